set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
REPS=3 STEPS=20 BENCH_ARGS="--scene scannet0000 --train-iters 0" LIBS="gateC= nogateC=PSVO_BA_DRAW_GATE=0 radixC=PSVO_PX_RADIX=1" bash scripts/gpu_ab_lib.sh || exit $?
REPS=3 STEPS=20 BENCH_ARGS="--scene multiroom --train-iters 0" LIBS="gateE= nogateE=PSVO_BA_DRAW_GATE=0" bash scripts/gpu_ab_lib.sh || exit $?
