set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
REPS=3 STEPS=20 BENCH_ARGS="--scene multiroom --train-iters 0" LIBS="nochunkE=proud-slam_amd/lib/ab/libpsvo_nochunk.so curE=" bash scripts/gpu_ab_lib.sh || exit $?
REPS=3 LIBS="nochunk=proud-slam_amd/lib/ab/libpsvo_nochunk.so cur=" bash scripts/gpu_ab_lib.sh || exit $?
