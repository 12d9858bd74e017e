set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
REPS=3 LIBS="cur= nogate=PSVO_BA_DRAW_GATE=0 nowait=proud-slam_amd/lib/ab/libpsvo_nowait.so" bash scripts/gpu_ab_lib.sh || exit $?
REPS=2 STEPS=20 BENCH_ARGS="--scene multiroom --train-iters 0" LIBS="ib4E=proud-slam_amd/lib/ab/libpsvo_ib4.so curE=" bash scripts/gpu_ab_lib.sh || exit $?
REPS=2 STEPS=20 BENCH_ARGS="--scene scannet0000 --train-iters 0" LIBS="ib4C=proud-slam_amd/lib/ab/libpsvo_ib4.so curC=" bash scripts/gpu_ab_lib.sh || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/r06o_prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --train-iters 100 > gpurun_out/r06o_prof_bench.json 2> gpurun_out/r06o_prof.err
echo "prof rc=$?"
python3 scripts/ba_timeline.py gpurun_out/r06o_prof/run_kernel_trace.csv -- -10 > gpurun_out/r06o_ba_timeline.txt 2>&1 || true
