set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
REPS=3 LIBS="r05=proud-slam_amd/lib/ab/libpsvo_r05.so cur= nobind=proud-slam_amd/lib/ab/libpsvo_nobind.so gate=PSVO_BA_DRAW_GATE=1 gr=PSVO_PX_RADIX=1,PSVO_BA_DRAW_GATE=1" bash scripts/gpu_ab_lib.sh || exit $?
echo "== E bench with PMC traffic"
timeout -k 10 600 python bench.py --scene multiroom --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06k_bench_E.json 2> gpurun_out/r06k_bench_E.err; rc=$?
echo "E rc=$rc"; tail -c 400 gpurun_out/r06k_bench_E.json; [ $rc -ne 0 ] && exit $rc
echo "== E kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06k_profE -o run -- python3 bench.py --scene multiroom --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --train-iters 0 > gpurun_out/r06k_profE_bench.json 2> gpurun_out/r06k_profE.err; rc=$?
echo "profE rc=$rc"
python3 scripts/ba_timeline.py gpurun_out/r06k_profE/run_kernel_trace.csv -- -10 > gpurun_out/r06k_E_timeline.txt 2>&1 || true
