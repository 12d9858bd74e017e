set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pixels.py tests/test_gpu_bundle_adjust.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06h_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r06h_pytest.log
[ $rc -ne 0 ] && exit $rc
REPS=3 LIBS="radix=PSVO_PX_RADIX=1 cur=" bash scripts/gpu_ab_lib.sh || exit $?
ROUND=r06h TESTS=0 BENCH=0 PROFILE=1 TL_ITERS="-30 -25" BENCH_ARGS="--train-iters 200" bash scripts/gpu_r06.sh
