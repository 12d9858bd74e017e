set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pixels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06i_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r06i_pytest.log
[ $rc -ne 0 ] && exit $rc
REPS=3 LIBS="radix=PSVO_PX_RADIX=1 cur=" bash scripts/gpu_ab_lib.sh || exit $?
