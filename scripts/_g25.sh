set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_bundle_adjust.py tests/test_gpu_pixels.py tests/test_gpu_rccl.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06u_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r06u_pytest.log
[ $rc -ne 0 ] && exit $rc
REPS=4 LIBS="prestop=proud-slam_amd/lib/ab/libpsvo_prestop.so cur=" bash scripts/gpu_ab_lib.sh || exit $?
