set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_bundle_adjust.py tests/test_gpu_rccl.py tests/test_gpu_dist_engine.py tests/test_gpu_share.py tests/test_gpu_lookback.py tests/test_gpu_dist_ba.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06q_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r06q_pytest.log
[ $rc -ne 0 ] && exit $rc
REPS=3 LIBS="presplit=proud-slam_amd/lib/ab/libpsvo_presplit.so cur=" bash scripts/gpu_ab_lib.sh || exit $?
