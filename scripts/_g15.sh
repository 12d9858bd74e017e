set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lookback.py tests/test_gpu_dist_engine.py tests/test_gpu_share.py tests/test_gpu_tree_pack.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06m_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r06m_pytest.log
[ $rc -ne 0 ] && exit $rc
REPS=2 STEPS=20 BENCH_ARGS="--scene multiroom --train-iters 0" LIBS="r05E=proud-slam_amd/lib/ab/libpsvo_r05.so curE=" bash scripts/gpu_ab_lib.sh || exit $?
REPS=3 LIBS="r05=proud-slam_amd/lib/ab/libpsvo_r05.so cur=" bash scripts/gpu_ab_lib.sh || exit $?
