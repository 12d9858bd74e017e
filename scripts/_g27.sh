set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_bundle_adjust.py tests/test_gpu_engine_fullsize_grads.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06w_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r06w_pytest.log
[ $rc -ne 0 ] && exit $rc
REPS=3 STEPS=20 BENCH_ARGS="--scene scannet0000 --train-iters 0" LIBS="preC=proud-slam_amd/lib/ab/libpsvo_pre256.so curC=" bash scripts/gpu_ab_lib.sh || exit $?
REPS=3 STEPS=20 BENCH_ARGS="--scene multiroom --train-iters 0" LIBS="preE=proud-slam_amd/lib/ab/libpsvo_pre256.so curE=" bash scripts/gpu_ab_lib.sh || exit $?
