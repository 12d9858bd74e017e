set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tree_pack.py tests/test_gpu_fullsize_parity.py tests/test_gpu_lookback.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06j_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r06j_pytest.log
[ $rc -ne 0 ] && exit $rc
echo "== E traversal A/B"
REPS=2 STEPS=20 BENCH_ARGS="--scene multiroom --train-iters 0" LIBS="preE=proud-slam_amd/lib/ab/libpsvo_pre2.so curE=" bash scripts/gpu_ab_lib.sh || exit $?
echo "== B draw placement A/B"
REPS=3 LIBS="radix=PSVO_PX_RADIX=1 cur= after=PSVO_BA_DRAW_AFTER_STEP=1 gate=PSVO_BA_DRAW_GATE=1 preB=proud-slam_amd/lib/ab/libpsvo_pre2.so smp1=proud-slam_amd/lib/ab/libpsvo_smp1.so smp3=proud-slam_amd/lib/ab/libpsvo_smp3.so r05=proud-slam_amd/lib/ab/libpsvo_r05.so" bash scripts/gpu_ab_lib.sh || exit $?
