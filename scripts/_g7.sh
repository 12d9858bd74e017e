set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_lookback.py tests/test_gpu_dist_engine.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06f_pytest.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/r06f_pytest.log
REPS=3 LIBS="r05=proud-slam_amd/lib/ab/libpsvo_r05.so cur= gate=PSVO_BA_DRAW_GATE=1" bash scripts/gpu_ab_lib.sh
