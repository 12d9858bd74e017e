#!/bin/bash
# round 4: engine tests, a rocprofv3 kernel trace of the default bench, and the K sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r04f}
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_bundle_adjust.py tests/test_gpu_sparse_adam.py -x -v -m gpu \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${R}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/${R}_pytest.log | tail -3
[ $rc -ne 0 ] && { tail -40 gpurun_out/${R}_pytest.log; exit $rc; }
PSVO_BA_PROFILE=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic \
    > gpurun_out/${R}_callprof.json 2> gpurun_out/${R}_callprof.err || exit $?
grep "ba-call" gpurun_out/${R}_callprof.err | tail -2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_prof -o run -- \
    python3 bench.py --steps 40 --warmup 5 --no-traffic --no-cpu-baseline > gpurun_out/${R}_prof_bench.json 2> gpurun_out/${R}_prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_ksweep.sh || exit $?
echo done
