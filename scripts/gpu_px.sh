#!/bin/bash
# pixel sampler + bundle-adjust tests, then the BA headline bench (short)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_pixels.py tests/test_gpu_bundle_adjust.py} -x -v -m gpu \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_px.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|PASSED|FAILED|Error" gpurun_out/pytest_px.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_px.json 2> gpurun_out/bench_px.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench_px.json; tail -3 gpurun_out/bench_px.err
