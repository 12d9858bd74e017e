#!/bin/bash
# round 4: the FAST draw's candidate path — pixel / BA tests, then A/B
# against the radix passes alone (PSVO_PX_CAND=0), interleaved, and a timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pixels.py tests/test_gpu_bundle_adjust.py -x -v -m gpu \
    -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r04pc_pytest.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r04pc_pytest.log | tail -3
[ $rc -ne 0 ] && { tail -40 gpurun_out/r04pc_pytest.log; exit $rc; }
VARIANTS="cand=PSVO_PX_CAND=1 radix=PSVO_PX_CAND=0" ROUND=r04pc bash scripts/gpu_r04r.sh || exit $?
PSVO_PX_CAND=1 ROUND=r04pct bash scripts/gpu_r04w.sh
