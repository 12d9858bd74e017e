#!/bin/bash
# round 4: pixel-draw tests, then the small-LDS draw histograms against the
# 16-KB ones (PSVO_PX_WIDE_LDS=1), interleaved, and a timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pixels.py tests/test_gpu_bundle_adjust.py -x -q -m gpu \
    -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r04px_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r04px_pytest.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="small=PSVO_AB_NONE=1 wide=PSVO_PX_WIDE_LDS=1" ROUND=r04px bash scripts/gpu_r04r.sh || exit $?
ROUND=r04pxt bash scripts/gpu_r04w.sh
