#!/bin/bash
# round 4: the whole GPU suite, then the query variants A/B (gpu_r04r.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r04t}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/${R}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/${R}_pytest.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" gpurun_out/${R}_pytest.log | head -20; tail -40 gpurun_out/${R}_pytest.log; exit $rc; }
ROUND=${R} bash scripts/gpu_r04r.sh
