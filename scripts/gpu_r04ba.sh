#!/bin/bash
# round 4: engine / bundle-adjust GPU tests, then one bench line with the
# bundle_adjust_frames call clock (PSVO_BA_PROFILE=1: where a call's fixed cost goes)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r04ba}
[ "${TESTS:-}" != none ] && { timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_engine.py tests/test_gpu_bundle_adjust.py tests/test_gpu_engine_fullsize_grads.py tests/test_gpu_dist_ba.py} \
    -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${R}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/${R}_pytest.log | tail -3
[ $rc -ne 0 ] && { tail -60 gpurun_out/${R}_pytest.log; exit $rc; }; }
PSVO_BA_PROFILE=1 timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-traffic \
    > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || exit $?
grep ba-call gpurun_out/${R}_bench.err | head -8
python3 -c "
import json
d=json.loads(open('gpurun_out/${R}_bench.json').read().strip().splitlines()[-1])
print(round(d['ms_per_step'],4), 'gpu', round(d['gpu_ms_per_step'],4), d['pace'])"
echo done
