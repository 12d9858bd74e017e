#!/bin/bash
# round 4: the look-back query (statistics / rank pass and sample scan inside
# the traversal / sampler launches) — its tests, then same-box A/B against the
# split kernels (PSVO_QUERY_SPLIT=1), interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r04q}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_engine.py tests/test_gpu_bundle_adjust.py tests/test_gpu_dist_ba.py tests/test_gpu_rccl.py tests/test_gpu_engine_fullsize_grads.py} \
    -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${R}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/${R}_pytest.log | tail -3
[ $rc -ne 0 ] && { tail -60 gpurun_out/${R}_pytest.log; exit $rc; }
for rep in $(seq ${REPS:-3}); do
  for v in lb=PSVO_AB_NONE=1 split=PSVO_QUERY_SPLIT=1; do
    n=${v%%=*}; e=${v#*=}
    env $e timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-traffic ${BENCH_ARGS:-} \
        > gpurun_out/${R}_${n}_${rep}.json 2> gpurun_out/${R}_${n}_${rep}.err || exit $?
    python3 -c "
import json
d=json.loads(open('gpurun_out/${R}_${n}_${rep}.json').read().strip().splitlines()[-1])
print('$n $rep', round(d['ms_per_step'],4), 'gpu', round(d['gpu_ms_per_step'],4), 'frac', round(d['roofline']['frac'],3), {k: round(v*1e3,1) for k, v in d['kernels_ms_overlapped'].items()})"
  done
done
echo done
