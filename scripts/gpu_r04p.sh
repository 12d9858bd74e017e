#!/bin/bash
# round 4: the W = 256 fused interpolation backward — its tests, then configs
# C and E with and without it (PSVO_IB256_FUSED=0), interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r04p}
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_bundle_adjust.py tests/test_gpu_engine_fullsize_grads.py \
    tests/test_gpu_engine.py -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${R}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/${R}_pytest.log | tail -3
[ $rc -ne 0 ] && { tail -60 gpurun_out/${R}_pytest.log; exit $rc; }
for rep in 1 2; do
  for sc in scannet0000 multiroom; do
    for v in fused=PSVO_AB_NONE=1 sep=PSVO_IB256_FUSED=0; do
      n=${v%%=*}; e=${v#*=}
      env $e timeout -k 10 500 python bench.py --scene $sc --steps 20 --warmup 5 --no-cpu-baseline --no-traffic \
          > gpurun_out/${R}_${sc}_${n}_${rep}.json 2> gpurun_out/${R}_${sc}_${n}_${rep}.err || exit $?
      python3 -c "
import json
d=json.loads(open('gpurun_out/${R}_${sc}_${n}_${rep}.json').read().strip().splitlines()[-1])
print('$sc $n $rep', round(d['ms_per_step'],4), round(d['value']/1e6,3), {k: round(v*1e3,1) for k, v in d['kernels_ms_overlapped'].items()})"
    done
  done
done
echo done
