#!/bin/bash
# round 4: query variants, same box, interleaved: both look-backs (default),
# the traversal's only (PSVO_LB_SAMPLER=0), that + the ray-major
# compaction-in-interpolation (PSVO_INTERP_RAYS=1), the split kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r04r}
for rep in $(seq ${REPS:-3}); do
  for v in ${VARIANTS:-lb=PSVO_AB_NONE=1 lbis=PSVO_LB_SAMPLER=0 lbis_ir=PSVO_LB_SAMPLER=0,PSVO_INTERP_RAYS=1 lb_ir=PSVO_INTERP_RAYS=1 split=PSVO_QUERY_SPLIT=1}; do
    n=${v%%=*}; e=${v#*=}; e=${e//,/ }
    env $e timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-traffic ${BENCH_ARGS:-} \
        > gpurun_out/${R}_${n}_${rep}.json 2> gpurun_out/${R}_${n}_${rep}.err || exit $?
    python3 -c "
import json
d=json.loads(open('gpurun_out/${R}_${n}_${rep}.json').read().strip().splitlines()[-1])
print('$n $rep', round(d['ms_per_step'],4), 'gpu', round(d['gpu_ms_per_step'],4), 'frac', round(d['roofline']['frac'],3), {k: round(v*1e3,1) for k, v in d['kernels_ms_overlapped'].items()})"
  done
done
echo done
