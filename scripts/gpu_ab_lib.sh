#!/bin/bash
# Same-box A/B of library builds or engine switches: LIBS="name=spec ..."
# where spec is a library path ('' = the product lib) or VAR=VALUE (an
# environment switch on the product lib); REPS rounds of one short bench line
# per entry, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in $(seq ${REPS:-3}); do
  for kv in ${LIBS}; do
    n=${kv%%=*}; p=${kv#*=}
    if [[ "$p" == *=* ]]; then envs="${p//,/ }"; lib=""; else envs="PSVO_AB_NONE=1"; lib="$p"; fi
    env PSVO_LIB_PATH=$lib $envs timeout -k 10 200 python bench.py --steps ${STEPS:-40} --warmup 5 --no-cpu-baseline \
        --no-traffic ${BENCH_ARGS:-} > gpurun_out/ablib_${n}_${rep}.json 2> gpurun_out/ablib_${n}_${rep}.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/ablib_${n}_${rep}.json'));print('$n', $rep, round(d['ms_per_step'],4), {k: round(v*1e3,1) for k,v in d['kernels_ms_overlapped'].items() if k in ('intersect','sample','select','interp_fwd','mlp_fwd','mlp_bwd')})"
  done
done
