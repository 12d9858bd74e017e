#!/bin/bash
# A/B of an engine environment switch on one box: VAR=name VALS="0 1" scripts/gpu_ab_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VALS:-0 1}; do
  t=${v//\//_}
  env $VAR=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$t.json 2> gpurun_out/ab_$t.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ab_$t.json'));print('$VAR=$v', round(d['ms_per_step'],4), [round(o['ms_per_step'],4) for o in d['other_path']], {k: round(v*1e3,1) for k, v in d['roofline']['parts_ms'].items()}, round(d['roofline']['frac'],3))"
done
if [ "${PROF:-0}" = "1" ]; then
  export $VAR=${PROF_VAL:-1}
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab_prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2>&1
  echo prof=$?
fi
