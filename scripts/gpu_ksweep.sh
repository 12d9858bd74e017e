#!/bin/bash
# Per-call overhead of bundle_adjust_frames: the default bench line at several
# K (iterations per call; the driver runs K = 20), one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in ${KS:-10 20 100}; do
  timeout -k 10 200 python bench.py --steps $k --warmup 5 --no-cpu-baseline --no-traffic ${BENCH_ARGS:-} \
      > gpurun_out/ksweep_${k}.json 2> gpurun_out/ksweep_${k}.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/ksweep_${k}.json'));print('K', $k, round(d['ms_per_step'],4), 'gpu', d.get('gpu_ms_per_step'), {k: v for k, v in (d.get('pace') or {}).items() if k != 'note'})"
done
