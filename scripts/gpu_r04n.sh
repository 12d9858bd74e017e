#!/bin/bash
# round 4: the default bench line and a rocprofv3 kernel trace of the same
# command; the bench's per-region kernel times against the trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r04n}
timeout -k 10 400 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/${R}_bench.err; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic ${BENCH_ARGS:-} > gpurun_out/${R}_prof_bench.json 2> gpurun_out/${R}_prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 scripts/parts_vs_rocprof.py gpurun_out/${R}_prof_bench.json gpurun_out/${R}_prof/run_kernel_trace.csv
python3 scripts/ba_timeline.py gpurun_out/${R}_prof/run_kernel_trace.csv > gpurun_out/${R}_ba_timeline.txt 2>&1 || true
python3 -c "
import json
d=json.loads(open('gpurun_out/${R}_bench.json').read().strip().splitlines()[-1])
print('bench', round(d['ms_per_step'],4), 'gpu', round(d['gpu_ms_per_step'],4), 'value', round(d['value']/1e6,3), 'frac', round(d['roofline']['frac'],3), 'mfma', round(d['roofline_mfma']['frac'],3))
print({k: round(v*1e3,1) for k, v in d['kernels_ms_overlapped'].items()})
"
echo done
