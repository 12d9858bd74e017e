#!/bin/bash
# round 4: kernel + HIP runtime trace of the default bench (when the host
# issues each launch of a headline iteration)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r04w}
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/${R}_prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic ${BENCH_ARGS:-} > gpurun_out/${R}_prof_bench.json 2> gpurun_out/${R}_prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
for it in 8 12 16; do python3 scripts/ba_timeline.py gpurun_out/${R}_prof/run_kernel_trace.csv $it > gpurun_out/${R}_ba_timeline_$it.txt 2>&1 || true; done
rm -f gpurun_out/${R}_prof/run_hip_api_trace.csv.gz
echo done
