#!/bin/bash
# Round-3 evidence on one GPU box: the default bench line (headline =
# bundle_adjust_frames as Mapping calls it; roofline from headline-mode
# kernel durations + in-run PMC passes; CPU baseline), then a rocprofv3
# --kernel-trace --stats run of the same command (--no-traffic: its PMC
# children are separate processes) whose k_interp_bwd / chain averages the
# bench's roofline must agree with.  Usage: ROUND=r03a scripts/gpu_round3.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${ROUND:-r03}
ARGS=${BENCH_ARGS:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python bench.py $ARGS > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_prof -o run -- \
    python3 bench.py --no-traffic --no-cpu-baseline $ARGS > gpurun_out/${R}_prof_bench.json 2> gpurun_out/${R}_prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
echo done
