#!/bin/bash
# Kernel trace of the bench headline (bundle_adjust_frames) and one
# iteration's timeline (scripts/ba_timeline.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-tl}
timeout -k 10 300 rocprofv3 --kernel-trace ${HIPTRACE:+--hip-runtime-trace} --output-format csv -d gpurun_out/${T}_trace -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic ${BENCH_ARGS:-} > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_trace.err
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/${T}_trace -name '*kernel_trace.csv' | head -1)
python3 scripts/ba_timeline.py "$f" ${ITER:-12} > gpurun_out/${T}_timeline.txt
cat gpurun_out/${T}_timeline.txt
