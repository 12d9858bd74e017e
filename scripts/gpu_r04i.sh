#!/bin/bash
# round 4 (session 2): same-box A/B host- vs device-sized forward, and a
# rocprofv3 kernel trace of the device-sized mode (timeline of one iteration)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r04i}
REPS=${REPS:-3} STEPS=${STEPS:-60} LIBS=${LIBS:-"host= dev=PSVO_DEV_SIZED=1"} bash scripts/gpu_ab_lib.sh || exit $?
for mode in ${TRACE_MODES:-dev}; do
  if [ $mode = dev ]; then export PSVO_DEV_SIZED=1; else unset PSVO_DEV_SIZED; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_prof_$mode -o run -- \
      python3 bench.py --steps 20 --warmup 5 --no-traffic --no-cpu-baseline > gpurun_out/${R}_prof_$mode.json 2> gpurun_out/${R}_prof_$mode.err
  rc=$?; echo "rocprof $mode rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 scripts/ba_timeline.py gpurun_out/${R}_prof_$mode/run_kernel_trace.csv > gpurun_out/${R}_timeline_$mode.txt 2>&1 || true
done
echo done
