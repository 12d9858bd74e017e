#!/bin/bash
# round 4: kernel-bound timing events with a device-scope release (default)
# against the system-scope one (PSVO_TIMING_SYSFENCE=1), then a rocprofv3
# kernel trace of the default line and its per-region comparison
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r04v}
VARIANTS="dev=PSVO_AB_NONE=1 sys=PSVO_TIMING_SYSFENCE=1" REPS=2 ROUND=$R bash scripts/gpu_r04r.sh || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/${R}_prof_bench.json 2> gpurun_out/${R}_prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 scripts/parts_vs_rocprof.py gpurun_out/${R}_prof_bench.json gpurun_out/${R}_prof/run_kernel_trace.csv
python3 scripts/parts_vs_rocprof.py gpurun_out/${R}_dev_1.json gpurun_out/${R}_prof/run_kernel_trace.csv
echo done
