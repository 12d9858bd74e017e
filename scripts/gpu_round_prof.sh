#!/bin/bash
# Round evidence on one GPU box: the unprofiled bench line (with the CPU
# baseline), a rocprofv3 --kernel-trace --stats run of the same command, the
# kernel trace split by engine mode, and the HBM traffic from separate
# FETCH_SIZE / WRITE_SIZE --pmc passes.  Usage: ROUND=r02 scripts/gpu_round_prof.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${ROUND:-r02}
ARGS=${BENCH_ARGS:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 20 --warmup 5 $ARGS > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_prof -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline $ARGS > gpurun_out/${R}_prof_bench.json 2> gpurun_out/${R}_prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 scripts/kernel_modes.py gpurun_out/${R}_prof/run_kernel_trace.csv gpurun_out/${R}_kernel_modes.json > /dev/null
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${R}_pmc_$c -o pmc --pmc $c -- \
      python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline $ARGS > gpurun_out/${R}_pmc_$c.log 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 scripts/traffic_summary.py gpurun_out/${R}_pmc_FETCH_SIZE/pmc_counter_collection.csv \
    gpurun_out/${R}_pmc_WRITE_SIZE/pmc_counter_collection.csv gpurun_out/${R}_traffic.json ${SCENE:-room0} > /dev/null
echo done
