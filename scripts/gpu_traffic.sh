#!/bin/bash
# HBM traffic per kernel from separate FETCH_SIZE / WRITE_SIZE passes
# (MI355X_MICROARCH.md: separate passes; FETCH_SIZE x2 on gfx950) → profiles/traffic.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_$c -o pmc --pmc $c -- \
      python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/pmc_$c.log 2>&1
  rc=$?; echo "$c rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 scripts/traffic_summary.py gpurun_out/pmc_FETCH_SIZE/pmc_counter_collection.csv \
    gpurun_out/pmc_WRITE_SIZE/pmc_counter_collection.csv gpurun_out/traffic.json
