#!/bin/bash
# Bench lines of the other BASELINE configs (C: ScanNet W=256 8x1024; E: multiroom W=256)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r02}
timeout -k 10 400 python bench.py --scene scannet0000 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${R}_bench_C.json 2> gpurun_out/${R}_bench_C.err
echo "C rc=$?"
timeout -k 10 500 python bench.py --scene multiroom --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${R}_bench_E.json 2> gpurun_out/${R}_bench_E.err
echo "E rc=$?"
