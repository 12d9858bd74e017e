#!/bin/bash
# W=256 decoder: correctness, kernel stats at config C's sample count, config C bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -x -q --timeout 120 -p no:cacheprovider > gpurun_out/m256_test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/m256_test.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/m256_base -o m -- \
    python3 scripts/mlp_bench.py --width 256 --m 524288 --iters 10 > gpurun_out/m256_base.log 2>&1
rc=$?; echo "stats rc=$rc"; tail -1 gpurun_out/m256_base.log
[ $rc -ne 0 ] && exit $rc
python3 scripts/prof_summary.py $(find gpurun_out/m256_base -name "*kernel_stats.csv" | head -1) 5
timeout -k 10 300 python bench.py --scene scannet0000 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_C_r2.json 2> gpurun_out/bench_C_r2.err
rc=$?; echo "benchC rc=$rc"
python3 -c "
import json; d=json.load(open('gpurun_out/bench_C_r2.json')); print(d['value'], d['ms_per_step'], d['roofline_mfma']['frac'], d['kernels_ms'])"
