#!/bin/bash
# W=256 decoder: correctness, then NC=1 (product) vs NC=2 (diag) kernel times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PSVO_LIB_PATH=$PWD/proud-slam_amd/lib/ab/libpsvo_nc2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -x -q --timeout 120 -p no:cacheprovider > gpurun_out/m256_test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/m256_test.log
[ $rc -ne 0 ] && exit $rc
for v in base nc2; do
  if [ $v = nc2 ]; then export PSVO_LIB_PATH=$PWD/proud-slam_amd/lib/ab/libpsvo_nc2.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/m256_$v -o m -- \
      python3 scripts/mlp_bench.py --width 256 --m 524288 --iters 10 > gpurun_out/m256_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; tail -1 gpurun_out/m256_$v.log
  [ $rc -ne 0 ] && exit $rc
  python3 scripts/prof_summary.py $(find gpurun_out/m256_$v -name "*kernel_stats.csv" | head -1) 5
done
