#!/bin/bash
# W = 256 decoder: correctness (vs torch fp32), then the kernels alone at
# config C's sample count under rocprofv3 --stats (LIBS: extra library
# builds to compare, name=path)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-m256b}
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py ${EXTRA_TESTS:-} -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${R}_test.log; [ $rc -ne 0 ] && { tail -30 gpurun_out/${R}_test.log; exit $rc; }
for kv in base= ${LIBS:-}; do
  n=${kv%%=*}; lib=${kv#*=}
  PSVO_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_$n -o m -- \
      python3 scripts/mlp_bench.py --width 256 --m ${M:-466287} --iters 10 > gpurun_out/${R}_$n.log 2>&1
  rc=$?; echo "$n rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/${R}_$n.log; exit $rc; }
  python3 scripts/prof_summary.py gpurun_out/${R}_$n/m_kernel_stats.csv 4
done
echo done
