#!/bin/bash
# PMC passes (one rocprofv3 run per counter set, kernel trace only) over
# scripts/mlp_bench.py; sets separated by ';' in PMC_SETS.  Output under
# gpurun_out/pmc_<i>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
IFS=';' read -ra SETS <<< "${PMC_SETS}"
for set in "${SETS[@]}"; do
  i=$((i + 1))
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_$i -o pmc --pmc $set -- \
      ${PMC_CMD:-python3 scripts/mlp_bench.py --iters 3} > gpurun_out/pmc_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
