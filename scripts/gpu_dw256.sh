#!/bin/bash
# k_dec256_dw workgroup split sweep (PSVO_DW256_W), decoder alone at config C's M
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in ${WS:-213,120,120,107}; do
  PSVO_DW256_W=$w timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dw_$w -o m -- \
      python3 scripts/mlp_bench.py --width 256 --m ${M:-466287} --iters 6 > gpurun_out/dw_$w.log 2>&1 || exit $?
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/dw_$w/m_kernel_stats.csv')):
    if 'k_dec256_dw(' in r['Name']: print('$w', round(float(r['AverageNs'])/1e3,1), 'us')"
done
