#!/bin/bash
# k_mlp_bwd3 diagnostics on one GPU box: phase stamps (diag build), then a
# kernel trace of the decoder alone at the bench's sample count.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
M=${M:-261107}
timeout -k 10 120 python scripts/mlp_stamps.py $M > gpurun_out/b3_stamps.txt 2>&1
rc=$?; cat gpurun_out/b3_stamps.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b3_prof -o mlp -- \
    python3 scripts/mlp_bench.py --m $M > gpurun_out/b3_prof.log 2>&1
rc=$?; tail -2 gpurun_out/b3_prof.log; [ $rc -ne 0 ] && exit $rc
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/b3_prof/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.1f} us")
PY
