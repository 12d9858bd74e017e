#!/bin/bash
# round 4: the scan -> compaction hole, kernel traces of switch variants
# (VARIANTS="name=VAR=V,VAR2=V2 ..."), median gap and iteration per variant
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r04k}
for kv in ${VARIANTS}; do
  n=${kv%%=*}; p=${kv#*=}; envs="${p//,/ }"
  env $envs timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${R}_$n -o run -- \
      python3 bench.py --steps 30 --warmup 5 --no-traffic --no-cpu-baseline > gpurun_out/${R}_$n.json 2> gpurun_out/${R}_$n.err
  rc=$?; [ $rc -ne 0 ] && { echo "$n rc=$rc"; tail -5 gpurun_out/${R}_$n.err; exit $rc; }
  python3 scripts/scan_gap.py gpurun_out/${R}_$n/run_kernel_trace.csv $n
done
echo done
