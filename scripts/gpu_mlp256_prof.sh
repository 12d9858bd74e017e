#!/bin/bash
# W=256 decoder kernels: kernel-trace stats, then SQ counter passes (separate runs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
M=${M:-524288}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/m256 -o m256 -- \
    python3 scripts/mlp_bench.py --width 256 --m $M --iters 10 > gpurun_out/m256.log 2>&1
rc=$?; echo "stats rc=$rc"; tail -2 gpurun_out/m256.log
[ $rc -ne 0 ] && exit $rc
python3 scripts/prof_summary.py $(find gpurun_out/m256 -name "*kernel_stats.csv" | head -1) 12
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/m256_pmc1 -o pmc \
    --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -- \
    python3 scripts/mlp_bench.py --width 256 --m $M --iters 2 > gpurun_out/m256_pmc1.log 2>&1
rc=$?; echo "pmc1 rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/m256_pmc2 -o pmc \
    --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -- \
    python3 scripts/mlp_bench.py --width 256 --m $M --iters 2 > gpurun_out/m256_pmc2.log 2>&1
rc=$?; echo "pmc2 rc=$rc"
exit 0
