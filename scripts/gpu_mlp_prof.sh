#!/bin/bash
# MLP kernel profiling: per-layer dW dispatches, then SQ counters (separate passes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
PSVO_DW_LAYER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mlp_layers -o mlp -- \
    python3 scripts/mlp_bench.py > gpurun_out/mlp_layers.log 2>&1
rc=$?; echo "layers rc=$rc"; cat gpurun_out/mlp_layers.log | tail -2
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/mlp_pmc1 -o pmc \
    --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -- \
    python3 scripts/mlp_bench.py --iters 3 > gpurun_out/mlp_pmc1.log 2>&1
rc=$?; echo "pmc1 rc=$rc"; tail -3 gpurun_out/mlp_pmc1.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/mlp_pmc2 -o pmc \
    --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -- \
    python3 scripts/mlp_bench.py --iters 3 > gpurun_out/mlp_pmc2.log 2>&1
rc=$?; echo "pmc2 rc=$rc"; tail -3 gpurun_out/mlp_pmc2.log
exit 0
