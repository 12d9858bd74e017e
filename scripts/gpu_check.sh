#!/bin/bash
# One GPU-box session: parity tests, a short bench, a rocprofv3 kernel trace.
# Stops at the first crash / timeout (exit codes other than 0/1 from pytest).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-20}
timeout -k 10 300 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 600 python bench.py --steps $STEPS --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
      python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
  rc=$?
  echo "rocprof rc=$rc"
  find gpurun_out/prof -name "*stats*" | head
fi
if [ "${DIST:-0}" = "1" ]; then
  # N>1 rehearsal: two ranks sharing the one GPU over gloo (the driver runs RCCL on 8 GPUs)
  PSVO_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 \
      > gpurun_out/bench_dist2.json 2> gpurun_out/bench_dist2.err
  rc=$?
  echo "dist2 rc=$rc"; cat gpurun_out/bench_dist2.json; tail -5 gpurun_out/bench_dist2.err
fi
