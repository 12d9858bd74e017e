#!/bin/bash
# Round-2 GPU session: selected / all GPU tests, the N=1 bench, a 2-rank
# launcher rehearsal over gloo on the one GPU.  Stops after any crash or time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-tests}
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -x -v -m gpu --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_r2.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|PASSED|FAILED|Error" gpurun_out/pytest_r2.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python bench.py --steps ${STEPS:-20} --warmup 5 > gpurun_out/bench_r2.json 2> gpurun_out/bench_r2.err
  rc=$?
  echo "bench rc=$rc"; cat gpurun_out/bench_r2.json; tail -5 gpurun_out/bench_r2.err
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ "${DIST:-0}" = "1" ]; then
  PSVO_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 3 \
      > gpurun_out/bench_dist2_r2.json 2> gpurun_out/bench_dist2_r2.err
  rc=$?
  echo "dist2 rc=$rc"; cat gpurun_out/bench_dist2_r2.json; tail -5 gpurun_out/bench_dist2_r2.err
fi
