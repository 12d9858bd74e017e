#!/bin/bash
# round 4: engine tests, A/B host- vs device-sized forward, kernel traces of both
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r04g}
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_bundle_adjust.py tests/test_gpu_sparse_adam.py -x -v -m gpu \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${R}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/${R}_pytest.log | tail -3
[ $rc -ne 0 ] && { tail -40 gpurun_out/${R}_pytest.log; exit $rc; }
REPS=3 STEPS=60 LIBS="host= dev=PSVO_DEV_SIZED=1" bash scripts/gpu_ab_lib.sh || exit $?
for mode in host dev; do
  if [ $mode = dev ]; then export PSVO_DEV_SIZED=1; else unset PSVO_DEV_SIZED; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_prof_$mode -o run -- \
      python3 bench.py --steps 40 --warmup 5 --no-traffic --no-cpu-baseline > gpurun_out/${R}_prof_$mode.json 2> gpurun_out/${R}_prof_$mode.err
  rc=$?; echo "rocprof $mode rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
echo done
