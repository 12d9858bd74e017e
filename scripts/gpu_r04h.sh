#!/bin/bash
# round 4 (session 2): the whole -m gpu suite, the default bench line (as the
# driver runs it: PMC passes + CPU baseline), a rocprofv3 kernel trace of the
# same command, then configs C and E.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r04h}
if [ "${TESTS:-all}" != "none" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 \
      --timeout-method thread > gpurun_out/${R}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/${R}_pytest.log | tail -3
  [ $rc -ne 0 ] && { tail -60 gpurun_out/${R}_pytest.log; exit $rc; }
fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/${R}_bench.err; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/${R}_prof_bench.json 2> gpurun_out/${R}_prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 scripts/ba_timeline.py gpurun_out/${R}_prof/run_kernel_trace.csv > gpurun_out/${R}_ba_timeline.txt 2>&1 || true
if [ "${CONFIGS:-1}" = "1" ]; then
  timeout -k 10 400 python bench.py --scene scannet0000 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${R}_bench_C.json 2> gpurun_out/${R}_bench_C.err
  rc=$?; echo "C rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 500 python bench.py --scene multiroom --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${R}_bench_E.json 2> gpurun_out/${R}_bench_E.err
  rc=$?; echo "E rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
echo done
