#!/bin/bash
# round 6: GPU suite + the default bench (+ optional rocprofv3 kernel trace).
# Stops at the first crash / timeout (pytest exit codes other than 0/1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r06}
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
      ${PYTEST_ARGS:-} > gpurun_out/${R}_pytest.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -25 gpurun_out/${R}_pytest.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 400 python bench.py --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS:-} > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err
  rc=$?
  echo "bench rc=$rc"; cat gpurun_out/${R}_bench.json; tail -3 gpurun_out/${R}_bench.err
  [ $rc -ne 0 ] && exit $rc
fi
if [ "${PROFILE:-0}" = "1" ]; then
  API=""; [ "${PROFILE_API:-0}" = "1" ] && API="--hip-runtime-trace"
  timeout -k 10 400 rocprofv3 --kernel-trace ${API} --stats --output-format csv -d gpurun_out/${R}_prof -o run -- \
      python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic ${BENCH_ARGS:-} \
      > gpurun_out/${R}_prof_bench.json 2> gpurun_out/${R}_prof.err
  rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
  for it in ${TL_ITERS:--30 -25}; do python3 scripts/ba_timeline.py gpurun_out/${R}_prof/run_kernel_trace.csv -- $it > gpurun_out/${R}_ba_timeline_$it.txt 2>&1 || true; done
  rm -f gpurun_out/${R}_prof/run_kernel_trace.csv.bak gpurun_out/${R}_prof/run_hip_api_trace.csv.bak
fi
if [ "${CONFIGS:-0}" = "1" ]; then  # C: ScanNet W=256 8x1024; E: multiroom W=256
  timeout -k 10 400 python bench.py --scene scannet0000 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic \
      > gpurun_out/${R}_bench_C.json 2> gpurun_out/${R}_bench_C.err
  rc=$?; echo "C rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 500 python bench.py --scene multiroom --steps 20 --warmup 5 --no-cpu-baseline --no-traffic \
      > gpurun_out/${R}_bench_E.json 2> gpurun_out/${R}_bench_E.err
  rc=$?; echo "E rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 - gpurun_out/${R}_bench_C.json gpurun_out/${R}_bench_E.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), d["ms_per_step"], d["gpu_ms_per_step"], d["config"].get("decoder_kept_fraction"),
          d["roofline_mfma"]["fwd_ms"], d["roofline_mfma"]["bwd_ms"])
PY
fi

if [ "${DIST:-0}" = "1" ]; then
  # N>1 rehearsal: two ranks sharing the one GPU over gloo (the driver runs RCCL on 8 GPUs)
  PSVO_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 ${DIST_ARGS:-} \
      > gpurun_out/${R}_bench_dist2.json 2> gpurun_out/${R}_bench_dist2.err
  rc=$?
  echo "dist2 rc=$rc"; tail -c 600 gpurun_out/${R}_bench_dist2.json; tail -5 gpurun_out/${R}_bench_dist2.err
fi
echo done
