#!/bin/bash
# round 4: BA / engine tests, then a rocprofv3 kernel-stats run of the default bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r04ps}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_bundle_adjust.py tests/test_gpu_engine.py tests/test_gpu_tracking.py} \
    -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${R}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/${R}_pytest.log | tail -3
[ $rc -ne 0 ] && { tail -60 gpurun_out/${R}_pytest.log; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic ${BENCH_ARGS:-} > gpurun_out/${R}_prof_bench.json 2> gpurun_out/${R}_prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 - <<'PY'
import csv, os
R = os.environ.get("R", "r04ps")
PY
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/${R}_prof/run_kernel_stats.csv')):
    n=r['Name']
    for k in ['k_pose_step_frames','k_intersect_sorted<true>','k_sample_fused','k_interp_fwd','k_mlp_fwd2','k_mlp_bwd3','k_composite_loss<4>','k_interp_rays_gx']:
        if k in n: print(k, r['Calls'], round(float(r['AverageNs'])/1000,2), round(float(r['MinNs'])/1000,2))
"
echo done
