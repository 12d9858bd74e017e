#!/bin/bash
# round 4: kernel + HIP runtime trace of the default bench (when the host
# issues each launch of a headline iteration)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r04w}
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/${R}_prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic ${BENCH_ARGS:-} > gpurun_out/${R}_prof_bench.json 2> gpurun_out/${R}_prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
for it in 8 12 16; do python3 scripts/ba_timeline.py gpurun_out/${R}_prof/run_kernel_trace.csv $it > gpurun_out/${R}_ba_timeline_$it.txt 2>&1 || true; done
# keep the API rows of one iteration's window only (the whole trace can exceed what gpurun copies back)
python3 - gpurun_out/${R}_prof <<'PY'
import csv, sys
d = sys.argv[1] + "/"
rows = sorted(csv.DictReader(open(d + "run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_pose_step_frames" in r["Kernel_Name"]]
if len(idx) > 13:
    t0, t1 = int(rows[idx[12]]["Start_Timestamp"]) - 4000000, int(rows[idx[13]]["Start_Timestamp"]) + 1000000
    api = list(csv.DictReader(open(d + "run_hip_api_trace.csv")))
    with open(d + "api_window.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(api[0].keys()))
        w.writeheader()
        w.writerows(r for r in api if t0 <= int(r["Start_Timestamp"]) <= t1)
PY
rm -f gpurun_out/${R}_prof/run_hip_api_trace.csv
echo done
