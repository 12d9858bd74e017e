"""The bench line's per-region kernel times (roofline.parts_ms: kernel-bound
HIP events of the UNPROFILED run) against a rocprofv3 kernel trace of the
same command: per region, the sum over its kernels of the median span of
their launches in the last N iterations (the marked headline iterations are
a run's last; the packed-tree traversal k_intersect_sorted<true> is the
headline's).
Usage: parts_vs_rocprof.py bench.json run_kernel_trace.csv [N]"""
import csv
import json
import re
import statistics
import sys

REGION = {"intersect": ("k_intersect_sorted<true>", "k_ray_stats_rank"), "sample": ("k_sample_fused", "k_scan_samples"),
          "points": ("k_sample_points", "k_compact_rays"),
          "interp_fwd": ("k_interp_fwd", "k_interp_fwd_rays", "k_points_interp")}
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
n_last = int(sys.argv[3]) if len(sys.argv) > 3 else 20
parts = d["roofline"]["parts_ms"]
rows = list(csv.DictReader(open(sys.argv[2])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the marked headline iterations are the run's last n_last: launches after
# the (n_last + 1)-th last look-ahead pose step (k_pose_step_frames)
pose = [int(r["Start_Timestamp"]) for r in rows if "k_pose_step_frames" in r["Kernel_Name"]]
t_from = pose[-(n_last + 1)] if len(pose) > n_last else 0
rows = [r for r in rows if int(r["Start_Timestamp"]) >= t_from]
dur = {}
for r in rows:
    m = re.search(r"(k_\w+)(<[^>(]*>)?", r["Kernel_Name"])
    if m:
        dur.setdefault(m.group(1) + (m.group(2) or ""), []).append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(f"{'region':12s} {'bench ms':>9s} {'rocprof ms':>10s} {'ratio':>6s}")
tb = tt = 0.0
for k, names in REGION.items():
    if k not in parts or parts[k] <= 0:
        continue
    tr = sum(statistics.median(dur[n]) / 1e3 for n in names if n in dur)
    b = parts[k]
    tb += b
    tt += tr
    print(f"{k:12s} {b:9.4f} {tr:10.4f} {b / tr if tr else float('nan'):6.3f}")
print(f"{'chain':12s} {tb:9.4f} {tt:10.4f} {tb / tt if tt else float('nan'):6.3f}")
