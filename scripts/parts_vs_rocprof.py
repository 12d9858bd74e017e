"""The bench line's per-region kernel times (roofline.parts_ms, kernel-bound
HIP events) against the rocprofv3 kernel trace of the same command: per
region, the mean per-iteration sum of its kernels' spans over the headline
iterations.  Usage: parts_vs_rocprof.py bench.json run_kernel_trace.csv"""
import csv
import json
import re
import statistics
import sys

REGION = {"intersect": ("k_intersect_sorted", "k_ray_stats_rank"), "sample": ("k_sample_fused", "k_scan_samples"),
          "points": ("k_sample_points", "k_compact_rays"),
          "interp_fwd": ("k_interp_fwd", "k_interp_fwd_rays", "k_points_interp")}
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
parts = d["roofline"]["parts_ms"]
rows = list(csv.DictReader(open(sys.argv[2])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = {}
for r in rows:
    m = re.search(r"k_\w+", r["Kernel_Name"])
    if m:
        dur.setdefault(m.group(0), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
# the headline iterations run k_intersect_sorted<true> (packed); per region the median span per launch
print(f"{'region':12s} {'bench ms':>9s} {'rocprof ms':>10s} {'ratio':>6s}")
for k, names in REGION.items():
    if k not in parts:
        continue
    tr = 0.0
    for n in names:
        if n in dur:
            tr += statistics.median(dur[n]) / 1e3
    b = parts[k]
    print(f"{k:12s} {b:9.4f} {tr:10.4f} {b / tr if tr else float('nan'):6.3f}")
