"""Kernel timeline of one bundle_adjust_frames iteration from a rocprofv3
kernel trace: start / end / duration (us, relative to the iteration's
look-ahead pose kernel: k_pose_step_frames, or k_pose_rays_frames before it
existed) and queue of every kernel; with a HIP runtime trace beside it
(rocprofv3 --hip-runtime-trace), also when the host issued each launch.
Usage: ba_timeline.py run_kernel_trace.csv [--] [iteration index; negative: from the last]"""
import csv
import os
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
argv = [a for a in sys.argv[1:] if a != "--"]  # (`--` lets a negative index through: from the end)
k = int(argv[1]) if len(argv) > 1 else 8
api = {}
hip = sys.argv[1].replace("kernel_trace.csv", "hip_api_trace.csv")
if os.path.exists(hip):
    for r in csv.DictReader(open(hip)):
        api[r["Correlation_Id"]] = int(r["Start_Timestamp"])
mark = "k_pose_step_frames" if any("k_pose_step_frames" in r["Kernel_Name"] for r in rows) else "k_pose_rays_frames"
idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
a, b = idx[k], idx[k + 1]
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a:b + 1]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
    name = m.group(1) if m else r["Kernel_Name"][:40]
    issued = api.get(r.get("Correlation_Id"))
    host = f"  host {(issued - t0) / 1e3:8.1f}" if issued is not None else ""
    print(f"{s / 1e3:8.1f} {e / 1e3:8.1f} {(e - s) / 1e3:7.1f}  q{r['Queue_Id']}  {name}{host}")
