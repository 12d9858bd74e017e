"""Median GPU idle time on the critical queue between the query's sample scan
and the step's next kernel (the compaction) in a rocprofv3 kernel trace, and
the median iteration period (k_pose_step_frames to k_pose_step_frames).
Usage: scan_gap.py run_kernel_trace.csv [label]"""
import csv
import re
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
gaps, nxt = [], {}
for i, r in enumerate(rows):
    if "k_scan_samples" not in r["Kernel_Name"]:
        continue
    for y in rows[i + 1:]:
        if y["Queue_Id"] == r["Queue_Id"]:
            m = re.search(r"k_\w+", y["Kernel_Name"])
            name = m.group(0) if m else y["Kernel_Name"][:30]
            if "compact" in name or "sample_points" in name or "interp_fwd" in name:
                gaps.append((int(y["Start_Timestamp"]) - int(r["End_Timestamp"])) / 1e3)
                nxt[name] = nxt.get(name, 0) + 1
            break
pose = [int(r["Start_Timestamp"]) for r in rows if "k_pose_step_frames" in r["Kernel_Name"]]
per = [(b - a) / 1e3 for a, b in zip(pose, pose[1:]) if (b - a) < 3e6]
lab = sys.argv[2] if len(sys.argv) > 2 else ""
print(f"{lab} scan->next gap median {statistics.median(gaps):.1f} us (n={len(gaps)}, {nxt}); "
      f"iteration median {statistics.median(per):.1f} us (n={len(per)})")
