"""GPU busy vs idle over the last N steps of a rocprofv3 kernel trace: one
step starts at each k_intersect_sorted launch."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n_last = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_intersect_sorted" in r["Kernel_Name"]]
steps = list(zip(starts[-n_last - 1:-1], starts[-n_last:]))
for a, b in steps:
    seg = rows[a:b]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    gaps = []
    for x, y in zip(seg, seg[1:]):
        g = int(y["Start_Timestamp"]) - int(x["End_Timestamp"])
        if g > 20000:
            gaps.append((g / 1e3, x["Kernel_Name"][:40], y["Kernel_Name"][:40]))
    print(f"step {(t1 - t0) / 1e3:8.1f} us  busy {busy / 1e3:8.1f} us  kernels {len(seg)}")
    for g in sorted(gaps, reverse=True)[:6]:
        print(f"    gap {g[0]:7.1f} us after {g[1]} before {g[2]}")
