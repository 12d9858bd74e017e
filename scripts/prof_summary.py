"""Print the top kernels of a rocprofv3 kernel_stats.csv (per-call average and total)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot / 1e6:.2f} ms")
for r in rows[:n]:
    print(f"{r['Name'][:72]:72s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1e3:8.1f}us "
          f"{float(r['TotalDurationNs']) / 1e6:7.2f}ms")
