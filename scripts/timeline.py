"""Per-kernel timeline of one engine step from a rocprofv3 kernel trace:
start offset / duration / stream of every kernel between two consecutive
k_composite_loss launches (the fused loss pass runs once per mapping step)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "k_composite_loss" in r["Kernel_Name"]]
if len(marks) < 3:
    sys.exit("fewer than 3 engine steps in the trace")
k = int(sys.argv[2]) if len(sys.argv) > 2 else -3
a, b = marks[k], marks[k + 1]
# start the window at the step's first decoder-forward predecessor: the sample_points launch before a
start = a
while start > 0 and "k_sample_points" not in rows[start]["Kernel_Name"]:
    start -= 1
end = b
while end > a and "k_sample_points" not in rows[end]["Kernel_Name"]:
    end -= 1
t0 = int(rows[start]["Start_Timestamp"])
t_end = int(rows[end]["Start_Timestamp"])
print(f"step window {(t_end - t0) / 1e3:.1f} us")
for r in rows[start:end]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("psvo::(anonymous namespace)::", "")[:48]
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  q{r['Queue_Id']:>3} s{r['Stream_Id']:>3}  {name}")
