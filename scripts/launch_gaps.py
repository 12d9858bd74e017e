"""Diagnostic: idle gaps on the engine's main queue and when the host issued
the kernel that ended each gap (rocprofv3 --kernel-trace --hip-runtime-trace
of bench.py).  Per kernel name on the busiest queue, over the last N
iterations: the median gap after the previous kernel on that queue and the
median (API end - previous kernel end) — negative: the host had queued it
before the queue ran dry.  Usage: launch_gaps.py <run_dir> [iterations]"""
import csv
import os
import statistics
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    n_it = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    K = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
    A = {int(a["Correlation_Id"]): a for a in csv.DictReader(open(os.path.join(d, "run_hip_api_trace.csv")))}
    K.sort(key=lambda k: int(k["Start_Timestamp"]))
    qcount = defaultdict(int)
    for k in K:
        qcount[k["Queue_Id"]] += 1
    q1 = max(qcount, key=qcount.get)
    main_q = [k for k in K if k["Queue_Id"] == q1]
    poses = [i for i, k in enumerate(main_q) if "k_pose_step_frames" in k["Kernel_Name"]]
    if len(poses) < 2:
        sys.exit("no iterations found")
    lo = poses[max(0, len(poses) - 1 - n_it)]
    gaps, issue = defaultdict(list), defaultdict(list)
    for i in range(lo + 1, poses[-1] + 1):
        k, prev = main_q[i], main_q[i - 1]
        name = k["Kernel_Name"].replace("psvo::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:40]
        g = (int(k["Start_Timestamp"]) - int(prev["End_Timestamp"])) / 1e3
        gaps[name].append(g)
        a = A.get(int(k["Correlation_Id"]))
        if a:
            issue[name].append((int(a["End_Timestamp"]) - int(prev["End_Timestamp"])) / 1e3)
    print(f"queue {q1}: {poses[-1] - lo} kernels over {min(n_it, len(poses) - 1)} iterations")
    print(f"{'kernel':42s} {'gap µs':>8s} {'issued µs':>10s}")
    for name in gaps:
        iss = f"{statistics.median(issue[name]):10.1f}" if issue[name] else f"{'-':>10s}"
        print(f"{name:42s} {statistics.median(gaps[name]):8.1f} {iss}")


if __name__ == "__main__":
    main()
