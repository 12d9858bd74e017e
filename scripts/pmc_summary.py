"""Per-kernel PMC summary of scripts/gpu_pmc.sh passes: mean counter value
per dispatch for the kernels named on the command line (substring match)."""
import csv
import glob
import sys
from collections import defaultdict

names = sys.argv[1:] or ["k_mlp_bwd3", "k_mlp_fwd2"]
acc = defaultdict(list)
for f in sorted(glob.glob("gpurun_out/pmc_*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = next((n for n in names if n in r["Kernel_Name"]), None)
        if k:
            acc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{k:14s} {c:34s} {sum(v) / len(v):16.4g}  ({len(v)} dispatches)")
