"""Per-kernel HBM bytes per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE
passes (KB units; FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 note)."""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return vals


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0].split("<")[0].split("::")[-1].strip() or name[:40]


fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
write = per_kernel(sys.argv[2], "WRITE_SIZE")
out = {"note": "bytes per launch, median over launches; fetch = 2 x FETCH_SIZE (gfx950), write = WRITE_SIZE",
       "kernels": {}}
for k in sorted(set(fetch) | set(write)):
    f = sorted(fetch.get(k, [0.0]))
    w = sorted(write.get(k, [0.0]))
    fm, wm = 2.0 * f[len(f) // 2], w[len(w) // 2]
    out["kernels"][short(k)] = {"fetch": fm, "write": wm, "total": fm + wm, "launches": len(f)}
K = out["kernels"]
if "k_interp_bwd" in K:
    out["interp_bwd_bytes_per_launch"] = K["k_interp_bwd"]["total"]
mlp = [n for n in ("k_mlp_prep", "k_mlp_fwd", "k_mlp_fwd2", "k_mlp_bwd_data", "k_mlp_bwd2", "k_mlp_dw",
                    "k_mlp_dw2", "k_mlp_dw_reduce") if n in K]
out["mlp_bytes_per_step"] = sum(K[n]["total"] for n in mlp)
qi = [n for n in ("k_intersect_sorted", "k_ray_stats_rank", "k_sample_fused", "k_scan_samples",
                  "k_sample_points", "k_interp_fwd", "k_interp_bwd") if n in K]
out["query_interp_bytes_per_step"] = sum(K[n]["total"] for n in qi)
out["scene"] = sys.argv[4] if len(sys.argv) > 4 else "room0"  # the bench scene the passes ran (gpu_traffic.sh: default)
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps({k: round(v["total"] / 1e6, 2) for k, v in K.items()}, indent=0))
