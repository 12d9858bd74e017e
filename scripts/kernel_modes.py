"""Per-kernel average duration split by engine mode, from one rocprofv3
kernel trace of bench.py: 'headline' steps (loss normalisers and embedding
backward on the aux stream, overlapping the decoder kernels) vs 'timed'
steps (the HIP-event breakdown run: every launch on one stream, so each
kernel's duration is its own).  The roofline numbers in bench.py come from
the timed steps; a plain --stats average mixes both modes (k_interp_bwd
co-resident with k_mlp_dw2 runs longer, by design)."""
import collections
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# a step = the launches from one k_sample_points (main stream) to the next
main_q = collections.Counter(r["Queue_Id"] for r in rows if "k_mlp_fwd2" in r["Kernel_Name"]).most_common(1)[0][0]
starts = [i for i, r in enumerate(rows) if "k_sample_points" in r["Kernel_Name"] and r["Queue_Id"] == main_q]
acc = {"headline": collections.defaultdict(list), "timed": collections.defaultdict(list)}
for a, b in zip(starts, starts[1:]):
    seg = rows[a:b]
    counts = [r for r in seg if "k_crit_counts" in r["Kernel_Name"]]
    if not counts:
        continue  # drop-in autograd path step
    mode = "timed" if counts[0]["Queue_Id"] == main_q else "headline"
    for r in seg:
        name = r["Kernel_Name"].replace("psvo::(anonymous namespace)::", "").split("(")[0]
        acc[mode][name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
out = {m: {k: {"avg_us": round(sum(v) / len(v), 2), "launches": len(v)} for k, v in sorted(d.items())}
       for m, d in acc.items()}
json.dump(out, open(sys.argv[2], "w"), indent=1)
for m in out:
    print(m)
    for k, v in out[m].items():
        print(f"  {k:40s} {v['avg_us']:9.2f} us  x{v['launches']}")
