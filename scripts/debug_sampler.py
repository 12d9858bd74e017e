"""Fused query path stage by stage on a golden fixture, synchronising and
printing after every launch (GPU debugging aid; run under `timeout`)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "proud-slam_amd"))
from psvo import _lib as L  # noqa: E402
from psvo.render_helpers import query_samples  # noqa: E402
from psvo.voxel_helpers import _intersect_sorted  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "A_voxels_center"
    g = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"))
    dev = "cuda"
    ro = torch.from_numpy(g["rays_o"]).to(dev)
    rd = torch.from_numpy(g["rays_d"]).to(dev)
    centres = torch.from_numpy(g["centres"]).to(dev)
    structure = torch.from_numpy(g["structure"]).to(dev)
    step = float(g["step_size"])
    print("intersect ...", flush=True)
    q = _intersect_sorted(ro, rd, centres, structure, float(g["voxel_size"]), float(g["max_distance"]), step)
    torch.cuda.synchronize()
    print("stats", q["stats"].cpu().tolist(), flush=True)
    ms = {"voxel_center_xyz": centres, "voxel_structure": structure}
    smp = query_samples(ro, rd, ms, step, float(g["voxel_size"]), float(g["max_distance"]),
                        noise=torch.from_numpy(g["noise"]))
    torch.cuda.synchronize()
    print("sampled r_hit", smp.r_hit, "s_max", smp.s_max, "m", smp.m, flush=True)
    z = smp.z_vals.cpu().numpy()
    print("z_vals match golden:", z.shape == g["z_vals"].shape and bool(np.allclose(z, g["z_vals"])), flush=True)


if __name__ == "__main__":
    main()
