"""Octree build + export: CPU builder (psvo.octree.Octree + map_states + H2D)
against the device builder (DeviceOctree + render arrays), per scene."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "proud-slam_amd"))
from psvo import synthetic as syn  # noqa: E402
from psvo.octree import DeviceOctree, Octree, map_states  # noqa: E402


def main():
    out = {}
    for name in sys.argv[1:] or ["room0", "multiroom"]:
        scene = {"room0": syn.room0, "multiroom": syn.multiroom}[name]()
        vox = syn.surface_voxels(scene, seed=0)
        emb = torch.zeros(1, device="cuda")
        t0 = time.perf_counter()
        cpu = Octree()
        cpu.init(scene.grid_dim, 16, scene.voxel_size, 8)
        cpu.insert(vox)
        ms = map_states(cpu, emb, scene.voxel_size, device="cuda")
        torch.cuda.synchronize()
        t_cpu = time.perf_counter() - t0
        vd = torch.from_numpy(vox).cuda()
        for rep in range(3):  # first call pays allocation / module load
            dev = DeviceOctree("cuda")
            dev.init(scene.grid_dim, 16, scene.voxel_size, 8, capacity=2 * len(vox) * 3)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            dev.insert(vd)
            t_ins = time.perf_counter() - t0
            msd = map_states(dev, emb, scene.voxel_size)
            torch.cuda.synchronize()
            t_dev = time.perf_counter() - t0
        same = all(torch.equal(ms[k], msd[k]) for k in ("voxel_center_xyz", "voxel_structure", "voxel_vertex_idx"))
        out[name] = {"voxels": int(len(vox)), "nodes": cpu.count_nodes(), "cpu_build_export_h2d_s": t_cpu,
                     "device_build_export_s": t_dev, "device_insert_s": t_ins, "speedup": t_cpu / t_dev, "identical": same}
        print(json.dumps({name: out[name]}), flush=True)


if __name__ == "__main__":
    main()
