"""Mesh extraction throughput (Mapping.extract_mesh →
MeshExtractor.create_mesh, res 8, require_color) on the synthetic room0 map:
SURFACE voxels per second for the device pipeline and its stages, and the
oracle's CPU restatement (torch-CPU get_scores + numpy marching cubes) on a
bounded voxel sample beside it."""
import json
import os
import sys
import time
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "proud-slam_amd"))
from psvo import synthetic as syn  # noqa: E402
from psvo.decoder import Decoder  # noqa: E402
from psvo.mesh import MeshExtractor, lattice_scores, marching_cubes_device, surface_states  # noqa: E402
from psvo.octree import Octree  # noqa: E402


def _timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps, out


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    scene = syn.room0()
    tree = Octree()
    tree.init(scene.grid_dim, 16, scene.voxel_size, 8)
    tree.insert(syn.surface_voxels(scene, seed=0))
    voxels, _, features = tree.export_arrays()
    gen = torch.Generator().manual_seed(0)
    emb = (torch.randn(voxels.shape[0], 16, generator=gen) * 0.3).cuda()
    torch.manual_seed(0)
    dec = Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none").cuda()
    sv, states = surface_states(torch.from_numpy(voxels), torch.from_numpy(features), emb, scene.voxel_size)
    n = sv.shape[0]
    vs = scene.voxel_size
    mx = MeshExtractor(types.SimpleNamespace(mapper_specs={"voxel_size": vs}))
    t_scores, _ = _timed(lambda: lattice_scores(dec, states, vs, 8), reps)
    t_sdf, (_, sdf) = _timed(lambda: lattice_scores(dec, states, vs, 8, with_rgb=False), reps)
    c = states["voxel_center_xyz"]
    t_mc, (v, f) = _timed(lambda: marching_cubes_device(c, sdf, vs, 8), reps)
    t_all, mesh = _timed(lambda: mx.create_mesh(dec, states, vs, sv, require_color=True, offset=-10, res=8), reps)
    out = {"surface_voxels": n, "lattice_points": n * 512, "vertices": int(v.shape[0]), "triangles": int(f.shape[0]),
           "ms": {"lattice_scores_rgb_sdf": 1e3 * t_scores, "lattice_sdf": 1e3 * t_sdf,
                  "marching_cubes": 1e3 * t_mc,
                  "create_mesh_with_colour": 1e3 * t_all},
           "voxels_per_s": n / t_all}
    # CPU oracle on a bounded sample
    from oracle import mesh_oracle as MO
    k = min(n, 256)
    params = {kk: vv.cpu() for kk, vv in dec.state_dict().items()}
    cc = c[:k].cpu()
    t0 = time.perf_counter()
    sc = MO.get_scores(params, cc, states["voxel_vertex_idx"][:k].cpu(), emb.cpu(), vs, 8)
    MO.marching_cubes(cc.numpy(), sc[..., 3].numpy(), vs)
    el = time.perf_counter() - t0
    out["cpu_oracle"] = {"voxels": k, "s": el, "voxels_per_s": k / el, "threads": torch.get_num_threads()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
