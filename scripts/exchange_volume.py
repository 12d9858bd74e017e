"""Data-parallel exchange volume per rank and step: embedding rows
one engine step touches (= rows SparseRowSum sends) vs the dense table a flat
all-reduce moves, on the bench's synthetic scenes."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "proud-slam_amd"))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="multiroom")
    a = ap.parse_args()
    args = bench.parse.__wrapped__() if hasattr(bench.parse, "__wrapped__") else None
    sys.argv = [sys.argv[0], "--scene", a.scene, "--pool", "2"]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    scene, tree, ms, emb, dec, batches = bench.build_scene(args, dev, 0)
    step_size, spr = bench.calibrate_step(ms, batches, args.samples_per_ray, scene.voxel_size)
    from psvo.engine import MappingEngine
    crit = {"rgb_weight": 0.5, "depth_weight": 1.0, "sdf_weight": 5000.0, "fs_weight": 10.0, "sdf_truncation": 0.1}
    eng = MappingEngine(ms, dec, scene.voxel_size, step_size, truncation=0.1, max_distance=10.0, criteria=crit,
                        max_depth=10.0, lr_emb=5e-3, lr_dec=5e-3)
    out = []
    for i, (ro, rd, rgb, depth) in enumerate(batches):
        eng.step(ro, rd, rgb, depth, seed=i, apply_adam=False)
        n = emb.shape[0]
        g = eng.grad_flat[: n * 16].view(n, 16)
        touched = int((g != 0).any(1).sum())
        out.append({"rows": n, "touched_rows": touched, "dense_bytes": n * 64,
                    "sparse_bytes_per_rank": touched * 68, "samples_per_hit_ray": spr})
    res = {"scene": a.scene, "nodes": tree.count_nodes(), "steps": out}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
