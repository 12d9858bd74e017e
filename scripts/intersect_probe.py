"""Diagnostic: the engine's intersect (k_intersect_sorted<packed> +
k_ray_stats_rank, the PSVO_TIME_INTERSECT region, serialised timing) on a
bench scene: ms per step, AABB tests and traversal rounds per ray
(PSVO_STAT_VISITS / PSVO_STAT_ROUNDS).  Usage: intersect_probe.py [scene]"""
import os
import sys
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "proud-slam_amd"))
import bench  # noqa: E402


def main():
    scene_name = sys.argv[1] if len(sys.argv) > 1 else "room0"
    args = types.SimpleNamespace(scene=scene_name, width=128, frames=4, rays_per_frame=1024)
    dev = torch.device("cuda")
    scene, tree, ms, emb, dec = bench.build_scene(args, dev, 0)
    kfs = bench.build_keyframes(args, scene, dev, 0)
    batches = bench.keyframe_batches(kfs, args.rays_per_frame, 4)
    from psvo.engine import MappingEngine
    step = {"room0": 0.0142, "multiroom": 0.0147}.get(scene_name, 0.015)
    eng = MappingEngine(ms, dec, scene.voxel_size, step, truncation=0.1, max_distance=10.0,
                        criteria={"rgb_weight": 0.5, "depth_weight": 1.0, "sdf_weight": 5000.0, "fs_weight": 10.0},
                        max_depth=10.0)
    for it in range(3):
        b = batches[it % len(batches)]
        eng.step(b[0][0], b[1][0], b[2][0], b[3][0], seed=it)
    eng.set_timing(True)
    vis = rounds = hits = 0
    n = 20
    for it in range(n):
        b = batches[it % len(batches)]
        eng.step(b[0][0], b[1][0], b[2][0], b[3][0], seed=100 + it)
        st = eng.last_stats
        vis += st[5]
        rounds += st[12]
        hits += st[1]
    torch.cuda.synchronize()
    t = eng.timing()
    R = b[0].shape[1]
    print(f"{scene_name}: intersect region {t['intersect'] * 1e3:.1f} us, sample {t['sample'] * 1e3:.1f} us, "
          f"AABB tests/ray {vis / n / R:.1f}, rounds/ray {rounds / n / R:.2f}, hit rays {hits / n:.0f} of {R}")
    eng.close()


if __name__ == "__main__":
    main()
