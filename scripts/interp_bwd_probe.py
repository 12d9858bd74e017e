"""k_interp_bwd variants at the bench's room0 size (4 x 1024 rays, step for
~64 samples/hit ray): one wave per ray vs 64-sample units, with and without
the embedding scatter (atomics), HIP-event timed."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "proud-slam_amd"))
from psvo import _lib as L  # noqa: E402
from psvo import synthetic as syn  # noqa: E402
from psvo.octree import Octree, map_states  # noqa: E402
from psvo.render_helpers import query_samples  # noqa: E402


def timed(fn, n=30):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1000.0


def main():
    w = syn.make_workload("room0", 4, 1024, seed=0)
    tree = Octree()
    tree.init(256, 16, 0.2, 8)
    tree.insert(w.voxels)
    emb = (torch.randn(max(20000, tree.count_nodes()), 16) * 0.01).cuda()
    ms = map_states(tree, emb, 0.2, device="cuda")
    ro, rd = w.rays_o.cuda(), w.rays_d.cuda()
    q = query_samples(ro, rd, ms, 0.00728, 0.2, 10.0, seed=1)
    R = ro.numel() // 3
    ns = (q.offsets[1:] - q.offsets[:-1]).float()
    print(f"r_hit {q.r_hit} M {q.m} S_max {q.s_max} mean {float(ns.mean()):.1f} p99 {float(ns.quantile(0.99)):.0f}")
    gf = torch.randn(q.m, 16, device="cuda")
    args = (q.offsets, q.rank_ray32, q.leaf, q.t, ro, rd, ms["voxel_center_xyz"], ms["voxel_vertex_idx"], emb, gf)
    ge, go, gd = torch.zeros_like(emb), torch.zeros(R, 3, device="cuda"), torch.zeros(R, 3, device="cuda")
    ws = torch.empty(int(L.lib().psvo_interp_bwd_workspace_floats(q.r_hit, q.s_max)), device="cuda")
    st = L.stream_of(torch.device("cuda"))
    res = {
        "per_ray_emb": timed(lambda: L.call("psvo_interp_bwd", st, q.r_hit, 16, 0.2, *args, ge, go, gd)),
        "per_ray_pose_only": timed(lambda: L.call("psvo_interp_bwd", st, q.r_hit, 16, 0.2, *args, None, go, gd)),
        "chunked_emb": timed(lambda: L.call("psvo_interp_bwd_chunked", st, q.r_hit, q.s_max, 16, 0.2, *args, ge, go,
                                            gd, ws)),
        "chunked_pose_only": timed(lambda: L.call("psvo_interp_bwd_chunked", st, q.r_hit, q.s_max, 16, 0.2, *args,
                                                  None, go, gd, ws)),
    }
    for k, v in res.items():
        print(f"{k:20s} {v:8.1f} us")


if __name__ == "__main__":
    main()
