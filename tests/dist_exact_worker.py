"""Worker for tests/test_gpu_dist_exact.py (run under torch.distributed.run,
2 ranks sharing cuda:0 over gloo).  Each rank renders its half of a room0
batch with psvo.dist.GlobalBatch + GlobalLossSums + GradBucket("sum"), then
rank 0 renders the whole batch in one process; every rank saves what it got
to <out>/rank{r}.pt and rank 0 saves <out>/single.pt for the test to compare."""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "proud-slam_amd"))

from psvo import synthetic as syn  # noqa: E402
from psvo.criterion import Criterion  # noqa: E402
from psvo.decoder import Decoder  # noqa: E402
from psvo.dist import GlobalBatch, GlobalLossSums, GradBucket  # noqa: E402
from psvo.octree import Octree, map_states  # noqa: E402
from psvo.render_helpers import render_rays  # noqa: E402

STEP, SEED = 0.01, 77


def render(tree, emb0, ro, rd, rgb, depth, crit, batch=None):
    dev = ro.device
    torch.manual_seed(0)
    dec = Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none").to(dev)
    emb = emb0.clone().to(dev).requires_grad_(True)
    ms = map_states(tree, emb, 0.2, device=dev)
    out = render_rays(ro, rd, ms, dec, None, STEP, 0.2, 0.1, 10, 10.0, seed=SEED, return_samples=True, batch=batch)
    loss, _ = crit(out, (rgb, depth), reduce_sums=GlobalLossSums() if batch is not None else None)
    loss.backward()
    params = [emb] + list(dec.parameters())
    if batch is not None:
        GradBucket(params, op="sum").allreduce()
    smp = out["samples"]
    return {"loss": loss.detach().cpu(), "s_idx": smp.s_idx.cpu(), "s_depth": smp.s_depth.cpu(),
            "z_vals": smp.z_vals.cpu(), "rank_ray": smp.rank_ray32.cpu(), "color": out["color"].detach().cpu(),
            "depth": out["depth"].detach().cpu(), "grads": [p.grad.detach().cpu() for p in params],
            "P": smp.P, "max_steps": smp.max_steps}


def main():
    out_dir = sys.argv[1]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    w = syn.make_workload("room0", 2, 700, seed=5)  # 1400 rays: K' = ceil(R_hit / 200) > 1 slots per block
    tree = Octree()
    tree.init(256, 16, 0.2, 8)
    tree.insert(w.voxels)
    g = torch.Generator().manual_seed(0)
    emb0 = torch.randn(max(20000, tree.count_nodes()), 16, generator=g) * 0.1
    crit = Criterion(type("A", (), {"criteria": {"rgb_weight": 0.5, "depth_weight": 1.0, "sdf_weight": 5000.0,
                                                 "fs_weight": 10.0, "sdf_truncation": 0.1},
                                    "data_specs": {"max_depth": 10.0}})())
    R = w.rays_o.shape[1]
    cut = [0, 611, R]  # uneven shards
    sl = slice(cut[rank], cut[rank + 1])
    ro, rd = w.rays_o[:, sl].to(dev), w.rays_d[:, sl].to(dev)
    rgb, depth = w.rgb.reshape(-1, 3)[sl].to(dev), w.depth.reshape(-1)[sl].to(dev)
    res = render(tree, emb0, ro, rd, rgb, depth, crit, batch=GlobalBatch())
    res["ray_off"] = cut[rank]
    torch.save(res, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    if rank == 0:
        ro, rd = w.rays_o.to(dev), w.rays_d.to(dev)
        single = render(tree, emb0, ro, rd, w.rgb.reshape(-1, 3).to(dev), w.depth.reshape(-1).to(dev), crit)
        torch.save(single, os.path.join(out_dir, "single.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
