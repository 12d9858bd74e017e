"""Worker for tests/test_gpu_dist_ba.py (torch.distributed.run, 2 ranks
sharing cuda:0 over gloo).  Data-parallel bundle_adjust_frames: rank r owns
keyframes [2r, 2r + 2) of a room0 keyframe graph (frame 0, stamp 0, fixed),
each iteration samples recorded pixel picks per keyframe, and the engine
computes the union-batch loss (psvo.dist.EngineExchange), the embedding /
decoder gradients are summed over ranks, every rank steps its own keyframe
poses; the next iteration's query is queued one step ahead (look-ahead).
Rank 0 then runs one process over all 4 keyframes with the same picks and
sampler seeds.  Results go to <out>/*.pt."""
import os
import sys
import types

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "proud-slam_amd"))

from psvo import render_helpers as RH  # noqa: E402
from psvo import synthetic as syn  # noqa: E402
from psvo.criterion import Criterion  # noqa: E402
from psvo.decoder import Decoder  # noqa: E402
from psvo.dist import EngineExchange, EngineGradExchange  # noqa: E402
from psvo.engine import MappingEngine  # noqa: E402
from psvo.octree import Octree, map_states  # noqa: E402
from psvo.pose import OptimizablePose  # noqa: E402

ITERS, N_RAYS, N_FRAMES, STEP = 3, 300, 4, 0.01
CRIT = {"rgb_weight": 0.5, "depth_weight": 1.0, "sdf_weight": 5000.0, "fs_weight": 10.0, "sdf_truncation": 0.1}


class PickFrame(syn.SyntheticFrame):
    """A keyframe whose sample_rays replays recorded picks (iteration-keyed)."""
    uniform_pixel_sampling = False

    def __init__(self, scene, T, f, dev):
        super().__init__(scene, T, scale=0.25, seed=f, device=dev)
        self.f, self.calls = f, 0
        self.stamp = f
        self.pose = OptimizablePose.from_matrix(T).to(dev)
        self.optim = torch.optim.Adam(self.pose.parameters(), lr=1e-3)
        self.get_pose = self.pose.matrix

    def sample_rays(self, n):
        g = torch.Generator().manual_seed(1000 * self.f + self.calls)
        self.calls += 1
        idx = torch.randperm(self.h * self.w, generator=g)[:n].sort().values.to(self.depth.device)
        m = torch.zeros(self.h * self.w, dtype=torch.bool, device=self.depth.device)
        m[idx] = True
        self.sample_mask = m.view(self.h, self.w)
        self.sample_idx = idx


def run(scene, tree, emb0, frames_ids, dev, exchange=None, sparse=False):
    torch.manual_seed(0)
    dec = Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none").to(dev)
    emb = emb0.clone().to(dev).requires_grad_(True)
    ms = map_states(tree, emb, scene.voxel_size, device=dev)
    poses = syn.camera_poses(scene, N_FRAMES, seed=31)
    kfs = [PickFrame(scene, poses[f], f, dev) for f in frames_ids]
    crit = Criterion(types.SimpleNamespace(criteria=dict(CRIT), data_specs={"max_depth": 10.0}))
    eo = torch.optim.Adam([emb], lr=5e-3)
    mo = torch.optim.Adam(dec.parameters(), lr=5e-3)
    eng = MappingEngine(ms, dec, scene.voxel_size, STEP, truncation=0.1, max_distance=10.0, criteria=CRIT,
                        max_depth=10.0, lr_emb=5e-3, lr_dec=5e-3)
    if exchange is not None:
        eng.set_exchange(exchange)
        # sparse: the row-sparse embedding exchange (config E's) forced on this small table
        eng.grad_exchange = EngineGradExchange(eng, op="sum", sparse_min_bytes=0 if sparse else 32 << 20)
    losses = []
    eng.ba_loss = True  # bundle_adjust_frames' steps return their loss (recorded below)
    orig = eng.step_frames

    def spy(*a, **k):
        out = orig(*a, **k)
        losses.append(float(out))
        return out

    eng.step_frames = spy
    RH.bundle_adjust_frames(kfs, ms, dec, None, crit, scene.voxel_size, STEP, N_rays=N_RAYS, num_iterations=ITERS,
                            embed_optim=eo, model_optim=mo, update_pose=True, engine=eng,
                            seed_fn=lambda it: 7777 + it)
    torch.cuda.synchronize()
    res = {"loss": losses, "emb": emb.detach().cpu(), "dec": [p.detach().cpu() for p in dec.parameters()],
           "poses": {f: kf.pose.data.detach().cpu() for f, kf in zip(frames_ids, kfs)},
           "modes": [] if eng.grad_exchange is None else [eng.grad_exchange.last_mode],
           "flags": None if eng.row_flags is None else eng.row_flags.cpu()}
    eng.close()
    return res


def main():
    out_dir = sys.argv[1]
    sparse = len(sys.argv) > 2 and sys.argv[2] == "sparse"
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    scene = syn.room0()
    tree = Octree()
    tree.init(scene.grid_dim, 16, scene.voxel_size, 8)
    tree.insert(syn.surface_voxels(scene, seed=0))
    emb0 = torch.randn(max(20000, tree.count_nodes()), 16, generator=torch.Generator().manual_seed(5)) * 0.1
    per = N_FRAMES // world
    mine = list(range(rank * per, (rank + 1) * per))
    res = run(scene, tree, emb0, mine, dev, EngineExchange(N_FRAMES * N_RAYS, device=dev), sparse=sparse)
    torch.save(res, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    if rank == 0:
        if sparse:
            os.environ["PSVO_SPARSE_ADAM"] = "0"  # the reference: one process, dense Adam on every row
        torch.save(run(scene, tree, emb0, list(range(N_FRAMES)), dev), os.path.join(out_dir, "single.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
