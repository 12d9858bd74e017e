"""Worker for tests/test_gpu_dist_engine.py (run under torch.distributed.run,
2 ranks sharing cuda:0 over gloo).  Each rank runs the native engine
(psvo_map_step) on its shard of one ray batch with psvo.dist.EngineExchange
(union-batch layout + normalisers) and sums the gradients over ranks; rank 0
then runs one engine on the whole batch.  Three iterations, the next batch's
query queued one step ahead as in bench.py.  Results go to <out>/*.pt."""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "proud-slam_amd"))

from psvo import synthetic as syn  # noqa: E402
from psvo.decoder import Decoder  # noqa: E402
from psvo.dist import EngineExchange, EngineGradExchange  # noqa: E402
from psvo.engine import MappingEngine  # noqa: E402
from psvo.octree import Octree, map_states  # noqa: E402

STEP, ITERS = 0.01, 3
CRIT = {"rgb_weight": 0.5, "depth_weight": 1.0, "sdf_weight": 5000.0, "fs_weight": 10.0}


def run(tree, emb0, batches, dev, exchange=None):
    torch.manual_seed(0)
    dec = Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none").to(dev)
    emb = emb0.clone().to(dev)
    ms = map_states(tree, emb, 0.2, device=dev)
    eng = MappingEngine(ms, dec, 0.2, STEP, truncation=0.1, max_distance=10.0, criteria=CRIT, max_depth=10.0)
    gx = None
    if exchange is not None:
        eng.set_exchange(exchange)
        gx = EngineGradExchange(eng, op="sum")
    res = {"loss": [], "grads": [], "stats": []}
    seeds = [101 + 7 * i for i in range(ITERS)]
    eng.query(batches[0][0], batches[0][1], seeds[0])
    for i in range(ITERS):
        ro, rd, rgb, depth = batches[i]
        if i + 1 < ITERS:
            eng.query(batches[i + 1][0], batches[i + 1][1], seeds[i + 1])
        loss = eng.step(ro, rd, rgb, depth, seed=seeds[i], apply_adam=False)
        if gx is not None:
            gx()
        res["grads"].append(eng.grad_flat.detach().cpu().clone())
        eng.adam()
        res["loss"].append(float(loss))
        res["stats"].append(list(eng.last_stats))
    torch.cuda.synchronize()
    res["emb"] = emb.cpu()
    res["dec"] = [p.detach().cpu() for p in dec.parameters()]
    eng.close()
    return res


def main():
    out_dir, scene, rays_per_frame, frames = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    cut0 = int(sys.argv[5])
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    ws = [syn.make_workload(scene, frames, rays_per_frame, seed=11 + i) for i in range(ITERS)]
    tree = Octree()
    tree.init(ws[0].scene.grid_dim, 16, ws[0].scene.voxel_size, 8)
    tree.insert(ws[0].voxels)
    g = torch.Generator().manual_seed(0)
    emb0 = torch.randn(max(20000, tree.count_nodes()), 16, generator=g) * 0.1
    R = ws[0].rays_o.shape[1]
    cut = [0, cut0, R]
    sl = slice(cut[rank], cut[rank + 1])

    def part(w, s):
        return (w.rays_o[0, s].contiguous().to(dev), w.rays_d[0, s].contiguous().to(dev),
                w.rgb.reshape(-1, 3)[s].contiguous().to(dev), w.depth.reshape(-1)[s].contiguous().to(dev))

    shard = [part(w, sl) for w in ws]
    res = run(tree, emb0, shard, dev, EngineExchange(R, device=dev))
    torch.save(res, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    if rank == 0:
        whole = [part(w, slice(0, R)) for w in ws]
        torch.save(run(tree, emb0, whole, dev), os.path.join(out_dir, "single.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
