"""Worker for tests/test_gpu_rccl.py: ONE rank on cuda:0 with an RCCL
("nccl") default process group and a gloo side group.  The native engine's
data-parallel protocol (psvo.dist.EngineExchange + EngineGradExchange) is
forced on for the single rank (force=True: every collective runs, as
identities), so the RCCL branch runs end to end — engine callback → the
operand's HIP stream wrapped as a torch ExternalStream → all_gather_into_tensor
/ all_reduce on the query communicator or the step's → the next kernel on the
same stream — and is compared with the same protocol over gloo and with the
engine without any exchange.  Engine-step loop (look-ahead queries, dense and
row-sparse gradient exchange) and bundle_adjust_frames (keyframe poses,
look-ahead).  Results go to <out>/<mode>.pt."""
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


def engine_loop(tree, emb0, batches, dev, exchange=None, sparse=False):
    torch.manual_seed(0)
    dec = Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none").to(dev)
    emb = emb0.clone().to(dev)
    ms = map_states(tree, emb, 0.2, device=dev)
    eng = MappingEngine(ms, dec, 0.2, STEP, truncation=0.1, max_distance=10.0, criteria=CRIT, max_depth=10.0)
    if exchange is not None:
        eng.set_exchange(exchange)
        if sparse:  # the row-sparse embedding exchange (config E's), forced for this small table
            eng.grad_exchange = EngineGradExchange(eng, sparse_min_bytes=0, op="sum", group=exchange.group,
                                                   force=True)
    res = {"loss": [], "grads": [], "stats": [], "modes": []}
    seeds = [101 + 7 * i for i in range(ITERS)]
    eng.query(batches[0][0], batches[0][1], seeds[0])
    for i in range(ITERS):
        ro, rd, rgb, depth = batches[i]
        if i + 1 < ITERS:  # queued on the side stream: its collectives overlap this step's
            eng.query(batches[i + 1][0], batches[i + 1][1], seeds[i + 1])
        loss = eng.step(ro, rd, rgb, depth, seed=seeds[i], apply_adam=False)
        if eng.grad_exchange is not None:
            eng.grad_exchange()
            res["modes"].append(eng.grad_exchange.last_mode)
        res["grads"].append(eng.grad_flat.detach().cpu().clone())
        eng.adam()
        res["loss"].append(float(loss))
        res["stats"].append(list(eng.last_stats))
    torch.cuda.synchronize()
    res["emb"] = emb.cpu()
    res["dec"] = [p.detach().cpu() for p in dec.parameters()]
    eng.close()
    return res


def ba_loop(tree, emb0, scene, dev, exchange=None):
    """bundle_adjust_frames on a prepared engine (the data-parallel call
    shape bench.py uses at N > 1): 3 keyframes, 512 rays each, 3 iterations."""
    import types
    from psvo import render_helpers as RH
    from psvo.criterion import Criterion
    from psvo.pose import OptimizablePose
    torch.manual_seed(0)
    dec = Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none").to(dev)
    emb = emb0.clone().to(dev).requires_grad_(True)
    ms = map_states(tree, emb, 0.2, device=dev)
    kfs = []
    for f, T in enumerate(syn.camera_poses(scene, 3, seed=5)):
        fr = syn.SyntheticFrame(scene, T, scale=0.25, seed=11 + f, device=dev)
        fr.stamp = f
        fr.pose = OptimizablePose.from_matrix(T).to(dev)
        fr.optim = torch.optim.Adam(fr.pose.parameters(), lr=1e-3)
        fr.get_pose = fr.pose.matrix
        kfs.append(fr)
    crit = Criterion(types.SimpleNamespace(criteria={**CRIT, "sdf_truncation": 0.1}, data_specs={"max_depth": 10.0}))
    eo = torch.optim.Adam([emb], lr=5e-3)
    mo = torch.optim.Adam(dec.parameters(), lr=5e-3)
    eng = MappingEngine(ms, dec, 0.2, STEP, truncation=0.1, max_distance=10.0, criteria=CRIT, max_depth=10.0)
    calls = []  # (op, count, stream) of every collective the engine issued
    if exchange is not None:
        eng.set_exchange(exchange)
        apply = exchange.apply

        def logged(op, in_off, out_off, count, stream=None):
            calls.append((int(op), int(count), int(stream or 0)))
            return apply(op, in_off, out_off, count, stream)
        exchange.apply = logged
    losses = []
    eng.ba_loss = True  # bundle_adjust_frames' steps return their loss (recorded below)
    eng.stats_hook = None
    orig = eng.step_frames

    def spy(*a, **k):
        out = orig(*a, **k)
        losses.append(float(out))  # the engine reuses the loss buffer
        return out
    eng.step_frames = spy
    RH.bundle_adjust_frames(kfs, ms, dec, None, crit, 0.2, STEP, N_rays=512, num_iterations=ITERS, embed_optim=eo,
                            model_optim=mo, update_pose=True, engine=eng, seed_fn=lambda it: 4242 + it)
    torch.cuda.synchronize()
    out = {"loss": losses, "emb": emb.detach().cpu(),
           "dec": [p.detach().cpu() for p in dec.parameters()],
           "poses": [kf.pose.data.detach().cpu() for kf in kfs], "calls": calls}
    eng.close()
    return out


def main():
    out_dir = sys.argv[1]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    assert dist.get_world_size() == 1
    gloo = dist.new_group([0], backend="gloo")
    ws = [syn.make_workload("room0", 2, 1024, seed=11 + i) for i in range(ITERS)]
    tree = Octree()
    tree.init(ws[0].scene.grid_dim, 16, ws[0].scene.voxel_size, 8)
    tree.insert(ws[0].voxels)
    g = torch.Generator().manual_seed(0)
    emb0 = torch.randn(max(20000, tree.count_nodes()), 16, generator=g) * 0.1
    R = ws[0].rays_o.shape[1]
    batches = [(w.rays_o[0].contiguous().to(dev), w.rays_d[0].contiguous().to(dev),
                w.rgb.reshape(-1, 3).contiguous().to(dev), w.depth.reshape(-1).contiguous().to(dev)) for w in ws]
    res = {
        "single": engine_loop(tree, emb0, batches, dev),
        "gloo": engine_loop(tree, emb0, batches, dev, EngineExchange(R, device=dev, group=gloo, force=True)),
        "nccl": engine_loop(tree, emb0, batches, dev, EngineExchange(R, device=dev, force=True)),
        "nccl_sparse": engine_loop(tree, emb0, batches, dev, EngineExchange(R, device=dev, force=True), sparse=True),
        "ba_single": ba_loop(tree, emb0, ws[0].scene, dev),
        "ba_gloo": ba_loop(tree, emb0, ws[0].scene, dev, EngineExchange(1536, device=dev, group=gloo, force=True)),
        "ba_nccl": ba_loop(tree, emb0, ws[0].scene, dev, EngineExchange(1536, device=dev, force=True)),
    }
    for k, v in res.items():
        torch.save(v, os.path.join(out_dir, f"{k}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
