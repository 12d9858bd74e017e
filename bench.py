"""Benchmark: rays/s for render + loss + backward (+ optimiser step) of the
Proud-SLAM mapping render-and-optimise iteration (render_helpers.py:609-676)
on synthetic Replica room0-shaped input (BASELINE.json configs[1]: 4096
rays/iter = 4 keyframes x 1024 rays, 1x MI355X; ~64 samples/ray).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One process per GPU; every rank renders its own 4096 rays against the
replicated octree (weak scaling) and the embedding + decoder gradients are
summed over ranks with one RCCL all-reduce per step.  Rank 0 prints one JSON
line.  Inputs (octree, embeddings, decoder, a pool of ray batches with GT)
are resident in HBM before timing starts.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "proud-slam_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "rays/sec render+backward, Replica room0, 64 samples/ray, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md: aggregate L2 (8 x 4 MiB) ≈34.5 TB/s
MFMA_F32_PEAK_TFS = 157.3  # MI355X_MICROARCH.md: f32-input MFMA (v_mfma_f32_32x32x2_f32) dense peak


def log(msg):
    """Progress on stderr (setup of the large scenes takes minutes)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--scene", default="room0")
    ap.add_argument("--frames", type=int, default=None,
                    help="keyframes x rays-per-frame = rays per iteration per GPU (default: 8 for scannet0000, else 4)")
    ap.add_argument("--rays-per-frame", type=int, default=1024)
    ap.add_argument("--width", type=int, default=None,
                    help="decoder width (default: the scene's config — 256 for scannet0000 / multiroom (ARKit), "
                         "else 128)")
    ap.add_argument("--samples-per-ray", type=float, default=64.0)
    ap.add_argument("--pool", type=int, default=8, help="distinct ray batches cycled through")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--path", choices=("ba", "step", "autograd"), default="ba",
                    help="headline: ba = the reference's bundle_adjust_frames API (keyframe poses optimised too; "
                         "dispatches to the native engine), step = the engine's psvo_map_step on pre-built "
                         "world-space ray batches, autograd = render_rays + Criterion + backward + Adam")
    ap.add_argument("--autograd", action="store_true", help="same as --path autograd")
    ap.add_argument("--exact-global-loss", action="store_true",
                    help="(kept for compatibility: N>1 always computes the union-batch loss)")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic.json"))
    a = ap.parse_args()
    if a.autograd:
        a.path = "autograd"
    a.autograd = a.path == "autograd"
    big = a.scene in ("scannet0000", "multiroom")  # configs/scannet/scannet.yaml:17, configs/arkit/arkit.yaml:17
    if a.width is None:
        a.width = 256 if big else 128
    if a.frames is None:
        a.frames = 8 if a.scene == "scannet0000" else 4
    return a


# per-scene Criterion / data specs (configs/replica/replica.yaml, configs/scannet/scannet.yaml:8-13)
SCENE_CRITERIA = {
    "scannet0000": ({"rgb_weight": 1.0, "depth_weight": 1.0, "sdf_weight": 5000.0, "fs_weight": 10.0,
                     "sdf_truncation": 0.1}, 5.0),
}
DEFAULT_CRITERIA = ({"rgb_weight": 0.5, "depth_weight": 1.0, "sdf_weight": 5000.0, "fs_weight": 10.0,
                     "sdf_truncation": 0.1}, 10.0)


def launch_workers(args):
    """`python bench.py --gpus N` (N > 1) without a torch.distributed launcher:
    start N ranks under torch.distributed.run as a child process (this parent
    never touches the GPU) and exit with its status."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1:
        # RCCL over xGMI; PSVO_DIST_BACKEND=gloo rehearses the N>1 path with
        # several ranks sharing one GPU (the device index wraps around)
        backend = os.environ.get("PSVO_DIST_BACKEND", "nccl")
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, local


def build_scene(args, device, rank):
    from psvo import synthetic as syn
    from psvo.octree import Octree, map_states
    from psvo.decoder import Decoder
    scene_fn = {"room0": syn.room0, "office0": syn.office0, "scannet0000": syn.scannet0000,
                "multiroom": syn.multiroom}[args.scene]
    scene = scene_fn()
    vox = syn.surface_voxels(scene, seed=0)
    tree = Octree()
    tree.init(scene.grid_dim, 16, scene.voxel_size, 8)
    tree.insert(vox)
    n_nodes = tree.count_nodes()
    num_embeddings = max(20000, n_nodes)  # replica.yaml:38 num_embeddings
    g = torch.Generator().manual_seed(0)
    emb = (torch.randn(num_embeddings, 16, generator=g) * 0.01).to(device).requires_grad_(True)  # mapping.py:80
    ms = map_states(tree, emb, scene.voxel_size, device=device)
    torch.manual_seed(0)
    dec = Decoder(depth=2, width=args.width, in_dim=16, skips=[], embedder="none").to(device)
    return scene, tree, ms, emb, dec


def build_keyframes(args, scene, device, rank):
    """This rank's keyframes: full-resolution synthetic RGB-D frames with
    their own poses (optimised by bundle_adjust_frames, lr 1e-3, frame.py:27)."""
    from psvo.pose import OptimizablePose
    from psvo.synthetic import SyntheticFrame, camera_poses
    out = []
    for f, T in enumerate(camera_poses(scene, args.frames, seed=1000 * rank + 77)):
        fr = SyntheticFrame(scene, T, scale=1.0, seed=7 * (rank * args.frames + f) + 1, device=device)
        fr.stamp = rank * args.frames + f  # the union batch's first keyframe (stamp 0) keeps its pose
        fr.pose = OptimizablePose.from_matrix(T).to(device)
        fr.optim = torch.optim.Adam(fr.pose.parameters(), lr=1e-3)
        fr.get_pose = fr.pose.matrix
        out.append(fr)
    return out


def keyframe_batches(kfs, n_per_frame, count):
    """`count` world-space ray batches as bundle_adjust_frames assembles them
    (render_helpers.py:620-633): n_per_frame gumbel-top-k pixels per keyframe,
    rays_d = dirs @ Rᵀ, rays_o = t, with the frames' rgb / depth — the pool the
    engine-step path cycles through, and the step-size calibration sample."""
    from psvo import sample_util
    out = []
    with torch.no_grad():
        for i in range(count):
            d, c, z = sample_util.sample_frames(kfs, n_per_frame, seed=7919 * i + 13)
            ro, rd = [], []
            for f, kf in enumerate(kfs):
                T = kf.get_pose()
                sl = slice(f * n_per_frame, (f + 1) * n_per_frame)
                rd.append(d[sl] @ T[:3, :3].transpose(0, 1))
                ro.append(T[:3, 3].reshape(1, 3).expand(n_per_frame, 3))
            out.append((torch.cat(ro).unsqueeze(0).contiguous(), torch.cat(rd).unsqueeze(0).contiguous(),
                        c.unsqueeze(0).contiguous(), z.unsqueeze(0).contiguous()))
    return out


def calibrate_step(ms, batches, target, voxel_size, world=1):
    """step_size so that the mean valid samples per hit ray ≈ target (SURVEY
    §8d), over the union of all ranks' batches."""
    from psvo.render_helpers import query_samples

    def mean_samples(step):
        # pooled over every batch the timed loop cycles through, so the timed
        # workload (not just batch 0) averages `target` samples per hit ray
        m = r = 0
        for i, b in enumerate(batches):
            s = query_samples(b[0], b[1], ms, step, voxel_size, 10.0, seed=1 + i)
            m += s.m
            r += s.r_hit
        if world > 1:
            t = torch.tensor([m, r], dtype=torch.float64, device=b[0].device)
            dist.all_reduce(t)
            m, r = float(t[0]), float(t[1])
        return m / r
    lo, hi = 0.001, 0.05
    for _ in range(18):
        mid = math.sqrt(lo * hi)
        if mean_samples(mid) > target:
            lo = mid
        else:
            hi = mid
    step = math.sqrt(lo * hi)
    return step, mean_samples(step)


class KernelTimer:
    """HIP events around chosen launches on the launching stream."""

    def __init__(self):
        self.events = {}
        self.enabled = False

    def __call__(self, name):
        timer = self

        class _Ctx:
            def __enter__(self_):
                if timer.enabled:
                    s = torch.cuda.Event(enable_timing=True)
                    s.record(torch.cuda.current_stream())
                    self_.s = s

            def __exit__(self_, *exc):
                if timer.enabled:
                    e = torch.cuda.Event(enable_timing=True)
                    e.record(torch.cuda.current_stream())
                    timer.events.setdefault(name, []).append((self_.s, e))
        return _Ctx()

    def mean_ms(self, name):
        ev = self.events.get(name, [])
        if not ev:
            return float("nan")
        return float(np.mean([s.elapsed_time(e) for s, e in ev]))


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _physical_cores():
    """Distinct (physical id, core id) pairs of /proc/cpuinfo: the host's physical cores."""
    cores, phys = set(), None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                phys = line.split(":", 1)[1].strip()
            elif line.startswith("core id"):
                cores.add((phys, line.split(":", 1)[1].strip()))
    except OSError:
        return None
    return len(cores) or None


def cpu_baseline(args, scene, tree, step_size, seconds):
    """Oracle (reference algorithm restated: C kernels + torch-CPU render /
    loss / autograd) on the host cores, bounded sample of the same workload."""
    from oracle import oracle as O
    from psvo import synthetic as syn
    voxels, children, features = tree.export_arrays()
    g = torch.Generator().manual_seed(0)
    emb = torch.randn(voxels.shape[0], 16, generator=g) * 0.01
    ms = O.map_states_from_export(voxels, children, features, scene.voxel_size, emb)
    params = O.decoder_params_init(args.width)
    poses = syn.camera_poses(scene, args.frames, seed=0)
    ro, rd, rgb, depth = syn.rays_for_frames(scene, poses, args.rays_per_frame, seed=0)
    t0 = time.time()
    n_it = 0
    while True:
        O.render_and_backward(ro, rd, rgb, depth, ms, params, step_size, scene.voxel_size,
                              generator=torch.Generator().manual_seed(n_it))
        n_it += 1
        if time.time() - t0 >= seconds or n_it >= 50:
            break
    dt = time.time() - t0
    rays = n_it * ro.shape[1]
    return {"value": rays / dt, "unit": "rays/s", "cores": int(torch.get_num_threads()), "kind": "port",
            "cpu_model": _cpu_model(), "host_physical_cores": _physical_cores(), "host_logical_cpus": os.cpu_count(),
            "process_cpu_share": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
            "sample": f"{n_it} iterations x {ro.shape[1]} rays ({args.scene}, {args.frames}x{args.rays_per_frame}), "
                      f"oracle C kernels (OpenMP over rays) + torch-CPU render/loss/backward, "
                      f"{torch.get_num_threads()} threads, {dt:.1f}s"}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_workers(args))
    world, rank, local = setup_dist(args)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    from psvo import _lib
    from psvo import render_helpers as RH
    from psvo.criterion import Criterion
    import types
    _lib.lib()

    log(f"scene {args.scene}: octree, embeddings, decoder W={args.width}")
    scene, tree, ms, emb, dec = build_scene(args, device, rank)
    log(f"{args.frames} keyframes ({tree.count_nodes()} octree nodes)")
    kfs = build_keyframes(args, scene, device, rank)
    batches = keyframe_batches(kfs, args.rays_per_frame, args.pool)
    log("step-size calibration")
    step_size, spr = calibrate_step(ms, batches, args.samples_per_ray, scene.voxel_size, world)
    log(f"step {step_size:.5f} m, {spr:.1f} samples / hit ray; timing the {args.path} path")
    crit_cfg, max_depth = SCENE_CRITERIA.get(args.scene, DEFAULT_CRITERIA)
    crit_args = types.SimpleNamespace(criteria=dict(crit_cfg), data_specs={"max_depth": max_depth})
    criterion = Criterion(crit_args)
    from psvo.optim import Adam  # torch.optim.Adam semantics, one HIP launch per step per optimiser
    embed_optim = Adam([emb], lr=5e-3)
    model_optim = Adam(dec.parameters(), lr=5e-3)
    params = [emb] + list(dec.parameters())
    timer = KernelTimer()
    _lib.KERNEL_TIMER = timer
    stats = {"n": 0, "m": 0, "r_hit": 0, "visits": 0, "s_max": 0}  # the marked (breakdown) runs
    head_stats = dict(stats)  # the headline bundle_adjust_frames iterations

    from psvo.dist import GlobalBatch, GlobalLossSums, GradBucket
    from psvo.engine import MappingEngine
    # N > 1: both paths form the loss of the union of the ranks' rays (global
    # sampler layout and normalisers) and sum the gradients with one flat
    # all-reduce per step
    bucket = GradBucket(params, op="sum")
    reducer = GlobalLossSums() if world > 1 else None
    gbatch = GlobalBatch() if world > 1 else None
    engine = MappingEngine(ms, dec, scene.voxel_size, step_size, truncation=0.1, max_distance=10.0,
                           criteria=crit_args.criteria, max_depth=max_depth, lr_emb=5e-3, lr_dec=5e-3)
    from psvo.dist import EngineExchange, EngineGradExchange
    if world > 1:
        # the loss of the union of all ranks' rays: union-batch
        # sampler layout and normalisers, gradients summed over ranks
        engine.set_exchange(EngineExchange(args.frames * args.rays_per_frame * world, device=device))
    exchange = EngineGradExchange(engine, op="sum")

    def record_stats(m, r_hit, visits, s_max, into=None):
        sd = stats if into is None else into
        sd["n"] += 1
        sd["m"] += m
        sd["r_hit"] += r_hit
        sd["visits"] += visits
        sd["s_max"] = max(sd["s_max"], s_max)

    def step_autograd(i, record=False):
        """The drop-in path: render_rays + Criterion + backward + Adam steps."""
        ro, rd, rgb, depth = batches[i % len(batches)]
        out = RH.render_rays(ro, rd, ms, dec, None, step_size, scene.voxel_size, 0.1, 10, 10.0, return_samples=True,
                             seed=7919 * i + 1, batch=gbatch)
        loss, _ = criterion(out, (rgb, depth), reduce_sums=reducer)
        embed_optim.zero_grad()  # set_to_none, as optim.zero_grad() in render_helpers.py:668
        model_optim.zero_grad()
        loss.backward()
        if world > 1:
            bucket.allreduce()
        embed_optim.step()
        model_optim.step()
        if record:
            s = out["samples"]
            record_stats(s.m, s.r_hit, s.visits, s.s_max)
        return loss

    eng_it = [0]  # engine iterations so far: the next batch is always the one already queued

    def eng_batch(it):
        # one seed for all ranks: the sampler noise is keyed by the union batch's logical row
        return batches[it % len(batches)], 1000003 + it

    def step_engine(i, record=False):
        """The same iteration as one native call (psvo_map_step); the next
        batch's ray query is queued first (psvo_map_query, side stream: it
        reads only rays + octree, so it overlaps this step).  With N > 1 the
        flat gradient bucket is all-reduced (RCCL) before the Adam steps."""
        it = eng_it[0]
        eng_it[0] += 1
        (ro, rd, rgb, depth), seed = eng_batch(it)
        if not engine._queued:
            engine.query(ro, rd, seed)
        (nro, nrd, _, _), nseed = eng_batch(it + 1)
        engine.query(nro, nrd, nseed)
        loss = engine.step(ro, rd, rgb, depth, seed=seed, apply_adam=(world == 1))
        if world > 1:
            exchange()  # flat RCCL all-reduce (row-sparse exchange for ≥ 32 MB tables), mean over ranks
            engine.adam()
        if record:
            st = engine.last_stats
            record_stats(st[4], st[9] if world > 1 else st[1], st[5], st[3])  # this rank's hit rays
        return loss

    def run(step_fn, steps, warmup, timed_hook=None):
        for i in range(warmup):
            step_fn(i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        if timed_hook:
            timed_hook(True)
        t0 = time.perf_counter()
        for i in range(steps):
            step_fn(warmup + i, record=timed_hook is not None)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if timed_hook:
            timed_hook(False)
        if world > 1:
            t = torch.tensor([el], device=device, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    # ---- bundle_adjust_frames (the reference's mapping API, render_helpers.py:
    # 559-676): this rank's keyframes — full-resolution synthetic RGB-D frames
    # with their own poses (optimised, lr 1e-3, frame.py:27) — each iteration
    # samples rays_per_frame pixels per keyframe (gumbel top-k on the device),
    # renders, back-propagates and steps every optimiser.  K steps = one call
    # with num_iterations = K (how Mapping calls it).
    ba_calls = [0]

    def run_ba(steps):
        engine.discard_queued()  # a look-ahead query of the engine-step runs
        call = ba_calls[0]
        ba_calls[0] += 1
        RH.bundle_adjust_frames(kfs, ms, dec, None, criterion, scene.voxel_size, step_size,
                                N_rays=args.rays_per_frame, num_iterations=steps, embed_optim=embed_optim,
                                model_optim=model_optim, update_pose=True, engine=engine,
                                seed_fn=lambda it: 1000003 * (call + 1) + it)  # same on every rank

    def timed_ba(steps, warmup, record=False):
        if warmup:
            run_ba(warmup)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        if record:
            engine.stats_hook = lambda st: record_stats(st[4], st[9] if world > 1 else st[1], st[5], st[3],
                                                        head_stats)
        run_ba(steps)
        engine.stats_hook = None
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], device=device, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    # the headline steps run without HIP-event markers (each costs a few µs of
    # GPU idle); the per-region breakdown comes from separate marked runs of
    # the engine step (pre-built ray batches, the same kernels)
    n_mark = max(5, min(args.steps, 20))
    kt_overlap = None
    others = []
    if args.path == "ba":
        elapsed = timed_ba(args.steps, args.warmup, record=True)
        path_desc = ("bundle_adjust_frames (drop-in API: per-iteration gumbel pixel sampling on the device, "
                     "keyframe poses optimised; dispatched to psvo_map_step_frames)")
    elif args.path == "autograd":
        elapsed = run(step_autograd, args.steps, args.warmup)
        path_desc = "drop-in autograd (render_rays + Criterion + backward + psvo.optim.Adam)"
    else:
        elapsed = run(step_engine, args.steps, args.warmup)
        path_desc = "native engine (psvo_map_step on pre-built world-space ray batches, next query one step ahead)"
    if args.path == "autograd":
        timer.enabled = True
        run(step_autograd, n_mark, 0, lambda on: None)
        timer.enabled = False
        kt = {k: timer.mean_ms(k) for k in MappingEngine.REGIONS}
    else:
        engine.set_timing(True)      # regions serialised on one stream
        run(step_engine, n_mark, 2, lambda on: None)
        kt = engine.timing()
        engine.set_timing("overlap")  # the same regions as the headline steps run them
        run(step_engine, n_mark, 0)
        kt_overlap = engine.timing()
        engine.set_timing(False)
    # the other paths, for reference (not the headline number)
    other_steps = max(5, min(args.steps, 20))
    rays_step = args.frames * args.rays_per_frame
    if world == 1:
        if args.path != "step":
            el2 = run(step_engine, other_steps, 2)
            others.append({"path": "native engine step (psvo_map_step, fixed poses, pre-built rays)",
                           "value": rays_step * other_steps / el2, "ms_per_step": 1000.0 * el2 / other_steps})
        if args.path != "autograd":
            el2 = run(step_autograd, other_steps, 2)
            others.append({"path": "drop-in autograd (render_rays + Criterion + backward + psvo.optim.Adam)",
                           "value": rays_step * other_steps / el2, "ms_per_step": 1000.0 * el2 / other_steps})
        if args.path != "ba":
            el2 = timed_ba(other_steps, 2)
            others.append({"path": "bundle_adjust_frames (native engine, poses optimised)",
                           "value": rays_step * other_steps / el2, "ms_per_step": 1000.0 * el2 / other_steps})
    other = others if others else {"path": "not run at N > 1 (the headline path only)"}
    rays_per_step = args.frames * args.rays_per_frame
    total_rays = rays_per_step * args.steps * world
    value = total_rays / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps

    # Rooflines.  Primary — the north star's "octree query+interp
    # kernel": algorithmic bytes per step = per ray 24 B + 48 B per AABB-tested
    # node (V counted by the kernel) + per valid sample 12 B (sampler output)
    # + 628 B (interp fwd) + 1,664 B (interp bwd), over the summed HIP-event
    # time of its launches (intersect + stats + hit rank, sampler + scan,
    # sample compaction, interp fwd, interp bwd).  Three fractions: the
    # algorithmic bytes against HBM (the contract's `frac`; > 1 would mean the
    # gathers are served from L2, and the bound is then reported as L2), the
    # same against the L2's ≈34.5 TB/s, and the PMC-counted HBM bytes
    # (FETCH_SIZE x 2 + WRITE_SIZE, profiles/traffic.json) against HBM.  Times
    # from the serialised marked run (`time_ms`) and as the headline steps
    # overlap them (`time_ms_overlapped`).  Secondary — the decoder (dominant
    # by time): fwd, δ chain and weight gradients are each W-dependent MACs per
    # sample (3 x 2 x MACs FLOP/sample), MFMA-bound.
    n_rec = max(stats["n"], 1)
    m_avg = stats["m"] / n_rec
    r_avg = stats["r_hit"] / n_rec
    v_avg = stats["visits"] / n_rec
    # the headline workload: the timed bundle_adjust_frames iterations' own
    # statistics (else the marked runs', which replay the headline's batches)
    hs = head_stats if head_stats["n"] else stats
    h_n = max(hs["n"], 1)
    h_m, h_r, h_v = hs["m"] / h_n, hs["r_hit"] / h_n, hs["visits"] / h_n
    if world > 1:  # per-GPU averages over the union of the ranks' batches (the calibration's population)
        t = torch.tensor([h_m, h_r, h_v], dtype=torch.float64, device=device)
        dist.all_reduce(t)
        h_m, h_r, h_v = (float(x) / world for x in t.cpu())
    q_keys = ("intersect", "sample", "points", "interp_fwd", "interp_bwd")
    q_parts = {k: kt[k] for k in q_keys}
    q_ms = sum(q_parts.values())
    q_ms_ov = sum(kt_overlap[k] for k in q_keys) if kt_overlap else None
    bytes_query = rays_step * 24.0 + v_avg * 48.0 + m_avg * 12.0
    bytes_qi = bytes_query + m_avg * (628.0 + 1664.0)
    traffic = {}
    if os.path.exists(args.traffic_json):
        try:
            traffic = json.load(open(args.traffic_json))
        except Exception:
            traffic = {}
        if traffic.get("scene", "room0") != args.scene:  # PMC passes of another scene: not this workload's bytes
            traffic = {}

    def bw_roof(kernel, alg_bytes, ms, ms_ov, counter_bytes, extra=None):
        gbs = alg_bytes / (ms * 1e-3) / 1e9 if ms and ms > 0 else None
        frac_hbm = gbs / HBM_PEAK_GBS if gbs else None
        bound, peak = ("hbm", HBM_PEAK_GBS) if (frac_hbm is None or frac_hbm <= 1.0) else ("l2", L2_PEAK_GBS)
        r = {"kernel": kernel, "bound": bound, "achieved": gbs, "peak": peak, "unit": "GB/s",
             "frac": gbs / peak if gbs else None, "traffic": counter_bytes,
             "algorithmic_bytes_per_launch": alg_bytes, "avg_launch_ms": ms, "time_ms_overlapped": ms_ov,
             "frac_hbm_algorithmic": frac_hbm,
             "frac_l2_algorithmic": gbs / L2_PEAK_GBS if gbs else None,
             "frac_hbm_counters": (counter_bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if (counter_bytes and ms) else None,
             "frac_hbm_algorithmic_overlapped": (alg_bytes / (ms_ov * 1e-3) / 1e9 / HBM_PEAK_GBS)
             if ms_ov and ms_ov > 0 else None}
        if extra:
            r.update(extra)
        for k, v in r.items():
            if k.startswith("frac") and v is not None and k != "frac_hbm_algorithmic" and \
                    k != "frac_hbm_algorithmic_overlapped":
                assert v <= 1.0, (kernel, k, v)
        return r

    roof_qi = bw_roof("octree query+interp (k_intersect_sorted+k_ray_stats_rank, k_sample_fused+k_scan_samples, "
                      "k_sample_points, k_interp_fwd, k_interp_bwd)", bytes_qi, q_ms, q_ms_ov,
                      traffic.get("query_interp_bytes_per_step"),
                      {"parts_ms": q_parts, "parts_ms_overlapped": {k: kt_overlap[k] for k in q_keys}
                       if kt_overlap else None, "visits_per_ray": v_avg / max(rays_step, 1),
                       "samples_per_hit_ray": m_avg / max(r_avg, 1)})
    roof_ib = bw_roof("k_interp_bwd", 1664.0 * m_avg, kt["interp_bwd"],
                      kt_overlap["interp_bwd"] if kt_overlap else None,
                      traffic.get("interp_bwd_bytes_per_launch"))
    mlp_f_ms, mlp_b_ms = kt["mlp_fwd"], kt["mlp_bwd"]
    mlp_ms = mlp_f_ms + mlp_b_ms
    w = args.width
    macs = 16 * w + w * w + w * 129 + 144 * w + w * 3  # nrgbd.py:80-146, depth 2, sdf_dim 128, in_dim 16
    flops_mlp = 3 * 2.0 * macs * m_avg
    mlp_tf = flops_mlp / (mlp_ms * 1e-3) / 1e12 if mlp_ms > 0 else None
    result = {
        "metric": METRIC,
        "value": value,
        "unit": "rays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (room0-shaped octree + Replica pinhole rays, analytic GT; random-init embeddings/decoder)",
        "config": {"workload": f"{args.scene}: {args.frames} keyframes x {args.rays_per_frame} rays/iter per GPU, "
                               f"{tree.count_nodes()} octree nodes, decoder W={args.width}, "
                               f"{h_m / max(h_r, 1):.1f} samples/hit ray (step {step_size:.5f} m)",
                   "rays_per_step_per_gpu": rays_per_step, "samples_per_step": h_m, "hit_rays_per_step": h_r,
                   "aabb_tests_per_step": h_v, "parallelism": f"dp{world} (ray-sharded, RCCL grad all-reduce)"},
        "roofline": roof_qi,
        "roofline_mfma": {"kernel": f"NRGBD decoder MLP W={w} fwd+bwd (fwd, δ chain, weight gradients)",
                          "bound": "mfma", "achieved": mlp_tf, "peak": MFMA_F32_PEAK_TFS, "unit": "TFLOP/s",
                          "frac": (mlp_tf / MFMA_F32_PEAK_TFS) if mlp_tf else None,
                          "traffic": traffic.get("mlp_bytes_per_step"),
                          "algorithmic_flops_per_launch": flops_mlp, "avg_launch_ms": mlp_ms,
                          "fwd_ms": mlp_f_ms, "bwd_ms": mlp_b_ms},
        "roofline_interp_bwd": roof_ib,
        "path": path_desc,
        "other_path": other,
        "kernels_ms": kt,
        "kernels_ms_overlapped": kt_overlap,
    }
    log("done timing")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("CPU baseline")
        result["cpu_baseline"] = cpu_baseline(args, scene, tree, step_size, args.cpu_baseline_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
