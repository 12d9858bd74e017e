"""Benchmark: rays/s for render + loss + backward (+ optimiser steps) of the
Proud-SLAM mapping render-and-optimise iteration — bundle_adjust_frames
(render_helpers.py:559-676) called exactly as Mapping.do_mapping calls it
(mapping.py:195-213: points encoder + its Adam, torch Adam optimisers on the
embeddings and decoder, keyframe pose optimisers) — on synthetic Replica
room0-shaped input (BASELINE.json configs[1]: 4096 rays/iter = 4 keyframes x
1024 rays, 1x MI355X; ~64 samples/ray).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--extras] [--no-traffic]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One process per GPU; every rank renders its own keyframes' 4096 rays against
the replicated octree (weak scaling); the loss is the union batch's and the
embedding + decoder gradients are summed over ranks.  Rank 0
prints one JSON line.  Inputs (octree, embeddings, decoder, full-resolution
keyframes) are resident in HBM before timing starts.  The roofline carries
kernel durations measured in the headline iterations and HBM bytes from two
PMC passes over the same iterations (rocprofv3 children, before the JSON).
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
TIMING_NOTE = ("headline mode, inside bundle_adjust_frames iterations: every kernel of a region timed by a HIP "
               "event pair bound to its own dispatch (hipExtLaunchKernel start / stop: the span rocprofv3 "
               "--kernel-trace reports, on the stream it runs on); a region = the sum of its kernels' spans "
               "(PSVO_TIMING_SPAN=1: first kernel's start to last kernel's end; PSVO_TIMING_MARKERS=1: marker "
               "events around the region)")


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
    ap.add_argument("--path", choices=("ba",), default="ba",
                    help="headline: the reference's bundle_adjust_frames API as Mapping calls it (the other paths: "
                         "--extras)")
    ap.add_argument("--extras", action="store_true",
                    help="also time the other paths (engine step on pre-built batches, drop-in autograd) and the "
                         "serialised one-stream kernel breakdown (not part of the default run, so that a profile "
                         "of the default command holds only headline-mode launches)")
    ap.add_argument("--no-traffic", action="store_true",
                    help="skip the PMC passes (rocprofv3 FETCH_SIZE / WRITE_SIZE children) that measure roofline.traffic")
    ap.add_argument("--train-iters", type=int, default=400,
                    help="untimed bundle_adjust_frames iterations on the same keyframes before the headline is "
                         "timed, so that it runs on a map in the state Mapping renders (trained: the sparse "
                         "decoder's class mix settles); stops early once the composited fraction is stable. "
                         "0: time the random-init map (the untrained figure is reported beside the trained one)")
    ap.add_argument("--probe", action="store_true", help=argparse.SUPPRESS)  # PMC child: headline iterations only
    ap.add_argument("--step-size", type=float, default=None, help=argparse.SUPPRESS)
    a = ap.parse_args()
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


def _cpu_threads():
    """Threads for the CPU baseline: the process's CPU share.  On the GPU box
    that share is 16 host CPUs per GPU (the box sets OMP_NUM_THREADS=16 for
    it), while the affinity mask shows the whole machine's CPUs; elsewhere the
    affinity mask."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return min(int(env), aff), f"OMP_NUM_THREADS={env}: the process's CPU share on this host " \
                                   f"(affinity mask {aff} CPUs is the whole machine's)"
    return aff, f"the process's affinity mask ({aff} CPUs)"


def cpu_baseline(args, scene, tree, step_size, seconds):
    """Oracle (reference algorithm restated: C kernels + torch-CPU render /
    loss / autograd) on the host cores, bounded sample of the same workload."""
    from oracle import oracle as O
    from psvo import synthetic as syn
    n_thr, why = _cpu_threads()
    torch.set_num_threads(n_thr)  # torch-CPU render / loss / autograd; the C kernels use OpenMP (same count)
    os.environ.setdefault("OMP_NUM_THREADS", str(n_thr))
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
            "cores_reason": why,
            "cpu_model": _cpu_model(), "host_physical_cores": _physical_cores(), "host_logical_cpus": os.cpu_count(),
            "process_affinity_cpus": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
            "sample": f"{n_it} iterations x {ro.shape[1]} rays ({args.scene}, {args.frames}x{args.rays_per_frame}), "
                      f"oracle C kernels (OpenMP over rays) + torch-CPU render/loss/backward, "
                      f"{torch.get_num_threads()} threads, {dt:.1f}s"}


CHAIN_KERNELS = ("k_intersect_sorted", "k_ray_stats_rank", "k_sample_fused", "k_scan_samples", "k_sample_points",
                 "k_interp_fwd", "k_points_interp", "k_interp_fwd_rays", "k_compact_rays")
# the kernels each timed region of the query + interp chain launches (for the
# per-region PMC traffic): intersect (+ its statistics / rank tail or pass),
# sampler (+ scan), compaction, interpolation (the headline's k_interp_fwd_rays
# does the compaction too)
REGION_KERNELS = {"intersect": ("k_intersect_sorted", "k_ray_stats_rank"),
                  "sample": ("k_sample_fused", "k_scan_samples"),
                  "points": ("k_sample_points", "k_compact_rays"),
                  "interp_fwd": ("k_interp_fwd", "k_interp_fwd_rays", "k_points_interp")}
MLP_KERNELS = ("k_mlp_prep", "k_mlp_fwd2", "k_mlp_bwd3", "k_mlp_bwd2", "k_mlp_dw2", "k_mlp_dw_reduce",
               "k_dec256_prep", "k_dec256_fwd", "k_dec256_bwd", "k_dec256_dw", "k_dec256_dw_reduce")


def _short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0].split("<")[0].split("::")[-1].strip() or name[:40]


def measure_traffic(args, step_size):
    """roofline.traffic, measured for this workload by this run: two rocprofv3
    PMC passes (FETCH_SIZE, then WRITE_SIZE: they cannot share a pass) over a
    child `bench.py --probe` that runs only the headline bundle_adjust_frames
    iterations with this run's step size.  Per kernel the median bytes per
    launch (FETCH_SIZE doubled: gfx950 tallies a 128-B streaming request as
    64 B, MI355X_MICROARCH.md §HBM; WRITE_SIZE as is; both count Infinity-
    Cache traffic).  Returns (dict or None, note)."""
    import csv
    import shutil
    import subprocess
    import tempfile
    from collections import defaultdict
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None, "rocprofv3 not found"
    out = {}
    with tempfile.TemporaryDirectory(prefix="psvo_pmc_") as tmp:
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, c)
            cmd = ["timeout", "-s", "KILL", "240", prof, "--pmc", c, "--output-format", "csv", "-d", d, "-o", "pmc",
                   "--", sys.executable, os.path.abspath(__file__), "--probe", "--step-size", repr(step_size),
                   "--scene", args.scene, "--frames", str(args.frames), "--rays-per-frame", str(args.rays_per_frame),
                   "--width", str(args.width), "--steps", "8", "--warmup", "2", "--no-cpu-baseline",
                   "--train-iters", str(args.train_iters_done)]
            env = dict(os.environ, TMPDIR=tmp)
            r = subprocess.run(cmd, env=env, capture_output=True, text=True)
            if r.returncode != 0:
                return None, f"{c} pass failed (rc {r.returncode}): {r.stderr[-300:]}"
            path = None
            for root, _, files in os.walk(d):
                for f in files:
                    if f.endswith("counter_collection.csv"):
                        path = os.path.join(root, f)
            if path is None:
                return None, f"{c} pass wrote no counter_collection.csv"
            vals = defaultdict(list)
            for row in csv.DictReader(open(path)):
                if row.get("Counter_Name") == c:
                    vals[_short(row["Kernel_Name"])].append(float(row["Counter_Value"]) * 1024.0)  # KB units
            # the trained map's launches: the last quarter of each kernel's (the probe trains first)
            vals = {k: v[len(v) - max(1, len(v) // 4):] if args.train_iters_done else v for k, v in vals.items()}
            out[c] = {k: sorted(v)[len(v) // 2] * (2.0 if c == "FETCH_SIZE" else 1.0) for k, v in vals.items()}
    kern = {}
    for k in set(out["FETCH_SIZE"]) | set(out["WRITE_SIZE"]):
        f, w = out["FETCH_SIZE"].get(k, 0.0), out["WRITE_SIZE"].get(k, 0.0)
        kern[k] = {"fetch": f, "write": w, "total": f + w}
    res = {"kernels": kern,
           "query_interp_bytes_per_step": sum(kern[k]["total"] for k in CHAIN_KERNELS if k in kern),
           "bwd_fused_bytes_per_launch": (kern.get("k_mlp_bwd3") or kern.get("k_interp_bwd") or {}).get("total"),
           "mlp_bytes_per_step": sum(kern[k]["total"] for k in MLP_KERNELS if k in kern)}
    return res, "measured by this run: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py --probe " \
                "(headline iterations), median bytes per launch, fetch = 2 x FETCH_SIZE (gfx950)"


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
    from psvo.point_feature import PointsResNet
    import types
    _lib.lib()

    log(f"scene {args.scene}: octree, embeddings, decoder W={args.width}")
    scene, tree, ms, emb, dec = build_scene(args, device, rank)
    log(f"{args.frames} keyframes ({tree.count_nodes()} octree nodes)")
    kfs = build_keyframes(args, scene, device, rank)
    if args.step_size is not None:
        step_size, spr = args.step_size, float("nan")
        batches = None
    else:
        batches = keyframe_batches(kfs, args.rays_per_frame, args.pool)
        log("step-size calibration")
        step_size, spr = calibrate_step(ms, batches, args.samples_per_ray, scene.voxel_size, world)
    log(f"step {step_size:.5f} m, {spr:.1f} samples / hit ray; timing the {args.path} path")
    crit_cfg, max_depth = SCENE_CRITERIA.get(args.scene, DEFAULT_CRITERIA)
    crit_args = types.SimpleNamespace(criteria=dict(crit_cfg), data_specs={"max_depth": max_depth})
    criterion = Criterion(crit_args)
    # Mapping's optimisers (mapping.py:81-82, 93) and its points encoder
    # (mapping.py:36, variations/resnet.py; never run by the render path)
    embed_optim = torch.optim.Adam([emb], lr=5e-3)
    model_optim = torch.optim.Adam(dec.parameters(), lr=5e-3)
    points_encoder = PointsResNet(16).to(device)
    points_encoder.train()
    resnet_optim = torch.optim.Adam(points_encoder.parameters(), lr=5e-3)
    stats = {"n": 0, "m": 0, "r_hit": 0, "visits": 0, "s_max": 0}  # the marked (breakdown) runs
    head_stats = dict(stats)  # the headline bundle_adjust_frames iterations

    from psvo.engine import MappingEngine
    from psvo.dist import EngineExchange
    # N > 1: the union batch's loss needs an engine with the
    # ranks' exchange, handed to bundle_adjust_frames; N = 1: the reference's
    # own call, dispatched to the native engine by bundle_adjust_frames itself
    dp_engine = None
    if world > 1:
        dp_engine = MappingEngine(ms, dec, scene.voxel_size, step_size, truncation=0.1, max_distance=max_depth,
                                  criteria=crit_args.criteria, max_depth=max_depth, lr_emb=5e-3, lr_dec=5e-3)
        dp_engine.set_exchange(EngineExchange(args.frames * args.rays_per_frame * world, device=device,
                                              max_rays_rank=args.frames * args.rays_per_frame))

    def record_stats(m, r_hit, visits, s_max, into=None):
        sd = stats if into is None else into
        sd["n"] += 1
        sd["m"] += m
        sd["r_hit"] += r_hit
        sd["visits"] += visits
        sd["s_max"] = max(sd["s_max"], s_max)

    # ---- bundle_adjust_frames as Mapping.do_mapping calls it (mapping.py:
    # 195-213; render_helpers.py:559-676): this rank's keyframes — full-
    # resolution synthetic RGB-D frames with their own poses (optimised, lr
    # 1e-3, frame.py:27) — each iteration samples rays_per_frame pixels per
    # keyframe (gumbel top-k on the device), renders, back-propagates and steps
    # every optimiser.  K steps = one call with num_iterations = K.
    ba_calls = [0]
    pace = {}  # the headline run's GPU-side period and the host's waits (timed_ba)

    def run_ba(steps):
        call = ba_calls[0]
        ba_calls[0] += 1
        if dp_engine is not None:
            dp_engine.discard_queued()
            RH.bundle_adjust_frames(kfs, ms, dec, points_encoder, criterion, scene.voxel_size, step_size,
                                    args.rays_per_frame, steps, 0.1, 10, max_depth, learning_rate=[1e-2, 1e-3],
                                    embed_optim=embed_optim, model_optim=model_optim, resnet_optim=resnet_optim,
                                    update_pose=True, engine=dp_engine,
                                    seed_fn=lambda it: 1000003 * (call + 1) + it)  # the same on every rank
        else:
            RH.bundle_adjust_frames(kfs, ms, dec, points_encoder, criterion, scene.voxel_size, step_size,
                                    args.rays_per_frame, steps, 0.1, 10, max_depth, learning_rate=[1e-2, 1e-3],
                                    embed_optim=embed_optim, model_optim=model_optim, resnet_optim=resnet_optim,
                                    update_pose=True)

    def head_engine():
        if dp_engine is not None:
            return dp_engine
        engs = list(RH._ENGINES.values())
        if len(engs) != 1:
            raise RuntimeError("bench: bundle_adjust_frames did not run on the native engine")
        return engs[0]

    sel_stats = {}

    def timed_ba(steps, warmup, record=False):
        if warmup:
            run_ba(warmup)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        eng = head_engine() if warmup else None
        clocked = False
        if record and eng is not None:
            eng.stats_hook = lambda st: record_stats(st[4], st[9] if world > 1 else st[1], st[5], st[3], head_stats)
            eng.select_stats(reset=True)  # the sparse decoder's kept / composited samples of the timed steps
        if record and eng is not None and os.environ.get("PSVO_BENCH_NO_CLOCK") != "1":
            try:  # an event at each step's entry on its stream: the GPU-side period
                eng.set_clock(steps)
                eng.host_wait_stats(reset=True)
                clocked = True
            except AttributeError:  # an older library (A/B runs) without the clock
                pass
        t0 = time.perf_counter()
        run_ba(steps)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if clocked:
            period, n_clk = eng.clock()
            eng.set_clock(0)
            w_us, w_calls, w_waited = eng.host_wait_stats(reset=True)
            pace.update(gpu_ms_per_step=period, clock_steps=n_clk,
                        host_wait_us_per_step=w_us / max(w_calls, 1), host_waits=w_calls,
                        host_waits_before_landing=w_waited)
        if eng is not None:
            eng.stats_hook = None
        if record and eng is not None:
            sel_stats.update(eng.select_stats())
        if world > 1:
            t = torch.tensor([el], device=device, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    def train_map(max_iters, chunk=50):
        """Untimed bundle_adjust_frames iterations on the same keyframes (the
        map as Mapping.spin leaves it for its next call, mapping.py:96-218):
        chunks of `chunk` until the composited fraction moves by < 0.01 between
        chunks (at least 2) or max_iters.  Returns [(iterations, composited
        fraction, kept fraction)] after each chunk."""
        trace, done, prev = [], 0, None
        m_acc = {"m": 0, "n": 0}
        while done < max_iters:
            n = min(chunk, max_iters - done)
            run_ba(n)  # the first call creates the engine
            done += n
            eng = head_engine()
            eng.select_stats(reset=True)
            eng.stats_hook = lambda st: (m_acc.__setitem__("m", m_acc["m"] + st[4]),
                                         m_acc.__setitem__("n", m_acc["n"] + 1))
            m_acc.update(m=0, n=0)
            run_ba(10)  # a short measured call: the class mix of the map as it now is
            done += 10
            eng.stats_hook = None
            sel = eng.select_stats(reset=True)
            m_step = m_acc["m"] / max(m_acc["n"], 1)
            comp = sel["composited_sum"] / max(sel["steps"], 1) / max(m_step, 1)
            kept = sel["kept_sum"] / max(sel["steps"], 1) / max(m_step, 1)
            if world > 1:  # one decision for all ranks (each call issues collectives): the ranks' mean
                t = torch.tensor([comp, kept], dtype=torch.float64, device=device)
                dist.all_reduce(t)
                comp, kept = (float(x) / world for x in t.cpu())
            trace.append((done, round(comp, 4), round(kept, 4)))
            if prev is not None and abs(comp - prev) < 0.01 and len(trace) >= 2:
                break
            prev = comp
        torch.cuda.synchronize()
        return trace

    if args.probe:  # PMC child (measure_traffic): the headline iterations only (after the same training)
        if args.train_iters > 0:
            run_ba(args.train_iters)
        run_ba(args.warmup + args.steps)
        torch.cuda.synchronize()
        return
    if args.path != "ba":
        raise SystemExit("bench.py: the headline is --path ba (the other paths run with --extras)")
    # the random-init map first (rounds 1-5 timed only this), then the map
    # trained on the same keyframes: the headline
    untrained, train_trace = None, []
    args.train_iters_done = 0
    if args.train_iters > 0:
        el_u = timed_ba(args.steps, max(1, args.warmup), record=True)
        hs_u = dict(head_stats)
        steps_u = sel_stats.get("steps", 0)
        m_u = hs_u["m"] / max(hs_u["n"], 1)
        untrained = {"value": args.frames * args.rays_per_frame * args.steps * world / el_u,
                     "ms_per_step": 1000.0 * el_u / args.steps, "gpu_ms_per_step": pace.get("gpu_ms_per_step"),
                     "decoder_kept_fraction": sel_stats["kept_sum"] / steps_u / m_u if steps_u and m_u else None,
                     "composited_fraction": sel_stats["composited_sum"] / steps_u / m_u if steps_u and m_u else None,
                     "samples_per_step": m_u}
        log(f"untrained map: {untrained['ms_per_step']:.4f} ms/step; training (untimed, <= {args.train_iters} it)")
        train_trace = train_map(args.train_iters)
        args.train_iters_done = train_trace[-1][0] if train_trace else 0
        log(f"trained {args.train_iters_done} iterations: composited / kept fraction {train_trace[-1][1:]}")
        for k in list(head_stats):
            head_stats[k] = 0
        sel_stats.clear()
        pace.clear()
    elapsed = timed_ba(args.steps, max(1, args.warmup), record=True)
    path_desc = ("bundle_adjust_frames as Mapping.do_mapping calls it (points encoder + its Adam, torch Adam "
                 "optimisers; per-iteration gumbel pixel sampling on the device, keyframe poses optimised) — "
                 "dispatched by bundle_adjust_frames to psvo_map_step_frames")
    eng = head_engine()
    # the kernels' durations as the headline runs them: HIP events on the
    # launching streams inside the same bundle_adjust_frames iterations
    n_mark = max(5, min(args.steps, 20))
    eng.set_timing("overlap")
    if world > 1:  # the exchanges' own durations, in the same marked iterations
        from psvo import dist as D
        D.TIMER = D.CollectiveTimer()
    timed_ba(n_mark, 0)
    kt_overlap = eng.timing()
    eng.set_timing(False)
    collectives = None
    if world > 1:
        coll_ms = D.TIMER.total_ms()
        collectives = {"collective_ms_per_step": coll_ms / n_mark, "collectives_per_step": D.TIMER.count / n_mark,
                       "backend": dist.get_backend(),
                       "timing": "HIP events around each RCCL call on its stream (gloo: host time of the "
                                 "host-staged call), marked iterations"}
        D.TIMER = None
    kt_serial = None
    others = []
    rays_step = args.frames * args.rays_per_frame
    if args.extras and world == 1:
        # the serialised one-stream breakdown and the other paths, on a separate
        # engine over pre-built world-space batches (fixed poses)
        if batches is None:
            batches = keyframe_batches(kfs, args.rays_per_frame, args.pool)
        from psvo.optim import Adam
        x_emb = emb.detach().clone().requires_grad_(True)
        x_ms = dict(ms, voxel_vertex_emb=x_emb)
        x_eo = Adam([x_emb], lr=5e-3)
        x_mo = Adam(dec.parameters(), lr=5e-3)
        engine = MappingEngine(x_ms, dec, scene.voxel_size, step_size, truncation=0.1, max_distance=max_depth,
                               criteria=crit_args.criteria, max_depth=max_depth, lr_emb=5e-3, lr_dec=5e-3)
        eng_it = [0]

        def step_engine(i, record=False):
            it = eng_it[0]
            eng_it[0] += 1
            ro, rd, rgb, depth = batches[it % len(batches)]
            seed = 1000003 + it
            if not engine._queued:
                engine.query(ro, rd, seed)
            nro, nrd, _, _ = batches[(it + 1) % len(batches)]
            engine.query(nro, nrd, seed + 1)
            loss = engine.step(ro, rd, rgb, depth, seed=seed)
            if record:
                st = engine.last_stats
                record_stats(st[4], st[1], st[5], st[3])
            return loss

        def step_autograd(i, record=False):
            ro, rd, rgb, depth = batches[i % len(batches)]
            out = RH.render_rays(ro, rd, x_ms, dec, None, step_size, scene.voxel_size, 0.1, 10, max_depth,
                                 return_samples=True, seed=7919 * i + 1)
            loss, _ = criterion(out, (rgb, depth))
            x_eo.zero_grad()
            x_mo.zero_grad()
            loss.backward()
            x_eo.step()
            x_mo.step()
            return loss

        def run(step_fn, steps, warmup, record=False):
            for i in range(warmup):
                step_fn(i)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(steps):
                step_fn(warmup + i, record)
            torch.cuda.synchronize()
            return time.perf_counter() - t0

        engine.set_timing(True)      # regions serialised on one stream
        run(step_engine, n_mark, 2, record=True)
        kt_serial = engine.timing()
        engine.set_timing(False)
        engine.discard_queued()
        other_steps = max(5, min(args.steps, 20))
        el2 = run(step_engine, other_steps, 2)
        others.append({"path": "native engine step (psvo_map_step, fixed poses, pre-built rays)",
                       "value": rays_step * other_steps / el2, "ms_per_step": 1000.0 * el2 / other_steps})
        engine.discard_queued()
        el2 = run(step_autograd, other_steps, 2)
        others.append({"path": "drop-in autograd (render_rays + Criterion + backward + psvo.optim.Adam)",
                       "value": rays_step * other_steps / el2, "ms_per_step": 1000.0 * el2 / other_steps})
        engine.close()
    rays_per_step = rays_step
    total_rays = rays_per_step * args.steps * world
    value = total_rays / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps

    # Rooflines.  Primary — the north star's "octree query+interp
    # kernel", as the kernels launched for it: algorithmic bytes per step =
    # per ray 24 B + 48 B per AABB-tested node (V counted by the kernel) + per
    # valid sample 12 B (sampler output) + 628 B (interp fwd), over the summed
    # durations of those launches AS THE HEADLINE RUNS THEM (HIP events on
    # their streams inside bundle_adjust_frames iterations: intersect + stats
    # + hit rank, sampler + scan, sample compaction, interp fwd).  The
    # interpolation BACKWARD (1,664 B / sample) runs inside the fused decoder
    # backward k_mlp_bwd3 (width 128), beside its MFMAs: it has no duration of
    # its own and is reported with that kernel (roofline_bwd_fused).  The
    # one-stream serialised durations are reported with --extras.  Traffic:
    # PMC-counted HBM bytes of the same iterations (measure_traffic).
    # Secondary — the decoder (dominant by time), MFMA-bound.
    hs = head_stats
    h_n = max(hs["n"], 1)
    h_m, h_r, h_v = hs["m"] / h_n, hs["r_hit"] / h_n, hs["visits"] / h_n
    if world > 1:  # per-GPU averages over the union of the ranks' batches
        t = torch.tensor([h_m, h_r, h_v], dtype=torch.float64, device=device)
        dist.all_reduce(t)
        h_m, h_r, h_v = (float(x) / world for x in t.cpu())
    fused_ib = args.width == 128  # interp bwd inside k_mlp_bwd3
    q_keys = ("intersect", "sample", "points", "interp_fwd") + (() if fused_ib else ("interp_bwd",))
    # a region the step did not mark (the headline has no separate compaction) counts 0
    q_parts = {k: max(kt_overlap[k], 0.0) for k in q_keys}
    q_ms = sum(q_parts.values())
    bytes_qi = rays_step * 24.0 + h_v * 48.0 + h_m * 12.0 + h_m * (628.0 + (0.0 if fused_ib else 1664.0))
    # the same byte model per region: traversal 24 B / ray + 48 B / AABB-tested node,
    # sampler output 12 B / sample, interpolation 628 B / sample (8 × 64-B vertex rows + 64-B feature
    # + the 12-B compacted sample), interp bwd 1,664 B / sample where it has a launch of its own
    region_bytes = {"intersect": rays_step * 24.0 + h_v * 48.0, "sample": h_m * 12.0, "points": 0.0,
                    "interp_fwd": h_m * 628.0, "interp_bwd": h_m * 1664.0}
    traffic, traffic_note = None, "not measured (N > 1 or --no-traffic)"
    if world == 1 and not args.no_traffic:
        log("PMC passes (roofline.traffic)")
        try:
            traffic, traffic_note = measure_traffic(args, step_size)
        except Exception as exc:  # noqa: BLE001 — the headline stands without it
            traffic, traffic_note = None, f"PMC passes failed: {type(exc).__name__}: {exc}"
    tr = traffic or {}

    def bw_roof(kernel, alg_bytes, ms, counter_bytes, ms_serial=None, extra=None):
        gbs = alg_bytes / (ms * 1e-3) / 1e9 if ms and ms > 0 else None
        r = {"kernel": kernel, "bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": gbs / HBM_PEAK_GBS if gbs else None, "traffic": counter_bytes,
             "algorithmic_bytes_per_launch": alg_bytes, "avg_launch_ms": ms,
             "timing": TIMING_NOTE,
             "frac_hbm_counters": (counter_bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if (counter_bytes and ms) else None,
             "frac_l2_algorithmic": gbs / L2_PEAK_GBS if gbs else None}
        if ms_serial:
            r["avg_launch_ms_serialised"] = ms_serial
            r["frac_serialised"] = alg_bytes / (ms_serial * 1e-3) / 1e9 / HBM_PEAK_GBS
        if extra:
            r.update(extra)
        return r

    lb = rays_step <= 16384  # the look-back query (svo_query.hip / lookback.h)
    lb_smp = lb and world == 1
    q_desc = ("k_intersect_sorted (hit ranks / statistics by in-launch look-back)" if lb
              else "k_intersect_sorted+k_ray_stats_rank")
    q_desc += (", k_sample_fused (sample scan, read-back and compaction by in-launch look-back)" if lb_smp
               else ", k_sample_fused+k_scan_samples")
    if lb_smp:
        i_desc = "k_interp_fwd"
    elif world > 1:
        i_desc = "k_sample_points, k_interp_fwd"
    else:
        i_desc = "k_compact_rays, k_interp_fwd"
    chain_desc = q_desc + ", " + i_desc
    kern_tr = tr.get("kernels") or {}
    per_region = {}
    for k in q_keys:
        ms_k = q_parts[k]
        if ms_k <= 0:
            continue
        frac_k = region_bytes[k] / (ms_k * 1e-3) / 1e9 / HBM_PEAK_GBS
        counted = sum(kern_tr[n]["total"] for n in REGION_KERNELS.get(k, ()) if n in kern_tr) if kern_tr else None
        cfrac = counted / (ms_k * 1e-3) / 1e9 / HBM_PEAK_GBS if counted else None
        per_region[k] = {"ms": ms_k, "algorithmic_bytes": region_bytes[k], "frac": frac_k,
                         "hbm_bytes_counted": counted, "frac_hbm_counters": cfrac,
                         # an algorithmic rate above the HBM peak cannot come from HBM: the table / tree
                         # reads hit the XCD L2s or the 256-MB MALL
                         "served_from": ("L2/MALL (algorithmic bytes exceed what HBM could deliver)" if frac_k > 1.0
                                         else "mostly L2/MALL (counted HBM bytes < 1/2 of algorithmic)"
                                         if counted is not None and counted < 0.5 * region_bytes[k] else "HBM")}
    roof_qi = bw_roof("octree query+interp (" + chain_desc + (")" if fused_ib else ", k_interp_bwd)"), bytes_qi,
                      q_ms, tr.get("query_interp_bytes_per_step"),
                      sum(kt_serial[k] for k in q_keys) if kt_serial else None,
                      {"parts_ms": q_parts, "parts_ms_serialised": {k: kt_serial[k] for k in q_keys}
                       if kt_serial else None, "per_region": per_region, "visits_per_ray": h_v / max(rays_step, 1),
                       "samples_per_hit_ray": h_m / max(h_r, 1), "traffic_note": traffic_note})
    mlp_f_ms, mlp_b_ms = kt_overlap["mlp_fwd"], kt_overlap["mlp_bwd"]
    mlp_ms = mlp_f_ms + mlp_b_ms
    w = args.width
    macs = 16 * w + w * w + w * 129 + 144 * w + w * 3  # nrgbd.py:80-146, depth 2, sdf_dim 128, in_dim 16
    trunk = 16 * w + w * w + w  # h1, h2 and the sdf row: what the sparse decoder runs on every sample
    flops_mlp = 3 * 2.0 * macs * h_m  # algorithmic: the reference's forward + δ chain + weight gradients, every sample
    steps_sel = sel_stats.get("steps", 0)
    kept = sel_stats["kept_sum"] / steps_sel if steps_sel else None  # per step (this rank)
    comp = sel_stats["composited_sum"] / steps_sel if steps_sel else None
    if world > 1 and kept is not None:
        t = torch.tensor([kept, comp], dtype=torch.float64, device=device)
        dist.all_reduce(t)
        kept, comp = (float(x) / world for x in t.cpu())
    # executed: the sdf trunk on every sample; the whole decoder forward and backward on the kept
    # ones — width 128 on the composited ones only, the trunk forward + backward (δ chain, dW1, dW2,
    # the sdf row of W3) on the kept samples that only the direct sdf loss reaches (class B); width
    # 128 reads the W2 layer's output (h2) the sdf trunk wrote instead of recomputing it
    two_class = w == 128 and kept is not None
    n_b = max(kept - comp, 0.0) if two_class else 0.0
    n_full = comp if two_class else kept
    w2 = w * w if two_class else 0  # the W2 layer, read rather than recomputed (two_class: width 128)
    flops_exec = (2.0 * trunk * h_m + 2.0 * (3 * macs - w2) * n_full + 2.0 * (3 * trunk - w2) * n_b) \
        if kept is not None else flops_mlp
    flops_bwd = (2 * 2.0 * macs * n_full + 2.0 * (3 * trunk - w2) * n_b) if kept is not None \
        else 2 * 2.0 * macs * h_m
    mlp_tf = flops_exec / (mlp_ms * 1e-3) / 1e12 if mlp_ms > 0 else None
    m_bwd = kept if kept is not None else h_m  # the samples the backward runs on
    if fused_ib:  # k_mlp_bwd3 (+ k_mlp_trunk_fb): δ chain + weight gradients + the interpolation backward
        b_tf = flops_bwd / (mlp_b_ms * 1e-3) / 1e12 if mlp_b_ms > 0 else None
        ib_gbs = 1664.0 * m_bwd / (mlp_b_ms * 1e-3) / 1e9 if mlp_b_ms > 0 else None
        roof_ib = {"kernel": "k_mlp_bwd3 + k_mlp_trunk_fb + k_mlp_dw_reduce (decoder delta chain, weight gradients, and the "
                             "interpolation backward: embedding scatter + dL/dx)",
                   "bound": "mfma", "achieved": b_tf, "peak": MFMA_F32_PEAK_TFS, "unit": "TFLOP/s",
                   "frac": b_tf / MFMA_F32_PEAK_TFS if b_tf else None,
                   "traffic": tr.get("bwd_fused_bytes_per_launch"), "avg_launch_ms": mlp_b_ms,
                   "flops_per_launch_executed": flops_bwd,
                   "samples_per_launch": m_bwd,
                   "interp_bwd_bytes": 1664.0 * m_bwd,
                   "interp_bwd_bytes_over_kernel_time_frac_hbm": ib_gbs / HBM_PEAK_GBS if ib_gbs else None,
                   "timing": TIMING_NOTE}
    else:
        roof_ib = bw_roof("k_interp_bwd", 1664.0 * m_bwd, kt_overlap["interp_bwd"],
                          tr.get("bwd_fused_bytes_per_launch"), kt_serial["interp_bwd"] if kt_serial else None)
    result = {
        "metric": METRIC,
        "value": value,
        "unit": "rays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        # the steady-state iteration period as the GPU ran it (events at each step's entry on its
        # stream) and how often the host had to wait for a query's statistics — a host that never
        # waits set the pace; one that waits on nearly every step was paced by the GPU
        "gpu_ms_per_step": pace.get("gpu_ms_per_step"),
        "pace": dict(pace, note="gpu_ms_per_step excludes each bundle_adjust_frames call's setup / write-back "
                                "and its first, un-pipelined iteration; ms_per_step is the wall clock of the call"),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": ("synthetic (room0-shaped octree + Replica pinhole RGB-D keyframes, analytic GT); embeddings / "
                 "decoder / poses trained from random init by %d untimed bundle_adjust_frames iterations on the "
                 "same keyframes before timing (map_state: %s)" % (args.train_iters_done, "trained"
                                                                   if args.train_iters_done else "random-init")),
        "config": {"workload": f"{args.scene}: {args.frames} keyframes x {args.rays_per_frame} rays/iter per GPU, "
                               f"{tree.count_nodes()} octree nodes, decoder W={args.width}, "
                               f"{h_m / max(h_r, 1):.1f} samples/hit ray (step {step_size:.5f} m)",
                   "rays_per_step_per_gpu": rays_per_step, "samples_per_step": h_m, "hit_rays_per_step": h_r,
                   "aabb_tests_per_step": h_v,
                   # the sparse decoder: samples whose gradients can be non-zero (the full decoder runs on
                   # these) and the composited ones (a compositing weight: z < z_min + truncation)
                   "decoder_kept_fraction": kept / h_m if kept is not None and h_m else None,
                   "composited_fraction": comp / h_m if comp is not None and h_m else None,
                   "map_state": "trained" if args.train_iters_done else "random-init",
                   "train_iterations": args.train_iters_done,
                   # (iterations so far, composited fraction, kept fraction) after each training chunk
                   "train_trace": train_trace,
                   "untrained": untrained,
                   "parallelism": f"dp{world} (ray-sharded, union-batch loss, "
                                  f"{dist.get_backend() if world > 1 else 'no'} collectives)"},
        "roofline": roof_qi,
        "roofline_mfma": {"kernel": f"NRGBD decoder MLP W={w} fwd+bwd (fwd, δ chain, weight gradients)",
                          "bound": "mfma", "achieved": mlp_tf, "peak": MFMA_F32_PEAK_TFS, "unit": "TFLOP/s",
                          "frac": (mlp_tf / MFMA_F32_PEAK_TFS) if mlp_tf else None,
                          "traffic": tr.get("mlp_bytes_per_step"),
                          "flops_executed_per_step": flops_exec,
                          "flops_algorithmic_per_step": flops_mlp,
                          "achieved_basis": "executed FLOPs (sdf trunk on every sample, the whole decoder forward + "
                                            "backward on the composited samples (W=256: on every kept sample), the "
                                            "trunk forward + backward on the other kept samples; W=128: the W2 "
                                            "layer's output read from the sdf trunk, not recomputed) / time",
                          "effective_algorithmic_tflops": flops_mlp / (mlp_ms * 1e-3) / 1e12 if mlp_ms > 0 else None,
                          "avg_launch_ms": mlp_ms,
                          "fwd_ms": mlp_f_ms, "bwd_ms": mlp_b_ms,
                          "timing": TIMING_NOTE},
        "roofline_bwd_fused" if fused_ib else "roofline_interp_bwd": roof_ib,
        "path": path_desc,
        "other_path": others if others else "run bench.py --extras for the engine-step and drop-in autograd paths",
        "kernels_ms_overlapped": kt_overlap,
        "kernels_ms_serialised": kt_serial,
        "traffic_kernels": tr.get("kernels"),
    }
    if collectives:
        result["collectives"] = collectives
        result["collective_ms_per_step"] = collectives["collective_ms_per_step"]
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
