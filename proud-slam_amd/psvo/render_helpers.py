"""MI355X render path with the reference's render_helpers API
(src/variations/render_helpers.py): render_rays, get_features_vox,
bundle_adjust_frames, track_frame, get_scores/eval_points helpers.

render_rays (render_helpers.py:351-556) runs as:

  ray_intersect_sorted  DFS + stable t_in sort + max_distance trim   (1 kernel)
  hit_rank              compaction order of hit rays                  (1 kernel)
  ── read back P, R_hit, max ceil(steps)  (sync 1; sizes the outputs) ──
  sample_rays           inverse-CDF sampling, reference [200,K',P] layout,
                        + per-ray sample offsets, S_max, M
  ── read back S_max, M  (sync 2; output shapes [R_hit, S_max]) ──
  sample_points         z_vals / mask and ray-major compact samples
  interp  (autograd)    x = o + d t, trilinear embedding gather   HIP fwd/bwd
  decoder               the caller's sdf_network (MLP)
  composite (autograd)  sdf→weights, rgb/depth                    HIP fwd/bwd

The reference needs ~10 host syncs per call and copies the
octree 256× per intersection; this path syncs twice and copies nothing.
"""
from __future__ import annotations

import ctypes
import os
from copy import deepcopy

import torch
import torch.nn.functional as F
from torch.autograd import Function

from . import _lib as L
from . import sample_util
from .voxel_helpers import MAX_DEPTH, N_MAX_HITS, _intersect_sorted

D_EMB = 16

_timed = L.timed  # per-launch HIP-event timer hook (psvo._lib.KERNEL_TIMER)


def ray(ray_start, ray_dir, depths):
    return ray_start + ray_dir * depths


def fill_in(shape, mask, input, initial=1.0):
    if isinstance(initial, torch.Tensor):
        output = initial.expand(*shape)
    else:
        output = input.new_ones(*shape) * initial
    return output.masked_scatter(mask.unsqueeze(-1).expand(*shape), input)


def masked_scatter(mask, x):
    B, K = mask.size()
    if x.dim() == 1:
        return x.new_zeros(B, K).masked_scatter(mask, x)
    return x.new_zeros(B, K, x.size(-1)).masked_scatter(mask.unsqueeze(-1).expand(B, K, x.size(-1)), x)


def masked_scatter_ones(mask, x):
    B, K = mask.size()
    if x.dim() == 1:
        return x.new_ones(B, K).masked_scatter(mask, x)
    return x.new_ones(B, K, x.size(-1)).masked_scatter(mask.unsqueeze(-1).expand(B, K, x.size(-1)), x)


# --------------------------------------------------------------------------
# autograd Functions over the HIP kernels
# --------------------------------------------------------------------------
class InterpSamples(Function):
    """feat[M,16] = trilinear(E, x = o[row] + d[row] t) — get_features_vox
    (render_helpers.py:104-156) fused with sampled_xyz (:436-437) and the
    hit-ray gather of rays_o / rays_d (row = ray_index[ray_of_sample], or
    ray_of_sample when ray_index is None).  Backward: d_emb (float atomics on
    whole 64-B rows), d_o / d_d per ray (wave reductions) at the rays' rows."""

    @staticmethod
    def forward(ctx, rays_o, rays_d, emb, leaf, t, ray_of_sample, offsets, centres, vertex_idx, voxel_size,
                ray_index=None):
        M = leaf.numel()
        feat = torch.empty((M, D_EMB), dtype=torch.float32, device=leaf.device)
        with _timed("interp_fwd"):
            L.call("psvo_interp_fwd", L.stream_of(leaf.device), M, D_EMB, float(voxel_size), leaf, t, ray_of_sample,
                   ray_index, rays_o, rays_d, centres, vertex_idx, emb, feat)
        ctx.save_for_backward(rays_o, rays_d, emb, leaf, t, offsets, centres, vertex_idx, ray_index)
        ctx.voxel_size = float(voxel_size)
        return feat

    @staticmethod
    def backward(ctx, grad_feat):
        rays_o, rays_d, emb, leaf, t, offsets, centres, vertex_idx, ray_index = ctx.saved_tensors
        dev = leaf.device
        r_hit = offsets.numel() - 1
        grad_feat = grad_feat.contiguous().float()
        # frozen embeddings (tracking): the kernel skips the scatter-add
        grad_emb = torch.zeros_like(emb) if ctx.needs_input_grad[2] else None
        need_od = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
        # rows of rays that hit nothing get zero gradient
        god = (torch.zeros if ray_index is not None else torch.empty)((2,) + tuple(rays_o.shape), dtype=torch.float32,
                                                                      device=dev)
        with _timed("interp_bwd"):
            L.call("psvo_interp_bwd", L.stream_of(dev), r_hit, D_EMB, ctx.voxel_size, offsets, ray_index, leaf, t,
                   rays_o, rays_d, centres, vertex_idx, emb, grad_feat, grad_emb, god[0], god[1])
        return (god[0] if need_od and ctx.needs_input_grad[0] else None,
                god[1] if need_od and ctx.needs_input_grad[1] else None,
                grad_emb if ctx.needs_input_grad[2] else None, None, None, None, None, None, None, None, None)


class CompositeRays(Function):
    """render_helpers.py:504-556: (sdf_s[M], rgb_s[M,3]) → padded sdf,
    weights [R_hit,S_max], color [R_hit,3], depth [R_hit], z_min [R_hit,1]."""

    @staticmethod
    def forward(ctx, sdf_s, rgb_s, z_vals, offsets, ray_ns, truncation):
        r_hit, s_max = z_vals.shape
        dev = z_vals.device
        sdf_s = sdf_s.contiguous().float()
        rgb_s = rgb_s.contiguous().float()
        sdf = torch.empty((r_hit, s_max), dtype=torch.float32, device=dev)
        weights = torch.empty((r_hit, s_max), dtype=torch.float32, device=dev)
        color = torch.empty((r_hit, 3), dtype=torch.float32, device=dev)
        depth = torch.empty((r_hit,), dtype=torch.float32, device=dev)
        z_min = torch.empty((r_hit, 1), dtype=torch.float32, device=dev)
        L.call("psvo_composite_fwd", L.stream_of(dev), r_hit, s_max, float(truncation), L.ptr(offsets), L.ptr(ray_ns),
               L.ptr(z_vals), L.ptr(sdf_s), L.ptr(rgb_s), L.ptr(sdf), L.ptr(weights), L.ptr(color), L.ptr(depth),
               L.ptr(z_min))
        ctx.save_for_backward(offsets, ray_ns, z_vals, sdf, weights, rgb_s)
        ctx.truncation = float(truncation)
        ctx.m = sdf_s.shape[0]
        ctx.mark_non_differentiable(z_min)
        return sdf, weights, color, depth, z_min

    @staticmethod
    def backward(ctx, g_sdf, g_weights, g_color, g_depth, g_zmin):
        offsets, ray_ns, z_vals, sdf, weights, rgb_s = ctx.saved_tensors
        r_hit, s_max = z_vals.shape
        dev = z_vals.device
        c = lambda g: None if g is None else g.contiguous().float()
        g_sdf_s = torch.empty((ctx.m,), dtype=torch.float32, device=dev)
        g_rgb_s = torch.empty((ctx.m, 3), dtype=torch.float32, device=dev)
        L.call("psvo_composite_bwd", L.stream_of(dev), r_hit, s_max, ctx.truncation, L.ptr(offsets), L.ptr(ray_ns),
               L.ptr(z_vals), L.ptr(sdf), L.ptr(weights), L.ptr(rgb_s), c(g_color), c(g_depth), c(g_weights),
               c(g_sdf), L.ptr(g_sdf_s), L.ptr(g_rgb_s))
        return g_sdf_s, g_rgb_s, None, None, None, None


# --------------------------------------------------------------------------
# query stages (no grad)
# --------------------------------------------------------------------------
class RaySamples:
    """Everything the differentiable part needs about one ray batch."""

    __slots__ = ("ray_mask", "r_hit", "P", "s_max", "m", "z_vals", "sample_mask", "leaf", "t",
                 "ray_of_sample", "offsets", "ray_ns", "rank_ray32", "s_idx", "s_depth", "s_dist", "visits", "max_steps")


def _global_rows(q, R, step_size, batch):
    """All-gather the per-ray hit lists and rank the global batch (dist.GlobalBatch):
    returns the global rank_ray / ray_rank / stats / hit arrays, this rank's
    first ray and first logical hit row, and the local hit count."""
    dev = q["ray_nv"].device
    sizes = batch.sizes(R)
    ray_off = sum(sizes[: batch.rank])
    g = {k: batch.gather_cat(q[k], sizes) for k in ("hit_idx", "hit_t0", "hit_t1", "ray_nv", "ray_dsum")}
    rg = sum(sizes)
    g["stats"] = torch.zeros_like(q["stats"])
    g["ray_rank"] = torch.empty((rg,), dtype=torch.int32, device=dev)
    g["rank_ray"] = torch.empty((rg,), dtype=torch.int32, device=dev)
    stream = L.stream_of(dev)
    L.call("psvo_ray_stats", stream, rg, L.ptr(g["ray_nv"]), L.ptr(g["ray_dsum"]), float(step_size), L.ptr(g["stats"]))
    L.call("psvo_hit_rank", stream, rg, L.ptr(g["ray_nv"]), L.ptr(g["ray_rank"]), L.ptr(g["rank_ray"]))
    counts = torch.stack([(g["ray_nv"][:ray_off] > 0).sum(), (q["ray_nv"] > 0).sum()]).to(torch.int32)
    return g, ray_off, counts


@torch.no_grad()
def query_samples(rays_o, rays_d, map_states, step_size, voxel_size, max_distance, noise=None, seed=None,
                  batch=None):
    """Intersection → sampling → compaction for rays_o/rays_d [1, R, 3].

    batch (psvo.dist.GlobalBatch, optional): sample inside the layout of all
    ranks' rays concatenated — the samples then equal the matching rows of a
    single-GPU run on the whole batch with the same seed / noise."""
    dev = rays_o.device
    R = rays_o.numel() // 3
    ray_rank = torch.empty((R,), dtype=torch.int32, device=dev)
    rank_ray = torch.empty((R,), dtype=torch.int32, device=dev)
    stream = L.stream_of(dev)
    exact = batch is not None and batch.world > 1
    with _timed("intersect"):
        q = _intersect_sorted(rays_o, rays_d, map_states["voxel_center_xyz"], map_states["voxel_structure"],
                              voxel_size, max_distance, step_size)
        if exact:
            g, ray_off, counts = _global_rows(q, R, step_size, batch)
        else:
            L.call("psvo_hit_rank", stream, R, L.ptr(q["ray_nv"]), L.ptr(ray_rank), L.ptr(rank_ray))
    if exact:
        st = torch.cat([g["stats"][:8], counts, q["stats"][5:8]]).cpu()  # sync 1
        P, rg_hit, max_ceil = int(st[0]), int(st[1]), int(st[2])
        row_begin, r_hit, visits, flags = int(st[8]), int(st[9]), int(st[10]), int(st[12])
        stats = g["stats"]
        rank_ray_s, hit_src = g["rank_ray"], g
        ray_rank = g["ray_rank"][ray_off:ray_off + R].clone()
        ray_rank = torch.where(ray_rank >= 0, ray_rank - row_begin, ray_rank)
        rank_ray[:r_hit] = g["rank_ray"][row_begin:row_begin + r_hit] - ray_off
        assert rg_hit > 0, "no ray hits the octree (render_helpers.py:388)"
    else:
        st = q["stats"].cpu()  # sync 1
        P, r_hit, max_ceil, visits, flags = int(st[0]), int(st[1]), int(st[2]), int(st[5]), int(st[7])
        row_begin, rg_hit, stats, rank_ray_s, hit_src = 0, r_hit, q["stats"], rank_ray, q
    if flags & 1:
        raise RuntimeError("octree deeper than the DFS level stack (15)")
    assert r_hit > 0, "no ray hits the octree (render_helpers.py:388)"
    max_steps = max_ceil + P
    s_idx = torch.empty((r_hit, max_steps), dtype=torch.int32, device=dev)
    s_depth = torch.empty((r_hit, max_steps), dtype=torch.float32, device=dev)
    s_dist = torch.empty((r_hit, max_steps), dtype=torch.float32, device=dev)
    ray_ns = torch.empty((r_hit,), dtype=torch.int32, device=dev)
    offsets = torch.empty((r_hit + 1,), dtype=torch.int32, device=dev)
    if noise is not None:
        noise = noise.to(device=dev, dtype=torch.float32).contiguous()
        kp = (rg_hit + 199) // 200
        if tuple(noise.shape) != (200, kp, max_steps):
            raise ValueError(f"noise must be [200, {kp}, {max_steps}], got {tuple(noise.shape)}")
    if seed is None:
        if exact:
            raise ValueError("query_samples: a GlobalBatch needs the same explicit seed (or noise) on every rank")
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    with _timed("sample"):
        L.call("psvo_sample_rays_range", stream, row_begin, r_hit, r_hit, max_steps, L.ptr(rank_ray_s),
               L.ptr(hit_src["hit_idx"]), L.ptr(hit_src["hit_t0"]), L.ptr(hit_src["hit_t1"]),
               L.ptr(hit_src["ray_dsum"]), float(step_size), L.ptr(noise), seed, L.ptr(stats), L.ptr(s_idx),
               L.ptr(s_depth), L.ptr(s_dist), L.ptr(ray_ns), L.ptr(offsets))
    st = stats.cpu()  # sync 2
    s_max, m = int(st[3]), int(st[4])
    if exact:  # pad to the global S_max: the composite's first sign change sees the sdf = 1 padding
        s_max = batch.max_int(s_max)
    if int(st[7]) & 2:
        raise RuntimeError("sampler exceeded max_steps")
    leaf = torch.empty((m,), dtype=torch.int32, device=dev)
    t = torch.empty((m,), dtype=torch.float32, device=dev)
    ray_of_sample = torch.empty((m,), dtype=torch.int32, device=dev)
    z_vals = torch.empty((r_hit, s_max), dtype=torch.float32, device=dev)
    mask = torch.empty((r_hit, s_max), dtype=torch.uint8, device=dev)
    with _timed("points"):
        L.call("psvo_sample_points", stream, r_hit, s_max, max_steps, L.ptr(s_idx), L.ptr(s_depth), L.ptr(ray_ns),
               L.ptr(offsets), L.ptr(leaf), L.ptr(t), L.ptr(ray_of_sample), L.ptr(z_vals), L.ptr(mask))
    out = RaySamples()
    out.ray_mask = (ray_rank >= 0).view(1, R)
    out.rank_ray32 = rank_ray[:r_hit]
    out.r_hit, out.P, out.s_max, out.m, out.visits, out.max_steps = r_hit, P, s_max, m, visits, max_steps
    out.z_vals, out.sample_mask = z_vals, mask  # uint8 [R_hit, S_max]
    out.leaf, out.t, out.ray_of_sample, out.offsets, out.ray_ns = leaf, t, ray_of_sample, offsets, ray_ns
    out.s_idx, out.s_depth, out.s_dist = s_idx, s_depth, s_dist
    return out


def render_rays(rays_o, rays_d, map_states, sdf_network, resnet, step_size, voxel_size, truncation, max_voxel_hit,
                max_distance, chunk_size=10000, profiler=None, return_raw=False, noise=None, seed=None,
                return_samples=False, batch=None):
    """render_helpers.py:351-556.  `noise` ([200, K', max_steps]) / `seed`
    select the sampler's uniform noise; by default it is drawn on the device
    from a seed taken from torch's CPU generator."""
    if profiler is not None:
        profiler.tick("ray_intersect")
    smp = query_samples(rays_o, rays_d, map_states, step_size, voxel_size, max_distance, noise, seed, batch)
    if profiler is not None:
        profiler.tok("ray_intersect")
    ro = rays_o.reshape(-1, 3).float().contiguous()
    rd = rays_d.reshape(-1, 3).float().contiguous()
    if smp.m == 0:
        return None, 0
    emb = map_states["voxel_vertex_emb"]
    feats = InterpSamples.apply(ro, rd, emb, smp.leaf, smp.t, smp.ray_of_sample, smp.offsets,
                                map_states["voxel_center_xyz"].float().contiguous(),
                                map_states["voxel_vertex_idx"].int().contiguous(), voxel_size, smp.rank_ray32)
    if profiler is not None:
        profiler.tick("render_core")
    field = sdf_network({"emb": feats, "dists": None})
    if profiler is not None:
        profiler.tok("render_core")
    sdf, weights, color, depth, z_min = CompositeRays.apply(field["sdf"], field["color"], smp.z_vals, smp.offsets,
                                                            smp.ray_ns, truncation)
    out = {
        "weights": weights,
        "color": color,
        "depth": depth,
        "z_vals": smp.z_vals,
        "sdf": sdf,
        "ray_mask": smp.ray_mask,
        "raw": z_min if return_raw else None,
        "rank_ray": smp.rank_ray32,  # hit-ray order for the fused Criterion (not in the reference dict)
    }
    if return_samples:
        out["samples"] = smp
    return out


@torch.enable_grad()
def get_features_vox(samples, map_states, voxel_size):
    """render_helpers.py:104-156 for arbitrary sample points (mesh / eval).
    sampled_point_xyz [M,3] is treated as o + 1·t with o = xyz, t = 0."""
    xyz = samples["sampled_point_xyz"].float().contiguous()
    idx = samples["sampled_point_voxel_idx"].int().contiguous()
    M = xyz.shape[0]
    dev = xyz.device
    zeros = torch.zeros((M,), dtype=torch.float32, device=dev)
    ray_of_sample = torch.arange(M, dtype=torch.int32, device=dev)
    offsets = torch.arange(M + 1, dtype=torch.int32, device=dev)
    feats = InterpSamples.apply(xyz, torch.ones_like(xyz), map_states["voxel_vertex_emb"], idx, zeros,
                                ray_of_sample, offsets, map_states["voxel_center_xyz"].float().contiguous(),
                                map_states["voxel_vertex_idx"].int().contiguous(), voxel_size)
    return {"dists": samples.get("sampled_point_distance"), "emb": feats}


@torch.no_grad()
def get_scores(sdf_network, map_states, voxel_size, bits=8):
    """render_helpers.py:243-294: decoder outputs on a bits³ grid per voxel."""
    feats = map_states["voxel_vertex_idx"]
    points = map_states["voxel_center_xyz"]
    values = map_states["voxel_vertex_emb"]
    chunk_size = 32
    res = bits
    lin = torch.linspace(-0.5, 0.5, res, device=points.device)
    xx, yy, zz = torch.meshgrid(lin, lin, lin, indexing="ij")
    grid_pts = torch.stack([xx, yy, zz], -1).float().reshape(1, -1, 3) * voxel_size
    outs = []
    for i in range(0, points.size(0), chunk_size):
        p = points[i:i + chunk_size]
        xyz = (grid_pts + p.unsqueeze(1)).reshape(-1, 3)
        idx = torch.arange(i, i + p.size(0), device=points.device)[:, None].expand(p.size(0), res ** 3).reshape(-1)
        fi = get_features_vox({"sampled_point_xyz": xyz, "sampled_point_voxel_idx": idx},
                              {"voxel_vertex_idx": feats, "voxel_center_xyz": points, "voxel_vertex_emb": values},
                              voxel_size)
        outs.append(sdf_network.get_values(fi["emb"]).reshape(-1, res ** 3, 4).detach().cpu())
    return torch.cat(outs, 0).view(-1, res, res, res, 4)


@torch.no_grad()
def eval_points(sdf_network, map_states, sampled_xyz, sampled_idx, voxel_size):
    """render_helpers.py:297-328."""
    sampled_idx = sampled_idx.reshape(-1)
    sampled_xyz = sampled_xyz.reshape(-1, 3)
    if sampled_xyz.shape[0] == 0:
        return None
    fi = get_features_vox({"sampled_point_xyz": sampled_xyz, "sampled_point_voxel_idx": sampled_idx}, map_states,
                          voxel_size)
    return sdf_network.get_values(fi["emb"]).reshape(-1, 4)[:, :3].detach().cpu()


# ---------------------------------------------------------------------------
# bundle_adjust_frames on the native engine (psvo_map_step_frames): one C
# call per iteration — rays from the keyframes' current poses, render, loss,
# backward, Adam(embeddings), Adam(decoder) and every keyframe's pose Adam —
# continuing the caller's optimisers' state (exp_avg / exp_avg_sq / step are
# read from and written back to them), so the drop-in loop and this path are
# interchangeable mid-run.
_ENGINES = {}


def _is_adam(opt):
    from .optim import Adam as PsvoAdam
    if not isinstance(opt, (torch.optim.Adam, PsvoAdam)) or len(opt.param_groups) != 1:
        return False
    g = opt.param_groups[0]
    return (not g.get("amsgrad", False) and g.get("weight_decay", 0.0) == 0.0 and not g.get("maximize", False)
            and not g.get("capturable", False) and not g.get("differentiable", False))


def _adam_state(opt, p):
    st = opt.state[p]
    if len(st) == 0:  # as Adam's lazy init
        st["step"] = torch.tensor(0.0)
        st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
    return st


def _engine_for(keyframe_graph, map_states, sdf_network, resnet, loss_criteria, embed_optim, model_optim,
                resnet_optim, voxel_size, step_size, truncation, max_distance, N_rays):
    """The cached MappingEngine for this map / decoder, or None when the
    call is outside what the native iteration covers (then the autograd loop
    below runs — the same kernels)."""
    from .engine import MappingEngine
    emb = map_states.get("voxel_vertex_emb")
    # resnet / resnet_optim (Mapping.do_mapping passes both, mapping.py:195-213) are accepted: the render
    # path never runs the point encoder (get_features_pcd is commented out, render_helpers.py:481), so its
    # parameters never get a gradient; bundle_adjust_frames checks that resnet_optim's step is a no-op
    if model_optim is None or embed_optim is None:
        return None
    if not (_is_adam(embed_optim) and _is_adam(model_optim)):
        return None
    if not (isinstance(emb, torch.Tensor) and emb.is_cuda and emb.dtype == torch.float32 and emb.is_contiguous()):
        return None
    if [p for p in embed_optim.param_groups[0]["params"]] != [emb]:
        return None
    params = sdf_network.fused_params() if hasattr(sdf_network, "fused_params") else None
    if params is None or not sdf_network.can_fuse(emb[:1]) or list(model_optim.param_groups[0]["params"]) != params:
        return None
    ge, gm = embed_optim.param_groups[0], model_optim.param_groups[0]
    if tuple(ge["betas"]) != tuple(gm["betas"]) or ge["eps"] != gm["eps"]:
        return None
    if not all(hasattr(loss_criteria, a) for a in ("rgb_weight", "depth_weight", "fs_weight", "sdf_weight",
                                                   "truncation", "max_dpeth")):
        return None
    # one truncation drives the engine's compositing and its loss: the render's (render_rays' argument)
    # and the criterion's (criteria sdf_truncation) must agree — Mapping passes the same value
    if float(truncation) != float(loss_criteria.truncation):
        return None
    if resnet_optim is not None:
        mine = {id(emb)} | {id(p) for p in params}
        if any(id(p) in mine for g in resnet_optim.param_groups for p in g["params"]):
            return None
    for kf in keyframe_graph:
        if not (hasattr(kf, "sample_rays") and hasattr(kf, "rays_d") and getattr(kf, "pose", None) is not None):
            return None
    key = (emb.data_ptr(), emb.shape[0], id(sdf_network), map_states["voxel_center_xyz"].data_ptr(),
           map_states["voxel_center_xyz"].shape[0], map_states["voxel_structure"].data_ptr(),
           map_states["voxel_vertex_idx"].data_ptr(), float(voxel_size), float(step_size), float(truncation),
           float(max_distance), float(loss_criteria.max_dpeth),
           tuple(float(getattr(loss_criteria, a)) for a in ("rgb_weight", "depth_weight", "fs_weight", "sdf_weight")))
    eng = _ENGINES.get(key)
    if eng is None:
        if len(_ENGINES) > 4:
            _ENGINES.clear()
        crit = {"rgb_weight": loss_criteria.rgb_weight, "depth_weight": loss_criteria.depth_weight,
                "fs_weight": loss_criteria.fs_weight, "sdf_weight": loss_criteria.sdf_weight}
        eng = MappingEngine(map_states, sdf_network, voxel_size, step_size, truncation=loss_criteria.truncation,
                            max_distance=max_distance, criteria=crit, max_depth=loss_criteria.max_dpeth,
                            betas=tuple(ge["betas"]), eps=ge["eps"])
        _ENGINES[key] = eng
    return eng


_SIDE_STREAMS = {}


def _side_stream(dev):
    """The pixel draws' stream, one per device for the process: creating a
    stream costs the host ≈ 0.35 ms, a third of a call's fixed cost
    (PSVO_BA_PROFILE=1, config B)."""
    key = torch.device(dev).index if torch.device(dev).index is not None else torch.cuda.current_device()
    s = _SIDE_STREAMS.get(key)
    if s is None:
        s = _SIDE_STREAMS[key] = torch.cuda.Stream(device=dev)
    return s


class _CallClock:
    """PSVO_BA_PROFILE=1: host timestamps of one bundle_adjust_frames call's
    phases (setup, each step's submission, write-back) to stderr — where a
    call's fixed cost goes (bench.py's per-call overhead)."""

    def __init__(self):
        import time
        self.on = os.environ.get("PSVO_BA_PROFILE") == "1"
        self.t0 = time.perf_counter()
        self.marks = []

    def __call__(self, what):
        if self.on:
            import time
            self.marks.append((what, time.perf_counter() - self.t0))

    def report(self):
        if self.on and self.marks:
            import sys
            sys.stderr.write("ba-call " + " ".join(f"{w}={t * 1e3:.3f}" for w, t in self.marks) + "\n")


def _pose_pack_key(kfs, pose_params, pose_st, upd, dev):
    """Identity + version of every tensor the packed poses / moments / steps
    are made from (an in-place write anywhere bumps a version)."""
    key = [str(dev), tuple(upd)]
    for f in range(len(kfs)):
        p = pose_params[f]
        key.append((id(p), p._version, p.data_ptr()))
        st = pose_st[f]
        if st is not None:
            for n in ("exp_avg", "exp_avg_sq", "step"):
                t = st[n]
                key.append((id(t), t._version, t.data_ptr()))
    return tuple(key)


def _bundle_adjust_engine(eng, keyframe_graph, embed_optim, model_optim, N_rays, num_iterations, update_pose,
                          noise, seed_fn=None, lookahead=True):
    clk = _CallClock()
    emb = eng.emb
    params = eng.params
    st_e = _adam_state(embed_optim, emb)
    st_d = [_adam_state(model_optim, p) for p in params]
    steps = {int(st_e["step"].item())} | {int(st["step"].item()) for st in st_d}
    if len(steps) != 1:
        return False  # parameters at different Adam steps: the engine steps them together
    adam_step = steps.pop()
    dev = emb.device
    # the keyframes' pose optimisers: checked (host only) before anything is
    # queued, so a call that falls back to the autograd loop has drawn nothing
    kfs = list(keyframe_graph)
    upd = [bool(kf.stamp != 0 and update_pose and getattr(kf, "optim", None) is not None) for kf in kfs]
    pose_params = [kf.pose.data for kf in kfs]
    pose_st = [None] * len(kfs)
    lr_pose = None
    for f, kf in enumerate(kfs):
        if not upd[f]:
            continue
        if not _is_adam(kf.optim):
            return False
        lr = kf.optim.param_groups[0]["lr"]
        if lr_pose is not None and lr != lr_pose:
            return False
        lr_pose = lr
        if tuple(kf.optim.param_groups[0]["betas"]) != tuple(embed_optim.param_groups[0]["betas"]):
            return False
        pose_st[f] = _adam_state(kf.optim, pose_params[f])
    clk("state")
    # keyframes whose sample_rays is the reference's uniform gumbel top-k
    # (frame.py:83-85) are sampled together in one native call with the
    # gathers fused (psvo.sample_util.sample_frames); others through their own
    # sample_rays and the boolean-mask gathers
    batched = all(getattr(kf, "uniform_pixel_sampling", False) for kf in kfs)
    cat = lambda xs: xs[0] if len(xs) == 1 else torch.cat(xs)  # noqa: E731

    def draw(it, out=None):
        """iteration it's pixels (dirs_cam, rgb, depth) and sampler seed, in
        the order the reference draws them (pixels, then the sampler noise)"""
        if batched:
            d_all, c_all, z_all = sample_util.sample_frames(kfs, N_rays, out=out)
        else:
            dirs, rgbs, depths = [], [], []
            for kf in kfs:
                kf.sample_rays(N_rays)
                idx = getattr(kf, "sample_idx", None)
                if idx is None:
                    idx = kf.sample_mask.reshape(-1).nonzero().squeeze(1)
                idx = idx.to(dev)
                if idx.numel() != N_rays:
                    raise RuntimeError("bundle_adjust_frames: sample_rays gave %d rays, expected %d"
                                       % (idx.numel(), N_rays))
                dirs.append(kf.rays_d.reshape(-1, 3).to(dev)[idx])
                rgbs.append(kf.rgb.reshape(-1, 3).to(dev)[idx])
                depths.append(kf.depth.reshape(-1).to(dev)[idx])
            d_all, c_all, z_all = cat(dirs), cat(rgbs), cat(depths)
        d_all = d_all.reshape(-1, 3).to(torch.float32).contiguous()
        nz = noise(it) if callable(noise) else None
        if seed_fn is not None:
            seed = int(seed_fn(it))
        else:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if nz is None else 0
        return d_all, c_all, z_all, nz, seed

    # the next iteration's pixels are drawn before this one's step, so the
    # engine queues its query right after this step's backward
    # (psvo_map_frames.next_dirs_cam); injected noise (tests) runs unpipelined.
    # Pipelined, the draws run on a stream of their own: they depend on nothing
    # the steps write, and on the step's stream they would sit between the
    # look-ahead query and the next render
    ahead = lookahead and not callable(noise)
    main = torch.cuda.current_stream(dev)
    side = _side_stream(dev) if ahead and num_iterations > 1 else None
    # the batched draws' output ring: draw j + 4 (queued on `side` at the top
    # of iteration j + 3) overwrites draw j's buffers, which step j reads on
    # main.  The host queues it only after step j + 2 read back its query's
    # statistics, which the look-ahead sampler queued on main after step
    # j + 1's backward writes — after all of step j (and the auxiliary work
    # step j joined into main) on the device: the ring needs no event.
    ring = []
    if side is not None and batched:
        nt = len(kfs) * N_rays
        for _ in range(4):
            r3 = (torch.empty(nt, 3, dtype=torch.float32, device=dev),
                  torch.empty(nt, 3, dtype=torch.float32, device=dev),
                  torch.empty(nt, dtype=torch.float32, device=dev))
            for t in r3:
                t.record_stream(side)  # freed at the call's end: after the side stream's draws
            ring.append(r3)
    if side is not None:
        side.wait_stream(main)  # the keyframes as the caller left them (and the ring's blocks)
    clk("side")

    # each next draw is queued as soon as its step is (beside the persistent
    # decoder kernels); ordered after the previous step's decoder backward it
    # measured slower (round 4, config B: 1.000-1.059 vs 0.985-1.000 ms)
    # PSVO_BA_DRAW_AFTER_STEP=1 (measured switch): each draw waits until the
    # previous step's kernels on the caller's stream are done, so that it runs
    # beside the next step's latency-bound query instead of beside the
    # persistent decoder backward
    after_step = os.environ.get("PSVO_BA_DRAW_AFTER_STEP") == "1"
    step_done = [None]

    def draw_ahead(it):
        if side is None:
            return draw(it), None
        if after_step and step_done[0] is not None:
            side.wait_event(step_done[0])
        # the batched draw writes into a ring of buffers made once per call
        # (below): no tensor of the loop is freed with record_stream(main),
        # whose allocator event — recorded on main at the free, with the
        # runtime's default system-scope release — put a marker packet between
        # the step's kernels: ≈ 15 µs of idle GPU per iteration between the
        # sampler and the interpolation, measured (rocprofv3 timeline, config B)
        bufs = ring[it % len(ring)] if ring else None
        with torch.cuda.stream(side):
            out = draw(it, bufs)
        if it == 0:
            clk("draw")
        if bufs is None:
            for t in out[:3]:
                t.record_stream(main)  # freed blocks are reused only after the steps that read them
        if it > 0:  # later draws are ordered by the engine (next_stream), no event needed
            return out, None
        ev = torch.cuda.Event()
        ev.record(side)
        return out, ev

    # the first pixels are queued first: the GPU draws them while the host
    # binds the optimiser state and packs the poses (the call's fixed cost)
    cur, cur_ready = draw_ahead(0)
    clk("draw0")
    eng.bind_adam(st_e["exp_avg"], st_e["exp_avg_sq"], [st["exp_avg"] for st in st_d],
                  [st["exp_avg_sq"] for st in st_d])
    clk("bind")
    eng.refresh_tree()  # the map may have grown / changed in place since the engine was made
    clk("tree")
    eng.set_lr(embed_optim.param_groups[0]["lr"], model_optim.param_groups[0]["lr"])
    # keyframe poses [F, 6] and their Adam state on the device — packed again
    # only when a tensor changed since this engine's last call wrote them back
    # (torch's version counters; the packed copies then still hold exactly the
    # written-back values): the repack's ~15 small torch ops were most of a
    # call's host setup
    pack_key = _pose_pack_key(kfs, pose_params, pose_st, upd, dev)
    cached = getattr(eng, "_pose_pack", None)
    if cached is not None and cached[0] == pack_key:
        poses, pm, pv, pstep = cached[1], cached[2], cached[3], list(cached[4])
    else:
        poses = torch.stack([p.detach().to(dev, torch.float32).reshape(6) for p in pose_params]).contiguous()
        pstep = [0] * len(kfs)
        zero6 = None
        m_rows, v_rows = [], []
        for f in range(len(kfs)):
            st = pose_st[f]
            if st is None:
                if zero6 is None:
                    zero6 = torch.zeros(6, dtype=torch.float32, device=dev)
                m_rows.append(zero6)
                v_rows.append(zero6)
                continue
            m_rows.append(st["exp_avg"].to(dev, torch.float32).reshape(6))
            v_rows.append(st["exp_avg_sq"].to(dev, torch.float32).reshape(6))
            pstep[f] = int(st["step"].item())
        pm = torch.stack(m_rows).contiguous()  # the poses' Adam moments [F, 6], one gather each
        pv = torch.stack(v_rows).contiguous()
    eng._pose_pack = None  # the packed copies change under the steps below
    if cur_ready is not None:
        main.wait_event(cur_ready)
    clk("poses")
    # batched draws run two iterations ahead, each queued after its step's
    # sample selection (psvo_engine_gate_stream), so that they overlap the
    # decoder instead of the latency-bound query / selection kernels:
    # config B 0.695 vs 0.722 ms per iteration ungated (profiles/r06_ab_draw.txt);
    # PSVO_BA_DRAW_GATE=0 queues each draw one ahead, ungated
    gate = (ahead and batched and os.environ.get("PSVO_BA_DRAW_GATE", "1") != "0"
            and hasattr(L.lib(), "psvo_engine_gate_stream"))  # (an older A/B build has no gate)
    pending = None
    if gate and num_iterations > 1:
        pending = draw_ahead(1)
    for it in range(num_iterations):
        # the engine orders the look-ahead's pose step (reads nxt's dirs) after
        # the draw queued on `side` (next_stream), and with it the next step
        if gate:
            nxt, _ = pending if pending is not None else (None, None)
        else:
            nxt, _ = draw_ahead(it + 1) if ahead and it + 1 < num_iterations else (None, None)
        d_all, c_all, z_all, nz, seed = cur
        adam_step += 1
        cur_steps = [pstep[f] + 1 if upd[f] else 0 for f in range(len(kfs))]
        dp = eng.grad_exchange is not None
        eng.step_frames(d_all, N_rays, poses, pm, pv, cur_steps, lr_pose or 0.0, c_all, z_all, seed, noise=nz,
                        adam_step=adam_step, apply_adam=not dp, next_dirs_cam=nxt[0] if nxt else None,
                        next_seed=nxt[4] if nxt else 0, next_stream=side if nxt else None,
                        want_loss=eng.ba_loss, next_depth=nxt[2] if nxt else None)
        if dp:  # data parallel: sum the union-batch gradient over ranks, then the same Adam everywhere
            eng.grad_exchange()
            eng.adam()
        pstep = [c if upd[f] else pstep[f] for f, c in enumerate(cur_steps)]
        if after_step and side is not None:
            step_done[0] = step_done[0] or torch.cuda.Event()
            step_done[0].record(main)
        if gate:  # the draw two ahead, behind this step's selection (the ring of 4 stays safe: see above)
            pending = None
            if it + 2 < num_iterations:
                L.call("psvo_engine_gate_stream", eng.handle, ctypes.c_void_p(side.cuda_stream))
                pending = draw_ahead(it + 2)
        cur = nxt if nxt is not None else (draw(it + 1) if it + 1 < num_iterations else None)
        if it < 2 or it == num_iterations - 1:
            clk(f"step{it}")
    if side is not None:
        main.wait_stream(side)  # frames' sample_mask / sample_idx of the last draw
    # write back: optimiser steps, pose parameters and their Adam state
    with torch.no_grad():
        for st in [st_e] + st_d:
            st["step"].fill_(float(adam_step))
        for f, kf in enumerate(kfs):
            if not upd[f]:
                continue
            pose_params[f].copy_(poses[f].to(pose_params[f].device).reshape(pose_params[f].shape))
            st = kf.optim.state[pose_params[f]]
            st["exp_avg"].copy_(pm[f].to(st["exp_avg"].device).reshape(st["exp_avg"].shape))
            st["exp_avg_sq"].copy_(pv[f].to(st["exp_avg_sq"].device).reshape(st["exp_avg_sq"].shape))
            st["step"].fill_(float(pstep[f]))
    # the caller's tensors now equal the packed copies: the next call reuses
    # them unless something writes the poses / their Adam state in between
    eng._pose_pack = (_pose_pack_key(kfs, pose_params, pose_st, upd, dev), poses, pm, pv, tuple(pstep))
    clk("writeback")
    clk.report()
    return True


def bundle_adjust_frames(keyframe_graph, map_states, sdf_network, resnet, loss_criteria, voxel_size, step_size,
                         N_rays=512, num_iterations=10, truncation=0.1, max_voxel_hit=10, max_distance=10,
                         learning_rate=[1e-2, 5e-3], embed_optim=None, model_optim=None, resnet_optim=None,
                         update_pose=True, noise=None, use_engine=True, engine=None, seed_fn=None, lookahead=True):
    """render_helpers.py:559-676 — mapping's render-and-optimise loop.

    Runs on the native engine (one psvo_map_step_frames call per iteration)
    whenever the optimisers are plain Adam over the map embeddings / fused
    decoder — including Mapping.do_mapping's call with the point encoder and
    its optimiser (mapping.py:195-213), which the reference's render path never
    runs (:481), so that optimiser's step is a no-op; otherwise the autograd
    loop below (same kernels).  Keywords beyond the reference signature:
    `noise` — a callable iteration → sampler noise [200, K', max_steps]
    (parity tests); `engine` — a prepared psvo.engine.MappingEngine to use
    (e.g. one with a data-parallel EngineExchange: every rank passes the
    keyframes of its share of the union batch); `seed_fn` — iteration →
    sampler seed (must agree across ranks when data parallel); `lookahead` —
    queue each next iteration's query beside the current step's weight
    gradients (the default; same results, tests compare both)."""
    if use_engine:
        eng = engine
        if resnet_optim is not None and num_iterations > 0:
            # the reference zero_grads every optimiser each iteration (:667-669): set_to_none leaves the
            # encoder's gradients None, backward never reaches them (:481), so its optim.step() (:674-676)
            # is a no-op — torch optimisers skip parameters whose grad is None.  Anything else (grads kept
            # as zero tensors: Adam would still move them by its momentum) takes the autograd loop.
            resnet_optim.zero_grad()
            if any(p.grad is not None for g in resnet_optim.param_groups for p in g["params"]):
                eng = None
                use_engine = False
    if use_engine:
        if eng is None:
            eng = _engine_for(keyframe_graph, map_states, sdf_network, resnet, loss_criteria, embed_optim,
                              model_optim, resnet_optim, voxel_size, step_size, truncation, max_distance, N_rays)
        if eng is not None and _bundle_adjust_engine(eng, keyframe_graph, embed_optim, model_optim, N_rays,
                                                     num_iterations, update_pose, noise, seed_fn, lookahead):
            return
        if engine is not None:
            raise RuntimeError("bundle_adjust_frames: the given engine cannot run this call (optimiser state)")
    optimizers = [embed_optim]
    if model_optim is not None:
        optimizers += [model_optim]
    if resnet_optim is not None:
        optimizers += [resnet_optim]
    for keyframe in keyframe_graph:
        if keyframe.stamp != 0 and update_pose:
            optimizers += [keyframe.optim]
    for _ in range(num_iterations):
        rays_o, rays_d, rgb_samples, depth_samples = [], [], [], []
        for frame in keyframe_graph:
            pose = frame.get_pose().cuda()
            frame.sample_rays(N_rays)
            sample_mask = frame.sample_mask.cuda()
            sampled_rays_d = frame.rays_d[sample_mask].cuda()
            R = pose[:3, :3].transpose(-1, -2)
            sampled_rays_d = sampled_rays_d @ R
            sampled_rays_o = pose[:3, 3].reshape(1, -1).expand_as(sampled_rays_d)
            rays_d += [sampled_rays_d]
            rays_o += [sampled_rays_o]
            rgb_samples += [frame.rgb.cuda()[sample_mask]]
            depth_samples += [frame.depth.cuda()[sample_mask]]
        rays_d = torch.cat(rays_d, dim=0).unsqueeze(0)
        rays_o = torch.cat(rays_o, dim=0).unsqueeze(0)
        rgb_samples = torch.cat(rgb_samples, dim=0).unsqueeze(0)
        depth_samples = torch.cat(depth_samples, dim=0).unsqueeze(0)
        final_outputs = render_rays(rays_o, rays_d, map_states, sdf_network, resnet, step_size, voxel_size,
                                    truncation, max_voxel_hit, max_distance,
                                    noise=noise(_) if callable(noise) else None)
        loss, _ = loss_criteria(final_outputs, (rgb_samples, depth_samples))
        for optim in optimizers:
            optim.zero_grad()
        loss.backward()
        for optim in optimizers:
            optim.step()


def track_frame(frame_pose, curr_frame, map_states, sdf_network, resnet, loss_criteria, voxel_size, N_rays=512,
                step_size=0.05, num_iterations=10, truncation=0.1, learning_rate=1e-3, max_voxel_hit=10,
                max_distance=10, profiler=None, depth_variance=False, noise=None):
    """render_helpers.py:679-761 — pose-only optimisation of one frame.
    noise: a callable iteration → the sampler noise (tests; the reference
    draws it inside InverseCDFRaySampling)."""
    init_pose = deepcopy(frame_pose).cuda()
    init_pose.requires_grad_(True)
    optim = torch.optim.Adam(init_pose.parameters(), lr=learning_rate)
    hit_mask = None
    for it in range(num_iterations):
        curr_frame.sample_rays(N_rays)
        sample_mask = curr_frame.sample_mask
        ray_dirs = curr_frame.rays_d[sample_mask].unsqueeze(0).cuda()
        rgb = curr_frame.rgb[sample_mask].cuda()
        depth = curr_frame.depth[sample_mask].cuda()
        ray_dirs_iter = (ray_dirs.squeeze(0) @ init_pose.rotation().transpose(-1, -2)).unsqueeze(0)
        ray_start_iter = init_pose.translation().reshape(1, 1, -1).expand_as(ray_dirs_iter).cuda().contiguous()
        final_outputs = render_rays(ray_start_iter, ray_dirs_iter, map_states, sdf_network, resnet, step_size,
                                    voxel_size, truncation, max_voxel_hit, max_distance,
                                    profiler=profiler if it == 0 else None,
                                    noise=noise(it) if callable(noise) else None)
        hit_mask = final_outputs["ray_mask"].view(N_rays)
        final_outputs["ray_mask"] = hit_mask
        loss, _ = loss_criteria(final_outputs, (rgb, depth), weight_depth_loss=depth_variance)
        optim.zero_grad()
        loss.backward()
        optim.step()
    return init_pose, optim, hit_mask
