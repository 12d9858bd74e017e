"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference's render-and-optimise hot path:
  octree export → ray/octree intersection → sort/trim → inverse-CDF sampling
  → trilinear interpolation → NRGBD decoder → SDF-weight compositing →
  Criterion loss → (torch-CPU autograd) backward.

Kernels come from svo_oracle.c (ctypes); the host-side logic is restated in
torch-CPU fp32 here, each function citing the reference lines it follows.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module.  The product package never does.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libsvo_oracle.so")
_lib = None

MAX_DEPTH = 10.0  # voxel_helpers.py:24
N_MAX_HITS = 50   # voxel_helpers.py:561 (max_voxel_hit is ignored by the reference)
SAMPLER_G = 200   # voxel_helpers.py:300
SAMPLER_CHUNK = 4 * SAMPLER_G  # voxel_helpers.py:331


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, i64, f32, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_float, ctypes.c_int
        L.oracle_octree_new.restype = vp
        L.oracle_octree_new.argtypes = [i32]
        L.oracle_octree_free.argtypes = [vp]
        L.oracle_octree_insert.argtypes = [vp, vp, i64]
        L.oracle_octree_count.restype = i64
        L.oracle_octree_count.argtypes = [vp]
        L.oracle_octree_export.argtypes = [vp, vp, vp, vp]
        L.oracle_svo_intersect.restype = i64
        L.oracle_svo_intersect.argtypes = [i64, vp, vp, vp, vp, f32, i32, vp, vp, vp]
        L.oracle_inverse_cdf.argtypes = [i32, i32, i32, i32, f32] + [vp] * 9
        L.oracle_ball_intersect.argtypes = [i32, i32, i32, f32, i32] + [vp] * 6
        L.oracle_aabb_intersect.argtypes = [i32, i32, i32, f32, i32] + [vp] * 6
        L.oracle_triangle_intersect.argtypes = [i32, i32, i32, f32, f32, i32] + [vp] * 6
        L.oracle_uniform_sampling.argtypes = [i32, i32, i32, i32, f32] + [vp] * 7
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.c_void_p)


# --------------------------------------------------------------------------
# Octree build / export — octree.cpp:104-294, :561-687; mapping.py:300-406
# --------------------------------------------------------------------------
class OracleOctree:
    def __init__(self, grid_dim: int):
        self._h = lib().oracle_octree_new(int(grid_dim))

    def insert(self, vox: np.ndarray):
        v = np.ascontiguousarray(vox, dtype=np.int32)
        lib().oracle_octree_insert(self._h, _ptr(v), int(v.shape[0]))

    def count(self) -> int:
        return int(lib().oracle_octree_count(self._h))

    def export(self):
        n = self.count()
        voxels = np.zeros((n, 4), np.float32)
        children = np.zeros((n, 8), np.float32)
        features = np.zeros((n, 8), np.int32)
        lib().oracle_octree_export(self._h, _ptr(voxels), _ptr(children), _ptr(features))
        return voxels, children, features

    def close(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.oracle_octree_free(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def map_states_from_export(voxels, children, features, voxel_size, embeddings):
    """mapping.py:328-377 — centres, [N,9] structure, vertex ids."""
    vox = torch.from_numpy(np.asarray(voxels, np.float32))
    ch = torch.from_numpy(np.asarray(children, np.float32))
    centres = (vox[:, :3] + vox[:, -1:] / 2) * voxel_size
    structure = torch.cat([ch, vox[:, -1:]], -1).int()
    return {
        "voxel_vertex_idx": torch.from_numpy(np.asarray(features, np.int32)),
        "voxel_center_xyz": centres.float(),
        "voxel_structure": structure,
        "voxel_vertex_emb": embeddings,
    }


# --------------------------------------------------------------------------
# Intersection — voxel_helpers.py:110-166 (kernel) + :557-595 (sort/trim)
# --------------------------------------------------------------------------
def svo_intersect_flat(ray_start, ray_dir, centres, structure, voxel_size, n_max=N_MAX_HITS):
    """Per-ray DFS hits in emission order; returns (idx, t_in, t_out, visits)."""
    rs = np.ascontiguousarray(ray_start, np.float32).reshape(-1, 3)
    rd = np.ascontiguousarray(ray_dir, np.float32).reshape(-1, 3)
    pts = np.ascontiguousarray(centres, np.float32)
    ch = np.ascontiguousarray(structure, np.int32)
    n = rs.shape[0]
    idx = np.empty((n, n_max), np.int32)
    t0 = np.empty((n, n_max), np.float32)
    t1 = np.empty((n, n_max), np.float32)
    visits = lib().oracle_svo_intersect(n, _ptr(rs), _ptr(rd), _ptr(pts), _ptr(ch), float(voxel_size), int(n_max),
                                        _ptr(idx), _ptr(t0), _ptr(t1))
    if visits < 0:
        raise RuntimeError("oracle DFS stack overflow")
    return idx, t0, t1, int(visits)


def ray_intersect_vox(rays_o, rays_d, centres, structure, voxel_size, max_distance=10.0):
    """voxel_helpers.py:557-595 with a stable sort on DFS emission order."""
    S, N = rays_o.shape[:2]
    idx, t0, t1, _ = svo_intersect_flat(rays_o.detach().reshape(-1, 3).numpy(), rays_d.detach().reshape(-1, 3).numpy(),
                                        centres.detach().numpy(), structure.numpy(), voxel_size)
    pts_idx = torch.from_numpy(idx).reshape(S, N, -1)
    min_depth = torch.from_numpy(t0).reshape(S, N, -1)
    max_depth = torch.from_numpy(t1).reshape(S, N, -1)
    miss = pts_idx.eq(-1)
    min_depth = min_depth.masked_fill(miss, max_distance)
    max_depth = max_depth.masked_fill(miss, max_distance)
    min_depth, order = torch.sort(min_depth, dim=-1, stable=True)
    max_depth = max_depth.gather(-1, order)
    pts_idx = pts_idx.gather(-1, order)
    pts_idx[min_depth > max_distance] = -1
    miss = pts_idx.eq(-1)
    min_depth = min_depth.masked_fill(miss, max_distance)
    max_depth = max_depth.masked_fill(miss, max_distance)
    P = int(pts_idx.ne(-1).sum(-1).max())
    out = {
        "min_depth": min_depth[..., :P],
        "max_depth": max_depth[..., :P],
        "intersected_voxel_idx": pts_idx[..., :P],
    }
    hits = out["intersected_voxel_idx"].ne(-1).any(-1)
    return out, hits


# --------------------------------------------------------------------------
# Sampling — voxel_helpers.py:288-374 (host wrapper) + :637-663 (ray_sample)
# --------------------------------------------------------------------------
def sampler_layout(n_rays):
    """K' (rays per sampler slot block) and the padded ray count H."""
    kp = int(math.ceil(n_rays / SAMPLER_G))
    return kp, kp * SAMPLER_G


def inverse_cdf_sampling(pts_idx, min_depth, max_depth, probs, steps, fixed_step_size=-1.0, noise=None,
                         deterministic=False, generator=None):
    """Returns (sampled_idx, depth, dists, noise_used) as the reference host
    wrapper does; `noise` (shape [200, K', max_steps]) may be injected."""
    N, P = pts_idx.shape
    kp, H = sampler_layout(N)
    if H > N:  # pad with copies of row 0 (voxel_helpers.py:303-310)
        pad = H - N
        pts_idx = torch.cat([pts_idx, pts_idx[:1].expand(pad, P)], 0)
        min_depth = torch.cat([min_depth, min_depth[:1].expand(pad, P)], 0)
        max_depth = torch.cat([max_depth, max_depth[:1].expand(pad, P)], 0)
        probs = torch.cat([probs, probs[:1].expand(pad, P)], 0)
        steps = torch.cat([steps, steps[:1].expand(pad)], 0)
    pts_idx = pts_idx.reshape(SAMPLER_G, kp, P).int().contiguous()
    min_depth = min_depth.reshape(SAMPLER_G, kp, P).float().contiguous()
    max_depth = max_depth.reshape(SAMPLER_G, kp, P).float().contiguous()
    probs = probs.reshape(SAMPLER_G, kp, P).float().contiguous()
    steps = steps.reshape(SAMPLER_G, kp).float().contiguous()
    max_steps = int(steps.ceil().long().max()) + P
    if noise is None:
        if deterministic:
            noise = torch.full((SAMPLER_G, kp, max_steps), 0.5)
        else:
            noise = torch.rand((SAMPLER_G, kp, max_steps), generator=generator).clamp(min=0.001, max=0.999)
    assert tuple(noise.shape) == (SAMPLER_G, kp, max_steps), (noise.shape, (SAMPLER_G, kp, max_steps))
    noise = noise.float().contiguous()
    parts = []
    for c0 in range(0, kp, SAMPLER_CHUNK):  # voxel_helpers.py:331-343
        c1 = min(kp, c0 + SAMPLER_CHUNK)
        w = c1 - c0
        a_idx = pts_idx[:, c0:c1].contiguous().numpy()
        a_lo = min_depth[:, c0:c1].contiguous().numpy()
        a_hi = max_depth[:, c0:c1].contiguous().numpy()
        a_nz = noise[:, c0:c1].contiguous().numpy()
        a_pr = probs[:, c0:c1].contiguous().numpy()
        a_st = steps[:, c0:c1].contiguous().numpy()
        o_idx = np.full((SAMPLER_G, w, max_steps), -1, np.int32)
        o_dep = np.zeros((SAMPLER_G, w, max_steps), np.float32)
        o_dis = np.zeros((SAMPLER_G, w, max_steps), np.float32)
        lib().oracle_inverse_cdf(SAMPLER_G, w, P, max_steps, float(fixed_step_size), _ptr(a_idx), _ptr(a_lo),
                                 _ptr(a_hi), _ptr(a_nz), _ptr(a_pr), _ptr(a_st), _ptr(o_idx), _ptr(o_dep),
                                 _ptr(o_dis))
        parts.append((torch.from_numpy(o_idx), torch.from_numpy(o_dep), torch.from_numpy(o_dis)))
    s_idx, s_dep, s_dis = [torch.cat([p[i] for p in parts], 1).reshape(H, -1)[:N] for i in range(3)]
    max_len = int(s_idx.ne(-1).sum(-1).max())
    return s_idx[:, :max_len], s_dep[:, :max_len], s_dis[:, :max_len], noise


def sequential_row_sums(dists):
    """Σ over the last dim, accumulated left to right in fp32 (the depth-sorted
    hit order).  torch leaves a reduction's order unspecified (CPU: vectorised
    cascade; CUDA: tree); this is the order the HIP kernel fixes."""
    d = dists.detach().numpy()
    acc = np.zeros(d.shape[:-1], np.float32)
    for j in range(d.shape[-1]):
        acc = (acc + d[..., j]).astype(np.float32)
    return torch.from_numpy(acc)


def ray_sample(intersection, step_size, noise=None, deterministic=False, generator=None, sum_order="torch"):
    """voxel_helpers.py:637-663.  sum_order "torch": dists.sum(-1) as the
    reference writes it (torch-CPU order); "sequential": sequential_row_sums."""
    idx = intersection["intersected_voxel_idx"]
    dists = (intersection["max_depth"] - intersection["min_depth"]).masked_fill(idx.eq(-1), 0)
    dsum = dists.sum(dim=-1) if sum_order == "torch" else sequential_row_sums(dists)
    probs = dists / dsum.unsqueeze(-1)
    steps = dsum / step_size
    s_idx, s_dep, s_dis, noise = inverse_cdf_sampling(idx, intersection["min_depth"], intersection["max_depth"],
                                                      probs, steps, -1.0, noise, deterministic, generator)
    s_dis = s_dis.clamp(min=0.0)
    s_dep = s_dep.masked_fill(s_idx.eq(-1), MAX_DEPTH)
    s_dis = s_dis.masked_fill(s_idx.eq(-1), 0.0)
    return {"sampled_point_depth": s_dep, "sampled_point_distance": s_dis, "sampled_point_voxel_idx": s_idx}, noise


# --------------------------------------------------------------------------
# Interpolation — render_helpers.py:46-156
# --------------------------------------------------------------------------
_CORNERS = torch.tensor([[(k >> 2) & 1, (k >> 1) & 1, k & 1] for k in range(8)], dtype=torch.float32)


def interp_features(xyz, leaf_idx, centres, vertex_idx, embeddings, voxel_size):
    """feats[M,16] = Σ_k w_k(p) E[vertex_idx[leaf, k]], p = (x-c)/voxel + 0.5."""
    li = leaf_idx.long()
    c = centres[li]
    e = embeddings[vertex_idx[li].long()]            # [M,8,D]
    p = ((xyz - c) / voxel_size + 0.5).unsqueeze(1)  # [M,1,3]
    q = _CORNERS.to(p.dtype).unsqueeze(0)
    w = (p * q + (1 - p) * (1 - q)).prod(dim=-1, keepdim=True)
    return (w * e).sum(1)


# --------------------------------------------------------------------------
# Decoder — nrgbd.py:80-146 for depth 2, embedder 'none', skips [] (all configs)
# --------------------------------------------------------------------------
def decoder_params_init(width=128, in_dim=16, sdf_dim=128, seed=0):
    """Same shapes/order as nrgbd.Decoder.state_dict(); nn.Linear default init."""
    g = torch.Generator().manual_seed(seed)

    def lin(i, o):
        bound = 1.0 / math.sqrt(i)
        w = (torch.rand((o, i), generator=g) * 2 - 1) * bound
        b = (torch.rand((o,), generator=g) * 2 - 1) * bound
        return w, b

    p = {}
    p["pts_linears.0.weight"], p["pts_linears.0.bias"] = lin(in_dim, width)
    p["pts_linears.1.weight"], p["pts_linears.1.bias"] = lin(width, width)
    p["sdf_out.weight"], p["sdf_out.bias"] = lin(width, 1 + sdf_dim)
    p["color_out.0.weight"], p["color_out.0.bias"] = lin(sdf_dim + in_dim, width)
    p["color_out.2.weight"], p["color_out.2.bias"] = lin(width, 3)
    return p


def decoder_forward(params, x):
    """nrgbd.py:116-146 → (color [M,3], sdf [M])."""
    F = torch.nn.functional
    h = F.relu(F.linear(x, params["pts_linears.0.weight"], params["pts_linears.0.bias"]))
    h = F.relu(F.linear(h, params["pts_linears.1.weight"], params["pts_linears.1.bias"]))
    o = F.linear(h, params["sdf_out.weight"], params["sdf_out.bias"])
    sdf, feat = o[:, :1], o[:, 1:]
    hc = F.relu(F.linear(torch.cat([feat, x], -1), params["color_out.0.weight"], params["color_out.0.bias"]))
    rgb = torch.sigmoid(F.linear(hc, params["color_out.2.weight"], params["color_out.2.bias"]))
    return rgb, sdf[:, 0]


def decoder_margins(params, x):
    """For decoder inputs x [n,16], in fp64: (relu, sdf) relative margins per
    sample.  relu: the smallest |a| / (Σ_j |W_ij h_j| + |b_i|) over the
    units of the three ReLU layers (pts_linears 0 / 1, color_out 0); sdf: the
    same ratio for the sdf output.  fp32 evaluates such a sum to within
    ~n·2^-24 of its denominator in any summation order, so a margin below
    ~1e-5 means two fp32 implementations can land on different sides of zero:
    a ReLU unit switches (the derivative jumps by the unit's whole
    contribution), or the sdf changes sign and the compositing's first sign
    change — hence z_min, the truncation window and every weight of the ray
    (render_helpers.py:531-545) — moves.  Discontinuities of the reference's
    own fp32 function."""
    F = torch.nn.functional
    p = {k: v.detach().double() for k, v in params.items()}
    x = x.detach().double()

    def layer(h, w, b):
        a = F.linear(h, w, b)
        den = F.linear(h.abs(), w.abs(), b.abs())
        return a, a.abs() / (den + 1e-300)

    a1, m1 = layer(x, p["pts_linears.0.weight"], p["pts_linears.0.bias"])
    a2, m2 = layer(a1.relu(), p["pts_linears.1.weight"], p["pts_linears.1.bias"])
    o, mo = layer(a2.relu(), p["sdf_out.weight"], p["sdf_out.bias"])
    _, m4 = layer(torch.cat([o[:, 1:], x], -1), p["color_out.0.weight"], p["color_out.0.bias"])
    relu = torch.minimum(torch.minimum(m1.amin(-1), m2.amin(-1)), m4.amin(-1))
    return relu, mo[:, 0]


def relu_margins(params, x):
    """decoder_margins' ReLU part."""
    return decoder_margins(params, x)[0]


# --------------------------------------------------------------------------
# render_rays — render_helpers.py:351-556
# --------------------------------------------------------------------------
def render_rays(rays_o, rays_d, map_states, decoder_params, step_size, voxel_size, truncation, max_distance,
                noise=None, deterministic=False, generator=None, sum_order="torch", dtype=torch.float32,
                capture=None):
    """dtype: the arithmetic of everything after the sampler (interpolation,
    decoder, compositing; the caller's criterion follows).  float32 is the
    reference; float64 gives the same function evaluated without fp32
    rounding at the same fp32 rays / depths / parameters (the intersection
    and the sampler always run in fp32, as the reference's kernels) — the
    yardstick for how far any fp32 summation order is from the exact value.
    capture (dict, optional): receives the decoder inputs "feats" [M,16]
    (ray-major sample order, gradients retained) and the per-ray sample
    offsets "offsets" [R_hit+1]."""
    intersection, hits = ray_intersect_vox(rays_o.detach().float(), rays_d.detach().float(),
                                           map_states["voxel_center_xyz"].float(),
                                           map_states["voxel_structure"], voxel_size, max_distance)
    assert hits.sum() > 0
    ray_mask = hits.view(1, -1)
    intersection = {k: v[ray_mask].reshape(-1, v.size(-1)) for k, v in intersection.items()}
    ro = rays_o[ray_mask].reshape(-1, 3)
    rd = rays_d[ray_mask].reshape(-1, 3)
    samples, noise = ray_sample(intersection, step_size, noise, deterministic, generator, sum_order)
    depth = samples["sampled_point_depth"]
    sidx = samples["sampled_point_voxel_idx"].long()
    mask = sidx.ne(-1)
    if dtype != torch.float32:
        ro, rd, depth = ro.to(dtype), rd.to(dtype), depth.to(dtype)
        decoder_params = {k: v.to(dtype) for k, v in decoder_params.items()}
    xyz = ro.unsqueeze(1) + rd.unsqueeze(1) * depth.unsqueeze(2)
    feats = interp_features(xyz[mask], sidx[mask], map_states["voxel_center_xyz"].to(dtype),
                            map_states["voxel_vertex_idx"], map_states["voxel_vertex_emb"].to(dtype), voxel_size)
    if capture is not None:
        if feats.requires_grad:
            feats.retain_grad()
        capture["feats"] = feats
        capture["offsets"] = torch.cat([torch.zeros(1, dtype=torch.long), mask.sum(-1).cumsum(0)])
    rgb_s, sdf_s = decoder_forward(decoder_params, feats)
    R, S = mask.shape
    sdf = torch.ones(R, S, dtype=dtype).masked_scatter(mask, sdf_s)
    colour = torch.zeros(R, S, 3, dtype=dtype).masked_scatter(mask.unsqueeze(-1).expand(R, S, 3), rgb_s)
    valid = mask.float()
    z = depth
    w = torch.sigmoid(sdf / truncation) * torch.sigmoid(-sdf / truncation)
    sign = sdf[:, 1:] * sdf[:, :-1]
    first = torch.argmax((sign < 0.0).float(), dim=1)[..., None]
    z_min = torch.gather(z, 1, first)
    # the comparison in fp32 as the reference makes it (exact for fp32 z; a dtype=float64 run keeps fp32's
    # discrete decisions)
    w = w * (z.float() < z_min.float() + truncation).to(w.dtype) * valid
    w = w / (w.sum(dim=-1, keepdim=True) + 1e-8)
    return {
        "weights": w,
        "color": (w[..., None] * colour).sum(-2),
        "depth": (w * z).sum(-1),
        "z_vals": z,
        "sdf": sdf,
        "ray_mask": ray_mask,
        "samples": samples,
        "sampled_xyz": xyz,
        "intersection": intersection,
        "noise": noise,
        "n_samples": int(mask.sum()),
    }


def ray_grads_from_dfeat(out, rays_o, rays_d, map_states, voxel_size, dfeat):
    """The interpolation backward alone, in fp64: per hit ray, d_o = Σ_s
    ∂feats_s/∂o · dfeat_s and d_d = Σ_s ∂feats_s/∂d · dfeat_s over the ray's
    samples (render_helpers.py:104-156 differentiated through xyz = o + d·z),
    for an arbitrary per-sample decoder-input gradient dfeat [M,16] in the
    ray-major sample order of `out` (a render_rays result).  Returns
    ([R_hit,3], [R_hit,3]) float64."""
    hit = out["ray_mask"].view(-1)
    ro = rays_o.reshape(-1, 3)[hit].detach().double().requires_grad_(True)
    rd = rays_d.reshape(-1, 3)[hit].detach().double().requires_grad_(True)
    sidx = out["samples"]["sampled_point_voxel_idx"].long()
    mask = sidx.ne(-1)
    z = out["z_vals"].detach().double()
    xyz = ro.unsqueeze(1) + rd.unsqueeze(1) * z.unsqueeze(2)
    feats = interp_features(xyz[mask], sidx[mask], map_states["voxel_center_xyz"].double(),
                            map_states["voxel_vertex_idx"], map_states["voxel_vertex_emb"].detach().double(),
                            voxel_size)
    g_o, g_d = torch.autograd.grad(feats, [ro, rd], grad_outputs=dfeat.detach().double())
    return g_o, g_d


# --------------------------------------------------------------------------
# Criterion — criterion.py:16-116 (weight_depth_loss=False path + median path)
# --------------------------------------------------------------------------
def criterion(outputs, rgb_gt, depth_gt, weights_cfg, truncation, max_depth, weight_depth_loss=False):
    ray_mask = outputs["ray_mask"]
    gt_depth = depth_gt[ray_mask]
    gt_color = rgb_gt[ray_mask]
    z = outputs["z_vals"]
    sdf = outputs["sdf"]
    color_loss = (gt_color - outputs["color"]).abs().mean()
    # masks from the fp32 values (a float64 run keeps the reference's discrete decisions)
    valid = (gt_depth.float() > 0.01) & (gt_depth.float() < max_depth)
    dl = (gt_depth - outputs["depth"]).abs()
    if weight_depth_loss:
        var = (outputs["weights"] * ((outputs["depth"].unsqueeze(-1) - z) ** 2)).sum(-1)
        tmp = dl / torch.sqrt(var + 1e-10)
        valid = (tmp < 10 * tmp.median()) & valid
    depth_loss = dl[valid].mean()
    d = gt_depth.unsqueeze(-1).expand(*z.shape)
    z32, d32 = z.float(), d.float()
    front = (z32 < d32 - truncation).to(z.dtype)
    back = (z32 > d32 + truncation).to(z.dtype)
    dmask = ((d32 > 0.0) & (d32 < max_depth)).to(z.dtype)
    sdf_mask = (1.0 - front) * (1.0 - back) * dmask
    n_fs = torch.count_nonzero(front).to(z.dtype)
    n_sdf = torch.count_nonzero(sdf_mask).to(z.dtype)
    fs_w = 1.0 - n_fs / (n_fs + n_sdf)
    sdf_w = 1.0 - n_sdf / (n_fs + n_sdf)
    fs_loss = torch.mean(torch.square(sdf * front - front)) * fs_w
    sdf_loss = torch.mean(torch.square((z + sdf * truncation) * sdf_mask - d * sdf_mask)) * sdf_w
    loss = (weights_cfg["rgb_weight"] * color_loss + weights_cfg["depth_weight"] * depth_loss
            + weights_cfg["fs_weight"] * fs_loss + weights_cfg["sdf_weight"] * sdf_loss)
    return loss, {"color_loss": color_loss, "depth_loss": depth_loss, "fs_loss": fs_loss, "sdf_loss": sdf_loss}


def criterion_sums(color, depth, sdf, z, gt_rgb_hit, gt_depth_hit, truncation, max_depth, pad_extra=0):
    """The eight additive partial sums the loss of criterion() decomposes into
    (csrc/criterion.hip layout): Σ|Δrgb|, Σ_valid|Δd|, n_valid, n_front,
    n_sdf, Σ fs², Σ sdf², 0 — differentiable torch ops.  pad_extra counts
    extra padded samples (z = 10, sdf = 1) per ray, as a shard with a smaller
    S_max than the global batch has them (criterion.py:70-116)."""
    d = gt_depth_hit.unsqueeze(-1).expand(*z.shape)
    front = (z < d - truncation).float()
    back = (z > d + truncation).float()
    dmask = ((d > 0.0) & (d < max_depth)).float()
    sm = (1.0 - front) * (1.0 - back) * dmask
    valid = ((gt_depth_hit > 0.01) & (gt_depth_hit < max_depth)).float()
    zero = color.new_zeros(())
    s = [(gt_rgb_hit - color).abs().sum(), ((gt_depth_hit - depth).abs() * valid).sum(), valid.sum(),
         front.sum(), sm.sum(), torch.square(sdf * front - front).sum(),
         torch.square((z + sdf * truncation) * sm - d * sm).sum(), zero]
    if pad_extra:
        zp = torch.full_like(gt_depth_hit, 10.0)
        fp = (zp < gt_depth_hit - truncation).float()
        bp = (zp > gt_depth_hit + truncation).float()
        smp = (1.0 - fp) * (1.0 - bp) * ((gt_depth_hit > 0.0) & (gt_depth_hit < max_depth)).float()
        s[3] = s[3] + pad_extra * fp.sum()
        s[4] = s[4] + pad_extra * smp.sum()
        s[6] = s[6] + pad_extra * torch.square((zp + truncation) * smp - gt_depth_hit * smp).sum()
    return torch.stack(s)


def criterion_from_sums(sums, n_hit, s_cols, weights_cfg):
    """Loss of criterion() from (all-reduced) sums over n_hit rays x s_cols columns."""
    color_loss = sums[0] / (3 * n_hit)
    depth_loss = sums[1] / sums[2]
    n_f, n_s = sums[3], sums[4]
    fs_loss = sums[5] / (n_hit * s_cols) * (1.0 - n_f / (n_f + n_s))
    sdf_loss = sums[6] / (n_hit * s_cols) * (1.0 - n_s / (n_f + n_s))
    loss = (weights_cfg["rgb_weight"] * color_loss + weights_cfg["depth_weight"] * depth_loss
            + weights_cfg["fs_weight"] * fs_loss + weights_cfg["sdf_weight"] * sdf_loss)
    return loss, {"color_loss": color_loss, "depth_loss": depth_loss, "fs_loss": fs_loss, "sdf_loss": sdf_loss}


REPLICA_CRITERIA = {"rgb_weight": 0.5, "depth_weight": 1.0, "sdf_weight": 5000.0, "fs_weight": 10.0}
SCANNET_CRITERIA = {"rgb_weight": 1.0, "depth_weight": 1.0, "sdf_weight": 5000.0, "fs_weight": 10.0}


def render_and_backward(rays_o, rays_d, rgb_gt, depth_gt, map_states, decoder_params, step_size, voxel_size,
                        truncation=0.1, max_distance=10.0, criteria=REPLICA_CRITERIA, noise=None,
                        deterministic=False, generator=None, rays_require_grad=True, sum_order="torch",
                        max_depth=None, dtype=torch.float32, capture=None):
    """One bundle-adjust iteration's differentiable part (render_helpers.py:648-671).

    Returns outputs, loss and grads for embeddings, decoder params, rays_o, rays_d
    (dtype: see render_rays; the gradients come back in that dtype)."""
    emb = map_states["voxel_vertex_emb"].detach().clone().requires_grad_(True)
    params = {k: v.detach().clone().requires_grad_(True) for k, v in decoder_params.items()}
    ro = rays_o.detach().clone().requires_grad_(rays_require_grad)
    rd = rays_d.detach().clone().requires_grad_(rays_require_grad)
    ms = dict(map_states)
    ms["voxel_vertex_emb"] = emb
    out = render_rays(ro, rd, ms, params, step_size, voxel_size, truncation, max_distance, noise, deterministic,
                      generator, sum_order, dtype, capture)
    loss, parts = criterion(out, rgb_gt.to(dtype), depth_gt.to(dtype), criteria, truncation,
                            max_distance if max_depth is None else max_depth)  # data_specs max_depth
    loss.backward()
    grads = {"embeddings": emb.grad, "rays_o": ro.grad, "rays_d": rd.grad}
    for k, v in params.items():
        grads[k] = v.grad
    return out, loss.detach(), parts, grads


# --------------------------------------------------------------------------
# bundle_adjust_frames — render_helpers.py:559-676 with keyframe poses
# (se3pose.py:8-98 restated below: [t | w], R = I + A[w]x + B[w]x^2, A / B as
# 10th-order Taylor series in theta)
# --------------------------------------------------------------------------
def _taylor(theta, first, step, nth=10):
    ans = torch.zeros_like(theta)
    denom = 1.0
    for i in range(nth + 1):
        if i > 0:
            denom *= step(i)
        ans = ans + (-1) ** i * theta ** (2 * i) / (denom * first)
    return ans


def se3_rotation(data):
    """se3pose.py:24-33 (rotation of pose parameters [t | w])."""
    w = data[3:]
    wx = torch.stack([torch.stack([torch.zeros(()), -w[2], w[1]]), torch.stack([w[2], torch.zeros(()), -w[0]]),
                      torch.stack([-w[1], w[0], torch.zeros(())])])
    theta = w.norm(dim=-1)[..., None, None]
    A = _taylor(theta, 1.0, lambda i: (2 * i) * (2 * i + 1))
    B = _taylor(theta, 2.0, lambda i: (2 * i + 1) * (2 * i + 2))
    return torch.eye(3) + A * wx + B * (wx @ wx)


def bundle_adjust(frames, picks, noises, map_states, decoder_params, poses0, stamps, step_size, voxel_size,
                  n_iters, lr_map=5e-3, lr_pose=1e-3, criteria=REPLICA_CRITERIA, truncation=0.1, max_distance=10.0):
    """frames: [(rays_d [H,W,3], rgb [H,W,3], depth [H,W])]; picks[it][f]:
    sorted pixel ids; noises[it]: the sampler noise of iteration it.  Adam
    (torch, CPU) on embeddings, decoder and the poses of frames with stamp != 0.
    Returns (losses, embeddings, decoder params, poses)."""
    emb = map_states["voxel_vertex_emb"].detach().clone().requires_grad_(True)
    params = {k: v.detach().clone().requires_grad_(True) for k, v in decoder_params.items()}
    poses = [torch.tensor(p, dtype=torch.float32).requires_grad_(True) for p in poses0]
    opts = [torch.optim.Adam([emb], lr=lr_map), torch.optim.Adam(list(params.values()), lr=lr_map)]
    opts += [torch.optim.Adam([poses[f]], lr=lr_pose) for f in range(len(frames)) if stamps[f] != 0]
    ms = dict(map_states)
    ms["voxel_vertex_emb"] = emb
    losses = []
    for it in range(n_iters):
        ro, rd, rgb, dep = [], [], [], []
        for f, (rays_d, rgb_f, depth_f) in enumerate(frames):
            idx = torch.as_tensor(picks[it][f]).long()
            R = se3_rotation(poses[f])
            d = rays_d.reshape(-1, 3)[idx] @ R.transpose(-1, -2)
            ro.append(poses[f][:3].reshape(1, -1).expand_as(d))
            rd.append(d)
            rgb.append(rgb_f.reshape(-1, 3)[idx])
            dep.append(depth_f.reshape(-1)[idx])
        rays_o, rays_d_w = torch.cat(ro)[None], torch.cat(rd)[None]
        out = render_rays(rays_o, rays_d_w, ms, params, step_size, voxel_size, truncation, max_distance,
                          noise=torch.as_tensor(noises[it]))
        loss, _ = criterion(out, torch.cat(rgb)[None], torch.cat(dep)[None], criteria, truncation, max_distance)
        for o in opts:
            o.zero_grad()
        loss.backward()
        for o in opts:
            o.step()
        losses.append(float(loss.detach()))
    return losses, emb.detach(), {k: v.detach() for k, v in params.items()}, torch.stack([p.detach() for p in poses])



def track_frame(rays_d_cam, rgb, depth, picks, noises, map_states, decoder_params, pose0, step_size, voxel_size,
                n_iters, lr=1e-3, criteria=REPLICA_CRITERIA, truncation=0.1, max_distance=10.0, max_depth=10.0,
                weight_depth_loss=True):
    """track_frame (render_helpers.py:679-761): pose-only Adam (torch, CPU)
    on one frame against the frozen map, rays = pose applied to the picked
    camera directions (:708-716), Criterion with weight_depth_loss (the
    depth-variance median filter, criterion.py:45-50).  picks[it]: sorted
    pixel ids; noises[it]: the sampler noise of iteration it.  Returns
    (losses, pose, the last iteration's hit mask)."""
    pose = torch.tensor(pose0, dtype=torch.float32).requires_grad_(True)
    opt = torch.optim.Adam([pose], lr=lr)
    params = {k: v.detach() for k, v in decoder_params.items()}
    ms = dict(map_states)
    ms["voxel_vertex_emb"] = map_states["voxel_vertex_emb"].detach()
    losses, hit = [], None
    for it in range(n_iters):
        idx = torch.as_tensor(picks[it]).long()
        d = rays_d_cam.reshape(-1, 3)[idx] @ se3_rotation(pose).transpose(-1, -2)
        ro = pose[:3].reshape(1, -1).expand_as(d)
        out = render_rays(ro[None], d[None], ms, params, step_size, voxel_size, truncation, max_distance,
                          noise=torch.as_tensor(noises[it]))
        loss, _ = criterion(out, rgb.reshape(-1, 3)[idx][None], depth.reshape(-1)[idx][None], criteria, truncation,
                            max_depth, weight_depth_loss=weight_depth_loss)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(float(loss.detach()))
        hit = out["ray_mask"].reshape(-1).clone()
    return losses, pose.detach(), hit


# ---------------------------------------------------------------- pixel sampling
def pixel_uniforms(seed, n_frames, n_pix):
    """The counter-based uniforms psvo_sample_pixels draws when no u is given
    (csrc/pixels.hip px_uniform: a 64-bit finaliser of seed·φ + f·2^40 + i,
    top 24 bits → [0, 1) like torch.rand).  numpy uint64 arithmetic wraps."""
    with np.errstate(over="ignore"):
        f = np.arange(n_frames, dtype=np.uint64)[:, None]
        i = np.arange(n_pix, dtype=np.uint64)[None, :]
        x = np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15) + (f << np.uint64(40)) + i
        x ^= x >> np.uint64(33)
        x *= np.uint64(0xFF51AFD7ED558CCD)
        x ^= x >> np.uint64(33)
        x *= np.uint64(0xC4CEB9FE1A85EC53)
        x ^= x >> np.uint64(33)
    top = ((x & np.uint64(0xFFFFFFFF)) >> np.uint64(8)).astype(np.float32)
    return top * np.float32(1.0 / 16777216.0)


def pixel_scores(mask, u):
    """sample_util.py:12-17 + :5-8 in f32: log(mask / (mask.sum() + 1e-7) +
    1e-7) + gumbel(u), one sum over the whole [B, H, W] mask."""
    mask = torch.as_tensor(mask, dtype=torch.float32)
    B = mask.shape[0]
    probs = mask / (mask.sum() + 1e-7)
    logp = torch.log(probs.reshape(B, -1) + 1e-7)
    u = torch.as_tensor(u, dtype=torch.float32).reshape(B, -1)
    return logp + (-torch.log(-torch.log(u + 1e-7) + 1e-7))


def sample_rays(mask, n, u):
    """sample_util.sample_rays (sample_util.py:12-20) with the uniforms
    gumbel_like draws given: the n top scores per frame, as ascending pixel
    indices [B, n] (the bool mask's pixels in row-major order).  Ties at the
    n-th score: lowest pixel index first (torch.topk leaves it unspecified)."""
    s = pixel_scores(mask, u).numpy()
    B = s.shape[0]
    out = np.empty((B, n), np.int64)
    for b in range(B):
        order = np.lexsort((np.arange(s.shape[1]), -s[b].astype(np.float64)))
        out[b] = np.sort(order[:n])
    return out


# ---------------------------------------------------------------------------
# The `grid` functions off the render path (SURVEY.md §8b import contract).
# Arrays in the reference layouts; outputs allocated as intersect.cpp /
# sample.cpp allocate them.
# ---------------------------------------------------------------------------

def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def ball_intersect(ray_start, ray_dir, points, radius, n_max):
    """intersect.cpp:15-42 + intersect_gpu.cu:13-73 → (idx, min_depth, max_depth) [b, m, n_max]."""
    rs, rd, pts = _f32(ray_start), _f32(ray_dir), _f32(points)
    b, m, n = rs.shape[0], rs.shape[1], pts.shape[1]
    idx = np.zeros((b, m, n_max), np.int32)
    lo = np.zeros((b, m, n_max), np.float32)
    hi = np.zeros((b, m, n_max), np.float32)
    lib().oracle_ball_intersect(b, n, m, float(radius), int(n_max), _ptr(rs), _ptr(rd), _ptr(pts), _ptr(idx),
                                _ptr(lo), _ptr(hi))
    return idx, lo, hi


def aabb_intersect(ray_start, ray_dir, points, voxelsize, n_max):
    """intersect.cpp:49-76 + intersect_gpu.cu:142-187 → (idx, min_depth, max_depth) [b, m, n_max]."""
    rs, rd, pts = _f32(ray_start), _f32(ray_dir), _f32(points)
    b, m, n = rs.shape[0], rs.shape[1], pts.shape[1]
    idx = np.zeros((b, m, n_max), np.int32)
    lo = np.zeros((b, m, n_max), np.float32)
    hi = np.zeros((b, m, n_max), np.float32)
    lib().oracle_aabb_intersect(b, n, m, float(voxelsize), int(n_max), _ptr(rs), _ptr(rd), _ptr(pts), _ptr(idx),
                                _ptr(lo), _ptr(hi))
    return idx, lo, hi


def triangle_intersect(ray_start, ray_dir, face_points, cagesize, blur, n_max):
    """intersect.cpp:119-146 + intersect_gpu.cu:273-369 → (idx [b,m,n_max], depth [b,m,3n_max], uv [b,m,2n_max])."""
    rs, rd, fp = _f32(ray_start), _f32(ray_dir), _f32(face_points)
    b, m, n = rs.shape[0], rs.shape[1], fp.shape[1]
    idx = np.zeros((b, m, n_max), np.int32)
    depth = np.zeros((b, m, 3 * n_max), np.float32)
    uv = np.zeros((b, m, 2 * n_max), np.float32)
    lib().oracle_triangle_intersect(b, n, m, float(cagesize), float(blur), int(n_max), _ptr(rs), _ptr(rd), _ptr(fp),
                                    _ptr(idx), _ptr(depth), _ptr(uv))
    return idx, depth, uv


def uniform_ray_sampling(pts_idx, min_depth, max_depth, uniform_noise, step_size, max_steps):
    """sample.cpp:21-54 + sample_gpu.cu:13-124 → (sampled_idx, depth, dists) [b, k, max_steps]."""
    pi = np.ascontiguousarray(pts_idx, dtype=np.int32)
    lo, hi, nz = _f32(min_depth), _f32(max_depth), _f32(uniform_noise)
    b, k, p = lo.shape
    s_idx = -np.ones((b, k, max_steps), np.int32)
    s_depth = np.zeros((b, k, max_steps), np.float32)
    s_dist = np.zeros((b, k, max_steps), np.float32)
    lib().oracle_uniform_sampling(b, k, p, int(max_steps), float(step_size), _ptr(pi), _ptr(lo), _ptr(hi), _ptr(nz),
                                  _ptr(s_idx), _ptr(s_depth), _ptr(s_dist))
    return s_idx, s_depth, s_dist


class _EasyNode:
    __slots__ = ("center", "depth", "index", "children")

    def __init__(self, center, depth, index):
        self.center, self.depth, self.index = center, depth, index
        self.children = [None] * 8


def build_octree(center, points, depth):
    """sparse_voxels/src/octree.cpp:12-164 (EasyOctree), pure Python (small
    inputs): centre compared and advanced in f32, leaves keep their point
    index, internal ids from total-1 down in BFS order.  Returns
    (centers i32 [total, 3], children i32 [total, 9])."""
    c0 = np.asarray(center, dtype=np.float32).reshape(3)
    pts = np.asarray(points, dtype=np.int64).reshape(-1, 3)
    root = _EasyNode(c0.copy(), int(depth), -1)

    def insert(p, point, index):  # octree.cpp:71-92
        diff = (point.astype(np.float32) > p.center).astype(np.int32)
        i = int(diff[0] + 2 * diff[1] + 4 * diff[2])
        if p.depth == 0:
            p.children[i] = _EasyNode(point.copy(), -1, index)
        else:
            if p.children[i] is None:
                length = 1 << (p.depth - 1)
                p.children[i] = _EasyNode((p.center + ((2 * diff - 1) * length).astype(np.float32)).astype(np.float32),
                                          p.depth - 1, -1)
            insert(p.children[i], point, index)

    for k in range(pts.shape[0]):
        insert(root, pts[k], k)

    def count(p):  # octree.cpp:94-111
        total, terminal = 1, 1 if p.depth == -1 else 0
        for c in p.children:
            if c is not None:
                a, t = count(c)
                total += a
                terminal += t
        return total, terminal

    total, terminal = count(root)
    centers = np.zeros((total, 3), np.int32)
    children = -np.ones((total, 9), np.int32)
    node_idx = total - 1
    root.index = node_idx
    queue = [root]
    head = 0
    while head < len(queue):  # octree.cpp:127-145
        node = queue[head]
        head += 1
        for i, c in enumerate(node.children):
            if c is not None:
                if c.depth > -1:
                    node_idx -= 1
                    c.index = node_idx
                queue.append(c)
                children[node.index, i] = c.index
        children[node.index, 8] = 1 << (node.depth + 1)
        centers[node.index] = np.trunc(np.asarray(node.center, dtype=np.float64)).astype(np.int32)
    assert node_idx == terminal  # octree.cpp:146
    return centers, children
