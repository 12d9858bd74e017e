"""Drop-in mirror of the reference's src/variations/voxel_helpers.py API on
libpsvo's HIP kernels: the render path (SparseVoxelOctreeRayIntersect,
InverseCDFRaySampling, ray_intersect_vox, ray_sample) and the helpers off it
(Ball/AABB/TriangleRayIntersect, UniformRaySampling, discretize_points,
build_easy_octree, ray_intersect_vox_AABB).

Differences from the reference that do not change results:
  * no G-fold replication of the octree before the DFS kernel
    (voxel_helpers.py:132-135 copies the tree up to 256 times per call);
    rays are independent, so one tree serves every ray;
  * the depth sort is stable on DFS emission order (torch.sort(stable=False)
    leaves equal-depth ties unspecified).
"""
from __future__ import annotations

import math

import torch
from torch.autograd import Function

import grid as _ext

from . import _lib as L

MAX_DEPTH = 10.0        # voxel_helpers.py:24
N_MAX_HITS = 50         # voxel_helpers.py:561
SAMPLER_G = 200         # voxel_helpers.py:300
SAMPLER_CHUNK = 4 * SAMPLER_G
STAT_WORDS = 16


class SparseVoxelOctreeRayIntersect(Function):
    """voxel_helpers.py:110-166: (voxelsize, n_max, points, children, ray_start, ray_dir)
    → (idx, min_depth, max_depth) [S, N, n_max], DFS emission order, non-differentiable."""

    @staticmethod
    def forward(ctx, voxelsize, n_max, points, children, ray_start, ray_dir):
        S, N = ray_start.shape[:2]
        rs = ray_start.reshape(1, S * N, 3).float().contiguous()
        rd = ray_dir.reshape(1, S * N, 3).float().contiguous()
        idx, lo, hi = _ext.svo_intersect(rs, rd, points.float().contiguous().unsqueeze(0),
                                         children.int().contiguous().unsqueeze(0), voxelsize, n_max)
        idx, lo, hi = idx.reshape(S, N, -1), lo.reshape(S, N, -1).type_as(ray_start), hi.reshape(S, N, -1).type_as(ray_start)
        ctx.mark_non_differentiable(idx, lo, hi)
        return idx, lo, hi

    @staticmethod
    def backward(ctx, a, b, c):
        return None, None, None, None, None, None


svo_ray_intersect = SparseVoxelOctreeRayIntersect.apply


class InverseCDFRaySampling(Function):
    """voxel_helpers.py:288-374 with the reference's [200, K', P] layout,
    row-0 padding and 800-slot launch chunks (the layout changes which rays
    get a trailing segment, sample_gpu.cu:224)."""

    @staticmethod
    def forward(ctx, pts_idx, min_depth, max_depth, probs, steps, fixed_step_size=-1, deterministic=False,
                noise=None):
        G, N, P = SAMPLER_G, pts_idx.size(0), pts_idx.size(1)
        H = int(math.ceil(N / G)) * G
        if H > N:
            pad = H - N
            pts_idx = torch.cat([pts_idx, pts_idx[:1].expand(pad, P)], 0)
            min_depth = torch.cat([min_depth, min_depth[:1].expand(pad, P)], 0)
            max_depth = torch.cat([max_depth, max_depth[:1].expand(pad, P)], 0)
            probs = torch.cat([probs, probs[:1].expand(pad, P)], 0)
            steps = torch.cat([steps, steps[:1].expand(pad)], 0)
        pts_idx = pts_idx.reshape(G, -1, P)
        min_depth = min_depth.reshape(G, -1, P)
        max_depth = max_depth.reshape(G, -1, P)
        probs = probs.reshape(G, -1, P)
        steps = steps.reshape(G, -1)
        max_steps = int(steps.ceil().long().max()) + P
        if noise is None:
            noise = min_depth.new_zeros(*min_depth.size()[:-1], max_steps)
            if deterministic:
                noise += 0.5
            else:
                noise = noise.uniform_().clamp(min=0.001, max=0.999)
        results = [
            _ext.inverse_cdf_sampling(
                pts_idx[:, i:i + SAMPLER_CHUNK].int().contiguous(),
                min_depth.float()[:, i:i + SAMPLER_CHUNK].contiguous(),
                max_depth.float()[:, i:i + SAMPLER_CHUNK].contiguous(),
                noise.float()[:, i:i + SAMPLER_CHUNK].contiguous(),
                probs.float()[:, i:i + SAMPLER_CHUNK].contiguous(),
                steps.float()[:, i:i + SAMPLER_CHUNK].contiguous(),
                fixed_step_size)
            for i in range(0, min_depth.size(1), SAMPLER_CHUNK)
        ]
        s_idx, s_dep, s_dis = [torch.cat([r[i] for r in results], 1) for i in range(3)]
        s_idx, s_dep, s_dis = s_idx.reshape(H, -1)[:N], s_dep.reshape(H, -1)[:N], s_dis.reshape(H, -1)[:N]
        max_len = int(s_idx.ne(-1).sum(-1).max())
        s_idx, s_dep, s_dis = s_idx[:, :max_len], s_dep[:, :max_len], s_dis[:, :max_len]
        ctx.mark_non_differentiable(s_idx, s_dep, s_dis)
        return s_idx, s_dep, s_dis

    @staticmethod
    def backward(ctx, a, b, c):
        return None, None, None, None, None, None, None, None


inverse_cdf_sampling = InverseCDFRaySampling.apply


class BallRayIntersect(Function):
    """voxel_helpers.py:27-46: (radius, n_max, points [S,n,3], ray_start, ray_dir [S,N,3])
    → (idx, min_depth, max_depth) [S, N, n_max], non-differentiable."""

    @staticmethod
    def forward(ctx, radius, n_max, points, ray_start, ray_dir):
        idx, lo, hi = _ext.ball_intersect(ray_start.float().contiguous(), ray_dir.float().contiguous(),
                                          points.float().contiguous(), radius, n_max)
        lo, hi = lo.type_as(ray_start), hi.type_as(ray_start)
        ctx.mark_non_differentiable(idx, lo, hi)
        return idx, lo, hi

    @staticmethod
    def backward(ctx, a, b, c):
        return None, None, None, None, None


ball_ray_intersect = BallRayIntersect.apply


class AABBRayIntersect(Function):
    """voxel_helpers.py:49-101: (voxelsize, n_max, points [n,3], ray_start, ray_dir [S,N,3])
    → (idx, min_depth, max_depth) [S, N, n_max].  One box list serves every
    ray (the reference copies it up to 2048 times, :55-74); its debug prints
    are not reproduced."""

    @staticmethod
    def forward(ctx, voxelsize, n_max, points, ray_start, ray_dir):
        S, N = ray_start.shape[:2]
        rs = ray_start.reshape(1, S * N, 3).float().contiguous()
        rd = ray_dir.reshape(1, S * N, 3).float().contiguous()
        idx, lo, hi = _ext.aabb_intersect(rs, rd, points.reshape(1, -1, 3).float().contiguous(), voxelsize, n_max)
        idx, lo, hi = idx.reshape(S, N, -1), lo.reshape(S, N, -1).type_as(ray_start), hi.reshape(S, N, -1).type_as(ray_start)
        ctx.mark_non_differentiable(idx, lo, hi)
        return idx, lo, hi

    @staticmethod
    def backward(ctx, a, b, c):
        return None, None, None, None, None


aabb_ray_intersect = AABBRayIntersect.apply


class TriangleRayIntersect(Function):
    """voxel_helpers.py:169-217: (cagesize, blur_ratio, n_max, points, faces, ray_start, ray_dir)
    → (idx [S,N,n_max], depth [S,N,n_max,3], uv [S,N,2·n_max])."""

    @staticmethod
    def forward(ctx, cagesize, blur_ratio, n_max, points, faces, ray_start, ray_dir):
        S, N = ray_start.shape[:2]
        rs = ray_start.reshape(1, S * N, 3).float().contiguous()
        rd = ray_dir.reshape(1, S * N, 3).float().contiguous()
        face_points = torch.nn.functional.embedding(faces.reshape(-1, 3), points.reshape(-1, 3))
        fp = face_points.reshape(1, -1, 9).float().contiguous()
        idx, depth, uv = _ext.triangle_intersect(rs, rd, fp, cagesize, blur_ratio, n_max)
        idx = idx.reshape(S, N, -1)
        depth = depth.type_as(ray_start).reshape(S, N, -1, 3)
        uv = uv.type_as(ray_start).reshape(S, N, -1)
        ctx.mark_non_differentiable(idx, depth, uv)
        return idx, depth, uv

    @staticmethod
    def backward(ctx, a, b, c):
        return None, None, None, None, None, None, None


triangle_ray_intersect = TriangleRayIntersect.apply


class UniformRaySampling(Function):
    """voxel_helpers.py:220-285: [256, K', P] layout with first-rows padding,
    max_steps = int(max_ray_length / step_size) + 2P, noise U[0,1) (0.5 when
    deterministic), trimmed to the longest valid row."""

    @staticmethod
    def forward(ctx, pts_idx, min_depth, max_depth, step_size, max_ray_length, deterministic=False, noise=None):
        G, N, P = 256, pts_idx.size(0), pts_idx.size(1)
        H = int(math.ceil(N / G)) * G
        if H > N:
            pts_idx = torch.cat([pts_idx, pts_idx[:H - N]], 0)
            min_depth = torch.cat([min_depth, min_depth[:H - N]], 0)
            max_depth = torch.cat([max_depth, max_depth[:H - N]], 0)
        pts_idx = pts_idx.reshape(G, -1, P)
        min_depth = min_depth.reshape(G, -1, P)
        max_depth = max_depth.reshape(G, -1, P)
        max_steps = int(max_ray_length / step_size) + min_depth.size(-1) * 2
        if noise is None:
            noise = min_depth.new_zeros(*min_depth.size()[:-1], max_steps)
            if deterministic:
                noise += 0.5
            else:
                noise = noise.uniform_()
        s_idx, s_dep, s_dis = _ext.uniform_ray_sampling(pts_idx.int().contiguous(), min_depth.float().contiguous(),
                                                        max_depth.float().contiguous(),
                                                        noise.float().reshape(G, -1, max_steps).contiguous(),
                                                        step_size, max_steps)
        s_dep, s_dis = s_dep.type_as(min_depth), s_dis.type_as(min_depth)
        s_idx, s_dep, s_dis = s_idx.reshape(H, -1)[:N], s_dep.reshape(H, -1)[:N], s_dis.reshape(H, -1)[:N]
        max_len = int(s_idx.ne(-1).sum(-1).max())
        s_idx, s_dep, s_dis = s_idx[:, :max_len], s_dep[:, :max_len], s_dis[:, :max_len]
        ctx.mark_non_differentiable(s_idx, s_dep, s_dis)
        return s_idx, s_dep, s_dis

    @staticmethod
    def backward(ctx, a, b, c):
        return None, None, None, None, None, None, None


uniform_ray_sampling = UniformRaySampling.apply


def discretize_points(voxel_points, voxel_size):
    """voxel_helpers.py:481-491: integer voxel indices from the minimum, and the mean residual."""
    minimal_voxel_point = voxel_points.min(dim=0, keepdim=True)[0]
    voxel_indices = ((voxel_points - minimal_voxel_point) / voxel_size).round_().long()
    residual = (voxel_points - voxel_indices.type_as(voxel_points) * voxel_size).mean(0, keepdim=True)
    return voxel_indices, residual


def build_easy_octree(points, half_voxel):
    """voxel_helpers.py:494-501: EasyOctree (grid.build_octree) over the discretised points."""
    coords, residual = discretize_points(points, half_voxel)
    ranges = coords.max(0)[0] - coords.min(0)[0]
    depths = torch.log2(ranges.max().float()).ceil_().long() - 1
    center = (coords.max(0)[0] + coords.min(0)[0]) / 2
    centers, children = _ext.build_octree(center, coords, int(depths))
    centers = centers.float() * half_voxel + residual
    return centers, children


@torch.no_grad()
def ray_intersect_vox_AABB(ray_start, ray_dir, flatten_centers, voxel_size, max_hits, max_distance=10.0):
    """voxel_helpers.py:598-634 (brute-force boxes, used by test_aabb.py):
    50 first hits in box order, sorted by t_in (stable here; the reference's
    torch.sort leaves ties unspecified), max_distance trim."""
    pts_idx, min_depth, max_depth = aabb_ray_intersect(voxel_size, N_MAX_HITS, flatten_centers, ray_start, ray_dir)
    min_depth.masked_fill_(pts_idx.eq(-1), max_distance)
    max_depth.masked_fill_(pts_idx.eq(-1), max_distance)
    min_depth, sorted_idx = min_depth.sort(dim=-1, stable=True)
    max_depth = max_depth.gather(-1, sorted_idx)
    pts_idx = pts_idx.gather(-1, sorted_idx)
    pts_idx[min_depth > max_distance] = -1
    min_depth.masked_fill_(pts_idx.eq(-1), max_distance)
    max_depth.masked_fill_(pts_idx.eq(-1), max_distance)
    max_hits = torch.max(pts_idx.ne(-1).sum(-1))
    min_depth = min_depth[..., :max_hits]
    max_depth = max_depth[..., :max_hits]
    pts_idx = pts_idx[..., :max_hits]
    hits = pts_idx.ne(-1).any(-1)
    return {"min_depth": min_depth, "max_depth": max_depth, "intersected_voxel_idx": pts_idx}, hits


def _intersect_sorted(rays_o, rays_d, centres, structure, voxel_size, max_distance, step_size=1.0):
    """Fused DFS + stable sort + trim (one kernel). Returns device buffers and
    the stats tensor (not yet read back)."""
    dev = rays_o.device
    R = rays_o.numel() // 3
    ro = rays_o.reshape(R, 3).float().contiguous()
    rd = rays_d.reshape(R, 3).float().contiguous()
    hit_idx = torch.empty((R, N_MAX_HITS), dtype=torch.int32, device=dev)
    hit_t0 = torch.empty((R, N_MAX_HITS), dtype=torch.float32, device=dev)
    hit_t1 = torch.empty((R, N_MAX_HITS), dtype=torch.float32, device=dev)
    ray_nv = torch.empty((R,), dtype=torch.int32, device=dev)
    ray_dsum = torch.empty((R,), dtype=torch.float32, device=dev)
    stats = torch.zeros((STAT_WORDS,), dtype=torch.int32, device=dev)
    L.call("psvo_ray_intersect_sorted", L.stream_of(dev), R, L.ptr(ro), L.ptr(rd), centres.float().contiguous(),
           structure.int().contiguous(), float(voxel_size), float(max_distance), float(step_size),
           L.ptr(hit_idx), L.ptr(hit_t0), L.ptr(hit_t1), L.ptr(ray_nv), L.ptr(ray_dsum), L.ptr(stats))
    return dict(ro=ro, rd=rd, hit_idx=hit_idx, hit_t0=hit_t0, hit_t1=hit_t1, ray_nv=ray_nv, ray_dsum=ray_dsum,
                stats=stats, R=R)


@torch.no_grad()
def ray_intersect_vox(ray_start, ray_dir, flatten_centers, flatten_children, voxel_size, max_hits,
                      max_distance=10.0):
    """voxel_helpers.py:557-595 (max_hits is ignored, as in the reference)."""
    S, N = ray_start.shape[:2]
    q = _intersect_sorted(ray_start, ray_dir, flatten_centers, flatten_children, voxel_size, max_distance)
    P = int(q["stats"][0].item())
    out = {
        "min_depth": q["hit_t0"][:, :P].reshape(S, N, P).type_as(ray_start),
        "max_depth": q["hit_t1"][:, :P].reshape(S, N, P).type_as(ray_start),
        "intersected_voxel_idx": q["hit_idx"][:, :P].reshape(S, N, P),
    }
    hits = out["intersected_voxel_idx"].ne(-1).any(-1)
    return out, hits


@torch.no_grad()
def ray_sample(intersection_outputs, step_size=0.01, fixed=False, noise=None):
    """voxel_helpers.py:637-663."""
    dists = (intersection_outputs["max_depth"] - intersection_outputs["min_depth"]).masked_fill(
        intersection_outputs["intersected_voxel_idx"].eq(-1), 0)
    intersection_outputs["probs"] = dists / dists.sum(dim=-1, keepdim=True)
    intersection_outputs["steps"] = dists.sum(-1) / step_size
    s_idx, s_dep, s_dis = inverse_cdf_sampling(intersection_outputs["intersected_voxel_idx"],
                                               intersection_outputs["min_depth"], intersection_outputs["max_depth"],
                                               intersection_outputs["probs"], intersection_outputs["steps"], -1,
                                               fixed, noise)
    s_dis = s_dis.clamp(min=0.0)
    s_dep.masked_fill_(s_idx.eq(-1), MAX_DEPTH)
    s_dis.masked_fill_(s_idx.eq(-1), 0.0)
    return {"sampled_point_depth": s_dep, "sampled_point_distance": s_dis, "sampled_point_voxel_idx": s_idx}
