"""Drop-in replacement for the reference's `grid` torch extension
(third_party/sparse_voxels, binding.cpp:10-20), backed by libpsvo.so (HIP,
gfx950).  `import grid as _ext` in voxel_helpers.py:22 keeps working when
proud-slam_amd/ is on sys.path.

Same names, argument order, shapes, dtypes, output allocation and
precondition errors (TORCH_CHECK → RuntimeError, include/utils.h:10-33) as
intersect.cpp / sample.cpp.  Kernel launch failures raise instead of the
reference's exit(-1) (cuda_utils.h:37-48).  Only the two functions on the
render path are implemented natively; the five the reference never calls
(ball/aabb/triangle intersect, uniform sampling, build_octree — SURVEY §2
row 3) raise NotImplementedError.
"""
from __future__ import annotations

import torch

from psvo import _lib as L


def svo_intersect(ray_start, ray_dir, points, children, voxelsize, n_max):
    """intersect.cpp:83-112 — returns (idx i32, min_depth f32, max_depth f32) [B, M, n_max]."""
    for t, n in ((ray_start, "ray_start"), (ray_dir, "ray_dir"), (points, "points"), (children, "children")):
        if not t.is_contiguous():
            raise RuntimeError(f"{n} must be a contiguous tensor")
    for t, n in ((ray_start, "ray_start"), (ray_dir, "ray_dir"), (points, "points")):
        if t.dtype != torch.float32:
            raise RuntimeError(f"{n} must be a float tensor")
    for t, n in ((ray_start, "ray_start"), (ray_dir, "ray_dir"), (points, "points"), (children, "children")):
        if not t.is_cuda:
            raise RuntimeError(f"{n} must be a CUDA tensor")
    if children.dtype != torch.int32:
        raise RuntimeError("children must be an int tensor")
    b, n, m = points.size(0), points.size(1), ray_start.size(1)
    shape = (ray_start.size(0), ray_start.size(1), int(n_max))
    idx = torch.zeros(shape, dtype=torch.int32, device=ray_start.device)
    min_depth = torch.zeros(shape, dtype=torch.float32, device=ray_start.device)
    max_depth = torch.zeros(shape, dtype=torch.float32, device=ray_start.device)
    L.call("psvo_svo_intersect", L.stream_of(ray_start.device), b, n, m, float(voxelsize), int(n_max),
           L.ptr(ray_start), L.ptr(ray_dir), L.ptr(points), L.ptr(children), L.ptr(idx), L.ptr(min_depth),
           L.ptr(max_depth))
    return idx, min_depth, max_depth


def inverse_cdf_sampling(pts_idx, min_depth, max_depth, uniform_noise, probs, steps, fixed_step_size):
    """sample.cpp:56-95 — returns (sampled_idx i32, depth f32, dists f32) [B, K, max_steps]."""
    for t, n in ((pts_idx, "pts_idx"), (min_depth, "min_depth"), (max_depth, "max_depth"), (probs, "probs"),
                 (steps, "steps"), (uniform_noise, "uniform_noise")):
        if not t.is_contiguous():
            raise RuntimeError(f"{n} must be a contiguous tensor")
    for t, n in ((min_depth, "min_depth"), (max_depth, "max_depth"), (uniform_noise, "uniform_noise"),
                 (probs, "probs"), (steps, "steps")):
        if t.dtype != torch.float32:
            raise RuntimeError(f"{n} must be a float tensor")
    if pts_idx.dtype != torch.int32:
        raise RuntimeError("pts_idx must be an int tensor")
    for t, n in ((pts_idx, "pts_idx"), (min_depth, "min_depth"), (max_depth, "max_depth"),
                 (uniform_noise, "uniform_noise"), (probs, "probs"), (steps, "steps")):
        if not t.is_cuda:
            raise RuntimeError(f"{n} must be a CUDA tensor")
    max_steps = uniform_noise.size(-1)
    b, k, p = min_depth.size(0), min_depth.size(1), min_depth.size(2)
    dev = pts_idx.device
    s_idx = -torch.ones((pts_idx.size(0), pts_idx.size(1), max_steps), dtype=torch.int32, device=dev)
    s_depth = torch.zeros((b, k, max_steps), dtype=torch.float32, device=dev)
    s_dist = torch.zeros((b, k, max_steps), dtype=torch.float32, device=dev)
    L.call("psvo_inverse_cdf_sampling", L.stream_of(dev), b, k, p, max_steps, float(fixed_step_size), L.ptr(pts_idx),
           L.ptr(min_depth), L.ptr(max_depth), L.ptr(uniform_noise), L.ptr(probs), L.ptr(steps), L.ptr(s_idx),
           L.ptr(s_depth), L.ptr(s_dist))
    return s_idx, s_depth, s_dist


def _not_on_path(name):
    def f(*args, **kwargs):
        raise NotImplementedError(f"grid.{name} is not on the render path (no caller in the reference run path; "
                                  f"SURVEY.md §2 row 3) and is not provided by the MI355X build")
    f.__name__ = name
    return f


ball_intersect = _not_on_path("ball_intersect")
aabb_intersect = _not_on_path("aabb_intersect")
triangle_intersect = _not_on_path("triangle_intersect")
uniform_ray_sampling = _not_on_path("uniform_ray_sampling")
build_octree = _not_on_path("build_octree")
