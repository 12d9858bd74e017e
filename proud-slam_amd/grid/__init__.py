"""Drop-in replacement for the reference's `grid` torch extension
(third_party/sparse_voxels, binding.cpp:10-20), backed by libpsvo.so (HIP,
gfx950).  `import grid as _ext` in voxel_helpers.py:22 keeps working when
proud-slam_amd/ is on sys.path.

Same names, argument order, shapes, dtypes, output allocation and
precondition errors (TORCH_CHECK → RuntimeError, include/utils.h:10-33) as
intersect.cpp / sample.cpp.  Kernel launch failures raise instead of the
reference's exit(-1) (cuda_utils.h:37-48).  The two render-path functions
run on csrc/svo_query.hip; the five off the path (ball / aabb / triangle
intersection, uniform sampling — csrc/grid_aux.hip — and build_octree, on
the host in csrc/grid_octree.cpp) keep the reference's semantics for code
such as src/variations/test_aabb.py.
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


def _check(tensors, floats=(), ints=()):
    """CHECK_CONTIGUOUS / CHECK_IS_FLOAT / CHECK_IS_INT / CHECK_CUDA (include/utils.h:10-33), in that order."""
    for t, n in tensors:
        if not t.is_contiguous():
            raise RuntimeError(f"{n} must be a contiguous tensor")
    for t, n in floats:
        if t.dtype != torch.float32:
            raise RuntimeError(f"{n} must be a float tensor")
    for t, n in ints:
        if t.dtype != torch.int32:
            raise RuntimeError(f"{n} must be an int tensor")
    for t, n in tensors:
        if not t.is_cuda:
            raise RuntimeError(f"{n} must be a CUDA tensor")


def _point_intersect(fn, ray_start, ray_dir, points, size, n_max):
    ts = ((ray_start, "ray_start"), (ray_dir, "ray_dir"), (points, "points"))
    _check(ts, floats=ts)
    b, n, m = points.size(0), points.size(1), ray_start.size(1)
    if ray_start.size(0) != b or ray_dir.shape != ray_start.shape:
        raise RuntimeError(f"{fn}: rays {tuple(ray_start.shape)} / {tuple(ray_dir.shape)} do not match "
                           f"points {tuple(points.shape)}")
    shape = (ray_start.size(0), ray_start.size(1), int(n_max))
    dev = ray_start.device
    idx = torch.zeros(shape, dtype=torch.int32, device=dev)
    lo = torch.zeros(shape, dtype=torch.float32, device=dev)
    hi = torch.zeros(shape, dtype=torch.float32, device=dev)
    L.call(f"psvo_{fn}", L.stream_of(dev), b, n, m, float(size), int(n_max), L.ptr(ray_start), L.ptr(ray_dir),
           L.ptr(points), L.ptr(idx), L.ptr(lo), L.ptr(hi))
    return idx, lo, hi


def ball_intersect(ray_start, ray_dir, points, radius, n_max):
    """intersect.cpp:15-42 — the first n_max balls of `radius` around `points`
    each ray passes (point order; a ball behind the origin counts, as in the
    reference): (idx i32, min_depth f32, max_depth f32) [B, M, n_max]."""
    return _point_intersect("ball_intersect", ray_start, ray_dir, points, radius, n_max)


def aabb_intersect(ray_start, ray_dir, points, voxelsize, n_max):
    """intersect.cpp:49-76 — the first n_max cubes of side `voxelsize` centred
    at `points` each ray enters (point order): (idx, min_depth, max_depth) [B, M, n_max]."""
    return _point_intersect("aabb_intersect", ray_start, ray_dir, points, voxelsize, n_max)


def triangle_intersect(ray_start, ray_dir, face_points, cagesize, blur, n_max):
    """intersect.cpp:119-146 — (idx i32 [B,M,n_max], depth f32 [B,M,3·n_max],
    uv f32 [B,M,2·n_max]): the first n_max faces hit (t > 0) in face order,
    sorted by t, with the cage offsets (-min(cage, gap/2), +min(cage, gap/2))."""
    ts = ((ray_start, "ray_start"), (ray_dir, "ray_dir"), (face_points, "face_points"))
    _check(ts, floats=ts)
    b, n, m = face_points.size(0), face_points.size(1), ray_start.size(1)
    if ray_start.size(0) != b or ray_dir.shape != ray_start.shape or face_points.size(-1) != 9:
        raise RuntimeError(f"triangle_intersect: rays {tuple(ray_start.shape)} do not match face_points "
                           f"{tuple(face_points.shape)} (expected [B, N, 9])")
    dev = ray_start.device
    idx = torch.zeros((ray_start.size(0), m, int(n_max)), dtype=torch.int32, device=dev)
    depth = torch.zeros((ray_start.size(0), m, int(n_max) * 3), dtype=torch.float32, device=dev)
    uv = torch.zeros((ray_start.size(0), m, int(n_max) * 2), dtype=torch.float32, device=dev)
    L.call("psvo_triangle_intersect", L.stream_of(dev), b, n, m, float(cagesize), float(blur), int(n_max),
           L.ptr(ray_start), L.ptr(ray_dir), L.ptr(face_points), L.ptr(idx), L.ptr(depth), L.ptr(uv))
    return idx, depth, uv


def uniform_ray_sampling(pts_idx, min_depth, max_depth, uniform_noise, step_size, max_steps):
    """sample.cpp:21-54 — (sampled_idx i32, depth f32, dists f32) [B, K, max_steps]:
    box boundaries merged with uniform steps, midpoints of the in-box intervals."""
    ts = ((pts_idx, "pts_idx"), (min_depth, "min_depth"), (max_depth, "max_depth"),
          (uniform_noise, "uniform_noise"))
    _check(ts, floats=ts[1:], ints=ts[:1])
    b, k, p = min_depth.size(0), min_depth.size(1), min_depth.size(2)
    if pts_idx.shape != min_depth.shape or max_depth.shape != min_depth.shape:
        raise RuntimeError("uniform_ray_sampling: pts_idx / min_depth / max_depth shapes differ")
    if uniform_noise.numel() < b * k * int(max_steps):
        raise RuntimeError(f"uniform_ray_sampling: uniform_noise {tuple(uniform_noise.shape)} is smaller than "
                           f"[{b}, {k}, {int(max_steps)}]")
    dev = pts_idx.device
    s_idx = -torch.ones((pts_idx.size(0), pts_idx.size(1), int(max_steps)), dtype=torch.int32, device=dev)
    s_depth = torch.zeros((b, k, int(max_steps)), dtype=torch.float32, device=dev)
    s_dist = torch.zeros((b, k, int(max_steps)), dtype=torch.float32, device=dev)
    L.call("psvo_uniform_ray_sampling", L.stream_of(dev), b, k, p, int(max_steps), float(step_size), L.ptr(pts_idx),
           L.ptr(min_depth), L.ptr(max_depth), L.ptr(uniform_noise), L.ptr(s_idx), L.ptr(s_depth), L.ptr(s_dist))
    return s_idx, s_depth, s_dist


def build_octree(center, points, depth):
    """octree.cpp:149-164 — EasyOctree over integer points [N, 3] under a root
    at `center` (3 values) of `depth`: (centers i32 [T, 3], children i32 [T, 9])
    on center's device.  Built on the host by libpsvo (the reference builds it
    on the host too, one Tensor::item() per comparison)."""
    import ctypes
    import time

    t0 = time.perf_counter()
    c = torch.as_tensor(center).detach().reshape(-1).to("cpu", torch.float32).contiguous()
    pts = torch.as_tensor(points).detach().to("cpu", torch.int64).reshape(-1, 3).contiguous()
    if c.numel() != 3:
        raise RuntimeError(f"build_octree: center must hold 3 values, got {c.numel()}")
    total, terminal = ctypes.c_int64(0), ctypes.c_int64(0)
    fn = L.lib().psvo_build_octree
    rc = fn(L.ptr(c), L.ptr(pts), pts.size(0), int(depth), 0, None, None, ctypes.byref(total), ctypes.byref(terminal))
    if rc != 0:
        if total.value >= 0 and depth >= 0:
            raise RuntimeError(f"build_octree: point {total.value} falls into an occupied leaf (duplicate points)")
        raise RuntimeError(f"build_octree: depth {depth} out of range [0, 29]")
    centers = torch.zeros((total.value, 3), dtype=torch.int32)
    children = -torch.ones((total.value, 9), dtype=torch.int32)
    rc = fn(L.ptr(c), L.ptr(pts), pts.size(0), int(depth), total.value, L.ptr(centers), L.ptr(children),
            ctypes.byref(total), ctypes.byref(terminal))
    if rc != 0:
        raise RuntimeError(f"build_octree failed (code {rc})")
    # the reference's report line (octree.cpp:160-161)
    print("Building EasyOctree done. total #nodes = %d, terminal #nodes = %d (time taken %f s)"
          % (total.value, terminal.value, time.perf_counter() - t0))
    dev = torch.as_tensor(center).device
    return centers.to(dev), children.to(dev)
