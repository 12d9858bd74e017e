"""Throughput of the off-path `grid` kernels (csrc/grid_aux.hip) at the
sizes the reference's helpers see: ray_intersect_vox_AABB over a room's
voxel centres (test_aabb.py), ball / triangle intersection over 10-20 k
primitives, uniform sampling of 4096 rays.  Prints one line per kernel:
average kernel time (HIP events on the launch stream), rays/s and primitive
tests/s, and the oracle's single-thread CPU rate on a ray sample.
Usage: grid_aux_bench.py [iterations]"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "proud-slam_amd")]

import grid  # noqa: E402
from oracle import oracle as O  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def cpu_rate(fn, rays):
    t = time.perf_counter()
    fn()
    return rays / (time.perf_counter() - t)


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    rng = np.random.default_rng(0)
    dev = "cuda"
    # room-like occupancy: 16 k voxel centres of a 0.2 m grid on a 64^3 lattice shell
    g = np.stack(np.meshgrid(*[np.arange(48)] * 3, indexing="ij"), -1).reshape(-1, 3)
    shell = (g.min(1) < 2) | (g.max(1) > 45)
    cent = ((g[shell][rng.permutation(shell.sum())[:16000]] + 0.5) * 0.2).astype(np.float32)[None]
    R = 4096
    o = np.tile(np.array([[[4.8, 4.8, 4.8]]], np.float32), (1, R, 1))
    d = rng.normal(size=(1, R, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    ro, rd, pc = to(o), to(d), to(cent)
    n = cent.shape[1]
    lines = []
    for name, size in (("aabb_intersect", 0.2), ("ball_intersect", 0.1)):
        f = getattr(grid, name)
        t = timed(lambda: f(ro, rd, pc, size, 50), iters)
        k = 64
        cpu = cpu_rate(lambda: getattr(O, name)(o[:, :k], d[:, :k], cent, size, 50), k)
        lines.append(f"{name:22s} rays {R} prims {n}: {t * 1e6:9.1f} us  {R / t / 1e6:8.2f} M rays/s  "
                     f"{R * n / t / 1e9:7.1f} G tests/s (upper bound: early exit at 50 hits)  "
                     f"cpu oracle {cpu / 1e3:7.2f} k rays/s (1 thread)")
    # triangles: 10 k small faces around the same shell
    F = 10000
    c = cent[0, rng.integers(0, n, F)]
    faces = (c[:, None, :] + rng.uniform(-0.15, 0.15, size=(F, 3, 3))).reshape(1, F, 9).astype(np.float32)
    fc = to(faces)
    t = timed(lambda: grid.triangle_intersect(ro, rd, fc, 0.1, 0.01, 50), iters)
    cpu = cpu_rate(lambda: O.triangle_intersect(o[:, :64], d[:, :64], faces, 0.1, 0.01, 50), 64)
    lines.append(f"{'triangle_intersect':22s} rays {R} faces {F}: {t * 1e6:9.1f} us  {R / t / 1e6:8.2f} M rays/s  "
                 f"{R * F / t / 1e9:7.1f} G tests/s  cpu oracle {cpu / 1e3:7.2f} k rays/s (1 thread)")
    # uniform sampling of the sorted AABB hits (the NSVF pipeline)
    idx, lo, hi = grid.aabb_intersect(ro, rd, pc, 0.2, 50)
    lo = lo.masked_fill(idx.eq(-1), 10.0)
    hi = hi.masked_fill(idx.eq(-1), 10.0)
    lo, order = lo.sort(dim=-1, stable=True)
    hi, idx = hi.gather(-1, order), idx.gather(-1, order)
    P = int(idx.ne(-1).sum(-1).max())
    pi, lo, hi = idx[..., :P].reshape(256, -1, P).contiguous(), lo[..., :P].reshape(256, -1, P).contiguous(), \
        hi[..., :P].reshape(256, -1, P).contiguous()
    ms = int(10.0 / 0.02) + 2 * P
    noise = torch.rand((256, R // 256, ms), device=dev)
    t = timed(lambda: grid.uniform_ray_sampling(pi, lo, hi, noise, 0.02, ms), iters)
    args = [a.cpu().numpy() for a in (pi, lo, hi, noise)]
    cpu = cpu_rate(lambda: O.uniform_ray_sampling(*args, 0.02, ms), R)
    lines.append(f"{'uniform_ray_sampling':22s} rays {R} P {P} steps {ms}: {t * 1e6:9.1f} us  "
                 f"{R / t / 1e6:8.2f} M rays/s  cpu oracle {cpu / 1e3:7.2f} k rays/s (1 thread)")
    pts = np.unique(rng.integers(0, 256, size=(300000, 3)), axis=0)
    cen = torch.tensor((pts.max(0) + pts.min(0)) / 2, dtype=torch.float32)
    t0 = time.perf_counter()
    grid.build_octree(cen, torch.from_numpy(pts), 7)
    lines.append(f"{'build_octree (host)':22s} {len(pts)} points depth 7: {(time.perf_counter() - t0) * 1e3:9.1f} ms")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
