"""The `grid` functions off the render path on the GPU (csrc/grid_aux.hip)
vs the oracle restatement, bit-exact: ball / aabb / triangle intersection
and uniform ray sampling, through the drop-in `grid` module and the
voxel_helpers mirror (AABBRayIntersect / ray_intersect_vox_AABB — what the
reference's src/variations/test_aabb.py runs — and UniformRaySampling).
The oracle is pinned by the known answers in test_grid_aux_oracle.py."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rays(rng, b, m, axis_frac=0.2):
    o = rng.uniform(-1, 1, size=(b, m, 3)).astype(np.float32)
    d = rng.normal(size=(b, m, 3)).astype(np.float32)
    # some rays with exact zero direction components (inf reciprocals in the slab test)
    k = int(m * axis_frac)
    d[:, :k, rng.integers(0, 3)] = 0.0
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    return o, d.astype(np.float32)


def _gpu(*arrays):
    return [torch.from_numpy(np.ascontiguousarray(a)).to(DEV) for a in arrays]


@pytest.mark.parametrize("fn", ["ball_intersect", "aabb_intersect"])
@pytest.mark.parametrize("b,m,n,n_max,size,seed", [
    (1, 1, 1, 1, 0.5, 0),
    (2, 301, 1000, 10, 0.4, 1),     # n_max saturates: first hits in point order only
    (3, 130, 333, 100, 0.25, 2),    # n not a multiple of the wave
    (1, 64, 5000, 50, 0.1, 3),      # >= 1024 points, n_max <= 128: four segment waves per ray
    (2, 150, 3000, 10, 0.5, 5),     # split mode, saturating inside the first segments
    (1, 97, 4097, 128, 0.3, 6),     # split mode at its n_max bound, ragged last segment
    (1, 50, 2000, 129, 0.3, 7),     # n_max past the split bound: one wave per ray
    (2, 17, 0, 4, 0.2, 4),          # no primitives: every idx -1
])
def test_point_intersect_matches_oracle(fn, b, m, n, n_max, size, seed):
    import grid
    rng = np.random.default_rng(seed)
    o, d = _rays(rng, b, m)
    pts = rng.uniform(-3, 3, size=(b, n, 3)).astype(np.float32)
    ref = getattr(O, fn)(o, d, pts, size, n_max)
    got = getattr(grid, fn)(*_gpu(o, d, pts), size, n_max)
    for g, r, name in zip(got, ref, ("idx", "min_depth", "max_depth")):
        np.testing.assert_array_equal(g.cpu().numpy(), r, err_msg=f"{fn} {name}")
    if n * m >= 1000:
        assert (ref[0] >= 0).any()


def _faces(rng, b, n, dup):
    c = rng.uniform(-2, 2, size=(b, n, 1, 3))
    f = (c + rng.uniform(-0.6, 0.6, size=(b, n, 3, 3))).reshape(b, n, 9).astype(np.float32)
    if dup:  # exact duplicates: equal depths, ordered by face index
        f[:, 1::7] = f[:, 0::7][:, :f[:, 1::7].shape[1]]
    return f


@pytest.mark.parametrize("b,m,n,n_max,blur,seed", [
    (1, 1, 3, 2, 0.0, 0),
    (2, 257, 700, 8, 0.05, 1),
    (1, 100, 2000, 64, 0.0, 2),
    (3, 33, 129, 200, 0.2, 3),
])
def test_triangle_intersect_matches_oracle(b, m, n, n_max, blur, seed):
    import grid
    rng = np.random.default_rng(seed)
    o, d = _rays(rng, b, m, axis_frac=0.0)
    o = o * 0.2 + np.array([0, 0, -4], np.float32)
    d = d * 0.3 + np.array([0, 0, 1], np.float32)
    d = (d / np.linalg.norm(d, axis=-1, keepdims=True)).astype(np.float32)
    f = _faces(rng, b, n, dup=True)
    ref = O.triangle_intersect(o, d, f, 0.1, blur, n_max)
    got = grid.triangle_intersect(*_gpu(o, d, f), 0.1, blur, n_max)
    for g, r, name in zip(got, ref, ("idx", "depth", "uv")):
        np.testing.assert_array_equal(g.cpu().numpy(), r, err_msg=name)
    if m > 1:
        assert (ref[0] >= 0).sum() > m


def _boxes(rng, b, k, p, frac_hit=0.8):
    """Sorted, touching-or-gapped boxes per ray (ray_intersect's layout:
    idx -1 and depth 10 after the valid prefix)."""
    idx = -np.ones((b, k, p), np.int32)
    lo = np.full((b, k, p), 10.0, np.float32)
    hi = np.full((b, k, p), 10.0, np.float32)
    for bi in range(b):
        for j in range(k):
            if rng.random() > frac_hit:
                continue
            c = int(rng.integers(1, p + 1))
            t = float(rng.uniform(0.5, 2.0))
            for i in range(c):
                if rng.random() < 0.5:
                    t += float(rng.uniform(0.0, 0.3))
                w = float(rng.uniform(0.05, 0.4))
                idx[bi, j, i] = int(rng.integers(0, 10000))
                lo[bi, j, i] = np.float32(t)
                hi[bi, j, i] = np.float32(t + w)
                t = float(hi[bi, j, i])
    return idx, lo, hi


@pytest.mark.parametrize("b,k,p,step,max_steps,seed", [
    (1, 1, 2, 0.3, 10, 0),
    (4, 50, 6, 0.05, 212, 1),     # int(10 / 0.05) + 2P: the reference's sizing
    (2, 77, 12, 0.02, 524, 2),
    (2, 40, 8, 0.05, 30, 3),      # too few steps: the merge stops at max_steps
    (1, 37, 4, 0.01, 1000, 4),    # rows too long for the LDS staging: merged in place in HBM
])
def test_uniform_sampling_matches_oracle(b, k, p, step, max_steps, seed):
    import grid
    rng = np.random.default_rng(seed)
    idx, lo, hi = _boxes(rng, b, k, p)
    noise = rng.random((b, k, max_steps), dtype=np.float32)
    noise[0, 0, :3] = 0.0  # exact-zero noise: the sample before the first box reads slot H-1
    ref = O.uniform_ray_sampling(idx, lo, hi, noise, step, max_steps)
    got = grid.uniform_ray_sampling(*_gpu(idx, lo, hi, noise), step, max_steps)
    for g, r, name in zip(got, ref, ("idx", "depth", "dists")):
        np.testing.assert_array_equal(g.cpu().numpy(), r, err_msg=name)
    assert (ref[0] >= 0).sum() > 0


def test_aabb_mirror_ray_intersect_vox_aabb_matches_oracle():
    """voxel_helpers.ray_intersect_vox_AABB (test_aabb.py's call) on a voxel
    grid: 50 first boxes in order, stable sort by t_in, max_distance trim."""
    from psvo.voxel_helpers import ray_intersect_vox_AABB
    rng = np.random.default_rng(11)
    g = np.stack(np.meshgrid(*[np.arange(12)] * 3, indexing="ij"), -1).reshape(-1, 3)
    keep = rng.random(len(g)) < 0.3
    centres = ((g[keep] + 0.5) * 0.2).astype(np.float32)
    o = np.tile(np.array([[[1.2, 1.2, -0.5]]], np.float32), (1, 500, 1))
    d = rng.normal(size=(1, 500, 3)).astype(np.float32) * 0.3
    d[..., 2] = 1.0
    out, hits = ray_intersect_vox_AABB(*_gpu(o, d), torch.from_numpy(centres).to(DEV), 0.2, 10, 10.0)
    idx, lo, hi = O.aabb_intersect(o, d, centres[None], 0.2, 50)
    lo = np.where(idx == -1, 10.0, lo).astype(np.float32)
    hi = np.where(idx == -1, 10.0, hi).astype(np.float32)
    order = np.argsort(lo, axis=-1, kind="stable")
    lo, hi, idx = (np.take_along_axis(a, order, -1) for a in (lo, hi, idx))
    idx[lo > 10.0] = -1
    P = int((idx != -1).sum(-1).max())
    np.testing.assert_array_equal(out["intersected_voxel_idx"].cpu().numpy(), idx[..., :P])
    np.testing.assert_array_equal(out["min_depth"].cpu().numpy(), np.where(idx == -1, 10.0, lo)[..., :P])
    np.testing.assert_array_equal(out["max_depth"].cpu().numpy(), np.where(idx == -1, 10.0, hi)[..., :P])
    np.testing.assert_array_equal(hits.cpu().numpy(), (idx != -1).any(-1))
    assert P > 3


def test_uniform_mirror_layout_matches_oracle():
    """UniformRaySampling: [256, K', P] layout, first-rows padding, 2P extra
    steps and the trim to the longest row."""
    from psvo.voxel_helpers import UniformRaySampling
    rng = np.random.default_rng(5)
    N, P = 600, 5
    idx, lo, hi = (a[0] for a in _boxes(rng, 1, N, P))
    s_idx, s_dep, s_dis = UniformRaySampling.apply(*_gpu(idx, lo, hi), 0.05, 10.0, True)
    H = 768
    pad = lambda a: np.concatenate([a, a[:H - N]], 0).reshape(256, -1, P)
    max_steps = int(10.0 / 0.05) + 2 * P
    noise = np.full((256, H // 256, max_steps), 0.5, np.float32)
    r_idx, r_dep, r_dis = (a.reshape(H, -1)[:N] for a in O.uniform_ray_sampling(pad(idx), pad(lo), pad(hi), noise,
                                                                                 0.05, max_steps))
    L = int((r_idx != -1).sum(-1).max())
    np.testing.assert_array_equal(s_idx.cpu().numpy(), r_idx[:, :L])
    np.testing.assert_array_equal(s_dep.cpu().numpy(), r_dep[:, :L])
    np.testing.assert_array_equal(s_dis.cpu().numpy(), r_dis[:, :L])
