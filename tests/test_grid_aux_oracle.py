"""The `grid` functions off the render path (ball / aabb /
triangle intersection, uniform ray sampling, build_octree), CPU side.

Parity anchor: the reference ships no test vectors for these and its CUDA
cannot be built here, so the oracle restatement (oracle/svo_oracle.c,
oracle/oracle.py) is pinned by known answers derived by hand from the
reference kernels (intersect_gpu.cu:13-369, sample_gpu.cu:13-124,
sparse_voxels/src/octree.cpp:12-164), including their quirks: a ball behind
the origin counts, the uniform sampler labels a gap sample with the previous
box and keeps only in-box midpoints, the triangle list is the first n_max
faces in face order then sorted.  build_octree runs on the host in libpsvo
(no GPU needed) and must equal the oracle's pure-Python EasyOctree exactly.
"""
import math

import numpy as np
import pytest
import torch

from oracle import oracle as O


def _ray(o, d):
    return np.array([[o]], np.float32), np.array([[d]], np.float32)


def test_ball_known_answer_including_ball_behind_origin():
    rs, rd = _ray([0, 0, 0], [1, 0, 0])
    pts = np.array([[[5, 0, 0], [5, 0.5, 0], [5, 2, 0], [-5, 0, 0]]], np.float32)
    idx, lo, hi = O.ball_intersect(rs, rd, pts, 1.0, 4)
    assert idx.tolist() == [[[0, 1, 3, -1]]]
    h = math.sqrt(0.75)
    np.testing.assert_allclose(lo[0, 0, :3], [4, 5 - h, 4], rtol=1e-6)
    np.testing.assert_allclose(hi[0, 0, :3], [6, 5 + h, 6], rtol=1e-6)
    assert lo[0, 0, 3] == 0 and hi[0, 0, 3] == 0  # unused slots keep the zeros


def test_ball_and_aabb_keep_first_n_max_in_point_order():
    rs, rd = _ray([0, 0, 0], [0, 0, 1])
    pts = np.array([[[0, 0, z] for z in (9, 3, 7, 5, 1)]], np.float32)
    idx, lo, _ = O.ball_intersect(rs, rd, pts, 0.5, 3)
    assert idx.tolist() == [[[0, 1, 2]]]
    np.testing.assert_allclose(lo[0, 0], [8.5, 2.5, 6.5])
    idx, lo, hi = O.aabb_intersect(rs, rd, pts, 1.0, 3)
    assert idx.tolist() == [[[0, 1, 2]]]
    np.testing.assert_allclose(lo[0, 0], [8.5, 2.5, 6.5])
    np.testing.assert_allclose(hi[0, 0], [9.5, 3.5, 7.5])


def test_aabb_known_answer():
    rs, rd = _ray([0, 0, 0], [1, 0, 0])
    pts = np.array([[[5, 0, 0], [5, 0.5, 0], [5, 2, 0], [-5, 0, 0], [0, 0, 0]]], np.float32)
    idx, lo, hi = O.aabb_intersect(rs, rd, pts, 2.0, 5)
    # box 2 misses in y, box 3 lies behind (t_out < 0), the origin's box clips at t = 0
    assert idx.tolist() == [[[0, 1, 4, -1, -1]]]
    np.testing.assert_array_equal(lo[0, 0, :3], [4, 4, 0])
    np.testing.assert_array_equal(hi[0, 0, :3], [6, 6, 1])


def test_triangle_known_answer_sorted_with_cage():
    rs, rd = _ray([0, 0, 0], [0, 0, 1])

    def tri(z, x0=-1.0):
        return [x0, -1, z, x0 + 4, -1, z, x0, 3, z]

    faces = np.array([[tri(3), tri(1), tri(5, x0=2.0), tri(2), tri(2)]], np.float32)
    idx, depth, uv = O.triangle_intersect(rs, rd, faces, 1.0, 0.0, 4)
    # face 2 misses; equal depths (faces 3, 4) keep face order
    assert idx.tolist() == [[[1, 3, 4, 0]]]
    d = depth.reshape(4, 3)
    np.testing.assert_allclose(d[:, 0], [1, 2, 2, 3])
    np.testing.assert_allclose(d[:, 1], [-1, -0.5, -0.0, -0.5])
    np.testing.assert_allclose(d[:, 2], [0.5, 0.0, 0.5, 1.0])
    np.testing.assert_allclose(uv.reshape(4, 2), 0.25)


def test_triangle_keeps_first_n_max_faces_not_nearest():
    rs, rd = _ray([0, 0, 0], [0, 0, 1])
    faces = np.array([[[-1, -1, z, 3, -1, z, -1, 3, z] for z in (4, 3, 2, 1)]], np.float32)
    idx, depth, _ = O.triangle_intersect(rs, rd, faces, 0.2, 0.0, 2)
    assert idx.tolist() == [[[1, 0]]]
    np.testing.assert_allclose(depth.reshape(2, 3), [[3, -0.2, 0.2], [4, -0.2, 0.2]])


def test_uniform_sampling_known_answer():
    # hand trace of sample_gpu.cu:13-124: boxes [1.0, 1.5] (id 0) and [2.0, 2.2]
    # (id 1), step 0.3, noise 0.5.  Merge: 1.0 1.15 1.45 1.5 1.75 2.0 2.05 2.2;
    # the midpoints inside a box survive (1.625 / 1.875 fall in the gap).
    pi = np.array([[[0, 1]]], np.int32)
    lo = np.array([[[1.0, 2.0]]], np.float32)
    hi = np.array([[[1.5, 2.2]]], np.float32)
    idx, dep, dist = O.uniform_ray_sampling(pi, lo, hi, np.full((1, 1, 10), 0.5, np.float32), 0.3, 10)
    assert idx.tolist() == [[[0, 0, 0, 1, 1, -1, -1, -1, -1, -1]]]
    np.testing.assert_allclose(dep[0, 0, :5], [1.075, 1.3, 1.475, 2.025, 2.125], rtol=1e-6)
    np.testing.assert_allclose(dist[0, 0, :5], [0.15, 0.3, 0.05, 0.05, 0.15], atol=1e-6)
    # the reference leaves its in-place scratch behind the valid prefix
    np.testing.assert_allclose(dep[0, 0, 5:8], [2.025, 2.125, 2.2], rtol=1e-6)


def test_uniform_sampling_miss_ray_is_empty():
    pi = -np.ones((1, 1, 3), np.int32)
    lo = np.full((1, 1, 3), 10.0, np.float32)
    idx, dep, dist = O.uniform_ray_sampling(pi, lo, lo.copy(), np.full((1, 1, 8), 0.5, np.float32), 0.1, 8)
    assert (idx == -1).all() and (dep == 0).all() and (dist == 0).all()


def test_build_octree_known_answer():
    pts = np.array([[0, 0, 0], [5, 5, 5], [1, 4, 2]])
    centers, children = O.build_octree([2.5, 2.5, 2.5], pts, 2)
    # root (id 9) → slots 0, 2, 7 → ids 8, 7, 6 in BFS order; leaves keep point ids;
    # centre -0.5 truncates to 0
    assert children[9].tolist() == [8, -1, 7, -1, -1, -1, -1, 6, 8]
    assert children[8].tolist() == [5, -1, -1, -1, -1, -1, -1, -1, 4]
    assert children[5].tolist() == [-1] * 7 + [0, 2]
    assert children[3].tolist() == [1] + [-1] * 7 + [2]
    assert children[0].tolist() == [-1] * 8 + [1]
    assert centers[9].tolist() == [2, 2, 2] and centers[5].tolist() == [0, 0, 0]
    assert centers[2].tolist() == [1, 4, 2]


def _unique_points(rng, n, span):
    pts = rng.integers(0, span, size=(n * 2, 3))
    pts = np.unique(pts, axis=0)
    rng.shuffle(pts)
    return pts[:n]


@pytest.mark.parametrize("n,span,seed", [(1, 4, 0), (40, 8, 1), (700, 64, 2), (3000, 200, 3)])
def test_host_build_octree_matches_oracle(n, span, seed):
    import grid
    rng = np.random.default_rng(seed)
    pts = _unique_points(rng, n, span)
    coords = torch.from_numpy(pts)
    ranges = coords.max(0)[0] - coords.min(0)[0]
    depth = max(int(torch.log2(ranges.max().float().clamp(min=2)).ceil_().long()) - 1, 0)
    center = (coords.max(0)[0] + coords.min(0)[0]) / 2
    c, ch = grid.build_octree(center, coords, depth)
    c_ref, ch_ref = O.build_octree(center.numpy(), pts, depth)
    assert c.dtype == torch.int32 and ch.dtype == torch.int32
    np.testing.assert_array_equal(c.numpy(), c_ref)
    np.testing.assert_array_equal(ch.numpy(), ch_ref)


def test_build_easy_octree_mirror_matches_oracle():
    from psvo.voxel_helpers import build_easy_octree, discretize_points
    rng = np.random.default_rng(7)
    pts = torch.from_numpy(_unique_points(rng, 500, 50)).float() * 0.1 + 0.03
    centers, children = build_easy_octree(pts, 0.1)
    coords, residual = discretize_points(pts, 0.1)
    ranges = coords.max(0)[0] - coords.min(0)[0]
    depth = int(torch.log2(ranges.max().float()).ceil_().long()) - 1
    c_ref, ch_ref = O.build_octree(((coords.max(0)[0] + coords.min(0)[0]) / 2).numpy(), coords.numpy(), depth)
    np.testing.assert_array_equal(children.numpy(), ch_ref)
    torch.testing.assert_close(centers, torch.from_numpy(c_ref).float() * 0.1 + residual, rtol=0, atol=0)


def test_build_octree_rejects_duplicates_and_bad_depth():
    import grid
    with pytest.raises(RuntimeError, match="duplicate"):
        grid.build_octree(torch.tensor([1.5, 1.5, 1.5]), torch.tensor([[0, 0, 0], [1, 1, 1], [0, 0, 0]]), 1)
    with pytest.raises(RuntimeError, match="depth"):
        grid.build_octree(torch.tensor([0.5, 0.5, 0.5]), torch.tensor([[0, 0, 0]]), -1)


def test_build_octree_empty_is_root_only():
    import grid
    c, ch = grid.build_octree(torch.tensor([4.0, 4.0, 4.0]), torch.zeros((0, 3), dtype=torch.long), 2)
    assert ch.tolist() == [[-1] * 8 + [8]] and c.tolist() == [[4, 4, 4]]
    c_ref, ch_ref = O.build_octree([4.0, 4.0, 4.0], np.zeros((0, 3), np.int64), 2)
    np.testing.assert_array_equal(ch.numpy(), ch_ref)


def test_grid_off_path_functions_reject_host_tensors():
    import grid
    r = torch.zeros((1, 4, 3))
    with pytest.raises(RuntimeError, match="CUDA"):
        grid.ball_intersect(r, r, torch.zeros((1, 5, 3)), 0.1, 4)
    with pytest.raises(RuntimeError, match="CUDA"):
        grid.aabb_intersect(r, r, torch.zeros((1, 5, 3)), 0.1, 4)
    with pytest.raises(RuntimeError, match="CUDA"):
        grid.triangle_intersect(r, r, torch.zeros((1, 5, 9)), 0.1, 0.0, 4)
    with pytest.raises(RuntimeError, match="int tensor"):
        grid.uniform_ray_sampling(torch.zeros((1, 4, 2)), torch.zeros((1, 4, 2)), torch.zeros((1, 4, 2)),
                                  torch.zeros((1, 4, 8)), 0.1, 8)
    with pytest.raises(RuntimeError, match="contiguous"):
        grid.aabb_intersect(torch.zeros((1, 3, 4)).transpose(1, 2), r, torch.zeros((1, 5, 3)), 0.1, 4)


def test_triangle_insertion_rotates_tied_runs():
    """intersect_gpu.cu:339-353 is not a stable sort: a shallower hit carries
    the head of each later run of equal depths to that run's end."""
    rs, rd = _ray([0, 0, 0], [0, 0, 1])
    faces = np.array([[[-1, -1, z, 3, -1, z, -1, 3, z] for z in (2, 2, 1, 2, 0.5)]], np.float32)
    idx, depth, _ = O.triangle_intersect(rs, rd, faces, 1.0, 0.0, 5)
    # run of depth 2: [0] → [0, 1] → rotate [1, 0] → [1, 0, 3] → rotate [0, 3, 1]
    assert idx.tolist() == [[[4, 2, 0, 3, 1]]]
    np.testing.assert_array_equal(depth.reshape(5, 3)[:, 0], [0.5, 1, 2, 2, 2])
