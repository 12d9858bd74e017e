"""Mesh extraction oracle, CPU only: get_scores /
eval_points pinned to the reference's own output (tests/golden/M_mesh_A.npz),
and the marching-cubes case table checked by construction — every
triangle edge on a sign-changing lattice edge, crack-free and consistently
wound across cubes, closed (Euler characteristic 2) around a sphere with
normals towards sdf > 0.  The skimage triangulation itself is parity
unpinned (absent third-party dependency, see oracle/mesh_oracle.py)."""
import ctypes
from collections import Counter

import numpy as np
import torch

from conftest import load_golden
from oracle import mesh_oracle as MO


def _params(g):
    return {k[len("dec."):]: torch.from_numpy(v) for k, v in g.items() if k.startswith("dec.")}


def test_get_scores_matches_reference():
    g = load_golden("M_mesh_A")
    out = MO.get_scores(_params(g), g["centres"], g["features"], g["embeddings"], float(g["voxel_size"]),
                        int(g["res"]))
    np.testing.assert_allclose(out.numpy(), g["scores"], rtol=0, atol=2e-6)


def test_eval_points_matches_reference():
    g = load_golden("M_mesh_A")
    rgb = MO.eval_points(_params(g), g["centres"], g["features"], g["embeddings"], g["points"], g["point_idx"],
                         float(g["voxel_size"]))
    np.testing.assert_allclose(rgb.numpy(), g["point_rgb"], rtol=0, atol=2e-6)


def test_lattice_linspace_matches_torch():
    """psvo_mesh_linspace (host entry point) = torch.linspace on the CPU, bit for bit."""
    from psvo import _lib as L
    for res in range(2, 17):
        out = (ctypes.c_float * res)()
        L.call("psvo_mesh_linspace", res, ctypes.cast(out, ctypes.c_void_p))
        np.testing.assert_array_equal(np.array(out[:], np.float32), torch.linspace(-0.5, 0.5, res).numpy())


def test_case_table_uses_exactly_the_crossing_edges():
    table, ends = MO.mc_table(), MO.edge_endpoints()
    for case in range(256):
        crossing = {e for e, (c0, c1, _) in enumerate(ends) if ((case >> c0) & 1) != ((case >> c1) & 1)}
        used = {e for tri in table[case] for e in tri}
        assert used == crossing, case
        assert len(table[case]) <= 12
    assert table[0] == [] and table[255] == []


def _edge_counts(faces):
    directed = Counter()
    for a, b, c in faces.tolist():
        for u, v in ((a, b), (b, c), (c, a)):
            directed[(u, v)] += 1
    return directed


def _check_crack_free(verts, faces, lo, hi):
    """Every directed edge once; an undirected edge is shared by two
    triangles (opposite directions) unless it lies on the lattice boundary."""
    d = _edge_counts(faces)
    assert max(d.values()) == 1
    on_bd = lambda i: bool(np.any(np.isclose(verts[i], lo, atol=1e-6) | np.isclose(verts[i], hi, atol=1e-6)))
    for (u, v) in d:
        if (v, u) not in d:
            assert on_bd(u) and on_bd(v), (u, v, verts[u], verts[v])


def test_device_case_table_equals_oracle_table():
    """csrc/mesh.hip builds its table at compile time from the same rule;
    the two independent codings agree entry for entry."""
    from psvo import _lib as L
    ntri = np.zeros(256, np.int8)
    tri = np.zeros((256, 36), np.int8)
    L.call("psvo_mesh_case_table", ctypes.c_void_p(ntri.ctypes.data), ctypes.c_void_p(tri.ctypes.data))
    for case, tris in enumerate(MO.mc_table()):
        assert ntri[case] == len(tris), case
        assert tri[case, :3 * len(tris)].reshape(-1, 3).tolist() == [list(t) for t in tris], case


def test_random_fields_are_crack_free_and_consistently_wound():
    rng = np.random.default_rng(0)
    for res in (2, 5, 8):
        sdf = rng.standard_normal((6, res, res, res)).astype(np.float32)
        sdf[1] = np.abs(sdf[1])  # all positive: skipped
        c = rng.uniform(0, 5, (6, 3)).astype(np.float32)
        verts, faces = MO.marching_cubes(c, sdf, 0.2)
        nv0 = 0
        for v in range(6):
            s = sdf[v]
            if s.min() > 0 or s.max() < 0:
                continue
            pos = s > 0
            n_cross = int((pos[1:] != pos[:-1]).sum() + (pos[:, 1:] != pos[:, :-1]).sum()
                          + (pos[:, :, 1:] != pos[:, :, :-1]).sum())
            vv = verts[nv0:nv0 + n_cross]
            ff = faces[(faces >= nv0).all(1) & (faces < nv0 + n_cross).all(1)] - nv0
            _check_crack_free(vv, ff, c[v] - 0.1, c[v] + 0.1)
            nv0 += n_cross
        assert nv0 == verts.shape[0]
        assert faces.min() >= 0 and faces.max() < verts.shape[0]


def test_sphere_is_closed_with_outward_normals():
    res, vs = 16, 1.0
    x = torch.linspace(-0.5, 0.5, res).numpy()
    xx, yy, zz = np.meshgrid(x, x, x, indexing="ij")
    ctr = np.array([0.03, -0.02, 0.01])
    sdf = (np.sqrt((xx - ctr[0]) ** 2 + (yy - ctr[1]) ** 2 + (zz - ctr[2]) ** 2) - 0.33).astype(np.float32)
    verts, faces = MO.marching_cubes(np.zeros((1, 3), np.float32), sdf[None], vs)
    edges = {tuple(sorted(e)) for f in faces.tolist() for e in ((f[0], f[1]), (f[1], f[2]), (f[2], f[0]))}
    assert verts.shape[0] - len(edges) + faces.shape[0] == 2  # a sphere
    _check_crack_free(verts, faces, -0.5, 0.5)
    a, b, c = verts[faces[:, 0]], verts[faces[:, 1]], verts[faces[:, 2]]
    n = np.cross(b - a, c - a)
    out = (a + b + c) / 3 - ctr
    assert ((n * out).sum(-1) > 0).all()  # towards sdf > 0
    r = np.linalg.norm(verts - ctr, axis=-1)
    assert np.abs(r - 0.33).max() < 0.01


def test_vertex_rows_follow_floor_division():
    vox = np.array([[3, 4, 5, 1], [0, 0, 0, 1], [3, 4, 6, 1]], np.float32)
    verts = np.array([[0.61, 0.81, 1.01], [0.01, 0.05, 0.19], [0.6, 0.8, 1.2], [-0.01, 0.0, 0.0]], np.float32)
    rows = MO.vertex_voxel_rows(verts, vox, 0.2)
    assert rows.tolist() == [0, 1, 2, -1]
