"""Mesh extraction on the device against the oracle:
lattice scores and point colours vs the reference's own get_scores /
eval_points output (golden M_mesh_A, decoder tolerance), marching cubes bit
for bit vs the oracle on the same sdf lattices (random fields at several
resolutions, the golden lattices), the vertex → voxel lookup vs the brute
force comparison of mesh_util.py:112-125, and create_mesh end to end."""
import types

import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import mesh_oracle as MO

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _decoder(g):
    from psvo.decoder import Decoder
    dec = Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none").to(DEV)
    dec.load_state_dict({k[len("dec."):]: torch.from_numpy(v) for k, v in g.items() if k.startswith("dec.")})
    return dec


def _states(g):
    return {"voxel_vertex_idx": torch.from_numpy(g["features"]).to(DEV),
            "voxel_center_xyz": torch.from_numpy(g["centres"]).to(DEV),
            "voxel_vertex_emb": torch.from_numpy(g["embeddings"]).to(DEV)}


def test_get_scores_matches_reference():
    from psvo.mesh import get_scores
    g = load_golden("M_mesh_A")
    out = get_scores(_decoder(g), _states(g), float(g["voxel_size"]), bits=int(g["res"]))
    assert out.shape == g["scores"].shape and out.device.type == "cpu"
    np.testing.assert_allclose(out.numpy(), g["scores"], rtol=0, atol=2e-5)


def test_eval_points_matches_reference():
    from psvo.mesh import eval_points
    g = load_golden("M_mesh_A")
    rgb = eval_points(_decoder(g), _states(g), torch.from_numpy(g["points"]), torch.from_numpy(g["point_idx"]),
                      float(g["voxel_size"]))
    np.testing.assert_allclose(rgb.numpy(), g["point_rgb"], rtol=0, atol=2e-5)


def test_sdf_only_decoder_is_bit_identical():
    """The sdf-only forward (mesh lattices) gives the full forward's sdf bit for bit."""
    from psvo.mesh import lattice_scores
    g = load_golden("M_mesh_A")
    dec, st = _decoder(g), _states(g)
    _, sdf_full = lattice_scores(dec, st, float(g["voxel_size"]), 8)
    rgb, sdf_only = lattice_scores(dec, st, float(g["voxel_size"]), 8, with_rgb=False)
    assert rgb is None
    assert torch.equal(sdf_full, sdf_only)
    # ragged sizes through the persistent loop: m not a multiple of the 256-sample tile
    from psvo.mesh import _decode, _decode_sdf
    feat = torch.randn(100003, 16, device=DEV) * 0.3
    out = torch.empty(100003, device=DEV)
    _decode_sdf(dec, feat, out)
    assert torch.equal(out, _decode(dec, feat)[1])


@pytest.mark.parametrize("res", [2, 5, 8, 16])
def test_marching_cubes_bit_exact_random(res):
    from psvo.mesh import marching_cubes_device
    rng = np.random.default_rng(res)
    n = 200 if res <= 8 else 40
    sdf = rng.standard_normal((n, res, res, res)).astype(np.float32)
    sdf[::7] = np.abs(sdf[::7])        # skipped voxels (no sign change)
    sdf[3::11] *= -1 if res > 2 else 1
    sdf[5, 0, 0, 0] = 0.0              # an exact zero (counts as "not +")
    c = rng.uniform(0, 30, (n, 3)).astype(np.float32)
    v_ref, f_ref = MO.marching_cubes(c, sdf, 0.2)
    v, f = marching_cubes_device(torch.from_numpy(c).to(DEV), torch.from_numpy(sdf).to(DEV), 0.2, res)
    np.testing.assert_array_equal(v.cpu().numpy(), v_ref)
    np.testing.assert_array_equal(f.cpu().numpy(), f_ref)


def test_marching_cubes_on_golden_lattices():
    from psvo.mesh import MeshExtractor
    g = load_golden("M_mesh_A")
    mx = MeshExtractor(types.SimpleNamespace(mapper_specs={"voxel_size": 0.2}))
    v, f = mx.marching_cubes(torch.from_numpy(g["centres"]).to(DEV), torch.from_numpy(g["scores"]))
    v_ref, f_ref = MO.marching_cubes(g["centres"], g["scores"][..., 3], 0.2)
    assert v_ref.shape[0] > 0
    np.testing.assert_array_equal(v, v_ref)
    np.testing.assert_array_equal(f, f_ref)


def test_vertex_rows_match_brute_force():
    from psvo.mesh import vertex_rows
    rng = np.random.default_rng(1)
    vox = np.unique(rng.integers(0, 40, (3000, 3)), axis=0)
    vox = np.concatenate([vox, np.ones((vox.shape[0], 1), np.int64)], 1).astype(np.float32)
    vox = vox[rng.permutation(vox.shape[0])]
    pts = rng.uniform(-0.5, 8.5, (20000, 3)).astype(np.float32)
    pts[:100] = (vox[:100, :3] * 0.2).astype(np.float32)  # exact voxel corners
    rows = vertex_rows(torch.from_numpy(vox).to(DEV), torch.from_numpy(pts).to(DEV), 0.2).cpu().numpy()
    ref = MO.vertex_voxel_rows(pts, vox, 0.2)
    np.testing.assert_array_equal(rows, ref)
    assert (ref >= 0).sum() > 400


def test_create_mesh_end_to_end():
    """room0 octree → SURFACE voxels → create_mesh(require_color): the device
    mesh equals the oracle's marching cubes on the device lattice sdf, colours
    equal the point-colour path at the oracle's vertex rows."""
    from psvo import synthetic as syn
    from psvo.decoder import Decoder
    from psvo.mesh import MeshExtractor, lattice_scores, surface_states
    from psvo.octree import Octree
    scene = syn.room0()
    tree = Octree()
    tree.init(scene.grid_dim, 16, scene.voxel_size, 8)
    tree.insert(syn.surface_voxels(scene, seed=0))
    voxels, _, features = tree.export_arrays()
    gen = torch.Generator().manual_seed(0)
    emb = (torch.randn(voxels.shape[0], 16, generator=gen) * 0.3).to(DEV)
    torch.manual_seed(0)
    dec = Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none").to(DEV)
    sv, states = surface_states(torch.from_numpy(voxels), torch.from_numpy(features), emb, scene.voxel_size)
    mx = MeshExtractor(types.SimpleNamespace(mapper_specs={"voxel_size": scene.voxel_size}))
    mesh = mx.create_mesh(dec, states, scene.voxel_size, sv, require_color=True, offset=-10, res=8)
    _, sdf = lattice_scores(dec, states, scene.voxel_size, 8)
    v_ref, f_ref = MO.marching_cubes(states["voxel_center_xyz"].cpu().numpy(), sdf.view(-1, 8, 8, 8).cpu().numpy(),
                                     scene.voxel_size)
    assert f_ref.shape[0] > 1000
    np.testing.assert_array_equal(mesh.vertices, v_ref - 10)
    np.testing.assert_array_equal(mesh.triangles, f_ref)
    pick = np.random.default_rng(0).choice(v_ref.shape[0], 3000, replace=False)
    rows = MO.vertex_voxel_rows(v_ref[pick], sv.cpu().numpy(), scene.voxel_size)
    assert (rows >= 0).mean() > 0.5
    ok = rows >= 0
    g_rgb = MO.eval_points({k: v.cpu() for k, v in dec.state_dict().items()}, states["voxel_center_xyz"].cpu(),
                           states["voxel_vertex_idx"].cpu(), emb.cpu(), v_ref[pick][ok], rows[ok], scene.voxel_size)
    np.testing.assert_allclose(mesh.vertex_colors[pick][ok], g_rgb.numpy(), rtol=0, atol=2e-5)
    assert (mesh.vertex_colors[pick][~ok] == 0).all()
    nrm = np.linalg.norm(mesh.vertex_normals, axis=-1)
    assert np.isfinite(nrm).all() and nrm.max() < 1 + 1e-4 and (np.abs(nrm - 1) < 1e-4).mean() > 0.99
