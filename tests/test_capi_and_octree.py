"""CPU-side checks of the product library: it loads, exports every symbol
include/psvo.h declares, and its CPU octree builder reproduces the oracle /
golden node numbering and export exactly.  No GPU compute calls."""
import os
import re

import numpy as np
import pytest
import torch

from psvo import _lib as L
from psvo.octree import Octree, map_states
from oracle import oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    src = open(os.path.join(REPO, "include", "psvo.h")).read()
    return sorted(set(re.findall(r"\b(psvo_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = L.lib()
    declared = _header_symbols()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(L.exported_symbols())
    assert lib.psvo_version().decode().startswith("psvo")


def test_library_links_torch_hip_runtime():
    maps = open("/proc/self/maps").read()
    libs = set(re.findall(r"\S*libamdhip64\S*", maps))
    assert len(libs) <= 1, libs


def test_octree_matches_golden(golden):
    name, g = golden
    t = Octree()
    t.init(int(g["grid_dim"]), 16, 0.2, 8)
    t.insert(torch.from_numpy(g["vox"]), None, None)
    v, c, f = t.export_arrays()
    np.testing.assert_array_equal(v, g["voxels"])
    np.testing.assert_array_equal(c, g["children"])
    np.testing.assert_array_equal(f, g["features"])
    assert t.count_nodes() == g["voxels"].shape[0]
    ms = map_states(t, torch.zeros(1), 0.2, device="cpu")
    np.testing.assert_array_equal(ms["voxel_center_xyz"].numpy(), g["centres"])
    np.testing.assert_array_equal(ms["voxel_structure"].numpy(), g["structure"])


@pytest.mark.parametrize("grid_dim,n,seed", [(16, 40, 0), (64, 600, 1), (256, 3000, 2), (1024, 2000, 3)])
def test_octree_matches_oracle_incremental(grid_dim, n, seed):
    """Several insert() calls with duplicates and FEATURE→SURFACE promotion."""
    rng = np.random.default_rng(seed)
    vox = rng.integers(0, grid_dim - 1, size=(n, 3)).astype(np.int32)
    vox = np.concatenate([vox, vox[: n // 4] + 1], 0).clip(0, grid_dim - 2).astype(np.int32)
    t, o = Octree(), O.OracleOctree(grid_dim)
    t.init(grid_dim, 16, 0.2, 8)
    for part in np.array_split(vox, 3):
        t.insert(part)
        o.insert(part)
    a, b = t.export_arrays(), o.export()
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    assert t.count_leaf_nodes() == int((b[2][:, 0] >= 0).sum())
    assert t.has_voxel(vox[0].tolist())
    assert 0.99 <= t.try_insert(vox[:10]) <= 1.0


def test_octree_pickle_replays_inserts():
    import pickle
    rng = np.random.default_rng(5)
    vox = rng.integers(0, 60, size=(200, 3)).astype(np.int32)
    t = Octree()
    t.init(64, 16, 0.2, 8)
    t.insert(vox)
    t2 = pickle.loads(pickle.dumps(t))
    for x, y in zip(t.export_arrays(), t2.export_arrays()):
        np.testing.assert_array_equal(x, y)


def test_grid_module_rejects_host_tensors():
    import grid
    x = torch.zeros(1, 4, 3)
    with pytest.raises(RuntimeError, match="CUDA"):
        grid.svo_intersect(x, x, torch.zeros(1, 2, 3), torch.zeros(1, 2, 9, dtype=torch.int32), 0.2, 50)
    with pytest.raises(RuntimeError, match="contiguous"):
        grid.svo_intersect(x.transpose(1, 2), x, x, x, 0.2, 50)
    with pytest.raises(RuntimeError, match="CUDA"):
        grid.ball_intersect(x, x, x, 0.1, 4)


def test_torchscript_octree_class_matches_python_octree():
    """torch.classes.svo.Octree (lib/libsvo_torch.so, the reference's
    TorchScript class: bindings.cpp:4-35) loaded the way mapping.py:18-19,
    86-87 loads it: insert, the counts, has_voxel / try_insert, the export
    and a pickle round trip (def_pickle replays the inserts) equal the Python
    psvo.octree.Octree on the same voxels."""
    import io
    import pickle
    from psvo import synthetic as syn
    torch.classes.load_library(os.path.join(REPO, "proud-slam_amd", "lib", "libsvo_torch.so"))
    vox = syn.surface_voxels(syn.room0(), seed=0)
    half = vox.shape[0] // 2
    t = torch.classes.svo.Octree()
    t.init(256, 16, 0.2, 8)
    ref = Octree()
    ref.init(256, 16, 0.2, 8)
    for part in (vox[:half], vox[half:]):
        pts = torch.from_numpy(part).int()
        t.insert(pts, pts, pts.float())  # mapping.py:292: (voxels, colors, points)
        ref.insert(part)
    assert t.count_nodes() == ref.count_nodes() and t.count_leaf_nodes() == ref.count_leaf_nodes()
    got = t.get_centres_and_children()
    want = ref.get_centres_and_children()
    assert len(got) == 5
    for a, b in zip(got[:3], want[:3]):
        assert torch.equal(a, b)
    assert tuple(got[3].shape) == (ref.count_nodes(), 8, 4) and tuple(got[4].shape) == (ref.count_nodes(), 8, 3)
    assert t.has_voxel(torch.from_numpy(vox[0]).int()) == ref.has_voxel(vox[0])
    probe = torch.from_numpy(vox[:64] + 1).int()
    assert t.try_insert(probe) == ref.try_insert(vox[:64] + 1)
    assert torch.equal(t.get_leaf_voxels(), ref.get_leaf_voxels())
    # pickling: the construction inputs, replayed into a fresh tree
    buf = io.BytesIO()
    torch.save(t, buf)  # the TorchScript pickler (def_pickle)
    buf.seek(0)
    t2 = torch.load(buf, weights_only=False)  # our own file, written above
    assert t2.count_nodes() == t.count_nodes()
    for a, b in zip(t2.get_centres_and_children()[:3], got[:3]):
        assert torch.equal(a, b)
    t3 = pickle.loads(pickle.dumps(t))
    assert torch.equal(t3.get_centres_and_children()[0], got[0])
    with pytest.raises(RuntimeError, match="not initialized"):
        torch.classes.svo.Octree().count_nodes()


def test_leaf_voxels_in_reference_dfs_order():
    """Octree::get_leaf_voxels (octree.cpp:480-505) walks the tree depth
    first in child-index order (cid = x-bit + 2·y-bit + 4·z-bit, octree.cpp
    :419-439) and emits only SURFACE leaves — not in creation order, and not
    the FEATURE corner leaves every insert adds.  Hand-built tree inserted
    in the reverse of that order (16³: every corner inside the grid)."""
    t = Octree()
    t.init(16, 16, 0.2, 8)
    t.insert(np.array([[7, 7, 7], [4, 0, 0], [0, 0, 0], [0, 4, 0]], dtype=np.int32))
    got = t.get_leaf_voxels()
    want = torch.tensor([[0, 0, 0], [4, 0, 0], [0, 4, 0], [7, 7, 7]], dtype=torch.float32)
    assert torch.equal(got, want)
    # the same order as a DFS over the exported child table, on a bigger tree
    from psvo import synthetic as syn
    vox = syn.surface_voxels(syn.room0(), seed=1)
    big = Octree()
    big.init(256, 16, 0.2, 8)
    big.insert(vox)
    v, c, f = big.export_arrays()
    order, stack = [], [0]
    while stack:
        nd = stack.pop()
        if f[nd, 0] >= 0:  # SURFACE rows carry their corner rows (features)
            order.append(v[nd, :3])
            continue
        stack.extend(int(k) for k in c[nd][::-1] if k >= 0)
    assert torch.equal(big.get_leaf_voxels(), torch.from_numpy(np.stack(order).astype(np.float32)))
    assert big.get_leaf_voxels().shape[0] == big.count_leaf_nodes()
