"""The device octree builder (psvo.octree.DeviceOctree, csrc/octree_gpu.hip)
against the CPU builder that the golden fixtures pin (Octree::insert,
octree.cpp:104-294; get_centres_and_children, :561-687): identical node ids,
types, links and corner features after incremental inserts with duplicates,
FEATURE→SURFACE promotion and capacity growth; map_states arrays
bit-identical; has_voxel / try_insert / leaf counts equal."""
import numpy as np
import pytest
import torch

from psvo.octree import DeviceOctree, Octree, map_states

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _batches(grid_dim, n, seed):
    rng = np.random.default_rng(seed)
    vox = rng.integers(0, grid_dim - 1, size=(n, 3)).astype(np.int32)
    vox = np.concatenate([vox, vox[: n // 4] + 1, vox[: n // 8]], 0).clip(0, grid_dim - 2).astype(np.int32)
    return np.array_split(vox, 3)


@pytest.mark.parametrize("grid_dim,n,seed,cap", [(16, 40, 0, 1024), (64, 600, 1, 1024), (256, 3000, 2, 1 << 16),
                                                 (1024, 4000, 3, 1024)])
def test_device_octree_matches_cpu_builder(grid_dim, n, seed, cap):
    cpu, dev = Octree(), DeviceOctree(DEV)
    cpu.init(grid_dim, 16, 0.2, 8)
    dev.init(grid_dim, 16, 0.2, 8, capacity=cap)  # small capacities force growth + rehash
    for part in _batches(grid_dim, n, seed):
        cpu.insert(part)
        dev.insert(torch.from_numpy(part))
        assert dev.count_nodes() == cpu.count_nodes()
        for a, b in zip(cpu.export_arrays(), dev.export_arrays()):
            np.testing.assert_array_equal(a, b.cpu().numpy())
    assert dev.count_leaf_nodes() == cpu.count_leaf_nodes()
    probe = _batches(grid_dim, 64, seed + 100)[0]
    for p in probe[:16]:
        assert dev.has_voxel(p.tolist()) == cpu.has_voxel(p.tolist())
    assert dev.try_insert(probe) == pytest.approx(cpu.try_insert(probe), abs=0)
    ms_c = map_states(cpu, torch.zeros(1), 0.2, device="cpu")
    ms_d = map_states(dev, torch.zeros(1, device=DEV), 0.2)
    for k in ("voxel_center_xyz", "voxel_structure", "voxel_vertex_idx"):
        assert torch.equal(ms_c[k], ms_d[k].cpu()), k


def test_device_octree_matches_golden(golden):
    name, g = golden
    t = DeviceOctree(DEV)
    t.init(int(g["grid_dim"]), 16, 0.2, 8)
    t.insert(torch.from_numpy(g["vox"]))
    v, c, f = (x.cpu().numpy() for x in t.export_arrays())
    np.testing.assert_array_equal(v, g["voxels"])
    np.testing.assert_array_equal(c, g["children"])
    np.testing.assert_array_equal(f, g["features"])
    ms = map_states(t, torch.zeros(1, device=DEV), 0.2)
    np.testing.assert_array_equal(ms["voxel_center_xyz"].cpu().numpy(), g["centres"])
    np.testing.assert_array_equal(ms["voxel_structure"].cpu().numpy(), g["structure"])


def test_device_octree_scene_scale():
    """A whole synthetic scene (config B shape) in one insert, then a second
    frame's voxels: same arrays as the CPU builder."""
    from psvo import synthetic as syn
    scene = syn.room0()
    vox = syn.surface_voxels(scene, seed=0)
    half = vox.shape[0] // 2
    cpu, dev = Octree(), DeviceOctree(DEV)
    cpu.init(scene.grid_dim, 16, scene.voxel_size, 8)
    dev.init(scene.grid_dim, 16, scene.voxel_size, 8)
    for part in (vox[:half], vox[half:]):
        cpu.insert(part)
        dev.insert(torch.from_numpy(np.ascontiguousarray(part)))
    for a, b in zip(cpu.export_arrays(), dev.export_arrays()):
        np.testing.assert_array_equal(a, b.cpu().numpy())
