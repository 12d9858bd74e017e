"""`svo.Octree` equivalent (torch.classes.svo.Octree, bindings.cpp:11-35) over
libpsvo's C++ builder.

Method names, argument meaning and outputs follow octree.cpp: node ids are
creation order (root 0), get_centres_and_children() returns
(voxels f32[N,4], children f32[N,8], features i32[N,8], pcd_xyz, pcd_color).
Per-node point samples (octree.cpp:198-239, read only by the disabled
get_features_pcd path, render_helpers.py:481) are not stored: the last two
outputs are zero tensors of the reference's shapes.  Pickling replays the
inserts like the reference's def_pickle (bindings.cpp:27-35).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L


def _zeros_view(n, k, c, device="cpu"):
    """[n, k, c] zeros without the memory: the per-node point samples the
    reference exports (octree.cpp:641-655) feed only disabled paths."""
    return torch.zeros((1, 1, 1), dtype=torch.float32, device=device).expand(n, k, c)


class Octree:
    def __init__(self):
        self._h = None
        self._inserted = []
        self.size = self.feat_dim = self.max_num = 0
        self.voxel_size = 0.0

    # octree.cpp:46-67
    def init(self, grid_dim, feat_dim, voxel_size, max_num=8):
        self.close()
        h = L.lib().psvo_octree_new(int(grid_dim), int(feat_dim), float(voxel_size), int(max_num))
        if not h:
            raise RuntimeError(f"Octree.init: grid_dim must be a power of two >= 2 (got {grid_dim})")
        self._h = h
        self.size, self.feat_dim, self.voxel_size, self.max_num = int(grid_dim), int(feat_dim), float(voxel_size), int(max_num)
        self._inserted = []

    def _check(self):
        if not self._h:
            raise RuntimeError("Octree not initialized!")

    @staticmethod
    def _as_int3(pts):
        a = pts.detach().cpu().numpy() if isinstance(pts, torch.Tensor) else np.asarray(pts)
        a = np.ascontiguousarray(a, dtype=np.int32)
        if a.ndim != 2 or a.shape[1] != 3:
            raise RuntimeError(f"Point dimensions mismatch: inputs are {a.shape[-1] if a.ndim else 0} expect 3")
        return a

    # octree.cpp:104-294
    def insert(self, pts, color=None, pcd=None):
        self._check()
        a = self._as_int3(pts)
        self._inserted.append(a)
        L.call("psvo_octree_insert", self._h, a.ctypes.data_as(L._vp), int(a.shape[0]))

    def try_insert(self, pts):
        self._check()
        a = self._as_int3(pts)
        return float(L.lib().psvo_octree_try_insert(self._h, a.ctypes.data_as(L._vp), int(a.shape[0])))

    def count_nodes(self):
        self._check()
        return int(L.lib().psvo_octree_count(self._h))

    def count_leaf_nodes(self):
        self._check()
        return int(L.lib().psvo_octree_count_leaves(self._h))

    def has_voxel(self, pts):
        self._check()
        p = pts.tolist() if isinstance(pts, torch.Tensor) else list(pts)
        if len(p) != 3:
            return False
        return bool(L.lib().psvo_octree_has_voxel(self._h, int(p[0]), int(p[1]), int(p[2])))

    def export_arrays(self):
        """(voxels, children, features) as numpy arrays (host)."""
        self._check()
        n = self.count_nodes()
        voxels = np.empty((n, 4), np.float32)
        children = np.empty((n, 8), np.float32)
        features = np.empty((n, 8), np.int32)
        L.call("psvo_octree_export", self._h, voxels.ctypes.data_as(L._vp), children.ctypes.data_as(L._vp),
               features.ctypes.data_as(L._vp))
        return voxels, children, features

    # octree.cpp:561-687
    def get_centres_and_children(self):
        v, c, f = self.export_arrays()
        n = v.shape[0]
        return (torch.from_numpy(v), torch.from_numpy(c), torch.from_numpy(f), _zeros_view(n, self.max_num, 4),
                _zeros_view(n, self.max_num, 3))

    def get_leaf_voxels(self):
        """SURFACE leaves' integer corners in the reference's depth-first
        child-index order (octree.cpp:480-505)."""
        n = L.lib().psvo_octree_leaf_voxels(self._h, None, 0)
        if n < 0:
            raise L.PsvoError("octree_leaf_voxels failed")
        out = torch.empty((n, 3), dtype=torch.float32)
        if n:
            L.lib().psvo_octree_leaf_voxels(self._h, out.data_ptr(), n)
        return out

    def close(self):
        if self._h:
            L.lib().psvo_octree_free(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __getstate__(self):
        return (self.size, self.feat_dim, self.voxel_size, [a.copy() for a in self._inserted], self.max_num)

    def __setstate__(self, state):
        self._h = None
        size, feat_dim, voxel_size, inserted, max_num = state
        self.init(size, feat_dim, voxel_size, max_num)
        for a in inserted:
            self.insert(a)


class DeviceOctree:
    """`svo.Octree` built on the device (csrc/octree_gpu.hip):
    the same node ids, types and links as Octree / octree.cpp:104-294 (creation
    order via a hash-and-scan construction), kept in HBM across inserts, and
    exported (get_centres_and_children, octree.cpp:561-687, or the renderer's
    map_states arrays) without a host walk or copy."""

    def __init__(self, device="cuda"):
        self.device = torch.device(device)
        self._h = None
        self.size = self.feat_dim = self.max_num = 0
        self.voxel_size = 0.0

    def init(self, grid_dim, feat_dim, voxel_size, max_num=8, capacity=1 << 16):
        self.close()
        h = L.lib().psvo_dtree_new(L.stream_of(self.device), int(grid_dim), int(capacity))
        if not h:
            raise RuntimeError(f"DeviceOctree.init: {L.lib().psvo_last_error().decode()}")
        self._h = h
        self.size, self.feat_dim, self.voxel_size, self.max_num = int(grid_dim), int(feat_dim), float(voxel_size), int(max_num)

    def _check(self):
        if not self._h:
            raise RuntimeError("Octree not initialized!")

    def _vox(self, pts):
        t = torch.as_tensor(pts)
        if t.dim() != 2 or t.shape[1] != 3:
            raise RuntimeError(f"Point dimensions mismatch: inputs are {t.shape[-1] if t.dim() else 0} expect 3")
        return t.to(device=self.device, dtype=torch.int32).contiguous()

    def insert(self, pts, color=None, pcd=None):
        self._check()
        v = self._vox(pts)
        L.call("psvo_dtree_insert", self._h, L.stream_of(self.device), v, v.shape[0])

    def count_nodes(self):
        self._check()
        return int(L.lib().psvo_dtree_count(self._h))

    def count_leaf_nodes(self):
        self._check()
        return int(L.lib().psvo_dtree_count_leaves(self._h, L.stream_of(self.device)))

    def _probe(self, pts, corners):
        v = self._vox(pts)
        hit = torch.empty((v.shape[0] * corners,), dtype=torch.int32, device=self.device)
        L.call("psvo_dtree_probe", self._h, L.stream_of(self.device), v, v.shape[0], corners, hit)
        return v, hit

    def has_voxel(self, pts):
        self._check()
        p = torch.as_tensor(pts).reshape(-1)
        if p.numel() != 3:
            return False
        return bool(self._probe(p.reshape(1, 3), 1)[1][0].item())

    def try_insert(self, pts):
        """octree.cpp:381-417: fraction of the distinct corner keys already present."""
        self._check()
        v, hit = self._probe(pts, 8)
        inc = torch.tensor([[0, 0, 0], [0, 0, 1], [0, 1, 0], [0, 1, 1], [1, 0, 0], [1, 0, 1], [1, 1, 0], [1, 1, 1]],
                           dtype=torch.int32, device=self.device)
        corners = (v[:, None, :] + inc[None]).reshape(-1, 3)
        uniq, inv = torch.unique(corners, dim=0, return_inverse=True)
        if uniq.shape[0] == 0:
            return 0.0
        present = torch.zeros((uniq.shape[0],), dtype=torch.int32, device=self.device).scatter_reduce(
            0, inv, hit, reduce="amax")
        return float(present.sum().item()) / float(uniq.shape[0])

    def export_arrays(self):
        """(voxels f32[N,4], children f32[N,8], features i32[N,8]) on the device."""
        self._check()
        n = self.count_nodes()
        v = torch.empty((n, 4), dtype=torch.float32, device=self.device)
        c = torch.empty((n, 8), dtype=torch.float32, device=self.device)
        f = torch.empty((n, 8), dtype=torch.int32, device=self.device)
        L.call("psvo_dtree_export", self._h, L.stream_of(self.device), float(self.voxel_size), v, c, f, None, None)
        return v, c, f

    def get_centres_and_children(self):
        v, c, f = self.export_arrays()
        n = v.shape[0]
        return (v, c, f, _zeros_view(n, self.max_num, 4, self.device), _zeros_view(n, self.max_num, 3, self.device))

    def render_arrays(self, voxel_size):
        """map_states' (voxel_center_xyz f32[N,3], voxel_structure i32[N,9],
        voxel_vertex_idx i32[N,8]) written directly by the export kernel."""
        self._check()
        n = self.count_nodes()
        centres = torch.empty((n, 3), dtype=torch.float32, device=self.device)
        structure = torch.empty((n, 9), dtype=torch.int32, device=self.device)
        features = torch.empty((n, 8), dtype=torch.int32, device=self.device)
        L.call("psvo_dtree_export", self._h, L.stream_of(self.device), float(voxel_size), None, None, features,
               centres, structure)
        return centres, structure, features

    def close(self):
        if self._h:
            L.lib().psvo_dtree_free(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def map_states(tree: Octree, embeddings: torch.Tensor, voxel_size: float, device=None):
    """Mapping.update_grid_pcd_features (mapping.py:300-406) without the
    pointcloud fields: centres, [N,9] structure, vertex ids on `device`.  A
    DeviceOctree hands over its device arrays directly."""
    if isinstance(tree, DeviceOctree):
        centres, structure, features = tree.render_arrays(voxel_size)
        n = centres.shape[0]
        dev = device if device is not None else embeddings.device
        return {
            "voxel_vertex_idx": features.to(dev),
            "voxel_center_xyz": centres.to(dev),
            "voxel_structure": structure.to(dev),
            "voxel_vertex_emb": embeddings,
            "pointclouds_xyz": _zeros_view(n, tree.max_num, 4),
            "pointclouds_color": _zeros_view(n, tree.max_num, 3),
        }
    voxels, children, features, pcd_xyz, pcd_color = tree.get_centres_and_children()
    centres = (voxels[:, :3] + voxels[:, -1:] / 2) * voxel_size
    structure = torch.cat([children, voxels[:, -1:]], -1).int()
    dev = device if device is not None else embeddings.device
    return {
        "voxel_vertex_idx": features.to(dev),
        "voxel_center_xyz": centres.float().to(dev),
        "voxel_structure": structure.to(dev),
        "voxel_vertex_emb": embeddings,
        "pointclouds_xyz": pcd_xyz,
        "pointclouds_color": pcd_color,
    }
