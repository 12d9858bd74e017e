"""Mesh extraction on the device: drop-ins for
render_helpers.get_scores / eval_points (render_helpers.py:243-328) and
utils.mesh_util.MeshExtractor (mesh_util.py:10-169), on csrc/mesh.hip.

The reference evaluates the decoder 32 voxels at a time with a device→host
copy per chunk, runs skimage marching cubes voxel by voxel on the host, and
finds each vertex's voxel by comparing it against every voxel (a [1000, N]
tensor per 1000 vertices).  Here: lattice features (one gather kernel) → the
fused decoder → marching cubes (count / offsets / emit kernels, one 16-byte
read-back for the output sizes) → a hash lookup of each vertex's voxel →
point features → the decoder for the colours; everything stays in HBM until
the mesh is returned.  The triangulation rule and its parity status are in
csrc/mesh.hip and DESIGN.md §6d.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L

_CHUNK_POINTS = 1 << 25  # lattice points per decoder call (2 GiB of features)


def _decode(sdf_network, feat):
    """[M, 16] features → (rgb [M, 3], sdf [M]) on the fused decoder (inference)."""
    out = sdf_network({"emb": feat})
    return out["color"], out["sdf"].reshape(-1)


def _decode_sdf(sdf_network, feat, out):
    """sdf only (Decoder.get_sdf): the fused decoder's sdf-only forward into `out`."""
    if not sdf_network.can_fuse(feat):
        out.copy_(sdf_network.get_values(feat)[:, 3])
        return
    w = sdf_network.W
    images = torch.empty((int(L.lib().psvo_mlp_image_floats_w(w)),), dtype=torch.float32, device=feat.device)
    ps = [p.detach() for p in sdf_network.fused_params()]
    L.call("psvo_mlp_fwd", L.stream_of(feat.device), feat.shape[0], w, feat, *ps, images, out, None, None, None)


def surface_states(voxels, features, embeddings, voxel_size):
    """Mapping.extract_mesh's selection (mapping.py:420-431): the rows whose 8
    corner features all exist (SURFACE voxels).  Returns (voxels [n, 4],
    encoder_states dict) on the embeddings' device."""
    dev = embeddings.device
    voxels = torch.as_tensor(voxels).to(dev)
    features = torch.as_tensor(features).to(dev)
    keep = ~features.eq(-1).any(-1)
    sv, sf = voxels[keep].float(), features[keep]
    centres = (sv[:, :3] + sv[:, -1:] / 2) * voxel_size
    return sv, {"voxel_vertex_idx": sf.int().contiguous(), "voxel_center_xyz": centres.float().contiguous(),
                "voxel_vertex_emb": embeddings}


def _states(map_states):
    c = map_states["voxel_center_xyz"].float().contiguous()
    vi = map_states["voxel_vertex_idx"].to(c.device).int().contiguous()
    emb = map_states["voxel_vertex_emb"].detach().to(c.device).float().contiguous()
    if not c.is_cuda:
        raise RuntimeError("psvo.mesh: map states must be on the GPU (HIP kernels only)")
    return c, vi, emb


@torch.no_grad()
def lattice_scores(sdf_network, map_states, voxel_size, res=8, with_rgb=True):
    """Device (rgb [n·res³, 3] or None, sdf [n·res³]) of every voxel's res³
    lattice; with_rgb=False runs the sdf-only decoder (what marching cubes
    reads)."""
    c, vi, emb = _states(map_states)
    n = c.shape[0]
    n3 = res ** 3
    rgb = torch.empty((n * n3, 3), dtype=torch.float32, device=c.device) if with_rgb else None
    sdf = torch.empty((n * n3,), dtype=torch.float32, device=c.device)
    step = max(1, _CHUNK_POINTS // n3)
    for v0 in range(0, n, step):
        v1 = min(n, v0 + step)
        feat = torch.empty(((v1 - v0) * n3, 16), dtype=torch.float32, device=c.device)
        L.call("psvo_mesh_grid_feat", L.stream_of(c.device), v1 - v0, res, float(voxel_size), c[v0:v1],
               vi[v0:v1], emb, feat)
        if with_rgb:
            r, s = _decode(sdf_network, feat)
            if v1 - v0 == n:
                return r, s
            rgb[v0 * n3:v1 * n3] = r
            sdf[v0 * n3:v1 * n3] = s
        else:
            _decode_sdf(sdf_network, feat, sdf[v0 * n3:v1 * n3])
    return rgb, sdf


@torch.no_grad()
def get_scores(sdf_network, map_states, voxel_size, bits=8):
    """render_helpers.py:243-294: [n, bits, bits, bits, 4] = [rgb | sdf] (host tensor, as the reference)."""
    rgb, sdf = lattice_scores(sdf_network, map_states, voxel_size, bits)
    return torch.cat([rgb, sdf[:, None]], -1).view(-1, bits, bits, bits, 4).cpu()


@torch.no_grad()
def point_colours(sdf_network, map_states, xyz, rows, voxel_size):
    """Device rgb [n, 3] at points xyz [n, 3] of voxel rows [n] (row < 0 → 0)."""
    c, vi, emb = _states(map_states)
    xyz = xyz.reshape(-1, 3).float().contiguous()
    rows = rows.reshape(-1).int().contiguous()
    feat = torch.empty((xyz.shape[0], 16), dtype=torch.float32, device=c.device)
    L.call("psvo_mesh_point_feat", L.stream_of(c.device), xyz.shape[0], float(voxel_size), xyz, rows, c, vi, emb,
           feat)
    rgb, _ = _decode(sdf_network, feat)
    return rgb * (rows >= 0).unsqueeze(-1).float()


@torch.no_grad()
def eval_points(sdf_network, map_states, sampled_xyz, sampled_idx, voxel_size):
    """render_helpers.py:297-328: rgb [n, 3] (host tensor, as the reference)."""
    dev = map_states["voxel_center_xyz"].device
    xyz = torch.as_tensor(sampled_xyz).to(dev).reshape(-1, 3)
    if xyz.shape[0] == 0:
        return None
    return point_colours(sdf_network, map_states, xyz, torch.as_tensor(sampled_idx).to(dev), voxel_size).cpu()


@torch.no_grad()
def marching_cubes_device(centres, sdf, voxel_size, res):
    """Device (verts f32 [V, 3], faces i32 [F, 3]) of the per-voxel meshes of
    sdf [n·res³] (voxel-major lattices), vertices in world coordinates."""
    centres = centres.float().contiguous()
    sdf = sdf.reshape(-1).float().contiguous()
    n = centres.shape[0]
    dev = centres.device
    if n == 0:
        return (torch.zeros((0, 3), dtype=torch.float32, device=dev),
                torch.zeros((0, 3), dtype=torch.int32, device=dev))
    if sdf.numel() != n * res ** 3:
        raise ValueError(f"marching_cubes: sdf has {sdf.numel()} values, expected {n} x {res}^3")
    nv = torch.empty(n, dtype=torch.int32, device=dev)
    nt = torch.empty(n, dtype=torch.int32, device=dev)
    vbase = torch.empty(n, dtype=torch.int64, device=dev)
    tbase = torch.empty(n, dtype=torch.int64, device=dev)
    totals = torch.empty(2, dtype=torch.int64, device=dev)
    st = L.stream_of(dev)
    L.call("psvo_mesh_mc_count", st, n, res, sdf, nv, nt, vbase, tbase, totals)
    n_v, n_f = (int(x) for x in totals.cpu())
    if n_v >= 2 ** 31:
        raise RuntimeError(f"marching_cubes: {n_v} vertices exceed int32 face indices")
    verts = torch.empty((n_v, 3), dtype=torch.float32, device=dev)
    faces = torch.empty((n_f, 3), dtype=torch.int32, device=dev)
    if n_v > 0:
        L.call("psvo_mesh_mc_emit", st, n, res, float(voxel_size), sdf, centres, nv, vbase, tbase, verts, faces)
    return verts, faces


@torch.no_grad()
def vertex_rows(voxels, verts, voxel_size):
    """Row of the voxel whose min corner equals vert // voxel (mesh_util.py:112-125), −1 if none."""
    voxels = voxels.float().contiguous()
    verts = verts.float().contiguous()
    dev = verts.device
    table = torch.empty(int(L.lib().psvo_mesh_vox_map_slots(voxels.shape[0])) * 4, dtype=torch.int32, device=dev)
    rows = torch.empty(verts.shape[0], dtype=torch.int32, device=dev)
    L.call("psvo_mesh_vertex_rows", L.stream_of(dev), voxels.shape[0], voxels, verts.shape[0], verts,
           float(voxel_size), table, rows)
    return rows


class Mesh:
    """The fields create_mesh fills in the reference's open3d TriangleMesh
    (mesh_util.py:135-146): vertices (offset applied), triangles,
    vertex_colors, vertex_normals (area-weighted, as compute_vertex_normals)."""

    def __init__(self, vertices, triangles, vertex_colors=None, vertex_normals=None):
        self.vertices, self.triangles = vertices, triangles
        self.vertex_colors, self.vertex_normals = vertex_colors, vertex_normals

    def __repr__(self):
        return f"Mesh({self.vertices.shape[0]} vertices, {self.triangles.shape[0]} triangles)"


def _vertex_normals(verts, faces):
    """Area-weighted vertex normals, unit length (open3d compute_vertex_normals)."""
    if faces.shape[0] == 0:
        return torch.zeros_like(verts)
    f = faces.long()
    a, b, c = verts[f[:, 0]], verts[f[:, 1]], verts[f[:, 2]]
    fn = torch.cross(b - a, c - a, dim=-1)
    vn = torch.zeros_like(verts)
    for k in range(3):
        vn.index_add_(0, f[:, k], fn)
    return vn / vn.norm(dim=-1, keepdim=True).clamp_min(1e-12)


class MeshExtractor:
    """utils.mesh_util.MeshExtractor (mesh_util.py:10-169) on the device."""

    def __init__(self, args):
        self.voxel_size = args.mapper_specs["voxel_size"]
        self.rays_d = None
        self.depth_points = None

    @torch.no_grad()
    def linearize_id(self, xyz, n_xyz):
        return xyz[:, 2] + n_xyz[-1] * xyz[:, 1] + (n_xyz[-1] * n_xyz[-2]) * xyz[:, 0]

    @torch.no_grad()
    def downsample_points(self, points, voxel_size=0.01):
        """open3d voxel_down_sample: the mean of the points in each occupied voxel."""
        p = np.asarray(points, np.float64)
        if p.shape[0] == 0:
            return p
        key = np.floor((p - p.min(0)) / voxel_size).astype(np.int64)
        _, inv = np.unique(key, axis=0, return_inverse=True)
        inv = inv.reshape(-1)
        out = np.zeros((inv.max() + 1, 3))
        np.add.at(out, inv, p)
        return out / np.bincount(inv)[:, None]

    @torch.no_grad()
    def get_rays(self, w=None, h=None, K=None):
        w = self.w if w is None else w
        h = self.h if h is None else h
        if K is None:
            K = np.eye(3)
            K[0, 0] = self.K[0, 0] * w / self.w
            K[1, 1] = self.K[1, 1] * h / self.h
            K[0, 2] = self.K[0, 2] * w / self.w
            K[1, 2] = self.K[1, 2] * h / self.h
        ix, iy = torch.meshgrid(torch.arange(w), torch.arange(h), indexing="xy")
        return torch.stack([(ix - K[0, 2]) / K[0, 0], (iy - K[1, 2]) / K[1, 1], torch.ones_like(ix)], -1).float()

    @torch.no_grad()
    def get_valid_points(self, frame_poses, depth_maps):
        def back_project(pose, depth):
            pose = torch.as_tensor(pose, dtype=torch.float32)
            pts = (self.rays_d * torch.as_tensor(depth).unsqueeze(-1)).reshape(-1, 3)
            return (pts @ pose[:3, :3].transpose(-1, -2) + pose[:3, 3]).cpu().numpy()

        if isinstance(frame_poses, list):
            pts = np.concatenate([back_project(frame_poses[i], depth_maps[i])
                                  for i in range(0, len(frame_poses), 5)], 0)
            return self.downsample_points(pts)
        pts = back_project(frame_poses, depth_maps)
        self.depth_points = pts if self.depth_points is None else np.concatenate([self.depth_points, pts], 0)
        self.depth_points = self.downsample_points(self.depth_points)
        return self.depth_points

    @torch.no_grad()
    def create_mesh(self, decoder, map_states, voxel_size, voxels, frame_poses=None, depth_maps=None,
                    clean_mseh=False, require_color=False, offset=-10, res=8):
        centres, _, _ = _states(map_states)
        _, sdf = lattice_scores(decoder, map_states, voxel_size, res, with_rgb=False)
        verts, faces = marching_cubes_device(centres, sdf, self.voxel_size, res)
        colours = None
        if require_color:
            rows = vertex_rows(torch.as_tensor(voxels).to(verts.device), verts, self.voxel_size)
            colours = point_colours(decoder, map_states, verts, rows, voxel_size)
        normals = _vertex_normals(verts, faces)
        v_np, f_np = verts.cpu().numpy(), faces.cpu().numpy()
        if clean_mseh:
            from scipy.spatial import cKDTree
            kdtree = cKDTree(self.get_valid_points(frame_poses, depth_maps))
            hit = kdtree.query_ball_point(v_np, voxel_size * 0.5, workers=12, return_length=True) > 0
            f_np = f_np[hit[f_np.reshape(-1)].reshape(-1, 3).any(-1)]
        return Mesh(v_np + offset, f_np, None if colours is None else colours.cpu().numpy(), normals.cpu().numpy())

    @torch.no_grad()
    def marching_cubes(self, voxels, sdf):
        """mesh_util.py:149-169 API: voxel centres [n, ≥3], scores [n, res, res, res, 4] → (verts, faces) numpy."""
        sdf = torch.as_tensor(sdf)
        res = sdf.shape[1]
        dev = voxels.device if isinstance(voxels, torch.Tensor) and voxels.is_cuda else torch.device("cuda")
        c = torch.as_tensor(voxels)[:, :3].to(dev)
        v, f = marching_cubes_device(c, sdf[..., 3].to(dev), self.voxel_size, res)
        return v.cpu().numpy(), f.cpu().numpy()
