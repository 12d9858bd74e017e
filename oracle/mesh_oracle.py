"""ORACLE — TEST INFRASTRUCTURE ONLY (mesh extraction).

CPU restatement of MeshExtractor.create_mesh (mesh_util.py:80-147) on the
SURFACE voxels Mapping.extract_mesh selects (mapping.py:420-440):
  get_scores      render_helpers.py:243-294  (lattice → features → decoder)
  eval_points     render_helpers.py:297-328
  marching_cubes  mesh_util.py:149-169       (per voxel, skipped without a sign change)
  vertex colours  mesh_util.py:108-133       (voxel of `vertex // voxel`, brute force)
get_scores / eval_points are pinned by tests/golden/M_mesh_A.npz (the
reference's own functions run in the container).  Marching cubes itself is
skimage.measure.marching_cubes in the reference — a third-party dependency
(requirements.txt:5, unpinned) that is not installed here, so the
triangulation is this module's table rule (the same rule csrc/mesh.hip
builds its table from, coded independently below) and is "parity unpinned"
against skimage; its vertex set (one vertex per sign-changing lattice edge,
linear interpolation) is the construction skimage uses too.
Only tests/ may import this module.
"""
from __future__ import annotations

import numpy as np
import torch

from . import oracle as O


# ------------------------------------------------------------ get_scores
def lattice(res):
    """torch.linspace(−.5, .5, res) meshgrid 'ij' → [res³, 3] (render_helpers.py:255-259)."""
    x = torch.linspace(-0.5, 0.5, res)
    xx, yy, zz = torch.meshgrid(x, x, x, indexing="ij")
    return torch.stack([xx, yy, zz], -1).float().reshape(-1, 3)


def get_scores(params, centres, features, embeddings, voxel_size, res=8):
    """[n, res, res, res, 4] = [rgb | sdf] (render_helpers.py:243-294)."""
    c = torch.as_tensor(centres, dtype=torch.float32)
    xyz = (lattice(res) * voxel_size).reshape(1, -1, 3) + c.unsqueeze(1)
    idx = torch.arange(c.shape[0])[:, None].expand(-1, res ** 3).reshape(-1)
    feats = O.interp_features(xyz.reshape(-1, 3), idx, c, torch.as_tensor(features),
                              torch.as_tensor(embeddings, dtype=torch.float32), voxel_size)
    rgb, sdf = O.decoder_forward(params, feats)
    return torch.cat([rgb, sdf[:, None]], -1).view(-1, res, res, res, 4)


def eval_points(params, centres, features, embeddings, points, idx, voxel_size):
    """rgb [n, 3] (render_helpers.py:297-328)."""
    feats = O.interp_features(torch.as_tensor(points, dtype=torch.float32), torch.as_tensor(idx),
                              torch.as_tensor(centres, dtype=torch.float32), torch.as_tensor(features),
                              torch.as_tensor(embeddings, dtype=torch.float32), voxel_size)
    rgb, _ = O.decoder_forward(params, feats)
    return rgb


# ------------------------------------------------------------ case table
# corner b = (b & 1, b >> 1 & 1, b >> 2 & 1) = (x, y, z); edge e = axis·4 +
# o1 + 2·o2 with (o1, o2) the corner offsets on the other two axes.
def _edge(c0, c1):
    axis = {1: 0, 2: 1, 4: 2}[c0 ^ c1]
    others = [a for a in range(3) if a != axis]
    return axis * 4 + ((c0 >> others[0]) & 1) + 2 * ((c0 >> others[1]) & 1)


def edge_endpoints():
    out = []
    for e in range(12):
        axis = e // 4
        others = [a for a in range(3) if a != axis]
        c0 = ((e & 1) << others[0]) | (((e >> 1) & 1) << others[1])
        out.append((c0, c0 | (1 << axis), axis))
    return out


def _face_walks():
    """Each cube face's corners, counter-clockwise seen from outside."""
    walks = []
    for axis in range(3):
        u, v = (axis + 1) % 3, (axis + 2) % 3  # e_u × e_v = e_axis
        square = [(0, 0), (1, 0), (1, 1), (0, 1)]
        for side in (0, 1):
            order = square if side else [square[0], square[3], square[2], square[1]]
            walks.append([(side << axis) | (a << u) | (b << v) for a, b in order])
    return walks


def _same_face(e1, e2):
    for c in _face_walks():
        f = {_edge(c[i], c[(i + 1) % 4]) for i in range(4)}
        if e1 in f and e2 in f:
            return True
    return False


def mc_table():
    """case → list of triangles (edge triples): per face, the iso-segment runs
    from the crossing where the CCW walk leaves the + corners to the one where
    it enters them (an ambiguous face isolates each + corner); segments chain
    into loops (listed from their lowest edge), each fanned from its first
    vertex whose diagonals stay off the cube faces."""
    walks = _face_walks()
    table = []
    for case in range(256):
        nxt = {}
        for c in walks:
            pos = [(case >> ci) & 1 for ci in c]
            if sum(pos) in (0, 4):
                continue
            ed = [_edge(c[i], c[(i + 1) % 4]) for i in range(4)]
            if sum(pos) == 2 and pos[0] == pos[2]:
                for i in range(4):
                    if pos[i]:
                        nxt[ed[i]] = ed[(i - 1) % 4]
            else:
                first = next(i for i in range(4) if pos[i] and not pos[(i - 1) % 4])
                last = next(i for i in range(4) if pos[i] and not pos[(i + 1) % 4])
                nxt[ed[last]] = ed[(first - 1) % 4]
        seen, tris = set(), []
        for s in sorted(nxt):
            if s in seen:
                continue
            loop, e = [], s
            while e not in seen:
                seen.add(e)
                loop.append(e)
                e = nxt[e]
            n = len(loop)
            # fan apex: the first loop vertex none of whose diagonals joins two
            # edges of one cube face (such a diagonal would lie in the face the
            # neighbouring cube triangulates too)
            a = next(a for a in range(n) if all(not _same_face(loop[a], loop[(a + i) % n]) for i in range(2, n - 1)))
            tris += [(loop[a], loop[(a + i) % n], loop[(a + i + 1) % n]) for i in range(1, n - 1)]
        table.append(tris)
    return table


# ------------------------------------------------------------ marching cubes
def marching_cubes(centres, sdf, voxel_size):
    """Per-voxel marching cubes over sdf [n, res, res, res] (mesh_util.py:149-169):
    vertices one per sign-changing lattice edge in slot order
    ((i·res + j)·res + k)·3 + axis, at t = v0/(v0 − v1), mapped to
    ((g·spacing) − 0.5)·voxel + centre; faces cube-major (i, j, k), table
    order within a cube; voxels without a sign change are skipped.
    Returns (verts f32 [V, 3], faces i32 [F, 3])."""
    table = mc_table()
    ends = edge_endpoints()
    sdf = np.asarray(sdf, np.float32)
    centres = np.asarray(centres, np.float32)
    n, res = sdf.shape[0], sdf.shape[1]
    r1 = res - 1
    sp = np.float32(1.0 / r1)
    vs = np.float32(voxel_size)
    all_v, all_f, nv = [], [], 0
    for v in range(n):
        s = sdf[v]
        if s.min() > 0 or s.max() < 0:
            continue
        pos = s > 0
        vid = -np.ones((res, res, res, 3), np.int64)
        verts = []
        # slot order: grid point (i, j, k) major, axis minor
        cross = np.zeros((res, res, res, 3), bool)
        cross[:-1, :, :, 0] = pos[:-1] != pos[1:]
        cross[:, :-1, :, 1] = pos[:, :-1] != pos[:, 1:]
        cross[:, :, :-1, 2] = pos[:, :, :-1] != pos[:, :, 1:]
        slots = np.argwhere(cross)  # lexicographic (i, j, k, axis) = slot order
        for q, (i, j, k, a) in enumerate(slots):
            vid[i, j, k, a] = q
            o = [i, j, k]
            o2 = list(o)
            o2[a] += 1
            v0, v1 = s[i, j, k], s[tuple(o2)]
            t = np.float32(v0 / np.float32(v0 - v1))
            g = [np.float32(np.float32(o[d]) + t) * sp if d == a else np.float32(o[d]) * sp for d in range(3)]
            verts.append([np.float32(np.float32(g[d] - np.float32(0.5)) * vs) + centres[v, d] for d in range(3)])
        if not verts:
            continue
        faces = []
        cases = np.zeros((r1, r1, r1), np.int64)
        for b in range(8):
            dx, dy, dz = b & 1, (b >> 1) & 1, (b >> 2) & 1
            cases |= pos[dx:dx + r1, dy:dy + r1, dz:dz + r1].astype(np.int64) << b
        for i, j, k in np.argwhere((cases != 0) & (cases != 255)):  # lexicographic cube order
            for tri in table[int(cases[i, j, k])]:
                f = []
                for e in tri:
                    c0, _, a = ends[e]
                    f.append(nv + vid[i + (c0 & 1), j + ((c0 >> 1) & 1), k + ((c0 >> 2) & 1), a])
                faces.append(f)
        all_v.append(np.asarray(verts, np.float32))
        if faces:
            all_f.append(np.asarray(faces, np.int64))
        nv += len(verts)
    if not all_v:
        return np.zeros((0, 3), np.float32), np.zeros((0, 3), np.int32)
    return (np.concatenate(all_v).astype(np.float32),
            (np.concatenate(all_f) if all_f else np.zeros((0, 3), np.int64)).astype(np.int32))


def vertex_voxel_rows(verts, voxels, voxel_size):
    """mesh_util.py:112-125: row of the voxel whose min corner equals
    verts // voxel (torch floor division), −1 if none."""
    vp = torch.floor_divide(torch.as_tensor(verts, dtype=torch.float32), voxel_size)
    vx = torch.as_tensor(voxels, dtype=torch.float32)[:, :3]
    eq = (vx.unsqueeze(0) == vp.unsqueeze(1)).all(-1)  # [V, N]
    has = eq.any(-1)
    first = torch.where(has, eq.float().argmax(-1), torch.full_like(has, -1, dtype=torch.long))
    return first.numpy()
