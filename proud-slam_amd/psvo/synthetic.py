"""Synthetic Replica/ScanNet-shaped scenes (no datasets exist offline).

A scene is a set of axis-aligned boxes in metres (a room shell seen from the
inside plus furniture), already carrying the reference's +10 m pose offset
(frame.py:24).  From it we derive:
  * integer surface voxels, in insertion order, for the octree builder
    (what Mapping.create_voxels_pointcloud feeds svo.insert, mapping.py:258-292);
  * pinhole rays with Replica intrinsics (replica.py:20-26; frame.py:43-58),
    gumbel top-k pixel selection (sample_util.py:4-20) and world transform as
    bundle_adjust_frames does (render_helpers.py:620-640);
  * analytic ground-truth depth / colour per ray.
Everything is seeded; nothing here is on the timed path.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch

REPLICA_K = dict(W=1200, H=680, fx=600.0, fy=600.0, cx=599.5, cy=339.5)
SCANNET_K = dict(W=628, H=468, fx=577.6, fy=578.7, cx=312.5, cy=235.4)  # depth intrinsics, crop 6


@dataclass
class Box:
    lo: np.ndarray
    hi: np.ndarray
    inside: bool = False  # True: the room shell, seen from inside


@dataclass
class Scene:
    boxes: list
    voxel_size: float = 0.2
    grid_dim: int = 256
    depth_noise: float = 0.0
    name: str = "room0"
    intrinsics: dict = field(default_factory=lambda: dict(REPLICA_K))


def room0(offset=10.0) -> Scene:
    """~8 x 6 x 3.2 m furnished living room (Replica room0 scale: ~15-20k
    octree nodes at 0.2 m voxels, under num_embeddings=20000)."""
    o = np.array([offset] * 3)
    b = [Box(o + [0.0, 0.0, 0.0], o + [8.0, 6.0, 3.2], inside=True),
         Box(o + [0.4, 0.3, 0.0], o + [2.8, 1.3, 0.85]),   # sofa
         Box(o + [0.4, 0.3, 0.85], o + [2.8, 0.5, 1.4]),   # sofa back
         Box(o + [3.0, 1.8, 0.0], o + [4.4, 2.8, 0.5]),    # coffee table
         Box(o + [7.3, 0.5, 0.0], o + [7.9, 2.9, 1.9]),    # cabinet
         Box(o + [5.2, 4.7, 0.0], o + [6.4, 5.7, 0.75]),   # side table
         Box(o + [0.2, 4.9, 0.0], o + [1.4, 5.9, 2.2]),    # shelf
         Box(o + [2.0, 5.4, 0.9], o + [4.5, 5.9, 1.0]),    # wall shelf
         Box(o + [6.0, 2.0, 0.0], o + [6.8, 2.8, 1.0]),    # armchair
         Box(o + [3.3, 3.6, 0.0], o + [3.7, 4.0, 1.6]),    # lamp
         Box(o + [2.5, 0.05, 1.2], o + [4.5, 0.15, 2.4]),  # picture frame
         Box(o + [4.6, 0.0, 2.7], o + [5.6, 6.0, 3.0])]    # ceiling beam
    return Scene(b, name="room0")


def office0(offset=10.0) -> Scene:
    o = np.array([offset] * 3)
    b = [Box(o + [0.0, 0.0, 0.0], o + [6.0, 6.5, 2.8], inside=True),
         Box(o + [0.5, 0.5, 0.0], o + [2.5, 1.5, 0.75]),
         Box(o + [3.5, 0.5, 0.0], o + [5.5, 1.5, 0.75]),
         Box(o + [0.5, 4.5, 0.0], o + [2.0, 6.2, 1.0]),
         Box(o + [4.5, 4.0, 0.0], o + [5.8, 6.3, 2.2]),
         Box(o + [2.6, 2.6, 0.0], o + [3.4, 3.4, 1.1])]
    return Scene(b, name="office0")


def scannet0000(offset=10.0) -> Scene:
    """Larger, noisier room (ScanNet scene0000_00 scale, depth noise ~1 cm)."""
    o = np.array([offset] * 3)
    b = [Box(o + [0.0, 0.0, 0.0], o + [9.0, 8.0, 3.0], inside=True),
         Box(o + [0.5, 0.5, 0.0], o + [2.5, 2.5, 0.6]),
         Box(o + [4.0, 0.4, 0.0], o + [6.5, 1.4, 0.9]),
         Box(o + [7.5, 3.0, 0.0], o + [8.8, 6.0, 2.0]),
         Box(o + [3.0, 5.0, 0.0], o + [5.0, 7.0, 0.75]),
         Box(o + [0.4, 6.0, 0.0], o + [1.5, 7.8, 1.8]),
         Box(o + [5.8, 6.2, 0.0], o + [7.0, 7.6, 1.2])]
    s = Scene(b, name="scannet0000", depth_noise=0.01)
    s.intrinsics = dict(SCANNET_K)
    return s


def multiroom(n_x=15, n_y=15, offset=10.0) -> Scene:
    """ARKit-style large scene (config E): a 15 x 15 grid of furnished rooms in
    a depth-10 tree (grid 1024) — > 1M SURFACE leaves, ~2.7M nodes, a ~170 MB
    embedding table."""
    boxes = []
    rng = np.random.default_rng(7)
    for i in range(n_x):
        for j in range(n_y):
            base = np.array([offset + 8.0 * i, offset + 7.0 * j, offset])
            boxes.append(Box(base, base + [7.5, 6.5, 3.0], inside=(i == 0 and j == 0)))
            for _ in range(4):
                lo = base + [rng.uniform(0.3, 5.5), rng.uniform(0.3, 4.5), 0.0]
                boxes.append(Box(lo, lo + [rng.uniform(0.5, 1.8), rng.uniform(0.5, 1.8), rng.uniform(0.4, 2.0)]))
    s = Scene(boxes, name="multiroom", grid_dim=1024)
    return s


def _face_points(box: Box, spacing: float):
    pts = []
    lo, hi = box.lo, box.hi
    for axis in range(3):
        a1, a2 = [a for a in range(3) if a != axis]
        u = np.arange(lo[a1], hi[a1] + 1e-9, spacing)
        v = np.arange(lo[a2], hi[a2] + 1e-9, spacing)
        uu, vv = np.meshgrid(u, v, indexing="ij")
        for c in (lo[axis], hi[axis]):
            p = np.zeros((uu.size, 3))
            p[:, axis] = c
            p[:, a1] = uu.ravel()
            p[:, a2] = vv.ravel()
            pts.append(p)
    return np.concatenate(pts, 0)


def surface_voxels(scene: Scene, spacing=None, seed=0) -> np.ndarray:
    """Integer voxel coords floor(p / voxel) of surface samples (mapping.py:264),
    de-duplicated in first-seen order (a mapping run inserts per frame; the
    octree's node numbering follows insertion order)."""
    rng = np.random.default_rng(seed)
    if spacing is None:  # 5 cm faces; half a voxel for the big multi-room scene
        spacing = 0.05 if scene.grid_dim <= 256 else scene.voxel_size * 0.5
    pts = np.concatenate([_face_points(b, spacing) for b in scene.boxes], 0)
    if scene.depth_noise > 0:
        pts = pts + rng.normal(0.0, scene.depth_noise, pts.shape)
    vox = np.floor(pts / scene.voxel_size).astype(np.int64)
    _, first = np.unique(vox, axis=0, return_index=True)
    vox = vox[np.sort(first)]
    assert vox.min() >= 0 and vox.max() < scene.grid_dim - 1, "scene must fit the grid"
    return vox.astype(np.int32)


def look_at(eye, target, up=(0.0, 0.0, 1.0)) -> np.ndarray:
    """Camera-to-world pose, OpenCV camera axes (x right, y down, z forward)."""
    eye, target, up = np.asarray(eye, float), np.asarray(target, float), np.asarray(up, float)
    z = target - eye
    z /= np.linalg.norm(z)
    x = np.cross(z, up)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    T = np.eye(4)
    T[:3, 0], T[:3, 1], T[:3, 2], T[:3, 3] = x, y, z, eye
    return T


def camera_poses(scene: Scene, n: int, seed=0) -> list:
    """Cameras at standing height inside the room shell looking at walls/furniture."""
    rng = np.random.default_rng(seed)
    room = [b for b in scene.boxes if b.inside][0]
    poses = []
    for _ in range(n):
        eye = room.lo + (room.hi - room.lo) * np.array([rng.uniform(0.3, 0.7), rng.uniform(0.3, 0.7), 0.0])
        eye[2] = room.lo[2] + rng.uniform(1.2, 1.8)
        ang = rng.uniform(0, 2 * math.pi)
        tgt = eye + np.array([math.cos(ang), math.sin(ang), rng.uniform(-0.6, -0.1)])
        poses.append(look_at(eye, tgt))
    return poses


def _ray_boxes(o, d, boxes):
    """First positive hit distance (in units of d) against the scene's boxes."""
    t_best = np.full(o.shape[0], np.inf)
    hit_box = np.full(o.shape[0], -1)
    for bi, b in enumerate(boxes):
        with np.errstate(divide="ignore", invalid="ignore"):
            inv = 1.0 / d
            t0 = (b.lo - o) * inv
            t1 = (b.hi - o) * inv
        tmin = np.nanmax(np.minimum(t0, t1), axis=1)
        tmax = np.nanmin(np.maximum(t0, t1), axis=1)
        t = tmax if b.inside else np.where(tmin > 1e-6, tmin, np.inf)
        ok = (tmax >= tmin) & (t > 1e-6) & (t < t_best)
        t_best = np.where(ok, t, t_best)
        hit_box = np.where(ok, bi, hit_box)
    return t_best, hit_box


def _ray_boxes_torch(o, d, boxes, device):
    """_ray_boxes in float64 torch on `device` (same IEEE operations, same
    result; the numpy loop takes minutes for a full frame of config E's
    1,125 boxes)."""
    o = torch.as_tensor(np.ascontiguousarray(o), dtype=torch.float64, device=device)
    d = torch.as_tensor(np.ascontiguousarray(d), dtype=torch.float64, device=device)
    inv = 1.0 / d
    t_best = torch.full((o.shape[0],), math.inf, dtype=torch.float64, device=device)
    hit_box = torch.full((o.shape[0],), -1, dtype=torch.int64, device=device)
    inf = torch.tensor(math.inf, dtype=torch.float64, device=device)
    for bi, b in enumerate(boxes):
        lo = torch.as_tensor(np.asarray(b.lo, np.float64), device=device)
        hi = torch.as_tensor(np.asarray(b.hi, np.float64), device=device)
        t0 = (lo - o) * inv
        t1 = (hi - o) * inv
        mn, mx = torch.minimum(t0, t1), torch.maximum(t0, t1)  # NaN propagates as in np.minimum / np.maximum
        tmin = torch.fmax(torch.fmax(mn[:, 0], mn[:, 1]), mn[:, 2])  # np.nanmax: NaN ignored
        tmax = torch.fmin(torch.fmin(mx[:, 0], mx[:, 1]), mx[:, 2])
        t = tmax if b.inside else torch.where(tmin > 1e-6, tmin, inf)
        ok = (tmax >= tmin) & (t > 1e-6) & (t < t_best)
        t_best = torch.where(ok, t, t_best)
        hit_box = torch.where(ok, torch.full_like(hit_box, bi), hit_box)
    return t_best.cpu().numpy(), hit_box.cpu().numpy()


def gumbel_topk_pixels(H, W, n, generator):
    """sample_util.py:4-20 on a uniform mask: n distinct pixel ids."""
    logp = torch.full((H * W,), math.log(1.0 / (H * W) + 1e-7))
    u = torch.rand(H * W, generator=generator)
    g = -torch.log(-torch.log(u + 1e-7) + 1e-7)
    return torch.topk(logp + g, n).indices.sort().values


def rays_for_frames(scene: Scene, poses, n_per_frame: int, seed=0):
    """World-space ray batch + analytic GT, as bundle_adjust_frames builds it."""
    K = scene.intrinsics
    g = torch.Generator().manual_seed(seed)
    rng = np.random.default_rng(seed + 1)
    R_o, R_d, GT_d, GT_c = [], [], [], []
    for T in poses:
        pix = gumbel_topk_pixels(K["H"], K["W"], n_per_frame, g).numpy()
        u = (pix % K["W"]).astype(np.float64)
        v = (pix // K["W"]).astype(np.float64)
        d_cam = np.stack([(u - K["cx"]) / K["fx"], (v - K["cy"]) / K["fy"], np.ones_like(u)], -1)
        Rm = T[:3, :3].astype(np.float32)
        d_world = (d_cam.astype(np.float32) @ Rm.T).astype(np.float32)
        o_world = np.broadcast_to(T[:3, 3].astype(np.float32), d_world.shape).copy()
        t, hb = _ray_boxes(o_world.astype(np.float64), d_world.astype(np.float64), scene.boxes)
        t = np.where(np.isfinite(t), t, 0.0)
        if scene.depth_noise > 0:
            t = t + rng.normal(0, scene.depth_noise, t.shape)
        p = o_world + d_world * t[:, None]
        col = 0.5 + 0.5 * np.sin(np.stack([1.3 * p[:, 0] + 0.7 * hb, 1.7 * p[:, 1], 2.1 * p[:, 2] + 0.3 * hb], -1))
        R_o.append(o_world)
        R_d.append(d_world)
        GT_d.append(t.astype(np.float32))
        GT_c.append(col.astype(np.float32))
    cat = lambda xs: torch.from_numpy(np.concatenate(xs, 0))
    return cat(R_o).unsqueeze(0), cat(R_d).unsqueeze(0), cat(GT_c).unsqueeze(0), cat(GT_d).unsqueeze(0)


class SyntheticFrame:
    """An RGBDFrame stand-in (frame.py:10-96 fields track_frame reads): camera
    ray directions rays_d [H, W, 3] (frame.py:48-58), analytic rgb / depth
    [H, W] of `scene` seen from pose T, and sample_rays(n) → sample_mask
    (gumbel top-k over the pixels, sample_util.py:4-20).  `scale` shrinks the
    Replica intrinsics to keep the frame small."""

    def __init__(self, scene: Scene, T, scale=0.25, seed=0, device="cuda"):
        K = scene.intrinsics
        H, W = int(K["H"] * scale), int(K["W"] * scale)
        fx, fy, cx, cy = K["fx"] * scale, K["fy"] * scale, K["cx"] * scale, K["cy"] * scale
        iy, ix = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
        d_cam = np.stack([(ix - cx) / fx, (iy - cy) / fy, np.ones_like(ix, dtype=np.float64)], -1).astype(np.float32)
        Rm = np.asarray(T, np.float64)[:3, :3]
        d_world = d_cam.reshape(-1, 3).astype(np.float64) @ Rm.T
        o_world = np.broadcast_to(np.asarray(T, np.float64)[:3, 3], d_world.shape)
        if torch.device(device).type == "cuda":
            t, hb = _ray_boxes_torch(o_world, d_world, scene.boxes, device)
        else:
            t, hb = _ray_boxes(o_world, d_world, scene.boxes)
        t = np.where(np.isfinite(t), t, 0.0)
        p = o_world + d_world * t[:, None]
        col = 0.5 + 0.5 * np.sin(np.stack([1.3 * p[:, 0] + 0.7 * hb, 1.7 * p[:, 1], 2.1 * p[:, 2] + 0.3 * hb], -1))
        self.h, self.w = H, W
        self.rays_d = torch.from_numpy(d_cam).to(device)
        self.rgb = torch.from_numpy(col.reshape(H, W, 3).astype(np.float32)).to(device)
        self.depth = torch.from_numpy(t.reshape(H, W).astype(np.float32)).to(device)
        self.gen = torch.Generator().manual_seed(seed)  # CPU: seeds for the device sampler, no sync
        self.sample_mask = None

    # sample_rays below is the reference's frame.sample_rays (uniform gumbel
    # top-k over all pixels): bundle_adjust_frames may sample these frames
    # together (psvo.sample_util.sample_frames)
    uniform_pixel_sampling = True

    def sample_rays(self, n):
        """frame.py:83-85: sample_rays(ones_like(depth)[None], n)[0] on the
        device (psvo.sample_util, gumbel top-k over a uniform distribution)."""
        from . import sample_util
        mask = torch.empty(self.h, self.w, dtype=torch.bool, device=self.depth.device)
        seed = int(torch.randint(0, 2 ** 62, (1,), generator=self.gen).item())
        idx = sample_util.sample_pixels(1, self.h * self.w, int(n), self.depth.device, seed=seed,
                                        frames=[(None, None, None, mask)])
        self.sample_mask = mask
        self.sample_idx = idx[0]  # the mask's pixels in row-major order (no host sync to gather them)


@dataclass
class Workload:
    scene: Scene
    voxels: np.ndarray
    poses: list
    rays_o: torch.Tensor
    rays_d: torch.Tensor
    rgb: torch.Tensor
    depth: torch.Tensor


def make_workload(kind="room0", n_frames=4, rays_per_frame=1024, seed=0) -> Workload:
    scene = {"room0": room0, "office0": office0, "scannet0000": scannet0000, "multiroom": multiroom}[kind]()
    vox = surface_voxels(scene, seed=seed)
    poses = camera_poses(scene, n_frames, seed=seed)
    ro, rd, rgb, depth = rays_for_frames(scene, poses, rays_per_frame, seed=seed)
    return Workload(scene, vox, poses, ro, rd, rgb, depth)
