"""src/utils/sample_util.py on the device (csrc/pixels.hip).

`sample_rays(mask, num_samples)` is the reference's drop-in (sample_util.py:
12-20): gumbel top-k sampling without replacement of `num_samples` pixels per
frame, probabilities ∝ mask (one sum over the whole [B, H, W] mask), as a
bool mask.  `sample_frames(frames, n)` is what bundle_adjust_frames does per
iteration with it (render_helpers.py:620-633: frame.sample_rays(N) on every
keyframe, then rays_d / rgb / depth gathered at the mask) for all keyframes in
one native call: the picked pixels' rows land in one concatenated batch, in
the order torch.cat([frame.rays_d[frame.sample_mask], ...]) gives.

The uniforms the gumbel noise is drawn from come from a counter-based
generator keyed by `seed` (drawn from torch's CPU generator when not given:
no device sync); `u=` injects them (parity tests against the reference's own
torch.rand_like draws, tests/golden/P_pixels.npz).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib as L

_PIXEL_FRAME = None


def _frame_struct():
    global _PIXEL_FRAME
    if _PIXEL_FRAME is None:
        class PixelFrame(ctypes.Structure):  # include/psvo.h psvo_pixel_frame
            _fields_ = [("dirs", ctypes.c_void_p), ("rgb", ctypes.c_void_p), ("depth", ctypes.c_void_p),
                        ("mask", ctypes.c_void_p)]
        _PIXEL_FRAME = PixelFrame
    return _PIXEL_FRAME


def _seed(seed):
    return int(torch.randint(0, 2 ** 62, (1,)).item()) if seed is None else int(seed) & (2 ** 64 - 1)


def _workspace(n_frames, n_pix, device):
    n = L.lib().psvo_sample_pixels_workspace_ints(n_frames, n_pix)
    return torch.empty(int(n), dtype=torch.int32, device=device)


def sample_pixels(n_frames, n_pix, k, device, weights=None, joint_sum=False, u=None, seed=None, frames=None,
                  out_dirs=None, out_rgb=None, out_depth=None):
    """psvo_sample_pixels: ascending picked pixel indices i64 [n_frames, k];
    `frames` — per-frame (dirs, rgb, depth, mask) tensors or None, gathered
    into out_* (see include/psvo.h)."""
    if not 1 <= k <= n_pix:
        raise ValueError(f"sample_pixels: cannot take {k} of {n_pix} pixels")
    if weights is not None:
        L.require_device_tensor(weights, "weights", torch.float32)
        if weights.numel() != n_frames * n_pix:
            raise ValueError("sample_pixels: weights must hold n_frames x n_pix values")
    if u is not None:
        u = u.to(device=device, dtype=torch.float32).contiguous()
        if u.numel() != n_frames * n_pix:
            raise ValueError("sample_pixels: u must hold n_frames x n_pix values")
    idx = torch.empty(n_frames, k, dtype=torch.int64, device=device)
    PF = _frame_struct()
    arr = (PF * n_frames)()
    keep = []
    if frames is not None:
        for f, (d, c, z, m) in enumerate(frames):
            for t in (d, c, z, m):
                if t is not None:
                    if not (t.is_cuda and t.is_contiguous()):
                        raise ValueError("sample_pixels: frame tensors must be contiguous device tensors")
                    keep.append(t)
            arr[f].dirs = d.data_ptr() if d is not None else None
            arr[f].rgb = c.data_ptr() if c is not None else None
            arr[f].depth = z.data_ptr() if z is not None else None
            arr[f].mask = m.data_ptr() if m is not None else None
    ws = _workspace(n_frames, n_pix, device)
    ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    rc = L.lib().psvo_sample_pixels(L.stream_of(device), n_frames, n_pix, k, ptr(weights), 1 if joint_sum else 0,
                                    ptr(u), _seed(seed), ctypes.cast(arr, ctypes.c_void_p), ptr(ws), ptr(idx),
                                    ptr(out_dirs), ptr(out_rgb), ptr(out_depth))
    if rc != 0:
        raise L.PsvoError(f"psvo_sample_pixels failed ({rc}): {L.lib().psvo_last_error().decode(errors='replace')}")
    return idx


def sample_rays(mask, num_samples, u=None, seed=None):
    """sample_util.sample_rays (sample_util.py:12-20): bool [B, H, W] with
    num_samples picked pixels per frame, probabilities ∝ mask."""
    if mask.dim() != 3:
        raise ValueError("sample_rays: mask must be [B, H, W]")
    B, H, W = mask.shape
    w = mask.reshape(B, H * W).to(torch.float32).contiguous()
    out = torch.empty(B, H, W, dtype=torch.bool, device=mask.device)
    frames = [(None, None, None, out[b]) for b in range(B)]
    sample_pixels(B, H * W, int(num_samples), mask.device, weights=w, joint_sum=True, u=u, seed=seed,
                  frames=frames)
    return out


def sample_frames(frames, n, seed=None, u=None, out=None):
    """frame.sample_rays(n) (frame.py:83-85: uniform over the frame's
    pixels) on every frame, plus the gathers of bundle_adjust_frames
    (render_helpers.py:625-633): sets each frame's sample_mask [H, W] and
    sample_idx [n] and returns (dirs [F·n, 3], rgb [F·n, 3], depth [F·n]) in
    torch.cat([frame.rays_d[frame.sample_mask], ...]) order (into `out` when
    given)."""
    frames = list(frames)
    F = len(frames)
    f0 = frames[0]
    dev = f0.depth.device
    H, W = f0.depth.shape[-2:]
    srcs = []
    for fr in frames:
        if tuple(fr.depth.shape[-2:]) != (H, W):
            raise ValueError("sample_frames: frames must share one resolution")
        for t in (fr.rays_d, fr.rgb, fr.depth):
            if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.device == dev):
                raise ValueError("sample_frames: rays_d / rgb / depth must be contiguous f32 on one device")
        m = torch.empty(H, W, dtype=torch.bool, device=dev)
        srcs.append((fr.rays_d, fr.rgb, fr.depth, m))
    if out is not None:  # the caller's (dirs, rgb, depth) buffers
        dirs, rgb, depth = out
        if not (tuple(dirs.shape) == (F * n, 3) and tuple(rgb.shape) == (F * n, 3) and tuple(depth.shape) == (F * n,)
                and all(t.dtype == torch.float32 and t.is_contiguous() and t.device == dev for t in out)):
            raise ValueError("sample_frames: out must be contiguous f32 [F*n, 3], [F*n, 3], [F*n] on the frames' device")
    else:
        dirs = torch.empty(F * n, 3, dtype=torch.float32, device=dev)
        rgb = torch.empty(F * n, 3, dtype=torch.float32, device=dev)
        depth = torch.empty(F * n, dtype=torch.float32, device=dev)
    idx = sample_pixels(F, H * W, int(n), dev, u=u, seed=seed, frames=srcs, out_dirs=dirs, out_rgb=rgb,
                        out_depth=depth)
    for f, fr in enumerate(frames):
        fr.sample_mask = srcs[f][3]
        fr.sample_idx = idx[f]
    return dirs, rgb, depth
