"""Optimisable SE(3) pose (the pose type track_frame optimises, se3pose.py:8-98):
parameters `data` = [t (3) | w (3)], w an axis-angle rotation,
R = I + A(θ)[w]× + B(θ)[w]×², A = sin θ/θ, B = (1 − cos θ)/θ² as 10th-order
Taylor series (smooth at θ = 0, so gradients through R are well defined).
from_matrix takes the log map the same way (θ from the trace, clamped away
from ±1).  Provided so tracking runs and tests are self-contained; the
drop-in track_frame takes the caller's own pose object unchanged."""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn


def _series(x, first_denom, step, nth=10):
    """Σ_{i≤nth} (−1)^i x^{2i} / d_i with d_0 = first_denom, d_i = d_{i−1}·step(i),
    by Horner's rule in y = x² (coefficients folded on the host: nth
    multiply-adds on the device instead of a power, divide and add per term)."""
    coef = []
    denom = float(first_denom)
    for i in range(nth + 1):
        if i > 0:
            denom *= step(i)
        coef.append((-1.0) ** i / denom)
    y = x * x
    out = torch.full_like(x, coef[-1])
    for c in reversed(coef[:-1]):
        out = torch.addcmul(torch.full_like(x, c), out, y)
    return out


def taylor_sin_over_x(x, nth=10):        # sin x / x
    return _series(x, 1.0, lambda i: (2 * i) * (2 * i + 1), nth)


def taylor_one_minus_cos_over_x2(x, nth=10):  # (1 − cos x) / x²
    return _series(x, 2.0, lambda i: (2 * i + 1) * (2 * i + 2), nth)


def skew(w):
    w0, w1, w2 = w.unbind(dim=-1)
    z = torch.zeros_like(w0)
    return torch.stack([torch.stack([z, -w2, w1], -1), torch.stack([w2, z, -w0], -1),
                        torch.stack([-w1, w0, z], -1)], -2)


class OptimizablePose(nn.Module):
    def __init__(self, init_pose):
        super().__init__()
        self.data = nn.Parameter(torch.as_tensor(init_pose, dtype=torch.float32).clone())

    def rotation(self):
        w = self.data[3:]
        wx = skew(w)
        theta = w.norm(dim=-1)[..., None, None]
        eye = torch.eye(3, device=w.device, dtype=torch.float32)
        return eye + taylor_sin_over_x(theta) * wx + taylor_one_minus_cos_over_x2(theta) * (wx @ wx)

    def translation(self):
        return self.data[:3]

    def matrix(self):
        rt = torch.eye(4, device=self.data.device)
        rt[:3, :3] = self.rotation()
        rt[:3, 3] = self.translation()
        return rt

    @staticmethod
    def log_rotation(r, eps=1e-7):
        trace = r[..., 0, 0] + r[..., 1, 1] + r[..., 2, 2]
        theta = ((trace - 1) / 2).clamp(-1 + eps, 1 - eps).acos()[..., None, None] % math.pi
        ln_r = (r - r.transpose(-2, -1)) / (2 * taylor_sin_over_x(theta) + 1e-8)
        return torch.stack([ln_r[..., 2, 1], ln_r[..., 0, 2], ln_r[..., 1, 0]], -1)

    @classmethod
    def from_matrix(cls, rt):
        rt = torch.as_tensor(np.asarray(rt) if not isinstance(rt, torch.Tensor) else rt, dtype=torch.float32)
        return cls(torch.cat([rt[:3, 3], cls.log_rotation(rt[:3, :3])], -1))
