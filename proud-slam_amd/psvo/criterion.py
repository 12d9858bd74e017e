"""Criterion with the reference's interface and loss (src/criterion.py:5-116).

Same constructor (args.criteria / args.data_specs), same forward signature
and the same padded-mean semantics over [R_hit, S_max].  loss_dict values
are converted to Python floats lazily (on first access) instead of five
`.item()` host syncs per call (criterion.py:39-67); bundle_adjust_frames and
track_frame discard the dict.

When `outputs` comes from psvo.render_helpers.render_rays (it carries the
hit-ray order `rank_ray`), the loss runs as libpsvo's criterion kernels
(csrc/criterion.hip): no boolean indexing, so no host syncs, and a
deterministic reduction.  weight_depth_loss (tracking's median filter) and
foreign output dicts use the PyTorch formulation below.
"""
from __future__ import annotations

import torch
import torch.nn as nn
from torch.autograd import Function

from . import _lib as L

CRIT_OUT_WORDS = 16
_USE_COLOR, _USE_DEPTH, _USE_SDF = 1, 2, 4


class CriterionLoss(Function):
    """(colour, depth, sdf) of the hit rays → scalar loss; the parts and the
    fs/sdf balance weights (f32[16], PSVO_CRIT_* words) are appended to `sink`.
    `reduce_sums` (optional) is applied to the f64[8] sums in place before the
    loss is formed — the data-parallel hook (all-reduce) of SURVEY §8e."""

    @staticmethod
    def forward(ctx, color, depth, sdf, z_vals, gt_rgb, gt_depth, rank_ray, cfg, reduce_sums=None, sink=None):
        tr, max_depth, rgb_w, depth_w, fs_w, sdf_w, flags = cfg
        r_hit, s_max = z_vals.shape
        dev = z_vals.device
        n_hit, s_cols, pad_extra = r_hit, s_max, 0
        if reduce_sums is not None:
            n_hit, s_cols = reduce_sums.global_shape(r_hit, s_max)
            pad_extra = s_cols - s_max
        ws = torch.empty((int(L.lib().psvo_criterion_workspace_floats(r_hit)),), dtype=torch.float32, device=dev)
        sums = torch.empty((8,), dtype=torch.float64, device=dev)
        out = torch.empty((CRIT_OUT_WORDS,), dtype=torch.float32, device=dev)
        stream = L.stream_of(dev)
        L.call("psvo_criterion_sums", stream, r_hit, s_max, pad_extra, tr, max_depth, L.ptr(rank_ray), L.ptr(gt_rgb),
               L.ptr(gt_depth), L.ptr(color), L.ptr(depth), L.ptr(sdf), L.ptr(z_vals), L.ptr(ws), L.ptr(sums))
        if reduce_sums is not None:
            reduce_sums(sums)
        L.call("psvo_criterion_finalize", stream, L.ptr(sums), n_hit, s_cols, rgb_w, depth_w, fs_w, sdf_w, tr, flags,
               L.ptr(out))
        ctx.save_for_backward(color, depth, sdf, z_vals, gt_rgb, gt_depth, rank_ray, out)
        ctx.cfg = cfg
        if sink is not None:
            sink.append(out)
        return out[0]

    @staticmethod
    def backward(ctx, g_loss):
        color, depth, sdf, z_vals, gt_rgb, gt_depth, rank_ray, out = ctx.saved_tensors
        tr, max_depth = ctx.cfg[0], ctx.cfg[1]
        r_hit, s_max = z_vals.shape
        dev = z_vals.device
        g = g_loss.detach().float().contiguous()
        g_color = torch.empty((r_hit, 3), dtype=torch.float32, device=dev)
        g_depth = torch.empty((r_hit,), dtype=torch.float32, device=dev)
        g_sdf = torch.empty((r_hit, s_max), dtype=torch.float32, device=dev)
        L.call("psvo_criterion_bwd", L.stream_of(dev), r_hit, s_max, tr, max_depth, L.ptr(rank_ray), L.ptr(gt_rgb),
               L.ptr(gt_depth), L.ptr(color), L.ptr(depth), L.ptr(sdf), L.ptr(z_vals), L.ptr(out), L.ptr(g),
               L.ptr(g_color), L.ptr(g_depth), L.ptr(g_sdf))
        return g_color, g_depth, g_sdf, None, None, None, None, None, None, None


class LazyLossDict(dict):
    """dict whose tensor values become floats when read."""

    def __getitem__(self, k):
        v = super().__getitem__(k)
        if isinstance(v, torch.Tensor):
            v = float(v.detach().item())
            super().__setitem__(k, v)
        return v

    def items(self):
        return [(k, self[k]) for k in self.keys()]

    def values(self):
        return [self[k] for k in self.keys()]


class Criterion(nn.Module):
    def __init__(self, args) -> None:
        super().__init__()
        self.args = args
        self.rgb_weight = args.criteria["rgb_weight"]
        self.depth_weight = args.criteria["depth_weight"]
        self.sdf_weight = args.criteria["sdf_weight"]
        self.fs_weight = args.criteria["fs_weight"]
        self.truncation = args.criteria["sdf_truncation"]
        self.max_dpeth = args.data_specs["max_depth"]

    def forward(self, outputs, obs, use_color_loss=True, use_depth_loss=True, compute_sdf_loss=True,
                weight_depth_loss=False, reduce_sums=None):
        if outputs.get("rank_ray") is not None and not weight_depth_loss and outputs["z_vals"].is_cuda:
            return self._forward_fused(outputs, obs, use_color_loss, use_depth_loss, compute_sdf_loss, reduce_sums)
        img, depth = obs
        loss = 0
        loss_dict = LazyLossDict()
        pred_depth = outputs["depth"]
        pred_color = outputs["color"]
        pred_sdf = outputs["sdf"]
        z_vals = outputs["z_vals"]
        ray_mask = outputs["ray_mask"]
        weights = outputs["weights"]
        gt_depth = depth[ray_mask]
        gt_color = img[ray_mask]
        if use_color_loss:
            color_loss = (gt_color - pred_color).abs().mean()
            loss += self.rgb_weight * color_loss
            loss_dict["color_loss"] = color_loss
        if use_depth_loss:
            valid_depth = (gt_depth > 0.01) & (gt_depth < self.max_dpeth)
            depth_loss = (gt_depth - pred_depth).abs()
            if weight_depth_loss:
                depth_var = torch.sum(weights * ((pred_depth.unsqueeze(-1) - z_vals) ** 2), -1)
                tmp = depth_loss / torch.sqrt(depth_var + 1e-10)
                valid_depth = (tmp < 10 * tmp.median()) & valid_depth
            depth_loss = depth_loss[valid_depth].mean()
            loss += self.depth_weight * depth_loss
            loss_dict["depth_loss"] = depth_loss
        if compute_sdf_loss:
            fs_loss, sdf_loss = self.get_sdf_loss(z_vals, gt_depth, pred_sdf, truncation=self.truncation,
                                                  loss_type="l2")
            loss += self.fs_weight * fs_loss
            loss += self.sdf_weight * sdf_loss
            loss_dict["fs_loss"] = fs_loss
            loss_dict["sdf_loss"] = sdf_loss
        loss_dict["loss"] = loss.detach() if isinstance(loss, torch.Tensor) else loss
        return loss, loss_dict

    def _forward_fused(self, outputs, obs, use_color, use_depth, use_sdf, reduce_sums):
        img, depth = obs
        flags = (_USE_COLOR if use_color else 0) | (_USE_DEPTH if use_depth else 0) | (_USE_SDF if use_sdf else 0)
        cfg = (float(self.truncation), float(self.max_dpeth), float(self.rgb_weight), float(self.depth_weight),
               float(self.fs_weight), float(self.sdf_weight), flags)
        dev = outputs["z_vals"].device
        gt_rgb = img.reshape(-1, 3).to(device=dev, dtype=torch.float32).contiguous()
        gt_depth = depth.reshape(-1).to(device=dev, dtype=torch.float32).contiguous()
        f = lambda t: t.float().contiguous()
        sink = []
        loss = CriterionLoss.apply(f(outputs["color"]), f(outputs["depth"]), f(outputs["sdf"]), f(outputs["z_vals"]),
                                   gt_rgb, gt_depth, outputs["rank_ray"], cfg, reduce_sums, sink)
        out = sink[0]
        parts = LazyLossDict()
        if use_color:
            parts["color_loss"] = out[1]
        if use_depth:
            parts["depth_loss"] = out[2]
        if use_sdf:
            parts["fs_loss"] = out[3]
            parts["sdf_loss"] = out[4]
        parts["loss"] = loss.detach()
        return loss, parts

    def compute_loss(self, x, y, mask=None, loss_type="l2"):
        if mask is None:
            mask = torch.ones_like(x).bool()
        if loss_type == "l1":
            return torch.mean(torch.abs(x - y)[mask])
        return torch.mean(torch.square(x - y)[mask])

    def get_masks(self, z_vals, depth, epsilon):
        front_mask = (z_vals < (depth - epsilon)).float()
        back_mask = (z_vals > (depth + epsilon)).float()
        depth_mask = ((depth > 0.0) & (depth < self.max_dpeth)).float()
        sdf_mask = (1.0 - front_mask) * (1.0 - back_mask) * depth_mask
        num_fs_samples = torch.count_nonzero(front_mask).float()
        num_sdf_samples = torch.count_nonzero(sdf_mask).float()
        num_samples = num_sdf_samples + num_fs_samples
        fs_weight = 1.0 - num_fs_samples / num_samples
        sdf_weight = 1.0 - num_sdf_samples / num_samples
        return front_mask, sdf_mask, fs_weight, sdf_weight

    def get_sdf_loss(self, z_vals, depth, predicted_sdf, truncation, loss_type="l2"):
        d = depth.unsqueeze(-1).expand(*z_vals.shape)
        front_mask, sdf_mask, fs_weight, sdf_weight = self.get_masks(z_vals, d, truncation)
        fs_loss = torch.mean(torch.square(predicted_sdf * front_mask - front_mask)) * fs_weight
        sdf_loss = torch.mean(torch.square((z_vals + predicted_sdf * truncation) * sdf_mask - d * sdf_mask)) * sdf_weight
        return fs_loss, sdf_loss
