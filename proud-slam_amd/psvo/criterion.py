"""Criterion with the reference's interface and loss (src/criterion.py:5-116).

Same constructor (args.criteria / args.data_specs), same forward signature
and the same padded-mean semantics over [R_hit, S_max].  loss_dict values
are converted to Python floats lazily (on first access) instead of five
`.item()` host syncs per call (criterion.py:39-67); bundle_adjust_frames and
track_frame discard the dict.
"""
from __future__ import annotations

import torch
import torch.nn as nn


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
                weight_depth_loss=False):
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
