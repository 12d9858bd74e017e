"""NRGBD decoder with the reference's module structure (src/variations/nrgbd.py:80-146),
so state_dicts load both ways.  Every shipped config uses depth 2,
embedder 'none', skips []:

  h = ReLU(L0(x)); h = ReLU(L1(h)); o = sdf_out(h) = [sdf | f(128)]
  rgb = σ(L5(ReLU(L4([f, x]))))

On a GPU forward() runs the fused fp32-MFMA kernels of libpsvo through
DecoderMLP: width 128 (every Replica config, csrc/mlp.hip) and width 256
(ScanNet / ARKit, configs/scannet/scannet.yaml:17, csrc/mlp256.hip).
get_values() (mesh extraction, no grad) uses the PyTorch layers.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.autograd import Function

from . import _lib as L


class DecoderMLP(Function):
    """(feat[M,16], W1,b1,...,W5,b5) → (sdf[M], rgb[M,3]) on libpsvo's fused
    MFMA kernels; backward gives dfeat and all ten parameter gradients.  The
    training forward keeps the activations the weight gradients need
    (2 KB/sample) so the backward never re-runs the forward."""

    @staticmethod
    def forward(ctx, feat, *params):
        feat = feat.contiguous().float()
        m = feat.shape[0]
        dev = feat.device
        sdf = torch.empty((m,), dtype=torch.float32, device=dev)
        rgb = torch.empty((m, 3), dtype=torch.float32, device=dev)
        ps = [p.contiguous() for p in params]
        # grad mode is off inside Function.forward: needs_input_grad tells what backward will want
        need_w = any(ctx.needs_input_grad[1:])           # weight gradients need the activations
        training = need_w or ctx.needs_input_grad[0]     # dfeat alone (frozen decoder) needs only the masks
        width = ps[0].shape[0]
        lib = L.lib()
        act = torch.empty((int(lib.psvo_mlp_act_floats(m, width)),), dtype=torch.float32,
                          device=dev) if need_w else None
        masks = torch.empty((int(lib.psvo_mlp_mask_words(m, width)),), dtype=torch.int64,
                            device=dev) if training else None
        images = torch.empty((int(lib.psvo_mlp_image_floats_w(width)),), dtype=torch.float32, device=dev)
        with L.timed("mlp_fwd"):
            L.call("psvo_mlp_fwd", L.stream_of(dev), m, width, feat, *ps, images, sdf, rgb, act, masks)
        if training:
            ctx.save_for_backward(feat, rgb, act, masks, images, *ps)
            ctx.need_w = need_w
            ctx.width = width
        return sdf, rgb

    @staticmethod
    def backward(ctx, g_sdf, g_rgb):
        feat, rgb, act, masks, images, *ps = ctx.saved_tensors
        m = feat.shape[0]
        dev = feat.device
        g_sdf = torch.zeros((m,), device=dev) if g_sdf is None else g_sdf.contiguous().float()
        g_rgb = torch.zeros((m, 3), device=dev) if g_rgb is None else g_rgb.contiguous().float()
        n_split = 256  # split-K workgroups of the weight gradients (one per CU)
        ws = torch.empty((int(L.lib().psvo_mlp_workspace_floats_w(m, ctx.width, n_split)),), dtype=torch.float32,
                         device=dev)
        dfeat = torch.empty((m, 16), dtype=torch.float32, device=dev)
        grads = [torch.empty_like(p) for p in ps] if ctx.need_w else [None] * len(ps)
        with L.timed("mlp_bwd"):
            L.call("psvo_mlp_bwd", L.stream_of(dev), m, ctx.width, feat, *ps, images, rgb, act, masks, g_sdf, g_rgb,
                   dfeat, *grads, 0, n_split, ws)
        return (dfeat if ctx.needs_input_grad[0] else None, *grads)


class _Same(nn.Module):
    def __init__(self, in_dim):
        super().__init__()
        self.embedding_size = in_dim

    def forward(self, x):
        return x


class Decoder(nn.Module):
    def __init__(self, depth=8, width=256, in_dim=3, sdf_dim=128, skips=[4], multires=6, embedder="nerf",
                 local_coord=False, **kwargs):
        super().__init__()
        if embedder != "none":
            raise NotImplementedError("only embedder='none' (every shipped config) is supported")
        self.D, self.W, self.skips = depth, width, list(skips)
        self.pe = _Same(in_dim)
        e = self.pe.embedding_size
        self.pts_linears = nn.ModuleList(
            [nn.Linear(e, width)] +
            [nn.Linear(width, width) if i not in self.skips else nn.Linear(width + e, width) for i in range(depth - 1)])
        self.sdf_out = nn.Linear(width, 1 + sdf_dim)
        self.color_out = nn.Sequential(nn.Linear(sdf_dim + e, width), nn.ReLU(), nn.Linear(width, 3), nn.Sigmoid())

    def get_values(self, x):
        x = self.pe(x)
        h = x
        for i, layer in enumerate(self.pts_linears):
            h = F.relu(layer(h))
            if i in self.skips:
                h = torch.cat([x, h], -1)
        o = self.sdf_out(h)
        sdf, feat = o[:, :1], o[:, 1:]
        rgb = self.color_out(torch.cat([feat, x], dim=-1))
        return torch.cat([rgb, sdf], dim=-1)

    def get_sdf(self, inputs):
        return self.get_values(inputs["emb"])[:, 3]

    def fused_params(self):
        l0, l1 = self.pts_linears
        return [l0.weight, l0.bias, l1.weight, l1.bias, self.sdf_out.weight, self.sdf_out.bias,
                self.color_out[0].weight, self.color_out[0].bias, self.color_out[2].weight, self.color_out[2].bias]

    def can_fuse(self, x):
        return (x.is_cuda and self.W in (128, 256) and self.D == 2 and not self.skips and x.shape[-1] == 16
                and self.sdf_out.out_features == 129)

    def forward(self, inputs):
        x = inputs["emb"]
        if self.can_fuse(x):
            sdf, rgb = DecoderMLP.apply(x, *self.fused_params())
            return {"color": rgb, "sdf": sdf}
        out = self.get_values(x)
        return {"color": out[:, :3], "sdf": out[:, 3]}
