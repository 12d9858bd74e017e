"""NRGBD decoder with the reference's module structure (src/variations/nrgbd.py:80-146),
so state_dicts load both ways.  Every shipped config uses depth 2,
embedder 'none', skips []:

  h = ReLU(L0(x)); h = ReLU(L1(h)); o = sdf_out(h) = [sdf | f(128)]
  rgb = σ(L5(ReLU(L4([f, x]))))

forward/get_values run the layers with PyTorch-ROCm GEMMs (hipBLASLt);
the render path calls forward({'emb': feats}) on all valid samples at once.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


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

    def forward(self, inputs):
        out = self.get_values(inputs["emb"])
        return {"color": out[:, :3], "sdf": out[:, 3]}
