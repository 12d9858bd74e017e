"""The points encoder Mapping hands to bundle_adjust_frames as `resnet`
(mapping.py:36 `get_resnet(args)` → variations/resnet.py PointsResNet with
replica.yaml:13-14 `resnet_specs: {feature_n: 16}`), with the reference's
module structure so its state_dict loads both ways.

The render path never runs it: render_rays' point-feature branch
(get_features_pcd) is commented out (render_helpers.py:481), so its
parameters never receive a gradient and Mapping's `resnet_optim`
(mapping.py:93) never moves them.  psvo.render_helpers.bundle_adjust_frames
accepts both and keeps the native engine (the optimiser's step is a no-op
torch itself would skip)."""
import torch
import torch.nn as nn


class PointsResNet(nn.Module):
    """variations/resnet.py: [x1 | y] (3 + 3 channels) → 64 → 128 → 256 → 512
    (ReLU after each) → fc → feature_n, per point."""

    def __init__(self, feature_n=16):
        super().__init__()
        self.resnet = nn.Sequential(nn.Linear(6, 64), nn.ReLU(inplace=False), nn.Linear(64, 128),
                                    nn.ReLU(inplace=False), nn.Linear(128, 256), nn.ReLU(inplace=False),
                                    nn.Linear(256, 512), nn.ReLU(inplace=False))
        self.fc = nn.Linear(512, feature_n)

    def forward(self, x1, y):
        x = torch.cat((x1, y), 2)
        x = self.resnet(x.reshape(-1, x.shape[2])).view(x1.size(0), x1.size(1), -1)
        return self.fc(x)
