"""psvo.point_feature.PointsResNet has the reference's module structure
(variations/resnet.py): the reference encoder's initial weights recorded in
tests/golden/BA_room0_resnet.npz load strictly, and the forward runs on the
reference's [B, N, 3] + [B, N, 3] inputs.  CPU only."""
import torch

from conftest import load_golden


def test_points_resnet_loads_reference_state():
    from psvo.point_feature import PointsResNet
    g = load_golden("BA_room0_resnet")
    m = PointsResNet(16)
    sd = {k[5:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("res0.")}
    m.load_state_dict(sd, strict=True)
    out = m(torch.rand(1, 7, 3), torch.rand(1, 7, 3))
    assert out.shape == (1, 7, 16)
