"""psvo.optim.Adam (one HIP launch per group) against torch.optim.Adam on the
same parameters and gradients over several steps (the
mapping loop's Adam(embeddings) / Adam(decoder))."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("wd", [0.0, 1e-2])
def test_adam_matches_torch(wd):
    from psvo.optim import Adam
    torch.manual_seed(0)
    shapes = [(20000, 16), (128, 16), (128,), (129, 128), (3,), (7, 5)]
    mine = [torch.randn(s, device=DEV) for s in shapes]
    ref = [p.clone() for p in mine]
    for p in mine + ref:
        p.requires_grad_(True)
    o1 = Adam(mine, lr=5e-3, weight_decay=wd)
    o2 = torch.optim.Adam(ref, lr=5e-3, weight_decay=wd)
    for it in range(6):
        for a, b in zip(mine, ref):
            g = torch.randn_like(a) * (10.0 ** (it % 3 - 1))
            a.grad = g.clone()
            b.grad = g.clone()
        o1.step()
        o2.step()
        for a, b in zip(mine, ref):
            torch.testing.assert_close(a, b, rtol=2e-6, atol=2e-7)
    for a, b in zip(mine, ref):
        s1, s2 = o1.state[a], o2.state[b]
        assert float(s1["step"]) == float(s2["step"]) == 6.0
        # torch's foreach path forms m with lerp, the kernel with β1·m + (1-β1)·g: rounding-level differences
        torch.testing.assert_close(s1["exp_avg"], s2["exp_avg"], rtol=1e-5, atol=2e-6)
        torch.testing.assert_close(s1["exp_avg_sq"], s2["exp_avg_sq"], rtol=1e-5, atol=1e-6)


def test_adam_state_dict_roundtrip_and_skips_none_grads():
    from psvo.optim import Adam
    p = torch.randn(100, device=DEV, requires_grad=True)
    q = torch.randn(10, device=DEV, requires_grad=True)
    o = Adam([p, q], lr=1e-2)
    p.grad = torch.ones_like(p)
    o.step()  # q has no grad: untouched, no state
    assert len(o.state[q]) == 0
    sd = o.state_dict()
    o2 = torch.optim.Adam([p, q], lr=1e-2)
    o2.load_state_dict(sd)
    assert torch.equal(o2.state[p]["exp_avg"], o.state[p]["exp_avg"])
