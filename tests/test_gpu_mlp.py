"""Fused fp32-MFMA decoder kernels vs a plain PyTorch fp32 reference of the
same op (nrgbd.Decoder layers; autograd for the backward).  Needs an MI355X."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("width", [128, 256])
@pytest.mark.parametrize("m", [1, 77, 1000, 4099])
def test_decoder_fused_matches_torch(m, width):
    from psvo.decoder import Decoder, DecoderMLP
    torch.manual_seed(m)
    dec = Decoder(depth=2, width=width, in_dim=16, skips=[], embedder="none").to(DEV)
    with torch.no_grad():
        for p in dec.parameters():
            p.mul_(3.0)  # wider pre-activations: exercise both ReLU sides and sigmoid tails
    x = (torch.randn(m, 16, device=DEV) * 2).requires_grad_(True)
    g_sdf = torch.randn(m, device=DEV)
    g_rgb = torch.randn(m, 3, device=DEV)
    # fused
    sdf, rgb = DecoderMLP.apply(x, *dec.fused_params())
    (sdf * g_sdf).sum().backward(retain_graph=True)
    (rgb * g_rgb).sum().backward()
    got = {"x": x.grad.clone()}
    for n, p in dec.named_parameters():
        got[n] = p.grad.clone()
        p.grad = None
    x.grad = None
    # reference (torch layers, fp32, TF32 off)
    torch.backends.cuda.matmul.allow_tf32 = False
    ref = dec.get_values(x)
    torch.testing.assert_close(sdf, ref[:, 3], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(rgb, ref[:, :3], rtol=1e-4, atol=1e-5)
    ((ref[:, 3] * g_sdf).sum() + (ref[:, :3] * g_rgb).sum()).backward()
    exp = {"x": x.grad}
    for n, p in dec.named_parameters():
        exp[n] = p.grad
    for k in exp:
        scale = exp[k].abs().max().item() + 1e-12
        err = (got[k] - exp[k]).abs().max().item()
        assert err <= 2e-4 * scale, (k, err, scale)


@pytest.mark.parametrize("width", [128, 256])
def test_decoder_fused_is_deterministic(width):
    from psvo.decoder import Decoder, DecoderMLP
    torch.manual_seed(0)
    dec = Decoder(depth=2, width=width, in_dim=16, skips=[], embedder="none").to(DEV)
    x = torch.randn(20000, 16, device=DEV, requires_grad=True)
    outs = []
    for _ in range(2):
        sdf, rgb = DecoderMLP.apply(x, *dec.fused_params())
        (sdf.sum() + rgb.sum()).backward()
        outs.append([x.grad.clone()] + [p.grad.clone() for p in dec.parameters()])
        x.grad = None
        for p in dec.parameters():
            p.grad = None
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("width", [128, 256])
def test_decoder_frozen_and_inference(width):
    """Frozen decoder (tracking: dfeat only, no activations kept) and the
    inference forward (no grad) give the training path's numbers."""
    from psvo.decoder import Decoder, DecoderMLP
    torch.manual_seed(5)
    dec = Decoder(depth=2, width=width, in_dim=16, skips=[], embedder="none").to(DEV)
    x = torch.randn(3001, 16, device=DEV)
    g_sdf = torch.randn(3001, device=DEV)
    g_rgb = torch.randn(3001, 3, device=DEV)
    xa = x.clone().requires_grad_(True)
    sdf, rgb = DecoderMLP.apply(xa, *dec.fused_params())
    ((sdf * g_sdf).sum() + (rgb * g_rgb).sum()).backward()
    xb = x.clone().requires_grad_(True)
    frozen = [p.detach() for p in dec.fused_params()]
    sdf2, rgb2 = DecoderMLP.apply(xb, *frozen)
    ((sdf2 * g_sdf).sum() + (rgb2 * g_rgb).sum()).backward()
    assert torch.equal(sdf, sdf2) and torch.equal(rgb, rgb2)
    assert torch.equal(xa.grad, xb.grad)
    with torch.no_grad():
        sdf3, rgb3 = DecoderMLP.apply(x, *frozen)
    assert torch.equal(sdf3, sdf2) and torch.equal(rgb3, rgb2)
