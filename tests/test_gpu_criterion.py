"""Fused Criterion kernels (csrc/criterion.hip) vs the PyTorch formulation of
src/criterion.py:17-116 on the same inputs, including the edge cases the
loss has (no valid depth, zero residuals, disabled terms) and the
data-parallel identity: shard sums (+ pad_extra) all-reduced == one GPU."""
import types

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _args(tr=0.05, max_depth=5.0):
    return types.SimpleNamespace(criteria={"rgb_weight": 0.5, "depth_weight": 1.0, "sdf_weight": 5000.0,
                                           "fs_weight": 10.0, "sdf_truncation": tr},
                                 data_specs={"max_depth": max_depth})


def _case(seed, R=400, r_hit=300, s_max=77, depth_fill=None):
    g = torch.Generator().manual_seed(seed)
    hit = torch.sort(torch.randperm(R, generator=g)[:r_hit]).values
    ray_mask = torch.zeros(R, dtype=torch.bool)
    ray_mask[hit] = True
    ns = torch.randint(1, s_max + 1, (r_hit,), generator=g)
    ns[0] = s_max
    z = torch.sort(torch.rand(r_hit, s_max, generator=g) * 6, dim=1).values
    col = torch.arange(s_max)[None, :]
    valid = col < ns[:, None]
    z = torch.where(valid, z, torch.full_like(z, 10.0))
    sdf = torch.where(valid, torch.randn(r_hit, s_max, generator=g) * 0.5, torch.ones_like(z))
    color = torch.rand(r_hit, 3, generator=g)
    depth = torch.rand(r_hit, generator=g) * 6
    gt_rgb = torch.rand(R, 3, generator=g)
    gt_depth = torch.rand(R, generator=g) * 6.5 - 0.3  # some <= 0.01, some >= max_depth
    if depth_fill is not None:
        gt_depth.fill_(depth_fill)
    gt_rgb[hit[:5]] = color[:5]  # exact zero residuals: sign(0) = 0
    return dict(hit=hit, ray_mask=ray_mask, z=z, sdf=sdf, color=color, depth=depth, gt_rgb=gt_rgb, gt_depth=gt_depth)


def _run(crit, c, fused, **kw):
    color = c["color"].to(DEV).requires_grad_(True)
    depth = c["depth"].to(DEV).requires_grad_(True)
    sdf = c["sdf"].to(DEV).requires_grad_(True)
    out = {"color": color, "depth": depth, "sdf": sdf, "z_vals": c["z"].to(DEV), "weights": None,
           "ray_mask": c["ray_mask"].to(DEV).view(1, -1)}
    if fused:
        out["rank_ray"] = c["hit"].to(DEV, torch.int32)
    loss, parts = crit(out, (c["gt_rgb"].to(DEV).view(1, -1, 3), c["gt_depth"].to(DEV).view(1, -1)), **kw)
    loss.backward()
    return loss, parts, color.grad, depth.grad, sdf.grad


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_fused_criterion_matches_torch(seed):
    from psvo.criterion import Criterion
    crit = Criterion(_args())
    c = _case(seed)
    lf, pf, *gf = _run(crit, c, True)
    lt, pt, *gt = _run(crit, c, False)
    np.testing.assert_allclose(float(lf), float(lt), rtol=2e-5)
    for k in ("color_loss", "depth_loss", "fs_loss", "sdf_loss"):
        np.testing.assert_allclose(pf[k], pt[k], rtol=2e-5, err_msg=k)
    for a, b in zip(gf, gt):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6 * b.abs().max().item())


def test_fused_criterion_flags_and_no_valid_depth():
    from psvo.criterion import Criterion
    crit = Criterion(_args())
    c = _case(5, depth_fill=0.0)  # no valid depth: depth loss NaN (empty mean), sdf_mask empty
    lf, pf, *gf = _run(crit, c, True, use_depth_loss=False)
    lt, pt, *gt = _run(crit, c, False, use_depth_loss=False)
    np.testing.assert_allclose(float(lf), float(lt), rtol=2e-5)
    assert "depth_loss" not in pf
    for a, b in zip(gf, gt):  # fs/sdf balance weights are 0/0 here: NaN sdf grads on both sides
        b = torch.zeros_like(a) if b is None else b  # unused depth: torch gives None, the kernel zeros
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-7, equal_nan=True)
    lf, pf, *_ = _run(crit, c, True)
    lt, pt, *_ = _run(crit, c, False)
    assert np.isnan(float(lf)) and np.isnan(float(lt))
    assert np.isnan(pf["depth_loss"]) and np.isnan(pt["depth_loss"])


def test_sharded_sums_equal_single_gpu():
    """Two shards with different S_max: local sums with pad_extra, summed,
    finalised on the global shape == the single-GPU loss; each shard's
    backward rows == the single-GPU rows."""
    from psvo import _lib as L
    from psvo.criterion import Criterion
    crit = Criterion(_args())
    c = _case(7, R=500, r_hit=400, s_max=90)
    # shard A = first 200 hit rays, trimmed to their own S_max (< 90)
    ns = (c["z"] < 10.0).sum(1)
    ns[:200] = torch.clamp(ns[:200], max=60)
    col = torch.arange(90)[None, :]
    keep = col < ns[:, None]
    c["z"] = torch.where(keep, c["z"], torch.full_like(c["z"], 10.0))
    c["sdf"] = torch.where(keep, c["sdf"], torch.ones_like(c["sdf"]))
    lt, pt, *gt = _run(crit, c, True)
    s_a = int(ns[:200].max())
    shards = [(slice(0, 200), s_a), (slice(200, 400), 90)]
    cfg = dict(tr=0.05, max_depth=5.0)
    sums = []
    dev_c = {k: v.to(DEV) for k, v in c.items()}
    for rows, s_loc in shards:
        r = rows.stop - rows.start
        z = dev_c["z"][rows, :s_loc].contiguous()
        sd = dev_c["sdf"][rows, :s_loc].contiguous()
        ws = torch.empty(int(L.lib().psvo_criterion_workspace_floats(r)), device=DEV)
        s = torch.empty(8, dtype=torch.float64, device=DEV)
        # tensors (not raw pointers) so that temporaries stay alive through the call
        L.call("psvo_criterion_sums", L.stream_of(), r, s_loc, 90 - s_loc, cfg["tr"], cfg["max_depth"],
               dev_c["hit"][rows].int().contiguous(), dev_c["gt_rgb"].contiguous(), dev_c["gt_depth"].contiguous(),
               dev_c["color"][rows].contiguous(), dev_c["depth"][rows].contiguous(), sd, z, ws, s)
        sums.append(s)
    tot = sums[0] + sums[1]
    out = torch.empty(16, device=DEV)
    L.call("psvo_criterion_finalize", L.stream_of(), L.ptr(tot), 400, 90, 0.5, 1.0, 10.0, 5000.0, cfg["tr"], 7,
           L.ptr(out))
    np.testing.assert_allclose(out[0].item(), float(lt), rtol=1e-6)
    # backward rows with the global coefficients
    g = torch.ones((), device=DEV)
    for rows, s_loc in shards:
        r = rows.stop - rows.start
        gc = torch.empty(r, 3, device=DEV)
        gd = torch.empty(r, device=DEV)
        gs = torch.empty(r, s_loc, device=DEV)
        L.call("psvo_criterion_bwd", L.stream_of(), r, s_loc, cfg["tr"], cfg["max_depth"],
               dev_c["hit"][rows].int().contiguous(), dev_c["gt_rgb"].contiguous(), dev_c["gt_depth"].contiguous(),
               dev_c["color"][rows].contiguous(), dev_c["depth"][rows].contiguous(),
               dev_c["sdf"][rows, :s_loc].contiguous(), dev_c["z"][rows, :s_loc].contiguous(), out, g, gc, gd, gs)
        torch.testing.assert_close(gc, gt[0][rows], rtol=1e-6, atol=0)
        torch.testing.assert_close(gd, gt[1][rows], rtol=1e-6, atol=0)
        torch.testing.assert_close(gs, gt[2][rows, :s_loc], rtol=1e-6, atol=1e-12)
        assert torch.all(gt[2][rows, s_loc:] == 0)


def test_fused_criterion_deterministic():
    from psvo.criterion import Criterion
    crit = Criterion(_args())
    c = _case(11, R=5000, r_hit=4096, s_max=200)
    a = _run(crit, c, True)
    b = _run(crit, c, True)
    assert float(a[0]) == float(b[0])
    for x, y in zip(a[2:], b[2:]):
        assert torch.equal(x, y)


@pytest.mark.parametrize("seed,s_max", [(0, 77), (1, 77), (2, 77), (3, 128), (4, 200), (5, 300), (6, 600)])
def test_composite_loss_matches_kernel_chain(seed, s_max):
    """psvo_composite_loss (+ psvo_criterion_coef / _reduce) == composite_fwd →
    criterion_sums → finalize → criterion_bwd → composite_bwd, bit for bit —
    for each of its register-cached (S_max ≤ 128, ≤ 256) and memory variants."""
    from psvo import _lib as L
    c = _case(seed, s_max=s_max)
    r_hit, s_max = c["z"].shape
    g = torch.Generator().manual_seed(100 + seed)
    ns = (c["z"] < 10.0).sum(1).to(torch.int32)
    offsets = torch.zeros(r_hit + 1, dtype=torch.int32)
    offsets[1:] = torch.cumsum(ns, 0)
    M = int(offsets[-1])
    sdf_s = (torch.randn(M, generator=g) * 0.3).to(DEV)
    rgb_s = torch.rand(M, 3, generator=g).to(DEV)
    z = c["z"].contiguous().to(DEV)
    rank_ray = c["hit"].to(torch.int32).to(DEV)
    gt_rgb, gt_depth = c["gt_rgb"].to(DEV), c["gt_depth"].to(DEV)
    offsets, ns = offsets.to(DEV), ns.to(DEV)
    tr, md = 0.05, 5.0
    w = (0.5, 1.0, 10.0, 5000.0)
    st = L.stream_of(DEV)
    f32 = dict(dtype=torch.float32, device=DEV)
    # the chain
    sdf, wts = torch.empty(r_hit, s_max, **f32), torch.empty(r_hit, s_max, **f32)
    col, dep, zmin = torch.empty(r_hit, 3, **f32), torch.empty(r_hit, **f32), torch.empty(r_hit, **f32)
    L.call("psvo_composite_fwd", st, r_hit, s_max, tr, L.ptr(offsets), L.ptr(ns), L.ptr(z), L.ptr(sdf_s),
           L.ptr(rgb_s), L.ptr(sdf), L.ptr(wts), L.ptr(col), L.ptr(dep), L.ptr(zmin))
    ws = torch.empty(r_hit * 8, **f32)
    sums = torch.empty(8, dtype=torch.float64, device=DEV)
    out = torch.zeros(16, **f32)
    L.call("psvo_criterion_sums", st, r_hit, s_max, 0, tr, md, L.ptr(rank_ray), L.ptr(gt_rgb), L.ptr(gt_depth),
           L.ptr(col), L.ptr(dep), L.ptr(sdf), L.ptr(z), L.ptr(ws), L.ptr(sums))
    L.call("psvo_criterion_finalize", st, L.ptr(sums), r_hit, s_max, *w, tr, 7, L.ptr(out))
    g_loss = torch.ones(1, **f32)
    gc, gd, gs = torch.empty(r_hit, 3, **f32), torch.empty(r_hit, **f32), torch.empty(r_hit, s_max, **f32)
    L.call("psvo_criterion_bwd", st, r_hit, s_max, tr, md, L.ptr(rank_ray), L.ptr(gt_rgb), L.ptr(gt_depth),
           L.ptr(col), L.ptr(dep), L.ptr(sdf), L.ptr(z), L.ptr(out), L.ptr(g_loss), L.ptr(gc), L.ptr(gd), L.ptr(gs))
    g_sdf_a, g_rgb_a = torch.empty(M, **f32), torch.empty(M, 3, **f32)
    L.call("psvo_composite_bwd", st, r_hit, s_max, tr, L.ptr(offsets), L.ptr(ns), L.ptr(z), L.ptr(sdf), L.ptr(wts),
           L.ptr(rgb_s), L.ptr(gc), L.ptr(gd), None, L.ptr(gs), L.ptr(g_sdf_a), L.ptr(g_rgb_a))
    # the fused pass
    ws2 = torch.full((r_hit * 8,), float("nan"), **f32)
    sums_c, sums2 = torch.empty(8, dtype=torch.float64, device=DEV), torch.empty(8, dtype=torch.float64, device=DEV)
    coef = torch.empty(4, **f32)
    out2 = torch.zeros(16, **f32)
    L.call("psvo_criterion_coef", st, r_hit, s_max, tr, md, L.ptr(rank_ray), L.ptr(gt_depth), L.ptr(z), *w, 7,
           L.ptr(ws2), L.ptr(sums_c), L.ptr(coef))
    col2, dep2 = torch.empty(r_hit, 3, **f32), torch.empty(r_hit, **f32)
    g_sdf_b, g_rgb_b = torch.empty(M, **f32), torch.empty(M, 3, **f32)
    L.call("psvo_composite_loss", st, r_hit, s_max, tr, md, L.ptr(offsets), L.ptr(ns), L.ptr(z), L.ptr(rank_ray),
           L.ptr(gt_rgb), L.ptr(gt_depth), L.ptr(sdf_s), L.ptr(rgb_s), L.ptr(coef), L.ptr(ws2), L.ptr(col2),
           L.ptr(dep2), L.ptr(g_sdf_b), L.ptr(g_rgb_b))
    L.call("psvo_criterion_reduce", st, r_hit, L.ptr(ws2), L.ptr(sums2))
    L.call("psvo_criterion_finalize", st, L.ptr(sums2), r_hit, s_max, *w, tr, 7, L.ptr(out2))
    torch.cuda.synchronize()
    assert torch.equal(coef, out[7:11]), (coef, out[7:11])
    assert torch.equal(col2, col) and torch.equal(dep2, dep)
    assert torch.equal(sums2, sums)
    assert torch.equal(out2, out)
    assert torch.equal(g_rgb_b, g_rgb_a)
    assert torch.equal(g_sdf_b, g_sdf_a), float((g_sdf_b - g_sdf_a).abs().max())
