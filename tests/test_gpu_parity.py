"""HIP path vs the oracle / golden vectors (needs an MI355X).

Bars:
  * octree hit / leaf indices, sample voxel ids, ray & sample masks: bit-exact;
  * sample depths: bit-exact on rays whose Σ(t_out - t_in) matches the
    golden's torch-CPU summation order (the only order-dependent input of the
    sampler), |Δz| ≤ 1e-5 relative on the rest;
  * fp32 outputs (sdf, weights, colour, depth, loss): rtol 1e-4 / atol 1e-5;
  * gradients: max|Δ| ≤ 2e-3 · max|ref| per tensor (float-atomic order and
    GEMM blocking differ from torch-CPU).
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _decoder(g):
    from psvo.decoder import Decoder
    dec = Decoder(depth=2, width=int(g["width"]), in_dim=16, skips=[], embedder="none", multires=0)
    dec.load_state_dict({k[4:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("dec.")})
    return dec.to(DEV)


def _map_states(g, emb):
    return {"voxel_vertex_idx": torch.from_numpy(g["features"]).to(DEV),
            "voxel_center_xyz": torch.from_numpy(g["centres"]).to(DEV),
            "voxel_structure": torch.from_numpy(g["structure"]).to(DEV),
            "voxel_vertex_emb": emb}


def _args(g):
    import types
    crit = dict(zip(("rgb_weight", "depth_weight", "fs_weight", "sdf_weight"), g["crit"].tolist()))
    crit["sdf_truncation"] = float(g["truncation"])
    return types.SimpleNamespace(criteria=crit, data_specs={"max_depth": float(g["max_depth"])})


def _torch_row_sums(g):
    idx = torch.from_numpy(g["hit_idx"]).reshape(-1, g["hit_idx"].shape[-1])
    d = (torch.from_numpy(g["hit_max"]) - torch.from_numpy(g["hit_min"])).reshape(idx.shape).masked_fill(idx.eq(-1), 0)
    seq = np.zeros(d.shape[0], np.float32)
    for j in range(d.shape[1]):
        seq = (seq + d[:, j].numpy()).astype(np.float32)
    return d.sum(-1).numpy(), seq


def test_grid_svo_intersect_matches_oracle(golden):
    import grid
    _, g = golden
    ro = torch.from_numpy(g["rays_o"]).to(DEV)
    rd = torch.from_numpy(g["rays_d"]).to(DEV)
    pts = torch.from_numpy(g["centres"]).to(DEV).unsqueeze(0)
    ch = torch.from_numpy(g["structure"]).to(DEV).unsqueeze(0)
    idx, lo, hi = grid.svo_intersect(ro, rd, pts, ch, 0.2, 50)
    np.testing.assert_array_equal(idx.cpu().numpy()[0], g["raw_idx"])
    np.testing.assert_array_equal(lo.cpu().numpy()[0], np.where(g["raw_idx"] >= 0, g["raw_t0"], 0))
    np.testing.assert_array_equal(hi.cpu().numpy()[0], np.where(g["raw_idx"] >= 0, g["raw_t1"], 0))



def test_grid_svo_intersect_reference_layout(golden):
    """grid.svo_intersect called exactly as an unchanged voxel_helpers.py
    calls it (SparseVoxelOctreeRayIntersect.forward, voxel_helpers.py:112-154):
    G = min(256, 2e9 / (points + children numel)) blocks, the rays padded by
    repeating the first H − N, reshaped to [G, K, 3], the octree expanded G
    times with .contiguous(); every batch b's rows against the C oracle,
    then the reference's reshape / trim back to [1, N, n_max]."""
    import grid
    _, g = golden
    ro = torch.from_numpy(g["rays_o"]).to(DEV)
    rd = torch.from_numpy(g["rays_d"]).to(DEV)
    points = torch.from_numpy(g["centres"]).to(DEV)
    children = torch.from_numpy(g["structure"]).to(DEV)
    G = min(256, int(2 * 10 ** 9 / (points.numel() + children.numel())))
    S, N = ro.shape[:2]
    K = int(np.ceil(N / G))
    H = K * G
    assert G > 1  # several blocks (padded rows where N is not a multiple of G)
    if H > N:
        ro = torch.cat([ro, ro[:, :H - N]], 1)
        rd = torch.cat([rd, rd[:, :H - N]], 1)
    ro, rd = ro.reshape(S * G, K, 3), rd.reshape(S * G, K, 3)
    pts = points.expand(S * G, *points.size()).contiguous()
    ch = children.expand(S * G, *children.size()).contiguous()
    idx, lo, hi = grid.svo_intersect(ro.float(), rd.float(), pts.float(), ch.int(), 0.2, 50)
    assert tuple(idx.shape) == (G, K, 50)
    pad = np.concatenate([np.arange(N), np.arange(H - N)])  # the ray each padded row repeats
    want_idx = g["raw_idx"][pad].reshape(G, K, 50)
    want_lo = np.where(g["raw_idx"] >= 0, g["raw_t0"], 0)[pad].reshape(G, K, 50)
    want_hi = np.where(g["raw_idx"] >= 0, g["raw_t1"], 0)[pad].reshape(G, K, 50)
    for b in range(G):  # batch by batch: each block reads its own copy of the tree
        np.testing.assert_array_equal(idx[b].cpu().numpy(), want_idx[b], err_msg=f"batch {b}")
        np.testing.assert_array_equal(lo[b].cpu().numpy(), want_lo[b], err_msg=f"batch {b}")
        np.testing.assert_array_equal(hi[b].cpu().numpy(), want_hi[b], err_msg=f"batch {b}")
    out = idx.reshape(S, H, -1)[:, :N]  # voxel_helpers.py:148-154
    np.testing.assert_array_equal(out.cpu().numpy()[0], g["raw_idx"])

def test_ray_intersect_vox_matches_golden(golden):
    from psvo.voxel_helpers import ray_intersect_vox
    _, g = golden
    out, hits = ray_intersect_vox(torch.from_numpy(g["rays_o"]).to(DEV), torch.from_numpy(g["rays_d"]).to(DEV),
                                  torch.from_numpy(g["centres"]).to(DEV), torch.from_numpy(g["structure"]).to(DEV),
                                  0.2, 10, 10.0)
    np.testing.assert_array_equal(out["intersected_voxel_idx"].cpu().numpy(), g["hit_idx"])
    np.testing.assert_array_equal(out["min_depth"].cpu().numpy(), g["hit_min"])
    np.testing.assert_array_equal(out["max_depth"].cpu().numpy(), g["hit_max"])
    np.testing.assert_array_equal(hits.cpu().numpy(), g["hits"])


def test_grid_inverse_cdf_matches_oracle():
    """Reference-layout sampler launch vs the C oracle on random hit lists."""
    import grid
    rng = np.random.default_rng(0)
    b, k, p = 7, 37, 6
    nb = rng.integers(0, p + 1, size=(b, k))
    idx = np.full((b, k, p), -1, np.int32)
    lo = np.full((b, k, p), 10.0, np.float32)
    hi = np.full((b, k, p), 10.0, np.float32)
    for i in range(b):
        for j in range(k):
            t = 0.5
            for h in range(nb[i, j]):
                a = t + rng.uniform(0.0, 0.3)
                w = rng.uniform(0.01, 0.35)
                idx[i, j, h], lo[i, j, h], hi[i, j, h] = rng.integers(0, 1000), a, a + w
                t = a + w
    d = np.where(idx >= 0, hi - lo, 0).astype(np.float32)
    s = d.sum(-1, keepdims=True).astype(np.float32)
    probs = (d / np.where(s > 0, s, 1)).astype(np.float32)
    steps = (s[..., 0] / np.float32(0.02)).astype(np.float32)
    ms = int(np.ceil(steps).max()) + p
    noise = rng.uniform(0.001, 0.999, size=(b, k, ms)).astype(np.float32)
    o_idx = np.full((b, k, ms), -1, np.int32)
    o_dep = np.zeros((b, k, ms), np.float32)
    o_dis = np.zeros((b, k, ms), np.float32)
    O.lib().oracle_inverse_cdf(b, k, p, ms, -1.0, *(O._ptr(a) for a in (idx, lo, hi, noise, probs, steps, o_idx,
                                                                         o_dep, o_dis)))
    t = lambda a: torch.from_numpy(a).to(DEV)
    g_idx, g_dep, g_dis = grid.inverse_cdf_sampling(t(idx), t(lo), t(hi), t(noise), t(probs), t(steps), -1.0)
    np.testing.assert_array_equal(g_idx.cpu().numpy(), o_idx)
    np.testing.assert_array_equal(g_dep.cpu().numpy(), o_dep)
    np.testing.assert_array_equal(g_dis.cpu().numpy(), o_dis)


def test_sampler_slot_quirk_known_answer_on_gpu():
    import grid
    b, k, p = 1, 8, 2
    t = lambda a: torch.tensor(a).to(DEV).contiguous()
    idx = t(np.tile(np.array([5, 9], np.int32), (b, k, 1)))
    lo = t(np.tile(np.array([1.0, 1.4], np.float32), (b, k, 1)))
    hi = t(np.tile(np.array([1.2, 1.6], np.float32), (b, k, 1)))
    probs = t(np.tile(np.array([0.5, 0.5], np.float32), (b, k, 1)))
    steps = t(np.full((b, k), 8.0, np.float32))
    noise = t(np.full((b, k, 10), 0.5, np.float32))
    s_idx, _, _ = grid.inverse_cdf_sampling(idx, lo, hi, noise, probs, steps, -1.0)
    assert (s_idx[0] != -1).sum(-1).tolist() == [10, 10, 10, 10, 9, 9, 9, 9]


def _run_product(g):
    from psvo.criterion import Criterion
    from psvo.render_helpers import render_rays
    emb = torch.from_numpy(g["embeddings"]).to(DEV).requires_grad_(True)
    dec = _decoder(g)
    ro = torch.from_numpy(g["rays_o"]).to(DEV).requires_grad_(True)
    rd = torch.from_numpy(g["rays_d"]).to(DEV).requires_grad_(True)
    out = render_rays(ro, rd, _map_states(g, emb), dec, None, float(g["step_size"]), 0.2, float(g["truncation"]), 10,
                      float(g["max_depth"]), noise=torch.from_numpy(g["noise"]), return_samples=True)
    crit = Criterion(_args(g))
    loss, parts = crit(out, (torch.from_numpy(g["rgb"]).to(DEV), torch.from_numpy(g["depth_gt"]).to(DEV)))
    loss.backward()
    grads = {"embeddings": emb.grad, "rays_o": ro.grad, "rays_d": rd.grad}
    for k, p in dec.named_parameters():
        grads["dec." + k] = p.grad
    return out, loss, parts, grads


def test_render_forward_matches_golden(golden):
    name, g = golden
    out, loss, parts, grads = _run_product(g)
    np.testing.assert_array_equal(out["ray_mask"].cpu().numpy(), g["ray_mask"])
    z = out["z_vals"].cpu().numpy()
    assert z.shape == g["z_vals"].shape, (z.shape, g["z_vals"].shape)
    torch_sum, seq_sum = _torch_row_sums(g)
    hit_rows = g["ray_mask"].reshape(-1)
    same_order = (torch_sum == seq_sum)[hit_rows]
    np.testing.assert_array_equal(z[same_order], g["z_vals"][same_order])
    np.testing.assert_allclose(z[~same_order], g["z_vals"][~same_order], rtol=1e-5, atol=1e-6)
    tol = dict(rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(out["sdf"].detach().cpu().numpy(), g["sdf"], **tol)
    np.testing.assert_allclose(out["weights"].detach().cpu().numpy(), g["weights"], **tol)
    np.testing.assert_allclose(out["color"].detach().cpu().numpy(), g["color"], **tol)
    np.testing.assert_allclose(out["depth"].detach().cpu().numpy(), g["depth"], **tol)
    np.testing.assert_allclose(float(loss), float(g["loss"]), rtol=1e-4)


def test_render_gradients_match_golden(golden):
    name, g = golden
    out, loss, parts, grads = _run_product(g)
    pairs = [("embeddings", "grad_embeddings"), ("rays_o", "grad_rays_o"), ("rays_d", "grad_rays_d")]
    pairs += [("dec." + k[len("grad_dec."):], k) for k in g if k.startswith("grad_dec.")]
    for mine, ref_key in pairs:
        got = grads[mine].detach().cpu().numpy()
        ref = g[ref_key]
        scale = np.abs(ref).max() + 1e-12
        err = np.abs(got - ref).max()
        assert err <= 2e-3 * scale, (name, mine, err, scale)


def test_interp_matches_torch_fp32_reference():
    """Numerics of the fused gather + trilinear kernel pair vs a plain
    PyTorch fp32 reference of the same op (autograd for the backward)."""
    from psvo.render_helpers import InterpSamples
    torch.manual_seed(0)
    n_nodes, n_rays, per = 500, 64, 37
    centres = (torch.rand(n_nodes, 3, device=DEV) * 4).float()
    vidx = torch.randint(0, 900, (n_nodes, 8), device=DEV, dtype=torch.int32)
    emb = torch.randn(900, 16, device=DEV, requires_grad=True)
    M = n_rays * per
    ray = torch.arange(n_rays, device=DEV, dtype=torch.int32).repeat_interleave(per)
    offsets = torch.arange(0, M + 1, per, device=DEV, dtype=torch.int32)
    # each ray crosses runs of samples inside 3 voxels (points stay inside
    # their voxel: trilinear weights in [0, 1] as on the render path)
    leaf = torch.randperm(n_nodes, device=DEV)[: n_rays * 3].to(torch.int32).view(n_rays, 3)  # distinct runs
    leaf = leaf.repeat_interleave(torch.tensor([12, 13, 12], device=DEV), dim=1).reshape(-1).contiguous()
    ro = (centres[leaf.view(n_rays, per)[:, 0].long()] - 0.05).detach().requires_grad_(True)
    rd = (torch.rand(n_rays, 3, device=DEV) * 0.02).requires_grad_(True)
    t = torch.sort(torch.rand(n_rays, per, device=DEV) * 3, dim=1).values.reshape(-1)
    # move each sample's leaf centre so that x = o + d t sits inside it
    x_s = (ro[ray.long()] + rd[ray.long()] * t[:, None]).detach()
    centres = centres.clone()
    centres[leaf.long()] = x_s + (torch.rand(M, 3, device=DEV) - 0.5) * 0.15
    feat = InterpSamples.apply(ro, rd, emb, leaf, t, ray, offsets, centres, vidx, 0.2)
    gout = torch.randn_like(feat)
    (feat * gout).sum().backward()
    g_mine = [x.grad.clone() for x in (emb, ro, rd)]
    for x in (emb, ro, rd):
        x.grad = None
    x = ro[ray.long()] + rd[ray.long()] * t[:, None]
    p = ((x - centres[leaf.long()]) / 0.2 + 0.5).unsqueeze(1)
    q = O._CORNERS.to(DEV).unsqueeze(0)
    w = (p * q + (1 - p) * (1 - q)).prod(-1, keepdim=True)
    ref = (w * emb[vidx[leaf.long()].long()]).sum(1)
    (ref * gout).sum().backward()
    torch.testing.assert_close(feat, ref, rtol=1e-5, atol=1e-5)
    for a, b in zip(g_mine, (emb.grad, ro.grad, rd.grad)):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4 * b.abs().max().item())


def test_full_size_properties():
    """BASELINE config B shape (4096 rays, room0, ~64 samples/ray): hit sets
    equal a brute-force AABB test over every SURFACE leaf (when < 50 hits),
    sample depths lie inside their hit intervals, weights are a partition of
    ≤ 1, gradients are finite, and indices are run-to-run deterministic."""
    from psvo import synthetic as syn
    from psvo.octree import Octree, map_states
    from psvo.decoder import Decoder
    from psvo.render_helpers import render_rays, query_samples
    w = syn.make_workload("room0", 4, 1024, seed=0)
    tree = Octree()
    tree.init(256, 16, 0.2, 8)
    tree.insert(w.voxels)
    emb = (torch.randn(tree.count_nodes(), 16, device=DEV) * 0.3).requires_grad_(True)
    ms = map_states(tree, emb, 0.2, device=DEV)
    ro, rd = w.rays_o.to(DEV), w.rays_d.to(DEV)
    s1 = query_samples(ro, rd, ms, 0.008, 0.2, 10.0, seed=7)
    s2 = query_samples(ro, rd, ms, 0.008, 0.2, 10.0, seed=7)
    assert torch.equal(s1.s_idx, s2.s_idx) and torch.equal(s1.z_vals, s2.z_vals)
    assert s1.m / s1.r_hit > 40
    # brute force: every SURFACE leaf box vs every ray, on CPU in float64
    leaves = torch.nonzero(ms["voxel_structure"][:, 8] == 1).squeeze(1)
    c = ms["voxel_center_xyz"][leaves].double().cpu()
    o64, d64 = ro[0].double().cpu(), rd[0].double().cpu()
    inv = 1.0 / d64
    t0 = ((c[None] - 0.1) - o64[:, None]) * inv[:, None]
    t1 = ((c[None] + 0.1) - o64[:, None]) * inv[:, None]
    tlo = torch.minimum(t0, t1).amax(-1).clamp(min=0)
    thi = torch.maximum(t0, t1).amin(-1)
    brute = (tlo < thi - 1e-5)  # strictly inside (grazing contacts excluded both ways)
    from psvo.voxel_helpers import _intersect_sorted
    q = _intersect_sorted(ro, rd, ms["voxel_center_xyz"], ms["voxel_structure"], 0.2, 10.0, 0.008)
    nv = q["ray_nv"].cpu()
    idx = q["hit_idx"].cpu()
    leaf_pos = {int(l): i for i, l in enumerate(leaves.tolist())}
    for r in range(0, ro.shape[1], 37):
        if nv[r] >= 50:
            continue
        mine = set(int(v) for v in idx[r, : nv[r]].tolist())
        exp = set(int(leaves[j]) for j in torch.nonzero(brute[r]).squeeze(1).tolist())
        assert exp <= mine, (r, exp - mine)
    out = render_rays(ro, rd, ms, Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none").to(DEV), None, 0.008, 0.2, 0.1, 10, 10.0)
    wsum = out["weights"].sum(-1)
    assert torch.all(wsum <= 1.0 + 1e-5)
    loss = out["color"].sum() + out["depth"].sum() + out["sdf"].sum()
    loss.backward()
    assert torch.isfinite(emb.grad).all()


@pytest.mark.parametrize("step", [0.0078, 0.05])
def test_fused_sampler_matches_oracle_full_size(step):
    """The wave-parallel fused sampler (one wave per hit ray) against the C
    oracle's serial restatement of sample_gpu.cu on BASELINE config B
    (room0, 4096 rays), fed the same intersections, probs and noise: sample
    indices, depths and distances bit-identical."""
    from psvo import synthetic as syn
    from psvo.octree import Octree, map_states
    from psvo.render_helpers import query_samples
    from psvo.voxel_helpers import _intersect_sorted
    w = syn.make_workload("room0", 4, 1024, seed=3)
    tree = Octree()
    tree.init(256, 16, 0.2, 8)
    tree.insert(w.voxels)
    ms = map_states(tree, torch.zeros(tree.count_nodes(), 16, device=DEV), 0.2, device=DEV)
    ro, rd = w.rays_o.to(DEV), w.rays_d.to(DEV)
    q = _intersect_sorted(ro, rd, ms["voxel_center_xyz"], ms["voxel_structure"], 0.2, 10.0, step)
    st = q["stats"].cpu()
    P, r_hit, max_ceil = int(st[0]), int(st[1]), int(st[2])
    hit = torch.nonzero(q["ray_nv"].cpu() > 0).squeeze(1)
    idx = q["hit_idx"].cpu()[hit, :P]
    t0 = q["hit_t0"].cpu()[hit, :P]
    t1 = q["hit_t1"].cpu()[hit, :P]
    dsum = q["ray_dsum"].cpu()[hit]
    dd = torch.where(idx != -1, t1 - t0, torch.zeros_like(t0))
    probs = torch.from_numpy(dd.numpy() / dsum.numpy()[:, None])
    steps = torch.from_numpy(dsum.numpy() / np.float32(step))
    kp = (r_hit + 199) // 200
    max_steps = max_ceil + P
    noise = torch.rand((200, kp, max_steps), generator=torch.Generator().manual_seed(5)).clamp(0.001, 0.999)
    o_idx, o_dep, o_dis, _ = O.inverse_cdf_sampling(idx, t0, t1, probs, steps, -1.0, noise)
    o_dis = o_dis.clamp(min=0.0)
    o_dep = o_dep.masked_fill(o_idx.eq(-1), O.MAX_DEPTH)
    o_dis = o_dis.masked_fill(o_idx.eq(-1), 0.0)
    smp = query_samples(ro, rd, ms, step, 0.2, 10.0, noise=noise)
    n = o_idx.shape[1]
    g_idx, g_dep, g_dis = smp.s_idx.cpu(), smp.s_depth.cpu(), smp.s_dist.cpu()
    assert smp.r_hit == r_hit and g_idx.shape[0] == o_idx.shape[0]
    np.testing.assert_array_equal(g_idx[:, :n].numpy(), o_idx.numpy())
    np.testing.assert_array_equal(g_dep[:, :n].numpy(), o_dep.numpy())
    np.testing.assert_array_equal(g_dis[:, :n].numpy(), o_dis.numpy())
    assert bool((g_idx[:, n:] == -1).all())


def test_config_e_multiroom_properties():
    """SURVEY §8 config E (multi-room scene, 1024³ grid, >1M surface leaves,
    depth-10 tree): hit sets contain every brute-force SURFACE leaf (rays with
    < 50 hits), indices are deterministic, one engine iteration over the
    2.7M-row embedding table gives a finite loss and touches only the rows the
    rays reach."""
    from psvo import synthetic as syn
    from psvo.octree import Octree, map_states
    from psvo.decoder import Decoder
    from psvo.engine import MappingEngine
    from psvo.render_helpers import query_samples
    from psvo.voxel_helpers import _intersect_sorted
    w = syn.make_workload("multiroom", 2, 512, seed=3)
    tree = Octree()
    tree.init(w.scene.grid_dim, 16, w.scene.voxel_size, 8)
    tree.insert(w.voxels)
    n_nodes = tree.count_nodes()
    assert n_nodes > 2_000_000
    emb = torch.randn(n_nodes, 16, device=DEV) * 0.1
    ms = map_states(tree, emb, w.scene.voxel_size, device=DEV)
    assert int((ms["voxel_structure"][:, 8] == 1).sum()) > 1_000_000
    ro, rd = w.rays_o.to(DEV), w.rays_d.to(DEV)
    vs = w.scene.voxel_size
    s1 = query_samples(ro, rd, ms, 0.008, vs, 10.0, seed=7)
    s2 = query_samples(ro, rd, ms, 0.008, vs, 10.0, seed=7)
    assert torch.equal(s1.s_idx, s2.s_idx) and torch.equal(s1.z_vals, s2.z_vals)
    q = _intersect_sorted(ro, rd, ms["voxel_center_xyz"], ms["voxel_structure"], vs, 10.0, 0.008)
    nv, idx = q["ray_nv"].cpu(), q["hit_idx"].cpu()
    leaves = torch.nonzero(ms["voxel_structure"][:, 8] == 1).squeeze(1)
    c = ms["voxel_center_xyz"][leaves].double().cpu()
    checked = 0
    for r in range(0, ro.shape[1], 61):
        if nv[r] >= 50:
            continue
        o64, d64 = ro[0, r].double().cpu(), rd[0, r].double().cpu()
        inv = 1.0 / d64
        t0 = ((c - vs / 2) - o64) * inv
        t1 = ((c + vs / 2) - o64) * inv
        tlo = torch.minimum(t0, t1).amax(-1).clamp(min=0)
        thi = torch.maximum(t0, t1).amin(-1)
        exp = set(int(leaves[j]) for j in torch.nonzero(tlo < thi - 1e-5).squeeze(1).tolist())
        mine = set(int(v) for v in idx[r, : nv[r]].tolist())
        assert exp <= mine, (r, exp - mine)
        checked += 1
    assert checked > 0
    dec = Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none").to(DEV)
    emb0 = emb.clone()
    eng = MappingEngine(ms, dec, vs, 0.008, truncation=0.1, max_distance=10.0, max_depth=10.0)
    loss = float(eng.step(ro, rd, w.rgb.to(DEV), w.depth.to(DEV), seed=5))
    assert loss == loss and abs(loss) < 1e30
    touched = (emb - emb0).abs().amax(-1) > 0
    reached = torch.zeros(n_nodes, dtype=torch.bool, device=DEV)
    hit = idx[torch.arange(idx.shape[1])[None, :] < nv[:, None]].unique().long().to(DEV)
    reached[ms["voxel_vertex_idx"][hit].reshape(-1).long()] = True
    assert int(touched.sum()) > 0
    assert not bool((touched & ~reached).any())
    eng.close()
