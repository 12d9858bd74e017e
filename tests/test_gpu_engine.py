"""The native mapping iteration (psvo.engine.MappingEngine → psvo_map_step)
against the autograd path (render_rays + Criterion + loss.backward() +
psvo.optim.Adam) on the same rays, seeds and initial state: with the dense
decoder the loss of the first iteration and the decoder update are
bit-identical (same kernels, same order; the decoder gradients are
deterministic); embeddings agree up to the order of the float atomics in the
interpolation backward.  The sparse decoder (the default) against the dense
one: the same forward bits, gradients up to the weight gradients' summation
order."""
import types

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup():
    from psvo import synthetic as syn
    from psvo.decoder import Decoder
    from psvo.octree import Octree, map_states
    w = syn.make_workload("room0", 2, 512, seed=4)
    tree = Octree()
    tree.init(256, 16, 0.2, 8)
    tree.insert(w.voxels)
    g = torch.Generator().manual_seed(0)
    emb0 = torch.randn(max(20000, tree.count_nodes()), 16, generator=g) * 0.1
    torch.manual_seed(0)
    dec = Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none").to(DEV)
    return w, tree, emb0, dec


def test_engine_matches_autograd_path():
    from copy import deepcopy
    from psvo.criterion import Criterion
    from psvo.engine import MappingEngine
    from psvo.octree import map_states
    from psvo.optim import Adam
    from psvo.render_helpers import render_rays
    w, tree, emb0, dec = _setup()
    ro, rd = w.rays_o.to(DEV), w.rays_d.to(DEV)
    rgb, depth = w.rgb.to(DEV), w.depth.to(DEV)
    step = 0.01
    crit = {"rgb_weight": 0.5, "depth_weight": 1.0, "sdf_weight": 5000.0, "fs_weight": 10.0}
    # autograd path
    dec_a = deepcopy(dec)
    emb_a = emb0.clone().to(DEV).requires_grad_(True)
    ms_a = map_states(tree, emb_a, 0.2, device=DEV)
    criterion = Criterion(types.SimpleNamespace(criteria=dict(crit, sdf_truncation=0.1),
                                                data_specs={"max_depth": 10.0}))
    oe, od = Adam([emb_a], lr=5e-3), Adam(dec_a.parameters(), lr=5e-3)
    losses_a = []
    for it in range(2):
        out = render_rays(ro, rd, ms_a, dec_a, None, step, 0.2, 0.1, 10, 10.0, seed=100 + it)
        loss, _ = criterion(out, (rgb, depth))
        oe.zero_grad()
        od.zero_grad()
        loss.backward()
        oe.step()
        od.step()
        losses_a.append(float(loss))
        if it == 0:
            dec_after1 = [p.detach().clone() for p in dec_a.fused_params()]
            emb_after1 = emb_a.detach().clone()
    # engine path
    dec_e = deepcopy(dec)
    emb_e = emb0.clone().to(DEV)
    ms_e = map_states(tree, emb_e, 0.2, device=DEV)
    eng = MappingEngine(ms_e, dec_e, 0.2, step, truncation=0.1, max_distance=10.0, criteria=crit, max_depth=10.0,
                        lr_emb=5e-3, lr_dec=5e-3)
    eng.set_paths(MappingEngine.PATH_DENSE_DECODER)  # every sample through the decoder, as autograd runs it
    losses_e = []
    for it in range(2):
        losses_e.append(float(eng.step(ro, rd, rgb, depth, seed=100 + it)))
        if it == 0:
            for a, b in zip(dec_e.fused_params(), dec_after1):
                assert torch.equal(a.detach(), b), "decoder update differs after one iteration"
            diff = (emb_e - emb_after1).abs()
            assert float(diff.max()) <= 2 * 5e-3 + 1e-6
            assert float((diff > 1e-6).float().mean()) < 1e-3
    assert losses_e[0] == losses_a[0]
    assert abs(losses_e[1] - losses_a[1]) <= 1e-4 * abs(losses_a[1])
    st = eng.last_stats
    assert st[1] > 0 and st[4] > 0  # R_hit, M
    eng.close()


@pytest.mark.parametrize("padded,sdf_shift", [(False, 0.0), (True, 0.0), (False, 0.5), (True, 0.5)])
def test_sparse_decoder_matches_dense(padded, sdf_shift):
    """The sparse decoder (the sdf trunk on every sample, the full decoder
    forward and backward on the kept samples only: composited or inside a
    loss mask, composite.hip k_select_samples) against the dense decoder on
    every sample, two psvo_map_step_frames iterations stopped before Adam
    from the same state and seeds, on the single-GPU chain and on the padded
    one (the data-parallel forward): the loss bit for bit (the forward's sdf
    and colours are the same bits), the statistics equal, the embedding /
    decoder gradients and the pose gradient up to the summation order of the
    weight gradients / the scatter.  A dropped sample's gradient is exactly
    zero.  The random decoder's sdf is negative nearly everywhere: the first
    sign change is at the padding (pad 1) and every sample is composited;
    shifted positive (sdf_shift) there is no sign change, z_min is the first
    sample and most samples are dropped."""
    from copy import deepcopy
    from psvo.engine import MappingEngine
    from psvo.octree import map_states
    w, tree, emb0, dec = _setup()
    dec = deepcopy(dec)
    with torch.no_grad():
        dec.sdf_out.bias[0] += sdf_shift
    n = 512
    poses, dirs = _frames_of(w, n)
    rgb, depth = w.rgb.reshape(-1, 3).to(DEV), w.depth.reshape(-1).to(DEV)
    crit = {"rgb_weight": 0.5, "depth_weight": 1.0, "sdf_weight": 5000.0, "fs_weight": 10.0}
    base = MappingEngine.PATH_PADDED if padded else 0
    runs = {}
    for mode in ("dense", "sparse"):
        e = emb0.clone().to(DEV)
        eng = MappingEngine(map_states(tree, e, 0.2, device=DEV), dec, 0.2, 0.01, truncation=0.1,
                            max_distance=10.0, criteria=crit, max_depth=10.0)
        eng.set_paths(base | (MappingEngine.PATH_DENSE_DECODER if mode == "dense" else 0))
        out = []
        for it in range(2):
            pg = torch.zeros(poses.shape[0], 8, device=DEV)
            loss = eng.step_frames(dirs, n, poses.clone(), torch.zeros_like(poses), torch.zeros_like(poses), [0, 1],
                                   1e-3, rgb, depth, seed=700 + it, apply_adam=False, pose_grad=pg, want_loss=True)
            torch.cuda.synchronize()
            out.append((float(loss), list(eng.last_stats), eng.grad_flat.cpu().clone(), pg.cpu()))
        if mode == "sparse":
            sel = eng.select_stats()
            m = out[-1][1][4]
            assert sel["steps"] == 2 and 0 < sel["composited"] <= sel["kept"] <= m, (sel, m)
            if sdf_shift > 0:
                assert sel["kept"] < 0.8 * m, (sel, m)  # the selection drops samples
        runs[mode] = out
        eng.close()
    n_emb = emb0.shape[0] * 16
    for (la, sa, ga, pa), (lb, sb, gb, pb) in zip(runs["dense"], runs["sparse"]):
        assert sa[:13] == sb[:13]
        assert la == lb, (la, lb)
        gd, gs = ga[n_emb:], gb[n_emb:]
        torch.testing.assert_close(gs, gd, rtol=1e-4, atol=1e-5 * float(gd.abs().max()))
        torch.testing.assert_close(gb[:n_emb], ga[:n_emb], rtol=1e-4, atol=1e-5 * float(ga[:n_emb].abs().max()))
        torch.testing.assert_close(pb, pa, rtol=0, atol=1e-4 * float(pa.abs().max()))


def test_device_sized_forward_capacity_fallback():
    """The device-sized forward (engine.cpp render: interpolation and sdf
    trunk queued before the host reads the query's statistics, sized by the
    sampler's device-side M within a capacity of 1.25 × the largest M seen):
    a batch 4 × larger than the last exceeds the capacity, the queued kernels
    write nothing and the host-sized launch runs instead; the next batch of
    that size fits.  Each step's loss bit for bit against the dense decoder
    (no device-sized forward), gradients as in test_sparse_decoder_matches_dense."""
    from psvo.engine import MappingEngine
    from psvo.octree import map_states
    w, tree, emb0, dec = _setup()
    rgb, depth = w.rgb.reshape(-1, 3).to(DEV), w.depth.reshape(-1).to(DEV)
    crit = {"rgb_weight": 0.5, "depth_weight": 1.0, "sdf_weight": 5000.0, "fs_weight": 10.0}
    sizes = [128, 512, 512, 128]
    runs = {}
    for mode in ("dense", "sparse"):
        eng = MappingEngine(map_states(tree, emb0.clone().to(DEV), 0.2, device=DEV), dec, 0.2, 0.01, truncation=0.1,
                            max_distance=10.0, criteria=crit, max_depth=10.0)
        eng.set_paths(MappingEngine.PATH_DENSE_DECODER if mode == "dense" else 0)
        out = []
        for it, n in enumerate(sizes):
            poses, dirs = _frames_of(w, n)
            pg = torch.zeros(poses.shape[0], 8, device=DEV)
            loss = eng.step_frames(dirs, n, poses.clone(), torch.zeros_like(poses), torch.zeros_like(poses), [0, 1],
                                   1e-3, rgb, depth, seed=900 + it, apply_adam=False, pose_grad=pg, want_loss=True)
            torch.cuda.synchronize()
            out.append((float(loss), list(eng.last_stats), eng.grad_flat.cpu().clone()))
        runs[mode] = out
        eng.close()
    n_emb = emb0.shape[0] * 16
    for (la, sa, ga), (lb, sb, gb) in zip(runs["dense"], runs["sparse"]):
        assert sa[:13] == sb[:13]
        assert la == lb, (la, lb)
        torch.testing.assert_close(gb[n_emb:], ga[n_emb:], rtol=1e-4, atol=1e-5 * float(ga[n_emb:].abs().max()))
        torch.testing.assert_close(gb[:n_emb], ga[:n_emb], rtol=1e-4, atol=1e-5 * float(ga[:n_emb].abs().max()))
    assert runs["sparse"][1][1][4] > 1.25 * runs["sparse"][0][1][4]  # the second batch is beyond the capacity


def test_engine_query_ahead_matches_inline():
    """psvo_map_query (next batch's intersection + sampling on the side stream,
    one step ahead) gives the same iterations as queries inline in the step."""
    from psvo import _lib as L
    from psvo.engine import MappingEngine
    from psvo.octree import map_states
    w, tree, emb0, dec = _setup()
    ro, rd, rgb, dep = (t.reshape(-1, t.shape[-1]) if t.dim() == 3 else t.reshape(-1)
                        for t in (w.rays_o, w.rays_d, w.rgb, w.depth))
    R = ro.shape[0]
    halves = [(ro[s].to(DEV).contiguous(), rd[s].to(DEV).contiguous(), rgb[s].to(DEV).contiguous(),
               dep[s].to(DEV).contiguous()) for s in (slice(0, R // 2), slice(R // 2, R))]
    crit = {"rgb_weight": 0.5, "depth_weight": 1.0, "sdf_weight": 5000.0, "fs_weight": 10.0}
    engines, embs, decs = [], [], []
    for _ in range(2):
        from copy import deepcopy
        d = deepcopy(dec)
        e = emb0.clone().to(DEV)
        engines.append(MappingEngine(map_states(tree, e, 0.2, device=DEV), d, 0.2, 0.01, truncation=0.1,
                                     max_distance=10.0, criteria=crit, max_depth=10.0))
        embs.append(e)
        decs.append(d)
    inline, ahead = engines
    n_it = 5
    la, lb = [], []
    for it in range(n_it):
        b = halves[it % 2]
        la.append(float(inline.step(*b, seed=50 + it)))
    stats_inline = inline.last_stats
    for it in range(n_it):
        b = halves[it % 2]
        if not ahead._queued:
            ahead.query(b[0], b[1], 50 + it)
        if it + 1 < n_it:
            nb = halves[(it + 1) % 2]
            ahead.query(nb[0], nb[1], 50 + it + 1)
        lb.append(float(ahead.step(*b, seed=50 + it)))
    assert ahead.last_stats == stats_inline
    assert la[0] == lb[0]
    np.testing.assert_allclose(lb, la, rtol=1e-4)
    for p, q in zip(decs[0].fused_params(), decs[1].fused_params()):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-4, atol=1e-6)
    # the embedding gradient is a float-atomic scatter whose order depends on
    # what runs beside it (the ahead engine's next query does): after step 1
    # the two differ by that order, amplified where Adam's second moment is tiny
    torch.testing.assert_close(embs[0], embs[1], rtol=1e-4, atol=5e-5)
    # a step whose batch is not the queued one is refused
    ahead.query(halves[0][0], halves[0][1], 7)
    with pytest.raises(RuntimeError):
        ahead.step(*halves[1], seed=7)
    with pytest.raises(RuntimeError, match="differ"):   # same rays, other seed: refused
        ahead.step(*halves[0], seed=8)
    for e in engines:
        e.close()


def test_failed_step_does_not_wedge_the_engine():
    """a queued batch whose step fails (here: no ray hits the
    octree) is consumed by the failed step; the next queued batch steps
    normally, and a step with other rays than the queued ones is refused."""
    from psvo._lib import PsvoError
    from psvo.engine import MappingEngine
    from psvo.octree import map_states
    w, tree, emb0, dec = _setup()
    ms = map_states(tree, emb0.clone().to(DEV), 0.2, device=DEV)
    eng = MappingEngine(ms, dec, 0.2, 0.01)
    ro, rd = w.rays_o.to(DEV), w.rays_d.to(DEV)
    rgb, depth = w.rgb.to(DEV), w.depth.to(DEV)
    miss_o = torch.full_like(ro, -50.0)   # far outside the scene, pointing away
    miss_d = torch.zeros_like(rd)
    miss_d[..., 0] = -1.0
    eng.query(miss_o, miss_d, 1)
    eng.query(ro, rd, 2)
    with pytest.raises(PsvoError, match="no ray hits"):
        eng.step(miss_o, miss_d, rgb, depth, seed=1)
    with pytest.raises(RuntimeError, match="differ"):
        eng.step(ro, rd, rgb, depth, seed=3)  # wrong seed for the queued batch
    loss = float(eng.step(ro, rd, rgb, depth, seed=2))
    assert np.isfinite(loss)
    assert int(eng.last_stats[1]) > 0
    loss2 = float(eng.step(ro, rd, rgb, depth, seed=4))  # nothing queued: fresh query
    assert np.isfinite(loss2)
    eng.close()


def _frames_of(w, n):
    """Keyframe poses [F, 6] and camera-frame directions of a workload's rays
    (world directions rotated back by each pose)."""
    from oracle import oracle as O
    from psvo.pose import OptimizablePose
    poses, dirs = [], []
    rd = w.rays_d[0].double()
    for f, T in enumerate(w.poses):
        p = OptimizablePose.from_matrix(np.asarray(T)).data.detach().double()
        poses.append(p.float())
        dirs.append((rd[f * n:(f + 1) * n] @ O.se3_rotation(p)).float())
    return torch.stack(poses).contiguous().to(DEV), torch.cat(dirs).contiguous().to(DEV)


def test_query_chain_variants_match_padded_path():
    """The mapping step's query / forward chain against the padded path the
    autograd route and the data-parallel step take (PATH_PADDED: k_sample_points
    writes the [R_hit, S_max] z / mask copy, the loss normalisers by
    k_crit_counts → reduce → coef on the aux stream), two
    psvo_map_step_frames iterations stopped before Adam from the same state
    and seeds, every variant:
      default_loss  z read from the sampler's rows (stride max_steps), the
                    ray-major compaction in the sampler's launch, the count chain;
      counts        + PSVO_STEP_NO_LOSS: the normalisers counted by the
                    sampler and turned into coefficients by its look-back scan;
      split         + PATH_QUERY_SPLIT: the statistics / rank pass and the
                    scan (with the counts) as kernels of their own, then
                    k_compact_rays.
    The same statistics, the decoder gradient bit for bit (it depends on the
    forward, the coefficients and the deterministic decoder backward only),
    the embedding gradient up to the scatter's float-atomic order, the pose
    gradient to 1e-5 of its max."""
    from psvo.engine import MappingEngine
    from psvo.octree import map_states
    w, tree, emb0, dec = _setup()
    n = 512
    poses, dirs = _frames_of(w, n)
    rgb, depth = w.rgb.reshape(-1, 3).to(DEV), w.depth.reshape(-1).to(DEV)
    crit = {"rgb_weight": 0.5, "depth_weight": 1.0, "sdf_weight": 5000.0, "fs_weight": 10.0}
    modes = {"padded": (MappingEngine.PATH_PADDED, True), "default_loss": (0, True), "counts": (0, False),
             "split": (MappingEngine.PATH_QUERY_SPLIT, False)}
    runs = {}
    for mode, (paths, want_loss) in modes.items():
        e = emb0.clone().to(DEV)
        eng = MappingEngine(map_states(tree, e, 0.2, device=DEV), dec, 0.2, 0.01, truncation=0.1,
                            max_distance=10.0, criteria=crit, max_depth=10.0)
        eng.set_paths(paths)
        out = []
        for it in range(2):
            pg = torch.zeros(poses.shape[0], 8, device=DEV)
            eng.step_frames(dirs, n, poses.clone(), torch.zeros_like(poses), torch.zeros_like(poses), [0, 1], 1e-3,
                            rgb, depth, seed=500 + it, apply_adam=False, pose_grad=pg, want_loss=want_loss)
            torch.cuda.synchronize()
            out.append((list(eng.last_stats), eng.grad_flat.cpu().clone(), pg.cpu()))
        runs[mode] = out
        eng.close()
    n_emb = emb0.shape[0] * 16
    for mode in modes:
        if mode == "padded":
            continue
        for (sa, ga, pa), (sb, gb, pb) in zip(runs["padded"], runs[mode]):
            assert sa[:13] == sb[:13], (mode, sa, sb)  # statistics (words past 12: zero)
            assert torch.equal(ga[n_emb:], gb[n_emb:]), mode  # decoder gradient: bit for bit
            torch.testing.assert_close(gb[:n_emb], ga[:n_emb], rtol=1e-5, atol=1e-6 * float(ga[:n_emb].abs().max()))
            torch.testing.assert_close(pb, pa, rtol=0, atol=1e-5 * float(pa.abs().max()))


def test_lookback_query_matches_split_kernels():
    """The query's statistics / rank pass and sample scan by decoupled look-
    back inside the traversal and sampler launches (the default) against the
    split kernels (PATH_QUERY_SPLIT: k_ray_stats_rank, k_scan_samples) on
    ragged batches — 1, 3, 5, 257 and 1,001 rays (a partial last workgroup,
    one to 251 workgroups: one to four tiles of 64, a partial last tile), a batch whose
first 600 rays miss the octree (leading workgroups with no hit ray) and
    4,096 rays (16 tiles): the same statistics words, the same loss (bit for bit) and the
    same decoder gradient; the embedding gradient up to the scatter's order."""
    from psvo.engine import MappingEngine
    from psvo.octree import map_states
    w, tree, emb0, dec = _setup()
    ro, rd = w.rays_o.reshape(-1, 3).to(DEV), w.rays_d.reshape(-1, 3).to(DEV)
    rgb, dep = w.rgb.reshape(-1, 3).to(DEV), w.depth.reshape(-1).to(DEV)
    g = torch.Generator().manual_seed(7)
    idx = torch.randint(0, ro.shape[0], (4096,), generator=g).to(DEV)
    ro4, rd4, rgb4, dep4 = ro[idx].contiguous(), rd[idx].contiguous(), rgb[idx].contiguous(), dep[idx].contiguous()
    miss = ro4.clone()
    miss[:600] = -50.0
    rdm = rd4.clone()
    rdm[:600] = torch.tensor([-1.0, 0.0, 0.0], device=DEV)
    batches = [(ro4[:k], rd4[:k], rgb4[:k], dep4[:k]) for k in (1, 3, 5, 257, 1001)]
    batches += [(miss, rdm, rgb4, dep4), (ro4, rd4, rgb4, dep4)]
    crit = {"rgb_weight": 0.5, "depth_weight": 1.0, "sdf_weight": 5000.0, "fs_weight": 10.0}
    runs = {}
    for split in ("0", "1"):
        eng = MappingEngine(map_states(tree, emb0.clone().to(DEV), 0.2, device=DEV), dec, 0.2, 0.01,
                            truncation=0.1, max_distance=10.0, criteria=crit, max_depth=10.0)
        eng.set_paths(MappingEngine.PATH_QUERY_SPLIT if split == "1" else 0)
        out = []
        for i, (o, d, c, z) in enumerate(batches):
            loss = float(eng.step(o.contiguous(), d.contiguous(), c.contiguous(), z.contiguous(), seed=900 + i,
                                  apply_adam=False))
            torch.cuda.synchronize()
            out.append((list(eng.last_stats), loss, eng.grad_flat.cpu().clone()))
        runs[split] = out
        eng.close()
    n_emb = emb0.shape[0] * 16
    for i, ((sa, la, ga), (sb, lb, gb)) in enumerate(zip(runs["1"], runs["0"])):
        assert sa[:13] == sb[:13], (i, sa, sb)
        assert sb[1] > 0, i
        assert la == lb, (i, la, lb)
        assert torch.equal(ga[n_emb:], gb[n_emb:]), i
        torch.testing.assert_close(gb[:n_emb], ga[:n_emb], rtol=1e-5, atol=1e-6 * float(ga[:n_emb].abs().max()))


def test_kernel_bound_region_timing():
    """psvo_engine_set_timing: every region's time is the sum of its kernels'
    own dispatch spans (hipExtLaunchKernel start / stop pairs) — positive for
    the regions the step runs, 0 for one that launched nothing, the query
    regions far below the decoder's, and the same results as an untimed run."""
    from psvo.engine import MappingEngine
    from psvo.octree import map_states
    w, tree, emb0, dec = _setup()
    ro, rd = w.rays_o.to(DEV), w.rays_d.to(DEV)
    rgb, depth = w.rgb.to(DEV), w.depth.to(DEV)
    crit = {"rgb_weight": 0.5, "depth_weight": 1.0, "sdf_weight": 5000.0, "fs_weight": 10.0}
    losses = []
    for timed in (False, "overlap", True):
        from copy import deepcopy
        emb = emb0.clone().to(DEV)
        ms = map_states(tree, emb, 0.2, device=DEV)
        eng = MappingEngine(ms, deepcopy(dec), 0.2, 0.01, truncation=0.1, max_distance=10.0, criteria=crit,
                            max_depth=10.0, lr_emb=5e-3, lr_dec=5e-3)
        if timed:
            eng.set_timing(timed)
        out = [float(eng.step(ro, rd, rgb, depth, seed=300 + it)) for it in range(3)]
        torch.cuda.synchronize()
        losses.append(out)
        if timed:
            t = eng.timing()
            for k in ("intersect", "sample", "interp_fwd", "mlp_fwd", "mlp_bwd"):
                assert t[k] > 0.0 and np.isfinite(t[k]), (k, t)
            assert t["intersect"] < t["mlp_fwd"] and t["sample"] < t["mlp_fwd"], t
            assert t["mlp_fwd"] < 1e3 and t["mlp_bwd"] < 1e3, t  # ms per step: a sane span, not an event mix-up
            eng.set_timing(False)
        eng.close()
    for other in losses[1:]:  # the first loss exactly; later ones up to the embedding scatter's atomic order
        assert other[0] == losses[0][0]
        np.testing.assert_allclose(other, losses[0], rtol=1e-4)
