"""The data-parallel engine's union-batch protocol at world 8, on the CPU over
gloo: eight ranks hold uneven shards of one batch's hit
rays — one shard EMPTY, cuts on the sampler's slot-0 rows — and run the
protocol the engine runs (include/psvo.h psvo_engine_set_exchange,
csrc/engine.cpp query_enqueue / map_step_impl) through
psvo.dist.EngineExchange.apply on the engine's exchange-buffer layout:

  1. ONE all-gather of the 8 statistics words + a hit-count byte per hit row
     (k_dist_pack, restated below);
  2. on every rank, the union layout (k_dist_layout: P, R_hit, max ⌈Σ/step⌉,
     the rank's first row, the first voxel id of the row after its last) and
     the [200·nch] slot-0 count table from the gathered bytes;
  3. each rank samples only its own rows of the union's [200, K', P] sampler
     layout (the oracle sampler, sample_gpu.cu:133-239), every other row of
     its view poisoned — slot-0 rows keep only their hit count — and
     next_col0;
  4. ONE all-gather of [S_max, 7 count words] (k_dist_counts / k_dist_smax):
     the union S_max and the Criterion's normaliser counts over the union's
     padded [R_hit, S_max] layout (criterion.py:70-101), the padding applied
     after the gather;
  5. the loss sums all-reduced (f64), and the decoder-stand-in's gradients
     summed over ranks.

Against one process on the concatenated batch: the same P, R_hit, S_max, M,
every rank's sample ids / depths bit-identical to its rows of the single
run, the loss to 1e-6, the summed gradients to 1e-5 — on every rank.  The
layout's word offsets are checked against psvo_engine_exchange_words."""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O

G, P, WORLD = 200, 6, 8
N_RAYS = 7400                     # K' = 37: slot-0 rows at multiples of 37
STEP = 0.4  # fewer samples than bins on many rays: the trailing segment reads slot 0 (sample_gpu.cu:224-237)
# rank 2 empty; every other shard starts at slot 1-6 of a sampler block whose
# slot-0 row the previous rank holds: its rays' trailing segments read that
# row's ids from the exchanged table (sample_gpu.cu:224-237, slots j·P + bin < K')
CUTS = [0, 37 * 3 + 1, 37 * 30 + 2, 37 * 30 + 2, 37 * 66 + 3, 37 * 133 + 4, 37 * 135 + 5, 37 * 189 + 6, 7400]
TR, MAX_D = 0.05, 5.0
assert len(CUTS) == WORLD + 1


def _batch():
    """The union batch's hit rays [N, P] (sorted, -1 / 10 fills), noise, GT."""
    rng = np.random.default_rng(1234)
    idx = np.full((N_RAYS, P), -1, np.int32)
    lo = np.full((N_RAYS, P), 10.0, np.float32)
    hi = np.full((N_RAYS, P), 10.0, np.float32)
    for r in range(N_RAYS):
        nb = P if rng.random() < 0.3 else int(rng.integers(1, P + 1))
        t = 0.5
        for h in range(nb):
            a = t + rng.uniform(0.0, 0.2)
            w = rng.uniform(0.01, 0.3)
            idx[r, h], lo[r, h], hi[r, h] = rng.integers(0, 5000), a, a + w
            t = a + w
    kp = (N_RAYS + G - 1) // G
    d = np.where(idx >= 0, hi - lo, 0).astype(np.float32)
    max_ceil = int(np.ceil(_row_sums(d) / np.float32(STEP)).max())
    noise = rng.uniform(0.001, 0.999, size=(G, kp, max_ceil + P)).astype(np.float32)
    gt_rgb = rng.uniform(0, 1, size=(N_RAYS, 3)).astype(np.float32)
    gt_d = rng.uniform(0.3, 4.0, size=N_RAYS).astype(np.float32)
    return idx, lo, hi, noise, gt_rgb, gt_d


def _row_sums(d):
    """Σ over a row left to right in f32 (k_intersect_sorted's dsum order)."""
    acc = np.zeros(d.shape[0], np.float32)
    for k in range(d.shape[1]):
        acc = (acc + d[:, k]).astype(np.float32)
    return acc


def _sample(idx, lo, hi, noise):
    """The oracle sampler over the whole logical layout (voxel_helpers.py:288-374
    padding to H rows with copies of row 0)."""
    n = idx.shape[0]
    kp = (n + G - 1) // G
    H = kp * G
    pad = lambda a: np.concatenate([a, np.repeat(a[:1], H - n, 0)], 0)  # noqa: E731
    idx, lo, hi = pad(idx), pad(lo), pad(hi)
    d = np.where(idx >= 0, hi - lo, 0).astype(np.float32)
    s = _row_sums(d)[:, None]
    probs = (d / np.where(s > 0, s, 1)).astype(np.float32)
    steps = (s[:, 0] / np.float32(STEP)).astype(np.float32)
    ms = noise.shape[-1]
    o_idx = np.full((G, kp, ms), -1, np.int32)
    o_dep = np.zeros((G, kp, ms), np.float32)
    o_dis = np.zeros((G, kp, ms), np.float32)
    r = lambda a: np.ascontiguousarray(a.reshape((G, kp) + a.shape[1:]))  # noqa: E731
    O.lib().oracle_inverse_cdf(G, kp, P, ms, -1.0, *(O._ptr(a) for a in (r(idx), r(lo), r(hi), noise, r(probs),
                                                                          r(steps), o_idx, o_dep, o_dis)))
    return o_idx.reshape(H, ms)[:n], o_dep.reshape(H, ms)[:n]


def _model():
    torch.manual_seed(5)
    return torch.nn.Linear(6, 4).double()


def _render_loss(model, s_idx, s_dep, gt_rgb, gt_d, s_cols):
    """A decoder stand-in on each valid sample (features from its voxel id and
    depth), softmax compositing over the ray's valid samples, and the
    Criterion's eight partial sums over the ray rows padded to s_cols columns
    (z = 10, sdf = 1 past the valid samples, as the engine pads them)."""
    n, s_loc = s_idx.shape
    valid = torch.from_numpy(s_idx != -1)
    z = torch.from_numpy(s_dep).double()
    z = torch.where(valid, z, torch.full_like(z, 10.0))
    vid = torch.from_numpy(s_idx).double()
    feats = torch.stack([torch.sin(vid * 0.37 + z), torch.cos(vid * 0.11 - z), z, torch.sin(3.0 * z),
                         torch.cos(vid * 0.05), torch.ones_like(z)], -1)
    out = model(feats)
    sdf = torch.where(valid, out[..., 0], torch.ones_like(z))
    w = torch.softmax(torch.where(valid, -sdf.abs(), torch.full_like(z, -1e4)), dim=1)
    color = (w.unsqueeze(-1) * torch.sigmoid(out[..., 1:])).sum(1)
    depth = (w * z).sum(1)
    return O.criterion_sums(color, depth, sdf, z, torch.from_numpy(gt_rgb).double(),
                            torch.from_numpy(gt_d).double(), TR, MAX_D, pad_extra=s_cols - s_loc)


def _layout(world, n_rays, n_rank=None):
    """EngineExchange's int32 word offsets (csrc/engine.cpp struct EngineExchange)."""
    cw = 8 + ((n_rank if n_rank else n_rays) + 3) // 4  # 8 words + a hit-count byte per ray of the shard
    q2_in = cw + world * cw
    q2_all = q2_in + 8
    table_off = (q2_all + world * 8 + 63) // 64 * 64
    kp = (n_rays + G - 1) // G
    nch = (kp + 799) // 800
    return dict(cw=cw, all=cw, q2_in=q2_in, q2_all=q2_all, table=table_off, nch=nch, words=table_off + G * nch)


def _pad_terms(d):
    """Per ray: does the MAX_DEPTH padding (z = 10) count as front / as in the
    sdf band (criterion.py:78-88 on the padded columns)."""
    zp = 10.0
    fp = zp < d - TR
    bp = zp > d + TR
    smp = ~fp & ~bp & (d > 0.0) & (d < MAX_D)
    return fp, smp


def _single():
    idx, lo, hi, noise, gt_rgb, gt_d = _batch()
    s_idx, s_dep = _sample(idx, lo, hi, noise)
    ns = (s_idx != -1).sum(1)
    s_max = int(ns.max())
    model = _model()
    sums = _render_loss(model, s_idx[:, :s_max], s_dep[:, :s_max], gt_rgb, gt_d, s_max)
    loss, _ = O.criterion_from_sums(sums, N_RAYS, s_max, O.REPLICA_CRITERIA)
    loss.backward()
    d = np.where(idx >= 0, hi - lo, 0).astype(np.float32)
    return dict(P=int((idx != -1).sum(1).max()), r_hit=N_RAYS, s_max=s_max, m=int(ns.sum()),
                max_ceil=int(np.ceil(_row_sums(d) / np.float32(STEP)).max()), s_idx=s_idx, s_dep=s_dep,
                loss=float(loss.detach()), grads=[p.grad.clone() for p in model.parameters()])


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from psvo.dist import XCH_GATHER_I32, XCH_QUERY, XCH_SUM_F64, EngineExchange, GradBucket
        idx, lo, hi, noise, gt_rgb, gt_d = _batch()
        a, b = CUTS[rank], CUTS[rank + 1]
        n_loc = b - a
        lay = _layout(world, N_RAYS)
        x = EngineExchange(max_rays_global=N_RAYS)
        xi, xf = x.buffers(lay["words"])
        assert x.max_rays_rank == N_RAYS
        # 1. this rank's words (k_dist_pack): R_hit, P, max ceil, first voxel id of its first row, flags,
        #    then a byte per hit row: its hit count — ONE all-gather
        d_loc = np.where(idx[a:b] >= 0, hi[a:b] - lo[a:b], 0).astype(np.float32)
        nv_loc = (idx[a:b] != -1).sum(1).astype(np.uint32)
        p_loc = int(nv_loc.max()) if n_loc else 0
        mc_loc = int(np.ceil(_row_sums(d_loc) / np.float32(STEP)).max()) if n_loc else 0
        cw = lay["cw"]
        xi[0:8] = torch.tensor([n_loc, p_loc, mc_loc, int(idx[a, 0]) if n_loc else -1, 0, 0, 0, 0],
                               dtype=torch.int32)
        packed = np.zeros(4 * (cw - 8), np.uint32)
        packed[:n_loc] = nv_loc
        packed = packed.reshape(-1, 4)
        words_nv = packed[:, 0] | (packed[:, 1] << 8) | (packed[:, 2] << 16) | (packed[:, 3] << 24)
        xi[8:cw] = torch.from_numpy(words_nv.view(np.int32))
        x.apply(XCH_GATHER_I32 | XCH_QUERY, 0, lay["all"], cw)
        gathered = xi[lay["all"]:lay["all"] + cw * world].view(world, cw).numpy()
        words = gathered[:, :8]
        # 2. union layout (k_dist_layout), on every rank from the gathered words alone
        r_hit = int(words[:, 0].sum())
        p_all = int(words[:, 1].max())
        mc_all = int(words[:, 2].max())
        begin = int(words[:rank, 0].sum())
        order = [r for r in range(rank + 1, world) if words[r, 0] > 0] + [r for r in range(world) if words[r, 0] > 0]
        next_col0 = int(words[order[0], 3]) if order else -1
        assert begin == a
        #    the slot-0 count table: row (blk, c) = hit count of logical row blk·K' + c·800 (its owner's byte)
        kp = (r_hit + G - 1) // G
        nch = lay["nch"]
        begins = np.concatenate([[0], np.cumsum(words[:, 0])])
        nv_bytes = gathered[:, 8:].view(np.uint32)
        table = np.zeros(G * nch, np.int64)
        for blk in range(G):
            for c in range(nch):
                lrow = blk * kp + c * 800
                lrow = lrow if lrow < r_hit else 0
                o = int(np.searchsorted(begins, lrow, side="right") - 1)
                j = lrow - int(begins[o])
                table[blk * nch + c] = (int(nv_bytes[o, j >> 2]) >> (8 * (j & 3))) & 0xFF
                assert table[blk * nch + c] == int((idx[lrow] != -1).sum())
        # 3. sample this rank's rows from its own hits + the table + next_col0; everything else poisoned
        rng = np.random.default_rng(77 + rank)
        v_idx = rng.integers(0, 5000, size=idx.shape).astype(np.int32)
        v_idx[rng.random(idx.shape) < 0.4] = -1
        v_lo = rng.uniform(0, 3, size=lo.shape).astype(np.float32)
        v_hi = (v_lo + 0.05).astype(np.float32)
        v_idx[a:b], v_lo[a:b], v_hi[a:b] = idx[a:b], lo[a:b], hi[a:b]
        for blk in range(G):
            for c in range(nch):
                lrow = blk * kp + c * 800
                if lrow < r_hit and not (a <= lrow < b):  # only the hit count survives: junk ids, then -1
                    nv = int(table[blk * nch + c])
                    v_idx[lrow] = -1
                    v_idx[lrow, :nv] = rng.integers(0, 5000, size=nv)
        if n_loc and b < r_hit:
            v_idx[b, 0] = next_col0
        elif n_loc:  # past the union's last row: the reference pads with copies of row 0
            v_idx[0, 0] = next_col0
        s_idx, s_dep = _sample(v_idx, v_lo, v_hi, noise)
        s_idx, s_dep = s_idx[a:b], s_dep[a:b]
        ns = (s_idx != -1).sum(1)
        s_loc = int(ns.max()) if n_loc else 0
        # 4. [S_max, counts] — ONE all-gather (k_dist_counts / k_dist_smax): the valid samples' counts and,
        #    per padding class, the rays and their Σ ns; the union S_max applied to the padding afterwards
        d = gt_d[a:b].astype(np.float64)
        valid_s = s_idx != -1
        z = s_dep.astype(np.float64)
        front = valid_s & (z < (d - TR)[:, None])
        back = valid_s & (z > (d + TR)[:, None])
        band = valid_s & ~front & ~back & ((d > 0.0) & (d < MAX_D))[:, None]
        fp, smp = _pad_terms(d)
        xi[lay["q2_in"]:lay["q2_in"] + 8] = torch.tensor(
            [s_loc, int(((d > 0.01) & (d < MAX_D)).sum()), int(front.sum()), int(band.sum()), int(fp.sum()),
             int(ns[fp].sum()), int(smp.sum()), int(ns[smp].sum())], dtype=torch.int32)
        x.apply(XCH_GATHER_I32 | XCH_QUERY, lay["q2_in"], lay["q2_all"], 8)
        g2 = xi[lay["q2_all"]:lay["q2_all"] + 8 * world].view(world, 8).numpy().astype(np.int64)
        s_max = int(g2[:, 0].max())
        c = g2[:, 1:].sum(0)
        counts = (float(c[0]), float(c[1] + s_max * c[3] - c[4]), float(c[2] + s_max * c[5] - c[6]))
        # 5. loss sums all-reduced (f64), the loss of the union; gradients summed over ranks
        model = _model()
        sums = _render_loss(model, s_idx[:, :s_loc], s_dep[:, :s_loc], gt_rgb[a:b], gt_d[a:b], s_max)
        xf[8:16] = sums.detach()  # the engine's loss half at offset 8
        x.apply(XCH_SUM_F64, 8, 8, 8)
        assert counts == tuple(float(v) for v in xf[10:13]), (counts, xf[10:13])  # n_valid, n_front, n_sdf
        sums_g = sums + (xf[8:16] - sums).detach()  # global values, local gradient paths
        loss, _ = O.criterion_from_sums(sums_g, r_hit, s_max, O.REPLICA_CRITERIA)
        loss.backward()
        GradBucket(model.parameters(), op="sum").allreduce()
        q.put((rank, dict(P=p_all, r_hit=r_hit, max_ceil=mc_all, s_max=s_max, m=int(ns.sum()), s_idx=s_idx,
                          s_dep=s_dep, loss=float(loss), grads=[p.grad.numpy().copy() for p in model.parameters()])))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_layout_matches_engine_exchange_words():
    from psvo import _lib as L
    for world, n, nr in ((1, 4096, 0), (2, 8192, 4096), (8, N_RAYS, 0), (8, 32768, 4096), (8, 200 * 800 + 1, 0),
                         (3, 1400, 789)):
        assert int(L.lib().psvo_engine_exchange_words(world, n, nr)) == _layout(world, n, nr)["words"]
    assert int(L.lib().psvo_engine_exchange_words(2, 100, 101)) == -1  # a shard larger than the union


def test_union_protocol_world8_equals_one_process():
    ref = _single()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=300) for _ in range(WORLD)], key=lambda t: t[0])
    for pr in procs:
        pr.join(timeout=300)
        assert pr.exitcode == 0
    assert CUTS[3] == CUTS[2]  # rank 2 holds no rays
    m_total = 0
    for rank, r in res:
        a, b = CUTS[rank], CUTS[rank + 1]
        assert (r["P"], r["r_hit"], r["max_ceil"], r["s_max"]) == (ref["P"], ref["r_hit"], ref["max_ceil"],
                                                                   ref["s_max"]), rank
        n = r["s_idx"].shape[1]
        np.testing.assert_array_equal(r["s_idx"], ref["s_idx"][a:b, :n])
        np.testing.assert_array_equal(r["s_dep"], ref["s_dep"][a:b, :n])
        assert (ref["s_idx"][a:b, n:] == -1).all()
        m_total += r["m"]
        assert abs(r["loss"] - ref["loss"]) <= 1e-6 * abs(ref["loss"]), (rank, r["loss"], ref["loss"])
        for g, gr in zip(r["grads"], ref["grads"]):
            torch.testing.assert_close(torch.from_numpy(g), gr, rtol=1e-5, atol=1e-9 * float(gr.abs().max()))
    assert m_total == ref["m"]
    # replicas identical
    for _, r in res[1:]:
        assert all(np.array_equal(g, h) for g, h in zip(r["grads"], res[0][1]["grads"]))
