"""CPU checks of the data-parallel engine's exchange protocol (include/psvo.h
psvo_engine_set_exchange; csrc/svo_query.hip k_dist_*).

1. Sufficiency: a rank samples its rows of the union batch's [200, K', P]
   layout from its own hit lists plus (a) the slot-0 rows' hit COUNTS (their
   voxel ids are read only as "== -1", and a row's hits are its prefix) and
   (b) the first voxel id of the row after its last — nothing else of other
   ranks' rows.  Checked with the oracle sampler (sample_gpu.cu:133-239
   restated): poisoning every other row — slot-0 rows down to junk ids over
   their hit prefix — except (b) leaves the shard's samples bit-identical.
2. psvo.dist.EngineExchange.apply over gloo, world size 2: all-gather and
   in-place sums on the exchange buffers, as the engine calls them."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O

G = 200


def _hits(n, p, rng, full_frac=0.3):
    idx = np.full((n, p), -1, np.int32)
    lo = np.full((n, p), 10.0, np.float32)
    hi = np.full((n, p), 10.0, np.float32)
    for r in range(n):
        nb = p if rng.random() < full_frac else int(rng.integers(1, p + 1))  # many rays with exactly P bins
        t = 0.5
        for h in range(nb):
            a = t + rng.uniform(0.0, 0.2)
            w = rng.uniform(0.01, 0.3)
            idx[r, h], lo[r, h], hi[r, h] = rng.integers(0, 5000), a, a + w
            t = a + w
    return idx, lo, hi


def _sample(idx, lo, hi, step, noise):
    """Oracle sampler over the whole logical layout (rows already padded to H)."""
    n, p = idx.shape
    d = np.where(idx >= 0, hi - lo, 0).astype(np.float32)
    s = d.sum(-1, keepdims=True, dtype=np.float32)
    probs = (d / np.where(s > 0, s, 1)).astype(np.float32)
    steps = (s[:, 0] / np.float32(step)).astype(np.float32)
    kp = n // G
    ms = noise.shape[-1]
    o_idx = np.full((G, kp, ms), -1, np.int32)
    o_dep = np.zeros((G, kp, ms), np.float32)
    o_dis = np.zeros((G, kp, ms), np.float32)
    r = lambda a: np.ascontiguousarray(a.reshape((G, kp) + a.shape[1:]))
    O.lib().oracle_inverse_cdf(G, kp, p, ms, -1.0, *(O._ptr(a) for a in (r(idx), r(lo), r(hi), noise, r(probs),
                                                                          r(steps), o_idx, o_dep, o_dis)))
    return o_idx.reshape(n, ms), o_dep.reshape(n, ms), o_dis.reshape(n, ms)


@pytest.mark.parametrize("step", [0.02, 0.4])  # many samples per bin / fewer samples than bins
@pytest.mark.parametrize("n,cuts", [(1400, [0, 611, 1400]), (8000, [0, 1, 41, 4001, 4082, 7993, 8000]),
                                    (7400, [0, 2467, 4934, 7400])])
def test_slot0_table_and_next_col0_suffice(n, cuts, step):
    """The trailing-segment quirk (sample_gpu.cu:224-237) reads slot 0's ids
    when a ray has fewer samples than bins, and the next row's first id when
    a ray has exactly P bins and its samples pass the last bin: rows whose
    block slot j < K'/P.  Shard ends are placed at such slots."""
    rng = np.random.default_rng(n + len(cuts))
    p = 6
    idx, lo, hi = _hits(n, p, rng, full_frac=0.7)
    kp = (n + G - 1) // G
    H = kp * G
    pad = lambda a: np.concatenate([a, np.repeat(a[:1], H - n, 0)], 0)  # voxel_helpers.py:303-310
    idx, lo, hi = pad(idx), pad(lo), pad(hi)
    d = np.where(idx >= 0, hi - lo, 0).astype(np.float32)
    ms = int(np.ceil(d.sum(-1, dtype=np.float32) / np.float32(step)).max()) + p
    noise = rng.uniform(0.001, 0.999, size=(G, kp, ms)).astype(np.float32)
    want = _sample(idx, lo, hi, step, noise)
    slot0_rows = {b * kp for b in range(G)}  # chunk 0 only: kp < 800
    for a, b in zip(cuts[:-1], cuts[1:]):
        # this rank's view: its rows, the slot-0 rows' hit counts (k_dist_layout's
        # table), the next row's first voxel id (next_col0); all else junk
        pi, pl, ph = idx.copy(), lo.copy(), hi.copy()
        other = np.ones(H, bool)
        other[a:b] = False
        junk = np.where(rng.random((H, p)) < 0.5, -1, rng.integers(0, 5000, size=(H, p))).astype(np.int32)
        jl = rng.uniform(0, 3, size=(H, p)).astype(np.float32)
        keep_idx = np.zeros((H, p), bool)
        keep_idx[b if b < H else 0, 0] = True
        sel = other[:, None] & ~keep_idx
        pi[sel] = junk[sel]
        for r in slot0_rows:  # only the count survives: other junk ids over the hit prefix, -1 after
            if other[r]:
                nv = int((idx[r] != -1).sum())
                pi[r] = -1
                pi[r, :nv] = rng.integers(0, 5000, size=nv) + 7
                if keep_idx[r, 0]:  # also the row after the shard: its first id (next_col0)
                    pi[r, 0] = idx[r, 0]
        pl[other] = jl[other]
        ph[other] = jl[other] + 0.05
        got = _sample(pi, pl, ph, step, noise)
        for w, g_ in zip(want, got):
            np.testing.assert_array_equal(g_[a:b], w[a:b])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _xch_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from psvo.dist import XCH_GATHER_I32, XCH_QUERY, XCH_SUM_F64, XCH_SUM_I32, EngineExchange
        x = EngineExchange(max_rays_global=4096)
        xi, xf = x.buffers(64)
        xi[0:8] = torch.arange(8, dtype=torch.int32) + 100 * rank
        x.apply(XCH_GATHER_I32 | XCH_QUERY, 0, 8, 8)
        xi[40:50] = rank + 1
        x.apply(XCH_SUM_I32 | XCH_QUERY, 40, 40, 10)
        xf[:] = torch.arange(16, dtype=torch.float64) * (rank + 1)
        x.apply(XCH_SUM_F64, 8, 8, 8)
        q.put((rank, xi.numpy().copy(), xf.numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_engine_exchange_apply_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_xch_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for pr in procs:
        pr.join(timeout=300)  # gloo teardown can be slow on a loaded host
        assert pr.exitcode == 0
    for rank, xi, xf in res:
        np.testing.assert_array_equal(xi[8:24], np.concatenate([np.arange(8), np.arange(8) + 100]))
        np.testing.assert_array_equal(xi[40:50], np.full(10, 3))
        np.testing.assert_array_equal(xf[:8], np.arange(8) * (rank + 1))  # untouched half
        np.testing.assert_array_equal(xf[8:], np.arange(8, 16) * 3.0)


def test_forced_exchange_needs_process_group():
    """force=True runs every collective even on one rank: without an
    initialised process group that must fail here, not inside a step's
    ctypes callback."""
    from psvo.dist import EngineExchange
    assert not (dist.is_available() and dist.is_initialized())
    with pytest.raises(RuntimeError, match="process group"):
        EngineExchange(max_rays_global=64, force=True)
    assert EngineExchange(max_rays_global=64).world == 1
