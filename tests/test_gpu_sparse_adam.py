"""Sparse-exact Adam on the embedding table (include/psvo.h emb_row_flags):
the engine marks the vertex rows its samples touch and steps only the rows
ever touched — an untouched row has g = m = v = 0, which torch's dense Adam
leaves unchanged.  Against the dense step (PSVO_SPARSE_ADAM=0) over three
engine iterations: the decoder bit for bit after the first (then to the
Adam bar), untouched rows bit-identical to
their initial values in both, touched rows to Adam's ulp-amplification bar
(the embedding gradient's float atomics), the flags a superset of the rows
that moved; and flags seeded from a carried-over optimiser state."""
import numpy as np
import pytest
import torch

from test_oracle_golden import adam_close

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("mixed", [False, True])
def test_sparse_adam_equals_dense(monkeypatch, mixed):
    """mixed: the first iteration runs as step(apply_adam=False) + adam() (the
    data-parallel pattern) on keyframe 0's rays only, the next two fused on
    keyframes 1-3 — rows touched only by the first must keep being stepped
    (their moments are non-zero) by the later sparse steps."""
    import test_gpu_fullsize_parity as F
    from psvo.decoder import Decoder
    from psvo.engine import MappingEngine
    c, w, ms, _ = F._setup("B")
    emb0 = ms["voxel_vertex_emb"].detach().clone()
    res = {}
    n1 = w.rays_o.shape[1] // 4
    for flag in ("0", "1"):
        monkeypatch.setenv("PSVO_SPARSE_ADAM", flag)
        torch.manual_seed(0)
        dec = Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none").to(DEV)
        emb = emb0.clone()
        eng = MappingEngine(dict(ms, voxel_vertex_emb=emb), dec, w.scene.voxel_size, c["step"])
        assert (eng.row_flags is not None) == (flag == "1")
        dec1 = None
        for it in range(3):
            if mixed:
                sl = slice(0, n1) if it == 0 else slice(n1, None)
                ro, rd, rgb, dep = (t[:, sl].contiguous().to(DEV) for t in (w.rays_o, w.rays_d, w.rgb, w.depth))
                eng.step(ro, rd, rgb, dep, seed=11 + it, apply_adam=it > 0)
                if it == 0:
                    eng.adam()
            else:
                eng.step(w.rays_o.to(DEV), w.rays_d.to(DEV), w.rgb.to(DEV), w.depth.to(DEV), seed=11 + it)
            if it == 0:  # the first update does not depend on the float-atomic embedding gradient
                dec1 = [p.detach().cpu().clone() for p in dec.parameters()]
        torch.cuda.synchronize()
        res[flag] = (emb.cpu(), dec1, eng.row_flags.cpu() if eng.row_flags is not None else None, eng.emb_m.cpu(),
                     [p.detach().cpu() for p in dec.parameters()])
        eng.close()
    (e_d, dec_d, _, m_d, d3_d), (e_s, dec_s, flags, m_s, d3_s) = res["0"], res["1"]
    assert all(torch.equal(a, b) for a, b in zip(dec_d, dec_s))
    for a, b in zip(d3_s, d3_d):
        adam_close(a.numpy(), b.numpy(), tight=1e-4, frac=0.99, max_abs=2.0 * 5e-3 * 3)
    e0 = emb0.cpu()
    moved = (e_d != e0).any(-1) | (e_s != e0).any(-1)
    live = (m_d != 0).any(-1)
    assert bool(moved.any()) and int(flags.sum()) < flags.numel()  # a real subset of the table
    assert bool(flags[moved].all()) and bool(flags[live].all())     # every row that moved / has moments is flagged
    assert torch.equal(e_s[~flags.bool()], e0[~flags.bool()])      # the rest is untouched ...
    assert torch.equal(e_d[~flags.bool()], e0[~flags.bool()])      # ... as the dense step leaves it
    rows = flags.bool()
    adam_close(e_s[rows].numpy(), e_d[rows].numpy(), tight=1e-5, frac=0.97, max_abs=2.0 * 5e-3 * 3)


def test_flags_from_carried_state():
    from psvo import _lib as L
    n = 5000
    g = torch.Generator().manual_seed(1)
    m = torch.zeros(n, 16)
    v = torch.zeros(n, 16)
    live = torch.randperm(n, generator=g)[:700]
    m[live[:400], 3] = 1e-3
    v[live[400:], 15] = 1e-6
    flags = torch.zeros(n, dtype=torch.uint8, device=DEV)
    flags[7] = 1  # already set: kept
    L.call("psvo_adam_flags_from_state", L.stream_of(flags.device), n, m.to(DEV), v.to(DEV), flags)
    torch.cuda.synchronize()
    want = torch.zeros(n, dtype=torch.uint8)
    want[live] = 1
    want[7] = 1
    assert torch.equal(flags.cpu(), want)


def test_one_rank_unforced_exchange_steps_every_row():
    """An exchange set on ONE rank without force (torchrun with one process,
    or a caller's own all-reduce): the step marks only its local flags and the
    gradient exchange returns early without marking the union, so Adam must
    not be row-sparse on the stale union flags (psvo_map_adam_ex: dense, then
    the flags refreshed from the moments).  Three iterations against the
    plain single-GPU engine: the same rows move, to Adam's ulp bar, and the
    union flags cover every row with moments."""
    import test_gpu_fullsize_parity as F
    from psvo.decoder import Decoder
    from psvo.dist import EngineExchange
    from psvo.engine import MappingEngine
    c, w, ms, _ = F._setup("B")
    emb0 = ms["voxel_vertex_emb"].detach().clone()
    res = {}
    for mode in ("plain", "exchange"):
        torch.manual_seed(0)
        dec = Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none").to(DEV)
        emb = emb0.clone()
        eng = MappingEngine(dict(ms, voxel_vertex_emb=emb), dec, w.scene.voxel_size, c["step"])
        if mode == "exchange":
            eng.set_exchange(EngineExchange(w.rays_o.shape[1], device=DEV))  # no process group: world 1
        args = (w.rays_o.to(DEV), w.rays_d.to(DEV), w.rgb.to(DEV), w.depth.to(DEV))
        for it in range(3):
            if mode == "exchange":
                eng.step(*args, seed=11 + it, apply_adam=False)
                eng.grad_exchange()
                eng.adam()
            else:
                eng.step(*args, seed=11 + it)
        torch.cuda.synchronize()
        res[mode] = (emb.cpu(), eng.row_flags.cpu(), eng.emb_m.cpu())
        eng.close()
    (e_p, f_p, m_p), (e_x, f_x, m_x) = res["plain"], res["exchange"]
    e0 = emb0.cpu()
    moved_p, moved_x = (e_p != e0).any(-1), (e_x != e0).any(-1)
    assert int(moved_p.sum()) > 100 and torch.equal(moved_p, moved_x)
    assert bool(f_x[(m_x != 0).any(-1)].all())  # every row with moments is flagged for later sparse steps
    adam_close(e_x[moved_p].numpy(), e_p[moved_p].numpy(), tight=1e-5, frac=0.97, max_abs=2.0 * 5e-3 * 3)
