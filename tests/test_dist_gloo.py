"""Data-parallel path on CPU (gloo, world_size 2): psvo.dist.GlobalLossSums
makes the sharded loss equal the single-process loss of the concatenated
batch (criterion.py's batch-global normalisers, padded to the global S_max),
and psvo.dist.GradBucket's one flat all-reduce makes the per-rank decoder
gradients sum to the single-process gradients."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O

R_HIT, S_MAX, TR, MAX_D = 96, 40, 0.05, 5.0


def _batch(seed=0):
    g = torch.Generator().manual_seed(seed)
    feats = torch.randn(R_HIT, S_MAX, 8, generator=g)
    ns = torch.randint(5, S_MAX + 1, (R_HIT,), generator=g)
    ns[:R_HIT // 2] = torch.clamp(ns[:R_HIT // 2], max=25)  # shard 0 has a smaller S_max
    z = torch.sort(torch.rand(R_HIT, S_MAX, generator=g) * 6, dim=1).values
    valid = torch.arange(S_MAX)[None, :] < ns[:, None]
    z = torch.where(valid, z, torch.full_like(z, 10.0))
    gt_rgb = torch.rand(R_HIT, 3, generator=g)
    gt_d = torch.rand(R_HIT, generator=g) * 5.5
    return feats, valid, z, gt_rgb, gt_d, ns


def _model():
    torch.manual_seed(1)
    return torch.nn.Linear(8, 4)


def _render(model, feats, valid, z):
    out = model(feats)
    sdf = torch.where(valid, out[..., 0], torch.ones_like(z))
    w = torch.softmax(torch.where(valid, -sdf.abs(), torch.full_like(z, -1e4)), dim=1)
    color = (w.unsqueeze(-1) * torch.sigmoid(out[..., 1:])).sum(1)
    depth = (w * z).sum(1)
    return color, depth, sdf


def _single():
    feats, valid, z, gt_rgb, gt_d, _ = _batch()
    model = _model()
    color, depth, sdf = _render(model, feats, valid, z)
    out = {"ray_mask": torch.ones(R_HIT, dtype=torch.bool), "z_vals": z, "sdf": sdf, "color": color, "depth": depth}
    loss, _ = O.criterion(out, gt_rgb, gt_d, O.REPLICA_CRITERIA, TR, MAX_D)
    loss.backward()
    return loss.detach(), [p.grad.clone() for p in model.parameters()]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from psvo.dist import GlobalLossSums, GradBucket, shard
        feats, valid, z, gt_rgb, gt_d, ns = _batch()
        b, e = shard(R_HIT, rank, world)
        s_loc = int(ns[b:e].max())  # this shard's own S_max
        feats, valid, z = feats[b:e, :s_loc], valid[b:e, :s_loc], z[b:e, :s_loc]
        model = _model()
        color, depth, sdf = _render(model, feats, valid, z)
        red = GlobalLossSums()
        n_hit, s_cols = red.global_shape(e - b, s_loc)
        sums = O.criterion_sums(color, depth, sdf, z, gt_rgb[b:e], gt_d[b:e], TR, MAX_D, pad_extra=s_cols - s_loc)
        tot = sums.detach().double().clone()
        red(tot)
        sums_g = sums + (tot.to(sums.dtype) - sums).detach()  # global values, local gradient paths
        loss, _ = O.criterion_from_sums(sums_g, n_hit, s_cols, O.REPLICA_CRITERIA)
        loss.backward()
        GradBucket(model.parameters(), op="sum").allreduce()
        # by value (numpy): tensors would travel as shared fds the exiting worker may close first
        q.put((rank, float(loss.detach()), n_hit, s_cols, [p.grad.numpy().copy() for p in model.parameters()]))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharded_global_loss_and_grad_bucket_match_single_process():
    loss1, grads1 = _single()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=300)  # gloo teardown can be slow on a loaded host
        assert p.exitcode == 0
    for rank, loss, n_hit, s_cols, grads in res:
        assert (n_hit, s_cols) == (R_HIT, S_MAX)
        assert abs(loss - float(loss1)) <= 1e-5 * abs(float(loss1))
        for a, b in zip(grads, grads1):
            torch.testing.assert_close(torch.from_numpy(a), b, rtol=1e-4, atol=1e-6 * float(b.abs().max()))
    # replicas stay identical
    for a, b in zip(res[0][4], res[1][4]):
        assert torch.equal(torch.from_numpy(a), torch.from_numpy(b))


class _TorchRowOps:
    """Test-only stand-in for psvo_rows_compact / psvo_rows_scatter_add on CPU
    tensors, to check SparseRowSum's exchange protocol over gloo (the device
    kernels themselves are checked in tests/test_gpu_rows.py)."""

    def workspace_ints(self, n_rows):
        return 1

    def compact(self, grad2d, ids, rows, count, workspace):
        nz = (grad2d != 0).any(1).nonzero().flatten()
        ids[: nz.numel()] = nz.to(torch.int32)
        rows[: nz.numel()] = grad2d[nz]
        count[0] = nz.numel()

    def scatter_add(self, ids, rows, grad2d):
        keep = ids >= 0
        grad2d[ids[keep].long()] += rows[keep]

    def compact_flagged(self, grad2d, flags, ids, rows, count, workspace):
        nz = (flags != 0).nonzero().flatten()
        ids[: nz.numel()] = nz.to(torch.int32)
        rows[: nz.numel()] = grad2d[nz]
        count[0] = nz.numel()

    def clear(self, ids, grad2d, flags):
        keep = ids[ids >= 0].long()
        grad2d[keep] = 0
        if flags is not None:
            flags[keep] = 0

    def mark(self, ids, flags):
        flags[ids[ids >= 0].long()] = 1

    def flags_from_grad(self, grad2d, flags):
        flags[(grad2d != 0).any(1)] = 1


def _sparse_grad(rank, n_rows, touched, seed):
    g = torch.Generator().manual_seed(seed + rank)
    grad = torch.zeros(n_rows, 16)
    idx = torch.randperm(n_rows, generator=g)[:touched]
    grad[idx] = torch.randn(touched, 16, generator=g)
    return grad


def _sparse_worker(rank, world, port, q, n_rows, touched):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from psvo.dist import SparseRowSum
        grad = _sparse_grad(rank, n_rows, touched, 7)
        mode = SparseRowSum(n_rows, 16, "cpu", ops=_TorchRowOps())(grad)
        q.put((rank, mode, grad.numpy().copy()))  # by value: the worker may exit before the get
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("touched,expect", [(40, "sparse"), (0, "sparse"), (900, "dense")])
def test_sparse_row_sum_protocol(touched, expect):
    """Row-sparse exchange (config E data parallelism): every rank ends with
    the sum of all ranks' gradients, bit-identical across ranks; the dense
    fallback when the lists would outweigh the table."""
    n_rows, world = 1000, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sparse_worker, args=(r, world, port, q, n_rows, touched)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=300)  # gloo teardown can be slow on a loaded host
        assert p.exitcode == 0
    want = sum(_sparse_grad(r, n_rows, touched, 7) for r in range(world))
    got = [torch.from_numpy(r[2]) for r in res]
    for (rank, mode, _), grad in zip(res, got):
        assert mode == expect
        torch.testing.assert_close(grad, want, rtol=1e-6, atol=1e-6)
    assert torch.equal(got[0], got[1]) and torch.equal(got[0], got[2])


def _flags_worker(rank, world, port, q, n_rows, touched):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from psvo.dist import SparseRowSum
        grad = _sparse_grad(rank, n_rows, touched, 11)
        local = (grad != 0).any(1).to(torch.uint8)
        local[rank] = 1  # a flagged row whose gradient is zero: listed, harmless
        union = torch.zeros(n_rows, dtype=torch.uint8)
        union[500] = 1   # sticky from earlier steps (identical on every rank)
        mode = SparseRowSum(n_rows, 16, "cpu", ops=_TorchRowOps())(grad, local=local, union=union)
        q.put((rank, mode, grad.numpy().copy(), local.numpy().copy(), union.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("touched,expect", [(40, "sparse"), (900, "dense")])
def test_sparse_row_sum_with_row_flags(touched, expect):
    """Sparse-exact Adam under data parallelism: with the engine's row flags
    the exchange finds a rank's rows from its `local` flags (no table scan),
    every rank ends with the summed gradient, the union flags mark every
    exchanged row (plus the sticky ones) identically on every rank — the set
    Adam steps — and `local` is cleared for the next step."""
    n_rows, world = 1000, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_flags_worker, args=(r, world, port, q, n_rows, touched)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    grads = [_sparse_grad(r, n_rows, touched, 11) for r in range(world)]
    want = sum(grads)
    touched_any = torch.zeros(n_rows, dtype=torch.bool)
    for g in grads:
        touched_any |= (g != 0).any(1)
    for rank, mode, grad, local, union in res:
        assert mode == expect
        torch.testing.assert_close(torch.from_numpy(grad), want, rtol=1e-6, atol=1e-6)
        assert not local.any()
        u = torch.from_numpy(union).bool()
        assert bool(u[500]) and bool((u | ~touched_any).all())  # every touched row flagged
        # nothing beyond the exchanged rows: touched, sticky, or (sparse) a listed zero row
        extra = u & ~touched_any
        extra[500] = False
        if expect == "sparse":
            extra[:world] = False
        assert not extra.any()
    assert all(np.array_equal(res[0][4], r[4]) for r in res) and all(np.array_equal(res[0][2], r[2]) for r in res)
