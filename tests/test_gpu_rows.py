"""Row-sparse gradient exchange kernels (csrc/rows.hip) vs torch on the
device: compaction order and content, scatter-add of several rank lists in
order (the SparseRowSum protocol's device half)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _compact(grad):
    from psvo import _lib as L
    n, w = grad.shape
    ids = torch.full((n,), -7, dtype=torch.int32, device=DEV)
    rows = torch.empty(n, w, device=DEV)
    count = torch.empty(1, dtype=torch.int32, device=DEV)
    ws = torch.empty(max(1, int(L.lib().psvo_rows_workspace_ints(n))), dtype=torch.int32, device=DEV)
    L.call("psvo_rows_compact", L.stream_of(DEV), n, w, grad, ws, ids, rows, count)
    k = int(count)
    return ids[:k], rows[:k]


@pytest.mark.parametrize("n_rows,touched", [(0, 0), (1, 1), (1023, 100), (1024, 1024), (250001, 30000),
                                            (70000, 0)])
def test_rows_compact_matches_torch(n_rows, touched):
    g = torch.Generator().manual_seed(n_rows + touched)
    grad = torch.zeros(n_rows, 16)
    if touched:
        idx = torch.randperm(n_rows, generator=g)[:touched]
        grad[idx] = torch.randn(touched, 16, generator=g)
        grad[idx[:3], :15] = 0.0  # rows with a single non-zero element
    grad = grad.to(DEV)
    ids, rows = _compact(grad)
    want = (grad != 0).any(1).nonzero().flatten()
    assert torch.equal(ids.long(), want)
    assert torch.equal(rows, grad[want])


@pytest.mark.parametrize("n_rows,touched", [(1, 1), (1023, 100), (250001, 30000), (70000, 0)])
def test_rows_flag_kernels_match_torch(n_rows, touched):
    """The data-parallel sparse-Adam half: compaction from a flag array
    (listing a flagged all-zero row too), clearing a list's rows and flags,
    marking a list, flags from a gradient's non-zero rows."""
    from psvo import _lib as L
    g = torch.Generator().manual_seed(n_rows + 2 * touched)
    grad = torch.zeros(n_rows, 16)
    flags = torch.zeros(n_rows, dtype=torch.uint8)
    if touched:
        idx = torch.randperm(n_rows, generator=g)[:touched]
        grad[idx] = torch.randn(touched, 16, generator=g)
        flags[idx] = 1
    flags[0] = 1  # flagged, possibly all-zero
    grad, flags = grad.to(DEV), flags.to(DEV)
    ids = torch.full((n_rows,), -7, dtype=torch.int32, device=DEV)
    rows = torch.empty(n_rows, 16, device=DEV)
    count = torch.empty(1, dtype=torch.int32, device=DEV)
    ws = torch.empty(max(1, int(L.lib().psvo_rows_workspace_ints(n_rows))), dtype=torch.int32, device=DEV)
    L.call("psvo_rows_compact_flagged", L.stream_of(DEV), n_rows, 16, grad, flags, ws, ids, rows, count)
    k = int(count)
    want = flags.nonzero().flatten()
    assert torch.equal(ids[:k].long(), want) and torch.equal(rows[:k], grad[want])
    nzf = torch.zeros(n_rows, dtype=torch.uint8, device=DEV)
    L.call("psvo_rows_flags_from_grad", L.stream_of(DEV), n_rows, 16, grad, nzf)
    assert torch.equal(nzf.bool(), (grad != 0).any(1))
    marks = torch.zeros(n_rows, dtype=torch.uint8, device=DEV)
    pad = torch.cat([ids[:k], torch.full((3,), -1, dtype=torch.int32, device=DEV)])
    L.call("psvo_rows_mark", L.stream_of(DEV), pad.shape[0], pad, marks)
    assert torch.equal(marks, flags)
    L.call("psvo_rows_clear", L.stream_of(DEV), pad.shape[0], 16, pad, grad, flags)
    assert not grad.any() and not flags.any()


def test_rows_scatter_add_in_rank_order():
    from psvo import _lib as L
    g = torch.Generator().manual_seed(3)
    n = 50000
    grads = []
    for r in range(4):
        x = torch.zeros(n, 16)
        idx = torch.randperm(n, generator=g)[:6000]
        x[idx] = torch.randn(6000, 16, generator=g)
        grads.append(x.to(DEV))
    out = torch.zeros(n, 16, device=DEV)
    for x in grads:
        ids, rows = _compact(x)
        pad_ids = torch.cat([ids, torch.full((5,), -1, dtype=torch.int32, device=DEV)])
        pad_rows = torch.cat([rows, torch.zeros(5, 16, device=DEV)])
        L.call("psvo_rows_scatter_add", L.stream_of(DEV), pad_ids.shape[0], 16, pad_ids, pad_rows, out)
    want = torch.zeros(n, 16, device=DEV)
    for x in grads:
        want += x
    assert torch.equal(out, want)  # same additions in the same order per element


def _rows_worker(rank, world, port, q, n_rows, touched):
    import os
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "proud-slam_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from psvo.dist import SparseRowSum
        g = torch.Generator().manual_seed(11 + rank)
        grad = torch.zeros(n_rows, 16)
        idx = torch.randperm(n_rows, generator=g)[:touched]
        grad[idx] = torch.randn(touched, 16, generator=g)
        grad = grad.to(DEV)
        mode = SparseRowSum(n_rows, 16, DEV)(grad)  # the HIP compaction / scatter kernels
        torch.cuda.synchronize()
        q.put((rank, mode, grad.cpu().numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_sparse_row_sum_two_ranks_device_kernels():
    """SparseRowSum with the device kernels, two ranks sharing the GPU (gloo):
    both ranks end with the sum of both gradients, bit-identical."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    n_rows, touched, world = 300000, 20000, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rows_worker, args=(r, world, port, q, n_rows, touched)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=150) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = torch.zeros(n_rows, 16)
    for r in range(world):
        g = torch.Generator().manual_seed(11 + r)
        x = torch.zeros(n_rows, 16)
        idx = torch.randperm(n_rows, generator=g)[:touched]
        x[idx] = torch.randn(touched, 16, generator=g)
        want += x
    got = [torch.from_numpy(r[2]) for r in res]
    assert all(r[1] == "sparse" for r in res)
    torch.testing.assert_close(got[0], want, rtol=1e-6, atol=1e-6)
    assert torch.equal(got[0], got[1])
