"""Data-parallel mapping over ranks: one process per GPU, the
global ray batch split across ranks, ONE fused all-reduce per iteration.

The reference is single-GPU; rays are independent through render and loss
apart from batch-global reductions, so a rank renders its own shard against
the replicated octree / embeddings / decoder and the only exchanges are

  * GradBucket.allreduce: embedding + decoder (+ pose) gradients flattened
    into one contiguous bucket and summed with a single RCCL all-reduce over
    xGMI (one large collective instead of one per tensor — the ring is
    per-link bandwidth bound, so fewer, larger messages win), then copied
    back.  Adam then runs redundantly and identically on every rank.
  * GlobalLossSums (optional, exact mode): the criterion's eight partial
    sums (csrc/criterion.hip) are all-reduced before the loss is formed, and
    every rank pads its [R_hit, S_max] block to the global S_max
    (pad_extra), so the sharded loss and its gradients equal the single-GPU
    loss of the concatenated batch (criterion.py:70-101 normalise by
    batch-global counts and the padded [R_hit, S_max] size).

Works with any torch.distributed backend: "nccl" (RCCL) on the GPUs, "gloo"
for the CPU tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


class CollectiveTimer:
    """Durations of the data-parallel engine's collectives (bench.py's
    collective_ms_per_step): RCCL ones by HIP events on the stream each runs
    on, gloo ones (host-staged, blocking) by the host clock."""

    def __init__(self):
        self.pairs = []     # (start, end) torch.cuda.Event
        self.host_s = 0.0   # gloo: seconds of host time
        self.count = 0

    def cuda(self, stream=None):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        self.pairs.append((a, b))
        self.count += 1
        return a, b

    def total_ms(self):
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in self.pairs) + 1e3 * self.host_s


TIMER = None  # a CollectiveTimer while the bench measures the exchanges


class _HostSpan:
    def __enter__(self):
        import time
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        import time
        if TIMER is not None:
            TIMER.host_s += time.perf_counter() - self.t0
            TIMER.count += 1
        return False


class GradBucket:
    """Flat all-reduce of the gradients of `params` (one collective).

    op="sum" matches the single-GPU gradient of a loss that is a SUM over
    shards (the exact global-loss mode, where each rank's loss already
    carries the global normalisation); op="mean" averages per-rank losses."""

    def __init__(self, params, op="sum", group=None):
        self.params = [p for p in params]
        self.op = op
        self.group = group
        self._flat = None

    def allreduce(self):
        ps = [p for p in self.params if p.grad is not None]
        if not ps or world() == 1:
            return
        n = sum(p.numel() for p in ps)
        dev, dt = ps[0].grad.device, ps[0].grad.dtype
        if self._flat is None or self._flat.numel() != n or self._flat.device != dev:
            self._flat = torch.empty(n, device=dev, dtype=dt)
        flat = self._flat
        off = 0
        for p in ps:
            k = p.numel()
            flat[off:off + k].copy_(p.grad.reshape(-1))
            off += k
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
        if self.op == "mean":
            flat.div_(world())
        off = 0
        for p in ps:
            k = p.numel()
            p.grad.copy_(flat[off:off + k].view_as(p.grad))
            off += k


class GlobalLossSums:
    """reduce_sums hook for psvo.criterion.Criterion / CriterionLoss: the
    loss of the union of all ranks' rays.

    global_shape(r_hit, s_max) all-reduces (Σ R_hit, max S_max) once per
    call; __call__(sums) all-reduces the f64[8] partial sums in place."""

    def __init__(self, group=None):
        self.group = group

    def global_shape(self, r_hit, s_max):
        if world() == 1:
            return r_hit, s_max
        t = torch.tensor([r_hit, -s_max], dtype=torch.int64, device=_coll_device(self.group))
        r = t.clone()
        dist.all_reduce(r[:1], op=dist.ReduceOp.SUM, group=self.group)
        dist.all_reduce(r[1:], op=dist.ReduceOp.MIN, group=self.group)  # max via min of negatives
        r = r.cpu()
        return int(r[0]), int(-r[1])

    def __call__(self, sums):
        if world() > 1:
            dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=self.group)


class GlobalBatch:
    """Exact data-parallel sampling: each rank samples
    its own hit rays inside the [200, K', P] layout of the CONCATENATED batch
    (ranks in order), with the global P / max_steps and noise keyed by the
    global logical index, so its samples equal the matching rows of a
    single-GPU run on the whole batch.  query_samples all-gathers the
    per-ray hit lists (idx / t_in / t_out / count / Σ) through gather_cat —
    P·12 B per ray, an exactness mode rather than the throughput path."""

    def __init__(self, group=None):
        self.group = group

    @property
    def world(self):
        return world()

    @property
    def rank(self):
        return dist.get_rank(self.group) if world() > 1 else 0

    def sizes(self, n):
        if world() == 1:
            return [int(n)]
        t = torch.tensor([int(n)], dtype=torch.int64, device=_coll_device(self.group))
        out = [torch.zeros_like(t) for _ in range(world())]
        dist.all_gather(out, t, group=self.group)
        return [int(x) for x in out]

    def max_int(self, v):
        if world() == 1:
            return int(v)
        t = torch.tensor([int(v)], dtype=torch.int64, device=_coll_device(self.group))
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return int(t)

    def gather_cat(self, t, sizes):
        """Concatenate every rank's `t` (first dims `sizes`) in rank order."""
        if world() == 1:
            return t
        dev = t.device
        stage = "cpu" if _backend(self.group) == "gloo" else dev
        n_max = max(sizes)
        pad = torch.zeros((n_max,) + tuple(t.shape[1:]), dtype=t.dtype, device=stage)
        pad[: t.shape[0]].copy_(t)
        out = [torch.empty_like(pad) for _ in range(world())]
        dist.all_gather(out, pad, group=self.group)
        return torch.cat([o[:k] for o, k in zip(out, sizes)], 0).to(dev)


def _coll_device(group=None):
    """Where small host-side collective operands live: the GPU for RCCL, the CPU for gloo."""
    return torch.device("cuda", torch.cuda.current_device()) if _backend(group) == "nccl" else torch.device("cpu")


def _backend(group=None):
    try:
        return dist.get_backend(group)
    except Exception:
        return "gloo"


def shard(n_total, rank, world_size):
    """Contiguous [begin, end) slice of n_total items for `rank`."""
    per = (n_total + world_size - 1) // world_size
    b = min(n_total, rank * per)
    return b, min(n_total, b + per)


class DeviceRowOps:
    """psvo_rows_compact / psvo_rows_scatter_add on the tensor's device (HIP)."""

    def __init__(self):
        from psvo import _lib as L
        self.L = L

    def compact(self, grad2d, ids, rows, count, workspace):
        self.L.call("psvo_rows_compact", self.L.stream_of(grad2d.device), grad2d.shape[0], grad2d.shape[1], grad2d,
                    workspace, ids, rows, count)

    def scatter_add(self, ids, rows, grad2d):
        self.L.call("psvo_rows_scatter_add", self.L.stream_of(grad2d.device), ids.shape[0], grad2d.shape[1], ids,
                    rows, grad2d)

    def compact_flagged(self, grad2d, flags, ids, rows, count, workspace):
        self.L.call("psvo_rows_compact_flagged", self.L.stream_of(grad2d.device), grad2d.shape[0], grad2d.shape[1],
                    grad2d, flags, workspace, ids, rows, count)

    def clear(self, ids, grad2d, flags):
        self.L.call("psvo_rows_clear", self.L.stream_of(grad2d.device), ids.shape[0], grad2d.shape[1], ids, grad2d,
                    flags)

    def mark(self, ids, flags):
        self.L.call("psvo_rows_mark", self.L.stream_of(flags.device), ids.shape[0], ids, flags)

    def flags_from_grad(self, grad2d, flags):
        self.L.call("psvo_rows_flags_from_grad", self.L.stream_of(grad2d.device), grad2d.shape[0], grad2d.shape[1],
                    grad2d, flags)

    def workspace_ints(self, n_rows):
        return int(self.L.lib().psvo_rows_workspace_ints(n_rows))


class SparseRowSum:
    """In-place all-reduce (sum) of a row-sparse gradient grad2d [n_rows, width]
    that exchanges only the rows a rank touched (a step's
    rays reach a few hundred thousand embedding rows of a multi-million-row
    table, so (id, row) pairs are a small fraction of the dense bytes a ring
    all-reduce moves).

    Protocol: compact the non-zero rows on the device (ascending ids), one
    host read of the count, all-gather the counts, all-gather the padded
    (id, row) lists, zero grad2d and scatter-add the lists in rank order — the
    same additions in the same order on every rank, so replicas stay
    bit-identical.  Falls back to a dense all-reduce when the padded lists
    would move more bytes than the table.  Returns "sparse" or "dense".

    With the engine's row flags (sparse-exact Adam under data parallelism):
    `local` u8[n_rows] = the rows this rank's step touched (its gradient is
    zero elsewhere) — the rows are found from those flags and the rank's own
    rows are zeroed before the lists are added back, so no pass touches the
    dense table; `union` u8[n_rows] (sticky, identical on every rank) gets
    every exchanged row marked, the set Adam then steps.  `local` is
    cleared for the next step."""

    def __init__(self, n_rows, width, device, group=None, ops=None, force=False):
        self.group = group
        self.force = bool(force)  # run the protocol on one rank too (tests)
        self.ops = ops if ops is not None else DeviceRowOps()
        self.ids = torch.empty(n_rows, dtype=torch.int32, device=device)
        self.rows = torch.empty(n_rows, width, dtype=torch.float32, device=device)
        self.count = torch.zeros(1, dtype=torch.int32, device=device)
        self.workspace = torch.empty(max(1, self.ops.workspace_ints(n_rows)), dtype=torch.int32, device=device)

    def __call__(self, grad2d, local=None, union=None):
        n_rows, width = grad2d.shape
        ws = dist.get_world_size(self.group) if dist.is_available() and dist.is_initialized() else 1
        if ws == 1 and not self.force:
            return "dense"
        if local is not None:
            self.ops.compact_flagged(grad2d, local, self.ids, self.rows, self.count, self.workspace)
        else:
            self.ops.compact(grad2d, self.ids, self.rows, self.count, self.workspace)
        stage = torch.device("cpu") if _backend(self.group) == "gloo" else grad2d.device
        cnt = self.count.to(stage, torch.int64)
        counts = [torch.empty_like(cnt) for _ in range(ws)]
        dist.all_gather(counts, cnt, group=self.group)
        counts = [int(c) for c in counts]
        n_max = max(counts)
        mine = int(counts[dist.get_rank(self.group) if self.group is not None else dist.get_rank()])
        if ws * n_max * (width + 1) >= n_rows * width and not (self.force and ws == 1):
            flat = grad2d if stage == grad2d.device else grad2d.to(stage)
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
            if flat is not grad2d:
                grad2d.copy_(flat)
            if union is not None:
                self.ops.flags_from_grad(grad2d, union)
            if local is not None:
                local.zero_()
            return "dense"
        if n_max == 0:  # no rank touched a row: the sum is zero (and gloo rejects empty gathers)
            if local is not None:
                self.ops.clear(self.ids[:mine], grad2d, local)
            else:
                grad2d.zero_()
            return "sparse"
        ids = torch.full((n_max,), -1, dtype=torch.int32, device=stage)
        rows = torch.zeros((n_max, width), dtype=torch.float32, device=stage)
        ids[:mine].copy_(self.ids[:mine])
        rows[:mine].copy_(self.rows[:mine])
        all_ids = [torch.empty_like(ids) for _ in range(ws)]
        all_rows = [torch.empty_like(rows) for _ in range(ws)]
        dist.all_gather(all_ids, ids, group=self.group)
        dist.all_gather(all_rows, rows, group=self.group)
        if local is not None:  # the gradient is zero outside this rank's listed rows
            self.ops.clear(self.ids[:mine], grad2d, local)
        else:
            grad2d.zero_()
        for r in range(ws):
            k = counts[r]
            if k:
                rid = all_ids[r][:k].to(grad2d.device)
                self.ops.scatter_add(rid, all_rows[r][:k].to(grad2d.device), grad2d)
                if union is not None:
                    self.ops.mark(rid, union)
        return "sparse"


XCH_GATHER_I32, XCH_SUM_I32, XCH_SUM_F64, XCH_QUERY = 1, 2, 3, 0x100


class EngineExchange:
    """The collectives of the data-parallel native engine (psvo_engine_set_exchange,
    include/psvo.h): the engine computes the loss of the UNION of all ranks'
    rays — bit-identical sample layout and normalisers to one GPU rendering the
    concatenated batch — and calls back here for its collectives, each on the
    HIP stream the engine produced the operand on: two all-gathers in the
    query phase (8 words + a hit-count byte per ray of the shard; S_max + the
    loss normalisers' counts), plus 8 doubles summed in the step when the
    query could not count the normalisers or the loss value is wanted.
    max_rays_rank: the largest shard a rank passes (default: the union's
    max_rays_global) — it sizes the first all-gather.

    With RCCL ("nccl") the query-phase collectives run on their own
    communicator (they are issued one step ahead, concurrently with the
    previous step's), so neither phase queues behind the other on one NCCL
    stream; with gloo (CPU rehearsal / tests) operands are staged through the
    host.  `apply` is the whole protocol and works on CPU tensors too."""

    def __init__(self, max_rays_global, device=None, group=None, query_group=None, force=False, max_rays_rank=None):
        # force: run every collective even on one rank (identities) — the
        # engine's data-parallel protocol end to end on a 1-rank communicator
        # (tests/test_gpu_rccl.py drives the RCCL branch this way)
        self.force = bool(force)
        on = dist.is_available() and dist.is_initialized()
        if self.force and not on:
            raise RuntimeError("EngineExchange(force=True) needs an initialised torch.distributed process group")
        self.world = dist.get_world_size(group) if on else 1
        self.rank = dist.get_rank(group) if on else 0
        self.max_rays_global = int(max_rays_global)
        self.max_rays_rank = int(max_rays_rank) if max_rays_rank is not None else self.max_rays_global
        self.group = group
        self.nccl = (self.world > 1 or self.force) and on and _backend(group) == "nccl"
        if query_group is None and self.nccl:
            query_group = dist.new_group(list(range(self.world)), backend="nccl")
        self.query_group = query_group if query_group is not None else group
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.xi32 = None
        self.xf64 = torch.zeros(16, dtype=torch.float64, device=self.device)  # include/psvo.h
        self.error = None
        self._cb = None

    def buffers(self, n_words):
        self.xi32 = torch.zeros(int(n_words), dtype=torch.int32, device=self.device)
        return self.xi32, self.xf64

    def apply(self, op, in_off, out_off, count, stream=None):
        """One collective of the engine protocol on xi32 / xf64 (see psvo.h)."""
        grp = self.query_group if (op & XCH_QUERY) else self.group
        op &= 0xFF
        buf = self.xf64 if op == XCH_SUM_F64 else self.xi32
        if op == XCH_GATHER_I32:
            src = buf[in_off:in_off + count]
            dst = buf[out_off:out_off + count * self.world]
        else:
            src = dst = buf[in_off:in_off + count]
        if self.world == 1 and not self.force:
            if op == XCH_GATHER_I32:
                dst.copy_(src)
            return
        if self.nccl:
            ctx = torch.cuda.stream(torch.cuda.ExternalStream(stream)) if stream else _nullctx()
            with ctx:
                ev = TIMER.cuda() if TIMER is not None else None
                if ev:
                    ev[0].record()
                if op == XCH_GATHER_I32:
                    dist.all_gather_into_tensor(dst, src, group=grp)
                else:
                    dist.all_reduce(dst, op=dist.ReduceOp.SUM, group=grp)
                if ev:
                    ev[1].record()
            return
        with _HostSpan():
            self._apply_gloo(op, src, dst, grp, stream)

    def _apply_gloo(self, op, src, dst, grp, stream):
        # gloo: stage through the host, ordered on the engine's stream
        if stream and src.is_cuda:
            torch.cuda.ExternalStream(stream).synchronize()
        h = src.cpu().clone()
        if op == XCH_GATHER_I32:
            parts = [torch.empty_like(h) for _ in range(self.world)]
            dist.all_gather(parts, h, group=grp)
            h = torch.cat(parts)
        else:
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=grp)
        if stream and dst.is_cuda:
            with torch.cuda.stream(torch.cuda.ExternalStream(stream)):
                dst.copy_(h)
        else:
            dst.copy_(h)

    def callback(self):
        """The psvo_exchange_fn handed to the engine (kept alive here)."""
        import ctypes
        if self._cb is None:
            proto = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                                     ctypes.c_int64, ctypes.c_void_p)

            def fn(user, op, in_off, out_off, count, stream):
                try:
                    self.apply(op, in_off, out_off, count, stream)
                    return 0
                except BaseException as exc:  # noqa: BLE001 — reported through the engine's error
                    self.error = exc
                    return 1
            self._cb = proto(fn)
        return self._cb


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


class EngineGradExchange:
    """The engine's per-step gradient exchange (MappingEngine.grad_flat =
    [embedding rows | decoder]): one flat all-reduce while the table is small
    (config B/D: 0.9 MB of embeddings — latency-bound, one collective is best),
    SparseRowSum on the embedding rows + a dense all-reduce of the decoder
    tail once the table reaches `sparse_min_bytes` (config E's multi-million-
    row table, where a step touches a small fraction of the rows).  The
    result is averaged over ranks (op "mean", as GradBucket)."""

    def __init__(self, engine, sparse_min_bytes=32 << 20, group=None, ops=None, op="mean", force=False):
        self.engine = engine
        self.group = group
        self.force = bool(force)  # collectives on one rank too (tests)
        self.op = op  # "sum": the engine's union-batch loss (EngineExchange) — gradients add up
        self.n_emb = int(engine.emb.shape[0])
        self.ops = ops if ops is not None else DeviceRowOps()
        self.sparse = None
        if self.n_emb * 16 * 4 >= sparse_min_bytes:
            self.sparse = SparseRowSum(self.n_emb, 16, engine.grad_flat.device, group=group, ops=ops,
                                       force=force)
        self.last_mode = "dense"
        self._rows_marked = False  # this step's exchange marked the union rows (MappingEngine.adam)

    def take_rows_marked(self):
        """True once after an exchange that marked every exchanged row into
        the engine's union flags: the next Adam step may be row-sparse."""
        m, self._rows_marked = self._rows_marked, False
        return m

    def __call__(self):
        self._rows_marked = False
        ws = dist.get_world_size(self.group) if dist.is_available() and dist.is_initialized() else 1
        if ws == 1 and not self.force:
            return  # no exchange ran: the engine's Adam steps the table densely
        if TIMER is None:
            return self._exchange(ws)
        if _backend(self.group) == "nccl":
            a, b = TIMER.cuda()
            a.record()
            self._exchange(ws)
            b.record()
        else:
            with _HostSpan():
                self._exchange(ws)

    def _exchange(self, ws):
        flat = self.engine.grad_flat
        n = self.n_emb * 16
        union, local = self.engine.row_flags, self.engine.row_local  # sparse-exact Adam (engine.set_exchange)
        if self.sparse is None:
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
            self.last_mode = "dense"
            if union is not None:  # the summed gradient's non-zero rows (a small table: one cheap pass)
                self.ops.flags_from_grad(flat[:n].view(self.n_emb, 16), union)
            if local is not None:
                local.zero_()
        else:
            self.last_mode = self.sparse(flat[:n].view(self.n_emb, 16), local=local, union=union)
            dist.all_reduce(flat[n:], op=dist.ReduceOp.SUM, group=self.group)
        self._rows_marked = union is not None
        if self.op == "mean":
            flat.div_(ws)
