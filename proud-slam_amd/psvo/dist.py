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
