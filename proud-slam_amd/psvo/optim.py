"""Adam for the mapping loop on libpsvo's multi-tensor kernel (csrc/optim.hip).

Drop-in for torch.optim.Adam as the reference uses it (render_helpers.py:
581-596: Adam(embeddings), Adam(decoder), per-keyframe pose Adam; lr /
betas / eps / weight_decay, amsgrad off): same constructor, param groups,
state keys ("step", "exp_avg", "exp_avg_sq") and state_dict, so checkpoints
move between the two.  Every step of every group is one kernel launch over
all its tensors.  Parameters that are not f32 CUDA tensors (or sparse grads)
raise — there is no PyTorch fallback.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib as L


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False):
        if amsgrad:
            raise NotImplementedError("psvo.optim.Adam: amsgrad is not supported (the reference does not use it)")
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameters: {betas}")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            ps, gs, ms, vs, ns = [], [], [], [], []
            step_no = None
            keep = []
            for p in group["params"]:
                if p.grad is None:
                    continue
                if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()):
                    raise RuntimeError("psvo.optim.Adam: parameters must be contiguous float32 CUDA tensors")
                if p.grad.is_sparse:
                    raise RuntimeError("psvo.optim.Adam: sparse gradients are not supported")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                s = int(st["step"].item())
                if step_no is None:
                    step_no = s
                elif s != step_no:  # tensors of one group at different step counts: launch separately
                    self._launch(group, [p], [p.grad], [st["exp_avg"]], [st["exp_avg_sq"]], s)
                    continue
                g = p.grad.contiguous()
                keep.append(g)
                ps.append(p)
                gs.append(g)
                ms.append(st["exp_avg"])
                vs.append(st["exp_avg_sq"])
            if ps:
                self._launch(group, ps, gs, ms, vs, step_no)
        return loss

    @staticmethod
    def _launch(group, ps, gs, ms, vs, step_no):
        n = len(ps)
        tables = [(ctypes.c_void_p * n)(*[t.data_ptr() for t in ts]) for ts in (ps, gs, ms, vs)]
        numel = (ctypes.c_int64 * n)(*[t.numel() for t in ps])
        vp = lambda a: ctypes.cast(a, ctypes.c_void_p)
        beta1, beta2 = group["betas"]
        L.call("psvo_adam_step", L.stream_of(ps[0].device), n, *[vp(a) for a in tables], vp(numel),
               float(group["lr"]), float(beta1), float(beta2), float(group["eps"]), float(group["weight_decay"]),
               int(step_no))
