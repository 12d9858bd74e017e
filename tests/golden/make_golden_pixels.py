"""Golden vectors for keyframe pixel sampling (container only: imports the
reference's own /root/reference/src/utils/sample_util.py, pure torch).

For each case the reference's sample_rays(mask, N) runs under
torch.manual_seed(seed); the uniforms it draws inside gumbel_like
(torch.rand_like, sample_util.py:5-6) are reproduced by re-seeding and drawing
torch.rand of the same shape, and stored with the picked pixel indices:

  P_pixels.npz   case{c}.mask   f32 [B, H, W]  the sampling weights
                 case{c}.u      f32 [B, H·W]   the uniforms rand_like drew
                 case{c}.idx    i64 [B, N]     picked pixels (ascending)
                 case{c}.n      N

Cases: a uniform frame (frame.py:84-85's torch.ones_like(depth)[None]) at
1/10 Replica size, two frames of a 0/1 mask with a hole (B = 2: one sum over
both frames, top-k per frame), and fractional weights.

Usage:  python tests/golden/make_golden_pixels.py
"""
import os
import sys

sys.dont_write_bytecode = True  # never write into /root/reference

import numpy as np
import torch

sys.path.insert(0, "/root/reference/src")
from utils.sample_util import sample_rays  # noqa: E402  (the reference's own function)

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "P_pixels.npz")


def case(mask, n, seed):
    torch.manual_seed(seed)
    m = sample_rays(mask, n)
    torch.manual_seed(seed)
    u = torch.rand(mask.shape[0], mask.shape[1] * mask.shape[2])  # = rand_like(logp) of sample_rays
    B = mask.shape[0]
    idx = torch.stack([torch.nonzero(m[b].reshape(-1)).squeeze(1) for b in range(B)])
    assert idx.shape == (B, n)
    return {"mask": mask.numpy().astype(np.float32), "u": u.numpy(), "idx": idx.numpy().astype(np.int64),
            "n": np.int64(n)}


def main():
    out = {}
    H, W = 68, 120
    cases = []
    cases.append((torch.ones(1, H, W), 1024, 11))
    m2 = torch.ones(2, H, W)
    m2[:, 20:40, 30:70] = 0.0
    cases.append((m2, 700, 12))
    g = torch.Generator().manual_seed(5)
    cases.append((torch.rand(1, H, W, generator=g) * 3.0, 512, 13))
    for c, (mask, n, seed) in enumerate(cases):
        for k, v in case(mask, n, seed).items():
            out[f"case{c}.{k}"] = v
    out["n_cases"] = np.int64(len(cases))
    np.savez_compressed(OUT, **out)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
