"""Decoder MLP kernels alone at the bench's sample count (profiling aid):
forward (training mode) + backward, `--iters` times on synthetic features."""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "proud-slam_amd"))
from psvo.decoder import Decoder  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=243614)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--width", type=int, default=128)
    a = ap.parse_args()
    torch.manual_seed(0)
    dec = Decoder(depth=2, width=a.width, in_dim=16, skips=[], embedder="none").cuda()
    x = (torch.randn(a.m, 16, device="cuda") * 0.3).requires_grad_(True)
    for i in range(a.iters + 3):
        if i == 3:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        out = dec({"emb": x})
        (out["sdf"].sum() + out["color"].sum()).backward()
    torch.cuda.synchronize()
    print(f"W={a.width} m={a.m} fwd+bwd {1e3 * (time.perf_counter() - t0) / a.iters:.3f} ms/iter")


if __name__ == "__main__":
    main()
