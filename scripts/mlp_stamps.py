"""Diagnostic: where k_mlp_fwd2 / k_mlp_bwd3 spend a tile / round (s_memtime stamps of
the lib/diag/libpsvo_stamps.so build, `make -C proud-slam_amd/csrc stamps`).
Read the SHARES of the segments, not the absolute time (the stamps fence the
code).  Prints per-segment mean cycles over (workgroup, wave, tile)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "proud-slam_amd"))
from psvo import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "proud-slam_amd", "lib", "diag", "libpsvo_stamps.so")
from psvo.decoder import Decoder  # noqa: E402

FWD = ["L1", "bar1", "L2", "bar2", "L3(+sdf)", "bar3(+stage,x)", "L4", "epilogue"]
B3 = ["P0", "bar0", "P1", "bar1", "P2", "bar2", "P3", "bar3"]


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 262963
    torch.manual_seed(0)
    dec = Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none").cuda()
    x = (torch.randn(m, 16, device="cuda") * 0.3).requires_grad_(True)
    for _ in range(4):
        out = dec({"emb": x})
        (out["sdf"].sum() + out["color"].sum()).backward()
    torch.cuda.synchronize()
    L = ctypes.CDLL(_lib.LIB_PATH)
    shape = (3, 256, 8, 8, 16)
    buf = np.zeros(shape, dtype=np.uint64)
    rc = L.psvo_debug_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_int64(buf.nbytes))
    assert rc == 0, rc
    n_wg_tiles = (m + 255) // 256
    for k, names in ((0, FWD),):
        st = buf[k].astype(np.int64)
        npts = len(names) + 1
        rows = []
        for wg in range(256):
            n_it = len(range(wg, n_wg_tiles, 256))
            for w in range(8):
                for it in range(min(n_it, 8)):
                    v = st[wg, w, it, :npts]
                    if v[0] == 0 or v[-1] == 0:
                        continue
                    rows.append(np.diff(v))
        d = np.array(rows, dtype=np.float64)
        tot = d.sum(1).mean()
        print(f"fwd2: {len(rows)} wave-tiles, mean tile {tot:.0f} cycles")
        for i, nm in enumerate(names):
            print(f"   {nm:16s} {d[:, i].mean():9.0f}  ({100 * d[:, i].mean() / tot:5.1f}%)  p90 {np.percentile(d[:, i], 90):9.0f}")
    b3_report(buf, m)


def b3_report(buf, m):
    """k_mlp_bwd3: per round, chain waves (0-3) and gradient waves (4-7) separately."""
    st = buf[1].astype(np.int64)
    n_units = (m + 15) // 16
    for role, waves in (("chain", range(4)), ("grad", range(4, 8))):
        rows = []
        for wg in range(256):
            u0, u1 = n_units * wg // 256, n_units * (wg + 1) // 256
            n_rounds = (u1 - u0 + 3) // 4
            for w in waves:
                for it in range(min(n_rounds, 8)):
                    v = st[wg, w, it, :9]
                    if v[0] == 0 or v[8] == 0:
                        continue
                    rows.append(np.diff(v))
        d = np.array(rows, dtype=np.float64)
        tot = d.sum(1).mean()
        print(f"bwd3 {role}: {len(rows)} wave-rounds, mean round {tot:.0f} cycles")
        for i, nm in enumerate(B3):
            print(f"   {nm:8s} {d[:, i].mean():9.0f}  ({100 * d[:, i].mean() / tot:5.1f}%)  p90 {np.percentile(d[:, i], 90):9.0f}")
        if role == "chain":  # sub-phase stamps 9..14 (0 where the code did not run)
            subs = []
            for wg in range(256):
                u0, u1 = n_units * wg // 256, n_units * (wg + 1) // 256
                for w in waves:
                    for it in range(min((u1 - u0 + 3) // 4, 8)):
                        subs.append(st[wg, w, it, :15])
            sv = np.array(subs, dtype=np.int64)
            for nm, a, b in (("P0 prep", 0, 9), ("P0 W4T", 9, 10), ("P0 dW1", 10, 1), ("P1 W3T", 2, 11),
                             ("P1 dW4x", 11, 3), ("P2 W2T", 4, 12), ("P2 loads", 12, 5), ("P3 W1T", 6, 13),
                             ("P3 interp", 13, 14), ("P3 scatter", 14, 7)):
                ok = (sv[:, a] > 0) & (sv[:, b] > 0)
                if ok.any():
                    print(f"     {nm:10s} {np.mean(sv[ok, b] - sv[ok, a]):9.0f}")


def dw_report(buf):
    """k_mlp_dw2: per-workgroup span and per-wave segment shares, by layer type."""
    st = buf[2, :, :, 0, :8].astype(np.int64)  # [wg][wave][start,end,wait,bar,issue,mfma,units,L]
    used = st[:, 0, 0] > 0
    t0 = st[used, :, 0].min()
    print("dw2: per layer type (0: W1+W5, 1: W2, 2: W3, 3: W4)")
    for L in range(4):
        sel = used & (st[:, 0, 7] == L)
        if not sel.any():
            continue
        span = (st[sel, :, 1].max(1) - t0)
        seg = st[sel][:, :, 2:6].sum(axis=(0, 1)).astype(np.float64)
        tot = seg.sum()
        units = st[sel, 0, 6]
        print(f"  L{L}: {int(sel.sum())} wgs, units/wg {units.min()}-{units.max()}, end {span.min()}-{span.max()} cycles, "
              f"wait {100 * seg[0] / tot:.1f}% bar {100 * seg[1] / tot:.1f}% issue {100 * seg[2] / tot:.1f}% "
              f"mfma {100 * seg[3] / tot:.1f}%  per-unit {tot / units.sum() / 8:.0f} cyc/wave")


if __name__ == "__main__":
    main()
