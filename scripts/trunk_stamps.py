"""Diagnostic: where k_mlp_trunk_fb (the sparse decoder's class-B trunk forward + backward) spends a
round — s_memtime stamps of the lib/diag/libpsvo_stamps.so build (`make -C
proud-slam_amd/csrc stamps`), recorded by the last launch of a short
bench.py run (config B).  Read the SHARES of the segments: the stamps fence
the code.  Usage: trunk_stamps.py [bench args...]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIAG = os.path.join(ROOT, "proud-slam_amd", "lib", "diag", "libpsvo_stamps.so")
os.environ["PSVO_LIB_PATH"] = DIAG
sys.path.insert(0, ROOT)

CHAIN = [("wait fwd (bar)", 0, 1), ("P: W2T", 1, 2), ("bar P", 2, 3), ("Q: W1T", 3, 4),
         ("Q: interp", 4, 5), ("Q: scatter", 5, 6)]
GRAD = [("bar top", 0, 1), ("P: dW2", 1, 2), ("bar P", 2, 3), ("Q: dW1 (xgrad)", 3, 4), ("Q: forward", 4, 6)]
B3 = [("P0", 0, 1), ("bar0", 1, 2), ("P1", 2, 3), ("bar1", 3, 4), ("P2", 4, 5), ("bar2", 5, 6), ("P3", 6, 7),
      ("bar3", 7, 8)]


def main():
    sys.argv = ["bench.py", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-traffic"] + sys.argv[1:]
    import bench  # noqa: E402
    bench.main()
    L = ctypes.CDLL(DIAG)
    buf = np.zeros((3, 256, 8, 8, 16), dtype=np.uint64)
    assert L.psvo_debug_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_int64(buf.nbytes)) == 0
    for kern, k, last, roles in (("trunk_fb", 2, 6, (("chain", range(4), CHAIN), ("grad", range(4, 8), GRAD))),
                                 ("bwd3", 1, 8, (("chain", range(4), B3), ("grad", range(4, 8), B3)))):
        report(buf[k].astype(np.int64), kern, last, roles)


def report(st, kern, last, roles):  # st: [wg][wave][round][stamp]
    for role, waves, segs in roles:
        v = st[:, list(waves)].reshape(-1, 16)
        ok = (v[:, 0] > 0) & (v[:, last] > 0)
        v = v[ok]
        tot = (v[:, last] - v[:, 0]).mean()
        print(f"{kern} {role}: {len(v)} wave-rounds, mean round {tot:.0f} cycles", file=sys.stderr)
        for nm, a, b in segs:
            good = (v[:, a] > 0) & (v[:, b] > 0)
            d = (v[good, b] - v[good, a]).astype(np.float64)
            print(f"   {nm:16s} {d.mean():9.0f}  ({100 * d.mean() / tot:5.1f}%)  p90 {np.percentile(d, 90):9.0f}",
                  file=sys.stderr)


if __name__ == "__main__":
    main()
