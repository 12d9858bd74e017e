"""Diagnostic: where k_sample_fused's time goes, per workgroup (s_memrealtime
stamps of the lib/diag/libpsvo_is_stamps.so build, `make -C
proud-slam_amd/csrc is_stamps`): entry, rays sampled, row stores drained,
look-back prefix known, compaction done — recorded by the last sampler
launch of a short bench.py run (config B).  Prints the launch's timeline
(first entry to last exit) and the per-segment distributions.
Usage: sampler_stamps.py [bench args...]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIAG = os.environ.get("PSVO_DIAG_LIB") or os.path.join(ROOT, "proud-slam_amd", "lib", "diag", "libpsvo_is_stamps.so")
os.environ["PSVO_LIB_PATH"] = DIAG
sys.path.insert(0, ROOT)


def main():
    sys.argv = ["bench.py", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-traffic"] + sys.argv[1:]
    import bench  # noqa: E402
    bench.main()
    L = ctypes.CDLL(DIAG)
    buf = np.zeros((4096, 8), dtype=np.uint64)
    assert L.psvo_debug_smp_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_int64(buf.nbytes)) == 0
    st = buf.astype(np.int64)
    # the last launch's workgroups: entry stamps within 1 ms of the latest entry
    t0 = st[:, 0]
    live = t0 > 0
    last = t0[live].max()
    sel = live & (t0 > last - 100000)  # 100 MHz: 1 ms
    s = st[sel] / 100.0  # µs
    base = s[:, 0].min()
    print(f"k_sample_fused: {sel.sum()} workgroups; entries span {s[:, 0].max() - base:.1f} us; "
          f"last exit {s[:, 4].max() - base:.1f} us after the first entry", file=sys.stderr)
    q = lambda x: " ".join(f"p{p}:{np.percentile(x, p):.1f}" for p in (10, 50, 90, 100))  # noqa: E731
    for nm, a, b in (("sample rays", 0, 1), ("  entry -> row loaded", 0, 5), ("  cdf + bin ends", 5, 6),
                     ("  interior samples", 6, 7), ("  ends + trailing", 7, 1),
                     ("drain + barrier", 1, 2), ("look-back", 2, 3), ("compaction", 3, 4), ("whole wg", 0, 4)):
        ok = (s[:, a] > 0) & (s[:, b] > 0)
        d = s[ok, b] - s[ok, a]
        print(f"   {nm:16s} mean {d.mean():6.2f} us  {q(d)}", file=sys.stderr)
    for k, nm in ((0, "entry"), (2, "prefix wait start"), (3, "prefix known"), (4, "exit")):
        print(f"   {nm:18s} (from first entry) {q(s[:, k] - base)}", file=sys.stderr)


if __name__ == "__main__":
    main()
