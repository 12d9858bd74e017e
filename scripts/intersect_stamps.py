"""Diagnostic: where a ray's k_intersect_sorted time goes (the s_memtime
segment counters of the lib/diag/libpsvo_is_stamps.so build, `make -C
proud-slam_amd/csrc is_stamps`), on the engine's last step of a bench scene.
Prints the distribution of per-ray cycles and rounds, and the segment shares
for all rays and for the slowest 10 %.  Usage: intersect_stamps.py [scene]"""
import ctypes
import os
import sys
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "proud-slam_amd"))
os.environ["PSVO_LIB_PATH"] = os.environ.get("PSVO_DIAG_LIB") or os.path.join(ROOT, "proud-slam_amd", "lib", "diag",
                                                                             "libpsvo_is_stamps.so")
from psvo import _lib  # noqa: E402
import bench  # noqa: E402

SEG = ["pop+load+aabb", "scan+push", "leaf merge", "sort+output"]


def main():
    scene_name = sys.argv[1] if len(sys.argv) > 1 else "room0"
    args = types.SimpleNamespace(scene=scene_name, width=128, frames=4, rays_per_frame=1024)
    dev = torch.device("cuda")
    scene, tree, ms, emb, dec = bench.build_scene(args, dev, 0)
    kfs = bench.build_keyframes(args, scene, dev, 0)
    batches = bench.keyframe_batches(kfs, args.rays_per_frame, 4)
    from psvo.engine import MappingEngine
    step = {"room0": 0.0142, "multiroom": 0.0147}.get(scene_name, 0.015)
    eng = MappingEngine(ms, dec, scene.voxel_size, step, truncation=0.1, max_distance=10.0,
                        criteria={"rgb_weight": 0.5, "depth_weight": 1.0, "sdf_weight": 5000.0, "fs_weight": 10.0},
                        max_depth=10.0)
    for it in range(6):
        b = batches[it % len(batches)]
        eng.step(b[0][0], b[1][0], b[2][0], b[3][0], seed=it)
    torch.cuda.synchronize()
    R = b[0].shape[1]
    L = ctypes.CDLL(_lib.LIB_PATH)
    buf = np.zeros((16384, 8), dtype=np.uint64)
    rc = L.psvo_debug_is_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_int64(buf.nbytes))
    assert rc == 0, rc
    d = buf[:R].astype(np.float64)
    d = d[d[:, 0] > 0]
    tot, rounds, lr, vis = d[:, 0], d[:, 5], d[:, 6], d[:, 7]
    q = lambda x: " ".join(f"{p}:{np.percentile(x, p):.0f}" for p in (50, 90, 99, 100))  # noqa: E731
    print(f"{scene_name}: {len(d)} rays; cycles/ray mean {tot.mean():.0f} ({q(tot)})")
    print(f"  rounds mean {rounds.mean():.2f} ({q(rounds)}); leaf rounds mean {lr.mean():.2f}; "
          f"AABB tests mean {vis.mean():.0f} ({q(vis)})")
    print(f"  cycles per round mean {(tot / np.maximum(rounds, 1)).mean():.0f}")
    slow = tot >= np.percentile(tot, 90)
    for name, sel in (("all rays", np.ones_like(slow)), ("slowest 10%", slow)):
        t = tot[sel].sum()
        parts = [d[sel, 1 + k].sum() / t * 100 for k in range(4)]
        other = 100 - sum(parts)
        print(f"  {name:12s} " + "  ".join(f"{n} {p:.1f}%" for n, p in zip(SEG, parts)) +
              f"  rest {other:.1f}%  | rounds {rounds[sel].mean():.1f}, leaf rounds {lr[sel].mean():.1f}")
    eng.close()


if __name__ == "__main__":
    main()
