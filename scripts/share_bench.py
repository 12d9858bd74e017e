"""Tracker <-> mapper state exchange throughput.

A mapper process publishes map_states + decoder `--versions` times; this
(tracker) process fetches each new snapshot into device tensors.  Timed per
snapshot: publish (mapper side, until the snapshot is visible) and fetch
(tracker side, until its private device copy is complete).

Beside it, the reference's mechanism restated (share.py:27-166 served by a
multiprocessing BaseManager, voxslam.py:28-33): update_share_data
(mapping.py:236-248) = {k: v.detach().cpu()} + deepcopy(decoder).cpu() set
through the manager proxy (pickle + deepcopy under the manager's lock);
do_tracking (tracking.py:114-125) = proxy get (deepcopy + pickle back) +
.cuda() per tensor.

Scenes: room0 (13.8 k nodes, 20 k x 16 embeddings, W=128 decoder) and a
config-E-sized map (2.74 M nodes, embeddings per node).

    python scripts/share_bench.py [--versions 20] [--scene room0|E|both]
"""
import argparse
import copy
import json
import multiprocessing as mp
import os
import sys
import time
from multiprocessing.managers import BaseManager

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "proud-slam_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

SCENES = {"room0": (13835, 20000), "E": (2740000, 2740000)}


def make_state(n_nodes, n_emb, v, dev):
    import torch
    return {
        "voxel_center_xyz": torch.full((n_nodes, 3), float(v), device=dev),
        "voxel_structure": torch.full((n_nodes, 9), v, dtype=torch.int32, device=dev),
        "voxel_vertex_idx": torch.full((n_nodes, 8), v, dtype=torch.int32, device=dev),
        "voxel_vertex_emb": torch.full((n_emb, 16), float(v), device=dev),
    }


def make_decoder():
    import torch
    from psvo.decoder import Decoder
    torch.manual_seed(0)
    return Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none").cuda()


class RefShare:
    """The reference's ShareData restated: deepcopy in and out under a lock,
    served by a BaseManager (pickled through a socket both ways)."""

    def __init__(self):
        self._states = None
        self._decoder = None
        self._stop = False

    def set_states(self, s):
        self._states = copy.deepcopy(s)

    def get_states(self):
        return copy.deepcopy(self._states)

    def set_decoder(self, d):
        self._decoder = copy.deepcopy(d)

    def get_decoder(self):
        return copy.deepcopy(self._decoder)

    def set_stop(self, v):
        self._stop = v

    def get_stop(self):
        return self._stop


class Mgr(BaseManager):
    pass


Mgr.register("RefShare", RefShare)


def mapper_ours(share, n_nodes, n_emb, versions, q):
    import torch
    torch.cuda.set_device(0)
    dec = make_decoder()
    states = [make_state(n_nodes, n_emb, v, "cuda") for v in (1, 2)]
    torch.cuda.synchronize()
    times = []
    for v in range(versions):
        t0 = time.perf_counter()
        share.decoder = dec
        share.states = states[v % 2]
        times.append(time.perf_counter() - t0)
        while share.version("voxels") < v + 1:   # the tracker acknowledges each snapshot on a spare channel
            time.sleep(0.0002)
    q.put(times)
    while not share.stop_tracking:
        time.sleep(0.005)
    share.close()


def mapper_ref(proxy, n_nodes, n_emb, versions, q, seen, published):
    import torch
    torch.cuda.set_device(0)
    dec = make_decoder()
    states = [make_state(n_nodes, n_emb, v, "cuda") for v in (1, 2)]
    torch.cuda.synchronize()
    times = []
    for v in range(versions):
        t0 = time.perf_counter()
        proxy.set_decoder(copy.deepcopy(dec).cpu())                        # mapping.py:238
        proxy.set_states({k: t.detach().cpu() for k, t in states[v % 2].items()})   # mapping.py:243-247
        times.append(time.perf_counter() - t0)
        published.value = v + 1
        while seen.value < v + 1:
            time.sleep(0.0002)
    q.put(times)


def run_ours(n_nodes, n_emb, versions):
    import torch
    from psvo.share import ShareData

    share = ShareData()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=mapper_ours, args=(share, n_nodes, n_emb, versions, q))
    p.start()
    fetch, last = [], 0
    dec, states = None, None
    ack = torch.zeros(1, device="cuda")
    t_end = time.time() + 600
    while last < versions and time.time() < t_end:
        if share.version("states") <= last:
            time.sleep(0.0002)
            continue
        t0 = time.perf_counter()
        dec = share.decoder                          # tracking.py:116
        r = share.fetch("states", after=last)        # tracking.py:120-125
        fetch.append(time.perf_counter() - t0)
        states, last = r
        share.voxels = ack                           # ack (not timed)
    ok = bool((states["voxel_structure"][:16] == (1 if versions % 2 else 2)).all())
    pub = q.get(timeout=120)
    share.stop_tracking = True
    p.join(timeout=60)
    share.close()
    return {"publish_ms": 1e3 * sorted(pub)[len(pub) // 2], "fetch_ms": 1e3 * sorted(fetch)[len(fetch) // 2],
            "snapshots": len(fetch), "contents_ok": ok}


def run_ref(n_nodes, n_emb, versions):
    import torch
    mgr = Mgr()
    mgr.start()
    proxy = mgr.RefShare()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    seen, published = ctx.Value("i", 0), ctx.Value("i", 0)
    p = ctx.Process(target=mapper_ref, args=(proxy, n_nodes, n_emb, versions, q, seen, published))
    p.start()
    fetch = []
    for v in range(versions):
        while published.value < v + 1:
            time.sleep(0.0002)
        t0 = time.perf_counter()
        dec = proxy.get_decoder().cuda()                                  # tracking.py:116
        st = {k: t.cuda() for k, t in proxy.get_states().items()}         # tracking.py:120-125
        torch.cuda.synchronize()
        fetch.append(time.perf_counter() - t0)
        seen.value = v + 1
        del dec, st
    pub = q.get(timeout=600)
    p.join(timeout=60)
    mgr.shutdown()
    return {"publish_ms": 1e3 * sorted(pub)[len(pub) // 2], "fetch_ms": 1e3 * sorted(fetch)[len(fetch) // 2],
            "snapshots": len(fetch)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--versions", type=int, default=20)
    ap.add_argument("--scene", default="both")
    ap.add_argument("--ref-versions", type=int, default=4)
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    scenes = ["room0", "E"] if a.scene == "both" else [a.scene]
    out = {}
    for sc in scenes:
        n_nodes, n_emb = SCENES[sc]
        mb = (n_nodes * (12 + 36 + 32) + n_emb * 64 + 54276 * 4) / 1e6
        ours = run_ours(n_nodes, n_emb, a.versions)
        print(f"[{sc}] ours {ours}", file=sys.stderr, flush=True)
        ref = run_ref(n_nodes, n_emb, a.ref_versions)
        print(f"[{sc}] reference mechanism {ref}", file=sys.stderr, flush=True)
        out[sc] = {"snapshot_MB": round(mb, 2), "nodes": n_nodes, "embeddings": n_emb, "device_ipc": ours,
                   "reference_manager_pickle": ref,
                   "speedup_round_trip": (ref["publish_ms"] + ref["fetch_ms"]) / (ours["publish_ms"] + ours["fetch_ms"]),
                   "fetch_GBps": mb / 1e3 / (ours["fetch_ms"] / 1e3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
