"""Device snapshots of ShareData on the GPU: same-process
round trips, a writer process publishing while this process reads over HIP
IPC (no torn snapshots, bit-exact contents, growing maps that force slot
reallocation), decoder modules, in-place refresh.

Reference behaviour: update_share_data (mapping.py:236-248) publishes the
decoder and every map_states tensor; do_tracking (tracking.py:114-125) takes a
private copy of each (ShareData getters deepcopy, share.py:41-47, :105-111)."""
import multiprocessing as mp
import time

import pytest
import torch

from psvo.decoder import Decoder
from psvo.share import ShareData

pytestmark = pytest.mark.gpu


def _states(v, n_nodes, dev):
    """A map_states-shaped snapshot whose every element encodes version v."""
    g = torch.Generator(device="cpu").manual_seed(v)
    return {
        "voxel_center_xyz": torch.full((n_nodes, 3), float(v), device=dev),
        "voxel_structure": torch.full((n_nodes, 9), v, dtype=torch.int32, device=dev),
        "voxel_vertex_idx": torch.full((n_nodes, 8), -v, dtype=torch.int32, device=dev),
        "voxel_vertex_emb": (torch.randn(20000, 16, generator=g) + v * 1000).to(dev),
    }


def _check_snapshot(st, ver):
    n = st["voxel_center_xyz"].shape[0]
    assert st["voxel_structure"].shape == (n, 9) and st["voxel_vertex_idx"].shape == (n, 8)
    assert bool((st["voxel_center_xyz"] == float(ver)).all()), f"torn snapshot at version {ver}"
    assert bool((st["voxel_structure"] == ver).all())
    assert bool((st["voxel_vertex_idx"] == -ver).all())
    ref = _states(ver, 1, "cpu")["voxel_vertex_emb"]
    assert torch.equal(st["voxel_vertex_emb"].cpu(), ref)


def test_same_process_round_trip():
    s = ShareData()
    try:
        assert s.states is None and s.fetch("states") is None
        st = _states(3, 5000, "cuda")
        assert s.publish("states", st) == 1
        got, ver = s.fetch("states")
        assert ver == 1 and s.fetch("states", after=ver) is None
        for k in st:
            assert torch.equal(got[k], st[k]) and got[k].data_ptr() != st[k].data_ptr()
        st["voxel_vertex_emb"].add_(1)          # the snapshot is a copy: later writes do not leak into it
        assert not torch.equal(s.states["voxel_vertex_emb"], st["voxel_vertex_emb"])
        # a CPU tensor (the reference's .cpu() setters) goes up once
        s.voxels = torch.arange(12, dtype=torch.float32).view(3, 4)
        v = s.voxels
        assert v.is_cuda and torch.equal(v.cpu(), torch.arange(12, dtype=torch.float32).view(3, 4))
        s.hash_voxel = None
        assert s.hash_voxel is None and s.version("hash_voxel") == 1
    finally:
        s.close()


def test_decoder_module_round_trip_and_refresh():
    torch.manual_seed(0)
    dec = Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none").cuda()
    s = ShareData()
    try:
        s.decoder = dec
        got = s.decoder
        assert type(got) is Decoder and next(got.parameters()).is_cuda
        x = torch.randn(300, 16, device="cuda")
        with torch.no_grad():
            a, b = dec.get_values(x), got.get_values(x)
        assert torch.equal(a, b)
        # in-place refresh of an earlier copy when the writer moves on
        with torch.no_grad():
            for p in dec.parameters():
                p.mul_(0.5)
        ver = s.publish("decoder", dec)
        ptrs = [p.data_ptr() for p in got.parameters()]
        out = s.fetch("decoder", after=1, into=got)
        assert out[1] == ver and out[0] is got and [p.data_ptr() for p in got.parameters()] == ptrs
        for p, q in zip(dec.parameters(), got.parameters()):
            assert torch.equal(p, q)
        with pytest.raises(ValueError):   # layout changes need a fresh fetch
            s.publish("states", _states(1, 10, "cuda"))
            s.fetch("states", into={"voxel_center_xyz": torch.empty(11, 3, device="cuda"),
                                     "voxel_structure": torch.empty(10, 9, dtype=torch.int32, device="cuda"),
                                     "voxel_vertex_idx": torch.empty(10, 8, dtype=torch.int32, device="cuda"),
                                     "voxel_vertex_emb": torch.empty(20000, 16, device="cuda")})
    finally:
        s.close()


def _writer(share, n_versions, q):
    import torch as T
    T.cuda.set_device(0)
    try:
        n = 4000
        for v in range(1, n_versions + 1):
            if v % 5 == 0:
                n = int(n * 1.7)                 # the map grows: slots reallocate (new IPC handles)
            share.states = _states(v, n, "cuda")
        q.put(("done", n))
        t0 = time.time()
        while not share.stop_tracking and time.time() - t0 < 60:   # keep the slots alive until the reader is done
            time.sleep(0.01)
    except BaseException as e:  # noqa: BLE001
        q.put(("error", repr(e)))
    finally:
        share.close()


def test_cross_process_snapshots_are_consistent():
    s = ShareData()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    n_versions = 40
    p = ctx.Process(target=_writer, args=(s, n_versions, q))
    p.start()
    try:
        seen, last, t0 = [], 0, time.time()
        while last < n_versions and time.time() - t0 < 90:
            r = s.fetch("states", after=last)
            if r is None:
                time.sleep(0.001)
                continue
            st, ver = r
            _check_snapshot(st, ver)
            assert ver > last
            seen.append(ver)
            last = ver
        assert last == n_versions, (seen, q.get(timeout=5) if not q.empty() else None)
        status = q.get(timeout=60)
        assert status[0] == "done", status
        assert s.states["voxel_center_xyz"].shape[0] == status[1]
    finally:
        s.stop_tracking = True
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
        s.close()
    assert p.exitcode == 0
