"""Data-parallel bundle_adjust_frames == one process on the union of the
keyframes: two ranks sharing cuda:0 over gloo each own two of
four room0 keyframes (tests/dist_ba_worker.py), three iterations with
recorded pixel picks, the same sampler seeds, pose updates and the
look-ahead query.  Against one process over all four keyframes: the same
union-batch loss every iteration (f64 partial-sum order), the same poses
(each rank steps the keyframes it owns), embeddings / decoder to Adam's
ulp-amplification bar, and replicas identical across ranks."""
import os
import socket
import subprocess
import sys

import pytest
import torch

from test_oracle_golden import adam_close

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("exchange", ["dense", "sparse"])
def test_bundle_adjust_sharded_keyframes_equal_single(tmp_path, exchange):
    """exchange "dense": one flat all-reduce of the gradient (room0's small
    table), the union row flags then taken from the summed gradient;
    "sparse": the row-sparse embedding exchange (config E's, forced here):
    each rank lists the rows its step marked, the union flags come from the
    exchanged lists — sparse-exact Adam on every rank, against one process
    running DENSE Adam (PSVO_SPARSE_ADAM=0)."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "dist_ba_worker.py"), str(tmp_path), exchange]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    single = torch.load(tmp_path / "single.pt", weights_only=True)
    ranks = [torch.load(tmp_path / f"rank{k}.pt", weights_only=True) for k in range(2)]
    for it, ls in enumerate(single["loss"]):
        for res in ranks:
            tol = 1e-6 if it == 0 else 1e-4
            assert abs(res["loss"][it] - ls) <= tol * abs(ls), (it, res["loss"][it], ls)
    for res in ranks:
        for f, p in res["poses"].items():
            torch.testing.assert_close(p, single["poses"][f], rtol=0, atol=1e-6)
    # replicas identical; the map against the single process (Adam bar)
    assert ranks[0]["modes"] == [exchange] and ranks[1]["modes"] == [exchange]
    assert ranks[0]["flags"] is not None and torch.equal(ranks[0]["flags"], ranks[1]["flags"])
    assert int(ranks[0]["flags"].sum()) < ranks[0]["flags"].numel()  # sparse: not every row stepped
    assert torch.equal(ranks[0]["emb"], ranks[1]["emb"])
    assert all(torch.equal(a, b) for a, b in zip(ranks[0]["dec"], ranks[1]["dec"]))
    bound = 2.0 * 5e-3 * len(single["loss"])
    e1, e0 = ranks[0]["emb"], single["emb"]
    adam_close(e1.numpy(), e0.numpy(), tight=1e-5, frac=0.97, max_abs=bound)
    for a, b in zip(ranks[0]["dec"], single["dec"]):
        adam_close(a.numpy(), b.numpy(), tight=1e-4, frac=0.99, max_abs=bound)
