"""Sharded == single-GPU on the same global batch: two ranks
sharing cuda:0 (gloo) each render their part of one room0 batch with
psvo.dist.GlobalBatch (global [200, K', P] sampler layout, global P /
max_steps, noise keyed by the global index), GlobalLossSums (batch-global
loss normalisers) and GradBucket("sum").  Against one process rendering the
whole batch: sample indices / depths are bit-identical row for row, the loss
agrees to f64-sum rounding and the gradients to fp32 summation order."""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_sharded_equals_single(tmp_path):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "dist_exact_worker.py"), str(tmp_path)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    single = torch.load(tmp_path / "single.pt", weights_only=True)
    ranks = [torch.load(tmp_path / f"rank{k}.pt", weights_only=True) for k in range(2)]
    row = 0
    for res in ranks:
        n = res["s_idx"].shape[0]
        assert res["P"] == single["P"] and res["max_steps"] == single["max_steps"]
        assert torch.equal(res["s_idx"], single["s_idx"][row:row + n])
        assert torch.equal(res["s_depth"], single["s_depth"][row:row + n])
        assert torch.equal(res["rank_ray"] + res["ray_off"], single["rank_ray"][row:row + n])
        assert torch.equal(res["z_vals"], single["z_vals"][row:row + n])  # padded to the global S_max
        torch.testing.assert_close(res["color"], single["color"][row:row + n], rtol=0, atol=2e-6)
        torch.testing.assert_close(res["depth"], single["depth"][row:row + n], rtol=0, atol=2e-5)
        row += n
    assert row == single["s_idx"].shape[0]
    for res in ranks:
        torch.testing.assert_close(res["loss"], single["loss"], rtol=1e-6, atol=0)
        for a, b in zip(res["grads"], single["grads"]):
            scale = float(b.abs().max()) + 1e-30
            assert float((a - b).abs().max()) <= 1e-4 * scale
