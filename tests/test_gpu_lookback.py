"""The in-launch look-back scans (csrc/lookback.h): helping and give-ups.

Since round 6 every look-back wait is for a workgroup that has started: a
waiter that finds a predecessor which has not started computes that block's
aggregate itself.  psvo_debug_set_lookback(mask, -1, delay_us) holds every
4th workgroup (and every tile's last) back at the chosen sites (1 traversal,
2 sampler, 4 sample selection) — as another queue's kernels holding the CUs
would — so that their successors help them: the results must be the same
bits, and the help counters must show that the path ran.  With a spin bound
of 0 every workgroup with a predecessor gives up at once: the engine must
then report the batch as failed — the traversal / sampler through the
query's statistics read-back, the sample selection (whose counts never reach
the host inside a step) at the engine's next read-back — write nothing out
of bounds, clear the report, and step normally once the bound is back."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _engine():
    from psvo import synthetic as syn
    from psvo.decoder import Decoder
    from psvo.engine import MappingEngine
    from psvo.octree import Octree, map_states
    from psvo.pose import OptimizablePose
    from oracle import oracle as O
    w = syn.make_workload("room0", 2, 512, seed=4)
    tree = Octree()
    tree.init(256, 16, 0.2, 8)
    tree.insert(w.voxels)
    g = torch.Generator().manual_seed(0)
    emb = (torch.randn(max(20000, tree.count_nodes()), 16, generator=g) * 0.1).to(DEV)
    torch.manual_seed(0)
    dec = Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none").to(DEV)
    crit = {"rgb_weight": 0.5, "depth_weight": 1.0, "sdf_weight": 5000.0, "fs_weight": 10.0}
    eng = MappingEngine(map_states(tree, emb, 0.2, device=DEV), dec, 0.2, 0.01, truncation=0.1, max_distance=10.0,
                        criteria=crit, max_depth=10.0)
    poses, dirs = [], []
    rd = w.rays_d[0].double()
    for f, T in enumerate(w.poses):
        p = OptimizablePose.from_matrix(np.asarray(T)).data.detach().double()
        poses.append(p.float())
        dirs.append((rd[f * 512:(f + 1) * 512] @ O.se3_rotation(p)).float())
    poses, dirs = torch.stack(poses).contiguous().to(DEV), torch.cat(dirs).contiguous().to(DEV)
    rgb, depth = w.rgb.reshape(-1, 3).to(DEV), w.depth.reshape(-1).to(DEV)

    def step(seed):
        loss = eng.step_frames(dirs, 512, poses.clone(), torch.zeros_like(poses), torch.zeros_like(poses), [0, 1],
                               1e-3, rgb, depth, seed=seed, apply_adam=False, want_loss=True)
        torch.cuda.synchronize()
        return float(loss)

    return eng, step


@pytest.fixture
def spin():
    from psvo import _lib as L
    yield lambda mask, bound, delay_us=0: L.call("psvo_debug_set_lookback", mask, bound, delay_us)
    L.call("psvo_debug_set_lookback", 0, -1, 0)


def _helps(reset=True):
    import ctypes
    from psvo import _lib as L
    out = (ctypes.c_int64 * 3)()
    L.call("psvo_debug_lb_helps", ctypes.cast(out, ctypes.c_void_p), int(reset))
    return list(out)


def test_unstarted_predecessors_are_helped_with_the_same_bits(spin):
    """Every 4th workgroup (and each tile's last) of all three look-back
    launches starts 300 µs late: the steps' losses, statistics and gradients
    equal an undelayed engine's bit for bit (gradients up to the order of the
    embedding scatter's float atomics), and each site helped."""
    eng, step = _engine()
    ref = [step(31 + i) for i in range(3)]
    ref_stats = list(eng.last_stats)
    ref_grad = eng.grad_flat.cpu().clone()
    eng.close()
    _helps(reset=True)
    spin(7, -1, 300)
    eng, step = _engine()
    got = [step(31 + i) for i in range(3)]
    spin(0, -1, 0)
    helps = _helps(reset=True)
    assert got == ref
    assert list(eng.last_stats)[:5] == ref_stats[:5]
    # (the embedding scatter's float atomics sum in arrival order: not bitwise)
    g = eng.grad_flat.cpu()
    torch.testing.assert_close(g, ref_grad, rtol=1e-4, atol=1e-6 * float(ref_grad.abs().max()))
    assert helps[0] > 0 and helps[1] > 0 and helps[2] > 0, helps
    eng.close()


@pytest.mark.parametrize("mask", [1, 2, 3])
def test_query_giveup_fails_the_step_and_recovers(spin, mask):
    from psvo._lib import PsvoError
    eng, step = _engine()
    ref = step(11)
    assert np.isfinite(ref)
    spin(mask, 0)
    with pytest.raises(PsvoError, match="look-back wait abandoned"):
        step(11)
    spin(0, -1)
    assert step(11) == ref  # descriptors re-zeroed, ticket counters consistent: the same bits
    assert eng.last_stats[1] > 0 and eng.last_stats[4] > 0
    eng.close()


def test_selection_giveup_is_reported_at_the_next_read_back(spin):
    from psvo._lib import PsvoError
    eng, step = _engine()
    ref = step(21)
    spin(4, 0)
    step(21)  # queued without a host round trip: the loss of dropped samples, no fault
    spin(0, -1)
    with pytest.raises(PsvoError, match="sample selection abandoned a look-back wait"):
        step(21)
    assert step(21) == ref  # reported once, cleared; the selection's descriptors re-zeroed
    eng.select_stats()  # nothing stale left in the counts either
    # the opt-in statistics call reports a give-up too, once
    spin(4, 0)
    step(21)
    spin(0, -1)
    with pytest.raises(RuntimeError, match="abandoned"):
        eng.select_stats()
    eng.select_stats()
    eng.close()


def test_many_launches_reuse_the_descriptors():
    """Tags keep the descriptor buffers valid without clearing: after 40 steps
    (three look-back launches each, on the same buffers) the engine still
    gives the loss a fresh engine gives on the same step."""
    eng, step = _engine()
    first = step(5)
    for it in range(40):
        step(100 + it)
    assert step(5) == first
    eng2, step2 = _engine()
    assert step2(5) == first
    eng.close()
    eng2.close()
