"""psvo_interp_bwd_chunked (64-sample work units, engine path) vs
psvo_interp_bwd (one wave per ray) on the same room0 samples: the same
embedding gradient and d_o / d_d up to fp32 summation order, across step
sizes that give short and very long rays (S_max up to several hundred)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("step", [0.02, 0.004])
def test_chunked_interp_bwd_matches(step):
    from psvo import _lib as L
    from psvo import synthetic as syn
    from psvo.octree import Octree, map_states
    from psvo.render_helpers import query_samples
    w = syn.make_workload("room0", 2, 512, seed=9)
    tree = Octree()
    tree.init(256, 16, 0.2, 8)
    tree.insert(w.voxels)
    g = torch.Generator().manual_seed(1)
    emb = (torch.randn(max(20000, tree.count_nodes()), 16, generator=g) * 0.1).to(DEV)
    ms = map_states(tree, emb, 0.2, device=DEV)
    ro, rd = w.rays_o.to(DEV), w.rays_d.to(DEV)
    q = query_samples(ro, rd, ms, step, 0.2, 10.0, seed=3)
    R = ro.numel() // 3
    assert q.s_max > 64  # long rays span several work units
    gf = torch.randn(q.m, 16, generator=g).to(DEV)
    args = (q.offsets, q.rank_ray32, q.leaf, q.t, ro, rd, ms["voxel_center_xyz"], ms["voxel_vertex_idx"], emb, gf)
    ge_a, go_a, gd_a = torch.zeros_like(emb), torch.zeros(R, 3, device=DEV), torch.zeros(R, 3, device=DEV)
    L.call("psvo_interp_bwd", L.stream_of(DEV), q.r_hit, 16, 0.2, *args, ge_a, go_a, gd_a)
    ge_b, go_b, gd_b = torch.zeros_like(emb), torch.zeros(R, 3, device=DEV), torch.zeros(R, 3, device=DEV)
    ws = torch.empty(int(L.lib().psvo_interp_bwd_workspace_floats(q.r_hit, q.s_max)), device=DEV)
    L.call("psvo_interp_bwd_chunked", L.stream_of(DEV), q.r_hit, q.s_max, 16, 0.2, *args, ge_b, go_b, gd_b, ws)
    torch.cuda.synchronize()
    for a, b in ((ge_a, ge_b), (go_a, go_b), (gd_a, gd_b)):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-5 * float(a.abs().max()))
