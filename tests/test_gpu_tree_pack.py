"""Packed octree records (csrc/tree_pack.hip) and the packed traversal
(k_intersect_sorted<PACKED>): the breadth-first records carry exactly the
reference arrays' centres / sides / child lists (every node once, siblings
contiguous in child-slot order, the root first), and the traversal over them
returns the reference-layout traversal's hits bit for bit — ids, t_in,
t_out, counts, Σ(t_out − t_in), visit counts — at configs B and E (2.7 M
nodes), on the engine's query path as well."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _pack(ms):
    from psvo import _lib as L
    c = ms["voxel_center_xyz"].float().contiguous()
    s = ms["voxel_structure"].int().contiguous()
    n = c.shape[0]
    packed = torch.empty(n * 32, dtype=torch.uint8, device=DEV)
    ws = torch.empty(int(L.lib().psvo_pack_tree_workspace_ints(n)), dtype=torch.int32, device=DEV)
    L.call("psvo_pack_tree", L.stream_of(c.device), n, c, s, ws, packed)
    return packed, c, s


def _intersect(ms, ro, rd, vs, step, packed=None):
    from psvo import _lib as L
    c = ms["voxel_center_xyz"].float().contiguous()
    s = ms["voxel_structure"].int().contiguous()
    R = ro.shape[0]
    out = dict(idx=torch.empty(R, 50, dtype=torch.int32, device=DEV), t0=torch.empty(R, 50, device=DEV),
               t1=torch.empty(R, 50, device=DEV), nv=torch.empty(R, dtype=torch.int32, device=DEV),
               ds=torch.empty(R, device=DEV), st=torch.zeros(16, dtype=torch.int32, device=DEV))
    if packed is None:
        L.call("psvo_ray_intersect_sorted", L.stream_of(ro.device), R, ro, rd, c, s, float(vs), 10.0, float(step),
               out["idx"], out["t0"], out["t1"], out["nv"], out["ds"], out["st"])
    else:
        L.call("psvo_ray_intersect_sorted_packed", L.stream_of(ro.device), R, ro, rd, packed, c, s, float(vs), 10.0,
               float(step), out["idx"], out["t0"], out["t1"], out["nv"], out["ds"], out["st"])
    torch.cuda.synchronize()
    return {k: v.cpu() for k, v in out.items()}


@pytest.mark.parametrize("name", ["B", "E"])
def test_packed_records_and_traversal(name):
    import test_gpu_fullsize_parity as F
    c, w, ms, _ = F._setup(name)
    packed, cen, st = _pack(ms)
    torch.cuda.synchronize()
    n = cen.shape[0]
    rec = packed.cpu().numpy().view(np.int32).reshape(n, 8)
    recf = packed.cpu().numpy().view(np.float32).reshape(n, 8)
    S = st.cpu().numpy()
    C = cen.cpu().numpy()
    # the nodes reachable from the root (the corner FEATURE nodes that only
    # carry vertex embeddings are in no child list and get no record)
    reach, lvl = [np.array([0])], np.array([0])
    while lvl.size:
        k = S[lvl, :8]
        lvl = k[k > -1]
        reach.append(lvl)
    starts = np.cumsum([0] + [r.size for r in reach])  # first record of each level
    reach = np.concatenate(reach)
    m = reach.size
    assert np.unique(reach).size == m
    rec, recf = rec[:m], recf[:m]
    ref_id, first, mask = rec[:, 4], rec[:, 5], rec[:, 6]
    assert ref_id[0] == 0  # the root first
    assert np.array_equal(ref_id, reach)  # breadth-first, every reachable node once
    assert np.array_equal(recf[:, :3], C[ref_id])  # same centre floats
    assert np.array_equal(rec[:, 3], S[ref_id, 8])  # same side
    # child lists: present children of the reference row, in slot order, at first + rank
    kids = S[ref_id, :8]
    present = kids > -1
    assert np.array_equal(mask, (present * (1 << np.arange(8))).sum(1))
    cnt = present.sum(1)
    has = cnt > 0
    assert np.all(first[~has] == -1)
    # siblings contiguous: the child blocks tile [1, m) in parent order
    assert first[has][0] == 1 and np.all(first[has][1:] == first[has][:-1] + cnt[has][:-1])
    assert first[has][-1] + cnt[has][-1] == m
    ch = cnt[has]
    pos = np.repeat(first[has] - (np.cumsum(ch) - ch), ch) + np.arange(ch.sum())
    child_ref = ref_id[pos]
    assert np.array_equal(child_ref, kids[has][present[has]])
    # spare word (the traversal's top start): the parent record for records
    # 1..127, 0 beyond; the root's = n_top | m << 16 with m the deepest level
    # >= 2 with <= 128 records above it, none a leaf (0: start at the root)
    parent = np.zeros(m, dtype=np.int64)
    parent[pos] = np.repeat(np.nonzero(has)[0], ch)
    top = min(m, 128)
    assert np.array_equal(rec[1:top, 7], parent[1:top])
    assert np.all(rec[top:, 7] == 0)
    word = 0
    for lv in range(2, len(starts)):
        n = starts[lv]
        if n > 128 or np.any(rec[:n, 3] == 1) or starts[lv] == starts[lv - 1]:
            break
        word = n | lv << 16
    assert rec[0, 7] == word and word > 0
    # traversal: bit-exact to the reference-layout kernel
    ro = w.rays_o.reshape(-1, 3).to(DEV).contiguous()
    rd = w.rays_d.reshape(-1, 3).to(DEV).contiguous()
    a = _intersect(ms, ro, rd, w.scene.voxel_size, c["step"])
    b = _intersect(ms, ro, rd, w.scene.voxel_size, c["step"], packed)
    for k in ("idx", "t0", "t1", "nv", "ds"):
        assert torch.equal(a[k], b[k]), k
    # P, R_hit, max ceil, spills, flags; the AABB-test count (a diagnostic)
    # may differ: the packed walk tests the top levels in full before any
    # prune can apply, the reference-layout one in key-ordered rounds, and
    # the packed walk's two-chunk rounds test a second chunk before the first
    # chunk's leaves can set the prune bound (config E: ≈ +2 %)
    keep = [0, 1, 2, 3, 4, 6, 7]
    assert torch.equal(a["st"][keep], b["st"][keep])
    va, vb = int(a["st"][5]), int(b["st"][5])
    assert abs(va - vb) <= 0.05 * va, (va, vb)
    assert int(a["st"][6]) == 0  # no serial-DFS fallback on either side


def test_engine_packed_query_matches_reference_layout(monkeypatch):
    """One engine step with the packed traversal equals one with the
    reference arrays: statistics and the updated decoder bit for bit."""
    import test_gpu_fullsize_parity as F
    from psvo.decoder import Decoder
    from psvo.engine import MappingEngine
    c, w, ms, _ = F._setup("B")
    res = []
    for flag in ("0", "1"):
        monkeypatch.setenv("PSVO_PACKED", flag)
        torch.manual_seed(0)
        dec = Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none").to(DEV)
        emb = ms["voxel_vertex_emb"].clone()
        eng = MappingEngine(dict(ms, voxel_vertex_emb=emb), dec, w.scene.voxel_size, c["step"])
        assert (eng.packed is not None) == (flag == "1")
        loss = eng.step(w.rays_o.to(DEV), w.rays_d.to(DEV), w.rgb.to(DEV), w.depth.to(DEV), seed=5)
        torch.cuda.synchronize()
        res.append((float(loss), eng.last_stats[:8], [p.detach().clone() for p in dec.parameters()]))
        eng.close()
    assert res[0][0] == res[1][0]
    assert res[0][1] == res[1][1]
    assert all(torch.equal(x, y) for x, y in zip(res[0][2], res[1][2]))
