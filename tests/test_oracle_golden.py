"""Pin the CPU oracle to golden vectors produced by the reference's own Python
path (tests/golden/make_golden.py).  CPU only."""
import pytest
import numpy as np
import torch

from conftest import load_golden
from oracle import oracle as O


def _decoder_params(g):
    return {k[len("dec."):]: torch.from_numpy(v) for k, v in g.items() if k.startswith("dec.")}


def _run_oracle(g):
    ms = O.map_states_from_export(g["voxels"], g["children"], g["features"], float(g["voxel_size"]),
                                  torch.from_numpy(g["embeddings"]))
    crit = dict(zip(("rgb_weight", "depth_weight", "fs_weight", "sdf_weight"), g["crit"].tolist()))
    return O.render_and_backward(torch.from_numpy(g["rays_o"]), torch.from_numpy(g["rays_d"]),
                                 torch.from_numpy(g["rgb"]), torch.from_numpy(g["depth_gt"]), ms, _decoder_params(g),
                                 float(g["step_size"]), float(g["voxel_size"]), float(g["truncation"]),
                                 float(g["max_depth"]), crit, noise=torch.from_numpy(g["noise"]))


def test_octree_export_matches_golden(golden):
    _, g = golden
    t = O.OracleOctree(int(g["grid_dim"]))
    t.insert(g["vox"])
    v, c, f = t.export()
    np.testing.assert_array_equal(v, g["voxels"])
    np.testing.assert_array_equal(c, g["children"])
    np.testing.assert_array_equal(f, g["features"])


def test_map_states_match_golden(golden):
    _, g = golden
    ms = O.map_states_from_export(g["voxels"], g["children"], g["features"], 0.2, None)
    np.testing.assert_array_equal(ms["voxel_center_xyz"].numpy(), g["centres"])
    np.testing.assert_array_equal(ms["voxel_structure"].numpy(), g["structure"])


def test_intersection_matches_golden(golden):
    _, g = golden
    out, hits = O.ray_intersect_vox(torch.from_numpy(g["rays_o"]), torch.from_numpy(g["rays_d"]),
                                    torch.from_numpy(g["centres"]), torch.from_numpy(g["structure"]), 0.2, 10.0)
    np.testing.assert_array_equal(out["intersected_voxel_idx"].numpy(), g["hit_idx"])
    np.testing.assert_array_equal(out["min_depth"].numpy(), g["hit_min"])
    np.testing.assert_array_equal(out["max_depth"].numpy(), g["hit_max"])
    np.testing.assert_array_equal(hits.numpy(), g["hits"])


def test_render_and_grads_match_golden(golden):
    name, g = golden
    out, loss, parts, grads = _run_oracle(g)
    # integer / index work and the sampler are bit-exact
    np.testing.assert_array_equal(out["ray_mask"].numpy(), g["ray_mask"])
    np.testing.assert_array_equal(out["z_vals"].detach().numpy(), g["z_vals"])
    # fp32 paths: same torch-CPU ops, only reduction order may differ
    tol = dict(rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(out["sdf"].detach().numpy(), g["sdf"], **tol)
    np.testing.assert_allclose(out["weights"].detach().numpy(), g["weights"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(out["color"].detach().numpy(), g["color"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(out["depth"].detach().numpy(), g["depth"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(float(loss), float(g["loss"]), rtol=1e-5)
    for k, ref in (("embeddings", g["grad_embeddings"]), ("rays_o", g["grad_rays_o"]), ("rays_d", g["grad_rays_d"])):
        got = grads[k].numpy()
        scale = np.abs(ref).max() + 1e-12
        assert np.abs(got - ref).max() <= 1e-4 * scale, (name, k, np.abs(got - ref).max(), scale)
    for k in [k for k in g if k.startswith("grad_dec.")]:
        got = grads[k[len("grad_dec."):]].numpy()
        ref = g[k]
        scale = np.abs(ref).max() + 1e-12
        assert np.abs(got - ref).max() <= 1e-4 * scale, (name, k, np.abs(got - ref).max(), scale)


def test_sampler_known_answer_slot_quirk():
    """SURVEY §8a-8, measured on the reference kernel: eight identical 2-hit
    rays launched as one K'=8 block give 10 valid samples in slots 0-3 and 9
    in the later slots (the trailing segment is only emitted when
    j*P + bin < K')."""
    b, k, p = 1, 8, 2
    idx = np.tile(np.array([5, 9], np.int32), (b, k, 1))
    lo = np.tile(np.array([1.0, 1.4], np.float32), (b, k, 1))
    hi = np.tile(np.array([1.2, 1.6], np.float32), (b, k, 1))
    probs = np.tile(np.array([0.5, 0.5], np.float32), (b, k, 1))
    steps = np.full((b, k), 8.0, np.float32)
    ms = 8 + p
    noise = np.full((b, k, ms), 0.5, np.float32)
    o_idx = np.full((b, k, ms), -1, np.int32)
    o_dep = np.zeros((b, k, ms), np.float32)
    o_dis = np.zeros((b, k, ms), np.float32)
    O.lib().oracle_inverse_cdf(b, k, p, ms, -1.0, *(O._ptr(a) for a in (idx, lo, hi, noise, probs, steps,
                                                                         o_idx, o_dep, o_dis)))
    counts = (o_idx[0] != -1).sum(-1)
    assert counts.tolist() == [10, 10, 10, 10, 9, 9, 9, 9]


def test_sampler_done_case_reads_next_slot():
    """When a ray's hits fill all P columns and its bins run out inside the
    main loop, the trailing emission takes pts_idx[H + P] = the NEXT slot's
    first voxel id (sample_gpu.cu:224-226), only while j*P + P < K'."""
    b, k, p = 1, 4, 1
    idx = np.array([[[3], [7], [11], [13]]], np.int32)
    lo = np.full((b, k, p), 1.0, np.float32)
    hi = np.full((b, k, p), 1.1, np.float32)
    probs = np.ones((b, k, p), np.float32)
    steps = np.full((b, k), 3.5, np.float32)   # ceil → 4 steps; the 4th cdf > 1 exhausts the bins
    ms = 4 + p
    noise = np.full((b, k, ms), 0.999, np.float32)
    o_idx = np.full((b, k, ms), -1, np.int32)
    o_dep = np.zeros((b, k, ms), np.float32)
    o_dis = np.zeros((b, k, ms), np.float32)
    O.lib().oracle_inverse_cdf(b, k, p, ms, -1.0, *(O._ptr(a) for a in (idx, lo, hi, noise, probs, steps,
                                                                         o_idx, o_dep, o_dis)))
    assert o_idx[0].tolist() == [[3, 3, 3, 3, 7], [7, 7, 7, 7, 11], [11, 11, 11, 11, 13], [13, 13, 13, 13, -1]]


BA_GOLDENS = ["BA_room0", "BA_room0_resnet", "BA_scannet_w256"]


def ba_settings(g):
    """(criteria dict, max_depth = max_distance) of a BA golden (mapping.py:61)."""
    from oracle import oracle as O
    if "crit" not in g:
        return dict(O.REPLICA_CRITERIA), 10.0
    names = ("rgb_weight", "depth_weight", "fs_weight", "sdf_weight")
    return dict(zip(names, (float(x) for x in g["crit"]))), float(g["max_depth"])


def _ba_inputs(name="BA_room0"):
    g = load_golden(name)
    n = int(g["n_nodes"])
    torch.manual_seed(int(g["emb_seed"]))
    emb0 = torch.randn(n, 16) * float(g["emb_std"])
    assert float(emb0.double().sum()) == float(g["emb0_checksum"])
    ms = {"voxel_vertex_idx": torch.from_numpy(g["features"]), "voxel_center_xyz": torch.from_numpy(g["centres"]),
          "voxel_structure": torch.from_numpy(g["structure"]), "voxel_vertex_emb": emb0}
    frames = [(torch.from_numpy(g[f"frame{i}.rays_d"]), torch.from_numpy(g[f"frame{i}.rgb"]),
               torch.from_numpy(g[f"frame{i}.depth"])) for i in range(3)]
    iters = int(g["iters"])
    picks = [[g[f"pick{it}.{i}"] for i in range(3)] for it in range(iters)]
    noises = [g[f"noise{it}"] for it in range(iters)]
    dec0 = {k[5:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("dec0.")}
    return g, emb0, ms, frames, picks, noises, dec0


@pytest.mark.parametrize("name", BA_GOLDENS)
def test_oracle_bundle_adjust_matches_reference(name):
    """The oracle's bundle_adjust_frames restatement (poses included) against
    the reference's own runs (BA_*: room0 W = 128, the same with the points
    encoder passed as Mapping.do_mapping passes it, ScanNet W = 256): losses
    of all 3 iterations, final keyframe poses (the first, stamp 0,
    unchanged), embeddings, decoder."""
    from oracle import oracle as O
    g, emb0, ms, frames, picks, noises, dec0 = _ba_inputs(name)
    crit, max_depth = ba_settings(g)
    losses, emb1, dec1, poses1 = O.bundle_adjust(frames, picks, noises, ms, dec0, g["pose0"], g["stamps"],
                                                 float(g["step_size"]), 0.2, int(g["iters"]), criteria=crit,
                                                 max_distance=max_depth)
    if "resnet_optim_states" in g:  # the encoder never gets a gradient: Adam never creates state for it
        assert int(g["resnet_optim_states"]) == 0 and bool(g["res_unchanged"])
    np.testing.assert_allclose(losses, g["losses"], rtol=1e-5)
    # W = 256: one pose element 5e-6 off (0.5 % of the pose lr) — summation order of the wider decoder's
    # per-sample terms, amplified by Adam's normalised step
    np.testing.assert_allclose(poses1.numpy(), g["poses1"], rtol=0, atol=1e-6 if name.startswith("BA_room0") else 1e-5)
    assert np.array_equal(poses1.numpy()[0], g["pose0"][0])
    rows = torch.from_numpy(g["emb_changed_rows"])
    changed = torch.nonzero((emb1 != emb0).any(-1)).squeeze(1)
    assert torch.equal(changed, rows)
    if name.startswith("BA_room0"):
        adam_close(emb1[rows].numpy(), g["emb1_changed"])
        for k, v in dec1.items():
            adam_close(v.numpy(), g["dec1." + k])
    else:
        # W = 256 (torch-CPU GEMMs of other shapes sum in another order than the reference's): measured
        # 98.8 % of embedding elements within 1e-6 / 99.6 % within 1e-5, the worst 0.16 lr (a near-zero
        # gradient's sign); decoder all but 2 elements within 1e-4
        adam_close(emb1[rows].numpy(), g["emb1_changed"], tight=1e-5, frac=0.99, max_abs=2 * 5e-3)
        for k, v in dec1.items():
            adam_close(v.numpy(), g["dec1." + k], tight=1e-4, frac=0.999, max_abs=2 * 5e-3)


def adam_close(got, ref, lr=5e-3, tight=1e-6, frac=0.98, max_abs=None):
    """Parameters after a few Adam steps.  Adam's step m / (sqrt(v) + eps) is
    ±lr for any gradient well above eps = 1e-8 whatever its size, so an
    element whose gradient is near zero (cancelling sums) moves by up to lr
    in either direction depending on rounding: a different summation order
    (float atomics on the GPU, torch-CPU here) flips a few of them.  The bar:
    >= frac of the elements (all but 2, for tiny tensors) within `tight`, every element within max_abs
    (default 0.1 lr: CPU-vs-CPU differences stay below a full step)."""
    d = np.abs(np.asarray(got, np.float64) - np.asarray(ref, np.float64))
    assert d.max() <= (0.1 * lr if max_abs is None else max_abs), d.max()
    # small tensors (biases, the rgb head): up to 2 flipped elements however few there are
    n_out = int((d > tight).sum())
    assert n_out <= max(2, (1.0 - frac) * d.size), ((d <= tight).mean(), n_out, d.size)


def test_oracle_pixel_sampling_matches_reference():
    """oracle.sample_rays against the reference's own sample_util.sample_rays
    (tests/golden/P_pixels.npz, make_golden_pixels.py): with the uniforms its
    torch.rand_like drew, the same picked pixels — uniform frame, a 0/1 mask
    over two frames (one joint sum), fractional weights."""
    from oracle import oracle as O
    g = load_golden("P_pixels")
    for c in range(int(g["n_cases"])):
        idx = O.sample_rays(g[f"case{c}.mask"], int(g[f"case{c}.n"]), g[f"case{c}.u"])
        assert np.array_equal(idx, g[f"case{c}.idx"]), c


def test_oracle_pixel_uniforms_are_uniform():
    from oracle import oracle as O
    u = O.pixel_uniforms(12345, 2, 100000)
    assert u.dtype == np.float32 and u.min() >= 0.0 and u.max() < 1.0
    assert abs(float(u.mean()) - 0.5) < 0.005
    assert not np.array_equal(u[0], u[1])


def test_track_frame_matches_reference_golden():
    """The oracle's tracking loop (render + Criterion with the median depth
    filter + pose Adam) against the reference's own track_frame with
    depth_variance=True (tests/golden/T_track.npz, tracking.py:130-147): the
    per-iteration losses, the final pose and the hit mask."""
    g = load_golden("T_track")
    ms = O.map_states_from_export(g["voxels"], g["children"], g["features"], float(g["voxel_size"]),
                                  torch.from_numpy(g["embeddings"]))
    iters = int(g["iters"])
    assert (g["depth_filter_dropped"] > 0).all()  # the median filter is exercised on every iteration
    losses, pose, hit = O.track_frame(torch.from_numpy(g["rays_d"]), torch.from_numpy(g["rgb"]),
                                      torch.from_numpy(g["depth"]), [g[f"pick{i}"] for i in range(iters)],
                                      [g[f"noise{i}"] for i in range(iters)], ms, _decoder_params(g), g["pose0"],
                                      float(g["step_size"]), float(g["voxel_size"]), iters, lr=float(g["lr"]),
                                      truncation=float(g["truncation"]), max_distance=float(g["max_distance"]),
                                      max_depth=float(g["max_depth"]), weight_depth_loss=True)
    np.testing.assert_allclose(losses, g["losses"], rtol=1e-5)
    # 1 % of one Adam step (lr 1e-3): the pose gradient's summation order (a few ulps at |t| ≈ 11)
    np.testing.assert_allclose(pose.numpy(), g["pose1"], rtol=0, atol=1e-5)
    np.testing.assert_array_equal(hit.numpy(), g["hit_mask"])
