"""Generate golden fixtures from the REFERENCE Python path (container only).

Runs /root/reference/src/variations/render_helpers.render_rays, the
reference Criterion and loss.backward() on small seeded inputs and stores
inputs, intermediates, outputs and gradients as .npz files in this directory.

The reference's `grid` CUDA extension cannot be built in this image (it needs
cuda.h / ATen-CUDA headers), so a stand-in `grid` module backed by the
oracle's C restatement (oracle/svo_oracle.c) is installed in sys.modules;
everything ABOVE the two kernels — batching/padding, sort/trim, probs/steps,
sampler host wrapper, interpolation, decoder, compositing, loss, autograd —
is the reference's own code.  Modules the path does not use (open3d, annoy,
tensorboardX) are replaced by empty stubs, torch.Tensor.cuda by identity
(CPU-only torch), and the reference's per-call np.savetxt debug dumps land in
a temp dir.  Noise drawn inside InverseCDFRaySampling is recorded so the
build can inject the same noise.

BA_*.npz: the reference's bundle_adjust_frames (3 keyframes, 3 iterations,
pose Adam on the non-first keyframes) — see run_ba_case / BA_CASES: room0
at W = 128, the same with the points encoder + its optimiser passed as
Mapping.do_mapping passes them, and ScanNet settings at W = 256.

T_track.npz: the reference's track_frame with depth_variance=True (the call
Tracking.do_tracking makes): per-iteration losses, noise and picks, the
median depth filter's dropped rays, the final pose and hit mask.

M_mesh_A.npz: the reference's get_scores / eval_points (mesh extraction's
lattice scores and vertex colours) on the A octree's first 40 SURFACE voxels.

Usage:  python tests/golden/make_golden.py [case ...]   (writes tests/golden/<case>.npz; all by default)
"""
from __future__ import annotations

import os
import sys
import tempfile
import types

sys.dont_write_bytecode = True  # never write into /root/reference

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "proud-slam_amd"))

from oracle import oracle as O  # noqa: E402
from psvo import synthetic as syn  # noqa: E402

OUT_DIR = os.path.dirname(os.path.abspath(__file__))


# ---------------------------------------------------------------- stubs
def _install_stubs(noise_log):
    for name in ("open3d", "tensorboardX", "annoy"):
        m = types.ModuleType(name)
        sys.modules[name] = m
    sys.modules["annoy"].AnnoyIndex = object
    sys.modules["tensorboardX"].SummaryWriter = object

    grid = types.ModuleType("grid")

    def svo_intersect(ray_start, ray_dir, points, children, voxelsize, n_max):
        B, K, _ = ray_start.shape
        # the reference replicates the tree B times; every copy is identical
        idx, t0, t1, _ = O.svo_intersect_flat(ray_start.reshape(-1, 3).numpy(), ray_dir.reshape(-1, 3).numpy(),
                                              points[0].contiguous().numpy(), children[0].contiguous().numpy(),
                                              voxelsize, n_max)
        return (torch.from_numpy(idx).reshape(B, K, n_max), torch.from_numpy(t0).reshape(B, K, n_max),
                torch.from_numpy(t1).reshape(B, K, n_max))

    def inverse_cdf_sampling(pts_idx, min_depth, max_depth, noise, probs, steps, fixed_step_size):
        b, k, p = pts_idx.shape
        ms = noise.shape[-1]
        noise_log.append(noise.clone())
        o_idx = np.full((b, k, ms), -1, np.int32)
        o_dep = np.zeros((b, k, ms), np.float32)
        o_dis = np.zeros((b, k, ms), np.float32)
        c = lambda t, dt: np.ascontiguousarray(t.numpy(), dtype=dt)
        O.lib().oracle_inverse_cdf(b, k, p, ms, float(fixed_step_size), O._ptr(c(pts_idx, np.int32)),
                                   O._ptr(c(min_depth, np.float32)), O._ptr(c(max_depth, np.float32)),
                                   O._ptr(c(noise, np.float32)), O._ptr(c(probs, np.float32)),
                                   O._ptr(c(steps, np.float32)), O._ptr(o_idx), O._ptr(o_dep), O._ptr(o_dis))
        return torch.from_numpy(o_idx), torch.from_numpy(o_dep), torch.from_numpy(o_dis)

    grid.svo_intersect = svo_intersect
    grid.inverse_cdf_sampling = inverse_cdf_sampling
    sys.modules["grid"] = grid
    torch.Tensor.cuda = lambda self, *a, **k: self
    sys.path.insert(0, os.path.join(REF, "src"))


def _reference_modules():
    import importlib
    rh = importlib.import_module("variations.render_helpers")
    nrgbd = importlib.import_module("variations.nrgbd")
    crit = importlib.import_module("criterion")
    return rh, nrgbd, crit


# ---------------------------------------------------------------- cases
def _octree(vox, grid_dim):
    t = O.OracleOctree(grid_dim)
    t.insert(vox)
    v, c, f = t.export()
    t.close()
    return v, c, f


def case_inputs(name):
    """Seeded inputs for each golden case."""
    g = np.random.default_rng(0)
    if name == "A_voxels_center":
        # the reference's only data fixture (875 real voxel centres, +10 m
        # offset) translated into a depth-6 (grid 64) octree — SURVEY §8d A.
        pts = np.loadtxt(os.path.join(REF, "src/variations/voxels_center.txt"))
        key = np.round(pts / 0.2).astype(np.int64)
        key = key - key.min(0) + 1
        vox, grid_dim = key.astype(np.int32), 64
        centre = (key.mean(0) + 0.5) * 0.2
        eye = centre + np.array([-2.5, -0.6, 0.4])
        T = syn.look_at(eye, centre)
        scene = syn.Scene([], grid_dim=grid_dim)
        K = scene.intrinsics
        gen = torch.Generator().manual_seed(0)
        pix = syn.gumbel_topk_pixels(K["H"], K["W"], 1024, gen).numpy()
        u, v = (pix % K["W"]).astype(np.float64), (pix // K["W"]).astype(np.float64)
        d = np.stack([(u - K["cx"]) / K["fx"], (v - K["cy"]) / K["fy"], np.ones_like(u)], -1).astype(np.float32)
        rd = d @ T[:3, :3].astype(np.float32).T
        ro = np.broadcast_to(T[:3, 3].astype(np.float32), rd.shape).copy()
        depth = g.uniform(1.5, 4.0, (1, 1024)).astype(np.float32)
        rgb = g.uniform(0, 1, (1, 1024, 3)).astype(np.float32)
        return dict(vox=vox, grid_dim=grid_dim, rays_o=ro[None], rays_d=rd[None], rgb=rgb, depth=depth,
                    step=0.02, width=128, emb_std=0.3, crit="replica", deterministic=False)
    if name in ("B_room0_small", "B_room0_det"):
        w = syn.make_workload("room0", n_frames=1, rays_per_frame=384, seed=3)
        ro, rd = w.rays_o.numpy(), w.rays_d.numpy()
        # grazing rays inside the floor voxel layer: > 50 leaf hits, DFS-order truncation
        n_graze = 8
        o = np.array([10.05, 10.07, 10.1], np.float32) + np.linspace(0, 0.06, n_graze)[:, None].astype(np.float32)
        dd = np.array([0.8, 0.6, 0.0], np.float32)[None].repeat(n_graze, 0)
        dd[:, 1] += np.linspace(0, 0.04, n_graze).astype(np.float32)
        ro = np.concatenate([ro, o[None]], 1)
        rd = np.concatenate([rd, dd[None]], 1)
        rgb = np.concatenate([w.rgb.numpy(), g.uniform(0, 1, (1, n_graze, 3)).astype(np.float32)], 1)
        depth = np.concatenate([w.depth.numpy(), np.full((1, n_graze), 3.0, np.float32)], 1)
        return dict(vox=w.voxels, grid_dim=256, rays_o=ro, rays_d=rd, rgb=rgb, depth=depth,
                    step=0.02 if name == "B_room0_small" else 0.012, width=128, emb_std=0.3, crit="replica",
                    deterministic=(name == "B_room0_det"))
    if name == "C_scannet_small":
        w = syn.make_workload("scannet0000", n_frames=1, rays_per_frame=256, seed=5)
        return dict(vox=w.voxels, grid_dim=256, rays_o=w.rays_o.numpy(), rays_d=w.rays_d.numpy(),
                    rgb=w.rgb.numpy(), depth=w.depth.numpy(), step=0.02, width=256, emb_std=0.3, crit="scannet",
                    deterministic=False)
    raise KeyError(name)


CASES = ["A_voxels_center", "B_room0_small", "B_room0_det", "C_scannet_small"]


def run_case(name, rh, nrgbd, crit_mod, noise_log):
    inp = case_inputs(name)
    voxels, children, features = _octree(inp["vox"], inp["grid_dim"])
    n_nodes = voxels.shape[0]
    torch.manual_seed(1234)
    emb = (torch.randn(n_nodes, 16) * inp["emb_std"]).requires_grad_(True)
    dec = nrgbd.Decoder(depth=2, width=inp["width"], in_dim=16, skips=[], embedder="none", multires=0)
    # map_states exactly as Mapping.update_grid_pcd_features builds them (mapping.py:328-377)
    vt = torch.from_numpy(voxels)
    centres = (vt[:, :3] + vt[:, -1:] / 2) * 0.2
    structure = torch.cat([torch.from_numpy(children), vt[:, -1:]], -1).int()
    map_states = {"voxel_vertex_idx": torch.from_numpy(features), "voxel_center_xyz": centres.float(),
                  "voxel_structure": structure, "voxel_vertex_emb": emb}
    ro = torch.from_numpy(np.ascontiguousarray(inp["rays_o"], np.float32)).requires_grad_(True)
    rd = torch.from_numpy(np.ascontiguousarray(inp["rays_d"], np.float32)).requires_grad_(True)
    args = types.SimpleNamespace(
        criteria={**(O.REPLICA_CRITERIA if inp["crit"] == "replica" else O.SCANNET_CRITERIA), "sdf_truncation": 0.1},
        data_specs={"max_depth": 10.0 if inp["crit"] == "replica" else 5.0})
    criterion = crit_mod.Criterion(args)
    noise_log.clear()
    torch.manual_seed(99)
    # deterministic=True is not reachable through render_rays (ray_sample passes
    # fixed=False); the det case calls the same path with noise forced to 0.5.
    if inp["deterministic"]:
        orig = torch.Tensor.uniform_
        torch.Tensor.uniform_ = lambda self, *a, **k: self.fill_(0.5)
    try:
        out = rh.render_rays(ro, rd, map_states, dec, None, inp["step"], 0.2, 0.1, 10, args.data_specs["max_depth"])
    finally:
        if inp["deterministic"]:
            torch.Tensor.uniform_ = orig
    rgb_gt = torch.from_numpy(inp["rgb"])
    depth_gt = torch.from_numpy(inp["depth"])
    loss, parts = criterion(out, (rgb_gt, depth_gt))
    loss.backward()
    noise = torch.cat(noise_log, 1).numpy() if len(noise_log) > 1 else noise_log[0].numpy()
    # also record the raw DFS hits and sorted/trimmed intersection
    from variations import voxel_helpers as vh
    inter, hits = vh.ray_intersect_vox(ro.detach(), rd.detach(), centres, structure, 0.2, 10, 10.0)
    raw_idx, raw_t0, raw_t1, visits = O.svo_intersect_flat(inp["rays_o"], inp["rays_d"], centres.numpy(),
                                                           structure.numpy(), 0.2)
    rec = dict(
        grid_dim=np.int64(inp["grid_dim"]), vox=inp["vox"], voxels=voxels, children=children, features=features,
        centres=centres.numpy(), structure=structure.numpy(), embeddings=emb.detach().numpy(),
        rays_o=inp["rays_o"], rays_d=inp["rays_d"], rgb=inp["rgb"], depth_gt=inp["depth"],
        step_size=np.float32(inp["step"]), voxel_size=np.float32(0.2), truncation=np.float32(0.1),
        max_distance=np.float32(10.0), max_depth=np.float32(args.data_specs["max_depth"]),
        crit=np.array([args.criteria[k] for k in ("rgb_weight", "depth_weight", "fs_weight", "sdf_weight")],
                      np.float32),
        width=np.int64(inp["width"]), noise=noise,
        raw_idx=raw_idx, raw_t0=raw_t0, raw_t1=raw_t1, visits=np.int64(visits),
        hit_idx=inter["intersected_voxel_idx"].numpy(), hit_min=inter["min_depth"].numpy(),
        hit_max=inter["max_depth"].numpy(), hits=hits.numpy(),
        z_vals=out["z_vals"].detach().numpy(), sdf=out["sdf"].detach().numpy(),
        weights=out["weights"].detach().numpy(), color=out["color"].detach().numpy(),
        depth=out["depth"].detach().numpy(), ray_mask=out["ray_mask"].numpy(),
        loss=np.float32(loss.item()),
        loss_parts=np.array([parts[k] for k in ("color_loss", "depth_loss", "fs_loss", "sdf_loss")], np.float32),
        grad_embeddings=emb.grad.numpy(), grad_rays_o=ro.grad.numpy(), grad_rays_d=rd.grad.numpy(),
    )
    for k, v in dec.state_dict().items():
        rec["dec." + k] = v.numpy()
    for k, p in dec.named_parameters():
        rec["grad_dec." + k] = p.grad.numpy()
    return rec


def run_mesh_case(rh, nrgbd):
    """get_scores / eval_points (render_helpers.py:243-328) on the SURFACE
    voxels Mapping.extract_mesh selects (mapping.py:420-431), for the first
    40 of them (two of get_scores' 32-voxel chunks)."""
    inp = case_inputs("A_voxels_center")
    voxels, children, features = _octree(inp["vox"], inp["grid_dim"])
    torch.manual_seed(4321)
    emb = torch.randn(voxels.shape[0], 16) * 0.3
    dec = nrgbd.Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none", multires=0)
    vt, ft = torch.from_numpy(voxels), torch.from_numpy(features)
    keep = ~ft.eq(-1).any(-1)
    sv, sf = vt[keep][:40], ft[keep][:40]
    centres = (sv[:, :3] + sv[:, -1:] / 2) * 0.2
    states = {"voxel_vertex_idx": sf, "voxel_center_xyz": centres, "voxel_vertex_emb": emb}
    with torch.no_grad():
        scores = rh.get_scores(dec, states, 0.2, bits=8)
        g = torch.Generator().manual_seed(7)
        idx = torch.randint(0, sv.shape[0], (300,), generator=g)
        pts = centres[idx] + (torch.rand(300, 3, generator=g) - 0.5) * 0.2
        colours = rh.eval_points(dec, states, pts, idx, 0.2)
    rec = dict(voxels=sv.numpy(), features=sf.numpy(), centres=centres.numpy(), embeddings=emb.numpy(),
               voxel_size=np.float32(0.2), res=np.int64(8), scores=scores.numpy(), points=pts.numpy(),
               point_idx=idx.numpy().astype(np.int64), point_rgb=colours.numpy())
    for k, v in dec.state_dict().items():
        rec["dec." + k] = v.numpy()
    return rec


BA_CASES = {
    # the round-2 golden: room0, W = 128, Replica criteria, no point encoder
    "BA_room0": dict(scene="room0", width=128, crit="replica", max_depth=10.0, n_rays=160, resnet=False),
    # the call Mapping.do_mapping makes (mapping.py:195-213): points_encoder
    # (variations/resnet.py PointsResNet, replica.yaml:13-14 feature_n 16) and
    # its Adam (mapping.py:93) passed as resnet / resnet_optim
    "BA_room0_resnet": dict(scene="room0", width=128, crit="replica", max_depth=10.0, n_rays=160, resnet=True),
    # ScanNet settings (scannet.yaml: W = 256, rgb_weight 1, max_depth 5 = max_distance, mapping.py:61)
    "BA_scannet_w256": dict(scene="scannet0000", width=256, crit="scannet", max_depth=5.0, n_rays=128,
                            resnet=True),
}


def _stub_torchvision():
    """variations/resnet.py imports torchvision.models at module level (for
    its commented-out ResNet-18 variant); the PointsResNet it defines is
    plain Linear/ReLU.  torchvision is not installed here: an empty stub."""
    if "torchvision" not in sys.modules:
        tv = types.ModuleType("torchvision")
        tv.models = types.ModuleType("torchvision.models")
        sys.modules["torchvision"] = tv
        sys.modules["torchvision.models"] = tv.models


def run_ba_case(rh, nrgbd, crit_mod, noise_log, name="BA_room0"):
    """The reference bundle_adjust_frames (render_helpers.py:559-676): 3
    keyframes (stamps 0, 5, 9 — the first pose stays fixed, :594-596) of a
    synthetic scene at a reduced resolution, n_rays per frame, 3 iterations,
    Adam(embeddings) / Adam(decoder) lr 5e-3 and each keyframe's pose Adam lr
    1e-3 (frame.py:27); with `resnet` the reference's PointsResNet and its
    Adam are passed as Mapping.do_mapping passes them.  Stub keyframes carry
    the reference's own se3pose.OptimizablePose and replay recorded pixel
    samples; the sampler noise of every iteration is recorded."""
    import importlib
    spec = BA_CASES[name]
    se3 = importlib.import_module("se3pose")
    scene = getattr(syn, spec["scene"])()
    vox = syn.surface_voxels(scene, seed=0)
    voxels, children, features = _octree(vox, 256)
    n_nodes = voxels.shape[0]
    Ts = syn.camera_poses(scene, 3, seed=17)
    frames = [syn.SyntheticFrame(scene, T, scale=0.06, seed=100 + i, device="cpu") for i, T in enumerate(Ts)]
    n_rays, iters = spec["n_rays"], 3
    gen = torch.Generator().manual_seed(5)
    picks = [[torch.randperm(f.h * f.w, generator=gen)[:n_rays].sort().values for f in frames] for _ in range(iters)]

    class KF:
        def __init__(self, i, fr, T, stamp):
            self.stamp = stamp
            self.rays_d, self.rgb, self.depth = fr.rays_d, fr.rgb, fr.depth
            self.h, self.w = fr.h, fr.w
            self.pose = se3.OptimizablePose.from_matrix(torch.tensor(T, dtype=torch.float32))
            self.optim = torch.optim.Adam(self.pose.parameters(), lr=1e-3)
            self.i, self.calls = i, 0

        def get_pose(self):
            return self.pose.matrix()

        def sample_rays(self, n):
            idx = picks[self.calls][self.i]
            self.calls += 1
            m = torch.zeros(self.h * self.w, dtype=torch.bool)
            m[idx] = True
            self.sample_mask = m.view(self.h, self.w)

    kfs = [KF(i, fr, T, st) for i, (fr, T, st) in enumerate(zip(frames, Ts, (0, 5, 9)))]
    pose0 = np.stack([kf.pose.data.detach().numpy().copy() for kf in kfs])
    torch.manual_seed(77)
    emb0 = torch.randn(n_nodes, 16) * 0.3
    emb = emb0.clone().requires_grad_(True)
    dec = nrgbd.Decoder(depth=2, width=spec["width"], in_dim=16, skips=[], embedder="none", multires=0)
    dec0 = {k: v.detach().clone().numpy() for k, v in dec.state_dict().items()}
    resnet, resnet_optim, res0 = None, None, {}
    if spec["resnet"]:
        _stub_torchvision()
        resnet = importlib.import_module("variations.resnet").PointsResNet(16)  # replica.yaml:13-14
        resnet.train()  # mapping.py:183
        resnet_optim = torch.optim.Adam(resnet.parameters(), lr=5e-3)  # mapping.py:93
        res0 = {k: v.detach().clone().numpy() for k, v in resnet.state_dict().items()}
    vt = torch.from_numpy(voxels)
    centres = (vt[:, :3] + vt[:, -1:] / 2) * 0.2
    structure = torch.cat([torch.from_numpy(children), vt[:, -1:]], -1).int()
    map_states = {"voxel_vertex_idx": torch.from_numpy(features), "voxel_center_xyz": centres.float(),
                  "voxel_structure": structure, "voxel_vertex_emb": emb}
    criteria = O.REPLICA_CRITERIA if spec["crit"] == "replica" else O.SCANNET_CRITERIA
    args = types.SimpleNamespace(criteria={**criteria, "sdf_truncation": 0.1},
                                 data_specs={"max_depth": spec["max_depth"]})
    crit = crit_mod.Criterion(args)
    losses = []

    def loss_rec(outputs, obs, **kw):
        loss, parts = crit(outputs, obs, **kw)
        losses.append(float(loss))
        return loss, parts
    embed_optim = torch.optim.Adam([emb], lr=5e-3)
    model_optim = torch.optim.Adam(dec.parameters(), lr=5e-3)
    noise_log.clear()
    torch.manual_seed(31)
    # positional order of mapping.py:195-213 (max_distance = data_specs max_depth, mapping.py:61)
    rh.bundle_adjust_frames(kfs, map_states, dec, resnet, loss_rec, 0.2, 0.02, n_rays, iters, 0.1, 10,
                            spec["max_depth"], embed_optim=embed_optim, model_optim=model_optim,
                            resnet_optim=resnet_optim, update_pose=True)
    assert len(noise_log) == iters, len(noise_log)
    emb1 = emb.detach()
    changed = torch.nonzero((emb1 != emb0).any(-1)).squeeze(1)
    rec = dict(voxels=voxels, children=children, features=features, centres=centres.numpy(),
               structure=structure.numpy(), n_nodes=np.int64(n_nodes), emb_seed=np.int64(77), emb_std=np.float32(0.3),
               emb0_checksum=np.float64(emb0.double().sum()), pose0=pose0, stamps=np.array([0, 5, 9], np.int64),
               poses1=np.stack([kf.pose.data.detach().numpy() for kf in kfs]),
               step_size=np.float32(0.02), n_rays=np.int64(n_rays), iters=np.int64(iters),
               losses=np.array(losses, np.float32), emb_changed_rows=changed.numpy().astype(np.int64),
               emb1_changed=emb1[changed].numpy())
    if name != "BA_room0":  # the round-2 file keeps its keys
        rec.update(width=np.int64(spec["width"]), max_depth=np.float32(spec["max_depth"]),
                   crit=np.array([criteria[k] for k in ("rgb_weight", "depth_weight", "fs_weight", "sdf_weight")],
                                 np.float32))
    if resnet is not None:
        # the reference never runs the encoder on this path (render_helpers.py:481 commented out): its
        # parameters never get a gradient and Adam never steps them (no state is created)
        rec["resnet_optim_states"] = np.int64(len(resnet_optim.state))
        for k, v in res0.items():
            rec["res0." + k] = v
        rec["res_unchanged"] = np.bool_(all(torch.equal(v, torch.from_numpy(res0[k]))
                                            for k, v in resnet.state_dict().items()))
    for i, fr in enumerate(frames):
        rec[f"frame{i}.rays_d"] = fr.rays_d.numpy()
        rec[f"frame{i}.rgb"] = fr.rgb.numpy()
        rec[f"frame{i}.depth"] = fr.depth.numpy()
    for it in range(iters):
        rec[f"noise{it}"] = noise_log[it].numpy()
        for i in range(len(frames)):
            rec[f"pick{it}.{i}"] = picks[it][i].numpy()
    for k, v in dec0.items():
        rec["dec0." + k] = v
    for k, v in dec.state_dict().items():
        rec["dec1." + k] = v.numpy()
    return rec


def track_setup():
    """The T_track case's inputs (also rebuilt by the tests): room0, one frame
    at 0.1 of the Replica resolution, a start pose perturbed from the frame's
    pose, N_rays pixels per iteration replayed from seeded permutations."""
    scene = syn.room0()
    vox = syn.surface_voxels(scene, seed=0)
    T = syn.camera_poses(scene, 1, seed=23)[0]
    from scipy.spatial.transform import Rotation as Rr
    dT = np.eye(4)
    dT[:3, :3] = Rr.from_rotvec([0.012, -0.02, 0.016]).as_matrix()
    dT[:3, 3] = [0.03, -0.015, 0.025]
    return scene, vox, T, T @ dT


def run_track_case(rh, nrgbd, crit_mod, noise_log):
    """The reference track_frame (render_helpers.py:679-761) with
    depth_variance=True — the call Tracking.do_tracking makes
    (tracking.py:130-147): Criterion(weight_depth_loss=True), the depth
    variance median filter (criterion.py:45-50) — 3 iterations of pose-only
    Adam (lr 1e-3) from a perturbed pose.  Per iteration: the loss, the
    sampler noise, the replayed pixel picks and how many hit rays the median
    filter dropped; then the final pose and the last hit mask."""
    import importlib
    se3 = importlib.import_module("se3pose")
    scene, vox, T, T0 = track_setup()
    voxels, children, features = _octree(vox, 256)
    n_nodes = voxels.shape[0]
    fr = syn.SyntheticFrame(scene, T, scale=0.1, seed=41, device="cpu")
    n_rays, iters = 256, 3
    gen = torch.Generator().manual_seed(9)
    picks = [torch.randperm(fr.h * fr.w, generator=gen)[:n_rays].sort().values for _ in range(iters)]

    class Frame:
        def __init__(self):
            self.rays_d, self.rgb, self.depth = fr.rays_d, fr.rgb, fr.depth
            self.calls = 0

        def sample_rays(self, n):
            idx = picks[self.calls]
            self.calls += 1
            m = torch.zeros(fr.h * fr.w, dtype=torch.bool)
            m[idx] = True
            self.sample_mask = m.view(fr.h, fr.w)

    torch.manual_seed(55)
    emb = torch.randn(n_nodes, 16) * 0.3
    dec = nrgbd.Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none", multires=0)
    for p in dec.parameters():
        p.requires_grad_(False)
    vt = torch.from_numpy(voxels)
    centres = (vt[:, :3] + vt[:, -1:] / 2) * 0.2
    structure = torch.cat([torch.from_numpy(children), vt[:, -1:]], -1).int()
    map_states = {"voxel_vertex_idx": torch.from_numpy(features), "voxel_center_xyz": centres.float(),
                  "voxel_structure": structure, "voxel_vertex_emb": emb}
    args = types.SimpleNamespace(criteria={**O.REPLICA_CRITERIA, "sdf_truncation": 0.1},
                                 data_specs={"max_depth": 10.0})
    crit = crit_mod.Criterion(args)
    losses, dropped = [], []

    def loss_rec(outputs, obs, **kw):
        loss, parts = crit(outputs, obs, **kw)
        losses.append(float(loss))
        with torch.no_grad():  # the hit rays criterion.py:45-50 drops from the depth loss
            gd = obs[1][outputs["ray_mask"]]
            valid = (gd > 0.01) & (gd < 10.0)
            dl = (gd - outputs["depth"]).abs()
            var = torch.sum(outputs["weights"] * ((outputs["depth"].unsqueeze(-1) - outputs["z_vals"]) ** 2), -1)
            tmp = dl / torch.sqrt(var + 1e-10)
            dropped.append(int((valid & ~(tmp < 10 * tmp.median())).sum()))
        return loss, parts
    pose0 = se3.OptimizablePose.from_matrix(torch.tensor(T0, dtype=torch.float32))
    p0 = pose0.data.detach().numpy().copy()
    noise_log.clear()
    torch.manual_seed(61)
    pose1, _, hit = rh.track_frame(pose0, Frame(), map_states, dec, None, loss_rec, 0.2, N_rays=n_rays,
                                   step_size=0.02, num_iterations=iters, truncation=0.1, learning_rate=1e-3,
                                   max_voxel_hit=10, max_distance=10, depth_variance=True)
    assert len(noise_log) == iters, len(noise_log)
    rec = dict(voxels=voxels, children=children, features=features, centres=centres.numpy(),
               structure=structure.numpy(), embeddings=emb.numpy(), rays_d=fr.rays_d.numpy(), rgb=fr.rgb.numpy(),
               depth=fr.depth.numpy(), pose0=p0, pose1=pose1.data.detach().numpy(), hit_mask=hit.numpy(),
               losses=np.array(losses, np.float32), depth_filter_dropped=np.array(dropped, np.int64),
               step_size=np.float32(0.02), voxel_size=np.float32(0.2), truncation=np.float32(0.1),
               max_distance=np.float32(10.0), max_depth=np.float32(10.0), lr=np.float32(1e-3),
               n_rays=np.int64(n_rays), iters=np.int64(iters),
               crit=np.array([O.REPLICA_CRITERIA[k] for k in ("rgb_weight", "depth_weight", "fs_weight",
                                                              "sdf_weight")], np.float32))
    for it in range(iters):
        rec[f"noise{it}"] = noise_log[it].numpy()
        rec[f"pick{it}"] = picks[it].numpy()
    for k, v in dec.state_dict().items():
        rec["dec." + k] = v.numpy()
    return rec


def main(only=()):
    """only: case names to (re)generate (default: all)."""
    want = (lambda n: not only or n in only)
    noise_log = []
    _install_stubs(noise_log)
    rh, nrgbd, crit_mod = _reference_modules()
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)  # render_rays np.savetxt()s every call (render_helpers.py:403-404)
        try:
            for name in CASES:
                if not want(name):
                    continue
                rec = run_case(name, rh, nrgbd, crit_mod, noise_log)
                path = os.path.join(OUT_DIR, f"{name}.npz")
                np.savez_compressed(path, **rec)
                print(f"{name}: nodes={rec['voxels'].shape[0]} rays={rec['rays_o'].shape[1]} "
                      f"R_hit={int(rec['hits'].sum())} P={rec['hit_idx'].shape[-1]} S={rec['z_vals'].shape[-1]} "
                      f"loss={float(rec['loss']):.6f} -> {os.path.relpath(path, REPO)} "
                      f"({os.path.getsize(path) // 1024} KiB)")
            for name in BA_CASES:
                if not want(name):
                    continue
                rec = run_ba_case(rh, nrgbd, crit_mod, noise_log, name)
                path = os.path.join(OUT_DIR, f"{name}.npz")
                np.savez_compressed(path, **rec)
                print(f"{name}: nodes={int(rec['n_nodes'])} losses={rec['losses'].tolist()} "
                      f"-> {os.path.relpath(path, REPO)} ({os.path.getsize(path) // 1024} KiB)")
            if want("T_track"):
                rec = run_track_case(rh, nrgbd, crit_mod, noise_log)
                path = os.path.join(OUT_DIR, "T_track.npz")
                np.savez_compressed(path, **rec)
                print(f"T_track: losses={rec['losses'].tolist()} dropped={rec['depth_filter_dropped'].tolist()} "
                      f"hits={int(rec['hit_mask'].sum())} -> {os.path.relpath(path, REPO)} "
                      f"({os.path.getsize(path) // 1024} KiB)")
            if not want("M_mesh_A"):
                return
            rec = run_mesh_case(rh, nrgbd)
            path = os.path.join(OUT_DIR, "M_mesh_A.npz")
            np.savez_compressed(path, **rec)
            print(f"M_mesh_A: voxels={rec['voxels'].shape[0]} scores={tuple(rec['scores'].shape)} "
                  f"-> {os.path.relpath(path, REPO)} ({os.path.getsize(path) // 1024} KiB)")
        finally:
            os.chdir(cwd)


if __name__ == "__main__":
    main(tuple(sys.argv[1:]))
