"""Pre-Adam gradient parity of the HEADLINE path at full size (VERDICT r3
item 1): psvo_map_step_frames — the call bundle_adjust_frames makes each
iteration, whose width-128 backward is the fused k_mlp_bwd3<true> (δ chain +
weight gradients + the interpolation backward: embedding scatter and dL/dx)
and whose width-256 backward is k_dec256_bwd / _dw + k_interp_bwd — stopped
before Adam (PSVO_STEP_NO_ADAM) and compared with the oracle
(oracle.render_and_backward: the reference's render_rays + Criterion +
loss.backward(), render_helpers.py:559-676 / :104-156, criterion.py:17-116)
on the same rays and sampler noise, at every BASELINE config:

  * the loss: rtol 1e-4;
  * grad_flat's embedding and decoder slices: ≤ 2e-3·max|ref| per tensor
    (float-atomic scatter / GEMM summation order) — the same bar as the
    autograd path's test_render_loss_grads_full_size;
  * per-ray d rays_o / d rays_d (psvo_engine_grad_rays, the sums the pose
    gradient is formed from): ≤ 2e-3·max on every hit ray except rays
    holding an fp32 near-tie — a ReLU pre-activation or the ray's sdf within
    1e-5 of zero in the fp64 oracle (oracle.decoder_margins), where any fp32
    order can land on either side (tests/test_gpu_fullsize_parity.py, part
    3) — which stay ≤ 2e-2·max, and at most 1 % of the rays are such;
  * the per-keyframe pose gradient (pose_grad [F, 8]): the exact (fp64)
    chain rays = (t, dirs·R(w)ᵀ) applied to the engine's own per-ray
    gradients to 1e-3·max (the f32 k_pose_grad_frames reduction), and against
    the same chain applied to the fp32 oracle's per-ray gradients to
    2e-3·max.

The rays are formed on the device from keyframe poses and camera-frame
directions (psvo_pose_rays_frames, as the engine forms them); the oracle is
fed exactly those rays."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

import test_gpu_fullsize_parity as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _keyframes(w, c):
    """Pose parameters [F, 6] of the workload's cameras and the camera-frame
    directions of its rays (world directions rotated back by each pose)."""
    from psvo.pose import OptimizablePose
    n = c["rays"]
    poses, dirs = [], []
    rd = w.rays_d[0].double()
    for f, T in enumerate(w.poses):
        p = OptimizablePose.from_matrix(np.asarray(T)).data.detach().double()
        R = O.se3_rotation(p)
        poses.append(p.float())
        dirs.append((rd[f * n:(f + 1) * n] @ R).float())
    return torch.stack(poses).contiguous(), torch.cat(dirs).contiguous()


def _pose_grad_from_rays(poses, dirs, g_o, g_d, n):
    """d loss / d pose [F, 6] through rays_o = t, rays_d = dirs·R(w)ᵀ (se3pose.py,
    oracle.se3_rotation), in fp64, from per-ray gradients."""
    out = []
    for f in range(poses.shape[0]):
        p = poses[f].double().clone().requires_grad_(True)
        R = O.se3_rotation(p)
        d = dirs[f * n:(f + 1) * n].double()
        ro = p[:3].expand(n, 3)
        rd = d @ R.transpose(0, 1)
        (ro * g_o[f * n:(f + 1) * n]).sum().add((rd * g_d[f * n:(f + 1) * n]).sum()).backward()
        out.append(p.grad.detach())
    return torch.stack(out)


@pytest.mark.parametrize("name", list(F.CONFIGS))
def test_engine_step_frames_grads_full_size(name):
    from psvo import _lib as L
    from psvo.decoder import Decoder
    from psvo.engine import MappingEngine
    c, w, ms, ms_cpu = F._setup(name)
    vs = w.scene.voxel_size
    n = c["rays"]
    n_f = c["frames"]
    R = n * n_f
    crit_w = O.SCANNET_CRITERIA if c["scene"] == "scannet0000" else O.REPLICA_CRITERIA
    params = O.decoder_params_init(c["width"], seed=4)
    poses, dirs = _keyframes(w, c)
    poses_d, dirs_d = poses.to(DEV), dirs.to(DEV)
    ro = torch.empty(R, 3, device=DEV)
    rd = torch.empty(R, 3, device=DEV)
    L.call("psvo_pose_rays_frames", L.stream_of(ro.device), R, n, poses_d, dirs_d, ro, rd)
    ro_c, rd_c = ro.cpu()[None], rd.cpu()[None]
    # sampler noise in the layout this batch's sampler reads ([200, K', max ⌈Σ/step⌉ + P])
    o_out, o_hits = O.ray_intersect_vox(ro_c, rd_c, ms_cpu["voxel_center_xyz"], ms_cpu["voxel_structure"], vs, 10.0)
    hit = o_hits.view(-1)
    inter = {k: v[0][hit] for k, v in o_out.items()}
    dists = (inter["max_depth"] - inter["min_depth"]).masked_fill(inter["intersected_voxel_idx"].eq(-1), 0)
    P = dists.shape[-1]
    max_steps = int(torch.ceil(O.sequential_row_sums(dists) / np.float32(c["step"])).max()) + P
    kp = (int(hit.sum()) + 199) // 200
    noise = torch.rand((200, kp, max_steps), generator=torch.Generator().manual_seed(17)).clamp(0.001, 0.999)
    rgb, depth = w.rgb.reshape(1, -1, 3), w.depth.reshape(1, -1)
    orc = {}
    for dt in (torch.float32, torch.float64):
        cap = {}
        res, loss_o, _, grads = O.render_and_backward(ro_c, rd_c, rgb, depth, ms_cpu, params, c["step"], vs, 0.1, 10.0,
                                                      crit_w, noise=noise, sum_order="sequential",
                                                      max_depth=c["max_depth"], dtype=dt, capture=cap)
        orc[dt] = (res, loss_o, grads, cap["feats"].detach())
    o_res, o_loss, o_grads, _ = orc[torch.float32]
    x_res64, _, _, x64 = orc[torch.float64]

    # ---- the engine: one psvo_map_step_frames, stopped before Adam
    dec = Decoder(depth=2, width=c["width"], in_dim=16, skips=[], embedder="none").to(DEV)
    dec.load_state_dict(params)
    emb = ms["voxel_vertex_emb"].clone()
    eng = MappingEngine(dict(ms, voxel_vertex_emb=emb), dec, vs, c["step"], truncation=0.1, max_distance=10.0,
                        criteria=crit_w, max_depth=c["max_depth"])
    pose_grad = torch.zeros(n_f, 8, device=DEV)
    pm = torch.zeros(n_f, 6, device=DEV)
    pv = torch.zeros(n_f, 6, device=DEV)
    loss = eng.step_frames(dirs_d, n, poses_d.clone(), pm, pv, [0] + [1] * (n_f - 1), 1e-3, rgb.to(DEV),
                           depth.to(DEV), seed=0, noise=noise, apply_adam=False, pose_grad=pose_grad)
    g_o = torch.empty(R, 3, device=DEV)
    g_d = torch.empty(R, 3, device=DEV)
    L.call("psvo_engine_grad_rays", eng.handle, L.stream_of(g_o.device), R, g_o, g_d)
    torch.cuda.synchronize()
    stats = eng.last_stats
    assert stats[1] == int(hit.sum()) and stats[0] == P
    assert stats[4] == int(o_res["samples"]["sampled_point_voxel_idx"].ne(-1).sum())  # M
    assert abs(float(loss) - float(o_loss)) <= 1e-4 * abs(float(o_loss)), (float(loss), float(o_loss))

    # grad_flat = [embeddings | W1, b1, ..., W5, b5] (fused_params order), pre-Adam
    names = {id(p): k for k, p in dec.named_parameters()}
    flat = eng.grad_flat.cpu()
    n_emb = emb.shape[0]
    pairs = [("embeddings", flat[:n_emb * 16].view(n_emb, 16), o_grads["embeddings"])]
    off = n_emb * 16
    for p in dec.fused_params():
        pairs.append((names[id(p)], flat[off:off + p.numel()].view(p.shape), o_grads[names[id(p)]]))
        off += p.numel()
    assert off == flat.numel()
    for k, a, b in pairs:
        scale = float(b.abs().max()) + 1e-12
        err = float((a - b).abs().max())
        assert err <= 2e-3 * scale, (k, err, scale)

    # per-ray d rays_o / d rays_d of the hit rays against the fp32 oracle
    got_o, got_d = g_o.cpu()[hit].double(), g_d.cpu()[hit].double()
    ref_o, ref_d = o_grads["rays_o"][0][hit].double(), o_grads["rays_d"][0][hit].double()
    offsets = torch.cat([torch.zeros(1, dtype=torch.long),
                         x_res64["samples"]["sampled_point_voxel_idx"].ne(-1).sum(-1).cumsum(0)])
    bad = torch.zeros(got_o.shape[0], dtype=torch.bool)
    for got, ref in ((got_o, ref_o), (got_d, ref_d)):
        scale = float(ref.abs().max())
        per_ray = (got - ref).abs().amax(-1)
        assert float(per_ray.max()) <= 2e-2 * scale, float(per_ray.max() / scale)
        bad |= per_ray > 2e-3 * scale
    for r in torch.nonzero(bad).squeeze(1).tolist():  # each must hold an fp32 near-tie (fp64 margins)
        relu_m, sdf_m = O.decoder_margins(params, x64[int(offsets[r]):int(offsets[r + 1])])
        assert bool((relu_m < 1e-5).any() or (sdf_m < 1e-5).any()), ("ray off the oracle with no near-tie", r)
    assert int(bad.sum()) <= max(4, 1e-2 * bad.shape[0]), int(bad.sum())

    # per-keyframe pose gradient
    pg = pose_grad.cpu()[:, :6].double()
    mine = _pose_grad_from_rays(poses, dirs, torch.where(hit[:, None], g_o.cpu().double(), 0.0),
                                torch.where(hit[:, None], g_d.cpu().double(), 0.0), n)
    assert float((pg - mine).abs().max()) <= 1e-3 * float(mine.abs().max()), (pg, mine)
    full_o = torch.zeros(R, 3, dtype=torch.float64)
    full_d = torch.zeros(R, 3, dtype=torch.float64)
    full_o[hit], full_d[hit] = ref_o, ref_d
    theirs = _pose_grad_from_rays(poses, dirs, full_o, full_d, n)
    assert float((pg - theirs).abs().max()) <= 2e-3 * float(theirs.abs().max()), (pg, theirs)
    eng.close()
