"""Diagnostic: per-ray d loss / d rays_o, rays_d of the tracking parity case
(tests/test_gpu_tracking.py::test_pose_gradient_matches_oracle) from the HIP
path, saved for comparison with the oracle on the CPU."""
import os
import sys
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "proud-slam_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_gpu_tracking as TT  # noqa: E402
from oracle import oracle as O  # noqa: E402
from psvo.criterion import Criterion  # noqa: E402
from psvo.decoder import Decoder  # noqa: E402
from psvo.render_helpers import render_rays  # noqa: E402

DEV = "cuda"
scene, ms_cpu, emb, T, frame = TT._setup()
frame.sample_rays(1024)
mask = frame.sample_mask
rgb, depth = frame.rgb[mask], frame.depth[mask]
params = O.decoder_params_init(128, seed=2)
pose_o = TT._perturbed(T)
ro_o, rd_o = TT._rays(pose_o, frame, mask.cpu())
ro_o = ro_o.detach().requires_grad_(True)
rd_o = rd_o.detach().requires_grad_(True)
out_o = O.render_rays(ro_o, rd_o, ms_cpu, params, 0.01, scene.voxel_size, 0.1, 10.0, deterministic=True)
loss_o, _ = O.criterion(out_o, rgb.cpu().view(1, -1, 3), depth.cpu().view(1, -1), O.REPLICA_CRITERIA, 0.1, 10.0)
loss_o.backward()
dec = Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none").to(DEV)
dec.load_state_dict(params)
ms = {"voxel_center_xyz": ms_cpu["voxel_center_xyz"].to(DEV), "voxel_structure": ms_cpu["voxel_structure"].to(DEV),
      "voxel_vertex_idx": ms_cpu["voxel_vertex_idx"].to(DEV), "voxel_vertex_emb": emb.to(DEV)}
ro = ro_o.detach().to(DEV).requires_grad_(True)
rd = rd_o.detach().to(DEV).requires_grad_(True)
out = render_rays(ro, rd, ms, dec, None, 0.01, scene.voxel_size, 0.1, 10, 10.0, noise=out_o["noise"])
crit = Criterion(types.SimpleNamespace(criteria=dict(TT.CRIT, sdf_truncation=0.1), data_specs={"max_depth": 10.0}))
out["ray_mask"] = out["ray_mask"].view(-1)
loss, _ = crit(out, (rgb, depth))
loss.backward()
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(REPO, "gpurun_out", "debug_track.npz"), g_ro=ro.grad.cpu().numpy(), g_rd=rd.grad.cpu().numpy(),
         g_ro_o=ro_o.grad.numpy(), g_rd_o=rd_o.grad.numpy(), z=out["z_vals"].detach().cpu().numpy(),
         z_o=out_o["z_vals"].detach().numpy(), mask=out["ray_mask"].cpu().numpy(), mask_o=out_o["ray_mask"].numpy(),
         loss=float(loss), loss_o=float(loss_o), depth=out["depth"].detach().cpu().numpy(),
         depth_o=out_o["depth"].detach().numpy())
print("loss", float(loss), float(loss_o))
