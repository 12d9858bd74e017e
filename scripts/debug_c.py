"""Diagnostic: config C full-size render + loss + backward, fused W=256
decoder vs the torch fp32 decoder, both against the oracle (per-ray rays_o /
rays_d gradients and the decoder input gradient)."""
import os
import sys
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "proud-slam_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_gpu_fullsize_parity as T  # noqa: E402
from oracle import oracle as O  # noqa: E402
from psvo.criterion import Criterion  # noqa: E402
from psvo.decoder import Decoder  # noqa: E402
from psvo.render_helpers import render_rays  # noqa: E402

DEV = "cuda"
name = sys.argv[1] if len(sys.argv) > 1 else "C"
c, w, ms, ms_cpu = T._setup(name)
vs = w.scene.voxel_size
crit_w = O.SCANNET_CRITERIA if c["scene"] == "scannet0000" else O.REPLICA_CRITERIA
params = O.decoder_params_init(c["width"], seed=4)
o_out, o_hits = T._oracle_intersection(w, ms_cpu, vs)
hit = o_hits.view(-1)
inter = {k: v[0][hit] for k, v in o_out.items()}
dists = (inter["max_depth"] - inter["min_depth"]).masked_fill(inter["intersected_voxel_idx"].eq(-1), 0)
P = dists.shape[-1]
max_steps = int(torch.ceil(O.sequential_row_sums(dists) / np.float32(c["step"])).max()) + P
kp = (int(hit.sum()) + 199) // 200
noise = torch.rand((200, kp, max_steps), generator=torch.Generator().manual_seed(13)).clamp(0.001, 0.999)
rgb, depth = w.rgb.reshape(1, -1, 3), w.depth.reshape(1, -1)
o_res, o_loss, _, o_grads = O.render_and_backward(w.rays_o, w.rays_d, rgb, depth, ms_cpu, params, c["step"], vs, 0.1,
                                                  10.0, crit_w, noise=noise, sum_order="sequential",
                                                  max_depth=c["max_depth"])
res = {}
for mode in ("fused", "torch"):
    dec = Decoder(depth=2, width=c["width"], in_dim=16, skips=[], embedder="none").to(DEV)
    dec.load_state_dict(params)
    if mode == "torch":
        dec.can_fuse = lambda x: False
    emb = ms["voxel_vertex_emb"].clone().requires_grad_(True)
    ms2 = dict(ms, voxel_vertex_emb=emb)
    ro = w.rays_o.to(DEV).requires_grad_(True)
    rd = w.rays_d.to(DEV).requires_grad_(True)
    out = render_rays(ro, rd, ms2, dec, None, c["step"], vs, 0.1, 10, 10.0, noise=noise)
    crit = Criterion(types.SimpleNamespace(criteria={**crit_w, "sdf_truncation": 0.1},
                                           data_specs={"max_depth": c["max_depth"]}))
    loss, _ = crit(out, (rgb.to(DEV), depth.to(DEV)))
    loss.backward()
    gro, grd = ro.grad.cpu()[0], rd.grad.cpu()[0]
    for k, a, b in (("rays_o", gro, o_grads["rays_o"][0]), ("rays_d", grd, o_grads["rays_d"][0]),
                    ("emb", emb.grad.cpu(), o_grads["embeddings"])):
        err = (a - b).abs()
        per = err.reshape(err.shape[0], -1).amax(-1)
        top = torch.topk(per, 5)
        print(mode, k, "max err", float(err.max()), "scale", float(b.abs().max()), "worst rows", top.indices.tolist(),
              [f"{v:.3g}" for v in top.values.tolist()])
    res[mode] = gro
    print(mode, "loss", float(loss), float(o_loss))
print("fused vs torch rays_o max", float((res["fused"] - res["torch"]).abs().max()))
