"""Diagnostic: where do config C's (W = 256) per-ray
rays_o / rays_d gradient outliers come from?

Runs config C's full-size render + Criterion + backward four ways on the same
rays, noise and parameters:
  o32  the oracle (torch-CPU fp32, the reference's arithmetic),
  o64  the oracle's same function in fp64 after the fp32 sampler
       (oracle.render_rays dtype=float64; fp32's discrete decisions kept),
  fused  the HIP path with the fused W = 256 decoder,
  torch  the HIP path with the decoder's torch fp32 layers,
and compares each fp32 run's per-ray gradients with o64 (the exact value of
the same function).  For the worst rays it then walks the chain sample by
sample — decoder input features, the decoder's upstream gradients (d sdf,
d rgb), its output gradient dfeat — against o64's intermediates, and reports
the smallest |pre-activation| of each ReLU layer on those samples (a mask
that fp32 rounding can flip).  Writes gpurun_out/debug_c256.json."""
import json
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

# ---- oracle runs, capturing the decoder's input / outputs and their gradients
cap = {}
_orig_dec = O.decoder_forward


def _dec_cap(p, x):
    x.retain_grad()
    r, s = _orig_dec(p, x)
    r.retain_grad()
    s.retain_grad()
    cap.update(x=x, rgb=r, sdf=s)
    return r, s


O.decoder_forward = _dec_cap
orc = {}
for dt in (torch.float32, torch.float64):
    cap.clear()
    res, loss, _, grads = O.render_and_backward(w.rays_o, w.rays_d, rgb, depth, ms_cpu, params, c["step"], vs, 0.1,
                                                10.0, crit_w, noise=noise, sum_order="sequential",
                                                max_depth=c["max_depth"], dtype=dt)
    orc[dt] = dict(loss=float(loss), grads=grads, x=cap["x"].detach(), dfeat=cap["x"].grad.detach(),
                   g_sdf=cap["sdf"].grad.detach(), g_rgb=cap["rgb"].grad.detach(),
                   mask=res["samples"]["sampled_point_voxel_idx"].ne(-1))
O.decoder_forward = _orig_dec
o64, o32 = orc[torch.float64], orc[torch.float32]
counts = o64["mask"].sum(-1)
offs = torch.cat([torch.zeros(1, dtype=torch.long), counts.cumsum(0)])
hit_rows = torch.nonzero(hit).squeeze(1)  # hit-ray i -> ray id

# ---- GPU runs
gpu = {}
for mode in ("fused", "torch"):
    dec = Decoder(depth=2, width=c["width"], in_dim=16, skips=[], embedder="none").to(DEV)
    dec.load_state_dict(params)
    if mode == "torch":
        dec.can_fuse = lambda x: False
    g = {}
    fwd = dec.forward

    def hooked(inputs, fwd=fwd, g=g):
        x = inputs["emb"]
        x.register_hook(lambda t: g.__setitem__("dfeat", t.detach().cpu()))
        out = fwd(inputs)
        out["sdf"].register_hook(lambda t: g.__setitem__("g_sdf", t.detach().cpu()))
        out["color"].register_hook(lambda t: g.__setitem__("g_rgb", t.detach().cpu()))
        g["x"] = x.detach().cpu()
        return out

    dec.forward = hooked
    emb = ms["voxel_vertex_emb"].clone().requires_grad_(True)
    ro = w.rays_o.to(DEV).requires_grad_(True)
    rd = w.rays_d.to(DEV).requires_grad_(True)
    out = render_rays(ro, rd, dict(ms, voxel_vertex_emb=emb), dec, None, c["step"], vs, 0.1, 10, 10.0, noise=noise)
    crit = Criterion(types.SimpleNamespace(criteria={**crit_w, "sdf_truncation": 0.1},
                                           data_specs={"max_depth": c["max_depth"]}))
    loss, _ = crit(out, (rgb.to(DEV), depth.to(DEV)))
    loss.backward()
    g.update(loss=float(loss), rays_o=ro.grad.cpu()[0], rays_d=rd.grad.cpu()[0], emb=emb.grad.cpu())
    gpu[mode] = g

report = {"config": name, "width": c["width"], "rays": int(w.rays_o.shape[1]), "r_hit": int(hit.sum()),
          "samples": int(offs[-1]), "loss": {"o64": o64["loss"], "o32": o32["loss"],
                                             "fused": gpu["fused"]["loss"], "torch": gpu["torch"]["loss"]}}


def per_ray(k, got):
    ref = o64["grads"][k][0].double()
    scale = float(ref.abs().max())
    err = (got.double() - ref).abs().reshape(ref.shape[0], -1).amax(-1) / scale
    return err


runs = {"o32": {"rays_o": o32["grads"]["rays_o"][0], "rays_d": o32["grads"]["rays_d"][0]},
        "fused": gpu["fused"], "torch": gpu["torch"]}
worst = {}
for k in ("rays_o", "rays_d"):
    report[k] = {}
    for r, v in runs.items():
        e = per_ray(k, v[k])
        top = torch.topk(e, 5)
        report[k][r] = {"max_rel": float(e.max()), "n_over_2e-3": int((e > 2e-3).sum()),
                        "n_over_1e-3": int((e > 1e-3).sum()), "p99.9": float(torch.quantile(e.float(), 0.999)),
                        "worst_rays": top.indices.tolist(), "worst_vals": [float(x) for x in top.values]}
        if r == "fused":
            worst[k] = top.indices.tolist()[:3]


def dec_preacts(x):
    """fp64 pre-activations of the three ReLU layers for features x [n,16]."""
    p = {k: v.double() for k, v in params.items()}
    F = torch.nn.functional
    a1 = F.linear(x, p["pts_linears.0.weight"], p["pts_linears.0.bias"])
    a2 = F.linear(a1.relu(), p["pts_linears.1.weight"], p["pts_linears.1.bias"])
    o = F.linear(a2.relu(), p["sdf_out.weight"], p["sdf_out.bias"])
    a4 = F.linear(torch.cat([o[:, 1:], x], -1), p["color_out.0.weight"], p["color_out.0.bias"])
    return a1, a2, a4


samples = []
for k, rays in worst.items():
    for ray in rays:
        i = int(torch.nonzero(hit_rows == ray).squeeze())
        a, b = int(offs[i]), int(offs[i + 1])
        rec = {"grad": k, "ray": ray, "hit_row": i, "n_samples": b - a}
        for q in ("x", "g_sdf", "g_rgb", "dfeat"):
            ref = o64[q][a:b].double()
            sc = float(ref.abs().max()) + 1e-300
            for r, src in (("o32", o32), ("fused", gpu["fused"]), ("torch", gpu["torch"])):
                got = src[q][a:b].double()
                d = (got - ref).abs().reshape(b - a, -1).amax(-1) / sc
                rec[f"{q}.{r}.max_rel"] = float(d.max())
                rec[f"{q}.{r}.argmax"] = int(d.argmax())
        # per-sample dfeat error of each run pushed through the exact (fp64) rest of the chain is what
        # the ray's d_o / d_d error would be if everything else were exact
        a1, a2, a4 = dec_preacts(o64["x"][a:b].double())
        for nm, t in (("h1", a1), ("h2", a2), ("c1", a4)):
            rec[f"min_abs_preact.{nm}"] = float(t.abs().min())
            # pre-activation flips between the fused run's features and the oracle's (fp64 layers on both)
            a1f, a2f, a4f = dec_preacts(gpu["fused"]["x"][a:b].double())
            tf = {"h1": a1f, "h2": a2f, "c1": a4f}[nm]
            rec[f"mask_flips_from_features.{nm}"] = int(((tf > 0) != (t > 0)).sum())
        samples.append(rec)
report["worst_ray_walk"] = samples

# decoder in isolation on ALL samples: each fp32 decoder's dfeat given o64's own inputs (x, g) vs fp64
x64, gs64, gr64 = o64["x"].double(), o64["g_sdf"].double(), o64["g_rgb"].double()


def dec_bwd(x, gs, gr, mode):
    if mode == "fp64":
        p = {k: v.double() for k, v in params.items()}
        xx = x.clone().requires_grad_(True)
        r, s = O.decoder_forward(p, xx)
        ((s * gs).sum() + (r * gr).sum()).backward()
        return xx.grad
    dec = Decoder(depth=2, width=c["width"], in_dim=16, skips=[], embedder="none").to(DEV)
    dec.load_state_dict(params)
    if mode == "torch":
        dec.can_fuse = lambda x: False
    xx = x.float().to(DEV).requires_grad_(True)
    out = dec({"emb": xx})
    ((out["sdf"] * gs.float().to(DEV)).sum() + (out["color"] * gr.float().to(DEV)).sum()).backward()
    return xx.grad.cpu().double()


ref = dec_bwd(x64, gs64, gr64, "fp64")
iso = {}
for mode in ("fused", "torch"):
    d = (dec_bwd(x64, gs64, gr64, mode) - ref).abs().amax(-1)
    mag = ref.abs().amax(-1) + 1e-30
    rel = d / mag
    iso[mode] = {"max_abs_over_global_max": float(d.max() / ref.abs().max()),
                 "per_sample_rel_p50": float(torch.quantile(rel.float()[:1_000_000], 0.5)),
                 "per_sample_rel_p99": float(torch.quantile(rel.float()[:1_000_000], 0.99)),
                 "per_sample_rel_max": float(rel.max())}
report["decoder_isolated_dfeat_vs_fp64"] = iso
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
with open(os.path.join(REPO, "gpurun_out", f"debug_{name}256.json"), "w") as f:
    json.dump(report, f, indent=1)
print(json.dumps(report, indent=1))
