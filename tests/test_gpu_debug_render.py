"""Tracking's debug render (tracking.py:162-215 render_debug_images; VERDICT
r1 weak #9): one render_rays call over a whole 200 x 160 frame (render_res
of configs/{replica,scannet,arkit}, 32,000 rays, chunk_size=5000,
return_raw=True, no autograd), then fill_in into depth / colour images —
against the oracle on the same rays and sampler noise.  chunk_size is the
reference's decoder batching (render_helpers.py:413-470); the fused decoder
needs none, and the result does not depend on it."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_debug_render_full_frame_matches_oracle():
    from psvo import synthetic as syn
    from psvo.decoder import Decoder
    from psvo.octree import Octree, map_states
    from psvo.render_helpers import fill_in, render_rays
    scene = syn.room0()
    tree = Octree()
    tree.init(scene.grid_dim, 16, scene.voxel_size, 8)
    tree.insert(syn.surface_voxels(scene, seed=0))
    emb = torch.randn(max(20000, tree.count_nodes()), 16, generator=torch.Generator().manual_seed(2)) * 0.1
    ms = map_states(tree, emb.to(DEV), scene.voxel_size, device=DEV)
    ms_cpu = {k: v.cpu() for k, v in ms.items()}
    # frame.get_rays(w, h) (frame.py:43-58) at render_res [200, 160]: intrinsics scaled to the grid
    w, h = 200, 160
    K = scene.intrinsics
    fx, fy = K["fx"] * w / K["W"], K["fy"] * h / K["H"]
    cx, cy = (K["cx"] + 0.5) * w / K["W"] - 0.5, (K["cy"] + 0.5) * h / K["H"] - 0.5
    iy, ix = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    d_cam = np.stack([(ix - cx) / fx, (iy - cy) / fy, np.ones_like(ix, dtype=np.float64)], -1).astype(np.float32)
    T = syn.camera_poses(scene, 1, seed=9)[0]
    R = torch.from_numpy(np.asarray(T[:3, :3], np.float32))
    rays_d = (torch.from_numpy(d_cam) @ R.transpose(-1, -2)).reshape(1, -1, 3).contiguous()
    rays_o = torch.from_numpy(np.asarray(T[:3, 3], np.float32)).reshape(1, 1, 3).expand_as(rays_d).contiguous()
    params = O.decoder_params_init(128, seed=3)
    step = 0.01
    o = O.render_rays(rays_o, rays_d, ms_cpu, params, step, scene.voxel_size, 0.1, 10.0, deterministic=False,
                      generator=torch.Generator().manual_seed(4), sum_order="sequential")
    dec = Decoder(depth=2, width=128, in_dim=16, skips=[], embedder="none").to(DEV)
    dec.load_state_dict(params)
    outs = []
    with torch.no_grad():
        for chunk in (5000, 20000):
            outs.append(render_rays(rays_o.to(DEV), rays_d.to(DEV), ms, dec, None, step, scene.voxel_size, 0.1, 10,
                                    10.0, chunk_size=chunk, return_raw=True, noise=o["noise"]))
    a, b = outs
    for k in ("ray_mask", "z_vals", "depth", "color", "raw"):
        assert torch.equal(a[k], b[k]), k  # chunk_size changes nothing
    out = a
    mask = out["ray_mask"].view(-1).cpu()
    assert torch.equal(mask, o["ray_mask"].view(-1))
    assert int(mask.sum()) > 20000  # most of the frame sees the room
    assert torch.equal(out["z_vals"].cpu(), o["z_vals"])
    torch.testing.assert_close(out["depth"].cpu(), o["depth"], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(out["color"].cpu(), o["color"], rtol=1e-4, atol=1e-5)
    # the images render_debug_images logs
    rdepth = fill_in((h, w, 1), out["ray_mask"].view(h, w), out["depth"], 0)
    rcolor = fill_in((h, w, 3), out["ray_mask"].view(h, w), out["color"], 0)
    odepth = fill_in((h, w, 1), o["ray_mask"].view(h, w), o["depth"], 0)
    ocolor = fill_in((h, w, 3), o["ray_mask"].view(h, w), o["color"], 0)
    torch.testing.assert_close(rdepth.cpu(), odepth, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rcolor.cpu(), ocolor, rtol=1e-4, atol=1e-5)
    assert out["raw"] is not None and out["raw"].shape[0] == int(mask.sum())
