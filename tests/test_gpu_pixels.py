"""Keyframe pixel sampling on the device (csrc/pixels.hip, psvo.sample_util)
against the reference's sample_util.sample_rays (sample_util.py:4-20).

- golden: the reference's own picks (tests/golden/P_pixels.npz) from the
  uniforms its torch.rand_like drew, injected here;
- full Replica frames (680 x 1200, 4 keyframes x 1024 picks, the bench's
  bundle_adjust_frames batch) with the counter-based uniforms, against the
  oracle fed the same uniforms (oracle.pixel_uniforms restates the generator);
- edge cases: every pixel, one pixel, a pixel count that is not a multiple of
  the block chunk, all-equal scores (ties taken in pixel order), zero weights.

Bar: the picked pixel sets are identical.  The scores are f32 logs; the device
logf and torch-CPU's log may differ in the last bit, which can swap two pixels
whose scores are within an ulp of the N-th score — the check allows a swap
only there (a few ulps of the threshold), and none happened when written.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _assert_same_picks(got, mask, u, n):
    ref = O.sample_rays(mask, n, u)
    got = np.asarray(got)
    assert got.shape == ref.shape
    s = O.pixel_scores(mask, u).numpy()
    for b in range(ref.shape[0]):
        assert np.all(np.diff(got[b]) > 0), "picks must be ascending and distinct"
        if np.array_equal(got[b], ref[b]):
            continue
        thr = np.sort(s[b])[::-1][n - 1]
        diff = np.setxor1d(got[b], ref[b])
        near = np.abs(s[b][diff].astype(np.float64) - thr) <= 4 * np.spacing(np.float32(abs(thr)))
        assert near.all(), (b, diff[~near][:8], s[b][diff[~near]][:8], thr)


def test_sample_rays_matches_reference_golden():
    from psvo import sample_util
    g = load_golden("P_pixels")
    for c in range(int(g["n_cases"])):
        mask = torch.from_numpy(g[f"case{c}.mask"])
        u = torch.from_numpy(g[f"case{c}.u"])
        n = int(g[f"case{c}.n"])
        out = sample_util.sample_rays(mask.to(DEV), n, u=u)
        assert out.dtype == torch.bool and out.shape == mask.shape
        got = np.stack([torch.nonzero(out[b].reshape(-1)).squeeze(1).cpu().numpy() for b in range(mask.shape[0])])
        assert got.shape == g[f"case{c}.idx"].shape, c
        _assert_same_picks(got, mask.numpy(), u.numpy(), n)
        assert np.array_equal(got, g[f"case{c}.idx"]), c


class _Frame:
    def __init__(self, H, W, seed):
        gen = torch.Generator().manual_seed(seed)
        self.rays_d = torch.randn(H, W, 3, generator=gen).to(DEV)
        self.rgb = torch.rand(H, W, 3, generator=gen).to(DEV)
        self.depth = (torch.rand(H, W, generator=gen) * 5).to(DEV)


@pytest.mark.parametrize("H,W,F,n", [(680, 1200, 4, 1024), (37, 53, 3, 100), (5, 7, 2, 35), (5, 7, 1, 1)])
def test_sample_frames_matches_oracle(H, W, F, n):
    """Full-size keyframes with the device generator: same picks as the
    oracle on the same uniforms, masks and sample_idx consistent, gathered
    rows = the frames' rows at the picks in torch.cat([f.x[f.sample_mask]]) order."""
    from psvo import sample_util
    frames = [_Frame(H, W, 100 + f) for f in range(F)]
    seed = 987654321
    dirs, rgb, depth = sample_util.sample_frames(frames, n, seed=seed)
    torch.cuda.synchronize()
    u = O.pixel_uniforms(seed, F, H * W)
    got = torch.stack([fr.sample_idx for fr in frames]).cpu().numpy()
    for f, fr in enumerate(frames):
        # frame.sample_rays normalises each frame on its own (B = 1 per frame)
        _assert_same_picks(got[f:f + 1], np.ones((1, H, W), np.float32), u[f:f + 1], n)
        m = fr.sample_mask
        assert m.shape == (H, W) and int(m.sum()) == n
        assert torch.equal(torch.nonzero(m.reshape(-1)).squeeze(1), fr.sample_idx)
        sl = slice(f * n, (f + 1) * n)
        assert torch.equal(dirs[sl], fr.rays_d[m])
        assert torch.equal(rgb[sl], fr.rgb[m])
        assert torch.equal(depth[sl], fr.depth[m])


def test_sample_pixels_edges():
    from psvo import sample_util
    H, W = 33, 41
    n_pix = H * W
    # every pixel
    idx = sample_util.sample_pixels(2, n_pix, n_pix, DEV, seed=3)
    assert torch.equal(idx.cpu(), torch.arange(n_pix).expand(2, -1))
    # all-equal scores: ties taken in pixel order
    u = torch.full((1, n_pix), 0.5)
    idx = sample_util.sample_pixels(1, n_pix, 100, DEV, u=u)
    assert torch.equal(idx.cpu()[0], torch.arange(100))
    # zero weights (a hole in the mask) with the device generator, against the oracle on the same uniforms
    w = torch.ones(1, H, W)
    w[0, :, 20:] = 0.0
    for n in (int((w > 0).sum()) - 3, int((w > 0).sum()) + 5):
        out = sample_util.sample_rays(w.to(DEV), n, seed=11)
        got = torch.nonzero(out.reshape(1, -1)[0]).squeeze(1).cpu().numpy()[None]
        _assert_same_picks(got, w.numpy(), O.pixel_uniforms(11, 1, n_pix), n)
    with pytest.raises(ValueError):
        sample_util.sample_pixels(1, 10, 11, DEV, seed=1)


def test_sample_frames_uniform_distribution():
    """Each pixel is picked with probability n / n_pix: per-row pick counts
    over 64 draws of 1024 from a 68 x 120 frame stay near their mean."""
    from psvo import sample_util
    H, W, n, reps = 68, 120, 1024, 64
    counts = torch.zeros(H * W, dtype=torch.int64, device=DEV)
    for r in range(reps):
        idx = sample_util.sample_pixels(1, H * W, n, DEV, seed=1000 + r)
        counts[idx[0]] += 1
    c = counts.view(H, W).sum(1).double().cpu()  # per image row
    mean = reps * n / H
    assert float((c - mean).abs().max()) < 6 * mean ** 0.5, (float(c.min()), float(c.max()), mean)


@pytest.mark.parametrize("H,W,F,n", [(680, 1200, 4, 1024), (240, 320, 3, 200), (68, 120, 2, 64)])
def test_candidate_band_draw_equals_radix_passes(H, W, F, n):
    """The candidate-band draw (k_px_cand + k_px_pick), its exact fallback
    (the band forced to miss) and the five radix passes give the same picks,
    masks and gathered rows, bit for bit."""
    from psvo import _lib as L
    from psvo import sample_util
    frames = [_Frame(H, W, 300 + f) for f in range(F)]
    outs = []
    try:
        for mode in (0, 1, 2):
            L.call("psvo_debug_set_pixel_draw", mode)
            for seed in (5, 77):
                d, c, z = sample_util.sample_frames(frames, n, seed=seed)
                outs.append((mode, seed, d.clone(), c.clone(), z.clone(),
                             torch.stack([fr.sample_idx for fr in frames]).clone(),
                             torch.stack([fr.sample_mask for fr in frames]).clone()))
    finally:
        L.call("psvo_debug_set_pixel_draw", 0)
    torch.cuda.synchronize()
    by_seed = {}
    for o in outs:
        by_seed.setdefault(o[1], []).append(o)
    for seed, group in by_seed.items():
        ref = group[1]  # the radix passes
        for o in group:
            for a, b in zip(o[2:], ref[2:]):
                assert torch.equal(a, b), (o[0], seed)
        u = O.pixel_uniforms(seed, F, H * W)
        for f in range(F):
            _assert_same_picks(ref[5][f:f + 1].cpu().numpy(), np.ones((1, H, W), np.float32), u[f:f + 1], n)
