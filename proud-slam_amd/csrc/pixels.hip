// Keyframe pixel sampling of the mapping loop on the device.
//
// Reference: every bundle_adjust_frames iteration (render_helpers.py:620-640)
// calls frame.sample_rays(N) per keyframe (frame.py:83-85), i.e.
// sample_util.sample_rays (sample_util.py:4-20):
//   p      = mask / (mask.sum() + 1e-7)                    (f32)
//   score  = log(p + 1e-7) + g,  g = −log(−log(u + 1e-7) + 1e-7),  u ~ U[0, 1)
//   picked = score.topk(N)  → a bool mask of the picked pixels
// then gathers rays_d / rgb / depth of the mask's pixels in row-major order.
// On the reference this is a full sort of H·W scores per keyframe per
// iteration (torch.topk) plus three boolean-mask gathers; here it is one
// radix select for all keyframes together, with the gathers fused into the
// compaction that writes the picked pixels:
//   k_px_hist<0>   scores → orderable u32 keys (stored: 4 B / pixel, read
//                  back by the later passes — three f32 logs per pixel cost
//                  more than the 4-B re-read); 4096-bin histogram of the top
//                  12 key bits (LDS, then one atomic per non-empty bin)
//   k_px_hist<1,2> every block re-derives the previous pass's pick from the
//                  global histogram (4096 bins, L2-resident), then histograms
//                  the next 12 / 8 bits of the keys sharing the picked prefix
//   k_px_count     the exact N-th largest key T: per block, keys > T and = T
//   k_px_write     keys > T, plus the first (N − #{> T}) keys = T in pixel
//                  order, written in pixel order (block offsets summed from
//                  the ≤ 256 block counts of the frame); idx, mask and the
//                  gathered rows
// HBM traffic per pixel: the key written once and read 4 times (20 B), the
// mask (1 B, optional), the weights (4 B, optional); plus the N gathered rows.
//
// The keyframe sampler's case (uniform weights, generated uniforms: the
// 24-bit integer behind u orders the scores, px_key_at FAST) draws k of
// n_pix ≫ k, so its k-th largest key lies near 2²⁴(1 − k/n_pix).  The
// candidate-band draw (round 6) needs one pass over the pixels, not five:
//   k_px_cand  every pixel's key from the counter hash (no memory read);
//              keys ≥ t0 — a band holding k + 8√k + 64 pixels on average —
//              in pixel order into a per-block segment of kPxSeg slots;
//              the mask zeroed
//   k_px_pick  one short 256-thread workgroup per frame: the segments into
//              registers (pixel order), the k-th largest key T among them by
//              two LDS histograms over the band, then the same pick rule as
//              k_px_write over the candidates only: idx, mask ones, the
//              gathered rows.
// Every key ≥ T is a candidate when the band holds ≥ k pixels, so the picks
// are k_px_write's, bit for bit.  A band that missed (fewer than k pixels
// in it: ≈ 8σ below the mean, p < 1e-15; or a full segment) is detected in
// k_px_pick, which then picks over every pixel of the frame itself (slow,
// exact: tests force it with psvo_debug_set_pixel_draw).
#include <hip/hip_runtime.h>

#include <stdlib.h>

#include "psvo_common.h"

namespace psvo {
namespace {

constexpr int kPxThreads = 256;
constexpr int kPxPer = 4;                       // consecutive pixels per thread per round
constexpr int kPxRound = kPxPer * kPxThreads;   // pixels per block per round
constexpr int kPxMaxBlocks = 256;               // blocks per frame
constexpr int kPxBins = 4096;    // 12-bit digits (the last pass: 8 bits)
constexpr int kPxMaxFrames = 32;
constexpr int kPxSeg = 64;            // candidate slots per k_px_cand block (≈ 7 used at the bench's draw)
constexpr int kPxPickRegs = 8;                         // k_px_pick (256 threads per frame): candidates per thread
constexpr int kPxCandMax = kPxThreads * kPxPickRegs;    // candidates k_px_pick holds in registers

struct PxFrames {
    psvo_pixel_frame f[kPxMaxFrames];
};

struct PxArgs {
    int64_t n_pix, k, chunk;     // pixels per frame, picks per frame, pixels per block (whole rounds)
    int nb;                      // blocks per frame
    const float *weights;        // [F, n_pix] or null (all ones)
    const float *u;              // [F, n_pix] or null (counter-based from seed)
    uint64_t seed;
    int joint_sum;               // normalise by the sum over all frames (sample_rays on a [B, H, W] mask)
    int n_frames;
    int *hist;                   // [3][F][4096]
    int *state;                  // [F][3][2]: (prefix, remaining) after passes 0, 1, 2
    int *counts;                 // [F][kPxMaxBlocks][2]: keys > T, keys = T
    double *wsum;                // [F][kPxMaxBlocks] partial weight sums
    uint32_t *keys;              // [F][n_pix] orderable score keys (written by pass 0)
    uint32_t t0;                 // candidate-band draw: the band's lowest key
    int *cand;                   // [F][kPxMaxBlocks][kPxSeg] candidate pixels, per block in pixel order
    int *ccount;                 // [F][kPxMaxBlocks] candidates per block (> kPxSeg: the segment overflowed)
};

__device__ __forceinline__ uint32_t px_mix32(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return (uint32_t)x;
}

// torch.rand_like's 24-bit uniform in [0, 1)
__device__ __forceinline__ float px_uniform(const PxArgs &a, int f, int64_t i) {
    if (a.u) return a.u[(int64_t)f * a.n_pix + i];
    const uint64_t key = a.seed * 0x9E3779B97F4A7C15ull + ((uint64_t)f << 40) + (uint64_t)i;
    return (float)(px_mix32(key) >> 8) * (1.0f / 16777216.0f);
}

// the reference's score in f32 (sample_util.py:5-9, :14-17), as an orderable key
__device__ __forceinline__ uint32_t px_key(const PxArgs &a, int f, int64_t i, float den) {
    const float w = a.weights ? a.weights[(int64_t)f * a.n_pix + i] : 1.0f;
    const float logp = logf(__fadd_rn(__fdiv_rn(w, den), 1e-7f));
    const float uu = px_uniform(a, f, i);
    const float g = -logf(__fadd_rn(-logf(__fadd_rn(uu, 1e-7f)), 1e-7f));
    const float s = __fadd_rn(logp, g);
    const uint32_t b = __float_as_uint(s);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

// Keys.  SCORE: the reference's f32 score (three logs) as a 32-bit key,
// computed and stored by pass 0, streamed back by the later passes.  FAST
// (uniform weights, generated uniforms — the keyframe sampler's case): the
// 24-bit integer m behind u = m·2⁻²⁴ itself, recomputed by every pass.  The score is a non-decreasing
// function of u when every pixel has the same weight (log p is one constant,
// g(u) and f32 rounding are monotone), so the n largest m are n largest
// scores — a tie in score is a tie topk breaks arbitrarily too — with no
// logs and no key array.
template <bool FAST, bool kCompute>
__device__ __forceinline__ uint32_t px_key_at(const PxArgs &a, int f, int64_t i, float den) {
    if constexpr (FAST) {
        const uint64_t key = a.seed * 0x9E3779B97F4A7C15ull + ((uint64_t)f << 40) + (uint64_t)i;
        return px_mix32(key) >> 8;
    } else if constexpr (kCompute) {
        const uint32_t k = px_key(a, f, i, den);
        a.keys[(int64_t)f * a.n_pix + i] = k;
        return k;
    } else {
        return a.keys[(int64_t)f * a.n_pix + i];
    }
}

// radix digits, most significant first: SCORE 12 / 12 / 8 bits, FAST 8 / 8 / 8
// (the 24-bit integer keys are uniform: with 8-bit digits a block flushes at
// most 256 bins to the global histogram, not ~2,600 of 4,096)
template <bool FAST>
constexpr int px_passes() { return 3; }
template <bool FAST>
constexpr int px_shift(int p) { return FAST ? 16 - 8 * p : (p == 0 ? 20 : (p == 1 ? 8 : 0)); }
template <bool FAST>
constexpr int px_width(int p) { return FAST ? 8 : (p == 2 ? 8 : 12); }

// mask.sum() + 1e-7 of the frame (or of all frames): fixed-order sum of the
// per-block partials (exact for 0/1 masks; weights null = all ones)
__device__ __forceinline__ float px_den(const PxArgs &a, int f) {
    double s;
    if (!a.weights) {
        s = (double)a.n_pix * (a.joint_sum ? a.n_frames : 1);
    } else {
        s = 0.0;
        const int f0 = a.joint_sum ? 0 : f, f1 = a.joint_sum ? a.n_frames : f + 1;
        for (int g = f0; g < f1; ++g)
            for (int b = 0; b < a.nb; ++b) s += a.wsum[g * kPxMaxBlocks + b];
    }
    return __fadd_rn((float)s, 1e-7f);
}

__global__ __launch_bounds__(kPxThreads) void k_px_wsum(PxArgs a) {
    __shared__ double part[kPxThreads / kWave];
    const int f = blockIdx.y, b = blockIdx.x;
    const int64_t i0 = (int64_t)b * a.chunk, i1 = min(a.n_pix, i0 + a.chunk);
    double s = 0.0;
    for (int64_t i = i0 + threadIdx.x; i < i1; i += kPxThreads) s += (double)a.weights[(int64_t)f * a.n_pix + i];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < kPxThreads / kWave; ++w) t += part[w];
        a.wsum[f * kPxMaxBlocks + b] = t;
    }
}

// Pick the bin holding the rem-th largest key of a histogram of 256 · BPT
// bins (highest bin first): bin → *bin_out, keys still needed inside it →
// *rem_out.  Thread t owns bins [BPT·t, BPT·t + BPT).
template <int BPT>
__device__ void px_select(const int *__restrict__ h, int rem, int *sh_suffix, int *bin_out, int *rem_out) {
    const int t = threadIdx.x;
    int v[BPT];
    int s = 0;
    for (int j = 0; j < BPT; ++j) {
        v[j] = h[t * BPT + j];
        s += v[j];
    }
    sh_suffix[t] = s;
    __syncthreads();
    // inclusive suffix sum over threads (Hillis-Steele from the top)
    for (int off = 1; off < kPxThreads; off <<= 1) {
        const int x = t + off < kPxThreads ? sh_suffix[t + off] : 0;
        __syncthreads();
        sh_suffix[t] += x;
        __syncthreads();
    }
    const int above = sh_suffix[t] - s;  // keys in the bins of threads t+1..
    if (above < rem && rem <= above + s) {
        int acc = above;
        for (int j = BPT - 1; j >= 0; --j) {
            if (acc + v[j] >= rem) {
                *bin_out = t * BPT + j;
                *rem_out = rem - acc;
                break;
            }
            acc += v[j];
        }
    }
    __syncthreads();
}

// the state after pass P − 1 (P ≥ 1): re-derived from the global histogram of
// pass P − 1 and the state after pass P − 2 (written by the previous kernel)
template <bool FAST, int P>
__device__ void px_state(const PxArgs &a, int f, int *sh_suffix, int *sh_res, uint32_t &prefix, int &rem) {
    uint32_t pfx = 0;
    int r = (int)a.k;
    if (P >= 2) {
        pfx = (uint32_t)a.state[(f * 3 + (P - 2)) * 2 + 0];
        r = a.state[(f * 3 + (P - 2)) * 2 + 1];
    }
    px_select<(1 << px_width<FAST>(P - 1)) / kPxThreads>(a.hist + ((int64_t)(P - 1) * a.n_frames + f) * kPxBins, r,
                                                         sh_suffix, &sh_res[0], &sh_res[1]);
    const uint32_t bin = (uint32_t)sh_res[0];
    // the key bits above px_shift(P − 1), fixed so far (after the last pass: the whole key)
    prefix = P == 1 ? bin : (pfx << px_width<FAST>(P - 1)) | bin;
    rem = sh_res[1];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        a.state[(f * 3 + (P - 1)) * 2 + 0] = (int)prefix;
        a.state[(f * 3 + (P - 1)) * 2 + 1] = rem;
    }
}

// pass P: histogram of digit P of the keys whose higher digits equal the
// prefix picked so far
// (a 16-KB LDS histogram whatever the digit: 1-KB histograms for the FAST
// digits, co-resident with the decoder forward, measured slower — the
// decoder loses more than the draw gains, profiles/r04px_ab_draw_lds.txt)
// SMALL (FAST only, PSVO_PX_SMALL_LDS=1, a measured switch): a 1-KB histogram, so the pass
// fits beside the traversal's 2 × 76.5 KB per CU (with PSVO_BA_DRAW_AFTER_STEP=1)
template <bool FAST, int P, bool SMALL = false>
__global__ __launch_bounds__(kPxThreads) void k_px_hist(PxArgs a) {
    static_assert(!SMALL || FAST, "the 1-KB histogram holds 8-bit digits");
    __shared__ int h[SMALL ? 256 : kPxBins];
    __shared__ int sh_suffix[kPxThreads];
    __shared__ int sh_res[2];
    constexpr int kShift = px_shift<FAST>(P);
    constexpr uint32_t kMask = (1u << px_width<FAST>(P)) - 1u;
    constexpr int kBins = 1 << px_width<FAST>(P);
    const int f = blockIdx.y, b = blockIdx.x;
    for (int j = threadIdx.x; j < kBins; j += kPxThreads) h[j] = 0;
    uint32_t prefix = 0;
    int rem = 0;
    if constexpr (P >= 1) px_state<FAST, P>(a, f, sh_suffix, sh_res, prefix, rem);
    __syncthreads();
    const float den = (!FAST && P == 0) ? px_den(a, f) : 0.0f;
    const int64_t i0 = (int64_t)b * a.chunk, i1 = min(a.n_pix, i0 + a.chunk);
    for (int64_t r0 = i0 + kPxPer * threadIdx.x; r0 < i1; r0 += kPxRound) {
#pragma unroll
        for (int q = 0; q < kPxPer; ++q) {
            const int64_t i = r0 + q;
            if (i >= i1) break;
            const uint32_t key = px_key_at<FAST, P == 0>(a, f, i, den);
            if constexpr (P == 0) {
                atomicAdd(&h[(key >> kShift) & kMask], 1);
            } else {
                if ((key >> px_shift<FAST>(P - 1)) == prefix) atomicAdd(&h[(key >> kShift) & kMask], 1);
            }
        }
    }
    __syncthreads();
    int *gh = a.hist + ((int64_t)P * a.n_frames + f) * kPxBins;
    for (int j = threadIdx.x; j < kBins; j += kPxThreads)
        if (h[j]) atomicAdd(&gh[j], h[j]);
}

// block sum of two counters (result valid in every thread)
__device__ __forceinline__ void px_block_sum2(int &x, int &y, int (*part)[kPxThreads / kWave]) {
    for (int o = 32; o > 0; o >>= 1) {
        x += __shfl_xor(x, o, 64);
        y += __shfl_xor(y, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        part[0][threadIdx.x >> 6] = x;
        part[1][threadIdx.x >> 6] = y;
    }
    __syncthreads();
    x = y = 0;
    for (int w = 0; w < kPxThreads / kWave; ++w) {
        x += part[0][w];
        y += part[1][w];
    }
    __syncthreads();
}

// the exact N-th largest key T of the frame; per block: keys > T, keys = T
template <bool FAST>
__global__ __launch_bounds__(kPxThreads) void k_px_count(PxArgs a) {
    __shared__ int sh_suffix[kPxThreads];
    __shared__ int sh_res[2];
    __shared__ int part[2][kPxThreads / kWave];
    const int f = blockIdx.y, b = blockIdx.x;
    uint32_t T;
    int rem;
    px_state<FAST, px_passes<FAST>()>(a, f, sh_suffix, sh_res, T, rem);
    const float den = 0.0f;
    const int64_t i0 = (int64_t)b * a.chunk, i1 = min(a.n_pix, i0 + a.chunk);
    int gt = 0, eq = 0;
    for (int64_t r0 = i0 + kPxPer * threadIdx.x; r0 < i1; r0 += kPxRound) {
#pragma unroll
        for (int q = 0; q < kPxPer; ++q) {
            const int64_t i = r0 + q;
            if (i >= i1) break;
            const uint32_t key = px_key_at<FAST, false>(a, f, i, den);
            gt += key > T;
            eq += key == T;
        }
    }
    px_block_sum2(gt, eq, part);
    if (threadIdx.x == 0) {
        a.counts[(f * kPxMaxBlocks + b) * 2 + 0] = gt;
        a.counts[(f * kPxMaxBlocks + b) * 2 + 1] = eq;
    }
}

// picked pixels in pixel order: index, mask and the gathered rows.  Pixel p
// is picked if key > T, or key = T and fewer than `ties` keys = T precede it;
// its output row = #{keys > T before p} + min(#{keys = T before p}, ties).
// Both counts come from one packed (eq << 16 | gt) block scan per round of
// 1024 pixels (4 consecutive pixels per thread).
template <bool FAST>
__global__ __launch_bounds__(kPxThreads) void k_px_write(PxArgs a, PxFrames fr, int64_t *__restrict__ idx,
                                                         float *__restrict__ out_dirs, float *__restrict__ out_rgb,
                                                         float *__restrict__ out_depth) {
    __shared__ int part[2][kPxThreads / kWave];
    __shared__ int wave_tot[kPxThreads / kWave];
    const int f = blockIdx.y, b = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int kLast = px_passes<FAST>() - 1;
    const uint32_t T = (uint32_t)a.state[(f * 3 + kLast) * 2 + 0];
    const int ties = a.state[(f * 3 + kLast) * 2 + 1];  // keys = T to take, in pixel order
    int gt_run = 0, eq_run = 0;                     // counts before this block, then before each round
    for (int j = threadIdx.x; j < b; j += kPxThreads) {
        gt_run += a.counts[(f * kPxMaxBlocks + j) * 2 + 0];
        eq_run += a.counts[(f * kPxMaxBlocks + j) * 2 + 1];
    }
    px_block_sum2(gt_run, eq_run, part);
    const float den = 0.0f;
    const psvo_pixel_frame F = fr.f[f];
    const int64_t i0 = (int64_t)b * a.chunk, i1 = min(a.n_pix, i0 + a.chunk);
    for (int64_t rr = i0; rr < i1; rr += kPxRound) {
        const int64_t r0 = rr + kPxPer * threadIdx.x;
        uint32_t key[kPxPer];
        int packed = 0;
#pragma unroll
        for (int q = 0; q < kPxPer; ++q) {
            key[q] = 0;
            if (r0 + q < i1) {
                key[q] = px_key_at<FAST, false>(a, f, r0 + q, den);
                packed += (key[q] > T ? 1 : 0) + (key[q] == T ? (1 << 16) : 0);
            }
        }
        // inclusive wave scan, then the waves before this one
        int inc = packed;
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(inc, o, 64);
            if (lane >= o) inc += v;
        }
        if (lane == 63) wave_tot[wave] = inc;
        __syncthreads();
        int before = inc - packed, round_tot = 0;
        for (int w = 0; w < kPxThreads / kWave; ++w) {
            if (w < wave) before += wave_tot[w];
            round_tot += wave_tot[w];
        }
        __syncthreads();
        int gt_b = gt_run + (before & 0xffff), eq_b = eq_run + (before >> 16);
        uint32_t mword = 0;
#pragma unroll
        for (int q = 0; q < kPxPer; ++q) {
            const int64_t i = r0 + q;
            if (i >= i1) break;
            const bool is_gt = key[q] > T, is_eq = key[q] == T;
            const bool pick = is_gt || (is_eq && eq_b < ties);
            if (pick) {
                const int64_t row = (int64_t)f * a.k + gt_b + min(eq_b, ties);
                if (idx) idx[row] = i;
                if (out_dirs && F.dirs)
                    for (int c = 0; c < 3; ++c) out_dirs[row * 3 + c] = F.dirs[i * 3 + c];
                if (out_rgb && F.rgb)
                    for (int c = 0; c < 3; ++c) out_rgb[row * 3 + c] = F.rgb[i * 3 + c];
                if (out_depth && F.depth) out_depth[row] = F.depth[i];
            }
            mword |= (pick ? 1u : 0u) << (8 * q);
            gt_b += is_gt;
            eq_b += is_eq;
        }
        if (F.mask && r0 < i1) {
            uint8_t *m = F.mask + r0;
            if (r0 + kPxPer <= i1 && ((uintptr_t)m & 3) == 0) {
                *reinterpret_cast<uint32_t *>(m) = mword;
            } else {
                for (int q = 0; q < kPxPer && r0 + q < i1; ++q) m[q] = (uint8_t)(mword >> (8 * q));
            }
        }
        gt_run += round_tot & 0xffff;
        eq_run += round_tot >> 16;
    }
}

// exclusive block scan of one int per thread (any block size ≤ 1024, whole
// waves); returns the prefix, *tot = the block's sum; sh: ≥ 16 ints
__device__ __forceinline__ int px_block_scan(int v, int *sh, int *tot) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    int inc = v;
    for (int o = 1; o < 64; o <<= 1) {
        const int x = __shfl_up(inc, o, 64);
        if (lane >= o) inc += x;
    }
    if (lane == 63) sh[wave] = inc;
    __syncthreads();
    int before = inc - v, t = 0;
    for (int w = 0; w < nw; ++w) {
        before += w < wave ? sh[w] : 0;
        t += sh[w];
    }
    __syncthreads();
    *tot = t;
    return before;
}

// the FAST key (the 24-bit integer behind the pixel's uniform)
__device__ __forceinline__ uint32_t px_hash(const PxArgs &a, int f, int64_t i) {
    return px_key_at<true, false>(a, f, i, 0.0f);
}

// k_px_cand: the band's pixels of block b of frame f, in pixel order; the mask zeroed
__global__ __launch_bounds__(kPxThreads) void k_px_cand(PxArgs a, PxFrames fr) {
    __shared__ int sh[kPxThreads / kWave];
    const int f = blockIdx.y, b = blockIdx.x;
    const int64_t i0 = (int64_t)b * a.chunk, i1 = min(a.n_pix, i0 + a.chunk);
    uint8_t *const mask = fr.f[f].mask;
    int *const seg = a.cand + ((int64_t)f * kPxMaxBlocks + b) * kPxSeg;
    int n = 0;  // candidates of the rounds before (uniform over the block)
    for (int64_t rr = i0; rr < i1; rr += kPxRound) {
        const int64_t r0 = rr + kPxPer * threadIdx.x;
        int flags = 0, c = 0;
#pragma unroll
        for (int q = 0; q < kPxPer; ++q) {
            if (r0 + q < i1 && px_hash(a, f, r0 + q) >= a.t0) {
                flags |= 1 << q;
                ++c;
            }
        }
        if (mask && r0 < i1) {
            uint8_t *m = mask + r0;
            if (r0 + kPxPer <= i1 && ((uintptr_t)m & 3) == 0) {
                *reinterpret_cast<uint32_t *>(m) = 0u;
            } else {
                for (int q = 0; q < kPxPer && r0 + q < i1; ++q) m[q] = 0;
            }
        }
        int tot;
        int pos = n + px_block_scan(c, sh, &tot);
#pragma unroll
        for (int q = 0; q < kPxPer; ++q)
            if ((flags >> q) & 1) {
                if (pos < kPxSeg) seg[pos] = (int)(r0 + q);
                ++pos;
            }
        n += tot;
    }
    if (threadIdx.x == 0) a.ccount[f * kPxMaxBlocks + b] = n;
}

// block sum (every thread gets it); sh: ≥ 16 ints
__device__ __forceinline__ int px_block_sum(int v, int *sh) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    int t = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += sh[w];
    __syncthreads();
    return t;
}

// the k-th largest of n keys key_at(e): the largest T with #{key ≥ T} ≥ k
template <typename KeyAt>
__device__ uint32_t px_kth(int64_t n, int64_t k, KeyAt key_at, int *sh) {
    uint32_t T = 0;
    for (int bit = 23; bit >= 0; --bit) {
        const uint32_t c = T | (1u << bit);
        int cnt = 0;
        for (int64_t e = threadIdx.x; e < n; e += blockDim.x) cnt += key_at(e) >= c;
        if (px_block_sum(cnt, sh) >= k) T = c;
    }
    return T;
}

// pick pixel i into output row `row`: idx, the mask's one, the gathered rows
__device__ __forceinline__ void px_emit(const PxArgs &a, const psvo_pixel_frame &F, int64_t row, int64_t i,
                                        int64_t *__restrict__ idx, float *__restrict__ out_dirs,
                                        float *__restrict__ out_rgb, float *__restrict__ out_depth) {
    if (idx) idx[row] = i;
    if (out_dirs && F.dirs)
        for (int c = 0; c < 3; ++c) out_dirs[row * 3 + c] = F.dirs[i * 3 + c];
    if (out_rgb && F.rgb)
        for (int c = 0; c < 3; ++c) out_rgb[row * 3 + c] = F.rgb[i * 3 + c];
    if (out_depth && F.depth) out_depth[row] = F.depth[i];
    if (F.mask) F.mask[i] = 1;
}

// the picks among n elements in pixel order (element e: key key_at(e), pixel
// pix_at(e)): key > T, or key = T and fewer than `ties` keys = T before it —
// k_px_write's rule; idx, mask ones, gathered rows
template <typename KeyAt, typename PixAt>
__device__ void px_pick_pass(const PxArgs &a, const psvo_pixel_frame &F, int f, int64_t n, uint32_t T, int ties,
                             KeyAt key_at, PixAt pix_at, int *sh, int64_t *__restrict__ idx,
                             float *__restrict__ out_dirs, float *__restrict__ out_rgb,
                             float *__restrict__ out_depth) {
    int gt_run = 0, eq_run = 0;
    for (int64_t base = 0; base < n; base += blockDim.x) {
        const int64_t e = base + threadIdx.x;
        uint32_t key = 0;
        int64_t i = 0;
        if (e < n) {
            key = key_at(e);
            i = pix_at(e);
        }
        const bool in = e < n, is_gt = in && key > T, is_eq = in && key == T;
        int tot;
        const int before = px_block_scan((is_gt ? 1 : 0) + (is_eq ? (1 << 16) : 0), sh, &tot);
        const int gt_b = gt_run + (before & 0xffff), eq_b = eq_run + (before >> 16);
        if (is_gt || (is_eq && eq_b < ties))
            px_emit(a, F, (int64_t)f * a.k + gt_b + min(eq_b, ties), i, idx, out_dirs, out_rgb, out_depth);
        gt_run += tot & 0xffff;
        eq_run += tot >> 16;
    }
}

// The bin of a histogram of 256 · BPT bins (thread t owns [BPT·t, BPT·t +
// BPT), highest bin first) holding the rem-th largest key: bin → res[0],
// keys still needed inside it → res[1] (every thread reads them after).
template <int BPT>
__device__ void px_select_fast(const int *h, int rem, int *sh, int *res) {
    const int t = threadIdx.x;
    int v[BPT];
    int s = 0;
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
        v[j] = h[t * BPT + j];
        s += v[j];
    }
    int tot;
    const int before = px_block_scan(s, sh, &tot);
    const int above = tot - before - s;  // keys in the bins of threads t+1..
    if (above < rem && rem <= above + s) {
        int acc = above;
        for (int j = BPT - 1; j >= 0; --j) {
            if (acc + v[j] >= rem) {
                res[0] = t * BPT + j;
                res[1] = rem - acc;
                break;
            }
            acc += v[j];
        }
    }
    __syncthreads();
}

// One short workgroup of 256 threads per frame (a long-lived one holds a CU
// slot a persistent decoder workgroup then waits for — measured: a one-wave
// pick of ≈ 40 µs cost ≈ 80 µs per step): the band's candidates into
// registers — element e = 256·r + t, pixel order — the k-th largest key T by
// two LDS histograms over the band (≤ 1,024 bins each: the band is at most
// 2¹⁸ keys wide, t0's eligibility), then k_px_write's pick rule in element
// order.  A band that missed: the same rule over every pixel (slow, exact).
__global__ __launch_bounds__(kPxThreads) void k_px_pick(PxArgs a, PxFrames fr, int64_t *__restrict__ idx,
                                                        float *__restrict__ out_dirs, float *__restrict__ out_rgb,
                                                        float *__restrict__ out_depth) {
    __shared__ int s_off[kPxMaxBlocks];
    __shared__ int s_hist[1024];
    __shared__ int sh[kPxThreads / kWave];
    __shared__ int s_res[2];
    const int f = blockIdx.x, t = threadIdx.x;
    const psvo_pixel_frame F = fr.f[f];
    // the segments' offsets in pixel order (nb ≤ 256 = the block)
    const int cnt = t < a.nb ? a.ccount[f * kPxMaxBlocks + t] : 0;
    int n_cand;
    const int off = px_block_scan(min(cnt, kPxSeg), sh, &n_cand);
    const bool full = __syncthreads_or(cnt > kPxSeg) != 0;
    if (t < a.nb) s_off[t] = off;
    for (int j = t; j < 1024; j += kPxThreads) s_hist[j] = 0;
    __syncthreads();
    if (!full && n_cand >= a.k && n_cand <= kPxCandMax) {
        uint32_t h[kPxPickRegs];
        int px[kPxPickRegs];
        // the band's width → the first histogram's shift (≤ 1,024 bins)
        const uint32_t width = 0x1000000u - a.t0;
        int s1 = 0;
        while ((width - 1) >> s1 >= 1024u) ++s1;
#pragma unroll
        for (int r = 0; r < kPxPickRegs; ++r) {
            const int e = r * kPxThreads + t;
            h[r] = 0;
            px[r] = 0;
            if (e < n_cand) {
                // the segment holding e: the last b with s_off[b] ≤ e (a run
                // of empty segments shares its successor's offset)
                int lo = 0, hi = a.nb - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (s_off[mid] <= e) lo = mid;
                    else hi = mid - 1;
                }
                px[r] = a.cand[((int64_t)f * kPxMaxBlocks + lo) * kPxSeg + (e - s_off[lo])];
                h[r] = px_hash(a, f, px[r]);
                atomicAdd(&s_hist[(h[r] - a.t0) >> s1], 1);
            }
        }
        __syncthreads();
        px_select_fast<4>(s_hist, (int)a.k, sh, s_res);
        const uint32_t b1 = (uint32_t)s_res[0];
        const int rem1 = s_res[1];
        for (int j = t; j < 1024; j += kPxThreads) s_hist[j] = 0;
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kPxPickRegs; ++r)
            if (r * kPxThreads + t < n_cand && ((h[r] - a.t0) >> s1) == b1)
                atomicAdd(&s_hist[(h[r] - a.t0) & ((1u << s1) - 1u)], 1);
        __syncthreads();
        px_select_fast<4>(s_hist, rem1, sh, s_res);
        const uint32_t T = a.t0 + ((b1 << s1) | (uint32_t)s_res[0]);
        const int ties = s_res[1];  // keys = T to take, in pixel order
        int gt_run = 0, eq_run = 0;
#pragma unroll
        for (int r = 0; r < kPxPickRegs; ++r) {
            if (r * kPxThreads < n_cand) {  // (block-uniform)
                const bool in = r * kPxThreads + t < n_cand;
                const bool is_gt = in && h[r] > T, is_eq = in && h[r] == T;
                int tot;
                const int before = px_block_scan((is_gt ? 1 : 0) + (is_eq ? (1 << 16) : 0), sh, &tot);
                const int gt_b = gt_run + (before & 0xffff), eq_b = eq_run + (before >> 16);
                if (is_gt || (is_eq && eq_b < ties))
                    px_emit(a, F, (int64_t)f * a.k + gt_b + min(eq_b, ties), px[r], idx, out_dirs, out_rgb,
                            out_depth);
                gt_run += tot & 0xffff;
                eq_run += tot >> 16;
            }
        }
        return;
    }
    // the band missed: every pixel of the frame (exact, slow — p < 1e-15 at
    // the bench's draw; forced in tests)
    auto key_at = [&](int64_t e) { return px_hash(a, f, e); };
    const uint32_t T = px_kth(a.n_pix, a.k, key_at, sh);
    int gt = 0;
    for (int64_t e = t; e < a.n_pix; e += kPxThreads) gt += key_at(e) > T;
    gt = px_block_sum(gt, sh);
    px_pick_pass(a, F, f, a.n_pix, T, (int)a.k - gt, key_at, [](int64_t e) { return e; }, sh, idx, out_dirs,
                 out_rgb, out_depth);
}

}  // namespace
}  // namespace psvo

using namespace psvo;

// tests only: 0 = the candidate-band draw where it applies, 1 = always the
// radix passes, 2 = the band forced to miss (k_px_pick's fallback);
// PSVO_PX_RADIX=1 starts at 1 (a measured switch: bench A/B)
static int g_px_draw_mode = getenv("PSVO_PX_RADIX") && *getenv("PSVO_PX_RADIX") == '1' ? 1 : 0;
extern "C" int psvo_debug_set_pixel_draw(int mode) {
    PSVO_REQUIRE(mode >= 0 && mode <= 2, "debug_set_pixel_draw: mode %d (0..2)", mode);
    g_px_draw_mode = mode;
    return PSVO_OK;
}

extern "C" int64_t psvo_sample_pixels_workspace_ints(int n_frames, int64_t n_pix) {
    return (int64_t)3 * n_frames * kPxBins + (int64_t)n_frames * 6 +
           (int64_t)n_frames * kPxMaxBlocks * 2 +
           (int64_t)n_frames * kPxMaxBlocks * 2 /* doubles */ + 2 /* alignment */ + (int64_t)n_frames * n_pix +
           (int64_t)n_frames * kPxMaxBlocks * (kPxSeg + 1) /* candidate segments + counts */;
}

extern "C" int psvo_sample_pixels(void *stream, int n_frames, int64_t n_pix, int64_t k, const float *weights,
                                  int joint_sum, const float *u, uint64_t seed, const psvo_pixel_frame *frames,
                                  int *workspace, int64_t *idx, float *out_dirs, float *out_rgb, float *out_depth) {
    PSVO_REQUIRE(n_frames >= 1 && n_frames <= kPxMaxFrames, "sample_pixels: %d frames (1..%d)", n_frames,
                 kPxMaxFrames);
    PSVO_REQUIRE(n_pix >= 1 && n_pix <= 0x7fffffff, "sample_pixels: bad pixel count %lld", (long long)n_pix);
    PSVO_REQUIRE(k >= 1 && k <= n_pix && k < 65536 * 64, "sample_pixels: cannot take %lld of %lld pixels",
                 (long long)k, (long long)n_pix);
    PSVO_REQUIRE(workspace != nullptr, "sample_pixels: null workspace");
    PxArgs a;
    a.n_pix = n_pix;
    a.k = k;
    // pixels per block: whole rounds of 1024, at most kPxMaxBlocks blocks per frame
    const int64_t per = (n_pix + kPxMaxBlocks - 1) / kPxMaxBlocks;
    a.chunk = ((per < kPxRound ? kPxRound : per) + kPxRound - 1) / kPxRound * kPxRound;
    a.nb = (int)((n_pix + a.chunk - 1) / a.chunk);
    a.weights = weights;
    a.u = u;
    a.seed = seed;
    a.t0 = 0;
    a.joint_sum = joint_sum ? 1 : 0;
    a.n_frames = n_frames;
    a.hist = workspace;
    a.state = a.hist + (int64_t)3 * n_frames * kPxBins;
    a.counts = a.state + (int64_t)n_frames * 6;
    int *wp = a.counts + (int64_t)n_frames * kPxMaxBlocks * 2;
    wp += ((uintptr_t)wp & 7) ? 1 : 0;
    a.wsum = reinterpret_cast<double *>(wp);
    a.keys = reinterpret_cast<uint32_t *>(a.wsum + (int64_t)n_frames * kPxMaxBlocks);
    a.cand = reinterpret_cast<int *>(a.keys + (int64_t)n_frames * n_pix);
    a.ccount = a.cand + (int64_t)n_frames * kPxMaxBlocks * kPxSeg;
    PxFrames fr = {};
    if (frames)
        for (int f = 0; f < n_frames; ++f) fr.f[f] = frames[f];
    hipStream_t st = as_stream(stream);
    const dim3 grid(a.nb, n_frames);
    if (!weights && !u && g_px_draw_mode != 1) {
        // the candidate band: k + 8√k + 64 pixels expected, ≤ 16 per block on
        // average (kPxSeg = 64 slots), ≤ 3/4 of kPxCandMax in all
        const double m = (double)k + 8.0 * sqrt((double)k) + 64.0;
        const double per_block = m * (double)a.chunk / (double)n_pix;
        const double t0 = 16777216.0 - ceil(m * 16777216.0 / (double)n_pix);
        if (t0 >= 1.0 && per_block <= 16.0 && m <= 0.75 * kPxCandMax) {
            a.t0 = g_px_draw_mode == 2 ? 0xffffffu : (uint32_t)t0;
            psvo::launch(k_px_cand, grid, dim3(kPxThreads), 0, st, a, fr);
            psvo::launch(k_px_pick, dim3(n_frames), dim3(kPxThreads), 0, st, a, fr, idx, out_dirs, out_rgb,
                         out_depth);
            return check_launch("sample_pixels");
        }
    }
    if (hipMemsetAsync(workspace, 0, sizeof(int) * (3 * n_frames * kPxBins), st) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "sample_pixels: memset failed");
    if (weights) psvo::launch(k_px_wsum, grid, dim3(kPxThreads), 0, st, a);
    if (!weights && !u) {  // uniform weights, generated uniforms: 24-bit integer keys
        static const bool small = getenv("PSVO_PX_SMALL_LDS") && *getenv("PSVO_PX_SMALL_LDS") == '1';
        if (small) {
            psvo::launch((k_px_hist<true, 0, true>), grid, dim3(kPxThreads), 0, st, a);
            psvo::launch((k_px_hist<true, 1, true>), grid, dim3(kPxThreads), 0, st, a);
            psvo::launch((k_px_hist<true, 2, true>), grid, dim3(kPxThreads), 0, st, a);
        } else {
            psvo::launch((k_px_hist<true, 0>), grid, dim3(kPxThreads), 0, st, a);
            psvo::launch((k_px_hist<true, 1>), grid, dim3(kPxThreads), 0, st, a);
            psvo::launch((k_px_hist<true, 2>), grid, dim3(kPxThreads), 0, st, a);
        }
        psvo::launch(k_px_count<true>, grid, dim3(kPxThreads), 0, st, a);
        psvo::launch(k_px_write<true>, grid, dim3(kPxThreads), 0, st, a, fr, idx, out_dirs, out_rgb, out_depth);
    } else {
        psvo::launch((k_px_hist<false, 0>), grid, dim3(kPxThreads), 0, st, a);
        psvo::launch((k_px_hist<false, 1>), grid, dim3(kPxThreads), 0, st, a);
        psvo::launch((k_px_hist<false, 2>), grid, dim3(kPxThreads), 0, st, a);
        psvo::launch(k_px_count<false>, grid, dim3(kPxThreads), 0, st, a);
        psvo::launch(k_px_write<false>, grid, dim3(kPxThreads), 0, st, a, fr, idx, out_dirs, out_rgb,
                           out_depth);
    }
    return check_launch("sample_pixels");
}
