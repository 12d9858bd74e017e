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

}  // namespace
}  // namespace psvo

using namespace psvo;

extern "C" int64_t psvo_sample_pixels_workspace_ints(int n_frames, int64_t n_pix) {
    return (int64_t)3 * n_frames * kPxBins + (int64_t)n_frames * 6 +
           (int64_t)n_frames * kPxMaxBlocks * 2 +
           (int64_t)n_frames * kPxMaxBlocks * 2 /* doubles */ + 2 /* alignment */ + (int64_t)n_frames * n_pix;
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
    a.joint_sum = joint_sum ? 1 : 0;
    a.n_frames = n_frames;
    a.hist = workspace;
    a.state = a.hist + (int64_t)3 * n_frames * kPxBins;
    a.counts = a.state + (int64_t)n_frames * 6;
    int *wp = a.counts + (int64_t)n_frames * kPxMaxBlocks * 2;
    wp += ((uintptr_t)wp & 7) ? 1 : 0;
    a.wsum = reinterpret_cast<double *>(wp);
    a.keys = reinterpret_cast<uint32_t *>(a.wsum + (int64_t)n_frames * kPxMaxBlocks);
    PxFrames fr = {};
    if (frames)
        for (int f = 0; f < n_frames; ++f) fr.f[f] = frames[f];
    hipStream_t st = as_stream(stream);
    if (hipMemsetAsync(workspace, 0, sizeof(int) * (3 * n_frames * kPxBins), st) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "sample_pixels: memset failed");
    const dim3 grid(a.nb, n_frames);
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
