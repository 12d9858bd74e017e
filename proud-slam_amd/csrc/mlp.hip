// NRGBD decoder (src/variations/nrgbd.py:80-146, depth 2, width 128, input
// 16, embedder 'none', skips [] — every shipped Replica config) as fused
// fp32-MFMA kernels for gfx950.
//
//   h1 = relu(W1 x + b1)           W1 [128,16]
//   h2 = relu(W2 h1 + b2)          W2 [128,128]
//   o  = W3 h2 + b3 = [sdf | f]    W3 [129,128]
//   c1 = relu(W4 [f; x] + b4)      W4 [128,144]
//   rgb = sigmoid(W5 c1 + b5)      W5 [3,128]
//
// Layout ("transposed" chain): a wave owns 32 samples and keeps every
// activation as feature-rows x sample-columns in v_mfma_f32_32x32x2_f32
// accumulator form — lane l holds sample l&31, register r of block b holds
// feature 32b + phi(r, l>>5), phi(r,h) = (r&3) + 8(r>>2) + 4h.  The next
// layer consumes that register directly as its B operand (k-pair
// {phi(r,0), phi(r,1)}), so the chain needs no LDS round trip and no
// shuffles; the A operand (weights) is read from LDS in a layout permuted to
// match (one ds_read_b128 feeds 4 MFMAs).  A workgroup = 4 waves = 128
// samples; each layer's weights are staged into LDS (≤ 73.7 KB) once per
// workgroup, two workgroups per CU.  fp32 in, fp32 accumulate (exact fmaf
// chains, no TF32-like rounding): the numerics class of the reference.
#include <hip/hip_runtime.h>

#include "psvo_common.h"

namespace psvo {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kW = 128;     // decoder width
constexpr int kIn = 16;     // embedding dim
constexpr int kNB = kW / 32;
constexpr int kTile = 128;  // samples per workgroup
constexpr int kThreads = 256;

// LDS carve (floats): small vectors first, then the staged weight image.
constexpr int kOffB1 = 0, kOffB2 = kOffB1 + 128, kOffB3 = kOffB2 + 128, kOffB4 = kOffB3 + 132,
              kOffB5 = kOffB4 + 128;                  // biases b1 b2 b3[129] b4 b5[3]
constexpr int kOffW3r0 = kOffB5 + 4, kOffW5 = kOffW3r0 + 128;  // W3 row 0 (sdf), W5 [3][128]
constexpr int kOffW = kOffW5 + 3 * 128;               // = 1032 floats (16-B aligned)
constexpr int kImgFwd = 128 * 144;                    // largest forward image (W4)
constexpr int kImgBwd = 160 * 128;                    // largest backward image (W4ᵀ, 5 x 4 blocks)
constexpr int kLdsFwd = (kOffW + kImgFwd) * 4;        // 77,856 B → 2 workgroups / CU
constexpr int kLdsBwd = (kOffW + kImgBwd) * 4;        // 86,048 B

__device__ __forceinline__ int phi(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// Position of M[i][k] (product row i, reduction index k fed from
// accumulator blocks) in the A-operand image [ib][kb][rg][lane][4].
__device__ __forceinline__ int perm_acc(int i, int k, int nkb) {
    const int ib = i >> 5, ii = i & 31;
    const int kb = k >> 5, kk = k & 31;
    const int r = (kk & 3) | ((kk >> 3) << 2);
    const int h = (kk >> 2) & 1;
    const int lane = ii + 32 * h;
    return ((((ib * nkb + kb) * 4 + (r >> 2)) * 64 + lane) << 2) + (r & 3);
}
// Same for a 16-wide reduction fed from the x registers: k-step t takes
// k = 2t + h, 8 steps grouped by 4: [ib][tg][lane][4].
__device__ __forceinline__ int perm_x(int i, int k) {
    const int ib = i >> 5, ii = i & 31;
    const int t = k >> 1, h = k & 1;
    const int lane = ii + 32 * h;
    return (((ib * 2 + (t >> 2)) * 64 + lane) << 2) + (t & 3);
}

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// acc[ob] += image(`wl`: NOUT x NIN blocks) · in[kb]
template <int NIN, int NOUT>
__device__ __forceinline__ void gemm_acc(const float *wl, const f32x16 (&in)[NIN], f32x16 (&acc)[NOUT], int lane) {
#pragma unroll
    for (int kb = 0; kb < NIN; ++kb) {
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) {
#pragma unroll
            for (int ob = 0; ob < NOUT; ++ob) {
                const float4 a = *reinterpret_cast<const float4 *>(wl + ((((ob * NIN + kb) * 4 + rg) * 64 + lane) << 2));
                acc[ob] = mfma(a.x, in[kb][4 * rg + 0], acc[ob]);
                acc[ob] = mfma(a.y, in[kb][4 * rg + 1], acc[ob]);
                acc[ob] = mfma(a.z, in[kb][4 * rg + 2], acc[ob]);
                acc[ob] = mfma(a.w, in[kb][4 * rg + 3], acc[ob]);
            }
        }
    }
}

// acc[ob] += image(perm_x) · x  (x[t] = x feature 2t + h)
__device__ __forceinline__ void gemm_x(const float *wl, const float (&x)[8], f32x16 (&acc)[kNB], int lane) {
#pragma unroll
    for (int tg = 0; tg < 2; ++tg) {
#pragma unroll
        for (int ob = 0; ob < kNB; ++ob) {
            const float4 a = *reinterpret_cast<const float4 *>(wl + (((ob * 2 + tg) * 64 + lane) << 2));
            acc[ob] = mfma(a.x, x[4 * tg + 0], acc[ob]);
            acc[ob] = mfma(a.y, x[4 * tg + 1], acc[ob]);
            acc[ob] = mfma(a.z, x[4 * tg + 2], acc[ob]);
            acc[ob] = mfma(a.w, x[4 * tg + 3], acc[ob]);
        }
    }
}

template <int N>
__device__ __forceinline__ void zero(f32x16 (&acc)[N]) {
#pragma unroll
    for (int b = 0; b < N; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[b][r] = 0.0f;
}

__device__ __forceinline__ void init_bias(f32x16 (&acc)[kNB], const float *b, int h) {
#pragma unroll
    for (int ob = 0; ob < kNB; ++ob)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[ob][r] = b[32 * ob + phi(r, h)];
}

// ReLU in place; returns the (value > 0) mask, bit 16b + r.
__device__ __forceinline__ uint64_t relu(f32x16 (&v)[kNB]) {
    uint64_t m = 0;
#pragma unroll
    for (int b = 0; b < kNB; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const bool pos = v[b][r] > 0.0f;
            v[b][r] = pos ? v[b][r] : 0.0f;
            m |= (uint64_t)pos << (16 * b + r);
        }
    return m;
}

__device__ __forceinline__ void apply_mask(f32x16 (&v)[kNB], uint64_t m) {
#pragma unroll
    for (int b = 0; b < kNB; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) v[b][r] = ((m >> (16 * b + r)) & 1) ? v[b][r] : 0.0f;
}

// Σ_k w[k] · v[k][sample] over this lane's 64 features (other half via partner lane)
__device__ __forceinline__ float row_dot(const float *w, const f32x16 (&v)[kNB], int h) {
    float s = 0.f;
#pragma unroll
    for (int b = 0; b < kNB; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) s += w[32 * b + phi(r, h)] * v[b][r];
    return s + __shfl_xor(s, 32, 64);
}

// Store an activation held in accumulator form as rows of a row-major
// [M][ld] matrix (sample s = lane's column): 16-B stores.
__device__ __forceinline__ void store_rows(float *dst, int64_t s, bool valid, int ld, const f32x16 (&v)[kNB], int h) {
    if (!valid) return;
    float *row = dst + s * ld;
#pragma unroll
    for (int b = 0; b < kNB; ++b)
#pragma unroll
        for (int rg = 0; rg < 4; ++rg)
            *reinterpret_cast<float4 *>(row + 32 * b + 8 * rg + 4 * h) =
                make_float4(v[b][4 * rg], v[b][4 * rg + 1], v[b][4 * rg + 2], v[b][4 * rg + 3]);
}

// Forward image of W[rows][cols] (global row-major, first row `row0`):
// columns < acc_cols come from accumulator blocks, the rest from x.
template <int NT>
__device__ __forceinline__ void stage_fwd(float *wl, const float *__restrict__ W, int rows, int cols, int row0,
                                          int acc_cols) {
    const int n = rows * cols;
    const int xbase = (rows >> 5) * (acc_cols >> 5) * 16 * 64;
    for (int e = threadIdx.x; e < n; e += NT) {
        const int o = e / cols, k = e - o * cols;
        const float v = W[(int64_t)(o + row0) * cols + k];
        wl[k < acc_cols ? perm_acc(o, k, acc_cols >> 5) : xbase + perm_x(o, k - acc_cols)] = v;
    }
}

// Backward (transposed) image of W[rows][cols]: product rows = columns of W
// (padded to `out_blocks` x 32), reduction over W's rows (from δ blocks).
template <int NT>
__device__ __forceinline__ void stage_bwd(float *wl, const float *__restrict__ W, int rows, int cols, int row0,
                                          int out_blocks) {
    const int nimg = out_blocks * (rows >> 5) * 1024;
    for (int e = threadIdx.x; e < nimg; e += NT) wl[e] = 0.0f;
    __syncthreads();
    const int n = rows * cols;
    for (int e = threadIdx.x; e < n; e += NT) {
        const int o = e / cols, k = e - o * cols;
        wl[perm_acc(k, o, rows >> 5)] = W[(int64_t)(o + row0) * cols + k];
    }
}

struct MlpParams {
    const float *w1, *b1, *w2, *b2, *w3, *b3, *w4, *b4, *w5, *b5;
};

__device__ __forceinline__ void stage_vectors(float *lds, const MlpParams &p) {
    for (int e = threadIdx.x; e < 128; e += kThreads) {
        lds[kOffB1 + e] = p.b1[e];
        lds[kOffB2 + e] = p.b2[e];
        lds[kOffB4 + e] = p.b4[e];
        lds[kOffW3r0 + e] = p.w3[e];  // W3 row 0 (sdf)
        lds[kOffW5 + e] = p.w5[e];
        lds[kOffW5 + 128 + e] = p.w5[128 + e];
        lds[kOffW5 + 256 + e] = p.w5[256 + e];
    }
    for (int e = threadIdx.x; e < 129; e += kThreads) lds[kOffB3 + e] = p.b3[e];
    if (threadIdx.x < 3) lds[kOffB5 + threadIdx.x] = p.b5[threadIdx.x];
}

__device__ __forceinline__ float sigmoidf(float x) { return 1.0f / (1.0f + expf(-x)); }

__device__ __forceinline__ void load_x(const float *__restrict__ feat, int64_t s, bool valid, int h, float (&x)[8]) {
    const float *fr = feat + (valid ? s : 0) * kIn;
#pragma unroll
    for (int t = 0; t < 8; ++t) x[t] = valid ? fr[2 * t + h] : 0.0f;
}

// ---------------------------------------------------------------------------
// forward: feat[M,16] → sdf[M], rgb[M,3]
__global__ __launch_bounds__(kThreads, 2) void k_mlp_fwd(int64_t m, const float *__restrict__ feat, MlpParams p,
                                                         float *__restrict__ sdf_out, float *__restrict__ rgb_out) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float *wl = lds + kOffW;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int h = lane >> 5;
    const int64_t s = (int64_t)blockIdx.x * kTile + wave * 32 + (lane & 31);
    const bool valid = s < m;
    float x[8];
    load_x(feat, s, valid, h, x);
    stage_vectors(lds, p);
    stage_fwd<kThreads>(wl, p.w1, 128, 16, 0, 0);
    __syncthreads();
    f32x16 a[kNB], bacc[kNB];
    init_bias(a, lds + kOffB1, h);
    gemm_x(wl, x, a, lane);
    relu(a);  // h1
    __syncthreads();
    stage_fwd<kThreads>(wl, p.w2, 128, 128, 0, 128);
    __syncthreads();
    init_bias(bacc, lds + kOffB2, h);
    gemm_acc<kNB, kNB>(wl, a, bacc, lane);
    relu(bacc);  // h2
    __syncthreads();
    stage_fwd<kThreads>(wl, p.w3, 128, 128, 1, 128);  // rows 1..128 → f
    __syncthreads();
    const float sdf = lds[kOffB3] + row_dot(lds + kOffW3r0, bacc, h);
    init_bias(a, lds + kOffB3 + 1, h);
    gemm_acc<kNB, kNB>(wl, bacc, a, lane);  // f
    __syncthreads();
    stage_fwd<kThreads>(wl, p.w4, 128, 144, 0, 128);  // [f | x]
    __syncthreads();
    init_bias(bacc, lds + kOffB4, h);
    gemm_acc<kNB, kNB>(wl, a, bacc, lane);
    gemm_x(wl + kNB * kNB * 16 * 64, x, bacc, lane);
    relu(bacc);  // c1
    float rgb[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = sigmoidf(lds[kOffB5 + c] + row_dot(lds + kOffW5 + 128 * c, bacc, h));
    if (valid && h == 0) {
        sdf_out[s] = sdf;
        rgb_out[s * 3 + 0] = rgb[0];
        rgb_out[s * 3 + 1] = rgb[1];
        rgb_out[s * 3 + 2] = rgb[2];
    }
}

// ---------------------------------------------------------------------------
// backward (data): recompute the forward, then chain the δ's down to dx.
// Writes the row-major operands of the weight gradients:
//   A1 = h1, A2 = h2, A3 = f, A4 = c1           [M][128]
//   D1 = δh1, D2 = δh2, D3 = δf, D4 = δc1       [M][128]   (post-ReLU-mask)
//   D5 = δ(rgb logits) [M][3];  dfeat [M][16]
struct BwdOut {
    float *a1, *a2, *a3, *a4, *d1, *d2, *d3, *d4, *d5, *dfeat;
};

constexpr int kThreadsBwd = 512;
constexpr int kTileBwd = 256;

__global__ __launch_bounds__(kThreadsBwd, 1) void k_mlp_bwd_data(int64_t m, const float *__restrict__ feat,
                                                                 MlpParams p, const float *__restrict__ g_sdf,
                                                                 const float *__restrict__ g_rgb, BwdOut o) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float *wl = lds + kOffW;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int h = lane >> 5;
    const int64_t s = (int64_t)blockIdx.x * kTileBwd + wave * 32 + (lane & 31);
    const bool valid = s < m;
    float x[8];
    load_x(feat, s, valid, h, x);
    stage_vectors(lds, p);
    // ---- recompute forward
    stage_fwd<kThreadsBwd>(wl, p.w1, 128, 16, 0, 0);
    __syncthreads();
    f32x16 a[kNB], bacc[kNB];
    init_bias(a, lds + kOffB1, h);
    gemm_x(wl, x, a, lane);
    const uint64_t m1 = relu(a);
    store_rows(o.a1, s, valid, 128, a, h);
    __syncthreads();
    stage_fwd<kThreadsBwd>(wl, p.w2, 128, 128, 0, 128);
    __syncthreads();
    init_bias(bacc, lds + kOffB2, h);
    gemm_acc<kNB, kNB>(wl, a, bacc, lane);
    const uint64_t m2 = relu(bacc);
    store_rows(o.a2, s, valid, 128, bacc, h);
    __syncthreads();
    stage_fwd<kThreadsBwd>(wl, p.w3, 128, 128, 1, 128);
    __syncthreads();
    init_bias(a, lds + kOffB3 + 1, h);
    gemm_acc<kNB, kNB>(wl, bacc, a, lane);  // f
    store_rows(o.a3, s, valid, 128, a, h);
    __syncthreads();
    stage_fwd<kThreadsBwd>(wl, p.w4, 128, 144, 0, 128);
    __syncthreads();
    init_bias(bacc, lds + kOffB4, h);
    gemm_acc<kNB, kNB>(wl, a, bacc, lane);
    gemm_x(wl + kNB * kNB * 16 * 64, x, bacc, lane);
    const uint64_t m4 = relu(bacc);  // c1
    store_rows(o.a4, s, valid, 128, bacc, h);
    float d5[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float y = sigmoidf(lds[kOffB5 + c] + row_dot(lds + kOffW5 + 128 * c, bacc, h));
        const float g = valid ? g_rgb[s * 3 + c] : 0.0f;
        d5[c] = g * (y * (1.0f - y));
    }
    if (valid && h == 0) {
        o.d5[s * 3 + 0] = d5[0];
        o.d5[s * 3 + 1] = d5[1];
        o.d5[s * 3 + 2] = d5[2];
    }
    // ---- δc1 = W5ᵀ δ5 ⊙ mask   (VALU)
#pragma unroll
    for (int b = 0; b < kNB; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int k = 32 * b + phi(r, h);
            const float v = lds[kOffW5 + k] * d5[0] + lds[kOffW5 + 128 + k] * d5[1] + lds[kOffW5 + 256 + k] * d5[2];
            bacc[b][r] = ((m4 >> (16 * b + r)) & 1) ? v : 0.0f;
        }
    store_rows(o.d4, s, valid, 128, bacc, h);
    // ---- [δf ; δx_c] = W4ᵀ δc1   (5 row blocks: f rows 0..127, x rows 128..143)
    __syncthreads();
    stage_bwd<kThreadsBwd>(wl, p.w4, 128, 144, 0, 5);
    __syncthreads();
    f32x16 t5[5];
    zero(t5);
    gemm_acc<kNB, 5>(wl, bacc, t5, lane);
    float dxc[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) dxc[r] = t5[4][r];
#pragma unroll
    for (int b = 0; b < kNB; ++b) a[b] = t5[b];  // δf
    store_rows(o.d3, s, valid, 128, a, h);
    const float dsdf = valid ? g_sdf[s] : 0.0f;
    // ---- δh2 = (W3[1:]ᵀ δf + W3[0]ᵀ δsdf) ⊙ mask
    __syncthreads();
    stage_bwd<kThreadsBwd>(wl, p.w3, 128, 128, 1, 4);
    __syncthreads();
#pragma unroll
    for (int b = 0; b < kNB; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) bacc[b][r] = lds[kOffW3r0 + 32 * b + phi(r, h)] * dsdf;
    gemm_acc<kNB, kNB>(wl, a, bacc, lane);
    apply_mask(bacc, m2);
    store_rows(o.d2, s, valid, 128, bacc, h);
    // ---- δh1 = W2ᵀ δh2 ⊙ mask
    __syncthreads();
    stage_bwd<kThreadsBwd>(wl, p.w2, 128, 128, 0, 4);
    __syncthreads();
    zero(a);
    gemm_acc<kNB, kNB>(wl, bacc, a, lane);
    apply_mask(a, m1);
    store_rows(o.d1, s, valid, 128, a, h);
    // ---- dx = W1ᵀ δh1 + δx_c   (one row block, rows 0..15 valid)
    __syncthreads();
    stage_bwd<kThreadsBwd>(wl, p.w1, 128, 16, 0, 1);
    __syncthreads();
    f32x16 t1[1];
    zero(t1);
    gemm_acc<kNB, 1>(wl, a, t1, lane);
    if (valid) {
        float *dst = o.dfeat + s * kIn;
#pragma unroll
        for (int rg = 0; rg < 2; ++rg)
            *reinterpret_cast<float4 *>(dst + 8 * rg + 4 * h) =
                make_float4(t1[0][4 * rg] + dxc[4 * rg], t1[0][4 * rg + 1] + dxc[4 * rg + 1],
                            t1[0][4 * rg + 2] + dxc[4 * rg + 2], t1[0][4 * rg + 3] + dxc[4 * rg + 3]);
    }
}

// ---------------------------------------------------------------------------
// backward (weights): dW[rows][cols] = Σ_s D[s][row] · A[s][col], db = Σ_s D[s].
// Split-K over samples; each workgroup writes a private slab (fixed-order,
// deterministic reduction in k_mlp_dw_reduce).
struct DwLayer {
    const float *D;   // [M][ldD], rows [d_row0, rows)
    const float *D0;  // optional row 0 column (δsdf) → D rows start at 1
    int ldD, rows;
    const float *A;   // [M][ldA], first a_cols columns
    const float *A2;  // [M][16] extra columns (x)
    int ldA, a_cols, cols;
    int slab_off;     // offset of this layer's (rows*cols + rows) in a slab
};
struct DwArgs {
    DwLayer L[5];
    int slab_stride;
};

constexpr int kDwChunk = 32;
constexpr int kDwLd = 160;  // padded LDS row (5 blocks)

__global__ __launch_bounds__(256) void k_mlp_dw(int64_t m, DwArgs args, int n_split, float *__restrict__ slabs) {
    __shared__ __attribute__((aligned(16))) float Dl[kDwChunk * kDwLd];
    __shared__ __attribute__((aligned(16))) float Al[kDwChunk * kDwLd];
    const DwLayer &L = args.L[blockIdx.y];
    const int split = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, i = lane & 31;
    const int RB = (L.rows + 31) >> 5, CB = (L.cols + 31) >> 5;
    const int nblk = RB * CB;
    const int64_t n_chunks = (m + kDwChunk - 1) / kDwChunk;
    const int64_t c_beg = n_chunks * split / n_split, c_end = n_chunks * (split + 1) / n_split;
    f32x16 acc[5];
    zero(acc);
    float bias = 0.0f;
    const int d_shift = L.D0 ? 1 : 0;
    for (int64_t c = c_beg; c < c_end; ++c) {
        const int64_t s0 = c * kDwChunk;
        __syncthreads();
        for (int e = threadIdx.x; e < kDwChunk * kDwLd; e += 256) {
            const int ss = e / kDwLd, col = e - ss * kDwLd;
            const int64_t sg = s0 + ss;
            float dv = 0.0f, av = 0.0f;
            if (sg < m) {
                if (col < L.rows) {
                    if (d_shift && col == 0)
                        dv = L.D0[sg];
                    else
                        dv = L.D[sg * L.ldD + col - d_shift];
                }
                if (col < L.a_cols)
                    av = L.A[sg * L.ldA + col];
                else if (col < L.cols)
                    av = L.A2[sg * 16 + (col - L.a_cols)];
            }
            Dl[e] = dv;
            Al[e] = av;
        }
        __syncthreads();
        if (threadIdx.x < L.rows) {
#pragma unroll 8
            for (int ss = 0; ss < kDwChunk; ++ss) bias += Dl[ss * kDwLd + threadIdx.x];
        }
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const int bid = wave + 4 * j;
            if (bid < nblk) {
                const int rb = bid / CB, cb = bid - rb * CB;
#pragma unroll 4
                for (int t = 0; t < kDwChunk / 2; ++t) {
                    const int row = 2 * t + h;
                    acc[j] = mfma(Dl[row * kDwLd + 32 * rb + i], Al[row * kDwLd + 32 * cb + i], acc[j]);
                }
            }
        }
    }
    float *slab = slabs + (int64_t)split * args.slab_stride + L.slab_off;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const int bid = wave + 4 * j;
        if (bid < nblk) {
            const int rb = bid / CB, cb = bid - rb * CB;
            const int col = 32 * cb + i;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = 32 * rb + phi(r, h);
                if (row < L.rows && col < L.cols) slab[row * L.cols + col] = acc[j][r];
            }
        }
    }
    if (threadIdx.x < L.rows) slab[L.rows * L.cols + threadIdx.x] = bias;
}

// grads[e] = Σ_split slabs[split][e], e over the packed (W, b) of all layers,
// scattered to the five (weight, bias) gradient buffers.
struct DwDst {
    float *w[5], *b[5];
    int off[5], rows[5], cols[5];
};

__global__ void k_mlp_dw_reduce(int n_split, int slab_stride, const float *__restrict__ slabs, DwDst dst,
                                int accumulate) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= slab_stride) return;
    float v = 0.0f;
    for (int sp = 0; sp < n_split; ++sp) v += slabs[(int64_t)sp * slab_stride + e];
#pragma unroll
    for (int l = 0; l < 5; ++l) {
        const int rel = e - dst.off[l];
        const int nw = dst.rows[l] * dst.cols[l];
        if (rel >= 0 && rel < nw + dst.rows[l]) {
            float *p = rel < nw ? dst.w[l] + rel : dst.b[l] + (rel - nw);
            *p = accumulate ? *p + v : v;
        }
    }
}

}  // namespace
}  // namespace psvo

using namespace psvo;

extern "C" int psvo_mlp_fwd(void *stream, int64_t m, int width, const float *feat, const float *w1, const float *b1,
                            const float *w2, const float *b2, const float *w3, const float *b3, const float *w4,
                            const float *b4, const float *w5, const float *b5, float *sdf, float *rgb) {
    PSVO_REQUIRE(width == kW, "mlp_fwd: width %d unsupported (fused path is width 128)", width);
    PSVO_REQUIRE(m >= 0, "mlp_fwd: m < 0");
    if (m == 0) return PSVO_OK;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_mlp_fwd),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, kLdsFwd);
        attr = true;
    }
    MlpParams p{w1, b1, w2, b2, w3, b3, w4, b4, w5, b5};
    hipLaunchKernelGGL(k_mlp_fwd, dim3(div_up(m, kTile)), dim3(kThreads), kLdsFwd, as_stream(stream), m, feat, p,
                       sdf, rgb);
    return check_launch("mlp_fwd");
}

// Packed slab layout (floats): per layer rows*cols weights then rows biases.
static void dw_layout(int off[5], int rows[5], int cols[5], int *stride) {
    const int R[5] = {128, 128, 129, 128, 3}, C[5] = {16, 128, 128, 144, 128};
    int o = 0;
    for (int l = 0; l < 5; ++l) {
        rows[l] = R[l];
        cols[l] = C[l];
        off[l] = o;
        o += R[l] * C[l] + R[l];
    }
    *stride = (o + 63) & ~63;
}

extern "C" int64_t psvo_mlp_workspace_floats(int64_t m, int n_split) {
    int off[5], rows[5], cols[5], stride;
    dw_layout(off, rows, cols, &stride);
    return m * (8 * 128 + 3 + 16) + (int64_t)n_split * stride;
}

// Full decoder backward: grads of the 10 parameters (overwritten, or added
// to when `accumulate`) and dfeat [M,16].  `workspace` holds the row-major
// activations / deltas and the split-K slabs (psvo_mlp_workspace_floats).
extern "C" int psvo_mlp_bwd(void *stream, int64_t m, int width, const float *feat, const float *w1, const float *b1,
                            const float *w2, const float *b2, const float *w3, const float *b3, const float *w4,
                            const float *b4, const float *w5, const float *b5, const float *g_sdf,
                            const float *g_rgb, float *dfeat, float *gw1, float *gb1, float *gw2, float *gb2,
                            float *gw3, float *gb3, float *gw4, float *gb4, float *gw5, float *gb5,
                            int accumulate, int n_split, float *workspace) {
    PSVO_REQUIRE(width == kW, "mlp_bwd: width %d unsupported (fused path is width 128)", width);
    PSVO_REQUIRE(m >= 0 && n_split > 0, "mlp_bwd: bad sizes");
    hipStream_t st = as_stream(stream);
    int off[5], rows[5], cols[5], stride;
    dw_layout(off, rows, cols, &stride);
    float *ws = workspace;
    BwdOut o;
    o.a1 = ws; ws += m * 128;
    o.a2 = ws; ws += m * 128;
    o.a3 = ws; ws += m * 128;
    o.a4 = ws; ws += m * 128;
    o.d1 = ws; ws += m * 128;
    o.d2 = ws; ws += m * 128;
    o.d3 = ws; ws += m * 128;
    o.d4 = ws; ws += m * 128;
    o.d5 = ws; ws += m * 3;
    ws += m * 16;  // reserved
    float *slabs = ws;
    o.dfeat = dfeat;
    MlpParams p{w1, b1, w2, b2, w3, b3, w4, b4, w5, b5};
    if (m > 0) {
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_mlp_bwd_data),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBwd);
            attr = true;
        }
        hipLaunchKernelGGL(k_mlp_bwd_data, dim3(div_up(m, kTileBwd)), dim3(kThreadsBwd), kLdsBwd, st, m, feat, p,
                           g_sdf, g_rgb, o);
        int rc = check_launch("mlp_bwd_data");
        if (rc) return rc;
    }
    DwArgs a;
    a.slab_stride = stride;
    a.L[0] = DwLayer{o.d1, nullptr, 128, 128, feat, nullptr, 16, 16, 16, off[0]};
    a.L[1] = DwLayer{o.d2, nullptr, 128, 128, o.a1, nullptr, 128, 128, 128, off[1]};
    a.L[2] = DwLayer{o.d3, g_sdf, 128, 129, o.a2, nullptr, 128, 128, 128, off[2]};
    a.L[3] = DwLayer{o.d4, nullptr, 128, 128, o.a3, feat, 128, 128, 144, off[3]};
    a.L[4] = DwLayer{o.d5, nullptr, 3, 3, o.a4, nullptr, 128, 128, 128, off[4]};
    hipLaunchKernelGGL(k_mlp_dw, dim3(n_split, 5), dim3(256), 0, st, m, a, n_split, slabs);
    int rc = check_launch("mlp_dw");
    if (rc) return rc;
    DwDst d;
    float *gw[5] = {gw1, gw2, gw3, gw4, gw5}, *gb[5] = {gb1, gb2, gb3, gb4, gb5};
    for (int l = 0; l < 5; ++l) {
        d.w[l] = gw[l];
        d.b[l] = gb[l];
        d.off[l] = off[l];
        d.rows[l] = rows[l];
        d.cols[l] = cols[l];
    }
    hipLaunchKernelGGL(k_mlp_dw_reduce, dim3(div_up(stride, 256)), dim3(256), 0, st, n_split, stride, slabs, d,
                       accumulate);
    return check_launch("mlp_dw_reduce");
}
