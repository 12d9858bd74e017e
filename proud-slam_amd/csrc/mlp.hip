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

#include <cstdlib>

#include "interp_fuse.h"
#include "psvo_common.h"

#ifdef PSVO_STAMPS
__device__ unsigned long long psvo_g_stamps[3][256][8][8][16];  // diagnostic build only
#endif

namespace psvo {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kW = 128;     // decoder width
constexpr int kIn = 16;     // embedding dim
constexpr int kNB = kW / 32;

// LDS carve (floats): small vectors first, then the staged weight image.
constexpr int kOffB1 = 0, kOffB2 = kOffB1 + 128, kOffB3 = kOffB2 + 128, kOffB4 = kOffB3 + 132,
              kOffB5 = kOffB4 + 128;                  // biases b1 b2 b3[129] b4 b5[3]
constexpr int kOffW3r0 = kOffB5 + 4, kOffW5 = kOffW3r0 + 128;  // W3 row 0 (sdf), W5 [3][128]
constexpr int kOffW = kOffW5 + 3 * 128;               // = 1032 floats (16-B aligned)
constexpr int kImgFwd = 128 * 144;                    // largest forward image (W4)

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

// acc[ob] += image(`wl`: NOUT x NIN blocks) · in[kb].  Software-pipelined:
// the NOUT operand groups of step (kb, rg) + 1 are read from LDS before the
// 4·NOUT MFMAs of step (kb, rg) issue (ob innermost, independent
// accumulators), and scheduling barriers per step keep the compiler from
// pulling those reads back next to their first use — so the LDS latency
// hides behind a step of MFMAs instead of stalling every 4 of them.  `st`
// (St::kN stores per step) drains a pending store queue between the reads
// and the MFMAs of each step — spread over the GEMM instead of a burst that
// fills the TA command FIFO and stalls the wave.
struct NoStore {
    static constexpr int kN = 0;
    __device__ __forceinline__ void operator()(int, int) const {}
};

template <int NIN, int NOUT, typename St = NoStore>
__device__ __forceinline__ void gemm_acc(const float *wl, const f32x16 (&in)[NIN], f32x16 (&acc)[NOUT], int lane,
                                         const St &st = St()) {
    constexpr int kSteps = NIN * 4;
    auto opnd = [&](int step, int ob) {
        const int kb = step >> 2, rg = step & 3;
        return *reinterpret_cast<const float4 *>(wl + ((((ob * NIN + kb) * 4 + rg) * 64 + lane) << 2));
    };
    float4 cur[NOUT];
#pragma unroll
    for (int ob = 0; ob < NOUT; ++ob) cur[ob] = opnd(0, ob);
#pragma unroll
    for (int step = 0; step < kSteps; ++step) {
        const int kb = step >> 2, rg = step & 3;
        float4 nxt[NOUT];
        if (step + 1 < kSteps) {
#pragma unroll
            for (int ob = 0; ob < NOUT; ++ob) nxt[ob] = opnd(step + 1, ob);
        }
        st(kb, rg);
#pragma unroll
        for (int ob = 0; ob < NOUT; ++ob) acc[ob] = mfma(cur[ob].x, in[kb][4 * rg + 0], acc[ob]);
#pragma unroll
        for (int ob = 0; ob < NOUT; ++ob) acc[ob] = mfma(cur[ob].y, in[kb][4 * rg + 1], acc[ob]);
#pragma unroll
        for (int ob = 0; ob < NOUT; ++ob) acc[ob] = mfma(cur[ob].z, in[kb][4 * rg + 2], acc[ob]);
#pragma unroll
        for (int ob = 0; ob < NOUT; ++ob) acc[ob] = mfma(cur[ob].w, in[kb][4 * rg + 3], acc[ob]);
        if (step + 1 < kSteps) __builtin_amdgcn_sched_group_barrier(0x100, NOUT, 0);  // the next step's reads
        if (St::kN > 0) __builtin_amdgcn_sched_group_barrier(0x040, St::kN, 0);      // queued stores
        __builtin_amdgcn_sched_group_barrier(0x008, 4 * NOUT, 0);                     // this step's MFMAs
        __builtin_amdgcn_sched_barrier(0);
        if (step + 1 < kSteps) {
#pragma unroll
            for (int ob = 0; ob < NOUT; ++ob) cur[ob] = nxt[ob];
        }
    }
}

// acc[ob] += image(perm_x) · x  (x[t] = x feature 2t + h).  `st` (a store
// queue of 16 slots, e.g. CfQueue: one 16-KB CF tile) drains 2 slots per k
// sub-step, between that sub-step's 4 MFMAs.
template <typename St = NoStore>
__device__ __forceinline__ void gemm_x(const float *wl, const float (&x)[8], f32x16 (&acc)[kNB], int lane,
                                       const St &st = St()) {
#pragma unroll
    for (int tg = 0; tg < 2; ++tg) {
        float4 a[kNB];
#pragma unroll
        for (int ob = 0; ob < kNB; ++ob) a[ob] = *reinterpret_cast<const float4 *>(wl + (((ob * 2 + tg) * 64 + lane) << 2));
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (St::kN > 0) {
                const int q = 2 * (4 * tg + c);
                st(q >> 2, q & 3);
                st((q + 1) >> 2, (q + 1) & 3);
            }
#pragma unroll
            for (int ob = 0; ob < kNB; ++ob) acc[ob] = mfma(a[ob][c], x[4 * tg + c], acc[ob]);
            if (St::kN > 0) {
                __builtin_amdgcn_sched_group_barrier(0x040, 2 * St::kN, 0);  // the queued stores
                __builtin_amdgcn_sched_group_barrier(0x008, kNB, 0);         // then this sub-step's MFMAs
                __builtin_amdgcn_sched_barrier(0);
            }
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

// ReLU in place; returns the (value > 0) mask, bit 16b + r.  No compares:
// y = max(v, 0), and t = (−u) & ~u (u = bits of y) has its sign bit set
// exactly for positive non-zero patterns (±0 clear), so no per-element
// compare results pile up in SGPR pairs (the compare form spilled ~300 SGPRs).
__device__ __forceinline__ uint64_t relu(f32x16 (&v)[kNB]) {
    uint32_t half[2] = {0u, 0u};
#pragma unroll
    for (int b = 0; b < kNB; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            // pinned in program order: the scheduler would otherwise hoist all
            // 64 element computations and keep them live at once
            float y = v[b][r];
            asm volatile("" : "+v"(y));
            y = fmaxf(y, 0.0f);
            v[b][r] = y;
            const uint32_t u = __float_as_uint(y);
            const uint32_t t = (0u - u) & ~u;
            half[b >> 1] |= (t >> 31) << (16 * (b & 1) + r);
            asm volatile("" : "+v"(half[b >> 1]));
        }
    return (uint64_t)half[0] | ((uint64_t)half[1] << 32);
}

__device__ __forceinline__ void apply_mask(f32x16 (&v)[kNB], uint64_t m) {
    const uint32_t half[2] = {(uint32_t)m, (uint32_t)(m >> 32)};
#pragma unroll
    for (int b = 0; b < kNB; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t keep = 0u - ((half[b >> 1] >> (16 * (b & 1) + r)) & 1u);
            v[b][r] = __uint_as_float(__float_as_uint(v[b][r]) & keep);
        }
}

// Σ_k w[k] · v[k][sample] over this lane's 64 features (other half via partner lane)
// (roundings spelled out — an fmaf chain and one add — so every kernel that
// uses it, e.g. the sdf-only and the training forward, gives the same bits
// whatever the compiler would contract around it)
__device__ __forceinline__ float row_dot(const float *w, const f32x16 (&v)[kNB], int h) {
    float s = 0.f;
#pragma unroll
    for (int b = 0; b < kNB; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) s = fmaf(w[32 * b + phi(r, h)], v[b][r], s);
    return __fadd_rn(s, __shfl_xor(s, 32, 64));
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

// load_rows' inverse: row `row` of a row-major [·][128] matrix into
// accumulator form (zeros when !valid)
__device__ __forceinline__ void load_rows(const float *__restrict__ src, int64_t row, bool valid, f32x16 (&v)[kNB],
                                          int h) {
    const float *p = src + (valid ? row : 0) * kW;
#pragma unroll
    for (int b = 0; b < kNB; ++b)
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) {
            float4 q = *reinterpret_cast<const float4 *>(p + 32 * b + 8 * rg + 4 * h);
            if (!valid) q = make_float4(0.f, 0.f, 0.f, 0.f);
            v[b][4 * rg] = q.x;
            v[b][4 * rg + 1] = q.y;
            v[b][4 * rg + 2] = q.z;
            v[b][4 * rg + 3] = q.w;
        }
}

// Activations and δ's the weight gradients consume are stored TILE-FEATURE
// major ("CF"): per 32-sample tile a [128 feature][32 slot] block (16 KB) in
// which tile-local sample c sits at position p = (c&1)·16 + c/2 (the two
// samples of one f32 MFMA k-step pair, 2t and 2t+1, at t and 16 + t) and the
// 8 16-B groups of a row are XOR-swizzled by feature (slot = g ^ (f/2)%8: any
// 16 consecutive rows then cover all 64 banks once per 16-B column).  That
// is exactly the weight-gradient kernel's LDS operand image (conflict-free
// 4-k-step ds_read_b128), so a tile lands there by straight 1-KB
// global_load_lds copies.  The producing wave writes its 32-sample tile
// register by register with buffer stores: each covers two 64-B runs of two
// feature rows.
constexpr int kCh = 64;                 // allocation granule: CF buffers hold whole 64-sample pairs of tiles
constexpr int kTileS = 32;              // samples per CF tile
constexpr int kCfTile = 128 * kTileS;   // floats per CF tile
constexpr int64_t kMaxSamples = (int64_t)131071 * kTileS;  // one CF matrix < 2 GiB (buffer offsets)

__device__ __forceinline__ int cf_row_slot(int row, int g) { return row * kTileS + ((g ^ ((row >> 1) & 7)) << 2); }

// Element (b, r) of a wave's accumulator tile lands at byte
//   tile·16384 + f·128 + 4·((((p>>2) ^ X) << 2) | (p&3)),  f = 32b + phi(r, h)
// with X = (f/2)%8 = 4((r>>2)&1) + 2h + ((r>>1)&1): per lane 4 XOR variants
// voff[((r>>1)&1) + 2((r>>2)&1)] (tile and 512h folded in) and a
// wave-uniform rest 4096b + 1024(r>>2) + 128(r&3) (soffset).
struct CfStore {
    int voff[4];
    bool ok;
    __device__ CfStore(int64_t tile, int lane, int64_t n_tiles) {
        ok = tile < n_tiles;
        const int c = lane & 31;
        const int p = (c & 1) * 16 + (c >> 1);
        const int hh = lane >> 5;
        const int base = (int)(tile * kCfTile * 4) + 512 * hh;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int xr = 4 * (v >> 1) + 2 * hh + (v & 1);
            voff[v] = base + 4 * ((((p >> 2) ^ xr) << 2) | (p & 3));
        }
    }
    __device__ __forceinline__ void store(const float *matrix, int64_t bytes, const f32x16 (&v)[kNB]) const {
        if (!ok) return;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(matrix), 0, (int)bytes, 0x00020000);
#pragma unroll
        for (int b = 0; b < kNB; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[b][r]), rs, voff[((r >> 1) & 1) + 2 * ((r >> 2) & 1)],
                                                      4096 * b + 1024 * (r >> 2) + 128 * (r & 3), 0);
    }
};

// Pending-store queue for gemm_acc: the tile `v` (the GEMM's input) into a CF
// matrix, 4 registers per GEMM step.  A disabled queue (or a tile past the
// allocation) gets an empty buffer range, so the hardware drops its stores
// without a branch in the MFMA stream.
struct CfQueue {
    static constexpr int kN = 4;
    const CfStore &c;
    const f32x16 (&v)[kNB];
    __amdgpu_buffer_rsrc_t rs;
    __device__ CfQueue(const CfStore &cs, const float *matrix, int64_t bytes, bool on, const f32x16 (&vv)[kNB])
        : c(cs), v(vv),
          rs(__builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(matrix), 0,
                                               __builtin_amdgcn_readfirstlane((on && cs.ok) ? (int)bytes : 0),
                                               0x00020000)) {}
    __device__ __forceinline__ void operator()(int kb, int rg) const {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r = 4 * rg + j;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[kb][r]), rs, c.voff[((r >> 1) & 1) + 2 * ((r >> 2) & 1)],
                                                  4096 * kb + 1024 * (r >> 2) + 128 * (r & 3), 0);
        }
    }
};

// ---------------------------------------------------------------------------
// Weight images: every layer's LDS operand image, laid out exactly as the
// kernels read it, built once per weight update by k_mlp_prep (a gather,
// coalesced writes) so that staging is a straight 16-B copy.
//   fwd: W1 (perm_x), W2, W3 rows 1..128 (perm_acc), W4 ([f | x])
//   bwd (k_mlp_bwd3's chain): W4ᵀ, W3[1:]ᵀ, W2ᵀ, W1ᵀ as 16 × 16 blocks
constexpr int kImgF1 = 0, kImgF2 = kImgF1 + 2048, kImgF3 = kImgF2 + 16384, kImgF4 = kImgF3 + 16384,
              kImgVec = kImgF4 + 18432,   // the small vectors in their LDS layout (kOffB1..kOffW), padded
              kVecPad = 1280,             // to whole 1-KB glds pieces
              // k_mlp_bwd3's chain (v_mfma_f32_16x16x4_f32, 16-sample units): Wᵀ as 16 × 16
              // blocks (ob, kb), lane (m, q) holding Wᵀ[16ob + m][16kb + 4q .. 4q + 3]
              kImgC4 = kImgVec + kVecPad,   // W4ᵀ: 9 × 8 blocks (144 rows: f and x)
              kImgC3 = kImgC4 + 9 * 8 * 256,  // W3[1:]ᵀ
              kImgC2 = kImgC3 + 8 * 8 * 256,  // W2ᵀ
              kImgC1 = kImgC2 + 8 * 8 * 256,  // W1ᵀ: 1 × 8 blocks
              // the trunk kernel's forward in the same chain layout (W, not Wᵀ):
              // lane (m, q) holding W[16ob + m][16kb + 4q .. 4q + 3]
              kImgT1 = kImgC1 + 8 * 256,    // W1: 8 × 1 blocks
              kImgT2 = kImgT1 + 8 * 256,    // W2: 8 × 8 blocks
              kImgTotal = kImgT2 + 8 * 8 * 256;  // 126,208 floats

__device__ __forceinline__ void inv_perm_acc(int pos, int nkb, int &i, int &k) {
    const int c = pos & 3, lane = (pos >> 2) & 63, rest = pos >> 8;
    const int rg = rest & 3, blk = rest >> 2;
    const int kb = blk % nkb, ib = blk / nkb;
    const int h = lane >> 5;
    i = ib * 32 + (lane & 31);
    k = kb * 32 + c + 4 * h + 8 * rg;
}
__device__ __forceinline__ void inv_perm_x(int pos, int &i, int &k) {
    const int c = pos & 3, lane = (pos >> 2) & 63, rest = pos >> 8;
    const int tg = rest & 1, ib = rest >> 1;
    i = ib * 32 + (lane & 31);
    k = 2 * (tg * 4 + c) + (lane >> 5);
}

struct MlpParams {
    const float *w1, *b1, *w2, *b2, *w3, *b3, *w4, *b4, *w5, *b5;
};

// element e (< kVecPad) of the vector image = LDS float e of stage_vectors' carve
__device__ __forceinline__ float vec_elem(const MlpParams &p, int e) {
    if (e < kOffB2) return p.b1[e - kOffB1];
    if (e < kOffB3) return p.b2[e - kOffB2];
    if (e < kOffB4) return e - kOffB3 < 129 ? p.b3[e - kOffB3] : 0.0f;
    if (e < kOffB5) return p.b4[e - kOffB4];
    if (e < kOffW3r0) return e - kOffB5 < 3 ? p.b5[e - kOffB5] : 0.0f;
    if (e < kOffW5) return p.w3[e - kOffW3r0];
    if (e < kOffW) return p.w5[e - kOffW5];
    return 0.0f;
}

__global__ __launch_bounds__(256) void k_mlp_prep(MlpParams p, float *__restrict__ img) {
    const float *w1 = p.w1, *w2 = p.w2, *w3 = p.w3, *w4 = p.w4;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kImgTotal) return;
    int i, k;
    float v = 0.0f;
    if (e >= kImgT1) {  // the trunk kernel's forward images: W[o][in], [ob][kb][lane (m, q)][4]
        const bool t1 = e < kImgT2;
        const int pos = e - (t1 ? kImgT1 : kImgT2);
        const int j = pos & 3, ln = (pos >> 2) & 63, blk = pos >> 8;
        const int nkb = t1 ? 1 : 8;
        const int o = 16 * (blk / nkb) + (ln & 15), in = 16 * (blk % nkb) + 4 * (ln >> 4) + j;
        img[e] = t1 ? p.w1[o * 16 + in] : w2[o * 128 + in];
        return;
    }
    if (e >= kImgC4) {  // chain16 images: [ob][kb][lane (m, q)][4]
        const int sec = e < kImgC3 ? 4 : e < kImgC2 ? 3 : e < kImgC1 ? 2 : 1;
        const int pos = e - (sec == 4 ? kImgC4 : sec == 3 ? kImgC3 : sec == 2 ? kImgC2 : kImgC1);
        const int j = pos & 3, ln = (pos >> 2) & 63, blk = pos >> 8;
        const int o = 16 * (blk >> 3) + (ln & 15), in = 16 * (blk & 7) + 4 * (ln >> 4) + j;  // Wᵀ[o][in]
        img[e] = sec == 4 ? w4[in * 144 + o] : sec == 3 ? w3[(1 + in) * 128 + o] : sec == 2 ? w2[in * 128 + o]
                                                                                             : p.w1[in * 16 + o];
        return;
    }
    if (e >= kImgVec) {
        img[e] = vec_elem(p, e - kImgVec);
        return;
    }
    if (e < kImgF2) {
        inv_perm_x(e - kImgF1, i, k);
        v = w1[i * 16 + k];
    } else if (e < kImgF3) {
        inv_perm_acc(e - kImgF2, 4, i, k);
        v = w2[i * 128 + k];
    } else if (e < kImgF4) {
        inv_perm_acc(e - kImgF3, 4, i, k);
        v = w3[(i + 1) * 128 + k];
    } else {
        const int pos = e - kImgF4;
        if (pos < 16384) {
            inv_perm_acc(pos, 4, i, k);
            v = w4[i * 144 + k];
        } else {
            inv_perm_x(pos - 16384, i, k);
            v = w4[i * 144 + 128 + k];
        }
    }
    img[e] = v;
}

// Barrier for LDS hazards only: waits for this wave's LDS operations, not for
// its global stores (__syncthreads' fence would also drain every outstanding
// activation store and glds before each layer).
__device__ __forceinline__ void raw_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS ops done (vmcnt left as is)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ float sigmoidf(float x) { return 1.0f / (1.0f + expf(-x)); }

__device__ __forceinline__ void load_x(const float *__restrict__ feat, int64_t s, bool valid, int h, float (&x)[8]) {
    const float *fr = feat + (valid ? s : 0) * kIn;
#pragma unroll
    for (int t = 0; t < 8; ++t) x[t] = valid ? fr[2 * t + h] : 0.0f;
}

// global → LDS copies (global_load_lds_*): LDS destination = wave-uniform
// base (M0) + lane × size.  Issued through inline asm so that the compiler's
// wait insertion does not treat them as LDS writes aliasing every ds_read
// (it would drain the prefetch with vmcnt(0) before each operand read); the
// kernel counts them itself (wait_vm).
__device__ __forceinline__ uint32_t lds_addr(const float *l) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float *)l;
}
__device__ __forceinline__ void glds16(const float *g, float *l) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds_addr(l)))
                 : "memory");
}

// streaming (nt) store of one float at base[i]: the slabs are read once, by
// the reduce kernel (a kernel boundary also pays ≈ dirty bytes ÷ 6 TB/s for
// what stays dirty in L2; measured: nt slab stores 0.99 -> 0.985 ms per BA
// iteration, write-through (sc1) ones no gain)
__device__ __forceinline__ void store_nt(float *base, int i, float v) { __builtin_nontemporal_store(v, base + i); }

// write C blocks to the slab (rows offset `row_off` in the layer's matrix)
template <int NR, int NC, bool NT = false>
__device__ __forceinline__ void dw_store(float *slab, int cols, int row_off, int max_col, const int (&rb)[NR],
                                         const int (&cb)[NC], const f32x16 (&acc)[NR][NC], int lane) {
    const int x = lane & 31, h = lane >> 5;
#pragma unroll
    for (int i = 0; i < NR; ++i)
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            const int col = 32 * cb[j] + x;
            if (col >= max_col) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                if (NT) {
                    store_nt(slab, (row_off + 32 * rb[i] + phi(r, h)) * cols + col, acc[i][j][r]);
                } else {
                    slab[(row_off + 32 * rb[i] + phi(r, h)) * cols + col] = acc[i][j][r];
                }
            }
        }
}

// s_waitcnt vmcnt(n) for this wave's global_load_lds copies (the kernels count them)
__device__ __forceinline__ void wait_vm(int n) {
    // s_waitcnt vmcnt(n) only (expcnt / lgkmcnt at their maxima); n <= 63
    asm volatile("" ::: "memory");
    switch (n) {
        case 0: __builtin_amdgcn_s_waitcnt(0x0F70); break;
        case 1: __builtin_amdgcn_s_waitcnt(0x0F71); break;
        case 8: __builtin_amdgcn_s_waitcnt(0x0F78); break;
        case 9: __builtin_amdgcn_s_waitcnt(0x0F79); break;
        case 16: __builtin_amdgcn_s_waitcnt(0x4F70); break;
        case 17: __builtin_amdgcn_s_waitcnt(0x4F71); break;
        case 18: __builtin_amdgcn_s_waitcnt(0x4F72); break;
        default: __builtin_amdgcn_s_waitcnt(0x0F70); break;  // conservative: everything
    }
    asm volatile("" ::: "memory");
}


// L = 0: W1 (MFMA) and W5 (VALU) share a workgroup (both are light: one
// 32x32 block per wave / three row dots); L = 1..3: W2, W3, W4.
struct DwGrid {
    int wg_begin[5];  // prefix over workgroup types (0: W1+W5, 1: W2, 2: W3, 3: W4) of split counts
    int n_split[5];   // slabs per weight matrix (W5 has W1's)
    int slab_off[5];  // float offset of matrix l's first slab
    int slab_len[5];  // rows*cols + rows
};

struct DwDst {
    float *w[5], *b[5];
    int rows[5], cols[5];
    int elem_begin[6];
};

// slabs_b (or null): k_mlp_trunk_fb's slabs (the same layout), whose W1, W2, W3
// row 0 and b3[0] elements are added (the rest of its slabs is not written).
// A workgroup sums 64 elements: wave k over the k-th quarter of the slabs
// (batches of 8 independent loads, lane = element: 256-B rows), then the
// quarters in order — a fixed order, so deterministic.  (One thread per
// element over all 2 × 256 slabs left ≈ 150 workgroups on 256 CUs, each
// thread with up to 512 loads in flight one batch at a time: 132 µs.)
constexpr int kDwRedEl = 64;
__device__ __forceinline__ float dw_sum_range(const float *__restrict__ p, int64_t stride, int b, int e) {
    float v = 0.0f;
    int sp = b;
    for (; sp + 8 <= e; sp += 8) {
        float q[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) q[u] = p[(sp + u) * stride];
#pragma unroll
        for (int u = 0; u < 8; ++u) v += q[u];
    }
    for (; sp < e; ++sp) v += p[sp * stride];
    return v;
}
__global__ __launch_bounds__(256) void k_mlp_dw_reduce(DwGrid g, const float *__restrict__ slabs, DwDst dst,
                                                       int accumulate, const float *__restrict__ slabs_b) {
    __shared__ float part[4][kDwRedEl];
    const int lane = threadIdx.x & 63, k = threadIdx.x >> 6;
    const int e = blockIdx.x * kDwRedEl + lane;
    const bool in = e < dst.elem_begin[5];
    int L = 0;
#pragma unroll
    for (int l = 1; l < 5; ++l) L += (e >= dst.elem_begin[l]);
    const int rel = in ? e - dst.elem_begin[L] : 0;
    const int n_split = g.n_split[L];
    const int64_t stride = g.slab_len[L];
    const int b = n_split * k / 4, en = n_split * (k + 1) / 4;
    float v = 0.0f;
    if (in) {
        v = dw_sum_range(slabs + g.slab_off[L] + rel, stride, b, en);
        if (slabs_b && (L < 2 || (L == 2 && (rel < 128 || rel == 129 * 128))))
            v += dw_sum_range(slabs_b + g.slab_off[L] + rel, stride, b, en);
    }
    part[k][lane] = v;
    __syncthreads();
    if (k != 0 || !in) return;
    v = ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
    const int nw = dst.rows[L] * dst.cols[L];
    float *out = rel < nw ? dst.w[L] + rel : dst.b[L] + (rel - nw);
    *out = accumulate ? *out + v : v;
}

// Diagnostic build only (-DPSVO_STAMPS, `make stamps`: lib/diag/): per-wave
// s_memtime stamps at the layer boundaries of k_mlp_fwd2 / k_mlp_bwd2, read
// through psvo_debug_stamps.  In the product library every PSVO_STAMP is empty.
#ifdef PSVO_STAMPS
constexpr int kStampIters = 8, kStampWgs = 256;  // psvo_g_stamps[2][256][8][8][16]
#define PSVO_STAMP_DECL int stit_ = 0
#define PSVO_STAMP(i)                                                                               \
    do {                                                                                            \
        __builtin_amdgcn_sched_barrier(0);                                                          \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                 \
        __builtin_amdgcn_sched_barrier(0);                                                          \
        if ((threadIdx.x & 63) == 0 && stit_ < kStampIters && blockIdx.x < kStampWgs)               \
            psvo_g_stamps[kStampK][blockIdx.x][threadIdx.x >> 6][stit_][i] = t_;                         \
    } while (0)
#define PSVO_STAMP_FLUSH(k) ++stit_
#else
#define PSVO_STAMP_DECL
#define PSVO_STAMP(i)
#define PSVO_STAMP_FLUSH(k)
#endif

// ---- k_mlp_fwd2's W4 layer, one 32-row output block at a time ----------
// Block OB's MFMAs carry the CF stores of f (its block OB, the layer input)
// and of c1 block OB-1 (finished, ReLU'd) — one store each per k-step — so
// the c1 tile no longer leaves in one 64-store burst that, issued by every
// wave of the chip at once, stalled the epilogue on HBM write drain; block
// OB's ReLU and mask bits run under block OB+1's MFMAs.  Per accumulator the
// MFMA order is unchanged: the same bits.
template <int OB>
struct L4Queue {
    static constexpr int kN = OB > 0 ? 2 : 1;
    const CfStore &c;
    const f32x16 (&f)[kNB];
    const f32x16 (&c1)[kNB];
    __amdgpu_buffer_rsrc_t rf, rc;
    __device__ L4Queue(const CfStore &cs, const float *fm, const float *cm, int64_t bytes, bool on,
                       const f32x16 (&ff)[kNB], const f32x16 (&cc)[kNB])
        : c(cs), f(ff), c1(cc),
          rf(__builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(fm), 0,
                                               __builtin_amdgcn_readfirstlane((on && cs.ok) ? (int)bytes : 0),
                                               0x00020000)),
          rc(__builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(cm), 0,
                                               __builtin_amdgcn_readfirstlane((on && cs.ok) ? (int)bytes : 0),
                                               0x00020000)) {}
    __device__ __forceinline__ void operator()(int kb, int rg) const {
        const int r = 4 * kb + rg;
        const int vo = c.voff[((r >> 1) & 1) + 2 * ((r >> 2) & 1)];
        const int so = 1024 * (r >> 2) + 128 * (r & 3);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(f[OB][r]), rf, vo, 4096 * OB + so, 0);
        if (OB > 0)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(c1[OB - 1][r]), rc, vo, 4096 * (OB - 1) + so, 0);
    }
};

// relu() restricted to block OB (same per-element sequence and mask bits)
template <int OB>
__device__ __forceinline__ void relu_block(f32x16 &v, uint32_t (&half)[2]) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        float y = v[r];
        asm volatile("" : "+v"(y));
        y = fmaxf(y, 0.0f);
        v[r] = y;
        const uint32_t u = __float_as_uint(y);
        const uint32_t t = (0u - u) & ~u;
        half[OB >> 1] |= (t >> 31) << (16 * (OB & 1) + r);
        asm volatile("" : "+v"(half[OB >> 1]));
    }
}

// bacc[OB] += W4 block OB · [f; x] (bias already in bacc), then its ReLU and
// mask bits (the rgb head's dots wait for all four blocks: until then f is
// live as the layer input and the registers are spoken for)
template <int OB>
__device__ __forceinline__ void l4_block(const float *wl, const f32x16 (&a)[kNB], const float (&x)[8],
                                         f32x16 (&bacc)[kNB], int lane, const L4Queue<OB> &q,
                                         uint32_t (&half)[2]) {
    f32x16 (&acc)[1] = *reinterpret_cast<f32x16(*)[1]>(&bacc[OB]);
    gemm_acc<kNB, 1>(wl + OB * kNB * 4 * 64 * 4, a, acc, lane, q);
    const float *wx = wl + kNB * kNB * 16 * 64;
#pragma unroll
    for (int tg = 0; tg < 2; ++tg) {
        const float4 w4 = *reinterpret_cast<const float4 *>(wx + (((OB * 2 + tg) * 64 + lane) << 2));
        acc[0] = mfma(w4.x, x[4 * tg + 0], acc[0]);
        acc[0] = mfma(w4.y, x[4 * tg + 1], acc[0]);
        acc[0] = mfma(w4.z, x[4 * tg + 2], acc[0]);
        acc[0] = mfma(w4.w, x[4 * tg + 3], acc[0]);
    }
    relu_block<OB>(bacc[OB], half);
}

// ---------------------------------------------------------------------------
// forward, persistent + double-buffered: one 512-thread workgroup per CU
// loops over 256-sample tiles (8 waves × 32 samples, the chain of k_mlp_fwd
// per wave).  The vectors and W1 stay resident in LDS; W2, W3, W4 stream
// through two 72-KB buffers with global_load_lds issued one layer ahead
// (W2 of the next tile during W4 of this one), so no wave waits for weight
// staging; each layer's activation stores are issued after the barrier that
// opens the next layer and drain behind its MFMAs.  LDS: 5 + 8 + 2 × 72 KB.
constexpr int kF2Waves = 8, kF2Threads = kF2Waves * 64, kF2Tile = kF2Waves * 32;
constexpr int kF2W1 = kVecPad, kF2Buf0 = kF2W1 + 2048, kF2Buf1 = kF2Buf0 + kImgFwd;
constexpr int kLdsFwd2 = (kF2Buf1 + kImgFwd) * 4;  // 160,768 B
static_assert(kLdsFwd2 <= 160 * 1024, "fwd2 LDS budget");
static_assert(kOffW <= kVecPad, "vector image");

__device__ __forceinline__ void stage8(float *dst, const float *img, int n_floats, int wave, int lane) {
    for (int c = wave; c < n_floats / 256; c += kF2Waves) glds16(img + (c * 64 + lane) * 4, dst + c * 256);
}

template <bool H2>
__global__ __launch_bounds__(kF2Threads, 1) void k_mlp_fwd2(int64_t m, const float *__restrict__ feat,
                                                            const float *__restrict__ img,
                                                            float *__restrict__ sdf_out, float *__restrict__ rgb_out,
                                                            float *__restrict__ act, uint64_t *__restrict__ masks,
                                                            const int *__restrict__ m_dev,
                                                            const float *__restrict__ h2_rows,
                                                            const int *__restrict__ h2_src) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    if (m_dev) m = __builtin_amdgcn_readfirstlane(*m_dev);  // the sparse decoder's kept samples (<= m)
    // h2_rows: h2 of every sample of the step (k_mlp_sdf2's, the same
    // instructions: the same bits), sample s's row h2_src[s] — the W2 layer
    // is read instead of recomputed (W3 / W4 stream through the buffers)
    constexpr bool h2_given = H2;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5;
    const bool save = act != nullptr;         // CF activations (weight gradients)
    const bool save_mask = masks != nullptr;  // ReLU masks (δ chain)
    const int64_t n_tiles = (m + kCh - 1) / kCh * 2;  // CF 32-sample tiles
    const int64_t tstride = n_tiles * 32 * 128;
    const int64_t tbytes = tstride * 4;
    // Balanced split: workgroup b owns the 32-sample units [u0, u1), so every
    // wave slot gets floor or ceil of n_units / (8 · grid) and the last
    // iteration is a partial one (waves past u1 skip their MFMAs but keep the
    // staging and barriers) instead of a whole extra 256-sample round on a
    // few CUs while the rest of the chip waits at the kernel boundary.
    const int64_t n_units = (m + kTileS - 1) / kTileS;
    const int64_t u0 = n_units * blockIdx.x / gridDim.x, u1 = n_units * (blockIdx.x + 1) / gridDim.x;
    const int n_it = (int)((u1 - u0 + kF2Waves - 1) / kF2Waves);
    auto buf = [&](int i) { return lds + ((i & 1) ? kF2Buf1 : kF2Buf0); };
    int seq = 0;  // staged layers so far: W(seq) sits in buf(seq)
    float xn[8];
    int srcn = 0;
    {
        const int64_t u = u0 + wave;
        const int64_t s = u * kTileS + (lane & 31);
        if (h2_given && u < u1 && s < m) srcn = h2_src[s];
        load_x(feat, h2_given ? (int64_t)srcn : s, u < u1 && s < m, h, xn);  // (h2 given: feat is the step's rows)
    }
    stage8(lds, img + kImgVec, kVecPad, wave, lane);
    stage8(lds + kF2W1, img + kImgF1, 2048, wave, lane);
    stage8(buf(0), img + (h2_given ? kImgF3 : kImgF2), 16384, wave, lane);
    wait_vm(0);
    raw_barrier();
    [[maybe_unused]] constexpr int kStampK = 0;
    PSVO_STAMP_DECL;
    for (int it = 0; it < n_it; ++it) {
        if (!H2) PSVO_STAMP(0);  // (the h2-reading instantiation: no stamps — the diagnostic build hit a backend error there)
        const int64_t u = u0 + (int64_t)it * kF2Waves + wave;
        const bool active = u < u1;  // wave-uniform
        const int64_t s = u * kTileS + (lane & 31);
        const bool valid = active && s < m;
        const bool more = it + 1 < n_it;
        float x[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = xn[i];
        const int src = srcn;
        const CfStore cfs(u, lane, n_tiles);
        f32x16 a[kNB], bacc[kNB];
        uint64_t m1 = 0, m2 = 0;
        float sdf = 0.f;
        // h2 read (its row of the step's h2): in flight under the W1 layer
        if (h2_given && active) load_rows(h2_rows, src, valid, bacc, h);
        // h1 = relu(W1 x + b1): resident W1
        if (active) {
            init_bias(a, lds + kOffB1, h);
            gemm_x(lds + kF2W1, x, a, lane);
            m1 = relu(a);
        }
        if (h2_given) {  // h1's stores; h2's mask
            if (active) {
                if (save) cfs.store(act, tbytes, a);
                m2 = relu(bacc);  // post-ReLU values: the same values and mask bits
            }
        } else {
            // h2 = relu(W2 h1 + b2)
            wait_vm(0);
            raw_barrier();
            stage8(buf(seq + 1), img + kImgF3, 16384, wave, lane);
            if (active) {
                init_bias(bacc, lds + kOffB2, h);
                gemm_acc<kNB, kNB>(buf(seq), a, bacc, lane, CfQueue(cfs, act, tbytes, save, a));  // + h1 stores
                m2 = relu(bacc);
            }
            ++seq;
        }
        // [sdf | f] = W3 h2 + b3
        wait_vm(0);
        raw_barrier();
        stage8(buf(seq + 1), img + kImgF4, 18432, wave, lane);
        if (active) {
            sdf = __fadd_rn(lds[kOffB3], row_dot(lds + kOffW3r0, bacc, h));
            init_bias(a, lds + kOffB3 + 1, h);
            gemm_acc<kNB, kNB>(buf(seq), bacc, a, lane, CfQueue(cfs, act + tstride, tbytes, save, bacc));  // + h2
        }
        ++seq;
        // c1 = relu(W4 [f; x] + b4); the next tile's W2 and x start loading
        wait_vm(0);
        raw_barrier();
        if (more) {
            stage8(buf(seq + 1), img + (h2_given ? kImgF3 : kImgF2), 16384, wave, lane);
            const int64_t un = u + kF2Waves;
            const int64_t sn = un * kTileS + (lane & 31);
            if (h2_given && un < u1 && sn < m) srcn = h2_src[sn];
            load_x(feat, h2_given ? (int64_t)srcn : sn, un < u1 && sn < m, h, xn);
        }
        if (!active) {
            ++seq;
            if (!H2) PSVO_STAMP(8);
            PSVO_STAMP_FLUSH(0);
            continue;
        }
        init_bias(bacc, lds + kOffB4, h);
        uint32_t half4[2] = {0u, 0u};
        {
            const float *wl4 = buf(seq);
            const float *fm = act + 2 * tstride, *cm = act + 3 * tstride;
            l4_block<0>(wl4, a, x, bacc, lane, L4Queue<0>(cfs, fm, cm, tbytes, save, a, bacc), half4);
            l4_block<1>(wl4, a, x, bacc, lane, L4Queue<1>(cfs, fm, cm, tbytes, save, a, bacc), half4);
            l4_block<2>(wl4, a, x, bacc, lane, L4Queue<2>(cfs, fm, cm, tbytes, save, a, bacc), half4);
            l4_block<3>(wl4, a, x, bacc, lane, L4Queue<3>(cfs, fm, cm, tbytes, save, a, bacc), half4);
            if (save && cfs.ok) {  // c1 block 3
                const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
                    const_cast<float *>(cm), 0, __builtin_amdgcn_readfirstlane((int)tbytes), 0x00020000);
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(bacc[3][r]), rc,
                                                          cfs.voff[((r >> 1) & 1) + 2 * ((r >> 2) & 1)],
                                                          4096 * 3 + 1024 * (r >> 2) + 128 * (r & 3), 0);
            }
        }
        ++seq;
        const uint64_t m4 = (uint64_t)half4[0] | ((uint64_t)half4[1] << 32);
        if (save_mask && valid) {
            uint64_t *mk = masks + (s * 2 + h) * 3;
            mk[0] = m1;
            mk[1] = m2;
            mk[2] = m4;
        }
        float rgb[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) rgb[c] = sigmoidf(lds[kOffB5 + c] + row_dot(lds + kOffW5 + 128 * c, bacc, h));
        if (valid && h == 0) {
            sdf_out[s] = sdf;
            rgb_out[s * 3 + 0] = rgb[0];
            rgb_out[s * 3 + 1] = rgb[1];
            rgb_out[s * 3 + 2] = rgb[2];
        }
        if (!H2) PSVO_STAMP(8);
        PSVO_STAMP_FLUSH(0);
    }
    wait_vm(0);
}

// sdf only (Decoder.get_sdf; mesh lattices): h1, h2 and the sdf row of W3 —
// 18.3 of the 53.7 k MACs per sample.  W1 and W2 stay resident (77 KB of
// LDS, no staging in the loop); the same instruction sequence as
// k_mlp_fwd2's first two layers, so the sdf is bit-identical to its output.
constexpr int kLdsSdf2 = (kF2Buf0 + 16384) * 4;

__global__ __launch_bounds__(kF2Threads, 1) void k_mlp_sdf2(int64_t m_host, const float *__restrict__ feat,
                                                            const float *__restrict__ img,
                                                            float *__restrict__ sdf_out, const int *__restrict__ m_dev,
                                                            float *__restrict__ h2_out) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    // m_dev: the count on the device, m_host the buffers' capacity (a larger
    // batch: nothing here, the host-sized launch after the read-back)
    int64_t m = m_dev ? (int64_t)__builtin_amdgcn_readfirstlane(*m_dev) : m_host;
    if (m > m_host) m = 0;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int h = lane >> 5;
    float *w2 = lds + kF2Buf0;
    // the balanced split of k_mlp_fwd2: workgroup b owns the
    // 32-sample tiles [u0, u1), wave w the tiles u0 + w, u0 + w + 8, …
    const int64_t n_units = (m + kTileS - 1) / kTileS;
    const int64_t u0 = n_units * blockIdx.x / gridDim.x, u1 = n_units * (blockIdx.x + 1) / gridDim.x;
    float xn[8];
    {
        const int64_t s = (u0 + wave) * kTileS + (lane & 31);
        load_x(feat, s, u0 + wave < u1 && s < m, h, xn);
    }
    stage8(lds, img + kImgVec, kVecPad, wave, lane);
    stage8(lds + kF2W1, img + kImgF1, 2048, wave, lane);
    stage8(w2, img + kImgF2, 16384, wave, lane);
    wait_vm(0);
    raw_barrier();
    for (int64_t u = u0 + wave; u < u1; u += kF2Waves) {  // no barriers below
        const int64_t s = u * kTileS + (lane & 31);
        const bool valid = s < m;
        float x[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = xn[i];
        if (u + kF2Waves < u1) {
            const int64_t sn = (u + kF2Waves) * kTileS + (lane & 31);
            load_x(feat, sn, sn < m, h, xn);
        }
        f32x16 a[kNB], bacc[kNB];
        init_bias(a, lds + kOffB1, h);
        gemm_x(lds + kF2W1, x, a, lane);
        (void)relu(a);
        init_bias(bacc, lds + kOffB2, h);
        gemm_acc<kNB, kNB>(w2, a, bacc, lane);
        (void)relu(bacc);
        const float sdf = __fadd_rn(lds[kOffB3], row_dot(lds + kOffW3r0, bacc, h));
        if (valid && h == 0) sdf_out[s] = sdf;
        if (h2_out) store_rows(h2_out, s, valid, kW, bacc, h);  // (the sparse decoder's later layers read it)
    }
    wait_vm(0);
}

// ---------------------------------------------------------------------------
// Fused backward: the δ chain AND the weight gradients in one persistent
// kernel, the δ's handed from the chain to the weight-gradient MFMAs through
// LDS instead of HBM (k_mlp_bwd2 + k_mlp_dw2 move 2 KB/sample of δ's out and
// back: ≈ 1.1 GB per step at config B).
//
// The chain needs features on the MFMA reduction axis (accumulator = next B
// operand, lane = sample); a weight gradient Σ_s δ[o][s] a[i][s] needs the
// samples there (lane = feature).  So every δ crosses lanes once: the chain
// wave writes its δ tile into LDS and the gradient MFMAs read it back
// transposed.  The chain runs v_mfma_f32_16x16x4_f32 on 16-sample units
// (an activation is 8 blocks × 4 = 32 registers, half of the 32-sample
// 32x32x2 form's 64 — the register file has to hold the weight-gradient
// accumulators too), lane (n, q) holding features 16·ob + 4q + j of sample n
// (j = register); its weights stream from L2 as MFMA A operands (Wᵀ images
// kImgC4..kImgC1, every CU reads the same 213 KB).
//
// One 8-wave workgroup per CU loops over rounds of four 16-sample units.
// Waves 0-3 (one per SIMD) run the chain of one unit each and own the
// gradients whose other operand is x or c1: W1 and the x columns of W4 (row
// block = wave), W5 (column block = wave); waves 4-7 (one per SIMD) own
// column block d = wave − 4 of W2, W3 and W4 (4 row blocks each, 192
// accumulator registers) and the biases of row block d.  A round is four
// phases separated by one barrier; a phase's exports are read in the next:
//   phase  chain wave c (unit u0 + 4r + c)                       gradient waves (the round's 4 units)
//   P0     δ5, δc1, x → LDS; δ[f; x] = W4ᵀ δc1; dW1 += δh1(r−1) ⊗ x
//   P1     δf, δsdf → LDS; δh2 = (W3ᵀ [δsdf; δf]) ⊙ m2;          dW4 += δc1 ⊗ f
//          dW4x += δc1 ⊗ x
//   P2     δh2 → LDS; δh1 = W2ᵀ δh2 ⊙ m1; dW5 += δ5 ⊗ c1         dW3 += [δsdf; δf] ⊗ h2
//   P3     δh1 → LDS; dfeat = W1ᵀ δh1 + δx_c (+ interp bwd)       dW2 += δh2 ⊗ h1
// plus a last P0 for the final round's dW1.  Per accumulator the MFMA
// order is fixed (rounds, units, k-steps in order): deterministic.  Each
// workgroup writes one slab of every layer; k_mlp_dw_reduce sums them.
//
// LDS image of a unit's δ (and of its x): 128 (16) rows × 16 slots, sample
// n at slot 8(n&1) + n/2 (k-step t of the 32x32x2 gradient MFMA takes
// samples 2t, 2t+1 — the CF tile's order), the four 16-B chunks of row r
// XOR-permuted by (r >> 2) & 3: the chain's ds_write_b32 (4 rows × 16
// slots) are at most 2-way, the gradient waves' ds_read_b128 (32 rows ×
// one chunk) conflict-free.
constexpr int kU = 16;                                  // samples per chain unit
constexpr int kUImg = 128 * kU;                         // a unit's δ image (8 KB)
constexpr int kB3Slot = kVecPad;                        // δ images [set 2][unit 4]
constexpr int kB3Small = kB3Slot + 2 * 4 * kUImg;       // per-sample rows [set 2][unit 4][4][16]: δ5 / δsdf
constexpr int kB3X = kB3Small + 2 * 4 * 4 * kU;         // x images [round parity 2][unit 4][16 × 16]
constexpr int kB3I = kB3X + 2 * 4 * 16 * kU;            // interpolation backward scatter staging [chain wave 4][512]
constexpr int kB3A = kB3I + 4 * 512;                    // chain accumulators dW1 / dW4x [chain wave 4][2][4][lane 64][4]
constexpr int kB3W5 = kB3A + 4 * 2 * 1024;              // gradient waves' dW5 / b5 partials [wave 4][lane 64][8]
constexpr int kLdsBwd3 = (kB3W5 + 4 * 64 * 8) * 4;      // 130,048 B
static_assert(kLdsBwd3 <= 160 * 1024, "bwd3 LDS budget");

typedef float f32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4v mfma16(float a, float b, f32x4v c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// 16-B buffer load: descriptor in SGPRs, one 32-bit lane offset + a
// wave-uniform byte offset (no 64-bit per-lane address arithmetic)
__device__ __forceinline__ float4 bload4(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const float *p, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(p), 0, (int)bytes, 0x00020000);
}

// acc[ob] += Wᵀ blocks (ob, kb) of the image at float offset `img_off` · in[kb]
// (16 × 16 × 4 MFMAs; the A operands stream from L2 through a ring D k-blocks deep)
template <int NKB, int NOB, int D>
__device__ __forceinline__ void gemm16(__amdgpu_buffer_rsrc_t rs, int img_off, const f32x4v (&in)[NKB],
                                       f32x4v (&acc)[NOB], int lane) {
    auto ld = [&](int kb, int ob) { return bload4(rs, lane * 16, (img_off + (ob * NKB + kb) * 256) * 4); };
    float4 ring[D + 1][NOB];
#pragma unroll
    for (int s = 0; s < D; ++s)
#pragma unroll
        for (int ob = 0; ob < NOB; ++ob) ring[s][ob] = ld(s, ob);
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
        const int cs = kb % (D + 1);
        if (kb + D < NKB) {
#pragma unroll
            for (int ob = 0; ob < NOB; ++ob) ring[(kb + D) % (D + 1)][ob] = ld(kb + D, ob);
        }
#pragma unroll
        for (int ob = 0; ob < NOB; ++ob) acc[ob] = mfma16(ring[cs][ob].x, in[kb][0], acc[ob]);
#pragma unroll
        for (int ob = 0; ob < NOB; ++ob) acc[ob] = mfma16(ring[cs][ob].y, in[kb][1], acc[ob]);
#pragma unroll
        for (int ob = 0; ob < NOB; ++ob) acc[ob] = mfma16(ring[cs][ob].z, in[kb][2], acc[ob]);
#pragma unroll
        for (int ob = 0; ob < NOB; ++ob) acc[ob] = mfma16(ring[cs][ob].w, in[kb][3], acc[ob]);
        if (kb + D < NKB) __builtin_amdgcn_sched_group_barrier(0x020, NOB, 0);  // the prefetch
        __builtin_amdgcn_sched_group_barrier(0x008, 4 * NOB, 0);                // this block's MFMAs
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int N>
__device__ __forceinline__ void zero4(f32x4v (&v)[N]) {
#pragma unroll
    for (int b = 0; b < N; ++b) v[b] = f32x4v{0.f, 0.f, 0.f, 0.f};
}

// ReLU mask of a 128-feature activation: feature 16·ob + 4q + j is bit
// 8·ob + j of w (the forward's mask word of lane-half q & 1, shifted by 4·(q >> 1))
__device__ __forceinline__ void mask16(f32x4v (&v)[8], uint64_t w) {
#pragma unroll
    for (int ob = 0; ob < 8; ++ob)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t keep = 0u - (uint32_t)((w >> (8 * ob + j)) & 1u);
            v[ob][j] = __uint_as_float(__float_as_uint(v[ob][j]) & keep);
        }
}

// a chain wave's activation → its unit image (rows 16·ob + 4q + j; `wb` = the
// lane's base: 64q + ((chunk ^ q) << 2) + word)
template <int NOB>
__device__ __forceinline__ void lds_u_store(float *img, int wb, const f32x4v (&v)[NOB]) {
#pragma unroll
    for (int ob = 0; ob < NOB; ++ob)
#pragma unroll
        for (int j = 0; j < 4; ++j) img[wb + 256 * ob + 16 * j] = v[ob][j];
}

struct BwdIn16 {
    uint64_t mk[3];  // the forward's mask words of lane-half q & 1
    float y[3], g[3], gs;
    float4 x;        // x features 4q .. 4q + 3
};

__device__ __forceinline__ void load_bwd_in16(const float *__restrict__ rgb_in, const uint64_t *__restrict__ masks,
                                              const float *__restrict__ g_sdf, const float *__restrict__ g_rgb,
                                              const float *__restrict__ feat, int64_t s, bool valid, int q,
                                              BwdIn16 &in, const int *__restrict__ x_src = nullptr) {
    const int64_t sv = valid ? s : 0;
    const uint64_t *mk = masks + (sv * 2 + (q & 1)) * 3;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        in.mk[i] = mk[i];
        in.y[i] = rgb_in[sv * 3 + i];
        in.g[i] = g_rgb[sv * 3 + i];
    }
    in.gs = g_sdf[sv];
    const int64_t xr = x_src ? (int64_t)x_src[sv] : sv;  // x_src: the sample's feature row (no compact copy)
    in.x = *reinterpret_cast<const float4 *>(feat + xr * kIn + 4 * q);
}

// chain wave: acc += δ rows [32c, 32c + 32) of the round's unit images ⊗ the
// units' x images (16 valid columns: lanes ≥ 16 feed zeros); bsum: Σ of the
// rows.  The accumulator lives in LDS between phases (`page`: [4][lane][4]
// floats, this wave's own): read, accumulated, written back — the same bits
// as a register-resident accumulator, 16 registers free in the other phases.
__device__ __forceinline__ void xgrad16(const float *dset, const float *xset, int c, int64_t ubase, int64_t u1,
                                        int lane, float *page, float *bsum) {
    const int i = lane & 31, h = lane >> 5;
    if (ubase >= u1) return;
    f32x16 acc;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float4 v = *reinterpret_cast<const float4 *>(page + (k * 64 + lane) * 4);
        acc[4 * k] = v.x;
        acc[4 * k + 1] = v.y;
        acc[4 * k + 2] = v.z;
        acc[4 * k + 3] = v.w;
    }
    const bool xv = i < 16;
    int ra[2], rx[2];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        ra[g] = i * kU + (((2 * h + g) ^ ((i >> 2) & 3)) << 2);
        rx[g] = (i & 15) * kU + (((2 * h + g) ^ (((i & 15) >> 2) & 3)) << 2);
    }
#pragma unroll
    for (int up = 0; up < 4; ++up) {
        if (ubase + up >= u1) break;  // wave-uniform
        const float *dl = dset + up * kUImg + 32 * c * kU;
        const float *xl = xset + up * 16 * kU;
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            const float4 a = *reinterpret_cast<const float4 *>(dl + ra[g]);
            float4 b = *reinterpret_cast<const float4 *>(xl + rx[g]);
            if (!xv) b = make_float4(0.f, 0.f, 0.f, 0.f);
            acc = mfma(a.x, b.x, acc);
            acc = mfma(a.y, b.y, acc);
            acc = mfma(a.z, b.z, acc);
            acc = mfma(a.w, b.w, acc);
            if (bsum) *bsum += (a.x + a.y) + (a.z + a.w);
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
        *reinterpret_cast<float4 *>(page + (k * 64 + lane) * 4) =
            make_float4(acc[4 * k], acc[4 * k + 1], acc[4 * k + 2], acc[4 * k + 3]);
}

// byte offset within a CF tile of lane (i, h)'s operand: row 32·blk + i,
// 16-B group h·4 + 2·hf + g (hf: the unit's half of the 32-sample tile).
// Computed, not selected from a table: a runtime index into a register
// array sends the array to scratch.
__device__ __forceinline__ int cf_voff(int blk, int lane, int hf, int g) {
    const int row = 32 * blk + (lane & 31);
    return (row * kTileS + ((((lane >> 5) * 4 + 2 * hf + g) ^ ((row >> 1) & 7)) << 2)) * 4;
}

// gradient wave c (P0, the previous round's units): dW5 column block c +=
// δ5 ⊗ c1 (VALU), b5 partials — in the phase where the gradient waves have
// no GEMM (on the chain, in P2, it lengthened the chain's longest phase); the
// c1 operands of two units in flight at a time
__device__ __forceinline__ void w5_grad(const float *sset, __amdgpu_buffer_rsrc_t c1m, int c, int64_t ubase,
                                        int64_t u1, int lane, float (&w5)[3], float (&b5)[3]) {
    const int h = lane >> 5;
#pragma unroll
    for (int pr = 0; pr < 4; ++pr) {
        float4 cl[1][2];
#pragma unroll
        for (int k = 0; k < 1; ++k) {
            int64_t u = ubase + pr + k;
            if (u >= u1) u = u1 - 1;  // in range (data unused)
#pragma unroll
            for (int g = 0; g < 2; ++g)
                cl[k][g] = bload4(c1m, cf_voff(c, lane, (int)(u & 1), g), (int)((u >> 1) * (kCfTile * 4)));
        }
#pragma unroll
        for (int k = 0; k < 1; ++k) {
            const int up = pr + k;
            if (ubase + up >= u1) break;
            const float *sl = sset + up * 4 * kU + 8 * h;
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) {
                    const float4 w = *reinterpret_cast<const float4 *>(sl + ch * kU + 4 * g);
                    const float4 a = cl[k][g];
                    w5[ch] += (a.x * w.x + a.y * w.y) + (a.z * w.z + a.w * w.w);
                    b5[ch] += (w.x + w.y) + (w.z + w.w);
                }
        }
    }
}

// gradient wave B operand: step q (unit q >> 1, k-group q & 1) of column block d
__device__ __forceinline__ float4 dw_bsrc(__amdgpu_buffer_rsrc_t act, int64_t ubase, int64_t u1, int d, int lane, int q) {
    int64_t u = ubase + (q >> 1);
    if (u >= u1) u = u1 - 1;  // in range (data unused)
    if (u < 0) u = 0;
    return bload4(act, cf_voff(d, lane, (int)(u & 1), q & 1), (int)((u >> 1) * (kCfTile * 4)));
}

// gradient wave, one job (a phase's layer): acc[ob] += δ (the round's unit
// images, all 4 row blocks) ⊗ the activation's column block d; bsum += Σ of
// row block d; EX = 2 (W3): row0 += δsdf ⊗ h2, b30 += Σ δsdf.  The B
// operands run through a 3-slot ring two steps ahead that continues into
// the next job (its first two loads are issued here, before the barrier):
// step q of a job with ring offset RO uses slot (RO + q) % 3.
template <int EX, int RO>
__device__ __forceinline__ void dw_job(float4 (&ring)[3], const float *dset, const float *sset,
                                       __amdgpu_buffer_rsrc_t act, int64_t ubase, bool on,
                                       __amdgpu_buffer_rsrc_t act_n, int64_t ubase_n, bool has_n, int64_t u1, int d,
                                       int lane, f32x16 (&acc)[kNB], float &bsum, float &row0, float &b30) {
    const int i = lane & 31, h = lane >> 5;
    int ra[2];
#pragma unroll
    for (int g = 0; g < 2; ++g) ra[g] = i * kU + (((2 * h + g) ^ ((i >> 2) & 3)) << 2);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int up = q >> 1, g = q & 1;
        const float4 b = ring[(RO + q) % 3];
        if (q + 2 < 8) ring[(RO + q + 2) % 3] = dw_bsrc(act, ubase, u1, d, lane, q + 2);
        else if (has_n) ring[(RO + q + 2) % 3] = dw_bsrc(act_n, ubase_n, u1, d, lane, q - 6);
        if (on && ubase + up < u1) {  // wave-uniform
            const float *dl = dset + up * kUImg;
            float4 a[kNB];
#pragma unroll
            for (int ob = 0; ob < kNB; ++ob) a[ob] = *reinterpret_cast<const float4 *>(dl + 32 * ob * kU + ra[g]);
#pragma unroll
            for (int ob = 0; ob < kNB; ++ob) acc[ob] = mfma(a[ob].x, b.x, acc[ob]);
#pragma unroll
            for (int ob = 0; ob < kNB; ++ob) acc[ob] = mfma(a[ob].y, b.y, acc[ob]);
#pragma unroll
            for (int ob = 0; ob < kNB; ++ob) acc[ob] = mfma(a[ob].z, b.z, acc[ob]);
#pragma unroll
            for (int ob = 0; ob < kNB; ++ob) acc[ob] = mfma(a[ob].w, b.w, acc[ob]);
            {  // row block d's sum: its own read (a[d] with a runtime d would put a[] in scratch)
                const float4 ad = *reinterpret_cast<const float4 *>(dl + 32 * d * kU + ra[g]);
                bsum += (ad.x + ad.y) + (ad.z + ad.w);
            }
            if (EX == 2) {
                const float4 w = *reinterpret_cast<const float4 *>(sset + up * 4 * kU + 8 * h + 4 * g);
                row0 += (b.x * w.x + b.y * w.y) + (b.z * w.z + b.w * w.w);
                b30 += (w.x + w.y) + (w.z + w.w);
            }
        }
    }
}

using ifuse::interp_bwd_unit;
using ifuse::scatter_unit;

struct Bwd3Src {
    const float *rgb, *g_sdf, *g_rgb, *feat;
    const uint64_t *masks;
    const float *act;  // CF [h1 | h2 | f | c1]
    float *dfeat;
    const int *x_src;  // or null: sample s's x is row x_src[s] of feat
};

// W = false (frozen decoder: dfeat only, e.g. tracking): all 8 waves run the
// chain (8 units per round), no exports, no gradients — the same chain
// arithmetic, so dfeat is bit-identical to the training call's.
//
// With ip.gx set (W only; the mapping engine) the chain wave also runs the
// interpolation backward of its unit in P3, right after dfeat (which is then
// not stored): the samples' leaf / ray / vertex rows load during P2, the 8
// embedding rows at the start of P3 (beside the W1ᵀ GEMM), then dL/dx per
// sample (ip.gx, summed per ray by k_interp_rays_gx) and the embedding
// scatter, summed over each leaf run of the unit first (k_interp_bwd's
// scheme: lanes own (corner, dim), whole 64-B rows per atomic instruction).
template <bool W>
__global__ __launch_bounds__(kF2Threads, 1) void k_mlp_bwd3(int64_t m, const float *__restrict__ img, Bwd3Src src,
                                                            DwGrid g, float *__restrict__ slabs, InterpFuse ip,
                                                            const int *__restrict__ m_dev) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    if (m_dev) m = __builtin_amdgcn_readfirstlane(*m_dev);  // the sparse decoder's kept samples (<= m)
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t n_tiles = (m + kCh - 1) / kCh * 2;  // CF tiles (32 samples)
    const int64_t tstride = n_tiles * kCfTile;
    const int64_t tb = tstride * 4;
    const int64_t n_units = (m + kU - 1) / kU;
    const int64_t u0 = n_units * blockIdx.x / gridDim.x, u1 = n_units * (blockIdx.x + 1) / gridDim.x;
    constexpr int kPer = W ? 4 : 8;  // units per round
    const int n_rounds = (int)((u1 - u0 + kPer - 1) / kPer);
    float *const slot = lds + kB3Slot, *const small = lds + kB3Small, *const xim = lds + kB3X;
    auto dset = [&](int s) { return slot + s * 4 * kUImg; };
    // the chain's 4 exports per round alternate over 2 sets (export e = 4r + phase → set e mod 2):
    // each is read in the phase after its write, the next write to its set is a phase later
    auto eset = [&](int e) { return dset(((e % 2) + 2) % 2); };
    auto sset = [&](int s) { return small + s * 4 * 4 * kU; };
    auto xset = [&](int par) { return xim + par * 4 * 16 * kU; };
    stage8(lds, img + kImgVec, kVecPad, wave, lane);
    wait_vm(0);
    raw_barrier();
    const int b = blockIdx.x;
    const int i = lane & 31, h = lane >> 5;
    if (!W || wave < 4) {
        // ================= chain wave c
        const __amdgpu_buffer_rsrc_t wrs = rsrc_of(img, (int64_t)kImgTotal * 4);
        const int c = wave;
        const int n = lane & 15, q = lane >> 4;
        const int sn = (n & 1) * 8 + (n >> 1);                     // the sample's slot
        const int wb = 64 * q + ((((sn >> 2) ^ q) << 2) | (sn & 3));  // + 256 ob + 16 j
        float *const page1 = lds + kB3A + c * 2048, *const page4x = page1 + 1024;  // dW1, dW4x accumulators
        if (W) {
#pragma unroll
            for (int k = 0; k < 8; ++k)
                *reinterpret_cast<float4 *>(page1 + (k * 64 + lane) * 4) = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        float b1p = 0.f;
        BwdIn16 nin;
        {
            const int64_t u = u0 + c;
            const int64_t s = u * kU + n;
            load_bwd_in16(src.rgb, src.masks, src.g_sdf, src.g_rgb, src.feat, s, u < u1 && s < m, q, nin, src.x_src);
        }
        [[maybe_unused]] constexpr int kStampK = 1;
        PSVO_STAMP_DECL;
        for (int r = 0; r <= n_rounds; ++r) {
            PSVO_STAMP(0);
            const int64_t ubase = u0 + kPer * (int64_t)r;
            const int64_t u = ubase + c;
            const bool active = r < n_rounds && u < u1;  // wave-uniform
            const int64_t s = u * kU + n;
            const bool valid = active && s < m;
            // ---- P0: δ5 / δc1 / x → LDS; δ[f; x] = W4ᵀ δc1; dW1 of the previous round
            f32x4v fa[8], fb[8], dxc[1];
            float dsdf = 0.f;
            uint64_t m1 = 0, m2 = 0;
            if (r < n_rounds) {
                const BwdIn16 in = nin;
                float d5[3];
#pragma unroll
                for (int ch = 0; ch < 3; ++ch)  // roundings spelled out: both instantiations give the same bits
                    d5[ch] = valid ? __fmul_rn(in.g[ch], __fmul_rn(in.y[ch], __fsub_rn(1.0f, in.y[ch]))) : 0.0f;
                dsdf = valid ? in.gs : 0.0f;
                const int sh = 4 * (q >> 1);
                m1 = valid ? in.mk[0] >> sh : 0;
                m2 = valid ? in.mk[1] >> sh : 0;
                const uint64_t m4 = valid ? in.mk[2] >> sh : 0;
                if (W) {
                    float *xl = xset(r & 1) + c * 16 * kU;
                    xl[wb + 0] = valid ? in.x.x : 0.f;
                    xl[wb + 16] = valid ? in.x.y : 0.f;
                    xl[wb + 32] = valid ? in.x.z : 0.f;
                    xl[wb + 48] = valid ? in.x.w : 0.f;
                }
                if (W && q == 0) {  // δ5: rows 0..2 of the round's small set (read by dW5 a round later)
                    float *sl = sset(r & 1) + c * 4 * kU;
#pragma unroll
                    for (int ch = 0; ch < 3; ++ch) sl[ch * kU + sn] = d5[ch];
                }
                if (active) {
#pragma unroll
                    for (int ob = 0; ob < 8; ++ob) {  // δc1 = W5ᵀ δ5 ⊙ mask
                        const int k = 16 * ob + 4 * q;
                        const float4 w0 = *reinterpret_cast<const float4 *>(lds + kOffW5 + k);
                        const float4 w1 = *reinterpret_cast<const float4 *>(lds + kOffW5 + 128 + k);
                        const float4 w2 = *reinterpret_cast<const float4 *>(lds + kOffW5 + 256 + k);
                        auto dot3 = [&](float a0, float a1, float a2) {
                            return fmaf(a2, d5[2], fmaf(a1, d5[1], __fmul_rn(a0, d5[0])));
                        };
                        fb[ob] = f32x4v{dot3(w0.x, w1.x, w2.x), dot3(w0.y, w1.y, w2.y), dot3(w0.z, w1.z, w2.z),
                                        dot3(w0.w, w1.w, w2.w)};
                    }
                    mask16(fb, m4);
                    if (W) lds_u_store<8>(eset(4 * r) + c * kUImg, wb, fb);
                    zero4(fa);
                    zero4(dxc);
                    gemm16<8, 4, 2>(wrs, kImgC4, fb, *reinterpret_cast<f32x4v(*)[4]>(&fa[0]), lane);  // δf
                    gemm16<8, 4, 2>(wrs, kImgC4 + 4 * 8 * 256, fb, *reinterpret_cast<f32x4v(*)[4]>(&fa[4]), lane);
                    gemm16<8, 1, 4>(wrs, kImgC4 + 8 * 8 * 256, fb, dxc, lane);  // δx_c
                }
            }
            if (W && r > 0) xgrad16(eset(4 * r - 1), xset((r - 1) & 1), c, ubase - 4, u1, lane, page1, &b1p);
            PSVO_STAMP(1);
            raw_barrier();
            PSVO_STAMP(2);
            if (r == n_rounds) break;
            // ---- P1: δf / δsdf → LDS; δh2 = W3ᵀ [δsdf; δf] ⊙ m2; dW4x, dW5
            if (W && q == 0) sset(r & 1)[c * 4 * kU + 3 * kU + sn] = dsdf;  // row 3
            if (active) {
                if (W) lds_u_store<8>(eset(4 * r + 1) + c * kUImg, wb, fa);
#pragma unroll
                for (int ob = 0; ob < 8; ++ob) {
                    const float4 w = *reinterpret_cast<const float4 *>(lds + kOffW3r0 + 16 * ob + 4 * q);
                    fb[ob] = f32x4v{__fmul_rn(w.x, dsdf), __fmul_rn(w.y, dsdf), __fmul_rn(w.z, dsdf), __fmul_rn(w.w, dsdf)};
                }
                gemm16<8, 4, 2>(wrs, kImgC3, fa, *reinterpret_cast<f32x4v(*)[4]>(&fb[0]), lane);
                gemm16<8, 4, 2>(wrs, kImgC3 + 4 * 8 * 256, fa, *reinterpret_cast<f32x4v(*)[4]>(&fb[4]), lane);
                mask16(fb, m2);  // δh2
            }
            if (W) {
                xgrad16(eset(4 * r), xset(r & 1), c, ubase, u1, lane, page4x, nullptr);
            }
            // the interpolation backward's sample data, one dependent level per phase
            const bool fuse = W && ip.gx != nullptr;  // uniform
            int lf = 0, ro = 0;
            float ts = 0.f;
            if (fuse && valid) {
                lf = ip.leaf[s];
                ro = ip.ray_of[s];
                ts = ip.t[s];
            }
            PSVO_STAMP(3);
            raw_barrier();
            PSVO_STAMP(4);
            // ---- P2: δh2 → LDS; δh1 = W2ᵀ δh2 ⊙ m1 (+ the interpolation backward's sample data)
            int4 vid0 = make_int4(0, 0, 0, 0), vid1 = make_int4(0, 0, 0, 0);
            float cen[3] = {0.f, 0.f, 0.f};
            int row = 0;
            if (fuse && valid) {
                vid0 = *reinterpret_cast<const int4 *>(ip.vertex_idx + (int64_t)lf * 8);
                vid1 = *reinterpret_cast<const int4 *>(ip.vertex_idx + (int64_t)lf * 8 + 4);
#pragma unroll
                for (int a = 0; a < 3; ++a) cen[a] = ip.centres[(int64_t)lf * 3 + a];
                row = ip.rank_ray[ro];
            }
            if (active) {
                if (W) lds_u_store<8>(eset(4 * r + 2) + c * kUImg, wb, fb);
                zero4(fa);
                gemm16<8, 4, 2>(wrs, kImgC2, fb, *reinterpret_cast<f32x4v(*)[4]>(&fa[0]), lane);
                gemm16<8, 4, 2>(wrs, kImgC2 + 4 * 8 * 256, fb, *reinterpret_cast<f32x4v(*)[4]>(&fa[4]), lane);
                mask16(fa, m1);  // δh1
            }
            float ro3[3] = {0.f, 0.f, 0.f}, rd3[3] = {0.f, 0.f, 0.f};
            float4 ev[8];
            if (fuse) {  // the 8 embedding rows (used in P3)
                const int vid[8] = {vid0.x, vid0.y, vid0.z, vid0.w, vid1.x, vid1.y, vid1.z, vid1.w};
#pragma unroll
                for (int k = 0; k < 8; ++k) ev[k] = reinterpret_cast<const float4 *>(ip.emb)[(int64_t)vid[k] * 4 + q];
                if (valid) {
#pragma unroll
                    for (int a = 0; a < 3; ++a) {
                        ro3[a] = ip.rays_o[(int64_t)row * 3 + a];
                        rd3[a] = ip.rays_d[(int64_t)row * 3 + a];
                    }
                }
            }
            PSVO_STAMP(5);
            raw_barrier();
            PSVO_STAMP(6);
            // ---- P3: δh1 → LDS; dfeat = W1ᵀ δh1 + δx_c; the next unit's inputs
            if (W && active) lds_u_store<8>(eset(4 * r + 3) + c * kUImg, wb, fa);
            if (r + 1 < n_rounds) {
                const int64_t un = u + kPer;
                const int64_t snx = un * kU + n;
                load_bwd_in16(src.rgb, src.masks, src.g_sdf, src.g_rgb, src.feat, snx, un < u1 && snx < m, q, nin,
                              src.x_src);
            }
            if (active) {
                f32x4v t1[1];
                zero4(t1);
                gemm16<8, 1, 4>(wrs, kImgC1, fa, t1, lane);
                const float4 gf = make_float4(__fadd_rn(t1[0][0], dxc[0][0]), __fadd_rn(t1[0][1], dxc[0][1]),
                                              __fadd_rn(t1[0][2], dxc[0][2]), __fadd_rn(t1[0][3], dxc[0][3]));
                if (!fuse) {
                    if (valid) *reinterpret_cast<float4 *>(src.dfeat + s * kIn + 4 * q) = gf;
                } else {
                    interp_bwd_unit(ip, lds + kB3I + c * 512, m, s, valid, n, q, ts, ro3, rd3, cen, vid0, vid1, ev,
                                    gf);
                    if (ip.grad_emb != nullptr) {
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the staging is this wave's own
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                        scatter_unit(ip, lds + kB3I + c * 512, u, m, lane, lf);
                    }
                }
            }
            PSVO_STAMP(7);
            raw_barrier();
            PSVO_STAMP(8);
            PSVO_STAMP_FLUSH(1);
        }
        if (!W) return;
        // ---- slabs: W1 row block c + b1; W4's x columns of row block c; W5 column block c (+ b5)
        float *s1 = slabs + g.slab_off[0] + (int64_t)b * g.slab_len[0];
        float *s4 = slabs + g.slab_off[3] + (int64_t)b * g.slab_len[3];
        if (i < 16) {
#pragma unroll
            for (int rr = 0; rr < 16; ++rr) {
                const int row = 32 * c + phi(rr, h);
                const int pos = ((rr >> 2) * 64 + lane) * 4 + (rr & 3);
                store_nt(s1, row * 16 + i, page1[pos]);
                store_nt(s4, row * 144 + 128 + i, page4x[pos]);
            }
        }
        const float bv = b1p + __shfl_xor(b1p, 32, 64);
        if (h == 0) store_nt(s1, 128 * 16 + 32 * c + i, bv);
    } else {
        // ================= gradient wave: column block d of W2 / W3 / W4, biases of row block d
        const int d = wave - 4;
        f32x16 acc2[kNB], acc3[kNB], acc4[kNB];
        zero(acc2);
        zero(acc3);
        zero(acc4);
        float b2p = 0.f, b3p = 0.f, b4p = 0.f, r0 = 0.f, b30 = 0.f, unused0 = 0.f, unused1 = 0.f;
        // dW5 / b5 partials live in LDS between rounds (registers are full with dW2..4)
        float *const page5 = lds + kB3W5 + d * 512 + lane * 8;
        *reinterpret_cast<float4 *>(page5) = make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<float4 *>(page5 + 4) = make_float4(0.f, 0.f, 0.f, 0.f);
        const __amdgpu_buffer_rsrc_t c1m = rsrc_of(src.act + 3 * tstride, tb);
        const __amdgpu_buffer_rsrc_t h1m = rsrc_of(src.act, tb), h2m = rsrc_of(src.act + tstride, tb),
                                     fm = rsrc_of(src.act + 2 * tstride, tb);
        [[maybe_unused]] constexpr int kStampK = 1;
        PSVO_STAMP_DECL;
        float4 ring[3];  // B operands, continuous across the jobs (see dw_job)
        ring[0] = dw_bsrc(fm, u0, u1, d, lane, 0);
        ring[1] = dw_bsrc(fm, u0, u1, d, lane, 1);
        for (int r = 0; r <= n_rounds; ++r) {
            const int64_t ubase = u0 + 4 * (int64_t)r;
            PSVO_STAMP(0);
            // P0: dW5 of the previous round (δ5 in its small set), beside the chain's W4ᵀ and dW1
            if (r > 0) {
                float w5[3] = {0.f, 0.f, 0.f}, b5[3] = {0.f, 0.f, 0.f};
                w5_grad(sset((r - 1) & 1), c1m, d, ubase - 4, u1, lane, w5, b5);
                float4 p0 = *reinterpret_cast<float4 *>(page5), p1 = *reinterpret_cast<float4 *>(page5 + 4);
                p0.x += w5[0]; p0.y += w5[1]; p0.z += w5[2];
                p1.x += b5[0]; p1.y += b5[1]; p1.z += b5[2];
                *reinterpret_cast<float4 *>(page5) = p0;
                *reinterpret_cast<float4 *>(page5 + 4) = p1;
            }
            PSVO_STAMP(1);
            raw_barrier();
            PSVO_STAMP(2);
            if (r == n_rounds) break;
            // P1: dW4 (δc1: export 0)
            dw_job<0, 0>(ring, eset(4 * r), nullptr, fm, ubase, true, h2m, ubase, true, u1, d, lane, acc4, b4p,
                         unused0, unused1);
            PSVO_STAMP(3);
            raw_barrier();
            PSVO_STAMP(4);
            // P2: dW3 (δf, δsdf: export 1)
            dw_job<2, 2>(ring, eset(4 * r + 1), sset(r & 1) + 3 * kU, h2m, ubase, true, h1m, ubase, true, u1, d, lane, acc3, b3p,
                         r0, b30);
            PSVO_STAMP(5);
            raw_barrier();
            PSVO_STAMP(6);
            // P3: dW2 (δh2: export 2), beside the chain's W1ᵀ and interpolation backward
            dw_job<0, 1>(ring, eset(4 * r + 2), nullptr, h1m, ubase, true, fm, ubase + 4, r + 1 < n_rounds, u1, d,
                         lane, acc2, b2p, unused0, unused1);
            PSVO_STAMP(7);
            raw_barrier();
            PSVO_STAMP(8);
            PSVO_STAMP_FLUSH(1);
        }
        const int rb[kNB] = {0, 1, 2, 3}, cb[1] = {d};
        float *s2 = slabs + g.slab_off[1] + (int64_t)b * g.slab_len[1];
        float *s3 = slabs + g.slab_off[2] + (int64_t)b * g.slab_len[2];
        float *s4 = slabs + g.slab_off[3] + (int64_t)b * g.slab_len[3];
        {
            f32x16 t[kNB][1];
#pragma unroll
            for (int k = 0; k < kNB; ++k) t[k][0] = acc2[k];
            dw_store<kNB, 1, true>(s2, 128, 0, 128, rb, cb, t, lane);
#pragma unroll
            for (int k = 0; k < kNB; ++k) t[k][0] = acc3[k];
            dw_store<kNB, 1, true>(s3, 128, 1, 128, rb, cb, t, lane);
#pragma unroll
            for (int k = 0; k < kNB; ++k) t[k][0] = acc4[k];
            dw_store<kNB, 1, true>(s4, 144, 0, 144, rb, cb, t, lane);
        }
        const float v2 = b2p + __shfl_xor(b2p, 32, 64), v3 = b3p + __shfl_xor(b3p, 32, 64),
                    v4 = b4p + __shfl_xor(b4p, 32, 64), vr0 = r0 + __shfl_xor(r0, 32, 64),
                    v30 = b30 + __shfl_xor(b30, 32, 64);
        if (h == 0) {
            store_nt(s2, 128 * 128 + 32 * d + i, v2);
            store_nt(s3, 129 * 128 + 1 + 32 * d + i, v3);
            store_nt(s4, 128 * 144 + 32 * d + i, v4);
            store_nt(s3, 32 * d + i, vr0);  // W3 row 0 (sdf)
        }
        if (d == 0 && lane == 0) store_nt(s3, 129 * 128, v30);
        // W5 column block d (+ b5)
        float *s5 = slabs + g.slab_off[4] + (int64_t)b * g.slab_len[4];
        const float4 p0 = *reinterpret_cast<const float4 *>(page5), p1 = *reinterpret_cast<const float4 *>(page5 + 4);
        const float w5[3] = {p0.x, p0.y, p0.z}, b5[3] = {p1.x, p1.y, p1.z};
        float v5[3], t5[3];
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            v5[ch] = w5[ch] + __shfl_xor(w5[ch], 32, 64);
            t5[ch] = b5[ch] + __shfl_xor(b5[ch], 32, 64);  // every lane of a half holds its half's Σ δ5
        }
        if (h == 0) {
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) store_nt(s5, ch * 128 + 32 * d + i, v5[ch]);
        }
        if (d == 0 && lane == 0) {
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) store_nt(s5, 3 * 128 + ch, t5[ch]);
        }
    }
}

// ---------------------------------------------------------------------------
// The sparse decoder's class B (samples whose only loss term is the direct
// one on their sdf — composite.hip k_select_samples): their colour head's δ's
// are exactly zero (g_rgb = 0, so δ5 = δc1 = δf = 0), so forward and backward
// need the trunk only:
//   h1 = relu(W1 x + b1),  h2 = relu(W2 h1 + b2)                       (forward)
//   δh2 = W3[0]ᵀ dsdf ⊙ [h2 > 0],  δh1 = W2ᵀ δh2 ⊙ [h1 > 0],  dfeat = W1ᵀ δh1
//   dW1 += δh1 ⊗ x,  dW2 += δh2 ⊗ h1,  W3 row 0 += dsdf · h2  (+ b1, b2, b3[0])
// 54 k MACs per sample, in ONE kernel that keeps the activations on chip (no
// activation round trip through HBM, no separate forward launch: the two
// measured 57 + 110 µs at config B).  The forward is recomputed here with the
// chain's 16 × 16 × 4 MFMAs (the sdf came from k_mlp_sdf2: the same values up
// to the accumulation order, which only the ReLU masks' ties could see).
// Rounds of four 16-sample units (unit u0 + 4r + k on chain wave k and
// gradient wave 4 + k), two phases each:
//   phase  chain wave c                                    gradient wave d
//   P(r)   δh2(r) from LDS; δh1 = W2ᵀ δh2 ⊙ [h1 > 0]       dW2 col block d += δh2(r) ⊗ h1(r)
//          → LDS                                           (both operands in LDS)
//   Q(r)   dfeat = W1ᵀ δh1 → the interpolation backward    dW1 row block d += δh1(r) ⊗ x(r); the
//          (dL/dx, the embedding scatter)                  forward of unit d of round r + 1: x → LDS,
//                                                          h1 = relu(W1 x + b1) → LDS (CF tile),
//                                                          h2 = relu(W2 h1 + b2), W3 row 0 += dsdf · h2,
//                                                          δh2 → LDS, the h1 mask words → LDS
// (the forward of round 0 before the loop).  A chain wave and a gradient
// wave share each SIMD's matrix unit: in P both run 128 × 128 GEMMs (W2ᵀ,
// dW2), in Q the gradient wave's forward overlaps the chain's latency-bound
// interpolation backward.  (The forward on the chain waves, with W2ᵀ in one
// phase: 42 k cycles per round, the chain alone in that phase for 62 % of
// it — s_memtime stamps, scripts/trunk_stamps.py.)  Writes one slab per
// workgroup of W1 (+ b1), W2 (+ b2) and W3's row 0 (+ b3[0]) in `slabs` (the
// DwGrid layout; k_mlp_dw_reduce adds these elements only).  m: the class's
// count on the device.
constexpr int kT4H2 = kVecPad;                 // δh2 unit images [unit 4]
constexpr int kT4H1 = kT4H2 + 4 * kUImg;       // δh1 unit images [unit 4]
constexpr int kT4CF = kT4H1 + 4 * kUImg;       // h1 as CF tiles [2] (the round's unit k → tile k / 2, half k % 2)
constexpr int kT4X = kT4CF + 2 * kCfTile;      // x images [round parity 2][unit 4][16 × 16]
constexpr int kT4I = kT4X + 2 * 4 * 16 * kU;   // interpolation backward staging [chain wave 4][512]
constexpr int kT4R = kT4I + 4 * 512;           // W3 row 0 / b3[0] partials [gradient wave 4][132]
constexpr int kT4M = kT4R + 4 * 132;           // h1 mask words [unit 4][lane 64] (u64)
constexpr int kLdsTrunk = (kT4M + 4 * 64 * 2) * 4;  // 123,968 B
static_assert(kLdsTrunk <= 160 * 1024, "trunk kernel LDS budget");

// Σ of v over the 16 lanes of the lane's DPP row (the chain's samples n of one
// q group), in every lane of the row: quad xor 1, xor 2, half-row mirror, row mirror
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row_sum16(float v) {
    v += dpp_mov<0xB1>(v);   // quad_perm [1, 0, 3, 2]
    v += dpp_mov<0x4E>(v);   // quad_perm [2, 3, 0, 1]
    v += dpp_mov<0x141>(v);  // row_half_mirror
    v += dpp_mov<0x140>(v);  // row_mirror
    return v;
}

__device__ __forceinline__ uint64_t relu16(f32x4v (&v)[8]) {
    uint64_t w = 0;
#pragma unroll
    for (int ob = 0; ob < 8; ++ob)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool on = v[ob][j] > 0.0f;
            w |= (uint64_t)on << (8 * ob + j);
            v[ob][j] = on ? v[ob][j] : 0.0f;
        }
    return w;
}

// gradient wave, dW2 += δh2 (the round's unit images) ⊗ h1 (the round's CF
// image in LDS), column block d — dw_job's arithmetic with both operands on chip
__device__ __forceinline__ void dw_job_lds(const float *dset, const float *cf, int64_t ubase, int64_t u1, int d,
                                           int lane, f32x16 (&acc)[kNB], float &bsum) {
    const int i = lane & 31, h = lane >> 5;
    int ra[2];
#pragma unroll
    for (int g = 0; g < 2; ++g) ra[g] = i * kU + (((2 * h + g) ^ ((i >> 2) & 3)) << 2);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int up = q >> 1, g = q & 1;
        if (ubase + up >= u1) break;  // wave-uniform
        const float4 b = *reinterpret_cast<const float4 *>(cf + (up >> 1) * kCfTile + cf_voff(d, lane, up & 1, g) / 4);
        const float *dl = dset + up * kUImg;
        float4 a[kNB];
#pragma unroll
        for (int ob = 0; ob < kNB; ++ob) a[ob] = *reinterpret_cast<const float4 *>(dl + 32 * ob * kU + ra[g]);
#pragma unroll
        for (int ob = 0; ob < kNB; ++ob) acc[ob] = mfma(a[ob].x, b.x, acc[ob]);
#pragma unroll
        for (int ob = 0; ob < kNB; ++ob) acc[ob] = mfma(a[ob].y, b.y, acc[ob]);
#pragma unroll
        for (int ob = 0; ob < kNB; ++ob) acc[ob] = mfma(a[ob].z, b.z, acc[ob]);
#pragma unroll
        for (int ob = 0; ob < kNB; ++ob) acc[ob] = mfma(a[ob].w, b.w, acc[ob]);
        const float4 ad = *reinterpret_cast<const float4 *>(dl + 32 * d * kU + ra[g]);
        bsum += (ad.x + ad.y) + (ad.z + ad.w);
    }
}

struct TrunkIn {
    float gs;
    float4 x;
    int src;  // the sample's h2 row (h2 given), else 0
};
__device__ __forceinline__ void load_trunk_in(const float *__restrict__ g_sdf, const float *__restrict__ feat,
                                              const int *__restrict__ src, int64_t s, bool valid, int q,
                                              TrunkIn &in) {
    const int64_t sv = valid ? s : 0;
    in.gs = g_sdf[sv];
    in.src = src && valid ? src[sv] : 0;
    in.x = *reinterpret_cast<const float4 *>(feat + (src ? (int64_t)in.src : sv) * kIn + 4 * q);  // (src: feat is
                                                                                                 // the step's rows)
}

template <int NOB>
__device__ __forceinline__ void lds_u_load(const float *img, int wb, f32x4v (&v)[NOB]) {
#pragma unroll
    for (int ob = 0; ob < NOB; ++ob)
#pragma unroll
        for (int j = 0; j < 4; ++j) v[ob][j] = img[wb + 256 * ob + 16 * j];
}

// acc[ob] += W blocks (ob, kb) of the image at `img_off` · in[kb] for NOB output
// blocks, streamed as one sequence of (output-block pair, kb) steps with the
// A-operand ring D steps deep running across the pairs (one ring fill per
// GEMM, not one per pair; 2 · 4 · (D + 1) ring registers)
template <int NKB, int NOB, int D>
__device__ __forceinline__ void gemm16_stream(__amdgpu_buffer_rsrc_t rs, int img_off, const f32x4v (&in)[NKB],
                                              f32x4v (&acc)[NOB], int lane) {
    static_assert(NOB % 2 == 0, "output blocks in pairs");
    constexpr int kSteps = NOB / 2 * NKB;
    auto ld = [&](int st, int i) {
        const int ob = 2 * (st / NKB) + i, kb = st % NKB;
        return bload4(rs, lane * 16, (img_off + (ob * NKB + kb) * 256) * 4);
    };
    float4 ring[D + 1][2];
#pragma unroll
    for (int st = 0; st < D; ++st)
#pragma unroll
        for (int i = 0; i < 2; ++i) ring[st][i] = ld(st, i);
#pragma unroll
    for (int st = 0; st < kSteps; ++st) {
        const int cs = st % (D + 1), ob = 2 * (st / NKB), kb = st % NKB;
        if (st + D < kSteps) {
#pragma unroll
            for (int i = 0; i < 2; ++i) ring[(st + D) % (D + 1)][i] = ld(st + D, i);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[ob + i] = mfma16(ring[cs][i].x, in[kb][0], acc[ob + i]);
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[ob + i] = mfma16(ring[cs][i].y, in[kb][1], acc[ob + i]);
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[ob + i] = mfma16(ring[cs][i].z, in[kb][2], acc[ob + i]);
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[ob + i] = mfma16(ring[cs][i].w, in[kb][3], acc[ob + i]);
        if (st + D < kSteps) __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);  // the prefetch
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);                      // this step's MFMAs
        __builtin_amdgcn_sched_barrier(0);
    }
}

// gradient wave k: the trunk forward of unit k of round r (chain layout: lane
// (n, q) holds features 16·ob + 4q + j of sample n) → x image, h1 CF tile,
// δh2 unit image, h1 mask words; W3 row 0 / b3[0] partials into `page3`
template <bool H2>
__device__ __forceinline__ void trunk_fwd_unit(float *lds, __amdgpu_buffer_rsrc_t wrs, const TrunkIn &in, int64_t u,
                                               int64_t u1, int64_t m, int k, int lane, int wb, float *xl,
                                               float *page3, float &b30p, const float *__restrict__ h2) {
    const int n = lane & 15, q = lane >> 4;
    const int64_t s = u * kU + n;
    const bool active = u < u1;  // wave-uniform
    const bool valid = active && s < m;
    const float dsdf = valid ? in.gs : 0.0f;
    const float4 xv = valid ? in.x : make_float4(0.f, 0.f, 0.f, 0.f);
    xl[wb + 0] = xv.x;
    xl[wb + 16] = xv.y;
    xl[wb + 32] = xv.z;
    xl[wb + 48] = xv.w;
    if (!active) return;
    f32x4v fb[8];
    f32x4v xin[1] = {f32x4v{xv.x, xv.y, xv.z, xv.w}};
    f32x4v hb[8];
#pragma unroll
    for (int ob = 0; ob < 8; ++ob) {
        const float4 bb = *reinterpret_cast<const float4 *>(lds + kOffB1 + 16 * ob + 4 * q);
        hb[ob] = f32x4v{bb.x, bb.y, bb.z, bb.w};
    }
    gemm16_stream<1, 8, 3>(wrs, kImgT1, xin, hb, lane);  // h1 = W1 x + b1
    if (H2) {  // h2 read: features 16 ob + 4q .. + 3 of the sample's row (in flight under h1's ReLU and stores)
        const float *row = h2 + (int64_t)in.src * kW;
#pragma unroll
        for (int ob = 0; ob < 8; ++ob) {
            float4 v = *reinterpret_cast<const float4 *>(row + 16 * ob + 4 * q);
            if (!valid) v = make_float4(0.f, 0.f, 0.f, 0.f);
            fb[ob] = f32x4v{v.x, v.y, v.z, v.w};
        }
    }
    const uint64_t m1 = relu16(hb);
    reinterpret_cast<uint64_t *>(lds + kT4M)[k * 64 + lane] = m1;
    {  // h1 → the CF tile (dW2's B operand; k_mlp_fwd2's layout): row 16 ob + 4q + j,
       // sample n at group 4 (n & 1) + 2 (k & 1) + n / 8, element (n / 2) & 3;
       // the row's swizzle (row >> 1) & 7 does not depend on ob
        const int grp = 4 * (n & 1) + 2 * (k & 1) + (n >> 3), el = (n >> 1) & 3;
        float *const tile = lds + kT4CF + (k >> 1) * kCfTile;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float *const cj = tile + (4 * q + j) * kTileS + ((grp ^ ((2 * q + (j >> 1)) & 7)) << 2) + el;
#pragma unroll
            for (int ob = 0; ob < 8; ++ob) cj[16 * ob * kTileS] = hb[ob][j];
        }
    }
    if (!H2) {
#pragma unroll
        for (int ob = 0; ob < 8; ++ob) {
            const float4 bb = *reinterpret_cast<const float4 *>(lds + kOffB2 + 16 * ob + 4 * q);
            fb[ob] = f32x4v{bb.x, bb.y, bb.z, bb.w};
        }
        // h2 = W2 h1 + b2: output-block pairs, one ring across them (beside the dW2
        // accumulators a ring over all 8 output blocks spills)
        gemm16_stream<8, 8, 3>(wrs, kImgT2, hb, fb, lane);
    }
    const uint64_t m2 = relu16(fb);
    {  // W3 row 0 += Σ_n dsdf · h2 (the unit's 16 samples by DPP row sums, into the page)
        f32x4v r0[8];
#pragma unroll
        for (int ob = 0; ob < 8; ++ob)
#pragma unroll
            for (int j = 0; j < 4; ++j) r0[ob][j] = row_sum16(fb[ob][j] * dsdf);
        if (n == 0) {
#pragma unroll
            for (int ob = 0; ob < 8; ++ob) {
                float4 *pp = reinterpret_cast<float4 *>(page3 + 16 * ob + 4 * q);
                const float4 o = *pp;
                *pp = make_float4(o.x + r0[ob][0], o.y + r0[ob][1], o.z + r0[ob][2], o.w + r0[ob][3]);
            }
        }
    }
    b30p += dsdf;
#pragma unroll
    for (int ob = 0; ob < 8; ++ob) {  // δh2 = W3[0]ᵀ dsdf ⊙ [h2 > 0] (k_mlp_bwd3's δf = 0 case)
        const float4 w = *reinterpret_cast<const float4 *>(lds + kOffW3r0 + 16 * ob + 4 * q);
        fb[ob] = f32x4v{__fmul_rn(w.x, dsdf), __fmul_rn(w.y, dsdf), __fmul_rn(w.z, dsdf), __fmul_rn(w.w, dsdf)};
    }
    mask16(fb, m2);
    lds_u_store<8>(lds + kT4H2 + k * kUImg, wb, fb);
}

template <bool H2>
__global__ __launch_bounds__(kF2Threads, 1) void k_mlp_trunk_fb(const int *__restrict__ m_dev,
                                                                const float *__restrict__ img,
                                                                const float *__restrict__ g_sdf,
                                                                const float *__restrict__ feat, DwGrid g,
                                                                float *__restrict__ slabs, InterpFuse ip,
                                                                const float *__restrict__ h2,
                                                                const int *__restrict__ h2_src) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int64_t m = __builtin_amdgcn_readfirstlane(*m_dev);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t n_units = (m + kU - 1) / kU;
    const int64_t u0 = n_units * blockIdx.x / gridDim.x, u1 = n_units * (blockIdx.x + 1) / gridDim.x;
    const int n_rounds = (int)((u1 - u0 + 3) / 4);
    float *const h2set = lds + kT4H2, *const h1set = lds + kT4H1, *const cf = lds + kT4CF;
    auto xset = [&](int par) { return lds + kT4X + (par & 1) * 4 * 16 * kU; };
    stage8(lds, img + kImgVec, kVecPad, wave, lane);
    wait_vm(0);
    raw_barrier();
    const int b = blockIdx.x;
    const int i = lane & 31, h = lane >> 5;
    const int n = lane & 15, q = lane >> 4;
    const int sn = (n & 1) * 8 + (n >> 1);                     // the sample's slot in a unit image
    const int wb = 64 * q + ((((sn >> 2) ^ q) << 2) | (sn & 3));  // + 256 ob + 16 j
    const __amdgpu_buffer_rsrc_t wrs = rsrc_of(img, (int64_t)kImgTotal * 4);
    const bool fuse = ip.gx != nullptr;  // uniform
    [[maybe_unused]] constexpr int kStampK = 2;
    PSVO_STAMP_DECL;
    if (wave < 4) {
        // ================= chain wave c
        const int c = wave;
        f32x4v w1acc[8];  // dW1 partials of this wave's units: rows 16 t + 4 (lane >> 4) + j, column lane & 15
        zero4(w1acc);
        float b1p[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // b1 partials: rows 16 t + (lane & 15)
        int lf_n = 0, ro_n = 0;
        float ts_n = 0.f;
        {
            const int64_t u = u0 + c;
            const int64_t s = u * kU + n;
            if (fuse && u < u1 && s < m) {
                lf_n = ip.leaf[s];
                ro_n = ip.ray_of[s];
                ts_n = ip.t[s];
            }
        }
        for (int r = 0; r < n_rounds; ++r) {
            PSVO_STAMP(0);
            const int64_t u = u0 + 4 * (int64_t)r + c;
            const bool active = u < u1;  // wave-uniform
            const int64_t s = u * kU + n;
            const bool valid = active && s < m;
            const int lf = lf_n, ro = ro_n;
            const float ts = ts_n;
            int4 vid0 = make_int4(0, 0, 0, 0), vid1 = make_int4(0, 0, 0, 0);
            float cen[3] = {0.f, 0.f, 0.f};
            int row = 0;
            if (fuse && valid) {
                vid0 = *reinterpret_cast<const int4 *>(ip.vertex_idx + (int64_t)lf * 8);
                vid1 = *reinterpret_cast<const int4 *>(ip.vertex_idx + (int64_t)lf * 8 + 4);
#pragma unroll
                for (int a = 0; a < 3; ++a) cen[a] = ip.centres[(int64_t)lf * 3 + a];
                row = ip.rank_ray[ro];
            }
            raw_barrier();  // the round's forward (gradient waves) is in LDS
            PSVO_STAMP(1);
            // ---- P: δh1 = W2ᵀ δh2 ⊙ [h1 > 0] → LDS
            f32x4v fa[8];
            if (active) {
                f32x4v fb[8];
                lds_u_load<8>(h2set + c * kUImg, wb, fb);
                const uint64_t m1 = reinterpret_cast<const uint64_t *>(lds + kT4M)[c * 64 + lane];
                zero4(fa);
                gemm16<8, 8, 2>(wrs, kImgC2, fb, fa, lane);  // one ring over all 8 output blocks
                mask16(fa, m1);
                lds_u_store<8>(h1set + c * kUImg, wb, fa);
            }
            PSVO_STAMP(2);
            raw_barrier();
            PSVO_STAMP(3);
            // ---- Q: dfeat = W1ᵀ δh1 → the interpolation backward; the next unit's inputs
            if (r + 1 < n_rounds) {
                const int64_t un = u + 4;
                const int64_t snx = un * kU + n;
                if (fuse && un < u1 && snx < m) {
                    lf_n = ip.leaf[snx];
                    ro_n = ip.ray_of[snx];
                    ts_n = ip.t[snx];
                }
            }
            if (active) {
                f32x4v t1[1];
                zero4(t1);
                gemm16<8, 1, 4>(wrs, kImgC1, fa, t1, lane);
                // dW1 += δh1 ⊗ x of this unit (16 × 16 × 4 MFMAs over its 16 samples: lane (m, kq)
                // feeds slots 4 kq .. 4 kq + 3 of row 16 t + m, one 16-B chunk of each image)
                {
                    const int mr = lane & 15, kq = lane >> 4;
                    const float *dl = h1set + c * kUImg, *xl = xset(r) + c * 16 * kU;
                    const float4 bx = *reinterpret_cast<const float4 *>(xl + mr * kU + ((kq ^ ((mr >> 2) & 3)) << 2));
#pragma unroll
                    for (int t = 0; t < 8; ++t) {
                        const int rw = 16 * t + mr;
                        const float4 a = *reinterpret_cast<const float4 *>(dl + rw * kU + ((kq ^ ((rw >> 2) & 3)) << 2));
                        w1acc[t] = mfma16(a.x, bx.x, w1acc[t]);
                        w1acc[t] = mfma16(a.y, bx.y, w1acc[t]);
                        w1acc[t] = mfma16(a.z, bx.z, w1acc[t]);
                        w1acc[t] = mfma16(a.w, bx.w, w1acc[t]);
                        b1p[t] += (a.x + a.y) + (a.z + a.w);
                    }
                }
                PSVO_STAMP(4);
                const float4 gf = make_float4(t1[0][0], t1[0][1], t1[0][2], t1[0][3]);
                if (fuse) {
                    float ro3[3] = {0.f, 0.f, 0.f}, rd3[3] = {0.f, 0.f, 0.f};
                    float4 ev[8];
                    const int vid[8] = {vid0.x, vid0.y, vid0.z, vid0.w, vid1.x, vid1.y, vid1.z, vid1.w};
#pragma unroll
                    for (int k = 0; k < 8; ++k) ev[k] = reinterpret_cast<const float4 *>(ip.emb)[(int64_t)vid[k] * 4 + q];
                    if (valid) {
#pragma unroll
                        for (int a = 0; a < 3; ++a) {
                            ro3[a] = ip.rays_o[(int64_t)row * 3 + a];
                            rd3[a] = ip.rays_d[(int64_t)row * 3 + a];
                        }
                    }
                    interp_bwd_unit(ip, lds + kT4I + c * 512, m, s, valid, n, q, ts, ro3, rd3, cen, vid0, vid1, ev,
                                    gf);
                    PSVO_STAMP(5);
                    if (ip.grad_emb != nullptr) {
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the staging is this wave's own
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                        scatter_unit(ip, lds + kT4I + c * 512, u, m, lane, lf);
                    }
                }
            }
            PSVO_STAMP(6);
            PSVO_STAMP_FLUSH(0);
        }
        // this wave's dW1 / b1 partials → LDS (the CF tiles and mask words: read in P only)
        float *const pw = lds + kT4CF + c * 2048;
#pragma unroll
        for (int t = 0; t < 8; ++t)
#pragma unroll
            for (int j = 0; j < 4; ++j) pw[(16 * t + 4 * (lane >> 4) + j) * 16 + (lane & 15)] = w1acc[t][j];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            float v = b1p[t];
            v += __shfl_xor(v, 16, 64);
            v += __shfl_xor(v, 32, 64);
            if (lane < 16) lds[kT4M + c * 128 + 16 * t + lane] = v;
        }
    } else {
        // ================= gradient wave: column block d of W2, row block d of W1, the forward of unit d
        const int d = wave - 4;
        f32x16 acc2[kNB];
        zero(acc2);
        float b2p = 0.f, b30p = 0.f;
        float *const page3 = lds + kT4R + d * 132;   // W3 row 0 (+ b3[0]) partials of this wave's units
        if (lane < 33) *reinterpret_cast<float4 *>(page3 + 4 * lane) = make_float4(0.f, 0.f, 0.f, 0.f);
        TrunkIn nin;
        auto load_in = [&](int r) {
            const int64_t u = u0 + 4 * (int64_t)r + d;
            const int64_t s = u * kU + n;
            load_trunk_in(g_sdf, feat, H2 ? h2_src : nullptr, s, u < u1 && s < m, q, nin);
        };
        if (n_rounds > 0) {  // the forward of round 0
            load_in(0);
            const TrunkIn in = nin;
            if (n_rounds > 1) load_in(1);
            trunk_fwd_unit<H2>(lds, wrs, in, u0 + d, u1, m, d, lane, wb, xset(0) + d * 16 * kU, page3, b30p, h2);
        }
        for (int r = 0; r < n_rounds; ++r) {
            PSVO_STAMP(0);
            const int64_t ubase = u0 + 4 * (int64_t)r;
            raw_barrier();
            PSVO_STAMP(1);
            // P (beside the chain's W2ᵀ): dW2 += δh2 ⊗ h1 of this round
            dw_job_lds(h2set, cf, ubase, u1, d, lane, acc2, b2p);
            PSVO_STAMP(2);
            raw_barrier();
            PSVO_STAMP(3);
            // Q (beside the chain's interpolation backward): the next round's forward
            PSVO_STAMP(4);
            if (r + 1 < n_rounds) {
                const TrunkIn in = nin;
                if (r + 2 < n_rounds) load_in(r + 2);
                trunk_fwd_unit<H2>(lds, wrs, in, ubase + 4 + d, u1, m, d, lane, wb, xset(r + 1) + d * 16 * kU,
                                   page3, b30p, h2);
            }
            PSVO_STAMP(6);
            PSVO_STAMP_FLUSH(0);
        }
        // b3[0]: Σ dsdf (every sample's in each of the 4 q rows: row 0's)
        const float bs = row_sum16(b30p);
        if (lane == 0) page3[128] = bs;
        const int rb[kNB] = {0, 1, 2, 3}, cb[1] = {d};
        float *s2 = slabs + g.slab_off[1] + (int64_t)b * g.slab_len[1];
        {
            f32x16 t[kNB][1];
#pragma unroll
            for (int k = 0; k < kNB; ++k) t[k][0] = acc2[k];
            dw_store<kNB, 1, true>(s2, 128, 0, 128, rb, cb, t, lane);
        }
        const float v2 = b2p + __shfl_xor(b2p, 32, 64);
        if (h == 0) store_nt(s2, 128 * 128 + 32 * d + i, v2);
    }
    // W3 row 0 (+ b3[0]): the gradient waves' pages; W1 (+ b1): the chain
    // waves' partials — each summed in wave order
    __syncthreads();
    {
        float *s1 = slabs + g.slab_off[0] + (int64_t)b * g.slab_len[0];
        for (int e = threadIdx.x; e < 128 * 16 + 128; e += kF2Threads) {
            float v = 0.f;
            if (e < 128 * 16) {
#pragma unroll
                for (int k = 0; k < 4; ++k) v += lds[kT4CF + k * 2048 + e];
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) v += lds[kT4M + k * 128 + e - 128 * 16];
            }
            store_nt(s1, e, v);
        }
    }
    if (wave >= 4) {
        const int d = wave - 4;
        float *s3 = slabs + g.slab_off[2] + (int64_t)b * g.slab_len[2];
        if (h == 0) {
            float v = 0.f;
#pragma unroll
            for (int k = 0; k < 4; ++k) v += lds[kT4R + k * 132 + 32 * d + i];
            store_nt(s3, 32 * d + i, v);
        }
        if (d == 0 && lane == 0) {
            float v = 0.f;
#pragma unroll
            for (int k = 0; k < 4; ++k) v += lds[kT4R + k * 132 + 128];
            store_nt(s3, 129 * 128, v);
        }
    }
}

static int device_cus() {
    static int cus = 0;
    if (cus == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    return cus;
}

}  // namespace
}  // namespace psvo

#ifdef PSVO_STAMPS
// copies the stamp array ([3 kernels][256 wg][8 waves][8 tiles][16 points] u64)
extern "C" int psvo_debug_stamps(void *dst, int64_t bytes) {
    if (bytes < (int64_t)sizeof(psvo_g_stamps)) return -1;
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(psvo_g_stamps), sizeof(psvo_g_stamps)) == hipSuccess ? 0 : -2;
}
#endif

using namespace psvo;

extern "C" int64_t psvo_mlp_image_floats(void) { return kImgTotal; }

// width-aware sizes (width 128: the CF layout above; width 256: mlp256.hip)
extern "C" int64_t psvo_mlp_image_floats_w(int width) {
    return width == 128 ? kImgTotal : width == 256 ? dec256_image_floats() : -1;
}
extern "C" int64_t psvo_mlp_act_floats(int64_t m, int width) {
    const int64_t mp = (m + kCh - 1) / kCh * kCh;
    return width == 128 ? mp * 4 * 128 : width == 256 ? dec256_act_floats(m) : -1;
}
extern "C" int64_t psvo_mlp_mask_words(int64_t m, int width) {
    return width == 128 ? m * 6 : width == 256 ? dec256_mask_words(m) : -1;
}

static int mlp_fwd_impl(void *stream, int64_t m, int width, const float *feat, const float *w1, const float *b1,
                            const float *w2, const float *b2, const float *w3, const float *b3, const float *w4,
                            const float *b4, const float *w5, const float *b5, float *images, float *sdf, float *rgb,
                            float *act, uint64_t *masks, bool images_ready, const int *m_dev = nullptr,
                            const H2Rows *h2 = nullptr) {
    if (width == 256) {
        PSVO_REQUIRE(m >= 0, "mlp_fwd: m < 0");
        PSVO_REQUIRE(images != nullptr, "mlp_fwd: images workspace required (psvo_mlp_image_floats_w floats)");
        PSVO_REQUIRE(act == nullptr || masks != nullptr, "mlp_fwd: act needs masks");
        PSVO_REQUIRE(m <= ((int64_t)1 << 31) / 256, "mlp_fwd: m = %lld too large", (long long)m);
        hipStream_t st = as_stream(stream);
        if (!images_ready) {
            const int rc = dec256_images(st, w1, b1, w2, b2, w3, b3, w4, b4, w5, b5, images);
            if (rc) return rc;
        }
        return dec256_fwd(st, m, feat, images, sdf, rgb, act, masks, m_dev);
    }
    PSVO_REQUIRE(width == kW, "mlp_fwd: width %d unsupported (fused paths: 128, 256)", width);
    PSVO_REQUIRE(m >= 0, "mlp_fwd: m < 0");
    PSVO_REQUIRE(images != nullptr, "mlp_fwd: images workspace required (psvo_mlp_image_floats floats)");
    PSVO_REQUIRE(act == nullptr || masks != nullptr, "mlp_fwd: act needs masks");
    PSVO_REQUIRE(m <= kMaxSamples, "mlp_fwd: m = %lld > %lld (32-bit CF offsets)", (long long)m,
                 (long long)kMaxSamples);
    if (m == 0) return PSVO_OK;
    hipStream_t st = as_stream(stream);
    MlpParams p{w1, b1, w2, b2, w3, b3, w4, b4, w5, b5};
    if (!images_ready) psvo::launch(k_mlp_prep, dim3(div_up(kImgTotal, 256)), dim3(256), 0, st, p, images);
    if (rgb == nullptr) {  // sdf only (inference)
        PSVO_REQUIRE(act == nullptr && masks == nullptr, "mlp_fwd: the sdf-only forward is inference only");
        static bool attr_s = false;
        if (!attr_s) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_mlp_sdf2),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, kLdsSdf2);
            attr_s = true;
        }
        const int64_t tiles = div_up(m, kF2Tile);
        const int grid = (int)(tiles < device_cus() ? tiles : device_cus());
        psvo::launch(k_mlp_sdf2, dim3(grid), dim3(kF2Threads), kLdsSdf2, st, m, feat, images, sdf, m_dev,
                     h2 ? h2->out : nullptr);
        return check_launch("mlp_fwd");
    }
    static bool attr2 = false;
    if (!attr2) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_mlp_fwd2<false>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, kLdsFwd2);
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_mlp_fwd2<true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, kLdsFwd2);
        attr2 = true;
    }
    const int64_t tiles = div_up(m, kF2Tile);  // ≥ 8 units per workgroup
    const int grid = (int)(tiles < device_cus() ? tiles : device_cus());
    PSVO_REQUIRE(!h2 || !h2->rows || h2->src, "mlp_fwd: h2 rows need their source index");
    const bool h2r = h2 && h2->rows;
    psvo::launch(h2r ? k_mlp_fwd2<true> : k_mlp_fwd2<false>, dim3(grid), dim3(kF2Threads), kLdsFwd2, st, m, feat,
                 images, sdf, rgb, act, masks, m_dev, h2r ? h2->rows : nullptr, h2r ? h2->src : nullptr);
    return check_launch("mlp_fwd");
}

namespace psvo {
int mlp_images(void *stream, int width, const float *w1, const float *b1, const float *w2, const float *b2,
               const float *w3, const float *b3, const float *w4, const float *b4, const float *w5, const float *b5,
               float *images) {
    if (width == 256) return dec256_images(as_stream(stream), w1, b1, w2, b2, w3, b3, w4, b4, w5, b5, images);
    MlpParams p{w1, b1, w2, b2, w3, b3, w4, b4, w5, b5};
    psvo::launch(k_mlp_prep, dim3(div_up(kImgTotal, 256)), dim3(256), 0, as_stream(stream), p, images);
    return check_launch("mlp_images");
}
int mlp_fwd_prepared(void *stream, int64_t m, int width, const float *feat, const float *w1, const float *b1,
                     const float *w2, const float *b2, const float *w3, const float *b3, const float *w4,
                     const float *b4, const float *w5, const float *b5, float *images, float *sdf, float *rgb,
                     float *act, uint64_t *masks, const int *m_dev, const H2Rows *h2) {
    return mlp_fwd_impl(stream, m, width, feat, w1, b1, w2, b2, w3, b3, w4, b4, w5, b5, images, sdf, rgb, act, masks,
                        true, m_dev, h2);
}
}  // namespace psvo

extern "C" int psvo_mlp_fwd(void *stream, int64_t m, int width, const float *feat, const float *w1, const float *b1,
                            const float *w2, const float *b2, const float *w3, const float *b3, const float *w4,
                            const float *b4, const float *w5, const float *b5, float *images, float *sdf, float *rgb,
                            float *act, uint64_t *masks) {
    return mlp_fwd_impl(stream, m, width, feat, w1, b1, w2, b2, w3, b3, w4, b4, w5, b5, images, sdf, rgb, act, masks,
                        false);
}

static const int kDwRows[5] = {128, 128, 129, 128, 3};
static const int kDwCols[5] = {16, 128, 128, 144, 128};
// k_mlp_bwd3: one workgroup per CU (at most one per round of 4 units), each
// writing a slab of every layer
static int bwd3_grid(int64_t m) {
    const int64_t rounds = (m + 4 * kU - 1) / (4 * kU);
    return (int)(rounds < device_cus() ? (rounds > 0 ? rounds : 1) : device_cus());
}
static void dw_grid_uniform(int n, DwGrid *g, int *slab_floats) {
    int off = 0;
    for (int l = 0; l < 5; ++l) {
        g->n_split[l] = n;
        g->slab_off[l] = off;
        g->slab_len[l] = kDwRows[l] * kDwCols[l] + kDwRows[l];
        off += n * g->slab_len[l];
    }
    *slab_floats = off;
}

extern "C" int64_t psvo_mlp_workspace_floats_w(int64_t m, int width, int n_split);

extern "C" int64_t psvo_mlp_workspace_floats(int64_t m, int n_split) {
    (void)n_split;  // k_mlp_bwd3 writes one slab per workgroup
    DwGrid g;
    int slab;
    dw_grid_uniform(bwd3_grid(m), &g, &slab);
    return m * 3 + 2 * (int64_t)slab;  // k_mlp_bwd3's slabs, then k_mlp_trunk_fb's (the sparse decoder's class B)
}

extern "C" int64_t psvo_mlp_workspace_floats_w(int64_t m, int width, int n_split) {
    return width == 128 ? psvo_mlp_workspace_floats(m, n_split) : width == 256 ? dec256_workspace_floats(m) : -1;
}

// Full decoder backward: grads of the 10 parameters (overwritten, or added
// to when `accumulate`) and dfeat [M,16], from the training forward's rgb,
// activations and masks.  `workspace`: δ operands + split-K slabs
// (psvo_mlp_workspace_floats).
namespace psvo {
int mlp_bwd(void *stream, int64_t m, int width, const float *feat, const float *w1, const float *b1, const float *w2,
            const float *b2, const float *w3, const float *b3, const float *w4, const float *b4, const float *w5,
            const float *b5, const float *images, const float *rgb, const float *act, const uint64_t *masks,
            const float *g_sdf, const float *g_rgb, float *dfeat, float *gw1, float *gb1, float *gw2, float *gb2,
            float *gw3, float *gb3, float *gw4, float *gb4, float *gw5, float *gb5, int accumulate, int n_split,
            float *workspace, hipEvent_t dfeat_ready, const InterpFuse *ip, hipStream_t reduce_stream,
            const int *m_dev, const TrunkBwd *tb, const int *x_src) {
    PSVO_REQUIRE(ip == nullptr || ((width == 256 || width == kW) && gw1 != nullptr),
                 "mlp_bwd: the fused interpolation backward needs a fused weight-gradient path");
    if (width == 256) {
        PSVO_REQUIRE(m >= 0, "mlp_bwd: bad sizes");
        PSVO_REQUIRE(images != nullptr && masks != nullptr, "mlp_bwd: images / masks of the training forward required");
        PSVO_REQUIRE(gw1 == nullptr || act != nullptr, "mlp_bwd: weight gradients need the forward's activations");
        float *gw[5] = {gw1, gw2, gw3, gw4, gw5}, *gb[5] = {gb1, gb2, gb3, gb4, gb5};
        return dec256_bwd(as_stream(stream), m, feat, images, rgb, act, masks, g_sdf, g_rgb, dfeat, gw, gb, accumulate,
                          workspace, dfeat_ready, ip, m_dev);
    }
    PSVO_REQUIRE(width == kW, "mlp_bwd: width %d unsupported (fused paths: 128, 256)", width);
    PSVO_REQUIRE(m >= 0 && n_split > 0, "mlp_bwd: bad sizes");
    PSVO_REQUIRE(images != nullptr, "mlp_bwd: images of the training forward required");
    const bool want_w = gw1 != nullptr;  // NULL weight gradients: δ chain / dfeat only (frozen decoder)
    PSVO_REQUIRE(!want_w || act != nullptr, "mlp_bwd: weight gradients need the forward's activations");
    hipStream_t st = as_stream(stream);
    DwGrid g;
    int slab_floats;
    float *gw[5] = {gw1, gw2, gw3, gw4, gw5}, *gb[5] = {gb1, gb2, gb3, gb4, gb5};
    PSVO_REQUIRE(tb == nullptr || (gw1 != nullptr && tb->m_dev && tb->g_sdf && tb->feat),
                 "mlp_bwd: the trunk backward needs the weight-gradient path and its inputs");
    float *slabs_b = nullptr;
    auto reduce = [&](float *slabs, hipStream_t rs) {
        DwDst d;
        int e = 0;
        for (int l = 0; l < 5; ++l) {
            d.w[l] = gw[l];
            d.b[l] = gb[l];
            d.rows[l] = kDwRows[l];
            d.cols[l] = kDwCols[l];
            d.elem_begin[l] = e;
            e += kDwRows[l] * kDwCols[l] + kDwRows[l];
        }
        d.elem_begin[5] = e;
        psvo::launch(k_mlp_dw_reduce, dim3(div_up(e, kDwRedEl)), dim3(256), 0, rs, g, slabs, d, accumulate,
                     static_cast<const float *>(slabs_b));
        return check_launch("mlp_dw_reduce");
    };
    {  // fused δ chain + weight gradients (or the chain alone: frozen decoder)
        static bool attr3 = false;
        if (!attr3) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_mlp_bwd3<true>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBwd3);
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_mlp_bwd3<false>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBwd3);
            attr3 = true;
        }
        Bwd3Src src{rgb, g_sdf, g_rgb, feat, masks, act, dfeat, x_src};
        if (!want_w) {
            if (m > 0) {
                const int64_t rounds = div_up(div_up(m, kU), 8);
                const int grid = (int)(rounds < device_cus() ? rounds : device_cus());
                psvo::launch(k_mlp_bwd3<false>, dim3(grid), dim3(kF2Threads), kLdsBwd3, st, m, images, src, g,
                             nullptr, InterpFuse{}, m_dev);
                const int rc = check_launch("mlp_bwd3");
                if (rc) return rc;
            }
            if (dfeat_ready && hipEventRecord(dfeat_ready, st) != hipSuccess)
                return set_error(PSVO_E_LAUNCH, "mlp_bwd: event record failed");
            return PSVO_OK;
        }
        const int grid = bwd3_grid(m);
        dw_grid_uniform(grid, &g, &slab_floats);
        float *slabs = workspace + m * 3;
        // dfeat_ready marks the last kernel's completion through its dispatch
        // (psvo::launch's stop event): no marker packet between the decoder's
        // backward and the per-ray sums that follow it on st
        static const bool bind_env = [] {
            const char *v = getenv("PSVO_BIND_DFEAT");
            return !(v && v[0] == '0');
        }();
        const bool trunk_last = tb && m > 0;
        bool bound = false;
        auto bind = [&](bool last) {
            if (last && bind_env && dfeat_ready) psvo::g_stop_event = dfeat_ready;
        };
        auto taken = [&](bool last) {
            if (last && bind_env && dfeat_ready) {
                bound = psvo::g_stop_event == nullptr;
                psvo::g_stop_event = nullptr;
            }
        };
        if (m > 0) {
            bind(!trunk_last);
            psvo::launch(k_mlp_bwd3<true>, dim3(grid), dim3(kF2Threads), kLdsBwd3, st, m, images, src, g, slabs,
                         ip ? *ip : InterpFuse{}, m_dev);
            taken(!trunk_last);
            const int rc = check_launch("mlp_bwd3");
            if (rc) return rc;
        } else if (hipMemsetAsync(slabs, 0, (size_t)slab_floats * sizeof(float), st) != hipSuccess) {
            return set_error(PSVO_E_LAUNCH, "mlp_bwd: memset failed");
        }
        if (tb && m > 0) {  // the sparse decoder's class B: the trunk forward + backward, its own slabs
            static bool attr_t = false;
            if (!attr_t) {
                (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_mlp_trunk_fb<true>),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, kLdsTrunk);
                (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_mlp_trunk_fb<false>),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, kLdsTrunk);
                attr_t = true;
            }
            slabs_b = slabs + slab_floats;
            PSVO_REQUIRE(!tb->h2 || tb->src, "mlp_bwd: the trunk's h2 rows need their source index");
            bind(true);
            psvo::launch(tb->h2 ? k_mlp_trunk_fb<true> : k_mlp_trunk_fb<false>, dim3(grid), dim3(kF2Threads), kLdsTrunk,
                         st, tb->m_dev, images, tb->g_sdf, tb->feat, g, slabs_b, tb->ip ? *tb->ip : InterpFuse{},
                         tb->h2, tb->src);
            taken(true);
            const int rc = check_launch("mlp_trunk_fb");
            if (rc) return rc;
        }
        if (dfeat_ready && !bound && hipEventRecord(dfeat_ready, st) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "mlp_bwd: event record failed");
        if (reduce_stream && reduce_stream != st) {  // the slab sum beside the caller's next work on st
            PSVO_REQUIRE(dfeat_ready != nullptr, "mlp_bwd: a separate reduce stream needs the dfeat_ready event");
            if (hipStreamWaitEvent(reduce_stream, dfeat_ready, 0) != hipSuccess)
                return set_error(PSVO_E_LAUNCH, "mlp_bwd: stream wait failed");
            return reduce(slabs, reduce_stream);
        }
        return reduce(slabs, st);
    }
}
}  // namespace psvo

namespace psvo {
// width 128: the interpolation backward runs inside k_mlp_bwd3; width 256:
// k_interp_bwd beside the weight-gradient kernel (measured faster than inside
// k_dec256_bwd: there the scatter's atomics overlap the dW MFMAs)
bool mlp_bwd_fuses_interp(int width) { return width == kW; }
bool mlp_bwd_split_tail(int width) { return width == kW; }
}  // namespace psvo

extern "C" int psvo_mlp_bwd(void *stream, int64_t m, int width, const float *feat, const float *w1, const float *b1,
                            const float *w2, const float *b2, const float *w3, const float *b3, const float *w4,
                            const float *b4, const float *w5, const float *b5, const float *images, const float *rgb,
                            const float *act, const uint64_t *masks, const float *g_sdf, const float *g_rgb, float *dfeat, float *gw1,
                            float *gb1, float *gw2, float *gb2, float *gw3, float *gb3, float *gw4, float *gb4,
                            float *gw5, float *gb5, int accumulate, int n_split, float *workspace) {
    return psvo::mlp_bwd(stream, m, width, feat, w1, b1, w2, b2, w3, b3, w4, b4, w5, b5, images, rgb, act, masks,
                         g_sdf, g_rgb, dfeat, gw1, gb1, gw2, gb2, gw3, gb3, gw4, gb4, gw5, gb5, accumulate, n_split,
                         workspace, nullptr);
}
