// NRGBD decoder at width 256 (src/variations/nrgbd.py:80-146, depth 2, input
// 16, sdf_dim 128, embedder 'none': configs/scannet/scannet.yaml:17 and
// configs/arkit/arkit.yaml:17) as fused fp32-MFMA kernels for gfx950.
//
//   h1 = relu(W1 x + b1)       W1 [256,16]      4,096 MAC / sample
//   h2 = relu(W2 h1 + b2)      W2 [256,256]    65,536
//   o  = W3 h2 + b3 = [sdf|f]  W3 [129,256]    33,024
//   c1 = relu(W4 [f; x] + b4)  W4 [256,144]    36,864
//   rgb = sigmoid(W5 c1 + b5)  W5 [3,256]         768
//
// Chain layout (v_mfma_f32_16x16x4_f32): a wave owns 16 samples; an
// activation of F features is F/16 blocks, each one f32x4 per lane in the
// MFMA accumulator form — lane l holds features 16b + 4(l>>4) + i (i = 0..3)
// of sample l&15 — and register i of block b is directly the B operand of
// the next layer's k-step (b, i) (k index l>>4 ↔ feature 16b + 4(l>>4) + i).
// The weights are the A operand, read from LDS in an image permuted to match:
// image[ib][ob][lane][i] = W[16ob + (l&15)][16ib + 4(l>>4) + i], one
// ds_read_b128 per 4 MFMAs.  W2 alone is 256 KB, so every layer's image
// streams through LDS in K-chunks (a few input blocks, ≤ 32 KB) in a ring of
// three buffers, two chunks in flight (global_load_lds), one barrier per
// chunk; the fwd / bwd kernels are persistent (one 8-wave workgroup per CU
// loops over 128-sample tiles) and the ring runs on across tiles.
//
// The weight gradients are split-K GEMMs over 16-sample tiles of stored
// activations and δ's: tile-feature-major [tile][F][16] with the 16-B groups
// of a row XOR-swizzled by a function of (row >> 2) & 3, which is the dW kernel's LDS
// operand image (conflict-free ds_read_b128 of 4 samples = 4 k-steps), so a
// tile lands by straight 1-KB copies.  Samples past M are zero inputs with
// zero gradients: they add nothing.
//
// fp32 in, fp32 accumulate: every product is an exact-f32 fmaf step (no
// TF32-like rounding), the numerics class of the reference's torch.float32.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "interp_fuse.h"
#include "psvo_common.h"

namespace psvo {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 8, kThreads = 64 * kWaves;
constexpr int kTileW = 16;                 // samples per wave
constexpr int kTileWG = kWaves * kTileW;   // samples per workgroup iteration
// The weight images stream through LDS in chunks of kIbPer input blocks
// (all of a layer's output blocks): 4 input blocks = 64 KB chunks in a ring
// of 2 (13 chunks, i.e. 13 workgroup barriers per tile); PSVO_DEC256_IBPER=2:
// 32 KB chunks in a ring of 3 (23 chunks), the earlier layout, for A/B.
#ifndef PSVO_DEC256_IBPER
#define PSVO_DEC256_IBPER 4
#endif
constexpr int kIbPer = PSVO_DEC256_IBPER;
static_assert(kIbPer == 2 || kIbPer == 4, "chunk width");
constexpr int kChunkFloats = kIbPer * 16 * 256;  // a chunk of the widest layer (16 output blocks)
constexpr int kRing = kIbPer == 4 ? 2 : 3;

// ---- weight images (floats) ----------------------------------------------
// forward: L1 [1][16], L2 [16][16], L3 [16][9], L4 [9][16], L5 [16][1]  ([ib][ob] blocks of 256 floats)
// backward: W5ᵀ [1][16], W4ᵀ [16][9], W3ᵀ [9][16], W2ᵀ [16][16], W1ᵀ [16][1]
constexpr int kBlk = 256;  // floats per (ib, ob) block: 64 lanes x 4
struct Img {
    int nib, nob, off;  // off in floats
};
constexpr Img kF1{1, 16, 0};
constexpr Img kF2{16, 16, kF1.off + 1 * 16 * kBlk};
constexpr Img kF3{16, 9, kF2.off + 16 * 16 * kBlk};
constexpr Img kF4{9, 16, kF3.off + 16 * 9 * kBlk};
constexpr Img kF5{16, 1, kF4.off + 9 * 16 * kBlk};
constexpr Img kB5{1, 16, kF5.off + 16 * 1 * kBlk};
constexpr Img kB4{16, 9, kB5.off + 1 * 16 * kBlk};
constexpr Img kB3{9, 16, kB4.off + 16 * 9 * kBlk};
constexpr Img kB2{16, 16, kB3.off + 9 * 16 * kBlk};
constexpr Img kB1{16, 1, kB2.off + 16 * 16 * kBlk};
// the sdf row alone (W3 row 0 as one output block: the same values as row 128
// of kF3's block 8), for the sdf trunk (k_dec256_trunk)
constexpr Img kS3{16, 1, kB1.off + 16 * 1 * kBlk};
constexpr int kImgMats = kS3.off + 16 * 1 * kBlk;
// bias vectors (forward order of the chain: b3 as [f rows | sdf | 0 pad], b5 padded to 16)
constexpr int kVB1 = 0, kVB2 = 256, kVB3 = 512, kVB4 = 512 + 144, kVB5 = kVB4 + 256, kVecN = kVB5 + 16;
constexpr int kImgTotal = kImgMats + kVecN;

// chunk plan of a program: chunk c covers input blocks [ib0, ib0 + nib) of image `img`
struct Chunk {
    int img_off, nob, ib0, nib;
};
__host__ __device__ constexpr Chunk chunk_of(Img im, int ib0, int nib) { return {im.off + ib0 * im.nob * kBlk, im.nob, ib0, nib}; }
__host__ __device__ constexpr int chunk_floats(Chunk c) { return c.nib * c.nob * kBlk; }

// chunks per layer: ceil(input blocks / kIbPer); L1 and L5 (one output /
// input block row) are one chunk each
constexpr int chunks_of(int nib) { return (nib + kIbPer - 1) / kIbPer; }
constexpr int kN16 = chunks_of(16), kN9 = chunks_of(9);
// forward: L1 | L2 (kN16) | L3 (kN16) | L4 (kN9) | L5
constexpr int kFwdL2 = 1, kFwdL3 = kFwdL2 + kN16, kFwdL4 = kFwdL3 + kN16, kFwdL5 = kFwdL4 + kN9,
              kFwdChunks = kFwdL5 + 1;
__host__ __device__ constexpr Chunk layer_chunk(Img im, int j) {
    return chunk_of(im, kIbPer * j, im.nib - kIbPer * j < kIbPer ? im.nib - kIbPer * j : kIbPer);
}
__host__ __device__ constexpr Chunk fwd_chunk(int c) {
    return c == 0         ? chunk_of(kF1, 0, 1)
           : c < kFwdL3   ? layer_chunk(kF2, c - kFwdL2)
           : c < kFwdL4   ? layer_chunk(kF3, c - kFwdL3)
           : c < kFwdL5   ? layer_chunk(kF4, c - kFwdL4)
                          : chunk_of(kF5, 0, 16);
}
// backward (data): W5ᵀ | W4ᵀ (kN16) | W3ᵀ (kN9) | W2ᵀ (kN16) | W1ᵀ
constexpr int kBwdL4 = 1, kBwdL3 = kBwdL4 + kN16, kBwdL2 = kBwdL3 + kN9, kBwdL1 = kBwdL2 + kN16,
              kBwdChunks = kBwdL1 + 1;
// the sdf trunk: L1 | L2 (kN16) | the sdf row
constexpr int kTrkL2 = 1, kTrkS3 = kTrkL2 + kN16, kTrkChunks = kTrkS3 + 1;
__host__ __device__ constexpr Chunk trunk_chunk(int c) {
    return c == 0 ? chunk_of(kF1, 0, 1) : c < kTrkS3 ? layer_chunk(kF2, c - kTrkL2) : chunk_of(kS3, 0, 16);
}
__host__ __device__ constexpr Chunk bwd_chunk(int c) {
    return c == 0         ? chunk_of(kB5, 0, 1)
           : c < kBwdL3   ? layer_chunk(kB4, c - kBwdL4)
           : c < kBwdL2   ? layer_chunk(kB3, c - kBwdL3)
           : c < kBwdL1   ? layer_chunk(kB2, c - kBwdL2)
                          : chunk_of(kB1, 0, 16);
}
static_assert(chunk_floats(chunk_of(kF5, 0, 16)) <= kChunkFloats && chunk_floats(chunk_of(kB1, 0, 16)) <= kChunkFloats,
              "one-chunk layers fit a ring buffer");

// effective (out x in) matrices of the images, from the torch parameters
struct Params {
    const float *w1, *b1, *w2, *b2, *w3, *b3, *w4, *b4, *w5, *b5;
};
__device__ float mat_at(const Params &p, int which, int o, int j) {
    switch (which) {
        case 0: return p.w1[o * 16 + j];                                               // W1   [256][16]
        case 1: return p.w2[o * 256 + j];                                              // W2   [256][256]
        case 2: return o < 128 ? p.w3[(o + 1) * 256 + j] : o == 128 ? p.w3[j] : 0.0f;  // [f rows; sdf; 0] x 256
        case 3: return p.w4[o * 144 + j];                                              // W4   [256][144]
        case 4: return o < 3 ? p.w5[o * 256 + j] : 0.0f;                               // W5 padded to 16 rows
        case 5: return j < 3 ? p.w5[j * 256 + o] : 0.0f;                               // W5ᵀ  [256][16 (3)]
        case 6: return p.w4[j * 144 + o];                                              // W4ᵀ  [144][256]
        case 7: return j < 128 ? p.w3[(j + 1) * 256 + o] : j == 128 ? p.w3[o] : 0.0f;  // W3ᵀ  [256][144]
        case 8: return p.w2[j * 256 + o];                                              // W2ᵀ
        case 9: return p.w1[j * 16 + o];                                               // W1ᵀ  [16][256]
        default: return o == 0 ? p.w3[j] : 0.0f;                                       // the sdf row [1 (16)][256]
    }
}

// one launch builds every image + the bias vectors (once per weight update)
__global__ __launch_bounds__(256) void k_dec256_prep(Params p, float *__restrict__ img) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= kImgTotal) return;
    if (e >= kImgMats) {
        const int v = e - kImgMats;
        float x;
        if (v < kVB2) x = p.b1[v];
        else if (v < kVB3) x = p.b2[v - kVB2];
        else if (v < kVB4) {
            const int r = v - kVB3;
            x = r < 128 ? p.b3[r + 1] : r == 128 ? p.b3[0] : 0.0f;
        } else if (v < kVB5) x = p.b4[v - kVB4];
        else x = (v - kVB5) < 3 ? p.b5[v - kVB5] : 0.0f;
        img[e] = x;
        return;
    }
    const Img ims[11] = {kF1, kF2, kF3, kF4, kF5, kB5, kB4, kB3, kB2, kB1, kS3};
    int which = 0;
    for (int k = 1; k < 11; ++k)
        if (e >= ims[k].off) which = k;
    const Img im = ims[which];
    const int r = e - im.off;
    const int i = r & 3, lane = (r >> 2) & 63, blk = r >> 8;
    const int ob = blk % im.nob, ib = blk / im.nob;
    const int o = 16 * ob + (lane & 15), j = 16 * ib + 4 * (lane >> 4) + i;
    img[e] = mat_at(p, which, o, j);  // fwd images 0..4, bwd 5..9, the sdf row 10
}

// ---- device helpers ------------------------------------------------------
__device__ __forceinline__ uint32_t lds_addr(const float *l) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float *)l;
}
// global → LDS 16 B per lane (LDS destination = wave-uniform base + lane x 16)
__device__ __forceinline__ void glds16(const float *g, float *l) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds_addr(l)))
                 : "memory");
}
// s_waitcnt vmcnt(N) lgkmcnt(0) (expcnt untouched); N < 64
template <int N>
__device__ __forceinline__ void wait_vm_lds() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70);
    asm volatile("" ::: "memory");
}
// all of this wave's global loads / stores and LDS ops done, then the workgroup barrier
__device__ __forceinline__ void chunk_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}
// the same with a uniform (SGPR) base and a 32-bit per-lane byte offset
__device__ __forceinline__ void glds16s(const float *base, uint32_t voff, float *l) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(base), "s"(__builtin_amdgcn_readfirstlane(lds_addr(l)))
                 : "memory");
}
// copy `floats` (multiple of 256) from global to an LDS buffer, spread over the
// NW waves.  The per-lane offset is made opaque here so that the compiler does
// not hoist one 64-bit address per chunk out of the tile loop (they spilled).
template <int NW>
__device__ __forceinline__ void stream_chunk(const float *__restrict__ src, float *dst, int floats, int wave,
                                             int lane) {
    uint32_t voff = (uint32_t)(wave * 256 + lane * 4) * 4u;
    asm volatile("" : "+v"(voff));
    for (int o = wave * 256; o < floats; o += NW * 256, voff += NW * 1024) glds16s(src, voff, dst + o);
}

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// The chain kernels: 8 waves (two per SIMD, ≤ 256 registers each), a wave
// owns NC = 1 group of 16 samples; every A operand (one ds_read_b128 = 4
// k-steps of one output block) feeds 4 x NC MFMAs.  Two waves per SIMD keep
// the MFMA pipe busy across one wave's barrier waits, ReLU passes and stores
// (4 waves x 2 groups, 512 registers each: fwd 1,309 -> 1,264 us, bwd 1,263
// -> 1,198 us at config C's 466 k samples; -DPSVO_DEC256_WAVES=4
// -DPSVO_DEC256_NC=2 builds that layout for A/B).
#ifndef PSVO_DEC256_NC
#define PSVO_DEC256_NC 1
#endif
#ifndef PSVO_DEC256_WAVES
#define PSVO_DEC256_WAVES 8
#endif
constexpr int kCWaves = PSVO_DEC256_WAVES, kCThreads = 64 * kCWaves, kNC = PSVO_DEC256_NC;
constexpr int kChainTile = kCWaves * kNC * kTileW;  // samples per chain-kernel workgroup iteration
static_assert(kTileWG % kChainTile == 0, "chain tile");

// acc[c][ob] += W(chunk: input blocks IB0.., NOB output blocks) · in[c][IB0 + ib]
// A operands in groups of up to 4 output blocks, read one group ahead; the
// schedule is pinned per group (left free, the compiler hoists every read of
// a chunk to its top); inside a group the MFMAs rotate over 4 x NC
// accumulators, so no two consecutive MFMAs share one.
template <int NOB, int NIN, int IB0, int NIB>
__device__ __forceinline__ void gemm_chunk(f32x4 (&acc)[kNC][NOB], const f32x4 (&in)[kNC][NIN], const float *buf,
                                           int lane, bool on = true) {
    static_assert(IB0 + NIB <= NIN, "chunk input blocks");
    if (!on) return;  // wave-uniform: a wave without samples in the last round
    constexpr int NG = (NOB + 3) / 4;
    constexpr int NSTEP = NIB * NG;
    f32x4 a[2][4];
    auto load = [&](int s, f32x4(&dst)[4]) {
        const int ib = s / NG, g = s % NG;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (4 * g + j < NOB) dst[j] = *reinterpret_cast<const f32x4 *>(buf + ((ib * NOB + 4 * g + j) * 64 + lane) * 4);
    };
    load(0, a[0]);
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) {
        __builtin_amdgcn_sched_barrier(0);
        if (s + 1 < NSTEP) load(s + 1, a[(s + 1) & 1]);
        const int ib = s / NG, g = s % NG;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int c = 0; c < kNC; ++c)
                    if (4 * g + j < NOB) acc[c][4 * g + j] = mfma(a[s & 1][j][i], in[c][IB0 + ib][i], acc[c][4 * g + j]);
    }
    __builtin_amdgcn_sched_barrier(0);
}

// bias image → accumulator init (lane holds features 16 ob + 4(l>>4) + i)
template <int NOB>
__device__ __forceinline__ void init_bias(f32x4 (&acc)[kNC][NOB], const float *vec, int lane) {
#pragma unroll
    for (int ob = 0; ob < NOB; ++ob) {
        const f32x4 b = *reinterpret_cast<const f32x4 *>(vec + 16 * ob + 4 * (lane >> 4));
#pragma unroll
        for (int c = 0; c < kNC; ++c) acc[c][ob] = b;
    }
}
template <int NOB>
__device__ __forceinline__ void zero(f32x4 (&acc)[kNC][NOB]) {
#pragma unroll
    for (int c = 0; c < kNC; ++c)
#pragma unroll
        for (int ob = 0; ob < NOB; ++ob) acc[c][ob] = f32x4{0.f, 0.f, 0.f, 0.f};
}
// ReLU in place; mask bit 4 ob + i = (value > 0), one word per sample group.
// No compares (mlp.hip's relu): y = max(v, 0) and (−u) & ~u (u = bits of y)
// has its sign bit set exactly for positive non-zero y — per-element compare
// results held as SGPR-pair lane masks spilled ~730 SGPRs to VGPR lanes here
// (v_writelane / v_readlane in the tile loop).
template <int NOB>
__device__ __forceinline__ void relu_mask(f32x4 (&acc)[kNC][NOB], uint64_t (&m)[kNC]) {
#pragma unroll
    for (int c = 0; c < kNC; ++c) {
        uint32_t half[2] = {0u, 0u};
#pragma unroll
        for (int ob = 0; ob < NOB; ++ob)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float y = acc[c][ob][i];
                asm volatile("" : "+v"(y));  // in program order: not all hoisted and kept live at once
                y = fmaxf(y, 0.0f);
                acc[c][ob][i] = y;
                const uint32_t u = __float_as_uint(y);
                const int bit = 4 * ob + i;
                half[bit >> 5] |= (((0u - u) & ~u) >> 31) << (bit & 31);
                asm volatile("" : "+v"(half[bit >> 5]));
            }
        m[c] = (uint64_t)half[0] | ((uint64_t)half[1] << 32);
    }
}
template <int NOB>
__device__ __forceinline__ void apply_mask(f32x4 (&acc)[kNC][NOB], const uint64_t (&m)[kNC]) {
#pragma unroll
    for (int c = 0; c < kNC; ++c) {
        const uint32_t half[2] = {(uint32_t)m[c], (uint32_t)(m[c] >> 32)};
#pragma unroll
        for (int ob = 0; ob < NOB; ++ob)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int bit = 4 * ob + i;
                const uint32_t keep = 0u - ((half[bit >> 5] >> (bit & 31)) & 1u);
                acc[c][ob][i] = __uint_as_float(__float_as_uint(acc[c][ob][i]) & keep);
            }
    }
}

// tile-feature-major store: feature f of sample n at f·16 + swz(f, n) in a
// 16-sample tile of a matrix with F rows (F·16 floats per tile).  For
// f = 16 ob + 4 g + i, (f >> 2) & 3 = g: the lane's offset within a 16-row
// block is one value, 64 g + swz; the rest are immediates.
// The 16-B group of samples 4q..4q+3 in row f sits at q ^ hsw((f >> 2) & 3):
// with hsw = {0, 2, 3, 1}, the dW kernel's ds_read_b128 (lane l: row
// 16 mb + (l & 15), group l >> 4) hits 16 distinct 16-B slots in each of
// ds_read_b128's four lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ...
// (MI355X_MICROARCH.md §LDS); the plain (f >> 2) & 3 left them 2-way.
__device__ __forceinline__ int hsw(int q) { return (0x78 >> (2 * q)) & 3; }
__device__ __forceinline__ int swz(int f, int n) { return ((((n >> 2) ^ hsw((f >> 2) & 3))) << 2) | (n & 3); }
template <int NOB>
__device__ __forceinline__ void store_tiles(float *__restrict__ mat, int64_t t16_0, int rows,
                                            const f32x4 (&acc)[kNC][NOB], int lane) {
    int off = 64 * (lane >> 4) + swz(4 * (lane >> 4), lane & 15);
    asm volatile("" : "+v"(off));  // keep the per-(ob, i) addresses from being hoisted out of the tile loop
#pragma unroll
    for (int c = 0; c < kNC; ++c) {
        float *p = mat + (t16_0 + c) * rows * 16 + off;
#pragma unroll
        for (int ob = 0; ob < NOB; ++ob)
#pragma unroll
            for (int i = 0; i < 4; ++i) __builtin_nontemporal_store(acc[c][ob][i], p + 256 * ob + 16 * i);
    }
}

__device__ __forceinline__ float sigmoidf(float x) { return 1.0f / (1.0f + expf(-x)); }

// per-tile activation / mask layout (act, masks)
struct Act {
    float *h1, *h2, *fx, *c1;  // [T16][F][16], F = 256, 256, 144, 256
    uint64_t *masks;           // [T16][3][64]  (h1, h2, c1)
};
struct Dlt {
    float *d1, *d2, *d3, *d4, *d5;  // δh1 [256], δh2 [256], [δf; g_sdf] [144], δc1 [256], δ5 [16] tiles
};

// The program's chunks run in order per tile.  Ring of 3: at chunk k the
// ring holds chunks k, k+1 and chunk k+2 is issued; ring of 2: chunk k+1 is
// issued into the buffer chunk k−1 held.  Either way the barrier first waits
// for every outstanding copy (vmcnt(0)), so a chunk lands while the one
// before it is computed; the next tile's first chunks are issued at the end
// of a tile.
struct Ring {
    float *ring;
    const float *img;
    int slot, wave, lane;
    bool more;
    template <int NCH, typename Plan>
    __device__ __forceinline__ const float *next(int k, Plan plan) {
        chunk_barrier();
        constexpr int kAhead = kRing - 1;
        const int k2 = k + kAhead;
        if (k2 < NCH || more) {
            const Chunk c = plan(k2 < NCH ? k2 : k2 - NCH);
            const float *src = img;
            asm volatile("" : "+s"(src));  // the chunk address is formed here, not hoisted (SGPR spills)
            stream_chunk<kCWaves>(src + c.img_off, ring + ((slot + kAhead) % kRing) * kChunkFloats, chunk_floats(c),
                                  wave, lane);
        }
        const float *b = ring + slot * kChunkFloats;
        slot = (slot + 1) % kRing;
        return b;
    }
    // the first kRing − 1 chunks of a program, before its first tile
    template <typename Plan>
    __device__ __forceinline__ void prime(Plan plan) {
#pragma unroll
        for (int c = 0; c < kRing - 1; ++c)
            stream_chunk<kCWaves>(img + plan(c).img_off, ring + c * kChunkFloats, chunk_floats(plan(c)), wave, lane);
    }
};

// chunks [C0, C0 + N) of one layer: input blocks [kIbPer·j, …) of `in` into `acc`
template <int NCH, int C0, int J, int N, int NOB, int NIN, typename Plan>
__device__ __forceinline__ void layer_chunks(Ring &R, f32x4 (&acc)[kNC][NOB], const f32x4 (&in)[kNC][NIN], Plan plan,
                                             int lane, bool on) {
    if constexpr (J < N) {
        constexpr int IB0 = J * kIbPer;
        constexpr int NIB = NIN - IB0 < kIbPer ? NIN - IB0 : kIbPer;
        gemm_chunk<NOB, NIN, IB0, NIB>(acc, in, R.next<NCH>(C0 + J, plan), lane, on);
        layer_chunks<NCH, C0, J + 1, N, NOB, NIN>(R, acc, in, plan, lane, on);
    }
}

// The chain kernels' work plan: rounds over the grid's wave slots, a wave's
// unit = kNC consecutive 16-sample tiles.  Every round but the last fills all
// slots (round r, workgroup b, wave w → tiles of 128-sample block r·G + b);
// the last round's units are spread over the workgroups first (unit
// w·G + b), so a partial round costs each workgroup one or two busy waves
// instead of whole tiles on a few workgroups (3,643 blocks on 256 workgroups:
// 15 → 14.5 tile times at config C).  A wave without a unit (t16 ≥ n16) skips
// the MFMAs and stores but still streams its share of the weight chunks.
struct ChainPlan {
    int64_t n16, full, rounds;
    __device__ ChainPlan(int64_t m) {
        n16 = (m + kTileW - 1) / kTileW;
        const int64_t slots = (int64_t)gridDim.x * kCWaves * kNC;
        full = n16 / slots;
        rounds = full + (n16 % slots ? 1 : 0);
    }
    __device__ int64_t t16(int64_t r, int wave) const {
        return r < full ? (((int64_t)r * gridDim.x + blockIdx.x) * kCWaves + wave) * kNC
                        : full * (int64_t)gridDim.x * kCWaves * kNC + ((int64_t)wave * gridDim.x + blockIdx.x) * kNC;
    }
};

// ---- forward ---------------------------------------------------------------
__global__ __launch_bounds__(kCThreads, 1) void k_dec256_fwd(int64_t m, int64_t n_tiles, const float *__restrict__ feat,
                                                             const float *__restrict__ img, float *__restrict__ sdf,
                                                             float *__restrict__ rgb, Act act,
                                                             const int *__restrict__ m_dev) {
    extern __shared__ __align__(16) float lds[];
    if (m_dev) m = __builtin_amdgcn_readfirstlane(*m_dev);  // the sparse decoder's kept samples (<= m)
    float *vec = lds;  // kVecN
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int e = threadIdx.x; e < kVecN; e += kCThreads) vec[e] = img[kImgMats + e];
    (void)n_tiles;
    const ChainPlan P(m);
    if (P.rounds == 0) return;
    Ring R{lds + ((kVecN + 63) / 64) * 64, img, 0, wave, lane, false};
    const int n = lane & 15, g = lane >> 4;
    auto plan = [](int c) { return fwd_chunk(c); };
    R.prime(plan);
    const bool train = act.h1 != nullptr;  // inference (no act): per-sample outputs only
    for (int64_t rd = 0; rd < P.rounds; ++rd) {
        R.more = rd + 1 < P.rounds;
        R.img = img;
        asm volatile("" : "+s"(R.img));  // chunk addresses are rebuilt per tile, not kept live across it
        const int64_t t16 = P.t16(rd, wave);  // this wave's first 16-sample tile
        const bool on = t16 < P.n16;          // wave-uniform
        f32x4 x[kNC][1];
#pragma unroll
        for (int c = 0; c < kNC; ++c) {
            const int64_t s = (t16 + c) * kTileW + n;
            x[c][0] = s < m ? *reinterpret_cast<const f32x4 *>(feat + s * 16 + 4 * g) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
        uint64_t m1[kNC], m2[kNC], m4[kNC];
        // L1, L2
        f32x4 h1[kNC][16], h2[kNC][16];
        init_bias(h1, vec + kVB1, lane);
        gemm_chunk<16, 1, 0, 1>(h1, x, R.next<kFwdChunks>(0, plan), lane, on);
        relu_mask(h1, m1);
        init_bias(h2, vec + kVB2, lane);
        layer_chunks<kFwdChunks, kFwdL2, 0, kN16>(R, h2, h1, plan, lane, on);
        if (train && on) store_tiles(act.h1, t16, 256, h1, lane);
        relu_mask(h2, m2);
        // L3: rows [f (blocks 0..7) | sdf (block 8, row 0)]
        f32x4 o3[kNC][9];
        init_bias(o3, vec + kVB3, lane);
        layer_chunks<kFwdChunks, kFwdL3, 0, kN16>(R, o3, h2, plan, lane, on);
        if (train && on) store_tiles(act.h2, t16, 256, h2, lane);
        float sdf_v[kNC];
        f32x4 fx[kNC][9];
#pragma unroll
        for (int c = 0; c < kNC; ++c) {
            sdf_v[c] = o3[c][8][0];  // row 128 = sdf (lanes with g == 0)
#pragma unroll
            for (int b = 0; b < 8; ++b) fx[c][b] = o3[c][b];
            fx[c][8] = x[c][0];
        }
        // L4
        f32x4 c1[kNC][16];
        init_bias(c1, vec + kVB4, lane);
        layer_chunks<kFwdChunks, kFwdL4, 0, kN9>(R, c1, fx, plan, lane, on);
        if (train && on) store_tiles(act.fx, t16, 144, fx, lane);
        relu_mask(c1, m4);
        // L5
        f32x4 o5[kNC][1];
        init_bias(o5, vec + kVB5, lane);
        gemm_chunk<1, 16, 0, 16>(o5, c1, R.next<kFwdChunks>(kFwdL5, plan), lane, on);
        if (train && on) store_tiles(act.c1, t16, 256, c1, lane);
#pragma unroll
        for (int c = 0; c < kNC; ++c) {
            if (act.masks && on) {
                uint64_t *mk = act.masks + (t16 + c) * 3 * 64;
                mk[lane] = m1[c];
                mk[64 + lane] = m2[c];
                mk[128 + lane] = m4[c];
            }
            const int64_t s = (t16 + c) * kTileW + n;
            if (on && s < m && g == 0) {
                sdf[s] = sdf_v[c];
                if (rgb) {
                    rgb[s * 3 + 0] = sigmoidf(o5[c][0][0]);
                    rgb[s * 3 + 1] = sigmoidf(o5[c][0][1]);
                    rgb[s * 3 + 2] = sigmoidf(o5[c][0][2]);
                }
            }
        }
    }
}

// ---- the sdf trunk: h1, h2 and the sdf row only (sparse decoder; sdf-only
// inference): 73.3 of 140.3 k MACs per sample.  The same chunks, MFMAs and
// order as k_dec256_fwd's L1 / L2, and the sdf row from kS3 — W3 row 0 as
// one output block — accumulated over the same k-steps in the same order as
// block 8 of k_dec256_fwd's L3: the same sdf bits.
__global__ __launch_bounds__(kCThreads, 1) void k_dec256_trunk(int64_t m, const float *__restrict__ feat,
                                                               const float *__restrict__ img,
                                                               float *__restrict__ sdf,
                                                               const int *__restrict__ m_dev) {
    extern __shared__ __align__(16) float lds[];
    // the device-sized forward (queued before the host reads the query's
    // statistics): the sampler's M; m is then the buffers' capacity — a
    // larger batch: nothing here, the host-sized launch after the read-back
    if (m_dev) {
        const int64_t md = __builtin_amdgcn_readfirstlane(*m_dev);
        m = md > m ? 0 : md;
    }
    float *vec = lds;  // kVecN
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int e = threadIdx.x; e < kVecN; e += kCThreads) vec[e] = img[kImgMats + e];
    const ChainPlan P(m);
    if (P.rounds == 0) return;
    Ring R{lds + ((kVecN + 63) / 64) * 64, img, 0, wave, lane, false};
    const int n = lane & 15, g = lane >> 4;
    auto plan = [](int c) { return trunk_chunk(c); };
    R.prime(plan);
    for (int64_t rd = 0; rd < P.rounds; ++rd) {
        R.more = rd + 1 < P.rounds;
        R.img = img;
        asm volatile("" : "+s"(R.img));
        const int64_t t16 = P.t16(rd, wave);
        const bool on = t16 < P.n16;  // wave-uniform
        f32x4 x[kNC][1];
#pragma unroll
        for (int c = 0; c < kNC; ++c) {
            const int64_t s = (t16 + c) * kTileW + n;
            x[c][0] = s < m ? *reinterpret_cast<const f32x4 *>(feat + s * 16 + 4 * g) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
        uint64_t m1[kNC], m2[kNC];
        f32x4 h1[kNC][16], h2[kNC][16];
        init_bias(h1, vec + kVB1, lane);
        gemm_chunk<16, 1, 0, 1>(h1, x, R.next<kTrkChunks>(0, plan), lane, on);
        relu_mask(h1, m1);
        init_bias(h2, vec + kVB2, lane);
        layer_chunks<kTrkChunks, kTrkL2, 0, kN16>(R, h2, h1, plan, lane, on);
        relu_mask(h2, m2);
        f32x4 o3[kNC][1];
        init_bias(o3, vec + kVB3 + 128, lane);  // block 8's biases: row 128 = the sdf's
        gemm_chunk<1, 16, 0, 16>(o3, h2, R.next<kTrkChunks>(kTrkS3, plan), lane, on);
#pragma unroll
        for (int c = 0; c < kNC; ++c) {
            const int64_t s = (t16 + c) * kTileW + n;
            if (on && s < m && g == 0) sdf[s] = o3[c][0][0];
        }
    }
}

// ---- backward (data) --------------------------------------------------------
// The fused interpolation backward of a wave's 16 samples (k_dec256_bwd's
// tile tail): the embedding rows and the ray are gathered here, then dL/dx and
// the scatter (interp_fuse.h).  Not inlined: inside the chain's loop the
// compiler ran out of registers (the activations' 190 plus the gathers), and
// at the tail of a tile nothing of the chain is live across the call.
__device__ __attribute__((noinline)) void interp_tail(const InterpFuse ip, float *stg, int64_t m, int64_t s,
                                                      bool valid, int n, int g, int lane, int64_t u, int lf, int row,
                                                      float ts, float c0, float c1, float c2, int4 vid0, int4 vid1,
                                                      float4 gf) {
    const float cen[3] = {c0, c1, c2};
    float ro3[3] = {0.f, 0.f, 0.f}, rd3[3] = {0.f, 0.f, 0.f};
    float4 ev[8];
    const int vid[8] = {vid0.x, vid0.y, vid0.z, vid0.w, vid1.x, vid1.y, vid1.z, vid1.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) ev[k] = reinterpret_cast<const float4 *>(ip.emb)[(int64_t)vid[k] * 4 + g];
    if (valid) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            ro3[a] = ip.rays_o[(int64_t)row * 3 + a];
            rd3[a] = ip.rays_d[(int64_t)row * 3 + a];
        }
    }
    ifuse::interp_bwd_unit(ip, stg, m, s, valid, n, g, ts, ro3, rd3, cen, vid0, vid1, ev, gf);
    if (ip.grad_emb != nullptr) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the staging is this wave's own
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        ifuse::scatter_unit(ip, stg, u, m, lane, lf);
    }
}

__global__ __launch_bounds__(kCThreads, 1) void k_dec256_bwd(int64_t m, int64_t n_tiles, const float *__restrict__ img,
                                                             const float *__restrict__ rgb,
                                                             const float *__restrict__ g_sdf,
                                                             const float *__restrict__ g_rgb, Act act, Dlt dl,
                                                             float *__restrict__ dfeat, InterpFuse ip,
                                                             const int *__restrict__ m_dev) {
    extern __shared__ __align__(16) float lds[];
    if (m_dev) m = __builtin_amdgcn_readfirstlane(*m_dev);  // the sparse decoder's kept samples (<= m)
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    (void)n_tiles;
    const ChainPlan P(m);
    if (P.rounds == 0) return;
    Ring R{lds, img, 0, wave, lane, false};
    const int n = lane & 15, g = lane >> 4;
    const bool want_w = dl.d1 != nullptr;
    // ip.gx set (the mapping engine, kNC = 1): the interpolation backward of
    // the wave's 16 samples right after their dfeat (k_mlp_bwd3's scheme,
    // interp_fuse.h) instead of a dfeat store and a k_interp_bwd launch
    // beside the weight-gradient kernel; its sample data loads one
    // dependent level per layer (leaf / ray / t, then the leaf's vertex rows
    // and centre, then the embedding rows and the ray) under the chain's MFMAs
    const bool fuse = kNC == 1 && ip.gx != nullptr;  // uniform
    float *const stg = lds + kRing * kChunkFloats + wave * 512;
    auto plan = [](int c) { return bwd_chunk(c); };
    R.prime(plan);
    for (int64_t rd = 0; rd < P.rounds; ++rd) {
        R.more = rd + 1 < P.rounds;
        R.img = img;
        asm volatile("" : "+s"(R.img));
        const int64_t t16 = P.t16(rd, wave);
        const bool on = t16 < P.n16;  // wave-uniform
        uint64_t m1[kNC], m2[kNC], m4[kNC];
        // δ of the rgb logits: g_rgb · σ' (rows 0..2 of a 16-row block, lanes g == 0)
        f32x4 d5[kNC][1];
        float gs[kNC];
#pragma unroll
        for (int c = 0; c < kNC; ++c) {
            const uint64_t *mk = act.masks + (on ? t16 + c : 0) * 3 * 64;
            m1[c] = on ? mk[lane] : 0;
            m2[c] = on ? mk[64 + lane] : 0;
            m4[c] = on ? mk[128 + lane] : 0;
            const int64_t s = (t16 + c) * kTileW + n;
            d5[c][0] = f32x4{0.f, 0.f, 0.f, 0.f};
            gs[c] = 0.0f;
            if (s < m) {
                gs[c] = g_sdf[s];
                if (g == 0) {
#pragma unroll
                    for (int i = 0; i < 3; ++i) {
                        const float r = rgb[s * 3 + i];
                        d5[c][0][i] = g_rgb[s * 3 + i] * (r * (1.0f - r));
                    }
                }
            }
        }
        const int64_t s0 = t16 * kTileW + n;  // this lane's sample (kNC = 1)
        const bool fvalid = fuse && on && s0 < m;
        int lf = 0, ro = 0;
        float ts = 0.f;
        if (fvalid) {
            lf = ip.leaf[s0];
            ro = ip.ray_of[s0];
            ts = ip.t[s0];
        }
        // δc1 = (W5ᵀ δ5) ⊙ m_c1
        f32x4 dc1[kNC][16];
        zero(dc1);
        gemm_chunk<16, 1, 0, 1>(dc1, d5, R.next<kBwdChunks>(0, plan), lane, on);
        apply_mask(dc1, m4);
        // δ[f; x] = W4ᵀ δc1
        f32x4 dfx[kNC][9];
        zero(dfx);
        layer_chunks<kBwdChunks, kBwdL4, 0, kN16>(R, dfx, dc1, plan, lane, on);
        int4 vid0 = make_int4(0, 0, 0, 0), vid1 = make_int4(0, 0, 0, 0);
        float cen[3] = {0.f, 0.f, 0.f};
        int row = 0;
        if (fvalid) {
            vid0 = *reinterpret_cast<const int4 *>(ip.vertex_idx + (int64_t)lf * 8);
            vid1 = *reinterpret_cast<const int4 *>(ip.vertex_idx + (int64_t)lf * 8 + 4);
#pragma unroll
            for (int a = 0; a < 3; ++a) cen[a] = ip.centres[(int64_t)lf * 3 + a];
            row = ip.rank_ray[ro];
        }
        if (want_w && on) {
            store_tiles(dl.d4, t16, 256, dc1, lane);
            store_tiles(dl.d5, t16, 16, d5, lane);
        }
        // δh2 = (W3ᵀ [δf; g_sdf]) ⊙ m_h2 (the sdf row as block 8's row 0)
        f32x4 dx[kNC][1];
#pragma unroll
        for (int c = 0; c < kNC; ++c) {
            dx[c][0] = dfx[c][8];
            dfx[c][8] = f32x4{g == 0 ? gs[c] : 0.0f, 0.f, 0.f, 0.f};
        }
        f32x4 dh2[kNC][16];
        zero(dh2);
        layer_chunks<kBwdChunks, kBwdL3, 0, kN9>(R, dh2, dfx, plan, lane, on);
        if (want_w && on) store_tiles(dl.d3, t16, 144, dfx, lane);
        apply_mask(dh2, m2);
        // δh1 = (W2ᵀ δh2) ⊙ m_h1
        f32x4 dh1[kNC][16];
        zero(dh1);
        layer_chunks<kBwdChunks, kBwdL2, 0, kN16>(R, dh1, dh2, plan, lane, on);
        if (want_w && on) store_tiles(dl.d2, t16, 256, dh2, lane);
        apply_mask(dh1, m1);
        // δx = W1ᵀ δh1 + the x rows of δ[f; x]
        gemm_chunk<1, 16, 0, 16>(dx, dh1, R.next<kBwdChunks>(kBwdL1, plan), lane, on);
        if (want_w && on) store_tiles(dl.d1, t16, 256, dh1, lane);
        if (fuse) {
            if (on) {  // dL/dx per sample (summed per ray by k_interp_rays_gx) and the embedding scatter
                const float4 gf = make_float4(dx[0][0][0], dx[0][0][1], dx[0][0][2], dx[0][0][3]);
                interp_tail(ip, stg, m, s0, fvalid, n, g, lane, t16, lf, row, ts, cen[0], cen[1], cen[2], vid0, vid1, gf);
            }
        } else {
#pragma unroll
            for (int c = 0; c < kNC; ++c) {
                const int64_t s = (t16 + c) * kTileW + n;
                if (on && s < m) *reinterpret_cast<f32x4 *>(dfeat + s * 16 + 4 * g) = dx[c][0];
            }
        }
    }
}

// ---- weight gradients ---------------------------------------------------------
// dW_L[m][n] = Σ_s A[m][s] B[n][s] (+ db_L[m] = Σ_s A[m][s]) over 16-sample tiles:
//   L2: A = δh2 (256), B = h1 (256); L3: A = [δf; g_sdf] (144), B = h2 (256);
//   L4: A = δc1 (256), B = [f; x] (144); L15: W1 (A = δh1, B = x rows of fx)
//   and W5 (A = δ5, B = c1) in one workgroup type.
// Workgroup = 8 waves; (layer, tile range); tiles stream through a 3-stage
// ring; wave w owns a fixed set of 16 x 16 output blocks in registers.
struct DwOps {
    const float *a[4], *b[4];  // per layer type: operand tile bases
    int fa[4], fb[4];          // rows per tile
    const float *a5, *b5;      // L15's second pair (δ5, c1)
};
struct DwPlan {
    int wg_begin[5];  // workgroups of type 0..3 = [wg_begin[t], wg_begin[t+1])
    int64_t n16;      // 16-sample tiles
    int slab_off[5];  // floats: slab of type t starts at slab_off[t] + (wg - wg_begin[t]) * slab_size[t]
    int slab_size[4];
};
// L3 / L4 workgroups (18 output blocks a wave) take kDwTpb 16-sample tiles
// per stage: one barrier per kDwTpb tiles (their per-tile MFMA work is about
// half of L2's 32 blocks); 3 stages of ≤ 12,800 floats
#ifndef PSVO_DW256_TPB
#define PSVO_DW256_TPB 2
#endif
constexpr int kDwTpb = PSVO_DW256_TPB;
constexpr int kDwSt = 6400 * kDwTpb > 8704 ? 6400 * kDwTpb : 8704;  // floats per stage
constexpr int kDwLds = 3 * kDwSt * 4;
static_assert(kDwLds <= 160 * 1024, "dw LDS budget");

// block ownership: wave w, layer type t → list of (mb, nb) with mb < MB_t, nb < NB_t
// L2 (16x16): mb 4(w>>1)..+3, nb 8(w&1)..+7    -> 32 blocks
// L3 (9x16):  all 9 mb, nb 2w, 2w+1              -> 18 blocks
// L4 (16x9):  mb 2w, 2w+1, all 9 nb              -> 18 blocks
// L15: W1 (16x1) mb 2w, 2w+1, nb 0; W5 (1x16) mb 0, nb 2w, 2w+1 -> 4 blocks
template <int MB, int NB>
__device__ __forceinline__ void dw_tile(f32x4 (&acc)[MB][NB], float (&bsum)[MB], bool do_bias, const float *sa,
                                        const float *sb, const int (&mb)[MB], const int (&nb)[NB], int lane) {
    const int r = lane & 15, g = lane >> 4;
    f32x4 av[MB], bv[NB];
#pragma unroll
    for (int i = 0; i < MB; ++i) {
        const int row = 16 * mb[i] + r;
        av[i] = *reinterpret_cast<const f32x4 *>(sa + row * 16 + ((g ^ hsw((row >> 2) & 3)) << 2));
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        const int row = 16 * nb[j] + r;
        bv[j] = *reinterpret_cast<const f32x4 *>(sb + row * 16 + ((g ^ hsw((row >> 2) & 3)) << 2));
    }
    if (do_bias) {
#pragma unroll
        for (int i = 0; i < MB; ++i) bsum[i] += (av[i][0] + av[i][1]) + (av[i][2] + av[i][3]);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < MB; ++i)
#pragma unroll
            for (int j = 0; j < NB; ++j) acc[i][j] = mfma(av[i][t], bv[j][t], acc[i][j]);
}

// C block (mb, nb) of a [rows][cols] slab: lane holds C[16 mb + 4 g + i][16 nb + (l & 15)]
template <int MB, int NB>
__device__ __forceinline__ void dw_store(float *slab, int cols, const f32x4 (&acc)[MB][NB], const int (&mb)[MB],
                                         const int (&nb)[NB], int lane) {
    const int c = lane & 15, g = lane >> 4;
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) slab[(16 * mb[i] + 4 * g + q) * cols + 16 * nb[j] + c] = acc[i][j][q];
}
// bias sums: Σ over the 4 lane groups, row 16 mb + (l & 15); written as column `cols - 1`? -> separate vector
template <int MB>
__device__ __forceinline__ void dw_store_bias(float *bias, const float (&bsum)[MB], const int (&mb)[MB], int lane) {
#pragma unroll
    for (int i = 0; i < MB; ++i) {
        float v = bsum[i];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        if (lane < 16) bias[16 * mb[i] + lane] = v;
    }
}

template <int T>
__device__ void dw_run(const DwOps &op, const DwPlan &pl, float *slabs, float *lds, int wg, int64_t t0, int64_t t1) {
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // stage layout: [A tile | B tile] (L15: [δh1 | x rows | δ5 | c1])
    constexpr int FA = T == 0 ? 256 : T == 1 ? 144 : T == 2 ? 256 : 256;
    constexpr int FB = T == 0 ? 256 : T == 1 ? 256 : T == 2 ? 144 : 16;
    constexpr int kStageF = T == 3 ? 256 * 16 + 16 * 16 + 16 * 16 + 256 * 16 : (FA + FB) * 16;
    constexpr int MB = T == 0 ? 4 : T == 1 ? 9 : T == 2 ? 2 : 2;
    constexpr int NB = T == 0 ? 8 : T == 1 ? 2 : T == 2 ? 9 : 1;
    int mb[MB], nb[NB];
#pragma unroll
    for (int i = 0; i < MB; ++i) mb[i] = T == 0 ? 4 * (wave >> 1) + i : T == 1 ? i : 2 * wave + i;
#pragma unroll
    for (int j = 0; j < NB; ++j) nb[j] = T == 0 ? 8 * (wave & 1) + j : T == 1 ? 2 * wave + j : T == 2 ? j : 0;
    f32x4 acc[MB][NB];
    float bsum[MB];
#pragma unroll
    for (int i = 0; i < MB; ++i) {
        bsum[i] = 0.0f;
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // L15's W5 part: mb 0 (δ5 rows), nb 2 wave, 2 wave + 1 of c1
    f32x4 acc5[1][2];
    float bsum5[1] = {0.0f};
    int mb5[1] = {0}, nb5[2] = {2 * wave, 2 * wave + 1};
    acc5[0][0] = acc5[0][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    // bias: in L2 / L3 the waves sharing rows split nothing: the wave with the
    // first column group sums (L2: w even; L3: w == 0; L4: every wave; L15: every wave, W5 on wave 0)
    const bool bias_main = T == 0 ? (wave & 1) == 0 : T == 1 ? wave == 0 : true;
    // a tile's 1-KB pieces (regions [A | B], L15 [δh1 | x rows | δ5 | c1]) are
    // dealt to the waves round robin, PER per wave (the last piece repeated
    // where the count does not divide: an identical copy to the same place),
    // so every wave has the same number of copies in flight and waits for
    // exactly one tile with a compile-time vmcnt
    constexpr int NP0 = T == 3 ? 16 : FA / 16, NP1 = T == 3 ? 1 : FB / 16, NP2 = T == 3 ? 1 : 0,
                  NP3 = T == 3 ? 16 : 0;
    constexpr int NPT = NP0 + NP1 + NP2 + NP3;
    constexpr int PER = (NPT + kWaves - 1) / kWaves;
    constexpr int TPB = (T == 1 || T == 2) ? kDwTpb : 1;  // tiles per stage
    // stage s holds tiles t0 + TPB·s + j; past t1 the last tile is copied again
    // (same copy count per wave) and not computed
    auto fill = [&](int64_t sg, float *st) {
#pragma unroll
        for (int j = 0; j < TPB; ++j) {
            int64_t t = t0 + TPB * sg + j;
            t = t < t1 ? t : t1 - 1;
            const float *base[4];
            if (T == 3) {
                base[0] = op.a[3] + t * 256 * 16;               // δh1
                base[1] = op.b[3] + t * 144 * 16 + 128 * 16;    // x rows of [f; x]
                base[2] = op.a5 + t * 16 * 16;                  // δ5
                base[3] = op.b5 + t * 256 * 16;                 // c1
            } else {
                base[0] = op.a[T] + t * FA * 16;
                base[1] = op.b[T] + t * FB * 16;
                base[2] = base[3] = base[0];
            }
            uint32_t voff = (uint32_t)lane * 16u;
            asm volatile("" : "+v"(voff));
#pragma unroll
            for (int k = 0; k < PER; ++k) {
                int p = wave + k * kWaves;
                p = p < NPT ? p : NPT - 1;
                const int r = p < NP0 ? 0 : p < NP0 + NP1 ? 1 : p < NP0 + NP1 + NP2 ? 2 : 3;
                const int q = p - (r == 0 ? 0 : r == 1 ? NP0 : r == 2 ? NP0 + NP1 : NP0 + NP1 + NP2);
                glds16s(base[r] + q * 256, voff, st + j * kStageF + p * 256);
            }
        }
    };
    static_assert(TPB * kStageF <= kDwSt && NPT * 256 == kStageF, "dw stage");
    const int64_t n_sg = t0 < t1 ? (t1 - t0 + TPB - 1) / TPB : 0;
    if (n_sg > 0) fill(0, lds);
    if (n_sg > 1) fill(1, lds + kDwSt);
    int slot = 0;
    for (int64_t sg = 0; sg < n_sg; ++sg) {
        // this wave's copies of stage sg landed (stage sg + 1's may be in flight), then all waves'
        if (sg + 1 < n_sg) wait_vm_lds<PER * TPB>(); else wait_vm_lds<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (sg + 2 < n_sg) fill(sg + 2, lds + ((slot + 2) % 3) * kDwSt);
        auto tile = [&](int j) {
            const float *st = lds + slot * kDwSt + j * kStageF;
            if (T == 3) {
                // x rows sit at stage row offset 256 (rows 128..143 of fx): block index 0 of a 16-row tile
                dw_tile<MB, NB>(acc, bsum, true, st, st + 4096 - 0, mb, nb, lane);
                dw_tile<1, 2>(acc5, bsum5, wave == 0, st + 4352, st + 4608, mb5, nb5, lane);
            } else {
                dw_tile<MB, NB>(acc, bsum, bias_main, st, st + FA * 16, mb, nb, lane);
            }
        };
        tile(0);
        if constexpr (TPB == 2) {
            __builtin_amdgcn_sched_barrier(0);  // the second tile's operand loads not hoisted into the first's MFMAs
            if (t0 + 2 * sg + 1 < t1) tile(1);  // uniform: the last stage's missing tile
        }
        slot = (slot + 1) % 3;
    }
    // slab: [rows][cols] weights then [rows] bias
    const int rows = T == 3 ? 256 : FA, cols = T == 3 ? 16 : FB;
    float *slab = slabs + pl.slab_off[T] + (int64_t)(wg - pl.wg_begin[T]) * pl.slab_size[T];
    dw_store<MB, NB>(slab, cols, acc, mb, nb, lane);
    if (bias_main) dw_store_bias<MB>(slab + rows * cols, bsum, mb, lane);
    if (T == 3) {
        float *slab5 = slab + rows * cols + rows;  // W5: [16][256] + bias [16]
        dw_store<1, 2>(slab5, 256, acc5, mb5, nb5, lane);
        if (wave == 0) dw_store_bias<1>(slab5 + 16 * 256, bsum5, mb5, lane);
    }
}

__global__ __launch_bounds__(kThreads, 1) void k_dec256_dw(DwOps op, DwPlan pl, float *__restrict__ slabs,
                                                            const int *__restrict__ m_dev) {
    extern __shared__ __align__(16) float lds[];
    const int wg = blockIdx.x;
    int t = 0;
    while (t < 3 && wg >= pl.wg_begin[t + 1]) ++t;
    const int nwg = pl.wg_begin[t + 1] - pl.wg_begin[t];
    const int k = wg - pl.wg_begin[t];
    // the sparse decoder: the kept samples' tiles (the plan's workgroups were sized for the upper bound)
    const int64_t n16 = m_dev ? (int64_t)((__builtin_amdgcn_readfirstlane(*m_dev) + kTileW - 1) / kTileW) : pl.n16;
    const int64_t per = (n16 + nwg - 1) / nwg;
    int64_t t0 = k * per, t1 = t0 + per < n16 ? t0 + per : n16;
    if (t0 > t1) t0 = t1;  // a workgroup past the kept tiles: an empty range, zero slabs
    switch (t) {
        case 0: dw_run<0>(op, pl, slabs, lds, wg, t0, t1); break;
        case 1: dw_run<1>(op, pl, slabs, lds, wg, t0, t1); break;
        case 2: dw_run<2>(op, pl, slabs, lds, wg, t0, t1); break;
        default: dw_run<3>(op, pl, slabs, lds, wg, t0, t1); break;
    }
}

// Σ over a layer's slabs → the torch parameter gradients (layout mapping of
// the chain: W3 rows [f | sdf], W5 padded to 16 rows)
struct DwOut {
    float *gw[5], *gb[5];
};
__global__ __launch_bounds__(256) void k_dec256_dw_reduce(DwPlan pl, const float *__restrict__ slabs, DwOut o,
                                                          int accumulate) {
    // element spaces: W2 (256x256 + 256), W3 (129x256 + 129), W4 (256x144 + 256), W1 (256x16 + 256), W5 (3x256 + 3)
    const int sizes[5] = {256 * 256 + 256, 129 * 256 + 129, 256 * 144 + 256, 256 * 16 + 256, 3 * 256 + 3};
    int e = blockIdx.x * 256 + threadIdx.x;
    int L = 0;
    while (L < 5 && e >= sizes[L]) e -= sizes[L++];
    if (L >= 5) return;
    const int T = L < 4 ? L : 3;
    const int nwg = pl.wg_begin[T + 1] - pl.wg_begin[T];
    const float *base = slabs + pl.slab_off[T];
    // (slab element, destination)
    int se;
    float *dst;
    if (L == 0) {  // W2
        se = e;
        dst = e < 65536 ? o.gw[1] + e : o.gb[1] + (e - 65536);
    } else if (L == 1) {  // W3: torch row r ↔ chain row r - 1 (r ≥ 1), row 0 ↔ chain row 128
        if (e < 129 * 256) {
            const int r = e / 256, c = e % 256;
            se = (r == 0 ? 128 : r - 1) * 256 + c;
            dst = o.gw[2] + e;
        } else {
            const int r = e - 129 * 256;
            se = 144 * 256 + (r == 0 ? 128 : r - 1);
            dst = o.gb[2] + r;
        }
    } else if (L == 2) {  // W4
        se = e;
        dst = e < 256 * 144 ? o.gw[3] + e : o.gb[3] + (e - 256 * 144);
    } else if (L == 3) {  // W1 (L15 slab head: [256][16] + [256])
        se = e;
        dst = e < 256 * 16 ? o.gw[0] + e : o.gb[0] + (e - 256 * 16);
    } else {  // W5 (L15 slab tail: [16][256] + [16])
        const int off5 = 256 * 16 + 256;
        se = e < 3 * 256 ? off5 + e : off5 + 16 * 256 + (e - 3 * 256);
        dst = e < 3 * 256 ? o.gw[4] + e : o.gb[4] + (e - 3 * 256);
    }
    double acc = 0.0;
    for (int k = 0; k < nwg; ++k) acc += (double)base[(int64_t)k * pl.slab_size[T] + se];
    *dst = accumulate ? *dst + (float)acc : (float)acc;
}

}  // namespace

// ---- host side -----------------------------------------------------------------
static int device_cus256() {
    static int cus = 0;
    if (cus == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    return cus;
}

int64_t dec256_tiles16(int64_t m) { return (m + kTileWG - 1) / kTileWG * kWaves; }
int64_t dec256_image_floats() { return kImgTotal; }
int64_t dec256_act_floats(int64_t m) { return dec256_tiles16(m) * 16 * (256 + 256 + 144 + 256); }
int64_t dec256_mask_words(int64_t m) { return dec256_tiles16(m) * 3 * 64; }

static void dw_plan(int64_t m, DwPlan *pl, int64_t *slab_floats) {
    const int64_t n16 = (m + kTileW - 1) / kTileW;  // tiles holding samples (all written by the chain kernels)
    pl->n16 = n16;
    // workgroups ∝ a type's time per sample on one CU: max(its FLOPs at the
    // CU's f32-MFMA rate (157.3 TF / 256), its operand bytes at a CU's share
    // of HBM (≈20 GB/s)) — L2: 131 kFLOP | 2,048 B, L3 / L4: 73.7 kFLOP |
    // 1,600 B, L1 + L5: 16.4 kFLOP | 2,112 B (memory-bound: by FLOPs alone it
    // got 14 workgroups and set the kernel's time)
    const int cus = device_cus256();
    // per-type weights measured at config C (466 k samples, one box, decoder
    // alone): {213,120,120,107} 1,310 us -> {213,130,130,60} 1,195-1,200 us —
    // the W1 / W5 type's byte-bound tiles finish early with fewer workgroups
    const int w[4] = {213, 130, 130, 60};
    const double wsum = (double)(w[0] + w[1] + w[2] + w[3]);
    // exactly `cus` workgroups (largest remainders): one more than the CUs
    // would run two of them back to back on one CU (104 KB of LDS each)
    int n[4], tot = 0;
    double rem[4];
    for (int t = 0; t < 4; ++t) {
        const double q = (double)cus * w[t] / wsum;
        n[t] = (int)q;
        rem[t] = q - n[t];
        tot += n[t];
    }
    while (tot < cus) {
        int b = 0;
        for (int t = 1; t < 4; ++t)
            if (rem[t] > rem[b]) b = t;
        n[b] += 1;
        rem[b] = -1.0;
        tot += 1;
    }
    for (int t = 0; t < 4; ++t) {
        if (n[t] < 1) n[t] = 1;
        if (n[t] > n16) n[t] = (int)(n16 > 0 ? n16 : 1);
    }
    pl->wg_begin[0] = 0;
    for (int t = 0; t < 4; ++t) pl->wg_begin[t + 1] = pl->wg_begin[t] + n[t];
    const int sz[4] = {256 * 256 + 256, 144 * 256 + 144, 256 * 144 + 256, 256 * 16 + 256 + 16 * 256 + 16};
    int64_t off = 0;
    for (int t = 0; t < 4; ++t) {
        pl->slab_off[t] = (int)off;
        pl->slab_size[t] = sz[t];
        off += (int64_t)n[t] * sz[t];
    }
    pl->slab_off[4] = (int)off;
    *slab_floats = off;
}

int64_t dec256_workspace_floats(int64_t m) {
    DwPlan pl;
    int64_t slab;
    dw_plan(m, &pl, &slab);
    return dec256_tiles16(m) * 16 * (256 + 256 + 144 + 256 + 16) + slab;
}

int dec256_images(hipStream_t st, const float *w1, const float *b1, const float *w2, const float *b2, const float *w3,
                  const float *b3, const float *w4, const float *b4, const float *w5, const float *b5, float *images) {
    Params p{w1, b1, w2, b2, w3, b3, w4, b4, w5, b5};
    psvo::launch(k_dec256_prep, dim3(div_up(kImgTotal, 256)), dim3(256), 0, st, p, images);
    return check_launch("dec256_images");
}

static int grid_for(int64_t n_tiles) {
    const int cus = device_cus256();
    return (int)(n_tiles < cus ? n_tiles : cus);
}

int dec256_fwd(hipStream_t st, int64_t m, const float *feat, const float *images, float *sdf, float *rgb, float *act,
               uint64_t *masks, const int *m_dev) {
    if (m == 0) return PSVO_OK;
    const int64_t n_tiles = (m + kChainTile - 1) / kChainTile;
    if (!rgb && !act && !masks) {  // sdf only: the trunk
        const int lds = (((kVecN + 63) / 64) * 64 + kRing * kChunkFloats) * 4;
        static bool tattr = false;
        if (!tattr) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_dec256_trunk),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, lds);
            tattr = true;
        }
        psvo::launch(k_dec256_trunk, dim3(grid_for(n_tiles)), dim3(kCThreads), lds, st, m, feat, images, sdf, m_dev);
        return check_launch("dec256_trunk");
    }
    const int64_t n16 = dec256_tiles16(m);
    Act a{};
    if (act) {
        a.h1 = act;
        a.h2 = a.h1 + n16 * 256 * 16;
        a.fx = a.h2 + n16 * 256 * 16;
        a.c1 = a.fx + n16 * 144 * 16;
    }
    a.masks = masks;
    const int lds = (((kVecN + 63) / 64) * 64 + kRing * kChunkFloats) * 4;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_dec256_fwd),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        attr = true;
    }
    psvo::launch(k_dec256_fwd, dim3(grid_for(n_tiles)), dim3(kCThreads), lds, st, m, n_tiles, feat, images, sdf,
                 rgb, a, m_dev);
    return check_launch("dec256_fwd");
}

int dec256_bwd(hipStream_t st, int64_t m, const float *feat, const float *images, const float *rgb, const float *act,
               const uint64_t *masks, const float *g_sdf, const float *g_rgb, float *dfeat, float *const gw[5],
               float *const gb[5], int accumulate, float *workspace, hipEvent_t dfeat_ready,
               const InterpFuse *ip, const int *m_dev) {
    PSVO_REQUIRE(ip == nullptr || (kNC == 1 && gw[0] != nullptr),
                 "dec256_bwd: the fused interpolation backward needs the weight-gradient path (1 group per wave)");
    (void)feat;
    const int64_t n_tiles = (m + kChainTile - 1) / kChainTile;
    const int64_t n16 = dec256_tiles16(m);
    Act a;
    a.h1 = const_cast<float *>(act);
    a.h2 = a.h1 + n16 * 256 * 16;
    a.fx = a.h2 + n16 * 256 * 16;
    a.c1 = a.fx + n16 * 144 * 16;
    a.masks = const_cast<uint64_t *>(masks);
    const bool want_w = gw[0] != nullptr;
    Dlt d{};
    float *ws = workspace;
    if (want_w) {
        d.d1 = ws; ws += n16 * 256 * 16;
        d.d2 = ws; ws += n16 * 256 * 16;
        d.d3 = ws; ws += n16 * 144 * 16;
        d.d4 = ws; ws += n16 * 256 * 16;
        d.d5 = ws; ws += n16 * 16 * 16;
    } else {
        ws += n16 * 16 * (256 + 256 + 144 + 256 + 16);
    }
    bool bound = false;
    if (m > 0) {
        const int lds = (kRing * kChunkFloats + kCWaves * 512) * 4;  // ring + per-wave scatter staging
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_dec256_bwd),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, lds);
            attr = true;
        }
        // dfeat_ready through the dispatch's stop event (no marker packet
        // between the backward and the weight-gradient kernel on st)
        static const bool bind_env = [] {
            const char *v = getenv("PSVO_BIND_DFEAT");
            return !(v && v[0] == '0');
        }();
        if (bind_env && dfeat_ready) psvo::g_stop_event = dfeat_ready;
        psvo::launch(k_dec256_bwd, dim3(grid_for(n_tiles)), dim3(kCThreads), lds, st, m, n_tiles, images, rgb,
                     g_sdf, g_rgb, a, d, dfeat, ip ? *ip : InterpFuse{}, m_dev);
        bound = bind_env && dfeat_ready && psvo::g_stop_event == nullptr;
        psvo::g_stop_event = nullptr;
        const int rc = check_launch("dec256_bwd");
        if (rc) return rc;
    }
    if (dfeat_ready && !bound && hipEventRecord(dfeat_ready, st) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "dec256_bwd: event record failed");
    if (!want_w) return PSVO_OK;
    DwPlan pl;
    int64_t slab_floats;
    dw_plan(m, &pl, &slab_floats);
    float *slabs = ws;
    DwOps op;
    op.a[0] = d.d2; op.b[0] = a.h1;   // L2
    op.a[1] = d.d3; op.b[1] = a.h2;   // L3
    op.a[2] = d.d4; op.b[2] = a.fx;   // L4
    op.a[3] = d.d1; op.b[3] = a.fx;   // L1 (x rows of fx)
    op.a5 = d.d5; op.b5 = a.c1;       // L5
    for (int t = 0; t < 4; ++t) op.fa[t] = op.fb[t] = 0;
    static bool dattr = false;
    if (!dattr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_dec256_dw),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, kDwLds);
        dattr = true;
    }
    if (m > 0) {
        psvo::launch(k_dec256_dw, dim3(pl.wg_begin[4]), dim3(kThreads), kDwLds, st, op, pl, slabs, m_dev);
        const int rc = check_launch("dec256_dw");
        if (rc) return rc;
    } else if (hipMemsetAsync(slabs, 0, slab_floats * sizeof(float), st) != hipSuccess) {
        return set_error(PSVO_E_LAUNCH, "dec256_bwd: memset failed");
    }
    DwOut o;
    for (int l = 0; l < 5; ++l) {
        o.gw[l] = gw[l];
        o.gb[l] = gb[l];
    }
    const int total = (256 * 256 + 256) + (129 * 256 + 129) + (256 * 144 + 256) + (256 * 16 + 256) + (3 * 256 + 3);
    psvo::launch(k_dec256_dw_reduce, dim3(div_up(total, 256)), dim3(256), 0, st, pl, slabs, o, accumulate);
    return check_launch("dec256_dw_reduce");
}

}  // namespace psvo
