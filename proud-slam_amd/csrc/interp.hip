// Trilinear interpolation of per-vertex embeddings at ray samples, forward
// and backward, on gfx950.
//
// Reference: render_helpers.py:104-156 (get_features_vox) with :86-99
// (get_embeddings_vox), :67-83 (offset_points) and :46-59 (trilinear_interp);
// the backward is what torch autograd derives for that graph
// (embedding_dense_backward scatter + d/dx of the weights), plus the
// broadcast backward of sampled_xyz = rays_o + rays_d * depth
// (render_helpers.py:436-437).
//
//   x = o[ray] + d[ray] * t            (per valid sample, ray-major order)
//   p = (x - centre[leaf]) / voxel + 0.5
//   w_k = Π_a (q_ka ? p_a : 1 - p_a),   k = 4 ix + 2 iy + iz  (meshgrid 'ij')
//   feat = Σ_k w_k E[vertex_idx[leaf, k]]
//
// Layout: embeddings are [E, 16] f32 = one 64-B row; four lanes own one
// sample and each moves 16 B (dims 4q..4q+3), so a wave-instruction reads
// sixteen 64-B rows — whole rows, never split across instructions.  The
// backward runs one wave per ray: the ray's samples are contiguous, the
// dL/dx reduction to d_o / d_d stays in registers (no atomics on rays), and
// the embedding scatter sums each leaf run first and then adds whole 64-B
// rows with global f32 atomics (one request per row and run).
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include "psvo_common.h"

namespace psvo {
namespace {

__device__ __forceinline__ void corner_weights(float px, float py, float pz, float w[8]) {
    const float ax[2] = {1.0f - px, px};
    const float ay[2] = {1.0f - py, py};
    const float az[2] = {1.0f - pz, pz};
#pragma unroll
    for (int k = 0; k < 8; ++k) w[k] = (ax[(k >> 2) & 1] * ay[(k >> 1) & 1]) * az[k & 1];
}

__device__ __forceinline__ void interp_one(int64_t s, int q, float voxel_size, const int *__restrict__ leaf,
                                           const float *__restrict__ t, const int *__restrict__ ray_of_sample,
                                           const int *__restrict__ ray_index, const float *__restrict__ rays_o,
                                           const float *__restrict__ rays_d, const float *__restrict__ centres,
                                           const int *__restrict__ vertex_idx, const float4 *__restrict__ emb,
                                           float4 *__restrict__ feat) {
    const int lf = leaf[s];
    const int r = ray_index ? ray_index[ray_of_sample[s]] : ray_of_sample[s];
    const float ts = t[s];
    float p[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float x = rays_o[(int64_t)r * 3 + a] + rays_d[(int64_t)r * 3 + a] * ts;
        p[a] = __fdiv_rn(x - centres[(int64_t)lf * 3 + a], voxel_size) + 0.5f;
    }
    float w[8];
    corner_weights(p[0], p[1], p[2], w);
    const int4 v0 = *reinterpret_cast<const int4 *>(vertex_idx + (int64_t)lf * 8);
    const int4 v1 = *reinterpret_cast<const int4 *>(vertex_idx + (int64_t)lf * 8 + 4);
    const int vid[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const float4 e = emb[(int64_t)vid[k] * 4 + q];
        acc.x = acc.x + w[k] * e.x;
        acc.y = acc.y + w[k] * e.y;
        acc.z = acc.z + w[k] * e.z;
        acc.w = acc.w + w[k] * e.w;
    }
    feat[s * 4 + q] = acc;
}

__global__ __launch_bounds__(256) void k_interp_fwd(int64_t m, float voxel_size, const int *__restrict__ leaf,
                                                    const float *__restrict__ t,
                                                    const int *__restrict__ ray_of_sample,
                                                    const int *__restrict__ ray_index,
                                                    const float *__restrict__ rays_o,
                                                    const float *__restrict__ rays_d,
                                                    const float *__restrict__ centres,
                                                    const int *__restrict__ vertex_idx,
                                                    const float4 *__restrict__ emb, float4 *__restrict__ feat,
                                                    const int *__restrict__ m_dev) {
    // m_dev: the sample count on the device (a launch queued before the host
    // knows it; m is then the buffers' capacity — a larger batch is left to
    // the host-sized launch after the read-back), the grid striding over it
    int64_t mm = m_dev ? (int64_t)*m_dev : m;
    if (mm > m) mm = 0;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < mm * 4;
         g += (int64_t)gridDim.x * blockDim.x)
        interp_one(g >> 2, (int)(g & 3), voxel_size, leaf, t, ray_of_sample, ray_index, rays_o, rays_d, centres,
                   vertex_idx, emb, feat);
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr int kInterpChunk = 64;  // samples per work unit of the chunked backward (4 passes)

struct BwdPass {  // per-wave LDS: one 16-sample pass, slot-minor so a lane reads 4 slots per ds_read_b128
    float w[8][16];    // trilinear weights [corner][slot]
    float g[16][16];   // grad_feat [dim][slot]
    int vid[16][8];    // vertex rows of the slot's leaf
};  // 2 KB per wave
// waves per k_interp_bwd workgroup: one — a 2-KB workgroup fits three times
// into the 6.4 KB of LDS the width-256 weight-gradient kernel (k_dec256_dw,
// 153.6 KB, one per CU) leaves free, so the embedding backward runs on every
// CU beside it; 4-wave (8-KB) workgroups fitted none of them
#ifndef PSVO_IB_WAVES
#define PSVO_IB_WAVES 1
#endif
constexpr int kIbWaves = PSVO_IB_WAVES;

// One wave per ray; 16 samples per pass, 4 lanes per sample (dims 4q..4q+3)
// for the gathers and dL/dx.  The embedding gradient is summed per leaf RUN
// (consecutive samples of the ray in the same voxel share the 8 vertex rows):
// lane j owns (corner j/16 + 4i, dim j%16), i = 0, 1, accumulates the run in
// registers across passes and flushes it when the leaf changes with two
// atomic instructions, each covering four whole 64-B rows — one memory-side
// request per row, the shape global f32 atomics run at full rate with
// (MI355X_MICROARCH.md, global float atomics).
// EMB = false: pose-only backward (tracking, frozen embeddings): d_o / d_d only
template <bool EMB>
__global__ __launch_bounds__(64 * kIbWaves) void k_interp_bwd(int64_t r_hit, float voxel_size, const int *__restrict__ offsets,
                                                    const int *__restrict__ ray_index,
                                                    const int *__restrict__ leaf, const float *__restrict__ t,
                                                    const float *__restrict__ rays_o,
                                                    const float *__restrict__ rays_d,
                                                    const float *__restrict__ centres,
                                                    const int *__restrict__ vertex_idx,
                                                    const float4 *__restrict__ emb,
                                                    const float4 *__restrict__ grad_feat,
                                                    float *__restrict__ grad_emb, float *__restrict__ grad_o,
                                                    float *__restrict__ grad_d, int chunk, int c_max,
                                                    float *__restrict__ part) {
    __shared__ BwdPass pass_all[kIbWaves];
    BwdPass &B = pass_all[threadIdx.x >> 6];
    const int lane = threadIdx.x & 63;
    // unit = one ray (chunk == 0) or chunk c of ray r (chunk samples each, c < c_max):
    // a long ray's samples spread over several waves instead of serialising
    // the launch behind its passes; partial d_o / d_d go to part[unit]
    const int64_t u = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t r = chunk ? u / c_max : u;
    if (r >= r_hit) return;
    // wave-uniform: scalar registers for the run loop
    const int rbeg = __builtin_amdgcn_readfirstlane(offsets[r]);
    const int rend = __builtin_amdgcn_readfirstlane(offsets[r + 1]);
    const int cidx = chunk ? (int)(u - r * c_max) : 0;
    const int beg = chunk ? min(rend, rbeg + cidx * chunk) : rbeg;
    const int end = chunk ? min(rend, beg + chunk) : rend;
    const int64_t ro_row = ray_index ? ray_index[r] : r;  // row of rays_o / rays_d / grad_o / grad_d
    const int q = lane & 3;
    const int sub = lane >> 2;
    const int ek0 = lane >> 4, ed = lane & 15;  // run accumulator slots: corners ek0, ek0 + 4; dim ed
    float o[3], d[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        o[a] = rays_o[ro_row * 3 + a];
        d[a] = rays_d[ro_row * 3 + a];
    }
    float go[3] = {0.f, 0.f, 0.f}, gd[3] = {0.f, 0.f, 0.f};
    int cur_leaf = -1, cur_v0 = 0, cur_v1 = 0;
    float acc0 = 0.f, acc1 = 0.f;
    for (int base = beg; base < end; base += 16) {
        const int s = base + sub;
        const bool active = s < end;
        float p[3] = {0.f, 0.f, 0.f};
        float w[8];
        int vid[8];
        float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
        float ts = 0.f;
        int lf = -1;
        if (active) {
            lf = leaf[s];
            ts = t[s];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const float x = o[a] + d[a] * ts;
                p[a] = __fdiv_rn(x - centres[(int64_t)lf * 3 + a], voxel_size) + 0.5f;
            }
            const int4 v0 = *reinterpret_cast<const int4 *>(vertex_idx + (int64_t)lf * 8);
            const int4 v1 = *reinterpret_cast<const int4 *>(vertex_idx + (int64_t)lf * 8 + 4);
            vid[0] = v0.x; vid[1] = v0.y; vid[2] = v0.z; vid[3] = v0.w;
            vid[4] = v1.x; vid[5] = v1.y; vid[6] = v1.z; vid[7] = v1.w;
            g = grad_feat[(int64_t)s * 4 + q];
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) vid[k] = 0;
        }
        corner_weights(p[0], p[1], p[2], w);
        // stage this pass for the run sums (each of the sample's 4 lanes writes a quarter)
        wave_lds_sync();  // the previous pass's readers are done
        if (EMB) {
            B.g[4 * q + 0][sub] = g.x;
            B.g[4 * q + 1][sub] = g.y;
            B.g[4 * q + 2][sub] = g.z;
            B.g[4 * q + 3][sub] = g.w;
            B.w[2 * q][sub] = w[2 * q];
            B.w[2 * q + 1][sub] = w[2 * q + 1];
            B.vid[sub][2 * q] = vid[2 * q];
            B.vid[sub][2 * q + 1] = vid[2 * q + 1];
        }
        // dL/dx for this lane's sample: eg_k = E[vid_k] · g
        float eg[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            float a = 0.f;
            if (active) {
                const float4 e = emb[(int64_t)vid[k] * 4 + q];
                a = e.x * g.x + e.y * g.y + e.z * g.z + e.w * g.w;
            }
            a += __shfl_xor(a, 1, 64);
            a += __shfl_xor(a, 2, 64);
            eg[k] = a;
        }
        if (active && q == 0) {
            const float ax[2] = {1.0f - p[0], p[0]};
            const float ay[2] = {1.0f - p[1], p[1]};
            const float az[2] = {1.0f - p[2], p[2]};
            float dp[3] = {0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int ix = (k >> 2) & 1, iy = (k >> 1) & 1, iz = k & 1;
                const float sx = ix ? 1.f : -1.f, sy = iy ? 1.f : -1.f, sz = iz ? 1.f : -1.f;
                dp[0] += sx * ay[iy] * az[iz] * eg[k];
                dp[1] += sy * ax[ix] * az[iz] * eg[k];
                dp[2] += sz * ax[ix] * ay[iy] * eg[k];
            }
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const float gx = __fdiv_rn(dp[a], voxel_size);
                go[a] += gx;
                gd[a] += gx * ts;
            }
        }
        wave_lds_sync();
        if (EMB) {
            // run sums over the pass's valid slots: the pass's weights and
            // gradients come into registers with 12 vector LDS reads, the
            // leaves as wave-uniform (scalar) loads, then the slot loop is
            // register-only (the leaf compare is wave-uniform)
            const int n_slots = min(16, end - base);
            float wa[16], wb[16], gv[16];
            int lfs[16];
#pragma unroll
            for (int sl = 0; sl < 16; ++sl) lfs[sl] = leaf[base + (sl < n_slots ? sl : 0)];
#pragma unroll
            for (int c4 = 0; c4 < 4; ++c4) {
                const float4 a = *reinterpret_cast<const float4 *>(&B.w[ek0][4 * c4]);
                const float4 b = *reinterpret_cast<const float4 *>(&B.w[ek0 + 4][4 * c4]);
                const float4 gg = *reinterpret_cast<const float4 *>(&B.g[ed][4 * c4]);
                wa[4 * c4] = a.x; wa[4 * c4 + 1] = a.y; wa[4 * c4 + 2] = a.z; wa[4 * c4 + 3] = a.w;
                wb[4 * c4] = b.x; wb[4 * c4 + 1] = b.y; wb[4 * c4 + 2] = b.z; wb[4 * c4 + 3] = b.w;
                gv[4 * c4] = gg.x; gv[4 * c4 + 1] = gg.y; gv[4 * c4 + 2] = gg.z; gv[4 * c4 + 3] = gg.w;
            }
#pragma unroll
            for (int sl = 0; sl < 16; ++sl) {
                if (sl < n_slots) {
                    if (lfs[sl] != cur_leaf) {
                        if (cur_leaf >= 0) {
                            atomicAdd(grad_emb + (int64_t)cur_v0 * 16 + ed, acc0);
                            atomicAdd(grad_emb + (int64_t)cur_v1 * 16 + ed, acc1);
                        }
                        cur_leaf = lfs[sl];
                        cur_v0 = B.vid[sl][ek0];
                        cur_v1 = B.vid[sl][ek0 + 4];
                        acc0 = 0.f;
                        acc1 = 0.f;
                    }
                    acc0 += wa[sl] * gv[sl];
                    acc1 += wb[sl] * gv[sl];
                }
            }
        }
    }
    if (EMB && cur_leaf >= 0) {
        atomicAdd(grad_emb + (int64_t)cur_v0 * 16 + ed, acc0);
        atomicAdd(grad_emb + (int64_t)cur_v1 * 16 + ed, acc1);
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        float x = go[a], y = gd[a];
#pragma unroll
        for (int sh = 32; sh > 0; sh >>= 1) {
            x += __shfl_xor(x, sh, 64);
            y += __shfl_xor(y, sh, 64);
        }
        go[a] = x;
        gd[a] = y;
    }
    if (lane == 0) {
        if (chunk) {
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                part[u * 6 + a] = go[a];
                part[u * 6 + 3 + a] = gd[a];
            }
        } else {
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                grad_o[ro_row * 3 + a] = go[a];
                grad_d[ro_row * 3 + a] = gd[a];
            }
        }
    }
}

// d_o / d_d of each ray = its chunks' partials summed in chunk order
__global__ __launch_bounds__(256) void k_interp_bwd_rays(int64_t r_hit, int c_max, const int *__restrict__ ray_index,
                                                         const float *__restrict__ part, float *__restrict__ grad_o,
                                                         float *__restrict__ grad_d) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= r_hit * 6) return;
    const int64_t r = e / 6;
    const int k = (int)(e - r * 6);
    float v = 0.f;
    for (int c = 0; c < c_max; ++c) v += part[(r * c_max + c) * 6 + k];
    const int64_t row = ray_index ? ray_index[r] : r;
    if (k < 3) grad_o[row * 3 + k] = v;
    else grad_d[row * 3 + k - 3] = v;
}

// d_o / d_d of each ray from its samples' dL/dx (the fused decoder backward's
// InterpFuse::gx): one wave per ray, lane l sums samples l, l + 64, ... in
// order, then a fixed shuffle tree — deterministic
__global__ __launch_bounds__(256) void k_interp_rays_gx(int64_t r_hit, const int *__restrict__ offsets,
                                                        const int *__restrict__ ray_index, const float *__restrict__ t,
                                                        const float *__restrict__ gx, float *__restrict__ grad_o,
                                                        float *__restrict__ grad_d, const int *__restrict__ offsets2,
                                                        const float *__restrict__ t2, const float *__restrict__ gx2) {
    const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (r >= r_hit) return;
    const int lane = threadIdx.x & 63;
    float go[3] = {0.f, 0.f, 0.f}, gd[3] = {0.f, 0.f, 0.f};
    for (int seg = 0; seg < (offsets2 ? 2 : 1); ++seg) {
        const int *of = seg ? offsets2 : offsets;
        const float *ts_ = seg ? t2 : t, *gx_ = seg ? gx2 : gx;
        const int beg = of[r], end = of[r + 1];
        for (int s = beg + lane; s < end; s += 64) {
            const float ts = ts_[s];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const float v = gx_[(int64_t)s * 3 + a];
                go[a] += v;
                gd[a] += v * ts;
            }
        }
    }
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int sh = 32; sh > 0; sh >>= 1) {
            go[a] += __shfl_xor(go[a], sh, 64);
            gd[a] += __shfl_xor(gd[a], sh, 64);
        }
    if (lane == 0) {
        const int64_t row = ray_index ? ray_index[r] : r;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            grad_o[row * 3 + a] = go[a];
            grad_d[row * 3 + a] = gd[a];
        }
    }
}

}  // namespace

int interp_rays_gx(hipStream_t st, int64_t r_hit, const int *offsets, const int *ray_index, const float *t,
                   const float *gx, float *grad_o, float *grad_d, const int *offsets2, const float *t2,
                   const float *gx2) {
    if (r_hit == 0) return PSVO_OK;
    psvo::launch(k_interp_rays_gx, dim3(div_up(r_hit, 4)), dim3(256), 0, st, r_hit, offsets, ray_index, t, gx,
                 grad_o, grad_d, offsets2, t2, gx2);
    return check_launch("interp_rays_gx");
}
}  // namespace psvo

using namespace psvo;

extern "C" int psvo_interp_fwd(void *stream, int64_t m, int d, float voxel_size, const int *leaf, const float *t,
                               const int *ray_of_sample, const int *ray_index, const float *rays_o, const float *rays_d,
                               const float *centres, const int *vertex_idx, const float *emb, float *feat) {
    PSVO_REQUIRE(d == 16, "interp_fwd: embedding dim %d unsupported (16 only)", d);
    PSVO_REQUIRE(m >= 0 && voxel_size > 0.f, "interp_fwd: bad sizes");
    if (m == 0) return PSVO_OK;
    psvo::launch(k_interp_fwd, dim3(div_up(m * 4, 256)), dim3(256), 0, as_stream(stream), m, voxel_size, leaf,
                       t, ray_of_sample, ray_index, rays_o, rays_d, centres, vertex_idx,
                       reinterpret_cast<const float4 *>(emb),
                       reinterpret_cast<float4 *>(feat), static_cast<const int *>(nullptr));
    return check_launch("interp_fwd");
}

namespace psvo {
// the interpolation over m_dev ≤ m_cap samples (the count on the device):
// one pass over at most 4,096 workgroups, striding
int interp_fwd_dev(hipStream_t st, int64_t m_cap, const int *m_dev, float voxel_size, const int *leaf, const float *t,
                   const int *ray_of_sample, const int *ray_index, const float *rays_o, const float *rays_d,
                   const float *centres, const int *vertex_idx, const float *emb, float *feat) {
    PSVO_REQUIRE(m_cap >= 0 && m_dev && voxel_size > 0.f, "interp_fwd_dev: bad arguments");
    if (m_cap == 0) return PSVO_OK;
    const int64_t blocks = div_up(m_cap * 4, 256);
    psvo::launch(k_interp_fwd, dim3((int)(blocks < 4096 ? blocks : 4096)), dim3(256), 0, st, m_cap, voxel_size, leaf,
                 t, ray_of_sample, ray_index, rays_o, rays_d, centres, vertex_idx,
                 reinterpret_cast<const float4 *>(emb), reinterpret_cast<float4 *>(feat), m_dev);
    return check_launch("interp_fwd_dev");
}
}  // namespace psvo


extern "C" int psvo_interp_bwd(void *stream, int64_t r_hit, int d, float voxel_size, const int *offsets,
                               const int *ray_index, const int *leaf, const float *t, const float *rays_o, const float *rays_d,
                               const float *centres, const int *vertex_idx, const float *emb,
                               const float *grad_feat, float *grad_emb, float *grad_o, float *grad_d) {
    PSVO_REQUIRE(d == 16, "interp_bwd: embedding dim %d unsupported (16 only)", d);
    PSVO_REQUIRE(r_hit >= 0 && voxel_size > 0.f, "interp_bwd: bad sizes");
    PSVO_REQUIRE(grad_o != nullptr && grad_d != nullptr, "interp_bwd: grad_o / grad_d required");
    if (r_hit == 0) return PSVO_OK;
    if (grad_emb)
        psvo::launch(k_interp_bwd<true>, dim3(div_up(r_hit, kIbWaves)), dim3(64 * kIbWaves), 0, as_stream(stream), r_hit,
                           voxel_size, offsets, ray_index, leaf, t, rays_o, rays_d, centres, vertex_idx,
                           reinterpret_cast<const float4 *>(emb), reinterpret_cast<const float4 *>(grad_feat),
                           grad_emb, grad_o, grad_d, 0, 1, nullptr);
    else
        psvo::launch(k_interp_bwd<false>, dim3(div_up(r_hit, kIbWaves)), dim3(64 * kIbWaves), 0, as_stream(stream), r_hit,
                           voxel_size, offsets, ray_index, leaf, t, rays_o, rays_d, centres, vertex_idx,
                           reinterpret_cast<const float4 *>(emb), reinterpret_cast<const float4 *>(grad_feat),
                           nullptr, grad_o, grad_d, 0, 1, nullptr);
    return check_launch("interp_bwd");
}

extern "C" int64_t psvo_interp_bwd_workspace_floats(int64_t r_hit, int s_max) {
    return r_hit * ((s_max + kInterpChunk - 1) / kInterpChunk) * 6;
}

extern "C" int psvo_interp_bwd_chunked(void *stream, int64_t r_hit, int s_max, int d, float voxel_size,
                                       const int *offsets, const int *ray_index, const int *leaf, const float *t,
                                       const float *rays_o, const float *rays_d, const float *centres,
                                       const int *vertex_idx, const float *emb, const float *grad_feat,
                                       float *grad_emb, float *grad_o, float *grad_d, float *workspace) {
    PSVO_REQUIRE(d == 16, "interp_bwd: embedding dim %d unsupported (16 only)", d);
    PSVO_REQUIRE(r_hit >= 0 && s_max > 0 && voxel_size > 0.f, "interp_bwd: bad sizes");
    PSVO_REQUIRE(grad_o != nullptr && grad_d != nullptr && workspace != nullptr,
                 "interp_bwd: grad_o / grad_d / workspace required");
    if (r_hit == 0) return PSVO_OK;
    const int c_max = (s_max + kInterpChunk - 1) / kInterpChunk;
    const int64_t units = r_hit * c_max;
    hipStream_t st = as_stream(stream);
    if (grad_emb)
        psvo::launch(k_interp_bwd<true>, dim3(div_up(units, kIbWaves)), dim3(64 * kIbWaves), 0, st, r_hit, voxel_size, offsets,
                           ray_index, leaf, t, rays_o, rays_d, centres, vertex_idx,
                           reinterpret_cast<const float4 *>(emb), reinterpret_cast<const float4 *>(grad_feat),
                           grad_emb, grad_o, grad_d, kInterpChunk, c_max, workspace);
    else
        psvo::launch(k_interp_bwd<false>, dim3(div_up(units, kIbWaves)), dim3(64 * kIbWaves), 0, st, r_hit, voxel_size, offsets,
                           ray_index, leaf, t, rays_o, rays_d, centres, vertex_idx,
                           reinterpret_cast<const float4 *>(emb), reinterpret_cast<const float4 *>(grad_feat),
                           nullptr, grad_o, grad_d, kInterpChunk, c_max, workspace);
    psvo::launch(k_interp_bwd_rays, dim3(div_up(r_hit * 6, 256)), dim3(256), 0, st, r_hit, c_max, ray_index,
                       workspace, grad_o, grad_d);
    return check_launch("interp_bwd_chunked");
}
