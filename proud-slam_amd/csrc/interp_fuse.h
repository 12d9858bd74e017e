// The interpolation backward (interp.hip's k_interp_bwd arithmetic) of one
// 16-sample unit on a decoder δ-chain wave, shared by the fused width-128
// (mlp.hip k_mlp_bwd3) and width-256 (mlp256.hip k_dec256_bwd) backwards:
// lane (n, q) holds sample n's dfeat dims 4q..4q+3 in both chains.
#pragma once

#include "psvo_common.h"

namespace psvo {
namespace ifuse {

constexpr int kU = 16;  // samples per chain unit

// The interpolation backward of one 16-sample unit on its chain wave (see
// k_mlp_bwd3): lane (n, q) holds sample n's dfeat dims 4q..4q+3 — k_interp_bwd's
// 4-lanes-per-sample layout, the same arithmetic (roundings spelled out as in
// interp.hip's contract(off)).  dL/dx goes to ip.gx; the embedding scatter's
// operands (w [8][16], g [16][16], vid [16][8]) are staged in `stg` for
// scatter_unit (the same wave, right after).
__device__ __forceinline__ void interp_bwd_unit(const InterpFuse &ip, float *stg, int64_t m, int64_t s, bool valid,
                                                int n, int q, float ts, const float (&o)[3], const float (&d)[3],
                                                const float (&cen)[3], int4 vid0, int4 vid1, const float4 (&ev)[8],
                                                float4 g) {
    float p[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float x = __fadd_rn(o[a], __fmul_rn(d[a], ts));
        p[a] = __fadd_rn(__fdiv_rn(__fsub_rn(x, cen[a]), ip.voxel_size), 0.5f);
    }
    const float ax[2] = {__fsub_rn(1.0f, p[0]), p[0]};
    const float ay[2] = {__fsub_rn(1.0f, p[1]), p[1]};
    const float az[2] = {__fsub_rn(1.0f, p[2]), p[2]};
    if (!valid) g = make_float4(0.f, 0.f, 0.f, 0.f);
    // dL/dx: eg_k = E[vid_k] · g over the sample's 4 lanes (n + 16q)
    float eg[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const float4 e = ev[k];
        float a = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(e.x, g.x), __fmul_rn(e.y, g.y)), __fmul_rn(e.z, g.z)),
                            __fmul_rn(e.w, g.w));
        a = __fadd_rn(a, __shfl_xor(a, 16, 64));
        a = __fadd_rn(a, __shfl_xor(a, 32, 64));
        eg[k] = a;
    }
    if (valid && q == 0) {
        float dp[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int ix = (k >> 2) & 1, iy = (k >> 1) & 1, iz = k & 1;
            const float sx = ix ? 1.f : -1.f, sy = iy ? 1.f : -1.f, sz = iz ? 1.f : -1.f;
            dp[0] = __fadd_rn(dp[0], __fmul_rn(__fmul_rn(__fmul_rn(sx, ay[iy]), az[iz]), eg[k]));
            dp[1] = __fadd_rn(dp[1], __fmul_rn(__fmul_rn(__fmul_rn(sy, ax[ix]), az[iz]), eg[k]));
            dp[2] = __fadd_rn(dp[2], __fmul_rn(__fmul_rn(__fmul_rn(sz, ax[ix]), ay[iy]), eg[k]));
        }
#pragma unroll
        for (int a = 0; a < 3; ++a) ip.gx[s * 3 + a] = __fdiv_rn(dp[a], ip.voxel_size);
    }
    if (ip.grad_emb == nullptr) return;
    // the scatter's operands: this lane's weights w[2q], w[2q + 1] and vertex rows
    float *Bw = stg, *Bg = stg + 128;
    int *Bv = reinterpret_cast<int *>(stg + 384);
    const int k0 = 2 * q, k1 = 2 * q + 1;
    const float w0 = __fmul_rn(__fmul_rn(ax[(k0 >> 2) & 1], ay[(k0 >> 1) & 1]), az[k0 & 1]);
    const float w1 = __fmul_rn(__fmul_rn(ax[(k1 >> 2) & 1], ay[(k1 >> 1) & 1]), az[k1 & 1]);
    Bg[(4 * q + 0) * 16 + n] = g.x;
    Bg[(4 * q + 1) * 16 + n] = g.y;
    Bg[(4 * q + 2) * 16 + n] = g.z;
    Bg[(4 * q + 3) * 16 + n] = g.w;
    Bw[k0 * 16 + n] = w0;
    Bw[k1 * 16 + n] = w1;
    Bv[n * 8 + k0] = q == 0 ? vid0.x : q == 1 ? vid0.z : q == 2 ? vid1.x : vid1.z;
    Bv[n * 8 + k1] = q == 0 ? vid0.y : q == 1 ? vid0.w : q == 2 ? vid1.y : vid1.w;
}

// The embedding scatter of one staged unit (interp_bwd_unit), summed per
// leaf run first (k_interp_bwd's scheme): lane j owns corners j >> 4 and
// (j >> 4) + 4 of dim j & 15, so a flush is two atomic instructions each
// covering four whole 64-B rows.
// `lf`: this lane's sample leaf (lane n holds sample n's: read with readlane,
// no memory access on the run loop's critical path)
__device__ __forceinline__ void scatter_unit(const InterpFuse &ip, const float *stg, int64_t u, int64_t m, int lane,
                                             int lf_lane) {
    const float *Bw = stg, *Bg = stg + 128;
    const int *Bv = reinterpret_cast<const int *>(stg + 384);
    const int64_t left = m - u * kU;
    const int n_slots = (int)(left < kU ? left : kU);
    const int ek0 = lane >> 4, ed = lane & 15;
    int cur = -1, cv0 = 0, cv1 = 0;
    float acc0 = 0.f, acc1 = 0.f;
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4) {  // four slots per LDS read (few live registers)
        if (4 * c4 >= n_slots) break;
        const float4 a4 = *reinterpret_cast<const float4 *>(Bw + ek0 * 16 + 4 * c4);
        const float4 b4 = *reinterpret_cast<const float4 *>(Bw + (ek0 + 4) * 16 + 4 * c4);
        const float4 g4 = *reinterpret_cast<const float4 *>(Bg + ed * 16 + 4 * c4);
        const float wa[4] = {a4.x, a4.y, a4.z, a4.w}, wb[4] = {b4.x, b4.y, b4.z, b4.w},
                    gv[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int sl = 4 * c4 + j;
            if (sl < n_slots) {
                const int lf = __builtin_amdgcn_readlane(lf_lane, sl);
                if (lf != cur) {
                    if (cur >= 0) {
                        atomicAdd(ip.grad_emb + (int64_t)cv0 * 16 + ed, acc0);
                        atomicAdd(ip.grad_emb + (int64_t)cv1 * 16 + ed, acc1);
                    }
                    cur = lf;
                    cv0 = Bv[sl * 8 + ek0];
                    cv1 = Bv[sl * 8 + ek0 + 4];
                    if (ip.row_flags != nullptr && ed == 0) {  // the rows this step touches (psvo_adam_mark_rows' set)
                        ip.row_flags[cv0] = 1;
                        ip.row_flags[cv1] = 1;
                    }
                    acc0 = 0.f;
                    acc1 = 0.f;
                }
                acc0 = __fadd_rn(acc0, __fmul_rn(wa[j], gv[j]));
                acc1 = __fadd_rn(acc1, __fmul_rn(wb[j], gv[j]));
            }
        }
    }
    if (cur >= 0) {
        atomicAdd(ip.grad_emb + (int64_t)cv0 * 16 + ed, acc0);
        atomicAdd(ip.grad_emb + (int64_t)cv1 * 16 + ed, acc1);
    }
}

}  // namespace ifuse
}  // namespace psvo
