// SDF-to-weight compositing per hit ray (forward + backward) on gfx950.
//
// Reference: render_helpers.py:504-556 —
//   sdf    = masked_scatter_ones(mask, sdf_s)        [R_hit, S]  (pad 1)
//   colour = masked_scatter(mask, rgb_s)              [R_hit, S, 3] (pad 0)
//   u      = σ(sdf/tr)·σ(-sdf/tr)
//   ind    = argmax(sdf[:,1:]·sdf[:,:-1] < 0)  (first sign change, 0 if none)
//   z_min  = z[ind];  w = u · [z < z_min + tr] · valid;  w /= Σw + 1e-8
//   rgb    = Σ w·colour;  depth = Σ w·z
// and the backward torch autograd derives for it (ind / the masks carry no
// gradient; padded sdf entries are constants).
//
// One wave per ray: a ray's S_max (≈100–600) samples stream through the 64
// lanes in strides; reductions are wave shuffles, so no LDS and no atomics.
#include <hip/hip_runtime.h>

#include "lookback.h"
#include "psvo_common.h"

namespace psvo {
namespace {

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) v += __shfl_xor(v, s, 64);
    return v;
}
__device__ __forceinline__ int wmin(int v) {
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) v = min(v, __shfl_xor(v, s, 64));
    return v;
}
__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// Backward per-sample pieces shared by k_composite_bwd and k_composite_loss,
// with the roundings spelled out (fmaf), so both kernels produce the same
// bits whatever the compiler would contract in either context.
// dL/dW_s = g_depth·z_s + g_w,s (+ g_colour·c_s for a valid sample)
__device__ __forceinline__ float comp_gw3(float gdp, float z, float gwx, bool has_c, float c0, float c1, float c2,
                                          float gr, float gg, float gb) {
    const float g = fmaf(gdp, z, gwx);
    return has_c ? fmaf(gb, c2, fmaf(gg, c1, fmaf(gr, c0, g))) : g;
}
__device__ __forceinline__ float comp_gw(float gdp, float z, float gwx, const float *c, float gr, float gg, float gb) {
    return c ? comp_gw3(gdp, z, gwx, true, c[0], c[1], c[2], gr, gg, gb) : comp_gw3(gdp, z, gwx, false, 0.f, 0.f,
                                                                                   0.f, gr, gg, gb);
}
// dL/dsdf_s through the weights (kept samples) plus the direct term g
__device__ __forceinline__ float comp_gsdf_sig(float gw, float dot, float tot, bool keep, float sp, float sn, float tr,
                                               float g) {
    const float gu = keep ? (gw - dot) / tot : 0.f;
    const float du = sp * sn * (sn - sp) / tr;
    return fmaf(gu, du, g);
}
__device__ __forceinline__ float comp_gsdf(float gw, float dot, float tot, bool keep, float sdf, float tr, float g) {
    const float a = sdf / tr;
    return comp_gsdf_sig(gw, dot, tot, keep, sigm(a), sigm(-a), tr, g);
}

__global__ __launch_bounds__(256) void k_composite_fwd(int64_t r_hit, int s_max, float tr,
                                                       const int *__restrict__ offsets,
                                                       const int *__restrict__ ray_ns,
                                                       const float *__restrict__ z_vals,
                                                       const float *__restrict__ sdf_s,
                                                       const float *__restrict__ rgb_s, float *__restrict__ sdf,
                                                       float *__restrict__ weights, float *__restrict__ color,
                                                       float *__restrict__ depth, float *__restrict__ z_min_out) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (r >= r_hit) return;
    const int off = offsets[r], ns = ray_ns[r];
    const float *z = z_vals + r * s_max;
    float *sd = sdf + r * s_max;
    float *wt = weights + r * s_max;
    // pass 1: padded sdf row + first sign change
    int first = s_max;
    for (int s = lane; s < s_max; s += 64) {
        const float v = s < ns ? sdf_s[off + s] : 1.0f;
        sd[s] = v;
        if (s + 1 < s_max) {
            const float v1 = (s + 1) < ns ? sdf_s[off + s + 1] : 1.0f;
            if (v1 * v < 0.0f) first = min(first, s);
        }
    }
    first = wmin(first);
    const int ind = first == s_max ? 0 : first;
    const float zmin = z[ind];
    // pass 2: unnormalised weights and their sum
    float tot = 0.f;
    for (int s = lane; s < s_max; s += 64) {
        const float v = sd[s];
        const float a = v / tr;
        float w = sigm(a) * sigm(-a);
        const bool keep = (z[s] < zmin + tr) && (s < ns);
        w = keep ? w : 0.0f;
        wt[s] = w;
        tot += w;
    }
    tot = wsum(tot) + 1e-8f;
    float cr = 0.f, cg = 0.f, cb = 0.f, dd = 0.f;
    for (int s = lane; s < s_max; s += 64) {
        const float w = wt[s] / tot;
        wt[s] = w;
        if (s < ns) {
            const float *c = rgb_s + (int64_t)(off + s) * 3;
            cr += w * c[0];
            cg += w * c[1];
            cb += w * c[2];
        }
        dd += w * z[s];
    }
    cr = wsum(cr);
    cg = wsum(cg);
    cb = wsum(cb);
    dd = wsum(dd);
    if (lane == 0) {
        color[r * 3 + 0] = cr;
        color[r * 3 + 1] = cg;
        color[r * 3 + 2] = cb;
        depth[r] = dd;
        if (z_min_out) z_min_out[r] = zmin;
    }
}

__global__ __launch_bounds__(256) void k_composite_bwd(int64_t r_hit, int s_max, float tr,
                                                       const int *__restrict__ offsets,
                                                       const int *__restrict__ ray_ns,
                                                       const float *__restrict__ z_vals,
                                                       const float *__restrict__ sdf,
                                                       const float *__restrict__ weights,
                                                       const float *__restrict__ rgb_s,
                                                       const float *__restrict__ g_color,
                                                       const float *__restrict__ g_depth,
                                                       const float *__restrict__ g_weights,
                                                       const float *__restrict__ g_sdf,
                                                       float *__restrict__ g_sdf_s, float *__restrict__ g_rgb_s) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (r >= r_hit) return;
    const int off = offsets[r], ns = ray_ns[r];
    const float *z = z_vals + r * s_max;
    const float *sd = sdf + r * s_max;
    const float *wt = weights + r * s_max;
    const float gr = g_color ? g_color[r * 3 + 0] : 0.f;
    const float gg = g_color ? g_color[r * 3 + 1] : 0.f;
    const float gb = g_color ? g_color[r * 3 + 2] : 0.f;
    const float gdp = g_depth ? g_depth[r] : 0.f;
    // dL/dW_s and Σ_s dL/dW_s · W_s
    float dot = 0.f, tot = 0.f;
    for (int s = lane; s < s_max; s += 64) {
        const float gw = comp_gw(gdp, z[s], g_weights ? g_weights[r * s_max + s] : 0.f,
                                 s < ns ? rgb_s + (int64_t)(off + s) * 3 : nullptr, gr, gg, gb);
        dot = fmaf(gw, wt[s], dot);
    }
    dot = wsum(dot);
    // T = Σ_kept u + 1e-8, the forward's normaliser (W_s = w_s / T); the
    // kept set is recomputed from the padded sdf row exactly as the forward.
    int first = s_max;
    for (int s = lane; s < s_max; s += 64) {
        if (s + 1 < s_max && sd[s + 1] * sd[s] < 0.0f) first = min(first, s);
    }
    first = wmin(first);
    const float zmin = z[first == s_max ? 0 : first];
    for (int s = lane; s < s_max; s += 64) {
        const float a = sd[s] / tr;
        const bool keep = (z[s] < zmin + tr) && (s < ns);
        tot += keep ? sigm(a) * sigm(-a) : 0.f;
    }
    tot = wsum(tot) + 1e-8f;
    for (int s = lane; s < ns; s += 64) {
        const float *c = rgb_s + (int64_t)(off + s) * 3;
        const float W = wt[s];
        const float gw = comp_gw(gdp, z[s], g_weights ? g_weights[r * s_max + s] : 0.f, c, gr, gg, gb);
        g_sdf_s[off + s] = comp_gsdf(gw, dot, tot, z[s] < zmin + tr, sd[s], tr, g_sdf ? g_sdf[r * s_max + s] : 0.f);
        float *gc = g_rgb_s + (int64_t)(off + s) * 3;
        gc[0] = W * gr;
        gc[1] = W * gg;
        gc[2] = W * gb;
    }
}

// Mapping step: compositing (k_composite_fwd), the Criterion's per-ray
// partial sums (k_crit_rays' colour / depth / fs / sdf slots; the count
// slots come from k_crit_counts), its backward with the precomputed
// coefficients (k_crit_bwd at d loss = 1) and the compositing backward
// (k_composite_bwd) in one wave per ray — the same arithmetic, four launches
// and the padded [R_hit, S_max] sdf / weight rows fewer.
//   coef = {c_colour, c_depth, c_fs, c_sdf} (k_crit_coef)
constexpr int kPartColor = 0, kPartDepth = 1, kPartQFs = 5, kPartQSdf = 6, kPartN = 8;

// criterion.hip's sample_terms, with its no-contraction arithmetic
struct CritTerms {
    float f, sm, xfs, ysdf;
};
__device__ __forceinline__ CritTerms crit_terms(float z, float p, float d, float tr, float max_depth) {
#pragma clang fp contract(off)
    CritTerms o;
    o.f = z < (d - tr) ? 1.0f : 0.0f;
    const float b = z > (d + tr) ? 1.0f : 0.0f;
    const float dm = (d > 0.0f && d < max_depth) ? 1.0f : 0.0f;
    o.sm = (1.0f - o.f) * (1.0f - b) * dm;
    o.xfs = p * o.f - o.f;
    o.ysdf = (z + p * tr) * o.sm - d * o.sm;
    return o;
}
__device__ __forceinline__ float crit_sq_add(float acc, float x) {
#pragma clang fp contract(off)
    return acc + x * x;
}
__device__ __forceinline__ float crit_grad(float cfs, float csdf, const CritTerms &t) {
#pragma clang fp contract(off)
    return cfs * t.xfs * t.f + csdf * t.ysdf * t.sm;
}

// J > 0: a ray's samples (s_max ≤ 64·J) are read once into registers —
// sample s = lane + 64j in slot j — and every pass runs from them; J = 0
// re-reads memory per pass (any s_max).  Same operations in the same order.
template <int J>
__global__ __launch_bounds__(256) void k_composite_loss(int64_t r_hit, int s_max, float tr, float max_depth,
                                                        const int *__restrict__ offsets,
                                                        const int *__restrict__ ray_ns,
                                                        const float *__restrict__ z_vals, int z_stride,
                                                        const int *__restrict__ rank_ray,
                                                        const float *__restrict__ gt_rgb,
                                                        const float *__restrict__ gt_depth,
                                                        const float *__restrict__ sdf_s,
                                                        const float *__restrict__ rgb_s,
                                                        const float *__restrict__ coef, float *__restrict__ part,
                                                        float *__restrict__ color, float *__restrict__ depth,
                                                        float *__restrict__ g_sdf_s, float *__restrict__ g_rgb_s,
                                                        int partials, const int *__restrict__ cidx) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (r >= r_hit) return;
    // the ray's ground truth and the coefficients depend on nothing computed
    // here: their loads go out first, beside the sample loads
    const int64_t orig = rank_ray[r];
    const int off = offsets[r], ns = ray_ns[r];
    // past the ray's ns valid samples every pass adds nothing (weights 0, no
    // sign change between padding sdfs of 1, colours masked): those passes
    // stop at ns — the same bits — and only the loss partials, which count
    // the padded samples (criterion.py:70-101), run to s_max
    const int lim = ns < s_max ? ns : s_max;
    const float d = gt_depth[orig];
    const float gt0 = gt_rgb[orig * 3 + 0], gt1 = gt_rgb[orig * 3 + 1], gt2 = gt_rgb[orig * 3 + 2];
    const float ccol = coef[0], cdep = coef[1], cfs = coef[2], csdf = coef[3];
    // the sampler row ([R, cap]: past its ns valid samples the padding
    // MAX_DEPTH is implied, the look-back sampler does not write it) or the
    // padded [R_hit, S_max] row
    const float *z = z_vals + r * z_stride;
    auto z_at = [&](int s) { return s < ns ? z[s] : kMaxDepthFill; };
    auto sdf_at = [&](int s) { return s < ns ? sdf_s[off + s] : 1.0f; };  // padded row (pad 1)
    // cidx (the sparse decoder, k_select_samples): the decoder ran on the
    // samples the backward needs only — sample s's colour and its gradients
    // live at cidx[off + s], and -1 marks a sample whose weight and loss
    // terms are zero (no colour read, no gradient written: both are 0)
    auto ci_at = [&](int s) { return s < ns ? (cidx ? cidx[off + s] : off + s) : -1; };
    constexpr int JR = J > 0 ? J : 1;
    float zr[JR], pr[JR], c0r[JR], c1r[JR], c2r[JR];
    if constexpr (J > 0) {
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int s = lane + 64 * j;
            zr[j] = s < s_max ? z_at(s) : 0.f;
            pr[j] = sdf_at(s);
            const int ci = ci_at(s);
            const bool v = ci >= 0;
            const float *c = rgb_s + (int64_t)(v ? ci : 0) * 3;
            c0r[j] = v ? c[0] : 0.f;
            c1r[j] = v ? c[1] : 0.f;
            c2r[j] = v ? c[2] : 0.f;
        }
    }
    auto Z = [&](int j, int s) {
        if constexpr (J > 0) return zr[j]; else return z_at(s);
    };
    auto P = [&](int j, int s) {
        if constexpr (J > 0) return pr[j]; else return sdf_at(s);
    };
    auto C = [&](int j, int s, int k) {
        if constexpr (J > 0) return k == 0 ? c0r[j] : (k == 1 ? c1r[j] : c2r[j]);
        else {
            const int ci = ci_at(s);
            return ci >= 0 ? rgb_s[(int64_t)ci * 3 + k] : 0.f;
        }
    };
#define PSVO_FOR_S(lim) for (int j = 0, s = lane; (J == 0 || j < J) && s < (lim); ++j, s += 64)
    // ---- forward (k_composite_fwd)
    // sdf of sample s + 1 (J > 0: the next lane's, or lane 0's of the next
    // slot — exchanged with every lane active, before the per-lane loops)
    float pn[JR];
    if constexpr (J > 0) {
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const float dn = __shfl_down(pr[j], 1, 64);
            const float nx = __shfl(pr[j + 1 < J ? j + 1 : j], 0, 64);
            pn[j] = lane < 63 ? dn : nx;
        }
    }
    int first = s_max;
    PSVO_FOR_S(lim) {
        const float v = P(j, s);
        float v1;
        if constexpr (J > 0) v1 = pn[j];
        else v1 = s + 1 < s_max ? sdf_at(s + 1) : 0.f;
        if (s + 1 < s_max && v1 * v < 0.0f) first = min(first, s);
    }
    first = wmin(first);
    const float zmin = z_at(first == s_max ? 0 : first);
    // σ(a), σ(−a) per sample (registers when J > 0: computed once, the same
    // bits as recomputing them in each pass)
    float spr[JR], snr[JR], wr[JR];
#pragma unroll
    for (int j = 0; j < JR; ++j) spr[j] = snr[j] = wr[j] = 0.f;
    float tot = 0.f;
    PSVO_FOR_S(lim) {
        const float a = P(j, s) / tr;
        const float sp = sigm(a), sn = sigm(-a);
        float w = sp * sn;
        const bool keep = (Z(j, s) < zmin + tr) && (s < ns);
        tot += keep ? w : 0.0f;
        if constexpr (J > 0) {
            spr[j] = sp;
            snr[j] = sn;
            wr[j] = keep ? w : 0.0f;
        }
    }
    tot = wsum(tot) + 1e-8f;
    if constexpr (J > 0) {
#pragma unroll
        for (int j = 0; j < J; ++j) wr[j] = wr[j] / tot;
    }
    auto weight_at = [&](int j, int s) {  // normalised weight W_s (0 outside the kept set)
        if constexpr (J > 0) {
            return wr[j];
        } else {
            const float a = P(j, s) / tr;
            const float w = sigm(a) * sigm(-a);
            const bool keep = (Z(j, s) < zmin + tr) && (s < ns);
            return (keep ? w : 0.0f) / tot;
        }
    };
    float cr = 0.f, cg = 0.f, cb = 0.f, dd = 0.f;
    PSVO_FOR_S(lim) {
        const float w = weight_at(j, s);
        if (s < ns) {
            cr += w * C(j, s, 0);
            cg += w * C(j, s, 1);
            cb += w * C(j, s, 2);
        }
        dd += w * Z(j, s);
    }
    cr = wsum(cr);
    cg = wsum(cg);
    cb = wsum(cb);
    dd = wsum(dd);
    // ---- loss partials (k_crit_rays) and d loss / d {colour, depth} (k_crit_bwd)
    float qfs = 0.f, qsdf = 0.f;
    if (partials) {  // the loss value's (not on the gradient path)
        PSVO_FOR_S(s_max) {
            const CritTerms t = crit_terms(Z(j, s), P(j, s), d, tr, max_depth);
            qfs = crit_sq_add(qfs, t.xfs);
            qsdf = crit_sq_add(qsdf, t.ysdf);
        }
        qfs = wsum(qfs);
        qsdf = wsum(qsdf);
    }
    const float rgb[3] = {cr, cg, cb};
    const float gt[3] = {gt0, gt1, gt2};
    float gcol[3], ac = 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float e = gt[c] - rgb[c];
        ac += fabsf(e);
        gcol[c] = -ccol * (e > 0.0f ? 1.0f : (e < 0.0f ? -1.0f : 0.0f));
    }
    const bool valid = d > 0.01f && d < max_depth;
    const float ed = d - dd;
    const float gdp = valid ? -cdep * (ed > 0.0f ? 1.0f : (ed < 0.0f ? -1.0f : 0.0f)) : 0.0f;
    if (lane == 0) {
        color[r * 3 + 0] = cr;
        color[r * 3 + 1] = cg;
        color[r * 3 + 2] = cb;
        depth[r] = dd;
        if (partials) {
            float *o = part + r * kPartN;
            o[kPartColor] = ac;
            o[kPartDepth] = valid ? fabsf(ed) : 0.0f;
            o[kPartQFs] = qfs;
            o[kPartQSdf] = qsdf;
            o[7] = 0.0f;
        }
    }
    // ---- compositing backward (k_composite_bwd, g_weights = 0)
    float dot = 0.f;
    PSVO_FOR_S(lim) {
        const bool v = s < ns;
        const float gw = comp_gw3(gdp, Z(j, s), 0.f, v, v ? C(j, s, 0) : 0.f, v ? C(j, s, 1) : 0.f,
                                  v ? C(j, s, 2) : 0.f, gcol[0], gcol[1], gcol[2]);
        dot = fmaf(gw, weight_at(j, s), dot);
    }
    dot = wsum(dot);
    PSVO_FOR_S(ns) {
        const float W = weight_at(j, s);
        const float zs = Z(j, s);
        const float gw = comp_gw3(gdp, zs, 0.f, true, C(j, s, 0), C(j, s, 1), C(j, s, 2), gcol[0], gcol[1], gcol[2]);
        const float p = P(j, s);
        const float gsdf = crit_grad(cfs, csdf, crit_terms(zs, p, d, tr, max_depth));  // k_crit_bwd's term
        const int gi = ci_at(s);
        if (gi < 0) continue;  // a dropped sample: both gradients are exactly 0
        if constexpr (J > 0)
            g_sdf_s[gi] = comp_gsdf_sig(gw, dot, tot, zs < zmin + tr, spr[j], snr[j], tr, gsdf);
        else
            g_sdf_s[gi] = comp_gsdf(gw, dot, tot, zs < zmin + tr, p, tr, gsdf);
        float *gc = g_rgb_s + (int64_t)gi * 3;
        gc[0] = W * gcol[0];
        gc[1] = W * gcol[1];
        gc[2] = W * gcol[2];
    }
#undef PSVO_FOR_S
}


// ---------------------------------------------------------------------------
// The sparse decoder's sample selection (engine): which samples the decoder
// backward needs, and how much of it.  A sample's gradients are exactly zero
// unless
//   - it is composited: z < z_min + tr (render_helpers.py:532-539; the only
//     samples with a weight, so the only ones whose colour reaches the loss,
//     :544, and whose sdf reaches it through the weights), or
//   - it lies in a loss mask: front (z < d − tr) or the sdf band
//     (criterion.py:78-116) — then only its sdf has a gradient (the direct
//     loss term), so its colour head (sdf_out's feature columns, W4, W5) has
//     no gradient and no use: the decoder TRUNK (h1, h2, the sdf row) is all
//     its backward needs.
// The rest (≈ 32 % at config B) get no loss term and no weight.  Class A
// (composited) goes to compact, ray-major indices [0, M_A) — the whole
// decoder runs on them —, class B (kept, not composited) to [cap, cap + M_B)
// — the trunk only (split = 0: every kept sample is class A, e.g. the width-256
// decoder).  cidx[s] is the sample's compact index (-1: dropped); the same
// per-sample arithmetic runs on either class, so the same colours, sdf and
// per-sample gradients: only the weight gradients' summation order changes.
// z_min, the masks and `first` are computed exactly as k_composite_loss
// computes them (same expressions, same padding).
//
// One wave per ray (rpw rays per wave when R_hit > 32,768: the look-back's
// 4,096 workgroups), 8 waves per workgroup (4: 15.7 µs at config B, 8: 14.6,
// 16: 17.4 — profiles/r05b{b,d,c}_kernel_stats.csv); the compact ray offsets of both
// classes by decoupled look-back over {A, B, composited} (lookback.h): one launch.
constexpr int kSelWaves = 8, kSelMaxRpw = 16;
struct SelectArgs {
    const float4 *feat;      // [M][16] the interpolated features (4 float4 per sample)
    const int *leaf, *ray_of;
    const float *t;
    int *cidx;               // [M]
    int *offa, *offb;        // [R_hit + 1] each: the classes' compact ray offsets (offb: split only)
    float4 *feat_c;          // [2 cap][16]: class A rows at [0, M_A), class B at [cap, cap + M_B)
    int *leaf_c, *ray_of_c;  // [2 cap]
    float *t_c;
    float *rgb_c;            // [2 cap][3] (split): class B's colours, written 0 (their weights are 0;
                             // the fused trunk kernel computes no colour head)
    int *src_c;              // [2 cap] or null: each kept sample's row in the step's sample order
    int64_t cap;             // class B's base index (the step's sample count M)
    int split;
    int *counts;             // [0] M_A, [1] M_B, [2] flags (look-back abandoned: bit 3), [3] pad, then u64
                             // running sums of kept / composited samples and of launches
    unsigned long long *desc;  // select_granules(r_hit): the ticket counter, aggregates, tile totals
    uint32_t tag;
    LbCtl ctl;                 // lookback.h (tests: psvo_debug_set_lookback)
    int *host_flag;            // coherent pinned word: bit 3 set by a workgroup that gave up its wait —
                               // the engine reports it at its next host read-back
};

// the ray's z_min (k_composite_loss's first sign change of the padded sdf row)
__device__ __forceinline__ float sel_zmin(int lane, int s_max, int ns, int off, const float *z,
                                          const float *__restrict__ sdf_s) {
    const int lim = ns < s_max ? ns : s_max;
    auto sdf_at = [&](int s) { return s < ns ? sdf_s[off + s] : 1.0f; };
    int first = s_max;
    for (int s = lane; s < lim; s += 64) {
        const float v = sdf_at(s);
        const float v1 = s + 1 < s_max ? sdf_at(s + 1) : 0.f;
        if (s + 1 < s_max && v1 * v < 0.0f) first = min(first, s);
    }
    first = wmin(first);
    const int f0 = first == s_max ? 0 : first;
    return f0 < ns ? z[f0] : kMaxDepthFill;
}

struct SelFlags {
    bool keep, comp;
};
__device__ __forceinline__ SelFlags sel_flags(float zs, float zmin, float d, float tr, float max_depth) {
#pragma clang fp contract(off)
    SelFlags o;
    o.comp = zs < zmin + tr;
    const bool f = zs < (d - tr);
    const bool b = zs > (d + tr);
    const bool dm = d > 0.0f && d < max_depth;
    o.keep = o.comp || f || (!b && dm);
    return o;
}

// look-back blocks this kernel helped (lookback.h; diagnostic: psvo_debug_lb_helps)
__device__ unsigned long long psvo_g_sel_helps;

__global__ __launch_bounds__(512) void k_select_samples(int64_t r_hit, int rpw, int s_max, float tr, float max_depth,
                                                        const int *__restrict__ offsets,
                                                        const int *__restrict__ ray_ns,
                                                        const float *__restrict__ z_vals, int z_stride,
                                                        const int *__restrict__ rank_ray,
                                                        const float *__restrict__ gt_depth,
                                                        const float *__restrict__ sdf_s, SelectArgs a) {
    __shared__ int s_na[kSelWaves * kSelMaxRpw], s_nb[kSelWaves * kSelMaxRpw];
    __shared__ int s_oa[kSelWaves * kSelMaxRpw], s_ob[kSelWaves * kSelMaxRpw];
    __shared__ float s_zmin[kSelWaves * kSelMaxRpw];
    __shared__ int s_nc[kSelWaves], s_base[2];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int blk = (int)blockIdx.x;
    lb_debug_delay(a.ctl, blk);
    if (threadIdx.x == 0) lb_mark_started<3>(a.desc, blk, (int)gridDim.x, a.tag);
    const int64_t r0 = ((int64_t)blk * kSelWaves + w) * rpw;
    const uint64_t below = (1ull << lane) - 1ull;
    const bool split = a.split != 0;
    // ---- count the classes per ray of block `cur` (the own block, or one
    // whose aggregate this workgroup computes for a successor: lookback.h)
    auto count_classes = [&](int cur) {
        const int64_t c0 = ((int64_t)cur * kSelWaves + w) * rpw;
        int nc_w = 0;
        for (int k = 0; k < rpw; ++k) {
            const int64_t r = c0 + k;
            int na = 0, nb = 0;
            float zmin = 0.f;
            if (r < r_hit) {
                const int off = offsets[r], ns = ray_ns[r];
                const float *z = z_vals + r * z_stride;
                const float d = gt_depth[rank_ray[r]];
                zmin = sel_zmin(lane, s_max, ns, off, z, sdf_s);
                for (int s0 = 0; s0 < ns; s0 += 64) {
                    const int s = s0 + lane;
                    SelFlags f{false, false};
                    if (s < ns) f = sel_flags(z[s], zmin, d, tr, max_depth);
                    const int nk = __popcll(__ballot(f.keep)), nc = __popcll(__ballot(f.comp && s < ns));
                    na += split ? nc : nk;
                    nb += split ? nk - nc : 0;
                    nc_w += nc;
                }
            }
            if (lane == 0) {
                s_na[w * rpw + k] = na;
                s_nb[w * rpw + k] = nb;
                s_zmin[w * rpw + k] = zmin;
            }
        }
        if (lane == 0) s_nc[w] = nc_w;
    };
    __shared__ int s_cmd;
    uint32_t own_agg[3] = {0u, 0u, 0u}, own_ex[3] = {0u, 0u, 0u};
    int rc = kLbDone, spins = 0;
    bool helped = false;
    for (int cur = blk;;) {  // pass loop: the own block, then any block helped
        count_classes(cur);
        __syncthreads();
        if (w == 0) {
            const int n_r = kSelWaves * rpw;
            int va = 0, vb = 0;
            for (int i = lane; i < n_r; i += 64) {
                va += s_na[i];
                vb += s_nb[i];
            }
            int c = lane < kSelWaves ? s_nc[lane] : 0;
#pragma unroll
            for (int sh = 32; sh > 0; sh >>= 1) {
                va += __shfl_xor(va, sh, 64);
                vb += __shfl_xor(vb, sh, 64);
                c += __shfl_xor(c, sh, 64);
            }
            const uint32_t agg[3] = {(uint32_t)va, (uint32_t)vb, (uint32_t)c};
            if (cur == blk) {
#pragma unroll
                for (int g = 0; g < 3; ++g) own_agg[g] = agg[g];
            } else {
                lb_publish<3>(a.desc, cur, lane, agg, a.tag);
                if (lane == 0) atomicAdd(&psvo_g_sel_helps, 1ull);
            }
            uint32_t ex[3];
            rc = lb_scan_help<3, 0u>(a.desc, blk, (int)gridDim.x, a.tag, lane, own_agg, ex, spins, a.ctl.spin_max);
            if (rc == kLbDone) {
#pragma unroll
                for (int g = 0; g < 3; ++g) own_ex[g] = ex[g];
            }
            if (lane == 0) s_cmd = rc;
        }
        __syncthreads();
        const int cmd = __builtin_amdgcn_readfirstlane(s_cmd);  // uniform (scalar addressing in the next pass)
        if (cmd < 0) break;
        cur = cmd;
        helped = true;
    }
    if (helped) {  // the LDS counts hold a helped block's: the own block's again
        count_classes(blk);
        __syncthreads();
    }
    if (w == 0 && lane == 0) {
        const bool ok = rc == kLbDone;
        const uint32_t(&ex)[3] = own_ex;
        const uint32_t(&agg)[3] = own_agg;
        s_base[0] = ok ? (int)ex[0] : -1;
        s_base[1] = (int)ex[1];
        if (blk == (int)gridDim.x - 1) {
            const uint32_t ta = ex[0] + agg[0], tb = ex[1] + agg[1], tc = ex[2] + agg[2];
            a.offa[r_hit] = ok ? (int)ta : 0;
            if (split) a.offb[r_hit] = ok ? (int)tb : 0;
            a.counts[0] = ok ? (int)ta : 0;  // an abandoned wait: empty compact batches
            a.counts[1] = ok ? (int)tb : 0;
            a.counts[3] = ok ? (int)tc : 0;  // composited (the statistics; split: = counts[0])
            unsigned long long *sums = reinterpret_cast<unsigned long long *>(a.counts + 4);
            sums[0] += ta + tb;  // one writer per launch, launches stream-ordered
            sums[1] += tc;
            sums[2] += 1;
        }
        if (!ok) {
            atomicOr(a.counts + 2, kLbFlagTimeout);
            if (a.host_flag)
                __hip_atomic_fetch_or(a.host_flag, kLbFlagTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // exclusive ray offsets of the workgroup's rays, per class
        int ra = s_base[0], rb = s_base[1];
        for (int i = 0; i < kSelWaves * rpw; ++i) {
            s_oa[i] = ra;
            s_ob[i] = rb;
            ra += s_na[i];
            rb += s_nb[i];
        }
    }
    __syncthreads();
    if (s_base[0] < 0) {  // the prefix is undefined: the rays' samples dropped, their compact
        // ranges empty or in bounds (the step is reported failed at the next read-back)
        for (int k = 0; k < rpw; ++k) {
            const int64_t r = r0 + k;
            if (r >= r_hit) break;
            const int off = offsets[r], ns = ray_ns[r];
            for (int s = lane; s < ns; s += 64) a.cidx[off + s] = -1;
            if (lane == 0) {
                a.offa[r] = 0;
                if (split) a.offb[r] = 0;
            }
        }
        return;
    }
    // ---- write: compact index of every sample, the kept samples' rows
    for (int k = 0; k < rpw; ++k) {
        const int64_t r = r0 + k;
        if (r >= r_hit) break;
        const int off = offsets[r], ns = ray_ns[r];
        const float *z = z_vals + r * z_stride;
        const float d = gt_depth[rank_ray[r]];
        const float zmin = s_zmin[w * rpw + k];
        int ba = s_oa[w * rpw + k], bb = s_ob[w * rpw + k];
        if (lane == 0) {
            a.offa[r] = ba;
            if (split) a.offb[r] = bb;
        }
        for (int s0 = 0; s0 < ns; s0 += 64) {
            const int s = s0 + lane;
            SelFlags f{false, false};
            if (s < ns) f = sel_flags(z[s], zmin, d, tr, max_depth);
            const bool in_a = split ? (f.comp && s < ns) : f.keep;
            const bool in_b = split && f.keep && !f.comp;
            const uint64_t bal_a = __ballot(in_a), bal_b = __ballot(in_b);
            const int64_t j = in_a ? (int64_t)(ba + __popcll(bal_a & below))
                                   : a.cap + bb + __popcll(bal_b & below);
            if (s < ns) a.cidx[off + s] = (in_a || in_b) ? (int)j : -1;
            if (in_a || in_b) {
                const int64_t src = off + s;
                a.leaf_c[j] = a.leaf[src];
                a.t_c[j] = a.t[src];
                a.ray_of_c[j] = (int)r;
                if (a.src_c) a.src_c[j] = (int)src;
                if (a.feat_c) {  // (null: the consumers read row src_c[j] of the step's features)
#pragma unroll
                    for (int q = 0; q < 4; ++q) a.feat_c[j * 4 + q] = a.feat[src * 4 + q];
                }
                if (in_b) {
#pragma unroll
                    for (int k = 0; k < 3; ++k) a.rgb_c[j * 3 + k] = 0.f;
                }
            }
            ba += __popcll(bal_a);
            bb += __popcll(bal_b);
        }
    }
}

}  // namespace
}  // namespace psvo

using namespace psvo;

extern "C" int psvo_composite_fwd(void *stream, int64_t r_hit, int s_max, float truncation, const int *offsets,
                                  const int *ray_ns, const float *z_vals, const float *sdf_s, const float *rgb_s,
                                  float *sdf, float *weights, float *color, float *depth, float *z_min) {
    PSVO_REQUIRE(r_hit >= 0 && s_max > 0 && truncation > 0.f, "composite_fwd: bad sizes");
    if (r_hit == 0) return PSVO_OK;
    psvo::launch(k_composite_fwd, dim3(div_up(r_hit, 4)), dim3(256), 0, as_stream(stream), r_hit, s_max,
                       truncation, offsets, ray_ns, z_vals, sdf_s, rgb_s, sdf, weights, color, depth, z_min);
    return check_launch("composite_fwd");
}

extern "C" int psvo_composite_bwd(void *stream, int64_t r_hit, int s_max, float truncation, const int *offsets,
                                  const int *ray_ns, const float *z_vals, const float *sdf, const float *weights,
                                  const float *rgb_s, const float *grad_color, const float *grad_depth,
                                  const float *grad_weights, const float *grad_sdf, float *grad_sdf_s,
                                  float *grad_rgb_s) {
    PSVO_REQUIRE(r_hit >= 0 && s_max > 0 && truncation > 0.f, "composite_bwd: bad sizes");
    if (r_hit == 0) return PSVO_OK;
    psvo::launch(k_composite_bwd, dim3(div_up(r_hit, 4)), dim3(256), 0, as_stream(stream), r_hit, s_max,
                       truncation, offsets, ray_ns, z_vals, sdf, weights, rgb_s, grad_color, grad_depth,
                       grad_weights, grad_sdf, grad_sdf_s, grad_rgb_s);
    return check_launch("composite_bwd");
}


extern "C" int psvo_composite_loss(void *stream, int64_t r_hit, int s_max, float truncation, float max_depth,
                                   const int *offsets, const int *ray_ns, const float *z_vals, const int *rank_ray,
                                   const float *gt_rgb, const float *gt_depth, const float *sdf_s,
                                   const float *rgb_s, const float *coef, float *workspace, float *color,
                                   float *depth, float *grad_sdf_s, float *grad_rgb_s) {
    return psvo::composite_loss_z(stream, r_hit, s_max, truncation, max_depth, offsets, ray_ns, z_vals, s_max,
                                  rank_ray, gt_rgb, gt_depth, sdf_s, rgb_s, coef, workspace, color, depth, grad_sdf_s,
                                  grad_rgb_s, true, nullptr);
}

int psvo::composite_loss_z(void *stream, int64_t r_hit, int s_max, float truncation, float max_depth,
                           const int *offsets, const int *ray_ns, const float *z_vals, int z_stride,
                           const int *rank_ray, const float *gt_rgb, const float *gt_depth, const float *sdf_s,
                           const float *rgb_s, const float *coef, float *workspace, float *color, float *depth,
                           float *grad_sdf_s, float *grad_rgb_s, bool partials, const int *cidx) {
    PSVO_REQUIRE(r_hit >= 0 && s_max > 0 && truncation > 0.f && z_stride >= s_max, "composite_loss: bad sizes");
    PSVO_REQUIRE(offsets && ray_ns && z_vals && rank_ray && gt_rgb && gt_depth && sdf_s && rgb_s && coef &&
                     workspace && color && depth && grad_sdf_s && grad_rgb_s,
                 "composite_loss: null pointer");
    if (r_hit == 0) return PSVO_OK;
    // samples cached in registers up to 64·8 per ray (room0 bench batches: S_max ≈ 200–300)
    auto kern = s_max <= 128   ? k_composite_loss<2>
                : s_max <= 256 ? k_composite_loss<4>
                : s_max <= 512 ? k_composite_loss<8>
                               : k_composite_loss<0>;
    psvo::launch(kern, dim3(div_up(r_hit, 4)), dim3(256), 0, as_stream(stream), r_hit, s_max, truncation,
                       max_depth, offsets, ray_ns, z_vals, z_stride, rank_ray, gt_rgb, gt_depth, sdf_s, rgb_s, coef,
                       workspace, color, depth, grad_sdf_s, grad_rgb_s, partials ? 1 : 0, cidx);
    return check_launch("composite_loss");
}

int psvo::select_samples(hipStream_t st, int64_t r_hit, int s_max, float truncation, float max_depth,
                         const int *offsets, const int *ray_ns, const float *z_vals, int z_stride, const int *rank_ray,
                         const float *gt_depth, const float *sdf_s, const float *feat, const int *leaf, const float *t,
                         const int *ray_of, int64_t cap, bool split, int *cidx, int *offa, int *offb, float *feat_c,
                         int *leaf_c, float *t_c, int *ray_of_c, float *rgb_c, int *src_c, int *counts,
                         unsigned long long *desc, uint32_t tag, int *host_flag) {
    PSVO_REQUIRE(r_hit >= 0 && s_max > 0 && truncation > 0.f && z_stride >= s_max && tag != 0 && cap > 0,
                 "select_samples: bad sizes");
    PSVO_REQUIRE(!split || (offb != nullptr && rgb_c != nullptr),
                 "select_samples: the split needs class B's offsets and colour rows");
    const int rpw = select_rays_per_wave(r_hit);
    PSVO_REQUIRE(rpw <= kSelMaxRpw, "select_samples: %lld hit rays exceed the selection's %d",
                 (long long)r_hit, kSelWaves * kSelMaxRpw * kLbMaxBlocks);
    if (r_hit == 0) return PSVO_OK;
    SelectArgs a{reinterpret_cast<const float4 *>(feat), leaf, ray_of, t, cidx, offa, offb,
                 reinterpret_cast<float4 *>(feat_c), leaf_c, ray_of_c, t_c, rgb_c, src_c, cap, split ? 1 : 0, counts, desc, tag,
                 lb_ctl(4), host_flag};
    psvo::launch(k_select_samples, dim3(div_up(r_hit, (int64_t)kSelWaves * rpw)), dim3(64 * kSelWaves), 0, st, r_hit,
                 rpw, s_max, truncation, max_depth, offsets, ray_ns, z_vals, z_stride, rank_ray, gt_depth, sdf_s, a);
    return check_launch("select_samples");
}

int psvo::lb_helps_select(int64_t *out1, bool reset) {
    unsigned long long h = 0;
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(&h, HIP_SYMBOL(psvo_g_sel_helps), sizeof(h)) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "debug_lb_helps: copy failed");
    *out1 = (int64_t)h;
    const unsigned long long z = 0;
    if (reset && hipMemcpyToSymbol(HIP_SYMBOL(psvo_g_sel_helps), &z, sizeof(z)) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "debug_lb_helps: reset failed");
    return PSVO_OK;
}

int psvo::select_rays_per_wave(int64_t r_hit) {
    const int64_t per = (int64_t)kSelWaves * kLbMaxBlocks;  // rays at one per wave
    return r_hit <= per ? 1 : (int)((r_hit + per - 1) / per);
}

int64_t psvo::select_granules(int64_t r_hit) {
    return lb_granules<3>(div_up(r_hit, (int64_t)kSelWaves * select_rays_per_wave(r_hit)));
}
