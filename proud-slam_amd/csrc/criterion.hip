// Mapping loss (Criterion) on the device, forward + backward, no host syncs.
//
// Reference: src/criterion.py:17-116 (forward :17-68, get_masks :78-101,
// get_sdf_loss :103-116).  With d = gt depth of the hit ray, z/p the padded
// [R_hit, S_max] z_vals / sdf rows:
//   colour = mean |gt_rgb − rgb|                          over R_hit·3
//   depth  = mean_{valid} |gt_d − depth|,  valid = 0.01 < d < max_depth
//   f  = [z < d − tr],  b = [z > d + tr],  dm = [0 < d < max_depth]
//   sm = (1−f)(1−b)dm
//   fs  = mean (p·f − f)²           · (1 − n_f/(n_f+n_s))   over R_hit·S_max
//   sdf = mean ((z + p·tr)·sm − d·sm)² · (1 − n_s/(n_f+n_s))
//   loss = rgb_w·colour + depth_w·depth + fs_w·fs + sdf_w·sdf
// The torch version needs three host syncs (boolean indexing) and ~40
// launches; here it is per-ray partial sums (one wave per ray), a fixed-order
// double reduction (deterministic), a one-thread finalise, and one backward
// pass.  The eight sums are exactly what a data-parallel run all-reduces to
// form the single-GPU loss of the global batch.
// Tracking's weight_depth_loss filter (criterion.py:45-49: valid &= tmp <
// 10·median(tmp)) is two more launches: per-ray tmp, and a one-block bitonic
// sort for the median; sums / bwd then take tmp and the threshold.
#include <hip/hip_runtime.h>

#include "psvo_common.h"

#pragma clang fp contract(off)

namespace psvo {
namespace {

enum { kSumColor = 0, kSumDepth, kNValid, kNFront, kNSdf, kSqFs, kSqSdf, kNSums = 8 };
enum { kFlagColor = 1, kFlagDepth = 2, kFlagSdf = 4 };
static_assert(kNValid == 2 && kNFront == 3 && kNSdf == 4, "svo_query.hip k_dist_smax writes these slots");
// out[] layout (PSVO_CRIT_* in psvo.h)
enum { kOutLoss = 0, kOutColor, kOutDepth, kOutFs, kOutSdf, kOutFsW, kOutSdfW, kOutCColor, kOutCDepth, kOutCFs,
       kOutCSdf };

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) v += __shfl_xor(v, s, 64);
    return v;
}

struct SampleTerms {
    float f, sm, xfs, ysdf;
};

__device__ __forceinline__ SampleTerms sample_terms(float z, float p, float d, float tr, float max_depth) {
    SampleTerms o;
    o.f = z < (d - tr) ? 1.0f : 0.0f;
    const float b = z > (d + tr) ? 1.0f : 0.0f;
    const float dm = (d > 0.0f && d < max_depth) ? 1.0f : 0.0f;
    o.sm = (1.0f - o.f) * (1.0f - b) * dm;
    o.xfs = p * o.f - o.f;
    o.ysdf = (z + p * tr) * o.sm - d * o.sm;
    return o;
}

// one wave per hit ray → part[r][8]
__global__ __launch_bounds__(256) void k_crit_rays(int64_t r_hit, int s_max, int pad_extra, float tr, float max_depth,
                                                   const int *__restrict__ rank_ray, const float *__restrict__ gt_rgb,
                                                   const float *__restrict__ gt_depth, const float *__restrict__ color,
                                                   const float *__restrict__ depth, const float *__restrict__ sdf,
                                                   const float *__restrict__ z_vals, const float *__restrict__ dtmp,
                                                   const float *__restrict__ dthr, float *__restrict__ part) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (r >= r_hit) return;
    const int64_t orig = rank_ray[r];
    const float d = gt_depth[orig];
    float nf = 0.f, ns = 0.f, qfs = 0.f, qsdf = 0.f;
    const float *z = z_vals + r * s_max;
    const float *p = sdf + r * s_max;
    for (int s = lane; s < s_max; s += 64) {
        const SampleTerms t = sample_terms(z[s], p[s], d, tr, max_depth);
        nf += t.f;
        ns += t.sm;
        qfs += t.xfs * t.xfs;
        qsdf += t.ysdf * t.ysdf;
    }
    nf = wsum(nf);
    ns = wsum(ns);
    qfs = wsum(qfs);
    qsdf = wsum(qsdf);
    if (lane == 0) {
        float ac = 0.f;
        for (int c = 0; c < 3; ++c) ac += fabsf(gt_rgb[orig * 3 + c] - color[r * 3 + c]);
        const bool valid = d > 0.01f && d < max_depth && (!dtmp || dtmp[r] < dthr[0]);
        if (pad_extra > 0) {  // padded samples of the global [R_hit, S_max] layout: z = 10, sdf = 1
            const SampleTerms t = sample_terms(10.0f, 1.0f, d, tr, max_depth);
            nf += t.f * pad_extra;
            ns += t.sm * pad_extra;
            qsdf += t.ysdf * t.ysdf * pad_extra;
        }
        float *o = part + r * kNSums;
        o[kSumColor] = ac;
        o[kSumDepth] = valid ? fabsf(d - depth[r]) : 0.0f;
        o[kNValid] = valid ? 1.0f : 0.0f;
        o[kNFront] = nf;
        o[kNSdf] = ns;
        o[kSqFs] = qfs;
        o[kSqSdf] = qsdf;
        o[7] = 0.0f;
    }
}

// fixed-order reduction of part[r_hit][8] → sums[8] (double): 256 virtual
// threads t each sum rows t, t+256, ..., then the pairwise tree
// x[t] += x[t + w], w = 128 .. 1.  One wave plays all 256 (lane l holds
// t = l + 64j, j = 0..3), so the two cross-wave levels are register adds and
// the in-wave levels shuffles — the same pairs as an LDS tree, no LDS: the
// engine runs this beside the persistent decoder kernels, whose LDS leaves
// no room for a workgroup that needs any until they end.
__global__ __launch_bounds__(64) void k_crit_reduce(int64_t r_hit, const float *__restrict__ part,
                                                    double *__restrict__ sums) {
    const int l = threadIdx.x;
    double acc[4][kNSums];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < kNSums; ++k) acc[j][k] = 0.0;
    static_assert(kNSums == 8, "two float4 per row");
    for (int64_t r0 = 0; r0 < r_hit; r0 += 256) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t r = r0 + l + 64 * j;
            if (r < r_hit) {
                const float4 a = reinterpret_cast<const float4 *>(part)[r * 2];
                const float4 b = reinterpret_cast<const float4 *>(part)[r * 2 + 1];
                acc[j][0] += (double)a.x; acc[j][1] += (double)a.y; acc[j][2] += (double)a.z; acc[j][3] += (double)a.w;
                acc[j][4] += (double)b.x; acc[j][5] += (double)b.y; acc[j][6] += (double)b.z; acc[j][7] += (double)b.w;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < kNSums; ++k) {
        double v = acc[0][k] + acc[2][k];       // w = 128: t = l adds t + 128
        const double v1 = acc[1][k] + acc[3][k];  //          t = l + 64 adds t + 128
        v += v1;                                  // w = 64
#pragma unroll
        for (int w = 32; w > 0; w >>= 1) {  // lanes < w read lane + w (still holding its level value)
            const double o = __shfl_down(v, w, 64);
            if (l < w) v += o;
        }
        if (l == 0) sums[k] = v;
    }
}

__global__ void k_crit_finalize(const double *__restrict__ sums, double n_hit, double n_cols, float rgb_w,
                                float depth_w, float fs_w, float sdf_w, float tr, int flags, float *__restrict__ out) {
    if (threadIdx.x != 0) return;
    const double n_el = n_hit * n_cols;
    const float color_loss = (float)(sums[kSumColor] / (3.0 * n_hit));
    const float n_valid = (float)sums[kNValid];
    const float depth_loss = (float)(sums[kSumDepth] / sums[kNValid]);  // 0/0 = NaN as torch's empty mean
    const float n_f = (float)sums[kNFront], n_s = (float)sums[kNSdf];
    const float n_tot = n_s + n_f;
    const float fs_weight = 1.0f - n_f / n_tot;
    const float sdf_weight = 1.0f - n_s / n_tot;
    const float fs_loss = (float)(sums[kSqFs] / n_el) * fs_weight;
    const float sdf_loss = (float)(sums[kSqSdf] / n_el) * sdf_weight;
    float loss = 0.0f;
    if (flags & kFlagColor) loss += rgb_w * color_loss;
    if (flags & kFlagDepth) loss += depth_w * depth_loss;
    if (flags & kFlagSdf) {
        loss += fs_w * fs_loss;
        loss += sdf_w * sdf_loss;
    }
    out[kOutLoss] = loss;
    out[kOutColor] = color_loss;
    out[kOutDepth] = depth_loss;
    out[kOutFs] = fs_loss;
    out[kOutSdf] = sdf_loss;
    out[kOutFsW] = fs_weight;
    out[kOutSdfW] = sdf_weight;
    // backward coefficients (d loss / d term per element, before the sign / residual factor)
    out[kOutCColor] = (flags & kFlagColor) ? (float)(rgb_w / (3.0 * n_hit)) : 0.0f;
    out[kOutCDepth] = (flags & kFlagDepth) ? depth_w / n_valid : 0.0f;
    out[kOutCFs] = (flags & kFlagSdf) ? (float)(2.0 * (double)(fs_w * fs_weight) / n_el) : 0.0f;
    out[kOutCSdf] = (flags & kFlagSdf) ? (float)(2.0 * (double)(sdf_w * sdf_weight) / n_el) * tr : 0.0f;
}

__device__ __forceinline__ float sgn(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }

__global__ __launch_bounds__(256) void k_crit_bwd(int64_t r_hit, int s_max, float tr, float max_depth,
                                                  const int *__restrict__ rank_ray, const float *__restrict__ gt_rgb,
                                                  const float *__restrict__ gt_depth, const float *__restrict__ color,
                                                  const float *__restrict__ depth, const float *__restrict__ sdf,
                                                  const float *__restrict__ z_vals, const float *__restrict__ coef,
                                                  const float *__restrict__ g_loss, const float *__restrict__ dtmp,
                                                  const float *__restrict__ dthr, float *__restrict__ g_color,
                                                  float *__restrict__ g_depth, float *__restrict__ g_sdf) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (r >= r_hit) return;
    const float g = g_loss[0];
    const int64_t orig = rank_ray[r];
    const float d = gt_depth[orig];
    const float cfs = g * coef[kOutCFs], csdf = g * coef[kOutCSdf];
    const float *z = z_vals + r * s_max;
    const float *p = sdf + r * s_max;
    float *gs = g_sdf + r * s_max;
    for (int s = lane; s < s_max; s += 64) {
        const SampleTerms t = sample_terms(z[s], p[s], d, tr, max_depth);
        gs[s] = cfs * t.xfs * t.f + csdf * t.ysdf * t.sm;
    }
    if (lane < 3) {
        g_color[r * 3 + lane] = -(g * coef[kOutCColor]) * sgn(gt_rgb[orig * 3 + lane] - color[r * 3 + lane]);
    } else if (lane == 3) {
        const bool valid = d > 0.01f && d < max_depth && (!dtmp || dtmp[r] < dthr[0]);
        g_depth[r] = valid ? -(g * coef[kOutCDepth]) * sgn(d - depth[r]) : 0.0f;
    }
}

// ---- mapping step, split by what each part depends on -------------------
// The loss's normalisers (n_valid, n_front, n_sdf) and hence every backward
// coefficient depend only on z_vals and the GT depth, not on the decoder: the
// engine counts them beside the decoder forward (k_crit_counts → reduce →
// k_crit_coef), and k_composite_loss (composite.hip) then runs compositing,
// the loss partials and the whole per-ray backward in one pass; the loss
// value itself (reduce + finalize) is off the critical path.

// one wave per hit ray: the count slots of part[r] (kNValid, kNFront, kNSdf)
__global__ __launch_bounds__(256) void k_crit_counts(int64_t r_hit, int s_max, float tr, float max_depth,
                                                     const int *__restrict__ rank_ray,
                                                     const float *__restrict__ gt_depth,
                                                     const float *__restrict__ z_vals, int z_stride,
                                                     const int *__restrict__ ray_ns, float *__restrict__ part) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (r >= r_hit) return;
    const float d = gt_depth[rank_ray[r]];
    const float *z = z_vals + r * z_stride;
    // ray_ns (sampler rows): past the ray's valid samples the padding
    // MAX_DEPTH is implied (the look-back sampler does not write it)
    const int n_in = ray_ns ? ray_ns[r] : s_max;
    float nf = 0.f, ns = 0.f;
    for (int s = lane; s < s_max; s += 64) {
        const SampleTerms t = sample_terms(s < n_in ? z[s] : kMaxDepthFill, 1.0f, d, tr, max_depth);
        nf += t.f;
        ns += t.sm;
    }
    nf = wsum(nf);
    ns = wsum(ns);
    if (lane == 0) {
        float *o = part + r * kNSums;
        o[kNValid] = (d > 0.01f && d < max_depth) ? 1.0f : 0.0f;
        o[kNFront] = nf;
        o[kNSdf] = ns;
    }
}

// data parallel: this rank's count words for the query's second all-gather
// (psvo_common.h dist_counts) — one wave per local hit row (sampler rows,
// valid prefix ray_ns), integer atomics (exact, order-free); the padding's
// terms stay per ray so the union S_max can be applied after the gather
__global__ __launch_bounds__(256) void k_dist_counts(const int *__restrict__ stats, const int *__restrict__ rank_ray,
                                                     const float *__restrict__ gt_depth,
                                                     const float *__restrict__ z_rows, int z_stride,
                                                     const int *__restrict__ ray_ns, float tr, float max_depth,
                                                     int *__restrict__ in) {
    __shared__ int red[7];
    if (blockIdx.x == 0 && threadIdx.x == 0) in[0] = stats[PSVO_STAT_S_MAX] | (gt_depth ? 0 : kDistNotCounted);
    if (!gt_depth) return;
    if (threadIdx.x < 7) red[threadIdx.x] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (r < stats[PSVO_STAT_R_HIT_LOCAL]) {
        const float d = gt_depth[rank_ray[r]];
        const float *z = z_rows + r * z_stride;
        const int n_in = ray_ns[r];
        float nf = 0.f, nsm = 0.f;
        for (int s = lane; s < n_in; s += 64) {
            const SampleTerms t = sample_terms(z[s], 1.0f, d, tr, max_depth);
            nf += t.f;
            nsm += t.sm;
        }
        nf = wsum(nf);
        nsm = wsum(nsm);
        if (lane == 0) {
            const SampleTerms pad = sample_terms(kMaxDepthFill, 1.0f, d, tr, max_depth);
            const int pf = pad.f != 0.0f, ps = pad.sm != 0.0f;
            atomicAdd(red + 0, (d > 0.01f && d < max_depth) ? 1 : 0);
            atomicAdd(red + 1, (int)nf);
            atomicAdd(red + 2, (int)nsm);
            atomicAdd(red + 3, pf);
            atomicAdd(red + 4, pf * n_in);
            atomicAdd(red + 5, ps);
            atomicAdd(red + 6, ps * n_in);
        }
    }
    __syncthreads();
    if (threadIdx.x < 7 && red[threadIdx.x] != 0) atomicAdd(in + 1 + threadIdx.x, red[threadIdx.x]);
}

// the backward coefficients of k_crit_finalize from the count sums alone
// (same arithmetic, so the two agree bit for bit)
__global__ void k_crit_coef(const double *__restrict__ sums, double n_hit, double n_cols, float rgb_w, float depth_w,
                            float fs_w, float sdf_w, float tr, int flags, float *__restrict__ coef) {
    if (threadIdx.x != 0) return;
    static_assert(kFlagColor == PSVO_CRIT_USE_COLOR && kFlagDepth == PSVO_CRIT_USE_DEPTH &&
                  kFlagSdf == PSVO_CRIT_USE_SDF, "flag bits");
    crit_coef_from_counts(sums[kNValid], sums[kNFront], sums[kNSdf], n_hit, n_cols, rgb_w, depth_w, fs_w, sdf_w, tr,
                          flags, coef);
}

// tracking's depth filter (criterion.py:45-50): per hit ray
//   tmp = |d − depth| / sqrt(Σ_s w_s (depth − z_s)² + 1e-10)
__global__ __launch_bounds__(256) void k_crit_depth_tmp(int64_t r_hit, int s_max, const int *__restrict__ rank_ray,
                                                        const float *__restrict__ gt_depth,
                                                        const float *__restrict__ depth,
                                                        const float *__restrict__ weights,
                                                        const float *__restrict__ z_vals, float *__restrict__ dtmp) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (r >= r_hit) return;
    const float pd = depth[r];
    float v = 0.f;
    for (int s = lane; s < s_max; s += 64) {
        const float e = pd - z_vals[r * s_max + s];
        v += weights[r * s_max + s] * (e * e);
    }
    v = wsum(v);
    if (lane == 0) dtmp[r] = fabsf(gt_depth[rank_ray[r]] - pd) / sqrtf(v + 1e-10f);
}

// threshold = 10 · median(tmp) (torch.median: the lower middle element,
// index (n−1)/2 of the sorted values): one block, bitonic sort in LDS
constexpr int kMedianMax = 16384;
__global__ __launch_bounds__(1024) void k_crit_depth_thr(int64_t r_hit, const float *__restrict__ dtmp,
                                                         float *__restrict__ dthr) {
    extern __shared__ float v[];
    int n2 = 1;
    while (n2 < r_hit) n2 <<= 1;
    for (int i = threadIdx.x; i < n2; i += blockDim.x) v[i] = i < r_hit ? dtmp[i] : __int_as_float(0x7f800000);
    __syncthreads();
    for (int k = 2; k <= n2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < n2; i += blockDim.x) {
                const int ij = i ^ j;
                if (ij > i) {
                    const float a = v[i], b = v[ij];
                    const bool up = (i & k) == 0;
                    if ((a > b) == up) {
                        v[i] = b;
                        v[ij] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
    if (threadIdx.x == 0) dthr[0] = 10.0f * v[(r_hit - 1) / 2];
}

}  // namespace
}  // namespace psvo

using namespace psvo;

extern "C" int64_t psvo_criterion_workspace_floats(int64_t r_hit) { return r_hit * kNSums; }

extern "C" int psvo_criterion_depth_filter(void *stream, int64_t r_hit, int s_max, const int *rank_ray,
                                           const float *gt_depth, const float *depth, const float *weights,
                                           const float *z_vals, float *dtmp, float *dthr) {
    PSVO_REQUIRE(r_hit > 0 && s_max > 0, "criterion_depth_filter: bad sizes");
    PSVO_REQUIRE(r_hit <= kMedianMax, "criterion_depth_filter: %lld hit rays > %d (single-block median)",
                 (long long)r_hit, kMedianMax);
    hipStream_t st = as_stream(stream);
    psvo::launch(k_crit_depth_tmp, dim3(div_up(r_hit, 4)), dim3(256), 0, st, r_hit, s_max, rank_ray, gt_depth,
                       depth, weights, z_vals, dtmp);
    int n2 = 1;
    while (n2 < r_hit) n2 <<= 1;
    psvo::launch(k_crit_depth_thr, dim3(1), dim3(1024), n2 * sizeof(float), st, r_hit, dtmp, dthr);
    return check_launch("criterion_depth_filter");
}

extern "C" int psvo_criterion_sums_ex(void *stream, int64_t r_hit, int s_max, int pad_extra, float truncation,
                                      float max_depth, const int *rank_ray, const float *gt_rgb, const float *gt_depth,
                                      const float *color, const float *depth, const float *sdf, const float *z_vals,
                                      const float *dtmp, const float *dthr, float *workspace, double *sums) {
    PSVO_REQUIRE(r_hit > 0 && s_max > 0 && pad_extra >= 0, "criterion_sums: bad sizes");
    PSVO_REQUIRE(rank_ray && gt_rgb && gt_depth && color && depth && sdf && z_vals && workspace && sums,
                 "criterion_sums: null pointer");
    PSVO_REQUIRE((dtmp == nullptr) == (dthr == nullptr), "criterion_sums: depth filter needs tmp and threshold");
    hipStream_t st = as_stream(stream);
    psvo::launch(k_crit_rays, dim3(div_up(r_hit, 4)), dim3(256), 0, st, r_hit, s_max, pad_extra, truncation,
                       max_depth, rank_ray, gt_rgb, gt_depth, color, depth, sdf, z_vals, dtmp, dthr, workspace);
    PSVO_REQUIRE(((uintptr_t)workspace & 15) == 0, "criterion: workspace must be 16-B aligned");
    psvo::launch(k_crit_reduce, dim3(1), dim3(64), 0, st, r_hit, workspace, sums);
    return check_launch("criterion_sums");
}

extern "C" int psvo_criterion_sums(void *stream, int64_t r_hit, int s_max, int pad_extra, float truncation,
                                   float max_depth, const int *rank_ray, const float *gt_rgb, const float *gt_depth,
                                   const float *color, const float *depth, const float *sdf, const float *z_vals,
                                   float *workspace, double *sums) {
    return psvo_criterion_sums_ex(stream, r_hit, s_max, pad_extra, truncation, max_depth, rank_ray, gt_rgb, gt_depth,
                                  color, depth, sdf, z_vals, nullptr, nullptr, workspace, sums);
}

extern "C" int psvo_criterion_coef(void *stream, int64_t r_hit, int s_max, float truncation, float max_depth,
                                   const int *rank_ray, const float *gt_depth, const float *z_vals, float rgb_w,
                                   float depth_w, float fs_w, float sdf_w, int flags, float *workspace, double *sums,
                                   float *coef) {
    PSVO_REQUIRE(r_hit > 0 && s_max > 0, "criterion_coef: bad sizes");
    PSVO_REQUIRE(rank_ray && gt_depth && z_vals && workspace && sums && coef, "criterion_coef: null pointer");
    return psvo::criterion_coef_z(stream, r_hit, s_max, truncation, max_depth, rank_ray, gt_depth, z_vals, s_max,
                                  nullptr, rgb_w, depth_w, fs_w, sdf_w, flags, workspace, sums, coef);
}

int psvo::criterion_coef_z(void *stream, int64_t r_hit, int s_max, float truncation, float max_depth,
                           const int *rank_ray, const float *gt_depth, const float *z_vals, int z_stride,
                           const int *ray_ns, float rgb_w, float depth_w, float fs_w, float sdf_w, int flags,
                           float *workspace, double *sums, float *coef) {
    PSVO_REQUIRE(z_stride >= s_max, "criterion_coef: z stride %d < S_max %d", z_stride, s_max);
    hipStream_t st = as_stream(stream);
    psvo::launch(k_crit_counts, dim3(div_up(r_hit, 4)), dim3(256), 0, st, r_hit, s_max, truncation, max_depth,
                       rank_ray, gt_depth, z_vals, z_stride, ray_ns, workspace);
    PSVO_REQUIRE(((uintptr_t)workspace & 15) == 0, "criterion: workspace must be 16-B aligned");
    psvo::launch(k_crit_reduce, dim3(1), dim3(64), 0, st, r_hit, workspace, sums);
    psvo::launch(k_crit_coef, dim3(1), dim3(64), 0, st, sums, (double)r_hit, (double)s_max, rgb_w, depth_w,
                       fs_w, sdf_w, truncation, flags, coef);
    return check_launch("criterion_coef");
}

namespace psvo {
// psvo_criterion_coef in two halves, so that a data-parallel engine can
// all-reduce the count sums (union-batch normalisers) between them
int criterion_counts(hipStream_t st, int64_t r_hit, int s_max, float truncation, float max_depth, const int *rank_ray,
                     const float *gt_depth, const float *z_vals, int z_stride, const int *ray_ns, float *workspace,
                     double *sums) {
    PSVO_REQUIRE(z_stride >= s_max, "criterion_counts: z stride %d < S_max %d", z_stride, s_max);
    if (r_hit > 0)
        psvo::launch(k_crit_counts, dim3(div_up(r_hit, 4)), dim3(256), 0, st, r_hit, s_max, truncation,
                           max_depth, rank_ray, gt_depth, z_vals, z_stride, ray_ns, workspace);
    PSVO_REQUIRE(((uintptr_t)workspace & 15) == 0, "criterion: workspace must be 16-B aligned");
    psvo::launch(k_crit_reduce, dim3(1), dim3(64), 0, st, r_hit, workspace, sums);
    return check_launch("criterion_counts");
}
int dist_counts(hipStream_t st, int64_t R, const int *stats, const int *rank_ray, const float *gt_depth,
                const float *z_rows, int z_stride, const int *ray_ns, float truncation, float max_depth, int *in) {
    const int64_t blocks = gt_depth ? (R + 3) / 4 : 1;
    psvo::launch(k_dist_counts, dim3((int)(blocks > 0 ? blocks : 1)), dim3(256), 0, st, stats, rank_ray, gt_depth,
                 z_rows, z_stride, ray_ns, truncation, max_depth, in);
    return check_launch("dist_counts");
}
int criterion_coef_from_sums(hipStream_t st, const double *sums, int64_t n_hit, int n_cols, float truncation,
                             float rgb_w, float depth_w, float fs_w, float sdf_w, int flags, float *coef) {
    psvo::launch(k_crit_coef, dim3(1), dim3(64), 0, st, sums, (double)n_hit, (double)n_cols, rgb_w, depth_w,
                       fs_w, sdf_w, truncation, flags, coef);
    return check_launch("criterion_coef");
}
}  // namespace psvo

extern "C" int psvo_criterion_reduce(void *stream, int64_t r_hit, const float *workspace, double *sums) {
    PSVO_REQUIRE(r_hit > 0 && workspace && sums, "criterion_reduce: bad arguments");
    PSVO_REQUIRE(((uintptr_t)workspace & 15) == 0, "criterion: workspace must be 16-B aligned");
    psvo::launch(k_crit_reduce, dim3(1), dim3(64), 0, as_stream(stream), r_hit, workspace, sums);
    return check_launch("criterion_reduce");
}

extern "C" int psvo_criterion_finalize(void *stream, const double *sums, int64_t n_hit, int s_max, float rgb_w,
                                       float depth_w, float fs_w, float sdf_w, float truncation, int flags,
                                       float *out) {
    PSVO_REQUIRE(n_hit > 0 && s_max > 0, "criterion_finalize: bad sizes");
    psvo::launch(k_crit_finalize, dim3(1), dim3(64), 0, as_stream(stream), sums, (double)n_hit, (double)s_max,
                       rgb_w, depth_w, fs_w, sdf_w, truncation, flags, out);
    return check_launch("criterion_finalize");
}

extern "C" int psvo_criterion_bwd_ex(void *stream, int64_t r_hit, int s_max, float truncation, float max_depth,
                                     const int *rank_ray, const float *gt_rgb, const float *gt_depth,
                                     const float *color, const float *depth, const float *sdf, const float *z_vals,
                                     const float *out, const float *g_loss, const float *dtmp, const float *dthr,
                                     float *g_color, float *g_depth, float *g_sdf) {
    PSVO_REQUIRE(r_hit > 0 && s_max > 0, "criterion_bwd: bad sizes");
    PSVO_REQUIRE((dtmp == nullptr) == (dthr == nullptr), "criterion_bwd: depth filter needs tmp and threshold");
    psvo::launch(k_crit_bwd, dim3(div_up(r_hit, 4)), dim3(256), 0, as_stream(stream), r_hit, s_max, truncation,
                       max_depth, rank_ray, gt_rgb, gt_depth, color, depth, sdf, z_vals, out, g_loss, dtmp, dthr,
                       g_color, g_depth, g_sdf);
    return check_launch("criterion_bwd");
}

extern "C" int psvo_criterion_bwd(void *stream, int64_t r_hit, int s_max, float truncation, float max_depth,
                                  const int *rank_ray, const float *gt_rgb, const float *gt_depth, const float *color,
                                  const float *depth, const float *sdf, const float *z_vals, const float *out,
                                  const float *g_loss, float *g_color, float *g_depth, float *g_sdf) {
    return psvo_criterion_bwd_ex(stream, r_hit, s_max, truncation, max_depth, rank_ray, gt_rgb, gt_depth, color, depth,
                                 sdf, z_vals, out, g_loss, nullptr, nullptr, g_color, g_depth, g_sdf);
}
