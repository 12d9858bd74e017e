// The `grid` extension's off-path entry points on gfx950: brute-force
// ray/ball, ray/box and ray/triangle intersection and NSVF uniform ray
// sampling.  The render path never calls them; they
// exist so code written against the reference's `grid` module — its own
// src/variations/test_aabb.py among it — runs unchanged.
//
// Reference behaviour restated (DARYL-GWZ/Proud-SLAM, third_party/sparse_voxels):
//   intersect_gpu.cu:13-73    ball test; first n_max hits in point order
//   intersect_gpu.cu:75-187   slab test (f_low 0, f_high 1e5); first n_max boxes in order
//   intersect_gpu.cu:273-362  Möller–Trumbore with blur; first n_max hits in face
//                             order, then ordered by depth (ties keep face order),
//                             then the cage offsets from the neighbour gaps
//   sample_gpu.cu:13-124      merge of box boundaries with uniform steps, midpoints,
//                             compaction of the in-box intervals
//
// MI355X design: the intersections give one wave per ray and test 64
// primitives per wave-step (coalesced 768-B / 2.3-KB reads of the primitive
// list); __ballot + mbcnt compact the hits in primitive order, so the wave
// stops as soon as n_max hits exist — the same prefix the reference's serial
// loop keeps.  The triangle kernel sorts its ≤ n_max hits in LDS by rank
// (count of smaller depths, ties broken by face order), which is the order
// the reference's insertion produces.  The uniform sampler is an in-place
// serial merge per ray, one lane per ray, exactly as the reference's.
//
// Arithmetic: contraction off and IEEE division / square root, matching the
// CPU oracle bit for bit (the reference uses __fdividef and nvcc's FMA
// contraction; DESIGN.md "parity").  sqrtf, not __fsqrt_rn: on this
// toolchain the latter lowers to the bare v_sqrt_f32 (1 ulp), sqrtf to the
// correctly rounded sequence.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include "psvo_common.h"

namespace psvo {
namespace {

constexpr int kGaWaves = 8;           // rays (waves) per workgroup of the point kernels
constexpr int kGaTile = 512;          // points per LDS tile (6 KB)
constexpr int kGaSegs = 4;            // split mode: waves (point segments) per ray
constexpr int kGaSplitHits = 128;     // split mode: per-segment hit list in LDS (n_max bound)
constexpr int kGaSplitMinN = 1024;    // split mode: shortest point list worth splitting
constexpr int kTriMaxHits = 2048;     // LDS bound of the triangle kernel's hit list

__device__ __forceinline__ int lanes_below(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// intersect_gpu.cu:75-140 — the comparisons of svo_query.hip's ray_aabb_nb:
// the reference's early-exit tests in order, the verdict accumulated so the
// wave runs one basic block per box instead of three divergent exits
__device__ __forceinline__ bool slab(const float o[3], const float inv[3], const float c[3], float half,
                                     float &t_lo, float &t_hi) {
    float lo_all = 0.0f, hi_all = 100000.0f;
    bool miss = false;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float lo = (c[a] - half - o[a]) * inv[a];
        const float hi = (c[a] + half - o[a]) * inv[a];
        const bool sw = hi < lo;
        const float l2 = sw ? hi : lo, h2 = sw ? lo : hi;
        miss = miss | (h2 < lo_all) | (l2 > hi_all);
        lo_all = (l2 > lo_all) ? l2 : lo_all;
        hi_all = (h2 < hi_all) ? h2 : hi_all;
        miss = miss | (lo_all > hi_all);
    }
    t_lo = lo_all;
    t_hi = hi_all;
    return !miss;
}

// Point primitives (ball centres, box centres) for the rays of one
// workgroup: kGaWaves rays, one per wave.  When the workgroup's rays share a
// batch (the usual case: a batch holds many rays) the primitive list streams
// once per workgroup through an LDS tile of kGaTile points instead of once
// per wave — the waves' L2 traffic, which bounds the brute-force scan, drops
// kGaWaves-fold.  `test(p, lo, hi)` decides the point at p[0..2].  Writes the
// first n_max hits in point order and -1 in the unused idx slots.
template <class Test>
__device__ __forceinline__ void point_hits(int64_t ray, int64_t total, int m, int n, int n_max,
                                           const float *__restrict__ points, const Test &test, int *idx_out,
                                           float *lo_out, float *hi_out) {
    __shared__ float tile[kGaTile * 3];
    const int lane = threadIdx.x % kWave;
    const int64_t ray0 = (int64_t)blockIdx.x * kGaWaves;
    const int64_t last = min(ray0 + kGaWaves, total) - 1;
    const bool active = ray < total;
    int *idx = idx_out + ray * n_max;
    float *lo_o = lo_out + ray * n_max, *hi_o = hi_out + ray * n_max;
    int cnt = 0;
    auto step = [&](const float *p, int k) {  // one wave-step over points k..k+63 (this lane: k)
        float lo = 0.0f, hi = 0.0f;
        const bool hit = k < n && test(p, lo, hi);
        const uint64_t mask = __ballot(hit);
        const int pos = cnt + lanes_below(mask);
        if (hit && pos < n_max) {
            idx[pos] = k;
            lo_o[pos] = lo;
            hi_o[pos] = hi;
        }
        cnt += __popcll(mask);
    };
    if (ray0 / m != last / m) {  // workgroup spans batches (block-uniform): direct loads
        if (!active) return;
        const float *pts = points + (ray / m) * n * 3;
        for (int k0 = 0; k0 < n && cnt < n_max; k0 += kWave) {
            const int k = min(k0 + lane, n - 1);
            step(pts + (int64_t)k * 3, k0 + lane);
        }
    } else {
        const float *pts = points + (ray0 / m) * n * 3;
        for (int t0 = 0; t0 < n; t0 += kGaTile) {
            if (!__syncthreads_or(active && cnt < n_max)) break;  // also orders the tile rewrite
            const int span = min(kGaTile, n - t0) * 3;
            for (int e = threadIdx.x; e < span; e += blockDim.x) tile[e] = pts[(int64_t)t0 * 3 + e];
            __syncthreads();
            if (active)
                for (int c = 0; c < kGaTile && t0 + c < n && cnt < n_max; c += kWave) step(tile + (c + lane) * 3, t0 + c + lane);
        }
        if (!active) return;
    }
    for (int l = min(cnt, n_max) + lane; l < n_max; l += kWave) idx[l] = -1;
}

// Split mode (n_max <= kGaSplitHits, long lists): each ray gets kGaSegs
// waves, each scanning one contiguous segment of the point list into its
// own LDS hit list (capped at n_max); the segment-0 wave then concatenates
// the lists in segment order and truncates at n_max — the first n_max hits
// in point order, as the serial loop keeps.  A few thousand rays are 4 waves
// per SIMD in the one-wave-per-ray layout; this gives each SIMD kGaSegs×
// as many waves to hide the per-step latency with.
template <class Test>
__device__ __forceinline__ void point_hits_split(int64_t ray, int64_t total, int m, int n, int n_max,
                                                 const float *__restrict__ points, const Test &test,
                                                 int *idx_out, float *lo_out, float *hi_out) {
    __shared__ int s_cnt[kGaWaves];
    __shared__ int s_k[kGaWaves * kGaSplitHits];
    __shared__ float s_lo[kGaWaves * kGaSplitHits], s_hi[kGaWaves * kGaSplitHits];
    const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    const int seg = wave % kGaSegs, grp = wave - seg;
    const bool active = ray < total;
    if (active) {
        const int seg_len = ((n + kGaSegs - 1) / kGaSegs + kWave - 1) / kWave * kWave;
        const int k_begin = seg * seg_len, k_end = min(n, k_begin + seg_len);
        const float *pts = points + (ray / m) * n * 3;
        int cnt = 0;
        for (int k0 = k_begin; k0 < k_end && cnt < n_max; k0 += kWave) {
            const int k = k0 + lane;
            float lo = 0.0f, hi = 0.0f;
            const bool hit = k < k_end && test(pts + (int64_t)k * 3, lo, hi);
            const uint64_t mask = __ballot(hit);
            const int pos = cnt + lanes_below(mask);
            if (hit && pos < n_max) {
                s_k[wave * kGaSplitHits + pos] = k;
                s_lo[wave * kGaSplitHits + pos] = lo;
                s_hi[wave * kGaSplitHits + pos] = hi;
            }
            cnt += __popcll(mask);
        }
        if (lane == 0) s_cnt[wave] = min(cnt, n_max);
    }
    __syncthreads();
    if (!active || seg != 0) return;
    int *idx = idx_out + ray * n_max;
    float *lo_o = lo_out + ray * n_max, *hi_o = hi_out + ray * n_max;
    int base = 0;
    for (int sgi = 0; sgi < kGaSegs && base < n_max; ++sgi) {
        const int src = (grp + sgi) * kGaSplitHits;
        const int take = min(s_cnt[grp + sgi], n_max - base);
        for (int q = lane; q < take; q += kWave) {
            idx[base + q] = s_k[src + q];
            lo_o[base + q] = s_lo[src + q];
            hi_o[base + q] = s_hi[src + q];
        }
        base += take;
    }
    for (int l = base + lane; l < n_max; l += kWave) idx[l] = -1;
}

template <bool SPLIT>
__global__ __launch_bounds__(kGaWaves *kWave) void k_ball_intersect(int b, int n, int m, float radius, int n_max,
                                                                     const float *__restrict__ ray_start,
                                                                     const float *__restrict__ ray_dir,
                                                                     const float *__restrict__ points, int *idx,
                                                                     float *min_depth, float *max_depth) {
    const int64_t total = (int64_t)b * m;
    const int64_t ray = SPLIT ? (int64_t)blockIdx.x * (kGaWaves / kGaSegs) + threadIdx.x / (kWave * kGaSegs)
                              : (int64_t)blockIdx.x * kGaWaves + threadIdx.x / kWave;
    const int64_t r = min(ray, total - 1);
    const float o[3] = {ray_start[r * 3], ray_start[r * 3 + 1], ray_start[r * 3 + 2]};
    const float w[3] = {ray_dir[r * 3], ray_dir[r * 3 + 1], ray_dir[r * 3 + 2]};
    const float r2max = radius * radius;
    auto test = [&](const float *p, float &lo, float &hi) {
        const float x = p[0] - o[0];
        const float y = p[1] - o[1];
        const float z = p[2] - o[2];
        const float d2 = x * x + y * y + z * z;
        const float proj = x * w[0] + y * w[1] + z * w[2];
        const float d2_proj = proj * proj;
        const float r2 = d2 - d2_proj;
        if (!(r2 < r2max)) return false;
        const float depth = sqrtf(d2_proj);
        const float blur = sqrtf(r2max - r2);
        lo = depth - blur;
        hi = depth + blur;
        return true;
    };
    if constexpr (SPLIT)
        point_hits_split(ray, total, m, n, n_max, points, test, idx, min_depth, max_depth);
    else
        point_hits(ray, total, m, n, n_max, points, test, idx, min_depth, max_depth);
}

template <bool SPLIT>
__global__ __launch_bounds__(kGaWaves *kWave) void k_aabb_intersect(int b, int n, int m, float voxelsize, int n_max,
                                                                     const float *__restrict__ ray_start,
                                                                     const float *__restrict__ ray_dir,
                                                                     const float *__restrict__ points, int *idx,
                                                                     float *min_depth, float *max_depth) {
    const int64_t total = (int64_t)b * m;
    const int64_t ray = SPLIT ? (int64_t)blockIdx.x * (kGaWaves / kGaSegs) + threadIdx.x / (kWave * kGaSegs)
                              : (int64_t)blockIdx.x * kGaWaves + threadIdx.x / kWave;
    const int64_t r = min(ray, total - 1);
    const float o[3] = {ray_start[r * 3], ray_start[r * 3 + 1], ray_start[r * 3 + 2]};
    float inv[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) inv[a] = __fdiv_rn(1.0f, ray_dir[r * 3 + a]);
    const float half = voxelsize * 0.5f;
    auto test = [&](const float *p, float &lo, float &hi) {
        // the reference keeps a box only when t_in > -1 (intersect_gpu.cu:176)
        return slab(o, inv, p, half, lo, hi) && lo > -1.0f;
    };
    if constexpr (SPLIT)
        point_hits_split(ray, total, m, n, n_max, points, test, idx, min_depth, max_depth);
    else
        point_hits(ray, total, m, n, n_max, points, test, idx, min_depth, max_depth);
}

struct F3 {
    float x, y, z;
};
__device__ __forceinline__ F3 sub(F3 a, F3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ float dot(F3 a, F3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ F3 cross(F3 a, F3 b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

// intersect_gpu.cu:273-305: t (> 0 to count), u, v
__device__ __forceinline__ bool ray_triangle(F3 o, F3 d, const float *f, float blur, float &t, float &u, float &v) {
    const F3 v0 = {f[0], f[1], f[2]}, v1 = {f[3], f[4], f[5]}, v2 = {f[6], f[7], f[8]};
    const F3 e1 = sub(v1, v0), e2 = sub(v2, v0), s = sub(o, v0);
    const F3 p = cross(d, e2);
    const float inv_det = __fdiv_rn(1.0f, dot(e1, p));
    u = dot(s, p) * inv_det;
    if ((u < 0.0f - blur) || (u > 1.0f + blur)) return false;
    const F3 q = cross(s, e1);
    v = dot(d, q) * inv_det;
    if ((v < 0.0f - blur) || (v > 1.0f + blur)) return false;
    if (((u + v) < 0.0f - blur) || ((u + v) > 1.0f + blur)) return false;
    t = dot(e2, q) * inv_det;
    return t > 0.0f;
}

// One wave per ray; the ≤ n_max hits live in LDS (dynamic, 20 B per slot).
__global__ __launch_bounds__(kWave) void k_triangle_intersect(int b, int n, int m, float cagesize, float blur,
                                                              int n_max, const float *__restrict__ ray_start,
                                                              const float *__restrict__ ray_dir,
                                                              const float *__restrict__ faces, int *idx_out,
                                                              float *depth_out, float *uv_out) {
    extern __shared__ float tri_lds[];
    int *h_k = reinterpret_cast<int *>(tri_lds);
    float *h_t = tri_lds + n_max;
    float *h_u = h_t + n_max;
    float *h_v = h_u + n_max;
    float *s_t = h_v + n_max;  // depths in sorted order
    const int lane = threadIdx.x;
    const int64_t ray = blockIdx.x;
    const int64_t bi = ray / m;
    const float *fp = faces + bi * n * 9;
    const F3 o = {ray_start[ray * 3], ray_start[ray * 3 + 1], ray_start[ray * 3 + 2]};
    const F3 d = {ray_dir[ray * 3], ray_dir[ray * 3 + 1], ray_dir[ray * 3 + 2]};
    int cnt = 0;
    for (int k0 = 0; k0 < n && cnt < n_max; k0 += kWave) {
        const int k = k0 + lane;
        float t = 0.0f, u = 0.0f, v = 0.0f;
        const bool hit = k < n && ray_triangle(o, d, fp + (int64_t)k * 9, blur, t, u, v);
        const uint64_t mask = __ballot(hit);
        const int pos = cnt + lanes_below(mask);
        if (hit && pos < n_max) {
            h_k[pos] = k;
            h_t[pos] = t;
            h_u[pos] = u;
            h_v[pos] = v;
        }
        cnt += __popcll(mask);
    }
    cnt = min(cnt, n_max);
    __syncthreads();
    int *idx = idx_out + ray * n_max;
    float *depth = depth_out + ray * n_max * 3;
    float *uv = uv_out + ray * n_max * 2;
    // Order of the reference's insertion (intersect_gpu.cu:339-353, strict <):
    // a hit goes before the first strictly deeper entry and the entry it
    // displaces is carried on, which moves the head of every later run of
    // equal depths to that run's end.  So a hit's slot is #(strictly
    // shallower hits); within a run of equal depths v the order is a queue
    // fed in face order — a hit of depth v appends, a shallower hit rotates
    // the queue by one.  Distinct depths (the usual case) place themselves;
    // the first hit of a tied run replays its queue, using the run's output
    // slots as the ring.
    for (int i = lane; i < cnt; i += kWave) {
        const float ti = h_t[i];
        int less = 0, eq_before = 0, eq = 0;
        for (int j = 0; j < cnt; ++j) {
            const float tj = h_t[j];
            less += tj < ti;
            eq += tj == ti;
            eq_before += (tj == ti) && (j < i);
        }
        if (eq == 1) {
            idx[less] = h_k[i];
            depth[less * 3] = ti;
            uv[less * 2] = h_u[i];
            uv[less * 2 + 1] = h_v[i];
            s_t[less] = ti;
        } else if (eq_before == 0) {
            int *ring = idx + less;  // hit numbers, later replaced by face ids
            int head = 0, len = 0;
            for (int j = i; j < cnt; ++j) {
                const float tj = h_t[j];
                if (tj == ti) {
                    ring[(head + len) % eq] = j;
                    ++len;
                } else if (tj < ti && len > 0) {
                    if (len < eq) ring[(head + len) % eq] = ring[head];
                    head = (head + 1) % eq;
                }
            }
            // slot q takes ring[(head + q) % eq]: park the hit numbers in the
            // min-cage words (rewritten below) so the ring can be overwritten
            for (int q = 0; q < eq; ++q) depth[(less + q) * 3 + 1] = __int_as_float(ring[(head + q) % eq]);
            for (int q = 0; q < eq; ++q) {
                const int hq = __float_as_int(depth[(less + q) * 3 + 1]);
                idx[less + q] = h_k[hq];
                depth[(less + q) * 3] = ti;
                uv[(less + q) * 2] = h_u[hq];
                uv[(less + q) * 2 + 1] = h_v[hq];
                s_t[less + q] = ti;
            }
        }
    }
    __syncthreads();
    // intersect_gpu.cu:354-368: half the gap to each neighbour, capped at cagesize
    for (int l = lane; l < cnt; l += kWave) {
        depth[l * 3 + 1] = (l == 0) ? -cagesize : -fminf(cagesize, 0.5f * (s_t[l] - s_t[l - 1]));
        depth[l * 3 + 2] = (l == cnt - 1) ? cagesize : fminf(cagesize, 0.5f * (s_t[l + 1] - s_t[l]));
    }
    for (int l = cnt + lane; l < n_max; l += kWave) idx[l] = -1;
}

// sample_gpu.cu:13-124, one lane per ray, in place in the output rows like
// the reference.  Two places where the reference leaves its own row are
// pinned here: reads past the row (pts_idx[H + umin - 1] at umin = 0, and
// umin past max_hits) read the neighbouring row of the flat array as the
// reference does (-1 outside the array), and writes past max_steps — the
// reference's write into the next ray's row, a race between lanes — are
// dropped.  The merge is bounded by its event count so NaN depths cannot
// spin it forever.
__global__ __launch_bounds__(kWave) void k_uniform_sampling(int b, int num_rays, int max_hits, int max_steps,
                                                          float step_size, const int *__restrict__ pts_idx,
                                                          const float *__restrict__ min_depth,
                                                          const float *__restrict__ max_depth,
                                                          const float *__restrict__ uniform_noise,
                                                          int *sampled_idx, float *sampled_depth,
                                                          float *sampled_dists) {
    const int64_t ray = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)b * num_rays;
    if (ray >= total) return;
    const int64_t n_idx = total * max_hits;
    const int64_t H = ray * max_hits, K = ray * max_steps;
    auto pidx = [&](int64_t at) { return (at >= 0 && at < n_idx) ? pts_idx[at] : -1; };
    auto mind = [&](int64_t at) { return (at >= 0 && at < n_idx) ? min_depth[at] : 0.0f; };
    int s = 0, ucur = 0, umin = 0, umax = 0;
    float curr_depth = 0.0f;
    const float d0 = min_depth[H];
    for (int guard = 0; guard <= max_steps + 2 * max_hits + 2; ++guard) {
        if (umax == max_hits || ucur == max_steps || pidx(H + umax) == -1) break;
        const float last_min = (umin < max_hits) ? min_depth[H + umin] : 10000.0f;
        const float last_max = (umax < max_hits) ? max_depth[H + umax] : 10000.0f;
        curr_depth = d0 + ((float)ucur + uniform_noise[K + ucur]) * step_size;
        float dep;
        int id;
        if (last_max <= curr_depth && last_max <= last_min) {
            dep = last_max;
            id = pidx(H + umax);
            ++umax;
        } else if (curr_depth <= last_min && curr_depth <= last_max) {
            dep = curr_depth;
            id = pidx(H + umin - 1);
            ++ucur;
        } else if (last_min <= curr_depth && last_min <= last_max) {
            dep = last_min;
            id = pidx(H + umin);
            ++umin;
        } else {
            continue;
        }
        if (s < max_steps) {
            sampled_depth[K + s] = dep;
            sampled_idx[K + s] = id;
        }
        ++s;
    }
    int step = 0;
    umin = 0;
    umax = 0;
    for (ucur = 0; ucur < max_steps - 1; ++ucur) {
        if (sampled_idx[K + ucur + 1] == -1) break;
        const float l_depth = sampled_depth[K + ucur];
        const float r_depth = sampled_depth[K + ucur + 1];
        const float mid = (l_depth + r_depth) * 0.5f;
        const float dist = r_depth - l_depth;
        sampled_depth[K + ucur] = mid;
        sampled_dists[K + ucur] = dist;
        if (umin < max_hits && mid >= mind(H + umin) && pidx(H + umin) > -1) ++umin;
        if (umax < max_hits && mid >= max_depth[H + umax] && pidx(H + umax) > -1) ++umax;
        if (umax == max_hits || pidx(H + umax) == -1) break;
        if (umin - 1 == umax && dist > 0.0f) {
            sampled_depth[K + step] = mid;
            sampled_dists[K + step] = dist;
            sampled_idx[K + step] = sampled_idx[K + ucur];
            ++step;
        }
    }
    for (int l = step; l < max_steps; ++l) sampled_idx[K + l] = -1;
}

}  // namespace
}  // namespace psvo

using namespace psvo;

extern "C" int psvo_ball_intersect(void *stream, int b, int n, int m, float radius, int n_max,
                                   const float *ray_start, const float *ray_dir, const float *points, int *idx,
                                   float *min_depth, float *max_depth) {
    PSVO_REQUIRE(b >= 0 && n >= 0 && m >= 0 && n_max > 0, "ball_intersect: bad sizes b=%d n=%d m=%d n_max=%d", b, n,
                 m, n_max);
    const int64_t total = (int64_t)b * m;
    if (total == 0) return PSVO_OK;
    if (n_max <= kGaSplitHits && n >= kGaSplitMinN)
        psvo::launch(k_ball_intersect<true>, dim3(div_up(total, kGaWaves / kGaSegs)), dim3(kGaWaves * kWave), 0,
                     as_stream(stream), b, n, m, radius, n_max, ray_start, ray_dir, points, idx, min_depth, max_depth);
    else
        psvo::launch(k_ball_intersect<false>, dim3(div_up(total, kGaWaves)), dim3(kGaWaves * kWave), 0, as_stream(stream), b,
                     n, m, radius, n_max, ray_start, ray_dir, points, idx, min_depth, max_depth);
    return check_launch("ball_intersect");
}

extern "C" int psvo_aabb_intersect(void *stream, int b, int n, int m, float voxelsize, int n_max,
                                   const float *ray_start, const float *ray_dir, const float *points, int *idx,
                                   float *min_depth, float *max_depth) {
    PSVO_REQUIRE(b >= 0 && n >= 0 && m >= 0 && n_max > 0, "aabb_intersect: bad sizes b=%d n=%d m=%d n_max=%d", b, n,
                 m, n_max);
    const int64_t total = (int64_t)b * m;
    if (total == 0) return PSVO_OK;
    if (n_max <= kGaSplitHits && n >= kGaSplitMinN)
        psvo::launch(k_aabb_intersect<true>, dim3(div_up(total, kGaWaves / kGaSegs)), dim3(kGaWaves * kWave), 0,
                     as_stream(stream), b, n, m, voxelsize, n_max, ray_start, ray_dir, points, idx, min_depth, max_depth);
    else
        psvo::launch(k_aabb_intersect<false>, dim3(div_up(total, kGaWaves)), dim3(kGaWaves * kWave), 0, as_stream(stream), b,
                     n, m, voxelsize, n_max, ray_start, ray_dir, points, idx, min_depth, max_depth);
    return check_launch("aabb_intersect");
}

extern "C" int psvo_triangle_intersect(void *stream, int b, int n, int m, float cagesize, float blur, int n_max,
                                       const float *ray_start, const float *ray_dir, const float *face_points,
                                       int *idx, float *depth, float *uv) {
    PSVO_REQUIRE(b >= 0 && n >= 0 && m >= 0 && n_max > 0, "triangle_intersect: bad sizes b=%d n=%d m=%d n_max=%d",
                 b, n, m, n_max);
    PSVO_REQUIRE(n_max <= kTriMaxHits, "triangle_intersect: n_max=%d exceeds %d", n_max, kTriMaxHits);
    const int64_t total = (int64_t)b * m;
    if (total == 0) return PSVO_OK;
    PSVO_REQUIRE(total <= 0x7fffffff, "triangle_intersect: %lld rays exceed the grid", (long long)total);
    psvo::launch(k_triangle_intersect, dim3((unsigned)total), dim3(kWave), (size_t)n_max * 5 * sizeof(float),
                 as_stream(stream), b, n, m, cagesize, blur, n_max, ray_start, ray_dir, face_points, idx, depth, uv);
    return check_launch("triangle_intersect");
}

extern "C" int psvo_uniform_ray_sampling(void *stream, int b, int num_rays, int max_hits, int max_steps,
                                         float step_size, const int *pts_idx, const float *min_depth,
                                         const float *max_depth, const float *uniform_noise, int *sampled_idx,
                                         float *sampled_depth, float *sampled_dists) {
    PSVO_REQUIRE(b >= 0 && num_rays >= 0 && max_hits > 0 && max_steps > 0,
                 "uniform_ray_sampling: bad sizes b=%d num_rays=%d max_hits=%d max_steps=%d", b, num_rays, max_hits,
                 max_steps);
    const int64_t total = (int64_t)b * num_rays;
    if (total == 0) return PSVO_OK;
    // one wave per workgroup: a few thousand serial rays spread over all CUs
    psvo::launch(k_uniform_sampling, dim3(div_up(total, kWave)), dim3(kWave), 0, as_stream(stream), b, num_rays,
                 max_hits, max_steps, step_size, pts_idx, min_depth, max_depth, uniform_noise, sampled_idx,
                 sampled_depth, sampled_dists);
    return check_launch("uniform_ray_sampling");
}
