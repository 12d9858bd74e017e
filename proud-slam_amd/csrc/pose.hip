// Camera pose of the tracking loop on the device.
//
// Reference: track_frame (render_helpers.py:679-761) optimises an SE(3) pose
// (se3pose.py:8-98; parameters [t | w], w axis-angle) through
//   rays_d = dirs_cam @ R(w)ᵀ,  rays_o = t           (render_helpers.py:714-716)
//   R = I + A(θ²)·W + B(θ²)·W²,  W = [w]×,  A = sin θ/θ,  B = (1 − cos θ)/θ²
// with A, B as 10th-order Taylor series in θ² (se3pose.py:27-44).  Two
// kernels: the world rays from the pose (one thread per ray, R recomputed per
// thread from the six parameters — 11 multiply-adds), and the pose gradient
// from the interpolation backward's per-ray grad_o / grad_d:
//   dL/dt   = Σ_r grad_o[r]
//   G_jk    = dL/dR_jk = Σ_r grad_d[r]_j · dir[r]_k
//   dL/dw_k = Σ_jk G_jk · (2w_k A′·W + A·E_k + 2w_k B′·W² + B·(E_k W + W E_k))_jk
// (E_k = [e_k]×, A′ = dA/d(θ²)), i.e. what autograd derives through
// rotation() — one block, a fixed-order reduction.
#include <hip/hip_runtime.h>

#include <cmath>

#include "psvo_common.h"

namespace psvo {
namespace {

constexpr int kSeriesN = 10;

// Horner evaluation of Σ_i (−1)^i y^i / d_i (d_0 = d0, d_i = d_{i−1}·step(i))
// and its derivative in y; `a` selects sin θ/θ (step (2i)(2i+1), d0 = 1) or
// (1 − cos θ)/θ² (step (2i+1)(2i+2), d0 = 2).
__device__ __forceinline__ void series(float y, bool a, float &p, float &dp) {
    float c[kSeriesN + 1];
    double den = a ? 1.0 : 2.0;
    for (int i = 0; i <= kSeriesN; ++i) {
        if (i > 0) den *= a ? (double)(2 * i) * (2 * i + 1) : (double)(2 * i + 1) * (2 * i + 2);
        c[i] = (float)((i & 1 ? -1.0 : 1.0) / den);
    }
    p = c[kSeriesN];
    dp = 0.f;
    for (int i = kSeriesN - 1; i >= 0; --i) {
        dp = dp * y + p;
        p = p * y + c[i];
    }
}

struct Rot {
    float w[3], W[3][3], W2[3][3], A, B, dA, dB;
    float R[3][3];
};

__device__ __forceinline__ void rotation(const float *__restrict__ pose, Rot &q) {
    q.w[0] = pose[3];
    q.w[1] = pose[4];
    q.w[2] = pose[5];
    const float y = q.w[0] * q.w[0] + q.w[1] * q.w[1] + q.w[2] * q.w[2];
    series(y, true, q.A, q.dA);
    series(y, false, q.B, q.dB);
    const float(&w)[3] = q.w;
    float W[3][3] = {{0.f, -w[2], w[1]}, {w[2], 0.f, -w[0]}, {-w[1], w[0], 0.f}};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            q.W[i][j] = W[i][j];
            q.W2[i][j] = W[i][0] * W[0][j] + W[i][1] * W[1][j] + W[i][2] * W[2][j];
        }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) q.R[i][j] = (i == j ? 1.f : 0.f) + q.A * q.W[i][j] + q.B * q.W2[i][j];
}

__global__ __launch_bounds__(256) void k_pose_rays(int64_t n, const float *__restrict__ pose,
                                                   const float *__restrict__ dirs, float *__restrict__ rays_o,
                                                   float *__restrict__ rays_d) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    Rot q;
    rotation(pose, q);
    const float d0 = dirs[r * 3 + 0], d1 = dirs[r * 3 + 1], d2 = dirs[r * 3 + 2];
    for (int j = 0; j < 3; ++j) {
        rays_d[r * 3 + j] = d0 * q.R[j][0] + d1 * q.R[j][1] + d2 * q.R[j][2];
        rays_o[r * 3 + j] = pose[j];
    }
}

constexpr int kGradThreads = 1024;

// bundle_adjust_frames (render_helpers.py:620-640): frame f's rays are
// [f·rpf, (f+1)·rpf), rays_d = dirs @ R(w_f)ᵀ, rays_o = t_f
__global__ __launch_bounds__(256) void k_pose_rays_frames(int64_t n, int64_t rpf, const float *__restrict__ poses,
                                                          const float *__restrict__ dirs, float *__restrict__ rays_o,
                                                          float *__restrict__ rays_d) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const float *pose = poses + (r / rpf) * 6;
    Rot q;
    rotation(pose, q);
    const float d0 = dirs[r * 3 + 0], d1 = dirs[r * 3 + 1], d2 = dirs[r * 3 + 2];
    for (int j = 0; j < 3; ++j) {
        rays_d[r * 3 + j] = d0 * q.R[j][0] + d1 * q.R[j][1] + d2 * q.R[j][2];
        rays_o[r * 3 + j] = pose[j];
    }
}

// dL/d[t | w] of one pose from Σ grad_o (tot[0..2]) and G = Σ grad_d ⊗ dir (tot[3..11])
__device__ void pose_chain(const float *__restrict__ pose, const float (&tot)[12], float *__restrict__ grad);

// Σ over the hit rays of ray range [ray_lo, ray_hi) (hit ranks keep ray order,
// so they are one contiguous run of rank_ray) → pose gradient; block = frame
// Σ over the frame's hit rays [lo, hi) (rank order, thread t: ranks t,
// t + kGradThreads, …) of d rays_o and of d rays_d ⊗ dir: the rank → ray
// reads of up to kPoseBatch ranks issued together, then their gradient rows,
// then the sums in rank order — the same additions as one rank at a time,
// without a dependent pair of memory round trips per rank
constexpr int kPoseBatch = 4;  // 8 spilled 14 VGPRs to scratch at 1,024 threads (128 VGPRs per lane)
__device__ __forceinline__ void frame_ray_sums(int64_t r_hit, const int *__restrict__ rank_ray, int64_t lo, int64_t hi,
                                               const float *__restrict__ dirs, const float *__restrict__ g_o,
                                               const float *__restrict__ g_d, float (&acc)[12]) {
    for (int64_t r0 = threadIdx.x; r0 < r_hit; r0 += (int64_t)kGradThreads * kPoseBatch) {
        int64_t row[kPoseBatch];
#pragma unroll
        for (int k = 0; k < kPoseBatch; ++k) {
            const int64_t r = r0 + (int64_t)k * kGradThreads;
            row[k] = r < r_hit ? rank_ray[r] : -1;
        }
        float go[kPoseBatch][3], gd[kPoseBatch][3], dir[kPoseBatch][3];
#pragma unroll
        for (int k = 0; k < kPoseBatch; ++k) {
            const bool in = row[k] >= lo && row[k] < hi;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                go[k][j] = in ? g_o[row[k] * 3 + j] : 0.f;
                gd[k][j] = in ? g_d[row[k] * 3 + j] : 0.f;
                dir[k][j] = in ? dirs[row[k] * 3 + j] : 0.f;
            }
        }
#pragma unroll
        for (int k = 0; k < kPoseBatch; ++k) {
            if (!(row[k] >= lo && row[k] < hi)) continue;
            for (int j = 0; j < 3; ++j) acc[j] += go[k][j];
            for (int j = 0; j < 3; ++j)
                for (int i = 0; i < 3; ++i) acc[3 + j * 3 + i] += gd[k][j] * dir[k][i];
        }
    }
}

__global__ __launch_bounds__(kGradThreads) void k_pose_grad_frames(int64_t r_hit, const int *__restrict__ rank_ray,
                                                                   int64_t rpf, const float *__restrict__ dirs,
                                                                   const float *__restrict__ g_o,
                                                                   const float *__restrict__ g_d,
                                                                   const float *__restrict__ poses,
                                                                   float *__restrict__ grads) {
    __shared__ float part[kGradThreads / 64][12];
    const int64_t lo = blockIdx.x * rpf, hi = lo + rpf;
    float acc[12] = {};
    frame_ray_sums(r_hit, rank_ray, lo, hi, dirs, g_o, g_d, acc);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int i = 0; i < 12; ++i) {
        float v = acc[i];
#pragma unroll
        for (int s = 32; s > 0; s >>= 1) v += __shfl_xor(v, s, 64);
        if (lane == 0) part[wv][i] = v;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    float tot[12] = {};
    for (int w = 0; w < kGradThreads / 64; ++w)
        for (int i = 0; i < 12; ++i) tot[i] += part[w][i];
    pose_chain(poses + blockIdx.x * 6, tot, grads + blockIdx.x * 8);
}

// The engine's per-frame sums (bundle_adjust_frames' look-ahead and its
// unpipelined step): thread t takes the frame's rays lo + t, lo + t + T, …
// directly — a hit ray is one with ray_rank >= 0, its gradient rows are read
// beside the rank (one memory round trip, not rank → ray → rows) — then the
// wave butterflies and the 16 wave partials summed by 12 threads in wave
// order: a fixed order, so every run gives the same bits.
__device__ __forceinline__ void frame_sums_direct(const int *__restrict__ ray_rank, int64_t lo, int64_t hi,
                                                  const float *__restrict__ dirs, const float *__restrict__ g_o,
                                                  const float *__restrict__ g_d, float (&part)[kGradThreads / 64][12],
                                                  float (&tot)[12]) {
    float acc[12] = {};
    for (int64_t r = lo + threadIdx.x; r < hi; r += kGradThreads) {
        const bool in = ray_rank[r] >= 0;  // the rows of a ray without hits are not written
        float go[3], gd[3], dir[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            go[j] = g_o[r * 3 + j];
            gd[j] = g_d[r * 3 + j];
            dir[j] = dirs[r * 3 + j];
        }
        if (!in) continue;
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[j] += go[j];
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int i = 0; i < 3; ++i) acc[3 + j * 3 + i] += gd[j] * dir[i];
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        float v = acc[i];
#pragma unroll
        for (int s = 32; s > 0; s >>= 1) v += __shfl_xor(v, s, 64);
        if (lane == 0) part[wv][i] = v;
    }
    __syncthreads();
    if (threadIdx.x < 12) {
        float t = 0.f;
        for (int w = 0; w < kGradThreads / 64; ++w) t += part[w][threadIdx.x];
        tot[threadIdx.x] = t;
    }
    __syncthreads();
}

__global__ __launch_bounds__(kGradThreads) void k_pose_grad_rays(const int *__restrict__ ray_rank, int64_t rpf,
                                                                 const float *__restrict__ dirs,
                                                                 const float *__restrict__ g_o,
                                                                 const float *__restrict__ g_d,
                                                                 const float *__restrict__ poses,
                                                                 float *__restrict__ grads) {
    __shared__ float part[kGradThreads / 64][12];
    __shared__ float tot[12];
    const int64_t lo = blockIdx.x * rpf;
    frame_sums_direct(ray_rank, lo, lo + rpf, dirs, g_o, g_d, part, tot);
    if (threadIdx.x != 0) return;
    float t[12];
    for (int i = 0; i < 12; ++i) t[i] = tot[i];
    pose_chain(poses + blockIdx.x * 6, t, grads + blockIdx.x * 8);
}

struct PoseStepArgs {
    int64_t step[kXchMaxFrames];
    float lr_bc1[kXchMaxFrames], bc2_sqrt[kXchMaxFrames];
};

// k_pose_grad_rays + k_adam on the frame's pose + k_pose_rays_frames for the
// frame's next rays, one block per frame (a frame's rays, gradient and pose
// are its own: no grid-wide dependency); the updated rotation is formed once
// (thread 0) and shared through LDS
__global__ __launch_bounds__(kGradThreads) void k_pose_step_frames(
    const int *__restrict__ ray_rank, int64_t rpf, const float *__restrict__ dirs, const float *__restrict__ g_o,
    const float *__restrict__ g_d, float *__restrict__ poses, float *__restrict__ pose_m, float *__restrict__ pose_v,
    PoseStepArgs a, float beta1, float beta2, float omb1, float omb2, float eps, float *__restrict__ grads,
    const float *__restrict__ next_dirs, float *__restrict__ rays_o, float *__restrict__ rays_d) {
    __shared__ float part[kGradThreads / 64][12];
    __shared__ float tot[12];
    __shared__ float rot_s[12];  // R row-major, then t
    __shared__ float pst[18];    // the frame's pose, Adam m, v (loaded beside the rays: no dependent
                                 // global round trips in the serial part)
    const int f = blockIdx.x;
    const int64_t lo = f * rpf, hi = lo + rpf;
    if (threadIdx.x >= 64 && threadIdx.x < 64 + 18) {  // (frame_sums_direct's barriers publish them)
        const int k = threadIdx.x - 64;
        pst[k] = k < 6 ? poses[f * 6 + k] : (pose_m ? (k < 12 ? pose_m[f * 6 + k - 6] : pose_v[f * 6 + k - 12]) : 0.f);
    }
    // the next rays' camera directions depend on nothing here: loaded first
    // (one thread per ray when rpf <= kGradThreads), beside the gradient rows
    const int64_t r1 = lo + threadIdx.x;
    float nd[3] = {0.f, 0.f, 0.f};
    if (rpf <= kGradThreads && r1 < hi)
        for (int j = 0; j < 3; ++j) nd[j] = next_dirs[r1 * 3 + j];
    frame_sums_direct(ray_rank, lo, hi, dirs, g_o, g_d, part, tot);
    if (threadIdx.x == 0) {
        float t[12];
        for (int i = 0; i < 12; ++i) t[i] = tot[i];
        float *g = grads + f * 8;
        float g6[8];
        pose_chain(pst, t, g6);
        for (int i = 0; i < 6; ++i) g[i] = g6[i];
        float p6[6];
        for (int i = 0; i < 6; ++i) p6[i] = pst[i];
        if (a.step[f] >= 1) {  // stamp 0 / update_pose False: fixed (render_helpers.py:594-596)
            for (int i = 0; i < 6; ++i) {
                float mi = pst[6 + i], vi = pst[12 + i];
                adam_elem(p6[i], g6[i], mi, vi, beta1, beta2, omb1, omb2, eps, 0.0f, a.lr_bc1[f], a.bc2_sqrt[f]);
                poses[f * 6 + i] = p6[i];
                pose_m[f * 6 + i] = mi;
                pose_v[f * 6 + i] = vi;
            }
        }
        Rot q;
        rotation(p6, q);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) rot_s[i * 3 + j] = q.R[i][j];
        for (int j = 0; j < 3; ++j) rot_s[9 + j] = p6[j];
    }
    __syncthreads();
    float R[3][3], t0[3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[i][j] = rot_s[i * 3 + j];
    for (int j = 0; j < 3; ++j) t0[j] = rot_s[9 + j];
    if (rpf <= kGradThreads) {
        if (r1 < hi)
            for (int j = 0; j < 3; ++j) {
                rays_d[r1 * 3 + j] = nd[0] * R[j][0] + nd[1] * R[j][1] + nd[2] * R[j][2];
                rays_o[r1 * 3 + j] = t0[j];
            }
        return;
    }
    for (int64_t r = lo + threadIdx.x; r < hi; r += kGradThreads) {
        const float d0 = next_dirs[r * 3 + 0], d1 = next_dirs[r * 3 + 1], d2 = next_dirs[r * 3 + 2];
        for (int j = 0; j < 3; ++j) {
            rays_d[r * 3 + j] = d0 * R[j][0] + d1 * R[j][1] + d2 * R[j][2];
            rays_o[r * 3 + j] = t0[j];
        }
    }
}

__global__ __launch_bounds__(kGradThreads) void k_pose_grad(int64_t r_hit, const int *__restrict__ rank_ray,
                                                            const float *__restrict__ dirs,
                                                            const float *__restrict__ g_o,
                                                            const float *__restrict__ g_d,
                                                            const float *__restrict__ pose, float *__restrict__ grad) {
    __shared__ float part[kGradThreads / 64][12];
    float acc[12] = {};
    for (int64_t r = threadIdx.x; r < r_hit; r += kGradThreads) {
        const int64_t row = rank_ray ? rank_ray[r] : r;
        float dir[3], gd[3];
        for (int j = 0; j < 3; ++j) {
            acc[j] += g_o[row * 3 + j];
            gd[j] = g_d[row * 3 + j];
            dir[j] = dirs[row * 3 + j];
        }
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 3; ++k) acc[3 + j * 3 + k] += gd[j] * dir[k];
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int i = 0; i < 12; ++i) {
        float v = acc[i];
#pragma unroll
        for (int s = 32; s > 0; s >>= 1) v += __shfl_xor(v, s, 64);
        if (lane == 0) part[wv][i] = v;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    float tot[12] = {};
    for (int w = 0; w < kGradThreads / 64; ++w)
        for (int i = 0; i < 12; ++i) tot[i] += part[w][i];
    pose_chain(pose, tot, grad);
}

__device__ void pose_chain(const float *__restrict__ pose, const float (&tot)[12], float *__restrict__ grad) {
    Rot q;
    rotation(pose, q);
    const float(&G)[3][3] = *reinterpret_cast<const float(*)[3][3]>(tot + 3);
    // Σ G∘W, Σ G∘W² and, per k, Σ G∘E_k, Σ G∘(E_k W + W E_k)
    float gw = 0.f, gw2 = 0.f;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            gw += G[i][j] * q.W[i][j];
            gw2 += G[i][j] * q.W2[i][j];
        }
    for (int k = 0; k < 3; ++k) {
        float e[3] = {0.f, 0.f, 0.f};
        e[k] = 1.f;
        const float E[3][3] = {{0.f, -e[2], e[1]}, {e[2], 0.f, -e[0]}, {-e[1], e[0], 0.f}};
        float ge = 0.f, gs = 0.f;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                ge += G[i][j] * E[i][j];
                float s = 0.f;
                for (int l = 0; l < 3; ++l) s += E[i][l] * q.W[l][j] + q.W[i][l] * E[l][j];
                gs += G[i][j] * s;
            }
        const float dy = 2.f * q.w[k];
        grad[3 + k] = dy * q.dA * gw + q.A * ge + dy * q.dB * gw2 + q.B * gs;
    }
    for (int j = 0; j < 3; ++j) grad[j] = tot[j];
}

}  // namespace
}  // namespace psvo

using namespace psvo;

extern "C" int psvo_pose_rays(void *stream, int64_t n, const float *pose, const float *dirs, float *rays_o,
                              float *rays_d) {
    PSVO_REQUIRE(n > 0, "pose_rays: bad size");
    PSVO_REQUIRE(pose && dirs && rays_o && rays_d, "pose_rays: null pointer");
    psvo::launch(k_pose_rays, dim3(div_up(n, 256)), dim3(256), 0, as_stream(stream), n, pose, dirs, rays_o,
                       rays_d);
    return check_launch("pose_rays");
}

extern "C" int psvo_pose_rays_frames(void *stream, int64_t n, int64_t rays_per_frame, const float *poses,
                                     const float *dirs, float *rays_o, float *rays_d) {
    PSVO_REQUIRE(n > 0 && rays_per_frame > 0 && n % rays_per_frame == 0, "pose_rays_frames: bad sizes");
    PSVO_REQUIRE(poses && dirs && rays_o && rays_d, "pose_rays_frames: null pointer");
    psvo::launch(k_pose_rays_frames, dim3(div_up(n, 256)), dim3(256), 0, as_stream(stream), n, rays_per_frame,
                       poses, dirs, rays_o, rays_d);
    return check_launch("pose_rays_frames");
}

extern "C" int psvo_pose_grad_frames(void *stream, int n_frames, int64_t rays_per_frame, int64_t r_hit,
                                     const int *rank_ray, const float *dirs, const float *g_o, const float *g_d,
                                     const float *poses, float *grads) {
    PSVO_REQUIRE(n_frames > 0 && rays_per_frame > 0 && r_hit >= 0, "pose_grad_frames: bad sizes");
    PSVO_REQUIRE(rank_ray && dirs && g_o && g_d && poses && grads, "pose_grad_frames: null pointer");
    psvo::launch(k_pose_grad_frames, dim3(n_frames), dim3(kGradThreads), 0, as_stream(stream), r_hit, rank_ray,
                       rays_per_frame, dirs, g_o, g_d, poses, grads);
    return check_launch("pose_grad_frames");
}

namespace psvo {
int pose_grad_frames_rays(hipStream_t st, int n_frames, int64_t rays_per_frame, const int *ray_rank,
                          const float *dirs, const float *g_o, const float *g_d, const float *poses, float *grads) {
    PSVO_REQUIRE(n_frames > 0 && rays_per_frame > 0, "pose_grad_frames: bad sizes");
    PSVO_REQUIRE(ray_rank && dirs && g_o && g_d && poses && grads, "pose_grad_frames: null pointer");
    psvo::launch(k_pose_grad_rays, dim3(n_frames), dim3(kGradThreads), 0, st, ray_rank, rays_per_frame, dirs, g_o,
                 g_d, poses, grads);
    return check_launch("pose_grad_frames");
}
int pose_step_frames(hipStream_t st, int n_frames, int64_t rays_per_frame, const int *ray_rank, const float *dirs,
                     const float *g_o, const float *g_d, float *poses, float *pose_m, float *pose_v,
                     const int64_t *steps, double lr, double beta1, double beta2, double eps, float *grads,
                     const float *next_dirs, float *rays_o, float *rays_d) {
    PSVO_REQUIRE(n_frames > 0 && n_frames <= kXchMaxFrames && rays_per_frame > 0, "pose_step_frames: bad sizes");
    PSVO_REQUIRE(ray_rank && dirs && g_o && g_d && poses && grads && next_dirs && rays_o && rays_d && steps,
                 "pose_step_frames: null pointer");
    PoseStepArgs a{};
    for (int f = 0; f < n_frames; ++f) {
        a.step[f] = steps[f];
        if (steps[f] < 1) continue;
        PSVO_REQUIRE(pose_m && pose_v, "pose_step_frames: pose Adam needs m / v");
        const double bc1 = 1.0 - std::pow(beta1, (double)steps[f]);  // as adam_launch forms them
        const double bc2 = 1.0 - std::pow(beta2, (double)steps[f]);
        a.lr_bc1[f] = (float)(lr / bc1);
        a.bc2_sqrt[f] = (float)std::sqrt(bc2);
    }
    psvo::launch(k_pose_step_frames, dim3(n_frames), dim3(kGradThreads), 0, st, ray_rank, rays_per_frame, dirs, g_o,
                 g_d, poses, pose_m, pose_v, a, (float)beta1, (float)beta2, (float)(1.0 - beta1), (float)(1.0 - beta2),
                 (float)eps, grads, next_dirs, rays_o, rays_d);
    return check_launch("pose_step_frames");
}
}  // namespace psvo

extern "C" int psvo_pose_grad(void *stream, int64_t r_hit, const int *rank_ray, const float *dirs, const float *g_o,
                              const float *g_d, const float *pose, float *grad) {
    PSVO_REQUIRE(r_hit >= 0, "pose_grad: bad size");
    PSVO_REQUIRE(dirs && g_o && g_d && pose && grad, "pose_grad: null pointer");
    psvo::launch(k_pose_grad, dim3(1), dim3(kGradThreads), 0, as_stream(stream), r_hit, rank_ray, dirs, g_o,
                       g_d, pose, grad);
    return check_launch("pose_grad");
}
