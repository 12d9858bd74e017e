// Adam step for many tensors in one launch (torch.optim.Adam semantics).
//
// Reference: the mapping loop steps torch.optim.Adam on the embeddings, the
// decoder and the keyframe poses every iteration (render_helpers.py:581-596,
// :668-672).  torch's foreach/fused implementations
// launch several multi-tensor kernels per optimizer; here every parameter
// tensor of a step is one grid: the tensor table travels in the kernel
// arguments, each 256-thread block takes a 4096-element slice of one tensor
// and streams (p, g, m, v) once — an HBM-bound 28 B per element.
//
//   g' = g + wd p
//   m  = β1 m + (1 − β1) g'
//   v  = β2 v + (1 − β2) g'²
//   p  = p − (lr / bc1) · m / (sqrt(v) / sqrt(bc2) + eps)
// with bc1 = 1 − β1^t, bc2 = 1 − β2^t and 1 − β (host, double, as torch
// forms them from Python floats) — torch's _fused_adam formulation
// (FusedAdamKernel), f32 arithmetic.
#include <hip/hip_runtime.h>

#include <cmath>

#include "psvo_common.h"

namespace psvo {
namespace {

constexpr int kAdamMaxTensors = 24;
constexpr int kAdamSlice = 1024;  // elements per block (4 per thread)

struct AdamTable {
    float *p[kAdamMaxTensors];
    const float *g[kAdamMaxTensors];
    float *m[kAdamMaxTensors];
    float *v[kAdamMaxTensors];
    int64_t n[kAdamMaxTensors];
    float lr_bc1[kAdamMaxTensors];  // lr / (1 - β1^t) per tensor
    float bc2_sqrt[kAdamMaxTensors];  // sqrt(1 - β2^t) per tensor (tensors may be at different steps t)
    int zero_grad[kAdamMaxTensors]; // write 0 into the gradient after use
    const uint8_t *rows[kAdamMaxTensors];  // per-16-element-row flags: only flagged rows are stepped (NULL: all)
    int block_begin[kAdamMaxTensors + 1];
    int count;
};

__global__ __launch_bounds__(256) void k_adam(AdamTable tab, float beta1, float beta2, float omb1, float omb2,
                                              float eps, float wd) {
    int ti = 0;
    while (ti + 1 < tab.count && (int)blockIdx.x >= tab.block_begin[ti + 1]) ++ti;
    const int64_t base = (int64_t)(blockIdx.x - tab.block_begin[ti]) * kAdamSlice;
    const int64_t n = tab.n[ti];
    float *__restrict__ p = tab.p[ti];
    float *__restrict__ g = const_cast<float *>(tab.g[ti]);
    const float lr_bc1 = tab.lr_bc1[ti];
    const float bc2_sqrt = tab.bc2_sqrt[ti];
    const bool zg = tab.zero_grad[ti] != 0;
    float *__restrict__ m = tab.m[ti];
    float *__restrict__ v = tab.v[ti];
    const uint8_t *__restrict__ rf = tab.rows[ti];
    for (int64_t i = base + threadIdx.x; i < base + kAdamSlice && i < n; i += 256) {
        if (rf && !rf[i >> 4]) continue;  // a row never touched: g = m = v = 0, the step leaves it as it is
        float pi = p[i], mi = m[i], vi = v[i];
        adam_elem(pi, g[i], mi, vi, beta1, beta2, omb1, omb2, eps, wd, lr_bc1, bc2_sqrt);
        p[i] = pi;
        m[i] = mi;
        v[i] = vi;
        if (zg) g[i] = 0.0f;
    }
}

// Rows touched by a step: every vertex row of the leaves its samples
// interpolate (render_helpers.py:104-156: the rows that can receive an
// embedding gradient).  Flags are sticky — once touched, a row's moments are
// non-zero and Adam must step it every iteration (torch.optim.Adam steps all
// elements); a row never touched has g = m = v = 0, which the dense step
// leaves bit-for-bit unchanged, so skipping it is exact.
__global__ __launch_bounds__(256) void k_adam_mark_rows(int64_t m, const int *__restrict__ leaf,
                                                        const int *__restrict__ vertex_idx, uint8_t *__restrict__ rf) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m * 8) return;
    const int64_t s = e >> 3;
    const int v = vertex_idx[(int64_t)leaf[s] * 8 + (e & 7)];
    if (v >= 0 && !rf[v]) rf[v] = 1;
}

// flags of rows whose moments are already non-zero (a bound optimiser state)
__global__ __launch_bounds__(256) void k_adam_flags_from_state(int64_t n_rows, const float *__restrict__ m,
                                                               const float *__restrict__ v, uint8_t *__restrict__ rf) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rows) return;
    bool nz = false;
    for (int c = 0; c < 16; c += 4) {
        const float4 a = *reinterpret_cast<const float4 *>(m + r * 16 + c);
        const float4 b = *reinterpret_cast<const float4 *>(v + r * 16 + c);
        nz |= a.x != 0.f || a.y != 0.f || a.z != 0.f || a.w != 0.f || b.x != 0.f || b.y != 0.f || b.z != 0.f ||
              b.w != 0.f;
    }
    if (nz) rf[r] = 1;
}

}  // namespace
}  // namespace psvo

using namespace psvo;

extern "C" int psvo_adam_mark_rows(void *stream, int64_t m, const int *leaf, const int *vertex_idx, uint8_t *flags) {
    PSVO_REQUIRE(m >= 0, "adam_mark_rows: bad size");
    if (m == 0) return PSVO_OK;
    PSVO_REQUIRE(leaf && vertex_idx && flags, "adam_mark_rows: null pointer");
    psvo::launch(psvo::k_adam_mark_rows, dim3(psvo::div_up(m * 8, 256)), dim3(256), 0, psvo::as_stream(stream),
                       m, leaf, vertex_idx, flags);
    return psvo::check_launch("adam_mark_rows");
}

extern "C" int psvo_adam_flags_from_state(void *stream, int64_t n_rows, const float *exp_avg,
                                          const float *exp_avg_sq, uint8_t *flags) {
    PSVO_REQUIRE(n_rows >= 0, "adam_flags_from_state: bad size");
    if (n_rows == 0) return PSVO_OK;
    PSVO_REQUIRE(exp_avg && exp_avg_sq && flags, "adam_flags_from_state: null pointer");
    PSVO_REQUIRE(((uintptr_t)exp_avg & 15) == 0 && ((uintptr_t)exp_avg_sq & 15) == 0,
                 "adam_flags_from_state: moments must be 16-B aligned");
    psvo::launch(psvo::k_adam_flags_from_state, dim3(psvo::div_up(n_rows, 256)), dim3(256), 0,
                       psvo::as_stream(stream), n_rows, exp_avg, exp_avg_sq, flags);
    return psvo::check_launch("adam_flags_from_state");
}

// One launch over n_tensors tensors (chunks of kAdamMaxTensors); per-tensor
// learning rate, optional per-tensor step number (`steps`, else `step` for
// all: the engine steps the map and the keyframe poses, each pose at its own
// Adam step, in one launch) and optional gradient zeroing (the engine's
// accumulation buffer is left zeroed for the next iteration's float atomics).
int psvo::adam_launch(hipStream_t st, int n_tensors, float *const *params, const float *const *grads,
                      float *const *exp_avg, float *const *exp_avg_sq, const int64_t *numel, const double *lr,
                      double beta1, double beta2, double eps, double weight_decay, int64_t step,
                      const int *zero_grad, const int64_t *steps, const uint8_t *const *row_flags) {
    PSVO_REQUIRE(n_tensors >= 0 && (steps || step >= 1), "adam_step: bad arguments (n_tensors=%d step=%lld)",
                 n_tensors, (long long)step);
    int t = 0;
    while (t < n_tensors) {
        AdamTable tab;
        tab.count = 0;
        int blocks = 0;
        for (; t < n_tensors && tab.count < kAdamMaxTensors; ++t) {
            if (numel[t] == 0) continue;
            PSVO_REQUIRE(params[t] && grads[t] && exp_avg[t] && exp_avg_sq[t], "adam_step: null pointer (tensor %d)",
                         t);
            const int64_t tt = steps ? steps[t] : step;
            PSVO_REQUIRE(tt >= 1, "adam_step: tensor %d at step %lld", t, (long long)tt);
            const double bc1 = 1.0 - std::pow(beta1, (double)tt);
            const double bc2 = 1.0 - std::pow(beta2, (double)tt);
            const int k = tab.count++;
            tab.p[k] = params[t];
            tab.g[k] = grads[t];
            tab.m[k] = exp_avg[t];
            tab.v[k] = exp_avg_sq[t];
            tab.n[k] = numel[t];
            tab.lr_bc1[k] = (float)(lr[t] / bc1);
            tab.bc2_sqrt[k] = (float)std::sqrt(bc2);
            tab.zero_grad[k] = zero_grad ? zero_grad[t] : 0;
            tab.rows[k] = row_flags ? row_flags[t] : nullptr;
            tab.block_begin[k] = blocks;
            blocks += (int)div_up(numel[t], kAdamSlice);
        }
        tab.block_begin[tab.count] = blocks;
        if (blocks == 0) continue;
        psvo::launch(k_adam, dim3(blocks), dim3(256), 0, st, tab, (float)beta1, (float)beta2,
                           (float)(1.0 - beta1), (float)(1.0 - beta2), (float)eps, (float)weight_decay);
        const int rc = check_launch("adam_step");
        if (rc) return rc;
    }
    return PSVO_OK;
}

extern "C" int psvo_adam_step(void *stream, int n_tensors, float *const *params, const float *const *grads,
                              float *const *exp_avg, float *const *exp_avg_sq, const int64_t *numel, double lr,
                              double beta1, double beta2, double eps, double weight_decay, int64_t step) {
    PSVO_REQUIRE(n_tensors >= 0 && n_tensors <= 4096, "adam_step: bad n_tensors=%d", n_tensors);
    double lrs[4096];
    for (int i = 0; i < n_tensors; ++i) lrs[i] = lr;
    return adam_launch(as_stream(stream), n_tensors, params, grads, exp_avg, exp_avg_sq, numel, lrs, beta1, beta2,
                       eps, weight_decay, step, nullptr);
}
