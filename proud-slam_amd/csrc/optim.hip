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
    for (int64_t i = base + threadIdx.x; i < base + kAdamSlice && i < n; i += 256) {
        float gi = g[i];
        float pi = p[i];
        if (wd != 0.0f) gi = gi + wd * pi;
        const float mi = beta1 * m[i] + omb1 * gi;
        const float vi = beta2 * v[i] + omb2 * gi * gi;
        const float denom = sqrtf(vi) / bc2_sqrt + eps;
        p[i] = pi - lr_bc1 * mi / denom;
        m[i] = mi;
        v[i] = vi;
        if (zg) g[i] = 0.0f;
    }
}

}  // namespace
}  // namespace psvo

using namespace psvo;

// One launch over n_tensors tensors (chunks of kAdamMaxTensors); per-tensor
// learning rate, optional per-tensor step number (`steps`, else `step` for
// all: the engine steps the map and the keyframe poses, each pose at its own
// Adam step, in one launch) and optional gradient zeroing (the engine's
// accumulation buffer is left zeroed for the next iteration's float atomics).
int psvo::adam_launch(hipStream_t st, int n_tensors, float *const *params, const float *const *grads,
                      float *const *exp_avg, float *const *exp_avg_sq, const int64_t *numel, const double *lr,
                      double beta1, double beta2, double eps, double weight_decay, int64_t step,
                      const int *zero_grad, const int64_t *steps) {
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
            tab.block_begin[k] = blocks;
            blocks += (int)div_up(numel[t], kAdamSlice);
        }
        tab.block_begin[tab.count] = blocks;
        if (blocks == 0) continue;
        hipLaunchKernelGGL(k_adam, dim3(blocks), dim3(256), 0, st, tab, (float)beta1, (float)beta2,
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
