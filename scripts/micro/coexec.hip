// Microbenchmark: do f32 MFMA (v_mfma_f32_16x16x4_f32) on waves 0-3 and
// packed f32 FMA (v_pk_fma_f32) on waves 4-7 of the same SIMDs run
// concurrently at their separate rates, or share one f32 datapath?
// mode 0: MFMA waves only, 1: VALU waves only, 2: both.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef float f32x2v __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(512, 1) void k(int mode, int iters, float *out) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const float a = threadIdx.x * 1e-3f, b = 1.0f - threadIdx.x * 1e-4f;
    if (wave < 4) {
        if (mode == 1) return;
        f32x4v c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
                c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
                c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
            }
        }
        f32x4v s = c0 + c1 + c2 + c3;
        out[blockIdx.x * 512 + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
    } else {
        if (mode == 0) return;
        f32x2v v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = f32x2v{a * j, b * j};
        const f32x2v m2 = {a, b}, c2 = {b, a};
        // one MFMA 16x16x4 = 1024 FMA per wave; one v_pk_fma = 128 FMA per wave:
        // 32 MFMAs per iteration = 256 pk_fma per iteration for equal FMA counts
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int j = 0; j < 32; ++j) {
#pragma unroll
                for (int t = 0; t < 8; ++t) v[t] = __builtin_elementwise_fma(v[t], m2, c2);
            }
        }
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[j][0] + v[j][1];
        out[blockIdx.x * 512 + threadIdx.x] = s;
    }
}

int main() {
    float *out;
    hipMalloc(&out, 1024 * 512 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 2000, blocks = 256;
    for (int rep = 0; rep < 2; ++rep)
        for (int mode = 0; mode < 3; ++mode) {
            hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, mode, 10, out);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, mode, iters, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double fma_per_side = (double)blocks * 4 * iters * 32 * 1024;  // per role
            const double fl = 2.0 * fma_per_side * (mode == 2 ? 2 : 1);
            printf("mode %d (%s): %.3f ms, %.1f TFLOP/s\n", mode, mode == 0 ? "mfma" : mode == 1 ? "valu" : "both", ms,
                   fl / ms / 1e9);
        }
    return 0;
}
