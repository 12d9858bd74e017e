// Diagnostic microbenchmark (not the product): the trunk backward's chain
// GEMM (δ[128 × 16 samples] = Wᵀ[128 × 128] · δ', v_mfma_f32_16x16x4_f32)
// with the A operands (a) streamed from L2 through a 2-deep ring of buffer
// loads — every CU reading the same 64-KB image, as k_mlp_bwd3 / k_mlp_bwd3t
// do — and (b) read from an LDS copy of the image.  One 4-wave workgroup per
// CU, N_ITER GEMMs per wave; prints µs per launch and the MFMA-cycle bound.
// Build: hipcc --offload-arch=gfx950 -O3 -o gemm16_bench gemm16_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f32x4v __attribute__((ext_vector_type(4)));

constexpr int kNKB = 8, kNOB = 8, kIter = 64;

__device__ __forceinline__ f32x4v mfma16(float a, float b, f32x4v c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float4 bload4(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}

template <int D>
__device__ __forceinline__ void gemm_l2(__amdgpu_buffer_rsrc_t rs, const f32x4v (&in)[kNKB], f32x4v (&acc)[kNOB],
                                        int lane) {
    auto ld = [&](int kb, int ob) { return bload4(rs, lane * 16, ((ob * kNKB + kb) * 256) * 4); };
    float4 ring[D + 1][kNOB];
#pragma unroll
    for (int s = 0; s < D; ++s)
#pragma unroll
        for (int ob = 0; ob < kNOB; ++ob) ring[s][ob] = ld(s, ob);
#pragma unroll
    for (int kb = 0; kb < kNKB; ++kb) {
        const int cs = kb % (D + 1);
        if (kb + D < kNKB) {
#pragma unroll
            for (int ob = 0; ob < kNOB; ++ob) ring[(kb + D) % (D + 1)][ob] = ld(kb + D, ob);
        }
#pragma unroll
        for (int ob = 0; ob < kNOB; ++ob) acc[ob] = mfma16(ring[cs][ob].x, in[kb][0], acc[ob]);
#pragma unroll
        for (int ob = 0; ob < kNOB; ++ob) acc[ob] = mfma16(ring[cs][ob].y, in[kb][1], acc[ob]);
#pragma unroll
        for (int ob = 0; ob < kNOB; ++ob) acc[ob] = mfma16(ring[cs][ob].z, in[kb][2], acc[ob]);
#pragma unroll
        for (int ob = 0; ob < kNOB; ++ob) acc[ob] = mfma16(ring[cs][ob].w, in[kb][3], acc[ob]);
    }
}

__device__ __forceinline__ void gemm_lds(const float *w, const f32x4v (&in)[kNKB], f32x4v (&acc)[kNOB], int lane) {
#pragma unroll
    for (int kb = 0; kb < kNKB; ++kb) {
        float4 a[kNOB];
#pragma unroll
        for (int ob = 0; ob < kNOB; ++ob)
            a[ob] = *reinterpret_cast<const float4 *>(w + (ob * kNKB + kb) * 256 + lane * 4);
#pragma unroll
        for (int ob = 0; ob < kNOB; ++ob) acc[ob] = mfma16(a[ob].x, in[kb][0], acc[ob]);
#pragma unroll
        for (int ob = 0; ob < kNOB; ++ob) acc[ob] = mfma16(a[ob].y, in[kb][1], acc[ob]);
#pragma unroll
        for (int ob = 0; ob < kNOB; ++ob) acc[ob] = mfma16(a[ob].z, in[kb][2], acc[ob]);
#pragma unroll
        for (int ob = 0; ob < kNOB; ++ob) acc[ob] = mfma16(a[ob].w, in[kb][3], acc[ob]);
    }
}

template <int MODE>  // 0: L2 ring D=2, 1: LDS, 2: L2 ring D=4
__global__ __launch_bounds__(256) void k_bench(const float *__restrict__ img, float *__restrict__ out) {
    extern __shared__ float lds[];
    const int lane = threadIdx.x & 63;
    if (MODE == 1) {
        for (int i = threadIdx.x * 4; i < 128 * 128; i += 256 * 4)
            *reinterpret_cast<float4 *>(lds + i) = *reinterpret_cast<const float4 *>(img + i);
        __syncthreads();
    }
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(img), 0, 128 * 128 * 4, 0x00020000);
    f32x4v in[kNKB], acc[kNOB];
#pragma unroll
    for (int k = 0; k < kNKB; ++k) in[k] = f32x4v{1e-3f * lane, 1.f, 0.5f, 0.25f};
#pragma unroll
    for (int o = 0; o < kNOB; ++o) acc[o] = f32x4v{0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < kIter; ++it) {
        if (MODE == 0) gemm_l2<2>(rs, in, acc, lane);
        if (MODE == 2) gemm_l2<4>(rs, in, acc, lane);
        if (MODE == 1) gemm_lds(lds, in, acc, lane);
#pragma unroll
        for (int k = 0; k < kNKB; ++k) in[k] = acc[k] * 1e-3f;  // a data dependency between iterations
    }
    float s = 0.f;
#pragma unroll
    for (int o = 0; o < kNOB; ++o) s += acc[o][0] + acc[o][1] + acc[o][2] + acc[o][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float *img, *out;
    hipMalloc(&img, 128 * 128 * 4);
    hipMalloc(&out, (size_t)cus * 2 * 256 * 4);
    std::vector<float> h(128 * 128);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 1e-3f * (float)(i % 97);
    hipMemcpy(img, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipFuncSetAttribute(reinterpret_cast<const void *>(&k_bench<1>), hipFuncAttributeMaxDynamicSharedMemorySize,
                        65536);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    // MFMA bound: per wave kIter GEMMs × 256 MFMAs × 32 cycles; 4 waves = one per SIMD
    const double mfma_cycles = (double)kIter * kNKB * kNOB * 4 * 32;
    for (int wgs_per_cu = 1; wgs_per_cu <= 2; ++wgs_per_cu) {
        const int grid = cus * wgs_per_cu;
        for (int mode = 0; mode < 3; ++mode) {
            auto run = [&]() {
                if (mode == 0) hipLaunchKernelGGL(k_bench<0>, dim3(grid), dim3(256), 0, 0, img, out);
                if (mode == 1) hipLaunchKernelGGL(k_bench<1>, dim3(grid), dim3(256), 65536, 0, img, out);
                if (mode == 2) hipLaunchKernelGGL(k_bench<2>, dim3(grid), dim3(256), 0, 0, img, out);
            };
            for (int w = 0; w < 3; ++w) run();
            hipDeviceSynchronize();
            hipEventRecord(a, 0);
            for (int r = 0; r < 10; ++r) run();
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            float ms = 0.f;
            hipEventElapsedTime(&ms, a, b);
            const double us = ms * 100.0;  // per launch
            printf("wgs/CU %d mode %s: %.1f us per launch; MFMA bound %.1f us at 2.4 GHz (x%d waves per SIMD)\n",
                   wgs_per_cu, mode == 0 ? "L2 ring D=2" : mode == 1 ? "LDS      " : "L2 ring D=4", us,
                   mfma_cycles * wgs_per_cu / 2.4e3, wgs_per_cu);
        }
    }
    return 0;
}
