// Diagnostic microbenchmark (not the product): does a kernel that stores a
// few words to pinned host memory (system-scope relaxed atomics, as the
// sampler's statistics read-back does) delay the next kernel on its stream?
// Kernel A: 1,024 workgroups write 8 MB of device data (as a sampler's rows),
// its last workgroup stores 16 words to (a) device memory or (b) pinned host
// memory; kernel B (one workgroup) follows.  The gap B.start − A.end is read
// from s_memrealtime stamps (100 MHz) taken in A's last store and at B's
// start.  Also: (c) B queued behind a hipStreamWaitEvent on an event another
// stream recorded long before (a satisfied cross-stream barrier).
// Build: hipcc --offload-arch=gfx950 -O3 -o hostwrite_gap hostwrite_gap.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ __forceinline__ unsigned long long rt() { return __builtin_amdgcn_s_memrealtime(); }

__global__ void k_a(float *rows, unsigned long long *dst, unsigned long long *stamp, int n_per) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    for (int i = 0; i < n_per; ++i) rows[(size_t)t * n_per + i] = (float)(t + i);
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x < 16) {
        __hip_atomic_store(dst + threadIdx.x, 0x100000000ull | threadIdx.x, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        if (threadIdx.x == 0) stamp[0] = rt();
    }
}

__global__ void k_b(unsigned long long *stamp) {
    if (threadIdx.x == 0) stamp[1] = rt();
}

__global__ void k_c() {}

// spins ~us microseconds (s_memrealtime, 100 MHz)
__global__ void k_spin(int us) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)us * 100ull) __builtin_amdgcn_s_sleep(2);
}

int main() {
    float *rows;
    unsigned long long *dev, *host, *stamp;
    hipMalloc(&rows, 1024 * 256 * 8 * sizeof(float));
    hipMalloc(&dev, 16 * 8);
    hipHostMalloc(&host, 16 * 8, hipHostMallocDefault);
    hipHostMalloc(&stamp, 2 * 8, hipHostMallocDefault);
    hipStream_t s, s2;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    hipEvent_t ev;
    hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventDisableSystemFence);
    hipEvent_t clk, mk;
    hipEventCreateWithFlags(&clk, hipEventReleaseToDevice);  // a timed marker, device-scope release
    hipEventCreateWithFlags(&mk, hipEventDisableTiming | hipEventDisableSystemFence);
    for (int mode = 0; mode < 8; ++mode) {
        double sum = 0.0;
        const int reps = 20;
        for (int r = 0; r < reps + 3; ++r) {
            if (mode & 2) {  // an event on another stream, satisfied long before
                hipLaunchKernelGGL(k_c, dim3(1), dim3(64), 0, s2);
                hipEventRecord(ev, s2);
                hipStreamSynchronize(s2);
            }
            hipLaunchKernelGGL(k_a, dim3(1024), dim3(256), 0, s, rows, (mode & 1) ? host : dev, stamp, 8);
            if (mode >= 4) hipEventRecord(mk, s);   // the query's done marker
            if (mode >= 6) hipEventRecord(clk, s);  // the step clock's timed marker
            if (mode >= 2 && (mode & 2)) hipStreamWaitEvent(s, ev, 0);
            hipLaunchKernelGGL(k_b, dim3(1), dim3(64), 0, s, stamp);
            hipStreamSynchronize(s);
            if (r >= 3) sum += (double)(stamp[1] - stamp[0]) / 100.0;  // 100 MHz → µs
        }
        printf("%s stats%s%s%s: gap A.last-store -> B.start %.2f us\n", (mode & 1) ? "host" : "device",
               (mode & 2) ? " + satisfied wait" : "", mode >= 4 ? " + marker" : "", mode >= 6 ? " + timed marker" : "",
               sum / reps);
    }
    // a cross-stream wait on an event NOT complete when the host queues it:
    // s2 spins `us` then records; s runs A (then waits, then B)
    for (int us : {2, 10, 30, 60}) {
        double sum = 0.0, a_dur = 0.0;
        const int reps = 20;
        for (int r = 0; r < reps + 3; ++r) {
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s2, us);
            hipEventRecord(ev, s2);
            hipLaunchKernelGGL(k_a, dim3(1024), dim3(256), 0, s, rows, dev, stamp, 64);
            hipStreamWaitEvent(s, ev, 0);
            hipLaunchKernelGGL(k_b, dim3(1), dim3(64), 0, s, stamp);
            hipStreamSynchronize(s);
            hipStreamSynchronize(s2);
            if (r >= 3) sum += (double)(stamp[1] - stamp[0]) / 100.0;
        }
        printf("pending cross-stream wait (other stream spins %d us): gap A.last-store -> B.start %.2f us\n", us,
               sum / reps);
    }
    return 0;
}
