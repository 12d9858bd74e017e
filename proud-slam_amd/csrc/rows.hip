// Row-sparse gradient exchange for data-parallel mapping on large maps
// (SURVEY §8e, config E): the embedding gradient of one step touches only the
// vertex rows of the leaves its rays sampled (≈ 8 rows per leaf visited), a
// small fraction of a ≥ 100 MB table, so ranks exchange (row id, row) pairs
// instead of all-reducing the dense table.
//   psvo_rows_compact:     ascending ids of the rows with a non-zero element,
//                          and those rows, packed (deterministic order)
//   psvo_rows_scatter_add: grad[ids[i]] += rows[i] for one rank's list (ids
//                          unique within a list: no atomics); applied rank by
//                          rank in the same order everywhere, so every replica
//                          forms the same sums bit for bit.
#include <hip/hip_runtime.h>

#include "psvo_common.h"

namespace psvo {
namespace {

constexpr int kRowsBlock = 1024;  // rows per block of the compaction scan

__device__ __forceinline__ bool row_nonzero(const float *__restrict__ g, int64_t r, int width) {
    bool nz = false;
    for (int c = 0; c < width; ++c) nz |= g[r * width + c] != 0.0f;
    return nz;
}

// the compaction's row predicate: a non-zero gradient row, or (flags given)
// a flagged row — the rows this rank's step touched (psvo_adam_mark_rows),
// found from n_rows bytes instead of the n_rows × width floats of the table
__device__ __forceinline__ bool row_taken(const float *__restrict__ g, const uint8_t *__restrict__ flags, int64_t r,
                                          int width) {
    return flags ? flags[r] != 0 : row_nonzero(g, r, width);
}

// pass 1: non-zero rows per block
__global__ __launch_bounds__(256) void k_rows_count(int64_t n_rows, int width, const float *__restrict__ g,
                                                    const uint8_t *__restrict__ flags, int *__restrict__ block_counts) {
    __shared__ int cnt;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    const int64_t r0 = (int64_t)blockIdx.x * kRowsBlock;
    int local = 0;
    for (int i = threadIdx.x; i < kRowsBlock; i += blockDim.x) {
        const int64_t r = r0 + i;
        if (r < n_rows && row_taken(g, flags, r, width)) ++local;
    }
    // wave reduction, then one LDS atomic per wave
    for (int s = 32; s > 0; s >>= 1) local += __shfl_xor(local, s, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(&cnt, local);
    __syncthreads();
    if (threadIdx.x == 0) block_counts[blockIdx.x] = cnt;
}

// pass 2: exclusive scan of the block counts (one block), total → count[0]
__global__ __launch_bounds__(1024) void k_rows_scan(int n_blocks, int *__restrict__ block_counts,
                                                    int *__restrict__ count) {
    __shared__ int part[1024];
    const int per = (n_blocks + 1023) / 1024;
    const int b0 = threadIdx.x * per;
    int s = 0;
    for (int i = 0; i < per && b0 + i < n_blocks; ++i) s += block_counts[b0 + i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // inclusive Hillis-Steele
        const int v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    int run = threadIdx.x > 0 ? part[threadIdx.x - 1] : 0;
    for (int i = 0; i < per && b0 + i < n_blocks; ++i) {
        const int c = block_counts[b0 + i];
        block_counts[b0 + i] = run;
        run += c;
    }
    if (threadIdx.x == 1023) count[0] = part[1023];
}

// pass 3: each block writes its non-zero rows in ascending order from its offset
__global__ __launch_bounds__(256) void k_rows_write(int64_t n_rows, int width, const float *__restrict__ g,
                                                    const uint8_t *__restrict__ flags,
                                                    const int *__restrict__ block_offsets, int *__restrict__ ids,
                                                    float *__restrict__ rows) {
    __shared__ int wave_base[4];
    const int64_t r0 = (int64_t)blockIdx.x * kRowsBlock;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int base = block_offsets[blockIdx.x];
    // 256 rows per round: thread t takes row r0 + round·256 + t; ranks by wave ballot + wave prefix
    for (int round = 0; round < kRowsBlock / 256; ++round) {
        const int64_t r = r0 + round * 256 + threadIdx.x;
        const bool nz = r < n_rows && row_taken(g, flags, r, width);
        const uint64_t bal = __ballot(nz);
        const int in_wave = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wave_base[wave] = __popcll(bal);
        __syncthreads();
        int before = base;
        for (int w = 0; w < wave; ++w) before += wave_base[w];
        const int total = wave_base[0] + wave_base[1] + wave_base[2] + wave_base[3];
        if (nz) {
            const int o = before + in_wave;
            ids[o] = (int)r;
            for (int c = 0; c < width; ++c) rows[(int64_t)o * width + c] = g[r * width + c];
        }
        base += total;
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_rows_scatter_add(int64_t n_list, int width, const int *__restrict__ ids,
                                                          const float *__restrict__ rows, float *__restrict__ g) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_list * width) return;
    const int64_t i = e / width;
    const int id = ids[i];
    if (id < 0) return;  // padding of a shorter list
    const int c = (int)(e - i * width);
    g[(int64_t)id * width + c] += rows[e];
}

// grad[ids[i]] = 0 and flags[ids[i]] = 0 (flags optional): a rank's own
// listed rows, before the lists are added back (sparse, no table pass)
__global__ __launch_bounds__(256) void k_rows_clear(int64_t n_list, int width, const int *__restrict__ ids,
                                                    float *__restrict__ g, uint8_t *__restrict__ flags) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_list * width) return;
    const int64_t i = e / width;
    const int id = ids[i];
    if (id < 0) return;
    const int c = (int)(e - i * width);
    g[(int64_t)id * width + c] = 0.0f;
    if (flags && c == 0) flags[id] = 0;
}

__global__ __launch_bounds__(256) void k_rows_mark(int64_t n_list, const int *__restrict__ ids,
                                                   uint8_t *__restrict__ flags) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_list) return;
    const int id = ids[i];
    if (id >= 0) flags[id] = 1;
}

__global__ __launch_bounds__(256) void k_rows_flags_from_grad(int64_t n_rows, int width, const float *__restrict__ g,
                                                              uint8_t *__restrict__ flags) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rows) return;
    if (row_nonzero(g, r, width)) flags[r] = 1;
}

}  // namespace
}  // namespace psvo

using namespace psvo;

extern "C" int64_t psvo_rows_workspace_ints(int64_t n_rows) { return (n_rows + kRowsBlock - 1) / kRowsBlock; }

static int rows_compact(void *stream, int64_t n_rows, int width, const float *grad, const uint8_t *flags,
                        int *workspace, int *ids, float *rows, int *count) {
    PSVO_REQUIRE(n_rows >= 0 && width > 0 && width <= 1024, "rows_compact: bad sizes");
    PSVO_REQUIRE(n_rows <= 0x7fffffff, "rows_compact: %lld rows exceed int32 ids", (long long)n_rows);
    PSVO_REQUIRE(count && (n_rows == 0 || (grad && workspace && ids && rows)), "rows_compact: null pointer");
    hipStream_t st = as_stream(stream);
    const int n_blocks = (int)psvo_rows_workspace_ints(n_rows);
    if (n_blocks == 0) {
        if (hipMemsetAsync(count, 0, sizeof(int), st) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "rows_compact: memset failed");
        return PSVO_OK;
    }
    psvo::launch(k_rows_count, dim3(n_blocks), dim3(256), 0, st, n_rows, width, grad, flags, workspace);
    psvo::launch(k_rows_scan, dim3(1), dim3(1024), 0, st, n_blocks, workspace, count);
    psvo::launch(k_rows_write, dim3(n_blocks), dim3(256), 0, st, n_rows, width, grad, flags, workspace, ids,
                       rows);
    return check_launch("rows_compact");
}

extern "C" int psvo_rows_compact(void *stream, int64_t n_rows, int width, const float *grad, int *workspace,
                                 int *ids, float *rows, int *count) {
    return rows_compact(stream, n_rows, width, grad, nullptr, workspace, ids, rows, count);
}

extern "C" int psvo_rows_compact_flagged(void *stream, int64_t n_rows, int width, const float *grad,
                                         const uint8_t *flags, int *workspace, int *ids, float *rows, int *count) {
    PSVO_REQUIRE(flags != nullptr || n_rows == 0, "rows_compact_flagged: flags required");
    return rows_compact(stream, n_rows, width, grad, flags, workspace, ids, rows, count);
}

extern "C" int psvo_rows_clear(void *stream, int64_t n_list, int width, const int *ids, float *grad, uint8_t *flags) {
    PSVO_REQUIRE(n_list >= 0 && width > 0, "rows_clear: bad sizes");
    PSVO_REQUIRE(n_list == 0 || (ids && grad), "rows_clear: null pointer");
    if (n_list == 0) return PSVO_OK;
    psvo::launch(k_rows_clear, dim3(div_up(n_list * width, 256)), dim3(256), 0, as_stream(stream), n_list,
                       width, ids, grad, flags);
    return check_launch("rows_clear");
}

extern "C" int psvo_rows_mark(void *stream, int64_t n_list, const int *ids, uint8_t *flags) {
    PSVO_REQUIRE(n_list >= 0, "rows_mark: bad size");
    PSVO_REQUIRE(n_list == 0 || (ids && flags), "rows_mark: null pointer");
    if (n_list == 0) return PSVO_OK;
    psvo::launch(k_rows_mark, dim3(div_up(n_list, 256)), dim3(256), 0, as_stream(stream), n_list, ids, flags);
    return check_launch("rows_mark");
}

extern "C" int psvo_rows_flags_from_grad(void *stream, int64_t n_rows, int width, const float *grad, uint8_t *flags) {
    PSVO_REQUIRE(n_rows >= 0 && width > 0, "rows_flags_from_grad: bad sizes");
    PSVO_REQUIRE(n_rows == 0 || (grad && flags), "rows_flags_from_grad: null pointer");
    if (n_rows == 0) return PSVO_OK;
    psvo::launch(k_rows_flags_from_grad, dim3(div_up(n_rows, 256)), dim3(256), 0, as_stream(stream), n_rows,
                       width, grad, flags);
    return check_launch("rows_flags_from_grad");
}

extern "C" int psvo_rows_scatter_add(void *stream, int64_t n_list, int width, const int *ids, const float *rows,
                                     float *grad) {
    PSVO_REQUIRE(n_list >= 0 && width > 0, "rows_scatter_add: bad sizes");
    PSVO_REQUIRE(n_list == 0 || (ids && rows && grad), "rows_scatter_add: null pointer");
    if (n_list == 0) return PSVO_OK;
    psvo::launch(k_rows_scatter_add, dim3(div_up(n_list * width, 256)), dim3(256), 0, as_stream(stream),
                       n_list, width, ids, rows, grad);
    return check_launch("rows_scatter_add");
}
