// The octree as the traversal reads it: one 32-B record per node, siblings
// contiguous, breadth-first.
//
// The reference hands the renderer two AoS rows per node
// (get_centres_and_children, octree.cpp:561-687 / mapping.py:328-347):
// centres f32[N,3] (12 B) and structure i32[N,9] (36 B, 8 child ids + side),
// in creation order.  A node visit of k_intersect_sorted therefore touches
// two unaligned rows in two arrays, and the up-to-8 children a wave pops
// together (one per lane) sit wherever insertion left them: on a map that
// does not fit in L2 (config E: 2.7 M nodes, 131 MB) every lane misses on its
// own lines.  The packed layout:
//
//   rec[i] = { float4 (cx, cy, cz, side as int bits),
//              int4   (reference node id, first child record, child mask, spare) }
//
// (spare: the traversal's start level for the root and the parent record for
// the next 127 records, k_pt_top; 0 elsewhere)
//
// in breadth-first order with a node's existing children at consecutive
// records first + rank(u) (rank = popcount(mask & ((1 << u) − 1))), so a
// wave's sibling candidates are one contiguous 32·k-byte span, and one node
// is two 16-B loads from one 32-B-aligned record.  Same floats and ids as
// the reference arrays, so the slab tests and the emitted ids are unchanged
// (tests/test_gpu_tree_pack.py holds the packed traversal bit-exact to the
// reference-layout one).
//
// Build: level-synchronous BFS from the root (node 0), per level three
// grids — child counts per block, one-block scan of the block sums (→ the
// next level's size, on the device), emit (records + the next level's
// reference ids) — launched for kMaxDepth levels with capacity-sized grids
// whose blocks past the level's size exit (no host read-back).
#include <hip/hip_runtime.h>

#include "psvo_common.h"

namespace psvo {
namespace {

constexpr int kPtBlock = 1024;  // nodes per block (256 threads x 4)
constexpr int kPtThreads = 256;
constexpr int kPtMaxDepth = 17;  // levels (the traversal's 16-level bound + the root)

struct PtWork {
    int *lists[2];  // reference ids of the nodes of the current / next level
    int *counts;    // children per node of the current level
    int *bsum;      // per-block sums → exclusive offsets
    int *meta;      // [level][2] = (first record, size)
};

__device__ __forceinline__ int child_mask(const int *__restrict__ row) {
    int m = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) m |= (row[u] > -1 ? 1 : 0) << u;
    return m;
}

__global__ __launch_bounds__(kPtThreads) void k_pt_count(int level, const int *__restrict__ structure, PtWork w) {
    __shared__ int part[kPtThreads / kWave];
    const int size = w.meta[level * 2 + 1];
    const int i0 = blockIdx.x * kPtBlock;
    if (i0 >= size) return;
    const int *cur = w.lists[level & 1];
    int s = 0;
    for (int i = i0 + threadIdx.x; i < i0 + kPtBlock && i < size; i += kPtThreads) {
        const int c = __popc(child_mask(structure + (int64_t)cur[i] * 9));
        w.counts[i] = c;
        s += c;
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, kWave);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int k = 0; k < kPtThreads / kWave; ++k) t += part[k];
        w.bsum[blockIdx.x] = t;
    }
}

// exclusive scan of the level's block sums (one block); the next level's
// first record and size
__global__ __launch_bounds__(1024) void k_pt_scan(int level, PtWork w) {
    __shared__ int part[1024];
    const int first = w.meta[level * 2 + 0], size = w.meta[level * 2 + 1];
    const int nb = (size + kPtBlock - 1) / kPtBlock;
    const int per = (nb + 1023) / 1024;
    const int b0 = threadIdx.x * per;
    int s = 0;
    for (int i = 0; i < per && b0 + i < nb; ++i) s += w.bsum[b0 + i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const int v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    int run = threadIdx.x > 0 ? part[threadIdx.x - 1] : 0;
    for (int i = 0; i < per && b0 + i < nb; ++i) {
        const int c = w.bsum[b0 + i];
        w.bsum[b0 + i] = run;
        run += c;
    }
    if (threadIdx.x == 1023 && level + 1 < kPtMaxDepth) {
        w.meta[(level + 1) * 2 + 0] = first + size;
        w.meta[(level + 1) * 2 + 1] = size > 0 ? part[1023] : 0;
    }
}

// records of the level's nodes; the next level's reference ids, each node's
// children at its first child's slot onward (ascending u)
__global__ __launch_bounds__(kPtThreads) void k_pt_emit(int level, const float *__restrict__ centres,
                                                        const int *__restrict__ structure, PtWork w,
                                                        PackRec *__restrict__ rec) {
    __shared__ int scan[kPtBlock];
    const int first = w.meta[level * 2 + 0], size = w.meta[level * 2 + 1];
    const int i0 = blockIdx.x * kPtBlock;
    if (i0 >= size) return;
    const int *cur = w.lists[level & 1];
    int *nxt = w.lists[(level + 1) & 1];
    // block-local exclusive scan of the child counts (node order)
    for (int k = threadIdx.x; k < kPtBlock; k += kPtThreads) scan[k] = (i0 + k < size) ? w.counts[i0 + k] : 0;
    __syncthreads();
    for (int off = 1; off < kPtBlock; off <<= 1) {
        int v[kPtBlock / kPtThreads];
#pragma unroll
        for (int q = 0; q < kPtBlock / kPtThreads; ++q) {
            const int k = threadIdx.x + q * kPtThreads;
            v[q] = k >= off ? scan[k - off] : 0;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kPtBlock / kPtThreads; ++q) scan[threadIdx.x + q * kPtThreads] += v[q];
        __syncthreads();
    }
    const int next_first = first + size;
    const int boff = w.bsum[blockIdx.x];
    for (int k = threadIdx.x; k < kPtBlock && i0 + k < size; k += kPtThreads) {
        const int i = i0 + k;
        const int node = cur[i];
        const int *row = structure + (int64_t)node * 9;
        const int m = child_mask(row);
        const int excl = boff + scan[k] - __popc(m);  // this node's first child, level-relative
        rec[first + i].c = make_float4(centres[(int64_t)node * 3 + 0], centres[(int64_t)node * 3 + 1],
                                       centres[(int64_t)node * 3 + 2], __int_as_float(row[8]));
        rec[first + i].i = make_int4(node, m ? next_first + excl : -1, m, 0);
        int g = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (row[u] > -1) nxt[excl + g++] = row[u];
    }
}

// The traversal's start level (svo_query.hip, top_start): the deepest level
// m >= 2 such that the records above it — [0, meta[m].first), breadth-first —
// number at most kTopMax and hold no leaf (side 1).  The root's spare word
// gets that count | m << 16 (0: start at the root); each other record among
// the first kTopMax gets its parent record.
constexpr int kTopMax = kPackTopMax;

__global__ __launch_bounds__(512) void k_pt_top(PtWork w, PackRec *__restrict__ rec) {
    __shared__ int leaf_at;
    const int total = w.meta[(kPtMaxDepth - 1) * 2 + 0] + w.meta[(kPtMaxDepth - 1) * 2 + 1];
    if (threadIdx.x == 0) leaf_at = kTopMax;
    __syncthreads();
    const int j = threadIdx.x;
    if (j < total && j < kTopMax) {
        if (__float_as_int(rec[j].c.w) == 1) atomicMin(&leaf_at, j);
        const int4 ri = rec[j].i;  // the parent link of each child among the first kTopMax records
        if (ri.y >= 0)
            for (int k = 0; k < __popc(ri.z) && ri.y + k < kTopMax; ++k) rec[ri.y + k].i.w = j;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int word = 0;
        for (int m = 2; m < kPtMaxDepth; ++m) {
            const int n = w.meta[m * 2 + 0];  // records of the levels above m
            if (n > kTopMax || n > leaf_at || w.meta[(m - 1) * 2 + 1] == 0) break;
            word = n | m << 16;
        }
        rec[0].i.w = word;
    }
}

__global__ void k_pt_init(PtWork w) {
    w.lists[0][0] = 0;  // the root is node 0 (the traversal's first candidate)
    w.meta[0] = 0;
    w.meta[1] = 1;
}

}  // namespace
}  // namespace psvo

using namespace psvo;

extern "C" int64_t psvo_pack_tree_workspace_ints(int64_t n_nodes) {
    const int64_t nb = (n_nodes + kPtBlock - 1) / kPtBlock;
    return 3 * n_nodes + nb + 2 * kPtMaxDepth + 16;
}

extern "C" int psvo_pack_tree(void *stream, int64_t n_nodes, const float *centres, const int *structure,
                              int *workspace, void *packed) {
    PSVO_REQUIRE(n_nodes >= 1 && n_nodes <= 0x7fffffff, "pack_tree: bad node count %lld", (long long)n_nodes);
    PSVO_REQUIRE(centres && structure && workspace && packed, "pack_tree: null pointer");
    PSVO_REQUIRE(((uintptr_t)packed & 15) == 0, "pack_tree: packed records must be 16-B aligned");
    hipStream_t st = as_stream(stream);
    PtWork w;
    int *p = workspace;
    w.lists[0] = p; p += n_nodes;
    w.lists[1] = p; p += n_nodes;
    w.counts = p; p += n_nodes;
    w.bsum = p; p += (n_nodes + kPtBlock - 1) / kPtBlock;
    w.meta = p;
    PackRec *rec = static_cast<PackRec *>(packed);
    if (hipMemsetAsync(w.meta, 0, sizeof(int) * 2 * kPtMaxDepth, st) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "pack_tree: memset failed");
    psvo::launch(k_pt_init, dim3(1), dim3(1), 0, st, w);
    const int nb = (int)((n_nodes + kPtBlock - 1) / kPtBlock);
    for (int level = 0; level < kPtMaxDepth; ++level) {
        psvo::launch(k_pt_count, dim3(nb), dim3(kPtThreads), 0, st, level, structure, w);
        psvo::launch(k_pt_scan, dim3(1), dim3(1024), 0, st, level, w);
        psvo::launch(k_pt_emit, dim3(nb), dim3(kPtThreads), 0, st, level, centres, structure, w, rec);
    }
    psvo::launch(k_pt_top, dim3(1), dim3(512), 0, st, w, rec);
    return check_launch("pack_tree");
}
