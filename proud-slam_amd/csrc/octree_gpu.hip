// Sparse voxel octree builder on the device: the same
// tree as octree.cpp / the reference's Octree::insert (octree.cpp:104-294) —
// node ids in CREATION ORDER, root 0, every voxel inserting itself as a
// SURFACE leaf and its 7 +1 corner neighbours as FEATURE leaves — and the
// export of get_centres_and_children (octree.cpp:561-687) plus the renderer's
// map_states arrays (mapping.py:300-406), without the per-frame CPU walk and
// host→device copy.
//
// Sequential semantics, parallel construction.  Walk w = 8·i + j (voxel i,
// corner j) visits depths d = 1..D; the sequential insert creates node
// (d, path prefix) at the FIRST walk (in w order) whose path reaches it, in
// the order (w, d).  So one insert call is:
//   1. every (w, d) hashes its node key into a device hash table (open
//      addressing, 64-bit CAS) and atomicMin's its walk index into the slot;
//      walks with j = 0 flag their leaf SURFACE;
//   2. (w, d) is a creator iff its slot has no node yet and holds min-walk w;
//   3. an exclusive scan of the creator flags in (w, d) order is exactly the
//      creation order: id = count + rank;
//   4. creators write their node (code of the creating walk, side, type) and
//      link themselves into their parent's child slot; SURFACE flags promote
//      leaves (FEATURE → SURFACE, octree.cpp:247-248).
// The table persists across inserts (existing nodes are never creators), so
// incremental inserts extend the tree exactly like repeated CPU inserts.
// Node arrays (code, side, type, child[8]) are struct-of-arrays in HBM;
// capacity doubles (with a rehash) when a batch could overflow it.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>

#include "psvo_common.h"

namespace psvo {
namespace {

constexpr int kDtMaxBits = 21;  // utils.h:12
constexpr int8_t kDtNonLeaf = -1, kDtSurface = 0, kDtFeature = 1;
constexpr uint64_t kEmptyKey = ~0ull;

__host__ __device__ __forceinline__ uint64_t dt_spread3(uint64_t v) {
    uint64_t x = v & 0x1fffffull;
    x = (x | x << 32) & 0x1f00000000ffffull;
    x = (x | x << 16) & 0x1f0000ff0000ffull;
    x = (x | x << 8) & 0x100f00f00f00f00full;
    x = (x | x << 4) & 0x10c30c30c30c30c3ull;
    x = (x | x << 2) & 0x1249249249249249ull;
    return x;
}
__device__ __forceinline__ uint64_t dt_squeeze3(uint64_t v) {
    uint64_t x = v & 0x1249249249249249ull;
    x = (x | x >> 2) & 0x10c30c30c30c30c3ull;
    x = (x | x >> 4) & 0x100f00f00f00f00full;
    x = (x | x >> 8) & 0x1f0000ff0000ffull;
    x = (x | x >> 16) & 0x1f00000000ffffull;
    x = (x | x >> 32) & 0x1fffffull;
    return x;
}
__device__ __forceinline__ uint64_t dt_prefix_mask(int i) {  // utils.h:56-77
    return i >= 20 ? 0x7fffffffffffffffull : ~((1ull << (60 - 3 * i)) - 1) & 0x7fffffffffffffffull;
}
__device__ __forceinline__ uint64_t dt_morton(int x, int y, int z) {  // utils.h (code of a corner)
    return (dt_spread3((uint64_t)(int64_t)x) | dt_spread3((uint64_t)(int64_t)y) << 1 |
            dt_spread3((uint64_t)(int64_t)z) << 2) &
           dt_prefix_mask(kDtMaxBits - 1);
}
// identity of the node at depth d on the path of (x, y, z): the path bits
// below size/2 (the walk ignores higher bits, octree.cpp:157-160) and d
__device__ __forceinline__ uint64_t dt_key(int x, int y, int z, int d, int D) {
    const int sh = D - d;
    const uint64_t m = (d >= 21) ? 0x1fffffull : ((1ull << d) - 1);
    const uint64_t xs = ((uint64_t)(uint32_t)x >> sh) & m, ys = ((uint64_t)(uint32_t)y >> sh) & m,
                   zs = ((uint64_t)(uint32_t)z >> sh) & m;
    return ((dt_spread3(xs) | dt_spread3(ys) << 1 | dt_spread3(zs) << 2) << 5) | (uint64_t)d;
}
__device__ __forceinline__ uint64_t dt_hash(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

struct DtTable {
    unsigned long long *key;
    unsigned int *minw;
    int *id;
    unsigned int *flags;
    uint64_t mask;  // capacity - 1 (power of two)
};

constexpr int kDtMaxProbe = 256;
constexpr uint64_t kDtNoSlot = ~0ull;

// slot of `k`, inserting it if absent; kDtNoSlot if the probe run exceeds
// kDtMaxProbe (the host grows the table and redoes the batch)
__device__ __forceinline__ uint64_t dt_insert(const DtTable &t, uint64_t k) {
    uint64_t s = dt_hash(k) & t.mask;
    for (int probe = 0; probe < kDtMaxProbe; ++probe) {
        const unsigned long long cur = t.key[s];
        if (cur == k) return s;
        if (cur == kEmptyKey) {
            const unsigned long long prev = atomicCAS(t.key + s, kEmptyKey, (unsigned long long)k);
            if (prev == kEmptyKey || prev == k) return s;
        }
        s = (s + 1) & t.mask;
    }
    return kDtNoSlot;
}
__device__ __forceinline__ int64_t dt_find(const DtTable &t, uint64_t k) {
    uint64_t s = dt_hash(k) & t.mask;
    for (int probe = 0; probe < kDtMaxProbe; ++probe) {
        const unsigned long long cur = t.key[s];
        if (cur == k) return (int64_t)s;
        if (cur == kEmptyKey) return -1;
        s = (s + 1) & t.mask;
    }
    return -1;
}

__constant__ int kDtIncX[8] = {0, 0, 0, 0, 1, 1, 1, 1};
__constant__ int kDtIncY[8] = {0, 0, 1, 1, 0, 0, 1, 1};
__constant__ int kDtIncZ[8] = {0, 1, 0, 1, 0, 1, 0, 1};

struct DtNodes {
    unsigned long long *code;
    int *side;
    int8_t *type;
    int *child;  // [cap][8]
};

__global__ void k_dt_fill(DtTable t, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > t.mask) return;
    t.key[i] = kEmptyKey;
    t.minw[i] = 0xffffffffu;
    t.id[i] = -1;
    t.flags[i] = 0;
    (void)n;
}
__global__ void k_dt_fill_child(int *child, int64_t from, int64_t to) {
    const int64_t i = from + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < to) child[i] = -1;
}

// (re)insert existing nodes [0, n) into a fresh table: key from the stored path
// (code of a node = prefix of its creating walk; the path bits are recovered
// from the code's coordinates)
__global__ void k_dt_rehash(DtTable t, DtNodes nd, int64_t n, int D) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t c = nd.code[i];
    const int x = (int)dt_squeeze3(c), y = (int)dt_squeeze3(c >> 1), z = (int)dt_squeeze3(c >> 2);
    const int d = D - (31 - __clz(nd.side[i]));  // side = size >> d
    const uint64_t s = dt_insert(t, dt_key(x, y, z, d, D));
    if (s == kDtNoSlot) return;  // cannot happen below load 1/2 (the table holds >= 2 slots per node)
    t.id[s] = (int)i;
    if (nd.type[i] == kDtSurface) t.flags[s] = 1u;
}

// 1. keys + min walk + SURFACE flags
__global__ void k_dt_walk(DtTable t, const int *__restrict__ vox, int64_t n_walks, int D, unsigned w_base,
                          int *__restrict__ overflow) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_walks * D) return;
    const int64_t w = e / D;
    const int d = (int)(e - w * D) + 1;
    const int64_t i = w >> 3;
    const int j = (int)(w & 7);
    const int x = vox[3 * i] + kDtIncX[j], y = vox[3 * i + 1] + kDtIncY[j], z = vox[3 * i + 2] + kDtIncZ[j];
    const uint64_t s = dt_insert(t, dt_key(x, y, z, d, D));
    if (s == kDtNoSlot) {
        *overflow = 1;
        return;
    }
    // the shallow keys are shared by nearly every walk: a plain read first
    // keeps the same-address atomics (which serialise) to the few that can win
    const unsigned wv = w_base + (unsigned)w;
    if (wv < __atomic_load_n(t.minw + s, __ATOMIC_RELAXED)) atomicMin(t.minw + s, wv);
    if (d == D && j == 0 && !(__atomic_load_n(t.flags + s, __ATOMIC_RELAXED) & 1u)) atomicOr(t.flags + s, 1u);
}

// 2. creator flags (w, d order)
__global__ void k_dt_flag(DtTable t, const int *__restrict__ vox, int64_t n_walks, int D, unsigned w_base,
                          int *__restrict__ flag) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_walks * D) return;
    const int64_t w = e / D;
    const int d = (int)(e - w * D) + 1;
    const int64_t i = w >> 3;
    const int j = (int)(w & 7);
    const int x = vox[3 * i] + kDtIncX[j], y = vox[3 * i + 1] + kDtIncY[j], z = vox[3 * i + 2] + kDtIncZ[j];
    const int64_t s = dt_find(t, dt_key(x, y, z, d, D));
    flag[e] = (s >= 0 && t.id[s] < 0 && t.minw[s] == w_base + (unsigned)w) ? 1 : 0;
}

// block-local exclusive scan + block totals; totals scanned by one block; offsets added
__global__ __launch_bounds__(1024) void k_dt_scan_local(const int *__restrict__ in, int64_t n, int *__restrict__ out,
                                                        int *__restrict__ totals) {
    __shared__ int ws[16];
    const int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x;
    const int v = i < n ? in[i] : 0;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int inc = v;
#pragma unroll
    for (int sh = 1; sh < 64; sh <<= 1) {
        const int t = __shfl_up(inc, sh, 64);
        if (lane >= sh) inc += t;
    }
    if (lane == 63) ws[w] = inc;
    __syncthreads();
    if (w == 0) {
        int s = lane < 16 ? ws[lane] : 0;
#pragma unroll
        for (int sh = 1; sh < 16; sh <<= 1) {
            const int t = __shfl_up(s, sh, 64);
            if (lane >= sh) s += t;
        }
        if (lane < 16) ws[lane] = s;
    }
    __syncthreads();
    const int excl = (w > 0 ? ws[w - 1] : 0) + inc - v;
    if (i < n) out[i] = excl;
    if (threadIdx.x == 1023) totals[blockIdx.x] = ws[15];
}
__global__ __launch_bounds__(1024) void k_dt_scan_totals(int *__restrict__ totals, int64_t nb, int *__restrict__ sum) {
    __shared__ int part[1024];
    const int64_t per = (nb + 1023) / 1024;
    const int64_t b0 = threadIdx.x * per, b1 = b0 + per < nb ? b0 + per : nb;
    int local = 0;
    for (int64_t b = b0; b < b1; ++b) local += totals[b];
    part[threadIdx.x] = local;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const int v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    int run = part[threadIdx.x] - local;
    for (int64_t b = b0; b < b1; ++b) {
        const int t = totals[b];
        totals[b] = run;
        run += t;
    }
    if (threadIdx.x == 1023) *sum = part[1023];
}
__global__ void k_dt_scan_add(int *__restrict__ out, int64_t n, const int *__restrict__ totals) {
    const int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x;
    if (i < n) out[i] += totals[blockIdx.x];
}

// 4a. creators: ids and node rows
__global__ void k_dt_create(DtTable t, DtNodes nd, const int *__restrict__ vox, int64_t n_walks, int D, int shift,
                            int size, const int *__restrict__ flag, const int *__restrict__ rank, int64_t count) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_walks * D || !flag[e]) return;
    const int64_t w = e / D;
    const int d = (int)(e - w * D) + 1;
    const int64_t i = w >> 3;
    const int j = (int)(w & 7);
    const int x = vox[3 * i] + kDtIncX[j], y = vox[3 * i + 1] + kDtIncY[j], z = vox[3 * i + 2] + kDtIncZ[j];
    const int64_t s = dt_find(t, dt_key(x, y, z, d, D));
    const int id = (int)(count + rank[e]);
    t.id[s] = id;
    nd.code[id] = dt_morton(x, y, z) & dt_prefix_mask(d + shift);
    nd.side[id] = size >> d;
    nd.type[id] = d == D ? kDtFeature : kDtNonLeaf;
}

// 4b. links (every id assigned) and SURFACE promotion
__global__ void k_dt_link(DtTable t, DtNodes nd, const int *__restrict__ vox, int64_t n_walks, int D, int size,
                          const int *__restrict__ flag) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_walks * D) return;
    const int64_t w = e / D;
    const int d = (int)(e - w * D) + 1;
    const int64_t i = w >> 3;
    const int j = (int)(w & 7);
    const int x = vox[3 * i] + kDtIncX[j], y = vox[3 * i + 1] + kDtIncY[j], z = vox[3 * i + 2] + kDtIncZ[j];
    if (flag[e]) {
        const int64_t s = dt_find(t, dt_key(x, y, z, d, D));
        const int parent = d == 1 ? 0 : t.id[dt_find(t, dt_key(x, y, z, d - 1, D))];
        const int edge = size >> d;
        const int cid = ((x & edge) > 0) + 2 * ((y & edge) > 0) + 4 * ((z & edge) > 0);
        nd.child[(int64_t)parent * 8 + cid] = t.id[s];
    }
    if (d == D && j == 0) nd.type[t.id[dt_find(t, dt_key(x, y, z, d, D))]] = kDtSurface;
}

// get_centres_and_children rows + the render arrays (mapping.py:328-372)
__global__ void k_dt_export(DtTable t, DtNodes nd, int64_t n, int D, float voxel_size, float *__restrict__ voxels,
                            float *__restrict__ children, int *__restrict__ features, float *__restrict__ centres,
                            int *__restrict__ structure) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int8_t ty = nd.type[i];
    const uint64_t c = nd.code[i];
    const int x = (int)dt_squeeze3(c), y = (int)dt_squeeze3(c >> 1), z = (int)dt_squeeze3(c >> 2);
    const int side = nd.side[i];
    const bool live = ty != kDtFeature;  // FEATURE rows are never reached by the reference BFS
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (live) {
        v[0] = (float)x;
        v[1] = (float)y;
        v[2] = (float)z;
        v[3] = (float)side;
    }
    if (voxels) {
#pragma unroll
        for (int k = 0; k < 4; ++k) voxels[i * 4 + k] = v[k];
    }
    if (centres) {  // (xyz + side/2) · voxel, as mapping.py:328 in fp32
#pragma unroll
        for (int k = 0; k < 3; ++k) centres[i * 3 + k] = __fmul_rn(__fadd_rn(v[k], __fmul_rn(v[3], 0.5f)), voxel_size);
    }
    int ch[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int cc = live ? nd.child[i * 8 + k] : -1;
        ch[k] = (cc >= 0 && nd.type[cc] != kDtFeature) ? cc : -1;
        if (children) children[i * 8 + k] = (float)ch[k];
        if (structure) structure[i * 9 + k] = ch[k];
    }
    if (structure) structure[i * 9 + 8] = (int)v[3];
    if (features) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            int f = -1;
            if (ty == kDtSurface) {  // find(corner) (octree.cpp:419-439): the leaf at the corner's path
                const int64_t s = dt_find(t, dt_key(x + kDtIncX[k], y + kDtIncY[k], z + kDtIncZ[k], D, D));
                f = s >= 0 ? t.id[s] : -1;
            }
            features[i * 8 + k] = f;
        }
    }
}

__global__ void k_dt_count_type(const int8_t *__restrict__ type, int64_t n, int8_t want, int *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int v = (i < n && type[i] == want) ? 1 : 0;
#pragma unroll
    for (int sh = 32; sh > 0; sh >>= 1) v += __shfl_xor(v, sh, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(out, v);
}

__global__ void k_dt_probe(DtTable t, const int *__restrict__ vox, int64_t n, int D, int corners, int *__restrict__ hit) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n * corners) return;
    const int64_t i = e / corners;
    const int j = (int)(e - i * corners);
    const int64_t s = dt_find(t, dt_key(vox[3 * i] + kDtIncX[j], vox[3 * i + 1] + kDtIncY[j], vox[3 * i + 2] + kDtIncZ[j], D, D));
    hit[e] = (s >= 0 && t.id[s] >= 0) ? 1 : 0;
}

}  // namespace
}  // namespace psvo

using namespace psvo;

struct psvo_dtree {
    int size = 0, D = 0, shift = 0;
    int64_t count = 0, cap = 0;
    unsigned w_next = 0;  // walk counter across inserts (min-walk order stays global)
    DtTable t{};
    DtNodes nd{};
    int *scratch = nullptr;  // flags | ranks | totals | sum | overflow
    int64_t scratch_n = 0;
};

namespace {

int dt_alloc_nodes(psvo_dtree *tr, int64_t cap, hipStream_t st) {
    DtNodes n{};
    if (hipMalloc(&n.code, cap * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&n.side, cap * sizeof(int)) != hipSuccess || hipMalloc(&n.type, cap * sizeof(int8_t)) != hipSuccess ||
        hipMalloc(&n.child, cap * 8 * sizeof(int)) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "dtree: out of device memory (%lld nodes)", (long long)cap);
    if (tr->count > 0) {
        (void)hipMemcpyAsync(n.code, tr->nd.code, tr->count * sizeof(unsigned long long), hipMemcpyDeviceToDevice, st);
        (void)hipMemcpyAsync(n.side, tr->nd.side, tr->count * sizeof(int), hipMemcpyDeviceToDevice, st);
        (void)hipMemcpyAsync(n.type, tr->nd.type, tr->count * sizeof(int8_t), hipMemcpyDeviceToDevice, st);
        (void)hipMemcpyAsync(n.child, tr->nd.child, tr->count * 8 * sizeof(int), hipMemcpyDeviceToDevice, st);
    }
    psvo::launch(k_dt_fill_child, dim3(div_up((cap - tr->count) * 8, 256)), dim3(256), 0, st, n.child,
                       tr->count * 8, cap * 8);
    if (tr->cap > 0) {
        (void)hipStreamSynchronize(st);
        (void)hipFree(tr->nd.code);
        (void)hipFree(tr->nd.side);
        (void)hipFree(tr->nd.type);
        (void)hipFree(tr->nd.child);
    }
    tr->nd = n;
    tr->cap = cap;
    return PSVO_OK;
}

int dt_alloc_table(psvo_dtree *tr, hipStream_t st, uint64_t min_slots) {
    uint64_t slots = 1024;
    while (slots < min_slots || slots < (uint64_t)tr->count * 2) slots <<= 1;
    DtTable t{};
    if (hipMalloc(&t.key, slots * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&t.minw, slots * sizeof(unsigned)) != hipSuccess || hipMalloc(&t.id, slots * sizeof(int)) != hipSuccess ||
        hipMalloc(&t.flags, slots * sizeof(unsigned)) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "dtree: out of device memory (hash table)");
    t.mask = slots - 1;
    psvo::launch(k_dt_fill, dim3(div_up((int64_t)slots, 256)), dim3(256), 0, st, t, slots);
    if (tr->count > 0)
        psvo::launch(k_dt_rehash, dim3(div_up(tr->count, 256)), dim3(256), 0, st, t, tr->nd, tr->count, tr->D);
    if (tr->t.key) {
        (void)hipStreamSynchronize(st);
        (void)hipFree(tr->t.key);
        (void)hipFree(tr->t.minw);
        (void)hipFree(tr->t.id);
        (void)hipFree(tr->t.flags);
    }
    tr->t = t;
    return PSVO_OK;
}

}  // namespace

extern "C" void *psvo_dtree_new(void *stream, int grid_dim, int64_t capacity) {
    if (grid_dim < 2 || (grid_dim & (grid_dim - 1)) || grid_dim > (1 << 16)) {
        set_error(PSVO_E_INVALID, "dtree_new: grid_dim must be a power of two in [2, 65536]");
        return nullptr;
    }
    hipStream_t st = as_stream(stream);
    psvo_dtree *tr = new psvo_dtree;
    tr->size = grid_dim;
    int D = 0;
    while ((1 << D) < grid_dim) ++D;
    tr->D = D;
    tr->shift = kDtMaxBits - D - 1;
    const int64_t cap0 = capacity > 1024 ? capacity : 1024;
    if (dt_alloc_nodes(tr, cap0, st) != PSVO_OK || dt_alloc_table(tr, st, (uint64_t)cap0 * 2) != PSVO_OK) {
        delete tr;
        return nullptr;
    }
    // root: id 0, code 0, side = grid_dim, key (d = 0)
    const unsigned long long zero = 0;
    const int side = grid_dim;
    const int8_t nl = kDtNonLeaf;
    (void)hipMemcpyAsync(tr->nd.code, &zero, sizeof(zero), hipMemcpyHostToDevice, st);
    (void)hipMemcpyAsync(tr->nd.side, &side, sizeof(side), hipMemcpyHostToDevice, st);
    (void)hipMemcpyAsync(tr->nd.type, &nl, sizeof(nl), hipMemcpyHostToDevice, st);
    tr->count = 1;
    psvo::launch(k_dt_rehash, dim3(1), dim3(64), 0, st, tr->t, tr->nd, (int64_t)1, tr->D);
    if (hipStreamSynchronize(st) != hipSuccess) {
        set_error(PSVO_E_LAUNCH, "dtree_new: device init failed");
        delete tr;
        return nullptr;
    }
    return tr;
}

extern "C" void psvo_dtree_free(void *tree) {
    psvo_dtree *tr = static_cast<psvo_dtree *>(tree);
    if (!tr) return;
    (void)hipDeviceSynchronize();
    (void)hipFree(tr->nd.code);
    (void)hipFree(tr->nd.side);
    (void)hipFree(tr->nd.type);
    (void)hipFree(tr->nd.child);
    (void)hipFree(tr->t.key);
    (void)hipFree(tr->t.minw);
    (void)hipFree(tr->t.id);
    (void)hipFree(tr->t.flags);
    (void)hipFree(tr->scratch);
    delete tr;
}

extern "C" int psvo_dtree_insert(void *tree, void *stream, const int *vox, int64_t n) {
    psvo_dtree *tr = static_cast<psvo_dtree *>(tree);
    PSVO_REQUIRE(tr != nullptr && n >= 0 && (n == 0 || vox != nullptr), "dtree_insert: bad arguments");
    if (n == 0) return PSVO_OK;
    hipStream_t st = as_stream(stream);
    const int64_t n_walks = n * 8, ne = n_walks * tr->D;
    PSVO_REQUIRE(ne < (int64_t)1 << 31 && (uint64_t)tr->w_next + (uint64_t)n_walks < 0xffffffffull,
                 "dtree_insert: batch too large (%lld voxels)", (long long)n);
    const int64_t nb = div_up(ne, 1024);
    const int64_t need = 2 * ne + nb + 2;
    if (need > tr->scratch_n) {
        (void)hipStreamSynchronize(st);
        (void)hipFree(tr->scratch);
        if (hipMalloc(&tr->scratch, need * sizeof(int)) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "dtree_insert: out of device memory");
        tr->scratch_n = need;
    }
    int *flag = tr->scratch, *rank = flag + ne, *totals = rank + ne, *sum = totals + nb, *overflow = sum + 1;
    const dim3 g(div_up(ne, 256)), b(256);
    // table: about 2.4 new nodes per voxel on surface scans; keep load <= 1/2
    // for that and grow (rehash from the node arrays, batch redone) if a
    // probe run still overflows
    uint64_t want = 2 * (uint64_t)(tr->count + 3 * n);
    for (int attempt = 0;; ++attempt) {
        if (want > tr->t.mask + 1) {
            int rc = dt_alloc_table(tr, st, want);
            if (rc) return rc;
        }
        int ov = 0;
        (void)hipMemsetAsync(overflow, 0, sizeof(int), st);
        psvo::launch(k_dt_walk, g, b, 0, st, tr->t, vox, n_walks, tr->D, tr->w_next, overflow);
        if (hipMemcpyAsync(&ov, overflow, sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "dtree_insert: walk failed (%s)", hipGetErrorString(hipGetLastError()));
        if (!ov) break;
        if (attempt >= 6) return set_error(PSVO_E_OVERFLOW, "dtree_insert: hash table overflow");
        want = 4 * (tr->t.mask + 1);
        int rc = dt_alloc_table(tr, st, want);
        if (rc) return rc;
    }
    psvo::launch(k_dt_flag, g, b, 0, st, tr->t, vox, n_walks, tr->D, tr->w_next, flag);
    psvo::launch(k_dt_scan_local, dim3(nb), dim3(1024), 0, st, flag, ne, rank, totals);
    psvo::launch(k_dt_scan_totals, dim3(1), dim3(1024), 0, st, totals, nb, sum);
    psvo::launch(k_dt_scan_add, dim3(nb), dim3(1024), 0, st, rank, ne, totals);
    int created = 0;
    if (hipMemcpyAsync(&created, sum, sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "dtree_insert: scan failed (%s)", hipGetErrorString(hipGetLastError()));
    if (tr->count + created > tr->cap) {  // node arrays: exactly what this batch creates
        int64_t cap = tr->cap;
        while (cap < tr->count + created) cap *= 2;
        int rc = dt_alloc_nodes(tr, cap, st);
        if (rc) return rc;
    }
    psvo::launch(k_dt_create, g, b, 0, st, tr->t, tr->nd, vox, n_walks, tr->D, tr->shift, tr->size, flag, rank,
                       tr->count);
    psvo::launch(k_dt_link, g, b, 0, st, tr->t, tr->nd, vox, n_walks, tr->D, tr->size, flag);
    tr->count += created;
    tr->w_next += (unsigned)n_walks;
    return check_launch("dtree_insert");
}

extern "C" int64_t psvo_dtree_count(void *tree) {
    const psvo_dtree *tr = static_cast<const psvo_dtree *>(tree);
    return tr ? tr->count : -1;
}

extern "C" int64_t psvo_dtree_count_leaves(void *tree, void *stream) {
    psvo_dtree *tr = static_cast<psvo_dtree *>(tree);
    if (!tr) return -1;
    hipStream_t st = as_stream(stream);
    int *out = tr->scratch;
    if (!out) {
        if (hipMalloc(&tr->scratch, 64 * sizeof(int)) != hipSuccess) return -1;
        tr->scratch_n = 64;
        out = tr->scratch;
    }
    (void)hipMemsetAsync(out, 0, sizeof(int), st);
    psvo::launch(k_dt_count_type, dim3(div_up(tr->count, 256)), dim3(256), 0, st, tr->nd.type, tr->count,
                       kDtSurface, out);
    int v = 0;
    (void)hipMemcpyAsync(&v, out, sizeof(int), hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) return -1;
    return v;
}

extern "C" int psvo_dtree_export(void *tree, void *stream, float voxel_size, float *voxels, float *children,
                                 int *features, float *centres, int *structure) {
    psvo_dtree *tr = static_cast<psvo_dtree *>(tree);
    PSVO_REQUIRE(tr != nullptr, "dtree_export: null tree");
    psvo::launch(k_dt_export, dim3(div_up(tr->count, 256)), dim3(256), 0, as_stream(stream), tr->t, tr->nd,
                       tr->count, tr->D, voxel_size, voxels, children, features, centres, structure);
    return check_launch("dtree_export");
}

extern "C" int psvo_dtree_probe(void *tree, void *stream, const int *vox, int64_t n, int corners, int *hit) {
    psvo_dtree *tr = static_cast<psvo_dtree *>(tree);
    PSVO_REQUIRE(tr != nullptr && n >= 0 && (corners == 1 || corners == 8), "dtree_probe: bad arguments");
    if (n == 0) return PSVO_OK;
    psvo::launch(k_dt_probe, dim3(div_up(n * corners, 256)), dim3(256), 0, as_stream(stream), tr->t, vox, n,
                       tr->D, corners, hit);
    return check_launch("dtree_probe");
}
