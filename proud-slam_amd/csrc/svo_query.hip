// Ray / sparse-voxel-octree query on gfx950: DFS intersection, stable
// depth sort, hit-ray ranking, inverse-CDF sampling and sample compaction.
//
// Reference behaviour restated (DARYL-GWZ/Proud-SLAM):
//   intersect_gpu.cu:75-140   slab AABB test
//   intersect_gpu.cu:191-270  DFS from node 0, children popped 7→0, ≤ n_max leaf hits
//   voxel_helpers.py:557-595  sort by t_in, max_distance trim, P = max valid hits
//   voxel_helpers.py:288-374  sampler host wrapper: G = 200 blocks × K' slots, 800-slot chunks
//   sample_gpu.cu:133-239     inverse-CDF kernel incl. its layout-dependent trailing segment
//   voxel_helpers.py:637-663  probs / steps, clamp + MAX_DEPTH fill
//   render_helpers.py:390-460 ray and sample compaction
//
// MI355X design: one lane per ray (rays are independent and divergent); the
// DFS keeps a per-level (node, remaining-children bitmask) stack and the
// ≤50-entry hit list in LDS, laid out [slot][lane] so the 64 lanes of a wave
// hit 64 distinct banks.  Per-launch statistics (P, R_hit, max steps, S_max,
// M) are wave-reduced and published with one atomic per wave, so the host
// reads them back once instead of the reference's sequence of host syncs.
//
// Arithmetic: traversal and sampler are compiled with FP contraction off and
// IEEE division so hit indices and sample depths reproduce the CPU oracle
// bit for bit (the reference CUDA uses __fdividef and nvcc's default FMA
// contraction; see DESIGN.md "parity").
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include "psvo_common.h"
#include "lookback.h"

namespace psvo {
namespace {

constexpr int kLevels = 16;  // octree depth <= 15 (grid_dim <= 32768)

__device__ __forceinline__ bool ray_aabb(const float o[3], const float inv[3], float cx, float cy, float cz,
                                         float half, float &t_lo, float &t_hi) {
    float lo_all = 0.0f, hi_all = 100000.0f;
    const float c[3] = {cx, cy, cz};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        float lo = (c[a] - half - o[a]) * inv[a];
        float hi = (c[a] + half - o[a]) * inv[a];
        if (hi < lo) {
            const float tmp = lo;
            lo = hi;
            hi = tmp;
        }
        if (hi < lo_all) return false;
        if (lo > hi_all) return false;
        lo_all = (lo > lo_all) ? lo : lo_all;
        hi_all = (hi < hi_all) ? hi : hi_all;
        if (lo_all > hi_all) return false;
    }
    t_lo = lo_all;
    t_hi = hi_all;
    return true;
}

// ray_aabb without the early exits: the same comparisons on the same values
// in the same order (NaNs included), the verdict accumulated instead of
// returned.  The traversal's node record is then consumed in one basic block,
// so the compiler cannot sink the y / z loads behind the x test (a second
// dependent memory round trip per round); t_lo / t_hi are set only on a hit.
__device__ __forceinline__ bool ray_aabb_nb(const float o[3], const float inv[3], float cx, float cy, float cz,
                                            float half, float &t_lo, float &t_hi) {
    float lo_all = 0.0f, hi_all = 100000.0f;
    bool miss = false;
    const float c[3] = {cx, cy, cz};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        float lo = (c[a] - half - o[a]) * inv[a];
        float hi = (c[a] + half - o[a]) * inv[a];
        const bool sw = hi < lo;
        const float l2 = sw ? hi : lo, h2 = sw ? lo : hi;
        miss = miss | (h2 < lo_all) | (l2 > hi_all);
        lo_all = (l2 > lo_all) ? l2 : lo_all;
        hi_all = (h2 < hi_all) ? h2 : hi_all;
        miss = miss | (lo_all > hi_all);
    }
    if (!miss) {
        t_lo = lo_all;
        t_hi = hi_all;
    }
    return !miss;
}

__device__ __forceinline__ int child_mask(const int *__restrict__ children, int node) {
    const int *row = children + (int64_t)node * 9;
    int m = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) m |= (row[u] > -1) ? (1 << u) : 0;
    return m;
}

// DFS of one ray over the flattened octree, emitting ≤ n_max leaf hits in
// the reference order into the LDS-resident list (stride kWave).
// Returns the number of AABB tests; *cnt the number of hits; *overflow if
// the level stack would exceed kLevels.
template <int STRIDE = kWave>
__device__ int dfs_ray(const float o[3], const float d[3], const float *__restrict__ points,
                       const int *__restrict__ children, float half_voxel, int n_max, int *l_node, int *l_mask,
                       int *h_idx, float *h_t0, float *h_t1, int *cnt_out, bool *overflow) {
    float inv[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) inv[a] = __fdiv_rn(1.0f, d[a]);
    int cnt = 0, visits = 0;
    int lvl = -1;
    {
        float t0, t1;
        const int side = children[8];
        ++visits;
        if (ray_aabb(o, inv, points[0], points[1], points[2], half_voxel * (float)side, t0, t1)) {
            if (side == 1) {
                h_idx[0] = 0;
                h_t0[0] = t0;
                h_t1[0] = t1;
                cnt = 1;
            } else {
                lvl = 0;
                l_node[0] = 0;
                l_mask[0] = child_mask(children, 0);
            }
        }
    }
    while (lvl >= 0 && cnt < n_max) {
        int m = l_mask[lvl * STRIDE];
        if (m == 0) {
            --lvl;
            continue;
        }
        const int u = 31 - __clz(m);
        l_mask[lvl * STRIDE] = m & ~(1 << u);
        const int k = children[(int64_t)l_node[lvl * STRIDE] * 9 + u];
        const float *pc = points + (int64_t)k * 3;
        const int side = children[(int64_t)k * 9 + 8];
        float t0, t1;
        ++visits;
        if (!ray_aabb(o, inv, pc[0], pc[1], pc[2], half_voxel * (float)side, t0, t1)) continue;
        if (side == 1) {
            h_idx[cnt * STRIDE] = k;
            h_t0[cnt * STRIDE] = t0;
            h_t1[cnt * STRIDE] = t1;
            ++cnt;
            continue;
        }
        if (lvl + 1 >= kLevels) {
            *overflow = true;
            break;
        }
        ++lvl;
        l_node[lvl * STRIDE] = k;
        l_mask[lvl * STRIDE] = child_mask(children, k);
    }
    *cnt_out = cnt;
    return visits;
}

// ---------------------------------------------------------------------------
// drop-in grid.svo_intersect: [b, m] rays against [b, n] trees.
__global__ __launch_bounds__(64) void k_svo_intersect_raw(int b, int n, int m, float voxelsize, int n_max,
                                                          const float *__restrict__ ray_start,
                                                          const float *__restrict__ ray_dir,
                                                          const float *__restrict__ points,
                                                          const int *__restrict__ children, int *__restrict__ idx,
                                                          float *__restrict__ min_depth,
                                                          float *__restrict__ max_depth) {
    __shared__ int l_node[kLevels * kWave];
    __shared__ int l_mask[kLevels * kWave];
    __shared__ int h_idx[kMaxHits * kWave];
    __shared__ float h_t0[kMaxHits * kWave];
    __shared__ float h_t1[kMaxHits * kWave];
    const int lane = threadIdx.x;
    const int64_t gid = (int64_t)blockIdx.x * kWave + lane;
    if (gid >= (int64_t)b * m) return;
    const int bi = (int)(gid / m);
    const float o[3] = {ray_start[gid * 3 + 0], ray_start[gid * 3 + 1], ray_start[gid * 3 + 2]};
    const float d[3] = {ray_dir[gid * 3 + 0], ray_dir[gid * 3 + 1], ray_dir[gid * 3 + 2]};
    int cnt = 0;
    bool overflow = false;
    const int nm = n_max < kMaxHits ? n_max : kMaxHits;
    dfs_ray(o, d, points + (int64_t)bi * n * 3, children + (int64_t)bi * n * 9, voxelsize * 0.5f, nm,
            l_node + lane, l_mask + lane, h_idx + lane, h_t0 + lane, h_t1 + lane, &cnt, &overflow);
    int *oi = idx + gid * n_max;
    float *omin = min_depth + gid * n_max;
    float *omax = max_depth + gid * n_max;
    for (int l = 0; l < n_max; ++l) {
        const bool v = l < cnt;
        oi[l] = v ? h_idx[l * kWave + lane] : -1;
        omin[l] = v ? h_t0[l * kWave + lane] : 0.0f;
        omax[l] = v ? h_t1[l * kWave + lane] : 0.0f;
    }
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) v = max(v, __shfl_xor(v, s, kWave));
    return v;
}
__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) v += __shfl_xor(v, s, kWave);
    return v;
}

// ---------------------------------------------------------------------------
// fused ray_intersect_vox: octree query → stable sort by t_in → max_distance
// trim, plus per-ray Σ(t_out - t_in) for the sampler's probs / steps.
//
// One wave per ray, KEY-ORDERED CHUNKED traversal instead of one-node-at-a-
// time DFS.  Every node has a path key Σ_d (7 − u_d)·8^(16−d); the
// reference's depth-first emission order (children popped 7→0,
// intersect_gpu.cu:191-270) is ascending key order, and the first n_max = 50
// leaves it emits are the 50 smallest leaf keys.  The wave keeps an LDS stack
// of untested candidates sorted by key (smallest on top) and each round pops
// up to 64 of them — one per lane — and tests them together: one dependent
// memory round trip per round (the candidate's centre and its whole
// structure row, children included, are independent loads), instead of one
// per AABB test.  Hit internal nodes push their existing children (keys
// ascending toward the top, so every child precedes every remaining
// candidate: preorder keys).  Once 50 leaves are known the 50th key bounds
// the search and every candidate beyond it is dropped (the DFS would never
// have reached it).  The stable sort by t_in breaks ties by key = DFS order.
// A round whose children would overflow the stack re-queues its tail lanes;
// a ray that cannot progress at all, or a tree deeper than the reference's
// 16-level stack, falls back to the serial DFS on lane 0 (same results,
// counted in stats[PSVO_STAT_SPILLS]).
constexpr int kStk = 512;    // candidate stack entries per ray
constexpr int kBfsL = 128;   // leaf list capacity (≤ 49 + 64 between compactions)
constexpr int kIsWaves = 8;  // waves (rays) per block
// the packed walk's two-chunk rounds (trace_pass TWO): for deep trees only —
// config E's traversal 73 → 67 µs, room0's +0.7 µs (profiles/r06_ab_two_chunk.txt)
constexpr int64_t kTwoChunkNodes = 1 << 18;

// Diagnostic build only (-DPSVO_IS_STAMPS, `make is_stamps`: lib/diag/): per
// ray, k_intersect_sorted's cycles by segment (s_memtime; scalar reads of the
// clock only), read through psvo_debug_is_stamps (scripts/intersect_stamps.py).
// Segments: [0] whole ray, [1] pop + node load + AABB test, [2] scan +
// re-queue + child push, [3] leaf merge, [4] final sort + output, [5] rounds,
// [6] rounds that found leaves, [7] AABB tests.  The product build has none.
#ifdef PSVO_IS_STAMPS
constexpr int kIsStampRays = 16384;
__device__ unsigned long long psvo_g_is_stamps[kIsStampRays][8];
#define IS_T(v)                                                                   \
    do {                                                                          \
        __builtin_amdgcn_sched_barrier(0);                                        \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory"); \
        __builtin_amdgcn_sched_barrier(0);                                        \
    } while (0)
#define IS_DECL unsigned long long is_t0 = 0, is_ta = 0, is_tb = 0, is_acc[5] = {0, 0, 0, 0, 0}, is_lr = 0
#define IS_MARK(var) IS_T(var)
#define IS_ADD(k, from, to) is_acc[k] += (to) - (from)
// k_sample_fused per workgroup (s_memrealtime, 100 MHz — one clock for all
// CUs): [0] entry, [1] its rays sampled (wave 0), [2] the row stores drained
// + barrier, [3] the look-back's prefix known (wave 0), [4] compaction done
__device__ unsigned long long psvo_g_smp_stamps[4096][8];
#define SMP_T(k)                                                                          \
    do {                                                                                  \
        __builtin_amdgcn_sched_barrier(0);                                                \
        const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                   \
        if ((threadIdx.x & 63) == 0 && w == 0) psvo_g_smp_stamps[blockIdx.x & 4095][k] = t_; \
        __builtin_amdgcn_sched_barrier(0);                                                \
    } while (0)
#define SMP_T0(k)                                                                         \
    do {                                                                                  \
        __builtin_amdgcn_sched_barrier(0);                                                \
        const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                   \
        if (threadIdx.x == 0) psvo_g_smp_stamps[blockIdx.x & 4095][k] = t_;               \
        __builtin_amdgcn_sched_barrier(0);                                                \
    } while (0)
#else
#define IS_DECL
#define IS_MARK(var)
#define IS_ADD(k, from, to)
#define SMP_T(k)
#define SMP_T0(k)
#endif

struct KeyLds {
    uint64_t skey[kStk];
    int snode[kStk];
    uint8_t sdep[kStk];
    uint64_t lkey[kBfsL];
    int lidx[kBfsL];
    float lt0[kBfsL], lt1[kBfsL];
    float hd[kMaxHits];  // t_out - t_in in sorted order
    int dfs_node[kLevels], dfs_mask[kLevels];
};

__device__ __forceinline__ uint64_t key_digit(int u, int depth) {
    return (uint64_t)(7 - u) << (3 * (kLevels - depth));
}

// inclusive prefix sum over the wave of v in [0, 16) (a node's child count):
// one ballot + lane-mask count per bit instead of six dependent cross-lane
// shuffles
__device__ __forceinline__ int wave_incl_scan16(int v) {
    int s = v;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const uint64_t m = __ballot((v >> b) & 1);
        s += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) << b;
    }
    return s;
}

// number of keys below k in the ascending list a[0, n), n <= 64: a
// branch-free binary search of 7 uniform steps (the leaf list is kept sorted
// by merging each round's leaves into it, so the prune's threshold — the 50th
// smallest key — is simply its last entry; no per-round selection)
__device__ __forceinline__ int count_below(const uint64_t *a, int n, uint64_t k) {
    int lo = 0;
#pragma unroll
    for (int step = kWave; step > 0; step >>= 1)
        if (lo + step <= n && a[lo + step - 1] < k) lo += step;
    return lo;
}


// The packed traversal's start below the root.  Every ray descends the same
// few top levels one round each (room0: 9 rounds per ray, one per level), so
// the records above the start level m (records [0, n_top), breadth-first,
// n_top <= 128; tree_pack.hip stores n_top and m in the root's spare word and
// the parent record in the others') are tested all at once — one round of
// independent loads — and "hit with every ancestor" is resolved by pointer
// jumping over the parent links (cross-lane, no LDS passes).  A node is
// tested by the reference's walk iff its parent passed (PSVO_STAT_VISITS
// counts exactly those).  The children of the passing level-(m−1) records
// are the level-m candidates, pushed in record order (within a level,
// breadth-first order is descending key order), the smallest key on top —
// the state the rounds would have reached, minus their latency.  The top
// levels hold no leaves (tree_pack.hip checks), so no prune can have applied.
// Returns the stack depth, or −1 (more than kStk candidates: the caller
// starts at the root).
__device__ int top_start(KeyLds &S, const PackRec *__restrict__ packed, const float o[3], const float inv[3],
                         float half, int n_top, int m, int lane, int &visits) {
    constexpr int kB = kPackTopMax / kWave;  // n_top <= kPackTopMax
    bool pa[kB];           // hit, then: hit and every ancestor hit
    int anc[kB], par[kB], first[kB], cmask[kB];
#pragma unroll
    for (int b = 0; b < kB; ++b) {
        const int j = b * kWave + lane;
        pa[b] = false;
        anc[b] = par[b] = -1;
        first[b] = -1;
        cmask[b] = 0;
        if (j < n_top) {
            const float4 pc = packed[j].c;
            const int4 pi = packed[j].i;
            float a = 0.f, t = 0.f;
            pa[b] = ray_aabb_nb(o, inv, pc.x, pc.y, pc.z, half * (float)__float_as_int(pc.w), a, t);
            par[b] = anc[b] = j == 0 ? -1 : pi.w;
            first[b] = pi.y;
            cmask[b] = pi.z;
        }
    }
    // pointer jumping: pa[j] = AND of the hits from j up to (excluding) anc[j]
    for (;;) {
        bool more = false;
#pragma unroll
        for (int b = 0; b < kB; ++b) more = more || anc[b] >= 0;
        if (!__ballot(more)) break;
        int wd[kB];
#pragma unroll
        for (int b = 0; b < kB; ++b) wd[b] = (anc[b] & 0x3FF) | (pa[b] ? 0x400 : 0);  // anc -1 → 0x3FF
        bool npa[kB];
        int nanc[kB];
#pragma unroll
        for (int b = 0; b < kB; ++b) {
            const int a = anc[b];
            int w = 0;
#pragma unroll
            for (int sb = 0; sb < kB; ++sb) {
                const int v = __shfl(wd[sb], a & (kWave - 1), kWave);
                if ((a >> 6) == sb) w = v;
            }
            npa[b] = a >= 0 ? (pa[b] && (w & 0x400)) : pa[b];
            nanc[b] = a >= 0 ? ((w & 0x3FF) == 0x3FF ? -1 : (w & 0x3FF)) : -1;
        }
#pragma unroll
        for (int b = 0; b < kB; ++b) {
            pa[b] = npa[b];
            anc[b] = nanc[b];
        }
    }
    // tested by the reference's walk: the root, and every node whose parent passed
    int tested = 0;
#pragma unroll
    for (int b = 0; b < kB; ++b) {
        const int p = par[b];
        bool parent_ok = false;
#pragma unroll
        for (int sb = 0; sb < kB; ++sb) {
            const int v = __shfl((int)pa[sb], p & (kWave - 1), kWave);
            if ((p >> 6) == sb) parent_ok = v != 0;
        }
        tested += (b * kWave + lane < n_top) && (b * kWave + lane == 0 || (p >= 0 && parent_ok)) ? 1 : 0;
    }
    // the level-m candidates: children of the passing level-(m-1) records
    // (those whose children lie past the top records), in record order.
    // Their keys: the candidate's rank in descending record order (= key
    // order within a level) in the level-m digit positions — the same order
    // as the path keys for every key this ray ever compares.
    int cnt[kB];
    int total = 0;
#pragma unroll
    for (int b = 0; b < kB; ++b) {
        cnt[b] = (pa[b] && first[b] >= n_top) ? __popc(cmask[b]) : 0;
        total += cnt[b];
    }
    total = wave_sum(total);
    if (total > kStk) return -1;
    const int shift = 3 * (kLevels - m);
    int run = 0;
#pragma unroll
    for (int b = 0; b < kB; ++b) {
        const int incl = wave_incl_scan16(cnt[b]);
        if (cnt[b]) {
            int g = run + incl - cnt[b];
            for (int k = 0; k < cnt[b]; ++k, ++g) {
                S.skey[g] = (uint64_t)(total - 1 - g) << shift;
                S.snode[g] = first[b] + k;
                S.sdep[g] = (uint8_t)m;
            }
        }
        run += __builtin_amdgcn_readlane(incl, kWave - 1);
    }
    visits += tested;
    return total;
}

// PACKED: candidates are records of the breadth-first packed tree
// (tree_pack.hip: centre + side and ref id / first child / child mask in one
// 32-B record, siblings contiguous) instead of reference node ids into the
// two AoS rows; the same floats, the same keys, the reference ids emitted.
// look-back blocks helped (lookback.h: a predecessor that had not started):
// [0] traversal, [1] sampler — diagnostic, read by psvo_debug_lb_helps
__device__ unsigned long long psvo_g_lb_helps[2];

// The per-ray work of k_intersect_sorted for the rays of block `cur` (one
// wave per ray): hit rows, ray_nv / ray_dsum, and the wave's totals in L.
// Inlined for the workgroup's own block; the look-back's help path calls
// trace_pass_help (not inlined: the own pass keeps its registers).
struct IsLds {
    int vis[kIsWaves], ov[kIsWaves], sp[kIsWaves], rd[kIsWaves], nv[kIsWaves], mc[kIsWaves], c0[kIsWaves];
};
template <bool PACKED, bool TWO = false>
__device__ __forceinline__ void trace_pass(int cur, int64_t n_rays, const float *__restrict__ rays_o,
                                           const float *__restrict__ rays_d, const float *__restrict__ centres,
                                           const int *__restrict__ structure, const PackRec *__restrict__ packed,
                                           float half, float max_distance, float step_size, int *__restrict__ hit_idx,
                                           float *__restrict__ hit_t0, float *__restrict__ hit_t1,
                                           int *__restrict__ ray_nv, float *__restrict__ ray_dsum, KeyLds &S,
                                           IsLds &L) {
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int64_t r = (int64_t)cur * kIsWaves + threadIdx.x / kWave;
    int visits = 0, rounds = 0;
    int w_nv = 0, w_mc = 0, w_c0 = -1;  // this wave's ray: valid hits, ⌈Σ/step⌉ (lane 0), first hit's id
    bool overflow_stack = false, spill = false;
    if (r < n_rays) {
        IS_DECL;
        IS_MARK(is_t0);
        const float o[3] = {rays_o[r * 3 + 0], rays_o[r * 3 + 1], rays_o[r * 3 + 2]};
        const float d[3] = {rays_d[r * 3 + 0], rays_d[r * 3 + 1], rays_d[r * 3 + 2]};
        float inv[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) inv[a] = __fdiv_rn(1.0f, d[a]);
        int nl = 0, sp = -1;
        bool bounded = false;
        uint64_t kbound = ~0ull;
        if constexpr (PACKED) {
            const int tw = packed[0].i.w;  // records above the start level | start level << 16 (0: none)
            if (tw > 0) sp = top_start(S, packed, o, inv, half, tw & 0xFFFF, tw >> 16, lane, visits);
        }
        if (sp < 0) {
            if (lane == 0) {  // the root is the first candidate
                S.skey[0] = 0;
                S.snode[0] = 0;
                S.sdep[0] = 0;
            }
            sp = 1;
        }
        wave_lds_sync();
        // merge one group's fresh leaves (keys ascending with the lane) into
        // the key-sorted list
        auto merge_leaves = [&](bool fresh, uint64_t key, int ref, float a, float b) {
            const uint64_t lb = __ballot(fresh);
            if (lb) {
                const int m = __popcll(lb), q = __popcll(lb & below);
                if (fresh) S.lkey[kWave + q] = key;  // scratch past the list (nl <= 50)
                const bool hold = lane < nl;
                uint64_t hk = 0;
                int hi = 0;
                float h0 = 0.f, h1 = 0.f;
                if (hold) {
                    hk = S.lkey[lane];
                    hi = S.lidx[lane];
                    h0 = S.lt0[lane];
                    h1 = S.lt1[lane];
                }
                wave_lds_sync();
                // final positions: own rank + the other list's keys below (keys are unique)
                const int pn = q + count_below(S.lkey, nl, key);
                const int po = lane + count_below(S.lkey + kWave, m, hk);
                wave_lds_sync();
                if (fresh && pn < kMaxHits) {
                    S.lkey[pn] = key;
                    S.lidx[pn] = ref;
                    S.lt0[pn] = a;
                    S.lt1[pn] = b;
                }
                if (hold && po < kMaxHits) {
                    S.lkey[po] = hk;
                    S.lidx[po] = hi;
                    S.lt0[po] = h0;
                    S.lt1[po] = h1;
                }
                nl = min(nl + m, kMaxHits);
                wave_lds_sync();
                if (nl == kMaxHits) {  // the 50 smallest keys kept; later candidates beyond them are dropped
                    kbound = S.lkey[kMaxHits - 1];
                    bounded = true;
                }
#ifdef PSVO_IS_STAMPS
                ++is_lr;
#endif
            } else {
                wave_lds_sync();
            }
        };
        while (sp > 0) {  // wave-uniform trip count
            ++rounds;
            IS_MARK(is_ta);
            const int n = min(sp, kWave);
            // PACKED: a full top chunk brings the next 64 entries along (group
            // B, one more record load in flight per lane); they are processed
            // in this round when every entry of both chunks is live and the
            // stack holds all their children — the heavy rays of a deep tree
            // (config E: up to ≈ 1,500 AABB tests) then walk half the rounds.
            // B's keys exceed A's and no B entry descends from an A entry, so
            // A's children stay above B's on the stack (key order); otherwise
            // B stays where it is, untouched (only read), for later rounds.
            const int nB = (PACKED && TWO) ? min(max(sp - kWave, 0), kWave) : 0;
            uint64_t key = 0, keyB = 0;
            int node = 0, dep = 0, nodeB = 0, depB = 0;
            if (lane < n) {
                const int e = sp - 1 - lane;
                key = S.skey[e];
                node = S.snode[e];
                dep = S.sdep[e];
            }
            if (lane < nB) {
                const int e = sp - 1 - kWave - lane;
                keyB = S.skey[e];
                nodeB = S.snode[e];
                depB = S.sdep[e];
            }
            // popped keys ascend with the lane: the live lanes are a prefix
            const bool live = lane < n && !(bounded && key > kbound);
            const int n_eff = __popcll(__ballot(live));
            const bool liveB = lane < nB && !(bounded && keyB > kbound);
            const bool two = nB > 0 && n_eff == kWave && __popcll(__ballot(liveB)) == nB;
            int row[8];
            int side = 0, first = 0, cmask = 0, ref = node;
            int sideB = 0, firstB = 0, cmaskB = 0, refB = nodeB;
            float a = 0.f, b = 0.f, aB = 0.f, bB = 0.f;
            bool hit = false, hitB = false;
            if (live) {
                if constexpr (PACKED) {
                    const float4 pc = packed[node].c;
                    const int4 pi = packed[node].i;
                    float4 pcB = make_float4(0.f, 0.f, 0.f, 0.f);
                    int4 piB = make_int4(0, 0, 0, 0);
                    if (two && liveB) {
                        pcB = packed[nodeB].c;
                        piB = packed[nodeB].i;
                    }
                    side = __float_as_int(pc.w);
                    ref = pi.x;
                    first = pi.y;
                    cmask = pi.z;
                    hit = ray_aabb_nb(o, inv, pc.x, pc.y, pc.z, half * (float)side, a, b);
                    if (two && liveB) {
                        sideB = __float_as_int(pcB.w);
                        refB = piB.x;
                        firstB = piB.y;
                        cmaskB = piB.z;
                        hitB = ray_aabb_nb(o, inv, pcB.x, pcB.y, pcB.z, half * (float)sideB, aB, bB);
                    }
                } else {
                    const int *rw = structure + (int64_t)node * 9;
#pragma unroll
                    for (int u = 0; u < 8; ++u) row[u] = rw[u];
                    side = rw[8];
                    const float *pc = centres + (int64_t)node * 3;
                    hit = ray_aabb_nb(o, inv, pc[0], pc[1], pc[2], half * (float)side, a, b);
                }
            }
            IS_MARK(is_tb);
            IS_ADD(1, is_ta, is_tb);
            const bool leaf = hit && side == 1;
            const bool inner = hit && side != 1;
            const bool leafB = hitB && sideB == 1;
            const bool innerB = hitB && sideB != 1;
            if (__ballot((inner && dep >= kLevels) || (innerB && depB >= kLevels))) {  // deeper than the reference's stack
                spill = true;
                break;
            }
            int c = 0, cB = 0;
            if (inner) {
                if constexpr (PACKED) {
                    c = __popc(cmask);
                } else {
#pragma unroll
                    for (int u = 0; u < 8; ++u) c += row[u] > -1;
                }
            }
            if (innerB) cB = __popc(cmaskB);
            const int incl = wave_incl_scan16(c);
            if (two) {
                const int inclB = wave_incl_scan16(cB);
                const int TA = __builtin_amdgcn_readlane(incl, kWave - 1);
                const int TB = __builtin_amdgcn_readlane(inclB, kWave - 1);
                const int floorB = sp - kWave - nB;
                if (floorB + TA + TB <= kStk) {  // (wave-uniform) both chunks accepted
                    wave_lds_sync();  // every lane has read its candidates before the stack is rewritten
                    // B's children, then A's on top, each in reverse key order
                    if (innerB) {
                        int g = inclB - cB;
                        const int cd = depB + 1;
#pragma unroll
                        for (int u = 7; u >= 0; --u) {
                            if ((cmaskB >> u) & 1) {
                                const int pos = floorB + (TB - 1 - g);
                                S.skey[pos] = keyB | key_digit(u, cd);
                                S.snode[pos] = firstB + __popc(cmaskB & ((1 << u) - 1));
                                S.sdep[pos] = (uint8_t)cd;
                                ++g;
                            }
                        }
                    }
                    if (inner) {
                        int g = incl - c;
                        const int cd = dep + 1;
#pragma unroll
                        for (int u = 7; u >= 0; --u) {
                            if ((cmask >> u) & 1) {
                                const int pos = floorB + TB + (TA - 1 - g);
                                S.skey[pos] = key | key_digit(u, cd);
                                S.snode[pos] = first + __popc(cmask & ((1 << u) - 1));
                                S.sdep[pos] = (uint8_t)cd;
                                ++g;
                            }
                        }
                    }
                    IS_MARK(is_ta);
                    IS_ADD(2, is_tb, is_ta);
                    visits += 1 + (liveB ? 1 : 0);
                    sp = floorB + TA + TB;
                    merge_leaves(leaf, key, ref, a, b);
                    merge_leaves(leafB, keyB, refB, aB, bB);
                    IS_MARK(is_tb);
                    IS_ADD(3, is_ta, is_tb);
                    continue;
                }
            }
            // a prune drops everything below the popped chunk (all keys > kbound)
            const int floor_ = (n_eff < n) ? 0 : sp - n;
            const bool ok = !live || floor_ + (n_eff - 1 - lane) + incl <= kStk;
            const uint64_t bad = __ballot(!ok);
            const int J = bad ? (int)__ffsll((unsigned long long)bad) - 1 : n_eff;  // accepted lanes [0, J)
            if (J == 0 && n_eff > 0) {
                spill = true;
                break;
            }
            const int T = J > 0 ? __builtin_amdgcn_readlane(incl, J - 1) : 0;
            const bool acc = lane < J;
            wave_lds_sync();  // every lane has read its candidate before the stack is rewritten
            if (live && !acc) {  // re-queued tail keeps its order on top of the floor
                const int pos = floor_ + (n_eff - 1 - lane);
                S.skey[pos] = key;
                S.snode[pos] = node;
                S.sdep[pos] = (uint8_t)dep;
            }
            const int base = floor_ + (n_eff - J);
            if (acc && inner) {
                int g = incl - c;  // rank of this lane's first (smallest-key) child
                const int cd = dep + 1;
#pragma unroll
                for (int u = 7; u >= 0; --u) {
                    const bool present = PACKED ? ((cmask >> u) & 1) != 0 : row[u] > -1;
                    if (present) {
                        const int pos = base + (T - 1 - g);
                        S.skey[pos] = key | key_digit(u, cd);
                        S.snode[pos] = PACKED ? first + __popc(cmask & ((1 << u) - 1)) : row[u];
                        S.sdep[pos] = (uint8_t)cd;
                        ++g;
                    }
                }
            }
            IS_MARK(is_ta);
            IS_ADD(2, is_tb, is_ta);
            visits += acc ? 1 : 0;
            sp = base + T;
            merge_leaves(acc && leaf, key, ref, a, b);
            IS_MARK(is_tb);
            IS_ADD(3, is_ta, is_tb);
        }
        if (spill) {  // serial DFS on lane 0 (reference order by construction; key = emission index)
            int cnt = 0;
            bool ov = false;
            if (lane == 0) {
                visits += dfs_ray<1>(o, d, centres, structure, half, kMaxHits, S.dfs_node, S.dfs_mask, S.lidx, S.lt0,
                                     S.lt1, &cnt, &ov);
                for (int i = 0; i < cnt; ++i) S.lkey[i] = (uint64_t)i;
            }
            cnt = __shfl(cnt, 0, kWave);
            overflow_stack = overflow_stack || __shfl((int)ov, 0, kWave);
            nl = cnt;
            wave_lds_sync();
        }
        IS_MARK(is_ta);
        // stable sort by t_in (ties: DFS order = key = list order, both paths
        // leave the list key-sorted), trim at max_distance; nl <= 50: one
        // entry per lane, the others' t_in read lane to lane
        int nv = 0;
        const float ti = lane < nl ? S.lt0[lane] : 0.f;
        int rank = 0;
        for (int j = 0; j < nl; ++j) {
            const float tj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ti), j));
            rank += (tj < ti) || (tj == ti && j < lane);
        }
        if (lane < nl) {
            const bool in = !(ti > max_distance);
            nv += in;
            const float bi = S.lt1[lane];
            S.hd[rank] = bi - ti;
            if (in) {
                hit_idx[r * kMaxHits + rank] = S.lidx[lane];
                hit_t0[r * kMaxHits + rank] = ti;
                hit_t1[r * kMaxHits + rank] = bi;
            }
        }
        nv = wave_sum(nv);
        {  // the first (nearest) hit's voxel id, for the sampler's by-rank copy
            const uint64_t m0 = __ballot(lane < nl && rank == 0 && !(ti > max_distance));
            const int c0 = __builtin_amdgcn_readlane(lane < nl ? S.lidx[lane] : -1, m0 ? __ffsll((unsigned long long)m0) - 1 : 0);
            w_c0 = m0 ? c0 : -1;
        }
        for (int l = nv + lane; l < kMaxHits; l += kWave) {
            hit_idx[r * kMaxHits + l] = -1;
            hit_t0[r * kMaxHits + l] = max_distance;
            hit_t1[r * kMaxHits + l] = max_distance;
        }
        wave_lds_sync();
        if (lane == 0) {
            float dsum = 0.0f;
            for (int l = 0; l < nv; ++l) dsum = dsum + S.hd[l];
            ray_nv[r] = nv;
            ray_dsum[r] = dsum;
            w_nv = nv;
            w_mc = nv > 0 ? (int)ceilf(__fdiv_rn(dsum, step_size)) : 0;  // k_ray_stats' arithmetic
        }
#ifdef PSVO_IS_STAMPS
        IS_MARK(is_tb);
        IS_ADD(4, is_ta, is_tb);
        const int is_vis = wave_sum(visits);
        if (lane == 0 && r < kIsStampRays) {
            psvo_g_is_stamps[r][0] = is_tb - is_t0;
            for (int k = 1; k < 5; ++k) psvo_g_is_stamps[r][k] = is_acc[k];
            psvo_g_is_stamps[r][5] = (unsigned long long)rounds;
            psvo_g_is_stamps[r][6] = is_lr;
            psvo_g_is_stamps[r][7] = (unsigned long long)is_vis;
        }
#endif
    }
    // visits / overflow: one atomic per block (per-ray P, R_hit and max ceil
    // are reduced by k_ray_stats: thousands of same-address atomics serialise
    // at the memory side)
    const int wvis = wave_sum(visits);
    const int wov = wave_max(overflow_stack ? 1 : 0);
    if (lane == 0) {
        L.vis[threadIdx.x / kWave] = wvis;
        L.ov[threadIdx.x / kWave] = wov;
        L.sp[threadIdx.x / kWave] = spill ? 1 : 0;
        L.rd[threadIdx.x / kWave] = rounds;  // wave-uniform
        L.nv[threadIdx.x / kWave] = w_nv;
        L.mc[threadIdx.x / kWave] = w_mc;
        L.c0[threadIdx.x / kWave] = w_c0;
    }
}

// A helped block's per-ray values for its aggregate (lookback.h: a
// predecessor that has not started), one wave per ray: the hits by the
// serial DFS (dfs_ray: the reference's emission order — the 50 smallest DFS
// keys the wave traversal keeps), then the same stable (t_in, DFS order)
// ranks, max_distance trim and left-to-right Σ(t_out − t_in) as trace_pass,
// so the hit count and ⌈Σ/step⌉ are the same bits; the AABB-test count is
// the DFS's (a statistic) and no rounds.  Nothing is written to the hit
// rows: the block's owner writes them when it runs.  Small on purpose — a
// second copy of the wave traversal here cost the own pass 3 µs.
__device__ __forceinline__ void help_trace_pass(int cur, int64_t n_rays, const float *rays_o, const float *rays_d,
                                             const float *centres, const int *structure, float half,
                                             float max_distance, float step_size, KeyLds &S, IsLds &L) {
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    const int64_t r = (int64_t)cur * kIsWaves + w;
    int nv = 0, mc = 0, visits = 0;
    if (r < n_rays) {
        const float o[3] = {rays_o[r * 3 + 0], rays_o[r * 3 + 1], rays_o[r * 3 + 2]};
        const float d[3] = {rays_d[r * 3 + 0], rays_d[r * 3 + 1], rays_d[r * 3 + 2]};
        int cnt = 0;
        bool ov = false;
        if (lane == 0)
            visits = dfs_ray<1>(o, d, centres, structure, half, kMaxHits, S.dfs_node, S.dfs_mask, S.lidx, S.lt0,
                                S.lt1, &cnt, &ov);
        cnt = __shfl(cnt, 0, kWave);
        visits = __shfl(visits, 0, kWave);
        wave_lds_sync();
        const float ti = lane < cnt ? S.lt0[lane] : 0.f;
        int rank = 0;
        for (int j = 0; j < cnt; ++j) {
            const float tj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ti), j));
            rank += (tj < ti) || (tj == ti && j < lane);
        }
        if (lane < cnt) S.hd[rank] = S.lt1[lane] - ti;
        nv = wave_sum(lane < cnt && !(ti > max_distance) ? 1 : 0);
        wave_lds_sync();
        if (lane == 0) {
            float dsum = 0.0f;
            for (int l = 0; l < nv; ++l) dsum = dsum + S.hd[l];
            mc = nv > 0 ? (int)ceilf(__fdiv_rn(dsum, step_size)) : 0;
        }
        mc = __shfl(mc, 0, kWave);
        wave_lds_sync();
    }
    if (lane == 0) {
        L.vis[w] = visits;
        L.rd[w] = 0;
        L.nv[w] = nv;
        L.mc[w] = mc;
    }
}

// wave 0: a block's aggregate {hit rays, P, max ⌈Σ/step⌉, AABB tests, rounds}
__device__ __forceinline__ void trace_agg(const IsLds &L, uint32_t (&agg)[5], uint64_t &hm) {
    const int lane = threadIdx.x & (kWave - 1);
    hm = __ballot(lane < kIsWaves && L.nv[lane] > 0);
    agg[0] = (uint32_t)__popcll(hm);
    agg[1] = agg[2] = agg[3] = agg[4] = 0u;
#pragma unroll
    for (int w = 0; w < kIsWaves; ++w) {
        agg[1] = max(agg[1], (uint32_t)L.nv[w]);
        agg[2] = max(agg[2], (uint32_t)L.mc[w]);
        agg[3] += (uint32_t)L.vis[w];
        agg[4] += (uint32_t)L.rd[w];
    }
}

template <bool PACKED, bool TWO = false>
__global__ __launch_bounds__(64 * kIsWaves) void k_intersect_sorted(int64_t n_rays, const float *__restrict__ rays_o,
                                                          const float *__restrict__ rays_d,
                                                          const float *__restrict__ centres,
                                                          const int *__restrict__ structure,
                                                          const PackRec *__restrict__ packed, float voxel_size,
                                                          float max_distance, float step_size,
                                                          int *__restrict__ hit_idx, float *__restrict__ hit_t0,
                                                          float *__restrict__ hit_t1, int *__restrict__ ray_nv,
                                                          float *__restrict__ ray_dsum, int *__restrict__ stats,
                                                          int *__restrict__ blk_out, int *__restrict__ ray_rank,
                                                          int *__restrict__ rank_ray, unsigned long long *lb_desc,
                                                          uint32_t lb_tag, int *__restrict__ nv_rank,
                                                          int *__restrict__ col0_rank, LbCtl ctl) {
    // lb_desc != nullptr: the statistics / hit-rank pass (k_ray_stats_rank)
    // runs in this launch by decoupled look-back (lookback.h): each workgroup
    // ranks its own hit rays, the last one writes P / R_hit / max ⌈Σ/step⌉.
    // A workgroup whose look-back finds a predecessor that has not started
    // traces that block's rays too (their aggregate: lookback.h) — the
    // pass loop below; `own` is the first pass.
    __shared__ KeyLds lds_all[kIsWaves];
    KeyLds &S = lds_all[threadIdx.x / kWave];
    const int lane = threadIdx.x & (kWave - 1);
    const int blk = (int)blockIdx.x;
    if (lb_desc) {
        lb_debug_delay(ctl, blk);
        if (threadIdx.x == 0) lb_mark_started<5>(lb_desc, blk, (int)gridDim.x, lb_tag);
    }
    const float half = voxel_size * 0.5f;
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    __shared__ IsLds L;
    __shared__ int s_cmd;
    trace_pass<PACKED, TWO>(blk, n_rays, rays_o, rays_d, centres, structure, packed, half, max_distance, step_size, hit_idx,
                       hit_t0, hit_t1, ray_nv, ray_dsum, S, L);
    __syncthreads();
    if (threadIdx.x == 0) {
        int v = 0, ov = 0, sps = 0, rd = 0;
        for (int w = 0; w < kIsWaves; ++w) {
            v += L.vis[w];
            ov |= L.ov[w];
            sps += L.sp[w];
            rd += L.rd[w];
        }
        if (lb_desc) {
            // summed by the look-back below
        } else if (blk_out) {  // summed by k_ray_stats_rank: no same-address atomics (they serialise at the memory side)
            blk_out[2 * blk] = v;
            blk_out[2 * blk + 1] = rd;
        } else {
            atomicAdd(stats + PSVO_STAT_VISITS, v);
            atomicAdd(stats + PSVO_STAT_ROUNDS, rd);
        }
        if (sps) atomicAdd(stats + PSVO_STAT_SPILLS, sps);
        if (ov) atomicOr(stats + 7, 1);
    }
    if (!lb_desc) return;
    // wave 0: the workgroup's aggregate → its exclusive prefix (lookback.h);
    // a predecessor that has not started: this workgroup traces that block's
    // rays too and publishes its aggregate (a helped block's statistics
    // arrive through it), then resumes its own look-back
    uint32_t own_agg[5], own_ex[5] = {0u, 0u, 0u, 0u, 0u};
    uint64_t own_hm = 0;
    int own_nv = 0, own_c0 = -1, lb_rc = kLbDone, spins = 0;
    if (threadIdx.x < kWave) {
        trace_agg(L, own_agg, own_hm);
        own_nv = lane < kIsWaves ? L.nv[lane] : 0;
        own_c0 = lane < kIsWaves ? L.c0[lane] : -1;
    }
    for (int cmd = -1;;) {  // one look-back call site; cmd ≥ 0: a block helped first
        if (cmd >= 0) {
            help_trace_pass(cmd, n_rays, rays_o, rays_d, centres, structure, half, max_distance, step_size, S, L);
            __syncthreads();
        }
        if (threadIdx.x < kWave) {
            if (cmd >= 0) {
                uint32_t agg[5];
                uint64_t hm;
                trace_agg(L, agg, hm);
                lb_publish<5>(lb_desc, cmd, lane, agg, lb_tag);
                if (lane == 0) atomicAdd(&psvo_g_lb_helps[0], 1ull);
            }
            lb_rc = lb_scan_help<5, 0b00110u>(lb_desc, blk, (int)gridDim.x, lb_tag, lane, own_agg, own_ex, spins,
                                               ctl.spin_max);
            if (lane == 0) s_cmd = lb_rc;
        }
        __syncthreads();
        cmd = __builtin_amdgcn_readfirstlane(s_cmd);
        if (cmd < 0) break;
    }
    if (threadIdx.x >= kWave) return;
    const bool ok = lb_rc == kLbDone;
    const uint32_t(&ex)[5] = own_ex;    // the exclusive prefix
    const uint32_t(&agg)[5] = own_agg;  // the own aggregate
    const int nv_l = own_nv;
    const uint64_t hm = own_hm;
    const int64_t rr = (int64_t)blk * kIsWaves + lane;
    if (lane < kIsWaves && rr < n_rays) {  // an abandoned wait (!ok) leaves `ex` undefined: no rank stores
        const int rk = (int)ex[0] + __popcll(hm & below);
        ray_rank[rr] = (nv_l > 0 && ok) ? rk : -1;
        if (nv_l > 0 && ok) {
            rank_ray[rk] = (int)rr;
            if (nv_rank) {  // by rank: the sampler's reads of other rows, one load each
                nv_rank[rk] = nv_l;
                col0_rank[rk] = own_c0;
            }
        }
    }
    if (lane == 0 && blk == (int)gridDim.x - 1) {  // the stats words were zeroed by the last read-back
        // an abandoned wait: no hit ray (the sampler then does nothing; the flag reports it)
        const int p = ok ? (int)max(ex[1], agg[1]) : 0, rh = ok ? (int)(ex[0] + agg[0]) : 0;
        const int mc = ok ? (int)max(ex[2], agg[2]) : 0;
        stats[PSVO_STAT_P] = p;
        stats[PSVO_STAT_R_HIT] = rh;
        stats[PSVO_STAT_MAX_CEIL] = mc;
        stats[kStatQuery + PSVO_STAT_P] = p;  // the sampler's copy (never re-zeroed inside its launch)
        stats[kStatQuery + PSVO_STAT_R_HIT] = rh;
        stats[kStatQuery + PSVO_STAT_MAX_CEIL] = mc;
        atomicAdd(stats + PSVO_STAT_VISITS, (int)(ex[3] + agg[3]));
        atomicAdd(stats + PSVO_STAT_ROUNDS, (int)(ex[4] + agg[4]));
    }
    if (!ok && lane == 0) atomicOr(stats + PSVO_STAT_FLAGS, kLbFlagTimeout);
}

// one wave, one word per lane (words <= 64)
__global__ void k_stats_to_host(int *__restrict__ stats, unsigned long long *host, int words, int seq, int zero) {
    const int i = threadIdx.x;
    if (i < words) {
        const int v = stats[i];
        if (zero) stats[i] = 0;  // ready for the query set's next use (no memset launch)
        stat_to_host(host, i, v, seq);
    }
}

// P (max valid hits), R_hit and max ceil(Σ/step) over the rays — one block.
__device__ void ray_stats_body(int64_t n, const int *__restrict__ ray_nv, const float *__restrict__ ray_dsum,
                               float step_size, int *__restrict__ stats) {
    int p = 0, hits = 0, mc = 0;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        const int nv = ray_nv[i];
        p = max(p, nv);
        hits += nv > 0;
        if (nv > 0) mc = max(mc, (int)ceilf(__fdiv_rn(ray_dsum[i], step_size)));
    }
    p = wave_max(p);
    hits = wave_sum(hits);
    mc = wave_max(mc);
    __shared__ int sp[16], sh[16], sm[16];
    const int w = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) {
        sp[w] = p;
        sh[w] = hits;
        sm[w] = mc;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < (int)(blockDim.x / kWave); ++k) {
            p = max(p, sp[k]);
            hits += sh[k];
            mc = max(mc, sm[k]);
        }
        stats[PSVO_STAT_P] = p;
        stats[PSVO_STAT_R_HIT] = hits;
        stats[PSVO_STAT_MAX_CEIL] = mc;
    }
}

__global__ __launch_bounds__(1024) void k_ray_stats(int64_t n, const int *__restrict__ ray_nv,
                                                    const float *__restrict__ ray_dsum, float step_size,
                                                    int *__restrict__ stats) {
    ray_stats_body(n, ray_nv, ray_dsum, step_size, stats);
}

// ---------------------------------------------------------------------------
// Single-workgroup exclusive scan (n ≲ 10^6): each thread owns a contiguous
// run; run totals scanned in LDS.
// Runs of up to kRegRun elements (n ≤ 8·1024 with 1024 threads) are read
// once, in one round of independent loads, and kept in registers (the
// general loop re-reads them after the barriers); `lmax`, if set, receives
// the thread's largest value.
constexpr int kRegRun = 8;

template <typename F>
__device__ void block_scan_runs(int64_t n, F value, int *__restrict__ out, int *total, int *lmax = nullptr) {
    // thread t scans the run [t·per, (t+1)·per); the run totals are scanned
    // with wave shuffles and one LDS pass over the ≤ 16 wave totals
    // (2 barriers instead of a 2·log2(1024)-barrier Hillis–Steele pass)
    __shared__ int s_wave[16];
    const int tid = threadIdx.x;
    const int nt = blockDim.x;
    const int lane = tid & (kWave - 1), w = tid / kWave, nw = nt / kWave;
    const int64_t per = (n + nt - 1) / nt;
    const int64_t beg = tid * per;
    const int64_t end = beg + per < n ? beg + per : n;
    const bool in_regs = per <= kRegRun;  // block-uniform
    int vals[kRegRun];
    int local = 0, mx = 0;
    if (in_regs) {
#pragma unroll
        for (int k = 0; k < kRegRun; ++k) vals[k] = beg + k < end ? value(beg + k) : 0;
#pragma unroll
        for (int k = 0; k < kRegRun; ++k) {
            local += vals[k];
            mx = max(mx, vals[k]);
        }
    } else {
        for (int64_t i = beg; i < end; ++i) {
            const int v = value(i);
            local += v;
            mx = max(mx, v);
        }
    }
    if (lmax) *lmax = mx;
    int incl = local;
#pragma unroll
    for (int sh = 1; sh < kWave; sh <<= 1) {
        const int t = __shfl_up(incl, sh, kWave);
        if (lane >= sh) incl += t;
    }
    if (lane == kWave - 1) s_wave[w] = incl;
    __syncthreads();
    if (w == 0) {
        int v = lane < nw ? s_wave[lane] : 0;
#pragma unroll
        for (int sh = 1; sh < 16; sh <<= 1) {
            const int t = __shfl_up(v, sh, kWave);
            if (lane >= sh) v += t;
        }
        if (lane < nw) s_wave[lane] = v;  // inclusive wave prefix
    }
    __syncthreads();
    int run = (w > 0 ? s_wave[w - 1] : 0) + incl - local;
    if (in_regs) {
#pragma unroll
        for (int k = 0; k < kRegRun; ++k)
            if (beg + k < end) {
                out[beg + k] = run;
                run += vals[k];
            }
    } else {
        for (int64_t i = beg; i < end; ++i) {
            out[i] = run;
            run += value(i);
        }
    }
    if (tid == nt - 1) *total = s_wave[nw - 1];
}

__device__ void hit_rank_body(int64_t n, const int *__restrict__ ray_nv, int *__restrict__ ray_rank,
                              int *__restrict__ rank_ray) {
    __shared__ int total;
    block_scan_runs(n, [&](int64_t i) { return ray_nv[i] > 0 ? 1 : 0; }, ray_rank, &total);
    __syncthreads();
    const int tid = threadIdx.x;
    for (int64_t i = tid; i < n; i += blockDim.x) {
        if (ray_nv[i] > 0) {
            rank_ray[ray_rank[i]] = (int)i;
        } else {
            ray_rank[i] = -1;
        }
    }
}

__global__ __launch_bounds__(1024) void k_hit_rank(int64_t n, const int *__restrict__ ray_nv,
                                                   int *__restrict__ ray_rank, int *__restrict__ rank_ray) {
    hit_rank_body(n, ray_nv, ray_rank, rank_ray);
}

// k_ray_stats + k_hit_rank in one launch (the engine's path).  Up to
// kRankPasses·1024 rays every input is read once, in one round of
// independent loads, and held in registers: ray i = k·1024 + t is thread t's
// pass k, its rank among the hit rays = the hit rays of the earlier passes +
// of the earlier waves of this pass (ballot counts in LDS, one scan) + the
// lower lanes (mbcnt).  The serial version (more rays) read ray_nv three
// times behind three barriers — dependent memory round trips on the
// critical path between the traversal and the sampler.
constexpr int kRankPasses = 8;

__global__ __launch_bounds__(1024) void k_ray_stats_rank(int64_t n, const int *__restrict__ ray_nv,
                                                         const float *__restrict__ ray_dsum, float step_size,
                                                         int *__restrict__ stats, int *__restrict__ ray_rank,
                                                         int *__restrict__ rank_ray, const int *__restrict__ blk_out,
                                                         int n_blk) {
    const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
    if (n <= (int64_t)kRankPasses * 1024 && n_blk <= 2048) {
        __shared__ int s_cnt[kRankPasses * 16];
        __shared__ int s_red[5][16];
        int nv[kRankPasses];
        float ds[kRankPasses];
        int v_blk = 0, r_blk = 0;
        if (blk_out) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int b = j * 1024 + tid;
                if (b < n_blk) {
                    v_blk += blk_out[2 * b];
                    r_blk += blk_out[2 * b + 1];
                }
            }
        }
#pragma unroll
        for (int k = 0; k < kRankPasses; ++k) {
            const int64_t i = (int64_t)k * 1024 + tid;
            nv[k] = i < n ? ray_nv[i] : 0;
            ds[k] = i < n ? ray_dsum[i] : 0.f;
        }
        int p = 0, mc = 0;
#pragma unroll
        for (int k = 0; k < kRankPasses; ++k) {
            p = max(p, nv[k]);
            if (nv[k] > 0) mc = max(mc, (int)ceilf(__fdiv_rn(ds[k], step_size)));
            const uint64_t m = __ballot(nv[k] > 0);
            if (lane == 0) s_cnt[k * 16 + w] = __popcll(m);
        }
        p = wave_max(p);
        mc = wave_max(mc);
        const int vs = wave_sum(v_blk), rs = wave_sum(r_blk);
        if (lane == 0) {
            s_red[0][w] = p;
            s_red[1][w] = mc;
            s_red[2][w] = vs;
            s_red[3][w] = rs;
        }
        __syncthreads();
        const int nw = blockDim.x / kWave;
        if (w == 0) {  // exclusive scan of the (pass, wave) hit counts, two per lane
            const int a0 = (lane * 2) / 16 < kRankPasses && (lane * 2) % 16 < nw ? s_cnt[lane * 2] : 0;
            const int a1 = (lane * 2 + 1) / 16 < kRankPasses && (lane * 2 + 1) % 16 < nw ? s_cnt[lane * 2 + 1] : 0;
            int incl = a0 + a1;
#pragma unroll
            for (int sh = 1; sh < kWave; sh <<= 1) {
                const int t = __shfl_up(incl, sh, kWave);
                if (lane >= sh) incl += t;
            }
            if (lane * 2 < kRankPasses * 16) {
                s_cnt[lane * 2] = incl - a0 - a1;
                s_cnt[lane * 2 + 1] = incl - a1;
            }
            if (lane == kWave - 1) s_red[4][0] = incl;  // hit rays
        }
        __syncthreads();
        if (tid == 0) {
            int pp = 0, mm = 0, vv = 0, rr = 0;
            for (int k = 0; k < nw; ++k) {
                pp = max(pp, s_red[0][k]);
                mm = max(mm, s_red[1][k]);
                vv += s_red[2][k];
                rr += s_red[3][k];
            }
            stats[PSVO_STAT_P] = pp;
            stats[PSVO_STAT_R_HIT] = s_red[4][0];
            stats[PSVO_STAT_MAX_CEIL] = mm;
            if (blk_out) {
                atomicAdd(stats + PSVO_STAT_VISITS, vv);
                atomicAdd(stats + PSVO_STAT_ROUNDS, rr);
            }
        }
#pragma unroll
        for (int k = 0; k < kRankPasses; ++k) {
            const int64_t i = (int64_t)k * 1024 + tid;
            const uint64_t m = __ballot(nv[k] > 0);
            if (i < n) {
                const int rk = s_cnt[k * 16 + w] +
                               (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                ray_rank[i] = nv[k] > 0 ? rk : -1;
                if (nv[k] > 0) rank_ray[rk] = (int)i;
            }
        }
        return;
    }
    if (blk_out) {  // the intersect blocks' AABB tests / traversal rounds
        int v = 0, rd = 0;
        for (int i = threadIdx.x; i < n_blk; i += blockDim.x) {
            v += blk_out[2 * i];
            rd += blk_out[2 * i + 1];
        }
        v = wave_sum(v);
        rd = wave_sum(rd);
        if ((threadIdx.x & (kWave - 1)) == 0) {
            atomicAdd(stats + PSVO_STAT_VISITS, v);  // 16 waves: 16 atomics
            atomicAdd(stats + PSVO_STAT_ROUNDS, rd);
        }
    }
    ray_stats_body(n, ray_nv, ray_dsum, step_size, stats);
    __syncthreads();
    hit_rank_body(n, ray_nv, ray_rank, rank_ray);
}

__global__ __launch_bounds__(1024) void k_scan_counts(int64_t n, const int *__restrict__ counts,
                                                      int *__restrict__ offsets) {
    __shared__ int total;
    block_scan_runs(n, [&](int64_t i) { return counts[i]; }, offsets, &total);
    __syncthreads();
    if (threadIdx.x == 0) offsets[n] = total;
}

// ---------------------------------------------------------------------------
// Sampler core shared by the drop-in launch and the fused path.  `Rows`
// abstracts where row elements come from: the drop-in kernel indexes a
// contiguous chunk exactly like the reference; the fused kernel maps the
// reference's logical [200, K', P] layout onto the compacted hit rays.
struct RawRows {
    const int *pts_idx;
    const float *min_depth, *max_depth, *probs;
    int H;
    __device__ int idx_at(int elem_from_H) const { return pts_idx[H + elem_from_H]; }
    __device__ int idx_slot0(int col) const { return pts_idx[col]; }
    __device__ float lo_at(int e) const { return min_depth[H + e]; }
    __device__ float hi_at(int e) const { return max_depth[H + e]; }
    __device__ float prob_at(int e) const { return probs[H + e]; }
    // bins of the ray's own row (e < max_hits)
    __device__ int own_idx(int e) const { return idx_at(e); }
    __device__ float own_lo(int e) const { return lo_at(e); }
    __device__ float own_hi(int e) const { return hi_at(e); }
    __device__ float own_prob(int e) const { return prob_at(e); }
};

struct FusedRows {
    const int *rank_ray;
    const int *hit_idx;
    const float *hit_t0, *hit_t1, *dsum;
    int P, r_hit;
    int own_row;   // logical row of this ray
    int base_row;  // logical row of slot 0 of this chunk of this block
    int jj;        // slot within the launch chunk
    __device__ int real(int lrow) const { return lrow < r_hit ? lrow : 0; }
    __device__ int64_t at(int elem_from_H) const {
        const int e = jj * P + elem_from_H;
        const int lrow = base_row + e / P;
        const int col = e % P;
        return (int64_t)rank_ray[real(lrow) - row_begin] * kMaxHits + col;
    }
    __device__ int idx_at(int e) const {
        if (fast) return e < P ? hit_idx[own_base + e] : next_c0;  // beyond the own row only (row + 1, col 0) is read
        if (slot0) {
            const int lrow = base_row + (jj * P + e) / P;
            if (lrow < row_begin || lrow >= row_end) return next_col0;  // only (own row + 1, col 0) is read
        }
        return hit_idx[at(e)];
    }
    __device__ int idx_slot0(int col) const {
        // the slot-0 row's valid hits are its prefix [0, nv): only "== -1" is asked
        if (fast) return col < slot0_nv ? 0 : -1;
        if (slot0) return col < slot0[slot0_row] ? 0 : -1;
        return hit_idx[(int64_t)rank_ray[real(base_row)] * kMaxHits + col];
    }
    __device__ float lo_at(int e) const { return hit_t0[at(e)]; }
    __device__ float hi_at(int e) const { return hit_t1[at(e)]; }
    __device__ float prob_at(int e) const {
        const int64_t a = at(e);
        const float dd = hit_idx[a] != -1 ? hit_t1[a] - hit_t0[a] : 0.0f;
        return __fdiv_rn(dd, dsum[rank_ray[real(own_row)]]);
    }
    // bins of the ray's own row (e < P): logical row own_row = i < r_hit, no division
    int64_t own_base;  // rank_ray[own_row] * kMaxHits
    float own_dsum;
    __device__ int own_idx(int e) const { return hit_idx[own_base + e]; }
    __device__ float own_lo(int e) const { return hit_t0[own_base + e]; }
    __device__ float own_hi(int e) const { return hit_t1[own_base + e]; }
    __device__ float own_prob(int e) const {
        const int64_t a = own_base + e;
        const float dd = hit_idx[a] != -1 ? hit_t1[a] - hit_t0[a] : 0.0f;
        return __fdiv_rn(dd, own_dsum);
    }
    // data-parallel engine: this rank holds only the logical rows
    // [row_begin, row_end) (rank_ray / hit_* are local); the sampler reads
    // other rows only as slot 0's hit counts (the slot-0 table, built from
    // the exchanged counts) and as the first voxel id of the row after its
    // own (next_col0)
    const int *slot0 = nullptr;  // [200 · nch] valid hits of each launch chunk's slot-0 row
    int slot0_row = 0;           // table row of (block, chunk)
    int row_begin = 0, row_end = 0, next_col0 = -1;
    // the engine's launches (the by-rank copies of the traversal: hit count
    // and first id per rank): the two reads of other rows preloaded with the
    // ray's own row — no rank → ray → row chain
    bool fast = false;
    int slot0_nv = 0, next_c0 = -1;
};

__device__ __forceinline__ uint32_t mix32(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return (uint32_t)x;
}

// inverse-CDF sampling of one ray; writes ≤ max_steps samples, returns count s.
template <typename Rows, typename Noise, typename Emit>
__device__ int sample_one(const Rows &rows, float steps_j, float fixed_step_size, int max_hits, int num_rays,
                          int H, int max_steps, Noise noise, Emit emit) {
    int bin = 0, s = 0;
    float lo_depth = rows.lo_at(0);
    float hi_depth = rows.hi_at(0);
    float lo_cdf = 0.0f;
    float hi_cdf = rows.prob_at(0);
    float step = (float)(1.0 / (double)steps_j);
    float z_low = lo_depth;
    const int total_steps = (int)ceilf(steps_j);
    bool done = false;
    if (fixed_step_size > 0.0f) step = fixed_step_size;
    for (int cs = 0; cs < total_steps; ++cs) {
        const float cdf = ((float)cs + noise(cs)) * step;
        while (cdf > hi_cdf) {
            if (s < max_steps) emit(s, rows.idx_at(bin), (hi_depth + z_low) * 0.5f, hi_depth - z_low);
            ++bin;
            ++s;
            if (bin >= max_hits || rows.idx_at(bin) == -1) {
                done = true;
                break;
            }
            lo_depth = rows.lo_at(bin);
            hi_depth = rows.hi_at(bin);
            lo_cdf = hi_cdf;
            hi_cdf = hi_cdf + rows.prob_at(bin);
            z_low = lo_depth;
        }
        if (done) break;
        const float u = __fdiv_rn(cdf - lo_cdf, hi_cdf - lo_cdf);
        const float z = lo_depth + u * (hi_depth - lo_depth);
        if (s < max_steps) emit(s, rows.idx_at(bin), (z + z_low) * 0.5f, z - z_low);
        z_low = z;
        ++s;
    }
    // sample_gpu.cu:224-237 verbatim semantics (see svo_oracle.c)
    while ((z_low < hi_depth) && (num_rays > (H + bin))) {
        if (s < max_steps) emit(s, rows.idx_at(bin), (hi_depth + z_low) * 0.5f, hi_depth - z_low);
        ++bin;
        ++s;
        if (bin >= max_hits || rows.idx_slot0(bin) == -1) break;
        lo_depth = rows.lo_at(bin);
        hi_depth = rows.hi_at(bin);
        z_low = lo_depth;
    }
    return s;
}

__global__ __launch_bounds__(64) void k_sample_raw(int b, int num_rays, int max_hits, int max_steps,
                                                   float fixed_step_size, const int *__restrict__ pts_idx,
                                                   const float *__restrict__ min_depth,
                                                   const float *__restrict__ max_depth,
                                                   const float *__restrict__ noise, const float *__restrict__ probs,
                                                   const float *__restrict__ steps, int *__restrict__ s_idx,
                                                   float *__restrict__ s_depth, float *__restrict__ s_dist) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (int64_t)b * num_rays) return;
    const int bi = (int)(gid / num_rays);
    const int j = (int)(gid % num_rays);
    const int64_t blk_h = (int64_t)bi * num_rays * max_hits;
    const int64_t blk_s = (int64_t)bi * num_rays * max_steps;
    RawRows rows{pts_idx + blk_h, min_depth + blk_h, max_depth + blk_h, probs + blk_h, j * max_hits};
    const int K = j * max_steps;
    const float *nz = noise + blk_s + K;
    int *oi = s_idx + blk_s + K;
    float *od = s_depth + blk_s + K;
    float *os = s_dist + blk_s + K;
    sample_one(
        rows, steps[(int64_t)bi * num_rays + j], fixed_step_size, max_hits, num_rays, j * max_hits, max_steps,
        [&](int cs) { return nz[cs]; },
        [&](int s, int v, float dep, float dis) {
            oi[s] = v;
            od[s] = dep;
            os[s] = dis;
        });
}

// Wave-parallel restatement of sample_one for one ray (one wave), valid when
// the cdf sequence ((cs + noise) * step) is non-decreasing — noise in [0, 1)
// and probs >= 0, which the fused path guarantees (probs are interval
// lengths / their sum; noise is clamped to [0.001, 0.999] or caller-given in
// [0, 1)).  The serial loop's output is a merge of two sorted streams:
//   interior sample cs in bin b(cs)   at position cs + b(cs)
//   end of bin b (bins it passed)     at position C_b + b
// with C_b = #{cs : !(cdf_cs > hcdf_b)} (first cs beyond bin b) and
// b(cs) = #{b : C_b <= cs}.  The trailing segment (sample_gpu.cu:224-237) is a
// run of consecutive bins whose first failing predicate a ballot finds.
// Every value is computed with the same float expressions as sample_one, so
// outputs are bit-identical to it.  Lane b owns bin b (max_hits <= 64).
struct WaveBins {  // per-wave LDS: bin b written by lane b, read by any lane
    float hc[kWave], lo[kWave], hi[kWave];
    int idx[kWave], c[kWave];
};


template <typename Rows, typename Noise, typename Emit>
__device__ int sample_wave(const Rows &rows, float steps_j, int max_hits, int num_rays, int H, Noise noise, Emit emit,
                           int lane, WaveBins &W) {
    const bool own = lane < max_hits;
    const int idx_b = own ? rows.own_idx(lane) : -1;
    const float lo_b = own ? rows.own_lo(lane) : 0.0f;
    const float hi_b = own ? rows.own_hi(lane) : 0.0f;
    const float prob_b = own ? rows.own_prob(lane) : 0.0f;
    // valid bins [0, nb): the serial loop stops at the first bin >= 1 with idx -1
    const uint64_t inval = __ballot(own && lane >= 1 && idx_b == -1);
    const int nb = inval ? min(__ffsll((unsigned long long)inval) - 1, max_hits) : max_hits;
    // hcdf_b: the serial running sum, same order of float additions
    SMP_T0(5);
    float acc = 0.0f, hcdf_b = 0.0f;
    for (int k = 0; k < nb; ++k) {
        const float pk = __shfl(prob_b, k, kWave);
        acc = (k == 0) ? pk : acc + pk;
        if (k == lane) hcdf_b = acc;
    }
    const float step = (float)(1.0 / (double)steps_j);
    const int total_steps = (int)ceilf(steps_j);
    auto cdf_at = [&](int cs) { return ((float)cs + noise(cs)) * step; };
    // C_b = first cs in [0, total_steps) with cdf_cs > hcdf_b (total_steps if none)
    int c_b = 0x7fffffff;  // bins past nb never end by cdf
    if (lane < nb) {
        int lo = 0, hi = total_steps;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (cdf_at(mid) > hcdf_b) hi = mid; else lo = mid + 1;
        }
        c_b = lo;
    }
    W.hc[lane] = hcdf_b;
    W.lo[lane] = lo_b;
    W.hi[lane] = hi_b;
    W.idx[lane] = idx_b;
    W.c[lane] = c_b;
    wave_lds_sync();
    SMP_T0(6);
    const int cs_end = W.c[nb - 1];  // first cs past the last valid bin
    const bool done = cs_end < total_steps;
    const int cs_lim = done ? cs_end : total_steps;
    // b(cs) = #{b < nb : C_b <= cs}; C_b is non-decreasing in b
    auto bin_of = [&](int cs) {
        int lo = 0, hi = nb;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (W.c[mid] <= cs) lo = mid + 1; else hi = mid;
        }
        return lo;
    };
    auto c_before = [&](int b) { return b == 0 ? 0 : W.c[b - 1]; };
    // z of interior sample c lying in bin b (sample_one: u, z)
    auto z_at = [&](int c, int b) {
        const float hc = W.hc[b];
        const float lc = b == 0 ? 0.0f : W.hc[b - 1];
        const float lo = W.lo[b], hi = W.hi[b];
        const float u = __fdiv_rn(cdf_at(c) - lc, hc - lc);
        return lo + u * (hi - lo);
    };
    // interior samples; z(cs - 1) comes from the neighbouring lane (the loop
    // bound is wave-uniform, so every lane takes part in the shuffles)
    float carry = 0.0f;
    for (int base = 0; base < cs_lim; base += kWave) {
        const int cs = base + lane;
        const bool act = cs < cs_lim;
        const int b = act ? bin_of(cs) : 0;
        const float z = act ? z_at(cs, b) : 0.0f;
        float zp = __shfl(z, lane > 0 ? lane - 1 : 0, kWave);
        if (lane == 0) zp = carry;
        carry = __shfl(z, kWave - 1, kWave);
        if (act) {
            const float z_low = cs == c_before(b) ? W.lo[b] : zp;
            emit(cs + b, W.idx[b], (z + z_low) * 0.5f, z - z_low);
        }
    }
    SMP_T0(7);
    // ends of the bins the main loop passed
    const int b_last = total_steps > 0 && !done ? bin_of(total_steps - 1) : 0;
    const int n_ends = done ? nb : b_last;
    // z_low at the end of bin b: its last interior sample, or lo_b if it has none
    auto end_z_low = [&](int b) { return W.c[b] > c_before(b) ? z_at(W.c[b] - 1, b) : W.lo[b]; };
    if (lane < n_ends) emit(c_b + lane, idx_b, (hi_b + end_z_low(lane)) * 0.5f, hi_b - end_z_low(lane));
    int s = cs_lim + n_ends;
    // trailing segment
    int bin0;
    float zl, hi_d;
    if (done) {
        bin0 = nb;
        zl = end_z_low(nb - 1);
        hi_d = W.hi[nb - 1];
    } else if (total_steps == 0) {
        bin0 = 0;
        zl = W.lo[0];
        hi_d = W.hi[0];
    } else {
        bin0 = b_last;
        zl = z_at(total_steps - 1, b_last);
        hi_d = W.hi[b_last];
    }
    if (zl < hi_d && num_rays > H + bin0) {
        const int v0 = bin0 < max_hits ? W.idx[bin0] : rows.idx_at(bin0);
        if (lane == 0) emit(s, v0, (hi_d + zl) * 0.5f, hi_d - zl);
        // bins k > bin0 continue while idx_slot0(k) != -1 && lo < hi && num_rays > H + k
        const bool cont = own && lane > bin0 && rows.idx_slot0(lane) != -1 && lo_b < hi_b && num_rays > H + lane;
        const uint64_t fail = ~__ballot(cont) & (~0ull << (bin0 + 1 < 64 ? bin0 + 1 : 63));
        const int k_end = bin0 + 1 >= 64 ? bin0 + 1 : (fail ? __ffsll((unsigned long long)fail) - 1 : 64);
        if (lane > bin0 && lane < k_end) emit(s + (lane - bin0), idx_b, (hi_b + lo_b) * 0.5f, hi_b - lo_b);
        s += k_end - bin0;
    }
    return s;
}

// Rows [row_begin, row_begin + n_rows) of the logical hit-ray order (n_rows <
// 0: through R_hit); ray i's outputs go to row i - row_begin.  A data-
// parallel rank samples its own rays inside the GLOBAL [200, K', P] layout
// this way: rank_ray / hit_* / dsum / stats then describe
// the all-gathered batch, and the noise key is the global logical index.
// the scan of the ray sample counts, the normaliser sums and the statistics
// read-back inside the sampler launch by decoupled look-back (single GPU;
// desc == nullptr: k_scan_samples runs after the launch instead)
struct SampleTail {
    int *offsets;              // [R_hit + 1] exclusive scan of ray_ns
    unsigned long long *host;  // PSVO_STAT_WORDS granules (stat_to_host)
    int seq;
    SampleCounts c;            // the Criterion's normalisers (c.gt_depth null: not counted)
    unsigned long long *desc;  // look-back descriptors (lookback.h), or null
    uint32_t tag;              // this launch's descriptor tag
    // with desc: the ray-major compacted samples (k_compact_rays' output:
    // leaf / t / ray_of_sample at offsets[r] + s, capacity R · max_steps_cap),
    // or null.  With desc the rows hold only their valid prefix (no padding:
    // every reader implies (-1, MAX_DEPTH) past the ray's count)
    int *leaf;
    float *t;
    int *ray_of;
    int *m_out;  // or null: the batch's sample count M, on the device (the step's device-sized forward)
    LbCtl ctl;   // lookback.h (tests: psvo_debug_set_lookback)
};
constexpr int kSmpStage = 256;  // a row's first samples staged in LDS for the in-launch compaction
constexpr int kSmpWaves = 8;    // k_sample_fused: waves (rays) per workgroup
// ray_cnt word: valid front / sdf samples (12 bits each), then whether a
// padded sample (z = MAX_DEPTH) is front / sdf, whether the ray's depth is valid
__device__ __forceinline__ int pack_counts(int nf, int nsm, bool pf, bool psm, bool valid) {
    return nf | (nsm << 12) | ((int)pf << 24) | ((int)psm << 25) | ((int)valid << 26);
}

// the sampler's look-back state (wave 0): the own block's aggregate {M,
// S_max, nf, nsm, Σ_pf ns, Σ_psm ns, pf | psm << 16, valid}, its lanes'
// in-block offsets, its exclusive prefix and the wait's state
struct SmpLb {  // in LDS: nothing of it stays in registers across the help passes
    uint32_t agg[kLbSmpGranules], ex[kLbSmpGranules];
    int before[kSmpWaves], rc, spins;
};
__device__ int smp_lb_pass(bool own, int cur, int blk, int nb, const int *s_ns, const int *s_cw, const SampleTail &tl,
                           SmpLb &lb);
__device__ void smp_lb_finish(int n, const SmpLb &lb, int *__restrict__ stats, const SampleTail &tl, int *s_off,
                              int st_word, int max_steps_cap, int blk);

// one ray of k_sample_fused; returns its valid-sample count, or -1 when the
// wave has no ray (the launch covers r_hit_cap rows)
template <bool HELP = false>
__device__ __forceinline__ int sample_fused_ray(int64_t row_begin, int64_t n_rows, int64_t r_hit_cap,
                                                int max_steps_cap, const int *__restrict__ rank_ray,
                                                const int *__restrict__ hit_idx, const float *__restrict__ hit_t0,
                                                const float *__restrict__ hit_t1, const float *__restrict__ ray_dsum,
                                                float step_size, const float *__restrict__ noise, uint64_t seed,
                                                int *__restrict__ stats, int *__restrict__ s_idx,
                                                float *__restrict__ s_depth, float *__restrict__ s_dist,
                                                const int *__restrict__ slot0, int slot0_nch,
                                                const int *__restrict__ nv_rank, const int *__restrict__ col0_rank,
                                                int &il_out, WaveBins &W, const SampleTail &tl, int &cnt_word,
                                                int *stage_i, float *stage_z, int blk, int wrow = -1);

__global__ __launch_bounds__(64 * kSmpWaves) void k_sample_fused(int64_t row_begin, int64_t n_rows, int64_t r_hit_cap,
                                                      int max_steps_cap,
                                                      const int *__restrict__ rank_ray,
                                                      const int *__restrict__ hit_idx,
                                                      const float *__restrict__ hit_t0,
                                                      const float *__restrict__ hit_t1,
                                                      const float *__restrict__ ray_dsum, float step_size,
                                                      const float *__restrict__ noise, uint64_t seed,
                                                      int *__restrict__ stats, int *__restrict__ s_idx,
                                                      float *__restrict__ s_depth, float *__restrict__ s_dist,
                                                      int *__restrict__ ray_ns, const int *__restrict__ slot0,
                                                      int slot0_nch, SampleTail tl, const int *__restrict__ nv_rank,
                                                      const int *__restrict__ col0_rank) {
    __shared__ WaveBins bins_all[kSmpWaves];
    // look-back mode (the engine's single-GPU query: row_begin 0, all rows):
    // the rows of this batch from the traversal's copy of its statistics
    // (kStatQuery: never re-zeroed inside this launch)
    const int blk = (int)blockIdx.x;
    const int *qp = stats + kStatQuery;
    const int n_lb = tl.desc && qp[PSVO_STAT_P] > 0 ? (int)min((int64_t)qp[PSVO_STAT_R_HIT], r_hit_cap) : 0;
    const int last_lb = n_lb > 0 ? (n_lb - 1) / kSmpWaves : 0;  // the workgroup holding the last row
    if (tl.desc && blk > last_lb) return;
    if (tl.desc) {
        lb_debug_delay(tl.ctl, blk);
        if (threadIdx.x == 0) lb_mark_started<kLbSmpGranules>(tl.desc, blk, last_lb + 1, tl.tag);
    }
    __shared__ int stage_i[kSmpWaves][kSmpStage];
    __shared__ float stage_z[kSmpWaves][kSmpStage];
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    SMP_T(0);
    const bool compact = tl.desc && tl.leaf;
    // the statistics words for the read-back, loaded now (the traversal's
    // are final; the one flag this launch adds is derived, not re-read):
    // no dependent round trip after the look-back in the last workgroup
    const int st_word = tl.desc && w == 0 && lane < PSVO_STAT_WORDS ? stats[lane] : 0;
    int il = 0, cnt_word = 0;
    int count = sample_fused_ray(row_begin, n_rows, r_hit_cap, max_steps_cap, rank_ray, hit_idx, hit_t0, hit_t1,
                                 ray_dsum, step_size, noise, seed, stats, s_idx, s_depth, s_dist, slot0, slot0_nch,
                                 nv_rank, col0_rank, il, bins_all[w], tl, cnt_word,
                                 compact ? stage_i[w] : nullptr, compact ? stage_z[w] : nullptr, blk);
    SMP_T(1);
    if (!tl.desc) {  // k_scan_samples reads them after the launch
        if (count >= 0 && lane == 0) {
            ray_ns[il] = count;
            if (tl.c.gt_depth) tl.c.ray_cnt[il] = cnt_word;
        }
        return;
    }
    __shared__ int s_ns[kSmpWaves], s_cw[kSmpWaves], s_off[kSmpWaves];
    if (lane == 0) {
        if (count >= 0) ray_ns[il] = count;
        s_ns[w] = count;  // -1: no row
        s_cw[w] = cnt_word;
    }
    // the counts publish before the rows' stores drain: a workgroup's
    // successors wait for its aggregate, not for its stores (measured: the
    // drain in front of the look-back cost up to 7 µs at the launch's tail)
    __syncthreads();
    SMP_T(2);
    __shared__ SmpLb lb;  // wave 0: the own block's aggregate / prefix
    if (w == 0) {
        // a predecessor that has not started: wave 0 counts its rows (one
        // per lane, the serial sampler) and publishes their aggregate, then
        // resumes its own look-back (lookback.h)
        __shared__ int s_hns[kSmpWaves], s_hcw[kSmpWaves];
        int rc = smp_lb_pass(true, blk, blk, last_lb + 1, s_ns, s_cw, tl, lb);
        while (rc >= 0) {
            if (lane < kSmpWaves) {
                int hil = 0, hcw = 0;
                const int hc = sample_fused_ray<true>(row_begin, n_rows, r_hit_cap, max_steps_cap, rank_ray, hit_idx,
                                                      hit_t0, hit_t1, ray_dsum, step_size, noise, seed, stats, s_idx,
                                                      s_depth, s_dist, slot0, slot0_nch, nv_rank, col0_rank, hil,
                                                      bins_all[0], tl, hcw, nullptr, nullptr, rc, lane);
                s_hns[lane] = hc;
                s_hcw[lane] = hcw;
            }
            rc = smp_lb_pass(false, rc, blk, last_lb + 1, s_hns, s_hcw, tl, lb);
        }
    }
    const int own_count = count, own_il = il;
    if (w == 0) smp_lb_finish(n_lb, lb, stats, tl, s_off, st_word, max_steps_cap, blk);
    SMP_T(3);
    if (!compact) return;
    // a row longer than the LDS stage is re-read below: this wave's own stores first
    if (own_count > kSmpStage) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // k_compact_rays' work: the row's valid prefix to its compacted place —
    // the first kSmpStage samples from LDS, the rest (rows longer than that)
    // read back from the row with sc1 loads (this wave's own stores, past L1)
    const int off = s_off[w];
    if (own_count <= 0 || off < 0) return;
    const int *oi = s_idx + (int64_t)own_il * max_steps_cap;
    const float *od = s_depth + (int64_t)own_il * max_steps_cap;
    for (int s = lane; s < own_count; s += kWave) {
        const bool st = s < kSmpStage;
        tl.leaf[off + s] = st ? stage_i[w][s] : ld_wt(oi + s);
        tl.t[off + s] = st ? stage_z[w][s] : ld_wt(od + s);
        tl.ray_of[off + s] = own_il;
    }
    SMP_T(4);
}

template <bool HELP>
__device__ __forceinline__ int sample_fused_ray(int64_t row_begin, int64_t n_rows, int64_t r_hit_cap,
                                                int max_steps_cap, const int *__restrict__ rank_ray,
                                                const int *__restrict__ hit_idx, const float *__restrict__ hit_t0,
                                                const float *__restrict__ hit_t1, const float *__restrict__ ray_dsum,
                                                float step_size, const float *__restrict__ noise, uint64_t seed,
                                                int *__restrict__ stats, int *__restrict__ s_idx,
                                                float *__restrict__ s_depth, float *__restrict__ s_dist,
                                                const int *__restrict__ slot0, int slot0_nch,
                                                const int *__restrict__ nv_rank, const int *__restrict__ col0_rank,
                                                int &il_out, WaveBins &W, const SampleTail &tl, int &cnt_word,
                                                int *stage_i, float *stage_z, int blk, int wrow) {
    // look-back mode: P / R_hit / max ⌈steps⌉ from the traversal's copy, which
    // no workgroup of this launch re-zeroes (a workgroup may start after the
    // last one zeroed the statistics: lookback.h helping)
    const int *qp = tl.desc ? stats + kStatQuery : stats;
    const int P = qp[PSVO_STAT_P];
    const int r_hit = qp[PSVO_STAT_R_HIT];
    const int max_steps = qp[PSVO_STAT_MAX_CEIL] + P;
    // the engine's launches (row_begin 0, or a data-parallel rank's own rows
    // indexed locally): the ray's rank → ray read beside the statistics words
    // the block's row of this wave (HELP: of this lane, wrow)
    if (wrow < 0) wrow = threadIdx.x / kWave;
    const int il_s = blk * (blockDim.x / kWave) + wrow;
    const int orig_s = (nv_rank && il_s < r_hit_cap) ? rank_ray[il_s] : 0;
    if (slot0) {  // data-parallel engine: the rank's rows, local rank_ray / hit arrays
        row_begin = stats[PSVO_STAT_ROW_BEGIN];
        n_rows = stats[PSVO_STAT_R_HIT_LOCAL];
    }
    const int lane = threadIdx.x & (kWave - 1);
    const int il = blk * (blockDim.x / kWave) + wrow;  // one ray per wave (HELP: per lane)
    const int i = (int)row_begin + il;                                        // logical row
    il_out = il;
    const int64_t n_own = n_rows < 0 ? (int64_t)r_hit - row_begin : n_rows;
    if (i >= r_hit || il >= n_own || il >= r_hit_cap || P <= 0) return -1;
    // (look-back mode: the last workgroup derives this flag; no atomics on `stats`)
    if (!tl.desc && max_steps > max_steps_cap && lane == 0 && il == 0) atomicOr(stats + PSVO_STAT_FLAGS, 2);
    const int kp = (r_hit + kSamplerG - 1) / kSamplerG;
    const int b = i / kp;
    const int j = i - b * kp;
    const int c = j / kSamplerChunk;
    const int jj = j - c * kSamplerChunk;
    const int nr = min(kSamplerChunk, kp - c * kSamplerChunk);
    const int orig = nv_rank ? orig_s : slot0 ? rank_ray[il] : rank_ray[i];
    // look-back mode (r_hit_cap = the batch's rays): a rank outside it only
    // after an abandoned look-back wait (flagged) — no row
    if (tl.desc && (orig < 0 || orig >= r_hit_cap)) return -1;
    const float dsum = ray_dsum[orig];
    FusedRows rows{rank_ray, hit_idx, hit_t0, hit_t1, ray_dsum, P, r_hit, i, b * kp + c * kSamplerChunk, jj,
                   (int64_t)orig * kMaxHits, dsum};
    if (slot0) {
        if (c >= slot0_nch) {  // the exchanged table covers slot0_nch launch chunks
            if (lane == 0) atomicOr(stats + PSVO_STAT_FLAGS, 4);
            return -1;
        }
        rows.slot0 = slot0;
        rows.slot0_row = b * slot0_nch + c;
        rows.row_begin = (int)row_begin;
        rows.row_end = (int)(row_begin + n_rows);
        rows.next_col0 = stats[PSVO_STAT_NEXT_COL0];
    }
    if (nv_rank) {  // the two reads of other rows, beside the own row's loads
        rows.fast = true;
        if (slot0) {
            rows.slot0_nv = slot0[rows.slot0_row];
            rows.next_c0 = il + 1 < n_rows ? col0_rank[il + 1] : rows.next_col0;
        } else {
            rows.slot0_nv = nv_rank[rows.base_row];  // base_row <= i < R_hit
            rows.next_c0 = col0_rank[i + 1 < r_hit ? i + 1 : 0];
        }
    }
    const float steps_j = __fdiv_rn(dsum, step_size);
    const int cap = max_steps < max_steps_cap ? max_steps : max_steps_cap;
    const bool nopad = tl.desc != nullptr;  // look-back mode: rows end at their valid prefix
    int *oi = s_idx + (int64_t)il * max_steps_cap;
    float *od = s_depth + (int64_t)il * max_steps_cap;
    float *os = s_dist ? s_dist + (int64_t)il * max_steps_cap : nullptr;  // the engine reads no distances
    const float *nz = noise ? noise + ((int64_t)b * kp + j) * max_steps : nullptr;
    const uint64_t key = seed * 0x9E3779B97F4A7C15ull + ((uint64_t)(b * kp + j) << 20);
    int count = 0;
    // the normalisers' per-sample terms (criterion.hip sample_terms) on the stored depths
    const bool counting = tl.c.gt_depth != nullptr;
    const float gd = counting ? tl.c.gt_depth[orig] : 0.f;
    const float lo_t = gd - tl.c.tr, hi_t = gd + tl.c.tr;
    const bool dm = gd > 0.0f && gd < tl.c.max_depth;
    int nf = 0, nsm = 0;
    auto noise_at = [&](int cs) {
        if (nz) return nz[cs];
        const float u = (float)(mix32(key + (uint64_t)cs) >> 8) * (1.0f / 16777216.0f);
        return fminf(fmaxf(u, 0.001f), 0.999f);
    };
    if constexpr (HELP) {
        // a helped row (lookback.h), one per lane: its count and count word
        // only, by the serial loop the wave sampler restates bit for bit
        // (sample_one) — small code; the row's owner writes it when it runs
        sample_one(rows, steps_j, 0.0f, P, nr, jj * P, cap, noise_at, [&](int s, int v, float dep, float) {
            if (s >= cap || v == -1) return;
            ++count;
            if (counting) {
                const bool f = dep < lo_t;
                nf += f;
                nsm += !f && !(dep > hi_t) && dm;
            }
        });
        if (counting) {
            const bool pf = kMaxDepthFill < lo_t;
            const bool psm = !pf && !(kMaxDepthFill > hi_t) && dm;
            cnt_word = pack_counts(nf, nsm, pf, psm, gd > 0.01f && gd < tl.c.max_depth);
        }
        return count;
    }
    const int s_end = sample_wave(
        rows, steps_j, P, nr, jj * P, noise_at,
        [&](int s, int v, float dep, float dis) {
            if (s >= cap) return;
            if (nopad && v == -1) return;  // the implied padding
            // voxel_helpers.py:654-656: clamp dists, MAX_DEPTH / 0 where idx == -1
            oi[s] = v;
            od[s] = v == -1 ? kMaxDepthFill : dep;
            if (os) os[s] = v == -1 ? 0.0f : fmaxf(dis, 0.0f);
            if (stage_i && s < kSmpStage) {  // v != -1 here (nopad)
                stage_i[s] = v;
                stage_z[s] = dep;
            }
            count += (v != -1);
            if (counting && v != -1) {
                const bool f = dep < lo_t;
                nf += f;
                nsm += !f && !(dep > hi_t) && dm;
            }
        },
        lane, W);
    const int s_written = nopad ? cap : s_end < cap ? s_end : cap;
    for (int s = s_written + lane; s < cap; s += kWave) {  // up to max_steps: readers stop at S_max <= max_steps
        oi[s] = -1;
        od[s] = kMaxDepthFill;
        if (os) os[s] = 0.0f;
    }
    if (counting) {
        const bool pf = kMaxDepthFill < lo_t;  // a padded sample: z = MAX_DEPTH
        const bool psm = !pf && !(kMaxDepthFill > hi_t) && dm;
        cnt_word = pack_counts(wave_sum(nf), wave_sum(nsm), pf, psm, gd > 0.01f && gd < tl.c.max_depth);
    }
    return wave_sum(count);
}

// k_scan_samples' work for one sampler workgroup (its 8 rows), wave 0 only,
// in two parts.  smp_lb_pass: the aggregate of block `cur`'s rows {M, S_max,
// and with the normalisers nf, nsm, Σ_pf ns, Σ_psm ns, pf | psm << 16,
// valid} — the own block's kept in `lb`, a helped block's published — then
// the own block's look-back (lookback.h lb_scan_help: returns the next block
// to help, or done / failed).  smp_lb_finish: its rows' offsets; the
// workgroup holding row n − 1 (block 0 when there is no row) writes
// offsets[n], the loss coefficients and the statistics read-back (granules,
// no system-scope release), and zeroes the device statistics for the next
// query.  Integer sums: exact, the same totals as k_scan_samples.
__device__ int smp_lb_pass(bool own, int cur, int blk, int nb, const int *s_ns, const int *s_cw, const SampleTail &tl,
                           SmpLb &lb) {
    constexpr int NG = kLbSmpGranules;
    const int lane = threadIdx.x & (kWave - 1);
    uint32_t agg[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) agg[g] = 0;
    int before = 0;  // samples of this workgroup's rows in front of lane's row
    const bool counting = tl.c.gt_depth != nullptr;
#pragma unroll
    for (int k = 0; k < kSmpWaves; ++k) {
        const int c = max(s_ns[k], 0);
        before += k < lane ? c : 0;
        agg[0] += (uint32_t)c;
        agg[1] = max(agg[1], (uint32_t)c);
        if (counting) {
            const int cw = s_ns[k] >= 0 ? s_cw[k] : 0;
            const int pf = (cw >> 24) & 1, psm = (cw >> 25) & 1;
            agg[2] += (uint32_t)(cw & 0xFFF);
            agg[3] += (uint32_t)((cw >> 12) & 0xFFF);
            agg[4] += pf ? (uint32_t)c : 0u;
            agg[5] += psm ? (uint32_t)c : 0u;
            agg[6] += (uint32_t)(pf | (psm << 16));
            agg[7] += (uint32_t)((cw >> 26) & 1);
        }
    }
    int spins = 0;
    if (own) {
#pragma unroll
        for (int g = 0; g < NG; ++g)
            if (lane == g) lb.agg[g] = agg[g];
        if (lane < kSmpWaves) lb.before[lane] = before;
    } else {
        lb_publish<NG>(tl.desc, cur, lane, agg, tl.tag);
        if (lane == 0) atomicAdd(&psvo_g_lb_helps[1], 1ull);
#pragma unroll
        for (int g = 0; g < NG; ++g) agg[g] = lb.agg[g];  // the own aggregate again
        spins = lb.spins;
    }
    uint32_t ex[NG];
    const int rc = lb_scan_help<NG, 0b10u>(tl.desc, blk, nb, tl.tag, lane, agg, ex, spins, tl.ctl.spin_max);
    if (lane == 0) {
        lb.rc = rc;
        lb.spins = spins;
    }
    if (rc == kLbDone) {
#pragma unroll
        for (int g = 0; g < NG; ++g)
            if (lane == g) lb.ex[g] = ex[g];
    }
    return rc;
}

__device__ void smp_lb_finish(int n, const SmpLb &lb, int *__restrict__ stats, const SampleTail &tl, int *s_off,
                              int st_word, int max_steps_cap, int blk) {
    const int lane = threadIdx.x & (kWave - 1);
    const bool ok = lb.rc == kLbDone;
    uint32_t ex[kLbSmpGranules], agg[kLbSmpGranules];
#pragma unroll
    for (int g = 0; g < kLbSmpGranules; ++g) {
        ex[g] = lb.ex[g];
        agg[g] = lb.agg[g];
    }
    const int last = n > 0 ? (n - 1) / kSmpWaves : 0;  // the workgroups past it returned without a descriptor
    const int il = blk * kSmpWaves + lane;
    const int before = lane < kSmpWaves ? lb.before[lane] : 0;
    // an abandoned wait (!ok: `ex` undefined) stores offset 0 (an in-bounds
    // range for any reader; the batch is reported failed) and the compaction
    // skips its rows
    if (lane < kSmpWaves) s_off[lane] = ok ? (int)ex[0] + before : -1;  // the in-launch compaction's
    if (lane < kSmpWaves && il < n) tl.offsets[il] = ok ? (int)ex[0] + before : 0;
    if (blk != last) return;
    const int tot = ok ? (int)(ex[0] + agg[0]) : 0;
    const int smax = ok ? (int)max(ex[1], agg[1]) : 0;
    if (lane == 0) {
        tl.offsets[n] = tot;
        if (tl.m_out) *tl.m_out = tot;  // an abandoned wait: no samples (the flag reports it)
    }
    if (tl.c.gt_depth && lane == 0) {  // the count sums over the padded [R_hit, S_max] layout (criterion.py:70-101)
        const uint32_t pp = ex[6] + agg[6];
        const long long t_nf = ex[2] + agg[2], t_nsm = ex[3] + agg[3], t_nspf = ex[4] + agg[4],
                        t_nspsm = ex[5] + agg[5], t_pf = pp & 0xFFFF, t_psm = pp >> 16, t_valid = ex[7] + agg[7];
        const long long n_f = t_nf + (long long)smax * t_pf - t_nspf;
        const long long n_s = t_nsm + (long long)smax * t_psm - t_nspsm;
        crit_coef_from_counts((double)t_valid, (double)n_f, (double)n_s, (double)n, (double)smax, tl.c.w_rgb,
                              tl.c.w_depth, tl.c.w_fs, tl.c.w_sdf, tl.c.tr, tl.c.crit_flags, tl.c.coef);
    }
    // the sampler's own flag (sample_fused_ray: max_steps beyond the rows' capacity)
    // (st_word: the last workgroup's load at its start — only it re-zeroes
    // the statistics, so its words are the traversal's; no dependent load here)
    const int max_steps = __shfl(st_word, PSVO_STAT_MAX_CEIL, kWave) + __shfl(st_word, PSVO_STAT_P, kWave);
    if (lane < PSVO_STAT_WORDS) {
        int v = lane == PSVO_STAT_S_MAX ? smax : lane == PSVO_STAT_M ? tot : st_word;
        if (lane == PSVO_STAT_FLAGS && n > 0 && max_steps > max_steps_cap) v |= 2;
        if (lane == PSVO_STAT_FLAGS && !ok) v |= kLbFlagTimeout;
        if (lane < kStatQuery) stats[lane] = 0;  // ready for the query set's next use (no memset launch)
        if (tl.host) stat_to_host(tl.host, lane, v, tl.seq);
    }
}

// offsets[0..R_hit] = exclusive scan of ray_ns; S_max and M into stats.  With
// `host` the statistics go to the host and `stats` is zeroed for the next
// query.
__global__ __launch_bounds__(1024) void k_scan_samples(int64_t row_begin, int64_t n_rows, int64_t r_hit_cap,
                                                       const int *__restrict__ ray_ns, int *__restrict__ offsets,
                                                       int *__restrict__ stats, int dist, unsigned long long *host,
                                                       int seq, SampleCounts cnt) {
    __shared__ int total;
    __shared__ int smax[16];
    __shared__ long long s_c[7][16];
    const int64_t n_own = dist ? (int64_t)stats[PSVO_STAT_R_HIT_LOCAL]
                               : n_rows < 0 ? (int64_t)stats[PSVO_STAT_R_HIT] - row_begin : n_rows;
    const int64_t n = max((int64_t)0, min(n_own, r_hit_cap));
    const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave, nw = blockDim.x / kWave;
    if ((n + blockDim.x - 1) / blockDim.x <= kRegRun) {
        // ≤ 8 rays per thread (R_hit ≤ 8,192): one round of independent loads —
        // the ray's sample count and its normaliser count word side by side —,
        // run sums / maxima / count sums in registers (32-bit: ≤ 8,192 rays of
        // ≤ 4,095 counts), one barrier, then the wave totals combined in
        // registers (every thread reads the ≤ 16 wave words it needs)
        __shared__ int s_wave[16], s_red[8][16];
        const int per = (int)((n + blockDim.x - 1) / blockDim.x);
        const int64_t beg = (int64_t)tid * per;
        int vals[kRegRun], cw[kRegRun];
#pragma unroll
        for (int k = 0; k < kRegRun; ++k) {
            const bool in = k < per && beg + k < n;
            vals[k] = in ? ray_ns[beg + k] : 0;
            cw[k] = in && cnt.gt_depth ? cnt.ray_cnt[beg + k] : 0;
        }
        int local = 0, mx = 0, c[7] = {0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < kRegRun; ++k) {
            local += vals[k];
            mx = max(mx, vals[k]);
            const int pf = (cw[k] >> 24) & 1, psm = (cw[k] >> 25) & 1;
            c[0] += cw[k] & 0xFFF;
            c[1] += (cw[k] >> 12) & 0xFFF;
            c[2] += pf;
            c[3] += psm;
            c[4] += (cw[k] >> 26) & 1;
            c[5] += pf ? vals[k] : 0;
            c[6] += psm ? vals[k] : 0;
        }
        int incl = local;
#pragma unroll
        for (int sh = 1; sh < kWave; sh <<= 1) {
            const int t = __shfl_up(incl, sh, kWave);
            if (lane >= sh) incl += t;
        }
        mx = wave_max(mx);
        if (cnt.gt_depth) {
#pragma unroll
            for (int k = 0; k < 7; ++k) c[k] = wave_sum(c[k]);
        }
        if (lane == kWave - 1) s_wave[w] = incl;
        if (lane == 0) {
            s_red[7][w] = mx;
#pragma unroll
            for (int k = 0; k < 7; ++k) s_red[k][w] = c[k];
        }
        __syncthreads();
        int before = 0, tot = 0;
        for (int k = 0; k < nw; ++k) {
            const int v = s_wave[k];
            before += k < w ? v : 0;
            tot += v;
        }
        int run = before + incl - local;
#pragma unroll
        for (int k = 0; k < kRegRun; ++k)
            if (k < per && beg + k < n) {
                offsets[beg + k] = run;
                run += vals[k];
            }
        if (w != 0) return;
        // wave 0: the block's maximum and count sums over the ≤ 16 wave words
        const bool wl = lane < nw;
        int bm = wl ? s_red[7][lane] : 0;
#pragma unroll
        for (int sh = 8; sh > 0; sh >>= 1) bm = max(bm, __shfl_xor(bm, sh, kWave));
        bm = __shfl(bm, 0, kWave);
        if (lane == 0) offsets[n] = tot;
        if (cnt.gt_depth) {
            int t[7];
#pragma unroll
            for (int k = 0; k < 7; ++k) {
                int v = wl ? s_red[k][lane] : 0;
#pragma unroll
                for (int sh = 8; sh > 0; sh >>= 1) v += __shfl_xor(v, sh, kWave);
                t[k] = v;
            }
            if (lane == 0) {  // the count sums over the padded [R_hit, S_max] layout → coefficients
                const long long n_f = (long long)t[0] + (long long)bm * t[2] - t[5];
                const long long n_s = (long long)t[1] + (long long)bm * t[3] - t[6];
                crit_coef_from_counts((double)t[4], (double)n_f, (double)n_s, (double)n, (double)bm, cnt.w_rgb,
                                      cnt.w_depth, cnt.w_fs, cnt.w_sdf, cnt.tr, cnt.crit_flags, cnt.coef);
            }
        }
        if (host) {  // the engine's read-back (every reader of stats is past the barrier)
            if (lane < PSVO_STAT_WORDS) {
                const int v = lane == PSVO_STAT_S_MAX ? bm : lane == PSVO_STAT_M ? tot : stats[lane];
                stats[lane] = 0;
                stat_to_host(host, lane, v, seq);
            }
        } else if (lane == 0) {
            stats[PSVO_STAT_S_MAX] = bm;
            stats[PSVO_STAT_M] = tot;
        }
        return;
    }
    int mx = 0;
    block_scan_runs(n, [&](int64_t i) { return ray_ns[i]; }, offsets, &total, &mx);
    mx = wave_max(mx);
    if (lane == 0) smax[w] = mx;
    if (cnt.gt_depth) {  // the loss normalisers' per-ray counts (k_sample_fused), exact integer sums
        long long c[7] = {};
        for (int64_t i0 = tid; i0 < n; i0 += (int64_t)blockDim.x * 8) {
            int cw[8], ns[8];  // one round of independent loads, then the sums
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int64_t i = i0 + (int64_t)k * blockDim.x;
                cw[k] = i < n ? cnt.ray_cnt[i] : 0;
                ns[k] = i < n ? ray_ns[i] : 0;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int pf = (cw[k] >> 24) & 1, psm = (cw[k] >> 25) & 1;
                c[0] += cw[k] & 0xFFF;
                c[1] += (cw[k] >> 12) & 0xFFF;
                c[2] += pf;
                c[3] += psm;
                c[4] += (cw[k] >> 26) & 1;
                c[5] += pf ? ns[k] : 0;
                c[6] += psm ? ns[k] : 0;
            }
        }
#pragma unroll
        for (int k = 0; k < 7; ++k) {
#pragma unroll
            for (int sh = 32; sh > 0; sh >>= 1) c[k] += __shfl_xor(c[k], sh, kWave);
            if (lane == 0) s_c[k][w] = c[k];
        }
    }
    __syncthreads();
    if (tid < kWave) {  // wave 0; with `host` one statistics word per lane (no serial copy loop)
        for (int k = 1; k < nw; ++k) mx = max(mx, smax[k]);
        const int tot = total;
        if (lane == 0) offsets[n] = tot;
        if (cnt.gt_depth && lane == 0) {  // the count sums over the padded [R_hit, S_max] layout → coefficients
            long long t[7];
            for (int k = 0; k < 7; ++k) {
                t[k] = 0;
                for (int q = 0; q < nw; ++q) t[k] += s_c[k][q];
            }
            const long long n_f = t[0] + (long long)mx * t[2] - t[5];
            const long long n_s = t[1] + (long long)mx * t[3] - t[6];
            crit_coef_from_counts((double)t[4], (double)n_f, (double)n_s, (double)n, (double)mx, cnt.w_rgb,
                                  cnt.w_depth, cnt.w_fs, cnt.w_sdf, cnt.tr, cnt.crit_flags, cnt.coef);
        }
        if (host) {  // the engine's read-back, as k_stats_to_host (every reader of stats is past the barrier)
            if (lane < PSVO_STAT_WORDS) {
                const int v = lane == PSVO_STAT_S_MAX ? mx : lane == PSVO_STAT_M ? tot : stats[lane];
                stats[lane] = 0;
                stat_to_host(host, lane, v, seq);
            }
        } else if (lane == 0) {
            stats[PSVO_STAT_S_MAX] = mx;
            stats[PSVO_STAT_M] = tot;
        }
    }
}

// ---------------------------------------------------------------------------
// z_vals / mask [R_hit, S_max] and ray-major compacted samples.
__global__ void k_sample_points(int64_t r_hit, int s_max, int cap, const int *__restrict__ s_idx,
                                const float *__restrict__ s_depth, const int *__restrict__ ray_ns,
                                const int *__restrict__ offsets, int *__restrict__ leaf, float *__restrict__ t,
                                int *__restrict__ ray_of_sample, float *__restrict__ z_vals,
                                uint8_t *__restrict__ mask) {
    // grid rows stride over the hit rays (no 64-bit division per element)
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= s_max) return;
    for (int64_t r = blockIdx.y; r < r_hit; r += gridDim.y) {
        const int64_t e = r * s_max + s;
        // valid samples form a prefix of each row; past it the padding
        // (-1, MAX_DEPTH) is implied — the look-back sampler does not write it
        const bool in = s < offsets[r + 1] - offsets[r];
        const int v = in ? s_idx[r * cap + s] : -1;
        const float z = in ? s_depth[r * cap + s] : kMaxDepthFill;
        z_vals[e] = z;
        mask[e] = v != -1;
        if (v != -1) {
            const int64_t o = offsets[r] + s;
            leaf[o] = v;
            t[o] = z;
            ray_of_sample[o] = (int)r;
        }
    }
}

// Ray-major sample compaction only (the engine's mapping path: the loss
// kernels read z from the sampler's rows, so no padded [R_hit, S_max] copy):
// one wave per hit ray copies the valid prefix of its sampler row to the
// compact arrays — ns ≈ 64 entries, not the S_max-wide row k_sample_points
// walks.
__global__ __launch_bounds__(256) void k_compact_rays(int64_t r_hit, int cap, const int *__restrict__ s_idx,
                                                      const float *__restrict__ s_depth,
                                                      const int *__restrict__ offsets, int *__restrict__ leaf,
                                                      float *__restrict__ t, int *__restrict__ ray_of_sample) {
    const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (r >= r_hit) return;
    const int lane = threadIdx.x & (kWave - 1);
    const int beg = offsets[r], ns = offsets[r + 1] - beg;
    for (int s = lane; s < ns; s += kWave) {
        leaf[beg + s] = s_idx[r * cap + s];
        t[beg + s] = s_depth[r * cap + s];
        ray_of_sample[beg + s] = (int)r;
    }
}

// ---------------------------------------------------------------------------
// Data-parallel query (engine.cpp): each rank samples
// its own hit rays inside the [200, K', P] layout of the union batch (ranks
// in order).  Besides P / R_hit / max ceil(steps) of the union, the sampler
// reads other ranks' rows in two places only (sample_gpu.cu:224-237): whether
// column k of each launch chunk's slot-0 row is a hit (idx_slot0(k) == -1 —
// a row's hits are its prefix, so that is k < the row's hit count) and the
// first voxel id of the row after a ray's own (a ray with exactly P bins).
// So ONE all-gather carries everything: per rank 8 words and the hit count
// of each of its hit rows (a byte each, rank order) — every rank then builds
// the union layout and the [200 · nch] slot-0 count table itself.
constexpr int kDistWords = 8;  // per rank: R_hit, P, max ceil, first voxel id of its first hit row, flags

// this rank's words: thread t packs the hit counts of its hit rows 4t..4t+3
__global__ __launch_bounds__(256) void k_dist_pack(const int *__restrict__ stats, const int *__restrict__ rank_ray,
                                                   const int *__restrict__ hit_idx, const int *__restrict__ ray_nv,
                                                   int *__restrict__ out, const int *__restrict__ nv_rank,
                                                   int flags_or) {
    const int r_hit = stats[PSVO_STAT_R_HIT];
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t == 0) {
        out[0] = r_hit;
        out[1] = stats[PSVO_STAT_P];
        out[2] = stats[PSVO_STAT_MAX_CEIL];
        out[3] = r_hit > 0 ? hit_idx[(int64_t)rank_ray[0] * kMaxHits] : -1;
        // e.g. a DFS-stack overflow on one rank: every rank fails together; and
        // PSVO_FLAG_UNION_UNCOUNTED from a rank whose query had no GT depths
        out[4] = stats[PSVO_STAT_FLAGS] | flags_or;
        for (int k = 5; k < kDistWords; ++k) out[k] = 0;
    }
    const int j0 = 4 * t;
    if (j0 >= r_hit) return;
    uint32_t w = 0;
    for (int k = 0; k < 4 && j0 + k < r_hit; ++k)  // nv <= 50
        w |= (uint32_t)(nv_rank ? nv_rank[j0 + k] : ray_nv[rank_ray[j0 + k]]) << (8 * k);
    out[kDistWords + t] = (int)w;
}

// union-batch statistics and the slot-0 count table from the gathered words
// (world x stride): table[b · nch + c] = hit count of logical row b·K' + c·800
// (row 0 past the union's end)
__global__ __launch_bounds__(256) void k_dist_layout(const int *__restrict__ all, int world, int rank, int stride,
                                                     int nch, int *__restrict__ stats, int *__restrict__ table,
                                                     int *__restrict__ q2_in) {
    int r_hit = 0;
    for (int r = 0; r < world; ++r) r_hit += all[r * stride];
    // this query's count words start at zero (k_dist_counts adds into them),
    // whatever an earlier query that failed before k_dist_smax left there
    if (q2_in && threadIdx.x >= 1 && threadIdx.x < kDistWords) q2_in[threadIdx.x] = 0;
    if (threadIdx.x == 0) {
        int p = 0, mc = 0, begin = 0, flags = 0;
        for (int r = 0; r < world; ++r) {
            const int *w = all + r * stride;
            if (r < rank) begin += w[0];
            p = max(p, w[1]);
            mc = max(mc, w[2]);
            flags |= w[4];
        }
        // the logical row after this rank's last: the next rank holding hit rows,
        // or (past the union's last row) row 0, as the reference's row-0 padding
        int next = -1;
        for (int r = rank + 1; r < world && next < 0; ++r)
            if (all[r * stride] > 0) next = r;
        for (int r = 0; r < world && next < 0; ++r)
            if (all[r * stride] > 0) next = r;
        stats[PSVO_STAT_R_HIT_LOCAL] = all[rank * stride];
        stats[PSVO_STAT_ROW_BEGIN] = begin;
        stats[PSVO_STAT_NEXT_COL0] = next >= 0 ? all[next * stride + 3] : -1;
        stats[PSVO_STAT_P] = p;
        stats[PSVO_STAT_R_HIT] = r_hit;
        stats[PSVO_STAT_MAX_CEIL] = mc;
        stats[PSVO_STAT_FLAGS] |= flags;
    }
    const int kp = (r_hit + kSamplerG - 1) / kSamplerG;
    for (int row = threadIdx.x; row < kSamplerG * nch; row += blockDim.x) {
        const int b = row / nch, c = row - b * nch;
        int lrow = b * kp + c * kSamplerChunk;
        if (lrow >= r_hit) lrow = 0;
        int nv = 0;
        if (r_hit > 0) {
            int o = 0, beg = 0;
            while (lrow >= beg + all[o * stride]) beg += all[o++ * stride];  // the owner: lrow < r_hit
            const int j = lrow - beg;
            nv = (int)(((uint32_t)all[o * stride + kDistWords + (j >> 2)] >> (8 * (j & 3))) & 0xffu);
        }
        table[row] = nv;
    }
}

// after the gather of [S_max, count words] (world x 8): the union S_max and,
// given the rank's counts (dist_counts), the union's normaliser sums —
// integers, so any summation order gives the single-GPU doubles; zeroes the
// rank's count words for the next query's atomics
__global__ void k_dist_smax(const int *__restrict__ all, int world, int *__restrict__ stats, int *__restrict__ in,
                            double *__restrict__ sums) {
    if (threadIdx.x != 0) return;
    int mx = 0;
    bool counted = true;  // every rank counted its rows against GT depths (k_dist_counts)
    for (int r = 0; r < world; ++r) {
        const int w0 = all[r * kDistWords];
        mx = max(mx, w0 & ~kDistNotCounted);
        counted = counted && !(w0 & kDistNotCounted);
    }
    stats[PSVO_STAT_S_MAX_LOCAL] = stats[PSVO_STAT_S_MAX];
    stats[PSVO_STAT_S_MAX] = mx;
    // the same on every rank: whether the step may take the union's count
    // sums from here or must count (and all-reduce) them itself
    if (!counted) stats[PSVO_STAT_FLAGS] |= PSVO_FLAG_UNION_UNCOUNTED;
    if (sums && counted) {
        long long c[7] = {0, 0, 0, 0, 0, 0, 0};
        for (int r = 0; r < world; ++r)
            for (int k = 0; k < 7; ++k) c[k] += all[r * kDistWords + 1 + k];
        // words: n_valid, Σ front, Σ sdf band (valid samples), rays whose padding is front,
        // Σ their ns, rays whose padding is in the band, Σ their ns (dist_counts)
        for (int k = 0; k < 8; ++k) sums[k] = 0.0;
        sums[2] = (double)c[0];                       // kNValid
        sums[3] = (double)(c[1] + mx * c[3] - c[4]);  // kNFront: + (S_max − ns) per padded-front ray
        sums[4] = (double)(c[2] + mx * c[5] - c[6]);  // kNSdf
    }
    for (int k = 1; k < kDistWords; ++k) in[k] = 0;
}

}  // namespace

}  // namespace psvo

using namespace psvo;

extern "C" int psvo_svo_intersect(void *stream, int b, int n, int m, float voxelsize, int n_max,
                                  const float *ray_start, const float *ray_dir, const float *points,
                                  const int *children, int *idx, float *min_depth, float *max_depth) {
    PSVO_REQUIRE(b >= 0 && n > 0 && m >= 0 && n_max > 0, "svo_intersect: bad sizes b=%d n=%d m=%d n_max=%d", b, n, m,
                 n_max);
    PSVO_REQUIRE(n_max <= kMaxHits, "svo_intersect: n_max=%d exceeds %d", n_max, kMaxHits);
    const int64_t total = (int64_t)b * m;
    if (total == 0) return PSVO_OK;
    psvo::launch(k_svo_intersect_raw, dim3(div_up(total, kWave)), dim3(kWave), 0, as_stream(stream), b, n, m,
                       voxelsize, n_max, ray_start, ray_dir, points, children, idx, min_depth, max_depth);
    return check_launch("svo_intersect");
}

extern "C" int psvo_inverse_cdf_sampling(void *stream, int b, int num_rays, int max_hits, int max_steps,
                                         float fixed_step_size, const int *pts_idx, const float *min_depth,
                                         const float *max_depth, const float *uniform_noise, const float *probs,
                                         const float *steps, int *sampled_idx, float *sampled_depth,
                                         float *sampled_dists) {
    PSVO_REQUIRE(b >= 0 && num_rays >= 0 && max_hits > 0 && max_steps > 0,
                 "inverse_cdf_sampling: bad sizes b=%d num_rays=%d max_hits=%d max_steps=%d", b, num_rays, max_hits,
                 max_steps);
    const int64_t total = (int64_t)b * num_rays;
    if (total == 0) return PSVO_OK;
    psvo::launch(k_sample_raw, dim3(div_up(total, kWave)), dim3(kWave), 0, as_stream(stream), b, num_rays,
                       max_hits, max_steps, fixed_step_size, pts_idx, min_depth, max_depth, uniform_noise, probs,
                       steps, sampled_idx, sampled_depth, sampled_dists);
    return check_launch("inverse_cdf_sampling");
}

extern "C" int psvo_ray_intersect_sorted(void *stream, int64_t n_rays, const float *rays_o, const float *rays_d,
                                         const float *centres, const int *structure, float voxel_size,
                                         float max_distance, float step_size, int *hit_idx, float *hit_t0,
                                         float *hit_t1, int *ray_nv, float *ray_dsum, int *stats) {
    PSVO_REQUIRE(n_rays >= 0, "ray_intersect_sorted: n_rays < 0");
    PSVO_REQUIRE(step_size > 0.0f && voxel_size > 0.0f, "ray_intersect_sorted: step/voxel must be > 0");
    if (n_rays == 0) return PSVO_OK;
    hipStream_t st = as_stream(stream);
    psvo::launch(k_intersect_sorted<false>, dim3(div_up(n_rays, kIsWaves)), dim3(kIsWaves * kWave), 0, st,
                       n_rays, rays_o, rays_d, centres, structure, nullptr, voxel_size, max_distance, step_size,
                       hit_idx, hit_t0, hit_t1, ray_nv, ray_dsum, stats, nullptr, nullptr, nullptr, nullptr, 0u,
                       nullptr, nullptr, LbCtl{});
    psvo::launch(k_ray_stats, dim3(1), dim3(1024), 0, st, n_rays, ray_nv, ray_dsum, step_size, stats);
    return check_launch("ray_intersect_sorted");
}

extern "C" int psvo_ray_intersect_sorted_packed(void *stream, int64_t n_rays, const float *rays_o, const float *rays_d,
                                                const void *packed, const float *centres, const int *structure,
                                                float voxel_size, float max_distance, float step_size, int *hit_idx,
                                                float *hit_t0, float *hit_t1, int *ray_nv, float *ray_dsum,
                                                int *stats) {
    PSVO_REQUIRE(n_rays >= 0, "ray_intersect_sorted_packed: n_rays < 0");
    PSVO_REQUIRE(step_size > 0.0f && voxel_size > 0.0f, "ray_intersect_sorted_packed: step/voxel must be > 0");
    PSVO_REQUIRE(packed && ((uintptr_t)packed & 15) == 0, "ray_intersect_sorted_packed: packed records (16-B aligned)");
    if (n_rays == 0) return PSVO_OK;
    hipStream_t st = as_stream(stream);
    // (the two-chunk walk: the same hits; the deep-tree parity tests run it here)
    psvo::launch(k_intersect_sorted<true, true>, dim3(div_up(n_rays, kIsWaves)), dim3(kIsWaves * kWave), 0, st,
                       n_rays, rays_o, rays_d, centres, structure, static_cast<const PackRec *>(packed), voxel_size,
                       max_distance, step_size, hit_idx, hit_t0, hit_t1, ray_nv, ray_dsum, stats, nullptr, nullptr,
                       nullptr, nullptr, 0u, nullptr, nullptr, LbCtl{});
    psvo::launch(k_ray_stats, dim3(1), dim3(1024), 0, st, n_rays, ray_nv, ray_dsum, step_size, stats);
    return check_launch("ray_intersect_sorted_packed");
}

namespace psvo {
// The statistics / rank pass and the sample scan: by default inside the
// traversal and sampler launches by decoupled look-back (lookback.h; up to
// kLbMaxRays rays: the packed pf / psm count granule); beyond that, and on
// the data-parallel sampler, as kernels of their own (k_ray_stats_rank,
// k_scan_samples).  The
// round-3 in-launch variant — the launch's last-arriving workgroup re-reading
// every ray — measured slower than the split kernels (one workgroup's
// dependent sc1 round trips) and is gone.
bool query_lookback(int64_t r) { return r > 0 && r <= kLbMaxRays; }
int64_t lookback_granules(int64_t r) {
    return lb_granules<kLbIsGranules>(div_up(r, kIsWaves)) + lb_granules<kLbSmpGranules>(div_up(r, kSmpWaves));
}
// the single-GPU sampler with the statistics read-back fused into its scan
// (one launch less before the host can size the rest of the step)
int sample_rays_to_host(hipStream_t st, int64_t r_hit_cap, int max_steps_cap, const int *rank_ray, const int *hit_idx,
                        const float *hit_t0, const float *hit_t1, const float *ray_dsum, float step_size,
                        const float *noise, uint64_t seed, int *stats, int *s_idx, float *s_depth, float *s_dist,
                        int *ray_ns, int *offsets, unsigned long long *host, int seq, const SampleCounts *counts, unsigned long long *lb_desc, uint32_t lb_tag, int *leaf,
                        float *t, int *ray_of, int *m_out, const int *nv_rank, const int *col0_rank) {
    PSVO_REQUIRE(r_hit_cap > 0 && max_steps_cap > 0 && offsets && ray_ns && host,
                 "sample_rays_to_host: bad arguments");
    PSVO_REQUIRE(!lb_desc || (r_hit_cap <= kLbMaxRays && lb_tag != 0), "sample_rays_to_host: look-back arguments");
    SampleTail tl{};
    if (counts) tl.c = *counts;
    tl.host = host;
    tl.seq = seq;
    if (lb_desc) {  // after the traversal's descriptors (lookback_granules)
        tl.offsets = offsets;
        tl.desc = lb_desc + lb_granules<kLbIsGranules>(div_up(r_hit_cap, kIsWaves));
        tl.tag = lb_tag;
        tl.ctl = lb_ctl(2);
        if (leaf && t && ray_of) {
            tl.leaf = leaf;
            tl.t = t;
            tl.ray_of = ray_of;
            tl.m_out = m_out;
        }
    }
    psvo::launch(k_sample_fused, dim3(div_up(r_hit_cap, kSmpWaves)), dim3(64 * kSmpWaves), 0, st, 0, -1, r_hit_cap, max_steps_cap,
                       rank_ray, hit_idx, hit_t0, hit_t1, ray_dsum, step_size, noise, seed, stats, s_idx, s_depth,
                       s_dist, ray_ns, nullptr, 0, tl, nv_rank, col0_rank);
    if (!lb_desc)
        psvo::launch(k_scan_samples, dim3(1), dim3(1024), 0, st, 0, -1, r_hit_cap, ray_ns, offsets, stats, 0,
                           host, seq, tl.c);
    return check_launch("sample_rays_to_host");
}

int stats_to_host(hipStream_t st, int *stats, unsigned long long *host, int words, int seq, bool zero) {
    psvo::launch(k_stats_to_host, dim3(1), dim3(64), 0, st, stats, host, words, seq, zero ? 1 : 0);
    return check_launch("stats_to_host");
}

// psvo_ray_intersect_sorted + psvo_hit_rank with the two single-block
// reductions fused into one launch (engine.cpp)
int intersect_ranked(hipStream_t st, int64_t n_rays, const float *rays_o, const float *rays_d, const float *centres,
                     const int *structure, float voxel_size, float max_distance, float step_size, int *hit_idx,
                     float *hit_t0, float *hit_t1, int *ray_nv, float *ray_dsum, int *stats, int *ray_rank,
                     int *rank_ray, const PackRec *packed, int *blk_out, unsigned long long *lb_desc,
                     uint32_t lb_tag, int *nv_rank, int *col0_rank, int64_t n_nodes) {
    PSVO_REQUIRE(n_rays >= 0, "intersect_ranked: n_rays < 0");
    PSVO_REQUIRE((nv_rank == nullptr) == (col0_rank == nullptr) && (!nv_rank || lb_desc),
                 "intersect_ranked: the by-rank copies come with the look-back pass");
    PSVO_REQUIRE(step_size > 0.0f && voxel_size > 0.0f, "intersect_ranked: step/voxel must be > 0");
    PSVO_REQUIRE(!lb_desc || (n_rays <= kLbMaxRays && lb_tag != 0), "intersect_ranked: look-back arguments");
    if (n_rays == 0) return PSVO_OK;
    // lb_desc: the statistics / rank pass inside the traversal launch (look-
    // back; the stats words are zero: memset / the last read-back)
    if (packed)
        psvo::launch(n_nodes >= kTwoChunkNodes ? k_intersect_sorted<true, true> : k_intersect_sorted<true, false>,
                     dim3(div_up(n_rays, kIsWaves)), dim3(kIsWaves * kWave), 0, st, n_rays, rays_o, rays_d, centres,
                     structure, packed, voxel_size, max_distance, step_size, hit_idx, hit_t0, hit_t1, ray_nv,
                     ray_dsum, stats, blk_out, ray_rank, rank_ray, lb_desc, lb_tag, nv_rank, col0_rank, lb_ctl(1));
    else
        psvo::launch(k_intersect_sorted<false>, dim3(div_up(n_rays, kIsWaves)), dim3(kIsWaves * kWave), 0, st,
                           n_rays, rays_o, rays_d, centres, structure, nullptr, voxel_size, max_distance, step_size,
                           hit_idx, hit_t0, hit_t1, ray_nv, ray_dsum, stats, blk_out, ray_rank, rank_ray, lb_desc,
                           lb_tag, nv_rank, col0_rank, lb_ctl(1));
    if (!lb_desc)
        psvo::launch(k_ray_stats_rank, dim3(1), dim3(1024), 0, st, n_rays, ray_nv, ray_dsum, step_size, stats,
                           ray_rank, rank_ray, blk_out, (int)div_up(n_rays, kIsWaves));
    return check_launch("intersect_ranked");
}
}  // namespace psvo

namespace psvo {
int dist_slot0_rows(int64_t max_rays_global) {
    const int64_t kp = (max_rays_global + kSamplerG - 1) / kSamplerG;
    return kSamplerG * (int)((kp + kSamplerChunk - 1) / kSamplerChunk);
}
int dist_count_words(int max_rays_rank) { return kDistWords + (max_rays_rank + 3) / 4; }
int dist_pack(hipStream_t st, int64_t R, const int *stats, const int *rank_ray, const int *hit_idx,
              const int *ray_nv, int *out, const int *nv_rank, int flags_or) {
    psvo::launch(k_dist_pack, dim3((int)div_up(div_up(R, 4), 256) + (R == 0)), dim3(256), 0, st, stats, rank_ray,
                 hit_idx, ray_nv, out, nv_rank, flags_or);
    return check_launch("dist_pack");
}
int dist_layout(hipStream_t st, const int *all, int world, int rank, int stride, int nch, int *stats, int *table,
                int *q2_in) {
    psvo::launch(k_dist_layout, dim3(1), dim3(256), 0, st, all, world, rank, stride, nch, stats, table, q2_in);
    return check_launch("dist_layout");
}
// the fused sampler + scan over this rank's rows (stats from dist_layout)
int dist_sample(hipStream_t st, int64_t r_hit_cap, int max_steps_cap, const int *rank_ray, const int *hit_idx,
                const float *hit_t0, const float *hit_t1, const float *ray_dsum, float step_size, uint64_t seed,
                int *stats, const int *table, int nch, int *s_idx, float *s_depth, float *s_dist, int *ray_ns,
                int *offsets, const int *nv_rank, const int *col0_rank) {
    if (r_hit_cap == 0) return PSVO_OK;
    psvo::launch(k_sample_fused, dim3(div_up(r_hit_cap, kSmpWaves)), dim3(64 * kSmpWaves), 0, st, 0, 0, r_hit_cap, max_steps_cap,
                       rank_ray, hit_idx, hit_t0, hit_t1, ray_dsum, step_size, nullptr, seed, stats, s_idx, s_depth,
                       s_dist, ray_ns, table, nch, SampleTail{}, nv_rank, col0_rank);
    psvo::launch(k_scan_samples, dim3(1), dim3(1024), 0, st, 0, 0, r_hit_cap, ray_ns, offsets, stats, 1,
                       nullptr, 0, SampleCounts{});
    return check_launch("dist_sample");
}
// the traversal's and sampler's helped-block counters (psvo_debug_lb_helps)
int lb_helps_query(int64_t *out2, bool reset) {
    unsigned long long h[2] = {0, 0};
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(h, HIP_SYMBOL(psvo_g_lb_helps), sizeof(h)) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "debug_lb_helps: copy failed");
    out2[0] = (int64_t)h[0];
    out2[1] = (int64_t)h[1];
    const unsigned long long z[2] = {0, 0};
    if (reset && hipMemcpyToSymbol(HIP_SYMBOL(psvo_g_lb_helps), z, sizeof(z)) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "debug_lb_helps: reset failed");
    return PSVO_OK;
}
int dist_smax(hipStream_t st, const int *all, int world, int *stats, int *in, double *sums) {
    psvo::launch(k_dist_smax, dim3(1), dim3(64), 0, st, all, world, stats, in, sums);
    return check_launch("dist_smax");
}
}  // namespace psvo

extern "C" int psvo_hit_rank(void *stream, int64_t n_rays, const int *ray_nv, int *ray_rank, int *rank_ray) {
    PSVO_REQUIRE(n_rays >= 0, "hit_rank: n_rays < 0");
    if (n_rays == 0) return PSVO_OK;
    psvo::launch(k_hit_rank, dim3(1), dim3(1024), 0, as_stream(stream), n_rays, ray_nv, ray_rank, rank_ray);
    return check_launch("hit_rank");
}

extern "C" int psvo_sample_rays_range(void *stream, int64_t row_begin, int64_t n_rows, int64_t r_hit_cap,
                                      int max_steps_cap, const int *rank_ray, const int *hit_idx,
                                      const float *hit_t0, const float *hit_t1, const float *ray_dsum,
                                      float step_size, const float *noise, uint64_t seed, int *stats, int *s_idx,
                                      float *s_depth, float *s_dist, int *ray_ns, int *offsets) {
    PSVO_REQUIRE(r_hit_cap >= 0 && max_steps_cap > 0, "sample_rays: bad caps");
    PSVO_REQUIRE(row_begin >= 0, "sample_rays: row_begin < 0");
    PSVO_REQUIRE(offsets != nullptr && ray_ns != nullptr, "sample_rays: ray_ns / offsets required");
    if (r_hit_cap == 0) return PSVO_OK;
    hipStream_t st = as_stream(stream);
    psvo::launch(k_sample_fused, dim3(div_up(r_hit_cap, kSmpWaves)), dim3(64 * kSmpWaves), 0, st, row_begin, n_rows, r_hit_cap,
                       max_steps_cap, rank_ray, hit_idx, hit_t0, hit_t1, ray_dsum, step_size, noise, seed, stats,
                       s_idx, s_depth, s_dist, ray_ns, nullptr, 0, SampleTail{}, static_cast<const int *>(nullptr),
                       static_cast<const int *>(nullptr));
    psvo::launch(k_scan_samples, dim3(1), dim3(1024), 0, st, row_begin, n_rows, r_hit_cap, ray_ns, offsets,
                       stats, 0, nullptr, 0, SampleCounts{});
    return check_launch("sample_rays");
}

extern "C" int psvo_sample_rays(void *stream, int64_t r_hit_cap, int max_steps_cap, const int *rank_ray,
                                const int *hit_idx, const float *hit_t0, const float *hit_t1, const float *ray_dsum,
                                float step_size, const float *noise, uint64_t seed, int *stats, int *s_idx,
                                float *s_depth, float *s_dist, int *ray_ns, int *offsets) {
    return psvo_sample_rays_range(stream, 0, -1, r_hit_cap, max_steps_cap, rank_ray, hit_idx, hit_t0, hit_t1,
                                  ray_dsum, step_size, noise, seed, stats, s_idx, s_depth, s_dist, ray_ns, offsets);
}

extern "C" int psvo_ray_stats(void *stream, int64_t n_rays, const int *ray_nv, const float *ray_dsum,
                              float step_size, int *stats) {
    PSVO_REQUIRE(n_rays >= 0 && step_size > 0.0f, "ray_stats: bad arguments");
    if (n_rays == 0) return PSVO_OK;
    psvo::launch(k_ray_stats, dim3(1), dim3(1024), 0, as_stream(stream), n_rays, ray_nv, ray_dsum, step_size,
                       stats);
    return check_launch("ray_stats");
}

extern "C" int psvo_scan_counts(void *stream, int64_t n, const int *counts, int *offsets) {
    PSVO_REQUIRE(n >= 0, "scan_counts: n < 0");
    psvo::launch(k_scan_counts, dim3(1), dim3(1024), 0, as_stream(stream), n, counts, offsets);
    return check_launch("scan_counts");
}

extern "C" int psvo_sample_points(void *stream, int64_t r_hit, int s_max, int max_steps_cap, const int *s_idx,
                                  const float *s_depth, const int *ray_ns, const int *offsets, int *leaf, float *t,
                                  int *ray_of_sample, float *z_vals, uint8_t *mask) {
    PSVO_REQUIRE(r_hit >= 0 && s_max >= 0 && s_max <= max_steps_cap, "sample_points: bad sizes");
    const int64_t total = r_hit * (int64_t)s_max;
    if (total == 0) return PSVO_OK;
    (void)ray_ns;
    const int bx = s_max <= 64 ? 64 : s_max <= 128 ? 128 : 256;
    const unsigned gy = (unsigned)(r_hit < 65535 ? r_hit : 65535);
    psvo::launch(k_sample_points, dim3(div_up(s_max, bx), gy), dim3(bx), 0, as_stream(stream), r_hit,
                       s_max, max_steps_cap, s_idx, s_depth, ray_ns, offsets, leaf, t, ray_of_sample, z_vals, mask);
    return check_launch("sample_points");
}

namespace psvo {
int compact_rays(hipStream_t st, int64_t r_hit, int cap, const int *s_idx, const float *s_depth, const int *offsets,
                 int *leaf, float *t, int *ray_of_sample) {
    PSVO_REQUIRE(r_hit >= 0 && cap > 0, "compact_rays: bad sizes");
    if (r_hit == 0) return PSVO_OK;
    psvo::launch(k_compact_rays, dim3(div_up(r_hit, 4)), dim3(256), 0, st, r_hit, cap, s_idx, s_depth, offsets,
                       leaf, t, ray_of_sample);
    return check_launch("compact_rays");
}

}  // namespace psvo

#ifdef PSVO_IS_STAMPS
extern "C" int psvo_debug_smp_stamps(void *dst, int64_t bytes) {
    if (bytes < (int64_t)sizeof(psvo::psvo_g_smp_stamps)) return -1;
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(psvo::psvo_g_smp_stamps), sizeof(psvo::psvo_g_smp_stamps)) ==
                   hipSuccess
               ? 0
               : -2;
}
extern "C" int psvo_debug_is_stamps(void *dst, int64_t bytes) {
    if (bytes < (int64_t)sizeof(psvo::psvo_g_is_stamps)) return -1;
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(psvo::psvo_g_is_stamps), sizeof(psvo::psvo_g_is_stamps)) == hipSuccess ? 0 : -2;
}
#endif
