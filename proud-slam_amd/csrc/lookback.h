// Single-pass workgroup scan by two-level look-back (MI355X: per-XCD L2s are
// not coherent, so every descriptor word crosses dies as an 8-byte granule).
//
// The query's two reductions over all rays of a batch — the hit-ray ranks
// with P / R_hit / max ⌈Σ/step⌉ (after the traversal) and the sample offsets
// with S_max / M and the loss normaliser counts (after the sampler) — used to
// be single-workgroup kernels of their own (k_ray_stats_rank, k_scan_samples)
// or the work of the launch's last-arriving workgroup (one workgroup reading
// every ray's value back, plus a same-address ticket per workgroup).  Here
// every workgroup of the producing launch publishes its aggregate, learns its
// exclusive prefix from its predecessors' descriptors and writes its own
// ranks / offsets; the workgroup holding the last item writes the totals.
//
// Descriptors: per workgroup (and per tile of 64 workgroups) NG granules
// {u32 value, u32 tag}, each written by ONE
// 8-byte agent-scope store (write-through: no release fence) and read with
// 8-byte agent-scope loads (sc1: past this CU's L1 and the non-coherent L2).
// A granule is valid when its tag equals the launch's tag: the host hands
// every launch a fresh tag, so the buffer never needs clearing.  Fields
// combine by sum, or by max where bit g of MAXMASK is set (all values ≥ 0,
// 0 is the identity of both).
//
// Progress: a workgroup waits only for lower-numbered workgroups.  On a
// multi-XCD part the workgroups are dealt round-robin to the XCDs and each
// XCD dispatches its share in index order, so on every XCD the lowest
// unfinished workgroup is resident once it holds a slot; a waiter can still
// spin while a lower workgroup of another XCD is queued behind a co-running
// kernel (e.g. the width-256 dW kernel at one workgroup per CU) — the wait
// then lasts as long as that kernel holds the CUs.  A wait that never ends
// (a bug) is abandoned after kLbSpinMax re-reads (≳ 1 s; 2^16, ≳ 65 ms, was
// reached once by two processes sharing one GPU in the data-parallel test —
// the other process's kernels held the CUs a queued lower workgroup needed
// for that long): lb_scan returns
// false, the caller raises PSVO_STAT_FLAGS bit 3, stores no rank / offset /
// compacted sample from the undefined prefix, and the engine reports the
// batch as failed — the grid still drains.
#pragma once
#include "psvo_common.h"

namespace psvo {

constexpr int kLbSpinMax = 1 << 20;
constexpr int kLbFlagTimeout = 8;  // PSVO_STAT_FLAGS bit 3

template <unsigned MAXMASK>
__device__ __forceinline__ uint32_t lb_comb(int g, uint32_t a, uint32_t b) {
    return ((MAXMASK >> g) & 1u) ? (a > b ? a : b) : a + b;
}

// lanes [0, NG) of the calling wave store granules g = lane of v (uniform)
template <int NG>
__device__ __forceinline__ void lb_store(unsigned long long *d, int lane, const uint32_t (&v)[NG], uint32_t tag) {
    uint32_t x = 0;
#pragma unroll
    for (int g = 0; g < NG; ++g)
        if (lane == g) x = v[g];
    if (lane < NG)
        __hip_atomic_store((g_u64 *)(d + lane), ((unsigned long long)tag << 32) | x, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// Wait until lanes [0, n) of the calling wave have read their granules
// src[lane·NG + g] tagged `tag`, then reduce them over the wave into `red`
// (every lane).  One round of independent loads per attempt; false: given up
// after kLbSpinMax attempts (`red` is then what the last attempt read).
template <int NG, unsigned MAXMASK>
__device__ __forceinline__ bool lb_gather(const unsigned long long *src, int n, uint32_t tag, int lane,
                                          uint32_t (&red)[NG]) {
    bool ok = true;
    uint32_t v[NG];
    for (int spins = 0;; ++spins) {
        bool mine = true;
#pragma unroll
        for (int g = 0; g < NG; ++g) v[g] = 0;
        if (lane < n) {
            unsigned long long q[NG];
#pragma unroll
            for (int g = 0; g < NG; ++g)
                q[g] = __hip_atomic_load((g_u64 *)(src + (size_t)lane * NG + g), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                v[g] = (uint32_t)q[g];
                mine = mine && (uint32_t)(q[g] >> 32) == tag;
            }
        }
        if (__ballot(!mine) == 0) break;
        if (spins + 1 >= kLbSpinMax) {
            ok = false;
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        uint32_t c = v[g];
#pragma unroll
        for (int sh = kWave / 2; sh > 0; sh >>= 1) c = lb_comb<MAXMASK>(g, c, (uint32_t)__shfl_xor((int)c, sh, kWave));
        red[g] = c;
    }
    return ok;
}

// Workgroup b's exclusive prefix `ex` over the nb workgroups of the launch
// (uniform over the calling wave, which must be whole; nb <= kLbMaxBlocks),
// in two levels of 64: b publishes its aggregate A[b]; it sums the aggregates
// of the workgroups in front of it in its tile of 64 (one round of loads);
// the tile's last workgroup publishes the tile's total T[b / 64]; b adds the
// totals of the tiles in front of its own (one more round).  Every wait is on
// lower-numbered workgroups, and after the last aggregate lands the prefixes
// are two load rounds away — a one-level look-back walks up to nb / 64
// dependent rounds when the workgroups finish together (measured: +7 µs for
// 1,024 traversal workgroups, +21 µs for 1,024 sampler workgroups).
// desc: [nb][NG] aggregates, then [nb / 64 rounded up][NG] tile totals.
constexpr int kLbMaxBlocks = kWave * kWave;

template <int NG>
__host__ __device__ constexpr int64_t lb_granules(int64_t nb) {
    return (nb + (nb + kWave - 1) / kWave) * NG;
}

template <int NG, unsigned MAXMASK>
__device__ __forceinline__ bool lb_scan(unsigned long long *desc, int b, int nb, uint32_t tag, int lane,
                                        const uint32_t (&agg)[NG], uint32_t (&ex)[NG]) {
    unsigned long long *tiles = desc + (size_t)nb * NG;
    const int t = b / kWave, b0 = t * kWave;
    lb_store<NG>(desc + (size_t)b * NG, lane, agg, tag);
    uint32_t e1[NG], e2[NG];
    bool ok = lb_gather<NG, MAXMASK>(desc + (size_t)b0 * NG, b - b0, tag, lane, e1);
    if (b - b0 == kWave - 1 || b == nb - 1) {  // the tile's total
        uint32_t tot[NG];
#pragma unroll
        for (int g = 0; g < NG; ++g) tot[g] = lb_comb<MAXMASK>(g, e1[g], agg[g]);
        lb_store<NG>(tiles + (size_t)t * NG, lane, tot, tag);
    }
    ok = lb_gather<NG, MAXMASK>(tiles, t, tag, lane, e2) && ok;
#pragma unroll
    for (int g = 0; g < NG; ++g) ex[g] = lb_comb<MAXMASK>(g, e2[g], e1[g]);
    return ok;
}

}  // namespace psvo
