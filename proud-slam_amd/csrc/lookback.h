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
// Progress (round 6): every wait is for a workgroup that is already resident.
// Round 5 waited for any lower-numbered workgroup, relying on the observed
// per-XCD in-order dispatch: a waiter on one XCD could spin on a lower
// workgroup of another XCD that was still queued behind another queue's
// kernels — two processes sharing one GPU (the reference's tracker + mapper
// deployment, the 2-rank data-parallel test) each filled CUs with waiters
// for workgroups the other one's waiters kept out (r05aj: `query look-back
// wait abandoned` after 2^16 re-reads).  Now each workgroup stores a STARTED
// granule {tag} as its first act.  A waiter that still misses a predecessor's
// aggregate after kLbHelpAfterUs of waiting checks that predecessor's started
// granule: if it has started, its aggregate follows its own work, which
// depends on nothing (keep waiting); if it has not, the waiter computes that
// workgroup's aggregate itself — the same deterministic per-item work on the
// same inputs, so the same bits — and publishes it (lb_scan_help returns the
// block to help; the caller's whole workgroup runs that block's items).  A
// missing tile total whose producer (the tile's last workgroup) has not
// started is summed by the waiter from the tile's aggregates, helping where
// needed.  So every wait ends whatever the dispatch order, the workgroup→XCD
// placement or what else holds the CUs, at no cost to the common case (one
// store per workgroup; a same-address ticket per workgroup, tried first,
// cost 1.5–6 µs per launch: 512 arrivals serialise at ≈ 11 ns each).  Items a
// helper computes are written again by their owner when it runs (the same
// bits); prefix-dependent outputs are written by each block's owner only.
// kLbSpinMax is a bug trap: lb_scan_help returns kLbFail after kLbSpinMax
// re-reads (≳ 0.3 s); the caller raises PSVO_STAT_FLAGS bit 3, stores no
// rank / offset / compacted sample from the undefined prefix, and the engine
// reports the batch as failed — the grid still drains.
// The help threshold is time, not re-reads: a predecessor that starts late
// because the CUs are briefly full (the draw, the decoder's prep kernels on
// other streams) is waited for — helping is the slow path (the traversal's
// help is a serial walk per ray: config E's traversal took 64 → 140 µs per
// launch with help after 16 re-reads, profiles/r06l_*); only a predecessor
// kept out for 100 µs — another queue holding the CUs — is helped.
#pragma once
#include "psvo_common.h"

namespace psvo {

constexpr int kLbSpinMax = 1 << 18;
constexpr int kLbHelpAfter = 16;   // re-reads between checks of the missing producers' started granules
constexpr uint64_t kLbHelpAfterTicks = 10000;  // kLbHelpAfterUs = 100 µs of waiting (s_memrealtime: 100 MHz)
constexpr int kLbFlagTimeout = 8;  // PSVO_STAT_FLAGS bit 3
constexpr int kLbDone = -1, kLbFail = -2;  // lb_scan_help's results (≥ 0: the block to help)

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

// Workgroup b's exclusive prefix over the nb workgroups of the launch, in
// two levels of 64: b publishes its aggregate A[b]; it sums the aggregates
// of the workgroups in front of it in its tile of 64 (one round of loads);
// the tile's last workgroup publishes the tile's total T[b / 64]; b adds the
// totals of the tiles in front of its own (one more round).  After the last
// aggregate lands the prefixes are two load rounds away — a one-level
// look-back walks up to nb / 64 dependent rounds when the workgroups finish
// together (measured: +7 µs for 1,024 traversal workgroups, +21 µs for 1,024
// sampler workgroups).
// desc: [nb][NG] aggregates, [nb / 64 rounded up][NG] tile totals, [nb]
// started granules.
constexpr int kLbMaxBlocks = kWave * kWave;

template <int NG>
__host__ __device__ constexpr int64_t lb_granules(int64_t nb) {
    return (nb + (nb + kWave - 1) / kWave) * NG + nb;
}

template <int NG>
__device__ __forceinline__ unsigned long long *lb_started_of(unsigned long long *desc, int nb) {
    return desc + (size_t)(nb + (nb + kWave - 1) / kWave) * NG;
}

// workgroup b's first act (one lane): its started granule
template <int NG>
__device__ __forceinline__ void lb_mark_started(unsigned long long *desc, int b, int nb, uint32_t tag) {
    __hip_atomic_store((g_u64 *)(lb_started_of<NG>(desc, nb) + b), (unsigned long long)tag << 32, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// Wait until lanes [0, n) of the calling wave have read their granules
// src[lane·NG + g] tagged `tag`, then reduce them over the wave into `red`
// (every lane).  Lane i's granules come from workgroup producer0 + i·pstride
// (capped at nb − 1).  Returns kLbDone; the lowest producer of a missing
// granule that has not started after kLbHelpAfterTicks of waiting (the
// caller helps it); or kLbFail after spin_max re-reads (the bug trap; tests:
// 0 = at once).
template <int NG, unsigned MAXMASK>
__device__ __forceinline__ int lb_gather(const unsigned long long *src, int n, uint32_t tag, int lane,
                                         uint32_t (&red)[NG], const unsigned long long *started, int producer0,
                                         int pstride, int nb, int &spins, int spin_max) {
    uint32_t v[NG];
    int rc = kLbDone;
    uint64_t t_wait = 0;  // when this gather first missed a granule
    for (;; ++spins) {
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
        const uint64_t missing = __ballot(!mine);
        if (missing == 0) break;
        if (spins + 1 >= spin_max) {
            rc = kLbFail;
            break;
        }
        if (t_wait == 0) t_wait = __builtin_amdgcn_s_memrealtime();
        if ((spins & (kLbHelpAfter - 1)) == kLbHelpAfter - 1 &&
            __builtin_amdgcn_s_memrealtime() - t_wait >= kLbHelpAfterTicks) {
            // which of the missing producers have not started
            const int p = min(producer0 + lane * pstride, nb - 1);
            bool unstarted = false;
            if (!mine) {
                const unsigned long long s = __hip_atomic_load((g_u64 *)(started + p), __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT);
                unstarted = (uint32_t)(s >> 32) != tag;
            }
            const uint64_t u = __ballot(unstarted);
            if (u) {
                rc = min(producer0 + (int)(__ffsll((unsigned long long)u) - 1) * pstride, nb - 1);
                break;
            }
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
    return rc;
}

// Workgroup b's exclusive prefix `ex` (uniform over the calling wave, which
// must be whole; nb <= kLbMaxBlocks), its aggregate `agg` published first.
// Returns kLbDone (ex valid), kLbFail (bug trap: ex undefined) or a block
// q ≥ 0 whose aggregate the caller must compute and publish (lb_publish)
// before calling again — re-entrant: a repeated call re-reads what landed.
template <int NG, unsigned MAXMASK>
__device__ __forceinline__ int lb_scan_help(unsigned long long *desc, int b, int nb, uint32_t tag, int lane,
                                            const uint32_t (&agg)[NG], uint32_t (&ex)[NG], int &spins,
                                            int spin_max = kLbSpinMax) {
    unsigned long long *tiles = desc + (size_t)nb * NG;
    const unsigned long long *started = lb_started_of<NG>(desc, nb);
    const int t = b / kWave, b0 = t * kWave;
    lb_store<NG>(desc + (size_t)b * NG, lane, agg, tag);
    uint32_t e1[NG], e2[NG];
    if (spin_max == 0 && b > 0) return kLbFail;  // tests: give up at once (psvo_debug_set_lb_spin bound 0)
    int rc = lb_gather<NG, MAXMASK>(desc + (size_t)b0 * NG, b - b0, tag, lane, e1, started, b0, 1, nb, spins,
                                    spin_max);
    if (rc != kLbDone) return rc;
    if (b - b0 == kWave - 1 || b == nb - 1) {  // the tile's total
        uint32_t tot[NG];
#pragma unroll
        for (int g = 0; g < NG; ++g) tot[g] = lb_comb<MAXMASK>(g, e1[g], agg[g]);
        lb_store<NG>(tiles + (size_t)t * NG, lane, tot, tag);
    }
    for (;;) {  // the tile totals in front: a missing one whose producer has not started is summed here
        rc = lb_gather<NG, MAXMASK>(tiles, t, tag, lane, e2, started, kWave - 1, kWave, nb, spins, spin_max);
        if (rc < 0) break;
        const int tt = rc / kWave;  // the tile of the unstarted producer (its last workgroup)
        uint32_t tot[NG];
        rc = lb_gather<NG, MAXMASK>(desc + (size_t)tt * kWave * NG, min(kWave, nb - tt * kWave), tag, lane, tot,
                                    started, tt * kWave, 1, nb, spins, spin_max);
        if (rc != kLbDone) return rc;
        lb_store<NG>(tiles + (size_t)tt * NG, lane, tot, tag);
    }
    if (rc != kLbDone) return rc;
#pragma unroll
    for (int g = 0; g < NG; ++g) ex[g] = lb_comb<MAXMASK>(g, e2[g], e1[g]);
    return kLbDone;
}

// per-launch look-back controls: the spin bound (kLbSpinMax; tests: smaller)
// and, tests only, a start delay for some workgroups (every 4th from 1 and
// every tile's last) that makes their successors help them
struct LbCtl {
    int spin_max;
    int delay_us;
};
__device__ __forceinline__ void lb_debug_delay(const LbCtl &c, int b) {
    if (c.delay_us > 0 && ((b & 3) == 1 || (b & (kWave - 1)) == kWave - 1)) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
        while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)c.delay_us * 100u) __builtin_amdgcn_s_sleep(127);
    }
}

// a helped block's aggregate (lanes [0, NG) of the calling wave)
template <int NG>
__device__ __forceinline__ void lb_publish(unsigned long long *desc, int q, int lane, const uint32_t (&agg)[NG],
                                           uint32_t tag) {
    lb_store<NG>(desc + (size_t)q * NG, lane, agg, tag);
}

}  // namespace psvo
