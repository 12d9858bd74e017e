// Native mapping-iteration engine: one C call runs a whole render-and-optimise
// iteration of the mapping loop (render_helpers.py:609-672 — render_rays,
// Criterion, loss.backward(), Adam(embeddings).step(), Adam(decoder).step())
// on one HIP stream: 24 kernel launches, two 32-byte stats read-backs that
// size the sample buffers, no host allocation after warm-up.  It strings
// together the same C-ABI entry points the PyTorch autograd path calls, so
// the two paths compute the same numbers; what it removes is the Python /
// autograd / allocator time between launches, which otherwise leaves the GPU
// idle behind every read-back.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <cmath>

#include <utility>
#include <vector>

#include "psvo_common.h"
#include "lookback.h"

namespace psvo {
namespace {

// buffers of one query (intersection + sampling of a ray batch): a query set
enum QSlot { kStats, kHitIdx, kHitT0, kHitT1, kRayNv, kRayDsum, kRayRank, kRankRay, kSIdx, kSDepth, kSDist, kRayNs,
             kOffsets, kBlkOut, kRayCnt, kCoefQ, kLbDesc, kLeafQ, kTQ, kRayOfQ, kDistSums, kMDev, kNvRank, kCol0Rank,
             kQSlots };
// buffers of the rest of a step
enum Slot {
    kLeaf, kT, kRayOf, kZ, kMask, kFeat, kImages, kSdfS, kRgbS, kAct, kMasks, kSdf, kWeights, kColor,
    kDepth, kZmin, kCritWs, kSums, kGLoss, kGColor, kGDepth, kGSdf, kGSdfS, kGRgbS, kMlpWs, kDfeat, kDecGrad,
    kGradEmb, kGradOD, kRaysO, kRaysD, kDTmp, kPoseGrad, kSumsC, kCoef, kIbWs,
    // the sparse decoder (select_samples): compact index, ray offsets, the kept samples' rows, counts, look-back
    kCidx, kOffB, kFeatB, kLeafB, kTB, kRayOfB, kSdfB, kSelCnt, kSelDesc,
    // its class B (the trunk only): ray offsets, activations and masks
    kOffB2, kH2, kSrcC, kSlots
};

struct Arena {
    void *p[kSlots] = {};
    size_t cap[kSlots] = {};
    uint32_t gen[kSlots] = {};  // allocations made for the slot (a new buffer may reuse a freed base address)
};

// One ray batch's query: its buffers, the pinned statistics it reads back
// and the events that order it against the steps.  psvo_map_query runs a
// query on the engine's side stream one step ahead (the query depends only on
// the rays and the octree, not on the embeddings / decoder the running step
// updates), so the step that consumes it finds its sizes already on the host.
struct QuerySet {
    Arena a;                      // slots kStats..kOffsets
    // coherent pinned {seq, value} granules: PSVO_STAT_WORDS for the read-back
    // after the sampler, PSVO_STAT_WORDS more for a data-parallel query's second
    unsigned long long *host_raw = nullptr;
    int host_stats[PSVO_STAT_WORDS] = {};     // the values of the last statistics that landed
    int seq = 0;                  // the flag value the current statistics carry
    hipStream_t qstream = nullptr;  // the stream the query was queued on
    const int *stats_zeroed = nullptr;  // the device statistics buffer a completed read-back left zeroed
    uint32_t lb_zero_gen = 0;           // the look-back descriptor allocation (Arena::gen) last zeroed (tags ≠ 0)
    bool compacted = false;             // the sampler compacted the samples (slots kLeafQ / kTQ / kRayOfQ)
    hipEvent_t done = nullptr;    // statistics landed (after the sampler)
    bool done_recorded = false;   // a query consumed on its own stream skips it (one packet less there)
    hipEvent_t freed = nullptr;   // the consuming step finished with the buffers
    bool freed_recorded = false;
    hipStream_t freed_on = nullptr;  // the stream `freed` was recorded on (a wait on that stream is implied)
    bool freed_lazy = false;         // released on freed_on, event not recorded yet (a consumer on
                                     // another stream records it then: a later point of freed_on)
    bool pending = false;
    int64_t R = 0;
    const float *ro = nullptr, *rd = nullptr;
    const float *dirs = nullptr;  // a psvo_map_step_frames look-ahead: the camera directions it was made from
    // the GT depths the sampler counted the Criterion's normalisers with
    // (coefficients in slot kCoefQ), or null: the step computes them itself
    const float *counts_gt = nullptr;
    uint64_t seed = 0;
    int max_steps = 0;
    // data parallel: the query's second half — dist_counts → the all-gather of
    // [S_max, count words] → dist_smax → the second read-back — on the
    // engine's q2 stream, issued by the step once its interpolation and sdf
    // trunk are queued (query_phase2), so it runs beside them instead of on
    // the pose → traversal → sampler → interpolation chain
    hipEvent_t p1 = nullptr;     // the first read-back's kernel done (bound to its dispatch)
    hipEvent_t done2 = nullptr;  // the second read-back done
    bool p2_pending = false;     // queued first half, second half not issued yet
    const float *p2_gt = nullptr;
    float p2_tr = 0.f, p2_max_depth = 0.f;
};

}  // namespace
}  // namespace psvo

// optional HIP-event timing of the roofline regions (PSVO_TIME_*)
struct EngineTimer {
    bool on = false;
    bool overlap = false;  // mode 2: events on the streams the regions run on, side streams kept
    bool pending = false;  // events of the last step not yet read
    bool markers = false;  // PSVO_TIMING_MARKERS=1: marker events around each region (the old timing)
    unsigned used = 0;     // regions the last step marked (a step may skip one: no compaction kernel)
    hipEvent_t ev[PSVO_TIME_REGIONS][2] = {};
    double ms[PSVO_TIME_REGIONS] = {};
    int64_t n[PSVO_TIME_REGIONS] = {};
    // kernel-bound timing (the default): the regions' kernels' own spans
    psvo::KernelClock kc;
    double kms[PSVO_TIME_REGIONS] = {};     // Σ kernel spans collected
    int64_t starts[PSVO_TIME_REGIONS] = {};  // region instances queued (a region's time = kms / starts)
};

// Data-parallel exchange (psvo_engine_set_exchange): the caller's collective
// callback and the device buffers it operates on.
struct EngineExchange {
    psvo_exchange_fn fn = nullptr;
    void *user = nullptr;
    int rank = 0, world = 1;
    int nch = 1;               // launch chunks the slot-0 table covers
    int cw = 8;                // words per rank of the query's first gather (dist_count_words(max_rays_rank))
    int64_t max_rays_rank = 0;
    int *xi32 = nullptr;       // psvo_engine_exchange_words(world, max_rays_global, max_rays_rank) int32
    double *xf64 = nullptr;    // 16 doubles: [0, 8) count sums, [8, 16) loss sums
    bool on() const { return fn != nullptr; }  // world 1 included: the one-rank protocol (tests)
    // int32 word offsets: [first gather: in | all ranks] [second gather: in | all ranks] [slot-0 count table]
    int64_t in_off() const { return 0; }
    int64_t all_off() const { return cw; }
    int64_t q2_in_off() const { return all_off() + (int64_t)world * cw; }
    int64_t q2_all_off() const { return q2_in_off() + psvo::kDistWordsPerRank; }
    int64_t table_off() const { return (q2_all_off() + (int64_t)world * psvo::kDistWordsPerRank + 63) / 64 * 64; }
    int64_t table_words() const { return (int64_t)psvo::kSamplerG * nch; }
    int call(int op, int64_t in, int64_t out, int64_t count, hipStream_t st, const char *what) const {
        const int rc = fn(user, op, in, out, count, st);
        if (rc != 0) return psvo::set_error(PSVO_E_LAUNCH, "exchange (%s) failed with %d", what, rc);
        return PSVO_OK;
    }
};

// psvo_engine_set_clock: an event on the caller's stream at the entry of
// every mapping step — the GPU reaches it when the previous step's work on
// that stream (through the look-ahead query) is done, so consecutive events
// are the iteration period as the GPU runs it
struct EngineClock {
    std::vector<hipEvent_t> ev;
    int n = 0;
    bool on = false;
};

struct psvo_engine {
    EngineExchange x;
    EngineClock clk;
    psvo::Arena a;
    psvo::QuerySet qs[2];           // FIFO of queries: head = the next step's
    int q_head = 0, q_count = 0;
    uint32_t lb_tag = 0;            // the last look-back descriptor tag handed out (lookback.h)
    hipStream_t side = nullptr;     // psvo_map_query's stream
    hipStream_t q2s = nullptr;      // data parallel: the queries' second halves (QuerySet::p2_pending)
    hipEvent_t in_ready = nullptr;  // the caller's stream position at psvo_map_query
    // the embedding backward runs on `aux` beside the decoder's weight
    // gradients (k_interp_bwd's 8-KB workgroups fit next to k_mlp_dw2's 152 KB)
    // (and the loss normalisers beside the decoder forward; data parallel,
    // also the loss value beside the decoder backward)
    hipStream_t aux = nullptr;
    // single GPU: the loss value (one-wave reduction, slow beside the
    // persistent decoder kernels) on its own stream, so it delays neither the
    // embedding backward on aux nor anything on the caller's stream
    hipStream_t lossq = nullptr;
    hipEvent_t dfeat_ready = nullptr, emb_done = nullptr, z_ready = nullptr, coef_ready = nullptr,
               grads_ready = nullptr, prep_fork = nullptr, prep_done = nullptr, loss_done = nullptr;
    // a look-ahead step's tail split (map_step_impl): the weight-gradient sum,
    // the optimiser step and the next decoder images on aux, while st runs the
    // pose step and the next query; every later reader of the weights on st
    // waits for adam_done first (render, before the interpolation)
    hipEvent_t adam_done = nullptr;
    bool bwd_recorded = false;     // dfeat_ready holds a step's decoder backward end (psvo_map_side_wait)
    bool adam_pending = false;
    hipEvent_t next_ready = nullptr;  // psvo_map_frames.next_stream's position at the call
    hipEvent_t draw_gate = nullptr;   // the last step's sample selection done (psvo_engine_gate_stream)
    hipEvent_t draw_gate_ev = nullptr;  // the event that marks it: draw_gate, or a timed step's clock event
    bool draw_gate_recorded = false;
    bool draw_gate_used = false;      // a caller gates on it: bind it to the selections from now on
    EngineTimer tm;
    // the decoder images a look-ahead step built on st after its Adam step,
    // for the decoder whose W[0] it names; consumed by the next
    // psvo_map_step_frames, dropped by every other call
    bool images_next = false;
    const float *images_w0 = nullptr;
    int paths = 0;                  // PSVO_PATH_* (psvo_engine_set_paths)
    int64_t m_early = 0;            // the device-sized forward's capacity (render): 1.25 × the largest M seen
    uint32_t sel_tag = 0;           // the sample selection's look-back descriptor tag
    uint32_t sel_zero_gen = 0;      // its descriptor allocation (Arena::gen) last zeroed
    int *host_flags = nullptr;      // coherent pinned: bit 3 = a sample selection gave up its look-back wait
    bool grads_clean = false;       // embedding-gradient buffer known to be zero (Adam zeroes it)
    const float *clean_buf = nullptr;  // ... and which buffer that is
};

using namespace psvo;

#define ENG_CALL(x)                     \
    do {                                \
        const int _rc = (x);            \
        if (_rc != PSVO_OK) return _rc; \
    } while (0)

namespace psvo {
thread_local KernelClock *g_kclock = nullptr;
}

namespace {

// device buffer of at least `bytes` for `slot`; growing synchronises the
// stream first (the old buffer may still be read by queued kernels)
void *arena_buf(Arena &a, hipStream_t st, int slot, size_t bytes, int *rc) {
    if (bytes == 0) bytes = 16;
    if (a.cap[slot] >= bytes) return a.p[slot];
    if (a.p[slot]) {
        (void)hipStreamSynchronize(st);
        (void)hipFree(a.p[slot]);
        a.p[slot] = nullptr;
        a.cap[slot] = 0;
    }
    const size_t cap = bytes + bytes / 4;  // headroom against per-step size jitter
    if (hipMalloc(&a.p[slot], cap) != hipSuccess) {
        *rc = set_error(PSVO_E_LAUNCH, "engine: hipMalloc(%zu) failed", cap);
        return nullptr;
    }
    a.cap[slot] = cap;
    a.gen[slot]++;
    return a.p[slot];
}

void *slot_buf(psvo_engine *e, hipStream_t st, int slot, size_t bytes, int *rc) {
    return arena_buf(e->a, st, slot, bytes, rc);
}

// block = false: only the pairs whose kernels have finished (a timed step's
// host must not wait for kernels it queued ahead); the rest move to the front
void timer_collect(psvo_engine *e, bool block = false) {
    EngineTimer &t = e->tm;
    if (!t.markers) {  // kernel-bound
        psvo::KernelClock &c = t.kc;
        auto ready = [&](hipEvent_t ev) {
            const hipError_t q = block ? hipEventSynchronize(ev) : hipEventQuery(ev);
            if (q == hipErrorNotReady && hipPeekAtLastError() == hipErrorNotReady) (void)hipGetLastError();  // not an error
            return q;
        };
        if (c.sum) {
            int w = 0;
            for (int i = 0; i < c.n; ++i) {
                const hipError_t q = ready(c.ev[i][1]);
                if (q == hipErrorNotReady) {
                    if (w != i) {
                        std::swap(c.ev[w][0], c.ev[i][0]);
                        std::swap(c.ev[w][1], c.ev[i][1]);
                        c.region[w] = c.region[i];
                    }
                    ++w;
                    continue;
                }
                float ms = 0.f;
                if (q == hipSuccess && hipEventElapsedTime(&ms, c.ev[i][0], c.ev[i][1]) == hipSuccess)
                    t.kms[c.region[i]] += ms;
                else
                    (void)hipGetLastError();  // not the next launch's error
            }
            c.n = w;
        } else {
            // closed instances in queue order; an unfinished one ends this pass
            // (its pairs and the later ones' stay until a later collection)
            int done = 0;
            for (; done < c.n_inst; ++done) {
                const psvo::KernelClock::Inst &I = c.inst[done];
                bool open = false;
                for (int d = 0; d < c.depth; ++d) open |= c.stack[d] == done;
                if (open) break;
                if (I.first < 0) continue;  // no kernel: the region's instance counts 0
                const hipError_t q = ready(c.ev[I.last][1]);
                if (q == hipErrorNotReady) break;
                float ms = 0.f;
                if (q == hipSuccess && hipEventElapsedTime(&ms, c.ev[I.first][0], c.ev[I.last][1]) == hipSuccess)
                    t.kms[I.region] += ms;
                else
                    (void)hipGetLastError();
            }
            if (done > 0) {  // drop the collected instances (the open ones keep their stack slots)
                for (int k = done; k < c.n_inst; ++k) c.inst[k - done] = c.inst[k];
                c.n_inst -= done;
                for (int d = 0; d < c.depth; ++d) c.stack[d] -= done;
            }
            if (c.n_inst == 0) c.n = 0;  // every pair read: the slots start over
        }
        t.pending = false;
        return;
    }
    if (!t.pending) return;
    for (int r = 0; r < PSVO_TIME_REGIONS; ++r) {
        if (!(t.used & (1u << r))) continue;  // never recorded: reading it would leave a sticky HIP error
        float ms = 0.f;
        if (hipEventSynchronize(t.ev[r][1]) == hipSuccess && hipEventElapsedTime(&ms, t.ev[r][0], t.ev[r][1]) == hipSuccess) {
            t.ms[r] += ms;
            t.n[r] += 1;
        } else {
            (void)hipGetLastError();  // not the next launch's error
        }
    }
    t.used = 0;
    t.pending = false;
}

inline void mark(psvo_engine *e, hipStream_t st, int region, int end) {
    EngineTimer &t = e->tm;
    if (!t.on) return;
    if (t.markers) {
        (void)hipEventRecord(t.ev[region][end], st);
        if (end) t.used |= 1u << region;
        return;
    }
    psvo::KernelClock &c = t.kc;
    if (!end) {
        if (c.n + 32 > psvo::KernelClock::kMax || c.n_inst + 2 > psvo::KernelClock::kMaxInst)
            timer_collect(e, true);  // room for the region's kernels
        t.starts[region] += 1;
        psvo::g_kclock = &c;
        c.streams[0] = st;  // the region's stream and the engine's side streams
        c.streams[1] = e->aux;
        c.streams[2] = e->lossq;
        c.streams[3] = e->side;
        if (c.depth >= 8) {
            c.overflow = true;
            return;
        }
        if (c.sum) {
            c.stack[c.depth++] = region;
        } else if (c.n_inst < psvo::KernelClock::kMaxInst) {
            c.inst[c.n_inst] = psvo::KernelClock::Inst{region, -1, -1};
            c.stack[c.depth++] = c.n_inst++;
        } else {
            c.overflow = true;
        }
    } else if (c.depth > 0) {
        c.depth--;
    }
}

// st waits for a split tail's optimiser step (map_step_impl) if one is pending
inline double now_ns() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e9 + t.tv_nsec;
}
// host_wait_us > 0: first poll the event from the host for up to that long
// (the device-sized forward is queued while the query still runs: a host
// that waits for the optimiser here keeps the cross-queue barrier — ≈ 20 µs
// of idle GPU between the sampler and the interpolation, measured — out of
// the stream)
int join_adam(psvo_engine *e, hipStream_t st, const char *who, double host_wait_us = 0.0) {
    if (!e->adam_pending) return PSVO_OK;
    // already done (the usual case: the optimiser step ran beside the query):
    // no barrier packet in front of the interpolation — the command processor
    // resolves even a satisfied cross-queue wait with a few µs of latency
    hipError_t q = hipEventQuery(e->adam_done);
    if (q == hipErrorNotReady && host_wait_us > 0.0) {
        const double t_end = now_ns() + host_wait_us * 1e3;
        while (q == hipErrorNotReady && now_ns() < t_end) q = hipEventQuery(e->adam_done);
    }
    if (q == hipSuccess) {
        e->adam_pending = false;
        return PSVO_OK;
    }
    if (q == hipErrorNotReady && hipPeekAtLastError() == hipErrorNotReady) (void)hipGetLastError();  // not an error
    if (hipStreamWaitEvent(st, e->adam_done, 0) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "%s: stream wait failed", who);
    e->adam_pending = false;
    return PSVO_OK;
}

// The host spins on the statistics granules the device writes (each word
// tagged with the query's seq, relaxed system-scope stores: stat_to_host) —
// it sees them as soon as they land, without the event's completion-signal
// round trip and without a system-scope release on the device; the event
// recorded after that kernel (or, without one, the query's stream) is still
// queried now and then so a failed stream ends the wait with its error.
// PSVO_HOST_WAIT_STATS=1: the host's time in these waits, printed when the
// engine is freed (is the iteration host-bound? a host that never waits is)
struct HostWait {
    double ns = 0;
    long calls = 0, spun = 0;
};
HostWait g_host_wait;
// every granule tagged `seq`: decode the values into out
bool stats_landed(const unsigned long long *raw, int seq, int *out) {
    int v[PSVO_STAT_WORDS];
    for (int k = 0; k < PSVO_STAT_WORDS; ++k) {
        const unsigned long long g = __atomic_load_n(raw + k, __ATOMIC_ACQUIRE);
        if ((int)(g >> 32) != seq) return false;
        v[k] = (int)(unsigned)g;
    }
    memcpy(out, v, sizeof(v));
    return true;
}
int spin_wait_impl(QuerySet &q, hipEvent_t ev, hipStream_t qs, const char *who, int part);
// part 0: the read-back after the sampler; 1: a data-parallel query's second
int spin_wait(QuerySet &q, hipEvent_t ev, hipStream_t qs, const char *who, int part = 0) {
    int tmp[PSVO_STAT_WORDS];
    const bool ready = stats_landed(q.host_raw + part * PSVO_STAT_WORDS, q.seq, tmp);
    const double t0 = now_ns();
    const int rc = spin_wait_impl(q, ev, qs, who, part);
    g_host_wait.ns += now_ns() - t0;
    g_host_wait.calls += 1;
    g_host_wait.spun += ready ? 0 : 1;
    return rc;
}
int spin_wait_impl(QuerySet &q, hipEvent_t ev, hipStream_t qs, const char *who, int part) {
    // the runtime query (error detection only) costs microseconds: at most one
    // per 0.5 ms of waiting, so the statistics are seen as soon as they land
    const unsigned long long *raw = q.host_raw + part * PSVO_STAT_WORDS;
    double next_query = now_ns() + 5e5;
    for (unsigned it = 1;; ++it) {
        if (stats_landed(raw, q.seq, q.host_stats)) return PSVO_OK;
        if ((it & 255) == 0 && now_ns() >= next_query) {
            next_query = now_ns() + 5e5;
            const hipError_t e = ev ? hipEventQuery(ev) : hipStreamQuery(qs);
            if (e == hipErrorNotReady) continue;
            if (e != hipSuccess) return set_error(PSVO_E_LAUNCH, "%s: stats read-back: %s", who, hipGetErrorString(e));
            // the event (no system-scope fence) may complete just before the
            // kernel's system-scope granule stores are visible: poll a while more
            for (unsigned k = 0; k < (1u << 22); ++k)
                if (stats_landed(raw, q.seq, q.host_stats)) return PSVO_OK;
            return set_error(PSVO_E_LAUNCH, "%s: stats read-back: event complete, granules not tagged %d", who,
                             q.seq);
        }
    }
}

int query_set_init(QuerySet &s) {
    if (s.host_raw) return PSVO_OK;
    if (hipHostMalloc(reinterpret_cast<void **>(&s.host_raw), 2 * PSVO_STAT_WORDS * sizeof(unsigned long long),
                      hipHostMallocCoherent | hipHostMallocMapped) !=
            hipSuccess ||
        // device-side ordering only: the statistics reach the host through the
        // scan kernel's own system-scope release (k_scan_samples / k_stats_to_host)
        hipEventCreateWithFlags(&s.done, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess ||
        hipEventCreateWithFlags(&s.freed, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess ||
        // (bound to a dispatch as its stop event: a timing event)
        hipEventCreateWithFlags(&s.p1, hipEventDisableSystemFence) != hipSuccess ||
        hipEventCreateWithFlags(&s.done2, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "engine: query set allocation failed");
    // tag 0: no statistics yet (seq from 1)
    memset(s.host_raw, 0, 2 * PSVO_STAT_WORDS * sizeof(unsigned long long));
    return PSVO_OK;
}

void query_set_free(QuerySet &s) {
    for (int k = 0; k < kQSlots; ++k)
        if (s.a.p[k]) (void)hipFree(s.a.p[k]);
    if (s.host_raw) (void)hipHostFree(s.host_raw);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.freed) (void)hipEventDestroy(s.freed);
    if (s.p1) (void)hipEventDestroy(s.p1);
    if (s.done2) (void)hipEventDestroy(s.done2);
}

}  // namespace

extern "C" psvo_engine *psvo_engine_new(void) {
    psvo_engine *e = new psvo_engine();
    for (auto &q : e->qs)
        if (query_set_init(q) != PSVO_OK) {
            psvo_engine_free(e);
            return nullptr;
        }
    return e;
}

extern "C" int psvo_engine_queued(psvo_engine *e) { return e ? e->q_count : 0; }

// Drop every queued query (their buffers are reused only after their side-
// stream work completed: the next query waits on the stream).
extern "C" int psvo_map_discard(psvo_engine *e) {
    PSVO_REQUIRE(e, "map_discard: null engine");
    e->images_next = false;
    // no caller stream to order: the optimiser step of a split tail completes here
    if (e->adam_pending) {
        if (hipEventSynchronize(e->adam_done) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "map_discard: optimiser step failed");
        e->adam_pending = false;
    }
    while (e->q_count > 0) {
        QuerySet &q = e->qs[e->q_head];
        // the stream the query was queued on: psvo_map_query's side stream,
        // or aux for a psvo_map_step_frames look-ahead
        hipStream_t qs = q.qstream;
        if (qs && hipEventRecord(q.freed, qs) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "map_discard: event record failed");
        q.freed_recorded = qs != nullptr;
        q.freed_lazy = false;
        q.freed_on = qs;
        q.pending = false;
        e->q_head ^= 1;
        e->q_count--;
    }
    return PSVO_OK;
}

static EngineExchange exchange_layout(int world, int64_t max_rays_global, int64_t max_rays_rank) {
    EngineExchange x;
    x.world = world;
    x.nch = dist_slot0_rows(max_rays_global) / kSamplerG;
    x.max_rays_rank = max_rays_rank > 0 ? max_rays_rank : max_rays_global;
    x.cw = dist_count_words((int)x.max_rays_rank);
    return x;
}

extern "C" int64_t psvo_engine_exchange_words(int world, int64_t max_rays_global, int64_t max_rays_rank) {
    if (world < 1 || max_rays_global < 1 || max_rays_rank < 0 || max_rays_rank > max_rays_global) return -1;
    const EngineExchange x = exchange_layout(world, max_rays_global, max_rays_rank);
    return x.table_off() + x.table_words();
}

extern "C" int psvo_engine_set_exchange(psvo_engine *e, int rank, int world, int64_t max_rays_global,
                                        int64_t max_rays_rank, psvo_exchange_fn fn, void *user, int *xi32,
                                        double *xf64) {
    PSVO_REQUIRE(e, "engine_set_exchange: null engine");
    PSVO_REQUIRE(world >= 1 && rank >= 0 && rank < world && max_rays_global >= 1 && max_rays_rank >= 0 &&
                     max_rays_rank <= max_rays_global,
                 "engine_set_exchange: bad rank %d / world %d / max_rays_global %lld / max_rays_rank %lld", rank,
                 world, (long long)max_rays_global, (long long)max_rays_rank);
    PSVO_REQUIRE(e->q_count == 0, "engine_set_exchange: queries are queued");
    PSVO_REQUIRE(!fn || (xi32 && xf64), "engine_set_exchange: exchange buffers required");
    e->x = exchange_layout(world, max_rays_global, max_rays_rank);
    e->x.fn = fn;
    e->x.user = user;
    e->x.rank = rank;
    e->x.xi32 = xi32;
    e->x.xf64 = xf64;
    return PSVO_OK;
}

extern "C" int psvo_engine_set_paths(psvo_engine *e, int paths) {
    PSVO_REQUIRE(e && (paths & ~(PSVO_PATH_QUERY_SPLIT | PSVO_PATH_PADDED | PSVO_PATH_DENSE_DECODER)) == 0, "engine_set_paths: bad arguments");
    PSVO_REQUIRE(e->q_count == 0, "engine_set_paths: queries are queued");
    e->paths = paths;
    return PSVO_OK;
}

extern "C" int psvo_engine_gate_stream(psvo_engine *e, void *stream) {
    PSVO_REQUIRE(e, "engine_gate_stream: null engine");
    e->draw_gate_used = true;  // (binding the event costs the selection's stream ≈ 5 µs: only for a gating caller)
    if (!e->draw_gate_recorded) return PSVO_OK;
    if (hipStreamWaitEvent(as_stream(stream), e->draw_gate_ev, 0) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "engine_gate_stream: stream wait failed");
    return PSVO_OK;
}

extern "C" int psvo_engine_select_stats(psvo_engine *e, void *stream, int64_t *out, int reset) {
    PSVO_REQUIRE(e && out, "engine_select_stats: null argument");
    for (int i = 0; i < 5; ++i) out[i] = 0;
    if (!e->a.p[kSelCnt]) return PSVO_OK;  // no sparse step yet
    hipStream_t st = as_stream(stream);
    int c[psvo::kSelCountInts];
    if (hipMemcpyAsync(c, e->a.p[kSelCnt], sizeof(c), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "engine_select_stats: copy failed");
    unsigned long long u[3];
    memcpy(u, c + 4, sizeof(u));
    out[0] = (int64_t)c[0] + c[1];  // kept: class A + class B
    out[1] = c[3];                  // composited
    out[2] = (int64_t)u[0];
    out[3] = (int64_t)u[1];
    out[4] = (int64_t)u[2];
    if (c[2] & psvo::kLbFlagTimeout) {  // reported once: the bit and the host word cleared
        if (hipMemsetAsync(static_cast<int *>(e->a.p[kSelCnt]) + 2, 0, sizeof(int), st) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "engine_select_stats: memset failed");
        if (e->host_flags) *(volatile int *)e->host_flags = 0;
        e->sel_zero_gen = 0;
        return set_error(PSVO_E_LAUNCH, "engine_select_stats: a sample selection's look-back wait was abandoned");
    }
    if (reset && hipMemsetAsync(static_cast<int *>(e->a.p[kSelCnt]) + 4, 0, 6 * sizeof(int), st) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "engine_select_stats: memset failed");
    return PSVO_OK;
}

extern "C" int psvo_engine_set_timing(psvo_engine *e, int on) {
    PSVO_REQUIRE(e, "engine_set_timing: null engine");
    EngineTimer &t = e->tm;
    const char *mk = getenv("PSVO_TIMING_MARKERS");
    if (on && !t.ev[0][0])
        for (int r = 0; r < PSVO_TIME_REGIONS; ++r)
            for (int k = 0; k < 2; ++k)
                // a device-scope release: a marker with the default system-scope one
                // writes the L2 back between the kernels it brackets (measured in the time)
                if (hipEventCreateWithFlags(&t.ev[r][k], hipEventReleaseToDevice) != hipSuccess)
                    return set_error(PSVO_E_LAUNCH, "engine_set_timing: hipEventCreate failed");
    // the kernel-bound pairs: device-scope release too — the stop event is
    // the kernel's own completion signal, and a system-scope release there
    // adds an L2 write-back to the span that the untimed kernel does not pay
    const unsigned kc_flags = hipEventReleaseToDevice;
    if (on && !t.kc.ev[0][0])
        for (int i = 0; i < psvo::KernelClock::kMax; ++i)
            for (int k = 0; k < 2; ++k)
                if (hipEventCreateWithFlags(&t.kc.ev[i][k], kc_flags) != hipSuccess)
                    return set_error(PSVO_E_LAUNCH, "engine_set_timing: hipEventCreate failed");
    timer_collect(e, true);
    if (psvo::g_kclock == &t.kc) psvo::g_kclock = nullptr;
    t.kc.depth = 0;
    t.kc.overflow = false;
    t.on = on != 0;
    t.overlap = on == 2;
    t.markers = mk && *mk == '1';
    const char *ks = getenv("PSVO_TIMING_SPAN");
    t.kc.sum = !(ks && *ks == '1');
    t.kc.n = 0;
    t.kc.n_inst = 0;
    for (int r = 0; r < PSVO_TIME_REGIONS; ++r) {
        t.ms[r] = 0.0;
        t.n[r] = 0;
        t.kms[r] = 0.0;
        t.starts[r] = 0;
    }
    return PSVO_OK;
}

extern "C" int psvo_engine_timing(psvo_engine *e, double *mean_ms) {
    PSVO_REQUIRE(e && mean_ms, "engine_timing: null argument");
    EngineTimer &t = e->tm;
    timer_collect(e, true);
    for (int r = 0; r < PSVO_TIME_REGIONS; ++r) {
        if (t.markers)
            mean_ms[r] = t.n[r] ? t.ms[r] / (double)t.n[r] : -1.0;
        else  // a region whose instances launched no kernel reads 0 (e.g. no separate compaction)
            mean_ms[r] = t.starts[r] ? t.kms[r] / (double)t.starts[r] : -1.0;
    }
    PSVO_REQUIRE(t.markers || !t.kc.overflow, "engine_timing: more kernels per step than timing slots");
    return PSVO_OK;
}

extern "C" int psvo_engine_set_clock(psvo_engine *e, int max_steps) {
    PSVO_REQUIRE(e && max_steps >= 0, "engine_set_clock: bad arguments");
    while ((int)e->clk.ev.size() < max_steps) {
        hipEvent_t ev;
        // device-scope release: the clock's marker sits between the query's scan
        // and the compaction on the critical stream (a system-scope one costs
        // an L2 write-back there)
        if (hipEventCreateWithFlags(&ev, hipEventReleaseToDevice) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "engine_set_clock: event failed");
        e->clk.ev.push_back(ev);
    }
    e->clk.n = 0;
    e->clk.on = max_steps > 0;
    return PSVO_OK;
}

extern "C" int psvo_engine_clock(psvo_engine *e, double *period_ms, int *n_steps) {
    PSVO_REQUIRE(e && period_ms && n_steps, "engine_clock: null argument");
    *period_ms = -1.0;
    *n_steps = e->clk.n;
    if (e->clk.n >= 2) {
        float ms = 0.f;
        hipEvent_t a = e->clk.ev[0], b = e->clk.ev[e->clk.n - 1];
        if (hipEventSynchronize(b) != hipSuccess || hipEventElapsedTime(&ms, a, b) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "engine_clock: event read failed");
        *period_ms = ms / (double)(e->clk.n - 1);
    }
    return PSVO_OK;
}

extern "C" int psvo_host_wait_stats(double *wait_us, long long *calls, long long *waited, int reset) {
    PSVO_REQUIRE(wait_us && calls && waited, "host_wait_stats: null argument");
    *wait_us = g_host_wait.ns / 1e3;
    *calls = g_host_wait.calls;
    *waited = g_host_wait.spun;
    if (reset) g_host_wait = HostWait();
    return PSVO_OK;
}

extern "C" void psvo_engine_free(psvo_engine *e) {
    if (!e) return;
    for (hipEvent_t ev : e->clk.ev) (void)hipEventDestroy(ev);
    static const bool report = getenv("PSVO_HOST_WAIT_STATS") && *getenv("PSVO_HOST_WAIT_STATS") == '1';
    if (report && g_host_wait.calls > 0)
        fprintf(stderr, "psvo: host waited for the query statistics %ld times (%ld not yet landed), %.1f us each\n",
                g_host_wait.calls, g_host_wait.spun, g_host_wait.ns / 1e3 / g_host_wait.calls);
    (void)hipDeviceSynchronize();
    for (int r = 0; r < PSVO_TIME_REGIONS; ++r)
        for (int k = 0; k < 2; ++k)
            if (e->tm.ev[r][k]) (void)hipEventDestroy(e->tm.ev[r][k]);
    if (psvo::g_kclock == &e->tm.kc) psvo::g_kclock = nullptr;
    for (int i = 0; i < psvo::KernelClock::kMax; ++i)
        for (int k = 0; k < 2; ++k)
            if (e->tm.kc.ev[i][k]) (void)hipEventDestroy(e->tm.kc.ev[i][k]);
    for (int s = 0; s < kSlots; ++s)
        if (e->a.p[s]) (void)hipFree(e->a.p[s]);
    for (auto &q : e->qs) query_set_free(q);
    if (e->side) (void)hipStreamDestroy(e->side);
    if (e->q2s) (void)hipStreamDestroy(e->q2s);
    if (e->aux) {
        (void)hipStreamSynchronize(e->aux);  // a pending tail split's optimiser step
        (void)hipStreamDestroy(e->aux);
    }
    if (e->lossq) (void)hipStreamDestroy(e->lossq);
    if (e->loss_done) (void)hipEventDestroy(e->loss_done);
    if (e->dfeat_ready) (void)hipEventDestroy(e->dfeat_ready);
    if (e->emb_done) (void)hipEventDestroy(e->emb_done);
    if (e->z_ready) (void)hipEventDestroy(e->z_ready);
    if (e->coef_ready) (void)hipEventDestroy(e->coef_ready);
    if (e->grads_ready) (void)hipEventDestroy(e->grads_ready);
    if (e->prep_fork) (void)hipEventDestroy(e->prep_fork);
    if (e->prep_done) (void)hipEventDestroy(e->prep_done);
    if (e->adam_done) (void)hipEventDestroy(e->adam_done);
    if (e->next_ready) (void)hipEventDestroy(e->next_ready);
    if (e->in_ready) (void)hipEventDestroy(e->in_ready);
    if (e->draw_gate) (void)hipEventDestroy(e->draw_gate);
    if (e->host_flags) (void)hipHostFree(e->host_flags);
    delete e;
}

#define ENG_BUF(T, name, slot, bytes)                                        \
    T *name = reinterpret_cast<T *>(slot_buf(e, st, slot, (bytes), &rc));   \
    if (!name) return rc;

// decoder parameter sizes (nrgbd.py:98-108, depth 2, in 16, sdf_dim 128) for width W
static void dec_sizes(int W, int64_t (&n)[10]) {
    const int64_t w = W;
    const int64_t v[10] = {w * 16, w, w * w, w, 129 * w, 129, w * 144, w, 3 * w, 3};
    for (int i = 0; i < 10; ++i) n[i] = v[i];
}
static int64_t dec_total(int W) {
    int64_t n[10], t = 0;
    dec_sizes(W, n);
    for (int i = 0; i < 10; ++i) t += n[i];
    return t;
}

extern "C" int64_t psvo_map_grad_floats(int64_t n_emb) { return n_emb * 16 + dec_total(128); }
extern "C" int64_t psvo_map_grad_floats_w(int64_t n_emb, int width) { return n_emb * 16 + dec_total(width); }

// grads: [embeddings (n_emb x 16) | W1, b1, ..., W5, b5]
// one launch for both optimisers (lr per tensor); the embedding gradient is
// zeroed as it is consumed — the next iteration's atomics accumulate into it
// the keyframe poses' Adam steps of a psvo_map_step_frames iteration, queued
// with the map's (one launch) or alone (data parallel: the map waits for the
// gradient all-reduce)
struct PoseAdam {
    int n = 0;
    float *p[kXchMaxFrames], *m[kXchMaxFrames], *v[kXchMaxFrames];
    const float *g[kXchMaxFrames];
    int64_t step[kXchMaxFrames];
    double lr = 0.0;
};

static int map_adam(hipStream_t st, const psvo_map_desc *d, float *grads, int64_t adam_step,
                    const PoseAdam *pa = nullptr, bool sparse_rows = false) {
    constexpr int kMax = 11 + kXchMaxFrames;
    float *p[kMax];
    const float *g[kMax];
    float *m[kMax], *v[kMax];
    int64_t n[kMax], steps[kMax];
    double lr[kMax];
    int zero[kMax];
    const uint8_t *rows[kMax] = {};
    if (sparse_rows) rows[0] = d->emb_row_flags;  // the embedding table: flagged rows only
    p[0] = d->emb;
    g[0] = grads;
    m[0] = d->emb_m;
    v[0] = d->emb_v;
    n[0] = d->n_emb * 16;
    lr[0] = d->lr_emb;
    zero[0] = 1;
    int64_t off = d->n_emb * 16;
    int64_t kDecSizes[10];
    dec_sizes(d->width, kDecSizes);
    for (int i = 0; i < 10; ++i) {
        p[1 + i] = d->dec[i];
        g[1 + i] = grads + off;
        m[1 + i] = d->dec_m[i];
        v[1 + i] = d->dec_v[i];
        n[1 + i] = kDecSizes[i];
        lr[1 + i] = d->lr_dec;
        zero[1 + i] = 0;  // overwritten by the decoder backward
        off += kDecSizes[i];
    }
    int cnt = 11;
    for (int i = 0; i < cnt; ++i) steps[i] = adam_step;
    for (int f = 0; pa && f < pa->n; ++f, ++cnt) {
        p[cnt] = pa->p[f];
        g[cnt] = pa->g[f];
        m[cnt] = pa->m[f];
        v[cnt] = pa->v[f];
        n[cnt] = 6;
        lr[cnt] = pa->lr;
        zero[cnt] = 0;
        steps[cnt] = pa->step[f];
    }
    return adam_launch(st, cnt, p, g, m, v, n, lr, d->beta1, d->beta2, d->eps, 0.0, adam_step, zero, steps, rows);
}

extern "C" int psvo_map_adam_ex(psvo_engine *e, void *stream, const psvo_map_desc *d, int64_t adam_step,
                                int flags) {
    PSVO_REQUIRE(e && d && d->grad_flat && adam_step >= 1, "map_adam: needs desc->grad_flat and adam_step >= 1");
    e->images_next = false;  // the weights may change before the next step
    hipStream_t st = as_stream(stream);
    ENG_CALL(join_adam(e, st, "map_adam"));
    // sparse-exact when the row flags hold every row with a gradient: a
    // single-GPU step marked its rows itself (also under PSVO_STEP_NO_ADAM);
    // data parallel, only the gradient exchange knows the union of all ranks'
    // rows, so the caller says it marked them (PSVO_ADAM_ROWS_EXCHANGED)
    const bool flags_complete = !e->x.on() || (flags & PSVO_ADAM_ROWS_EXCHANGED);
    const bool sparse = d->emb_row_flags != nullptr && flags_complete;
    ENG_CALL(map_adam(st, d, d->grad_flat, adam_step, nullptr, sparse));
    if (d->emb_row_flags && !sparse) {
        // dense step under the exchange without a union mark (one unforced
        // rank, a caller's own all-reduce): keep the flags sticky-complete —
        // every row whose moments are now non-zero — so a later sparse step
        // still steps them; this rank's marks are spent
        ENG_CALL(psvo_adam_flags_from_state(st, d->n_emb, d->emb_m, d->emb_v, d->emb_row_flags));
        if (d->emb_row_local && hipMemsetAsync(d->emb_row_local, 0, (size_t)d->n_emb, st) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "map_adam: memset failed");
    }
    e->grads_clean = true;
    return PSVO_OK;
}

extern "C" int psvo_map_adam(psvo_engine *e, void *stream, const psvo_map_desc *d, int64_t adam_step) {
    return psvo_map_adam_ex(e, stream, d, adam_step, 0);
}

namespace {

// what one render (query + forward) leaves for the loss and the backward
struct Render {
    int64_t r_hit = 0, m = 0;
    int s_max = 0;
    int *rank_ray, *ray_rank, *ray_ns, *offsets, *leaf, *ray_of;
    float *tt, *z_vals, *feat, *images, *sdf_s, *rgb_s, *act, *sdf, *weights, *color, *depth;
    uint64_t *masks;
    bool z_recorded = false;  // e->z_ready marks the sample compaction on st (aux has not waited yet)
    int z_stride = 0;         // row stride of z_vals: s_max (padded copy) or the sampler's row capacity
    bool sparse = false;      // the decoder ran the sdf trunk only (sdf_s): the rest after select_samples
    float *h2 = nullptr;      // (sparse, width 128) every sample's h2 rows [m][128] from the sdf trunk
};

constexpr int64_t kW128 = 128;  // h2 row length (the width-128 decoder)

#define Q_BUF(T, name, slot, bytes)                                              \
    T *name = reinterpret_cast<T *>(arena_buf(q.a, st, slot, (bytes), &rc));    \
    if (!name) return rc;

// A data-parallel query's second half (QuerySet::p2_pending) on the q2
// stream, forked at the first read-back: the rank's [S_max, count words]
// (dist_counts), their all-gather on the query communicator, the union S_max
// and normaliser sums (dist_smax), the second read-back.  Nothing on the
// step's stream waits for it: the host does (render, before the first launch
// sized by S_max), and aux before it reads the sums.
int query_phase2(psvo_engine *e, QuerySet &q, const char *who) {
    if (!q.p2_pending) return PSVO_OK;
    q.p2_pending = false;
    const EngineExchange &x = e->x;
    if (!e->q2s && hipStreamCreateWithFlags(&e->q2s, hipStreamNonBlocking) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "%s: stream creation failed", who);
    hipStream_t s2 = e->q2s;
    int *stats = static_cast<int *>(q.a.p[kStats]);
    int *in = x.xi32 + x.q2_in_off();
    // (the count words start at zero, whatever a failed earlier half left)
    if (hipStreamWaitEvent(s2, q.p1, 0) != hipSuccess ||
        hipMemsetAsync(in + 1, 0, (kDistWordsPerRank - 1) * sizeof(int), s2) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "%s: stream ordering failed", who);
    ENG_CALL(dist_counts(s2, q.R, stats, static_cast<const int *>(q.a.p[kRankRay]), q.p2_gt,
                         static_cast<const float *>(q.a.p[kSDepth]), q.max_steps,
                         static_cast<const int *>(q.a.p[kRayNs]), q.p2_tr, q.p2_max_depth, in));
    ENG_CALL(x.call(PSVO_XCH_GATHER_I32 | PSVO_XCH_QUERY, x.q2_in_off(), x.q2_all_off(), kDistWordsPerRank, s2,
                    "S_max + counts"));
    ENG_CALL(dist_smax(s2, x.xi32 + x.q2_all_off(), x.world, stats, in,
                       q.p2_gt ? static_cast<double *>(q.a.p[kDistSums]) : nullptr));
    ENG_CALL(psvo::stats_to_host(s2, stats, q.host_raw + PSVO_STAT_WORDS, PSVO_STAT_WORDS, q.seq));
    q.stats_zeroed = stats;
    if (hipEventRecord(q.done2, s2) != hipSuccess) return set_error(PSVO_E_LAUNCH, "%s: event record failed", who);
    return PSVO_OK;
}

// every queued second half, oldest query first; `st` then follows them
int flush_phase2(psvo_engine *e, hipStream_t st, const char *who) {
    for (int k = 0; k < 2; ++k) {
        QuerySet &o = e->qs[e->q_head ^ k];
        if (!o.p2_pending) continue;
        ENG_CALL(query_phase2(e, o, who));
        if (hipStreamWaitEvent(st, o.done2, 0) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "%s: stream ordering failed", who);
    }
    return PSVO_OK;
}

// The query half of render_rays (render_helpers.py:363-413): intersection,
// hit ranks and sampling of one ray batch into query set `q` on stream `st`,
// then the 32-byte statistics read-back (event q.done).  The sampler reads P,
// R_hit and max ⌈steps⌉ from `stats` on the device; its buffers are [R, cap]
// with cap ≥ max_steps = max ⌈Σ(t_out − t_in)/step⌉ + P, bounded by 50 leaf
// intervals of at most a voxel diagonal (rows are written only up to
// max_steps; an overflow is flagged and reported by the consumer).
int query_enqueue(psvo_engine *e, hipStream_t st, QuerySet &q, const psvo_map_desc *d, int64_t R,
                  const float *rays_o, const float *rays_d, uint64_t seed, const char *who,
                  const float *noise = nullptr, bool record_done = true, const float *counts_gt = nullptr) {
    int rc = PSVO_OK;
    // data parallel: an earlier query's second half first — every rank issues
    // the collectives in query order, and this query's kernels follow that
    // half's reads of the buffers they overwrite
    ENG_CALL(flush_phase2(e, st, who));
    Q_BUF(int, stats, kStats, PSVO_STAT_WORDS * sizeof(int));
    if (q.stats_zeroed != stats && hipMemsetAsync(stats, 0, PSVO_STAT_WORDS * sizeof(int), st) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "%s: memset failed", who);
    q.stats_zeroed = nullptr;  // until this query's read-back is queued
    Q_BUF(int, hit_idx, kHitIdx, R * kMaxHits * sizeof(int));
    Q_BUF(float, hit_t0, kHitT0, R * kMaxHits * sizeof(float));
    Q_BUF(float, hit_t1, kHitT1, R * kMaxHits * sizeof(float));
    Q_BUF(int, ray_nv, kRayNv, R * sizeof(int));
    Q_BUF(float, ray_dsum, kRayDsum, R * sizeof(float));
    Q_BUF(int, ray_rank, kRayRank, R * sizeof(int));
    Q_BUF(int, rank_ray, kRankRay, R * sizeof(int));
    mark(e, st, PSVO_TIME_INTERSECT, 0);
    Q_BUF(int, blk_out, kBlkOut, (size_t)(R + 3) / 4 * 2 * sizeof(int));  // per intersect block: tests, rounds
    const EngineExchange &x = e->x;
    // the statistics / rank pass and the sample scan inside the traversal and
    // sampler launches (decoupled look-back; the sampler's only on one GPU)
    unsigned long long *lb = nullptr;
    uint32_t tag = 0;
    if (psvo::query_lookback(R) && !(e->paths & PSVO_PATH_QUERY_SPLIT)) {
        const size_t lb_bytes = (size_t)psvo::lookback_granules(R) * sizeof(unsigned long long);
        lb = reinterpret_cast<unsigned long long *>(arena_buf(q.a, st, kLbDesc, lb_bytes, &rc));
        if (!lb) return rc;
        // fresh memory (or after a reported failure): no stale granule may
        // carry a future tag, and the ticket counters start at 0 (lookback.h)
        if (q.lb_zero_gen != q.a.gen[kLbDesc]) {
            if (hipMemsetAsync(lb, 0, q.a.cap[kLbDesc], st) != hipSuccess)
                return set_error(PSVO_E_LAUNCH, "%s: memset failed", who);
            q.lb_zero_gen = q.a.gen[kLbDesc];
        }
        e->lb_tag = e->lb_tag == 0xffffffffu ? 1u : e->lb_tag + 1u;
        tag = e->lb_tag;
    }
    // with the look-back: each rank's hit count and first voxel id by rank
    // (the sampler's only reads of other rows, one load each)
    int *nv_rank = nullptr, *col0_rank = nullptr;
    if (lb) {
        Q_BUF(int, nr_, kNvRank, R * sizeof(int));
        Q_BUF(int, c0_, kCol0Rank, R * sizeof(int));
        nv_rank = nr_, col0_rank = c0_;
    }
    ENG_CALL(psvo::intersect_ranked(st, R, rays_o, rays_d, d->centres, d->structure, d->voxel_size,
                                    d->max_distance, d->step_size, hit_idx, hit_t0, hit_t1, ray_nv, ray_dsum, stats,
                                    ray_rank, rank_ray, static_cast<const PackRec *>(d->packed), blk_out, lb, tag,
                                    nv_rank, col0_rank, d->n_nodes));
    if (x.on() && noise) return set_error(PSVO_E_INVALID, "%s: injected sampler noise is single-GPU only", who);
    if (x.on()) {  // union-batch layout: ONE all-gather (8 words + the hit rows' counts), then local
        if (R > x.max_rays_rank)
            return set_error(PSVO_E_INVALID, "%s: %lld rays exceed the exchange's max_rays_rank %lld", who,
                             (long long)R, (long long)x.max_rays_rank);
        // (a query without GT depths: the step counts the normalisers itself —
        // on every rank, decided from the gathered flags)
        ENG_CALL(dist_pack(st, R, stats, rank_ray, hit_idx, ray_nv, x.xi32 + x.in_off(), nv_rank,
                           counts_gt ? 0 : psvo::PSVO_FLAG_UNION_UNCOUNTED));
        ENG_CALL(x.call(PSVO_XCH_GATHER_I32 | PSVO_XCH_QUERY, x.in_off(), x.all_off(), x.cw, st, "query layout"));
        ENG_CALL(dist_layout(st, x.xi32 + x.all_off(), x.world, x.rank, x.cw, x.nch, stats, x.xi32 + x.table_off(),
                             nullptr));
    }
    mark(e, st, PSVO_TIME_INTERSECT, 1);
    const int max_steps = (int)ceil(kMaxHits * 1.7321 * 1.001 * (double)d->voxel_size / (double)d->step_size) +
                          kMaxHits + 1;
    Q_BUF(int, s_idx, kSIdx, (size_t)R * max_steps * sizeof(int));
    Q_BUF(float, s_depth, kSDepth, (size_t)R * max_steps * sizeof(float));
    // the sampler's distance rows (render_helpers' sampled_dists) are not read
    // on this path: the sampler skips them (nullptr)
    float *const s_dist = nullptr;
    Q_BUF(int, ray_ns, kRayNs, (size_t)R * sizeof(int));
    Q_BUF(int, offsets, kOffsets, (size_t)(R + 1) * sizeof(int));
    mark(e, st, PSVO_TIME_SAMPLE, 0);
    if (x.on()) {
        ENG_CALL(dist_sample(st, R, max_steps, rank_ray, hit_idx, hit_t0, hit_t1, ray_dsum, d->step_size, seed, stats,
                             x.xi32 + x.table_off(), x.nch, s_idx, s_depth, s_dist, ray_ns, offsets, nv_rank,
                             col0_rank));
        // S_max of the union (every rank pads its [R_hit, S_max] blocks to it)
        // and, given the step's GT depths, the loss normalisers' counts: ONE
        // all-gather of 8 words, in the query's second half (query_phase2)
        if (counts_gt) {
            Q_BUF(double, qs_, kDistSums, 8 * sizeof(double));
            (void)qs_;
        }
        q.p2_gt = counts_gt;
        q.p2_tr = d->truncation;
        q.p2_max_depth = d->max_depth;
    }
    q.seq = q.seq == 0x7fffffff ? 1 : q.seq + 1;
    q.counts_gt = x.on() ? counts_gt : nullptr;  // data parallel: the union's count sums in kDistSums
    q.compacted = false;
    if (!x.on()) {  // the sampler's scan does the read-back (and, given the GT depths, the loss normalisers)
        psvo::SampleCounts sc{};
        // the per-ray counts pack into 12-bit fields (svo_query.hip pack_counts):
        // rows that may hold more than 4095 samples count in the step instead (k_crit_counts)
        const bool counts = counts_gt != nullptr && max_steps <= 4095;
        if (counts) {
            Q_BUF(int, ray_cnt, kRayCnt, (size_t)R * sizeof(int));
            Q_BUF(float, coefq, kCoefQ, 4 * sizeof(float));
            sc = psvo::SampleCounts{counts_gt, ray_cnt, coefq, d->truncation, d->max_depth, d->w_rgb, d->w_depth,
                                    d->w_fs, d->w_sdf,
                                    PSVO_CRIT_USE_COLOR | PSVO_CRIT_USE_DEPTH | PSVO_CRIT_USE_SDF};
            q.counts_gt = counts_gt;
        }
        // look-back sampler: the ray-major compaction in the same launch
        // (capacity R · max_steps: every row fits); otherwise k_compact_rays after the read-back
        int *leaf_q = nullptr, *ray_of_q = nullptr, *m_dev = nullptr;
        float *t_q = nullptr;
        if (lb) {
            const size_t cap = (size_t)R * max_steps;
            Q_BUF(int, lq_, kLeafQ, cap * sizeof(int));
            Q_BUF(float, tq_, kTQ, cap * sizeof(float));
            Q_BUF(int, rq_, kRayOfQ, cap * sizeof(int));
            Q_BUF(int, md_, kMDev, sizeof(int));
            leaf_q = lq_, t_q = tq_, ray_of_q = rq_, m_dev = md_;
        }
        ENG_CALL(psvo::sample_rays_to_host(st, R, max_steps, rank_ray, hit_idx, hit_t0, hit_t1, ray_dsum,
                                           d->step_size, noise, seed, stats, s_idx, s_depth, s_dist, ray_ns, offsets,
                                           q.host_raw, q.seq, counts ? &sc : nullptr, lb, tag, leaf_q, t_q,
                                           ray_of_q, m_dev, nv_rank, col0_rank));
        q.compacted = leaf_q != nullptr;
    }
    mark(e, st, PSVO_TIME_SAMPLE, 1);
    if (x.on()) {
        // the first read-back (the shard's sizes and the union's R_hit / P /
        // flags), the words kept for the second half, whose stream forks here
        psvo::g_stop_event = q.p1;
        const int rb = psvo::stats_to_host(st, stats, q.host_raw, PSVO_STAT_WORDS, q.seq, false);
        const bool bound = psvo::g_stop_event == nullptr;
        psvo::g_stop_event = nullptr;
        ENG_CALL(rb);
        if (!bound && hipEventRecord(q.p1, st) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "%s: event record failed", who);
        q.p2_pending = true;
    }
    q.stats_zeroed = x.on() ? nullptr : stats;  // (data parallel: the second read-back zeroes them)
    q.done_recorded = record_done;
    if (record_done && hipEventRecord(q.done, st) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "%s: stats read-back failed", who);
    q.qstream = st;
    q.R = R;
    q.ro = rays_o;
    q.rd = rays_d;
    q.dirs = nullptr;
    q.seed = seed;
    q.max_steps = max_steps;
    return PSVO_OK;
}

// A query set for a step on `st` over (R, rays, seed): the queued one
// psvo_map_query prepared for exactly this batch, or a fresh query enqueued
// on `st` itself.
int take_query(psvo_engine *e, hipStream_t st, const psvo_map_desc *d, int64_t R, const float *rays_o,
               const float *rays_d, uint64_t seed, const char *who, QuerySet **out, const float *noise = nullptr,
               const float *counts_gt = nullptr) {
    if (e->q_count > 0) {
        QuerySet &q = e->qs[e->q_head];
        if (q.R != R || q.ro != rays_o || q.rd != rays_d || q.seed != seed)
            return set_error(PSVO_E_INVALID, "%s: rays / seed differ from the batch queued by psvo_map_query", who);
        // the step's kernels read the query's outputs: order the streams
        if (q.qstream != st) {
            // a look-ahead queued without the event: its stream's position now (at or after the query)
            if (!q.done_recorded && hipEventRecord(q.done, q.qstream) != hipSuccess)
                return set_error(PSVO_E_LAUNCH, "%s: event record failed", who);
            q.done_recorded = true;
            if (hipStreamWaitEvent(st, q.done, 0) != hipSuccess)
                return set_error(PSVO_E_LAUNCH, "%s: stream wait failed", who);
        }
        *out = &q;
        return PSVO_OK;
    }
    QuerySet &q = e->qs[e->q_head];
    ENG_CALL(query_enqueue(e, st, q, d, R, rays_o, rays_d, seed, who, noise, true, counts_gt));
    *out = &q;
    return PSVO_OK;
}

// Give back the head query set once the step's kernels are queued.
int release_query(psvo_engine *e, hipStream_t st, QuerySet *q);

// `s` waits until the set's last consumer is done with its buffers (nothing
// when that consumer ran on `s` itself)
int freed_wait(QuerySet &q, hipStream_t s) {
    if (q.freed_lazy) {
        if (q.freed_on == s) return PSVO_OK;
        if (hipEventRecord(q.freed, q.freed_on) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "engine: event record failed");
        q.freed_lazy = false;
        q.freed_recorded = true;
    }
    if (q.freed_recorded && q.freed_on != s && hipStreamWaitEvent(s, q.freed, 0) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "engine: stream ordering failed");
    return PSVO_OK;
}

// Drops the step's query set if the step fails after take_query: without it a
// failed batch (no hit ray, sampler overflow) would stay at the FIFO head and
// every later step would be refused as "rays differ from the queued batch".
struct QueryGuard {
    psvo_engine *e;
    hipStream_t st;
    QuerySet *q = nullptr;
    ~QueryGuard() {
        if (q) (void)release_query(e, st, q);
    }
    int release() {
        QuerySet *x = q;
        q = nullptr;
        return release_query(e, st, x);
    }
};

int release_query(psvo_engine *e, hipStream_t st, QuerySet *q) {
    // no marker packet on st now (between two kernels one costs ≈ 5 µs):
    // a consumer on another stream records it when it needs it (freed_wait)
    q->freed_lazy = true;
    q->freed_recorded = false;
    q->freed_on = st;
    if (e->q_count > 0 && q == &e->qs[e->q_head]) {
        q->pending = false;
        e->q_head ^= 1;
        e->q_count--;
    }
    return PSVO_OK;
}

// Work beside the main stream on `aux` (timed runs in mode 1: everything on
// the caller's stream, in dependency order).
bool engine_overlap(psvo_engine *e) { return !e->tm.on || e->tm.overlap; }
int ensure_aux(psvo_engine *e) {
    if (e->aux) return PSVO_OK;
    hipEvent_t *evs[] = {&e->dfeat_ready, &e->emb_done, &e->z_ready, &e->coef_ready, &e->grads_ready,
                         &e->prep_fork, &e->prep_done, &e->loss_done, &e->adam_done, &e->next_ready};
    if (hipStreamCreateWithFlags(&e->aux, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&e->lossq, hipStreamNonBlocking) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "engine: aux stream creation failed");
    // stream-ordering events on one device: no system-scope fence (its L2
    // write-back, ≈ dirty bytes ÷ 6 TB/s, would sit between the kernels)
    for (hipEvent_t *ev : evs)  // (dfeat_ready may be bound to a dispatch as its stop event, like q.p1)
        if (hipEventCreateWithFlags(ev, (ev == &e->dfeat_ready ? 0 : hipEventDisableTiming) |
                                            hipEventDisableSystemFence) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "engine: event creation failed");
    return PSVO_OK;
}
// `st` waits for `ev` recorded on `from` now (no-op when from == st)
int fork_join(hipStream_t from, hipStream_t st, hipEvent_t ev) {
    if (from == st) return PSVO_OK;
    if (hipEventRecord(ev, from) != hipSuccess || hipStreamWaitEvent(st, ev, 0) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "engine: stream ordering failed");
    return PSVO_OK;
}

// A sample selection (k_select_samples) that gave up its look-back wait set
// bit 3 of the pinned host word: its step's loss and gradients were formed
// without the abandoned workgroups' samples.  Reported at the engine's next
// host read-back (the following step's statistics, or select_stats) — the
// step itself queues everything without a host round trip — and cleared
// once reported; the descriptors are re-zeroed before the next selection.
int select_failed(psvo_engine *e, const char *who) {
    if (!e->host_flags) return PSVO_OK;
    volatile int *f = e->host_flags;
    if (!(*f & psvo::kLbFlagTimeout)) return PSVO_OK;
    *f = 0;
    e->sel_zero_gen = 0;
    return set_error(PSVO_E_LAUNCH, "%s: the previous step's sample selection abandoned a look-back wait", who);
}

// render_rays (render_helpers.py:363-556) on the device, after the query:
// sample compaction (sized by the query's read-back), interpolation, decoder,
// compositing.  want_act: keep the decoder activations for weight gradients
// (mapping); tracking keeps only the masks.
int render(psvo_engine *e, hipStream_t st, const psvo_map_desc *d, QuerySet &qset, const float *rays_o,
           const float *rays_d, bool want_act, int *stats_out, const char *who, Render &o,
           bool fused_loss = false, bool need_z_event = true, bool sparse = false) {
    int rc = PSVO_OK;
    void *stream = st;
    const int max_steps = qset.max_steps;
    const int *rank_ray = static_cast<const int *>(qset.a.p[kRankRay]);
    const int *s_idx = static_cast<const int *>(qset.a.p[kSIdx]);
    const float *s_depth = static_cast<const float *>(qset.a.p[kSDepth]);
    const int *ray_ns = static_cast<const int *>(qset.a.p[kRayNs]);
    const int *offsets = static_cast<const int *>(qset.a.p[kOffsets]);
    float *const *W = d->dec;
    const int width = d->width;
    ENG_BUF(float, images, kImages, psvo_mlp_image_floats_w(width) * sizeof(float));
    // the decoder's operand images depend only on the weights (the previous
    // step's Adam is ordered before them on st): built on aux while the host
    // waits for the query's read-back (psvo_map_step)
    const bool prebuilt = fused_loss && e->images_next && e->images_w0 == W[0];
    e->images_next = false;
    const bool early_images = fused_loss && engine_overlap(e) && !prebuilt;
    if (early_images) {
        ENG_CALL(fork_join(st, e->aux, e->prep_fork));
        ENG_CALL(mlp_images(e->aux, width, W[0], W[1], W[2], W[3], W[4], W[5], W[6], W[7], W[8], W[9], images));
        if (hipEventRecord(e->prep_done, e->aux) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "%s: event record failed", who);
    }
    const bool dist = e->x.on();
    // the mapping step: no padded [R_hit, S_max] copy — the loss kernels read
    // z from the sampler's depth rows (stride max_steps; the union S_max of a
    // data-parallel step is at most every rank's max_steps) and the samples
    // are compacted ray-major (by the look-back sampler in its own launch,
    // else k_compact_rays: a wave per hit ray over its ≈ 64 valid entries);
    // tracking and PSVO_PATH_PADDED: the padded copy the autograd path makes
    // (k_sample_points)
    const bool rays_path = fused_loss && want_act && !(e->paths & PSVO_PATH_PADDED);
    // The device-sized forward: the interpolation and the sdf trunk queued
    // BEFORE the host waits for the query's statistics, sized on the device
    // (the sampler's M, kMDev) within a capacity grown from earlier batches —
    // the GPU runs them straight after the sampler instead of after the
    // host's read-back and launch (≈ 19 µs of idle GPU per step at config B).
    // A batch beyond the capacity makes them write nothing; the host then
    // runs them sized by the read-back, as without this path.
    const int64_t m_early = std::min<int64_t>(e->m_early, (int64_t)qset.R * max_steps);
    const bool early = rays_path && sparse && qset.compacted && qset.a.p[kMDev] && m_early > 0 &&
                       (early_images || prebuilt) && !(e->paths & PSVO_PATH_QUERY_SPLIT);
    float *feat_e = nullptr, *sdf_e = nullptr, *h2_e = nullptr;
    // the sparse decoder (width 128): the sdf trunk hands every sample's h2 to
    // the later layers (k_mlp_fwd2 / k_mlp_trunk_fb read it instead of
    // recomputing the W2 layer); width 256's trunk (k_dec256_trunk) is
    // device-sized too (round 6: C / E lost 22–37 µs per step to the host's
    // read-back before the interpolation)
    const bool want_h2 = sparse && width == 128;
    if (early) {
        const int *m_dev = static_cast<const int *>(qset.a.p[kMDev]);
        ENG_BUF(float, fe, kFeat, m_early * 16 * sizeof(float));
        ENG_BUF(float, se, kSdfS, m_early * sizeof(float));
        feat_e = fe;
        sdf_e = se;
        if (want_h2) {  // (width 256: its trunk keeps no h2)
            ENG_BUF(float, he, kH2, m_early * kW128 * sizeof(float));
            h2_e = he;
        }
        ENG_CALL(join_adam(e, st, who, 2000.0));
        mark(e, st, PSVO_TIME_INTERP_FWD, 0);
        ENG_CALL(psvo::interp_fwd_dev(st, m_early, m_dev, d->voxel_size, static_cast<const int *>(qset.a.p[kLeafQ]),
                                      static_cast<const float *>(qset.a.p[kTQ]),
                                      static_cast<const int *>(qset.a.p[kRayOfQ]), rank_ray, rays_o, rays_d,
                                      d->centres, d->vertex_idx, d->emb, feat_e));
        mark(e, st, PSVO_TIME_INTERP_FWD, 1);
        mark(e, st, PSVO_TIME_MLP_FWD, 0);
        if (early_images && hipStreamWaitEvent(st, e->prep_done, 0) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "%s: stream wait failed", who);
        const psvo::H2Rows h2o{h2_e, nullptr, nullptr};
        ENG_CALL(mlp_fwd_prepared(stream, m_early, width, feat_e, W[0], W[1], W[2], W[3], W[4], W[5], W[6], W[7],
                                  W[8], W[9], images, sdf_e, nullptr, nullptr, nullptr, m_dev, &h2o));
        // the loss normalisers need only z (the sampler's rows): aux may start
        // them after these (a marker in front of them delays the interpolation)
        if (engine_overlap(e) && need_z_event) {
            if (hipEventRecord(e->z_ready, st) != hipSuccess)
                return set_error(PSVO_E_LAUNCH, "%s: event record failed", who);
            o.z_recorded = true;
        }
    }
    ENG_CALL(spin_wait(qset, qset.done_recorded ? qset.done : nullptr, qset.qstream, who));
    timer_collect(e);  // the previous step's events completed before this read-back
    const int *hs = qset.host_stats;
    // data-parallel: this rank's hit rays, padded to the union's S_max
    const int r_hit = dist ? hs[PSVO_STAT_R_HIT_LOCAL] : hs[PSVO_STAT_R_HIT];
    if (hs[PSVO_STAT_FLAGS] & 8) {
        qset.lb_zero_gen = 0;  // the next query re-zeroes the descriptors and ticket counters
        return set_error(PSVO_E_LAUNCH, "%s: query look-back wait abandoned", who);
    }
    ENG_CALL(select_failed(e, who));
    if (hs[PSVO_STAT_FLAGS] & 1) return set_error(PSVO_E_OVERFLOW, "%s: octree deeper than the DFS stack", who);
    if (hs[PSVO_STAT_FLAGS] & 4) return set_error(PSVO_E_OVERFLOW, "%s: union batch exceeds max_rays_global", who);
    if (hs[PSVO_STAT_R_HIT] == 0)
        return set_error(PSVO_E_INVALID, "%s: no ray hits the octree (render_helpers.py:388)", who);
    const int64_t M = hs[PSVO_STAT_M];
    if (hs[PSVO_STAT_FLAGS] & 2) return set_error(PSVO_E_OVERFLOW, "%s: sampler exceeded max_steps", who);
    // data parallel: the union S_max comes with the query's second half
    // (query_phase2) — the mapping step waits for it only after queueing the
    // interpolation and the sdf trunk, which do not need it; the padded
    // paths (and an empty shard, which still joins the collectives) now
    auto phase2 = [&]() -> int {
        ENG_CALL(query_phase2(e, qset, who));
        ENG_CALL(spin_wait(qset, qset.done2, e->q2s, who, 1));
        return PSVO_OK;
    };
    const bool p2_late = dist && rays_path && r_hit > 0 && M > 0;
    if (dist && !p2_late) ENG_CALL(phase2());
    const int s_max = hs[PSVO_STAT_S_MAX];
    if (stats_out && !p2_late) memcpy(stats_out, hs, PSVO_STAT_WORDS * sizeof(int));
    o.r_hit = r_hit;
    o.m = M;
    o.s_max = s_max;
    if (dist && (r_hit == 0 || M == 0)) return PSVO_OK;  // an empty shard still joins the collectives
    if (M == 0) return set_error(PSVO_E_INVALID, "%s: no valid samples", who);
    // the device-sized forward covered this batch (else: it wrote nothing, run it host-sized below)
    const bool early_done = early && M <= m_early;
    if (rays_path && sparse) e->m_early = std::max<int64_t>(e->m_early, M + M / 4);
    ENG_BUF(int, leaf, kLeaf, M * sizeof(int));
    ENG_BUF(float, tt, kT, M * sizeof(float));
    ENG_BUF(int, ray_of, kRayOf, M * sizeof(int));
    ENG_BUF(float, feat, kFeat, M * 16 * sizeof(float));
    if (early_done && feat != feat_e) return set_error(PSVO_E_LAUNCH, "%s: feature buffer moved", who);
    float *z_vals = nullptr;
    if (!early) o.z_recorded = false;
    if (rays_path) {
        if (qset.compacted) {  // the sampler compacted in its launch (look-back offsets)
            leaf = static_cast<int *>(qset.a.p[kLeafQ]);
            tt = static_cast<float *>(qset.a.p[kTQ]);
            ray_of = static_cast<int *>(qset.a.p[kRayOfQ]);
        }
        // the loss normalisers need only z: aux may start them now (a
        // marker packet on st: none when aux has nothing to wait for)
        if (engine_overlap(e) && need_z_event && !o.z_recorded) {
            if (hipEventRecord(e->z_ready, st) != hipSuccess)
                return set_error(PSVO_E_LAUNCH, "%s: event record failed", who);
            o.z_recorded = true;
        }
        if (!qset.compacted) {
            mark(e, st, PSVO_TIME_POINTS, 0);
            ENG_CALL(psvo::compact_rays(st, r_hit, max_steps, s_idx, s_depth, offsets, leaf, tt, ray_of));
            mark(e, st, PSVO_TIME_POINTS, 1);
        }
        z_vals = const_cast<float *>(s_depth);
        o.z_stride = max_steps;
    } else {
        const size_t RS = (size_t)r_hit * s_max;
        ENG_BUF(float, z_b, kZ, RS * sizeof(float));
        ENG_BUF(uint8_t, smask, kMask, RS);
        mark(e, st, PSVO_TIME_POINTS, 0);
        ENG_CALL(psvo_sample_points(stream, r_hit, s_max, max_steps, s_idx, s_depth, ray_ns, offsets, leaf, tt,
                                    ray_of, z_b, smask));
        mark(e, st, PSVO_TIME_POINTS, 1);
        // the loss normalisers can start now (psvo_map_step, on aux)
        if (fused_loss && engine_overlap(e)) {
            if (hipEventRecord(e->z_ready, st) != hipSuccess)
                return set_error(PSVO_E_LAUNCH, "%s: event record failed", who);
            o.z_recorded = true;
        }
        z_vals = z_b;
        o.z_stride = s_max;
    }
    // ---- forward: interpolation, decoder (after the previous step's
    // optimiser step when its tail ran on aux)
    ENG_CALL(join_adam(e, st, who));
    if (!early_done) {  // (a batch beyond the device-sized forward's capacity: its region is already marked)
        if (!early) mark(e, st, PSVO_TIME_INTERP_FWD, 0);
        ENG_CALL(psvo_interp_fwd(stream, M, 16, d->voxel_size, leaf, tt, ray_of, rank_ray, rays_o, rays_d, d->centres,
                                 d->vertex_idx, d->emb, feat));
        if (!early) mark(e, st, PSVO_TIME_INTERP_FWD, 1);
    }
    ENG_BUF(float, sdf_s, kSdfS, M * sizeof(float));
    if (early_done && sdf_s != sdf_e) return set_error(PSVO_E_LAUNCH, "%s: sdf buffer moved", who);
    float *h2_s = nullptr;
    if (want_h2) {
        ENG_BUF(float, hb, kH2, M * kW128 * sizeof(float));
        if (early_done && hb != h2_e) return set_error(PSVO_E_LAUNCH, "%s: h2 buffer moved", who);
        h2_s = hb;
    }
    float *rgb_s = nullptr, *act = nullptr;
    uint64_t *masks = nullptr;
    // sparse: the sdf trunk (h1, h2, the sdf row: 18.6 of 53.8 k MACs per
    // sample) on every sample — the compositing weights need every sdf — and
    // the full decoder later, on the samples select_samples keeps
    o.sparse = sparse;
    if (!sparse) {
        ENG_BUF(float, rgb_b, kRgbS, M * 3 * sizeof(float));
        rgb_s = rgb_b;
        if (want_act) {
            ENG_BUF(float, abuf, kAct, (size_t)psvo_mlp_act_floats(M, width) * sizeof(float));
            act = abuf;
        }
        ENG_BUF(uint64_t, mbuf, kMasks, (size_t)psvo_mlp_mask_words(M, width) * sizeof(uint64_t));
        masks = mbuf;
    }
    if (!early) mark(e, st, PSVO_TIME_MLP_FWD, 0);  // (the device-sized forward opened it)
    o.h2 = nullptr;
    if (early_done) {
        o.h2 = h2_s;
    } else if (early_images || prebuilt) {
        if (early_images && hipStreamWaitEvent(st, e->prep_done, 0) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "%s: stream wait failed", who);
        const psvo::H2Rows h2o{h2_s, nullptr, nullptr};
        ENG_CALL(mlp_fwd_prepared(stream, M, width, feat, W[0], W[1], W[2], W[3], W[4], W[5], W[6], W[7], W[8], W[9],
                                  images, sdf_s, rgb_s, act, masks, nullptr, &h2o));
        o.h2 = h2_s;
    } else {
        ENG_CALL(psvo_mlp_fwd(stream, M, width, feat, W[0], W[1], W[2], W[3], W[4], W[5], W[6], W[7], W[8], W[9],
                              images, sdf_s, rgb_s, act, masks));
    }
    // sparse: the region stays open over the selection (its own, nested
    // region) and the compact forward (map_step_impl closes it)
    if (!sparse) mark(e, st, PSVO_TIME_MLP_FWD, 1);
    o.rank_ray = const_cast<int *>(rank_ray);
    o.ray_rank = static_cast<int *>(qset.a.p[kRayRank]);
    o.ray_ns = const_cast<int *>(ray_ns);
    o.offsets = const_cast<int *>(offsets);
    o.leaf = leaf;
    o.ray_of = ray_of;
    o.tt = tt;
    o.z_vals = z_vals;
    o.feat = feat;
    o.images = images;
    o.sdf_s = sdf_s;
    o.rgb_s = rgb_s;
    o.act = act;
    o.masks = masks;
    if (p2_late) {
        ENG_CALL(phase2());
        o.s_max = hs[PSVO_STAT_S_MAX];
        if (stats_out) memcpy(stats_out, hs, PSVO_STAT_WORDS * sizeof(int));
    }
    if (fused_loss) return PSVO_OK;  // compositing is part of psvo_composite_loss
    const size_t RS = (size_t)r_hit * s_max;
    ENG_BUF(float, sdf, kSdf, RS * sizeof(float));
    ENG_BUF(float, weights, kWeights, RS * sizeof(float));
    ENG_BUF(float, color, kColor, (size_t)r_hit * 3 * sizeof(float));
    ENG_BUF(float, depth, kDepth, (size_t)r_hit * sizeof(float));
    ENG_BUF(float, z_min, kZmin, (size_t)r_hit * sizeof(float));
    ENG_CALL(psvo_composite_fwd(stream, r_hit, s_max, d->truncation, offsets, ray_ns, z_vals, sdf_s, rgb_s, sdf,
                                weights, color, depth, z_min));
    o.sdf = sdf;
    o.weights = weights;
    o.color = color;
    o.depth = depth;
    return PSVO_OK;
}

// Criterion forward + backward to the per-sample decoder gradients (d loss =
// 1); dtmp/dthr: tracking's median depth filter or NULL.
int loss_backward(psvo_engine *e, hipStream_t st, const psvo_map_desc *d, const Render &q, const float *gt_rgb,
                  const float *gt_depth, const float *dtmp, const float *dthr, float *loss_out, float **g_sdf_s_out,
                  float **g_rgb_s_out) {
    int rc = PSVO_OK;
    void *stream = st;
    const int64_t r_hit = q.r_hit, M = q.m;
    const int s_max = q.s_max;
    const size_t RS = (size_t)r_hit * s_max;
    ENG_BUF(float, crit_ws, kCritWs, psvo_criterion_workspace_floats(r_hit) * sizeof(float));
    ENG_BUF(double, sums, kSums, 8 * sizeof(double));
    ENG_CALL(psvo_criterion_sums_ex(stream, r_hit, s_max, 0, d->truncation, d->max_depth, q.rank_ray, gt_rgb,
                                    gt_depth, q.color, q.depth, q.sdf, q.z_vals, dtmp, dthr, crit_ws, sums));
    ENG_CALL(psvo_criterion_finalize(stream, sums, r_hit, s_max, d->w_rgb, d->w_depth, d->w_fs, d->w_sdf,
                                     d->truncation, PSVO_CRIT_USE_COLOR | PSVO_CRIT_USE_DEPTH | PSVO_CRIT_USE_SDF,
                                     loss_out));
    ENG_BUF(float, g_loss, kGLoss, sizeof(float));
    if (hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(g_loss), 0x3F800000 /* 1.0f */, 1, st) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "engine: g_loss fill failed");
    ENG_BUF(float, g_color, kGColor, (size_t)r_hit * 3 * sizeof(float));
    ENG_BUF(float, g_depth, kGDepth, (size_t)r_hit * sizeof(float));
    ENG_BUF(float, g_sdf, kGSdf, RS * sizeof(float));
    ENG_CALL(psvo_criterion_bwd_ex(stream, r_hit, s_max, d->truncation, d->max_depth, q.rank_ray, gt_rgb, gt_depth,
                                   q.color, q.depth, q.sdf, q.z_vals, loss_out, g_loss, dtmp, dthr, g_color, g_depth,
                                   g_sdf));
    ENG_BUF(float, g_sdf_s, kGSdfS, M * sizeof(float));
    ENG_BUF(float, g_rgb_s, kGRgbS, M * 3 * sizeof(float));
    ENG_CALL(psvo_composite_bwd(stream, r_hit, s_max, d->truncation, q.offsets, q.ray_ns, q.z_vals, q.sdf, q.weights,
                                q.rgb_s, g_color, g_depth, nullptr, g_sdf, g_sdf_s, g_rgb_s));
    *g_sdf_s_out = g_sdf_s;
    *g_rgb_s_out = g_rgb_s;
    return PSVO_OK;
}

}  // namespace

namespace {
// the keyframe poses' part of an iteration (psvo_map_step_frames): per-frame
// gradient from the rays' grad_o / grad_d, then each optimised pose's Adam
int frames_update(psvo_engine *e, hipStream_t st, const psvo_map_desc *d, const psvo_map_frames *fr,
                  const Render &q, const float *grad_od, int64_t R, PoseAdam *pa) {
    int rc = PSVO_OK;
    float *pg = fr->pose_grad;
    if (!pg) {
        ENG_BUF(float, gbuf, kPoseGrad, (size_t)fr->n_frames * 8 * sizeof(float));
        pg = gbuf;
    }
    // data parallel: a keyframe belongs to one rank (each rank passes its own
    // keyframes), so its rays — and its whole pose gradient of the union-batch
    // loss — are local: no exchange
    ENG_CALL(psvo::pose_grad_frames_rays(st, fr->n_frames, fr->rays_per_frame, q.ray_rank, fr->dirs_cam, grad_od,
                                         grad_od + R * 3, fr->poses, pg));
    pa->n = 0;
    pa->lr = fr->lr_pose;
    for (int f = 0; f < fr->n_frames; ++f) {
        if (fr->pose_step[f] < 1) continue;  // stamp 0 / update_pose False: no optimiser (render_helpers.py:594-596)
        const int k = pa->n++;
        pa->p[k] = fr->poses + f * 6;
        pa->m[k] = fr->pose_m + f * 6;
        pa->v[k] = fr->pose_v + f * 6;
        pa->g[k] = pg + f * 8;
        pa->step[k] = fr->pose_step[f];
    }
    return PSVO_OK;
}

// the poses' Adam steps on their own (one launch, each pose at its own step)
int pose_adam(hipStream_t st, const psvo_map_desc *d, const PoseAdam &pa) {
    if (pa.n == 0) return PSVO_OK;
    int64_t n6[kXchMaxFrames];
    double lr[kXchMaxFrames];
    int zero[kXchMaxFrames];
    for (int k = 0; k < pa.n; ++k) {
        n6[k] = 6;
        lr[k] = pa.lr;
        zero[k] = 0;
    }
    return adam_launch(st, pa.n, pa.p, pa.g, pa.m, pa.v, n6, lr, d->beta1, d->beta2, d->eps, 0.0, 1, zero,
                       const_cast<int64_t *>(pa.step));
}

// The next iteration's query, queued on `ps` after this step's pose update:
// its rays (the updated poses applied to next_dirs_cam) into the engine's ray
// buffers — this step's last reader of them, the embedding backward, ran
// earlier on `ps` — then intersection + sampling into the free query set.
int frames_lookahead(psvo_engine *e, hipStream_t st, const psvo_map_desc *d, const psvo_map_frames *fr,
                     int64_t R, const Render &cur, const float *grad_od, bool record_done) {
    int rc = PSVO_OK;
    PSVO_REQUIRE(e->q_count == 0, "map_step_frames: a query is already queued");
    QuerySet &q = e->qs[e->q_head];
    // the set's last consumer ran on st itself: stream order suffices (no wait
    // packet between the backward and the pose step)
    ENG_CALL(freed_wait(q, st));
    ENG_BUF(float, rays_o, kRaysO, (size_t)R * 3 * sizeof(float));
    ENG_BUF(float, rays_d, kRaysD, (size_t)R * 3 * sizeof(float));
    float *pg = fr->pose_grad;
    if (!pg) {
        ENG_BUF(float, gbuf, kPoseGrad, (size_t)fr->n_frames * 8 * sizeof(float));
        pg = gbuf;
    }
    // this step's pose gradient, each optimised pose's Adam step and the next
    // rays from the updated poses: one launch (frames_update + pose_adam +
    // psvo_pose_rays_frames, the same arithmetic)
    ENG_CALL(psvo::pose_step_frames(st, fr->n_frames, fr->rays_per_frame, cur.ray_rank, fr->dirs_cam,
                                    grad_od, grad_od + R * 3, fr->poses, fr->pose_m, fr->pose_v, fr->pose_step,
                                    fr->lr_pose, d->beta1, d->beta2, d->eps, pg, fr->next_dirs_cam, rays_o, rays_d));
    ENG_CALL(query_enqueue(e, st, q, d, R, rays_o, rays_d, fr->next_seed, "map_step_frames (look-ahead)", nullptr,
                           record_done, fr->next_gt_depth));
    q.dirs = fr->next_dirs_cam;
    q.pending = true;
    e->q_count++;
    return PSVO_OK;
}
}  // namespace

static int map_step_impl(psvo_engine *e, hipStream_t st, const psvo_map_desc *d, int64_t n_rays, const float *rays_o,
                         const float *rays_d, const float *gt_rgb, const float *gt_depth, const float *noise,
                         uint64_t seed, int64_t adam_step, int flags, float *loss_out, int *stats_out,
                         const psvo_map_frames *fr) {
    PSVO_REQUIRE(e && d && rays_o && rays_d && gt_rgb && gt_depth && loss_out, "map_step: null argument");
    PSVO_REQUIRE(n_rays > 0 && adam_step >= 1, "map_step: bad sizes");
    PSVO_REQUIRE(d->width == 128 || d->width == 256, "map_step: decoder width %d unsupported (fused: 128, 256)",
                 d->width);
    int rc = PSVO_OK;
    const int64_t R = n_rays;
    Render q;
    QuerySet *qset = nullptr;
    // the normalisers from the query — single GPU the sampler's tail, data
    // parallel the query's second gather — only when the loss value is not
    // wanted (its reduction reads the counts k_crit_counts writes into the
    // loss partials)
    const bool want_loss = !(flags & PSVO_STEP_NO_LOSS);
    const float *counts_gt = !want_loss ? gt_depth : nullptr;
    ENG_CALL(take_query(e, st, d, R, rays_o, rays_d, seed, "map_step", &qset, noise, counts_gt));
    QueryGuard guard{e, st, qset};
    const bool overlap = engine_overlap(e);
    if (overlap) ENG_CALL(ensure_aux(e));
    hipStream_t ax = overlap ? e->aux : st;  // side work: loss normalisers / value, embedding backward
    // the look-ahead's inputs made on another stream: its position now, waited
    // for by the look-ahead's pose step only (psvo_map_frames.next_stream)
    const bool wait_next = fr && fr->next_dirs_cam && fr->next_stream && as_stream(fr->next_stream) != st;
    if (wait_next) {
        ENG_CALL(ensure_aux(e));
        if (hipEventRecord(e->next_ready, as_stream(fr->next_stream)) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "map_step: event record failed");
    }
    // The two cross-stream waits this step needs on st — the previous step's
    // optimiser (before the interpolation reads the embeddings: render) and
    // the draw of the next pixels (before the look-ahead's pose step) — sit
    // where their consumers are.  Queued here, in front of the render, both
    // measured slower (round 4, config B: 0.941 vs 0.928-0.932 ms per
    // iteration): the next draw co-runs with the persistent decoder kernels
    // and ends late, so the render then waits for it.
    const int crit_flags = PSVO_CRIT_USE_COLOR | PSVO_CRIT_USE_DEPTH | PSVO_CRIT_USE_SDF;
    // aux waits for z only to count the normalisers itself, or to mark the
    // rows the width-256 backward's scatter will touch
    const bool coef_known = counts_gt && qset->counts_gt == counts_gt;
    const bool need_z = !coef_known || e->x.on() ||
                        (d->emb_row_flags && !psvo::mlp_bwd_fuses_interp(d->width));
    // the sparse decoder: render runs the sdf trunk only
    const bool sparse_dec = !(e->paths & PSVO_PATH_DENSE_DECODER);
    ENG_CALL(render(e, st, d, *qset, rays_o, rays_d, true, stats_out, "map_step", q, true, need_z, sparse_dec));
    // (the step clock's marker is recorded after the optimiser step, below:
    // on st between two dependent kernels a marker costs ≈ 5 µs, measured)
    if (q.z_recorded && hipStreamWaitEvent(ax, e->z_ready, 0) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "map_step: stream wait failed");
    const int64_t M = q.m;
    const int64_t r_hit = q.r_hit;
    const int s_max = q.s_max;
    // data-parallel: the loss of the union batch (criterion.py:70-101 normalise
    // by batch-global counts and the padded [R_hit, S_max] size): count sums
    // and loss sums are all-reduced, the rank's gradients are its part of the
    // union-batch gradient (the caller sums them over ranks)
    const EngineExchange &x = e->x;
    const bool dist = x.on();
    const bool empty = dist && (r_hit == 0 || M == 0);
    const int64_t n_hit = dist ? qset->host_stats[PSVO_STAT_R_HIT] : r_hit;
    // ---- the sparse decoder: the samples whose gradients can be non-zero
    // get compact indices (composite.hip k_select_samples) — class A
    // (composited) at [0, M_A): the whole decoder forward; width 128, class B
    // (only the direct sdf loss term) at [M, M + M_B): the trunk's
    // forward + backward in one kernel (k_mlp_trunk_fb) — sized on the device (the counts never
    // reach the host)
    float *const *W = d->dec;
    Render qb = q;  // what the loss pass and the backward read per sample: the kept samples when sparse
    int *cidx = nullptr, *sel_cnt = nullptr;
    const bool two_class = q.sparse && d->width == 128;
    int *offb = nullptr;
    const int *h2_src = nullptr;  // the kept samples' rows of q.h2 (class A at [0, M), B at [M, 2 M))
    if (q.sparse && !empty) {
        const int64_t M2 = 2 * M;  // the compact rows: class A at [0, M), class B at [M, 2 M)
        ENG_BUF(int, cx, kCidx, M * sizeof(int));
        ENG_BUF(int, offa, kOffB, (size_t)(r_hit + 1) * sizeof(int));
        // the compact feature copy: width 256 only (width 128 reads the step's rows by src_c)
        float *feat_c = nullptr;
        if (!q.h2) {
            ENG_BUF(float, fc, kFeatB, M2 * 16 * sizeof(float));
            feat_c = fc;
        }
        ENG_BUF(int, leaf_c, kLeafB, M2 * sizeof(int));
        ENG_BUF(float, t_c, kTB, M2 * sizeof(float));
        ENG_BUF(int, ray_of_c, kRayOfB, M2 * sizeof(int));
        ENG_BUF(int, cnt, kSelCnt, psvo::kSelCountInts * sizeof(int));
        ENG_BUF(unsigned long long, desc, kSelDesc,
                (size_t)psvo::select_granules(r_hit) * sizeof(unsigned long long));
        if (e->sel_zero_gen != e->a.gen[kSelDesc]) {  // fresh memory: no stale granule may carry a future tag
            if (hipMemsetAsync(desc, 0, e->a.cap[kSelDesc], st) != hipSuccess ||
                hipMemsetAsync(cnt, 0, psvo::kSelCountInts * sizeof(int), st) != hipSuccess)
                return set_error(PSVO_E_LAUNCH, "map_step: memset failed");
            e->sel_zero_gen = e->a.gen[kSelDesc];
        }
        if (!e->host_flags) {
            if (hipHostMalloc(reinterpret_cast<void **>(&e->host_flags), sizeof(int),
                              hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
                return set_error(PSVO_E_LAUNCH, "map_step: pinned allocation failed");
            *e->host_flags = 0;
        }
        if (two_class) {
            ENG_BUF(int, ob, kOffB2, (size_t)(r_hit + 1) * sizeof(int));
            offb = ob;
        }
        ENG_BUF(float, rgb_c, kRgbS, M2 * 3 * sizeof(float));
        int *src_c = nullptr;
        if (q.h2) {
            ENG_BUF(int, sc, kSrcC, M2 * sizeof(int));
            src_c = sc;
        }
        e->sel_tag = e->sel_tag == 0xffffffffu ? 1u : e->sel_tag + 1u;
        mark(e, st, PSVO_TIME_SELECT, 0);
        if (e->draw_gate_used && !e->draw_gate &&
            hipEventCreateWithFlags(&e->draw_gate, hipEventDisableSystemFence) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "map_step: event creation failed");
        psvo::g_stop_event = e->draw_gate_used ? e->draw_gate : nullptr;  // bound to the selection's dispatch
        psvo::g_stop_share = true;  // (a timed step: the clock's stop event of the selection, no marker)
        psvo::g_stop_bound = nullptr;
        const int sel_rc = psvo::select_samples(st, r_hit, s_max, d->truncation, d->max_depth, q.offsets, q.ray_ns,
                                                q.z_vals, q.z_stride, q.rank_ray, gt_depth, q.sdf_s, q.feat, q.leaf,
                                                q.tt, q.ray_of, M, two_class, cx, offa, offb, feat_c, leaf_c, t_c,
                                                ray_of_c, rgb_c, src_c, cnt, desc, e->sel_tag, e->host_flags);
        if (e->draw_gate_used && psvo::g_stop_event == nullptr && psvo::g_stop_bound) {  // (consumed: launched)
            e->draw_gate_ev = psvo::g_stop_bound;
            e->draw_gate_recorded = true;
        }
        psvo::g_stop_event = nullptr;
        psvo::g_stop_share = false;
        ENG_CALL(sel_rc);
        mark(e, st, PSVO_TIME_SELECT, 1);
        ENG_BUF(float, sdf_b, kSdfB, M * sizeof(float));
        ENG_BUF(float, act, kAct, (size_t)psvo_mlp_act_floats(M, d->width) * sizeof(float));
        ENG_BUF(uint64_t, masks, kMasks, (size_t)psvo_mlp_mask_words(M, d->width) * sizeof(uint64_t));
        const psvo::H2Rows h2r{nullptr, q.h2, src_c};
        ENG_CALL(mlp_fwd_prepared(st, M, d->width, src_c ? q.feat : feat_c, W[0], W[1], W[2], W[3], W[4], W[5], W[6],
                                  W[7], W[8], W[9], q.images, sdf_b, rgb_c, act, masks, cnt, src_c ? &h2r : nullptr));
        h2_src = src_c;
        mark(e, st, PSVO_TIME_MLP_FWD, 1);
        qb.offsets = offa;
        qb.leaf = leaf_c;
        qb.tt = t_c;
        qb.ray_of = ray_of_c;
        qb.feat = src_c ? q.feat : feat_c;  // (src_c: x of kept sample j is row src_c[j])
        qb.rgb_s = rgb_c;
        qb.act = act;
        qb.masks = masks;
        cidx = cx;
        sel_cnt = cnt;
    }
    // ---- loss and backward (d loss = 1): normalisers on aux (after the
    // sampler, beside the decoder forward), then one fused per-ray pass
    ENG_BUF(float, crit_ws, kCritWs, psvo_criterion_workspace_floats(r_hit) * sizeof(float));
    double *sums_c = x.xf64, *sums = x.xf64 ? x.xf64 + 8 : nullptr;
    if (!dist) {
        ENG_BUF(double, sc, kSumsC, 8 * sizeof(double));
        ENG_BUF(double, sl, kSums, 8 * sizeof(double));
        sums_c = sc;
        sums = sl;
    }
    // the sampler counted the normalisers for exactly this GT (its tail wrote the coefficients)
    const bool coef_q = !dist && counts_gt && qset->counts_gt == counts_gt;
    // data parallel: the query gathered the union's counts — decided from the
    // gathered words (PSVO_FLAG_UNION_UNCOUNTED), the same on every rank, so
    // that all ranks issue the same collectives (psvo_map_query's counts_gt
    // must hold the step's GT depths: psvo.h)
    const bool sums_q = dist && counts_gt && qset->counts_gt != nullptr &&
                        !(qset->host_stats[PSVO_STAT_FLAGS] & psvo::PSVO_FLAG_UNION_UNCOUNTED);
    float *coef = coef_q ? static_cast<float *>(qset->a.p[kCoefQ]) : nullptr;
    if (!coef_q) {
        ENG_BUF(float, cbuf, kCoef, 4 * sizeof(float));
        coef = cbuf;
    }
    ENG_BUF(float, color, kColor, (size_t)r_hit * 3 * sizeof(float));
    ENG_BUF(float, depth, kDepth, (size_t)r_hit * sizeof(float));
    const int64_t m_rows = q.sparse ? 2 * M : M;  // per-sample gradient rows (the sparse decoder: at cidx)
    ENG_BUF(float, g_sdf_s, kGSdfS, m_rows * sizeof(float));
    ENG_BUF(float, g_rgb_s, kGRgbS, m_rows * 3 * sizeof(float));
    // sparse-exact Adam (single GPU): the rows this step can touch, beside the
    // decoder — marked whenever the flags exist, also when the caller runs the
    // Adam step itself (PSVO_STEP_NO_ADAM, then psvo_map_adam): a later fused
    // step must still find these rows (their moments are non-zero from now on)
    const bool mark_rows = d->emb_row_flags && !dist;
    const bool sparse_rows = mark_rows && !(flags & PSVO_STEP_NO_ADAM);
    // data parallel: this rank's rows into emb_row_local (the row-sparse
    // exchange lists them; the union flags come from what it exchanged)
    uint8_t *const mark_into = mark_rows ? d->emb_row_flags : (dist ? d->emb_row_local : nullptr);
    if (dist) {
        if (sums_q) {
            sums_c = static_cast<double *>(qset->a.p[kDistSums]);
            // (landed on the host before this launch; the wait orders it formally)
            if (hipStreamWaitEvent(ax, qset->done2, 0) != hipSuccess)
                return set_error(PSVO_E_LAUNCH, "map_step: stream wait failed");
        } else {
            ENG_CALL(criterion_counts(ax, empty ? 0 : r_hit, s_max, d->truncation, d->max_depth, q.rank_ray,
                                      gt_depth, q.z_vals, q.z_stride, q.z_stride == s_max ? nullptr : q.ray_ns,
                                      crit_ws, sums_c));
            ENG_CALL(x.call(PSVO_XCH_SUM_F64, 0, 0, 8, ax, "loss normalisers"));
        }
        ENG_CALL(criterion_coef_from_sums(ax, sums_c, n_hit, s_max, d->truncation, d->w_rgb, d->w_depth, d->w_fs,
                                          d->w_sdf, crit_flags, coef));
    } else if (!coef_q) {
        ENG_CALL(psvo::criterion_coef_z(ax, r_hit, s_max, d->truncation, d->max_depth, q.rank_ray, gt_depth,
                                        q.z_vals, q.z_stride, q.ray_ns, d->w_rgb,
                                        d->w_depth, d->w_fs, d->w_sdf, crit_flags, crit_ws, sums_c, coef));
    }
    if (!coef_q) ENG_CALL(fork_join(ax, st, e->coef_ready));
    // after the normalisers: the fused loss pass waits for them, Adam for the marks
    // (width 128: the fused backward's embedding scatter flags the rows it touches instead — the mark
    // kernel beside the decoder forward slowed it by ≈ 17 µs)
    const bool marks_in_bwd = psvo::mlp_bwd_fuses_interp(d->width);
    if (mark_into && !empty && !marks_in_bwd)
        ENG_CALL(psvo_adam_mark_rows(ax, M, q.leaf, d->vertex_idx, mark_into));
    if (!empty)
        ENG_CALL(psvo::composite_loss_z(st, r_hit, s_max, d->truncation, d->max_depth, q.offsets, q.ray_ns,
                                        q.z_vals, q.z_stride, q.rank_ray, gt_rgb, gt_depth, q.sdf_s, qb.rgb_s, coef,
                                        crit_ws, color, depth, g_sdf_s, g_rgb_s, want_loss || dist, cidx));
    // the loss value (not on the gradient path), beside the decoder backward:
    // data parallel on aux (its collective), single GPU on its own stream,
    // joined into st before the optimiser step (loss_out / crit_ws ordered)
    // PSVO_STEP_NO_LOSS: the caller does not read the value (bundle_adjust_frames
    // discards it, render_helpers.py:662-676): no reduction, no collective (every
    // rank passes the same flags)
    hipStream_t lq = (overlap && !dist) ? e->lossq : ax;
    if (want_loss) {
        ENG_CALL(fork_join(st, lq, e->grads_ready));
        if (!empty) {
            ENG_CALL(psvo_criterion_reduce(lq, r_hit, crit_ws, sums));
        } else if (hipMemsetAsync(sums, 0, 8 * sizeof(double), lq) != hipSuccess) {
            return set_error(PSVO_E_LAUNCH, "map_step: memset failed");
        }
        if (dist) ENG_CALL(x.call(PSVO_XCH_SUM_F64, 8, 8, 8, lq, "loss sums"));
        ENG_CALL(psvo_criterion_finalize(lq, sums, n_hit, s_max, d->w_rgb, d->w_depth, d->w_fs, d->w_sdf,
                                         d->truncation, crit_flags, loss_out));
        if (lq != ax && hipEventRecord(e->loss_done, lq) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "map_step: event record failed");
    }
    const bool join_loss = want_loss && lq != ax;
    const int n_split = 256;
    ENG_BUF(float, mlp_ws, kMlpWs, psvo_mlp_workspace_floats_w(M, d->width, n_split) * sizeof(float));
    ENG_BUF(float, dfeat, kDfeat, M * 16 * sizeof(float));
    // gradients: the caller's flat buffer (data-parallel all-reduce) or the arena
    float *grads = d->grad_flat;
    if (!grads) {
        ENG_BUF(float, gbuf, kDecGrad, psvo_map_grad_floats_w(d->n_emb, d->width) * sizeof(float));
        grads = gbuf;
    }
    float *grad_emb = grads;
    float *G[10];
    {
        int64_t kDecSizes[10];
        dec_sizes(d->width, kDecSizes);
        int64_t off = d->n_emb * 16;
        for (int i = 0; i < 10; ++i) {
            G[i] = grads + off;
            off += kDecSizes[i];
        }
    }
    ENG_BUF(float, grad_od, kGradOD, (size_t)R * 6 * sizeof(float));
    if (empty) {  // no samples on this rank: its part of the gradient is zero
        ENG_CALL(fork_join(ax, st, e->emb_done));
        if (hipMemsetAsync(grads, 0, (size_t)psvo_map_grad_floats_w(d->n_emb, d->width) * sizeof(float), st) !=
            hipSuccess)
            return set_error(PSVO_E_LAUNCH, "map_step: memset failed");
        e->grads_clean = false;
        ENG_CALL(guard.release());
        if (!(flags & PSVO_STEP_NO_ADAM)) ENG_CALL(map_adam(st, d, grads, adam_step));
        if (e->clk.on && e->clk.n < (int)e->clk.ev.size() && hipEventRecord(e->clk.ev[e->clk.n++], st) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "map_step: event record failed");
        return PSVO_OK;
    }
    // width 128: the interpolation backward runs inside the fused decoder
    // backward (embedding scatter into grad_emb, dL/dx per sample), then only
    // the per-ray d_o / d_d sums remain; otherwise k_interp_bwd after dfeat
    const bool fuse_ib = psvo::mlp_bwd_fuses_interp(d->width);
    // look-ahead with the fused backward (single GPU or the caller's Adam
    // skipped): the tail splits — st runs the per-ray d_o / d_d sums, the pose
    // step and the next query right after the decoder backward; aux sums the
    // weight-gradient slabs, steps the optimiser and builds the next decoder
    // images beside them (the next step's render waits for adam_done)
    const bool ahead = fr && fr->next_dirs_cam;
    const bool split = psvo::mlp_bwd_split_tail(d->width) && overlap && ahead && !(flags & PSVO_STEP_NO_ADAM);
    const bool emb_dirty = !(e->grads_clean && e->clean_buf == grad_emb);
    if (fuse_ib && emb_dirty && hipMemsetAsync(grad_emb, 0, (size_t)d->n_emb * 16 * sizeof(float), st) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "map_step: memset failed");
    float *gx = nullptr;
    if (fuse_ib) {
        ENG_BUF(float, gxb, kIbWs, (size_t)m_rows * 3 * sizeof(float));
        gx = gxb;
    }
    const psvo::InterpFuse ipf{qb.leaf,  qb.ray_of,    q.rank_ray, d->vertex_idx, qb.tt, rays_o, rays_d, d->centres,
                               d->emb,   d->voxel_size, grad_emb,   gx,            mark_into};
    mark(e, st, PSVO_TIME_MLP_BWD, 0);
    // the sparse decoder's class B: its rows at [M, 2 M) of the compact arrays
    const psvo::InterpFuse ipf_b{qb.leaf + M, qb.ray_of + M, q.rank_ray, d->vertex_idx, qb.tt + M, rays_o, rays_d,
                                 d->centres, d->emb, d->voxel_size, grad_emb, gx ? gx + 3 * M : nullptr, mark_into};
    const psvo::TrunkBwd tbw{sel_cnt ? sel_cnt + 1 : nullptr, g_sdf_s + M, h2_src ? qb.feat : qb.feat + M * 16,
                             fuse_ib ? &ipf_b : nullptr, h2_src ? q.h2 : nullptr, h2_src ? h2_src + M : nullptr};
    ENG_CALL(mlp_bwd(st, M, d->width, qb.feat, W[0], W[1], W[2], W[3], W[4], W[5], W[6], W[7], W[8], W[9], q.images,
                     qb.rgb_s, qb.act, qb.masks, g_sdf_s, g_rgb_s, dfeat, G[0], G[1], G[2], G[3], G[4], G[5], G[6],
                     G[7], G[8], G[9], 0, n_split, mlp_ws, overlap ? e->dfeat_ready : nullptr,
                     fuse_ib ? &ipf : nullptr, split ? ax : nullptr, sel_cnt, two_class ? &tbw : nullptr, h2_src));
    mark(e, st, PSVO_TIME_MLP_BWD, 1);
    if (overlap) e->bwd_recorded = true;  // mlp_bwd recorded dfeat_ready on st
    // embedding backward: after dfeat (the fused kernel), beside the weight-gradient reduce
    hipStream_t eb = split ? st : ax;
    if (overlap && eb != st && hipStreamWaitEvent(eb, e->dfeat_ready, 0) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "map_step: stream wait failed");
    if (!fuse_ib && emb_dirty &&
        hipMemsetAsync(grad_emb, 0, (size_t)d->n_emb * 16 * sizeof(float), eb) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "map_step: memset failed");
    e->grads_clean = false;
    e->clean_buf = grad_emb;
    if (fuse_ib) {
        mark(e, eb, PSVO_TIME_INTERP_BWD, 0);
        ENG_CALL(psvo::interp_rays_gx(eb, q.r_hit, qb.offsets, q.rank_ray, qb.tt, gx, grad_od, grad_od + R * 3,
                                      two_class ? offb : nullptr, two_class ? qb.tt + M : nullptr,
                                      two_class ? gx + 3 * M : nullptr));
        mark(e, eb, PSVO_TIME_INTERP_BWD, 1);
    } else {
        mark(e, eb, PSVO_TIME_INTERP_BWD, 0);
        ENG_BUF(float, ib_ws2, kIbWs, psvo_interp_bwd_workspace_floats(q.r_hit, q.s_max) * sizeof(float));
        ENG_CALL(psvo_interp_bwd_chunked(eb, q.r_hit, q.s_max, 16, d->voxel_size, qb.offsets, q.rank_ray, qb.leaf,
                                         qb.tt, rays_o, rays_d, d->centres, d->vertex_idx, d->emb, dfeat, grad_emb,
                                         grad_od, grad_od + R * 3, ib_ws2));
        mark(e, eb, PSVO_TIME_INTERP_BWD, 1);
    }
    if (overlap && eb != st &&
        (hipEventRecord(e->emb_done, eb) != hipSuccess || hipStreamWaitEvent(st, e->emb_done, 0) != hipSuccess))
        return set_error(PSVO_E_LAUNCH, "map_step: stream join failed");
    // the loss value's reads of crit_ws before the next step's writes: through
    // st, or (split) through aux's optimiser step, which the next render waits
    // for; split, st joins it too once the look-ahead is queued (below)
    if (join_loss && hipStreamWaitEvent(split ? ax : st, e->loss_done, 0) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "map_step: stream join failed");
    e->tm.pending = e->tm.on;
    ENG_CALL(guard.release());
    PoseAdam pa;
    // look-ahead (psvo_map_frames.next_dirs_cam): the poses' gradient and
    // Adam step right after the embedding backward on its stream, then the
    // next iteration's rays + query there too — beside this step's weight
    // gradients and the map's Adam
    if (ahead) {
        if (wait_next && hipStreamWaitEvent(eb, e->next_ready, 0) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "map_step: stream wait failed");
        // queued on the step's own stream (split tail): consumed there, no event
        ENG_CALL(frames_lookahead(e, eb, d, fr, R, q, grad_od, eb != st));
    } else if (fr) {
        ENG_CALL(frames_update(e, st, d, fr, q, grad_od, R, &pa));
    }
    // ---- optimiser steps, the poses' with the map's (the map's are skipped
    // when the caller all-reduces the gradients first)
    if (!(flags & PSVO_STEP_NO_ADAM)) {
        hipStream_t os = split ? ax : st;
        ENG_CALL(map_adam(os, d, grads, adam_step, &pa, sparse_rows));
        e->grads_clean = true;
        if (ahead) {  // the next iteration's decoder images, while the look-ahead query runs
            ENG_BUF(float, images, kImages, psvo_mlp_image_floats_w(d->width) * sizeof(float));
            ENG_CALL(mlp_images(os, d->width, W[0], W[1], W[2], W[3], W[4], W[5], W[6], W[7], W[8], W[9], images));
            e->images_next = true;
            e->images_w0 = W[0];
        }
        if (split) {
            if (hipEventRecord(e->adam_done, ax) != hipSuccess)
                return set_error(PSVO_E_LAUNCH, "map_step: event record failed");
            e->adam_pending = true;
        }
    } else {
        ENG_CALL(pose_adam(st, d, pa));
    }
    // the step clock: after the optimiser step, on the stream that ran it (a
    // look-ahead step's: aux, where nothing waits behind the marker) — the
    // same point of every step
    if (e->clk.on && e->clk.n < (int)e->clk.ev.size() &&
        hipEventRecord(e->clk.ev[e->clk.n++], (split && !(flags & PSVO_STEP_NO_ADAM)) ? ax : st) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "map_step: event record failed");
    // split tail: loss_out is written on the loss stream; the caller reads it
    // on st (the loss pass ends long before the look-ahead's pose step, so
    // this wait, queued behind the look-ahead, costs nothing).  The weights
    // stay pending on aux until the next engine call or psvo_map_join.
    if (split && join_loss && hipStreamWaitEvent(st, e->loss_done, 0) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "map_step: stream join failed");
    return PSVO_OK;
}

extern "C" int psvo_engine_grad_rays(psvo_engine *e, void *stream, int64_t n_rays, float *grad_o, float *grad_d) {
    PSVO_REQUIRE(e && grad_o && grad_d && n_rays > 0, "engine_grad_rays: bad arguments");
    const size_t bytes = (size_t)n_rays * 3 * sizeof(float);
    PSVO_REQUIRE(e->a.p[kGradOD] && e->a.cap[kGradOD] >= 2 * bytes, "engine_grad_rays: no step of %lld rays ran",
                 (long long)n_rays);
    const float *g = static_cast<const float *>(e->a.p[kGradOD]);
    hipStream_t st = as_stream(stream);
    if (hipMemcpyAsync(grad_o, g, bytes, hipMemcpyDeviceToDevice, st) != hipSuccess ||
        hipMemcpyAsync(grad_d, g + n_rays * 3, bytes, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "engine_grad_rays: copy failed");
    return PSVO_OK;
}

extern "C" int psvo_map_side_wait(psvo_engine *e, void *stream) {
    PSVO_REQUIRE(e, "map_side_wait: null engine");
    if (!e->dfeat_ready || !e->bwd_recorded) return PSVO_OK;
    if (hipStreamWaitEvent(as_stream(stream), e->dfeat_ready, 0) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "map_side_wait: stream wait failed");
    return PSVO_OK;
}

extern "C" int psvo_map_join(psvo_engine *e, void *stream) {
    PSVO_REQUIRE(e, "map_join: null engine");
    return join_adam(e, as_stream(stream), "map_join");
}

extern "C" int psvo_map_step(psvo_engine *e, void *stream, const psvo_map_desc *d, int64_t n_rays,
                             const float *rays_o, const float *rays_d, const float *gt_rgb, const float *gt_depth,
                             uint64_t seed, int64_t adam_step, int flags, float *loss_out, int *stats_out) {
    return map_step_impl(e, as_stream(stream), d, n_rays, rays_o, rays_d, gt_rgb, gt_depth, nullptr, seed, adam_step,
                         flags, loss_out, stats_out, nullptr);
}

extern "C" int psvo_map_step_frames(psvo_engine *e, void *stream, const psvo_map_desc *d, const psvo_map_frames *fr,
                                    const float *gt_rgb, const float *gt_depth, const float *noise, uint64_t seed,
                                    int64_t adam_step, int flags, float *loss_out, int *stats_out) {
    PSVO_REQUIRE(e && d && fr && fr->dirs_cam && fr->poses && fr->pose_step, "map_step_frames: null argument");
    PSVO_REQUIRE(fr->n_frames > 0 && fr->rays_per_frame > 0, "map_step_frames: bad sizes");
    PSVO_REQUIRE(fr->n_frames <= kXchMaxFrames, "map_step_frames: at most %d keyframes per call (rank)",
                 kXchMaxFrames);
    for (int f = 0; f < fr->n_frames; ++f)
        PSVO_REQUIRE(fr->pose_step[f] < 1 || (fr->pose_m && fr->pose_v), "map_step_frames: pose Adam needs m / v");
    PSVO_REQUIRE(!(fr->next_dirs_cam && noise), "map_step_frames: look-ahead needs drawn (not injected) noise");
    hipStream_t st = as_stream(stream);
    int rc = PSVO_OK;
    const int64_t R = (int64_t)fr->n_frames * fr->rays_per_frame;
    if (e->q_count > 0) {  // the previous call's look-ahead: rays and query made from the updated poses
        const QuerySet &q = e->qs[e->q_head];
        PSVO_REQUIRE(q.dirs != nullptr && q.dirs == fr->dirs_cam && q.R == R && q.seed == seed && !noise,
                     "map_step_frames: dirs_cam / seed differ from the previous call's next_dirs_cam / next_seed");
        return map_step_impl(e, st, d, R, q.ro, q.rd, gt_rgb, gt_depth, nullptr, seed, adam_step, flags, loss_out,
                             stats_out, fr);
    }
    ENG_BUF(float, rays_o, kRaysO, (size_t)R * 3 * sizeof(float));
    ENG_BUF(float, rays_d, kRaysD, (size_t)R * 3 * sizeof(float));
    ENG_CALL(psvo_pose_rays_frames(st, R, fr->rays_per_frame, fr->poses, fr->dirs_cam, rays_o, rays_d));
    return map_step_impl(e, st, d, R, rays_o, rays_d, gt_rgb, gt_depth, noise, seed, adam_step, flags, loss_out,
                         stats_out, fr);
}

extern "C" int psvo_map_query(psvo_engine *e, void *stream, const psvo_map_desc *d, int64_t n_rays,
                              const float *rays_o, const float *rays_d, uint64_t seed) {
    PSVO_REQUIRE(e && d && rays_o && rays_d && n_rays > 0, "map_query: bad arguments");
    e->images_next = false;  // the weights may change before the next step
    PSVO_REQUIRE(e->q_count < 2, "map_query: two queries already queued (run psvo_map_step)");
    hipStream_t st = as_stream(stream);
    if (!e->side) {
        if (hipStreamCreateWithFlags(&e->side, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&e->in_ready, hipEventDisableTiming) != hipSuccess)
            return set_error(PSVO_E_LAUNCH, "map_query: side stream creation failed");
    }
    QuerySet &q = e->qs[(e->q_head + e->q_count) & 1];
    // the rays were produced on the caller's stream; the set's buffers may
    // still be read by the step that consumed it last
    if (hipEventRecord(e->in_ready, st) != hipSuccess || hipStreamWaitEvent(e->side, e->in_ready, 0) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "map_query: stream ordering failed");
    ENG_CALL(freed_wait(q, e->side));
    // (a buffer that must grow syncs the side stream first, which includes that wait)
    ENG_CALL(query_enqueue(e, e->side, q, d, n_rays, rays_o, rays_d, seed, "map_query"));
    q.pending = true;
    e->q_count++;
    return PSVO_OK;
}

extern "C" int psvo_track_step(psvo_engine *e, void *stream, const psvo_map_desc *d, int64_t n_rays,
                               const float *dirs_cam, const float *gt_rgb, const float *gt_depth, float *pose,
                               float *pose_m, float *pose_v, double lr, const float *noise, uint64_t seed,
                               int64_t adam_step, int flags, float *pose_grad, float *loss_out, int *stats_out) {
    PSVO_REQUIRE(e && d && dirs_cam && gt_rgb && gt_depth && pose && loss_out, "track_step: null argument");
    e->images_next = false;  // the weights may change before the next step
    PSVO_REQUIRE(n_rays > 0 && adam_step >= 1, "track_step: bad sizes");
    PSVO_REQUIRE(d->width == 128 || d->width == 256, "track_step: decoder width %d unsupported (fused: 128, 256)",
                 d->width);
    PSVO_REQUIRE((flags & PSVO_STEP_NO_ADAM) || (pose_m && pose_v), "track_step: Adam needs pose_m / pose_v");
    hipStream_t st = as_stream(stream);
    int rc = PSVO_OK;
    const int64_t R = n_rays;
    // ---- world rays from the pose (render_helpers.py:714-716)
    ENG_BUF(float, rays_o, kRaysO, (size_t)R * 3 * sizeof(float));
    ENG_BUF(float, rays_d, kRaysD, (size_t)R * 3 * sizeof(float));
    ENG_CALL(psvo_pose_rays(stream, R, pose, dirs_cam, rays_o, rays_d));
    Render q;
    PSVO_REQUIRE(e->q_count == 0, "track_step: the engine has queued mapping queries");
    PSVO_REQUIRE(!e->x.on(), "track_step: tracking runs on one GPU (SURVEY §8e: its median filter is global)");
    QuerySet *qset = nullptr;
    ENG_CALL(take_query(e, st, d, R, rays_o, rays_d, seed, "track_step", &qset, noise));
    QueryGuard guard{e, st, qset};
    ENG_CALL(render(e, st, d, *qset, rays_o, rays_d, false, stats_out, "track_step", q));
    // ---- loss (optionally with the median depth filter) and backward
    float *dtmp = nullptr, *dthr = nullptr;
    if (flags & PSVO_TRACK_DEPTH_FILTER) {
        ENG_BUF(float, tbuf, kDTmp, (size_t)q.r_hit * sizeof(float) + 64);
        dtmp = tbuf;
        dthr = tbuf + ((q.r_hit + 15) / 16) * 16;
        ENG_CALL(psvo_criterion_depth_filter(stream, q.r_hit, q.s_max, q.rank_ray, gt_depth, q.depth, q.weights,
                                             q.z_vals, dtmp, dthr));
    }
    float *g_sdf_s, *g_rgb_s;
    ENG_CALL(loss_backward(e, st, d, q, gt_rgb, gt_depth, dtmp, dthr, loss_out, &g_sdf_s, &g_rgb_s));
    // frozen map: decoder backward to the features only, interpolation
    // backward to the rays only (no embedding scatter)
    const int64_t M = q.m;
    ENG_BUF(float, dfeat, kDfeat, M * 16 * sizeof(float));
    const int n_split = 256;
    ENG_BUF(float, mlp_ws, kMlpWs, psvo_mlp_workspace_floats_w(M, d->width, n_split) * sizeof(float));
    float *const *W = d->dec;
    mark(e, st, PSVO_TIME_MLP_BWD, 0);
    ENG_CALL(psvo_mlp_bwd(stream, M, d->width, q.feat, W[0], W[1], W[2], W[3], W[4], W[5], W[6], W[7], W[8], W[9],
                          q.images, q.rgb_s, nullptr, q.masks, g_sdf_s, g_rgb_s, dfeat, nullptr, nullptr, nullptr,
                          nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, n_split, mlp_ws));
    mark(e, st, PSVO_TIME_MLP_BWD, 1);
    ENG_BUF(float, grad_od, kGradOD, (size_t)R * 6 * sizeof(float));
    mark(e, st, PSVO_TIME_INTERP_BWD, 0);
    ENG_CALL(psvo_interp_bwd(stream, q.r_hit, 16, d->voxel_size, q.offsets, q.rank_ray, q.leaf, q.tt, rays_o, rays_d,
                             d->centres, d->vertex_idx, d->emb, dfeat, nullptr, grad_od, grad_od + R * 3));
    mark(e, st, PSVO_TIME_INTERP_BWD, 1);
    e->tm.pending = e->tm.on;
    ENG_CALL(guard.release());
    // ---- pose gradient through rotation() and the pose's Adam step
    if (!pose_grad) {
        ENG_BUF(float, gbuf, kPoseGrad, 8 * sizeof(float));
        pose_grad = gbuf;
    }
    ENG_CALL(psvo_pose_grad(stream, q.r_hit, q.rank_ray, dirs_cam, grad_od, grad_od + R * 3, pose, pose_grad));
    if (!(flags & PSVO_STEP_NO_ADAM)) {
        int64_t n6 = 6;
        int zero = 0;
        const float *g = pose_grad;
        ENG_CALL(adam_launch(st, 1, &pose, &g, &pose_m, &pose_v, &n6, &lr, d->beta1, d->beta2, d->eps, 0.0, adam_step,
                             &zero));
    }
    return PSVO_OK;
}
