// Internal helpers shared by the psvo HIP translation units (gfx950 only).
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/psvo.h"

namespace psvo {

// Kernel-bound timing (the engine's timed regions, psvo_engine_set_timing):
// while a region is armed every kernel launched through psvo::launch gets
// events bound to its own dispatch (hipExtLaunchKernel) — no marker packets
// between the kernels.  Default: every kernel gets a (start, stop) pair and
// a region is the sum of its kernels' spans (what rocprofv3's kernel trace
// reports for them); PSVO_TIMING_SPAN=1: an instance of a region is timed
// from its first kernel's start to its last kernel's end (only the first
// kernel carries a start event; the gaps between the kernels count).  One
// host thread queues a timed step; regions nest (the innermost open instance
// owns a launch).
struct KernelClock {
    static constexpr int kMax = 192, kMaxInst = 64;
    hipEvent_t ev[kMax][2] = {};
    int region[kMax] = {};        // sum mode: the pair's region
    int n = 0;                    // pairs taken since the last full collection
    struct Inst {
        int region, first, last;  // pair indices (−1: no kernel yet)
    } inst[kMaxInst] = {};
    int n_inst = 0;
    int stack[8] = {};            // open instances (span mode) / regions (sum mode), innermost last
    int depth = 0;
    bool sum = false;
    bool overflow = false;        // more launches / instances than slots: the surplus ran untimed
    hipStream_t streams[4] = {};  // the arming engine's streams: launches on any other stream are not its own
    bool owns(hipStream_t st) const {
        for (hipStream_t s : streams)
            if (s == st) return true;
        return false;
    }
};
// engine.cpp: set while an engine with timing on queues a step, on the thread
// that queues it (another thread's launches, e.g. a tracking engine's, are
// never attributed to it)
extern thread_local KernelClock *g_kclock;

// set by the engine around one launch: that launch's completion records this
// event (bound to the dispatch, no marker packet), unless a kernel clock
// needs the slot — then it is recorded right after the launch, or, with
// g_stop_share, not at all: g_stop_bound names the clock's stop event, which
// marks the same completion (the caller waits on that one before the clock
// reuses it)
extern thread_local hipEvent_t g_stop_event;
extern thread_local bool g_stop_share;
extern thread_local hipEvent_t g_stop_bound;

template <typename... KArgs, typename... A>
inline void launch(void (*k)(KArgs...), dim3 grid, dim3 block, uint32_t lds, hipStream_t st, A &&...a) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    KernelClock *c = g_kclock;
    if (c && c->depth > 0 && c->owns(st)) {
        if (c->n < KernelClock::kMax) {
            const int i = c->n++;
            e1 = c->ev[i][1];
            if (c->sum) {
                c->region[i] = c->stack[c->depth - 1];
                e0 = c->ev[i][0];
            } else {
                KernelClock::Inst &I = c->inst[c->stack[c->depth - 1]];
                if (I.first < 0) {
                    I.first = i;
                    e0 = c->ev[i][0];
                }
                I.last = i;
            }
        } else {
            c->overflow = true;
        }
    }
    hipEvent_t late = nullptr;
    if (g_stop_event) {
        if (!e1)
            e1 = g_stop_bound = g_stop_event;
        else if (g_stop_share)
            g_stop_bound = e1;
        else
            late = g_stop_bound = g_stop_event;
        g_stop_event = nullptr;
    }
    hipExtLaunchKernelGGL(k, grid, block, lds, st, e0, e1, 0u, static_cast<KArgs>(a)...);
    if (late) (void)hipEventRecord(late, st);
}

// Set the thread-local error message; returns `code` for tail calls.
int set_error(int code, const char *fmt, ...);

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// Check the most recent launch.  Never exits the process (the reference's
// CUDA_CHECK_ERRORS calls exit(-1), cuda_utils.h:37-48): the binding raises.
int check_launch(const char *what);

// the look-back controls of site 1 (traversal), 2 (sampler) or 4 (sample
// selection): lookback.h's kLbSpinMax and no delay unless
// psvo_debug_set_lookback set them
struct LbCtl;
LbCtl lb_ctl(int site);
// look-back blocks helped (lookback.h): traversal + sampler, selection
int lb_helps_query(int64_t *out2, bool reset);
int lb_helps_select(int64_t *out1, bool reset);

// multi-tensor Adam launch (optim.hip): per-tensor lr, optional per-tensor
// step numbers (steps: else `step` for all), optional gradient zeroing
int adam_launch(hipStream_t st, int n_tensors, float *const *params, const float *const *grads, float *const *exp_avg,
                float *const *exp_avg_sq, const int64_t *numel, const double *lr, double beta1, double beta2,
                double eps, double weight_decay, int64_t step, const int *zero_grad, const int64_t *steps = nullptr,
                const uint8_t *const *row_flags = nullptr);

constexpr int kWave = 64;
constexpr int kMaxHits = 50;        // voxel_helpers.py:561 (n_max hard-coded)
constexpr int kSamplerG = 200;      // voxel_helpers.py:300
constexpr int kSamplerChunk = 800;  // voxel_helpers.py:331 (4 * G)
constexpr float kMaxDepthFill = 10.0f;  // voxel_helpers.py:24 MAX_DEPTH

inline int div_up(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// records the packed traversal's top start tests per ray (two per lane;
// svo_query.hip top_start, tree_pack.hip k_pt_top): more would cost more
// AABB work than the rounds they save (room0's first 512 records: five times
// the tests of a whole walk)
#ifndef PSVO_PACK_TOP_MAX
#define PSVO_PACK_TOP_MAX 128
#endif
constexpr int kPackTopMax = PSVO_PACK_TOP_MAX;  // a multiple of 64, <= 512

// one octree node as the packed traversal reads it (tree_pack.hip)
struct PackRec {  // 32 B, 16-B aligned
    float4 c;     // centre x, y, z; side (int bits)
    int4 i;       // reference node id, first child record (-1: none), child mask, spare (tree_pack.hip)
};

// the query's statistics words → coherent pinned host memory as {seq, value}
// granules (stat_to_host; zeroing them on the device): the engine's host
// thread polls the tags instead of waiting for an event (svo_query.hip)
// zero: clear the words read (the query set's next use needs no memset);
// false for a first read-back that later kernels of the query still extend
int stats_to_host(hipStream_t st, int *stats, unsigned long long *host, int words, int seq, bool zero = true);
// the same granules from the statistics' device copy, which stays as it is
// The Criterion's normalisers (criterion.py:70-101: the valid-depth rays and
// the front / sdf samples over the padded [R_hit, S_max] layout) depend only
// on the samples' depths and the rays' GT depth, so the sampler counts them
// per ray as it emits samples (ray_cnt i32[R]) and its last workgroup turns
// the sums into the backward coefficients coef f32[4] (crit_coef_from_counts:
// k_crit_coef's bits).  gt_depth null: not counted.
struct SampleCounts {
    const float *gt_depth;
    int *ray_cnt;
    float *coef;
    float tr, max_depth, w_rgb, w_depth, w_fs, w_sdf;
    int crit_flags;
};
// psvo_sample_rays (single GPU, whole batch) whose scan also does
// stats_to_host's read-back (svo_query.hip); with counts also the
// normalisers.  lb_desc (query_lookback): the scan runs inside the sampler
// launch by look-back (lookback.h) over the descriptors after the
// traversal's (lookback_granules(r_hit_cap) granules, tag ≠ 0 fresh per
// query), the rows hold only their valid prefix, and with leaf / t / ray_of
// (capacity r_hit_cap · max_steps_cap) the launch also does k_compact_rays'
// compaction
int sample_rays_to_host(hipStream_t st, int64_t r_hit_cap, int max_steps_cap, const int *rank_ray, const int *hit_idx,
                        const float *hit_t0, const float *hit_t1, const float *ray_dsum, float step_size,
                        const float *noise, uint64_t seed, int *stats, int *s_idx, float *s_depth, float *s_dist,
                        int *ray_ns, int *offsets, unsigned long long *host, int seq,
                        const SampleCounts *counts = nullptr, unsigned long long *lb_desc = nullptr,
                        uint32_t lb_tag = 0, int *leaf = nullptr, float *t = nullptr, int *ray_of = nullptr,
                        int *m_out = nullptr,  // with the compaction: M on the device
                        const int *nv_rank = nullptr, const int *col0_rank = nullptr);  // intersect_ranked's copies
// whether a query of r rays runs its statistics / rank pass and its sample
// scan by look-back (up to kLbMaxRays rays), and its descriptor granules
constexpr int64_t kLbMaxRays = 16384;  // 8 rays per workgroup: 2,048 workgroups, within lookback.h's 64 · 64
constexpr int kLbIsGranules = 5, kLbSmpGranules = 8;
// statistics words [kStatQuery, +3): the traversal's P / R_hit / max ⌈steps⌉
// again, for the look-back sampler — never zeroed by a read-back, so a
// sampler workgroup that starts after the launch's last one zeroed words
// [0, kStatQuery) still reads this batch's values (lookback.h helping)
constexpr int kStatQuery = 13;
static_assert(kStatQuery + 3 <= PSVO_STAT_WORDS, "statistics words");
bool query_lookback(int64_t r);
int64_t lookback_granules(int64_t r);

// one element of the Adam step (k_adam; optim.hip's formulation), shared so
// the fused pose step (pose.hip) computes the same bits
__device__ __forceinline__ void adam_elem(float &p, float g, float &m, float &v, float beta1, float beta2, float omb1,
                                          float omb2, float eps, float wd, float lr_bc1, float bc2_sqrt) {
    if (wd != 0.0f) g = g + wd * p;
    const float mi = beta1 * m + omb1 * g;
    const float vi = beta2 * v + omb2 * g * g;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p = p - lr_bc1 * mi / denom;
    m = mi;
    v = vi;
}

// the bundle-adjust pose work (pose.hip), over each frame's rays directly
// (ray_rank[r] >= 0: a hit ray; the engine's sums — one fixed order for both
// calls): the frames' pose gradients (k_pose_grad_rays), and the
// look-ahead's whole pose step in one launch, one block per keyframe — the
// gradient, its Adam step when steps[f] >= 1 (k_adam's arithmetic, lr / bc1
// and sqrt(bc2) formed on the host as adam_launch does), then the frame's
// next rays (k_pose_rays_frames) from the updated pose
// the interpolation forward over the device's sample count m_dev <= m_cap
// (interp.hip; psvo_interp_fwd's arithmetic)
int interp_fwd_dev(hipStream_t st, int64_t m_cap, const int *m_dev, float voxel_size, const int *leaf, const float *t,
                   const int *ray_of_sample, const int *ray_index, const float *rays_o, const float *rays_d,
                   const float *centres, const int *vertex_idx, const float *emb, float *feat);
int pose_grad_frames_rays(hipStream_t st, int n_frames, int64_t rays_per_frame, const int *ray_rank,
                          const float *dirs, const float *g_o, const float *g_d, const float *poses, float *grads);
int pose_step_frames(hipStream_t st, int n_frames, int64_t rays_per_frame, const int *ray_rank, const float *dirs,
                     const float *g_o, const float *g_d, float *poses, float *pose_m, float *pose_v,
                     const int64_t *steps, double lr, double beta1, double beta2, double eps, float *grads,
                     const float *next_dirs, float *rays_o, float *rays_d);

int intersect_ranked(hipStream_t st, int64_t n_rays, const float *rays_o, const float *rays_d, const float *centres,
                     const int *structure, float voxel_size, float max_distance, float step_size, int *hit_idx,
                     float *hit_t0, float *hit_t1, int *ray_nv, float *ray_dsum, int *stats, int *ray_rank,
                     int *rank_ray, const PackRec *packed = nullptr, int *blk_out = nullptr,
                     unsigned long long *lb_desc = nullptr, uint32_t lb_tag = 0,
                     int *nv_rank = nullptr, int *col0_rank = nullptr, int64_t n_nodes = 0);  // look-back: by-rank hit count, first id

// data-parallel query (svo_query.hip): rows of the slot-0 count table for a
// union batch of at most max_rays_global rays; the words one rank
// contributes to the query's first all-gather (8 words + a hit-count byte per
// hit row, for at most max_rays_rank rays); pack them; union statistics +
// slot-0 count table from the gathered words; the sampler over the rank's
// rows; after the second all-gather ([S_max, 7 count words] per rank) the
// union S_max and normaliser sums
constexpr int kDistWordsPerRank = 8;
// word 0 of a rank's second-gather words: its S_max, with this bit set when
// it did not count its rows (no GT depths given to its query)
constexpr int kDistNotCounted = 1 << 30;
// PSVO_STAT_FLAGS bit set by k_dist_smax when some rank did not count: every
// rank then counts in its step (one decision for all ranks, so all issue the
// same collectives)
constexpr int PSVO_FLAG_UNION_UNCOUNTED = 16;
int dist_slot0_rows(int64_t max_rays_global);
int dist_count_words(int max_rays_rank);
int dist_pack(hipStream_t st, int64_t R, const int *stats, const int *rank_ray, const int *hit_idx,
              const int *ray_nv, int *out, const int *nv_rank = nullptr, int flags_or = 0);
// (q2_in: this rank's words of the second gather, whose count words it
// zeroes, or null: the caller zeroes them on the stream of dist_counts)
int dist_layout(hipStream_t st, const int *all, int world, int rank, int stride, int nch, int *stats, int *table,
                int *q2_in);
int dist_sample(hipStream_t st, int64_t r_hit_cap, int max_steps_cap, const int *rank_ray, const int *hit_idx,
                const float *hit_t0, const float *hit_t1, const float *ray_dsum, float step_size, uint64_t seed,
                int *stats, const int *table, int nch, int *s_idx, float *s_depth, float *s_dist, int *ray_ns,
                int *offsets, const int *nv_rank = nullptr, const int *col0_rank = nullptr);
int dist_smax(hipStream_t st, const int *all, int world, int *stats, int *in, double *sums);
// this rank's words of the second gather: in[0] = S_max of its rows; given
// the GT depths, in[1..7] += n_valid, Σ front / Σ sdf-band over the valid
// samples, and per padding class (front, band: sample_terms of the MAX_DEPTH
// fill) the rays and their Σ ns — in[1..7] zeroed before (criterion.hip)
int dist_counts(hipStream_t st, int64_t R, const int *stats, const int *rank_ray, const float *gt_depth,
                const float *z_rows, int z_stride, const int *ray_ns, float truncation, float max_depth, int *in);

// psvo_criterion_coef split at the count sums (criterion.hip)
int criterion_counts(hipStream_t st, int64_t r_hit, int s_max, float truncation, float max_depth, const int *rank_ray,
                     const float *gt_depth, const float *z_vals, int z_stride, const int *ray_ns, float *workspace,
                     double *sums);
int criterion_coef_from_sums(hipStream_t st, const double *sums, int64_t n_hit, int n_cols, float truncation,
                             float rgb_w, float depth_w, float fs_w, float sdf_w, int flags, float *coef);

// psvo_criterion_coef / psvo_composite_loss reading z from rows of stride
// z_stride >= s_max (the sampler's [R, cap] depth rows, the engine's mapping
// path: no padded [R_hit, S_max] copy; ray_ns: the rows' valid samples, past
// which MAX_DEPTH is implied — the look-back sampler writes no padding)
int criterion_coef_z(void *stream, int64_t r_hit, int s_max, float truncation, float max_depth, const int *rank_ray,
                     const float *gt_depth, const float *z_vals, int z_stride, const int *ray_ns, float rgb_w,
                     float depth_w, float fs_w, float sdf_w, int flags, float *workspace, double *sums, float *coef);
int composite_loss_z(void *stream, int64_t r_hit, int s_max, float truncation, float max_depth, const int *offsets,
                     const int *ray_ns, const float *z_vals, int z_stride, const int *rank_ray, const float *gt_rgb,
                     const float *gt_depth, const float *sdf_s, const float *rgb_s, const float *coef,
                     float *workspace, float *color, float *depth, float *grad_sdf_s, float *grad_rgb_s,
                     bool partials = true,  // false: no loss partials (the loss value is not wanted)
                     const int *cidx = nullptr);  // the sparse decoder's compact sample index (select_samples)
// The sparse decoder's sample selection (composite.hip k_select_samples):
// the samples whose gradients can be non-zero get compact, ray-major indices
// cidx[s] (-1: dropped) — class A (composited: the whole decoder) at
// [0, M_A), class B (only a loss term: the decoder trunk) at [cap, cap + M_B)
// (split = false: every kept sample in class A) —, the classes' compact ray
// offsets offa / offb [R_hit + 1] and compact copies of their features /
// leaf / t / ray ([2 cap] arrays; split: class B's colour rows of rgb_c
// [2 cap][3] are written 0 — their composite weights are 0; src_c [2 cap],
// if not null: each kept sample's index in the step's sample order).  counts[0] = M_A, counts[1] = M_B (the
// compact decoder launches read them on the device), counts[2] |= 8 if the
// look-back wait was abandoned (then both are 0; with host_flag — coherent
// pinned memory — bit 3 is also set there for the host); counts + 4: u64 running
// sums of kept / composited samples and of launches (kSelCountInts ints,
// zeroed once).  desc: select_granules(r_hit) granules, zeroed once; tag
// fresh per launch (≠ 0).
constexpr int kSelCountInts = 10;
int select_samples(hipStream_t st, int64_t r_hit, int s_max, float truncation, float max_depth, const int *offsets,
                   const int *ray_ns, const float *z_vals, int z_stride, const int *rank_ray, const float *gt_depth,
                   const float *sdf_s, const float *feat, const int *leaf, const float *t, const int *ray_of,
                   int64_t cap, bool split, int *cidx, int *offa, int *offb, float *feat_c, int *leaf_c, float *t_c,
                   int *ray_of_c, float *rgb_c, int *src_c, int *counts, unsigned long long *desc, uint32_t tag,
                   int *host_flag = nullptr);
int select_rays_per_wave(int64_t r_hit);
int64_t select_granules(int64_t r_hit);
// sample compaction alone, one wave per hit ray (svo_query.hip k_compact_rays):
// the valid prefix of each sampler row → leaf / t / ray_of_sample at offsets[r] + s
int compact_rays(hipStream_t st, int64_t r_hit, int cap, const int *s_idx, const float *s_depth, const int *offsets,
                 int *leaf, float *t, int *ray_of_sample);

// width-256 decoder (mlp256.hip): sizes, operand images, forward (act /
// masks NULL: inference), backward (gw[0] NULL: δ chain to dfeat only)
int64_t dec256_tiles16(int64_t m);
int64_t dec256_image_floats();
int64_t dec256_act_floats(int64_t m);
int64_t dec256_mask_words(int64_t m);
int64_t dec256_workspace_floats(int64_t m);
int dec256_images(hipStream_t st, const float *w1, const float *b1, const float *w2, const float *b2, const float *w3,
                  const float *b3, const float *w4, const float *b4, const float *w5, const float *b5, float *images);
// rgb, act and masks all null: the sdf trunk only (k_dec256_trunk, the same sdf
// bits).  m_dev: the sample count read on the device (<= m; buffers sized for m)
int dec256_fwd(hipStream_t st, int64_t m, const float *feat, const float *images, float *sdf, float *rgb, float *act,
               uint64_t *masks, const int *m_dev = nullptr);
struct InterpFuse;
// ip (the mapping engine's width-256 step): the interpolation backward runs
// inside the δ-chain kernel (dfeat is then not stored), as at width 128
int dec256_bwd(hipStream_t st, int64_t m, const float *feat, const float *images, const float *rgb, const float *act,
               const uint64_t *masks, const float *g_sdf, const float *g_rgb, float *dfeat, float *const gw[5],
               float *const gb[5], int accumulate, float *workspace, hipEvent_t dfeat_ready,
               const InterpFuse *ip = nullptr, const int *m_dev = nullptr);

constexpr int kXchMaxFrames = 64;  // keyframes per psvo_map_step_frames call

// ---- in-launch hand-offs between workgroups --------------------------------
// (cdna_hip_programming.md §6 G16, sc1 form; the per-XCD L2s are not
// coherent).  Every word another workgroup reads in the same launch is stored
// write-through (sc1: a relaxed agent-scope atomic store on a global pointer)
// and read back with sc1 loads, so no release / acquire fence (an L2
// write-back / invalidate) is needed (lookback.h's descriptors).
typedef __attribute__((address_space(1))) int g_i32;
typedef __attribute__((address_space(1))) float g_f32;
typedef __attribute__((address_space(1))) unsigned long long g_u64;
__device__ __forceinline__ void st_wt(int *p, int v) {
    __hip_atomic_store((g_i32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(float *p, float v) {
    __hip_atomic_store((g_f32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_wt(const int *p) {
    return __hip_atomic_load((g_i32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float *p) {
    return __hip_atomic_load((g_f32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// query statistics to the host: PSVO_STAT_WORDS 8-byte granules {seq, value}
// written by relaxed system-scope stores into coherent pinned memory — each
// word carries its own tag, so no system-scope release (an L2 write-back on
// the critical stream) orders them; the host polls until every tag is seq
__device__ __forceinline__ void stat_to_host(unsigned long long *host, int word, int v, int seq) {
    __hip_atomic_store((g_u64 *)(host + word), ((unsigned long long)(unsigned)seq << 32) | (unsigned)v,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// the Criterion's backward coefficients from the batch's count sums
// (criterion.py:70-101; k_crit_coef and the sampler's tail share this, so
// both give the same bits): coef = {colour, depth, fs, sdf}; flags PSVO_CRIT_USE_*
__device__ __forceinline__ void crit_coef_from_counts(double n_valid_d, double n_f_d, double n_s_d, double n_hit,
                                                      double n_cols, float rgb_w, float depth_w, float fs_w,
                                                      float sdf_w, float tr, int flags, float *coef) {
    const double n_el = n_hit * n_cols;
    const float n_valid = (float)n_valid_d;
    const float n_f = (float)n_f_d, n_s = (float)n_s_d;
    const float n_tot = n_s + n_f;
    const float fs_weight = 1.0f - n_f / n_tot;
    const float sdf_weight = 1.0f - n_s / n_tot;
    coef[0] = (flags & PSVO_CRIT_USE_COLOR) ? (float)(rgb_w / (3.0 * n_hit)) : 0.0f;
    coef[1] = (flags & PSVO_CRIT_USE_DEPTH) ? depth_w / n_valid : 0.0f;
    coef[2] = (flags & PSVO_CRIT_USE_SDF) ? (float)(2.0 * (double)(fs_w * fs_weight) / n_el) : 0.0f;
    coef[3] = (flags & PSVO_CRIT_USE_SDF) ? (float)(2.0 * (double)(sdf_w * sdf_weight) / n_el) * tr : 0.0f;
}

// The interpolation backward (interp.hip's k_interp_bwd: embedding scatter
// and dL/dx) folded into the width-128 fused decoder backward, per 16-sample
// unit right after its dfeat: grad_emb (zeroed by the caller) += the
// trilinear scatter, gx[M][3] = dL/dx of every sample (psvo_interp_rays_gx
// sums them per ray into d_o / d_d).  Engine only (mlp_bwd `ip`).
struct InterpFuse {
    const int *leaf, *ray_of, *rank_ray, *vertex_idx;
    const float *t, *rays_o, *rays_d, *centres, *emb;
    float voxel_size;
    float *grad_emb;
    float *gx;
    uint8_t *row_flags;  // or null: every embedding row the scatter touches is flagged (sparse-exact Adam)
};

// d_o / d_d of every hit ray from the samples' dL/dx (InterpFuse::gx);
// offsets2 / t2 / gx2 (or null): a second segment of each ray (the sparse
// decoder's class B), summed after the first
int interp_rays_gx(hipStream_t st, int64_t r_hit, const int *offsets, const int *ray_index, const float *t,
                   const float *gx, float *grad_o, float *grad_d, const int *offsets2 = nullptr,
                   const float *t2 = nullptr, const float *gx2 = nullptr);

// psvo_mlp_bwd that records `dfeat_ready` (if not null) on the stream once
// dfeat is written, before the weight-gradient kernels are queued; with `ip`
// (width 128, fused backward) it also runs the interpolation backward and
// dfeat is not stored.  m_dev (width 128; the sparse decoder): the sample
// count is read on the device (select_samples' counts[0] <= m; the buffers
// are sized for m).
// the sparse decoder's class B (k_mlp_trunk_fb after k_mlp_bwd3, width 128:
// the trunk's forward recomputed and its backward in one kernel): its count
// on the device, dL/dsdf, the features and the fused interpolation backward
struct TrunkBwd {
    const int *m_dev;
    const float *g_sdf, *feat;
    const InterpFuse *ip;
    const float *h2 = nullptr;  // or: the step's h2 rows (H2Rows) and each class-B sample's row —
    const int *src = nullptr;   // the W2 layer is read instead of recomputed; feat then holds the
                                // step's rows too (x of sample s: row src[s])
};
int mlp_bwd(void *stream, int64_t m, int width, const float *feat, const float *w1, const float *b1, const float *w2,
            const float *b2, const float *w3, const float *b3, const float *w4, const float *b4, const float *w5,
            const float *b5, const float *images, const float *rgb, const float *act, const uint64_t *masks,
            const float *g_sdf, const float *g_rgb, float *dfeat, float *gw1, float *gb1, float *gw2, float *gb2,
            float *gw3, float *gb3, float *gw4, float *gb4, float *gw5, float *gb5, int accumulate, int n_split,
            float *workspace, hipEvent_t dfeat_ready, const InterpFuse *ip = nullptr,
            hipStream_t reduce_stream = nullptr, const int *m_dev = nullptr, const TrunkBwd *tb = nullptr,
            const int *x_src = nullptr);  // x_src (width 128): sample s's x is row x_src[s] of feat
// whether mlp_bwd can take `ip` for this width (the fused width-128 backward is built and selected)
bool mlp_bwd_fuses_interp(int width);
// the look-ahead's split tail (psvo_map_step_frames): the weight-gradient
// slab sum and the optimiser on the side stream beside the next query — width
// 128 only (the width-256 weight-gradient kernel holds every CU)
bool mlp_bwd_split_tail(int width);

// the decoder's LDS operand images (k_mlp_prep) on their own, and
// psvo_mlp_fwd without rebuilding them (the engine prepares them on its aux
// stream beside the sampler / interpolation kernels)
int mlp_images(void *stream, int width, const float *w1, const float *b1, const float *w2, const float *b2,
               const float *w3, const float *b3, const float *w4, const float *b4, const float *w5, const float *b5,
               float *images);
// the sparse decoder's h2 hand-over (width 128): the sdf-only forward
// (rgb == nullptr) writes every sample's h2 as row-major rows into `out`
// [m][128]; the full forward (k_mlp_fwd2) reads sample s's h2 from row src[s]
// of `rows` instead of recomputing the W2 layer (the same instructions made
// it: the same bits) — and its x from row src[s] of `feat` (the step's
// features, no compact copy)
struct H2Rows {
    float *out = nullptr;
    const float *rows = nullptr;
    const int *src = nullptr;
};
int mlp_fwd_prepared(void *stream, int64_t m, int width, const float *feat, const float *w1, const float *b1,
                     const float *w2, const float *b2, const float *w3, const float *b3, const float *w4,
                     const float *b4, const float *w5, const float *b5, float *images, float *sdf, float *rgb,
                     float *act, uint64_t *masks, const int *m_dev = nullptr,
                     const H2Rows *h2 = nullptr);  // m_dev: as mlp_bwd (width 128)

}  // namespace psvo

#define PSVO_REQUIRE(cond, ...)                                       \
    do {                                                              \
        if (!(cond)) return ::psvo::set_error(PSVO_E_INVALID, __VA_ARGS__); \
    } while (0)
