/*
 * psvo — MI355X-native sparse-voxel-octree renderer: C ABI.
 *
 * Plain pointers and sizes only; every device pointer is HBM memory owned by
 * the caller; every call is asynchronous on `stream` (a hipStream_t passed as
 * void*) and returns PSVO_OK or an error code (psvo_last_error() gives the
 * message).  No call allocates, frees or synchronises, so callers may capture
 * sequences into a hipGraph.
 *
 * Reference interfaces replaced (DARYL-GWZ/Proud-SLAM):
 *   psvo_svo_intersect            grid.svo_intersect
 *                                 third_party/sparse_voxels/src/intersect.cpp:83-112,
 *                                 intersect_gpu.cu:191-270, :415-426
 *   psvo_inverse_cdf_sampling     grid.inverse_cdf_sampling
 *                                 third_party/sparse_voxels/src/sample.cpp:56-95,
 *                                 sample_gpu.cu:133-239, :255-269
 *   psvo_ball_intersect / psvo_aabb_intersect / psvo_triangle_intersect
 *                                 grid.ball_intersect / aabb_intersect / triangle_intersect
 *                                 intersect.cpp:15-42, :49-76, :119-146; intersect_gpu.cu:13-187, :273-362
 *   psvo_uniform_ray_sampling     grid.uniform_ray_sampling sample.cpp:21-54, sample_gpu.cu:13-124
 *   psvo_build_octree             grid.build_octree octree.cpp:12-164 (CPU, host memory)
 *   psvo_ray_intersect_sorted     voxel_helpers.ray_intersect_vox (voxel_helpers.py:557-595)
 *                                 + SparseVoxelOctreeRayIntersect (:110-166), fused
 *   psvo_hit_rank / psvo_sample_rays / psvo_sample_points
 *                                 render_helpers.render_rays ray/sample compaction
 *                                 (render_helpers.py:390-460) + voxel_helpers.ray_sample
 *                                 (voxel_helpers.py:637-663) + InverseCDFRaySampling (:288-374)
 *   psvo_interp_fwd / _bwd        render_helpers.get_features_vox (render_helpers.py:104-156)
 *                                 forward and its autograd backward
 *   psvo_composite_fwd / _bwd     render_helpers.render_rays compositing (render_helpers.py:504-556)
 *   psvo_mlp_fwd / _bwd           variations/nrgbd.Decoder forward + autograd backward
 *                                 (nrgbd.py:80-146), fused fp32 MFMA
 *   psvo_criterion_*              criterion.Criterion.forward + autograd backward
 *                                 (criterion.py:17-116)
 *   psvo_adam_step                torch.optim.Adam.step of the mapping loop
 *                                 (render_helpers.py:581-596, :668-672)
 *   psvo_map_step                 one bundle_adjust_frames iteration (render_helpers.py:609-672):
 *                                 render_rays + Criterion + backward + both Adam steps
 *   psvo_share_*                  share.ShareData (src/share.py:27-166) served by a BaseManager
 *                                 (voxslam.py:28-33): update_share_data (mapping.py:236-248) /
 *                                 do_tracking (tracking.py:114-125) state exchange, device-resident
 *   psvo_octree_*                 torch.classes.svo.Octree (third_party/sparse_octree/src/bindings.cpp:4-35,
 *                                 octree.cpp:104-294, :561-687) — CPU builder, host memory
 */
#ifndef PSVO_H
#define PSVO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    PSVO_OK = 0,
    PSVO_E_INVALID = 1,   /* bad argument (shape / size / null pointer) */
    PSVO_E_LAUNCH = 2,    /* HIP launch or runtime error */
    PSVO_E_OVERFLOW = 3,  /* DFS stack overflow (reference: assert(ptr < 256)) */
    PSVO_E_BUSY = 4,      /* share channel: no free slot within the timeout */
    PSVO_E_SYSTEM = 5     /* share channel: shared-memory / OS error */
};

const char *psvo_last_error(void);
const char *psvo_version(void);

/* ---- drop-in `grid` kernels (reference layouts) ----------------------- */

/* ray_start/ray_dir f32[b,m,3]; points f32[b,n,3]; children i32[b,n,9];
 * outputs idx i32 / min_depth f32 / max_depth f32 [b,m,n_max] (idx -1 when
 * unused; depths 0 there).  Hits in DFS emission order, children popped 7→0. */
int psvo_svo_intersect(void *stream, int b, int n, int m, float voxelsize, int n_max, const float *ray_start,
                       const float *ray_dir, const float *points, const int *children, int *idx, float *min_depth,
                       float *max_depth);

/* One reference launch over a contiguous [b, num_rays, max_hits] chunk; the
 * outputs [b, num_rays, max_steps] must be pre-filled (-1 / 0 / 0). */
int psvo_inverse_cdf_sampling(void *stream, int b, int num_rays, int max_hits, int max_steps,
                              float fixed_step_size, const int *pts_idx, const float *min_depth,
                              const float *max_depth, const float *uniform_noise, const float *probs,
                              const float *steps, int *sampled_idx, float *sampled_depth, float *sampled_dists);

/* The `grid` functions off the render path (csrc/grid_aux.hip), reference
 * layouts; outputs pre-filled by the caller as the reference allocates them
 * (zeros; -1 for sampled_idx).  ball / aabb: the first n_max hits in point
 * order, idx -1 after.  triangle: face_points f32[b,n,9]; the first n_max
 * hits in face order sorted by depth (ties in face order); depth
 * f32[b,m,3·n_max] = (t, -gap/2 capped, +gap/2 capped), uv f32[b,m,2·n_max];
 * n_max <= 2048.  uniform sampling: pts_idx/min/max [b,num_rays,max_hits],
 * noise and outputs [b,num_rays,max_steps]. */
int psvo_ball_intersect(void *stream, int b, int n, int m, float radius, int n_max, const float *ray_start,
                        const float *ray_dir, const float *points, int *idx, float *min_depth, float *max_depth);
int psvo_aabb_intersect(void *stream, int b, int n, int m, float voxelsize, int n_max, const float *ray_start,
                        const float *ray_dir, const float *points, int *idx, float *min_depth, float *max_depth);
int psvo_triangle_intersect(void *stream, int b, int n, int m, float cagesize, float blur, int n_max,
                            const float *ray_start, const float *ray_dir, const float *face_points, int *idx,
                            float *depth, float *uv);
int psvo_uniform_ray_sampling(void *stream, int b, int num_rays, int max_hits, int max_steps, float step_size,
                              const int *pts_idx, const float *min_depth, const float *max_depth,
                              const float *uniform_noise, int *sampled_idx, float *sampled_depth,
                              float *sampled_dists);
/* grid.build_octree on the host: n int64 points [n,3] under a root centred at
 * center[3] (f32) of the given depth.  Sets *total (nodes) and *terminal
 * (leaves = n); writes centers i32[total,3] and children i32[total,9] only
 * when capacity >= total (call with capacity 0 first to size them).
 * PSVO_E_INVALID for depth outside [0, 29] or two points in one leaf slot
 * (*total = the second point's index). */
int psvo_build_octree(const float *center, const int64_t *points, int64_t n, int depth, int64_t capacity,
                      int *centers, int *children, int64_t *total, int64_t *terminal);

/* ---- fused render path ------------------------------------------------ */

/* Device-side statistics written by the query stages (int32 words).       */
enum {
    PSVO_STAT_P = 0,         /* max valid hits over rays (voxel_helpers.py:582) */
    PSVO_STAT_R_HIT = 1,     /* rays with >= 1 hit */
    PSVO_STAT_MAX_CEIL = 2,  /* max ceil(steps) over hit rays (voxel_helpers.py:320) */
    PSVO_STAT_S_MAX = 3,     /* max valid samples per ray (voxel_helpers.py:359) */
    PSVO_STAT_M = 4,         /* total valid samples */
    PSVO_STAT_VISITS = 5,    /* AABB tests performed (traffic accounting) */
    PSVO_STAT_SPILLS = 6,    /* rays that fell back to the serial DFS (diagnostic) */
    PSVO_STAT_FLAGS = 7,     /* bit 0: DFS stack overflow; bit 1: sampler exceeded max_steps */
    /* data-parallel engine (psvo_engine_set_exchange): words 0..3 then describe
     * the GLOBAL batch (P, R_hit, max ceil, S_max over all ranks) and these the
     * rank's own rows */
    PSVO_STAT_ROW_BEGIN = 8,     /* first global logical hit row of this rank */
    PSVO_STAT_R_HIT_LOCAL = 9,   /* this rank's hit rays */
    PSVO_STAT_NEXT_COL0 = 10,    /* first voxel id of the global row after this rank's last */
    PSVO_STAT_S_MAX_LOCAL = 11,  /* this rank's max valid samples per ray */
    PSVO_STAT_ROUNDS = 12,       /* traversal rounds of the wave-per-ray intersect, summed over rays (diagnostic) */
    PSVO_STAT_WORDS = 16
};

/* DFS + stable sort by t_in + max_distance trim for R rays.  hit_* are
 * [R, 50] (sorted valid prefix, then -1 / max_distance fills); ray_nv[R]
 * valid-hit count; ray_dsum[R] = Σ(t_out - t_in) in sorted order.
 * `stats` (PSVO_STAT_WORDS int32, zeroed by the caller) receives P, R_hit,
 * max ceil(Σ/step) and the visit count. */
int psvo_ray_intersect_sorted(void *stream, int64_t n_rays, const float *rays_o, const float *rays_d,
                              const float *centres, const int *structure, float voxel_size, float max_distance,
                              float step_size, int *hit_idx, float *hit_t0, float *hit_t1, int *ray_nv,
                              float *ray_dsum, int *stats);

/* The octree breadth-first with siblings contiguous, one 32-B record per
 * node {f32 cx, cy, cz, side (int bits) | i32 reference id, first child
 * record, child mask, 0} (csrc/tree_pack.hip), built on the device from the
 * reference arrays: packed = n_nodes x 32 B (16-B aligned), workspace
 * psvo_pack_tree_workspace_ints(n_nodes) ints.  Valid until the map changes. */
int64_t psvo_pack_tree_workspace_ints(int64_t n_nodes);
int psvo_pack_tree(void *stream, int64_t n_nodes, const float *centres, const int *structure, int *workspace,
                   void *packed);
/* psvo_ray_intersect_sorted reading the packed records (same results, the
 * reference ids); centres / structure serve the serial-DFS fallback. */
int psvo_ray_intersect_sorted_packed(void *stream, int64_t n_rays, const float *rays_o, const float *rays_d,
                                     const void *packed, const float *centres, const int *structure, float voxel_size,
                                     float max_distance, float step_size, int *hit_idx, float *hit_t0, float *hit_t1,
                                     int *ray_nv, float *ray_dsum, int *stats);

/* ray_rank[R] = rank among hit rays or -1; rank_ray[R_hit] = original ray. */
int psvo_hit_rank(void *stream, int64_t n_rays, const int *ray_nv, int *ray_rank, int *rank_ray);

/* Inverse-CDF sampling of the R_hit hit rays with the reference's logical
 * [200, K', P] layout (K' = ceil(R_hit/200), 800-slot launch chunks): P,
 * R_hit and max_steps are read from `stats` on the device.  noise is either
 * NULL (counter-based uniform from `seed`, clamped to [0.001, 0.999]) or
 * f32[200, K', max_steps] with values in [0, 1).  Outputs [R_hit,
 * max_steps_cap] with max_steps_cap >= stats[P] + stats[MAX_CEIL]; per-ray
 * valid counts to ray_ns[R_hit], their exclusive scan to offsets[R_hit+1];
 * S_max / M into stats. */
int psvo_sample_rays(void *stream, int64_t r_hit_cap, int max_steps_cap, const int *rank_ray, const int *hit_idx,
                     const float *hit_t0, const float *hit_t1, const float *ray_dsum, float step_size,
                     const float *noise, uint64_t seed, int *stats, int *s_idx, float *s_depth, float *s_dist,
                     int *ray_ns, int *offsets);

/* psvo_sample_rays for the logical hit rows [row_begin, row_begin + n_rows)
 * (n_rows < 0: through R_hit), outputs at row - row_begin.  rank_ray,
 * hit_*, ray_dsum and stats (P / R_hit / max ceil) describe the GLOBAL ray
 * batch (all ranks' rays concatenated): a data-parallel rank samples its own
 * rays inside the single-GPU [200, K', P] layout — the sampler quirks of
 * voxel_helpers.py:300-317 / sample_gpu.cu:224-237 and the noise depend on
 * the global slot.  S_max / M of the range go to stats. */
int psvo_sample_rays_range(void *stream, int64_t row_begin, int64_t n_rows, int64_t r_hit_cap, int max_steps_cap,
                           const int *rank_ray, const int *hit_idx, const float *hit_t0, const float *hit_t1,
                           const float *ray_dsum, float step_size, const float *noise, uint64_t seed, int *stats,
                           int *s_idx, float *s_depth, float *s_dist, int *ray_ns, int *offsets);

/* P, R_hit and max ceil(Σ(t_out - t_in) / step) of n_rays intersected rays
 * into stats (the reduction psvo_ray_intersect_sorted ends with). */
int psvo_ray_stats(void *stream, int64_t n_rays, const int *ray_nv, const float *ray_dsum, float step_size,
                   int *stats);

/* Exclusive scan of per-ray sample counts → sample offsets. */
int psvo_scan_counts(void *stream, int64_t n, const int *counts, int *offsets);

/* Compact valid samples (ray-major): leaf[M], t[M], ray[M]; z_vals and mask
 * [R_hit, S_max] (z = 10 where invalid, render_helpers.py:418-460). */
int psvo_sample_points(void *stream, int64_t r_hit, int s_max, int max_steps_cap, const int *s_idx,
                       const float *s_depth, const int *ray_ns, const int *offsets, int *leaf, float *t,
                       int *ray_of_sample, float *z_vals, uint8_t *mask);

/* Trilinear interpolation of vertex embeddings at x = o[row] + d[row]*t with
 * row = ray_index[ray_of_sample] (ray_index NULL: row = ray_of_sample).
 * centres f32[N,3]; vertex_idx i32[N,8]; emb f32[E,D] with D == 16. */
int psvo_interp_fwd(void *stream, int64_t m, int d, float voxel_size, const int *leaf, const float *t,
                    const int *ray_of_sample, const int *ray_index, const float *rays_o, const float *rays_d,
                    const float *centres, const int *vertex_idx, const float *emb, float *feat);

/* Backward of psvo_interp_fwd given grad_feat[M,D]: accumulates into
 * grad_emb[E,D] (float atomics, caller zeroes) and writes grad_o / grad_d at
 * the rows ray_index[r] (or r) of the R_hit hit rays (other rows untouched).
 * Samples must be ray-major (offsets[R_hit+1]). */
int psvo_interp_bwd(void *stream, int64_t r_hit, int d, float voxel_size, const int *offsets, const int *ray_index,
                    const int *leaf, const float *t, const float *rays_o, const float *rays_d, const float *centres,
                    const int *vertex_idx, const float *emb, const float *grad_feat, float *grad_emb, float *grad_o,
                    float *grad_d);

/* psvo_interp_bwd with each ray's samples split into 64-sample work units
 * (one wave each), so the launch is not serialised behind the longest rays;
 * the per-unit d_o / d_d partials (workspace f32[psvo_interp_bwd_workspace_
 * floats(r_hit, s_max)]) are summed per ray in unit order (deterministic).
 * Same embedding gradient; d_o / d_d equal up to fp32 summation order. */
int64_t psvo_interp_bwd_workspace_floats(int64_t r_hit, int s_max);
int psvo_interp_bwd_chunked(void *stream, int64_t r_hit, int s_max, int d, float voxel_size, const int *offsets,
                            const int *ray_index, const int *leaf, const float *t, const float *rays_o,
                            const float *rays_d, const float *centres, const int *vertex_idx, const float *emb,
                            const float *grad_feat, float *grad_emb, float *grad_o, float *grad_d, float *workspace);

/* SDF-to-weight compositing (render_helpers.py:504-556) per hit ray.
 * sdf_s[M], rgb_s[M,3] per valid sample; outputs sdf/weights [R_hit,S_max]
 * (sdf padded with 1), color [R_hit,3], depth [R_hit]. */
int psvo_composite_fwd(void *stream, int64_t r_hit, int s_max, float truncation, const int *offsets,
                       const int *ray_ns, const float *z_vals, const float *sdf_s, const float *rgb_s,
                       float *sdf, float *weights, float *color, float *depth, float *z_min);

/* Backward of psvo_composite_fwd: given grad_color[R_hit,3], grad_depth[R_hit],
 * grad_weights[R_hit,S_max] (may be NULL) and grad_sdf[R_hit,S_max] (may be
 * NULL), writes grad_sdf_s[M] and grad_rgb_s[M,3]. */
int psvo_composite_bwd(void *stream, int64_t r_hit, int s_max, float truncation, const int *offsets,
                       const int *ray_ns, const float *z_vals, const float *sdf, const float *weights,
                       const float *rgb_s, const float *grad_color, const float *grad_depth,
                       const float *grad_weights, const float *grad_sdf, float *grad_sdf_s, float *grad_rgb_s);

/* Mapping-step fusion of psvo_composite_fwd, psvo_criterion_sums' per-ray
 * partials, psvo_criterion_bwd (d loss = 1) and psvo_composite_bwd
 * (grad_weights = 0) in one pass per hit ray — same arithmetic.  coef f32[4]
 * = the backward coefficients from psvo_criterion_coef; workspace as
 * psvo_criterion_sums' (the count slots already filled by
 * psvo_criterion_coef; this fills the others, so psvo_criterion_reduce +
 * psvo_criterion_finalize then give the loss).  Writes color [R_hit,3],
 * depth [R_hit], grad_sdf_s [M], grad_rgb_s [M,3]. */
int psvo_composite_loss(void *stream, int64_t r_hit, int s_max, float truncation, float max_depth,
                        const int *offsets, const int *ray_ns, const float *z_vals, const int *rank_ray,
                        const float *gt_rgb, const float *gt_depth, const float *sdf_s, const float *rgb_s,
                        const float *coef, float *workspace, float *color, float *depth, float *grad_sdf_s,
                        float *grad_rgb_s);

/* ---- NRGBD decoder (nrgbd.py:80-146; width 128 or 256, in 16, depth 2) -- */
/* Weights in torch nn.Linear layout ([out][in] row-major): W1[128,16],
 * W2[128,128], W3[129,128] (row 0 = sdf), W4[128,144] ([f | x] columns),
 * W5[3,128].  Forward: feat[M,16] → sdf[M], rgb[M,3] (sigmoid applied).
 * `images` (psvo_mlp_image_floats() floats) receives the weights' LDS operand
 * images, rebuilt by every call; psvo_mlp_bwd reuses them (same weights).
 * Training mode: masks u64[M][2][3] (ReLU masks, needed by any psvo_mlp_bwd)
 * and act f32[4][ceil(M/64)*64*128] (h1, h2, f, c1 in 32-sample CF tiles, see
 * mlp.hip; needed only for weight gradients) are written when non-NULL;
 * act requires masks.  Inference: both NULL; rgb NULL as well: the sdf
 * alone (Decoder.get_sdf, mesh lattices — h1, h2 and W3's sdf row only).
 * Width 256 (W1[256,16], W2[256,256], W3[129,256], W4[256,144], W5[3,256];
 * mlp256.hip): images psvo_mlp_image_floats_w(256), act / masks as sized by
 * psvo_mlp_act_floats / psvo_mlp_mask_words (16-sample tiles); rgb NULL
 * skips only the rgb stores. */
int64_t psvo_mlp_image_floats(void);
/* width-aware sizes (width 128 or 256; -1 otherwise): operand images, the
 * training forward's activations (act) and ReLU masks (u64 words), the
 * backward's workspace */
int64_t psvo_mlp_image_floats_w(int width);
int64_t psvo_mlp_act_floats(int64_t m, int width);
int64_t psvo_mlp_mask_words(int64_t m, int width);
int64_t psvo_mlp_workspace_floats_w(int64_t m, int width, int n_split);
int psvo_mlp_fwd(void *stream, int64_t m, int width, const float *feat, const float *w1, const float *b1,
                 const float *w2, const float *b2, const float *w3, const float *b3, const float *w4,
                 const float *b4, const float *w5, const float *b5, float *images, float *sdf, float *rgb,
                 float *act, uint64_t *masks);

/* Floats of device workspace psvo_mlp_bwd needs for m samples. */
int64_t psvo_mlp_workspace_floats(int64_t m, int n_split);

/* Backward given g_sdf[M], g_rgb[M,3] and the training forward's rgb / act /
 * masks: writes dfeat[M,16] and the 10 parameter gradients (overwrite, or
 * add when `accumulate`); split-K over ~n_split sample ranges with a
 * deterministic slab reduction.  gw1 == NULL (frozen decoder, e.g.
 * tracking): dfeat only — act may then be NULL and the other gradient
 * pointers are ignored. */
int psvo_mlp_bwd(void *stream, int64_t m, int width, const float *feat, const float *w1, const float *b1,
                 const float *w2, const float *b2, const float *w3, const float *b3, const float *w4,
                 const float *b4, const float *w5, const float *b5, const float *images, const float *rgb,
                 const float *act, const uint64_t *masks, const float *g_sdf, const float *g_rgb, float *dfeat, float *gw1, float *gb1,
                 float *gw2, float *gb2, float *gw3, float *gb3, float *gw4, float *gb4, float *gw5, float *gb5,
                 int accumulate, int n_split, float *workspace);

/* ---- mapping loss (criterion.py:17-116) ------------------------------ */
/* out[] words written by psvo_criterion_finalize */
enum {
    PSVO_CRIT_LOSS = 0, PSVO_CRIT_COLOR = 1, PSVO_CRIT_DEPTH = 2, PSVO_CRIT_FS = 3, PSVO_CRIT_SDF = 4,
    PSVO_CRIT_FS_WEIGHT = 5, PSVO_CRIT_SDF_WEIGHT = 6, /* 7..10: backward coefficients */
    PSVO_CRIT_OUT_WORDS = 16
};
enum { PSVO_CRIT_USE_COLOR = 1, PSVO_CRIT_USE_DEPTH = 2, PSVO_CRIT_USE_SDF = 4 };

/* Floats of workspace psvo_criterion_sums needs. */
int64_t psvo_criterion_workspace_floats(int64_t r_hit);

/* Loss sums over the R_hit hit rays: gt_rgb f32[R,3] / gt_depth f32[R] are
 * indexed through rank_ray[R_hit]; colour [R_hit,3], depth [R_hit], sdf and
 * z_vals [R_hit,S_max] as psvo_composite_fwd / psvo_sample_points produce.
 * sums f64[8] = {Σ|Δrgb|, Σ_valid |Δd|, n_valid, n_front, n_sdf, Σ fs², Σ sdf², 0}
 * (fixed-order, deterministic).  pad_extra > 0 adds that many padded samples
 * (z = 10, sdf = 1) per ray — for a shard whose S_max is below the global
 * one, so that all-reduced sums equal the single-GPU sums. */
int psvo_criterion_sums(void *stream, int64_t r_hit, int s_max, int pad_extra, float truncation, float max_depth,
                        const int *rank_ray, const float *gt_rgb, const float *gt_depth, const float *color,
                        const float *depth, const float *sdf, const float *z_vals, float *workspace, double *sums);

/* Loss and its parts from (possibly all-reduced) sums over n_hit rays ×
 * s_max columns; flags = PSVO_CRIT_USE_* terms; out f32[PSVO_CRIT_OUT_WORDS]. */
int psvo_criterion_finalize(void *stream, const double *sums, int64_t n_hit, int s_max, float rgb_w, float depth_w,
                            float fs_w, float sdf_w, float truncation, int flags, float *out);

/* The Criterion's normalisers depend only on z_vals and the GT depth
 * (criterion.py:78-101): counts n_valid / n_front / n_sdf into workspace's
 * count slots, their sums into sums f64[8], and the backward coefficients
 * coef f32[4] = {c_colour, c_depth, c_fs, c_sdf} exactly as
 * psvo_criterion_finalize derives them — before the decoder has run. */
int psvo_criterion_coef(void *stream, int64_t r_hit, int s_max, float truncation, float max_depth,
                        const int *rank_ray, const float *gt_depth, const float *z_vals, float rgb_w, float depth_w,
                        float fs_w, float sdf_w, int flags, float *workspace, double *sums, float *coef);
/* Fixed-order reduction of the workspace's per-ray partials into sums f64[8]. */
int psvo_criterion_reduce(void *stream, int64_t r_hit, const float *workspace, double *sums);

/* Backward given g_loss (device scalar): g_color [R_hit,3], g_depth [R_hit],
 * g_sdf [R_hit,S_max]. */
int psvo_criterion_bwd(void *stream, int64_t r_hit, int s_max, float truncation, float max_depth, const int *rank_ray,
                       const float *gt_rgb, const float *gt_depth, const float *color, const float *depth,
                       const float *sdf, const float *z_vals, const float *out, const float *g_loss, float *g_color,
                       float *g_depth, float *g_sdf);

/* Tracking's weight_depth_loss filter (criterion.py:45-49) over the R_hit
 * hit rays (R_hit ≤ 16384): dtmp f32[R_hit] = |gt_d − depth| /
 * sqrt(Σ_s w·(depth − z)² + 1e-10) from psvo_composite_fwd's weights, and
 * dthr f32[1] = 10 · torch.median(dtmp) (lower middle element). */
int psvo_criterion_depth_filter(void *stream, int64_t r_hit, int s_max, const int *rank_ray, const float *gt_depth,
                                const float *depth, const float *weights, const float *z_vals, float *dtmp,
                                float *dthr);
/* psvo_criterion_sums / _bwd with the depth filter: a ray's depth term is
 * valid only if also dtmp[r] < dthr[0] (both NULL: no filter). */
int psvo_criterion_sums_ex(void *stream, int64_t r_hit, int s_max, int pad_extra, float truncation, float max_depth,
                           const int *rank_ray, const float *gt_rgb, const float *gt_depth, const float *color,
                           const float *depth, const float *sdf, const float *z_vals, const float *dtmp,
                           const float *dthr, float *workspace, double *sums);
int psvo_criterion_bwd_ex(void *stream, int64_t r_hit, int s_max, float truncation, float max_depth,
                          const int *rank_ray, const float *gt_rgb, const float *gt_depth, const float *color,
                          const float *depth, const float *sdf, const float *z_vals, const float *out,
                          const float *g_loss, const float *dtmp, const float *dthr, float *g_color, float *g_depth,
                          float *g_sdf);

/* ---- camera pose (tracking, csrc/pose.hip) ---------------------------- */
/* pose f32[6] = [t | w] (se3pose.py:8-98, R = I + A·[w]× + B·[w]×², Taylor
 * A/B): rays_o[r] = t, rays_d[r] = R·dirs[r] (render_helpers.py:714-716). */
int psvo_pose_rays(void *stream, int64_t n, const float *pose, const float *dirs, float *rays_o, float *rays_d);
/* grad f32[6] = dL/d[t | w] from per-ray grad_o / grad_d of the R_hit hit
 * rays at rows rank_ray[r] (psvo_interp_bwd's output), through rotation(). */
/* Several keyframes (bundle_adjust_frames, render_helpers.py:620-640): poses
 * f32[F][6], frame f owns rays [f·rays_per_frame, (f+1)·rays_per_frame);
 * grads f32[F][8] ([dL/dt | dL/dw | 0 0]) over each frame's hit rays. */
int psvo_pose_rays_frames(void *stream, int64_t n, int64_t rays_per_frame, const float *poses, const float *dirs,
                          float *rays_o, float *rays_d);
int psvo_pose_grad_frames(void *stream, int n_frames, int64_t rays_per_frame, int64_t r_hit, const int *rank_ray,
                          const float *dirs, const float *g_o, const float *g_d, const float *poses, float *grads);
int psvo_pose_grad(void *stream, int64_t r_hit, const int *rank_ray, const float *dirs, const float *g_o,
                   const float *g_d, const float *pose, float *grad);

/* ---- mesh extraction (csrc/mesh.hip; mesh_util.py:80-169) -------------
 * On the SURFACE voxels (centres f32[n,3], vertex_idx i32[n,8]) of
 * Mapping.extract_mesh (mapping.py:420-431). */
/* The marching-cubes case table (host copy): ntri[256], tri[256][36] cube
 * edge ids (edge = axis·4 + o1 + 2·o2; corner b = (b&1, b>>1&1, b>>2&1)). */
int psvo_mesh_case_table(int8_t *ntri, int8_t *tri);
/* torch.linspace(-0.5, 0.5, res) as the CPU computes it (host call). */
int psvo_mesh_linspace(int res, float *out);
/* get_scores' lattice features (render_helpers.py:243-294): feat f32[n·res³,16],
 * voxel-major, lattice (i,j,k) row-major, x = lin[i,j,k]·voxel + centre. */
int psvo_mesh_grid_feat(void *stream, int64_t n_vox, int res, float voxel_size, const float *centres,
                        const int *vertex_idx, const float *emb, float *feat);
/* eval_points' features (render_helpers.py:297-328) at xyz f32[n,3] in voxel
 * rows row i32[n] (row < 0: zero features). */
int psvo_mesh_point_feat(void *stream, int64_t n, float voxel_size, const float *xyz, const int *row,
                         const float *centres, const int *vertex_idx, const float *emb, float *feat);
/* Marching cubes over sdf f32[n·res³] (res ≤ 16), per voxel, skipping voxels
 * without a sign change (mesh_util.py:149-169): count vertices nv / triangles
 * nt i32[n], exclusive offsets vbase / tbase i64[n] and totals i64[2] = {V, F}
 * (device); then emit verts f32[V,3] = ((lattice pos)/(res−1) − ½)·voxel +
 * centre and faces i32[F,3] (vertex ids, voxel-major, normals towards sdf > 0). */
int psvo_mesh_mc_count(void *stream, int64_t n_vox, int res, const float *sdf, int *nv, int *nt, int64_t *vbase,
                       int64_t *tbase, int64_t *totals);
int psvo_mesh_mc_emit(void *stream, int64_t n_vox, int res, float voxel_size, const float *sdf, const float *centres,
                      const int *nv, const int64_t *vbase, const int64_t *tbase, float *verts, int *faces);
/* Vertex colours' voxel lookup (mesh_util.py:112-125): row[v] = the row of
 * voxels f32[n,4] whose min corner equals verts[v] // voxel (torch floor
 * division), −1 if none; table: i32[4·psvo_mesh_vox_map_slots(n)] scratch. */
int64_t psvo_mesh_vox_map_slots(int64_t n_vox);
int psvo_mesh_vertex_rows(void *stream, int64_t n_vox, const float *voxels, int64_t n_verts, const float *verts,
                          float voxel_size, int *table, int *row);

/* ---- optimiser ------------------------------------------------------- */
/* One Adam step (torch.optim.Adam, amsgrad off) over n_tensors f32 tensors:
 * host arrays of device pointers and element counts; `step` is the step
 * number after increment (bias corrections 1 - beta^step). */
/* Sparse-exact Adam support for the embedding table (16 floats per row):
 * mark the vertex rows of M samples' leaves (leaf i32[M], vertex_idx
 * i32[N,8]) in flags u8[n_emb]; flag the rows whose Adam moments are
 * non-zero (a state carried over from an optimiser). */
int psvo_adam_mark_rows(void *stream, int64_t m, const int *leaf, const int *vertex_idx, uint8_t *flags);
int psvo_adam_flags_from_state(void *stream, int64_t n_rows, const float *exp_avg, const float *exp_avg_sq,
                               uint8_t *flags);
int psvo_adam_step(void *stream, int n_tensors, float *const *params, const float *const *grads,
                   float *const *exp_avg, float *const *exp_avg_sq, const int64_t *numel, double lr, double beta1,
                   double beta2, double eps, double weight_decay, int64_t step);

/* ---- native mapping iteration ---------------------------------------- */
typedef struct psvo_engine psvo_engine;  /* owns a device workspace arena */

typedef struct psvo_map_desc {
    /* map (device): centres f32[N,3], structure i32[N,9], vertex_idx i32[N,8] */
    int64_t n_nodes;
    const float *centres;
    const int *structure;
    const int *vertex_idx;
    /* embeddings f32[n_emb,16] and their Adam moments (updated in place) */
    float *emb;
    int64_t n_emb;
    float *emb_m, *emb_v;
    /* decoder W1,b1,...,W5,b5 (psvo_mlp_fwd layout) and Adam moments */
    float *dec[10];
    float *dec_m[10];
    float *dec_v[10];
    int width; /* 128 (Replica) or 256 (ScanNet / ARKit) */
    float voxel_size, step_size, max_distance, truncation, max_depth;
    float w_rgb, w_depth, w_fs, w_sdf; /* Criterion weights (criterion.py:8-13) */
    double lr_emb, lr_dec, beta1, beta2, eps;
    /* optional flat gradient buffer f32[psvo_map_grad_floats(n_emb)]:
     * [embeddings | W1, b1, ..., W5, b5]; NULL = engine-owned */
    float *grad_flat;
    /* optional psvo_pack_tree records of this map: the query traverses them
     * (same results); NULL = the reference arrays */
    const void *packed;
    /* optional u8[n_emb] sticky flags of the embedding rows ever touched: a
     * single-GPU step marks its samples' vertex rows and Adam steps only the
     * flagged rows (an untouched row has g = m = v = 0: the dense step leaves
     * it unchanged, so the result is the same).  Initialise from a bound
     * optimiser state with psvo_adam_flags_from_state.  NULL = dense Adam.
     * Data parallel: the step does not mark them (every rank must hold the
     * union of all ranks' rows); the gradient exchange marks the rows it
     * exchanged (psvo_rows_mark / psvo_rows_flags_from_grad) and
     * psvo_map_adam steps the flagged rows. */
    uint8_t *emb_row_flags;
    /* optional u8[n_emb], data parallel only: the rows THIS rank's step
     * touched (marked by the step, cleared by the exchange,
     * psvo_rows_compact_flagged / psvo_rows_clear): the row-sparse exchange
     * finds them without a pass over the gradient table. */
    uint8_t *emb_row_local;
} psvo_map_desc;

/* psvo_map_step / psvo_map_step_frames flags: NO_ADAM stops after the
 * gradients (then psvo_map_adam); NO_LOSS skips the loss value (loss_out is
 * not written — the gradients do not need it; data parallel, every rank must
 * pass the same flags: the loss sums' collective is skipped too) */
enum { PSVO_STEP_NO_ADAM = 1, PSVO_STEP_NO_LOSS = 4 };

int64_t psvo_map_grad_floats(int64_t n_emb);                 /* width 128 */
int64_t psvo_map_grad_floats_w(int64_t n_emb, int width);

/* ---- keyframe pixel sampling (csrc/pixels.hip) ----------------------------
 * Replaces sample_util.sample_rays (src/utils/sample_util.py:4-20) as called
 * by frame.sample_rays (src/frame.py:83-85) for every keyframe in every
 * bundle_adjust_frames iteration (render_helpers.py:620-640), plus the three
 * boolean-mask gathers that follow it (:625-633).  Per frame f: the k pixels
 * of [n_pix] with the largest score log(w/(Σw + 1e-7) + 1e-7) +
 * g(u), g(u) = −log(−log(u + 1e-7) + 1e-7), all in f32 as the reference
 * computes them; weights NULL = all ones (frame.py:84); Σw over the frame, or
 * over all frames when joint_sum (sample_rays on a [B, H, W] mask); u f32
 * [F, n_pix] when given (parity), else a counter-based 24-bit uniform from
 * seed.  Ties at the k-th score are taken in pixel order.  Outputs, in pixel
 * (= row-major mask) order: idx i64[F, k]; per frame the bool mask and the
 * gathered rows of dirs / rgb / depth into out_* [F·k, 3] / [F·k, 3] / [F·k]
 * (any NULL skips it).  workspace: psvo_sample_pixels_workspace_ints ints. */
typedef struct psvo_pixel_frame {
    const float *dirs;   /* [n_pix, 3] camera ray directions (frame.rays_d), or NULL */
    const float *rgb;    /* [n_pix, 3], or NULL */
    const float *depth;  /* [n_pix], or NULL */
    uint8_t *mask;       /* [n_pix] bool out (frame.sample_mask), or NULL */
} psvo_pixel_frame;
int64_t psvo_sample_pixels_workspace_ints(int n_frames, int64_t n_pix);
int psvo_sample_pixels(void *stream, int n_frames, int64_t n_pix, int64_t k, const float *weights, int joint_sum,
                       const float *u, uint64_t seed, const psvo_pixel_frame *frames, int *workspace, int64_t *idx,
                       float *out_dirs, float *out_rgb, float *out_depth);

/* ---- row-sparse gradient exchange (data parallel on large maps, §8e) ---- */
/* Ints of workspace psvo_rows_compact needs for n_rows rows. */
int64_t psvo_rows_workspace_ints(int64_t n_rows);
/* Pack the rows of grad f32[n_rows, width] with a non-zero element: ids
 * i32[count] ascending, rows f32[count, width]; count → device int.  Replaces
 * the dense all-reduce of the embedding gradient (GradBucket / the engine's
 * flat bucket) when a step touches few rows of a large table. */
int psvo_rows_compact(void *stream, int64_t n_rows, int width, const float *grad, int *workspace, int *ids,
                      float *rows, int *count);
/* grad[ids[i]] += rows[i] for i < n_list (ids unique within the list; ids < 0
 * are padding and skipped).  Applying every rank's list in rank order gives
 * every rank the same sums, bit for bit. */
int psvo_rows_scatter_add(void *stream, int64_t n_list, int width, const int *ids, const float *rows, float *grad);
/* psvo_rows_compact over the rows with flags[r] != 0 (n_rows bytes read, not
 * the table; a flagged all-zero row is listed too). */
int psvo_rows_compact_flagged(void *stream, int64_t n_rows, int width, const float *grad, const uint8_t *flags,
                              int *workspace, int *ids, float *rows, int *count);
/* grad[ids[i]] = 0 and, if flags, flags[ids[i]] = 0 for i < n_list (ids < 0 skipped). */
int psvo_rows_clear(void *stream, int64_t n_list, int width, const int *ids, float *grad, uint8_t *flags);
/* flags[ids[i]] = 1 for i < n_list (ids < 0 skipped). */
int psvo_rows_mark(void *stream, int64_t n_list, const int *ids, uint8_t *flags);
/* flags[r] = 1 for every row of grad f32[n_rows, width] with a non-zero element. */
int psvo_rows_flags_from_grad(void *stream, int64_t n_rows, int width, const float *grad, uint8_t *flags);

psvo_engine *psvo_engine_new(void);
void psvo_engine_free(psvo_engine *e);
/* Data-parallel mapping: one process per GPU, each rank steps
 * its own shard of the ray batch and the engine computes the loss of the
 * UNION batch — the single-GPU result on all ranks' rays concatenated in rank
 * order.  The engine calls `fn` for each collective, on the stream the
 * operands were produced on (the collective must be ordered on it):
 *   PSVO_XCH_GATHER_I32: xi32[out + r·count + k] = rank r's xi32[in + k]
 *   PSVO_XCH_SUM_I32 / _F64: in-place sum of xi32 / xf64 [in, in + count)
 * PSVO_XCH_QUERY is or-ed into ops issued by psvo_map_query or a
 * psvo_map_step_frames look-ahead (they may run concurrently with the
 * previous step's: use a separate communicator).
 * xi32: psvo_engine_exchange_words(world, max_rays_global, max_rays_rank)
 * device int32 (max_rays_global: rays of the union batch; max_rays_rank:
 * of one rank's shard, 0 = max_rays_global; a larger shard fails the query);
 * xf64: 16 device doubles (count sums, loss sums).  Returns non-zero on
 * failure.  Exchanged per step, query phase: ONE all-gather of 8 words + a
 * hit-count byte per hit ray of the rank (ceil(max_rays_rank / 4) words) —
 * the union layout and the sampler's slot-0 table follow on every rank —
 * then ONE all-gather of 8 words after the sampler (S_max and, when the
 * step's GT depth was known at query time and the loss value is not wanted,
 * the loss normalisers' counts) — issued by the consuming step once its
 * interpolation is queued, on a stream of the engine's own (`stream` is then
 * not the query's), and before the next query's first gather; step phase: the normaliser counts (8
 * doubles summed) only when some rank's query could not count them (one
 * decision for all ranks, from the gathered words: every rank issues the same
 * collectives; a query that counted used the GT depths it was given, which
 * must be the step's), the loss sums
 * (8 doubles) only when the loss value is wanted; then the caller sums
 * grad_flat over ranks (PSVO_STEP_NO_ADAM) before psvo_map_adam.  A non-NULL fn turns
 * the protocol on for any world, 1 included (the collectives are then
 * identities: a one-rank communicator drives the whole callback path —
 * tests/test_gpu_rccl.py); fn NULL turns it off. */
enum { PSVO_XCH_GATHER_I32 = 1, PSVO_XCH_SUM_I32 = 2, PSVO_XCH_SUM_F64 = 3, PSVO_XCH_QUERY = 0x100 };
typedef int (*psvo_exchange_fn)(void *user, int op, int64_t in_off, int64_t out_off, int64_t count, void *stream);
int64_t psvo_engine_exchange_words(int world, int64_t max_rays_global, int64_t max_rays_rank);
int psvo_engine_set_exchange(psvo_engine *e, int rank, int world, int64_t max_rays_global, int64_t max_rays_rank,
                             psvo_exchange_fn fn, void *user, int *xi32, double *xf64);

/* Queries psvo_map_query queued and no step has consumed yet (0..2).  A step
 * that fails after picking up its queued query still consumes it. */
int psvo_engine_queued(psvo_engine *e);
/* Drop the queued queries (e.g. the look-ahead query of a loop that ended). */
int psvo_map_discard(psvo_engine *e);

/* Which production kernels a mapping step runs, for cross-checks (each form
 * also runs by default elsewhere): PSVO_PATH_QUERY_SPLIT — the query's
 * statistics / rank pass and its sample scan as kernels of their own
 * (k_ray_stats_rank, k_scan_samples: queries above 16,384 rays and the
 * data-parallel sampler) instead of inside the traversal and sampler launches;
 * PSVO_PATH_PADDED — the padded [R_hit, S_max] z copy and the loss
 * normalisers counted in the step (the data-parallel / tracking forward);
 * PSVO_PATH_DENSE_DECODER — the width-128 decoder forward and backward on
 * every sample (the tracking / autograd form) instead of the sparse decoder
 * (the sdf trunk on every sample, the full decoder on the samples whose
 * gradients can be non-zero: composited or inside a loss mask). */
enum { PSVO_PATH_QUERY_SPLIT = 1, PSVO_PATH_PADDED = 2, PSVO_PATH_DENSE_DECODER = 4 };
int psvo_engine_set_paths(psvo_engine *e, int paths);   /* with no query queued */

/* The sparse decoder's sample selection (synchronises `stream`, which must
 * order the engine's steps): out[0] / out[1] kept / composited samples of the
 * last step, out[2] / out[3] their sums since the last reset, out[4] the steps
 * summed; reset != 0 zeroes the sums.  An abandoned look-back wait of any
 * step is reported as an error. */
int psvo_engine_select_stats(psvo_engine *e, void *stream, int64_t *out, int reset);

/* `stream` waits until the last mapping step's sample selection (the sparse
 * decoder's k_select_samples) has run — nothing if no step has.  The
 * keyframe pixel draws of bundle_adjust_frames queue behind it, so that
 * their latency-bound passes run beside the decoder forward / backward
 * instead of beside the selection's look-back. */
int psvo_engine_gate_stream(psvo_engine *e, void *stream);

/* Tests only: the in-launch look-back scans of the sites in `mask` (1
 * traversal, 2 sampler, 4 sample selection) get a spin bound of spin_bound
 * re-reads instead of the bug-trap bound (0: every workgroup with a
 * predecessor gives up at once; -1: the default), and with delay_us > 0 every
 * 4th workgroup (from 1) and every 64th (the tiles' last) waits that long
 * before it starts, so that its successors compute its aggregate themselves
 * (the path a workgroup kept off the CUs by other work takes).  mask 0: the
 * defaults.  Process-wide; takes effect at the next launch. */
int psvo_debug_set_lookback(int mask, int spin_bound, int delay_us);
/* Tests only: look-back blocks helped so far ([0] traversal, [1] sampler,
 * [2] sample selection); reset != 0 zeroes them.  Synchronises the device. */
int psvo_debug_lb_helps(int64_t *out3, int reset);
/* Tests only: psvo_sample_pixels' draw for uniform weights and generated
 * uniforms — 0: the candidate-band draw where it applies (the default), 1:
 * always the radix passes, 2: the band forced to miss (its exact fallback).
 * The three give the same picks.  Process-wide. */
int psvo_debug_set_pixel_draw(int mode);

/* Optional HIP-event timing of the roofline regions (on the launch stream). */
enum { PSVO_TIME_MLP_FWD = 0, PSVO_TIME_MLP_BWD = 1, PSVO_TIME_INTERP_FWD = 2, PSVO_TIME_INTERP_BWD = 3,
       PSVO_TIME_INTERSECT = 4, PSVO_TIME_SAMPLE = 5, PSVO_TIME_POINTS = 6, PSVO_TIME_SELECT = 7,
       PSVO_TIME_REGIONS = 8 };
int psvo_engine_set_timing(psvo_engine *e, int on);        /* resets the accumulators; on = 1: regions serialised
                                                           on one stream, 2: as run (side streams overlap) */
int psvo_engine_timing(psvo_engine *e, double *mean_ms);   /* mean ms per region, -1 if none */
/* The iteration period as the GPU runs it: with max_steps > 0 every mapping
 * step records an event after its optimiser step, on the stream that runs it
 * (the caller's, or the engine's aux stream for a look-ahead step's split
 * tail: the same point of every step; up to max_steps;
 * resets the count; 0 turns it off); psvo_engine_clock gives the mean time
 * between the first and the last recorded event per step (-1 if fewer than
 * two) — synchronises on the last event. */
int psvo_engine_set_clock(psvo_engine *e, int max_steps);
int psvo_engine_clock(psvo_engine *e, double *period_ms, int *n_steps);
/* The host's waits for query statistics (all engines of the process): total
 * microseconds, calls, and calls that found them not yet landed (the GPU set
 * the pace); reset != 0 zeroes the counters. */
int psvo_host_wait_stats(double *wait_us, long long *calls, long long *waited, int reset);

/* One iteration on n_rays rays (rays_o/rays_d f32[R,3], gt_rgb f32[R,3],
 * gt_depth f32[R]): sampler noise from `seed`; Adam bias corrections for
 * step number `adam_step`; flags PSVO_STEP_NO_ADAM stops after the
 * gradients (into desc->grad_flat) so that ranks can all-reduce them and
 * then call psvo_map_adam.  loss_out: device f32[PSVO_CRIT_OUT_WORDS]
 * (PSVO_CRIT_* words); stats_out: host int[PSVO_STAT_WORDS] or NULL.  Two
 * stats read-backs synchronise the stream; everything else is queued. */
/* Queue the query (intersection + sampling + statistics read-back) of the
 * NEXT batch on the engine's side stream, ordered after `stream`'s current
 * position: the step that consumes it (psvo_map_step with the same rays,
 * n_rays and seed) then starts without a read-back stall, and the query runs
 * beside the current step's decoder kernels.  At most two queued; the rays
 * must stay valid until the consuming step. */
int psvo_map_query(psvo_engine *e, void *stream, const psvo_map_desc *d, int64_t n_rays, const float *rays_o,
                   const float *rays_d, uint64_t seed);
int psvo_map_step(psvo_engine *e, void *stream, const psvo_map_desc *d, int64_t n_rays, const float *rays_o,
                  const float *rays_d, const float *gt_rgb, const float *gt_depth, uint64_t seed, int64_t adam_step,
                  int flags, float *loss_out, int *stats_out);

/* One tracking iteration (track_frame's loop body, render_helpers.py:
 * 708-722): world rays from pose f32[6] (device) and camera-frame dirs_cam
 * f32[R,3], render against the frozen map / decoder of `d` (emb, dec read
 * only), Criterion (+ the median depth filter with PSVO_TRACK_DEPTH_FILTER),
 * backward to the pose only, and torch.optim.Adam on the pose (lr, d->beta1,
 * d->beta2, d->eps; moments pose_m / pose_v f32[6]) unless
 * PSVO_STEP_NO_ADAM.  pose_grad: device f32[6] out or NULL.  One stats
 * read-back; loss_out / stats_out as psvo_map_step. */
/* bundle_adjust_frames with update_pose (render_helpers.py:559-676): the
 * iteration's rays come from the keyframes' current poses — frame f's rays
 * are [f·rays_per_frame, (f+1)·rays_per_frame): rays_o = t_f, rays_d =
 * dirs_cam @ R(w_f)ᵀ (:620-640) — and after the backward every keyframe with
 * pose_step[f] ≥ 1 takes its pose Adam step (its own step number, lr_pose;
 * frame.py:27 keyframe.optim) beside Adam(embeddings) / Adam(decoder).
 * poses / pose_m / pose_v: device f32[F][6], updated in place; pose_step:
 * host int64[F] (0: the frame's pose is fixed — stamp 0 or update_pose
 * False); pose_grad: device f32[F][8] output or NULL.  noise: the sampler's
 * uniform noise f32[200, K', max_steps] (voxel_helpers.py:323-328) or NULL
 * (drawn from seed).  No queued psvo_map_query may be pending.  Data parallel
 * (psvo_engine_set_exchange): the keyframes are split over the ranks — each
 * rank passes its own keyframes, whose rays form its part of the union batch
 * (rank order) — so every pose gradient of the union-batch loss is local (no
 * pose exchange); every rank steps the poses it owns.  At most 64 keyframes per call.
 * Look-ahead: with next_dirs_cam (the next iteration's camera directions,
 * same layout; no injected noise) the call also queues the next iteration's
 * query — its rays need this step's pose update, which runs right after the
 * decoder backward, so the next rays, intersection and sampling overlap this
 * step's weight-gradient sum and optimiser step.  The next call must pass
 * dirs_cam == this next_dirs_cam and seed == next_seed; an unconsumed
 * look-ahead is dropped by psvo_map_discard.  next_stream (or NULL: the
 * call's stream): the stream next_dirs_cam (and the next call's gt_rgb /
 * gt_depth) is being produced on; the step orders only its look-ahead pose
 * step after the work queued there so far, not the whole iteration. */
typedef struct psvo_map_frames {
    int n_frames;
    int64_t rays_per_frame;
    const float *dirs_cam;
    float *poses, *pose_m, *pose_v;
    const int64_t *pose_step;
    double lr_pose;
    float *pose_grad;
    const float *next_dirs_cam;  /* NULL: no look-ahead */
    uint64_t next_seed;
    void *next_stream;           /* hipStream_t producing next_dirs_cam, or NULL */
    /* optional: the next call's gt_depth (same storage).  On one GPU with
     * PSVO_STEP_NO_LOSS the look-ahead's sampler then also counts the
     * Criterion's normalisers (criterion.py:70-101), so the next step needs no
     * separate count pass; NULL: the next step counts them itself.  The
     * values are read when the look-ahead runs: they must not change until
     * the consuming call (its counts would no longer match; the engine
     * matches only the pointer).  Rows that may exceed 4095 samples are
     * counted in the next step instead. */
    const float *next_gt_depth;
} psvo_map_frames;
int psvo_map_step_frames(psvo_engine *e, void *stream, const psvo_map_desc *d, const psvo_map_frames *frames,
                         const float *gt_rgb, const float *gt_depth, const float *noise, uint64_t seed,
                         int64_t adam_step, int flags, float *loss_out, int *stats_out);

/* One tracking iteration (track_frame's loop body, render_helpers.py:708-722)
 * on camera-frame directions: world rays from pose [t | w], render, Criterion
 * (PSVO_TRACK_DEPTH_FILTER: weight_depth_loss, the median depth filter),
 * backward to the pose only and its Adam step.  noise: the sampler's uniform
 * noise [200, K', max_steps] as the reference draws it (tests), or NULL:
 * drawn on the device from `seed`. */
enum { PSVO_TRACK_DEPTH_FILTER = 2 };
int psvo_track_step(psvo_engine *e, void *stream, const psvo_map_desc *d, int64_t n_rays, const float *dirs_cam,
                    const float *gt_rgb, const float *gt_depth, float *pose, float *pose_m, float *pose_v, double lr,
                    const float *noise, uint64_t seed, int64_t adam_step, int flags, float *pose_grad,
                    float *loss_out, int *stats_out);

/* Both Adam steps of the iteration from desc->grad_flat (one launch; the
 * embedding gradient is zeroed as it is consumed).  With emb_row_flags the
 * embedding step is row-sparse when the flags are known to hold every row
 * with a gradient: always on one GPU (the step marked them); in data-parallel
 * mode (psvo_engine_set_exchange) only with PSVO_ADAM_ROWS_EXCHANGED — the
 * caller's gradient exchange marked the union of all ranks' rows
 * (psvo_rows_mark / psvo_rows_flags_from_grad).  Otherwise the step is dense
 * and the flags are refreshed from the moments (psvo_adam_flags_from_state)
 * and emb_row_local cleared.  psvo_map_adam = psvo_map_adam_ex(…, 0). */
enum { PSVO_ADAM_ROWS_EXCHANGED = 1 };
int psvo_map_adam(psvo_engine *e, void *stream, const psvo_map_desc *d, int64_t adam_step);
int psvo_map_adam_ex(psvo_engine *e, void *stream, const psvo_map_desc *d, int64_t adam_step, int flags);
/* `stream` waits for the optimiser step a look-ahead psvo_map_step_frames
 * left running on the engine's side stream (its weights are pending until
 * then; every engine call joins it itself). */
int psvo_map_join(psvo_engine *e, void *stream);
/* `stream` waits for the end of the last mapping step's decoder backward
 * (its δ chain; a no-op before the first step).  The pipelined
 * bundle_adjust_frames loop queues its next keyframe pixel draw behind it,
 * so the draw runs beside the latency-bound look-ahead query instead of
 * beside the persistent decoder kernels. */
int psvo_map_side_wait(psvo_engine *e, void *stream);
/* The last mapping step's per-ray loss gradients d rays_o / d rays_d (the
 * interpolation backward's ray sums, what the keyframe pose gradient is
 * formed from) into grad_o / grad_d f32[n_rays, 3], original ray order; rows
 * of rays that hit nothing are undefined.  n_rays must be that step's. */
int psvo_engine_grad_rays(psvo_engine *e, void *stream, int64_t n_rays, float *grad_o, float *grad_d);

/* ---- octree builder on the device (csrc/octree_gpu.hip) ----------------
 * The same tree as psvo_octree_* (Octree::insert, octree.cpp:104-294: ids in
 * creation order, root 0, SURFACE leaf + 7 FEATURE corner leaves per voxel)
 * built in HBM by a hash-and-scan construction, incrementally across
 * inserts; export writes get_centres_and_children (octree.cpp:561-687) and /
 * or the renderer's map_states arrays (mapping.py:328-372) on the device.
 * vox / hit / outputs are device pointers; rows = psvo_dtree_count(). */
void *psvo_dtree_new(void *stream, int grid_dim, int64_t capacity);
void psvo_dtree_free(void *tree);
int psvo_dtree_insert(void *tree, void *stream, const int *vox, int64_t n);
int64_t psvo_dtree_count(void *tree);
int64_t psvo_dtree_count_leaves(void *tree, void *stream);
/* any output may be NULL: voxels f32[N,4], children f32[N,8], features i32[N,8]
 * (get_centres_and_children), centres f32[N,3] = (xyz + side/2)·voxel_size,
 * structure i32[N,9] = [children | side] (map_states) */
int psvo_dtree_export(void *tree, void *stream, float voxel_size, float *voxels, float *children, int *features,
                      float *centres, int *structure);
/* hit[i·corners + j] = leaf at voxel i's corner j exists (corners 1: has_voxel,
 * 8: the corner keys try_insert counts, octree.cpp:381-474) */
int psvo_dtree_probe(void *tree, void *stream, const int *vox, int64_t n, int corners, int *hit);

/* ---- tracker <-> mapper state exchange (csrc/share.cpp) ----------------
 * A POSIX shared-memory block `name` ("/…") holds a robust process-shared
 * mutex, PSVO_SHARE_FLAGS int flags (stop_mapping / stop_tracking), the
 * tracked trajectory and PSVO_SHARE_CHANNELS channels of 3 device slots.  A
 * slot is a device allocation of the publishing process exported with
 * hipIpcGetMemHandle; publish copies D2D into a slot no reader holds and makes
 * it the latest (one stream sync); readers pin the latest slot, copy D2D into
 * their own buffers and unpin.  Unlike the kernels above, publish / read
 * synchronise `stream` (the snapshot must be complete before it is visible). */
#define PSVO_SHARE_CHANNELS 8
#define PSVO_SHARE_FLAGS 8
#define PSVO_SHARE_META_CAP 65536
#define PSVO_SHARE_TRAJ_CAP 65536
#define PSVO_SHARE_POSE_DIM 8   /* trajectory row = [n, pose[0..n), 0...], n <= 7 */
int64_t psvo_share_block_bytes(void);
void *psvo_share_create(const char *name);  /* NULL on error (psvo_last_error) */
void *psvo_share_attach(const char *name);
void psvo_share_detach(void *share);        /* frees this process's slots, closes its IPC mappings */
int psvo_share_unlink(const char *name);
int psvo_share_set_flag(void *share, int i, int value);
int psvo_share_get_flag(void *share, int i);   /* -1 on bad arguments */
int psvo_share_push_pose(void *share, const double *pose, int n);
int64_t psvo_share_trajectory(void *share, double *out, int64_t cap);  /* rows [cap, 8]; returns the pose count */
/* writer: n device buffers -> a free slot of `channel` at 256-B aligned
 * offsets (written to offsets[n]) + opaque meta; *version = new version */
int psvo_share_publish(void *share, void *stream, int channel, int n, const void *const *srcs, const int64_t *bytes,
                       const void *meta, int64_t meta_len, int timeout_ms, int64_t *offsets, uint64_t *version);
/* reader: 1 = pinned the latest snapshot newer than `after` (slot, version,
 * meta, used bytes, device base pointer filled), 0 = nothing newer, < 0 = -error */
int psvo_share_acquire(void *share, int channel, uint64_t after, int *slot, uint64_t *version, void *meta,
                       int64_t meta_cap, int64_t *meta_len, int64_t *used, void **base);
int psvo_share_read(void *share, void *stream, int channel, int slot, int n, void *const *dsts,
                    const int64_t *offsets, const int64_t *bytes, const void *base);
int psvo_share_release(void *share, int channel, int slot);
uint64_t psvo_share_version(void *share, int channel);   /* latest version, 0 = none */

/* ---- octree builder (CPU, host memory) -------------------------------- */
void *psvo_octree_new(int grid_dim, int feat_dim, double voxel_size, int max_points_per_leaf);
void psvo_octree_free(void *tree);
int psvo_octree_insert(void *tree, const int *vox, int64_t n);
int64_t psvo_octree_count(void *tree);
int64_t psvo_octree_count_leaves(void *tree);
/* voxels f32[N,4], children f32[N,8], features i32[N,8] as
 * Octree::get_centres_and_children (octree.cpp:561-687) */
int psvo_octree_export(void *tree, float *voxels, float *children, int *features);
int psvo_octree_has_voxel(void *tree, int x, int y, int z);
double psvo_octree_try_insert(void *tree, const int *vox, int64_t n);
/* Octree::get_leaf_voxels (octree.cpp:480-505): the integer corner of every
 * SURFACE leaf, in the reference's depth-first child-index (0..7) order, into
 * out f32[cap, 3]; returns the number of leaves (-1 on error), writing at
 * most cap of them. */
int64_t psvo_octree_leaf_voxels(void *tree, float *out, int64_t cap);

#ifdef __cplusplus
}
#endif

#endif /* PSVO_H */
