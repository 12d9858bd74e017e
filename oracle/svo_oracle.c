/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference's octree builder, ray/octree
 * intersector and inverse-CDF sampler.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library, and only as the
 * checker / CPU baseline.  The product path (proud-slam_amd/) never links or
 * calls it.
 *
 * Parity anchor:
 *   - the reference CUDA sources cannot be built in this image (they need
 *     cuda.h / ATen CUDA headers), so the kernels are RESTATED here;
 *   - the Python side of the reference is imported at golden-generation time
 *     (tests/golden/make_golden.py) with this library standing in for the
 *     `grid` extension, which pins everything above the kernels;
 *   - the sampler's layout quirk is pinned by the known-answer case measured
 *     on the reference kernel during the survey.
 *
 * Arithmetic: compiled with -ffp-contract=off; divisions are IEEE
 * (the reference uses __fdividef, ≤2 ulp — see DESIGN.md §parity).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Morton codes: restates third_party/sparse_octree/src/utils.h:12-124       */
/* ------------------------------------------------------------------------ */
#define OR_MAX_BITS 21

static uint64_t or_mask(int i) /* utils.h:56-77, MASK[i] */
{
    uint64_t m = 0x7000000000000000ull;
    uint64_t acc = m;
    for (int k = 1; k <= i; ++k) acc |= (m >> (3 * k));
    return acc;
}

static uint64_t or_spread(uint64_t v) /* utils.h:79-88 expand() */
{
    uint64_t x = v & 0x1fffffull;
    x = (x | x << 32) & 0x1f00000000ffffull;
    x = (x | x << 16) & 0x1f0000ff0000ffull;
    x = (x | x << 8) & 0x100f00f00f00f00full;
    x = (x | x << 4) & 0x10c30c30c30c30c3ull;
    x = (x | x << 2) & 0x1249249249249249ull;
    return x;
}

static uint64_t or_gather(uint64_t v) /* utils.h:90-99 compact() */
{
    uint64_t x = v & 0x1249249249249249ull;
    x = (x | x >> 2) & 0x10c30c30c30c30c3ull;
    x = (x | x >> 4) & 0x100f00f00f00f00full;
    x = (x | x >> 8) & 0x1f0000ff0000ffull;
    x = (x | x >> 16) & 0x1f00000000ffffull;
    x = (x | x >> 32) & 0x1fffffull;
    return x;
}

static uint64_t or_encode(int x, int y, int z) /* utils.h:101-124 */
{
    uint64_t c = or_spread((uint64_t)(int64_t)x) | (or_spread((uint64_t)(int64_t)y) << 1) |
                 (or_spread((uint64_t)(int64_t)z) << 2);
    return c & or_mask(OR_MAX_BITS - 1);
}

static void or_decode(uint64_t code, int out[3]) /* utils.h:113-119 */
{
    out[0] = (int)or_gather(code);
    out[1] = (int)or_gather(code >> 1);
    out[2] = (int)or_gather(code >> 2);
}

/* ------------------------------------------------------------------------ */
/* Pointer octree: restates octree.cpp:46-67 (init), 104-294 (insert),      */
/* 419-439 (find_octant), 541-559 (count), 561-687 (export)                 */
/* ------------------------------------------------------------------------ */
enum { OR_NONLEAF = -1, OR_SURFACE = 0, OR_FEATURE = 1 }; /* octree.h:16-21 */

static const int OR_INCR_X[8] = {0, 0, 0, 0, 1, 1, 1, 1}; /* octree.cpp:12-14 */
static const int OR_INCR_Y[8] = {0, 0, 1, 1, 0, 0, 1, 1};
static const int OR_INCR_Z[8] = {0, 1, 0, 1, 0, 1, 0, 1};

typedef struct OrNode {
    uint64_t code;
    unsigned side;
    int index;
    int type;
    int is_leaf;
    struct OrNode *child[8];
} OrNode;

typedef struct OrTree {
    int size;
    int max_level;
    int next_index;
    OrNode *root;
    OrNode **pool;
    int64_t n_pool, cap_pool;
} OrTree;

static OrNode *or_new_node(OrTree *t)
{
    OrNode *n = (OrNode *)calloc(1, sizeof(OrNode));
    n->index = t->next_index++; /* octree.h:41 index_ = next_index_++ */
    n->type = OR_NONLEAF;
    if (t->n_pool == t->cap_pool) {
        t->cap_pool = t->cap_pool ? 2 * t->cap_pool : 1024;
        t->pool = (OrNode **)realloc(t->pool, (size_t)t->cap_pool * sizeof(OrNode *));
    }
    t->pool[t->n_pool++] = n;
    return n;
}

void *oracle_octree_new(int grid_dim)
{
    OrTree *t = (OrTree *)calloc(1, sizeof(OrTree));
    t->size = grid_dim;
    t->max_level = (int)log2((double)grid_dim); /* octree.cpp:55 */
    t->root = or_new_node(t);                     /* octree.cpp:57-60 */
    t->root->side = (unsigned)grid_dim;
    t->root->is_leaf = 0;
    return t;
}

void oracle_octree_free(void *h)
{
    OrTree *t = (OrTree *)h;
    if (!t) return;
    for (int64_t i = 0; i < t->n_pool; ++i) free(t->pool[i]);
    free(t->pool);
    free(t);
}

/* octree.cpp:139-293: every input voxel inserts itself (j==0, SURFACE) and
 * its 7 +1 corner neighbours (FEATURE unless later inserted as j==0). */
void oracle_octree_insert(void *h, const int *vox, int64_t n)
{
    OrTree *t = (OrTree *)h;
    const int shift = OR_MAX_BITS - t->max_level - 1;
    for (int64_t i = 0; i < n; ++i) {
        for (int j = 0; j < 8; ++j) {
            const int x = vox[3 * i + 0] + OR_INCR_X[j];
            const int y = vox[3 * i + 1] + OR_INCR_Y[j];
            const int z = vox[3 * i + 2] + OR_INCR_Z[j];
            const uint64_t key = or_encode(x, y, z);
            OrNode *nd = t->root;
            unsigned edge = (unsigned)t->size / 2;
            for (int d = 1; d <= t->max_level; edge /= 2, ++d) {
                const int cid = ((x & (int)edge) > 0) + 2 * ((y & (int)edge) > 0) + 4 * ((z & (int)edge) > 0);
                OrNode *c = nd->child[cid];
                if (!c) {
                    const int leaf = (d == t->max_level);
                    c = or_new_node(t);
                    c->code = key & or_mask(d + shift);
                    c->side = edge;
                    c->is_leaf = leaf;
                    c->type = leaf ? (j == 0 ? OR_SURFACE : OR_FEATURE) : OR_NONLEAF;
                    nd->child[cid] = c;
                } else if (c->type == OR_FEATURE && j == 0) {
                    c->type = OR_SURFACE; /* octree.cpp:247-248 */
                }
                nd = c;
            }
        }
    }
}

static OrNode *or_find(OrTree *t, int x, int y, int z) /* octree.cpp:419-439 */
{
    OrNode *nd = t->root;
    unsigned edge = (unsigned)t->size / 2;
    for (int d = 1; d <= t->max_level; edge /= 2, ++d) {
        const int cid = ((x & (int)edge) > 0) + 2 * ((y & (int)edge) > 0) + 4 * ((z & (int)edge) > 0);
        OrNode *c = nd->child[cid];
        if (!c) return NULL;
        nd = c;
    }
    return nd;
}

/* octree.cpp:541-559: every node counts, FEATURE leaves included */
int64_t oracle_octree_count(void *h)
{
    OrTree *t = (OrTree *)h;
    return t->n_pool;
}

/* octree.cpp:561-687.  voxels f32[N,4] (min corner xyz, side), children
 * f32[N,8] (-1 = absent or FEATURE), features i32[N,8] (corner leaf ids,
 * SURFACE rows only).  Rows are indexed by creation index; FEATURE rows are
 * never visited and keep their fill values. */
void oracle_octree_export(void *h, float *voxels, float *children, int *features)
{
    OrTree *t = (OrTree *)h;
    const int64_t n = t->n_pool;
    memset(voxels, 0, (size_t)n * 4 * sizeof(float));
    for (int64_t i = 0; i < n * 8; ++i) {
        children[i] = -1.0f;
        features[i] = -1;
    }
    OrNode **queue = (OrNode **)malloc((size_t)n * sizeof(OrNode *));
    int64_t head = 0, tail = 0;
    queue[tail++] = t->root;
    while (head < tail) {
        OrNode *nd = queue[head++];
        int xyz[3];
        or_decode(nd->code, xyz);
        float *v = voxels + (int64_t)nd->index * 4;
        v[0] = (float)xyz[0];
        v[1] = (float)xyz[1];
        v[2] = (float)xyz[2];
        v[3] = (float)nd->side;
        if (nd->type == OR_SURFACE) {
            for (int k = 0; k < 8; ++k) {
                OrNode *c = or_find(t, (int)v[0] + OR_INCR_X[k], (int)v[1] + OR_INCR_Y[k], (int)v[2] + OR_INCR_Z[k]);
                if (c) features[(int64_t)nd->index * 8 + k] = c->index;
            }
        }
        for (int k = 0; k < 8; ++k) {
            OrNode *c = nd->child[k];
            if (c && c->type != OR_FEATURE) {
                queue[tail++] = c;
                children[(int64_t)nd->index * 8 + k] = (float)c->index;
            }
        }
    }
    free(queue);
}

/* ------------------------------------------------------------------------ */
/* Ray / AABB slab test: restates intersect_gpu.cu:75-140                    */
/* ------------------------------------------------------------------------ */
static int or_ray_aabb(const float o[3], const float dir[3], const float c[3], float half, float *t0, float *t1)
{
    float lo_all = 0.0f, hi_all = 100000.0f;
    for (int d = 0; d < 3; ++d) {
        const float inv = 1.0f / dir[d];
        float lo = (c[d] - half - o[d]) * inv;
        float hi = (c[d] + half - o[d]) * inv;
        if (hi < lo) {
            float tmp = lo;
            lo = hi;
            hi = tmp;
        }
        if (hi < lo_all) return 0;
        if (lo > hi_all) return 0;
        lo_all = (lo > lo_all) ? lo : lo_all;
        hi_all = (hi < hi_all) ? hi : hi_all;
        if (lo_all > hi_all) return 0;
    }
    *t0 = lo_all;
    *t1 = hi_all;
    return 1;
}

/* intersect_gpu.cu:191-270 for a flat ray list (the reference's G-fold batch
 * copy only replicates the tree; rays are independent).  Returns the number
 * of AABB tests performed (V, for the bench's byte accounting). */
int64_t oracle_svo_intersect(int64_t n_rays, const float *ray_start, const float *ray_dir, const float *points,
                             const int *children9, float voxelsize, int n_max, int *idx, float *min_depth,
                             float *max_depth)
{
    const float half_voxel = voxelsize * 0.5f;
    int64_t visits = 0;
    int overflow = 0;
    /* rays are independent: OpenMP over rays (the CPU baseline's threads) */
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : visits) reduction(| : overflow)
    for (int64_t r = 0; r < n_rays; ++r) {
        int *oi = idx + r * n_max;
        float *omin = min_depth + r * n_max;
        float *omax = max_depth + r * n_max;
        for (int l = 0; l < n_max; ++l) {
            oi[l] = -1;
            omin[l] = 0.0f;
            omax[l] = 0.0f;
        }
        int stack[256 + 8]; /* pushes of the last popped node may pass 256 before the check */
        int ptr = 0, cnt = 0;
        stack[0] = 0; /* root is node 0 (intersect_gpu.cu:232) */
        while (ptr > -1 && cnt < n_max) {
            if (ptr >= 256) { /* reference: assert(ptr < 256) */
                overflow = 1;
                break;
            }
            const int k = stack[ptr--];
            ++visits;
            const int side = children9[(int64_t)k * 9 + 8];
            float t0, t1;
            if (!or_ray_aabb(ray_start + 3 * r, ray_dir + 3 * r, points + (int64_t)k * 3, half_voxel * (float)side, &t0, &t1))
                continue;
            if (side == 1) {
                oi[cnt] = k;
                omin[cnt] = t0;
                omax[cnt] = t1;
                ++cnt;
                continue;
            }
            for (int u = 0; u < 8; ++u) {
                const int ch = children9[(int64_t)k * 9 + u];
                if (ch > -1) stack[++ptr] = ch;
            }
        }
    }
    return overflow ? -1 : visits;
}

/* ------------------------------------------------------------------------ */
/* Inverse-CDF sampler: restates sample_gpu.cu:133-239 for ONE launch over  */
/* a contiguous [b, num_rays, max_hits] chunk (sample.cpp:56-95).  Outputs  */
/* must be pre-filled by the caller (idx -1, depth 0, dists 0) as           */
/* sample.cpp:80-89 does.  Reproduces the layout-dependent trailing-segment */
/* quirks verbatim, including the slot-0 read at :231.    */
/* ------------------------------------------------------------------------ */
void oracle_inverse_cdf(int b, int num_rays, int max_hits, int max_steps, float fixed_step_size, const int *pts_idx0,
                        const float *min_depth0, const float *max_depth0, const float *noise0, const float *probs0,
                        const float *steps0, int *out_idx0, float *out_depth0, float *out_dists0)
{
    for (int bi = 0; bi < b; ++bi) {
        const int *pts_idx = pts_idx0 + (int64_t)bi * num_rays * max_hits;
        const float *min_depth = min_depth0 + (int64_t)bi * num_rays * max_hits;
        const float *max_depth = max_depth0 + (int64_t)bi * num_rays * max_hits;
        const float *probs = probs0 + (int64_t)bi * num_rays * max_hits;
        const float *steps = steps0 + (int64_t)bi * num_rays;
        const float *noise = noise0 + (int64_t)bi * num_rays * max_steps;
        int *out_idx = out_idx0 + (int64_t)bi * num_rays * max_steps;
        float *out_depth = out_depth0 + (int64_t)bi * num_rays * max_steps;
        float *out_dists = out_dists0 + (int64_t)bi * num_rays * max_steps;
        /* rays write disjoint rows (the slot-0 / next-slot reads are reads) */
#pragma omp parallel for schedule(dynamic, 64)
        for (int j = 0; j < num_rays; ++j) {
            const int H = j * max_hits, K = j * max_steps;
            int bin = 0, s = 0;
            float lo_depth = min_depth[H];
            float hi_depth = max_depth[H];
            float lo_cdf = 0.0f;
            float hi_cdf = probs[H];
            float step = (float)(1.0 / (double)steps[j]);
            float z_low = lo_depth;
            const int total_steps = (int)ceilf(steps[j]);
            int done = 0;
            if (fixed_step_size > 0.0f) step = fixed_step_size;
            for (int cs = 0; cs < total_steps; ++cs) {
                const float cdf = ((float)cs + noise[K + cs]) * step;
                while (cdf > hi_cdf) {
                    out_idx[K + s] = pts_idx[H + bin];
                    out_dists[K + s] = hi_depth - z_low;
                    out_depth[K + s] = (hi_depth + z_low) * 0.5f;
                    ++bin;
                    ++s;
                    if (bin >= max_hits || pts_idx[H + bin] == -1) {
                        done = 1;
                        break;
                    }
                    lo_depth = min_depth[H + bin];
                    hi_depth = max_depth[H + bin];
                    lo_cdf = hi_cdf;
                    hi_cdf = hi_cdf + probs[H + bin];
                    z_low = lo_depth;
                }
                if (done) break;
                const float u = (cdf - lo_cdf) / (hi_cdf - lo_cdf);
                const float z = lo_depth + u * (hi_depth - lo_depth);
                out_idx[K + s] = pts_idx[H + bin];
                out_dists[K + s] = z - z_low;
                out_depth[K + s] = (z + z_low) * 0.5f;
                z_low = z;
                ++s;
            }
            /* sample_gpu.cu:224 — `~done` is always true; the slot test uses
             * the per-launch ray count, and :231 reads slot 0's row. */
            while ((z_low < hi_depth) && (num_rays > (H + bin))) {
                out_idx[K + s] = pts_idx[H + bin];
                out_dists[K + s] = hi_depth - z_low;
                out_depth[K + s] = (hi_depth + z_low) * 0.5f;
                ++bin;
                ++s;
                if (bin >= max_hits || pts_idx[bin] == -1) break;
                lo_depth = min_depth[H + bin];
                hi_depth = max_depth[H + bin];
                z_low = lo_depth;
            }
        }
    }
}

/* ------------------------------------------------------------------------ */
/* The `grid` functions off the render path (they must exist  */
/* for import compatibility; test_aabb.py calls aabb_intersect).  Serial     */
/* loops in the reference's own structure, one ray at a time.                */
/* ------------------------------------------------------------------------ */

/* intersect_gpu.cu:13-73 (pow(p, 2) is the correctly rounded square p*p) */
void oracle_ball_intersect(int b, int n, int m, float radius, int n_max, const float *ray_start,
                           const float *ray_dir, const float *points, int *idx, float *min_depth, float *max_depth)
{
    const float radius2 = radius * radius;
    for (int64_t r = 0; r < (int64_t)b * m; ++r) {
        const float *pts = points + (r / m) * n * 3;
        const float *o = ray_start + r * 3, *w = ray_dir + r * 3;
        int *id = idx + r * n_max;
        float *lo = min_depth + r * n_max, *hi = max_depth + r * n_max;
        for (int l = 0; l < n_max; ++l) id[l] = -1;
        for (int k = 0, cnt = 0; k < n && cnt < n_max; ++k) {
            float x = pts[k * 3 + 0] - o[0];
            float y = pts[k * 3 + 1] - o[1];
            float z = pts[k * 3 + 2] - o[2];
            float d2 = x * x + y * y + z * z;
            float p = x * w[0] + y * w[1] + z * w[2];
            float d2_proj = p * p;
            float r2 = d2 - d2_proj;
            if (r2 < radius2) {
                id[cnt] = k;
                float depth = sqrtf(d2_proj);
                float blur = sqrtf(radius2 - r2);
                lo[cnt] = depth - blur;
                hi[cnt] = depth + blur;
                ++cnt;
            }
        }
    }
}

/* intersect_gpu.cu:142-187 over or_ray_aabb (a miss is (-1,-1); kept when t_in > -1) */
void oracle_aabb_intersect(int b, int n, int m, float voxelsize, int n_max, const float *ray_start,
                           const float *ray_dir, const float *points, int *idx, float *min_depth, float *max_depth)
{
    const float half = voxelsize * 0.5f;
    for (int64_t r = 0; r < (int64_t)b * m; ++r) {
        const float *pts = points + (r / m) * n * 3;
        int *id = idx + r * n_max;
        float *lo = min_depth + r * n_max, *hi = max_depth + r * n_max;
        for (int l = 0; l < n_max; ++l) id[l] = -1;
        for (int k = 0, cnt = 0; k < n && cnt < n_max; ++k) {
            float t0 = -1.0f, t1 = -1.0f;
            if (!or_ray_aabb(ray_start + r * 3, ray_dir + r * 3, pts + k * 3, half, &t0, &t1)) t0 = t1 = -1.0f;
            if (t0 > -1.0f) {
                id[cnt] = k;
                lo[cnt] = t0;
                hi[cnt] = t1;
                ++cnt;
            }
        }
    }
}

static void or_sub(const float a[3], const float b[3], float o[3])
{
    o[0] = a[0] - b[0];
    o[1] = a[1] - b[1];
    o[2] = a[2] - b[2];
}
static float or_dot(const float a[3], const float b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static void or_cross(const float a[3], const float b[3], float o[3]) /* cutil_math.h:424-427 */
{
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

/* RayTriangleIntersection intersect_gpu.cu:273-305: returns (t, u, v), t = -1 on a miss */
static void or_ray_triangle(const float o[3], const float d[3], const float *f, float blur, float tuv[3])
{
    float e1[3], e2[3], s[3], p[3], q[3];
    or_sub(f + 3, f, e1);
    or_sub(f + 6, f, e2);
    or_sub(o, f, s);
    or_cross(d, e2, p);
    float det = 1.0f / or_dot(e1, p);
    float u = or_dot(s, p) * det;
    tuv[0] = -1.0f;
    tuv[1] = tuv[2] = 0.0f;
    if ((u < 0.0f - blur) || (u > 1.0f + blur)) return;
    or_cross(s, e1, q);
    float v = or_dot(d, q) * det;
    if ((v < 0.0f - blur) || (v > 1.0f + blur)) return;
    if (((u + v) < 0.0f - blur) || ((u + v) > 1.0f + blur)) return;
    tuv[0] = or_dot(e2, q) * det;
    tuv[1] = u;
    tuv[2] = v;
}

/* intersect_gpu.cu:307-369: insertion while collecting, then the cage offsets */
void oracle_triangle_intersect(int b, int n, int m, float cagesize, float blur, int n_max, const float *ray_start,
                               const float *ray_dir, const float *face_points, int *idx, float *depth, float *uv)
{
    for (int64_t r = 0; r < (int64_t)b * m; ++r) {
        const float *fp = face_points + (r / m) * n * 9;
        int *id = idx + r * n_max;
        float *dp = depth + r * n_max * 3, *uvr = uv + r * n_max * 2;
        for (int l = 0; l < n_max; ++l) id[l] = -1;
        int cnt = 0;
        for (int k = 0; k < n && cnt < n_max; ++k) {
            float tuv[3];
            or_ray_triangle(ray_start + r * 3, ray_dir + r * 3, fp + (int64_t)k * 9, blur, tuv);
            if (tuv[0] > 0) {
                int ki = k;
                float d = tuv[0], u = tuv[1], v = tuv[2], tf;
                int ti;
                for (int l = 0; l < cnt; l++) {
                    if (d < dp[l * 3]) {
                        ti = ki; ki = id[l]; id[l] = ti;
                        tf = d; d = dp[l * 3]; dp[l * 3] = tf;
                        tf = u; u = uvr[l * 2]; uvr[l * 2] = tf;
                        tf = v; v = uvr[l * 2 + 1]; uvr[l * 2 + 1] = tf;
                    }
                }
                id[cnt] = ki;
                dp[cnt * 3] = d;
                uvr[cnt * 2] = u;
                uvr[cnt * 2 + 1] = v;
                cnt++;
            }
        }
        for (int l = 0; l < cnt; l++) {
            dp[l * 3 + 1] = (l == 0) ? -cagesize : -fminf(cagesize, (float)(.5 * (dp[l * 3] - dp[l * 3 - 3])));
            dp[l * 3 + 2] = (l == cnt - 1) ? cagesize : fminf(cagesize, (float)(.5 * (dp[l * 3 + 3] - dp[l * 3])));
        }
    }
}

/* sample_gpu.cu:13-124 for every ray of the flat [b, num_rays] layout.  Reads
 * past a ray's row go to the neighbouring row as in the reference (-1 / 0
 * outside the array); writes past max_steps (a cross-row race there) are
 * dropped; the merge stops after max_steps + 2·max_hits + 3 rounds. */
void oracle_uniform_sampling(int b, int num_rays, int max_hits, int max_steps, float step_size,
                             const int *pts_idx, const float *min_depth, const float *max_depth,
                             const float *uniform_noise, int *sampled_idx, float *sampled_depth, float *sampled_dists)
{
    const int64_t total = (int64_t)b * num_rays, n_idx = total * max_hits;
#define OR_PIDX(at) (((at) >= 0 && (at) < n_idx) ? pts_idx[(at)] : -1)
    for (int64_t j = 0; j < total; ++j) {
        const int64_t H = j * max_hits, K = j * max_steps;
        int s = 0, ucur = 0, umin = 0, umax = 0, guard = 0;
        float last_min_depth, last_max_depth, curr_depth = 0.0f;
        while (guard++ <= max_steps + 2 * max_hits + 2) {
            if ((umax == max_hits) || (ucur == max_steps) || (OR_PIDX(H + umax) == -1)) break;
            last_min_depth = (umin < max_hits) ? min_depth[H + umin] : 10000.0f;
            last_max_depth = (umax < max_hits) ? max_depth[H + umax] : 10000.0f;
            if (ucur < max_steps) curr_depth = min_depth[H] + ((float)ucur + uniform_noise[K + ucur]) * step_size;
            if ((last_max_depth <= curr_depth) && (last_max_depth <= last_min_depth)) {
                if (s < max_steps) {
                    sampled_depth[K + s] = last_max_depth;
                    sampled_idx[K + s] = OR_PIDX(H + umax);
                }
                umax++;
                s++;
                continue;
            }
            if ((curr_depth <= last_min_depth) && (curr_depth <= last_max_depth)) {
                if (s < max_steps) {
                    sampled_depth[K + s] = curr_depth;
                    sampled_idx[K + s] = OR_PIDX(H + umin - 1);
                }
                ucur++;
                s++;
                continue;
            }
            if ((last_min_depth <= curr_depth) && (last_min_depth <= last_max_depth)) {
                if (s < max_steps) {
                    sampled_depth[K + s] = last_min_depth;
                    sampled_idx[K + s] = OR_PIDX(H + umin);
                }
                umin++;
                s++;
                continue;
            }
        }
        float l_depth, r_depth;
        int step = 0;
        for (ucur = 0, umin = 0, umax = 0; ucur < max_steps - 1; ucur++) {
            if (sampled_idx[K + ucur + 1] == -1) break;
            l_depth = sampled_depth[K + ucur];
            r_depth = sampled_depth[K + ucur + 1];
            sampled_depth[K + ucur] = (l_depth + r_depth) * .5f;
            sampled_dists[K + ucur] = (r_depth - l_depth);
            if ((umin < max_hits) && (sampled_depth[K + ucur] >= min_depth[H + umin]) && (pts_idx[H + umin] > -1))
                umin++;
            if ((umax < max_hits) && (sampled_depth[K + ucur] >= max_depth[H + umax]) && (pts_idx[H + umax] > -1))
                umax++;
            if ((umax == max_hits) || (pts_idx[H + umax] == -1)) break;
            if ((umin - 1 == umax) && (sampled_dists[K + ucur] > 0)) {
                sampled_depth[K + step] = sampled_depth[K + ucur];
                sampled_dists[K + step] = sampled_dists[K + ucur];
                sampled_idx[K + step] = sampled_idx[K + ucur];
                step++;
            }
        }
        for (int l = step; l < max_steps; l++) sampled_idx[K + l] = -1;
    }
#undef OR_PIDX
}
