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
