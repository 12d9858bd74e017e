// Mesh extraction on the device.
//
// Reference: MeshExtractor.create_mesh (mesh_util.py:80-147) on the SURFACE
// voxels Mapping.extract_mesh selects (mapping.py:420-440):
//   get_scores (render_helpers.py:243-294): per voxel a res³ lattice
//     x = linspace(−.5, .5, res)[i,j,k] · voxel + centre  (meshgrid 'ij'),
//     trilinear features (get_features_vox) → Decoder.get_values → [rgb | sdf]
//   marching_cubes (mesh_util.py:149-169): per voxel with a sign change,
//     skimage.measure.marching_cubes(sdf, 0, spacing 1/(res−1)), vertices
//     (v − 0.5)·voxel + centre, faces offset by the running vertex count
//   colour (mesh_util.py:108-133): each vertex's voxel = the SURFACE voxel
//     whose min corner equals vertex // voxel, rgb = eval_points there
//     (render_helpers.py:297-328), 0 when there is none.
// The reference evaluates 32 voxels per decoder call with a device→host copy
// each and runs skimage per voxel on the host; here the lattice features are
// one gather kernel (then the fused decoder), and marching cubes is two
// block-per-voxel kernels around a scan: count (vertices = sign-changing
// lattice edges, triangles from the case table), exclusive offsets, emit.
//
// Case table: built at compile time from one rule (no stored table).  A
// lattice corner is "+" when sdf > 0.  On each cube face, walked
// counter-clockwise seen from outside, the iso-line runs from the crossing
// where the walk leaves the + region to the one where it enters it; a face
// with two diagonal + corners (ambiguous) separates the + corners.  Those
// directed segments chain into closed loops (each crossing edge leaves one
// face and enters its neighbour), listed from their lowest edge, each fanned
// from its first vertex whose diagonals stay off the cube faces.
// Faces resolve the same way from both cubes that share them, so the surface
// is crack-free, and triangles wind with their normal towards + (free
// space).  skimage's Lewiner tables are not vendored in the reference (an
// absent third-party dependency): the vertex set — one vertex per
// sign-changing edge at t = v0/(v0 − v1) — is the same construction, the
// triangulation of ambiguous cubes is this rule's.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include "psvo_common.h"

namespace psvo {
namespace {

constexpr int kMcMaxTri = 12;  // bound checked by the table builder below

struct McTables {
    int8_t ntri[256];
    int8_t tri[256][kMcMaxTri * 3];  // cube edge ids
    int8_t edge_corner[12][2];       // endpoint corners, low then high along the edge's axis
    int8_t edge_axis[12];
};

// corner b = (b&1, b>>1&1, b>>2&1) = (x, y, z) offsets
// edge e = axis·4 + o1 + 2·o2, (o1, o2) the offsets on the other two axes in
// increasing axis order
constexpr int edge_of(int c0, int c1) {
    const int d = c0 ^ c1;
    const int axis = d == 1 ? 0 : (d == 2 ? 1 : 2);
    const int a1 = axis == 0 ? 1 : 0, a2 = axis == 2 ? 1 : 2;
    return axis * 4 + ((c0 >> a1) & 1) + 2 * ((c0 >> a2) & 1);
}

// two cube edges on a common face: parallel with one shared offset, or
// perpendicular and touching a common corner's face
constexpr bool same_face(int e1, int e2) {
    int f1 = 0, f2 = 0;  // bitmask of the faces (axis·2 + side) containing each edge
    for (int k = 0; k < 2; ++k) {
        const int e = k ? e2 : e1;
        const int axis = e / 4, a1 = axis == 0 ? 1 : 0, a2 = axis == 2 ? 1 : 2;
        const int m = (1 << (a1 * 2 + (e & 1))) | (1 << (a2 * 2 + ((e >> 1) & 1)));
        if (k) f2 = m; else f1 = m;
    }
    return (f1 & f2) != 0;
}

constexpr McTables make_mc_tables() {
    McTables t{};
    for (int e = 0; e < 12; ++e) {
        const int axis = e / 4, a1 = axis == 0 ? 1 : 0, a2 = axis == 2 ? 1 : 2;
        const int c0 = ((e & 1) << a1) | (((e >> 1) & 1) << a2);
        t.edge_corner[e][0] = (int8_t)c0;
        t.edge_corner[e][1] = (int8_t)(c0 | (1 << axis));
        t.edge_axis[e] = (int8_t)axis;
    }
    for (int cs = 0; cs < 256; ++cs) {
        int next[12] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
        for (int axis = 0; axis < 3; ++axis) {
            for (int side = 0; side < 2; ++side) {
                // (u, v) = the next two axes cyclically, u × v = +axis; CCW about
                // the outward normal (±axis) seen from outside
                const int au = (axis + 1) % 3, av = (axis + 2) % 3;
                const int uv[4][2] = {{0, 0}, {1, 0}, {1, 1}, {0, 1}};
                int c[4] = {0, 0, 0, 0};
                for (int i = 0; i < 4; ++i) {
                    const int k = side ? i : (4 - i) % 4;  // reversed walk for the −axis face
                    c[i] = (side << axis) | (uv[k][0] << au) | (uv[k][1] << av);
                }
                int pos[4] = {0, 0, 0, 0}, npos = 0;
                for (int i = 0; i < 4; ++i) {
                    pos[i] = (cs >> c[i]) & 1;
                    npos += pos[i];
                }
                if (npos == 0 || npos == 4) continue;
                int ed[4] = {0, 0, 0, 0};
                for (int i = 0; i < 4; ++i) ed[i] = edge_of(c[i], c[(i + 1) % 4]);
                if (npos == 2 && pos[0] == pos[2]) {
                    for (int i = 0; i < 4; ++i)
                        if (pos[i]) next[ed[i]] = ed[(i + 3) % 4];
                } else {
                    int first = 0, last = 0;
                    for (int i = 0; i < 4; ++i) {
                        if (pos[i] && !pos[(i + 3) % 4]) first = i;
                        if (pos[i] && !pos[(i + 1) % 4]) last = i;
                    }
                    next[ed[last]] = ed[(first + 3) % 4];
                }
            }
        }
        bool seen[12] = {};
        int n = 0;
        for (int s = 0; s < 12; ++s) {
            if (next[s] < 0 || seen[s]) continue;
            int loop[12] = {}, len = 0;
            for (int e = s; !seen[e]; e = next[e]) {
                seen[e] = true;
                loop[len++] = e;
            }
            // fan apex: the first loop vertex none of whose diagonals joins two
            // edges of one cube face (such a diagonal would lie in a face the
            // neighbouring cube triangulates too)
            int apex = -1;
            for (int a = 0; a < len && apex < 0; ++a) {
                bool ok = true;
                for (int i = 2; i + 1 < len; ++i) ok = ok && !same_face(loop[a], loop[(a + i) % len]);
                if (ok) apex = a;
            }
            if (apex < 0) apex = len;  // cannot happen (every loop has one): makes the constexpr build fail
            for (int i = 1; i + 1 < len; ++i) {
                t.tri[cs][3 * n + 0] = (int8_t)loop[apex];
                t.tri[cs][3 * n + 1] = (int8_t)loop[(apex + i) % len];
                t.tri[cs][3 * n + 2] = (int8_t)loop[(apex + i + 1) % len];
                ++n;
            }
        }
        t.ntri[cs] = (int8_t)n;
    }
    return t;
}

constexpr McTables kMcHost = make_mc_tables();
constexpr int mc_max_tri() {
    int m = 0;
    for (int c = 0; c < 256; ++c) m = kMcHost.ntri[c] > m ? kMcHost.ntri[c] : m;
    return m;
}
static_assert(mc_max_tri() <= kMcMaxTri, "case table bound");
static_assert(kMcHost.ntri[0] == 0 && kMcHost.ntri[255] == 0 && kMcHost.ntri[1] == 1, "case table sanity");

__constant__ McTables kMc = make_mc_tables();

constexpr int kMcThreads = 256;
constexpr int kMcMaxRes = 16;

__device__ __forceinline__ int block_excl_scan(int v, int *lds_w, int &total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
        const int y = __shfl_up(x, s, 64);
        if (lane >= s) x += y;
    }
    if (lane == 63) lds_w[wv] = x;
    __syncthreads();
    int base = 0;
    total = 0;
    for (int w = 0; w < kMcThreads / 64; ++w) {
        if (w < wv) base += lds_w[w];
        total += lds_w[w];
    }
    __syncthreads();
    return base + x - v;
}

struct McLds {
    float s[kMcMaxRes * kMcMaxRes * kMcMaxRes];
    short vid[3 * kMcMaxRes * kMcMaxRes * kMcMaxRes];
    int red[2][kMcThreads / 64];
};

// edge slot q = ((i·res + j)·res + k)·3 + axis; valid when the +axis
// neighbour exists and the two values straddle 0 (one > 0, the other not)
__device__ __forceinline__ bool crossing(const float *s, int res, int q) {
    const int g = q / 3, a = q - 3 * g;
    const int coord = a == 0 ? g / (res * res) : (a == 1 ? (g / res) % res : g % res);
    if (coord >= res - 1) return false;
    const int stride = a == 0 ? res * res : (a == 1 ? res : 1);
    return (s[g] > 0.f) != (s[g + stride] > 0.f);
}

__device__ __forceinline__ int cube_case(const float *s, int res, int c) {
    const int r1 = res - 1;
    const int i = c / (r1 * r1), j = (c / r1) % r1, k = c % r1;
    int cs = 0;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const int g = ((i + (b & 1)) * res + j + ((b >> 1) & 1)) * res + k + ((b >> 2) & 1);
        cs |= (s[g] > 0.f ? 1 : 0) << b;
    }
    return cs;
}

// load one voxel's lattice; false when the reference skips it (min > 0 or
// max < 0, mesh_util.py:156-157)
__device__ bool load_voxel(McLds &L, const float *__restrict__ sdf, int64_t v, int n3) {
    float mn = 3.4e38f, mx = -3.4e38f;
    for (int g = threadIdx.x; g < n3; g += kMcThreads) {
        const float x = sdf[v * n3 + g];
        L.s[g] = x;
        mn = fminf(mn, x);
        mx = fmaxf(mx, x);
    }
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) {
        mn = fminf(mn, __shfl_xor(mn, s, 64));
        mx = fmaxf(mx, __shfl_xor(mx, s, 64));
    }
    __shared__ float red[2][kMcThreads / 64];
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = mn;
        red[1][threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    mn = red[0][0];
    mx = red[1][0];
    for (int w = 1; w < kMcThreads / 64; ++w) {
        mn = fminf(mn, red[0][w]);
        mx = fmaxf(mx, red[1][w]);
    }
    return !(mn > 0.f || mx < 0.f);
}

__global__ __launch_bounds__(kMcThreads) void k_mc_count(int64_t n_vox, int res, const float *__restrict__ sdf,
                                                         int *__restrict__ nv, int *__restrict__ nt) {
    __shared__ McLds L;
    const int64_t v = blockIdx.x;
    const int n3 = res * res * res, r1 = res - 1;
    if (!load_voxel(L, sdf, v, n3)) {
        if (threadIdx.x == 0) nv[v] = nt[v] = 0;
        return;
    }
    int cv = 0, ct = 0;
    for (int q = threadIdx.x; q < 3 * n3; q += kMcThreads) cv += crossing(L.s, res, q) ? 1 : 0;
    for (int c = threadIdx.x; c < r1 * r1 * r1; c += kMcThreads) ct += kMc.ntri[cube_case(L.s, res, c)];
    int tv = 0, tt = 0;
    (void)block_excl_scan(cv, L.red[0], tv);
    (void)block_excl_scan(ct, L.red[1], tt);
    if (threadIdx.x == 0) {
        nv[v] = tv;
        nt[v] = tt;
    }
}

// exclusive offsets of nv / nt (one block, chunks of kMcThreads·8); totals[2]
__global__ __launch_bounds__(kMcThreads) void k_mc_offsets(int64_t n, const int *__restrict__ nv,
                                                           const int *__restrict__ nt, int64_t *__restrict__ vbase,
                                                           int64_t *__restrict__ tbase, int64_t *__restrict__ totals) {
    __shared__ int red[2][kMcThreads / 64];
    constexpr int kPer = 8;
    int64_t run_v = 0, run_t = 0;
    for (int64_t c0 = 0; c0 < n; c0 += (int64_t)kMcThreads * kPer) {
        const int64_t b = c0 + (int64_t)threadIdx.x * kPer;
        int lv = 0, lt = 0;
        for (int i = 0; i < kPer; ++i)
            if (b + i < n) {
                lv += nv[b + i];
                lt += nt[b + i];
            }
        int tv = 0, tt = 0;
        const int ev = block_excl_scan(lv, red[0], tv);
        const int et = block_excl_scan(lt, red[1], tt);
        int64_t ov = run_v + ev, ot = run_t + et;
        for (int i = 0; i < kPer; ++i)
            if (b + i < n) {
                vbase[b + i] = ov;
                tbase[b + i] = ot;
                ov += nv[b + i];
                ot += nt[b + i];
            }
        run_v += tv;
        run_t += tt;
    }
    if (threadIdx.x == 0) {
        totals[0] = run_v;
        totals[1] = run_t;
    }
}

__global__ __launch_bounds__(kMcThreads) void k_mc_emit(int64_t n_vox, int res, float voxel_size,
                                                        const float *__restrict__ sdf,
                                                        const float *__restrict__ centres,
                                                        const int *__restrict__ nv, const int64_t *__restrict__ vbase,
                                                        const int64_t *__restrict__ tbase, float *__restrict__ verts,
                                                        int *__restrict__ faces) {
    __shared__ McLds L;
    const int64_t v = blockIdx.x;
    if (nv[v] == 0) return;
    const int n3 = res * res * res, r1 = res - 1, nq = 3 * n3;
    (void)load_voxel(L, sdf, v, n3);
    // vertex ids: a contiguous run of slots per thread, block-scanned
    const int per = (nq + kMcThreads - 1) / kMcThreads;
    const int q0 = threadIdx.x * per;
    int cnt = 0;
    for (int q = q0; q < q0 + per && q < nq; ++q) cnt += crossing(L.s, res, q) ? 1 : 0;
    int tot = 0;
    int id = block_excl_scan(cnt, L.red[0], tot);
    const int64_t vb = vbase[v];
    const float sp = (float)(1.0 / (double)r1);
    const float cx[3] = {centres[v * 3 + 0], centres[v * 3 + 1], centres[v * 3 + 2]};
    for (int q = q0; q < q0 + per && q < nq; ++q) {
        if (!crossing(L.s, res, q)) continue;
        L.vid[q] = (short)id;
        const int g = q / 3, a = q - 3 * g;
        const int ijk[3] = {g / (res * res), (g / res) % res, g % res};
        const int stride = a == 0 ? res * res : (a == 1 ? res : 1);
        const float v0 = L.s[g], v1 = L.s[g + stride];
        const float t = v0 / (v0 - v1);
        float* o = verts + (vb + id) * 3;
        for (int d = 0; d < 3; ++d) {
            const float gcoord = d == a ? ((float)ijk[d] + t) * sp : (float)ijk[d] * sp;
            o[d] = (gcoord - 0.5f) * voxel_size + cx[d];
        }
        ++id;
    }
    __syncthreads();
    // triangles: per-thread cube runs, block-scanned
    const int ncube = r1 * r1 * r1;
    const int cper = (ncube + kMcThreads - 1) / kMcThreads;
    const int cb = threadIdx.x * cper;
    int tc = 0;
    for (int c = cb; c < cb + cper && c < ncube; ++c) tc += kMc.ntri[cube_case(L.s, res, c)];
    int ttot = 0;
    int64_t tri = tbase[v] + block_excl_scan(tc, L.red[1], ttot);
    for (int c = cb; c < cb + cper && c < ncube; ++c) {
        const int cs = cube_case(L.s, res, c);
        const int n = kMc.ntri[cs];
        if (n == 0) continue;
        const int i = c / (r1 * r1), j = (c / r1) % r1, k = c % r1;
        for (int u = 0; u < n; ++u) {
            for (int w = 0; w < 3; ++w) {
                const int e = kMc.tri[cs][3 * u + w];
                const int c0 = kMc.edge_corner[e][0];
                const int g = ((i + (c0 & 1)) * res + j + ((c0 >> 1) & 1)) * res + k + ((c0 >> 2) & 1);
                faces[tri * 3 + w] = (int)(vb + L.vid[g * 3 + kMc.edge_axis[e]]);
            }
            ++tri;
        }
    }
}

// lattice features: x = lin[i,j,k]·voxel + centre, p = (x − centre)/voxel + ½
// (render_helpers.py:253-283 → get_embeddings_vox :86-99); four lanes per
// point, 16 B each (as k_interp_fwd)
struct Lin {
    float v[kMcMaxRes];
};

__device__ __forceinline__ void corner_w(const float p[3], float w[8]) {
    const float ax[2] = {1.0f - p[0], p[0]};
    const float ay[2] = {1.0f - p[1], p[1]};
    const float az[2] = {1.0f - p[2], p[2]};
#pragma unroll
    for (int k = 0; k < 8; ++k) w[k] = (ax[(k >> 2) & 1] * ay[(k >> 1) & 1]) * az[k & 1];
}

__device__ __forceinline__ float4 gather_interp(const float p[3], const int *__restrict__ vrow,
                                                const float4 *__restrict__ emb, int q) {
    float w[8];
    corner_w(p, w);
    const int4 v0 = *reinterpret_cast<const int4 *>(vrow);
    const int4 v1 = *reinterpret_cast<const int4 *>(vrow + 4);
    const int vid[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const float4 e = emb[(int64_t)vid[k] * 4 + q];
        acc.x = acc.x + w[k] * e.x;
        acc.y = acc.y + w[k] * e.y;
        acc.z = acc.z + w[k] * e.z;
        acc.w = acc.w + w[k] * e.w;
    }
    return acc;
}

__global__ __launch_bounds__(256) void k_grid_feat(int64_t n_pts, int res, float voxel_size, Lin lin,
                                                   const float *__restrict__ centres,
                                                   const int *__restrict__ vertex_idx,
                                                   const float4 *__restrict__ emb, float4 *__restrict__ feat) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t s = gid >> 2;
    const int q = (int)(gid & 3);
    if (s >= n_pts) return;
    const int n3 = res * res * res;
    const int64_t v = s / n3;
    const int l = (int)(s - v * n3);
    const int ijk[3] = {l / (res * res), (l / res) % res, l % res};
    float p[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float c = centres[v * 3 + a];
        const float x = lin.v[ijk[a]] * voxel_size + c;
        p[a] = __fdiv_rn(x - c, voxel_size) + 0.5f;
    }
    feat[s * 4 + q] = gather_interp(p, vertex_idx + v * 8, emb, q);
}

// eval_points (render_helpers.py:297-328): features at given points x with
// their voxel rows (row < 0: zeros)
__global__ __launch_bounds__(256) void k_point_feat(int64_t n, float voxel_size, const float *__restrict__ xyz,
                                                    const int *__restrict__ row, const float *__restrict__ centres,
                                                    const int *__restrict__ vertex_idx,
                                                    const float4 *__restrict__ emb, float4 *__restrict__ feat) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t s = gid >> 2;
    const int q = (int)(gid & 3);
    if (s >= n) return;
    const int64_t v = row[s];
    if (v < 0) {  // no voxel (the reference leaves the colour 0): zero features, masked by the caller
        feat[s * 4 + q] = make_float4(0.f, 0.f, 0.f, 0.f);
        return;
    }
    float p[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) p[a] = __fdiv_rn(xyz[s * 3 + a] - centres[v * 3 + a], voxel_size) + 0.5f;
    feat[s * 4 + q] = gather_interp(p, vertex_idx + v * 8, emb, q);
}

// torch's floor division of floats (c10 div_floor_floating): the vertex's
// voxel coordinate `points // voxel_size` (mesh_util.py:115)
__device__ __forceinline__ float div_floor(float a, float b) {
    const float mod = fmodf(a, b);
    float div = (a - mod) / b;
    if (mod != 0.f && ((b < 0.f) != (mod < 0.f))) div -= 1.0f;
    float fl;
    if (div != 0.f) {
        fl = floorf(div);
        if (div - fl > 0.5f) fl += 1.0f;
    } else {
        fl = copysignf(0.f, a / b);
    }
    return fl;
}

// open-addressing map voxel min corner → SURFACE row (keys from the
// exported voxels, integral floats)
__device__ __forceinline__ uint32_t key_hash(int x, int y, int z) {
    uint32_t h = (uint32_t)x * 73856093u ^ (uint32_t)y * 19349663u ^ (uint32_t)z * 83492791u;
    h ^= h >> 16;
    h *= 0x7feb352du;
    h ^= h >> 15;
    return h;
}

__global__ void k_vox_map_insert(int64_t n, const float *__restrict__ voxels, int cap_mask, int4 *__restrict__ table) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int x = (int)voxels[r * 4 + 0], y = (int)voxels[r * 4 + 1], z = (int)voxels[r * 4 + 2];
    uint32_t h = key_hash(x, y, z) & (uint32_t)cap_mask;
    for (;;) {
        // claim with the row (−1 = empty); the first row with a key wins ties
        // exactly as the reference's sort picks the lowest matching index
        int *slot = reinterpret_cast<int *>(table + h);
        const int prev = atomicCAS(slot + 3, -1, (int)r);
        if (prev == -1) {
            slot[0] = x;
            slot[1] = y;
            slot[2] = z;
            return;
        }
        h = (h + 1) & (uint32_t)cap_mask;
    }
}

__global__ void k_vertex_rows(int64_t n, float voxel_size, const float *__restrict__ verts, int cap_mask,
                              const int4 *__restrict__ table, int *__restrict__ row) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    float f[3];
    for (int a = 0; a < 3; ++a) f[a] = div_floor(verts[s * 3 + a], voxel_size);
    int best = -1;
    if (fabsf(f[0]) < 1e9f && fabsf(f[1]) < 1e9f && fabsf(f[2]) < 1e9f) {
        const int x = (int)f[0], y = (int)f[1], z = (int)f[2];
        uint32_t h = key_hash(x, y, z) & (uint32_t)cap_mask;
        for (;;) {
            const int4 e = table[h];
            if (e.w == -1) break;
            if (e.x == x && e.y == y && e.z == z && (best < 0 || e.w < best)) best = e.w;
            h = (h + 1) & (uint32_t)cap_mask;
        }
    }
    row[s] = best;
}

}  // namespace
}  // namespace psvo

using namespace psvo;

extern "C" int psvo_mesh_linspace(int res, float *out) {
    PSVO_REQUIRE(res >= 2 && res <= kMcMaxRes && out, "mesh_linspace: res %d outside [2, %d]", res, kMcMaxRes);
    // torch.linspace(−.5, .5, res) on the CPU: start + step·i for the first
    // half, end − step·(res−1−i) for the rest, each one rounding
    const float start = -0.5f, end = 0.5f;
    const float step = (end - start) / (float)(res - 1);
    for (int i = 0; i < res; ++i)
        out[i] = i < res / 2 ? fmaf(step, (float)i, start) : fmaf(-step, (float)(res - 1 - i), end);
    return PSVO_OK;
}

extern "C" int psvo_mesh_case_table(int8_t *ntri, int8_t *tri) {
    PSVO_REQUIRE(ntri && tri, "mesh_case_table: null pointer");
    for (int c = 0; c < 256; ++c) {
        ntri[c] = kMcHost.ntri[c];
        for (int i = 0; i < kMcMaxTri * 3; ++i) tri[c * kMcMaxTri * 3 + i] = kMcHost.tri[c][i];
    }
    return PSVO_OK;
}

extern "C" int psvo_mesh_grid_feat(void *stream, int64_t n_vox, int res, float voxel_size, const float *centres,
                                   const int *vertex_idx, const float *emb, float *feat) {
    PSVO_REQUIRE(n_vox >= 0 && res >= 2 && res <= kMcMaxRes && voxel_size > 0.f, "mesh_grid_feat: bad sizes");
    if (n_vox == 0) return PSVO_OK;
    PSVO_REQUIRE(centres && vertex_idx && emb && feat, "mesh_grid_feat: null pointer");
    Lin lin{};
    (void)psvo_mesh_linspace(res, lin.v);
    const int64_t n = n_vox * res * res * res;
    psvo::launch(k_grid_feat, dim3(div_up(n * 4, 256)), dim3(256), 0, as_stream(stream), n, res, voxel_size,
                       lin, centres, vertex_idx, reinterpret_cast<const float4 *>(emb),
                       reinterpret_cast<float4 *>(feat));
    return check_launch("mesh_grid_feat");
}

extern "C" int psvo_mesh_point_feat(void *stream, int64_t n, float voxel_size, const float *xyz, const int *row,
                                    const float *centres, const int *vertex_idx, const float *emb, float *feat) {
    PSVO_REQUIRE(n >= 0 && voxel_size > 0.f, "mesh_point_feat: bad sizes");
    if (n == 0) return PSVO_OK;
    psvo::launch(k_point_feat, dim3(div_up(n * 4, 256)), dim3(256), 0, as_stream(stream), n, voxel_size, xyz,
                       row, centres, vertex_idx, reinterpret_cast<const float4 *>(emb),
                       reinterpret_cast<float4 *>(feat));
    return check_launch("mesh_point_feat");
}

extern "C" int psvo_mesh_mc_count(void *stream, int64_t n_vox, int res, const float *sdf, int *nv, int *nt,
                                  int64_t *vbase, int64_t *tbase, int64_t *totals) {
    PSVO_REQUIRE(n_vox > 0 && res >= 2 && res <= kMcMaxRes, "mesh_mc_count: bad sizes");
    PSVO_REQUIRE(sdf && nv && nt && vbase && tbase && totals, "mesh_mc_count: null pointer");
    hipStream_t st = as_stream(stream);
    psvo::launch(k_mc_count, dim3((unsigned)n_vox), dim3(kMcThreads), 0, st, n_vox, res, sdf, nv, nt);
    psvo::launch(k_mc_offsets, dim3(1), dim3(kMcThreads), 0, st, n_vox, nv, nt, vbase, tbase, totals);
    return check_launch("mesh_mc_count");
}

extern "C" int psvo_mesh_mc_emit(void *stream, int64_t n_vox, int res, float voxel_size, const float *sdf,
                                 const float *centres, const int *nv, const int64_t *vbase, const int64_t *tbase,
                                 float *verts, int *faces) {
    PSVO_REQUIRE(n_vox > 0 && res >= 2 && res <= kMcMaxRes && voxel_size > 0.f, "mesh_mc_emit: bad sizes");
    PSVO_REQUIRE(sdf && centres && nv && vbase && tbase, "mesh_mc_emit: null pointer");
    psvo::launch(k_mc_emit, dim3((unsigned)n_vox), dim3(kMcThreads), 0, as_stream(stream), n_vox, res,
                       voxel_size, sdf, centres, nv, vbase, tbase, verts, faces);
    return check_launch("mesh_mc_emit");
}

extern "C" int64_t psvo_mesh_vox_map_slots(int64_t n_vox) {
    int64_t cap = 1024;
    while (cap < 2 * n_vox) cap <<= 1;
    return cap;
}

extern "C" int psvo_mesh_vertex_rows(void *stream, int64_t n_vox, const float *voxels, int64_t n_verts,
                                     const float *verts, float voxel_size, int *table, int *row) {
    PSVO_REQUIRE(n_vox >= 0 && n_verts >= 0 && voxel_size > 0.f, "mesh_vertex_rows: bad sizes");
    PSVO_REQUIRE(psvo_mesh_vox_map_slots(n_vox) <= (1LL << 30), "mesh_vertex_rows: too many voxels");
    if (n_verts == 0) return PSVO_OK;
    hipStream_t st = as_stream(stream);
    const int64_t cap = psvo_mesh_vox_map_slots(n_vox);
    if (hipMemsetAsync(table, 0xFF, (size_t)cap * 16, st) != hipSuccess)
        return set_error(PSVO_E_LAUNCH, "mesh_vertex_rows: memset failed");
    if (n_vox > 0)
        psvo::launch(k_vox_map_insert, dim3(div_up(n_vox, 256)), dim3(256), 0, st, n_vox, voxels,
                           (int)(cap - 1), reinterpret_cast<int4 *>(table));
    psvo::launch(k_vertex_rows, dim3(div_up(n_verts, 256)), dim3(256), 0, st, n_verts, voxel_size, verts,
                       (int)(cap - 1), reinterpret_cast<const int4 *>(table), row);
    return check_launch("mesh_vertex_rows");
}
