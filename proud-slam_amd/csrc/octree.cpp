// Sparse voxel octree builder (CPU, host memory) behind the psvo C-ABI.
//
// Mirrors torch.classes.svo.Octree (third_party/sparse_octree/src/bindings.cpp:4-35):
// insert() semantics of octree.cpp:104-294 (every voxel inserts itself as a
// SURFACE leaf and its 7 +1 corner neighbours as FEATURE leaves, node ids in
// creation order, root = 0) and the export of get_centres_and_children()
// (octree.cpp:561-687): rows indexed by node id; FEATURE rows untouched;
// children = -1 when absent or FEATURE; features = the corner leaves of
// SURFACE rows.
//
// Data layout: nodes live in flat struct-of-arrays vectors (code, side,
// type, 8 int32 child ids) instead of the reference's heap pointer tree, so
// insertion walks contiguous memory and export is a single linear pass (every
// non-FEATURE node is BFS-reachable from the root, so no queue is needed).
// The node arrays map 1:1 onto the device layout the render kernels read.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <set>
#include <vector>

#include "../../include/psvo.h"

namespace {

constexpr int kMaxBits = 21;  // utils.h:12
constexpr int kIncX[8] = {0, 0, 0, 0, 1, 1, 1, 1};
constexpr int kIncY[8] = {0, 0, 1, 1, 0, 0, 1, 1};
constexpr int kIncZ[8] = {0, 1, 0, 1, 0, 1, 0, 1};
enum : int8_t { kNonLeaf = -1, kSurface = 0, kFeature = 1 };

inline uint64_t spread3(uint64_t v) {
    uint64_t x = v & 0x1fffffull;
    x = (x | x << 32) & 0x1f00000000ffffull;
    x = (x | x << 16) & 0x1f0000ff0000ffull;
    x = (x | x << 8) & 0x100f00f00f00f00full;
    x = (x | x << 4) & 0x10c30c30c30c30c3ull;
    x = (x | x << 2) & 0x1249249249249249ull;
    return x;
}
inline uint64_t squeeze3(uint64_t v) {
    uint64_t x = v & 0x1249249249249249ull;
    x = (x | x >> 2) & 0x10c30c30c30c30c3ull;
    x = (x | x >> 4) & 0x100f00f00f00f00full;
    x = (x | x >> 8) & 0x1f0000ff0000ffull;
    x = (x | x >> 16) & 0x1f00000000ffffull;
    x = (x | x >> 32) & 0x1fffffull;
    return x;
}
// MASK[i] of utils.h:56-77: the top 3(i+1) bits below bit 63.
inline uint64_t prefix_mask(int i) { return i >= 20 ? 0x7fffffffffffffffull : ~((1ull << (60 - 3 * i)) - 1) & 0x7fffffffffffffffull; }
inline uint64_t morton(int x, int y, int z) {
    return (spread3((uint64_t)(int64_t)x) | spread3((uint64_t)(int64_t)y) << 1 | spread3((uint64_t)(int64_t)z) << 2) &
           prefix_mask(kMaxBits - 1);
}

struct Tree {
    int size = 0, feat_dim = 0, max_level = 0, max_points = 8;
    double voxel_size = 0.0;
    std::vector<uint64_t> code;
    std::vector<uint32_t> side;
    std::vector<int8_t> type;
    std::vector<int32_t> child;  // 8 per node
    std::set<uint64_t> keys;     // all inserted corner keys (try_insert overlap)

    int add(uint64_t c, uint32_t s, int8_t t) {
        const int id = (int)code.size();
        code.push_back(c);
        side.push_back(s);
        type.push_back(t);
        child.insert(child.end(), 8, -1);
        return id;
    }
    int find(int x, int y, int z) const {  // octree.cpp:419-439
        int nd = 0;
        unsigned edge = (unsigned)size / 2;
        for (int d = 1; d <= max_level; edge /= 2, ++d) {
            const int cid = ((x & (int)edge) > 0) + 2 * ((y & (int)edge) > 0) + 4 * ((z & (int)edge) > 0);
            const int c = child[(size_t)nd * 8 + cid];
            if (c < 0) return -1;
            nd = c;
        }
        return nd;
    }
};

}  // namespace

extern "C" void *psvo_octree_new(int grid_dim, int feat_dim, double voxel_size, int max_points_per_leaf) {
    if (grid_dim < 2 || (grid_dim & (grid_dim - 1))) return nullptr;
    Tree *t = new Tree;
    t->size = grid_dim;
    t->feat_dim = feat_dim;
    t->voxel_size = voxel_size;
    t->max_points = max_points_per_leaf;
    t->max_level = (int)std::log2((double)grid_dim);
    t->add(0, (uint32_t)grid_dim, kNonLeaf);  // root, id 0
    return t;
}

extern "C" void psvo_octree_free(void *tree) { delete static_cast<Tree *>(tree); }

extern "C" int psvo_octree_insert(void *tree, const int *vox, int64_t n) {
    Tree *t = static_cast<Tree *>(tree);
    if (!t || (n > 0 && !vox)) return PSVO_E_INVALID;
    const int shift = kMaxBits - t->max_level - 1;
    t->code.reserve(t->code.size() + (size_t)n * 2);
    for (int64_t i = 0; i < n; ++i) {
        for (int j = 0; j < 8; ++j) {
            const int x = vox[3 * i] + kIncX[j], y = vox[3 * i + 1] + kIncY[j], z = vox[3 * i + 2] + kIncZ[j];
            const uint64_t key = morton(x, y, z);
            t->keys.insert(key);
            int nd = 0;
            unsigned edge = (unsigned)t->size / 2;
            for (int d = 1; d <= t->max_level; edge /= 2, ++d) {
                const int cid = ((x & (int)edge) > 0) + 2 * ((y & (int)edge) > 0) + 4 * ((z & (int)edge) > 0);
                int c = t->child[(size_t)nd * 8 + cid];
                if (c < 0) {
                    const bool leaf = d == t->max_level;
                    c = t->add(key & prefix_mask(d + shift), edge, leaf ? (j == 0 ? kSurface : kFeature) : kNonLeaf);
                    t->child[(size_t)nd * 8 + cid] = c;
                } else if (t->type[c] == kFeature && j == 0) {
                    t->type[c] = kSurface;
                }
                nd = c;
            }
        }
    }
    return PSVO_OK;
}

extern "C" int64_t psvo_octree_count(void *tree) {
    const Tree *t = static_cast<Tree *>(tree);
    return t ? (int64_t)t->code.size() : -1;
}

extern "C" int64_t psvo_octree_count_leaves(void *tree) {  // octree.cpp:712-736 (SURFACE leaves)
    const Tree *t = static_cast<Tree *>(tree);
    if (!t) return -1;
    int64_t n = 0;
    for (int8_t ty : t->type) n += ty == kSurface;
    return n;
}

extern "C" int psvo_octree_export(void *tree, float *voxels, float *children, int *features) {
    const Tree *t = static_cast<Tree *>(tree);
    if (!t || !voxels || !children || !features) return PSVO_E_INVALID;
    const size_t n = t->code.size();
    std::memset(voxels, 0, n * 4 * sizeof(float));
    for (size_t i = 0; i < n * 8; ++i) {
        children[i] = -1.0f;
        features[i] = -1;
    }
    for (size_t i = 0; i < n; ++i) {
        if (t->type[i] == kFeature) continue;  // never reached by the reference BFS
        const int x = (int)squeeze3(t->code[i]), y = (int)squeeze3(t->code[i] >> 1), z = (int)squeeze3(t->code[i] >> 2);
        voxels[i * 4 + 0] = (float)x;
        voxels[i * 4 + 1] = (float)y;
        voxels[i * 4 + 2] = (float)z;
        voxels[i * 4 + 3] = (float)t->side[i];
        if (t->type[i] == kSurface)
            for (int k = 0; k < 8; ++k) features[i * 8 + k] = t->find(x + kIncX[k], y + kIncY[k], z + kIncZ[k]);
        for (int k = 0; k < 8; ++k) {
            const int c = t->child[i * 8 + k];
            if (c >= 0 && t->type[c] != kFeature) children[i * 8 + k] = (float)c;
        }
    }
    return PSVO_OK;
}

extern "C" int psvo_octree_has_voxel(void *tree, int x, int y, int z) {  // octree.cpp:441-474
    const Tree *t = static_cast<Tree *>(tree);
    return t ? (t->find(x, y, z) >= 0) : 0;
}

extern "C" double psvo_octree_try_insert(void *tree, const int *vox, int64_t n) {  // octree.cpp:381-417
    const Tree *t = static_cast<Tree *>(tree);
    if (!t) return -1.0;
    std::set<uint64_t> tmp;
    for (int64_t i = 0; i < n; ++i)
        for (int j = 0; j < 8; ++j) tmp.insert(morton(vox[3 * i] + kIncX[j], vox[3 * i + 1] + kIncY[j], vox[3 * i + 2] + kIncZ[j]));
    if (tmp.empty()) return 0.0;
    size_t hit = 0;
    for (uint64_t k : tmp) hit += t->keys.count(k);
    return (double)hit / (double)tmp.size();
}

// octree.cpp:480-505 get_leaf_voxel_recursive: a node that is a SURFACE leaf
// emits its corner, any other node recurses into children 0..7 in order
// (FEATURE leaves have no children: nothing).  Iterative, explicit stack.
extern "C" int64_t psvo_octree_leaf_voxels(void *tree, float *out, int64_t cap) {
    const Tree *t = static_cast<Tree *>(tree);
    if (!t || (cap > 0 && !out)) return -1;
    int64_t n = 0;
    std::vector<int> stack{0};
    while (!stack.empty()) {
        const int nd = stack.back();
        stack.pop_back();
        if (t->type[nd] == kSurface) {
            if (n < cap) {
                out[n * 3 + 0] = (float)squeeze3(t->code[nd]);
                out[n * 3 + 1] = (float)squeeze3(t->code[nd] >> 1);
                out[n * 3 + 2] = (float)squeeze3(t->code[nd] >> 2);
            }
            ++n;
            continue;
        }
        for (int k = 7; k >= 0; --k) {  // pushed 7..0: child 0 is visited first
            const int c = t->child[(size_t)nd * 8 + k];
            if (c >= 0) stack.push_back(c);
        }
    }
    return n;
}
