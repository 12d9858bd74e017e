// grid.build_octree: the NSVF "EasyOctree" over integer voxel coordinates
// (CPU, host memory) behind the psvo C-ABI.
//
// Restates third_party/sparse_voxels/src/octree.cpp:12-164:
//   insert (:71-92)    descend from the root; child slot = (x>c.x) + 2(y>c.y) + 4(z>c.z),
//                      compared in f32 (the centre is a float tensor); a missing
//                      child at depth d gets centre c + (2·diff − 1)·2^(d−1);
//                      at depth 0 the point itself becomes the leaf, id = point index
//   finalize (:113-147) BFS from the root: the root takes id total−1 and every
//                      further internal node the next lower id in BFS order;
//                      children[id] = child ids (−1 absent), [8] = 2^(depth+1)
//                      (1 for leaves); centres cast to int32 (truncation)
//
// The reference keeps heap nodes and calls Tensor::item() three times per
// level per point; here the nodes are one flat vector indexed by int, so a
// million points insert in tens of milliseconds.  Where the reference
// breaks — a point landing in an occupied leaf slot (it orphans the earlier
// leaf, then trips its node-count assert or indexes past its outputs) or a
// negative depth (1 << −1) — this returns PSVO_E_INVALID instead.
#include <cstddef>
#include <cstdint>
#include <vector>

#include "../../include/psvo.h"

namespace {

struct EasyNode {
    float c[3];   // internal centre (f32 arithmetic, as the reference's float tensor)
    int64_t p[3]; // leaf: the point itself
    int depth;    // -1 for leaves
    int index;
    int child[8];
};

int build(const float *center, const int64_t *pts, int64_t n, int depth, std::vector<EasyNode> &nodes,
          int64_t *bad) {
    EasyNode root{};
    for (int a = 0; a < 3; ++a) root.c[a] = center[a];
    root.depth = depth;
    root.index = -1;
    for (int &c : root.child) c = -1;
    nodes.clear();
    nodes.reserve((size_t)(n + 1) * 2);
    nodes.push_back(root);
    for (int64_t k = 0; k < n; ++k) {
        const int64_t *q = pts + 3 * k;
        int u = 0;
        for (;;) {
            int diff[3];
            for (int a = 0; a < 3; ++a) diff[a] = (float)q[a] > nodes[u].c[a] ? 1 : 0;
            const int slot = diff[0] + 2 * diff[1] + 4 * diff[2];
            if (nodes[u].depth == 0) {
                if (nodes[u].child[slot] >= 0) {
                    *bad = k;
                    return PSVO_E_INVALID;
                }
                EasyNode leaf{};
                for (int a = 0; a < 3; ++a) leaf.p[a] = q[a];
                leaf.depth = -1;
                leaf.index = (int)k;
                for (int &c : leaf.child) c = -1;
                nodes[u].child[slot] = (int)nodes.size();
                nodes.push_back(leaf);
                break;
            }
            if (nodes[u].child[slot] < 0) {
                const int len = 1 << (nodes[u].depth - 1);
                EasyNode in{};
                for (int a = 0; a < 3; ++a) in.c[a] = nodes[u].c[a] + (float)((2 * diff[a] - 1) * len);
                in.depth = nodes[u].depth - 1;
                in.index = -1;
                for (int &c : in.child) c = -1;
                nodes[u].child[slot] = (int)nodes.size();
                nodes.push_back(in);
            }
            u = nodes[u].child[slot];
        }
    }
    return PSVO_OK;
}

}  // namespace

extern "C" int psvo_build_octree(const float *center, const int64_t *points, int64_t n, int depth,
                                 int64_t capacity, int *centers, int *children, int64_t *total,
                                 int64_t *terminal) {
    if (!center || !total || !terminal || n < 0 || (n > 0 && !points)) return PSVO_E_INVALID;
    if (depth < 0 || depth > 29 || n > 0x7ffffffe) return PSVO_E_INVALID;
    std::vector<EasyNode> nodes;
    int64_t bad = -1;
    if (build(center, points, n, depth, nodes, &bad) != PSVO_OK) {
        *total = bad;
        *terminal = -1;
        return PSVO_E_INVALID;
    }
    const int64_t nt = (int64_t)nodes.size();
    *total = nt;
    *terminal = n;
    if (capacity < nt) return PSVO_OK;
    if (!centers || !children) return PSVO_E_INVALID;
    for (int64_t i = 0; i < nt * 3; ++i) centers[i] = 0;
    for (int64_t i = 0; i < nt * 9; ++i) children[i] = -1;
    // BFS: FIFO over node slots (a vector with a read cursor)
    std::vector<int> queue;
    queue.reserve((size_t)nt);
    int next = (int)nt - 1;
    nodes[0].index = next;
    queue.push_back(0);
    for (size_t head = 0; head < queue.size(); ++head) {
        const EasyNode &v = nodes[queue[head]];
        int *row = children + (int64_t)v.index * 9;
        for (int i = 0; i < 8; ++i) {
            const int c = v.child[i];
            if (c < 0) continue;
            if (nodes[c].depth > -1) nodes[c].index = --next;
            queue.push_back(c);
            row[i] = nodes[c].index;
        }
        row[8] = 1 << (v.depth + 1);
        int *cr = centers + (int64_t)v.index * 3;
        for (int a = 0; a < 3; ++a) cr[a] = v.depth < 0 ? (int)(int32_t)v.p[a] : (int)v.c[a];
    }
    return PSVO_OK;
}
