// torch.classes.svo.Octree — the reference's TorchScript class
// (third_party/sparse_octree/src/bindings.cpp:4-35, loaded by
// mapping.py:18-19 with torch.classes.load_library and constructed at
// mapping.py:86-87) over libpsvo's CPU builder (octree.cpp, psvo_octree_*):
// the same method names, argument meaning and outputs, so an unchanged
// mapping.py works with only the library path changed.
//
// Node ids are the reference's creation order (octree.cpp:9, root 0);
// get_centres_and_children returns (voxels f32[N,4], children f32[N,8],
// features i32[N,8], pcd_xyz f32[N,K,4], pcd_color f32[N,K,3]) as
// octree.cpp:561-687 does.  The per-node point samples (octree.cpp:198-239)
// feed only the disabled get_features_pcd path (render_helpers.py:481): the
// last two outputs are zeros of the reference's shapes.  def_pickle replays
// the inserts (bindings.cpp:27-35 pickles the tree's construction inputs).
#include <torch/custom_class.h>
#include <torch/script.h>

#include <tuple>
#include <vector>

#include "psvo.h"

namespace {

struct SvoOctree : torch::CustomClassHolder {
    void *h = nullptr;
    int64_t size = 0, feat_dim = 0, max_num = 8;
    double voxel_size = 0.0;
    std::vector<torch::Tensor> inserted;  // the int32 [n, 3] voxel batches, in insert order

    SvoOctree() = default;
    ~SvoOctree() override { release(); }

    void release() {
        if (h) psvo_octree_free(h);
        h = nullptr;
    }
    void check() const { TORCH_CHECK(h != nullptr, "Octree not initialized!"); }

    // octree.cpp:46-67
    void init(int64_t grid_dim, int64_t feat_dim_, double voxel_size_, int64_t max_num_) {
        release();
        h = psvo_octree_new((int)grid_dim, (int)feat_dim_, voxel_size_, (int)max_num_);
        TORCH_CHECK(h != nullptr, "Octree.init: grid_dim must be a power of two >= 2 (got ", grid_dim, ")");
        size = grid_dim;
        feat_dim = feat_dim_;
        voxel_size = voxel_size_;
        max_num = max_num_;
        inserted.clear();
    }

    static torch::Tensor as_int3(const torch::Tensor &pts) {
        TORCH_CHECK(pts.dim() == 2 && pts.size(1) == 3, "Point dimensions mismatch: inputs are ",
                    pts.dim() ? pts.size(-1) : 0, " expect 3");
        return pts.detach().to(torch::kCPU, torch::kInt32).contiguous();
    }

    // octree.cpp:104-294 (colors / pcd: the point samples, not stored)
    void insert(torch::Tensor pts, torch::Tensor color, torch::Tensor pcd) {
        (void)color;
        (void)pcd;
        check();
        torch::Tensor a = as_int3(pts);
        const int rc = psvo_octree_insert(h, a.data_ptr<int>(), a.size(0));
        TORCH_CHECK(rc == PSVO_OK, "Octree.insert: ", psvo_last_error());
        inserted.push_back(a.clone());
    }

    // octree.cpp:381-417
    double try_insert(torch::Tensor pts) {
        check();
        torch::Tensor a = as_int3(pts);
        return psvo_octree_try_insert(h, a.data_ptr<int>(), a.size(0));
    }

    int64_t count_nodes() {
        check();
        return psvo_octree_count(h);
    }
    int64_t count_leaf_nodes() {
        check();
        return psvo_octree_count_leaves(h);
    }

    bool has_voxel(torch::Tensor pts) {
        check();
        torch::Tensor p = pts.detach().to(torch::kCPU, torch::kInt64).reshape({-1});
        if (p.numel() != 3) return false;
        auto a = p.accessor<int64_t, 1>();
        return psvo_octree_has_voxel(h, (int)a[0], (int)a[1], (int)a[2]) != 0;
    }

    std::tuple<torch::Tensor, torch::Tensor, torch::Tensor> arrays() {
        check();
        const int64_t n = psvo_octree_count(h);
        torch::Tensor v = torch::empty({n, 4}, torch::kFloat32), c = torch::empty({n, 8}, torch::kFloat32),
                      f = torch::empty({n, 8}, torch::kInt32);
        const int rc = psvo_octree_export(h, v.data_ptr<float>(), c.data_ptr<float>(), f.data_ptr<int>());
        TORCH_CHECK(rc == PSVO_OK, "Octree.get_centres_and_children: ", psvo_last_error());
        return {v, c, f};
    }

    // octree.cpp:561-687
    std::tuple<torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor> get_centres_and_children() {
        auto [v, c, f] = arrays();
        const int64_t n = v.size(0);
        return {v, c, f, torch::zeros({n, max_num, 4}, torch::kFloat32), torch::zeros({n, max_num, 3}, torch::kFloat32)};
    }

    // the SURFACE leaves' integer corners in the reference's depth-first
    // child-index order (octree.cpp:480-505)
    torch::Tensor get_leaf_voxels() {
        check();
        const int64_t n = psvo_octree_leaf_voxels(h, nullptr, 0);
        TORCH_CHECK(n >= 0, "Octree.get_leaf_voxels: ", psvo_last_error());
        torch::Tensor v = torch::empty({n, 3}, torch::kFloat32);
        TORCH_CHECK(psvo_octree_leaf_voxels(h, v.data_ptr<float>(), n) == n, "Octree.get_leaf_voxels failed");
        return v;
    }

    using State = std::tuple<int64_t, int64_t, double, std::vector<torch::Tensor>, int64_t>;
    State getstate() const { return State(size, feat_dim, voxel_size, inserted, max_num); }
};

}  // namespace

TORCH_LIBRARY(svo, m) {
    m.class_<SvoOctree>("Octree")
        .def(torch::init<>())
        .def("init", &SvoOctree::init)
        .def("insert", &SvoOctree::insert)
        .def("try_insert", &SvoOctree::try_insert)
        .def("count_nodes", &SvoOctree::count_nodes)
        .def("count_leaf_nodes", &SvoOctree::count_leaf_nodes)
        .def("has_voxel", &SvoOctree::has_voxel)
        .def("get_centres_and_children", &SvoOctree::get_centres_and_children)
        .def("get_leaf_voxels", &SvoOctree::get_leaf_voxels)
        .def_pickle(
            // __getstate__: the construction inputs (bindings.cpp:27-30)
            [](const c10::intrusive_ptr<SvoOctree> &self) -> SvoOctree::State { return self->getstate(); },
            // __setstate__: a new tree with the inserts replayed in order (bindings.cpp:31-34)
            [](SvoOctree::State st) {
                auto t = c10::make_intrusive<SvoOctree>();
                t->init(std::get<0>(st), std::get<1>(st), std::get<2>(st), std::get<4>(st));
                for (const torch::Tensor &a : std::get<3>(st)) t->insert(a, a, a);
                return t;
            });
}
