// bvh_build.cpp — binned-SAH BVH2 for the software traversal kernels.
//
// The reference builds one BLAS with one GEOMETRY_DESC per mesh plus an identity TLAS instance
// (DXRPathTracer.cpp:2331-2488) and lets the driver choose the tree.  Here the tree is built on the
// host once per scene: 32-bin SAH over triangle centroids, leaves of <= 8 triangles (<= 4 preferred),
// depth capped so the per-lane LDS traversal stack (kTraversalStack entries) can never overflow.
// Child boxes are padded outward so that the (fast, FMA-using) slab test on the GPU is conservative:
// the exact triangle test alone decides hits, which keeps results independent of the tree.
#include "bvh_build.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>

namespace dxrpt {
namespace {

struct Box {
    float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
    float hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    void grow(const Box& b) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], b.lo[k]);
            hi[k] = std::max(hi[k], b.hi[k]);
        }
    }
    void grow(const float* p) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], p[k]);
            hi[k] = std::max(hi[k], p[k]);
        }
    }
    bool empty() const { return lo[0] > hi[0]; }
    double area() const {
        if (empty()) return 0.0;
        double dx = double(hi[0]) - lo[0], dy = double(hi[1]) - lo[1], dz = double(hi[2]) - lo[2];
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
};

constexpr int kBins = 32;
constexpr int kPreferLeaf = 4;
constexpr uint32_t kMaxDepth = kTraversalStack;  // a node at depth d has at most d stack entries above it

struct Task {
    int32_t node;    // node whose child slot we fill
    int slot;        // 0 or 1
    uint32_t begin, end, depth;
};

struct Builder {
    const float* pos;
    std::vector<Box> tri_box;
    std::vector<float> cen;  // 3 per tri
    std::vector<uint32_t> refs;
    std::vector<BvhNode> nodes;
    float pad_abs = 0.f;
    uint32_t max_depth = 0, num_leaves = 0;
    double sah_sum = 0.0;  // sum over nodes of area * cost contribution

    Box range_box(uint32_t b, uint32_t e) const {
        Box r;
        for (uint32_t i = b; i < e; ++i) r.grow(tri_box[refs[i]]);
        return r;
    }

    void write_child(int32_t node, int slot, const Box& bx, int32_t child) {
        BvhNode& n = nodes[node];
        float lo[3], hi[3];
        if (bx.empty()) {
            for (int k = 0; k < 3; ++k) { lo[k] = FLT_MAX; hi[k] = -FLT_MAX; }
        } else {
            for (int k = 0; k < 3; ++k) {
                float m = std::max(std::fabs(bx.lo[k]), std::fabs(bx.hi[k]));
                float p = m * 7.62939453125e-06f + pad_abs;  // |coord| * 2^-17 + scene-relative term
                lo[k] = bx.lo[k] - p;
                hi[k] = bx.hi[k] + p;
            }
        }
        float* ab = slot == 0 ? n.a : n.b;
        ab[0] = lo[0]; ab[1] = hi[0]; ab[2] = lo[1]; ab[3] = hi[1];
        n.c[slot * 2 + 0] = lo[2];
        n.c[slot * 2 + 1] = hi[2];
        n.d[slot] = child;
    }

    int32_t new_node() {
        BvhNode n;
        std::memset(&n, 0, sizeof(n));
        nodes.push_back(n);
        return int32_t(nodes.size() - 1);
    }

    // Returns the split position (refs partitioned) or 0 when the range should become a leaf.
    uint32_t split(uint32_t b, uint32_t e, uint32_t depth, const Box& bounds) {
        const uint32_t n = e - b;
        if (n <= 1) return 0;
        Box cb;
        for (uint32_t i = b; i < e; ++i) cb.grow(&cen[3 * refs[i]]);
        const double leaf_cost = double(n);
        double best_cost = DBL_MAX;
        int best_axis = -1, best_bin = -1;
        const double inv_area = bounds.area() > 0 ? 1.0 / bounds.area() : 0.0;
        for (int ax = 0; ax < 3; ++ax) {
            float ext = cb.hi[ax] - cb.lo[ax];
            if (!(ext > 0.f)) continue;
            Box bb[kBins];
            uint32_t bc[kBins] = {};
            const float scale = float(kBins) / ext;
            for (uint32_t i = b; i < e; ++i) {
                uint32_t t = refs[i];
                int k = int((cen[3 * t + ax] - cb.lo[ax]) * scale);
                k = std::min(std::max(k, 0), kBins - 1);
                bc[k]++;
                bb[k].grow(tri_box[t]);
            }
            double right_area[kBins];
            uint32_t right_cnt[kBins];
            Box acc;
            uint32_t cnt = 0;
            for (int k = kBins - 1; k > 0; --k) {
                acc.grow(bb[k]);
                cnt += bc[k];
                right_area[k] = acc.area();
                right_cnt[k] = cnt;
            }
            acc = Box();
            cnt = 0;
            for (int k = 0; k < kBins - 1; ++k) {
                acc.grow(bb[k]);
                cnt += bc[k];
                if (cnt == 0 || right_cnt[k + 1] == 0) continue;
                double c = 1.0 + (acc.area() * cnt + right_area[k + 1] * right_cnt[k + 1]) * inv_area;
                if (c < best_cost) {
                    best_cost = c;
                    best_axis = ax;
                    best_bin = k;
                }
            }
        }
        const bool must_split = n > uint32_t(kMaxLeafTris);
        if (!must_split && n <= uint32_t(kPreferLeaf) && leaf_cost <= best_cost) return 0;
        if (!must_split && depth + 1 >= kMaxDepth) return 0;
        // Depth budget: halving splits need `levels` more levels to reach <= kMaxLeafTris; once the SAH
        // split could no longer meet the cap, fall back to object-median splits.
        uint32_t levels = 0;
        for (uint32_t m = (n + kMaxLeafTris - 1) / kMaxLeafTris; m > 1; m = (m + 1) / 2) ++levels;
        const bool tight = depth + levels + 3 >= kMaxDepth;
        if (best_axis >= 0 && !tight && (must_split || best_cost < leaf_cost)) {
            const float ext = cb.hi[best_axis] - cb.lo[best_axis];
            const float scale = float(kBins) / ext;
            auto mid = std::partition(refs.begin() + b, refs.begin() + e, [&](uint32_t t) {
                int k = int((cen[3 * t + best_axis] - cb.lo[best_axis]) * scale);
                k = std::min(std::max(k, 0), kBins - 1);
                return k <= best_bin;
            });
            uint32_t m = uint32_t(mid - refs.begin());
            if (m > b && m < e) return m;
        }
        if (!must_split) return 0;
        // Object-median fallback (degenerate centroids): split by index along the widest axis.
        int ax = 0;
        for (int k = 1; k < 3; ++k)
            if (cb.hi[k] - cb.lo[k] > cb.hi[ax] - cb.lo[ax]) ax = k;
        uint32_t m = b + n / 2;
        std::nth_element(refs.begin() + b, refs.begin() + m, refs.begin() + e, [&](uint32_t x, uint32_t y) {
            float cx = cen[3 * x + ax], cy = cen[3 * y + ax];
            return cx < cy || (cx == cy && x < y);
        });
        return m;
    }
};

}  // namespace

bool build_bvh(const float* tri_positions, uint32_t ntris, BvhBuildResult& out, std::string& err) {
    if (ntris == 0) {
        err = "build_bvh: scene has no triangles";
        return false;
    }
    if (ntris >= (1u << 28)) {
        err = "build_bvh: too many triangles (leaf encoding holds 2^28)";
        return false;
    }
    Builder B;
    B.pos = tri_positions;
    B.tri_box.resize(ntris);
    B.cen.resize(size_t(ntris) * 3);
    B.refs.resize(ntris);
    Box scene;
    for (uint32_t t = 0; t < ntris; ++t) {
        Box bx;
        for (int v = 0; v < 3; ++v) bx.grow(tri_positions + size_t(t) * 9 + v * 3);
        B.tri_box[t] = bx;
        for (int k = 0; k < 3; ++k) B.cen[3 * t + k] = 0.5f * (bx.lo[k] + bx.hi[k]);
        B.refs[t] = t;
        scene.grow(bx);
    }
    float ext = 0.f;
    for (int k = 0; k < 3; ++k) ext = std::max(ext, scene.hi[k] - scene.lo[k]);
    B.pad_abs = ext * 1e-6f + 1e-7f;
    B.nodes.reserve(size_t(ntris) * 2 / 3 + 16);

    const double root_area = scene.area() > 0 ? scene.area() : 1.0;
    double sah = 0.0;
    int32_t root = B.new_node();
    std::vector<Task> stack;
    // The root always is an internal node: split the whole range (or put everything in child 0).
    {
        uint32_t m = B.split(0, ntris, 0, scene);
        if (m == 0) {
            B.write_child(root, 0, scene, encode_leaf(0, ntris));
            B.write_child(root, 1, Box(), encode_leaf(0, 1));
            B.num_leaves = 1;
            sah = 1.0 + ntris;
            B.max_depth = 1;
        } else {
            stack.push_back({root, 1, m, ntris, 1});
            stack.push_back({root, 0, 0, m, 1});
            sah = 1.0;
        }
    }
    while (!stack.empty()) {
        Task t = stack.back();
        stack.pop_back();
        Box bx = B.range_box(t.begin, t.end);
        B.max_depth = std::max(B.max_depth, t.depth);
        uint32_t m = (t.depth + 1 >= kMaxDepth && t.end - t.begin <= uint32_t(kMaxLeafTris))
                         ? 0
                         : B.split(t.begin, t.end, t.depth, bx);
        if (m == 0) {
            if (t.end - t.begin > uint32_t(kMaxLeafTris)) {
                err = "build_bvh: cannot form a leaf within the depth cap";
                return false;
            }
            B.write_child(t.node, t.slot, bx, encode_leaf(t.begin, t.end - t.begin));
            B.num_leaves++;
            sah += bx.area() / root_area * double(t.end - t.begin);
        } else {
            if (t.depth + 1 > kMaxDepth) {
                err = "build_bvh: depth cap exceeded";
                return false;
            }
            int32_t nn = B.new_node();
            B.write_child(t.node, t.slot, bx, nn);
            sah += bx.area() / root_area * 1.0;
            stack.push_back({nn, 1, m, t.end, t.depth + 1});
            stack.push_back({nn, 0, t.begin, m, t.depth + 1});
        }
    }
    out.nodes = std::move(B.nodes);
    out.tri_order = std::move(B.refs);
    out.max_depth = B.max_depth;
    out.num_leaves = B.num_leaves;
    out.sah_cost = sah;
    return true;
}

}  // namespace dxrpt
