// bvh_build.cpp — binned-SAH binary tree, emitted as BVH2 or as a compressed BVH8.
//
// The reference builds one BLAS with one GEOMETRY_DESC per mesh plus an identity TLAS instance
// (DXRPathTracer.cpp:2331-2488) and lets the driver choose the tree.  Here the tree is built on the
// host once per scene: 32-bin SAH over triangle centroids, small leaves, and a depth budget that
// falls back to object-median splits so the per-lane LDS traversal stacks can never overflow.
// Child boxes are padded outward so that the (fast, FMA-using) slab tests on the GPU are
// conservative: the exact triangle test alone decides hits, which keeps results independent of the
// tree (the parity oracle builds its own).
#include "bvh_build.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <chrono>

namespace dxrpt {
namespace {

// Builder threads: BvhBuildParams::threads, else the host's CPUs capped at 16 (the GPU box's job gets 16
// CPUs of its host; more threads would only time-slice them).  Results never depend on the count.
unsigned build_threads(const BvhBuildParams* params) {
    if (params && params->threads) return params->threads;
    return std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
}

// Fork-join pool for the builders' independent subtrees.  A thread that waits for a task it spawned runs
// queued tasks meanwhile (so nested waits cannot deadlock); workers take the oldest tasks -- the largest
// subtrees, spawned nearest the root -- which spreads the big pieces over them.
class TaskPool {
public:
    explicit TaskPool(unsigned n) {
        for (unsigned i = 1; i < n; ++i) th_.emplace_back([this] { work(); });
    }
    ~TaskPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (std::thread& t : th_) t.join();
    }
    bool parallel() const { return !th_.empty(); }
    void submit(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> g(m_);
            q_.push_back(std::move(f));
        }
        cv_.notify_one();
    }
    // Runs queued tasks until `done` is set, newest first (most likely the awaited task or its own children;
    // the workers take the oldest, largest ones).
    void wait(const std::atomic<bool>& done) {
        while (!done.load(std::memory_order_acquire)) {
            std::function<void()> f;
            {
                std::lock_guard<std::mutex> g(m_);
                if (!q_.empty()) {
                    f = std::move(q_.back());
                    q_.pop_back();
                }
            }
            if (f) f();
            else std::this_thread::yield();
        }
    }

private:
    void work() {
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [this] { return stop_ || !q_.empty(); });
                if (stop_ && q_.empty()) return;
                f = std::move(q_.front());
                q_.pop_front();
            }
            f();
        }
    }
    std::mutex m_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
    std::vector<std::thread> th_;
    bool stop_ = false;
};

// task(k) for k in [0, K): 1..K-1 on the pool, 0 inline.  Returns only once every task has ended -- also
// when one throws, since the queued tasks reference the caller's frame -- and then rethrows bad_alloc.
// Every task the pool runs is wrapped like this (or catches for itself), so no exception leaves
// TaskPool::wait, which runs other fork-joins' tasks inline.
template <class F>
void fork_join(TaskPool& pool, size_t K, F&& task) {
    std::atomic<size_t> left{K > 1 ? K - 1 : 0};
    std::atomic<bool> done{K <= 1}, failed{false};
    for (size_t k = 1; k < K; ++k)
        pool.submit([&, k] {
            try {
                task(k);
            } catch (...) {
                failed.store(true);
            }
            if (left.fetch_sub(1) == 1) done.store(true, std::memory_order_release);
        });
    try {
        task(size_t(0));
    } catch (...) {
        failed.store(true);
    }
    pool.wait(done);
    if (failed.load()) throw std::bad_alloc();
}

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

// SAH bins per axis (object and spatial splits); r03: 64 bins measured within +-1 % (a 1/8 share +2.5 %)
constexpr int kBins = 32;
// spatial-split search when the object split's child overlap exceeds this fraction of the root area
// (r03: 1e-6 / 1e-4 measured +1-3 %)
constexpr double kSbvhAlpha = 1e-5;
constexpr uint32_t kMaxDepth2 = kTraversalStack;  // a BVH2 node at depth d has <= d stack entries above it

// Generic binary tree node.
struct TNode {
    Box box;
    int32_t child[2] = {-1, -1};
    uint32_t first = 0, count = 0;  // leaf when count > 0
    uint32_t begin = 0, end = 0;    // triangle (refs) range of the whole subtree
};

struct Builder {
    std::vector<Box> tri_box;
    std::vector<float> cen;
    std::vector<uint32_t> refs;
    std::vector<TNode> tree;
    uint32_t leaf_max = kMaxLeafTris;
    uint32_t prefer_leaf = 4;
    uint32_t depth_cap = kMaxDepth2;

    Box range_box(uint32_t b, uint32_t e) const {
        Box r;
        for (uint32_t i = b; i < e; ++i) r.grow(tri_box[refs[i]]);
        return r;
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
        const bool must_split = n > leaf_max;
        if (!must_split && n <= prefer_leaf && leaf_cost <= best_cost) return 0;
        if (!must_split && depth + 1 >= depth_cap) return 0;
        // Depth budget: halving splits need `levels` more levels to reach <= leaf_max; once the SAH
        // split could no longer meet the cap, fall back to object-median splits.
        uint32_t levels = 0;
        for (uint32_t m = (n + leaf_max - 1) / leaf_max; m > 1; m = (m + 1) / 2) ++levels;
        const bool tight = depth + levels + 3 >= depth_cap;
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

    // Builds the binary tree; tree[0] is the root (may be a leaf).
    bool build(uint32_t ntris, std::string& err, double& sah) {
        struct Task {
            int32_t node;
            uint32_t begin, end, depth;
        };
        tree.clear();
        tree.reserve(size_t(ntris) * 2 / 3 + 16);
        tree.emplace_back();
        std::vector<Task> stack{{0, 0, ntris, 0}};
        const double root_area = std::max(range_box(0, ntris).area(), 1e-30);
        sah = 0.0;
        while (!stack.empty()) {
            Task t = stack.back();
            stack.pop_back();
            Box bx = range_box(t.begin, t.end);
            tree[t.node].box = bx;
            tree[t.node].begin = t.begin;
            tree[t.node].end = t.end;
            uint32_t m = split(t.begin, t.end, t.depth, bx);
            if (m == 0) {
                if (t.end - t.begin > leaf_max) {
                    err = "build_bvh: cannot form a leaf within the depth cap";
                    return false;
                }
                tree[t.node].first = t.begin;
                tree[t.node].count = t.end - t.begin;
                sah += bx.area() / root_area * double(t.end - t.begin);
            } else {
                if (t.depth + 1 > depth_cap) {
                    err = "build_bvh: depth cap exceeded";
                    return false;
                }
                int32_t c0 = int32_t(tree.size()), c1 = c0 + 1;
                tree.emplace_back();
                tree.emplace_back();
                tree[t.node].child[0] = c0;
                tree[t.node].child[1] = c1;
                sah += bx.area() / root_area;
                stack.push_back({c1, m, t.end, t.depth + 1});
                stack.push_back({c0, t.begin, m, t.depth + 1});
            }
        }
        return true;
    }
};

double tree_sah(const std::vector<TNode>& tree);

// Spatial-split binary builder (SBVH, Stich et al. 2009) for the BVH8 path: at nodes whose best
// object split leaves overlapping children, it also bins the node box into slabs, clips each
// triangle reference to the slabs it crosses, and may split along a plane, duplicating straddling
// references (with clipped boxes) into both children.  Cuts the child-box overlap that long thin
// architectural triangles cause, hence node visits per ray.  Duplicates are harmless for the
// traversal: a triangle tested twice yields the same hit (tie rule: smaller t, then smaller id).
//
// Duplication budget (r05): every subtree carries its own allowance of extra references.  A node may search
// a spatial split while its allowance is positive; what is left after its split is shared by its children
// in proportion to their reference counts (as Embree's spatial-split builder shares its "extended range").
// No decision depends on the order in which subtrees are built, so the subtrees of large nodes are built
// in parallel (TaskPool) and the tree is the same for any thread count.  (r04 spent one global allowance in
// depth-first order: the left half of the scene took all of it, and the build was serial.)
struct SpatialBuilder {
    struct Ref {
        uint32_t tri;
        Box box;
    };
    const float* pos = nullptr;  // ntris * 9
    const uint8_t* keep_whole = nullptr;  // per triangle: never split (BvhBuildParams::keep_whole)
    std::vector<TNode> tree;
    std::vector<uint32_t> refs;  // leaf order, duplicates allowed
    uint32_t depth_cap = 32;
    double root_area = 1.0;
    double alpha = kSbvhAlpha;  // overlap / root area that enables a spatial search
    size_t ref_budget = 0;       // maximum references of the whole tree (duplication budget)
    double sah = 0.0;            // binary tree, C_trav = 1, C_tri = 1, relative to the root area
    unsigned threads = 1;
    // subtrees of at least this many references are built as their own tasks
    static constexpr size_t kTaskRefs = 2048;

    // Splits `r` at `plane` on `axis` into the parts of its triangle on each side (boxes clipped to r.box).
    void split_ref(const Ref& r, int axis, float plane, Box& left, Box& right) const {
        left = Box();
        right = Box();
        const float* v = pos + size_t(r.tri) * 9;
        for (int i = 0; i < 3; ++i) {
            const float* a = v + 3 * i;
            const float* b = v + 3 * ((i + 1) % 3);
            if (a[axis] <= plane) left.grow(a);
            if (a[axis] >= plane) right.grow(a);
            if ((a[axis] < plane && b[axis] > plane) || (b[axis] < plane && a[axis] > plane)) {
                const float t = std::min(std::max((plane - a[axis]) / (b[axis] - a[axis]), 0.0f), 1.0f);
                float p[3];
                for (int k = 0; k < 3; ++k) p[k] = a[k] + (b[k] - a[k]) * t;
                p[axis] = plane;
                left.grow(p);
                right.grow(p);
            }
        }
        for (int k = 0; k < 3; ++k) {
            left.lo[k] = std::max(left.lo[k], r.box.lo[k]);
            left.hi[k] = std::min(left.hi[k], r.box.hi[k]);
            right.lo[k] = std::max(right.lo[k], r.box.lo[k]);
            right.hi[k] = std::min(right.hi[k], r.box.hi[k]);
        }
        left.hi[axis] = std::min(left.hi[axis], plane);
        right.lo[axis] = std::max(right.lo[axis], plane);
    }

    TaskPool* pool = nullptr;
    // nodes of at least two chunks of this many references bin and partition them in parallel
    static constexpr size_t kChunkRefs = 8192;

    // f(k, begin, end) for the K chunks of [0, n) (K = 1 without a pool or for small n), on the pool; returns
    // K.  Every chunk's results go to slot k, merged by the caller in chunk order: the same as one pass.
    template <class F>
    size_t chunked(size_t n, F&& f) const {
        const size_t K = pool && pool->parallel() ? std::min<size_t>(size_t(threads) * 2u, n / kChunkRefs) : 1u;
        if (K <= 1) {
            f(size_t(0), size_t(0), n);
            return 1;
        }
        fork_join(*pool, K, [&](size_t k) { f(k, n * k / K, n * (k + 1) / K); });
        return K;
    }

    size_t max_chunks(size_t n) const {
        return pool && pool->parallel() ? std::max<size_t>(1, std::min<size_t>(size_t(threads) * 2u, n / kChunkRefs)) : 1u;
    }

    Box bounds_of(const std::vector<Ref>& rs) const {
        if (max_chunks(rs.size()) == 1) {
            Box bx;
            for (const Ref& r : rs) bx.grow(r.box);
            return bx;
        }
        std::vector<Box> part(max_chunks(rs.size()));
        const size_t K = chunked(rs.size(), [&](size_t k, size_t b, size_t e) {
            for (size_t i = b; i < e; ++i) part[k].grow(rs[i].box);
        });
        Box bx;
        for (size_t k = 0; k < K; ++k) bx.grow(part[k]);
        return bx;
    }

    struct ObjSplit {
        double cost = DBL_MAX;
        int axis = -1, bin = -1;
        Box left, right;
        float lo = 0.f, scale = 0.f;
    };

    struct AxisBins {
        Box bb[3][kBins];
        uint32_t enter[3][kBins] = {}, exit_[3][kBins] = {};  // object binning: counts in enter
    };

    ObjSplit object_split(const std::vector<Ref>& rs) const {
        ObjSplit best;
        const size_t nk = max_chunks(rs.size());
        Box cb_local;
        std::vector<Box> cb_heap(nk > 1 ? nk : 0);
        Box* cbs = nk > 1 ? cb_heap.data() : &cb_local;
        size_t K = chunked(rs.size(), [&](size_t k, size_t b, size_t e) {
            for (size_t i = b; i < e; ++i) {
                float c[3];
                for (int a = 0; a < 3; ++a) c[a] = 0.5f * (rs[i].box.lo[a] + rs[i].box.hi[a]);
                cbs[k].grow(c);
            }
        });
        Box cb;
        for (size_t k = 0; k < K; ++k) cb.grow(cbs[k]);
        float scale[3];
        bool live[3];
        for (int ax = 0; ax < 3; ++ax) {
            const float ext = cb.hi[ax] - cb.lo[ax];
            live[ax] = ext > 0.f;
            scale[ax] = live[ax] ? float(kBins) / ext : 0.f;
        }
        if (!live[0] && !live[1] && !live[2]) return best;
        AxisBins local;
        std::vector<AxisBins> heap(nk > 1 ? nk : 0);
        AxisBins* part = nk > 1 ? heap.data() : &local;
        K = chunked(rs.size(), [&](size_t k, size_t b, size_t e) {
            AxisBins& P = part[k];
            for (size_t i = b; i < e; ++i) {
                const Ref& r = rs[i];
                for (int ax = 0; ax < 3; ++ax) {
                    if (!live[ax]) continue;
                    int j = int((0.5f * (r.box.lo[ax] + r.box.hi[ax]) - cb.lo[ax]) * scale[ax]);
                    j = std::min(std::max(j, 0), kBins - 1);
                    P.enter[ax][j]++;
                    P.bb[ax][j].grow(r.box);
                }
            }
        });
        for (size_t k = 1; k < K; ++k)
            for (int ax = 0; ax < 3; ++ax)
                for (int j = 0; j < kBins; ++j) {
                    part[0].bb[ax][j].grow(part[k].bb[ax][j]);
                    part[0].enter[ax][j] += part[k].enter[ax][j];
                }
        const AxisBins& P = part[0];
        for (int ax = 0; ax < 3; ++ax) {
            if (!live[ax]) continue;
            const Box* bb = P.bb[ax];
            const uint32_t* bc = P.enter[ax];
            Box racc[kBins];
            uint32_t rcnt[kBins];
            Box acc;
            uint32_t cnt = 0;
            for (int k = kBins - 1; k > 0; --k) {
                acc.grow(bb[k]);
                cnt += bc[k];
                racc[k] = acc;
                rcnt[k] = cnt;
            }
            acc = Box();
            cnt = 0;
            for (int k = 0; k < kBins - 1; ++k) {
                acc.grow(bb[k]);
                cnt += bc[k];
                if (cnt == 0 || rcnt[k + 1] == 0) continue;
                const double c = acc.area() * cnt + racc[k + 1].area() * rcnt[k + 1];
                if (c < best.cost) {
                    best.cost = c;
                    best.axis = ax;
                    best.bin = k;
                    best.left = acc;
                    best.right = racc[k + 1];
                    best.lo = cb.lo[ax];
                    best.scale = scale[ax];
                }
            }
        }
        return best;
    }

    struct SpatSplit {
        double cost = DBL_MAX;
        int axis = -1;
        float plane = 0.f;
    };

    SpatSplit spatial_split(const std::vector<Ref>& rs, const Box& nb) const {
        SpatSplit best;
        float lo[3], bs[3];
        bool live[3];
        for (int ax = 0; ax < 3; ++ax) {
            lo[ax] = nb.lo[ax];
            const float ext = nb.hi[ax] - nb.lo[ax];
            live[ax] = ext > 0.f;
            bs[ax] = ext / float(kBins);
        }
        const size_t nk = max_chunks(rs.size());
        AxisBins local;
        std::vector<AxisBins> heap(nk > 1 ? nk : 0);
        AxisBins* part = nk > 1 ? heap.data() : &local;
        const size_t K = chunked(rs.size(), [&](size_t k, size_t b, size_t e) {
            AxisBins& P = part[k];
            for (int ax = 0; ax < 3; ++ax) {
                if (!live[ax]) continue;
                Box* bb = P.bb[ax];
                uint32_t* enter = P.enter[ax];
                uint32_t* exit_ = P.exit_[ax];
                for (size_t i = b; i < e; ++i) {
                    const Ref& r = rs[i];
                    if (keep_whole && keep_whole[r.tri]) {  // goes whole to the side of its centroid
                        int c = int((0.5f * (r.box.lo[ax] + r.box.hi[ax]) - lo[ax]) / bs[ax]);
                        c = std::min(std::max(c, 0), kBins - 1);
                        bb[c].grow(r.box);
                        enter[c]++;
                        exit_[c]++;
                        continue;
                    }
                    int b0 = int((r.box.lo[ax] - lo[ax]) / bs[ax]), b1 = int((r.box.hi[ax] - lo[ax]) / bs[ax]);
                    b0 = std::min(std::max(b0, 0), kBins - 1);
                    b1 = std::min(std::max(b1, b0), kBins - 1);
                    Ref cur = r;
                    for (int j = b0; j < b1; ++j) {
                        Box L, R;
                        split_ref(cur, ax, lo[ax] + bs[ax] * float(j + 1), L, R);
                        bb[j].grow(L);
                        cur.box = R;
                    }
                    bb[b1].grow(cur.box);
                    enter[b0]++;
                    exit_[b1]++;
                }
            }
        });
        for (size_t k = 1; k < K; ++k)
            for (int ax = 0; ax < 3; ++ax)
                for (int j = 0; j < kBins; ++j) {
                    part[0].bb[ax][j].grow(part[k].bb[ax][j]);
                    part[0].enter[ax][j] += part[k].enter[ax][j];
                    part[0].exit_[ax][j] += part[k].exit_[ax][j];
                }
        for (int ax = 0; ax < 3; ++ax) {
            if (!live[ax]) continue;
            const Box* bb = part[0].bb[ax];
            const uint32_t* enter = part[0].enter[ax];
            const uint32_t* exit_ = part[0].exit_[ax];
            Box racc[kBins];
            uint32_t rcnt[kBins];
            Box acc;
            uint32_t cnt = 0;
            for (int k = kBins - 1; k > 0; --k) {
                acc.grow(bb[k]);
                cnt += exit_[k];
                racc[k] = acc;
                rcnt[k] = cnt;
            }
            acc = Box();
            cnt = 0;
            for (int k = 0; k < kBins - 1; ++k) {
                acc.grow(bb[k]);
                cnt += enter[k];
                if (cnt == 0 || rcnt[k + 1] == 0) continue;
                const double c = acc.area() * cnt + racc[k + 1].area() * rcnt[k + 1];
                if (c < best.cost) {
                    best.cost = c;
                    best.axis = ax;
                    best.plane = lo[ax] + bs[ax] * float(k + 1);
                }
            }
        }
        return best;
    }

    static void concat(std::vector<std::vector<Ref>>& parts, size_t K, std::vector<Ref>& out) {
        if (K == 1) {
            out.swap(parts[0]);
            return;
        }
        size_t total = 0;
        for (size_t k = 0; k < K; ++k) total += parts[k].size();
        out.reserve(total);
        for (size_t k = 0; k < K; ++k) out.insert(out.end(), parts[k].begin(), parts[k].end());
    }

    // Partitions the references of a node (bounds nb, at `depth`, duplication allowance `budget`) into L
    // and R; returns the number of references it duplicated.
    size_t split_node(std::vector<Ref>& rs, const Box& nb, uint32_t depth, size_t budget, std::vector<Ref>& L,
                      std::vector<Ref>& R, Box& lb, Box& rb) const {
        const size_t n = rs.size();
        uint32_t levels = 0;
        for (size_t m = n; m > 1; m = (m + 1) / 2) ++levels;
        const bool tight = depth + levels + 3 >= depth_cap;
        size_t dup = 0;
        if (!tight) {
            const ObjSplit os = object_split(rs);
            SpatSplit ss;
            if (os.axis >= 0) {
                Box ov;
                for (int k = 0; k < 3; ++k) {
                    ov.lo[k] = std::max(os.left.lo[k], os.right.lo[k]);
                    ov.hi[k] = std::min(os.left.hi[k], os.right.hi[k]);
                }
                bool overlap = true;
                for (int k = 0; k < 3; ++k) overlap = overlap && ov.lo[k] <= ov.hi[k];
                if (overlap && ov.area() > alpha * root_area && budget > 0) ss = spatial_split(rs, nb);
            } else {
                if (budget > 0) ss = spatial_split(rs, nb);  // no object split separates these centroids
            }
            if (ss.axis >= 0 && ss.cost < os.cost) {
                const size_t nk = max_chunks(n);
                std::vector<std::vector<Ref>> Lk(nk), Rk(nk);
                std::vector<size_t> dk(nk, 0);
                std::vector<Box> lbk(nk), rbk(nk);
                if (nk == 1) {
                    Lk[0].reserve(n / 2 + 16);
                    Rk[0].reserve(n / 2 + 16);
                }
                const size_t K = chunked(n, [&](size_t k, size_t b, size_t e) {
                    auto left = [&](const Ref& r) {
                        Lk[k].push_back(r);
                        lbk[k].grow(r.box);
                    };
                    auto right = [&](const Ref& r) {
                        Rk[k].push_back(r);
                        rbk[k].grow(r.box);
                    };
                    for (size_t i = b; i < e; ++i) {
                        const Ref& r = rs[i];
                        if (r.box.hi[ss.axis] <= ss.plane) left(r);
                        else if (r.box.lo[ss.axis] >= ss.plane) right(r);
                        else {
                            Box bl, br;
                            const bool whole = keep_whole && keep_whole[r.tri];
                            if (!whole) split_ref(r, ss.axis, ss.plane, bl, br);
                            if (!whole && !bl.empty() && !br.empty() && bl.lo[ss.axis] <= bl.hi[ss.axis] && br.lo[ss.axis] <= br.hi[ss.axis]) {
                                left(Ref{r.tri, bl});
                                right(Ref{r.tri, br});
                                dk[k]++;
                            } else if (0.5f * (r.box.lo[ss.axis] + r.box.hi[ss.axis]) < ss.plane) {
                                left(r);
                            } else {
                                right(r);
                            }
                        }
                    }
                });
                concat(Lk, K, L);
                concat(Rk, K, R);
                for (size_t k = 0; k < K; ++k) {
                    dup += dk[k];
                    lb.grow(lbk[k]);
                    rb.grow(rbk[k]);
                }
                if (L.empty() || R.empty()) {
                    L.clear();
                    R.clear();
                    dup = 0;
                    lb = rb = Box();
                }
            }
            if (L.empty() && os.axis >= 0) {
                const size_t nk = max_chunks(n);
                std::vector<std::vector<Ref>> Lk(nk), Rk(nk);
                if (nk == 1) {
                    Lk[0].reserve(n / 2 + 16);
                    Rk[0].reserve(n / 2 + 16);
                }
                const size_t K = chunked(n, [&](size_t k, size_t b, size_t e) {
                    for (size_t i = b; i < e; ++i) {
                        const Ref& r = rs[i];
                        int j = int((0.5f * (r.box.lo[os.axis] + r.box.hi[os.axis]) - os.lo) * os.scale);
                        j = std::min(std::max(j, 0), kBins - 1);
                        (j <= os.bin ? Lk[k] : Rk[k]).push_back(r);
                    }
                });
                concat(Lk, K, L);
                concat(Rk, K, R);
                if (L.empty() || R.empty()) {
                    L.clear();
                    R.clear();
                } else {  // the bins' boxes on each side of the chosen plane: exactly the children's bounds
                    lb = os.left;
                    rb = os.right;
                }
            }
        }
        if (L.empty()) {  // object median along the widest centroid axis
            Box cb;
            for (const Ref& r : rs) {
                float c[3];
                for (int k = 0; k < 3; ++k) c[k] = 0.5f * (r.box.lo[k] + r.box.hi[k]);
                cb.grow(c);
            }
            int ax = 0;
            for (int k = 1; k < 3; ++k)
                if (cb.hi[k] - cb.lo[k] > cb.hi[ax] - cb.lo[ax]) ax = k;
            const size_t m = n / 2;
            std::nth_element(rs.begin(), rs.begin() + m, rs.end(), [&](const Ref& x, const Ref& y) {
                const float cx = x.box.lo[ax] + x.box.hi[ax], cy = y.box.lo[ax] + y.box.hi[ax];
                return cx < cy || (cx == cy && x.tri < y.tri);
            });
            L.assign(rs.begin(), rs.begin() + m);
            R.assign(rs.begin() + m, rs.end());
            lb = bounds_of(L);
            rb = bounds_of(R);
        }
        return dup;
    }

    // A subtree built by one task: node 0 its root, children after their parent; a child index kExternal | k
    // is the root of kids[k], a subtree built by a task of its own.  Stitched into one array at the end
    // (stitch): every node is copied once, whatever the nesting of tasks.
    static constexpr int32_t kExternal = int32_t(1u << 30);
    struct Sub {
        std::vector<TNode> nodes;
        std::vector<uint32_t> refs;
        std::vector<std::unique_ptr<Sub>> kids;
        size_t node_off = 0, ref_off = 0;  // in the stitched arrays
        bool deep = false;  // the depth cap was exceeded
        bool oom = false;   // a task ran out of memory
    };

    // Builds the subtree of `rs` (consumed; bounds nb) into out; returns the index of its root.  Children of at
    // least kTaskRefs references each are built as tasks -- by size alone, so the task structure and the tree
    // are the same for any thread count.
    int32_t build_rec(Sub& out, std::vector<Ref>& rs, const Box& nb, uint32_t depth, size_t budget) {
        const int32_t idx = int32_t(out.nodes.size());
        out.nodes.emplace_back();
        out.nodes[size_t(idx)].box = nb;
        const size_t n = rs.size();
        if (n <= 1) {
            TNode& t = out.nodes[size_t(idx)];
            t.first = uint32_t(out.refs.size());
            t.count = uint32_t(n);
            for (const Ref& r : rs) out.refs.push_back(r.tri);
            return idx;
        }
        if (depth + 1 > depth_cap) {
            out.deep = true;
            return idx;
        }
        std::vector<Ref> L, R;
        Box lb, rb;
        const size_t dup = split_node(rs, nb, depth, budget, L, R, lb, rb);
        std::vector<Ref>().swap(rs);
        // the allowance left after this split, shared in proportion to the children's references
        const size_t rest = budget > dup ? budget - dup : 0;
        const size_t bl = size_t(double(rest) * double(L.size()) / double(L.size() + R.size()));
        const size_t br = rest - bl;
        int32_t c0, c1;
        if (pool && L.size() >= kTaskRefs && R.size() >= kTaskRefs) {
            Sub* sr = new Sub;
            c1 = kExternal | int32_t(out.kids.size());
            out.kids.emplace_back(sr);
            std::atomic<bool> done{false};
            pool->submit([&, sr] {
                try {
                    build_rec(*sr, R, rb, depth + 1, br);
                } catch (...) {  // bad_alloc: reported by the caller, never thrown across threads
                    sr->oom = true;
                }
                done.store(true, std::memory_order_release);
            });
            try {
                c0 = build_rec(out, L, lb, depth + 1, bl);
            } catch (...) {  // the task references R, rb and done on this frame: let it end first
                pool->wait(done);
                throw;
            }
            pool->wait(done);
        } else {
            c0 = build_rec(out, L, lb, depth + 1, bl);
            c1 = build_rec(out, R, rb, depth + 1, br);
        }
        out.nodes[size_t(idx)].child[0] = c0;
        out.nodes[size_t(idx)].child[1] = c1;
        return idx;
    }

    // The task subtrees in one array (tree, refs): subtree blocks in the order root, then breadth-first over
    // the task tree; copied in parallel, external child indices resolved to their subtree's block.
    void stitch(Sub& root, TaskPool& tp, bool& deep, bool& oom) {
        std::vector<Sub*> subs{&root};
        for (size_t i = 0; i < subs.size(); ++i)
            for (auto& k : subs[i]->kids) subs.push_back(k.get());
        size_t nn = 0, nr = 0;
        for (Sub* x : subs) {
            x->node_off = nn;
            x->ref_off = nr;
            nn += x->nodes.size();
            nr += x->refs.size();
            deep |= x->deep;
            oom |= x->oom;
        }
        if (deep || oom) return;
        tree.resize(nn);
        refs.resize(nr);
        // every worker returns before this frame ends (fork_join): a worker the pool starts late still reads
        // `cursor`
        std::atomic<size_t> cursor{0};
        fork_join(tp, threads, [&](size_t) {
            for (size_t i; (i = cursor.fetch_add(1)) < subs.size();) {
                const Sub& x = *subs[i];
                for (size_t j = 0; j < x.nodes.size(); ++j) {
                    TNode t = x.nodes[j];
                    if (t.count) t.first += uint32_t(x.ref_off);
                    else
                        for (int c = 0; c < 2; ++c)
                            t.child[c] = (t.child[c] & kExternal) ? int32_t(x.kids[size_t(t.child[c] & ~kExternal)]->node_off)
                                                                  : t.child[c] + int32_t(x.node_off);
                    tree[x.node_off + j] = t;
                }
                std::copy(x.refs.begin(), x.refs.end(), refs.begin() + std::ptrdiff_t(x.ref_off));
            }
        });
    }

    bool build(uint32_t ntris, const std::vector<Box>& tri_box, std::string& err) {
        std::vector<Ref> all(ntris);
        for (uint32_t t = 0; t < ntris; ++t) all[t] = Ref{t, tri_box[t]};
        bool deep = false, oom = false;
        {
            TaskPool tp(threads);
            pool = &tp;
            const Box rb = bounds_of(all);
            root_area = std::max(rb.area(), 1e-30);
            Sub root;
            root.nodes.reserve(size_t(ntris) / 2 + 16);
            try {
                build_rec(root, all, rb, 0, ref_budget > ntris ? ref_budget - ntris : 0);
                stitch(root, tp, deep, oom);
            } catch (...) {
                oom = true;
            }
            pool = nullptr;
        }
        if (oom) {
            err = "build_bvh: out of memory";
            return false;
        }
        if (deep) {
            err = "build_bvh: depth cap exceeded";
            return false;
        }
        // (begin / end are not kept: the treelet pass and the collapse count and gather references by walking)
        sah = tree_sah(tree);
        return true;
    }
};

// Outward padding so that GPU slab tests with FMA rounding stay conservative.
Box padded(const Box& bx, float pad_abs) {
    if (bx.empty()) return bx;
    Box o;
    for (int k = 0; k < 3; ++k) {
        float m = std::max(std::fabs(bx.lo[k]), std::fabs(bx.hi[k]));
        float p = m * 7.62939453125e-06f + pad_abs;  // |coord| * 2^-17 + scene-relative term
        o.lo[k] = bx.lo[k] - p;
        o.hi[k] = bx.hi[k] + p;
    }
    return o;
}

// ---- treelet restructuring (Karras & Aila 2013) ---------------------------------------------------------
// Bottom-up, every internal node R roots a treelet: its two children, then repeatedly the treelet leaf of
// largest surface area replaced by its two children, up to kTreeletLeaves leaves.  A dynamic programme over
// the subsets of those leaves finds the binary topology of least SAH cost (C_node * area + the children's
// costs; a treelet leaf keeps its subtree and its cost), and the treelet's internal nodes are rewired into
// it when that is cheaper.  Leaves, their references and boxes are unchanged, so the tree is over the same
// geometry and traversal results cannot change (the triangle tests alone decide hits); the tree is then
// renumbered in depth-first order (children after parents, subtree references contiguous) for the
// collapse.  Costs: C_node = 1, C_tri = 1 per reference, as the SBVH's split search.
constexpr int kTreeletLeaves = 7;

// Restructures the treelet rooted at internal node r (cost[] holds every node's subtree SAH cost, its
// descendants' already final).  Touches only r's subtree.
void restructure_treelet(std::vector<TNode>& tree, std::vector<double>& cost, int32_t r) {
    constexpr int kMaxSub = 1 << kTreeletLeaves;
    double area[kMaxSub], best[kMaxSub];
    uint8_t split[kMaxSub];
    int32_t leaves[kTreeletLeaves], internals[kTreeletLeaves];
    int nl = 2, ni = 1;
    leaves[0] = tree[size_t(r)].child[0];
    leaves[1] = tree[size_t(r)].child[1];
    internals[0] = r;
    while (nl < kTreeletLeaves) {  // expand the treelet leaf of largest area
        int bi = -1;
        double ba = -1.0;
        for (int i = 0; i < nl; ++i)
            if (!tree[size_t(leaves[i])].count && tree[size_t(leaves[i])].box.area() > ba) {
                ba = tree[size_t(leaves[i])].box.area();
                bi = i;
            }
        if (bi < 0) break;
        const int32_t x = leaves[bi];
        internals[ni++] = x;
        leaves[bi] = tree[size_t(x)].child[0];
        leaves[nl++] = tree[size_t(x)].child[1];
    }
    if (nl < 3) return;  // two leaves have one topology
    const int full = (1 << nl) - 1;
    Box sbox[kMaxSub];  // the union of a subset's leaf boxes: the subset without its lowest leaf, grown by it
    for (int sset = 1; sset <= full; ++sset) {
        const int low = __builtin_ctz(unsigned(sset));
        sbox[sset] = sbox[sset & (sset - 1)];
        sbox[sset].grow(tree[size_t(leaves[low])].box);
        area[sset] = sbox[sset].area();
    }
    for (int i = 0; i < nl; ++i) best[1 << i] = cost[size_t(leaves[i])];
    // a proper subset of S is numerically smaller than S: increasing order is a valid DP order
    for (int sset = 1; sset <= full; ++sset) {
        if ((sset & (sset - 1)) == 0) continue;
        const int low = sset & -sset;
        double bc = DBL_MAX;
        int bp = 0;
        for (int p = (sset - 1) & sset; p; p = (p - 1) & sset) {  // partitions {P, S \ P} with S's lowest leaf in P
            if (!(p & low)) continue;
            const double c = best[p] + best[sset ^ p];
            if (c < bc) {
                bc = c;
                bp = p;
            }
        }
        best[sset] = area[sset] + bc;
        split[sset] = uint8_t(bp);
    }
    if (!(best[full] < cost[size_t(r)] * (1.0 - 1e-9))) return;
    // rewire: the new topology's internal nodes reuse the treelet's (r stays the root), assigned in the
    // pre-order of the new topology
    struct Rewire {
        std::vector<TNode>& tree;
        std::vector<double>& cost;
        const int32_t* leaves;
        const int32_t* internals;
        const uint8_t* split;
        const double* best;
        int next;
        int32_t build(int sset) {
            if ((sset & (sset - 1)) == 0) return leaves[__builtin_ctz(unsigned(sset))];
            const int32_t idx = internals[next++];
            const int p = split[sset];
            const int32_t x = build(p), y = build(sset ^ p);
            TNode& t = tree[size_t(idx)];
            t.child[0] = x;
            t.child[1] = y;
            t.box = tree[size_t(x)].box;
            t.box.grow(tree[size_t(y)].box);
            cost[size_t(idx)] = best[sset];
            return idx;
        }
    };
    Rewire{tree, cost, leaves, internals, split, best, 0}.build(full);
}

// Breadth-first order of the tree's nodes from the root (level_end[l]: end of level l in bfs).
void bfs_levels(const std::vector<TNode>& tree, std::vector<int32_t>& bfs, std::vector<size_t>& level_end) {
    bfs.clear();
    level_end.clear();
    bfs.reserve(tree.size());
    bfs.push_back(0);
    for (size_t b = 0; b < bfs.size();) {
        const size_t e = bfs.size();
        for (size_t i = b; i < e; ++i) {
            const TNode& t = tree[size_t(bfs[i])];
            if (!t.count) {
                bfs.push_back(t.child[0]);
                bfs.push_back(t.child[1]);
            }
        }
        level_end.push_back(e);
        b = e;
    }
}

// f(i) for i in [b, e) on the pool in chunks (serial below a threshold); returns after every call.
template <class F>
void parallel_range(TaskPool& pool, unsigned threads, size_t b, size_t e, F&& f) {
    const size_t n = e - b;
    const size_t K = pool.parallel() && n >= 4096 ? std::min<size_t>(size_t(threads) * 4u, n / 1024u) : 1u;
    if (K <= 1) {
        for (size_t i = b; i < e; ++i) f(i);
        return;
    }
    fork_join(pool, K, [&](size_t k) {
        for (size_t i = b + n * k / K; i < b + n * (k + 1) / K; ++i) f(i);
    });
}

// Leaves, references and node slots are kept; only the topology of internal nodes changes, so the tree is not
// renumbered: the collapse gathers each wide leaf's references by walking its (at most three-reference)
// binary subtree left to right, the order of a depth-first renumbering.
void restructure_treelets(std::vector<TNode>& tree, const std::vector<uint32_t>& refs, int passes, const uint8_t* alpha,
                          unsigned threads) {
    const size_t nn = tree.size();
    if (nn < 3) return;
    std::vector<double> cost(nn, 0.0);
    std::vector<uint8_t> fixed(nn, 0);  // subtree holds an alpha-tested reference: left as built
    const unsigned hw = std::max(1u, threads);
    TaskPool pool(hw);
    std::vector<int32_t> bfs;
    std::vector<size_t> level_end;
    // post-order of the subtree at `root`, internal nodes only
    auto post_order = [&](int32_t root, std::vector<int32_t>& order) {
        order.clear();
        std::vector<std::pair<int32_t, bool>> st{{root, false}};
        while (!st.empty()) {
            auto [n, done] = st.back();
            st.pop_back();
            if (tree[size_t(n)].count) continue;
            if (done) {
                order.push_back(n);
                continue;
            }
            st.push_back({n, true});
            st.push_back({tree[size_t(n)].child[1], false});
            st.push_back({tree[size_t(n)].child[0], false});
        }
    };
    for (int pass = 0; pass < passes; ++pass) {
        // costs bottom-up over the current topology, one breadth-first level at a time (deepest first)
        bfs_levels(tree, bfs, level_end);
        for (size_t l = level_end.size(); l-- > 0;) {
            parallel_range(pool, hw, l ? level_end[l - 1] : 0, level_end[l], [&](size_t i) {
                const size_t n = size_t(bfs[i]);
                const TNode& t = tree[n];
                if (t.count) {
                    cost[n] = t.box.area() * double(t.count);
                    uint8_t f = 0;
                    if (alpha)
                        for (uint32_t k = 0; k < t.count; ++k) f |= alpha[refs[t.first + k]];
                    fixed[n] = f;
                } else {
                    cost[n] = t.box.area() + cost[size_t(t.child[0])] + cost[size_t(t.child[1])];
                    fixed[n] = fixed[size_t(t.child[0])] | fixed[size_t(t.child[1])];
                }
            });
        }
        // disjoint subtrees at the cut depth are restructured in parallel (each bottom-up), the levels above
        // serially, deepest level first (every node after its descendants, as a post-order)
        constexpr size_t kCut = 7;
        std::vector<int32_t> roots;
        if (level_end.size() > kCut)
            for (size_t i = level_end[kCut - 1]; i < level_end[kCut]; ++i)
                if (!tree[size_t(bfs[i])].count) roots.push_back(bfs[i]);
        std::atomic<size_t> cursor{0};
        fork_join(pool, roots.empty() ? 1 : hw, [&](size_t) {
            std::vector<int32_t> order;
            for (size_t k; (k = cursor.fetch_add(1)) < roots.size();) {
                post_order(roots[k], order);
                for (int32_t n : order)
                    if (!fixed[size_t(n)]) restructure_treelet(tree, cost, n);
            }
        });
        for (size_t l = std::min(kCut, level_end.size()); l-- > 0;)
            for (size_t i = l ? level_end[l - 1] : 0; i < level_end[l]; ++i) {
                const int32_t n = bfs[i];
                if (!tree[size_t(n)].count && !fixed[size_t(n)]) restructure_treelet(tree, cost, n);
            }
    }
}

double tree_sah(const std::vector<TNode>& tree) {
    const double ra = std::max(tree[0].box.area(), 1e-30);
    double sah = 0.0;
    for (const TNode& t : tree) sah += t.box.area() / ra * (t.count ? double(t.count) : 1.0);
    return sah;
}

// ---- BVH2 emission -------------------------------------------------------------------------------------
struct Emit2 {
    const std::vector<TNode>& tree;
    float pad;
    std::vector<BvhNode> nodes;
    uint32_t max_depth = 0, leaves = 0;

    void write_child(uint32_t node, int slot, const Box& b, int32_t link) {
        BvhNode& n = nodes[node];
        Box p = padded(b, pad);
        float lo[3], hi[3];
        for (int k = 0; k < 3; ++k) {
            lo[k] = b.empty() ? FLT_MAX : p.lo[k];
            hi[k] = b.empty() ? -FLT_MAX : p.hi[k];
        }
        float* ab = slot == 0 ? n.a : n.b;
        ab[0] = lo[0]; ab[1] = hi[0]; ab[2] = lo[1]; ab[3] = hi[1];
        n.c[slot * 2 + 0] = lo[2];
        n.c[slot * 2 + 1] = hi[2];
        n.d[slot] = link;
    }
    int32_t link_of(int32_t t, uint32_t depth) {
        const TNode& tn = tree[t];
        if (tn.count) {
            leaves++;
            return encode_leaf(tn.first, tn.count);
        }
        uint32_t idx = uint32_t(nodes.size());
        nodes.emplace_back();
        std::memset(&nodes.back(), 0, sizeof(BvhNode));
        max_depth = std::max(max_depth, depth);
        for (int s = 0; s < 2; ++s) {
            int32_t c = tn.child[s];
            int32_t l = link_of(c, depth + 1);
            write_child(idx, s, tree[c].box, l);
        }
        return int32_t(idx);
    }
    void run() {
        const TNode& root = tree[0];
        if (root.count) {  // the root is always an internal node: leaf in child 0, empty child 1
            nodes.emplace_back();
            std::memset(&nodes.back(), 0, sizeof(BvhNode));
            write_child(0, 0, root.box, encode_leaf(root.first, root.count));
            write_child(0, 1, Box(), encode_leaf(0, 1));
            leaves = 1;
            max_depth = 1;
        } else {
            link_of(0, 0);
        }
    }
};

// ---- BVH8 emission -------------------------------------------------------------------------------------
struct Emit8 {
    const std::vector<TNode>& tree;
    const std::vector<uint32_t>& refs;
    float pad;
    std::vector<Bvh8Node> nodes;
    std::vector<uint32_t> tri_order;
    uint32_t max_depth = 0, leaves = 0;

    static float sgn(int o, int bit) { return (o & bit) ? -1.0f : 1.0f; }

    // SAH-optimal collapse of the binary tree into the 8-wide tree (Ylitie et al. 2017, sec. 3.1),
    // by dynamic programming over (binary node n, i = number of wide-node slots it may occupy):
    //   C(n, 1)  = min(leaf: A(n) * C_prim * tris(n)  [tris(n) <= kMaxLeafTris8],
    //                  node: A(n) * C_node + D(n, 8))
    //   D(n, i)  = min_k C(left, k) + C(right, i - k)     (split the slots between the children)
    //   C(n, i)  = min(C(n, i - 1), D(n, i))              (i >= 2)
    // C_prim / C_node: the traversal is memory-latency bound and each triangle test is a dependent
    // round trip like a node visit, so a triangle is priced at 1.5 node visits (tuned on the GPU).
    double kCNode = 1.0, kCPrim = 1.5;  // set from BvhBuildParams::leaf_cost
    std::vector<double> cost;     // [n * 8 + i], i in 1..7 (index 0: D(n, 8) for the node case)
    std::vector<uint8_t> pick;    // [n * 8 + i]: i == 1: 0 leaf / 1 node; i >= 2: 0 = use C(n, i-1), k = split
    std::vector<uint8_t> dsplit;  // k of D(n, 8)

    std::vector<uint32_t> ntri;   // references of each binary node's subtree
    bool is_leaf(int32_t t) const { return pick[size_t(t) * 8 + 1] == 0; }

    // The references of binary subtree t, left to right (a wide leaf: at most kMaxLeafTris8 of them).
    void leaf_refs(int32_t t, std::vector<uint32_t>& out) const {
        const TNode& n = tree[size_t(t)];
        if (n.count) {
            for (uint32_t i = 0; i < n.count; ++i) out.push_back(refs[n.first + i]);
            return;
        }
        leaf_refs(n.child[0], out);
        leaf_refs(n.child[1], out);
    }

    // C / D of binary node ni (its children's already final).
    void solve_node(size_t ni) {
        const TNode& n = tree[ni];
        const double A = n.box.area();
        double* C = &cost[ni * 8];
        uint8_t* P = &pick[ni * 8];
        const uint32_t nt = ntri[ni] = n.count ? n.count : ntri[size_t(n.child[0])] + ntri[size_t(n.child[1])];
        const double leaf = nt <= uint32_t(kMaxLeafTris8) ? A * kCPrim * double(nt) : DBL_MAX;
        if (n.count) {  // binary leaf
            for (int i = 1; i < 8; ++i) { C[i] = leaf; P[i] = 0; }
            C[0] = DBL_MAX;
            return;
        }
        const double* L = &cost[size_t(n.child[0]) * 8];
        const double* R = &cost[size_t(n.child[1]) * 8];
        auto D = [&](int i, uint8_t& bk) {
            double best = DBL_MAX;
            for (int k = 1; k < i; ++k) {
                double c = L[k] + R[i - k];
                if (c < best) { best = c; bk = uint8_t(k); }
            }
            return best;
        };
        uint8_t k8 = 1;
        const double d8 = D(8, k8);
        dsplit[ni] = k8;
        C[0] = d8;
        const double node = A * kCNode + d8;
        C[1] = std::min(leaf, node);
        P[1] = leaf <= node ? 0 : 1;
        for (int i = 2; i < 8; ++i) {
            uint8_t k = 1;
            const double d = D(i, k);
            if (d < C[i - 1]) { C[i] = d; P[i] = k; }
            else { C[i] = C[i - 1]; P[i] = 0; }
        }
    }

    // Every node's C / D, bottom-up: the binary tree's breadth-first levels, deepest first, each level's
    // nodes in parallel (a node reads only its children's results).
    void solve(TaskPool& pool) {
        const size_t nn = tree.size();
        cost.assign(nn * 8, 0.0);
        pick.assign(nn * 8, 0);
        dsplit.assign(nn, 0);
        ntri.assign(nn, 0);
        std::vector<int32_t> bfs;
        std::vector<size_t> level_end;
        bfs_levels(tree, bfs, level_end);
        for (size_t l = level_end.size(); l-- > 0;)
            parallel_range(pool, threads, l ? level_end[l - 1] : 0, level_end[l], [&](size_t i) { solve_node(size_t(bfs[i])); });
    }

    // Children of binary subtree t occupying at most i slots.
    void expand(int32_t t, int i, std::vector<int32_t>& ch) const {
        while (i > 1 && pick[size_t(t) * 8 + i] == 0) --i;
        if (i == 1 || tree[t].count) {
            ch.push_back(t);
            return;
        }
        const int k = pick[size_t(t) * 8 + i];
        expand(tree[t].child[0], k, ch);
        expand(tree[t].child[1], i - k, ch);
    }

    // The wide node for binary subtree t: its children per D(t, 8).
    void gather_children(int32_t t, std::vector<int32_t>& ch) const {
        ch.clear();
        if (tree[t].count) {
            ch.push_back(t);
            return;
        }
        const int k = dsplit[t];
        expand(tree[t].child[0], k, ch);
        expand(tree[t].child[1], 8 - k, ch);
    }

    // The wide node for binary subtree t, except its child and triangle bases: slot assignment, quantised
    // child boxes, leaf metadata.  Depends on t alone, so the nodes of a level are planned in parallel.
    struct Plan {
        Bvh8Node node;
        int32_t slot_of[8];
        uint32_t n_internal = 0, n_tris = 0;
    };

    void plan(int32_t t, Plan& P) const {
        P.n_internal = P.n_tris = 0;
        std::vector<int32_t> ch;
        gather_children(t, ch);
        // slot assignment: slot s is nearest for rays of octant 7 ^ s (greedy auction on centroids)
        Box nb;
        for (int32_t c : ch) nb.grow(tree[c].box);
        float pc[3];
        for (int k = 0; k < 3; ++k) pc[k] = 0.5f * (nb.lo[k] + nb.hi[k]);
        int32_t* slot_of = P.slot_of;
        std::fill(slot_of, slot_of + 8, -1);
        bool used[8] = {false, false, false, false, false, false, false, false};
        bool taken[8] = {false, false, false, false, false, false, false, false};
        float cost_cs[8][8];
        for (size_t c = 0; c < ch.size(); ++c) {
            const Box& b = tree[ch[c]].box;
            float off[3];
            for (int k = 0; k < 3; ++k) off[k] = 0.5f * (b.lo[k] + b.hi[k]) - pc[k];
            for (int s = 0; s < 8; ++s) {
                const int o = 7 ^ s;  // the octant for which slot s is visited first
                cost_cs[c][s] = -(off[0] * sgn(o, 4) + off[1] * sgn(o, 2) + off[2] * sgn(o, 1));
            }
        }
        for (size_t round = 0; round < ch.size(); ++round) {
            float best = -FLT_MAX;
            int bc = -1, bs = -1;
            for (size_t c = 0; c < ch.size(); ++c) {
                if (used[c]) continue;
                for (int s = 0; s < 8; ++s) {
                    if (taken[s]) continue;
                    if (cost_cs[c][s] > best) { best = cost_cs[c][s]; bc = int(c); bs = s; }
                }
            }
            used[bc] = true;
            taken[bs] = true;
            slot_of[bs] = ch[bc];
        }
        Bvh8Node& n = P.node;
        std::memset(&n, 0, sizeof(Bvh8Node));
        // quantisation frame: padded union box
        Box pb[8];
        Box ub;
        for (int s = 0; s < 8; ++s)
            if (slot_of[s] >= 0) {
                pb[s] = padded(tree[slot_of[s]].box, pad);
                ub.grow(pb[s]);
            }
        float scale[3];
        for (int k = 0; k < 3; ++k) {
            n.p[k] = ub.lo[k];
            float ext = ub.hi[k] - ub.lo[k];
            int e = -100;
            if (ext > 0.0f) {
                e = int(std::ceil(std::log2(double(ext) / 255.0)));
                e = std::max(e, -100);
            }
            for (;;) {  // make every child fit in [0, 255] quanta with float decode p + q * 2^e
                scale[k] = std::ldexp(1.0f, e);
                bool ok = true;
                for (int s = 0; s < 8 && ok; ++s) {
                    if (slot_of[s] < 0) continue;
                    double qh = std::ceil((double(pb[s].hi[k]) - n.p[k]) / scale[k]);
                    if (qh > 255.0) ok = false;
                    else if (std::fmaf(float(qh), scale[k], n.p[k]) < pb[s].hi[k] && qh + 1.0 > 255.0) ok = false;
                }
                if (ok) break;
                ++e;
            }
            n.e[k] = uint8_t(e + 127);
        }
        uint32_t tri_off = 0;
        for (int s = 0; s < 8; ++s) {
            if (slot_of[s] < 0) {  // empty slot: an inverted box the slab test never enters, meta 0
                for (int k = 0; k < 3; ++k) {
                    n.qlo[k][s] = 255;
                    n.qhi[k][s] = 0;
                }
                continue;
            }
            for (int k = 0; k < 3; ++k) {
                double ql = std::floor((double(pb[s].lo[k]) - n.p[k]) / scale[k]);
                double qh = std::ceil((double(pb[s].hi[k]) - n.p[k]) / scale[k]);
                ql = std::min(std::max(ql, 0.0), 255.0);
                qh = std::min(std::max(qh, 0.0), 255.0);
                while (ql > 0.0 && std::fmaf(float(ql), scale[k], n.p[k]) > pb[s].lo[k]) ql -= 1.0;
                while (qh < 255.0 && std::fmaf(float(qh), scale[k], n.p[k]) < pb[s].hi[k]) qh += 1.0;
                n.qlo[k][s] = uint8_t(ql);
                n.qhi[k][s] = uint8_t(qh);
            }
            if (is_leaf(slot_of[s])) {
                const uint32_t cnt = ntri[size_t(slot_of[s])];
                n.meta[s] = uint8_t((cnt << 5) | tri_off);
                tri_off += cnt;
            } else {
                n.imask |= uint8_t(1u << s);
                n.meta[s] = uint8_t(kMetaInternal | s);
                P.n_internal++;
            }
        }
        P.n_tris = tri_off;
    }

    // Breadth-first emission: the wide nodes of each level are contiguous and the top levels come
    // first, so a prefix of the node array is the top of the tree (the levels every ray visits stay
    // together in the caches).  A node's internal children stay contiguous.  Each level is planned in
    // parallel, then numbered in level order -- the numbering of one serial breadth-first pass.
    struct Pending {
        uint32_t idx;
        int32_t t;
    };
    unsigned threads = 1;

    void run() {
        TaskPool pool(threads);
        solve(pool);
        nodes.emplace_back();
        std::vector<Pending> level{{0u, 0}}, next;
        std::vector<Plan> plans;
        for (uint32_t depth = 0; !level.empty(); ++depth) {
            max_depth = std::max(max_depth, depth);
            plans.resize(level.size());
            const size_t K = pool.parallel() && level.size() >= 64 ? std::min<size_t>(size_t(threads) * 4u, level.size() / 16u) : 1u;
            if (K <= 1) {
                for (size_t i = 0; i < level.size(); ++i) plan(level[i].t, plans[i]);
            } else {
                const size_t n = level.size();
                fork_join(pool, K, [&](size_t k) {
                    for (size_t i = n * k / K; i < n * (k + 1) / K; ++i) plan(level[i].t, plans[i]);
                });
            }
            next.clear();
            for (size_t i = 0; i < level.size(); ++i) {
                const Plan& P = plans[i];
                const uint32_t base_child = uint32_t(nodes.size());
                nodes.resize(nodes.size() + P.n_internal);
                Bvh8Node& n = nodes[level[i].idx];
                n = P.node;
                n.base_child = base_child;
                n.base_tri = uint32_t(tri_order.size());
                uint32_t rank = 0;
                for (int s = 0; s < 8; ++s) {
                    const int32_t c = P.slot_of[s];
                    if (c < 0) continue;
                    if (is_leaf(c)) {
                        leaf_refs(c, tri_order);
                        leaves++;
                    } else {
                        next.push_back({base_child + rank++, c});
                    }
                }
            }
            level.swap(next);
        }
    }
};

}  // namespace

bool build_bvh(const float* tri_positions, uint32_t ntris, int width, BvhBuildResult& out, std::string& err,
               const BvhBuildParams* params) {
    if (ntris == 0) {
        err = "build_bvh: scene has no triangles";
        return false;
    }
    if (ntris >= (1u << 28)) {
        err = "build_bvh: too many triangles (leaf encoding holds 2^28)";
        return false;
    }
    if (width != 2 && width != 8) {
        err = "build_bvh: width must be 2 or 8";
        return false;
    }
    Builder B;
    // BVH8: full binary split (single-triangle leaves); the collapse forms the wide leaves.
    B.leaf_max = width == 8 ? 1u : uint32_t(kMaxLeafTris);
    B.prefer_leaf = width == 8 ? 1u : 4u;
    B.depth_cap = kMaxDepth2;
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
    const float pad = ext * 1e-6f + 1e-7f;
    out = BvhBuildResult();
    if (width == 2) {
        double sah = 0.0;
        if (!B.build(ntris, err, sah)) return false;
        out.sah_cost = sah;
        Emit2 E{B.tree, pad, {}, 0, 0};
        E.run();
        out.nodes = std::move(E.nodes);
        out.tri_order = std::move(B.refs);
        out.max_depth = E.max_depth;
        out.num_leaves = E.leaves;
        return true;
    }
    // BVH8: the SAH collapse does not bound the wide depth, so tighten the binary tree's depth cap
    // until the wide tree fits the traversal stack (kTraversalStack8 entries).
    static const uint32_t kCaps[] = {32u, 30u, 28u, 26u, 24u, 22u, 20u};
    const uint32_t max_depth8 = params && params->max_wide_depth ? params->max_wide_depth : uint32_t(kTraversalStack8) - 1u;
    std::vector<uint32_t> caps;
    if (params && params->binary_depth_cap) caps.push_back(params->binary_depth_cap);
    else caps.assign(std::begin(kCaps), std::end(kCaps));
    uint32_t last_depth = 0;
    const bool spatial = !params || params->spatial_splits;
    const uint32_t tp_param = params ? params->treelet_passes : BvhBuildParams().treelet_passes;
    // the treelet passes re-wire subtrees without regard to the depth cap: when no cap gives a shallow enough
    // tree with them, the caps are tried again without them
    std::vector<std::pair<uint32_t, uint32_t>> tries;  // (binary depth cap, treelet passes)
    for (uint32_t tp : {tp_param, 0u}) {
        if (tp == 0u && tp_param == 0u && !tries.empty()) break;
        for (uint32_t cap : caps) tries.push_back({cap, spatial ? tp : 0u});
        if (!spatial) break;
    }
    {
        for (const auto& [cap, tp] : tries) {
            double sah = 0.0;
            SpatialBuilder SB;
            const std::vector<TNode>* tree = &B.tree;
            const std::vector<uint32_t>* refs = &B.refs;
            double ph[3] = {0.0, 0.0, 0.0};
            auto tick = std::chrono::steady_clock::now();
            auto lap = [&](int k) {
                const auto now = std::chrono::steady_clock::now();
                ph[k] = std::chrono::duration<double, std::milli>(now - tick).count();
                tick = now;
            };
            if (spatial) {
                SB.pos = tri_positions;
                SB.keep_whole = params ? params->keep_whole : nullptr;
                SB.depth_cap = cap;
                SB.threads = build_threads(params);
                SB.ref_budget = size_t(double(ntris) * (params ? params->ref_budget : BvhBuildParams().ref_budget));
                if (!SB.build(ntris, B.tri_box, err)) return false;
                lap(0);
                if (tp > 0) restructure_treelets(SB.tree, SB.refs, int(tp), params ? params->keep_whole : nullptr, SB.threads);
                lap(1);
                sah = tp > 0 ? tree_sah(SB.tree) : SB.sah;
                tree = &SB.tree;
                refs = &SB.refs;
            } else {
                for (uint32_t t = 0; t < ntris; ++t) B.refs[t] = t;
                B.depth_cap = cap;
                if (!B.build(ntris, err, sah)) return false;
                lap(0);
            }
            Emit8 E{*tree, *refs, pad, {}, {}, 0, 0, 1.0, params ? params->leaf_cost : BvhBuildParams().leaf_cost, {}, {}, {}, {}};
            E.threads = build_threads(params);
            E.run();
            lap(2);
            last_depth = E.max_depth;
            if (E.max_depth > max_depth8) continue;
            if (E.tri_order.size() != refs->size()) {
                err = "build_bvh: BVH8 emission lost triangles";
                return false;
            }
            out.sah_cost = sah;
            out.wide_sah = (tree->front().box.area() + E.cost[0]) / tree->front().box.area();
            out.nodes8 = std::move(E.nodes);
            out.tri_order = std::move(E.tri_order);
            out.max_depth = E.max_depth;
            out.num_leaves = E.leaves;
            out.binary_depth_cap = cap;
            out.treelet_passes = spatial ? tp : 0u;
            for (int k = 0; k < 3; ++k) out.phase_ms[k] = ph[k];
            return true;
        }
    }
    err = "build_bvh: BVH8 deeper than the traversal stack (" + std::to_string(last_depth) + ")";
    return false;
}

}  // namespace dxrpt
