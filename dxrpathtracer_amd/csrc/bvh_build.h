// bvh_build.h — host BVH builders (replace the driver-side DXR BLAS build invoked at
// DXRPathTracer.cpp:2465-2473 with PREFER_FAST_TRACE).
//
// One binned-SAH binary tree is built over all triangles; it is then emitted either as the BVH2
// layout (BvhNode, 64 B) or collapsed into the compressed 8-wide layout (Bvh8Node, 80 B).
#pragma once
#include <stdint.h>
#include <string>
#include <vector>

#include "pt_layout.h"

namespace dxrpt {

struct BvhBuildResult {
    std::vector<BvhNode> nodes;       // BVH2: nodes[0] is the root; DFS order
    std::vector<Bvh8Node> nodes8;     // BVH8: nodes8[0] is the root
    std::vector<uint32_t> tri_order;  // leaf order -> global triangle id (BVH8 with spatial splits:
                                      // a triangle may appear more than once)
    uint32_t max_depth = 0;           // of the emitted layout
    uint32_t num_leaves = 0;
    double sah_cost = 0.0;            // binary tree, C_trav = 1, C_tri = 1, relative to root area
    double wide_sah = 0.0;            // BVH8: the collapse's cost (C_node = 1, C_tri = leaf_cost), relative to root area
    uint32_t binary_depth_cap = 0;    // BVH8: depth cap of the binary tree that was collapsed
    uint32_t treelet_passes = 0;      // BVH8: treelet passes of the tree that was collapsed
    double phase_ms[3] = {0.0, 0.0, 0.0};  // BVH8: binary (SBVH) build, treelet passes, collapse + emission
};

// Optional builder parameters (diagnostics; the product uses the defaults).
struct BvhBuildParams {
    uint32_t binary_depth_cap = 0;  // BVH8: force this binary depth cap (0: tighten until the tree fits)
    uint32_t max_wide_depth = 0;    // BVH8: accepted wide depth (0: kTraversalStack8 - 1)
    bool spatial_splits = true;     // BVH8: SBVH spatial splits
    double ref_budget = 1.15;       // BVH8: maximum triangle references / triangles with spatial splits
                                    // (r04: 2.0 is C4 -11 % but the Sponza proxy's tree one level
                                    // deeper, metric +0.8 %, slowest 1/8 share +5 %;
                                    // profiles/r04_ab_split_budget.txt, r04_shares_budget200.txt)
    double leaf_cost = 1.5;         // BVH8 collapse: SAH cost of a triangle test relative to a node visit
                                    // (latency-bound traversal: each test is a dependent memory round trip)
    // per global triangle, non-zero: never cut by a spatial split (an alpha-tested triangle: every extra
    // reference is another opacity test); null: every triangle may be split
    const uint8_t* keep_whole = nullptr;
    // BVH8 with spatial splits: passes of treelet restructuring (Karras & Aila 2013) of the binary tree
    // before the collapse (0: none; DXRPT_OPT_TREELET_PASSES).  r04: 1 pass -2.3 % metric, -1.4..-2.0 %
    // C2/C3/C5, C4 +0.6 %; 2 passes C4 +6 % (profiles/r04_ab_treelet.txt)
#ifndef DXRPT_TREELET_PASSES
#define DXRPT_TREELET_PASSES 1
#endif
    uint32_t treelet_passes = DXRPT_TREELET_PASSES;
    // host threads of the build (0: the host's CPUs, at most 16); the tree does not depend on it
    unsigned threads = 0;
};

// tri_positions: ntris * 9 floats (v0.xyz, v1.xyz, v2.xyz) in global triangle order.
// width 2 -> BVH2 (leaves <= kMaxLeafTris), width 8 -> compressed BVH8 (leaves <= kMaxLeafTris8).
// Deterministic: the same input always yields the same tree, whatever the thread count.
// BVH8: the binary depth cap is tightened until the wide tree fits kTraversalStack8 - 1 levels; at each cap a
// tree whose treelet passes made it too deep is first rebuilt without them.
bool build_bvh(const float* tri_positions, uint32_t ntris, int width, BvhBuildResult& out, std::string& err,
               const BvhBuildParams* params = nullptr);

}  // namespace dxrpt
