// bvh_build.h — host binned-SAH BVH2 builder (replaces the driver-side DXR BLAS build invoked at
// DXRPathTracer.cpp:2465-2473 with PREFER_FAST_TRACE).
#pragma once
#include <stdint.h>
#include <string>
#include <vector>

#include "pt_layout.h"

namespace dxrpt {

struct BvhBuildResult {
    std::vector<BvhNode> nodes;       // nodes[0] is the root; DFS order
    std::vector<uint32_t> tri_order;  // leaf order -> global triangle id
    uint32_t max_depth = 0;
    uint32_t num_leaves = 0;
    double sah_cost = 0.0;            // C_trav = 1, C_tri = 1, relative to root area
};

// tri_positions: ntris * 9 floats (v0.xyz, v1.xyz, v2.xyz) in global triangle order.
// Deterministic: the same input always yields the same tree.
bool build_bvh(const float* tri_positions, uint32_t ntris, BvhBuildResult& out, std::string& err);

}  // namespace dxrpt
