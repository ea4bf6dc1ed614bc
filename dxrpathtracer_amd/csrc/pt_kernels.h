// pt_kernels.h — launch interface of the wavefront kernels (pt_kernels.hip), used by dxrpt_api.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dxrpt.h"
#include "pt_layout.h"

namespace dxrpt {

// Per-frame wavefront buffers (all indexed as documented; sized for `capacity` paths).
//   path slot p in [0, num_paths): one path per pixel of the rendered tiles
//     ps_thr[p]  float4  (path throughput rgb, payload roughness)          RayTrace.hlsl:63-71
//     ps_rad[p]  float4  (radiance rgb accumulated so far, bits(isDiffuse))
//     ps_pix[p]  uint2   (global pixel index y*W+x, accumulation index)
//   queue index i in [0, q_count[d]) at radiance depth d (PathLength):
//     q_org[d&1][i] float4 (origin xyz, tmax)       rays in SoA-of-float4: one dwordx4 per lane
//     q_dir[d&1][i] float4 (direction xyz, bits(path slot))
//     hit[i]        float4 (b1, b2, bits(global tri id) or ~0u on miss, bits(geometry index))
//   shadow slot k of path p lives at [k * capacity + p]; sh_n[p] = pending slots of path p:
//     sh_org  float4 (origin xyz, tmax)
//     sh_dir  float4 (direction xyz, tmin)
//     sh_con  float4 (contribution rgb = pathThroughput * CalcLighting or sky*throughput, bits(force_opaque));
//                    k_shadow multiplies it by the visibility in place
//   sh_queue[j]   uint32 slot id of the j-th shadow ray of the current depth (compacted)
struct FrameBuffers {
    float4* ps_thr = nullptr;
    float4* ps_rad = nullptr;
    uint2* ps_pix = nullptr;
    float4* q_org[2] = {nullptr, nullptr};
    float4* q_dir[2] = {nullptr, nullptr};
    float4* hit = nullptr;
    uint32_t* sh_n = nullptr;
    uint32_t* sh_queue = nullptr;
    float4* sh_org = nullptr;
    float4* sh_dir = nullptr;
    float4* sh_con = nullptr;
    uint32_t* counters = nullptr;  // [0..15] queue counts by depth, [16..31] shadow ray counts by depth
    uint32_t capacity = 0;         // paths
    uint32_t shadow_slots = 0;     // slots per queue entry
};

struct SceneDev {
    const BvhNode* nodes = nullptr;     // width 2
    const Bvh8Node* nodes8 = nullptr;   // width 8
    const TriRecord* tris = nullptr;
    const dxrpt_mesh_vertex* vertices = nullptr;
    const uint32_t* indices = nullptr;
    const dxrpt_geometry_info* geoinfo = nullptr;
    const dxrpt_material* materials = nullptr;
    const TexDesc* texdesc = nullptr;
    const uint32_t* texels = nullptr;
    const uint16_t* sky = nullptr;
    const float* lut = nullptr;  // [0..255] unorm, [256..511] sRGB->linear
    uint32_t sky_res = 0;
    uint32_t num_textures = 0;
    int width = 8;  // BVH width actually built: 2 or 8
};

struct FrameParams {
    dxrpt_ray_trace_constants rtc;
    dxrpt_app_settings set;
    const dxrpt_spot_light* lights;  // device copy of LightConstants.Lights
    const dxrpt_tile* tiles;         // device copy
    const uint32_t* tile_prefix;     // num_tiles + 1 prefix sums of tile pixel counts
    float4* accum;
    uint32_t num_tiles;
    uint32_t num_paths;
    uint32_t width, height;
    unsigned long long* trav;        // non-null: count traversal work ([0..1] closest node/tri, [2..3] shadow)
    uint32_t persistent_blocks;      // grid of the persistent BVH8 traversal kernels; 0 = one thread per ray
    uint32_t refill_lanes;           // persistent kernels: refill once this many lanes of a wave are idle
};

// Kernel sequence of one frame: raygen, then (trace, shade, shadow) per depth 1..L-1, then accumulate.
// When `ev` is non-null, 2 + 3(L-1) + 1 events are recorded: before raygen and after each launch.
inline int frame_event_count(int L) { return 2 + 3 * (L - 1) + 1; }
hipError_t launch_frame(const SceneDev& scene, const FrameBuffers& fb, const FrameParams& fp, hipStream_t stream,
                        hipEvent_t* ev);

// Closest-hit / any-hit queries on arbitrary rays (dxrpt_trace_rays): rays are (o.xyz, tmin),
// (d.xyz, tmax) pairs; hits are (t, b1, b2, bits(global tri)) with t = -1 and tri = ~0 on miss.
hipError_t launch_trace_rays(const SceneDev& scene, const float4* rays, uint32_t n, uint32_t flags, float4* hits,
                             hipStream_t stream);

}  // namespace dxrpt
