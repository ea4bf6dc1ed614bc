// pt_kernels.h — launch interface of the path tracer's kernels (pt_kernels.hip), used by dxrpt_api.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dxrpt.h"
#include "pt_layout.h"

namespace dxrpt {

// Word index of texel (x, y) relative to TexDesc::offset; tiles_x = ceil(width / tile width).
__host__ __device__ __attribute__((always_inline)) inline uint32_t tex_tile_word(uint32_t x, uint32_t y, uint32_t tiles_x,
                                                                                 bool r8) {
    if (r8) return ((y >> 3) * tiles_x + (x >> 4)) * kTexTileWords + (y & 7u) * 4u + ((x & 15u) >> 2);
    return ((y >> 2) * tiles_x + (x >> 3)) * kTexTileWords + (y & 3u) * 8u + (x & 7u);
}

// Queue counters are sharded: a producer wave appends to one shard of the queue (wave % kQueueShards in
// the wavefront passes, its screen run in the split schedule), so concurrent waves spread their atomics
// over kQueueShards addresses instead of one.  Shard s of a queue owns positions [s * cap, (s + 1) * cap);
// consumers enumerate item i of the queue by walking the shard counts (queue_pos in pt_kernels.hip).
constexpr uint32_t kQueueShards = 64;
constexpr uint32_t kMaxDepthQueues = 16;  // radiance queues 0..15 by depth, shadow queues 16..31

// Radiance ray queue of one depth (SoA of 16-B words: one dwordx4 per lane, coalesced).  The path
// state travels with its ray, so every per-depth kernel reads and writes it at the queue position.
//   org[pos] float4 (origin xyz, tmax)
//   dir[pos] float4 (direction xyz, bits(path slot p) -- split schedule: bits(accumulation index))
//   thr[pos] float4 (path throughput rgb, payload roughness)                RayTrace.hlsl:63-71
//   rad[pos] float4 (radiance rgb accumulated so far, bits(payload IsDiffuse))
//   pix[pos] uint32 global pixel index y*W+x (CMJ pattern seed)
struct RayQueue {
    float4* org = nullptr;
    float4* dir = nullptr;
    float4* thr = nullptr;
    float4* rad = nullptr;
    uint32_t* pix = nullptr;
};

// Per-frame buffers.
//   path slot p in [0, num_paths): one path per pixel of the rendered tiles
//     ps_pix[p]  uint2   (global pixel index, accumulation index), written by raygen (wavefront)
//     px_rad[p]  float4  final path radiance (wavefront)
//   queue position pos in [0, qsize) of depth d (sharded layout, see above):
//     q[d&1]     RayQueue
//     hit[pos]   float4 (b1, b2, bits(global tri id) or ~0u on miss, bits(geometry index))     (wavefront)
//     fwd[pos]   uint32 position of the path's continuation ray in queue d+1, ~0u if the path ended
//     sh_n[pos]  uint32 number of shadow rays the vertex emitted; ray k lives in slot k * qsize + pos
//                (megakernel schedules: pos = the path slot / the tail's dense queue index):
//       sh_org  float4 (origin xyz, tmax)
//       sh_dir  float4 (direction xyz, tmin)
//       sh_con  float4 (contribution rgb = pathThroughput * CalcLighting or sky*throughput,
//                       bits(force_opaque)); k_shadow multiplies it by the visibility in place
//   sh_queue[spos]  uint32 slot id of a queued shadow ray (sharded layout with shard capacity cap_s)
struct FrameBuffers {
    uint2* ps_pix = nullptr;
    float4* px_rad = nullptr;
    RayQueue q[2];
    float4* hit = nullptr;
    uint32_t* fwd = nullptr;
    uint32_t* sh_n = nullptr;
    uint32_t* sh_queue = nullptr;
    float4* sh_org = nullptr;
    float4* sh_dir = nullptr;
    float4* sh_con = nullptr;
    uint32_t* counters = nullptr;  // [queue][shard]: 2 * kMaxDepthQueues * kQueueShards
    // megakernel frames: the other counter set of the ping-pong pair (the next frame's), zeroed by the
    // frame's first kernel's workgroup 0 -- so the next frame needs no fill launch (null: nothing to zero)
    uint32_t* counters_next = nullptr;
    bool counters_clean = false;   // counters already zero: launch_frame skips its fill
    uint32_t capacity = 0;         // paths
    uint32_t cap_r = 0;            // queue shard capacity (multiple of 64)
    uint32_t qsize = 0;            // kQueueShards * cap_r >= capacity
    uint32_t shadow_slots = 0;     // slots per queue position; shadow shard capacity = shadow_slots * cap_r
};

// Shard capacity for producers of at most `paths` items (one wave of producers adds <= 64 items per
// queue).  Wavefront passes: waves w, w + kQueueShards, ... share a shard.  Split schedule: shard
// w * kQueueShards / nw holds <= ceil(nw / kQueueShards) consecutive waves.  +1 wave of slack.
inline uint32_t queue_shard_capacity(uint32_t paths) {
    const uint32_t nw = (paths + 63u) / 64u;
    return 64u * ((nw + kQueueShards - 1u) / kQueueShards + 1u);
}

struct SceneDev {
    const Bvh8Node* nodes8 = nullptr;
    const TriRecord* tris = nullptr;
    const float4* tri_verts = nullptr;  // per global triangle: 3 MeshVertex records = 12 float4
    const GeoShade* geoshade = nullptr;  // per geometry: its material's textures, resolved
    const uint32_t* texels = nullptr;
    const uint16_t* sky = nullptr;
    const float* lut = nullptr;  // [0..255] unorm, [256..511] sRGB->linear
    const uint32_t* omm = nullptr;  // opacity micromap, kOmmWords per alpha-tested triangle slot (pt_layout.h); null: off
    uint32_t sky_res = 0;
    // LDS traversal stack, ints per lane: two words (node-group base, hit/internal masks) per entry,
    // entries = min(tree depth + 1, kStackLds8).  Less LDS per workgroup -> more resident waves.
    uint32_t stack_ints = 2u * kStackLds8;
    // group-stack entries kStackLds8 .. kTraversalStack8-1: [entry * spill_stride + global thread]
    uint2* spill8 = nullptr;
    uint32_t spill_stride = 0;  // >= the global thread count of every traversal launch using this slab
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
    unsigned long long* trav;        // non-null: count traversal work ([0..1] closest node/tri, [2..3] shadow, [4] hits)
    unsigned long long* wave_clock;  // census frames, non-null: per-wave (start, end) s_memrealtime stamps
    uint32_t packet;                 // wave-coherent traversal: bit 0/1 closest/any hit at depth 1, bit 2/3 at depth >= 2
    uint32_t timing_mask;            // per-kernel timing events: kinds (1 << DXRPT_K_*) bracketed
    uint32_t megakernel;             // 1: the frame runs as megakernel(s) (k_path, or k_path_head + k_path_tail)
    uint32_t megakernel_occupancy;   // k_path / k_path_head register budget: 4..7 waves per SIMD
    uint32_t num_cus;
    // DXRPT_OPT_WAVE_ORDER (k_path): wave w of the launch traces the paths of wave slot wave_order[w] (a
    // permutation, costliest first, built from the previous frame; null: identity).  Non-null wave_cost:
    // each wave slot's duration class (kWaveClasses log-scale classes of its s_memrealtime span, 0 =
    // costliest) goes to wave_cost[slot] and is counted in wave_hist[class].
    const uint32_t* wave_order;
    uint32_t* wave_cost;
    uint32_t* wave_hist;
    // Megakernel, path-ordered frames (DXRPT_OPT_XCD_CHUNK): workgroup i runs on XCD i mod 8, so the
    // kernel maps it to pixel block (8 t + (i mod 8 + t) mod 8) C + (i / 8) mod C, t = (i / 8) / C: each
    // XCD (own L2) takes runs of C consecutive 8x8 blocks, runs dealt to the XCDs in rotation.  0: block i.
    uint32_t xcd_chunk;
    // Depth-split megakernel (DXRPT_OPT_MEGAKERNEL_SPLIT): 1 = k_path_head (depth 1) then one compacting
    // k_path_tail per further depth; 0 = the single k_path.  tail_occupancy: the tails' register budget.
    uint32_t split;
    uint32_t tail_occupancy;
    // Overlapped frames (DXRPT_OPT_FRAME_OVERLAP): the megakernel schedules write each path's radiance to
    // stage[accumulation index] instead of blending it into accum; launch_accum_stage blends the frame's
    // paths afterwards.  Null: blend in the kernel.
    float4* stage = nullptr;
    uint32_t accum_extent = 0;  // 1 + the largest accumulation index of the tiles (DXRPT_DEBUG range checks)
};

constexpr uint32_t kWaveClasses = 256;
// words of one counter set: the sharded queue counters, padded to 16 B
constexpr uint32_t kCounterWords = 2 * 16 * 64 + 16;

// Kernel sequence of one wavefront frame: raygen, then (trace, shade, shadow, resolve) per depth 1..L-1,
// then accumulate.  With `aux` and 2 * kMaxDepthQueues `fork_ev` events, each depth's any-hit pass runs
// on `aux` concurrently with the next depth's closest-hit pass.  When `ev` is non-null (per-kernel
// timing), launch slot i = raygen, 1 + 4(d-1) + {trace, shade, shadow, resolve}, 1 + 4(L-1) =
// accumulate is bracketed by events ev[2i], ev[2i+1] on the stream it runs on.  A megakernel frame
// (fp.megakernel) records ev[0], ev[1] around its launches.
inline int frame_event_count(int L) { return 2 * (2 + 4 * (L - 1)); }
// Builds `order` (n wave slots, costliest first) from the classes in `cls` and their histogram `hist`
// (kWaveClasses counts) with `cursor` (kWaveClasses zeros) as scratch, and zeroes `hist_next` and
// `cursor_next` (the next frame's).  Order within a class is unspecified: it only schedules.
hipError_t launch_wave_order(const uint32_t* cls, const uint32_t* hist, uint32_t* cursor, uint32_t* hist_next,
                             uint32_t* cursor_next, uint32_t* order, uint32_t n, hipStream_t stream);

// *sched_out (if non-null) receives the DXRPT_SCHED_* bits of the schedule launched.
hipError_t launch_frame(const SceneDev& scene, const FrameBuffers& fb, const FrameParams& fp, hipStream_t stream,
                        hipEvent_t* ev, hipStream_t aux = nullptr, hipEvent_t* fork_ev = nullptr,
                        uint32_t* sched_out = nullptr);

// Lightmap baking (BakeRayGen) over a width x height lightmap.  launch_bake_compact lists the texels
// inside a UV island (pos.w != 0; the others are skipped by BakeRayGen) into list[0, *count), so the
// bake waves carry only live texels; launch_bake then traces list entries [first, first + span)
// (threads past *count exit), shadow slots indexed by entry - first (FrameBuffers sized for >= span
// paths).  Ray counts are added to fb.counters (the caller zeroes them once per bake pass).  fp
// carries the constants (rtc.TotalNumPixels = width * height, rtc.CurrSampleIdx = the bake sample
// index), settings, lights.
struct BakeArgs {
    const float4* pos;   // surface map: world position, w = 1 inside a UV island (0 outside)
    const float4* nrm;   // surface map: world normal
    float4* accum;       // rgb sum of valid samples, w = valid sample count (in/out)
    float4* lightmap;    // rgb average, w = 1
    const uint32_t* list;   // live texel indices (launch_bake_compact)
    const uint32_t* count;  // number of list entries (device)
    uint32_t width, height, first, span;
};
hipError_t launch_bake_compact(const float4* pos, uint32_t texels, uint32_t* list, uint32_t* count, hipStream_t stream);
hipError_t launch_bake(const SceneDev& scene, const FrameBuffers& fb, const FrameParams& fp, const BakeArgs& b,
                       hipStream_t stream);

// Closest-hit / any-hit queries on arbitrary rays (dxrpt_trace_rays): rays are (o.xyz, tmin),
// (d.xyz, tmax) pairs; hits are (t, b1, b2, bits(global tri)) with t = -1 and tri = ~0 on miss.
hipError_t launch_trace_rays(const SceneDev& scene, const float4* rays, uint32_t n, uint32_t flags, float4* hits,
                             hipStream_t stream);

// Global thread count of the largest traversal launch of a frame (sizes the stack spill slab): one
// lane per path slot in the megakernel schedules, one per possible shadow ray in the wavefront's.
uint32_t frame_traversal_threads(uint32_t num_paths, uint32_t shadow_slots, bool megakernel);
uint32_t trace_rays_threads(uint32_t n);

// Primary-only AOV of the frame's tiles into fp.accum (one float4 per path slot's accumulation index).
hipError_t launch_primary_aov(const SceneDev& scene, const FrameBuffers& fb, const FrameParams& fp, hipStream_t stream);
// RaygenShader's progressive blend (RayTrace.hlsl:140-148) of an overlapped frame's stage into fp.accum
// (the fp.num_paths paths of fp.tiles).
hipError_t launch_accum_stage(const FrameParams& fp, hipStream_t stream);

// SampleCMJ2D on device cases (x = sampleIdx, y = numSamplesX, z = numSamplesY, w = pattern) -> out.
hipError_t launch_sample_cmj(const uint4* cases, uint32_t n, float2* out, hipStream_t stream);

// DXRPT_DEBUG builds: the range-check record since the last call (synchronises the device, zeroes it;
// dxrpt_get_debug_record); word 7 = 1 in debug builds.
constexpr int kDebugWords = 8;
hipError_t read_debug_record(uint32_t out[kDebugWords]);
// DXRPT_DIAG_PHASES builds: the per-phase lane ticks since the last call (synchronises the device, zeroes them).
constexpr int kPhaseClockWords = 24;  // [0, 8) k_path, [8, 16) k_path_head, [16, 24) k_path_tail
hipError_t read_phase_ticks(unsigned long long out[kPhaseClockWords]);

}  // namespace dxrpt
