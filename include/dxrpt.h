/*
 * dxrpt.h — C ABI of the MI355X-native path tracer (gfx950 / HIP).
 *
 * This is the drop-in boundary for the reference's DXR `DispatchRays` path
 * (WANG-Ruipeng/DXRPathTracer).  Every entry point below replaces one piece of
 * the reference's D3D12 binding of that path; the replaced interface is cited
 * as file:line relative to the reference tree.
 *
 *   reference                                   replaced by
 *   ------------------------------------------  --------------------------------
 *   Model::CreateBuffers vertex/index SRVs      dxrpt_set_scene
 *     (SampleFramework12/v1.02/Graphics/Model.cpp:851-881)
 *   GeometryInfo buffer (DXRPathTracer.cpp:2363-2367, 2477-2484)
 *   Material SRV table (MeshRenderer.cpp:158-186)
 *   LoadMaterialResources texture SRVs         dxrpt_add_texture
 *     (Graphics/Model.cpp:104-149)
 *   SkyCache::CubeMap (Graphics/Skybox.cpp:160-201)   dxrpt_set_sky
 *   BuildRTAccelerationStructure               dxrpt_build_bvh
 *     (DXRPathTracer.cpp:2331-2488)
 *   RenderRayTracing / DispatchRays(W,H,1)     dxrpt_render
 *     (DXRPathTracer.cpp:2024-2090)
 *   HUD ray count (DXRPathTracer.cpp:2171-2174) dxrpt_get_stats
 *   DXCall/Exception (Exceptions.h:260-290)    int status + dxrpt_last_error
 *
 * Conventions
 *   - All functions return 0 (DXRPT_OK) on success, a negative DXRPT_E_* code on
 *     failure; no C++ exception crosses the ABI.  dxrpt_last_error() returns a
 *     human-readable description of the last failure on that context.
 *   - Host pointers are only read during the call (scene data is deep-copied to
 *     device memory owned by the context).
 *   - The accumulation target is CALLER-owned device memory (the reference's
 *     `rtTarget` RGBA32F UAV, DXRPathTracer.cpp:919-927).
 *   - dxrpt_render only enqueues work on `stream` (a hipStream_t, or NULL for
 *     the default stream); the caller synchronises.
 *   - Stream ordering: every call that reads or writes context-owned buffers or the accumulation
 *     target (dxrpt_render, dxrpt_render_aov, dxrpt_trace_rays, dxrpt_bake_lightmap,
 *     dxrpt_post_process) runs after all such work the context enqueued before it, on whatever stream
 *     the caller passes: a call on a different stream than the previous call first makes its stream
 *     wait for the previous stream's work (one command queue, as the reference's, Graphics/DX12.cpp:
 *     263-305).  Overlapped frames (DXRPT_OPT_FRAME_OVERLAP) keep this: a frame's result is in `accum`
 *     once the stream of its call reaches the point where dxrpt_render returned.
 *   - One host thread per context.
 */
#ifndef DXRPT_H_
#define DXRPT_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DXRPT_ABI_VERSION 4

/* ---- status codes ---------------------------------------------------------------------------- */
#define DXRPT_OK 0
#define DXRPT_E_INVALID_ARG (-1)
#define DXRPT_E_HIP (-2)
#define DXRPT_E_NO_DEVICE (-3)
#define DXRPT_E_STATE (-4)      /* call out of order (e.g. render before build_bvh) */
#define DXRPT_E_OOM (-5)
#define DXRPT_E_UNSUPPORTED (-6)

/* ---- limits mirrored from AppSettings.hlsl:53-60 ----------------------------------------------- */
#define DXRPT_MAX_SPOT_LIGHTS 32u           /* MaxSpotLights (AppSettings.hlsl:53) */
#define DXRPT_MAX_PATH_LENGTH 8u            /* MaxPathLengthSetting (AppSettings.hlsl:60) */
#define DXRPT_SPOT_SHADOW_NEAR_CLIP 0.1f    /* SpotShadowNearClip (AppSettings.hlsl:56) */
#define DXRPT_INVALID_INDEX 0xFFFFFFFFu     /* Material.Opacity when no opacity map (MeshRenderer.cpp:158-186) */

/* ---- texture formats (dxrpt_add_texture) ------------------------------------------------------ */
#define DXRPT_TEX_RGBA8_UNORM 0u  /* 4 x u8, linear */
#define DXRPT_TEX_RGBA8_SRGB 1u   /* 4 x u8, rgb sRGB-decoded per texel (ForceSRGB albedo, Model.cpp:140) */
#define DXRPT_TEX_R8_UNORM 2u     /* 1 x u8 (e.g. BC4 opacity decoded on the host) */

/* ---- POD types, byte-identical to the reference layouts ---------------------------------------- */

/* MeshVertex, 64 B: SampleFramework12/v1.02/Graphics/Model.h:25-67, Shaders/RayTracing.hlsl:13-21 */
typedef struct dxrpt_mesh_vertex {
    float Position[3];
    float Normal[3];
    float UV[2];
    float Tangent[3];
    float Bitangent[3];
    float LightmapUV[2];
} dxrpt_mesh_vertex;

/* GeometryInfo, 16 B: DXRPathTracer/SharedTypes.h:58-64 */
typedef struct dxrpt_geometry_info {
    uint32_t VtxOffset;   /* in vertices */
    uint32_t IdxOffset;   /* in indices (not bytes) */
    uint32_t MaterialIdx;
    uint32_t PadTo16Bytes;
} dxrpt_geometry_info;

/* Material, 24 B: DXRPathTracer/SharedTypes.h:30-38.  Each field is a texture index returned by
 * dxrpt_add_texture (the reference stores SRV descriptor indices). Opacity == DXRPT_INVALID_INDEX
 * marks the geometry opaque (D3D12_RAYTRACING_GEOMETRY_FLAG_OPAQUE, DXRPathTracer.cpp:2348,2361). */
typedef struct dxrpt_material {
    uint32_t Albedo;
    uint32_t Normal;
    uint32_t Roughness;
    uint32_t Metallic;
    uint32_t Opacity;
    uint32_t Emissive;
} dxrpt_material;

/* SpotLight, 48 B: DXRPathTracer/SharedTypes.h:40-48 */
typedef struct dxrpt_spot_light {
    float Position[3];
    float AngularAttenuationX;
    float Direction[3];
    float AngularAttenuationY;
    float Intensity[3];
    float Range;
} dxrpt_spot_light;

/* LightConstants, 3584 B: DXRPathTracer.cpp:131-135, RayTrace.hlsl:46-50 */
typedef struct dxrpt_light_constants {
    dxrpt_spot_light Lights[DXRPT_MAX_SPOT_LIGHTS];
    float ShadowMatrices[DXRPT_MAX_SPOT_LIGHTS][16];
} dxrpt_light_constants;

/* RayTraceConstants, 156 B: DXRPathTracer.cpp:145-165, RayTrace.hlsl:24-44.
 * InvViewProjection is row-major and used with the row-vector convention mul(float4, M).
 * The five *Idx fields are bindless SRV indices in the reference; here the context owns the
 * buffers and they are ignored (kept for layout identity). */
typedef struct dxrpt_ray_trace_constants {
    float InvViewProjection[16];
    float SunDirectionWS[3];
    float CosSunAngularRadius;
    float SunIrradiance[3];
    float SinSunAngularRadius;
    float SunRenderColor[3];
    uint32_t Padding;
    float CameraPosWS[3];
    uint32_t CurrSampleIdx;
    uint32_t TotalNumPixels;
    uint32_t VtxBufferIdx;
    uint32_t IdxBufferIdx;
    uint32_t GeometryInfoBufferIdx;
    uint32_t MaterialBufferIdx;
    uint32_t SkyTextureIdx;
    uint32_t NumLights;
} dxrpt_ray_trace_constants;

/* AppSettingsCBuffer, 124 B: DXRPathTracer/AppSettings.h:97-128 (bool32 -> uint32_t), defaults in
 * AppSettings.cpp:95-208 (dxrpt_default_settings fills them). */
typedef struct dxrpt_app_settings {
    uint32_t EnableSun;
    uint32_t EnableSky;
    uint32_t SunAreaLightApproximation;
    float SunSize;
    float SunDirection[3];
    int32_t MSAAMode;
    uint32_t RenderLights;
    uint32_t EnableRayTracing;
    uint32_t ClampRoughness;
    uint32_t AvoidCausticPaths;
    int32_t SqrtNumSamples;
    int32_t MaxPathLength;
    int32_t MaxAnyHitPathLength;
    float Exposure;
    float BloomExposure;
    float BloomMagnitude;
    float BloomBlurSigma;
    uint32_t EnableAlbedoMaps;
    uint32_t EnableNormalMaps;
    uint32_t EnableDiffuse;
    uint32_t EnableSpecular;
    uint32_t EnableDirect;
    uint32_t EnableIndirect;
    uint32_t EnableIndirectSpecular;
    uint32_t ApplyMultiscatteringEnergyCompensation;
    float RoughnessScale;
    float MetallicScale;
    uint32_t EnableWhiteFurnaceMode;
    uint32_t EnableLightMapRender;
} dxrpt_app_settings;

/* A screen-space tile of the W x H image rendered by one dxrpt_render call.  Pixel (x, y) of the
 * tile (x0 <= x < x0+w, y0 <= y < y0+h) is written to
 *     accum[accum_offset + (y - y0) * accum_pitch + (x - x0)]      (float4 units)
 * The CMJ pattern always uses the GLOBAL pixel index y * W + x and TotalNumPixels (RayTrace.hlsl:85-96),
 * so any tiling produces bit-identical pixels.  A NULL tile list means one full-frame tile with
 * accum_offset 0 and accum_pitch W (the reference's rtTarget). */
typedef struct dxrpt_tile {
    uint32_t x0, y0, w, h;
    uint64_t accum_offset;
    uint32_t accum_pitch;
    uint32_t pad;
} dxrpt_tile;

/* Kernel kinds for the per-kernel timings in dxrpt_stats. */
#define DXRPT_K_RAYGEN 0
#define DXRPT_K_TRACE 1       /* closest-hit traversal of radiance rays (all depths) */
#define DXRPT_K_SHADE 2
#define DXRPT_K_SHADOW 3      /* any-hit traversal of shadow rays (all depths) */
#define DXRPT_K_ACCUMULATE 4
#define DXRPT_K_RESOLVE 5     /* adds visibility-weighted shadow contributions to path radiance */
#define DXRPT_K_PATH 6        /* megakernel frames (DXRPT_OPT_MEGAKERNEL_PATHS): all of the frame's launches */
#define DXRPT_K_PATH_HEAD 7   /* depth-split frames: k_path_head (raygen + depth 1) */
#define DXRPT_K_PATH_TAIL 8   /* depth-split frames: the k_path_tail launches (depths >= 2), back to back */
#define DXRPT_K_COUNT 9

/* Counters of the last dxrpt_render call (read back with a stream sync in dxrpt_get_stats), plus
 * per-kernel HIP-event timings accumulated since dxrpt_reset_timing (DXRPT_OPT_KERNEL_TIMING). */
typedef struct dxrpt_stats {
    uint64_t pixels;                   /* paths started */
    uint64_t radiance_rays;            /* closest-hit rays traced (all depths) */
    uint64_t shadow_rays;              /* any-hit rays traced */
    uint64_t nominal_rays;             /* W*H*(1+2(L-1)) of the rendered pixels, DXRPathTracer.cpp:2171 */
    uint64_t radiance_rays_per_depth[DXRPT_MAX_PATH_LENGTH];
    uint64_t shadow_rays_per_depth[DXRPT_MAX_PATH_LENGTH];
    /* DXRPT_OPT_COUNT_TRAVERSAL only (last render): BVH node and triangle-record FETCHES of the schedule
       that ran -- one per lane per visit in per-lane traversals, one per wave per visit in the
       wave-coherent packet traversals (scalar loads) */
    uint64_t node_visits_radiance, tri_tests_radiance, node_visits_shadow, tri_tests_shadow;
    /* DXRPT_OPT_KERNEL_TIMING only: summed kernel durations (ms) and launches since the last reset */
    double kernel_ms[DXRPT_K_COUNT];
    uint64_t kernel_launches[DXRPT_K_COUNT];
    uint64_t timed_frames;
    double frame_ms;                   /* summed raygen-start -> accumulate-end time of the timed frames */
    /* The schedule the last dxrpt_render ran (DXRPT_SCHED_* bits), the paths each 64-lane wave of its
       megakernel carried (64; 0 for the wavefront passes), its register budget in waves per SIMD (the
       head's on a depth-split frame) and the tails' (depth-split frames, else 0). */
    uint32_t schedule;
    uint32_t paths_per_wave;
    uint32_t occupancy;
    uint32_t tail_occupancy;
    /* DXRPT_OPT_COUNT_TRAVERSAL on a megakernel frame: radiance rays that hit a triangle (the vertices
       PathTrace shades); the other radiance rays ran MissShader.  0 otherwise. */
    uint64_t radiance_hits;
    /* DXRPT_OPT_COUNT_TRAVERSAL: the part of the census above that belongs to depth-1 vertices (the split
       schedule's head kernel; the rest is its tails'): node and triangle fetches of closest-hit and of
       any-hit rays, and (megakernel census) radiance hits. */
    uint64_t census_depth1[5];
    /* Materials of the scene's geometries shaded from one packed normal / metallic / roughness tap
       (DXRPT_OPT_PACKED_TAPS), and the packed textures built for them. */
    uint32_t packed_materials;
    uint32_t packed_textures;
    /* Geometry texture references inlined as constants (1 x 1 maps, DXRPT_OPT_PACKED_TAPS bit 1). */
    uint32_t inlined_maps;
    uint32_t reserved0;
} dxrpt_stats;
#define DXRPT_SCHED_MEGAKERNEL 1u    /* k_path (or the split head/tail kernels): no wavefront passes */
/* 2u (path groups) and 64u (two concurrent halves) are retired (ABI 3) */
#define DXRPT_SCHED_ORDER_KERNEL 4u  /* the cost-ordered instantiation ran (it records wave costs) */
#define DXRPT_SCHED_COST_ORDERED 8u  /* ... and started the waves in a cost order built by earlier frames */
#define DXRPT_SCHED_CENSUS 16u       /* the counting (DXRPT_OPT_COUNT_TRAVERSAL) instantiation */
#define DXRPT_SCHED_SPLIT 32u        /* depth-split megakernel: k_path_head then compacted k_path_tail */
#define DXRPT_SCHED_OVERLAP 128u     /* overlapped with its neighbour frames (DXRPT_OPT_FRAME_OVERLAP) */

/* BVH summary (dxrpt_get_bvh_info). */
typedef struct dxrpt_bvh_info {
    uint32_t num_nodes;
    uint32_t num_leaves;
    uint32_t num_tris;
    uint32_t max_depth;
    uint32_t node_bytes;      /* bytes per node of the layout traversed on the GPU */
    uint32_t tri_bytes;       /* bytes per leaf triangle record */
    uint32_t width;           /* 8: compressed BVH8, 80-B nodes */
    uint32_t num_refs;        /* leaf triangle references (spatial splits reference a triangle more than once) */
    double build_ms;          /* host build time, dxrpt_build_bvh call to return (replaces the timed BLAS/TLAS
                                 build, DXRPathTracer.cpp:2465-2473, logged at :1499-1500) */
    double sah_cost;
    /* ABI 4: the parts of build_ms -- binary SBVH, treelet passes, BVH8 collapse and emission, and the rest
       (triangle records, per-triangle vertices, uploads) -- and the build's shape */
    double phase_ms[4];
    double wide_sah;          /* SAH cost of the BVH8 collapse (node visit 1, triangle test DXRPT_OPT_LEAF_COST) */
    uint32_t binary_depth_cap;  /* the binary depth cap the accepted tree was built with */
    uint32_t treelet_passes;  /* treelet passes of the accepted tree (0 when they made it too deep) */
    uint32_t threads;         /* builder threads (DXRPT_OPT_BVH_THREADS); the tree does not depend on them */
    uint32_t ref_budget_pct;  /* spatial-split reference budget, percent of the triangles (DXRPT_OPT_SPATIAL_SPLITS) */
} dxrpt_bvh_info;

typedef struct dxrpt_ctx dxrpt_ctx;

/* ---- lifecycle -------------------------------------------------------------------------------- */
/* Capability check at create: gfx9xx device with >= 64 KiB LDS (replaces the SM 6.6 / DXR 1.1 checks
 * of Graphics/DX12.cpp:141-165). */
int dxrpt_create(int hip_device, dxrpt_ctx** out_ctx);
int dxrpt_destroy(dxrpt_ctx* ctx);
const char* dxrpt_last_error(const dxrpt_ctx* ctx);
int dxrpt_abi_version(void);
/* Fill `s` with the reference defaults (AppSettings.cpp:95-208). */
void dxrpt_default_settings(dxrpt_app_settings* s);

/* ---- scene ------------------------------------------------------------------------------------ */
/* Vertex/index/geometry/material tables (Model.cpp:851-881, DXRPathTracer.cpp:2363-2367).
 * idx_bytes is 2 (R16_UINT) or 4 (R32_UINT); indices are mesh-local, offset by VtxOffset. */
int dxrpt_set_scene(dxrpt_ctx* ctx,
                    const dxrpt_mesh_vertex* vertices, uint32_t num_vertices,
                    const void* indices, uint32_t idx_bytes, uint32_t num_indices,
                    const dxrpt_geometry_info* geometries, uint32_t num_geometries,
                    const dxrpt_material* materials, uint32_t num_materials);
/* Adds a w x h texture (mip 0) of format DXRPT_TEX_*; out_index receives the index to store in
 * dxrpt_material fields.  Indices are assigned 0, 1, 2, ... in call order. */
int dxrpt_add_texture(dxrpt_ctx* ctx, uint32_t w, uint32_t h, uint32_t fmt, const void* texels,
                      uint32_t* out_index);
/* Sky cubemap: 6 faces (+x,-x,+y,-y,+z,-z) of res x res RGBA16F texels, face-major then row-major
 * (the SkyCache::CubeMap layout, Graphics/Skybox.cpp:160-201). */
int dxrpt_set_sky(dxrpt_ctx* ctx, const uint16_t* rgba16f_cube, uint32_t res);
/* Builds the acceleration structure over the scene set by dxrpt_set_scene (one BLAS over all
 * geometries + identity instance in the reference; here one binned-SAH BVH over all triangles).
 * Fails with DXRPT_E_INVALID_ARG when the node or triangle-record array would reach 4 GiB (the
 * kernels address records by 32-bit byte offsets: about 80 M triangle references). */
int dxrpt_build_bvh(dxrpt_ctx* ctx);
int dxrpt_get_bvh_info(const dxrpt_ctx* ctx, dxrpt_bvh_info* info);

/* ---- options ----------------------------------------------------------------------------------
 * Retired in ABI 3 (measured slower or neutral on MI355X; DESIGN.md §7a holds the table and the A/B
 * records): 3 BVH_WIDTH, 4-7 wave-pool traversal, 8-11 and 14-15 wavefront launch shapes and budgets,
 * 16 CONCURRENCY, 17 TRAVERSAL_PIPELINE, 19 LDS_NODES, 21 XCD_MAPPING, 22 PACKET_SWITCH,
 * 26 MEGAKERNEL_PERSISTENT, 27 MEGAKERNEL_LANES (path groups), 30 SPLIT_UNITS, 35 SPLIT_PARTS,
 * 38 SPLIT_BINS, 39 SPLIT_ALPHA.  dxrpt_set_option rejects them with DXRPT_E_UNSUPPORTED, ids that were
 * never assigned with DXRPT_E_INVALID_ARG.  The list, once (the library and the tests read it here): */
#define DXRPT_RETIRED_OPTIONS {3u, 4u, 5u, 6u, 7u, 8u, 9u, 10u, 11u, 14u, 15u, 16u, 17u, 19u, 21u, 22u, 26u, 27u, 30u, 35u, 38u, 39u}
#define DXRPT_OPT_COUNT_TRAVERSAL 1u  /* 1: instrumented kernels of the same schedule count node / triangle
                                         fetches (slower; images identical) */
#define DXRPT_OPT_KERNEL_TIMING 2u    /* 1: record hipEvents around the launches of dxrpt_render */
#define DXRPT_OPT_SPATIAL_SPLITS 12u  /* BVH8 build: spatial-split reference budget in percent of the triangle count
                                         (101..400; <= 100 disables spatial splits; default 115) */
#define DXRPT_OPT_LEAF_COST 13u       /* BVH8 build: triangle-test cost in percent of a node visit (default 150) */
#define DXRPT_OPT_PACKET_TRAVERSAL 18u /* BVH8 wave-coherent traversal (the 64 rays of a wave share one node
                                          sequence fetched with scalar loads) per pass, bit mask: 1 = closest
                                          hit at depth 1 (primary rays), 2 = any hit at depth 1 (megakernel:
                                          the sun shadow rays of the primary hits), 4 = closest hit at depth
                                          >= 2, 8 = any hit at depth >= 2 (wavefront only); default 3.
                                          Identical results. */
#define DXRPT_OPT_KERNEL_TIMING_MASK 20u /* kernel kinds bracketed by events when DXRPT_OPT_KERNEL_TIMING is on
                                            (bit 1 << DXRPT_K_*, default all); the frame span is always timed.
                                            Fewer events, less timing overhead in the measured frames. */
#define DXRPT_OPT_MEGAKERNEL_PATHS 23u /* frames of at most this many path vertices (paths x (MaxPathLength-1);
                                            default 0xFFFFFFFF: every frame) run as megakernels, one lane per
                                            path (the single k_path, or the depth-split k_path_head +
                                            k_path_tail); larger frames run the wavefront passes (one kernel
                                            per stage and depth, compacted queues between depths).  0 = always
                                            the wavefront.  Identical results. */
#define DXRPT_OPT_MEGAKERNEL_OCCUPANCY 24u /* megakernel register budget in waves/SIMD: 0 = by frame size
                                              (default: 7 above 600,000 paths, 5 from 300,000 with overlapped
                                              frames, else 4; the split head 5, or 7 above
                                              1,500,000 paths with three frames in flight), or 4..7 */
#define DXRPT_OPT_BAKE_CHUNK 25u /* texels per dxrpt_bake_lightmap launch (default 2^21; bounds the
                                    per-texel shadow-slot buffers).  Identical results. */
#define DXRPT_OPT_WAVE_CLOCKS 28u /* 1: with DXRPT_OPT_COUNT_TRAVERSAL, the megakernel census frame also
                                     records each wave's start and end time (s_memrealtime, 100 MHz),
                                     read with dxrpt_get_wave_clocks (diagnostic: where a frame's tail
                                     comes from); without it, a cost-ordered frame (DXRPT_OPT_WAVE_ORDER)
                                     records each wave slot's stamps.  Images identical. */
#define DXRPT_OPT_WAVE_ORDER 29u     /* 1: megakernel frames start their costliest waves first -- each
                                     wave's duration class is recorded every frame and a small pass
                                     orders the next frame's waves by it (progressive frames cost alike),
                                     so the frame does not end on long waves started last.  The order
                                     resets when the frame's tiles or path count change.  0: waves in
                                     path order.  2 (default): 1 for frames of at most 3 rounds of
                                     resident waves (1.5 with overlapped frames; a GPU's share of a
                                     multi-GPU frame), else 0.  Images identical in every mode. */
#define DXRPT_OPT_XCD_CHUNK 31u      /* path-ordered megakernel frames: each XCD (its own L2) takes runs of
                                        this many consecutive 8x8 pixel blocks, runs dealt to the 8 XCDs
                                        in rotation (default 8; 0: block i on workgroup i, i.e.
                                        neighbouring blocks on different XCDs).  Identical results. */
#define DXRPT_OPT_WAVE_ORDER_PERIOD 32u /* cost-ordered frames: every this-many-th frame records its waves'
                                           durations and rebuilds the order, the frames between reuse it
                                           (default 256, sixteen SqrtNumSamples^2 = 16 cycles of
                                           progressive frames, ~60 ms of a GPU's 1/8 band share; 1 = every
                                           frame).  Identical results. */
#define DXRPT_OPT_MEGAKERNEL_SPLIT 33u /* 1: megakernel frames run as one kernel per path depth -- a head
                                          kernel runs raygen and depth 1 of every camera path, then per
                                          further depth one kernel runs the surviving paths, compacted into
                                          full waves (wave64 ballot, one atomic per wave), with the path
                                          state in the queue instead of registers and its own register
                                          budget.  0: the single k_path.  2 (default): by frame size --
                                          frames of >= 2M path vertices (paths x (L-1)) with overlapped
                                          frames, >= 8M without.  Identical results. */
#define DXRPT_OPT_TAIL_OCCUPANCY 34u   /* register budget of the split schedule's tail kernels in waves/SIMD:
                                          0 = 7 (or DXRPT_OPT_MEGAKERNEL_OCCUPANCY when set), 4..7 */
#define DXRPT_OPT_OPACITY_MICROMAP 36u /* 1 (default): candidates on alpha-tested geometry first read a
                                          micromap word of their triangle (built on the host from the
                                          opacity map: per barycentric cell, "every tap here accepts",
                                          "every tap here rejects" or "tap"), and skip the opacity tap of
                                          AnyHitShader (RayTrace.hlsl:485-507) where the cell decides it.
                                          0: always tap.  Identical results. */
#define DXRPT_OPT_FRAME_OVERLAP 37u    /* 3 (default): by frame size -- three frames in flight for
                                          depth-split frames and frames of at most 600k paths (a GPU's band
                                          share), two for larger single-kernel frames; 1: two, 2: three.
                                          Consecutive megakernel frames rotate over internal streams with
                                          their own path buffers and stage their radiance; the caller's
                                          stream blends a frame's stage (RaygenShader's progressive rule,
                                          RayTrace.hlsl:140-148) once it is done, so the next frames' waves
                                          fill the previous frame's drain.  dxrpt_render still returns with
                                          every launch enqueued, and the target is complete when the
                                          caller's stream reaches that point (see "Stream ordering" above).
                                          The streams want hardware queues of their own: a host with more
                                          busy streams than GPU_MAX_HW_QUEUES (4 by default) minus three
                                          should raise it.  0: one frame at a time on the
                                          caller's stream.  Identical results. */
#define DXRPT_OPT_TREELET_PASSES 40u /* BVH8 build: passes of treelet restructuring (Karras & Aila 2013:
                                        every 7-leaf treelet of the binary SBVH re-wired to its SAH-optimal
                                        topology; subtrees holding alpha-tested triangles are left as
                                        built) before the collapse to BVH8, 0..8 (default 1).  Identical
                                        results (the closest hit does not depend on the tree); only node
                                        visits change. */
#define DXRPT_OPT_BVH_THREADS 41u    /* BVH8 build: host threads (0 = default: the host's CPUs, at most 16).
                                        The tree is the same for every count (ABI 4: the spatial-split budget
                                        is shared between subtrees in proportion to their references, so
                                        subtrees build independently). */
#define DXRPT_OPT_PACKED_TAPS 42u    /* Material taps from fewer loads, identical results.  Bit 0: a
                                        material whose normal, metallic and roughness maps are each W x H
                                        or 1 x 1 (normal RGBA8 unorm, the others R8 or RGBA8 unorm) is
                                        shaded from one host-built RGBA8 texture (normal.rg, metallic,
                                        roughness): one bilinear tap instead of three, same texels and
                                        weights.  Bit 1: a 1 x 1 map (albedo, normal, roughness, metallic,
                                        emissive) travels inline in the shading record, so its tap reads
                                        no memory.  Default 3; 0: a tap per map. */
int dxrpt_set_option(dxrpt_ctx* ctx, uint32_t option, uint64_t value);
/* Zeroes the accumulated kernel timings. */
int dxrpt_reset_timing(dxrpt_ctx* ctx);

/* ---- the hot path ----------------------------------------------------------------------------- */
/* One sample per pixel for every pixel of `tiles` (one DispatchRays(W,H,1)), progressively
 * accumulated into `accum` (device float4): accum = lerp(new, accum, s/(s+1)), s = CurrSampleIdx
 * (RayTrace.hlsl:140-148).  rtc->TotalNumPixels must equal W*H.  `stream` is a hipStream_t.
 * `tiles` NULL: the full W x H frame into accum[y*W + x].  Otherwise tile k's pixel (lx, ly) is image pixel
 * (x0 + lx, y0 + ly) accumulated at accum[accum_offset + ly*accum_pitch + lx]; tiles must lie inside
 * the image; zero-area tiles are skipped, and a list without pixels (num_tiles 0, e.g. a rank of an
 * N-GPU partition that holds no band) returns DXRPT_OK and enqueues nothing. */
int dxrpt_render(dxrpt_ctx* ctx,
                 const dxrpt_ray_trace_constants* rtc,
                 const dxrpt_app_settings* settings,
                 const dxrpt_light_constants* lights,
                 float* accum, uint32_t width, uint32_t height,
                 const dxrpt_tile* tiles, uint32_t num_tiles,
                 void* stream);
/* Primary-only AOV (debug plumbing): for every pixel of `tiles` (NULL: the full frame;
 * addressing as dxrpt_render), RaygenShader's primary ray (CMJ set 0 of rtc->CurrSampleIdx), its closest
 * hit (alpha-tested iff MaxAnyHitPathLength >= 1) and the albedo PathTrace takes there
 * (RayTrace.hlsl:180-183): out = (albedo rgb, 1) on a hit, (0, 0, 0, 0) on a miss.  Overwrites `out`
 * (device float4), no accumulation.  Stream-ordered. */
int dxrpt_render_aov(dxrpt_ctx* ctx, const dxrpt_ray_trace_constants* rtc, const dxrpt_app_settings* settings, float* out,
                     uint32_t width, uint32_t height, const dxrpt_tile* tiles, uint32_t num_tiles, void* stream);
/* ---- post-processing (the consumer of the accumulation buffer) --------------------------------
 * PostProcessor::Render (DXRPathTracer/PostProcessor.cpp:43-92, PostProcessing.hlsl): half-res bloom
 * (2x2 gather, 2 x separable 14-tap Gaussian in RGBA16F), exposure 2^Exposure / FP16Scale and the
 * filmic ALU tone map, from `accum` (device float4 W*H, the dxrpt_render target) into `out` (device,
 * W*H float4 or RGBA8 UNORM).  Uses settings->Exposure, BloomExposure, BloomMagnitude, BloomBlurSigma.
 * Needs no scene; scratch buffers are owned by ctx.  Stream-ordered like dxrpt_render. */
#define DXRPT_POST_FLOAT4 0u
#define DXRPT_POST_RGBA8 1u
int dxrpt_post_process(dxrpt_ctx* ctx, const dxrpt_app_settings* settings, const float* accum, uint32_t width,
                       uint32_t height, void* out, uint32_t out_format, void* stream);
/* Synchronises the context's last stream and returns the counters of the last dxrpt_render. */
int dxrpt_get_stats(dxrpt_ctx* ctx, dxrpt_stats* out);
/* Diagnostic (DXRPT_OPT_WAVE_CLOCKS, megakernel frames): the last render's per-slot (start, end)
 * s_memrealtime stamps.  On a census frame (+ DXRPT_OPT_COUNT_TRAVERSAL, always the 64-lane per-path
 * kernel) slot w = paths [64 w, 64 w + 64) in path-slot order; on a cost-ordered frame slot w = the
 * paths [L w, L w + L) with L = the frame's paths per wave (64, or the path-group width).  A render that
 * records no stamps leaves *num_waves = 0.  Copies min(max_waves, slots) pairs into out[2 w],
 * out[2 w + 1] and the slot count into *num_waves. */
int dxrpt_get_wave_clocks(dxrpt_ctx* ctx, uint64_t* out, uint32_t max_waves, uint32_t* num_waves);
/* Diagnostic of kernel builds made with -DDXRPT_DIAG_PHASES=1 (zeros in the shipped build): lane time,
 * in s_memrealtime ticks (100 MHz) summed over every lane, spent in each phase of a camera path since the
 * last call; reads and zeroes the sums (synchronises the device).  Three sets of 8 (ABI 4):
 *   out[0..7]   the single k_path: 0 raygen + depth-1 closest hit, 1 depth-1 shading, 2 depth-1 shadow rays,
 *               3/4/5 the same at depth 2, 6 depths >= 3, 7 accumulation and waiting for the wave's other
 *               lanes after the path ended;
 *   out[8..15]  k_path_head and out[16..23] k_path_tail (all depths): 0 ray setup + closest hit, 1 shading
 *               (path_vertex), 2 continuation push, 3 / 4 / 5 shadow slot 0 / 1 / >= 2, 6 radiance hand-off,
 *               7 waiting for the wave's other lanes. */
#define DXRPT_PHASE_CLOCKS 24
int dxrpt_get_phase_clocks(dxrpt_ctx* ctx, uint64_t out[DXRPT_PHASE_CLOCKS]);

/* Range-check record of kernel builds made with -DDXRPT_DEBUG=1 (`make variant NAME=debug
 * EXTRA=-DDXRPT_DEBUG=1`; the shipped build returns zeros with out[7] = 0).  Every queued path state a
 * depth-split tail reads and every stage entry an overlapped frame's blend reads is checked before use;
 * a failing lane is counted and does nothing else.  Reads and zeroes the record (synchronises the device):
 *   out[0] violations, out[1] the first one's kind (DXRPT_DEBUG_*), out[2] its depth (-1 = the blend),
 *   out[3] its lane index, out[4] the bad value, out[5] its bound, out[6] queue entries checked,
 *   out[7] 1 in a debug build. */
#define DXRPT_DEBUG_WORDS 8
#define DXRPT_DEBUG_QUEUE_POS 1u   /* queue position >= the queue's capacity */
#define DXRPT_DEBUG_TMAX 2u        /* queued TMax neither FP32Max nor (depth-2 queue) the ended mark -1 */
#define DXRPT_DEBUG_ACCUM_INDEX 3u /* accumulation index >= the tile list's extent */
#define DXRPT_DEBUG_PIXEL 4u       /* CMJ pixel index >= width x height */
int dxrpt_get_debug_record(dxrpt_ctx* ctx, uint32_t out[DXRPT_DEBUG_WORDS]);

/* TraceRay on arbitrary rays against the built acceleration structure (the DXR TraceRay call sites
 * RayTrace.hlsl:138,258,305,407,425 without the shading).  `rays` (device) holds num_rays pairs of
 * float4: (origin.xyz, tmin), (direction.xyz, tmax).  `hits` (device) receives one float4 per ray:
 *   closest-hit (flags bit0 = 0): (t, b1, b2, bits(global triangle id)), t = -1 and id = ~0 on miss;
 *   any-hit     (flags bit0 = 1): (+1 occluded / -1 visible, 0, 0, ~0).
 * flags bit1 = run the alpha-test any-hit on non-opaque geometry (i.e. not RAY_FLAG_FORCE_OPAQUE).
 * The global triangle id is GeometryInfo.IdxOffset/3 + PrimitiveIndex(). */
#define DXRPT_TRACE_ANY_HIT 1u
#define DXRPT_TRACE_ALPHA 2u
int dxrpt_trace_rays(dxrpt_ctx* ctx, const float* rays, uint32_t num_rays, uint32_t flags, float* hits,
                     void* stream);

/* SampleCMJ2D (Shaders/Sampling.hlsl:322-331, the sampler of RayTrace.hlsl:85-90) evaluated by the GPU
 * path's own code on num_cases device cases of 4 uint32 (sampleIdx, numSamplesX, numSamplesY, pattern);
 * out (device) receives 2 floats per case.  Pins the kernels' sampler against the reference's vectors. */
int dxrpt_sample_cmj(dxrpt_ctx* ctx, const uint32_t* cases, uint32_t num_cases, float* out, void* stream);

/* The opacity micromap words (DXRPT_OPT_OPACITY_MICROMAP; host only, no context or GPU needed) of
 * num_tris triangles with vertex UVs uvs[6t .. 6t+5] = (u0, v0, u1, v1, u2, v2) on one opacity map given
 * as dxrpt_add_texture takes it (w x h, fmt, row-major texels): words[W t .. W t + W-1], W =
 * DXRPT_OMM_WORDS, hold 2 bits per barycentric cell c at bit 2 (c mod 16) of word c / 16, cells
 * i = floor(S b1), j = floor(S b2) (S = DXRPT_OMM_SPLIT) clamped to i + j <= S-1, numbered row-major by
 * i: 1 = AnyHitShader accepts every hit in the cell, 2 = rejects every hit, 0 = tap.  Exposed so the
 * verdicts can be checked against the oracle's AnyHitShader without a GPU. */
#define DXRPT_OMM_SPLIT 32u
#define DXRPT_OMM_WORDS 33u
int dxrpt_opacity_micromap(const float* uvs, uint32_t num_tris, uint32_t w, uint32_t h, uint32_t fmt, const void* texels,
                           uint32_t* words);

/* ---- multi-GPU frame (no reference counterpart: the reference is single-GPU) -------
 * The frame is split into screen tiles across the GPUs of a node, one process and context per GPU: rank
 * r renders its tiles (dxrpt_render with its tile list; accum_offset/pitch address its compact slab),
 * dxrpt_gather_slabs moves every slab to rank 0 over RCCL (grouped ncclSend / ncclRecv: each xGMI link
 * carries one rank's slab, all at once), and rank 0 scatters the gathered slabs into the W x H frame
 * with dxrpt_unpermute.  CMJ seeds use global pixel indices, so the result is the single-GPU frame. */
#define DXRPT_COMM_ID_BYTES 128
/* An RCCL unique id (ncclGetUniqueId) for dxrpt_comm_create; rank 0 makes it and sends the 128 bytes to
 * the other ranks by any means (MPI, a file, torch.distributed in the Python driver). */
int dxrpt_comm_unique_id(void* id);
/* RCCL communicator of `nranks` ranks on HIP device `hip_device` (ncclCommInitRank; collective: every rank
 * calls it with the same id).  *comm is an ncclComm_t, released with dxrpt_comm_destroy. */
int dxrpt_comm_create(int hip_device, int nranks, int rank, const void* id, void** comm);
int dxrpt_comm_destroy(void* comm);
/* The number of ranks of the RCCL communicator (ncclCommCount) and this process's rank in it
 * (ncclCommUserRank): what the gather runs over, for the multi-GPU bench line. */
int dxrpt_comm_info(void* comm, int* nranks, int* rank);
/* Collective frame-end gather: rank r sends counts[r] float4 pixels of its device `slab`; rank 0 receives
 * all ranks' slabs back to back into its device `gathered` (rank r at sum(counts[0..r-1]) float4s; its
 * own slab is copied on `stream`).  Every rank passes the same counts[nranks]; stream-ordered. */
int dxrpt_gather_slabs(void* comm, const float* slab, const uint64_t* counts, float* gathered, void* stream);
/* Un-permute: the pixels of `tiles` (host array; tile pixel (lx, ly) read at src[accum_offset + ly *
 * accum_pitch + lx], float4 units) written to the row-major width x height device frame `dst` at
 * (x0 + lx, y0 + ly).  For a gathered frame: every rank's tiles with accum_offset += the rank's slab
 * offset in `gathered`.  The tile list is cached on the device while it is unchanged. */
int dxrpt_unpermute(const float* src, const dxrpt_tile* tiles, uint32_t num_tiles, float* dst, uint32_t width,
                    uint32_t height, void* stream);
/* Message of the last failed dxrpt_comm_* / dxrpt_gather_slabs / dxrpt_unpermute call of this thread. */
const char* dxrpt_multi_last_error(void);
/* Releases this thread's dxrpt_unpermute scratch (device tile lists, after their last launch); also done by
 * dxrpt_comm_destroy.  Call it before the HIP runtime shuts down (a scratch still held at thread exit is left
 * to the process teardown). */
int dxrpt_multi_release(void);

/* ---- lightmap baking (the second consumer of PathTrace) ----------------------------------------
 * One progressive bake pass: BakeRayGen (DXRPathTracer/Baking.hlsl:336-465) as dispatched by
 * DXRPathTracer::RenderBakingPass_Progressive (DXRPathTracer.cpp:1895-1991), one thread per texel of
 * a width x height lightmap (all device float4, row-major):
 *   surface_pos    world position, w != 0 inside a UV island (SurfaceMap.hlsl SV_Target0; w = 0 skips)
 *   surface_normal world normal (SV_Target1)
 *   accum          in/out: rgb = sum of the valid samples, w = their count (g_AccumulationBuffer)
 *   lightmap       out: rgb = accum average, w = 1 (g_BakedLightMap); marker colours for bad texels
 * A cosine-hemisphere ray around the normal (CMJ set 0 at the texel index, sample rtc->CurrSampleIdx)
 * is traced as the first ray of a diffuse path (PathTrace with the scene's lights and sky), clamped
 * against the running average (x10 luminance) and accumulated if valid.  rtc->TotalNumPixels must be
 * width*height (DXRPathTracer.cpp:1934-1935).  Clear accum and lightmap to 0 before sample 0.
 * Stream-ordered like dxrpt_render; dxrpt_get_stats afterwards reports the pass (pixels = texels,
 * the radiance/shadow rays its paths traced). */
int dxrpt_bake_lightmap(dxrpt_ctx* ctx, const dxrpt_ray_trace_constants* rtc, const dxrpt_app_settings* settings,
                        const dxrpt_light_constants* lights, const float* surface_pos, const float* surface_normal,
                        float* accum, float* lightmap, uint32_t width, uint32_t height, void* stream);
/* DenoiseCS (DenoiseMedian.hlsl:52-102, FilterRadius 1 as bound by DXRPathTracer.cpp:2106): each
 * texel's clamped 3x3 neighbourhood of `in` (device float4 W*H) sorted by luminance
 * (0.299, 0.587, 0.114) with a stable insertion sort; the 5th (median) rgb, alpha 1, into `out`. */
int dxrpt_denoise_median(dxrpt_ctx* ctx, const float* in, float* out, uint32_t width, uint32_t height, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DXRPT_H_ */
