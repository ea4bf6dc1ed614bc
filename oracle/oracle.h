/* oracle.h — C interface of the CPU parity oracle (TEST INFRASTRUCTURE ONLY; see oracle.cpp).
 * Structs restate the reference layouts directly (SharedTypes.h, RayTracing.hlsl, AppSettings.h,
 * DXRPathTracer.cpp:145-165); they are byte-compatible with include/dxrpt.h but deliberately do not
 * include it, so the checker does not depend on product headers. */
#ifndef ORACLE_H_
#define ORACLE_H_
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_TEX_RGBA8_UNORM 0u
#define ORACLE_TEX_RGBA8_SRGB 1u
#define ORACLE_TEX_R8_UNORM 2u

typedef struct oracle_vertex { float Position[3], Normal[3], UV[2], Tangent[3], Bitangent[3], LightmapUV[2]; } oracle_vertex;
typedef struct oracle_geometry_info { uint32_t VtxOffset, IdxOffset, MaterialIdx, PadTo16Bytes; } oracle_geometry_info;
typedef struct oracle_material { uint32_t Albedo, Normal, Roughness, Metallic, Opacity, Emissive; } oracle_material;
typedef struct oracle_spot_light {
    float Position[3]; float AngularAttenuationX; float Direction[3]; float AngularAttenuationY; float Intensity[3]; float Range;
} oracle_spot_light;
typedef struct oracle_texture { uint32_t width, height, fmt, pad; const void* texels; } oracle_texture;
typedef struct oracle_ray_trace_constants {
    float InvViewProjection[16];
    float SunDirectionWS[3]; float CosSunAngularRadius;
    float SunIrradiance[3]; float SinSunAngularRadius;
    float SunRenderColor[3]; uint32_t Padding;
    float CameraPosWS[3]; uint32_t CurrSampleIdx;
    uint32_t TotalNumPixels;
    uint32_t VtxBufferIdx, IdxBufferIdx, GeometryInfoBufferIdx, MaterialBufferIdx, SkyTextureIdx, NumLights;
} oracle_ray_trace_constants;
typedef struct oracle_app_settings {
    uint32_t EnableSun, EnableSky, SunAreaLightApproximation; float SunSize; float SunDirection[3]; int32_t MSAAMode;
    uint32_t RenderLights, EnableRayTracing, ClampRoughness, AvoidCausticPaths;
    int32_t SqrtNumSamples, MaxPathLength, MaxAnyHitPathLength;
    float Exposure, BloomExposure, BloomMagnitude, BloomBlurSigma;
    uint32_t EnableAlbedoMaps, EnableNormalMaps, EnableDiffuse, EnableSpecular, EnableDirect, EnableIndirect,
        EnableIndirectSpecular, ApplyMultiscatteringEnergyCompensation;
    float RoughnessScale, MetallicScale;
    uint32_t EnableWhiteFurnaceMode, EnableLightMapRender;
} oracle_app_settings;
typedef struct oracle_stats { uint64_t radiance_rays, shadow_rays, node_visits, tri_tests; } oracle_stats;
typedef struct oracle_scene oracle_scene;

void oracle_cmj2d(uint32_t sample_idx, uint32_t nx, uint32_t ny, uint32_t pattern, float out[2]);
void oracle_sincos(float x, float out[2]);
/* Sampling.hlsl:72-114 SquareToConcentricDiskMapping (out 2 per input), 181-196 SampleDirectionCosineHemisphere
 * (out 3 per input) on n (x, y) pairs; BRDF.hlsl:89-92 GGX_V1 on n (m2, nDotX) pairs (out 1 per input). */
void oracle_concentric_disk(const float* xy, uint32_t n, float* out);
void oracle_cosine_hemisphere(const float* uv, uint32_t n, float* out);
void oracle_ggx_v1(const float* m2_ndotx, uint32_t n, float* out);
void oracle_fresnel(const float* in, uint32_t n, float* out);
void oracle_ggx_specular(const float* in, uint32_t n, float* out);
/* Arrays must outlive the scene (not copied), except indices which are widened into the scene. */
oracle_scene* oracle_scene_create(const oracle_vertex* vertices, uint32_t num_vertices, const void* indices, uint32_t idx_bytes,
                                  uint32_t num_indices, const oracle_geometry_info* geometries, uint32_t num_geometries,
                                  const oracle_material* materials, uint32_t num_materials, const oracle_texture* textures,
                                  uint32_t num_textures, const uint16_t* sky_cube, uint32_t sky_res);
void oracle_scene_destroy(oracle_scene* scene);
double oracle_scene_build_ms(const oracle_scene* scene);
/* Renders one sample for the pixels of the crop [x0,x0+w) x [y0,y0+h) of a width x height image into
 * accum (w*h float4, crop-local row-major), with the progressive lerp of RayTrace.hlsl:143-148. */
int oracle_render(const oracle_scene* scene, const oracle_ray_trace_constants* rtc, const oracle_app_settings* settings,
                  const oracle_spot_light* lights, uint32_t width, uint32_t height, uint32_t x0, uint32_t y0, uint32_t w,
                  uint32_t h, float* accum, uint32_t threads, oracle_stats* out_stats);
/* Primary-only AOV (C1 plumbing) of the crop: per pixel (albedo rgb, 1) at the primary ray's closest hit,
 * (0, 0, 0, 0) on a miss; out is w*h float4, crop-local row-major. */
int oracle_render_aov(const oracle_scene* scene, const oracle_ray_trace_constants* rtc, const oracle_app_settings* settings,
                      uint32_t width, uint32_t height, uint32_t x0, uint32_t y0, uint32_t w, uint32_t h, float* out);
/* One bake pass (Baking.hlsl BakeRayGen) over texels [first, first + count) of a width x height
 * lightmap: pos/nrm/accum/lightmap are W*H float4 (same meaning as dxrpt_bake_lightmap). */
int oracle_bake(const oracle_scene* scene, const oracle_ray_trace_constants* rtc, const oracle_app_settings* settings,
                const oracle_spot_light* lights, const float* pos, const float* nrm, uint32_t width, uint32_t height,
                uint32_t first, uint32_t count, float* accum, float* lightmap, uint32_t threads, oracle_stats* out_stats);
/* DenoiseMedian.hlsl DenoiseCS, FilterRadius 1: in/out W*H float4. */
void oracle_median3x3(const float* in, float* out, uint32_t width, uint32_t height);
/* rays: n x 8 floats (o.xyz, tmin, d.xyz, tmax); hits: n x 4 (same encoding as dxrpt_trace_rays). */
int oracle_trace_rays(const oracle_scene* scene, const float* rays, uint32_t n, uint32_t flags, float* hits);
int oracle_alpha_accepts(const oracle_scene* scene, const uint32_t* gtri, const float* bary, uint32_t n, uint8_t* out);

#ifdef __cplusplus
}
#endif
#endif
