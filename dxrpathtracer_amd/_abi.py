"""ctypes mirror of include/dxrpt.h and include/dxrpt_host.h.

Struct layouts are the reference's (see the header comments); sizes are asserted at import so a
header edit that is not mirrored here fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")
# libdxrpt.so from another directory (A/B of kernel builds, scripts/ab.sh); the host library
# always comes from LIB_DIR
KERNEL_LIB_DIR = os.environ.get("DXRPT_KERNEL_LIB_DIR") or LIB_DIR

u32 = C.c_uint32
i32 = C.c_int32
f32 = C.c_float

DXRPT_OK = 0
DXRPT_INVALID_INDEX = 0xFFFFFFFF
DXRPT_MAX_SPOT_LIGHTS = 32
DXRPT_MAX_PATH_LENGTH = 8
DXRPT_COMM_ID_BYTES = 128
TEX_RGBA8_UNORM, TEX_RGBA8_SRGB, TEX_R8_UNORM = 0, 1, 2
TRACE_ANY_HIT, TRACE_ALPHA = 1, 2
SCENE_SPONZA, SCENE_SUNTEMPLE, SCENE_BOXTEST, SCENE_WHITEFURNACE, SCENE_STRONGHOLD = 0, 1, 2, 3, 4


class MeshVertex(C.Structure):
    _fields_ = [("Position", f32 * 3), ("Normal", f32 * 3), ("UV", f32 * 2), ("Tangent", f32 * 3),
                ("Bitangent", f32 * 3), ("LightmapUV", f32 * 2)]


class GeometryInfo(C.Structure):
    _fields_ = [("VtxOffset", u32), ("IdxOffset", u32), ("MaterialIdx", u32), ("PadTo16Bytes", u32)]


class Material(C.Structure):
    _fields_ = [("Albedo", u32), ("Normal", u32), ("Roughness", u32), ("Metallic", u32), ("Opacity", u32),
                ("Emissive", u32)]


class SpotLight(C.Structure):
    _fields_ = [("Position", f32 * 3), ("AngularAttenuationX", f32), ("Direction", f32 * 3),
                ("AngularAttenuationY", f32), ("Intensity", f32 * 3), ("Range", f32)]


class LightConstants(C.Structure):
    _fields_ = [("Lights", SpotLight * DXRPT_MAX_SPOT_LIGHTS), ("ShadowMatrices", (f32 * 16) * DXRPT_MAX_SPOT_LIGHTS)]


class RayTraceConstants(C.Structure):
    _fields_ = [("InvViewProjection", f32 * 16), ("SunDirectionWS", f32 * 3), ("CosSunAngularRadius", f32),
                ("SunIrradiance", f32 * 3), ("SinSunAngularRadius", f32), ("SunRenderColor", f32 * 3),
                ("Padding", u32), ("CameraPosWS", f32 * 3), ("CurrSampleIdx", u32), ("TotalNumPixels", u32),
                ("VtxBufferIdx", u32), ("IdxBufferIdx", u32), ("GeometryInfoBufferIdx", u32),
                ("MaterialBufferIdx", u32), ("SkyTextureIdx", u32), ("NumLights", u32)]


class AppSettings(C.Structure):
    _fields_ = [("EnableSun", u32), ("EnableSky", u32), ("SunAreaLightApproximation", u32), ("SunSize", f32),
                ("SunDirection", f32 * 3), ("MSAAMode", i32), ("RenderLights", u32), ("EnableRayTracing", u32),
                ("ClampRoughness", u32), ("AvoidCausticPaths", u32), ("SqrtNumSamples", i32),
                ("MaxPathLength", i32), ("MaxAnyHitPathLength", i32), ("Exposure", f32), ("BloomExposure", f32),
                ("BloomMagnitude", f32), ("BloomBlurSigma", f32), ("EnableAlbedoMaps", u32),
                ("EnableNormalMaps", u32), ("EnableDiffuse", u32), ("EnableSpecular", u32), ("EnableDirect", u32),
                ("EnableIndirect", u32), ("EnableIndirectSpecular", u32),
                ("ApplyMultiscatteringEnergyCompensation", u32), ("RoughnessScale", f32), ("MetallicScale", f32),
                ("EnableWhiteFurnaceMode", u32), ("EnableLightMapRender", u32)]


class Tile(C.Structure):
    _fields_ = [("x0", u32), ("y0", u32), ("w", u32), ("h", u32), ("accum_offset", C.c_uint64),
                ("accum_pitch", u32), ("pad", u32)]


K_RAYGEN, K_TRACE, K_SHADE, K_SHADOW, K_ACCUMULATE, K_RESOLVE, K_PATH, K_PATH_HEAD, K_PATH_TAIL, K_COUNT = range(10)
KERNEL_NAMES = ("k_raygen", "k_trace", "k_shade", "k_shadow", "k_accumulate", "k_resolve", "k_path", "k_path_head",
                "k_path_tail")
ABI_VERSION = 4
# dxrpt_set_option ids (include/dxrpt.h); the ids missing here were retired in ABI 3 (DXRPT_E_UNSUPPORTED)
OPT_COUNT_TRAVERSAL = 1
OPT_KERNEL_TIMING = 2
OPT_SPATIAL_SPLITS = 12
OPT_LEAF_COST = 13
OPT_PACKET_TRAVERSAL = 18
OPT_KERNEL_TIMING_MASK = 20
OPT_MEGAKERNEL_PATHS = 23
OPT_MEGAKERNEL_OCCUPANCY = 24
OPT_BAKE_CHUNK = 25
OPT_WAVE_CLOCKS = 28
OPT_WAVE_ORDER = 29
OPT_XCD_CHUNK = 31
OPT_WAVE_ORDER_PERIOD = 32
OPT_MEGAKERNEL_SPLIT = 33
OPT_TAIL_OCCUPANCY = 34
OPT_OPACITY_MICROMAP = 36
OPT_FRAME_OVERLAP = 37
OPT_TREELET_PASSES = 40
OPT_BVH_THREADS = 41
OPT_PACKED_TAPS = 42
# include/dxrpt.h DXRPT_RETIRED_OPTIONS (tests/test_abi.py checks the two lists agree)
RETIRED_OPTIONS = (3, 4, 5, 6, 7, 8, 9, 10, 11, 14, 15, 16, 17, 19, 21, 22, 26, 27, 30, 35, 38, 39)
DXRPT_E_INVALID_ARG, DXRPT_E_HIP, DXRPT_E_NO_DEVICE, DXRPT_E_STATE, DXRPT_E_OOM = -1, -2, -3, -4, -5
DXRPT_E_UNSUPPORTED = -6
# context defaults (dxrpt_api.hip)
POST_FLOAT4, POST_RGBA8 = 0, 1  # dxrpt_post_process output formats
DEFAULT_PACKET_TRAVERSAL = 3
DEFAULT_MEGAKERNEL_PATHS = 0xFFFFFFFF
DEFAULT_MEGAKERNEL_OCCUPANCY = 0
DEFAULT_BAKE_CHUNK = 1 << 21
DEFAULT_XCD_CHUNK = 8
DEFAULT_WAVE_ORDER_PERIOD = 256
DEFAULT_OPACITY_MICROMAP = 1
DEFAULT_PACKED_TAPS = 3  # bit 0 packed normal/metallic/roughness maps, bit 1 inlined 1 x 1 maps
DEFAULT_FRAME_OVERLAP = 3
DEFAULT_WAVE_ORDER = 2  # by frame size
DEFAULT_MEGAKERNEL_SPLIT = 2  # by frame size
DEFAULT_TAIL_OCCUPANCY = 0
# opacity micromap (pt_layout.h kOmm*): cells per barycentric axis, verdicts
OMM_SPLIT = 32  # include/dxrpt.h DXRPT_OMM_SPLIT
OMM_WORDS = 33  # DXRPT_OMM_WORDS
OMM_UNKNOWN, OMM_OPAQUE, OMM_TRANSPARENT = 0, 1, 2


class Stats(C.Structure):
    _fields_ = [("pixels", C.c_uint64), ("radiance_rays", C.c_uint64), ("shadow_rays", C.c_uint64),
                ("nominal_rays", C.c_uint64), ("radiance_rays_per_depth", C.c_uint64 * DXRPT_MAX_PATH_LENGTH),
                ("shadow_rays_per_depth", C.c_uint64 * DXRPT_MAX_PATH_LENGTH),
                ("node_visits_radiance", C.c_uint64), ("tri_tests_radiance", C.c_uint64),
                ("node_visits_shadow", C.c_uint64), ("tri_tests_shadow", C.c_uint64),
                ("kernel_ms", C.c_double * K_COUNT), ("kernel_launches", C.c_uint64 * K_COUNT),
                ("timed_frames", C.c_uint64), ("frame_ms", C.c_double), ("schedule", u32), ("paths_per_wave", u32),
                ("occupancy", u32), ("tail_occupancy", u32), ("radiance_hits", C.c_uint64),
                ("census_depth1", C.c_uint64 * 5), ("packed_materials", C.c_uint32), ("packed_textures", C.c_uint32),
                ("inlined_maps", C.c_uint32), ("reserved0", C.c_uint32)]


# dxrpt_stats.schedule bits
SCHED_MEGAKERNEL, SCHED_ORDER_KERNEL, SCHED_COST_ORDERED, SCHED_CENSUS, SCHED_SPLIT, SCHED_OVERLAP = 1, 4, 8, 16, 32, 128


class BvhInfo(C.Structure):
    _fields_ = [("num_nodes", u32), ("num_leaves", u32), ("num_tris", u32), ("max_depth", u32),
                ("node_bytes", u32), ("tri_bytes", u32), ("width", u32), ("num_refs", u32), ("build_ms", C.c_double),
                ("sah_cost", C.c_double), ("phase_ms", C.c_double * 4), ("wide_sah", C.c_double),
                ("binary_depth_cap", u32), ("treelet_passes", u32), ("threads", u32), ("ref_budget_pct", u32)]


BVH_PHASES = ("sbvh", "treelet", "collapse", "records_upload")  # dxrpt_bvh_info.phase_ms
PHASE_CLOCKS = 24  # dxrpt_get_phase_clocks: [0:8] k_path, [8:16] k_path_head, [16:24] k_path_tail
DEBUG_WORDS = 8  # dxrpt_get_debug_record (DXRPT_DEBUG builds)
DEBUG_QUEUE_POS, DEBUG_TMAX, DEBUG_ACCUM_INDEX, DEBUG_PIXEL = 1, 2, 3, 4


class HostTexture(C.Structure):
    _fields_ = [("width", u32), ("height", u32), ("fmt", u32), ("pad", u32), ("texels", C.c_void_p)]


class ModelLoadSettings(C.Structure):
    _fields_ = [("file_path", C.c_char_p), ("texture_dir", C.c_char_p), ("scene_scale", f32), ("force_srgb", u32),
                ("merge_meshes", u32)]


class HostScene(C.Structure):
    _fields_ = [("vertices", C.POINTER(MeshVertex)), ("num_vertices", u32), ("idx_bytes", u32),
                ("indices", C.c_void_p), ("num_indices", u32), ("num_geometries", u32),
                ("geometries", C.POINTER(GeometryInfo)), ("materials", C.POINTER(Material)),
                ("num_materials", u32), ("num_textures", u32), ("textures", C.POINTER(HostTexture)),
                ("spot_lights", C.POINTER(SpotLight)), ("num_spot_lights", u32), ("scene_id", u32),
                ("camera_position", f32 * 3), ("camera_rotation", f32 * 2), ("sun_direction", f32 * 3),
                ("white_furnace", u32), ("seed", C.c_uint64), ("num_triangles", C.c_uint64),
                ("internal", C.c_void_p)]


for _t, _n in ((MeshVertex, 64), (GeometryInfo, 16), (Material, 24), (SpotLight, 48), (LightConstants, 3584),
               (RayTraceConstants, 156), (AppSettings, 124), (Tile, 32)):
    assert C.sizeof(_t) == _n, f"{_t.__name__} is {C.sizeof(_t)} B, expected {_n}"

# Every symbol include/dxrpt.h declares (checked by tests/test_abi.py).
DXRPT_SYMBOLS = ("dxrpt_abi_version", "dxrpt_default_settings", "dxrpt_create", "dxrpt_destroy", "dxrpt_last_error",
                 "dxrpt_set_scene", "dxrpt_add_texture", "dxrpt_set_sky", "dxrpt_build_bvh", "dxrpt_get_bvh_info",
                 "dxrpt_render", "dxrpt_get_stats", "dxrpt_trace_rays", "dxrpt_set_option", "dxrpt_reset_timing",
                 "dxrpt_post_process", "dxrpt_bake_lightmap", "dxrpt_denoise_median", "dxrpt_get_wave_clocks",
                 "dxrpt_get_phase_clocks", "dxrpt_get_debug_record", "dxrpt_sample_cmj", "dxrpt_render_aov", "dxrpt_comm_unique_id", "dxrpt_comm_create",
                 "dxrpt_comm_destroy", "dxrpt_comm_info", "dxrpt_gather_slabs", "dxrpt_unpermute", "dxrpt_multi_last_error",
                 "dxrpt_multi_release", "dxrpt_opacity_micromap")
DXRPT_HOST_SYMBOLS = ("dxrpt_host_scene_create", "dxrpt_host_scene_load", "dxrpt_host_scene_destroy", "dxrpt_host_last_error",
                      "dxrpt_host_inv_view_projection", "dxrpt_host_sky_create", "dxrpt_host_fill_constants",
                      "dxrpt_host_float_to_half", "dxrpt_host_half_to_float", "dxrpt_host_hosek_load",
                      "dxrpt_host_hosek_load_tables", "dxrpt_host_texture_load", "dxrpt_host_texture_free",
                      "dxrpt_host_set_asset_dir",
                      "dxrpt_host_hosek_destroy", "dxrpt_host_hosek_last_error", "dxrpt_host_sky_create_hosek",
                      "dxrpt_host_hosek_rgb_radiance", "dxrpt_host_hosek_solar_radiance", "dxrpt_host_spectrum_to_rgb",
                      "dxrpt_host_spectrum_from_rgb_reflectance", "dxrpt_host_lightmap_charts",
                      "dxrpt_host_surface_map")

_lib = None
_host = None


def _load(name: str, where: str = LIB_DIR) -> C.CDLL:
    path = os.path.join(where, name)
    if not os.path.exists(path):
        raise ImportError(f"{path} is missing: build it with `make -C dxrpathtracer_amd/csrc` "
                          f"(or __graft_entry__.build()); there is no fallback implementation")
    return C.CDLL(path)


def lib() -> C.CDLL:
    """libdxrpt.so: the HIP path tracer (fails loudly if not built)."""
    global _lib
    if _lib is None:
        L = _load("libdxrpt.so", KERNEL_LIB_DIR)
        P = C.c_void_p
        L.dxrpt_abi_version.restype = C.c_int
        L.dxrpt_default_settings.argtypes = [C.POINTER(AppSettings)]
        L.dxrpt_default_settings.restype = None
        L.dxrpt_create.argtypes = [C.c_int, C.POINTER(P)]
        L.dxrpt_destroy.argtypes = [P]
        L.dxrpt_last_error.argtypes = [P]
        L.dxrpt_last_error.restype = C.c_char_p
        L.dxrpt_set_scene.argtypes = [P, C.POINTER(MeshVertex), u32, P, u32, u32, C.POINTER(GeometryInfo), u32,
                                      C.POINTER(Material), u32]
        L.dxrpt_add_texture.argtypes = [P, u32, u32, u32, P, C.POINTER(u32)]
        L.dxrpt_set_sky.argtypes = [P, P, u32]
        L.dxrpt_build_bvh.argtypes = [P]
        L.dxrpt_get_bvh_info.argtypes = [P, C.POINTER(BvhInfo)]
        L.dxrpt_render.argtypes = [P, C.POINTER(RayTraceConstants), C.POINTER(AppSettings),
                                   C.POINTER(LightConstants), P, u32, u32, C.POINTER(Tile), u32, P]
        L.dxrpt_get_stats.argtypes = [P, C.POINTER(Stats)]
        L.dxrpt_get_wave_clocks.argtypes = [P, C.POINTER(C.c_uint64), C.c_uint32, C.POINTER(C.c_uint32)]
        L.dxrpt_get_phase_clocks.argtypes = [P, C.POINTER(C.c_uint64)]
        L.dxrpt_get_debug_record.argtypes = [P, C.POINTER(u32)]
        L.dxrpt_trace_rays.argtypes = [P, P, u32, u32, P, P]
        L.dxrpt_post_process.argtypes = [P, C.POINTER(AppSettings), P, u32, u32, P, u32, P]
        L.dxrpt_set_option.argtypes = [P, u32, C.c_uint64]
        L.dxrpt_bake_lightmap.argtypes = [P, C.POINTER(RayTraceConstants), C.POINTER(AppSettings),
                                          C.POINTER(LightConstants), P, P, P, P, u32, u32, P]
        L.dxrpt_denoise_median.argtypes = [P, P, P, u32, u32, P]
        L.dxrpt_reset_timing.argtypes = [P]
        L.dxrpt_sample_cmj.argtypes = [P, P, u32, P, P]
        L.dxrpt_render_aov.argtypes = [P, C.POINTER(RayTraceConstants), C.POINTER(AppSettings), P, u32, u32,
                                       C.POINTER(Tile), u32, P]
        L.dxrpt_comm_unique_id.argtypes = [P]
        L.dxrpt_comm_create.argtypes = [C.c_int, C.c_int, C.c_int, P, C.POINTER(P)]
        L.dxrpt_comm_destroy.argtypes = [P]
        if hasattr(L, "dxrpt_comm_info"):  # ABI 3 (absent from older builds loaded for A/B runs)
            L.dxrpt_comm_info.argtypes = [P, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.dxrpt_gather_slabs.argtypes = [P, P, C.POINTER(C.c_uint64), P, P]
        L.dxrpt_unpermute.argtypes = [P, C.POINTER(Tile), u32, P, u32, u32, P]
        L.dxrpt_multi_last_error.restype = C.c_char_p
        if hasattr(L, "dxrpt_multi_release"):  # ABI 4
            L.dxrpt_multi_release.argtypes = []
        L.dxrpt_opacity_micromap.argtypes = [P, u32, u32, u32, u32, P, P]
        _lib = L
    return _lib


def host() -> C.CDLL:
    """libdxrpt_host.so: scene/camera/sky inputs (host only)."""
    global _host
    if _host is None:
        H = _load("libdxrpt_host.so")
        P = C.c_void_p
        H.dxrpt_host_scene_create.argtypes = [u32, C.c_uint64, u32, C.POINTER(C.POINTER(HostScene))]
        H.dxrpt_host_scene_load.argtypes = [u32, C.POINTER(ModelLoadSettings), C.POINTER(C.POINTER(HostScene))]
        H.dxrpt_host_scene_destroy.argtypes = [C.POINTER(HostScene)]
        H.dxrpt_host_scene_destroy.restype = None
        H.dxrpt_host_last_error.restype = C.c_char_p
        H.dxrpt_host_inv_view_projection.argtypes = [C.POINTER(f32), f32, f32, f32, f32, f32, f32, C.POINTER(f32)]
        H.dxrpt_host_inv_view_projection.restype = None
        H.dxrpt_host_sky_create.argtypes = [C.POINTER(f32), f32, f32, C.POINTER(f32), u32, P, C.POINTER(f32),
                                            C.POINTER(f32)]
        H.dxrpt_host_fill_constants.argtypes = [C.POINTER(f32), C.POINTER(f32), C.POINTER(AppSettings),
                                                C.POINTER(f32), C.POINTER(f32), u32, u32, u32, u32,
                                                C.POINTER(RayTraceConstants)]
        H.dxrpt_host_fill_constants.restype = None
        H.dxrpt_host_float_to_half.argtypes = [f32]
        H.dxrpt_host_float_to_half.restype = C.c_uint16
        H.dxrpt_host_half_to_float.argtypes = [C.c_uint16]
        H.dxrpt_host_half_to_float.restype = f32
        H.dxrpt_host_hosek_load.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(P)]
        H.dxrpt_host_hosek_load_tables.argtypes = [C.c_char_p, C.POINTER(P)]
        H.dxrpt_host_texture_load.argtypes = [C.c_char_p, u32, C.POINTER(HostTexture)]
        H.dxrpt_host_texture_free.argtypes = [C.POINTER(HostTexture)]
        H.dxrpt_host_texture_free.restype = None
        H.dxrpt_host_set_asset_dir.argtypes = [C.c_char_p]
        H.dxrpt_host_hosek_destroy.argtypes = [P]
        H.dxrpt_host_hosek_destroy.restype = None
        H.dxrpt_host_hosek_last_error.restype = C.c_char_p
        H.dxrpt_host_sky_create_hosek.argtypes = [P, C.POINTER(f32), f32, f32, C.POINTER(f32), u32, P, C.POINTER(f32),
                                                  C.POINTER(f32)]
        d = C.c_double
        H.dxrpt_host_hosek_rgb_radiance.argtypes = [P, d, d, d, d, d, C.c_int]
        H.dxrpt_host_hosek_rgb_radiance.restype = d
        H.dxrpt_host_hosek_solar_radiance.argtypes = [P, d, d, d, d, d, d]
        H.dxrpt_host_hosek_solar_radiance.restype = d
        H.dxrpt_host_spectrum_to_rgb.argtypes = [P, C.POINTER(f32), C.POINTER(f32)]
        H.dxrpt_host_spectrum_to_rgb.restype = None
        H.dxrpt_host_spectrum_from_rgb_reflectance.argtypes = [P, C.POINTER(f32), C.POINTER(f32)]
        H.dxrpt_host_spectrum_from_rgb_reflectance.restype = None
        H.dxrpt_host_lightmap_charts.argtypes = [C.POINTER(HostScene), u32, C.POINTER(MeshVertex), P]
        H.dxrpt_host_surface_map.argtypes = [C.POINTER(MeshVertex), u32, P, u32, u32, u32, P, P]
        _host = H
    return _host


def default_settings() -> AppSettings:
    """AppSettings defaults (AppSettings.cpp:95-208), filled by libdxrpt_host-free Python so the
    CPU tests need no GPU library; must equal dxrpt_default_settings (tests/test_abi.py)."""
    s = AppSettings()
    s.EnableSun = 1
    s.EnableSky = 1
    s.SunAreaLightApproximation = 1
    s.SunSize = 1.0
    s.SunDirection[:] = (0.26, 0.987, -0.16)
    s.MSAAMode = 2
    s.RenderLights = 1
    s.EnableRayTracing = 1
    s.ClampRoughness = 0
    s.AvoidCausticPaths = 0
    s.SqrtNumSamples = 4
    s.MaxPathLength = 3
    s.MaxAnyHitPathLength = 1
    s.Exposure = -14.0
    s.BloomExposure = -4.0
    s.BloomMagnitude = 1.0
    s.BloomBlurSigma = 2.5
    s.EnableAlbedoMaps = 1
    s.EnableNormalMaps = 1
    s.EnableDiffuse = 1
    s.EnableSpecular = 1
    s.EnableDirect = 1
    s.EnableIndirect = 1
    s.EnableIndirectSpecular = 0
    s.ApplyMultiscatteringEnergyCompensation = 1
    s.RoughnessScale = 1.0
    s.MetallicScale = 1.0
    s.EnableWhiteFurnaceMode = 0
    s.EnableLightMapRender = 1
    return s
