"""ctypes binding of the CPU parity oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg as the checker / CPU baseline, never by the product (dxrpathtracer_amd).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


class OracleStats(C.Structure):
    _fields_ = [("radiance_rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("node_visits", C.c_uint64),
                ("tri_tests", C.c_uint64)]


class OracleTexture(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("fmt", C.c_uint32), ("pad", C.c_uint32),
                ("texels", C.c_void_p)]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        P = C.c_void_p
        L.oracle_cmj2d.argtypes = [C.c_uint32] * 4 + [C.POINTER(C.c_float)]
        L.oracle_cmj2d.restype = None
        L.oracle_sincos.argtypes = [C.c_float, C.POINTER(C.c_float)]
        L.oracle_sincos.restype = None
        L.oracle_scene_create.argtypes = [P, C.c_uint32, P, C.c_uint32, C.c_uint32, P, C.c_uint32, P, C.c_uint32,
                                          P, C.c_uint32, P, C.c_uint32]
        L.oracle_scene_create.restype = P
        L.oracle_scene_destroy.argtypes = [P]
        L.oracle_scene_destroy.restype = None
        L.oracle_scene_build_ms.argtypes = [P]
        L.oracle_scene_build_ms.restype = C.c_double
        L.oracle_render.argtypes = [P, P, P, P] + [C.c_uint32] * 6 + [P, C.c_uint32, C.POINTER(OracleStats)]
        L.oracle_trace_rays.argtypes = [P, P, C.c_uint32, C.c_uint32, P]
        L.oracle_alpha_accepts.argtypes = [P, P, P, C.c_uint32, P]
        L.oracle_render_aov.argtypes = [P, P, P] + [C.c_uint32] * 6 + [P]
        L.oracle_bake.argtypes = [P, P, P, P, P, P] + [C.c_uint32] * 4 + [P, P, C.c_uint32, C.POINTER(OracleStats)]
        L.oracle_median3x3.argtypes = [P, P, C.c_uint32, C.c_uint32]
        L.oracle_median3x3.restype = None
        for fn in ("oracle_concentric_disk", "oracle_cosine_hemisphere", "oracle_ggx_v1", "oracle_fresnel",
                   "oracle_ggx_specular"):
            getattr(L, fn).argtypes = [P, C.c_uint32, P]
            getattr(L, fn).restype = None
        _lib = L
    return _lib


def cmj2d(sample_idx: int, nx: int, ny: int, pattern: int) -> tuple[float, float]:
    out = (C.c_float * 2)()
    lib().oracle_cmj2d(sample_idx, nx, ny, pattern & 0xFFFFFFFF, out)
    return out[0], out[1]


def sincos(x: float) -> tuple[float, float]:
    out = (C.c_float * 2)()
    lib().oracle_sincos(x, out)
    return out[0], out[1]


def _batched(fn: str, pairs, width: int, arity: int = 2):
    import numpy as np
    a = np.ascontiguousarray(pairs, dtype=np.float32).reshape(-1, arity)
    out = np.zeros((a.shape[0], width), dtype=np.float32)
    getattr(lib(), fn)(a.ctypes.data, a.shape[0], out.ctypes.data)
    return out


def concentric_disk(xy):
    """SquareToConcentricDiskMapping (Sampling.hlsl:72-114) on an (n, 2) array -> (n, 2) float32."""
    return _batched("oracle_concentric_disk", xy, 2)


def cosine_hemisphere(uv):
    """SampleDirectionCosineHemisphere (Sampling.hlsl:181-196) on an (n, 2) array -> (n, 3) float32."""
    return _batched("oracle_cosine_hemisphere", uv, 3)


def ggx_v1(m2_ndotx):
    """GGX_V1 (BRDF.hlsl:89-92) on an (n, 2) array of (m2, nDotX) -> (n,) float32."""
    return _batched("oracle_ggx_v1", m2_ndotx, 1)[:, 0]


def fresnel(args):
    """Fresnel (BRDF.hlsl:16-24) on an (n, 9) array of (specAlbedo, h, l) -> (n, 3) float32."""
    return _batched("oracle_fresnel", args, 3, 9)


def ggx_specular(args):
    """GGXSpecular (BRDF.hlsl:128-145) on an (n, 13) array of (m, n, h, v, l) -> (n,) float32."""
    return _batched("oracle_ggx_specular", args, 1, 13)[:, 0]


class OracleScene:
    """The oracle's own copy of a dxrpathtracer_amd.scene.Scene (plus its own BVH)."""

    def __init__(self, scene, sky):
        L = lib()
        self._keep = (scene, sky)
        self._tex = (OracleTexture * max(1, len(scene.textures)))()
        for i, (w, h, fmt, data) in enumerate(scene.textures):
            self._tex[i] = OracleTexture(w, h, fmt, 0, data.ctypes.data)
        self.ptr = L.oracle_scene_create(scene.vertices.ctypes.data, scene.vertices.shape[0], scene.indices.ctypes.data,
                                         scene.idx_bytes, scene.indices.size, scene.geometries.ctypes.data,
                                         scene.geometries.shape[0], scene.materials.ctypes.data,
                                         scene.materials.shape[0], C.cast(self._tex, C.c_void_p),
                                         len(scene.textures), sky.cube.ctypes.data, sky.res)
        self.build_ms = L.oracle_scene_build_ms(self.ptr)

    def close(self):
        if self.ptr:
            lib().oracle_scene_destroy(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def render(self, rtc, settings, lights, width, height, crop=None, accum=None, threads=0):
        """One sample over `crop` = (x0, y0, w, h); returns (accum (h, w, 4) float32, OracleStats)."""
        x0, y0, w, h = crop if crop is not None else (0, 0, width, height)
        if accum is None:
            accum = np.zeros((h, w, 4), dtype=np.float32)
        assert accum.dtype == np.float32 and accum.flags.c_contiguous and accum.shape == (h, w, 4)
        st = OracleStats()
        rc = lib().oracle_render(self.ptr, C.addressof(rtc), C.addressof(settings),
                                 C.addressof(lights) if lights is not None else None, width, height, x0, y0, w, h,
                                 accum.ctypes.data, threads, C.byref(st))
        if rc != 0:
            raise RuntimeError("oracle_render failed")
        return accum, st

    def render_aov(self, rtc, settings, width, height, crop=None):
        """Primary-only AOV over `crop`: (h, w, 4) float32 = (albedo rgb, 1) on a hit, 0 on a miss."""
        x0, y0, w, h = crop if crop is not None else (0, 0, width, height)
        out = np.zeros((h, w, 4), dtype=np.float32)
        rc = lib().oracle_render_aov(self.ptr, C.addressof(rtc), C.addressof(settings), width, height, x0, y0, w, h,
                                     out.ctypes.data)
        if rc != 0:
            raise RuntimeError("oracle_render_aov failed")
        return out

    def trace_rays(self, rays: np.ndarray, flags: int) -> np.ndarray:
        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 8)
        hits = np.zeros((rays.shape[0], 4), dtype=np.float32)
        lib().oracle_trace_rays(self.ptr, rays.ctypes.data, rays.shape[0], flags, hits.ctypes.data)
        return hits

    def alpha_accepts(self, gtri: np.ndarray, bary: np.ndarray) -> np.ndarray:
        """AnyHitShader's verdict (RayTrace.hlsl:485-507) per (global triangle, b1, b2): True = accept."""
        gtri = np.ascontiguousarray(gtri, dtype=np.uint32)
        bary = np.ascontiguousarray(bary, dtype=np.float32).reshape(-1, 2)
        out = np.zeros(gtri.shape[0], dtype=np.uint8)
        if lib().oracle_alpha_accepts(self.ptr, gtri.ctypes.data, bary.ctypes.data, gtri.shape[0], out.ctypes.data) != 0:
            raise ValueError("oracle_alpha_accepts: triangle id out of range")
        return out.astype(bool)

    def bake(self, rtc, settings, lights, pos, nrm, accum, lightmap, first=0, count=None, threads=0):
        """One BakeRayGen pass over texels [first, first + count); updates accum / lightmap (H, W, 4) in place."""
        h, w = pos.shape[:2]
        for a in (pos, nrm, accum, lightmap):
            assert a.dtype == np.float32 and a.flags.c_contiguous and a.shape == (h, w, 4)
        count = w * h - first if count is None else count
        st = OracleStats()
        rc = lib().oracle_bake(self.ptr, C.addressof(rtc), C.addressof(settings),
                               C.addressof(lights) if lights is not None else None, pos.ctypes.data, nrm.ctypes.data,
                               w, h, first, count, accum.ctypes.data, lightmap.ctypes.data, threads, C.byref(st))
        if rc != 0:
            raise RuntimeError("oracle_bake failed")
        return st


def median3x3(img: np.ndarray) -> np.ndarray:
    """DenoiseCS (FilterRadius 1) of an (H, W, 4) float32 image."""
    img = np.ascontiguousarray(img, dtype=np.float32)
    out = np.empty_like(img)
    lib().oracle_median3x3(img.ctypes.data, out.ctypes.data, img.shape[1], img.shape[0])
    return out
