"""DXRPathTracer host driver over the C ABI (libdxrpt.so).

Mirrors the reference's path-tracer-facing methods of class DXRPathTracer (DXRPathTracer.h:32-202):
InitializeScene (DXRPathTracer.cpp:932-985), BuildRTAccelerationStructure (2331-2488), the sample-index
/ restart bookkeeping of Update (1416-1461) and RenderRayTracing (2024-2090).  There is no CPU
fallback: every method goes through the HIP library and raises on a non-zero status.
"""
from __future__ import annotations

import ctypes as C

from . import _abi as A
from .scene import Scene, Sky, make_constants, make_lights


class DxrptError(RuntimeError):
    pass


class DXRPathTracer:
    def __init__(self, device: int = 0):
        self._L = A.lib()
        self._ctx = C.c_void_p()
        rc = self._L.dxrpt_create(device, C.byref(self._ctx))
        if rc != A.DXRPT_OK:
            raise DxrptError(f"dxrpt_create({device}) failed with status {rc}")
        self.rt_curr_sample_idx = 0
        self.rt_should_restart = True
        self.scene: Scene | None = None
        self.sky: Sky | None = None

    def _check(self, rc: int, what: str):
        if rc != A.DXRPT_OK:
            msg = self._L.dxrpt_last_error(self._ctx)
            raise DxrptError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

    def close(self):
        if self._ctx:
            self._L.dxrpt_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- InitializeScene (DXRPathTracer.cpp:932-985) + material/texture tables --------------------
    def initialize_scene(self, scene: Scene, sky: Sky):
        L = self._L
        for (w, h, fmt, data) in scene.textures:
            idx = C.c_uint32()
            self._check(L.dxrpt_add_texture(self._ctx, w, h, fmt, data.ctypes.data, C.byref(idx)), "dxrpt_add_texture")
        s = scene._host
        self._check(L.dxrpt_set_scene(self._ctx, s.vertices, s.num_vertices, s.indices, s.idx_bytes, s.num_indices,
                                      s.geometries, s.num_geometries, s.materials, s.num_materials), "dxrpt_set_scene")
        self.set_sky(sky)
        self.scene = scene
        self.rt_should_restart = True

    def set_sky(self, sky: Sky):
        self._check(self._L.dxrpt_set_sky(self._ctx, sky.cube.ctypes.data, sky.res), "dxrpt_set_sky")
        self.sky = sky

    def build_rt_acceleration_structure(self) -> A.BvhInfo:
        self._check(self._L.dxrpt_build_bvh(self._ctx), "dxrpt_build_bvh")
        return self.bvh_info()

    def bvh_info(self) -> A.BvhInfo:
        info = A.BvhInfo()
        self._check(self._L.dxrpt_get_bvh_info(self._ctx, C.byref(info)), "dxrpt_get_bvh_info")
        return info

    # ---- Update restart logic (DXRPathTracer.cpp:1416-1461) ----------------------------------------
    def restart(self):
        self.rt_should_restart = True

    def update(self):
        if self.rt_should_restart:
            self.rt_curr_sample_idx = 0
            self.rt_should_restart = False

    # ---- RenderRayTracing (DXRPathTracer.cpp:2024-2090) ---------------------------------------------
    def render_ray_tracing(self, accum_ptr: int, width: int, height: int, settings: A.AppSettings,
                           tiles=None, stream: int = 0, sample_idx: int | None = None,
                           lights: A.LightConstants | None = None) -> bool:
        """Enqueues one DispatchRays(W,H,1) equivalent.  Returns False (and does nothing) once the
        sample count reached SqrtNumSamples^2 (DXRPathTracer.cpp:2027-2028)."""
        idx = self.rt_curr_sample_idx if sample_idx is None else sample_idx
        if idx >= settings.SqrtNumSamples * settings.SqrtNumSamples:
            return False
        rtc = make_constants(self.scene, settings, self.sky, width, height, idx)
        self.render_raw(rtc, settings, accum_ptr, width, height, tiles, stream,
                        lights if lights is not None else make_lights(self.scene))
        if sample_idx is None:
            self.rt_curr_sample_idx += 1
        return True

    def render_raw(self, rtc: A.RayTraceConstants, settings: A.AppSettings, accum_ptr: int, width: int,
                   height: int, tiles=None, stream: int = 0, lights: A.LightConstants | None = None):
        tarr, nt = None, 0
        if isinstance(tiles, C.Array):
            # a ctypes Tile array built once by the caller (BandLayout.tile_array: an N-GPU block partition
            # has thousands of tiles, marshalling them every frame would starve the GPU)
            tarr, nt = (tiles if len(tiles) else (A.Tile * 1)()), len(tiles)
        elif tiles is not None:  # a list of Tile / tuples: marshalled on every call, so later edits to it are seen
            tarr = (A.Tile * max(1, len(tiles)))()  # an empty list: a non-null array of 0 tiles (no pixels)
            for i, t in enumerate(tiles):
                tarr[i] = t if isinstance(t, A.Tile) else A.Tile(*t)
            nt = len(tiles)
        lp = C.byref(lights) if lights is not None else None
        self._check(self._L.dxrpt_render(self._ctx, C.byref(rtc), C.byref(settings), lp, C.c_void_p(accum_ptr),
                                         width, height, tarr, nt, C.c_void_p(stream)), "dxrpt_render")

    def render_aov(self, rtc: A.RayTraceConstants, settings: A.AppSettings, out_ptr: int, width: int, height: int,
                   tiles=None, stream: int = 0):
        """Primary-only AOV (dxrpt_render_aov): (albedo rgb, 1) at each pixel's primary hit, 0 on a miss."""
        tarr, nt = None, 0
        if tiles is not None:
            tarr = tiles if isinstance(tiles, C.Array) and len(tiles) else \
                (A.Tile * max(1, len(tiles)))(*[t if isinstance(t, A.Tile) else A.Tile(*t) for t in tiles])
            nt = len(tiles)
        self._check(self._L.dxrpt_render_aov(self._ctx, C.byref(rtc), C.byref(settings), C.c_void_p(out_ptr), width,
                                             height, tarr, nt, C.c_void_p(stream)), "dxrpt_render_aov")

    def set_option(self, option: int, value: int):
        self._check(self._L.dxrpt_set_option(self._ctx, option, value), "dxrpt_set_option")

    def reset_timing(self):
        self._check(self._L.dxrpt_reset_timing(self._ctx), "dxrpt_reset_timing")

    def stats(self) -> A.Stats:
        st = A.Stats()
        self._check(self._L.dxrpt_get_stats(self._ctx, C.byref(st)), "dxrpt_get_stats")
        return st

    def wave_clocks(self):
        """Per-wave (start, end) s_memrealtime stamps (100 MHz ticks) of the last census frame rendered
        with OPT_COUNT_TRAVERSAL + OPT_WAVE_CLOCKS (megakernel), as a (waves, 2) uint64 array."""
        import numpy as np
        n = C.c_uint32()
        self._check(self._L.dxrpt_get_wave_clocks(self._ctx, None, 0, C.byref(n)), "dxrpt_get_wave_clocks")
        out = np.zeros((n.value, 2), dtype=np.uint64)
        if n.value:
            self._check(self._L.dxrpt_get_wave_clocks(self._ctx, out.ctypes.data_as(C.POINTER(C.c_uint64)), n.value,
                                                      C.byref(n)), "dxrpt_get_wave_clocks")
        return out

    def debug_record(self):
        """The range-check record since the last call (kernel builds with -DDXRPT_DEBUG=1; zeros and
        is_debug_build False otherwise), see dxrpt_get_debug_record: a dict of the 8 words."""
        out = (C.c_uint32 * A.DEBUG_WORDS)()
        self._check(self._L.dxrpt_get_debug_record(self._ctx, out), "dxrpt_get_debug_record")
        v = list(out)
        return {"violations": v[0], "kind": v[1], "depth": v[2] - (1 << 32) if v[2] >= 1 << 31 else v[2],
                "lane": v[3], "value": v[4], "bound": v[5], "checked": v[6], "is_debug_build": bool(v[7])}

    def phase_clocks(self):
        """Lane ticks per camera-path phase since the last call (kernel builds with -DDXRPT_DIAG_PHASES=1;
        zeros otherwise), see dxrpt_get_phase_clocks: 24 values, [0:8] k_path, [8:16] k_path_head, [16:24]
        k_path_tail."""
        out = (C.c_uint64 * A.PHASE_CLOCKS)()
        self._check(self._L.dxrpt_get_phase_clocks(self._ctx, out), "dxrpt_get_phase_clocks")
        return [int(v) for v in out]

    def post_process(self, settings: A.AppSettings, accum_ptr: int, width: int, height: int, out_ptr: int,
                     out_format: int = A.POST_FLOAT4, stream: int = 0):
        """PostProcessor::Render (PostProcessor.cpp:43-92): bloom + exposure + filmic tone map of the
        accumulation buffer into `out` (device W*H float4 or RGBA8)."""
        self._check(A.lib().dxrpt_post_process(self._ctx, C.byref(settings), accum_ptr, width, height, out_ptr,
                                               out_format, stream), "dxrpt_post_process")

    def trace_rays(self, rays_ptr: int, n: int, flags: int, hits_ptr: int, stream: int = 0):
        self._check(self._L.dxrpt_trace_rays(self._ctx, C.c_void_p(rays_ptr), n, flags, C.c_void_p(hits_ptr),
                                             C.c_void_p(stream)), "dxrpt_trace_rays")

    # ---- lightmap baking (DXRPathTracer.cpp:1993-2022, 1895-1991, 2092-2125) --------------------------
    def bake_lightmap(self, settings: A.AppSettings, surface_pos_ptr: int, surface_normal_ptr: int, accum_ptr: int,
                      lightmap_ptr: int, width: int, height: int, sample_idx: int, stream: int = 0,
                      lights: A.LightConstants | None = None):
        """RenderBakingPass_Progressive: one BakeRayGen pass (sample `sample_idx`) over a width x height
        lightmap; all pointers are device float4 arrays.  The caller clears accum/lightmap before sample 0
        and advances sample_idx (bakingSampleIndex++, DXRPathTracer.cpp:2020)."""
        rtc = make_constants(self.scene, settings, self.sky, width, height, sample_idx)
        lc = lights if lights is not None else make_lights(self.scene)
        self._check(self._L.dxrpt_bake_lightmap(self._ctx, C.byref(rtc), C.byref(settings), C.byref(lc),
                                                C.c_void_p(surface_pos_ptr), C.c_void_p(surface_normal_ptr),
                                                C.c_void_p(accum_ptr), C.c_void_p(lightmap_ptr), width, height,
                                                C.c_void_p(stream)), "dxrpt_bake_lightmap")

    def denoise_median(self, in_ptr: int, out_ptr: int, width: int, height: int, stream: int = 0):
        """RenderLightmapMedianPass: DenoiseCS (3x3 luminance median) from `in` into `out` (device float4)."""
        self._check(self._L.dxrpt_denoise_median(self._ctx, C.c_void_p(in_ptr), C.c_void_p(out_ptr), width, height,
                                                 C.c_void_p(stream)), "dxrpt_denoise_median")

