"""Host scene inputs: wraps libdxrpt_host.so (scenes, camera, sky) with numpy views.

Reference roles: Model::GenerateBoxTestScene / CreateWithAssimp (Graphics/Model.cpp:435-780), the
per-scene camera/sun tables (DXRPathTracer.cpp:83-98), FirstPersonCamera (Graphics/Camera.cpp:202-229)
and SkyCache::Init (Graphics/Skybox.cpp:48-215).
"""
from __future__ import annotations

import ctypes as C
import math
import os
from dataclasses import dataclass

import numpy as np

from . import _abi as A

SPONZA_SEED = 0x53504F4E5A41  # "SPONZA" 
SCENE_NAMES = {"sponza": A.SCENE_SPONZA, "suntemple": A.SCENE_SUNTEMPLE, "boxtest": A.SCENE_BOXTEST,
               "whitefurnace": A.SCENE_WHITEFURNACE, "stronghold": A.SCENE_STRONGHOLD}
# The reference's asset table (DXRPathTracer.cpp:83-95): model path (relative to the reference checkout's
# Content/Models), texture dir (relative to the model), scene scale.  Sponza / SunTemple are absent from
# the snapshot (procedural proxies); Stronghold is theInn.fbx.
SCENE_ASSETS = {
    A.SCENE_SPONZA: ("Sponza/Sponza_NoSpotLight.fbx", None, 0.01),
    A.SCENE_SUNTEMPLE: ("SunTemple/SunTemple.fbx", "Textures", 0.005),
    A.SCENE_WHITEFURNACE: ("WhiteFurnace/WhiteFurnace.fbx", None, 1.0),
    A.SCENE_STRONGHOLD: ("theInn/source/theInn.fbx", "../textures", 0.1),
}

# DXRPathTracer.cpp:265 camera.Initialize(aspect, Pi_4, 0.1f, 100.0f)
CAMERA_FOV = math.pi / 4
CAMERA_NEAR = 0.1
CAMERA_FAR = 100.0
# AppSettings.cpp:104-113 sky defaults
DEFAULT_TURBIDITY = 2.0
DEFAULT_GROUND_ALBEDO = (0.25, 0.25, 0.25)
SKY_RES = 128  # Skybox.cpp:164


DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def _host():
    """libdxrpt_host.so with the packaged asset directory set (the SunTemple proxy's opacity maps)."""
    H = A.host()
    if not getattr(H, "_asset_dir_set", False):
        H.dxrpt_host_set_asset_dir(DATA_DIR.encode())
        H._asset_dir_set = True
    return H


class Scene:
    """A host scene (vertices, indices, geometries, materials, textures, lights + camera/sun pose)."""

    def __init__(self, scene: str | int = "boxtest", seed: int = SPONZA_SEED, detail: int = 0, model_path: str | None = None,
                 texture_dir: str | None = None, scene_scale: float | None = None):
        """A built-in scene (proxy / BoxTest), or with `model_path` a model file loaded like
        Model::CreateWithAssimp (dxrpt_host_scene_load; texture_dir and scene_scale default to the
        reference's table for the scene id)."""
        sid = SCENE_NAMES[scene] if isinstance(scene, str) else int(scene)
        H = _host()
        p = C.POINTER(A.HostScene)()
        if model_path is None:
            rc = H.dxrpt_host_scene_create(sid, seed, detail, C.byref(p))
            what = f"dxrpt_host_scene_create({sid})"
        else:
            _, tdir, scale = SCENE_ASSETS.get(sid, (None, None, 1.0))
            st = A.ModelLoadSettings(model_path.encode(), (texture_dir if texture_dir is not None else tdir or "").encode(),
                                     scale if scene_scale is None else scene_scale, 1, 0)
            rc = H.dxrpt_host_scene_load(sid, C.byref(st), C.byref(p))
            what = f"dxrpt_host_scene_load({model_path})"
        if rc != 0:
            raise RuntimeError(f"{what} failed: {H.dxrpt_host_last_error().decode()}")
        self._p = p
        s = p.contents
        self.scene_id = sid
        self.num_triangles = int(s.num_triangles)
        self.vertices = np.frombuffer((C.c_uint8 * (64 * s.num_vertices)).from_address(C.cast(s.vertices, C.c_void_p).value),
                                      dtype=np.float32).reshape(s.num_vertices, 16)
        idt = np.uint16 if s.idx_bytes == 2 else np.uint32
        self.indices = np.frombuffer((C.c_uint8 * (s.idx_bytes * s.num_indices)).from_address(s.indices), dtype=idt)
        self.geometries = np.frombuffer((C.c_uint8 * (16 * s.num_geometries)).from_address(
            C.cast(s.geometries, C.c_void_p).value), dtype=np.uint32).reshape(s.num_geometries, 4)
        self.materials = np.frombuffer((C.c_uint8 * (24 * s.num_materials)).from_address(
            C.cast(s.materials, C.c_void_p).value), dtype=np.uint32).reshape(s.num_materials, 6)
        self.textures = []
        for i in range(s.num_textures):
            t = s.textures[i]
            nbytes = t.width * t.height * (1 if t.fmt == A.TEX_R8_UNORM else 4)
            data = np.frombuffer((C.c_uint8 * nbytes).from_address(t.texels), dtype=np.uint8)
            self.textures.append((int(t.width), int(t.height), int(t.fmt), data))
        self.spot_lights = [s.spot_lights[i] for i in range(s.num_spot_lights)]
        self.camera_position = tuple(s.camera_position)
        self.camera_rotation = tuple(s.camera_rotation)
        self.sun_direction = tuple(s.sun_direction)
        self.white_furnace = bool(s.white_furnace)
        self._host = s

    @classmethod
    def from_reference(cls, scene: str | int, reference_root: str | None = None) -> "Scene":
        """The scene's model file from a reference checkout (Content/Models, DXRPathTracer.cpp:83-95)."""
        import os
        sid = SCENE_NAMES[scene] if isinstance(scene, str) else int(scene)
        root = reference_root or os.environ.get("DXRPT_REFERENCE_ROOT", "/root/reference")
        rel = SCENE_ASSETS[sid][0]
        return cls(sid, model_path=os.path.join(root, "Content", "Models", rel))

    def close(self):
        if self._p:
            A.host().dxrpt_host_scene_destroy(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def idx_bytes(self) -> int:
        return int(self._host.idx_bytes)

    def texture_bytes(self) -> int:
        return sum(d.nbytes for _, _, _, d in self.textures)

    # ---- camera + sky ---------------------------------------------------------------------------
    def inv_view_projection(self, width: int, height: int) -> np.ndarray:
        out = (C.c_float * 16)()
        pos = (C.c_float * 3)(*self.camera_position)
        A.host().dxrpt_host_inv_view_projection(pos, self.camera_rotation[0], self.camera_rotation[1], CAMERA_FOV,
                                                width / height, CAMERA_NEAR, CAMERA_FAR, out)
        return np.array(out, dtype=np.float32)

    def settings(self, **overrides) -> A.AppSettings:
        s = A.default_settings()
        s.SunDirection[:] = self.sun_direction          # AppSettings::SunDirection.SetValue (DXRPathTracer.cpp:963)
        s.EnableWhiteFurnaceMode = 1 if self.white_furnace else 0  # DXRPathTracer.cpp:935
        for k, v in overrides.items():
            if k == "SunDirection":
                s.SunDirection[:] = v
            else:
                setattr(s, k, v)
        return s


@dataclass
class Sky:
    cube: np.ndarray          # uint16, 6*res*res*4 (RGBA16F)
    res: int
    sun_irradiance: tuple
    sun_render_color: tuple
    model: str = "analytic"


class HosekData:
    """The Hosek-Wilkie tables.  Default: the packaged table file (dxrpt_host_hosek_load_tables,
    data/hosek_tables.bin, generated by scripts/make_hosek_tables.py).  With `hosek_dir` +
    `spectrum_source`: parsed out of the reference's ArHosekSkyModelData_RGB.h / _Spectral.h and
    Graphics/Spectrum.cpp (dxrpt_host_hosek_load; tests use it to check the packaged file)."""

    def __init__(self, table_file: str | None = None, hosek_dir: str | None = None, spectrum_source: str | None = None):
        H = A.host()
        self._p = C.c_void_p()
        if hosek_dir is not None:
            rc = H.dxrpt_host_hosek_load(hosek_dir.encode(), spectrum_source.encode(), C.byref(self._p))
        else:
            rc = H.dxrpt_host_hosek_load_tables((table_file or HOSEK_TABLES).encode(), C.byref(self._p))
        if rc != 0:
            raise RuntimeError(H.dxrpt_host_hosek_last_error().decode())

    @property
    def handle(self):
        return self._p

    def rgb_radiance(self, turbidity, albedo, elevation, theta, gamma, channel):
        return A.host().dxrpt_host_hosek_rgb_radiance(self._p, turbidity, albedo, elevation, theta, gamma, channel)

    def solar_radiance(self, solar_elevation, turbidity, albedo, theta, gamma, wavelength):
        return A.host().dxrpt_host_hosek_solar_radiance(self._p, solar_elevation, turbidity, albedo, theta, gamma,
                                                        wavelength)

    def spectrum_to_rgb(self, spectrum):
        sp = (C.c_float * 60)(*spectrum)
        out = (C.c_float * 3)()
        A.host().dxrpt_host_spectrum_to_rgb(self._p, sp, out)
        return tuple(out)

    def spectrum_from_rgb(self, rgb):
        out = (C.c_float * 60)()
        A.host().dxrpt_host_spectrum_from_rgb_reflectance(self._p, (C.c_float * 3)(*rgb), out)
        return list(out)

    def __del__(self):
        if getattr(self, "_p", None):
            A.host().dxrpt_host_hosek_destroy(self._p)
            self._p = None


HOSEK_TABLES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "hosek_tables.bin")


def reference_hosek_sources():
    """The reference checkout's dataset sources ($DXRPT_REFERENCE_ROOT, default /root/reference), or None.
    Only tests use them, to check the packaged tables; the product never reads the reference."""
    root = os.path.join(os.environ.get("DXRPT_REFERENCE_ROOT", "/root/reference"), "SampleFramework12", "v1.02")
    hd, sp = os.path.join(root, "HosekSky"), os.path.join(root, "Graphics", "Spectrum.cpp")
    ok = all(os.path.isfile(p) for p in (os.path.join(hd, "ArHosekSkyModelData_RGB.h"),
                                          os.path.join(hd, "ArHosekSkyModelData_Spectral.h"), sp))
    return (hd, sp) if ok else None


_HOSEK = []


def load_hosek() -> HosekData:
    """The process-wide HosekData from the packaged tables (raises if the file is missing)."""
    if not _HOSEK:
        _HOSEK.append(HosekData())
    return _HOSEK[0]


def make_sky(settings: A.AppSettings, turbidity: float = DEFAULT_TURBIDITY,
             ground_albedo=DEFAULT_GROUND_ALBEDO, res: int = SKY_RES, model: str = "hosek") -> Sky:
    """SkyCache::Init.  model: "hosek" (the reference's Hosek-Wilkie sky from the packaged tables, the
    default) or "analytic" (a Preetham proxy, kept for A/B and for turbidity above the solar fit)."""
    cube = np.zeros(6 * res * res * 4, dtype=np.uint16)
    irr = (C.c_float * 3)()
    ren = (C.c_float * 3)()
    sun = (C.c_float * 3)(*settings.SunDirection)
    alb = (C.c_float * 3)(*ground_albedo)
    H = A.host()
    if model == "hosek":
        rc = H.dxrpt_host_sky_create_hosek(load_hosek().handle, sun, settings.SunSize, turbidity, alb, res,
                                           cube.ctypes.data, irr, ren)
        if rc != 0:
            raise RuntimeError(H.dxrpt_host_hosek_last_error().decode())
        return Sky(cube, res, tuple(irr), tuple(ren), "hosek")
    if model != "analytic":
        raise ValueError(f"unknown sky model {model!r}")
    rc = H.dxrpt_host_sky_create(sun, settings.SunSize, turbidity, alb, res, cube.ctypes.data, irr, ren)
    if rc != 0:
        raise RuntimeError("dxrpt_host_sky_create failed")
    return Sky(cube, res, tuple(irr), tuple(ren), "analytic")


def make_constants(scene: Scene, settings: A.AppSettings, sky: Sky, width: int, height: int,
                   sample_idx: int) -> A.RayTraceConstants:
    """RenderRayTracing's constant fill (DXRPathTracer.cpp:2048-2067)."""
    inv = (C.c_float * 16)(*scene.inv_view_projection(width, height))
    pos = (C.c_float * 3)(*scene.camera_position)
    rtc = A.RayTraceConstants()
    nl = min(len(scene.spot_lights), A.DXRPT_MAX_SPOT_LIGHTS)
    A.host().dxrpt_host_fill_constants(inv, pos, C.byref(settings), (C.c_float * 3)(*sky.sun_irradiance),
                                       (C.c_float * 3)(*sky.sun_render_color), sample_idx, width, height, nl,
                                       C.byref(rtc))
    return rtc


def make_lights(scene: Scene) -> A.LightConstants:
    lc = A.LightConstants()
    for i, l in enumerate(scene.spot_lights[:A.DXRPT_MAX_SPOT_LIGHTS]):
        lc.Lights[i] = l
    return lc


def nominal_rays(width: int, height: int, max_path_length: int) -> int:
    """HUD ray count, DXRPathTracer.cpp:2171."""
    return width * height * (1 + (max_path_length - 1) * 2)


# ---- lightmap bake inputs ----------------------------------------------------------------------------
def lightmap_charts(scene: Scene, resolution: int) -> tuple[np.ndarray, np.ndarray]:
    """The lightmapped mesh (dxrpt_host_lightmap_charts; the reference uses xatlas, Model.cpp:608-715):
    (vertices (3T, 16) float32 in the MeshVertex layout with LightmapUV set, indices (3T,) uint32)."""
    n = (int(scene._host.num_indices) // 3) * 3
    verts = np.zeros((n, 16), dtype=np.float32)
    idx = np.zeros(n, dtype=np.uint32)
    rc = A.host().dxrpt_host_lightmap_charts(scene._p, resolution,
                                             verts.ctypes.data_as(C.POINTER(A.MeshVertex)), idx.ctypes.data)
    if rc != 0:
        raise ValueError(f"dxrpt_host_lightmap_charts: {n // 3} charts do not fit a {resolution}^2 lightmap")
    return verts, idx


def surface_map(vertices: np.ndarray, indices: np.ndarray, width: int, height: int) -> tuple[np.ndarray, np.ndarray]:
    """RenderSurfaceMap (dxrpt_host_surface_map): (position (H, W, 4), normal (H, W, 4)) float32."""
    vertices = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 16)
    indices = np.ascontiguousarray(indices, dtype=np.uint32)
    pos = np.empty((height, width, 4), dtype=np.float32)
    nrm = np.empty((height, width, 4), dtype=np.float32)
    rc = A.host().dxrpt_host_surface_map(vertices.ctypes.data_as(C.POINTER(A.MeshVertex)), vertices.shape[0],
                                         indices.ctypes.data, indices.size, width, height, pos.ctypes.data,
                                         nrm.ctypes.data)
    if rc != 0:
        raise ValueError("dxrpt_host_surface_map: bad arguments (index out of range or size)")
    return pos, nrm
