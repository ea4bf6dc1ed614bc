"""CPU: host-side inputs (scenes, camera, sky, fp16) and the screen-space band partition."""
import ctypes as C
import math

import numpy as np
import pytest

import dxrpathtracer_amd as D
import dxrpathtracer_amd._abi as A
from dxrpathtracer_amd.distributed import band_layout, source_index
from tests._common import scene_bundle


def test_boxtest_geometry_is_the_reference_scene():
    # Model::GenerateBoxTestScene (Graphics/Model.cpp:761-780) + InitBox (235-343)
    sc, _ = scene_bundle("boxtest")
    assert sc.vertices.shape == (48, 16) and sc.indices.dtype == np.uint16 and sc.indices.size == 72
    assert sc.geometries.tolist() == [[0, 0, 0, 0], [24, 36, 0, 0]]
    pos = sc.vertices[:, 0:3]
    np.testing.assert_array_equal(pos[:24].min(0), [-1, 0.5, -1])
    np.testing.assert_array_equal(pos[:24].max(0), [1, 2.5, 1])
    np.testing.assert_array_equal(pos[24:].min(0), [-5, -0.125, -5])
    np.testing.assert_array_equal(pos[24:].max(0), [5, 0.125, 5])
    np.testing.assert_array_equal(sc.indices[:6], [0, 1, 2, 2, 3, 0])
    np.testing.assert_array_equal(sc.indices[36:42], [0, 1, 2, 2, 3, 0])  # mesh-local
    # top face: N=(0,1,0), T=(1,0,0), B=(0,0,-1); uv(0,0) at (-1,1,1)
    np.testing.assert_array_equal(sc.vertices[0], [-1, 2.5, 1, 0, 1, 0, 0, 0, 1, 0, 0, 0, 0, -1, 0, 0])
    assert sc.camera_position == (0.0, 2.5, -10.0)
    assert sc.num_triangles == 24


def test_scene_tables():
    # DXRPathTracer.cpp:96-98
    sp, _ = scene_bundle("sponza")
    assert sp.camera_position == pytest.approx((-11.5, 1.85, -0.45))
    assert sp.camera_rotation == pytest.approx((0.0, 1.544))
    assert sp.sun_direction == pytest.approx((0.26, 0.987, -0.16))
    st, _ = scene_bundle("suntemple")
    assert st.sun_direction == pytest.approx((-0.133022308, 0.642787635, 0.75440651))
    wf, _ = scene_bundle("whitefurnace")
    assert wf.white_furnace and wf.settings().EnableWhiteFurnaceMode == 1


def test_sponza_proxy_size_and_determinism():
    sp, _ = scene_bundle("sponza")
    assert 230_000 <= sp.num_triangles <= 300_000, sp.num_triangles  # ~Crytek Sponza scale
    assert 15 <= sp.materials.shape[0] <= 30
    assert any(m[4] != A.DXRPT_INVALID_INDEX for m in sp.materials)  # alpha-tested leaves
    assert len(sp.spot_lights) == 0  # Sponza_NoSpotLight.fbx (DXRPathTracer.cpp:86)
    again = D.Scene("sponza")
    np.testing.assert_array_equal(again.vertices, sp.vertices)
    np.testing.assert_array_equal(again.indices, sp.indices)
    other = D.Scene("sponza", seed=7)
    assert not np.array_equal(other.vertices, sp.vertices) or not all(
        np.array_equal(a[3], b[3]) for a, b in zip(other.textures, sp.textures))
    # every geometry's indices stay inside its vertex range
    g = sp.geometries
    ends = list(g[1:, 1]) + [sp.indices.size]
    vend = list(g[1:, 0]) + [sp.vertices.shape[0]]
    for k in range(g.shape[0]):
        ii = sp.indices[g[k, 1]:ends[k]]
        assert ii.max() + g[k, 0] < vend[k]


def test_suntemple_proxy_has_alpha_foliage():
    st, _ = scene_bundle("suntemple")
    opaque = [m[4] == A.DXRPT_INVALID_INDEX for m in st.materials]
    assert not all(opaque)
    assert st.num_triangles > 100_000


def test_half_conversion_is_round_to_nearest_even():
    H = A.host()
    rng = np.random.default_rng(0)
    xs = np.concatenate([rng.standard_normal(20000).astype(np.float32) * 1e3,
                         rng.standard_normal(5000).astype(np.float32) * 1e-5,
                         np.array([0.0, -0.0, 65504.0, 65520.0, 1e9, 6.1e-5, 5.96e-8, np.inf, -np.inf], np.float32)])
    for x in xs:
        assert H.dxrpt_host_float_to_half(float(x)) == int(np.float16(x).view(np.uint16)), x
    for h in range(0, 65536, 7):
        if (h & 0x7C00) == 0x7C00 and (h & 0x3FF):
            continue  # NaN payloads
        assert H.dxrpt_host_half_to_float(h) == float(np.uint16(h).view(np.float16)), h


def test_camera_unprojects_the_view_axis():
    sc, _ = scene_bundle("sponza")
    M = sc.inv_view_projection(1920, 1080).reshape(4, 4).astype(np.float64)
    near = np.array([0, 0, 0, 1.0]) @ M
    far = np.array([0, 0, 1, 1.0]) @ M
    near, far = near[:3] / near[3], far[:3] / far[3]
    d = (far - near) / np.linalg.norm(far - near)
    yaw = 1.544  # forward = (sin yaw, 0, cos yaw) for pitch 0 (XMQuaternionRotationRollPitchYaw)
    np.testing.assert_allclose(d, [math.sin(yaw), 0, math.cos(yaw)], atol=1e-5)
    np.testing.assert_allclose(near, np.array(sc.camera_position) + 0.1 * d, atol=1e-4)
    np.testing.assert_allclose(np.linalg.norm(far - near), 100 - 0.1, rtol=1e-4)


def test_sky_cube_layout_and_sun():
    sc, sky = scene_bundle("sponza")
    assert sky.cube.size == 6 * 128 * 128 * 4
    px = sky.cube.view(np.float16).astype(np.float32).reshape(6, 128, 128, 4)
    assert np.all(px[..., 3] == 1.0)
    assert np.isfinite(px).all() and (px[..., :3] >= 0).all()
    # +y face (zenith) is brighter than -y face (clamped at the horizon)
    assert px[2, ..., :3].mean() > 0
    assert sky.sun_irradiance[0] > 10 and sky.sun_render_color[0] <= 65000
    st = sc.settings()
    rtc = D.make_constants(sc, st, sky, 64, 32, 3)
    assert rtc.TotalNumPixels == 64 * 32 and rtc.CurrSampleIdx == 3
    assert math.isclose(rtc.CosSunAngularRadius, math.cos(math.radians(1.0)), rel_tol=1e-7)
    n = math.sqrt(0.26 ** 2 + 0.987 ** 2 + 0.16 ** 2)
    assert rtc.SunDirectionWS[1] == pytest.approx(0.987 / n)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_band_layout_covers_every_pixel_once(world):
    W, H = 37, 1080
    lay = band_layout(W, H, world)
    assert sum(lay.counts) == W * H
    idx = source_index(lay)
    assert len(idx) == W * H and len(set(idx)) == W * H
    assert max(idx) < world * lay.max_count
    for r in range(world):
        owned = sum(t.w * t.h for t in lay.tiles[r])
        assert owned == lay.counts[r]


def test_asset_dir_defaults_next_to_the_library():
    # a C caller that never calls dxrpt_host_set_asset_dir still finds the packaged SunTemple opacity
    # maps (../data next to libdxrpt_host.so); a missing asset is an argument/IO error, not "out of memory"
    import subprocess
    import sys
    code = r"""
import ctypes as C, os, sys
lib = C.CDLL(os.path.join(sys.argv[1], "libdxrpt_host.so"))
lib.dxrpt_host_last_error.restype = C.c_char_p
out = C.c_void_p()
rc = lib.dxrpt_host_scene_create(1, C.c_uint64(0), 1, C.byref(out))   # DXRPT_SCENE_SUNTEMPLE, small detail
assert rc == 0, (rc, lib.dxrpt_host_last_error())
lib.dxrpt_host_scene_destroy(out)
assert lib.dxrpt_host_set_asset_dir(b"/nonexistent") == 0
rc = lib.dxrpt_host_scene_create(1, C.c_uint64(0), 1, C.byref(out))
assert rc == -1 and b"opacity map" in lib.dxrpt_host_last_error(), (rc, lib.dxrpt_host_last_error())
print("ok")
"""
    import dxrpathtracer_amd._abi as A
    r = subprocess.run([sys.executable, "-c", code, A.LIB_DIR], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr
