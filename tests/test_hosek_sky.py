"""Hosek-Wilkie sky (the reference's SkyCache::Init sky, host/hosek.cpp) on CPU.

Pins: the reference's own sky code compiled verbatim (tests/golden/make_hosek_reference.py: the whole of
HosekSky/ArHosekSkyModel.cpp and Graphics/Spectrum.cpp, SkyCache::Init / Sample's statements from
Graphics/Skybox.cpp:31-154,254-269, DirectXMath's four Float3 ops restated from its SSE2 paths) ->
tests/golden/hosek_reference.npz: SunIrradiance, SunRenderColor and every FP16 texel of the full
6 x 128 x 128 cube for the scenes' skies, plus a 6 x 16 x 16 sweep over turbidity 1..10, coloured albedo and
sun elevation -- matched BIT FOR BIT (tolerance 0).  Also the zenith probe of SURVEY.md 8(c) (3.04945) and
regression vectors of this restatement (tests/golden/hosek_sky.json).  The tables come from the packaged
file (data/hosek_tables.bin), so these tests run without the reference checkout; where the checkout is
present, the packaged file is checked against the reference's dataset sources table by table.
"""
import json
import math
import os

import numpy as np
import pytest

import dxrpathtracer_amd as D
import dxrpathtracer_amd._abi as A

HOSEK = D.scene.load_hosek()
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "hosek_sky.json")
REFERENCE = os.path.join(os.path.dirname(__file__), "golden", "hosek_reference.npz")


def _f32(x):
    return np.float32(x)


def test_zenith_probe_matches_reference():
    s = np.array([0.26, 0.987, -0.16], dtype=np.float32)
    s = s / _f32(np.sqrt(_f32(s[0] * s[0] + s[1] * s[1]) + _f32(s[2] * s[2])))
    theta_s = _f32(np.arccos(_f32(max(s[1], _f32(1e-5)))))
    elevation = _f32(_f32(1.570796327) - theta_s)
    r = HOSEK.rgb_radiance(2.0, 0.25, float(elevation), 0.0, float(theta_s), 0)
    v = _f32(_f32(_f32(r) * _f32(683.0)) * _f32(2.0 ** -10))
    assert abs(float(v) - 3.04945) < 1e-5


def _sky(p, res):
    import ctypes as C
    cube = np.zeros(6 * res * res * 4, dtype=np.uint16)
    irr, ren = (C.c_float * 3)(), (C.c_float * 3)()
    rc = A.host().dxrpt_host_sky_create_hosek(HOSEK.handle, (C.c_float * 3)(*p[:3]), float(p[3]), float(p[4]),
                                              (C.c_float * 3)(*p[5:8]), res, cube.ctypes.data, irr, ren)
    assert rc == 0, A.host().dxrpt_host_hosek_last_error()
    return np.array(irr, np.float32), np.array(ren, np.float32), cube.reshape(6, res, res, 4)


def test_sky_matches_reference_skycache_bit_for_bit():
    """SkyCache::Init + Sample of the reference, compiled verbatim (make_hosek_reference.py): sun irradiance,
    sun render colour and every FP16 cube texel identical (tolerance 0) for each case."""
    g = np.load(REFERENCE)
    names = [str(n) for n in g["names"]]
    assert {"sponza", "suntemple"} <= set(names) and len(names) >= 8
    for i, name in enumerate(names):
        p, res = g["params"][i], int(g["res"][i])
        irr, ren, cube = _sky(p, res)
        np.testing.assert_array_equal(irr.view(np.uint32), g[f"{name}_sun_irradiance"].view(np.uint32), err_msg=name)
        np.testing.assert_array_equal(ren.view(np.uint32), g[f"{name}_sun_render_color"].view(np.uint32), err_msg=name)
        # the reference's texels: XMStoreHalf4 of Sample()'s float32 radiance (round to nearest even), alpha 1
        ref = g[f"{name}_cube_f16"] if f"{name}_cube_f16" in g.files else g[f"{name}_cube"].astype(np.float16).view(np.uint16)
        assert ref.shape == (6, res, res, 3)
        np.testing.assert_array_equal(cube[..., :3], ref, err_msg=name)
        assert (cube[..., 3] == 0x3C00).all()
        if f"{name}_cube_f32_every8" in g.files:  # the stored float32 samples are the texels' source values
            np.testing.assert_array_equal(g[f"{name}_cube_f32_every8"].astype(np.float16).view(np.uint16), ref[:, 4::8, 4::8])


def test_radiance_depends_on_view_and_sun_angles_only():
    a = HOSEK.rgb_radiance(3.0, 0.1, 0.6, 0.4, 0.9, 1)
    assert a == HOSEK.rgb_radiance(3.0, 0.1, 0.6, 0.4, 0.9, 1)
    assert a > 0.0
    # brighter towards the sun (gamma -> 0) at fixed theta
    assert HOSEK.rgb_radiance(3.0, 0.1, 0.6, 0.4, 0.05, 1) > a
    # turbidity interpolation is continuous across integer knots
    lo = HOSEK.rgb_radiance(2.0 - 1e-9, 0.1, 0.6, 0.4, 0.9, 0)
    hi = HOSEK.rgb_radiance(2.0, 0.1, 0.6, 0.4, 0.9, 0)
    assert abs(lo - hi) <= 1e-6 * abs(hi)


def test_solar_radiance_positive_inside_disc_and_zero_spectrum_outside_range():
    inside = HOSEK.solar_radiance(0.8, 2.0, 0.25, 0.7, 0.001, 550.0)
    outside = HOSEK.solar_radiance(0.8, 2.0, 0.25, 0.7, 0.5, 550.0)  # off the disc: sky only
    assert inside > outside > 0.0
    # wavelengths beyond the 320..720 nm datasets: the sky part returns 0 (ArHosekSkyModel.cpp:529-530)
    assert HOSEK.solar_radiance(0.8, 2.0, 0.25, 0.7, 0.5, 719.0) > 0.0


def test_spectrum_conversions():
    assert HOSEK.spectrum_from_rgb((0.0, 0.0, 0.0)) == [0.0] * 60
    assert HOSEK.spectrum_to_rgb([0.0] * 60) == (0.0, 0.0, 0.0)
    # grey reflectance: white basis only, scaled by 0.94 (Spectrum.cpp:113-153)
    g = HOSEK.spectrum_from_rgb((0.25, 0.25, 0.25))
    w = HOSEK.spectrum_from_rgb((1.0, 1.0, 1.0))
    np.testing.assert_allclose(np.array(g), np.array(w) * 0.25, rtol=1e-6)
    # the equal-energy spectrum has Y = 1 (ToXYZ normalises by the CIE Y integral) and is reddish in sRGB
    rgb = HOSEK.spectrum_to_rgb([1.0] * 60)
    y = 0.212671 * rgb[0] + 0.715160 * rgb[1] + 0.072169 * rgb[2]
    assert abs(y - 1.0) < 0.01 and rgb[0] > rgb[1] > rgb[2]


def test_sky_matches_regression_vectors():
    gold = json.load(open(GOLDEN))
    for name, g in gold["scenes"].items():
        st = D.Scene(name).settings()
        sky = D.make_sky(st, model="hosek")
        assert sky.model == "hosek"
        np.testing.assert_array_equal(np.float32(sky.sun_irradiance), np.float32(g["sun_irradiance"]))
        np.testing.assert_array_equal(np.float32(sky.sun_render_color), np.float32(g["sun_render_color"]))
        cube = sky.cube.reshape(6, sky.res, sky.res, 4)
        for key, texel in g["texels"].items():
            s, y, x = map(int, key.split(","))
            assert [int(v) for v in cube[s, y, x]] == texel, (name, key)
        assert int(sky.cube.astype(np.uint64).sum()) == g["cube_u16_sum"]


def test_sky_cube_layout_and_sun_constants():
    st = D.Scene("sponza").settings()
    sky = D.make_sky(st, model="hosek", res=32)
    cube = sky.cube.view(np.float16).reshape(6, 32, 32, 4).astype(np.float32)
    assert np.isfinite(cube).all() and (cube[..., :3] > 0).all()
    assert (cube[..., 3] == 1.0).all()
    # the cube excludes the sun; the sun render colour is irradiance / (pi sin^2(1 deg)) clamped to FP16Max
    assert max(sky.sun_render_color) == 65000.0
    ratio = np.array(sky.sun_render_color) / np.array(sky.sun_irradiance)
    np.testing.assert_allclose(ratio, ratio[0], rtol=1e-5)
    # +y face centre (zenith) is bluer than red
    z = cube[2, 16, 16]
    assert z[2] > z[0]


def test_missing_dataset_is_an_error_not_a_crash(tmp_path):
    import ctypes as C
    p = C.c_void_p()
    rc = A.host().dxrpt_host_hosek_load(str(tmp_path).encode(), str(tmp_path / "none.cpp").encode(), C.byref(p))
    assert rc != 0 and not p.value
    assert b"cannot read" in A.host().dxrpt_host_hosek_last_error()
    rc = A.host().dxrpt_host_hosek_load_tables(str(tmp_path / "none.bin").encode(), C.byref(p))
    assert rc != 0 and not p.value
    assert b"cannot read" in A.host().dxrpt_host_hosek_last_error()


def test_truncated_table_file_is_rejected(tmp_path):
    import ctypes as C
    blob = open(D.scene.HOSEK_TABLES, "rb").read()
    for cut in (4, 12, len(blob) // 2, len(blob) - 1):
        f = tmp_path / f"cut{cut}.bin"
        f.write_bytes(blob[:cut])
        p = C.c_void_p()
        assert A.host().dxrpt_host_hosek_load_tables(str(f).encode(), C.byref(p)) != 0 and not p.value
        assert b"malformed" in A.host().dxrpt_host_hosek_last_error()


def test_default_sky_is_hosek():
    assert D.make_sky(D.Scene("sponza").settings(), res=8).model == "hosek"


@pytest.mark.skipif(D.scene.reference_hosek_sources() is None, reason="reference checkout not present")
def test_packaged_tables_match_reference_sources():
    """The packaged table file and the reference's dataset sources give the same model, bit for bit."""
    src = D.scene.HosekData(None, *D.scene.reference_hosek_sources())
    for args in ((2.0, 0.25, 0.9, 0.3, 0.7, 0), (7.5, 0.6, 0.1, 1.2, 0.05, 2), (1.0, 0.0, 1.5, 0.0, 1.5, 1)):
        assert HOSEK.rgb_radiance(*args) == src.rgb_radiance(*args)
    for wl in (400.0, 455.0, 550.0, 699.0):
        assert HOSEK.solar_radiance(0.8, 3.3, 0.4, 0.7, 0.001, wl) == src.solar_radiance(0.8, 3.3, 0.4, 0.7, 0.001, wl)
    assert HOSEK.spectrum_from_rgb((0.2, 0.5, 0.9)) == src.spectrum_from_rgb((0.2, 0.5, 0.9))
    assert HOSEK.spectrum_to_rgb([float(i) for i in range(60)]) == src.spectrum_to_rgb([float(i) for i in range(60)])


def test_turbidity_above_fit_range_is_rejected():
    st = D.Scene("sponza").settings()
    with pytest.raises(RuntimeError, match="turbidity"):
        D.make_sky(st, turbidity=12.0, model="hosek")
    assert math.isfinite(D.make_sky(st, turbidity=12.0, model="analytic").sun_irradiance[0])
