"""GPU parity of the lightmap baker (dxrpt_bake_lightmap, dxrpt_denoise_median) against the oracle.

Same gate as the renders (tests/_common.py: per-texel RGB within 1e-4 relative), on surface maps
rasterised from the chart atlas of BoxTest (whole lightmap) and of the Sponza proxy (a texel band the
oracle finishes in seconds; the GPU bakes the whole map).  Sample counts > 1 exercise the firefly
clamp against the running average; the valid-sample counts (accum.w) must match exactly.
"""
import numpy as np
import pytest

import dxrpathtracer_amd as D
import dxrpathtracer_amd._abi as A
from dxrpathtracer_amd.scene import lightmap_charts, surface_map
from dxrpathtracer_amd.tracer import DXRPathTracer
from oracle import pyoracle as O
from tests._common import RTOL, oracle_scene, rel_err, scene_bundle

pytestmark = pytest.mark.gpu

_T = {}


def tracer(name):
    if name not in _T:
        sc, sky = scene_bundle(name)
        t = DXRPathTracer(0)
        t.initialize_scene(sc, sky)
        t.build_rt_acceleration_structure()
        _T[name] = t
    return _T[name]


def _maps(name, res):
    sc, _ = scene_bundle(name)
    verts, idx = lightmap_charts(sc, res)
    return surface_map(verts, idx, res, res)


def _gpu_bake(torch, name, pos, nrm, st, samples, chunk=None):
    t = tracer(name)
    H, W = pos.shape[:2]
    if chunk is not None:
        t.set_option(A.OPT_BAKE_CHUNK, chunk)
    dpos = torch.from_numpy(pos.reshape(-1, 4)).cuda()
    dnrm = torch.from_numpy(nrm.reshape(-1, 4)).cuda()
    acc = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
    lm = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
    try:
        for s in samples:
            t.bake_lightmap(st, dpos.data_ptr(), dnrm.data_ptr(), acc.data_ptr(), lm.data_ptr(), W, H, s,
                            torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    finally:
        if chunk is not None:
            t.set_option(A.OPT_BAKE_CHUNK, A.DEFAULT_BAKE_CHUNK)
    return acc.cpu().numpy().reshape(H, W, 4), lm.cpu().numpy().reshape(H, W, 4)


def _oracle_bake(name, pos, nrm, st, samples, first=0, count=None):
    sc, sky = scene_bundle(name)
    H, W = pos.shape[:2]
    acc = np.zeros_like(pos)
    lm = np.zeros_like(pos)
    for s in samples:
        rtc = D.make_constants(sc, st, sky, W, H, s)
        oracle_scene(name).bake(rtc, st, D.make_lights(sc), pos, nrm, acc, lm, first=first, count=count)
    return acc, lm


def _check(gpu, ref, what, rows=None):
    ga, gl = gpu
    ra, rl = ref
    if rows is not None:
        ga, gl, ra, rl = ga[rows], gl[rows], ra[rows], rl[rows]
    np.testing.assert_array_equal(ga[..., 3], ra[..., 3], err_msg=f"{what}: valid-sample counts differ")
    np.testing.assert_array_equal(gl[..., 3], rl[..., 3], err_msg=f"{what}: lightmap alpha differs")
    for g, r, name in ((ga, ra, "accum"), (gl, rl, "lightmap")):
        assert np.isfinite(g).all(), f"{what} {name}: non-finite texels"
        e = rel_err(g[..., :3], r[..., :3])
        if e.max() > RTOL:
            i = tuple(np.argwhere(e > RTOL)[0][:2])
            raise AssertionError(f"{what} {name}: {int((e > RTOL).any(axis=-1).sum())} texels exceed rel {RTOL} "
                                 f"(max {e.max():.3e}); first {i} gpu={g[i]} ref={r[i]}")


@pytest.mark.parametrize("samples", [[0], [0, 1, 2, 3]])
def test_bake_boxtest_matches_oracle(torch_cuda, samples):
    pos, nrm = _maps("boxtest", 64)
    sc, _ = scene_bundle("boxtest")
    st = sc.settings(SqrtNumSamples=4)
    gpu = _gpu_bake(torch_cuda, "boxtest", pos, nrm, st, samples)
    ref = _oracle_bake("boxtest", pos, nrm, st, samples)
    _check(gpu, ref, f"boxtest 64^2 samples {samples}")
    assert (gpu[0][..., 3] > 0).sum() > 1000  # most covered texels took valid samples


@pytest.mark.parametrize("L", [2, 3, 5])
def test_bake_sponza_band_matches_oracle(torch_cuda, L):
    res = 2048
    pos, nrm = _maps("sponza", res)
    sc, _ = scene_bundle("sponza")
    st = sc.settings(MaxPathLength=L)
    samples = [0, 1]
    gpu = _gpu_bake(torch_cuda, "sponza", pos, nrm, st, samples)
    y0, nrows = 700, 12  # a band of 24k texels across many charts
    ref = _oracle_bake("sponza", pos, nrm, st, samples, first=y0 * res, count=nrows * res)
    _check(gpu, ref, f"sponza {res}^2 L={L} rows {y0}..{y0 + nrows}", rows=slice(y0, y0 + nrows))
    assert (pos[y0:y0 + nrows, :, 3] > 0).sum() > 5000


def test_bake_markers_and_chunking(torch_cuda):
    pos, nrm = _maps("boxtest", 64)
    pos[0, 0] = (np.inf, 0, 0, 1)
    nrm[0, 1] = 0
    pos[0, 1, 3] = 1
    nrm[0, 2] = (np.nan, 0, 0, 1)
    pos[0, 2, 3] = 1
    sc, _ = scene_bundle("boxtest")
    st = sc.settings()
    a = _gpu_bake(torch_cuda, "boxtest", pos, nrm, st, [0, 1])
    ref = _oracle_bake("boxtest", pos, nrm, st, [0, 1])
    np.testing.assert_array_equal(a[1][0, :3], ref[1][0, :3])
    np.testing.assert_array_equal(a[1][0, 0], [0, 0, 1, 1])
    np.testing.assert_array_equal(a[1][0, 1], [0, 0, 0, 1])
    np.testing.assert_array_equal(a[1][0, 2], [1, 0, 1, 1])
    b = _gpu_bake(torch_cuda, "boxtest", pos, nrm, st, [0, 1], chunk=100)  # 41 launches, ragged tail
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])


@pytest.mark.parametrize("W,H", [(1, 1), (7, 5), (512, 256)])
def test_median_denoise_matches_oracle(torch_cuda, W, H):
    torch = torch_cuda
    rng = np.random.default_rng(W * 31 + H)
    img = np.exp(rng.normal(0, 1.5, size=(H, W, 4))).astype(np.float32)
    img[H // 2:, : W // 2] = 0.25  # luminance ties
    t = tracer("boxtest")
    din = torch.from_numpy(img.reshape(-1, 4)).cuda()
    dout = torch.zeros_like(din)
    t.denoise_median(din.data_ptr(), dout.data_ptr(), W, H, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dout.cpu().numpy().reshape(H, W, 4), O.median3x3(img))
    with pytest.raises(RuntimeError):
        t.denoise_median(din.data_ptr(), din.data_ptr(), W, H, 0)
