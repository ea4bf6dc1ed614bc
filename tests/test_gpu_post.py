"""GPU parity of dxrpt_post_process (the consumer of the accumulation buffer) against oracle/post.py."""
import numpy as np
import pytest

import dxrpathtracer_amd as D
import dxrpathtracer_amd._abi as A
from dxrpathtracer_amd.tracer import DXRPathTracer
from oracle import post as P
from tests._common import scene_bundle

pytestmark = pytest.mark.gpu


def _hdr(rng, H, W):
    # radiance in the FP16Scale-prescaled units of the accumulation buffer (sun-lit ~ 0.1 .. 100)
    img = np.exp(rng.normal(0.0, 2.0, size=(H, W, 4))).astype(np.float32)
    img[..., 3] = 1.0
    return img


@pytest.mark.parametrize("W,H", [(64, 48), (97, 33), (1920, 1080)])
@pytest.mark.parametrize("fmt", [A.POST_FLOAT4, A.POST_RGBA8])
def test_post_process_matches_oracle(torch_cuda, W, H, fmt):
    torch = torch_cuda
    rng = np.random.default_rng(W * 1000 + H)
    img = _hdr(rng, H, W)
    st = A.default_settings()
    st.Exposure = -11.5
    st.BloomExposure = -3.0
    st.BloomMagnitude = 0.75
    st.BloomBlurSigma = 1.8
    t = DXRPathTracer(0)
    try:
        acc = torch.from_numpy(img.reshape(-1, 4)).cuda()
        out = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda") if fmt == A.POST_FLOAT4 else \
            torch.zeros((H * W,), dtype=torch.int32, device="cuda")
        t.post_process(st, acc.data_ptr(), W, H, out.data_ptr(), fmt, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    finally:
        t.close()
    ref = P.post_process(img, st.Exposure, st.BloomExposure, st.BloomMagnitude, st.BloomBlurSigma,
                         rgba8=fmt == A.POST_RGBA8)
    if fmt == A.POST_FLOAT4:
        got = out.cpu().numpy().reshape(H, W, 4)
        np.testing.assert_allclose(got, ref, rtol=1e-6, atol=0)
    else:
        got = out.cpu().numpy().view(np.uint8).reshape(H, W, 4)
        np.testing.assert_array_equal(got, ref)


def test_post_process_of_a_rendered_frame(torch_cuda):
    # the drop-in chain: dxrpt_render's accumulation buffer straight into dxrpt_post_process
    torch = torch_cuda
    W, H = 160, 90
    sc, sky = scene_bundle("sponza")
    st = sc.settings(MaxPathLength=3)
    t = DXRPathTracer(0)
    try:
        t.initialize_scene(sc, sky)
        t.build_rt_acceleration_structure()
        acc = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        for k in range(2):
            t.render_raw(D.make_constants(sc, st, sky, W, H, k), st, acc.data_ptr(), W, H, stream=s,
                         lights=D.make_lights(sc))
        out = torch.zeros((H * W,), dtype=torch.int32, device="cuda")
        t.post_process(st, acc.data_ptr(), W, H, out.data_ptr(), A.POST_RGBA8, s)
        torch.cuda.synchronize()
    finally:
        t.close()
    got = out.cpu().numpy().view(np.uint8).reshape(H, W, 4)
    ref = P.post_process(acc.cpu().numpy().reshape(H, W, 4), st.Exposure, st.BloomExposure, st.BloomMagnitude,
                         st.BloomBlurSigma, rgba8=True)
    np.testing.assert_array_equal(got, ref)
    assert got[..., :3].mean() > 5  # a lit image, not black


def test_post_process_rejects_bad_arguments(torch_cuda):
    torch = torch_cuda
    t = DXRPathTracer(0)
    try:
        acc = torch.zeros((4, 4), dtype=torch.float32, device="cuda")
        with pytest.raises(Exception, match="2 x 2"):
            t.post_process(A.default_settings(), acc.data_ptr(), 1, 4, acc.data_ptr())
        with pytest.raises(Exception, match="format"):
            t.post_process(A.default_settings(), acc.data_ptr(), 2, 2, acc.data_ptr(), 7)
    finally:
        t.close()
