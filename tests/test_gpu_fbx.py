"""GPU parity on a scene ingested through dxrpt_host_scene_load (FBX + BC1/BC4 DDS textures, or a PNG
albedo and a JPEG opacity -- the WIC formats -- alpha tested through the TransparentColor -> opacity
slot): the HIP path against the CPU oracle on the same loaded inputs.  The scene is a synthetic FBX written by the test (the reference's assets do not travel
to the GPU box)."""
import numpy as np
import pytest

import dxrpathtracer_amd as D
import dxrpathtracer_amd._abi as A
from dxrpathtracer_amd.tracer import DXRPathTracer
from oracle import pyoracle as O
from tests import fbx_util as F
from tests._common import assert_parity

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("images", ["dds", "png"])
@pytest.mark.parametrize("max_any_hit", [1, 3])
@pytest.mark.parametrize("mega", [0, A.DEFAULT_MEGAKERNEL_PATHS])  # wavefront passes / one-kernel frame
def test_fbx_scene_matches_oracle(torch_cuda, tmp_path, max_any_hit, mega, images):
    torch = torch_cuda
    if images == "png":
        pytest.importorskip("PIL.Image")
    sc = D.Scene(A.SCENE_BOXTEST, model_path=F.box_room_fbx(str(tmp_path), images=images))
    assert sc.materials[0][4] != 0xFFFFFFFF  # opacity map present: alpha-tested geometry
    st = sc.settings(MaxPathLength=4, MaxAnyHitPathLength=max_any_hit)
    sky = D.make_sky(st)
    W, H = 160, 96
    t = DXRPathTracer(0)
    t.set_option(A.OPT_MEGAKERNEL_PATHS, mega)
    try:
        t.initialize_scene(sc, sky)
        t.build_rt_acceleration_structure()
        for s in (0, 3):
            rtc = D.make_constants(sc, st, sky, W, H, s)
            acc = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
            t.render_raw(rtc, st, acc.data_ptr(), W, H, stream=torch.cuda.current_stream().cuda_stream,
                         lights=D.make_lights(sc))
            torch.cuda.synchronize()
            gpu = acc.cpu().numpy().reshape(H, W, 4)
            ref, _ = O.OracleScene(sc, sky).render(rtc, st, D.make_lights(sc), W, H)
            assert_parity(gpu, ref, f"fbx room s{s} anyhit{max_any_hit}")
            assert np.isfinite(gpu).all() and gpu[..., :3].max() > 0
    finally:
        t.close()
