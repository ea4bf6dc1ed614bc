"""GPU: the overlapped-frame scratch audit ("Per-frame scratch under overlapped frames").

Every shipped overlapped schedule -- the metric frame (depth-split, three frames in flight), C3 (L=8,
five tails a frame), C2 720p, the 1/2 share (split) and the cost-ordered 1/8 share (order rebuilt every
frame and every 2nd, the r05 ADVICE hazard) -- renders many frames back to back with no host sync, and
the kernels' range-check record (dxrpt_get_debug_record) must stay empty.  In the shipped build the checks
are compiled out (the record is all zeros, is_debug_build False); the same file under the debug kernels
(DXRPT_KERNEL_LIB_DIR=ab/debug, built by `make variant NAME=debug EXTRA=-DDXRPT_DEBUG=1`) checks every
queue entry a tail reads and every stage entry a blend reads: scripts/debug_build_run.sh, record in
profiles/r06_debug_build.txt."""
import numpy as np
import pytest

import dxrpathtracer_amd as D
import dxrpathtracer_amd._abi as A
from dxrpathtracer_amd.distributed import band_layout
from dxrpathtracer_amd.tracer import DXRPathTracer
from tests._common import scene_bundle

pytestmark = pytest.mark.gpu

CASES = [  # id, W, H, L, share (world, rank) or None, frames, options
    ("metric", 1920, 1080, 3, None, 24, ()),
    ("c3", 1920, 1080, 8, None, 12, ()),
    ("c2", 1280, 720, 3, None, 24, ()),
    ("half_share", 1920, 1080, 3, (2, 1), 24, ()),
    ("eighth_share_period1", 1920, 1080, 3, (8, 5), 40, ((A.OPT_WAVE_ORDER_PERIOD, 1),)),
    ("eighth_share_period2", 1920, 1080, 3, (8, 2), 40, ((A.OPT_WAVE_ORDER_PERIOD, 2),)),
    ("eighth_share_default", 1920, 1080, 3, (8, 7), 40, ()),
]


@pytest.mark.parametrize("name,W,H,L,share,frames,options", CASES, ids=[c[0] for c in CASES])
def test_overlapped_schedules_pass_the_range_checks(torch_cuda, name, W, H, L, share, frames, options):
    torch = torch_cuda
    sc, sky = scene_bundle("sponza")
    st = sc.settings(MaxPathLength=L)
    lights = D.make_lights(sc)
    tiles, n = None, W * H
    if share is not None:
        lay = band_layout(W, H, share[0])
        tiles, n = lay.tile_array(share[1]), lay.counts[share[1]]
    t = DXRPathTracer(0)
    try:
        t.initialize_scene(sc, sky)
        t.build_rt_acceleration_structure()
        for o, v in options:
            t.set_option(o, v)
        t.debug_record()  # zero the record
        acc = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        for f in range(frames):
            t.render_raw(D.make_constants(sc, st, sky, W, H, f % 16), st, acc.data_ptr(), W, H, tiles=tiles,
                         stream=stream, lights=lights)
        torch.cuda.synchronize()
        s = t.stats()
        assert s.schedule & A.SCHED_OVERLAP, s.schedule
        rec = t.debug_record()
        assert rec["violations"] == 0, rec
        if rec["is_debug_build"]:
            # the tails checked at least every queued entry of every frame (the split schedules), and the
            # blends every path; the single k_path frames have no queues
            if s.schedule & A.SCHED_SPLIT:
                assert rec["checked"] >= frames * n * 0.9, rec
            print(f"debug build: {name} {frames} frames, {rec['checked']} queue entries checked, 0 violations")
        else:
            assert rec == {"violations": 0, "kind": 0, "depth": 0, "lane": 0, "value": 0, "bound": 0, "checked": 0,
                           "is_debug_build": False}, rec
        assert np.isfinite(acc.cpu().numpy()).all()
    finally:
        t.close()
