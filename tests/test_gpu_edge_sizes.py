"""GPU parity at degenerate frame sizes and tile lists, on every schedule (SURVEY.md 8(c) edge cases).

Frames of 1x1, a single row, a single column and odd sizes below one wave (partial last waves, a split
tail queue holding one path, cost-ordered frames of one wave), tile lists with an empty tile, and two
accumulated samples, against the oracle's full frame -- through the shipped megakernel schedules
(overlapped frames on and off, the depth-split schedule forced on, cost-ordered waves) and the
wavefront passes.  Gate: tests/_common.py (1e-4 relative).
"""
import numpy as np
import pytest

import dxrpathtracer_amd as D
import dxrpathtracer_amd._abi as A
from dxrpathtracer_amd.tracer import DXRPathTracer
from tests._common import assert_parity, oracle_scene, scene_bundle

pytestmark = pytest.mark.gpu

SIZES = [(1, 1), (3, 1), (1, 5), (7, 9), (65, 1), (63, 2), (129, 3)]
SCHEDULES = {
    "overlap": {},
    "no_overlap": {A.OPT_FRAME_OVERLAP: 0},
    "split": {A.OPT_MEGAKERNEL_SPLIT: 1},
    "split_no_overlap": {A.OPT_MEGAKERNEL_SPLIT: 1, A.OPT_FRAME_OVERLAP: 0},
    "ordered": {A.OPT_WAVE_ORDER: 1, A.OPT_WAVE_ORDER_PERIOD: 1},
    "wavefront": {A.OPT_MEGAKERNEL_PATHS: 0},
}
_TRACERS = {}


def tracer(name, schedule):
    key = (name, schedule)
    if key not in _TRACERS:
        sc, sky = scene_bundle(name)
        t = DXRPathTracer(0)
        t.initialize_scene(sc, sky)
        t.build_rt_acceleration_structure()
        for o, v in SCHEDULES[schedule].items():
            t.set_option(o, v)
        _TRACERS[key] = t
    return _TRACERS[key]


def render(torch, name, schedule, W, H, st, samples, tiles=None, n_out=None):
    sc, sky = scene_bundle(name)
    t = tracer(name, schedule)
    n = n_out if n_out is not None else W * H
    acc = torch.zeros((max(n, 1), 4), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for s in range(samples):
        t.render_raw(D.make_constants(sc, st, sky, W, H, s), st, acc.data_ptr(), W, H, tiles=tiles, stream=stream,
                     lights=D.make_lights(sc))
    torch.cuda.synchronize()
    return acc.cpu().numpy()[:n]


def oracle_frame(name, W, H, st, samples):
    sc, sky = scene_bundle(name)
    ref = None
    for s in range(samples):
        ref, _ = oracle_scene(name).render(D.make_constants(sc, st, sky, W, H, s), st, D.make_lights(sc), W, H,
                                           accum=ref)
    return ref


@pytest.mark.parametrize("schedule", sorted(SCHEDULES))
@pytest.mark.parametrize("L", [3, 8])
def test_degenerate_frame_sizes(torch_cuda, schedule, L):
    sc, _ = scene_bundle("sponza")
    st = sc.settings(MaxPathLength=L)
    for (W, H) in SIZES:
        out = render(torch_cuda, "sponza", schedule, W, H, st, 2)
        ref = oracle_frame("sponza", W, H, st, 2)
        assert_parity(out.reshape(H, W, 4), ref, f"sponza {W}x{H} L{L} {schedule}")


@pytest.mark.parametrize("schedule", sorted(SCHEDULES))
def test_tile_lists_with_empty_and_single_pixel_tiles(torch_cuda, schedule):
    """An empty tile between a 1x1 tile and a 5x3 tile (accum offsets packed), on a 64x48 frame."""
    W, H = 64, 48
    sc, _ = scene_bundle("suntemple")
    st = sc.settings()
    tiles = [A.Tile(10, 7, 1, 1, 0, 1, 0), A.Tile(30, 30, 0, 4, 1, 0, 0), A.Tile(40, 20, 5, 3, 1, 5, 0)]
    out = render(torch_cuda, "suntemple", schedule, W, H, st, 1, tiles=tiles, n_out=16)
    ref = oracle_frame("suntemple", W, H, st, 1)
    assert_parity(out[0:1].reshape(1, 1, 4), ref[7:8, 10:11], f"1x1 tile {schedule}")
    assert_parity(out[1:16].reshape(3, 5, 4), ref[20:23, 40:45], f"5x3 tile {schedule}")


@pytest.mark.parametrize("schedule", ["overlap", "no_overlap", "wavefront"])
def test_tile_lists_without_pixels_render_nothing(torch_cuda, schedule):
    """An empty tile list (a rank of an N-GPU partition with no band) or one of zero-area tiles: the call
    succeeds, writes no pixel, and the next frame is unaffected (include/dxrpt.h, dxrpt_render)."""
    torch = torch_cuda
    sc, sky = scene_bundle("boxtest")
    st = sc.settings()
    t = tracer("boxtest", schedule)
    stream = torch.cuda.current_stream().cuda_stream
    acc = torch.full((4, 4), 7.0, dtype=torch.float32, device="cuda")
    for tiles in ([], [A.Tile(3, 3, 0, 0, 0, 0, 0), A.Tile(5, 1, 4, 0, 0, 4, 0)]):
        t.render_raw(D.make_constants(sc, st, sky, 16, 16, 0), st, acc.data_ptr(), 16, 16, tiles=tiles, stream=stream,
                     lights=D.make_lights(sc))
    torch.cuda.synchronize()
    assert np.all(acc.cpu().numpy() == 7.0)
    out = render(torch, "boxtest", schedule, 16, 16, st, 1)
    assert_parity(out.reshape(16, 16, 4), oracle_frame("boxtest", 16, 16, st, 1), f"boxtest 16x16 after empty lists {schedule}")


def test_tile_outside_the_image_is_an_error(torch_cuda):
    import torch
    sc, sky = scene_bundle("boxtest")
    st = sc.settings()
    t = tracer("boxtest", "overlap")
    acc = torch.zeros((64, 4), dtype=torch.float32, device="cuda")
    with pytest.raises(RuntimeError, match="outside the image"):
        t.render_raw(D.make_constants(sc, st, sky, 16, 16, 0), st, acc.data_ptr(), 16, 16,
                     tiles=[A.Tile(12, 0, 8, 8, 0, 8, 0)], stream=torch.cuda.current_stream().cuda_stream,
                     lights=D.make_lights(sc))
