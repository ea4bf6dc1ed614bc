"""GPU parity of the STEADY-STATE shipped schedule: consecutive progressive frames through one fresh,
untouched context, as bench.py and every rank of an N-GPU run render them.

Defaults (r03, overlapped frames, DXRPT_OPT_FRAME_OVERLAP 1): every megakernel frame stages its radiance
and is blended on the caller's stream; 64-lane waves at every size; a frame of at most 1.5 rounds of
resident waves (a GPU's 1/8 share of the metric frame) runs the cost-ordered instantiation -- frame 0
records its wave costs in path order, frames 1+ start their waves in the cost order built from them
(DXRPT_OPT_WAVE_ORDER, default "by frame size") -- larger ones path order.  With overlap off the cost
order holds up to 3 rounds.  Each test renders >= 3
consecutive frames (RaygenShader over
DispatchRays(W, H, 1), RayTrace.hlsl:92-149) into ONE accumulation target, checks after every frame
that the schedule it expects actually ran (dxrpt_stats.schedule / paths_per_wave), and compares the
accumulated crops with the oracle accumulated the same way (the progressive rule, RayTrace.hlsl:140-148).
Gate: tests/_common.py (1e-4 relative).
"""
import numpy as np
import pytest

import dxrpathtracer_amd as D
import dxrpathtracer_amd._abi as A
from dxrpathtracer_amd.distributed import band_layout
from dxrpathtracer_amd.tracer import DXRPathTracer
from tests._common import assert_parity, oracle_scene, scene_bundle

pytestmark = pytest.mark.gpu


def _fresh(name):
    sc, sky = scene_bundle(name)
    t = DXRPathTracer(0)
    t.initialize_scene(sc, sky)
    t.build_rt_acceleration_structure()
    return t


def _band_crops(lay, rank, n=4, w=128):
    """(crop, slab offset of its first pixel, slab pitch) for n bands of the rank spread over its list."""
    tiles = lay.rank_tiles(rank)
    picks = sorted({0, len(tiles) // 3, (2 * len(tiles)) // 3, len(tiles) - 1})[:n]
    out = []
    for k, i in enumerate(picks):
        t = tiles[i]
        x0 = t.x0 + (k * 397) % (t.w - w)
        out.append(((x0, t.y0, w, t.h), t.accum_offset + (x0 - t.x0), t.accum_pitch))
    return out


def _frame_crops(W, H):
    c = 64
    crops = [(0, 0, c, c), (W - c, H - c, c, c), (W // 2 - 48, H // 2 - 32, 96, 64), (W // 3, H - 40, 80, 40)]
    return [(cr, cr[1] * W + cr[0], W) for cr in crops]


def _steady_frames(torch, name, W, H, L, frames, crops, tiles=None, n_out=None, expect=None, options=()):
    sc, sky = scene_bundle(name)
    st = sc.settings(MaxPathLength=L)
    lights = D.make_lights(sc)
    t = _fresh(name)
    for opt, val in options:
        t.set_option(opt, val)
    n = W * H if n_out is None else n_out
    acc = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
    refs = [None] * len(crops)
    stream = torch.cuda.current_stream().cuda_stream
    scheds = []
    try:
        for f in range(frames):
            rtc = D.make_constants(sc, st, sky, W, H, f)
            t.render_raw(rtc, st, acc.data_ptr(), W, H, tiles=tiles, stream=stream, lights=lights)
            torch.cuda.synchronize()
            s = t.stats()
            scheds.append((s.schedule, s.paths_per_wave))
            if expect is not None:
                expect(f, s)
            out = acc.cpu().numpy()
            for k, ((x0, y0, w, h), off, pitch) in enumerate(crops):
                refs[k], _ = oracle_scene(name).render(rtc, st, lights, W, H, crop=(x0, y0, w, h), accum=refs[k])
                rows = np.array([[off + yy * pitch + xx for xx in range(w)] for yy in range(h)])
                assert_parity(out[rows], refs[k], f"{name} {W}x{H} L{L} frame {f} crop {(x0, y0, w, h)}")
    finally:
        t.close()
    return scheds


def _expect(lanes, ordered, overlap=True, split=False):
    def check(f, s):
        assert s.schedule & A.SCHED_MEGAKERNEL and not s.schedule & A.SCHED_CENSUS, s.schedule
        # from 1.5M path vertices (three frames in flight; 2M with two) the depth-split schedule, one part
        assert bool(s.schedule & A.SCHED_SPLIT) == split, f"frame {f}: schedule {s.schedule}"
        assert bool(s.schedule & A.SCHED_OVERLAP) == overlap, f"frame {f}: schedule {s.schedule}"
        assert bool(s.schedule & A.SCHED_ORDER_KERNEL) == ordered, \
            f"frame {f}: the {'cost-ordered' if ordered else 'path-ordered'} instantiation did not run ({s.schedule})"
        # frame 0 builds the order from its own wave costs; frames 1+ start their waves in that order
        assert bool(s.schedule & A.SCHED_COST_ORDERED) == (ordered and f > 0), f"frame {f}: schedule {s.schedule}"
        assert s.paths_per_wave == lanes, (f, s.paths_per_wave)
    return check


def test_c2_720p_L3_consecutive_frames(torch_cuda):
    # BASELINE.json configs[1]: 921,600 paths x 2 vertices (>= 1.5M with three frames in flight, r05) -> the
    # depth-split schedule, overlapped
    W, H = 1280, 720
    _steady_frames(torch_cuda, "sponza", W, H, 3, 3, _frame_crops(W, H), expect=_expect(64, False, split=True))


@pytest.mark.parametrize("name", ["sponza", "suntemple"])
def test_metric_1080p_L3_consecutive_frames(torch_cuda, name):
    # the bench's workload (BASELINE.json metric) and configs[3]: 2.07M paths x 2 vertices -> the
    # depth-split schedule (k_path_head + the compacted depth-2 k_path_tail), overlapped, four frames
    W, H = 1920, 1080
    _steady_frames(torch_cuda, name, W, H, 3, 4, _frame_crops(W, H), expect=_expect(64, False, split=True))


@pytest.mark.parametrize("world,rank,lanes,ordered,overlap", [(8, 5, 64, True, 1), (8, 0, 64, True, 1),
                                                              (2, 1, 64, False, 1), (8, 5, 64, True, 0),
                                                              (4, 1, 64, False, 1), (8, 2, 64, True, 3),
                                                              (4, 1, 64, False, 3), (2, 0, 64, False, 3)])
def test_metric_band_share_consecutive_frames(torch_cuda, world, rank, lanes, ordered, overlap):
    # one GPU's share of the metric frame (bench.py --gpus N): 1/8 = 259,200 paths (4,050 waves, one round
    # at 4 waves/SIMD: cost-ordered from its second frame), 1/4 = 518,400 (1.6 rounds at 5 waves/SIMD with
    # two frames in flight: path order, r04),
    # 1/2 = 1,036,800 paths (path order); overlap off: the 1/8 share one frame at a time
    W, H = 1920, 1080
    lay = band_layout(W, H, world)
    # the 1/2 share (2.07M path vertices) runs the depth-split schedule when frames overlap
    _steady_frames(torch_cuda, "sponza", W, H, 3, 3, _band_crops(lay, rank), tiles=lay.rank_tiles(rank),
                   n_out=lay.counts[rank], expect=_expect(lanes, ordered, bool(overlap), split=world == 2 and bool(overlap)),
                   options=((A.OPT_FRAME_OVERLAP, overlap),))


def test_c5_4k_L6_gpu_share_consecutive_frames(torch_cuda):
    # BASELINE.json configs[4]: what each of the 8 GPUs renders -- a 1/8 band share of 3840x2160 at
    # MaxPathLength 6 (1,036,800 paths x 5 vertices: the depth-split schedule) on the default schedule,
    # three consecutive frames
    W, H = 3840, 2160
    lay = band_layout(W, H, 8)
    _steady_frames(torch_cuda, "sponza", W, H, 6, 3, _band_crops(lay, 3, w=96), tiles=lay.rank_tiles(3),
                   n_out=lay.counts[3], expect=_expect(64, False, split=True))


def test_c3_1080p_L8_sixteen_samples(torch_cuda):
    # BASELINE.json configs[2]: "16 spp" = SqrtNumSamples 4 -> CurrSampleIdx 0..15 accumulated into one
    # target through the shipped context (DXRPathTracer.cpp:2027-2028, 2089), compared after every frame
    W, H = 1920, 1080
    crops = [((x0, y0, 48, 48), y0 * W + x0, W) for (x0, y0) in ((0, 0), (936, 516), (1500, 880), (300, 1032))]

    def check(f, s):
        # 2.07M paths x 7 vertices: the depth-split schedule as one part (default by frame size),
        # overlapped with the neighbour frames
        assert s.schedule & A.SCHED_MEGAKERNEL and s.paths_per_wave == 64, (f, s.schedule, s.paths_per_wave)
        assert s.schedule & A.SCHED_SPLIT, (f, s.schedule)
        assert s.schedule & A.SCHED_OVERLAP, (f, s.schedule)

    _steady_frames(torch_cuda, "sponza", W, H, 8, 16, crops, expect=check)


@pytest.mark.parametrize("W,H,L,frames,share", [(1280, 720, 3, 20, None), (1920, 1080, 3, 20, (8, 5)),
                                                (1920, 1080, 3, 6, None), (1920, 1080, 4, 18, (4, 1)),
                                                (1920, 1080, 8, 5, None), (3840, 2160, 6, 3, None),
                                                (1920, 1080, 8, 5, (2, 1))])
def test_overlapped_frames_are_bit_identical(torch_cuda, W, H, L, frames, share):
    # DXRPT_OPT_FRAME_OVERLAP: back-to-back frames (no host sync between them, as bench.py and every rank
    # render them) rotate over two or three sets of internal streams and stage their radiance; the caller's
    # stream blends each stage in frame order (RayTrace.hlsl:140-148).  (Cost-order rebuilds with frames in
    # flight: test_overlapped_order_rebuilds_are_bit_identical.) 1080p L=3 and L=8 and
    # 4K L=6 run the depth-split schedule overlapped against k_path / the split one frame at a time.  The
    # accumulated target must equal the one-frame-at-a-time schedule's bit for bit.
    torch = torch_cuda
    sc, sky = scene_bundle("sponza")
    st = sc.settings(MaxPathLength=L)
    lights = D.make_lights(sc)
    tiles, n = None, W * H
    if share is not None:
        lay = band_layout(W, H, share[0])
        tiles, n = lay.tile_array(share[1]), lay.counts[share[1]]
    consts = [D.make_constants(sc, st, sky, W, H, f % 16) for f in range(frames)]
    stream = torch.cuda.current_stream().cuda_stream
    out = []
    for overlap in (0, 1, 2, 3):  # one frame at a time, two / three frames in flight, by frame size (default)
        t = _fresh("sponza")
        try:
            t.set_option(A.OPT_FRAME_OVERLAP, overlap)
            acc = torch.full((n, 4), 0.5, dtype=torch.float32, device="cuda")
            for f in range(frames):
                t.render_raw(consts[f], st, acc.data_ptr(), W, H, tiles=tiles, stream=stream, lights=lights)
            torch.cuda.synchronize()
            s = t.stats()
            assert bool(s.schedule & A.SCHED_OVERLAP) == bool(overlap), s.schedule
            out.append(acc.cpu().numpy())
        finally:
            t.close()
    for o in out[1:]:
        np.testing.assert_array_equal(o, out[0])


@pytest.mark.parametrize("overlap,period", [(2, 1), (2, 2), (1, 1), (3, 2)])
def test_overlapped_order_rebuilds_are_bit_identical(torch_cuda, overlap, period):
    # a cost-order rebuild (launch_wave_order at the end of an ordered frame) must be seen by
    # the next frame of EVERY slot -- with three frames in flight frame f+2 runs on a third stream.  A 1/8
    # band share (cost-ordered), rebuilds every 1 or 2 frames, 24 frames back to back with no host sync,
    # equals the same frames one at a time bit for bit (a torn permutation would run some waves twice and
    # blend others' stale stage pixels)
    torch = torch_cuda
    W, H, L, frames = 1920, 1080, 3, 24
    sc, sky = scene_bundle("sponza")
    st = sc.settings(MaxPathLength=L)
    lights = D.make_lights(sc)
    lay = band_layout(W, H, 8)
    tiles, n = lay.tile_array(3), lay.counts[3]
    consts = [D.make_constants(sc, st, sky, W, H, f % 16) for f in range(frames)]
    stream = torch.cuda.current_stream().cuda_stream
    out = []
    for ov in (0, overlap):
        t = _fresh("sponza")
        try:
            t.set_option(A.OPT_FRAME_OVERLAP, ov)
            t.set_option(A.OPT_WAVE_ORDER, 1)
            t.set_option(A.OPT_WAVE_ORDER_PERIOD, period)
            acc = torch.full((n, 4), 0.5, dtype=torch.float32, device="cuda")
            for f in range(frames):
                t.render_raw(consts[f], st, acc.data_ptr(), W, H, tiles=tiles, stream=stream, lights=lights)
            torch.cuda.synchronize()
            s = t.stats()
            assert s.schedule & A.SCHED_COST_ORDERED, s.schedule
            assert bool(s.schedule & A.SCHED_OVERLAP) == bool(ov), s.schedule
            out.append(acc.cpu().numpy())
        finally:
            t.close()
    np.testing.assert_array_equal(out[1], out[0])


def _frames(torch, W, H, L, frames, overlap, streams=None, between=None, name="sponza", lights_of=None):
    """`frames` back-to-back frames into one target through a fresh context with DXRPT_OPT_FRAME_OVERLAP
    `overlap`, no host sync between them: frame f on streams[f % len(streams)] (torch streams; default the
    current one), between(t, f) called before frame f, lights_of(f) the frame's (rtc.NumLights, lights)."""
    sc, sky = scene_bundle(name)
    st = sc.settings(MaxPathLength=L)
    t = _fresh(name)
    try:
        t.set_option(A.OPT_FRAME_OVERLAP, overlap)
        acc = torch.full((W * H, 4), 0.5, dtype=torch.float32, device="cuda")
        streams = streams or [torch.cuda.current_stream()]
        for st_ in streams:  # the target was written on the current stream
            st_.wait_stream(torch.cuda.current_stream())
        for f in range(frames):
            if between is not None:
                between(t, f)
            rtc = D.make_constants(sc, st, sky, W, H, f % 16)
            lights = D.make_lights(sc)
            if lights_of is not None:
                rtc.NumLights, lights = lights_of(f, sc, lights)
            t.render_raw(rtc, st, acc.data_ptr(), W, H, stream=streams[f % len(streams)].cuda_stream, lights=lights)
        torch.cuda.synchronize()
        return acc.cpu().numpy(), t.stats()
    finally:
        t.close()


@pytest.mark.parametrize("W,H,L,overlap", [(1280, 720, 3, 1), (1920, 1080, 3, 1), (320, 180, 5, 1), (1920, 1080, 3, 3),
                                           (320, 180, 5, 2)])
def test_overlapped_frames_on_alternating_streams(torch_cuda, W, H, L, overlap):
    # include/dxrpt.h "Stream ordering": a caller that submits consecutive frames on two streams (a ring of
    # command queues) still gets the frames in submission order -- each call on a new stream first waits
    # for the previous stream -- so the progressive blend (order dependent) equals the one-stream,
    # one-frame-at-a-time result bit for bit, over >= 6 frames (1080p: the depth-split schedule)
    torch = torch_cuda
    ref, _ = _frames(torch, W, H, L, 8, 0)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    got, s = _frames(torch, W, H, L, 8, overlap, streams=streams)
    assert s.schedule & A.SCHED_OVERLAP, s.schedule
    np.testing.assert_array_equal(got, ref)
    got0, _ = _frames(torch, W, H, L, 8, 0, streams=streams)
    np.testing.assert_array_equal(got0, ref)


def test_census_frame_between_overlapped_frames(torch_cuda):
    # a non-overlapped frame (here a census frame, DXRPT_OPT_COUNT_TRAVERSAL) between
    # overlapped frames, with no host sync, runs after them and before the next one (it shares the BVH8
    # stack-spill slab and, through the stream, the target): the frames equal the one-at-a-time result
    torch = torch_cuda
    W, H = 1920, 1080

    def census_on_3(t, f):
        t.set_option(A.OPT_COUNT_TRAVERSAL, 1 if f in (3, 4) else 0)

    ref, _ = _frames(torch, W, H, 3, 8, 0)
    got, s = _frames(torch, W, H, 3, 8, 1, between=census_on_3)
    np.testing.assert_array_equal(got, ref)
    got2, _ = _frames(torch, 1280, 720, 3, 8, 1, between=census_on_3)
    ref2, _ = _frames(torch, 1280, 720, 3, 8, 0)
    np.testing.assert_array_equal(got2, ref2)


@pytest.mark.parametrize("name,W,H", [("boxtest", 256, 256), ("sponza", 640, 360)])
def test_light_count_changes_between_overlapped_frames(torch_cuda, name, W, H):
    # frames in flight with different shadow-slot counts (spot lights toggled between frames)
    # keep their own buffers and stack-spill slabs: equal to the one-frame-at-a-time result
    torch = torch_cuda
    import math

    def lights_of(f, sc, lights):
        n = (0, 2, 3, 0, 1, 3, 2, 0)[f % 8]
        for i in range(3):
            L = lights.Lights[i]
            p, d = [((1.5, 4.0, -2.0), (-0.3, -1.0, 0.4)), ((-2.5, 1.5, -1.5), (0.8, -0.2, 0.5)),
                    ((0.5, 3.0, 2.0), (0.0, -1.0, -0.2))][i]
            nn = math.sqrt(sum(x * x for x in d))
            L.Position[:] = p
            L.Direction[:] = tuple(-x / nn for x in d)
            L.Intensity[:] = (50.0, 45.0, 37.5)
            L.AngularAttenuationX, L.AngularAttenuationY, L.Range = math.cos(0.3), math.cos(0.6), 7.5
        return n, lights

    ref, _ = _frames(torch, W, H, 4, 8, 0, name=name, lights_of=lights_of)
    got, _ = _frames(torch, W, H, 4, 8, 1, name=name, lights_of=lights_of)
    np.testing.assert_array_equal(got, ref)
