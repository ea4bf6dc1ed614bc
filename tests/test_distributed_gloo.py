"""CPU, world_size 2 (gloo): the multi-GPU path's partition + frame-end gather + un-permute.

Each rank renders only its row bands (here with the CPU oracle standing in for the HIP kernel, which
tests/test_gpu_parity.py checks separately with the same tiles) into a compact slab; rank 0 gathers
the slabs and must reproduce the single-rank frame bit for bit, because CMJ seeds use global pixel
indices (RayTrace.hlsl:85-96)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, H, q, kind="bands"):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import dxrpathtracer_amd as D
        from dxrpathtracer_amd.distributed import gather_frame, screen_layout, source_index
        from tests._common import oracle_scene, scene_bundle
        sc, sky = scene_bundle("boxtest")
        st = sc.settings(MaxPathLength=3)
        rtc = D.make_constants(sc, st, sky, W, H, 1)
        lay = screen_layout(W, H, world, kind)
        local = np.zeros((lay.max_count, 4), dtype=np.float32)
        orc = oracle_scene("boxtest")
        for t in lay.rank_tiles(rank):
            img, _ = orc.render(rtc, st, D.make_lights(sc), W, H, crop=(t.x0, t.y0, t.w, t.h))
            local[t.accum_offset:t.accum_offset + t.w * t.h] = img.reshape(-1, 4)
        full = torch.zeros((W * H, 4), dtype=torch.float32) if rank == 0 else None
        idx = torch.tensor(source_index(lay), dtype=torch.long) if rank == 0 else None
        gather_frame(torch.from_numpy(local), lay, rank, full, idx)
        if rank == 0:
            ref, _ = orc.render(rtc, st, D.make_lights(sc), W, H)
            q.put(bool(np.array_equal(full.numpy().reshape(H, W, 4), ref)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,kind", [(2, "bands"), (2, "blocks"), (3, "blocks")])
def test_band_gather_reproduces_single_rank_frame(world, kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    W, H = 52, 76  # 10 bands of 8 rows / 7 x 10 blocks of 8 x 8, the last row and column partial
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, q, kind)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    assert q.get(timeout=10) is True


def _worker_pipelined(rank, world, port, W, H, q):
    # PipelinedGather over 3 frames with different slab contents: after submit(f+1) rank 0's frame
    # buffer holds frame f exactly; after flush() the last frame
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dxrpathtracer_amd.distributed import PipelinedGather, screen_layout, source_index
        lay = screen_layout(W, H, world, "blocks")
        full = torch.zeros((W * H, 4), dtype=torch.float32) if rank == 0 else None
        idx = torch.tensor(source_index(lay), dtype=torch.long) if rank == 0 else None
        pg = PipelinedGather(lay, rank, full, idx)

        def frame_image(f):  # the full frame every rank "renders" its bands of, frame f
            return (np.arange(W * H * 4, dtype=np.float32).reshape(H, W, 4) + 1000.0 * f)

        local = torch.zeros((lay.max_count, 4), dtype=torch.float32)
        ok = True
        for f in range(3):
            img = frame_image(f)
            for t in lay.rank_tiles(rank):
                local[t.accum_offset:t.accum_offset + t.w * t.h] = torch.from_numpy(
                    img[t.y0:t.y0 + t.h, t.x0:t.x0 + t.w].reshape(-1, 4))
            pg.submit(local)
            local.fill_(-1.0)  # the next frame overwrites the accumulation buffer: the snapshot must hold
            if rank == 0 and f > 0:
                ok &= bool(np.array_equal(full.numpy().reshape(H, W, 4), frame_image(f - 1)))
        pg.flush()
        if rank == 0:
            ok &= bool(np.array_equal(full.numpy().reshape(H, W, 4), frame_image(2)))
            q.put(ok)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_pipelined_gather_delivers_every_frame(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    W, H = 40, 56
    procs = [ctx.Process(target=_worker_pipelined, args=(r, world, port, W, H, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    assert q.get(timeout=10) is True


def test_band_partition_is_balanced():
    # 8-row bands at the metric's 1920x1080: every rank within 1 % of the mean pixel count at 2, 4, 8 ranks
    # (pixel balance only: the band height itself is chosen by the slowest rank's measured share time,
    # distributed.BAND_ROWS)
    from dxrpathtracer_amd.distributed import band_layout
    for world in (2, 4, 8):
        lay = band_layout(1920, 1080, world)
        assert sum(lay.counts) == 1920 * 1080
        assert max(lay.counts) <= 1.01 * (1920 * 1080 / world), (world, lay.counts)
        assert all(t.h % 8 == 0 for r in range(world) for t in lay.rank_tiles(r))


def test_block_partition_covers_image_and_spreads_rows():
    # the block partition (--layout blocks; bands are the default): every pixel exactly once, equal block counts, each rank's blocks drawn
    # from (nearly) every block row, so clustered expensive rows (foliage) are shared by all ranks
    from dxrpathtracer_amd.distributed import block_layout, source_index
    for W, H, world in ((1920, 1080, 8), (1920, 1080, 2), (1366, 767, 3), (64, 8, 8)):
        lay = block_layout(W, H, world)
        idx = source_index(lay)
        assert sorted(idx) == sorted(set(idx)) and len(idx) == W * H
        nblocks = [len(lay.rank_tiles(r)) for r in range(world)]
        assert max(nblocks) - min(nblocks) <= 1
        again = block_layout(W, H, world)  # deterministic
        key = lambda L: [[(t.x0, t.y0, t.w, t.h, t.accum_offset) for t in L.rank_tiles(r)] for r in range(world)]
        assert key(lay) == key(again)
    lay = block_layout(1920, 1080, 8)
    for r in range(8):
        rows = {t.y0 // 8 for t in lay.rank_tiles(r)}
        assert len(rows) >= 0.95 * 135


def test_tile_array_matches_rank_tiles():
    # BandLayout.tile_array: the ctypes array render_raw passes straight to dxrpt_render (built once)
    from dxrpathtracer_amd.distributed import band_layout, block_layout, gathered_tiles
    for lay in (band_layout(1920, 1080, 8), block_layout(333, 187, 3)):
        for r in range(lay.world):
            arr = lay.tile_array(r)
            assert arr is lay.tile_array(r)
            got = [(t.x0, t.y0, t.w, t.h, t.accum_offset, t.accum_pitch) for t in arr]
            want = [(t.x0, t.y0, t.w, t.h, t.accum_offset, t.accum_pitch) for t in lay.rank_tiles(r)]
            assert got == want
        # dxrpt_unpermute's list: every rank's tiles, offsets moved to the rank's slab in the gathered buffer
        gt = gathered_tiles(lay)
        assert len(gt) == sum(len(lay.rank_tiles(r)) for r in range(lay.world))
        assert sum(t.w * t.h for t in gt) == lay.width * lay.height
        ends = sorted((t.accum_offset, t.accum_offset + t.h * t.accum_pitch) for t in gt)
        assert ends[0][0] == 0 and all(a[1] <= b[0] for a, b in zip(ends, ends[1:]))


def _worker_native_fail(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dxrpathtracer_amd.distributed import NativeGather, band_layout
        try:
            NativeGather(band_layout(64, 32, world), rank, 0, None)
            q.put((rank, "built"))
        except RuntimeError as e:
            q.put((rank, "raised", str(e)[:200]))
    finally:
        dist.destroy_process_group()


@pytest.mark.skipif(torch.cuda.is_available(), reason="needs a host without a usable GPU (the RCCL communicator must fail)")
def test_native_gather_failure_is_collective():
    # On a host where the RCCL communicator cannot be built, NativeGather raises on EVERY rank (the ranks
    # all-gather their device checks before anything collective in RCCL, rank 0's unique-id failure is
    # broadcast, dxrpt_comm_create's result is all-gathered) instead of leaving the other ranks blocked in
    # the next collective -- so bench.py can fall back to torch.distributed.gather.
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_native_fail, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    got = sorted(q.get(timeout=10) for _ in range(world))
    assert [g[:2] for g in got] == [(r, "raised") for r in range(world)], got
