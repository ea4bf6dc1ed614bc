"""GPU: the multi-GPU frame behind the C ABI -- dxrpt_unpermute against the partition's
source_index, and the RCCL gather path (dxrpt_comm_create / dxrpt_gather_slabs / dxrpt_unpermute through
distributed.NativeGather) on a one-rank communicator, which must reproduce the single-GPU frame bit for
bit.  More ranks need more GPUs: the N-GPU runs are the driver's (bench.py --gpus N)."""
import ctypes as C
import os
import socket

import numpy as np
import pytest

import dxrpathtracer_amd as D
import dxrpathtracer_amd._abi as A
from dxrpathtracer_amd.distributed import NativeGather, band_layout, block_layout, gathered_tiles, source_index
from dxrpathtracer_amd.tracer import DXRPathTracer
from tests._common import scene_bundle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind,W,H,world", [("bands", 1920, 1080, 8), ("blocks", 333, 187, 3), ("bands", 100, 50, 2)])
def test_unpermute_matches_source_index(torch_cuda, kind, W, H, world):
    torch = torch_cuda
    lay = (band_layout if kind == "bands" else block_layout)(W, H, world)
    rng = np.random.default_rng(7)
    slabs = [rng.standard_normal((lay.counts[r], 4)).astype(np.float32) for r in range(world)]
    gathered = np.concatenate(slabs)
    # expected frame from source_index (rank r's slab at r * max_count in the padded layout)
    padded = np.zeros((world * lay.max_count, 4), np.float32)
    for r in range(world):
        padded[r * lay.max_count:r * lay.max_count + lay.counts[r]] = slabs[r]
    want = padded[np.array(source_index(lay))]
    tiles = gathered_tiles(lay)
    tarr = (A.Tile * len(tiles))(*tiles)
    src = torch.from_numpy(gathered).cuda()
    dst = torch.full((W * H, 4), -7.0, dtype=torch.float32, device="cuda")
    rc = A.lib().dxrpt_unpermute(C.c_void_p(src.data_ptr()), tarr, len(tiles), C.c_void_p(dst.data_ptr()), W, H,
                                 C.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, A.lib().dxrpt_multi_last_error()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dst.cpu().numpy(), want)
    # a tile outside the frame is rejected before any launch
    bad = (A.Tile * 1)(A.Tile(W - 4, 0, 8, 1, 0, 8, 0))
    assert A.lib().dxrpt_unpermute(C.c_void_p(src.data_ptr()), bad, 1, C.c_void_p(dst.data_ptr()), W, H, None) != 0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_native_gather_one_rank_equals_full_frame(torch_cuda):
    torch = torch_cuda
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        W, H = 480, 270
        sc, sky = scene_bundle("sponza")
        st = sc.settings(MaxPathLength=3)
        lay = band_layout(W, H, 1)
        t = DXRPathTracer(0)
        t.initialize_scene(sc, sky)
        t.build_rt_acceleration_structure()
        stream = torch.cuda.current_stream().cuda_stream
        lights = D.make_lights(sc)
        ref = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
        slab = torch.zeros((lay.counts[0], 4), dtype=torch.float32, device="cuda")
        full = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
        ng = NativeGather(lay, 0, 0, full)
        frames = []
        for f in range(3):
            rtc = D.make_constants(sc, st, sky, W, H, f)
            t.render_raw(rtc, st, ref.data_ptr(), W, H, stream=stream, lights=lights)
            t.render_raw(rtc, st, slab.data_ptr(), W, H, tiles=lay.rank_tiles(0), stream=stream, lights=lights)
            ng.submit(slab)
            frames.append(ref.clone())
            if f:  # frame f - 1 is complete in `full` once frame f was submitted
                torch.cuda.synchronize()
                np.testing.assert_array_equal(full.cpu().numpy(), frames[f - 1].cpu().numpy())
        ng.flush()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(full.cpu().numpy(), frames[-1].cpu().numpy())
        ng.close()
        t.close()
    finally:
        dist.destroy_process_group()
