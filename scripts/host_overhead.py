#!/usr/bin/env python3
"""Host cost per frame of the bench loop (one MI355X): is the Python/ctypes submission of a frame
cheaper than the GPU time of a GPU's share?  A rank of an 8-GPU metric run renders a 1/8 band share
(~0.3-0.36 ms of GPU time) and submits its slab to the frame-end gather every frame; if the host took
longer than that per frame, the N-GPU frame would be host-bound.

Prints, for each case, the wall-clock time of the submission loop per frame (host, before the final
synchronize) and the GPU time per frame (events on the render stream):
  share8      render_raw of the rank's 1/8 band share (rank 2), no gather
  share8+ng   the same plus NativeGather.submit of a slab through a one-rank RCCL communicator
              (dxrpt_gather_slabs + dxrpt_unpermute: the calls rank 0 makes every frame)

    python scripts/host_overhead.py [--frames 64]
"""
import argparse
import os
import socket
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    import dxrpathtracer_amd as D
    from dxrpathtracer_amd.distributed import NativeGather, band_layout
    from dxrpathtracer_amd.tracer import DXRPathTracer

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    W, H, L = 1920, 1080, 3
    sc = D.Scene("sponza")
    st = sc.settings(MaxPathLength=L)
    sky = D.make_sky(st)
    t = DXRPathTracer(0)
    t.initialize_scene(sc, sky)
    t.build_rt_acceleration_structure()
    lights = D.make_lights(sc)
    consts = [D.make_constants(sc, st, sky, W, H, s) for s in range(16)]
    stream = torch.cuda.current_stream()
    lay8 = band_layout(W, H, 8)
    tiles, n = lay8.tile_array(2), lay8.counts[2]
    acc = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
    # a one-rank gather of a slab of the share's size (one rank's calls; the slab is the share's)
    lay1 = band_layout(W, n // W if n % W == 0 else (n + W - 1) // W, 1)
    full = torch.zeros((lay1.counts[0], 4), dtype=torch.float32, device="cuda")
    ng = NativeGather(lay1, 0, 0, full)
    slab = torch.zeros((lay1.counts[0], 4), dtype=torch.float32, device="cuda")

    def run(label, gather):
        for f in range(8):
            t.render_raw(consts[f % 16], st, acc.data_ptr(), W, H, tiles=tiles, stream=stream.cuda_stream, lights=lights)
            if gather:
                ng.submit(slab)
        if gather:
            ng.flush()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        h0 = time.perf_counter()
        for f in range(args.frames):
            t.render_raw(consts[f % 16], st, acc.data_ptr(), W, H, tiles=tiles, stream=stream.cuda_stream, lights=lights)
            if gather:
                ng.submit(slab)
        if gather:
            ng.flush()
        h1 = time.perf_counter()
        b.record(stream)
        torch.cuda.synchronize()
        host = (h1 - h0) / args.frames * 1e3
        gpu = a.elapsed_time(b) / args.frames
        print(f"{label:12s} host {host:.4f} ms/frame  gpu {gpu:.4f} ms/frame  "
              f"({'host-bound' if host > 0.9 * gpu else 'GPU-bound'})", flush=True)

    for _ in range(2):
        run("share8", False)
        run("share8+ng", True)
    ng.close()
    t.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
