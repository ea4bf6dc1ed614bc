#!/usr/bin/env python3
"""Experiment: a frame split into K independent parts (row bands b -> part b % K), each part rendered
by its own context on its own stream, all parts concurrent.  Measures whether the parts' passes fill
each other's tails (ms/frame vs the one-context frame).  Sponza proxy 1920x1080 L=3.

    python scripts/ab_split.py [--frames 32] [--parts 1,2,3,4]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--parts", default="1,2,3,4")
    ap.add_argument("--shards", default="", help="also time rank 0's band share of an N-way split, e.g. 2,4,8")
    ap.add_argument("--share-parts", default="2,4", help="rank 0's share split into k concurrent parts")
    ap.add_argument("--config", default="metric", choices=["metric", "c2", "c3", "c4", "c5"])
    ap.add_argument("--msplit", type=int, default=None, help="DXRPT_OPT_MEGAKERNEL_SPLIT for every context")
    ap.add_argument("--occ", type=int, default=None)
    ap.add_argument("--tail-occ", type=int, default=None)
    ap.add_argument("--wave-order", type=int, default=None)
    ap.add_argument("--part-layout", default="bands", choices=["bands", "halves"],
                    help="parts = interleaved 8-row bands, or contiguous row ranges")
    args = ap.parse_args()
    import torch
    import dxrpathtracer_amd as D
    from dxrpathtracer_amd.distributed import band_layout
    from dxrpathtracer_amd.tracer import DXRPathTracer

    import dxrpathtracer_amd._abi as A
    name, W, H, L = {"metric": ("sponza", 1920, 1080, 3), "c2": ("sponza", 1280, 720, 3), "c3": ("sponza", 1920, 1080, 8),
                     "c4": ("suntemple", 1920, 1080, 3), "c5": ("sponza", 3840, 2160, 6)}[args.config]
    sc = D.Scene(name)
    st = sc.settings(MaxPathLength=L)
    sky = D.make_sky(st)
    lights = D.make_lights(sc)
    consts = [D.make_constants(sc, st, sky, W, H, s) for s in range(16)]
    kmax = max(int(k) for k in args.parts.split(","))
    tracers = []
    for _ in range(kmax):
        t = DXRPathTracer(0)
        for opt, v in ((A.OPT_MEGAKERNEL_SPLIT, args.msplit), (A.OPT_MEGAKERNEL_OCCUPANCY, args.occ),
                       (A.OPT_TAIL_OCCUPANCY, args.tail_occ), (A.OPT_WAVE_ORDER, args.wave_order)):
            if v is not None:
                t.set_option(opt, v)
        t.initialize_scene(sc, sky)
        t.build_rt_acceleration_structure()
        tracers.append(t)
    main_s = torch.cuda.current_stream()
    streams = [torch.cuda.Stream() for _ in range(kmax)]
    res = {}
    for rnd in range(args.rounds):
        for k in (int(x) for x in args.parts.split(",")):
            lay = band_layout(W, H, k)
            if args.part_layout == "halves" and k > 1:  # contiguous row ranges (multiples of 8 rows)
                rows = [((H // 8) * r // k) * 8 for r in range(k)] + [H]
                lay.tiles = [[A.Tile(0, rows[r], W, rows[r + 1] - rows[r], 0, W, 0)] for r in range(k)]
                lay.counts = [W * (rows[r + 1] - rows[r]) for r in range(k)]
            accs = [torch.zeros((max(1, lay.counts[r]), 4), dtype=torch.float32, device="cuda") for r in range(k)]

            def frame(f):
                if k == 1:
                    tracers[0].render_raw(consts[f % 16], st, accs[0].data_ptr(), W, H, stream=main_s.cuda_stream,
                                          lights=lights)
                    return
                for r in range(k):
                    streams[r].wait_stream(main_s)
                    tracers[r].render_raw(consts[f % 16], st, accs[r].data_ptr(), W, H, tiles=lay.rank_tiles(r),
                                          stream=streams[r].cuda_stream, lights=lights)
                for r in range(k):
                    main_s.wait_stream(streams[r])

            for f in range(4):
                frame(f)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for f in range(args.frames):
                frame(f)
            torch.cuda.synchronize()
            res.setdefault(k, []).append((time.perf_counter() - t0) / args.frames * 1e3)
    for k, v in res.items():
        print(f"{args.config} {args.part_layout} msplit={args.msplit} occ={args.occ}/{args.tail_occ} order={args.wave_order} parts {k}: ms/frame " + " ".join(f"{x:.3f}" for x in v) + f"  min {min(v):.3f}")
    # one rank's share of an N-GPU frame (what each GPU renders at N GPUs, before the gather)
    for n in (int(x) for x in args.shards.split(",") if x):
        lay = band_layout(W, H, n)
        acc = torch.zeros((lay.counts[0], 4), dtype=torch.float32, device="cuda")
        ts = []
        for rnd in range(args.rounds):
            for f in range(4):
                tracers[0].render_raw(consts[f % 16], st, acc.data_ptr(), W, H, tiles=lay.rank_tiles(0),
                                      stream=main_s.cuda_stream, lights=lights)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for f in range(args.frames):
                tracers[0].render_raw(consts[f % 16], st, acc.data_ptr(), W, H, tiles=lay.rank_tiles(0),
                                      stream=main_s.cuda_stream, lights=lights)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) / args.frames * 1e3)
        print(f"rank-0 share of {n} GPUs ({lay.counts[0]} px): ms/frame {min(ts):.3f}  "
              f"(ideal {res.get(1, [float('nan')])[0] / n:.3f})")
        import dxrpathtracer_amd._abi as A
        t = tracers[0]
        t.set_option(A.OPT_KERNEL_TIMING, 1)
        t.reset_timing()
        for f in range(args.frames):
            t.render_raw(consts[f % 16], st, acc.data_ptr(), W, H, tiles=lay.rank_tiles(0), stream=main_s.cuda_stream,
                         lights=lights)
        torch.cuda.synchronize()
        s_ = t.stats()
        t.set_option(A.OPT_KERNEL_TIMING, 0)
        nf = max(1, s_.timed_frames)
        print("   per frame (events): span %.3f ms; " % (s_.frame_ms / nf) + ", ".join(
            f"{A.KERNEL_NAMES[k]} {s_.kernel_ms[k] / nf:.3f} ({s_.kernel_launches[k] // nf}x)" for k in range(A.K_COUNT)))
        # the share split into k concurrent parts (tile i -> part i % k), one context + stream each
        for k in (int(x) for x in args.share_parts.split(",") if x):
            if k > kmax:
                continue
            parts = [[] for _ in range(k)]
            offs = [0] * k
            for i, tl in enumerate(lay.rank_tiles(0)):
                r = i % k
                parts[r].append(A.Tile(tl.x0, tl.y0, tl.w, tl.h, offs[r], tl.w, 0))
                offs[r] += tl.w * tl.h
            accs = [torch.zeros((max(1, offs[r]), 4), dtype=torch.float32, device="cuda") for r in range(k)]

            def frame(f):
                for r in range(k):
                    streams[r].wait_stream(main_s)
                    tracers[r].render_raw(consts[f % 16], st, accs[r].data_ptr(), W, H, tiles=parts[r],
                                          stream=streams[r].cuda_stream, lights=lights)
                for r in range(k):
                    main_s.wait_stream(streams[r])
            ts = []
            for rnd in range(args.rounds):
                for f in range(4):
                    frame(f)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for f in range(args.frames):
                    frame(f)
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) / args.frames * 1e3)
            print(f"   share of {n} GPUs in {k} concurrent parts: ms/frame {min(ts):.3f}")
    for t in tracers:
        t.close()


if __name__ == "__main__":
    main()
