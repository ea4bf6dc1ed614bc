#!/usr/bin/env python3
"""ms/frame of the default (shipped) schedule on a BASELINE config, for A/B of kernel builds
(DXRPT_KERNEL_LIB_DIR picks the libdxrpt.so).  Prints one line: label, median and mean ms/frame of
`--rounds` x `--frames` frames (HIP events on the render stream), counted rays per frame.

    python scripts/time_frames.py [--label x] [--config metric|c2|c3|c4|c5] [--share N --rank r]
"""
import argparse
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
CONFIGS = {"metric": ("sponza", 1920, 1080, 3), "c2": ("sponza", 1280, 720, 3), "c3": ("sponza", 1920, 1080, 8),
           "c4": ("suntemple", 1920, 1080, 3), "c5": ("sponza", 3840, 2160, 6)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--label", default=os.environ.get("DXRPT_KERNEL_LIB_DIR", "default"))
    ap.add_argument("--config", default="metric", choices=sorted(CONFIGS))
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--share", type=int, default=1)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--layout", default="bands", choices=["blocks", "bands", "blocks-raster", "blocks-lpt", "bands-balanced"],
                    help="screen partition of --share (blocks-raster: 8x8 tiles in raster order, block k -> rank k %% N)")
    ap.add_argument("--any-hit", type=int, default=None, help="MaxAnyHitPathLength override")
    ap.add_argument("--packet", type=int, default=None, help="DXRPT_OPT_PACKET_TRAVERSAL override")
    ap.add_argument("--occ", type=int, default=None, help="DXRPT_OPT_MEGAKERNEL_OCCUPANCY override")
    ap.add_argument("--tile", default=None, help="x,y,w,h: render only this rectangle (one tile)")
    ap.add_argument("--band", type=int, default=None, help="band height of --layout bands (default BAND_ROWS)")
    ap.add_argument("--lanes", type=int, default=None, help="DXRPT_OPT_MEGAKERNEL_LANES override")
    ap.add_argument("--wave-order", type=int, default=None, help="DXRPT_OPT_WAVE_ORDER override")
    ap.add_argument("--split", type=int, default=None, help="DXRPT_OPT_SPLIT_UNITS override (per mille)")
    ap.add_argument("--xcd-chunk", type=int, default=None, help="DXRPT_OPT_XCD_CHUNK override (blocks)")
    ap.add_argument("--mega-paths", type=int, default=None, help="DXRPT_OPT_MEGAKERNEL_PATHS override (path vertices)")
    ap.add_argument("--order-period", type=int, default=None, help="DXRPT_OPT_WAVE_ORDER_PERIOD override (frames)")
    ap.add_argument("--msplit", type=int, default=None, help="DXRPT_OPT_MEGAKERNEL_SPLIT override (0 off, 1 on, 2 by size)")
    ap.add_argument("--tail-occ", type=int, default=None, help="DXRPT_OPT_TAIL_OCCUPANCY override")
    ap.add_argument("--omm", type=int, default=None, help="DXRPT_OPT_OPACITY_MICROMAP override")
    ap.add_argument("--overlap", type=int, default=None, help="DXRPT_OPT_FRAME_OVERLAP override (0 off, 1 two frames in flight, 2 three)")
    ap.add_argument("--leaf-cost", type=int, default=None, help="DXRPT_OPT_LEAF_COST before the BVH build (percent)")
    ap.add_argument("--spatial", type=int, default=None, help="DXRPT_OPT_SPATIAL_SPLITS before the BVH build (percent)")
    ap.add_argument("--split-alpha", type=int, default=None, help="DXRPT_OPT_SPLIT_ALPHA before the BVH build")
    ap.add_argument("--bins", type=int, default=None, help="DXRPT_OPT_SPLIT_BINS override (split frames)")
    ap.add_argument("--parts", type=int, default=None, help="DXRPT_OPT_SPLIT_PARTS override (split frames)")
    ap.add_argument("--max-path", type=int, default=None, help="MaxPathLength override (a cost breakdown by depth)")
    ap.add_argument("--phases", action="store_true",
                    help="print the per-phase lane-time split of the timed frames (kernel builds with -DDXRPT_DIAG_PHASES=1)")
    args = ap.parse_args()
    import torch
    import dxrpathtracer_amd as D
    from dxrpathtracer_amd.distributed import screen_layout
    from dxrpathtracer_amd.tracer import DXRPathTracer

    name, W, H, L = CONFIGS[args.config]
    L = L if args.max_path is None else args.max_path
    sc = D.Scene(name)
    st = sc.settings(MaxPathLength=L, **({} if args.any_hit is None else {"MaxAnyHitPathLength": args.any_hit}))
    sky = D.make_sky(st)
    t = DXRPathTracer(0)
    import dxrpathtracer_amd._abi as A
    if args.packet is not None:
        t.set_option(A.OPT_PACKET_TRAVERSAL, args.packet)
    if args.occ is not None:
        t.set_option(A.OPT_MEGAKERNEL_OCCUPANCY, args.occ)
    if args.wave_order is not None:
        t.set_option(A.OPT_WAVE_ORDER, args.wave_order)
    if args.lanes is not None:
        t.set_option(A.OPT_MEGAKERNEL_LANES, args.lanes)
    if args.split is not None:
        t.set_option(A.OPT_SPLIT_UNITS, args.split)
    if args.xcd_chunk is not None:
        t.set_option(A.OPT_XCD_CHUNK, args.xcd_chunk)
    if args.mega_paths is not None:
        t.set_option(A.OPT_MEGAKERNEL_PATHS, args.mega_paths)
    if args.order_period is not None:
        t.set_option(A.OPT_WAVE_ORDER_PERIOD, args.order_period)
    if args.msplit is not None:
        t.set_option(A.OPT_MEGAKERNEL_SPLIT, args.msplit)
    if args.tail_occ is not None:
        t.set_option(A.OPT_TAIL_OCCUPANCY, args.tail_occ)
    if args.omm is not None:
        t.set_option(A.OPT_OPACITY_MICROMAP, args.omm)
    if args.overlap is not None:
        t.set_option(A.OPT_FRAME_OVERLAP, args.overlap)
    if args.parts is not None:
        t.set_option(A.OPT_SPLIT_PARTS, args.parts)
    if args.bins is not None:
        t.set_option(A.OPT_SPLIT_BINS, args.bins)
    if args.leaf_cost is not None:
        t.set_option(A.OPT_LEAF_COST, args.leaf_cost)
    if args.spatial is not None:
        t.set_option(A.OPT_SPATIAL_SPLITS, args.spatial)
    if args.split_alpha is not None:
        t.set_option(A.OPT_SPLIT_ALPHA, args.split_alpha)
    t.initialize_scene(sc, sky)
    t.build_rt_acceleration_structure()
    tiles, n = None, W * H
    if args.tile:
        from dxrpathtracer_amd import _abi as AA
        x, y, w, h = (int(v) for v in args.tile.split(","))
        tiles, n = [AA.Tile(x, y, w, h, 0, w, 0)], w * h
    elif args.layout == "blocks-lpt":  # 8x8 block tiles, costliest first (one census frame's wave clocks)
        from dxrpathtracer_amd import _abi as AA
        import numpy as np
        acc0 = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
        t.set_option(A.OPT_COUNT_TRAVERSAL, 1)
        t.set_option(A.OPT_WAVE_CLOCKS, 1)
        t.render_raw(D.make_constants(sc, st, sky, W, H, 0), st, acc0.data_ptr(), W, H,
                     stream=torch.cuda.current_stream().cuda_stream, lights=D.make_lights(sc))
        torch.cuda.synchronize()
        wc = t.wave_clocks().astype(np.int64)
        t.set_option(A.OPT_WAVE_CLOCKS, 0)
        t.set_option(A.OPT_COUNT_TRAVERSAL, 0)
        bw = (W + 7) // 8
        order = np.argsort(-(wc[:, 1] - wc[:, 0]), kind="stable")  # wave w of the full frame = block w
        tiles = [AA.Tile(int(b % bw) * 8, int(b // bw) * 8, 8, 8, 64 * k, 8, 0) for k, b in enumerate(order)]
        n = 64 * len(tiles)
        tiles = (AA.Tile * len(tiles))(*tiles)
    elif args.layout == "blocks-raster":  # the whole frame as 8x8 block tiles in raster order (tile-count A/B)
        from dxrpathtracer_amd import _abi as AA
        tiles = [AA.Tile(x, y, 8, 8, (y // 8 * (W // 8) + x // 8) * 64, 8, 0) for y in range(0, H, 8) for x in range(0, W, 8)]
        if args.share > 1:
            tiles = tiles[args.rank::args.share]
            tiles = [AA.Tile(t.x0, t.y0, 8, 8, 64 * k, 8, 0) for k, t in enumerate(tiles)]
        n = 64 * len(tiles)
        tiles = (AA.Tile * len(tiles))(*tiles)
    elif args.layout == "bands-balanced" and args.share > 1:  # bands dealt by one census frame's costs
        import numpy as np
        from dxrpathtracer_amd.distributed import balanced_band_layout, band_costs_from_wave_clocks
        acc0 = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
        t.set_option(A.OPT_COUNT_TRAVERSAL, 1)
        t.set_option(A.OPT_WAVE_CLOCKS, 1)
        t.render_raw(D.make_constants(sc, st, sky, W, H, 0), st, acc0.data_ptr(), W, H,
                     stream=torch.cuda.current_stream().cuda_stream, lights=D.make_lights(sc))
        torch.cuda.synchronize()
        costs = band_costs_from_wave_clocks(W, H, t.wave_clocks())
        t.set_option(A.OPT_WAVE_CLOCKS, 0)
        t.set_option(A.OPT_COUNT_TRAVERSAL, 0)
        lay = balanced_band_layout(W, H, args.share, costs)
        tiles, n = lay.tile_array(args.rank), lay.counts[args.rank]
    elif args.share > 1:
        from dxrpathtracer_amd.distributed import band_layout
        lay = (band_layout(W, H, args.share, args.band) if args.layout == "bands" and args.band
               else screen_layout(W, H, args.share, args.layout))
        tiles, n = lay.tile_array(args.rank), lay.counts[args.rank]
    acc = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
    consts = [D.make_constants(sc, st, sky, W, H, s) for s in range(16)]
    lights = D.make_lights(sc)
    stream = torch.cuda.current_stream()
    for f in range(5):
        t.render_raw(consts[f % 16], st, acc.data_ptr(), W, H, tiles=tiles, stream=stream.cuda_stream, lights=lights)
    torch.cuda.synchronize()
    if args.phases:
        t.phase_clocks()  # zero the sums of the warm-up frames
    rounds = []
    for r in range(args.rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for f in range(args.frames):
            t.render_raw(consts[f % 16], st, acc.data_ptr(), W, H, tiles=tiles, stream=stream.cuda_stream, lights=lights)
        b.record(stream)
        torch.cuda.synchronize()
        rounds.append(a.elapsed_time(b) / args.frames)
    s = t.stats()
    print(f"{args.label:24s} {args.config}{'' if args.max_path is None else f' L={L}'}{'' if args.wave_order is None else f' order={args.wave_order}'}{'' if args.split is None else f' split={args.split}'}{'' if args.xcd_chunk is None else f' xcd={args.xcd_chunk}'}{'' if args.mega_paths is None else f' mega={args.mega_paths}'}{'' if args.order_period is None else f' period={args.order_period}'}{'' if args.msplit is None else f' msplit={args.msplit}'}{'' if args.occ is None else f' occ={args.occ}'}{'' if args.tail_occ is None else f' tocc={args.tail_occ}'}{'' if args.omm is None else f' omm={args.omm}'}{'' if args.overlap is None else f' ovl={args.overlap}'}{'' if args.parts is None else f' parts={args.parts}'}{'' if args.bins is None else f' bins={args.bins}'}{'' if args.leaf_cost is None else f' leaf={args.leaf_cost}'}{'' if args.spatial is None else f' sbvh={args.spatial}'}{'' if args.split_alpha is None else f' salpha={args.split_alpha}'} share 1/{args.share} r{args.rank} {args.layout if args.share > 1 else ''}{args.band or ''}{' tile ' + args.tile if args.tile else ''}: median {statistics.median(rounds):.4f} "
          f"mean {statistics.mean(rounds):.4f} min {min(rounds):.4f} ms/frame  rays {s.radiance_rays + s.shadow_rays} sched {s.schedule} ppw {s.paths_per_wave}",
          flush=True)
    if args.phases:
        ph = t.phase_clocks()
        tot = float(sum(ph)) or 1.0
        names = ("d1 trace", "d1 shade", "d1 shadow", "d2 trace", "d2 shade", "d2 shadow", "d>=3", "end/idle")
        print("  phases (share of lane time): " + ", ".join(f"{nm} {v / tot:.3f}" for nm, v in zip(names, ph)), flush=True)
    t.close()


if __name__ == "__main__":
    main()
