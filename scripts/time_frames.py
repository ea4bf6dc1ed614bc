#!/usr/bin/env python3
"""ms/frame of the default (shipped) schedule on a BASELINE config, for A/B of kernel builds
(DXRPT_KERNEL_LIB_DIR picks the libdxrpt.so) and of context options.  Prints one line: label, median and
mean ms/frame of `--rounds` x `--frames` back-to-back frames (HIP events on the render stream), counted
rays per frame, the schedule bits.  --kernels adds the per-launch kernel timings of those frames
(DXRPT_OPT_KERNEL_TIMING; with overlapped frames the spans overlap their neighbours').

    python scripts/time_frames.py [--label x] [--config metric|c2|c3|c4|c5] [--share N --rank r]
                                  [--opt NAME=VALUE ...] [--kernels]
"""
import argparse
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
CONFIGS = {"metric": ("sponza", 1920, 1080, 3), "c2": ("sponza", 1280, 720, 3), "c3": ("sponza", 1920, 1080, 8),
           "c4": ("suntemple", 1920, 1080, 3), "c5": ("sponza", 3840, 2160, 6)}
BUILD_OPTIONS = ("LEAF_COST", "SPATIAL_SPLITS", "TREELET_PASSES")  # set before the BVH build


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--label", default=os.environ.get("DXRPT_KERNEL_LIB_DIR", "default"))
    ap.add_argument("--config", default="metric", choices=sorted(CONFIGS))
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--share", type=int, default=1)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--layout", default="bands", choices=["bands", "blocks"])
    ap.add_argument("--tile", default=None, help="x,y,w,h: render only this rectangle (one tile)")
    ap.add_argument("--max-path", type=int, default=None, help="MaxPathLength override (a cost breakdown by depth)")
    ap.add_argument("--any-hit", type=int, default=None, help="MaxAnyHitPathLength override")
    ap.add_argument("--opt", action="append", default=[],
                    help="NAME=VALUE: dxrpt_set_option(DXRPT_OPT_NAME, VALUE), e.g. FRAME_OVERLAP=0, TAIL_OCCUPANCY=6")
    ap.add_argument("--kernels", action="store_true", help="also print per-launch kernel timings (head / tail / path)")
    ap.add_argument("--side-stream", action="store_true",
                    help="mimic NativeGather's streams: per frame a slab copy on a side stream after the render, "
                         "waited for by the render stream one frame later")
    ap.add_argument("--cur-copy", action="store_true",
                    help="per frame a slab snapshot copy on the render stream (a gather on the caller's stream)")
    ap.add_argument("--phases", action="store_true",
                    help="print the per-phase lane-time split of the timed frames (kernel builds with -DDXRPT_DIAG_PHASES=1)")
    args = ap.parse_args()
    import torch
    import dxrpathtracer_amd as D
    import dxrpathtracer_amd._abi as A
    from dxrpathtracer_amd.distributed import screen_layout
    from dxrpathtracer_amd.tracer import DXRPathTracer

    name, W, H, L = CONFIGS[args.config]
    L = L if args.max_path is None else args.max_path
    sc = D.Scene(name)
    st = sc.settings(MaxPathLength=L, **({} if args.any_hit is None else {"MaxAnyHitPathLength": args.any_hit}))
    sky = D.make_sky(st)
    t = DXRPathTracer(0)
    opts = [(o.split("=")[0].upper(), int(o.split("=")[1], 0)) for o in args.opt]
    for k, v in opts:
        if k in BUILD_OPTIONS:
            t.set_option(getattr(A, "OPT_" + k), v)
    t.initialize_scene(sc, sky)
    t.build_rt_acceleration_structure()
    for k, v in opts:
        if k not in BUILD_OPTIONS:
            t.set_option(getattr(A, "OPT_" + k), v)
    tiles, n = None, W * H
    if args.tile:
        x, y, w, h = (int(v) for v in args.tile.split(","))
        tiles, n = [A.Tile(x, y, w, h, 0, w, 0)], w * h
    elif args.share > 1:
        lay = screen_layout(W, H, args.share, args.layout)
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
    if args.kernels:
        t.set_option(A.OPT_KERNEL_TIMING, 1)
        t.reset_timing()
    side = torch.cuda.Stream() if args.side_stream else None
    snap = torch.empty_like(acc) if side is not None else None
    pend = None

    cur_snap = torch.empty_like(acc) if args.cur_copy else None

    def frame_end():
        nonlocal pend
        if cur_snap is not None:
            cur_snap.copy_(acc)
        if side is None:
            return
        side.wait_stream(stream)
        with torch.cuda.stream(side):
            snap.copy_(acc)
        ev = torch.cuda.Event()
        ev.record(side)
        if pend is not None:
            stream.wait_event(pend)
        pend = ev

    rounds = []
    for r in range(args.rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for f in range(args.frames):
            t.render_raw(consts[f % 16], st, acc.data_ptr(), W, H, tiles=tiles, stream=stream.cuda_stream, lights=lights)
            frame_end()
        b.record(stream)
        torch.cuda.synchronize()
        rounds.append(a.elapsed_time(b) / args.frames)
    s = t.stats()
    desc = " ".join(args.opt) + (f" L={L}" if args.max_path is not None else "")
    desc += (" side-stream" if args.side_stream else "") + (" cur-copy" if args.cur_copy else "")
    where = f"share 1/{args.share} r{args.rank} {args.layout}" if args.share > 1 else ("tile " + args.tile if args.tile else "full")
    print(f"{args.label:24s} {args.config} {desc} {where}: median {statistics.median(rounds):.4f} "
          f"mean {statistics.mean(rounds):.4f} min {min(rounds):.4f} ms/frame  rays {s.radiance_rays + s.shadow_rays} "
          f"sched {s.schedule} occ {s.occupancy}/{s.tail_occupancy}", flush=True)
    if args.kernels:
        parts = []
        for k in (A.K_PATH, A.K_PATH_HEAD, A.K_PATH_TAIL):
            if s.kernel_launches[k]:
                parts.append(f"{A.KERNEL_NAMES[k]} {s.kernel_ms[k] / s.kernel_launches[k]:.4f} ms x{s.kernel_launches[k] / s.timed_frames:g}/frame")
        print("  per launch: " + ", ".join(parts), flush=True)
    if args.phases:
        ph = t.phase_clocks()
        names = ("d1 trace", "d1 shade", "d1 shadow", "d2 trace", "d2 shade", "d2 shadow", "d>=3", "end/idle")
        split = ("trace", "shade", "push", "shadow0", "shadow1", "shadow2+", "handoff", "idle")
        for label, part, nm in (("k_path", ph[0:8], names), ("k_path_head", ph[8:16], split), ("k_path_tail", ph[16:24], split)):
            tot = float(sum(part))
            if tot:
                print(f"  {label} phases (share of lane time, {tot / 1e8 / args.rounds / args.frames:.4g} lane-s/frame): "
                      + ", ".join(f"{n} {v / tot:.3f}" for n, v in zip(nm, part)), flush=True)
    t.close()


if __name__ == "__main__":
    main()
