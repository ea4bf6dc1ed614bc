#!/usr/bin/env python3
"""A/B of traversal variants in ONE process (interleaved rounds, median per variant), on the bench
workload (Sponza proxy 1920x1080, L=3).  Prints per-kernel ms per frame from the HIP-event timings.

    python scripts/ab_variants.py [--frames 16] [--rounds 3] [--variants w8m0,w8m1r16,...]
variant syntax: letter+number tokens, e.g. w8m0b64o7 (w width, m mode, r refill lanes, k chunks per
wave, p postpone lanes, b trace block, o occupancy; see KEYS for the rest, e.g. l megakernel lanes)
"""
import argparse
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


KEYS = {"w": "width", "m": "mode", "r": "refill", "k": "chunks", "p": "postpone", "b": "block", "o": "occ",
        "s": "sblock", "q": "socc", "x": "spatial", "c": "leafcost", "h": "hocc", "g": "sgrid",
        "j": "conc", "t": "pipe", "a": "packet", "n": "ldsnodes", "z": "xcd", "u": "pswitch", "e": "mega", "v": "megaocc", "y": "persist", "l": "lanes"}
DEFAULTS = {"width": 8, "mode": 0, "refill": 16, "chunks": 4, "postpone": 0, "block": 64, "occ": 7, "sblock": 256,
            "socc": 0, "spatial": 150, "leafcost": 150, "hocc": 8, "sgrid": 0, "conc": 1, "pipe": 0, "packet": 3, "ldsnodes": 0, "xcd": 0, "pswitch": 0, "mega": 1, "megaocc": 0, "persist": 0, "lanes": 64}
BUILD_KEYS = ("width", "spatial", "leafcost")  # a separate context (BVH) per combination


def parse(v):
    """'w8m1r16k4p16b64o7' -> dict(width, mode, refill, chunks, postpone, block, occ); unspecified keys
    take DEFAULTS."""
    import re
    out = dict(DEFAULTS)
    pos = 0
    for m in re.finditer(r"([a-z])(\d+)", v):
        if m.start() != pos or m[1] not in KEYS:
            raise SystemExit(f"bad variant {v}")
        out[KEYS[m[1]]] = int(m[2])
        pos = m.end()
    if pos != len(v):
        raise SystemExit(f"bad variant {v}")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="w2m0,w8m0,w8m1r16,w8m1r32,w8m1r48")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--L", type=int, default=3)
    ap.add_argument("--scene", default="sponza")
    ap.add_argument("--share", type=int, default=1, help="render one rank's band share of an N-GPU frame")
    ap.add_argument("--rank", type=int, default=0, help="which rank's share (--share > 1)")
    ap.add_argument("--band", type=int, default=0, help="band rows of the partition (0: distributed.BAND_ROWS)")
    args = ap.parse_args()
    import torch
    import dxrpathtracer_amd as D
    import dxrpathtracer_amd._abi as A
    from dxrpathtracer_amd.tracer import DXRPathTracer

    W, H = args.width, args.height
    sc = D.Scene(args.scene)
    st = sc.settings(MaxPathLength=args.L)
    sky = D.make_sky(st)
    tracers = {}
    for bk in sorted({tuple(parse(v)[k] for k in BUILD_KEYS) for v in args.variants.split(",")}):
        t = DXRPathTracer(0)
        t.set_option(A.OPT_BVH_WIDTH, bk[0])
        t.set_option(A.OPT_SPATIAL_SPLITS, bk[1])
        t.set_option(A.OPT_LEAF_COST, bk[2])
        t.initialize_scene(sc, sky)
        info = t.build_rt_acceleration_structure()
        print(f"bvh {bk}: {info.num_nodes} nodes depth {info.max_depth} build {info.build_ms:.0f} ms", flush=True)
        tracers[bk] = t
    accum = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
    tiles = None
    if args.share > 1:
        from dxrpathtracer_amd.distributed import band_layout
        tiles = band_layout(W, H, args.share, **({'band': args.band} if args.band else {})).rank_tiles(args.rank)
    consts = [D.make_constants(sc, st, sky, W, H, s) for s in range(16)]
    lights = D.make_lights(sc)
    sh = torch.cuda.current_stream().cuda_stream
    res = {v: [] for v in args.variants.split(",")}
    for rnd in range(args.rounds):
        for v in res:
            o = parse(v)
            t = tracers[tuple(o[k] for k in BUILD_KEYS)]
            t.set_option(A.OPT_POSTPONE_TRIS, o["postpone"])
            t.set_option(A.OPT_TRAVERSAL_MODE, o["mode"])
            t.set_option(A.OPT_REFILL_LANES, o["refill"])
            t.set_option(A.OPT_CHUNKS_PER_WAVE, o["chunks"])
            t.set_option(A.OPT_TRACE_BLOCK, o["block"])
            t.set_option(A.OPT_OCCUPANCY, o["occ"])
            t.set_option(A.OPT_SHADOW_OCCUPANCY, o["hocc"])
            t.set_option(A.OPT_SHADOW_GRID, o["sgrid"])
            t.set_option(A.OPT_CONCURRENCY, o["conc"])
            t.set_option(A.OPT_TRAVERSAL_PIPELINE, o["pipe"])
            t.set_option(A.OPT_PACKET_TRAVERSAL, o["packet"])
            t.set_option(A.OPT_LDS_NODES, o["ldsnodes"])
            t.set_option(A.OPT_XCD_MAPPING, o["xcd"])
            t.set_option(A.OPT_PACKET_SWITCH, o["pswitch"])
            t.set_option(A.OPT_MEGAKERNEL_PATHS, 1 << 30 if o["mega"] else 0)
            t.set_option(A.OPT_MEGAKERNEL_OCCUPANCY, o["megaocc"])
            t.set_option(A.OPT_MEGAKERNEL_PERSISTENT, o["persist"])
            t.set_option(A.OPT_MEGAKERNEL_LANES, o["lanes"])
            t.set_option(A.OPT_SHADE_BLOCK, o["sblock"])
            t.set_option(A.OPT_SHADE_OCCUPANCY, o["socc"])
            for f in range(3):
                t.render_raw(consts[f], st, accum.data_ptr(), W, H, tiles=tiles, stream=sh, lights=lights)
            torch.cuda.synchronize()
            # wall-clock pass without per-kernel timing (which serialises the concurrent passes)
            t0 = time.perf_counter()
            for f in range(args.frames):
                t.render_raw(consts[f % 16], st, accum.data_ptr(), W, H, tiles=tiles, stream=sh, lights=lights)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / args.frames * 1e3
            # per-kernel breakdown pass
            t.set_option(A.OPT_KERNEL_TIMING, 1)
            t.reset_timing()
            for f in range(args.frames):
                t.render_raw(consts[f % 16], st, accum.data_ptr(), W, H, tiles=tiles, stream=sh, lights=lights)
            torch.cuda.synchronize()
            s = t.stats()
            t.set_option(A.OPT_KERNEL_TIMING, 0)
            n = max(1, s.timed_frames)
            res[v].append((wall, [s.kernel_ms[k] / n for k in range(A.K_COUNT)]))
    print(f"{args.scene} {W}x{H} L={args.L} share 1/{args.share} rank {args.rank}: median of {args.rounds} rounds x {args.frames} frames (ms/frame)")
    print(f"{'variant':12s} {'wall':>8s} " + " ".join(f"{k:>12s}" for k in A.KERNEL_NAMES))
    for v, rows in res.items():
        wall = statistics.median(r[0] for r in rows)
        ks = [statistics.median(r[1][k] for r in rows) for k in range(A.K_COUNT)]
        print(f"{v:12s} {wall:8.3f} " + " ".join(f"{x:12.3f}" for x in ks))


if __name__ == "__main__":
    main()
