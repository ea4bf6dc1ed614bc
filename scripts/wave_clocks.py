#!/usr/bin/env python3
"""Where a frame's (or a GPU share's) time goes, wave by wave: one census frame of the megakernel with
per-wave start/end stamps (DXRPT_OPT_COUNT_TRAVERSAL + DXRPT_OPT_WAVE_CLOCKS, s_memrealtime 100 MHz).
Prints the frame span, the distribution of wave durations and the slowest waves with their 8x8
pixel blocks.

    python scripts/wave_clocks.py [--config metric] [--share 8 --rank 2] [--json out.json]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from scripts.time_frames import CONFIGS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="metric", choices=sorted(CONFIGS))
    ap.add_argument("--share", type=int, default=1)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--layout", default="bands", choices=["blocks", "bands"])
    ap.add_argument("--frames", type=int, default=3, help="census frames (the last one is reported)")
    ap.add_argument("--json", default=None)
    ap.add_argument("--occ", type=int, default=0, help="megakernel occupancy (0: default by size)")
    ap.add_argument("--ordered", action="store_true", help="time the default (cost-ordered) frames, not a census")
    ap.add_argument("--slots", type=int, default=256 * 4 * 7, help="resident wave slots (CUs x SIMDs x waves/SIMD)")
    args = ap.parse_args()
    import torch
    import dxrpathtracer_amd as D
    import dxrpathtracer_amd._abi as A
    from dxrpathtracer_amd.distributed import screen_layout
    from dxrpathtracer_amd.tracer import DXRPathTracer

    name, W, H, L = CONFIGS[args.config]
    sc = D.Scene(name)
    st = sc.settings(MaxPathLength=L)
    sky = D.make_sky(st)
    t = DXRPathTracer(0)
    t.initialize_scene(sc, sky)
    t.build_rt_acceleration_structure()
    tiles, n = None, W * H
    if args.share > 1:
        lay = screen_layout(W, H, args.share, args.layout)
        tiles, n = lay.rank_tiles(args.rank), lay.counts[args.rank]
    acc = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    if not args.ordered:  # census frame (path order); --ordered: the shipped cost-ordered frames
        t.set_option(A.OPT_COUNT_TRAVERSAL, 1)
    t.set_option(A.OPT_WAVE_CLOCKS, 1)
    if args.occ:
        t.set_option(A.OPT_MEGAKERNEL_OCCUPANCY, args.occ)
    for f in range(args.frames):
        t.render_raw(D.make_constants(sc, st, sky, W, H, f), st, acc.data_ptr(), W, H, tiles=tiles, stream=stream,
                     lights=D.make_lights(sc))
    torch.cuda.synchronize()
    wc = t.wave_clocks().astype(np.int64)
    s = t.stats()
    t0 = wc[:, 0].min()
    start = (wc[:, 0] - t0) * 0.01  # us
    end = (wc[:, 1] - t0) * 0.01
    dur = end - start
    order = np.argsort(-dur)
    # block position of wave w: the tiles are walked in order, 64 paths per wave (8x8 blocks when the
    # tile is a multiple of 8 in both sizes)
    tl = tiles if tiles else [A.Tile(0, 0, W, H, 0, W, 0)]
    blocks = []
    for tt in tl:
        bw, bh = (tt.w + 7) // 8, (tt.h + 7) // 8
        for b in range(bw * bh):
            blocks.append((tt.x0 + (b % bw) * 8, tt.y0 + (b // bw) * 8))
    per = max(1, round(n / len(wc)))  # paths per wave
    res = {"config": args.config, "ordered": bool(args.ordered), "paths_per_wave": per, "share": args.share, "rank": args.rank, "layout": args.layout, "waves": int(len(wc)),
           "span_us": float(end.max()), "last_start_us": float(start.max()),
           "dur_us": {q: float(np.percentile(dur, p)) for q, p in (("min", 0), ("p50", 50), ("p90", 90), ("p99", 99),
                                                                      ("max", 100))},
           "mean_us": float(dur.mean()),
           "slowest": [{"wave": int(w), "block_xy": blocks[w * per // 64] if w * per // 64 < len(blocks) else None,
                        "start_us": round(float(start[w]), 1), "dur_us": round(float(dur[w]), 1)} for w in order[:12]],
           # resident-slot utilisation: wave time / (slots x span), and waves alive at fractions of the span
           "slots": int(args.slots), "busy_frac": float(dur.sum() / (args.slots * end.max())),
           "alive_at": {f"{q}%": int(((start <= end.max() * q / 100) & (end > end.max() * q / 100)).sum())
                        for q in (25, 50, 75, 85, 90, 95, 98)},
           "nodes_per_path": round((s.node_visits_radiance + s.node_visits_shadow) / max(1, n), 2)}
    print(json.dumps(res))
    if args.json:
        np.save(args.json.replace(".json", ".npy"), np.stack([start, end], 1))
        json.dump(res, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
