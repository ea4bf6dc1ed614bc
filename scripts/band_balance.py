#!/usr/bin/env python3
"""Cost-balanced band shares vs round-robin bands (r05 diagnostic for the 8-GPU tail).

1. One census frame of the full image with per-wave clocks (DXRPT_OPT_WAVE_CLOCKS): each 8x8 block's wave
   duration, summed per 8-row band -> a per-band cost.
2. Bands dealt to N ranks by LPT on that cost (distributed.balanced_band_layout) vs round robin.
3. Every rank's share of both layouts timed as scripts/time_frames.py does (fresh context per share).

    python scripts/band_balance.py [--config metric] [--world 8] [--rounds 3] [--frames 32]
"""
import argparse
import os
import statistics
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from scripts.time_frames import CONFIGS  # noqa: E402


def band_costs(D, A, sc, st, sky, W, H):
    import torch
    from dxrpathtracer_amd.tracer import DXRPathTracer
    t = DXRPathTracer(0)
    t.initialize_scene(sc, sky)
    t.build_rt_acceleration_structure()
    acc = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
    t.set_option(A.OPT_COUNT_TRAVERSAL, 1)
    t.set_option(A.OPT_WAVE_CLOCKS, 1)
    for f in range(3):
        t.render_raw(D.make_constants(sc, st, sky, W, H, f), st, acc.data_ptr(), W, H,
                     stream=torch.cuda.current_stream().cuda_stream, lights=D.make_lights(sc))
    torch.cuda.synchronize()
    wc = t.wave_clocks().astype(np.int64)
    t.close()
    dur = (wc[:, 1] - wc[:, 0]) * 0.01  # us
    nbx = (W + 7) // 8
    nb = (H + 7) // 8
    cost = np.zeros(nb)
    for w, d in enumerate(dur[: nbx * nb]):  # wave w = 8x8 block w (row-major blocks of the full frame)
        cost[w // nbx] += d
    return cost


def time_share(D, A, sc, st, sky, W, H, tiles, n, rounds, frames):
    import torch
    from dxrpathtracer_amd.tracer import DXRPathTracer
    t = DXRPathTracer(0)
    t.initialize_scene(sc, sky)
    t.build_rt_acceleration_structure()
    arr = (A.Tile * len(tiles))(*tiles)
    acc = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
    consts = [D.make_constants(sc, st, sky, W, H, s) for s in range(16)]
    lights = D.make_lights(sc)
    stream = torch.cuda.current_stream()
    for f in range(5):
        t.render_raw(consts[f % 16], st, acc.data_ptr(), W, H, tiles=arr, stream=stream.cuda_stream, lights=lights)
    torch.cuda.synchronize()
    res = []
    for r in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for f in range(frames):
            t.render_raw(consts[f % 16], st, acc.data_ptr(), W, H, tiles=arr, stream=stream.cuda_stream, lights=lights)
        b.record(stream)
        torch.cuda.synchronize()
        res.append(a.elapsed_time(b) / frames)
    t.close()
    return statistics.median(res)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="metric", choices=sorted(CONFIGS))
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--frames", type=int, default=32)
    args = ap.parse_args()
    import dxrpathtracer_amd as D
    import dxrpathtracer_amd._abi as A
    from dxrpathtracer_amd.distributed import band_layout, balanced_band_layout

    name, W, H, L = CONFIGS[args.config]
    sc = D.Scene(name)
    st = sc.settings(MaxPathLength=L)
    sky = D.make_sky(st)
    cost = band_costs(D, A, sc, st, sky, W, H)
    print("band cost (us of wave time): total %.0f, min %.1f, max %.1f, p50 %.1f" %
          (cost.sum(), cost.min(), cost.max(), np.median(cost)), flush=True)
    rr = band_layout(W, H, args.world)
    bal = balanced_band_layout(W, H, args.world, cost.tolist())
    for lab, lay in (("round-robin", rr), ("balanced", bal)):
        times = []
        for r in range(args.world):
            pred = sum(cost[t.y0 // 8] for t in lay.tiles[r])
            ms = time_share(D, A, sc, st, sky, W, H, lay.tiles[r], lay.counts[r], args.rounds, args.frames)
            times.append(ms)
            print(f"{lab:12s} {args.config} 1/{args.world} r{r}: {ms:.4f} ms  bands {len(lay.tiles[r])}  "
                  f"pixels {lay.counts[r]}  predicted cost {pred:.0f}", flush=True)
        print(f"{lab:12s} {args.config} 1/{args.world}: slowest {max(times):.4f} mean {statistics.mean(times):.4f} "
              f"spread {(max(times) - min(times)) / max(times):.3f}", flush=True)


if __name__ == "__main__":
    main()
