#!/usr/bin/env python3
"""Traversal census of one screen tile (or the full frame) of a BASELINE config: node and triangle-record
fetches of the timed megakernel schedule (per lane in per-lane traversals, per wave in packet traversals,
DXRPT_OPT_COUNT_TRAVERSAL), per path and per ray -- where a slow block's work goes.

    python scripts/tile_census.py [--config metric] [--tile x,y,w,h] [--max-path L]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from scripts.time_frames import CONFIGS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="metric", choices=sorted(CONFIGS))
    ap.add_argument("--tile", default=None)
    ap.add_argument("--max-path", type=int, default=None)
    ap.add_argument("--any-hit", type=int, default=None)
    args = ap.parse_args()
    import torch
    import dxrpathtracer_amd as D
    import dxrpathtracer_amd._abi as A
    from dxrpathtracer_amd.tracer import DXRPathTracer

    name, W, H, L = CONFIGS[args.config]
    L = L if args.max_path is None else args.max_path
    sc = D.Scene(name)
    st = sc.settings(MaxPathLength=L, **({} if args.any_hit is None else {"MaxAnyHitPathLength": args.any_hit}))
    sky = D.make_sky(st)
    t = DXRPathTracer(0)
    t.initialize_scene(sc, sky)
    t.build_rt_acceleration_structure()
    tiles, n = None, W * H
    if args.tile:
        x, y, w, h = (int(v) for v in args.tile.split(","))
        tiles, n = [A.Tile(x, y, w, h, 0, w, 0)], w * h
    acc = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
    t.set_option(A.OPT_COUNT_TRAVERSAL, 1)
    t.render_raw(D.make_constants(sc, st, sky, W, H, 0), st, acc.data_ptr(), W, H, tiles=tiles,
                 stream=torch.cuda.current_stream().cuda_stream, lights=D.make_lights(sc))
    torch.cuda.synchronize()
    s = t.stats()
    rr, sr = max(1, s.radiance_rays), max(1, s.shadow_rays)
    print(f"{args.config} L={L} tile {args.tile or 'full'}: paths {n}  radiance rays/path {s.radiance_rays / n:.2f} "
          f"shadow rays/path {s.shadow_rays / n:.2f}  node fetches/path {(s.node_visits_radiance + s.node_visits_shadow) / n:.1f} "
          f"(radiance {s.node_visits_radiance / rr:.1f}/ray, shadow {s.node_visits_shadow / sr:.1f}/ray)  "
          f"tri fetches/path {(s.tri_tests_radiance + s.tri_tests_shadow) / n:.1f} "
          f"(radiance {s.tri_tests_radiance / rr:.1f}/ray, shadow {s.tri_tests_shadow / sr:.1f}/ray)", flush=True)
    t.close()


if __name__ == "__main__":
    main()
