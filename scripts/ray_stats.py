#!/usr/bin/env python3
"""Per-depth radiance / shadow ray counts of one frame of a BASELINE config (dxrpt_get_stats), and the
per-wave averages (64 paths per wave).  usage: python scripts/ray_stats.py [--config metric]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from scripts.time_frames import CONFIGS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="metric", choices=sorted(CONFIGS))
    args = ap.parse_args()
    import torch
    import dxrpathtracer_amd as D
    from dxrpathtracer_amd.tracer import DXRPathTracer
    name, W, H, L = CONFIGS[args.config]
    sc = D.Scene(name)
    st = sc.settings(MaxPathLength=L)
    sky = D.make_sky(st)
    t = DXRPathTracer(0)
    t.initialize_scene(sc, sky)
    t.build_rt_acceleration_structure()
    acc = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
    t.render_raw(D.make_constants(sc, st, sky, W, H, 0), st, acc.data_ptr(), W, H,
                 stream=torch.cuda.current_stream().cuda_stream, lights=D.make_lights(sc))
    torch.cuda.synchronize()
    s = t.stats()
    waves = (W * H + 63) // 64
    for d in range(1, L):
        r, sh = s.radiance_rays_per_depth[d], s.shadow_rays_per_depth[d]
        print(f"{args.config} depth {d}: radiance {r} ({r / waves:.1f}/wave)  shadow {sh} ({sh / waves:.1f}/wave)")


if __name__ == "__main__":
    main()
