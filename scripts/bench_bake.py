"""Lightmap bake throughput: RenderBakingPass_Progressive at the reference's
LightMapResolution 4096 (DXRPathTracer.cpp:111) over the Sponza proxy's chart atlas, MaxPathLength 3.

One "step" = one bake pass (one cosine-hemisphere sample per covered texel, DispatchRays(4096, 4096)).
Prints one JSON line: texel samples/s, rays/s (counted by the path's own counters), ms per pass and
the CPU oracle on a bounded texel sample for scale.  Inputs are resident in HBM before timing.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import dxrpathtracer_amd as D  # noqa: E402
import dxrpathtracer_amd._abi as A  # noqa: E402
from dxrpathtracer_amd.scene import lightmap_charts, surface_map  # noqa: E402
from dxrpathtracer_amd.tracer import DXRPathTracer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--res", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--path-length", type=int, default=3)
    ap.add_argument("--scene", default="sponza")
    ap.add_argument("--cpu-texels", type=int, default=20000)
    args = ap.parse_args()
    res = args.res
    sc = D.Scene(args.scene)
    st = sc.settings(MaxPathLength=args.path_length)
    sky = D.make_sky(st)
    t0 = time.time()
    verts, idx = lightmap_charts(sc, res)
    pos, nrm = surface_map(verts, idx, res, res)
    raster_s = time.time() - t0
    covered = int((pos[..., 3] != 0).sum())
    tr = DXRPathTracer(0)
    tr.initialize_scene(sc, sky)
    tr.build_rt_acceleration_structure()
    dev = torch.device("cuda", 0)
    dpos = torch.from_numpy(pos.reshape(-1, 4)).to(dev)
    dnrm = torch.from_numpy(nrm.reshape(-1, 4)).to(dev)
    acc = torch.zeros((res * res, 4), dtype=torch.float32, device=dev)
    lm = torch.zeros_like(acc)
    den = torch.zeros_like(acc)
    stream = torch.cuda.current_stream().cuda_stream
    for s in range(args.warmup):
        tr.bake_lightmap(st, dpos.data_ptr(), dnrm.data_ptr(), acc.data_ptr(), lm.data_ptr(), res, res, s, stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for s in range(args.warmup, args.warmup + args.steps):
        tr.bake_lightmap(st, dpos.data_ptr(), dnrm.data_ptr(), acc.data_ptr(), lm.data_ptr(), res, res, s, stream)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    stats = tr.stats()  # ray counters of the last bake pass
    # median denoise of the result
    m0, m1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    m0.record()
    for _ in range(10):
        tr.denoise_median(lm.data_ptr(), den.data_ptr(), res, res, stream)
    m1.record()
    torch.cuda.synchronize()
    median_ms = m0.elapsed_time(m1) / 10
    samples = acc[:, 3].sum().item()
    cpu = None
    if args.cpu_texels > 0:
        from oracle import pyoracle as O
        osc = O.OracleScene(sc, sky)
        rtc = D.make_constants(sc, st, sky, res, res, 0)
        ca, cl = np.zeros_like(pos), np.zeros_like(pos)
        first = (res // 2) * res
        n = args.cpu_texels
        cov = int((pos.reshape(-1, 4)[first:first + n, 3] != 0).sum())
        th = min(16, os.cpu_count() or 1)
        c0 = time.time()
        osc.bake(rtc, st, D.make_lights(sc), pos, nrm, ca, cl, first=first, count=n, threads=th)
        cs = time.time() - c0
        cpu = {"value": cov / cs / 1e6, "unit": "M texel samples/s", "cores": th, "kind": "port",
               "sample": f"{n} texels ({cov} covered) of the same map, one bake pass"}
    out = {"metric": "lightmap bake texel samples/s", "value": covered / (ms * 1e-3) / 1e6,
           "unit": "M texel samples/s", "ms_per_pass": ms, "steps": args.steps, "warmup": args.warmup,
           "higher_is_better": True, "dtype": "f32", "data": "synthetic (seeded proxy + chart atlas)",
           "config": {"workload": f"{args.scene} lightmap {res}x{res} L={args.path_length}",
                      "covered_texels": covered, "raster_s": round(raster_s, 2)},
           "valid_samples_per_covered_texel": samples / covered,
           "rays_per_pass": int(stats.radiance_rays + stats.shadow_rays),
           "Mrays_s": (stats.radiance_rays + stats.shadow_rays) / (ms * 1e-3) / 1e6,
           "median_denoise_ms": median_ms,
           "median_denoise_GBps": res * res * 16 * 2 / (median_ms * 1e-3) / 1e9,
           "cpu_baseline": cpu}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
