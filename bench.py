#!/usr/bin/env python3
"""Benchmark of the path tracer on BASELINE.json's metric config: Sponza(-proxy) 1920x1080,
MaxPathLength 3, one sample per pixel per frame with progressive accumulation.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

A step is one frame (DispatchRays(1920,1080,1) equivalent, DXRPathTracer.cpp:2024-2090) over the whole
image.  With N ranks the image is split into 8-row bands, band b -> rank b % N (distributed.band_layout;
--layout blocks: 8x8-pixel blocks dealt in a seeded random order) and every frame ends
with an RCCL gather of the rank slabs to rank 0 plus the un-permute: total work per
frame is fixed, so scaling is "strong".  The gather of frame f runs on the render stream, which with
overlapped frames carries only the blends, while frames f+1.. render on the library's slot streams
(distributed.NativeGather); the last frame's gather is inside the timed region.  value = nominal
Mrays/s of the whole job (W*H*(1+2(L-1)) rays per frame, the reference's HUD formula
DXRPathTracer.cpp:2171) over the max-over-ranks time.  Rank 0 prints one JSON line; with N > 1 it carries
every rank's render time, the gather's and un-permute's times and RCCL's rank count ("multi_gpu").
roofline: the dominant kernel's SURVEY.md 8(d) bytes per launch over its average launch duration from a
frame-at-a-time pass (HIP events, DXRPT_OPT_FRAME_OVERLAP 0); the overlapped frame-interval rate beside it.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
# Overlapped frames run on up to three internal streams of libdxrpt, which with the render stream fill the
# HIP runtime's default four hardware queues per process; a multi-GPU rank adds RCCL's and
# torch.distributed's streams.  Give those queues of their own rather than sharing one with a frame slot
# (set before torch initialises HIP; INTEGRATION.md "Streams").
if int(os.environ.get("WORLD_SIZE", "1")) > 1:
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

WIDTH, HEIGHT, PATH_LENGTH = 1920, 1080, 3
SCENE = "sponza"
# BASELINE.json configs, selectable with --config (the default is the metric's; the others are the
# parity configs, timed the same way for the record): name -> (scene, width, height, path length)
CONFIGS = {"metric": ("sponza", 1920, 1080, 3), "c2": ("sponza", 1280, 720, 3), "c3": ("sponza", 1920, 1080, 8),
           "c4": ("suntemple", 1920, 1080, 3), "c5": ("sponza", 3840, 2160, 6)}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "Mrays/sec + ms/frame, Sponza 1920x1080 path-length 3 at 1/2/4/8 GPU"
ACCUM_BYTES = 32  # RaygenShader's progressive blend: 16-B read + 16-B write per path


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def usable_cpus():
    """(threads to use, detail): the CPUs this process may run on -- its affinity mask, capped by a
    cgroup v2 CPU quota (cpu.max) when one is set (a GPU box grants a job a share of the host)."""
    host = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = host
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    n = aff if quota is None else max(1, min(aff, int(quota + 0.5)))
    return n, {"host_cpus": host, "affinity_cpus": aff, "cgroup_cpu_quota": quota}


def cpu_baseline(scene, sky, settings, threads):
    """The CPU oracle (scalar C++ restatement, own BVH) on a bounded sample: one full 1920x1080 L=3
    frame at CurrSampleIdx 0 on `threads` host threads (default: every CPU the process may use, one
    worker per core as SURVEY.md 8(d) asks), plus a single-thread figure on a 1920x68 band of the
    same frame."""
    import dxrpathtracer_amd as D
    from oracle import pyoracle as O
    cpus = usable_cpus()
    if threads <= 0:
        threads = cpus[0]
    orc = O.OracleScene(scene, sky)
    rtc = D.make_constants(scene, settings, sky, WIDTH, HEIGHT, 0)
    lights = D.make_lights(scene)
    t0 = time.perf_counter()
    _, st = orc.render(rtc, settings, lights, WIDTH, HEIGHT, threads=threads)
    dt = time.perf_counter() - t0
    band = (0, HEIGHT // 2 - 34, WIDTH, 68)
    t1 = time.perf_counter()
    orc.render(rtc, settings, lights, WIDTH, HEIGHT, crop=band, threads=1)
    dt1 = time.perf_counter() - t1
    per_px = 1 + 2 * (PATH_LENGTH - 1)
    nominal = WIDTH * HEIGHT * per_px
    return {"value": round(nominal / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"one full {WIDTH}x{HEIGHT} L={PATH_LENGTH} frame (sample 0) of the same scene, "
                      f"{dt:.2f} s wall, {st.radiance_rays + st.shadow_rays} rays traced, oracle BVH",
            "frame_s": round(dt, 3),
            "single_thread_Mrays_s": round(band[2] * band[3] * per_px / dt1 / 1e6, 3),
            "single_thread_sample": f"{band[2]}x{band[3]} band at rows {band[1]}..{band[1] + band[3] - 1}, {dt1:.2f} s",
            "cpu_model": cpu_model(), **cpus[1]}


def pmc_kernels(config):
    """Per-kernel, per-LAUNCH counters of the non-overlapped launch profile of this config (the newest
    profiles/<round>_launch_<config>.json, written by scripts/pmc_summary.py over scripts/profile.sh's
    rocprofv3 passes of scripts/launch_profile.py): {kernel kind: summary}."""
    import glob
    for p in sorted(glob.glob(os.path.join(REPO, "profiles", f"*_launch_{config}.json")), reverse=True):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("config") == f"{SCENE}-proxy {WIDTH}x{HEIGHT} L={PATH_LENGTH}":
            return d, os.path.basename(p)
    return {}, None


def full_formula_bytes(c, settings, bvh):
    """SURVEY.md 8(d)'s algorithmic bytes of a set of rays, term by term as the survey writes them:
      per ray: 32 B in (o, d, tmax, flags) + 16 B hit out (radiance) or 4 B visibility (shadow)
               + N_node x S_node + N_tri x S_tri (the census' fetches of the timed schedule)
      per radiance hit: 12 (3 indices) + 192 (3 vertices) + 16 (GeometryInfo) + 24 (Material)
               + taps x 4 texels x 4 B (RGBA8: normal, albedo if enabled; metallic, roughness, emissive)
               + 64 (path-state RMW) + 32 (next-ray write) + 32 (shadow-ray write)
      per miss: 4 x 8 B (FP16 cube bilinear)
      + 32 B accumulation RMW per path that ends.
    `c`: radiance_rays, shadow_rays, node_fetches, tri_fetches, hits, paths_ending.  Alpha-test opacity
    taps of any-hit candidates are not counted (a lower bound for C4)."""
    hits = int(c["hits"])
    misses = int(c["radiance_rays"]) - hits
    taps = 3 + int(settings.EnableNormalMaps) + int(settings.EnableAlbedoMaps)
    per_hit = 12 + 192 + 16 + 24 + taps * 16 + 64 + 32 + 32
    terms = {
        "radiance_ray_io": int(c["radiance_rays"]) * (32 + 16),
        "shadow_ray_io": int(c["shadow_rays"]) * (32 + 4),
        "bvh_node_fetches": int(c["node_fetches"]) * int(bvh.node_bytes),
        "triangle_fetches": int(c["tri_fetches"]) * int(bvh.tri_bytes),
        "radiance_hit_shading": hits * per_hit,
        "miss_sky_taps": misses * 32,
        "accumulation": ACCUM_BYTES * int(c["paths_ending"]),
    }
    return sum(terms.values()), {"terms": terms, "counts": {k: int(v) for k, v in c.items()}, "misses": misses,
                                 "taps_per_hit": taps, "bytes_per_hit": per_hit}


def census_parts(census, pixels, L):
    """The census of one frame split by kernel: the split schedule's head runs every depth-1 vertex, its
    tails every deeper one (the single k_path runs both).  Depth-1 counts are dxrpt_stats.census_depth1;
    a path ends in the head iff it has no depth-2 ray."""
    rr = [int(census.radiance_rays_per_depth[d]) for d in range(8)]
    sr = [int(census.shadow_rays_per_depth[d]) for d in range(8)]
    d1 = [int(v) for v in census.census_depth1]
    tot = {"radiance_rays": int(census.radiance_rays), "shadow_rays": int(census.shadow_rays),
           "node_fetches": int(census.node_visits_radiance + census.node_visits_shadow),
           "tri_fetches": int(census.tri_tests_radiance + census.tri_tests_shadow),
           "hits": int(census.radiance_hits), "paths_ending": int(pixels)}
    ends_head = int(pixels) - (rr[2] if L > 2 else 0)
    head = {"radiance_rays": rr[1], "shadow_rays": sr[1], "node_fetches": d1[0] + d1[2], "tri_fetches": d1[1] + d1[3],
            "hits": d1[4], "paths_ending": ends_head}
    tail = {k: tot[k] - head[k] for k in tot}
    return {"frame": tot, "head": head, "tail": tail}


def schedule_name(bits, A):
    if not bits & A.SCHED_MEGAKERNEL:
        return "wavefront passes"
    if bits & A.SCHED_SPLIT:
        return "depth-split megakernel (k_path_head + k_path_tail per depth)" + (
            ", overlapped frames" if bits & A.SCHED_OVERLAP else "")
    s = "megakernel (k_path)"
    if bits & A.SCHED_COST_ORDERED:
        s += ", cost-ordered waves"
    if bits & A.SCHED_OVERLAP:
        s += ", overlapped frames"
    return s


def percentile(v, q):
    return float(np.percentile(np.asarray(v, dtype=np.float64), q)) if len(v) else None


def paced_latency(torch, stream, render, frames, ahead):
    """Frame latency with at most `ahead` frames submitted and not yet blended -- the reference's
    swap-chain bound (RenderLatency = 2, Graphics/DX12.h:21): before submitting frame f the host waits for
    frame f-ahead's blend.  Per frame: host submit time -> GPU completion of the event after its blend on
    the caller's stream, both on the host clock (GPU event times are anchored at a reference event recorded
    on the idle GPU at a known host time; `anchor_us` bounds that anchor's own launch delay).  Returns p50 /
    p99 / max latency and the paced pass's ms per frame."""
    torch.cuda.synchronize()
    ref = torch.cuda.Event(enable_timing=True)
    h0 = time.perf_counter()
    ref.record(stream)
    ref.synchronize()
    anchor_us = (time.perf_counter() - h0) * 1e6
    subs, done = [], []
    for f in range(frames):
        if f >= ahead:
            done[f - ahead].synchronize()
        subs.append(time.perf_counter())
        render(f)
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        done.append(e)
    torch.cuda.synchronize()
    end = [h0 + ref.elapsed_time(e) * 1e-3 for e in done]
    lat = [(t - h) * 1e3 for t, h in zip(end, subs)]
    return {"frames_in_flight_cap": ahead, "p50_ms": round(percentile(lat, 50), 4), "p99_ms": round(percentile(lat, 99), 4),
            "max_ms": round(max(lat), 4), "ms_per_frame": round((end[-1] - subs[0]) * 1e3 / frames, 4),
            "frames": frames, "anchor_us": round(anchor_us, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0: every usable CPU)")
    ap.add_argument("--config", default="metric", choices=sorted(CONFIGS))
    ap.add_argument("--layout", default="bands", choices=["bands", "blocks"],
                    help="N-GPU screen partition: round-robin 8-row bands (default) or a seeded 8x8-block deal")
    ap.add_argument("--gather", default="native", choices=["native", "torch"],
                    help="N-GPU frame-end gather: the C ABI's RCCL send/recv + un-permute kernel (default) or "
                         "torch.distributed.gather + index_select")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1: nccl (= RCCL, one rank per GPU; the default) or gloo "
                         "(a rehearsal of the N-rank control flow on fewer GPUs: ranks share devices round robin, the "
                         "native RCCL gather refuses two ranks on one GPU, so the torch gather runs staged through host)")
    ap.add_argument("--phase-timeout", type=float, default=300.0,
                    help="seconds any one phase (setup, a collective, the timed frames) may take on a rank before "
                         "every rank is ended with a JSON error line")
    args = ap.parse_args()
    global SCENE, WIDTH, HEIGHT, PATH_LENGTH
    SCENE, WIDTH, HEIGHT, PATH_LENGTH = CONFIGS[args.config]
    metric = METRIC if args.config == "metric" else \
        f"Mrays/sec + ms/frame, {SCENE.capitalize()} {WIDTH}x{HEIGHT} path-length {PATH_LENGTH} (BASELINE config {args.config})"

    import torch
    import torch.distributed as dist
    from dxrpathtracer_amd.watchdog import Watchdog, default_store

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    # every rank ends non-zero with a JSON error line on any failure or stuck collective (watchdog.py); the
    # rendezvous store carries the abort to the other ranks
    wd = Watchdog(rank, world, None, metric)
    try:
        with wd.phase("init", args.phase_timeout):
            # one rank per GPU (the driver's launch); a gloo rehearsal may put several ranks on one device
            device = local_rank if args.dist_backend == "nccl" else local_rank % max(1, torch.cuda.device_count())
            torch.cuda.set_device(device)
            if world > 1:
                if args.dist_backend == "nccl":
                    dist.init_process_group("nccl", device_id=torch.device("cuda", device))
                else:
                    dist.init_process_group("gloo")
                wd.store = default_store()
        run(args, metric, world, rank, device, wd)
    except BaseException as e:  # noqa: BLE001 -- any failure ends every rank (SystemExit from argparse aside)
        import traceback
        traceback.print_exc()
        wd.fail(f"{type(e).__name__}: {e}")
    wd.close()


def run(args, metric, world, rank, device, wd):
    import torch
    import torch.distributed as dist
    import dxrpathtracer_amd as D
    import dxrpathtracer_amd._abi as A
    from dxrpathtracer_amd.distributed import NativeGather, PipelinedGather, screen_layout, source_index
    from dxrpathtracer_amd.tracer import DXRPathTracer

    T = args.phase_timeout
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream

    # ---- scene + acceleration structure (untimed, like the reference's InitializeScene + AS build)
    with wd.phase("setup", T):
        t0 = time.perf_counter()
        scene = D.Scene(SCENE)
        settings = scene.settings(MaxPathLength=PATH_LENGTH)
        sky = D.make_sky(settings)
        tracer = DXRPathTracer(device)
        tracer.initialize_scene(scene, sky)
        bvh = tracer.build_rt_acceleration_structure()
        setup_s = time.perf_counter() - t0
        lights = D.make_lights(scene)
        lay = screen_layout(WIDTH, HEIGHT, world, args.layout)
        tiles = lay.tile_array(rank) if world > 1 else None
        n_local = lay.counts[rank] if world > 1 else WIDTH * HEIGHT
        accum = torch.zeros((max(lay.max_count, n_local), 4), dtype=torch.float32, device="cuda")
        full = idx = None
        if world > 1 and rank == 0:
            full = torch.zeros((WIDTH * HEIGHT, 4), dtype=torch.float32, device="cuda")
            if args.gather == "torch":
                idx = torch.tensor(source_index(lay), dtype=torch.long, device="cuda")
        consts = [D.make_constants(scene, settings, sky, WIDTH, HEIGHT, s) for s in range(16)]

    # frame-end gather of the band slabs to rank 0 (RCCL), overlapped with the next frame's render
    pg = None
    gather_used = None
    if world > 1:
        with wd.phase("communicator", T):
            gather_used = args.gather
            if args.gather == "native":
                try:
                    pg = NativeGather(lay, rank, device, full, timing=True)
                except RuntimeError as e:  # e.g. an RCCL communicator that cannot be built on this node
                    # every rank takes the same branch (NativeGather's checks and results are all-gathered)
                    log(f"native gather unavailable ({e}); falling back to torch.distributed.gather")
                    gather_used = f"torch (native failed: {e})"
            if pg is None:
                if idx is None and rank == 0:
                    idx = torch.tensor(source_index(lay), dtype=torch.long, device="cuda")
                pg = PipelinedGather(lay, rank, full, idx)

    def render(f):
        tracer.render_raw(consts[f % 16], settings, accum.data_ptr(), WIDTH, HEIGHT, tiles=tiles, stream=sh,
                          lights=lights)

    def frame(f):
        render(f)
        if pg is not None:
            pg.submit(accum)

    def flush():
        if pg is not None:
            pg.flush()

    with wd.phase("census + per-launch timing", T):
        # ---- traversal work census (instrumented kernels, untimed): nodes / triangles per ray, split by the
        # kernel that traces them (depth 1: the split schedule's head; deeper: its tails).  The census runs
        # the counting instantiations of the schedule the timed frames run (k_path_head / k_path_tail with
        # kCount on depth-split frames; the single k_path's census walks the order of the register budget it
        # stands for), asserted below against the timed schedule.
        tracer.set_option(A.OPT_COUNT_TRAVERSAL, 1)
        frame(0)
        flush()
        census = tracer.stats()
        tracer.set_option(A.OPT_COUNT_TRAVERSAL, 0)

        # ---- per-launch kernel durations (untimed pass): the shipped kernels one frame at a time
        # (DXRPT_OPT_FRAME_OVERLAP 0), so each launch's HIP-event span is the launch alone -- with overlapped
        # frames a launch shares the GPU with the neighbour frames for part of its span.  The events are on
        # the stream the kernels run on (the render stream when frames do not overlap).  The pass pins the
        # timed frames' schedule (split or single k_path, register budgets, wave order), which the by-size
        # defaults would otherwise pick differently without overlap.
        for f in range(3):
            frame(f)
        flush()
        torch.cuda.synchronize()
        timed = tracer.stats()
        assert census.schedule & A.SCHED_CENSUS, census.schedule
        assert bool(census.schedule & A.SCHED_SPLIT) == bool(timed.schedule & A.SCHED_SPLIT), (census.schedule, timed.schedule)
        if not timed.schedule & A.SCHED_SPLIT:
            assert (census.occupancy <= 5) == (timed.occupancy <= 5), (census.occupancy, timed.occupancy)
        pinned = {A.OPT_MEGAKERNEL_SPLIT: 1 if timed.schedule & A.SCHED_SPLIT else 0,
                  A.OPT_MEGAKERNEL_OCCUPANCY: int(timed.occupancy),
                  A.OPT_TAIL_OCCUPANCY: int(timed.tail_occupancy) if timed.schedule & A.SCHED_SPLIT else 0,
                  A.OPT_WAVE_ORDER: 1 if timed.schedule & A.SCHED_ORDER_KERNEL else 0}
        for o, v in pinned.items():
            tracer.set_option(o, v)
        tracer.set_option(A.OPT_FRAME_OVERLAP, 0)
        for f in range(3):
            frame(f)
        flush()
        torch.cuda.synchronize()
        tracer.set_option(A.OPT_KERNEL_TIMING_MASK, (1 << A.K_COUNT) - 1)
        tracer.set_option(A.OPT_KERNEL_TIMING, 1)
        tracer.reset_timing()
        for f in range(min(args.steps, 32)):
            frame(f)
        flush()
        torch.cuda.synchronize()
        launches = tracer.stats()
        tracer.set_option(A.OPT_KERNEL_TIMING, 0)
        same = ~(A.SCHED_OVERLAP | A.SCHED_COST_ORDERED)
        assert launches.schedule & same == timed.schedule & same, (launches.schedule, timed.schedule)
        tracer.set_option(A.OPT_FRAME_OVERLAP, A.DEFAULT_FRAME_OVERLAP)
        for o, v in ((A.OPT_MEGAKERNEL_SPLIT, A.DEFAULT_MEGAKERNEL_SPLIT), (A.OPT_MEGAKERNEL_OCCUPANCY, A.DEFAULT_MEGAKERNEL_OCCUPANCY),
                     (A.OPT_TAIL_OCCUPANCY, A.DEFAULT_TAIL_OCCUPANCY), (A.OPT_WAVE_ORDER, A.DEFAULT_WAVE_ORDER)):
            tracer.set_option(o, v)
        per_launch = {A.KERNEL_NAMES[k]: {"avg_ms": launches.kernel_ms[k] / launches.kernel_launches[k],
                                          "launches_per_frame": launches.kernel_launches[k] / max(1, launches.timed_frames)}
                      for k in range(A.K_COUNT) if launches.kernel_launches[k]}
        frame_at_a_time_ms = launches.frame_ms / max(1, launches.timed_frames)

    with wd.phase("warmup + render-only throughput", T):
        for f in range(args.warmup):
            frame(f)
        flush()
        torch.cuda.synchronize()
        # this rank's own steady-state render throughput (no gather, no barrier): K back-to-back frames of
        # the shipped schedule, elapsed / K -- a throughput interval, not a per-frame event span (with frames
        # in flight a span on the render stream measures waits and the blend, not the frame)
        t_r = time.perf_counter()
        for f in range(args.steps):
            render(args.warmup + f)
        torch.cuda.synchronize()
        render_only_ms = (time.perf_counter() - t_r) / args.steps * 1e3

    # ---- timed region: the shipped defaults (overlapped frames), nothing but the frames between the
    # barrier + synchronize brackets.  (Through r06's first runs the loop also recorded two timing events per
    # frame on the render stream; each timing event is a marker packet the stream's queue has to pass, and
    # they cost 1-5 % of the interval -- C2 0.696 vs 0.663 ms render-only.  The per-frame spans now come from
    # their own untimed pass below; BENCH_TIMED_SPANS=1 puts the events back into the timed loop for an A/B.)
    spans_in_timed = os.environ.get("BENCH_TIMED_SPANS", "0") == "1"

    def span_pass(base):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        for f in range(args.steps):
            ev[f][0].record(stream)
            frame(base + f)
            ev[f][1].record(stream)
        return ev

    with wd.phase("timed frames", T):
        if hasattr(pg, "reset_times"):
            pg.reset_times()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t_start = time.perf_counter()
        if spans_in_timed:
            ev = span_pass(args.warmup)
        else:
            for f in range(args.steps):
                frame(args.warmup + f)
        flush()  # the last frame's gather + un-permute are inside the timed region
        torch.cuda.synchronize()
        local_elapsed = time.perf_counter() - t_start  # this rank, before the closing barrier
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t_start
        # the gather's own spans over the timed frames only (the span and latency passes below submit more)
        g_times = pg.times() if (world > 1 and hasattr(pg, "times")) else (None, None, 0)
    stats = tracer.stats()

    with wd.phase("frame spans", T):
        # per-frame event spans on the render stream (diagnostic, untimed): the same K frames again
        span_ms_per_frame = None
        if not spans_in_timed:
            torch.cuda.synchronize()
            t_s = time.perf_counter()
            ev = span_pass(args.warmup)
            flush()
            torch.cuda.synchronize()
            span_ms_per_frame = (time.perf_counter() - t_s) / args.steps * 1e3

    with wd.phase("frame latency", T):
        # paced passes (untimed for the headline): the reference's two frames of latency, and three (the
        # library's frames in flight)
        latency = [paced_latency(torch, stream, render, 48, ahead) for ahead in (2, 3)]
        # a progressive viewer's reset -> first image on an otherwise idle GPU (one frame, nothing in flight)
        idle = []
        for k in range(5):
            torch.cuda.synchronize()
            h = time.perf_counter()
            render(k)
            torch.cuda.synchronize()
            idle.append((time.perf_counter() - h) * 1e3)

    multi = None
    with wd.phase("collect", T):
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if args.dist_backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        frame_ms = np.array([a.elapsed_time(b) for a, b in ev])  # per frame on the render stream (incl. the gather's)
        nominal_per_frame = WIDTH * HEIGHT * (1 + 2 * (PATH_LENGTH - 1))
        ms_per_step = elapsed / args.steps * 1e3
        value = nominal_per_frame * args.steps / elapsed / 1e6
        if world > 1:
            per_rank = [None] * world
            dist.all_gather_object(per_rank, (render_only_ms, local_elapsed / args.steps * 1e3, n_local, device))
            g_ms, u_ms, g_frames = g_times
            render_max = max(v[0] for v in per_rank)
            multi = {"render_ms_per_rank": [round(v[0], 4) for v in per_rank], "render_ms_max": round(render_max, 4),
                     "render_ms_min": round(min(v[0] for v in per_rank), 4),
                     "render_what": "each rank's steady-state render throughput interval: elapsed / K over K "
                                    "back-to-back frames of its share, no gather, no barrier (bench.py run)",
                     "timed_ms_per_rank": [round(v[1], 4) for v in per_rank],
                     "timed_what": "each rank's own elapsed / K of the timed frames (with its gathers), before the "
                                   "closing barrier",
                     "share_pixels_per_rank": [int(v[2]) for v in per_rank],
                     "gather": gather_used,
                     "gather_ms": None if g_ms is None else round(g_ms, 4),
                     "unpermute_ms": None if u_ms is None else round(u_ms, 4),
                     "gather_frames_timed": g_frames,
                     "rccl_ranks": getattr(pg, "comm_ranks", None),
                     "dist_backend": args.dist_backend,
                     "devices": [int(v[3]) for v in per_rank],
                     "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "runtime default (4)"),
                     # the part of the job's frame interval the gather adds beyond the slowest rank's own
                     # render throughput (difference of throughput intervals)
                     "gather_exposed_ms": round(ms_per_step - render_max, 4),
                     "gather_how": "dxrpt_gather_slabs (grouped ncclSend/ncclRecv of every rank's slab to rank 0) "
                                   "timed with events on the render stream, dxrpt_unpermute on rank 0's render stream"}

    # ---- roofline of the dominant kernel, per launch (SURVEY.md 8(d) bytes / the launch's own duration)
    parts = census_parts(census, n_local, PATH_LENGTH)
    part_bytes = {k: full_formula_bytes(v, settings, bvh) for k, v in parts.items()}
    frame_bytes = part_bytes["frame"][0]
    kern = {}
    if "k_path_head" in per_launch:  # the depth-split schedule: head (depth 1) and tails (depths >= 2)
        for name, part in (("k_path_head", "head"), ("k_path_tail", "tail")):
            if name in per_launch:
                n = per_launch[name]["launches_per_frame"]
                kern[name] = {"bytes_per_launch": part_bytes[part][0] / n, "avg_launch_ms": per_launch[name]["avg_ms"],
                              "launches_per_frame": n, "bytes_part": part}
    elif "k_path" in per_launch:
        kern["k_path"] = {"bytes_per_launch": frame_bytes, "avg_launch_ms": per_launch["k_path"]["avg_ms"],
                          "launches_per_frame": 1.0, "bytes_part": "frame"}
    for k, e in kern.items():
        e["achieved"] = e["bytes_per_launch"] / (e["avg_launch_ms"] * 1e-3) / 1e9
        e["frac"] = e["achieved"] / HBM_PEAK_GBS
    dominant = max(kern, key=lambda k: kern[k]["avg_launch_ms"] * kern[k]["launches_per_frame"]) if kern else None
    pmc, pmc_src = pmc_kernels(args.config)
    pk = pmc.get("kernels_by_kind") or {}
    for k, e in kern.items():
        c = pk.get(k, {})
        e["pmc_avg_launch_ms"] = c.get("avg_ms")
        e["traffic"] = c.get("l2_fabric_bytes_per_launch")
        e["write_bytes"] = c.get("write_bytes_per_launch")
        e["l2_hit_rate"] = c.get("l2_hit_rate")
        e["wait_any_per_wave_cycle"] = c.get("wait_any_per_wave_cycle")
        e["valu_lane_utilisation"] = c.get("valu_lane_utilisation")
    d = kern.get(dominant, {})
    wait_frac = d.get("wait_any_per_wave_cycle")
    achieved = d.get("achieved", 0.0)
    # what limits the kernel, from its counters: waves parked on s_waitcnt for much of their cycles with
    # HBM far from its peak = latency of dependent loads (the roofline is still priced against HBM)
    limiter = "latency" if (wait_frac is not None and wait_frac > 0.3 and achieved < 0.6 * HBM_PEAK_GBS) else "hbm"
    # the shipped throughput rate: this rank's frame bytes over the job's frame interval (elapsed / K, a
    # throughput interval -- never a median of event spans, which with frames in flight bunch around the
    # blends); cross-checked against the mean of the render-stream frame spans
    fi_ms = ms_per_step
    fi_gbs = frame_bytes / (fi_ms * 1e-3) / 1e9
    span_mean = float(frame_ms.mean())
    fi_consistent = abs(span_mean - fi_ms) <= 0.05 * fi_ms
    assert fi_gbs <= HBM_PEAK_GBS, f"frame-interval rate {fi_gbs:.0f} GB/s above the HBM peak: a timing error"
    if not fi_consistent:
        log(f"warning: mean frame span {span_mean:.4f} ms vs frame interval {fi_ms:.4f} ms (> 5 % apart)")

    def r4(v):
        return round(v, 4) if isinstance(v, float) else v

    result = None
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            with wd.phase("cpu baseline", max(T, 600.0)):
                cpu = cpu_baseline(scene, sky, settings, args.cpu_threads)
        result = {
            "metric": metric,
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic: seeded procedural {SCENE.capitalize()} proxy ({'Sponza.fbx' if SCENE == 'sponza' else 'SunTemple.fbx'} "
                    "absent from the reference snapshot)",
            "config": {"workload": f"{SCENE}-proxy {WIDTH}x{HEIGHT} L={PATH_LENGTH} 1spp/frame progressive",
                       "width": WIDTH, "height": HEIGHT, "max_path_length": PATH_LENGTH,
                       "sqrt_num_samples": 4, "triangles": scene.num_triangles, "sky": sky.model,
                       "parallelism": (f"screen {args.layout} x{world} + RCCL gather ({gather_used})" if world > 1
                                       else "single GPU")},
            # the roofline this kernel is priced against (no MFMA on this path); "limiter": what its counters
            # say holds it below that roof
            "roofline": {"bound": "hbm", "limiter": limiter, "kernel": dominant,
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": d.get("traffic"),
                         "traffic_kind": "L2->fabric bytes per launch (rocprofv3 FETCH_SIZE + WRITE_SIZE, raw, no x2 "
                                         "read correction): Infinity-Cache hits included, so not HBM bytes",
                         "traffic_source": pmc_src,
                         "bytes_per_launch": int(d.get("bytes_per_launch", 0)),
                         "bytes_formula": "SURVEY.md 8(d) full formula over the rays this kernel traces (census split "
                                          "by depth: head = depth 1, tails = depths >= 2)",
                         "avg_launch_ms": r4(d.get("avg_launch_ms", 0.0)),
                         "achieved_over": "the kernel's average launch duration: HIP events on its stream in a "
                                          "frame-at-a-time pass (DXRPT_OPT_FRAME_OVERLAP 0) inside bench.py",
                         "pmc_avg_launch_ms": d.get("pmc_avg_launch_ms"),
                         "l2_hit_rate": d.get("l2_hit_rate"), "hbm_write_bytes": d.get("write_bytes"),
                         "wait_any_per_wave_cycle": wait_frac,
                         "valu_lane_utilisation": d.get("valu_lane_utilisation"),
                         "per_kernel": {k: {kk: r4(vv) for kk, vv in e.items()} for k, e in kern.items()},
                         # the shipped throughput rate: the frame's bytes over the job's frame interval
                         # (elapsed / K with up to three frames in flight: not a launch duration)
                         "frame_interval": {"bytes": int(frame_bytes), "ms": round(fi_ms, 4),
                                            "what": "elapsed / steps of the timed region (ms_per_step)",
                                            "achieved": round(fi_gbs, 1), "frac": round(fi_gbs / HBM_PEAK_GBS, 4),
                                            "mean_frame_span_ms": round(span_mean, 4),
                                            "span_pass": "timed loop" if spans_in_timed else
                                            "an untimed pass of the same K frames with two timing events per frame",
                                            "span_pass_ms_per_frame": r4(span_ms_per_frame),
                                            "consistent_within_5pct": bool(fi_consistent),
                                            "frame_at_a_time_ms": round(frame_at_a_time_ms, 4)}},
            "cpu_baseline": cpu,
            # the headline counts the reference's HUD rays (W*H*(1+2(L-1)) per frame); the kernels skip
            # shadow rays whose pending contribution is exactly 0 (identical image), so fewer are traced:
            "nominal_rays_per_frame": nominal_per_frame,
            "counted_rays_per_frame": int(stats.radiance_rays + stats.shadow_rays),
            "counted_Mrays_s": round((stats.radiance_rays + stats.shadow_rays) * args.steps / elapsed / 1e6, 2)
            if world == 1 else None,
            "multi_gpu": multi,
            "detail": {
                "per_launch_kernel_ms": {k: {kk: round(vv, 4) for kk, vv in v.items()} for k, v in per_launch.items()},
                "schedule": schedule_name(stats.schedule, A),
                "schedule_bits": int(stats.schedule),
                "frame_at_a_time_schedule_bits": int(launches.schedule),
                "occupancy": {"head_or_path": int(stats.occupancy), "tail": int(stats.tail_occupancy)},
                "algorithmic_bytes": {k: v[1] for k, v in part_bytes.items()},
                # per-frame event spans on the render stream: with frames in flight they measure the waits for
                # the slot streams and the blend, so they bunch (median << mean); only the mean is a rate
                "frame_span_ms": {"mean": round(span_mean, 4), "median": round(float(np.median(frame_ms)), 4),
                                  "max": round(float(frame_ms.max()), 4)},
                "render_only_ms_per_frame": round(render_only_ms, 4),
                # submit -> blended latency (the reference bounds it at RenderLatency = 2 frames,
                # Graphics/DX12.h:21); unpaced submission has no bounded latency (the host runs ahead)
                "frame_latency": {"paced": latency,
                                  "idle_gpu_one_frame_ms": {"median": round(float(np.median(idle)), 4),
                                                            "max": round(float(max(idle)), 4)}},
                "census": {"what": "node / triangle-record fetches of the timed schedule (per lane in per-lane "
                                   "traversals, per wave in packet traversals), one instrumented frame of the "
                                   "timed kernels' counting instantiations",
                           "kernels": ("k_path_head<count> + k_path_tail<7,count>" if census.schedule & A.SCHED_SPLIT
                                       else f"k_path<{5 if census.occupancy <= 5 else 7},count>"),
                           "schedule_bits": int(census.schedule),
                           "node_fetches_radiance": int(census.node_visits_radiance),
                           "tri_fetches_radiance": int(census.tri_tests_radiance),
                           "node_fetches_shadow": int(census.node_visits_shadow),
                           "tri_fetches_shadow": int(census.tri_tests_shadow),
                           "depth1": [int(v) for v in census.census_depth1],
                           "radiance_rays_per_depth": [int(v) for v in census.radiance_rays_per_depth],
                           "shadow_rays_per_depth": [int(v) for v in census.shadow_rays_per_depth],
                           "node_bytes": int(bvh.node_bytes), "tri_bytes": int(bvh.tri_bytes),
                           "accum_bytes_per_pixel": ACCUM_BYTES, "pixels": int(n_local)},
                "node_fetches_per_radiance_ray": round(census.node_visits_radiance / max(1, census.radiance_rays), 2),
                "tri_fetches_per_radiance_ray": round(census.tri_tests_radiance / max(1, census.radiance_rays), 2),
                "node_fetches_per_shadow_ray": round(census.node_visits_shadow / max(1, census.shadow_rays), 2),
                "tri_fetches_per_shadow_ray": round(census.tri_tests_shadow / max(1, census.shadow_rays), 2),
                "bvh": {"nodes": bvh.num_nodes, "refs": bvh.num_refs, "max_depth": bvh.max_depth,
                        "build_ms": round(bvh.build_ms, 1),
                        "build_phase_ms": {n: round(bvh.phase_ms[i], 1) for i, n in enumerate(A.BVH_PHASES)},
                        "build_threads": bvh.threads, "binary_depth_cap": bvh.binary_depth_cap,
                        "treelet_passes": bvh.treelet_passes, "ref_budget_pct": bvh.ref_budget_pct,
                        "sah": round(bvh.sah_cost, 2), "wide_sah": round(bvh.wide_sah, 3)},
                # material taps actually issued per hit: the SURVEY 8(d) byte formula keeps five taps; packed
                # normal/metallic/roughness maps and inlined 1 x 1 maps (DXRPT_OPT_PACKED_TAPS) read fewer
                "material_maps": {"packed_materials": int(stats.packed_materials),
                                  "packed_textures": int(stats.packed_textures),
                                  "inlined_maps": int(stats.inlined_maps)},
                "setup_s": round(setup_s, 2),
            },
        }
        print(json.dumps(result), flush=True)
    with wd.phase("teardown", T):
        if world > 1:
            if hasattr(pg, "close"):
                pg.close()
            dist.barrier()
            dist.destroy_process_group()
        tracer.close()


if __name__ == "__main__":
    main()
