#!/usr/bin/env python3
"""Benchmark of the path tracer on BASELINE.json's metric config: Sponza(-proxy) 1920x1080,
MaxPathLength 3, one sample per pixel per frame with progressive accumulation.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

A step is one frame (DispatchRays(1920,1080,1) equivalent, DXRPathTracer.cpp:2024-2090) over the whole
image.  With N ranks the image is split into 8-row bands, band b -> rank b % N (distributed.band_layout;
--layout blocks: 8x8-pixel blocks dealt in a seeded random order) and every frame ends
with an RCCL gather of the rank slabs to rank 0 plus the un-permute: total work per
frame is fixed, so scaling is "strong".  The gather of frame f runs on RCCL's stream while frame f+1
renders (distributed.PipelinedGather); the last frame's gather is inside the timed region.  value = nominal Mrays/s of the whole job (W*H*(1+2(L-1))
rays per frame, the reference's HUD formula DXRPathTracer.cpp:2171) over the max-over-ranks time.
Rank 0 prints one JSON line.
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

WIDTH, HEIGHT, PATH_LENGTH = 1920, 1080, 3
SCENE = "sponza"
# BASELINE.json configs, selectable with --config (the default is the metric's; the others are the
# parity configs, timed the same way for the record): name -> (scene, width, height, path length)
CONFIGS = {"metric": ("sponza", 1920, 1080, 3), "c2": ("sponza", 1280, 720, 3), "c3": ("sponza", 1920, 1080, 8),
           "c4": ("suntemple", 1920, 1080, 3), "c5": ("sponza", 3840, 2160, 6)}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "Mrays/sec + ms/frame, Sponza 1920x1080 path-length 3 at 1/2/4/8 GPU"
# Algorithmic bytes, per ray, plus the BVH nodes (80 B) and triangle records (48 B) it
# visits (counted by the instrumented kernels):
#   k_trace  (closest hit): 32 B ray in (2 x float4) + 16 B hit out
#   k_shadow (any hit):     4 B queue entry + 48 B shadow slot in (origin, direction, contribution);
#                           the 16-B contribution write of occluded rays is not counted (lower bound)
#   k_path   (megakernel, one launch per frame): all of the above + 32 B accumulation RMW per pixel
RAY_IN_BYTES, HIT_OUT_BYTES = 32, 16
SHADOW_IN_BYTES = 52
ACCUM_BYTES = 32


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


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` (k_trace / k_shadow) from the committed rocprofv3 PMC summary, if
    one exists for this config (profiles/*_pmc_<kernel>.json, written by scripts/pmc_summary.py)."""
    import glob
    for p in sorted(glob.glob(os.path.join(REPO, "profiles", f"*_pmc_{kernel}.json")), reverse=True):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("config") == f"{SCENE}-proxy {WIDTH}x{HEIGHT} L={PATH_LENGTH}":
            return d, os.path.basename(p)
    return {}, None


def pmc_frame(config):
    """Per-FRAME counters of the megakernel schedule (k_path, or the split schedule's head + tails) from
    the newest committed summary for this config (profiles/<round>_pmc_frame_<config>.json, written by
    scripts/pmc_summary.py over scripts/profile.sh's rocprofv3 passes)."""
    import glob
    for p in sorted(glob.glob(os.path.join(REPO, "profiles", f"*_pmc_frame_{config}.json")), reverse=True):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("config") == f"{SCENE}-proxy {WIDTH}x{HEIGHT} L={PATH_LENGTH}":
            return d, os.path.basename(p)
    return {}, None


def full_formula_bytes(census, settings, bvh, pixels):
    """SURVEY.md 8(d)'s algorithmic bytes of one frame, term by term as the survey writes them:
      per ray: 32 B in (o, d, tmax, flags) + 16 B hit out (radiance) or 4 B visibility (shadow)
               + N_node x S_node + N_tri x S_tri (the census' fetches of the timed schedule)
      per radiance hit: 12 (3 indices) + 192 (3 vertices) + 16 (GeometryInfo) + 24 (Material)
               + taps x 4 texels x 4 B (RGBA8: normal, albedo if enabled; metallic, roughness, emissive)
               + 64 (path-state RMW) + 32 (next-ray write) + 32 (shadow-ray write)
      per miss: 4 x 8 B (FP16 cube bilinear)
      + 32 B accumulation RMW per pixel.
    Alpha-test opacity taps of any-hit candidates are not counted (a lower bound for C4)."""
    hits = int(census.radiance_hits)
    misses = int(census.radiance_rays) - hits
    taps = 3 + int(settings.EnableNormalMaps) + int(settings.EnableAlbedoMaps)
    per_hit = 12 + 192 + 16 + 24 + taps * 16 + 64 + 32 + 32
    terms = {
        "radiance_ray_io": int(census.radiance_rays) * (32 + 16),
        "shadow_ray_io": int(census.shadow_rays) * (32 + 4),
        "bvh_node_fetches": int(census.node_visits_radiance + census.node_visits_shadow) * int(bvh.node_bytes),
        "triangle_fetches": int(census.tri_tests_radiance + census.tri_tests_shadow) * int(bvh.tri_bytes),
        "radiance_hit_shading": hits * per_hit,
        "miss_sky_taps": misses * 32,
        "accumulation": ACCUM_BYTES * int(pixels),
    }
    return sum(terms.values()), {"terms": terms, "radiance_hits": hits, "misses": misses,
                                 "taps_per_hit": taps, "bytes_per_hit": per_hit}


def schedule_name(bits, ppw, A):
    if not bits & A.SCHED_MEGAKERNEL:
        return "wavefront passes"
    if bits & A.SCHED_SPLIT:
        return ("depth-split megakernel (k_path_head + k_path_tail per depth)"
                + (", two concurrent halves" if bits & A.SCHED_PARTS else "")
                + (", overlapped frames" if bits & A.SCHED_OVERLAP else ""))
    s = "megakernel (k_path)"
    if bits & A.SCHED_PATH_GROUPS:
        s += f", path groups ({ppw} paths per wave)"
    if bits & A.SCHED_COST_ORDERED:
        s += ", cost-ordered waves"
    if bits & A.SCHED_OVERLAP:
        s += ", overlapped frames"
    return s


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
    args = ap.parse_args()
    global SCENE, WIDTH, HEIGHT, PATH_LENGTH
    SCENE, WIDTH, HEIGHT, PATH_LENGTH = CONFIGS[args.config]
    metric = METRIC if args.config == "metric" else \
        f"Mrays/sec + ms/frame, {SCENE.capitalize()} {WIDTH}x{HEIGHT} path-length {PATH_LENGTH} (BASELINE config {args.config})"

    import torch
    import torch.distributed as dist
    import dxrpathtracer_amd as D
    import dxrpathtracer_amd._abi as A
    from dxrpathtracer_amd.distributed import NativeGather, PipelinedGather, screen_layout, source_index
    from dxrpathtracer_amd.tracer import DXRPathTracer

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream

    # ---- scene + acceleration structure (untimed, like the reference's InitializeScene + AS build)
    t0 = time.perf_counter()
    scene = D.Scene(SCENE)
    settings = scene.settings(MaxPathLength=PATH_LENGTH)
    sky = D.make_sky(settings)
    tracer = DXRPathTracer(local_rank)
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
        gather_used = args.gather
        if args.gather == "native":
            try:
                pg = NativeGather(lay, rank, local_rank, full)
            except RuntimeError as e:  # e.g. an RCCL communicator that cannot be built on this node
                # every rank takes the same branch (dxrpt_comm_create is collective: it fails on all ranks)
                log(f"native gather unavailable ({e}); falling back to torch.distributed.gather")
                gather_used = f"torch (native failed: {e})"
        if pg is None:
            if idx is None and rank == 0:
                idx = torch.tensor(source_index(lay), dtype=torch.long, device="cuda")
            pg = PipelinedGather(lay, rank, full, idx)

    def frame(f):
        tracer.render_raw(consts[f % 16], settings, accum.data_ptr(), WIDTH, HEIGHT, tiles=tiles, stream=sh,
                          lights=lights)
        if pg is not None:
            pg.submit(accum)

    def flush():
        if pg is not None:
            pg.flush()

    # ---- traversal work census (instrumented kernels, untimed): nodes / triangles per ray
    tracer.set_option(A.OPT_COUNT_TRAVERSAL, 1)
    frame(0)
    flush()
    census = tracer.stats()
    tracer.set_option(A.OPT_COUNT_TRAVERSAL, 0)

    for f in range(args.warmup):
        frame(f)
    flush()
    torch.cuda.synchronize()

    # ---- per-kernel breakdown (all kinds, untimed pass before the timed region): picks the dominant
    # kernel whose roofline is reported.  ~26 events per frame cost ~0.1 ms of frame time, so the timed
    # region below brackets only the dominant kernel's launches (plus the frame span).
    tracer.set_option(A.OPT_KERNEL_TIMING_MASK, (1 << A.K_COUNT) - 1)
    tracer.set_option(A.OPT_KERNEL_TIMING, 1)
    tracer.reset_timing()
    for f in range(min(args.steps, 16)):
        frame(f)
    flush()
    torch.cuda.synchronize()
    breakdown = tracer.stats()
    kms = {A.KERNEL_NAMES[k]: breakdown.kernel_ms[k] for k in range(A.K_COUNT)}
    dominant = max(kms, key=kms.get)
    roof_kernel = dominant if dominant in ("k_trace", "k_shadow", "k_path") else "k_trace"
    K_ROOF = {"k_trace": A.K_TRACE, "k_shadow": A.K_SHADOW, "k_path": A.K_PATH}[roof_kernel]

    # ---- timed region: production schedule (any-hit / closest-hit stream overlap), events on the
    # launching streams around the roofline kernel's launches only
    tracer.set_option(A.OPT_KERNEL_TIMING_MASK, 1 << K_ROOF)
    tracer.reset_timing()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for f in range(args.steps):
        ev[f][0].record(stream)
        frame(args.warmup + f)
        ev[f][1].record(stream)
    flush()  # the last frame's gather + un-permute are inside the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    stats = tracer.stats()
    tracer.set_option(A.OPT_KERNEL_TIMING, 0)
    roof_ms_avg = stats.kernel_ms[K_ROOF] / max(1, stats.kernel_launches[K_ROOF])
    gpu_frame_ms = stats.frame_ms / max(1, stats.timed_frames)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    frame_ms = np.array([a.elapsed_time(b) for a, b in ev])  # per frame on the render stream
    nominal_per_frame = WIDTH * HEIGHT * (1 + 2 * (PATH_LENGTH - 1))
    ms_per_step = elapsed / args.steps * 1e3
    value = nominal_per_frame * args.steps / elapsed / 1e6

    # ---- roofline of the dominant kernel (measured live with HIP events on its launching stream)
    launches_per_frame = PATH_LENGTH - 1  # one closest-hit and one any-hit pass per depth
    trace_bytes_frame = (census.radiance_rays * (RAY_IN_BYTES + HIT_OUT_BYTES)
                         + census.node_visits_radiance * bvh.node_bytes + census.tri_tests_radiance * bvh.tri_bytes)
    shadow_bytes_frame = (census.shadow_rays * SHADOW_IN_BYTES
                          + census.node_visits_shadow * bvh.node_bytes + census.tri_tests_shadow * bvh.tri_bytes)
    # k_path (the whole frame in one launch, rays and path state in registers): the node and triangle
    # FETCHES its census counted (per lane in the per-lane traversals, once per wave in the packet
    # traversals) + the accumulation RMW; the shading gathers are not counted, so it is a lower bound
    fetch_bytes_frame = ((census.node_visits_radiance + census.node_visits_shadow) * bvh.node_bytes
                         + (census.tri_tests_radiance + census.tri_tests_shadow) * bvh.tri_bytes)
    path_bytes_lower = fetch_bytes_frame + ACCUM_BYTES * n_local
    path_bytes_full, full_detail = full_formula_bytes(census, settings, bvh, n_local)
    # k_path: the survey's full formula (census of the timed schedule); the fetch-only figure stays beside it
    roof_bytes = {"k_trace": trace_bytes_frame / launches_per_frame, "k_shadow": shadow_bytes_frame / launches_per_frame,
                  "k_path": path_bytes_full}[roof_kernel]
    achieved_launch = roof_bytes / (roof_ms_avg * 1e-3) / 1e9
    # Overlapped frames (DXRPT_SCHED_OVERLAP): a launch's event span runs from its stream becoming ready
    # (while the previous frame still holds the GPU) to its end, so it overlaps its neighbours' spans; the
    # steady-state frame interval (per-frame events on the render stream) is the time the GPU spends per
    # launch, and prices the kernel's bytes.  Without overlap the two agree.
    frame_interval_ms = float(np.median(np.array([a.elapsed_time(b) for a, b in ev])))
    overlapped = bool(stats.schedule & A.SCHED_OVERLAP)
    achieved = roof_bytes / (frame_interval_ms * 1e-3) / 1e9 if overlapped and roof_kernel == "k_path" else achieved_launch
    pmc, traffic_src = pmc_traffic(roof_kernel)
    traffic = pmc.get("hbm_bytes_per_launch")
    l2_hit = pmc.get("l2_hit_rate")
    wait_frac = pmc.get("wait_any_per_wave_cycle")
    write_bytes = pmc.get("hbm_write_bytes_per_launch")
    if roof_kernel == "k_path":  # per-frame PMC summary of the megakernel schedule of this config
        fr, src = pmc_frame(args.config)
        if fr:
            traffic, traffic_src = fr.get("hbm_bytes_per_frame"), src
            l2_hit, wait_frac, write_bytes = fr.get("l2_hit_rate"), fr.get("wait_any_per_wave_cycle"), fr.get("hbm_write_bytes")
            pmc = {"kernel": " + ".join(fr.get("kernels", []))}
    # what limits the kernel, from its counters: waves parked on s_waitcnt for most of their cycles with
    # HBM far from its peak = latency of dependent loads (the roofline below is still priced against HBM)
    bound = "latency" if (wait_frac is not None and wait_frac > 0.3 and achieved < 0.6 * HBM_PEAK_GBS) else "hbm"
    # the other traversal kernel, from the breakdown pass (for the record; wavefront schedule only)
    other = "k_shadow" if roof_kernel == "k_trace" else "k_trace"
    K_OTHER = A.K_SHADOW if other == "k_shadow" else A.K_TRACE
    other_ms = breakdown.kernel_ms[K_OTHER] / max(1, breakdown.kernel_launches[K_OTHER])
    other_bytes = (shadow_bytes_frame if other == "k_shadow" else trace_bytes_frame) / launches_per_frame
    other_pmc, _ = pmc_traffic(other)

    result = None
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(scene, sky, settings, args.cpu_threads)
        frames = breakdown.timed_frames or 1
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
            "roofline": {"bound": bound, "roofline_kind": "hbm",
                         "kernel": ("k_path_head + k_path_tail (one frame)" if roof_kernel == "k_path" and stats.schedule & A.SCHED_SPLIT
                                    else roof_kernel), "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "bytes_per_launch": int(roof_bytes),
                         "bytes_formula": "SURVEY.md 8(d) full formula" if roof_kernel == "k_path" else "per-ray I/O + fetches",
                         "bytes_fetch_lower_bound": int(path_bytes_lower) if roof_kernel == "k_path" else None,
                         "frac_fetch_lower_bound": round(path_bytes_lower / (roof_bytes / achieved * 1e-9) / 1e9 / HBM_PEAK_GBS, 4)
                         if roof_kernel == "k_path" else None,
                         "avg_launch_ms": round(roof_ms_avg, 4), "traffic_source": traffic_src,
                         "traffic_kernel": pmc.get("kernel"), "l2_hit_rate": l2_hit,
                         "hbm_write_bytes": write_bytes, "wait_any_per_wave_cycle": wait_frac,
                         # overlapped frames (DXRPT_SCHED_OVERLAP): a launch shares the GPU with its
                         # neighbour frames for part of its event span, so the per-launch figure above
                         # understates the kernel; the steady-state frame interval prices the same bytes
                         "frames_overlap": overlapped,
                         "achieved_over": "steady-state frame interval (median per-frame events)" if overlapped
                         and roof_kernel == "k_path" else "average launch span (HIP events on the launching stream)",
                         "frame_interval_ms": round(frame_interval_ms, 4),
                         "achieved_launch_span": round(achieved_launch, 1),
                         "frac_launch_span": round(achieved_launch / HBM_PEAK_GBS, 4)},
            "cpu_baseline": cpu,
            # the headline counts the reference's HUD rays (W*H*(1+2(L-1)) per frame); the kernels skip
            # shadow rays whose pending contribution is exactly 0 (identical image), so fewer are traced:
            "nominal_rays_per_frame": nominal_per_frame,
            "counted_rays_per_frame": int(stats.radiance_rays + stats.shadow_rays),
            "counted_Mrays_s": round((stats.radiance_rays + stats.shadow_rays) * args.steps / elapsed / 1e6, 2)
            if world == 1 else None,
            "detail": {
                "kernel_ms_per_frame": {k: round(v / frames, 4) for k, v in kms.items()},
                "dominant_kernel": dominant,
                "roofline_other": {"kernel": other, "bytes_per_launch": int(other_bytes),
                                   "avg_launch_ms": round(other_ms, 4),
                                   "achieved_GBs": round(other_bytes / (other_ms * 1e-3) / 1e9, 1),
                                   "traffic": other_pmc.get("hbm_bytes_per_launch"),
                                   "l2_hit_rate": other_pmc.get("l2_hit_rate")} if other_ms > 0 else None,
                "schedule": schedule_name(stats.schedule, stats.paths_per_wave, A),
                "schedule_bits": int(stats.schedule),
                "algorithmic_bytes": full_detail,
                "gpu_frame_ms_events": round(gpu_frame_ms, 4),
                "kernel_breakdown_note": "kernel_ms_per_frame from a separate all-kernel event pass before the timed region",
                "frame_ms": {"mean": round(float(frame_ms.mean()), 4), "median": round(float(np.median(frame_ms)), 4),
                             "max": round(float(frame_ms.max()), 4)},
                "census": {"what": "node / triangle-record fetches of the timed schedule (per lane in per-lane "
                                   "traversals, per wave in packet traversals), one instrumented frame",
                           "node_fetches_radiance": int(census.node_visits_radiance),
                           "tri_fetches_radiance": int(census.tri_tests_radiance),
                           "node_fetches_shadow": int(census.node_visits_shadow),
                           "tri_fetches_shadow": int(census.tri_tests_shadow),
                           "node_bytes": int(bvh.node_bytes), "tri_bytes": int(bvh.tri_bytes),
                           "accum_bytes_per_pixel": ACCUM_BYTES, "pixels": int(n_local)},
                "node_fetches_per_radiance_ray": round(census.node_visits_radiance / max(1, census.radiance_rays), 2),
                "tri_fetches_per_radiance_ray": round(census.tri_tests_radiance / max(1, census.radiance_rays), 2),
                "node_fetches_per_shadow_ray": round(census.node_visits_shadow / max(1, census.shadow_rays), 2),
                "tri_fetches_per_shadow_ray": round(census.tri_tests_shadow / max(1, census.shadow_rays), 2),
                "bvh": {"nodes": bvh.num_nodes, "max_depth": bvh.max_depth, "build_ms": round(bvh.build_ms, 1),
                        "sah": round(bvh.sah_cost, 2)},
                "setup_s": round(setup_s, 2),
            },
        }
        print(json.dumps(result), flush=True)
    if world > 1:
        if hasattr(pg, "close"):
            pg.close()
        dist.barrier()
        dist.destroy_process_group()
    tracer.close()


if __name__ == "__main__":
    main()
