"""Screen-space sharding across GPUs of one node + the frame-end gather.

The reference is single-GPU; every pixel's path is independent and the CMJ pattern uses only the
GLOBAL pixel index (RayTrace.hlsl:85-96), so any partition of the image renders bit-identical pixels.
Rank r path-traces its share of the image -- bands b = r, r+N, r+2N, ... of `band` full rows
(band_layout, the default), or 8x8 pixel blocks dealt in a seeded random order (block_layout) -- into a
compact local buffer (dxrpt_tile accum_offset/pitch), and rank 0 gathers the slabs
(torch.distributed: RCCL over xGMI on the GPU node, gloo in the CPU tests) and un-permutes them into
the full RGBA32F frame.
"""
from __future__ import annotations

from dataclasses import dataclass

from . import _abi as A

# 8-row bands (one 8x8-pixel-block row per band, the megakernel's wave footprint): 1080 rows over 8
# ranks = 135 bands, 17 or 16 per rank.  Chosen by the SLOWEST rank's share, which is what an N-GPU
# frame waits for: all 8 ranks' 1/8 shares with the shipped schedule take at most 0.557 ms with 8-row,
# 0.575 with 16-row and 0.595 with 32-row bands (profiles/r02_ab_band_height_all_ranks.txt).
BAND_ROWS = 8


@dataclass
class BandLayout:
    width: int
    height: int
    world: int
    band: int
    tiles: list          # tiles[r] = list of dxrpt Tile for rank r (compact accum offsets)
    counts: list         # pixels owned by each rank
    max_count: int       # padded slab size (pixels) used by the equal-size gather

    def rank_tiles(self, rank: int):
        return self.tiles[rank]

    def tile_array(self, rank: int):
        """Rank `rank`'s tiles as a ctypes Tile array, built once per layout and rank (DXRPathTracer.render_raw
        passes it to dxrpt_render without re-marshalling).  Layouts are not edited after construction."""
        cache = self.__dict__.setdefault("_arrays", {})
        if rank not in cache:
            t = self.tiles[rank]
            cache[rank] = (A.Tile * len(t))(*t)
        return cache[rank]


def band_layout(width: int, height: int, world: int, band: int = BAND_ROWS) -> BandLayout:
    tiles = [[] for _ in range(world)]
    counts = [0] * world
    for b, y0 in enumerate(range(0, height, band)):
        r = b % world
        h = min(band, height - y0)
        tiles[r].append(A.Tile(0, y0, width, h, counts[r], width, 0))
        counts[r] += width * h
    return BandLayout(width, height, world, band, tiles, counts, max(counts))


def balanced_band_layout(width: int, height: int, world: int, costs, band: int = BAND_ROWS) -> BandLayout:
    """Bands dealt to the ranks by cost (longest-processing-time first): bands in decreasing `costs[b]`
    (ties: lower band first), each to the rank with the least cost so far (ties: lower rank).  Every rank
    renders its bands top to bottom.  Deterministic: every rank computes the same layout from the same
    costs (e.g. per-band wave time of an earlier frame, scripts/band_balance.py)."""
    nb = (height + band - 1) // band
    if len(costs) != nb:
        raise ValueError(f"balanced_band_layout: {len(costs)} costs for {nb} bands")
    load = [0.0] * world
    owner = [0] * nb
    for b in sorted(range(nb), key=lambda b: (-float(costs[b]), b)):
        r = min(range(world), key=lambda r: (load[r], r))
        owner[b] = r
        load[r] += float(costs[b])
    tiles = [[] for _ in range(world)]
    counts = [0] * world
    for b in range(nb):
        r, y0 = owner[b], b * band
        h = min(band, height - y0)
        tiles[r].append(A.Tile(0, y0, width, h, counts[r], width, 0))
        counts[r] += width * h
    return BandLayout(width, height, world, band, tiles, counts, max(counts))


def _mix64(x: int) -> int:
    """splitmix64 finaliser: the partition's only source of pseudo-randomness (deterministic)."""
    x = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return x ^ (x >> 31)


def block_layout(width: int, height: int, world: int, block: int = 8, seed: int = 0x5EED) -> BandLayout:
    """Cost-spreading partition: the image's block x block pixel blocks (one megakernel wave each) are
    dealt to the ranks in a seeded pseudo-random order, round robin, so every rank receives an equal
    number of blocks drawn from the whole image.  The expensive blocks of a frame -- measured with
    scripts/wave_clocks.py: alpha-tested foliage, clustered in a few block rows -- land on all ranks
    instead of on the one that owns those rows, which is what an N-GPU frame waits for.  Each rank
    renders its blocks in raster order (tiles of block x block pixels, compact in its slab); pixels,
    CMJ seeds and results are those of the full frame (global pixel indices)."""
    nbx, nby = (width + block - 1) // block, (height + block - 1) // block
    order = sorted(range(nbx * nby), key=lambda b: (_mix64(b ^ (seed << 32)), b))
    owner = [0] * (nbx * nby)
    for k, b in enumerate(order):
        owner[b] = k % world
    tiles = [[] for _ in range(world)]
    counts = [0] * world
    for b in range(nbx * nby):
        r = owner[b]
        x0, y0 = (b % nbx) * block, (b // nbx) * block
        w, h = min(block, width - x0), min(block, height - y0)
        tiles[r].append(A.Tile(x0, y0, w, h, counts[r], w, 0))
        counts[r] += w * h
    return BandLayout(width, height, world, block, tiles, counts, max(counts))


def screen_layout(width: int, height: int, world: int, kind: str = "bands") -> BandLayout:
    """The multi-GPU screen partition: "bands" (band_layout, default) or "blocks" (block_layout).  Measured
    per-rank times of a 1080p frame's 1/8 shares before cost-ordered waves
    (profiles/r02_shares_path_groups_default.txt): bands 0.62-0.69 ms, blocks 0.66-0.70 -- a share ends
    with its slowest waves, not with its pixel count; with cost-ordered waves every rank's band share
    takes 0.53-0.56 ms (profiles/r02_shares_all_ranks_default.txt)."""
    if kind == "bands":
        return band_layout(width, height, world)
    if kind == "blocks":
        return block_layout(width, height, world)
    raise ValueError(f"unknown screen layout {kind!r}")


def source_index(layout: BandLayout):
    """For every pixel of the full frame (row-major), its row in the gathered (world * max_count)
    buffer.  Returned as a Python list; callers turn it into a device index tensor once."""
    idx = [0] * (layout.width * layout.height)
    for r in range(layout.world):
        base = r * layout.max_count
        for t in layout.tiles[r]:
            for yy in range(t.h):
                dst = (t.y0 + yy) * layout.width + t.x0
                src = base + t.accum_offset + yy * t.accum_pitch
                idx[dst:dst + t.w] = range(src, src + t.w)
    return idx


def gather_frame(local, layout: BandLayout, rank: int, full=None, src_index=None, group=None):
    """Collective: every rank passes its (max_count, 4) float32 slab; rank 0 receives all slabs and
    writes the un-permuted frame into `full` ((H*W, 4) tensor) using `src_index` (LongTensor)."""
    import torch
    import torch.distributed as dist
    if layout.world == 1:
        if full is not None:
            full.copy_(local[: layout.width * layout.height])
        return full
    # rank 0 receives the slabs straight into one (world * max_count, 4) buffer (contiguous row blocks)
    allbuf = torch.empty((layout.world * local.shape[0], 4), dtype=local.dtype, device=local.device) if rank == 0 else None
    dist.gather(local, list(allbuf.chunk(layout.world)) if rank == 0 else None, dst=0, group=group)
    if rank == 0:
        torch.index_select(allbuf, 0, src_index, out=full)
    return full


class PipelinedGather:
    """The frame-end gather overlapped with the next frame's render.

    submit(local) snapshots the rank's slab into one of two staging buffers (a device copy ordered
    after the frame's kernels on the current stream) and starts the gather of that snapshot as an
    asynchronous collective (RCCL runs it on its own stream), then completes the PREVIOUS frame's
    gather: its wait orders the un-permute into `full` on the current stream.  The collective of frame
    f therefore runs while frame f+1 renders, instead of between them (the render of f+1 only needs the
    accumulation buffer, which the snapshot freed).  flush() completes the last frame.  Rank 0's
    `full` holds frame f's image once submit(f+1) or flush() has returned to the stream."""

    def __init__(self, layout: BandLayout, rank: int, full=None, src_index=None, group=None):
        self.layout, self.rank, self.full, self.src_index, self.group = layout, rank, full, src_index, group
        self.staging = None
        self.recv = None
        self.pending = None
        self.count = 0
        # gloo (the CPU tests, bench.py's --dist-backend gloo rehearsal): device slabs are staged through host
        # memory, the collective runs on host tensors
        import torch.distributed as dist
        self.host = layout.world > 1 and dist.is_initialized() and dist.get_backend(group) == "gloo"

    def submit(self, local):
        import torch
        import torch.distributed as dist
        if self.layout.world == 1:
            if self.full is not None:
                self.full.copy_(local[: self.layout.width * self.layout.height])
            return
        if self.staging is None:
            dev = "cpu" if self.host else local.device
            self.staging = [torch.empty(local.shape, dtype=local.dtype, device=dev) for _ in range(2)]
            if self.rank == 0:  # each frame's slabs land in one contiguous buffer: no concatenation copy
                w = self.layout.world
                self.recv = [torch.empty((w * local.shape[0], 4), dtype=local.dtype, device=dev) for _ in range(2)]
        k = self.count % 2
        self.count += 1
        self.staging[k].copy_(local)
        work = dist.gather(self.staging[k], list(self.recv[k].chunk(self.layout.world)) if self.rank == 0 else None,
                           dst=0, group=self.group, async_op=True)
        prev, self.pending = self.pending, (work, k)
        if prev is not None:
            self._finish(prev)

    def flush(self):
        if self.pending is not None:
            self._finish(self.pending)
            self.pending = None

    def _finish(self, pend):
        import torch
        work, k = pend
        work.wait()
        if self.rank == 0:
            if self.recv[k].device != self.full.device:  # host-staged (gloo): un-permute on the host, one copy back
                if getattr(self, "_src_host", None) is None:
                    self._src_host = self.src_index.to(self.recv[k].device)
                self.full.copy_(torch.index_select(self.recv[k], 0, self._src_host))
            else:
                torch.index_select(self.recv[k], 0, self.src_index, out=self.full)


def gathered_tiles(layout: BandLayout):
    """Every rank's tiles with accum_offset moved to the rank's slab in the gathered buffer of
    dxrpt_gather_slabs (rank r's slab at sum(counts[:r]) pixels): the tile list of dxrpt_unpermute."""
    out, base = [], 0
    for r in range(layout.world):
        for t in layout.tiles[r]:
            out.append(A.Tile(t.x0, t.y0, t.w, t.h, base + t.accum_offset, t.accum_pitch, 0))
        base += layout.counts[r]
    return out


class NativeGather:
    """The frame-end gather through the C ABI (libdxrpt.so): an RCCL communicator of the
    job's ranks made by dxrpt_comm_create (rank 0's unique id broadcast over torch.distributed, the only
    thing torch does here), grouped ncclSend / ncclRecv of every rank's slab into one contiguous buffer on
    rank 0 (dxrpt_gather_slabs) and the un-permute kernel into the W x H frame (dxrpt_unpermute) -- the
    sequence a C++ host runs.  Frame f's slab is snapshotted and gathered on the render
    stream and un-permuted there once frame f+1 is submitted (or at flush()).  With overlapped frames (the
    default) the render stream carries only the frames' blends: the frames themselves run on the
    library's slot streams, which the gather does not block, so frame f+1.. render while frame f gathers.
    side_stream=True gathers on a stream of its own instead (for one-frame-at-a-time rendering on the
    render stream; r05: with overlapped frames the extra stream and its cross-stream waits cost the 1/8
    share 0.244 -> 0.27-0.35 ms, profiles/r05_ab_overlap_side.txt, r05_ab_overlap_hwq.txt)."""

    def __init__(self, layout: BandLayout, rank: int, device: int, full=None, group=None, timing: bool = False,
                 side_stream: bool = False, lib=None):
        import ctypes as C
        import torch.distributed as dist
        self.layout, self.rank, self.full = layout, rank, full
        # `lib`: the C ABI (libdxrpt.so); the CPU tests pass a stub communicator with the same entry points
        self.L = lib if lib is not None else A.lib()
        uid = C.create_string_buffer(A.DXRPT_COMM_ID_BYTES)
        # Failures BEFORE ncclCommInitRank are made collective, so every rank raises together (a caller may
        # then fall back to another gather) instead of the others blocking inside the collective init: the
        # ranks first agree that each one's device and arguments are valid, then rank 0 makes the id.  A
        # rank that fails inside ncclCommInitRank itself still leaves the others blocked there (RCCL's
        # blocking init), which no check before it can cover.
        ready = self._device_ready(device) and 0 <= rank < layout.world
        flags = [None] * layout.world
        dist.all_gather_object(flags, bool(ready), group=group)
        if not all(flags):
            raise RuntimeError(f"native gather: ranks {[r for r, v in enumerate(flags) if not v]} cannot use their "
                               "device; not creating the RCCL communicator")
        obj = [None]
        if rank == 0:
            rc = self.L.dxrpt_comm_unique_id(uid)
            obj = [bytes(uid.raw) if rc == A.DXRPT_OK else ("error", self._msg(rc))]
        dist.broadcast_object_list(obj, src=0, group=group)
        if isinstance(obj[0], tuple):
            raise RuntimeError(f"dxrpt_comm_unique_id failed on rank 0: {obj[0][1]}")
        uid = C.create_string_buffer(obj[0], A.DXRPT_COMM_ID_BYTES)
        self.comm = C.c_void_p()
        rc = self.L.dxrpt_comm_create(device, layout.world, rank, uid, C.byref(self.comm))
        # the communicator's own view (what RCCL runs the gather over) is checked in the same collective as
        # the create result, so every rank raises or continues together
        nr, rk = C.c_int(), C.c_int()
        rc_info = self.L.dxrpt_comm_info(self.comm, C.byref(nr), C.byref(rk)) if rc == A.DXRPT_OK else rc
        mine = (rc == A.DXRPT_OK, rc_info == A.DXRPT_OK and nr.value == layout.world and rk.value == rank)
        oks = [None] * layout.world
        dist.all_gather_object(oks, mine, group=group)
        if not all(a and b for a, b in oks):
            if rc == A.DXRPT_OK:
                self.L.dxrpt_comm_destroy(self.comm)
            self.comm = C.c_void_p()
            bad_create = [r for r, v in enumerate(oks) if not v[0]]
            bad_info = [r for r, v in enumerate(oks) if v[0] and not v[1]]
            raise RuntimeError(f"native gather: dxrpt_comm_create failed on ranks {bad_create}, dxrpt_comm_info "
                               f"disagreed on ranks {bad_info}: "
                               f"{self._msg(rc if rc != A.DXRPT_OK else rc_info) if not all(mine) else 'see those ranks'}")
        self.comm_ranks, self.comm_rank = nr.value, rk.value  # what RCCL runs the gather over
        self.counts = (C.c_uint64 * layout.world)(*layout.counts)
        self.tiles = gathered_tiles(layout)
        self.tarr = (A.Tile * len(self.tiles))(*self.tiles)
        self.total = sum(layout.counts)
        self.side = self._new_stream() if side_stream else None
        self.staging = None
        self.recv = None
        self.pending = None
        self.count = 0
        # timing=True: events around each frame's dxrpt_gather_slabs (side stream) and dxrpt_unpermute
        # (render stream), read by times() once the frames are done
        self.timing = timing
        self.gather_ev, self.unpermute_ev = [], []

    # device seams (the CPU tests' stub subclass replaces these four; the product path is HIP through torch)
    def _device_ready(self, device):
        import torch
        return torch.cuda.is_available() and 0 <= device < torch.cuda.device_count()

    def _new_stream(self):
        import torch
        return torch.cuda.Stream()

    def _current_stream(self):
        import torch
        return torch.cuda.current_stream()

    def _event(self, timing=False):
        import torch
        return torch.cuda.Event(enable_timing=timing)

    def _synchronize(self):
        import torch
        torch.cuda.synchronize()

    def _msg(self, rc):
        msg = self.L.dxrpt_multi_last_error()
        return f"({rc}) {msg.decode() if msg else ''}"

    def _check(self, rc, what):
        if rc != A.DXRPT_OK:
            raise RuntimeError(f"{what} failed {self._msg(rc)}")

    def submit(self, local):
        import ctypes as C
        import torch
        cur = self._current_stream()
        n = self.layout.counts[self.rank]
        if self.staging is None:
            self.staging = [torch.empty((n, 4), dtype=torch.float32, device=local.device) for _ in range(2)]
            if self.rank == 0:
                self.recv = [torch.empty((self.total, 4), dtype=torch.float32, device=local.device) for _ in range(2)]
        k = self.count % 2
        self.count += 1
        self.staging[k].copy_(local[:n])
        gs = self.side if self.side is not None else cur
        if self.side is not None:
            self.side.wait_stream(cur)
        if self.timing:
            g0, g1 = self._event(True), self._event(True)
            g0.record(gs)
        self._check(self.L.dxrpt_gather_slabs(self.comm, C.c_void_p(self.staging[k].data_ptr()), self.counts,
                                              C.c_void_p(self.recv[k].data_ptr()) if self.rank == 0 else None,
                                              C.c_void_p(gs.cuda_stream)), "dxrpt_gather_slabs")
        ev = self._event()
        ev.record(gs)
        if self.timing:
            g1.record(gs)
            self.gather_ev.append((g0, g1))
        prev, self.pending = self.pending, (ev, k)
        if prev is not None:
            self._finish(prev)

    def flush(self):
        if self.pending is not None:
            self._finish(self.pending)
            self.pending = None

    def _finish(self, pend):
        import ctypes as C
        ev, k = pend
        cur = self._current_stream()
        cur.wait_event(ev)
        if self.rank == 0:
            if self.timing:
                u0, u1 = self._event(True), self._event(True)
                u0.record(cur)
            self._check(self.L.dxrpt_unpermute(C.c_void_p(self.recv[k].data_ptr()), self.tarr, len(self.tiles),
                                               C.c_void_p(self.full.data_ptr()), self.layout.width, self.layout.height,
                                               C.c_void_p(cur.cuda_stream)), "dxrpt_unpermute")
            if self.timing:
                u1.record(cur)
                self.unpermute_ev.append((u0, u1))

    def reset_times(self):
        self.gather_ev, self.unpermute_ev = [], []

    def times(self):
        """(mean ms of dxrpt_gather_slabs on the side stream, mean ms of dxrpt_unpermute on rank 0's render
        stream, frames) over the frames submitted since reset_times(); call after the frames are done."""
        import statistics
        g = [a.elapsed_time(b) for a, b in self.gather_ev]
        u = [a.elapsed_time(b) for a, b in self.unpermute_ev]
        return (statistics.mean(g) if g else None, statistics.mean(u) if u else None, len(g))

    def close(self):
        if self.comm:
            self.flush()
            self._synchronize()
            self._check(self.L.dxrpt_comm_destroy(self.comm), "dxrpt_comm_destroy")
            self.comm = None
            # the un-permute scratch of this thread, released while the HIP runtime is up
            self._check(self.L.dxrpt_multi_release(), "dxrpt_multi_release")
