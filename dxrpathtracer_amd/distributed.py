"""Screen-space sharding across GPUs of one node + the frame-end gather.

The reference is single-GPU; every pixel's path is independent and the CMJ pattern uses only the
GLOBAL pixel index (RayTrace.hlsl:85-96), so any partition of the image renders bit-identical pixels.
Rank r path-traces bands b = r, r+N, r+2N, ... of `band` full rows into a compact local buffer
(dxrpt_tile accum_offset/pitch), and rank 0 gathers the slabs (torch.distributed: RCCL over xGMI on
the GPU node, gloo in the CPU tests) and un-permutes them into the full RGBA32F frame.
"""
from __future__ import annotations

from dataclasses import dataclass

from . import _abi as A

BAND_ROWS = 16


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


def band_layout(width: int, height: int, world: int, band: int = BAND_ROWS) -> BandLayout:
    tiles = [[] for _ in range(world)]
    counts = [0] * world
    for b, y0 in enumerate(range(0, height, band)):
        r = b % world
        h = min(band, height - y0)
        tiles[r].append(A.Tile(0, y0, width, h, counts[r], width, 0))
        counts[r] += width * h
    return BandLayout(width, height, world, band, tiles, counts, max(counts))


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
    gather_list = [torch.empty_like(local) for _ in range(layout.world)] if rank == 0 else None
    dist.gather(local, gather_list, dst=0, group=group)
    if rank == 0:
        allbuf = torch.cat(gather_list, dim=0)
        torch.index_select(allbuf, 0, src_index, out=full)
    return full
