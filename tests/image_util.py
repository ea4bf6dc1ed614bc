"""Test-side PNG writer (every colour type / bit depth, optional Adam7) and a ctypes helper that decodes a
file through dxrpt_host_texture_load.  Test infrastructure only."""
from __future__ import annotations

import ctypes as C
import struct
import zlib

import numpy as np

import dxrpathtracer_amd._abi as A

ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]


def _chunk(tag: bytes, body: bytes) -> bytes:
    return struct.pack(">I", len(body)) + tag + body + struct.pack(">I", zlib.crc32(tag + body) & 0xFFFFFFFF)


def _pack_row(samples: np.ndarray, depth: int) -> bytes:
    """samples: 1-D array of channel samples of one row (interleaved)."""
    if depth == 8:
        return samples.astype(np.uint8).tobytes()
    if depth == 16:
        return samples.astype(">u2").tobytes()
    per = 8 // depth
    out = bytearray((len(samples) + per - 1) // per)
    for i, v in enumerate(samples):
        out[i // per] |= int(v) << (8 - depth - (i % per) * depth)
    return bytes(out)


def _filter(raw_rows: list[bytes], bpp: int, rng) -> bytes:
    """Each row gets a random filter type (0..4), so the decoder's five unfilters are all exercised."""
    out = bytearray()
    prev = bytes(len(raw_rows[0])) if raw_rows else b""
    for row in raw_rows:
        ft = int(rng.integers(0, 5))
        enc = bytearray(len(row))
        for i, x in enumerate(row):
            a = row[i - bpp] if i >= bpp else 0
            b = prev[i]
            c = prev[i - bpp] if i >= bpp else 0
            if ft == 0:
                pred = 0
            elif ft == 1:
                pred = a
            elif ft == 2:
                pred = b
            elif ft == 3:
                pred = (a + b) >> 1
            else:
                p = a + b - c
                pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                pred = a if pa <= pb and pa <= pc else (b if pb <= pc else c)
            enc[i] = (x - pred) & 0xFF
        out += bytes([ft]) + enc
        prev = row
    return bytes(out)


def write_png(path, samples: np.ndarray, ctype: int, depth: int, palette=None, trns: bytes | None = None,
              interlace: bool = False, seed: int = 0):
    """samples: (H, W, channels) integer array at the file's depth (palette indices for ctype 3)."""
    rng = np.random.default_rng(seed)
    h, w, nc = samples.shape
    bpp = max(1, nc * depth // 8)
    passes = ADAM7 if interlace else [(0, 0, 1, 1)]
    data = b""
    for x0, y0, dx, dy in passes:
        sub = samples[y0::dy, x0::dx]
        if sub.shape[0] == 0 or sub.shape[1] == 0:
            continue
        rows = [_pack_row(sub[y].reshape(-1), depth) for y in range(sub.shape[0])]
        data += _filter(rows, bpp, rng)
    png = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 1 if interlace else 0))
    if palette is not None:
        png += _chunk(b"PLTE", bytes(np.asarray(palette, np.uint8).reshape(-1)))
    if trns is not None:
        png += _chunk(b"tRNS", trns)
    # split IDAT in two chunks (decoders must concatenate them)
    z = zlib.compress(data, 9)
    png += _chunk(b"IDAT", z[: len(z) // 2]) + _chunk(b"IDAT", z[len(z) // 2:]) + _chunk(b"IEND", b"")
    open(path, "wb").write(png)


def decode(path, srgb: bool = False):
    """(RGBA8 or R8 array, fmt) through dxrpt_host_texture_load; raises RuntimeError with the library's error."""
    H = A.host()
    t = A.HostTexture()
    rc = H.dxrpt_host_texture_load(str(path).encode(), 1 if srgb else 0, C.byref(t))
    if rc != 0:
        raise RuntimeError(H.dxrpt_host_last_error().decode())
    try:
        ch = 1 if t.fmt == A.TEX_R8_UNORM else 4
        n = t.width * t.height * ch
        arr = np.ctypeslib.as_array((C.c_uint8 * n).from_address(t.texels)).copy()
    finally:
        H.dxrpt_host_texture_free(C.byref(t))
    return arr.reshape(t.height, t.width, ch) if ch == 4 else arr.reshape(t.height, t.width), int(t.fmt)
