"""Test helpers for the FBX ingest (dxrpt_host_scene_load): a minimal binary FBX 7.4 writer for
synthetic scenes, an independent reader of the raw geometry arrays, and a DDS writer (BC1 / BC4 /
uncompressed) for material textures.  Test infrastructure only."""
from __future__ import annotations

import struct
import zlib

import numpy as np


# ---- FBX writer ---------------------------------------------------------------------------------------
def _prop(v):
    if isinstance(v, tuple) and v[0] == "arr":  # ("arr", type, values)
        t, vals = v[1], v[2]
        fmt = {"d": "d", "f": "f", "i": "i", "l": "q", "b": "B"}[t]
        raw = struct.pack(f"<{len(vals)}{fmt}", *vals)
        comp = zlib.compress(raw)
        return t.encode() + struct.pack("<III", len(vals), 1, len(comp)) + comp
    if isinstance(v, str):
        b = v.encode("latin1")
        return b"S" + struct.pack("<I", len(b)) + b
    if isinstance(v, bytes):
        return b"R" + struct.pack("<I", len(v)) + v
    if isinstance(v, float):
        return b"D" + struct.pack("<d", v)
    if isinstance(v, int):
        return (b"L" + struct.pack("<q", v)) if abs(v) >= 2 ** 31 else (b"I" + struct.pack("<i", v))
    raise TypeError(v)


def _node(name, props=(), children=(), base=0):
    """Node record at absolute offset `base` (FBX 7.4: 32-bit end offsets)."""
    pb = b"".join(_prop(p) for p in props)
    nb = name.encode()
    head_len = 12 + 1 + len(nb) + len(pb)
    body = b""
    off = base + head_len
    for c in children:
        cb = _node(c[0], c[1], c[2], off)
        body += cb
        off += len(cb)
    if children:
        body += b"\0" * 13
    end = base + head_len + len(body)
    return struct.pack("<III", end, len(props), len(pb)) + bytes([len(nb)]) + nb + pb + body


def write_fbx(path, nodes):
    """nodes: list of (name, props, children) top-level records."""
    out = bytearray(b"Kaydara FBX Binary  \0\x1a\0" + struct.pack("<I", 7400))
    for n in nodes:
        out += _node(n[0], n[1], n[2], len(out))
    out += b"\0" * 13
    with open(path, "wb") as f:
        f.write(bytes(out))


def arr(t, vals):
    return ("arr", t, list(vals))


def mesh_fbx(path, positions, polygons, normals_pv, uvs, uv_index, material_tex=None, tangents_pv=None,
             binormals_pv=None, material_slots=None):
    """A one-model FBX: `polygons` lists of vertex indices; normals_pv per polygon vertex (Direct);
    uvs + uv_index (IndexToDirect); optional material with a DiffuseColor texture file name, or
    `material_slots` = {FBX material property (DiffuseColor, TransparentColor, ...): file name}."""
    pvi = []
    for poly in polygons:
        pvi += list(poly[:-1]) + [~poly[-1]]
    geo_children = [
        ("Vertices", [arr("d", np.asarray(positions, np.float64).ravel())], []),
        ("PolygonVertexIndex", [arr("i", pvi)], []),
        ("LayerElementNormal", [0], [("MappingInformationType", ["ByPolygonVertex"], []),
                                     ("ReferenceInformationType", ["Direct"], []),
                                     ("Normals", [arr("d", np.asarray(normals_pv, np.float64).ravel())], [])]),
        ("LayerElementUV", [0], [("MappingInformationType", ["ByPolygonVertex"], []),
                                 ("ReferenceInformationType", ["IndexToDirect"], []),
                                 ("UV", [arr("d", np.asarray(uvs, np.float64).ravel())], []),
                                 ("UVIndex", [arr("i", uv_index)], [])]),
    ]
    if tangents_pv is not None:
        geo_children.append(("LayerElementTangent", [0], [("MappingInformationType", ["ByPolygonVertex"], []),
                                                          ("ReferenceInformationType", ["Direct"], []),
                                                          ("Tangents", [arr("d", np.asarray(tangents_pv).ravel())], [])]))
        geo_children.append(("LayerElementBinormal", [0], [("MappingInformationType", ["ByPolygonVertex"], []),
                                                           ("ReferenceInformationType", ["Direct"], []),
                                                           ("Binormals", [arr("d", np.asarray(binormals_pv).ravel())], [])]))
    objects = [("Geometry", [1001, "Mesh\0\x01Geometry", "Mesh"], geo_children),
               ("Model", [2001, "Mesh\0\x01Model", "Mesh"], [])]
    conns = [("C", ["OO", 2001, 0], []), ("C", ["OO", 1001, 2001], [])]
    slots = dict(material_slots or {})
    if material_tex is not None:
        slots["DiffuseColor"] = material_tex
    if slots:
        objects.append(("Material", [3001, "mat\0\x01Material", ""], []))
        conns.append(("C", ["OO", 3001, 2001], []))
        for k, (prop, fname) in enumerate(slots.items()):
            objects.append(("Texture", [4001 + k, "tex\0\x01Texture", ""], [("FileName", ["C:\\some\\dir\\" + fname], []),
                                                                          ("RelativeFilename", [fname], [])]))
            conns.append(("C", ["OP", 4001 + k, 3001, prop], []))
    write_fbx(path, [("FBXHeaderExtension", [], [("FBXVersion", [7400], [])]),
                     ("Objects", [], objects), ("Connections", [], conns)])


# ---- independent raw reader (geometry arrays only) ----------------------------------------------------
def read_fbx_arrays(path):
    """{node name: numpy array} of every array property in the file (first occurrence per name)."""
    d = open(path, "rb").read()
    ver = struct.unpack_from("<I", d, 23)[0]
    out = {}

    def rec(off):
        if ver >= 7500:
            end, nprops, _ = struct.unpack_from("<QQQ", d, off)
            off += 24
        else:
            end, nprops, _ = struct.unpack_from("<III", d, off)
            off += 12
        nl = d[off]
        off += 1
        name = d[off:off + nl].decode("latin1")
        off += nl
        if end == 0:
            return None, off
        for _ in range(nprops):
            t = chr(d[off])
            off += 1
            if t in "YCIFDL":
                off += {"Y": 2, "C": 1, "I": 4, "F": 4, "D": 8, "L": 8}[t]
            elif t in "SR":
                off += 4 + struct.unpack_from("<I", d, off)[0]
            else:
                n, enc, clen = struct.unpack_from("<III", d, off)
                off += 12
                raw = d[off:off + clen]
                off += clen
                if enc:
                    raw = zlib.decompress(raw)
                dt = {"f": np.float32, "d": np.float64, "i": np.int32, "l": np.int64, "b": np.uint8}[t]
                out.setdefault(name, np.frombuffer(raw, dtype=dt, count=n))
        while off < end:
            c, off = rec(off)
            if c is None:
                break
        return name, end

    off = 27
    while off < len(d):
        n, off = rec(off)
        if n is None:
            break
    return out


# ---- DDS writer ---------------------------------------------------------------------------------------
def write_dds(path, width, height, fourcc=None, data=b"", bgrx=False):
    """Legacy-header DDS: fourcc b'DXT1' / b'BC4U' blocks in `data`, or 32-bit BGRX/BGRA texels."""
    flags = 0x1 | 0x2 | 0x4 | 0x1000
    if fourcc:
        pf = struct.pack("<II4sIIIII", 32, 0x4, fourcc, 0, 0, 0, 0, 0)
    else:
        pf = struct.pack("<II4sIIIII", 32, 0x40 | (0 if bgrx else 0x1), b"\0\0\0\0", 32, 0xFF0000, 0xFF00, 0xFF,
                         0 if bgrx else 0xFF000000)
    hdr = struct.pack("<IIIIIII", 124, flags, height, width, 0, 0, 1) + b"\0" * 44 + pf + struct.pack("<IIIII", 0x1000, 0, 0, 0, 0)
    with open(path, "wb") as f:
        f.write(b"DDS " + hdr + data)


def bc4_decode_block(b):
    """Python restatement of the BC4 block rule (D3D functional spec) for the tests."""
    r0, r1 = b[0], b[1]
    if r0 > r1:
        pal = [r0, r1] + [((7 - i) * r0 + i * r1 + 3) // 7 for i in range(1, 7)]
    else:
        pal = [r0, r1] + [((5 - i) * r0 + i * r1 + 2) // 5 for i in range(1, 5)] + [0, 255]
    bits = int.from_bytes(bytes(b[2:8]), "little")
    return [pal[(bits >> (3 * i)) & 7] for i in range(16)]


def box_room_fbx(directory, images="dds"):
    """A synthetic scene for the GPU ingest test: floor, back and side walls, a box and an alpha-tested
    card (TransparentColor -> opacity), albedo and opacity from BC1 / BC4 DDS files (images="dds") or
    from a PNG albedo and a greyscale JPEG opacity (images="png", the WIC formats; needs PIL for the
    JPEG).  Geometry is given in the renderer's (left-handed) frame and written with z mirrored, as an
    FBX exporter would store it."""
    import os
    quads = []  # (4 corners, normal)

    def quad(a, b, c, d, n):
        quads.append(([a, b, c, d], n))
    quad((-5, 0, -5), (5, 0, -5), (5, 0, 5), (-5, 0, 5), (0, 1, 0))          # floor
    quad((-5, 0, 5), (5, 0, 5), (5, 6, 5), (-5, 6, 5), (0, 0, -1))           # back wall
    quad((-5, 0, -5), (-5, 0, 5), (-5, 6, 5), (-5, 6, -5), (1, 0, 0))        # left wall
    quad((5, 0, 5), (5, 0, -5), (5, 6, -5), (5, 6, 5), (-1, 0, 0))           # right wall
    for (lo, hi) in [((-1.0, 0.0, -1.0), (1.0, 2.0, 1.0))]:
        x0, y0, z0 = lo
        x1, y1, z1 = hi
        quad((x0, y1, z0), (x1, y1, z0), (x1, y1, z1), (x0, y1, z1), (0, 1, 0))
        quad((x0, y0, z0), (x0, y1, z0), (x1, y1, z0), (x1, y0, z0), (0, 0, -1))
        quad((x0, y0, z1), (x1, y0, z1), (x1, y1, z1), (x0, y1, z1), (0, 0, 1))
        quad((x0, y0, z0), (x0, y0, z1), (x0, y1, z1), (x0, y1, z0), (-1, 0, 0))
        quad((x1, y0, z0), (x1, y1, z0), (x1, y1, z1), (x1, y0, z1), (1, 0, 0))
    pos, polys, normals, uv_index = [], [], [], []
    uvs = [(0.0, 0.0), (1.0, 0.0), (1.0, 1.0), (0.0, 1.0)]
    for corners, n in quads:
        base = len(pos)
        pos += [(x, y, -z) for (x, y, z) in corners]
        polys.append([base, base + 1, base + 2, base + 3])
        normals += [(n[0], n[1], -n[2])] * 4
        uv_index += [0, 1, 2, 3]
    # an 8x8 BC1 albedo (4 blocks of different colours) and an 8x8 BC4 opacity (left half opaque)
    blocks = []
    for c0 in (0xF800, 0x07E0, 0x001F, 0xFFE0):
        blocks.append(struct.pack("<HHI", c0, 0x8410, 0x5A5A5A5A))
    write_dds(os.path.join(directory, "albedo.dds"), 8, 8, fourcc=b"DXT1", data=b"".join(blocks))
    op = []
    for bx in range(4):
        v = 255 if bx % 2 == 0 else 0
        op.append(bytes([v, v, 0, 0, 0, 0, 0, 0]))
    write_dds(os.path.join(directory, "opacity.dds"), 8, 8, fourcc=b"BC4U", data=b"".join(op))
    slots = {"DiffuseColor": "albedo.dds", "TransparentColor": "opacity.dds"}
    if images == "png":
        import numpy as np
        from PIL import Image
        from tests.image_util import write_png
        yy, xx = np.mgrid[0:16, 0:16]
        rgb = np.stack([(xx * 16) % 256, (yy * 16) % 256, ((xx ^ yy) * 32) % 256], -1)
        write_png(os.path.join(directory, "albedo.png"), rgb, 2, 8, interlace=True)
        mask = np.where((xx // 4 + yy // 4) % 2 == 0, 255, 0).astype(np.uint8)
        Image.fromarray(mask, "L").save(os.path.join(directory, "opacity.jpg"), quality=90)
        slots = {"DiffuseColor": "albedo.png", "TransparentColor": "opacity.jpg"}
    path = os.path.join(directory, "room.fbx")
    mesh_fbx(path, pos, polys, normals, uvs, uv_index, material_slots=slots)
    return path
