#!/usr/bin/env python3
"""Packages the SunTemple foliage opacity maps the SunTemple proxy (BASELINE config C4) alpha-tests with.

SURVEY.md 8(d): the proxy's foliage cards use the reference's real BC4 opacity maps,
Content/Models/SunTemple/Textures/T_M_Tree_Branches_0_A.dds (1024^2) and T_Soul_Tree011M_Inst_0_A.dds
(2048^2).  Run once where the reference checkout exists:

    python scripts/make_suntemple_opacity.py [--reference /root/reference]

Each file's mip 0 is decoded by this repository's BC4 decoder (dxrpt_host_texture_load, host/dds.cpp)
and stored as dxrpathtracer_amd/data/suntemple/<name>.r8z: "DXR8", u32 width, u32 height (little
endian), then the zlib-compressed width*height R8 texels (read by host/image.cpp load_r8z).  The files
are texture data (content), not code.
"""
import argparse
import os
import struct
import sys
import zlib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
NAMES = ("T_M_Tree_Branches_0_A", "T_Soul_Tree011M_Inst_0_A")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default=os.environ.get("DXRPT_REFERENCE_ROOT", "/root/reference"))
    args = ap.parse_args()
    from tests import image_util as I
    out_dir = os.path.join(REPO, "dxrpathtracer_amd", "data", "suntemple")
    os.makedirs(out_dir, exist_ok=True)
    for n in NAMES:
        src = os.path.join(args.reference, "Content", "Models", "SunTemple", "Textures", n + ".dds")
        img, fmt = I.decode(src)
        assert img.ndim == 2, f"{src}: expected a single-channel (BC4) texture"
        h, w = img.shape
        blob = b"DXR8" + struct.pack("<II", w, h) + zlib.compress(img.tobytes(), 9)
        dst = os.path.join(out_dir, n + ".r8z")
        open(dst, "wb").write(blob)
        print(f"{dst}: {w}x{h}, {len(blob)} bytes, {100.0 * (img >= 90).mean():.1f}% texels >= 0.35")


if __name__ == "__main__":
    main()
