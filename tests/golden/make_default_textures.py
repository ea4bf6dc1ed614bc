"""Regenerates tests/golden/default_textures.json from the reference's 1x1 DDS files (run in the
build container, where /root/reference exists).  Output is RGBA bytes per texture."""
import json
import os
import struct
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/Content/Textures"


def decode(path):
    b = open(path, "rb").read()
    assert b[:4] == b"DDS "
    hdr = struct.unpack("<31I", b[4:128])
    h, w = hdr[2], hdr[3]
    pf_flags, bits, rmask, gmask, bmask = hdr[19], hdr[21], hdr[22], hdr[23], hdr[24]
    assert (w, h, bits) == (1, 1, 32) and (rmask, gmask, bmask) == (0xFF0000, 0xFF00, 0xFF), (path, hdr)
    px = struct.unpack("<I", b[128:132])[0]
    return [(px >> 16) & 0xFF, (px >> 8) & 0xFF, px & 0xFF, 255]  # X8 reads as alpha 1


if __name__ == "__main__":
    out = {n: decode(os.path.join(REF, n + ".dds"))
           for n in ("DefaultBaseColor", "DefaultNormalMap", "DefaultRoughness", "DefaultBlack")}
    print(json.dumps(out, indent=2))
