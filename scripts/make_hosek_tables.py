#!/usr/bin/env python3
"""Generates dxrpathtracer_amd/data/hosek_tables.bin: the constant tables the Hosek-Wilkie sky needs.

Run once, in a container that has the reference checkout:

    python scripts/make_hosek_tables.py [--reference /root/reference]

The tables are published data of two models, not code:
  * Hosek & Wilkie 2012/2013 sky model fits (SampleFramework12/v1.02/HosekSky/ArHosekSkyModelData_RGB.h,
    ArHosekSkyModelData_Spectral.h): datasetRGB{1,2,3} (1080 doubles each), datasetRGBRad{1,2,3} (120),
    dataset<wl> / datasetRad<wl> / solarDataset<wl> (1800) / limbDarkeningDataset<wl> (6) for the 11
    wavelengths 320..720 nm;
  * CIE 1931 colour matching functions and Smits' RGB->spectrum reflectance bases as pbrt-v3 tabulates
    them (Graphics/Spectrum.cpp:205-1095): CIE_lambda/X/Y/Z (471 floats), RGB2SpectLambda and the seven
    RGBRefl2Spect* bases (32 floats).

File format (little endian): 8-byte magic "DXRPTHK1", u32 record count, then per record: u32 name length,
name bytes, u32 element type (0 = float64, 1 = float32), u32 element count, the elements.  Read by
dxrpt_host_hosek_load_tables (csrc/host/hosek.cpp).  The float32 tables are rounded from the decimal
literal through double, as the source-parsing loader (dxrpt_host_hosek_load) does.
"""
from __future__ import annotations

import argparse
import os
import re
import struct

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "dxrpathtracer_amd", "data", "hosek_tables.bin")
WAVELENGTHS = [320 + 40 * i for i in range(11)]
REFL = ["White", "Cyan", "Magenta", "Yellow", "Red", "Green", "Blue"]
NUM = re.compile(r"[-+]?(?:\d+\.?\d*|\.\d+)(?:[eE][-+]?\d+)?")


def strip_comments(src: str) -> str:
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    return re.sub(r"//[^\n]*", " ", src)


def named_array(src: str, name: str) -> list[float]:
    """The initializer of `<type> name[...] = { ... };` as floats (first definition)."""
    m = re.search(r"(?<![A-Za-z0-9_])" + re.escape(name) + r"\s*\[[^\]]*\]\s*=\s*\{([^}]*)\}", src)
    if not m:
        raise KeyError(name)
    return [float(t) for t in NUM.findall(m.group(1))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default=os.environ.get("DXRPT_REFERENCE_ROOT", "/root/reference"))
    ap.add_argument("--out", default=OUT)
    args = ap.parse_args()
    sf = os.path.join(args.reference, "SampleFramework12", "v1.02")
    rgb = strip_comments(open(os.path.join(sf, "HosekSky", "ArHosekSkyModelData_RGB.h")).read())
    spec = strip_comments(open(os.path.join(sf, "HosekSky", "ArHosekSkyModelData_Spectral.h")).read())
    sp = strip_comments(open(os.path.join(sf, "Graphics", "Spectrum.cpp")).read())

    records = []  # (name, type, values)

    def take(src, name, n, kind):
        v = named_array(src, name)
        if len(v) != n:
            raise ValueError(f"{name}: {len(v)} elements, expected {n}")
        records.append((name, kind, v))

    for c in (1, 2, 3):
        take(rgb, f"datasetRGB{c}", 1080, 0)
        take(rgb, f"datasetRGBRad{c}", 120, 0)
    for wl in WAVELENGTHS:
        take(spec, f"dataset{wl}", 1080, 0)
        take(spec, f"datasetRad{wl}", 120, 0)
        take(spec, f"solarDataset{wl}", 1800, 0)
        take(spec, f"limbDarkeningDataset{wl}", 6, 0)
    for name in ("CIE_lambda", "CIE_X", "CIE_Y", "CIE_Z"):
        take(sp, name, 471, 1)
    take(sp, "RGB2SpectLambda", 32, 1)
    for r in REFL:
        take(sp, f"RGBRefl2Spect{r}", 32, 1)

    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "wb") as f:
        f.write(b"DXRPTHK1")
        f.write(struct.pack("<I", len(records)))
        for name, kind, v in records:
            nb = name.encode()
            f.write(struct.pack("<I", len(nb)) + nb + struct.pack("<II", kind, len(v)))
            f.write(np.asarray(v, dtype="<f8" if kind == 0 else "<f4").tobytes())
    print(f"wrote {args.out}: {len(records)} tables, {os.path.getsize(args.out)} bytes")


if __name__ == "__main__":
    main()
