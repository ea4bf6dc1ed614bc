#!/usr/bin/env python3
"""Generates tests/golden/cmj_reference.json from the reference's own CMJ code.

The reference's C++ correlated multi-jittered sampler (SampleFramework12/v1.02/Graphics/Sampling.cpp:
383-432: CMJPermute, CMJRandFloat, SampleCMJ2D -- the CPU twin of Shaders/Sampling.hlsl:282-331 that
RayTrace.hlsl's SamplePoint calls) is read out of the checkout at generation time, compiled verbatim
with g++ into oracle/_ref/ (git-ignored) and run on a grid of cases:
  * every sample index 0 .. N-1 of square and non-square grids (numSamplesX x numSamplesY),
  * patterns = setIdx * TotalNumPixels + pixelIdx (u32 wrap, RayTrace.hlsl:85-90) for the BASELINE
    frame sizes, several pixels and path depths, plus arbitrary 32-bit patterns.
The only text added around the extracted functions is the two type names they use (`uint32`, `Float2`,
defined in the reference's SF12 headers, which pull in Windows headers and are not compiled here).
Values are stored as float32 bit patterns, so the test is bit-exact.

    python tests/golden/make_cmj_golden.py          (needs /root/reference and g++)
"""
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = "/root/reference/SampleFramework12/v1.02/Graphics/Sampling.cpp"
OUT_DIR = os.path.join(REPO, "oracle", "_ref")
GOLDEN = os.path.join(REPO, "tests", "golden", "cmj_reference.json")

PRELUDE = """#include <cstdint>
#include <cstdio>
typedef uint32_t uint32;
struct Float2 { float x, y; Float2(float a, float b) : x(a), y(b) {} };
"""
DRIVER = r"""
#include <cstring>
int main() {
    unsigned s, nx, ny, pat;
    while (std::scanf("%u %u %u %u", &s, &nx, &ny, &pat) == 4) {
        Float2 v = SampleCMJ2D(s, nx, ny, pat);
        uint32_t bx, by;
        std::memcpy(&bx, &v.x, 4);
        std::memcpy(&by, &v.y, 4);
        std::printf("%u %u\n", bx, by);
    }
    return 0;
}
"""


def extract(text: str) -> str:
    """The reference's CMJPermute .. end of SampleCMJ2D, verbatim."""
    a = text.index("static uint32 CMJPermute(")
    m = re.search(r"Float2 SampleCMJ2D\(uint32 sampleIdx[^)]*\)\s*\{", text[a:])
    b = a + m.end()
    depth = 1
    while depth:
        depth += {"{": 1, "}": -1}.get(text[b], 0)
        b += 1
    return text[a:b]


def cases():
    out = []
    grids = [(4, 4), (1, 1), (2, 2), (2, 3), (3, 2), (5, 7), (7, 5), (8, 8), (16, 1), (1, 16), (3, 11)]
    sizes = [(1920, 1080), (1280, 720), (3840, 2160), (256, 256)]
    pixels = [0, 1, 1000, 65535, 1919, 1036799]
    for nx, ny in grids:
        n = nx * ny
        pats = []
        for (w, h) in sizes:
            tp = w * h
            for px in pixels:
                if px < tp:
                    for set_idx in (0, 1, 2, 7):
                        pats.append((set_idx * tp + px) & 0xFFFFFFFF)
        pats += [0xFFFFFFFF, 0x80000000, 0xDEADBEEF, 0x12345678, 7 * 8294400 + 8294399]
        pats = sorted(set(pats))
        step = max(1, len(pats) // 24)
        for pat in pats[::step]:
            for s in range(n):
                out.append((s, nx, ny, pat))
    return out


def main():
    if not os.path.isfile(SRC):
        sys.exit(f"{SRC} not found: the generator needs the reference checkout")
    os.makedirs(OUT_DIR, exist_ok=True)
    cpp = os.path.join(OUT_DIR, "cmj_gen.cpp")
    exe = os.path.join(OUT_DIR, "cmj_gen")
    with open(cpp, "w") as f:
        f.write(PRELUDE + "\n" + extract(open(SRC, encoding="utf-8", errors="replace").read()) + "\n" + DRIVER)
    subprocess.run(["g++", "-O0", "-ffp-contract=off", "-fno-fast-math", "-o", exe, cpp], check=True)
    cs = cases()
    res = subprocess.run([exe], input="\n".join(" ".join(map(str, c)) for c in cs), capture_output=True, text=True,
                         check=True).stdout.split("\n")
    rows = []
    for c, r in zip(cs, res):
        bx, by = (int(v) for v in r.split())
        rows.append([*c, bx, by])
    assert len(rows) == len(cs)
    json.dump({
        "source": "SampleFramework12/v1.02/Graphics/Sampling.cpp:383-432 (CMJPermute, CMJRandFloat, SampleCMJ2D), "
                  "extracted verbatim from the checkout and compiled with g++ -O0 -ffp-contract=off by "
                  "tests/golden/make_cmj_golden.py",
        "columns": ["sample_idx", "num_samples_x", "num_samples_y", "pattern", "x_f32_bits", "y_f32_bits"],
        "cases": rows,
        # the four probes recorded by the survey, kept for reference
        "total_num_pixels": 2073600,
        "pixel_idx": 1000,
        "sqrt_num_samples": 4,
        "probes": [
            {"sample_idx": 0, "set_idx": 0, "value": [0.0882263333, 0.919450641]},
            {"sample_idx": 0, "set_idx": 1, "value": [0.182110727, 0.600448847]},
            {"sample_idx": 1, "set_idx": 0, "value": [0.203955621, 0.65700686]},
            {"sample_idx": 2, "set_idx": 1, "value": [0.656626701, 0.510319352]},
        ],
    }, open(GOLDEN, "w"), separators=(",", ":"))
    print(f"{len(rows)} cases -> {GOLDEN}")


if __name__ == "__main__":
    main()
