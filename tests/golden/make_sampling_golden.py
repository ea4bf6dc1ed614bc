#!/usr/bin/env python3
"""Generates tests/golden/sampling_reference.npz from the reference's own sampling and BRDF C++ code.

The reference's C++ twins of the shader functions the path tracer uses -- read out of the checkout at
generation time, compiled verbatim with g++ into oracle/_ref/ (git-ignored) and run on dense input grids:
  * SampleFramework12/v1.02/Graphics/Sampling.cpp:167-210  SquareToConcentricDiskMapping
    (statement-identical to Shaders/Sampling.hlsl:72-114, the kernels' sample_cosine_hemisphere first half)
  * Sampling.cpp:264-279  SampleDirectionCosineHemisphere  (Sampling.hlsl:181-196; RayTrace.hlsl:333's
    diffuse lobe, Baking.hlsl's bake ray)
  * Graphics/BRDF.h:39-42  GGX_V1  (BRDF.hlsl:89-92, inside GGXVisibility / CalcLighting)
  * the constant `Pi` of SF12_Math.h:551, read from the same checkout.
The only text added around the extracted functions is a types-only prelude: the SF12 vector types the
functions use (Float2, Float3 with their plain constructors -- SF12_Math.h pulls in DirectXMath and Windows
headers, so it is not compiled here) and the standard headers (<cmath>, <algorithm>).
Two builds of the same extracted text:
  build "libm"  -- std::cos / std::sin are glibc's, as written;
  build "det"   -- the same text with the prelude routing std::cos / std::sin to the deterministic sin/cos the
                   oracle and the kernels define (pt_math.h pt_sincos, oracle.cpp sincos_det; a diagnostic build:
                   it shows that every other operation of the reference's arithmetic is reproduced bit for bit).
Values are stored as float32 bit patterns.

    python tests/golden/make_sampling_golden.py          (needs /root/reference and g++)
"""
import os
import re
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SF12 = "/root/reference/SampleFramework12/v1.02"
OUT_DIR = os.path.join(REPO, "oracle", "_ref", "sampling")
GOLDEN = os.path.join(REPO, "tests", "golden", "sampling_reference.npz")

PRELUDE = """#include <cmath>
#include <cstdint>
#include <cstdio>
#include <algorithm>
#include <math.h>
struct Float2 { float x, y; Float2() : x(0), y(0) {} };
struct Float3 { float x, y, z; Float3() : x(0), y(0), z(0) {} Float3(float a, float b, float c) : x(a), y(b), z(c) {} };
"""
# build "det": std::cos / std::sin resolve to the oracle's sincos_det (oracle/oracle.cpp:81-94, the same
# Cody-Waite reduction + minimax polynomials as pt_math.h)
DET_TRIG = """
namespace std {
inline void dxrpt_det_sincos(float x, float* s, float* c) {
    float j = std::rint(x * 0.636619772f);
    int q = int(j);
    float y = ((x - j * 1.5703125f) - j * 4.837512969970703125e-4f) - j * 7.549789954891882e-8f;
    float z = y * y;
    float sp = y + (y * z) * (-1.6666654611e-1f + z * (8.3321608736e-3f + z * -1.9515295891e-4f));
    float cp = (1.0f - 0.5f * z) + (z * z) * (4.166664568298827e-2f + z * (-1.388731625493765e-3f + z * 2.443315711809948e-5f));
    switch (q & 3) {
        case 0: *s = sp; *c = cp; break;
        case 1: *s = cp; *c = -sp; break;
        case 2: *s = -sp; *c = -cp; break;
        default: *s = -cp; *c = sp; break;
    }
}
inline float dxrpt_det_cos(float x) { float s, c; dxrpt_det_sincos(x, &s, &c); return c; }
inline float dxrpt_det_sin(float x) { float s, c; dxrpt_det_sincos(x, &s, &c); return s; }
}
#define cos dxrpt_det_cos
#define sin dxrpt_det_sin
"""
DRIVER = r"""
#include <cstring>
static uint32_t bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
int main() {
    char op;
    float a, b;
    while (std::scanf(" %c %a %a", &op, &a, &b) == 3) {
        if (op == 'd') { Float2 r = SquareToConcentricDiskMapping(a, b); std::printf("%u %u\n", bits(r.x), bits(r.y)); }
        else if (op == 'h') { Float3 r = SampleDirectionCosineHemisphere(a, b); std::printf("%u %u %u\n", bits(r.x), bits(r.y), bits(r.z)); }
        else { std::printf("%u\n", bits(GGX_V1(a, b))); }
    }
    return 0;
}
"""


def extract_function(text: str, signature_regex: str) -> str:
    """The function whose signature matches, verbatim through its closing brace."""
    m = re.search(signature_regex, text)
    if not m:
        raise SystemExit(f"not found: {signature_regex}")
    a = m.start()
    b = text.index("{", m.end() - 1) + 1
    depth = 1
    while depth:
        depth += {"{": 1, "}": -1}.get(text[b], 0)
        b += 1
    return text[a:b]


def reference_source() -> str:
    sampling = open(os.path.join(SF12, "Graphics", "Sampling.cpp"), encoding="utf-8", errors="replace").read()
    brdf = open(os.path.join(SF12, "Graphics", "BRDF.h"), encoding="utf-8", errors="replace").read()
    math_h = open(os.path.join(SF12, "SF12_Math.h"), encoding="utf-8", errors="replace").read()
    pi = re.search(r"const float Pi = [0-9.]+f;", math_h).group(0)
    parts = [pi,
             extract_function(sampling, r"Float2 SquareToConcentricDiskMapping\(float x, float y\)\s*\{"),
             extract_function(sampling, r"Float3 SampleDirectionCosineHemisphere\(float u1, float u2\)\s*\{"),
             extract_function(brdf, r"inline float GGX_V1\(float m2, float nDotX\)\s*\{")]
    return "\n".join(parts)


def inputs():
    rng = np.random.default_rng(0x5A3)
    g = np.linspace(0.0, 1.0, 65, dtype=np.float32)
    grid = np.stack(np.meshgrid(g, g, indexing="ij"), -1).reshape(-1, 2)
    # CMJ-like inputs in [0, 1), the disk's region borders (a = +-b), the centre and exact halves
    rnd = rng.random((2048, 2), dtype=np.float32)
    diag = np.stack([g, g], -1)
    anti = np.stack([g, 1.0 - g], -1).astype(np.float32)
    special = np.array([[0.5, 0.5], [0.5, 0.0], [0.0, 0.5], [1.0, 0.5], [0.5, 1.0], [0.0, 0.0], [1.0, 1.0],
                        [np.nextafter(np.float32(0.5), np.float32(1)), 0.5], [0.5, np.nextafter(np.float32(0.5), np.float32(0))],
                        [0.99999994, 0.99999994], [1e-7, 0.75]], dtype=np.float32)
    uv = np.concatenate([grid, rnd, diag, anti, special]).astype(np.float32)
    # GGX_V1: m2 = roughness^2 in [0, 1], nDotX in [0, 1] (saturated dot products)
    m = np.concatenate([grid, rnd, np.array([[0.0, 0.0], [0.0, 1.0], [1.0, 0.0], [1e-8, 1e-8]], dtype=np.float32)])
    return uv, m.astype(np.float32)


def build(src: str, extra: str, name: str) -> str:
    os.makedirs(OUT_DIR, exist_ok=True)
    cpp = os.path.join(OUT_DIR, f"{name}.cpp")
    with open(cpp, "w") as f:
        f.write(PRELUDE + extra + "\n// ---- extracted from the reference checkout ----\n" + src + "\n" + DRIVER)
    exe = os.path.join(OUT_DIR, name)
    # /fp:precise (the reference's MSVC default): no FMA contraction
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", cpp, "-o", exe, "-lm"], check=True)
    return exe


def run(exe: str, uv, m):
    lines = [f"d {float(a).hex()} {float(b).hex()}" for a, b in uv] + [f"h {float(a).hex()} {float(b).hex()}" for a, b in uv] + \
            [f"v {float(a).hex()} {float(b).hex()}" for a, b in m]
    out = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True, check=True).stdout.split("\n")
    n = len(uv)
    disk = np.array([[int(v) for v in out[i].split()] for i in range(n)], dtype=np.uint32)
    hemi = np.array([[int(v) for v in out[n + i].split()] for i in range(n)], dtype=np.uint32)
    v1 = np.array([int(out[2 * n + i]) for i in range(len(m))], dtype=np.uint32)
    return disk, hemi, v1


def main():
    if not os.path.isdir(SF12):
        sys.exit("needs the reference checkout at /root/reference")
    src = reference_source()
    uv, m = inputs()
    exe_libm = build(src, "", "sampling_libm")
    exe_det = build(src, DET_TRIG, "sampling_det")
    d0, h0, v0 = run(exe_libm, uv, m)
    d1, h1, v1 = run(exe_det, uv, m)
    np.savez_compressed(GOLDEN, uv=uv, m2_ndotx=m, disk_libm=d0, hemi_libm=h0, ggx_v1_libm=v0, disk_det=d1, hemi_det=h1,
                        ggx_v1_det=v1,
                        source=np.array("Graphics/Sampling.cpp:167-210,264-279; Graphics/BRDF.h:39-42; SF12_Math.h:551 "
                                        "(compiled verbatim by tests/golden/make_sampling_golden.py)"))
    print(f"wrote {GOLDEN}: {len(uv)} (x, y) inputs, {len(m)} (m2, nDotX) inputs")


if __name__ == "__main__":
    main()
