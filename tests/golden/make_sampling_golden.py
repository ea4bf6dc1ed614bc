#!/usr/bin/env python3
"""Generates tests/golden/sampling_reference.npz from the reference's own sampling and BRDF C++ code.

The reference's C++ twins of the shader functions the path tracer uses -- read out of the checkout at
generation time, compiled verbatim with g++ into oracle/_ref/ (git-ignored) and run on dense input grids:
  * SampleFramework12/v1.02/Graphics/Sampling.cpp:167-210  SquareToConcentricDiskMapping
    (statement-identical to Shaders/Sampling.hlsl:72-114, the kernels' sample_cosine_hemisphere first half)
  * Sampling.cpp:264-279  SampleDirectionCosineHemisphere  (Sampling.hlsl:181-196; RayTrace.hlsl:333's
    diffuse lobe, Baking.hlsl's bake ray)
  * Graphics/BRDF.h:39-42  GGX_V1  (BRDF.hlsl:89-92, inside GGXVisibility / CalcLighting)
  * Graphics/BRDF.h:17-26  Fresnel(specAlbedo, h, l)  (statement-identical to BRDF.hlsl:16-24; CalcLighting's)
  * Graphics/BRDF.h:59-77  GGX_Specular  (BRDF.hlsl:128-145's GGXSpecular up to one association: the C++
    divides by Pi * Square(x), the HLSL by (Pi * x) * x -- so a stated bound, never bit equality)
The SF12 types and scalar helpers they use come from tests/golden/make_hosek_reference.py's verbatim
extracts of SF12_Math.{h,cpp} (types-only layouts, DirectXMath's Float3 ops restated from its SSE2 paths).
Two builds of the same extracted text:
  build "libm"  -- std::cos / std::sin / std::pow are glibc's, as written;
  build "det"   -- the same text with std::cos / std::sin routed to the deterministic sin/cos the oracle and the
                   kernels define (pt_math.h pt_sincos, oracle.cpp sincos_det) and std::pow(x, 5) to the
                   (x*x)*(x*x)*x the HLSL pow(x, 5) is defined as here (pt_math.h pow5; a diagnostic build: it
                   shows that every other operation of the reference's arithmetic is reproduced bit for bit).
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

PRELUDE = """#include "PCH.h"
#include "..\\\\SF12_Math.h"
using namespace SampleFramework12;
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
inline float dxrpt_det_pow(float x, float e) { if (e != 5.0f) std::abort(); float x2 = x * x; return (x2 * x2) * x; }
}
#define cos dxrpt_det_cos
#define sin dxrpt_det_sin
#define pow dxrpt_det_pow
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
        else if (op == 'v') { std::printf("%u\n", bits(GGX_V1(a, b))); }
        else if (op == 'f') {  // a, b read above are specAlbedo.x, .y; then z, h, l
            float r[7];
            for (float& v : r) if (std::scanf(" %a", &v) != 1) return 2;
            Float3 f = Fresnel(Float3(a, b, r[0]), Float3(r[1], r[2], r[3]), Float3(r[4], r[5], r[6]));
            std::printf("%u %u %u\n", bits(f.x), bits(f.y), bits(f.z));
        } else {  // 's': m, n.x read above; then n.yz, h, v, l
            float r[11];
            for (float& v : r) if (std::scanf(" %a", &v) != 1) return 2;
            std::printf("%u\n", bits(GGX_Specular(a, Float3(b, r[0], r[1]), Float3(r[2], r[3], r[4]), Float3(r[5], r[6], r[7]),
                                                    Float3(r[8], r[9], r[10]))));
        }
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
    parts = [extract_function(math_h, r"template<typename T> T Square\(T x\)\s*\{"),extract_function(sampling, r"Float2 SquareToConcentricDiskMapping\(float x, float y\)\s*\{"),
             extract_function(sampling, r"Float3 SampleDirectionCosineHemisphere\(float u1, float u2\)\s*\{"),
             extract_function(brdf, r"inline float GGX_V1\(float m2, float nDotX\)\s*\{"),
             extract_function(brdf, r"inline Float3 Fresnel\(Float3 specAlbedo, Float3 h, Float3 l\)\s*\{"),
             extract_function(brdf, r"inline float GGX_Specular\(float m, const Float3& n, const Float3& h, const Float3& v, "
                                    r"const Float3& l\)\s*\{")]
    return "namespace SampleFramework12 {\n" + "\n".join(parts) + "\n}\n"


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


def unit(rng, n):
    v = rng.normal(size=(n, 3)).astype(np.float32)
    return (v / np.linalg.norm(v, axis=1, keepdims=True)).astype(np.float32)


def brdf_inputs():
    """Fresnel: (specAlbedo in [0, 1]^3 -- some below the 0.1 % fade --, unit h, unit l); GGX_Specular: (m in
    (0, 1], unit n, h = normalize(v + l), unit v, unit l), the way CalcLighting forms them."""
    rng = np.random.default_rng(0xB2DF)
    n = 4096
    spec = rng.random((n, 3), dtype=np.float32)
    spec[: n // 8] *= np.float32(0.004)
    spec[n // 8: n // 8 + 16] = np.float32(0.0)
    spec[n // 8 + 16: n // 8 + 32] = np.float32(1.0)
    fres = np.concatenate([spec, unit(rng, n), unit(rng, n)], axis=1).astype(np.float32)
    mr = rng.random((n, 1), dtype=np.float32) * np.float32(0.999) + np.float32(0.001)
    nn, v, l = unit(rng, n), unit(rng, n), unit(rng, n)
    h = v + l
    h = (h / np.linalg.norm(h, axis=1, keepdims=True)).astype(np.float32)
    spec_in = np.concatenate([mr, nn, h, v, l], axis=1).astype(np.float32)
    return fres, spec_in


def sf12():
    """The SF12 types and scalar members (verbatim extracts + DirectXMath's Float3 ops restated) written by
    tests/golden/make_hosek_reference.py: (include dir, compiled sf12_math object)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_hosek_reference", os.path.join(os.path.dirname(__file__),
                                                                                         "make_hosek_reference.py"))
    H = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(H)
    os.makedirs(H.INC, exist_ok=True)
    H.sources()
    obj = os.path.join(OUT_DIR, "sf12_math.o")
    os.makedirs(OUT_DIR, exist_ok=True)
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-w", "-I", H.INC, "-c",
                    os.path.join(H.OUT_DIR, "sf12_math.cpp"), "-o", obj], check=True)
    return H.INC, obj


def build(src: str, extra: str, name: str, inc: str, obj: str) -> str:
    os.makedirs(OUT_DIR, exist_ok=True)
    cpp = os.path.join(OUT_DIR, f"{name}.cpp")
    with open(cpp, "w") as f:
        f.write(PRELUDE + extra + "\n// ---- extracted from the reference checkout ----\n" + src + "\n" + DRIVER)
    exe = os.path.join(OUT_DIR, name)
    # /fp:precise (the reference's MSVC default): no FMA contraction
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-w", "-I", inc, cpp, obj, "-o", exe,
                    "-lm"], check=True)
    return exe


def hexs(row):
    return " ".join(float(v).hex() for v in row)


def run(exe: str, uv, m, fres, spec_in):
    lines = [f"d {hexs(r)}" for r in uv] + [f"h {hexs(r)}" for r in uv] + [f"v {hexs(r)}" for r in m] + \
            [f"f {hexs(r)}" for r in fres] + [f"s {hexs(r)}" for r in spec_in]
    out = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True, check=True).stdout.split("\n")
    n, k = len(uv), 0

    def take(count, width=None):
        nonlocal k
        rows = out[k:k + count]
        k += count
        if width is None:
            return np.array([int(r) for r in rows], dtype=np.uint32)
        return np.array([[int(v) for v in r.split()] for r in rows], dtype=np.uint32)
    return take(n, 2), take(n, 3), take(len(m)), take(len(fres), 3), take(len(spec_in))


def main():
    if not os.path.isdir(SF12):
        sys.exit("needs the reference checkout at /root/reference")
    src = reference_source()
    uv, m = inputs()
    fres, spec_in = brdf_inputs()
    inc, obj = sf12()
    exe_libm = build(src, "", "sampling_libm", inc, obj)
    exe_det = build(src, DET_TRIG, "sampling_det", inc, obj)
    d0, h0, v0, f0, s0 = run(exe_libm, uv, m, fres, spec_in)
    d1, h1, v1, f1, s1 = run(exe_det, uv, m, fres, spec_in)
    np.savez_compressed(GOLDEN, uv=uv, m2_ndotx=m, disk_libm=d0, hemi_libm=h0, ggx_v1_libm=v0, disk_det=d1, hemi_det=h1,
                        ggx_v1_det=v1, fresnel_in=fres, fresnel_libm=f0, fresnel_det=f1, ggx_spec_in=spec_in,
                        ggx_spec_libm=s0, ggx_spec_det=s1,
                        source=np.array("Graphics/Sampling.cpp:167-210,264-279; Graphics/BRDF.h:17-26,39-42,59-77; "
                                        "SF12_Math.h/.cpp (compiled verbatim by tests/golden/make_sampling_golden.py)"))
    print(f"wrote {GOLDEN}: {len(uv)} (x, y) inputs, {len(m)} (m2, nDotX) inputs, {len(fres)} Fresnel and "
          f"{len(spec_in)} GGX_Specular inputs")


if __name__ == "__main__":
    main()
