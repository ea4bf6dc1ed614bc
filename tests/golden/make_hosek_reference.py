#!/usr/bin/env python3
"""Generates tests/golden/hosek_reference.npz from the reference's own sky code (SkyCache::Init + Sample).

Compiled with g++ into oracle/_ref/hosek/ (git-ignored), from the reference checkout at generation time:
  * HosekSky/ArHosekSkyModel.cpp            -- the whole file, verbatim (the model, its datasets via its own
                                                #includes of ArHosekSkyModelData_*.h)
  * Graphics/Spectrum.cpp (+ Spectrum.h)    -- the whole file, verbatim (SampledSpectrum::Init / FromRGB / ToRGB)
  * SF12_Math.cpp  Float3 constructors, arithmetic operators, Float3::Clamp, Float3::Perpendicular,
                   Float3x3(r0, r1, r2)                                   (functions extracted verbatim)
  * SF12_Math.h    the constants and Lerp / Min / Max / Clamp / Saturate / DegToRad   (extracted verbatim)
  * PCH.h          the integer typedefs (extracted verbatim); Assert.h the release Assert_ block (verbatim)
  * Graphics/Sampling.cpp  SampleDirectionCone, SampleDirectionCone_PDF               (extracted verbatim)
  * Graphics/Textures.cpp  MapXYSToDirection                                          (extracted verbatim)
  * Graphics/Skybox.cpp    PhysicalSunSize / CosPhysicalSunSize / AngleBetween / IrradianceIntegral (:31-46),
                           SkyCache::Init's statements :50-56 and :64-154 (after its up-to-date check and
                           Shutdown) and SkyCache::Sample's body :254-269 -- verbatim, around the SkyCache
                           members declared as plain variables.
Added text (types only, plus the one absent third-party dependency):
  * the SF12 struct layouts (Float2, Float3, Float3x3 -- SF12_Math.h also pulls in DirectXMath and Windows
    headers, so it is not compiled itself) and the standard headers PCH.h would bring (with <math.h>, so an
    unqualified sqrt(float) resolves to the float overload as under MSVC's <cmath>);
  * DirectXMath (Windows SDK; not in the checkout) behind Float3::Dot / Cross / Normalize / Transform(Float3x3),
    restated from its published SSE2 paths: XMVector3Dot = (x*x' + y*y') + z*z'; XMVector3Cross = products then
    differences; XMVector3Normalize = v / sqrt(dot); XMVector3TransformCoord with a 3x3 (r3 = (0,0,0,1)) =
    ((z*r2 + r3) + y*r1) + x*r0, then / w (= 1).
Outputs per case: SunIrradiance, SunRenderColor (float32) and the cube as the reference stores it.  The scenes'
skies (full 6 x 128 x 128): the FP16 texels -- Sample()'s float32 radiance through DirectXMath's XMStoreHalf4,
whose scalar path (XMConvertFloatToHalf) rounds to nearest even like numpy's float16 cast, used here -- plus
Sample()'s float32 radiance on every 8th texel row and column.  The sweep cases (6 x 16 x 16): the float32
radiance of every texel.

    python tests/golden/make_hosek_reference.py          (needs /root/reference and g++)
"""
import os
import re
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
SF12 = "/root/reference/SampleFramework12/v1.02"
OUT_DIR = os.path.join(REPO, "oracle", "_ref", "hosek")
INC = os.path.join(OUT_DIR, "inc")
GOLDEN = os.path.join(REPO, "tests", "golden", "hosek_reference.npz")
# the sky inputs: (name, sun direction, sun size (deg), turbidity, ground albedo, cube resolution).  The three
# scenes' skies (their AppSettings sun, the defaults turbidity 2 / albedo 0.25 of DXRPathTracer's settings),
# then a sweep over the model's inputs (turbidity 1..10 -- the solar fit's range --, coloured albedo, low and
# high sun, a sun below the horizon that Init saturates to y = 0, a non-unit direction).
SCENE_RES = 128
SWEEP_RES = 16
SWEEP = [
    ("t1_high", (0.1, 0.95, 0.3), 1.0, 1.0, (0.0, 0.0, 0.0)),
    ("t3_mid", (0.5, 0.5, -0.7), 0.5, 3.0, (0.8, 0.2, 0.1)),
    ("t5_low", (-0.9, 0.12, 0.2), 2.0, 5.5, (0.25, 0.5, 0.75)),
    ("t7_grazing", (0.0, 0.02, 1.0), 1.0, 7.25, (1.0, 1.0, 1.0)),
    ("t10_mid", (0.3, 0.6, 0.2), 3.0, 10.0, (0.1, 0.1, 0.1)),
    ("below_horizon", (0.6, -0.3, 0.4), 1.0, 2.0, (0.25, 0.25, 0.25)),
    ("unnormalised", (2.0, 5.0, -1.0), 0.27, 4.0, (0.4, 0.3, 0.2)),
]


def read(p):
    return open(os.path.join(SF12, p), encoding="utf-8", errors="replace").read()


def extract_function(text, signature_regex):
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


def between(text, start, end, include_end=True):
    """Verbatim text from the first `start` through the first `end` after it."""
    a = text.index(start)
    b = text.index(end, a) + (len(end) if include_end else 0)
    return text[a:b]


def body(fn):
    return fn[fn.index("{") + 1:fn.rindex("}")]


def write(path, text):
    with open(path, "w") as f:
        f.write(text)


def sources():
    pch, assert_h, math_h, math_cpp = read("PCH.h"), read("Assert.h"), read("SF12_Math.h"), read("SF12_Math.cpp")
    sampling, textures, skybox = read("Graphics/Sampling.cpp"), read("Graphics/Textures.cpp"), read("Graphics/Skybox.cpp")
    typedefs = "\n".join(re.findall(r"^typedef \w+ \w+;$", pch, re.M))
    write(os.path.join(INC, "PCH.h"), "#pragma once\n#include <cmath>\n#include <cstdint>\n#include <cstdio>\n#include <cstdlib>\n"
          "#include <cstring>\n#include <limits>\n#include <vector>\n#include <algorithm>\n#include <ostream>\n#include <utility>\n"
          "#include <stdint.h>\n#include <wchar.h>\n#include <math.h>\n// ---- PCH.h, verbatim ----\n" + typedefs + "\n")
    write(os.path.join(INC, "..\\\\Assert.h"), "#pragma once\n// ---- Assert.h, verbatim (release: Assert_ is empty) ----\n" +
          between(assert_h, "#ifdef _DEBUG", "#define StaticAssertMsg_(x, msg)\n#endif") + "\n")
    # SF12_Math.h: types only, then its constants and scalar templates verbatim
    helpers = between(math_h, "const float Pi = ", "inline Float3 Saturate(Float3 val)", include_end=False)
    helpers += extract_function(math_h, r"inline Float3 Saturate\(Float3 val\)\s*\{") + "\n\n"
    helpers += extract_function(math_h, r"inline float DegToRad\(float deg\)\s*\{") + "\n"
    write(os.path.join(INC, "..\\\\SF12_Math.h"), """#pragma once
#include "PCH.h"
#include "..\\\\Assert.h"
namespace SampleFramework12 {
// ---- types only (SF12_Math.h's layouts; the DirectXMath members dropped) ----
struct Float2 { float x, y; };
struct Float3x3;
struct Float3 {
    float x, y, z;
    Float3(); Float3(float x); Float3(float x, float y, float z);
    Float3& operator+=(const Float3& other); Float3 operator+(const Float3& other) const;
    Float3& operator+=(float other); Float3 operator+(float other) const;
    Float3& operator-=(const Float3& other); Float3 operator-(const Float3& other) const;
    Float3& operator-=(float s); Float3 operator-(float s) const;
    Float3& operator*=(const Float3& other); Float3 operator*(const Float3& other) const;
    Float3& operator*=(float s); Float3 operator*(float s) const;
    Float3& operator/=(const Float3& other); Float3 operator/(const Float3& other) const;
    Float3& operator/=(float s); Float3 operator/(float s) const;
    bool operator==(const Float3& other) const; bool operator!=(const Float3& other) const;
    Float3 operator-() const;
    static float Dot(const Float3& a, const Float3& b);
    static Float3 Cross(const Float3& a, const Float3& b);
    static Float3 Normalize(const Float3& a);
    static Float3 Transform(const Float3& v, const Float3x3& m);
    static Float3 Clamp(const Float3& val, const Float3& min, const Float3& max);
    static Float3 Perpendicular(const Float3& v);
};
Float3 operator*(float a, const Float3& b);
struct Float3x3 {
    float _11, _12, _13;
    float _21, _22, _23;
    float _31, _32, _33;
    Float3x3(const Float3& r0, const Float3& r1, const Float3& r2);
};
// ---- SF12_Math.h, verbatim ----
""" + helpers + "}\n")
    # SF12_Math.cpp: the scalar Float3 / Float3x3 members verbatim, DirectXMath's four restated
    ops = between(math_cpp, "Float3::Float3()\n", "Float3::Float3(Float2 xy, float z_)", include_end=False)
    ops += between(math_cpp, "Float3& Float3::operator+=(const Float3& other)", "XMVECTOR Float3::ToSIMD() const", include_end=False)
    ops += extract_function(math_cpp, r"Float3 Float3::Clamp\(const Float3& val, const Float3& min, const Float3& max\)\s*\{") + "\n\n"
    ops += extract_function(math_cpp, r"Float3 Float3::Perpendicular\(const Float3& vec\)\s*\{") + "\n\n"
    ops += extract_function(math_cpp, r"Float3x3::Float3x3\(const Float3& r0, const Float3& r1, const Float3& r2\)\s*\{") + "\n"
    write(os.path.join(OUT_DIR, "sf12_math.cpp"), """#include "PCH.h"
#include "..\\\\SF12_Math.h"
namespace SampleFramework12 {
// ---- DirectXMath (absent third-party dependency), restated from its SSE2 paths ----
float Float3::Dot(const Float3& a, const Float3& b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
Float3 Float3::Cross(const Float3& a, const Float3& b) {
    Float3 r; r.x = a.y * b.z - a.z * b.y; r.y = a.z * b.x - a.x * b.z; r.z = a.x * b.y - a.y * b.x; return r; }
Float3 Float3::Normalize(const Float3& a) {
    float l = std::sqrt((a.x * a.x + a.y * a.y) + a.z * a.z);
    Float3 r; if (l == 0.0f) return r;  // XMVector3Normalize: zero length -> zero vector
    r.x = a.x / l; r.y = a.y / l; r.z = a.z / l; return r; }
Float3 Float3::Transform(const Float3& v, const Float3x3& m) {
    float rx = v.z * m._31 + 0.0f, ry = v.z * m._32 + 0.0f, rz = v.z * m._33 + 0.0f, rw = v.z * 0.0f + 1.0f;
    rx = v.y * m._21 + rx; ry = v.y * m._22 + ry; rz = v.y * m._23 + rz; rw = v.y * 0.0f + rw;
    rx = v.x * m._11 + rx; ry = v.x * m._12 + ry; rz = v.x * m._13 + rz; rw = v.x * 0.0f + rw;
    return Float3(rx / rw, ry / rw, rz / rw); }
// ---- SF12_Math.cpp, verbatim ----
""" + ops + "}\n")
    init = extract_function(skybox, r"bool SkyCache::Init\(const Float3& sunDirection_, float sunSize, const Float3& groundAlbedo_, float turbidity, bool createCubemap\)\s*\{")
    init_a = between(init, "Float3 sunDirection = sunDirection_;", "sunSize = Max(sunSize, 0.01f);")
    init_b = between(init, "Shutdown();", "SunRenderColor = Float3::Clamp(sunColor, 0.0f, FP16Max);")[len("Shutdown();"):]
    sample = extract_function(skybox, r"Float3 SkyCache::Sample\(Float3 sampleDir\) const\s*\{")
    statics = between(skybox, "// Actual physical size of the sun", "return Pi * sinTheta * sinTheta;\n}")
    write(os.path.join(OUT_DIR, "sky_driver.cpp"), """#include "PCH.h"
#include "..\\\\SF12_Math.h"
#include "ArHosekSkyModel.h"
#include "Spectrum.h"
namespace SampleFramework12 {
// ---- Graphics/Sampling.cpp, Graphics/Textures.cpp: verbatim ----
""" + extract_function(sampling, r"Float3 SampleDirectionCone\(float u1, float u2, float cosThetaMax\)\s*\{") + "\n\n" +
          extract_function(sampling, r"float SampleDirectionCone_PDF\(float cosThetaMax\)\s*\{") + "\n\n" +
          extract_function(textures, r"Float3 MapXYSToDirection\(uint64 x, uint64 y, uint64 s, uint64 width, uint64 height\)\s*\{") + """

// ---- Graphics/Skybox.cpp :31-46, verbatim ----
""" + statics + """

// SkyCache's members (Skybox.h) as plain variables
ArHosekSkyModelState* StateR = nullptr;
ArHosekSkyModelState* StateG = nullptr;
ArHosekSkyModelState* StateB = nullptr;
float Turbidity = 0.0f, Elevation = 0.0f, SunSize = 0.0f;
Float3 SunDirection, Albedo, SunRadiance, SunIrradiance, SunRenderColor;

void SkyInit(const Float3& sunDirection_, float sunSize, const Float3& groundAlbedo_, float turbidity)
{
    // ---- SkyCache::Init (Skybox.cpp:50-56, 64-154), verbatim ----
    """ + init_a + "\n" + init_b + """
}

Float3 SkySample(Float3 sampleDir)
{
    // ---- SkyCache::Sample (Skybox.cpp:254-269), verbatim ----
""" + body(sample) + """
}
}  // namespace SampleFramework12

using namespace SampleFramework12;
int main(int argc, char** argv)
{
    SampledSpectrum::Init();  // App.cpp:45
    float sx, sy, sz, size, turb, ax, ay, az;
    unsigned res;
    if (std::scanf("%a %a %a %a %a %a %a %a %u", &sx, &sy, &sz, &size, &turb, &ax, &ay, &az, &res) != 9) return 2;
    SkyInit(Float3(sx, sy, sz), size, Float3(ax, ay, az), turb);
    FILE* f = std::fopen(argv[1], "wb");
    const float head[6] = {SunIrradiance.x, SunIrradiance.y, SunIrradiance.z, SunRenderColor.x, SunRenderColor.y, SunRenderColor.z};
    std::fwrite(head, 4, 6, f);
    for (uint64 s = 0; s < 6; ++s)
        for (uint64 y = 0; y < res; ++y)
            for (uint64 x = 0; x < res; ++x) {
                Float3 r = SkySample(MapXYSToDirection(x, y, s, res, res));  // Skybox.cpp:176-177
                std::fwrite(&r, 4, 3, f);
            }
    std::fclose(f);
    arhosekskymodelstate_free(StateR);
    arhosekskymodelstate_free(StateG);
    arhosekskymodelstate_free(StateB);
    return 0;
}
""")


def build():
    os.makedirs(INC, exist_ok=True)
    sources()
    flags = ["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-w", "-I", INC,
             "-I", os.path.join(SF12, "HosekSky"), "-I", os.path.join(SF12, "Graphics")]
    objs = []
    for src in (os.path.join(SF12, "HosekSky", "ArHosekSkyModel.cpp"), os.path.join(SF12, "Graphics", "Spectrum.cpp"),
                os.path.join(OUT_DIR, "sf12_math.cpp"), os.path.join(OUT_DIR, "sky_driver.cpp")):
        o = os.path.join(OUT_DIR, os.path.basename(src) + ".o")
        subprocess.run(flags + ["-c", src, "-o", o], check=True)
        objs.append(o)
    exe = os.path.join(OUT_DIR, "sky_reference")
    subprocess.run(["g++", *objs, "-o", exe, "-lm"], check=True)
    return exe


def run(exe, sun, size, turb, albedo, res):
    out = os.path.join(OUT_DIR, "out.bin")
    args = [*sun, size, turb, *albedo]
    subprocess.run([exe, out], input=" ".join(float(np.float32(v)).hex() for v in args) + f" {res}\n", text=True, check=True)
    v = np.fromfile(out, dtype=np.float32)
    return v[:3].copy(), v[3:6].copy(), v[6:].reshape(6, res, res, 3)


def main():
    if not os.path.isdir(SF12):
        sys.exit("needs the reference checkout at /root/reference")
    import dxrpathtracer_amd as D
    exe = build()
    cases = []
    for name in ("sponza", "suntemple", "boxtest"):
        st = D.Scene(name).settings()
        if any(tuple(st.SunDirection) == c[1] and float(st.SunSize) == c[2] for c in cases):
            continue  # the same sky as an earlier scene's
        cases.append((name, tuple(st.SunDirection), float(st.SunSize), float(D.scene.DEFAULT_TURBIDITY),
                      tuple(D.scene.DEFAULT_GROUND_ALBEDO), SCENE_RES))
    cases += [(n, s, z, t, a, SWEEP_RES) for n, s, z, t, a in SWEEP]
    out = {"names": np.array([c[0] for c in cases]),
           "params": np.array([[*c[1], c[2], c[3], *c[4]] for c in cases], dtype=np.float32),
           "res": np.array([c[5] for c in cases], dtype=np.int32),
           "source": np.array("HosekSky/ArHosekSkyModel.cpp, Graphics/Spectrum.cpp (whole files); SF12_Math.{h,cpp}, "
                              "Graphics/{Sampling,Textures}.cpp, Graphics/Skybox.cpp:31-46,50-56,64-154,254-269 "
                              "(compiled verbatim by tests/golden/make_hosek_reference.py)")}
    for name, sun, size, turb, alb, res in cases:
        irr, ren, cube = run(exe, sun, size, turb, alb, res)
        out[f"{name}_sun_irradiance"] = irr
        out[f"{name}_sun_render_color"] = ren
        if res == SCENE_RES:
            out[f"{name}_cube_f16"] = cube.astype(np.float16).view(np.uint16)
            out[f"{name}_cube_f32_every8"] = cube[:, 4::8, 4::8].copy()
        else:
            out[f"{name}_cube"] = cube
        print(f"{name:14s} irradiance {irr} render {ren} cube {cube.shape}")
    np.savez_compressed(GOLDEN, **out)
    print(f"wrote {GOLDEN} ({os.path.getsize(GOLDEN)} bytes)")


if __name__ == "__main__":
    main()
