// oracle.cpp — CPU restatement of the reference DXR path tracer (the parity ORACLE).
//
// TEST INFRASTRUCTURE ONLY.  This file is the checker for the MI355X kernels in
// dxrpathtracer_amd/csrc.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
// load it, and only to check or to time the CPU baseline.  The product never links or calls it.
//
// It restates, scalar and recursive like the reference, with every function citing the reference
// file:line it follows (paths relative to the reference tree):
//   DXRPathTracer/RayTrace.hlsl            RaygenShader 92-149, PathTrace 151-441, GetHitSurface 444-464,
//                                          GetGeometryMaterial 467-474, ClosestHit 476-483, AnyHit 485-507,
//                                          Miss 509-530, ShadowHit/Miss 532-542, SamplePoint 85-90
//   SampleFramework12/v1.02/Shaders/BRDF.hlsl      16-24, 89-145, 209-261
//   SampleFramework12/v1.02/Shaders/Sampling.hlsl  72-114, 131-154, 181-196, 282-331
//   SampleFramework12/v1.02/Shaders/RayTracing.hlsl 13-53, Shaders/Constants.hlsl 13-27
// It owns its own acceleration structure (a binned-SAH BVH built here, not the product's), so the
// closest hit is checked independently of the product's tree: hits are decided only by the exact
// triangle test and the tie rule (smallest t, then smallest global triangle id).
//
// Conventions that the reference leaves to D3D/driver rounding (parity UNPINNED against D3D, fixed
// identically here and in dxrpathtracer_amd/csrc/pt_math.h): dot order (x+y)+z, normalize = v/sqrt,
// pow(x,5) = x^2*x^2*x, sin/cos = the Cody-Waite/minimax pair below, bilinear wrap texture filter,
// cube face selection + per-face bilinear clamp, Moller-Trumbore two-sided triangle test.
// Compiled with -ffp-contract=off -fno-fast-math: every expression rounds exactly as written.
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

#include "oracle.h"

namespace {

// ---- Shaders/Constants.hlsl:13-27 ----------------------------------------------------------------
const float kPi = 3.141592654f;
const float kFP32Max = 3.402823466e+38f;
const float kFP16Max = 65000.0f;
const float kRayTMin = 0.00001f;            // RayTrace.hlsl:243, 382
const float kSpotShadowNearClip = 0.1f;     // AppSettings.hlsl:56
const uint32_t kNone = 0xFFFFFFFFu;

struct F3 {
    float x, y, z;
};
inline F3 f3(float x, float y, float z) { return F3{x, y, z}; }
inline F3 operator+(F3 a, F3 b) { return F3{a.x + b.x, a.y + b.y, a.z + b.z}; }
inline F3 operator-(F3 a, F3 b) { return F3{a.x - b.x, a.y - b.y, a.z - b.z}; }
inline F3 operator*(F3 a, F3 b) { return F3{a.x * b.x, a.y * b.y, a.z * b.z}; }
inline F3 operator*(F3 a, float s) { return F3{a.x * s, a.y * s, a.z * s}; }
inline F3 operator-(F3 a) { return F3{-a.x, -a.y, -a.z}; }
inline float dot(F3 a, F3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
inline F3 cross(F3 a, F3 b) { return F3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline float length(F3 a) { return std::sqrt(dot(a, a)); }
inline F3 normalize(F3 a) {
    float l = std::sqrt(dot(a, a));
    return F3{a.x / l, a.y / l, a.z / l};
}
inline float saturate(float x) { return std::fmin(std::fmax(x, 0.0f), 1.0f); }
inline float lerp(float a, float b, float t) { return a + t * (b - a); }
// HLSL reflect(i, n) = i - 2 * n * dot(i, n)
inline F3 reflect(F3 i, F3 n) {
    float d = dot(i, n);
    return F3{i.x - (2.0f * n.x) * d, i.y - (2.0f * n.y) * d, i.z - (2.0f * n.z) * d};
}
inline float pow5(float x) {
    float x2 = x * x;
    return (x2 * x2) * x;
}
// HLSL smoothstep
inline float smoothstep(float a, float b, float x) {
    float t = saturate((x - a) / (b - a));
    return t * t * (3.0f - 2.0f * t);
}

void sincos_det(float x, float* s, float* c) {
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

// ---- Sampling.hlsl:282-331 --------------------------------------------------------------------------
uint32_t CMJPermute(uint32_t i, uint32_t l, uint32_t p) {
    uint32_t w = l - 1;
    w |= w >> 1;
    w |= w >> 2;
    w |= w >> 4;
    w |= w >> 8;
    w |= w >> 16;
    do {
        i ^= p;
        i *= 0xe170893du;
        i ^= p >> 16;
        i ^= (i & w) >> 4;
        i ^= p >> 8;
        i *= 0x0929eb3fu;
        i ^= p >> 23;
        i ^= (i & w) >> 1;
        i *= 1u | p >> 27;
        i *= 0x6935fa69u;
        i ^= (i & w) >> 11;
        i *= 0x74dcb303u;
        i ^= (i & w) >> 2;
        i *= 0x9e501cc3u;
        i ^= (i & w) >> 2;
        i *= 0xc860a3dfu;
        i &= w;
        i ^= i >> 5;
    } while (i >= l);
    return (i + p) % l;
}
float CMJRandFloat(uint32_t i, uint32_t p) {
    i ^= p;
    i ^= i >> 17;
    i ^= i >> 10;
    i *= 0xb36534e5u;
    i ^= i >> 12;
    i ^= i >> 21;
    i *= 0x93fc4795u;
    i ^= 0xdf6e307fu;
    i ^= i >> 17;
    i *= 1u | p >> 18;
    return float(i) * (1.0f / 4294967808.0f);
}
void SampleCMJ2D(uint32_t sampleIdx, uint32_t numSamplesX, uint32_t numSamplesY, uint32_t pattern, float out[2]) {
    uint32_t N = numSamplesX * numSamplesY;
    sampleIdx = CMJPermute(sampleIdx, N, pattern * 0x51633e2du);
    uint32_t sx = CMJPermute(sampleIdx % numSamplesX, numSamplesX, pattern * 0x68bc21ebu);
    uint32_t sy = CMJPermute(sampleIdx / numSamplesX, numSamplesY, pattern * 0x02e5be93u);
    float jx = CMJRandFloat(sampleIdx, pattern * 0x967a889bu);
    float jy = CMJRandFloat(sampleIdx, pattern * 0x368cc8b7u);
    out[0] = (float(sx) + (float(sy) + jx) / float(numSamplesY)) / float(numSamplesX);
    out[1] = (float(sampleIdx) + jy) / float(N);
}

// ---- Sampling.hlsl:72-114 (SquareToConcentricDiskMapping), 181-196 (cosine hemisphere) ---------------
void SquareToConcentricDiskMapping(float x, float y, float out[2]) {
    float phi = 0.0f;
    float r = 0.0f;
    float a = 2.0f * x - 1.0f;
    float b = 2.0f * y - 1.0f;
    if (a > -b) {
        if (a > b) {
            r = a;
            phi = (kPi / 4.0f) * (b / a);
        } else {
            r = b;
            phi = (kPi / 4.0f) * (2.0f - (a / b));
        }
    } else {
        if (a < b) {
            r = -a;
            phi = (kPi / 4.0f) * (4.0f + (b / a));
        } else {
            r = -b;
            if (b != 0)
                phi = (kPi / 4.0f) * (6.0f - (a / b));
            else
                phi = 0;
        }
    }
    float s, c;
    sincos_det(phi, &s, &c);
    out[0] = r * c;
    out[1] = r * s;
}
F3 SampleDirectionCosineHemisphere(float u1, float u2) {
    float uv[2];
    SquareToConcentricDiskMapping(u1, u2, uv);
    float u = uv[0], v = uv[1];
    float r = u * u + v * v;
    return F3{u, v, std::sqrt(std::fmax(0.0f, 1.0f - r))};
}
// Sampling.hlsl:131-154
F3 SampleGGXVisibleNormal(F3 wo, float ax, float ay, float u1, float u2) {
    F3 v = normalize(F3{wo.x * ax, wo.y * ay, wo.z});
    F3 t1 = (v.z < 0.999f) ? normalize(cross(v, F3{0, 0, 1})) : F3{1, 0, 0};
    F3 t2 = cross(t1, v);
    float a = 1.0f / (1.0f + v.z);
    float r = std::sqrt(u1);
    float phi = (u2 < a) ? (u2 / a) * kPi : kPi + ((u2 - a) / (1.0f - a)) * kPi;
    float s, c;
    sincos_det(phi, &s, &c);
    float p1 = r * c;
    float p2 = (r * s) * ((u2 < a) ? 1.0f : v.z);
    F3 n = (t1 * p1 + t2 * p2) + v * std::sqrt(std::fmax(0.0f, (1.0f - p1 * p1) - p2 * p2));
    return normalize(F3{ax * n.x, ay * n.y, std::fmax(0.0f, n.z)});
}

// ---- BRDF.hlsl ---------------------------------------------------------------------------------------
F3 Fresnel(F3 specAlbedo, F3 h, F3 l) {  // 16-24
    float p = pow5(1.0f - saturate(dot(l, h)));
    float fade = saturate(dot(specAlbedo, F3{333.0f, 333.0f, 333.0f}));
    return F3{(specAlbedo.x + (1.0f - specAlbedo.x) * p) * fade, (specAlbedo.y + (1.0f - specAlbedo.y) * p) * fade,
              (specAlbedo.z + (1.0f - specAlbedo.z) * p) * fade};
}
float GGXV1(float m2, float nDotX) { return 1.0f / (nDotX + std::sqrt(m2 + ((1 - m2) * nDotX) * nDotX)); }  // 89-92
float GGXVisibility(float m2, float nDotL, float nDotV) { return GGXV1(m2, nDotL) * GGXV1(m2, nDotV); }  // 97-100
float SmithGGXMasking(F3 n, F3 l, F3 v, float a2) {  // 102-109
    (void)l;
    float dotNV = saturate(dot(n, v));
    float denomC = std::sqrt(a2 + ((1.0f - a2) * dotNV) * dotNV) + dotNV;
    return (2.0f * dotNV) / denomC;
}
float SmithGGXMaskingShadowing(F3 n, F3 l, F3 v, float a2) {  // 111-120
    float dotNL = saturate(dot(n, l));
    float dotNV = saturate(dot(n, v));
    float denomA = dotNV * std::sqrt(a2 + ((1.0f - a2) * dotNL) * dotNL);
    float denomB = dotNL * std::sqrt(a2 + ((1.0f - a2) * dotNV) * dotNV);
    return ((2.0f * dotNL) * dotNV) / (denomA + denomB);
}
float GGXSpecular(float m, F3 n, F3 h, F3 v, F3 l) {  // 128-145
    float nDotH = saturate(dot(n, h));
    float nDotL = saturate(dot(n, l));
    float nDotV = saturate(dot(n, v));
    float m2 = m * m;
    float x = (nDotH * nDotH) * (m2 - 1) + 1;
    float d = m2 / ((kPi * x) * x);
    float vis = GGXVisibility(m2, nDotL, nDotV);
    return d * vis;
}
float GGXEnvironmentBRDFScale(float nDotV, float sqrtRoughness) {  // 209-224 (.x)
    const float nDotV2 = nDotV * nDotV;
    const float sqrtRoughness2 = sqrtRoughness * sqrtRoughness;
    const float sqrtRoughness3 = sqrtRoughness2 * sqrtRoughness;
    const float delta = ((0.991086418474895f + (0.412367709802119f * sqrtRoughness) * nDotV2) -
                         (0.363848256078895f * sqrtRoughness2)) -
                        ((0.758634385642633f * nDotV) * sqrtRoughness2);
    const float bias = saturate(((0.0306613448029984f * sqrtRoughness) +
                                 0.0238299731830387f / ((0.0272458171384516f + sqrtRoughness3) + nDotV2)) -
                                0.0454747751719356f);
    return saturate(delta - bias);
}
F3 CalcLighting(F3 normal, F3 lightDir, F3 peakIrradiance, F3 diffuseAlbedo, F3 specularAlbedo, float roughness,
                F3 positionWS, F3 cameraPosWS, F3 msEnergyCompensation) {  // 241-261
    F3 lighting = diffuseAlbedo * (1.0f / 3.14159f);
    F3 view = normalize(cameraPosWS - positionWS);
    const float nDotL = saturate(dot(normal, lightDir));
    if (nDotL > 0.0f) {
        F3 h = normalize(view + lightDir);
        F3 fresnel = Fresnel(specularAlbedo, h, lightDir);
        float specular = GGXSpecular(roughness, normal, h, view, lightDir);
        lighting = lighting + (fresnel * specular) * msEnergyCompensation;
    }
    return (lighting * nDotL) * peakIrradiance;
}

// ---- scene, textures, sky -----------------------------------------------------------------------------
struct Tex {
    uint32_t w, h, fmt;
    const uint8_t* data;
};

struct Scene {
    const oracle_vertex* vtx = nullptr;
    std::vector<uint32_t> idx;
    const oracle_geometry_info* geo = nullptr;
    uint32_t ngeo = 0;
    const oracle_material* mat = nullptr;
    uint32_t nmat = 0;
    std::vector<Tex> tex;
    const uint16_t* sky = nullptr;
    uint32_t sky_res = 0;
    float lut_unorm[256], lut_srgb[256];
    // triangles in global order: v0, e1, e2; geometry; opaque flag
    std::vector<float> tv;  // 9 per tri
    std::vector<uint32_t> tgeom;
    std::vector<uint8_t> topaque;
    // BVH
    struct Node {
        float lo[3], hi[3];
        uint32_t left;   // internal: index of the left child (right = left + 1); leaf: first ref
        uint32_t count;  // 0 internal, > 0 leaf
    };
    std::vector<Node> nodes;
    std::vector<uint32_t> refs;
};

float half_to_float(uint16_t h) {
    uint32_t sign = uint32_t(h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1Fu, m = h & 0x3FFu;
    uint32_t x;
    if (e == 0) {
        if (m == 0)
            x = sign;
        else {
            int k = 0;
            while (!(m & 0x400u)) { m <<= 1; ++k; }
            x = sign | (uint32_t(127 - 15 + 1 - k) << 23) | ((m & 0x3FFu) << 13);
        }
    } else if (e == 31) {
        x = sign | 0x7F800000u | (m << 13);
    } else {
        x = sign | ((e - 15 + 127) << 23) | (m << 13);
    }
    float f;
    std::memcpy(&f, &x, 4);
    return f;
}

struct T4 {
    float r, g, b, a;
};

inline int wrap(int i, uint32_t n) {
    int m = i % int(n);
    return m < 0 ? m + int(n) : m;
}

T4 texel(const Scene& S, const Tex& t, int x, int y) {
    const size_t i = size_t(y) * t.w + size_t(x);
    T4 o;
    if (t.fmt == ORACLE_TEX_R8_UNORM) {
        float v = S.lut_unorm[t.data[i]];
        o.r = v; o.g = v; o.b = v; o.a = 1.0f;
    } else {
        const uint8_t* p = t.data + i * 4;
        const float* l = t.fmt == ORACLE_TEX_RGBA8_SRGB ? S.lut_srgb : S.lut_unorm;
        o.r = l[p[0]];
        o.g = l[p[1]];
        o.b = l[p[2]];
        o.a = S.lut_unorm[p[3]];
    }
    return o;
}

// SampleLevel(MeshSampler, uv, 0): bilinear, wrap, mip 0 (see file header)
T4 SampleTex(const Scene& S, uint32_t idx, float u, float v) {
    const Tex& t = S.tex[idx];
    float x = u * float(t.w) - 0.5f;
    float y = v * float(t.h) - 0.5f;
    float x0 = std::floor(x), y0 = std::floor(y);
    float fx = x - x0, fy = y - y0;
    int ix0 = wrap(int(x0), t.w), ix1 = wrap(int(x0) + 1, t.w);
    int iy0 = wrap(int(y0), t.h), iy1 = wrap(int(y0) + 1, t.h);
    T4 a = texel(S, t, ix0, iy0), b = texel(S, t, ix1, iy0), c = texel(S, t, ix0, iy1), d = texel(S, t, ix1, iy1);
    return T4{lerp(lerp(a.r, b.r, fx), lerp(c.r, d.r, fx), fy), lerp(lerp(a.g, b.g, fx), lerp(c.g, d.g, fx), fy),
              lerp(lerp(a.b, b.b, fx), lerp(c.b, d.b, fx), fy), lerp(lerp(a.a, b.a, fx), lerp(c.a, d.a, fx), fy)};
}

// TextureCube.SampleLevel(LinearSampler, dir, 0): major axis face (x, then y, then z on ties),
// bilinear clamped to the face.
F3 SampleSky(const Scene& S, F3 d) {
    float ax = std::fabs(d.x), ay = std::fabs(d.y), az = std::fabs(d.z);
    int face;
    float ma, sc, tc;
    if (ax >= ay && ax >= az) {
        face = d.x >= 0.0f ? 0 : 1; ma = ax; sc = d.x >= 0.0f ? -d.z : d.z; tc = -d.y;
    } else if (ay >= az) {
        face = d.y >= 0.0f ? 2 : 3; ma = ay; sc = d.x; tc = d.y >= 0.0f ? d.z : -d.z;
    } else {
        face = d.z >= 0.0f ? 4 : 5; ma = az; sc = d.z >= 0.0f ? d.x : -d.x; tc = -d.y;
    }
    const uint32_t R = S.sky_res;
    float u = (sc / ma + 1.0f) * 0.5f, v = (tc / ma + 1.0f) * 0.5f;
    float x = u * float(R) - 0.5f, y = v * float(R) - 0.5f;
    float x0 = std::floor(x), y0 = std::floor(y);
    float fx = x - x0, fy = y - y0;
    const int rmax = int(R) - 1;
    int ix0 = std::min(std::max(int(x0), 0), rmax), ix1 = std::min(std::max(int(x0) + 1, 0), rmax);
    int iy0 = std::min(std::max(int(y0), 0), rmax), iy1 = std::min(std::max(int(y0) + 1, 0), rmax);
    const uint16_t* f = S.sky + size_t(face) * R * R * 4;
    auto at = [&](int xx, int yy, int ch) { return half_to_float(f[(size_t(yy) * R + xx) * 4 + ch]); };
    F3 o;
    o.x = lerp(lerp(at(ix0, iy0, 0), at(ix1, iy0, 0), fx), lerp(at(ix0, iy1, 0), at(ix1, iy1, 0), fx), fy);
    o.y = lerp(lerp(at(ix0, iy0, 1), at(ix1, iy0, 1), fx), lerp(at(ix0, iy1, 1), at(ix1, iy1, 1), fx), fy);
    o.z = lerp(lerp(at(ix0, iy0, 2), at(ix1, iy0, 2), fx), lerp(at(ix0, iy1, 2), at(ix1, iy1, 2), fx), fy);
    return o;
}

// ---- Shaders/RayTracing.hlsl:43-53 + RayTrace.hlsl:444-464 -----------------------------------------
struct Surf {
    F3 pos, n, t, b;
    float u, v;
};
inline float BarycentricLerp(float v0, float v1, float v2, F3 b) { return (v0 * b.x + v1 * b.y) + v2 * b.z; }

Surf GetHitSurface(const Scene& S, uint32_t geometryIdx, uint32_t primIdx, float b1, float b2) {
    const F3 bary = F3{(1 - b1) - b2, b1, b2};
    const oracle_geometry_info& gi = S.geo[geometryIdx];
    const uint32_t i0 = S.idx[primIdx * 3 + gi.IdxOffset + 0];
    const uint32_t i1 = S.idx[primIdx * 3 + gi.IdxOffset + 1];
    const uint32_t i2 = S.idx[primIdx * 3 + gi.IdxOffset + 2];
    const oracle_vertex& v0 = S.vtx[i0 + gi.VtxOffset];
    const oracle_vertex& v1 = S.vtx[i1 + gi.VtxOffset];
    const oracle_vertex& v2 = S.vtx[i2 + gi.VtxOffset];
    auto L3 = [&](const float* a, const float* b, const float* c) {
        return F3{BarycentricLerp(a[0], b[0], c[0], bary), BarycentricLerp(a[1], b[1], c[1], bary),
                  BarycentricLerp(a[2], b[2], c[2], bary)};
    };
    Surf s;
    s.pos = L3(v0.Position, v1.Position, v2.Position);
    s.n = normalize(L3(v0.Normal, v1.Normal, v2.Normal));
    s.u = BarycentricLerp(v0.UV[0], v1.UV[0], v2.UV[0], bary);
    s.v = BarycentricLerp(v0.UV[1], v1.UV[1], v2.UV[1], bary);
    s.t = normalize(L3(v0.Tangent, v1.Tangent, v2.Tangent));
    s.b = normalize(L3(v0.Bitangent, v1.Bitangent, v2.Bitangent));
    return s;
}

// ---- acceleration structure ---------------------------------------------------------------------------
// Moller-Trumbore, two-sided; bit-identical arithmetic to dxrpathtracer_amd/csrc/pt_kernels.hip.
bool intersect_triangle(F3 o, F3 d, F3 v0, F3 e1, F3 e2, float* t, float* u, float* v) {
    F3 pvec = cross(d, e2);
    float det = dot(e1, pvec);
    if (det == 0.0f) return false;
    float inv = 1.0f / det;
    F3 tvec = o - v0;
    float uu = dot(tvec, pvec) * inv;
    if (uu < 0.0f || uu > 1.0f) return false;
    F3 qvec = cross(tvec, e1);
    float vv = dot(d, qvec) * inv;
    if (vv < 0.0f || uu + vv > 1.0f) return false;
    *t = dot(e2, qvec) * inv;
    *u = uu;
    *v = vv;
    return true;
}

void build_bvh(Scene& S) {
    const uint32_t n = uint32_t(S.tgeom.size());
    std::vector<float> lo(size_t(n) * 3), hi(size_t(n) * 3), cen(size_t(n) * 3);
    for (uint32_t t = 0; t < n; ++t) {
        const float* v = &S.tv[size_t(t) * 9];
        for (int k = 0; k < 3; ++k) {
            float a = v[k], b = v[k] + v[3 + k], c = v[k] + v[6 + k];
            lo[3 * t + k] = std::min(a, std::min(b, c));
            hi[3 * t + k] = std::max(a, std::max(b, c));
            cen[3 * t + k] = 0.5f * (lo[3 * t + k] + hi[3 * t + k]);
        }
    }
    S.refs.resize(n);
    for (uint32_t i = 0; i < n; ++i) S.refs[i] = i;
    S.nodes.clear();
    S.nodes.reserve(size_t(n) * 2);
    struct Job { uint32_t node, b, e; };
    std::vector<Job> st;
    S.nodes.push_back(Scene::Node{});
    st.push_back({0, 0, n});
    float ext = 0.f;
    while (!st.empty()) {
        Job j = st.back();
        st.pop_back();
        Scene::Node nd;
        for (int k = 0; k < 3; ++k) { nd.lo[k] = FLT_MAX; nd.hi[k] = -FLT_MAX; }
        float clo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, chi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (uint32_t i = j.b; i < j.e; ++i) {
            uint32_t t = S.refs[i];
            for (int k = 0; k < 3; ++k) {
                nd.lo[k] = std::min(nd.lo[k], lo[3 * t + k]);
                nd.hi[k] = std::max(nd.hi[k], hi[3 * t + k]);
                clo[k] = std::min(clo[k], cen[3 * t + k]);
                chi[k] = std::max(chi[k], cen[3 * t + k]);
            }
        }
        if (j.node == 0) ext = std::max(nd.hi[0] - nd.lo[0], std::max(nd.hi[1] - nd.lo[1], nd.hi[2] - nd.lo[2]));
        // conservative padding so the slab test never rejects a box that holds an accepted hit
        for (int k = 0; k < 3; ++k) {
            float m = std::max(std::fabs(nd.lo[k]), std::fabs(nd.hi[k]));
            float p = m * 1e-5f + ext * 1e-6f + 1e-7f;
            nd.lo[k] -= p;
            nd.hi[k] += p;
        }
        const uint32_t cnt = j.e - j.b;
        uint32_t mid = j.b;
        if (cnt > 4) {
            // 16-bin SAH over the widest centroid axis
            int ax = 0;
            for (int k = 1; k < 3; ++k)
                if (chi[k] - clo[k] > chi[ax] - clo[ax]) ax = k;
            const float w = chi[ax] - clo[ax];
            if (w > 0.f) {
                const int NB = 16;
                uint32_t bc[NB] = {};
                float blo[NB][3], bhi[NB][3];
                for (int b = 0; b < NB; ++b)
                    for (int k = 0; k < 3; ++k) { blo[b][k] = FLT_MAX; bhi[b][k] = -FLT_MAX; }
                auto bin = [&](uint32_t t) { return std::min(NB - 1, std::max(0, int((cen[3 * t + ax] - clo[ax]) / w * NB))); };
                for (uint32_t i = j.b; i < j.e; ++i) {
                    uint32_t t = S.refs[i];
                    int b = bin(t);
                    bc[b]++;
                    for (int k = 0; k < 3; ++k) {
                        blo[b][k] = std::min(blo[b][k], lo[3 * t + k]);
                        bhi[b][k] = std::max(bhi[b][k], hi[3 * t + k]);
                    }
                }
                auto area = [](const float* l, const float* h) {
                    if (l[0] > h[0]) return 0.0;
                    double x = double(h[0]) - l[0], y = double(h[1]) - l[1], z = double(h[2]) - l[2];
                    return x * y + y * z + z * x;
                };
                double best = 1e300;
                int bestb = -1;
                for (int s = 1; s < NB; ++s) {
                    float l0[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, h0[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
                    float l1[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, h1[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
                    uint32_t c0 = 0, c1 = 0;
                    for (int b = 0; b < NB; ++b) {
                        float* L = b < s ? l0 : l1;
                        float* H = b < s ? h0 : h1;
                        (b < s ? c0 : c1) += bc[b];
                        for (int k = 0; k < 3; ++k) { L[k] = std::min(L[k], blo[b][k]); H[k] = std::max(H[k], bhi[b][k]); }
                    }
                    if (!c0 || !c1) continue;
                    double c = area(l0, h0) * c0 + area(l1, h1) * c1;
                    if (c < best) { best = c; bestb = s; }
                }
                if (bestb > 0)
                    mid = uint32_t(std::partition(S.refs.begin() + j.b, S.refs.begin() + j.e,
                                                  [&](uint32_t t) { return bin(t) < bestb; }) - S.refs.begin());
            }
            if (mid == j.b || mid == j.e) {
                mid = j.b + cnt / 2;
                std::nth_element(S.refs.begin() + j.b, S.refs.begin() + mid, S.refs.begin() + j.e, [&](uint32_t x, uint32_t y) {
                    return cen[3 * x + ax] < cen[3 * y + ax] || (cen[3 * x + ax] == cen[3 * y + ax] && x < y);
                });
            }
        }
        if (cnt <= 4) {
            nd.left = j.b;
            nd.count = cnt;
            S.nodes[j.node] = nd;
        } else {
            nd.left = uint32_t(S.nodes.size());
            nd.count = 0;
            S.nodes[j.node] = nd;
            S.nodes.push_back(Scene::Node{});
            S.nodes.push_back(Scene::Node{});
            st.push_back({nd.left + 1, mid, j.e});
            st.push_back({nd.left, j.b, mid});
        }
    }
}

struct Stats {
    uint64_t radiance_rays = 0, shadow_rays = 0, node_visits = 0, tri_tests = 0;
};

struct Hit {
    float t, b1, b2;
    uint32_t tri;
};

bool AlphaAccepts(const Scene& S, uint32_t geom, uint32_t gtri, float b1, float b2);

// TraceRay: closest hit (smallest t, ties -> smallest global tri) or, for shadow rays
// (ACCEPT_FIRST_HIT_AND_END_SEARCH), any accepted hit.  alpha = !RAY_FLAG_FORCE_OPAQUE.
bool TraceRay(const Scene& S, F3 o, F3 d, float tmin, float tmax, bool anyHit, bool alpha, Hit& h, Stats& st) {
    h.t = tmax;
    h.tri = kNone;
    h.b1 = h.b2 = 0.0f;
    F3 inv = F3{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    uint32_t stack[128];
    int sp = 0;
    stack[sp++] = 0;
    while (sp > 0) {
        const Scene::Node& n = S.nodes[stack[--sp]];
        st.node_visits++;
        float t0 = tmin, t1 = h.t;
        bool miss = false;
        const float oo[3] = {o.x, o.y, o.z}, ii[3] = {inv.x, inv.y, inv.z};
        for (int k = 0; k < 3 && !miss; ++k) {
            float a = (n.lo[k] - oo[k]) * ii[k], b = (n.hi[k] - oo[k]) * ii[k];
            if (std::isnan(a) || std::isnan(b)) continue;  // d == 0 and o on the slab plane: treat as inside
            if (a > b) std::swap(a, b);
            t0 = std::max(t0, a);
            t1 = std::min(t1, b);
            if (t0 > t1) miss = true;
        }
        if (miss) continue;
        if (n.count == 0) {
            stack[sp++] = n.left + 1;
            stack[sp++] = n.left;
            continue;
        }
        for (uint32_t k = 0; k < n.count; ++k) {
            const uint32_t gtri = S.refs[n.left + k];
            const float* v = &S.tv[size_t(gtri) * 9];
            st.tri_tests++;
            float t, u, w;
            if (!intersect_triangle(o, d, F3{v[0], v[1], v[2]}, F3{v[3], v[4], v[5]}, F3{v[6], v[7], v[8]}, &t, &u, &w)) continue;
            if (!(t >= tmin)) continue;
            if (anyHit) {
                if (!(t <= tmax)) continue;
            } else if (!(t < h.t || (t == h.t && gtri < h.tri))) {
                continue;
            }
            const uint32_t geom = S.tgeom[gtri];
            if (alpha && !S.topaque[gtri] && !AlphaAccepts(S, geom, gtri, u, w)) continue;
            h.t = t;
            h.tri = gtri;
            h.b1 = u;
            h.b2 = w;
            if (anyHit) return true;
        }
    }
    return h.tri != kNone;
}

// AnyHitShader / ShadowAnyHitShader, RayTrace.hlsl:485-507
bool AlphaAccepts(const Scene& S, uint32_t geom, uint32_t gtri, float b1, float b2) {
    const oracle_geometry_info& gi = S.geo[geom];
    const oracle_material& m = S.mat[gi.MaterialIdx];
    if (m.Opacity == kNone) return true;
    const uint32_t primIdx = gtri - gi.IdxOffset / 3;
    const Surf s = GetHitSurface(S, geom, primIdx, b1, b2);
    return !(SampleTex(S, m.Opacity, s.u, s.v).r < 0.35f);
}

// ---- the path tracer (RayTrace.hlsl) ------------------------------------------------------------------
struct Ctx {
    const Scene& S;
    const oracle_ray_trace_constants& rtc;
    const oracle_app_settings& set;
    const oracle_spot_light* lights;
    uint32_t numLights;
    Stats& st;
};

struct PrimaryPayload {  // RayTrace.hlsl:63-71
    F3 Radiance;
    float Roughness;
    uint32_t PathLength;
    uint32_t PixelIdx;
    uint32_t SampleSetIdx;
    bool IsDiffuse;
};

void SamplePoint(const Ctx& C, uint32_t pixelIdx, uint32_t& setIdx, float out[2]) {  // 85-90
    const uint32_t permutation = setIdx * C.rtc.TotalNumPixels + pixelIdx;
    setIdx += 1;
    SampleCMJ2D(C.rtc.CurrSampleIdx, uint32_t(C.set.SqrtNumSamples), uint32_t(C.set.SqrtNumSamples), permutation, out);
}

float TraceShadow(const Ctx& C, F3 o, F3 d, float tmin, float tmax, bool forceOpaque) {
    Hit h;
    C.st.shadow_rays++;
    return TraceRay(C.S, o, d, tmin, tmax, true, !forceOpaque, h, C.st) ? 0.0f : 1.0f;  // ShadowHit/Miss 532-542
}

void TraceRadiance(const Ctx& C, F3 o, F3 d, float tmin, float tmax, bool forceOpaque, PrimaryPayload& payload);

F3 PathTrace(const Ctx& C, const Surf& hitSurface, const oracle_material& material, PrimaryPayload inPayload, F3 incomingRayOriginWS,
             F3 incomingRayDirWS) {
    const oracle_app_settings& A = C.set;
    const oracle_ray_trace_constants& R = C.rtc;
    const Scene& S = C.S;
    if ((!A.EnableDiffuse && !A.EnableSpecular) || (!A.EnableDirect && !A.EnableIndirect)) return F3{0, 0, 0};
    if (inPayload.PathLength > 1 && !A.EnableIndirect) return F3{0, 0, 0};
    // float3x3 tangentToWorld = float3x3(T, B, N): rows
    F3 row0 = hitSurface.t, row1 = hitSurface.b, row2 = hitSurface.n;
    const F3 positionWS = hitSurface.pos;
    F3 normalWS = hitSurface.n;
    if (A.EnableNormalMaps) {
        T4 nm = SampleTex(S, material.Normal, hitSurface.u, hitSurface.v);
        F3 normalTS;
        normalTS.x = nm.r * 2.0f - 1.0f;
        normalTS.y = nm.g * 2.0f - 1.0f;
        normalTS.z = std::sqrt(1.0f - saturate(normalTS.x * normalTS.x + normalTS.y * normalTS.y));
        normalWS = normalize((row0 * normalTS.x + row1 * normalTS.y) + row2 * normalTS.z);  // mul(normalTS, tangentToWorld)
        row2 = normalWS;
    }
    F3 baseColor = F3{1.0f, 1.0f, 1.0f};
    if (A.EnableAlbedoMaps && !A.EnableWhiteFurnaceMode) {
        T4 a = SampleTex(S, material.Albedo, hitSurface.u, hitSurface.v);
        baseColor = F3{a.r, a.g, a.b};
    }
    const float metallic = saturate((A.EnableWhiteFurnaceMode ? 1.0f : SampleTex(S, material.Metallic, hitSurface.u, hitSurface.v).r) * A.MetallicScale);
    const bool enableDiffuse = (A.EnableDiffuse && metallic < 1.0f) || A.EnableWhiteFurnaceMode;
    const bool enableSpecular = (A.EnableSpecular && (A.EnableIndirectSpecular ? !(A.AvoidCausticPaths && inPayload.IsDiffuse) : (inPayload.PathLength == 1)));
    if (enableDiffuse == false && enableSpecular == false) return F3{0, 0, 0};
    const float sqrtRoughness = saturate((A.EnableWhiteFurnaceMode ? 1.0f : SampleTex(S, material.Roughness, hitSurface.u, hitSurface.v).r) * A.RoughnessScale);
    const F3 diffuseAlbedo = F3{lerp(baseColor.x, 0.0f, metallic), lerp(baseColor.y, 0.0f, metallic), lerp(baseColor.z, 0.0f, metallic)} * (enableDiffuse ? 1.0f : 0.0f);
    const F3 specularAlbedo = F3{lerp(0.03f, baseColor.x, metallic), lerp(0.03f, baseColor.y, metallic), lerp(0.03f, baseColor.z, metallic)} * (enableSpecular ? 1.0f : 0.0f);
    float roughness = sqrtRoughness * sqrtRoughness;
    if (A.ClampRoughness) roughness = std::fmax(roughness, inPayload.Roughness);
    F3 msEnergyCompensation = F3{1.0f, 1.0f, 1.0f};
    if (A.ApplyMultiscatteringEnergyCompensation) {
        float Ess = GGXEnvironmentBRDFScale(saturate(dot(normalWS, -incomingRayDirWS)), sqrtRoughness);
        float k = 1.0f / Ess - 1.0f;
        msEnergyCompensation = F3{1.0f + specularAlbedo.x * k, 1.0f + specularAlbedo.y * k, 1.0f + specularAlbedo.z * k};
    }
    F3 radiance = F3{0, 0, 0};
    if (!A.EnableWhiteFurnaceMode) {
        T4 e = SampleTex(S, material.Emissive, hitSurface.u, hitSurface.v);
        radiance = F3{e.r, e.g, e.b};
    }
    // Sun, 224-262
    if (A.EnableSun && !A.EnableWhiteFurnaceMode) {
        const F3 D = F3{R.SunDirectionWS[0], R.SunDirectionWS[1], R.SunDirectionWS[2]};
        F3 sunDirection = D;
        if (A.SunAreaLightApproximation) {
            F3 Rr = reflect(incomingRayDirWS, normalWS);
            float r = R.SinSunAngularRadius;
            float d = R.CosSunAngularRadius;
            float DDotR = dot(D, Rr);
            F3 Sv = Rr - D * DDotR;
            sunDirection = DDotR < d ? normalize(D * d + normalize(Sv) * r) : Rr;
        }
        const float vis = TraceShadow(C, positionWS, D, kRayTMin, kFP32Max, inPayload.PathLength > uint32_t(A.MaxAnyHitPathLength));
        radiance = radiance + CalcLighting(normalWS, sunDirection, F3{R.SunIrradiance[0], R.SunIrradiance[1], R.SunIrradiance[2]},
                                           diffuseAlbedo, specularAlbedo, roughness, positionWS, incomingRayOriginWS, msEnergyCompensation) * vis;
    }
    // Spot lights, 265-313
    if (A.RenderLights) {
        for (uint32_t li = 0; li < C.numLights; ++li) {
            const oracle_spot_light& sl = C.lights[li];
            F3 surfaceToLight = F3{sl.Position[0], sl.Position[1], sl.Position[2]} - positionWS;
            float distanceToLight = length(surfaceToLight);
            surfaceToLight = F3{surfaceToLight.x / distanceToLight, surfaceToLight.y / distanceToLight, surfaceToLight.z / distanceToLight};
            float angleFactor = saturate(dot(surfaceToLight, F3{sl.Direction[0], sl.Direction[1], sl.Direction[2]}));
            float angularAttenuation = smoothstep(sl.AngularAttenuationY, sl.AngularAttenuationX, angleFactor);
            float d = distanceToLight / sl.Range;
            float falloff = saturate(1.0f - (d * d * d * d));
            falloff = (falloff * falloff) / (distanceToLight * distanceToLight + 1.0f);
            angularAttenuation *= falloff;
            if (angularAttenuation > 0.0f) {
                const float vis = TraceShadow(C, positionWS + normalWS * 0.01f, surfaceToLight, kSpotShadowNearClip,
                                              distanceToLight - kSpotShadowNearClip, inPayload.PathLength > uint32_t(A.MaxAnyHitPathLength));
                F3 intensity = F3{sl.Intensity[0], sl.Intensity[1], sl.Intensity[2]} * angularAttenuation;
                radiance = radiance + CalcLighting(normalWS, surfaceToLight, intensity, diffuseAlbedo, specularAlbedo, roughness,
                                                   positionWS, incomingRayOriginWS, msEnergyCompensation) * vis;
            }
        }
    }
    // BRDF sampling, 315-376
    float brdfSample[2];
    SamplePoint(C, inPayload.PixelIdx, inPayload.SampleSetIdx, brdfSample);
    F3 throughput = F3{0, 0, 0};
    F3 rayDirTS = F3{0, 0, 0};
    float selector = brdfSample[0];
    if (enableSpecular == false)
        selector = 0.0f;
    else if (enableDiffuse == false)
        selector = 1.0f;
    if (selector < 0.5f) {
        if (enableSpecular) brdfSample[0] *= 2.0f;
        rayDirTS = SampleDirectionCosineHemisphere(brdfSample[0], brdfSample[1]);
        throughput = diffuseAlbedo;
    } else {
        if (enableDiffuse) brdfSample[0] = (brdfSample[0] - 0.5f) * 2.0f;
        // mul(incomingRayDirWS, transpose(tangentToWorld)) = (dot(d,row0), dot(d,row1), dot(d,row2))
        F3 incomingRayDirTS = normalize(F3{dot(incomingRayDirWS, row0), dot(incomingRayDirWS, row1), dot(incomingRayDirWS, row2)});
        F3 microfacetNormalTS = SampleGGXVisibleNormal(-incomingRayDirTS, roughness, roughness, brdfSample[0], brdfSample[1]);
        F3 sampleDirTS = reflect(incomingRayDirTS, microfacetNormalTS);
        F3 normalTS = F3{0.0f, 0.0f, 1.0f};
        F3 F = A.EnableWhiteFurnaceMode ? F3{1, 1, 1} : Fresnel(specularAlbedo, microfacetNormalTS, sampleDirTS);
        float G1 = SmithGGXMasking(normalTS, sampleDirTS, -incomingRayDirTS, roughness * roughness);
        float G2 = SmithGGXMaskingShadowing(normalTS, sampleDirTS, -incomingRayDirTS, roughness * roughness);
        throughput = F * (G2 / G1);
        rayDirTS = sampleDirTS;
        if (A.ApplyMultiscatteringEnergyCompensation) {
            float Ess = GGXEnvironmentBRDFScale(saturate(dot(normalTS, -incomingRayDirWS)), sqrtRoughness);  // 361: space-mixing quirk
            float k = 1.0f / Ess - 1.0f;
            throughput = throughput * F3{1.0f + specularAlbedo.x * k, 1.0f + specularAlbedo.y * k, 1.0f + specularAlbedo.z * k};
        }
    }
    const F3 rayDirWS = normalize((row0 * rayDirTS.x + row1 * rayDirTS.y) + row2 * rayDirTS.z);  // mul(rayDirTS, tangentToWorld)
    if (enableDiffuse && enableSpecular) throughput = throughput * 2.0f;
    if (inPayload.PathLength == 1 && !A.EnableDirect) radiance = F3{0, 0, 0};
    if (A.EnableIndirect && (int(inPayload.PathLength) + 1 < A.MaxPathLength) && !A.EnableWhiteFurnaceMode) {
        PrimaryPayload payload;
        payload.Radiance = F3{0, 0, 0};
        payload.PathLength = inPayload.PathLength + 1;
        payload.PixelIdx = inPayload.PixelIdx;
        payload.SampleSetIdx = inPayload.SampleSetIdx;
        payload.IsDiffuse = (selector < 0.5f);
        payload.Roughness = roughness;
        TraceRadiance(C, positionWS, rayDirWS, kRayTMin, kFP32Max, payload.PathLength > uint32_t(A.MaxAnyHitPathLength), payload);
        radiance = radiance + payload.Radiance * throughput;
    } else {
        const float vis = TraceShadow(C, positionWS, rayDirWS, kRayTMin, kFP32Max, inPayload.PathLength + 1 > uint32_t(A.MaxAnyHitPathLength));
        if (A.EnableWhiteFurnaceMode) {
            radiance = throughput;
        } else {
            F3 skyRadiance = A.EnableSky ? SampleSky(S, rayDirWS) : F3{0, 0, 0};
            radiance = radiance + (skyRadiance * vis) * throughput;
        }
    }
    return radiance;
}

// TraceRay(radiance) -> ClosestHitShader (476-483) or MissShader (509-530)
void TraceRadiance(const Ctx& C, F3 o, F3 d, float tmin, float tmax, bool forceOpaque, PrimaryPayload& payload) {
    Hit h;
    C.st.radiance_rays++;
    if (TraceRay(C.S, o, d, tmin, tmax, false, !forceOpaque, h, C.st)) {
        const uint32_t geom = C.S.tgeom[h.tri];
        const oracle_geometry_info& gi = C.S.geo[geom];
        const Surf s = GetHitSurface(C.S, geom, h.tri - gi.IdxOffset / 3, h.b1, h.b2);
        payload.Radiance = PathTrace(C, s, C.S.mat[gi.MaterialIdx], payload, o, d);
    } else {
        const oracle_app_settings& A = C.set;
        if (A.EnableWhiteFurnaceMode) {
            payload.Radiance = F3{1, 1, 1};
        } else {
            payload.Radiance = A.EnableSky ? SampleSky(C.S, d) : F3{0, 0, 0};
            if (payload.PathLength == 1) {
                float cosSunAngle = dot(d, F3{C.rtc.SunDirectionWS[0], C.rtc.SunDirectionWS[1], C.rtc.SunDirectionWS[2]});
                if (cosSunAngle >= C.rtc.CosSunAngularRadius)
                    payload.Radiance = F3{C.rtc.SunRenderColor[0], C.rtc.SunRenderColor[1], C.rtc.SunRenderColor[2]};
            }
        }
    }
}

// The primary-only AOV of pixel (x, y) (SURVEY.md 8(d), C1 plumbing): RaygenShader's ray (92-126), its
// closest hit, and the hit surface's albedo tap as PathTrace takes it (RayTrace.hlsl:180-183: the
// albedo map when EnableAlbedoMaps and not furnace, else 1); out = (albedo rgb, 1) on a hit, 0 on a miss.
void PrimaryAov(const Ctx& C, uint32_t x, uint32_t y, uint32_t W, uint32_t H, float out[4]) {
    const uint32_t pixelIdx = y * W + x;
    uint32_t sampleSetIdx = 0;
    float s[2];
    SamplePoint(C, pixelIdx, sampleSetIdx, s);
    float rx = float(x) + s[0], ry = float(y) + s[1];
    float ncx = rx / (float(W) * 0.5f) - 1.0f, ncy = ry / (float(H) * 0.5f) - 1.0f;
    ncy *= -1.0f;
    const float* M = C.rtc.InvViewProjection;
    float a[4], b[4];
    for (int j = 0; j < 4; ++j) {
        a[j] = ((ncx * M[0 * 4 + j] + ncy * M[1 * 4 + j]) + 0.0f * M[2 * 4 + j]) + 1.0f * M[3 * 4 + j];
        b[j] = ((ncx * M[0 * 4 + j] + ncy * M[1 * 4 + j]) + 1.0f * M[2 * 4 + j]) + 1.0f * M[3 * 4 + j];
    }
    F3 start = F3{a[0] / a[3], a[1] / a[3], a[2] / a[3]};
    F3 end = F3{b[0] / b[3], b[1] / b[3], b[2] / b[3]};
    F3 rayDir = normalize(end - start);
    float rayLength = length(end - start);
    Hit h;
    C.st.radiance_rays++;
    out[0] = out[1] = out[2] = out[3] = 0.0f;
    if (TraceRay(C.S, start, rayDir, 0.0f, rayLength, false, !(1u > uint32_t(C.set.MaxAnyHitPathLength)), h, C.st)) {
        const uint32_t geom = C.S.tgeom[h.tri];
        const oracle_geometry_info& gi = C.S.geo[geom];
        const Surf sf = GetHitSurface(C.S, geom, h.tri - gi.IdxOffset / 3, h.b1, h.b2);
        F3 base = F3{1.0f, 1.0f, 1.0f};
        if (C.set.EnableAlbedoMaps && !C.set.EnableWhiteFurnaceMode) {
            T4 t = SampleTex(C.S, C.S.mat[gi.MaterialIdx].Albedo, sf.u, sf.v);
            base = F3{t.r, t.g, t.b};
        }
        out[0] = base.x;
        out[1] = base.y;
        out[2] = base.z;
        out[3] = 1.0f;
    }
}

// RaygenShader, 92-149: returns the clamped radiance of pixel (x, y)
F3 Raygen(const Ctx& C, uint32_t x, uint32_t y, uint32_t W, uint32_t H) {
    const uint32_t pixelIdx = y * W + x;
    uint32_t sampleSetIdx = 0;
    float s[2];
    SamplePoint(C, pixelIdx, sampleSetIdx, s);
    float rx = float(x) + s[0], ry = float(y) + s[1];
    float ncx = rx / (float(W) * 0.5f) - 1.0f, ncy = ry / (float(H) * 0.5f) - 1.0f;
    ncy *= -1.0f;
    const float* M = C.rtc.InvViewProjection;
    float a[4], b[4];
    for (int j = 0; j < 4; ++j) {
        a[j] = ((ncx * M[0 * 4 + j] + ncy * M[1 * 4 + j]) + 0.0f * M[2 * 4 + j]) + 1.0f * M[3 * 4 + j];
        b[j] = ((ncx * M[0 * 4 + j] + ncy * M[1 * 4 + j]) + 1.0f * M[2 * 4 + j]) + 1.0f * M[3 * 4 + j];
    }
    F3 start = F3{a[0] / a[3], a[1] / a[3], a[2] / a[3]};
    F3 end = F3{b[0] / b[3], b[1] / b[3], b[2] / b[3]};
    F3 rayDir = normalize(end - start);
    float rayLength = length(end - start);
    PrimaryPayload payload;
    payload.Radiance = F3{0, 0, 0};
    payload.Roughness = 0.0f;
    payload.PathLength = 1;
    payload.PixelIdx = pixelIdx;
    payload.SampleSetIdx = sampleSetIdx;
    payload.IsDiffuse = false;
    TraceRadiance(C, start, rayDir, 0.0f, rayLength, payload.PathLength > uint32_t(C.set.MaxAnyHitPathLength), payload);
    return F3{std::fmin(std::fmax(payload.Radiance.x, 0.0f), kFP16Max), std::fmin(std::fmax(payload.Radiance.y, 0.0f), kFP16Max),
              std::fmin(std::fmax(payload.Radiance.z, 0.0f), kFP16Max)};
}

// BakeRayGen, DXRPathTracer/Baking.hlsl:336-465 (its PathTrace/miss/hit shaders, Baking.hlsl:96-330,
// are RayTrace.hlsl's; the shared PathTrace/TraceRadiance above serve both).  Updates texel i of
// accum/lightmap (float4 each); a texel outside every UV island (pos.w == 0) is left untouched.
inline float Luminance(F3 c) { return dot(c, F3{0.299f, 0.587f, 0.114f}); }

void BakeTexel(const Ctx& C, uint32_t i, const float* pos, const float* nrm, float* accum, float* lightmap) {
    const float* P4 = pos + size_t(i) * 4;
    float* out = lightmap + size_t(i) * 4;
    if (P4[3] == 0.0f) return;  // 351-354
    const F3 worldPos = F3{P4[0], P4[1], P4[2]};
    auto put = [&](float r, float g, float b) { out[0] = r; out[1] = g; out[2] = b; out[3] = 1.0f; };
    if (std::isinf(worldPos.x) || std::isinf(worldPos.y) || std::isinf(worldPos.z)) return put(0, 0, 1);  // 357-361
    const F3 worldNormalVec = F3{nrm[size_t(i) * 4], nrm[size_t(i) * 4 + 1], nrm[size_t(i) * 4 + 2]};
    if (dot(worldNormalVec, worldNormalVec) < 0.0001f) return put(0, 0, 0);  // 363-369
    const F3 worldNormal = normalize(worldNormalVec);
    uint32_t sampleSetIdx = 0;
    // 376-379: tangentToWorld rows (tangent, bitangent, normal)
    const F3 up = std::fabs(worldNormal.z) < 0.999f ? F3{0, 0, 1} : F3{1, 0, 0};
    const F3 tangent = normalize(cross(up, worldNormal));
    const F3 bitangent = cross(worldNormal, tangent);
    float hs[2];
    SamplePoint(C, i, sampleSetIdx, hs);  // 382 (pixelIdx = y * W + x = i)
    const F3 rayDirTS = SampleDirectionCosineHemisphere(hs[0], hs[1]);
    const F3 rayDir = (tangent * rayDirTS.x + bitangent * rayDirTS.y) + worldNormal * rayDirTS.z;  // 386
    const F3 origin = worldPos + rayDir * 0.00001f;                                                    // 390
    auto bad = [](F3 v) {
        return std::isinf(v.x) || std::isinf(v.y) || std::isinf(v.z) || std::isnan(v.x) || std::isnan(v.y) || std::isnan(v.z);
    };
    if (bad(origin) || bad(rayDir) || length(rayDir) < 0.001f) return put(1, 0, 1);  // 395-396, 415-419
    PrimaryPayload payload;
    payload.Radiance = F3{0, 0, 0};
    payload.Roughness = 0.0f;
    payload.PathLength = 1;
    payload.PixelIdx = i;
    payload.SampleSetIdx = sampleSetIdx;
    payload.IsDiffuse = true;
    TraceRadiance(C, origin, rayDir, 0.0001f, kFP32Max, payload.PathLength > uint32_t(C.set.MaxAnyHitPathLength), payload);
    F3 newSampleColor = payload.Radiance;
    float* acc = accum + size_t(i) * 4;
    F3 colorSum = F3{acc[0], acc[1], acc[2]};
    float validSampleCount = acc[3];
    if (validSampleCount >= 1.0f) {  // 431-447: firefly clamp at 10x the running average's luminance
        const F3 averageColor = F3{colorSum.x / validSampleCount, colorSum.y / validSampleCount, colorSum.z / validSampleCount};
        const float averageLuminance = Luminance(averageColor) + 0.001f;
        const float sampleLuminance = Luminance(newSampleColor);
        if (sampleLuminance > averageLuminance * 10.0f) newSampleColor = newSampleColor * (averageLuminance * 10.0f / sampleLuminance);
    }
    const bool isNan = std::isnan(newSampleColor.x) || std::isnan(newSampleColor.y) || std::isnan(newSampleColor.z);
    const bool isTooDark = Luminance(newSampleColor) < 0.0001f;
    if (!isNan && !isTooDark) {  // 454-458
        colorSum = colorSum + newSampleColor;
        validSampleCount += 1.0f;
    }
    acc[0] = colorSum.x; acc[1] = colorSum.y; acc[2] = colorSum.z; acc[3] = validSampleCount;
    F3 averageColor = F3{0, 0, 0};
    if (validSampleCount > 0.0f)
        averageColor = F3{colorSum.x / validSampleCount, colorSum.y / validSampleCount, colorSum.z / validSampleCount};
    put(averageColor.x, averageColor.y, averageColor.z);  // 465
}

struct OracleScene {
    Scene S;
    double build_ms = 0;
};

}  // namespace

extern "C" {

void oracle_cmj2d(uint32_t sample_idx, uint32_t nx, uint32_t ny, uint32_t pattern, float out[2]) {
    SampleCMJ2D(sample_idx, nx, ny, pattern, out);
}

void oracle_sincos(float x, float out[2]) { sincos_det(x, &out[0], &out[1]); }

// Batched evaluations of the sampling / BRDF helpers for the reference-compiled golden vectors
// (tests/golden/make_sampling_golden.py): n inputs each.
void oracle_concentric_disk(const float* xy, uint32_t n, float* out) {
    for (uint32_t i = 0; i < n; ++i) SquareToConcentricDiskMapping(xy[2 * i], xy[2 * i + 1], out + 2 * i);
}
void oracle_cosine_hemisphere(const float* uv, uint32_t n, float* out) {
    for (uint32_t i = 0; i < n; ++i) {
        const F3 d = SampleDirectionCosineHemisphere(uv[2 * i], uv[2 * i + 1]);
        out[3 * i] = d.x;
        out[3 * i + 1] = d.y;
        out[3 * i + 2] = d.z;
    }
}
void oracle_ggx_v1(const float* m2_ndotx, uint32_t n, float* out) {
    for (uint32_t i = 0; i < n; ++i) out[i] = GGXV1(m2_ndotx[2 * i], m2_ndotx[2 * i + 1]);
}
// in: n x (specAlbedo xyz, h xyz, l xyz); out: n x rgb
void oracle_fresnel(const float* in, uint32_t n, float* out) {
    for (uint32_t i = 0; i < n; ++i) {
        const float* a = in + 9 * i;
        const F3 f = Fresnel(F3{a[0], a[1], a[2]}, F3{a[3], a[4], a[5]}, F3{a[6], a[7], a[8]});
        out[3 * i] = f.x;
        out[3 * i + 1] = f.y;
        out[3 * i + 2] = f.z;
    }
}
// in: n x (m, n xyz, h xyz, v xyz, l xyz); out: n
void oracle_ggx_specular(const float* in, uint32_t n, float* out) {
    for (uint32_t i = 0; i < n; ++i) {
        const float* a = in + 13 * i;
        out[i] = GGXSpecular(a[0], F3{a[1], a[2], a[3]}, F3{a[4], a[5], a[6]}, F3{a[7], a[8], a[9]}, F3{a[10], a[11], a[12]});
    }
}

oracle_scene* oracle_scene_create(const oracle_vertex* vertices, uint32_t num_vertices, const void* indices, uint32_t idx_bytes,
                                  uint32_t num_indices, const oracle_geometry_info* geometries, uint32_t num_geometries,
                                  const oracle_material* materials, uint32_t num_materials, const oracle_texture* textures,
                                  uint32_t num_textures, const uint16_t* sky_cube, uint32_t sky_res) {
    auto t0 = std::chrono::steady_clock::now();
    std::unique_ptr<OracleScene> O(new OracleScene());
    Scene& S = O->S;
    S.vtx = vertices;
    S.idx.resize(num_indices);
    for (uint32_t i = 0; i < num_indices; ++i)
        S.idx[i] = idx_bytes == 2 ? static_cast<const uint16_t*>(indices)[i] : static_cast<const uint32_t*>(indices)[i];
    S.geo = geometries;
    S.ngeo = num_geometries;
    S.mat = materials;
    S.nmat = num_materials;
    for (uint32_t i = 0; i < num_textures; ++i)
        S.tex.push_back(Tex{textures[i].width, textures[i].height, textures[i].fmt, static_cast<const uint8_t*>(textures[i].texels)});
    S.sky = sky_cube;
    S.sky_res = sky_res;
    for (int i = 0; i < 256; ++i) {
        S.lut_unorm[i] = float(i) / 255.0f;
        double c = double(i) / 255.0;
        S.lut_srgb[i] = float(c <= 0.04045 ? c / 12.92 : std::pow((c + 0.055) / 1.055, 2.4));
    }
    const uint32_t ntri = num_indices / 3;
    S.tv.resize(size_t(ntri) * 9);
    S.tgeom.assign(ntri, 0);
    S.topaque.assign(ntri, 1);
    for (uint32_t g = 0; g < num_geometries; ++g) {
        const uint32_t b = geometries[g].IdxOffset / 3;
        const uint32_t e = g + 1 < num_geometries ? geometries[g + 1].IdxOffset / 3 : ntri;
        const bool opaque = materials[geometries[g].MaterialIdx].Opacity == kNone;
        for (uint32_t t = b; t < e; ++t) {
            S.tgeom[t] = g;
            S.topaque[t] = opaque ? 1 : 0;
            const float* p[3];
            for (int k = 0; k < 3; ++k) p[k] = vertices[S.idx[size_t(t) * 3 + k] + geometries[g].VtxOffset].Position;
            float* o = &S.tv[size_t(t) * 9];
            for (int k = 0; k < 3; ++k) {
                o[k] = p[0][k];
                o[3 + k] = p[1][k] - p[0][k];
                o[6 + k] = p[2][k] - p[0][k];
            }
        }
    }
    build_bvh(S);
    O->build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return reinterpret_cast<oracle_scene*>(O.release());
}

void oracle_scene_destroy(oracle_scene* s) { delete reinterpret_cast<OracleScene*>(s); }

double oracle_scene_build_ms(const oracle_scene* s) { return reinterpret_cast<const OracleScene*>(s)->build_ms; }

int oracle_render(const oracle_scene* scene, const oracle_ray_trace_constants* rtc, const oracle_app_settings* settings,
                  const oracle_spot_light* lights, uint32_t width, uint32_t height, uint32_t x0, uint32_t y0, uint32_t w,
                  uint32_t h, float* accum, uint32_t threads, oracle_stats* out_stats) {
    const Scene& S = reinterpret_cast<const OracleScene*>(scene)->S;
    if (x0 + w > width || y0 + h > height) return -1;
    if (threads == 0) threads = std::max(1u, std::thread::hardware_concurrency());
    const uint32_t nl = (settings->RenderLights && lights) ? std::min(rtc->NumLights, 32u) : 0u;
    std::atomic<uint32_t> next_row{0};
    std::vector<Stats> stats(threads);
    auto worker = [&](uint32_t tid) {
        Ctx C{S, *rtc, *settings, lights, nl, stats[tid]};
        for (;;) {
            uint32_t r = next_row.fetch_add(1);
            if (r >= h) break;
            for (uint32_t c = 0; c < w; ++c) {
                F3 rad = Raygen(C, x0 + c, y0 + r, width, height);
                // RayTrace.hlsl:143-148
                const float lerpFactor = float(rtc->CurrSampleIdx) / (float(rtc->CurrSampleIdx) + 1.0f);
                float* px = accum + (size_t(r) * w + c) * 4;
                px[0] = lerp(rad.x, px[0], lerpFactor);
                px[1] = lerp(rad.y, px[1], lerpFactor);
                px[2] = lerp(rad.z, px[2], lerpFactor);
                px[3] = 1.0f;
            }
        }
    };
    std::vector<std::thread> pool;
    for (uint32_t t = 1; t < threads; ++t) pool.emplace_back(worker, t);
    worker(0);
    for (auto& t : pool) t.join();
    if (out_stats) {
        std::memset(out_stats, 0, sizeof(*out_stats));
        for (const Stats& s : stats) {
            out_stats->radiance_rays += s.radiance_rays;
            out_stats->shadow_rays += s.shadow_rays;
            out_stats->node_visits += s.node_visits;
            out_stats->tri_tests += s.tri_tests;
        }
    }
    return 0;
}

int oracle_render_aov(const oracle_scene* scene, const oracle_ray_trace_constants* rtc, const oracle_app_settings* settings,
                      uint32_t width, uint32_t height, uint32_t x0, uint32_t y0, uint32_t w, uint32_t h, float* out) {
    const Scene& S = reinterpret_cast<const OracleScene*>(scene)->S;
    if (x0 + w > width || y0 + h > height) return -1;
    Stats st;
    Ctx C{S, *rtc, *settings, nullptr, 0u, st};
    for (uint32_t r = 0; r < h; ++r)
        for (uint32_t c = 0; c < w; ++c) PrimaryAov(C, x0 + c, y0 + r, width, height, out + (size_t(r) * w + c) * 4);
    return 0;
}

int oracle_bake(const oracle_scene* scene, const oracle_ray_trace_constants* rtc, const oracle_app_settings* settings,
                const oracle_spot_light* lights, const float* pos, const float* nrm, uint32_t width, uint32_t height,
                uint32_t first, uint32_t count, float* accum, float* lightmap, uint32_t threads, oracle_stats* out_stats) {
    const Scene& S = reinterpret_cast<const OracleScene*>(scene)->S;
    if (uint64_t(first) + count > uint64_t(width) * height) return -1;
    if (threads == 0) threads = std::max(1u, std::thread::hardware_concurrency());
    const uint32_t nl = (settings->RenderLights && lights) ? std::min(rtc->NumLights, 32u) : 0u;
    std::atomic<uint32_t> next{0};
    std::vector<Stats> stats(threads);
    auto worker = [&](uint32_t tid) {
        Ctx C{S, *rtc, *settings, lights, nl, stats[tid]};
        for (;;) {
            const uint32_t b = next.fetch_add(256);
            if (b >= count) break;
            for (uint32_t k = b; k < std::min(count, b + 256u); ++k) BakeTexel(C, first + k, pos, nrm, accum, lightmap);
        }
    };
    std::vector<std::thread> pool;
    for (uint32_t t = 1; t < threads; ++t) pool.emplace_back(worker, t);
    worker(0);
    for (auto& t : pool) t.join();
    if (out_stats) {
        std::memset(out_stats, 0, sizeof(*out_stats));
        for (const Stats& st : stats) {
            out_stats->radiance_rays += st.radiance_rays;
            out_stats->shadow_rays += st.shadow_rays;
            out_stats->node_visits += st.node_visits;
            out_stats->tri_tests += st.tri_tests;
        }
    }
    return 0;
}

// DenoiseCS, DXRPathTracer/DenoiseMedian.hlsl:52-102 with FilterRadius 1 (DXRPathTracer.cpp:2106).
void oracle_median3x3(const float* in, float* out, uint32_t width, uint32_t height) {
    for (uint32_t y = 0; y < height; ++y)
        for (uint32_t x = 0; x < width; ++x) {
            F3 nb[9];
            int index = 0;
            for (int dy = -1; dy <= 1; ++dy)
                for (int dx = -1; dx <= 1; ++dx) {
                    const int cx = std::min(std::max(int(x) + dx, 0), int(width) - 1);
                    const int cy = std::min(std::max(int(y) + dy, 0), int(height) - 1);
                    const float* v = in + (size_t(cy) * width + cx) * 4;
                    nb[index++] = F3{v[0], v[1], v[2]};
                }
            for (int i = 1; i < 9; ++i) {  // 83-95
                const F3 key = nb[i];
                const float keyLuminance = Luminance(key);
                int j = i - 1;
                while (j >= 0 && Luminance(nb[j]) > keyLuminance) {
                    nb[j + 1] = nb[j];
                    j = j - 1;
                }
                nb[j + 1] = key;
            }
            float* o = out + (size_t(y) * width + x) * 4;
            o[0] = nb[4].x; o[1] = nb[4].y; o[2] = nb[4].z; o[3] = 1.0f;
        }
}

// AnyHitShader's verdict (AlphaAccepts, RayTrace.hlsl:485-507) for n candidates (global triangle id,
// barycentrics b1, b2): out[i] = 1 accept, 0 reject.  Checks the GPU path's opacity micromap.
int oracle_alpha_accepts(const oracle_scene* scene, const uint32_t* gtri, const float* bary, uint32_t n, uint8_t* out) {
    const Scene& S = reinterpret_cast<const OracleScene*>(scene)->S;
    for (uint32_t i = 0; i < n; ++i) {
        if (gtri[i] >= S.tgeom.size()) return -1;
        out[i] = AlphaAccepts(S, S.tgeom[gtri[i]], gtri[i], bary[2 * i], bary[2 * i + 1]) ? 1u : 0u;
    }
    return 0;
}

int oracle_trace_rays(const oracle_scene* scene, const float* rays, uint32_t n, uint32_t flags, float* hits) {
    const Scene& S = reinterpret_cast<const OracleScene*>(scene)->S;
    Stats st;
    for (uint32_t i = 0; i < n; ++i) {
        const float* r = rays + size_t(i) * 8;
        Hit h;
        const bool any = (flags & 1u) != 0, alpha = (flags & 2u) != 0;
        bool hit = TraceRay(S, F3{r[0], r[1], r[2]}, F3{r[4], r[5], r[6]}, r[3], r[7], any, alpha, h, st);
        float* o = hits + size_t(i) * 4;
        uint32_t tri = hit && !any ? h.tri : kNone;
        if (any) {
            o[0] = hit ? 1.0f : -1.0f;
            o[1] = o[2] = 0.0f;
        } else {
            o[0] = hit ? h.t : -1.0f;
            o[1] = hit ? h.b1 : 0.0f;
            o[2] = hit ? h.b2 : 0.0f;
        }
        std::memcpy(&o[3], &tri, 4);
    }
    return 0;
}

}  // extern "C"
