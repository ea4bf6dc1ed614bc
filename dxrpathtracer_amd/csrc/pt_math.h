// pt_math.h — gfx950 device restatement of the path tracer's shader library.
//
// Every function restates an HLSL function of the reference with an explicit evaluation order.
// The library is compiled with -ffp-contract=off and correctly-rounded f32 divide/sqrt, so each
// expression rounds exactly as written; the CPU oracle (oracle/oracle.cpp) restates the same
// HLSL independently with the same order, which is what makes per-pixel parity checkable.
// Conventions fixed here (the D3D rounding is driver/vendor-defined and therefore unpinned):
//   dot(a,b)      = (a.x*b.x + a.y*b.y) + a.z*b.z
//   normalize(v)  = v / sqrt(dot(v,v))          (HLSL: v * rsqrt(dot(v,v)))
//   pow(x, 5)     = (x*x)*(x*x)*x               (BRDF.hlsl:18)
//   sin/cos       = pt_sincos (Cody-Waite + minimax, identical on host and device)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PT_DEV __device__ __forceinline__

namespace dxrpt {

// Shaders/Constants.hlsl:13-27
constexpr float kPi = 3.141592654f;
constexpr float kFP32Max = 3.402823466e+38f;
constexpr float kFP16Max = 65000.0f;

struct f3 {
    float x, y, z;
};
PT_DEV f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
PT_DEV f3 add(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
PT_DEV f3 sub(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
PT_DEV f3 mul(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
PT_DEV f3 scl(f3 a, float s) { return f3{a.x * s, a.y * s, a.z * s}; }
PT_DEV f3 neg(f3 a) { return f3{-a.x, -a.y, -a.z}; }
PT_DEV float dot3(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
PT_DEV f3 cross3(f3 a, f3 b) {
    return f3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
PT_DEV float len3(f3 a) { return sqrtf(dot3(a, a)); }
PT_DEV f3 normalize3(f3 a) {
    float l = sqrtf(dot3(a, a));
    return f3{a.x / l, a.y / l, a.z / l};
}
PT_DEV float saturate(float x) { return fminf(fmaxf(x, 0.0f), 1.0f); }
PT_DEV float lerpf(float a, float b, float t) { return a + t * (b - a); }
PT_DEV f3 lerp3(f3 a, f3 b, float t) { return f3{lerpf(a.x, b.x, t), lerpf(a.y, b.y, t), lerpf(a.z, b.z, t)}; }
// reflect(i, n) = i - 2 * n * dot(i, n)
PT_DEV f3 reflect3(f3 i, f3 n) {
    float d = dot3(i, n);
    return f3{i.x - (2.0f * n.x) * d, i.y - (2.0f * n.y) * d, i.z - (2.0f * n.z) * d};
}
PT_DEV float pow5(float x) {
    float x2 = x * x;
    return (x2 * x2) * x;
}
PT_DEV float smoothstepf(float a, float b, float x) {
    float t = saturate((x - a) / (b - a));
    return t * t * (3.0f - 2.0f * t);
}
PT_DEV f3 ld3(const float4& v) { return f3{v.x, v.y, v.z}; }

// Deterministic sin/cos: quadrant reduction by pi/2 (3-term Cody-Waite), Cephes minimax kernels.
PT_DEV void pt_sincos(float x, float* s, float* c) {
    float j = rintf(x * 0.636619772f);
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

// ---- Shaders/Sampling.hlsl:282-331 (Kensler correlated multi-jittered sampling) ------------------
PT_DEV uint32_t cmj_permute(uint32_t i, uint32_t l, uint32_t p) {
    uint32_t w = l - 1;
    w |= w >> 1;
    w |= w >> 2;
    w |= w >> 4;
    w |= w >> 8;
    w |= w >> 16;
    do {
        i ^= p; i *= 0xe170893du;
        i ^= p >> 16;
        i ^= (i & w) >> 4;
        i ^= p >> 8; i *= 0x0929eb3fu;
        i ^= p >> 23;
        i ^= (i & w) >> 1; i *= 1u | p >> 27;
        i *= 0x6935fa69u;
        i ^= (i & w) >> 11; i *= 0x74dcb303u;
        i ^= (i & w) >> 2; i *= 0x9e501cc3u;
        i ^= (i & w) >> 2; i *= 0xc860a3dfu;
        i &= w;
        i ^= i >> 5;
    } while (i >= l);
    return (i + p) % l;
}
PT_DEV float cmj_randfloat(uint32_t i, uint32_t p) {
    i ^= p;
    i ^= i >> 17;
    i ^= i >> 10; i *= 0xb36534e5u;
    i ^= i >> 12;
    i ^= i >> 21; i *= 0x93fc4795u;
    i ^= 0xdf6e307fu;
    i ^= i >> 17; i *= 1u | p >> 18;
    return float(i) * (1.0f / 4294967808.0f);
}
// DXRPT_CMJ_POW2 (r06): grids whose nx and ny are powers of two (SqrtNumSamples 1, 2, 4, 8, 16, ...: every
// BASELINE config uses 4) take the same arithmetic with the integer % and / as masks and shifts and the float
// divisions as multiplications by the exact reciprocal 2^-k -- bit-identical results (x / 2^k == x * 2^-k in
// binary floating point without underflow, which these values in [0, N] cannot reach), without the
// integer-division sequences (v_rcp_iflag + quarter-rate v_mul_hi/v_mul_lo) and the IEEE divide expansions.
// The grid size is wave-uniform, so the test is a scalar branch.
#ifndef DXRPT_CMJ_POW2
#define DXRPT_CMJ_POW2 1
#endif
PT_DEV uint32_t cmj_permute_pow2(uint32_t i, uint32_t l, uint32_t p) {  // l = 2^k: w = l - 1, one round
    const uint32_t w = l - 1u;
    i ^= p; i *= 0xe170893du;
    i ^= p >> 16;
    i ^= (i & w) >> 4;
    i ^= p >> 8; i *= 0x0929eb3fu;
    i ^= p >> 23;
    i ^= (i & w) >> 1; i *= 1u | p >> 27;
    i *= 0x6935fa69u;
    i ^= (i & w) >> 11; i *= 0x74dcb303u;
    i ^= (i & w) >> 2; i *= 0x9e501cc3u;
    i ^= (i & w) >> 2; i *= 0xc860a3dfu;
    i &= w;
    i ^= i >> 5;
    return (i + p) & w;  // i <= w after the mask (i >> 5 only clears bits), so the loop's test never repeats
}
PT_DEV void sample_cmj2d(uint32_t sampleIdx, uint32_t nx, uint32_t ny, uint32_t pattern, float* ox, float* oy) {
    uint32_t N = nx * ny;
    if (DXRPT_CMJ_POW2 && ((nx & (nx - 1u)) | (ny & (ny - 1u))) == 0u && nx != 0u && ny != 0u) {
        const uint32_t kx = uint32_t(__builtin_ctz(nx));
        sampleIdx = cmj_permute_pow2(sampleIdx, N, pattern * 0x51633e2du);
        uint32_t sx = cmj_permute_pow2(sampleIdx & (nx - 1u), nx, pattern * 0x68bc21ebu);
        uint32_t sy = cmj_permute_pow2(sampleIdx >> kx, ny, pattern * 0x02e5be93u);
        float jx = cmj_randfloat(sampleIdx, pattern * 0x967a889bu);
        float jy = cmj_randfloat(sampleIdx, pattern * 0x368cc8b7u);
        // 1 / 2^k as a float: exact (k < 32 here)
        const float rnx = __uint_as_float((127u - kx) << 23), rny = __uint_as_float((127u - uint32_t(__builtin_ctz(ny))) << 23);
        const float rN = __uint_as_float((127u - uint32_t(__builtin_ctz(N))) << 23);
        *ox = (float(sx) + (float(sy) + jx) * rny) * rnx;
        *oy = (float(sampleIdx) + jy) * rN;
        return;
    }
    sampleIdx = cmj_permute(sampleIdx, N, pattern * 0x51633e2du);
    uint32_t sx = cmj_permute(sampleIdx % nx, nx, pattern * 0x68bc21ebu);
    uint32_t sy = cmj_permute(sampleIdx / nx, ny, pattern * 0x02e5be93u);
    float jx = cmj_randfloat(sampleIdx, pattern * 0x967a889bu);
    float jy = cmj_randfloat(sampleIdx, pattern * 0x368cc8b7u);
    *ox = (float(sx) + (float(sy) + jx) / float(ny)) / float(nx);
    *oy = (float(sampleIdx) + jy) / float(N);
}

// ---- Shaders/Sampling.hlsl:72-114, 181-196 --------------------------------------------------------
PT_DEV void square_to_concentric_disk(float x, float y, float* ou, float* ov) {
    float phi = 0.0f, r = 0.0f;
    float a = 2.0f * x - 1.0f;
    float b = 2.0f * y - 1.0f;
    if (a > -b) {
        if (a > b) { r = a; phi = (kPi / 4.0f) * (b / a); }
        else { r = b; phi = (kPi / 4.0f) * (2.0f - (a / b)); }
    } else {
        if (a < b) { r = -a; phi = (kPi / 4.0f) * (4.0f + (b / a)); }
        else {
            r = -b;
            if (b != 0.0f) phi = (kPi / 4.0f) * (6.0f - (a / b));
            else phi = 0.0f;
        }
    }
    float s, c;
    pt_sincos(phi, &s, &c);
    *ou = r * c;
    *ov = r * s;
}
PT_DEV f3 sample_cosine_hemisphere(float u1, float u2) {
    float u, v;
    square_to_concentric_disk(u1, u2, &u, &v);
    float r = u * u + v * v;
    return f3{u, v, sqrtf(fmaxf(0.0f, 1.0f - r))};
}
// Sampling.hlsl:131-154
PT_DEV f3 sample_ggx_visible_normal(f3 wo, float ax, float ay, float u1, float u2) {
    f3 v = normalize3(f3{wo.x * ax, wo.y * ay, wo.z});
    f3 t1 = (v.z < 0.999f) ? normalize3(cross3(v, f3{0.0f, 0.0f, 1.0f})) : f3{1.0f, 0.0f, 0.0f};
    f3 t2 = cross3(t1, v);
    float a = 1.0f / (1.0f + v.z);
    float r = sqrtf(u1);
    float phi = (u2 < a) ? (u2 / a) * kPi : kPi + ((u2 - a) / (1.0f - a)) * kPi;
    float s, c;
    pt_sincos(phi, &s, &c);
    float p1 = r * c;
    float p2 = (r * s) * ((u2 < a) ? 1.0f : v.z);
    float w = sqrtf(fmaxf(0.0f, (1.0f - p1 * p1) - p2 * p2));
    f3 n = add(add(scl(t1, p1), scl(t2, p2)), scl(v, w));
    return normalize3(f3{ax * n.x, ay * n.y, fmaxf(0.0f, n.z)});
}

// ---- Shaders/BRDF.hlsl ------------------------------------------------------------------------------
// Fresnel, BRDF.hlsl:16-24
PT_DEV f3 fresnel(f3 specAlbedo, f3 h, f3 l) {
    float p = pow5(1.0f - saturate(dot3(l, h)));
    float fade = saturate(dot3(specAlbedo, f3{333.0f, 333.0f, 333.0f}));
    f3 f;
    f.x = (specAlbedo.x + (1.0f - specAlbedo.x) * p) * fade;
    f.y = (specAlbedo.y + (1.0f - specAlbedo.y) * p) * fade;
    f.z = (specAlbedo.z + (1.0f - specAlbedo.z) * p) * fade;
    return f;
}
// GGXV1 / GGXVisibility, BRDF.hlsl:89-100
PT_DEV float ggx_v1(float m2, float nDotX) { return 1.0f / (nDotX + sqrtf(m2 + ((1.0f - m2) * nDotX) * nDotX)); }
// SmithGGXMasking, BRDF.hlsl:102-109 (n = +z in tangent space)
PT_DEV float smith_ggx_masking(float dotNVraw, float a2) {
    float dotNV = saturate(dotNVraw);
    float denomC = sqrtf(a2 + ((1.0f - a2) * dotNV) * dotNV) + dotNV;
    return (2.0f * dotNV) / denomC;
}
// SmithGGXMaskingShadowing, BRDF.hlsl:111-120
PT_DEV float smith_ggx_masking_shadowing(float dotNLraw, float dotNVraw, float a2) {
    float dotNL = saturate(dotNLraw);
    float dotNV = saturate(dotNVraw);
    float denomA = dotNV * sqrtf(a2 + ((1.0f - a2) * dotNL) * dotNL);
    float denomB = dotNL * sqrtf(a2 + ((1.0f - a2) * dotNV) * dotNV);
    return ((2.0f * dotNL) * dotNV) / (denomA + denomB);
}
// GGXSpecular, BRDF.hlsl:128-145
PT_DEV float ggx_specular(float m, f3 n, f3 h, f3 v, f3 l) {
    float nDotH = saturate(dot3(n, h));
    float nDotL = saturate(dot3(n, l));
    float nDotV = saturate(dot3(n, v));
    float m2 = m * m;
    float x = (nDotH * nDotH) * (m2 - 1.0f) + 1.0f;
    float d = m2 / ((kPi * x) * x);
    float vis = ggx_v1(m2, nDotL) * ggx_v1(m2, nDotV);
    return d * vis;
}
// GGXEnvironmentBRDFScaleBias, BRDF.hlsl:209-224 (returns the scale = Ess)
PT_DEV float ggx_env_brdf_scale(float nDotV, float sqrtRoughness) {
    const float nDotV2 = nDotV * nDotV;
    const float s2 = sqrtRoughness * sqrtRoughness;
    const float s3 = s2 * sqrtRoughness;
    const float delta = ((0.991086418474895f + (0.412367709802119f * sqrtRoughness) * nDotV2) -
                         0.363848256078895f * s2) -
                        (0.758634385642633f * nDotV) * s2;
    const float bias = saturate((0.0306613448029984f * sqrtRoughness +
                                 0.0238299731830387f / ((0.0272458171384516f + s3) + nDotV2)) -
                                0.0454747751719356f);
    return saturate(delta - bias);
}
// CalcLighting, BRDF.hlsl:241-261
PT_DEV f3 calc_lighting(f3 normal, f3 lightDir, f3 peakIrradiance, f3 diffuseAlbedo, f3 specularAlbedo,
                        float roughness, f3 positionWS, f3 cameraPosWS, f3 msEC) {
    f3 lighting = scl(diffuseAlbedo, 1.0f / 3.14159f);
    f3 view = normalize3(sub(cameraPosWS, positionWS));
    const float nDotL = saturate(dot3(normal, lightDir));
    if (nDotL > 0.0f) {
        f3 h = normalize3(add(view, lightDir));
        f3 fr = fresnel(specularAlbedo, h, lightDir);
        float specular = ggx_specular(roughness, normal, h, view, lightDir);
        lighting = add(lighting, mul(scl(fr, specular), msEC));
    }
    return mul(scl(lighting, nDotL), peakIrradiance);
}

}  // namespace dxrpt
