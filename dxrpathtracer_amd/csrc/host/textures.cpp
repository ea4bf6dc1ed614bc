// textures.cpp — procedural material textures for the Sponza/SunTemple proxies.
//
// The reference loads DDS/PNG/JPG textures through DirectXTex/WIC (Graphics/Textures.cpp:38-172);
// the Sponza textures are not in the snapshot (README.md:14).  Each proxy material gets tileable,
// seeded albedo (sRGB), tangent-space normal, roughness and metallic maps (and an opacity map for
// alpha-tested cards), generated from periodic value noise so that wrap sampling has no seams.
#include <algorithm>
#include <cmath>
#include <cstring>

#include "scene_builder.h"

namespace dxrpt_host {

namespace {

inline uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU;
    x ^= x >> 15; x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}
inline float hashf(int ix, int iy, uint32_t seed) {
    uint32_t h = hash32(uint32_t(ix) * 0x8da6b343u ^ hash32(uint32_t(iy) * 0xd8163841u ^ seed));
    return float(h >> 8) * (1.0f / 16777216.0f);
}
inline float smooth(float t) { return t * t * (3.0f - 2.0f * t); }
inline int pmod(int a, int p) { int m = a % p; return m < 0 ? m + p : m; }

// Periodic value noise, period `p` lattice cells over [0,1).
float vnoise(float x, float y, int p, uint32_t seed) {
    float fx = x * p, fy = y * p;
    int ix = int(std::floor(fx)), iy = int(std::floor(fy));
    float tx = smooth(fx - ix), ty = smooth(fy - iy);
    float a = hashf(pmod(ix, p), pmod(iy, p), seed), b = hashf(pmod(ix + 1, p), pmod(iy, p), seed);
    float c = hashf(pmod(ix, p), pmod(iy + 1, p), seed), d = hashf(pmod(ix + 1, p), pmod(iy + 1, p), seed);
    return (a + (b - a) * tx) + ((c + (d - c) * tx) - (a + (b - a) * tx)) * ty;
}
float fbm(float x, float y, int p, int oct, uint32_t seed) {
    float s = 0, amp = 0.5f, norm = 0;
    for (int o = 0; o < oct; ++o) {
        s += amp * vnoise(x, y, p << o, seed + 1013u * o);
        norm += amp;
        amp *= 0.5f;
    }
    return s / norm;
}

struct Sample {
    float h;         // height for the normal map, [0,1]
    float c;         // albedo multiplier
    float rough;     // roughness offset
    float opacity;   // 1 opaque
};

Sample eval(Pattern p, float u, float v, uint32_t seed) {
    Sample s{0.5f, 1.0f, 0.0f, 1.0f};
    switch (p) {
        case Pattern::StoneTiles: {
            const int n = 4;
            float fu = u * n, fv = v * n;
            int iu = int(fu), iv = int(fv);
            float du = std::min(fu - iu, 1.0f - (fu - iu)), dv = std::min(fv - iv, 1.0f - (fv - iv));
            float edge = std::min(du, dv);
            float grout = edge < 0.03f ? 1.0f : 0.0f;
            float jit = hashf(iu, iv, seed);
            float nz = fbm(u, v, 8, 4, seed);
            s.h = grout ? 0.2f : 0.7f + 0.3f * nz;
            s.c = grout ? 0.55f : 0.8f + 0.25f * jit + 0.15f * (nz - 0.5f);
            s.rough = grout ? 0.2f : 0.1f * (nz - 0.5f);
            break;
        }
        case Pattern::Bricks: {
            const int rows = 8, cols = 4;
            float fv = v * rows;
            int iv = int(fv);
            float fu = u * cols + (iv & 1 ? 0.5f : 0.0f);
            int iu = int(std::floor(fu));
            float du = std::min(fu - std::floor(fu), 1.0f - (fu - std::floor(fu))) * 2.0f;
            float dv = std::min(fv - iv, 1.0f - (fv - iv));
            bool mortar = du < 0.04f || dv < 0.06f;
            float jit = hashf(pmod(iu, cols), iv, seed);
            float nz = fbm(u, v, 16, 3, seed);
            s.h = mortar ? 0.25f : 0.75f + 0.25f * nz;
            s.c = mortar ? 0.7f : 0.75f + 0.35f * jit + 0.1f * (nz - 0.5f);
            s.rough = mortar ? 0.15f : 0.0f;
            break;
        }
        case Pattern::Marble: {
            float t = fbm(u, v, 4, 5, seed);
            float vein = std::fabs(std::sin((u + v) * 6.2831853f * 2.0f + t * 9.0f));
            s.c = 0.75f + 0.25f * std::pow(vein, 0.3f);
            s.h = 0.5f + 0.1f * t;
            s.rough = -0.1f * vein;
            break;
        }
        case Pattern::Plaster: {
            float t = fbm(u, v, 8, 5, seed);
            s.c = 0.85f + 0.2f * (t - 0.5f);
            s.h = t;
            break;
        }
        case Pattern::Fabric: {
            const float N = 64.0f * 3.14159265f;
            float a = std::sin(u * N), b = std::sin(v * N);
            float weave = 0.5f + 0.25f * (a * (b > 0 ? 1.0f : -1.0f)) + 0.25f * b;
            float t = fbm(u, v, 4, 3, seed);
            s.c = 0.8f + 0.2f * weave + 0.1f * (t - 0.5f);
            s.h = weave;
            s.rough = 0.1f;
            break;
        }
        case Pattern::Wood: {
            float t = fbm(u, v, 4, 4, seed);
            float ring = 0.5f + 0.5f * std::sin((u * 20.0f + t * 6.0f) * 6.2831853f);
            s.c = 0.7f + 0.3f * ring;
            s.h = 0.5f + 0.2f * ring;
            break;
        }
        case Pattern::Metal: {
            float t = fbm(u * 0.1f, v, 32, 3, seed);
            s.c = 0.9f + 0.1f * t;
            s.h = 0.5f + 0.05f * t;
            s.rough = 0.15f * (t - 0.5f);
            break;
        }
        case Pattern::Leaves: {
            // 6 x 6 elliptical leaves per tile; opacity outside them
            const int n = 6;
            float fu = u * n, fv = v * n;
            int iu = int(fu), iv = int(fv);
            float lu = fu - iu - 0.5f, lv = fv - iv - 0.5f;
            float ang = hashf(iu, iv, seed) * 3.14159f;
            float ca = std::cos(ang), sa = std::sin(ang);
            float ru = ca * lu + sa * lv, rv = -sa * lu + ca * lv;
            float e = (ru * ru) / 0.16f + (rv * rv) / 0.04f;
            bool in = e < 1.0f;
            s.opacity = in ? 1.0f : 0.0f;
            s.c = 0.7f + 0.3f * hashf(iu, iv, seed + 7);
            s.h = in ? 1.0f - e : 0.0f;
            break;
        }
        case Pattern::Ceramic: {
            float t = fbm(u, v, 4, 3, seed);
            s.c = 0.9f + 0.1f * t;
            s.h = 0.5f;
            s.rough = -0.05f;
            break;
        }
        case Pattern::Roof: {
            const int rows = 10;
            float fv = v * rows;
            int iv = int(fv);
            float t = fv - iv;
            float nz = fbm(u, v, 8, 3, seed);
            s.h = t;
            s.c = 0.7f + 0.3f * t + 0.1f * (nz - 0.5f);
            break;
        }
    }
    return s;
}

inline uint8_t to_u8(float x) { return uint8_t(std::lround(std::min(std::max(x, 0.0f), 1.0f) * 255.0f)); }

}  // namespace

Texture solid_rgba(uint8_t r, uint8_t g, uint8_t b, uint8_t a, uint32_t fmt) {
    Texture t;
    t.w = t.h = 1;
    t.fmt = fmt;
    t.data = {r, g, b, a};
    return t;
}

Texture solid_r8(uint8_t v) {
    Texture t;
    t.w = t.h = 1;
    t.fmt = DXRPT_TEX_R8_UNORM;
    t.data = {v};
    return t;
}

MaterialTextures make_material_textures(Pattern p, uint64_t seed, uint32_t size, float r, float g, float b,
                                        float rough_base, float metal, bool with_opacity) {
    const uint32_t N = size;
    const uint32_t sd = uint32_t(seed ^ (seed >> 32));
    std::vector<Sample> S(size_t(N) * N);
    for (uint32_t y = 0; y < N; ++y)
        for (uint32_t x = 0; x < N; ++x) S[size_t(y) * N + x] = eval(p, (x + 0.5f) / N, (y + 0.5f) / N, sd);
    MaterialTextures mt;
    mt.albedo.w = mt.albedo.h = N;
    mt.albedo.fmt = DXRPT_TEX_RGBA8_SRGB;
    mt.albedo.data.resize(size_t(N) * N * 4);
    mt.normal.w = mt.normal.h = N;
    mt.normal.fmt = DXRPT_TEX_RGBA8_UNORM;
    mt.normal.data.resize(size_t(N) * N * 4);
    mt.roughness.w = mt.roughness.h = N;
    mt.roughness.fmt = DXRPT_TEX_R8_UNORM;
    mt.roughness.data.resize(size_t(N) * N);
    const float strength = 4.0f;
    for (uint32_t y = 0; y < N; ++y)
        for (uint32_t x = 0; x < N; ++x) {
            const Sample& s = S[size_t(y) * N + x];
            uint8_t* a = &mt.albedo.data[(size_t(y) * N + x) * 4];
            a[0] = to_u8(r * s.c);
            a[1] = to_u8(g * s.c);
            a[2] = to_u8(b * s.c);
            a[3] = 255;
            const float hl = S[size_t(y) * N + (x + N - 1) % N].h, hr = S[size_t(y) * N + (x + 1) % N].h;
            const float hd = S[size_t((y + N - 1) % N) * N + x].h, hu = S[size_t((y + 1) % N) * N + x].h;
            float nx = -(hr - hl) * strength, ny = -(hu - hd) * strength, nz = 1.0f;
            float l = std::sqrt(nx * nx + ny * ny + nz * nz);
            uint8_t* n = &mt.normal.data[(size_t(y) * N + x) * 4];
            n[0] = to_u8(nx / l * 0.5f + 0.5f);
            n[1] = to_u8(ny / l * 0.5f + 0.5f);
            n[2] = to_u8(nz / l * 0.5f + 0.5f);
            n[3] = 255;
            // roughness maps store sqrt(roughness) (RayTrace.hlsl:198, 202)
            mt.roughness.data[size_t(y) * N + x] = to_u8(rough_base + s.rough);
        }
    mt.metallic = solid_r8(to_u8(metal));
    if (with_opacity) {
        mt.opacity.w = mt.opacity.h = N;
        mt.opacity.fmt = DXRPT_TEX_R8_UNORM;
        mt.opacity.data.resize(size_t(N) * N);
        for (size_t i = 0; i < size_t(N) * N; ++i) mt.opacity.data[i] = to_u8(S[i].opacity);
    }
    return mt;
}

}  // namespace dxrpt_host
