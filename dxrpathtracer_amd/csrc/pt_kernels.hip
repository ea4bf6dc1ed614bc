// pt_kernels.hip — wavefront path tracer for gfx950 (MI355X).
//
// Replaces the recursive DXR pipeline of DXRPathTracer/RayTrace.hlsl (RaygenShader 92-149,
// PathTrace 151-441, ClosestHit 476-483, AnyHit 485-507, Miss 509-530, ShadowHit/Miss 532-542)
// with one kernel per stage and depth:
//
//   k_raygen        (1 thread / pixel)       CMJ set-0 jitter, unproject, primary ray -> queue[1]
//   for d = 1 .. MaxPathLength-1:            (d = PathLength of the radiance rays in queue[d])
//     k_trace       (1 thread / queued ray)  closest hit; alpha-tested any-hit iff d <= MaxAnyHitPathLength
//     k_shade       (1 thread / queued ray)  miss: sky/sun disc.  hit: PathTrace -> emissive, sun/spot
//                                            shadow rays with their pending CalcLighting terms, BRDF
//                                            sample, continuation ray (wave64 ballot compaction into
//                                            queue[d+1]) or the final sky-visibility ray
//     k_shadow      (1 thread / queued ray)  any-hit traversal of that ray's shadow rays, adds
//                                            contribution * visibility to the path's radiance
//   k_accumulate    (1 thread / pixel)       clamp to FP16Max, lerp into the RGBA32F target
//
// Recursion becomes a loop: path throughput (product of the BRDF throughputs of earlier vertices)
// is carried in the path state so every term can be added to the pixel directly.  Each path owns
// its pixel's radiance, every add happens in one thread in a fixed order: results are deterministic
// run to run and independent of the tiling.
//
// BVH traversal: BVH2 or compressed BVH8 (pt_layout.h), one ray per lane, per-lane stack in LDS sized
// to the built tree's depth (SceneDev::stack_ints x 4 B x 256 lanes per workgroup, dynamic shared
// memory), exact Moller-Trumbore triangle test (same arithmetic as the oracle) behind conservative
// (padded) slab tests.
#include <hip/hip_runtime.h>

#include "pt_kernels.h"
#include "pt_math.h"

namespace dxrpt {

constexpr int kBlock = 256;
constexpr uint32_t kMiss = 0xFFFFFFFFu;
constexpr float kRayTMin = 0.00001f;          // RayTrace.hlsl:243, 382
constexpr float kSpotShadowNearClip = 0.1f;   // AppSettings.hlsl:56

PT_DEV uint32_t fbits(float f) { return __float_as_uint(f); }
PT_DEV float bitsf(uint32_t u) { return __uint_as_float(u); }

// Per-lane traversal stacks in LDS: wave w of the workgroup owns S.stack_ints x 64 ints, entry j of
// lane l at [j * 64 + l] (conflict-free, and the stride is a compile-time constant so every stack
// access is one ds_read/ds_write with an immediate offset).  The LDS address space is explicit so
// the spill path (global) never merges with it into flat accesses.
typedef __attribute__((address_space(3))) int lds_int;
constexpr int kStkStride = 64;
#ifndef DXRPT_STACK_REMAT
#define DXRPT_STACK_REMAT 0
#endif
#ifndef DXRPT_STACK_TID
#define DXRPT_STACK_TID 1
#endif
PT_DEV lds_int* lane_stack(const SceneDev& S, int* stack) {
#if DXRPT_STACK_REMAT
    // the wave's part scalar, the lane's from mbcnt: cheap to recompute, so the compiler need not keep
    // (or spill) a per-lane base across the path
    const uint32_t wave = uint32_t(__builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6)));
    return (lds_int*)(stack) + wave * S.stack_ints * 64u + uint32_t(__lane_id());
#else
    return (lds_int*)(stack) + (threadIdx.x >> 6) * S.stack_ints * 64u + (threadIdx.x & 63u);
#endif
}

// ---- texture sampling ---------------------------------------------------------------------------
// SampleLevel(MeshSampler, uv, 0): MeshSampler is anisotropic x16 with WRAP addressing
// (Graphics/DX12_Helpers.cpp:327-338); at LOD 0 on mip 0 this is defined here as bilinear with
// wrap, texel centres at (i + 0.5) / size, weights lerp(lerp(t00,t10,fx), lerp(t01,t11,fx), fy).
PT_DEV int wrap_coord(int i, uint32_t n) {
    if ((n & (n - 1u)) == 0u) return i & int(n - 1u);
    int m = i % int(n);
    return m < 0 ? m + int(n) : m;
}

typedef float f2v __attribute__((ext_vector_type(2)));

struct Texel4 {
    float r, g, b, a;
};

// DXRPT_LDS_LUT: the 512-entry decode table (unorm, sRGB) is copied to the workgroup's LDS at kernel
// start (lut_fill), so a texel's decode is an LDS read instead of a dependent global-memory gather.
// Every kernel that samples textures (shading, alpha-tested traversal) calls lut_fill first.
#ifndef DXRPT_LDS_LUT
#define DXRPT_LDS_LUT 1
#endif
#if DXRPT_LDS_LUT
__shared__ float g_lut[512];
#endif

PT_DEV void lut_fill(const SceneDev& S) {
#if DXRPT_LDS_LUT
    for (uint32_t i = threadIdx.x; i < 512u; i += blockDim.x) g_lut[i] = S.lut[i];
    __syncthreads();
#endif
}

PT_DEV float lut_at(const SceneDev& S, uint32_t i) {
#if DXRPT_LDS_LUT
    return g_lut[i];
#else
    return S.lut[i];
#endif
}

PT_DEV Texel4 fetch_texel(const SceneDev& S, const TexDesc& td, int x, int y) {
    const bool r8 = td.fmt == DXRPT_TEX_R8_UNORM;
    const uint32_t tiles_x = (td.width + (r8 ? kTexTileW8 : kTexTileW32) - 1u) / (r8 ? kTexTileW8 : kTexTileW32);
    const uint32_t word = tex_tile_word(uint32_t(x), uint32_t(y), tiles_x, r8);
    Texel4 t;
    if (r8) {
        uint32_t w = S.texels[td.offset + word];
        float v = lut_at(S, (w >> ((uint32_t(x) & 3u) * 8u)) & 0xFFu);
        t.r = v; t.g = v; t.b = v; t.a = 1.0f;
    } else {
        uint32_t w = S.texels[td.offset + word];
        const uint32_t l = td.fmt == DXRPT_TEX_RGBA8_SRGB ? 256u : 0u;
        t.r = lut_at(S, l + (w & 0xFFu));
        t.g = lut_at(S, l + ((w >> 8) & 0xFFu));
        t.b = lut_at(S, l + ((w >> 16) & 0xFFu));
        t.a = lut_at(S, w >> 24);
    }
    return t;
}

PT_DEV Texel4 sample_tex_desc(const SceneDev& S, const TexDesc td, float u, float v);

PT_DEV Texel4 sample_tex(const SceneDev& S, uint32_t texIdx, float u, float v) {
    return sample_tex_desc(S, S.texdesc[texIdx], u, v);
}

PT_DEV TexDesc tex_desc(GeoTex g) {
    TexDesc td;
    td.offset = g.offset;
    td.width = g.whf & 0x7FFFu;
    td.height = (g.whf >> 15) & 0x7FFFu;
    td.fmt = g.whf >> 30;
    return td;
}

PT_DEV Texel4 sample_tex_desc(const SceneDev& S, const TexDesc td, float u, float v) {
    float x = u * float(td.width) - 0.5f;
    float y = v * float(td.height) - 0.5f;
    float x0 = floorf(x), y0 = floorf(y);
    float fx = x - x0, fy = y - y0;
    int ix0 = wrap_coord(int(x0), td.width), ix1 = wrap_coord(int(x0) + 1, td.width);
    int iy0 = wrap_coord(int(y0), td.height), iy1 = wrap_coord(int(y0) + 1, td.height);
    Texel4 t00 = fetch_texel(S, td, ix0, iy0), t10 = fetch_texel(S, td, ix1, iy0);
    Texel4 t01 = fetch_texel(S, td, ix0, iy1), t11 = fetch_texel(S, td, ix1, iy1);
    Texel4 r;
    r.r = lerpf(lerpf(t00.r, t10.r, fx), lerpf(t01.r, t11.r, fx), fy);
    r.g = lerpf(lerpf(t00.g, t10.g, fx), lerpf(t01.g, t11.g, fx), fy);
    r.b = lerpf(lerpf(t00.b, t10.b, fx), lerpf(t01.b, t11.b, fx), fy);
    r.a = lerpf(lerpf(t00.a, t10.a, fx), lerpf(t01.a, t11.a, fx), fy);
    return r;
}

// Sky cube SampleLevel(LinearSampler, dir, 0) (RayTrace.hlsl:434, 521): LinearSampler is
// linear/clamp (DX12_Helpers.cpp:282-293).  Defined here as: D3D major-axis face selection (ties
// resolve x before y before z), bilinear within the face, clamped to the face edge.
PT_DEV float half_to_float(uint16_t h) { return float(__builtin_bit_cast(_Float16, h)); }

PT_DEV f3 sample_sky(const SceneDev& S, f3 d) {
    float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    int face;
    float ma, sc, tc;
    if (ax >= ay && ax >= az) {
        face = d.x >= 0.0f ? 0 : 1; ma = ax; sc = d.x >= 0.0f ? -d.z : d.z; tc = -d.y;
    } else if (ay >= az) {
        face = d.y >= 0.0f ? 2 : 3; ma = ay; sc = d.x; tc = d.y >= 0.0f ? d.z : -d.z;
    } else {
        face = d.z >= 0.0f ? 4 : 5; ma = az; sc = d.z >= 0.0f ? d.x : -d.x; tc = -d.y;
    }
    const float res = float(S.sky_res);
    float u = (sc / ma + 1.0f) * 0.5f;
    float v = (tc / ma + 1.0f) * 0.5f;
    float x = u * res - 0.5f, y = v * res - 0.5f;
    float x0 = floorf(x), y0 = floorf(y);
    float fx = x - x0, fy = y - y0;
    const int rmax = int(S.sky_res) - 1;
    int ix0 = min(max(int(x0), 0), rmax), ix1 = min(max(int(x0) + 1, 0), rmax);
    int iy0 = min(max(int(y0), 0), rmax), iy1 = min(max(int(y0) + 1, 0), rmax);
    const uint16_t* base = S.sky + size_t(face) * S.sky_res * S.sky_res * 4u;
    const ushort4* t = reinterpret_cast<const ushort4*>(base);
    ushort4 a = t[iy0 * S.sky_res + ix0], b = t[iy0 * S.sky_res + ix1];
    ushort4 c = t[iy1 * S.sky_res + ix0], e = t[iy1 * S.sky_res + ix1];
    f3 r;
    r.x = lerpf(lerpf(half_to_float(a.x), half_to_float(b.x), fx), lerpf(half_to_float(c.x), half_to_float(e.x), fx), fy);
    r.y = lerpf(lerpf(half_to_float(a.y), half_to_float(b.y), fx), lerpf(half_to_float(c.y), half_to_float(e.y), fx), fy);
    r.z = lerpf(lerpf(half_to_float(a.z), half_to_float(b.z), fx), lerpf(half_to_float(c.z), half_to_float(e.z), fx), fy);
    return r;
}

// ---- hit surface (RayTrace.hlsl:444-474, Shaders/RayTracing.hlsl:43-53) --------------------------
struct Surface {
    f3 pos, n, t, b;
    float u, v;
};

PT_DEV float bary_lerp(float a, float b, float c, float w0, float w1, float w2) { return (a * w0 + b * w1) + c * w2; }

PT_DEV Surface get_hit_surface(const SceneDev& S, uint32_t gtri, float b1, float b2) {
    const float w0 = (1.0f - b1) - b2;
    // the triangle's vertices idx[gtri*3 + k] + VtxOffset, copied contiguously at build time
    const float4* V = S.tri_verts + size_t(gtri) * 12u;
    float4 q[3][4];
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int j = 0; j < 4; ++j) q[k][j] = V[k * 4 + j];
    // MeshVertex layout: q[.][0] = pos.xyz, n.x ; [1] = n.yz, uv ; [2] = t.xyz, b.x ; [3] = b.yz, lmuv
    Surface s;
    s.pos = f3{bary_lerp(q[0][0].x, q[1][0].x, q[2][0].x, w0, b1, b2), bary_lerp(q[0][0].y, q[1][0].y, q[2][0].y, w0, b1, b2),
               bary_lerp(q[0][0].z, q[1][0].z, q[2][0].z, w0, b1, b2)};
    s.n = normalize3(f3{bary_lerp(q[0][0].w, q[1][0].w, q[2][0].w, w0, b1, b2), bary_lerp(q[0][1].x, q[1][1].x, q[2][1].x, w0, b1, b2),
                        bary_lerp(q[0][1].y, q[1][1].y, q[2][1].y, w0, b1, b2)});
    s.u = bary_lerp(q[0][1].z, q[1][1].z, q[2][1].z, w0, b1, b2);
    s.v = bary_lerp(q[0][1].w, q[1][1].w, q[2][1].w, w0, b1, b2);
    s.t = normalize3(f3{bary_lerp(q[0][2].x, q[1][2].x, q[2][2].x, w0, b1, b2), bary_lerp(q[0][2].y, q[1][2].y, q[2][2].y, w0, b1, b2),
                        bary_lerp(q[0][2].z, q[1][2].z, q[2][2].z, w0, b1, b2)});
    s.b = normalize3(f3{bary_lerp(q[0][2].w, q[1][2].w, q[2][2].w, w0, b1, b2), bary_lerp(q[0][3].x, q[1][3].x, q[2][3].x, w0, b1, b2),
                        bary_lerp(q[0][3].y, q[1][3].y, q[2][3].y, w0, b1, b2)});
    return s;
}

// AnyHitShader / ShadowAnyHitShader (RayTrace.hlsl:485-507): opacity.x < 0.35 -> IgnoreHit.
// The opacity tap of AnyHitShader split in two, so several candidates' texel loads are in flight
// together (traverse8_packet's two-triangle steps): issue computes the bilinear footprint and loads its
// four texel words, finish decodes and filters channel r exactly as sample_tex_desc(...).r does.
struct OpacityTap {
    uint32_t w00, w10, w01, w11;  // texel words
    uint32_t s0, s1;              // byte shift of column ix0 / ix1 (R8: x & 3; RGBA8: 0)
    uint32_t lut;                 // decode table base (0 unorm, 256 sRGB)
    float fx, fy;
};

PT_DEV OpacityTap opacity_issue(const SceneDev& S, const TexDesc td, float u, float v) {
    float x = u * float(td.width) - 0.5f;
    float y = v * float(td.height) - 0.5f;
    float x0 = floorf(x), y0 = floorf(y);
    OpacityTap t;
    t.fx = x - x0;
    t.fy = y - y0;
    const int ix0 = wrap_coord(int(x0), td.width), ix1 = wrap_coord(int(x0) + 1, td.width);
    const int iy0 = wrap_coord(int(y0), td.height), iy1 = wrap_coord(int(y0) + 1, td.height);
    const bool r8 = td.fmt == DXRPT_TEX_R8_UNORM;
    const uint32_t tiles_x = (td.width + (r8 ? kTexTileW8 : kTexTileW32) - 1u) / (r8 ? kTexTileW8 : kTexTileW32);
    const uint32_t* T = S.texels + td.offset;
    t.w00 = T[tex_tile_word(uint32_t(ix0), uint32_t(iy0), tiles_x, r8)];
    t.w10 = T[tex_tile_word(uint32_t(ix1), uint32_t(iy0), tiles_x, r8)];
    t.w01 = T[tex_tile_word(uint32_t(ix0), uint32_t(iy1), tiles_x, r8)];
    t.w11 = T[tex_tile_word(uint32_t(ix1), uint32_t(iy1), tiles_x, r8)];
    t.s0 = r8 ? (uint32_t(ix0) & 3u) * 8u : 0u;
    t.s1 = r8 ? (uint32_t(ix1) & 3u) * 8u : 0u;
    t.lut = td.fmt == DXRPT_TEX_RGBA8_SRGB ? 256u : 0u;
    return t;
}

PT_DEV float opacity_finish(const SceneDev& S, const OpacityTap& t) {
    const float a = lut_at(S, t.lut + ((t.w00 >> t.s0) & 0xFFu)), b = lut_at(S, t.lut + ((t.w10 >> t.s1) & 0xFFu));
    const float c = lut_at(S, t.lut + ((t.w01 >> t.s0) & 0xFFu)), d = lut_at(S, t.lut + ((t.w11 >> t.s1) & 0xFFu));
    return lerpf(lerpf(a, b, t.fx), lerpf(c, d, t.fx), t.fy);
}

// Opacity micromap (pt_layout.h kOmm*): the word holding the cell of a candidate at barycentrics
// (b1, b2) of the triangle in micromap slot `slot` (TriRecord flags >> 1), and its verdict
// (kOmmOpaque / kOmmTransparent decide AnyHitShader without its tap, kOmmUnknown: tap).
struct OmmProbe {
    uint32_t word, shift;
};
PT_DEV OmmProbe omm_probe(const SceneDev& S, uint32_t slot, float b1, float b2) {
    OmmProbe p{0u, 0u};
    if (S.omm && b1 + b2 <= 2.0f) {  // NaN barycentrics: the tap decides
        const uint32_t c = omm_cell(b1, b2);
        p.word = S.omm[size_t(slot) * kOmmWords + (c >> 4)];
        p.shift = 2u * (c & 15u);
    }
    return p;
}
PT_DEV uint32_t omm_verdict(const OmmProbe& p) { return (p.word >> p.shift) & 3u; }

#ifndef DXRPT_ALPHA_ONE_TRIP
#define DXRPT_ALPHA_ONE_TRIP 1
#endif
PT_DEV bool alpha_accepts(const SceneDev& S, uint32_t geom, uint32_t gtri, uint32_t slot, float b1, float b2) {
    const GeoTex opacity = S.geoshade[geom].opacity;
    const float2* V = reinterpret_cast<const float2*>(S.tri_verts + size_t(gtri) * 12u);
    float2 uv[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) uv[k] = V[k * 8 + 3];  // float2 #3 of MeshVertex k = UV
    const OmmProbe om = omm_probe(S, slot, b1, b2);
#if DXRPT_ALPHA_ONE_TRIP
    // the opacity descriptor, the UVs and the micromap word in one memory round trip (a triangle that
    // reaches here is alpha tested, so its geometry has an opacity map; otherwise they are unused)
    asm volatile("" ::"v"(opacity.offset), "v"(opacity.whf), "v"(uv[0].x), "v"(uv[0].y), "v"(uv[1].x), "v"(uv[1].y),
                 "v"(uv[2].x), "v"(uv[2].y), "v"(om.word));
#endif
    if (opacity.whf == 0u) return true;
    const uint32_t verdict = omm_verdict(om);
    if (verdict != kOmmUnknown) return verdict == kOmmOpaque;
    const float w0 = (1.0f - b1) - b2;
    float u = bary_lerp(uv[0].x, uv[1].x, uv[2].x, w0, b1, b2);
    float v = bary_lerp(uv[0].y, uv[1].y, uv[2].y, w0, b1, b2);
    return !(sample_tex_desc(S, tex_desc(opacity), u, v).r < 0.35f);
}

// ---- traversal ------------------------------------------------------------------------------------
// Moller-Trumbore, two-sided (no culling flags are set in the reference, Timing.txt:3).  The
// arithmetic below is bit-identical to oracle/oracle.cpp:intersect_triangle.
PT_DEV bool intersect_triangle(f3 o, f3 d, f3 v0, f3 e1, f3 e2, float* t, float* u, float* v) {
    f3 pvec = cross3(d, e2);
    float det = dot3(e1, pvec);
    if (det == 0.0f) return false;
    float inv = 1.0f / det;
    f3 tvec = sub(o, v0);
    float uu = dot3(tvec, pvec) * inv;
    if (uu < 0.0f || uu > 1.0f) return false;
    f3 qvec = cross3(tvec, e1);
    float vv = dot3(d, qvec) * inv;
    if (vv < 0.0f || uu + vv > 1.0f) return false;
    *t = dot3(e2, qvec) * inv;
    *u = uu;
    *v = vv;
    return true;
}

struct HitRec {
    float t, b1, b2;
    uint32_t tri;   // global triangle id, kMiss if none
    uint32_t geom;
};

// One candidate triangle (the "intersection + any-hit" stage of a DXR traversal).  Returns true
// when an any-hit ray is done (accepted occluder).  Closest hit: smallest t, ties -> smallest global
// triangle id, which makes the result independent of traversal order.
// A leaf-ordered triangle record: v0, e1, e2 as float4 (.w = global tri id / geometry / flags).
struct TriRec {
    float4 p0, p1, p2;
};

// Keeps a loaded record in registers at this point: the compiler otherwise sinks the v0 load behind
// the det != 0 branch, which costs a second dependent round trip per triangle.
PT_DEV void pin_tri(const TriRec& r) {
    asm volatile("" ::"v"(r.p0.x), "v"(r.p0.y), "v"(r.p0.z), "v"(r.p0.w), "v"(r.p1.x), "v"(r.p1.y), "v"(r.p1.z),
                 "v"(r.p1.w), "v"(r.p2.x), "v"(r.p2.y), "v"(r.p2.z), "v"(r.p2.w));
}

// DXRPT_PIN_LOADS: a record's words come from one 64-bit base address (immediate offsets) and are
// all in registers before the first test uses them -- one memory round trip per record.
#ifndef DXRPT_PIN_LOADS
#define DXRPT_PIN_LOADS 1
#endif

PT_DEV TriRec load_tri_raw(const SceneDev& S, uint32_t rec) {
    const float4* T = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(S.tris) + size_t(rec) * 48u);
    return TriRec{T[0], T[1], T[2]};
}

PT_DEV TriRec load_tri(const SceneDev& S, uint32_t rec) {
#if DXRPT_PIN_LOADS
    const TriRec r = load_tri_raw(S, rec);
    pin_tri(r);
    return r;
#else
    const float4* T = reinterpret_cast<const float4*>(S.tris);
    return TriRec{T[rec * 3 + 0], T[rec * 3 + 1], T[rec * 3 + 2]};
#endif
}

template <bool kAnyHit>
PT_DEV bool test_tri_rec(const SceneDev& S, const TriRec& r, f3 o, f3 d, float tmin, float tmax, bool alpha, HitRec& h) {
    const float4 p0 = r.p0, p1 = r.p1, p2 = r.p2;
    float t, u, v;
    if (!intersect_triangle(o, d, ld3(p0), ld3(p1), ld3(p2), &t, &u, &v)) return false;
    const uint32_t gtri = fbits(p0.w);
    if (!(t >= tmin)) return false;
    if (kAnyHit) {
        if (!(t <= tmax)) return false;
    } else {
        if (!(t < h.t || (t == h.t && gtri < h.tri))) return false;
    }
    const uint32_t geom = fbits(p1.w);
    if (alpha && !(fbits(p2.w) & kTriOpaque) && !alpha_accepts(S, geom, gtri, fbits(p2.w) >> 1, u, v)) return false;
    h.t = t;
    h.tri = gtri;
    h.b1 = u;
    h.b2 = v;
    h.geom = geom;
    return kAnyHit;
}

// The geometric part of test_tri_rec: the triangle is a candidate if the ray hits it inside
// [tmin, tmax] (any hit) or ahead of the current best (closest hit); alpha and acceptance follow.
template <bool kAnyHit>
PT_DEV bool tri_candidate(const TriRec& r, f3 o, f3 d, float tmin, float tmax, const HitRec& h, float& t, float& u,
                          float& v) {
    if (!intersect_triangle(o, d, ld3(r.p0), ld3(r.p1), ld3(r.p2), &t, &u, &v)) return false;
    if (!(t >= tmin)) return false;
    if (kAnyHit) return t <= tmax;
    const uint32_t gtri = fbits(r.p0.w);
    return t < h.t || (t == h.t && gtri < h.tri);
}

template <bool kAnyHit>
PT_DEV bool test_triangle(const SceneDev& S, uint32_t rec, f3 o, f3 d, float tmin, float tmax, bool alpha, HitRec& h) {
    return test_tri_rec<kAnyHit>(S, load_tri(S, rec), o, d, tmin, tmax, alpha, h);
}

PT_DEV f3 safe_inverse(f3 d) {
    f3 inv;
    inv.x = 1.0f / (fabsf(d.x) > 1e-20f ? d.x : copysignf(1e-20f, d.x));
    inv.y = 1.0f / (fabsf(d.y) > 1e-20f ? d.y : copysignf(1e-20f, d.y));
    inv.z = 1.0f / (fabsf(d.z) > 1e-20f ? d.z : copysignf(1e-20f, d.z));
    return inv;
}

// BVH2 traversal ("while-while", Aila & Laine 2009): nearer child first, farther pushed on a per-lane
// LDS stack (stk[sp * kStkStride]).
template <bool kAnyHit, bool kCount>
PT_DEV bool traverse2(const SceneDev& S, f3 o, f3 d, float tmin, float tmax, bool alpha, lds_int* stk, HitRec& h,
                      uint32_t& nvisit, uint32_t& ntest) {
    const f3 inv = safe_inverse(d);
    const f3 ood = mul(o, inv);
    int node = 0;
    int sp = 0;
    const float4* N = reinterpret_cast<const float4*>(S.nodes);
    while (true) {
        while (node >= 0) {
            if (kCount) ++nvisit;
            const float4 a = N[node * 4 + 0];
            const float4 b = N[node * 4 + 1];
            const float4 c = N[node * 4 + 2];
            const int4 ch = reinterpret_cast<const int4*>(N)[node * 4 + 3];
            const float tmx = h.t;
            float l0x = __builtin_fmaf(a.x, inv.x, -ood.x), h0x = __builtin_fmaf(a.y, inv.x, -ood.x);
            float l0y = __builtin_fmaf(a.z, inv.y, -ood.y), h0y = __builtin_fmaf(a.w, inv.y, -ood.y);
            float l0z = __builtin_fmaf(c.x, inv.z, -ood.z), h0z = __builtin_fmaf(c.y, inv.z, -ood.z);
            float l1x = __builtin_fmaf(b.x, inv.x, -ood.x), h1x = __builtin_fmaf(b.y, inv.x, -ood.x);
            float l1y = __builtin_fmaf(b.z, inv.y, -ood.y), h1y = __builtin_fmaf(b.w, inv.y, -ood.y);
            float l1z = __builtin_fmaf(c.z, inv.z, -ood.z), h1z = __builtin_fmaf(c.w, inv.z, -ood.z);
            float n0 = fmaxf(fmaxf(fminf(l0x, h0x), fminf(l0y, h0y)), fmaxf(fminf(l0z, h0z), tmin));
            float f0 = fminf(fminf(fmaxf(l0x, h0x), fmaxf(l0y, h0y)), fminf(fmaxf(l0z, h0z), tmx));
            float n1 = fmaxf(fmaxf(fminf(l1x, h1x), fminf(l1y, h1y)), fmaxf(fminf(l1z, h1z), tmin));
            float f1 = fminf(fminf(fmaxf(l1x, h1x), fmaxf(l1y, h1y)), fminf(fmaxf(l1z, h1z), tmx));
            const bool hit0 = n0 <= f0, hit1 = n1 <= f1;
            if (hit0 && hit1) {
                int first = ch.x, second = ch.y;
                if (n1 < n0) { first = ch.y; second = ch.x; }
                stk[sp * kStkStride] = second;
                ++sp;
                node = first;
            } else if (hit0 || hit1) {
                node = hit0 ? ch.x : ch.y;
            } else {
                if (sp == 0) return kAnyHit ? false : h.tri != kMiss;
                --sp;
                node = stk[sp * kStkStride];
            }
        }
        const uint32_t code = ~uint32_t(node);
        const uint32_t first = code >> 3, count = (code & 7u) + 1u;
        for (uint32_t k = 0; k < count; ++k) {
            if (kCount) ++ntest;
            if (test_triangle<kAnyHit>(S, first + k, o, d, tmin, tmax, alpha, h)) return true;
        }
        if (sp == 0) return kAnyHit ? false : h.tri != kMiss;
        --sp;
        node = stk[sp * kStkStride];
    }
}

// Compressed BVH8 traversal (Ylitie, Karras & Laine 2017, adapted to one ray per wave64 lane).
// A node visit intersects all 8 quantised child boxes at once; internal hits form a "node group"
// (base_child, hit bits keyed by slot ^ octant, imask) visited highest key first (near to far), leaf
// hits are tested right away.  The rest of a group is pushed when descending: <= 1 push per level,
// 2 x 4 B per entry in LDS (stk[2 sp * kStkStride], stk[(2 sp + 1) * kStkStride]).
// The traversal is a resumable state machine (Ray8 + node + sp) so persistent kernels can advance
// every lane by one node visit per iteration and refill lanes whose ray finished.
struct Ray8 {
    f3 o, d, inv, ood;
    float tmin, tmax;
    uint32_t oct;
    bool alpha;
};

PT_DEV void ray8_init(Ray8& R, f3 o, f3 d, float tmin, float tmax, bool alpha, HitRec& h) {
    R.o = o;
    R.d = d;
    R.inv = safe_inverse(d);
    R.ood = mul(o, R.inv);
    R.tmin = tmin;
    R.tmax = tmax;
    R.oct = (R.inv.x < 0.0f ? 4u : 0u) | (R.inv.y < 0.0f ? 2u : 0u) | (R.inv.z < 0.0f ? 1u : 0u);
    R.alpha = alpha;
    h.t = tmax;
    h.tri = kMiss;
    h.b1 = h.b2 = 0.0f;
    h.geom = 0;
}

// Visits `node`: its hit leaf triangles become the pending group (tbase, tbits); then selects the next
// node (pops when the current group is exhausted).  Returns false when no node is left to visit.  The
// pending triangles must be tested (trav8_tris) before the next node visit, so that the visit order
// and hence the result are the same however tests and visits of different lanes are interleaved.
// Group stack: `sp` entries; the top one lives in registers (`tos`), entries 0 .. sp-2 in LDS
// (first kStackLds8) and in the thread's global spill slab (deeper), so a pop hands over the next
// group at once and the LDS refill of `tos` overlaps the next node fetch.
// DXRPT_STACK_TID (the megakernel's 64-thread workgroups, stk == nullptr): the lane's stack base is
// recomputed at every access from the lane id (volatile asm: never kept live across the path, so it is
// never spilled and reloaded from scratch on a push or pop).
PT_DEV lds_int* stack_base(lds_int* stk) {
#if DXRPT_STACK_TID
    if (stk == nullptr) {
        extern __shared__ int stack[];
        uint32_t lane;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
        return (lds_int*)(stack) + lane;
    }
#endif
    return stk;
}

PT_DEV void stack8_store(const SceneDev& S, lds_int* stk, int j, uint2 e) {
    if (j < kStackLds8) {
        stk = stack_base(stk);
        stk[(2 * j) * kStkStride] = int(e.x);
        stk[(2 * j + 1) * kStkStride] = int(e.y);
    } else {  // rare: deep entries spill to this thread's global slab
        S.spill8[size_t(j - kStackLds8) * S.spill_stride + blockIdx.x * blockDim.x + threadIdx.x] = e;
    }
}

PT_DEV uint2 stack8_load(const SceneDev& S, const lds_int* stk, int j) {
    if (j < kStackLds8) {
        stk = const_cast<lds_int*>(stack_base(const_cast<lds_int*>(stk)));
        return make_uint2(uint32_t(stk[(2 * j) * kStkStride]), uint32_t(stk[(2 * j + 1) * kStkStride]));
    }
    return S.spill8[size_t(j - kStackLds8) * S.spill_stride + blockIdx.x * blockDim.x + threadIdx.x];
}

// The 80-B node as five 16-B words (pt_layout.h Bvh8Node).
struct Node8Words {
    uint4 w0, w1, w2, w3, w4;
};

// The first `n` nodes (the top levels: the builder emits breadth first) copied to LDS by the
// workgroup (node_cache_fill); visits there read LDS instead of issuing vector memory loads.
struct NodeCache {
    const uint4* lds;
    uint32_t n;
};

PT_DEV Node8Words load_node8(const SceneDev& S, uint32_t node) {
#if DXRPT_PIN_LOADS
    const uint4* N = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(S.nodes8) + size_t(node) * kNode8Stride);
    const Node8Words w{N[0], N[1], N[2], N[3], N[4]};
    // the leaf metadata (w1.zw) is otherwise loaded behind the leaf-hit branch: a second round trip
    asm volatile("" ::"v"(w.w0.x), "v"(w.w0.y), "v"(w.w0.z), "v"(w.w0.w), "v"(w.w1.x), "v"(w.w1.y), "v"(w.w1.z),
                 "v"(w.w1.w), "v"(w.w2.x), "v"(w.w2.y), "v"(w.w2.z), "v"(w.w2.w), "v"(w.w3.x), "v"(w.w3.y),
                 "v"(w.w3.z), "v"(w.w3.w), "v"(w.w4.x), "v"(w.w4.y), "v"(w.w4.z), "v"(w.w4.w));
    return w;
#else
    const uint4* N = reinterpret_cast<const uint4*>(S.nodes8);
    return Node8Words{N[node * kNode8Words + 0], N[node * kNode8Words + 1], N[node * kNode8Words + 2], N[node * kNode8Words + 3], N[node * kNode8Words + 4]};
#endif
}

PT_DEV Node8Words load_node8(const SceneDev& S, const NodeCache& nc, uint32_t node) {
    if (node < nc.n) {
        const uint4* L = nc.lds;
        return Node8Words{L[node * kNode8Words + 0], L[node * kNode8Words + 1], L[node * kNode8Words + 2], L[node * kNode8Words + 3], L[node * kNode8Words + 4]};
    }
    return load_node8(S, node);
}

// Copies the top `n` nodes into `lds` (all threads of the workgroup; ends with a barrier).
PT_DEV NodeCache node_cache_fill(const SceneDev& S, uint4* lds, uint32_t n) {
    const uint4* N = reinterpret_cast<const uint4*>(S.nodes8);
    for (uint32_t j = threadIdx.x; j < n * kNode8Words; j += blockDim.x) lds[j] = N[j];
    __syncthreads();
    return NodeCache{lds, n};
}

// Slot mask of the node's children whose quantised box the ray enters within [tmin, tmx].
PT_DEV uint32_t box8_hits(const Ray8& R, const Node8Words& W, float tmx) {
    const uint4 w0 = W.w0, w2 = W.w2, w3 = W.w3, w4 = W.w4;
    const float ax = __uint_as_float((w0.w & 0xFFu) << 23) * R.inv.x;
    const float ay = __uint_as_float(((w0.w >> 8) & 0xFFu) << 23) * R.inv.y;
    const float az = __uint_as_float(((w0.w >> 16) & 0xFFu) << 23) * R.inv.z;
    const float bx = __builtin_fmaf(__uint_as_float(w0.x), R.inv.x, -R.ood.x);
    const float by = __builtin_fmaf(__uint_as_float(w0.y), R.inv.y, -R.ood.y);
    const float bz = __builtin_fmaf(__uint_as_float(w0.z), R.inv.z, -R.ood.z);
    // Near/far quantised planes per axis chosen once per node from the ray octant (Ylitie et al. 2017,
    // sec. 3.2): with inv >= 0 the near plane of every child is qlo, else qhi, so this equals the
    // min/max of the two slab distances.  Words: w2 = (qlo_x 0-3, 4-7, qlo_y 0-3, 4-7),
    // w3 = (qlo_z .., qhi_x ..), w4 = (qhi_y .., qhi_z ..).
    const bool sxn = (R.oct & 4u) != 0u, syn = (R.oct & 2u) != 0u, szn = (R.oct & 1u) != 0u;
    const uint32_t nx0 = sxn ? w3.z : w2.x, nx1 = sxn ? w3.w : w2.y, fx0 = sxn ? w2.x : w3.z, fx1 = sxn ? w2.y : w3.w;
    const uint32_t ny0 = syn ? w4.x : w2.z, ny1 = syn ? w4.y : w2.w, fy0 = syn ? w2.z : w4.x, fy1 = syn ? w2.w : w4.y;
    const uint32_t nz0 = szn ? w4.z : w3.x, nz1 = szn ? w4.w : w3.y, fz0 = szn ? w3.x : w4.z, fz1 = szn ? w3.y : w4.w;
    uint32_t hm = 0;  // hit children, slot space
    // near and far plane of one axis in one packed FMA (v_pk_fma_f32): (qn, qf) * (a, a) + (b, b)
    const f2v A2x = {ax, ax}, A2y = {ay, ay}, A2z = {az, az};
    const f2v B2x = {bx, bx}, B2y = {by, by}, B2z = {bz, bz};
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const uint32_t sh = 8u * uint32_t(c & 3);
        const f2v qx = {float(((c < 4 ? nx0 : nx1) >> sh) & 0xFFu), float(((c < 4 ? fx0 : fx1) >> sh) & 0xFFu)};
        const f2v qy = {float(((c < 4 ? ny0 : ny1) >> sh) & 0xFFu), float(((c < 4 ? fy0 : fy1) >> sh) & 0xFFu)};
        const f2v qz = {float(((c < 4 ? nz0 : nz1) >> sh) & 0xFFu), float(((c < 4 ? fz0 : fz1) >> sh) & 0xFFu)};
        const f2v tx = __builtin_elementwise_fma(qx, A2x, B2x);
        const f2v ty = __builtin_elementwise_fma(qy, A2y, B2y);
        const f2v tz = __builtin_elementwise_fma(qz, A2z, B2z);
        const float tn = fmaxf(fmaxf(tx.x, ty.x), fmaxf(tz.x, R.tmin));
        const float tf = fminf(fminf(tx.y, ty.y), fminf(tz.y, tmx));
        // empty slots carry inverted boxes (qlo 255, qhi 0: never entered) and meta 0 (no triangles)
        hm |= uint32_t(tn <= tf) << c;
    }
    return hm;
}

// Node visit on already-loaded words (lets the caller issue the next node's loads early).
template <bool kCount>
PT_DEV bool trav8_node_w(const SceneDev& S, const Ray8& R, const Node8Words& W, uint32_t& node, int& sp, lds_int* stk,
                         uint2& tos, const HitRec& h, uint32_t& tbase, uint32_t& tbits, uint32_t& nvisit) {
    if (kCount) ++nvisit;
    const uint4 w0 = W.w0, w1 = W.w1;
    const uint32_t hm = box8_hits(R, W, h.t);  // hit children, slot space
    const uint32_t imask = w0.w >> 24;
    // internal hits to key space (bit slot ^ oct): three conditional bit-group swaps
    uint32_t ihits = hm & imask;
    if (R.oct & 1u) ihits = ((ihits & 0x55u) << 1) | ((ihits >> 1) & 0x55u);
    if (R.oct & 2u) ihits = ((ihits & 0x33u) << 2) | ((ihits >> 2) & 0x33u);
    if (R.oct & 4u) ihits = ((ihits & 0x0Fu) << 4) | ((ihits >> 4) & 0x0Fu);
    // leaf hits -> triangle bits ((count << 5) | offset per leaf slot)
    uint32_t thits = 0;
    uint32_t lh = hm & ~imask;
    const unsigned long long meta = (static_cast<unsigned long long>(w1.w) << 32) | w1.z;
    while (lh) {
        const uint32_t c = uint32_t(__builtin_ctz(lh));
        lh &= lh - 1u;
        const uint32_t m = uint32_t(meta >> (8u * c)) & 0xFFu;
        thits |= ((1u << (m >> 5)) - 1u) << (m & 31u);
    }
    tbase = w1.y;
    tbits = thits;
    uint32_t gbase = w1.x;
    uint32_t gword = (ihits << 24) | imask;
    while (true) {
        if (gword >> 24) {
            const uint32_t k = 31u - uint32_t(__builtin_clz(gword));
            gword &= ~(1u << k);
            const uint32_t slot = (k - 24u) ^ R.oct;
            node = gbase + uint32_t(__builtin_popcount(gword & 0xFFu & ((1u << slot) - 1u)));
            if (gword >> 24) {  // push the rest of the group
                if (sp > 0) stack8_store(S, stk, sp - 1, tos);
                tos = make_uint2(gbase, gword);
                ++sp;
            }
            return true;
        }
        if (sp == 0) return false;
        gbase = tos.x;  // pop
        gword = tos.y;
        if (--sp > 0) tos = stack8_load(S, stk, sp - 1);
    }
}

template <bool kCount>
PT_DEV bool trav8_node(const SceneDev& S, const Ray8& R, uint32_t& node, int& sp, lds_int* stk, uint2& tos, const HitRec& h,
                       uint32_t& tbase, uint32_t& tbits, uint32_t& nvisit, const NodeCache& nc = NodeCache{nullptr, 0u}) {
    return trav8_node_w<kCount>(S, R, load_node8(S, nc, node), node, sp, stk, tos, h, tbase, tbits, nvisit);
}

// Tests the pending triangle group.  Returns true when an any-hit ray found an occluder.
template <bool kAnyHit, bool kCount>
PT_DEV bool trav8_tris(const SceneDev& S, const Ray8& R, uint32_t tbase, uint32_t tbits, HitRec& h, uint32_t& ntest) {
    while (tbits) {
        const uint32_t b = uint32_t(__builtin_ctz(tbits));
        tbits &= tbits - 1u;
        if (kCount) ++ntest;
        if (test_triangle<kAnyHit>(S, tbase + b, R.o, R.d, R.tmin, R.tmax, R.alpha, h)) return true;
    }
    return false;
}

// Tests the pending group two records at a time: both records are loaded before either test, so a
// lane pays one memory round trip per pair.  Tests still run in bit order (same results).
template <bool kAnyHit, bool kCount>
PT_DEV bool trav8_tris2(const SceneDev& S, const Ray8& R, uint32_t tbase, uint32_t tbits, HitRec& h, uint32_t& ntest) {
    while (tbits) {
        const uint32_t b0 = uint32_t(__builtin_ctz(tbits));
        tbits &= tbits - 1u;
        const bool two = tbits != 0u;
        const uint32_t b1 = two ? uint32_t(__builtin_ctz(tbits)) : b0;
        tbits &= tbits - 1u;
        const TriRec ra = load_tri_raw(S, tbase + b0);
        const TriRec rb = load_tri_raw(S, tbase + b1);
        pin_tri(ra);
        pin_tri(rb);
        if (kCount) ntest += two ? 2u : 1u;
        if (test_tri_rec<kAnyHit>(S, ra, R.o, R.d, R.tmin, R.tmax, R.alpha, h)) return true;
        if (two && test_tri_rec<kAnyHit>(S, rb, R.o, R.d, R.tmin, R.tmax, R.alpha, h)) return true;
    }
    return false;
}

// Traversal with the memory round trips overlapped (kPipe bit 0: triangle pairs, bit 1: the next
// node's words are loaded right after its address is known, before the current node's triangle
// tests).  Visit order, tests and results are those of traverse8.
template <bool kAnyHit, bool kCount, int kPipe>
PT_DEV bool traverse8_pipe(const SceneDev& S, f3 o, f3 d, float tmin, float tmax, bool alpha, lds_int* stk, HitRec& h,
                           uint32_t& nvisit, uint32_t& ntest, const NodeCache& nc) {
    Ray8 R;
    ray8_init(R, o, d, tmin, tmax, alpha, h);
    uint32_t node = 0;
    int sp = 0;
    uint2 tos = make_uint2(0u, 0u);
    Node8Words w = load_node8(S, nc, 0);
    while (true) {
        uint32_t tbase = 0, tbits = 0;
        const bool more = trav8_node_w<kCount>(S, R, w, node, sp, stk, tos, h, tbase, tbits, nvisit);
        if (kPipe & 2) w = load_node8(S, nc, node);
        if (tbits) {
            const bool done = (kPipe & 1) ? trav8_tris2<kAnyHit, kCount>(S, R, tbase, tbits, h, ntest)
                                          : trav8_tris<kAnyHit, kCount>(S, R, tbase, tbits, h, ntest);
            if (done) return true;
        }
        if (!more) break;
        if (!(kPipe & 2)) w = load_node8(S, nc, node);
    }
    return h.tri != kMiss;
}

// ---- wave-coherent ("packet") BVH8 traversal ------------------------------------------------------
// The 64 rays of a wave walk ONE node sequence: a child is entered when any live lane's ray enters its
// box (each lane tests with its own ray and its own closest t), leaf triangles hit by any lane are
// tested by every live lane.  Node and triangle addresses are therefore wave-uniform and are fetched
// with scalar loads (constant address space -> s_load through the scalar cache), so the traversal
// issues no vector memory instructions at all; the vector memory pipeline (TA/TD), which bounds the
// per-lane traversal, is left to the shading passes.  The group stack is wave-uniform too: entry j
// lives in lane j of two VGPRs (push = v_cndmask, pop = v_readlane), no LDS.
// Each lane tests a superset of the leaves its own traversal would test, and closest hit is the
// minimum (t, triangle id) over tested triangles while any-hit is a boolean over them, so the results
// are those of traverse8 bit for bit.  Pays off for coherent rays (primary rays of an 8x8 pixel block,
// their sun shadow rays); incoherent rays visit the union of their paths.
typedef unsigned int U32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(4))) const U32x4 ConstU4;

PT_DEV uint4 u4(U32x4 v) { return make_uint4(v.x, v.y, v.z, v.w); }
PT_DEV float4 f4(U32x4 v) {
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}

PT_DEV Node8Words load_node8_uniform(const SceneDev& S, uint32_t node) {
    ConstU4* N = (ConstU4*)(S.nodes8);  // NOLINT: generic -> constant address space
    const uint32_t b = node * kNode8Words;
    return Node8Words{u4(N[b + 0]), u4(N[b + 1]), u4(N[b + 2]), u4(N[b + 3]), u4(N[b + 4])};
}

PT_DEV TriRec load_tri_uniform(const SceneDev& S, uint32_t rec) {
    ConstU4* T = (ConstU4*)(S.tris);  // NOLINT
    const uint32_t b = rec * 3u;
    return TriRec{f4(T[b + 0]), f4(T[b + 1]), f4(T[b + 2])};
}

// A triangle's opacity map and vertex UVs when the triangle is wave-uniform (packet traversal):
// scalar loads of GeoShade::opacity and the three MeshVertex::UV of its vertex record.
struct AlphaInputs {
    GeoTex op;
    float2 uv0, uv1, uv2;
    PT_DEV float u(float b1, float b2) const { return bary_lerp(uv0.x, uv1.x, uv2.x, (1.0f - b1) - b2, b1, b2); }
    PT_DEV float v(float b1, float b2) const { return bary_lerp(uv0.y, uv1.y, uv2.y, (1.0f - b1) - b2, b1, b2); }
};
typedef unsigned int U32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(4))) const U32x2 ConstU2;

PT_DEV AlphaInputs alpha_inputs_uniform(const SceneDev& S, uint32_t geom, uint32_t gtri) {
    ConstU2* G = (ConstU2*)(S.geoshade);   // NOLINT: 6 GeoTex per geometry, opacity last
    ConstU2* V = (ConstU2*)(S.tri_verts);  // NOLINT: 3 x 64-B MeshVertex per triangle, UV = 8-B word 3
    const U32x2 op = G[geom * 6u + 5u];
    const U32x2 a = V[gtri * 24u + 3u], b = V[gtri * 24u + 11u], c = V[gtri * 24u + 19u];
    AlphaInputs ai;
    ai.op = GeoTex{op.x, op.y};
    ai.uv0 = make_float2(__uint_as_float(a.x), __uint_as_float(a.y));
    ai.uv1 = make_float2(__uint_as_float(b.x), __uint_as_float(b.y));
    ai.uv2 = make_float2(__uint_as_float(c.x), __uint_as_float(c.y));
    return ai;
}

PT_DEV uint32_t wave_or8(uint32_t m) {
    uint32_t u = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) u |= uint32_t(__ballot((m >> c) & 1u) != 0ull) << c;
    return u;
}

// `live`: this lane holds a ray (lanes past the end of the queue join with live = false).  Returns
// this lane's result like traverse8 (h.tri != kMiss: hit / occluded).
// Adaptive mode (switch_pct > 0): the wave tracks the fraction of its live lanes that enter some child
// of each visited node; once that fraction, over all visits so far (>= kSwitchMinVisits), falls below
// switch_pct percent, the packet is incoherent and the wave continues one ray per lane (traverse8_from
// from the root, keeping each lane's best hit as its bound: it tests every triangle the lane's own
// traversal would, so the result is still that of traverse8).
constexpr uint32_t kSwitchMinVisits = 4;

// DXRPT_PACKET_PREFETCH: the packet traversal selects its next node right after the box test and loads
// it while the current node's leaf triangles are tested (same visit order and bounds, same results).
// DXRPT_PACKET_VCHUNK: the packet traversal loads a node's pending triangle records as 64-dword vector
// chunks (lane j: dword j) and reads them with readlane, instead of scalar loads of one record or pair
// per round trip (the tris buffer is padded by six records so a chunk never reads past it).
#ifndef DXRPT_PACKET_VCHUNK
#define DXRPT_PACKET_VCHUNK 0
#endif
// DXRPT_TRAV_PRIO: wave priority (s_setprio) while a wave runs a per-lane traversal (0: off).
#ifndef DXRPT_TRAV_PRIO
#define DXRPT_TRAV_PRIO 0
#endif
// DXRPT_ORDER_XCD: cost-ordered frames also deal runs of xcd_chunk consecutive order positions to the XCDs.
#ifndef DXRPT_ORDER_XCD
#define DXRPT_ORDER_XCD 0
#endif
#ifndef DXRPT_PACKET_PREFETCH
#define DXRPT_PACKET_PREFETCH 0
#endif

template <bool kAnyHit>
PT_DEV bool traverse8_from(const SceneDev& S, const Ray8& R, lds_int* stk, HitRec& h);

// kCount: node / triangle FETCHES are counted in *cnt (cnt[0] nodes, cnt[1] triangles) by the wave's
// first live lane -- a packet fetches each node and triangle once per wave (scalar loads).
// kPair: leaf triangles two at a time (both records, both geometric tests against the bound at the
// step's start -- a superset of the sequential candidates --, both opacity taps in flight, acceptance in
// order with the live bound: the hits of testing them one after the other, with one alpha round trip
// per pair).  Used by the path-group kernel, whose small frames end with alpha-tested foliage waves.
template <bool kAnyHit, bool kCount = false, bool kPair = false>
PT_DEV bool traverse8_packet(const SceneDev& S, f3 o, f3 d, float tmin, float tmax, bool alpha, bool live, HitRec& h,
                             uint32_t switch_pct = 0u, lds_int* stk = nullptr, uint32_t* cnt = nullptr) {
    Ray8 R;
    ray8_init(R, o, d, tmin, tmax, alpha, h);
    unsigned long long lv = __ballot(live);
    if (lv == 0ull) return false;
    uint32_t visits = 0, lanes_live = 0, lanes_useful = 0;  // wave-uniform coherence census
    // key order of the first live lane's octant for the whole wave (any order gives the same results)
    const uint32_t oct = uint32_t(__builtin_amdgcn_readlane(int(R.oct), __ffsll(static_cast<long long>(lv)) - 1));
    const uint32_t lane = uint32_t(__lane_id());
    const bool counter = kCount && lane == uint32_t(__ffsll(static_cast<long long>(lv)) - 1);
    uint32_t sbase = 0, sword = 0;  // stack entry j in lane j
    uint32_t sp = 0;
    uint32_t node = 0;
#if DXRPT_PACKET_VCHUNK
    const bool full = __ballot(1) == ~0ull;  // every lane loads its chunk dword
#endif
#if DXRPT_PACKET_PREFETCH
    Node8Words W = load_node8_uniform(S, 0u);
#endif
    while (true) {
#if !DXRPT_PACKET_PREFETCH
        const Node8Words W = load_node8_uniform(S, node);
#endif
        if (counter) ++cnt[0];
        const uint32_t hm = live ? box8_hits(R, W, h.t) : 0u;
        const uint32_t um = wave_or8(hm);
        if (switch_pct) {
            ++visits;
            lanes_live += uint32_t(__popcll(__ballot(live)));
            lanes_useful += uint32_t(__popcll(__ballot(hm != 0u)));
            if (visits >= kSwitchMinVisits && lanes_useful * 100u < lanes_live * switch_pct) {
                if (live) traverse8_from<kAnyHit>(S, R, stk, h);
                return h.tri != kMiss;
            }
        }
        const uint32_t imask = W.w0.w >> 24;
        // leaf triangles hit by any lane: (count << 5) | offset per leaf slot
        uint32_t tbits = 0;
        uint32_t lh = um & ~imask;
        const unsigned long long meta = (static_cast<unsigned long long>(W.w1.w) << 32) | W.w1.z;
        while (lh) {
            const uint32_t c = uint32_t(__builtin_ctz(lh));
            lh &= lh - 1u;
            const uint32_t m = uint32_t(meta >> (8u * c)) & 0xFFu;
            tbits |= ((1u << (m >> 5)) - 1u) << (m & 31u);
        }
        const uint32_t tbase = W.w1.y;
#if DXRPT_PACKET_VCHUNK
        if (full && tbits) {
            // the pending records (contiguous from tbase) in 64-dword chunks, one vector load per chunk:
            // lane j holds dword j; each record is then read lane by lane (readlane) -- one memory round
            // trip for up to five records instead of one per scalar-loaded pair
            const uint32_t* TD = reinterpret_cast<const uint32_t*>(S.tris);
            uint32_t lo = tbase + uint32_t(__builtin_ctz(tbits));
            uint32_t chunk = TD[size_t(lo) * 12u + lane];
            while (tbits) {
                const uint32_t b = uint32_t(__builtin_ctz(tbits));
                tbits &= tbits - 1u;
                const uint32_t rec = tbase + b;
                uint32_t off = (rec - lo) * 12u;
                if (off + 12u > 64u) {
                    lo = rec;
                    chunk = TD[size_t(lo) * 12u + lane];
                    off = 0u;
                }
                auto rl = [&](uint32_t k) { return __uint_as_float(uint32_t(__builtin_amdgcn_readlane(int(chunk), int(off + k)))); };
                TriRec r;
                r.p0 = make_float4(rl(0), rl(1), rl(2), rl(3));
                r.p1 = make_float4(rl(4), rl(5), rl(6), rl(7));
                r.p2 = make_float4(rl(8), rl(9), rl(10), rl(11));
                if (counter) ++cnt[1];
                if (live && test_tri_rec<kAnyHit>(S, r, R.o, R.d, R.tmin, R.tmax, R.alpha, h)) live = false;  // occluded
            }
        }
#endif
#if DXRPT_PACKET_PREFETCH
        uint32_t ihits = um & imask;
        if (oct & 1u) ihits = ((ihits & 0x55u) << 1) | ((ihits >> 1) & 0x55u);
        if (oct & 2u) ihits = ((ihits & 0x33u) << 2) | ((ihits >> 2) & 0x33u);
        if (oct & 4u) ihits = ((ihits & 0x0Fu) << 4) | ((ihits >> 4) & 0x0Fu);
        uint32_t gbase = W.w1.x;
        uint32_t gword = (ihits << 24) | imask;
        bool found = false;
        while (true) {
            if (gword >> 24) {
                const uint32_t k = 31u - uint32_t(__builtin_clz(gword));
                gword &= ~(1u << k);
                const uint32_t slot = (k - 24u) ^ oct;
                node = gbase + uint32_t(__builtin_popcount(gword & 0xFFu & ((1u << slot) - 1u)));
                if (gword >> 24) {  // push the rest of the group
                    if (lane == sp) {
                        sbase = gbase;
                        sword = gword;
                    }
                    ++sp;
                }
                found = true;
                break;
            }
            if (sp == 0u) break;
            --sp;
            gbase = uint32_t(__builtin_amdgcn_readlane(int(sbase), int(sp)));
            gword = uint32_t(__builtin_amdgcn_readlane(int(sword), int(sp)));
        }
        // the next node is known before this node's triangles are tested (their hits only tighten the
        // bound its box test will use): its words are in flight while they are
        Node8Words Wn = W;
        if (found) Wn = load_node8_uniform(S, node);
#endif
        while (kPair && tbits) {
            const uint32_t b0 = uint32_t(__builtin_ctz(tbits));
            tbits &= tbits - 1u;
            const bool two = tbits != 0u;
            const uint32_t b1 = two ? uint32_t(__builtin_ctz(tbits)) : b0;
            if (two) tbits &= tbits - 1u;
            const TriRec r0 = load_tri_uniform(S, tbase + b0), r1 = load_tri_uniform(S, tbase + b1);
            if (counter) cnt[1] += two ? 2u : 1u;
            float t0 = 0.0f, u0 = 0.0f, v0 = 0.0f, t1 = 0.0f, u1 = 0.0f, v1 = 0.0f;
            const bool c0 = live && tri_candidate<kAnyHit>(r0, R.o, R.d, R.tmin, R.tmax, h, t0, u0, v0);
            const bool c1 = two && live && tri_candidate<kAnyHit>(r1, R.o, R.d, R.tmin, R.tmax, h, t1, u1, v1);
            // AnyHitShader (RayTrace.hlsl:485-507) for candidates on alpha-tested geometry
            const bool n0 = c0 && R.alpha && !(fbits(r0.p2.w) & kTriOpaque);
            const bool n1 = c1 && R.alpha && !(fbits(r1.p2.w) & kTriOpaque);
            float o0 = 1.0f, o1 = 1.0f;
            const bool any0 = __ballot(n0) != 0ull, any1 = __ballot(n1) != 0ull;
            if (any0 || any1) {
                OpacityTap q0{}, q1{};
                bool m0 = false, m1 = false;
                // lanes whose micromap cell decides skip the tap (o = 0: reject; 1: accept)
                if (any0) {
                    const AlphaInputs ai = alpha_inputs_uniform(S, fbits(r0.p1.w), fbits(r0.p0.w));
                    const OmmProbe pr = omm_probe(S, fbits(r0.p2.w) >> 1, u0, v0);  // per lane, same round trip
                    const uint32_t vd = n0 && ai.op.whf != 0u ? omm_verdict(pr) : kOmmOpaque;
                    m0 = n0 && ai.op.whf != 0u && vd == kOmmUnknown;
                    if (vd == kOmmTransparent) o0 = 0.0f;
                    if (m0) q0 = opacity_issue(S, tex_desc(ai.op), ai.u(u0, v0), ai.v(u0, v0));
                }
                if (any1) {
                    const AlphaInputs ai = alpha_inputs_uniform(S, fbits(r1.p1.w), fbits(r1.p0.w));
                    const OmmProbe pr = omm_probe(S, fbits(r1.p2.w) >> 1, u1, v1);
                    const uint32_t vd = n1 && ai.op.whf != 0u ? omm_verdict(pr) : kOmmOpaque;
                    m1 = n1 && ai.op.whf != 0u && vd == kOmmUnknown;
                    if (vd == kOmmTransparent) o1 = 0.0f;
                    if (m1) q1 = opacity_issue(S, tex_desc(ai.op), ai.u(u1, v1), ai.v(u1, v1));
                }
                if (m0) o0 = opacity_finish(S, q0);
                if (m1) o1 = opacity_finish(S, q1);
            }
            if (c0 && !(o0 < 0.35f) && (kAnyHit || t0 < h.t || (t0 == h.t && fbits(r0.p0.w) < h.tri))) {
                h.t = t0;
                h.tri = fbits(r0.p0.w);
                h.b1 = u0;
                h.b2 = v0;
                h.geom = fbits(r0.p1.w);
                if (kAnyHit) live = false;  // occluded
            }
            if (c1 && live && !(o1 < 0.35f) && (kAnyHit || t1 < h.t || (t1 == h.t && fbits(r1.p0.w) < h.tri))) {
                h.t = t1;
                h.tri = fbits(r1.p0.w);
                h.b1 = u1;
                h.b2 = v1;
                h.geom = fbits(r1.p1.w);
                if (kAnyHit) live = false;
            }
        }
        while (!kPair && tbits) {
            const uint32_t b = uint32_t(__builtin_ctz(tbits));
            tbits &= tbits - 1u;
            const TriRec r = load_tri_uniform(S, tbase + b);
            if (counter) ++cnt[1];
            if (live && test_tri_rec<kAnyHit>(S, r, R.o, R.d, R.tmin, R.tmax, R.alpha, h)) live = false;  // occluded
        }
#if DXRPT_PACKET_PREFETCH
        if (kAnyHit && __ballot(live) == 0ull) break;
        if (!found) break;
        W = Wn;
#else
        if (kAnyHit && __ballot(live) == 0ull) break;
        uint32_t ihits = um & imask;
        if (oct & 1u) ihits = ((ihits & 0x55u) << 1) | ((ihits >> 1) & 0x55u);
        if (oct & 2u) ihits = ((ihits & 0x33u) << 2) | ((ihits >> 2) & 0x33u);
        if (oct & 4u) ihits = ((ihits & 0x0Fu) << 4) | ((ihits >> 4) & 0x0Fu);
        uint32_t gbase = W.w1.x;
        uint32_t gword = (ihits << 24) | imask;
        bool found = false;
        while (true) {
            if (gword >> 24) {
                const uint32_t k = 31u - uint32_t(__builtin_clz(gword));
                gword &= ~(1u << k);
                const uint32_t slot = (k - 24u) ^ oct;
                node = gbase + uint32_t(__builtin_popcount(gword & 0xFFu & ((1u << slot) - 1u)));
                if (gword >> 24) {  // push the rest of the group
                    if (lane == sp) {
                        sbase = gbase;
                        sword = gword;
                    }
                    ++sp;
                }
                found = true;
                break;
            }
            if (sp == 0u) break;
            --sp;
            gbase = uint32_t(__builtin_amdgcn_readlane(int(sbase), int(sp)));
            gword = uint32_t(__builtin_amdgcn_readlane(int(sword), int(sp)));
        }
        if (!found) break;
#endif
    }
    return h.tri != kMiss;
}

// One node visit and its triangles.  Returns true when the ray is finished: h.tri != kMiss means hit
// (closest) / occluded (any-hit).
template <bool kAnyHit, bool kCount>
PT_DEV bool trav8_step(const SceneDev& S, const Ray8& R, uint32_t& node, int& sp, lds_int* stk, uint2& tos, HitRec& h,
                       uint32_t& nvisit, uint32_t& ntest, const NodeCache& nc) {
    uint32_t tbase = 0, tbits = 0;
    const bool more = trav8_node<kCount>(S, R, node, sp, stk, tos, h, tbase, tbits, nvisit, nc);
    if (tbits && trav8_tris<kAnyHit, kCount>(S, R, tbase, tbits, h, ntest)) return true;
    return !more;
}

template <bool kAnyHit, bool kCount>
PT_DEV bool traverse8(const SceneDev& S, f3 o, f3 d, float tmin, float tmax, bool alpha, lds_int* stk, HitRec& h,
                      uint32_t& nvisit, uint32_t& ntest, const NodeCache& nc) {
    Ray8 R;
    ray8_init(R, o, d, tmin, tmax, alpha, h);
    uint32_t node = 0;
    int sp = 0;
    uint2 tos = make_uint2(0u, 0u);
#if DXRPT_TRAV_PRIO
    __builtin_amdgcn_s_setprio(DXRPT_TRAV_PRIO);  // traversing waves issue their next fetch first
#endif
    while (!trav8_step<kAnyHit, kCount>(S, R, node, sp, stk, tos, h, nvisit, ntest, nc)) {
    }
#if DXRPT_TRAV_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    return h.tri != kMiss;
}

// Per-lane traversal from the root with the lane's current best hit kept as the bound.
template <bool kAnyHit>
PT_DEV bool traverse8_from(const SceneDev& S, const Ray8& R, lds_int* stk, HitRec& h) {
    uint32_t node = 0, nv = 0, nt = 0;
    int sp = 0;
    uint2 tos = make_uint2(0u, 0u);
    while (!trav8_step<kAnyHit, false>(S, R, node, sp, stk, tos, h, nv, nt, NodeCache{nullptr, 0u})) {
    }
    return h.tri != kMiss;
}

// Two any-hit rays of one lane down ONE node sequence (DXRPT_SHADOW_PAIRS).  A vertex's sun and
// sky-visibility rays both start at the hit position (RayTrace.hlsl:241-244, 415-425), so they cross the
// same nodes around it; walked one after the other they fetch those nodes twice and chain two traversals'
// round trips.  Here a child is entered when either live ray enters its box (each ray tested against its
// own [tmin, tmax]) and every live ray tests each triangle of the visited leaves until it finds an
// occluder (then it drops out of the box tests).  An any-hit answer is whether some accepted hit lies in
// [tmin, tmax] among the triangles its own traversal (traverse8<true>) would test; the union visits a
// superset of those and tests them exactly, so each answer is that traversal's, for any two rays.
// live: bit 0 ray a, bit 1 ray b.  Returns the occluded bits.  kCount: node and triangle-record fetches
// (shared by both rays) into nvisit / ntest.
// The pair keeps each ray lean (origin, direction, inverse, interval, alpha flag): the box-test terms
// o * inv and the octant are recomputed per node visit -- the same products ray8_init forms, so the same
// box hits -- which keeps the pair inside the traversal's register budget.
struct RayLean {
    f3 o, d, inv;
    float tmin, tmax;
    bool alpha;
};

PT_DEV void ray_lean_init(RayLean& R, f3 o, f3 d, float tmin, float tmax, bool alpha) {
    R.o = o;
    R.d = d;
    R.inv = safe_inverse(d);
    R.tmin = tmin;
    R.tmax = tmax;
    R.alpha = alpha;
}

PT_DEV uint32_t lean_oct(const RayLean& R) {
    return (R.inv.x < 0.0f ? 4u : 0u) | (R.inv.y < 0.0f ? 2u : 0u) | (R.inv.z < 0.0f ? 1u : 0u);
}

PT_DEV uint32_t box8_hits_lean(const RayLean& L, const Node8Words& W) {
    Ray8 R;
    R.o = L.o;
    R.d = L.d;
    R.inv = L.inv;
    R.ood = mul(L.o, L.inv);
    R.tmin = L.tmin;
    R.tmax = L.tmax;
    R.oct = lean_oct(L);
    R.alpha = L.alpha;
    return box8_hits(R, W, L.tmax);
}

template <bool kCount>
PT_DEV uint32_t traverse8_anyhit2(const SceneDev& S, const RayLean& Ra, const RayLean& Rb, uint32_t live, lds_int* stk,
                                  uint32_t& nvisit, uint32_t& ntest) {
    uint32_t occ = 0;
    if (!live) return occ;
    const uint32_t oct = lean_oct((live & 1u) ? Ra : Rb);  // child order of the walk (any order: same answers)
    uint32_t node = 0;
    int sp = 0;
    uint2 tos = make_uint2(0u, 0u);
    while (true) {
        if (kCount) ++nvisit;
        const uint4* N = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(S.nodes8) + size_t(node) * kNode8Stride);
        const Node8Words W{N[0], N[1], N[2], N[3], N[4]};  // not pinned: the pair's registers are scarce
        uint32_t hm = 0;
        if (live & 1u) hm |= box8_hits_lean(Ra, W);
        if (live & 2u) hm |= box8_hits_lean(Rb, W);
        // the group logic of trav8_node_w on the union mask, keyed by `oct`
        const uint4 w0 = W.w0, w1 = W.w1;
        const uint32_t imask = w0.w >> 24;
        uint32_t ihits = hm & imask;
        if (oct & 1u) ihits = ((ihits & 0x55u) << 1) | ((ihits >> 1) & 0x55u);
        if (oct & 2u) ihits = ((ihits & 0x33u) << 2) | ((ihits >> 2) & 0x33u);
        if (oct & 4u) ihits = ((ihits & 0x0Fu) << 4) | ((ihits >> 4) & 0x0Fu);
        uint32_t tbits = 0;
        uint32_t lh = hm & ~imask;
        const unsigned long long meta = (static_cast<unsigned long long>(w1.w) << 32) | w1.z;
        while (lh) {
            const uint32_t c = uint32_t(__builtin_ctz(lh));
            lh &= lh - 1u;
            const uint32_t m = uint32_t(meta >> (8u * c)) & 0xFFu;
            tbits |= ((1u << (m >> 5)) - 1u) << (m & 31u);
        }
        const uint32_t tbase = w1.y;
        uint32_t gbase = w1.x;
        uint32_t gword = (ihits << 24) | imask;
        bool more = false;
        while (true) {
            if (gword >> 24) {
                const uint32_t k = 31u - uint32_t(__builtin_clz(gword));
                gword &= ~(1u << k);
                const uint32_t slot = (k - 24u) ^ oct;
                node = gbase + uint32_t(__builtin_popcount(gword & 0xFFu & ((1u << slot) - 1u)));
                if (gword >> 24) {
                    if (sp > 0) stack8_store(S, stk, sp - 1, tos);
                    tos = make_uint2(gbase, gword);
                    ++sp;
                }
                more = true;
                break;
            }
            if (sp == 0) break;
            gbase = tos.x;
            gword = tos.y;
            if (--sp > 0) tos = stack8_load(S, stk, sp - 1);
        }
        while (tbits) {
            const uint32_t b = uint32_t(__builtin_ctz(tbits));
            tbits &= tbits - 1u;
            if (kCount) ++ntest;
            const TriRec r = load_tri(S, tbase + b);
            // one inlined test for both rays (the ray's fields selected), not two copies of the alpha test
            uint32_t todo = live;
#pragma nounroll
            while (todo) {
                const uint32_t j = uint32_t(__builtin_ctz(todo));
                todo &= todo - 1u;
                const bool jb = j != 0u;
                const f3 o = jb ? Rb.o : Ra.o, d = jb ? Rb.d : Ra.d;
                HitRec h;
                if (test_tri_rec<true>(S, r, o, d, jb ? Rb.tmin : Ra.tmin, jb ? Rb.tmax : Ra.tmax, jb ? Rb.alpha : Ra.alpha, h)) {
                    live &= ~(1u << j);
                    occ |= 1u << j;
                }
            }
            if (!live) return occ;
        }
        if (!more) return occ;
    }
}

// DXRPT_SHADOW_PAIRS: a vertex's per-lane shadow rays go two slots at a time through traverse8_anyhit2
// -- 1: in the split schedule's tails, 2: there and in k_path / k_bake (trace_path); 0: one slot at a
// time through traverse8<true> everywhere.  Same answers either way.
#ifndef DXRPT_SHADOW_PAIRS
#define DXRPT_SHADOW_PAIRS 0
#endif

template <int W, bool kAnyHit, bool kCount, int kPipe = 0>
PT_DEV bool traverse(const SceneDev& S, f3 o, f3 d, float tmin, float tmax, bool alpha, lds_int* stk, HitRec& h,
                     uint32_t& nvisit, uint32_t& ntest, const NodeCache& nc = NodeCache{nullptr, 0u}) {
    h.t = tmax;
    h.tri = kMiss;
    h.b1 = h.b2 = 0.0f;
    h.geom = 0;
    if (W == 8) {
        if (kPipe & 3) return traverse8_pipe<kAnyHit, kCount, kPipe & 3>(S, o, d, tmin, tmax, alpha, stk, h, nvisit, ntest, nc);
        return traverse8<kAnyHit, kCount>(S, o, d, tmin, tmax, alpha, stk, h, nvisit, ntest, nc);
    }
    return traverse2<kAnyHit, kCount>(S, o, d, tmin, tmax, alpha, stk, h, nvisit, ntest);
}


// ---- kernels --------------------------------------------------------------------------------------
struct KArgs {
    SceneDev S;
    FrameBuffers F;
    FrameParams P;
};

PT_DEV const uint32_t* radiance_counts(const FrameBuffers& F, int depth) { return F.counters + uint32_t(depth) * kQueueShards; }
PT_DEV const uint32_t* shadow_counts(const FrameBuffers& F, int depth) {
    return F.counters + (kMaxDepthQueues + uint32_t(depth)) * kQueueShards;
}

// Item count of a sharded queue (wave-uniform: the counts are read with scalar loads).
PT_DEV uint32_t queue_total(const uint32_t* __restrict__ cnt) {
    uint32_t t = 0;
#pragma unroll
    for (uint32_t s = 0; s < kQueueShards; ++s) t += cnt[s];
    return t;
}

// Position of item i (< queue_total) of a sharded queue with shard capacity cap: the items of shard 0
// come first, then shard 1, ...  Any item order across lanes.
PT_DEV uint32_t queue_pos_any(const uint32_t* __restrict__ cnt, uint32_t cap, uint32_t i) {
    uint32_t pos = 0, base = 0;
#pragma unroll
    for (uint32_t s = 0; s < kQueueShards; ++s) {
        const uint32_t c = cnt[s];
        if (i >= base && i - base < c) pos = s * cap + (i - base);
        base += c;
    }
    return pos;
}

// Same, for lanes holding consecutive items (i grows with the lane id, so the first active lane holds
// the smallest): a wave-uniform scalar scan finds the shard of that item, then each lane steps
// forward over the (few) shards its own item lies past.
PT_DEV uint32_t queue_pos(const uint32_t* __restrict__ cnt, uint32_t cap, uint32_t i) {
    const uint32_t i0 = uint32_t(__builtin_amdgcn_readfirstlane(int(i)));
    uint32_t s = 0, base = 0;
    while (s + 1u < kQueueShards && base + cnt[s] <= i0) base += cnt[s++];
    while (s + 1u < kQueueShards && base + cnt[s] <= i) base += cnt[s++];
    return s * cap + (i - base);
}

// Append to shard `region_base + oct` (region_base wave-uniform, oct per lane in 0..7): the lanes of each
// octant form one group (three ballots), each group's first lane reserves the group's run with one atomic
// -- at most 8 lanes of one vector atomic per wave.  Returns this lane's position (meaningful where `want`).
PT_DEV uint32_t queue_append_oct(uint32_t* counters, uint32_t cap, bool want, uint32_t region_base, uint32_t oct) {
    const unsigned long long m = __ballot(want);
    const unsigned long long b4 = __ballot(want && (oct & 4u)), b2 = __ballot(want && (oct & 2u)),
                             b1 = __ballot(want && (oct & 1u));
    const unsigned long long same = m & ((oct & 4u) ? b4 : ~b4) & ((oct & 2u) ? b2 : ~b2) & ((oct & 1u) ? b1 : ~b1);
    const int lane = __lane_id();
    const int leader = want ? __ffsll(static_cast<long long>(same)) - 1 : lane;
    const uint32_t shard = region_base + oct;
    uint32_t base = 0;
    if (want && lane == leader) base = atomicAdd(&counters[shard], uint32_t(__popcll(same)));
    base = uint32_t(__shfl(int(base), leader));
    return shard * cap + base + uint32_t(__popcll(same & ((1ull << lane) - 1ull)));
}

// Wave-aggregated append to `shard` (wave-uniform) of a queue: one atomic per wave.  Returns the
// position of this lane's item (only meaningful where `want`).  Must be called by all active lanes.
PT_DEV uint32_t queue_append(uint32_t* counters, uint32_t cap, bool want, uint32_t shard) {
    const unsigned long long m = __ballot(want);
    const int lane = __lane_id();
    const int leader = __ffsll(static_cast<long long>(__ballot(1))) - 1;
    uint32_t base = 0;
    if (lane == leader && m != 0ull) base = atomicAdd(&counters[shard], uint32_t(__popcll(m)));
    base = __shfl(base, leader);
    return shard * cap + base + uint32_t(__popcll(m & ((1ull << lane) - 1ull)));
}

// ---- XCD-aware work mapping -----------------------------------------------------------------------
// MI355X dispatches workgroups round-robin over its 8 XCDs (block b -> XCD b % 8), and each XCD has its
// own 4 MB L2.  With FrameParams::xcd_map the queue of a pass is cut into 8 contiguous ranges of
// workgroups and XCD x runs range x (xcd_block), and producers append their rays to the shards of their
// own range (region_shard: shards 8r .. 8r+7 belong to range r), so range r of every queue holds the
// paths of one screen region (the primary queue is written in pixel-block order) and each XCD's L2
// works on the BVH nodes, triangles and texels of its region only.  The b % 8 placement is an
// affinity, not a guarantee (MI355X_MICROARCH.md): every mapping here is a bijection, so the placement
// only affects speed.  Without xcd_map: identity blocks, shard = wave % kQueueShards.
constexpr uint32_t kXcds = 8;
static_assert(kQueueShards == kXcds * 8u, "xcd_map: 8 shards per XCD range");

// Logical workgroup of this block when nb workgroups cover the pass; false: no work for this block.
PT_DEV bool xcd_block(bool xcd, uint32_t nb, uint32_t& lb) {
    const uint32_t b = blockIdx.x;
    if (!xcd) {
        lb = b;
        return b < nb;
    }
    const uint32_t x = b % kXcds, k = b / kXcds, q = nb / kXcds, r = nb % kXcds;
    if (k >= q + (x < r ? 1u : 0u)) return false;
    lb = x * q + min(x, r) + k;
    return true;
}

// Shard of logical wave lw of a pass over nw waves.
PT_DEV __host__ uint32_t region_shard(bool xcd, uint32_t lw, uint32_t nw) {
    return xcd ? (uint32_t((uint64_t(lw) * kXcds) / nw) * 8u + (lw & 7u)) : lw % kQueueShards;
}

// First queue item of this lane (i = lb * blockDim + threadIdx) for a pass over n items; false if the
// whole workgroup is past the end.  lw_out: the lane's logical wave.
PT_DEV bool xcd_item(bool xcd, uint32_t n, uint32_t& i, uint32_t& lw) {
    const uint32_t bd = blockDim.x;
    uint32_t lb;
    if (!xcd_block(xcd, (n + bd - 1u) / bd, lb)) return false;
    i = lb * bd + threadIdx.x;
    lw = i >> 6;
    return true;
}

// RaygenShader's ray (RayTrace.hlsl:92-126, SamplePoint 85-90) for path slot p: the tile and pixel of
// the slot, CMJ set-0 jitter, near/far-plane unprojection.
struct PrimaryRay {
    f3 start, dir;
    float length;
    uint32_t pixelIdx, accumIdx;
};

// Path slot p -> its pixel (x, y) and accumulation index: the tile by binary search over the prefix
// table, then the pixel inside the tile.
struct PathPixel {
    uint32_t x, y, accumIdx;
};
PT_DEV PathPixel path_pixel(const KArgs& A, uint32_t p) {
    uint32_t lo = 0, hi = A.P.num_tiles;
    while (hi - lo > 1u) {
        uint32_t mid = (lo + hi) >> 1;
        if (A.P.tile_prefix[mid] <= p) lo = mid; else hi = mid;
    }
    const dxrpt_tile tl = A.P.tiles[lo];
    const uint32_t local = p - A.P.tile_prefix[lo];
    uint32_t lx, ly;
    if ((tl.w & 7u) == 0u && (tl.h & 7u) == 0u) {
        // one wave = one 8x8 pixel block (blocks row-major in the tile): coherent primary rays.
        // Only the path-slot order changes; pixels, CMJ seeds and outputs do not.
        const uint32_t blk = local >> 6, in = local & 63u, bw = tl.w >> 3;
        lx = (blk % bw) * 8u + (in & 7u);
        ly = (blk / bw) * 8u + (in >> 3);
    } else {
        lx = local % tl.w;
        ly = local / tl.w;
    }
    return PathPixel{tl.x0 + lx, tl.y0 + ly, uint32_t(tl.accum_offset) + ly * tl.accum_pitch + lx};
}

PT_DEV PrimaryRay primary_ray(const KArgs& A, uint32_t p) {
    const PathPixel pp = path_pixel(A, p);
    const uint32_t x = pp.x, y = pp.y;
    const uint32_t pixelIdx = y * A.P.width + x;
    const uint32_t accumIdx = pp.accumIdx;

    const uint32_t nS = uint32_t(A.P.set.SqrtNumSamples);
    float sx, sy;
    sample_cmj2d(A.P.rtc.CurrSampleIdx, nS, nS, 0u * A.P.rtc.TotalNumPixels + pixelIdx, &sx, &sy);
    const float px = float(x) + sx, py = float(y) + sy;
    float ncx = px / (float(A.P.width) * 0.5f) - 1.0f;
    float ncy = py / (float(A.P.height) * 0.5f) - 1.0f;
    ncy *= -1.0f;
    const float* M = A.P.rtc.InvViewProjection;
    float s[4], e[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        s[j] = ((ncx * M[0 * 4 + j] + ncy * M[1 * 4 + j]) + 0.0f * M[2 * 4 + j]) + 1.0f * M[3 * 4 + j];
        e[j] = ((ncx * M[0 * 4 + j] + ncy * M[1 * 4 + j]) + 1.0f * M[2 * 4 + j]) + 1.0f * M[3 * 4 + j];
    }
    const f3 start = f3{s[0] / s[3], s[1] / s[3], s[2] / s[3]};
    const f3 end = f3{e[0] / e[3], e[1] / e[3], e[2] / e[3]};
    const f3 diff = sub(end, start);
    const f3 dir = normalize3(diff);
    const float rayLength = len3(diff);
    return PrimaryRay{start, dir, rayLength, pixelIdx, accumIdx};
}

// RaygenShader, RayTrace.hlsl:92-126 (+ SamplePoint 85-90).  Path slot p goes to the queue-1 position
// a wave-ordered append of its wave w = p / 64 would have produced (shard region_shard(w), waves of
// one shard in order); the shard counts are analytic.
__global__ __launch_bounds__(kBlock) void k_raygen(KArgs A) {
    const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t P = A.P.num_paths;
    const bool xcd = A.P.xcd_map != 0u;
    const uint32_t nw = (P + 63u) / 64u;
    if (p == 0) {
        uint32_t* cnt = A.F.counters + 1u * kQueueShards;
        for (uint32_t s = 0; s < kQueueShards; ++s) {
            uint32_t waves = 0;
            if (!xcd) {
                waves = s < nw ? (nw - 1u - s) / kQueueShards + 1u : 0u;
            } else {  // waves of region r = s / 8 are [ceil(r nw / 8), ceil((r + 1) nw / 8)), those = s mod 8
                const uint32_t r = s / 8u, sub = s % 8u;
                const uint32_t b = uint32_t((uint64_t(r) * nw + kXcds - 1u) / kXcds);
                const uint32_t e = uint32_t((uint64_t(r + 1u) * nw + kXcds - 1u) / kXcds);
                const uint32_t f = b + ((sub + 8u - b % 8u) % 8u);
                waves = f < e ? (e - 1u - f) / 8u + 1u : 0u;
            }
            uint32_t items = waves * 64u;
            if (nw > 0u && region_shard(xcd, nw - 1u, nw) == s) items -= nw * 64u - P;
            cnt[s] = items;
        }
    }
    if (p >= P) return;
    const PrimaryRay pr = primary_ray(A, p);
    const f3 start = pr.start, dir = pr.dir;
    const float rayLength = pr.length;
    const uint32_t pixelIdx = pr.pixelIdx, accumIdx = pr.accumIdx;
    const uint32_t w = p >> 6;
    uint32_t widx;  // index of wave w among the waves of its shard
    if (!xcd) {
        widx = w / kQueueShards;
    } else {
        const uint32_t r = uint32_t((uint64_t(w) * kXcds) / nw);
        const uint32_t b = uint32_t((uint64_t(r) * nw + kXcds - 1u) / kXcds);
        widx = (w - (b + ((w % 8u + 8u - b % 8u) % 8u))) / 8u;
    }
    const uint32_t pos = region_shard(xcd, w, nw) * A.F.cap_r + widx * 64u + (p & 63u);
    const RayQueue& Q = A.F.q[1];
    Q.org[pos] = make_float4(start.x, start.y, start.z, rayLength);
    Q.dir[pos] = make_float4(dir.x, dir.y, dir.z, bitsf(p));
    Q.thr[pos] = make_float4(1.0f, 1.0f, 1.0f, 0.0f);
    Q.rad[pos] = make_float4(0.0f, 0.0f, 0.0f, bitsf(0u));
    Q.pix[pos] = pixelIdx;
    A.F.ps_pix[p] = make_uint2(pixelIdx, accumIdx);
}

// kOcc > 0 asks the compiler for kOcc resident waves per SIMD (register budget 512 / kOcc).
// Workgroups of 64..256 threads (FrameParams::trace_block).
template <bool kCount, int W, int kOcc, int kPipe = 0>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kOcc > 0 ? kOcc : 1)))
void k_trace(KArgs A, int depth) {
    lut_fill(A.S);
    extern __shared__ int stack[];  // S.stack_ints per lane, lane-interleaved, then the node cache
    NodeCache nc{nullptr, 0u};
    if (W == 8 && !kCount && (kPipe & 4))  // LDS node cache: a separate instantiation, so that the
        // default kernels' node loads are plain global loads (no LDS/global pointer select -> flat loads)
        nc = node_cache_fill(A.S, reinterpret_cast<uint4*>(stack + A.S.stack_ints * blockDim.x), A.P.lds_nodes);
    const uint32_t* cnt = radiance_counts(A.F, depth);
    const uint32_t n = queue_total(cnt);
    uint32_t i, lw;
    if (!xcd_item(A.P.xcd_map != 0u, n, i, lw) || i >= n) return;
    const uint32_t pos = queue_pos(cnt, A.F.cap_r, i);
    const float4 o4 = A.F.q[depth & 1].org[pos];
    const float4 d4 = A.F.q[depth & 1].dir[pos];
    // Primary rays start at TMin 0 (RayTrace.hlsl:118); continuation rays at 1e-5 (:382).
    const float tmin = depth == 1 ? 0.0f : kRayTMin;
    // RAY_FLAG_FORCE_OPAQUE iff PathLength > MaxAnyHitPathLength (RayTrace.hlsl:132, 401)
    const bool alpha = depth <= A.P.set.MaxAnyHitPathLength;
    HitRec h;
    uint32_t nv = 0, nt = 0;
    traverse<W, false, kCount, kPipe>(A.S, ld3(o4), ld3(d4), tmin, o4.w, alpha, lane_stack(A.S, stack), h, nv, nt, nc);
    A.F.hit[pos] = make_float4(h.b1, h.b2, bitsf(h.tri), bitsf(h.geom));
    if (kCount) {
        atomicAdd(&A.P.trav[0], (unsigned long long)nv);
        atomicAdd(&A.P.trav[1], (unsigned long long)nt);
    }
}

// Shadow ray k of the vertex at queue position pos lives in slot [k * qsize + pos]; k_shadow multiplies
// its contribution by the visibility in place and k_resolve adds the slots, in k order, to the path's
// radiance (deterministic, no atomics on radiance).
PT_DEV void emit_shadow(const KArgs& A, uint32_t pos, uint32_t& n, f3 o, f3 d, float tmin, float tmax, f3 contrib,
                        bool forceOpaque) {
    const size_t s = size_t(n) * A.F.qsize + pos;
    A.F.sh_org[s] = make_float4(o.x, o.y, o.z, tmax);
    A.F.sh_dir[s] = make_float4(d.x, d.y, d.z, tmin);
    A.F.sh_con[s] = make_float4(contrib.x, contrib.y, contrib.z, bitsf(forceOpaque ? 1u : 0u));
    ++n;
}

PT_DEV bool nonzero3(f3 c) { return !(c.x == 0.0f && c.y == 0.0f && c.z == 0.0f); }

// A vertex's per-lane shadow rays in slots k0 .. nsh-1 (per-slot buffers at slot_p), two slots at a time
// through traverse8_anyhit2 (the wave walks the pairs together); contribution * visibility is added to
// rad in slot order -- the sum of the one-slot-at-a-time loop.  cnt: any-hit node / triangle fetches.
template <bool kCount>
PT_DEV void shadow_pairs(const KArgs& A, uint32_t slot_p, uint32_t k0, uint32_t nsh, lds_int* stk, float4& rad,
                         uint32_t& nvisit, uint32_t& ntest) {
    for (uint32_t k = k0; __ballot(k < nsh) != 0ull; k += 2u) {
        const uint32_t live = (k < nsh ? 1u : 0u) | (k + 1u < nsh ? 2u : 0u);
        const size_t sa = size_t(k) * A.F.qsize + slot_p, sb = sa + A.F.qsize;
        RayLean Ra, Rb;
        if (live & 1u) {
            const float4 o4 = A.F.sh_org[sa], d4 = A.F.sh_dir[sa];
            ray_lean_init(Ra, ld3(o4), ld3(d4), d4.w, o4.w, fbits(A.F.sh_con[sa].w) == 0u);
        }
        if (live & 2u) {
            const float4 o4 = A.F.sh_org[sb], d4 = A.F.sh_dir[sb];
            ray_lean_init(Rb, ld3(o4), ld3(d4), d4.w, o4.w, fbits(A.F.sh_con[sb].w) == 0u);
        }
        const uint32_t occ = traverse8_anyhit2<kCount>(A.S, Ra, Rb, live, stk, nvisit, ntest);
        if (live & 1u) {
            const float4 c4 = A.F.sh_con[sa];
            rad.x += (occ & 1u) ? c4.x * 0.0f : c4.x;
            rad.y += (occ & 1u) ? c4.y * 0.0f : c4.y;
            rad.z += (occ & 1u) ? c4.z * 0.0f : c4.z;
        }
        if (live & 2u) {
            const float4 c4 = A.F.sh_con[sb];
            rad.x += (occ & 2u) ? c4.x * 0.0f : c4.x;
            rad.y += (occ & 2u) ? c4.y * 0.0f : c4.y;
            rad.z += (occ & 2u) ? c4.z * 0.0f : c4.z;
        }
    }
}

// Shadow ray kinds, in the order a vertex emits them (RayTrace.hlsl:224-262, 265-313, 415-425).
constexpr int kShadowSun = 0, kShadowSpot = 1, kShadowSky = 2;

// One path vertex: MissShader (RayTrace.hlsl:509-530) or ClosestHitShader -> PathTrace (151-441) for the
// ray (inOrigin, inDir) of path depth `depth` with hit record `hit` (b1, b2, tri, geom).  Shadow rays
// go to emit(kind, origin, dir, tmin, tmax, pending contribution = pathThr * CalcLighting (or sky *
// throughput), force_opaque) in the reference's order (sun, spot lights, final sky visibility); the
// local radiance and the continuation come back in O.  Shared by k_shade (wavefront: emit queues the
// shadow ray) and k_path (megakernel: emit traces it at once).
struct VertexIn {
    f3 inOrigin, inDir, pathThr;
    float payloadRoughness;  // payload.Roughness (RayTrace.hlsl:70)
    bool payloadIsDiffuse;   // payload.IsDiffuse (RayTrace.hlsl:69)
    uint32_t pix;            // global pixel index (CMJ pattern)
    float4 hit;
};
struct VertexOut {
    f3 local = f3{0.0f, 0.0f, 0.0f};
    bool cont = false;
    f3 nextThr = f3{0.0f, 0.0f, 0.0f};
    f3 nextOrigin = f3{0.0f, 0.0f, 0.0f}, nextDir = f3{0.0f, 0.0f, 0.0f};
    float nextRoughness = 0.0f;
    bool nextIsDiffuse = false;
};

template <class Emit>
PT_DEV void path_vertex(const KArgs& A, int depth, const VertexIn& V, Emit&& emit, VertexOut& O) {
    const dxrpt_app_settings& set = A.P.set;
    const dxrpt_ray_trace_constants& rtc = A.P.rtc;
    const float4 hit = V.hit;
    const f3 pathThr = V.pathThr;
    const f3 inDir = V.inDir;
    const f3 inOrigin = V.inOrigin;
    const bool furnace = set.EnableWhiteFurnaceMode != 0;
    const uint32_t tri = fbits(hit.z);

    if (tri == kMiss) {
        // MissShader
        if (furnace) {
            O.local = f3{1.0f, 1.0f, 1.0f};
        } else {
            O.local = set.EnableSky ? sample_sky(A.S, inDir) : f3{0.0f, 0.0f, 0.0f};
            if (depth == 1) {
                float cosSunAngle = dot3(inDir, f3{rtc.SunDirectionWS[0], rtc.SunDirectionWS[1], rtc.SunDirectionWS[2]});
                if (cosSunAngle >= rtc.CosSunAngularRadius)
                    O.local = f3{rtc.SunRenderColor[0], rtc.SunRenderColor[1], rtc.SunRenderColor[2]};
            }
        }
    } else do {
        // PathTrace early outs (RayTrace.hlsl:153-158): local radiance 0, the path ends.
        if ((!set.EnableDiffuse && !set.EnableSpecular) || (!set.EnableDirect && !set.EnableIndirect)) break;
        if (depth > 1 && !set.EnableIndirect) break;
        const uint32_t geom = fbits(hit.w);
        const Surface surf = get_hit_surface(A.S, tri, hit.x, hit.y);
        const GeoShade mat = A.S.geoshade[geom];  // GetGeometryMaterial (RayTrace.hlsl:467-474), resolved
        const f3 T = surf.t, Bt = surf.b;
        f3 Nrow = surf.n;
        const f3 positionWS = surf.pos;
        f3 normalWS = surf.n;
        if (set.EnableNormalMaps) {
            Texel4 nm = sample_tex_desc(A.S, tex_desc(mat.normal), surf.u, surf.v);
            f3 nts;
            nts.x = nm.r * 2.0f - 1.0f;
            nts.y = nm.g * 2.0f - 1.0f;
            nts.z = sqrtf(1.0f - saturate(nts.x * nts.x + nts.y * nts.y));
            normalWS = normalize3(add(add(scl(T, nts.x), scl(Bt, nts.y)), scl(surf.n, nts.z)));
            Nrow = normalWS;
        }
        f3 baseColor = f3{1.0f, 1.0f, 1.0f};
        if (set.EnableAlbedoMaps && !furnace) {
            Texel4 a = sample_tex_desc(A.S, tex_desc(mat.albedo), surf.u, surf.v);
            baseColor = f3{a.r, a.g, a.b};
        }
        const float metallic = saturate((furnace ? 1.0f : sample_tex_desc(A.S, tex_desc(mat.metallic), surf.u, surf.v).r) * set.MetallicScale);
        const bool enableDiffuse = (set.EnableDiffuse && metallic < 1.0f) || furnace;
        const bool payloadIsDiffuse = V.payloadIsDiffuse;
        const bool enableSpecular =
            set.EnableSpecular && (set.EnableIndirectSpecular ? !(set.AvoidCausticPaths && payloadIsDiffuse) : (depth == 1));
        if (!enableDiffuse && !enableSpecular) break;
        const float sqrtRoughness = saturate((furnace ? 1.0f : sample_tex_desc(A.S, tex_desc(mat.roughness), surf.u, surf.v).r) * set.RoughnessScale);
        const float dsel = enableDiffuse ? 1.0f : 0.0f, ssel = enableSpecular ? 1.0f : 0.0f;
        const f3 diffuseAlbedo = scl(f3{lerpf(baseColor.x, 0.0f, metallic), lerpf(baseColor.y, 0.0f, metallic), lerpf(baseColor.z, 0.0f, metallic)}, dsel);
        const f3 specularAlbedo = scl(f3{lerpf(0.03f, baseColor.x, metallic), lerpf(0.03f, baseColor.y, metallic), lerpf(0.03f, baseColor.z, metallic)}, ssel);
        float roughness = sqrtRoughness * sqrtRoughness;
        if (set.ClampRoughness) roughness = fmaxf(roughness, V.payloadRoughness);
        f3 msEC = f3{1.0f, 1.0f, 1.0f};
        if (set.ApplyMultiscatteringEnergyCompensation) {
            const float Ess = ggx_env_brdf_scale(saturate(dot3(normalWS, neg(inDir))), sqrtRoughness);
            const float k = 1.0f / Ess - 1.0f;
            msEC = f3{1.0f + specularAlbedo.x * k, 1.0f + specularAlbedo.y * k, 1.0f + specularAlbedo.z * k};
        }
        if (!furnace) {
            Texel4 em = sample_tex_desc(A.S, tex_desc(mat.emissive), surf.u, surf.v);
            O.local = f3{em.r, em.g, em.b};
        }
        const bool directZero = (depth == 1 && !set.EnableDirect);  // RayTrace.hlsl:385-386
        const bool shadowOpaque = depth > set.MaxAnyHitPathLength;
        // Sun (RayTrace.hlsl:224-262)
        if (set.EnableSun && !furnace && !directZero) {
            const f3 D = f3{rtc.SunDirectionWS[0], rtc.SunDirectionWS[1], rtc.SunDirectionWS[2]};
            f3 sunDirection = D;
            if (set.SunAreaLightApproximation) {
                const f3 R = reflect3(inDir, normalWS);
                const float r = rtc.SinSunAngularRadius;
                const float dd = rtc.CosSunAngularRadius;
                const float DDotR = dot3(D, R);
                const f3 Sv = sub(R, scl(D, DDotR));
                sunDirection = DDotR < dd ? normalize3(add(scl(D, dd), scl(normalize3(Sv), r))) : R;
            }
            const f3 c = calc_lighting(normalWS, sunDirection, f3{rtc.SunIrradiance[0], rtc.SunIrradiance[1], rtc.SunIrradiance[2]},
                                       diffuseAlbedo, specularAlbedo, roughness, positionWS, inOrigin, msEC);
            if (nonzero3(c))
                emit(kShadowSun, positionWS, D, kRayTMin, kFP32Max, mul(pathThr, c), shadowOpaque);
        }
        // Spot lights (RayTrace.hlsl:265-313)
        if (set.RenderLights && !furnace && !directZero) {
            for (uint32_t l = 0; l < rtc.NumLights; ++l) {
                const dxrpt_spot_light sl = A.P.lights[l];
                const f3 lp = f3{sl.Position[0], sl.Position[1], sl.Position[2]};
                f3 surfaceToLight = sub(lp, positionWS);
                const float distanceToLight = len3(surfaceToLight);
                surfaceToLight = f3{surfaceToLight.x / distanceToLight, surfaceToLight.y / distanceToLight, surfaceToLight.z / distanceToLight};
                const float angleFactor = saturate(dot3(surfaceToLight, f3{sl.Direction[0], sl.Direction[1], sl.Direction[2]}));
                float angularAttenuation = smoothstepf(sl.AngularAttenuationY, sl.AngularAttenuationX, angleFactor);
                const float dn = distanceToLight / sl.Range;
                float falloff = saturate(1.0f - (dn * dn * dn * dn));
                falloff = (falloff * falloff) / (distanceToLight * distanceToLight + 1.0f);
                angularAttenuation *= falloff;
                if (angularAttenuation > 0.0f) {
                    const f3 intensity = scl(f3{sl.Intensity[0], sl.Intensity[1], sl.Intensity[2]}, angularAttenuation);
                    const f3 c = calc_lighting(normalWS, surfaceToLight, intensity, diffuseAlbedo, specularAlbedo, roughness,
                                               positionWS, inOrigin, msEC);
                    if (nonzero3(c))
                        emit(kShadowSpot, add(positionWS, scl(normalWS, 0.01f)), surfaceToLight, kSpotShadowNearClip,
                                    distanceToLight - kSpotShadowNearClip, mul(pathThr, c), shadowOpaque);
                }
            }
        }
        if (directZero) O.local = f3{0.0f, 0.0f, 0.0f};
        // BRDF importance sampling (RayTrace.hlsl:315-376); sample set = PathLength
        float bx, by;
        sample_cmj2d(rtc.CurrSampleIdx, uint32_t(set.SqrtNumSamples), uint32_t(set.SqrtNumSamples),
                     uint32_t(depth) * rtc.TotalNumPixels + V.pix, &bx, &by);
        f3 throughput, rayDirTS;
        float selector = bx;
        if (!enableSpecular) selector = 0.0f;
        else if (!enableDiffuse) selector = 1.0f;
        if (selector < 0.5f) {
            if (enableSpecular) bx *= 2.0f;
            rayDirTS = sample_cosine_hemisphere(bx, by);
            throughput = diffuseAlbedo;
        } else {
            if (enableDiffuse) bx = (bx - 0.5f) * 2.0f;
            const f3 inTS = normalize3(f3{dot3(inDir, T), dot3(inDir, Bt), dot3(inDir, Nrow)});
            const f3 mTS = sample_ggx_visible_normal(neg(inTS), roughness, roughness, bx, by);
            const f3 sampleDirTS = reflect3(inTS, mTS);
            const f3 F = furnace ? f3{1.0f, 1.0f, 1.0f} : fresnel(specularAlbedo, mTS, sampleDirTS);
            const float a2 = roughness * roughness;
            const float G1 = smith_ggx_masking(-inTS.z, a2);
            const float G2 = smith_ggx_masking_shadowing(sampleDirTS.z, -inTS.z, a2);
            throughput = scl(F, G2 / G1);
            rayDirTS = sampleDirTS;
            if (set.ApplyMultiscatteringEnergyCompensation) {
                // dot(normalTS, -incomingRayDirWS): the reference mixes spaces here (RayTrace.hlsl:361)
                const float Ess = ggx_env_brdf_scale(saturate(-inDir.z), sqrtRoughness);
                const float k = 1.0f / Ess - 1.0f;
                throughput = mul(throughput, f3{1.0f + specularAlbedo.x * k, 1.0f + specularAlbedo.y * k, 1.0f + specularAlbedo.z * k});
            }
        }
        const f3 rayDirWS = normalize3(add(add(scl(T, rayDirTS.x), scl(Bt, rayDirTS.y)), scl(Nrow, rayDirTS.z)));
        if (enableDiffuse && enableSpecular) throughput = scl(throughput, 2.0f);
        if (set.EnableIndirect && (depth + 1 < set.MaxPathLength) && !furnace) {
            O.cont = true;
            O.nextThr = mul(pathThr, throughput);
            O.nextOrigin = positionWS;
            O.nextDir = rayDirWS;
            O.nextRoughness = roughness;
            O.nextIsDiffuse = selector < 0.5f;
        } else if (furnace) {
            O.local = throughput;  // RayTrace.hlsl:427-430 (visibility unused)
        } else {
            const f3 sky = set.EnableSky ? sample_sky(A.S, rayDirWS) : f3{0.0f, 0.0f, 0.0f};
            const f3 c = mul(sky, throughput);
            if (nonzero3(c))
                emit(kShadowSky, positionWS, rayDirWS, kRayTMin, kFP32Max, mul(pathThr, c),
                            depth + 1 > set.MaxAnyHitPathLength);
        }
    } while (false);
}

// MissShader (RayTrace.hlsl:509-530) and ClosestHitShader -> PathTrace (151-441).
// kOcc > 0: register budget for kOcc waves per SIMD; workgroups of FrameParams::shade_block threads.
template <int kOcc>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kOcc > 0 ? kOcc : 1)))
void k_shade(KArgs A, int depth) {
    lut_fill(A.S);
    const uint32_t* cnt = radiance_counts(A.F, depth);
    const uint32_t nq = queue_total(cnt);
    const bool xcd = A.P.xcd_map != 0u;
    uint32_t i, lw;
    if (!xcd_item(xcd, nq, i, lw) || i >= nq) return;
    // the wave's shard in the queues it produces (all lanes of a wave share lw)
    const uint32_t shard = region_shard(xcd, lw, (nq + 63u) / 64u);
    const uint32_t pos = queue_pos(cnt, A.F.cap_r, i);
    const RayQueue& Q = A.F.q[depth & 1];
    const float4 o4 = Q.org[pos];
    const float4 d4 = Q.dir[pos];
    const uint32_t pathSlot = fbits(d4.w);
    const float4 thr4 = Q.thr[pos];
    float4 rad4 = Q.rad[pos];
    const f3 pathThr = ld3(thr4);
    uint32_t nsh = 0;
    VertexIn V;
    V.inOrigin = ld3(o4);
    V.inDir = ld3(d4);
    V.pathThr = pathThr;
    V.payloadRoughness = thr4.w;
    V.payloadIsDiffuse = (fbits(rad4.w) & 1u) != 0u;
    V.pix = Q.pix[pos];
    V.hit = A.F.hit[pos];
    VertexOut O;
    path_vertex(A, depth, V, [&](int, f3 o, f3 d, float tmin, float tmax, f3 c, bool fo) {
        emit_shadow(A, pos, nsh, o, d, tmin, tmax, c, fo);
    }, O);
    const f3 local = O.local;
    const bool cont = O.cont;
    const f3 nextThr = O.nextThr, nextOrigin = O.nextOrigin, nextDir = O.nextDir;
    const float nextRoughness = O.nextRoughness;
    const bool nextIsDiffuse = O.nextIsDiffuse;

    // Always add (also when zero): keeps NaN/inf propagation identical to the recursive form.
    rad4.x += pathThr.x * local.x;
    rad4.y += pathThr.y * local.y;
    rad4.z += pathThr.z * local.z;
    A.F.sh_n[pos] = nsh;

    // wave64 compaction (ballot + popcount + one atomic per wave and shard) of the shadow rays into the
    // shadow queue of this depth and of the continuation rays into queue[depth+1]
    uint32_t* shcnt = A.F.counters + (kMaxDepthQueues + uint32_t(depth)) * kQueueShards;
    const uint32_t cap_s = A.F.shadow_slots * A.F.cap_r;
    {
        // one atomic for all of the wave's shadow rays: ray k of every lane after rays 0..k-1 of all lanes
        const int lane = __lane_id();
        const unsigned long long lt = (1ull << lane) - 1ull;
        uint32_t total = 0;
        for (uint32_t k = 0;; ++k) {
            const unsigned long long m = __ballot(nsh > k);
            if (m == 0ull) break;
            total += uint32_t(__popcll(m));
        }
        const int leader = __ffsll(static_cast<long long>(__ballot(1))) - 1;
        uint32_t base = 0;
        if (lane == leader && total != 0u) base = atomicAdd(&shcnt[shard], total);
        base = uint32_t(__shfl(int(base), leader)) + shard * cap_s;
        for (uint32_t k = 0;; ++k) {
            const unsigned long long m = __ballot(nsh > k);
            if (m == 0ull) break;
            if (nsh > k) A.F.sh_queue[base + uint32_t(__popcll(m & lt))] = k * A.F.qsize + pos;
            base += uint32_t(__popcll(m));
        }
    }
    const uint32_t npos = queue_append(A.F.counters + uint32_t(depth + 1) * kQueueShards, A.F.cap_r, cont, shard);
    if (cont) {
        const RayQueue& N = A.F.q[(depth + 1) & 1];
        N.org[npos] = make_float4(nextOrigin.x, nextOrigin.y, nextOrigin.z, kFP32Max);
        N.dir[npos] = make_float4(nextDir.x, nextDir.y, nextDir.z, bitsf(pathSlot));
        N.thr[npos] = make_float4(nextThr.x, nextThr.y, nextThr.z, nextRoughness);
        N.rad[npos] = make_float4(rad4.x, rad4.y, rad4.z, bitsf(nextIsDiffuse ? 1u : 0u));  // payload.IsDiffuse
        N.pix[npos] = Q.pix[pos];
        A.F.fwd[pos] = npos;
    } else {
        A.F.px_rad[pathSlot] = rad4;
        A.F.fwd[pos] = ~0u;
    }
}

// ShadowHitShader / ShadowMissShader / ShadowAnyHitShader (RayTrace.hlsl:497-507, 532-542):
// one thread per queued shadow ray (grid-stride); occluded -> contribution * 0 (keeps NaN/Inf).
template <bool kCount, int W, int kOcc, int kPipe = 0>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kOcc > 0 ? kOcc : 1)))
void k_shadow(KArgs A, int depth) {
    lut_fill(A.S);
    extern __shared__ int stack[];  // S.stack_ints per lane, lane-interleaved, then the node cache
    NodeCache nc{nullptr, 0u};
    if (W == 8 && !kCount && (kPipe & 4))  // LDS node cache: a separate instantiation, so that the
        // default kernels' node loads are plain global loads (no LDS/global pointer select -> flat loads)
        nc = node_cache_fill(A.S, reinterpret_cast<uint4*>(stack + A.S.stack_ints * blockDim.x), A.P.lds_nodes);
    const uint32_t* cnt = shadow_counts(A.F, depth);
    const uint32_t count = queue_total(cnt);
    const uint32_t cap_s = A.F.shadow_slots * A.F.cap_r;
    uint32_t nv = 0, nt = 0;
    uint32_t lb;
    const uint32_t nb = min((count + blockDim.x - 1u) / blockDim.x, gridDim.x);
    if (!xcd_block(A.P.xcd_map != 0u, nb, lb)) return;
    for (uint32_t i = lb * blockDim.x + threadIdx.x; i < count; i += gridDim.x * blockDim.x) {
        const uint32_t slot = A.F.sh_queue[queue_pos(cnt, cap_s, i)];
        const float4 o4 = A.F.sh_org[slot];
        const float4 d4 = A.F.sh_dir[slot];
        const float4 c4 = A.F.sh_con[slot];
        HitRec h;
        const bool occluded =
            traverse<W, true, kCount, kPipe>(A.S, ld3(o4), ld3(d4), d4.w, o4.w, fbits(c4.w) == 0u, lane_stack(A.S, stack), h, nv, nt, nc);
        if (occluded) A.F.sh_con[slot] = make_float4(c4.x * 0.0f, c4.y * 0.0f, c4.z * 0.0f, c4.w);
    }
    if (kCount) {
        atomicAdd(&A.P.trav[2], (unsigned long long)nv);
        atomicAdd(&A.P.trav[3], (unsigned long long)nt);
    }
}

// Packet variants of k_trace / k_shadow (traverse8_packet): one item per lane, whole waves exit
// past the end of the queue, the rest run with live = false on the surplus lanes.
template <int kOcc>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kOcc > 0 ? kOcc : 1)))
void k_trace_packet(KArgs A, int depth) {
    lut_fill(A.S);
    const uint32_t* cnt = radiance_counts(A.F, depth);
    const uint32_t n = queue_total(cnt);
    uint32_t i, lw;
    if (!xcd_item(A.P.xcd_map != 0u, n, i, lw) || (i & ~63u) >= n) return;
    const bool live = i < n;
    const uint32_t pos = live ? queue_pos(cnt, A.F.cap_r, i) : 0u;
    float4 o4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), d4 = make_float4(0.0f, 0.0f, 1.0f, 0.0f);
    if (live) {
        o4 = A.F.q[depth & 1].org[pos];
        d4 = A.F.q[depth & 1].dir[pos];
    }
    const float tmin = depth == 1 ? 0.0f : kRayTMin;
    const bool alpha = depth <= A.P.set.MaxAnyHitPathLength;
    HitRec h;
    extern __shared__ int stack[];  // per-lane stacks for the adaptive fallback (FrameParams::packet_switch)
    traverse8_packet<false>(A.S, ld3(o4), ld3(d4), tmin, o4.w, alpha, live, h, A.P.packet_switch, lane_stack(A.S, stack));
    if (live) A.F.hit[pos] = make_float4(h.b1, h.b2, bitsf(h.tri), bitsf(h.geom));
}

template <int kOcc>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kOcc > 0 ? kOcc : 1)))
void k_shadow_packet(KArgs A, int depth) {
    lut_fill(A.S);
    const uint32_t* cnt = shadow_counts(A.F, depth);
    const uint32_t n = queue_total(cnt);
    uint32_t i, lw;
    if (!xcd_item(A.P.xcd_map != 0u, n, i, lw) || (i & ~63u) >= n) return;
    const bool live = i < n;
    const uint32_t cap_s = A.F.shadow_slots * A.F.cap_r;
    const uint32_t slot = live ? A.F.sh_queue[queue_pos(cnt, cap_s, i)] : 0u;
    float4 o4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), d4 = make_float4(0.0f, 0.0f, 1.0f, 0.0f), c4 = o4;
    if (live) {
        o4 = A.F.sh_org[slot];
        d4 = A.F.sh_dir[slot];
        c4 = A.F.sh_con[slot];
    }
    HitRec h;
    extern __shared__ int stack[];
    const bool occluded = traverse8_packet<true>(A.S, ld3(o4), ld3(d4), d4.w, o4.w, fbits(c4.w) == 0u, live, h,
                                                 A.P.packet_switch, lane_stack(A.S, stack));
    if (live && occluded) A.F.sh_con[slot] = make_float4(c4.x * 0.0f, c4.y * 0.0f, c4.z * 0.0f, c4.w);
}

// Adds the visibility-weighted shadow contributions of each depth-d vertex, in slot order, to the
// radiance of its path: in the continuation ray's queue entry, or in px_rad if the path ended.
__global__ __launch_bounds__(kBlock) void k_resolve(KArgs A, int depth) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t* cnt = radiance_counts(A.F, depth);
    if (i >= queue_total(cnt)) return;
    const uint32_t pos = queue_pos(cnt, A.F.cap_r, i);
    const uint32_t n = A.F.sh_n[pos];
    if (n == 0u) return;
    const uint32_t f = A.F.fwd[pos];
    float4* dst = f != ~0u ? &A.F.q[(depth + 1) & 1].rad[f] : &A.F.px_rad[fbits(A.F.q[depth & 1].dir[pos].w)];
    float4 r = *dst;
    for (uint32_t k = 0; k < n; ++k) {
        const float4 c = A.F.sh_con[size_t(k) * A.F.qsize + pos];
        r.x += c.x;
        r.y += c.y;
        r.z += c.z;
    }
    *dst = r;
}

// Wave-pool BVH8 traversal for the radiance (kShadow = false) and shadow (true) queues of one depth.
// Wave w owns the queue items [w * K * 64, (w + 1) * K * 64) (K = chunks_per_wave consecutive 64-ray
// chunks) and advances every lane by one node visit per iteration; lanes whose ray finished are
// refilled from the pool once >= refill lanes are idle (Aila & Laine 2009, "replacing terminated
// rays"), so a wave's time follows the pool's total work instead of K times its slowest ray.  The
// grid covers the queue; the dispatcher balances waves across CUs.  No atomics.
template <bool kCount, bool kShadow>
__global__ __launch_bounds__(kBlock) void k_traverse8p(KArgs A, int depth) {
    lut_fill(A.S);
    extern __shared__ int stack[];  // S.stack_ints per lane, lane-interleaved (launch_lds_bytes)
    lds_int* stk = lane_stack(A.S, stack);
    const uint32_t* cnt = kShadow ? shadow_counts(A.F, depth) : radiance_counts(A.F, depth);
    const uint32_t cap = kShadow ? A.F.shadow_slots * A.F.cap_r : A.F.cap_r;
    const uint32_t count = queue_total(cnt);
    const uint32_t wave = blockIdx.x * (kBlock / 64u) + threadIdx.x / 64u;
    const uint32_t pool = A.P.chunks_per_wave * 64u;
    const uint32_t begin = wave * pool;
    if (begin >= count) return;
    const uint32_t end = min(count, begin + pool);
    uint32_t next = begin;
    const uint32_t refill = A.P.refill_lanes;
    const unsigned long long lt = (1ull << __lane_id()) - 1ull;
    // Radiance rays: FORCE_OPAQUE iff PathLength > MaxAnyHitPathLength (RayTrace.hlsl:132, 401);
    // primary rays start at TMin 0 (:118), continuation rays at 1e-5 (:382).
    const bool alphaR = depth <= A.P.set.MaxAnyHitPathLength;
    const float tminR = depth == 1 ? 0.0f : kRayTMin;
    const uint32_t postpone = A.P.postpone_tris;
    bool active = false, more = false;
    uint32_t item = 0, tbase = 0, tbits = 0;
    uint2 tos = make_uint2(0u, 0u);
    Ray8 R;
    HitRec h;
    uint32_t node = 0;
    int sp = 0;
    uint32_t nv = 0, nt = 0;
    while (true) {
        const unsigned long long idle = __ballot(!active);
        const uint32_t nidle = uint32_t(__popcll(idle));
        if (next < end && nidle >= refill) {
            if (!active) {
                const uint32_t j = next + uint32_t(__popcll(idle & lt));
                if (j < end) {
                    const uint32_t pos = queue_pos_any(cnt, cap, j);
                    if (kShadow) {
                        item = A.F.sh_queue[pos];
                        const float4 o4 = A.F.sh_org[item];
                        const float4 d4 = A.F.sh_dir[item];
                        const bool alpha = fbits(A.F.sh_con[item].w) == 0u;
                        ray8_init(R, ld3(o4), ld3(d4), d4.w, o4.w, alpha, h);
                    } else {
                        item = pos;
                        const float4 o4 = A.F.q[depth & 1].org[pos];
                        const float4 d4 = A.F.q[depth & 1].dir[pos];
                        ray8_init(R, ld3(o4), ld3(d4), tminR, o4.w, alphaR, h);
                    }
                    node = 0;
                    sp = 0;
                    tbits = 0;
                    more = true;
                    active = true;
                }
            }
            next += nidle;
        }
        if (__ballot(active) == 0ull) {
            if (next >= end) break;
            continue;
        }
        bool finished = false;
        if (postpone == 0u) {  // triangles inline with their node visit
            if (active) {
                more = trav8_node<kCount>(A.S, R, node, sp, stk, tos, h, tbase, tbits, nv);
                const bool occ = tbits && trav8_tris<kShadow, kCount>(A.S, R, tbase, tbits, h, nt);
                tbits = 0;
                finished = occ || !more;
            }
        } else {
            // Triangle postponement (Ylitie et al. 2017, sec. 4): pending groups wait until >= postpone
            // lanes hold one (or no lane can visit a node), then those lanes test them together.
            const uint32_t ntri = uint32_t(__popcll(__ballot(active && tbits != 0u)));
            const bool node_lane = active && tbits == 0u && more;
            const uint32_t nnode = uint32_t(__popcll(__ballot(node_lane)));
            if (ntri >= postpone || nnode == 0u) {
                if (active && tbits != 0u) {
                    const bool occ = trav8_tris<kShadow, kCount>(A.S, R, tbase, tbits, h, nt);
                    tbits = 0;
                    finished = occ || !more;
                }
            } else if (node_lane) {
                more = trav8_node<kCount>(A.S, R, node, sp, stk, tos, h, tbase, tbits, nv);
                finished = !more && tbits == 0u;
            }
        }
        if (finished) {
            active = false;
            if (kShadow) {
                if (h.tri != kMiss) {  // occluded: contribution * 0 (keeps NaN/Inf like the reference)
                    const float4 c4 = A.F.sh_con[item];
                    A.F.sh_con[item] = make_float4(c4.x * 0.0f, c4.y * 0.0f, c4.z * 0.0f, c4.w);
                }
            } else {
                A.F.hit[item] = make_float4(h.b1, h.b2, bitsf(h.tri), bitsf(h.geom));
            }
        }
    }
    if (kCount) {
        atomicAdd(&A.P.trav[kShadow ? 2 : 0], (unsigned long long)nv);
        atomicAdd(&A.P.trav[kShadow ? 3 : 1], (unsigned long long)nt);
    }
}

// RayTrace.hlsl:140-148
// RaygenShader's clamp and progressive blend (RayTrace.hlsl:140-148) of path radiance r into accum[a].
PT_DEV void accumulate_pixel(const KArgs& A, uint32_t a, float4 r) {
    const float rx = fminf(fmaxf(r.x, 0.0f), kFP16Max);
    const float ry = fminf(fmaxf(r.y, 0.0f), kFP16Max);
    const float rz = fminf(fmaxf(r.z, 0.0f), kFP16Max);
    const float s = float(A.P.rtc.CurrSampleIdx);
    const float f = s / (s + 1.0f);
    const float4 cur = A.P.accum[a];
    A.P.accum[a] = make_float4(lerpf(rx, cur.x, f), lerpf(ry, cur.y, f), lerpf(rz, cur.z, f), 1.0f);
}

// A finished camera path's radiance: into the accumulation target, or -- frames that overlap their
// neighbours (DXRPT_OPT_FRAME_OVERLAP) -- into the frame's stage at the same index, blended by
// k_accum_stage once the previous frame's blend is done (same arithmetic, same order per pixel).
PT_DEV void finish_pixel(const KArgs& A, uint32_t a, float4 r) {
    if (A.P.stage) {
        A.P.stage[a] = r;
        return;
    }
    accumulate_pixel(A, a, r);
}

__global__ __launch_bounds__(kBlock) void k_accum_stage(KArgs A) {
    const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= A.P.num_paths) return;
    const uint32_t a = path_pixel(A, p).accumIdx;
    accumulate_pixel(A, a, A.P.stage[a]);
}

__global__ __launch_bounds__(kBlock) void k_accumulate(KArgs A) {
    const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= A.P.num_paths) return;
    accumulate_pixel(A, A.F.ps_pix[p].y, A.F.px_rad[p]);
}

// ---- megakernel (small frames) --------------------------------------------------------------------
// One thread per path runs the whole frame: raygen, then per depth the closest hit, path_vertex (the
// same shading code as k_shade) and the vertex's shadow rays (any hit, in slot order), then the
// accumulation.  There are no pass boundaries, so a frame costs its slowest WAVE's path instead of the
// sum over passes of each pass's slowest wave -- what limits a GPU's share of a frame split over 8
// GPUs (too few waves per pass to hide the dependent node-fetch chains).  The radiance of a path is
// summed in the wavefront's order (local terms, then each vertex's shadow contributions in slot
// order), so frames are bit-identical to the wavefront schedule.  Shadow rays go through the same
// per-slot buffers (slot k * qsize + path), so any number of spot lights works.  Ray counts are
// added to the queue counters (shard = wave % kQueueShards) for dxrpt_get_stats.
PT_DEV void count_rays(uint32_t* counters, uint32_t n) {
    const int lane = __lane_id();
    const int leader = __ffsll(static_cast<long long>(__ballot(1))) - 1;
    // wave sum of n (n <= 2 + lights): popcounts of the per-bit ballots
    uint32_t total = 0;
#pragma unroll
    for (int b = 0; b < 8; ++b) total += uint32_t(__popcll(__ballot((n >> b) & 1u))) << b;
    const uint32_t shard = ((blockIdx.x * blockDim.x + threadIdx.x) >> 6) % kQueueShards;
    if (lane == leader && total) atomicAdd(&counters[shard], total);
}

// DXRPT_SHADOW_MODE 0: every shadow ray of a vertex goes through the per-slot buffers (global memory)
// and the wave walks the slots; 1: the sun and sky-visibility rays stay in registers.
#ifndef DXRPT_SHADOW_MODE
#define DXRPT_SHADOW_MODE 0
#endif
// Memory-overlap mode of the megakernel's per-lane traversals (traverse8_pipe kPipe bits: 1 triangle
// pairs, 2 next node loaded before the current node's triangles); closest hit / any hit.
// Diagnostic builds only (never shipped; they change the image): 1 = shadow rays are not traced
// (every shadow ray unoccluded), to price their share of a frame.
#ifndef DXRPT_DIAG_NO_SHADOW
#define DXRPT_DIAG_NO_SHADOW 0
#endif
// 1: the depth-1 packet shadow traversal takes only sun rays (0: slot 0 whatever its kind, the r01-r02 rule).
#ifndef DXRPT_SUN0_CHECK
#define DXRPT_SUN0_CHECK 1
#endif
#ifndef DXRPT_MEGA_PIPE_CH
#define DXRPT_MEGA_PIPE_CH 0
#endif
#ifndef DXRPT_MEGA_PIPE_AH
#define DXRPT_MEGA_PIPE_AH 0
#endif
// The same traversal pipelining (traverse8_pipe kPipe bits) for the split schedule's per-lane closest hit
// (k_path_tail) and per-lane shadow rays (vertex_shadows), separately.  r03 A/B
// (profiles/r03_ab_split_pipe.txt): closest-hit triangle pairs (1) -0.8..-1.0 % on the metric, C3, C4 and
// C5's share; the next-node prefetch (2, 3) and any-hit pairs / prefetch lose 3-35 %.
// The split head's packet traversals with leaf triangles two at a time (traverse8_packet kPair): bit 0
// the primary closest hit, bit 1 the depth-1 sun shadow rays.
#ifndef DXRPT_HEAD_PACKET_PAIR
#define DXRPT_HEAD_PACKET_PAIR 0
#endif
#ifndef DXRPT_SPLIT_PIPE_CH
#define DXRPT_SPLIT_PIPE_CH 1
#endif
#ifndef DXRPT_SPLIT_PIPE_AH
#define DXRPT_SPLIT_PIPE_AH 0
#endif

// DXRPT_CHAIN_SHADOWS: a lane's per-lane shadow rays (slots k0 .. n-1) are traced back to back in ONE
// loop -- a lane that finishes ray k starts ray k+1 at its next step, instead of idling until the
// wave's slowest ray k is done (nested per-lane loops re-converge after every ray).  Each ray is
// exactly traverse<8, true>'s (ray8_init, then trav8_step until done), taken and added to the
// radiance in slot order, so the result is the slot loop's.
#ifndef DXRPT_CHAIN_SHADOWS
#define DXRPT_CHAIN_SHADOWS 0
#endif

// DXRPT_DIAG_PHASES (diagnostic builds only; dxrpt_get_phase_clocks): each lane of the full-frame
// megakernel sums the s_memrealtime ticks it spends in each phase of its path (the clock is wave-wide, so
// a lane masked off while others finish a loop is charged to the phase that loop belongs to, and a lane
// whose path ended waits in phase 7); wave sums go to g_phase_ticks with one atomic per phase per wave.
#ifndef DXRPT_DIAG_PHASES
#define DXRPT_DIAG_PHASES 0
#endif
struct PhaseAcc {
    uint32_t a[8];
    uint32_t t;
};
__device__ unsigned long long g_phase_ticks[8];
PT_DEV void phase_mark(PhaseAcc* pa, int k) {
#if DXRPT_DIAG_PHASES
    if (pa) {
        const uint32_t now = uint32_t(__builtin_amdgcn_s_memrealtime());
        pa->a[k] += now - pa->t;
        pa->t = now;
    }
#endif
}
PT_DEV void phase_flush(PhaseAcc* pa) {
#if DXRPT_DIAG_PHASES
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        uint32_t v = pa->a[k];
        for (int off = 32; off > 0; off >>= 1) v += uint32_t(__shfl_xor(int(v), off));
        if ((threadIdx.x & 63u) == 0u) atomicAdd(&g_phase_ticks[k], (unsigned long long)v);
    }
#endif
}

template <bool kCount>
PT_DEV void shadow_rays_chained(const KArgs& A, uint32_t slot_p, uint32_t k0, uint32_t n, lds_int* stk, float4& rad,
                                uint32_t* cnt, const NodeCache& nc) {
    uint32_t k = k0;
    Ray8 R;
    HitRec h;
    uint32_t node = 0;
    int sp = 0;
    uint2 tos = make_uint2(0u, 0u);
    f3 c = f3{0.0f, 0.0f, 0.0f};
    auto start = [&](uint32_t kk) {
        const size_t slot = size_t(kk) * A.F.qsize + slot_p;
        const float4 o4 = A.F.sh_org[slot], d4 = A.F.sh_dir[slot], c4 = A.F.sh_con[slot];
        ray8_init(R, ld3(o4), ld3(d4), d4.w, o4.w, fbits(c4.w) == 0u, h);
        c = ld3(c4);
        node = 0;
        sp = 0;
        tos = make_uint2(0u, 0u);
    };
    if (k < n) start(k);
    while (k < n) {
        if (trav8_step<true, kCount>(A.S, R, node, sp, stk, tos, h, cnt[2], cnt[3], nc)) {
            const bool occluded = h.tri != kMiss;
            rad.x += occluded ? c.x * 0.0f : c.x;
            rad.y += occluded ? c.y * 0.0f : c.y;
            rad.z += occluded ? c.z * 0.0f : c.z;
            if (++k < n) start(k);
        }
    }
}

// One path from its first ray (PathLength 1) to its end: per depth the closest hit, path_vertex and
// the vertex's shadow rays in slot order -- the megakernel's per-thread loop, shared by k_path (camera
// paths) and k_bake (lightmap texels).  `slot_p` (< F.qsize) indexes the per-slot shadow buffers, `pix`
// is the CMJ pattern index; `packet` bit 0 / bit 1: wave-coherent traversal for the depth-1 closest hit
// / the depth-1 sun shadow rays (all lanes must be active at depth 1 then).  Returns the radiance.
// kBake: the first ray is BakeRayGen's (TMin 0.0001, IsDiffuse, no packets) instead of RaygenShader's.
// nc: the workgroup's LDS copy of the top BVH8 nodes for the per-lane traversals (n = 0: none).
// kCount: census of the traversal work (cnt[0..1] closest-hit node / triangle fetches, cnt[2..3] any
// hit; per-lane traversals fetch per lane, packet traversals once per wave).
template <bool kBake, bool kCount = false>
PT_DEV float4 trace_path(const KArgs& A, uint32_t slot_p, uint32_t pix, f3 org, f3 dir, float tmax, lds_int* stk,
                         uint32_t packet_mask, const NodeCache& nc = NodeCache{nullptr, 0u}, uint32_t* cnt = nullptr,
                         PhaseAcc* pa = nullptr) {
    const dxrpt_app_settings& set = A.P.set;
    const float tmin1 = kBake ? 0.0001f : 0.0f;
    const bool isDiffuse1 = kBake;
    const uint32_t packet = kBake ? 0u : packet_mask;
    uint32_t unused[5] = {0u, 0u, 0u, 0u, 0u};
    if (!kCount) cnt = unused;
    f3 thr = f3{1.0f, 1.0f, 1.0f};
    float payloadRoughness = 0.0f;
    bool payloadIsDiffuse = isDiffuse1;
    float4 rad = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const int L = set.MaxPathLength < 2 ? 2 : set.MaxPathLength;
    for (int d = 1; d <= L - 1; ++d) {
        count_rays(A.F.counters + uint32_t(d) * kQueueShards, 1u);
        HitRec h;
        if (d == 1 && (packet & 1u))  // coherent primary rays: wave-coherent traversal (same results)
            traverse8_packet<false, kCount>(A.S, org, dir, tmin1, tmax, d <= set.MaxAnyHitPathLength, true, h, 0u, nullptr, cnt);
        else
            traverse<8, false, kCount, DXRPT_MEGA_PIPE_CH>(A.S, org, dir, d == 1 ? tmin1 : kRayTMin, tmax, d <= set.MaxAnyHitPathLength, stk, h,
                                       cnt[0], cnt[1], nc);
        phase_mark(pa, d == 1 ? 0 : d == 2 ? 3 : 6);
        if (kCount && h.tri != kMiss) ++cnt[4];  // radiance hits: the vertices PathTrace shades
        VertexIn V;
        V.inOrigin = org;
        V.inDir = dir;
        V.pathThr = thr;
        V.payloadRoughness = payloadRoughness;
        V.payloadIsDiffuse = payloadIsDiffuse;
        V.pix = pix;
        V.hit = make_float4(h.b1, h.b2, bitsf(h.tri), bitsf(h.geom));
#if DXRPT_SHADOW_MODE == 0
        VertexOut O;
        uint32_t nsh = 0;
        bool sun0 = false;  // slot 0 holds the sun's shadow ray (the sun is emitted first when at all)
        path_vertex(A, d, V, [&](int kind, f3 o, f3 dd, float tmn, float tmx, f3 c, bool fo) {
            sun0 |= kind == kShadowSun || !DXRPT_SUN0_CHECK;
            emit_shadow(A, slot_p, nsh, o, dd, tmn, tmx, c, fo);
        }, O);
        count_rays(A.F.counters + (kMaxDepthQueues + uint32_t(d)) * kQueueShards, nsh);
        phase_mark(pa, d == 1 ? 1 : d == 2 ? 4 : 6);
        rad.x += thr.x * O.local.x;
        rad.y += thr.y * O.local.y;
        rad.z += thr.z * O.local.z;
        // ShadowHit/Miss/AnyHit: contribution * visibility, slot by slot.  The wave walks the slots
        // together; at depth 1 (packet bit 1) the sun shadow rays of an 8x8 pixel block's primary hits
        // -- one direction, nearby origins -- take the wave-coherent traversal.  A lane whose sun term
        // is zero has another kind of ray in slot 0 (a spot light's, or at MaxPathLength 2 the sky
        // visibility ray, random directions): it traces per lane, after the packet.
#if DXRPT_CHAIN_SHADOWS
        uint32_t k0 = 0;
        if (d == 1 && (packet & 2u) && !DXRPT_DIAG_NO_SHADOW) {  // slot 0 of the sun lanes: one packet
            const bool live = nsh > 0u && sun0;
            const size_t slot = slot_p;
            float4 o4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), d4 = make_float4(0.0f, 0.0f, 1.0f, 0.0f), c4 = o4;
            if (live) {
                o4 = A.F.sh_org[slot];
                d4 = A.F.sh_dir[slot];
                c4 = A.F.sh_con[slot];
            }
            HitRec hs;
            const bool occluded = traverse8_packet<true, kCount>(A.S, ld3(o4), ld3(d4), d4.w, o4.w, fbits(c4.w) == 0u, live,
                                                                 hs, 0u, nullptr, cnt + 2);
            if (live) {
                rad.x += occluded ? c4.x * 0.0f : c4.x;
                rad.y += occluded ? c4.y * 0.0f : c4.y;
                rad.z += occluded ? c4.z * 0.0f : c4.z;
                k0 = 1u;
            }
        }
        if (!DXRPT_DIAG_NO_SHADOW) shadow_rays_chained<kCount>(A, slot_p, k0, nsh, stk, rad, cnt, nc);
#elif DXRPT_SHADOW_PAIRS >= 2
        // slot 0 of a depth-1 vertex through the packet traversal (sun lanes), the rest two at a time
        uint32_t k0 = 0;
        if (d == 1 && (packet & 2u) && !DXRPT_DIAG_NO_SHADOW) {
            const bool live = nsh > 0u;
            float4 o4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), d4 = make_float4(0.0f, 0.0f, 1.0f, 0.0f), c4 = o4;
            if (live) {
                o4 = A.F.sh_org[slot_p];
                d4 = A.F.sh_dir[slot_p];
                c4 = A.F.sh_con[slot_p];
            }
            HitRec hs;
            bool occluded = traverse8_packet<true, kCount>(A.S, ld3(o4), ld3(d4), d4.w, o4.w, fbits(c4.w) == 0u,
                                                           live && sun0, hs, 0u, nullptr, cnt + 2);
            if (live && !sun0)
                occluded = traverse<8, true, kCount, DXRPT_MEGA_PIPE_AH>(A.S, ld3(o4), ld3(d4), d4.w, o4.w, fbits(c4.w) == 0u, stk, hs, cnt[2], cnt[3], nc);
            if (live) {
                rad.x += occluded ? c4.x * 0.0f : c4.x;
                rad.y += occluded ? c4.y * 0.0f : c4.y;
                rad.z += occluded ? c4.z * 0.0f : c4.z;
            }
            k0 = 1u;
        }
        if (!DXRPT_DIAG_NO_SHADOW) shadow_pairs<kCount>(A, slot_p, k0, nsh, stk, rad, cnt[2], cnt[3]);
#else
        for (uint32_t k = 0; !DXRPT_DIAG_NO_SHADOW && __ballot(k < nsh) != 0ull; ++k) {
            const bool live = k < nsh;
            const size_t slot = size_t(k) * A.F.qsize + slot_p;
            float4 o4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), d4 = make_float4(0.0f, 0.0f, 1.0f, 0.0f), c4 = o4;
            if (live) {
                o4 = A.F.sh_org[slot];
                d4 = A.F.sh_dir[slot];
                c4 = A.F.sh_con[slot];
            }
            HitRec hs;
            bool occluded = false;
            const bool pk = d == 1 && k == 0 && (packet & 2u);
            if (pk)
                occluded = traverse8_packet<true, kCount>(A.S, ld3(o4), ld3(d4), d4.w, o4.w, fbits(c4.w) == 0u, live && sun0, hs,
                                                          0u, nullptr, cnt + 2);
            if (live && !(pk && sun0))
                occluded = traverse<8, true, kCount, DXRPT_MEGA_PIPE_AH>(A.S, ld3(o4), ld3(d4), d4.w, o4.w, fbits(c4.w) == 0u, stk, hs, cnt[2], cnt[3], nc);
            if (live) {
                rad.x += occluded ? c4.x * 0.0f : c4.x;
                rad.y += occluded ? c4.y * 0.0f : c4.y;
                rad.z += occluded ? c4.z * 0.0f : c4.z;
            }
        }
#endif
#else
        VertexOut O;
        // The vertex's sun and sky-visibility rays stay in registers: both start at the hit position
        // with TMin 1e-5 / TMax FP32Max (RayTrace.hlsl:241-244, 415-425), the sun's direction is the
        // wave-uniform SunDirectionWS, so a ray is its pending contribution (+ the sky direction).
        // Spot-light rays (any number) go through the per-slot buffers.
        uint32_t nsh = 0, nspot = 0;
        bool hasSun = false, hasSky = false;
        f3 cSun = f3{0.0f, 0.0f, 0.0f}, cSky = cSun, shOrg = cSun, skyDir = cSun;
        path_vertex(A, d, V, [&](int kind, f3 o, f3 dd, float tmn, float tmx, f3 c, bool fo) {
            ++nsh;
            if (kind == kShadowSun) {
                hasSun = true;
                cSun = c;
                shOrg = o;
            } else if (kind == kShadowSky) {
                hasSky = true;
                cSky = c;
                shOrg = o;
                skyDir = dd;
            } else {
                emit_shadow(A, slot_p, nspot, o, dd, tmn, tmx, c, fo);
            }
        }, O);
        count_rays(A.F.counters + (kMaxDepthQueues + uint32_t(d)) * kQueueShards, nsh);
        rad.x += thr.x * O.local.x;
        rad.y += thr.y * O.local.y;
        rad.z += thr.z * O.local.z;
        // ShadowHit/Miss/AnyHit: contribution * visibility, in the emission order (sun, spots, sky).
        // At depth 1 (packet bit 1) the sun shadow rays of an 8x8 pixel block's primary hits -- one
        // direction, nearby origins -- take the wave-coherent traversal.
        const f3 sunD = f3{A.P.rtc.SunDirectionWS[0], A.P.rtc.SunDirectionWS[1], A.P.rtc.SunDirectionWS[2]};
        const bool sunAlpha = !(d > set.MaxAnyHitPathLength), skyAlpha = !(d + 1 > set.MaxAnyHitPathLength);
        if (__ballot(hasSun) != 0ull) {
            HitRec hs;
            bool occluded = false;
            if (d == 1 && (packet & 2u))
                occluded = traverse8_packet<true, kCount>(A.S, shOrg, sunD, kRayTMin, kFP32Max, sunAlpha, hasSun, hs, 0u, nullptr, cnt + 2);
            else if (hasSun)
                occluded = traverse<8, true, kCount, DXRPT_MEGA_PIPE_AH>(A.S, shOrg, sunD, kRayTMin, kFP32Max, sunAlpha, stk, hs, cnt[2], cnt[3], nc);
            if (hasSun) {
                rad.x += occluded ? cSun.x * 0.0f : cSun.x;
                rad.y += occluded ? cSun.y * 0.0f : cSun.y;
                rad.z += occluded ? cSun.z * 0.0f : cSun.z;
            }
        }
        for (uint32_t k = 0; __ballot(k < nspot) != 0ull; ++k) {
            if (k < nspot) {
                const size_t slot = size_t(k) * A.F.qsize + slot_p;
                const float4 o4 = A.F.sh_org[slot], d4 = A.F.sh_dir[slot], c4 = A.F.sh_con[slot];
                HitRec hs;
                const bool occluded =
                    traverse<8, true, kCount, DXRPT_MEGA_PIPE_AH>(A.S, ld3(o4), ld3(d4), d4.w, o4.w, fbits(c4.w) == 0u, stk, hs, cnt[2], cnt[3], nc);
                rad.x += occluded ? c4.x * 0.0f : c4.x;
                rad.y += occluded ? c4.y * 0.0f : c4.y;
                rad.z += occluded ? c4.z * 0.0f : c4.z;
            }
        }
        if (hasSky) {
            HitRec hs;
            const bool occluded = traverse<8, true, kCount, DXRPT_MEGA_PIPE_AH>(A.S, shOrg, skyDir, kRayTMin, kFP32Max, skyAlpha, stk, hs, cnt[2], cnt[3], nc);
            rad.x += occluded ? cSky.x * 0.0f : cSky.x;
            rad.y += occluded ? cSky.y * 0.0f : cSky.y;
            rad.z += occluded ? cSky.z * 0.0f : cSky.z;
        }
#endif
        phase_mark(pa, d == 1 ? 2 : d == 2 ? 5 : 6);
        if (!O.cont) break;
        org = O.nextOrigin;
        dir = O.nextDir;
        tmax = kFP32Max;
        thr = O.nextThr;
        payloadRoughness = O.nextRoughness;
        payloadIsDiffuse = O.nextIsDiffuse;
    }
    return rad;
}

// DXRPT_GROUP_PAIRS: the path-group traversal tests a leaf's triangles two at a time -- both records in
// one memory round trip, both geometric tests against the bound at the pair's start (a superset of the
// sequential candidates), both candidates' alpha inputs (opacity descriptor + UVs) and then both
// opacity taps in flight together, acceptance in order with the live bound: the hits of testing them one
// after the other, in half the dependent round trips (the slowest waves of a small frame are
// alpha-tested shadow rays through foliage).
#ifndef DXRPT_GROUP_PAIRS
#define DXRPT_GROUP_PAIRS 1
#endif

// The alpha inputs of triangle `gtri` on geometry `geom` for a per-lane candidate (issued, not waited on).
struct LaneAlpha {
    GeoTex op;
    float2 uv0, uv1, uv2;
    OmmProbe omm;
};
PT_DEV LaneAlpha lane_alpha_issue(const SceneDev& S, uint32_t geom, uint32_t gtri, uint32_t slot, float b1, float b2) {
    LaneAlpha a;
    a.op = S.geoshade[geom].opacity;
    const float2* V = reinterpret_cast<const float2*>(S.tri_verts + size_t(gtri) * 12u);
    a.uv0 = V[3];
    a.uv1 = V[11];
    a.uv2 = V[19];
    a.omm = omm_probe(S, slot, b1, b2);
    return a;
}

// Opacity of a per-lane candidate at barycentrics (b1, b2): AnyHitShader's tap (alpha_accepts), split
// so two candidates' taps can be in flight together.
PT_DEV OpacityTap lane_alpha_tap(const SceneDev& S, const LaneAlpha& a, float b1, float b2) {
    const float w0 = (1.0f - b1) - b2;
    const float u = bary_lerp(a.uv0.x, a.uv1.x, a.uv2.x, w0, b1, b2);
    const float v = bary_lerp(a.uv0.y, a.uv1.y, a.uv2.y, w0, b1, b2);
    return opacity_issue(S, tex_desc(a.op), u, v);
}

PT_DEV bool trav8_tris_pairs(const SceneDev& S, const Ray8& R, uint32_t tbase, uint32_t tbits, HitRec& h, bool any) {
    while (tbits) {
        const uint32_t b0 = uint32_t(__builtin_ctz(tbits));
        tbits &= tbits - 1u;
        const bool two = tbits != 0u;
        const uint32_t b1 = two ? uint32_t(__builtin_ctz(tbits)) : b0;
        if (two) tbits &= tbits - 1u;
        const TriRec r0 = load_tri_raw(S, tbase + b0), r1 = load_tri_raw(S, tbase + b1);
        pin_tri(r0);
        pin_tri(r1);
        float t0 = 0.0f, u0 = 0.0f, v0 = 0.0f, t1 = 0.0f, u1 = 0.0f, v1 = 0.0f;
        const bool c0 = any ? tri_candidate<true>(r0, R.o, R.d, R.tmin, R.tmax, h, t0, u0, v0)
                            : tri_candidate<false>(r0, R.o, R.d, R.tmin, R.tmax, h, t0, u0, v0);
        const bool c1 = two && (any ? tri_candidate<true>(r1, R.o, R.d, R.tmin, R.tmax, h, t1, u1, v1)
                                    : tri_candidate<false>(r1, R.o, R.d, R.tmin, R.tmax, h, t1, u1, v1));
        if (!c0 && !c1) continue;
        const bool n0 = c0 && R.alpha && !(fbits(r0.p2.w) & kTriOpaque);
        const bool n1 = c1 && R.alpha && !(fbits(r1.p2.w) & kTriOpaque);
        float o0 = 1.0f, o1 = 1.0f;
        if (n0 || n1) {  // AnyHitShader (RayTrace.hlsl:485-507) for the candidates on alpha-tested geometry
            const LaneAlpha a0 = lane_alpha_issue(S, fbits(r0.p1.w), fbits(r0.p0.w), fbits(r0.p2.w) >> 1, u0, v0);
            const LaneAlpha a1 = lane_alpha_issue(S, fbits(r1.p1.w), fbits(r1.p0.w), fbits(r1.p2.w) >> 1, u1, v1);
            asm volatile("" ::"v"(a0.op.offset), "v"(a0.op.whf), "v"(a0.uv0.x), "v"(a0.uv0.y), "v"(a0.uv1.x), "v"(a0.uv1.y),
                         "v"(a0.uv2.x), "v"(a0.uv2.y), "v"(a1.op.offset), "v"(a1.op.whf), "v"(a1.uv0.x), "v"(a1.uv0.y),
                         "v"(a1.uv1.x), "v"(a1.uv1.y), "v"(a1.uv2.x), "v"(a1.uv2.y));
            asm volatile("" ::"v"(a0.omm.word), "v"(a1.omm.word));
            // a candidate whose micromap cell decides skips the tap (o = 0: reject; 1: accept)
            const uint32_t vd0 = n0 && a0.op.whf != 0u ? omm_verdict(a0.omm) : kOmmOpaque;
            const uint32_t vd1 = n1 && a1.op.whf != 0u ? omm_verdict(a1.omm) : kOmmOpaque;
            if (vd0 == kOmmTransparent) o0 = 0.0f;
            if (vd1 == kOmmTransparent) o1 = 0.0f;
            const bool m0 = n0 && a0.op.whf != 0u && vd0 == kOmmUnknown, m1 = n1 && a1.op.whf != 0u && vd1 == kOmmUnknown;
            OpacityTap q0{}, q1{};
            if (m0) q0 = lane_alpha_tap(S, a0, u0, v0);
            if (m1) q1 = lane_alpha_tap(S, a1, u1, v1);
            if (m0) o0 = opacity_finish(S, q0);
            if (m1) o1 = opacity_finish(S, q1);
        }
        if (c0 && !(o0 < 0.35f) && (any || t0 < h.t || (t0 == h.t && fbits(r0.p0.w) < h.tri))) {
            h.t = t0;
            h.tri = fbits(r0.p0.w);
            h.b1 = u0;
            h.b2 = v0;
            h.geom = fbits(r0.p1.w);
            if (any) return true;
        }
        if (c1 && !(o1 < 0.35f) && (any || t1 < h.t || (t1 == h.t && fbits(r1.p0.w) < h.tri))) {
            h.t = t1;
            h.tri = fbits(r1.p0.w);
            h.b1 = u1;
            h.b2 = v1;
            h.geom = fbits(r1.p1.w);
            if (any) return true;
        }
    }
    return false;
}

// Per-lane BVH8 traversal whose kind is a lane value (closest hit, or any hit when `any`): the
// path-group schedule below runs a continuation ray and shadow rays in one loop.  Same node order and
// triangle tests as traverse<8, any, false>, so the same hit / visibility.
PT_DEV bool traverse8_rt(const SceneDev& S, f3 o, f3 d, float tmin, float tmax, bool alpha, bool any, lds_int* stk,
                         HitRec& h) {
    h.t = tmax;
    h.tri = kMiss;
    h.b1 = h.b2 = 0.0f;
    h.geom = 0;
    Ray8 R;
    ray8_init(R, o, d, tmin, tmax, alpha, h);
    uint32_t node = 0, nv = 0;
    int sp = 0;
    uint2 tos = make_uint2(0u, 0u);
    while (true) {
        uint32_t tbase = 0, tbits = 0;
        const bool more = trav8_node<false>(S, R, node, sp, stk, tos, h, tbase, tbits, nv);
        bool done = false;
        if (DXRPT_GROUP_PAIRS && tbits) done = trav8_tris_pairs(S, R, tbase, tbits, h, any);
        while (!DXRPT_GROUP_PAIRS && tbits) {
            const uint32_t b = uint32_t(__builtin_ctz(tbits));
            tbits &= tbits - 1u;
            const TriRec r = load_tri(S, tbase + b);
            if (any ? test_tri_rec<true>(S, r, R.o, R.d, R.tmin, R.tmax, R.alpha, h)
                    : test_tri_rec<false>(S, r, R.o, R.d, R.tmin, R.tmax, R.alpha, h)) {
                done = true;
                break;
            }
        }
        if (done || !more) break;
    }
    return h.tri != kMiss;
}

// Path-group schedule (DXRPT_OPT_MEGAKERNEL_LANES g < 64): each path is carried by 64/g lanes of its
// wave (lanes l, l+g, ...) that all run its shading (identical values, so identical control flow);
// after a vertex, its continuation ray and its shadow rays are independent traversals, handed out to
// the group's lanes round by round (item 0 = continuation, then the shadow slots), so a path's chain of
// dependent traversals shortens (L=3 with the sun: R1 | R2+S1 | S2+V2 = 3 rounds instead of 5).  The
// results are gathered back over the group with lane shuffles and summed in the reference's slot
// order, so the frame equals trace_path's bit for bit.  Only member 0 counts rays (and, in
// camera_path, writes the pixel).
PT_DEV float4 trace_path_group(const KArgs& A, uint32_t slot_p, uint32_t pix, f3 org, f3 dir, float tmax, lds_int* stk,
                               uint32_t g) {
    const dxrpt_app_settings& set = A.P.set;
    const uint32_t lane = uint32_t(__lane_id());
    const uint32_t member = lane / g, gsize = 64u / g, leader = lane & (g - 1u);
    const bool quiet = member != 0u;
    const uint32_t packet = __ballot(1) != ~0ull ? 0u : (A.P.packet & 1u);
    f3 thr = f3{1.0f, 1.0f, 1.0f};
    float payloadRoughness = 0.0f;
    bool payloadIsDiffuse = false;
    float4 rad = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const int L = set.MaxPathLength < 2 ? 2 : set.MaxPathLength;
    HitRec h;
    uint32_t nv = 0, nt = 0;
    for (int d = 1; d <= L - 1; ++d) {
        count_rays(A.F.counters + uint32_t(d) * kQueueShards, quiet ? 0u : 1u);
        if (d == 1) {  // the primary ray: every member traces it (packets while the wave is full)
            if (packet)
                traverse8_packet<false, false, true>(A.S, org, dir, 0.0f, tmax, d <= set.MaxAnyHitPathLength, true, h);
            else
                traverse<8, false, false>(A.S, org, dir, 0.0f, tmax, d <= set.MaxAnyHitPathLength, stk, h, nv, nt);
        }
        VertexIn V;
        V.inOrigin = org;
        V.inDir = dir;
        V.pathThr = thr;
        V.payloadRoughness = payloadRoughness;
        V.payloadIsDiffuse = payloadIsDiffuse;
        V.pix = pix;
        V.hit = make_float4(h.b1, h.b2, bitsf(h.tri), bitsf(h.geom));
        VertexOut O;
        uint32_t nsh = 0;
        path_vertex(A, d, V, [&](int, f3 o, f3 dd, float tmn, float tmx, f3 c, bool fo) {
            emit_shadow(A, slot_p, nsh, o, dd, tmn, tmx, c, fo);
        }, O);
        count_rays(A.F.counters + (kMaxDepthQueues + uint32_t(d)) * kQueueShards, quiet ? 0u : nsh);
        rad.x += thr.x * O.local.x;
        rad.y += thr.y * O.local.y;
        rad.z += thr.z * O.local.z;
        const uint32_t first = O.cont ? 1u : 0u, items = first + nsh;
        uint32_t occ_lo = 0, occ_hi = 0;  // occlusion bit per shadow slot (<= 2 + 32 lights)
        HitRec hn;
        hn.t = 0.0f;
        hn.b1 = hn.b2 = 0.0f;
        hn.tri = kMiss;
        hn.geom = 0;
        for (uint32_t r = 0; __ballot(r * gsize < items) != 0ull; ++r) {
            const uint32_t item = r * gsize + member;
            if (item < items) {
                f3 o, dd;
                float tmn, tmx;
                bool alpha, any;
                if (item < first) {  // the continuation ray (PathLength d + 1)
                    o = O.nextOrigin;
                    dd = O.nextDir;
                    tmn = kRayTMin;
                    tmx = kFP32Max;
                    alpha = d + 1 <= set.MaxAnyHitPathLength;
                    any = false;
                } else {
                    const size_t slot = size_t(item - first) * A.F.qsize + slot_p;
                    const float4 o4 = A.F.sh_org[slot], d4 = A.F.sh_dir[slot];
                    o = ld3(o4);
                    dd = ld3(d4);
                    tmn = d4.w;
                    tmx = o4.w;
                    alpha = fbits(A.F.sh_con[slot].w) == 0u;
                    any = true;
                }
                HitRec ht;
                const bool hit = traverse8_rt(A.S, o, dd, tmn, tmx, alpha, any, stk, ht);
                if (item < first) {
                    hn = ht;
                } else if (hit) {
                    const uint32_t k = item - first;
                    if (k < 32u) occ_lo |= 1u << k; else occ_hi |= 1u << (k - 32u);
                }
            }
        }
        // gather over the group: occlusion bits (OR over members), the continuation hit (member 0)
        for (uint32_t off = g; off < 64u; off <<= 1) {
            occ_lo |= uint32_t(__shfl_xor(int(occ_lo), int(off)));
            occ_hi |= uint32_t(__shfl_xor(int(occ_hi), int(off)));
        }
        h.b1 = __shfl(hn.b1, int(leader));
        h.b2 = __shfl(hn.b2, int(leader));
        h.tri = uint32_t(__shfl(int(hn.tri), int(leader)));
        h.geom = uint32_t(__shfl(int(hn.geom), int(leader)));
        for (uint32_t k = 0; k < nsh; ++k) {  // ShadowHit/Miss: contribution * visibility, in slot order
            const float4 c4 = A.F.sh_con[size_t(k) * A.F.qsize + slot_p];
            const bool occluded = ((k < 32u ? occ_lo >> k : occ_hi >> (k - 32u)) & 1u) != 0u;
            rad.x += occluded ? c4.x * 0.0f : c4.x;
            rad.y += occluded ? c4.y * 0.0f : c4.y;
            rad.z += occluded ? c4.z * 0.0f : c4.z;
        }
        if (!O.cont) break;
        org = O.nextOrigin;
        dir = O.nextDir;
        thr = O.nextThr;
        payloadRoughness = O.nextRoughness;
        payloadIsDiffuse = O.nextIsDiffuse;
    }
    return rad;
}

// Path p of a wave whose paths are 64-aligned (p & ~63 .. p | 63).  Packets need every lane of the wave
// (the packet stack lives one entry per lane): a partial last wave (num_paths % 64 != 0) traverses one
// ray per lane -- a wave-uniform scalar test, the other waves keep their packets (same results).
template <bool kCount = false>
PT_DEV void camera_path(const KArgs& A, uint32_t p, lds_int* stk, const NodeCache& nc = NodeCache{nullptr, 0u},
                        uint32_t* cnt = nullptr, PhaseAcc* pa = nullptr) {
    const PrimaryRay pr = primary_ray(A, p);
    const uint32_t packet = (p | 63u) < A.P.num_paths ? A.P.packet : 0u;
    const float4 rad = trace_path<false, kCount>(A, p, pr.pixelIdx, pr.start, pr.dir, pr.length, stk, packet, nc, cnt, pa);
    finish_pixel(A, pr.accumIdx, rad);
}

// A path of a path group (DXRPT_OPT_MEGAKERNEL_LANES; g paths per wave): only member 0 writes the pixel.
PT_DEV void camera_path_group(const KArgs& A, uint32_t p, lds_int* stk, bool member0, uint32_t g) {
    const PrimaryRay pr = primary_ray(A, p);
    const float4 rad = trace_path_group(A, p, pr.pixelIdx, pr.start, pr.dir, pr.length, stk, g);
    if (member0) finish_pixel(A, pr.accumIdx, rad);
}

// A vertex's shadow rays (ShadowHit/Miss/AnyHit, RayTrace.hlsl:497-507, 532-542) walked slot by slot by
// the wave, contribution * visibility added to rad in slot order -- trace_path's walk (the depth-1 sun
// rays of a full wave through the packet traversal, packet bit 1).
PT_DEV void vertex_shadows(const KArgs& A, int d, uint32_t slot_p, uint32_t nsh, bool sun0, uint32_t packet,
                           float4& rad) {
    uint32_t nv = 0, nt = 0;
#if DXRPT_SHADOW_PAIRS
    // depth >= 2 (the tails: the sun and sky-visibility rays of the last vertex share their origin): two
    // slots at a time.  The head (d == 1, a constant there) keeps the slot loop below.
    if (d > 1) {
        shadow_pairs<false>(A, slot_p, 0u, nsh, nullptr, rad, nv, nt);
        return;
    }
#endif
    for (uint32_t k = 0; __ballot(k < nsh) != 0ull; ++k) {
        const bool live = k < nsh;
        const size_t slot = size_t(k) * A.F.qsize + slot_p;
        float4 o4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), d4 = make_float4(0.0f, 0.0f, 1.0f, 0.0f), c4 = o4;
        if (live) {
            o4 = A.F.sh_org[slot];
            d4 = A.F.sh_dir[slot];
            c4 = A.F.sh_con[slot];
        }
        HitRec hs;
        bool occluded = false;
        const bool pk = d == 1 && k == 0 && (packet & 2u);
        if (pk)
            occluded = traverse8_packet<true, false, (DXRPT_HEAD_PACKET_PAIR & 2) != 0>(A.S, ld3(o4), ld3(d4), d4.w, o4.w, fbits(c4.w) == 0u, live && sun0, hs);
        if (live && !(pk && sun0))
            occluded = traverse<8, true, false, DXRPT_SPLIT_PIPE_AH>(A.S, ld3(o4), ld3(d4), d4.w, o4.w, fbits(c4.w) == 0u, nullptr, hs, nv, nt);
        if (live) {
            rad.x += occluded ? c4.x * 0.0f : c4.x;
            rad.y += occluded ? c4.y * 0.0f : c4.y;
            rad.z += occluded ? c4.z * 0.0f : c4.z;
        }
    }
}

// DXRPT_MEGA_STAGE: k_path's camera path with the path state kept in memory instead of registers across
// the traversals -- the split schedule's staging inside the single kernel.  FrameBuffers::q[0] at the
// path slot p (unused by megakernel frames) holds the continuation: org (origin, bits(accumulation
// index)), dir (direction, bits(CMJ pattern)), thr (throughput, payload Roughness), rad (radiance so
// far, bits(payload IsDiffuse)).  The continuation is stored before the vertex's shadow rays are
// traced (only the radiance sum is live across them) and re-read after the next closest-hit traversal
// (only the ray and p are live across it).  Same arithmetic in the same order as trace_path.
#ifndef DXRPT_MEGA_STAGE
#define DXRPT_MEGA_STAGE 0
#endif
PT_DEV void camera_path_staged(const KArgs& A, uint32_t p) {
    const dxrpt_app_settings& set = A.P.set;
    const RayQueue& Q = A.F.q[0];
    const int L = set.MaxPathLength < 2 ? 2 : set.MaxPathLength;
    bool cont;
    bool nextDiffuse;
    float4 rad;
    {   // depth 1: RaygenShader's ray, packet traversals while the wave is full
        const PrimaryRay pr = primary_ray(A, p);
        const uint32_t packet = (p | 63u) < A.P.num_paths ? A.P.packet : 0u;
        count_rays(A.F.counters + 1u * kQueueShards, 1u);
        HitRec h;
        uint32_t nv = 0, nt = 0;
        if (packet & 1u)
            traverse8_packet<false, false>(A.S, pr.start, pr.dir, 0.0f, pr.length, 1 <= set.MaxAnyHitPathLength, true, h);
        else
            traverse<8, false, false>(A.S, pr.start, pr.dir, 0.0f, pr.length, 1 <= set.MaxAnyHitPathLength, nullptr, h, nv, nt);
        VertexIn V;
        V.inOrigin = pr.start;
        V.inDir = pr.dir;
        V.pathThr = f3{1.0f, 1.0f, 1.0f};
        V.payloadRoughness = 0.0f;
        V.payloadIsDiffuse = false;
        V.pix = pr.pixelIdx;
        V.hit = make_float4(h.b1, h.b2, bitsf(h.tri), bitsf(h.geom));
        VertexOut O;
        uint32_t nsh = 0;
        bool sun0 = false;
        path_vertex(A, 1, V, [&](int kind, f3 o, f3 dd, float tmn, float tmx, f3 c, bool fo) {
            sun0 |= kind == kShadowSun || !DXRPT_SUN0_CHECK;
            emit_shadow(A, p, nsh, o, dd, tmn, tmx, c, fo);
        }, O);
        count_rays(A.F.counters + (kMaxDepthQueues + 1u) * kQueueShards, nsh);
        cont = O.cont;
        nextDiffuse = O.nextIsDiffuse;
        if (cont) {
            Q.org[p] = make_float4(O.nextOrigin.x, O.nextOrigin.y, O.nextOrigin.z, bitsf(pr.accumIdx));
            Q.dir[p] = make_float4(O.nextDir.x, O.nextDir.y, O.nextDir.z, bitsf(pr.pixelIdx));
            Q.thr[p] = make_float4(O.nextThr.x, O.nextThr.y, O.nextThr.z, O.nextRoughness);
        }
        rad = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        rad.x += 1.0f * O.local.x;
        rad.y += 1.0f * O.local.y;
        rad.z += 1.0f * O.local.z;
        vertex_shadows(A, 1, p, nsh, sun0, packet, rad);
        if (!cont) {
            accumulate_pixel(A, pr.accumIdx, rad);
            return;
        }
    }
    for (int d = 2; d <= L - 1; ++d) {
        Q.rad[p] = make_float4(rad.x, rad.y, rad.z, bitsf(nextDiffuse ? 1u : 0u));
        count_rays(A.F.counters + uint32_t(d) * kQueueShards, 1u);
        HitRec h;
        {
            const float4 o4 = Q.org[p], d4 = Q.dir[p];
            uint32_t nv = 0, nt = 0;
            traverse<8, false, false>(A.S, ld3(o4), ld3(d4), kRayTMin, kFP32Max, d <= set.MaxAnyHitPathLength, nullptr, h, nv, nt);
        }
        const float4 o4 = Q.org[p], d4 = Q.dir[p], t4 = Q.thr[p], r4 = Q.rad[p];
        const uint32_t accumIdx = fbits(o4.w);
        VertexIn V;
        V.inOrigin = ld3(o4);
        V.inDir = ld3(d4);
        V.pathThr = ld3(t4);
        V.payloadRoughness = t4.w;
        V.payloadIsDiffuse = (fbits(r4.w) & 1u) != 0u;
        V.pix = fbits(d4.w);
        V.hit = make_float4(h.b1, h.b2, bitsf(h.tri), bitsf(h.geom));
        VertexOut O;
        uint32_t nsh = 0;
        path_vertex(A, d, V, [&](int, f3 o, f3 dd, float tmn, float tmx, f3 c, bool fo) {
            emit_shadow(A, p, nsh, o, dd, tmn, tmx, c, fo);
        }, O);
        count_rays(A.F.counters + (kMaxDepthQueues + uint32_t(d)) * kQueueShards, nsh);
        cont = O.cont;
        nextDiffuse = O.nextIsDiffuse;
        if (cont) {
            Q.org[p] = make_float4(O.nextOrigin.x, O.nextOrigin.y, O.nextOrigin.z, bitsf(accumIdx));
            Q.dir[p] = make_float4(O.nextDir.x, O.nextDir.y, O.nextDir.z, d4.w);
            Q.thr[p] = make_float4(O.nextThr.x, O.nextThr.y, O.nextThr.z, O.nextRoughness);
        }
        rad = make_float4(r4.x, r4.y, r4.z, 0.0f);
        rad.x += V.pathThr.x * O.local.x;
        rad.y += V.pathThr.y * O.local.y;
        rad.z += V.pathThr.z * O.local.z;
        vertex_shadows(A, d, p, nsh, false, 0u, rad);
        if (!cont) {
            accumulate_pixel(A, accumIdx, rad);
            return;
        }
    }
}

// Cost-ordered dispatch (FrameParams::wave_order / wave_cost): the hardware starts waves in launch order,
// so a frame ends with the waves started last; running the costliest wave slots (last frame's
// durations: the image changes little between progressive frames) first leaves short ones for the
// end and shortens the tail in which resident slots run dry (scripts/wave_clocks.py busy_frac).
// Which lanes trace which paths is unchanged -- only the order of whole waves -- so images are equal.
struct WaveSlot {
    uint32_t slot;
    unsigned long long t0;
};

// FrameParams::xcd_chunk: position of launch index i (of n, one wave per workgroup, workgroup i on XCD
// i mod 8) when each XCD takes runs of C consecutive positions, the runs dealt in rotation: run t of
// XCD x is run 8 t + (x + t) mod 8.  A bijection on [0, n) (the last partial group stays in order).
PT_DEV uint32_t xcd_position(uint32_t i, uint32_t n, uint32_t C) {
    const uint32_t full = n / (8u * C) * (8u * C);
    const uint32_t k = i >> 3, t = k / C;
    return i < full ? (t * 8u + (((i & 7u) + t) & 7u)) * C + k % C : i;
}

PT_DEV WaveSlot wave_slot(const KArgs& A, uint32_t* half = nullptr) {
    WaveSlot ws;
    uint32_t w = uint32_t(__builtin_amdgcn_readfirstlane(int((blockIdx.x * blockDim.x + threadIdx.x) >> 6)));
    if (half) {  // path groups: the costliest split_units slots run as two half waves each (half 1, 2)
        const uint32_t k = A.P.split_units;
        *half = w < 2u * k ? 1u + (w & 1u) : 0u;
        w = w < 2u * k ? w >> 1 : w - k;
    }
    ws.slot = w;
    if (A.P.wave_order) {
#if DXRPT_ORDER_XCD
        // the cost order's neighbours (same class, path order within it) on one XCD
        if (A.P.xcd_chunk && !(half && A.P.split_units)) w = xcd_position(w, gridDim.x * (blockDim.x >> 6), A.P.xcd_chunk);
#endif
        ws.slot = A.P.wave_order[w];
    }
    ws.t0 = A.P.wave_cost ? __builtin_amdgcn_s_memrealtime() : 0ull;
    return ws;
}

// A split slot (half 1 / 2) keeps its unsplit class: half 1 counts it again in the histogram, so the
// next order holds it among the costliest (its clock stamps are half 1's).
PT_DEV void wave_slot_split_done(const KArgs& A, const WaveSlot& ws, uint32_t half) {
    if (!A.P.wave_cost || half != 1u || (threadIdx.x & 63u) != 0u) return;
    atomicAdd(&A.P.wave_hist[A.P.wave_cost[ws.slot]], 1u);
    if (A.P.wave_clock) {
        A.P.wave_clock[2 * ws.slot] = ws.t0;
        A.P.wave_clock[2 * ws.slot + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

PT_DEV void wave_slot_done(const KArgs& A, const WaveSlot& ws) {
    if (!A.P.wave_cost) return;
    const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - ws.t0;
    // class: 16 octaves (2^4 .. 2^19 ticks of 10 ns) x 16 steps within an octave, costliest = 0
    const uint32_t d = dt > 0xFFFFFull ? 0xFFFFFu : uint32_t(dt) | 16u;
    const uint32_t lg = 31u - uint32_t(__builtin_clz(d));
    const uint32_t key = (lg - 4u) * 16u + ((d << (31u - lg)) >> 27 & 15u);
    if ((threadIdx.x & 63u) == 0u) {  // vector store and atomic from lane 0
        A.P.wave_cost[ws.slot] = kWaveClasses - 1u - key;
        atomicAdd(&A.P.wave_hist[kWaveClasses - 1u - key], 1u);
        if (A.P.wave_clock) {  // DXRPT_OPT_WAVE_CLOCKS on an ordered frame: the slot's start and end
            A.P.wave_clock[2 * ws.slot] = ws.t0;
            A.P.wave_clock[2 * ws.slot + 1] = ws.t0 + dt;
        }
    }
}

// One thread per wave slot, kWaveClasses threads per workgroup: the class offsets (exclusive scan of
// the histogram, per workgroup), ranks within the workgroup (LDS atomics), one global reservation per
// (workgroup, class).
__global__ __launch_bounds__(kWaveClasses) void k_wave_order(const uint32_t* cls, const uint32_t* hist, uint32_t* cursor,
                                                             uint32_t* hist_next, uint32_t* cursor_next, uint32_t* order,
                                                             uint32_t n) {
    __shared__ uint32_t scan[kWaveClasses], lcount[kWaveClasses], lbase[kWaveClasses];
    const uint32_t t = threadIdx.x;
    uint32_t v = hist[t];
    const uint32_t own = v;
    scan[t] = v;
    lcount[t] = 0u;
    for (uint32_t off = 1; off < kWaveClasses; off <<= 1) {
        __syncthreads();
        const uint32_t add = t >= off ? scan[t - off] : 0u;
        __syncthreads();
        scan[t] = v = v + add;
    }
    __syncthreads();
    scan[t] = v - own;
    const uint32_t i = blockIdx.x * kWaveClasses + t;
    uint32_t c = 0, r = 0;
    if (i < n) {
        c = cls[i];
        r = atomicAdd(&lcount[c], 1u);
    }
    __syncthreads();
    if (lcount[t]) lbase[t] = atomicAdd(&cursor[t], lcount[t]);
    __syncthreads();
    if (i < n) order[scan[c] + lbase[c] + r] = i;
    if (blockIdx.x == 0u) {
        hist_next[t] = 0u;
        cursor_next[t] = 0u;
    }
}

hipError_t launch_wave_order(const uint32_t* cls, const uint32_t* hist, uint32_t* cursor, uint32_t* hist_next,
                             uint32_t* cursor_next, uint32_t* order, uint32_t n, hipStream_t stream) {
    hipLaunchKernelGGL(k_wave_order, dim3((n + kWaveClasses - 1u) / kWaveClasses), dim3(kWaveClasses), 0, stream, cls,
                       hist, cursor, hist_next, cursor_next, order, n);
    return hipGetLastError();
}

// kPersistent: a grid sized to the resident waves; each wave takes the next 64 paths (one 8x8 pixel
// block) from a frame counter until the frame is done, so no wave idles while a long one finishes.
// kLds: the workgroup first copies the top A.P.lds_nodes BVH8 nodes (breadth-first, so the levels
// every ray visits) behind the stacks; the per-lane traversals read those from LDS.
// kGroup: path groups of 64 / A.P.mega_lanes lanes (its own instantiation, so the default kernel's
// register allocation does not carry the group schedule).
// kOrder: the cost-ordered dispatch (wave_slot); its own instantiation, so that the path-ordered
// kernel of large frames keeps its code (the indirection costs it ~2 %).
template <int kOcc, bool kPersistent, bool kLds = false, bool kGroup = false, bool kCount = false, bool kOrder = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kOcc > 0 ? kOcc : 1)))
void k_path(KArgs A) {
    if (A.F.counters_next && blockIdx.x == 0u)  // the next frame's counter set (this stream's previous frame's)
        for (uint32_t i = threadIdx.x; i < kCounterWords; i += blockDim.x) A.F.counters_next[i] = 0u;
    lut_fill(A.S);
    extern __shared__ int stack[];
#if DXRPT_STACK_TID
    lds_int* stk = nullptr;  // 64-thread workgroups: the base is the lane's, recomputed per access (stack_base)
#else
    lds_int* stk = lane_stack(A.S, stack);
#endif
    if (kGroup) {  // mega_lanes paths per wave, each traced by 64 / mega_lanes lanes
        const uint32_t lane = threadIdx.x & 63u;
        uint32_t half = 0;
        const WaveSlot ws = wave_slot(A, &half);
        // a split slot's half h traces paths [(h - 1) g, h g) of the slot with g = mega_lanes / 2
        const uint32_t g = half ? A.P.mega_lanes >> 1 : A.P.mega_lanes;
        const uint32_t q = ws.slot * A.P.mega_lanes + (half ? (half - 1u) * g : 0u) + (lane & (g - 1u));
        if (q < A.P.num_paths) camera_path_group(A, q, stk, lane < g, g);
        if (half) wave_slot_split_done(A, ws, half);
        else wave_slot_done(A, ws);
        return;
    }
    if (!kPersistent && !kLds && !kCount && kOrder) {
        const WaveSlot ws = wave_slot(A);
        const uint32_t p = (ws.slot << 6) | (threadIdx.x & 63u);
        if (p < A.P.num_paths) {
            if (DXRPT_MEGA_STAGE) camera_path_staged(A, p);
            else camera_path(A, p, stk);
        }
        wave_slot_done(A, ws);
        return;
    }
    if (!kPersistent) {
        const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
        if (kLds) {
            const NodeCache nc = node_cache_fill(A.S, reinterpret_cast<uint4*>(stack + A.S.stack_ints * blockDim.x),
                                                 A.P.lds_nodes);
            if (p < A.P.num_paths) camera_path(A, p, stk, nc);
            return;
        }
        if (kCount) {  // census (DXRPT_OPT_COUNT_TRAVERSAL): wave sums, one 64-bit atomic per counter per wave
            const unsigned long long t0 = A.P.wave_clock ? __builtin_amdgcn_s_memrealtime() : 0ull;
            uint32_t cnt[5] = {0u, 0u, 0u, 0u, 0u};
            if (p < A.P.num_paths) camera_path<true>(A, p, stk, NodeCache{nullptr, 0u}, cnt);
            if (A.P.wave_clock && (threadIdx.x & 63u) == 0u && p < A.P.num_paths) {  // vector stores from lane 0
                const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
                A.P.wave_clock[2 * (p >> 6)] = t0;
                A.P.wave_clock[2 * (p >> 6) + 1] = t1;
            }
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                uint32_t v = cnt[k];
                for (int off = 32; off > 0; off >>= 1) v += uint32_t(__shfl_xor(int(v), off));
                if ((threadIdx.x & 63u) == 0u) atomicAdd(&A.P.trav[k], (unsigned long long)v);
            }
            return;
        }
#if DXRPT_DIAG_PHASES
        PhaseAcc pa = {{0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}, uint32_t(__builtin_amdgcn_s_memrealtime())};
        if (p < A.P.num_paths) camera_path(A, p, stk, NodeCache{nullptr, 0u}, nullptr, &pa);
        phase_mark(&pa, 7);
        phase_flush(&pa);
        return;
#endif
        if (A.P.xcd_chunk) {  // XCD-local runs of blocks (FrameParams::xcd_chunk); the tail stays in order
            // run t of XCD x is chunk 8 t + (x + t) mod 8: the XCDs' chunks rotate from run to run, so no
            // XCD keeps the same screen columns (a fixed deal makes stripes of unequal cost)
            const uint32_t q = xcd_position(blockIdx.x, gridDim.x, A.P.xcd_chunk) * blockDim.x + threadIdx.x;
            if (q < A.P.num_paths) {
                if (DXRPT_MEGA_STAGE) camera_path_staged(A, q);
                else camera_path(A, q, stk);
            }
            return;
        }
        if (p >= A.P.num_paths) return;
        if (DXRPT_MEGA_STAGE) camera_path_staged(A, p);
        else camera_path(A, p, stk);
        return;
    }
    uint32_t* work = A.F.counters + 2 * kMaxDepthQueues * kQueueShards;
    const uint32_t lane = threadIdx.x & 63u;
    for (;;) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(work, 64u);
        base = __builtin_amdgcn_readfirstlane(__shfl(base, 0));
        if (base >= A.P.num_paths) break;  // uniform: every wave reaches it once the counter passes the frame
        if (base + lane < A.P.num_paths) camera_path(A, base + lane, stk);
    }
}

// ---- depth-split megakernel (FrameParams::split) ---------------------------------------------
// The frame as one megakernel launch per path depth: k_path_head runs every camera path from raygen
// through its first vertex (packet primaries and depth-1 sun shadows: the coherent part); k_path_tail(d)
// runs depth d of the paths still alive.  Between depths the surviving paths are compacted -- wave64
// ballot + popcount, one atomic per wave on a sharded counter -- into a queue whose entries carry the
// whole path state, so every tail wave is full of live paths (the single k_path keeps a lane per path
// for all L - 1 depths, idle once its path ended), and the path state lives in the queue rather than in
// registers across the traversals: a tail keeps only the queue position and the ray across its
// closest-hit traversal and re-reads the rest afterwards, and every kernel queues the continuation
// BEFORE tracing the vertex's shadow rays, so only the radiance sum is live across them.  Each kernel
// has its own register budget (FrameParams::megakernel_occupancy / tail_occupancy).  A path's radiance
// is k_path's sum, continued term by term from the queued partial sum, so frames are bit-identical.
// Queue of depth d (RayQueue q[d & 1], counters d, shard = producer wave mod kQueueShards):
//   org (origin xyz, FP32Max)   dir (direction xyz, bits(accumulation index))
//   thr (throughput rgb, payload Roughness)   rad (radiance so far, bits(payload IsDiffuse))   pix (CMJ pattern)
// The queued count of depth d is that depth's radiance-ray count (dxrpt_get_stats).

// Queues the continuation of a vertex (all active lanes must call; `cont` selects) into queue d + 1;
// returns its position.  The radiance word is written later (split_finish), after the shadow rays.
// Producer wave w of nw (in screen order) appends to shard w * 64 / nw: each shard holds a contiguous
// run of screen blocks, so the next depth's waves, which take the queue in shard order, sweep the
// image like the head's (neighbouring origins resident together share the BVH nodes and texels in
// cache), while the waves running at any time still spread their atomics over several shards.
// split_bins: shard 8 r + octant(continuation direction), r = the producer's screen region (8, in producer
// order): a tail wave then holds rays of one octant from one region -- the same near-to-far child order
// and nearby origins, so its lanes walk similar node sequences (fewer idle lanes, more shared lines).
PT_DEV uint32_t split_push(const KArgs& A, int d, bool cont, const VertexOut& O, uint32_t pix, uint32_t accumIdx,
                           uint32_t w, uint32_t nw) {
    uint32_t* ctr = A.F.counters + uint32_t(d + 1) * kQueueShards;
    uint32_t pos;
    if (A.P.split_bins) {
        const uint32_t region = uint32_t((uint64_t(w) * (kQueueShards / kSplitBins)) / nw);
        const uint32_t oct = (O.nextDir.x < 0.0f ? 4u : 0u) | (O.nextDir.y < 0.0f ? 2u : 0u) | (O.nextDir.z < 0.0f ? 1u : 0u);
        pos = queue_append_oct(ctr, A.F.cap_q, cont, region * kSplitBins, oct);
    } else {
        pos = queue_append(ctr, A.F.cap_q, cont, uint32_t((uint64_t(w) * kQueueShards) / nw));
    }
    if (cont) {
        const RayQueue& Q = A.F.q[(d + 1) & 1];
        Q.org[pos] = make_float4(O.nextOrigin.x, O.nextOrigin.y, O.nextOrigin.z, kFP32Max);
        Q.dir[pos] = make_float4(O.nextDir.x, O.nextDir.y, O.nextDir.z, bitsf(accumIdx));
        Q.thr[pos] = make_float4(O.nextThr.x, O.nextThr.y, O.nextThr.z, O.nextRoughness);
        Q.pix[pos] = pix;
    }
    return pos;
}

// The vertex's radiance sum: into its queued continuation, or the pixel if the path ended here.
PT_DEV void split_finish(const KArgs& A, int d, bool cont, uint32_t qpos, bool nextDiffuse, uint32_t accumIdx,
                         const float4& rad) {
    if (cont)
        A.F.q[(d + 1) & 1].rad[qpos] = make_float4(rad.x, rad.y, rad.z, bitsf(nextDiffuse ? 1u : 0u));
    else
        finish_pixel(A, accumIdx, rad);
}

// Raygen + depth 1 of every camera path (one 64-path 8x8 block per wave, XCD runs as k_path).
template <int kOcc>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kOcc > 0 ? kOcc : 1)))
void k_path_head(KArgs A) {
    if (A.F.counters_next && blockIdx.x == 0u)  // the next frame's counter set (see k_path)
        for (uint32_t i = threadIdx.x; i < kCounterWords; i += blockDim.x) A.F.counters_next[i] = 0u;
    lut_fill(A.S);
    const uint32_t blk = A.P.xcd_chunk ? xcd_position(blockIdx.x, gridDim.x, A.P.xcd_chunk) : blockIdx.x;
    const uint32_t p = blk * blockDim.x + threadIdx.x;  // path slot within this launch (shadow-slot index)
    if (p >= A.P.num_paths) return;
    const dxrpt_app_settings& set = A.P.set;
    const PrimaryRay pr = primary_ray(A, A.P.path_base + p);
    const uint32_t packet = (p | 63u) < A.P.num_paths ? A.P.packet : 0u;
    count_rays(A.F.counters + 1u * kQueueShards, 1u);
    HitRec h;
    uint32_t nv = 0, nt = 0;
    if (packet & 1u)  // coherent primary rays: wave-coherent traversal (same results)
        traverse8_packet<false, false, (DXRPT_HEAD_PACKET_PAIR & 1) != 0>(A.S, pr.start, pr.dir, 0.0f, pr.length, 1 <= set.MaxAnyHitPathLength, true, h);
    else
        traverse<8, false, false>(A.S, pr.start, pr.dir, 0.0f, pr.length, 1 <= set.MaxAnyHitPathLength, nullptr, h, nv, nt);
    VertexIn V;
    V.inOrigin = pr.start;
    V.inDir = pr.dir;
    V.pathThr = f3{1.0f, 1.0f, 1.0f};
    V.payloadRoughness = 0.0f;
    V.payloadIsDiffuse = false;
    V.pix = pr.pixelIdx;
    V.hit = make_float4(h.b1, h.b2, bitsf(h.tri), bitsf(h.geom));
    VertexOut O;
    uint32_t nsh = 0;
    bool sun0 = false;
    path_vertex(A, 1, V, [&](int kind, f3 o, f3 dd, float tmn, float tmx, f3 c, bool fo) {
        sun0 |= kind == kShadowSun || !DXRPT_SUN0_CHECK;
        emit_shadow(A, p, nsh, o, dd, tmn, tmx, c, fo);
    }, O);
    count_rays(A.F.counters + (kMaxDepthQueues + 1u) * kQueueShards, nsh);
    const bool cont = O.cont;
    const bool nextDiffuse = O.nextIsDiffuse;
    const uint32_t qpos = split_push(A, 1, cont, O, pr.pixelIdx, pr.accumIdx, blk, gridDim.x);
    float4 rad = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    rad.x += 1.0f * O.local.x;
    rad.y += 1.0f * O.local.y;
    rad.z += 1.0f * O.local.z;
    vertex_shadows(A, 1, p, nsh, sun0, packet, rad);
    split_finish(A, 1, cont, qpos, nextDiffuse, pr.accumIdx, rad);
}

// Depth d of the paths queued for it (one per lane); waves past the queued count exit at once (the grid
// covers every path of the frame).
template <int kOcc>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kOcc > 0 ? kOcc : 1)))
void k_path_tail(KArgs A, int d) {
    const uint32_t* cnt = A.F.counters + uint32_t(d) * kQueueShards;
    const uint32_t n = queue_total(cnt);
    const uint32_t nw = (n + 63u) / 64u;  // waves with work
    // wave j of the queue: XCD runs of A.P.xcd_chunk consecutive queue chunks among the nw live waves
    // (workgroup b runs on XCD b mod 8; the grid's surplus workgroups exit at once)
    if (blockIdx.x >= nw) return;
    const uint32_t j = A.P.xcd_chunk ? xcd_position(blockIdx.x, nw, A.P.xcd_chunk) : blockIdx.x;
    lut_fill(A.S);
    const uint32_t i = j * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const dxrpt_app_settings& set = A.P.set;
    const uint32_t pos = queue_pos(cnt, A.F.cap_q, i);
    const RayQueue& Q = A.F.q[d & 1];
    HitRec h;
    {
        const float4 o4 = Q.org[pos], d4 = Q.dir[pos];
        uint32_t nv = 0, nt = 0;
        traverse<8, false, false, DXRPT_SPLIT_PIPE_CH>(A.S, ld3(o4), ld3(d4), kRayTMin, o4.w, d <= set.MaxAnyHitPathLength, nullptr, h, nv, nt);
    }
    // the rest of the path state comes back from the queue after the traversal (the radiance so far only
    // once the vertex is shaded: it is not live across path_vertex)
    const float4 o4 = Q.org[pos], d4 = Q.dir[pos], t4 = Q.thr[pos];
    const float rw = reinterpret_cast<const float*>(Q.rad + pos)[3];
    const uint32_t accumIdx = fbits(d4.w);
    VertexIn V;
    V.inOrigin = ld3(o4);
    V.inDir = ld3(d4);
    V.pathThr = ld3(t4);
    V.payloadRoughness = t4.w;
    V.payloadIsDiffuse = (fbits(rw) & 1u) != 0u;
    V.pix = Q.pix[pos];
    V.hit = make_float4(h.b1, h.b2, bitsf(h.tri), bitsf(h.geom));
    VertexOut O;
    uint32_t nsh = 0;
    path_vertex(A, d, V, [&](int, f3 o, f3 dd, float tmn, float tmx, f3 c, bool fo) {
        emit_shadow(A, i, nsh, o, dd, tmn, tmx, c, fo);  // shadow slots by the dense index (< qsize)
    }, O);
    count_rays(A.F.counters + (kMaxDepthQueues + uint32_t(d)) * kQueueShards, nsh);
    const bool cont = O.cont;
    const bool nextDiffuse = O.nextIsDiffuse;
    const int L = set.MaxPathLength < 2 ? 2 : set.MaxPathLength;
    const uint32_t qpos = d + 1 <= L - 1 ? split_push(A, d, cont, O, V.pix, accumIdx, j, nw) : 0u;
    const float4 r4 = Q.rad[pos];
    float4 rad = make_float4(r4.x, r4.y, r4.z, 0.0f);
    rad.x += V.pathThr.x * O.local.x;
    rad.y += V.pathThr.y * O.local.y;
    rad.z += V.pathThr.z * O.local.z;
    vertex_shadows(A, d, i, nsh, false, 0u, rad);
    split_finish(A, d, cont, qpos, nextDiffuse, accumIdx, rad);
}

// ---- lightmap baking (Baking.hlsl:336-465, BakeRayGen) -------------------------------------------
// One thread per lightmap texel of the chunk [first, first + count): the surface map's world position
// and normal (SurfaceMap.hlsl raster), a tangent frame from the normal, CMJ set 0 at the texel index
// (TotalNumPixels = the lightmap's texel count, DXRPathTracer.cpp:1934-1935), a cosine-hemisphere ray
// traced as a PathLength-1 diffuse path (the same trace_path as the camera paths), the firefly clamp
// against the running average and the valid-sample accumulation (rgb sum, count), then the average
// into the lightmap.  Bad inputs write the reference's marker colours.
PT_DEV float luma(float3 c) { return (c.x * 0.299f + c.y * 0.587f) + c.z * 0.114f; }

template <int kOcc>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kOcc > 0 ? kOcc : 1)))
void k_bake(KArgs A, BakeArgs B) {
    lut_fill(A.S);
    extern __shared__ int stack[];
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B.span || B.first + i >= *B.count) return;
    const uint32_t texel = B.list[B.first + i];
    const float4 pos4 = B.pos[texel];  // w != 0: inside a UV island (Baking.hlsl:351-354 in the compaction)
    const f3 worldPos = f3{pos4.x, pos4.y, pos4.z};
    if (isinf(worldPos.x) || isinf(worldPos.y) || isinf(worldPos.z)) {
        B.lightmap[texel] = make_float4(0.0f, 0.0f, 1.0f, 1.0f);
        return;
    }
    const float4 n4 = B.nrm[texel];
    const f3 nv = f3{n4.x, n4.y, n4.z};
    if (dot3(nv, nv) < 0.0001f) {
        B.lightmap[texel] = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
        return;
    }
    const f3 N = normalize3(nv);
    const f3 up = fabsf(N.z) < 0.999f ? f3{0.0f, 0.0f, 1.0f} : f3{1.0f, 0.0f, 0.0f};
    const f3 T = normalize3(cross3(up, N));
    const f3 Bt = cross3(N, T);
    float sx, sy;
    const uint32_t nS = uint32_t(A.P.set.SqrtNumSamples);
    sample_cmj2d(A.P.rtc.CurrSampleIdx, nS, nS, 0u * A.P.rtc.TotalNumPixels + texel, &sx, &sy);
    const f3 dTS = sample_cosine_hemisphere(sx, sy);
    const f3 dir = add(add(scl(T, dTS.x), scl(Bt, dTS.y)), scl(N, dTS.z));  // mul(dirTS, float3x3(T, B, N))
    const f3 origin = add(worldPos, scl(dir, 0.00001f));
    const bool badO = isinf(origin.x) || isinf(origin.y) || isinf(origin.z) || isnan(origin.x) || isnan(origin.y) || isnan(origin.z);
    const bool badD = isinf(dir.x) || isinf(dir.y) || isinf(dir.z) || isnan(dir.x) || isnan(dir.y) || isnan(dir.z) ||
                      len3(dir) < 0.001f;
    if (badO || badD) {
        B.lightmap[texel] = make_float4(1.0f, 0.0f, 1.0f, 1.0f);
        return;
    }
#if DXRPT_STACK_TID
    const float4 r = trace_path<true>(A, i, texel, origin, dir, kFP32Max, nullptr, 0u);  // 64-thread workgroups
#else
    const float4 r = trace_path<true>(A, i, texel, origin, dir, kFP32Max, lane_stack(A.S, stack), 0u);
#endif
    float3 c = make_float3(r.x, r.y, r.z);
    const float4 prev = B.accum[texel];
    float3 sum = make_float3(prev.x, prev.y, prev.z);
    float n = prev.w;
    if (n >= 1.0f) {  // firefly clamp against the running average (x10 its luminance)
        const float3 avg = make_float3(sum.x / n, sum.y / n, sum.z / n);
        const float avgL = luma(avg) + 0.001f;
        const float sL = luma(c);
        if (sL > avgL * 10.0f) {
            const float k = avgL * 10.0f / sL;
            c = make_float3(c.x * k, c.y * k, c.z * k);
        }
    }
    const bool valid = !(isnan(c.x) || isnan(c.y) || isnan(c.z)) && !(luma(c) < 0.0001f);
    if (valid) {
        sum = make_float3(sum.x + c.x, sum.y + c.y, sum.z + c.z);
        n += 1.0f;
    }
    B.accum[texel] = make_float4(sum.x, sum.y, sum.z, n);
    const float3 avg = n > 0.0f ? make_float3(sum.x / n, sum.y / n, sum.z / n) : make_float3(0.0f, 0.0f, 0.0f);
    B.lightmap[texel] = make_float4(avg.x, avg.y, avg.z, 1.0f);
}

// Arbitrary ray queries (dxrpt_trace_rays): flags bit0 = any-hit (shadow) semantics,
// bit1 = alpha test enabled (not FORCE_OPAQUE).
template <int W>
__global__ __launch_bounds__(kBlock) void k_trace_rays(SceneDev S, const float4* rays, uint32_t n, uint32_t flags, float4* hits) {
    lut_fill(S);
    extern __shared__ int stack[];  // S.stack_ints per lane, lane-interleaved (launch_lds_bytes)
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float4 a = rays[2 * i], b = rays[2 * i + 1];
    HitRec h;
    uint32_t nv = 0, nt = 0;
    const bool alpha = (flags & 2u) != 0u;
    if (flags & 1u) {
        bool occ = traverse<W, true, false>(S, ld3(a), ld3(b), a.w, b.w, alpha, lane_stack(S, stack), h, nv, nt);
        hits[i] = make_float4(occ ? 1.0f : -1.0f, 0.0f, 0.0f, bitsf(kMiss));
    } else {
        bool any = traverse<W, false, false>(S, ld3(a), ld3(b), a.w, b.w, alpha, lane_stack(S, stack), h, nv, nt);
        hits[i] = any ? make_float4(h.t, h.b1, h.b2, bitsf(h.tri)) : make_float4(-1.0f, 0.0f, 0.0f, bitsf(kMiss));
    }
}

static inline uint32_t grid_for(uint32_t n) { return (n + kBlock - 1) / kBlock; }

// Grid of the wave-pool kernel over a queue of at most n items (4 waves per workgroup).
static inline uint32_t pool_grid(uint32_t n, uint32_t chunks_per_wave) {
    const uint32_t waves = (n + 64u * chunks_per_wave - 1u) / (64u * chunks_per_wave);
    return (waves + kBlock / 64u - 1u) / (kBlock / 64u);
}

uint32_t frame_traversal_threads(uint32_t num_paths, uint32_t shadow_slots, uint32_t chunks_per_wave) {
    const uint32_t gs = grid_for(num_paths * shadow_slots);
    uint32_t g = std::max(grid_for(num_paths), gs);
    if (chunks_per_wave)
        g = std::max(g, std::max(pool_grid(num_paths, chunks_per_wave), pool_grid(num_paths * shadow_slots, chunks_per_wave)));
    return g * kBlock;
}

uint32_t trace_rays_threads(uint32_t n) { return grid_for(n) * kBlock; }

template <int kOcc>
static void launch_head(const KArgs& A, uint32_t g, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL((k_path_head<kOcc>), dim3(g), dim3(64), lds, s, A);
}
template <int kOcc>
static void launch_tail(const KArgs& A, uint32_t g, size_t lds, hipStream_t s, int d) {
    hipLaunchKernelGGL((k_path_tail<kOcc>), dim3(g), dim3(64), lds, s, A, d);
}

// The depth-split schedule (FrameParams::split): the head, then one tail launch per depth.
static void launch_split(const KArgs& A, uint32_t gm, size_t lds, hipStream_t s) {
    const FrameParams& fp = A.P;
    const int L = fp.set.MaxPathLength < 2 ? 2 : fp.set.MaxPathLength;
    switch (fp.megakernel_occupancy) {
        case 8: launch_head<8>(A, gm, lds, s); break;
        case 7: launch_head<7>(A, gm, lds, s); break;
        case 6: launch_head<6>(A, gm, lds, s); break;
        case 5: launch_head<5>(A, gm, lds, s); break;
        default: launch_head<4>(A, gm, lds, s); break;
    }
    for (int d = 2; d <= L - 1; ++d) {
        switch (fp.tail_occupancy) {
            case 8: launch_tail<8>(A, gm, lds, s, d); break;
            case 7: launch_tail<7>(A, gm, lds, s, d); break;
            case 6: launch_tail<6>(A, gm, lds, s, d); break;
            case 5: launch_tail<5>(A, gm, lds, s, d); break;
            default: launch_tail<4>(A, gm, lds, s, d); break;
        }
    }
}

hipError_t launch_split_part(const SceneDev& scene, const FrameBuffers& fb, const FrameParams& fp, hipStream_t stream) {
    if (!fb.counters_clean) {
        const hipError_t e = hipMemsetAsync(fb.counters, 0, kCounterWords * sizeof(uint32_t), stream);
        if (e != hipSuccess) return e;
    }
    if (fp.num_paths == 0) return hipSuccess;
    KArgs A{scene, fb, fp};
    const size_t lds = size_t(scene.stack_ints) * 64u * sizeof(int);
    launch_split(A, (fp.num_paths + 63u) / 64u, lds, stream);
    return hipGetLastError();
}

hipError_t launch_accum_stage(const FrameParams& fp, hipStream_t stream) {
    if (fp.num_paths == 0 || !fp.stage) return hipSuccess;
    KArgs A{SceneDev{}, FrameBuffers{}, fp};
    hipLaunchKernelGGL(k_accum_stage, dim3((fp.num_paths + kBlock - 1u) / kBlock), dim3(kBlock), 0, stream, A);
    return hipGetLastError();
}

hipError_t launch_frame(const SceneDev& scene, const FrameBuffers& fb, const FrameParams& fp, hipStream_t stream,
                        hipEvent_t* ev, hipStream_t aux, hipEvent_t* fork_ev, uint32_t* sched_out) {
    KArgs A{scene, fb, fp};
    uint32_t sched_local = 0;
    uint32_t& sched = sched_out ? *sched_out : sched_local;
    sched = 0;
    A.P.lds_nodes = scene.width == 8 ? std::min(fp.lds_nodes, scene.num_nodes) : 0u;
    const uint32_t g = grid_for(fp.num_paths);
    const size_t lds = size_t(scene.stack_ints) * kBlock * sizeof(int);
    const bool count = fp.trav != nullptr;
    // per-kernel timing: launch slot i (raygen, then trace/shade/shadow/resolve per depth, then
    // accumulate) is bracketed by ev[2i], ev[2i+1] recorded on the stream the kernel runs on
    // (the frame's first start and last stop events are always recorded: they bracket the frame)
    const int L_ = fp.set.MaxPathLength < 2 ? 2 : fp.set.MaxPathLength;
    const int last_slot = 1 + 4 * (L_ - 1);
    auto timed = [&](int slot) {
        static const uint32_t kinds[4] = {DXRPT_K_TRACE, DXRPT_K_SHADE, DXRPT_K_SHADOW, DXRPT_K_RESOLVE};
        const uint32_t kind = slot == 0 ? DXRPT_K_RAYGEN : slot == last_slot ? DXRPT_K_ACCUMULATE : kinds[(slot - 1) % 4];
        return (fp.timing_mask >> kind) & 1u;
    };
    auto start = [&](int slot, hipStream_t st) {
        if (ev && (slot == 0 || timed(slot))) (void)hipEventRecord(ev[2 * slot], st);
    };
    auto stop = [&](int slot, hipStream_t st) {
        if (ev && (slot == last_slot || timed(slot))) (void)hipEventRecord(ev[2 * slot + 1], st);
    };
    auto slot_of = [](int d, int kind) { return 1 + 4 * (d - 1) + kind; };  // kind 0 trace 1 shade 2 shadow 3 resolve
    static_assert(kCounterWords >= 2 * kMaxDepthQueues * kQueueShards + 1 && kCounterWords % 4 == 0, "counter set");
    hipError_t e = fb.counters_clean ? hipSuccess : hipMemsetAsync(fb.counters, 0, kCounterWords * sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    if (fp.megakernel) {  // whole frame in k_path (timing: ev[0], ev[1] bracket the k_path launch)
        // one wave per workgroup: the per-lane stack base is the lane's (DXRPT_STACK_TID, stack_base)
        const uint32_t tb = 64u;
        const size_t ldsm = size_t(scene.stack_ints) * tb * sizeof(int);
        // mega_lanes < 64 (per-lane path, no persistent grid / LDS nodes): 64 threads per mega_lanes paths.
        // A census frame always runs the 64-lane per-path kernel (one wave per 64 paths).
        const bool twins = fp.mega_lanes < 64u && !fp.mega_persistent && !A.P.lds_nodes && !A.P.trav;
        const uint64_t threads = twins ? ((uint64_t(fp.num_paths) + fp.mega_lanes - 1u) / fp.mega_lanes + fp.split_units) * 64u
                                       : fp.num_paths;
        const uint32_t gm = uint32_t((threads + tb - 1u) / tb);
        const bool ordered = (fp.wave_cost || fp.wave_order) && fp.megakernel_occupancy >= 4 && fp.megakernel_occupancy <= 7;
        sched = DXRPT_SCHED_MEGAKERNEL;
        if (ev) (void)hipEventRecord(ev[0], stream);
        if (A.P.trav) {  // census frame (DXRPT_OPT_COUNT_TRAVERSAL): same schedule, counting instantiation
            sched |= DXRPT_SCHED_CENSUS;
            hipLaunchKernelGGL((k_path<7, false, false, false, true>), dim3(gm), dim3(tb), ldsm, stream, A);
        }
        else if (fp.split && !fp.mega_persistent && !A.P.lds_nodes && !twins && !ordered) {
            sched |= DXRPT_SCHED_SPLIT;
            launch_split(A, gm, ldsm, stream);
        }
        else if (fp.mega_persistent && tb == 64u) {
            const uint32_t gp = std::min(gm, fp.mega_persistent * fp.num_cus);
            // the same register budgets as the non-persistent kernel (A/B at equal occupancy)
            if (fp.megakernel_occupancy >= 7) hipLaunchKernelGGL((k_path<7, true>), dim3(gp), dim3(tb), ldsm, stream, A);
            else if (fp.megakernel_occupancy == 6) hipLaunchKernelGGL((k_path<6, true>), dim3(gp), dim3(tb), ldsm, stream, A);
            else if (fp.megakernel_occupancy == 4) hipLaunchKernelGGL((k_path<4, true>), dim3(gp), dim3(tb), ldsm, stream, A);
            else hipLaunchKernelGGL((k_path<5, true>), dim3(gp), dim3(tb), ldsm, stream, A);
        }
        else if (A.P.lds_nodes) {
            const size_t ldsn = ldsm + size_t(A.P.lds_nodes) * kNode8Stride;
            if (fp.megakernel_occupancy >= 7) hipLaunchKernelGGL((k_path<7, false, true>), dim3(gm), dim3(tb), ldsn, stream, A);
            else if (fp.megakernel_occupancy == 6) hipLaunchKernelGGL((k_path<6, false, true>), dim3(gm), dim3(tb), ldsn, stream, A);
            else if (fp.megakernel_occupancy == 5) hipLaunchKernelGGL((k_path<5, false, true>), dim3(gm), dim3(tb), ldsn, stream, A);
            else hipLaunchKernelGGL((k_path<4, false, true>), dim3(gm), dim3(tb), ldsn, stream, A);
        }
        else if (twins) {  // (cost ordering by FrameParams::wave_order / wave_cost, null: off)
            sched |= DXRPT_SCHED_PATH_GROUPS | (fp.wave_cost || fp.wave_order ? DXRPT_SCHED_ORDER_KERNEL : 0u) |
                     (fp.wave_order ? DXRPT_SCHED_COST_ORDERED : 0u);
            if (fp.megakernel_occupancy >= 7) hipLaunchKernelGGL((k_path<7, false, false, true>), dim3(gm), dim3(tb), ldsm, stream, A);
            else if (fp.megakernel_occupancy == 6) hipLaunchKernelGGL((k_path<6, false, false, true>), dim3(gm), dim3(tb), ldsm, stream, A);
            else if (fp.megakernel_occupancy == 5) hipLaunchKernelGGL((k_path<5, false, false, true>), dim3(gm), dim3(tb), ldsm, stream, A);
            else hipLaunchKernelGGL((k_path<4, false, false, true>), dim3(gm), dim3(tb), ldsm, stream, A);
        }
        else if (ordered) {  // cost-ordered waves
            sched |= DXRPT_SCHED_ORDER_KERNEL | (fp.wave_order ? DXRPT_SCHED_COST_ORDERED : 0u);
            if (fp.megakernel_occupancy == 7) hipLaunchKernelGGL((k_path<7, false, false, false, false, true>), dim3(gm), dim3(tb), ldsm, stream, A);
            else if (fp.megakernel_occupancy == 6) hipLaunchKernelGGL((k_path<6, false, false, false, false, true>), dim3(gm), dim3(tb), ldsm, stream, A);
            else if (fp.megakernel_occupancy == 5) hipLaunchKernelGGL((k_path<5, false, false, false, false, true>), dim3(gm), dim3(tb), ldsm, stream, A);
            else hipLaunchKernelGGL((k_path<4, false, false, false, false, true>), dim3(gm), dim3(tb), ldsm, stream, A);
        }
        else if (fp.megakernel_occupancy == 8) hipLaunchKernelGGL((k_path<8, false>), dim3(gm), dim3(tb), ldsm, stream, A);
        else if (fp.megakernel_occupancy == 7) hipLaunchKernelGGL((k_path<7, false>), dim3(gm), dim3(tb), ldsm, stream, A);
        else if (fp.megakernel_occupancy == 6) hipLaunchKernelGGL((k_path<6, false>), dim3(gm), dim3(tb), ldsm, stream, A);
        else if (fp.megakernel_occupancy == 4) hipLaunchKernelGGL((k_path<4, false>), dim3(gm), dim3(tb), ldsm, stream, A);
        else if (fp.megakernel_occupancy == 5) hipLaunchKernelGGL((k_path<5, false>), dim3(gm), dim3(tb), ldsm, stream, A);
        else hipLaunchKernelGGL((k_path<0, false>), dim3(gm), dim3(tb), ldsm, stream, A);  // 3: the compiler's budget
        if (ev) (void)hipEventRecord(ev[1], stream);
        return hipGetLastError();
    }
    start(0, stream);
    hipLaunchKernelGGL(k_raygen, dim3(g), dim3(kBlock), 0, stream, A);
    stop(0, stream);
    const int L = fp.set.MaxPathLength < 2 ? 2 : fp.set.MaxPathLength;
    const uint32_t tb = fp.trace_block;
    const uint32_t gt = (fp.num_paths + tb - 1u) / tb;
    // any-hit grid: one thread per queued shadow ray (upper bound num_paths * slots; surplus waves
    // exit at once), or a grid-stride loop over a capped grid of shadow_grid 256-thread equivalents
    const uint32_t gst_full = (fp.num_paths * fb.shadow_slots + tb - 1u) / tb;
    const uint32_t gst = fp.shadow_grid ? std::min<uint32_t>(gst_full, fp.shadow_grid * (kBlock / tb)) : gst_full;
    const size_t ldst = size_t(scene.stack_ints) * tb * sizeof(int);
    const size_t ldsc = ldst + size_t(A.P.lds_nodes) * kNode8Stride;  // + the node cache (uncounted BVH8 kernels)
    const bool w8 = scene.width == 8;
    const bool pers = w8 && fp.chunks_per_wave > 0;
    const uint32_t gp = pers ? pool_grid(fp.num_paths, fp.chunks_per_wave) : 0u;
    const uint32_t gps = pers ? pool_grid(fp.num_paths * fb.shadow_slots, fp.chunks_per_wave) : 0u;
    // one-thread-per-ray traversal kernels: <count, width, occupancy>
    auto trace = [&](int d, hipStream_t st) {
#define DXRPT_LAUNCH(K, C, W, O, GG) hipLaunchKernelGGL((K<C, W, O>), dim3(GG), dim3(tb), ldst, st, A, d)
#define DXRPT_LAUNCH_P(K, O, GG)                                                                              \
    switch (A.P.lds_nodes ? 4u : fp.pipeline) {                                                            \
        case 4: hipLaunchKernelGGL((K<false, 8, O, 4>), dim3(GG), dim3(tb), ldsc, st, A, d); break;         \
        case 1: hipLaunchKernelGGL((K<false, 8, O, 1>), dim3(GG), dim3(tb), ldsc, st, A, d); break;         \
        case 2: hipLaunchKernelGGL((K<false, 8, O, 2>), dim3(GG), dim3(tb), ldsc, st, A, d); break;         \
        case 3: hipLaunchKernelGGL((K<false, 8, O, 3>), dim3(GG), dim3(tb), ldsc, st, A, d); break;         \
        default: hipLaunchKernelGGL((K<false, 8, O, 0>), dim3(GG), dim3(tb), ldsc, st, A, d); break;        \
    }
        const bool shadow = d < 0;
        d = shadow ? -d : d;
        const uint32_t G = shadow ? gst_full : gt;
        // packet traversal: bit 0 closest hit at depth 1, bit 1 any hit at depth 1, bits 2/3 deeper
        const uint32_t pbit = (shadow ? 2u : 1u) << (d == 1 ? 0 : 2);
        if (w8 && !count && (fp.packet & pbit)) {
            const uint32_t occ = shadow ? fp.shadow_occupancy : fp.occupancy;
            if (shadow) {
                if (occ == 7) hipLaunchKernelGGL((k_shadow_packet<7>), dim3(G), dim3(tb), ldst, st, A, d);
                else if (occ == 8) hipLaunchKernelGGL((k_shadow_packet<8>), dim3(G), dim3(tb), ldst, st, A, d);
                else hipLaunchKernelGGL((k_shadow_packet<0>), dim3(G), dim3(tb), ldst, st, A, d);
            } else {
                if (occ == 7) hipLaunchKernelGGL((k_trace_packet<7>), dim3(G), dim3(tb), ldst, st, A, d);
                else if (occ == 8) hipLaunchKernelGGL((k_trace_packet<8>), dim3(G), dim3(tb), ldst, st, A, d);
                else hipLaunchKernelGGL((k_trace_packet<0>), dim3(G), dim3(tb), ldst, st, A, d);
            }
            return;
        }
        const uint32_t G2 = shadow ? gst : gt;
        if (!w8) {
            if (shadow) { if (count) DXRPT_LAUNCH(k_shadow, true, 2, 0, G2); else DXRPT_LAUNCH(k_shadow, false, 2, 0, G2); }
            else { if (count) DXRPT_LAUNCH(k_trace, true, 2, 0, G2); else DXRPT_LAUNCH(k_trace, false, 2, 0, G2); }
        } else if (count) {
            if (shadow) DXRPT_LAUNCH(k_shadow, true, 8, 0, G2); else DXRPT_LAUNCH(k_trace, true, 8, 0, G2);
        } else {
            const uint32_t occ = shadow ? fp.shadow_occupancy : fp.occupancy;
            if (occ == 7) { if (shadow) DXRPT_LAUNCH_P(k_shadow, 7, G2) else DXRPT_LAUNCH_P(k_trace, 7, G2) }
            else if (occ == 8) { if (shadow) DXRPT_LAUNCH_P(k_shadow, 8, G2) else DXRPT_LAUNCH_P(k_trace, 8, G2) }
            else { if (shadow) DXRPT_LAUNCH_P(k_shadow, 0, G2) else DXRPT_LAUNCH_P(k_trace, 0, G2) }
        }
#undef DXRPT_LAUNCH
#undef DXRPT_LAUNCH_P
    };
    auto radiance = [&](int d, hipStream_t st) {
        start(slot_of(d, 0), st);
        if (pers) {
            if (count) hipLaunchKernelGGL((k_traverse8p<true, false>), dim3(gp), dim3(kBlock), lds, st, A, d);
            else hipLaunchKernelGGL((k_traverse8p<false, false>), dim3(gp), dim3(kBlock), lds, st, A, d);
        } else {
            trace(d, st);
        }
        stop(slot_of(d, 0), st);
    };
    auto shadow = [&](int d, hipStream_t st) {
        start(slot_of(d, 2), st);
        if (pers) {
            if (count) hipLaunchKernelGGL((k_traverse8p<true, true>), dim3(gps), dim3(kBlock), lds, st, A, d);
            else hipLaunchKernelGGL((k_traverse8p<false, true>), dim3(gps), dim3(kBlock), lds, st, A, d);
        } else {
            trace(-d, st);
        }
        stop(slot_of(d, 2), st);
    };
    // Fork/join (aux != null): k_shadow(d) and k_trace(d+1) both only need k_shade(d), so the any-hit
    // pass runs on `aux` concurrently with the next closest-hit pass; k_resolve(d) joins both before
    // k_shade(d+1).
    const bool fork = aux != nullptr && fork_ev != nullptr;
    for (int d = 1; d <= L - 1; ++d) {
        if (d == 1 || !fork) radiance(d, stream);
        start(slot_of(d, 1), stream);
        {
            const uint32_t sb = fp.shade_block, gsh = (fp.num_paths + sb - 1u) / sb;
            switch (fp.shade_occupancy) {
                case 6: hipLaunchKernelGGL((k_shade<6>), dim3(gsh), dim3(sb), 0, stream, A, d); break;
                case 7: hipLaunchKernelGGL((k_shade<7>), dim3(gsh), dim3(sb), 0, stream, A, d); break;
                case 8: hipLaunchKernelGGL((k_shade<8>), dim3(gsh), dim3(sb), 0, stream, A, d); break;
                default: hipLaunchKernelGGL((k_shade<0>), dim3(gsh), dim3(sb), 0, stream, A, d); break;
            }
        }
        stop(slot_of(d, 1), stream);
        if (fork) {
            if ((e = hipEventRecord(fork_ev[2 * d], stream)) != hipSuccess) return e;
            if ((e = hipStreamWaitEvent(aux, fork_ev[2 * d], 0)) != hipSuccess) return e;
            shadow(d, aux);
            if ((e = hipEventRecord(fork_ev[2 * d + 1], aux)) != hipSuccess) return e;
            if (d + 1 <= L - 1) radiance(d + 1, stream);
            if ((e = hipStreamWaitEvent(stream, fork_ev[2 * d + 1], 0)) != hipSuccess) return e;
        } else {
            shadow(d, stream);
        }
        start(slot_of(d, 3), stream);
        hipLaunchKernelGGL(k_resolve, dim3(g), dim3(kBlock), 0, stream, A, d);
        stop(slot_of(d, 3), stream);
    }
    start(slot_of(L, 0), stream);
    hipLaunchKernelGGL(k_accumulate, dim3(g), dim3(kBlock), 0, stream, A);
    stop(slot_of(L, 0), stream);
    return hipGetLastError();
}

// Live-texel list: one ballot + one atomic per wave; the order of the waves' segments does not matter
// (every texel is independent and keeps its own CMJ pattern index).
__global__ __launch_bounds__(256) void k_bake_compact(const float4* __restrict__ pos, uint32_t texels,
                                                      uint32_t* __restrict__ list, uint32_t* __restrict__ count) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    const bool live = t < texels && pos[t].w != 0.0f;
    const uint64_t m = __ballot(live);
    if (m == 0ull) return;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t leader = uint32_t(__ffsll((unsigned long long)m) - 1);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(count, uint32_t(__popcll(m)));
    base = __shfl(base, int(leader));
    if (live) list[base + uint32_t(__popcll(m & ((1ull << lane) - 1ull)))] = t;
}

hipError_t launch_bake_compact(const float4* pos, uint32_t texels, uint32_t* list, uint32_t* count, hipStream_t stream) {
    hipError_t e = hipMemsetAsync(count, 0, sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_bake_compact, dim3((texels + 255u) / 256u), dim3(256), 0, stream, pos, texels, list, count);
    return hipGetLastError();
}

hipError_t launch_bake(const SceneDev& scene, const FrameBuffers& fb, const FrameParams& fp, const BakeArgs& b,
                       hipStream_t stream) {
    if (b.span == 0) return hipSuccess;
    KArgs A{scene, fb, fp};
    const uint32_t tb = 64;
    const size_t lds = size_t(scene.stack_ints) * tb * sizeof(int);
    const dim3 g((b.span + tb - 1u) / tb);
    if (fp.megakernel_occupancy >= 7) hipLaunchKernelGGL((k_bake<7>), g, dim3(tb), lds, stream, A, b);
    else if (fp.megakernel_occupancy == 6) hipLaunchKernelGGL((k_bake<6>), g, dim3(tb), lds, stream, A, b);
    else if (fp.megakernel_occupancy == 5) hipLaunchKernelGGL((k_bake<5>), g, dim3(tb), lds, stream, A, b);
    else hipLaunchKernelGGL((k_bake<4>), g, dim3(tb), lds, stream, A, b);
    return hipGetLastError();
}

hipError_t launch_trace_rays(const SceneDev& scene, const float4* rays, uint32_t n, uint32_t flags, float4* hits,
                             hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const size_t lds = size_t(scene.stack_ints) * kBlock * sizeof(int);
    if (scene.width == 8)
        hipLaunchKernelGGL((k_trace_rays<8>), dim3(grid_for(n)), dim3(kBlock), lds, stream, scene, rays, n, flags, hits);
    else
        hipLaunchKernelGGL((k_trace_rays<2>), dim3(grid_for(n)), dim3(kBlock), lds, stream, scene, rays, n, flags, hits);
    return hipGetLastError();
}

// Primary-only AOV (SURVEY.md 8(d), C1 plumbing): RaygenShader's ray for path slot p (the tiles of the
// call), its closest hit (packet traversal on full waves, as k_path's depth 1), and the albedo tap
// PathTrace takes at the hit (RayTrace.hlsl:180-183); out[accumIdx] = (albedo rgb, 1) on a hit, 0 on a
// miss.  No shading, no accumulation: a debug view of the ray-generation / traversal / surface plumbing.
__global__ __launch_bounds__(64) void k_primary_aov(KArgs A) {
    lut_fill(A.S);
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= A.P.num_paths) return;
    const PrimaryRay pr = primary_ray(A, p);
    HitRec h;
    uint32_t nv = 0, nt = 0;
    const bool alpha = 1 <= A.P.set.MaxAnyHitPathLength;
    if ((p | 63u) < A.P.num_paths && (A.P.packet & 1u))
        traverse8_packet<false, false>(A.S, pr.start, pr.dir, 0.0f, pr.length, alpha, true, h);
    else
        traverse<8, false, false>(A.S, pr.start, pr.dir, 0.0f, pr.length, alpha, nullptr, h, nv, nt);
    float4 out = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (h.tri != kMiss) {
        out.w = 1.0f;
        if (A.P.set.EnableAlbedoMaps && !A.P.set.EnableWhiteFurnaceMode) {
            const Surface surf = get_hit_surface(A.S, h.tri, h.b1, h.b2);
            const Texel4 a = sample_tex_desc(A.S, tex_desc(A.S.geoshade[h.geom].albedo), surf.u, surf.v);
            out.x = a.r;
            out.y = a.g;
            out.z = a.b;
        } else {
            out.x = out.y = out.z = 1.0f;
        }
    }
    A.P.accum[pr.accumIdx] = out;
}

hipError_t launch_primary_aov(const SceneDev& scene, const FrameBuffers& fb, const FrameParams& fp, hipStream_t stream) {
    if (fp.num_paths == 0) return hipSuccess;
    KArgs A{scene, fb, fp};
    const size_t lds = size_t(scene.stack_ints) * 64u * sizeof(int);
    hipLaunchKernelGGL(k_primary_aov, dim3((fp.num_paths + 63u) / 64u), dim3(64), lds, stream, A);
    return hipGetLastError();
}

// SampleCMJ2D (Sampling.hlsl:322-331) on arbitrary (sampleIdx, numSamplesX, numSamplesY, pattern) cases.
__global__ __launch_bounds__(kBlock) void k_sample_cmj(const uint4* cases, uint32_t n, float2* out) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint4 c = cases[i];
    float x, y;
    sample_cmj2d(c.x, c.y, c.z, c.w, &x, &y);
    out[i] = make_float2(x, y);
}

hipError_t launch_sample_cmj(const uint4* cases, uint32_t n, float2* out, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_sample_cmj, dim3(grid_for(n)), dim3(kBlock), 0, stream, cases, n, out);
    return hipGetLastError();
}

hipError_t read_phase_ticks(unsigned long long out[8]) {
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) return e;
    if ((e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase_ticks), 8 * sizeof(unsigned long long))) != hipSuccess) return e;
    const unsigned long long zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_phase_ticks), zero, sizeof(zero));
}

}  // namespace dxrpt
