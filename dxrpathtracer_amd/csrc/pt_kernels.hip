// pt_kernels.hip — the path tracer's gfx950 (MI355X) kernels.
//
// Replaces the recursive DXR pipeline of DXRPathTracer/RayTrace.hlsl (RaygenShader 92-149,
// PathTrace 151-441, ClosestHit 476-483, AnyHit 485-507, Miss 509-530, ShadowHit/Miss 532-542).
// Recursion becomes a loop over path depth; the per-vertex shading is ONE device function
// (path_vertex) run by three schedules that produce bit-identical frames:
//
//   depth-split megakernel (default for frames of >= 2M path vertices)
//     k_path_head      1 lane / camera path: raygen, packet primary, path_vertex(1), continuation
//                      compacted into queue[2] (wave64 ballot + one atomic per wave), the vertex's
//                      shadow rays, radiance into the queue entry (or the pixel)
//     k_path_tail(d)   1 lane / queued path of depth d: per-lane closest hit, path_vertex(d), ...
//   single megakernel k_path (smaller frames): one lane per path for every depth, no queues
//   wavefront passes (DXRPT_OPT_MEGAKERNEL_PATHS 0), one kernel per stage and depth:
//     k_raygen, then per depth k_trace, k_shade, k_shadow (concurrent with the next k_trace),
//     k_resolve, and k_accumulate
//
// Each path's radiance is a fixed-order sum done by the lane that owns it: results are deterministic
// run to run and independent of the tiling, the schedule and the launch shape.
//
// BVH traversal: compressed BVH8 (pt_layout.h), one ray per lane with a group stack whose top lives in
// registers, the next kStackLds8 entries in LDS (lane-interleaved) and deeper ones in a global slab;
// the primary rays and depth-1 sun shadow rays of an 8x8 pixel block walk one node sequence per wave
// with scalar loads (traverse8_packet).  Exact two-sided Moller-Trumbore behind conservative (padded)
// quantised box tests, identical to the oracle's arithmetic.
//
// Every traversal kernel runs 64-thread workgroups (one wave): a lane's LDS stack base is its lane id
// (stack_base), recomputed at every access so it is never kept live (and never spilled).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "pt_kernels.h"
#include "pt_math.h"

namespace dxrpt {

constexpr int kBlock = 256;                   // streaming kernels (raygen, shade, resolve, accumulate)
constexpr int kWave = 64;                     // traversal kernels: one wave per workgroup
constexpr uint32_t kMiss = 0xFFFFFFFFu;
constexpr float kRayTMin = 0.00001f;          // RayTrace.hlsl:243, 382
constexpr float kSpotShadowNearClip = 0.1f;   // AppSettings.hlsl:56
constexpr int kStkStride = 64;                // LDS stack: entry j of lane l at [j * 64 + l]

PT_DEV uint32_t fbits(float f) { return __float_as_uint(f); }
PT_DEV float bitsf(uint32_t u) { return __uint_as_float(u); }

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

// The 512-entry decode table (unorm, sRGB) is copied to the workgroup's LDS at kernel start
// (lut_fill): a texel's decode is an LDS read instead of a dependent global-memory gather.  Every
// kernel that samples textures (shading, alpha-tested traversal) calls lut_fill first.
__shared__ float g_lut[512];

// The table by LDS DMA (r05): global_load_lds_dwordx4 -- 16 B per lane, 1 KB per instruction -- the whole
// table by every wave (identical values: no barrier needed between a workgroup's waves), then one
// vmcnt(0), so the table is in before anything else runs.  No VGPR round trip, no ds_write, no barrier:
// metric / C2 / C4 -2 %.  kDma false: the plain copy (the non-last split tails of long paths keep it: the
// DMA form there cost C3 +1.8 %, C5 +1.3 %, profiles/r05_ab_lutdma*.txt -- measured, not understood).
template <bool kDma = true>
PT_DEV void lut_fill(const SceneDev& S) {
    if (kDma) {
        const char* src = reinterpret_cast<const char*>(S.lut) + (threadIdx.x & 63u) * 16u;
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(g_lut), 16, 0, 0);
        __builtin_amdgcn_global_load_lds(src + 1024, (__attribute__((address_space(3))) void*)(g_lut + 256), 16, 0, 0);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) (expcnt, lgkmcnt left at their maxima)
    } else {
        for (uint32_t i = threadIdx.x; i < 512u; i += blockDim.x) g_lut[i] = S.lut[i];
        __syncthreads();
    }
}

// A texel's word in the tiled pool (pt_kernels.h tex_tile_word), branch-free in the format: both tilings'
// addresses are computed and one selected, so a bilinear tap's four loads issue back to back.  (r05: with
// the format test as a branch -- the format is per lane -- the compiler serialised the four loads, each
// behind an s_waitcnt vmcnt(0) of the one before: four dependent memory round trips per tap, in every
// material tap and every AnyHitShader opacity tap.)
PT_DEV uint32_t tex_word(uint32_t x, uint32_t y, uint32_t tiles_x, bool r8) {
    const uint32_t a = ((y >> 3) * tiles_x + (x >> 4)) * kTexTileWords + (y & 7u) * 4u + ((x & 15u) >> 2);
    const uint32_t b = ((y >> 2) * tiles_x + (x >> 3)) * kTexTileWords + (y & 3u) * 8u + (x & 7u);
    return r8 ? a : b;
}

// Decode of one loaded texel word (the LDS table, unorm or sRGB), branch-free in the format: R8 -> (v, v, v, 1)
// with v = the texel's byte, RGBA8 -> the four channels (alpha always unorm).
PT_DEV Texel4 decode_texel(uint32_t w, bool r8, uint32_t l, uint32_t x) {
    const uint32_t b0 = r8 ? ((w >> ((x & 3u) * 8u)) & 0xFFu) : l + (w & 0xFFu);
    const uint32_t b1 = r8 ? b0 : l + ((w >> 8) & 0xFFu);
    const uint32_t b2 = r8 ? b0 : l + ((w >> 16) & 0xFFu);
    Texel4 t;
    t.r = g_lut[b0];
    t.g = g_lut[b1];
    t.b = g_lut[b2];
    const float a = g_lut[w >> 24];
    t.a = r8 ? 1.0f : a;
    return t;
}

// A 1 x 1 map's reference carries its texel word instead of a pool offset (DXRPT_OPT_PACKED_TAPS bit 1,
// pt_layout.h kTexInline): its bilinear tap reads no memory -- the same word four times, the same weights,
// so the same value, NaN for a NaN / Inf UV included.
PT_DEV bool tex_inline(const TexDesc& td) { return td.inl; }

// kInline: the reference may be an inlined 1 x 1 map (material maps; never the opacity map, whose
// AnyHitShader tap runs inside the traversal loops and keeps the plain form)
template <bool kInline = true>
PT_DEV TexDesc tex_desc(GeoTex g) {
    TexDesc td;
    td.offset = g.offset;
    td.width = g.whf & 0x7FFFu;
    td.height = (g.whf >> 15) & 0x7FFFu;
    td.fmt = g.whf >> 30;
    td.inl = kInline && (g.whf & 0x3FFFFFFFu) == 0u;  // width = height = 0: an inlined 1 x 1 map
    if (td.inl) td.width = td.height = 1u;
    return td;
}

// The per-texel form (a format branch per texel): the split tails' material taps keep it -- the
// branch-free form above costs them 5-10 % (r05, profiles/r05_ab_taps.txt), while it saves 2-5 % in the
// head, the single k_path and the alpha tests.
PT_DEV Texel4 fetch_texel(const SceneDev& S, const TexDesc& td, int x, int y, bool inl = false) {
    const bool r8 = td.fmt == DXRPT_TEX_R8_UNORM;
    const uint32_t tiles_x = (td.width + (r8 ? kTexTileW8 : kTexTileW32) - 1u) / (r8 ? kTexTileW8 : kTexTileW32);
    const uint32_t word = tex_tile_word(uint32_t(x), uint32_t(y), tiles_x, r8);
    Texel4 t;
    uint32_t w;
    if (inl)  // a 1 x 1 map inlined in its reference (tex_inline)
        w = td.offset;
    else
        w = S.texels[td.offset + word];
    if (r8) {
        float v = g_lut[(w >> ((uint32_t(x) & 3u) * 8u)) & 0xFFu];
        t.r = v; t.g = v; t.b = v; t.a = 1.0f;
    } else {
        const uint32_t l = td.fmt == DXRPT_TEX_RGBA8_SRGB ? 256u : 0u;
        t.r = g_lut[l + (w & 0xFFu)];
        t.g = g_lut[l + ((w >> 8) & 0xFFu)];
        t.b = g_lut[l + ((w >> 16) & 0xFFu)];
        t.a = g_lut[w >> 24];
    }
    return t;
}

template <bool kGrouped = true, bool kInline = true>
PT_DEV Texel4 sample_tex_desc(const SceneDev& S, const TexDesc td, float u, float v) {
    const bool inl = kInline && tex_inline(td);
    if (!kGrouped) {
        float x = u * float(td.width) - 0.5f;
        float y = v * float(td.height) - 0.5f;
        float x0 = floorf(x), y0 = floorf(y);
        float fx = x - x0, fy = y - y0;
        int ix0 = wrap_coord(int(x0), td.width), ix1 = wrap_coord(int(x0) + 1, td.width);
        int iy0 = wrap_coord(int(y0), td.height), iy1 = wrap_coord(int(y0) + 1, td.height);
        Texel4 t00, t10, t01, t11;
        if (inl) {
            t00 = t10 = t01 = t11 = fetch_texel(S, td, 0, 0, true);
        } else {
            t00 = fetch_texel(S, td, ix0, iy0);
            t10 = fetch_texel(S, td, ix1, iy0);
            t01 = fetch_texel(S, td, ix0, iy1);
            t11 = fetch_texel(S, td, ix1, iy1);
        }
        Texel4 r;
        r.r = lerpf(lerpf(t00.r, t10.r, fx), lerpf(t01.r, t11.r, fx), fy);
        r.g = lerpf(lerpf(t00.g, t10.g, fx), lerpf(t01.g, t11.g, fx), fy);
        r.b = lerpf(lerpf(t00.b, t10.b, fx), lerpf(t01.b, t11.b, fx), fy);
        r.a = lerpf(lerpf(t00.a, t10.a, fx), lerpf(t01.a, t11.a, fx), fy);
        return r;
    }
    float x = u * float(td.width) - 0.5f;
    float y = v * float(td.height) - 0.5f;
    float x0 = floorf(x), y0 = floorf(y);
    float fx = x - x0, fy = y - y0;
    int ix0 = wrap_coord(int(x0), td.width), ix1 = wrap_coord(int(x0) + 1, td.width);
    int iy0 = wrap_coord(int(y0), td.height), iy1 = wrap_coord(int(y0) + 1, td.height);
    const bool r8 = td.fmt == DXRPT_TEX_R8_UNORM;
    const uint32_t tiles_x = r8 ? (td.width + kTexTileW8 - 1u) / kTexTileW8 : (td.width + kTexTileW32 - 1u) / kTexTileW32;
    uint32_t w00, w10, w01, w11;
    if (inl) {
        w00 = w10 = w01 = w11 = td.offset;
    } else {
        const uint32_t* T = S.texels + td.offset;
        w00 = T[tex_word(uint32_t(ix0), uint32_t(iy0), tiles_x, r8)];
        w10 = T[tex_word(uint32_t(ix1), uint32_t(iy0), tiles_x, r8)];
        w01 = T[tex_word(uint32_t(ix0), uint32_t(iy1), tiles_x, r8)];
        w11 = T[tex_word(uint32_t(ix1), uint32_t(iy1), tiles_x, r8)];
    }
    const uint32_t l = td.fmt == DXRPT_TEX_RGBA8_SRGB ? 256u : 0u;
    Texel4 t00 = decode_texel(w00, r8, l, uint32_t(ix0)), t10 = decode_texel(w10, r8, l, uint32_t(ix1));
    Texel4 t01 = decode_texel(w01, r8, l, uint32_t(ix0)), t11 = decode_texel(w11, r8, l, uint32_t(ix1));
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

// AnyHitShader / ShadowAnyHitShader (RayTrace.hlsl:485-507): opacity.x < 0.35 -> IgnoreHit.
// kGA: the opacity tap's four texel loads grouped (sample_tex_desc<true>); the split tails keep the per-texel
// form (r05: grouped, the tails' traversal loops ran 8-10 % slower although their rays skip the alpha test by
// default; k_path, the head and the other kernels gain 1-4 %, profiles/r05_ab_taps*.txt).
template <bool kGA = true>
PT_DEV bool alpha_accepts(const SceneDev& S, uint32_t geom, uint32_t gtri, uint32_t slot, float b1, float b2) {
    const GeoTex opacity = S.geoshade[geom].opacity;
    const float2* V = reinterpret_cast<const float2*>(S.tri_verts + size_t(gtri) * 12u);
    float2 uv[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) uv[k] = V[k * 8 + 3];  // float2 #3 of MeshVertex k = UV
    const OmmProbe om = omm_probe(S, slot, b1, b2);
    // the opacity descriptor, the UVs and the micromap word in one memory round trip (a triangle that
    // reaches here is alpha tested, so its geometry has an opacity map; otherwise they are unused)
    asm volatile("" ::"v"(opacity.offset), "v"(opacity.whf), "v"(uv[0].x), "v"(uv[0].y), "v"(uv[1].x), "v"(uv[1].y),
                 "v"(uv[2].x), "v"(uv[2].y), "v"(om.word));
    if (opacity.whf == 0u) return true;
    const uint32_t verdict = omm_verdict(om);
    if (verdict != kOmmUnknown) return verdict == kOmmOpaque;
    const float w0 = (1.0f - b1) - b2;
    float u = bary_lerp(uv[0].x, uv[1].x, uv[2].x, w0, b1, b2);
    float v = bary_lerp(uv[0].y, uv[1].y, uv[2].y, w0, b1, b2);
    return !(sample_tex_desc<kGA, false>(S, tex_desc<false>(opacity), u, v).r < 0.35f);
}

// ---- triangles ------------------------------------------------------------------------------------
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

// Byte offsets of node / triangle records as 32-bit values (DXRPT_ADDR32, r06): the loads take the array's
// SGPR base plus a 32-bit VGPR offset ("saddr" form: one VGPR per address, no 64-bit add), and the offset is
// two full-rate shift-adds instead of a quarter-rate v_mad_u64_u32 (LLVM lowers x * 80 / x * 48 to
// v_mul_lo_u32 or the 64-bit multiply-add; the asm keeps the shift-add form).  dxrpt_build_bvh refuses trees
// whose node or triangle-record array reaches 4 GiB, so the offsets cannot wrap.
#ifndef DXRPT_ADDR32
#define DXRPT_ADDR32 1
#endif
PT_DEV uint32_t shl_add(uint32_t a, uint32_t b) {  // (a << 4) + b
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, 4, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
PT_DEV uint32_t tri_offset(uint32_t rec) { return shl_add(rec, rec << 5); }  // rec * 48
PT_DEV uint32_t node_offset(uint32_t node) {
    return kNode8Stride == 80u ? shl_add(node, node << 6) : node * kNode8Stride;  // node * 80
}

// A record's words come from one base address (immediate offsets).
PT_DEV TriRec load_tri_raw(const SceneDev& S, uint32_t rec) {
    const float4* T = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(S.tris) +
                                                      (DXRPT_ADDR32 ? size_t(tri_offset(rec)) : size_t(rec) * 48u));
    return TriRec{T[0], T[1], T[2]};
}

// ... and are all in registers before the first test uses them: one memory round trip per record.
PT_DEV TriRec load_tri(const SceneDev& S, uint32_t rec) {
    const TriRec r = load_tri_raw(S, rec);
    pin_tri(r);
    return r;
}

// One candidate triangle (the "intersection + any-hit" stage of a DXR traversal).  Returns true
// when an any-hit ray is done (accepted occluder).  Closest hit: smallest t, ties -> smallest global
// triangle id, which makes the result independent of traversal order.
template <bool kAnyHit, bool kGA = true>
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
    if (alpha && !(fbits(p2.w) & kTriOpaque) && !alpha_accepts<kGA>(S, geom, gtri, fbits(p2.w) >> 1, u, v)) return false;
    h.t = t;
    h.tri = gtri;
    h.b1 = u;
    h.b2 = v;
    h.geom = geom;
    return kAnyHit;
}

PT_DEV f3 safe_inverse(f3 d) {
    f3 inv;
    inv.x = 1.0f / (fabsf(d.x) > 1e-20f ? d.x : copysignf(1e-20f, d.x));
    inv.y = 1.0f / (fabsf(d.y) > 1e-20f ? d.y : copysignf(1e-20f, d.y));
    inv.z = 1.0f / (fabsf(d.z) > 1e-20f ? d.z : copysignf(1e-20f, d.z));
    return inv;
}

// ---- per-lane BVH8 traversal ----------------------------------------------------------------------
// Compressed BVH8 (Ylitie, Karras & Laine 2017, adapted to one ray per wave64 lane).  A node visit
// intersects all 8 quantised child boxes at once; internal hits form a "node group" (base_child, hit
// bits keyed by slot ^ octant, imask) visited highest key first (near to far), leaf hits are tested
// right away.  The rest of a group is pushed when descending: <= 1 push per level.
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

// Group stack: `sp` entries; the top one lives in registers (`tos`), entries 0 .. sp-2 in LDS (first
// kStackLds8, 2 x 4 B each) and in the thread's global spill slab (deeper), so a pop hands over the
// next group at once and the LDS refill of `tos` overlaps the next node fetch.  The lane's LDS base is
// recomputed at every access from the lane id (volatile asm: never kept live across the path, so it is
// never spilled and reloaded from scratch on a push or pop).  One wave per workgroup.
typedef __attribute__((address_space(3))) int lds_int;

PT_DEV lds_int* stack_base() {
    extern __shared__ int stack[];
    uint32_t lane;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
    return (lds_int*)(stack) + lane;
}

PT_DEV void stack8_store(const SceneDev& S, int j, uint2 e) {
    if (j < kStackLds8) {
        lds_int* stk = stack_base();
        stk[(2 * j) * kStkStride] = int(e.x);
        stk[(2 * j + 1) * kStkStride] = int(e.y);
    } else {  // rare: deep entries spill to this thread's global slab
        S.spill8[size_t(j - kStackLds8) * S.spill_stride + blockIdx.x * blockDim.x + threadIdx.x] = e;
    }
}

PT_DEV uint2 stack8_load(const SceneDev& S, int j) {
    if (j < kStackLds8) {
        const lds_int* stk = stack_base();
        return make_uint2(uint32_t(stk[(2 * j) * kStkStride]), uint32_t(stk[(2 * j + 1) * kStkStride]));
    }
    return S.spill8[size_t(j - kStackLds8) * S.spill_stride + blockIdx.x * blockDim.x + threadIdx.x];
}

// The 80-B node as five 16-B words (pt_layout.h Bvh8Node), from one 64-bit base with immediate offsets
// and pinned in registers (the leaf metadata w1.zw is otherwise loaded behind the leaf-hit branch: a
// second round trip).
struct Node8Words {
    uint4 w0, w1, w2, w3, w4;
};

PT_DEV Node8Words load_node8(const SceneDev& S, uint32_t node) {
    const uint4* N = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(S.nodes8) +
                                                    (DXRPT_ADDR32 ? size_t(node_offset(node)) : size_t(node) * kNode8Stride));
    const Node8Words w{N[0], N[1], N[2], N[3], N[4]};
    asm volatile("" ::"v"(w.w0.x), "v"(w.w0.y), "v"(w.w0.z), "v"(w.w0.w), "v"(w.w1.x), "v"(w.w1.y), "v"(w.w1.z),
                 "v"(w.w1.w), "v"(w.w2.x), "v"(w.w2.y), "v"(w.w2.z), "v"(w.w2.w), "v"(w.w3.x), "v"(w.w3.y),
                 "v"(w.w3.z), "v"(w.w3.w), "v"(w.w4.x), "v"(w.w4.y), "v"(w.w4.z), "v"(w.w4.w));
    return w;
}

// Slot mask of the node's children whose quantised box the ray enters within [tmin, tmx].  kNearest:
// also the slot of the internal child entered first (smallest entry distance; *nslot, 8 if none).
// DXRPT_NEAR_KEYS (r06): kNearest's choice as the unsigned minimum of per-child keys -- the entry distance's
// bits (tn >= tmin >= 0 in every caller: bit order = value order) with the slot in the low 3 mantissa bits, a
// missed child's key all ones -- instead of a compare-and-select chain per child (5 VALU each: the internal-bit
// test, the compare, two selects).  2 (shipped): the minimum over every hit child; a leaf winner falls back to
// the octant order.  0: the chain.  Closest-hit results do not depend on the visit order (minimum (t, triangle
// id)), so frames are bit-identical; node-visit counts move.  Same box, interleaved (profiles/r06_ab_boxtest.txt):
// metric -0.3 %, C4 -0.9 %, C2 -1.0 %, C3 -0.4 %, the 1/8 share -1.4 %; excluding leaves from the minimum through
// bit 31 of their keys (measured as mode 1, removed) was even to +0.6 %.
#ifndef DXRPT_NEAR_KEYS
#define DXRPT_NEAR_KEYS 2
#endif
// kInfT (r06, DXRPT_AH_INF): an any-hit walk's box test without the TMax clamp -- hit <=> !(tn > tf) &&
// !(tmin > tf): 4 VALU per child instead of 5 (max, max3, min, min3, compare).  For rays with TMax = FP32Max (the
// sun's and the sky-visibility rays, RayTrace.hlsl:258,425) it differs from the clamped test only where tf is
// +inf or NaN, where it accepts; for any ray it accepts a superset of the clamped test's children, and the
// triangle test still enforces TMax, so the any-hit result -- a boolean over the occluders in [TMin, TMax] -- is
// the same: frames are bit-identical.  DXRPT_AH_INF 1: the chained sun / sky rays (metric -2.0 %, C4 -1.9 %, C2
// -2.7 %, C3 even, 1/8 share -0.6 %, r06_ab_boxtest.txt); 2 (shipped): also the sun packets (metric -0.6 %,
// r06_ab_boxtest2.txt).  Measured and removed: the per-lane sun rays of frames without spot lights on the kInfT
// form too (a second per-lane any-hit walk behind a NumLights branch; spot rays must keep the clamp, their TMax
// culls) -- in every kernel it raised the head's spills 34 -> 82 VGPRs (even to +0.5 %), in the tails and the
// single k_path only it was even to +0.6 % (r06_ab_inf3.txt).
#ifndef DXRPT_AH_INF
#define DXRPT_AH_INF 2
#endif
// kUOct (the packet walks, DXRPT_PACKET_UOCT): `uoct` is the octant of every live lane's ray, a wave-uniform
// value -- with the node words in SGPRs (scalar loads) the near / far word selection is then scalar.
template <bool kNearest = false, bool kInfT = false, bool kUOct = false>
PT_DEV uint32_t box8_hits(const Ray8& R, const Node8Words& W, float tmx, uint32_t* nslot = nullptr, uint32_t uoct = 0u) {
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
    const uint32_t boct = kUOct ? uoct : R.oct;
    const bool sxn = (boct & 4u) != 0u, syn = (boct & 2u) != 0u, szn = (boct & 1u) != 0u;
    const uint32_t nx0 = sxn ? w3.z : w2.x, nx1 = sxn ? w3.w : w2.y, fx0 = sxn ? w2.x : w3.z, fx1 = sxn ? w2.y : w3.w;
    const uint32_t ny0 = syn ? w4.x : w2.z, ny1 = syn ? w4.y : w2.w, fy0 = syn ? w2.z : w4.x, fy1 = syn ? w2.w : w4.y;
    const uint32_t nz0 = szn ? w4.z : w3.x, nz1 = szn ? w4.w : w3.y, fz0 = szn ? w3.x : w4.z, fz1 = szn ? w3.y : w4.w;
    uint32_t hm = 0;  // hit children, slot space
    const uint32_t imask = w0.w >> 24;
    float best_tn = kFP32Max;
    uint32_t best_c = 8u;
    uint32_t best_key = 0xFFFFFFFFu;
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
        float tn, tf;
        bool hit;
        if (kInfT) {
            tn = fmaxf(fmaxf(tx.x, ty.x), tz.x);
            tf = fminf(fminf(tx.y, ty.y), tz.y);
            hit = !(tn > tf) && !(R.tmin > tf);
        } else {
            tn = fmaxf(fmaxf(tx.x, ty.x), fmaxf(tz.x, R.tmin));
            tf = fminf(fminf(tx.y, ty.y), fminf(tz.y, tmx));
            hit = tn <= tf;
        }
        // empty slots carry inverted boxes (qlo 255, qhi 0: never entered) and meta 0 (no triangles)
        hm |= uint32_t(hit) << c;
        if (kNearest && DXRPT_NEAR_KEYS) {
            const uint32_t key = (fbits(tn) & ~7u) | uint32_t(c);
            best_key = __builtin_elementwise_min(best_key, hit ? key : 0xFFFFFFFFu);
        } else if (kNearest && hit && ((imask >> c) & 1u) && tn < best_tn) {
            best_tn = tn;
            best_c = uint32_t(c);
        }
    }
    if (kNearest && DXRPT_NEAR_KEYS) {
        best_c = best_key & 7u;
        if (best_key == 0xFFFFFFFFu || !((imask >> best_c) & 1u)) best_c = 8u;
    }
    if (kNearest) *nslot = best_c;
    return hm;
}

// Internal hits (slot space) to key space (bit slot ^ oct): three conditional bit-group swaps.
PT_DEV uint32_t key_order(uint32_t ihits, uint32_t oct) {
    if (oct & 1u) ihits = ((ihits & 0x55u) << 1) | ((ihits >> 1) & 0x55u);
    if (oct & 2u) ihits = ((ihits & 0x33u) << 2) | ((ihits >> 2) & 0x33u);
    if (oct & 4u) ihits = ((ihits & 0x0Fu) << 4) | ((ihits >> 4) & 0x0Fu);
    return ihits;
}

// Leaf hits -> triangle bits ((count << 5) | offset per leaf slot).
PT_DEV uint32_t leaf_tri_bits(uint32_t lh, const uint4& w1) {
    uint32_t thits = 0;
    const unsigned long long meta = (static_cast<unsigned long long>(w1.w) << 32) | w1.z;
    while (lh) {
        const uint32_t c = uint32_t(__builtin_ctz(lh));
        lh &= lh - 1u;
        const uint32_t m = uint32_t(meta >> (8u * c)) & 0xFFu;
        thits |= ((1u << (m >> 5)) - 1u) << (m & 31u);
    }
    return thits;
}

// Visits the node whose words are W: its hit leaf triangles become the pending group (tbase, tbits);
// then selects the next node (pops when the current group is exhausted).  Returns false when no node
// is left to visit.  The pending triangles are tested before the next node visit, so the visit order
// and hence the result are the same however tests and visits of different lanes interleave.
// Child visit order: closest-hit rays near to far (key = slot ^ octant, highest first), any-hit rays far
// to near (key octant inverted): a shadow ray leaves a surface and its occluders lie away from that
// surface, so it meets one after fewer node visits (r04: SIMT replay -22 % node visits, -30 % triangle
// tests per Sponza shadow ray; metric 1.78 -> 1.61 ms, profiles/r04_ab_farfirst.txt).  An any-hit result
// is a boolean over every occluder, so the order does not change it.
template <bool kAnyHit>
PT_DEV uint32_t key_octant(uint32_t oct) { return kAnyHit ? oct ^ 7u : oct; }

template <bool kCount, bool kAnyHit = false, bool kNearest = false, bool kInfT = false>
PT_DEV bool trav8_node(const SceneDev& S, const Ray8& R, const Node8Words& W, uint32_t& node, int& sp, uint2& tos,
                       const HitRec& h, uint32_t& tbase, uint32_t& tbits, uint32_t& nvisit) {
    if (kCount) ++nvisit;
    const uint4 w0 = W.w0, w1 = W.w1;
    uint32_t nslot = 8u;
    // kNearest picks the nearest hit internal child for closest-hit rays (any-hit rays ignore it: their
    // farthest-entry-first variant was +0.7..1.4 % on C3 / C5, profiles/r04_ab_farthest.txt)
    constexpr bool kPick = kNearest && !kAnyHit;
    const uint32_t hm = box8_hits<kPick, kInfT>(R, W, h.t, &nslot);  // hit children, slot space
    const uint32_t imask = w0.w >> 24;
    const uint32_t koct = key_octant<kAnyHit>(R.oct);
    const uint32_t ihits = key_order(hm & imask, koct);
    tbase = w1.y;
    tbits = leaf_tri_bits(hm & ~imask, w1);
    uint32_t gbase = w1.x;
    uint32_t gword = (ihits << 24) | imask;
    if (kPick && nslot < 8u) {  // the nearest internal child first, the rest as a group
        gword &= ~(1u << (24u + (nslot ^ koct)));
        node = gbase + uint32_t(__builtin_popcount(imask & ((1u << nslot) - 1u)));
        if (gword >> 24) {
            if (sp > 0) stack8_store(S, sp - 1, tos);
            tos = make_uint2(gbase, gword);
            ++sp;
        }
        return true;
    }
    while (true) {
        if (gword >> 24) {
            const uint32_t k = 31u - uint32_t(__builtin_clz(gword));
            gword &= ~(1u << k);
            const uint32_t slot = (k - 24u) ^ koct;
            node = gbase + uint32_t(__builtin_popcount(gword & 0xFFu & ((1u << slot) - 1u)));
            if (gword >> 24) {  // push the rest of the group
                if (sp > 0) stack8_store(S, sp - 1, tos);
                tos = make_uint2(gbase, gword);
                ++sp;
            }
            return true;
        }
        if (sp == 0) return false;
        gbase = tos.x;  // pop
        gword = tos.y;
        if (--sp > 0) tos = stack8_load(S, sp - 1);
    }
}

// Tests the pending triangle group.  Returns true when an any-hit ray found an occluder.
template <bool kAnyHit, bool kCount, bool kGA = true>
PT_DEV bool trav8_tris(const SceneDev& S, const Ray8& R, uint32_t tbase, uint32_t tbits, HitRec& h, uint32_t& ntest) {
    while (tbits) {
        const uint32_t b = uint32_t(__builtin_ctz(tbits));
        tbits &= tbits - 1u;
        if (kCount) ++ntest;
        if (test_tri_rec<kAnyHit, kGA>(S, load_tri(S, tbase + b), R.o, R.d, R.tmin, R.tmax, R.alpha, h)) return true;
    }
    return false;
}

// The pending group two records at a time: both records are loaded before either test, so a lane pays
// one memory round trip per pair.  Tests still run in bit order (same results).
template <bool kAnyHit, bool kCount, bool kGA = true>
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
        if (test_tri_rec<kAnyHit, kGA>(S, ra, R.o, R.d, R.tmin, R.tmax, R.alpha, h)) return true;
        if (two && test_tri_rec<kAnyHit, kGA>(S, rb, R.o, R.d, R.tmin, R.tmax, R.alpha, h)) return true;
    }
    return false;
}

// One ray per lane from the root.  kPairs: leaf triangles two at a time (trav8_tris2; the split tails'
// closest hit, r03: -0.8..-1.0 %).  kNearest (closest hit): each node descends into its nearest hit
// internal child first (exact entry distance) and keeps the others as one octant-ordered group -- fewer
// node visits and triangle tests, for a few more registers in the box test, so only kernels with the
// budget use it (r04: the split tails and k_path at <= 5 waves/SIMD; k_path<7> spills, C2 +9 %).
// Returns h.tri != kMiss (hit / occluded).
//
// DXRPT_IFIF (r06): the wave's loop interleaves the two halves of a lane's walk ("if-if", Aila & Laine 2009)
// instead of running each visit's triangle group to completion before the next visit ("while-while"): an
// iteration visits one node on the lanes with no pending triangle and tests one triangle (two with kPairs)
// on the lanes holding some.  A lane's own sequence -- visit, its group's triangles in bit order, next
// visit -- is unchanged, so results and census counts are identical; only which lanes share an iteration
// changes (a lane with three leaf triangles no longer holds the wave's other lanes for three tests).
// r06 A/B (profiles/r06_ab_ifif.txt, r06_ab_ifif2.txt, same box, interleaved): metric 1.391 -> 1.370 ms, tail
// 1.115 -> 1.092 ms per launch, C3 -3.3 %, C4 -2.1 %, C2 -2.2 %, the 1/8 share -2.8 %.  A variant running
// only one of the two halves per iteration, chosen wave-uniformly by the lanes ready for each, was no better
// (the weights tried: even to -3 %, worse at 1:1); nor did one fetch per iteration serving both kinds of
// lane (a node's words or a triangle record through the same loads): +9 % metric, tail +14 %
// (profiles/r06_ab_unified.txt).
#ifndef DXRPT_IFIF
#define DXRPT_IFIF 1
#endif
// kSpec (with DXRPT_IFIF): speculative visits -- a lane holding a pending triangle group also visits its next
// node in the same iteration, queueing the new group behind the pending one (one slot).  The lane's
// node-visit and triangle-test sequences keep their order; only a closest-hit ray's culling may use a less
// tight t (visits can run ahead of tests), so results are identical and census counts may differ.  On in the
// single k_path (the band shares' kernel: 1/8 share -1.3..-2 %, 1/4 -2 %), off in the split head and tails
// (metric +1..3 %; profiles/r06_ab_spec*.txt).  DXRPT_SPEC_PATH 0 turns it off in k_path too.
#ifndef DXRPT_SPEC_PATH
#define DXRPT_SPEC_PATH 1
#endif
template <bool kAnyHit, bool kCount, bool kPairs = false, bool kNearest = false, bool kGA = true, bool kSpec = false,
          bool kInfT = false>
PT_DEV bool traverse8(const SceneDev& S, f3 o, f3 d, float tmin, float tmax, bool alpha, HitRec& h, uint32_t& nvisit,
                      uint32_t& ntest) {
    Ray8 R;
    ray8_init(R, o, d, tmin, tmax, alpha, h);
    uint32_t node = 0;
    int sp = 0;
    uint2 tos = make_uint2(0u, 0u);
#if DXRPT_IFIF
    uint32_t tbase = 0, tbits = 0;
    bool more = true;
    uint32_t qbase = 0, qbits = 0;  // kSpec: a second, queued triangle group
    while (true) {
        if (kSpec) {
            // speculative visit (kSpec): a lane holding a pending group keeps visiting while the queue slot
            // is free; the groups are tested in visit order
            if (tbits == 0u && qbits == 0u && !more) break;
            if (more && qbits == 0u) {
                uint32_t nb = 0, nbits = 0;
                more = trav8_node<kCount, kAnyHit, kNearest, kInfT>(S, R, load_node8(S, node), node, sp, tos, h, nb, nbits, nvisit);
                if (tbits == 0u) {
                    tbase = nb;
                    tbits = nbits;
                } else {
                    qbase = nb;
                    qbits = nbits;
                }
            }
        } else if (tbits == 0u) {
            if (!more) break;
            more = trav8_node<kCount, kAnyHit, kNearest, kInfT>(S, R, load_node8(S, node), node, sp, tos, h, tbase, tbits, nvisit);
        }
        if (kSpec && tbits == 0u && qbits) {
            tbase = qbase;
            tbits = qbits;
            qbits = 0u;
        }
        if (tbits) {
            const uint32_t b0 = uint32_t(__builtin_ctz(tbits));
            tbits &= tbits - 1u;
            if (kPairs) {
                const bool two = tbits != 0u;
                const uint32_t b1 = two ? uint32_t(__builtin_ctz(tbits)) : b0;
                tbits &= tbits - 1u;
                const TriRec ra = load_tri_raw(S, tbase + b0);
                const TriRec rb = load_tri_raw(S, tbase + b1);
                pin_tri(ra);
                pin_tri(rb);
                if (kCount) ntest += two ? 2u : 1u;
                if (test_tri_rec<kAnyHit, kGA>(S, ra, R.o, R.d, R.tmin, R.tmax, R.alpha, h)) return true;
                if (two && test_tri_rec<kAnyHit, kGA>(S, rb, R.o, R.d, R.tmin, R.tmax, R.alpha, h)) return true;
            } else {
                if (kCount) ++ntest;
                if (test_tri_rec<kAnyHit, kGA>(S, load_tri(S, tbase + b0), R.o, R.d, R.tmin, R.tmax, R.alpha, h)) return true;
            }
        }
    }
    return h.tri != kMiss;
#else
    while (true) {
        uint32_t tbase = 0, tbits = 0;
        const bool more = trav8_node<kCount, kAnyHit, kNearest, kInfT>(S, R, load_node8(S, node), node, sp, tos, h, tbase,
                                                                       tbits, nvisit);
        if (tbits) {
            const bool done = kPairs ? trav8_tris2<kAnyHit, kCount, kGA>(S, R, tbase, tbits, h, ntest)
                                     : trav8_tris<kAnyHit, kCount, kGA>(S, R, tbase, tbits, h, ntest);
            if (done) return true;
        }
        if (!more) break;
    }
    return h.tri != kMiss;
#endif
}

// ---- wave-coherent ("packet") BVH8 traversal ------------------------------------------------------
// The 64 rays of a wave walk ONE node sequence: a child is entered when any live lane's ray enters its
// box (each lane tests with its own ray and its own closest t), leaf triangles hit by any lane are
// tested by every live lane.  Node and triangle addresses are therefore wave-uniform and are fetched
// with scalar loads (constant address space -> s_load through the scalar cache), so the traversal
// issues no vector memory instructions; the group stack is wave-uniform too: entry j lives in lane j
// of two VGPRs (push = v_cndmask, pop = v_readlane), no LDS.
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

PT_DEV uint32_t wave_or8(uint32_t m) {
    uint32_t u = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) u |= uint32_t(__ballot((m >> c) & 1u) != 0ull) << c;
    return u;
}

// `live`: this lane holds a ray (lanes past the end join with live = false).  kFar: any-hit packets walk far
// to near (the head's depth-1 sun shadows: metric -1 %); k_path at <= 5 waves/SIMD walks them near to far
// (1/8 share -3.5 %, profiles/r04_ab_packet_order.txt).  Returns this lane's
// result like traverse8 (h.tri != kMiss: hit / occluded).  kCount: node / triangle FETCHES are counted
// in cnt[0] / cnt[1] by the wave's first live lane (a packet fetches each once per wave).
// kUOct: every live lane's ray has the octant `oct0` (the box test's near / far selection is then scalar).
template <bool kAnyHit, bool kCount, bool kFar, bool kInfT, bool kUOct>
PT_DEV bool packet_walk(const SceneDev& S, const Ray8& R, bool live, unsigned long long lv, uint32_t oct0, HitRec& h,
                        uint32_t* cnt) {
    // key order of the first live lane's octant for the whole wave (any order gives the same results;
    // any-hit rays far to near, key_octant)
    const uint32_t oct = key_octant<kAnyHit && kFar>(oct0);
    const uint32_t lane = uint32_t(__lane_id());
    const bool counter = kCount && lane == uint32_t(__ffsll(static_cast<long long>(lv)) - 1);
    uint32_t sbase = 0, sword = 0;  // stack entry j in lane j
    uint32_t sp = 0;
    uint32_t node = 0;
    while (true) {
        const Node8Words W = load_node8_uniform(S, node);
        if (counter) ++cnt[0];
        const uint32_t hm = live ? box8_hits<false, kInfT, kUOct>(R, W, h.t, nullptr, oct0) : 0u;
        const uint32_t um = wave_or8(hm);
        const uint32_t imask = W.w0.w >> 24;
        uint32_t tbits = leaf_tri_bits(um & ~imask, W.w1);  // leaf triangles hit by any lane
        const uint32_t tbase = W.w1.y;
        while (tbits) {
            const uint32_t b = uint32_t(__builtin_ctz(tbits));
            tbits &= tbits - 1u;
            const TriRec r = load_tri_uniform(S, tbase + b);
            if (counter) ++cnt[1];
            if (live && test_tri_rec<kAnyHit>(S, r, R.o, R.d, R.tmin, R.tmax, R.alpha, h)) live = false;  // occluded
        }
        if (kAnyHit && __ballot(live) == 0ull) break;
        uint32_t gbase = W.w1.x;
        uint32_t gword = (key_order(um & imask, oct) << 24) | imask;
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
    }
    return h.tri != kMiss;
}

// DXRPT_PACKET_UOCT (r06): a packet whose live lanes share one ray octant -- always the sun's shadow rays (one
// direction, kOctMode 1), mostly an 8x8 block's primary rays (kOctMode 2 tests it per packet) -- walks with the
// octant's near / far node words chosen by scalar selects on the SGPR node words: 24 VALU fewer per visit (12
// copies of node words into VGPRs and 12 per-lane selects).  kOctMode 0: per-lane selection only.
#ifndef DXRPT_PACKET_UOCT
#define DXRPT_PACKET_UOCT 1
#endif
template <bool kAnyHit, bool kCount = false, bool kFar = true, bool kInfT = false, int kOctMode = 2>
PT_DEV bool traverse8_packet(const SceneDev& S, f3 o, f3 d, float tmin, float tmax, bool alpha, bool live, HitRec& h,
                             uint32_t* cnt = nullptr) {
    Ray8 R;
    ray8_init(R, o, d, tmin, tmax, alpha, h);
    const unsigned long long lv = __ballot(live);
    if (lv == 0ull) return false;
    const uint32_t oct0 = uint32_t(__builtin_amdgcn_readlane(int(R.oct), __ffsll(static_cast<long long>(lv)) - 1));
    if constexpr (DXRPT_PACKET_UOCT && kOctMode == 1) {
        return packet_walk<kAnyHit, kCount, kFar, kInfT, true>(S, R, live, lv, oct0, h, cnt);
    } else {
        if (DXRPT_PACKET_UOCT && kOctMode == 2 && __ballot(live && R.oct != oct0) == 0ull)
            return packet_walk<kAnyHit, kCount, kFar, kInfT, true>(S, R, live, lv, oct0, h, cnt);
        return packet_walk<kAnyHit, kCount, kFar, kInfT, false>(S, R, live, lv, oct0, h, cnt);
    }
}

// ---- queues ---------------------------------------------------------------------------------------
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

// Position of item i (< queue_total) of a sharded queue with shard capacity cap, for lanes holding
// consecutive items (i grows with the lane id, so the first active lane holds the smallest): a
// wave-uniform scalar scan finds the shard of that item, then each lane steps forward over the (few)
// shards its own item lies past.  The items of shard 0 come first, then shard 1, ...
PT_DEV uint32_t queue_pos(const uint32_t* __restrict__ cnt, uint32_t cap, uint32_t i) {
    const uint32_t i0 = uint32_t(__builtin_amdgcn_readfirstlane(int(i)));
    uint32_t s = 0, base = 0;
    while (s + 1u < kQueueShards && base + cnt[s] <= i0) base += cnt[s++];
    while (s + 1u < kQueueShards && base + cnt[s] <= i) base += cnt[s++];
    return s * cap + (i - base);
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

// ---- ray generation -------------------------------------------------------------------------------
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

// RaygenShader, RayTrace.hlsl:92-126 (+ SamplePoint 85-90), wavefront schedule.  Path slot p goes to the
// queue-1 position a wave-ordered append of its wave w = p / 64 would have produced (shard
// w % kQueueShards, waves of one shard in order); the shard counts are analytic.
__global__ __launch_bounds__(kBlock) void k_raygen(KArgs A) {
    const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t P = A.P.num_paths;
    const uint32_t nw = (P + 63u) / 64u;
    if (p == 0) {
        uint32_t* cnt = A.F.counters + 1u * kQueueShards;
        for (uint32_t s = 0; s < kQueueShards; ++s) {
            const uint32_t waves = s < nw ? (nw - 1u - s) / kQueueShards + 1u : 0u;
            uint32_t items = waves * 64u;
            if (nw > 0u && (nw - 1u) % kQueueShards == s) items -= nw * 64u - P;
            cnt[s] = items;
        }
    }
    if (p >= P) return;
    const PrimaryRay pr = primary_ray(A, p);
    const uint32_t w = p >> 6;
    const uint32_t pos = (w % kQueueShards) * A.F.cap_r + (w / kQueueShards) * 64u + (p & 63u);
    const RayQueue& Q = A.F.q[1];
    Q.org[pos] = make_float4(pr.start.x, pr.start.y, pr.start.z, pr.length);
    Q.dir[pos] = make_float4(pr.dir.x, pr.dir.y, pr.dir.z, bitsf(p));
    Q.thr[pos] = make_float4(1.0f, 1.0f, 1.0f, 0.0f);
    Q.rad[pos] = make_float4(0.0f, 0.0f, 0.0f, bitsf(0u));
    Q.pix[pos] = pr.pixelIdx;
    A.F.ps_pix[p] = make_uint2(pr.pixelIdx, pr.accumIdx);
}

// ---- the path vertex (shared by every schedule) -----------------------------------------------------
// Shadow ray k of the vertex at queue position pos lives in slot [k * qsize + pos].
// DXRPT_NT (r06): the depth-split kernels read the per-frame streams a last time -- the queued path state after
// the traversal, the shadow-slot records -- with the nontemporal cache policy (`global_load ... nt`), so those
// lines go first when the XCD's L2 needs room and BVH nodes and triangle records stay.  Same box, interleaved
// (profiles/r06_ab_nt.txt): metric -0.4..-0.6 %, C4 -0.5..-1.0 %, C2 -0.5..-0.7 %, C3 even; the single k_path
// (band shares) keeps plain loads (+0.4 % there).  Nontemporal STORES of the same streams lost 1.5-2.5 %; the
// tails' first (pre-traversal) queue reads and the blend's stage reads nontemporal too were neutral.
// DXRPT_NT_CHAIN: the chained shadow loop's slot origin / direction words (read once, right after the shading
// wrote them) as well: metric -1.2..-1.3 %, C4 -1.2..-1.3 %, C2 -1.1..-1.8 %, C3 -0.3 % (r06_ab_nt_chain.txt).
#ifndef DXRPT_NT
#define DXRPT_NT 1
#endif
typedef float v4f_t __attribute__((ext_vector_type(4)));
template <bool kNT>
PT_DEV float4 ld4(const float4* p) {
    if (kNT) {
        const v4f_t t = __builtin_nontemporal_load(reinterpret_cast<const v4f_t*>(p));
        return make_float4(t.x, t.y, t.z, t.w);
    }
    return *p;
}
template <bool kNT>
PT_DEV uint32_t ld1(const uint32_t* p) { return kNT ? __builtin_nontemporal_load(p) : *p; }
constexpr bool kSplitNT = DXRPT_NT != 0;
#ifndef DXRPT_NT_CHAIN
#define DXRPT_NT_CHAIN 1
#endif

PT_DEV void emit_shadow(const KArgs& A, uint32_t pos, uint32_t& n, f3 o, f3 d, float tmin, float tmax, f3 contrib,
                        bool forceOpaque) {
    const size_t s = size_t(n) * A.F.qsize + pos;
    A.F.sh_org[s] = make_float4(o.x, o.y, o.z, tmax);
    A.F.sh_dir[s] = make_float4(d.x, d.y, d.z, tmin);
    A.F.sh_con[s] = make_float4(contrib.x, contrib.y, contrib.z, bitsf(forceOpaque ? 1u : 0u));
    ++n;
}

PT_DEV bool nonzero3(f3 c) { return !(c.x == 0.0f && c.y == 0.0f && c.z == 0.0f); }

// Shadow ray kinds, in the order a vertex emits them (RayTrace.hlsl:224-262, 265-313, 415-425).
constexpr int kShadowSun = 0, kShadowSpot = 1, kShadowSky = 2;

// One path vertex: MissShader (RayTrace.hlsl:509-530) or ClosestHitShader -> PathTrace (151-441) for the
// ray (inOrigin, inDir) of path depth `depth` with hit record `hit` (b1, b2, tri, geom).  Shadow rays
// go to emit(kind, origin, dir, tmin, tmax, pending contribution = pathThr * CalcLighting (or sky *
// throughput), force_opaque) in the reference's order (sun, spot lights, final sky visibility); the
// local radiance and the continuation come back in O.
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

template <bool kGroupedTaps = true, class Emit>
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
        // packed material (DXRPT_OPT_PACKED_TAPS, pt_layout.h kTexFmtPackedNMR): the normal map's tap also
        // carries metallic (.b) and roughness (.a) -- one bilinear tap for the three.  texMetal / texRough
        // hold the maps' values (furnace: 1, no tap), so both forms leave the same two floats live.
        const TexDesc ntd = tex_desc(mat.normal);
        const bool packedNMR = ntd.fmt == kTexFmtPackedNMR;
        float texMetal = 1.0f, texRough = 1.0f;
        if (set.EnableNormalMaps || (packedNMR && !furnace)) {
            const Texel4 nm = sample_tex_desc<kGroupedTaps>(A.S, ntd, surf.u, surf.v);
            if (packedNMR && !furnace) {
                texMetal = nm.b;
                texRough = nm.a;
            }
            if (set.EnableNormalMaps) {
                f3 nts;
                nts.x = nm.r * 2.0f - 1.0f;
                nts.y = nm.g * 2.0f - 1.0f;
                nts.z = sqrtf(1.0f - saturate(nts.x * nts.x + nts.y * nts.y));
                normalWS = normalize3(add(add(scl(T, nts.x), scl(Bt, nts.y)), scl(surf.n, nts.z)));
                Nrow = normalWS;
            }
        }
        f3 baseColor = f3{1.0f, 1.0f, 1.0f};
        if (set.EnableAlbedoMaps && !furnace) {
            Texel4 a = sample_tex_desc<kGroupedTaps>(A.S, tex_desc(mat.albedo), surf.u, surf.v);
            baseColor = f3{a.r, a.g, a.b};
        }
        if (!furnace && !packedNMR) texMetal = sample_tex_desc<kGroupedTaps>(A.S, tex_desc(mat.metallic), surf.u, surf.v).r;
        const float metallic = saturate(texMetal * set.MetallicScale);
        const bool enableDiffuse = (set.EnableDiffuse && metallic < 1.0f) || furnace;
        const bool payloadIsDiffuse = V.payloadIsDiffuse;
        const bool enableSpecular =
            set.EnableSpecular && (set.EnableIndirectSpecular ? !(set.AvoidCausticPaths && payloadIsDiffuse) : (depth == 1));
        if (!enableDiffuse && !enableSpecular) break;
        if (!furnace && !packedNMR) texRough = sample_tex_desc<kGroupedTaps>(A.S, tex_desc(mat.roughness), surf.u, surf.v).r;
        const float sqrtRoughness = saturate(texRough * set.RoughnessScale);
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
            Texel4 em = sample_tex_desc<kGroupedTaps>(A.S, tex_desc(mat.emissive), surf.u, surf.v);
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

// ---- wavefront passes (DXRPT_OPT_MEGAKERNEL_PATHS 0) ---------------------------------------------
// Closest hit of the depth's queued radiance rays, one per lane.
template <bool kCount>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(7))) void k_trace(KArgs A, int depth) {
    lut_fill(A.S);
    const uint32_t* cnt = radiance_counts(A.F, depth);
    const uint32_t n = queue_total(cnt);
    const uint32_t i = blockIdx.x * kWave + threadIdx.x;
    if (i >= n) return;
    const uint32_t pos = queue_pos(cnt, A.F.cap_r, i);
    const float4 o4 = A.F.q[depth & 1].org[pos];
    const float4 d4 = A.F.q[depth & 1].dir[pos];
    // Primary rays start at TMin 0 (RayTrace.hlsl:118); continuation rays at 1e-5 (:382).
    const float tmin = depth == 1 ? 0.0f : kRayTMin;
    // RAY_FLAG_FORCE_OPAQUE iff PathLength > MaxAnyHitPathLength (RayTrace.hlsl:132, 401)
    const bool alpha = depth <= A.P.set.MaxAnyHitPathLength;
    HitRec h;
    uint32_t nv = 0, nt = 0;
    traverse8<false, kCount>(A.S, ld3(o4), ld3(d4), tmin, o4.w, alpha, h, nv, nt);
    A.F.hit[pos] = make_float4(h.b1, h.b2, bitsf(h.tri), bitsf(h.geom));
    if (kCount) {  // census counters: [0..4] depth-1 vertices, [5..9] deeper
        atomicAdd(&A.P.trav[(depth == 1 ? 0 : 5) + 0], (unsigned long long)nv);
        atomicAdd(&A.P.trav[(depth == 1 ? 0 : 5) + 1], (unsigned long long)nt);
    }
}

// MissShader (RayTrace.hlsl:509-530) and ClosestHitShader -> PathTrace (151-441) of the depth's queue:
// shadow rays into the per-slot buffers and the depth's shadow queue, the continuation into queue[d+1]
// (wave64 ballot + popcount, one atomic per wave and shard), the radiance so far along with it.
__global__ __launch_bounds__(kBlock) void k_shade(KArgs A, int depth) {
    lut_fill(A.S);
    const uint32_t* cnt = radiance_counts(A.F, depth);
    const uint32_t nq = queue_total(cnt);
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= nq) return;
    const uint32_t shard = (i >> 6) % kQueueShards;  // the wave's shard in the queues it produces
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
    // Always add (also when zero): keeps NaN/inf propagation identical to the recursive form.
    rad4.x += pathThr.x * O.local.x;
    rad4.y += pathThr.y * O.local.y;
    rad4.z += pathThr.z * O.local.z;
    A.F.sh_n[pos] = nsh;

    // one atomic for all of the wave's shadow rays: ray k of every lane after rays 0..k-1 of all lanes
    uint32_t* shcnt = A.F.counters + (kMaxDepthQueues + uint32_t(depth)) * kQueueShards;
    const uint32_t cap_s = A.F.shadow_slots * A.F.cap_r;
    {
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
    const uint32_t npos = queue_append(A.F.counters + uint32_t(depth + 1) * kQueueShards, A.F.cap_r, O.cont, shard);
    if (O.cont) {
        const RayQueue& N = A.F.q[(depth + 1) & 1];
        N.org[npos] = make_float4(O.nextOrigin.x, O.nextOrigin.y, O.nextOrigin.z, kFP32Max);
        N.dir[npos] = make_float4(O.nextDir.x, O.nextDir.y, O.nextDir.z, bitsf(pathSlot));
        N.thr[npos] = make_float4(O.nextThr.x, O.nextThr.y, O.nextThr.z, O.nextRoughness);
        N.rad[npos] = make_float4(rad4.x, rad4.y, rad4.z, bitsf(O.nextIsDiffuse ? 1u : 0u));  // payload.IsDiffuse
        N.pix[npos] = Q.pix[pos];
        A.F.fwd[pos] = npos;
    } else {
        A.F.px_rad[pathSlot] = rad4;
        A.F.fwd[pos] = ~0u;
    }
}

// ShadowHitShader / ShadowMissShader / ShadowAnyHitShader (RayTrace.hlsl:497-507, 532-542): one lane per
// queued shadow ray; occluded -> contribution * 0 in place (keeps NaN/Inf).
template <bool kCount>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(8))) void k_shadow(KArgs A, int depth) {
    lut_fill(A.S);
    const uint32_t* cnt = shadow_counts(A.F, depth);
    const uint32_t count = queue_total(cnt);
    const uint32_t i = blockIdx.x * kWave + threadIdx.x;
    if (i >= count) return;
    const uint32_t slot = A.F.sh_queue[queue_pos(cnt, A.F.shadow_slots * A.F.cap_r, i)];
    const float4 o4 = A.F.sh_org[slot];
    const float4 d4 = A.F.sh_dir[slot];
    const float4 c4 = A.F.sh_con[slot];
    HitRec h;
    uint32_t nv = 0, nt = 0;
    if (traverse8<true, kCount>(A.S, ld3(o4), ld3(d4), d4.w, o4.w, fbits(c4.w) == 0u, h, nv, nt))
        A.F.sh_con[slot] = make_float4(c4.x * 0.0f, c4.y * 0.0f, c4.z * 0.0f, c4.w);
    if (kCount) {
        atomicAdd(&A.P.trav[(depth == 1 ? 0 : 5) + 2], (unsigned long long)nv);
        atomicAdd(&A.P.trav[(depth == 1 ? 0 : 5) + 3], (unsigned long long)nt);
    }
}

// Packet variants of k_trace / k_shadow (traverse8_packet): one item per lane, whole waves exit past the
// end of the queue, the rest run with live = false on the surplus lanes.
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(7))) void k_trace_packet(KArgs A, int depth) {
    lut_fill(A.S);
    const uint32_t* cnt = radiance_counts(A.F, depth);
    const uint32_t n = queue_total(cnt);
    const uint32_t i = blockIdx.x * kWave + threadIdx.x;
    if ((i & ~63u) >= n) return;
    const bool live = i < n;
    const uint32_t pos = live ? queue_pos(cnt, A.F.cap_r, i) : 0u;
    float4 o4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), d4 = make_float4(0.0f, 0.0f, 1.0f, 0.0f);
    if (live) {
        o4 = A.F.q[depth & 1].org[pos];
        d4 = A.F.q[depth & 1].dir[pos];
    }
    HitRec h;
    traverse8_packet<false>(A.S, ld3(o4), ld3(d4), depth == 1 ? 0.0f : kRayTMin, o4.w, depth <= A.P.set.MaxAnyHitPathLength,
                            live, h);
    if (live) A.F.hit[pos] = make_float4(h.b1, h.b2, bitsf(h.tri), bitsf(h.geom));
}

__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(8))) void k_shadow_packet(KArgs A, int depth) {
    lut_fill(A.S);
    const uint32_t* cnt = shadow_counts(A.F, depth);
    const uint32_t n = queue_total(cnt);
    const uint32_t i = blockIdx.x * kWave + threadIdx.x;
    if ((i & ~63u) >= n) return;
    const bool live = i < n;
    const uint32_t slot = live ? A.F.sh_queue[queue_pos(cnt, A.F.shadow_slots * A.F.cap_r, i)] : 0u;
    float4 o4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), d4 = make_float4(0.0f, 0.0f, 1.0f, 0.0f), c4 = o4;
    if (live) {
        o4 = A.F.sh_org[slot];
        d4 = A.F.sh_dir[slot];
        c4 = A.F.sh_con[slot];
    }
    HitRec h;
    const bool occluded = traverse8_packet<true>(A.S, ld3(o4), ld3(d4), d4.w, o4.w, fbits(c4.w) == 0u, live, h);
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
// DXRPT_DEBUG builds (make variant NAME=debug EXTRA=-DDXRPT_DEBUG=1; dxrpt_get_debug_record): the queued
// path state every tail lane reads and the stage entry every blend reads are range-checked before use --
// queue position < qsize, the queued TMax (FP32Max; the direct-mapped depth-2 queue also -1 = ended),
// accumulation index < the tile list's extent, pixel index < W x H -- the hazard class of the r05 fault
// (a frame reading another overlapped frame's scratch).  A failing lane counts the violation, the first
// one is recorded, and the lane does nothing else.  No device trap: a trapping wave ends the process with
// a queue error, on a shared box; the host reads the record (and tests assert it is empty).
#ifndef DXRPT_DEBUG
#define DXRPT_DEBUG 0
#endif
// [0] violations, [1] first kind (DXRPT_DEBUG_*), [2] its depth, [3] its lane index, [4] the bad value,
// [5] its bound, [6] entries checked, [7] reserved (the host sets 1 in debug builds)
__device__ uint32_t g_debug[kDebugWords];
PT_DEV bool debug_ok(bool ok, uint32_t kind, int d, uint32_t lane_idx, uint32_t value, uint32_t bound) {
#if DXRPT_DEBUG
    if (ok) return true;
    if (atomicAdd(&g_debug[0], 1u) == 0u) {
        g_debug[1] = kind;
        g_debug[2] = uint32_t(d);
        g_debug[3] = lane_idx;
        g_debug[4] = value;
        g_debug[5] = bound;
    }
    return false;
#else
    (void)ok, (void)kind, (void)d, (void)lane_idx, (void)value, (void)bound;
    return true;
#endif
}
PT_DEV void debug_count(uint32_t n) {
#if DXRPT_DEBUG
    if ((threadIdx.x & 63u) == 0u && n) atomicAdd(&g_debug[6], n);
#else
    (void)n;
#endif
}

PT_DEV void finish_pixel(const KArgs& A, uint32_t a, float4 r) {
    if (DXRPT_DEBUG && !debug_ok(a < A.P.accum_extent, DXRPT_DEBUG_ACCUM_INDEX, 0, 0u, a, A.P.accum_extent)) return;
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
    if (DXRPT_DEBUG && !debug_ok(a < A.P.accum_extent, DXRPT_DEBUG_ACCUM_INDEX, -1, p, a, A.P.accum_extent)) return;
    accumulate_pixel(A, a, A.P.stage[a]);
}

__global__ __launch_bounds__(kBlock) void k_accumulate(KArgs A) {
    const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= A.P.num_paths) return;
    accumulate_pixel(A, A.F.ps_pix[p].y, A.F.px_rad[p]);
}

// ---- megakernel --------------------------------------------------------------------------------------
// One lane per path runs the whole frame: raygen, then per depth the closest hit, path_vertex and the
// vertex's shadow rays (any hit, in slot order), then the accumulation -- no passes, no queues; a frame
// costs its slowest WAVE's path instead of the sum over passes of each pass's slowest wave.  The
// radiance is summed in the wavefront's order (local terms, then each vertex's shadow contributions in
// slot order), so frames are bit-identical to it.  Shadow rays go through the same per-slot buffers
// (slot k * qsize + path), so any number of spot lights works.  Ray counts are added to the queue
// counters (shard = wave % kQueueShards) for dxrpt_get_stats.
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
constexpr int kPhaseSets = 3;
// Three sets of 8 phases: [0, 8) the single k_path (above), [8, 16) k_path_head, [16, 24) k_path_tail --
// 0 ray setup + closest hit, 1 shading (path_vertex), 2 continuation push, 3 / 4 / 5 shadow slot 0 / 1 /
// >= 2 (sun, sky visibility or first spot light, the rest), 6 radiance hand-off, 7 waiting for the wave's
// other lanes after the lane's path ended.
__device__ unsigned long long g_phase_ticks[kPhaseSets * 8];
PT_DEV void phase_mark(PhaseAcc* pa, int k) {
#if DXRPT_DIAG_PHASES
    if (pa) {
        const uint32_t now = uint32_t(__builtin_amdgcn_s_memrealtime());
        pa->a[k] += now - pa->t;
        pa->t = now;
    }
#endif
}
PT_DEV void phase_flush(PhaseAcc* pa, int set = 0) {
#if DXRPT_DIAG_PHASES
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        uint32_t v = pa->a[k];
        for (int off = 32; off > 0; off >>= 1) v += uint32_t(__shfl_xor(int(v), off));
        if ((threadIdx.x & 63u) == 0u) atomicAdd(&g_phase_ticks[set * 8 + k], (unsigned long long)v);
    }
#endif
}
PT_DEV PhaseAcc phase_start() {
    PhaseAcc pa = {{0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}, 0u};
#if DXRPT_DIAG_PHASES
    pa.t = uint32_t(__builtin_amdgcn_s_memrealtime());
#endif
    return pa;
}

// A vertex's shadow rays (ShadowHit/Miss/AnyHit, RayTrace.hlsl:497-507, 532-542) in its per-slot buffers
// at slot_p, walked slot by slot by the wave; contribution * visibility is added to rad in slot order.
// At depth 1 (packet bit 1) the sun shadow rays of an 8x8 pixel block's primary hits -- one direction,
// nearby origins -- take the wave-coherent traversal (all lanes active).  A lane whose slot 0 holds another
// kind of ray (a spot light's, or at MaxPathLength 2 the sky visibility ray: random directions) traces it
// per lane, after the packet.  cnt[2..3]: the census' any-hit node / triangle fetches.
template <bool kCount, bool kNear = false, bool kGA = true, bool kSpec = false, bool kNT = kSplitNT>
PT_DEV void vertex_shadows(const KArgs& A, int d, uint32_t slot_p, uint32_t nsh, bool sun0, uint32_t packet, float4& rad,
                           uint32_t* cnt, PhaseAcc* pa = nullptr) {
    uint32_t unused[4] = {0u, 0u, 0u, 0u};
    if (!kCount) cnt = unused;
    for (uint32_t k = 0; __ballot(k < nsh) != 0ull; phase_mark(pa, 3 + int(k < 2u ? k : 2u)), ++k) {
        const bool live = k < nsh;
        const size_t slot = size_t(k) * A.F.qsize + slot_p;
        float4 o4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), d4 = make_float4(0.0f, 0.0f, 1.0f, 0.0f), c4 = o4;
        if (live) {
            o4 = ld4<kNT>(A.F.sh_org + slot);
            d4 = ld4<kNT>(A.F.sh_dir + slot);
            c4 = ld4<kNT>(A.F.sh_con + slot);
        }
        HitRec hs;
        bool occluded = false;
        const bool pk = d == 1 && k == 0 && (packet & 2u);
        if (pk)
            occluded = traverse8_packet<true, kCount, !kNear, DXRPT_AH_INF >= 2, 1>(A.S, ld3(o4), ld3(d4), d4.w, o4.w, fbits(c4.w) == 0u,
                                                                          live && sun0, hs, cnt + 2);
        if (live && !(pk && sun0))
            occluded = traverse8<true, kCount, false, kNear, kGA, kSpec>(A.S, ld3(o4), ld3(d4), d4.w, o4.w, fbits(c4.w) == 0u, hs,
                                                                     cnt[2], cnt[3]);
        if (live) {
            rad.x += occluded ? c4.x * 0.0f : c4.x;
            rad.y += occluded ? c4.y * 0.0f : c4.y;
            rad.z += occluded ? c4.z * 0.0f : c4.z;
        }
    }
}

// A vertex's (at most) two shadow rays in ONE per-lane traversal loop (r05).  Without spot lights a vertex
// emits at most the sun's shadow ray (exact SunDirectionWS, RayTrace.hlsl:242-258) and, at the path's last
// vertex, the sky-visibility ray (:415-425); both leave positionWS with TMin 1e-5 and TMax FP32Max.  A lane
// traces them back to back: when its first ray is decided (an accepted occluder, or the stack runs empty) it
// restarts from the root with the second direction while the wave's other lanes go on, so the wave waits for
// the slowest lane's SUM of the two traversals instead of the slowest first ray plus the slowest second ray.
// Each any-hit result is a boolean over every occluder of its ray, so the visibilities -- and the radiance,
// added in slot order after the loop -- are those of vertex_shadows bit for bit; so are the census counts
// (cnt[2..3]: the same node visits and triangle tests per ray).  Requires nsh <= 2 and the rays of a frame
// without spot lights (A.P.rtc.NumLights == 0).
#ifndef DXRPT_CHAIN_SHADOWS
#define DXRPT_CHAIN_SHADOWS 1
#endif
#ifndef DXRPT_CHAIN_RELOAD
#define DXRPT_CHAIN_RELOAD 0
#endif
#ifndef DXRPT_CHAIN_PAIRS
#define DXRPT_CHAIN_PAIRS 0
#endif

template <bool kCount, bool kGA = true, bool kSpec = false, bool kNT = kSplitNT>
PT_DEV void vertex_shadows_chained(const KArgs& A, uint32_t slot_p, uint32_t nsh, float4& rad, uint32_t* cnt,
                                   PhaseAcc* pa = nullptr) {
    uint32_t unused[4] = {0u, 0u, 0u, 0u};
    if (!kCount) cnt = unused;
    const size_t s0 = slot_p, s1 = size_t(A.F.qsize) + slot_p;
    bool active = nsh > 0u;
    uint32_t occ = 0u;  // bit k: the ray of slot k is occluded
    if (active) {
        // the slots' origin / direction words are read this once (DXRPT_NT_CHAIN: nontemporal); their
        // contribution words again after the loop
        const float4 o4 = ld4<kNT && DXRPT_NT_CHAIN>(A.F.sh_org + s0), d4 = ld4<kNT && DXRPT_NT_CHAIN>(A.F.sh_dir + s0);
#if DXRPT_CHAIN_RELOAD
        // the second ray read back from its slot when the lane switches to it: nothing of it held in
        // registers across the first ray's traversal (tail spills 84 -> 43 VGPRs) -- but the reload's round
        // trip stalls the wave: metric +0.6..0.8 %, tail 1.122 -> 1.135 ms (r06, profiles/r06_ab_chain_reload.txt)
#else
        const float4 d41 = nsh > 1u ? ld4<kNT && DXRPT_NT_CHAIN>(A.F.sh_dir + s1) : d4;
        const bool alpha1 = nsh > 1u ? fbits(A.F.sh_con[s1].w) == 0u : false;
        const f3 o = ld3(o4), dir1 = ld3(d41);
#endif
        const bool alpha0 = fbits(A.F.sh_con[s0].w) == 0u;
        Ray8 R;
        HitRec h;
        ray8_init(R, ld3(o4), ld3(d4), d4.w, o4.w, alpha0, h);
        uint32_t node = 0, k = 0;
        int sp = 0;
        uint2 tos = make_uint2(0u, 0u);
#if DXRPT_IFIF
        uint32_t tbase = 0, tbits = 0;
        bool more = true;
        uint32_t qbase = 0, qbits = 0;  // kSpec: the queued group
#endif
        while (active) {
#if DXRPT_IFIF
            // if-if (traverse8): one node visit or one triangle test per lane and iteration
            bool hit = false;
            if (kSpec) {
                if (more && qbits == 0u) {
                    uint32_t nb = 0, nbits = 0;
                    more = trav8_node<kCount, true, false, DXRPT_AH_INF >= 1>(A.S, R, load_node8(A.S, node), node, sp, tos, h, nb, nbits, cnt[2]);
                    if (tbits == 0u) {
                        tbase = nb;
                        tbits = nbits;
                    } else {
                        qbase = nb;
                        qbits = nbits;
                    }
                }
                if (tbits == 0u && qbits) {
                    tbase = qbase;
                    tbits = qbits;
                    qbits = 0u;
                }
            } else if (tbits == 0u) {  // (a lane here holds a pending triangle or may visit: more is true)
                more = trav8_node<kCount, true, false, DXRPT_AH_INF >= 1>(A.S, R, load_node8(A.S, node), node, sp, tos, h, tbase, tbits, cnt[2]);
            }
            if (tbits) {
                const uint32_t b = uint32_t(__builtin_ctz(tbits));
                tbits &= tbits - 1u;
#if DXRPT_CHAIN_PAIRS
                const bool two = tbits != 0u;  // a second record loaded with the first (one round trip)
                const uint32_t b1 = two ? uint32_t(__builtin_ctz(tbits)) : b;
                const TriRec ra = load_tri_raw(A.S, tbase + b), rb = load_tri_raw(A.S, tbase + b1);
                pin_tri(ra);
                pin_tri(rb);
                if (kCount) ++cnt[3];
                hit = test_tri_rec<true, kGA>(A.S, ra, R.o, R.d, R.tmin, R.tmax, R.alpha, h);
                if (!hit && two) {
                    tbits &= tbits - 1u;
                    if (kCount) ++cnt[3];
                    hit = test_tri_rec<true, kGA>(A.S, rb, R.o, R.d, R.tmin, R.tmax, R.alpha, h);
                }
#else
                if (kCount) ++cnt[3];
                hit = test_tri_rec<true, kGA>(A.S, load_tri(A.S, tbase + b), R.o, R.d, R.tmin, R.tmax, R.alpha, h);
#endif
            }
            if (hit || (!more && tbits == 0u && qbits == 0u)) {
                tbits = 0u;
                qbits = 0u;
                more = true;
#else
            uint32_t tbase = 0, tbits = 0;
            const bool more = trav8_node<kCount, true, false, DXRPT_AH_INF >= 1>(A.S, R, load_node8(A.S, node), node, sp, tos, h, tbase, tbits, cnt[2]);
            const bool hit = tbits != 0u && trav8_tris<true, kCount, kGA>(A.S, R, tbase, tbits, h, cnt[3]);
            if (hit || !more) {
#endif
                occ |= uint32_t(hit) << k;
                if (++k < nsh) {  // the second ray: same origin, TMin, TMax
#if DXRPT_CHAIN_RELOAD
                    const float4 o41 = A.F.sh_org[s1], d41 = A.F.sh_dir[s1];
                    ray8_init(R, ld3(o41), ld3(d41), d41.w, o41.w, fbits(A.F.sh_con[s1].w) == 0u, h);
#else
                    ray8_init(R, o, dir1, d4.w, o4.w, alpha1, h);
#endif
                    node = 0;
                    sp = 0;
                    tos = make_uint2(0u, 0u);
                } else {
                    active = false;
                }
            }
        }
    }
    phase_mark(pa, 3);
    for (uint32_t k = 0; k < nsh; ++k) {  // slot order, as vertex_shadows
        const float4 c4 = ld4<kNT>(A.F.sh_con + size_t(k) * A.F.qsize + slot_p);
        const bool occluded = (occ >> k) & 1u;
        rad.x += occluded ? c4.x * 0.0f : c4.x;
        rad.y += occluded ? c4.y * 0.0f : c4.y;
        rad.z += occluded ? c4.z * 0.0f : c4.z;
    }
}

// One path from its first ray (PathLength 1) to its end: per depth the closest hit, path_vertex and the
// vertex's shadow rays in slot order -- the megakernel's per-thread loop, shared by k_path (camera paths)
// and k_bake (lightmap texels).  `slot_p` (< F.qsize) indexes the per-slot shadow buffers, `pix` is the
// CMJ pattern index; `packet` bit 0 / bit 1: wave-coherent traversal for the depth-1 closest hit / the
// depth-1 sun shadow rays (all lanes must be active at depth 1 then).  Returns the radiance.
// kBake: the first ray is BakeRayGen's (TMin 0.0001, IsDiffuse, no packets) instead of RaygenShader's.
// kCount: census of the traversal work, cnt[0..4] for depth-1 vertices and cnt[5..9] for deeper ones:
// closest-hit node / triangle fetches, any-hit node / triangle fetches, radiance hits (per-lane traversals
// fetch per lane, packet traversals once per wave).
template <bool kBake, bool kCount = false, bool kNearest = false>
PT_DEV float4 trace_path(const KArgs& A, uint32_t slot_p, uint32_t pix, f3 org, f3 dir, float tmax, uint32_t packet_mask,
                         uint32_t* cnt = nullptr, PhaseAcc* pa = nullptr) {
    const dxrpt_app_settings& set = A.P.set;
    const float tmin1 = kBake ? 0.0001f : 0.0f;
    const uint32_t packet = kBake ? 0u : packet_mask;
    uint32_t unused[5] = {0u, 0u, 0u, 0u, 0u};
    f3 thr = f3{1.0f, 1.0f, 1.0f};
    float payloadRoughness = 0.0f;
    bool payloadIsDiffuse = kBake;
    float4 rad = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const int L = set.MaxPathLength < 2 ? 2 : set.MaxPathLength;
    for (int d = 1; d <= L - 1; ++d) {
        count_rays(A.F.counters + uint32_t(d) * kQueueShards, 1u);
        uint32_t* cd = kCount ? cnt + (d == 1 ? 0 : 5) : unused;
        HitRec h;
        if (d == 1 && (packet & 1u))  // coherent primary rays: wave-coherent traversal (same results)
            traverse8_packet<false, kCount>(A.S, org, dir, tmin1, tmax, d <= set.MaxAnyHitPathLength, true, h, cd);
        else
            traverse8<false, kCount, false, kNearest, true, DXRPT_SPEC_PATH != 0>(A.S, org, dir, d == 1 ? tmin1 : kRayTMin, tmax, d <= set.MaxAnyHitPathLength, h, cd[0],
                                     cd[1]);
        phase_mark(pa, d == 1 ? 0 : d == 2 ? 3 : 6);
        if (kCount && h.tri != kMiss) ++cd[4];  // radiance hits: the vertices PathTrace shades
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
        bool sun0 = false;  // slot 0 holds the sun's shadow ray (the sun is emitted first when at all)
        // material taps grouped where the budget has the registers (<= 5 waves/SIMD; k_path<7> +2.8 %, r05)
        path_vertex<kNearest>(A, d, V, [&](int kind, f3 o, f3 dd, float tmn, float tmx, f3 c, bool fo) {
            sun0 |= kind == kShadowSun;
            emit_shadow(A, slot_p, nsh, o, dd, tmn, tmx, c, fo);
        }, O);
        count_rays(A.F.counters + (kMaxDepthQueues + uint32_t(d)) * kQueueShards, nsh);
        phase_mark(pa, d == 1 ? 1 : d == 2 ? 4 : 6);
        rad.x += thr.x * O.local.x;
        rad.y += thr.y * O.local.y;
        rad.z += thr.z * O.local.z;
        // depth >= 2 (the depth-1 sun shadows of full waves take the packet traversal): the vertex's rays
        // chained in one loop where the budget has the registers (kNearest: <= 5 waves/SIMD)
        if (kNearest && DXRPT_CHAIN_SHADOWS && A.P.rtc.NumLights == 0u && (d > 1 || !(packet & 2u)))
            vertex_shadows_chained<kCount, true, DXRPT_SPEC_PATH != 0, false>(A, slot_p, nsh, rad, kCount ? cd : nullptr);
        else
            vertex_shadows<kCount, kNearest, true, DXRPT_SPEC_PATH != 0, false>(A, d, slot_p, nsh, sun0, packet, rad, cd);
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

// Path p of a wave whose paths are 64-aligned (p & ~63 .. p | 63).  Packets need every lane of the wave
// (the packet stack lives one entry per lane): a partial last wave (num_paths % 64 != 0) traverses one
// ray per lane -- a wave-uniform scalar test, the other waves keep their packets (same results).
template <bool kCount = false, bool kNearest = false>
PT_DEV void camera_path(const KArgs& A, uint32_t p, uint32_t* cnt = nullptr, PhaseAcc* pa = nullptr) {
    const PrimaryRay pr = primary_ray(A, p);
    const uint32_t packet = (p | 63u) < A.P.num_paths ? A.P.packet : 0u;
    const float4 rad = trace_path<false, kCount, kNearest>(A, p, pr.pixelIdx, pr.start, pr.dir, pr.length, packet, cnt, pa);
    finish_pixel(A, pr.accumIdx, rad);
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

PT_DEV WaveSlot wave_slot(const KArgs& A) {
    WaveSlot ws;
    const uint32_t w = uint32_t(__builtin_amdgcn_readfirstlane(int((blockIdx.x * blockDim.x + threadIdx.x) >> 6)));
    ws.slot = A.P.wave_order ? A.P.wave_order[w] : w;
    ws.t0 = A.P.wave_cost ? __builtin_amdgcn_s_memrealtime() : 0ull;
    return ws;
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

// The single megakernel, one wave per workgroup.  kCount: the census instantiation
// (DXRPT_OPT_COUNT_TRAVERSAL; wave sums, one 64-bit atomic per counter per wave, optional per-wave clock
// stamps).  kOrder: the cost-ordered dispatch (wave_slot); its own instantiation, so that the
// path-ordered kernel of large frames keeps its code (the indirection costs it ~2 %).  Otherwise
// path-ordered with XCD-local runs of blocks (FrameParams::xcd_chunk).
template <int kOcc, bool kCount = false, bool kOrder = false>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(kOcc))) void k_path(KArgs A) {
    constexpr bool kNear = kOcc <= 5;  // nearest-child-first closest hits where the register budget allows
    if (A.F.counters_next && blockIdx.x == 0u)  // the next frame's counter set (this stream's previous frame's)
        for (uint32_t i = threadIdx.x; i < kCounterWords; i += blockDim.x) A.F.counters_next[i] = 0u;
    lut_fill(A.S);
    if (kOrder) {
        const WaveSlot ws = wave_slot(A);
        const uint32_t p = (ws.slot << 6) | (threadIdx.x & 63u);
        if (p < A.P.num_paths) camera_path<false, kNear>(A, p);
        wave_slot_done(A, ws);
        return;
    }
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (kCount) {
        const unsigned long long t0 = A.P.wave_clock ? __builtin_amdgcn_s_memrealtime() : 0ull;
        uint32_t cnt[10] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
        if (p < A.P.num_paths) camera_path<true, kNear>(A, p, cnt);
        if (A.P.wave_clock && (threadIdx.x & 63u) == 0u && p < A.P.num_paths) {  // vector stores from lane 0
            const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
            A.P.wave_clock[2 * (p >> 6)] = t0;
            A.P.wave_clock[2 * (p >> 6) + 1] = t1;
        }
#pragma unroll
        for (int k = 0; k < 10; ++k) {
            uint32_t v = cnt[k];
            for (int off = 32; off > 0; off >>= 1) v += uint32_t(__shfl_xor(int(v), off));
            if ((threadIdx.x & 63u) == 0u) atomicAdd(&A.P.trav[k], (unsigned long long)v);
        }
        return;
    }
#if DXRPT_DIAG_PHASES
    PhaseAcc pa = {{0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}, uint32_t(__builtin_amdgcn_s_memrealtime())};
    if (p < A.P.num_paths) camera_path<false, kNear>(A, p, nullptr, &pa);
    phase_mark(&pa, 7);
    phase_flush(&pa);
    return;
#endif
    // XCD-local runs of blocks (FrameParams::xcd_chunk); the tail stays in order.  Run t of XCD x is chunk
    // 8 t + (x + t) mod 8: the XCDs' chunks rotate from run to run, so no XCD keeps the same screen columns.
    const uint32_t q = A.P.xcd_chunk ? xcd_position(blockIdx.x, gridDim.x, A.P.xcd_chunk) * blockDim.x + threadIdx.x : p;
    if (q < A.P.num_paths) camera_path<false, kNear>(A, q);
}

// ---- depth-split megakernel (FrameParams::split) ---------------------------------------------
// The frame as one megakernel launch per path depth: k_path_head runs every camera path from raygen
// through its first vertex (packet primaries and depth-1 sun shadows: the coherent part); k_path_tail(d)
// runs depth d of the paths still alive.  Between depths the surviving paths are compacted -- wave64
// ballot + popcount, one atomic per wave on a sharded counter -- into a queue whose entries carry the
// whole path state, so every tail wave is full of live paths, and the path state lives in the queue
// rather than in registers across the traversals: a tail keeps only the queue position and the ray
// across its closest-hit traversal and re-reads the rest afterwards, and every kernel queues the
// continuation BEFORE tracing the vertex's shadow rays, so only the radiance sum is live across them.
// Each kernel has its own register budget (FrameParams::megakernel_occupancy / tail_occupancy).  A path's
// radiance is k_path's sum, continued term by term from the queued partial sum: frames are bit-identical.
// Queue of depth d (RayQueue q[d & 1], counters d):
//   org (origin xyz, FP32Max)   dir (direction xyz, bits(accumulation index))
//   thr (throughput rgb, payload Roughness)   rad (radiance so far, bits(payload IsDiffuse))   pix (CMJ pattern)
// The queued count of depth d is that depth's radiance-ray count (dxrpt_get_stats).

// Queues the continuation of a vertex (all active lanes must call; `cont` selects) into queue d + 1;
// returns its position.  The radiance word is written later (split_finish), after the shadow rays.
// Producer wave w of nw (in screen order) appends to shard w * 64 / nw: each shard holds a contiguous
// run of screen blocks, so the next depth's waves, which take the queue in shard order, sweep the
// image like the head's (neighbouring origins resident together share the BVH nodes and texels in
// cache), while the waves running at any time still spread their atomics over several shards.
PT_DEV uint32_t split_push(const KArgs& A, int d, bool cont, const VertexOut& O, uint32_t pix, uint32_t accumIdx,
                           uint32_t w, uint32_t nw) {
    const uint32_t pos = queue_append(A.F.counters + uint32_t(d + 1) * kQueueShards, A.F.cap_r, cont,
                                      uint32_t((uint64_t(w) * kQueueShards) / nw));
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

// Census of a depth-split frame (kCount): each lane's node / triangle fetches and radiance hits (cnt[0..4]
// depth 1 in the head, cnt[5..9] deeper in the tails, as trace_path counts them), summed over the wave and
// added with one 64-bit atomic per counter per wave.  All lanes of the wave must call.
PT_DEV void census_flush(const KArgs& A, const uint32_t (&cnt)[10]) {
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        uint32_t v = cnt[k];
        for (int off = 32; off > 0; off >>= 1) v += uint32_t(__shfl_xor(int(v), off));
        if ((threadIdx.x & 63u) == 0u && v) atomicAdd(&A.P.trav[k], (unsigned long long)v);
    }
}

// Raygen + depth 1 of camera path p (the head's per-lane body).
template <bool kCount>
PT_DEV void head_path(const KArgs& A, uint32_t p, uint32_t* cnt, PhaseAcc* pa = nullptr) {
    const dxrpt_app_settings& set = A.P.set;
    const PrimaryRay pr = primary_ray(A, p);
    const uint32_t packet = (p | 63u) < A.P.num_paths ? A.P.packet : 0u;
    count_rays(A.F.counters + 1u * kQueueShards, 1u);
    HitRec h;
    uint32_t nv = 0, nt = 0;
    if (packet & 1u)  // coherent primary rays: wave-coherent traversal (same results)
        traverse8_packet<false, kCount>(A.S, pr.start, pr.dir, 0.0f, pr.length, 1 <= set.MaxAnyHitPathLength, true, h, cnt);
    else
        traverse8<false, kCount>(A.S, pr.start, pr.dir, 0.0f, pr.length, 1 <= set.MaxAnyHitPathLength, h, nv, nt);
    if (kCount) {
        cnt[0] += nv;
        cnt[1] += nt;
        if (h.tri != kMiss) ++cnt[4];
    }
    phase_mark(pa, 0);
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
        sun0 |= kind == kShadowSun;
        emit_shadow(A, p, nsh, o, dd, tmn, tmx, c, fo);
    }, O);
    count_rays(A.F.counters + (kMaxDepthQueues + 1u) * kQueueShards, nsh);
    phase_mark(pa, 1);
    const bool cont = O.cont;
    const bool nextDiffuse = O.nextIsDiffuse;
    // the depth-2 queue is direct-mapped: entry p for path slot p (>= 99 % of camera paths continue, so a
    // compacting append buys no density), written without the append's returning atomic -- the head waited
    // on it (8.5 % of its lane time, r05_phases2.txt) -- and an ended path marks its entry (TMax -1) for the
    // tail to skip.  The queue counter still counts the rays (dxrpt_stats).  r05: metric -1.9 %, C2 / C4
    // -1 %, the 1/2 share -1.4 % (profiles/r05_ab_direct.txt).
    const uint32_t qpos = p;
    count_rays(A.F.counters + 2u * kQueueShards, cont ? 1u : 0u);
    if (set.MaxPathLength > 2) {  // a depth-2 tail reads the queue
        const RayQueue& Q = A.F.q[0];
        if (cont) {
            Q.org[p] = make_float4(O.nextOrigin.x, O.nextOrigin.y, O.nextOrigin.z, kFP32Max);
            Q.dir[p] = make_float4(O.nextDir.x, O.nextDir.y, O.nextDir.z, bitsf(pr.accumIdx));
            Q.thr[p] = make_float4(O.nextThr.x, O.nextThr.y, O.nextThr.z, O.nextRoughness);
            Q.pix[p] = pr.pixelIdx;
        } else {
            Q.org[p] = make_float4(0.0f, 0.0f, 0.0f, -1.0f);
        }
    }

    float4 rad = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    rad.x += 1.0f * O.local.x;
    rad.y += 1.0f * O.local.y;
    rad.z += 1.0f * O.local.z;
    phase_mark(pa, 2);
    vertex_shadows<kCount>(A, 1, p, nsh, sun0, packet, rad, cnt, pa);
    split_finish(A, 1, cont, qpos, nextDiffuse, pr.accumIdx, rad);
    phase_mark(pa, 6);
}

// Raygen + depth 1 of every camera path (one 64-path 8x8 block per wave, XCD runs as k_path).  kCount: the
// census instantiation of the same code (the traversal orders of the timed head: packet primaries, depth-1
// sun shadows far to near).
template <int kOcc, bool kCount = false>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(kOcc))) void k_path_head(KArgs A) {
    if (A.F.counters_next && blockIdx.x == 0u)  // the next frame's counter set (see k_path)
        for (uint32_t i = threadIdx.x; i < kCounterWords; i += blockDim.x) A.F.counters_next[i] = 0u;
    lut_fill(A.S);
    const uint32_t blk = A.P.xcd_chunk ? xcd_position(blockIdx.x, gridDim.x, A.P.xcd_chunk) : blockIdx.x;
    const uint32_t p = blk * blockDim.x + threadIdx.x;  // path slot (shadow-slot index)
    if (!kCount) {
#if DXRPT_DIAG_PHASES
        PhaseAcc pa = phase_start();
        if (p < A.P.num_paths) head_path<false>(A, p, nullptr, &pa);
        phase_mark(&pa, 7);
        phase_flush(&pa, 1);
#else
        if (p < A.P.num_paths) head_path<false>(A, p, nullptr);
#endif
        return;
    }
    uint32_t cnt[10] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    if (p < A.P.num_paths) head_path<true>(A, p, cnt);
    census_flush(A, cnt);
}

#ifndef DXRPT_TAIL_PAIRS
#define DXRPT_TAIL_PAIRS 1  // the tails' closest hits test leaf triangles two per iteration (trav8_tris2)
#endif
// Depth d of queued path i (the tail's per-lane body; j = the lane's queue wave, nw = waves with work).
template <bool kCount, bool kLast>
PT_DEV void tail_path(const KArgs& A, int d, uint32_t i, uint32_t j, uint32_t nw, const uint32_t* cnt_q, uint32_t* cnt,
                      PhaseAcc* pa = nullptr) {
    const dxrpt_app_settings& set = A.P.set;
    const bool direct = d == 2;  // the head's direct-mapped queue (entry = path slot)
    const uint32_t pos = direct ? i : queue_pos(cnt_q, A.F.cap_r, i);
    const RayQueue& Q = A.F.q[d & 1];
    if (DXRPT_DEBUG && !debug_ok(pos < A.F.qsize, DXRPT_DEBUG_QUEUE_POS, d, i, pos, A.F.qsize)) return;
    HitRec h;
    {
        const float4 o4 = Q.org[pos], d4 = Q.dir[pos];  // read again after the traversal (nontemporal there)
        if (DXRPT_DEBUG) {  // the queued state before it is used (the lane then does nothing else)
            const bool ended = direct && o4.w == -1.0f;
            const uint32_t a = fbits(d4.w), px = ended ? 0u : Q.pix[pos];
            if (!debug_ok(ended || o4.w == kFP32Max, DXRPT_DEBUG_TMAX, d, i, fbits(o4.w), fbits(kFP32Max)) ||
                !debug_ok(ended || a < A.P.accum_extent, DXRPT_DEBUG_ACCUM_INDEX, d, i, a, A.P.accum_extent) ||
                !debug_ok(ended || px < A.P.width * A.P.height, DXRPT_DEBUG_PIXEL, d, i, px, A.P.width * A.P.height))
                return;
        }
        if (direct && !(o4.w >= 0.0f)) return;  // the path ended at depth 1
        uint32_t nv = 0, nt = 0;
        traverse8<false, kCount, DXRPT_TAIL_PAIRS != 0, true, false>(A.S, ld3(o4), ld3(d4), kRayTMin, o4.w, d <= set.MaxAnyHitPathLength,
                                                                   h, nv, nt);
        if (kCount) {
            cnt[5] += nv;
            cnt[6] += nt;
            if (h.tri != kMiss) ++cnt[9];
        }
    }
    phase_mark(pa, 0);
    // the rest of the path state comes back from the queue after the traversal (the radiance so far only
    // once the vertex is shaded: it is not live across path_vertex)
    const float4 o4 = ld4<kSplitNT>(Q.org + pos), d4 = ld4<kSplitNT>(Q.dir + pos), t4 = ld4<kSplitNT>(Q.thr + pos);
    const float rw = reinterpret_cast<const float*>(Q.rad + pos)[3];
    const uint32_t accumIdx = fbits(d4.w);
    VertexIn V;
    V.inOrigin = ld3(o4);
    V.inDir = ld3(d4);
    V.pathThr = ld3(t4);
    V.payloadRoughness = t4.w;
    V.payloadIsDiffuse = (fbits(rw) & 1u) != 0u;
    V.pix = ld1<kSplitNT>(Q.pix + pos);
    V.hit = make_float4(h.b1, h.b2, bitsf(h.tri), bitsf(h.geom));
    VertexOut O;
    uint32_t nsh = 0;
    // per-texel taps (r05: the grouped form is neutral here even with two taps per hit, r05_ab_tailgrp.txt)
    path_vertex<false>(A, d, V, [&](int, f3 o, f3 dd, float tmn, float tmx, f3 c, bool fo) {
        emit_shadow(A, i, nsh, o, dd, tmn, tmx, c, fo);  // shadow slots by the dense index (< qsize)
    }, O);
    count_rays(A.F.counters + (kMaxDepthQueues + uint32_t(d)) * kQueueShards, nsh);
    phase_mark(pa, 1);
    // the last depth's vertices never continue (path_vertex: depth + 1 < MaxPathLength); stating it
    // (cont = false for kLast) frees registers across the shadow loop -- spills 79 -> 46 VGPRs -- but measured
    // 0.5-0.9 % slower (r06_ab_lastcont.txt)
    const bool cont = O.cont;
    const bool nextDiffuse = O.nextIsDiffuse;
    const int L = set.MaxPathLength < 2 ? 2 : set.MaxPathLength;
    const uint32_t qpos = d + 1 <= L - 1 ? split_push(A, d, cont, O, V.pix, accumIdx, j, nw) : 0u;
    const float4 r4 = ld4<kSplitNT>(Q.rad + pos);
    float4 rad = make_float4(r4.x, r4.y, r4.z, 0.0f);
    rad.x += V.pathThr.x * O.local.x;
    rad.y += V.pathThr.y * O.local.y;
    rad.z += V.pathThr.z * O.local.z;
    phase_mark(pa, 2);
    // the last depth's vertices emit the sun's and the sky-visibility ray: chained (wave-uniform test: no spot
    // lights, <= 2 rays per vertex); the other depths have at most the sun's and keep the slot loop, in
    // instantiations without the chained code (its registers cost the single-ray tails 2-3 %, r05)
    if (kLast && DXRPT_CHAIN_SHADOWS && A.P.rtc.NumLights == 0u)
        vertex_shadows_chained<kCount, false>(A, i, nsh, rad, kCount ? cnt + 5 : nullptr, pa);
    else
        vertex_shadows<kCount, true, false>(A, d, i, nsh, false, 0u, rad, kCount ? cnt + 5 : nullptr, pa);
    split_finish(A, d, cont, qpos, nextDiffuse, accumIdx, rad);
    phase_mark(pa, 6);
}

// Depth d of the paths queued for it (one per lane); waves past the queued count exit at once (the grid
// covers every path of the frame).  kCount: the census instantiation (the tails' traversal orders: closest
// hits nearest child first with triangle pairs, any-hit rays far to near).
template <int kOcc, bool kCount = false, bool kLast = false>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(kOcc))) void k_path_tail(KArgs A, int d) {
    const uint32_t* cnt_q = A.F.counters + uint32_t(d) * kQueueShards;
    const uint32_t n = d == 2 ? A.P.num_paths : queue_total(cnt_q);  // depth 2: every path slot (direct-mapped)
    const uint32_t nw = (n + 63u) / 64u;  // waves with work
    // wave j of the queue: XCD runs of A.P.xcd_chunk consecutive queue chunks among the nw live waves
    // (workgroup b runs on XCD b mod 8; the grid's surplus workgroups exit at once)
    if (blockIdx.x >= nw) return;
    const uint32_t j = A.P.xcd_chunk ? xcd_position(blockIdx.x, nw, A.P.xcd_chunk) : blockIdx.x;
    lut_fill<kLast>(A.S);  // the plain copy in the non-last tails (DMA there: C3 +1.8 %, C5 +1.3 %)
    const uint32_t i = j * blockDim.x + threadIdx.x;
    if (DXRPT_DEBUG) debug_count(n - j * 64u < 64u ? n - j * 64u : 64u);
    if (!kCount) {
#if DXRPT_DIAG_PHASES
        PhaseAcc pa = phase_start();
        if (i < n) tail_path<false, kLast>(A, d, i, j, nw, cnt_q, nullptr, &pa);
        phase_mark(&pa, 7);
        phase_flush(&pa, 2);
#else
        if (i < n) tail_path<false, kLast>(A, d, i, j, nw, cnt_q, nullptr);
#endif
        return;
    }
    uint32_t cnt[10] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    if (i < n) tail_path<true, kLast>(A, d, i, j, nw, cnt_q, cnt);
    census_flush(A, cnt);
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
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(kOcc))) void k_bake(KArgs A, BakeArgs B) {
    lut_fill(A.S);
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
    const float4 r = trace_path<true>(A, i, texel, origin, dir, kFP32Max, 0u);
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
__global__ __launch_bounds__(kWave) void k_trace_rays(SceneDev S, const float4* rays, uint32_t n, uint32_t flags, float4* hits) {
    lut_fill(S);
    const uint32_t i = blockIdx.x * kWave + threadIdx.x;
    if (i >= n) return;
    const float4 a = rays[2 * i], b = rays[2 * i + 1];
    HitRec h;
    uint32_t nv = 0, nt = 0;
    const bool alpha = (flags & 2u) != 0u;
    if (flags & 1u) {
        const bool occ = traverse8<true, false>(S, ld3(a), ld3(b), a.w, b.w, alpha, h, nv, nt);
        hits[i] = make_float4(occ ? 1.0f : -1.0f, 0.0f, 0.0f, bitsf(kMiss));
    } else {
        const bool any = traverse8<false, false>(S, ld3(a), ld3(b), a.w, b.w, alpha, h, nv, nt);
        hits[i] = any ? make_float4(h.t, h.b1, h.b2, bitsf(h.tri)) : make_float4(-1.0f, 0.0f, 0.0f, bitsf(kMiss));
    }
}

// ---- launches -------------------------------------------------------------------------------------
static inline uint32_t grid_for(uint32_t n, uint32_t block) { return (n + block - 1u) / block; }

uint32_t frame_traversal_threads(uint32_t num_paths, uint32_t shadow_slots, bool megakernel) {
    // megakernel schedules: one lane per path slot (k_path, k_path_head, k_path_tail, k_bake); the
    // wavefront's any-hit pass: one lane per queued shadow ray
    const uint64_t n = megakernel ? uint64_t(num_paths) : uint64_t(num_paths) * std::max<uint32_t>(shadow_slots, 1u);
    return uint32_t(((n + kWave - 1u) / kWave) * kWave);
}

uint32_t trace_rays_threads(uint32_t n) { return grid_for(n, kWave) * kWave; }

// Kernel instantiations by register budget (waves per SIMD): the megakernels take 4..7.
#define DXRPT_OCC_SWITCH(occ, launch) \
    switch (occ) {                     \
        case 7: launch(7); break;      \
        case 6: launch(6); break;      \
        case 5: launch(5); break;      \
        default: launch(4); break;     \
    }

// The depth-split schedule (FrameParams::split): the head, then one tail launch per depth; head_ev
// (per-kernel timing) is recorded between them.
// census: the counting instantiations of the shipped budgets (head 5, tails 7), whose traversal code is
// the timed kernels' -- their counts are the fetches of the schedule bench.py times (verdict r04 #2).
static void launch_split(const KArgs& A, uint32_t gm, size_t lds, hipStream_t s, hipEvent_t head_ev, bool census) {
    const FrameParams& fp = A.P;
    const int L = fp.set.MaxPathLength < 2 ? 2 : fp.set.MaxPathLength;
    if (census) {
        hipLaunchKernelGGL((k_path_head<5, true>), dim3(gm), dim3(kWave), lds, s, A);
        for (int d = 2; d <= L - 1; ++d) {
            if (d < L - 1) hipLaunchKernelGGL((k_path_tail<7, true, false>), dim3(gm), dim3(kWave), lds, s, A, d);
            else hipLaunchKernelGGL((k_path_tail<7, true, true>), dim3(gm), dim3(kWave), lds, s, A, d);
        }
        return;
    }
#define DXRPT_HEAD(O) hipLaunchKernelGGL((k_path_head<O>), dim3(gm), dim3(kWave), lds, s, A)
    DXRPT_OCC_SWITCH(fp.megakernel_occupancy, DXRPT_HEAD)
#undef DXRPT_HEAD
    if (head_ev) (void)hipEventRecord(head_ev, s);
    for (int d = 2; d <= L - 1; ++d) {  // the last depth's tail: its own instantiation (chained shadow rays)
#define DXRPT_TAIL(O) hipLaunchKernelGGL((k_path_tail<O, false, false>), dim3(gm), dim3(kWave), lds, s, A, d)
#define DXRPT_TAIL_LAST(O) hipLaunchKernelGGL((k_path_tail<O, false, true>), dim3(gm), dim3(kWave), lds, s, A, d)
        if (d < L - 1) {
            DXRPT_OCC_SWITCH(fp.tail_occupancy, DXRPT_TAIL)
        } else {
            DXRPT_OCC_SWITCH(fp.tail_occupancy, DXRPT_TAIL_LAST)
        }
#undef DXRPT_TAIL
#undef DXRPT_TAIL_LAST
    }
}

hipError_t launch_accum_stage(const FrameParams& fp, hipStream_t stream) {
    if (fp.num_paths == 0 || !fp.stage) return hipSuccess;
    KArgs A{SceneDev{}, FrameBuffers{}, fp};
    hipLaunchKernelGGL(k_accum_stage, dim3(grid_for(fp.num_paths, kBlock)), dim3(kBlock), 0, stream, A);
    return hipGetLastError();
}

hipError_t launch_frame(const SceneDev& scene, const FrameBuffers& fb, const FrameParams& fp, hipStream_t stream,
                        hipEvent_t* ev, hipStream_t aux, hipEvent_t* fork_ev, uint32_t* sched_out) {
    KArgs A{scene, fb, fp};
    uint32_t sched_local = 0;
    uint32_t& sched = sched_out ? *sched_out : sched_local;
    sched = 0;
    const uint32_t g = grid_for(fp.num_paths, kBlock);
    const size_t lds = size_t(scene.stack_ints) * kWave * sizeof(int);  // one wave's LDS stacks
    const bool count = fp.trav != nullptr;
    static_assert(kCounterWords >= 2 * kMaxDepthQueues * kQueueShards && kCounterWords % 4 == 0, "counter set");
    hipError_t e = fb.counters_clean ? hipSuccess : hipMemsetAsync(fb.counters, 0, kCounterWords * sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    if (fp.megakernel) {  // timing: ev[0], ev[1] bracket the frame's megakernel launches (ev[2]: after the head)
        const uint32_t gm = grid_for(fp.num_paths, kWave);
        const bool ordered = fp.wave_cost || fp.wave_order;
        sched = DXRPT_SCHED_MEGAKERNEL;
        if (ev) (void)hipEventRecord(ev[0], stream);
        if (count && fp.split && !ordered && !fp.wave_clock) {
            // census frame (DXRPT_OPT_COUNT_TRAVERSAL) of a depth-split frame: the counting head and tails
            sched |= DXRPT_SCHED_CENSUS | DXRPT_SCHED_SPLIT;
            launch_split(A, gm, lds, stream, nullptr, true);
        } else if (count) {  // census frame of the single kernel: its counting instantiation, with the
                             // traversal orders of the budget it stands for (k_path<5> walks closest hits
                             // nearest-first and packet shadows near to far like k_path at <= 5 waves/SIMD;
                             // k_path<7> like k_path at 6-7); with wave clocks, split frames count here too
            sched |= DXRPT_SCHED_CENSUS;
            if ((fp.split && !ordered) || fp.megakernel_occupancy <= 5)
                hipLaunchKernelGGL((k_path<5, true>), dim3(gm), dim3(kWave), lds, stream, A);
            else
                hipLaunchKernelGGL((k_path<7, true>), dim3(gm), dim3(kWave), lds, stream, A);
        } else if (fp.split && !ordered) {
            sched |= DXRPT_SCHED_SPLIT;
            launch_split(A, gm, lds, stream, ev ? ev[2] : nullptr, false);
        } else if (ordered) {  // cost-ordered waves
            sched |= DXRPT_SCHED_ORDER_KERNEL | (fp.wave_order ? DXRPT_SCHED_COST_ORDERED : 0u);
#define DXRPT_PATH(O) hipLaunchKernelGGL((k_path<O, false, true>), dim3(gm), dim3(kWave), lds, stream, A)
            DXRPT_OCC_SWITCH(fp.megakernel_occupancy, DXRPT_PATH)
#undef DXRPT_PATH
        } else {
#define DXRPT_PATH(O) hipLaunchKernelGGL((k_path<O>), dim3(gm), dim3(kWave), lds, stream, A)
            DXRPT_OCC_SWITCH(fp.megakernel_occupancy, DXRPT_PATH)
#undef DXRPT_PATH
        }
        if (ev) (void)hipEventRecord(ev[1], stream);
        return hipGetLastError();
    }
    // wavefront passes; per-kernel timing: launch slot i (raygen, then trace/shade/shadow/resolve per depth,
    // then accumulate) is bracketed by ev[2i], ev[2i+1] recorded on the stream the kernel runs on (the
    // frame's first start and last stop events are always recorded: they bracket the frame)
    const int L = fp.set.MaxPathLength < 2 ? 2 : fp.set.MaxPathLength;
    const int last_slot = 1 + 4 * (L - 1);
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
    start(0, stream);
    hipLaunchKernelGGL(k_raygen, dim3(g), dim3(kBlock), 0, stream, A);
    stop(0, stream);
    const uint32_t gt = grid_for(fp.num_paths, kWave);
    const uint32_t gst = grid_for(fp.num_paths * fb.shadow_slots, kWave);  // one lane per queued shadow ray (bound)
    // one lane per ray; packet traversal: bit 0 closest hit at depth 1, bit 1 any hit at depth 1, bits 2/3 deeper
    auto radiance = [&](int d, hipStream_t st) {
        start(slot_of(d, 0), st);
        if (!count && (fp.packet & (1u << (d == 1 ? 0 : 2)))) hipLaunchKernelGGL(k_trace_packet, dim3(gt), dim3(kWave), lds, st, A, d);
        else if (count) hipLaunchKernelGGL((k_trace<true>), dim3(gt), dim3(kWave), lds, st, A, d);
        else hipLaunchKernelGGL((k_trace<false>), dim3(gt), dim3(kWave), lds, st, A, d);
        stop(slot_of(d, 0), st);
    };
    auto shadow = [&](int d, hipStream_t st) {
        start(slot_of(d, 2), st);
        if (!count && (fp.packet & (2u << (d == 1 ? 0 : 2)))) hipLaunchKernelGGL(k_shadow_packet, dim3(gst), dim3(kWave), lds, st, A, d);
        else if (count) hipLaunchKernelGGL((k_shadow<true>), dim3(gst), dim3(kWave), lds, st, A, d);
        else hipLaunchKernelGGL((k_shadow<false>), dim3(gst), dim3(kWave), lds, st, A, d);
        stop(slot_of(d, 2), st);
    };
    // Fork/join: k_shadow(d) and k_trace(d+1) both only need k_shade(d), so the any-hit pass runs on `aux`
    // concurrently with the next closest-hit pass; k_resolve(d) joins both before k_shade(d+1).
    const bool fork = aux != nullptr && fork_ev != nullptr;
    for (int d = 1; d <= L - 1; ++d) {
        if (d == 1 || !fork) radiance(d, stream);
        start(slot_of(d, 1), stream);
        hipLaunchKernelGGL(k_shade, dim3(g), dim3(kBlock), 0, stream, A, d);
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
    const size_t lds = size_t(scene.stack_ints) * kWave * sizeof(int);
    const dim3 g(grid_for(b.span, kWave));
#define DXRPT_BAKE(O) hipLaunchKernelGGL((k_bake<O>), g, dim3(kWave), lds, stream, A, b)
    DXRPT_OCC_SWITCH(fp.megakernel_occupancy, DXRPT_BAKE)
#undef DXRPT_BAKE
    return hipGetLastError();
}

hipError_t launch_trace_rays(const SceneDev& scene, const float4* rays, uint32_t n, uint32_t flags, float4* hits,
                             hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const size_t lds = size_t(scene.stack_ints) * kWave * sizeof(int);
    hipLaunchKernelGGL(k_trace_rays, dim3(grid_for(n, kWave)), dim3(kWave), lds, stream, scene, rays, n, flags, hits);
    return hipGetLastError();
}

// Primary-only AOV (SURVEY.md 8(d), C1 plumbing): RaygenShader's ray for path slot p (the tiles of the
// call), its closest hit (packet traversal on full waves, as k_path's depth 1), and the albedo tap
// PathTrace takes at the hit (RayTrace.hlsl:180-183); out[accumIdx] = (albedo rgb, 1) on a hit, 0 on a
// miss.  No shading, no accumulation: a debug view of the ray-generation / traversal / surface plumbing.
__global__ __launch_bounds__(kWave) void k_primary_aov(KArgs A) {
    lut_fill(A.S);
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= A.P.num_paths) return;
    const PrimaryRay pr = primary_ray(A, p);
    HitRec h;
    uint32_t nv = 0, nt = 0;
    const bool alpha = 1 <= A.P.set.MaxAnyHitPathLength;
    if ((p | 63u) < A.P.num_paths && (A.P.packet & 1u))
        traverse8_packet<false>(A.S, pr.start, pr.dir, 0.0f, pr.length, alpha, true, h);
    else
        traverse8<false, false>(A.S, pr.start, pr.dir, 0.0f, pr.length, alpha, h, nv, nt);
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
    const size_t lds = size_t(scene.stack_ints) * kWave * sizeof(int);
    hipLaunchKernelGGL(k_primary_aov, dim3(grid_for(fp.num_paths, kWave)), dim3(kWave), lds, stream, A);
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
    hipLaunchKernelGGL(k_sample_cmj, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, stream, cases, n, out);
    return hipGetLastError();
}

hipError_t read_debug_record(uint32_t out[kDebugWords]) {
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) return e;
    if ((e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_debug), kDebugWords * sizeof(uint32_t))) != hipSuccess) return e;
    out[7] = DXRPT_DEBUG ? 1u : 0u;
    const uint32_t zero[kDebugWords] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_debug), zero, sizeof(zero));
}

hipError_t read_phase_ticks(unsigned long long out[kPhaseClockWords]) {
    static_assert(kPhaseClockWords == kPhaseSets * 8, "phase clock sets");
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) return e;
    if ((e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase_ticks), kPhaseClockWords * sizeof(unsigned long long))) != hipSuccess)
        return e;
    const unsigned long long zero[kPhaseClockWords] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_phase_ticks), zero, sizeof(zero));
}

}  // namespace dxrpt
