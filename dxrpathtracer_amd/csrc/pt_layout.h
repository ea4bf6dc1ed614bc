// pt_layout.h — device-memory layouts shared by the host-side builders (bvh_build.cpp,
// dxrpt_api.hip) and the gfx950 kernels (pt_kernels.hip).  Plain C++ PODs only.
//
// HBM layout of one context (all arrays 256-B aligned, built once per scene):
//   nodes     BvhNode[num_nodes]        64 B   BVH2, two child AABBs per node (replaces the DXR BLAS,
//                                              DXRPathTracer.cpp:2331-2488)
//   tris      TriRecord[num_tris]       48 B   leaf-ordered triangles: v0, e1=v1-v0, e2=v2-v0 + ids
//   vertices  dxrpt_mesh_vertex[nv]     64 B   AoS, exactly the reference MeshVertex (Model.h:25-67)
//   indices   uint32[ni]                 4 B   mesh-local, R16 inputs are widened on upload
//   geoinfo   dxrpt_geometry_info[ng]   16 B
//   materials dxrpt_material[nm]        24 B
//   texdesc   TexDesc[nt]               16 B   -> texels (one pool of 32-bit words)
//   sky       uint16[6*res*res*4]        8 B/texel RGBA16F cube
// Per-frame (wavefront) buffers are described in pt_kernels.hip.
#pragma once
#include <stdint.h>

namespace dxrpt {

// BVH2 node, 64 B (four 16-B words, read with two/four dwordx4 loads).
//   a = (c0.lo.x, c0.hi.x, c0.lo.y, c0.hi.y)
//   b = (c1.lo.x, c1.hi.x, c1.lo.y, c1.hi.y)
//   c = (c0.lo.z, c0.hi.z, c1.lo.z, c1.hi.z)
//   d = (child0, child1, 0, 0): child >= 0 -> internal node index;
//       child < 0 -> leaf, ~child = (first_tri << 3) | (count - 1), 1 <= count <= 8.
struct BvhNode {
    float a[4];
    float b[4];
    float c[4];
    int32_t d[4];
};
static_assert(sizeof(BvhNode) == 64, "BvhNode must be 64 B");

constexpr int kMaxLeafTris = 8;
constexpr int kTraversalStack = 32;   // LDS stack entries per lane; builder caps depth to fit.

__attribute__((always_inline)) inline int32_t encode_leaf(uint32_t first, uint32_t count) {
    return ~static_cast<int32_t>((first << 3) | (count - 1u));
}

// Compressed 8-wide node, 80 B (five 16-B words), after Ylitie et al. 2017 ("Efficient incoherent
// ray traversal on GPUs through compressed wide BVHs"): child boxes quantised to 8 bits against the
// node's origin p and per-axis power-of-two scales 2^(e-127).
//   w0 = (p.x, p.y, p.z, e.x | e.y<<8 | e.z<<16 | imask<<24)     imask bit s = slot s is internal
//   w1 = (base_child, base_tri, meta[0..3], meta[4..7])
//   w2..w4 = qlo_x[8], qlo_y[8], qlo_z[8], qhi_x[8], qhi_y[8], qhi_z[8]
// meta[s]: 0 = empty; 0x80 | s = internal child (stored at base_child + popcount(imask below s));
//          (count << 5) | offset = leaf with count (1..3) triangles at base_tri + offset (offset < 24).
// Slots are assigned so that visiting keys (slot ^ octant(ray)) from high to low is roughly
// front-to-back: slot s is the nearest child for rays whose octant is 7 ^ s.
struct Bvh8Node {
    float p[3];
    uint8_t e[3];
    uint8_t imask;
    uint32_t base_child;
    uint32_t base_tri;
    uint8_t meta[8];
    uint8_t qlo[3][8];
    uint8_t qhi[3][8];
};
static_assert(sizeof(Bvh8Node) == 80, "Bvh8Node must be 80 B");
// Device stride of a node: 80 (packed) or 128 (one node per 128-B cache line, 48 B of padding; the
// A/B of DESIGN.md §7).  The builder's array is always packed; the upload pads.
#ifndef DXRPT_NODE_STRIDE
#define DXRPT_NODE_STRIDE 80
#endif
constexpr uint32_t kNode8Stride = DXRPT_NODE_STRIDE;
constexpr uint32_t kNode8Words = kNode8Stride / 16u;  // 16-B words
static_assert(kNode8Stride == 80u || kNode8Stride == 128u, "node stride 80 or 128");

constexpr int kMaxLeafTris8 = 3;
constexpr int kTraversalStack8 = 16;  // group-stack entries per lane; the builder caps BVH8 depth to fit.
constexpr int kStackLds8 = 6;         // of which the first entries live in LDS, the rest in a global slab
                                      // (traversals deeper than 6 pending groups are rare: see DESIGN.md)
constexpr uint8_t kMetaInternal = 0x80;

// Leaf triangle record, 48 B.
//   p0 = (v0.x, v0.y, v0.z, bits(gtri))      gtri = global triangle id = IdxOffset/3 + PrimitiveIndex
//   p1 = (e1.x, e1.y, e1.z, bits(geometry))  geometry = GeometryIndex()
//   p2 = (e2.x, e2.y, e2.z, bits(flags))     flags bit0 = opaque geometry; on alpha-tested geometry
//                                            bits 1..31 = the triangle's opacity micromap slot
struct TriRecord {
    float p0[4];
    float p1[4];
    float p2[4];
};
static_assert(sizeof(TriRecord) == 48, "TriRecord must be 48 B");

constexpr uint32_t kTriOpaque = 1u;

// Texture descriptor, 16 B.  Texels live in one pool of 32-bit words starting at `offset`, in
// 128-B tiles (one L2 line) laid out row-major by tile; width and height are padded up to whole tiles
// (padding texels are never sampled: coordinates wrap at the true size).
//   fmt DXRPT_TEX_RGBA8_*: one word per texel (r | g<<8 | b<<16 | a<<24), 8 x 4 texels per tile
//   fmt DXRPT_TEX_R8_UNORM: four texels per word (x & 3 selects the byte), 16 x 8 texels per tile
struct TexDesc {
    uint32_t offset;
    uint32_t width;
    uint32_t height;
    uint32_t fmt;
    bool inl = false;  // device view of an inlined 1 x 1 map (GeoTex whf width = height = 0): offset = its texel word
};

// Packed material taps (DXRPT_OPT_PACKED_TAPS): a material whose normal map (RGBA8 unorm) and metallic and
// roughness maps (R8 or RGBA8 unorm, .r read) have one size gets a host-built RGBA8 unorm texture
// (normal.r, normal.g, metallic, roughness), referenced from GeoShade::normal with this format tag: one
// bilinear tap instead of three, the same texels, weights and decode (unorm) for every channel.
constexpr uint32_t kTexFmtPackedNMR = 3u;

// A texture reference packed into 8 B: `offset` as in TexDesc, whf = width | height << 15 | fmt << 30
// (width, height <= 32767); whf == 0: no texture.
// An inlined 1 x 1 map (DXRPT_OPT_PACKED_TAPS bit 1, not for opacity): whf's width and height are 0 and
// `offset` is the map's texel word (the pool word: RGBA8, or R8 in byte 0), so its tap reads no memory.
struct GeoTex {
    uint32_t offset;
    uint32_t whf;
};

// Per-geometry shading record, 48 B (three 16-B words): the geometry's material textures resolved
// (GeometryInfo.MaterialIdx -> Material -> texture descriptors, RayTrace.hlsl:467-474, 497), so a hit
// reaches its texels in two dependent loads (this record, then the texels) instead of four.
struct GeoShade {
    GeoTex albedo, normal, roughness, metallic, emissive, opacity;  // opacity.whf == 0: opaque
};
static_assert(sizeof(GeoShade) == 48, "GeoShade must be 48 B");

constexpr uint32_t kTexTileWords = 32;  // 128 B
constexpr uint32_t kTexTileW32 = 8, kTexTileH32 = 4;
constexpr uint32_t kTexTileW8 = 16, kTexTileH8 = 8;

// Opacity micromap (DXRPT_OPT_OPACITY_MICROMAP, built by omm.cpp): kOmmWords 32-bit words per triangle
// of alpha-tested geometry, at slot (TriRecord flags >> 1) -- a candidate reads the one word holding its
// cell, issued with the UV and descriptor loads of its tap.  The triangle's barycentric domain is cut
// into kOmmSplit x kOmmSplit square cells (b1, b2) of which kOmmCells touch the triangle; cell c holds
// 2 bits at bit 2(c & 15) of word c >> 4: kOmmOpaque / kOmmTransparent when AnyHitShader's opacity tap
// (RayTrace.hlsl:485-507: bilinear, wrap, mip 0, `.x < 0.35` rejects) has the same verdict at every
// point of the cell, kOmmUnknown otherwise (the tap decides).  A verdict is an exact shortcut of the tap,
// never an approximation: the builder checks every texel any point of the cell can filter.
constexpr uint32_t kOmmSplit = 32;  // include/dxrpt.h DXRPT_OMM_SPLIT
constexpr uint32_t kOmmCells = kOmmSplit * (kOmmSplit + 1u) / 2u;  // 528
constexpr uint32_t kOmmWords = (2u * kOmmCells + 31u) / 32u;        // 33 words = 132 B per triangle
constexpr uint32_t kOmmUnknown = 0u, kOmmOpaque = 1u, kOmmTransparent = 2u;

// The cell of barycentrics (b1, b2), b1, b2 >= 0, b1 + b2 <= 1 (the triangle test guarantees it up to
// rounding): row i = floor(b1 * kOmmSplit), column j = floor(b2 * kOmmSplit), clamped into the triangle;
// rows are stored one after another (row i holds kOmmSplit - i cells).
#if defined(__HIPCC__)
__host__ __device__
#endif
inline uint32_t omm_cell(float b1, float b2) {
    uint32_t i = uint32_t(b1 * float(kOmmSplit)), j = uint32_t(b2 * float(kOmmSplit));
    i = i < kOmmSplit - 1u ? i : kOmmSplit - 1u;
    j = j < kOmmSplit - 1u - i ? j : kOmmSplit - 1u - i;
    return i * (2u * kOmmSplit + 1u - i) / 2u + j;
}



}  // namespace dxrpt
