// dds.cpp — DDS texture files, mip 0 (the path tracer samples LOD 0 only: RayTrace.hlsl:467-474).
//
// The reference decodes textures with DirectXTex (July 2017, prebuilt, Graphics/Textures.cpp:38-172;
// its source is not vendored): DDS files are uploaded in their stored DXGI format and filtered by the
// GPU sampler.  Restated here for the formats the reference's content uses:
//   * uncompressed 32-bit RGB(A) with channel masks (Content/Textures/Default*.dds: B8G8R8X8, the
//     X channel reads as alpha 1) and 8-bit luminance/alpha;
//   * BC1 (DXT1), BC3 (DXT5), BC4 (BC4U/ATI1: the SunTemple opacity maps), BC5 (BC5U/ATI2), decoded to
//     RGBA8 / R8 with the D3D block-decompression rules (BC1 3-colour mode when c0 <= c1; BC4/BC5
//     8-value mode when r0 > r1, else 6 values + 0 and 255; interpolants rounded as integers, the
//     unorm formula of the D3D functional spec up to its rounding, which is parity-unpinned).
// Legacy headers and the DX10 extension header are both read.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "scene_builder.h"

namespace dxrpt_host {

namespace {

uint32_t rd32(const uint8_t* p) { return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24; }

uint32_t fourcc(const char* s) { return uint32_t(uint8_t(s[0])) | uint32_t(uint8_t(s[1])) << 8 | uint32_t(uint8_t(s[2])) << 16 | uint32_t(uint8_t(s[3])) << 24; }

// value of a masked channel scaled to 8 bits (mask 0 -> `def`)
uint8_t channel(uint32_t px, uint32_t mask, uint8_t def) {
    if (!mask) return def;
    int shift = 0;
    while (!((mask >> shift) & 1u)) ++shift;
    const uint32_t m = mask >> shift;
    const uint32_t v = (px >> shift) & m;
    return uint8_t((v * 255u + m / 2u) / m);
}

void rgb565(uint16_t c, int& r, int& g, int& b) {
    r = ((c >> 11) & 31) * 255 / 31;
    g = ((c >> 5) & 63) * 255 / 63;
    b = (c & 31) * 255 / 31;
}

// BC1 colour block -> 16 RGBA texels (alpha from the 3-colour mode's transparent index unless `opaque`)
void bc1_block(const uint8_t* b, uint8_t out[16][4], bool opaque4) {
    const uint16_t c0 = uint16_t(b[0] | b[1] << 8), c1 = uint16_t(b[2] | b[3] << 8);
    int pal[4][4];
    rgb565(c0, pal[0][0], pal[0][1], pal[0][2]);
    rgb565(c1, pal[1][0], pal[1][1], pal[1][2]);
    pal[0][3] = pal[1][3] = 255;
    if (c0 > c1 || opaque4) {
        for (int k = 0; k < 3; ++k) {
            pal[2][k] = (2 * pal[0][k] + pal[1][k] + 1) / 3;
            pal[3][k] = (pal[0][k] + 2 * pal[1][k] + 1) / 3;
        }
        pal[2][3] = pal[3][3] = 255;
    } else {
        for (int k = 0; k < 3; ++k) {
            pal[2][k] = (pal[0][k] + pal[1][k]) / 2;
            pal[3][k] = 0;
        }
        pal[2][3] = 255;
        pal[3][3] = 0;
    }
    const uint32_t idx = rd32(b + 4);
    for (int i = 0; i < 16; ++i) {
        const int s = (idx >> (2 * i)) & 3;
        for (int k = 0; k < 4; ++k) out[i][k] = uint8_t(pal[s][k]);
    }
}

// BC4 (BC3 alpha) block -> 16 unorm8 values
void bc4_block(const uint8_t* b, uint8_t out[16]) {
    const int r0 = b[0], r1 = b[1];
    int pal[8];
    pal[0] = r0;
    pal[1] = r1;
    if (r0 > r1) {
        for (int i = 1; i < 7; ++i) pal[i + 1] = ((7 - i) * r0 + i * r1 + 3) / 7;
    } else {
        for (int i = 1; i < 5; ++i) pal[i + 1] = ((5 - i) * r0 + i * r1 + 2) / 5;
        pal[6] = 0;
        pal[7] = 255;
    }
    uint64_t bits = 0;
    for (int i = 0; i < 6; ++i) bits |= uint64_t(b[2 + i]) << (8 * i);
    for (int i = 0; i < 16; ++i) out[i] = uint8_t(pal[(bits >> (3 * i)) & 7u]);
}

}  // namespace

bool load_dds(const std::string& path, bool srgb, Texture& tex, std::string& err) {
    std::ifstream f(path, std::ios::binary);
    if (!f) {
        err = "cannot open " + path;
        return false;
    }
    std::vector<uint8_t> d((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (d.size() < 128 || rd32(d.data()) != fourcc("DDS ")) {
        err = path + ": not a DDS file";
        return false;
    }
    const uint8_t* h = d.data() + 4;
    const uint32_t height = rd32(h + 8), width = rd32(h + 12);
    const uint8_t* pf = h + 72;  // DDS_PIXELFORMAT
    const uint32_t pf_flags = rd32(pf + 4), cc = rd32(pf + 8), bits = rd32(pf + 12);
    const uint32_t rm = rd32(pf + 16), gm = rd32(pf + 20), bm = rd32(pf + 24), am = rd32(pf + 28);
    size_t off = 128;
    enum { UNC, BC1, BC3, BC4, BC5 } kind = UNC;
    if (pf_flags & 0x4u) {  // DDPF_FOURCC
        uint32_t dxgi = 0;
        if (cc == fourcc("DX10")) {
            if (d.size() < 148) { err = path + ": truncated DX10 header"; return false; }
            dxgi = rd32(d.data() + 128);
            off = 148;
        }
        if (cc == fourcc("DXT1") || dxgi == 71 || dxgi == 72) kind = BC1;
        else if (cc == fourcc("DXT5") || dxgi == 77 || dxgi == 78) kind = BC3;
        else if (cc == fourcc("BC4U") || cc == fourcc("ATI1") || dxgi == 80) kind = BC4;
        else if (cc == fourcc("BC5U") || cc == fourcc("ATI2") || dxgi == 83) kind = BC5;
        else if (dxgi == 28 || dxgi == 29 || dxgi == 87 || dxgi == 88 || dxgi == 91 || dxgi == 93)
            kind = UNC;  // R8G8B8A8 / B8G8R8A8 / B8G8R8X8 (_SRGB): masks synthesised below
        else {
            err = path + ": unsupported DDS format (fourcc/DXGI)";
            return false;
        }
    }
    tex.w = width;
    tex.h = height;
    if (kind == UNC) {
        uint32_t r_m = rm, g_m = gm, b_m = bm, a_m = am, bpp = bits;
        if (pf_flags & 0x4u) {  // DX10 uncompressed
            const uint32_t dxgi = rd32(d.data() + 128);
            const bool bgra = !(dxgi == 28 || dxgi == 29);
            r_m = bgra ? 0x00FF0000u : 0x000000FFu;
            g_m = 0x0000FF00u;
            b_m = bgra ? 0x000000FFu : 0x00FF0000u;
            a_m = (dxgi == 88 || dxgi == 93) ? 0u : 0xFF000000u;
            bpp = 32;
        } else if (!(pf_flags & 0x40u) && !(pf_flags & 0x20000u) && !(pf_flags & 0x2u)) {
            err = path + ": unsupported DDS pixel format";
            return false;
        }
        if (bpp != 32 && bpp != 8) {
            err = path + ": unsupported bit count";
            return false;
        }
        const size_t bytes = size_t(width) * height * (bpp / 8);
        if (d.size() < off + bytes) { err = path + ": truncated"; return false; }
        if (bpp == 8) {  // L8 / A8 -> R8
            tex.fmt = DXRPT_TEX_R8_UNORM;
            tex.data.assign(d.begin() + off, d.begin() + off + bytes);
            return true;
        }
        tex.fmt = srgb ? DXRPT_TEX_RGBA8_SRGB : DXRPT_TEX_RGBA8_UNORM;
        tex.data.resize(size_t(width) * height * 4);
        for (size_t i = 0; i < size_t(width) * height; ++i) {
            const uint32_t px = rd32(d.data() + off + 4 * i);
            tex.data[4 * i + 0] = channel(px, r_m, 0);
            tex.data[4 * i + 1] = channel(px, g_m, 0);
            tex.data[4 * i + 2] = channel(px, b_m, 0);
            tex.data[4 * i + 3] = channel(px, a_m, 255);  // X8 / no alpha: alpha 1
        }
        return true;
    }
    const uint32_t bw = (width + 3) / 4, bh = (height + 3) / 4;
    const size_t block = (kind == BC1 || kind == BC4) ? 8 : 16;
    if (d.size() < off + size_t(bw) * bh * block) { err = path + ": truncated"; return false; }
    const bool r8 = kind == BC4;
    tex.fmt = r8 ? DXRPT_TEX_R8_UNORM : (srgb ? DXRPT_TEX_RGBA8_SRGB : DXRPT_TEX_RGBA8_UNORM);
    tex.data.assign(size_t(width) * height * (r8 ? 1 : 4), 0);
    for (uint32_t by = 0; by < bh; ++by)
        for (uint32_t bx = 0; bx < bw; ++bx) {
            const uint8_t* b = d.data() + off + (size_t(by) * bw + bx) * block;
            uint8_t px[16][4];
            if (kind == BC1) {
                bc1_block(b, px, false);
            } else if (kind == BC3) {
                uint8_t a[16];
                bc4_block(b, a);
                bc1_block(b + 8, px, true);
                for (int i = 0; i < 16; ++i) px[i][3] = a[i];
            } else if (kind == BC4) {
                uint8_t r[16];
                bc4_block(b, r);
                for (int i = 0; i < 16; ++i) px[i][0] = r[i];
            } else {  // BC5: red, green; blue 0, alpha 1
                uint8_t r[16], g[16];
                bc4_block(b, r);
                bc4_block(b + 8, g);
                for (int i = 0; i < 16; ++i) {
                    px[i][0] = r[i];
                    px[i][1] = g[i];
                    px[i][2] = 0;
                    px[i][3] = 255;
                }
            }
            for (int i = 0; i < 16; ++i) {
                const uint32_t x = bx * 4 + uint32_t(i & 3), y = by * 4 + uint32_t(i >> 2);
                if (x >= width || y >= height) continue;
                const size_t t = size_t(y) * width + x;
                if (r8) tex.data[t] = px[i][0];
                else std::memcpy(&tex.data[4 * t], px[i], 4);
            }
        }
    return true;
}

}  // namespace dxrpt_host
