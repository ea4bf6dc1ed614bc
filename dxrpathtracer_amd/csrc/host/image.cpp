// image.cpp — PNG and baseline-JPEG decoding for scene ingest, plus the by-format dispatcher.
//
// The reference loads every non-DDS texture through WIC (Graphics/Textures.cpp:38-172: LoadFromWICFile
// into R8G8B8A8, _SRGB when forceSRGB, then GenerateMipMaps).  WIC is a Windows component, so its
// decoders are restated here from the format specifications:
//   PNG  (ISO/IEC 15948): IHDR/PLTE/tRNS/IDAT/IEND, zlib inflate (the image's libz), the five scanline
//        filters, Adam7 interlacing, bit depths 1/2/4/8/16 of all five colour types -> RGBA8.
//        Lossless, so the texels are exactly the file's (16-bit samples keep their high byte).
//   JPEG (ITU-T T.81): baseline and extended sequential Huffman DCT (SOF0/SOF1), 8-bit samples, 1 or 3
//        components, any sampling factors up to 4x4, restart intervals, JFIF YCbCr -> RGB.  Chroma
//        upsampling and the colour conversion follow libjpeg (triangle "fancy" upsampling for 2:1,
//        16-bit fixed-point YCbCr); the inverse DCT is an exact float IDCT rounded once, so texels
//        agree with libjpeg's integer IDCT to +-3.  WIC's decoder is not specified, so JPEG texels
//        are parity-unpinned against the reference (the path tracer samples whatever texels it is
//        given, so GPU-vs-oracle parity is unaffected).
// Progressive/arithmetic JPEG, 12-bit JPEG and PNG gamma/colour-profile chunks are rejected or ignored.
#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <iterator>

#include "scene_builder.h"

namespace dxrpt_host {

namespace {

bool read_all(const std::string& path, std::vector<uint8_t>& d, std::string& err) {
    std::ifstream f(path, std::ios::binary);
    if (!f) {
        err = "cannot open " + path;
        return false;
    }
    d.assign((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    return true;
}

uint32_t be32(const uint8_t* p) { return uint32_t(p[0]) << 24 | uint32_t(p[1]) << 16 | uint32_t(p[2]) << 8 | p[3]; }
uint16_t be16(const uint8_t* p) { return uint16_t(uint16_t(p[0]) << 8 | p[1]); }

// ---- PNG ---------------------------------------------------------------------------------------------
uint8_t paeth(int a, int b, int c) {
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    return uint8_t(pa <= pb && pa <= pc ? a : (pb <= pc ? b : c));
}

// Reverses the scanline filters of one (sub)image in place: rows of 1 + stride bytes.
bool unfilter(uint8_t* data, uint32_t rows, size_t stride, uint32_t bpp, std::vector<uint8_t>& out) {
    out.assign(size_t(rows) * stride, 0);
    for (uint32_t y = 0; y < rows; ++y) {
        const uint8_t ft = data[size_t(y) * (stride + 1)];
        const uint8_t* in = data + size_t(y) * (stride + 1) + 1;
        uint8_t* cur = out.data() + size_t(y) * stride;
        const uint8_t* prev = y ? cur - stride : nullptr;
        for (size_t i = 0; i < stride; ++i) {
            const int a = i >= bpp ? cur[i - bpp] : 0, b = prev ? prev[i] : 0, c = (prev && i >= bpp) ? prev[i - bpp] : 0;
            int v = in[i];
            switch (ft) {
                case 0: break;
                case 1: v += a; break;
                case 2: v += b; break;
                case 3: v += (a + b) >> 1; break;
                case 4: v += paeth(a, b, c); break;
                default: return false;
            }
            cur[i] = uint8_t(v);
        }
    }
    return true;
}

bool load_png_mem(const std::vector<uint8_t>& d, const std::string& path, Texture& tex, std::string& err) {
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
    if (d.size() < 33 || std::memcmp(d.data(), sig, 8) != 0) {
        err = path + ": not a PNG file";
        return false;
    }
    uint32_t w = 0, h = 0, depth = 0, ctype = 0, interlace = 0;
    std::vector<uint8_t> idat, plte, trns;
    size_t p = 8;
    bool seen_ihdr = false, seen_iend = false;
    while (p + 12 <= d.size()) {
        const uint32_t len = be32(&d[p]);
        if (p + 12 + size_t(len) > d.size()) break;
        const char* type = reinterpret_cast<const char*>(&d[p + 4]);
        const uint8_t* body = &d[p + 8];
        if (std::memcmp(type, "IHDR", 4) == 0 && len >= 13) {
            w = be32(body);
            h = be32(body + 4);
            depth = body[8];
            ctype = body[9];
            interlace = body[12];
            if (body[10] != 0 || body[11] != 0) {
                err = path + ": unknown PNG compression/filter method";
                return false;
            }
            seen_ihdr = true;
        } else if (std::memcmp(type, "PLTE", 4) == 0) {
            plte.assign(body, body + len);
        } else if (std::memcmp(type, "tRNS", 4) == 0) {
            trns.assign(body, body + len);
        } else if (std::memcmp(type, "IDAT", 4) == 0) {
            idat.insert(idat.end(), body, body + len);
        } else if (std::memcmp(type, "IEND", 4) == 0) {
            seen_iend = true;
            break;
        }
        p += 12 + size_t(len);
    }
    const int channels[7] = {1, 0, 3, 1, 2, 0, 4};
    if (!seen_ihdr || !seen_iend || idat.empty() || w == 0 || h == 0 || w > 16384 || h > 16384 || ctype > 6 ||
        channels[ctype] == 0 || interlace > 1) {
        err = path + ": malformed or unsupported PNG";
        return false;
    }
    const bool depth_ok = (ctype == 0 && (depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16)) ||
                          (ctype == 3 && (depth == 1 || depth == 2 || depth == 4 || depth == 8)) ||
                          ((ctype == 2 || ctype == 4 || ctype == 6) && (depth == 8 || depth == 16));
    if (!depth_ok || (ctype == 3 && plte.empty())) {
        err = path + ": invalid PNG bit depth / palette";
        return false;
    }
    const uint32_t nc = uint32_t(channels[ctype]);
    const uint32_t bits_px = nc * depth, bpp = std::max(1u, bits_px / 8);
    // Adam7 passes (x0, y0, dx, dy); one pass covering everything when not interlaced
    static const uint32_t adam7[7][4] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4}, {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};
    const uint32_t npass = interlace ? 7u : 1u;
    size_t raw_size = 0;
    for (uint32_t k = 0; k < npass; ++k) {
        const uint32_t x0 = interlace ? adam7[k][0] : 0, y0 = interlace ? adam7[k][1] : 0;
        const uint32_t dx = interlace ? adam7[k][2] : 1, dy = interlace ? adam7[k][3] : 1;
        const uint32_t pw = w > x0 ? (w - x0 + dx - 1) / dx : 0, ph = h > y0 ? (h - y0 + dy - 1) / dy : 0;
        if (pw && ph) raw_size += size_t(ph) * (1 + (size_t(pw) * bits_px + 7) / 8);
    }
    std::vector<uint8_t> raw(raw_size);
    uLongf got = uLongf(raw_size);
    if (uncompress(raw.data(), &got, idat.data(), uLong(idat.size())) != Z_OK || got != raw_size) {
        err = path + ": corrupt PNG image data (inflate)";
        return false;
    }
    tex.w = w;
    tex.h = h;
    tex.data.assign(size_t(w) * h * 4, 0);
    size_t off = 0;
    std::vector<uint8_t> rows;
    for (uint32_t k = 0; k < npass; ++k) {
        const uint32_t x0 = interlace ? adam7[k][0] : 0, y0 = interlace ? adam7[k][1] : 0;
        const uint32_t dx = interlace ? adam7[k][2] : 1, dy = interlace ? adam7[k][3] : 1;
        const uint32_t pw = w > x0 ? (w - x0 + dx - 1) / dx : 0, ph = h > y0 ? (h - y0 + dy - 1) / dy : 0;
        if (!pw || !ph) continue;
        const size_t stride = (size_t(pw) * bits_px + 7) / 8;
        if (!unfilter(raw.data() + off, ph, stride, bpp, rows)) {
            err = path + ": bad PNG filter type";
            return false;
        }
        off += size_t(ph) * (stride + 1);
        for (uint32_t y = 0; y < ph; ++y) {
            const uint8_t* r = rows.data() + size_t(y) * stride;
            for (uint32_t x = 0; x < pw; ++x) {
                uint32_t s[4] = {0, 0, 0, 0};  // samples at the file's depth
                for (uint32_t c = 0; c < nc; ++c) {
                    if (depth == 8) s[c] = r[size_t(x) * nc + c];
                    else if (depth == 16) s[c] = be16(r + (size_t(x) * nc + c) * 2);
                    else {  // 1/2/4-bit grey or palette: packed MSB first
                        const size_t bit = size_t(x) * depth;
                        s[c] = (r[bit >> 3] >> (8 - depth - (bit & 7))) & ((1u << depth) - 1u);
                    }
                }
                uint8_t* o = &tex.data[(size_t(y0 + y * dy) * w + x0 + x * dx) * 4];
                auto to8 = [&](uint32_t v) -> uint8_t {
                    if (depth == 16) return uint8_t(v >> 8);
                    if (depth == 8) return uint8_t(v);
                    return uint8_t(v * 255u / ((1u << depth) - 1u));
                };
                uint8_t a = 255;
                if (ctype == 3) {
                    const uint32_t i = s[0];
                    if (size_t(i) * 3 + 2 < plte.size()) {
                        o[0] = plte[i * 3];
                        o[1] = plte[i * 3 + 1];
                        o[2] = plte[i * 3 + 2];
                    }
                    if (i < trns.size()) a = trns[i];
                } else if (ctype == 0 || ctype == 4) {
                    o[0] = o[1] = o[2] = to8(s[0]);
                    if (ctype == 4) a = to8(s[1]);
                    else if (trns.size() >= 2 && s[0] == be16(trns.data())) a = 0;
                } else {
                    o[0] = to8(s[0]);
                    o[1] = to8(s[1]);
                    o[2] = to8(s[2]);
                    if (ctype == 6) a = to8(s[3]);
                    else if (trns.size() >= 6 && s[0] == be16(&trns[0]) && s[1] == be16(&trns[2]) && s[2] == be16(&trns[4])) a = 0;
                }
                o[3] = a;
            }
        }
    }
    return true;
}

// ---- JPEG (baseline / extended sequential Huffman) --------------------------------------------------
const uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                             41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                             30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Huffman {
    // canonical codes: for each length L, codes [mincode[L], maxcode[L]] map to values from valptr[L]
    int32_t mincode[17] = {}, maxcode[17] = {}, valptr[17] = {};
    uint8_t vals[256] = {};
    bool defined = false;
};

struct Component {
    uint32_t id = 0, h = 1, v = 1, tq = 0, td = 0, ta = 0;
    int32_t pred = 0;
    uint32_t bw = 0, bh = 0;          // blocks per line / column of this component (padded to MCUs)
    std::vector<uint8_t> pixels;      // bw*8 x bh*8 decoded samples
};

struct BitReader {
    const uint8_t* d;
    size_t n, p;
    uint32_t acc = 0;
    int bits = 0;
    bool marker = false;  // hit a marker: feed zeros
    int32_t get(int k) {
        while (bits < k) {
            uint32_t byte = 0;
            if (!marker && p < n) {
                byte = d[p];
                if (byte == 0xFF) {
                    const uint8_t nx = p + 1 < n ? d[p + 1] : 0;
                    if (nx == 0x00) p += 2;
                    else { marker = true; byte = 0; }
                } else {
                    ++p;
                }
            }
            acc = (acc << 8) | byte;
            bits += 8;
        }
        const int32_t v = int32_t((acc >> (bits - k)) & ((1u << k) - 1u));
        bits -= k;
        return v;
    }
    void reset() {  // byte-align after a restart marker
        acc = 0;
        bits = 0;
        marker = false;
    }
};

int decode_huff(BitReader& br, const Huffman& h) {
    int32_t code = 0;
    for (int L = 1; L <= 16; ++L) {
        code = (code << 1) | br.get(1);
        if (h.maxcode[L] >= 0 && code <= h.maxcode[L] && code >= h.mincode[L]) return h.vals[h.valptr[L] + code - h.mincode[L]];
    }
    return -1;
}

int32_t extend(int32_t v, int t) { return t == 0 ? 0 : (v < (1 << (t - 1)) ? v - (1 << t) + 1 : v); }

// Separable float inverse DCT of one block (coefficients in natural order, dequantised), level shift,
// rounding to nearest and clamping to [0, 255].
void idct8x8(const float in[64], uint8_t* out, size_t stride) {
    static float cosv[8][8];
    static bool init = false;
    if (!init) {
        for (int x = 0; x < 8; ++x)
            for (int u = 0; u < 8; ++u)
                cosv[x][u] = float((u == 0 ? std::sqrt(0.125) : 0.5) * std::cos((2.0 * x + 1.0) * u * 3.14159265358979323846 / 16.0));
        init = true;
    }
    float tmp[64];
    for (int y = 0; y < 8; ++y)
        for (int u = 0; u < 8; ++u) {  // rows: along v
            float s = 0.0f;
            for (int v = 0; v < 8; ++v) s += cosv[y][v] * in[v * 8 + u];
            tmp[y * 8 + u] = s;
        }
    for (int y = 0; y < 8; ++y)
        for (int x = 0; x < 8; ++x) {
            float s = 0.0f;
            for (int u = 0; u < 8; ++u) s += cosv[x][u] * tmp[y * 8 + u];
            const float v = std::nearbyint(s + 128.0f);
            out[size_t(y) * stride + x] = uint8_t(std::min(255.0f, std::max(0.0f, v)));
        }
}

bool load_jpeg_mem(const std::vector<uint8_t>& d, const std::string& path, Texture& tex, std::string& err) {
    if (d.size() < 4 || d[0] != 0xFF || d[1] != 0xD8) {
        err = path + ": not a JPEG file";
        return false;
    }
    uint16_t qt[4][64] = {};
    Huffman hdc[4], hac[4];
    std::vector<Component> comps;
    uint32_t width = 0, height = 0, restart = 0;
    bool frame = false, done = false;
    size_t p = 2;
    auto fail = [&](const std::string& m) {
        err = path + ": " + m;
        return false;
    };
    while (p + 4 <= d.size() && !done) {
        if (d[p] != 0xFF) return fail("bad JPEG marker");
        const uint8_t m = d[p + 1];
        if (m == 0xFF) { ++p; continue; }
        if (m == 0xD8 || m == 0x01 || (m >= 0xD0 && m <= 0xD7)) { p += 2; continue; }
        if (m == 0xD9) break;
        const uint32_t len = be16(&d[p + 2]);
        if (len < 2 || p + 2 + len > d.size()) return fail("truncated JPEG segment");
        const uint8_t* s = &d[p + 4];
        const uint32_t n = len - 2;
        if (m == 0xDB) {  // DQT
            for (uint32_t q = 0; q < n;) {
                const uint32_t pq = s[q] >> 4, tq = s[q] & 15u;
                if (pq > 1 || tq > 3) return fail("bad quantisation table id / precision");
                if (q + 1 + 64 * (pq + 1) > n) return fail("truncated quantisation table");
                ++q;
                for (int k = 0; k < 64; ++k) {
                    qt[tq][kZigzag[k]] = pq ? be16(s + q + 2 * k) : s[q + k];
                }
                q += pq ? 128 : 64;
            }
        } else if (m == 0xC4) {  // DHT
            for (uint32_t q = 0; q + 17 <= n;) {
                const uint32_t tc = s[q] >> 4, th = s[q] & 15u;
                if (tc > 1 || th > 3) return fail("bad Huffman table class / id");
                Huffman& H = tc ? hac[th] : hdc[th];
                uint32_t total = 0;
                for (int L = 1; L <= 16; ++L) total += s[q + L];
                if (total > 256 || q + 17 + total > n) return fail("bad Huffman table");
                std::memcpy(H.vals, s + q + 17, total);
                int32_t code = 0, k = 0;
                for (int L = 1; L <= 16; ++L) {
                    const int cnt = s[q + L];
                    H.valptr[L] = k;
                    H.mincode[L] = code;
                    code += cnt;
                    k += cnt;
                    H.maxcode[L] = cnt ? code - 1 : -1;
                    code <<= 1;
                }
                H.defined = true;
                q += 17 + total;
            }
        } else if (m == 0xDD) {  // DRI
            if (n < 2) return fail("truncated restart interval");
            restart = be16(s);
        } else if (m == 0xC0 || m == 0xC1) {  // SOF0 / SOF1
            if (n < 6) return fail("truncated frame header");
            if (s[0] != 8) return fail("only 8-bit JPEG samples are supported");
            height = be16(s + 1);
            width = be16(s + 3);
            const uint32_t nc = s[5];
            if ((nc != 1 && nc != 3) || width == 0 || height == 0 || width > 16384 || height > 16384)
                return fail("unsupported JPEG frame (components / size)");
            if (n < 6 + 3 * nc) return fail("truncated frame header");
            comps.resize(nc);
            for (uint32_t c = 0; c < nc; ++c) {
                comps[c].id = s[6 + 3 * c];
                comps[c].h = s[7 + 3 * c] >> 4;
                comps[c].v = s[7 + 3 * c] & 15u;
                comps[c].tq = s[8 + 3 * c];
                if (comps[c].tq > 3) return fail("bad quantisation table id");
                if (comps[c].h < 1 || comps[c].h > 4 || comps[c].v < 1 || comps[c].v > 4) return fail("bad sampling factors");
            }
            frame = true;
        } else if ((m >= 0xC2 && m <= 0xCF) && m != 0xC4 && m != 0xC8 && m != 0xCC) {
            return fail("progressive / lossless / arithmetic JPEG is not supported");
        } else if (m == 0xDA) {  // SOS: one interleaved scan with every component (baseline)
            if (!frame) return fail("scan before frame header");
            if (n < 1) return fail("truncated scan header");
            const uint32_t ns = s[0];
            if (ns != comps.size()) return fail("non-interleaved sequential scans are not supported");
            if (n < 1 + 2 * ns + 3) return fail("truncated scan header");
            for (uint32_t k = 0; k < ns; ++k) {
                const uint32_t cid = s[1 + 2 * k];
                auto it = std::find_if(comps.begin(), comps.end(), [&](const Component& c) { return c.id == cid; });
                if (it == comps.end()) return fail("scan names an unknown component");
                it->td = s[2 + 2 * k] >> 4;
                it->ta = s[2 + 2 * k] & 15u;
                if (it->td > 3 || it->ta > 3) return fail("bad Huffman table id in scan");
                if (!hdc[it->td].defined || !hac[it->ta].defined) return fail("scan uses an undefined Huffman table");
            }
            uint32_t hmax = 1, vmax = 1;
            for (const Component& c : comps) {
                hmax = std::max(hmax, c.h);
                vmax = std::max(vmax, c.v);
            }
            if (comps.size() == 1) hmax = vmax = comps[0].h = comps[0].v = 1;  // single component: no interleave
            const uint32_t mcux = (width + 8 * hmax - 1) / (8 * hmax), mcuy = (height + 8 * vmax - 1) / (8 * vmax);
            for (Component& c : comps) {
                c.bw = mcux * c.h;
                c.bh = mcuy * c.v;
                c.pixels.assign(size_t(c.bw) * 8 * c.bh * 8, 0);
                c.pred = 0;
            }
            BitReader br{d.data(), d.size(), p + 2 + len};
            float coef[64];
            uint32_t mcus = 0;
            for (uint32_t my = 0; my < mcuy; ++my)
                for (uint32_t mx = 0; mx < mcux; ++mx) {
                    if (restart && mcus && mcus % restart == 0) {  // RSTn: byte-align, skip the marker
                        br.reset();
                        while (br.p + 1 < br.n && !(br.d[br.p] == 0xFF && br.d[br.p + 1] >= 0xD0 && br.d[br.p + 1] <= 0xD7)) ++br.p;
                        br.p += 2;
                        for (Component& c : comps) c.pred = 0;
                    }
                    ++mcus;
                    for (Component& c : comps)
                        for (uint32_t by = 0; by < c.v; ++by)
                            for (uint32_t bx = 0; bx < c.h; ++bx) {
                                int32_t blk[64] = {};
                                const int t = decode_huff(br, hdc[c.td]);
                                if (t < 0 || t > 11) return fail("corrupt JPEG data (DC)");
                                c.pred += extend(t ? br.get(t) : 0, t);
                                blk[0] = c.pred;
                                for (int k = 1; k < 64;) {
                                    const int rs = decode_huff(br, hac[c.ta]);
                                    if (rs < 0) return fail("corrupt JPEG data (AC)");
                                    const int r = rs >> 4, sz = rs & 15;
                                    if (sz == 0) {
                                        if (r != 15) break;  // EOB
                                        k += 16;
                                        continue;
                                    }
                                    k += r;
                                    if (k > 63) return fail("corrupt JPEG data (AC run)");
                                    blk[kZigzag[k]] = extend(br.get(sz), sz);
                                    ++k;
                                }
                                for (int k = 0; k < 64; ++k) coef[k] = float(blk[k] * int32_t(qt[c.tq][k]));
                                const size_t stride = size_t(c.bw) * 8;
                                const size_t x0 = (size_t(mx) * c.h + bx) * 8, y0 = (size_t(my) * c.v + by) * 8;
                                idct8x8(coef, c.pixels.data() + y0 * stride + x0, stride);
                            }
                }
            done = true;
            break;
        }
        p += 2 + len;
    }
    if (!done) return fail("no image scan");
    uint32_t hmax = 1, vmax = 1;
    for (const Component& c : comps) {
        hmax = std::max(hmax, c.h);
        vmax = std::max(vmax, c.v);
    }
    // every component at full resolution: libjpeg's "fancy" (triangle) upsampling for the 2:1 cases,
    // sample replication otherwise
    std::vector<std::vector<uint8_t>> full(comps.size());
    for (size_t c = 0; c < comps.size(); ++c) {
        const Component& C = comps[c];
        const uint32_t rh = hmax / C.h, rv = vmax / C.v;
        const uint32_t dw = (width * C.h + hmax - 1) / hmax, dh = (height * C.v + vmax - 1) / vmax;  // downsampled size
        const size_t stride = size_t(C.bw) * 8;
        auto in = [&](uint32_t x, uint32_t y) -> int { return C.pixels[size_t(std::min(y, dh - 1)) * stride + std::min(x, dw - 1)]; };
        std::vector<uint8_t>& F = full[c];
        F.resize(size_t(width) * height);
        for (uint32_t y = 0; y < height; ++y) {
            uint8_t* o = &F[size_t(y) * width];
            if ((rh == 2 || rh == 1) && (rv == 2 || rv == 1) && !(rh == 1 && rv == 1) && dw >= 2) {
                const uint32_t iy = y / rv;
                // vertical neighbour row (rv == 2): the row above for even output rows, below for odd
                const uint32_t ny = rv == 2 ? ((y & 1u) ? std::min(iy + 1, dh - 1) : (iy ? iy - 1 : 0)) : iy;
                for (uint32_t x = 0; x < width; ++x) {
                    const uint32_t ix = x / rh;
                    int v;
                    if (rv == 1) {  // h2v1 (jdsample.c h2v1_fancy_upsample)
                        const int cur = in(ix, iy);
                        if (x & 1u) v = ix + 1 < dw ? (cur * 3 + in(ix + 1, iy) + 2) >> 2 : cur;
                        else v = ix > 0 ? (cur * 3 + in(ix - 1, iy) + 1) >> 2 : cur;
                    } else if (rh == 1) {  // h1v2
                        v = (in(ix, iy) * 3 + in(ix, ny) + ((y & 1u) ? 2 : 1)) >> 2;
                    } else {  // h2v2 (h2v2_fancy_upsample): column sums 3 * near row + far row
                        const int cs = in(ix, iy) * 3 + in(ix, ny);
                        if (x & 1u) v = ix + 1 < dw ? (cs * 3 + (in(ix + 1, iy) * 3 + in(ix + 1, ny)) + 7) >> 4 : (cs * 4 + 7) >> 4;
                        else v = ix > 0 ? (cs * 3 + (in(ix - 1, iy) * 3 + in(ix - 1, ny)) + 8) >> 4 : (cs * 4 + 8) >> 4;
                    }
                    o[x] = uint8_t(v);
                }
            } else {
                for (uint32_t x = 0; x < width; ++x) o[x] = uint8_t(in(x * C.h / hmax, y * C.v / vmax));
            }
        }
    }
    tex.w = width;
    tex.h = height;
    tex.data.assign(size_t(width) * height * 4, 255);
    // JFIF YCbCr -> RGB in libjpeg's fixed point (jdcolor.c: 16 fraction bits, rounded tables)
    auto fix = [](double x) { return int32_t(x * 65536.0 + 0.5); };
    for (size_t i = 0; i < size_t(width) * height; ++i) {
        uint8_t* o = &tex.data[i * 4];
        if (comps.size() == 1) {
            o[0] = o[1] = o[2] = full[0][i];
            continue;
        }
        const int32_t Y = full[0][i], cb = int32_t(full[1][i]) - 128, cr = int32_t(full[2][i]) - 128;
        const int32_t r = Y + ((fix(1.40200) * cr + 32768) >> 16);
        const int32_t g = Y + ((-fix(0.34414) * cb + 32768 - fix(0.71414) * cr) >> 16);
        const int32_t b = Y + ((fix(1.77200) * cb + 32768) >> 16);
        o[0] = uint8_t(std::min(255, std::max(0, r)));
        o[1] = uint8_t(std::min(255, std::max(0, g)));
        o[2] = uint8_t(std::min(255, std::max(0, b)));
    }
    return true;
}

}  // namespace

bool load_png(const std::string& path, bool srgb, Texture& tex, std::string& err) {
    std::vector<uint8_t> d;
    if (!read_all(path, d, err) || !load_png_mem(d, path, tex, err)) return false;
    tex.fmt = srgb ? DXRPT_TEX_RGBA8_SRGB : DXRPT_TEX_RGBA8_UNORM;
    return true;
}

bool load_jpeg(const std::string& path, bool srgb, Texture& tex, std::string& err) {
    std::vector<uint8_t> d;
    if (!read_all(path, d, err) || !load_jpeg_mem(d, path, tex, err)) return false;
    tex.fmt = srgb ? DXRPT_TEX_RGBA8_SRGB : DXRPT_TEX_RGBA8_UNORM;
    return true;
}

bool load_r8z(const std::string& path, Texture& tex, std::string& err) {
    std::vector<uint8_t> d;
    if (!read_all(path, d, err)) return false;
    if (d.size() < 12 || std::memcmp(d.data(), "DXR8", 4) != 0) {
        err = path + ": not an R8 asset file";
        return false;
    }
    uint32_t w, h;
    std::memcpy(&w, &d[4], 4);
    std::memcpy(&h, &d[8], 4);
    if (w == 0 || h == 0 || w > 16384 || h > 16384) {
        err = path + ": bad R8 asset size";
        return false;
    }
    tex.w = w;
    tex.h = h;
    tex.fmt = DXRPT_TEX_R8_UNORM;
    tex.data.resize(size_t(w) * h);
    uLongf got = uLongf(tex.data.size());
    if (uncompress(tex.data.data(), &got, d.data() + 12, uLong(d.size() - 12)) != Z_OK || got != tex.data.size()) {
        err = path + ": corrupt R8 asset data";
        return false;
    }
    return true;
}

// LoadTexture (Graphics/Textures.cpp:38-172): DDS through the DDS loader, everything else through the
// image decoders (WIC in the reference), chosen by the file's signature.
bool load_image(const std::string& path, bool srgb, Texture& tex, std::string& err) {
    std::ifstream f(path, std::ios::binary);
    if (!f) {
        err = "cannot open " + path;
        return false;
    }
    uint8_t magic[8] = {};
    f.read(reinterpret_cast<char*>(magic), 8);
    if (std::memcmp(magic, "DDS ", 4) == 0) return load_dds(path, srgb, tex, err);
    if (magic[0] == 0x89 && magic[1] == 'P' && magic[2] == 'N' && magic[3] == 'G') return load_png(path, srgb, tex, err);
    if (magic[0] == 0xFF && magic[1] == 0xD8) return load_jpeg(path, srgb, tex, err);
    err = path + ": unsupported image format (DDS, PNG and JPEG are decoded)";
    return false;
}

}  // namespace dxrpt_host
