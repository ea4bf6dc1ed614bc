// omm.cpp — opacity micromap builder (host side of DXRPT_OPT_OPACITY_MICROMAP).
//
// AnyHitShader / ShadowAnyHitShader (RayTrace.hlsl:485-507) reject a candidate hit when the bilinear
// mip-0 tap of the opacity map at the hit's interpolated UV is below 0.35.  Alpha-tested foliage and
// cloth cards are mostly texels far from that threshold, so over most of a triangle the verdict is the
// same at every point: this builder finds, per barycentric cell (pt_layout.h kOmm*), whether every tap
// the kernel can take there reads only texels >= kOpaqueMin (accept) or only texels <= kTransparentMax
// (reject).  The kernels then skip the UV interpolation and the texel round trip for those candidates;
// cells with any texel near the threshold or mixed texels stay kOmmUnknown and are tapped as before, so
// every hit, miss and occlusion is bit-identical with and without the micromap.
//
// Conservativeness (what makes a verdict exact):
//  * barycentrics: the kernel's cell comes from floor(b1 * kOmmSplit), floor(b2 * kOmmSplit) of the float
//    barycentrics (omm_cell), so a point of cell (i, j) lies in [i/N, (i+1)/N] x [j/N, (j+1)/N] up to the
//    rounding of one product; the clamped cells of the hypotenuse row hold points with b1 + b2 <= 1 up
//    to rounding, i.e. inside the same box.  The box is widened by kBaryEps.
//  * UV: u = (u0 w0 + u1 b1) + u2 b2 with w0 = (1 - b1) - b2 (bary_lerp, no contraction) is affine in
//    (b1, b2), so over the box it lies between the values at the four corners; the float evaluation
//    error is below 8 ulp of |u0| + |u1| + |u2| (kUvRel bounds it).
//  * texels: the tap's columns are floor(u W - 0.5) and the next one (wrap addressing), so the
//    footprint of a u interval [ulo, uhi] is columns floor(ulo W - 0.5 - m) .. floor(uhi W - 0.5 + m) + 1
//    (m covers the rounding of u W - 0.5); rows alike.
//  * filtering: lerp(lerp(a, b, fx), lerp(c, d, fx), fy) of four values >= 0.3501 is >= 0.35 in float
//    (each lerp stays within its endpoints up to one rounding of ~3e-8), and of four values <= 0.3499 is
//    < 0.35.  Decoded texels are k/255 (or their sRGB decode), never inside (0.3499, 0.3501) for unorm.
#include "omm.h"

#include <cmath>
#include <cstring>

#include "pt_layout.h"

namespace dxrpt {

namespace {
constexpr float kOpaqueMin = 0.3501f;
constexpr float kTransparentMax = 0.3499f;
constexpr double kBaryEps = 1e-6;
constexpr double kUvRel = 1e-6;
}  // namespace

float omm_decode(uint32_t lut_base, uint32_t b) {
    if (lut_base == 0u) return float(b) / 255.0f;
    const double c = double(b) / 255.0;
    return float(c <= 0.04045 ? c / 12.92 : std::pow((c + 0.055) / 1.055, 2.4));
}

OpacityField::OpacityField(uint32_t w, uint32_t h, std::vector<float> values) : w_(w), h_(h) {
    const size_t pitch = size_t(w) + 1u;
    sat_op_.assign(pitch * (size_t(h) + 1u), 0u);
    sat_tr_.assign(pitch * (size_t(h) + 1u), 0u);
    for (uint32_t y = 0; y < h; ++y) {
        uint32_t row_op = 0, row_tr = 0;
        for (uint32_t x = 0; x < w; ++x) {
            const float v = values[size_t(y) * w + x];
            row_op += v >= kOpaqueMin ? 1u : 0u;
            row_tr += v <= kTransparentMax ? 1u : 0u;
            sat_op_[(y + 1u) * pitch + x + 1u] = sat_op_[y * pitch + x + 1u] + row_op;
            sat_tr_[(y + 1u) * pitch + x + 1u] = sat_tr_[y * pitch + x + 1u] + row_tr;
        }
    }
}

uint64_t OpacityField::count(const std::vector<uint32_t>& sat, int64_t x0, int64_t x1, int64_t y0, int64_t y1) const {
    // inclusive rectangle inside [0, w) x [0, h)
    const size_t p = size_t(w_) + 1u;
    return uint64_t(sat[size_t(y1 + 1) * p + size_t(x1 + 1)]) - sat[size_t(y0) * p + size_t(x1 + 1)] -
           sat[size_t(y1 + 1) * p + size_t(x0)] + sat[size_t(y0) * p + size_t(x0)];
}

uint32_t OpacityField::verdict(int64_t x0, int64_t x1, int64_t y0, int64_t y1) const {
    // wrapped column / row ranges: at most two intervals each
    auto split = [](int64_t a, int64_t b, int64_t n, int64_t iv[2][2]) {
        if (b - a + 1 >= n) {
            iv[0][0] = 0;
            iv[0][1] = n - 1;
            return 1;
        }
        const int64_t s = ((a % n) + n) % n, len = b - a + 1;
        if (s + len <= n) {
            iv[0][0] = s;
            iv[0][1] = s + len - 1;
            return 1;
        }
        iv[0][0] = s;
        iv[0][1] = n - 1;
        iv[1][0] = 0;
        iv[1][1] = s + len - 1 - n;
        return 2;
    };
    int64_t cx[2][2], cy[2][2];
    const int nx = split(x0, x1, w_, cx), ny = split(y0, y1, h_, cy);
    uint64_t area = 0, op = 0, tr = 0;
    for (int a = 0; a < nx; ++a)
        for (int b = 0; b < ny; ++b) {
            area += uint64_t(cx[a][1] - cx[a][0] + 1) * uint64_t(cy[b][1] - cy[b][0] + 1);
            op += count(sat_op_, cx[a][0], cx[a][1], cy[b][0], cy[b][1]);
            tr += count(sat_tr_, cx[a][0], cx[a][1], cy[b][0], cy[b][1]);
        }
    if (op == area) return kOmmOpaque;
    if (tr == area) return kOmmTransparent;
    return kOmmUnknown;
}

void omm_triangle(const OpacityField& F, const float* uv, uint32_t* out) {
    for (uint32_t k = 0; k < kOmmWords; ++k) out[k] = 0u;
    for (int k = 0; k < 6; ++k)
        if (!std::isfinite(uv[k]) || std::fabs(uv[k]) > 1e6f) return;  // all unknown
    const double u0 = uv[0], v0 = uv[1], u1 = uv[2], v1 = uv[3], u2 = uv[4], v2 = uv[5];
    const double W = F.width(), H = F.height();
    const double du = kUvRel * (std::fabs(u0) + std::fabs(u1) + std::fabs(u2) + 1.0);
    const double dv = kUvRel * (std::fabs(v0) + std::fabs(v1) + std::fabs(v2) + 1.0);
    const double N = kOmmSplit;
    uint32_t c = 0;
    for (uint32_t i = 0; i < kOmmSplit; ++i)
        for (uint32_t j = 0; j + i < kOmmSplit; ++j, ++c) {
            const double b1[2] = {i / N - kBaryEps, (i + 1) / N + kBaryEps};
            const double b2[2] = {j / N - kBaryEps, (j + 1) / N + kBaryEps};
            double ulo = INFINITY, uhi = -INFINITY, vlo = INFINITY, vhi = -INFINITY;
            for (double p : b1)
                for (double q : b2) {
                    const double u = u0 + p * (u1 - u0) + q * (u2 - u0);
                    const double v = v0 + p * (v1 - v0) + q * (v2 - v0);
                    ulo = std::fmin(ulo, u);
                    uhi = std::fmax(uhi, u);
                    vlo = std::fmin(vlo, v);
                    vhi = std::fmax(vhi, v);
                }
            // texel coordinate x = u W - 0.5 in float: rounding of the product and the subtraction
            const double mx = (std::fmax(std::fabs(ulo), std::fabs(uhi)) * W + 1.0) * 1e-6 + 1e-3;
            const double my = (std::fmax(std::fabs(vlo), std::fabs(vhi)) * H + 1.0) * 1e-6 + 1e-3;
            const int64_t x0 = int64_t(std::floor((ulo - du) * W - 0.5 - mx));
            const int64_t x1 = int64_t(std::floor((uhi + du) * W - 0.5 + mx)) + 1;
            const int64_t y0 = int64_t(std::floor((vlo - dv) * H - 0.5 - my));
            const int64_t y1 = int64_t(std::floor((vhi + dv) * H - 0.5 + my)) + 1;
            const uint32_t s = F.verdict(x0, x1, y0, y1);
            out[c >> 4] |= s << (2u * (c & 15u));
        }
}

}  // namespace dxrpt
