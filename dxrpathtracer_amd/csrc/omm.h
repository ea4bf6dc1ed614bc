// omm.h — opacity micromap builder (host).  See pt_layout.h (kOmm*) for the device format.
#pragma once
#include <stdint.h>

#include <vector>

namespace dxrpt {

// One opacity map, decoded to the float AnyHitShader filters (channel r through the unorm / sRGB table
// the kernels use), row-major w x h, plus summed-area tables of its "certainly opaque" and "certainly
// transparent" texels.
class OpacityField {
  public:
    OpacityField(uint32_t w, uint32_t h, std::vector<float> values);
    uint32_t width() const { return w_; }
    uint32_t height() const { return h_; }
    // Verdict (kOmmOpaque / kOmmTransparent / kOmmUnknown) of every bilinear tap whose footprint lies in
    // texel columns [x0, x1] x rows [y0, y1] (inclusive, unwrapped: wrap addressing is applied here).
    uint32_t verdict(int64_t x0, int64_t x1, int64_t y0, int64_t y1) const;

  private:
    uint64_t count(const std::vector<uint32_t>& sat, int64_t x0, int64_t x1, int64_t y0, int64_t y1) const;
    uint32_t w_, h_;
    std::vector<uint32_t> sat_op_, sat_tr_;  // (w + 1) x (h + 1) inclusive prefix counts
};

// The kOmmWords words of one triangle with vertex UVs uv[0..5] = (u0, v0, u1, v1, u2, v2) on `field`.
void omm_triangle(const OpacityField& field, const float* uv, uint32_t* out);

// Decoded opacity of texel byte b (lut_base 0: unorm, 256: sRGB; the table of dxrpt_api.hip make_lut).
float omm_decode(uint32_t lut_base, uint32_t b);

}  // namespace dxrpt
