// sky.cpp — sky cubemap + sun constants (the SkyCache::Init role, Graphics/Skybox.cpp:48-215).
//
// The reference evaluates the Hosek-Wilkie RGB model (HosekSky/ArHosekSkyModel.cpp:604-656) per
// cube texel and integrates the spectral solar radiance over the sun disc.  Those coefficient
// tables are not reproduced here; this file is a documented PROXY with the same inputs, outputs,
// units and cube layout: Preetham-Shirley-Smits (1999) sky luminance/chromaticity (Perez model)
// and a Beer-Lambert sun (Rayleigh + Angstrom aerosol), both pre-scaled by FP16Scale = 2^-10 like
// the reference (Skybox.cpp:125, 269).  The path tracer consumes the cube as opaque input data, so
// parity of the hot path does not depend on which sky model produced it.
//
// Kept from the reference exactly: sun direction handling (y saturated, normalised; Skybox.cpp:51-53),
// AngleBetween's clamp of the cosine at 1e-5 (Skybox.cpp:33-36), the texel -> direction map
// MapXYSToDirection (Graphics/Textures.cpp:585-616), the SunRenderColor rule
// (irradiance / (pi sin^2(SunSize)), max component clamped to FP16Max; Skybox.cpp:142-154).
#include <algorithm>
#include <cmath>
#include <cstring>

#include "scene_builder.h"

namespace {

constexpr double kFP16Scale = 0.0009765625;  // Shaders/Constants.hlsl:27
constexpr double kFP16Max = 65000.0;

double angle_between(const double a[3], const double b[3]) {
    double d = a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
    return std::acos(std::max(d, 0.00001));
}

struct Perez {
    double A, B, C, D, E;
    double f(double theta, double gamma) const {
        double ct = std::cos(theta), cg = std::cos(gamma);
        return (1.0 + A * std::exp(B / ct)) * (1.0 + C * std::exp(D * gamma) + E * cg * cg);
    }
};

struct Preetham {
    Perez pY, px, py;
    double Yz, xz, yz, thetaS;
    double sun[3];

    Preetham(const double sun_dir[3], double T) {
        std::memcpy(sun, sun_dir, sizeof(sun));
        const double up[3] = {0, 1, 0};
        thetaS = angle_between(sun_dir, up);
        pY = {0.1787 * T - 1.4630, -0.3554 * T + 0.4275, -0.0227 * T + 5.3251, 0.1206 * T - 2.5771, -0.0670 * T + 0.3703};
        px = {-0.0193 * T - 0.2592, -0.0665 * T + 0.0008, -0.0004 * T + 0.2125, -0.0641 * T - 0.8989, -0.0033 * T + 0.0452};
        py = {-0.0167 * T - 0.2608, -0.0950 * T + 0.0092, -0.0079 * T + 0.2102, -0.0441 * T - 1.6537, -0.0109 * T + 0.0529};
        const double chi = (4.0 / 9.0 - T / 120.0) * (M_PI - 2.0 * thetaS);
        Yz = ((4.0453 * T - 4.9710) * std::tan(chi) - 0.2155 * T + 2.4192) * 1000.0;  // kcd/m^2 -> cd/m^2
        const double t = thetaS, t2 = t * t, t3 = t2 * t, T2 = T * T;
        xz = T2 * (0.00166 * t3 - 0.00375 * t2 + 0.00209 * t) + T * (-0.02903 * t3 + 0.06377 * t2 - 0.03202 * t + 0.00394) +
             (0.11693 * t3 - 0.21196 * t2 + 0.06052 * t + 0.25886);
        yz = T2 * (0.00275 * t3 - 0.00610 * t2 + 0.00317 * t) + T * (-0.04214 * t3 + 0.08970 * t2 - 0.04153 * t + 0.00516) +
             (0.15346 * t3 - 0.26756 * t2 + 0.06670 * t + 0.26688);
    }

    // Linear sRGB radiance in cd/m^2-equivalent units for direction d (unit vector).
    void radiance(const double d[3], double rgb[3]) const {
        const double up[3] = {0, 1, 0};
        const double theta = angle_between(d, up);
        const double gamma = angle_between(d, sun);
        const double Y = Yz * pY.f(theta, gamma) / pY.f(0.0, thetaS);
        const double x = xz * px.f(theta, gamma) / px.f(0.0, thetaS);
        const double y = yz * py.f(theta, gamma) / py.f(0.0, thetaS);
        const double X = x / y * Y, Z = (1.0 - x - y) / y * Y;
        rgb[0] = std::max(0.0, 3.2404542 * X - 1.5371385 * Y - 0.4985314 * Z);
        rgb[1] = std::max(0.0, -0.9692660 * X + 1.8760108 * Y + 0.0415560 * Z);
        rgb[2] = std::max(0.0, 0.0556434 * X - 0.2040259 * Y + 1.0572252 * Z);
    }
};

// MapXYSToDirection, Graphics/Textures.cpp:585-616
void map_xys_to_direction(uint32_t x, uint32_t y, uint32_t s, uint32_t w, uint32_t h, double out[3]) {
    float u = ((float(x) + 0.5f) / float(w)) * 2.0f - 1.0f;
    float v = ((float(y) + 0.5f) / float(h)) * 2.0f - 1.0f;
    v *= -1.0f;
    float d[3] = {0, 0, 0};
    switch (s) {
        case 0: d[0] = 1.0f; d[1] = v; d[2] = -u; break;
        case 1: d[0] = -1.0f; d[1] = v; d[2] = u; break;
        case 2: d[0] = u; d[1] = 1.0f; d[2] = -v; break;
        case 3: d[0] = u; d[1] = -1.0f; d[2] = v; break;
        case 4: d[0] = u; d[1] = v; d[2] = 1.0f; break;
        default: d[0] = -u; d[1] = v; d[2] = -1.0f; break;
    }
    double l = std::sqrt(double(d[0]) * d[0] + double(d[1]) * d[1] + double(d[2]) * d[2]);
    for (int k = 0; k < 3; ++k) out[k] = d[k] / l;
}

void normalize_sun(const float in[3], double out[3]) {
    double s[3] = {in[0], std::min(std::max(double(in[1]), 0.0), 1.0), in[2]};
    double l = std::sqrt(s[0] * s[0] + s[1] * s[1] + s[2] * s[2]);
    if (l == 0) { out[0] = 0; out[1] = 1; out[2] = 0; return; }
    for (int k = 0; k < 3; ++k) out[k] = s[k] / l;
}

}  // namespace

extern "C" {

uint16_t dxrpt_host_float_to_half(float f) {
    uint32_t x;
    std::memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t mant = x & 0x7FFFFFu;
    int32_t exp = int32_t((x >> 23) & 0xFFu);
    if (exp == 0xFF) return uint16_t(sign | 0x7C00u | (mant ? 0x200u : 0u));  // inf / nan
    int32_t e = exp - 127 + 15;
    if (e >= 31) return uint16_t(sign | 0x7C00u);                              // overflow -> inf
    if (e <= 0) {                                                              // subnormal / zero
        if (e < -10) return uint16_t(sign);
        mant |= 0x800000u;
        const uint32_t shift = uint32_t(14 - e);
        uint32_t hm = mant >> shift;
        const uint32_t rem = mant & ((1u << shift) - 1u), half = 1u << (shift - 1);
        if (rem > half || (rem == half && (hm & 1u))) ++hm;
        return uint16_t(sign | hm);
    }
    uint32_t hm = mant >> 13;
    const uint32_t rem = mant & 0x1FFFu;
    uint32_t h = sign | (uint32_t(e) << 10) | hm;
    if (rem > 0x1000u || (rem == 0x1000u && (hm & 1u))) ++h;  // carries into the exponent correctly
    return uint16_t(h);
}

float dxrpt_host_half_to_float(uint16_t h) {
    const uint32_t sign = uint32_t(h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1Fu, mant = h & 0x3FFu;
    uint32_t x;
    if (exp == 0) {
        if (mant == 0) x = sign;
        else {
            int e = -1;
            do { ++e; mant <<= 1; } while (!(mant & 0x400u));
            x = sign | (uint32_t(127 - 15 - e) << 23) | ((mant & 0x3FFu) << 13);
        }
    } else if (exp == 31) {
        x = sign | 0x7F800000u | (mant << 13);
    } else {
        x = sign | ((exp - 15 + 127) << 23) | (mant << 13);
    }
    float f;
    std::memcpy(&f, &x, 4);
    return f;
}

int dxrpt_host_sky_create(const float sun_direction[3], float sun_size_deg, float turbidity,
                          const float ground_albedo[3], uint32_t res, uint16_t* out_cube,
                          float out_sun_irradiance[3], float out_sun_render_color[3]) {
    (void)ground_albedo;  // the Preetham proxy has no ground albedo term
    if (!sun_direction || res == 0 || !out_cube || !out_sun_irradiance || !out_sun_render_color) return DXRPT_E_INVALID_ARG;
    const double T = std::min(std::max(double(turbidity), 1.0), 32.0);
    const double sunSize = std::max(double(sun_size_deg), 0.01);
    double sun[3];
    normalize_sun(sun_direction, sun);
    Preetham sky(sun, std::min(T, 10.0));

    // Sun irradiance on a surface facing the sun: top-of-atmosphere RGB (scaled to the reference's
    // 683 * 100 * 2^-10 photometric convention) times Beer-Lambert transmittance along the air mass.
    const double thetaS_deg = sky.thetaS * 180.0 / M_PI;
    const double airmass = 1.0 / (std::cos(sky.thetaS) + 0.15 * std::pow(std::max(93.885 - thetaS_deg, 1e-3), -1.253));
    const double beta = 0.04608 * T - 0.04586;
    const double lambda_um[3] = {0.680, 0.550, 0.440};
    const double toa = 128000.0 * kFP16Scale;  // ~128 klx solar illuminance
    for (int k = 0; k < 3; ++k) {
        double tauR = 0.008735 * std::pow(lambda_um[k], -4.08);
        double tauA = beta * std::pow(lambda_um[k], -1.3);
        out_sun_irradiance[k] = float(toa * std::exp(-airmass * (tauR + tauA)));
    }
    // SunRenderColor (Skybox.cpp:142-154)
    const double sinS = std::sin(sunSize * M_PI / 180.0);
    const double integral = M_PI * sinS * sinS;
    double col[3], mx = 0;
    for (int k = 0; k < 3; ++k) {
        col[k] = out_sun_irradiance[k] / integral;
        mx = std::max(mx, col[k]);
    }
    for (int k = 0; k < 3; ++k) {
        if (mx > kFP16Max) col[k] *= kFP16Max / mx;
        out_sun_render_color[k] = float(std::min(std::max(col[k], 0.0), kFP16Max));
    }
    // Cube texels (Skybox.cpp:160-201): radiance * FP16Scale -> Half4(rgb, 1)
    for (uint32_t s = 0; s < 6; ++s)
        for (uint32_t y = 0; y < res; ++y)
            for (uint32_t x = 0; x < res; ++x) {
                double d[3], rgb[3];
                map_xys_to_direction(x, y, s, res, res, d);
                sky.radiance(d, rgb);
                uint16_t* t = out_cube + ((size_t(s) * res + y) * res + x) * 4;
                for (int k = 0; k < 3; ++k) t[k] = dxrpt_host_float_to_half(float(rgb[k] * kFP16Scale));
                t[3] = dxrpt_host_float_to_half(1.0f);
            }
    return DXRPT_OK;
}

}  // extern "C"
