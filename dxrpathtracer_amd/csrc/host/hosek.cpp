// hosek.cpp — the reference's sky: Hosek-Wilkie sky model + spectral solar disc, integrated the way
// SkyCache::Init does (SampleFramework12/v1.02/Graphics/Skybox.cpp:48-215, Sample 252-270).
//
// Restated here (not copied): the model evaluation of HosekSky/ArHosekSkyModel.cpp —
//   ArHosekSkyModel_CookConfiguration          :149-229  (quintic Bezier in elevation^(1/3), lerp in
//                                                         turbidity and ground albedo)
//   ArHosekSkyModel_CookRadianceConfiguration  :231-291
//   ArHosekSkyModel_GetRadianceInternal        :293-306  (the 9-parameter extended Perez formula)
//   arhosekskymodelstate_alloc_init            :310-345, arhosekskymodel_radiance :521-566
//   arhosek_rgb_skymodelstate_alloc_init       :604-637, arhosek_tristim_skymodel_radiance :639-652
//   arhosekskymodel_sr_internal                :658-687, ..._solar_radiance_internal2 :689-791,
//   arhosekskymodel_solar_radiance             :793-818
// and the pbrt-v3 spectral helpers of Graphics/Spectrum.{h,cpp} that SkyCache::Init uses
// (AverageSpectrumSamples :74-110, SampledSpectrum::Init / ToXYZ / ToRGB Spectrum.h:296-375,
// FromRGB(Reflectance) Spectrum.cpp:113-185, XYZToRGB Spectrum.h:51-55).
//
// The model's coefficient tables (published with the model: RGB and spectral datasets, solar
// radiance and limb darkening fits) and the CIE 1931 / Smits RGB-to-spectrum tables are DATA: they
// ship with the package as dxrpathtracer_amd/data/hosek_tables.bin (written once by
// scripts/make_hosek_tables.py from the reference's HosekSky/ArHosekSkyModelData_{RGB,Spectral}.h and
// Graphics/Spectrum.cpp) and are read from that file at run time (dxrpt_host_hosek_load_tables), like
// a scene asset; nothing reads the reference checkout at run time.
//
// Arithmetic follows the reference's types: doubles inside the model, floats in SkyCache::Init
// (Float3 ops as DirectXMath's SSE2 paths: dot = (x*x + y*y) + z*z, normalize = v / sqrt(dot),
// cross from exact products, XMVector3TransformCoord with a 3x3 = ((z*r2 + y*r1) + x*r0)).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../../include/dxrpt_host.h"
#include "scene_builder.h"

namespace {

constexpr double kMathPi = 3.141592653589793;  // ArHosekSkyModel.cpp:119
constexpr float kPi = 3.141592654f;            // SF12_Math.h:551
constexpr float kPi_2 = 1.570796327f;          // SF12_Math.h:553
constexpr float kFP16Scale = 0.0009765625f;    // SF12_Math.h:562
constexpr float kFP16Max = 65000.0f;           // SF12_Math.h:559
constexpr int kNumSpectral = 60;               // Spectrum.h:43-45: 60 samples over [400, 700) nm
constexpr int kLambdaStart = 400, kLambdaEnd = 700;
constexpr float kCIEYIntegral = 106.856895f;   // Spectrum.h:76

// ---- named numeric arrays from a C/C++ source ------------------------------------------------------
bool read_file(const std::string& path, std::string& out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::ostringstream ss;
    ss << f.rdbuf();
    out = ss.str();
    return true;
}

// The initializer list of `<type> name[...] = { ... };` as doubles.  Returns false if not found.
bool named_array(const std::string& src, const std::string& name, std::vector<double>& out) {
    size_t p = 0;
    while ((p = src.find(name, p)) != std::string::npos) {
        const bool start_ok = p == 0 || !(std::isalnum(uint8_t(src[p - 1])) || src[p - 1] == '_');
        size_t q = p + name.size();
        p = q;
        if (!start_ok) continue;
        while (q < src.size() && std::isspace(uint8_t(src[q]))) ++q;
        if (q >= src.size() || src[q] != '[') continue;
        q = src.find(']', q);
        if (q == std::string::npos) return false;
        ++q;
        while (q < src.size() && std::isspace(uint8_t(src[q]))) ++q;
        if (q >= src.size() || src[q] != '=') continue;
        q = src.find('{', q);
        if (q == std::string::npos) return false;
        ++q;
        out.clear();
        while (q < src.size() && src[q] != '}') {
            const char c = src[q];
            if (c == '/' && q + 1 < src.size() && src[q + 1] == '/') {
                q = src.find('\n', q);
                if (q == std::string::npos) return false;
            } else if (c == '/' && q + 1 < src.size() && src[q + 1] == '*') {
                q = src.find("*/", q);
                if (q == std::string::npos) return false;
                q += 2;
            } else if (std::isdigit(uint8_t(c)) || c == '-' || c == '+' || c == '.') {
                char* end = nullptr;
                const double v = std::strtod(src.c_str() + q, &end);
                if (end == src.c_str() + q) return false;
                out.push_back(v);
                q = size_t(end - src.c_str());
                if (q < src.size() && (src[q] == 'f' || src[q] == 'F')) ++q;
            } else {
                ++q;
            }
        }
        return !out.empty();
    }
    return false;
}

// ---- Float3 (SF12 / DirectXMath SSE2 semantics) -------------------------------------------------
struct F3 {
    float x, y, z;
};
float dot(F3 a, F3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
F3 normalize(F3 a) {
    const float l = std::sqrt(dot(a, a));
    return {a.x / l, a.y / l, a.z / l};
}
F3 cross(F3 a, F3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
float saturate(float v) { return std::min(std::max(v, 0.0f), 1.0f); }
// Skybox.cpp:35-38
float angle_between(F3 a, F3 b) { return std::acos(std::max(dot(a, b), 0.00001f)); }
// SF12_Math.cpp:456-476
F3 perpendicular(F3 v) {
    const float x = std::abs(v.x), y = std::abs(v.y), z = std::abs(v.z);
    const float m = std::min(std::min(x, y), z);
    F3 p;
    if (m == x) p = cross(v, F3{1.0f, 0.0f, 0.0f});
    else if (m == y) p = cross(v, F3{0.0f, 1.0f, 0.0f});
    else p = cross(v, F3{0.0f, 0.0f, 1.0f});
    return normalize(p);
}
// XMVector3TransformCoord(v, Float3x3(r0, r1, r2)): ((z*r2 + (0,0,0)) + y*r1) + x*r0, w = 1
F3 transform(F3 v, F3 r0, F3 r1, F3 r2) {
    F3 t{v.z * r2.x + 0.0f, v.z * r2.y + 0.0f, v.z * r2.z + 0.0f};
    t = F3{v.y * r1.x + t.x, v.y * r1.y + t.y, v.y * r1.z + t.z};
    t = F3{v.x * r0.x + t.x, v.x * r0.y + t.y, v.x * r0.z + t.z};
    return t;
}
float lerpf(float x, float y, float s) { return x + (y - x) * s; }  // SF12_Math.h:570-573
float deg_to_rad(float d) { return d * (1.0f / 180.0f) * 3.14159265359f; }  // SF12_Math.h:663-666

}  // namespace

// ---- datasets --------------------------------------------------------------------------------------
struct dxrpt_host_hosek {
    std::vector<double> rgb[3], rgbRad[3];
    std::vector<double> spec[11], specRad[11], solar[11], limb[11];
    std::vector<float> cieLambda, cieX, cieY, cieZ, rgbLambda, refl[7];  // white cyan magenta yellow red green blue
    // SampledSpectrum::Init products
    float X[kNumSpectral], Y[kNumSpectral], Z[kNumSpectral], R[7][kNumSpectral];
};

namespace {

enum { kWhite, kCyan, kMagenta, kYellow, kRed, kGreen, kBlue };

// Spectrum.cpp:74-110
float average_spectrum_samples(const float* lambda, const float* vals, int n, float lambdaStart, float lambdaEnd) {
    if (lambdaEnd <= lambda[0]) return vals[0];
    if (lambdaStart >= lambda[n - 1]) return vals[n - 1];
    if (n == 1) return vals[0];
    float sum = 0;
    if (lambdaStart < lambda[0]) sum += vals[0] * (lambda[0] - lambdaStart);
    if (lambdaEnd > lambda[n - 1]) sum += vals[n - 1] * (lambdaEnd - lambda[n - 1]);
    int i = 0;
    while (lambdaStart > lambda[i + 1]) ++i;
    auto interp = [lambda, vals](float w, int k) {
        const float t = (w - lambda[k]) / (lambda[k + 1] - lambda[k]);
        return (1 - t) * vals[k] + t * vals[k + 1];  // SpectrumLerp, Spectrum.h:98
    };
    for (; i + 1 < n && lambdaEnd >= lambda[i]; ++i) {
        const float s0 = std::max(lambdaStart, lambda[i]);
        const float s1 = std::min(lambdaEnd, lambda[i + 1]);
        sum += 0.5f * (interp(s0, i) + interp(s1, i)) * (s1 - s0);
    }
    return sum / (lambdaEnd - lambdaStart);
}

float spectrum_lerp(float t, float v1, float v2) { return (1 - t) * v1 + t * v2; }

// SampledSpectrum::Init (Spectrum.h:296-360), the reflectance tables only
void spectrum_init(dxrpt_host_hosek& H) {
    for (int i = 0; i < kNumSpectral; ++i) {
        const float wl0 = spectrum_lerp(float(i) / float(kNumSpectral), float(kLambdaStart), float(kLambdaEnd));
        const float wl1 = spectrum_lerp(float(i + 1) / float(kNumSpectral), float(kLambdaStart), float(kLambdaEnd));
        const int nc = int(H.cieLambda.size());
        H.X[i] = average_spectrum_samples(H.cieLambda.data(), H.cieX.data(), nc, wl0, wl1);
        H.Y[i] = average_spectrum_samples(H.cieLambda.data(), H.cieY.data(), nc, wl0, wl1);
        H.Z[i] = average_spectrum_samples(H.cieLambda.data(), H.cieZ.data(), nc, wl0, wl1);
        const int nr = int(H.rgbLambda.size());
        for (int k = 0; k < 7; ++k) H.R[k][i] = average_spectrum_samples(H.rgbLambda.data(), H.refl[k].data(), nr, wl0, wl1);
    }
}

// SampledSpectrum::FromRGB(rgb, Reflectance), Spectrum.cpp:113-153 + Clamp()
void spectrum_from_rgb_reflectance(const dxrpt_host_hosek& H, const float rgb[3], float out[kNumSpectral]) {
    float r[kNumSpectral] = {};
    auto add = [&](float a, int table) {
        for (int i = 0; i < kNumSpectral; ++i) r[i] += H.R[table][i] * a;  // (a * s) = s * a, then +=
    };
    if (rgb[0] <= rgb[1] && rgb[0] <= rgb[2]) {
        add(rgb[0], kWhite);
        if (rgb[1] <= rgb[2]) { add(rgb[1] - rgb[0], kCyan); add(rgb[2] - rgb[1], kBlue); }
        else { add(rgb[2] - rgb[0], kCyan); add(rgb[1] - rgb[2], kGreen); }
    } else if (rgb[1] <= rgb[0] && rgb[1] <= rgb[2]) {
        add(rgb[1], kWhite);
        if (rgb[0] <= rgb[2]) { add(rgb[0] - rgb[1], kMagenta); add(rgb[2] - rgb[0], kBlue); }
        else { add(rgb[2] - rgb[1], kMagenta); add(rgb[0] - rgb[2], kRed); }
    } else {
        add(rgb[2], kWhite);
        if (rgb[0] <= rgb[1]) { add(rgb[0] - rgb[2], kYellow); add(rgb[1] - rgb[0], kGreen); }
        else { add(rgb[1] - rgb[2], kYellow); add(rgb[0] - rgb[1], kRed); }
    }
    for (int i = 0; i < kNumSpectral; ++i) {
        r[i] *= .94f;
        out[i] = std::min(std::max(r[i], 0.0f), INFINITY);
    }
}

// SampledSpectrum::ToRGB = XYZToRGB(ToXYZ) (Spectrum.h:51-55, 362-385)
void spectrum_to_rgb(const dxrpt_host_hosek& H, const float c[kNumSpectral], float rgb[3]) {
    float xyz[3] = {0.f, 0.f, 0.f};
    for (int i = 0; i < kNumSpectral; ++i) {
        xyz[0] += H.X[i] * c[i];
        xyz[1] += H.Y[i] * c[i];
        xyz[2] += H.Z[i] * c[i];
    }
    const float scale = float(kLambdaEnd - kLambdaStart) / float(kCIEYIntegral * kNumSpectral);
    xyz[0] *= scale;
    xyz[1] *= scale;
    xyz[2] *= scale;
    rgb[0] = 3.240479f * xyz[0] - 1.537150f * xyz[1] - 0.498535f * xyz[2];
    rgb[1] = -0.969256f * xyz[0] + 1.875991f * xyz[1] + 0.041556f * xyz[2];
    rgb[2] = 0.055648f * xyz[0] - 0.204043f * xyz[1] + 1.057311f * xyz[2];
}

// ---- the model -------------------------------------------------------------------------------------
struct HState {
    double configs[11][9];
    double radiances[11];
    double turbidity, albedo, elevation, solar_radius;
};

// Bernstein weights of the quintic in t = (elevation / (pi/2))^(1/3), in the reference's term order
double quintic(const double* m, int stride, double s) {
    return std::pow(1.0 - s, 5.0) * m[0] + 5.0 * std::pow(1.0 - s, 4.0) * s * m[stride] +
           10.0 * std::pow(1.0 - s, 3.0) * std::pow(s, 2.0) * m[2 * stride] +
           10.0 * std::pow(1.0 - s, 2.0) * std::pow(s, 3.0) * m[3 * stride] +
           5.0 * (1.0 - s) * std::pow(s, 4.0) * m[4 * stride] + std::pow(s, 5.0) * m[5 * stride];
}

// ArHosekSkyModel.cpp:149-229 (config, 9 x 6 Bezier control points per turbidity, 10 turbidities x 2
// albedos) and :231-291 (radiance scale, 6 per turbidity).  `stride` 9 or 1, `block` 54 or 6.
void cook(const double* dataset, double* out, int n, int block, double turbidity, double albedo, double solar_elevation) {
    const int int_turbidity = int(turbidity);
    const double turbidity_rem = turbidity - double(int_turbidity);
    const double s = std::pow(solar_elevation / (kMathPi / 2.0), (1.0 / 3.0));
    const double* m = dataset + (block * (int_turbidity - 1));
    for (int i = 0; i < n; ++i) out[i] = (1.0 - albedo) * (1.0 - turbidity_rem) * quintic(m + i, n, s);
    m = dataset + (block * 10 + block * (int_turbidity - 1));
    for (int i = 0; i < n; ++i) out[i] += (albedo) * (1.0 - turbidity_rem) * quintic(m + i, n, s);
    if (int_turbidity == 10) return;
    m = dataset + (block * (int_turbidity));
    for (int i = 0; i < n; ++i) out[i] += (1.0 - albedo) * (turbidity_rem)*quintic(m + i, n, s);
    m = dataset + (block * 10 + block * (int_turbidity));
    for (int i = 0; i < n; ++i) out[i] += (albedo) * (turbidity_rem)*quintic(m + i, n, s);
}

// ArHosekSkyModel.cpp:293-306
double radiance_internal(const double* c, double theta, double gamma) {
    const double expM = std::exp(c[4] * gamma);
    const double rayM = std::cos(gamma) * std::cos(gamma);
    const double mieM = (1.0 + std::cos(gamma) * std::cos(gamma)) / std::pow((1.0 + c[8] * c[8] - 2.0 * c[8] * std::cos(gamma)), 1.5);
    const double zenith = std::sqrt(std::cos(theta));
    return (1.0 + c[0] * std::exp(c[1] / (std::cos(theta) + 0.01))) *
           (c[2] + c[3] * expM + c[5] * rayM + c[6] * mieM + c[7] * zenith);
}

void init_state(HState& st, const std::vector<double>* cfg, const std::vector<double>* rad, int channels, double turbidity,
                double albedo, double elevation, double solar_radius) {
    st.solar_radius = solar_radius;
    st.turbidity = turbidity;
    st.albedo = albedo;
    st.elevation = elevation;
    for (int c = 0; c < channels; ++c) {
        cook(cfg[c].data(), st.configs[c], 9, 54, turbidity, albedo, elevation);
        double r = 0.0;
        cook(rad[c].data(), &r, 1, 6, turbidity, albedo, elevation);
        st.radiances[c] = r;
    }
}

// arhosek_rgb_skymodelstate_alloc_init (:604-637): TERRESTRIAL_SOLAR_RADIUS = (0.51 deg) / 2
void rgb_state(const dxrpt_host_hosek& H, HState& st, double turbidity, double albedo, double elevation) {
    init_state(st, H.rgb, H.rgbRad, 3, turbidity, albedo, elevation, ((0.51 * (kMathPi / 180.0)) / 2.0));
}

// arhosekskymodelstate_alloc_init (:310-345)
void spectral_state(const dxrpt_host_hosek& H, HState& st, double solar_elevation, double turbidity, double albedo) {
    init_state(st, H.spec, H.specRad, 11, turbidity, albedo, solar_elevation, (0.51 * (kMathPi / 180.0)) / 2.0);
}

// arhosek_tristim_skymodel_radiance (:639-652)
double tristim_radiance(const HState& st, double theta, double gamma, int channel) {
    return radiance_internal(st.configs[channel], theta, gamma) * st.radiances[channel];
}

// arhosekskymodel_radiance (:521-566); emission correction factors are 1
double spectral_radiance(const HState& st, double theta, double gamma, double wavelength) {
    const int low_wl = int((wavelength - 320.0) / 40.0);
    if (low_wl < 0 || low_wl >= 11) return 0.0f;
    const double interp = std::fmod((wavelength - 320.0) / 40.0, 1.0);
    const double val_low = radiance_internal(st.configs[low_wl], theta, gamma) * st.radiances[low_wl] * 1.0;
    if (interp < 1e-6) return val_low;
    double result = (1.0 - interp) * val_low;
    if (low_wl + 1 < 11) result += interp * radiance_internal(st.configs[low_wl + 1], theta, gamma) * st.radiances[low_wl + 1] * 1.0;
    return result;
}

// arhosekskymodel_sr_internal (:658-687): 45 cubic pieces per turbidity
double sr_internal(const dxrpt_host_hosek& H, int turbidity, int wl, double elevation) {
    const int pieces = 45, order = 4;
    int pos = int(std::pow(2.0 * elevation / kMathPi, 1.0 / 3.0) * pieces);
    if (pos > 44) pos = 44;
    const double break_x = std::pow((double(pos) / double(pieces)), 3.0) * (kMathPi * 0.5);
    const double* coefs = H.solar[wl].data() + (order * pieces * turbidity + order * (pos + 1) - 1);
    double res = 0.0;
    const double x = elevation - break_x;
    double x_exp = 1.0;
    for (int i = 0; i < order; ++i) {
        res += x_exp * *coefs--;
        x_exp *= x;
    }
    return res * 1.0;
}

// arhosekskymodel_solar_radiance_internal2 (:689-791)
double solar_radiance_internal2(const dxrpt_host_hosek& H, const HState& st, double wavelength, double elevation, double gamma) {
    int turb_low = int(st.turbidity) - 1;
    double turb_frac = st.turbidity - double(turb_low + 1);
    if (turb_low == 9) {
        turb_low = 8;
        turb_frac = 1.0;
    }
    int wl_low = int((wavelength - 320.0) / 40.0);
    double wl_frac = std::fmod(wavelength, 40.0) / 40.0;
    if (wl_low == 10) {
        wl_low = 9;
        wl_frac = 1.0;
    }
    double direct_radiance =
        (1.0 - turb_frac) * ((1.0 - wl_frac) * sr_internal(H, turb_low, wl_low, elevation) +
                             wl_frac * sr_internal(H, turb_low, wl_low + 1, elevation)) +
        turb_frac * ((1.0 - wl_frac) * sr_internal(H, turb_low + 1, wl_low, elevation) +
                     wl_frac * sr_internal(H, turb_low + 1, wl_low + 1, elevation));
    double ld[6];
    for (int i = 0; i < 6; i++) ld[i] = (1.0 - wl_frac) * H.limb[wl_low][i] + wl_frac * H.limb[wl_low + 1][i];
    const double sol_rad_sin = std::sin(st.solar_radius);
    const double ar2 = 1 / (sol_rad_sin * sol_rad_sin);
    const double singamma = std::sin(gamma);
    double sc2 = 1.0 - ar2 * singamma * singamma;
    if (sc2 < 0.0) sc2 = 0.0;
    const double sampleCosine = std::sqrt(sc2);
    const double darkeningFactor = ld[0] + ld[1] * sampleCosine + ld[2] * std::pow(sampleCosine, 2.0) +
                                   ld[3] * std::pow(sampleCosine, 3.0) + ld[4] * std::pow(sampleCosine, 4.0) +
                                   ld[5] * std::pow(sampleCosine, 5.0);
    direct_radiance *= darkeningFactor;
    return direct_radiance;
}

// arhosekskymodel_solar_radiance (:793-818)
double solar_radiance(const dxrpt_host_hosek& H, const HState& st, double theta, double gamma, double wavelength) {
    const double direct = solar_radiance_internal2(H, st, wavelength, ((kMathPi / 2.0) - theta), gamma);
    const double inscattered = spectral_radiance(st, theta, gamma, wavelength);
    return direct + inscattered;
}

// Graphics/Textures.cpp:585-616
F3 map_xys_to_direction(uint64_t x, uint64_t y, uint64_t s, uint64_t width, uint64_t height) {
    const float u = ((x + 0.5f) / float(width)) * 2.0f - 1.0f;
    float v = ((y + 0.5f) / float(height)) * 2.0f - 1.0f;
    v *= -1.0f;
    F3 dir{0.0f, 0.0f, 0.0f};
    switch (s) {
        case 0: dir = normalize(F3{1.0f, v, -u}); break;
        case 1: dir = normalize(F3{-1.0f, v, u}); break;
        case 2: dir = normalize(F3{u, 1.0f, -v}); break;
        case 3: dir = normalize(F3{u, -1.0f, v}); break;
        case 4: dir = normalize(F3{u, v, 1.0f}); break;
        case 5: dir = normalize(F3{-u, v, -1.0f}); break;
    }
    return dir;
}

thread_local std::string g_hosek_err;

}  // namespace

extern "C" {

const char* dxrpt_host_hosek_last_error(void) { return g_hosek_err.c_str(); }

}  // extern "C"

namespace {

// Fills every table of `H` through `get(name, values)` (false: missing).  Model tables are doubles,
// the Spectrum.cpp tables are float literals.
template <class Get>
bool fill_tables(dxrpt_host_hosek& H, Get get, const char* who) {
    auto need = [&](const std::string& name, std::vector<double>& v, size_t n) {
        if (!get(name, v) || v.size() != n) {
            g_hosek_err = std::string(who) + ": array " + name + " missing or of unexpected size";
            return false;
        }
        return true;
    };
    auto needf = [&](const std::string& name, std::vector<float>& v, size_t n) {
        std::vector<double> d;
        if (!need(name, d, n)) return false;
        v.assign(d.begin(), d.end());
        return true;
    };
    bool ok = true;
    for (int c = 0; c < 3 && ok; ++c)
        ok = need("datasetRGB" + std::to_string(c + 1), H.rgb[c], 1080) &&
             need("datasetRGBRad" + std::to_string(c + 1), H.rgbRad[c], 120);
    for (int w = 0; w < 11 && ok; ++w) {
        const std::string wl = std::to_string(320 + 40 * w);
        ok = need("dataset" + wl, H.spec[w], 1080) && need("datasetRad" + wl, H.specRad[w], 120) &&
             need("solarDataset" + wl, H.solar[w], 1800) && need("limbDarkeningDataset" + wl, H.limb[w], 6);
    }
    static const char* refl[7] = {"RGBRefl2SpectWhite", "RGBRefl2SpectCyan", "RGBRefl2SpectMagenta", "RGBRefl2SpectYellow",
                                  "RGBRefl2SpectRed",   "RGBRefl2SpectGreen", "RGBRefl2SpectBlue"};
    ok = ok && needf("CIE_lambda", H.cieLambda, 471) && needf("CIE_X", H.cieX, 471) && needf("CIE_Y", H.cieY, 471) &&
         needf("CIE_Z", H.cieZ, 471) && needf("RGB2SpectLambda", H.rgbLambda, 32);
    for (int k = 0; k < 7 && ok; ++k) ok = needf(refl[k], H.refl[k], 32);
    if (ok) spectrum_init(H);
    return ok;
}

}  // namespace

extern "C" {

int dxrpt_host_hosek_load(const char* hosek_dir, const char* spectrum_source, dxrpt_host_hosek** out) {
    if (!hosek_dir || !spectrum_source || !out) {
        g_hosek_err = "dxrpt_host_hosek_load: null argument";
        return -1;
    }
    *out = nullptr;
    std::string rgb, spec, sp;
    const std::string dir(hosek_dir);
    if (!read_file(dir + "/ArHosekSkyModelData_RGB.h", rgb) || !read_file(dir + "/ArHosekSkyModelData_Spectral.h", spec) ||
        !read_file(spectrum_source, sp)) {
        g_hosek_err = "dxrpt_host_hosek_load: cannot read the dataset sources under " + dir + " / " + spectrum_source;
        return -1;
    }
    auto get = [&](const std::string& name, std::vector<double>& v) {
        const std::string& src = name.rfind("dataset", 0) == 0 && name.find("RGB") != std::string::npos ? rgb
                                 : (name.rfind("dataset", 0) == 0 || name.rfind("solar", 0) == 0 || name.rfind("limb", 0) == 0)
                                     ? spec
                                     : sp;
        return named_array(src, name, v);
    };
    auto* H = new dxrpt_host_hosek();
    if (!fill_tables(*H, get, "dxrpt_host_hosek_load")) {
        delete H;
        return -1;
    }
    *out = H;
    return 0;
}

// The packaged tables (dxrpathtracer_amd/data/hosek_tables.bin, scripts/make_hosek_tables.py):
// "DXRPTHK1", u32 count, then {u32 name length, name, u32 type (0 f64 / 1 f32), u32 count, data}.
int dxrpt_host_hosek_load_tables(const char* path, dxrpt_host_hosek** out) {
    if (!path || !out) {
        g_hosek_err = "dxrpt_host_hosek_load_tables: null argument";
        return -1;
    }
    *out = nullptr;
    std::string blob;
    if (!read_file(path, blob)) {
        g_hosek_err = std::string("dxrpt_host_hosek_load_tables: cannot read ") + path;
        return -1;
    }
    std::vector<std::pair<std::string, std::vector<double>>> tables;
    size_t p = 0;
    auto u32 = [&](uint32_t& v) {
        if (p + 4 > blob.size()) return false;
        std::memcpy(&v, blob.data() + p, 4);
        p += 4;
        return true;
    };
    uint32_t count = 0;
    bool ok = blob.size() >= 12 && blob.compare(0, 8, "DXRPTHK1") == 0;
    p = 8;
    ok = ok && u32(count);
    for (uint32_t i = 0; ok && i < count; ++i) {
        uint32_t nlen = 0, type = 0, n = 0;
        ok = u32(nlen) && p + nlen <= blob.size();
        if (!ok) break;
        std::string name = blob.substr(p, nlen);
        p += nlen;
        ok = u32(type) && u32(n) && type <= 1;
        const size_t esz = type == 0 ? 8 : 4;
        ok = ok && p + size_t(n) * esz <= blob.size();
        if (!ok) break;
        std::vector<double> v(n);
        for (uint32_t k = 0; k < n; ++k) {
            if (type == 0) {
                std::memcpy(&v[k], blob.data() + p + size_t(k) * 8, 8);
            } else {
                float f;
                std::memcpy(&f, blob.data() + p + size_t(k) * 4, 4);
                v[k] = f;
            }
        }
        p += size_t(n) * esz;
        tables.emplace_back(std::move(name), std::move(v));
    }
    if (!ok || p != blob.size()) {
        g_hosek_err = std::string("dxrpt_host_hosek_load_tables: malformed table file ") + path;
        return -1;
    }
    auto get = [&](const std::string& name, std::vector<double>& v) {
        for (auto& t : tables)
            if (t.first == name) {
                v = t.second;
                return true;
            }
        return false;
    };
    auto* H = new dxrpt_host_hosek();
    if (!fill_tables(*H, get, "dxrpt_host_hosek_load_tables")) {
        delete H;
        return -1;
    }
    *out = H;
    return 0;
}

void dxrpt_host_hosek_destroy(dxrpt_host_hosek* h) { delete h; }

double dxrpt_host_hosek_rgb_radiance(const dxrpt_host_hosek* H, double turbidity, double albedo, double elevation,
                                     double theta, double gamma, int channel) {
    HState st;
    rgb_state(*H, st, turbidity, albedo, elevation);
    return tristim_radiance(st, theta, gamma, channel);
}

double dxrpt_host_hosek_solar_radiance(const dxrpt_host_hosek* H, double solar_elevation, double turbidity, double albedo,
                                       double theta, double gamma, double wavelength) {
    HState st;
    spectral_state(*H, st, solar_elevation, turbidity, albedo);
    return solar_radiance(*H, st, theta, gamma, wavelength);
}

void dxrpt_host_spectrum_to_rgb(const dxrpt_host_hosek* H, const float spectrum[60], float rgb[3]) {
    spectrum_to_rgb(*H, spectrum, rgb);
}

void dxrpt_host_spectrum_from_rgb_reflectance(const dxrpt_host_hosek* H, const float rgb[3], float spectrum[60]) {
    spectrum_from_rgb_reflectance(*H, rgb, spectrum);
}

// SkyCache::Init (Skybox.cpp:48-215) with createCubemap = true; the SH / SG projections of the cube
// (:158-211) feed the raster path only and are not computed.
int dxrpt_host_sky_create_hosek(const dxrpt_host_hosek* H, const float sun_direction[3], float sun_size_deg,
                                float turbidity, const float ground_albedo[3], uint32_t res, uint16_t* out_cube,
                                float out_sun_irradiance[3], float out_sun_render_color[3]) {
    if (!H || !sun_direction || !ground_albedo || !out_sun_irradiance || !out_sun_render_color || (res && !out_cube)) {
        g_hosek_err = "dxrpt_host_sky_create_hosek: null argument";
        return -1;
    }
    F3 sunDirection{sun_direction[0], sun_direction[1], sun_direction[2]};
    F3 groundAlbedo{ground_albedo[0], ground_albedo[1], ground_albedo[2]};
    sunDirection.y = saturate(sunDirection.y);
    sunDirection = normalize(sunDirection);
    turbidity = std::min(std::max(turbidity, 1.0f), 32.0f);
    groundAlbedo = F3{saturate(groundAlbedo.x), saturate(groundAlbedo.y), saturate(groundAlbedo.z)};
    const float sunSize = std::max(sun_size_deg, 0.01f);
    // (:64-67, repeated after the up-to-date check)
    sunDirection.y = saturate(sunDirection.y);
    sunDirection = normalize(sunDirection);
    if (turbidity > 10.0f) {
        g_hosek_err = "dxrpt_host_sky_create_hosek: the solar radiance fit covers turbidity 1..10";
        return -1;
    }
    const F3 up{0.0f, 1.0f, 0.0f};
    const float thetaS = angle_between(sunDirection, up);
    const float elevation = kPi_2 - thetaS;
    HState stR, stG, stB;
    rgb_state(*H, stR, turbidity, groundAlbedo.x, elevation);
    rgb_state(*H, stG, turbidity, groundAlbedo.y, elevation);
    rgb_state(*H, stB, turbidity, groundAlbedo.z, elevation);

    // sun irradiance: 8 x 8 stratified samples of the 0.27-degree physical sun (:78-130)
    const float albedo3[3] = {groundAlbedo.x, groundAlbedo.y, groundAlbedo.z};
    float groundAlbedoSpectrum[kNumSpectral];
    spectrum_from_rgb_reflectance(*H, albedo3, groundAlbedoSpectrum);
    std::vector<HState> skyStates(kNumSpectral);
    for (int i = 0; i < kNumSpectral; ++i)  // the reference passes thetaS as the solar elevation (:84)
        spectral_state(*H, skyStates[i], thetaS, turbidity, groundAlbedoSpectrum[i]);
    F3 sunIrradiance{0.0f, 0.0f, 0.0f};
    const F3 sunDirX = perpendicular(sunDirection);
    const F3 sunDirY = cross(sunDirection, sunDirX);
    const float physicalSunSize = deg_to_rad(0.27f);  // Skybox.cpp:32-33
    const float cosPhysicalSunSize = std::cos(physicalSunSize);
    const uint64_t NumSamples = 8;
    for (uint64_t x = 0; x < NumSamples; ++x) {
        for (uint64_t y = 0; y < NumSamples; ++y) {
            const float u1 = (x + 0.5f) / NumSamples;
            const float u2 = (y + 0.5f) / NumSamples;
            // SampleDirectionCone (Graphics/Sampling.cpp:282-288)
            const float cosTheta = (1.0f - u1) + u1 * cosPhysicalSunSize;
            const float sinTheta = std::sqrt(1.0f - cosTheta * cosTheta);
            const float phi = u2 * 2.0f * kPi;
            F3 sampleDir{std::cos(phi) * sinTheta, std::sin(phi) * sinTheta, cosTheta};
            sampleDir = transform(sampleDir, sunDirX, sunDirY, sunDirection);
            const float sampleThetaS = angle_between(sampleDir, up);
            const float sampleGamma = angle_between(sampleDir, sunDirection);
            float solarRadiance[kNumSpectral];
            for (int i = 0; i < kNumSpectral; ++i) {
                const float wavelength = lerpf(float(kLambdaStart), float(kLambdaEnd), i / float(kNumSpectral));
                solarRadiance[i] = float(solar_radiance(*H, skyStates[i], sampleThetaS, sampleGamma, wavelength));
            }
            float rgb[3];
            spectrum_to_rgb(*H, solarRadiance, rgb);
            F3 sampleRadiance{rgb[0] * kFP16Scale, rgb[1] * kFP16Scale, rgb[2] * kFP16Scale};
            const float w = saturate(dot(sampleDir, sunDirection));
            sunIrradiance = F3{sunIrradiance.x + sampleRadiance.x * w, sunIrradiance.y + sampleRadiance.y * w,
                               sunIrradiance.z + sampleRadiance.z * w};
        }
    }
    const float pdf = 1.0f / (2.0f * kPi * (1.0f - cosPhysicalSunSize));  // SampleDirectionCone_PDF
    const float mc = (1.0f / NumSamples) * (1.0f / NumSamples) * (1.0f / pdf);
    sunIrradiance = F3{sunIrradiance.x * mc, sunIrradiance.y * mc, sunIrradiance.z * mc};
    const float lum = 683.0f * 100.0f;
    sunIrradiance = F3{sunIrradiance.x * lum, sunIrradiance.y * lum, sunIrradiance.z * lum};
    // (:140-154)
    const float st = std::sin(deg_to_rad(sunSize));
    const float integral = kPi * st * st;
    F3 sunColor{sunIrradiance.x / integral, sunIrradiance.y / integral, sunIrradiance.z / integral};
    const float maxc = std::max(sunColor.x, std::max(sunColor.y, sunColor.z));
    if (maxc > kFP16Max) sunColor = F3{sunColor.x * (kFP16Max / maxc), sunColor.y * (kFP16Max / maxc), sunColor.z * (kFP16Max / maxc)};
    out_sun_irradiance[0] = sunIrradiance.x;
    out_sun_irradiance[1] = sunIrradiance.y;
    out_sun_irradiance[2] = sunIrradiance.z;
    out_sun_render_color[0] = std::min(std::max(sunColor.x, 0.0f), kFP16Max);
    out_sun_render_color[1] = std::min(std::max(sunColor.y, 0.0f), kFP16Max);
    out_sun_render_color[2] = std::min(std::max(sunColor.z, 0.0f), kFP16Max);

    // cube: SkyCache::Sample per texel centre (:158-180, 252-270), FP16 texels, alpha 1
    for (uint64_t s = 0; s < 6; ++s)
        for (uint64_t y = 0; y < res; ++y)
            for (uint64_t x = 0; x < res; ++x) {
                const F3 dir = map_xys_to_direction(x, y, s, res, res);
                const float gamma = angle_between(dir, sunDirection);
                const float theta = angle_between(dir, up);
                float r = float(tristim_radiance(stR, theta, gamma, 0));
                float g = float(tristim_radiance(stG, theta, gamma, 1));
                float b = float(tristim_radiance(stB, theta, gamma, 2));
                r *= 683.0f;
                g *= 683.0f;
                b *= 683.0f;
                const size_t idx = ((s * res + y) * res + x) * 4u;
                out_cube[idx + 0] = dxrpt_host_float_to_half(r * kFP16Scale);
                out_cube[idx + 1] = dxrpt_host_float_to_half(g * kFP16Scale);
                out_cube[idx + 2] = dxrpt_host_float_to_half(b * kFP16Scale);
                out_cube[idx + 3] = dxrpt_host_float_to_half(1.0f);
            }
    return 0;
}

}  // extern "C"
