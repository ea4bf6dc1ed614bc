// camera.cpp — FirstPersonCamera matrices and the RenderRayTracing constant fill.
//
// Graphics/Camera.cpp:202-229: orientation = XMQuaternionRotationRollPitchYaw(xRot, yRot, 0),
// world = rotation (rows right/up/forward) + translation, view = inverse(world),
// projection = XMMatrixPerspectiveFovLH(fov, aspect, near, far).  DXRPathTracer.cpp:2049 passes
// Float4x4::Invert(camera.ViewProjectionMatrix()).  DirectXMath is not available here; the matrices
// are evaluated in double and rounded once (the reference's float SIMD rounding is unpinned, and the
// matrix is an input that fixtures store verbatim).
#include <cmath>
#include <cstring>

#include "scene_builder.h"

namespace {

void mat_mul(const double a[16], const double b[16], double o[16]) {
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) {
            double s = 0;
            for (int k = 0; k < 4; ++k) s += a[r * 4 + k] * b[k * 4 + c];
            o[r * 4 + c] = s;
        }
}

bool mat_inv(const double m[16], double inv[16]) {
    double a[4][8];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 8; ++c) a[r][c] = c < 4 ? m[r * 4 + c] : (c - 4 == r ? 1.0 : 0.0);
    for (int c = 0; c < 4; ++c) {
        int p = c;
        for (int r = c + 1; r < 4; ++r)
            if (std::fabs(a[r][c]) > std::fabs(a[p][c])) p = r;
        if (a[p][c] == 0.0) return false;
        if (p != c)
            for (int k = 0; k < 8; ++k) std::swap(a[p][k], a[c][k]);
        double d = a[c][c];
        for (int k = 0; k < 8; ++k) a[c][k] /= d;
        for (int r = 0; r < 4; ++r) {
            if (r == c) continue;
            double f = a[r][c];
            for (int k = 0; k < 8; ++k) a[r][k] -= f * a[c][k];
        }
    }
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) inv[r * 4 + c] = a[r][c + 4];
    return true;
}

}  // namespace

extern "C" {

void dxrpt_host_inv_view_projection(const float position[3], float xrot, float yrot, float fov, float aspect,
                                    float nearz, float farz, float out[16]) {
    // FirstPersonCamera::SetXRotation clamps pitch to [-pi/2, pi/2] (Camera.cpp:219-223)
    double p = std::fmin(std::fmax(double(xrot), -M_PI / 2), M_PI / 2), y = double(yrot);
    double cp = std::cos(p), sp = std::sin(p), cy = std::cos(y), sy = std::sin(y);
    // Rows of Rx(pitch) * Ry(yaw) (row-vector convention, LH): right, up, forward
    double R[3] = {cy, 0.0, -sy};
    double U[3] = {sp * sy, cp, sp * cy};
    double F[3] = {cp * sy, -sp, cp * cy};
    double P[3] = {position[0], position[1], position[2]};
    double view[16] = {R[0], U[0], F[0], 0,
                       R[1], U[1], F[1], 0,
                       R[2], U[2], F[2], 0,
                       -(P[0] * R[0] + P[1] * R[1] + P[2] * R[2]),
                       -(P[0] * U[0] + P[1] * U[1] + P[2] * U[2]),
                       -(P[0] * F[0] + P[1] * F[1] + P[2] * F[2]), 1};
    double h = 1.0 / std::tan(0.5 * double(fov));
    double w = h / double(aspect);
    double q = double(farz) / (double(farz) - double(nearz));
    double proj[16] = {w, 0, 0, 0,
                       0, h, 0, 0,
                       0, 0, q, 1,
                       0, 0, -q * double(nearz), 0};
    double vp[16], inv[16];
    mat_mul(view, proj, vp);
    if (!mat_inv(vp, inv)) {
        std::memset(out, 0, 16 * sizeof(float));
        return;
    }
    for (int i = 0; i < 16; ++i) out[i] = float(inv[i]);
}

void dxrpt_host_fill_constants(const float inv_view_projection[16], const float camera_position[3],
                               const dxrpt_app_settings* s, const float sun_irradiance[3],
                               const float sun_render_color[3], uint32_t curr_sample_idx, uint32_t width,
                               uint32_t height, uint32_t num_lights, dxrpt_ray_trace_constants* out) {
    std::memset(out, 0, sizeof(*out));
    std::memcpy(out->InvViewProjection, inv_view_projection, 16 * sizeof(float));
    // AppSettings::SunDirection is a DirectionSetting: stored normalised (Settings.cpp:370, 519)
    double sx = s->SunDirection[0], sy = s->SunDirection[1], sz = s->SunDirection[2];
    double l = std::sqrt(sx * sx + sy * sy + sz * sz);
    out->SunDirectionWS[0] = float(sx / l);
    out->SunDirectionWS[1] = float(sy / l);
    out->SunDirectionWS[2] = float(sz / l);
    const double rad = double(s->SunSize) * M_PI / 180.0;  // DegToRad(SunSize), DXRPathTracer.cpp:2053-2054
    out->CosSunAngularRadius = float(std::cos(rad));
    out->SinSunAngularRadius = float(std::sin(rad));
    std::memcpy(out->SunIrradiance, sun_irradiance, 3 * sizeof(float));
    std::memcpy(out->SunRenderColor, sun_render_color, 3 * sizeof(float));
    std::memcpy(out->CameraPosWS, camera_position, 3 * sizeof(float));
    out->CurrSampleIdx = curr_sample_idx;
    out->TotalNumPixels = width * height;
    out->VtxBufferIdx = out->IdxBufferIdx = out->GeometryInfoBufferIdx = out->MaterialBufferIdx = out->SkyTextureIdx = 0;
    out->NumLights = num_lights;
}

}  // extern "C"
