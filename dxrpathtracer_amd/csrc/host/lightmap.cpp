// lightmap.cpp — the bake's host-side inputs: lightmap UVs and the surface map.
//
// The reference unwraps the model with xatlas (Graphics/Model.cpp:608-715, a third-party library the
// image does not have) into a "lightmapped" copy of the mesh: new vertices per chart corner carrying
// LightmapUV, 32-bit indices, the meshes drawn in order.  dxrpt_host_lightmap_charts produces a mesh
// of the same shape with the simplest valid atlas (every triangle its own chart, two per grid cell);
// any caller-made atlas (xatlas output, an FBX's second UV set) works the same way.
//
// dxrpt_host_surface_map is RenderSurfaceMap (DXRPathTracer.cpp:1845-1893) with SurfaceMap.hlsl: the
// lightmapped mesh rasterised at LightmapUV (VSMain: clip = (2u - 1, 2(1 - v) - 1, 0.5, 1)), no culling,
// no depth test, no blending (DXRPathTracer.cpp:673-677), so the last triangle drawn over a texel
// wins; PSMain writes (WorldPos, 1) and (normalize(WorldNormal), 1).  Rasterisation follows the D3D
// rules: vertices snapped to 1/256 pixel, coverage sampled at pixel centres, the top-left fill rule;
// attributes are interpolated linearly (w = 1) with the barycentrics of the snapped triangle.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/dxrpt_host.h"

namespace {

// Edge function of (a -> b) at p, all in 1/256-pixel fixed point.
inline int64_t edge(int64_t ax, int64_t ay, int64_t bx, int64_t by, int64_t px, int64_t py) {
    return (bx - ax) * (py - ay) - (by - ay) * (px - ax);
}

// Top-left rule in the y-down raster, edges oriented so the interior is positive (edge() > 0): a
// "top" edge is horizontal with the interior below it (runs +x), a "left" edge runs up (-y).
inline bool top_left(int64_t ax, int64_t ay, int64_t bx, int64_t by) {
    const int64_t dx = bx - ax, dy = by - ay;
    return (dy == 0 && dx > 0) || dy < 0;
}

inline int64_t snap(float s) { return int64_t(std::nearbyint(double(s) * 256.0)); }

}  // namespace

extern "C" {

int dxrpt_host_lightmap_charts(const dxrpt_host_scene* scene, uint32_t resolution, dxrpt_mesh_vertex* out_vertices,
                               uint32_t* out_indices) {
    if (!scene || !out_vertices || !out_indices || resolution < 8) return DXRPT_E_INVALID_ARG;
    const uint64_t ntri = scene->num_indices / 3u;
    const uint64_t pairs = (ntri + 1u) / 2u;
    const uint32_t G = std::max<uint32_t>(1u, uint32_t(std::ceil(std::sqrt(double(pairs)))));
    const double cell = double(resolution) / double(G);
    if (cell < 4.0) return DXRPT_E_INVALID_ARG;  // charts smaller than 4 texels: resolution too low
    auto index = [&](uint64_t i) -> uint32_t {
        return scene->idx_bytes == 2 ? static_cast<const uint16_t*>(scene->indices)[i]
                                     : static_cast<const uint32_t*>(scene->indices)[i];
    };
    uint64_t t = 0;
    for (uint32_t g = 0; g < scene->num_geometries; ++g) {
        const dxrpt_geometry_info& gi = scene->geometries[g];
        const uint64_t end = g + 1 < scene->num_geometries ? scene->geometries[g + 1].IdxOffset / 3u : ntri;
        for (; t < end; ++t) {
            const uint64_t pair = t / 2u;
            const double x0 = double(pair % G) * cell, y0 = double(pair / G) * cell;
            // even triangle: lower-left half of the cell; odd: upper-right half; 1-2 texels of gutter
            double c[3][2];
            if ((t & 1u) == 0) {
                c[0][0] = x0 + 1.0;        c[0][1] = y0 + 1.0;
                c[1][0] = x0 + cell - 2.0; c[1][1] = y0 + 1.0;
                c[2][0] = x0 + 1.0;        c[2][1] = y0 + cell - 2.0;
            } else {
                c[0][0] = x0 + cell - 1.0; c[0][1] = y0 + cell - 1.0;
                c[1][0] = x0 + 2.0;        c[1][1] = y0 + cell - 1.0;
                c[2][0] = x0 + cell - 1.0; c[2][1] = y0 + 2.0;
            }
            for (int k = 0; k < 3; ++k) {
                dxrpt_mesh_vertex v = scene->vertices[index(t * 3u + uint64_t(k)) + gi.VtxOffset];
                v.LightmapUV[0] = float(c[k][0] / double(resolution));
                v.LightmapUV[1] = float(c[k][1] / double(resolution));
                out_vertices[t * 3u + uint64_t(k)] = v;
                out_indices[t * 3u + uint64_t(k)] = uint32_t(t * 3u + uint64_t(k));
            }
        }
    }
    return DXRPT_OK;
}

int dxrpt_host_surface_map(const dxrpt_mesh_vertex* vertices, uint32_t num_vertices, const uint32_t* indices,
                           uint32_t num_indices, uint32_t width, uint32_t height, float* out_pos, float* out_normal) {
    if (!vertices || !indices || !out_pos || !out_normal || width == 0 || height == 0 || width > 32768 || height > 32768)
        return DXRPT_E_INVALID_ARG;
    const size_t n = size_t(width) * height * 4u;
    std::memset(out_pos, 0, n * sizeof(float));  // ClearRenderTargetView(0, 0, 0, 0)
    std::memset(out_normal, 0, n * sizeof(float));
    for (uint32_t t = 0; t + 2 < num_indices; t += 3) {
        const dxrpt_mesh_vertex* v[3];
        int64_t X[3], Y[3];
        for (int k = 0; k < 3; ++k) {
            const uint32_t i = indices[t + uint32_t(k)];
            if (i >= num_vertices) return DXRPT_E_INVALID_ARG;
            v[k] = &vertices[i];
            // VSMain clip position, then the viewport transform to pixels
            const float cx = v[k]->LightmapUV[0] * 2.0f - 1.0f;
            const float cy = (1.0f - v[k]->LightmapUV[1]) * 2.0f - 1.0f;
            X[k] = snap((cx + 1.0f) * 0.5f * float(width));
            Y[k] = snap((1.0f - cy) * 0.5f * float(height));
        }
        int64_t area = edge(X[0], Y[0], X[1], Y[1], X[2], Y[2]);
        if (area == 0) continue;
        int a = 1, b = 2;  // orient so the interior is positive (no culling: both windings draw)
        if (area < 0) {
            std::swap(a, b);
            area = -area;
        }
        const int64_t minx = std::min({X[0], X[1], X[2]}), maxx = std::max({X[0], X[1], X[2]});
        const int64_t miny = std::min({Y[0], Y[1], Y[2]}), maxy = std::max({Y[0], Y[1], Y[2]});
        // pixel centres (px + 0.5) * 256 inside the box
        const int64_t px0 = std::max<int64_t>(0, (minx - 128 + 255) >> 8), px1 = std::min<int64_t>(width - 1, (maxx - 128) >> 8);
        const int64_t py0 = std::max<int64_t>(0, (miny - 128 + 255) >> 8), py1 = std::min<int64_t>(height - 1, (maxy - 128) >> 8);
        const bool tl0 = top_left(X[a], Y[a], X[b], Y[b]);  // edge opposite vertex 0
        const bool tl1 = top_left(X[b], Y[b], X[0], Y[0]);  // opposite a
        const bool tl2 = top_left(X[0], Y[0], X[a], Y[a]);  // opposite b
        for (int64_t py = py0; py <= py1; ++py)
            for (int64_t px = px0; px <= px1; ++px) {
                const int64_t sx = px * 256 + 128, sy = py * 256 + 128;
                const int64_t w0 = edge(X[a], Y[a], X[b], Y[b], sx, sy);
                const int64_t wa = edge(X[b], Y[b], X[0], Y[0], sx, sy);
                const int64_t wb = edge(X[0], Y[0], X[a], Y[a], sx, sy);
                if (w0 < 0 || wa < 0 || wb < 0) continue;
                if ((w0 == 0 && !tl0) || (wa == 0 && !tl1) || (wb == 0 && !tl2)) continue;
                float l[3];
                l[0] = float(double(w0) / double(area));
                l[a] = float(double(wa) / double(area));
                l[b] = float(double(wb) / double(area));
                float* P = out_pos + (size_t(py) * width + size_t(px)) * 4u;
                float* N = out_normal + (size_t(py) * width + size_t(px)) * 4u;
                float nn[3];
                for (int c = 0; c < 3; ++c) {
                    P[c] = (v[0]->Position[c] * l[0] + v[1]->Position[c] * l[1]) + v[2]->Position[c] * l[2];
                    nn[c] = (v[0]->Normal[c] * l[0] + v[1]->Normal[c] * l[1]) + v[2]->Normal[c] * l[2];
                }
                P[3] = 1.0f;
                const float len = std::sqrt((nn[0] * nn[0] + nn[1] * nn[1]) + nn[2] * nn[2]);
                N[0] = nn[0] / len;
                N[1] = nn[1] / len;
                N[2] = nn[2] / len;
                N[3] = 1.0f;
            }
    }
    return DXRPT_OK;
}

}  // extern "C"
