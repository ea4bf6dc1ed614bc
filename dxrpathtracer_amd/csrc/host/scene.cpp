// scene.cpp — host scene inputs: BoxTest (exact), WhiteFurnace/Sponza/SunTemple proxies, primitives.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <dlfcn.h>
#include <memory>
#include <mutex>
#include <string>

#include "scene_builder.h"

namespace dxrpt_host {

namespace {
thread_local std::string g_last_error;
// Packaged-asset directory (dxrpt_host_set_asset_dir); unset, it defaults to ../data next to this
// library (dxrpathtracer_amd/lib/libdxrpt_host.so -> dxrpathtracer_amd/data).
std::mutex g_asset_mutex;
std::string g_asset_dir;
bool g_asset_dir_set = false;

std::string default_asset_dir() {
    Dl_info info{};
    if (dladdr(reinterpret_cast<void*>(&dxrpt_host_set_asset_dir), &info) && info.dli_fname) {
        std::string lib = info.dli_fname;
        const size_t slash = lib.find_last_of('/');
        return (slash == std::string::npos ? std::string(".") : lib.substr(0, slash)) + "/../data";
    }
    return std::string();
}

struct SceneStore {
    dxrpt_host_scene pub{};
    SceneBuilder B;
    std::vector<uint16_t> idx16;
    std::vector<dxrpt_host_texture> views;
};

// Default 1x1 textures, Graphics/Model.cpp:74-82 -> Content/Textures/*.dds (B8G8R8X8_UNORM).
// Texel bytes read from the files (B,G,R,X): DefaultBaseColor c0 c0 c0, DefaultNormalMap ff 7f 7f,
// DefaultRoughness 40 40 40, DefaultBlack 00 00 00; X reads as alpha 1.
Texture default_base_color(bool srgb) { return solid_rgba(0xC0, 0xC0, 0xC0, 0xFF, srgb ? DXRPT_TEX_RGBA8_SRGB : DXRPT_TEX_RGBA8_UNORM); }
Texture default_normal() { return solid_rgba(0x7F, 0x7F, 0xFF, 0xFF); }
Texture default_roughness() { return solid_rgba(0x40, 0x40, 0x40, 0xFF); }
Texture default_black() { return solid_rgba(0x00, 0x00, 0x00, 0xFF); }

// Mesh::InitBox (Graphics/Model.cpp:235-343) with identity orientation:
// 24 vertices (4 per face: +y, -y, -z ("front"), +z ("back"), -x ("left"), +x ("right")), 36 indices
// (0,1,2, 2,3,0 per face); Position = corner * dimensions/2 + position.
void init_box(SceneBuilder& B, V3 dim, V3 pos, uint32_t material) {
    struct Cv { float p[3], n[3], uv[2], t[3], b[3]; };
    static const Cv k[24] = {
        // Top
        {{-1, 1, 1}, {0, 1, 0}, {0, 0}, {1, 0, 0}, {0, 0, -1}},
        {{1, 1, 1}, {0, 1, 0}, {1, 0}, {1, 0, 0}, {0, 0, -1}},
        {{1, 1, -1}, {0, 1, 0}, {1, 1}, {1, 0, 0}, {0, 0, -1}},
        {{-1, 1, -1}, {0, 1, 0}, {0, 1}, {1, 0, 0}, {0, 0, -1}},
        // Bottom
        {{-1, -1, -1}, {0, -1, 0}, {0, 0}, {1, 0, 0}, {0, 0, 1}},
        {{1, -1, -1}, {0, -1, 0}, {1, 0}, {1, 0, 0}, {0, 0, 1}},
        {{1, -1, 1}, {0, -1, 0}, {1, 1}, {1, 0, 0}, {0, 0, 1}},
        {{-1, -1, 1}, {0, -1, 0}, {0, 1}, {1, 0, 0}, {0, 0, 1}},
        // Front
        {{-1, 1, -1}, {0, 0, -1}, {0, 0}, {1, 0, 0}, {0, -1, 0}},
        {{1, 1, -1}, {0, 0, -1}, {1, 0}, {1, 0, 0}, {0, -1, 0}},
        {{1, -1, -1}, {0, 0, -1}, {1, 1}, {1, 0, 0}, {0, -1, 0}},
        {{-1, -1, -1}, {0, 0, -1}, {0, 1}, {1, 0, 0}, {0, -1, 0}},
        // Back
        {{1, 1, 1}, {0, 0, 1}, {0, 0}, {-1, 0, 0}, {0, -1, 0}},
        {{-1, 1, 1}, {0, 0, 1}, {1, 0}, {-1, 0, 0}, {0, -1, 0}},
        {{-1, -1, 1}, {0, 0, 1}, {1, 1}, {-1, 0, 0}, {0, -1, 0}},
        {{1, -1, 1}, {0, 0, 1}, {0, 1}, {-1, 0, 0}, {0, -1, 0}},
        // Left
        {{-1, 1, 1}, {-1, 0, 0}, {0, 0}, {0, 0, -1}, {0, -1, 0}},
        {{-1, 1, -1}, {-1, 0, 0}, {1, 0}, {0, 0, -1}, {0, -1, 0}},
        {{-1, -1, -1}, {-1, 0, 0}, {1, 1}, {0, 0, -1}, {0, -1, 0}},
        {{-1, -1, 1}, {-1, 0, 0}, {0, 1}, {0, 0, -1}, {0, -1, 0}},
        // Right
        {{1, 1, -1}, {1, 0, 0}, {0, 0}, {0, 0, 1}, {0, -1, 0}},
        {{1, 1, 1}, {1, 0, 0}, {1, 0}, {0, 0, 1}, {0, -1, 0}},
        {{1, -1, 1}, {1, 0, 0}, {1, 1}, {0, 0, 1}, {0, -1, 0}},
        {{1, -1, -1}, {1, 0, 0}, {0, 1}, {0, 0, 1}, {0, -1, 0}},
    };
    const V3 s = dim * 0.5f;
    B.begin_mesh(material);
    for (int i = 0; i < 24; ++i) {
        V3 p{k[i].p[0] * s.x, k[i].p[1] * s.y, k[i].p[2] * s.z};
        p = p + pos;
        B.vtx(p, V3{k[i].n[0], k[i].n[1], k[i].n[2]}, k[i].uv[0], k[i].uv[1], V3{k[i].t[0], k[i].t[1], k[i].t[2]},
              V3{k[i].b[0], k[i].b[1], k[i].b[2]});
    }
    for (uint32_t f = 0; f < 6; ++f) {
        B.tri(4 * f + 0, 4 * f + 1, 4 * f + 2);
        B.tri(4 * f + 2, 4 * f + 3, 4 * f + 0);
    }
    B.end_mesh();
}

// Model::GenerateBoxTestScene (Graphics/Model.cpp:761-780): one material whose albedo "White.png"
// and normal "Hex.png" do not exist in Content/Textures, so LoadMaterialResources (104-149) falls back
// to the default textures, forceSRGB = false.  Texture order = load order:
// 0 DefaultBaseColor, 1 DefaultNormalMap, 2 DefaultRoughness, 3 DefaultBlack (metallic + emissive).
void build_boxtest(SceneBuilder& B) {
    uint32_t t0 = B.add_texture(default_base_color(false));
    uint32_t t1 = B.add_texture(default_normal());
    uint32_t t2 = B.add_texture(default_roughness());
    uint32_t t3 = B.add_texture(default_black());
    uint32_t m = B.add_material(t0, t1, t2, t3, DXRPT_INVALID_INDEX, t3);
    init_box(B, V3{2.0f, 2.0f, 2.0f}, V3{0.0f, 1.5f, 0.0f}, m);
    init_box(B, V3{10.0f, 0.25f, 10.0f}, V3{0.0f, 0.0f, 0.0f}, m);
}

// WhiteFurnace scene: the reference loads Content/Models/WhiteFurnace/WhiteFurnace.fbx (1 mesh,
// 9,902 vertices); the FBX loader is SURVEY 8(f) next #1.  Proxy: a UV sphere of similar vertex count,
// default textures (the furnace mode ignores all textures except normal maps, RayTrace.hlsl:182-198).
void build_whitefurnace_proxy(SceneBuilder& B) {
    uint32_t t0 = B.add_texture(default_base_color(true));
    uint32_t t1 = B.add_texture(default_normal());
    uint32_t t2 = B.add_texture(default_roughness());
    uint32_t t3 = B.add_texture(default_black());
    uint32_t m = B.add_material(t0, t1, t2, t3, DXRPT_INVALID_INDEX, t3);
    const int seg = 110, rings = 89;
    const float R = 1.0f;
    B.begin_mesh(m);
    for (int j = 0; j <= rings; ++j) {
        float th = float(M_PI) * float(j) / rings;
        for (int i = 0; i <= seg; ++i) {
            float ph = 2.0f * float(M_PI) * float(i) / seg;
            V3 n{std::sin(th) * std::cos(ph), std::cos(th), std::sin(th) * std::sin(ph)};
            V3 t = normalize(V3{-std::sin(ph), 0.0f, std::cos(ph)});
            V3 b = normalize(cross(n, t));
            if (j == 0 || j == rings) b = V3{std::cos(ph), 0.0f, std::sin(ph)};
            B.vtx(n * R, n, float(i) / seg, float(j) / rings, t, b);
        }
    }
    for (int j = 0; j < rings; ++j)
        for (int i = 0; i < seg; ++i) {
            uint32_t a = j * (seg + 1) + i, b = a + 1, c = a + (seg + 1), d = c + 1;
            B.tri(a, c, b);
            B.tri(b, c, d);
        }
    B.end_mesh();
}

}  // namespace

// ---- primitives --------------------------------------------------------------------------------------
void SceneBuilder::grid(V3 o, V3 U, V3 V, V3 n, int nu, int nv, float us, float vs) {
    const V3 t = normalize(U), b = normalize(V);
    const uint32_t base = local_count();
    for (int j = 0; j <= nv; ++j)
        for (int i = 0; i <= nu; ++i) {
            float s = float(i) / nu, r = float(j) / nv;
            vtx(o + U * s + V * r, n, s * us, r * vs, t, b);
        }
    for (int j = 0; j < nv; ++j)
        for (int i = 0; i < nu; ++i) {
            uint32_t a = base + j * (nu + 1) + i, bb = a + 1, c = a + (nu + 1), d = c + 1;
            tri(a, bb, d);
            tri(d, c, a);
        }
}

void SceneBuilder::box(V3 lo, V3 hi, float uvs) {
    const V3 e = hi - lo;
    // +y, -y, +x, -x, +z, -z
    grid(V3{lo.x, hi.y, hi.z}, V3{e.x, 0, 0}, V3{0, 0, -e.z}, V3{0, 1, 0}, 1, 1, e.x * uvs, e.z * uvs);
    grid(V3{lo.x, lo.y, lo.z}, V3{e.x, 0, 0}, V3{0, 0, e.z}, V3{0, -1, 0}, 1, 1, e.x * uvs, e.z * uvs);
    grid(V3{hi.x, hi.y, lo.z}, V3{0, 0, e.z}, V3{0, -e.y, 0}, V3{1, 0, 0}, 1, 1, e.z * uvs, e.y * uvs);
    grid(V3{lo.x, hi.y, hi.z}, V3{0, 0, -e.z}, V3{0, -e.y, 0}, V3{-1, 0, 0}, 1, 1, e.z * uvs, e.y * uvs);
    grid(V3{hi.x, hi.y, hi.z}, V3{-e.x, 0, 0}, V3{0, -e.y, 0}, V3{0, 0, 1}, 1, 1, e.x * uvs, e.y * uvs);
    grid(V3{lo.x, hi.y, lo.z}, V3{e.x, 0, 0}, V3{0, -e.y, 0}, V3{0, 0, -1}, 1, 1, e.x * uvs, e.y * uvs);
}

void SceneBuilder::cylinder(V3 c, float r, float h, int seg, int rings, float flute_amp, int flutes, float uvs) {
    const uint32_t base = local_count();
    const float circ = 2.0f * float(M_PI) * r;
    for (int j = 0; j <= rings; ++j) {
        float y = h * float(j) / rings;
        for (int i = 0; i <= seg; ++i) {
            float ph = 2.0f * float(M_PI) * float(i) / seg;
            float rr = r * (1.0f - flute_amp * 0.5f * (1.0f - std::cos(ph * flutes)));
            float drr = -r * flute_amp * 0.5f * flutes * std::sin(ph * flutes);
            V3 dir{std::cos(ph), 0.0f, std::sin(ph)};
            V3 tang{-std::sin(ph), 0.0f, std::cos(ph)};
            // surface tangent along phi: d/dph (rr*dir) = drr*dir + rr*tang
            V3 dp = dir * drr + tang * rr;
            V3 t = normalize(dp);
            V3 n = normalize(cross(t, V3{0, 1, 0}));  // outward
            if (dot(n, dir) < 0) n = n * -1.0f;
            V3 b{0, 1, 0};
            vtx(c + dir * rr + V3{0, y, 0}, n, float(i) / seg * circ * uvs, y * uvs, t, b);
        }
    }
    for (int j = 0; j < rings; ++j)
        for (int i = 0; i < seg; ++i) {
            uint32_t a = base + j * (seg + 1) + i, b = a + 1, cc = a + (seg + 1), d = cc + 1;
            tri(a, cc, b);
            tri(b, cc, d);
        }
}

void SceneBuilder::arch(V3 centre, V3 axis, V3 depth_dir, float r_in, float r_out, float depth, int seg, float uvs) {
    const V3 up{0, 1, 0};
    const V3 a = normalize(axis), dd = normalize(depth_dir);
    // front/back faces (annulus), inner intrados, outer extrados
    for (int side = 0; side < 2; ++side) {
        const V3 off = dd * (side == 0 ? 0.0f : depth);
        const V3 n = side == 0 ? dd * -1.0f : dd;
        const uint32_t base = local_count();
        for (int i = 0; i <= seg; ++i) {
            float th = float(M_PI) * float(i) / seg;
            V3 dir = a * std::cos(th) + up * std::sin(th);
            V3 pin = centre + off + dir * r_in, pout = centre + off + dir * r_out;
            vtx(pin, n, dot(pin - centre, a) * uvs, pin.y * uvs, a, up);
            vtx(pout, n, dot(pout - centre, a) * uvs, pout.y * uvs, a, up);
        }
        for (int i = 0; i < seg; ++i) {
            uint32_t p0 = base + 2 * i, p1 = p0 + 1, p2 = p0 + 2, p3 = p0 + 3;
            if (side == 0) { tri(p0, p1, p3); tri(p3, p2, p0); }
            else { tri(p0, p3, p1); tri(p3, p0, p2); }
        }
    }
    for (int surf = 0; surf < 2; ++surf) {
        const float r = surf == 0 ? r_in : r_out;
        const uint32_t base = local_count();
        for (int i = 0; i <= seg; ++i) {
            float th = float(M_PI) * float(i) / seg;
            V3 dir = a * std::cos(th) + up * std::sin(th);
            V3 n = surf == 0 ? dir * -1.0f : dir;
            V3 t = normalize(a * -std::sin(th) + up * std::cos(th));
            for (int k = 0; k < 2; ++k) {
                V3 p = centre + dir * r + dd * (k * depth);
                vtx(p, n, th * r * uvs, k * depth * uvs, t, dd);
            }
        }
        for (int i = 0; i < seg; ++i) {
            uint32_t p0 = base + 2 * i, p1 = p0 + 1, p2 = p0 + 2, p3 = p0 + 3;
            if (surf == 0) { tri(p0, p2, p1); tri(p1, p2, p3); }
            else { tri(p0, p1, p2); tri(p2, p1, p3); }
        }
    }
}

void SceneBuilder::lathe(V3 c, const std::vector<std::pair<float, float>>& prof, int seg, float uvs) {
    const uint32_t base = local_count();
    const int np = int(prof.size());
    for (int j = 0; j < np; ++j) {
        const int jp = std::max(0, j - 1), jn = std::min(np - 1, j + 1);
        float dr = prof[jn].first - prof[jp].first, dy = prof[jn].second - prof[jp].second;
        for (int i = 0; i <= seg; ++i) {
            float ph = 2.0f * float(M_PI) * float(i) / seg;
            V3 dir{std::cos(ph), 0.0f, std::sin(ph)};
            V3 tang{-std::sin(ph), 0.0f, std::cos(ph)};
            V3 along = normalize(dir * dr + V3{0, dy, 0});
            V3 n = normalize(cross(tang, along));
            if (dot(n, dir) < 0 && prof[j].first > 0) n = n * -1.0f;
            vtx(c + dir * prof[j].first + V3{0, prof[j].second, 0}, n, float(i) / seg * 4.0f, prof[j].second * uvs, tang, along);
        }
    }
    for (int j = 0; j + 1 < np; ++j)
        for (int i = 0; i < seg; ++i) {
            uint32_t a = base + j * (seg + 1) + i, b = a + 1, cc = a + (seg + 1), d = cc + 1;
            tri(a, cc, b);
            tri(b, cc, d);
        }
}

void SceneBuilder::cloth(V3 top_left, V3 axis, float width, float height, int nu, int nv, float amp, float waves,
                         V3 normal_dir) {
    const V3 a = normalize(axis), nd = normalize(normal_dir);
    const uint32_t base = local_count();
    for (int j = 0; j <= nv; ++j) {
        float t = float(j) / nv;
        float sag = amp * (0.35f + 0.65f * t);
        for (int i = 0; i <= nu; ++i) {
            float s = float(i) / nu;
            float ph = 2.0f * float(M_PI) * waves * s;
            float off = sag * std::sin(ph);
            float doff = sag * 2.0f * float(M_PI) * waves * std::cos(ph) / width;
            V3 p = top_left + a * (s * width) + V3{0, -t * height, 0} + nd * off;
            V3 tx = normalize(a + nd * doff);
            V3 n = normalize(cross(V3{0, -1, 0}, tx));
            if (dot(n, nd) < 0) n = n * -1.0f;
            vtx(p, n, s * 2.0f, t * 3.0f, tx, V3{0, -1, 0});
        }
    }
    for (int j = 0; j < nv; ++j)
        for (int i = 0; i < nu; ++i) {
            uint32_t a0 = base + j * (nu + 1) + i, b = a0 + 1, c = a0 + (nu + 1), d = c + 1;
            tri(a0, b, d);
            tri(d, c, a0);
        }
}

}  // namespace dxrpt_host

namespace dxrpt_host {
size_t load_fbx_scene(const std::string& path, const std::string& texture_dir, float scene_scale, bool force_srgb,
                      SceneBuilder& B);
namespace {
// SceneCameraPositions / Rotations / SunDirections, DXRPathTracer.cpp:96-98 (index = Scenes enum)
const float kCamPos[DXRPT_SCENE_COUNT][3] = {{-11.5f, 1.85f, -0.45f}, {-1.0f, 5.5f, 12.0f}, {0.0f, 2.5f, -10.0f},
                                             {0.0f, 0.0f, -3.0f}, {0.0f, 0.0f, -30.0f}};
const float kCamRot[DXRPT_SCENE_COUNT][2] = {{0.0f, 1.544f}, {0.2f, 3.0f}, {0.0f, 0.0f}, {0.0f, 0.0f}, {0.0f, 0.0f}};
const float kSunDir[DXRPT_SCENE_COUNT][3] = {{0.26f, 0.987f, -0.16f}, {-0.133022308f, 0.642787635f, 0.75440651f},
                                             {0.26f, 0.987f, -0.16f}, {0.0f, 1.0f, 0.0f}, {-0.218f, 0.5f, -0.839f}};

// Fills the public view of a built scene.
void publish(SceneStore& St, uint32_t scene_id, uint64_t seed, bool idx16) {
    SceneBuilder& B = St.B;
    dxrpt_host_scene& P = St.pub;
    P.scene_id = scene_id;
    P.seed = seed;
    std::memcpy(P.camera_position, kCamPos[scene_id], sizeof(P.camera_position));
    std::memcpy(P.camera_rotation, kCamRot[scene_id], sizeof(P.camera_rotation));
    std::memcpy(P.sun_direction, kSunDir[scene_id], sizeof(P.sun_direction));
    P.white_furnace = scene_id == DXRPT_SCENE_WHITEFURNACE ? 1u : 0u;  // DXRPathTracer.cpp:935
    P.vertices = B.vertices.data();
    P.num_vertices = uint32_t(B.vertices.size());
    if (idx16) {
        St.idx16.assign(B.indices.begin(), B.indices.end());
        P.idx_bytes = 2;
        P.indices = St.idx16.data();
    } else {
        P.idx_bytes = 4;
        P.indices = B.indices.data();
    }
    P.num_indices = uint32_t(B.indices.size());
    P.geometries = B.geos.data();
    P.num_geometries = uint32_t(B.geos.size());
    P.materials = B.mats.data();
    P.num_materials = uint32_t(B.mats.size());
    St.views.resize(B.textures.size());
    for (size_t i = 0; i < B.textures.size(); ++i) {
        St.views[i].width = B.textures[i].w;
        St.views[i].height = B.textures[i].h;
        St.views[i].fmt = B.textures[i].fmt;
        St.views[i].texels = B.textures[i].data.data();
    }
    P.textures = St.views.data();
    P.num_textures = uint32_t(St.views.size());
    P.spot_lights = B.lights.empty() ? nullptr : B.lights.data();
    P.num_spot_lights = uint32_t(B.lights.size());
    P.num_triangles = B.indices.size() / 3;
    P.internal = &St;
}
}  // namespace

std::string asset_dir() {
    std::lock_guard<std::mutex> lock(g_asset_mutex);
    if (!g_asset_dir_set) {
        g_asset_dir = default_asset_dir();
        g_asset_dir_set = true;
    }
    return g_asset_dir;
}

}  // namespace dxrpt_host

using namespace dxrpt_host;

extern "C" {

const char* dxrpt_host_last_error(void) { return g_last_error.c_str(); }

int dxrpt_host_set_asset_dir(const char* dir) {
    if (!dir) return DXRPT_E_INVALID_ARG;
    std::lock_guard<std::mutex> lock(g_asset_mutex);
    g_asset_dir = dir;
    g_asset_dir_set = true;
    return DXRPT_OK;
}

int dxrpt_host_texture_load(const char* path, uint32_t force_srgb, dxrpt_host_texture* out) {
    if (!path || !out) return DXRPT_E_INVALID_ARG;
    std::memset(out, 0, sizeof(*out));
    Texture t;
    std::string err;
    if (!load_image(path, force_srgb != 0, t, err)) {
        g_last_error = err;
        return DXRPT_E_INVALID_ARG;
    }
    void* px = std::malloc(t.data.size());
    if (!px) {
        g_last_error = "dxrpt_host_texture_load: out of memory";
        return DXRPT_E_INVALID_ARG;
    }
    std::memcpy(px, t.data.data(), t.data.size());
    out->width = t.w;
    out->height = t.h;
    out->fmt = t.fmt;
    out->texels = px;
    return DXRPT_OK;
}

void dxrpt_host_texture_free(dxrpt_host_texture* tex) {
    if (!tex) return;
    std::free(const_cast<void*>(tex->texels));
    tex->texels = nullptr;
}

int dxrpt_host_scene_create(uint32_t scene_id, uint64_t seed, uint32_t detail, dxrpt_host_scene** out) {
    if (!out) return DXRPT_E_INVALID_ARG;
    *out = nullptr;
    try {
        std::unique_ptr<SceneStore> S(new SceneStore());
        SceneBuilder& B = S->B;
        switch (scene_id) {
            case DXRPT_SCENE_SPONZA: build_sponza_proxy(B, seed, detail); break;
            case DXRPT_SCENE_SUNTEMPLE: build_suntemple_proxy(B, seed, detail); break;
            case DXRPT_SCENE_BOXTEST: build_boxtest(B); break;
            case DXRPT_SCENE_WHITEFURNACE: build_whitefurnace_proxy(B); break;
            default: g_last_error = "dxrpt_host_scene_create: unknown scene id"; return DXRPT_E_INVALID_ARG;
        }
        // IndexType::Index16Bit for BoxTest (Model.cpp:770)
        publish(*S, scene_id, seed, scene_id == DXRPT_SCENE_BOXTEST);
        *out = &S.release()->pub;
        return DXRPT_OK;
    } catch (const std::bad_alloc&) {
        g_last_error = "dxrpt_host_scene_create: out of memory";
        return DXRPT_E_OOM;
    } catch (const std::exception& e) {  // e.g. a packaged asset that cannot be read
        g_last_error = e.what();
        return DXRPT_E_INVALID_ARG;
    }
}

int dxrpt_host_scene_load(uint32_t scene_id, const dxrpt_host_model_settings* settings, dxrpt_host_scene** out) {
    if (!out || !settings || !settings->file_path) return DXRPT_E_INVALID_ARG;
    *out = nullptr;
    try {
        if (scene_id >= DXRPT_SCENE_COUNT) {
            g_last_error = "dxrpt_host_scene_load: unknown scene id";
            return DXRPT_E_INVALID_ARG;
        }
        if (settings->merge_meshes) {
            g_last_error = "dxrpt_host_scene_load: MergeMeshes (PreTransformVertices) is not supported";
            return DXRPT_E_INVALID_ARG;
        }
        std::unique_ptr<SceneStore> S(new SceneStore());
        // ModelLoadSettings::TextureDir is relative to the model file's directory (Model.cpp:551)
        std::string path = settings->file_path;
        const size_t slash = path.find_last_of('/');
        std::string dir = slash == std::string::npos ? std::string() : path.substr(0, slash + 1);
        std::string tdir = dir;
        if (settings->texture_dir && settings->texture_dir[0]) {
            tdir = dir + settings->texture_dir;
            if (tdir.back() != '/') tdir += '/';
        }
        const size_t max_indices =
            load_fbx_scene(path, tdir, settings->scene_scale, settings->force_srgb != 0, S->B);
        publish(*S, scene_id, 0, max_indices <= 0xFFFF);  // Model.cpp:561-573
        *out = &S.release()->pub;
        return DXRPT_OK;
    } catch (const std::exception& e) {
        g_last_error = e.what();
        return DXRPT_E_INVALID_ARG;
    }
}

void dxrpt_host_scene_destroy(dxrpt_host_scene* scene) {
    if (!scene) return;
    delete static_cast<SceneStore*>(scene->internal);
}

}  // extern "C"
