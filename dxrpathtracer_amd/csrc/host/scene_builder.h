// scene_builder.h — internal mesh/material/texture accumulation for the host scene generators.
#pragma once
#include <stdint.h>

#include <cmath>
#include <string>
#include <vector>

#include "../../../include/dxrpt.h"
#include "../../../include/dxrpt_host.h"

namespace dxrpt_host {

struct V3 {
    float x = 0, y = 0, z = 0;
    V3() = default;
    V3(float a, float b, float c) : x(a), y(b), z(c) {}
};
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 operator*(float s, V3 a) { return {a.x * s, a.y * s, a.z * s}; }
inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline V3 normalize(V3 a) {
    float l = std::sqrt(dot(a, a));
    return l > 0 ? a * (1.0f / l) : a;
}

struct Texture {
    uint32_t w = 1, h = 1, fmt = DXRPT_TEX_RGBA8_UNORM;
    std::vector<uint8_t> data;
};

// splitmix64: the only RNG of the proxies.
struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed) {}
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    float uniform() { return float(next() >> 40) * (1.0f / 16777216.0f); }
    float range(float a, float b) { return a + (b - a) * uniform(); }
};

struct SceneBuilder {
    std::vector<dxrpt_mesh_vertex> vertices;
    std::vector<uint32_t> indices;
    std::vector<dxrpt_geometry_info> geos;
    std::vector<dxrpt_material> mats;
    std::vector<Texture> textures;
    std::vector<dxrpt_spot_light> lights;
    // current mesh
    uint32_t cur_vtx = 0, cur_idx = 0, cur_mat = 0;
    bool in_mesh = false;

    uint32_t add_texture(Texture&& t) {
        textures.push_back(std::move(t));
        return uint32_t(textures.size() - 1);
    }
    uint32_t add_material(uint32_t albedo, uint32_t normal, uint32_t rough, uint32_t metal, uint32_t opacity,
                          uint32_t emissive) {
        dxrpt_material m{albedo, normal, rough, metal, opacity, emissive};
        mats.push_back(m);
        return uint32_t(mats.size() - 1);
    }
    void begin_mesh(uint32_t material) {
        cur_vtx = uint32_t(vertices.size());
        cur_idx = uint32_t(indices.size());
        cur_mat = material;
        in_mesh = true;
    }
    uint32_t local_count() const { return uint32_t(vertices.size()) - cur_vtx; }
    // Returns the mesh-local index of the new vertex.
    uint32_t vtx(V3 p, V3 n, float u, float v, V3 t, V3 b) {
        dxrpt_mesh_vertex mv{};
        mv.Position[0] = p.x; mv.Position[1] = p.y; mv.Position[2] = p.z;
        mv.Normal[0] = n.x; mv.Normal[1] = n.y; mv.Normal[2] = n.z;
        mv.UV[0] = u; mv.UV[1] = v;
        mv.Tangent[0] = t.x; mv.Tangent[1] = t.y; mv.Tangent[2] = t.z;
        mv.Bitangent[0] = b.x; mv.Bitangent[1] = b.y; mv.Bitangent[2] = b.z;
        vertices.push_back(mv);
        return uint32_t(vertices.size()) - 1 - cur_vtx;
    }
    void tri(uint32_t a, uint32_t b, uint32_t c) {
        indices.push_back(a);
        indices.push_back(b);
        indices.push_back(c);
    }
    void end_mesh() {
        if (indices.size() > cur_idx) {
            dxrpt_geometry_info g{cur_vtx, cur_idx, cur_mat, 0};
            geos.push_back(g);
        } else {
            vertices.resize(cur_vtx);
        }
        in_mesh = false;
    }

    // ---- primitives (all emit into the current mesh) ---------------------------------------------
    // Planar grid: P(s,t) = o + s*U + t*V, s,t in [0,1]; normal n; nu x nv quads; uv = (s*us, t*vs).
    void grid(V3 o, V3 U, V3 V, V3 n, int nu, int nv, float us, float vs);
    // Axis-aligned box with outward faces, uv scaled by `uvs` per metre.
    void box(V3 lo, V3 hi, float uvs);
    // Cylinder along +y: base centre c, radius r, height h, seg x rings, optional flutes (amplitude).
    void cylinder(V3 c, float r, float h, int seg, int rings, float flute_amp, int flutes, float uvs);
    // Arch: half annulus in the plane spanned by `axis` (horizontal) and +y, extruded along `depth_dir`.
    void arch(V3 centre, V3 axis, V3 depth_dir, float r_in, float r_out, float depth, int seg, float uvs);
    // Surface of revolution around +y through profile points (radius, height).
    void lathe(V3 c, const std::vector<std::pair<float, float>>& prof, int seg, float uvs);
    // Hanging cloth: a width x height sheet in the plane (axis, -y), waves along axis; double-sided
    // is NOT emitted (the reference's geometry is single-sheet, culling is off).
    void cloth(V3 top_left, V3 axis, float width, float height, int nu, int nv, float amp, float waves, V3 normal_dir);
};

// textures.cpp
Texture solid_rgba(uint8_t r, uint8_t g, uint8_t b, uint8_t a, uint32_t fmt = DXRPT_TEX_RGBA8_UNORM);
Texture solid_r8(uint8_t v);
enum class Pattern { StoneTiles, Bricks, Marble, Plaster, Fabric, Wood, Metal, Leaves, Ceramic, Roof };
struct MaterialTextures {
    Texture albedo, normal, roughness, metallic, opacity;
};
MaterialTextures make_material_textures(Pattern p, uint64_t seed, uint32_t size, float r, float g, float b,
                                        float rough_base, float metal, bool with_opacity);




// sponza_proxy.cpp
void build_sponza_proxy(SceneBuilder& B, uint64_t seed, uint32_t detail);
void build_suntemple_proxy(SceneBuilder& B, uint64_t seed, uint32_t detail);

// Texture files (dds.cpp, image.cpp): LoadTexture's decoders (Graphics/Textures.cpp:38-172).
bool load_dds(const std::string& path, bool srgb, Texture& tex, std::string& err);
bool load_png(const std::string& path, bool srgb, Texture& tex, std::string& err);
bool load_jpeg(const std::string& path, bool srgb, Texture& tex, std::string& err);
bool load_image(const std::string& path, bool srgb, Texture& tex, std::string& err);  // by file signature

// Packaged assets (dxrpt_host_set_asset_dir): the directory holding suntemple/*.r8z.
std::string asset_dir();
// An R8 image stored as "DXR8", u32 width, u32 height, zlib stream of width*height bytes.
bool load_r8z(const std::string& path, Texture& tex, std::string& err);

}  // namespace dxrpt_host
