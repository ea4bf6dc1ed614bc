// sponza_proxy.cpp — seeded procedural stand-ins for the absent Sponza / SunTemple assets.
//
// The reference renders Content/Models/Sponza/Sponza_NoSpotLight.fbx (DXRPathTracer.cpp:86, scale
// 0.01) and SunTemple.fbx (scale 0.005); both files are stripped from the snapshot
// (.MISSING_LARGE_BLOBS:1-4).  These generators build scenes of the same role and scale for the
// same camera poses (DXRPathTracer.cpp:96-98): a two-storey colonnaded atrium open to the sky with
// arches, balconies, drapes and alpha-tested plants (~0.26 M triangles, ~20 materials, no spot
// lights), and a pillared temple hall with alpha-tested foliage.  All randomness comes from
// splitmix64 seeded with `seed` (default 0x53504F4E5A41, "SPONZA").
#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <string>

#include "scene_builder.h"

namespace dxrpt_host {

namespace {

struct Mat {
    uint32_t id;
};

uint32_t add_pbr(SceneBuilder& B, Pattern p, uint64_t seed, uint32_t size, float r, float g, float b, float rough,
                 float metal, bool alpha, uint32_t black) {
    MaterialTextures t = make_material_textures(p, seed, size, r, g, b, rough, metal, alpha);
    uint32_t ia = B.add_texture(std::move(t.albedo));
    uint32_t in = B.add_texture(std::move(t.normal));
    uint32_t ir = B.add_texture(std::move(t.roughness));
    uint32_t im = B.add_texture(std::move(t.metallic));
    uint32_t io = alpha ? B.add_texture(std::move(t.opacity)) : DXRPT_INVALID_INDEX;
    return B.add_material(ia, in, ir, im, io, black);
}

// A PBR material whose opacity map is a packaged asset (asset_dir()/<file>, an .r8z R8 image).
uint32_t add_pbr_asset_opacity(SceneBuilder& B, Pattern p, uint64_t seed, uint32_t size, float r, float g, float b,
                               float rough, float metal, const char* file, uint32_t black) {
    MaterialTextures t = make_material_textures(p, seed, size, r, g, b, rough, metal, false);
    Texture op;
    std::string err;
    const std::string dir = asset_dir();
    const std::string path = dir + "/suntemple/" + file;
    if (dir.empty() || !load_r8z(path, op, err))
        throw std::runtime_error("SunTemple proxy: cannot load the packaged opacity map " + path +
                                 " (default: ../data next to libdxrpt_host.so; dxrpt_host_set_asset_dir overrides): " + err);
    uint32_t ia = B.add_texture(std::move(t.albedo));
    uint32_t in = B.add_texture(std::move(t.normal));
    uint32_t ir = B.add_texture(std::move(t.roughness));
    uint32_t im = B.add_texture(std::move(t.metallic));
    uint32_t io = B.add_texture(std::move(op));
    return B.add_material(ia, in, ir, im, io, black);
}

int scaled(int base, uint32_t detail) { return detail == 0 ? base : std::max(3, int(base * detail / 4)); }

// A leaf card: a subdivided quad facing `n`, centred at c, size w x h, slight curl.
void leaf_card(SceneBuilder& B, V3 c, V3 right, V3 up, float w, float h, int sub, float curl) {
    const V3 n = normalize(cross(right, up));
    const uint32_t base = B.local_count();
    for (int j = 0; j <= sub; ++j)
        for (int i = 0; i <= sub; ++i) {
            float s = float(i) / sub - 0.5f, t = float(j) / sub - 0.5f;
            float bend = curl * (s * s * 4.0f);
            V3 p = c + right * (s * w) + up * (t * h) + n * bend;
            B.vtx(p, n, float(i) / sub, float(j) / sub, normalize(right), normalize(up));
        }
    for (int j = 0; j < sub; ++j)
        for (int i = 0; i < sub; ++i) {
            uint32_t a = base + j * (sub + 1) + i, b = a + 1, cc = a + (sub + 1), d = cc + 1;
            B.tri(a, b, d);
            B.tri(d, cc, a);
        }
}

void plant(SceneBuilder& B, Rng& rng, V3 base, uint32_t vase_mat, uint32_t leaf_mat, int seg, int cards, int sub) {
    std::vector<std::pair<float, float>> prof;
    const int np = 24;
    for (int k = 0; k < np; ++k) {
        float t = float(k) / (np - 1);
        float r = 0.25f + 0.18f * std::sin(t * 3.14159f) - 0.08f * t + (k == np - 1 ? 0.04f : 0.0f);
        prof.push_back({r, t * 0.9f});
    }
    prof.push_back({0.2f, 0.9f});
    B.begin_mesh(vase_mat);
    B.lathe(base, prof, seg, 1.0f);
    B.end_mesh();
    B.begin_mesh(leaf_mat);
    for (int k = 0; k < cards; ++k) {
        float ang = rng.range(0.0f, 6.2831853f);
        float tilt = rng.range(0.2f, 1.0f);
        float len = rng.range(0.5f, 0.9f);
        V3 dir{std::cos(ang), 0.0f, std::sin(ang)};
        V3 right = normalize(cross(V3{0, 1, 0}, dir));
        V3 up = normalize(dir * std::sin(tilt) + V3{0, 1, 0} * std::cos(tilt));
        V3 c = base + V3{0, 0.9f, 0} + up * (len * 0.5f) + dir * 0.1f;
        leaf_card(B, c, right, up, 0.45f, len, sub, 0.05f);
    }
    B.end_mesh();
}

}  // namespace

void build_sponza_proxy(SceneBuilder& B, uint64_t seed, uint32_t detail) {
    Rng rng(seed);
    const uint32_t TS = 512;
    const uint32_t black = B.add_texture(solid_rgba(0, 0, 0, 255));  // DefaultBlack emissive
    // ~20 materials (Sponza has 25 in the reference asset set)
    const uint32_t mFloor = add_pbr(B, Pattern::StoneTiles, rng.next(), TS, 0.62f, 0.58f, 0.52f, 0.75f, 0.0f, false, black);
    const uint32_t mColumn = add_pbr(B, Pattern::Marble, rng.next(), TS, 0.85f, 0.82f, 0.76f, 0.45f, 0.0f, false, black);
    const uint32_t mColumnB = add_pbr(B, Pattern::Plaster, rng.next(), TS, 0.70f, 0.66f, 0.58f, 0.7f, 0.0f, false, black);
    const uint32_t mArch = add_pbr(B, Pattern::Bricks, rng.next(), TS, 0.66f, 0.50f, 0.38f, 0.8f, 0.0f, false, black);
    const uint32_t mWall = add_pbr(B, Pattern::Plaster, rng.next(), TS, 0.78f, 0.72f, 0.62f, 0.85f, 0.0f, false, black);
    const uint32_t mWall2 = add_pbr(B, Pattern::Bricks, rng.next(), TS, 0.72f, 0.62f, 0.50f, 0.85f, 0.0f, false, black);
    const uint32_t mCeil = add_pbr(B, Pattern::Wood, rng.next(), TS, 0.45f, 0.32f, 0.22f, 0.6f, 0.0f, false, black);
    const uint32_t mRoof = add_pbr(B, Pattern::Roof, rng.next(), TS, 0.55f, 0.30f, 0.22f, 0.7f, 0.0f, false, black);
    const uint32_t mRed = add_pbr(B, Pattern::Fabric, rng.next(), TS, 0.62f, 0.08f, 0.07f, 0.9f, 0.0f, false, black);
    const uint32_t mGreen = add_pbr(B, Pattern::Fabric, rng.next(), TS, 0.10f, 0.45f, 0.15f, 0.9f, 0.0f, false, black);
    const uint32_t mBlue = add_pbr(B, Pattern::Fabric, rng.next(), TS, 0.10f, 0.18f, 0.55f, 0.9f, 0.0f, false, black);
    const uint32_t mVase = add_pbr(B, Pattern::Ceramic, rng.next(), TS, 0.55f, 0.35f, 0.25f, 0.35f, 0.0f, false, black);
    const uint32_t mLeaf = add_pbr(B, Pattern::Leaves, rng.next(), TS, 0.20f, 0.45f, 0.12f, 0.7f, 0.0f, true, black);
    const uint32_t mBalus = add_pbr(B, Pattern::Marble, rng.next(), TS, 0.80f, 0.78f, 0.72f, 0.5f, 0.0f, false, black);
    const uint32_t mMetal = add_pbr(B, Pattern::Metal, rng.next(), 256, 0.75f, 0.62f, 0.40f, 0.35f, 1.0f, false, black);
    const uint32_t mSlab = add_pbr(B, Pattern::StoneTiles, rng.next(), TS, 0.55f, 0.52f, 0.48f, 0.8f, 0.0f, false, black);
    const uint32_t mDark = add_pbr(B, Pattern::Plaster, rng.next(), TS, 0.35f, 0.32f, 0.30f, 0.9f, 0.0f, false, black);
    const uint32_t mGold = add_pbr(B, Pattern::Metal, rng.next(), 256, 0.95f, 0.78f, 0.35f, 0.25f, 1.0f, false, black);
    const uint32_t mStoneB = add_pbr(B, Pattern::Bricks, rng.next(), TS, 0.60f, 0.58f, 0.55f, 0.85f, 0.0f, false, black);
    const uint32_t mPlinth = add_pbr(B, Pattern::Marble, rng.next(), TS, 0.50f, 0.48f, 0.45f, 0.4f, 0.0f, false, black);

    const float X0 = -18.0f, X1 = 18.0f, Z1 = 9.0f, ZC = 4.0f;
    const float H1 = 5.7f, H1t = 6.0f, H2 = 11.0f, H2t = 11.3f, HW = 12.5f;
    // ---- floor (courtyard + aisles)
    B.begin_mesh(mFloor);
    B.grid(V3{X0, 0.0f, Z1}, V3{X1 - X0, 0, 0}, V3{0, 0, -2 * Z1}, V3{0, 1, 0}, scaled(128, detail), scaled(64, detail), 24.0f, 12.0f);
    B.end_mesh();
    // ---- outer walls
    B.begin_mesh(mWall);
    B.grid(V3{X0, HW, Z1}, V3{X1 - X0, 0, 0}, V3{0, -HW, 0}, V3{0, 0, -1}, 36, 12, 12.0f, 4.0f);   // z = +9 facing -z
    B.grid(V3{X1, HW, -Z1}, V3{X0 - X1, 0, 0}, V3{0, -HW, 0}, V3{0, 0, 1}, 36, 12, 12.0f, 4.0f);   // z = -9 facing +z
    B.end_mesh();
    B.begin_mesh(mWall2);
    B.grid(V3{X1, HW, Z1}, V3{0, 0, -2 * Z1}, V3{0, -HW, 0}, V3{-1, 0, 0}, 18, 12, 6.0f, 4.0f);   // east end
    B.grid(V3{X0, HW, -Z1}, V3{0, 0, 2 * Z1}, V3{0, -HW, 0}, V3{1, 0, 0}, 18, 12, 6.0f, 4.0f);    // west end
    B.end_mesh();
    // ---- first-floor slabs, balconies and roofs over both aisles (courtyard open to the sky)
    for (int side = -1; side <= 1; side += 2) {
        const float za = side * ZC, zb = side * Z1;
        const float zlo = std::min(za, zb), zhi = std::max(za, zb);
        B.begin_mesh(mSlab);
        B.box(V3{X0, H1, zlo - (side < 0 ? 0.0f : 0.6f)}, V3{X1, H1t, zhi + (side < 0 ? 0.6f : 0.0f)}, 0.5f);
        B.end_mesh();
        B.begin_mesh(mCeil);
        B.box(V3{X0, H2, zlo}, V3{X1, H2t, zhi}, 0.5f);
        B.end_mesh();
        B.begin_mesh(mRoof);
        B.grid(V3{X0, H2t + 1.2f, za}, V3{X1 - X0, 0, 0}, V3{0, -1.2f, zb - za}, normalize(V3{0, 1.0f, side * 1.2f / (Z1 - ZC)}), 36, 4, 12.0f, 3.0f);
        B.end_mesh();
        // wall band above the upper arches
        B.begin_mesh(mStoneB);
        B.box(V3{X0, 10.2f, za - 0.45f}, V3{X1, H2t + 1.2f, za + 0.45f}, 0.5f);
        B.box(V3{X0, 4.5f + 1.2f - 0.5f, za - 0.45f}, V3{X1, H1, za + 0.45f}, 0.5f);
        B.end_mesh();
    }
    // ---- colonnades: ground floor (fluted marble) and upper floor, arches between columns
    const int ncol = 11;
    const float spacing = 2.4f;
    const int segG = scaled(48, detail), ringsG = scaled(32, detail);
    const int segU = scaled(40, detail), ringsU = scaled(24, detail);
    for (int side = -1; side <= 1; side += 2) {
        const float z = side * ZC;
        for (int c = 0; c < ncol; ++c) {
            const float x = -12.0f + spacing * c;
            B.begin_mesh(mColumn);
            B.cylinder(V3{x, 0.35f, z}, 0.42f, 4.3f, segG, ringsG, 0.08f, 16, 0.6f);
            B.end_mesh();
            B.begin_mesh(mPlinth);
            std::vector<std::pair<float, float>> basep = {{0.0f, 0.0f}, {0.62f, 0.0f}, {0.62f, 0.18f}, {0.52f, 0.24f}, {0.48f, 0.30f}, {0.44f, 0.36f}, {0.42f, 0.36f}};
            B.lathe(V3{x, 0.0f, z}, basep, segG, 1.0f);
            std::vector<std::pair<float, float>> capp = {{0.42f, 4.65f}, {0.46f, 4.72f}, {0.55f, 4.85f}, {0.62f, 4.95f}, {0.66f, 5.05f}, {0.66f, 5.2f}, {0.0f, 5.2f}};
            B.lathe(V3{x, 0.0f, z}, capp, segG, 1.0f);
            B.end_mesh();
            B.begin_mesh(mColumnB);
            B.cylinder(V3{x, H1t, z}, 0.28f, 3.8f, segU, ringsU, 0.0f, 1, 0.6f);
            std::vector<std::pair<float, float>> capu = {{0.28f, H1t + 3.8f}, {0.34f, H1t + 3.9f}, {0.42f, H1t + 4.05f}, {0.42f, H1t + 4.2f}, {0.0f, H1t + 4.2f}};
            B.lathe(V3{x, 0.0f, z}, capu, segU, 1.0f);
            B.end_mesh();
            if (c + 1 < ncol) {
                B.begin_mesh(mArch);
                B.arch(V3{x + spacing * 0.5f, 5.2f, z - 0.45f}, V3{1, 0, 0}, V3{0, 0, 1}, 0.78f, 1.2f, 0.9f, scaled(48, detail), 0.5f);
                B.arch(V3{x + spacing * 0.5f, H1t + 4.2f, z - 0.45f}, V3{1, 0, 0}, V3{0, 0, 1}, 0.78f, 1.2f, 0.9f, scaled(48, detail), 0.5f);
                B.end_mesh();
            }
        }
        // balustrade on the first floor edge
        B.begin_mesh(mBalus);
        const int nb = 60;
        const int bseg = scaled(16, detail);
        for (int k = 0; k < nb; ++k) {
            const float x = -13.0f + 26.0f * (k + 0.5f) / nb;
            std::vector<std::pair<float, float>> bp = {{0.0f, H1t}, {0.09f, H1t}, {0.09f, H1t + 0.08f}, {0.06f, H1t + 0.2f}, {0.1f, H1t + 0.45f},
                                                       {0.07f, H1t + 0.7f}, {0.05f, H1t + 0.85f}, {0.09f, H1t + 0.95f}, {0.0f, H1t + 0.95f}};
            B.lathe(V3{x, 0.0f, side * (ZC + 0.2f)}, bp, bseg, 1.0f);
        }
        B.box(V3{-13.0f, H1t + 0.95f, side * (ZC + 0.2f) - 0.15f}, V3{13.0f, H1t + 1.1f, side * (ZC + 0.2f) + 0.15f}, 1.0f);
        B.end_mesh();
        // drapes hanging from the upper floor into the courtyard side of the aisle
        const uint32_t drape[3] = {mRed, mGreen, mBlue};
        for (int k = 0; k < 5; ++k) {
            const float x = -10.8f + spacing * 2 * k + 0.35f;
            B.begin_mesh(drape[(k + (side > 0 ? 1 : 0)) % 3]);
            B.cloth(V3{x, H2 - 0.3f, side * (ZC + 0.9f)}, V3{1, 0, 0}, 1.6f, 4.6f, scaled(48, detail), scaled(32, detail), 0.12f, 3.0f,
                    V3{0, 0, float(-side)});
            B.end_mesh();
        }
        // wall niches with bronze sconces along the aisle walls
        for (int k = 0; k < 12; ++k) {
            const float x = -16.5f + 3.0f * k;
            B.begin_mesh(mDark);
            B.box(V3{x - 0.6f, 1.5f, side * Z1 - (side > 0 ? 0.25f : 0.0f)}, V3{x + 0.6f, 3.5f, side * Z1 + (side < 0 ? 0.25f : 0.0f)}, 1.0f);
            B.end_mesh();
            B.begin_mesh(mGold);
            B.cylinder(V3{x, 2.2f, side * (Z1 - 0.45f)}, 0.08f, 0.6f, scaled(24, detail), 4, 0.0f, 1, 1.0f);
            B.end_mesh();
        }
    }
    // ---- far (east) wall decoration: big arch + metal chains hanging in the courtyard
    B.begin_mesh(mArch);
    B.arch(V3{X1 - 0.8f, 6.5f, -3.0f}, V3{0, 0, 1}, V3{1, 0, 0}, 2.4f, 3.0f, 0.8f, scaled(64, detail), 0.5f);
    B.end_mesh();
    B.begin_mesh(mMetal);
    for (int k = 0; k < 6; ++k) {
        const float x = -10.0f + 4.0f * k;
        B.cylinder(V3{x, 7.5f, 0.0f}, 0.025f, 5.0f, scaled(12, detail), 24, 0.0f, 1, 1.0f);
        B.cylinder(V3{x, 7.0f, 0.0f}, 0.35f, 0.5f, scaled(32, detail), 4, 0.0f, 1, 1.0f);
    }
    B.end_mesh();
    // ---- plants in vases along the courtyard (alpha-tested leaves, the any-hit path)
    for (int k = 0; k < 8; ++k) {
        const float x = -10.5f + 3.0f * k;
        const float z = (k & 1) ? 2.8f : -2.8f;
        plant(B, rng, V3{x, 0.0f, z}, mVase, mLeaf, scaled(48, detail), 48, scaled(4, detail));
    }
}

void build_suntemple_proxy(SceneBuilder& B, uint64_t seed, uint32_t detail) {
    Rng rng(seed ^ 0x53554E54454D50ull);  // "SUNTEMP"
    const uint32_t TS = 512;
    const uint32_t black = B.add_texture(solid_rgba(0, 0, 0, 255));
    const uint32_t mFloor = add_pbr(B, Pattern::Marble, rng.next(), TS, 0.55f, 0.50f, 0.45f, 0.35f, 0.0f, false, black);
    const uint32_t mWall = add_pbr(B, Pattern::Bricks, rng.next(), TS, 0.70f, 0.58f, 0.45f, 0.8f, 0.0f, false, black);
    const uint32_t mPillar = add_pbr(B, Pattern::Marble, rng.next(), TS, 0.80f, 0.74f, 0.62f, 0.4f, 0.0f, false, black);
    const uint32_t mRoof = add_pbr(B, Pattern::Wood, rng.next(), TS, 0.35f, 0.25f, 0.18f, 0.7f, 0.0f, false, black);
    const uint32_t mGold = add_pbr(B, Pattern::Metal, rng.next(), 256, 0.95f, 0.75f, 0.30f, 0.3f, 1.0f, false, black);
    // foliage: procedural albedo / normal / roughness, the reference's own BC4 opacity maps (SURVEY.md
    // 8(d): Content/Models/SunTemple/Textures, packaged by scripts/make_suntemple_opacity.py)
    const uint32_t mLeafA = add_pbr_asset_opacity(B, Pattern::Leaves, rng.next(), TS, 0.25f, 0.40f, 0.10f, 0.7f, 0.0f,
                                                  "T_M_Tree_Branches_0_A.r8z", black);
    const uint32_t mLeafB = add_pbr_asset_opacity(B, Pattern::Leaves, rng.next(), TS, 0.45f, 0.35f, 0.10f, 0.7f, 0.0f,
                                                  "T_Soul_Tree011M_Inst_0_A.r8z", black);
    const uint32_t mBark = add_pbr(B, Pattern::Wood, rng.next(), TS, 0.30f, 0.22f, 0.15f, 0.9f, 0.0f, false, black);
    const float X = 9.0f, Z0 = -24.0f, Z1 = 16.0f, H = 11.0f;
    B.begin_mesh(mFloor);
    B.grid(V3{-X, 0.0f, Z1}, V3{2 * X, 0, 0}, V3{0, 0, Z0 - Z1}, V3{0, 1, 0}, scaled(64, detail), scaled(128, detail), 8.0f, 16.0f);
    B.end_mesh();
    B.begin_mesh(mWall);
    B.grid(V3{-X, H, Z1}, V3{0, 0, Z0 - Z1}, V3{0, -H, 0}, V3{1, 0, 0}, 64, 16, 16.0f, 4.0f);
    B.grid(V3{X, H, Z0}, V3{0, 0, Z1 - Z0}, V3{0, -H, 0}, V3{-1, 0, 0}, 64, 16, 16.0f, 4.0f);
    B.grid(V3{X, H, Z0}, V3{-2 * X, 0, 0}, V3{0, -H, 0}, V3{0, 0, 1}, 32, 16, 8.0f, 4.0f);
    B.end_mesh();
    // roof beams with skylight gaps
    B.begin_mesh(mRoof);
    for (int k = 0; k < 20; ++k) {
        const float z = Z0 + 2.0f * k;
        B.box(V3{-X, H, z}, V3{X, H + 0.6f, z + 1.1f}, 0.5f);
    }
    B.end_mesh();
    const int seg = scaled(48, detail), rings = scaled(32, detail);
    for (int r = 0; r < 2; ++r)
        for (int k = 0; k < 9; ++k) {
            const float x = r == 0 ? -5.5f : 5.5f, z = Z0 + 3.0f + 4.0f * k;
            B.begin_mesh(mPillar);
            B.cylinder(V3{x, 0.0f, z}, 0.6f, H, seg, rings, 0.06f, 20, 0.5f);
            B.end_mesh();
            B.begin_mesh(mGold);
            std::vector<std::pair<float, float>> cap = {{0.6f, H - 0.6f}, {0.75f, H - 0.4f}, {0.9f, H - 0.2f}, {0.9f, H}, {0.0f, H}};
            B.lathe(V3{x, 0.0f, z}, cap, seg, 1.0f);
            B.end_mesh();
        }
    // trees: trunks + dense alpha-tested foliage cards (the any-hit heavy part of C4)
    for (int t = 0; t < 10; ++t) {
        const float x = rng.range(-7.5f, 7.5f), z = rng.range(-18.0f, 8.0f);
        if (std::fabs(x) > 4.5f && std::fabs(x) < 6.5f) continue;
        B.begin_mesh(mBark);
        B.cylinder(V3{x, 0.0f, z}, 0.18f, 3.5f, scaled(24, detail), 12, 0.0f, 1, 1.0f);
        B.end_mesh();
        B.begin_mesh(t & 1 ? mLeafA : mLeafB);
        const int cards = 260;
        for (int k = 0; k < cards; ++k) {
            float ang = rng.range(0.0f, 6.2831853f), el = rng.range(-0.6f, 1.2f);
            float rr = rng.range(0.3f, 1.8f);
            V3 dir{std::cos(ang) * std::cos(el), std::sin(el), std::sin(ang) * std::cos(el)};
            V3 c = V3{x, 3.8f, z} + dir * rr;
            V3 right = normalize(cross(V3{0, 1, 0}, dir) + V3{0.01f, 0, 0});
            V3 up = normalize(cross(dir, right));
            leaf_card(B, c, right, up, 0.8f, 0.8f, scaled(4, detail), 0.08f);
        }
        B.end_mesh();
    }
}

}  // namespace dxrpt_host
