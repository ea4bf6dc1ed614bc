// bvh_stats — host-side BVH quality report for the builder (no GPU needed).
//
// Builds the BVH2 and BVH8 layouts of a host scene exactly as dxrpt_build_bvh does, then walks them with
// a scalar restatement of the device traversal (same node decode, same visit order) for three ray sets:
// primary camera rays, one cosine-distributed bounce per primary hit, and sun shadow rays from the
// primary hits.  Prints node visits and triangle tests per ray, the quantities the traversal kernels'
// VALU cost scales with, so builder changes can be compared on CPU before spending GPU time.
//
//   make tools && ./build/bvh_stats [scene_id=0] [grid_w=320] [grid_h=180] [binary_depth_cap] [ref_budget]
// (grid_w and grid_h multiples of 8)
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include "../../../include/dxrpt.h"
#include "../../../include/dxrpt_host.h"
#include "../bvh_build.h"

using namespace dxrpt;

namespace {

struct V3 {
    float x, y, z;
};
V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V3 norm(V3 a) {
    float l = sqrtf(dot(a, a));
    return {a.x / l, a.y / l, a.z / l};
}

struct Counters {
    std::vector<uint64_t> keys;  // optional per-ray sort keys (bounce rays)
    uint64_t rays = 0, nodes = 0, tris = 0, hits = 0, alpha_tris = 0;
    uint64_t stack_hist[40] = {};  // rays by maximum stack occupancy
    std::vector<std::vector<uint8_t>> seqs;  // per ray: triangles tested at each node visit, in order
};

struct Scene {
    std::vector<float> pos;  // ntris * 9
    std::vector<uint8_t> alpha;  // per triangle: alpha-tested material (kept whole by the builder)
    uint32_t ntris = 0;
};

float hit_tri(const Scene& S, uint32_t t, V3 o, V3 d, float tmin, float tmax) {
    const float* p = &S.pos[size_t(t) * 9];
    V3 v0{p[0], p[1], p[2]}, v1{p[3], p[4], p[5]}, v2{p[6], p[7], p[8]};
    V3 e1 = sub(v1, v0), e2 = sub(v2, v0);
    V3 pv = cross(d, e2);
    float det = dot(e1, pv);
    if (det == 0.0f) return -1.0f;
    float inv = 1.0f / det;
    V3 tv = sub(o, v0);
    float u = dot(tv, pv) * inv;
    if (u < 0.0f || u > 1.0f) return -1.0f;
    V3 qv = cross(tv, e1);
    float v = dot(d, qv) * inv;
    if (v < 0.0f || u + v > 1.0f) return -1.0f;
    float tt = dot(e2, qv) * inv;
    return (tt >= tmin && tt < tmax) ? tt : -1.0f;
}

// Scalar BVH8 traversal: the same decode and visit order as trav8_step (pt_kernels.hip).
float trace8(const Scene& S, const BvhBuildResult& B, V3 o, V3 d, float tmin, float tmax, bool any, Counters& c,
             uint32_t* out_tri) {
    V3 inv{1.0f / (fabsf(d.x) > 1e-20f ? d.x : copysignf(1e-20f, d.x)), 1.0f / (fabsf(d.y) > 1e-20f ? d.y : copysignf(1e-20f, d.y)),
           1.0f / (fabsf(d.z) > 1e-20f ? d.z : copysignf(1e-20f, d.z))};
    V3 ood{o.x * inv.x, o.y * inv.y, o.z * inv.z};
    // key octant: near to far for closest hits, far to near for any-hit rays (pt_kernels.hip key_octant)
    const uint32_t oct = ((inv.x < 0 ? 4u : 0u) | (inv.y < 0 ? 2u : 0u) | (inv.z < 0 ? 1u : 0u)) ^ (any ? 7u : 0u);
    float best = tmax;
    uint32_t best_tri = ~0u;
    std::vector<std::pair<uint32_t, uint32_t>> stk;
    uint32_t node = 0;
    size_t max_sp = 0;
    c.rays++;
    c.seqs.emplace_back();
    std::vector<uint8_t>& seq = c.seqs.back();
    struct Hist {
        Counters& c;
        size_t& m;
        ~Hist() { c.stack_hist[std::min<size_t>(m, 39)]++; }
    } hist{c, max_sp};
    for (;;) {
        c.nodes++;
        const Bvh8Node& n = B.nodes8[node];
        float a[3], b[3];
        const float* invp = &inv.x;
        const float* oodp = &ood.x;
        for (int k = 0; k < 3; ++k) {
            uint32_t eb = uint32_t(n.e[k]) << 23;
            float sc;
            memcpy(&sc, &eb, 4);
            a[k] = sc * invp[k];
            b[k] = fmaf(n.p[k], invp[k], -oodp[k]);
        }
        uint32_t ihits = 0, thits = 0;
        // child order of closest-hit rays (env SIM_ORDER): 3 (default) nearest hit internal child first, the
        // rest as one octant-keyed group (the split tails, k_path at <= 5 waves/SIMD); 0 octant key order
        // (k_path<6/7>); 1 / 2 every child sorted by entry distance (any-hit: far first / widest first);
        // 4 as 3, and any-hit rays take the hit internal child with the farthest entry first.
        // Any-hit rays: far-to-near octant order in modes 0 and 3 (pt_kernels.hip key_octant).
        static const int sim_order = getenv("SIM_ORDER") ? atoi(getenv("SIM_ORDER")) : 3;
        std::pair<float, uint32_t> exact[8];
        int nex = 0;
        for (int s = 0; s < 8; ++s) {
            uint32_t m = n.meta[s];
            if (!m) continue;
            float tn = tmin, tf = best;
            for (int k = 0; k < 3; ++k) {
                float t0 = fmaf(float(n.qlo[k][s]), a[k], b[k]), t1 = fmaf(float(n.qhi[k][s]), a[k], b[k]);
                tn = std::max(tn, std::min(t0, t1));
                tf = std::min(tf, std::max(t0, t1));
            }
            if (tn > tf) continue;
            if (m & kMetaInternal) {
                ihits |= 1u << ((m & 7u) ^ oct);
                exact[nex++] = {any ? (sim_order == 2 ? -(tf - tn) : -tn) : tn, m & 7u};
            } else thits |= ((1u << (m >> 5)) - 1u) << (m & 31u);
        }
        if (sim_order != 3 && sim_order != 4 && sim_order && nex) {  // exact order: push all but the first, far end first
            std::sort(exact, exact + nex);
            // children slots: node index = base_child + rank of slot among internal slots
            for (int e = nex - 1; e >= 1; --e) {
                uint32_t slot = exact[e].second;
                stk.push_back({n.base_child + uint32_t(__builtin_popcount(n.imask & ((1u << slot) - 1u))), 0xFFFFFFFFu});
            }
            max_sp = std::max(max_sp, stk.size());
        }
        seq.push_back(uint8_t(__builtin_popcount(thits)));
        while (thits) {
            uint32_t bit = __builtin_ctz(thits);
            thits &= thits - 1;
            c.tris++;
            uint32_t t = B.tri_order[n.base_tri + bit];
            c.alpha_tris += S.alpha[t];
            float tt = hit_tri(S, t, o, d, tmin, best);
            if (tt >= 0.0f) {
                best = tt;
                best_tri = t;
                if (any) {
                    c.hits++;
                    if (out_tri) *out_tri = t;
                    return best;
                }
            }
        }
        if (sim_order == 3 || sim_order == 4) {  // nearest internal child first (closest hit; mode 4: any-hit
                                                  // rays the farthest entry first), the rest as an octant-keyed group
            if ((!any || sim_order == 4) && nex) {
                int bi = 0;
                for (int e = 1; e < nex; ++e) if (exact[e].first < exact[bi].first) bi = e;
                const uint32_t slot = exact[bi].second;
                const uint32_t rest = ihits & ~(1u << (slot ^ oct));
                if (rest) stk.push_back({n.base_child, (rest << 24) | n.imask});
                max_sp = std::max(max_sp, stk.size());
                node = n.base_child + uint32_t(__builtin_popcount(n.imask & ((1u << slot) - 1u)));
                continue;
            }
        }
        if (sim_order == 1 || sim_order == 2) {
            // test the leaf triangles first (already done above), then go to the nearest internal child
            if (nex) {
                node = n.base_child + uint32_t(__builtin_popcount(n.imask & ((1u << exact[0].second) - 1u)));
                continue;
            }
            for (;;) {
                if (stk.empty()) {
                    if (best_tri != ~0u) c.hits++;
                    if (out_tri) *out_tri = best_tri;
                    return best_tri != ~0u ? best : -1.0f;
                }
                node = stk.back().first;
                stk.pop_back();
                break;
            }
            continue;
        }
        uint32_t gbase = n.base_child, gword = (ihits << 24) | n.imask;
        for (;;) {
            if (gword >> 24) {
                uint32_t k = 31u - __builtin_clz(gword);
                gword &= ~(1u << k);
                uint32_t slot = (k - 24u) ^ oct;
                node = gbase + __builtin_popcount(gword & 0xFFu & ((1u << slot) - 1u));
                if (gword >> 24) stk.push_back({gbase, gword});
                max_sp = std::max(max_sp, stk.size());
                break;
            }
            if (stk.empty()) {
                if (best_tri != ~0u) c.hits++;
                if (out_tri) *out_tri = best_tri;
                return best_tri != ~0u ? best : -1.0f;
            }
            gbase = stk.back().first;
            gword = stk.back().second;
            stk.pop_back();
        }
    }
}

uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
float rnd(uint64_t& s) { return float(splitmix(s) >> 40) * (1.0f / 16777216.0f); }

// SIMT replay of the recorded traversals: waves of 64 lanes over consecutive rays (the device queue
// order), one node visit per lane per iteration.  Policies:
//   inline   : a lane tests the triangles of the node it just visited in the same iteration (today)
//   postpone : triangles wait until >= T lanes have some (or no lane can visit a node), then all
//              those lanes test theirs together (Ylitie et al. 2017, sec. 4)
//   pool K/R : a wave owns K * 64 rays and refills idle lanes once >= R are idle
// Cost units: C_node per node iteration, C_tri per triangle-loop trip, C_refill per refill.
struct Policy {
    const char* name;
    int postpone_T;  // 0 = inline
    int pool_chunks;
    int refill;
};
double simulate(const std::vector<std::vector<uint8_t>>& seqs, const Policy& P) {
    const double Cn = 250.0, Ct = 90.0, Cr = 150.0;
    double cost = 0.0;
    const size_t pool = size_t(64) * P.pool_chunks;
    for (size_t base = 0; base < seqs.size(); base += pool) {
        const size_t end = std::min(seqs.size(), base + pool);
        size_t next = base;
        const std::vector<uint8_t>* seq[64] = {};
        size_t j[64] = {};
        int pend[64] = {};
        bool active[64] = {};
        for (;;) {
            int idle = 0;
            for (int l = 0; l < 64; ++l) idle += !active[l];
            if (next < end && (idle >= P.refill || idle == 64)) {
                for (int l = 0; l < 64 && next < end; ++l)
                    if (!active[l]) {
                        seq[l] = &seqs[next++];
                        j[l] = 0;
                        pend[l] = 0;
                        active[l] = !seq[l]->empty();
                    }
                cost += Cr;
            }
            int nact = 0;
            for (int l = 0; l < 64; ++l) nact += active[l];
            if (!nact) {
                if (next >= end) break;
                continue;
            }
            if (P.postpone_T == 0) {
                int mk = 0;
                for (int l = 0; l < 64; ++l)
                    if (active[l]) {
                        mk = std::max(mk, int((*seq[l])[j[l]]));
                        if (++j[l] == seq[l]->size()) active[l] = false;
                    }
                cost += Cn + Ct * mk;
            } else {
                int ntri = 0, nnode = 0, mk = 0;
                for (int l = 0; l < 64; ++l) {
                    if (!active[l]) continue;
                    if (pend[l]) { ntri++; mk = std::max(mk, pend[l]); }
                    else nnode++;
                }
                if (ntri >= P.postpone_T || nnode == 0) {
                    cost += Ct * mk;
                    for (int l = 0; l < 64; ++l)
                        if (active[l] && pend[l]) {
                            pend[l] = 0;
                            if (j[l] == seq[l]->size()) active[l] = false;
                        }
                } else {
                    cost += Cn;
                    for (int l = 0; l < 64; ++l)
                        if (active[l] && !pend[l]) {
                            pend[l] = (*seq[l])[j[l]];
                            if (++j[l] == seq[l]->size() && !pend[l]) active[l] = false;
                        }
                }
            }
        }
    }
    return cost;
}

void simulate_all(const char* name, const Counters& c) {
    static const Policy kPolicies[] = {
        {"inline", 0, 1, 64},      {"postpone8", 8, 1, 64},    {"postpone16", 16, 1, 64},
        {"postpone32", 32, 1, 64}, {"pool2r16", 0, 2, 16},     {"pool4r16", 0, 4, 16},
        {"pool4r32", 0, 4, 32},    {"pool8r16", 0, 8, 16},     {"pool4r16+pp16", 16, 4, 16},
        {"pool8r16+pp16", 16, 8, 16}, {"pool4r8", 0, 4, 8},
    };
    double ideal = 0.0;
    for (const auto& s : c.seqs) {
        ideal += 250.0 * s.size();
        for (uint8_t k : s) ideal += 90.0 * k;
    }
    ideal /= 64.0;
    double base = 0.0;
    printf("  %-8s SIMT cost / ideal (lower is better):", name);
    for (const Policy& P : kPolicies) {
        double v = simulate(c.seqs, P);
        if (&P == &kPolicies[0]) base = v;
        printf(" %s %.2f", P.name, v / ideal);
    }
    printf("  [inline = %.0f units/ray]\n", base / c.seqs.size());
}

void report(const char* name, const Counters& c) {
    printf("  %-9s rays %8llu  nodes/ray %6.2f  tris/ray %6.2f (alpha %5.2f)  hit %5.1f%%  stack>4 %.3f%% >6 %.4f%% >8 %.5f%% max ",
           name, (unsigned long long)c.rays, double(c.nodes) / c.rays, double(c.tris) / c.rays, double(c.alpha_tris) / c.rays,
           100.0 * c.hits / c.rays,
           [&] { uint64_t n = 0; for (int i = 5; i < 40; ++i) n += c.stack_hist[i]; return 100.0 * n / c.rays; }(),
           [&] { uint64_t n = 0; for (int i = 7; i < 40; ++i) n += c.stack_hist[i]; return 100.0 * n / c.rays; }(),
           [&] { uint64_t n = 0; for (int i = 9; i < 40; ++i) n += c.stack_hist[i]; return 100.0 * n / c.rays; }());
    int mx = 0;
    for (int i = 0; i < 40; ++i)
        if (c.stack_hist[i]) mx = i;
    printf("%d\n", mx);
}

}  // namespace

int main(int argc, char** argv) {
    const uint32_t scene_id = argc > 1 ? uint32_t(atoi(argv[1])) : 0u;
    {   // packaged assets: dxrpathtracer_amd/data, two levels above this binary (csrc/build/bvh_stats)
        std::string dir(argv[0]);
        dir = dir.find('/') == std::string::npos ? std::string(".") : dir.substr(0, dir.rfind('/'));
        dxrpt_host_set_asset_dir((dir + "/../../data").c_str());
    }
    const uint32_t gw = argc > 2 ? uint32_t(atoi(argv[2])) : 320u;
    const uint32_t gh = argc > 3 ? uint32_t(atoi(argv[3])) : 180u;
    BvhBuildParams params;  // argv[4]: binary depth cap to explore (0: default; the wide depth is then unbounded)
    if (argc > 4 && atoi(argv[4]) > 0) {
        params.binary_depth_cap = uint32_t(atoi(argv[4]));
        params.max_wide_depth = 1000u;
    }
    if (argc > 5) {  // argv[5]: spatial-split reference budget (0: no spatial splits)
        params.ref_budget = atof(argv[5]);
        params.spatial_splits = params.ref_budget > 0.0;
    }
    if (argc > 6) params.treelet_passes = uint32_t(atoi(argv[6]));  // argv[6]: treelet restructuring passes
    if (argc > 7) params.threads = unsigned(atoi(argv[7]));  // argv[7]: builder threads (0: auto)
    dxrpt_host_scene* hs = nullptr;
    if (dxrpt_host_scene_create(scene_id, 0, 0, &hs) != 0) {
        fprintf(stderr, "scene: %s\n", dxrpt_host_last_error());
        return 1;
    }
    Scene S;
    S.ntris = hs->num_indices / 3;
    S.pos.resize(size_t(S.ntris) * 9);
    for (uint32_t g = 0; g < hs->num_geometries; ++g) {
        const dxrpt_geometry_info& gi = hs->geometries[g];
        uint32_t end = g + 1 < hs->num_geometries ? hs->geometries[g + 1].IdxOffset / 3 : S.ntris;
        for (uint32_t t = gi.IdxOffset / 3; t < end; ++t)
            for (int k = 0; k < 3; ++k) {
                uint32_t idx = hs->idx_bytes == 2 ? static_cast<const uint16_t*>(hs->indices)[t * 3 + k]
                                                  : static_cast<const uint32_t*>(hs->indices)[t * 3 + k];
                memcpy(&S.pos[size_t(t) * 9 + k * 3], hs->vertices[idx + gi.VtxOffset].Position, 12);
            }
    }
    S.alpha.assign(S.ntris, 0u);
    for (uint32_t g = 0; g < hs->num_geometries; ++g) {
        uint32_t end = g + 1 < hs->num_geometries ? hs->geometries[g + 1].IdxOffset / 3 : S.ntris;
        if (hs->materials[hs->geometries[g].MaterialIdx].Opacity != DXRPT_INVALID_INDEX)
            for (uint32_t t = hs->geometries[g].IdxOffset / 3; t < end; ++t) S.alpha[t] = 1u;
    }
    params.keep_whole = S.alpha.data();  // as dxrpt_build_bvh
    printf("scene %u: %u triangles\n", scene_id, S.ntris);
    BvhBuildResult B;
    std::string err;
    auto t0 = std::chrono::steady_clock::now();
    if (!build_bvh(S.pos.data(), S.ntris, 8, B, err, &params)) {
        fprintf(stderr, "build: %s\n", err.c_str());
        return 1;
    }
    double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    uint64_t slots = 0, leaf_tris = 0, leaves = 0;
    for (const Bvh8Node& n : B.nodes8)
        for (int s = 0; s < 8; ++s)
            if (n.meta[s]) {
                slots++;
                if (!(n.meta[s] & kMetaInternal)) {
                    leaves++;
                    leaf_tris += n.meta[s] >> 5;
                }
            }
    {   // FNV-1a over the emitted layout: identical trees for any thread count
        uint64_t h = 1469598103934665603ull;
        auto mix = [&](const void* p, size_t n) {
            const uint8_t* b = static_cast<const uint8_t*>(p);
            for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
        };
        mix(B.nodes8.data(), B.nodes8.size() * sizeof(Bvh8Node));
        mix(B.tri_order.data(), B.tri_order.size() * sizeof(uint32_t));
        printf("layout hash %016llx (%zu nodes, %zu refs)\n", (unsigned long long)h, B.nodes8.size(), B.tri_order.size());
    }
    printf("phases: sbvh %.0f treelet %.0f collapse %.0f ms (treelet passes %u)\n", B.phase_ms[0], B.phase_ms[1], B.phase_ms[2], B.treelet_passes);
    printf("BVH8: %zu nodes, depth %u (binary cap %u), %.2f children/node, %llu leaves, %.2f tris/leaf, build %.0f ms, SAH(bin) %.2f SAH(wide) %.2f\n",
           B.nodes8.size(), B.max_depth, B.binary_depth_cap, double(slots) / B.nodes8.size(), (unsigned long long)leaves,
           double(leaf_tris) / leaves, ms, B.sah_cost, B.wide_sah);

    float M[16];
    dxrpt_host_inv_view_projection(hs->camera_position, hs->camera_rotation[0], hs->camera_rotation[1], 3.14159265f / 4.0f,
                                   16.0f / 9.0f, 0.1f, 100.0f, M);
    V3 sun = norm({hs->sun_direction[0], hs->sun_direction[1], hs->sun_direction[2]});
    float scene_lo[3] = {3.4e38f, 3.4e38f, 3.4e38f}, scene_hi[3] = {-3.4e38f, -3.4e38f, -3.4e38f};
    for (size_t i = 0; i < S.pos.size(); ++i) {
        scene_lo[i % 3] = std::min(scene_lo[i % 3], S.pos[i]);
        scene_hi[i % 3] = std::max(scene_hi[i % 3], S.pos[i]);
    }
    Counters prim, bounce, shadow;
    uint64_t rng = 12345;
    // rays in the device's order: 8x8 pixel blocks (one wave each), blocks row-major
    for (uint32_t pix = 0; pix < gw * gh; ++pix) {
            const uint32_t blk = pix / 64, in = pix % 64, bw = gw / 8;
            const uint32_t x = (blk % bw) * 8 + in % 8, y = (blk / bw) * 8 + in / 8;
            float ncx = (x + 0.5f) / gw * 2.0f - 1.0f, ncy = -((y + 0.5f) / gh * 2.0f - 1.0f);
            float s[4], e[4];
            for (int j = 0; j < 4; ++j) {
                s[j] = ncx * M[j] + ncy * M[4 + j] + M[12 + j];
                e[j] = ncx * M[j] + ncy * M[4 + j] + M[8 + j] + M[12 + j];
            }
            V3 o{s[0] / s[3], s[1] / s[3], s[2] / s[3]};
            V3 en{e[0] / e[3], e[1] / e[3], e[2] / e[3]};
            V3 dd = sub(en, o);
            float len = sqrtf(dot(dd, dd));
            V3 d = norm(dd);
            uint32_t tri = ~0u;
            float t = trace8(S, B, o, d, 0.0f, len, false, prim, &tri);
            if (t < 0.0f) continue;
            V3 p{o.x + d.x * t, o.y + d.y * t, o.z + d.z * t};
            const float* v = &S.pos[size_t(tri) * 9];
            V3 nrm = norm(cross(sub({v[3], v[4], v[5]}, {v[0], v[1], v[2]}), sub({v[6], v[7], v[8]}, {v[0], v[1], v[2]})));
            if (dot(nrm, d) > 0.0f) nrm = {-nrm.x, -nrm.y, -nrm.z};
            trace8(S, B, p, sun, 1e-4f, 3.4e38f, true, shadow, nullptr);
            // cosine-distributed bounce around the facing normal
            float r1 = rnd(rng), r2 = rnd(rng);
            float r = sqrtf(r1), phi = 6.2831853f * r2;
            V3 tt = fabsf(nrm.x) > 0.5f ? norm(cross(nrm, {0, 1, 0})) : norm(cross(nrm, {1, 0, 0}));
            V3 bb = cross(nrm, tt);
            float lx = r * cosf(phi), ly = r * sinf(phi), lz = sqrtf(std::max(0.0f, 1.0f - r1));
            V3 bd = norm({tt.x * lx + bb.x * ly + nrm.x * lz, tt.y * lx + bb.y * ly + nrm.y * lz, tt.z * lx + bb.z * ly + nrm.z * lz});
            trace8(S, B, p, bd, 1e-4f, 3.4e38f, false, bounce, nullptr);
            {   // sort key: direction octant (3 bits) | 30-bit Morton code of the origin in the scene box
                auto q = [](float v, float lo, float hi) {
                    float t = (v - lo) / (hi - lo);
                    return uint32_t(std::min(std::max(t, 0.0f), 0.999999f) * 1024.0f);
                };
                auto spread = [](uint64_t v) {
                    uint64_t r = 0;
                    for (int b = 0; b < 10; ++b) r |= ((v >> b) & 1ull) << (3 * b);
                    return r;
                };
                const float* lo = scene_lo;
                const float* hi = scene_hi;
                uint64_t m = spread(q(p.x, lo[0], hi[0])) | (spread(q(p.y, lo[1], hi[1])) << 1) | (spread(q(p.z, lo[2], hi[2])) << 2);
                uint64_t oct = (bd.x < 0 ? 4u : 0u) | (bd.y < 0 ? 2u : 0u) | (bd.z < 0 ? 1u : 0u);
                // finer direction bin: 4x4 cells on the octant's face of the direction cube
                float ax = fabsf(bd.x), ay = fabsf(bd.y), az = fabsf(bd.z);
                uint32_t face = ax >= ay && ax >= az ? 0 : (ay >= az ? 1 : 2);
                float u = face == 0 ? ay / ax : ax / (face == 1 ? ay : az), v = face == 2 ? ay / az : az / (face == 0 ? ax : ay);
                uint64_t dbin = (face << 4) | (uint32_t(std::min(u, 0.999f) * 4) << 2) | uint32_t(std::min(v, 0.999f) * 4);
                bounce.keys.push_back((oct << 60) | (dbin << 52) | (uint64_t(bounce.keys.size()) << 0) | (m << 22) * 0);
                bounce.keys.back() = (oct << 61) | (dbin << 55) | (m << 25);
            }
        }
    report("primary", prim);
    report("bounce", bounce);
    report("shadow", shadow);
    simulate_all("primary", prim);
    simulate_all("bounce", bounce);
    {   // the same bounce rays re-ordered by sort keys
        auto reorder = [&](const char* nm, auto keyfn) {
            std::vector<size_t> idx(bounce.seqs.size());
            for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
            std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return keyfn(a) < keyfn(b); });
            Counters c2;
            c2.rays = bounce.rays;
            for (size_t i : idx) c2.seqs.push_back(bounce.seqs[i]);
            simulate_all(nm, c2);
        };
        reorder("b:oct", [&](size_t i) { return bounce.keys[i] >> 61; });
        reorder("b:oct+dir", [&](size_t i) { return bounce.keys[i] >> 55; });
        reorder("b:oct+org", [&](size_t i) { return (bounce.keys[i] >> 61 << 40) | ((bounce.keys[i] >> 25) & ((1ull << 30) - 1)); });
        reorder("b:o+d+org", [&](size_t i) { return bounce.keys[i]; });
        reorder("b:org", [&](size_t i) { return (bounce.keys[i] >> 25) & ((1ull << 30) - 1); });
    }
    simulate_all("shadow", shadow);
    // relative VALU cost model of the BVH8 kernels (~225 ops per node visit, ~80 per triangle test)
    auto cost = [](const Counters& c) { return (225.0 * c.nodes + 80.0 * c.tris) / c.rays; };
    printf("  cost model (VALU ops/ray): primary %.0f bounce %.0f shadow %.0f\n", cost(prim), cost(bounce), cost(shadow));
    dxrpt_host_scene_destroy(hs);
    return 0;
}
