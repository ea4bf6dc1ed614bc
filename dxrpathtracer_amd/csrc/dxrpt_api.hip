// dxrpt_api.hip — the C ABI (include/dxrpt.h): context, scene upload, BVH build, render.
//
// Host-side counterpart of DXRPathTracer::BuildRTAccelerationStructure (DXRPathTracer.cpp:2331-2488)
// and DXRPathTracer::RenderRayTracing (DXRPathTracer.cpp:2024-2090).  No exception crosses the ABI:
// every entry point catches, stores a message for dxrpt_last_error and returns a DXRPT_E_* code.
//
// Stream ordering (include/dxrpt.h "Stream ordering"): the reference records every frame into one
// command queue (Graphics/DX12.cpp:263-305), so each frame sees the previous one's result.  Here every
// call that enqueues work runs after all work this context enqueued before it, whatever stream the caller
// passes: a call on a stream other than the previous call's first makes its stream wait on an event
// recorded at the end of the previous one (enter_stream).  Overlapped frames run on two internal slot
// streams and blend on the caller's stream, so the chain of caller streams orders them too.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <map>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/dxrpt.h"
#include "bvh_build.h"
#include "omm.h"
#include "pt_kernels.h"
#include "pt_layout.h"
#include "post_kernels.h"

using namespace dxrpt;

namespace {

struct ApiError : std::runtime_error {
    int code;
    ApiError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIP_CHECK(expr)                                                                                   \
    do {                                                                                                  \
        hipError_t e_ = (expr);                                                                           \
        if (e_ != hipSuccess)                                                                             \
            throw ApiError(DXRPT_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));                \
    } while (0)

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    void ensure(size_t n) {
        if (n <= bytes && p) return;
        release();
        if (n == 0) n = 16;
        hipError_t e = hipMalloc(&p, n);
        if (e != hipSuccess) throw ApiError(DXRPT_E_OOM, "hipMalloc(" + std::to_string(n) + "): " + hipGetErrorString(e));
        bytes = n;
    }
    void upload(const void* src, size_t n) {
        ensure(n);
        if (n) HIP_CHECK(hipMemcpy(p, src, n, hipMemcpyHostToDevice));
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

// Depth-split schedule by frame size (DXRPT_OPT_MEGAKERNEL_SPLIT 2): frames of at least this many path
// vertices (paths x (L - 1)); with overlapped frames the next frames fill the per-depth kernels' drains,
// so the split pays from fewer vertices -- the more frames in flight, the fewer (r05 with
// three in flight: 720p L=3, 1.84M vertices, 0.770 -> 0.699 ms split; the 1/4 share, 1.04M, +5 %:
// profiles/r05_ab_share_knobs.txt).
constexpr uint64_t kSplitMinVertices = 8000000;
constexpr uint64_t kSplitMinVerticesOverlap2 = 2000000;  // two frames in flight
constexpr uint64_t kSplitMinVerticesOverlap3 = 1500000;  // three
// DXRPT_OPT_FRAME_OVERLAP: up to three frames in flight, frame f on slot f % (frames in flight)
#ifndef DXRPT_OVERLAP_SLOTS
#define DXRPT_OVERLAP_SLOTS 3
#endif
constexpr uint32_t kOverlapSlots = DXRPT_OVERLAP_SLOTS;
static_assert(kOverlapSlots >= 3 && kOverlapSlots < 32, "DXRPT_OPT_FRAME_OVERLAP 2 needs three slots; the gate mask is 32 bits");
constexpr uint32_t kOverlapBySize = 3;  // DXRPT_OPT_FRAME_OVERLAP value: frames in flight by frame size
// BVH8 stack-spill slabs: 0 = work on the caller's stream, 1 + k = overlap slot k
constexpr uint32_t kSpillSlabs = 1 + kOverlapSlots;
constexpr uint32_t kTravCounters = 10;  // census: [0..4] depth-1 vertices, [5..9] deeper (dxrpt_stats)

}  // namespace

struct dxrpt_ctx {
    int device = 0;
    std::string err;
    // host copies of the scene
    std::vector<dxrpt_mesh_vertex> vertices;
    std::vector<uint32_t> indices;
    std::vector<dxrpt_geometry_info> geos;
    std::vector<dxrpt_material> mats;
    std::vector<TexDesc> texdesc;
    std::vector<uint32_t> texels;
    bool scene_set = false, bvh_built = false, sky_set = false, tex_dirty = true, geoshade_dirty = true;
    uint32_t sky_res = 0;
    // device copies
    DevBuf d_texels, d_sky, d_lut, d_nodes8, d_tris, d_geoshade;
    DevBuf d_lights, d_tiles, d_tile_prefix;
    DevBuf p_bloom0, p_bloom1;  // post-processing scratch (RGBA16F half-res)
    DevBuf d_tri_verts;  // per global triangle: its 3 MeshVertex records (3 x 64 B), built with the BVH
    // per-frame buffers of work on the caller's stream (wavefront passes, non-overlapped megakernel frames)
    DevBuf f_pix, f_pxrad, f_hit, f_fwd, f_shn, f_shq, f_shorg, f_shdir, f_shcon, f_counters;
    DevBuf f_q[2][5];  // RayQueue org, dir, thr, rad, pix per depth parity
    FrameBuffers fb;
    uint32_t ctr_set = 0;                 // counter set of the next frame (f_counters holds two)
    bool ctr_clean[2] = {false, false};   // set known to be zero (zeroed by the previous megakernel frame)
    dxrpt_bvh_info bvh{};
    std::vector<dxrpt_tile> tiles_cache;
    std::vector<dxrpt_spot_light> lights_cache;
    dxrpt_stats last{};
    int last_L = 0;
    bool rendered = false;
    bool last_counted = false;  // the last render ran a counting (census) frame: dxrpt_get_stats reads d_trav
    // stream ordering: the stream of the last enqueuing call, whether anything may still be in flight
    hipStream_t last_stream = nullptr;
    bool have_last = false;
    bool inflight = false;
    hipEvent_t chain_ev = nullptr;
    // options
    bool opt_count = false, opt_timing = false;
    uint32_t opt_timing_mask = (1u << DXRPT_K_COUNT) - 1u;  // DXRPT_OPT_KERNEL_TIMING_MASK
    uint32_t num_cus = 256;
    uint32_t opt_packet = 3;        // DXRPT_OPT_PACKET_TRAVERSAL
    hipStream_t aux = nullptr;      // wavefront any-hit pass stream (created on first use)
    std::vector<hipEvent_t> fork_ev;
    uint32_t opt_mega_paths = 0xFFFFFFFFu;  // DXRPT_OPT_MEGAKERNEL_PATHS (path vertices; default: every frame)
    uint32_t opt_mega_occ = 0;              // DXRPT_OPT_MEGAKERNEL_OCCUPANCY (0 = by frame size)
    uint32_t opt_tail_occ = 0;              // DXRPT_OPT_TAIL_OCCUPANCY (0 = 7, or the megakernel's when set)
    uint32_t opt_bake_chunk = 1u << 21;     // DXRPT_OPT_BAKE_CHUNK (texels per bake launch)
    uint32_t opt_split = 2;                 // DXRPT_OPT_MEGAKERNEL_SPLIT (0 off, 1 on, 2 by frame size)
    uint32_t opt_omm = 1;                   // DXRPT_OPT_OPACITY_MICROMAP
    uint32_t opt_packed = 3;                // DXRPT_OPT_PACKED_TAPS (bit 0: packed NMR maps, bit 1: inlined 1 x 1 maps)
    std::vector<uint32_t> texels_packed;    // packed normal/metallic/roughness textures, after `texels` on the device
    uint32_t packed_materials = 0, packed_textures = 0;  // of the current shading records (dxrpt_stats)
    uint32_t inlined_refs = 0;  // geometry texture references inlined (1 x 1 maps)
    uint32_t opt_overlap = kOverlapBySize;  // DXRPT_OPT_FRAME_OVERLAP
    // overlapped frames: frame f runs on slot f % kOverlapSlots -- its own stream, path buffers, counters,
    // stage and BVH8 stack-spill slab -- and stages its radiance (d_stage); the caller's stream blends the
    // stage once the frame is done, so frame f+1's waves start while frame f drains
    struct Slot {
        DevBuf q[2][5], shorg, shdir, shcon, counters, stage;
        FrameBuffers fb;
        uint32_t ctr_set = 0;
        bool ctr_clean[2] = {false, false};
        hipStream_t stream = nullptr;
        hipEvent_t done = nullptr;        // the slot's last frame (and its order pass) is done
        hipEvent_t stage_free = nullptr;  // caller's stream: the slot's last stage has been blended
        bool stage_used = false;
    };
    Slot slot[kOverlapSlots];
    hipEvent_t ovl_fork = nullptr;  // the first overlapped frame after other work starts behind the caller's stream
    bool ovl_active = false;        // the slot streams run overlapped frames (no fork needed)
    hipEvent_t ovl_gate = nullptr;  // frames on the other slots wait for it (a rebuilt wave order)
    uint32_t ovl_gate_pending = 0;  // bit k: slot k's next frame has not yet waited on ovl_gate
    uint32_t ovl_parity = 0;
    uint32_t ovl_slots = 0;  // frames in flight of the current rotation (2 or 3)
    std::vector<const uint32_t*> stat_counters;  // counter set of the last frame
    uint32_t accum_extent = 0;  // 1 + the largest accumulation index of the current tile list (stage size)
    DevBuf d_omm;                           // kOmmWords per micromap slot (pt_layout.h kOmm*)
    std::vector<uint32_t> omm_tris;         // slot -> global triangle (alpha-tested geometry), set by the BVH build
    bool omm_dirty = true, omm_any = false; // any: some triangle has a verdict (else d_omm is not read)
    BvhBuildParams build_params;    // DXRPT_OPT_SPATIAL_SPLITS, DXRPT_OPT_LEAF_COST, DXRPT_OPT_TREELET_PASSES
    DevBuf d_trav;   // kTravCounters x u64 census counters (DXRPT_OPT_COUNT_TRAVERSAL)
    DevBuf d_wclock;  // 2 x u64 per wave (DXRPT_OPT_WAVE_CLOCKS)
    bool opt_wave_clocks = false;
    uint32_t wclock_waves = 0;
    // DXRPT_OPT_WAVE_ORDER: per wave slot, the last frame's duration and the order built from it
    uint32_t opt_wave_order = 2;  // 0 off, 1 on, 2 by frame size (see render)
    uint32_t opt_xcd_chunk = 8;       // DXRPT_OPT_XCD_CHUNK (r02: 1080p 2.100 -> 2.075 ms, C4 2.276 -> 2.252)
    DevBuf d_wave_cost, d_wave_order, d_wave_hist;  // hist: 2 frames x (histogram, cursor) x kWaveClasses
    uint32_t order_parity = 0;
    uint64_t order_key = 0;     // (waves, tiles generation) the order was built for
    bool order_ready = false;   // d_wave_order holds an order for order_key
    uint32_t order_frame = 0;   // ordered frames since the order (re)started
    uint32_t opt_order_period = 256; // DXRPT_OPT_WAVE_ORDER_PERIOD (r02: 1/8 share 0.549 -> 0.534 ms at 16;
                                     // r04: 16 -> 64, slowest 1/8 shares -1.3..-2.5 %: a recording frame costs
                                     // ~0.26 ms, profiles/r04_ab_order_period.txt; r05, three frames in flight:
                                     // 64 -> 256, 1/8 shares -2.6 % -- the rebuild also waits for the other
                                     // slots' frames; 256 frames are ~60 ms of a 1/8 share,
                                     // profiles/r05_ab_order_period.txt)
    uint64_t tiles_gen = 0;     // bumped whenever the tile list changes
    DevBuf d_spill;  // BVH8 traversal stack entries beyond the LDS part (deep trees only), kSpillSlabs slabs
    uint32_t spill_threads = 0;  // per-slab stride: the largest traversal launch seen
    DevBuf d_bake_list;  // live lightmap texels of the last bake pass + their count
    // kernel timing: a ring of per-frame event sets, harvested lazily
    struct FrameEvents {
        std::vector<hipEvent_t> ev;
        int L = 0;
        uint32_t mask = 0;  // kernel kinds whose events were recorded
        bool pending = false;
        bool mega = false;   // megakernel frame: ev[0], ev[1] bracket its launches
        bool split = false;  // ... the depth-split schedule: ev[2] after the head
    };
    std::vector<FrameEvents> ring;
    size_t ring_head = 0;
    double kernel_ms[DXRPT_K_COUNT] = {};
    uint64_t kernel_launches[DXRPT_K_COUNT] = {};
    uint64_t timed_frames = 0;
    double frame_ms = 0.0;

    ~dxrpt_ctx() {
        for (Slot& P : slot)
            if (P.stream) (void)hipStreamSynchronize(P.stream);
        if (have_last) (void)hipStreamSynchronize(last_stream);
        if (aux) (void)hipStreamSynchronize(aux);
        DevBuf* all[] = {&d_texels, &d_sky, &d_lut, &d_geoshade, &d_nodes8, &d_tris, &d_tri_verts, &d_lights, &d_tiles,
                         &d_tile_prefix, &f_pix, &f_pxrad, &f_hit, &f_fwd, &f_shn, &f_shq, &f_shorg, &f_shdir, &f_shcon,
                         &f_counters, &p_bloom0, &p_bloom1, &d_wclock, &d_omm, &d_trav, &d_spill, &d_bake_list,
                         &d_wave_cost, &d_wave_order, &d_wave_hist};
        for (DevBuf* b : all) b->release();
        for (auto& qb : f_q)
            for (DevBuf& b : qb) b.release();
        for (auto& f : ring)
            for (hipEvent_t e : f.ev) (void)hipEventDestroy(e);
        if (aux) (void)hipStreamDestroy(aux);
        for (hipEvent_t e : fork_ev) (void)hipEventDestroy(e);
        for (Slot& P : slot) {
            for (auto& qb : P.q)
                for (DevBuf& b : qb) b.release();
            P.shorg.release();
            P.shdir.release();
            P.shcon.release();
            P.counters.release();
            P.stage.release();
            if (P.stream) (void)hipStreamDestroy(P.stream);
            if (P.done) (void)hipEventDestroy(P.done);
            if (P.stage_free) (void)hipEventDestroy(P.stage_free);
        }
        if (ovl_fork) (void)hipEventDestroy(ovl_fork);
        if (ovl_gate) (void)hipEventDestroy(ovl_gate);
        if (chain_ev) (void)hipEventDestroy(chain_ev);
    }
};

namespace {

template <class F>
int guarded(dxrpt_ctx* ctx, F&& f) {
    try {
        if (ctx) HIP_CHECK(hipSetDevice(ctx->device));
        f();
        return DXRPT_OK;
    } catch (const ApiError& e) {
        if (ctx) ctx->err = e.what();
        return e.code;
    } catch (const std::bad_alloc&) {
        if (ctx) ctx->err = "host out of memory";
        return DXRPT_E_OOM;
    } catch (const std::exception& e) {
        if (ctx) ctx->err = e.what();
        return DXRPT_E_INVALID_ARG;
    }
}

void require(bool c, const std::string& msg, int code = DXRPT_E_INVALID_ARG) {
    if (!c) throw ApiError(code, msg);
}

// 256-entry decode tables: [0,256) unorm c/255, [256,512) sRGB -> linear (IEC 61966-2-1), computed in
// double and rounded once; oracle/oracle.cpp builds the same table the same way.
std::vector<float> make_lut() {
    std::vector<float> l(512);
    for (uint32_t i = 0; i < 256; ++i) {
        l[i] = omm_decode(0u, i);
        l[256 + i] = omm_decode(256u, i);
    }
    return l;
}

// Waits until nothing this context enqueued is in flight: before anything in-flight work reads is
// replaced or freed (scene, texture, tile, light and buffer uploads, buffer growth, the cost order's
// restart).  The caller streams form one chain (enter_stream), so the last one covers the older ones.
void drain_frames(dxrpt_ctx* c) {
    if (!c->inflight) return;
    for (dxrpt_ctx::Slot& P : c->slot)
        if (P.stream) HIP_CHECK(hipStreamSynchronize(P.stream));
    if (c->have_last) HIP_CHECK(hipStreamSynchronize(c->last_stream));
    c->inflight = false;
    c->ovl_active = false;
}

// Every enqueuing call starts here: on a stream other than the previous call's, the new stream first
// waits for everything the previous one carries (which, through the blends, includes every overlapped
// frame).  Afterwards `s` is the context's stream until the next call.
void enter_stream(dxrpt_ctx* c, hipStream_t s) {
    if (c->inflight && c->have_last && s != c->last_stream) {
        if (!c->chain_ev) HIP_CHECK(hipEventCreateWithFlags(&c->chain_ev, hipEventDisableTiming));
        HIP_CHECK(hipEventRecord(c->chain_ev, c->last_stream));
        HIP_CHECK(hipStreamWaitEvent(s, c->chain_ev, 0));
    }
    c->last_stream = s;
    c->have_last = true;
}

// BVH8 stack-spill slab `slab` (0: the caller's stream, 1 + k: overlap slot k) for launches of up to
// `threads` global threads.  Every slab has the stride of the largest launch seen, so frames in flight
// on different slots never share entries whatever their sizes; growing it waits for in-flight frames.
void ensure_spill(dxrpt_ctx* c, uint32_t threads) {
    if (c->bvh.max_depth + 1u <= uint32_t(kStackLds8) || threads <= c->spill_threads) return;
    drain_frames(c);
    const size_t per = size_t(kTraversalStack8 - kStackLds8) * threads;
    c->d_spill.ensure(per * kSpillSlabs * sizeof(uint2));
    c->spill_threads = threads;
}

// Device view of the scene; `slab` selects the BVH8 stack-spill slab (ensure_spill sized it).
SceneDev scene_dev(dxrpt_ctx* c, uint32_t slab) {
    SceneDev s;
    s.nodes8 = c->d_nodes8.as<Bvh8Node>();
    const uint32_t entries = c->bvh.max_depth + 1u;
    s.stack_ints = 2u * std::min<uint32_t>(entries, uint32_t(kStackLds8));
    if (entries > uint32_t(kStackLds8)) {
        s.spill8 = c->d_spill.as<uint2>() + size_t(kTraversalStack8 - kStackLds8) * c->spill_threads * slab;
        s.spill_stride = c->spill_threads;
    }
    s.tris = c->d_tris.as<TriRecord>();
    s.tri_verts = c->d_tri_verts.as<float4>();
    s.geoshade = c->d_geoshade.as<GeoShade>();
    s.texels = c->d_texels.as<uint32_t>();
    s.sky = c->d_sky.as<uint16_t>();
    s.lut = c->d_lut.as<float>();
    s.sky_res = c->sky_res;
    s.omm = c->opt_omm && c->omm_any ? c->d_omm.as<uint32_t>() : nullptr;
    return s;
}

// The opacity micromap of every triangle on alpha-tested geometry (omm.cpp), one slot per triangle in
// the order the BVH build numbered them (TriRecord flags >> 1), rebuilt when the texture set changes.
// Triangles whose opacity map is missing or huge keep all-unknown words (always tapped).
void build_omm(dxrpt_ctx* c) {
    const uint32_t ntris = uint32_t(c->indices.size() / 3), ng = uint32_t(c->geos.size());
    const size_t nslots = c->omm_tris.size();
    std::vector<uint32_t> words(nslots * kOmmWords, 0u);
    std::vector<std::unique_ptr<OpacityField>> fields(c->texdesc.size());
    std::vector<uint32_t> tri_geom(ntris, 0u);
    for (uint32_t g = 0; g < ng; ++g) {
        const uint32_t end = g + 1 < ng ? c->geos[g + 1].IdxOffset / 3 : ntris;
        for (uint32_t t = c->geos[g].IdxOffset / 3; t < end && t < ntris; ++t) tri_geom[t] = g;
    }
    bool any = false;
    for (size_t slot = 0; slot < nslots; ++slot) {
        const uint32_t t = c->omm_tris[slot], g = tri_geom[t];
        const uint32_t op = c->mats[c->geos[g].MaterialIdx].Opacity;
        if (op >= c->texdesc.size()) continue;  // no such texture (always accepts): never probed
        const TexDesc& d = c->texdesc[op];
        if (size_t(d.width) * d.height > (size_t(1) << 24)) continue;  // > 16 M texels: tapped as before
        if (!fields[op]) {
            const bool r8 = d.fmt == DXRPT_TEX_R8_UNORM;
            const uint32_t lut = d.fmt == DXRPT_TEX_RGBA8_SRGB ? 256u : 0u;
            const uint32_t tiles_x = (d.width + (r8 ? kTexTileW8 : kTexTileW32) - 1u) / (r8 ? kTexTileW8 : kTexTileW32);
            float dec[256];
            for (uint32_t b = 0; b < 256; ++b) dec[b] = omm_decode(lut, b);
            std::vector<float> v(size_t(d.width) * d.height);
            const uint32_t* T = c->texels.data() + d.offset;
            for (uint32_t y = 0; y < d.height; ++y)
                for (uint32_t x = 0; x < d.width; ++x) {
                    const uint32_t w = T[tex_tile_word(x, y, tiles_x, r8)];
                    v[size_t(y) * d.width + x] = dec[(r8 ? w >> (8u * (x & 3u)) : w) & 0xFFu];
                }
            fields[op] = std::make_unique<OpacityField>(d.width, d.height, std::move(v));
        }
        float uv[6];
        for (int k = 0; k < 3; ++k) {  // indices were range-checked by the BVH build
            const dxrpt_mesh_vertex& mv = c->vertices[size_t(c->indices[size_t(t) * 3 + k]) + c->geos[g].VtxOffset];
            uv[2 * k] = mv.UV[0];
            uv[2 * k + 1] = mv.UV[1];
        }
        uint32_t* w = &words[slot * kOmmWords];
        omm_triangle(*fields[op], uv, w);
        for (uint32_t k = 0; k < kOmmWords; ++k) any = any || w[k] != 0u;
    }
    if (any) c->d_omm.upload(words.data(), words.size() * sizeof(uint32_t));
    c->omm_any = any;
    c->omm_dirty = false;
}

// DXRPT_OPT_PACKED_TAPS: one RGBA8 unorm texture (normal.r, normal.g, metallic, roughness) per distinct
// (normal, metallic, roughness) triple of the geometries' materials that qualifies -- normal RGBA8 unorm,
// metallic and roughness R8 or RGBA8 unorm (their .r is what the shading reads), each either W x H or
// 1 x 1 -- in the tiled layout, appended to the device pool after `texels`.  A 1 x 1 map is a constant:
// its bilinear tap is lerp(c, c, f) = c for any finite weight, and a NaN / Inf weight (a NaN / Inf UV)
// is NaN at either size, so spreading it over W x H gives the same value.  Returns material index ->
// packed reference (whf with format kTexFmtPackedNMR), {0, 0} where the material keeps three taps.
std::vector<GeoTex> build_packed(dxrpt_ctx* c) {
    std::vector<GeoTex> out(c->mats.size(), GeoTex{0u, 0u});
    c->texels_packed.clear();
    c->packed_materials = c->packed_textures = 0;
    if (!(c->opt_packed & 1u)) return out;
    std::map<std::array<uint32_t, 3>, GeoTex> made;
    std::vector<bool> used(c->mats.size(), false);
    for (const dxrpt_geometry_info& g : c->geos)
        if (g.MaterialIdx < c->mats.size()) used[g.MaterialIdx] = true;
    const size_t nt = c->texdesc.size();
    auto unorm_r = [](const TexDesc& d) { return d.fmt == DXRPT_TEX_R8_UNORM || d.fmt == DXRPT_TEX_RGBA8_UNORM; };
    for (size_t mi = 0; mi < c->mats.size(); ++mi) {
        if (!used[mi]) continue;
        const dxrpt_material& m = c->mats[mi];
        if (m.Normal >= nt || m.Metallic >= nt || m.Roughness >= nt) continue;
        const TexDesc &N = c->texdesc[m.Normal], &M = c->texdesc[m.Metallic], &R = c->texdesc[m.Roughness];
        if (N.fmt != DXRPT_TEX_RGBA8_UNORM || !unorm_r(M) || !unorm_r(R)) continue;
        const uint32_t w = std::max({N.width, M.width, R.width}), h = std::max({N.height, M.height, R.height});
        auto fits = [&](const TexDesc& d) { return (d.width == w && d.height == h) || (d.width == 1 && d.height == 1); };
        if (!fits(N) || !fits(M) || !fits(R)) continue;
        const std::array<uint32_t, 3> key{m.Normal, m.Metallic, m.Roughness};
        auto it = made.find(key);
        if (it == made.end()) {
            const uint32_t tx32 = (w + kTexTileW32 - 1) / kTexTileW32, ty32 = (h + kTexTileH32 - 1) / kTexTileH32;
            const size_t at = c->texels_packed.size();
            const size_t base = c->texels.size() + at;
            require(base + size_t(tx32) * ty32 * kTexTileWords < (size_t(1) << 32),
                    "packed textures: texel pool exceeds 2^32 words");
            c->texels_packed.resize(at + size_t(tx32) * ty32 * kTexTileWords, 0u);
            // texel (x, y) of map d (its own tiling; a 1 x 1 map's only texel)
            auto word_of = [&](const TexDesc& d, uint32_t x, uint32_t y) {
                if (d.width == 1 && d.height == 1) x = y = 0;
                const uint32_t* T = c->texels.data() + d.offset;
                if (d.fmt == DXRPT_TEX_R8_UNORM) {
                    const uint32_t t8 = (d.width + kTexTileW8 - 1) / kTexTileW8;
                    return (T[tex_tile_word(x, y, t8, true)] >> (8u * (x & 3u))) & 0xFFu;
                }
                return T[tex_tile_word(x, y, (d.width + kTexTileW32 - 1) / kTexTileW32, false)];
            };
            uint32_t* dst = c->texels_packed.data() + at;
            for (uint32_t y = 0; y < h; ++y)
                for (uint32_t x = 0; x < w; ++x)
                    dst[tex_tile_word(x, y, tx32, false)] =
                        (word_of(N, x, y) & 0xFFFFu) | ((word_of(M, x, y) & 0xFFu) << 16) | ((word_of(R, x, y) & 0xFFu) << 24);
            it = made.emplace(key, GeoTex{uint32_t(base), w | (h << 15) | (kTexFmtPackedNMR << 30)}).first;
        }
        out[mi] = it->second;
        ++c->packed_materials;
    }
    c->packed_textures = uint32_t(made.size());
    return out;
}

void upload_textures(dxrpt_ctx* c) {
    const bool shade = c->geoshade_dirty && !c->geos.empty();
    if ((c->omm_dirty && c->opt_omm && c->bvh_built) || c->tex_dirty || shade) drain_frames(c);
    if (c->omm_dirty && c->opt_omm && c->bvh_built) build_omm(c);
    std::vector<GeoTex> packed;
    if (c->tex_dirty || shade) {
        // the texel pool: the added textures, then the packed ones of the current materials
        if (!c->geos.empty()) {
            packed = build_packed(c);
        } else {
            c->texels_packed.clear();
            c->packed_materials = c->packed_textures = 0;
        }
        const size_t n0 = c->texels.size() * sizeof(uint32_t), n1 = c->texels_packed.size() * sizeof(uint32_t);
        c->d_texels.ensure(n0 + n1);
        if (n0) HIP_CHECK(hipMemcpy(c->d_texels.p, c->texels.data(), n0, hipMemcpyHostToDevice));
        if (n1) HIP_CHECK(hipMemcpy(static_cast<char*>(c->d_texels.p) + n0, c->texels_packed.data(), n1, hipMemcpyHostToDevice));
        c->tex_dirty = false;
        c->geoshade_dirty = true;
    }
    if (!c->geoshade_dirty || c->geos.empty()) return;
    // per-geometry shading records (pt_layout.h GeoShade): GeometryInfo.MaterialIdx -> Material -> the
    // texture descriptors, resolved once on the host; a material index that names no added texture
    // resolves to "none" (the render path rejects such materials before it launches; an opacity of
    // DXRPT_INVALID_INDEX is the reference's "opaque")
    auto ref = [&](uint32_t t) {
        GeoTex g{0u, 0u};
        if (t < c->texdesc.size()) {
            const TexDesc& d = c->texdesc[t];
            g.offset = d.offset;
            g.whf = d.width | (d.height << 15) | (d.fmt << 30);
        }
        return g;
    };
    std::vector<GeoShade> gs(c->geos.size());
    c->inlined_refs = 0;
    for (size_t g = 0; g < c->geos.size(); ++g) {
        const uint32_t mi = c->geos[g].MaterialIdx;
        const dxrpt_material& m = c->mats[mi];
        gs[g] = GeoShade{ref(m.Albedo), ref(m.Normal), ref(m.Roughness), ref(m.Metallic), ref(m.Emissive), ref(m.Opacity)};
        if (mi < packed.size() && packed[mi].whf) gs[g].normal = packed[mi];  // (normal.rg, metallic, roughness)
        if (c->opt_packed & 2u)  // 1 x 1 maps inline (pt_layout.h GeoTex): their taps read no memory
            for (GeoTex* r : {&gs[g].albedo, &gs[g].normal, &gs[g].roughness, &gs[g].metallic, &gs[g].emissive}) {
                if ((r->whf & 0x3FFFFFFFu) != (1u | (1u << 15))) continue;
                const size_t n0 = c->texels.size();
                r->offset = r->offset < n0 ? c->texels[r->offset] : c->texels_packed[r->offset - n0];
                r->whf &= 0xC0000000u;  // width = height = 0, format kept
                ++c->inlined_refs;
            }
    }
    c->d_geoshade.upload(gs.data(), gs.size() * sizeof(GeoShade));
    c->geoshade_dirty = false;
}

// Do buffers for `paths` paths with `slots` shadow slots fit f?
bool frame_fits(const FrameBuffers& f, uint32_t paths, uint32_t slots) {
    return paths <= f.capacity && slots <= f.shadow_slots && f.counters;
}

// Queue + shadow-slot buffers of `f` for `paths` paths and `slots` shadow slots (grown, never shrunk).
// q: the two RayQueue parities; sh*: the shadow slots.
void alloc_frame(FrameBuffers& f, DevBuf (&q)[2][5], DevBuf& shorg, DevBuf& shdir, DevBuf& shcon, uint32_t paths,
                 uint32_t slots) {
    const uint32_t cap = std::max(paths, f.capacity);
    const uint32_t sl = std::max(slots, std::max(f.shadow_slots, 2u));
    const uint32_t cap_r = queue_shard_capacity(cap);
    const size_t qsize = size_t(kQueueShards) * cap_r;
    require(qsize * sl < (size_t(1) << 32), "frame too large for 32-bit shadow slot ids", DXRPT_E_INVALID_ARG);
    for (int b = 0; b < 2; ++b) {
        for (int k = 0; k < 4; ++k) q[b][k].ensure(qsize * 16);
        q[b][4].ensure(qsize * 4);
        f.q[b].org = q[b][0].as<float4>();
        f.q[b].dir = q[b][1].as<float4>();
        f.q[b].thr = q[b][2].as<float4>();
        f.q[b].rad = q[b][3].as<float4>();
        f.q[b].pix = q[b][4].as<uint32_t>();
    }
    shorg.ensure(qsize * sl * 16);
    shdir.ensure(qsize * sl * 16);
    shcon.ensure(qsize * sl * 16);
    f.sh_org = shorg.as<float4>();
    f.sh_dir = shdir.as<float4>();
    f.sh_con = shcon.as<float4>();
    f.capacity = cap;
    f.cap_r = cap_r;
    f.qsize = uint32_t(qsize);
    f.shadow_slots = sl;
}

// Buffers of work on the caller's stream (drains first when they grow: in-flight work may read them).
void ensure_frame(dxrpt_ctx* c, uint32_t paths, uint32_t slots) {
    FrameBuffers& f = c->fb;
    if (frame_fits(f, paths, slots)) return;
    drain_frames(c);
    alloc_frame(f, c->f_q, c->f_shorg, c->f_shdir, c->f_shcon, paths, slots);
    const size_t qsize = f.qsize, sl = f.shadow_slots;
    c->f_pix.ensure(size_t(f.capacity) * 8);
    c->f_pxrad.ensure(size_t(f.capacity) * 16);
    c->f_hit.ensure(qsize * 16);
    c->f_fwd.ensure(qsize * 4);
    c->f_shn.ensure(qsize * 4);
    c->f_shq.ensure(qsize * sl * 4);
    if (!c->f_counters.p) {  // two counter sets (ping-pong across megakernel frames), both dirty at first
        c->f_counters.ensure(2 * kCounterWords * sizeof(uint32_t));
        c->ctr_clean[0] = c->ctr_clean[1] = false;
    }
    f.ps_pix = c->f_pix.as<uint2>();
    f.px_rad = c->f_pxrad.as<float4>();
    f.hit = c->f_hit.as<float4>();
    f.fwd = c->f_fwd.as<uint32_t>();
    f.sh_n = c->f_shn.as<uint32_t>();
    f.sh_queue = c->f_shq.as<uint32_t>();
    f.counters = c->f_counters.as<uint32_t>() + c->ctr_set * kCounterWords;
}

// Overlap slot k (stream, events, queues, shadow slots, counters, stage) for `paths` paths; drains first
// when a buffer grows.
void ensure_slot(dxrpt_ctx* c, uint32_t k, uint32_t paths, uint32_t slots, size_t stage_bytes) {
    dxrpt_ctx::Slot& P = c->slot[k];
    if (!P.stream) {
        HIP_CHECK(hipStreamCreateWithFlags(&P.stream, hipStreamNonBlocking));
        HIP_CHECK(hipEventCreateWithFlags(&P.done, hipEventDisableTiming));
        HIP_CHECK(hipEventCreateWithFlags(&P.stage_free, hipEventDisableTiming));
    }
    if (!c->ovl_fork) HIP_CHECK(hipEventCreateWithFlags(&c->ovl_fork, hipEventDisableTiming));
    if (!c->ovl_gate) HIP_CHECK(hipEventCreateWithFlags(&c->ovl_gate, hipEventDisableTiming));
    const bool fits = frame_fits(P.fb, paths, slots) && P.stage.bytes >= stage_bytes;
    if (fits) return;
    drain_frames(c);
    if (!frame_fits(P.fb, paths, slots)) {
        alloc_frame(P.fb, P.q, P.shorg, P.shdir, P.shcon, paths, slots);
        if (!P.counters.p) {
            P.counters.ensure(2 * kCounterWords * sizeof(uint32_t));
            P.ctr_clean[0] = P.ctr_clean[1] = false;
            P.fb.counters = P.counters.as<uint32_t>();
        }
    }
    P.stage.ensure(stage_bytes);
}

// Adds one timed frame's event intervals to the per-kernel sums (blocks until the frame is done).
void harvest(dxrpt_ctx* c, dxrpt_ctx::FrameEvents& f) {
    if (!f.pending) return;
    HIP_CHECK(hipEventSynchronize(f.ev[f.mega ? 1 : frame_event_count(f.L) - 1]));
    auto span = [&](int a, int b) {
        float ms = 0.f;
        HIP_CHECK(hipEventElapsedTime(&ms, f.ev[a], f.ev[b]));
        return double(ms);
    };
    if (f.mega) {
        if ((f.mask >> DXRPT_K_PATH) & 1u) {
            c->kernel_ms[DXRPT_K_PATH] += span(0, 1);
            c->kernel_launches[DXRPT_K_PATH]++;
        }
        if (f.split) {  // the head, then the tails back to back on the same stream
            if ((f.mask >> DXRPT_K_PATH_HEAD) & 1u) {
                c->kernel_ms[DXRPT_K_PATH_HEAD] += span(0, 2);
                c->kernel_launches[DXRPT_K_PATH_HEAD]++;
            }
            if ((f.mask >> DXRPT_K_PATH_TAIL) & 1u && f.L > 2) {
                c->kernel_ms[DXRPT_K_PATH_TAIL] += span(2, 1);
                c->kernel_launches[DXRPT_K_PATH_TAIL] += uint64_t(f.L - 2);
            }
        }
        c->frame_ms += span(0, 1);
        c->timed_frames++;
        f.pending = false;
        return;
    }
    auto slot = [&](int i) { return span(2 * i, 2 * i + 1); };
    auto add = [&](int kind, int i) {
        if (!((f.mask >> kind) & 1u)) return;
        c->kernel_ms[kind] += slot(i);
        c->kernel_launches[kind]++;
    };
    add(DXRPT_K_RAYGEN, 0);
    static const int kinds[4] = {DXRPT_K_TRACE, DXRPT_K_SHADE, DXRPT_K_SHADOW, DXRPT_K_RESOLVE};
    for (int d = 1; d <= f.L - 1; ++d)
        for (int k = 0; k < 4; ++k) add(kinds[k], 1 + 4 * (d - 1) + k);
    const int acc = 1 + 4 * (f.L - 1);
    add(DXRPT_K_ACCUMULATE, acc);
    const int e = 2 * acc;
    c->frame_ms += span(0, e + 1);
    c->timed_frames++;
    f.pending = false;
}

void harvest_all(dxrpt_ctx* c) {
    for (auto& f : c->ring) harvest(c, f);
}

}  // namespace

// f(i) for i in [0, n) on up to `threads` host threads in contiguous chunks (the BVH build's per-triangle
// record and vertex copies; each i writes only its own outputs).
template <class F>
static void host_parallel(uint32_t n, unsigned threads, F&& f) {
    const unsigned k = std::max(1u, std::min(threads, n / 16384u));
    if (k <= 1) {
        for (uint32_t i = 0; i < n; ++i) f(i);
        return;
    }
    std::vector<std::thread> th;
    for (unsigned j = 1; j < k; ++j)
        th.emplace_back([&, j] {
            for (uint32_t i = uint32_t(uint64_t(n) * j / k); i < uint32_t(uint64_t(n) * (j + 1) / k); ++i) f(i);
        });
    for (uint32_t i = 0; i < uint32_t(uint64_t(n) / k); ++i) f(i);
    for (std::thread& t : th) t.join();
}

extern "C" {

int dxrpt_abi_version(void) { return DXRPT_ABI_VERSION; }

void dxrpt_default_settings(dxrpt_app_settings* s) {
    if (!s) return;
    std::memset(s, 0, sizeof(*s));
    // AppSettings.cpp:95-208
    s->EnableSun = 1;
    s->EnableSky = 1;
    s->SunAreaLightApproximation = 1;
    s->SunSize = 1.0f;
    s->SunDirection[0] = 0.26f;
    s->SunDirection[1] = 0.987f;
    s->SunDirection[2] = -0.16f;
    s->MSAAMode = 2;  // MSAA4x (raster only)
    s->RenderLights = 1;
    s->EnableRayTracing = 1;
    s->ClampRoughness = 0;
    s->AvoidCausticPaths = 0;
    s->SqrtNumSamples = 4;
    s->MaxPathLength = 3;
    s->MaxAnyHitPathLength = 1;
    s->Exposure = -14.0f;
    s->BloomExposure = -4.0f;
    s->BloomMagnitude = 1.0f;
    s->BloomBlurSigma = 2.5f;
    s->EnableAlbedoMaps = 1;
    s->EnableNormalMaps = 1;
    s->EnableDiffuse = 1;
    s->EnableSpecular = 1;
    s->EnableDirect = 1;
    s->EnableIndirect = 1;
    s->EnableIndirectSpecular = 0;
    s->ApplyMultiscatteringEnergyCompensation = 1;
    s->RoughnessScale = 1.0f;
    s->MetallicScale = 1.0f;
    s->EnableWhiteFurnaceMode = 0;
    s->EnableLightMapRender = 1;
}

int dxrpt_create(int hip_device, dxrpt_ctx** out_ctx) {
    if (!out_ctx) return DXRPT_E_INVALID_ARG;
    *out_ctx = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return DXRPT_E_NO_DEVICE;
    if (hip_device < 0 || hip_device >= n) return DXRPT_E_INVALID_ARG;
    dxrpt_ctx* c = new (std::nothrow) dxrpt_ctx();
    if (!c) return DXRPT_E_OOM;
    c->device = hip_device;
    int rc = guarded(c, [&] {
        hipDeviceProp_t prop;
        HIP_CHECK(hipGetDeviceProperties(&prop, hip_device));
        require(std::strncmp(prop.gcnArchName, "gfx9", 4) == 0,
                std::string("unsupported device architecture ") + prop.gcnArchName, DXRPT_E_UNSUPPORTED);
        require(prop.sharedMemPerBlock >= 64 * 1024, "device LDS per workgroup < 64 KiB", DXRPT_E_UNSUPPORTED);
        c->num_cus = uint32_t(prop.multiProcessorCount);
        std::vector<float> lut = make_lut();
        c->d_lut.upload(lut.data(), lut.size() * sizeof(float));
    });
    if (rc != DXRPT_OK) {
        delete c;
        return rc;
    }
    *out_ctx = c;
    return DXRPT_OK;
}

int dxrpt_destroy(dxrpt_ctx* ctx) {
    if (!ctx) return DXRPT_E_INVALID_ARG;
    (void)hipSetDevice(ctx->device);
    delete ctx;
    return DXRPT_OK;
}

const char* dxrpt_last_error(const dxrpt_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

// include/dxrpt.h DXRPT_RETIRED_OPTIONS: the one list of retired ids
static bool option_retired(uint32_t option) {
    static const uint32_t kRetired[] = DXRPT_RETIRED_OPTIONS;
    for (uint32_t r : kRetired)
        if (r == option) return true;
    return false;
}

int dxrpt_set_option(dxrpt_ctx* ctx, uint32_t option, uint64_t value) {
    if (!ctx) return DXRPT_E_INVALID_ARG;
    return guarded(ctx, [&] {
        if (option == DXRPT_OPT_COUNT_TRAVERSAL) {
            ctx->opt_count = value != 0;
            if (ctx->opt_count) ctx->d_trav.ensure(kTravCounters * sizeof(unsigned long long));
        } else if (option == DXRPT_OPT_KERNEL_TIMING) {
            ctx->opt_timing = value != 0;
        } else if (option == DXRPT_OPT_SPATIAL_SPLITS) {
            require(value <= 400, "dxrpt_set_option: spatial-split budget must be 0..400 (percent of triangles)");
            ctx->build_params.spatial_splits = value > 100;
            ctx->build_params.ref_budget = double(value) / 100.0;
        } else if (option == DXRPT_OPT_LEAF_COST) {
            require(value >= 5 && value <= 1000, "dxrpt_set_option: leaf cost must be 5..1000 (percent of a node visit)");
            ctx->build_params.leaf_cost = double(value) / 100.0;
        } else if (option == DXRPT_OPT_PACKET_TRAVERSAL) {
            require(value <= 15, "dxrpt_set_option: packet traversal mask must be 0..15");
            ctx->opt_packet = uint32_t(value);
        } else if (option == DXRPT_OPT_KERNEL_TIMING_MASK) {
            require(value != 0 && value < (1u << DXRPT_K_COUNT), "dxrpt_set_option: timing mask must select kernel kinds");
            ctx->opt_timing_mask = uint32_t(value);
        } else if (option == DXRPT_OPT_WAVE_CLOCKS) {
            ctx->opt_wave_clocks = value != 0;
        } else if (option == DXRPT_OPT_WAVE_ORDER) {
            require(value <= 2, "dxrpt_set_option: wave order must be 0, 1 or 2");
            drain_frames(ctx);  // an in-flight frame may read the order
            ctx->opt_wave_order = uint32_t(value);
            ctx->order_ready = false;
        } else if (option == DXRPT_OPT_XCD_CHUNK) {
            require(value <= 4096, "dxrpt_set_option: XCD chunk must be 0..4096 blocks");
            ctx->opt_xcd_chunk = uint32_t(value);
        } else if (option == DXRPT_OPT_WAVE_ORDER_PERIOD) {
            require(value >= 1 && value <= 1024, "dxrpt_set_option: wave order period must be 1..1024 frames");
            ctx->opt_order_period = uint32_t(value);
        } else if (option == DXRPT_OPT_MEGAKERNEL_PATHS) {
            ctx->opt_mega_paths = value > 0xFFFFFFFFull ? 0xFFFFFFFFu : uint32_t(value);
        } else if (option == DXRPT_OPT_MEGAKERNEL_OCCUPANCY) {
            require(value == 0 || (value >= 4 && value <= 7), "dxrpt_set_option: megakernel occupancy must be 0 or 4..7");
            ctx->opt_mega_occ = uint32_t(value);
        } else if (option == DXRPT_OPT_TAIL_OCCUPANCY) {
            require(value == 0 || (value >= 4 && value <= 7), "dxrpt_set_option: tail occupancy must be 0 or 4..7");
            ctx->opt_tail_occ = uint32_t(value);
        } else if (option == DXRPT_OPT_BAKE_CHUNK) {
            require(value >= 64 && value <= (1u << 26), "dxrpt_set_option: bake chunk must be 64..2^26 texels");
            ctx->opt_bake_chunk = uint32_t(value);
        } else if (option == DXRPT_OPT_MEGAKERNEL_SPLIT) {
            require(value <= 2, "dxrpt_set_option: megakernel split must be 0 (off), 1 (on) or 2 (by frame size)");
            ctx->opt_split = uint32_t(value);
        } else if (option == DXRPT_OPT_FRAME_OVERLAP) {
            require(value <= kOverlapBySize,
                    "dxrpt_set_option: frame overlap must be 0 (off), 1 (two frames in flight), 2 (three) or 3 (by frame size)");
            if (uint32_t(value) != ctx->opt_overlap) {  // the slot rotation restarts
                drain_frames(ctx);
                ctx->ovl_parity = 0;
            }
            ctx->opt_overlap = uint32_t(value);
        } else if (option == DXRPT_OPT_TREELET_PASSES) {
            require(value <= 8, "dxrpt_set_option: treelet passes must be 0..8");
            ctx->build_params.treelet_passes = uint32_t(value);
        } else if (option == DXRPT_OPT_OPACITY_MICROMAP) {
            require(value <= 1, "dxrpt_set_option: opacity micromap must be 0 (off) or 1 (on)");
            drain_frames(ctx);  // in-flight frames may read the micromap
            ctx->opt_omm = uint32_t(value);
        } else if (option == DXRPT_OPT_PACKED_TAPS) {
            require(value <= 3, "dxrpt_set_option: packed taps must be 0..3 (bit 0: packed maps, bit 1: inlined 1 x 1 maps)");
            if (uint32_t(value) != ctx->opt_packed) {  // the shading records (and the packed texels) change
                drain_frames(ctx);
                ctx->opt_packed = uint32_t(value);
                ctx->tex_dirty = true;
                ctx->geoshade_dirty = true;
            }
        } else if (option == DXRPT_OPT_BVH_THREADS) {
            require(value <= 256, "dxrpt_set_option: BVH build threads must be 0 (default) or 1..256");
            ctx->build_params.threads = unsigned(value);
        } else if (option_retired(option)) {
            throw ApiError(DXRPT_E_UNSUPPORTED, "dxrpt_set_option: option " + std::to_string(option) +
                                                    " was retired in ABI 3 (measured slower or neutral; DESIGN.md §7a)");
        } else {
            throw ApiError(DXRPT_E_INVALID_ARG, "dxrpt_set_option: unknown option " + std::to_string(option));
        }
    });
}

int dxrpt_reset_timing(dxrpt_ctx* ctx) {
    if (!ctx) return DXRPT_E_INVALID_ARG;
    return guarded(ctx, [&] {
        harvest_all(ctx);
        for (int k = 0; k < DXRPT_K_COUNT; ++k) {
            ctx->kernel_ms[k] = 0.0;
            ctx->kernel_launches[k] = 0;
        }
        ctx->timed_frames = 0;
        ctx->frame_ms = 0.0;
    });
}

int dxrpt_set_scene(dxrpt_ctx* ctx, const dxrpt_mesh_vertex* vertices, uint32_t num_vertices, const void* indices,
                    uint32_t idx_bytes, uint32_t num_indices, const dxrpt_geometry_info* geometries,
                    uint32_t num_geometries, const dxrpt_material* materials, uint32_t num_materials) {
    if (!ctx) return DXRPT_E_INVALID_ARG;
    return guarded(ctx, [&] {
        drain_frames(ctx);
        require(vertices && indices && geometries && materials, "dxrpt_set_scene: null array");
        require(idx_bytes == 2 || idx_bytes == 4, "dxrpt_set_scene: idx_bytes must be 2 or 4");
        require(num_indices % 3 == 0 && num_indices > 0, "dxrpt_set_scene: num_indices must be a positive multiple of 3");
        require(num_geometries > 0 && num_materials > 0, "dxrpt_set_scene: empty geometry/material table");
        ctx->vertices.assign(vertices, vertices + num_vertices);
        ctx->indices.resize(num_indices);
        if (idx_bytes == 2) {
            const uint16_t* s = static_cast<const uint16_t*>(indices);
            for (uint32_t i = 0; i < num_indices; ++i) ctx->indices[i] = s[i];
        } else {
            std::memcpy(ctx->indices.data(), indices, size_t(num_indices) * 4);
        }
        ctx->geos.assign(geometries, geometries + num_geometries);
        ctx->mats.assign(materials, materials + num_materials);
        for (uint32_t g = 0; g < num_geometries; ++g) {
            const dxrpt_geometry_info& gi = geometries[g];
            require(gi.IdxOffset % 3 == 0 && gi.IdxOffset < num_indices, "dxrpt_set_scene: bad IdxOffset in geometry " + std::to_string(g));
            require(gi.MaterialIdx < num_materials, "dxrpt_set_scene: bad MaterialIdx in geometry " + std::to_string(g));
        }
        ctx->geoshade_dirty = true;
        ctx->omm_dirty = true;
        ctx->scene_set = true;
        ctx->bvh_built = false;
    });
}

int dxrpt_add_texture(dxrpt_ctx* ctx, uint32_t w, uint32_t h, uint32_t fmt, const void* texels, uint32_t* out_index) {
    if (!ctx) return DXRPT_E_INVALID_ARG;
    return guarded(ctx, [&] {
        drain_frames(ctx);
        require(texels && w > 0 && h > 0, "dxrpt_add_texture: empty texture");
        require(w <= 16384 && h <= 16384, "dxrpt_add_texture: texture larger than 16384");
        require(fmt <= DXRPT_TEX_R8_UNORM, "dxrpt_add_texture: unknown format");
        TexDesc d;
        d.offset = uint32_t(ctx->texels.size());
        d.width = w;
        d.height = h;
        d.fmt = fmt;
        // 128-B tiles (pt_layout.h TexDesc): a bilinear footprint usually falls in one cache line
        const bool r8 = fmt == DXRPT_TEX_R8_UNORM;
        const uint32_t tw = r8 ? kTexTileW8 : kTexTileW32, th = r8 ? kTexTileH8 : kTexTileH32;
        const uint32_t tiles_x = (w + tw - 1) / tw, tiles_y = (h + th - 1) / th;
        const size_t at = ctx->texels.size();
        ctx->texels.resize(at + size_t(tiles_x) * tiles_y * kTexTileWords, 0u);
        uint32_t* dst = ctx->texels.data() + at;
        for (uint32_t y = 0; y < h; ++y)
            for (uint32_t x = 0; x < w; ++x) {
                const size_t word = tex_tile_word(x, y, tiles_x, r8);
                if (r8) {
                    const uint32_t b = static_cast<const uint8_t*>(texels)[size_t(y) * w + x];
                    dst[word] |= b << (8u * (x & 3u));
                } else {
                    dst[word] = static_cast<const uint32_t*>(texels)[size_t(y) * w + x];
                }
            }
        require(ctx->texels.size() < (size_t(1) << 32), "dxrpt_add_texture: texel pool exceeds 2^32 words");
        if (out_index) *out_index = uint32_t(ctx->texdesc.size());
        ctx->texdesc.push_back(d);
        ctx->tex_dirty = true;
        ctx->omm_dirty = true;
    });
}

int dxrpt_set_sky(dxrpt_ctx* ctx, const uint16_t* cube, uint32_t res) {
    if (!ctx) return DXRPT_E_INVALID_ARG;
    return guarded(ctx, [&] {
        drain_frames(ctx);
        require(cube && res > 0 && res <= 4096, "dxrpt_set_sky: bad cube");
        ctx->d_sky.upload(cube, size_t(res) * res * 6 * 4 * sizeof(uint16_t));
        ctx->sky_res = res;
        ctx->sky_set = true;
    });
}

int dxrpt_build_bvh(dxrpt_ctx* ctx) {
    if (!ctx) return DXRPT_E_INVALID_ARG;
    return guarded(ctx, [&] {
        drain_frames(ctx);
        require(ctx->scene_set, "dxrpt_build_bvh: no scene (call dxrpt_set_scene first)", DXRPT_E_STATE);
        auto t0 = std::chrono::steady_clock::now();
        // Global triangle list: gtri = IdxOffset/3 + PrimitiveIndex for every geometry.
        const uint32_t ntris = uint32_t(ctx->indices.size() / 3);
        std::vector<uint32_t> tri_geom(ntris, 0xFFFFFFFFu);
        const uint32_t ng = uint32_t(ctx->geos.size());
        for (uint32_t g = 0; g < ng; ++g) {
            uint32_t begin = ctx->geos[g].IdxOffset / 3;
            uint32_t end = (g + 1 < ng) ? ctx->geos[g + 1].IdxOffset / 3 : ntris;
            require(end >= begin, "dxrpt_build_bvh: geometries must be sorted by IdxOffset");
            for (uint32_t t = begin; t < end; ++t) tri_geom[t] = g;
        }
        for (uint32_t t = 0; t < ntris; ++t) {
            require(tri_geom[t] != 0xFFFFFFFFu, "dxrpt_build_bvh: triangle not covered by any geometry");
            for (int k = 0; k < 3; ++k)
                require(ctx->indices[size_t(t) * 3 + k] + uint64_t(ctx->geos[tri_geom[t]].VtxOffset) < ctx->vertices.size(),
                        "dxrpt_build_bvh: index out of range");
        }
        const unsigned threads = ctx->build_params.threads ? ctx->build_params.threads
                                                          : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        std::vector<float> pos(size_t(ntris) * 9);
        host_parallel(ntris, threads, [&](uint32_t t) {
            const uint32_t g = tri_geom[t];
            for (int k = 0; k < 3; ++k)
                std::memcpy(&pos[size_t(t) * 9 + k * 3], ctx->vertices[ctx->indices[size_t(t) * 3 + k] + ctx->geos[g].VtxOffset].Position, 12);
        });
        BvhBuildResult res;
        std::string err;
        // spatial splits leave alpha-tested triangles whole: each extra reference of one is another
        // AnyHitShader opacity test (r03: SAH 67.5 -> 63.1 on the Sponza proxy, metric -2.4 %, C4 -1.3 %)
        std::vector<uint8_t> alpha_tri(ntris);
        for (uint32_t t = 0; t < ntris; ++t)
            alpha_tri[t] = ctx->mats[ctx->geos[tri_geom[t]].MaterialIdx].Opacity != DXRPT_INVALID_INDEX ? 1u : 0u;
        BvhBuildParams bp = ctx->build_params;
        bp.keep_whole = alpha_tri.data();
        if (!build_bvh(pos.data(), ntris, 8, res, err, &bp)) throw ApiError(DXRPT_E_INVALID_ARG, err);
        // one record per leaf reference (spatial splits may reference a triangle more than once)
        const uint32_t nrefs = uint32_t(res.tri_order.size());
        // opacity micromap slots: the triangles of alpha-tested geometry in global order
        std::vector<uint32_t> slot_of(ntris, 0u);
        ctx->omm_tris.clear();
        for (uint32_t t = 0; t < ntris; ++t)
            if (alpha_tri[t]) {
                slot_of[t] = uint32_t(ctx->omm_tris.size());
                ctx->omm_tris.push_back(t);
            }
        // the kernels address node and triangle records by 32-bit byte offsets (pt_kernels.hip DXRPT_ADDR32)
        require(res.nodes8.size() * size_t(kNode8Stride) < (size_t(1) << 32) && size_t(nrefs) * sizeof(TriRecord) < (size_t(1) << 32),
                "dxrpt_build_bvh: the BVH's node or triangle-record array reaches 4 GiB (32-bit record offsets)");
        std::vector<TriRecord> tris(nrefs);
        host_parallel(nrefs, threads, [&](uint32_t i) {
            const uint32_t t = res.tri_order[i];
            const float* v = &pos[size_t(t) * 9];
            TriRecord& r = tris[i];
            const uint32_t g = tri_geom[t];
            uint32_t flags = alpha_tri[t] ? slot_of[t] << 1 : kTriOpaque;
            r.p0[0] = v[0]; r.p0[1] = v[1]; r.p0[2] = v[2];
            r.p1[0] = v[3] - v[0]; r.p1[1] = v[4] - v[1]; r.p1[2] = v[5] - v[2];
            r.p2[0] = v[6] - v[0]; r.p2[1] = v[7] - v[1]; r.p2[2] = v[8] - v[2];
            std::memcpy(&r.p0[3], &t, 4);
            std::memcpy(&r.p1[3], &g, 4);
            std::memcpy(&r.p2[3], &flags, 4);
        });
        if (kNode8Stride == sizeof(Bvh8Node)) {
            ctx->d_nodes8.upload(res.nodes8.data(), res.nodes8.size() * sizeof(Bvh8Node));
        } else {  // padded device layout (pt_layout.h kNode8Stride)
            std::vector<uint8_t> padded(res.nodes8.size() * size_t(kNode8Stride), 0u);
            for (size_t i = 0; i < res.nodes8.size(); ++i)
                std::memcpy(padded.data() + i * kNode8Stride, &res.nodes8[i], sizeof(Bvh8Node));
            ctx->d_nodes8.upload(padded.data(), padded.size());
        }
        ctx->d_tris.upload(tris.data(), tris.size() * sizeof(TriRecord));
        {   // shading-side copy of each triangle's vertices: one contiguous 192-B record per gtri, so a
            // hit gathers 2 cache lines in one round trip instead of 3 indices then 3 vertices
            std::vector<dxrpt_mesh_vertex> tv(size_t(ntris) * 3);
            host_parallel(ntris, threads, [&](uint32_t t) {
                for (int k = 0; k < 3; ++k)
                    tv[size_t(t) * 3 + k] = ctx->vertices[ctx->indices[size_t(t) * 3 + k] + ctx->geos[tri_geom[t]].VtxOffset];
            });
            ctx->d_tri_verts.upload(tv.data(), tv.size() * sizeof(dxrpt_mesh_vertex));
        }
        auto t1 = std::chrono::steady_clock::now();
        ctx->bvh = dxrpt_bvh_info{};
        ctx->bvh.num_nodes = uint32_t(res.nodes8.size());
        ctx->bvh.num_leaves = res.num_leaves;
        ctx->bvh.num_tris = ntris;
        ctx->bvh.max_depth = res.max_depth;
        ctx->bvh.node_bytes = uint32_t(sizeof(Bvh8Node));
        ctx->bvh.width = 8u;
        ctx->bvh.tri_bytes = sizeof(TriRecord);
        ctx->bvh.build_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        ctx->bvh.sah_cost = res.sah_cost;
        ctx->bvh.num_refs = nrefs;
        for (int k = 0; k < 3; ++k) ctx->bvh.phase_ms[k] = res.phase_ms[k];
        ctx->bvh.phase_ms[3] = std::max(0.0, ctx->bvh.build_ms - res.phase_ms[0] - res.phase_ms[1] - res.phase_ms[2]);
        ctx->bvh.wide_sah = res.wide_sah;
        ctx->bvh.binary_depth_cap = res.binary_depth_cap;
        ctx->bvh.treelet_passes = res.treelet_passes;
        ctx->bvh.threads = bp.threads ? bp.threads : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        ctx->bvh.ref_budget_pct = bp.spatial_splits ? uint32_t(bp.ref_budget * 100.0 + 0.5) : 0u;
        ctx->spill_threads = 0;  // the depth may have changed: the next launch re-sizes the spill slabs
        ctx->bvh_built = true;
        ctx->omm_dirty = true;
        ctx->omm_any = false;
    });
}

int dxrpt_get_bvh_info(const dxrpt_ctx* ctx, dxrpt_bvh_info* info) {
    if (!ctx || !info) return DXRPT_E_INVALID_ARG;
    if (!ctx->bvh_built) return DXRPT_E_STATE;
    *info = ctx->bvh;
    return DXRPT_OK;
}

// The call's tile list (NULL: the full frame) validated and uploaded with its pixel prefix sums (only when it
// changed); returns the number of paths (pixels).  Tiles of zero area are valid and dropped; a list with no
// pixels at all returns 0 before touching the device (the caller then enqueues nothing).
uint32_t prepare_tiles(dxrpt_ctx* ctx, const dxrpt_tile* tiles, uint32_t num_tiles, uint32_t width, uint32_t height,
                       const char* who) {
    std::vector<dxrpt_tile> tl;
    if (!tiles) {
        dxrpt_tile t{};
        t.x0 = 0; t.y0 = 0; t.w = width; t.h = height; t.accum_offset = 0; t.accum_pitch = width;
        tl.push_back(t);
    } else {
        for (uint32_t k = 0; k < num_tiles; ++k) {
            const dxrpt_tile& t = tiles[k];
            require(uint64_t(t.x0) + t.w <= width && uint64_t(t.y0) + t.h <= height,
                    std::string(who) + ": tile " + std::to_string(k) + " outside the image");
            if (t.w > 0 && t.h > 0) tl.push_back(t);
        }
        if (tl.empty()) return 0u;
    }
    std::vector<uint32_t> prefix(tl.size() + 1, 0);
    uint64_t total = 0;
    for (size_t k = 0; k < tl.size(); ++k) {
        const dxrpt_tile& t = tl[k];
        require(t.w > 0 && t.h > 0 && uint64_t(t.x0) + t.w <= width && uint64_t(t.y0) + t.h <= height,
                std::string(who) + ": tile " + std::to_string(k) + " outside the image");
        require(t.accum_pitch >= t.w, std::string(who) + ": tile accum_pitch < width");
        require(t.accum_offset + uint64_t(t.h - 1) * t.accum_pitch + t.w <= 0xFFFFFFFFull,
                std::string(who) + ": accumulation index exceeds 32 bits");
        prefix[k] = uint32_t(total);
        total += uint64_t(t.w) * t.h;
        require(total < 0x7FFFFFFFull, std::string(who) + ": too many pixels in one call");
    }
    prefix[tl.size()] = uint32_t(total);
    uint64_t extent = 0;
    for (const dxrpt_tile& t : tl) extent = std::max<uint64_t>(extent, t.accum_offset + uint64_t(t.h - 1) * t.accum_pitch + t.w);
    ctx->accum_extent = uint32_t(extent);
    if (tl.size() != ctx->tiles_cache.size() || std::memcmp(tl.data(), ctx->tiles_cache.data(), tl.size() * sizeof(dxrpt_tile)) != 0) {
        drain_frames(ctx);
        ctx->d_tiles.upload(tl.data(), tl.size() * sizeof(dxrpt_tile));
        ctx->d_tile_prefix.upload(prefix.data(), prefix.size() * sizeof(uint32_t));
        ctx->tiles_cache = tl;
        ++ctx->tiles_gen;
    }
    return uint32_t(total);
}

int dxrpt_render_aov(dxrpt_ctx* ctx, const dxrpt_ray_trace_constants* rtc, const dxrpt_app_settings* settings, float* out,
                     uint32_t width, uint32_t height, const dxrpt_tile* tiles, uint32_t num_tiles, void* stream) {
    if (!ctx) return DXRPT_E_INVALID_ARG;
    return guarded(ctx, [&] {
        require(ctx->bvh_built, "dxrpt_render_aov: acceleration structure not built", DXRPT_E_STATE);
        require(rtc && settings && out, "dxrpt_render_aov: null argument");
        require(width > 0 && height > 0, "dxrpt_render_aov: empty image");
        require(uint64_t(width) * height == rtc->TotalNumPixels, "dxrpt_render_aov: TotalNumPixels != width*height");
        require(settings->SqrtNumSamples >= 1, "dxrpt_render_aov: SqrtNumSamples must be >= 1");
        const hipStream_t s = static_cast<hipStream_t>(stream);
        enter_stream(ctx, s);
        upload_textures(ctx);
        const uint32_t paths = prepare_tiles(ctx, tiles, num_tiles, width, height, "dxrpt_render_aov");
        if (paths == 0u) return;  // a tile list without pixels: nothing to do
        ensure_spill(ctx, frame_traversal_threads(paths, 1u, true));
        FrameParams fp{};
        fp.rtc = *rtc;
        fp.set = *settings;
        fp.tiles = ctx->d_tiles.as<dxrpt_tile>();
        fp.tile_prefix = ctx->d_tile_prefix.as<uint32_t>();
        fp.accum = reinterpret_cast<float4*>(out);
        fp.num_tiles = uint32_t(ctx->tiles_cache.size());
        fp.num_paths = paths;
        fp.width = width;
        fp.height = height;
        fp.packet = ctx->opt_packet;
        HIP_CHECK(launch_primary_aov(scene_dev(ctx, 0), ctx->fb, fp, s));
        ctx->ovl_active = false;  // the next overlapped frame starts behind this call (slab 0)
        ctx->inflight = true;
    });
}

int dxrpt_render(dxrpt_ctx* ctx, const dxrpt_ray_trace_constants* rtc, const dxrpt_app_settings* settings,
                 const dxrpt_light_constants* lights, float* accum, uint32_t width, uint32_t height,
                 const dxrpt_tile* tiles, uint32_t num_tiles, void* stream) {
    if (!ctx) return DXRPT_E_INVALID_ARG;
    return guarded(ctx, [&] {
        require(ctx->bvh_built, "dxrpt_render: acceleration structure not built", DXRPT_E_STATE);
        require(ctx->sky_set, "dxrpt_render: sky cubemap not set", DXRPT_E_STATE);
        require(rtc && settings && accum, "dxrpt_render: null argument");
        require(width > 0 && height > 0, "dxrpt_render: empty image");
        require(uint64_t(width) * height == rtc->TotalNumPixels, "dxrpt_render: TotalNumPixels != width*height");
        require(settings->SqrtNumSamples >= 1, "dxrpt_render: SqrtNumSamples must be >= 1");
        require(settings->MaxPathLength >= 1 && settings->MaxPathLength <= int(DXRPT_MAX_PATH_LENGTH),
                "dxrpt_render: MaxPathLength must be in [1, 8]");
        const bool useLights = settings->RenderLights && rtc->NumLights > 0;
        require(!useLights || (lights && rtc->NumLights <= DXRPT_MAX_SPOT_LIGHTS), "dxrpt_render: bad lights");
        for (const dxrpt_material& m : ctx->mats) {
            const uint32_t nt = uint32_t(ctx->texdesc.size());
            require(m.Albedo < nt && m.Normal < nt && m.Roughness < nt && m.Metallic < nt && m.Emissive < nt &&
                        (m.Opacity == DXRPT_INVALID_INDEX || m.Opacity < nt),
                    "dxrpt_render: material references a texture that was not added");
        }
        const hipStream_t s = static_cast<hipStream_t>(stream);
        enter_stream(ctx, s);
        upload_textures(ctx);
        const uint32_t paths = prepare_tiles(ctx, tiles, num_tiles, width, height, "dxrpt_render");
        if (paths == 0u) {  // a tile list without pixels (e.g. a rank of a tiny frame): nothing to do, and the
                            // stats of this call are empty (not the previous frame's)
            std::memset(&ctx->last, 0, sizeof(ctx->last));
            ctx->last_L = 0;
            ctx->last_counted = false;
            ctx->stat_counters.clear();
            ctx->rendered = true;
            return;
        }
        const uint32_t nl = useLights ? rtc->NumLights : 0u;
        if (nl) {
            std::vector<dxrpt_spot_light> L(lights->Lights, lights->Lights + nl);
            if (L.size() != ctx->lights_cache.size() || std::memcmp(L.data(), ctx->lights_cache.data(), nl * sizeof(dxrpt_spot_light)) != 0) {
                drain_frames(ctx);
                ctx->d_lights.upload(L.data(), nl * sizeof(dxrpt_spot_light));
                ctx->lights_cache = L;
            }
        }
        const uint32_t slots = 2u + nl;  // shadow slots per vertex: sun, spot lights, final sky visibility
        const int L = settings->MaxPathLength < 2 ? 2 : settings->MaxPathLength;
        FrameParams fp{};
        fp.rtc = *rtc;
        fp.rtc.NumLights = nl;
        fp.set = *settings;
        fp.lights = nl ? ctx->d_lights.as<dxrpt_spot_light>() : nullptr;
        fp.tiles = ctx->d_tiles.as<dxrpt_tile>();
        fp.tile_prefix = ctx->d_tile_prefix.as<uint32_t>();
        fp.accum = reinterpret_cast<float4*>(accum);
        fp.num_tiles = uint32_t(ctx->tiles_cache.size());
        fp.num_paths = paths;
        fp.accum_extent = ctx->accum_extent;
        fp.width = width;
        fp.height = height;
        fp.xcd_chunk = ctx->opt_xcd_chunk;
        fp.packet = ctx->opt_packet;
        fp.timing_mask = ctx->opt_timing_mask;
        fp.num_cus = ctx->num_cus;
        // megakernel schedules for every frame by default: DXRPT_OPT_MEGAKERNEL_PATHS bounds them by path
        // vertices = paths x (L-1); the wavefront passes (the north star's per-stage kernels) stay selectable
        // (DXRPT_OPT_MEGAKERNEL_PATHS 0) and parity-tested at full size
        const uint64_t vertices = uint64_t(paths) * uint64_t(L - 1);
        fp.megakernel = vertices <= ctx->opt_mega_paths ? 1u : 0u;
        // register budget by frame size (measured on the Sponza proxy 1080p L=3 and its band shares): more
        // resident waves hide more latency once a frame has waves for several rounds; a GPU's 1/8 share fits
        // in one round at 4 waves/SIMD without spills.  r03 with overlapped frames: 600k+ paths 7, 300k-600k
        // 6 (a 1/4 share 0.560 -> 0.520 ms), below 4 (1/8 share 0.305 / 0.317 / 0.329 ms at 4 / 5 / 6).  r04:
        // 300k-600k 5, where k_path walks closest hits nearest-child-first (1/4 share 0.474 -> 0.466 ms,
        // profiles/r04_ab_mid_frames.txt)
        fp.megakernel_occupancy = ctx->opt_mega_occ ? ctx->opt_mega_occ
                                : paths > 600000u ? 7u
                                : (ctx->opt_overlap && paths > 300000u ? 5u : 4u);
        // depth-split schedule (k_path_head + one compacting k_path_tail per depth): it wins where there are
        // many path vertices per frame and loses on short paths, where each kernel's drain is a larger part
        // of its time -- unless overlapped frames fill the drains (r03: from 2M vertices, the metric's 1/2
        // share 0.961 -> 0.939 ms; 720p, C3's 1/8 share and the 1/4 share stay k_path, +1.4 / +2.2 / +10.6 %
        // split; profiles/r03_ab_msplit*.txt, r03_ab_split_small.txt)
        const uint64_t split_min = !ctx->opt_overlap ? kSplitMinVertices
                                 : ctx->opt_overlap == 1u ? kSplitMinVerticesOverlap2 : kSplitMinVerticesOverlap3;
        const bool split_by_size = vertices >= split_min;
        fp.split = fp.megakernel && (ctx->opt_split == 1u || (ctx->opt_split == 2u && split_by_size)) ? 1u : 0u;
        // split budgets: the head 5 waves/SIMD (96 VGPRs, no spills; r03: metric -0.2 %, C3 -0.4 %, C5's share
        // -1.0 %, C4 +0.5 % against 7), 6 (80 VGPRs) for frames above 1.5M paths with three frames in flight
        // (r05: metric -0.6 %, C4 -0.9 %; the 1/2 share +0.9 %, C5's share +0.6 %, profiles/r05_ab_occ3.txt),
        // 7 (72 VGPRs) there since the if-if traversal loops (r06: metric -0.9..-1.4 %, C4 -0.6 %, C3 even,
        // profiles/r06_ab_budgets.txt, r06_ab_split_budgets.txt); the tails 7 (72 VGPRs; 6: +2-3 %)
        if (fp.split && !ctx->opt_mega_occ)
            fp.megakernel_occupancy = !ctx->opt_overlap ? 6u : (ctx->opt_overlap != 1u && paths > 1500000u ? 7u : 5u);
        fp.tail_occupancy = ctx->opt_tail_occ ? ctx->opt_tail_occ : (ctx->opt_mega_occ ? fp.megakernel_occupancy : 7u);
        ctx->wclock_waves = 0;  // set again below only by a frame that records stamps
        // Overlapped frames (DXRPT_OPT_FRAME_OVERLAP, megakernel frames): frame parity ov runs on slot ov --
        // its stream, buffers, counters and BVH8 stack-spill slab -- and stages its radiance; the caller's
        // stream blends the stage after it, so the next frame (the other parity) may start as soon as it is
        // launched, filling this frame's drain.  Census and wave-clock frames run on the caller's stream.
        const bool overlap = ctx->opt_overlap && fp.megakernel && !ctx->opt_count && !ctx->opt_wave_clocks && paths > 0;
        ensure_spill(ctx, frame_traversal_threads(paths, slots, fp.megakernel != 0));
        // frames in flight: three where the frame's waves leave the GPU idle for much of their span -- band
        // shares (one round of waves: a 1/8 share 0.316 -> 0.244 ms) and the depth-split frames, whose tails
        // drain several times per frame -- two for the large single-kernel frames (720p: 3 is +1 %)
        // (profiles/r05_ab_overlap_depth.txt, r05_ab_overlap_cur.txt)
        if (overlap) {
            const uint32_t want = ctx->opt_overlap == kOverlapBySize ? (fp.split || paths <= 600000u ? kOverlapSlots : 2u)
                                                                     : ctx->opt_overlap + 1u;
            if (want != ctx->ovl_slots) {  // the rotation restarts
                drain_frames(ctx);
                ctx->ovl_parity = 0;
                ctx->ovl_slots = want;
            }
        }
        const uint32_t ov = ctx->ovl_parity;
        dxrpt_ctx::Slot& P = ctx->slot[ov];
        hipStream_t fs = s;  // the frame's stream
        if (overlap) {
            ensure_slot(ctx, ov, paths, slots, size_t(ctx->accum_extent) * 16u);
            fs = P.stream;
            if (!ctx->ovl_active) {  // after other work: start behind the caller's stream
                HIP_CHECK(hipEventRecord(ctx->ovl_fork, s));
                HIP_CHECK(hipStreamWaitEvent(fs, ctx->ovl_fork, 0));
                for (dxrpt_ctx::Slot& Q : ctx->slot) Q.stage_used = false;
                ctx->ovl_gate_pending = 0;
            }
            if (P.stage_used) HIP_CHECK(hipStreamWaitEvent(fs, P.stage_free, 0));  // the stage's previous blend
            // the new wave order: every slot's next frame after a rebuild waits for it, not just the next
            // frame's -- with three in flight frame f+2 runs on a third stream that would otherwise see only
            // its own slot's stage_free (the blend of frame f-1) and could read the order mid-rewrite
            if (ctx->ovl_gate_pending & (1u << ov)) HIP_CHECK(hipStreamWaitEvent(fs, ctx->ovl_gate, 0));
            ctx->ovl_gate_pending &= ~(1u << ov);
        } else {
            ensure_frame(ctx, paths, slots);
        }
        if (ctx->opt_count) {
            fp.trav = ctx->d_trav.as<unsigned long long>();
            HIP_CHECK(hipMemsetAsync(fp.trav, 0, kTravCounters * sizeof(unsigned long long), s));
            if (ctx->opt_wave_clocks && fp.megakernel) {  // census: the 64-lane kernel, one slot per 64 paths
                ctx->wclock_waves = (paths + 63u) / 64u;
                ctx->d_wclock.ensure(size_t(ctx->wclock_waves) * 2 * sizeof(unsigned long long));
                fp.wave_clock = ctx->d_wclock.as<unsigned long long>();
            }
        }
        // cost-ordered waves (the single k_path only).  By frame size (2): frames of at most 3 rounds of
        // resident waves -- with overlapped frames 1.5 -- whose end is a large part of their time (a GPU's
        // share of a multi-GPU frame); larger frames keep path order, where concurrent neighbouring blocks
        // share more cache than the shorter tail saves (profiles/r02_ab_wave_order.txt; r03: 1/2 share
        // 1.004 -> 0.980 ms, 720p 0.925 -> 0.896 without it, the 1/8 share 0.329 -> 0.305 with it).
        uint32_t order_waves = 0;
        bool order_pass = false;
        const uint32_t waves = (paths + 63u) / 64u;
        const uint64_t rounds_slots = uint64_t(ctx->num_cus) * 4u * fp.megakernel_occupancy;
        const bool order_size = ctx->opt_overlap ? 2u * uint64_t(waves) <= 3u * rounds_slots : waves <= 3u * rounds_slots;
        const bool order_on = !fp.split && (ctx->opt_wave_order == 1 || (ctx->opt_wave_order == 2 && order_size));
        if (order_on && fp.megakernel && !ctx->opt_count) {
            order_waves = waves;
            const uint64_t key = (uint64_t(order_waves) << 32) ^ ctx->tiles_gen;
            if (key != ctx->order_key || !ctx->order_ready || ctx->d_wave_order.bytes < size_t(order_waves) * sizeof(uint32_t))
                drain_frames(ctx);  // the other slot's frame may still read the order / record classes
            ctx->d_wave_cost.ensure(size_t(order_waves) * sizeof(uint32_t));
            ctx->d_wave_order.ensure(size_t(order_waves) * sizeof(uint32_t));
            ctx->d_wave_hist.ensure(4 * kWaveClasses * sizeof(uint32_t));
            if (key != ctx->order_key || !ctx->order_ready) {  // (re)start: path order, zeroed histograms
                ctx->order_key = key;
                ctx->order_ready = false;
                ctx->order_parity = 0;
                ctx->order_frame = 0;
                HIP_CHECK(hipMemsetAsync(ctx->d_wave_hist.p, 0, 4 * kWaveClasses * sizeof(uint32_t), fs));
            }
            // every opt_order_period-th ordered frame records its wave classes and rebuilds the order
            // (progressive frames cost alike); the frames between reuse it -- no recording atomics, no pass
            order_pass = ctx->opt_wave_clocks || ctx->order_frame % ctx->opt_order_period == 0u;
            fp.wave_cost = order_pass ? ctx->d_wave_cost.as<uint32_t>() : nullptr;
            fp.wave_hist = order_pass ? ctx->d_wave_hist.as<uint32_t>() + ctx->order_parity * 2 * kWaveClasses : nullptr;
            fp.wave_order = ctx->order_ready ? ctx->d_wave_order.as<uint32_t>() : nullptr;
            if (ctx->opt_wave_clocks) {  // per-slot stamps of an ordered frame (diagnostic)
                ctx->wclock_waves = order_waves;
                ctx->d_wclock.ensure(size_t(order_waves) * 2 * sizeof(unsigned long long));
                fp.wave_clock = ctx->d_wclock.as<unsigned long long>();
            }
        }
        hipEvent_t* ev = nullptr;
        if (ctx->opt_timing) {
            if (ctx->ring.empty()) ctx->ring.resize(64);
            dxrpt_ctx::FrameEvents& f = ctx->ring[ctx->ring_head];
            ctx->ring_head = (ctx->ring_head + 1) % ctx->ring.size();
            harvest(ctx, f);  // recycles the oldest slot (blocks only if it is still in flight)
            const int need = frame_event_count(L);
            while (int(f.ev.size()) < need) {
                hipEvent_t e;
                HIP_CHECK(hipEventCreate(&e));
                f.ev.push_back(e);
            }
            f.L = L;
            f.mask = ctx->opt_timing_mask;
            f.pending = true;
            f.mega = fp.megakernel != 0;
            f.split = fp.megakernel && fp.split && !ctx->opt_count && !order_waves;
            ev = f.ev.data();
        }
        hipStream_t aux = nullptr;
        if (!fp.megakernel) {  // the wavefront's any-hit passes run on an internal stream
            if (!ctx->aux) {
                HIP_CHECK(hipStreamCreateWithFlags(&ctx->aux, hipStreamNonBlocking));
                ctx->fork_ev.resize(2 * kMaxDepthQueues);
                for (auto& e : ctx->fork_ev) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            }
            aux = ctx->aux;
        }
        uint32_t sched = 0;
        if (overlap) {
            fp.stage = P.stage.as<float4>();
            const uint32_t cur = P.ctr_set;
            uint32_t* cb = P.counters.as<uint32_t>();
            P.fb.counters = cb + cur * kCounterWords;
            P.fb.counters_clean = P.ctr_clean[cur];
            P.fb.counters_next = cb + (1u - cur) * kCounterWords;  // zeroed in-kernel for this slot's next frame
            HIP_CHECK(launch_frame(scene_dev(ctx, 1u + ov), P.fb, fp, fs, ev, nullptr, nullptr, &sched));
            P.ctr_clean[cur] = false;
            P.ctr_clean[1u - cur] = true;
            P.ctr_set = 1u - cur;
            P.fb.counters_next = nullptr;
            P.fb.counters_clean = false;
            ctx->stat_counters.assign(1, P.fb.counters);
        } else {
            // counter sets: this frame's is fb.counters (read by dxrpt_get_stats); a megakernel frame zeroes
            // the other one in-kernel, so the next frame skips the fill launch
            uint32_t* cbase = ctx->f_counters.as<uint32_t>();
            const uint32_t cur = ctx->ctr_set;
            ctx->fb.counters = cbase + cur * kCounterWords;
            ctx->fb.counters_clean = ctx->ctr_clean[cur];
            ctx->fb.counters_next = fp.megakernel ? cbase + (1u - cur) * kCounterWords : nullptr;
            HIP_CHECK(launch_frame(scene_dev(ctx, 0), ctx->fb, fp, s, ev, aux, aux ? ctx->fork_ev.data() : nullptr, &sched));
            ctx->ctr_clean[cur] = false;
            if (fp.megakernel) {
                ctx->ctr_clean[1u - cur] = true;
                ctx->ctr_set = 1u - cur;
            }
            ctx->fb.counters_next = nullptr;
            ctx->fb.counters_clean = false;
            ctx->stat_counters.assign(1, ctx->fb.counters);
        }
        if (overlap) sched |= DXRPT_SCHED_OVERLAP;
        if (order_waves) ++ctx->order_frame;
        if (order_waves && order_pass) {  // the next frames' order from this frame's wave classes (after the frame events)
            uint32_t* h = ctx->d_wave_hist.as<uint32_t>();
            uint32_t* cur = h + ctx->order_parity * 2 * kWaveClasses;
            uint32_t* nxt = h + (1u - ctx->order_parity) * 2 * kWaveClasses;
            // overlapped: the other slot's frame may still read the order being rewritten
            if (overlap)
                for (uint32_t k = 0; k < kOverlapSlots; ++k)
                    if (k != ov && ctx->slot[k].stage_used) HIP_CHECK(hipStreamWaitEvent(fs, ctx->slot[k].done, 0));
            HIP_CHECK(launch_wave_order(fp.wave_cost, cur, cur + kWaveClasses, nxt, nxt + kWaveClasses,
                                        ctx->d_wave_order.as<uint32_t>(), order_waves, fs));
            ctx->order_ready = true;
            ctx->order_parity ^= 1u;
            if (overlap) {  // and the next frame of every other slot reads the new order
                HIP_CHECK(hipEventRecord(ctx->ovl_gate, fs));
                ctx->ovl_gate_pending = ((1u << kOverlapSlots) - 1u) & ~(1u << ov);
            }
        }
        if (overlap) {  // the caller's stream blends the stage once the frame is done
            HIP_CHECK(hipEventRecord(P.done, fs));
            HIP_CHECK(hipStreamWaitEvent(s, P.done, 0));
            HIP_CHECK(launch_accum_stage(fp, s));
            HIP_CHECK(hipEventRecord(P.stage_free, s));
            P.stage_used = true;
            ctx->ovl_parity = (ctx->ovl_parity + 1u) % ctx->ovl_slots;
            ctx->ovl_active = true;
        } else {
            // the next overlapped frame starts behind this one: it used slab 0 and, through the stream
            // chain, runs after every earlier overlapped frame
            ctx->ovl_active = false;
        }
        ctx->inflight = true;
        ctx->last_L = L;
        std::memset(&ctx->last, 0, sizeof(ctx->last));
        ctx->last.pixels = paths;
        ctx->last.nominal_rays = uint64_t(paths) * uint64_t(1 + (L - 1) * 2);
        ctx->last.schedule = sched;
        ctx->last.paths_per_wave = fp.megakernel ? 64u : 0u;
        ctx->last.occupancy = fp.megakernel ? fp.megakernel_occupancy : 0u;
        ctx->last.tail_occupancy = (sched & DXRPT_SCHED_SPLIT) ? fp.tail_occupancy : 0u;
        ctx->last_counted = fp.trav != nullptr;
        ctx->rendered = true;
    });
}

int dxrpt_get_stats(dxrpt_ctx* ctx, dxrpt_stats* out) {
    if (!ctx || !out) return DXRPT_E_INVALID_ARG;
    return guarded(ctx, [&] {
        require(ctx->rendered, "dxrpt_get_stats: nothing rendered yet", DXRPT_E_STATE);
        drain_frames(ctx);
        uint32_t shards[2 * kMaxDepthQueues * kQueueShards];
        uint32_t cnt[2 * kMaxDepthQueues] = {};
        for (const uint32_t* set : ctx->stat_counters) {
            HIP_CHECK(hipMemcpy(shards, set, sizeof(shards), hipMemcpyDeviceToHost));
            for (uint32_t q = 0; q < 2 * kMaxDepthQueues; ++q)
                for (uint32_t k = 0; k < kQueueShards; ++k) cnt[q] += shards[q * kQueueShards + k];
        }
        dxrpt_stats s = ctx->last;
        s.packed_materials = ctx->packed_materials;
        s.packed_textures = ctx->packed_textures;
        s.inlined_maps = ctx->inlined_refs;
        for (int d = 1; d < ctx->last_L && d < int(DXRPT_MAX_PATH_LENGTH); ++d) {
            s.radiance_rays_per_depth[d] = cnt[d];
            s.shadow_rays_per_depth[d] = cnt[16 + d];
            s.radiance_rays += cnt[d];
            s.shadow_rays += cnt[16 + d];
        }
        if (ctx->last_counted && ctx->d_trav.p) {
            unsigned long long tr[kTravCounters];
            HIP_CHECK(hipMemcpy(tr, ctx->d_trav.p, sizeof(tr), hipMemcpyDeviceToHost));
            const bool mega = (s.schedule & DXRPT_SCHED_CENSUS) != 0;  // the megakernel census counts hits
            s.node_visits_radiance = tr[0] + tr[5];
            s.tri_tests_radiance = tr[1] + tr[6];
            s.node_visits_shadow = tr[2] + tr[7];
            s.tri_tests_shadow = tr[3] + tr[8];
            s.radiance_hits = mega ? tr[4] + tr[9] : 0u;
            for (int k = 0; k < 5; ++k) s.census_depth1[k] = (k < 4 || mega) ? tr[k] : 0u;
        }
        harvest_all(ctx);
        for (int k = 0; k < DXRPT_K_COUNT; ++k) {
            s.kernel_ms[k] = ctx->kernel_ms[k];
            s.kernel_launches[k] = ctx->kernel_launches[k];
        }
        s.timed_frames = ctx->timed_frames;
        s.frame_ms = ctx->frame_ms;
        *out = s;
    });
}

int dxrpt_get_wave_clocks(dxrpt_ctx* ctx, uint64_t* out, uint32_t max_waves, uint32_t* num_waves) {
    if (!ctx || !num_waves) return DXRPT_E_INVALID_ARG;
    return guarded(ctx, [&] {
        require(ctx->rendered, "dxrpt_get_wave_clocks: nothing rendered yet", DXRPT_E_STATE);
        drain_frames(ctx);
        *num_waves = ctx->wclock_waves;
        const uint32_t n = std::min(max_waves, ctx->wclock_waves);
        if (n && out) HIP_CHECK(hipMemcpy(out, ctx->d_wclock.p, size_t(n) * 2 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    });
}

int dxrpt_get_phase_clocks(dxrpt_ctx* ctx, uint64_t out[DXRPT_PHASE_CLOCKS]) {
    if (!ctx || !out) return DXRPT_E_INVALID_ARG;
    return guarded(ctx, [&] {
        static_assert(kPhaseClockWords == DXRPT_PHASE_CLOCKS, "include/dxrpt.h DXRPT_PHASE_CLOCKS");
        unsigned long long t[kPhaseClockWords];
        HIP_CHECK(read_phase_ticks(t));
        for (int k = 0; k < kPhaseClockWords; ++k) out[k] = t[k];
    });
}

int dxrpt_get_debug_record(dxrpt_ctx* ctx, uint32_t out[DXRPT_DEBUG_WORDS]) {
    if (!ctx || !out) return DXRPT_E_INVALID_ARG;
    return guarded(ctx, [&] {
        static_assert(kDebugWords == DXRPT_DEBUG_WORDS, "include/dxrpt.h DXRPT_DEBUG_WORDS");
        HIP_CHECK(read_debug_record(out));
    });
}

int dxrpt_trace_rays(dxrpt_ctx* ctx, const float* rays, uint32_t num_rays, uint32_t flags, float* hits, void* stream) {
    if (!ctx) return DXRPT_E_INVALID_ARG;
    return guarded(ctx, [&] {
        require(ctx->bvh_built, "dxrpt_trace_rays: acceleration structure not built", DXRPT_E_STATE);
        require(num_rays == 0 || (rays && hits), "dxrpt_trace_rays: null argument");
        const hipStream_t s = static_cast<hipStream_t>(stream);
        enter_stream(ctx, s);
        upload_textures(ctx);
        ensure_spill(ctx, trace_rays_threads(num_rays));
        HIP_CHECK(launch_trace_rays(scene_dev(ctx, 0), reinterpret_cast<const float4*>(rays), num_rays, flags,
                                    reinterpret_cast<float4*>(hits), s));
        ctx->ovl_active = false;
        ctx->inflight = true;
    });
}

int dxrpt_opacity_micromap(const float* uvs, uint32_t num_tris, uint32_t w, uint32_t h, uint32_t fmt, const void* texels,
                           uint32_t* words) {
    static_assert(kOmmWords == DXRPT_OMM_WORDS && kOmmSplit == DXRPT_OMM_SPLIT, "include/dxrpt.h DXRPT_OMM_*");
    if (!uvs || !texels || !words || w == 0 || h == 0 || fmt > DXRPT_TEX_R8_UNORM) return DXRPT_E_INVALID_ARG;
    if (size_t(w) * h > (size_t(1) << 26)) return DXRPT_E_INVALID_ARG;
    try {
        const uint32_t lut = fmt == DXRPT_TEX_RGBA8_SRGB ? 256u : 0u;
        std::vector<float> v(size_t(w) * h);
        for (size_t i = 0; i < v.size(); ++i) {
            const uint32_t b = fmt == DXRPT_TEX_R8_UNORM ? static_cast<const uint8_t*>(texels)[i]
                                                         : static_cast<const uint32_t*>(texels)[i] & 0xFFu;
            v[i] = omm_decode(lut, b);
        }
        const OpacityField f(w, h, std::move(v));
        for (uint32_t t = 0; t < num_tris; ++t) omm_triangle(f, uvs + size_t(t) * 6u, words + size_t(t) * kOmmWords);
        return DXRPT_OK;
    } catch (const std::bad_alloc&) {
        return DXRPT_E_OOM;
    }
}

int dxrpt_sample_cmj(dxrpt_ctx* ctx, const uint32_t* cases, uint32_t num_cases, float* out, void* stream) {
    if (!ctx) return DXRPT_E_INVALID_ARG;
    return guarded(ctx, [&] {
        require(num_cases == 0 || (cases && out), "dxrpt_sample_cmj: null argument");
        HIP_CHECK(launch_sample_cmj(reinterpret_cast<const uint4*>(cases), num_cases, reinterpret_cast<float2*>(out),
                                    static_cast<hipStream_t>(stream)));
    });
}

// PostProcessor::Render (DXRPathTracer/PostProcessor.cpp:43-92): bloom + exposure + filmic tone map.
int dxrpt_post_process(dxrpt_ctx* ctx, const dxrpt_app_settings* settings, const float* accum, uint32_t width,
                       uint32_t height, void* out, uint32_t out_format, void* stream) {
    if (!ctx) return DXRPT_E_INVALID_ARG;
    return guarded(ctx, [&] {
        require(settings && accum && out, "dxrpt_post_process: null argument");
        require(width >= 2 && height >= 2, "dxrpt_post_process: image must be at least 2 x 2");
        require(out_format == DXRPT_POST_FLOAT4 || out_format == DXRPT_POST_RGBA8, "dxrpt_post_process: bad output format");
        const hipStream_t s = static_cast<hipStream_t>(stream);
        enter_stream(ctx, s);  // after the frames whose blends write `accum`
        const size_t half = size_t(width / 2) * (height / 2) * 8u;
        if (ctx->p_bloom0.bytes < half) drain_frames(ctx);  // an earlier post pass may still use the scratch
        ctx->p_bloom0.ensure(half);
        ctx->p_bloom1.ensure(half);
        PostParams p{};
        p.accum = accum;
        p.bloom0 = ctx->p_bloom0.p;
        p.bloom1 = ctx->p_bloom1.p;
        p.out = out;
        p.width = width;
        p.height = height;
        p.out_format = out_format;
        // PostProcessing.hlsl:21-25, 125-130; evaluated in double, rounded to float
        const double sigma = double(settings->BloomBlurSigma);
        const double g = 1.0 / std::sqrt(2.0 * 3.14159 * sigma * sigma);
        for (int k = 0; k < 14; ++k) {
            const int d = k - 7;
            p.weights.w[k] = float(g * std::exp(-double(d * d) / (2.0 * sigma * sigma)));
        }
        p.bloom_magnitude = settings->BloomMagnitude;
        p.bloom_exp2 = float(std::exp2(double(settings->BloomExposure)));
        p.exposure_scale = float(std::exp2(double(settings->Exposure)) / 0.0009765625);
        HIP_CHECK(launch_post_process(p, s));
        ctx->inflight = true;
    });
}

// DXRPathTracer::RenderBakingPass_Progressive (DXRPathTracer.cpp:1895-1991): one DispatchRays(W, H) of
// BakeRayGen over the surface map.  The dispatch is cut into chunks of texels so the per-texel shadow
// slots stay bounded; every texel is independent, so the chunking changes nothing in the results.
int dxrpt_bake_lightmap(dxrpt_ctx* ctx, const dxrpt_ray_trace_constants* rtc, const dxrpt_app_settings* settings,
                        const dxrpt_light_constants* lights, const float* surface_pos, const float* surface_normal,
                        float* accum, float* lightmap, uint32_t width, uint32_t height, void* stream) {
    if (!ctx) return DXRPT_E_INVALID_ARG;
    return guarded(ctx, [&] {
        require(ctx->bvh_built, "dxrpt_bake_lightmap: acceleration structure not built", DXRPT_E_STATE);
        require(ctx->sky_set, "dxrpt_bake_lightmap: sky cubemap not set", DXRPT_E_STATE);
        require(rtc && settings && surface_pos && surface_normal && accum && lightmap, "dxrpt_bake_lightmap: null argument");
        require(width > 0 && height > 0, "dxrpt_bake_lightmap: empty lightmap");
        require(uint64_t(width) * height < 0x7FFFFFFFull, "dxrpt_bake_lightmap: lightmap too large");
        require(uint64_t(width) * height == rtc->TotalNumPixels, "dxrpt_bake_lightmap: TotalNumPixels != width*height");
        require(settings->SqrtNumSamples >= 1, "dxrpt_bake_lightmap: SqrtNumSamples must be >= 1");
        require(settings->MaxPathLength >= 1 && settings->MaxPathLength <= int(DXRPT_MAX_PATH_LENGTH),
                "dxrpt_bake_lightmap: MaxPathLength must be in [1, 8]");
        const bool useLights = settings->RenderLights && rtc->NumLights > 0;
        require(!useLights || (lights && rtc->NumLights <= DXRPT_MAX_SPOT_LIGHTS), "dxrpt_bake_lightmap: bad lights");
        const hipStream_t s = static_cast<hipStream_t>(stream);
        enter_stream(ctx, s);
        upload_textures(ctx);
        const uint32_t nl = useLights ? rtc->NumLights : 0u;
        if (nl) {
            std::vector<dxrpt_spot_light> L(lights->Lights, lights->Lights + nl);
            if (L.size() != ctx->lights_cache.size() || std::memcmp(L.data(), ctx->lights_cache.data(), nl * sizeof(dxrpt_spot_light)) != 0) {
                drain_frames(ctx);
                ctx->d_lights.upload(L.data(), nl * sizeof(dxrpt_spot_light));
                ctx->lights_cache = L;
            }
        }
        const uint32_t total = width * height;
        const uint32_t chunk = std::min<uint32_t>(total, ctx->opt_bake_chunk);
        ensure_frame(ctx, chunk, 2u + nl);
        ensure_spill(ctx, frame_traversal_threads(chunk, 2u + nl, true));
        if (ctx->d_bake_list.bytes < size_t(total) * sizeof(uint32_t) + 64) drain_frames(ctx);
        ctx->d_bake_list.ensure(size_t(total) * sizeof(uint32_t) + 64);
        FrameParams fp{};
        fp.rtc = *rtc;
        fp.rtc.NumLights = nl;
        fp.set = *settings;
        fp.lights = nl ? ctx->d_lights.as<dxrpt_spot_light>() : nullptr;
        fp.num_paths = chunk;
        // (the bake's incoherent first rays: 6 beat 7 at 2M-texel chunks, 19.0 vs 20.3 ms per 4096^2 pass)
        fp.megakernel_occupancy = ctx->opt_mega_occ ? ctx->opt_mega_occ : (chunk > 1500000u ? 6u : (chunk > 300000u ? 5u : 4u));
        fp.width = width;
        fp.height = height;
        const SceneDev sd = scene_dev(ctx, 0);
        BakeArgs b;
        b.pos = reinterpret_cast<const float4*>(surface_pos);
        b.nrm = reinterpret_cast<const float4*>(surface_normal);
        b.accum = reinterpret_cast<float4*>(accum);
        b.lightmap = reinterpret_cast<float4*>(lightmap);
        b.width = width;
        b.height = height;
        b.list = ctx->d_bake_list.as<uint32_t>();
        b.count = b.list + total;  // the entry count lives after the list
        HIP_CHECK(launch_bake_compact(b.pos, total, const_cast<uint32_t*>(b.list), const_cast<uint32_t*>(b.count), s));
        ctx->fb.counters = ctx->f_counters.as<uint32_t>() + ctx->ctr_set * kCounterWords;
        ctx->fb.counters_next = nullptr;
        HIP_CHECK(hipMemsetAsync(ctx->fb.counters, 0, kCounterWords * sizeof(uint32_t), s));
        ctx->ctr_clean[ctx->ctr_set] = false;
        ctx->stat_counters.assign(1, ctx->fb.counters);
        // the live count stays on the device (no host sync): launches cover every texel, and chunks
        // past the live count exit at once
        for (uint32_t first = 0; first < total; first += chunk) {
            b.first = first;
            b.span = std::min(chunk, total - first);
            HIP_CHECK(launch_bake(sd, ctx->fb, fp, b, s));
        }
        // dxrpt_get_stats then reports this pass: texels and the rays its paths traced
        ctx->ovl_active = false;
        ctx->inflight = true;
        ctx->last_L = settings->MaxPathLength < 2 ? 2 : settings->MaxPathLength;
        std::memset(&ctx->last, 0, sizeof(ctx->last));
        ctx->last.pixels = total;
        ctx->rendered = true;
    });
}

// DXRPathTracer::RenderLightmapMedianPass (DXRPathTracer.cpp:2092-2125): DenoiseCS with FilterRadius 1.
int dxrpt_denoise_median(dxrpt_ctx* ctx, const float* in, float* out, uint32_t width, uint32_t height, void* stream) {
    if (!ctx) return DXRPT_E_INVALID_ARG;
    return guarded(ctx, [&] {
        require(in && out, "dxrpt_denoise_median: null argument");
        require(in != out, "dxrpt_denoise_median: in and out must not alias");
        require(width > 0 && height > 0 && uint64_t(width) * height < 0x7FFFFFFFull, "dxrpt_denoise_median: bad size");
        HIP_CHECK(launch_median3x3(reinterpret_cast<const float4*>(in), reinterpret_cast<float4*>(out), width, height,
                                   static_cast<hipStream_t>(stream)));
    });
}

}  // extern "C"
