// dxrpt_render — a C++ host above the C ABI (include/dxrpt.h + include/dxrpt_host.h), no Python.
//
// The reference's application loop for the path tracer, restated headless:
//   DXRPathTracer::InitializeScene     (DXRPathTracer.cpp:932-985)  -> dxrpt_host_scene_create, Hosek sky,
//                                                                      dxrpt_add_texture / dxrpt_set_scene /
//                                                                      dxrpt_set_sky
//   BuildRTAccelerationStructure       (DXRPathTracer.cpp:2331-2488) -> dxrpt_build_bvh
//   RenderRayTracing + DispatchRays    (DXRPathTracer.cpp:2024-2090) -> dxrpt_host_fill_constants +
//                                                                      dxrpt_render, once per frame
//   PostProcessor::Render              (DXRPathTracer.cpp:1561-1564) -> dxrpt_post_process (RGBA8)
// and, with --world N, the screen-band sharding of an N-GPU frame with the frame-end gather of
// SURVEY.md 8(e) (dxrpt_comm_create, dxrpt_gather_slabs, dxrpt_unpermute): every rank is its own
// process (rank r on HIP device --device), rank 0 writes the RCCL unique id to --uid-file and the other
// ranks read it (the "any means" of dxrpt_comm_unique_id).  Rank 0 ends each frame with the whole
// W x H frame in its buffer.
//
//   dxrpt_render [--scene sponza|suntemple|boxtest|whitefurnace] [--width W] [--height H]
//                [--path-length L] [--frames N] [--warmup K] [--device d]
//                [--world N --rank r --uid-file PATH] [--dump-accum FILE] [--ppm FILE]
//
// Frame f uses CurrSampleIdx = f mod SqrtNumSamples^2 (the bench's steady state; the reference stops at
// SqrtNumSamples^2 samples, DXRPathTracer.cpp:2027-2028).  Prints one JSON line per rank: ms/frame
// (HIP events on the render stream around the timed frames) and nominal Mrays/s
// (W*H*(1 + 2(L-1)) per frame, DXRPathTracer.cpp:2171).  --dump-accum writes the final accumulation
// target (rank 0: the gathered frame) as raw float32 RGBA; --ppm the post-processed frame.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

#include "../../../include/dxrpt.h"
#include "../../../include/dxrpt_host.h"

namespace {

constexpr uint64_t kSponzaSeed = 0x53504F4E5A41ull;  // dxrpathtracer_amd/scene.py SPONZA_SEED
constexpr float kFov = 3.14159265358979323846f / 4.0f, kNear = 0.1f, kFar = 100.0f;  // DXRPathTracer.cpp:265
constexpr float kTurbidity = 2.0f;                     // AppSettings.cpp:104-113
constexpr uint32_t kSkyRes = 128;                      // Skybox.cpp:164
constexpr uint32_t kBandRows = 8;                      // distributed.BAND_ROWS

void die(const char* what, const char* msg) {
    std::fprintf(stderr, "dxrpt_render: %s failed: %s\n", what, msg ? msg : "");
    std::exit(1);
}

void check(int rc, const char* what) {
    if (rc != DXRPT_OK) die(what, dxrpt_last_error(nullptr));
}

void check_multi(int rc, const char* what) {
    if (rc != DXRPT_OK) die(what, dxrpt_multi_last_error());
}

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) die(what, hipGetErrorString(e));
}

std::string exe_dir() {
    char buf[4096];
    const ssize_t n = readlink("/proc/self/exe", buf, sizeof(buf) - 1);
    if (n <= 0) return ".";
    buf[n] = 0;
    std::string p(buf);
    const size_t s = p.rfind('/');
    return s == std::string::npos ? "." : p.substr(0, s);
}

// Round-robin 8-row bands (distributed.band_layout): band b -> rank b mod N, packed in the rank's slab.
struct Bands {
    std::vector<std::vector<dxrpt_tile>> tiles;  // per rank
    std::vector<uint64_t> counts;                // pixels per rank
};

Bands band_layout(uint32_t W, uint32_t H, uint32_t world) {
    Bands b;
    b.tiles.resize(world);
    b.counts.assign(world, 0);
    uint32_t band = 0;
    for (uint32_t y0 = 0; y0 < H; y0 += kBandRows, ++band) {
        const uint32_t r = band % world, h = std::min(kBandRows, H - y0);
        dxrpt_tile t{};
        t.x0 = 0;
        t.y0 = y0;
        t.w = W;
        t.h = h;
        t.accum_offset = b.counts[r];
        t.accum_pitch = W;
        b.tiles[r].push_back(t);
        b.counts[r] += uint64_t(W) * h;
    }
    return b;
}

void write_file(const char* path, const void* data, size_t bytes) {
    FILE* f = std::fopen(path, "wb");
    if (!f || std::fwrite(data, 1, bytes, f) != bytes) die("write", path);
    std::fclose(f);
}

}  // namespace

int main(int argc, char** argv) {
    std::string scene_name = "sponza", uid_file, dump, ppm;
    uint32_t W = 1920, H = 1080, L = 3, frames = 32, warmup = 5, world = 1, rank = 0;
    int device = 0;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto val = [&]() -> const char* {
            if (i + 1 >= argc) die("arguments", ("missing value for " + a).c_str());
            return argv[++i];
        };
        if (a == "--scene") scene_name = val();
        else if (a == "--width") W = uint32_t(std::atoi(val()));
        else if (a == "--height") H = uint32_t(std::atoi(val()));
        else if (a == "--path-length") L = uint32_t(std::atoi(val()));
        else if (a == "--frames") frames = uint32_t(std::atoi(val()));
        else if (a == "--warmup") warmup = uint32_t(std::atoi(val()));
        else if (a == "--device") device = std::atoi(val());
        else if (a == "--world") world = uint32_t(std::atoi(val()));
        else if (a == "--rank") rank = uint32_t(std::atoi(val()));
        else if (a == "--uid-file") uid_file = val();
        else if (a == "--dump-accum") dump = val();
        else if (a == "--ppm") ppm = val();
        else die("arguments", ("unknown option " + a).c_str());
    }
    uint32_t scene_id = DXRPT_SCENE_SPONZA;
    if (scene_name == "suntemple") scene_id = DXRPT_SCENE_SUNTEMPLE;
    else if (scene_name == "boxtest") scene_id = DXRPT_SCENE_BOXTEST;
    else if (scene_name == "whitefurnace") scene_id = DXRPT_SCENE_WHITEFURNACE;
    else if (scene_name != "sponza") die("arguments", ("unknown scene " + scene_name).c_str());
    if (world < 1 || rank >= world || (world > 1 && uid_file.empty())) die("arguments", "--world N needs --rank < N and --uid-file");
    if (L < 2 || L > DXRPT_MAX_PATH_LENGTH || frames == 0) die("arguments", "--path-length 2..8, --frames >= 1");

    // ---- InitializeScene: scene, settings, sky (host) ------------------------------------------
    dxrpt_host_scene* sc = nullptr;
    if (dxrpt_host_scene_create(scene_id, kSponzaSeed, 0, &sc) != DXRPT_OK) die("dxrpt_host_scene_create", dxrpt_host_last_error());
    dxrpt_app_settings st;
    dxrpt_default_settings(&st);
    std::memcpy(st.SunDirection, sc->sun_direction, sizeof(st.SunDirection));  // DXRPathTracer.cpp:963
    st.EnableWhiteFurnaceMode = sc->white_furnace ? 1 : 0;                     // DXRPathTracer.cpp:935
    st.MaxPathLength = int32_t(L);
    const std::string tables = exe_dir() + "/../data/hosek_tables.bin";
    dxrpt_host_hosek* hosek = nullptr;
    if (dxrpt_host_hosek_load_tables(tables.c_str(), &hosek) != DXRPT_OK) die("dxrpt_host_hosek_load_tables", dxrpt_host_hosek_last_error());
    std::vector<uint16_t> cube(size_t(6) * kSkyRes * kSkyRes * 4);
    float sun_irr[3], sun_ren[3];
    const float albedo[3] = {0.25f, 0.25f, 0.25f};
    if (dxrpt_host_sky_create_hosek(hosek, st.SunDirection, st.SunSize, kTurbidity, albedo, kSkyRes, cube.data(), sun_irr,
                                    sun_ren) != DXRPT_OK)
        die("dxrpt_host_sky_create_hosek", dxrpt_host_hosek_last_error());
    dxrpt_light_constants lights{};
    const uint32_t nl = std::min<uint32_t>(sc->num_spot_lights, DXRPT_MAX_SPOT_LIGHTS);
    for (uint32_t l = 0; l < nl; ++l) lights.Lights[l] = sc->spot_lights[l];
    float inv_vp[16];
    dxrpt_host_inv_view_projection(sc->camera_position, sc->camera_rotation[0], sc->camera_rotation[1], kFov,
                                   float(W) / float(H), kNear, kFar, inv_vp);

    // ---- the path tracer context: textures, scene, sky, acceleration structure -------------------
    hip_check(hipSetDevice(device), "hipSetDevice");
    dxrpt_ctx* ctx = nullptr;
    check(dxrpt_create(device, &ctx), "dxrpt_create");
    for (uint32_t t = 0; t < sc->num_textures; ++t) {
        const dxrpt_host_texture& tx = sc->textures[t];
        uint32_t idx = 0;
        check(dxrpt_add_texture(ctx, tx.width, tx.height, tx.fmt, tx.texels, &idx), "dxrpt_add_texture");
    }
    check(dxrpt_set_scene(ctx, sc->vertices, sc->num_vertices, sc->indices, sc->idx_bytes, sc->num_indices, sc->geometries,
                          sc->num_geometries, sc->materials, sc->num_materials),
          "dxrpt_set_scene");
    check(dxrpt_set_sky(ctx, cube.data(), kSkyRes), "dxrpt_set_sky");
    check(dxrpt_build_bvh(ctx), "dxrpt_build_bvh");

    // ---- frame buffers, the rank's share and the gather ------------------------------------------
    const Bands lay = band_layout(W, H, world);
    const uint64_t n_local = world > 1 ? lay.counts[rank] : uint64_t(W) * H;
    hipStream_t stream;
    hip_check(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "hipStreamCreate");
    float *accum = nullptr, *gathered = nullptr, *full = nullptr;
    hip_check(hipMalloc(&accum, n_local * 16), "hipMalloc");
    hip_check(hipMemset(accum, 0, n_local * 16), "hipMemset");
    void* comm = nullptr;
    std::vector<dxrpt_tile> all_tiles;  // every rank's tiles, offsets into the gathered buffer
    if (world > 1) {
        char uid[DXRPT_COMM_ID_BYTES];
        if (rank == 0) {
            check_multi(dxrpt_comm_unique_id(uid), "dxrpt_comm_unique_id");
            const std::string tmp = uid_file + ".tmp";
            write_file(tmp.c_str(), uid, sizeof(uid));
            if (std::rename(tmp.c_str(), uid_file.c_str()) != 0) die("rename", uid_file.c_str());
        } else {
            for (int tries = 0;; ++tries) {  // rank 0 publishes the id atomically (rename)
                FILE* f = std::fopen(uid_file.c_str(), "rb");
                if (f) {
                    const size_t got = std::fread(uid, 1, sizeof(uid), f);
                    std::fclose(f);
                    if (got == sizeof(uid)) break;
                }
                if (tries > 6000) die("uid file", uid_file.c_str());
                std::this_thread::sleep_for(std::chrono::milliseconds(10));
            }
        }
        check_multi(dxrpt_comm_create(device, int(world), int(rank), uid, &comm), "dxrpt_comm_create");
        if (rank == 0) {
            hip_check(hipMalloc(&gathered, uint64_t(W) * H * 16), "hipMalloc");
            hip_check(hipMalloc(&full, uint64_t(W) * H * 16), "hipMalloc");
            hip_check(hipMemset(full, 0, uint64_t(W) * H * 16), "hipMemset");
            uint64_t base = 0;
            for (uint32_t r = 0; r < world; ++r) {
                for (dxrpt_tile t : lay.tiles[r]) {
                    t.accum_offset += base;
                    all_tiles.push_back(t);
                }
                base += lay.counts[r];
            }
        }
    }
    const dxrpt_tile* tiles = world > 1 ? lay.tiles[rank].data() : nullptr;
    const uint32_t ntiles = world > 1 ? uint32_t(lay.tiles[rank].size()) : 0u;
    const uint32_t spp = uint32_t(st.SqrtNumSamples * st.SqrtNumSamples);

    auto frame = [&](uint32_t f) {
        dxrpt_ray_trace_constants rtc;
        dxrpt_host_fill_constants(inv_vp, sc->camera_position, &st, sun_irr, sun_ren, f % spp, W, H, nl, &rtc);
        check(dxrpt_render(ctx, &rtc, &st, &lights, accum, W, H, tiles, ntiles, stream), "dxrpt_render");
        if (world > 1) {  // frame-end gather to rank 0 and the un-permute into the W x H frame (stream-ordered)
            check_multi(dxrpt_gather_slabs(comm, accum, lay.counts.data(), gathered, stream), "dxrpt_gather_slabs");
            if (rank == 0)
                check_multi(dxrpt_unpermute(gathered, all_tiles.data(), uint32_t(all_tiles.size()), full, W, H, stream),
                            "dxrpt_unpermute");
        }
    };

    // ---- RenderRayTracing, frame after frame -------------------------------------------------------
    uint32_t f = 0;
    for (; f < warmup; ++f) frame(f);
    hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
    hipEvent_t e0, e1;
    hip_check(hipEventCreate(&e0), "hipEventCreate");
    hip_check(hipEventCreate(&e1), "hipEventCreate");
    hip_check(hipEventRecord(e0, stream), "hipEventRecord");
    for (uint32_t k = 0; k < frames; ++k, ++f) frame(f);
    hip_check(hipEventRecord(e1, stream), "hipEventRecord");
    hip_check(hipEventSynchronize(e1), "hipEventSynchronize");
    float ms = 0.0f;
    hip_check(hipEventElapsedTime(&ms, e0, e1), "hipEventElapsedTime");
    dxrpt_stats stats;
    check(dxrpt_get_stats(ctx, &stats), "dxrpt_get_stats");
    const double ms_frame = double(ms) / frames;
    const double nominal = double(W) * H * (1 + 2 * (L - 1));
    std::printf("{\"tool\": \"dxrpt_render\", \"scene\": \"%s\", \"width\": %u, \"height\": %u, \"max_path_length\": %u, "
                "\"frames\": %u, \"world\": %u, \"rank\": %u, \"pixels_local\": %llu, \"ms_per_frame\": %.4f, "
                "\"nominal_Mrays_s\": %.2f, \"schedule_bits\": %u, \"triangles\": %llu}\n",
                scene_name.c_str(), W, H, L, frames, world, rank, (unsigned long long)n_local, ms_frame,
                nominal / (ms_frame * 1e-3) / 1e6, stats.schedule, (unsigned long long)sc->num_triangles);

    // ---- outputs (rank 0 holds the whole frame) ------------------------------------------------------
    const float* frame_buf = world > 1 ? full : accum;
    if (rank == 0 && !dump.empty()) {
        std::vector<float> host(uint64_t(W) * H * 4);
        hip_check(hipMemcpy(host.data(), frame_buf, host.size() * 4, hipMemcpyDeviceToHost), "hipMemcpy");
        write_file(dump.c_str(), host.data(), host.size() * 4);
    }
    if (rank == 0 && !ppm.empty()) {  // PostProcessor::Render -> RGBA8, written as binary PPM
        void* ldr = nullptr;
        hip_check(hipMalloc(&ldr, uint64_t(W) * H * 4), "hipMalloc");
        check(dxrpt_post_process(ctx, &st, frame_buf, W, H, ldr, DXRPT_POST_RGBA8, stream), "dxrpt_post_process");
        std::vector<uint8_t> rgba(uint64_t(W) * H * 4), rgb(uint64_t(W) * H * 3);
        hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
        hip_check(hipMemcpy(rgba.data(), ldr, rgba.size(), hipMemcpyDeviceToHost), "hipMemcpy");
        for (uint64_t p = 0; p < uint64_t(W) * H; ++p) std::memcpy(&rgb[3 * p], &rgba[4 * p], 3);
        FILE* o = std::fopen(ppm.c_str(), "wb");
        if (!o) die("open", ppm.c_str());
        std::fprintf(o, "P6\n%u %u\n255\n", W, H);
        std::fwrite(rgb.data(), 1, rgb.size(), o);
        std::fclose(o);
        hip_check(hipFree(ldr), "hipFree");
    }
    if (comm) check_multi(dxrpt_comm_destroy(comm), "dxrpt_comm_destroy");
    hip_check(hipFree(accum), "hipFree");
    if (gathered) hip_check(hipFree(gathered), "hipFree");
    if (full) hip_check(hipFree(full), "hipFree");
    check(dxrpt_destroy(ctx), "dxrpt_destroy");
    dxrpt_host_hosek_destroy(hosek);
    dxrpt_host_scene_destroy(sc);
    return 0;
}
