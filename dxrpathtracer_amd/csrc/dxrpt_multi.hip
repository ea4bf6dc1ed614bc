// dxrpt_multi.hip — the multi-GPU frame behind the C ABI (include/dxrpt.h).
//
// The reference renders one frame on one GPU (DispatchRays(W, H, 1), DXRPathTracer.cpp:2077-2085).  Here
// a frame is split into screen tiles across the GPUs of a node (one process / context per GPU): rank r
// renders its tiles with dxrpt_render into a compact slab, the slabs go to rank 0 over RCCL (xGMI on an
// MI355X node) with grouped point-to-point sends -- each link carries only its own rank's slab, every
// sender at once -- and rank 0 scatters them into the W x H frame with the un-permute kernel.  CMJ seeds
// use global pixel indices (RayTrace.hlsl:85-96), so the gathered frame equals the single-GPU frame bit
// for bit.  The communicator is created here from a unique id the caller distributes (MPI, a file, or
// torch.distributed in the Python driver), so a C++ host needs nothing but this library.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/dxrpt.h"

namespace {

constexpr int kBlock = 256;

// One thread per pixel of the tile list (prefix = exclusive pixel prefix sums, num_tiles + 1 entries):
// tile pixel (lx, ly) is read at src[accum_offset + ly * accum_pitch + lx] and written to the frame at
// dst[(y0 + ly) * width + x0 + lx].
__global__ __launch_bounds__(kBlock) void k_unpermute(const float4* __restrict__ src, const dxrpt_tile* __restrict__ tiles,
                                                      const uint32_t* __restrict__ prefix, uint32_t num_tiles,
                                                      float4* __restrict__ dst, uint32_t width) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= prefix[num_tiles]) return;
    uint32_t lo = 0, hi = num_tiles;
    while (hi - lo > 1u) {
        const uint32_t mid = (lo + hi) >> 1;
        if (prefix[mid] <= i) lo = mid; else hi = mid;
    }
    const dxrpt_tile t = tiles[lo];
    const uint32_t local = i - prefix[lo];
    const uint32_t lx = local % t.w, ly = local / t.w;
    dst[size_t(t.y0 + ly) * width + t.x0 + lx] = src[t.accum_offset + size_t(ly) * t.accum_pitch + lx];
}

struct MultiError : std::runtime_error {
    int code;
    MultiError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw MultiError(DXRPT_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

void nccl_check(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw MultiError(DXRPT_E_HIP, std::string(what) + ": " + ncclGetErrorString(r));
}

// Scratch of the un-permute (device tile list + prefix) per thread and HIP device, reused across frames.
// `done` is recorded after each launch that reads it: a new tile list waits for it before overwriting or
// freeing the buffer (the last launch may still be queued on a non-blocking caller stream).  It is released
// by dxrpt_multi_release (or dxrpt_comm_destroy) on the thread that used it; a scratch still held at thread
// exit is left to the process teardown -- no HIP call from a thread_local destructor, which may run after
// the HIP runtime or RCCL is gone.
struct UnpermuteScratch {
    int device = -1;
    void* buf = nullptr;
    size_t bytes = 0;
    hipEvent_t done = nullptr;
    std::vector<dxrpt_tile> tiles;
    void release() {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (device >= 0) hip_check(hipSetDevice(device), "hipSetDevice");
        if (done) {
            hip_check(hipEventSynchronize(done), "hipEventSynchronize");
            hip_check(hipEventDestroy(done), "hipEventDestroy");
            done = nullptr;
        }
        if (buf) hip_check(hipFree(buf), "hipFree");
        buf = nullptr;
        bytes = 0;
        tiles.clear();
        if (cur >= 0) (void)hipSetDevice(cur);
    }
};
thread_local std::vector<std::unique_ptr<UnpermuteScratch>> g_scratch;

void release_scratch() {
    for (auto& s : g_scratch) s->release();
    g_scratch.clear();
}
thread_local std::string g_err;

UnpermuteScratch& scratch_for_current_device() {
    int dev = 0;
    hip_check(hipGetDevice(&dev), "hipGetDevice");
    for (auto& s : g_scratch)
        if (s->device == dev) return *s;
    g_scratch.push_back(std::make_unique<UnpermuteScratch>());
    g_scratch.back()->device = dev;
    hip_check(hipEventCreateWithFlags(&g_scratch.back()->done, hipEventDisableTiming), "hipEventCreate");
    return *g_scratch.back();
}

template <class F>
int guarded(F&& f) {
    try {
        f();
        return DXRPT_OK;
    } catch (const MultiError& e) {
        g_err = e.what();
        return e.code;
    } catch (const std::bad_alloc&) {
        g_err = "host out of memory";
        return DXRPT_E_OOM;
    } catch (const std::exception& e) {
        g_err = e.what();
        return DXRPT_E_INVALID_ARG;
    }
}

void require(bool c, const std::string& m) {
    if (!c) throw MultiError(DXRPT_E_INVALID_ARG, m);
}

}  // namespace

extern "C" {

const char* dxrpt_multi_last_error(void) { return g_err.c_str(); }

int dxrpt_unpermute(const float* src, const dxrpt_tile* tiles, uint32_t num_tiles, float* dst, uint32_t width,
                    uint32_t height, void* stream) {
    return guarded([&] {
        require(src && dst && (tiles || num_tiles == 0), "dxrpt_unpermute: null argument");
        if (num_tiles == 0) return;
        UnpermuteScratch& s = scratch_for_current_device();
        std::vector<uint32_t> prefix(num_tiles + 1, 0u);
        uint64_t total = 0;
        for (uint32_t k = 0; k < num_tiles; ++k) {
            const dxrpt_tile& t = tiles[k];
            require(t.w > 0 && t.h > 0 && uint64_t(t.x0) + t.w <= width && uint64_t(t.y0) + t.h <= height,
                    "dxrpt_unpermute: tile " + std::to_string(k) + " outside the frame");
            require(t.accum_pitch >= t.w, "dxrpt_unpermute: tile accum_pitch < width");
            prefix[k] = uint32_t(total);
            total += uint64_t(t.w) * t.h;
            require(total < 0x7FFFFFFFull, "dxrpt_unpermute: too many pixels");
        }
        prefix[num_tiles] = uint32_t(total);
        const bool same = s.tiles.size() == num_tiles &&
                          std::memcmp(s.tiles.data(), tiles, num_tiles * sizeof(dxrpt_tile)) == 0;
        const size_t tb = num_tiles * sizeof(dxrpt_tile), pb = prefix.size() * sizeof(uint32_t);
        if (!same) {  // upload the tile list once per distinct list (a frame-rate caller reuses it)
            hip_check(hipEventSynchronize(s.done), "hipEventSynchronize");  // the previous list's last reader
            if (tb + pb > s.bytes) {
                if (s.buf) hip_check(hipFree(s.buf), "hipFree");
                s.buf = nullptr;
                hip_check(hipMalloc(&s.buf, tb + pb), "hipMalloc");
                s.bytes = tb + pb;
            }
            hip_check(hipMemcpy(s.buf, tiles, tb, hipMemcpyHostToDevice), "hipMemcpy tiles");
            hip_check(hipMemcpy(static_cast<char*>(s.buf) + tb, prefix.data(), pb, hipMemcpyHostToDevice), "hipMemcpy prefix");
            s.tiles.assign(tiles, tiles + num_tiles);
        }
        const dxrpt_tile* dt = static_cast<const dxrpt_tile*>(s.buf);
        const uint32_t* dp = reinterpret_cast<const uint32_t*>(static_cast<const char*>(s.buf) + tb);
        hipLaunchKernelGGL(k_unpermute, dim3(uint32_t((total + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                           static_cast<hipStream_t>(stream), reinterpret_cast<const float4*>(src), dt, dp, num_tiles,
                           reinterpret_cast<float4*>(dst), width);
        hip_check(hipGetLastError(), "k_unpermute");
        hip_check(hipEventRecord(s.done, static_cast<hipStream_t>(stream)), "hipEventRecord");
    });
}

int dxrpt_comm_unique_id(void* id) {
    return guarded([&] {
        require(id != nullptr, "dxrpt_comm_unique_id: null argument");
        ncclUniqueId u;
        nccl_check(ncclGetUniqueId(&u), "ncclGetUniqueId");
        std::memcpy(id, &u, sizeof(u));
    });
}

int dxrpt_comm_create(int hip_device, int nranks, int rank, const void* id, void** comm) {
    return guarded([&] {
        require(id && comm && nranks >= 1 && rank >= 0 && rank < nranks, "dxrpt_comm_create: bad argument");
        hip_check(hipSetDevice(hip_device), "hipSetDevice");
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        ncclComm_t c = nullptr;
        nccl_check(ncclCommInitRank(&c, nranks, u, rank), "ncclCommInitRank");
        *comm = c;
    });
}

int dxrpt_comm_destroy(void* comm) {
    return guarded([&] {
        if (comm) nccl_check(ncclCommDestroy(static_cast<ncclComm_t>(comm)), "ncclCommDestroy");
        release_scratch();
    });
}

int dxrpt_multi_release(void) {
    return guarded([&] { release_scratch(); });
}

int dxrpt_comm_info(void* comm, int* nranks, int* rank) {
    return guarded([&] {
        require(comm && nranks && rank, "dxrpt_comm_info: null argument");
        nccl_check(ncclCommCount(static_cast<ncclComm_t>(comm), nranks), "ncclCommCount");
        nccl_check(ncclCommUserRank(static_cast<ncclComm_t>(comm), rank), "ncclCommUserRank");
    });
}

int dxrpt_gather_slabs(void* comm, const float* slab, const uint64_t* counts, float* gathered, void* stream) {
    return guarded([&] {
        require(comm && counts, "dxrpt_gather_slabs: null argument");
        ncclComm_t c = static_cast<ncclComm_t>(comm);
        int nranks = 0, rank = 0;
        nccl_check(ncclCommCount(c, &nranks), "ncclCommCount");
        nccl_check(ncclCommUserRank(c, &rank), "ncclCommUserRank");
        require(counts[rank] == 0 || slab, "dxrpt_gather_slabs: null slab");
        require(rank != 0 || gathered, "dxrpt_gather_slabs: rank 0 needs the gathered buffer");
        hipStream_t s = static_cast<hipStream_t>(stream);
        if (rank == 0) {
            uint64_t off = 0;
            nccl_check(ncclGroupStart(), "ncclGroupStart");
            for (int r = 0; r < nranks; ++r) {
                const size_t n = size_t(counts[r]) * 4u;  // float4 pixels -> floats
                if (r == 0) {
                    if (n && gathered + off != slab)
                        hip_check(hipMemcpyAsync(gathered + off, slab, n * sizeof(float), hipMemcpyDeviceToDevice, s),
                                  "hipMemcpyAsync own slab");
                } else if (n) {
                    nccl_check(ncclRecv(gathered + off, n, ncclFloat, r, c, s), "ncclRecv");
                }
                off += n;
            }
            nccl_check(ncclGroupEnd(), "ncclGroupEnd");
        } else if (counts[rank]) {
            nccl_check(ncclSend(slab, size_t(counts[rank]) * 4u, ncclFloat, 0, c, s), "ncclSend");
        }
    });
}

}  // extern "C"
