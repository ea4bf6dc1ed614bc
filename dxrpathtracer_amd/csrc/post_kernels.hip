// post_kernels.hip — the post-processing stage that consumes the path tracer's accumulation buffer
// (PostProcessor::Render, DXRPathTracer/PostProcessor.cpp:43-92; shaders DXRPathTracer/PostProcessing.hlsl).
//
//   k_bloom_down   half-res Bloom pass (:83-99): Gather of the 2x2 footprint, (((c0 + c1) + c2) + c3) / 4
//   k_blur         BlurH / BlurV (:110-118, Blur :29-54): 14 point taps i = -7..6 (asymmetric, as the
//                  reference), un-normalised Gaussian weights; run H, V, H, V (:74-85)
//   k_tonemap      ToneMap (:121-137): point-sampled radiance + bilinear bloom * BloomMagnitude *
//                  2^BloomExposure, * 2^Exposure / FP16Scale, filmic ALU curve (:57-62)
//
// The bloom chain lives in RGBA16F like the reference's temp targets (PostProcessor.cpp:62-69), so each
// pass rounds its output to half.  Sampler behaviour is defined here (D3D leaves filter precision to
// the hardware): PointSampler / LinearSampler are clamp-addressed (DX12_Helpers.cpp:312-317), texel
// of a point sample = floor(coord * size), bilinear at coord * size - 0.5 with float weights, Gather
// order (x0,y1), (x1,y1), (x1,y0), (x0,y0).  Gaussian weights and exposure scales are computed once on
// the host (double, rounded to float).  HBM-bound and tiny (1080p: 33 MB read, 8-33 MB written).
#include <hip/hip_runtime.h>

#include "post_kernels.h"

namespace dxrpt {

namespace {

constexpr int kPostBlock = 256;

__device__ __forceinline__ float lerp_pp(float a, float b, float t) { return a + t * (b - a); }

__device__ __forceinline__ float4 load_h4(const ushort4* p, uint32_t i) {
    const ushort4 h = p[i];
    return make_float4(float(__builtin_bit_cast(_Float16, h.x)), float(__builtin_bit_cast(_Float16, h.y)),
                       float(__builtin_bit_cast(_Float16, h.z)), float(__builtin_bit_cast(_Float16, h.w)));
}

__device__ __forceinline__ ushort4 to_h4(float4 v) {
    return make_ushort4(__builtin_bit_cast(uint16_t, _Float16(v.x)), __builtin_bit_cast(uint16_t, _Float16(v.y)),
                        __builtin_bit_cast(uint16_t, _Float16(v.z)), __builtin_bit_cast(uint16_t, _Float16(v.w)));
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return min(max(v, lo), hi); }

// Bloom (PostProcessing.hlsl:83-99): output pixel (x, y) of the bw x bh target at uv = ((x+.5)/bw, (y+.5)/bh);
// GatherRed/Green/Blue(LinearSampler) on the W x H input.
__global__ __launch_bounds__(kPostBlock) void k_bloom_down(const float4* __restrict__ in, uint32_t W, uint32_t H,
                                                           ushort4* __restrict__ out, uint32_t bw, uint32_t bh) {
    const uint32_t i = blockIdx.x * kPostBlock + threadIdx.x;
    if (i >= bw * bh) return;
    const uint32_t x = i % bw, y = i / bw;
    const float u = (float(x) + 0.5f) / float(bw), v = (float(y) + 0.5f) / float(bh);
    const int x0 = int(floorf(u * float(W) - 0.5f)), y0 = int(floorf(v * float(H) - 0.5f));
    const int xa = clampi(x0, 0, int(W) - 1), xb = clampi(x0 + 1, 0, int(W) - 1);
    const int ya = clampi(y0, 0, int(H) - 1), yb = clampi(y0 + 1, 0, int(H) - 1);
    const float4 c0 = in[size_t(yb) * W + xa], c1 = in[size_t(yb) * W + xb];
    const float4 c2 = in[size_t(ya) * W + xb], c3 = in[size_t(ya) * W + xa];
    float3 r = make_float3(0.0f, 0.0f, 0.0f);
    r.x = (((r.x + c0.x) + c1.x) + c2.x) + c3.x;
    r.y = (((r.y + c0.y) + c1.y) + c2.y) + c3.y;
    r.z = (((r.z + c0.z) + c1.z) + c2.z) + c3.z;
    out[i] = to_h4(make_float4(r.x / 4.0f, r.y / 4.0f, r.z / 4.0f, 1.0f));
}

// Blur (PostProcessing.hlsl:29-54) along x (dx = 1) or y (dx = 0) of a w x h RGBA16F image.
__global__ __launch_bounds__(kPostBlock) void k_blur(const ushort4* __restrict__ in, ushort4* __restrict__ out, uint32_t w,
                                                     uint32_t h, int dx, PostWeights wt) {
    const uint32_t i = blockIdx.x * kPostBlock + threadIdx.x;
    if (i >= w * h) return;
    const uint32_t x = i % w, y = i / w;
    const float u = (float(x) + 0.5f) / float(w), v = (float(y) + 0.5f) / float(h);
    float4 c = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
    for (int k = 0; k < 14; ++k) {
        const int t = k - 7;
        // texCoord += (i / inputSize) * texScale; point sample = floor(texCoord * size), clamped
        const float tu = u + (float(t) / float(w)) * float(dx);
        const float tv = v + (float(t) / float(h)) * float(1 - dx);
        const int sx = clampi(int(floorf(tu * float(w))), 0, int(w) - 1);
        const int sy = clampi(int(floorf(tv * float(h))), 0, int(h) - 1);
        const float4 s = load_h4(in, uint32_t(sy) * w + uint32_t(sx));
        const float g = wt.w[k];
        c.x += s.x * g;
        c.y += s.y * g;
        c.z += s.z * g;
        c.w += s.w * g;
    }
    out[i] = to_h4(c);
}

// ToneMapFilmicALU (PostProcessing.hlsl:57-62)
__device__ __forceinline__ float filmic(float c) {
    c = fmaxf(0.0f, c - 0.004f);
    return (c * (6.2f * c + 0.5f)) / (c * (6.2f * c + 1.7f) + 0.06f);
}

// ToneMap (PostProcessing.hlsl:121-137); out_format 0: float4, 1: RGBA8 UNORM (saturate, x255, round to even).
__global__ __launch_bounds__(kPostBlock) void k_tonemap(const float4* __restrict__ in, const ushort4* __restrict__ bloom,
                                                        uint32_t W, uint32_t H, uint32_t bw, uint32_t bh, float bloom_mag,
                                                        float bloom_exp2, float exposure_scale, void* out, uint32_t out_format) {
    const uint32_t i = blockIdx.x * kPostBlock + threadIdx.x;
    if (i >= W * H) return;
    const uint32_t x = i % W, y = i / W;
    const float4 p = in[i];
    const float u = (float(x) + 0.5f) / float(W), v = (float(y) + 0.5f) / float(H);
    const float tx = u * float(bw) - 0.5f, ty = v * float(bh) - 0.5f;
    const float fx0 = floorf(tx), fy0 = floorf(ty);
    const float fx = tx - fx0, fy = ty - fy0;
    const int xa = clampi(int(fx0), 0, int(bw) - 1), xb = clampi(int(fx0) + 1, 0, int(bw) - 1);
    const int ya = clampi(int(fy0), 0, int(bh) - 1), yb = clampi(int(fy0) + 1, 0, int(bh) - 1);
    const float4 t00 = load_h4(bloom, uint32_t(ya) * bw + uint32_t(xa)), t10 = load_h4(bloom, uint32_t(ya) * bw + uint32_t(xb));
    const float4 t01 = load_h4(bloom, uint32_t(yb) * bw + uint32_t(xa)), t11 = load_h4(bloom, uint32_t(yb) * bw + uint32_t(xb));
    const float bx = lerp_pp(lerp_pp(t00.x, t10.x, fx), lerp_pp(t01.x, t11.x, fx), fy);
    const float by = lerp_pp(lerp_pp(t00.y, t10.y, fx), lerp_pp(t01.y, t11.y, fx), fy);
    const float bz = lerp_pp(lerp_pp(t00.z, t10.z, fx), lerp_pp(t01.z, t11.z, fx), fy);
    float r = p.x + (bx * bloom_mag) * bloom_exp2;
    float g = p.y + (by * bloom_mag) * bloom_exp2;
    float b = p.z + (bz * bloom_mag) * bloom_exp2;
    r = filmic(r * exposure_scale);
    g = filmic(g * exposure_scale);
    b = filmic(b * exposure_scale);
    if (out_format == 0) {
        static_cast<float4*>(out)[i] = make_float4(r, g, b, 1.0f);
    } else {
        const uint32_t R = uint32_t(rintf(fminf(fmaxf(r, 0.0f), 1.0f) * 255.0f));
        const uint32_t G = uint32_t(rintf(fminf(fmaxf(g, 0.0f), 1.0f) * 255.0f));
        const uint32_t B = uint32_t(rintf(fminf(fmaxf(b, 0.0f), 1.0f) * 255.0f));
        static_cast<uint32_t*>(out)[i] = R | (G << 8) | (B << 16) | (255u << 24);
    }
}

uint32_t blocks(uint64_t n) { return uint32_t((n + kPostBlock - 1) / kPostBlock); }

}  // namespace

// DenoiseCS (DenoiseMedian.hlsl:49-102): the 3x3 neighbourhood (coordinates clamped to the image) sorted
// by luminance with the shader's insertion sort, the middle element (index 4) written with alpha 1.
// The insertion sort is unrolled into compare-and-swap steps with static indices (the array stays in
// registers): inserting element a walks j = a-1 .. 0 and swaps while the element before is brighter;
// the `moving` flag stops the walk exactly where the shader's while loop stops (NaN keys included).
__global__ __launch_bounds__(kPostBlock) void k_median3x3(const float4* __restrict__ in, float4* __restrict__ out,
                                                          uint32_t w, uint32_t h) {
    const uint32_t i = blockIdx.x * kPostBlock + threadIdx.x;
    if (i >= w * h) return;
    const int x = int(i % w), y = int(i / w);
    float3 nb[9];
    float lum[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const int cx = min(max(x + (k % 3) - 1, 0), int(w) - 1), cy = min(max(y + (k / 3) - 1, 0), int(h) - 1);
        const float4 v = in[size_t(cy) * w + cx];
        nb[k] = make_float3(v.x, v.y, v.z);
        lum[k] = (v.x * 0.299f + v.y * 0.587f) + v.z * 0.114f;
    }
#pragma unroll
    for (int a = 1; a < 9; ++a) {
        bool moving = true;
#pragma unroll
        for (int j = a - 1; j >= 0; --j) {
            moving = moving && (lum[j] > lum[j + 1]);
            const float3 lo = nb[j], hi = nb[j + 1];
            const float ll = lum[j], lh = lum[j + 1];
            nb[j] = moving ? hi : lo;
            nb[j + 1] = moving ? lo : hi;
            lum[j] = moving ? lh : ll;
            lum[j + 1] = moving ? ll : lh;
        }
    }
    out[i] = make_float4(nb[4].x, nb[4].y, nb[4].z, 1.0f);
}

hipError_t launch_median3x3(const float4* in, float4* out, uint32_t w, uint32_t h, hipStream_t stream) {
    hipLaunchKernelGGL(k_median3x3, dim3(blocks(uint64_t(w) * h)), dim3(kPostBlock), 0, stream, in, out, w, h);
    return hipGetLastError();
}

hipError_t launch_post_process(const PostParams& p, hipStream_t stream) {
    const uint32_t bw = p.width / 2, bh = p.height / 2;
    if (bw > 0 && bh > 0) {
        hipLaunchKernelGGL(k_bloom_down, dim3(blocks(uint64_t(bw) * bh)), dim3(kPostBlock), 0, stream,
                           static_cast<const float4*>(p.accum), p.width, p.height, static_cast<ushort4*>(p.bloom0), bw, bh);
        for (int it = 0; it < 2; ++it) {  // PostProcessor.cpp:74-85
            hipLaunchKernelGGL(k_blur, dim3(blocks(uint64_t(bw) * bh)), dim3(kPostBlock), 0, stream,
                               static_cast<const ushort4*>(p.bloom0), static_cast<ushort4*>(p.bloom1), bw, bh, 1, p.weights);
            hipLaunchKernelGGL(k_blur, dim3(blocks(uint64_t(bw) * bh)), dim3(kPostBlock), 0, stream,
                               static_cast<const ushort4*>(p.bloom1), static_cast<ushort4*>(p.bloom0), bw, bh, 0, p.weights);
        }
    }
    hipLaunchKernelGGL(k_tonemap, dim3(blocks(uint64_t(p.width) * p.height)), dim3(kPostBlock), 0, stream,
                       static_cast<const float4*>(p.accum), static_cast<const ushort4*>(p.bloom0), p.width, p.height,
                       bw > 0 ? bw : 1u, bh > 0 ? bh : 1u, p.bloom_magnitude, p.bloom_exp2, p.exposure_scale, p.out,
                       p.out_format);
    return hipGetLastError();
}

}  // namespace dxrpt
