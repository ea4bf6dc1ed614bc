// post_kernels.h — launch interface of the post-processing stage (post_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dxrpt {

// Gaussian weights of taps i = -7..6 (CalcGaussianWeight, PostProcessing.hlsl:21-25).
struct PostWeights {
    float w[14];
};

struct PostParams {
    const void* accum;       // W*H float4: the path tracer's accumulation buffer
    void* bloom0;            // (W/2)*(H/2) RGBA16F scratch (the bloom result ends here)
    void* bloom1;            // (W/2)*(H/2) RGBA16F scratch
    void* out;               // W*H float4 (out_format 0) or RGBA8 (1)
    uint32_t width, height;  // >= 2 each
    uint32_t out_format;
    float bloom_magnitude;   // AppSettings.BloomMagnitude
    float bloom_exp2;        // 2^BloomExposure
    float exposure_scale;    // 2^Exposure / FP16Scale
    PostWeights weights;
};

hipError_t launch_post_process(const PostParams& p, hipStream_t stream);

// DenoiseMedian.hlsl (FilterRadius 1): luminance-median of each texel's clamped 3x3 neighbourhood.
hipError_t launch_median3x3(const float4* in, float4* out, uint32_t w, uint32_t h, hipStream_t stream);

}  // namespace dxrpt
