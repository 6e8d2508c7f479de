// Shared helpers for the gfx950 kernel library (error state, launch checks, activations,
// wave-64 reductions).  Wave size is hard-coded to 64 (CDNA).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/ducosy_hip.h"

namespace dcs {

void set_error(const std::string& msg);

inline int fail(int code, const char* what) {
    set_error(what);
    return code;
}

inline int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error(std::string(what) + ": " + hipGetErrorString(e));
        return (int)e;
    }
    return DCS_OK;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
// records inside a registered range-record arena (dcs_range_arena_register) are zeroed by the
// caller in bulk, once per reuse of the arena
bool in_range_arena(const void* p);
// zero an f16x3 range record before its producer's atomic maxima (a no-op for rng == nullptr and
// for records of a registered arena)
inline int range_zero(float* rng, hipStream_t s) {
    if (!rng || in_range_arena(rng)) return 0;
    const hipError_t e = hipMemsetAsync(rng, 0, DCS_RANGE_PARTS * sizeof(float), s);
    return e == hipSuccess ? 0 : fail((int)e, "range record memset failed");
}
inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

constexpr int WAVE = 64;

__device__ __forceinline__ float act_apply(float v, int act) {
    // act >= DCS_ACT_AFFINE assumed to have been preceded by the affine map
    if (act == DCS_ACT_RELU) return v > 0.f ? v : 0.f;
    if (act == DCS_ACT_LRELU) return v > 0.f ? v : 0.2f * v;
    if (act == DCS_ACT_TANH) return tanhf(v);
    return v;
}

// derivative of act at pre-activation value v (relu'(0) = 0 as in torch threshold_backward)
__device__ __forceinline__ float act_grad(float v, int act) {
    if (act == DCS_ACT_RELU) return v > 0.f ? 1.f : 0.f;
    if (act == DCS_ACT_LRELU) return v > 0.f ? 1.f : 0.2f;
    return 1.f;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// f16x3 range record (include/ducosy_hip.h DCS_RANGE_PARTS): a producer kernel folds the max
// |value| it wrote into rng[block % DCS_RANGE_PARTS] by an atomic max on the float bits
// (non-negative floats order as unsigned ints); the ABI call zeroed rng first (range_zero).
// m: this lane's max |value|; every lane of the wave calls it (the reduction shuffles).
__device__ __forceinline__ void range_note(float* __restrict__ rng, float m) {
    if (!rng) return;  // kernel argument: wave-uniform
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0)
        atomicMax(reinterpret_cast<unsigned int*>(rng) + ((blockIdx.x + blockIdx.y * 7919u) & (DCS_RANGE_PARTS - 1)),
                  __float_as_uint(m));
}
__device__ __forceinline__ float absmax4(const float4& v) {
    return fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// block-wide sum for 256-thread blocks; result valid in every thread
__device__ __forceinline__ float block_sum_256(float v, float* red /* >= 4 floats */) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    float r = red[0] + red[1] + red[2] + red[3];
    return r;
}

__device__ __forceinline__ double block_sum_256_d(double v, double* red) {
    v = wave_sum_d(v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }

__device__ __forceinline__ float sgnf(float x) { return (x > 0.f) ? 1.f : ((x < 0.f) ? -1.f : 0.f); }

// Per-chunk InstanceNorm statistics of one (image, channel): count, mean, sum of squared
// deviations, and the maximum with its first pixel index.  Written by the statistics pass
// (norm.hip) or by the conv rows epilogue (conv.hip), merged by in_stats_finalize8_kernel.
struct Part {
    float cnt, mean, m2, mx;
    int amax;
    int pad[3];
};

// Partial sums of the InstanceNorm backward over a chunk of one image's pixels, per channel:
// a = sum g, b = sum g * xhat with g = da * act'(xhat) (norm.hip in_bwd_*; the window data gradient's
// epilogue and the ring fold write them too, conv_win.hip / conv.hip)
struct Sum2 {
    float a, b;
};

}  // namespace dcs
