// Device helpers shared by the convolution kernels (conv.hip, conv_win.hip): MFMA operand vector
// types, the f16x3 operand split and scale exponent, the XCD-aware workgroup order.
#pragma once
#include "common.hpp"

namespace dcs {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx8 __attribute__((ext_vector_type(8)));
typedef float f32x4v __attribute__((ext_vector_type(4)));

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

// f16x3 split: v' = v * 2^s (exact), hi = fp16(v'), lo = fp16(v' - hi) (the residual is exact in
// fp32; |v' - hi - lo| <= 2^-22 |v'| while |v'| < 2^15 and lo is normal, else an absolute
// 2^-25 floor from the fp16 denormals, far below the tensor's 2^15 top)
__device__ __forceinline__ void split8h(const float4& a, const float4& b, float sc, f16x8& hi, f16x8& lo) {
    const floatx8 f = floatx8{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w} * sc;
    hi = __builtin_convertvector(f, f16x8);
    lo = __builtin_convertvector(f - __builtin_convertvector(hi, floatx8), f16x8);
}
__device__ __forceinline__ void split4h(const float4& a, float sc, f16x4& hi, f16x4& lo) {
    const f32x4v f = f32x4v{a.x, a.y, a.z, a.w} * sc;
    hi = __builtin_convertvector(f, f16x4);
    lo = __builtin_convertvector(f - __builtin_convertvector(hi, f32x4v), f16x4);
}

// f16x3 operand exponent: s with max|operand| * 2^s < 2^15, from the n (<= 1024) partial
// maxima of the operand's range record (every wave reduces them itself; wave-uniform result)
__device__ __forceinline__ int f16x3_exp(const float* __restrict__ rng, int n) {
    const int lane = threadIdx.x & 63;
    float m = 0.f;
    for (int i = lane; i < n; i += 64) m = fmaxf(m, rng[i]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    int e = 0;
    (void)frexpf(m, &e);  // m = f * 2^e, 0.5 <= f < 1 (e = 0 for m = 0)
    int sh = 15 - e;
    sh = sh < -100 ? -100 : (sh > 100 ? 100 : sh);
    return __builtin_amdgcn_readfirstlane(sh);
}

__device__ __forceinline__ int xcd_remap(int L, int T) {
    // bijective: blocks L, L+8, ... share an XCD under round-robin dispatch
    const int xcd = L & 7, q = T >> 3, r = T & 7;
    const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + (L >> 3);
}

}  // namespace dcs
