// Device helpers shared by the convolution kernels (conv.hip, conv_win.hip, conv_subpix.hip): MFMA operand vector
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

// Sub-pixel phase weights (conv_subpix.hip): for nearest-x2 upsample + 3x3 zero-pad conv weights
// w[Cout][Cin][3][3], output phase (py, px) at source offset (u, t) sums the 3x3 taps that land on that
// source pixel: rows 0 | 1,2 for phase 0, 0,1 | 2 for phase 1 (likewise columns) -- the upsample folded
// into the weights, four taps per phase instead of nine.
__device__ __forceinline__ float subpix_tapsum(const float* __restrict__ w, int Cin, int co, int ci, int py, int px,
                                               int u, int t) {
    const int ya = py ? (u ? 2 : 0) : (u ? 1 : 0), yb = py ? (u ? 2 : 1) : (u ? 2 : 0);
    const int xa = px ? (t ? 2 : 0) : (t ? 1 : 0), xb = px ? (t ? 2 : 1) : (t ? 2 : 0);
    const float* wp = w + ((long long)co * Cin + ci) * 9;
    float s = 0.f;
    for (int ty = ya; ty <= yb; ++ty)
        for (int tx = xa; tx <= xb; ++tx) s += wp[ty * 3 + tx];
    return s;
}
// B of the forward: virtual row v = (column tile (px, 64-channel block), row phase py, channel), k =
// (16-channel slice, u, t, channel).  B of the data gradient: row = input channel ci, k = (phase, slice
// of the output channels, window offset (1 - u, 1 - t), channel).  [4 Cout or Cin rows][4 Cin or 4 Cout]
__device__ __forceinline__ float subpix_value(const float* __restrict__ w, int Cout, int Cin, int dgrad, int v, int k) {
    const int rem = k & 63, tap = rem >> 4;
    if (!dgrad) {
        const int cblk = Cout >> 6;
        const int ntile = v >> 7, py = (v >> 6) & 1;
        const int px = ntile / cblk, co = (ntile - px * cblk) * 64 + (v & 63);
        return subpix_tapsum(w, Cin, co, (k >> 6) * 16 + (rem & 15), py, px, tap >> 1, tap & 1);
    }
    const int nslice = Cout >> 4, it = k >> 6;
    const int ph = it / nslice, co = (it - ph * nslice) * 16 + (rem & 15);
    return subpix_tapsum(w, Cin, co, v, ph >> 1, ph & 1, 1 - (tap >> 1), 1 - (tap & 1));
}

}  // namespace dcs
