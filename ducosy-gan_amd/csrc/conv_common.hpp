// Device helpers shared by the convolution kernels (conv.hip, conv_win.hip, conv_subpix.hip): MFMA operand vector
// types, the f16x3 operand split and scale exponent, the XCD-aware workgroup order.
#pragma once
#include <type_traits>
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
// maxima of the operand's range record (every wave reduces them itself; wave-uniform result).  All
// sixteen loads of a lane in flight at once (buffer loads past n read 0, the identity of a max over
// maxima >= 0): one memory round trip at a kernel's start instead of one per 128 partials; the wave
// maximum by DPP within rows of 16 lanes, then the four row maxima
static_assert(DCS_RANGE_PARTS <= 1024, "f16x3_exp reduces at most 16 x 64 partial maxima");
__device__ __forceinline__ int f16x3_exp(const float* __restrict__ rng, int n) {
    const int lane = threadIdx.x & 63;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(rng), (short)0, n * 4, 0x00020000);
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (lane + 64 * k) * 4, 0, 0));
    float m = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) m = fmaxf(m, v[k]);
    auto dpp_max = [](float x, auto ctrl) {
        const int y = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), decltype(ctrl)::value, 0xf, 0xf, true);
        return fmaxf(x, __builtin_bit_cast(float, y));
    };
    m = dpp_max(m, std::integral_constant<int, 0xb1>{});   // quad_perm (1, 0, 3, 2)
    m = dpp_max(m, std::integral_constant<int, 0x4e>{});   // quad_perm (2, 3, 0, 1)
    m = dpp_max(m, std::integral_constant<int, 0x124>{});  // row_ror 4
    m = dpp_max(m, std::integral_constant<int, 0x128>{});  // row_ror 8
    const auto rl = [&](int l) { return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, m), l)); };
    m = fmaxf(fmaxf(rl(0), rl(16)), fmaxf(rl(32), rl(48)));
    int e = 0;
    (void)frexpf(m, &e);  // m = f * 2^e, 0.5 <= f < 1 (e = 0 for m = 0)
    int sh = 15 - e;
    sh = sh < -100 ? -100 : (sh > 100 ? 100 : sh);
    return __builtin_amdgcn_readfirstlane(sh);
}

// ring copies of the residual data gradient's padded-grid ring written by conv_win.hip's ring16_kernel
// (one per tap; the ring buffer, dcs_conv_dgrad_reflect_ring_size, holds at least this many)
constexpr int RG_COPIES = 3;

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
// stride-2 3x3 zero-pad-1 convolution (the Generator's down-convolutions) on the same kernels: the
// kernel row ty a window offset reaches for parity class a (or -1: none).  Data gradient (phase
// kernel, offset u from the source row above): a = 0 takes ty = 1 at u = 1; a = 1 takes ty = 2 at
// u = 0 and ty = 0 at u = 1.  Forward (class kernel, offset o from the class row of the output row):
// a = 0 takes ty = 1 at o = 0; a = 1 takes ty = 0 at o = 0 and ty = 2 at o = 1.
__device__ __forceinline__ int s2_dgrad_tap(int a, int u) { return a ? (u ? 0 : 2) : (u ? 1 : -1); }
__device__ __forceinline__ int s2_fwd_tap(int a, int o) { return a ? (o ? 2 : 0) : (o ? -1 : 1); }
// 4x4 stride-2 pad-1 (the PatchGAN layers): every (class, offset) pair is a tap.  Data gradient: a = 0
// takes ty = 3 at u = 0 and 1 at u = 1, a = 1 takes 2 at u = 0 and 0 at u = 1; forward: a = 0 takes 1 at
// o = 0 and 3 at o = 1, a = 1 takes 0 at o = 0 and 2 at o = 1.
__device__ __forceinline__ int k4_dgrad_tap(int a, int u) { return a ? (u ? 0 : 2) : (u ? 1 : 3); }
__device__ __forceinline__ int k4_fwd_tap(int a, int o) { return a ? (o ? 2 : 0) : (o ? 3 : 1); }

// B of the window phase kernels (conv_subpix.hip), kind:
//  0: sub-pixel forward, [4 Cout][4 Cin]: virtual row v = (column tile (px, 64-channel block), row
//     phase py, channel), k = (16-channel slice, u, t, channel);
//  1: sub-pixel data gradient, [Cin][16 Cout]: row = input channel, k = (phase, slice of the output
//     channels, window offset (1 - u, 1 - t), channel);
//  2: stride-2 data gradient, [4 Cin][4 Cout]: kind 0's layout over dx's parity classes;
//  3: stride-2 forward, [Cout][16 Cin]: kind 1's layout over the source's parity classes;
//  4 / 5: the 4x4 stride-2 convolution's forward / data gradient in kind 3's / kind 2's layout.
__device__ __forceinline__ float subpix_value(const float* __restrict__ w, int Cout, int Cin, int kind, int v, int k) {
    const int rem = k & 63, tap = rem >> 4;
    if (kind == 0 || kind == 2 || kind == 5) {
        const int Cv = kind == 0 ? Cout : Cin;  // the kernel's output channels
        const int cblk = Cv >> 6;
        const int ntile = v >> 7, py = (v >> 6) & 1;
        const int px = ntile / cblk, oc = (ntile - px * cblk) * 64 + (v & 63);
        const int rc = (k >> 6) * 16 + (rem & 15);  // reduction channel
        if (kind == 0) return subpix_tapsum(w, Cin, oc, rc, py, px, tap >> 1, tap & 1);
        if (kind == 5) return w[((long long)rc * Cin + oc) * 16 + k4_dgrad_tap(py, tap >> 1) * 4 + k4_dgrad_tap(px, tap & 1)];
        const int ty = s2_dgrad_tap(py, tap >> 1), tx = s2_dgrad_tap(px, tap & 1);
        return (ty < 0 || tx < 0) ? 0.f : w[((long long)rc * Cin + oc) * 9 + ty * 3 + tx];
    }
    const int nslice = (kind == 1 ? Cout : Cin) >> 4, it = k >> 6;
    const int ph = it / nslice, rc = (it - ph * nslice) * 16 + (rem & 15);
    if (kind == 1) return subpix_tapsum(w, Cin, rc, v, ph >> 1, ph & 1, 1 - (tap >> 1), 1 - (tap & 1));
    if (kind == 4) return w[((long long)v * Cin + rc) * 16 + k4_fwd_tap(ph >> 1, tap >> 1) * 4 + k4_fwd_tap(ph & 1, tap & 1)];
    const int ty = s2_fwd_tap(ph >> 1, tap >> 1), tx = s2_fwd_tap(ph & 1, tap & 1);
    return (ty < 0 || tx < 0) ? 0.f : w[((long long)v * Cin + rc) * 9 + ty * 3 + tx];
}
// shapes each kind takes (the kernels' channel tiling)
inline bool subpix_pack_ok(int Cout, int Cin, int kind) {
    if (Cout <= 0 || Cin <= 0 || 16LL * Cout * Cin >= (1LL << 30) || kind < 0 || kind > 5) return false;
    switch (kind) {
        case 0: return Cout % 64 == 0 && Cin % 16 == 0;
        case 1: return Cout % 16 == 0 && Cin % 128 == 0;
        case 2: case 5: return Cin % 64 == 0 && Cout % 16 == 0;
        default: return Cout % 128 == 0 && Cin % 16 == 0;  // 3, 4
    }
}
// rows and k of a kind's planes (rows x K = 16 Cout Cin)
__device__ __host__ __forceinline__ int subpix_K(int Cout, int Cin, int kind) {
    return kind == 0 ? 4 * Cin : kind == 1 ? 16 * Cout : (kind == 2 || kind == 5) ? 4 * Cout : 16 * Cin;
}

}  // namespace dcs
