// Convolution family for the DuCoSy-GAN hot path on gfx950 (MI355X).
//
// Every nn.Conv2d of modules/model.py (Generator :94-112, ResidualBlockWithCBAM :72-80,
// Discriminator :122-129) in forward, data-gradient and weight-gradient form is one
// implicit GEMM on the f32 MFMA (v_mfma_f32_32x32x2_f32, exact fp32):
//
//   rows pass   out[m][n] = sum_k  A[m][k] * B[k][n]
//       m = output pixel, k = (tap, source channel), n = output channel
//       A is gathered on the fly from the NHWC source (reflection/zero padding, nearest
//       x2 upsampling, channel-concat of two sources, stride 1/2, and stride-2 transposed
//       "parity classes" are all folded into the gather — never materialised), with the
//       previous layer's InstanceNorm + ReLU/LeakyReLU applied as a per-(n,c) prologue.
//       B is the packed weight matrix.
//   wgrad pass  dW[co][k] = sum_pixels dy[p][co] * A[p][k], split over pixels, partial
//       slabs reduced deterministically by a second kernel.
//
// Tiling: 256-thread workgroups (4 waves as 2x2), BM x BN output tile, BK = 32, register-
// staged double-buffered LDS ([k][m] layouts, m contiguous, padded by 4 floats), each wave
// owns (BM/2)x(BN/2) = 2x2 or 2x1 32x32 MFMA accumulators.
#include "common.hpp"
#include "conv_common.hpp"

namespace dcs {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// MFMA operand modes (dcs_conv_desc.mma): exact f32 (v_mfma_f32_32x32x2_f32), bf16 operands
// (v_mfma_f32_32x32x16_bf16, f32 accumulation: BASELINE config 5's half-precision MFMA path),
// and bf16x3 (each f32 operand split into hi + lo bf16, three MFMAs hi*hi + hi*lo + lo*hi:
// ~2^-16 relative per product instead of 2^-24, at 3/16 of the f32-MFMA cycles per FLOP).
constexpr int MMA_F32 = 0, MMA_BF16 = 1, MMA_BF16X3 = 3, MMA_BF16X6 = 6;
// internal: DCS_MMA_BF16 on the bf16x6 pipeline with its three LDS planes used as three
// consecutive 16-k sub-tiles (48 k per barrier, one product each), for the residual convs
constexpr int MMA_BF16P = 2;
// f16x3 (DCS_MMA_F16X3): fp32 operands scaled by a power of two and split into hi + lo fp16,
// three products on v_mfma_f32_32x32x16_f16 (include/ducosy_hip.h)
constexpr int MMA_F16X3 = 7;
// f16 (DCS_MMA_F16): the f16x3 staging with the hi planes only, one product (hi*hi) per fragment
constexpr int MMA_F16 = 8;
#ifndef DCS_BF16_BUFGATHER
#define DCS_BF16_BUFGATHER 1  // branch-free buffer-descriptor gather in the bf16 rows pass
#endif

// bf16 LDS rows of the rows pass: 32 k of hi (+ 32 k of lo for bf16x3) + 8 pad elements;
// 80-B / 144-B pitches keep the per-lane 16-B fragment reads conflict-free.
template <int MMA>
constexpr int lde_bf16() { return MMA == MMA_BF16X3 ? 72 : 40; }

// split 8 floats into hi (round-to-nearest bf16, one v_cvt_pk_bf16_f32 per pair) and, for
// bf16x3, lo = bf16(v - hi) with hi re-expanded by bit shifts (bf16 -> f32 is exact)
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
template <int MMA>
__device__ __forceinline__ void split8(const float4& a, const float4& b, bf16x8& hi, bf16x8& lo) {
    const floatx8 f = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    hi = __builtin_convertvector(f, bf16x8);
    if constexpr (MMA == MMA_BF16X3) {
        u32x4v w;
        __builtin_memcpy(&w, &hi, 16);
        floatx8 r;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            r[2 * q] = f[2 * q] - __uint_as_float(w[q] << 16);
            r[2 * q + 1] = f[2 * q + 1] - __uint_as_float(w[q] & 0xffff0000u);
        }
        lo = __builtin_convertvector(r, bf16x8);
    }
}

// three-way split for bf16x6: v = hi + mid + lo (each bf16, residuals exact in f32); the six
// products that matter (all but mid*lo, lo*mid, lo*lo, each <= 2^-27 relative) give ~2^-24
// relative error per product: fp32-class.  Each rounded pair is re-expanded from its packed
// register (low half << 16, high half & 0xffff0000): one op per value instead of a second
// single-value conversion plus a shift
__device__ __forceinline__ floatx8 unpack8(const bf16x8& h) {
    u32x4v w;
    __builtin_memcpy(&w, &h, 16);
    floatx8 r;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        r[2 * q] = __uint_as_float(w[q] << 16);
        r[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
    }
    return r;
}
__device__ __forceinline__ void split8x3(const float4& a, const float4& b, bf16x8& hi, bf16x8& mid, bf16x8& lo) {
    const floatx8 f = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    hi = __builtin_convertvector(f, bf16x8);
    const floatx8 r1 = f - unpack8(hi);
    mid = __builtin_convertvector(r1, bf16x8);
    const floatx8 r2 = r1 - unpack8(mid);
    lo = __builtin_convertvector(r2, bf16x8);
}

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x4v unpack4(const bf16x4& h) {
    u32x2v w;
    __builtin_memcpy(&w, &h, 8);
    return f32x4v{__uint_as_float(w[0] << 16), __uint_as_float(w[0] & 0xffff0000u),
                  __uint_as_float(w[1] << 16), __uint_as_float(w[1] & 0xffff0000u)};
}
__device__ __forceinline__ void split4x3(const float4& a, bf16x4& hi, bf16x4& mid, bf16x4& lo) {
    const f32x4v f = {a.x, a.y, a.z, a.w};
    hi = __builtin_convertvector(f, bf16x4);
    const f32x4v r1 = f - unpack4(hi);
    mid = __builtin_convertvector(r1, bf16x4);
    const f32x4v r2 = r1 - unpack4(mid);
    lo = __builtin_convertvector(r2, bf16x4);
}

constexpr int BK = 32;
constexpr int NT = 256;
#ifndef DCS_X6_BK
#define DCS_X6_BK 16
#endif
#ifndef DCS_TAG2
#define DCS_TAG2 1  // TAG-2 instances (no prologue / epilogue activation) for the generic x6 / f16x3 passes
#endif
#ifndef DCS_WGRAD_WIN
#define DCS_WGRAD_WIN 1  // f16x3 residual weight gradient on the rolling-window kernel (conv_win.hip)
#endif
#ifndef DCS_WGRAD_X6
#define DCS_WGRAD_X6 1  // bf16x6 weight-gradient kernel in the bf16x6 mode
#endif
#ifndef DCS_WGRAD_X6_CO64
#define DCS_WGRAD_X6_CO64 1  // ... also for 64 output channels in the fp16 modes (128-row tile, half masked): f16x3 up2 at bs 16
                             // 2.15 ms vs 2.48 ms f32 (bf16x6 was 3.49 ms: off there), profiles/r03d
#endif
#ifndef DCS_X6_BN64
#define DCS_X6_BN64 1  // bf16x6 rows also for 64-column tiles
#endif
#ifndef DCS_X6_V4
#define DCS_X6_V4 1  // bf16x6 rows also for the 4-channel NHWC gather (stem, PatchGAN layer 0)
#endif
#ifndef DCS_X6_PIPE
#define DCS_X6_PIPE 1  // bf16x6 rows: global loads two k-tiles ahead (two register sets)
#endif
#ifndef DCS_X6_SELGATHER
#define DCS_X6_SELGATHER 1  // bf16x6 rows: gather address by selects, no exec-mask branch
#endif
#ifndef DCS_X6_STORE_FIRST
#define DCS_X6_STORE_FIRST 1  // bf16x6 rows: stage the next tile before folding the chain
#endif
#ifndef DCS_KSLICE_ALL
#define DCS_KSLICE_ALL 1  // bf16x6 rows: slice-major K walk for every 16-channel-aligned source
#endif
#ifndef DCS_X6_SGB
#define DCS_X6_SGB 5  // bf16x6 residual rows: VALU instructions scheduled after each MFMA (0 = compiler)
#endif
#ifndef DCS_WGRAD_SGB
#define DCS_WGRAD_SGB 5  // bf16x6 weight gradient: VALU instructions scheduled after each MFMA
#endif
#ifndef DCS_X6_SGB0
#define DCS_X6_SGB0 0  // ... the same for the other bf16x6 rows kernels
#endif
#ifndef DCS_BF16P
#define DCS_BF16P 1  // half-precision residual convs on the x6 pipeline (48 k per barrier)
#endif
#ifndef DCS_BF16P_ROWS
#define DCS_BF16P_ROWS 1  // the residual rows passes too (else the plain bf16 rows kernel)
#endif
#ifndef DCS_BF16P_BM256
#define DCS_BF16P_BM256 1  // ... on 256-row tiles where they divide the pixels
#endif
#ifndef DCS_WGRAD_REDUCE_UNROLL
#define DCS_WGRAD_REDUCE_UNROLL 8
#endif
#ifndef DCS_X6_OCC
#define DCS_X6_OCC 2  // bf16x6 rows: workgroups per CU the register budget is sized for
#endif
#ifndef DCS_H3_NSUB
#define DCS_H3_NSUB 2  // f16x3 rows, 128-column tiles: 16-k sub-tiles per barrier (64-column tiles: 1)
#endif
#ifndef DCS_WGRAD_X6_V4
#define DCS_WGRAD_X6_V4 1  // fp16 modes: 4-channel-source weight gradients (stem, PatchGAN layer 0) on the x6 kernel
#endif
#ifndef DCS_TAG4
#define DCS_TAG4 1  // the Generator stem's rows instance: per-row reflected offset tables, compile-time 7x7 x 4
#endif
#ifndef DCS_TAG3
#define DCS_TAG3 1  // PatchGAN layers 1-3: rows / x6 weight-gradient instances with the IN + LeakyReLU gather fixed
#endif
#ifndef DCS_UWALK
#define DCS_UWALK 1  // slice-major rows gathers: the (tap, slice) walk in uniform registers (no per-lane tap decode)
#endif
#ifndef DCS_X6_BM256
#define DCS_X6_BM256 1  // bf16x6 residual rows: 256 x 128 tiles (512 threads)
#endif


// ---------------------------------------------------------------------------------------
// geometry helpers
// ---------------------------------------------------------------------------------------
struct ClassGeom {
    int My, Mx, ntaps, ry, rx;
};

__device__ __host__ inline ClassGeom class_geom(const dcs_conv_desc& d, int z) {
    ClassGeom g;
    if (!d.parity) {
        g.My = d.Ho; g.Mx = d.Wo; g.ntaps = d.KH * d.KW; g.ry = 0; g.rx = 0;
    } else if (d.parity == 2) {  // sub-pixel phases of nearest-x2 upsample + 3x3 conv
        g.ry = z >> 1; g.rx = z & 1;
        g.My = d.Hs; g.Mx = d.Ws; g.ntaps = 4;
    } else {
        g.ry = z >> 1; g.rx = z & 1;
        g.My = (d.Ho - g.ry + 1) >> 1;
        g.Mx = (d.Wo - g.rx + 1) >> 1;
        int ty0 = (g.ry + d.pt) & 1, tx0 = (g.rx + d.pl) & 1;
        int nty = (d.KH - ty0 + 1) >> 1, ntx = (d.KW - tx0 + 1) >> 1;
        g.ntaps = nty * ntx;
    }
    return g;
}

// tap j of class z -> offset added to the row's base source coordinate, and the packed tap
__device__ __forceinline__ void tap_decode(const dcs_conv_desc& d, const ClassGeom& g, int j,
                                           int& ady, int& adx, int& btap) {
    if (!d.parity) {
        int ty = j / d.KW, tx = j - ty * d.KW;
        ady = ty; adx = tx; btap = j;
    } else if (d.parity == 2) {  // phase (ry, rx), 2x2 taps at source offsets r-1+{0,1}
        const int jy = j >> 1, jx = j & 1;
        ady = g.ry - 1 + jy; adx = g.rx - 1 + jx;
        btap = (2 * g.ry + g.rx) * 4 + j;
    } else {
        int ty0 = (g.ry + d.pt) & 1, tx0 = (g.rx + d.pl) & 1;
        int ntx = (d.KW - tx0 + 1) >> 1;
        int jy = j / ntx, jx = j - jy * ntx;
        int ty = ty0 + 2 * jy, tx = tx0 + 2 * jx;
        ady = (g.ry + d.pt - ty) >> 1;  // exact (even numerator)
        adx = (g.rx + d.pl - tx) >> 1;
        btap = ty * d.KW + tx;
    }
}

// virtual coordinate -> source coordinate (padding + nearest upsampling); false = zero pad
__device__ __forceinline__ bool map_coord(int v, int Hv, int up, int mode, int& s) {
    if (v < 0 || v >= Hv) {
        if (mode == DCS_PAD_ZERO) return false;
        v = v < 0 ? -v : 2 * (Hv - 1) - v;
    }
    s = up == 2 ? (v >> 1) : v;
    return true;
}

// Branch-free variant for the vectorised gathers: returns validity, writes the source coordinate.
__device__ __forceinline__ bool map_coord_sel(int v, int Hv, int up, int mode, int& s) {
    const bool inside = (unsigned)v < (unsigned)Hv;
    const int r = v < 0 ? -v : 2 * (Hv - 1) - v;
    const int c = inside ? v : r;
    s = up == 2 ? (c >> 1) : c;
    return inside || mode == DCS_PAD_REFLECT;
}

// Source reads of the vectorised gathers go through a raw buffer descriptor: a 32-bit byte
// offset per lane, and the hardware range check returns zeros for offset OOB_OFF, so zero
// padding and rows past the end need no branches (the host keeps every source < 2 GiB).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int OOB_OFF = 0x7fffffff - 64;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t src_rsrc(const float* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, 0x7fffff00, 0x00020000);
}

__device__ __forceinline__ float2 buf_load2(__amdgpu_buffer_rsrc_t r, int byte_off) {
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, byte_off, 0, 0);
    float2 f;
    __builtin_memcpy(&f, &v, 8);
    return f;
}

__device__ __forceinline__ float4 buf_load4(__amdgpu_buffer_rsrc_t r, int byte_off) {
    u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0);
    float4 f;
    __builtin_memcpy(&f, &v, 16);
    return f;
}

struct RowInfo {
    int n, by, bx;        // image, base virtual source coords
    long long out_off;    // element offset of the output pixel (channel 0), -1 if invalid
};

// fold (conv_rows_kernel of dcs_conv_dgrad_reflect only): see the fold branches below
__device__ __forceinline__ RowInfo row_info(const dcs_conv_desc& d, const ClassGeom& g, int m, int fold = 0) {
    // 32-bit index math: the host guarantees N*My*Mx < 2^31
    RowInfo r;
    if (fold == 2) {
        // the one-pixel ring of the (H+2) x (W+2) padded grid only (dcs_conv_dgrad_reflect_win: the
        // interior comes from the window kernel), rows in the ring buffer's order: top row, bottom
        // row, then (left, right) of rows 1..H; out_off indexes the ring buffer
        // The rows are enumerated segment by segment over the whole batch (every image's top row,
        // then every bottom row, left column, right column), so a 128-row tile lies in one segment
        // and reads only that segment's kernel row / column of taps (ring_tap_mask)
        const int H = d.Ho - 2, ringlen = 2 * d.Wo + 2 * H;
        if (m >= ringlen * d.N) { r.n = 0; r.by = -100000; r.bx = -100000; r.out_off = -1; return r; }
        int n, idx, oy, ox;
        const int sw = d.N * d.Wo, sh = d.N * H;
        if (m < 2 * sw) {  // top / bottom rows
            const int u = m < sw ? m : m - sw;
            n = u / d.Wo;
            ox = u - n * d.Wo;
            oy = m < sw ? 0 : d.Ho - 1;
            idx = (m < sw ? 0 : d.Wo) + ox;
        } else {           // left / right columns of rows 1 .. H
            const int v = m - 2 * sw, right = v >= sh ? 1 : 0, u = right ? v - sh : v;
            n = u / H;
            oy = 1 + (u - n * H);
            ox = right ? d.Wo - 1 : 0;
            idx = 2 * d.Wo + 2 * (oy - 1) + right;
        }
        r.n = n;
        r.by = oy * d.stride - d.pt;
        r.bx = ox * d.stride - d.pl;
        r.out_off = ((long long)n * ringlen + idx) * d.Co;
        return r;
    }
    const int per = g.My * g.Mx;
    if (m >= per * d.N) { r.n = 0; r.by = -100000; r.bx = -100000; r.out_off = -1; return r; }
    const int n = m / per;
    const int rem = m - n * per;
    const int qy = rem / g.Mx, qx = rem - qy * g.Mx;
    int oy, ox;
    if (!d.parity) {
        oy = qy; ox = qx;
        r.by = oy * d.stride - d.pt;
        r.bx = ox * d.stride - d.pl;
    } else {
        oy = 2 * qy + g.ry; ox = 2 * qx + g.rx;
        r.by = qy; r.bx = qx;
    }
    r.n = n;
    if (fold) {
        // dcs_conv_dgrad_reflect (pad 1): interior pixels of the (H+2) x (W+2) padded grid go to
        // the unpadded N x H x W tensor, the one-pixel ring to the ring area behind it
        const int H = d.Ho - 2, W = d.Wo - 2;
        if (oy >= 1 && oy <= H && ox >= 1 && ox <= W) {
            r.out_off = ((long long)(n * H + oy - 1) * W + ox - 1) * d.Co;
        } else {
            const int ring = 2 * d.Wo + 2 * H;
            const int idx = oy == 0 ? ox : (oy == d.Ho - 1 ? d.Wo + ox : 2 * d.Wo + 2 * (oy - 1) + (ox == 0 ? 0 : 1));
            r.out_off = ((long long)d.N * H * W + (long long)n * ring + idx) * d.Co;
        }
        return r;
    }
    r.out_off = ((long long)(n * d.Ho + oy) * d.Wo + ox) * d.Co;
    return r;
}

__device__ __forceinline__ float4 affine_act4(float4 v, const float* sc, const float* sh, int act) {
    float4 s = *reinterpret_cast<const float4*>(sc);
    float4 b = *reinterpret_cast<const float4*>(sh);
    v.x = act_apply(fmaf(v.x, s.x, b.x), act);
    v.y = act_apply(fmaf(v.y, s.y, b.y), act);
    v.z = act_apply(fmaf(v.z, s.z, b.z), act);
    v.w = act_apply(fmaf(v.w, s.w, b.w), act);
    return v;
}

// gather 4 consecutive source channels (c..c+3, same tap) for a row; Cs % 4 == 0, s_c == 1
__device__ __forceinline__ float4 gather4(const dcs_conv_desc& d, const float* __restrict__ src,
                                          const float* __restrict__ psc, const float* __restrict__ psh,
                                          int n, int vy, int vx, int c) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    int sy, sx;
    const int Hv = d.Hs * d.up, Wv = d.Ws * d.up;
    if (map_coord(vy, Hv, d.up, d.pad_mode, sy) && map_coord(vx, Wv, d.up, d.pad_mode, sx)) {
        v = *reinterpret_cast<const float4*>(src + n * d.s_n + sy * d.s_h + sx * d.s_w + c);
        if (d.pro_act != DCS_ACT_NONE) {
            long long o = (long long)n * d.Cs + c;
            v = affine_act4(v, psc + o, psh + o, d.pro_act);
        }
    }
    return v;
}

// gather one source element (general strides, concat of two sources)
__device__ __forceinline__ float gather1(const dcs_conv_desc& d, const float* __restrict__ src,
                                         const float* __restrict__ src2,
                                         const float* __restrict__ psc, const float* __restrict__ psh,
                                         int n, int vy, int vx, int c) {
    int sy, sx;
    const int Hv = d.Hs * d.up, Wv = d.Ws * d.up;
    if (!(map_coord(vy, Hv, d.up, d.pad_mode, sy) && map_coord(vx, Wv, d.up, d.pad_mode, sx)))
        return 0.f;
    float v;
    if (c < d.csplit)
        v = src[n * d.s_n + (long long)c * d.s_c + sy * d.s_h + sx * d.s_w];
    else
        v = src2[n * d.s2_n + (long long)(c - d.csplit) * d.s2_c + sy * d.s2_h + sx * d.s2_w];
    if (d.pro_act != DCS_ACT_NONE) {
        long long o = (long long)n * d.Cs + c;
        v = act_apply(fmaf(v, psc[o], psh[o]), d.pro_act);
    }
    return v;
}

// ---------------------------------------------------------------------------------------
// weight packing
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ float pack_value(const float* __restrict__ w, int Cout, int Cin, int KH, int KW,
                                           int kind, int ci_count, int Kpad, int ncols, int nmajor, long long idx) {
    // element (k, col) of the logical [Kpad][ncols] GEMM B matrix; stored N-major
    // ([ncols][Kpad], MFMA rows pass) or K-major ([Kpad][ncols], narrow kernels)
    int k, col;
    if (nmajor) { col = (int)(idx / Kpad); k = (int)(idx - (long long)col * Kpad); }
    else { k = (int)(idx / ncols); col = (int)(idx - (long long)k * ncols); }
    int taps = KH * KW;
    if (kind & DCS_PACK_KSLICE) {  // K rows in slice-major order: k' = (c/16)*taps*16 + tap*16 + c%16
        kind &= 7;
        const int C = kind == 0 ? Cin : Cout;  // reduction channels per tap
        const int per = taps * 16;
        if (k < taps * C) {
            const int slice = k / per, rem = k - slice * per;
            const int tap = rem >> 4, cs = rem & 15;
            k = tap * C + slice * 16 + cs;
        } else {
            k = 1 << 30;  // K padding: zero
        }
    }
    float v = 0.f;
    if (kind == 3 || kind == 4) {
        // nearest-x2 upsample + 3x3 conv (zero pad 1) split into sub-pixel phases; each
        // phase/tap weight is a sum of original taps.  Row sets per (phase r, tap a):
        //   kind 3 (forward, class z = 2ry+rx, tap j = 2a+b): S(0,0)={0} S(0,1)={1,2} S(1,0)={0,1} S(1,1)={2}
        //   kind 4 (adjoint = 4x4 stride-2 pad-1 conv over dy, tap u): T(0)={2} T(1)={1,2} T(2)={0,1} T(3)={0}
        // encoded as [first, last] original-tap ranges.
        const int C1 = kind == 3 ? Cin : Cout;   // reduction channels per packed tap
        const int pt = k / C1, c1 = k - pt * C1;
        int y0, y1, x0, x1;
        bool ok;
        if (kind == 3) {
            const int z = pt >> 2, j = pt & 3;
            const int ry = z >> 1, rx = z & 1, a = j >> 1, b = j & 1;
            ok = pt < 16 && col < Cout;
            y0 = ry == 0 ? (a == 0 ? 0 : 1) : (a == 0 ? 0 : 2);
            y1 = ry == 0 ? (a == 0 ? 0 : 2) : (a == 0 ? 1 : 2);
            x0 = rx == 0 ? (b == 0 ? 0 : 1) : (b == 0 ? 0 : 2);
            x1 = rx == 0 ? (b == 0 ? 0 : 2) : (b == 0 ? 1 : 2);
        } else {
            const int u = pt >> 2, vv = pt & 3;
            ok = pt < 16 && col < ci_count;
            y0 = u == 0 ? 2 : (u == 1 ? 1 : 0);
            y1 = u == 0 ? 2 : (u == 3 ? 0 : (u == 1 ? 2 : 1));
            x0 = vv == 0 ? 2 : (vv == 1 ? 1 : 0);
            x1 = vv == 0 ? 2 : (vv == 3 ? 0 : (vv == 1 ? 2 : 1));
        }
        if (ok) {
            const int co = kind == 3 ? col : c1, ci = kind == 3 ? c1 : col;
            const float* wp = w + ((long long)co * Cin + ci) * 9;
            float acc = 0.f;
            for (int ty = y0; ty <= y1; ++ty)
                for (int tx = x0; tx <= x1; ++tx) acc += wp[ty * 3 + tx];
            v = acc;
        }
    } else if (kind == 5) {  // B[(tap)*ci_count + ci][co], zero for ci >= Cin (padded source)
        int tap = k / ci_count, ci = k - tap * ci_count;
        if (tap < taps && col < Cout && ci < Cin) {
            int ty = tap / KW, tx = tap - ty * KW;
            v = w[(((long long)col * Cin + ci) * KH + ty) * KW + tx];
        }
    } else if (kind == 0) {  // B[(tap)*Cin + ci][co]
        int tap = k / Cin, ci = k - tap * Cin;
        if (tap < taps && col < Cout) {
            int ty = tap / KW, tx = tap - ty * KW;
            v = w[(((long long)col * Cin + ci) * KH + ty) * KW + tx];
        }
    } else {  // B[(tap)*Cout + co][ci]
        int tap = k / Cout, co = k - tap * Cout;
        if (tap < taps && col < ci_count) {
            int ty = tap / KW, tx = tap - ty * KW;
            if (kind == 1) { ty = KH - 1 - ty; tx = KW - 1 - tx; }
            v = w[(((long long)co * Cin + col) * KH + ty) * KW + tx];
        }
    }
    return v;
}

__global__ void pack_weights_kernel(const float* __restrict__ w, int Cout, int Cin, int KH, int KW,
                                    int kind, int ci_count, int Kpad, int ncols, int nmajor,
                                    float* __restrict__ out) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)Kpad * ncols) return;
    out[idx] = pack_value(w, Cout, Cin, KH, KW, kind, ci_count, Kpad, ncols, nmajor, idx);
}

// the same over a DCS_RANGE_PARTS-block grid-stride walk, each block also writing the max
// |value| it packed (the rng_b range record of an f16x3 rows pass over these weights)
__global__ __launch_bounds__(256) void pack_weights_r_kernel(const float* __restrict__ w, int Cout, int Cin, int KH,
                                                             int KW, int kind, int ci_count, int Kpad, int ncols,
                                                             int nmajor, float* __restrict__ out,
                                                             float* __restrict__ rng) {
    const long long total = (long long)Kpad * ncols;
    float m = 0.f;
    for (long long idx = (long long)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
        const float v = pack_value(w, Cout, Cin, KH, KW, kind, ci_count, Kpad, ncols, nmajor, idx);
        out[idx] = v;
        m = fmaxf(m, fabsf(v));
    }
    __shared__ float red[4];
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) rng[blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (blockIdx.x == 0)  // a grid smaller than the record: the remaining partial maxima are zero
        for (int i = gridDim.x + threadIdx.x; i < DCS_RANGE_PARTS; i += blockDim.x) rng[i] = 0.f;
}

// ---------------------------------------------------------------------------------------
// rows pass: implicit GEMM on v_mfma_f32_32x32x2_f32
//
// LDS holds both operands k-contiguous ([row][32 k + 4 pad], 144-B rows: conflict-free for
// ds_read_b128).  A k-tile of 32 is consumed in 16 MFMA k-steps with a permuted k order:
// at step s, lane half h (lanes 0-31 / 32-63) supplies k = 16h + s for both A and B, so each
// lane fetches its whole k-tile of fragments with 4 ds_read_b128 per 32x32 block, issued
// before the 64 MFMAs of the tile (no per-step lgkmcnt waits).  The global loads of the next
// k-tile are in flight during the MFMAs (register staging, one barrier per k-tile).
// Workgroups are remapped XCD-aware: each XCD walks a contiguous range of (M tile, N tile)
// pairs with the N tiles of one M tile adjacent, so im2col re-reads hit the XCD's L2.
// ---------------------------------------------------------------------------------------
constexpr int LDK = BK + 4;  // padded k row (floats)


// One k-tile (32 k) of MFMAs.  Two-level fp32 summation: the 16 k-steps of a tile chain into
// a fresh accumulator that is then added to the running total, so a K-long reduction is a
// 32-long chain plus a K/32-long chain instead of one K-long fma chain (K = 2304 for the
// residual conv): ~4x smaller rounding growth for 64 extra VGPRs and 64 v_add per tile.
template <int IM, int JN, int Q0 = 0, int Q1 = 4>
__device__ __forceinline__ void mfma_steps(const float4 (&af)[IM][4], const float4 (&bf)[JN][4],
                                           floatx16 (&t)[IM][JN]) {
#pragma unroll
    for (int q = Q0; q < Q1; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int i = 0; i < IM; ++i)
#pragma unroll
                for (int j = 0; j < JN; ++j) {
                    const float a = e == 0 ? af[i][q].x : e == 1 ? af[i][q].y : e == 2 ? af[i][q].z : af[i][q].w;
                    const float b = e == 0 ? bf[j][q].x : e == 1 ? bf[j][q].y : e == 2 ? bf[j][q].z : bf[j][q].w;
                    if (q == 0 && e == 0) {
                        floatx16 zero = {};
                        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, zero, 0, 0, 0);
                    } else {
                        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, t[i][j], 0, 0, 0);
                    }
                }
}

template <int IM, int JN, int Q0, int Q1>
__device__ __forceinline__ void mfma_chain(const float4 (&af)[IM][4], const float4 (&bf)[JN][4],
                                           floatx16 (&t)[IM][JN]) {
#pragma unroll
    for (int q = Q0; q < Q1; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int i = 0; i < IM; ++i)
#pragma unroll
                for (int j = 0; j < JN; ++j) {
                    const float a = e == 0 ? af[i][q].x : e == 1 ? af[i][q].y : e == 2 ? af[i][q].z : af[i][q].w;
                    const float b = e == 0 ? bf[j][q].x : e == 1 ? bf[j][q].y : e == 2 ? bf[j][q].z : bf[j][q].w;
                    t[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, t[i][j], 0, 0, 0);
                }
}

template <int IM, int JN>
__device__ __forceinline__ void acc_add(floatx16 (&acc)[IM][JN], const floatx16 (&t)[IM][JN]) {
#pragma unroll
    for (int i = 0; i < IM; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j) acc[i][j] += t[i][j];
}

template <int IM, int JN>
__device__ __forceinline__ void mfma_ktile(const float4 (&af)[IM][4], const float4 (&bf)[JN][4],
                                           floatx16 (&acc)[IM][JN]) {
    floatx16 t[IM][JN];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int i = 0; i < IM; ++i)
#pragma unroll
                for (int j = 0; j < JN; ++j) {
                    const float a = e == 0 ? af[i][q].x : e == 1 ? af[i][q].y : e == 2 ? af[i][q].z : af[i][q].w;
                    const float b = e == 0 ? bf[j][q].x : e == 1 ? bf[j][q].y : e == 2 ? bf[j][q].z : bf[j][q].w;
                    if (q == 0 && e == 0) {
                        floatx16 zero = {};
                        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, zero, 0, 0, 0);
                    } else {
                        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, t[i][j], 0, 0, 0);
                    }
                }
#pragma unroll
    for (int i = 0; i < IM; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j) acc[i][j] += t[i][j];
}

// TAG 1: the residual-block geometry (3x3, stride 1, no upsampling, regular rows, 256 source
// channels) is compiled in, so the per-k-tile tap decode and coordinate mapping fold to
// constants; the padding mode (reflect forward, zero for the dgrad) stays a runtime value.
template <int TAG>
__device__ __forceinline__ dcs_conv_desc specialise(dcs_conv_desc d) {
#ifndef DCS_NO_SPECIALISE
    if constexpr (TAG == 1) {  // the residual-block convs: no prologue / epilogue activation
        d.KH = 3; d.KW = 3; d.stride = 1; d.up = 1; d.parity = 0;
        d.Cs = 256; d.csplit = 256; d.s_c = 1;
        d.pro_act = DCS_ACT_NONE; d.epi_act = DCS_ACT_NONE;
    }
    if constexpr (TAG == 2) {  // zero padding, no upsampling in the gather, no prologue / epilogue
        // activation: the runtime activation dispatch (and its tanh) leaves the k-loop, and the gather
        // address is linear in the tap (the reflection / upsampling coordinate maps compile away)
        d.pro_act = DCS_ACT_NONE; d.epi_act = DCS_ACT_NONE;
        d.pad_mode = DCS_PAD_ZERO; d.up = 1;
    }
    if constexpr (TAG == 4) {  // the Generator stem: 7x7 reflect-padded conv over the packed NHWC x 4 image
        d.KH = 7; d.KW = 7; d.Cs = 4; d.csplit = 4; d.s_c = 1; d.stride = 1; d.up = 1; d.parity = 0;
        d.pad_mode = DCS_PAD_REFLECT; d.pro_act = DCS_ACT_NONE; d.epi_act = DCS_ACT_NONE;
    }
    if constexpr (TAG == 3) {  // the PatchGAN layers 1-3: the gather applies IN + LeakyReLU of the
        // previous layer (compile-time activation), zero padding, no upsampling, no epilogue activation
        d.pro_act = DCS_ACT_LRELU; d.epi_act = DCS_ACT_NONE;
        d.pad_mode = DCS_PAD_ZERO; d.up = 1;
    }
#endif
    return d;
}

// InstanceNorm statistics of a rows tile, fused into the epilogue (dcs_conv_rows_in_stats): the
// tile's BM rows lie in one image (the host requires rows-per-image % BM == 0), so each of its
// columns contributes one Part (mean / M2 / max over BM pixels): chunk (z, tile) of image n, where
// z is the sub-pixel phase of a parity-2 forward (one class otherwise).  A lane holds
// 32 rows of one column per 32-column block (IM blocks of 16): two-pass mean / M2 in registers,
// the partner lane (lane ^ 32) merged by shuffle, the BM/64 waves along M through LDS, all in a
// fixed order (deterministic).  The value is the stored one (bias and epilogue activation).
template <int BM, int BN, int IM, int JN>
__device__ __forceinline__ void rows_in_stats(const dcs_conv_desc& d, const floatx16 (&acc)[IM][JN],
                                              const float* __restrict__ bias, int n0, long long m0, const ClassGeom& g,
                                              int z, int wm, int wn, int lane, int tid, float* lds,
                                              Part* __restrict__ parts) {
    constexpr int WN = BN / 2, WMN = BM / 64;
    static_assert(IM == 2, "64-row waves");
    Part* sp = reinterpret_cast<Part*>(lds);  // [WMN][BN]; the k-loop's last barrier freed the LDS
    const int hi = lane >> 5;
    const long long per = (long long)g.My * g.Mx;  // rows of one image (of one phase)
    const int base = (int)(m0 % per);              // the tile's first row within its image
    const int ncls = d.parity == 2 ? 4 : 1;
    auto pixel = [&](int row) {  // output pixel index within the image
        if (d.parity != 2) return base + row;
        const int q = base + row, qy = q / g.Mx, qx = q - (q / g.Mx) * g.Mx;
        return (2 * qy + g.ry) * d.Wo + 2 * qx + g.rx;
    };
#pragma unroll
    for (int j = 0; j < JN; ++j) {
        const int colL = wn * WN + j * 32 + (lane & 31), col = n0 + colL;
        const float bv = (bias && col < d.Co) ? bias[col] : 0.f;
        auto val = [&](int i, int r) {
            float v = acc[i][j][r] + bv;
            if (d.epi_act != DCS_ACT_NONE) v = act_apply(v, d.epi_act);
            return v;
        };
        float s = 0.f, mx = -INFINITY;
        int am = 0;
#pragma unroll
        for (int i = 0; i < IM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {  // rows increase with (i, r): strict > keeps the first maximum
                const float v = val(i, r);
                s += v;
                if (v > mx) { mx = v; am = pixel(wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi); }
            }
        float mean = s * (1.f / 32.f), m2 = 0.f;
#pragma unroll
        for (int i = 0; i < IM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float dv = val(i, r) - mean;
                m2 = fmaf(dv, dv, m2);
            }
        const float mb = __shfl_xor(mean, 32, 64), m2b = __shfl_xor(m2, 32, 64), mxb = __shfl_xor(mx, 32, 64);
        const int amb = __shfl_xor(am, 32, 64);
        if (hi == 0) {  // left operand: this lane; equal counts (32 + 32)
            const float dl = mb - mean;
            Part p;
            p.cnt = 64.f;
            p.mean = mean + 0.5f * dl;
            p.m2 = m2 + m2b + dl * dl * 16.f;
            p.mx = mx;
            p.amax = am;
            if (mxb > mx || (mxb == mx && amb < am)) { p.mx = mxb; p.amax = amb; }
            p.pad[0] = p.pad[1] = p.pad[2] = 0;
            sp[wm * BN + colL] = p;
        }
    }
    __syncthreads();
    if (tid < BN && n0 + tid < d.Co) {
        Part a = sp[tid];
#pragma unroll
        for (int w = 1; w < WMN; ++w) {
            const Part b = sp[w * BN + tid];
            const float tot = a.cnt + b.cnt, dl = b.mean - a.mean;
            a.mean += dl * (b.cnt / tot);
            a.m2 += b.m2 + dl * dl * (a.cnt * b.cnt / tot);
            a.cnt = tot;
            if (b.mx > a.mx || (b.mx == a.mx && b.amax < a.amax)) { a.mx = b.mx; a.amax = b.amax; }
        }
        const long long tiles = per / BM, n = m0 / per;
        parts[((n * ncls + z) * tiles + base / BM) * d.Co + n0 + tid] = a;
    }
}

// VEC: 0 scalar gather (any layout), 1 = 16 consecutive k of one tap per thread (Cs % 16 == 0),
//      2 = four float4 taps per thread over a 4-channel NHWC source (Cs == 4, the stem)
// BM = 256 (bf16x6, 128 columns): 512 threads as 4 x 2 waves of 64 x 64, one workgroup per CU;
// every staged weight k-tile then feeds twice the pixels (0.75 of the 128-row tile's bytes per MFMA)
// bf16x6 rows k-loop body: the fragment reads first, then each MFMA followed by DCS_X6_SGB
// VALU instructions (the next tile's split and address arithmetic), then the LDS stores, so the
// split runs in the shadow of the wave's own MFMAs instead of after them (0 = compiler order)
template <int NMFMA, int NV, int NDSR = 12, int NDSW = 6>
__device__ __forceinline__ void x6_interleave() {
    if constexpr (NV > 0) {
        __builtin_amdgcn_sched_group_barrier(0x100, NDSR, 0);  // DS read
#pragma unroll
        for (int i = 0; i < NMFMA; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);  // VALU
        }
        __builtin_amdgcn_sched_group_barrier(0x200, NDSW, 0);  // DS write
    }
}

template <int BM, int BN, int VEC, int TAG, int MMA = MMA_F32>
__global__ __launch_bounds__(2 * BM, (MMA == MMA_BF16X6 || MMA == MMA_F16X3 || MMA == MMA_F16) ? (BM == 256 ? 2 : DCS_X6_OCC) : 2) void conv_rows_kernel(
    const dcs_conv_desc din, const float* __restrict__ src, const float* __restrict__ src2,
    const float* __restrict__ wp, const float* __restrict__ bias, const float* __restrict__ psc,
    const float* __restrict__ psh, float* __restrict__ out_, int gx, int gy, Part* __restrict__ parts, int fold_) {
    const dcs_conv_desc d = specialise<TAG>(din);
    // fold_ = mode (bits 0-1: 0 none, 1 interior + ring, 2 ring rows only) | K splits << 2 (ring rows:
    // the grid's z index is the split, each split writes its own copy of the ring, summed by the fold)
    const int fold = fold_ & 3;
    const int ksplit = (fold_ >> 2) > 1 ? (fold_ >> 2) : 1;
    static_assert(BM == 128 || (BM == 256 && (MMA == MMA_BF16X6 || MMA == MMA_BF16P || MMA == MMA_F16X3 || MMA == MMA_F16) && BN == 128 && VEC == 1),
                  "A loader: 2 threads per row; 256-row tiles only for the x6 128-column kernel");
    constexpr int NTH = 2 * BM;                    // threads (two per A row)
    constexpr int WM = 64, WN = BN / 2;            // per-wave tile
    constexpr int IM = WM / 32, JN = WN / 32;      // 32x32 blocks per wave
    constexpr int BTPR = NTH / BN;                 // B loader threads per row (2 or 4)
    // bf16: 64-deep k-tiles (twice the MFMA work per round of global loads: the bf16 passes are
    // load-latency bound at 32); f32 and bf16x3 (LDS budget) keep 32
    // f16x3 (H3): two fp16 planes; the vectorised gathers stage two 16-k sub-tiles per barrier
    // (32 k: the MFMAs per barrier of the 16-k bf16x6 tile), the 4-channel stem one
    constexpr bool H3 = MMA == MMA_F16X3 || MMA == MMA_F16;
    constexpr bool F1 = MMA == MMA_F16;  // f16: hi planes only, one product
    constexpr int NSUB = (H3 && VEC == 1 && BN == 128) ? DCS_H3_NSUB : 1;  // 16-k sub-tiles per k-tile (split-at-store modes)
    constexpr int BKT = MMA == MMA_BF16X6 ? DCS_X6_BK : (MMA == MMA_BF16P ? 48 : (H3 ? 16 * NSUB : BK));  // x6: 3 LDS planes, 16-deep tiles keep 2 blocks/CU
    constexpr bool X6L = MMA == MMA_BF16X6 || MMA == MMA_BF16P || H3;  // the x6 LDS planes and pipeline
    constexpr bool X6F = MMA == MMA_BF16X6 || H3;  // operands split at the LDS store (prologue deferred there)
    constexpr int NSLOT = H3 ? 2 * NSUB : 3;       // LDS planes per buffer: [plane][sub] (H3), else 3
    constexpr int AKPT = BKT / 2;                  // k per A-loader thread (2 threads per row)
    constexpr int ACH = AKPT / 4;                  // float4 per A-loader thread
    constexpr int BKPT = BKT / BTPR;               // k per B-loader thread
    constexpr int BCH = BKPT / 4;                  // float4 per B-loader thread
    constexpr int KT2 = 128 / BKT;                 // k-tiles per inner accumulation chain (128 k)
    // bf16 elements per LDS row: planes of BKT k (hi [, mid] [, lo]) + 8 pad; pitches 80 / 144 /
    // 112 B keep the 16-B fragment reads conflict-free
    constexpr int NPL = MMA == MMA_BF16X6 ? 3 : (MMA == MMA_BF16X3 ? 2 : 1);
    constexpr int LDE = NPL * BKT + 8;
    // x6: three planes [plane][buf][BM+BN rows][16 bf16], the 16-B halves of a row swapped on
    // odd groups of 8 rows, so both the 8-lane ds_write_b128 groups and the 16-lane
    // ds_read_b128 groups hit 64 distinct banks (MI355X_MICROARCH.md LDS table)
    constexpr int LDS_FLOATS = MMA == MMA_F32 ? 2 * (BM + BN) * LDK
                             : X6L ? NSLOT * 2 * (BM + BN) * 16 / 2 : (BM + BN) * LDE;

    // f32: As[2][BM][LDK] | Bs[2][BN][LDK];  bf16 modes: Ah[2][BM][LDE] | Bh[2][BN][LDE]
    __shared__ __attribute__((aligned(16))) float lds[LDS_FLOATS];
    auto As = reinterpret_cast<float (*)[BM][LDK]>(lds);
    auto Bs = reinterpret_cast<float (*)[BN][LDK]>(lds + 2 * BM * LDK);
    __bf16* const Ah = reinterpret_cast<__bf16*>(lds);
    __bf16* const Bh = Ah + 2 * BM * LDE;
    // x6 plane offset (bf16 elements) of (plane, buffer, tile row, 8-k half)
    auto x6o = [](int pl, int buf, int row, int h) {
        return ((pl * 2 + buf) * (BM + BN) + row) * 16 + 8 * (h ^ ((row >> 3) & 1));
    };
    __shared__ long long rowoff[BM];
    // bf16x6 prologue (TAG 0): the per-(image, channel) scale / shift of the <= 2 images a tile
    // spans, staged once, so the affine at the LDS store reads LDS instead of issuing global
    // loads that would wait behind the prefetched gathers
    constexpr bool PRO_LDS = X6F && (TAG == 0 || TAG == 3);
    // TAG 4 (stem): the reflected source row / column offsets of each A row's 7 kernel rows and 7
    // kernel columns, computed once per workgroup (14 coordinate maps per row instead of 2 per tap
    // per k-tile); a tap's gather offset is one row entry + one column entry
    constexpr bool STEMT = TAG == 4 && VEC == 2;
    __shared__ int stab[STEMT ? 2 * BM * 7 : 1];
    constexpr int PRO_CMAX = 512;
    __shared__ __attribute__((aligned(16))) float prol[PRO_LDS ? 4 * PRO_CMAX : 4];

    const int T = gridDim.x;
    const int L = xcd_remap(blockIdx.x, T);
    const int ntile = L % gy;
    const int rest = L / gy;
    const int mtile = rest % gx;
    const int z = ksplit > 1 ? 0 : rest / gx;
    const int ks = ksplit > 1 ? rest / gx : 0;
    const ClassGeom g = class_geom(d, z);
    const long long M = fold == 2 ? (long long)d.N * (2 * d.Wo + 2 * (d.Ho - 2)) : (long long)g.My * g.Mx * d.N;
    float* __restrict__ const out = out_ + (long long)ks * M * d.Co;
    const long long m0 = (long long)mtile * BM;
    if (m0 >= M) return;
    const int n0 = ntile * BN;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;

    // A loader: one row, 16 consecutive k (VEC: Cs % 16 == 0, so the 16 k share one tap); BF16P:
    // 8 k of each of the tile's three 16-k sub-tiles
    const int arow = tid >> 1, akq = (tid & 1) * ((MMA == MMA_BF16P || NSUB > 1) ? 8 : AKPT);
    const RowInfo ri = row_info(d, g, (int)(m0 + arow), fold);
    const bool rvalid = ri.out_off >= 0;
    if ((tid & 1) == 0) rowoff[arow] = ri.out_off;
    if constexpr (STEMT) {  // thread pair of a row: even lane the 7 row offsets, odd lane the 7 column offsets
        const int Hv0 = d.Hs * d.up, Wv0 = d.Ws * d.up;
#pragma unroll
        for (int t7 = 0; t7 < 7; ++t7) {
            int c;
            if ((tid & 1) == 0) {
                map_coord(ri.by + t7, Hv0, d.up, d.pad_mode, c);
                stab[arow * 7 + t7] = c * (int)d.s_h;
            } else {
                map_coord(ri.bx + t7, Wv0, d.up, d.pad_mode, c);
                stab[BM * 7 + arow * 7 + t7] = c * (int)d.s_w;
            }
        }
        __syncthreads();
    }
    // B loader: one output channel row, BKPT consecutive k
    const int brow = tid / BTPR, bkq = (tid % BTPR) * ((MMA == MMA_BF16P || NSUB > 1) ? 16 / BTPR : BKPT);
    const float* bsrc = wp + (long long)(n0 + brow) * d.ldb;

    // taps this tile needs (ring rows of a padded-grid data gradient, TAG 1 fold 2: a segment of the ring
    // reads one kernel row or column; every other launch: all taps)
    int tapmask = (1 << g.ntaps) - 1, ntap_act = g.ntaps;
    if constexpr (TAG == 1 && H3) {
        if (fold == 2) {
            const int Hr = d.Ho - 2, sw = d.N * d.Wo, sh = d.N * Hr;
            auto seg_mask = [&](long long m) {  // (ty, tx) bit ty * 3 + tx of the taps segment m's rows read
                return m < sw ? 0x1C0 : (m < 2 * sw ? 0x007 : (m < 2 * sw + sh ? 0x124 : 0x049));
            };
            const long long mlast = (m0 + BM < M ? m0 + BM : M) - 1;
            int msk = 0;
            for (int sgi = 0; sgi < 4; ++sgi) {  // the segments between the tile's first and last row
                const long long sb = sgi == 0 ? 0 : (sgi == 1 ? sw : (sgi == 2 ? 2 * sw : 2 * sw + sh));
                const long long se = sgi == 0 ? sw : (sgi == 1 ? 2 * sw : (sgi == 2 ? 2 * sw + sh : 2 * sw + 2 * sh));
                if (sb <= mlast && se > m0) msk |= seg_mask(sb);
            }
            tapmask = __builtin_amdgcn_readfirstlane(msk);
            ntap_act = __builtin_popcount(tapmask);
        }
    }
    const int K = ntap_act * d.Cs;
    const int nkt_all = (K + BKT - 1) / BKT;
    const int kper = (nkt_all + ksplit - 1) / ksplit;
    const int kt_beg = ks * kper;                                         // this split's k-tiles
    const int nkt = kt_beg + kper < nkt_all ? kt_beg + kper : nkt_all;  // (exclusive end)
    const int kb0 = kt_beg * BKT;
    const int Hv = d.Hs * d.up, Wv = d.Ws * d.up;
    const float* srow = src + ri.n * d.s_n;
    const long long so = (long long)ri.n * d.Cs;
    const __amdgpu_buffer_rsrc_t arsrc = src_rsrc(src);
    // f16x3 operand scales 2^ea, 2^eb and the exponent that undoes them in the epilogue
    float asc = 1.f, bsc = 1.f;
    int eab = 0;
    if constexpr (H3) {
        const int ea = f16x3_exp(d.rng_a, d.rng_a_n), eb = f16x3_exp(d.rng_b, d.rng_b_n);
        asc = __builtin_ldexpf(1.f, ea);
        bsc = __builtin_ldexpf(1.f, eb);
        eab = -(ea + eb);
    }
    bool pro_lds = false;  // block-uniform
    int pro_base = 0;      // n_lo * Cs: psc/psh index of prol[0]
    if constexpr (PRO_LDS) {
        if (d.pro_act != DCS_ACT_NONE && d.Cs <= PRO_CMAX && d.parity != 2) {
            const long long per = (long long)g.My * g.Mx;
            const int n_lo = (int)(m0 / per);
            const int n_hi = (int)(((m0 + BM < M ? m0 + BM : M) - 1) / per);
            if (n_hi - n_lo <= 1) {
                pro_lds = true;
                pro_base = n_lo * d.Cs;
                for (int i = tid; i < 2 * d.Cs; i += NTH) {
                    const bool ok = n_lo + i / d.Cs < d.N;
                    prol[i] = ok ? psc[pro_base + i] : 0.f;
                    prol[2 * PRO_CMAX + i] = ok ? psh[pro_base + i] : 0.f;
                }
            }
        }
        __syncthreads();
    }

    // incremental (tap, channel) state of the next k-tile to load, for A and B.  TAG 1 (the
    // residual convs) runs the DCS_KORDER_SLICE K order: all taps of a 16-channel slice, then
    // the next slice, so the source rows a slice gathers are re-read by its next taps from
    // L1/L2 instead of after a sweep over all channels (the dispatch requires d.korder == SLICE)
    // TAG 0 bf16x6 kernels with 16-channel-aligned sources walk the same slice-major order over
    // tap-major packed weights (KSB: the B column is rebuilt from (tap, channel) per k-tile)
    constexpr bool KSB = TAG != 1 && X6F && VEC == 1 && DCS_KSLICE_ALL;
    constexpr bool KS = TAG == 1 || KSB;
    int aj, ac;
    if constexpr (KS) {
        const int p0 = (kb0 + akq) >> 4;
        aj = p0 % g.ntaps;
        ac = (p0 / g.ntaps) * 16 + (akq & 15);
    } else {
        aj = (kb0 + akq) / d.Cs;
        ac = (kb0 + akq) - ((kb0 + akq) / d.Cs) * d.Cs;
    }
    int bj, bc;
    if constexpr (KSB) {
        const int p0 = (kb0 + bkq) >> 4;
        bj = p0 % g.ntaps;
        bc = (p0 / g.ntaps) * 16 + (bkq & 15);
    } else {
        bj = (kb0 + bkq) / d.Cs;
        bc = (kb0 + bkq) - ((kb0 + bkq) / d.Cs) * d.Cs;
    }
    auto advance = [&](int& j, int& c) {
        if constexpr (KS) {
            j += BKT / 16;
            while (j >= g.ntaps) { j -= g.ntaps; c += 16; }
        } else {
            c += BKT;
            while (c >= d.Cs) { c -= d.Cs; ++j; }
        }
    };
    // Uniform tap walk of the slice-major order (KS): every thread of the workgroup walks the same
    // (tap, 16-channel slice) sequence, only the channel within the slice (akq / bkq & 15) differs
    // per lane.  The walk state lives in SGPRs (readfirstlane at init, scalar selects per step) and
    // the tap's kernel position is tracked as (ty, tx) instead of decoded from j per sub-tile: the
    // per-lane decode (an integer division by KW for A and again for B) was ~20 % of the VALU
    // instructions of the non-residual rows kernels, which are VALU bound.
    int wntx, wnty, wty0 = 0, wtx0 = 0;  // taps of this class along x / y; parity-1 first taps
    if (!d.parity) {
        wntx = d.KW; wnty = d.KH;
    } else if (d.parity == 2) {
        wntx = 2; wnty = 2;
    } else {
        wty0 = (g.ry + d.pt) & 1; wtx0 = (g.rx + d.pl) & 1;
        wntx = (d.KW - wtx0 + 1) >> 1; wnty = (d.KH - wty0 + 1) >> 1;
    }
    struct Walk {
        int ty, tx, cs;  // tap position within the class, first channel of the slice
    };
    auto walk_init = [&](int p0) {  // p0: index of the first 16-k step (uniform)
        Walk w;
        int j = p0 % ntap_act;
        if constexpr (TAG == 1 && H3) {  // the j-th tap of the mask
            int t = 0;
            for (int q = 0; q < g.ntaps; ++q)
                if ((tapmask >> q) & 1) {
                    if (j == 0) { t = q; break; }
                    --j;
                }
            j = t;
        }
        w.cs = __builtin_amdgcn_readfirstlane((p0 / ntap_act) * 16);
        w.ty = __builtin_amdgcn_readfirstlane(j / wntx);
        w.tx = __builtin_amdgcn_readfirstlane(j - (j / wntx) * wntx);
        return w;
    };
    auto walk_step1 = [&](Walk& w) {
        const bool wx = w.tx + 1 == wntx;
        const bool wy = wx && w.ty + 1 == wnty;
        w.tx = wx ? 0 : w.tx + 1;
        w.ty = wy ? 0 : (wx ? w.ty + 1 : w.ty);
        w.cs += wy ? 16 : 0;
    };
    auto walk_step = [&](Walk& w) {
        walk_step1(w);
        if constexpr (TAG == 1 && H3) {  // skip the taps outside the mask (uniform; a no-op for a full mask)
            while (!((tapmask >> (w.ty * wntx + w.tx)) & 1)) walk_step1(w);
        }
    };
    // (ady, adx): source offset of the tap; bt: its column block in the packed weights (tap_decode).
    // All three are affine in (ty, tx) with per-class constants (parity 1: ady = (ry + pt - ty0) / 2
    // - ty, the numerator being even), so the walk needs no per-step case analysis.
    int woy, wsy, wox, wsx, wb0, wbty, wbtx;
    if (!d.parity) {
        woy = 0; wsy = 1; wox = 0; wsx = 1; wb0 = 0; wbty = d.KW; wbtx = 1;
    } else if (d.parity == 2) {
        woy = g.ry - 1; wsy = 1; wox = g.rx - 1; wsx = 1; wb0 = (2 * g.ry + g.rx) * 4; wbty = 2; wbtx = 1;
    } else {
        woy = (g.ry + d.pt - wty0) >> 1; wsy = -1; wox = (g.rx + d.pl - wtx0) >> 1; wsx = -1;
        wb0 = wty0 * d.KW + wtx0; wbty = 2 * d.KW; wbtx = 2;
    }
    auto walk_tap = [&](const Walk& w, int& ady, int& adx, int& bt) {
        ady = woy + wsy * w.ty;
        adx = wox + wsx * w.tx;
        bt = wb0 + wbty * w.ty + wbtx * w.tx;
    };
    constexpr bool UWALK = KS && DCS_UWALK;
    Walk wa = walk_init(kb0 >> 4), wb = wa;
    const int alo = akq & 15, blo = bkq & 15;
    // linear gather (zero padding, no upsampling): the lane's element offset of tap (0, 0) at channel
    // alo of the slice; a tap adds ady * s_h + adx * s_w + slice base (uniform)
    const bool lin = d.pad_mode == DCS_PAD_ZERO && d.up == 1;
    const int abase = ri.n * (int)d.s_n + ri.by * (int)d.s_h + ri.bx * (int)d.s_w + alo;
    // one 16-k sub-tile step (NSUB > 1); equal to advance for 16-k tiles
    auto advance16 = [&](int& j, int& c) {
        if constexpr (KS) {
            j += 1;
            if (j >= g.ntaps) { j -= g.ntaps; c += 16; }
        } else {
            c += 16;
            while (c >= d.Cs) { c -= d.Cs; ++j; }
        }
    };

    float4 ra[ACH];
    float4 rb[BCH];

    // pa: bf16x6 defers the prologue affine to the LDS store (a load consumed at once would make
    // the next tile's gather wait); it records the channel offset into psc/psh, -1 for none
    auto load_a = [&](int kt, auto& dst, int (&pa)[NSUB]) {
#pragma unroll
        for (int q = 0; q < NSUB; ++q) pa[q] = -1;
        if (STEMT) {  // the stem: 49 taps, reflected offsets from the per-row table, branch-free
#pragma unroll
            for (int e = 0; e < ACH; ++e) {
                const int j = aj + e;
                const int ty = j / 7, tx = j - (j / 7) * 7;
                const bool ok = rvalid && j < 49;
                const int o = ok ? (ri.n * (int)d.s_n + stab[arow * 7 + ty] + stab[BM * 7 + arow * 7 + tx]) * 4 : OOB_OFF;
                dst[e] = buf_load4(arsrc, ok ? o : OOB_OFF);
            }
            aj += BKT / 4;
        } else if (VEC == 2) {  // Cs == 4: taps aj .. aj+ACH-1, one float4 each (no prologue)
#pragma unroll
            for (int e = 0; e < ACH; ++e) dst[e] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (rvalid) {
#pragma unroll
                for (int e = 0; e < ACH; ++e) {
                    const int j = aj + e;
                    if (j < g.ntaps) {
                        int ady, adx, bt;
                        tap_decode(d, g, j, ady, adx, bt);
                        int sy, sx;
                        if (map_coord(ri.by + ady, Hv, d.up, d.pad_mode, sy) &&
                            map_coord(ri.bx + adx, Wv, d.up, d.pad_mode, sx))
                            dst[e] = *reinterpret_cast<const float4*>(srow + sy * d.s_h + sx * d.s_w);
                    }
                }
            }
            aj += BKT / 4;
        } else if (MMA == MMA_BF16P) {
            // three 16-k sub-tiles (slice-major: the next tap of the slice each), 8 k per thread
#pragma unroll
            for (int sub = 0; sub < 3; ++sub) {
                const bool kin = aj < g.ntaps && ac < d.Cs;
                int ady, adx, bt, sy = 0, sx = 0;
                tap_decode(d, g, kin ? aj : 0, ady, adx, bt);
                const bool yok = map_coord_sel(ri.by + ady, Hv, d.up, d.pad_mode, sy);
                const bool xok = map_coord_sel(ri.bx + adx, Wv, d.up, d.pad_mode, sx);
                const int off = (kin && rvalid && yok && xok)
                                    ? (ri.n * (int)d.s_n + sy * (int)d.s_h + sx * (int)d.s_w + ac) * 4
                                    : OOB_OFF;
                dst[2 * sub] = buf_load4(arsrc, off);
                dst[2 * sub + 1] = buf_load4(arsrc, off + 16);
                const bool wrap = aj + 1 >= g.ntaps;
                aj = wrap ? 0 : aj + 1;
                ac += wrap ? 16 : 0;
            }
        } else if (VEC && NSUB > 1) {
            // f16x3: NSUB 16-k sub-tiles (the next tap of the slice, or the next 16 channels), 8 k
            // per thread each, by the branch-free select gather of the bf16x6 tiles below
#pragma unroll
            for (int sub = 0; sub < NSUB; ++sub) {
                int ady, adx, bt, sy = 0, sx = 0, c;
                bool kin;
                if constexpr (UWALK) {
                    kin = wa.cs < d.Cs;
                    walk_tap(wa, ady, adx, bt);
                    c = wa.cs + alo;
                } else {
                    kin = aj < g.ntaps && ac < d.Cs;
                    tap_decode(d, g, kin ? aj : 0, ady, adx, bt);
                    c = ac;
                }
                int off;
                if (UWALK && lin) {  // zero padding, no upsampling: lane base + uniform tap offset
                    const int vy = ri.by + ady, vx = ri.bx + adx;
                    const bool ok = kin && rvalid && (unsigned)vy < (unsigned)Hv && (unsigned)vx < (unsigned)Wv;
                    off = ok ? (abase + ady * (int)d.s_h + adx * (int)d.s_w + wa.cs) * 4 : OOB_OFF;
                } else {
                    const bool yok = map_coord_sel(ri.by + ady, Hv, d.up, d.pad_mode, sy);
                    const bool xok = map_coord_sel(ri.bx + adx, Wv, d.up, d.pad_mode, sx);
                    off = (kin && rvalid && yok && xok) ? (ri.n * (int)d.s_n + sy * (int)d.s_h + sx * (int)d.s_w + c) * 4
                                                        : OOB_OFF;
                }
                dst[2 * sub] = buf_load4(arsrc, off);
                dst[2 * sub + 1] = buf_load4(arsrc, off + 16);
                if (d.pro_act != DCS_ACT_NONE && off != OOB_OFF) pa[sub] = (int)so + c;
                if constexpr (UWALK) walk_step(wa);
                else advance16(aj, ac);
            }
        } else if (VEC && MMA != MMA_F32 && DCS_BF16_BUFGATHER) {
            // bf16 modes: branch-free gather through a buffer descriptor (OOB -> zeros)
            int sy = 0, sx = 0, off = OOB_OFF;
            // past the last k-tile (the x6 pipeline's unconditional prefetch) the walk leaves the
            // range through aj (tap-major) or through ac (slice-major): both must stay in range
            int c = ac;
            if constexpr (UWALK && X6F && DCS_X6_SELGATHER && BKT == 16) {
                const bool kin = wa.cs < d.Cs;
                int ady, adx, bt;
                walk_tap(wa, ady, adx, bt);
                c = wa.cs + alo;
                if (lin) {
                    const int vy = ri.by + ady, vx = ri.bx + adx;
                    const bool ok = kin && rvalid && (unsigned)vy < (unsigned)Hv && (unsigned)vx < (unsigned)Wv;
                    off = ok ? (abase + ady * (int)d.s_h + adx * (int)d.s_w + wa.cs) * 4 : OOB_OFF;
                } else {
                    const bool yok = map_coord_sel(ri.by + ady, Hv, d.up, d.pad_mode, sy);
                    const bool xok = map_coord_sel(ri.bx + adx, Wv, d.up, d.pad_mode, sx);
                    off = (kin && rvalid && yok && xok) ? (ri.n * (int)d.s_n + sy * (int)d.s_h + sx * (int)d.s_w + c) * 4
                                                        : OOB_OFF;
                }
            } else if constexpr (X6F && DCS_X6_SELGATHER) {
                // select form (tap 0 stands in for a tap past the end): no exec-mask branch
                // splits the k-loop body, so the scheduler can spread the next tile's split
                // arithmetic over this tile's MFMAs
                const bool kin = aj < g.ntaps && ac < d.Cs;
                int ady, adx, bt;
                tap_decode(d, g, kin ? aj : 0, ady, adx, bt);
                const bool yok = map_coord_sel(ri.by + ady, Hv, d.up, d.pad_mode, sy);
                const bool xok = map_coord_sel(ri.bx + adx, Wv, d.up, d.pad_mode, sx);
                off = (kin && rvalid && yok && xok) ? (ri.n * (int)d.s_n + sy * (int)d.s_h + sx * (int)d.s_w + ac) * 4
                                                    : OOB_OFF;
            } else if (aj < g.ntaps && ac < d.Cs) {
                int ady, adx, bt;
                tap_decode(d, g, aj, ady, adx, bt);
                const bool yok = map_coord_sel(ri.by + ady, Hv, d.up, d.pad_mode, sy);
                const bool xok = map_coord_sel(ri.bx + adx, Wv, d.up, d.pad_mode, sx);
                if (rvalid && yok && xok) off = (ri.n * (int)d.s_n + sy * (int)d.s_h + sx * (int)d.s_w + ac) * 4;
            }
#pragma unroll
            for (int i = 0; i < ACH; ++i) dst[i] = buf_load4(arsrc, off + 16 * i);
            if constexpr (X6F) {
                if (d.pro_act != DCS_ACT_NONE && off != OOB_OFF) pa[0] = (int)so + c;
            } else if (d.pro_act != DCS_ACT_NONE && off != OOB_OFF) {
#pragma unroll
                for (int i = 0; i < ACH; ++i) dst[i] = affine_act4(dst[i], psc + so + ac + 4 * i, psh + so + ac + 4 * i, d.pro_act);
            }
            if constexpr (UWALK && X6F && DCS_X6_SELGATHER && BKT == 16) {
                walk_step(wa);
            } else {
                advance(aj, ac);
            }
        } else if (VEC) {
            // (a buffer-descriptor variant of this gather, as in the wgrad pass, measured 3-7 %
            //  slower here: invalid taps would issue loads that the branch now skips)
#pragma unroll
            for (int i = 0; i < ACH; ++i) dst[i] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (rvalid && aj < g.ntaps && ac < d.Cs) {
                int ady, adx, bt;
                tap_decode(d, g, aj, ady, adx, bt);
                int sy, sx;
                if (map_coord(ri.by + ady, Hv, d.up, d.pad_mode, sy) &&
                    map_coord(ri.bx + adx, Wv, d.up, d.pad_mode, sx)) {
                    const float* sp = srow + sy * d.s_h + sx * d.s_w + ac;
#pragma unroll
                    for (int i = 0; i < ACH; ++i) dst[i] = *reinterpret_cast<const float4*>(sp + 4 * i);
                    if (d.pro_act != DCS_ACT_NONE) {
#pragma unroll
                        for (int i = 0; i < ACH; ++i) dst[i] = affine_act4(dst[i], psc + so + ac + 4 * i, psh + so + ac + 4 * i, d.pro_act);
                    }
                }
            }
            advance(aj, ac);
        } else {
#pragma unroll
            for (int i = 0; i < ACH; ++i) {
                float e[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    int k = kt * BKT + akq + 4 * i + q;
                    int j = k / d.Cs, c = k - j * d.Cs;
                    e[q] = 0.f;
                    if (rvalid && j < g.ntaps) {
                        int ady, adx, bt;
                        tap_decode(d, g, j, ady, adx, bt);
                        e[q] = gather1(d, src, src2, psc, psh, ri.n, ri.by + ady, ri.bx + adx, c);
                    }
                }
                dst[i] = make_float4(e[0], e[1], e[2], e[3]);
            }
        }
    };
    const __amdgpu_buffer_rsrc_t brsrc = src_rsrc(wp);
    // f16x3 / f16 with pre-split weights (d.b_h3, dcs_pack_split_h3): B is staged without a split,
    // rows [r][hi | lo][ldb] halves; the fp32 pack (wp) is then not read
    const bool bpre = H3 && d.b_h3 != nullptr;
    const __amdgpu_buffer_rsrc_t b3rsrc = src_rsrc(reinterpret_cast<const float*>(d.b_h3));
    auto load_b = [&](int kt, auto& dst) {
        if constexpr (MMA == MMA_BF16P) {  // slice-major packed B: the tile's 48 k are consecutive
            constexpr int BQ = BCH / 3;      // float4 per sub-tile: 2 (256 threads) or 1 (512)
#pragma unroll
            for (int sub = 0; sub < 3; ++sub) {
                const long long col = (long long)kt * BKT + 16 * sub + bkq;
                const int off = col < d.ldb ? (int)(((long long)(n0 + brow) * d.ldb + col) * 4) : OOB_OFF;
#pragma unroll
                for (int q = 0; q < BQ; ++q) dst[BQ * sub + q] = buf_load4(brsrc, off + 16 * q);
            }
            return;
        }
        if constexpr (NSUB > 1) {  // f16x3 sub-tiles: BKPT / NSUB k of each 16-k sub-tile
            constexpr int BQ = BCH / NSUB;
#pragma unroll
            for (int sub = 0; sub < NSUB; ++sub) {
                long long col;
                bool ok = true;
                if constexpr (TAG == 1 && H3 && DCS_UWALK) {  // the (masked) slice-major walk: 9 taps x 16 per slice
                    ok = wb.cs < d.Cs;
                    col = (long long)(wb.cs >> 4) * (9 * 16) + (wb.ty * 3 + wb.tx) * 16 + blo;
                    walk_step(wb);
                } else if (!d.parity && !KSB) {
                    col = (long long)kt * BKT + 16 * sub + bkq;
                } else if constexpr (KSB && DCS_UWALK) {
                    ok = wb.cs < d.Cs;
                    int ady, adx, bt;
                    walk_tap(wb, ady, adx, bt);
                    col = bt * d.Cs + wb.cs + blo;
                    walk_step(wb);
                } else {
                    ok = bj < g.ntaps && bc < d.Cs;
                    int ady, adx, bt = 0;
                    if (ok) tap_decode(d, g, bj, ady, adx, bt);
                    col = (long long)bt * d.Cs + bc;
                    advance16(bj, bc);
                }
                if (bpre) {  // 8 k: hi (16 B) into dst[2 sub], lo into dst[2 sub + 1]; 4 k: hi in .xy, lo in .zw
                    const int oh = (ok && col < d.ldb) ? (int)(((long long)(n0 + brow) * 2 * d.ldb + col) * 2) : OOB_OFF;
                    const int ol = oh == OOB_OFF ? OOB_OFF : oh + 2 * d.ldb;
                    if constexpr (BQ == 2) {
                        dst[BQ * sub] = buf_load4(b3rsrc, oh);
                        // (f16: the lo slot zero, not left unwritten -- a partly written array was kept in
                        // scratch memory)
                        dst[BQ * sub + 1] = F1 ? make_float4(0.f, 0.f, 0.f, 0.f) : buf_load4(b3rsrc, ol);
                    } else {
                        const float2 h = buf_load2(b3rsrc, oh);
                        float2 l = make_float2(0.f, 0.f);
                        if constexpr (!F1) l = buf_load2(b3rsrc, ol);
                        dst[BQ * sub] = make_float4(h.x, h.y, l.x, l.y);
                    }
                } else {
                    const int off = (ok && col < d.ldb) ? (int)(((long long)(n0 + brow) * d.ldb + col) * 4) : OOB_OFF;
#pragma unroll
                    for (int q = 0; q < BQ; ++q) dst[BQ * sub + q] = buf_load4(brsrc, off + 16 * q);
                }
            }
            return;
        }
        long long col;
        bool ok = true;
        if (!d.parity && !KSB) {
            col = kt * BKT + bkq;
        } else if constexpr (KSB && DCS_UWALK && X6F && DCS_BF16_BUFGATHER && BKT == 16) {
            ok = wb.cs < d.Cs;
            int ady, adx, bt;
            walk_tap(wb, ady, adx, bt);
            col = bt * d.Cs + wb.cs + blo;
            walk_step(wb);
        } else {  // the BKPT k of this thread share one tap (Cs % 16 == 0)
            ok = bj < g.ntaps && bc < d.Cs;
            int ady, adx, bt = 0;
            if (ok) tap_decode(d, g, bj, ady, adx, bt);
            col = (long long)bt * d.Cs + bc;
            advance(bj, bc);
        }
        if (H3 && BCH == 1 && bpre) {  // 4 k: hi (8 B) in .xy, lo in .zw
            const int oh = (ok && col < d.ldb) ? (int)(((long long)(n0 + brow) * 2 * d.ldb + col) * 2) : OOB_OFF;
            const float2 h = buf_load2(b3rsrc, oh);
            float2 l = make_float2(0.f, 0.f);
            if constexpr (!F1) l = buf_load2(b3rsrc, oh == OOB_OFF ? OOB_OFF : oh + 2 * d.ldb);
            dst[0] = make_float4(h.x, h.y, l.x, l.y);
            return;
        }
        if constexpr (X6F && DCS_BF16_BUFGATHER) {  // branch-free: k-tiles past the end read zeros
            const int off = (ok && col < d.ldb) ? (int)(((long long)(n0 + brow) * d.ldb + col) * 4) : OOB_OFF;
#pragma unroll
            for (int i = 0; i < BCH; ++i) dst[i] = buf_load4(brsrc, off + 16 * i);
        } else {
#pragma unroll
            for (int i = 0; i < BCH; ++i)
                dst[i] = (ok && col < d.ldb) ? *reinterpret_cast<const float4*>(bsrc + col + 4 * i)
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto store_tiles = [&](int buf, const auto& sa0, const auto& sb, const int (&pa)[NSUB]) {
        float4 sa[ACH];
#pragma unroll
        for (int i = 0; i < ACH; ++i) sa[i] = sa0[i];
        if constexpr (X6F) {
            constexpr int AQ = ACH / NSUB;  // float4 of one sub-tile
#pragma unroll
            for (int sub = 0; sub < NSUB; ++sub) {
                const int pq = pa[sub];
                if (d.pro_act != DCS_ACT_NONE && pq >= 0) {
                    if (pro_lds) {
                        const int q = pq - pro_base;
#pragma unroll
                        for (int i = 0; i < AQ; ++i)
                            sa[AQ * sub + i] = affine_act4(sa[AQ * sub + i], prol + q + 4 * i, prol + 2 * PRO_CMAX + q + 4 * i, d.pro_act);
                    } else {
#pragma unroll
                        for (int i = 0; i < AQ; ++i)
                            sa[AQ * sub + i] = affine_act4(sa[AQ * sub + i], psc + pq + 4 * i, psh + pq + 4 * i, d.pro_act);
                    }
                }
            }
        }
        if constexpr (MMA == MMA_F32) {
#pragma unroll
            for (int i = 0; i < ACH; ++i) *reinterpret_cast<float4*>(&As[buf][arow][akq + 4 * i]) = sa[i];
#pragma unroll
            for (int i = 0; i < BCH; ++i) *reinterpret_cast<float4*>(&Bs[buf][brow][bkq + 4 * i]) = sb[i];
        } else if constexpr (MMA == MMA_BF16P) {
            static_assert(BKT == 48 && ACH == 6 && (BCH == 6 || BCH == 3) && BN == 128,
                          "bf16p tiles: 3 x 16 k, 8 A and 8 / 4 B per thread each");
#pragma unroll
            for (int sub = 0; sub < 3; ++sub) {
                const floatx8 fa = {sa[2 * sub].x, sa[2 * sub].y, sa[2 * sub].z, sa[2 * sub].w,
                                    sa[2 * sub + 1].x, sa[2 * sub + 1].y, sa[2 * sub + 1].z, sa[2 * sub + 1].w};
                *reinterpret_cast<bf16x8*>(Ah + x6o(sub, buf, arow, akq >> 3)) = __builtin_convertvector(fa, bf16x8);
                if constexpr (BCH == 6) {
                    const floatx8 fb = {sb[2 * sub].x, sb[2 * sub].y, sb[2 * sub].z, sb[2 * sub].w,
                                        sb[2 * sub + 1].x, sb[2 * sub + 1].y, sb[2 * sub + 1].z, sb[2 * sub + 1].w};
                    *reinterpret_cast<bf16x8*>(Ah + x6o(sub, buf, BM + brow, bkq >> 3)) = __builtin_convertvector(fb, bf16x8);
                } else {  // 512 threads: 4 k of B per thread, the 8-byte half of a 16-byte chunk
                    const float4 v = sb[sub];
                    const f32x4v f4 = {v.x, v.y, v.z, v.w};
                    *reinterpret_cast<bf16x4*>(Ah + x6o(sub, buf, BM + brow, bkq >> 3) + 4 * ((bkq >> 2) & 1)) =
                        __builtin_convertvector(f4, bf16x4);
                }
            }
        } else if constexpr (H3) {
            // planes [hi | lo] x sub-tiles: slot = plane * NSUB + sub
            static_assert(ACH == 2 * NSUB && (BCH == 2 * NSUB || BCH == NSUB), "f16x3 tiles: 8 A and 8 / 4 B per thread per sub-tile");
#pragma unroll
            for (int sub = 0; sub < NSUB; ++sub) {
                f16x8 hi, lo;
                split8h(sa[2 * sub], sa[2 * sub + 1], asc, hi, lo);
                *reinterpret_cast<f16x8*>(Ah + x6o(sub, buf, arow, akq >> 3)) = hi;
                if constexpr (!F1) *reinterpret_cast<f16x8*>(Ah + x6o(NSUB + sub, buf, arow, akq >> 3)) = lo;
                if constexpr (BCH == 2 * NSUB) {
                    if (bpre) {
                        hi = __builtin_bit_cast(f16x8, sb[2 * sub]);
                        lo = __builtin_bit_cast(f16x8, sb[2 * sub + 1]);
                    } else {
                        split8h(sb[2 * sub], sb[2 * sub + 1], bsc, hi, lo);
                    }
                    *reinterpret_cast<f16x8*>(Ah + x6o(sub, buf, BM + brow, bkq >> 3)) = hi;
                    if constexpr (!F1) *reinterpret_cast<f16x8*>(Ah + x6o(NSUB + sub, buf, BM + brow, bkq >> 3)) = lo;
                } else {  // 4 k of B per thread: the 8-byte half of a 16-byte chunk
                    f16x4 h4, l4;
                    if (bpre) {
                        h4 = __builtin_bit_cast(f16x4, make_float2(sb[sub].x, sb[sub].y));
                        l4 = __builtin_bit_cast(f16x4, make_float2(sb[sub].z, sb[sub].w));
                    } else {
                        split4h(sb[sub], bsc, h4, l4);
                    }
                    const int q = 4 * ((bkq >> 2) & 1);
                    *reinterpret_cast<f16x4*>(Ah + x6o(sub, buf, BM + brow, bkq >> 3) + q) = h4;
                    if constexpr (!F1) *reinterpret_cast<f16x4*>(Ah + x6o(NSUB + sub, buf, BM + brow, bkq >> 3) + q) = l4;
                }
            }
        } else if constexpr (MMA == MMA_BF16X6) {
            static_assert(BKT == 16 && ACH == 2 && (BCH == 2 || BCH == 1), "x6 tiles: 16 k, 8 / 4 per loader thread");
            bf16x8 hi, mid, lo;
            split8x3(sa[0], sa[1], hi, mid, lo);
            *reinterpret_cast<bf16x8*>(Ah + x6o(0, buf, arow, akq >> 3)) = hi;
            *reinterpret_cast<bf16x8*>(Ah + x6o(1, buf, arow, akq >> 3)) = mid;
            *reinterpret_cast<bf16x8*>(Ah + x6o(2, buf, arow, akq >> 3)) = lo;
            if constexpr (BCH == 2) {
                split8x3(sb[0], sb[1], hi, mid, lo);
                *reinterpret_cast<bf16x8*>(Ah + x6o(0, buf, BM + brow, bkq >> 3)) = hi;
                *reinterpret_cast<bf16x8*>(Ah + x6o(1, buf, BM + brow, bkq >> 3)) = mid;
                *reinterpret_cast<bf16x8*>(Ah + x6o(2, buf, BM + brow, bkq >> 3)) = lo;
            } else {  // 64-column tiles: 4 k per thread, the 8-byte half of a 16-byte chunk
                bf16x4 h4, m4, l4;
                split4x3(sb[0], h4, m4, l4);
                const int sub = 4 * ((bkq >> 2) & 1);
                *reinterpret_cast<bf16x4*>(Ah + x6o(0, buf, BM + brow, bkq >> 3) + sub) = h4;
                *reinterpret_cast<bf16x4*>(Ah + x6o(1, buf, BM + brow, bkq >> 3) + sub) = m4;
                *reinterpret_cast<bf16x4*>(Ah + x6o(2, buf, BM + brow, bkq >> 3) + sub) = l4;
            }
        } else {
            bf16x8 hi, lo;
            __bf16* a = Ah + (buf * BM + arow) * LDE;
#pragma unroll
            for (int i = 0; i < ACH / 2; ++i) {
                split8<MMA>(sa[2 * i], sa[2 * i + 1], hi, lo);
                *reinterpret_cast<bf16x8*>(a + akq + 8 * i) = hi;
                if constexpr (MMA == MMA_BF16X3) *reinterpret_cast<bf16x8*>(a + 32 + akq + 8 * i) = lo;
            }
            __bf16* b = Bh + (buf * BN + brow) * LDE;
#pragma unroll
            for (int i = 0; i < BCH / 2; ++i) {
                split8<MMA>(sb[2 * i], sb[2 * i + 1], hi, lo);
                *reinterpret_cast<bf16x8*>(b + bkq + 8 * i) = hi;
                if constexpr (MMA == MMA_BF16X3) *reinterpret_cast<bf16x8*>(b + 32 + bkq + 8 * i) = lo;
            }
        }
    };

    floatx16 acc[IM][JN], t[IM][JN];
#pragma unroll
    for (int i = 0; i < IM; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) { acc[i][j][r] = 0.f; t[i][j][r] = 0.f; }

    int pa0[NSUB], pa1[NSUB];
    load_a(kt_beg, ra, pa0);
    load_b(kt_beg, rb);
    store_tiles(0, ra, rb, pa0);
    __syncthreads();

    const int l32 = lane & 31, lk = (lane >> 5) * 16;
    if constexpr (MMA != MMA_F32) {
        // k-step s of a k-tile: lane (r, h) supplies A[row r][16s + 8h + 0..7] and
        // B[16s + 8h + 0..7][col r] (v_mfma_f32_32x32x16_bf16 operand map)
        constexpr int NST = BKT / 16;
        const int kh = (lane >> 5) * 8;
        auto step = [&](int cur, int st) {
            if constexpr (MMA == MMA_BF16P) {  // three 16-k sub-tiles, one product each, into acc
#pragma unroll
                for (int sub = 0; sub < 3; ++sub) {
                    bf16x8 fa[IM], fb[JN];
#pragma unroll
                    for (int i = 0; i < IM; ++i)
                        fa[i] = *reinterpret_cast<const bf16x8*>(Ah + x6o(sub, cur, wm * WM + i * 32 + l32, kh >> 3));
#pragma unroll
                    for (int j = 0; j < JN; ++j)
                        fb[j] = *reinterpret_cast<const bf16x8*>(Ah + x6o(sub, cur, BM + wn * WN + j * 32 + l32, kh >> 3));
#pragma unroll
                    for (int i = 0; i < IM; ++i)
#pragma unroll
                        for (int j = 0; j < JN; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
                }
                return;
            }
            if constexpr (H3) {  // per sub-tile: lo*hi, hi*lo, hi*hi (smallest terms first)
#pragma unroll
                for (int sub = 0; sub < NSUB; ++sub) {
                    f16x8 fah[IM], fal[IM], fbh[JN], fbl[JN];
#pragma unroll
                    for (int i = 0; i < IM; ++i) {
                        const int row = wm * WM + i * 32 + l32;
                        fah[i] = *reinterpret_cast<const f16x8*>(Ah + x6o(sub, cur, row, kh >> 3));
                        if constexpr (!F1) fal[i] = *reinterpret_cast<const f16x8*>(Ah + x6o(NSUB + sub, cur, row, kh >> 3));
                    }
#pragma unroll
                    for (int j = 0; j < JN; ++j) {
                        const int row = BM + wn * WN + j * 32 + l32;
                        fbh[j] = *reinterpret_cast<const f16x8*>(Ah + x6o(sub, cur, row, kh >> 3));
                        if constexpr (!F1) fbl[j] = *reinterpret_cast<const f16x8*>(Ah + x6o(NSUB + sub, cur, row, kh >> 3));
                    }
#pragma unroll
                    for (int i = 0; i < IM; ++i)
#pragma unroll
                        for (int j = 0; j < JN; ++j) {
                            if constexpr (!F1) {
                                t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fal[i], fbh[j], t[i][j], 0, 0, 0);
                                t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fah[i], fbl[j], t[i][j], 0, 0, 0);
                            }
                            t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fah[i], fbh[j], t[i][j], 0, 0, 0);
                        }
                }
                return;
            }
            bf16x8 ah[IM], bh[JN], al[IM], bl[JN], am[IM], bm[JN];
#pragma unroll
            for (int i = 0; i < IM; ++i) {
                if constexpr (MMA == MMA_BF16X6) {
                    const int row = wm * WM + i * 32 + l32;
                    ah[i] = *reinterpret_cast<const bf16x8*>(Ah + x6o(0, cur, row, kh >> 3));
                    am[i] = *reinterpret_cast<const bf16x8*>(Ah + x6o(1, cur, row, kh >> 3));
                    al[i] = *reinterpret_cast<const bf16x8*>(Ah + x6o(2, cur, row, kh >> 3));
                } else {
                    const __bf16* a = Ah + (cur * BM + wm * WM + i * 32 + l32) * LDE + 16 * st + kh;
                    ah[i] = *reinterpret_cast<const bf16x8*>(a);
                    if constexpr (MMA == MMA_BF16X3) al[i] = *reinterpret_cast<const bf16x8*>(a + 32);
                }
            }
#pragma unroll
            for (int j = 0; j < JN; ++j) {
                if constexpr (MMA == MMA_BF16X6) {
                    const int row = BM + wn * WN + j * 32 + l32;
                    bh[j] = *reinterpret_cast<const bf16x8*>(Ah + x6o(0, cur, row, kh >> 3));
                    bm[j] = *reinterpret_cast<const bf16x8*>(Ah + x6o(1, cur, row, kh >> 3));
                    bl[j] = *reinterpret_cast<const bf16x8*>(Ah + x6o(2, cur, row, kh >> 3));
                } else {
                    const __bf16* b = Bh + (cur * BN + wn * WN + j * 32 + l32) * LDE + 16 * st + kh;
                    bh[j] = *reinterpret_cast<const bf16x8*>(b);
                    if constexpr (MMA == MMA_BF16X3) bl[j] = *reinterpret_cast<const bf16x8*>(b + 32);
                }
            }
#pragma unroll
            for (int i = 0; i < IM; ++i)
#pragma unroll
                for (int j = 0; j < JN; ++j) {
                    if constexpr (MMA == MMA_BF16X6) {  // smallest terms first
                        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bm[j], t[i][j], 0, 0, 0);
                        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], t[i][j], 0, 0, 0);
                        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], t[i][j], 0, 0, 0);
                        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bh[j], t[i][j], 0, 0, 0);
                        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bm[j], t[i][j], 0, 0, 0);
                        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], t[i][j], 0, 0, 0);
                    } else if constexpr (MMA == MMA_BF16X3) {
                        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], t[i][j], 0, 0, 0);
                        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], t[i][j], 0, 0, 0);
                        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], t[i][j], 0, 0, 0);
                    } else {  // bf16: operand rounding dominates, one accumulation level
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                    }
                }
        };
        auto fold_t = [&](int kt) {  // close the inner accumulation chain every KT2 k-tiles
            if (MMA != MMA_BF16 && MMA != MMA_BF16P && ((kt % KT2) == KT2 - 1 || kt + 1 == nkt)) {
#pragma unroll
                for (int i = 0; i < IM; ++i)
#pragma unroll
                    for (int j = 0; j < JN; ++j) {
                        acc[i][j] += t[i][j];
#pragma unroll
                        for (int r = 0; r < 16; ++r) t[i][j][r] = 0.f;
                    }
            }
        };
        if constexpr (X6L && DCS_X6_PIPE) {
            // two register sets: tile kt+2's gather is in flight while tile kt computes, so
            // staging tile kt+1 waits only for loads issued a whole k-tile earlier
            // The loads are issued unconditionally (k-tiles past the end gather zeros from the
            // buffer descriptors): a load under a branch makes the compiler's vmcnt bookkeeping
            // assume it may be missing and wait for every load at the next LDS store.
            float4 ra2[ACH], rb2[BCH];
            int pa2[NSUB];
            load_a(kt_beg + 1, ra, pa1);
            load_b(kt_beg + 1, rb);
            for (int kt = kt_beg; kt < nkt; kt += 2) {
                load_a(kt + 2, ra2, pa2);
                load_b(kt + 2, rb2);
                step(0, 0);
                if (DCS_X6_STORE_FIRST) {
                    // staging before the chain fold and unconditional (a tile past the end is
                    // zeros into a buffer nobody reads again): one basic block with the MFMAs
                    store_tiles(1, ra, rb, pa1);
                    x6_interleave<IM * JN * (MMA == MMA_BF16P ? 3 : (H3 ? (F1 ? 1 : 3) * NSUB : 6)), (TAG == 1 && X6F) ? DCS_X6_SGB : DCS_X6_SGB0,
                                  H3 ? (IM + JN) * (F1 ? 1 : 2) * NSUB : 12, H3 ? (F1 ? 2 : 4) * NSUB : 6>();
                    fold_t(kt);
                } else {
                    fold_t(kt);
                    if (kt + 1 < nkt) store_tiles(1, ra, rb, pa1);
                }
                __syncthreads();
                if (kt + 1 >= nkt) break;
                load_a(kt + 3, ra, pa1);
                load_b(kt + 3, rb);
                step(1, 0);
                if (DCS_X6_STORE_FIRST) {
                    store_tiles(0, ra2, rb2, pa2);
                    x6_interleave<IM * JN * (MMA == MMA_BF16P ? 3 : (H3 ? (F1 ? 1 : 3) * NSUB : 6)), (TAG == 1 && X6F) ? DCS_X6_SGB : DCS_X6_SGB0,
                                  H3 ? (IM + JN) * (F1 ? 1 : 2) * NSUB : 12, H3 ? (F1 ? 2 : 4) * NSUB : 6>();
                    fold_t(kt + 1);
                } else {
                    fold_t(kt + 1);
                    if (kt + 2 < nkt) store_tiles(0, ra2, rb2, pa2);
                }
                __syncthreads();
            }
        } else {
            for (int kt = kt_beg; kt < nkt; ++kt) {
                const int cur = (kt - kt_beg) & 1;
#pragma unroll
                for (int st = 0; st < NST / 2; ++st) step(cur, st);
                if (kt + 1 < nkt) { load_a(kt + 1, ra, pa1); load_b(kt + 1, rb); }
#pragma unroll
                for (int st = NST / 2; st < NST; ++st) step(cur, st);
                fold_t(kt);
                if (kt + 1 < nkt) store_tiles(cur ^ 1, ra, rb, pa1);
                __syncthreads();
            }
        }
    } else
    for (int kt = kt_beg; kt < nkt; ++kt) {
        const int cur = (kt - kt_beg) & 1;
        float4 af[IM][4], bf[JN][4];
#pragma unroll
        for (int i = 0; i < IM; ++i)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                af[i][q] = *reinterpret_cast<const float4*>(&As[cur][wm * WM + i * 32 + l32][lk + 4 * q]);
#pragma unroll
        for (int j = 0; j < JN; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                bf[j][q] = *reinterpret_cast<const float4*>(&Bs[cur][wn * WN + j * 32 + l32][lk + 4 * q]);
        // MFMAs of the tile in two halves with the next tile's gather in between; the inner
        // chain t spans KT2 k-tiles (two-level summation, see mfma_ktile)
        mfma_chain<IM, JN, 0, 2>(af, bf, t);
        if (kt + 1 < nkt) { load_a(kt + 1, ra, pa1); load_b(kt + 1, rb); }
        mfma_chain<IM, JN, 2, 4>(af, bf, t);
        if ((kt % KT2) == KT2 - 1 || kt + 1 == nkt) {
#pragma unroll
            for (int i = 0; i < IM; ++i)
#pragma unroll
                for (int j = 0; j < JN; ++j) {
                    acc[i][j] += t[i][j];
#pragma unroll
                    for (int r = 0; r < 16; ++r) t[i][j][r] = 0.f;
                }
        }
        if (kt + 1 < nkt) store_tiles(cur ^ 1, ra, rb, pa1);
        __syncthreads();
    }

    if constexpr (H3) {  // undo the operand scales (exact powers of two)
#pragma unroll
        for (int i = 0; i < IM; ++i)
#pragma unroll
            for (int j = 0; j < JN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = __builtin_ldexpf(acc[i][j][r], eab);
    }
    // epilogue: + bias, activation, NHWC store; in the reflection-fold data gradient
    // (fold, dcs_conv_dgrad_reflect) src2 carries the residual addend of the interior pixels
    const float* addend = fold ? src2 : nullptr;
    const long long interior = fold ? (long long)d.N * (d.Ho - 2) * (d.Wo - 2) * d.Co : 0;
#pragma unroll
    for (int j = 0; j < JN; ++j) {
        const int col = n0 + wn * WN + j * 32 + l32;
        if (col >= d.Co) continue;
        const float bv = bias ? bias[col] : 0.f;
#pragma unroll
        for (int i = 0; i < IM; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                const long long off = rowoff[row];
                if (off < 0) continue;
                float v = acc[i][j][r] + bv;
                if (d.epi_act != DCS_ACT_NONE) v = act_apply(v, d.epi_act);
                if (addend && off < interior) v += addend[off + col];
                out[off + col] = v;
            }
        }
    }
    if (parts) rows_in_stats<BM, BN, IM, JN>(d, acc, bias, n0, m0, g, z, wm, wn, lane, tid, lds, parts);
}

// ---------------------------------------------------------------------------------------
// wgrad pass: dW[co][k] = sum_p dy[p][co] * A[p][k]  (split over pixels -> partial slabs)
// ---------------------------------------------------------------------------------------
// Both operands arrive pixel-major (k-major), so LDS keeps them as [k][m] / [k][n] rows
// (m/n contiguous, padded by 4): every loader thread moves float4 runs straight from global
// to LDS (8 threads per pixel row, one pixel decode per thread per k-tile).  A lane's MFMA
// operands are single floats down a column ([2s+h][m]); all 16 k-steps of a tile are read
// into registers before the tile's MFMAs so LDS latency is paid once per tile.
template <int BM, int BN, int VEC, int TAG>
__global__ __launch_bounds__(NT, 2) void conv_wgrad_kernel(
    const dcs_conv_desc din, const float* __restrict__ dy, const float* __restrict__ src,
    const float* __restrict__ src2, const float* __restrict__ psc, const float* __restrict__ psh,
    float* __restrict__ ws, int kt_per_split, int gn, int gm) {
    const dcs_conv_desc d = specialise<TAG>(din);
    constexpr int WM = BM / 2, WN = BN / 2;
    constexpr int IM = WM / 32, JN = WN / 32;
    constexpr int LDA = BM + 4, LDB = BN + 4;
    constexpr int ACH = (BK * BM / 4) / NT;
    constexpr int BCH = (BK * BN / 4) / NT;

    __shared__ __attribute__((aligned(16))) float As[2][BK][LDA];
    __shared__ __attribute__((aligned(16))) float Bs[2][BK][LDB];

    // sub-pixel descriptors (parity 2, VEC only) run one GEMM per phase z: dy rows are the
    // phase's output pixels (2qy+ry, 2qx+rx), columns its 4 taps x Cs
    const int ncls = d.parity == 2 ? 4 : 1;
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int ntile = L % gn;
    const int mtile = (L / gn) % gm;
    const int z = (L / (gn * gm)) % ncls;
    const int split = L / (gn * gm * ncls);
    const ClassGeom g = class_geom(d, z);
    const long long P = (long long)g.My * g.Mx * d.N;   // pixels (reduction)
    const int Ktot = g.ntaps * d.Cs;                    // GEMM N
    const int m0 = mtile * BM;                          // output channel tile
    const int n0 = ntile * BN;                          // (tap, ci) tile
    const long long nkt_all = (P + BK - 1) / BK;
    const long long kt_beg = (long long)split * kt_per_split;
    long long kt_end = kt_beg + kt_per_split;
    if (kt_end > nkt_all) kt_end = nkt_all;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int kr = tid >> 3;
    const int ac0 = (tid & 7) * (BM / 8), bc0 = (tid & 7) * (BN / 8);

    float4 ra[ACH];
    float4 rb[BCH];

    // B columns of this thread are fixed for the whole kernel: with VEC (Cs % 16 == 0) its
    // BN/8 consecutive columns share one tap -> decode once.
    const int nb0 = n0 + bc0;
    const bool bcol_ok = nb0 < Ktot;
    int bady = 0, badx = 0, bchan = 0;
    // VEC == 2 (Cs == 4): the thread's 16 columns are 4 taps x 4 channels
    int q4y[4] = {0, 0, 0, 0}, q4x[4] = {0, 0, 0, 0};
    bool q4ok[4] = {false, false, false, false};
    if (VEC == 2) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int j = nb0 / 4 + e;
            q4ok[e] = nb0 + 4 * e < Ktot;
            int bt;
            if (q4ok[e]) tap_decode(d, g, j, q4y[e], q4x[e], bt);
        }
    } else if (VEC && bcol_ok) {
        const int j = nb0 / d.Cs;
        bchan = nb0 - j * d.Cs;
        int bt;
        tap_decode(d, g, j, bady, badx, bt);
    }
    const int Hv = d.Hs * d.up, Wv = d.Ws * d.up;
    const __amdgpu_buffer_rsrc_t rsrc = src_rsrc(src);
    // incremental pixel state of the NEXT k-tile row this thread loads (p = kt*BK + kr)
    int pn = 0, pqy = 0, pqx = 0;
    {
        const long long p = kt_beg * BK + kr;
        if (p < P) {
            const int per = g.My * g.Mx;
            pn = (int)(p / per);
            const int rem = (int)(p - (long long)pn * per);
            pqy = rem / g.Mx;
            pqx = rem - pqy * g.Mx;
        }
    }
    auto advance_pix = [&]() {
        pqx += BK;
        while (pqx >= g.Mx) { pqx -= g.Mx; if (++pqy == g.My) { pqy = 0; ++pn; } }
    };

    auto load_a = [&](long long kt) {  // dy rows: [p][co]
        long long p = kt * BK + kr;
        const int co = m0 + ac0;
        const bool ok = p < P;
        if (d.parity == 2) p = ((long long)pn * d.Ho + 2 * pqy + g.ry) * d.Wo + 2 * pqx + g.rx;
#pragma unroll
        for (int i = 0; i < ACH; ++i)
            ra[i] = (ok && co + 4 * i < d.Co) ? *reinterpret_cast<const float4*>(dy + p * d.Co + co + 4 * i)
                                              : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    auto load_b = [&](long long kt) {  // gathered source rows: [p][(tap, ci)]
        const long long p = kt * BK + kr;
#pragma unroll
        for (int i = 0; i < BCH; ++i) rb[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (VEC == 2) {
            const int by = pqy * d.stride - d.pt, bx = pqx * d.stride - d.pl;
            const int rowoff = pn * (int)d.s_n;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                int sy, sx;
                const bool yok = map_coord_sel(by + q4y[e], Hv, d.up, d.pad_mode, sy);
                const bool xok = map_coord_sel(bx + q4x[e], Wv, d.up, d.pad_mode, sx);
                const bool ok = p < P && q4ok[e] && yok && xok;
                rb[e] = buf_load4(rsrc, ok ? (rowoff + sy * (int)d.s_h + sx * (int)d.s_w) * 4 : OOB_OFF);
            }
            advance_pix();
        } else if (VEC) {
            // the thread's BN/8 columns share one tap (Cs % 16 == 0); bcol_ok covers all of them
            // sub-pixel phases: the tap offsets already include the padding
            const int vy = d.parity == 2 ? pqy + bady : pqy * d.stride - d.pt + bady;
            const int vx = d.parity == 2 ? pqx + badx : pqx * d.stride - d.pl + badx;
            int sy, sx;
            const bool yok = map_coord_sel(vy, Hv, d.up, d.pad_mode, sy);
            const bool xok = map_coord_sel(vx, Wv, d.up, d.pad_mode, sx);
            const bool ok = p < P && bcol_ok && yok && xok;
            const int off = ok ? (pn * (int)d.s_n + sy * (int)d.s_h + sx * (int)d.s_w + bchan) * 4 : OOB_OFF;
#pragma unroll
            for (int i = 0; i < BCH; ++i) rb[i] = buf_load4(rsrc, off + 16 * i);
            if (d.pro_act != DCS_ACT_NONE) {
                const long long o = (long long)pn * d.Cs + bchan;
#pragma unroll
                for (int i = 0; i < BCH; ++i) {
                    const float4 v = affine_act4(rb[i], psc + o + 4 * i, psh + o + 4 * i, d.pro_act);
                    rb[i] = ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
            advance_pix();
        } else if (p < P) {
            const RowInfo ri = row_info(d, g, (int)p);
#pragma unroll
            for (int i = 0; i < BCH; ++i) {
                float e[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    e[q] = 0.f;
                    const int n1 = nb0 + 4 * i + q;
                    if (n1 < Ktot) {
                        int j = n1 / d.Cs, c = n1 - j * d.Cs;
                        int ady, adx, bt;
                        tap_decode(d, g, j, ady, adx, bt);
                        e[q] = gather1(d, src, src2, psc, psh, ri.n, ri.by + ady, ri.bx + adx, c);
                    }
                }
                rb[i] = make_float4(e[0], e[1], e[2], e[3]);
            }
        }
    };
    // LDS column swizzle phys(c) = c ^ (((c >> 5) & 3) << 2): the 8 lanes of a ds_write_b128
    // group store columns 16t + 4i (t = 0..7), which would hit only two 4-bank slots; XOR-ing
    // bits 2-3 with (c >> 5) spreads them over all 8 slots.  A fragment read (32 consecutive
    // columns of one 32-aligned group) sees a fixed permutation, so it stays conflict-free.
    auto swz = [](int c) { return c ^ (((c >> 5) & 3) << 2); };
    int aoff[ACH], boff[BCH];
#pragma unroll
    for (int i = 0; i < ACH; ++i) aoff[i] = swz(ac0 + 4 * i);
#pragma unroll
    for (int i = 0; i < BCH; ++i) boff[i] = swz(bc0 + 4 * i);
    auto store_tiles = [&](int buf) {
#pragma unroll
        for (int i = 0; i < ACH; ++i) *reinterpret_cast<float4*>(&As[buf][kr][aoff[i]]) = ra[i];
#pragma unroll
        for (int i = 0; i < BCH; ++i) *reinterpret_cast<float4*>(&Bs[buf][kr][boff[i]]) = rb[i];
    };

    constexpr int KT2 = 4;  // k-tiles per inner accumulation chain (two-level summation)
    floatx16 acc[IM][JN], t[IM][JN];
#pragma unroll
    for (int i = 0; i < IM; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) { acc[i][j][r] = 0.f; t[i][j][r] = 0.f; }

    if (kt_beg < kt_end) {
        load_a(kt_beg);
        load_b(kt_beg);
        store_tiles(0);
    }
    __syncthreads();
    const int l32 = lane & 31, lh = lane >> 5;
    // swizzled fragment columns (see store_tiles): group g = c >> 5 permutes l32 by XOR
    int acol[IM], bcol[JN];
#pragma unroll
    for (int i = 0; i < IM; ++i) {
        const int c = wm * WM + i * 32;
        acol[i] = swz(c + l32);
    }
#pragma unroll
    for (int j = 0; j < JN; ++j) {
        const int c = wn * WN + j * 32;
        bcol[j] = swz(c + l32);
    }
    for (long long kt = kt_beg; kt < kt_end; ++kt) {
        const int cur = (int)((kt - kt_beg) & 1);
        // fragments of all 16 k-steps (lane half h takes k = 2s + h)
        float4 af[IM][4], bf[JN][4];
#pragma unroll
        for (int i = 0; i < IM; ++i)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float* a = &As[cur][8 * q + lh][acol[i]];
                af[i][q] = make_float4(a[0], a[2 * LDA], a[4 * LDA], a[6 * LDA]);
            }
#pragma unroll
        for (int j = 0; j < JN; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float* b = &Bs[cur][8 * q + lh][bcol[j]];
                bf[j][q] = make_float4(b[0], b[2 * LDB], b[4 * LDB], b[6 * LDB]);
            }
        if constexpr (VEC != 0) {
            mfma_chain<IM, JN, 0, 2>(af, bf, t);
            if (kt + 1 < kt_end) { load_a(kt + 1); load_b(kt + 1); }
            mfma_chain<IM, JN, 2, 4>(af, bf, t);
            const long long rel = kt - kt_beg;
            if ((rel % KT2) == KT2 - 1 || kt + 1 == kt_end) {
#pragma unroll
                for (int i = 0; i < IM; ++i)
#pragma unroll
                    for (int j = 0; j < JN; ++j) {
                        acc[i][j] += t[i][j];
#pragma unroll
                        for (int r = 0; r < 16; ++r) t[i][j][r] = 0.f;
                    }
            }
        } else {  // small-Cs gathers (stem, first PatchGAN layer): short K chains, one level
            mfma_chain<IM, JN, 0, 4>(af, bf, acc);
            if (kt + 1 < kt_end) { load_a(kt + 1); load_b(kt + 1); }
        }
        if (kt + 1 < kt_end) store_tiles(cur ^ 1);
        __syncthreads();
    }

    float* slab = ws + ((long long)split * ncls + z) * d.Co * Ktot;
#pragma unroll
    for (int j = 0; j < JN; ++j) {
        const int col = n0 + wn * WN + j * 32 + l32;
        if (col >= Ktot) continue;
#pragma unroll
        for (int i = 0; i < IM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                if (row < d.Co) slab[(long long)row * Ktot + col] = acc[i][j][r];
            }
    }
}


// dw[co][ci][ty][tx] = sum_s ws[s][co][(ty*KW+tx)*Cs + ci].  Threads walk the slabs in
// their own (co, tap, ci) order so the nsplit reads per output are coalesced; each output is
// written once (scattered into OIHW).  Fixed split order: deterministic.
__global__ void wgrad_reduce_kernel(const float* __restrict__ ws, int nsplit, int Co, int Cs, int KH,
                                    int KW, int Cw, float* __restrict__ dw) {
    long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const int taps = KH * KW;
    const long long Ktot = (long long)taps * Cs;
    const long long total = (long long)Co * Ktot;
    if (idx >= total) return;
    const int co = (int)(idx / Ktot);
    const int k = (int)(idx - (long long)co * Ktot);
    const int tap = k / Cs, ci = k - tap * Cs;
    float s = 0.f;
    if (ci >= Cw) return;  // zero-padded source channel (no weight)
    // loads hoisted 8 at a time, the additions kept in split order (bit-identical sums)
#pragma unroll DCS_WGRAD_REDUCE_UNROLL
    for (int q = 0; q < nsplit; ++q) s += ws[(long long)q * total + idx];
    dw[((long long)co * Cw + ci) * taps + tap] = s;
}

// ---------------------------------------------------------------------------------------
// narrow rows (Co <= 4): one thread per output pixel, weights in LDS
// ---------------------------------------------------------------------------------------
template <int NO, bool VEC>
__global__ __launch_bounds__(256) void conv_rows_narrow_kernel(
    const dcs_conv_desc d, const float* __restrict__ src, const float* __restrict__ src2,
    const float* __restrict__ wp, const float* __restrict__ bias, const float* __restrict__ psc,
    const float* __restrict__ psh, float* __restrict__ out, int Krows) {
    extern __shared__ __attribute__((aligned(16))) float wl[];  // [Krows][NO]
    for (int i = threadIdx.x; i < Krows * NO; i += blockDim.x) {
        int k = i / NO, o = i - k * NO;
        wl[i] = wp[(long long)k * d.ldb + o];
    }
    __syncthreads();
    const int z = blockIdx.y;
    const ClassGeom g = class_geom(d, z);
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    const RowInfo ri = row_info(d, g, m);
    if (ri.out_off < 0) return;
    float acc[NO];
#pragma unroll
    for (int o = 0; o < NO; ++o) acc[o] = 0.f;
    for (int j = 0; j < g.ntaps; ++j) {
        int ady, adx, bt;
        tap_decode(d, g, j, ady, adx, bt);
        const float* wt = wl + (long long)bt * d.Cs * NO;
        if (VEC) {
            int sy, sx;
            const int Hv = d.Hs * d.up, Wv = d.Ws * d.up;
            if (!(map_coord(ri.by + ady, Hv, d.up, d.pad_mode, sy) &&
                  map_coord(ri.bx + adx, Wv, d.up, d.pad_mode, sx)))
                continue;
            const float* sp = src + ri.n * d.s_n + sy * d.s_h + sx * d.s_w;
            const long long so = (long long)ri.n * d.Cs;
            for (int c = 0; c < d.Cs; c += 4) {
                float4 v = *reinterpret_cast<const float4*>(sp + c);
                if (d.pro_act != DCS_ACT_NONE) v = affine_act4(v, psc + so + c, psh + so + c, d.pro_act);
#pragma unroll
                for (int o = 0; o < NO; ++o) {
                    acc[o] = fmaf(v.x, wt[(c + 0) * NO + o], acc[o]);
                    acc[o] = fmaf(v.y, wt[(c + 1) * NO + o], acc[o]);
                    acc[o] = fmaf(v.z, wt[(c + 2) * NO + o], acc[o]);
                    acc[o] = fmaf(v.w, wt[(c + 3) * NO + o], acc[o]);
                }
            }
        } else {
            for (int c = 0; c < d.Cs; ++c) {
                float v = gather1(d, src, src2, psc, psh, ri.n, ri.by + ady, ri.bx + adx, c);
#pragma unroll
                for (int o = 0; o < NO; ++o) acc[o] = fmaf(v, wt[c * NO + o], acc[o]);
            }
        }
    }
#pragma unroll
    for (int o = 0; o < NO; ++o) {
        if (o >= d.Co) break;
        float v = acc[o] + (bias ? bias[o] : 0.f);
        if (d.epi_act != DCS_ACT_NONE) v = act_apply(v, d.epi_act);
        out[ri.out_off + o] = v;
    }
}

// narrow wgrad: partial[s][o][k] = sum_{p in split s} dy[p][o] * A[p][k]
template <int NO, bool VEC>
__global__ __launch_bounds__(256) void conv_wgrad_narrow_kernel(
    const dcs_conv_desc d, const float* __restrict__ dy, const float* __restrict__ src,
    const float* __restrict__ src2, const float* __restrict__ psc, const float* __restrict__ psh,
    float* __restrict__ ws, long long pix_per_split) {
    const ClassGeom g = class_geom(d, 0);
    const long long P = (long long)g.My * g.Mx * d.N;
    const int Ktot = g.ntaps * d.Cs;
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int split = blockIdx.y;
    const long long p0 = (long long)split * pix_per_split;
    long long p1 = p0 + pix_per_split;
    if (p1 > P) p1 = P;
    if (k >= Ktot) return;
    const int j = k / d.Cs, c = k - j * d.Cs;
    int ady, adx, bt;
    tap_decode(d, g, j, ady, adx, bt);
    float acc[NO];
#pragma unroll
    for (int o = 0; o < NO; ++o) acc[o] = 0.f;
    for (long long p = p0; p < p1; ++p) {
        RowInfo ri = row_info(d, g, (int)p);
        float v = gather1(d, src, src2, psc, psh, ri.n, ri.by + ady, ri.bx + adx, c);
        const float* dp = dy + p * d.Co;
#pragma unroll
        for (int o = 0; o < NO; ++o) acc[o] = fmaf(dp[o], v, acc[o]);
    }
    float* slab = ws + (long long)split * d.Co * Ktot;
#pragma unroll
    for (int o = 0; o < NO; ++o)
        if (o < d.Co) slab[(long long)o * Ktot + k] = acc[o];
}

// ---------------------------------------------------------------------------------------
// padding / upsampling adjoints
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int reflect_pre(int i, int H, int pad, int* a) {
    // padded positions a with reflect(a - pad) == i
    int n = 0;
    a[n++] = i + pad;
    if (i >= 1 && i <= pad) a[n++] = pad - i;
    if (i >= H - 1 - pad && i <= H - 2) a[n++] = 2 * (H - 1) - i + pad;
    return n;
}

__global__ void reflect_fold_kernel(const float* __restrict__ dxp, const float* __restrict__ add,
                                    float* __restrict__ dx, int N, int H, int W, int C4, int pad) {
    // 32-bit index math (the host guarantees N*(H+2p)*(W+2p)*C4 < 2^31)
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int total = N * H * W * C4;
    if (idx >= total) return;
    const int c4 = idx % C4;
    int t = idx / C4;
    const int j = t % W; t /= W;
    const int i = t % H;
    const int n = t / H;
    const int Hp = H + 2 * pad, Wp = W + 2 * pad;
    int ay[3], ax[3];
    int ny = reflect_pre(i, H, pad, ay), nx = reflect_pre(j, W, pad, ax);
    float4 s = add ? reinterpret_cast<const float4*>(add)[idx] : make_float4(0.f, 0.f, 0.f, 0.f);
    for (int p = 0; p < ny; ++p)
        for (int q = 0; q < nx; ++q) {
            float4 v = reinterpret_cast<const float4*>(dxp)[((n * Hp + ay[p]) * Wp + ax[q]) * C4 + c4];
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
    reinterpret_cast<float4*>(dx)[idx] = s;
}

__global__ void reflect_fold_scalar_kernel(const float* __restrict__ dxp, const float* __restrict__ add,
                                           float* __restrict__ dx, int N, int H, int W, int C, int pad) {
    long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    long long total = (long long)N * H * W * C;
    if (idx >= total) return;
    int c = (int)(idx % C);
    long long t = idx / C;
    int j = (int)(t % W); t /= W;
    int i = (int)(t % H);
    int n = (int)(t / H);
    const int Hp = H + 2 * pad, Wp = W + 2 * pad;
    int ay[3], ax[3];
    int ny = reflect_pre(i, H, pad, ay), nx = reflect_pre(j, W, pad, ax);
    float s = add ? add[idx] : 0.f;
    for (int p = 0; p < ny; ++p)
        for (int q = 0; q < nx; ++q) s += dxp[(((long long)n * Hp + ay[p]) * Wp + ax[q]) * C + c];
    dx[idx] = s;
}

// ring fold of dcs_conv_dgrad_reflect (pad 1): dx[y][x] += the ring entries of the padded
// grid that reflect onto (y, x) (rows 1 and H-2, columns 1 and W-2), in reflect_pre order; the
// conv epilogue already stored the interior contribution (plus the addend).  One thread per
// (image, target pixel, 4 channels); targets: the two rows over every column, then the two
// columns over the remaining rows.
__global__ void reflect_ring_fold_kernel(const float* __restrict__ ring, float* __restrict__ dx, int N, int H, int W,
                                         int C4, int nsplit) {
    const int ntgt = 2 * W + 2 * (H - 2);
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)N * ntgt * C4) return;
    const int c4 = (int)(idx % C4);
    const int t = (int)((idx / C4) % ntgt);
    const int n = (int)(idx / ((long long)C4 * ntgt));
    int y, x;
    if (t < 2 * W) {
        y = t < W ? 1 : H - 2;
        x = t < W ? t : t - W;
    } else {
        const int u = t - 2 * W;  // rows 0, 2..H-3, H-1 (rows 1 and H-2 are covered above)
        const int rr = u >> 1;
        y = rr == 0 ? 0 : (rr <= H - 4 ? rr + 1 : H - 1);
        x = (u & 1) ? W - 2 : 1;
    }
    const int Hp = H + 2, Wp = W + 2, ringlen = 2 * Wp + 2 * H;
    int ay[3], ax[3];
    const int ny = reflect_pre(y, H, 1, ay), nx = reflect_pre(x, W, 1, ax);
    float4* o = reinterpret_cast<float4*>(dx) + (((long long)n * H + y) * W + x) * C4 + c4;
    float4 s = *o;
    for (int p = 0; p < ny; ++p)
        for (int q = 0; q < nx; ++q) {
            const int yp = ay[p], xp = ax[q];
            if (yp >= 1 && yp <= H && xp >= 1 && xp <= W) continue;  // interior: in the epilogue
            const int ri = yp == 0 ? xp : (yp == Hp - 1 ? Wp + xp : 2 * Wp + 2 * (yp - 1) + (xp == 0 ? 0 : 1));
            for (int q = 0; q < nsplit; ++q) {  // the K splits' ring copies, in split order
                const float4 v = reinterpret_cast<const float4*>(ring)[(((long long)q * N + n) * ringlen + ri) * C4 + c4];
                s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
            }
        }
    *o = s;
}

__global__ void upsample2_grad_kernel(const float* __restrict__ du, float* __restrict__ dx, int N, int H,
                                      int W, int C4) {
    long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    long long total = (long long)N * H * W * C4;
    if (idx >= total) return;
    int c4 = (int)(idx % C4);
    long long t = idx / C4;
    int j = (int)(t % W); t /= W;
    int i = (int)(t % H);
    int n = (int)(t / H);
    const float4* u = reinterpret_cast<const float4*>(du);
    const long long W2 = 2LL * W;
    long long b = (((long long)n * 2 * H + 2 * i) * W2 + 2 * j) * C4 + c4;
    float4 a0 = u[b], a1 = u[b + C4], a2 = u[b + W2 * C4], a3 = u[b + W2 * C4 + C4];
    reinterpret_cast<float4*>(dx)[idx] =
        make_float4(a0.x + a1.x + a2.x + a3.x, a0.y + a1.y + a2.y + a3.y, a0.z + a1.z + a2.z + a3.z,
                    a0.w + a1.w + a2.w + a3.w);
}

// ---------------------------------------------------------------------------------------
// host-side validation and dispatch
// ---------------------------------------------------------------------------------------
static int validate(const dcs_conv_desc* d, bool rows) {
    if (!d) return fail(DCS_E_INVALID, "null descriptor");
    if (d->N <= 0 || d->Hs <= 0 || d->Ws <= 0 || d->Cs <= 0 || d->Ho <= 0 || d->Wo <= 0 || d->Co <= 0)
        return fail(DCS_E_INVALID, "conv: non-positive dimension");
    if (d->KH <= 0 || d->KW <= 0 || d->KH * d->KW > 64) return fail(DCS_E_INVALID, "conv: bad kernel");
    if (d->up != 1 && d->up != 2) return fail(DCS_E_INVALID, "conv: up must be 1 or 2");
    if (d->stride != 1 && d->stride != 2) return fail(DCS_E_INVALID, "conv: stride must be 1 or 2");
    if (d->parity < 0 || d->parity > 2) return fail(DCS_E_INVALID, "conv: parity must be 0, 1 or 2");
    if (d->parity == 1 && (d->stride != 2 || d->up != 1 || d->pad_mode != DCS_PAD_ZERO))
        return fail(DCS_E_INVALID, "conv: parity rows need stride 2, no upsample, zero pad");
    if (d->parity == 2 && (d->stride != 1 || d->up != 1 || d->pad_mode != DCS_PAD_ZERO || d->KH != 3 ||
                           d->KW != 3 || d->Ho != 2 * d->Hs || d->Wo != 2 * d->Ws))
        return fail(DCS_E_INVALID, "conv: sub-pixel rows describe nearest-x2 + 3x3 zero-pad conv (up=1, Ho=2Hs)");
    if (d->pad_mode == DCS_PAD_REFLECT && (d->pt >= d->Hs * d->up || d->pl >= d->Ws * d->up))
        return fail(DCS_E_INVALID, "conv: reflect pad larger than the input");
    if (d->csplit < 0 || d->csplit > d->Cs) return fail(DCS_E_INVALID, "conv: bad csplit");
    if (d->cw < 0 || d->cw > d->Cs) return fail(DCS_E_INVALID, "conv: bad cw (weight channels)");
    if (d->mma != MMA_F32 && d->mma != MMA_BF16 && d->mma != MMA_BF16X3 && d->mma != MMA_BF16X6 && d->mma != MMA_F16X3 &&
        d->mma != MMA_F16)
        return fail(DCS_E_INVALID, "conv: mma must be DCS_MMA_F32, DCS_MMA_BF16, DCS_MMA_BF16X3, DCS_MMA_BF16X6, DCS_MMA_F16X3 or DCS_MMA_F16");
    if ((d->mma == MMA_F16X3 || d->mma == MMA_F16) && (!d->rng_a || !d->rng_b || d->rng_a_n <= 0 || d->rng_b_n <= 0 ||
                                d->rng_a_n > 1024 || d->rng_b_n > 1024))
        return fail(DCS_E_INVALID, "conv: DCS_MMA_F16X3 / DCS_MMA_F16 need the operand range records rng_a / rng_b (1..1024 partial maxima)");
    if (!d->parity) {
        // output dims must be those of the forward conv over the virtual input
        int Hv = d->Hs * d->up, Wv = d->Ws * d->up;
        (void)Hv; (void)Wv;
    }
    (void)rows;
    return DCS_OK;
}

// 4-channel NHWC source (the packed stem input): float4 per tap, 16-byte aligned pixels
static bool vec4_ok(const dcs_conv_desc* d, const float* src) {
    const long long extent = (long long)(d->N - 1) * d->s_n + (long long)(d->Hs - 1) * d->s_h +
                             (long long)(d->Ws - 1) * d->s_w + d->Cs;
    return d->Cs == 4 && d->s_c == 1 && d->csplit == 4 && (d->s_w % 4 == 0) && (d->s_h % 4 == 0) &&
           (d->s_n % 4 == 0) && ((reinterpret_cast<uintptr_t>(src) & 15) == 0) && d->s_n >= 0 && d->s_h >= 0 &&
           d->s_w >= 0 && extent * 4 < (long long)OOB_OFF - 64;
}

static bool vec_ok(const dcs_conv_desc* d, const float* src) {
    // the vectorised gathers address the source through a buffer descriptor with 32-bit byte
    // offsets: every element they can touch must lie below 2 GiB (minus the OOB sentinel)
    const long long extent = (long long)(d->N - 1) * d->s_n + (long long)(d->Hs - 1) * d->s_h +
                             (long long)(d->Ws - 1) * d->s_w + d->Cs;
    return (d->Cs % 16 == 0) && d->s_c == 1 && d->csplit == d->Cs &&
           (d->s_w % 4 == 0) && (d->s_h % 4 == 0) && (d->s_n % 4 == 0) &&
           ((reinterpret_cast<uintptr_t>(src) & 15) == 0) && extent * 4 < (long long)OOB_OFF - 64 &&
           d->s_n >= 0 && d->s_h >= 0 && d->s_w >= 0;
}

// LDS-tiled single-output-channel kernels (conv_narrow.hip)
bool narrow_tiled_ok(const dcs_conv_desc& d, const float* src);
int launch_narrow_rows_tiled(const dcs_conv_desc& d, const float* src, const float* wp, const float* bias,
                             const float* psc, const float* psh, float* out, hipStream_t s);
bool narrow_small_ok(const dcs_conv_desc& d, const float* src);
int launch_narrow_rows_small(const dcs_conv_desc& d, const float* src, const float* wp, const float* bias,
                             const float* psc, const float* psh, float* out, hipStream_t s);
bool narrow_wgrad_tiled_ok(const dcs_conv_desc& d, const float* src);
int narrow_wgrad_tiled_blocks(const dcs_conv_desc& d);
int launch_narrow_wgrad_tiled(const dcs_conv_desc& d, const float* dy, const float* src, const float* psc,
                              const float* psh, float* part, hipStream_t s);

}  // namespace dcs

using namespace dcs;

extern "C" int dcs_pack_weights_r(const float* w, int Cout, int Cin, int KH, int KW, int kind, int ci_count,
                                  int Kpad, int ncols, int nmajor, float* out, float* rng, void* stream);
namespace {
// blocks of a per-pack range / pack launch: one element per thread, at most one block per range-record
// slot (a small pack no longer dispatches 512 mostly idle blocks; ~8 elements per thread measured slower)
unsigned pack_blocks(long long total) {
    const long long b = cdiv(total, 256);
    return (unsigned)(b < 1 ? 1 : (b > DCS_RANGE_PARTS ? DCS_RANGE_PARTS : b));
}
}  // namespace
extern "C" int dcs_pack_weights(const float* w, int Cout, int Cin, int KH, int KW, int kind, int ci_count,
                                int Kpad, int ncols, int nmajor, float* out, void* stream) {
    return dcs_pack_weights_r(w, Cout, Cin, KH, KW, kind, ci_count, Kpad, ncols, nmajor, out, nullptr, stream);
}

namespace {
const char* pack_args_error(const float* w, int Cout, int Cin, int KH, int KW, int kind, int ci_count, int Kpad,
                            int ncols, const float* out) {
    if (!w || !out || Cout <= 0 || Cin <= 0 || KH <= 0 || KW <= 0 || Kpad <= 0 || ncols <= 0 || ci_count <= 0 ||
        (kind != 5 && ci_count > Cin) || (kind == 5 && ci_count < Cin) || kind < 0 ||
        (kind & 7) > 5 || (kind & ~(7 | DCS_PACK_KSLICE)) ||
        ((kind & DCS_PACK_KSLICE) && (((kind & 7) != 0 && (kind & 7) != 1) ||
                                      ((kind & 7) == 0 ? Cin : Cout) % 16 != 0)))
        return "pack_weights: bad arguments";
    if ((kind == 3 || kind == 4) && (KH != 3 || KW != 3)) return "pack_weights: sub-pixel kinds need 3x3";
    return nullptr;
}
}  // namespace

extern "C" int dcs_pack_weights_r(const float* w, int Cout, int Cin, int KH, int KW, int kind, int ci_count,
                                  int Kpad, int ncols, int nmajor, float* out, float* rng, void* stream) {
    if (const char* err = pack_args_error(w, Cout, Cin, KH, KW, kind, ci_count, Kpad, ncols, out))
        return fail(DCS_E_INVALID, err);
    long long total = (long long)Kpad * ncols;
    if (rng)
        hipLaunchKernelGGL(pack_weights_r_kernel, dim3(pack_blocks(total)), dim3(256), 0, as_stream(stream), w, Cout, Cin,
                           KH, KW, kind, ci_count, Kpad, ncols, nmajor, out, rng);
    else
        hipLaunchKernelGGL(pack_weights_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, as_stream(stream), w,
                           Cout, Cin, KH, KW, kind, ci_count, Kpad, ncols, nmajor, out);
    return check_launch("pack_weights");
}

namespace dcs {
// pre-split B of the f16x3 / f16 rows pass: out[r][0][k] = hi, out[r][1][k] = lo of wpack[r][k] * 2^eb, eb the
// exponent the rows kernel derives from the same range record (f16x3_exp), so the split is the one it would
// do at staging (split8h)
__global__ __launch_bounds__(256) void pack_split_h3_kernel(const float* __restrict__ wp, long long total, int ldb,
                                                            const float* __restrict__ rng, int rng_n,
                                                            _Float16* __restrict__ out) {
    const float sc = __builtin_ldexpf(1.f, f16x3_exp(rng, rng_n));
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
        const long long r = i / ldb, k = i - r * ldb;
        const float v = wp[i] * sc;
        const _Float16 h = (_Float16)v;
        out[2 * r * ldb + k] = h;
        out[(2 * r + 1) * ldb + k] = (_Float16)(v - (float)h);
    }
}
}  // namespace dcs

extern "C" int dcs_pack_split_h3(const float* wpack, int rows, int ldb, const float* rng, int rng_n, void* out,
                                 void* stream) {
    if (!wpack || !rng || !out || rows <= 0 || ldb <= 0 || rng_n <= 0) return fail(DCS_E_INVALID, "pack_split_h3: bad arguments");
    const long long total = (long long)rows * ldb;
    const long long blocks = cdiv(total, 256) < 1024 ? cdiv(total, 256) : 1024;
    hipLaunchKernelGGL(pack_split_h3_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), wpack, total, ldb,
                       rng, rng_n, reinterpret_cast<_Float16*>(out));
    return check_launch("pack_split_h3");
}

namespace dcs {
namespace {
// batched weight packs (dcs_pack_batch): block -> job by a binary search over the jobs' first blocks
__device__ __forceinline__ int pack_job_of(const dcs_pack_job* __restrict__ jobs, int njobs, int b, bool second) {
    int lo = 0, hi = njobs - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        const int start = second ? jobs[mid].p0 : jobs[mid].b0;
        if (start <= b) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// launch 1: each pack and its range record (kind >= 0), or the range of the raw weights of a window pack
__global__ __launch_bounds__(256) void pack_batch1_kernel(const dcs_pack_job* __restrict__ jobs, int njobs) {
    const int j = pack_job_of(jobs, njobs, blockIdx.x, false);
    const dcs_pack_job& jb = jobs[j];
    const int lb = blockIdx.x - jb.b0, nb = jb.b1;
    float m = 0.f;
    float* rng;
    if (jb.h3 == 2) {  // sub-pixel phase weights: the range of the combined values
        const long long n = 16LL * jb.Cout * jb.Cin;
        const int K = subpix_K(jb.Cout, jb.Cin, jb.h3_flip);
        for (long long i = (long long)lb * 256 + threadIdx.x; i < n; i += (long long)nb * 256) {
            const int v = (int)(i / K);
            m = fmaxf(m, fabsf(subpix_value(jb.w, jb.Cout, jb.Cin, jb.h3_flip, v, (int)(i - (long long)v * K))));
        }
        rng = jb.h3_scratch;
    } else if (jb.h3) {
        const long long n = (long long)jb.Cout * jb.Cin * 9;
        for (long long i = (long long)lb * 256 + threadIdx.x; i < n; i += (long long)nb * 256) m = fmaxf(m, fabsf(jb.w[i]));
        rng = jb.h3_scratch;
    } else {
        const long long total = (long long)jb.Kpad * jb.ncols;
        for (long long idx = (long long)lb * 256 + threadIdx.x; idx < total; idx += (long long)nb * 256) {
            const float v = pack_value(jb.w, jb.Cout, jb.Cin, jb.KH, jb.KW, jb.kind, jb.ci_count, jb.Kpad, jb.ncols,
                                       jb.nmajor, idx);
            jb.out[idx] = v;
            m = fmaxf(m, fabsf(v));
        }
        rng = jb.rng;
    }
    if (!rng) return;  // block-uniform
    __shared__ float red[4];
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) rng[lb] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (lb == 0)
        for (int i = nb + threadIdx.x; i < DCS_RANGE_PARTS; i += blockDim.x) rng[i] = 0.f;
}

// launch 2: the pre-split planes of a pack (dcs_pack_split_h3), or the hi / lo planes of a window pack
// (dcs_pack_weights_h3), each with the exponent of the range record launch 1 wrote
__global__ __launch_bounds__(256) void pack_batch2_kernel(const dcs_pack_job* __restrict__ jobs, int njobs) {
    const int j = pack_job_of(jobs, njobs, blockIdx.x, true);
    const dcs_pack_job& jb = jobs[j];
    const int lb = blockIdx.x - jb.p0, nb = jb.p1;
    if (jb.h3 == 2) {
        const int e = f16x3_exp(jb.h3_scratch, DCS_RANGE_PARTS);
        const float sc = __builtin_ldexpf(1.f, e);
        if (lb == 0 && threadIdx.x == 0) jb.h3_wexp[0] = e;
        const long long total = 16LL * jb.Cout * jb.Cin;
        const int K = subpix_K(jb.Cout, jb.Cin, jb.h3_flip);
        _Float16* oh = reinterpret_cast<_Float16*>(jb.h3_hi);
        _Float16* ol = reinterpret_cast<_Float16*>(jb.h3_lo);
        for (long long i = (long long)lb * 256 + threadIdx.x; i < total; i += (long long)nb * 256) {
            const int v = (int)(i / K);
            const float f = subpix_value(jb.w, jb.Cout, jb.Cin, jb.h3_flip, v, (int)(i - (long long)v * K)) * sc;
            const _Float16 h = (_Float16)f;
            oh[i] = h;
            ol[i] = (_Float16)(f - (float)h);
        }
    } else if (jb.h3) {
        const int e = f16x3_exp(jb.h3_scratch, DCS_RANGE_PARTS);
        const float sc = __builtin_ldexpf(1.f, e);
        if (lb == 0 && threadIdx.x == 0) jb.h3_wexp[0] = e;
        const int C = jb.h3_flip ? jb.Cout : jb.Cin;
        const int K = 9 * C;
        const long long total = (long long)jb.h3_ncols * K;
        _Float16* oh = reinterpret_cast<_Float16*>(jb.h3_hi);
        _Float16* ol = reinterpret_cast<_Float16*>(jb.h3_lo);
        for (long long idx = (long long)lb * 256 + threadIdx.x; idx < total; idx += (long long)nb * 256) {
            const int col = (int)(idx / K), k = (int)(idx - (long long)col * K);
            const int slice = k / 144, rem = k - slice * 144;
            const int tap = rem >> 4, c = slice * 16 + (rem & 15);
            const int ty = tap / 3, tx = tap - 3 * (tap / 3);
            float v = 0.f;
            if (!jb.h3_flip) {
                if (col < jb.Cout) v = jb.w[(((long long)col * jb.Cin + c) * 3 + ty) * 3 + tx];
            } else {
                if (col < jb.Cin) v = jb.w[(((long long)c * jb.Cin + col) * 3 + (2 - ty)) * 3 + (2 - tx)];
            }
            const float f = v * sc;
            const _Float16 h = (_Float16)f, l = (_Float16)(f - (float)h);
            oh[idx] = h;
            ol[idx] = l;
            if (jb.h3_flip) {  // the tap-major copy behind the planes (as conv_win.hip's pack_h3_kernel)
                const long long t = total + (long long)col * K + tap * C + c;
                oh[t] = h;
                ol[t] = l;
            }
        }
    } else {
        const float sc = __builtin_ldexpf(1.f, f16x3_exp(jb.rng, DCS_RANGE_PARTS));
        const long long total = (long long)jb.ncols * jb.Kpad;
        _Float16* out = reinterpret_cast<_Float16*>(jb.planes);
        for (long long i = (long long)lb * 256 + threadIdx.x; i < total; i += (long long)nb * 256) {
            const long long r = i / jb.Kpad, k = i - r * jb.Kpad;
            const float v = jb.out[i] * sc;
            const _Float16 h = (_Float16)v;
            out[2 * r * jb.Kpad + k] = h;
            out[(2 * r + 1) * jb.Kpad + k] = (_Float16)(v - (float)h);
        }
    }
}
}  // namespace
}  // namespace dcs

// block counts: about one element per thread, at most one block per range-record slot in launch 1 (a
// record's partial maxima then depend on the grid, their maximum - the only thing a consumer reads -
// does not, so every pack, exponent and plane equals the per-pack calls')
extern "C" int dcs_pack_plan(dcs_pack_job* jobs, int njobs, int* g1, int* g2) {
    if (!jobs || njobs <= 0 || !g1 || !g2) return fail(DCS_E_INVALID, "pack_plan: bad arguments");
    long long b = 0, p = 0;
    for (int i = 0; i < njobs; ++i) {
        dcs_pack_job& jb = jobs[i];
        if (!jb.w) return fail(DCS_E_INVALID, "pack_plan: job without weights");
        long long n1, n2 = 0, cap2 = 1;
        if (jb.h3 == 2) {
            if (!jb.h3_hi || !jb.h3_lo || !jb.h3_wexp || !jb.h3_scratch || !subpix_pack_ok(jb.Cout, jb.Cin, jb.h3_flip))
                return fail(DCS_E_INVALID, "pack_plan: window phase-kernel job (dcs_pack_subpix_h3's shape rules)");
            n1 = n2 = cdiv(16LL * jb.Cout * jb.Cin, 2048);  // dcs_pack_subpix_h3's launches
            cap2 = 256;
        } else if (jb.h3) {
            if (!jb.h3_hi || !jb.h3_lo || !jb.h3_wexp || !jb.h3_scratch || jb.Cout <= 0 || jb.Cin <= 0 ||
                (jb.h3_flip ? jb.Cout : jb.Cin) % 16 != 0 || jb.h3_ncols < (jb.h3_flip ? jb.Cin : jb.Cout))
                return fail(DCS_E_INVALID, "pack_plan: window job (3x3, reduction channels % 16 == 0)");
            n1 = cdiv((long long)jb.Cout * jb.Cin * 9, 2048);  // dcs_pack_weights_h3's range launch
            n2 = cdiv((long long)jb.h3_ncols * 9 * (jb.h3_flip ? jb.Cout : jb.Cin), 2048);
            cap2 = 256;
        } else {
            if (const char* err = pack_args_error(jb.w, jb.Cout, jb.Cin, jb.KH, jb.KW, jb.kind, jb.ci_count, jb.Kpad,
                                                  jb.ncols, jb.out))
                return fail(DCS_E_INVALID, err);
            n1 = cdiv((long long)jb.Kpad * jb.ncols, 256);
            if (jb.planes) {
                if (!jb.rng || !jb.nmajor) return fail(DCS_E_INVALID, "pack_plan: planes need an N-major pack with a range record");
                n2 = cdiv((long long)jb.ncols * jb.Kpad, 256);
                cap2 = 1024;
            }
        }
        n1 = n1 < 1 ? 1 : (n1 > DCS_RANGE_PARTS ? DCS_RANGE_PARTS : n1);
        n2 = n2 > cap2 ? cap2 : n2;
        jb.b0 = (int)b; jb.b1 = (int)n1;
        jb.p0 = (int)p; jb.p1 = (int)n2;
        b += n1;
        p += n2;
    }
    *g1 = (int)b;
    *g2 = (int)p;
    return 0;
}

extern "C" int dcs_pack_batch(const dcs_pack_job* jobs_dev, int njobs, int g1, int g2, void* stream) {
    if (!jobs_dev || njobs <= 0 || g1 <= 0 || g2 < 0) return fail(DCS_E_INVALID, "pack_batch: bad arguments");
    hipStream_t s = as_stream(stream);
    hipLaunchKernelGGL(pack_batch1_kernel, dim3((unsigned)g1), dim3(256), 0, s, jobs_dev, njobs);
    int e = check_launch("pack_batch1");
    if (e || g2 == 0) return e;
    hipLaunchKernelGGL(pack_batch2_kernel, dim3((unsigned)g2), dim3(256), 0, s, jobs_dev, njobs);
    return check_launch("pack_batch2");
}

namespace dcs {
int conv_rows_impl(const dcs_conv_desc* dp, const float* src, const float* src2, const float* wpack, const float* bias,
                   const float* psc, const float* psh, float* out, Part* parts, int* bm_used, void* stream,
                   int fold = 0);
// K splits of the ring-rows pass (fold 2) of a padded-grid data gradient: enough workgroups for two
// per CU, at least 4 k-tiles per split, at most 8 ring copies
int ring_ksplit(const dcs_conv_desc& d) {
    const long long M = (long long)d.N * (2 * d.Wo + 2 * (d.Ho - 2));
    const long long tiles = cdiv(M, 128) * cdiv(d.Co, d.Co > 64 ? 128 : 64);
    // a ring segment reads one kernel row or column (the masked walk of conv_rows_kernel, fold 2)
    const long long nkt = cdiv((long long)(d.KH > d.KW ? d.KH : d.KW) * d.Cs, 32);
    long long k = cdiv(512, tiles);
    if (k > 8) k = 8;
    while (k > 1 && nkt / k < 8) --k;
    return k < 1 ? 1 : (int)k;
}
}  // namespace dcs
namespace dcs {
int conv_rows_impl(const dcs_conv_desc* dp, const float* src, const float* src2, const float* wpack, const float* bias,
                   const float* psc, const float* psh, float* out, Part* parts, int* bm_used, void* stream,
                   int fold) {
    int e = validate(dp, true);
    if (e) return e;
    const dcs_conv_desc& d = *dp;
    if (!src || !wpack || !out) return fail(DCS_E_INVALID, "conv_rows: null pointer");
    if (d.pro_act != DCS_ACT_NONE && (!psc || !psh)) return fail(DCS_E_INVALID, "conv_rows: missing prologue");
    if (d.csplit < d.Cs && !src2) return fail(DCS_E_INVALID, "conv_rows: missing src2");
    const int BN = d.Co > 64 ? 128 : 64;
    if (d.ldb % BK != 0) return fail(DCS_E_INVALID, "conv_rows: ldb (packed K) must be a multiple of 32");
    if (d.parity && d.Cs % 16 != 0) return fail(DCS_E_INVALID, "conv_rows: parity rows need Cs % 16 == 0");
    if (d.Co % 4 != 0) return fail(DCS_E_INVALID, "conv_rows: Co must be a multiple of 4 (use the narrow path)");
    long long Mmax = 0;
    const int ncls = d.parity ? 4 : 1;
    for (int z = 0; z < ncls; ++z) {
        ClassGeom g = class_geom(d, z);
        long long M = (long long)g.My * g.Mx * d.N;
        if (M > Mmax) Mmax = M;
    }
    if (fold == 2) Mmax = (long long)d.N * (2 * d.Wo + 2 * (d.Ho - 2));  // ring rows only
    const int gx = (int)cdiv(Mmax, 128), gy = (int)cdiv(d.Co, BN);
    // ring rows (fold 2): K split over the grid's z so the few ring tiles fill the chip (each split
    // writes its own ring copy; reflect_ring_fold sums them)
    const int ksplit = fold == 2 ? ring_ksplit(d) : 1;
    const int fold_arg = fold | (ksplit > 1 ? ksplit << 2 : 0);
    dim3 grid((unsigned)(gx * gy * ncls * ksplit));
    if (bm_used) *bm_used = 128;
    const bool vec = vec_ok(dp, src);
    const bool v4 = !vec && vec4_ok(dp, src) && d.pro_act == DCS_ACT_NONE && !d.parity;
    const bool res_geom = d.Cs == 256 && d.Co == 256 && d.KH == 3 && d.KW == 3 && !d.parity && d.up == 1 &&
                          d.stride == 1 && d.pro_act == DCS_ACT_NONE && d.epi_act == DCS_ACT_NONE;
    // the residual-geometry kernels (TAG 1) run the slice-major K order, every other kernel the
    // tap-major one: the weights must have been packed to match
    const bool res = res_geom && d.korder == DCS_KORDER_SLICE;
    if (d.korder == DCS_KORDER_SLICE && !(res_geom && vec_ok(dp, src)))
        return fail(DCS_E_INVALID, "conv_rows: DCS_KORDER_SLICE is implemented for the 256-channel 3x3 stride-1 "
                                   "residual geometry with a vectorisable source");
    if (d.korder != DCS_KORDER_TAP && d.korder != DCS_KORDER_SLICE) return fail(DCS_E_INVALID, "conv_rows: bad korder");
    hipStream_t s = as_stream(stream);
    const bool x6f = d.mma == MMA_BF16X6 || d.mma == MMA_F16X3 || d.mma == MMA_F16;  // split-at-store pipelines
    const bool plain = DCS_TAG2 && d.pro_act == DCS_ACT_NONE && d.epi_act == DCS_ACT_NONE && d.pad_mode == DCS_PAD_ZERO &&
                       d.up == 1;
    const bool lrelu = DCS_TAG3 && d.pro_act == DCS_ACT_LRELU && d.epi_act == DCS_ACT_NONE && d.pad_mode == DCS_PAD_ZERO &&
                       d.up == 1;  // TAG 2 instances
#define DCS_ROWS_X6F(BM_, BN_, VEC_, TAG_, G)                                                                          \
    if (d.mma == MMA_F16X3)                                                                                          \
        hipLaunchKernelGGL((conv_rows_kernel<BM_, BN_, VEC_, TAG_, MMA_F16X3>), G, dim3(2 * BM_), 0, s, d, src, src2, \
                           wpack, bias, psc, psh, out, gxx, gy, parts, fold_arg);                                        \
    else if (d.mma == MMA_F16)                                                                                       \
        hipLaunchKernelGGL((conv_rows_kernel<BM_, BN_, VEC_, TAG_, MMA_F16>), G, dim3(2 * BM_), 0, s, d, src, src2,   \
                           wpack, bias, psc, psh, out, gxx, gy, parts, fold_arg);                                        \
    else                                                                                                             \
        hipLaunchKernelGGL((conv_rows_kernel<BM_, BN_, VEC_, TAG_, MMA_BF16X6>), G, dim3(2 * BM_), 0, s, d, src, src2, \
                           wpack, bias, psc, psh, out, gxx, gy, parts, fold_arg);
    if (vec && x6f && (BN == 128 || DCS_X6_BN64)) {  // x6 / f16x3: 128- or 64-column tiles
        // 256-row tiles where they divide the pixels evenly (the forward over whole 128 x 128
        // images); the 130 x 130 padded data gradient keeps 128-row tiles (measured: its partial
        // last dispatch round and zero-padded border rows make the big tile 7 % slower there)
        int gxx = gx;
        if (BN == 128 && res && DCS_X6_BM256 && Mmax % 256 == 0 && (!parts || ((long long)d.Ho * d.Wo) % 256 == 0)) {
            gxx = (int)cdiv(Mmax, 256);
            const dim3 grid2((unsigned)(gxx * gy));
            DCS_ROWS_X6F(256, 128, 1, 1, grid2)
            if (bm_used) *bm_used = 256;
        } else if (BN == 128 && res) { DCS_ROWS_X6F(128, 128, 1, 1, grid) }
        else if (BN == 128 && plain) { DCS_ROWS_X6F(128, 128, 1, 2, grid) }
        else if (BN == 128 && lrelu) { DCS_ROWS_X6F(128, 128, 1, 3, grid) }
        else if (BN == 128) { DCS_ROWS_X6F(128, 128, 1, 0, grid) }
        else if (plain) { DCS_ROWS_X6F(128, 64, 1, 2, grid) }
        else if (lrelu) { DCS_ROWS_X6F(128, 64, 1, 3, grid) }
        else { DCS_ROWS_X6F(128, 64, 1, 0, grid) }
        return check_launch("conv_rows");
    }
    if (v4 && x6f && DCS_X6_V4) {  // 4-channel stem / PatchGAN layer 0
        const int gxx = gx;
        const bool stem = DCS_TAG4 && d.KH == 7 && d.KW == 7 && d.Cs == 4 && d.stride == 1 && d.up == 1 && !d.parity &&
                          d.pad_mode == DCS_PAD_REFLECT && d.pro_act == DCS_ACT_NONE && d.epi_act == DCS_ACT_NONE;
        if (BN == 128 && plain) { DCS_ROWS_X6F(128, 128, 2, 2, grid) }
        else if (BN == 128) { DCS_ROWS_X6F(128, 128, 2, 0, grid) }
        else if (plain) { DCS_ROWS_X6F(128, 64, 2, 2, grid) }
        else if (stem) { DCS_ROWS_X6F(128, 64, 2, 4, grid) }
        else { DCS_ROWS_X6F(128, 64, 2, 0, grid) }
        return check_launch("conv_rows");
    }
#undef DCS_ROWS_X6F
    if (vec && d.mma == MMA_BF16 && res && BN == 128 && DCS_BF16P && DCS_BF16P_ROWS && d.ldb % 48 == 0) {
        // residual convs in the half-precision mode: the x6 pipeline, 48 k per barrier; 256-row
        // tiles where they divide the pixels (the forward)
        if (DCS_BF16P_BM256 && Mmax % 256 == 0 && (!parts || ((long long)d.Ho * d.Wo) % 256 == 0)) {
            const int gx2 = (int)cdiv(Mmax, 256);
            hipLaunchKernelGGL((conv_rows_kernel<256, 128, 1, 1, MMA_BF16P>), dim3((unsigned)(gx2 * gy)), dim3(512), 0, s,
                               d, src, src2, wpack, bias, psc, psh, out, gx2, gy, parts, fold_arg);
            if (bm_used) *bm_used = 256;
        } else {
            hipLaunchKernelGGL((conv_rows_kernel<128, 128, 1, 1, MMA_BF16P>), grid, dim3(NT), 0, s, d, src, src2, wpack,
                               bias, psc, psh, out, gx, gy, parts, fold_arg);
        }
        return check_launch("conv_rows");
    }
    const bool mma_ok = vec && (d.mma == MMA_BF16X3 || (d.mma == MMA_BF16 && d.Cs % 64 == 0 && d.ldb % 64 == 0));
    if (mma_ok) {  // bf16 operand modes (vectorised gathers; else exact f32)
#define DCS_ROWS_MMA(M)                                                                                              \
    if (BN == 128 && res) hipLaunchKernelGGL((conv_rows_kernel<128, 128, 1, 1, M>), grid, dim3(NT), 0, s, d, src, src2, wpack, bias, psc, psh, out, gx, gy, parts, fold_arg); \
    else if (BN == 128) hipLaunchKernelGGL((conv_rows_kernel<128, 128, 1, 0, M>), grid, dim3(NT), 0, s, d, src, src2, wpack, bias, psc, psh, out, gx, gy, parts, fold_arg);  \
    else hipLaunchKernelGGL((conv_rows_kernel<128, 64, 1, 0, M>), grid, dim3(NT), 0, s, d, src, src2, wpack, bias, psc, psh, out, gx, gy, parts, fold_arg);
        if (d.mma == MMA_BF16) { DCS_ROWS_MMA(MMA_BF16) } else { DCS_ROWS_MMA(MMA_BF16X3) }
#undef DCS_ROWS_MMA
        return check_launch("conv_rows");
    }
    if (BN == 128) {
        if (vec && res) hipLaunchKernelGGL((conv_rows_kernel<128, 128, 1, 1>), grid, dim3(NT), 0, s, d, src, src2, wpack, bias, psc, psh, out, gx, gy, parts, fold_arg);
        else if (vec) hipLaunchKernelGGL((conv_rows_kernel<128, 128, 1, 0>), grid, dim3(NT), 0, s, d, src, src2, wpack, bias, psc, psh, out, gx, gy, parts, fold_arg);
        else if (v4) hipLaunchKernelGGL((conv_rows_kernel<128, 128, 2, 0>), grid, dim3(NT), 0, s, d, src, src2, wpack, bias, psc, psh, out, gx, gy, parts, fold_arg);
        else hipLaunchKernelGGL((conv_rows_kernel<128, 128, 0, 0>), grid, dim3(NT), 0, s, d, src, src2, wpack, bias, psc, psh, out, gx, gy, parts, fold_arg);
    } else {
        if (vec) hipLaunchKernelGGL((conv_rows_kernel<128, 64, 1, 0>), grid, dim3(NT), 0, s, d, src, src2, wpack, bias, psc, psh, out, gx, gy, parts, fold_arg);
        else if (v4) hipLaunchKernelGGL((conv_rows_kernel<128, 64, 2, 0>), grid, dim3(NT), 0, s, d, src, src2, wpack, bias, psc, psh, out, gx, gy, parts, fold_arg);
        else hipLaunchKernelGGL((conv_rows_kernel<128, 64, 0, 0>), grid, dim3(NT), 0, s, d, src, src2, wpack, bias, psc, psh, out, gx, gy, parts, fold_arg);
    }
    return check_launch("conv_rows");
}
}  // namespace dcs

extern "C" int dcs_conv_rows(const dcs_conv_desc* dp, const float* src, const float* src2, const float* wpack,
                             const float* bias, const float* psc, const float* psh, float* out, void* stream) {
    return conv_rows_impl(dp, src, src2, wpack, bias, psc, psh, out, nullptr, nullptr, stream);
}

namespace {
// parity 0 rows, or the sub-pixel forward's four phases (each phase's rows per image % 128)
bool rows_stats_ok(const dcs_conv_desc& d) {
    if (d.parity == 1 || d.Co <= 4 || d.Co % 4 != 0) return false;
    const ClassGeom g = class_geom(d, 0);
    return ((long long)g.My * g.Mx) % 128 == 0;
}
}  // namespace

extern "C" size_t dcs_conv_rows_in_stats_parts_size(const dcs_conv_desc* dp) {
    if (!dp || !rows_stats_ok(*dp)) return 0;
    return (size_t)dp->N * ((size_t)dp->Ho * dp->Wo / 128) * dp->Co * sizeof(Part);  // phases: 4 x (Ho*Wo/4)
}

extern "C" int dcs_conv_rows_in_stats(const dcs_conv_desc* dp, const float* src, const float* src2, const float* wpack,
                                      const float* bias, const float* psc, const float* psh, float* out, void* parts,
                                      size_t parts_bytes, int* nchunk, void* stream) {
    if (!dp || !parts || !nchunk) return fail(DCS_E_INVALID, "conv_rows_in_stats: null pointer");
    if (!rows_stats_ok(*dp))
        return fail(DCS_E_INVALID, "conv_rows_in_stats: needs parity 0 / 2 rows, Co > 4 and rows per image % 128 == 0");
    if (parts_bytes < dcs_conv_rows_in_stats_parts_size(dp))
        return fail(DCS_E_WORKSPACE, "conv_rows_in_stats: parts buffer too small");
    int bm = 128;
    const int e = conv_rows_impl(dp, src, src2, wpack, bias, psc, psh, out, reinterpret_cast<Part*>(parts), &bm, stream);
    if (e) return e;
    const ClassGeom g = class_geom(*dp, 0);
    *nchunk = (int)((dp->parity == 2 ? 4 : 1) * (long long)g.My * g.Mx / bm);
    return 0;
}

namespace {
// sub-pixel wgrad: dW[co][ci][ty][tx] = sum over splits and the 4 phases z of the phase tap
// (jy, jx) whose weight sum contains (ty, tx): jy = ry ? (ty == 2) : (ty > 0), same for x.
__global__ void wgrad_subpixel_fold_kernel(const float* __restrict__ ws, int nsplit, int Co, int Cs,
                                           float* __restrict__ dw) {
    long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long total = (long long)Co * Cs * 9;
    if (idx >= total) return;
    const int t = (int)(idx % 9);
    const long long r = idx / 9;
    const int ci = (int)(r % Cs), co = (int)(r / Cs);
    const int ty = t / 3, tx = t - 3 * ty;
    const long long Ktot = 4ll * Cs, slab = (long long)Co * Ktot;
    float s = 0.f;
    for (int q = 0; q < nsplit; ++q)
#pragma unroll
        for (int z = 0; z < 4; ++z) {
            const int ry = z >> 1, rx = z & 1;
            const int jy = ry ? (ty == 2) : (ty > 0), jx = rx ? (tx == 2) : (tx > 0);
            s += ws[((long long)q * 4 + z) * slab + (long long)co * Ktot + (jy * 2 + jx) * Cs + ci];
        }
    dw[idx] = s;
}

// bf16x6 weight gradient (dcs_conv_desc.mma == DCS_MMA_BF16X6, vectorised sources, parity 0):
// dW[co][(tap, ci)] = sum_p dy[p][co] * src(p + tap)[ci] with each fp32 operand split into
// hi + mid + lo bf16 (split8x3) once, when the tile is staged, and the six products of the
// rows pass on v_mfma_f32_32x32x16_bf16.  Both operands are staged pixel-major
// ([16 pixels][128 columns] per plane, as they arrive from HBM); the MFMA wants 8 consecutive
// pixels of one column per lane, which ds_read_b64_tr_b16 delivers from that image (two 4-row
// transposed reads per fragment, cdna_hip_programming.md T10).  Row pitch 320 B: the 8-lane
// ds_write_b128 groups and the 32-lane transposed-read halves both cover all banks.  Same
// pixel walk, split partition (16-pixel tiles, twice the count) and partial slabs as
// conv_wgrad_kernel.
typedef short shortx4 __attribute__((ext_vector_type(4)));
typedef short shortx8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) shortx4 lds_shortx4;

// MMA == MMA_BF16P (the half-precision mode): the three planes hold three consecutive 16-pixel
// sub-tiles converted to bf16 (48 pixels per barrier, one product each, one accumulation level).
// V4: 4-channel NHWC source (the packed stem image + masks, PatchGAN layer 0): a thread's 8
// columns are channels 0-3 of two consecutive taps, one float4 gather each
template <int TAG, int MMA = MMA_BF16X6, bool V4 = false>
__global__ __launch_bounds__(NT, 2) void conv_wgrad_x6_kernel(
    const dcs_conv_desc din, const float* __restrict__ dy, const float* __restrict__ src,
    const float* __restrict__ psc, const float* __restrict__ psh, float* __restrict__ ws, int kt_per_split,
    int gn, int gm) {
    const dcs_conv_desc d = specialise<TAG>(din);
    constexpr bool H3 = MMA == MMA_F16X3 || MMA == MMA_F16;
    constexpr bool F1 = MMA == MMA_F16;  // f16: hi planes only, one product
    constexpr int NSUB = MMA == MMA_BF16P ? 3 : (H3 ? 2 : 1);  // 16-pixel sub-tiles per k-tile
    constexpr int NSLOT = H3 ? 2 * NSUB : 3;     // LDS planes per operand and buffer (f16x3: [hi|lo][sub])
    constexpr int BM = 128, BN = 128, BKP = 16;  // output channels x (tap, ci) columns x pixels per k-tile
    constexpr int WM = BM / 2, WN = BN / 2, IM = WM / 32, JN = WN / 32;
    constexpr int PITCH = 160;                   // bf16 per LDS row
    constexpr int KT2 = 8 / NSUB > 0 ? 8 / NSUB : 1;  // k-tiles per inner accumulation chain (128 pixels)
    __shared__ __attribute__((aligned(16))) __bf16 X[2 * NSLOT * 2 * BKP * PITCH];  // [A|B][plane][buf][pix][col]
    auto xo = [](int op, int pl, int buf, int pix, int col) {
        return (((op * NSLOT + pl) * 2 + buf) * BKP + pix) * PITCH + col;
    };
    float asc = 1.f, bsc = 1.f;  // f16x3 operand scales (dy, source) and the epilogue's exponent
    int eab = 0;
    if constexpr (H3) {
        const int ea = f16x3_exp(d.rng_a, d.rng_a_n), eb = f16x3_exp(d.rng_b, d.rng_b_n);
        asc = __builtin_ldexpf(1.f, ea);
        bsc = __builtin_ldexpf(1.f, eb);
        eab = -(ea + eb);
    }

    // sub-pixel descriptors (parity 2) run one GEMM per phase z, as in conv_wgrad_kernel
    const int ncls = d.parity == 2 ? 4 : 1;
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int ntile = L % gn;
    const int mtile = (L / gn) % gm;
    const int z = (L / (gn * gm)) % ncls;
    const int split = L / (gn * gm * ncls);
    const ClassGeom g = class_geom(d, z);
    const long long P = (long long)g.My * g.Mx * d.N;
    const int Ktot = g.ntaps * d.Cs;
    const int m0 = mtile * BM, n0 = ntile * BN;
    const long long nkt_all = (P + BKP - 1) / BKP;
    long long kt_beg = (long long)split * kt_per_split;
    long long kt_end = kt_beg + kt_per_split;
    if (kt_end > nkt_all) kt_end = nkt_all;
    // pixels of this split; BF16P / f16x3 walk them in NSUB x 16-pixel k-tiles numbered from 0
    const long long px_beg = kt_beg * BKP;
    const long long px_end = kt_end * BKP < P ? kt_end * BKP : P;
    if constexpr (NSUB > 1) {
        kt_end = px_end > px_beg ? (px_end - px_beg + NSUB * BKP - 1) / (NSUB * BKP) : 0;
        kt_beg = 0;
    }

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int kr = tid >> 4;        // the tile's pixel row this thread stages
    const int cc = (tid & 15) * 8;  // its 8 columns (of A: output channels; of B: (tap, ci))
    const int nb0 = n0 + cc;
    const bool bcol_ok = nb0 < Ktot;
    int bady = 0, badx = 0, bchan = 0;
    int bady1 = 0, badx1 = 0;  // V4: the second tap of the thread's columns
    bool bok1 = false;
    if constexpr (V4) {
        if (bcol_ok) {
            int bt;
            tap_decode(d, g, nb0 >> 2, bady, badx, bt);
            bok1 = (nb0 >> 2) + 1 < g.ntaps;
            if (bok1) tap_decode(d, g, (nb0 >> 2) + 1, bady1, badx1, bt);
        }
    } else if (bcol_ok) {  // the 8 columns share one tap (Cs % 16 == 0)
        const int j = nb0 / d.Cs;
        bchan = nb0 - j * d.Cs;
        int bt;
        tap_decode(d, g, j, bady, badx, bt);
    }
    const int Hv = d.Hs * d.up, Wv = d.Ws * d.up;
    const __amdgpu_buffer_rsrc_t rsrc = src_rsrc(src);
    int pn = 0, pqy = 0, pqx = 0;  // pixel of the next k-tile row this thread loads
    {
        const long long p = px_beg + kr;
        if (p < P) {
            const int per = g.My * g.Mx;
            pn = (int)(p / per);
            const int rem = (int)(p - (long long)pn * per);
            pqy = rem / g.Mx;
            pqx = rem - pqy * g.Mx;
        }
    }
    // Two register sets: the global loads of tile kt+2 are issued while tile kt is multiplied and
    // consumed (split + stored to LDS) only at the end of tile kt+1, two tiles of MFMA work later.
    float4 ra0[2 * NSUB], rb0[2 * NSUB], ra1[2 * NSUB], rb1[2 * NSUB];
    // Branch-free loads (buffer loads; out-of-range offsets read zeros) so that the wait for one
    // register set never waits for the other; the prologue affine is applied at the store.
    const __amdgpu_buffer_rsrc_t dyrsrc = src_rsrc(dy);
    int pro0[NSUB], pro1[NSUB];  // per set and sub-tile: pixel-image channel offset of the prologue, -1 = none
    auto load = [&](long long kt, float4 (&ra)[2 * NSUB], float4 (&rb)[2 * NSUB], int (&pro)[NSUB]) {
#pragma unroll
      for (int sub = 0; sub < NSUB; ++sub) {
        // 32-bit pixel / offset arithmetic: the dispatch requires dy < 2 GiB (dy_small), so every
        // pixel index and byte offset of dy fits (64-bit products here were ~10 % of the VALU)
        int p = NSUB > 1 ? (int)px_beg + (int)kt * (NSUB * BKP) + sub * BKP + kr : (int)kt * BKP + kr;
        const bool pok = p < (NSUB > 1 ? (int)px_end : (int)P);
        const int co = m0 + cc;
        if (d.parity == 2) p = (pn * d.Ho + 2 * pqy + g.ry) * d.Wo + 2 * pqx + g.rx;  // phase pixel
#pragma unroll
        for (int i = 0; i < 2; ++i)
            ra[2 * sub + i] = buf_load4(dyrsrc, (pok && co + 4 * i < d.Co) ? (p * d.Co + co + 4 * i) * 4 : OOB_OFF);
        // sub-pixel phases: the tap offsets already include the padding
        const int vy = d.parity == 2 ? pqy + bady : pqy * d.stride - d.pt + bady;
        const int vx = d.parity == 2 ? pqx + badx : pqx * d.stride - d.pl + badx;
        int sy, sx;
        const bool yok = map_coord_sel(vy, Hv, d.up, d.pad_mode, sy);
        const bool xok = map_coord_sel(vx, Wv, d.up, d.pad_mode, sx);
        const bool ok = pok && bcol_ok && yok && xok;
        const int off = ok ? (pn * (int)d.s_n + sy * (int)d.s_h + sx * (int)d.s_w + bchan) * 4 : OOB_OFF;
        if constexpr (V4) {
            const int vy1 = d.parity == 2 ? pqy + bady1 : pqy * d.stride - d.pt + bady1;
            const int vx1 = d.parity == 2 ? pqx + badx1 : pqx * d.stride - d.pl + badx1;
            int sy1, sx1;
            const bool ok1 = pok && bok1 && map_coord_sel(vy1, Hv, d.up, d.pad_mode, sy1) &&
                             map_coord_sel(vx1, Wv, d.up, d.pad_mode, sx1);
            rb[2 * sub] = buf_load4(rsrc, off);
            rb[2 * sub + 1] = buf_load4(rsrc, ok1 ? (pn * (int)d.s_n + sy1 * (int)d.s_h + sx1 * (int)d.s_w) * 4 : OOB_OFF);
        } else {
#pragma unroll
            for (int i = 0; i < 2; ++i) rb[2 * sub + i] = buf_load4(rsrc, off + 16 * i);
        }
        pro[sub] = (d.pro_act != DCS_ACT_NONE && ok) ? pn * d.Cs + bchan : -1;
        // next k-tile: at most one row wrap (the dispatch requires Mx >= BKP), as selects so the
        // tile body stays one basic block
        pqx += BKP;
        const bool wx = pqx >= g.Mx;
        pqx -= wx ? g.Mx : 0;
        pqy += wx ? 1 : 0;
        const bool wy = pqy == g.My;
        pqy = wy ? 0 : pqy;
        pn += wy ? 1 : 0;
      }
    };
    auto store = [&](int buf, const float4 (&ra)[2 * NSUB], const float4 (&rbl)[2 * NSUB], const int (&pro)[NSUB]) {
        if constexpr (H3) {  // slot = plane * NSUB + sub
#pragma unroll
            for (int sub = 0; sub < NSUB; ++sub) {
                f16x8 hi, lo;
                split8h(ra[2 * sub], ra[2 * sub + 1], asc, hi, lo);
                *reinterpret_cast<f16x8*>(X + xo(0, sub, buf, kr, cc)) = hi;
                if constexpr (!F1) *reinterpret_cast<f16x8*>(X + xo(0, NSUB + sub, buf, kr, cc)) = lo;
                float4 rb[2] = {rbl[2 * sub], rbl[2 * sub + 1]};
                if (d.pro_act != DCS_ACT_NONE && pro[sub] >= 0) {
#pragma unroll
                    for (int i = 0; i < 2; ++i)
                        rb[i] = affine_act4(rb[i], psc + pro[sub] + 4 * i, psh + pro[sub] + 4 * i, d.pro_act);
                }
                split8h(rb[0], rb[1], bsc, hi, lo);
                *reinterpret_cast<f16x8*>(X + xo(1, sub, buf, kr, cc)) = hi;
                if constexpr (!F1) *reinterpret_cast<f16x8*>(X + xo(1, NSUB + sub, buf, kr, cc)) = lo;
            }
            return;
        }
        if constexpr (MMA == MMA_BF16P) {
#pragma unroll
            for (int sub = 0; sub < NSUB; ++sub) {
                const floatx8 fa = {ra[2 * sub].x, ra[2 * sub].y, ra[2 * sub].z, ra[2 * sub].w,
                                    ra[2 * sub + 1].x, ra[2 * sub + 1].y, ra[2 * sub + 1].z, ra[2 * sub + 1].w};
                *reinterpret_cast<bf16x8*>(X + xo(0, sub, buf, kr, cc)) = __builtin_convertvector(fa, bf16x8);
                float4 rb[2] = {rbl[2 * sub], rbl[2 * sub + 1]};
                if (d.pro_act != DCS_ACT_NONE && pro[sub] >= 0) {
#pragma unroll
                    for (int i = 0; i < 2; ++i)
                        rb[i] = affine_act4(rb[i], psc + pro[sub] + 4 * i, psh + pro[sub] + 4 * i, d.pro_act);
                }
                const floatx8 fb = {rb[0].x, rb[0].y, rb[0].z, rb[0].w, rb[1].x, rb[1].y, rb[1].z, rb[1].w};
                *reinterpret_cast<bf16x8*>(X + xo(1, sub, buf, kr, cc)) = __builtin_convertvector(fb, bf16x8);
            }
            return;
        }
        bf16x8 hi, mid, lo;
        split8x3(ra[0], ra[1], hi, mid, lo);
        *reinterpret_cast<bf16x8*>(X + xo(0, 0, buf, kr, cc)) = hi;
        *reinterpret_cast<bf16x8*>(X + xo(0, 1, buf, kr, cc)) = mid;
        *reinterpret_cast<bf16x8*>(X + xo(0, 2, buf, kr, cc)) = lo;
        float4 rb[2] = {rbl[0], rbl[1]};
        if (d.pro_act != DCS_ACT_NONE && pro[0] >= 0) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
                rb[i] = affine_act4(rb[i], psc + pro[0] + 4 * i, psh + pro[0] + 4 * i, d.pro_act);
        }
        split8x3(rb[0], rb[1], hi, mid, lo);
        *reinterpret_cast<bf16x8*>(X + xo(1, 0, buf, kr, cc)) = hi;
        *reinterpret_cast<bf16x8*>(X + xo(1, 1, buf, kr, cc)) = mid;
        *reinterpret_cast<bf16x8*>(X + xo(1, 2, buf, kr, cc)) = lo;
    };
    // transposed fragment of columns col0 .. col0+31, all 16 pixels: lane (r, h) receives
    // pixels 8h .. 8h+7 of column col0 + r.  In a 16-lane group, lane 4q+p addresses pixel
    // row q (+4 for the second read), columns 4p .. 4p+3.
    const int g16 = lane >> 4;
    const int rpix = 8 * (g16 >> 1) + ((lane & 15) >> 2);
    const int rcol = 16 * (g16 & 1) + 4 * (lane & 3);
    auto frag16 = [&](int op, int pl, int buf, int col0) {
        const __bf16* p0 = X + xo(op, pl, buf, rpix, col0 + rcol);
        const shortx4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_shortx4*)(p0));
        const shortx4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_shortx4*)(p0 + 4 * PITCH));
        return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
    };
    auto frag = [&](int op, int pl, int buf, int col0) { return __builtin_bit_cast(bf16x8, frag16(op, pl, buf, col0)); };
    auto fragh = [&](int op, int pl, int buf, int col0) { return __builtin_bit_cast(f16x8, frag16(op, pl, buf, col0)); };

    floatx16 acc[IM][JN], t[IM][JN];
#pragma unroll
    for (int i = 0; i < IM; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) { acc[i][j][r] = 0.f; t[i][j][r] = 0.f; }

    auto tile = [&](long long kt, float4 (&nra)[2 * NSUB], float4 (&nrb)[2 * NSUB], int (&npro)[NSUB],
                    const float4 (&ora)[2 * NSUB], const float4 (&orb)[2 * NSUB], const int (&opro)[NSUB]) {
        const int cur = (int)((kt - kt_beg) & 1);
        if constexpr (H3) {
#pragma unroll
            for (int sub = 0; sub < NSUB; ++sub) {
                f16x8 ah[IM], al[IM], bh[JN], bl[JN];
#pragma unroll
                for (int i = 0; i < IM; ++i) {
                    ah[i] = fragh(0, sub, cur, wm * WM + i * 32);
                    if constexpr (!F1) al[i] = fragh(0, NSUB + sub, cur, wm * WM + i * 32);
                }
#pragma unroll
                for (int j = 0; j < JN; ++j) {
                    bh[j] = fragh(1, sub, cur, wn * WN + j * 32);
                    if constexpr (!F1) bl[j] = fragh(1, NSUB + sub, cur, wn * WN + j * 32);
                }
                if (sub == 0) load(kt + 2, nra, nrb, npro);  // unconditional (see below)
#pragma unroll
                for (int i = 0; i < IM; ++i)
#pragma unroll
                    for (int j = 0; j < JN; ++j) {
                        if constexpr (!F1) {
                            t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], t[i][j], 0, 0, 0);
                            t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], t[i][j], 0, 0, 0);
                        }
                        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], t[i][j], 0, 0, 0);
                    }
            }
            store(cur ^ 1, ora, orb, opro);
            if constexpr (DCS_WGRAD_SGB > 0) {
                __builtin_amdgcn_sched_group_barrier(0x100, 2 * (IM + JN) * (F1 ? 1 : 2) * NSUB, 0);  // DS read
#pragma unroll
                for (int i = 0; i < IM * JN * (F1 ? 1 : 3) * NSUB; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, DCS_WGRAD_SGB, 0);
                }
                __builtin_amdgcn_sched_group_barrier(0x200, (F1 ? 2 : 4) * NSUB, 0);  // DS write
            }
            const long long rel = kt - kt_beg;
            if ((rel % KT2) == KT2 - 1 || kt + 1 == kt_end) {
#pragma unroll
                for (int i = 0; i < IM; ++i)
#pragma unroll
                    for (int j = 0; j < JN; ++j) {
                        acc[i][j] += t[i][j];
#pragma unroll
                        for (int r = 0; r < 16; ++r) t[i][j][r] = 0.f;
                    }
            }
            __syncthreads();
            return;
        }
        if constexpr (MMA == MMA_BF16P) {
#pragma unroll
            for (int sub = 0; sub < NSUB; ++sub) {
                bf16x8 fa[IM], fb[JN];
#pragma unroll
                for (int i = 0; i < IM; ++i) fa[i] = frag(0, sub, cur, wm * WM + i * 32);
#pragma unroll
                for (int j = 0; j < JN; ++j) fb[j] = frag(1, sub, cur, wn * WN + j * 32);
                if (sub == 0) load(kt + 2, nra, nrb, npro);
#pragma unroll
                for (int i = 0; i < IM; ++i)
#pragma unroll
                    for (int j = 0; j < JN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
            }
            store(cur ^ 1, ora, orb, opro);
            __syncthreads();
            return;
        }
        bf16x8 ah[IM], am[IM], al[IM], bh[JN], bm[JN], bl[JN];
#pragma unroll
        for (int i = 0; i < IM; ++i) {
            const int c0 = wm * WM + i * 32;
            ah[i] = frag(0, 0, cur, c0);
            am[i] = frag(0, 1, cur, c0);
            al[i] = frag(0, 2, cur, c0);
        }
#pragma unroll
        for (int j = 0; j < JN; ++j) {
            const int c0 = wn * WN + j * 32;
            bh[j] = frag(1, 0, cur, c0);
            bm[j] = frag(1, 1, cur, c0);
            bl[j] = frag(1, 2, cur, c0);
        }
        load(kt + 2, nra, nrb, npro);  // unconditional (past the range: zeros or unused), so the
                                        // vmcnt bookkeeping stays exact across the loop
#pragma unroll
        for (int i = 0; i < IM; ++i)
#pragma unroll
            for (int j = 0; j < JN; ++j) {  // smallest terms first, as in the rows pass
                t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bm[j], t[i][j], 0, 0, 0);
                t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], t[i][j], 0, 0, 0);
                t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], t[i][j], 0, 0, 0);
                t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bh[j], t[i][j], 0, 0, 0);
                t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bm[j], t[i][j], 0, 0, 0);
                t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], t[i][j], 0, 0, 0);
            }
        // stage tile kt+1 before the chain fold, unconditionally (past the range: a buffer nobody
        // reads again), with the split spread over this tile's MFMAs
        store(cur ^ 1, ora, orb, opro);
        if constexpr (DCS_WGRAD_SGB > 0) {
            __builtin_amdgcn_sched_group_barrier(0x100, 24, 0);  // DS read (transposed fragments)
#pragma unroll
            for (int i = 0; i < IM * JN * 6; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, DCS_WGRAD_SGB, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x200, 6, 0);  // DS write
        }
        const long long rel = kt - kt_beg;
        if ((rel % KT2) == KT2 - 1 || kt + 1 == kt_end) {
#pragma unroll
            for (int i = 0; i < IM; ++i)
#pragma unroll
                for (int j = 0; j < JN; ++j) {
                    acc[i][j] += t[i][j];
#pragma unroll
                    for (int r = 0; r < 16; ++r) t[i][j][r] = 0.f;
                }
        }
        __syncthreads();
    };
    if (kt_beg < kt_end) {
        load(kt_beg, ra0, rb0, pro0);
        store(0, ra0, rb0, pro0);
        load(kt_beg + 1, ra1, rb1, pro1);
    }
    __syncthreads();
    for (long long kt = kt_beg; kt < kt_end; kt += 2) {
        tile(kt, ra0, rb0, pro0, ra1, rb1, pro1);  // tile kt+1 waits in set 1; tile kt+2 lands in set 0
        if (kt + 1 < kt_end) tile(kt + 1, ra1, rb1, pro1, ra0, rb0, pro0);
    }

    if constexpr (H3) {  // undo the operand scales (exact powers of two)
#pragma unroll
        for (int i = 0; i < IM; ++i)
#pragma unroll
            for (int j = 0; j < JN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = __builtin_ldexpf(acc[i][j][r], eab);
    }
    float* slab = ws + ((long long)split * ncls + z) * d.Co * Ktot;
    const int l32 = lane & 31;
#pragma unroll
    for (int j = 0; j < JN; ++j) {
        const int col = n0 + wn * WN + j * 32 + l32;
        if (col >= Ktot) continue;
#pragma unroll
        for (int i = 0; i < IM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                if (row < d.Co) slab[(long long)row * Ktot + col] = acc[i][j][r];
            }
    }
}

struct WgradPlan {
    int BM, BN, nsplit, kt_per_split;
    long long Ktot;
};
WgradPlan wgrad_plan(const dcs_conv_desc& d) {
    WgradPlan p;
    ClassGeom g = class_geom(d, 0);
    long long P = (long long)g.My * g.Mx * d.N;
    p.Ktot = (long long)g.ntaps * d.Cs;
    p.BM = d.Co > 64 ? 128 : 64;
    p.BN = 128;
    const long long tiles = cdiv(d.Co, p.BM) * cdiv(p.Ktot, p.BN) * (d.parity == 2 ? 4 : 1);
    const long long nkt = cdiv(P, BK);
    // Workgroups run in rounds of `slots` (256 CUs x blocks per CU: 3 for the vectorised BM=64
    // kernel, else 2, by VGPR budget) and every block streams the same number of k-tiles, so a grid of
    // tiles*nsplit blocks costs ceil(blocks/slots) rounds.  Pick the split count that
    // fills the rounds best (>= 8 k-tiles per split, <= 256 splits), preferring fewer splits
    // (less partial-slab traffic) among equally full choices.
    const bool vec_shape = (d.Cs % 16 == 0 || d.Cs == 4) && d.s_c == 1 && d.csplit == d.Cs;  // minus alignment
    const long long slots = 256 * (p.BM == 64 && vec_shape ? 3 : 2);
    long long maxs = cdiv(nkt, 8);
    if (maxs > 256) maxs = 256;
    if (maxs < 1) maxs = 1;
    long long best = 1;
    double best_score = -1.0;
    for (long long ns = 1; ns <= maxs; ++ns) {
        const long long kps = cdiv(nkt, ns);
        const long long nsr = cdiv(nkt, kps);            // splits actually used
        const long long blocks = tiles * nsr;
        const long long rounds = cdiv(blocks, slots);
        // time ~ rounds * k-tiles per block (+ a small per-block epilogue cost)
        const double cost = (double)rounds * (double)(kps + 2);
        const double score = 1.0 / cost;
        if (score > best_score * 1.0001) { best_score = score; best = ns; }
    }
    p.kt_per_split = (int)cdiv(nkt, best);
    p.nsplit = (int)cdiv(nkt, p.kt_per_split);
    return p;
}
}  // namespace

// conv_win.hip: the f16x3 window weight gradient of the residual 3x3 convs
namespace dcs {
#ifndef DCS_X6_F16_TAG3  // the f16 PatchGAN weight gradients on the LeakyReLU-prologue instance (TAG 3) as in f16x3,
                         // not the generic one: bit-identical, f16 step 128.26 -> 127.73 ms (profiles/r06/ab/r06aq_*)
#define DCS_X6_F16_TAG3 1
#endif
bool wgrad_win_check(const dcs_conv_desc& d);
size_t wgrad_win_workspace_size(const dcs_conv_desc& d);
int wgrad_win_launch(const dcs_conv_desc& d, const float* dy, const float* x, float* ws, hipStream_t s);
// conv_subpix.hip: the f16x3 window weight gradients of the up- and stride-2 convolutions (a VARIANT build
// with EXTRA=-DDCS_SUBPIX_WGRAD=0 runs the x6 kernels instead, for A/B)
#ifndef DCS_SUBPIX_WGRAD
#define DCS_SUBPIX_WGRAD 1
#endif
bool subpix_wgrad_check(const dcs_conv_desc& d);
size_t subpix_wgrad_workspace_size(const dcs_conv_desc& d);
int subpix_wgrad_launch(const dcs_conv_desc& d, const float* dy, const float* x, float* ws, hipStream_t s);
// conv_subpix.hip: the f16x3 window weight gradient of the stride-2 convolutions (3x3 and 4x4)
bool s2_wgrad_check(const dcs_conv_desc& d);
size_t s2_wgrad_workspace_size(const dcs_conv_desc& d);
int s2_wgrad_launch(const dcs_conv_desc& d, const float* dy, const float* x, const float* psc, const float* psh,
                    float* ws, hipStream_t s);
}  // namespace dcs

extern "C" size_t dcs_conv_wgrad_workspace_size(const dcs_conv_desc* dp) {
    if (!dp) return 0;
    WgradPlan p = wgrad_plan(*dp);
    size_t n = (size_t)p.nsplit * (dp->parity == 2 ? 4 : 1) * dp->Co * p.Ktot * sizeof(float);
    if (DCS_WGRAD_WIN && wgrad_win_check(*dp)) {
        const size_t nw = wgrad_win_workspace_size(*dp);
        n = nw > n ? nw : n;
    }
    if (DCS_SUBPIX_WGRAD && subpix_wgrad_check(*dp)) {
        const size_t nw = subpix_wgrad_workspace_size(*dp);
        n = nw > n ? nw : n;
    }
    if (DCS_SUBPIX_WGRAD && s2_wgrad_check(*dp)) {
        const size_t nw = s2_wgrad_workspace_size(*dp);
        n = nw > n ? nw : n;
    }
    return n;
}

extern "C" int dcs_conv_wgrad(const dcs_conv_desc* dp, const float* dy, const float* x, const float* x2,
                              const float* psc, const float* psh, float* dw, void* ws, size_t ws_bytes,
                              void* stream) {
    int e = validate(dp, false);
    if (e) return e;
    const dcs_conv_desc& d = *dp;
    if (d.parity == 1) return fail(DCS_E_INVALID, "conv_wgrad: describe the forward conv (parity 0 or 2)");
    if (!dy || !x || !dw || !ws) return fail(DCS_E_INVALID, "conv_wgrad: null pointer");
    if (d.Co % 4 != 0) return fail(DCS_E_INVALID, "conv_wgrad: Co must be a multiple of 4");
    if (ws_bytes < dcs_conv_wgrad_workspace_size(dp)) return fail(DCS_E_WORKSPACE, "conv_wgrad: workspace too small");
    WgradPlan p = wgrad_plan(d);
    const int gn = (int)cdiv(p.Ktot, p.BN), gm = (int)cdiv(d.Co, p.BM);
    const int ncls = d.parity == 2 ? 4 : 1;
    dim3 grid((unsigned)(gn * gm * p.nsplit * ncls));
    const bool vec = vec_ok(dp, x);
    if (d.parity == 2 && !vec) return fail(DCS_E_INVALID, "conv_wgrad: sub-pixel rows need a vectorisable source");
    hipStream_t s = as_stream(stream);
    float* w = reinterpret_cast<float*>(ws);
    if (DCS_WGRAD_WIN && wgrad_win_check(d)) {  // f16x3 residual geometry: the rolling-window kernel
        const int ns = wgrad_win_launch(d, dy, x, w, s);
        if (ns < 0) return -ns;
        const long long total = (long long)d.Co * 9 * d.Cs;
        hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s, w, ns, d.Co, d.Cs,
                           3, 3, d.Cs, dw);
        return check_launch("conv_wgrad_reduce");
    }
    if (DCS_SUBPIX_WGRAD && subpix_wgrad_check(d) && !x2) {  // f16x3 up-convolution: the rolling-window phase kernel
        const int ns = subpix_wgrad_launch(d, dy, x, w, s);
        if (ns < 0) return -ns;
        const long long tot9 = (long long)d.Co * d.Cs * 9;
        hipLaunchKernelGGL(wgrad_subpixel_fold_kernel, dim3((unsigned)cdiv(tot9, 256)), dim3(256), 0, s, w, ns, d.Co,
                           d.Cs, dw);
        return check_launch("wgrad_subpixel_fold");
    }
    if (DCS_SUBPIX_WGRAD && s2_wgrad_check(d) && !x2) {  // f16x3 stride-2 conv: the rolling class-window kernel
        const int ns = s2_wgrad_launch(d, dy, x, psc, psh, w, s);
        if (ns < 0) return -ns;
        const long long total = (long long)d.Co * d.KH * d.KW * d.Cs;
        hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s, w, ns, d.Co, d.Cs,
                           d.KH, d.KW, d.Cs, dw);
        return check_launch("conv_wgrad_reduce");
    }
    const bool res = d.Cs == 256 && d.KH == 3 && d.KW == 3 && d.up == 1 && d.stride == 1 && !d.parity &&
                     d.pro_act == DCS_ACT_NONE && d.epi_act == DCS_ACT_NONE;
    const bool v4 = !vec && vec4_ok(dp, x) && d.pro_act == DCS_ACT_NONE && !d.parity;
    const bool dy_small = (long long)d.N * d.Ho * d.Wo * d.Co * 4 < (long long)OOB_OFF - 64;
    // (the bf16 and bf16x3 modes run the bf16x6 weight gradient: a bf16 MFMA weight gradient measured
    // slower than the exact f32 one at every layer, its 8-pixel walk per thread VALU bound)
    if (DCS_WGRAD_X6_V4 && (d.mma == MMA_F16X3 || d.mma == MMA_F16) && v4 && d.Cs == 4 && !d.parity && dy_small &&
               d.pro_act == DCS_ACT_NONE && (p.BM == 128 || d.Co == 64) && class_geom(d, 0).Mx >= 16) {
        // 4-channel sources (stem, PatchGAN layer 0) on the fp16 x6 pipeline: two taps per thread's 8 columns
        const bool plain = DCS_TAG2 && d.pad_mode == DCS_PAD_ZERO && d.up == 1;
        if (d.mma == MMA_F16X3) {
            if (plain) hipLaunchKernelGGL((conv_wgrad_x6_kernel<2, MMA_F16X3, true>), grid, dim3(NT), 0, s, d, dy, x, psc, psh, w, 2 * p.kt_per_split, gn, gm);
            else hipLaunchKernelGGL((conv_wgrad_x6_kernel<0, MMA_F16X3, true>), grid, dim3(NT), 0, s, d, dy, x, psc, psh, w, 2 * p.kt_per_split, gn, gm);
        } else {
            if (plain) hipLaunchKernelGGL((conv_wgrad_x6_kernel<2, MMA_F16, true>), grid, dim3(NT), 0, s, d, dy, x, psc, psh, w, 2 * p.kt_per_split, gn, gm);
            else hipLaunchKernelGGL((conv_wgrad_x6_kernel<0, MMA_F16, true>), grid, dim3(NT), 0, s, d, dy, x, psc, psh, w, 2 * p.kt_per_split, gn, gm);
        }
    } else if (d.mma != MMA_F32 && vec && dy_small && (p.BM == 128 || (d.Co == 64 && DCS_WGRAD_X6_CO64 && (d.mma == MMA_F16X3 || d.mma == MMA_F16))) &&
               d.parity != 1 && class_geom(d, 0).Mx >= 16 && DCS_WGRAD_X6) {  // one row wrap per tile
        // 16-pixel tiles: twice the tile count per split, the same pixel ranges and slabs.  (The
        // 64-output-channel layers could run the 128-row tile half masked: slower than f32.)
        const bool plain = DCS_TAG2 && d.pro_act == DCS_ACT_NONE && d.pad_mode == DCS_PAD_ZERO && d.up == 1;
        const bool lrelu = DCS_TAG3 && d.pro_act == DCS_ACT_LRELU && d.pad_mode == DCS_PAD_ZERO && d.up == 1;
        if (d.mma == MMA_F16X3) {  // f16x3: two 16-pixel sub-tiles per barrier
            if (res) hipLaunchKernelGGL((conv_wgrad_x6_kernel<1, MMA_F16X3>), grid, dim3(NT), 0, s, d, dy, x, psc, psh, w, 2 * p.kt_per_split, gn, gm);
            else if (plain) hipLaunchKernelGGL((conv_wgrad_x6_kernel<2, MMA_F16X3>), grid, dim3(NT), 0, s, d, dy, x, psc, psh, w, 2 * p.kt_per_split, gn, gm);
            else if (lrelu) hipLaunchKernelGGL((conv_wgrad_x6_kernel<3, MMA_F16X3>), grid, dim3(NT), 0, s, d, dy, x, psc, psh, w, 2 * p.kt_per_split, gn, gm);
            else hipLaunchKernelGGL((conv_wgrad_x6_kernel<0, MMA_F16X3>), grid, dim3(NT), 0, s, d, dy, x, psc, psh, w, 2 * p.kt_per_split, gn, gm);
        } else if (d.mma == MMA_F16) {  // f16: the same pipeline, one product
            if (res) hipLaunchKernelGGL((conv_wgrad_x6_kernel<1, MMA_F16>), grid, dim3(NT), 0, s, d, dy, x, psc, psh, w, 2 * p.kt_per_split, gn, gm);
            else if (plain) hipLaunchKernelGGL((conv_wgrad_x6_kernel<2, MMA_F16>), grid, dim3(NT), 0, s, d, dy, x, psc, psh, w, 2 * p.kt_per_split, gn, gm);
            else if (lrelu && DCS_X6_F16_TAG3) hipLaunchKernelGGL((conv_wgrad_x6_kernel<3, MMA_F16>), grid, dim3(NT), 0, s, d, dy, x, psc, psh, w, 2 * p.kt_per_split, gn, gm);
            else hipLaunchKernelGGL((conv_wgrad_x6_kernel<0, MMA_F16>), grid, dim3(NT), 0, s, d, dy, x, psc, psh, w, 2 * p.kt_per_split, gn, gm);
        } else if (d.mma == MMA_BF16 && DCS_BF16P) {  // half precision: one product, 48 pixels per barrier
            if (res) hipLaunchKernelGGL((conv_wgrad_x6_kernel<1, MMA_BF16P>), grid, dim3(NT), 0, s, d, dy, x, psc, psh, w, 2 * p.kt_per_split, gn, gm);
            else hipLaunchKernelGGL((conv_wgrad_x6_kernel<0, MMA_BF16P>), grid, dim3(NT), 0, s, d, dy, x, psc, psh, w, 2 * p.kt_per_split, gn, gm);
        } else if (res) hipLaunchKernelGGL((conv_wgrad_x6_kernel<1>), grid, dim3(NT), 0, s, d, dy, x, psc, psh, w, 2 * p.kt_per_split, gn, gm);
        else hipLaunchKernelGGL((conv_wgrad_x6_kernel<0>), grid, dim3(NT), 0, s, d, dy, x, psc, psh, w, 2 * p.kt_per_split, gn, gm);
    } else if (p.BM == 128) {
        if (vec && res) hipLaunchKernelGGL((conv_wgrad_kernel<128, 128, 1, 1>), grid, dim3(NT), 0, s, d, dy, x, x2, psc, psh, w, p.kt_per_split, gn, gm);
        else if (vec) hipLaunchKernelGGL((conv_wgrad_kernel<128, 128, 1, 0>), grid, dim3(NT), 0, s, d, dy, x, x2, psc, psh, w, p.kt_per_split, gn, gm);
        else if (v4) hipLaunchKernelGGL((conv_wgrad_kernel<128, 128, 2, 0>), grid, dim3(NT), 0, s, d, dy, x, x2, psc, psh, w, p.kt_per_split, gn, gm);
        else hipLaunchKernelGGL((conv_wgrad_kernel<128, 128, 0, 0>), grid, dim3(NT), 0, s, d, dy, x, x2, psc, psh, w, p.kt_per_split, gn, gm);
    } else {
        if (vec) hipLaunchKernelGGL((conv_wgrad_kernel<64, 128, 1, 0>), grid, dim3(NT), 0, s, d, dy, x, x2, psc, psh, w, p.kt_per_split, gn, gm);
        else if (v4) hipLaunchKernelGGL((conv_wgrad_kernel<64, 128, 2, 0>), grid, dim3(NT), 0, s, d, dy, x, x2, psc, psh, w, p.kt_per_split, gn, gm);
        else hipLaunchKernelGGL((conv_wgrad_kernel<64, 128, 0, 0>), grid, dim3(NT), 0, s, d, dy, x, x2, psc, psh, w, p.kt_per_split, gn, gm);
    }
    e = check_launch("conv_wgrad");
    if (e) return e;
    if (d.parity == 2) {
        const long long tot9 = (long long)d.Co * d.Cs * 9;
        hipLaunchKernelGGL(wgrad_subpixel_fold_kernel, dim3((unsigned)cdiv(tot9, 256)), dim3(256), 0, s, w, p.nsplit,
                           d.Co, d.Cs, dw);
        return check_launch("wgrad_subpixel_fold");
    }
    long long total = (long long)d.Co * p.Ktot;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s, w, p.nsplit, d.Co,
                       d.Cs, d.KH, d.KW, d.cw > 0 ? d.cw : d.Cs, dw);
    return check_launch("conv_wgrad_reduce");
}

extern "C" int dcs_conv_rows_narrow(const dcs_conv_desc* dp, const float* src, const float* src2,
                                    const float* wpack, const float* bias, const float* psc, const float* psh,
                                    float* out, void* stream) {
    int e = validate(dp, true);
    if (e) return e;
    const dcs_conv_desc& d = *dp;
    if (!src || !wpack || !out) return fail(DCS_E_INVALID, "conv_rows_narrow: null pointer");
    if (d.Co > 4) return fail(DCS_E_INVALID, "conv_rows_narrow: Co must be <= 4");
    if (d.ldb < d.Co) return fail(DCS_E_INVALID, "conv_rows_narrow: ldb < Co");
    const int NO = d.Co <= 1 ? 1 : 4;
    const int Krows = d.KH * d.KW * d.Cs;
    size_t lds = (size_t)Krows * NO * sizeof(float);
    if (lds > 64 * 1024) return fail(DCS_E_INVALID, "conv_rows_narrow: weights exceed 64 KiB of LDS");
    long long Mmax = 0;
    const int ncls = d.parity ? 4 : 1;
    for (int z = 0; z < ncls; ++z) {
        ClassGeom g = class_geom(d, z);
        long long M = (long long)g.My * g.Mx * d.N;
        if (M > Mmax) Mmax = M;
    }
    hipStream_t s = as_stream(stream);
    if (narrow_small_ok(d, src)) return launch_narrow_rows_small(d, src, wpack, bias, psc, psh, out, s);
    if (narrow_tiled_ok(d, src)) return launch_narrow_rows_tiled(d, src, wpack, bias, psc, psh, out, s);
    dim3 grid((unsigned)cdiv(Mmax, 256), ncls);
    const bool vec = vec_ok(dp, src);
    // the kernel reads wp[k*ldb + o] for o < NO: ldb must cover NO columns
    if (d.ldb < NO) return fail(DCS_E_INVALID, "conv_rows_narrow: ldb must be >= 4 when Co > 1");
    if (NO == 1) {
        if (vec) hipLaunchKernelGGL((conv_rows_narrow_kernel<1, true>), grid, dim3(256), lds, s, d, src, src2, wpack, bias, psc, psh, out, Krows);
        else hipLaunchKernelGGL((conv_rows_narrow_kernel<1, false>), grid, dim3(256), lds, s, d, src, src2, wpack, bias, psc, psh, out, Krows);
    } else {
        if (vec) hipLaunchKernelGGL((conv_rows_narrow_kernel<4, true>), grid, dim3(256), lds, s, d, src, src2, wpack, bias, psc, psh, out, Krows);
        else hipLaunchKernelGGL((conv_rows_narrow_kernel<4, false>), grid, dim3(256), lds, s, d, src, src2, wpack, bias, psc, psh, out, Krows);
    }
    return check_launch("conv_rows_narrow");
}

namespace {
long long narrow_pix_per_split(const dcs_conv_desc& d, int* nsplit) {
    ClassGeom g = class_geom(d, 0);
    long long P = (long long)g.My * g.Mx * d.N;
    long long Ktot = (long long)g.ntaps * d.Cs;
    long long kb = cdiv(Ktot, 256);
    long long want = cdiv(2048, kb);
    long long ns = want < P ? want : P;
    if (ns < 1) ns = 1;
    if (ns > 4096) ns = 4096;
    long long pps = cdiv(P, ns);
    *nsplit = (int)cdiv(P, pps);
    return pps;
}
}  // namespace

extern "C" size_t dcs_conv_wgrad_narrow_workspace_size(const dcs_conv_desc* dp) {
    if (!dp) return 0;
    int ns;
    narrow_pix_per_split(*dp, &ns);
    ClassGeom g = class_geom(*dp, 0);
    size_t naive = (size_t)ns * dp->Co * g.ntaps * dp->Cs * sizeof(float);
    size_t tiled = (size_t)narrow_wgrad_tiled_blocks(*dp) * g.ntaps * dp->Cs * sizeof(float);
    return naive > tiled ? naive : tiled;
}

extern "C" int dcs_conv_wgrad_narrow(const dcs_conv_desc* dp, const float* dy, const float* x, const float* x2,
                                     const float* psc, const float* psh, float* dw, void* ws, size_t ws_bytes,
                                     void* stream) {
    int e = validate(dp, false);
    if (e) return e;
    const dcs_conv_desc& d = *dp;
    if (d.parity || d.Co > 4) return fail(DCS_E_INVALID, "conv_wgrad_narrow: forward conv with Co <= 4 expected");
    if (!dy || !x || !dw || !ws) return fail(DCS_E_INVALID, "conv_wgrad_narrow: null pointer");
    if (ws_bytes < dcs_conv_wgrad_narrow_workspace_size(dp)) return fail(DCS_E_WORKSPACE, "conv_wgrad_narrow: workspace too small");
    int ns;
    long long pps = narrow_pix_per_split(d, &ns);
    ClassGeom g = class_geom(d, 0);
    long long Ktot = (long long)g.ntaps * d.Cs;
    dim3 grid((unsigned)cdiv(Ktot, 256), ns);
    hipStream_t s = as_stream(stream);
    float* w = reinterpret_cast<float*>(ws);
    if (narrow_wgrad_tiled_ok(d, x)) {
        e = launch_narrow_wgrad_tiled(d, dy, x, psc, psh, w, s);
        if (e) return e;
        hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)cdiv(Ktot, 256)), dim3(256), 0, s, w,
                           narrow_wgrad_tiled_blocks(d), 1, d.Cs, d.KH, d.KW, d.cw > 0 ? d.cw : d.Cs, dw);
        return check_launch("narrow_wgrad_tiled_reduce");
    }
    if (d.Co == 1) hipLaunchKernelGGL((conv_wgrad_narrow_kernel<1, false>), grid, dim3(256), 0, s, d, dy, x, x2, psc, psh, w, pps);
    else if (d.Co == 2) hipLaunchKernelGGL((conv_wgrad_narrow_kernel<2, false>), grid, dim3(256), 0, s, d, dy, x, x2, psc, psh, w, pps);
    else if (d.Co == 3) hipLaunchKernelGGL((conv_wgrad_narrow_kernel<3, false>), grid, dim3(256), 0, s, d, dy, x, x2, psc, psh, w, pps);
    else hipLaunchKernelGGL((conv_wgrad_narrow_kernel<4, false>), grid, dim3(256), 0, s, d, dy, x, x2, psc, psh, w, pps);
    e = check_launch("conv_wgrad_narrow");
    if (e) return e;
    long long total = (long long)d.Co * Ktot;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s, w, ns, d.Co, d.Cs,
                       d.KH, d.KW, d.cw > 0 ? d.cw : d.Cs, dw);
    return check_launch("conv_wgrad_narrow_reduce");
}

__global__ void pack_nhwc4_kernel(const float* __restrict__ x, int c1, const float* __restrict__ x2, int c2,
                                  long long HW, long long total, float4* __restrict__ out, float* __restrict__ rng) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;  // pixel index n*HW + hw
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (p < total) {
        const long long n = p / HW, hw = p - n * HW;
        for (int c = 0; c < c1; ++c) v[c] = x[(n * c1 + c) * HW + hw];
        for (int c = 0; c < c2; ++c) v[c1 + c] = x2[(n * c2 + c) * HW + hw];
        out[p] = make_float4(v[0], v[1], v[2], v[3]);
    }
    range_note(rng, absmax4(make_float4(v[0], v[1], v[2], v[3])));  // every lane
}

extern "C" int dcs_pack_nhwc4(const float* x, int c1, const float* x2, int c2, int N, int H, int W, float* out,
                              float* rng, void* stream) {
    if (!x || !out || c1 < 1 || c2 < 0 || c1 + c2 > 4 || (c2 > 0 && !x2) || N <= 0 || H <= 0 || W <= 0 ||
        (reinterpret_cast<uintptr_t>(out) & 15))
        return fail(DCS_E_INVALID, "pack_nhwc4: bad arguments");
    if (int e = range_zero(rng, as_stream(stream))) return e;
    const long long HW = (long long)H * W, total = (long long)N * HW;
    hipLaunchKernelGGL(pack_nhwc4_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, as_stream(stream), x, c1,
                       x2, c2, HW, total, reinterpret_cast<float4*>(out), rng);
    return check_launch("pack_nhwc4");
}

extern "C" int dcs_reflect_fold(const float* dxpad, const float* addend, float* dx, int N, int H, int W, int C,
                                int pad, void* stream) {
    if (!dxpad || !dx || N <= 0 || H <= 0 || W <= 0 || C <= 0 || pad < 0 || pad > 3 || pad >= H || pad >= W)
        return fail(DCS_E_INVALID, "reflect_fold: bad arguments");
    hipStream_t s = as_stream(stream);
    if (C % 4 == 0 && (long long)N * (H + 2 * pad) * (W + 2 * pad) * (C / 4) < (1LL << 31)) {
        long long total = (long long)N * H * W * (C / 4);
        hipLaunchKernelGGL(reflect_fold_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s, dxpad, addend, dx,
                           N, H, W, C / 4, pad);
    } else {
        long long total = (long long)N * H * W * C;
        hipLaunchKernelGGL(reflect_fold_scalar_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s, dxpad,
                           addend, dx, N, H, W, C, pad);
    }
    return check_launch("reflect_fold");
}

extern "C" size_t dcs_conv_dgrad_reflect_ring_size(const dcs_conv_desc* dp) {
    if (!dp || dp->Ho < 6 || dp->Wo < 6) return 0;
    // the window path's ring pass writes one ring copy per K split
    const int copies = ring_ksplit(*dp) > RG_COPIES ? ring_ksplit(*dp) : RG_COPIES;  // (conv_win.hip's ring16_kernel)
    return (size_t)copies * dp->N * (2 * dp->Wo + 2 * (dp->Ho - 2)) * dp->Co * sizeof(float);
}

extern "C" int dcs_conv_dgrad_reflect(const dcs_conv_desc* dp, const float* dy, const float* wpack,
                                      const float* addend, float* dx, float* ring, void* stream) {
    if (!dp || !dy || !wpack || !dx || !ring) return fail(DCS_E_INVALID, "conv_dgrad_reflect: null pointer");
    const dcs_conv_desc& d = *dp;
    if (d.parity || d.stride != 1 || d.up != 1 || d.pad_mode != DCS_PAD_ZERO ||
        d.pt != d.KH - 1 || d.pl != d.KW - 1 || d.pro_act != DCS_ACT_NONE || d.epi_act != DCS_ACT_NONE ||
        d.Ho != d.Hs + 2 || d.Wo != d.Ws + 2 || d.KH != 3 || d.KW != 3 ||
        d.csplit < d.Cs || d.Co % 4 != 0 || d.Ho < 6 || d.Wo < 6)
        return fail(DCS_E_INVALID, "conv_dgrad_reflect: 3x3 stride-1 data gradient onto the pad-1 grid expected "
                                   "(Ho = Hs + 2, pt = pl = 2, zero pad, no activations)");
    if (ring != dx + (long long)d.N * (d.Ho - 2) * (d.Wo - 2) * d.Co)
        return fail(DCS_E_INVALID, "conv_dgrad_reflect: ring must directly follow dx (one allocation)");
    int e = conv_rows_impl(&d, dy, addend, wpack, nullptr, nullptr, nullptr, dx, nullptr, nullptr, stream, 1);
    if (e) return e;
    const int H = d.Ho - 2, W = d.Wo - 2, C4 = d.Co / 4;
    const long long total = (long long)d.N * (2 * W + 2 * (H - 2)) * C4;
    hipLaunchKernelGGL(reflect_ring_fold_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, as_stream(stream), ring,
                       dx, d.N, H, W, C4, 1);
    return check_launch("reflect_ring_fold");
}

// The same fold, and the InstanceNorm-backward partial sums of the folded pixels (the window data
// gradient's epilogue leaves rows 1, H - 2 and columns 1, W - 2 to it): block (n, chunk fc) folds the
// targets fc * tpc .. of image n, 256 / C4 targets at a time, and writes per channel sum g and
// sum g * xhat over them (g = final da * act'(xhat), xhat = y * sc + sh) to parts chunk chunk0 + fc,
// reduced over the block's target lanes in a fixed order.
__global__ __launch_bounds__(256) void reflect_ring_fold_ibw_kernel(const float* __restrict__ ring, float* __restrict__ dx,
                                                                    int N, int H, int W, int C4, int nsplit,
                                                                    const float* __restrict__ yin,
                                                                    const float* __restrict__ sc,
                                                                    const float* __restrict__ sh, int act,
                                                                    Sum2* __restrict__ parts, int nchunk, int chunk0,
                                                                    int nfc) {
    const int n = blockIdx.x / nfc, fc = blockIdx.x - n * nfc;
    const int ntgt = 2 * W + 2 * (H - 2);
    const int tpc = (ntgt + nfc - 1) / nfc;
    const int lanes = 256 / C4, c4 = threadIdx.x % C4, tl = threadIdx.x / C4;
    const int Hp = H + 2, Wp = W + 2, ringlen = 2 * Wp + 2 * H;
    const int C = 4 * C4;
    const float4 s4 = *reinterpret_cast<const float4*>(sc + (long long)n * C + 4 * c4);
    const float4 b4 = *reinterpret_cast<const float4*>(sh + (long long)n * C + 4 * c4);
    float sa[4] = {0.f, 0.f, 0.f, 0.f}, sb[4] = {0.f, 0.f, 0.f, 0.f};
    const int t1 = (fc + 1) * tpc < ntgt ? (fc + 1) * tpc : ntgt;
    for (int t = fc * tpc + tl; t < t1; t += lanes) {
        int y, x;
        if (t < 2 * W) {
            y = t < W ? 1 : H - 2;
            x = t < W ? t : t - W;
        } else {
            const int u = t - 2 * W;
            const int rr = u >> 1;
            y = rr == 0 ? 0 : (rr <= H - 4 ? rr + 1 : H - 1);
            x = (u & 1) ? W - 2 : 1;
        }
        int ay[3], ax[3];
        const int ny = reflect_pre(y, H, 1, ay), nx = reflect_pre(x, W, 1, ax);
        const long long pix = ((long long)n * H + y) * W + x;
        float4* o = reinterpret_cast<float4*>(dx) + pix * C4 + c4;
        float4 v = *o;
        for (int p = 0; p < ny; ++p)
            for (int q = 0; q < nx; ++q) {
                const int yp = ay[p], xp = ax[q];
                if (yp >= 1 && yp <= H && xp >= 1 && xp <= W) continue;
                const int ri = yp == 0 ? xp : (yp == Hp - 1 ? Wp + xp : 2 * Wp + 2 * (yp - 1) + (xp == 0 ? 0 : 1));
                for (int qq = 0; qq < nsplit; ++qq) {
                    const float4 r = reinterpret_cast<const float4*>(ring)[(((long long)qq * N + n) * ringlen + ri) * C4 + c4];
                    v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
                }
            }
        *o = v;
        const float4 y4 = reinterpret_cast<const float4*>(yin)[pix * C4 + c4];
        const float dv[4] = {v.x, v.y, v.z, v.w}, yv[4] = {y4.x, y4.y, y4.z, y4.w};
        const float s_[4] = {s4.x, s4.y, s4.z, s4.w}, b_[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float xh = fmaf(yv[e], s_[e], b_[e]);
            const float g = dv[e] * act_grad(xh, act);
            sa[e] += g;
            sb[e] = fmaf(g, xh, sb[e]);
        }
    }
    __shared__ float red[8][256];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        red[e][threadIdx.x] = sa[e];
        red[4 + e][threadIdx.x] = sb[e];
    }
    __syncthreads();
    if (tl == 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float a = 0.f, b = 0.f;
            for (int l = 0; l < lanes; ++l) {
                a += red[e][l * C4 + c4];
                b += red[4 + e][l * C4 + c4];
            }
            parts[((long long)n * nchunk + chunk0 + fc) * C + 4 * c4 + e] = Sum2{a, b};
        }
    }
}

namespace dcs {
// fold + IN-backward partial sums of the folded pixels (reflect_ring_fold_ibw_kernel); C / 4 divides 256
int reflect_ring_fold_ibw(const float* ring, float* dx, int N, int H, int W, int C, int nsplit, const float* y,
                          const float* sc, const float* sh, int act, Sum2* parts, int nchunk, int chunk0, int nfc,
                          hipStream_t s) {
    const int C4 = C / 4;
    if (C % 4 || 256 % C4) return fail(DCS_E_INVALID, "reflect_ring_fold_ibw: C / 4 must divide 256");
    hipLaunchKernelGGL(reflect_ring_fold_ibw_kernel, dim3((unsigned)(N * nfc)), dim3(256), 0, s, ring, dx, N, H, W, C4,
                       nsplit, y, sc, sh, act, parts, nchunk, chunk0, nfc);
    return check_launch("reflect_ring_fold_ibw");
}

// fold the padded grid's ring (dcs_conv_dgrad_reflect's ring layout) onto dx's border (H x W interior)
int reflect_ring_fold(const float* ring, float* dx, int N, int H, int W, int C, int nsplit, hipStream_t s) {
    const int C4 = C / 4;
    const long long total = (long long)N * (2 * W + 2 * (H - 2)) * C4;
    hipLaunchKernelGGL(reflect_ring_fold_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s, ring, dx, N, H, W, C4,
                       nsplit);
    return check_launch("reflect_ring_fold");
}
}  // namespace dcs

extern "C" int dcs_upsample2_grad(const float* dup, float* dx, int N, int H, int W, int C, void* stream) {
    if (!dup || !dx || N <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 4 != 0)
        return fail(DCS_E_INVALID, "upsample2_grad: bad arguments (C % 4 == 0 required)");
    long long total = (long long)N * H * W * (C / 4);
    hipLaunchKernelGGL(upsample2_grad_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, as_stream(stream),
                       dup, dx, N, H, W, C / 4);
    return check_launch("upsample2_grad");
}
