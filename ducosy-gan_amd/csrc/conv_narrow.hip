// LDS-tiled single-output-channel convolutions on gfx950 (Co == 1):
//   * the Generator head (modules/model.py:112: ReflectionPad(3) + Conv 7x7 64->1 + Tanh),
//   * the input-image gradient of the stem (dgrad of Conv 7x7 cin->64, channel 0 only),
//   * the PatchGAN last layer (modules/model.py:129: Conv 4x4 512->1),
// forward rows and weight gradient.  A GEMM with N = 1 wastes 31/32 of every MFMA, so these
// run on the VALU: a block stages a (16+KH-1) x (64+KW-1) halo of 8 source channels in LDS
// (prologue InstanceNorm+ReLU and reflection/zero padding applied while staging), each
// thread then produces 4 horizontally adjacent outputs with a sliding register window
// (10 float4 source reads feed 28 float4 dot products per tap row).
#include "common.hpp"

namespace dcs {

constexpr int NT_TH = 16, NT_TW = 64, NT_CC = 8, NT_XT = 4;
#ifndef DCS_NARROW_TY_UNROLL
#define DCS_NARROW_TY_UNROLL 1
#endif
#ifndef DCS_NARROW_WAVES
#define DCS_NARROW_WAVES 3  // waves per SIMD the head forward is compiled for (3 blocks of 4 waves per CU)
#endif

// Halo coordinate -> source coordinate.  Halo pixels that only feed masked outputs (tile
// overhang past Ho/Wo) can lie more than one reflection away: clamp them into the tensor so
// every staged read stays in bounds (their values are never used).
__device__ __forceinline__ bool nmap(int v, int Hs, int mode, int& s) {
    if (v < 0 || v >= Hs) {
        if (mode == DCS_PAD_ZERO) return false;
        v = v < 0 ? -v : 2 * (Hs - 1) - v;
        v = v < 0 ? 0 : (v >= Hs ? Hs - 1 : v);
    }
    s = v;
    return true;
}

// stage the halo of channel chunk c0 into LDS: lin[(hy*HW_ + hx)*8 + c]
template <int KH, int KW>
__device__ __forceinline__ void stage_halo(const dcs_conv_desc& d, const float* __restrict__ src,
                                           const float* __restrict__ psc, const float* __restrict__ psh,
                                           int n, int oy0, int ox0, int c0, float* lin) {
    constexpr int HH = NT_TH + KH - 1, HW_ = NT_TW + KW - 1;
    const long long so = (long long)n * d.Cs + c0;
    for (int i = threadIdx.x; i < HH * HW_ * 2; i += blockDim.x) {
        const int pix = i >> 1, half = i & 1;
        const int hy = pix / HW_, hx = pix - hy * HW_;
        int sy, sx;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (nmap(oy0 + hy - d.pt, d.Hs, d.pad_mode, sy) && nmap(ox0 + hx - d.pl, d.Ws, d.pad_mode, sx)) {
            v = *reinterpret_cast<const float4*>(src + n * d.s_n + sy * d.s_h + sx * d.s_w + c0 + half * 4);
            if (d.pro_act != DCS_ACT_NONE) {
                const float* s = psc + so + half * 4;
                const float* b = psh + so + half * 4;
                v.x = act_apply(fmaf(v.x, s[0], b[0]), d.pro_act);
                v.y = act_apply(fmaf(v.y, s[1], b[1]), d.pro_act);
                v.z = act_apply(fmaf(v.z, s[2], b[2]), d.pro_act);
                v.w = act_apply(fmaf(v.w, s[3], b[3]), d.pro_act);
            }
        }
        *reinterpret_cast<float4*>(lin + pix * NT_CC + half * 4) = v;
    }
}

__device__ __forceinline__ float dot4(float4 a, float4 b, float acc) {
    acc = fmaf(a.x, b.x, acc);
    acc = fmaf(a.y, b.y, acc);
    acc = fmaf(a.z, b.z, acc);
    return fmaf(a.w, b.w, acc);
}

template <int KH, int KW>
__global__ __launch_bounds__(256, DCS_NARROW_WAVES) void narrow_rows_tiled_kernel(const dcs_conv_desc d, const float* __restrict__ src,
                                                                const float* __restrict__ wp,
                                                                const float* __restrict__ bias,
                                                                const float* __restrict__ psc,
                                                                const float* __restrict__ psh,
                                                                float* __restrict__ out) {
    constexpr int HH = NT_TH + KH - 1, HW_ = NT_TW + KW - 1;
    __shared__ __attribute__((aligned(16))) float lin[HH * HW_ * NT_CC];
    __shared__ __attribute__((aligned(16))) float lw[KH * KW * NT_CC];
    const int n = blockIdx.z;
    const int oy0 = blockIdx.y * NT_TH, ox0 = blockIdx.x * NT_TW;
    const int r = threadIdx.x >> 4, cg = threadIdx.x & 15;
    float acc[NT_XT] = {0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < d.Cs; c0 += NT_CC) {
        __syncthreads();
        stage_halo<KH, KW>(d, src, psc, psh, n, oy0, ox0, c0, lin);
        for (int i = threadIdx.x; i < KH * KW * NT_CC; i += blockDim.x) {
            const int t = i / NT_CC, c = i - t * NT_CC;
            lw[i] = wp[((long long)t * d.Cs + c0 + c) * d.ldb];
        }
        __syncthreads();
        // tap rows not unrolled and 3 waves per SIMD (<= 168 VGPRs, was 238): 3 blocks of 50 KB LDS
        // fit a CU instead of 2
#pragma unroll DCS_NARROW_TY_UNROLL
        for (int ty = 0; ty < KH; ++ty) {
            const float* row = lin + ((r + ty) * HW_ + cg * NT_XT) * NT_CC;
#pragma unroll DCS_NARROW_TY_UNROLL
            for (int q = 0; q < 2; ++q) {
                float4 v[NT_XT + KW - 1];
#pragma unroll
                for (int i = 0; i < NT_XT + KW - 1; ++i) v[i] = *reinterpret_cast<const float4*>(row + i * NT_CC + q * 4);
#pragma unroll
                for (int tx = 0; tx < KW; ++tx) {
                    const float4 w = *reinterpret_cast<const float4*>(lw + (ty * KW + tx) * NT_CC + q * 4);
#pragma unroll
                    for (int j = 0; j < NT_XT; ++j) acc[j] = dot4(v[j + tx], w, acc[j]);
                }
            }
        }
    }
    const int oy = oy0 + r;
    if (oy >= d.Ho) return;
    const float b = bias ? bias[0] : 0.f;
#pragma unroll
    for (int j = 0; j < NT_XT; ++j) {
        const int ox = ox0 + cg * NT_XT + j;
        if (ox < d.Wo) {
            float v = acc[j] + b;
            if (d.epi_act != DCS_ACT_NONE) v = act_apply(v, d.epi_act);
            out[((long long)n * d.Ho + oy) * d.Wo + ox] = v;
        }
    }
}

// weight gradient, Co == 1: part[block][t*Cs + c] = sum over the block's tiles of
// dy[p] * src(p + t)[c].  Each block walks tiles with a grid stride; per thread the
// accumulators of its (tap, channel) items of every chunk stay in registers.
template <int KH, int KW, int NCH>
__global__ __launch_bounds__(256) void narrow_wgrad_tiled_kernel(const dcs_conv_desc d, const float* __restrict__ dy,
                                                                 const float* __restrict__ src,
                                                                 const float* __restrict__ psc,
                                                                 const float* __restrict__ psh,
                                                                 float* __restrict__ part, int tiles_x,
                                                                 int tiles_y) {
    constexpr int HH = NT_TH + KH - 1, HW_ = NT_TW + KW - 1;
    constexpr int ITEMS = KH * KW * NT_CC;           // per chunk
    constexpr int IPT = (ITEMS + 255) / 256;         // items per thread per chunk
    __shared__ __attribute__((aligned(16))) float lin[HH * HW_ * NT_CC];
    __shared__ float ldy[NT_TH * NT_TW];
    float acc[NCH][IPT];
#pragma unroll
    for (int k = 0; k < NCH; ++k)
#pragma unroll
        for (int q = 0; q < IPT; ++q) acc[k][q] = 0.f;
    const int ntiles = tiles_x * tiles_y * d.N;
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int n = tile / (tiles_x * tiles_y);
        const int rem = tile - n * tiles_x * tiles_y;
        const int oy0 = (rem / tiles_x) * NT_TH, ox0 = (rem % tiles_x) * NT_TW;
        __syncthreads();
        for (int i = threadIdx.x; i < NT_TH * NT_TW; i += blockDim.x) {
            const int yy = oy0 + i / NT_TW, xx = ox0 + i % NT_TW;
            ldy[i] = (yy < d.Ho && xx < d.Wo) ? dy[((long long)n * d.Ho + yy) * d.Wo + xx] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
            __syncthreads();
            stage_halo<KH, KW>(d, src, psc, psh, n, oy0, ox0, k * NT_CC, lin);
            __syncthreads();
#pragma unroll
            for (int q = 0; q < IPT; ++q) {
                const int it = threadIdx.x + q * 256;
                if (it < ITEMS) {
                    const int t = it / NT_CC, c = it - t * NT_CC;
                    const int ty = t / KW, tx = t - ty * KW;
                    float a = 0.f;
                    for (int yy = 0; yy < NT_TH; ++yy) {
                        const float* row = lin + ((yy + ty) * HW_ + tx) * NT_CC + c;
                        const float* g = ldy + yy * NT_TW;
#pragma unroll 8
                        for (int xx = 0; xx < NT_TW; ++xx) a = fmaf(g[xx], row[xx * NT_CC], a);
                    }
                    acc[k][q] += a;
                }
            }
        }
    }
#pragma unroll
    for (int k = 0; k < NCH; ++k)
#pragma unroll
        for (int q = 0; q < IPT; ++q) {
            const int it = threadIdx.x + q * 256;
            if (it < ITEMS) {
                const int t = it / NT_CC, c = it - t * NT_CC;
                part[(long long)blockIdx.x * (KH * KW * d.Cs) + (long long)t * d.Cs + k * NT_CC + c] = acc[k][q];
            }
        }
}

// weight gradient, Co == 1, with a register window along x: thread (row group rg, ty, c) keeps
// the KW tap sums of (ty, tx = 0..KW-1, c) and walks the tile's pixel rows of its group; each
// staged source value it reads feeds KW multiply-adds (the per-item kernel above read one LDS
// value per multiply-add).  Per-thread sums persist across the block's tiles; the row groups are
// added in a fixed order at the end (deterministic).  Same partial layout as the kernel above.
template <int KH, int KW, int NCH>
__global__ __launch_bounds__(256) void narrow_wgrad_win_kernel(const dcs_conv_desc d, const float* __restrict__ dy,
                                                               const float* __restrict__ src,
                                                               const float* __restrict__ psc,
                                                               const float* __restrict__ psh,
                                                               float* __restrict__ part, int tiles_x, int tiles_y) {
    constexpr int HH = NT_TH + KH - 1, HW_ = NT_TW + KW - 1;
    constexpr int ITEMS = KH * NT_CC;            // (ty, c) pairs per chunk
    constexpr int RG = 256 / ITEMS;              // row groups (4 for 7x7)
    constexpr int RPG = (NT_TH + RG - 1) / RG;   // tile rows per group
    __shared__ __attribute__((aligned(16))) float lin[HH * HW_ * NT_CC];
    __shared__ float ldy[NT_TH * NT_TW];
    const int rg = threadIdx.x / ITEMS, item = threadIdx.x - (threadIdx.x / ITEMS) * ITEMS;
    const bool live = rg < RG;
    const int ty = item / NT_CC, c = item - (item / NT_CC) * NT_CC;
    float acc[NCH][KW];
#pragma unroll
    for (int k = 0; k < NCH; ++k)
#pragma unroll
        for (int tx = 0; tx < KW; ++tx) acc[k][tx] = 0.f;
    const int ntiles = tiles_x * tiles_y * d.N;
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int n = tile / (tiles_x * tiles_y);
        const int rem = tile - n * tiles_x * tiles_y;
        const int oy0 = (rem / tiles_x) * NT_TH, ox0 = (rem % tiles_x) * NT_TW;
        __syncthreads();
        for (int i = threadIdx.x; i < NT_TH * NT_TW; i += blockDim.x) {
            const int yy = oy0 + i / NT_TW, xx = ox0 + i % NT_TW;
            ldy[i] = (yy < d.Ho && xx < d.Wo) ? dy[((long long)n * d.Ho + yy) * d.Wo + xx] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
            __syncthreads();
            stage_halo<KH, KW>(d, src, psc, psh, n, oy0, ox0, k * NT_CC, lin);
            __syncthreads();
            if (live) {
                for (int r = 0; r < RPG; ++r) {
                    const int yy = rg * RPG + r;
                    if (yy >= NT_TH) break;
                    const float* row = lin + (yy + ty) * HW_ * NT_CC + c;
                    const float* g = ldy + yy * NT_TW;
                    float w[KW];
#pragma unroll
                    for (int tx = 0; tx < KW - 1; ++tx) w[tx] = row[tx * NT_CC];
#pragma unroll
                    for (int xx = 0; xx < NT_TW; ++xx) {
                        w[(xx + KW - 1) % KW] = row[(xx + KW - 1) * NT_CC];
                        const float gv = g[xx];
#pragma unroll
                        for (int tx = 0; tx < KW; ++tx) acc[k][tx] = fmaf(gv, w[(xx + tx) % KW], acc[k][tx]);
                    }
                }
            }
        }
    }
    // add the row groups in order, through LDS (one chunk at a time)
    float* red = lin;  // [RG][ITEMS][KW]
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
        __syncthreads();
        if (live)
#pragma unroll
            for (int tx = 0; tx < KW; ++tx) red[(rg * ITEMS + item) * KW + tx] = acc[k][tx];
        __syncthreads();
        for (int i = threadIdx.x; i < ITEMS * KW; i += blockDim.x) {
            const int it = i / KW, tx = i - (i / KW) * KW;
            float sum = 0.f;
            for (int q = 0; q < RG; ++q) sum += red[(q * ITEMS + it) * KW + tx];
            const int tyy = it / NT_CC, cc = it - (it / NT_CC) * NT_CC;
            part[(long long)blockIdx.x * (KH * KW * d.Cs) + (long long)(tyy * KW + tx) * d.Cs + k * NT_CC + cc] = sum;
        }
    }
}

// One output channel over many input channels on small images (the PatchGAN last layer,
// modules/model.py:129: Conv 4x4 512->1 on 32 x 32): a tiled kernel gets one block per 16 x 64
// output tile, 32 blocks for a batch of 16, so here one WAVE computes one output pixel, its 64
// lanes splitting the channels (CPL each; a tap's pixel row is one coalesced 2 KiB read), the
// weights of the lane's channels held in registers, the prologue (IN + LeakyReLU of the
// previous layer) applied per element, then a fixed-order cross-lane sum.
template <int KH, int KW, int CPL>
__global__ __launch_bounds__(256) void narrow_rows_small_kernel(const dcs_conv_desc d, const float* __restrict__ src,
                                                                const float* __restrict__ wp,
                                                                const float* __restrict__ bias,
                                                                const float* __restrict__ psc,
                                                                const float* __restrict__ psh,
                                                                float* __restrict__ out) {
    static_assert(CPL % 4 == 0, "float4 channel groups");
    const int lane = threadIdx.x & 63;
    const int c0 = lane * CPL;
    float w[KH * KW][CPL];
#pragma unroll
    for (int t = 0; t < KH * KW; ++t)
#pragma unroll
        for (int j = 0; j < CPL; ++j) w[t][j] = wp[((long long)t * d.Cs + c0 + j) * d.ldb];
    const float b = bias ? bias[0] : 0.f;
    const long long P = (long long)d.N * d.Ho * d.Wo;
    const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long long nwaves = ((long long)gridDim.x * blockDim.x) >> 6;
    for (long long p = wave; p < P; p += nwaves) {
        const int n = (int)(p / ((long long)d.Ho * d.Wo));
        const int rem = (int)(p - (long long)n * d.Ho * d.Wo);
        const int oy = rem / d.Wo, ox = rem - (rem / d.Wo) * d.Wo;
        float sc[CPL], sh[CPL];
        if (d.pro_act != DCS_ACT_NONE) {
#pragma unroll
            for (int j = 0; j < CPL; ++j) {
                sc[j] = psc[(long long)n * d.Cs + c0 + j];
                sh[j] = psh[(long long)n * d.Cs + c0 + j];
            }
        }
        float acc = 0.f;
#pragma unroll
        for (int ty = 0; ty < KH; ++ty) {
            const int iy = oy * d.stride + ty - d.pt;
            if (iy < 0 || iy >= d.Hs) continue;  // zero padding
#pragma unroll
            for (int tx = 0; tx < KW; ++tx) {
                const int ix = ox * d.stride + tx - d.pl;
                if (ix < 0 || ix >= d.Ws) continue;
                const float* sp = src + n * d.s_n + iy * d.s_h + ix * d.s_w + c0;
#pragma unroll
                for (int j4 = 0; j4 < CPL / 4; ++j4) {
                    const float4 v4 = *reinterpret_cast<const float4*>(sp + 4 * j4);
                    const float v[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int j = 4 * j4 + e;
                        const float a = d.pro_act != DCS_ACT_NONE ? act_apply(fmaf(v[e], sc[j], sh[j]), d.pro_act) : v[e];
                        acc = fmaf(a, w[ty * KW + tx][j], acc);
                    }
                }
            }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
        if (lane == 0) {
            float v = acc + b;
            if (d.epi_act != DCS_ACT_NONE) v = act_apply(v, d.epi_act);
            out[p] = v;
        }
    }
}

bool narrow_small_ok(const dcs_conv_desc& d, const float* src) {
    return !d.parity && d.Co == 1 && d.up == 1 && d.pad_mode == DCS_PAD_ZERO && d.KH == 4 && d.KW == 4 &&
           (d.Cs == 256 || d.Cs == 512) && d.s_c == 1 && d.csplit == d.Cs && d.s_w % 4 == 0 && d.s_h % 4 == 0 &&
           d.s_n % 4 == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0 && (long long)d.Ho * d.Wo <= 64 * 64;
}

int launch_narrow_rows_small(const dcs_conv_desc& d, const float* src, const float* wp, const float* bias,
                             const float* psc, const float* psh, float* out, hipStream_t s) {
    const long long P = (long long)d.N * d.Ho * d.Wo;
    long long blocks = cdiv(P, 4);  // one wave per pixel, 4 waves per block
    if (blocks > 2048) blocks = 2048;
    if (d.Cs == 512)
        hipLaunchKernelGGL((narrow_rows_small_kernel<4, 4, 8>), dim3((unsigned)blocks), dim3(256), 0, s, d, src, wp, bias,
                           psc, psh, out);
    else
        hipLaunchKernelGGL((narrow_rows_small_kernel<4, 4, 4>), dim3((unsigned)blocks), dim3(256), 0, s, d, src, wp, bias,
                           psc, psh, out);
    return check_launch("narrow_rows_small");
}

bool narrow_tiled_ok(const dcs_conv_desc& d, const float* src) {
    return !d.parity && d.Co == 1 && d.up == 1 && d.stride == 1 && d.Cs % NT_CC == 0 && d.s_c == 1 &&
           d.csplit == d.Cs && (d.s_w % 4 == 0) && (d.s_h % 4 == 0) && (d.s_n % 4 == 0) &&
           ((reinterpret_cast<uintptr_t>(src) & 15) == 0) &&
           ((d.KH == 7 && d.KW == 7) || (d.KH == 4 && d.KW == 4));
}

int launch_narrow_rows_tiled(const dcs_conv_desc& d, const float* src, const float* wp, const float* bias,
                             const float* psc, const float* psh, float* out, hipStream_t s) {
    dim3 grid((unsigned)cdiv(d.Wo, NT_TW), (unsigned)cdiv(d.Ho, NT_TH), d.N);
    if (d.KH == 7)
        hipLaunchKernelGGL((narrow_rows_tiled_kernel<7, 7>), grid, dim3(256), 0, s, d, src, wp, bias, psc, psh, out);
    else
        hipLaunchKernelGGL((narrow_rows_tiled_kernel<4, 4>), grid, dim3(256), 0, s, d, src, wp, bias, psc, psh, out);
    return check_launch("narrow_rows_tiled");
}

bool narrow_wgrad_tiled_ok(const dcs_conv_desc& d, const float* src) {
    return narrow_tiled_ok(d, src) && d.KH == 7 && d.Cs == 64;
}

#ifndef DCS_NARROW_WGRAD_BLOCKS
#define DCS_NARROW_WGRAD_BLOCKS 768  // 3 blocks of 53 KB LDS per CU on 256 CUs
#endif
int narrow_wgrad_tiled_blocks(const dcs_conv_desc& d) {
    long long tiles = cdiv(d.Wo, NT_TW) * cdiv(d.Ho, NT_TH) * d.N;
    return (int)(tiles < DCS_NARROW_WGRAD_BLOCKS ? tiles : DCS_NARROW_WGRAD_BLOCKS);
}

int launch_narrow_wgrad_tiled(const dcs_conv_desc& d, const float* dy, const float* src, const float* psc,
                              const float* psh, float* part, hipStream_t s) {
    const int tx = (int)cdiv(d.Wo, NT_TW), ty = (int)cdiv(d.Ho, NT_TH);
#ifdef DCS_NARROW_WGRAD_ITEMS  // A/B: one LDS read per multiply-add
    hipLaunchKernelGGL((narrow_wgrad_tiled_kernel<7, 7, 8>), dim3(narrow_wgrad_tiled_blocks(d)), dim3(256), 0, s, d,
                       dy, src, psc, psh, part, tx, ty);
#else
    hipLaunchKernelGGL((narrow_wgrad_win_kernel<7, 7, 8>), dim3(narrow_wgrad_tiled_blocks(d)), dim3(256), 0, s, d,
                       dy, src, psc, psh, part, tx, ty);
#endif
    return check_launch("narrow_wgrad_tiled");
}

// Data gradient of a KxK convolution whose OUTPUT has one channel (the Generator head,
// modules/model.py:112: ReflectionPad(3) + Conv 7x7 64->1), onto the unpadded input:
//   dx[n][y][x][c] = sum_{ty,tx} W[c][ty][tx] * g[n][y][x][ty][tx],
//   g = sum over the padded positions (a, b) that pad to (y, x) of dy[n][a-ty][b-tx]
// (zero outside dy).  The padding adjoint (reflection fold) is applied to the one-channel dy
// before the channel expansion, so the 64-channel padded gradient is never materialised, and
// the K*K*C MACs per pixel run on the VALU with the weights as wave-uniform scalar operands
// (an N = 1 GEMM would waste 31/32 of every MFMA).  One thread per input pixel, all C channels.
__device__ __forceinline__ int pad_preimages(int i, int H, int pad, int mode, int* a) {
    int n = 0;
    a[n++] = i + pad;
    if (mode == DCS_PAD_REFLECT) {
        if (i >= 1 && i <= pad) a[n++] = pad - i;
        if (i >= H - 1 - pad && i <= H - 2) a[n++] = 2 * (H - 1) - i + pad;
    }
    return n;
}

template <int C, int K>
__global__ __launch_bounds__(256) void dgrad_c1_kernel(const float* __restrict__ dy, int N, int H, int W,
                                                       const float* __restrict__ wk, int mode,
                                                       float* __restrict__ dx) {
    constexpr int pad = (K - 1) / 2;
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (long long)N * H * W) return;
    const int n = (int)(p / ((long long)H * W));
    const int rem = (int)(p - (long long)n * H * W);
    const int y = rem / W, x = rem - (rem / W) * W;
    // interior pixels (one preimage — reflection also maps rows 1..pad and H-1-pad..H-2 — and
    // every tap inside dy) take unconditional loads
    const bool inner = y > pad && y < H - 1 - pad && x > pad && x < W - 1 - pad;
    int ay[3], ax[3], ny = 1, nx = 1;
    if (!inner) {
        ny = pad_preimages(y, H, pad, mode, ay);
        nx = pad_preimages(x, W, pad, mode, ax);
    }
    const float* d = dy + (long long)n * H * W;
    float acc[C];
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = 0.f;
#pragma unroll 1
    for (int ty = 0; ty < K; ++ty) {
        float g[K];
        if (inner) {
            const float* b = d + (long long)(y + pad - ty) * W + x + pad;
#pragma unroll
            for (int tx = 0; tx < K; ++tx) g[tx] = b[-tx];
        } else {
#pragma unroll
            for (int tx = 0; tx < K; ++tx) {
                float s = 0.f;
                for (int i = 0; i < ny; ++i) {
                    const int r = ay[i] - ty;
                    if ((unsigned)r >= (unsigned)H) continue;
                    for (int j = 0; j < nx; ++j) {
                        const int q = ax[j] - tx;
                        if ((unsigned)q < (unsigned)W) s += d[(long long)r * W + q];
                    }
                }
                g[tx] = s;
            }
        }
#pragma unroll
        for (int tx = 0; tx < K; ++tx) {
            const float* wt = wk + (ty * K + tx) * C;  // wave-uniform: scalar loads
#pragma unroll
            for (int c = 0; c < C; ++c) acc[c] = fmaf(wt[c], g[tx], acc[c]);
        }
    }
    float4* o = reinterpret_cast<float4*>(dx + p * C);
#pragma unroll
    for (int c = 0; c < C / 4; ++c) o[c] = make_float4(acc[4 * c], acc[4 * c + 1], acc[4 * c + 2], acc[4 * c + 3]);
}


// Data gradient onto ONE input channel (the image channel of the Generator stem, Conv 7x7
// cin->64 with ReflectionPad(3); the PatchGAN's first layer, Conv 4x4 s2 1->64), in two passes
// instead of a 64->1 transposed convolution that re-gathers every dy pixel for every output:
//   pass 1 (per dy pixel q): z[t][q] = sum_c W[c][0][t] * dy[q][c]        (K*K dot products of C)
//   pass 2 (per input pixel): dx[y][x] = sum over the padded positions (a, b) that pad to (y, x)
//          and the taps t = (ty, tx) with (a - ty) and (b - tx) divisible by the stride of
//          z[t][((a-ty)/s, (b-tx)/s)]
// z is tap-planar ([K*K][Q]) so that both passes touch it with unit stride across the lanes.
// Pass 1 stages 64 dy pixels x 32 channels at a time through LDS (coalesced 128-B row segments
// in, one pixel row per lane out).
template <int T, int C>
__global__ __launch_bounds__(64) void to1_zproj_kernel(const float* __restrict__ dy, long long Q,
                                                       const float* __restrict__ wk, float* __restrict__ z) {
    constexpr int HC = 32, PITCH = HC + 4, SEG = HC / 4;  // channels per stage, LDS row pitch (floats)
    static_assert(C == 2 * HC, "two staging rounds");
    __shared__ __attribute__((aligned(16))) float sm[64 * PITCH];
    const long long q0 = (long long)blockIdx.x * 64;
    const int lane = threadIdx.x;
    float4 row[C / 4];  // this lane's dy pixel, all channels
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int k = 0; k < SEG; ++k) {
            const int idx = k * 64 + lane, pix = idx / SEG, c4 = idx - (idx / SEG) * SEG;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (q0 + pix < Q) v = *reinterpret_cast<const float4*>(dy + (q0 + pix) * C + h * HC + 4 * c4);
            *reinterpret_cast<float4*>(sm + pix * PITCH + 4 * c4) = v;
        }
        __syncthreads();
#pragma unroll
        for (int c4 = 0; c4 < SEG; ++c4) row[h * SEG + c4] = *reinterpret_cast<const float4*>(sm + lane * PITCH + 4 * c4);
        __syncthreads();
    }
    const long long q = q0 + lane;
    const bool live = q < Q;
    // tap-outer: one tap's C weights (wave-uniform scalar loads) against the register row
#pragma unroll 7
    for (int t = 0; t < T; ++t) {
        const float* w = wk + t * C;
        float a0 = 0.f, a1 = 0.f;  // two chains
#pragma unroll
        for (int c4 = 0; c4 < C / 4; c4 += 2) {
            a0 = fmaf(w[4 * c4 + 0], row[c4].x, fmaf(w[4 * c4 + 1], row[c4].y,
                 fmaf(w[4 * c4 + 2], row[c4].z, fmaf(w[4 * c4 + 3], row[c4].w, a0))));
            a1 = fmaf(w[4 * c4 + 4], row[c4 + 1].x, fmaf(w[4 * c4 + 5], row[c4 + 1].y,
                 fmaf(w[4 * c4 + 6], row[c4 + 1].z, fmaf(w[4 * c4 + 7], row[c4 + 1].w, a1))));
        }
        if (live) z[t * Q + q] = a0 + a1;
    }
}

// taps of one axis that reach padded position a: all K (stride 1), or the K/2 of a's parity
// (stride 2, K even)
template <int K, int S>
__global__ __launch_bounds__(256) void to1_gather_kernel(const float* __restrict__ z, int N, int Hy, int Wy, int pt,
                                                         int pl, int mode, int H, int W, float* __restrict__ dx) {
    static_assert(S == 1 || (S == 2 && K % 2 == 0), "stride-2 taps come in parity pairs");
    constexpr int KS = K / S;
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (long long)N * H * W) return;
    const int n = (int)(p / ((long long)H * W));
    const int rem = (int)(p - (long long)n * H * W);
    const int y = rem / W, x = rem - (rem / W) * W;
    int ay[3], ax[3];
    const int ny = pad_preimages(y, H, pt, mode, ay), nx = pad_preimages(x, W, pl, mode, ax);
    const long long Q = (long long)N * Hy * Wy;
    const float* zn = z + (long long)n * Hy * Wy;
    float s = 0.f;
    for (int i = 0; i < ny; ++i) {
        const int a = ay[i];
#pragma unroll
        for (int my = 0; my < KS; ++my) {
            const int ty = S == 2 ? (a & 1) + 2 * my : my;
            const int u = a - ty;
            if (u < 0) continue;
            const int oy = S == 2 ? (u >> 1) : u;
            if (oy >= Hy) continue;
            for (int j = 0; j < nx; ++j) {
                const int b = ax[j];
#pragma unroll
                for (int mx = 0; mx < KS; ++mx) {
                    const int tx = S == 2 ? (b & 1) + 2 * mx : mx;
                    const int v = b - tx;
                    const int ox = S == 2 ? (v >> 1) : v;
                    if (v >= 0 && ox < Wy) s += zn[(ty * K + tx) * Q + (long long)oy * Wy + ox];
                }
            }
        }
    }
    dx[p] = s;
}

}  // namespace dcs

using namespace dcs;

extern "C" size_t dcs_conv_dgrad_to1_workspace_size(int N, int Hy, int Wy, int K) {
    return (size_t)N * Hy * Wy * K * K * sizeof(float);
}

// dy: NHWC [N][Hy][Wy][C] (C = 64); wk[(ty*K + tx)*C + c] = W[c][0][ty][tx] (dcs_pack_weights kind 2,
// nmajor 0, ncols 1, ci_count 1); dx: [N][H][W], the unpadded input of the forward conv (stride s,
// padding pt/pl of pad_mode, Hy = (H + 2*pt - K)/s + 1).
extern "C" int dcs_conv_dgrad_to1(const float* dy, int N, int Hy, int Wy, int C, const float* wk, int K, int stride,
                                  int pt, int pl, int pad_mode, int H, int W, float* dx, void* ws, size_t ws_bytes,
                                  void* stream) {
    if (!dy || !wk || !dx || !ws || N <= 0 || Hy <= 0 || Wy <= 0 || H <= 0 || W <= 0 || (stride != 1 && stride != 2) ||
        pt < 0 || pl < 0 || (pad_mode != DCS_PAD_ZERO && pad_mode != DCS_PAD_REFLECT) ||
        (pad_mode == DCS_PAD_REFLECT && (pt >= H || pl >= W)) || (reinterpret_cast<uintptr_t>(dy) & 15))
        return fail(DCS_E_INVALID, "conv_dgrad_to1: bad arguments");
    if (C != 64 || !((K == 7 && stride == 1) || (K == 4 && stride == 2)))
        return fail(DCS_E_INVALID, "conv_dgrad_to1: C == 64 and (K, stride) = (7, 1) or (4, 2)");
    if (ws_bytes < dcs_conv_dgrad_to1_workspace_size(N, Hy, Wy, K))
        return fail(DCS_E_WORKSPACE, "conv_dgrad_to1: workspace too small");
    hipStream_t s = as_stream(stream);
    float* z = reinterpret_cast<float*>(ws);
    const long long Q = (long long)N * Hy * Wy;
    if (K == 7) hipLaunchKernelGGL((to1_zproj_kernel<49, 64>), dim3((unsigned)cdiv(Q, 64)), dim3(64), 0, s, dy, Q, wk, z);
    else hipLaunchKernelGGL((to1_zproj_kernel<16, 64>), dim3((unsigned)cdiv(Q, 64)), dim3(64), 0, s, dy, Q, wk, z);
    int e = check_launch("conv_dgrad_to1_zproj");
    if (e) return e;
    const dim3 grid((unsigned)cdiv((long long)N * H * W, 256));
    if (K == 7) hipLaunchKernelGGL((to1_gather_kernel<7, 1>), grid, dim3(256), 0, s, z, N, Hy, Wy, pt, pl, pad_mode, H, W, dx);
    else hipLaunchKernelGGL((to1_gather_kernel<4, 2>), grid, dim3(256), 0, s, z, N, Hy, Wy, pt, pl, pad_mode, H, W, dx);
    return check_launch("conv_dgrad_to1_gather");
}

// wk: the forward conv's K-major packed weights ([K*K][C] x 1 column: dcs_pack_weights kind 0,
// nmajor 0, ncols 1), i.e. wk[(ty*K + tx)*C + c] = W[0][c][ty][tx].
extern "C" int dcs_conv_dgrad_c1(const float* dy, int N, int H, int W, const float* wk, int C, int K, int pad,
                                 int pad_mode, float* dx, void* stream) {
    if (!dy || !wk || !dx || N <= 0 || H <= 0 || W <= 0 || K <= 0 || K > 9 || pad < 0 || pad >= K ||
        (pad_mode != DCS_PAD_ZERO && pad_mode != DCS_PAD_REFLECT) || (pad_mode == DCS_PAD_REFLECT && (pad >= H || pad >= W)) ||
        (reinterpret_cast<uintptr_t>(dx) & 15))
        return fail(DCS_E_INVALID, "conv_dgrad_c1: bad arguments");
    if (2 * pad != K - 1) return fail(DCS_E_INVALID, "conv_dgrad_c1: 'same' convolutions only (2*pad == K-1)");
    const long long total = (long long)N * H * W;
    const dim3 grid((unsigned)cdiv(total, 256));
    hipStream_t s = as_stream(stream);
#define DCS_C1(CC, KK) hipLaunchKernelGGL((dgrad_c1_kernel<CC, KK>), grid, dim3(256), 0, s, dy, N, H, W, wk, pad_mode, dx)
    if (C == 64 && K == 7) DCS_C1(64, 7);
    else if (C == 64 && K == 3) DCS_C1(64, 3);
    else if (C == 32 && K == 7) DCS_C1(32, 7);
    else if (C == 32 && K == 3) DCS_C1(32, 3);
    else return fail(DCS_E_INVALID, "conv_dgrad_c1: C must be 32 or 64 and K 3 or 7");
#undef DCS_C1
    return check_launch("conv_dgrad_c1");
}
