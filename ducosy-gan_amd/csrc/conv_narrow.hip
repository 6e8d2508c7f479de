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
__global__ __launch_bounds__(256) void narrow_rows_tiled_kernel(const dcs_conv_desc d, const float* __restrict__ src,
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
#pragma unroll
        for (int ty = 0; ty < KH; ++ty) {
            const float* row = lin + ((r + ty) * HW_ + cg * NT_XT) * NT_CC;
#pragma unroll
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

int narrow_wgrad_tiled_blocks(const dcs_conv_desc& d) {
    long long tiles = cdiv(d.Wo, NT_TW) * cdiv(d.Ho, NT_TH) * d.N;
    return (int)(tiles < 512 ? tiles : 512);
}

int launch_narrow_wgrad_tiled(const dcs_conv_desc& d, const float* dy, const float* src, const float* psc,
                              const float* psh, float* part, hipStream_t s) {
    const int tx = (int)cdiv(d.Wo, NT_TW), ty = (int)cdiv(d.Ho, NT_TH);
    hipLaunchKernelGGL((narrow_wgrad_tiled_kernel<7, 7, 8>), dim3(narrow_wgrad_tiled_blocks(d)), dim3(256), 0, s, d,
                       dy, src, psc, psh, part, tx, ty);
    return check_launch("narrow_wgrad_tiled");
}

}  // namespace dcs
