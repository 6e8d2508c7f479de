// Nearest-x2 upsample + 3x3 zero-pad convolution (the Generator's up-convolutions,
// modules/model.py:112-120 Upsample + Conv2d) on f16x3 operands, the source window of a tile staged once
// per 16-channel slice.
//
// Output pixel (2i + py, 2j + px) reads source rows {i - 1, i} (py = 0) or {i, i + 1} (py = 1) and
// likewise for columns: each of the four phases is a 2x2 convolution of the LOW-resolution source with
// weights that sum the 3x3 taps landing on the same source pixel (subpix_value, conv_common.hpp).
// conv.hip's rows pass runs the phases as four classes and gathers A per k-tile (every source value
// fetched and split four times per phase); here a workgroup owns 256 source pixels (R = 256 / TW rows
// of a TW-wide strip) x 128 virtual output columns, and per 16-channel slice stages the
// (R + 2) x (TW + 2) source window once (zero outside the image) for 2 phases x 4 taps.
//
// Virtual columns: a column tile is (px, 64-channel block); its halves are the row phases py = 0, 1.
// Waves w and w + 4 (one SIMD) own the same 64 pixels in the two row phases; each wave runs 4 taps
// (u, t) x 2 x 2 blocks x 3 products per slice, so no wave idles on a tap another phase needs.
// B arrives pre-split (dcs_pack_subpix_h3: hi / lo fp16 planes [4 Co][4 C], k = slice * 64 + u * 32 +
// t * 16 + c).  One fp32 chain per slice (64 k), added to the running sum (two-level, as conv.hip).
// LDS: window [2][2 planes][520 px][16] + B [2][2 planes][4 taps][128 rows x 16 + 48] halves (131 KB).
//
// Data gradient (MODE 1): dx[i][j] = sum over phases (py, px) and offsets (u, t) of
// dy[2 (i + 1 - py - u) + py][2 (j + 1 - px - t) + px] . W_phase[u][t]^T: per phase a 2x2 convolution of
// the phase's dy sub-grid (every other dy pixel) with the transposed phase weights.  The k loop runs
// over (phase, 16-channel slice of dy); each iteration stages the phase's (R + 1) x (TW + 1) dy window and
// its B slice, and every wave runs the 4 offsets of that phase (8 waves = 4 pixel x 2 channel blocks of
// a 256-pixel x 128-input-channel tile).
#include "common.hpp"
#include "conv_common.hpp"

#ifndef DCS_SP_BDMA  // B slices by LDS-DMA (global_load_lds_dwordx4) instead of registers + ds_write, and idle window
                     // units storing to a dummy slot so no load sinks into a branch: ~20 VGPRs fewer and every
                     // load issued at the top of the slice, bit-identical, but no faster per launch (kbench) and
                     // 0.5 % slower in the f16x3 step (profiles/r06/ab/r06ak_*): the phase kernels' 0.33 MFMA
                     // busy is not the staging loads' latency; off
#define DCS_SP_BDMA 0
#endif
#ifndef DCS_SP_PAIR_DG  // the up-conv data gradient paired too, with one window register set (two: 2-3 % slower):
                        // up1 / up2 data gradient 0.239 / 0.264 -> 0.230 / 0.250 ms per launch, bit-identical, step
                        // within noise (profiles/r06/ab/r06al_*)
#define DCS_SP_PAIR_DG 1
#endif
#ifndef DCS_SP_PAIR  // f16: two k iterations per barrier in the window phase kernel (0: one, as f16x3): 3-7 % per
                     // launch, bit-identical
#define DCS_SP_PAIR 1
#endif

namespace dcs {
namespace {

constexpr int SP_NT = 512, SP_BN = 128;
constexpr int SP_PIX = 520;                 // window pixels: (256 / TW + 2) * (TW + 2) <= 520 for 16 <= TW <= 128
constexpr int SP_SLOT = 128 * 16 + 48;      // halves per B tap slot (the four slots of a row on distinct banks)
constexpr int SP_UNITS = (2 * SP_PIX + SP_NT - 1) / SP_NT;

struct SubArgs {
    int N, Hs, Ws, C, Co;  // MODE 0: source NHWC [N][Hs][Ws][C], output [N][2 Hs][2 Ws][Co];
                           // MODE 1: dy [N][2 Hs][2 Ws][C], dx [N][Hs][Ws][Co]
    int R, TW, tiles_x, tiles;  // tile = R rows x TW columns of the source; tiles per row band / image
    int gy, cblk;          // column tiles (MODE 0: 4 Co / 128, MODE 1: Co / 128), 64-channel blocks (Co / 64)
    int rng_n;
    int pro_act;           // PRO: the source prologue's activation (DCS_ACT_AFFINE / _RELU / _LRELU)
};
constexpr int SP_PROC = 512;  // PRO: source channels the prologue table holds

// the InstanceNorm backward's partial sums of a data gradient's output da (a layer a = act(IN(y)) whose
// input gradient this is): per (chunk, channel) sum g and sum g * xhat, g = da * act'(xhat),
// xhat = y * scale + shift (the same quantities as conv_win.hip's IbwArgs)
struct PhIbw {
    const float* y;
    const float* sc;
    const float* sh;
    Sum2* parts;  // [N][nchunk][Co]
    int act;
};

// one global_load_lds_dwordx4 (lane L's 16 bytes at LDS byte address lds + 16 L; inline asm as
// conv_win.hip's win_glds: the kernel retires it with its own vmcnt wait before the publishing barrier)
__device__ __forceinline__ void sp_glds(const void* base, unsigned voff, unsigned lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(base), "s"(lds)
                 : "memory");
}

// window: pixel pairs swap on odd groups of 8 pixels, 16-byte halves on odd groups of 16 (conflict-free
// reads of every other pixel: the MFMA row blocks interleave, as conv_win.hip)
__device__ __forceinline__ int sp_woff(int buf, int pl, int wpix, int h) {
    return ((buf * 2 + pl) * SP_PIX + (wpix ^ ((wpix >> 3) & 1))) * 16 + 8 * (h ^ ((wpix >> 4) & 1));
}
__device__ __forceinline__ int sp_boff(int buf, int pl, int tap, int row, int h) {
    return ((buf * 2 + pl) * 4 + tap) * SP_SLOT + row * 16 + 8 * (h ^ ((row >> 3) & 1));
}

// NP 3: f16x3 (lo*hi + hi*lo + hi*hi), 1: f16 (hi planes only); MODE 0: phases over the output columns
// (sub-pixel forward; S2: the stride-2 data gradient), MODE 1: phases over k (sub-pixel data gradient;
// S2: the stride-2 forward).  S2 kernels skip the (phase, offset) pairs no 3x3 tap reaches (weights 0).
// PXC >= 0: the launch covers the column tiles of column phase PXC only (the stride-2 data gradient runs
// one launch per phase, so the phase's skipped column offset is known at compile time)
// PRO (MODE 1): the source is y of a layer a = act(y * scale + shift) (per image and channel, the
// PatchGAN's InstanceNorm + LeakyReLU): the window staging applies it, zero padding outside the image.
// IBW: the IN-backward partial sums of the output (data gradients; chunk = (tile, phase) as the statistics)
template <int NP, int MODE, int S2, int PXC = -1, int PRO = 0, int IBW = 0>
__global__ __launch_bounds__(SP_NT, 1) void subpix_win_kernel(SubArgs a, const float* __restrict__ src,
                                                              const _Float16* __restrict__ wh,
                                                              const _Float16* __restrict__ wl,
                                                              const float* __restrict__ rng,
                                                              const int* __restrict__ wexp, float* __restrict__ out,
                                                              Part* __restrict__ parts, const float* __restrict__ psc,
                                                              const float* __restrict__ psh, PhIbw ib) {
    // f16 (NP 1, DCS_SP_PAIR): a slice is only 16 MFMAs per wave, so two iterations run per barrier, the
    // second one's window and B in the planes f16x3 gives its lo halves (same sums in the same order)
    // Two window register sets (both loads in flight from the barrier) for the up-conv forward; the other
    // launches reuse one (the second window loaded after the first one's store): two spill in the stride-2
    // and prologue kernels and measured slower in the up-conv data gradient
    constexpr bool PAIR = NP == 1 && DCS_SP_PAIR && (MODE == 0 || S2 || DCS_SP_PAIR_DG);
    constexpr bool WR2 = !S2 && !PRO && MODE == 0;
    constexpr int NI = PAIR ? 2 : 1;  // iterations per barrier
    __shared__ __attribute__((aligned(16))) _Float16 smem[2 * 2 * SP_PIX * 16 + 2 * 2 * 4 * SP_SLOT];
    __shared__ __attribute__((aligned(16))) float pro_s[PRO ? 2 * SP_PROC : 4];  // [scale | shift][channel]
    _Float16* const Wn = smem;
    _Float16* const Bs = smem + 2 * 2 * SP_PIX * 16;

    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int gyl = PXC >= 0 ? a.cblk : a.gy;
    const int ntile = (PXC >= 0 ? PXC * a.cblk : 0) + L % gyl, mt = L / gyl;
    const int n = mt / a.tiles, tile = mt - n * a.tiles;
    const int tyi = tile / a.tiles_x, txi = tile - tyi * a.tiles_x;
    const int y0 = tyi * a.R, x0 = txi * a.TW;
    const int px = MODE == 0 ? ntile / a.cblk : 0, cb = ntile - px * a.cblk;
    const int n0 = ntile * SP_BN;  // first (virtual) B row of the tile
    const int TW = a.TW, WP = MODE == 0 ? a.TW + 2 : a.TW + 1, C = a.C;
    const int nslice = C / 16, nit = MODE == 0 ? nslice : 4 * nslice;
    const int K = 64 * nit;
    const int npix = (MODE == 0 ? a.R + 2 : a.R + 1) * WP;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid & 3, py = wid >> 2;  // MODE 1: py is the wave's 64-channel half of the tile
    const int l32 = lane & 31, kh = lane >> 5;

    // the source exponent (ea, asc) and the PRO table are read in the prologue, beside the first
    // staging loads
    int ea = 0;
    float asc = 1.f;
    const int eb = __builtin_amdgcn_readfirstlane(wexp[0]);

    // window staging units (pixel, 8-channel half).  MODE 0: byte offset of the unit's channel 0 (-1:
    // zero).  MODE 1: the byte offset of the unit's dy pixel (2 (y0 + row), 2 (x0 + column)) at phase
    // (0, 0), and in uvm the phases (qy, qx) whose pixel (2 (y0 + row) - qy, 2 (x0 + column) - qx) is in
    // the image (bit 2 qy + qx); a phase moves the pixel by a block-uniform (qy 2 Ws + qx) C * 4 bytes
    int uoff[SP_UNITS], uvm[SP_UNITS];
    const float rwp = 1.f / (float)WP;
#pragma unroll
    for (int q = 0; q < SP_UNITS; ++q) {
        const int u = tid + q * SP_NT;
        const int wpix = u >> 1, h = u & 1;
        uoff[q] = -1;
        uvm[q] = 0;
        if (wpix < npix) {
            // wpix / WP by a float reciprocal: exact, (wpix + 0.5) / WP stays >= 0.5 / WP from an integer
            const int wr = (int)(((float)wpix + 0.5f) * rwp), wc = wpix - wr * WP;
            if constexpr (MODE == 0) {
                const int sy = y0 - 1 + wr, sx = x0 - 1 + wc;
                if (sy >= 0 && sy < a.Hs && sx >= 0 && sx < a.Ws) uoff[q] = (((n * a.Hs + sy) * a.Ws + sx) * C + 8 * h) * 4;
            } else {
                uoff[q] = (((n * 2 * a.Hs + 2 * (y0 + wr)) * 2 * a.Ws + 2 * (x0 + wc)) * C + 8 * h) * 4;
#pragma unroll
                for (int ph = 0; ph < 4; ++ph) {
                    const int cy = y0 - (ph >> 1) + wr, cx = x0 - (ph & 1) + wc;
                    if (cy >= 0 && cy < a.Hs && cx >= 0 && cx < a.Ws) uvm[q] |= 1 << ph;
                }
            }
        }
    }
    const __amdgpu_buffer_rsrc_t srsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, 0x7fffff00, 0x00020000);
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    constexpr int NWR = PAIR && WR2 ? 2 : 1;
    float4 wr_[NWR][SP_UNITS][2];
    int vmask[NWR] = {}, vit[NWR] = {};  // PRO: the staged units inside the image, and their iteration
    auto unit_off = [&](int q, int it) {  // byte offset of unit q's 8 channels at iteration it (OOB: zero)
        if constexpr (MODE == 0) {
            return uoff[q] >= 0 ? uoff[q] + it * 64 : 0x7fffffbf;
        } else {
            const int ph = it / nslice, s = it - ph * nslice;  // (block-uniform)
            const int pshift = (s * 16 - ((ph >> 1) * 2 * a.Ws + (ph & 1)) * C) * 4;
            return (uvm[q] >> ph) & 1 ? uoff[q] + pshift : 0x7fffffbf;
        }
    };
    auto win_load = [&](int it, int p) {  // into register set p
        if constexpr (PRO) { vmask[p] = 0; vit[p] = it; }
#pragma unroll
        for (int q = 0; q < SP_UNITS; ++q) {
            const int off = unit_off(q, it);
            if constexpr (PRO) vmask[p] |= (off != 0x7fffffbf) << q;
            u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(srsrc, off, 0, 0);
            u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(srsrc, off + 16, 0, 0);
            __builtin_memcpy(&wr_[p][q][0], &v0, 16);
            __builtin_memcpy(&wr_[p][q][1], &v1, 16);
        }
    };
    auto win_store = [&](int buf, int p, int pl) {  // register set p: the hi plane into plane pl, f16x3 also the lo
#pragma unroll
        for (int q = 0; q < SP_UNITS; ++q) {
            const int u = tid + q * SP_NT;
            const int wpix = u >> 1, h = u & 1;
            float4 (&wr)[2] = wr_[p][q];
            // DCS_SP_BDMA: idle units store too, into the B tap slot's padding (never read): a store under a
            // branch lets the compiler sink the unit's load into the branch, right before its wait
            const bool live = wpix < npix;
            if (DCS_SP_BDMA || live) {
                if constexpr (PRO) {  // a = act(y * scale + shift) inside the image, 0 in the padding
                    const int c0 = (vit[p] % nslice) * 16 + 8 * h;
                    const float4 s0 = *reinterpret_cast<const float4*>(pro_s + c0);
                    const float4 s1 = *reinterpret_cast<const float4*>(pro_s + c0 + 4);
                    const float4 b0 = *reinterpret_cast<const float4*>(pro_s + SP_PROC + c0);
                    const float4 b1 = *reinterpret_cast<const float4*>(pro_s + SP_PROC + c0 + 4);
                    const bool ok = (vmask[p] >> q) & 1;
                    auto f = [&](float v, float sc, float sh) { return ok ? act_apply(fmaf(v, sc, sh), a.pro_act) : 0.f; };
                    wr[0] = make_float4(f(wr[0].x, s0.x, b0.x), f(wr[0].y, s0.y, b0.y),
                                        f(wr[0].z, s0.z, b0.z), f(wr[0].w, s0.w, b0.w));
                    wr[1] = make_float4(f(wr[1].x, s1.x, b1.x), f(wr[1].y, s1.y, b1.y),
                                        f(wr[1].z, s1.z, b1.z), f(wr[1].w, s1.w, b1.w));
                }
                f16x8 hi, lo;
                split8h(wr[0], wr[1], asc, hi, lo);
                constexpr int DUMMY = 2 * 2 * SP_PIX * 16 + 128 * 16;  // (buffer 0, plane 0, tap 0) padding row
                *reinterpret_cast<f16x8*>(Wn + (live ? sp_woff(buf, pl, wpix, h) : DUMMY)) = hi;
                if constexpr (NP == 3) *reinterpret_cast<f16x8*>(Wn + (live ? sp_woff(buf, 1, wpix, h) : DUMMY)) = lo;
            }
        }
    };
    // B slice: 2 planes x 128 rows x 64 k = 2048 16-byte chunks, 4 per thread (chunks 0, 1 the hi
    // plane, 2, 3 the lo plane: f16 loads only the first two); chunk -> (plane, row, tap, half) with
    // (tap, half) fastest (the 128 contiguous bytes of a row).  S2: the chunks of (row, tap) pairs the
    // MFMA loop skips load nothing (an out-of-range buffer offset reads zero without a fetch): 7 of the
    // 16 (phase, tap) pairs of the forward, up to 5 of 8 of a data gradient launch.  PAIR: chunks 2, 3
    // are the hi plane of the next iteration (clamped to the last)
    constexpr int NBC = NP == 3 || PAIR ? 4 : 2;
    const __amdgpu_buffer_rsrc_t bhr = __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16*>(wh), (short)0, 0x7fffff00, 0x00020000);
    const __amdgpu_buffer_rsrc_t blr = __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16*>(NP == 3 ? wl : wh), (short)0, 0x7fffff00, 0x00020000);
    int bg[NBC], bl[NBC], bt[NBC];
#pragma unroll
    for (int i = 0; i < NBC; ++i) {
        const int q = tid + i * SP_NT;
        const int pl = q >> 10, rem = q & 1023;
        const int row = rem >> 3, c8 = rem & 7;
        bg[i] = ((n0 + row) * K + c8 * 8) * 2;  // byte offset in the plane
        bl[i] = sp_boff(0, pl, c8 >> 1, row, c8 & 1);
        bt[i] = (c8 >> 1) | ((row >> 6) << 2);  // tap (u, t) and the row's 64-row half (MODE 0: py)
    }
    u32x4 br[NBC];
    auto b_load = [&](int it0) {
#pragma unroll
        for (int i = 0; i < NBC; ++i) {
            const int it = PAIR && i >= 2 ? (it0 + 1 < nit ? it0 + 1 : it0) : it0;
            const int kb = it * 128;  // bytes
            bool skip = false;
            if constexpr (S2) {
                const int u = (bt[i] >> 1) & 1, t = bt[i] & 1;
                if constexpr (MODE == 0) {
                    skip = ((bt[i] >> 2) == 0 && u == 0) || (PXC == 0 && t == 0);
                } else {
                    const int ph = it / nslice;
                    skip = ((ph >> 1) == 0 && u == 1) || ((ph & 1) == 0 && t == 1);
                }
            }
            br[i] = __builtin_amdgcn_raw_buffer_load_b128(i < 2 ? bhr : blr, skip ? 0x7fffffbf : bg[i] + kb, 0, 0);
        }
    };
    // DCS_SP_BDMA: the same slice as 1 KB blocks (plane, tap, 32-row block) by LDS-DMA, NBC per wave
    // (block c = wave * NBC + i).  A block's LDS image is lane-linear (lane L -> row L / 2, half slot L % 2),
    // so sp_boff's swizzle moves to the source: lane L fetches half (L % 2) ^ bit 3 of its row.  S2: the
    // blocks of skipped (row half, tap) pairs are not fetched (wave-uniform; the MFMA loop never reads them)
    constexpr bool BDMA = DCS_SP_BDMA;
    const unsigned dlane = 2u * (unsigned)((n0 + (lane >> 1)) * K + 8 * ((lane & 1) ^ ((lane >> 4) & 1)));
    unsigned dsu[NBC], ddst[NBC];
    int dbt[NBC], dpl[NBC];
    {
        const unsigned bs_lds = (unsigned)(uintptr_t)(__attribute__((address_space(3))) _Float16*)Bs;
        const int w = __builtin_amdgcn_readfirstlane(wid);
#pragma unroll
        for (int i = 0; i < NBC; ++i) {
            const int c = w * NBC + i, pl = c >> 4, tap = (c >> 2) & 3, rb = c & 3;
            dsu[i] = 2u * (unsigned)(rb * 32 * K + tap * 16);
            ddst[i] = __builtin_amdgcn_readfirstlane(bs_lds + 2u * (unsigned)((pl * 4 + tap) * SP_SLOT + rb * 32 * 16));
            dbt[i] = tap | ((rb >> 1) << 2);  // as bt: tap (u, t) and the 64-row half
            dpl[i] = pl;
        }
    }
    auto b_dma = [&](int it0, int buf) {  // slice it0 (PAIR: and it0 + 1 in plane 1) into buffer buf
#pragma unroll
        for (int i = 0; i < NBC; ++i) {
            const int it = PAIR && dpl[i] ? (it0 + 1 < nit ? it0 + 1 : it0) : it0;
            bool skip = false;
            if constexpr (S2) {
                const int u = (dbt[i] >> 1) & 1, t = dbt[i] & 1;
                if constexpr (MODE == 0) {
                    skip = ((dbt[i] >> 2) == 0 && u == 0) || (PXC == 0 && t == 0);
                } else {
                    const int ph = it / nslice;
                    skip = ((ph >> 1) == 0 && u == 1) || ((ph & 1) == 0 && t == 1);
                }
            }
            if (!skip)
                sp_glds(NP == 3 && dpl[i] ? wl : wh, dlane + (dsu[i] + 2u * (unsigned)(it * 64)),
                        ddst[i] + 2u * (unsigned)(buf * 8 * SP_SLOT));
        }
    };
    auto b_store = [&](int buf) {
        const int boff = buf * 8 * SP_SLOT;
#pragma unroll
        for (int i = 0; i < NBC; ++i) *reinterpret_cast<u32x4*>(Bs + boff + bl[i]) = br[i];
    };

    // row block i holds source pixels 2m + i of the wave's 64 (TW even: a pair shares a row), so block 0
    // at column offset t + 1 reads the fragment block 1 reads at t.  Window pixel of the lane's block-0
    // pixel at tap (u, t) = (0, 0): MODE 0 (phase (py, px)): window row qy + py + u, column qx + px + t;
    // MODE 1 (window offset (o_r, o_c) = (1 - u, 1 - t)): row qy + o_r, column qx + o_c
    int wbe;
    {
        const int q = wm * 64 + 2 * l32;
        const int qy = q >> __builtin_ctz(TW);
        wbe = MODE == 0 ? (qy + py) * WP + (q - qy * TW) + px : qy * WP + (q - qy * TW);
    }

    floatx16 acc[2][2], t[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) { acc[i][j][r] = 0.f; t[i][j][r] = 0.f; }

    // prologue: every load of iteration 0 (and the exponent's, the PRO table's) in flight before the
    // first store
    win_load(0, 0);
    if constexpr (PAIR && WR2) win_load(nit > 1 ? 1 : 0, 1);
    if constexpr (BDMA) b_dma(0, 0);
    else b_load(0);
    if constexpr (PRO) {  // the image's prologue scale / shift (published by the barrier below)
        for (int c = tid; c < C; c += SP_NT) {
            pro_s[c] = psc[(long long)n * C + c];
            pro_s[SP_PROC + c] = psh[(long long)n * C + c];
        }
        __syncthreads();
    }
    ea = f16x3_exp(rng, a.rng_n);
    asc = __builtin_ldexpf(1.f, ea);
    win_store(0, 0, 0);
    if constexpr (PAIR && !WR2) win_load(nit > 1 ? 1 : 0, 0);
    if constexpr (PAIR) win_store(0, WR2 ? 1 : 0, 1);
    if constexpr (BDMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else b_store(0);
    __syncthreads();

    f16x8 fh[3], fl[3];
    // one k iteration s (its hi plane pl) over the staged buffer
    auto iter = [&](int buf, int s, int pl) {
    #pragma unroll
            for (int tap = 0; tap < 4; ++tap) {
                const int u = tap >> 1, tx = tap & 1;
                // S2: the pairs no tap reaches (wave-uniform: py per wave, px per workgroup, the class per
                // iteration)
                bool skip_row = false, skip_col = false;
                if constexpr (S2 && MODE == 0) {
                    skip_row = py == 0 && u == 0;
                    skip_col = PXC == 0 && tx == 0;  // (both runtime: the allocator spills)
                } else if constexpr (S2) {
                    const int ph = s / nslice;
                    skip_row = (ph >> 1) == 0 && u == 1;
                    skip_col = (ph & 1) == 0 && tx == 1;
                }
                if (skip_row) continue;
                f16x8 ah[2], al[2], bh[2], bl_[2];
                if (tx == 0) {  // fragments of window pixels wbe + u * WP + 0 .. 2 (block i, offset t: f = t + i)
    #pragma unroll
                    for (int f = 0; f < 3; ++f) {
                        const int wpix = wbe + u * WP + f;
                        fh[f] = *reinterpret_cast<const f16x8*>(Wn + sp_woff(buf, pl, wpix, kh));
                        if constexpr (NP == 3) fl[f] = *reinterpret_cast<const f16x8*>(Wn + sp_woff(buf, 1, wpix, kh));
                    }
                }
                if (skip_col) continue;
    #pragma unroll
                for (int i = 0; i < 2; ++i) {
                    ah[i] = fh[tx + i];
                    if constexpr (NP == 3) al[i] = fl[tx + i];
                }
    #pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int row = py * 64 + j * 32 + l32;
                    bh[j] = *reinterpret_cast<const f16x8*>(Bs + sp_boff(buf, pl, tap, row, kh));
                    if constexpr (NP == 3) bl_[j] = *reinterpret_cast<const f16x8*>(Bs + sp_boff(buf, 1, tap, row, kh));
                }
    #pragma unroll
                for (int i = 0; i < 2; ++i)
    #pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        if constexpr (NP == 3) {
                            t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], t[i][j], 0, 0, 0);
                            t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl_[j], t[i][j], 0, 0, 0);
                        }
                        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], t[i][j], 0, 0, 0);
                    }
            }
    };
    if constexpr (!PAIR) {
        for (int s = 0; s < nit; ++s) {
            const int buf = s & 1, sn = s + 1 < nit ? s + 1 : s;
            win_load(sn, 0);  // unconditional (clamped): a load under a branch would force vmcnt(0) below
            if constexpr (BDMA) b_dma(sn, buf ^ 1);
            else b_load(sn);
    #pragma unroll
            for (int tap = 0; tap < 4; ++tap) {
                const int u = tap >> 1, tx = tap & 1;
                // S2: the pairs no tap reaches (wave-uniform: py per wave, px per workgroup, the class per
                // iteration)
                bool skip_row = false, skip_col = false;
                if constexpr (S2 && MODE == 0) {
                    skip_row = py == 0 && u == 0;
                    skip_col = PXC == 0 && tx == 0;  // (both runtime: the allocator spills)
                } else if constexpr (S2) {
                    const int ph = s / nslice;
                    skip_row = (ph >> 1) == 0 && u == 1;
                    skip_col = (ph & 1) == 0 && tx == 1;
                }
                if (skip_row) continue;
                f16x8 ah[2], al[2], bh[2], bl_[2];
                if (tx == 0) {  // fragments of window pixels wbe + u * WP + 0 .. 2 (block i, offset t: f = t + i)
    #pragma unroll
                    for (int f = 0; f < 3; ++f) {
                        const int wpix = wbe + u * WP + f;
                        fh[f] = *reinterpret_cast<const f16x8*>(Wn + sp_woff(buf, 0, wpix, kh));
                        if constexpr (NP == 3) fl[f] = *reinterpret_cast<const f16x8*>(Wn + sp_woff(buf, 1, wpix, kh));
                    }
                }
                if (skip_col) continue;
    #pragma unroll
                for (int i = 0; i < 2; ++i) {
                    ah[i] = fh[tx + i];
                    if constexpr (NP == 3) al[i] = fl[tx + i];
                }
    #pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int row = py * 64 + j * 32 + l32;
                    bh[j] = *reinterpret_cast<const f16x8*>(Bs + sp_boff(buf, 0, tap, row, kh));
                    if constexpr (NP == 3) bl_[j] = *reinterpret_cast<const f16x8*>(Bs + sp_boff(buf, 1, tap, row, kh));
                }
    #pragma unroll
                for (int i = 0; i < 2; ++i)
    #pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        if constexpr (NP == 3) {
                            t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], t[i][j], 0, 0, 0);
                            t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl_[j], t[i][j], 0, 0, 0);
                        }
                        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], t[i][j], 0, 0, 0);
                    }
            }
            // the other buffers were last read before the previous barrier
            win_store(buf ^ 1, 0, 0);
            if constexpr (BDMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            else b_store(buf ^ 1);
            __syncthreads();
            if ((s & 1) || s + 1 == nit) {  // close the accumulation chain every two iterations (128 k)
    #pragma unroll
                for (int i = 0; i < 2; ++i)
    #pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        acc[i][j] += t[i][j];
    #pragma unroll
                        for (int r = 0; r < 16; ++r) t[i][j][r] = 0.f;
                    }
            }
        }
    } else {
        for (int s0 = 0; s0 < nit; s0 += NI) {
            const int buf = (s0 / NI) & 1, sn = s0 + NI < nit ? s0 + NI : s0, sn1 = sn + 1 < nit ? sn + 1 : sn;
            win_load(sn, 0);  // unconditional (clamped): a load under a branch would force vmcnt(0) below
            if constexpr (PAIR && WR2) win_load(sn1, 1);
            if constexpr (BDMA) b_dma(sn, buf ^ 1);
            else b_load(sn);
            iter(buf, s0, 0);
            // the other buffers were last read before the previous barrier
            win_store(buf ^ 1, 0, 0);
            if constexpr (PAIR && !WR2) win_load(sn1, 0);  // (one register set: the second window after the first's store)
            if constexpr (PAIR) {
                if (s0 + 1 < nit) iter(buf, s0 + 1, 1);  // (block-uniform)
                win_store(buf ^ 1, WR2 ? 1 : 0, 1);
            }
            if constexpr (BDMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            else b_store(buf ^ 1);
            __syncthreads();
            const int s = s0 + NI - 1;  // the barrier's last iteration
            if ((s & 1) || s + 1 >= nit) {  // close the accumulation chain every two iterations (128 k)
    #pragma unroll
                for (int i = 0; i < 2; ++i)
    #pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        acc[i][j] += t[i][j];
    #pragma unroll
                        for (int r = 0; r < 16; ++r) t[i][j][r] = 0.f;
                    }
            }
        }
    }

    // epilogue: undo the operand scales, NHWC store, IN statistics.  MODE 0: the phase's pixels of the
    // 2 Hs x 2 Ws output, channels co0 + j * 32 + lane; MODE 1: the Hs x Ws output, channels n0 + py * 64 + ...
    const int eab = -(ea + eb);
    const int Wo = MODE == 0 ? 2 * a.Ws : a.Ws;
    // output pixel index within the image (increasing along r, then i); TW is a power of two and
    // every product below fits 24 bits (index math off the slow 32-bit multiplier)
    const int tws = __builtin_ctz(TW);
    auto opix = [&](int i, int r) {
        const int q = wm * 64 + 2 * ((r & 3) + 8 * (r >> 2) + 4 * kh) + i;
        const int qy = q >> tws, qx = q & (TW - 1);
        if constexpr (MODE == 0) return (int)__umul24(2 * (y0 + qy) + py, Wo) + 2 * (x0 + qx) + px;
        else return (int)__umul24(y0 + qy, Wo) + x0 + qx;
    };
    const long long obase = (long long)n * (MODE == 0 ? 4LL : 1LL) * a.Hs * a.Ws * a.Co;
    float* const outn = out + obase;  // the image's output (32-bit offsets below)
    const int co0 = MODE == 0 ? cb * 64 : n0 + py * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                acc[i][j][r] = __builtin_ldexpf(acc[i][j][r], eab);
                outn[(int)__umul24(opix(i, r), a.Co) + co0 + j * 32 + l32] = acc[i][j][r];
            }
    if constexpr (IBW) {  // per WG column: sums over the wave's 64 pixels, then the 4 pixel waves in order
        Sum2* ss = reinterpret_cast<Sum2*>(smem);  // [4][128]; the loop's last barrier freed the LDS
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int ch = co0 + j * 32 + l32;
            const float sc = ib.sc[(long long)n * a.Co + ch], sh = ib.sh[(long long)n * a.Co + ch];
            float yv[2][16];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) yv[i][r] = ib.y[obase + (int)__umul24(opix(i, r), a.Co) + ch];
            float sa = 0.f, sb = 0.f;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float xh = fmaf(yv[i][r], sc, sh);
                    const float g = acc[i][j][r] * act_grad(xh, ib.act);
                    sa += g;
                    sb = fmaf(g, xh, sb);
                }
            sa += __shfl_xor(sa, 32, 64);  // the same operand pair on both lanes: order-free
            sb += __shfl_xor(sb, 32, 64);
            if (kh == 0) ss[wm * SP_BN + py * 64 + j * 32 + l32] = Sum2{sa, sb};
        }
        __syncthreads();
        if (tid < SP_BN) {
            Sum2 t = ss[tid];
#pragma unroll
            for (int w = 1; w < 4; ++w) {
                t.a += ss[w * SP_BN + tid].a;
                t.b += ss[w * SP_BN + tid].b;
            }
            if constexpr (MODE == 0)
                ib.parts[((long long)n * 4 * a.tiles + tile * 4 + px * 2 + (tid >> 6)) * a.Co + co0 + (tid & 63)] = t;
            else
                ib.parts[((long long)n * a.tiles + tile) * a.Co + n0 + tid] = t;
        }
        return;
    }
    if (!parts) return;  // kernel argument: block-uniform
    // per virtual column: count / mean / M2 / max / first argmax over the wave's 64 pixels, then the
    // four pixel waves merged in a fixed order; chunk = (tile, px, py) of the image
    Part* sp = reinterpret_cast<Part*>(smem);  // [4][128]; the loop's last barrier freed the LDS
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        float s = 0.f, mx = -INFINITY;
        int am = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r)  // increasing pixel order (first maximum)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const float v = acc[i][j][r];
                s += v;
                if (v > mx) { mx = v; am = opix(i, r); }
            }
        const float mean = s * (1.f / 32.f);
        float m2 = 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float dv = acc[i][j][r] - mean;
                m2 = fmaf(dv, dv, m2);
            }
        const float mb = __shfl_xor(mean, 32, 64), m2b = __shfl_xor(m2, 32, 64), mxb = __shfl_xor(mx, 32, 64);
        const int amb = __shfl_xor(am, 32, 64);
        if (kh == 0) {
            const float dl = mb - mean;
            Part p;
            p.cnt = 64.f;
            p.mean = mean + 0.5f * dl;
            p.m2 = m2 + m2b + dl * dl * 16.f;
            p.mx = mx;
            p.amax = am;
            if (mxb > mx || (mxb == mx && amb < am)) { p.mx = mxb; p.amax = amb; }
            p.pad[0] = p.pad[1] = p.pad[2] = 0;
            sp[wm * SP_BN + py * 64 + j * 32 + l32] = p;
        }
    }
    __syncthreads();
    if (tid < SP_BN) {
        Part p = sp[tid];
#pragma unroll
        for (int w = 1; w < 4; ++w) {
            const Part b = sp[w * SP_BN + tid];
            const float tot = p.cnt + b.cnt, dl = b.mean - p.mean;
            p.mean += dl * (b.cnt / tot);
            p.m2 += b.m2 + dl * dl * (p.cnt * b.cnt / tot);
            p.cnt = tot;
            if (b.mx > p.mx || (b.mx == p.mx && b.amax < p.amax)) { p.mx = b.mx; p.amax = b.amax; }
        }
        if constexpr (MODE == 0) {
            const int nchunk = 4 * a.tiles;
            const int chunk = tile * 4 + px * 2 + (tid >> 6);
            parts[((long long)n * nchunk + chunk) * a.Co + co0 + (tid & 63)] = p;
        } else {
            parts[((long long)n * a.tiles + tile) * a.Co + n0 + tid] = p;
        }
    }
}

// sub-pixel B pack: the range of the combined weights, then every block derives the exponent and
// writes the hi / lo planes ([4 Cout][4 Cin] forward, [Cin][16 Cout] data gradient)
__global__ __launch_bounds__(256) void subpix_range_kernel(const float* __restrict__ w, int Cout, int Cin, int kind,
                                                           float* __restrict__ parts) {
    const long long total = 16LL * Cout * Cin;
    const int K = subpix_K(Cout, Cin, kind);
    float m = 0.f;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
        const int v = (int)(i / K);
        m = fmaxf(m, fabsf(subpix_value(w, Cout, Cin, kind, v, (int)(i - (long long)v * K))));
    }
    __shared__ float red[4];
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) parts[blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (blockIdx.x == 0)
        for (int i = gridDim.x + threadIdx.x; i < DCS_RANGE_PARTS; i += blockDim.x) parts[i] = 0.f;
}

__global__ __launch_bounds__(256) void subpix_pack_kernel(const float* __restrict__ w, int Cout, int Cin, int kind,
                                                          const float* __restrict__ parts,
                                                          _Float16* __restrict__ oh, _Float16* __restrict__ ol,
                                                          int* __restrict__ wexp) {
    const int e = f16x3_exp(parts, DCS_RANGE_PARTS);
    const float sc = __builtin_ldexpf(1.f, e);
    if (blockIdx.x == 0 && threadIdx.x == 0) wexp[0] = e;
    const long long total = 16LL * Cout * Cin;
    const int K = subpix_K(Cout, Cin, kind);
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
        const int v = (int)(i / K);
        const float f = subpix_value(w, Cout, Cin, kind, v, (int)(i - (long long)v * K)) * sc;
        const _Float16 h = (_Float16)f;
        oh[i] = h;
        ol[i] = (_Float16)(f - (float)h);
    }
}

// ---------------------------------------------------------------------------------------
// Weight gradient of the up-convolutions on a rolling source window (f16x3), per phase:
//   dWp[py][px][u][t][co][ci] = sum_{i, j} dy[2i + py][2j + px][co] * src[i + py + u - 1][j + px + t - 1][ci]
// folded onto the 3x3 taps by conv.hip's wgrad_subpixel_fold_kernel (slabs [split][phase][co][(u, t), ci]).
// conv.hip's x6 weight gradient runs the phases as four classes of a 128 x 128 (co, (tap, ci)) tile and
// gathers the source per tap column group.  Here a workgroup owns 32 co x 64 ci x all 16 (phase, tap)
// pairs and walks a 64-pixel-wide strip of the low-resolution grid row by row: per row it stages the two
// dy rows of the strip (128 px each, de-interleaved by column phase) and ONE new source row segment
// (66 px with the halo) into a ring of four rows, split into hi / lo fp16 once; wave (phase, ci block)
// reads its dy fragment once per 16-pixel sub-tile and its four taps' source fragments at a per-tap
// (ring slot, pixel) offset.  MFMA: M = co (32), N = ci (32), K = 16 low-resolution pixels; fragments
// by ds_read_b64_tr_b16 as conv_win.hip's weight gradient (source ring: its 64-channel swizzled
// layout; dy: 32-channel rows, conflict-free unswizzled).  Two-level accumulation over row pairs.
constexpr int SW_NT = 512, SW_SW = 64, SW_WP = SW_SW + 2;
constexpr int SW_XROW = 2 * SW_WP * 64;      // halves per ring slot (2 planes x 66 px x 64 ci)
constexpr int SW_DPH = 2 * SW_SW * 32;       // halves per (py, px) dy region (2 planes x 64 px x 32 co)
constexpr int SW_DBUF = 4 * SW_DPH;          // halves per dy buffer (4 phases)
constexpr int SW_XU = (SW_WP * 8 + SW_NT - 1) / SW_NT;  // source-row (pixel, 8-channel unit)s per thread: 2

struct SWArgs {
    int N, H, W, C, Co;  // source NHWC [N][H][W][C] (low resolution); dy NHWC [N][2H][2W][Co]
    int strips, rchunks, rows_per;
    int gco, gci;        // 32-channel co tiles, 64-channel ci tiles
    int rng_a_n, rng_b_n;
};

__device__ __forceinline__ int sw_swz(int pix) { return ((pix >> 1) & 1) << 2; }

typedef short swshortx4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) swshortx4 lds_swshortx4;

// fragment of 8 consecutive pixels of one channel per lane from a pixel-major image of `pitch` halves
// per pixel (two transposed 4-pixel reads)
template <int PITCH>
__device__ __forceinline__ f16x8 sw_frag(const _Float16* p) {
    const swshortx4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_swshortx4*)(p));
    const swshortx4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_swshortx4*)(p + 4 * PITCH));
    return __builtin_bit_cast(f16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int NP>
__global__ __launch_bounds__(SW_NT, 1) void subpix_wgrad_kernel(SWArgs a, const float* __restrict__ dy,
                                                                const float* __restrict__ src,
                                                                const float* __restrict__ rnga,
                                                                const float* __restrict__ rngb,
                                                                float* __restrict__ ws) {
    __shared__ __attribute__((aligned(16))) _Float16 smem[4 * SW_XROW + 2 * SW_DBUF];
    _Float16* const Xr = smem;                 // [4][2][66][64]
    _Float16* const Dy = smem + 4 * SW_XROW;   // [2][py][px][2][64][32]

    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int ntile = a.gco * a.gci;
    const int tile = L % ntile, split = L / ntile;
    const int co0 = (tile % a.gco) * 32, ci0 = (tile / a.gco) * 64;
    const int rc = split % a.rchunks, rest = split / a.rchunks;
    const int strip = rest % a.strips, n = rest / a.strips;
    const int x0 = strip * SW_SW;
    const int H = a.H, W = a.W, C = a.C, Co = a.Co;
    const int y_beg = rc * a.rows_per;
    const int y_end = y_beg + a.rows_per < H ? y_beg + a.rows_per : H;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int cib = wid & 1, ph = wid >> 1, py = ph >> 1, px = ph & 1;

    const int ea = f16x3_exp(rnga, a.rng_a_n), eb = f16x3_exp(rngb, a.rng_b_n);
    const float asc = __builtin_ldexpf(1.f, ea), bsc = __builtin_ldexpf(1.f, eb);

    const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dy), (short)0, 0x7fffff00, 0x00020000);
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, 0x7fffff00, 0x00020000);
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    constexpr int OOB = 0x7fffffbf;

    // dy: 2 rows x 128 px x 4 units (8 co) = 1024 units, 2 per thread: unit -> (row phase, column
    // phase, low-res pixel j, unit) with the unit fastest, then j (8 lanes write 128 contiguous bytes)
    int doff[2], dls[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int u = tid + q * SW_NT;
        const int cu = u & 3, j = (u >> 2) & 63, qx = (u >> 8) & 1, qy = u >> 9;
        doff[q] = (qy * 2 * W + 2 * (x0 + j) + qx) * Co * 4 + (co0 + 8 * cu) * 4;  // + row 2y base
        dls[q] = (qy * 2 + qx) * SW_DPH + j * 32 + 8 * cu;
    }
    // source row segment: 66 px (halo included) x 8 units; byte offset within the row (-1: none)
    int xoff[SW_XU], xls[SW_XU];
#pragma unroll
    for (int q = 0; q < SW_XU; ++q) {
        const int u = tid + q * SW_NT, wc = u >> 3, cu = u & 7;
        xoff[q] = -1;
        xls[q] = -1;
        if (wc < SW_WP) {
            const int sx = x0 - 1 + wc;
            if (sx >= 0 && sx < W) xoff[q] = (sx * C + ci0 + 8 * cu) * 4;
            xls[q] = wc * 64 + 8 * (cu ^ sw_swz(wc));
        }
    }
    float4 dr[2][2], xr[SW_XU][2];
    auto ld_dy = [&](int y) {  // dy rows 2y, 2y + 1
        const int rb = ((n * 2 * H + 2 * y) * 2 * W) * Co * 4;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(drs, rb + doff[q], 0, 0);
            u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(drs, rb + doff[q] + 16, 0, 0);
            __builtin_memcpy(&dr[q][0], &v0, 16);
            __builtin_memcpy(&dr[q][1], &v1, 16);
        }
    };
    auto ld_x = [&](int r) {  // logical source row r in [-1, H]: zero outside the image
        const bool ok = r >= 0 && r < H;
        const int rb = ((n * H + (ok ? r : 0)) * W) * C * 4;
#pragma unroll
        for (int q = 0; q < SW_XU; ++q) {
            const int off = (ok && xoff[q] >= 0) ? rb + xoff[q] : OOB;
            u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0);
            u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(xrs, off + 16, 0, 0);
            __builtin_memcpy(&xr[q][0], &v0, 16);
            __builtin_memcpy(&xr[q][1], &v1, 16);
        }
    };
    auto st_dy = [&](int buf) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            f16x8 hi, lo;
            split8h(dr[q][0], dr[q][1], asc, hi, lo);
            *reinterpret_cast<f16x8*>(Dy + buf * SW_DBUF + dls[q]) = hi;
            if constexpr (NP == 3) *reinterpret_cast<f16x8*>(Dy + buf * SW_DBUF + dls[q] + SW_SW * 32) = lo;
        }
    };
    auto st_x = [&](int slot) {
#pragma unroll
        for (int q = 0; q < SW_XU; ++q) {
            if (xls[q] >= 0) {
                f16x8 hi, lo;
                split8h(xr[q][0], xr[q][1], bsc, hi, lo);
                *reinterpret_cast<f16x8*>(Xr + slot * SW_XROW + xls[q]) = hi;
                if constexpr (NP == 3) *reinterpret_cast<f16x8*>(Xr + slot * SW_XROW + SW_WP * 64 + xls[q]) = lo;
            }
        }
    };

    // transposed-read lane offsets (halves), as conv_win.hip's weight gradient
    const int g16 = lane >> 4;
    const int rpix = 8 * (g16 >> 1) + ((lane & 15) >> 2);
    const int rcol = 16 * (g16 & 1) + 4 * (lane & 3);
    const int aoff = ph * SW_DPH + rpix * 32 + rcol;  // dy region of the wave's phase, its 32 co
    int boff[2];
    {
        const int cb = 32 * cib + rcol;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int p = rpix + px + t;  // window column j + px + t
            boff[t] = p * 64 + 8 * ((cb >> 3) ^ sw_swz(p)) + (cb & 7);
        }
    }

    floatx16 acc[4], tq[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) { acc[i][r] = 0.f; tq[i][r] = 0.f; }

    // prologue: source rows y_beg-1 .. y_beg+1 into their ring slots, dy rows of y_beg into buffer 0
#pragma unroll 1
    for (int r = y_beg - 1; r <= y_beg + 1; ++r) {
        ld_x(r);
        st_x(r & 3);
    }
    ld_dy(y_beg);
    st_dy(y_beg & 1);
    __syncthreads();

#pragma unroll 1
    for (int y = y_beg; y < y_end; ++y) {
        ld_dy(y + 1 < y_end ? y + 1 : y);  // unconditional (clamped / zero past the image)
        ld_x(y + 2);
        const _Float16* const Db = Dy + (y & 1) * SW_DBUF;
        const _Float16* Xs[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) Xs[u] = Xr + ((y + 3 + py + u) & 3) * SW_XROW;  // row y + py + u - 1
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // 16-pixel sub-tiles of the strip
            f16x8 ah, al;
            ah = sw_frag<32>(Db + aoff + k * 16 * 32);
            if constexpr (NP == 3) al = sw_frag<32>(Db + SW_SW * 32 + aoff + k * 16 * 32);
#pragma unroll
            for (int tap = 0; tap < 4; ++tap) {
                const int u = tap >> 1, t = tap & 1;
                f16x8 bh, bl;
                bh = sw_frag<64>(Xs[u] + boff[t] + k * 16 * 64);
                if constexpr (NP == 3) {
                    bl = sw_frag<64>(Xs[u] + SW_WP * 64 + boff[t] + k * 16 * 64);
                    tq[tap] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, tq[tap], 0, 0, 0);
                    tq[tap] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, tq[tap], 0, 0, 0);
                }
                tq[tap] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, tq[tap], 0, 0, 0);
            }
            // stage the rows loaded above into the buffers this row does not read: mid-row (f16x3), or
            // after the row's MFMAs (f16: a third of the MFMAs hid too little of the loads' latency)
            if (k == (NP == 1 ? 3 : 1)) {
                st_dy((y + 1) & 1);
                st_x((y + 2) & 3);
            }
        }
        if (((y - y_beg) & 1) == 1 || y + 1 == y_end) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                acc[i] += tq[i];
#pragma unroll
                for (int r = 0; r < 16; ++r) tq[i][r] = 0.f;
            }
        }
        __syncthreads();
    }

    // epilogue: undo the operand scales, slab [split][phase][co][(u, t) * C + ci]
    const int eab = -(ea + eb);
    const long long Ktot = 4LL * C;
    float* const slab = ws + ((long long)split * 4 + ph) * Co * Ktot;
    const int col = ci0 + 32 * cib + (lane & 31);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = co0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            slab[(long long)row * Ktot + i * C + col] = __builtin_ldexpf(acc[i][r], eab);
        }
}

// ---------------------------------------------------------------------------------------
// Weight gradient of the stride-2 convolutions (down-convs 3x3, PatchGAN 4x4; zero pad 1) on a rolling
// window of the full-resolution source (f16x3):
//   dW[co][ci][ty][tx] = sum_{i, j} dy[i][j][co] * x[2i + ty - 1][2j + tx - 1][ci]
// A workgroup owns 64 co x 32 ci x all KK taps and walks a 64-pixel strip of the low-resolution grid row
// by row.  Per row it stages the dy row segment (64 px x 64 co, conv_win.hip's swizzled pixel-major
// layout) and the two new source rows 2i + 1, 2i + 2 of the strip, each split by column parity into an
// odd array O[p] = x[2 (x0 + p) - 1] and an even array E[p] = x[2 (x0 + p)] (65 px x 32 ci, 64-byte
// pixel rows), into a ring of six rows; tap (ty, tx) reads row 2i + ty - 1 at O[j + tx / 2] (tx even) or
// E[j + (tx - 1) / 2] (tx odd).  Waves: 2 co blocks x 4 tap groups (4x4: four taps each; 3x3: 3, 2, 2, 2),
// M = co (32), N = ci (32), K = 16 low-resolution pixels; fragments by ds_read_b64_tr_b16.  An optional
// source prologue a = act(y * scale + shift) (the PatchGAN's IN + LeakyReLU) is applied at staging, zero
// in the padding.  Partial slabs [split][co][tap * C + ci] for conv.hip's wgrad_reduce_kernel.
constexpr int S2W_NT = 512, S2W_SW = 64, S2W_P = 65;
constexpr int S2W_XCLS = 2 * S2W_P * 32;     // halves per (row, class): 2 planes x 65 px x 32 ci
constexpr int S2W_XROW = 2 * S2W_XCLS;       // halves per ring slot (2 classes)
constexpr int S2W_DROW = 2 * S2W_SW * 64;    // halves per dy buffer (2 planes x 64 px x 64 co)
constexpr int S2W_XU = (2 * S2W_P * 4 + S2W_NT - 1) / S2W_NT;  // source (class, pixel, 8-ci unit)s per thread per row

struct S2WArgs {
    int N, H, W, C, Co;  // dy NHWC [N][H][W][Co] (low resolution); source [N][2H][2W][C]
    int KK;              // 3 or 4
    int strips, rchunks, rows_per;
    int gco, gci;        // 64-channel co tiles, 32-channel ci tiles
    int rng_a_n, rng_b_n;
    int pro_act;
};

template <int NP, int KK, int PRO>
__global__ __launch_bounds__(S2W_NT, 1) void s2_wgrad_kernel(S2WArgs a, const float* __restrict__ dy,
                                                             const float* __restrict__ src,
                                                             const float* __restrict__ rnga,
                                                             const float* __restrict__ rngb,
                                                             const float* __restrict__ psc,
                                                             const float* __restrict__ psh, float* __restrict__ ws) {
    __shared__ __attribute__((aligned(16))) _Float16 smem[6 * S2W_XROW + 2 * S2W_DROW];
    _Float16* const Xr = smem;                 // [6 rows][class][2 planes][65 px][32 ci]
    _Float16* const Dy = smem + 6 * S2W_XROW;  // [2][2 planes][64 px][64 co]

    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int ntile = a.gco * a.gci;
    const int tile = L % ntile, split = L / ntile;
    const int co0 = (tile % a.gco) * 64, ci0 = (tile / a.gco) * 32;
    const int rc = split % a.rchunks, rest = split / a.rchunks;
    const int strip = rest % a.strips, n = rest / a.strips;
    const int x0 = strip * S2W_SW;
    const int H = a.H, W = a.W, C = a.C, Co = a.Co;
    const int y_beg = rc * a.rows_per;
    const int y_end = y_beg + a.rows_per < H ? y_beg + a.rows_per : H;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int cob = wid & 1, grp = wid >> 1;
    constexpr int NT = KK == 4 ? 4 : 3;  // taps per wave (3x3: 3, 2, 2, 2)
    const int t0 = KK == 4 ? grp * 4 : (grp == 0 ? 0 : 1 + 2 * grp);
    const int nt = KK == 4 ? 4 : (grp == 0 ? 3 : 2);

    const int ea = f16x3_exp(rnga, a.rng_a_n), eb = f16x3_exp(rngb, a.rng_b_n);
    const float asc = __builtin_ldexpf(1.f, ea), bsc = __builtin_ldexpf(1.f, eb);
    // PRO: the scale / shift of this thread's 8 source channels (every unit of a thread has the same
    // 8-channel group: unit index % 4 == tid % 4), kept in registers
    float psv[PRO ? 8 : 1], pbv[PRO ? 8 : 1];
    if constexpr (PRO) {
        const int c0 = ci0 + 8 * (tid & 3);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            psv[k] = psc[(long long)n * C + c0 + k];
            pbv[k] = psh[(long long)n * C + c0 + k];
        }
    }

    const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dy), (short)0, 0x7fffff00, 0x00020000);
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, 0x7fffff00, 0x00020000);
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    constexpr int OOB = 0x7fffffbf;

    // dy row segment: 64 px x 8 units, one per thread
    int doff, dls;
    {
        const int pix = tid >> 3, cu = tid & 7;
        doff = ((x0 + pix) * Co + co0 + 8 * cu) * 4;
        dls = pix * 64 + 8 * (cu ^ sw_swz(pix));
    }
    // source row segment: 2 classes x 65 px x 4 units; unit -> (class, p, cu); byte offset within the row
    // of the full-resolution column (-1: outside the image), LDS offset within the slot (-1: none)
    const int W2 = 2 * W;
    int xoff[S2W_XU], xls[S2W_XU];
#pragma unroll
    for (int q = 0; q < S2W_XU; ++q) {
        const int u = tid + q * S2W_NT;
        const int cu = u & 3, p = (u >> 2) % S2W_P, cls = (u >> 2) / S2W_P;  // cls 0: odd, 1: even
        xoff[q] = -1;
        xls[q] = -1;
        if (cls < 2) {
            const int col = cls == 0 ? 2 * (x0 + p) - 1 : 2 * (x0 + p);
            if (col >= 0 && col < W2) xoff[q] = (col * C + ci0 + 8 * cu) * 4;
            xls[q] = cls * S2W_XCLS + p * 32 + 8 * cu;
        }
    }
    float4 dr[2], xr[2][S2W_XU][2];
    auto ld_dy = [&](int y) {
        const int rb = ((n * H + y) * W) * Co * 4;
        u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(drs, rb + doff, 0, 0);
        u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(drs, rb + doff + 16, 0, 0);
        __builtin_memcpy(&dr[0], &v0, 16);
        __builtin_memcpy(&dr[1], &v1, 16);
    };
    auto ld_x = [&](int slot, int r) {  // full-resolution source row r (zero outside the image)
        const bool ok = r >= 0 && r < 2 * H;
        const int rb = ((n * 2 * H + (ok ? r : 0)) * W2) * C * 4;
#pragma unroll
        for (int q = 0; q < S2W_XU; ++q) {
            const int off = (ok && xoff[q] >= 0) ? rb + xoff[q] : OOB;
            u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0);
            u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(xrs, off + 16, 0, 0);
            __builtin_memcpy(&xr[slot][q][0], &v0, 16);
            __builtin_memcpy(&xr[slot][q][1], &v1, 16);
        }
    };
    auto st_dy = [&](int buf) {
        f16x8 hi, lo;
        split8h(dr[0], dr[1], asc, hi, lo);
        *reinterpret_cast<f16x8*>(Dy + buf * S2W_DROW + dls) = hi;
        if constexpr (NP == 3) *reinterpret_cast<f16x8*>(Dy + buf * S2W_DROW + S2W_SW * 64 + dls) = lo;
    };
    auto st_x = [&](int slot, int rs, int r) {  // register set rs -> ring slot of row r
        const bool ok = r >= 0 && r < 2 * H;
#pragma unroll
        for (int q = 0; q < S2W_XU; ++q) {
            if (xls[q] >= 0) {
                float4 v0 = xr[rs][q][0], v1 = xr[rs][q][1];
                if constexpr (PRO) {  // the prologue applies inside the image only (0 in the padding); the
                    // selection sits here, not after the load, so the row prefetch is not waited on early
                    const bool in = ok && xoff[q] >= 0;
                    auto f = [&](float v, int k) { return in ? act_apply(fmaf(v, psv[k], pbv[k]), a.pro_act) : 0.f; };
                    v0 = make_float4(f(v0.x, 0), f(v0.y, 1), f(v0.z, 2), f(v0.w, 3));
                    v1 = make_float4(f(v1.x, 4), f(v1.y, 5), f(v1.z, 6), f(v1.w, 7));
                }
                f16x8 hi, lo;
                split8h(v0, v1, bsc, hi, lo);
                const int cls = xls[q] >= S2W_XCLS ? 1 : 0;
                const int base = slot * S2W_XROW + cls * S2W_XCLS;
                const int off = xls[q] - cls * S2W_XCLS;
                *reinterpret_cast<f16x8*>(Xr + base + off) = hi;
                if constexpr (NP == 3) *reinterpret_cast<f16x8*>(Xr + base + S2W_P * 32 + off) = lo;
            }
        }
    };

    // transposed-read lane offsets (halves), as conv_win.hip's weight gradient
    const int g16 = lane >> 4;
    const int rpix = 8 * (g16 >> 1) + ((lane & 15) >> 2);
    const int rcol = 16 * (g16 & 1) + 4 * (lane & 3);
    int aoff;
    {
        const int c = 32 * cob + rcol;
        aoff = rpix * 64 + 8 * ((c >> 3) ^ sw_swz(rpix)) + (c & 7);
    }
    // per tap of the wave: ring row offset (ty - 1 relative to 2i) and class array offset
    int tdy[NT], tb[NT];
#pragma unroll
    for (int k = 0; k < NT; ++k) {
        const int tap = t0 + (k < nt ? k : 0);
        const int ty = tap / KK, tx = tap - (tap / KK) * KK;
        tdy[k] = ty - 1;
        const int cls = (tx & 1) ? 1 : 0;  // tx odd: even class (column 2j + tx - 1 even)
        const int po = (tx & 1) ? (tx - 1) / 2 : tx / 2;
        tb[k] = cls * S2W_XCLS + (rpix + po) * 32 + rcol;
    }

    floatx16 acc[NT], tq[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) { acc[i][r] = 0.f; tq[i][r] = 0.f; }

    auto slot_of = [](int r) { return ((r % 6) + 6) % 6; };
    // prologue: rows 2 y_beg - 1 .. 2 y_beg + KK - 2 into their slots, dy row y_beg into buffer 0
#pragma unroll 1
    for (int r = 2 * y_beg - 1; r <= 2 * y_beg + KK - 2; ++r) {
        ld_x(0, r);
        st_x(slot_of(r), 0, r);
    }
    ld_dy(y_beg);
    st_dy(y_beg & 1);
    __syncthreads();

#pragma unroll 1
    for (int y = y_beg; y < y_end; ++y) {
        // next step's rows in flight: dy row y + 1 and source rows 2y + KK - 1, 2y + KK
        const int rn = 2 * y + KK - 1;
        ld_dy(y + 1 < y_end ? y + 1 : y);
        ld_x(0, rn);
        ld_x(1, rn + 1);
        const _Float16* const Db = Dy + (y & 1) * S2W_DROW;
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // 16-pixel sub-tiles of the strip
            f16x8 ah, al;
            ah = sw_frag<64>(Db + aoff + k * 16 * 64);
            if constexpr (NP == 3) al = sw_frag<64>(Db + S2W_SW * 64 + aoff + k * 16 * 64);
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                if (t < nt) {
                    const _Float16* xs = Xr + slot_of(2 * y + tdy[t]) * S2W_XROW + tb[t] + k * 16 * 32;
                    f16x8 bh, bl;
                    bh = sw_frag<32>(xs);
                    if constexpr (NP == 3) {
                        bl = sw_frag<32>(xs + S2W_P * 32);
                        tq[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, tq[t], 0, 0, 0);
                        tq[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, tq[t], 0, 0, 0);
                    }
                    tq[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, tq[t], 0, 0, 0);
                }
            }
        }
        // stage the loaded rows into the slots this row does not read (rows 2y - 3, 2y - 2 modulo 6)
        st_dy((y + 1) & 1);
        st_x(slot_of(rn), 0, rn);
        st_x(slot_of(rn + 1), 1, rn + 1);
        if (((y - y_beg) & 1) == 1 || y + 1 == y_end) {
#pragma unroll
            for (int i = 0; i < NT; ++i) {
                acc[i] += tq[i];
#pragma unroll
                for (int r = 0; r < 16; ++r) tq[i][r] = 0.f;
            }
        }
        __syncthreads();
    }

    // epilogue: undo the operand scales, slab [split][co][tap * C + ci]
    const int eab = -(ea + eb);
    const long long Ktot = (long long)KK * KK * C;
    float* const slab = ws + (long long)split * Co * Ktot;
    const int col = ci0 + (lane & 31);
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        if (i < nt) {
            const int tap = t0 + i;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = co0 + 32 * cob + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                slab[(long long)row * Ktot + tap * C + col] = __builtin_ldexpf(acc[i][r], eab);
            }
        }
    }
}

struct SWPlan {
    int strips, rchunks, rows_per, nsplit;
};
int rolling_rchunks(long long base, int rows);
SWPlan sw_plan(const dcs_conv_desc& d) {
    SWPlan p;
    p.strips = d.Ws / SW_SW;
    const long long base = (long long)d.N * p.strips * (d.Co / 32) * (d.Cs / 64);
    const int rch = rolling_rchunks(base, d.Hs);
    p.rows_per = (int)cdiv(d.Hs, rch);
    p.rchunks = (int)cdiv(d.Hs, p.rows_per);
    p.nsplit = d.N * p.strips * p.rchunks;
    return p;
}

// the epilogues index an image's output with 24-bit pixel products and 32-bit element offsets
// (__umul24(opix, Co)): every output pixel index and element offset of one image must fit
bool out_geom(const dcs_conv_desc& d) {
    return (long long)d.Ho * d.Wo < (1LL << 24) && (long long)d.Ho * d.Wo * d.Co < 0x7fffff00LL;
}

bool tile_geom(int N, int Hs, int Ws, SubArgs* a) {
    const int TW = Ws < 128 ? Ws : 128;
    if (N <= 0 || Hs <= 0 || TW < 16 || 256 % TW || Ws % TW || Hs % (256 / TW)) return false;  // (TW even)
    if (a) {
        a->N = N; a->Hs = Hs; a->Ws = Ws;
        a->TW = TW; a->R = 256 / TW; a->tiles_x = Ws / TW; a->tiles = (Hs / a->R) * a->tiles_x;
    }
    return true;
}

bool subpix_geom(const dcs_conv_desc& d, SubArgs* a) {
    const bool ok = d.parity == 2 && d.up == 1 && d.stride == 1 && d.KH == 3 && d.KW == 3 &&
                    d.pad_mode == DCS_PAD_ZERO && d.pt == 1 && d.pl == 1 && d.Ho == 2 * d.Hs && d.Wo == 2 * d.Ws &&
                    d.N > 0 && d.Hs > 0 && d.Ws > 0 && d.Cs % 16 == 0 && d.Cs > 0 && d.Co % 64 == 0 && d.Co > 0 &&
                    d.s_c == 1 && d.s_w == d.Cs && d.s_h == (long long)d.Ws * d.Cs &&
                    d.s_n == (long long)d.Hs * d.Ws * d.Cs && d.csplit == d.Cs && d.pro_act == DCS_ACT_NONE &&
                    d.epi_act == DCS_ACT_NONE && (d.mma == DCS_MMA_F16X3 || d.mma == DCS_MMA_F16) && d.rng_a &&
                    d.rng_a_n > 0 && d.rng_a_n <= 1024 && (long long)d.N * d.Hs * d.Ws * d.Cs * 4 < 0x7fffff00LL - 64 &&
                    16LL * d.Co * d.Cs < (1LL << 30);
    if (!ok || !out_geom(d) || !tile_geom(d.N, d.Hs, d.Ws, a)) return false;
    if (a) { a->C = d.Cs; a->Co = d.Co; a->gy = d.Co / 32; a->cblk = d.Co / 64; a->rng_n = d.rng_a_n; }
    return true;
}

// the data gradient's descriptor (modules/hip/ops.py dgrad, the rows pass's form): source = dy [N][Hs][Ws][Cs]
// (the forward's output), a 4x4 stride-2 zero-pad-1 conv onto dx [N][Ho][Wo][Co] with Hs = 2 Ho, Ws = 2 Wo
bool subpix_dgrad_geom(const dcs_conv_desc& d, SubArgs* a) {
    const bool ok = d.parity == 0 && d.up == 1 && d.stride == 2 && d.KH == 4 && d.KW == 4 &&
                    d.pad_mode == DCS_PAD_ZERO && d.pt == 1 && d.pl == 1 && d.Hs == 2 * d.Ho && d.Ws == 2 * d.Wo &&
                    d.N > 0 && d.Ho > 0 && d.Wo > 0 && d.Cs % 16 == 0 && d.Cs > 0 && d.Co % 128 == 0 && d.Co > 0 &&
                    d.s_c == 1 && d.s_w == d.Cs && d.s_h == (long long)d.Ws * d.Cs &&
                    d.s_n == (long long)d.Hs * d.Ws * d.Cs && d.csplit == d.Cs && d.pro_act == DCS_ACT_NONE &&
                    d.epi_act == DCS_ACT_NONE && (d.mma == DCS_MMA_F16X3 || d.mma == DCS_MMA_F16) && d.rng_a &&
                    d.rng_a_n > 0 && d.rng_a_n <= 1024 && (long long)d.N * d.Hs * d.Ws * d.Cs * 4 < 0x7fffff00LL - 64 &&
                    16LL * d.Co * d.Cs < (1LL << 30);
    if (!ok || !out_geom(d) || !tile_geom(d.N, d.Ho, d.Wo, a)) return false;
    if (a) { a->C = d.Cs; a->Co = d.Co; a->gy = d.Co / 128; a->cblk = d.Co / 64; a->rng_n = d.rng_a_n; }
    return true;
}

// the down-convolutions (stride-2 3x3 zero-pad-1, the rows pass's descriptors): forward (parity 0, source
// [N][Hs][Ws][Cs] with Hs = 2 Ho) on the class kernel (MODE 1), data gradient (parity 1, dy [N][Hs][Ws][Cs]
// onto dx [N][2 Hs][2 Ws][Co]) on the phase kernel (MODE 0)
bool s2_geom(const dcs_conv_desc& d, SubArgs* a) {
    const bool k3 = d.KH == 3 && d.KW == 3, k4 = d.KH == 4 && d.KW == 4;
    const bool pro_ok = d.pro_act == DCS_ACT_NONE ||
                        (d.parity == 0 && d.Cs <= SP_PROC &&
                         (d.pro_act == DCS_ACT_AFFINE || d.pro_act == DCS_ACT_RELU || d.pro_act == DCS_ACT_LRELU));
    const bool common = d.up == 1 && d.stride == 2 && (k3 || k4) && d.pad_mode == DCS_PAD_ZERO &&
                        d.pt == 1 && d.pl == 1 && d.N > 0 && d.Hs > 0 && d.Ws > 0 && d.Cs % 16 == 0 && d.Cs > 0 &&
                        d.s_c == 1 && d.s_w == d.Cs && d.s_h == (long long)d.Ws * d.Cs &&
                        d.s_n == (long long)d.Hs * d.Ws * d.Cs && d.csplit == d.Cs && pro_ok &&
                        d.epi_act == DCS_ACT_NONE && (d.mma == DCS_MMA_F16X3 || d.mma == DCS_MMA_F16) && d.rng_a &&
                        d.rng_a_n > 0 && d.rng_a_n <= 1024 && (long long)d.N * d.Hs * d.Ws * d.Cs * 4 < 0x7fffff00LL - 64 &&
                        d.Co > 0 && 16LL * d.Co * d.Cs < (1LL << 30);
    if (!common || !out_geom(d)) return false;
    if (d.parity == 0) {  // forward
        if (d.Hs != 2 * d.Ho || d.Ws != 2 * d.Wo || d.Co % 128 || !tile_geom(d.N, d.Ho, d.Wo, a)) return false;
        if (a) { a->C = d.Cs; a->Co = d.Co; a->gy = d.Co / 128; a->cblk = d.Co / 64; a->rng_n = d.rng_a_n; a->pro_act = d.pro_act; }
        return true;
    }
    if (d.parity == 1) {  // data gradient
        if (d.Ho != 2 * d.Hs || d.Wo != 2 * d.Ws || d.Co % 64 || !tile_geom(d.N, d.Hs, d.Ws, a)) return false;
        if (a) { a->C = d.Cs; a->Co = d.Co; a->gy = d.Co / 32; a->cblk = d.Co / 64; a->rng_n = d.rng_a_n; a->pro_act = 0; }
        return true;
    }
    return false;
}

}  // namespace
}  // namespace dcs

using namespace dcs;

extern "C" int dcs_subpix_win_ok(const dcs_conv_desc* dp) { return dp && subpix_geom(*dp, nullptr) ? 1 : 0; }

extern "C" size_t dcs_subpix_win_parts_size(const dcs_conv_desc* dp) {
    SubArgs a;
    if (!dp || !subpix_geom(*dp, &a)) return 0;
    return (size_t)a.N * 4 * a.tiles * a.Co * sizeof(Part);
}

extern "C" int dcs_subpix_win(const dcs_conv_desc* dp, const float* src, const void* w_hi, const void* w_lo,
                              const int* wexp, float* out, void* parts, size_t parts_bytes, int* nchunk, void* stream) {
    if (!dp || !src || !w_hi || !w_lo || !wexp || !out) return fail(DCS_E_INVALID, "subpix_win: null pointer");
    SubArgs a;
    if (!subpix_geom(*dp, &a))
        return fail(DCS_E_INVALID, "subpix_win: needs a sub-pixel rows descriptor (parity 2: nearest-x2 + 3x3 zero-pad "
                                   "conv) over contiguous NHWC, Cs % 16 == 0, Co % 64 == 0, min(Ws, 128) dividing 256 "
                                   "and Ws, Hs % (256 / min(Ws, 128)) == 0, f16x3 / f16 with the source range record");
    if (parts) {
        if (!nchunk || parts_bytes < dcs_subpix_win_parts_size(dp))
            return fail(DCS_E_WORKSPACE, "subpix_win: parts buffer too small");
        *nchunk = 4 * a.tiles;
    }
    const unsigned blocks = (unsigned)((long long)a.N * a.tiles * a.gy);
    hipStream_t s = as_stream(stream);
    const _Float16* h = reinterpret_cast<const _Float16*>(w_hi);
    const _Float16* l = reinterpret_cast<const _Float16*>(w_lo);
    if (dp->mma == DCS_MMA_F16)
        hipLaunchKernelGGL((subpix_win_kernel<1, 0, 0>), dim3(blocks), dim3(SP_NT), 0, s, a, src, h, l, dp->rng_a, wexp,
                           out, reinterpret_cast<Part*>(parts), nullptr, nullptr, PhIbw{});
    else
        hipLaunchKernelGGL((subpix_win_kernel<3, 0, 0>), dim3(blocks), dim3(SP_NT), 0, s, a, src, h, l, dp->rng_a, wexp,
                           out, reinterpret_cast<Part*>(parts), nullptr, nullptr, PhIbw{});
    return check_launch("subpix_win");
}

extern "C" int dcs_subpix_win_dgrad_ok(const dcs_conv_desc* dp) { return dp && subpix_dgrad_geom(*dp, nullptr) ? 1 : 0; }

extern "C" int dcs_subpix_win_dgrad(const dcs_conv_desc* dp, const float* dy, const void* w_hi, const void* w_lo,
                                    const int* wexp, float* dx, void* stream) {
    if (!dp || !dy || !w_hi || !w_lo || !wexp || !dx) return fail(DCS_E_INVALID, "subpix_win_dgrad: null pointer");
    SubArgs a;
    if (!subpix_dgrad_geom(*dp, &a))
        return fail(DCS_E_INVALID, "subpix_win_dgrad: needs the sub-pixel data-gradient descriptor (4x4 stride-2 "
                                   "zero-pad-1 over contiguous NHWC dy, Hs = 2 Ho), Cs % 16 == 0, Co % 128 == 0, "
                                   "min(Wo, 128) dividing 256 and Wo, Ho % (256 / min(Wo, 128)) == 0, f16x3 / f16 with "
                                   "the dy range record");
    const unsigned blocks = (unsigned)((long long)a.N * a.tiles * a.gy);
    hipStream_t s = as_stream(stream);
    const _Float16* h = reinterpret_cast<const _Float16*>(w_hi);
    const _Float16* l = reinterpret_cast<const _Float16*>(w_lo);
    if (dp->mma == DCS_MMA_F16)
        hipLaunchKernelGGL((subpix_win_kernel<1, 1, 0>), dim3(blocks), dim3(SP_NT), 0, s, a, dy, h, l, dp->rng_a, wexp, dx,
                           nullptr, nullptr, nullptr, PhIbw{});
    else
        hipLaunchKernelGGL((subpix_win_kernel<3, 1, 0>), dim3(blocks), dim3(SP_NT), 0, s, a, dy, h, l, dp->rng_a, wexp, dx,
                           nullptr, nullptr, nullptr, PhIbw{});
    return check_launch("subpix_win_dgrad");
}

extern "C" int dcs_pack_subpix_h3(const float* w, int Cout, int Cin, int kind, void* out_hi, void* out_lo,
                                  float* scratch, int* wexp, void* stream) {
    if (!w || !out_hi || !out_lo || !scratch || !wexp || !subpix_pack_ok(Cout, Cin, kind))
        return fail(DCS_E_INVALID, "pack_subpix_h3: bad arguments (kind 0: Cout % 64, Cin % 16; 1: Cout % 16, "
                                   "Cin % 128; 2: Cin % 64, Cout % 16; 3: Cout % 128, Cin % 16)");
    hipStream_t s = as_stream(stream);
    const long long total = 16LL * Cout * Cin;
    const long long rb = cdiv(total, 2048) < DCS_RANGE_PARTS ? cdiv(total, 2048) : DCS_RANGE_PARTS;
    hipLaunchKernelGGL(subpix_range_kernel, dim3((unsigned)rb), dim3(256), 0, s, w, Cout, Cin, kind, scratch);
    int e = check_launch("pack_subpix_h3 range");
    if (e) return e;
    const long long pb = cdiv(total, 2048) < 256 ? cdiv(total, 2048) : 256;
    hipLaunchKernelGGL(subpix_pack_kernel, dim3((unsigned)pb), dim3(256), 0, s, w, Cout, Cin, kind, scratch,
                       reinterpret_cast<_Float16*>(out_hi), reinterpret_cast<_Float16*>(out_lo), wexp);
    return check_launch("pack_subpix_h3");
}

namespace dcs {
// conv.hip's dcs_conv_wgrad: d describes the forward up-convolution (parity 2, the rows pass's form)
bool subpix_wgrad_check(const dcs_conv_desc& d) {
    return (d.mma == DCS_MMA_F16X3 || d.mma == DCS_MMA_F16) && d.parity == 2 && d.up == 1 && d.stride == 1 &&
           d.KH == 3 && d.KW == 3 && d.pad_mode == DCS_PAD_ZERO && d.pt == 1 && d.pl == 1 && d.Ho == 2 * d.Hs &&
           d.Wo == 2 * d.Ws && d.Cs % 64 == 0 && d.Co % 32 == 0 && d.Ws % SW_SW == 0 && d.Hs >= 1 && d.s_c == 1 &&
           d.s_w == d.Cs && d.s_h == (long long)d.Ws * d.Cs && d.s_n == (long long)d.Hs * d.Ws * d.Cs &&
           d.csplit == d.Cs && (d.cw == 0 || d.cw == d.Cs) && d.pro_act == DCS_ACT_NONE && d.rng_a && d.rng_b &&
           d.rng_a_n > 0 && d.rng_a_n <= 1024 && d.rng_b_n > 0 && d.rng_b_n <= 1024 &&
           (long long)d.N * d.Hs * d.Ws * d.Cs * 4 < 0x7fffff00LL - 64 &&
           (long long)d.N * d.Ho * d.Wo * d.Co * 4 < 0x7fffff00LL - 64;
}

size_t subpix_wgrad_workspace_size(const dcs_conv_desc& d) {
    const SWPlan p = sw_plan(d);
    return (size_t)p.nsplit * 4 * d.Co * 4 * d.Cs * sizeof(float);
}

// partial slabs into ws (subpix_wgrad_workspace_size bytes, wgrad_subpixel_fold_kernel's layout); returns the
// split count (< 0: error).  rng_a: dy's range record, rng_b: the source's.
int subpix_wgrad_launch(const dcs_conv_desc& d, const float* dy, const float* x, float* ws, hipStream_t s) {
    const SWPlan p = sw_plan(d);
    SWArgs a;
    a.N = d.N; a.H = d.Hs; a.W = d.Ws; a.C = d.Cs; a.Co = d.Co;
    a.strips = p.strips; a.rchunks = p.rchunks; a.rows_per = p.rows_per;
    a.gco = d.Co / 32; a.gci = d.Cs / 64;
    a.rng_a_n = d.rng_a_n; a.rng_b_n = d.rng_b_n;
    const unsigned blocks = (unsigned)((long long)p.nsplit * a.gco * a.gci);
    if (d.mma == DCS_MMA_F16)
        hipLaunchKernelGGL(subpix_wgrad_kernel<1>, dim3(blocks), dim3(SW_NT), 0, s, a, dy, x, d.rng_a, d.rng_b, ws);
    else
        hipLaunchKernelGGL(subpix_wgrad_kernel<3>, dim3(blocks), dim3(SW_NT), 0, s, a, dy, x, d.rng_a, d.rng_b, ws);
    const int e = check_launch("subpix_wgrad");
    return e ? -e : p.nsplit;
}
}  // namespace dcs

extern "C" int dcs_stride2_win_ok(const dcs_conv_desc* dp) { return dp && s2_geom(*dp, nullptr) ? 1 : 0; }

extern "C" size_t dcs_stride2_win_parts_size(const dcs_conv_desc* dp) {
    SubArgs a;
    if (!dp || dp->parity != 0 || !s2_geom(*dp, &a)) return 0;
    return (size_t)a.N * a.tiles * a.Co * sizeof(Part);
}

extern "C" int dcs_stride2_win(const dcs_conv_desc* dp, const float* src, const float* pro_scale,
                               const float* pro_shift, const void* w_hi, const void* w_lo, const int* wexp, float* out,
                               void* parts, size_t parts_bytes, int* nchunk, void* stream) {
    if (!dp || !src || !w_hi || !w_lo || !wexp || !out) return fail(DCS_E_INVALID, "stride2_win: null pointer");
    SubArgs a;
    if (!s2_geom(*dp, &a))
        return fail(DCS_E_INVALID, "stride2_win: needs a stride-2 3x3 or 4x4 zero-pad-1 rows descriptor over contiguous "
                                   "NHWC (parity 0: forward, Co % 128 == 0, an optional affine / ReLU / LeakyReLU "
                                   "prologue for Cs <= 512; parity 1: data gradient, Co % 64 == 0), Cs % 16 == 0, the "
                                   "low-resolution grid tileable (min(W, 128) dividing 256 and W), f16x3 / f16 with "
                                   "the source range record");
    const bool pro = dp->pro_act != DCS_ACT_NONE;
    if (pro && (!pro_scale || !pro_shift)) return fail(DCS_E_INVALID, "stride2_win: prologue needs scale and shift");
    if (parts) {
        if (dp->parity != 0 || !nchunk || parts_bytes < dcs_stride2_win_parts_size(dp))
            return fail(DCS_E_WORKSPACE, "stride2_win: statistics only for the forward, parts buffer too small");
        *nchunk = a.tiles;
    }
    const unsigned blocks = (unsigned)((long long)a.N * a.tiles * a.gy);
    hipStream_t s = as_stream(stream);
    const _Float16* h = reinterpret_cast<const _Float16*>(w_hi);
    const _Float16* l = reinterpret_cast<const _Float16*>(w_lo);
    Part* pp = reinterpret_cast<Part*>(parts);
    const bool f16 = dp->mma == DCS_MMA_F16;
    const bool k3 = dp->KH == 3;  // 3x3: the unreached (class, offset) pairs skipped; 4x4: every pair a tap
#define DCS_S2_FWD(NP_, S2_, PRO_)                                                                                   \
    hipLaunchKernelGGL((subpix_win_kernel<NP_, 1, S2_, -1, PRO_>), dim3(blocks), dim3(SP_NT), 0, s, a, src, h, l,      \
                       dp->rng_a, wexp, out, pp, pro_scale, pro_shift, PhIbw{})
#define DCS_S2_DG(NP_, S2_, PXC_)                                                                                    \
    hipLaunchKernelGGL((subpix_win_kernel<NP_, 0, S2_, PXC_>), dim3(blocks / 2), dim3(SP_NT), 0, s, a, src, h, l,     \
                       dp->rng_a, wexp, out, nullptr, nullptr, nullptr, PhIbw{})
    if (dp->parity == 0) {
        if (f16) {
            if (k3) { if (pro) DCS_S2_FWD(1, 1, 1); else DCS_S2_FWD(1, 1, 0); }
            else { if (pro) DCS_S2_FWD(1, 0, 1); else DCS_S2_FWD(1, 0, 0); }
        } else {
            if (k3) { if (pro) DCS_S2_FWD(3, 1, 1); else DCS_S2_FWD(3, 1, 0); }
            else { if (pro) DCS_S2_FWD(3, 0, 1); else DCS_S2_FWD(3, 0, 0); }
        }
    } else {  // one launch per column phase
        if (f16) {
            if (k3) { DCS_S2_DG(1, 1, 0); DCS_S2_DG(1, 1, 1); } else { DCS_S2_DG(1, 0, 0); DCS_S2_DG(1, 0, 1); }
        } else {
            if (k3) { DCS_S2_DG(3, 1, 0); DCS_S2_DG(3, 1, 1); } else { DCS_S2_DG(3, 0, 0); DCS_S2_DG(3, 0, 1); }
        }
    }
#undef DCS_S2_FWD
#undef DCS_S2_DG
    return check_launch("stride2_win");
}

namespace dcs {
namespace {
// row chunks per strip: the count that minimises (dispatch rounds of one workgroup per CU) x (rows per
// workgroup), >= 8 rows per chunk, fewer chunks (less slab traffic) on ties
int rolling_rchunks(long long base, int rows) {
    const int maxch = rows / 8 > 0 ? rows / 8 : 1;
    int best = 1;
    long long best_cost = -1;
    for (int rch = 1; rch <= maxch && rch <= 64; ++rch) {
        const long long cost = cdiv(base * rch, 256) * cdiv(rows, rch);
        if (best_cost < 0 || cost < best_cost) { best_cost = cost; best = rch; }
    }
    return best;
}

SWPlan s2w_plan(const dcs_conv_desc& d) {
    SWPlan p;
    p.strips = d.Wo / S2W_SW;
    const long long base = (long long)d.N * p.strips * (d.Co / 64) * (d.Cs / 32);
    const int rch = rolling_rchunks(base, d.Ho);
    p.rows_per = (int)cdiv(d.Ho, rch);
    p.rchunks = (int)cdiv(d.Ho, p.rows_per);
    p.nsplit = d.N * p.strips * p.rchunks;
    return p;
}
}  // namespace

// conv.hip's dcs_conv_wgrad: d describes the forward stride-2 conv (parity 0; source [N][Hs][Ws][Cs], Hs = 2 Ho)
bool s2_wgrad_check(const dcs_conv_desc& d) {
    // (the PatchGAN's 4x4 layers measured slower here than on the x6 kernel in the bench step's 8-image
    // calls: 217 vs 174 us, profiles/r04af; the kernel takes them, the dispatch keeps them on x6)
    return (d.mma == DCS_MMA_F16X3 || d.mma == DCS_MMA_F16) && d.parity == 0 && d.up == 1 && d.stride == 2 &&
           d.KH == 3 && d.KW == 3 && d.pad_mode == DCS_PAD_ZERO && d.pt == 1 &&
           d.pl == 1 && d.Hs == 2 * d.Ho && d.Ws == 2 * d.Wo && d.Cs % 32 == 0 && d.Co % 64 == 0 &&
           d.Wo % S2W_SW == 0 && d.Ho >= 1 && d.s_c == 1 && d.s_w == d.Cs && d.s_h == (long long)d.Ws * d.Cs &&
           d.s_n == (long long)d.Hs * d.Ws * d.Cs && d.csplit == d.Cs && (d.cw == 0 || d.cw == d.Cs) &&
           (d.pro_act == DCS_ACT_NONE || d.pro_act == DCS_ACT_AFFINE || d.pro_act == DCS_ACT_RELU ||
            d.pro_act == DCS_ACT_LRELU) &&
           d.rng_a && d.rng_b && d.rng_a_n > 0 && d.rng_a_n <= 1024 && d.rng_b_n > 0 && d.rng_b_n <= 1024 &&
           (long long)d.N * d.Hs * d.Ws * d.Cs * 4 < 0x7fffff00LL - 64 &&
           (long long)d.N * d.Ho * d.Wo * d.Co * 4 < 0x7fffff00LL - 64;
}

size_t s2_wgrad_workspace_size(const dcs_conv_desc& d) {
    const SWPlan p = s2w_plan(d);
    return (size_t)p.nsplit * d.Co * d.KH * d.KW * d.Cs * sizeof(float);
}

// partial slabs [split][co][tap * C + ci] into ws; returns the split count (< 0: error).  rng_a: dy's range
// record, rng_b: the (prologued) source's.
int s2_wgrad_launch(const dcs_conv_desc& d, const float* dy, const float* x, const float* psc, const float* psh,
                    float* ws, hipStream_t s) {
    const SWPlan p = s2w_plan(d);
    S2WArgs a;
    a.N = d.N; a.H = d.Ho; a.W = d.Wo; a.C = d.Cs; a.Co = d.Co; a.KK = d.KH;
    a.strips = p.strips; a.rchunks = p.rchunks; a.rows_per = p.rows_per;
    a.gco = d.Co / 64; a.gci = d.Cs / 32;
    a.rng_a_n = d.rng_a_n; a.rng_b_n = d.rng_b_n; a.pro_act = d.pro_act;
    const bool pro = d.pro_act != DCS_ACT_NONE;
    if (pro && (!psc || !psh)) return -fail(DCS_E_INVALID, "conv_wgrad: prologue needs scale and shift");
    const unsigned blocks = (unsigned)((long long)p.nsplit * a.gco * a.gci);
    const bool f16 = d.mma == DCS_MMA_F16;
#define DCS_S2W(NP_, KK_, PRO_) \
    hipLaunchKernelGGL((s2_wgrad_kernel<NP_, KK_, PRO_>), dim3(blocks), dim3(S2W_NT), 0, s, a, dy, x, d.rng_a, d.rng_b, psc, psh, ws)
    if (f16) { if (pro) DCS_S2W(1, 3, 1); else DCS_S2W(1, 3, 0); }  // (3x3 only: s2_wgrad_check)
    else { if (pro) DCS_S2W(3, 3, 1); else DCS_S2W(3, 3, 0); }
#undef DCS_S2W
    const int e = check_launch("s2_wgrad");
    return e ? -e : p.nsplit;
}
}  // namespace dcs

namespace {
// chunks per image of the fused IN-backward partial sums: the subpixel data gradient (MODE 1) writes one
// per tile, the stride-2 data gradient (MODE 0) one per (tile, column phase, row phase)
bool phase_ibw_geom(const dcs_conv_desc& d, int subpixel, SubArgs* a, int* nchunk) {
    if (subpixel ? !subpix_dgrad_geom(d, a) : (d.parity != 1 || !s2_geom(d, a))) return false;
    *nchunk = subpixel ? a->tiles : 4 * a->tiles;
    return true;
}
}  // namespace

extern "C" size_t dcs_phase_win_dgrad_inbwd_parts_size(const dcs_conv_desc* dp, int subpixel) {
    SubArgs a;
    int nch = 0;
    if (!dp || !phase_ibw_geom(*dp, subpixel, &a, &nch)) return 0;
    return (size_t)a.N * nch * a.Co * sizeof(Sum2);
}

extern "C" int dcs_phase_win_dgrad_inbwd(const dcs_conv_desc* dp, int subpixel, const float* dy, const void* w_hi,
                                         const void* w_lo, const int* wexp, float* dx, const float* y,
                                         const float* scale, const float* shift, int act, void* parts,
                                         size_t parts_bytes, int* nchunk, void* stream) {
    if (!dp || !dy || !w_hi || !w_lo || !wexp || !dx || !y || !scale || !shift || !parts || !nchunk)
        return fail(DCS_E_INVALID, "phase_win_dgrad_inbwd: null pointer");
    SubArgs a;
    int nch = 0;
    if (!phase_ibw_geom(*dp, subpixel, &a, &nch))
        return fail(DCS_E_INVALID, "phase_win_dgrad_inbwd: a dcs_subpix_win_dgrad (subpixel = 1) or dcs_stride2_win "
                                   "data-gradient (subpixel = 0, parity 1) descriptor expected");
    if (act != DCS_ACT_AFFINE && act != DCS_ACT_RELU && act != DCS_ACT_LRELU)
        return fail(DCS_E_INVALID, "phase_win_dgrad_inbwd: act must be DCS_ACT_AFFINE / _RELU / _LRELU");
    if (parts_bytes < dcs_phase_win_dgrad_inbwd_parts_size(dp, subpixel))
        return fail(DCS_E_WORKSPACE, "phase_win_dgrad_inbwd: parts buffer too small");
    *nchunk = nch;
    const PhIbw ib{y, scale, shift, reinterpret_cast<Sum2*>(parts), act};
    const unsigned blocks = (unsigned)((long long)a.N * a.tiles * a.gy);
    hipStream_t s = as_stream(stream);
    const _Float16* h = reinterpret_cast<const _Float16*>(w_hi);
    const _Float16* l = reinterpret_cast<const _Float16*>(w_lo);
    const bool f16 = dp->mma == DCS_MMA_F16;
    if (subpixel) {
        if (f16) hipLaunchKernelGGL((subpix_win_kernel<1, 1, 0, -1, 0, 1>), dim3(blocks), dim3(SP_NT), 0, s, a, dy, h, l, dp->rng_a, wexp, dx, nullptr, nullptr, nullptr, ib);
        else hipLaunchKernelGGL((subpix_win_kernel<3, 1, 0, -1, 0, 1>), dim3(blocks), dim3(SP_NT), 0, s, a, dy, h, l, dp->rng_a, wexp, dx, nullptr, nullptr, nullptr, ib);
        return check_launch("subpix_win_dgrad_inbwd");
    }
    const bool k3 = dp->KH == 3;
#define DCS_S2_DGI(NP_, S2_, PXC_)                                                                                   \
    hipLaunchKernelGGL((subpix_win_kernel<NP_, 0, S2_, PXC_, 0, 1>), dim3(blocks / 2), dim3(SP_NT), 0, s, a, dy, h, l, \
                       dp->rng_a, wexp, dx, nullptr, nullptr, nullptr, ib)
    if (f16) {
        if (k3) { DCS_S2_DGI(1, 1, 0); DCS_S2_DGI(1, 1, 1); } else { DCS_S2_DGI(1, 0, 0); DCS_S2_DGI(1, 0, 1); }
    } else {
        if (k3) { DCS_S2_DGI(3, 1, 0); DCS_S2_DGI(3, 1, 1); } else { DCS_S2_DGI(3, 0, 0); DCS_S2_DGI(3, 0, 1); }
    }
#undef DCS_S2_DGI
    return check_launch("stride2_win_dgrad_inbwd");
}
