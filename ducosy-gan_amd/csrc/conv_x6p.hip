// Pre-split bf16x6 implicit-GEMM convolution rows pass for the 256-channel 3x3 residual convs
// (modules/model.py:72-80: ReflectionPad(1) + Conv 3x3 256->256, forward and the stride-1
// data gradient), with the operands staged by LDS-DMA.
//
// The bf16x6 product (conv.hip: each fp32 operand v = hi + mid + lo in bf16, six MFMAs per
// product, fp32 accumulation) needs every operand element in three bf16 planes.  conv.hip's
// rows kernel splits on the fly, so each activation element is split 9 (taps) x 2 (column
// tiles) times and each weight once per pixel tile, and the split, the conversion and the
// ds_write staging are 7 VALU instructions per MFMA.  Here the operands are split ONCE
// (dcs_split_x6: fp32 -> interleaved planes [.. C/8][hi, mid, lo][8]) and the k-tiles move from
// HBM/L2 straight into LDS with buffer_load ... lds (one 16-B piece per lane; out-of-range
// offsets read as zeros, which is the zero padding), three stages deep, one barrier per
// k-tile and no register staging.  The per-k-tile VALU left is the DMA address arithmetic.
//
// Tile: 128 output pixels x 128 output channels per 256-thread workgroup, 4 waves as 2 x 2,
// each wave 64 x 64 (2 x 2 blocks of v_mfma_f32_32x32x16_bf16); k-tiles of 16 (one 32-byte
// row per plane and operand row).  Two-level fp32 summation as in conv.hip (inner chains of
// 128 k).  LDS per stage: [A|B][plane][128 rows][16 bf16], the 16-byte halves of a row swapped
// on odd groups of 8 rows so the fragment reads are conflict-free; the DMA fetches the swapped
// half instead (its LDS destination is lane-linear).
#include "common.hpp"

#include <cstdlib>

namespace dcs {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx8 __attribute__((ext_vector_type(8)));

constexpr int XP_BM = 128, XP_BN = 128, XP_BK = 16, XP_NT = 256;
constexpr int XP_STAGES = 3;
constexpr int XP_PLANE_BYTES = 128 * 32;                    // 128 rows x 16 bf16
constexpr int XP_STAGE_BYTES = 2 * 3 * XP_PLANE_BYTES;      // A and B, three planes: 24 KiB
constexpr unsigned XP_OOB = 0x80000000u;                    // > num_records: reads as zeros
constexpr int XP_KT2 = 8;                                   // k-tiles per inner accumulation chain

__device__ __forceinline__ __amdgpu_buffer_rsrc_t xp_rsrc(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7ffff000, 0x00020000);
}

// fp32 -> three bf16 planes, 8 consecutive elements per group: out[g] = {hi[8], mid[8], lo[8]}
__global__ void split_x6_kernel(const float4* __restrict__ src, uint4* __restrict__ dst, long long ngroups) {
    const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= ngroups) return;
    const float4 a = src[2 * g], b = src[2 * g + 1];
    const floatx8 f = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const bf16x8 hi = __builtin_convertvector(f, bf16x8);
    const floatx8 r1 = f - __builtin_convertvector(hi, floatx8);
    const bf16x8 mid = __builtin_convertvector(r1, bf16x8);
    const floatx8 r2 = r1 - __builtin_convertvector(mid, floatx8);
    const bf16x8 lo = __builtin_convertvector(r2, bf16x8);
    uint4 h, m, l;
    __builtin_memcpy(&h, &hi, 16);
    __builtin_memcpy(&m, &mid, 16);
    __builtin_memcpy(&l, &lo, 16);
    dst[3 * g] = h;
    dst[3 * g + 1] = m;
    dst[3 * g + 2] = l;
}

__device__ __forceinline__ void xp_dma(__amdgpu_buffer_rsrc_t r, unsigned char* lds, unsigned voff) {
#ifndef DCS_XP_NODMA  // skeleton probe: timing experiments only (wrong results)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
#endif
}

__device__ __forceinline__ void xp_barrier() {
#ifndef DCS_XP_NOBAR  // skeleton probe
    __builtin_amdgcn_s_barrier();
#endif
    asm volatile("" ::: "memory");
}

template <bool REFLECT, int IL>
__global__ __launch_bounds__(XP_NT, 2) void conv_rows_x6p_kernel(const dcs_conv_desc d, const __bf16* __restrict__ srcp,
                                                               const __bf16* __restrict__ wpp,
                                                               float* __restrict__ out, int gx, int gy) {
    // one LDS array (a second __shared__ object can make hipcc drain the DMA queue early)
    __shared__ __attribute__((aligned(16))) unsigned char lds[XP_STAGES * XP_STAGE_BYTES];

    const int T = gridDim.x;
    const int xcd = blockIdx.x & 7, q8 = T >> 3, r8 = T & 7;
    const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
    const int ntile = L % gy, mtile = L / gy;
    const int M = d.N * d.Ho * d.Wo;
    const int m0 = mtile * XP_BM, n0 = ntile * XP_BN;
    if (m0 >= M || mtile >= gx) return;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int Cs = d.Cs, KW = d.KW;
    const int nkt = d.KH * KW * Cs / XP_BK;
    const int kt_per_tap = Cs / XP_BK;

    // ---- DMA lanes: wave wid stages rows 32*wid .. +31 of A and of B; lane = (row, 16-B slot)
    const int lrow = 32 * wid + (lane >> 1);
    const int slot = lane & 1;
    const int half = slot ^ ((lrow >> 3) & 1);  // which 8-k half of the row this slot holds
    // A: the output pixel of this lane's row
    const int m = m0 + lrow;
    const bool mvalid = m < M;
    const int per = d.Ho * d.Wo;
    const int an = mvalid ? m / per : 0;
    const int arem = m - an * per;
    const int aoy = arem / d.Wo, aox = arem - (arem / d.Wo) * d.Wo;
    const unsigned pix_bytes = (unsigned)Cs * 6u;
    auto tap_base = [&](int j) -> unsigned {
        const int ty = j / KW, tx = j - (j / KW) * KW;
        int vy = aoy + ty - d.pt, vx = aox + tx - d.pl;
        bool ok = mvalid;
        if (REFLECT) {
            vy = vy < 0 ? -vy : (vy >= d.Hs ? 2 * (d.Hs - 1) - vy : vy);
            vx = vx < 0 ? -vx : (vx >= d.Ws ? 2 * (d.Ws - 1) - vx : vx);
        } else {
            ok = ok && (unsigned)vy < (unsigned)d.Hs && (unsigned)vx < (unsigned)d.Ws;
        }
        return ok ? (unsigned)((an * d.Hs + vy) * d.Ws + vx) * pix_bytes + (unsigned)half * 48u : XP_OOB;
    };
    // B: packed weights [ncols][Kpad] split to [ncols][Kpad/8][3][8]
    const unsigned bbase = (unsigned)(n0 + lrow) * (unsigned)d.ldb * 6u + (unsigned)half * 48u;
    const __amdgpu_buffer_rsrc_t ra = xp_rsrc(srcp), rb = xp_rsrc(wpp);

    int dj = 0, dc = 0;            // (tap, k-tile within the tap) of the next k-tile to stage
    unsigned abase = tap_base(0);
    auto issue = [&](int kt, int stage) {
        unsigned char* s = lds + stage * XP_STAGE_BYTES + wid * 1024;
        unsigned ao = abase == XP_OOB ? XP_OOB : abase + (unsigned)dc * 96u;
        unsigned bo = bbase + (unsigned)kt * 96u;
#ifdef DCS_XP_L2PROBE  // skeleton probe: every A piece from a 64 KiB window (L2/L1 hits), B from 64 KiB
        ao &= 0xffffu;
        bo &= 0xffffu;
#endif
#pragma unroll
        for (int q = 0; q < 3; ++q) xp_dma(ra, s + q * XP_PLANE_BYTES, ao + 16u * q);
#pragma unroll
        for (int q = 0; q < 3; ++q) xp_dma(rb, s + (3 + q) * XP_PLANE_BYTES, bo + 16u * q);
        if (++dc == kt_per_tap) {
            dc = 0;
            ++dj;
            if (dj < d.KH * KW) abase = tap_base(dj);
        }
    };

    floatx16 acc[2][2], t[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) { acc[i][j][r] = 0.f; t[i][j][r] = 0.f; }

    // fragment addresses: lane (r = lane & 31, hh = lane >> 5) reads k 8hh..8hh+7 of its row
    const int l32 = lane & 31, hh = lane >> 5;
    int aoff[2], boff[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int row = wm * 64 + i * 32 + l32;
        aoff[i] = row * 32 + 16 * (hh ^ ((row >> 3) & 1));
        const int col = wn * 64 + i * 32 + l32;
        boff[i] = 3 * XP_PLANE_BYTES + col * 32 + 16 * (hh ^ ((col >> 3) & 1));
    }

    issue(0, 0);
    if (nkt > 1) issue(1, 1);
    int stage = 0;
    auto mfma6 = [&](const bf16x8 (&ah)[2], const bf16x8 (&am)[2], const bf16x8 (&al)[2], const bf16x8 (&bh)[2],
                     const bf16x8 (&bm)[2], const bf16x8 (&bl)[2], int i, int j) {  // smallest terms first
        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bm[j], t[i][j], 0, 0, 0);
        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], t[i][j], 0, 0, 0);
        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], t[i][j], 0, 0, 0);
        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bh[j], t[i][j], 0, 0, 0);
        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bm[j], t[i][j], 0, 0, 0);
        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], t[i][j], 0, 0, 0);
    };
    if constexpr (IL == 2) {
        // software-pipelined: the fragments of k-tile kt+1 are read from LDS while the MFMAs of
        // k-tile kt run (two register sets); the wait and barrier sit between the two MFMA halves.
        // Iteration kt: MFMAs (i = 0) of kt | own DMA kt+1 landed, barrier, DMA kt+2 into the stage
        // of kt-1 (last read before this barrier), fragments of kt+1 | MFMAs (i = 1) of kt.
        bf16x8 fa[2][3][2], fb[2][3][2];
        auto rd = [&](int set, int st) {
            const unsigned char* sb = lds + st * XP_STAGE_BYTES;
#pragma unroll
            for (int q = 0; q < 3; ++q)
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    fa[set][q][i] = *reinterpret_cast<const bf16x8*>(sb + q * XP_PLANE_BYTES + aoff[i]);
                    fb[set][q][i] = *reinterpret_cast<const bf16x8*>(sb + q * XP_PLANE_BYTES + boff[i]);
                }
        };
        auto m6 = [&](int set, int i, int j) {
            t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[set][1][i], fb[set][1][j], t[i][j], 0, 0, 0);
            t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[set][2][i], fb[set][0][j], t[i][j], 0, 0, 0);
            t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[set][0][i], fb[set][2][j], t[i][j], 0, 0, 0);
            t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[set][1][i], fb[set][0][j], t[i][j], 0, 0, 0);
            t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[set][0][i], fb[set][1][j], t[i][j], 0, 0, 0);
            t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[set][0][i], fb[set][0][j], t[i][j], 0, 0, 0);
        };
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6) : "memory");
        if (nkt == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        xp_barrier();
        rd(0, 0);
#ifdef DCS_XP_NOLDS
        rd(1, 1);
#endif
        for (int kt = 0; kt < nkt; kt += 2) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int k = kt + u;
                if (k < nkt) {
                    m6(u, 0, 0);
                    m6(u, 0, 1);
                    __builtin_amdgcn_sched_barrier(0);
                    if (k + 1 < nkt) {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        xp_barrier();
                        int s1 = stage + 1;
                        if (s1 >= XP_STAGES) s1 -= XP_STAGES;
                        if (k + 2 < nkt) {
                            int s2 = s1 + 1;
                            if (s2 >= XP_STAGES) s2 -= XP_STAGES;
                            issue(k + 2, s2);
                        }
#ifndef DCS_XP_NOLDS  // skeleton probe: fragments stay in registers
                        rd(u ^ 1, s1);
#endif
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    m6(u, 1, 0);
                    m6(u, 1, 1);
                    if ((k % XP_KT2) == XP_KT2 - 1 || k + 1 == nkt) {
#pragma unroll
                        for (int i = 0; i < 2; ++i)
#pragma unroll
                            for (int j = 0; j < 2; ++j) {
                                acc[i][j] += t[i][j];
#pragma unroll
                                for (int r = 0; r < 16; ++r) t[i][j][r] = 0.f;
                            }
                    }
                    if (++stage == XP_STAGES) stage = 0;
                }
            }
        }
    } else
    for (int kt = 0; kt < nkt; ++kt) {
        // this wave's pieces of k-tile kt have landed (those of kt + 1 may still fly); the
        // barrier makes every wave's pieces visible and frees the stage read at kt - 1
        if (kt + 1 < nkt) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (!IL && kt + 2 < nkt) {
            int s2 = stage + 2;
            if (s2 >= XP_STAGES) s2 -= XP_STAGES;
            issue(kt + 2, s2);
        }
        const unsigned char* sb = lds + stage * XP_STAGE_BYTES;
        bf16x8 ah[2], am[2], al[2], bh[2], bm[2], bl[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            ah[i] = *reinterpret_cast<const bf16x8*>(sb + aoff[i]);
            am[i] = *reinterpret_cast<const bf16x8*>(sb + XP_PLANE_BYTES + aoff[i]);
            al[i] = *reinterpret_cast<const bf16x8*>(sb + 2 * XP_PLANE_BYTES + aoff[i]);
            bh[i] = *reinterpret_cast<const bf16x8*>(sb + boff[i]);
            bm[i] = *reinterpret_cast<const bf16x8*>(sb + XP_PLANE_BYTES + boff[i]);
            bl[i] = *reinterpret_cast<const bf16x8*>(sb + 2 * XP_PLANE_BYTES + boff[i]);
        }
        if constexpr (IL) {
            // the stage's fragments are in flight first; the DMA pieces of k-tile kt + 2 go out
            // between the MFMA groups (an LDS-DMA issue stalls the wave for tens of cycles)
            mfma6(ah, am, al, bh, bm, bl, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (kt + 2 < nkt) {
                int s2 = stage + 2;
                if (s2 >= XP_STAGES) s2 -= XP_STAGES;
                issue(kt + 2, s2);
            }
            __builtin_amdgcn_sched_barrier(0);
            mfma6(ah, am, al, bh, bm, bl, 0, 1);
            mfma6(ah, am, al, bh, bm, bl, 1, 0);
            mfma6(ah, am, al, bh, bm, bl, 1, 1);
        } else {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) mfma6(ah, am, al, bh, bm, bl, i, j);
        }
        if ((kt % XP_KT2) == XP_KT2 - 1 || kt + 1 == nkt) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    acc[i][j] += t[i][j];
#pragma unroll
                    for (int r = 0; r < 16; ++r) t[i][j][r] = 0.f;
                }
        }
        if (++stage == XP_STAGES) stage = 0;
    }

    // epilogue: NHWC fp32 store (output pixel index == GEMM row for regular rows)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int col = n0 + wn * 64 + j * 32 + l32;
        if (col >= d.Co) continue;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
                if (row < M) out[(long long)row * d.Co + col] = acc[i][j][r];
            }
    }
}


// ---------------------------------------------------------------------------------------
// Big-tile variant: 256 pixels x 128 channels per 256-thread workgroup, ONE workgroup per CU
// (one wave per SIMD), each wave 128 x 64 (4 x 2 blocks: 48 MFMAs per k-tile, twice the work
// per staged byte of the 128 x 128 tile's waves), a four-stage LDS ring (36 KiB per stage,
// DMA three k-tiles ahead) and the fragments of k-tile kt + 1 read from LDS into a second
// register set while the MFMAs of k-tile kt run, so one wave keeps its SIMD's matrix pipe fed:
//   iteration kt:  [DMA k-tile kt+3 between the first four MFMA groups]  MFMAs rows 0-63
//                  wait own DMA kt+1, barrier, ds_read fragments of kt+1  MFMAs rows 64-127
// Stage (kt+3) % 4 == (kt-1) % 4 was last read before the barrier of iteration kt-1, which
// every wave has passed when it issues the DMA.
// ---------------------------------------------------------------------------------------
constexpr int X2_BM = 256, X2_BN = 128, X2_STAGES = 4;
constexpr int X2_APLANE = X2_BM * 32, X2_BPLANE = X2_BN * 32;
constexpr int X2_STAGE_BYTES = 3 * X2_APLANE + 3 * X2_BPLANE;  // 36 KiB

template <bool REFLECT>
__global__ __launch_bounds__(XP_NT, 1) void conv_rows_x6p2_kernel(const dcs_conv_desc d, const __bf16* __restrict__ srcp,
                                                                const __bf16* __restrict__ wpp,
                                                                float* __restrict__ out, int gx, int gy) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[X2_STAGES * X2_STAGE_BYTES];

    const int T = gridDim.x;
    const int xcd = blockIdx.x & 7, q8 = T >> 3, r8 = T & 7;
    const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
    const int ntile = L % gy, mtile = L / gy;
    const int M = d.N * d.Ho * d.Wo;
    const int m0 = mtile * X2_BM, n0 = ntile * X2_BN;
    if (m0 >= M || mtile >= gx) return;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int Cs = d.Cs, KW = d.KW;
    const int nkt = d.KH * KW * Cs / XP_BK;
    const int kt_per_tap = Cs / XP_BK;
    const int slot = lane & 1;

    // ---- DMA lanes.  A: wave wid stages rows 64*wid + 32*p + lane/2 (p = 0, 1); B: rows 32*wid + lane/2
    const int per = d.Ho * d.Wo;
    const unsigned pix_bytes = (unsigned)Cs * 6u;
    int an[2], aoy[2], aox[2], ahalf[2];
    bool mvalid[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int row = 64 * wid + 32 * p + (lane >> 1);
        const int m = m0 + row;
        mvalid[p] = m < M;
        an[p] = mvalid[p] ? m / per : 0;
        const int rem = m - an[p] * per;
        aoy[p] = rem / d.Wo;
        aox[p] = rem - aoy[p] * d.Wo;
        ahalf[p] = slot ^ ((row >> 3) & 1);
    }
    auto tap_base = [&](int p, int j) -> unsigned {
        const int ty = j / KW, tx = j - (j / KW) * KW;
        int vy = aoy[p] + ty - d.pt, vx = aox[p] + tx - d.pl;
        bool ok = mvalid[p];
        if (REFLECT) {
            vy = vy < 0 ? -vy : (vy >= d.Hs ? 2 * (d.Hs - 1) - vy : vy);
            vx = vx < 0 ? -vx : (vx >= d.Ws ? 2 * (d.Ws - 1) - vx : vx);
        } else {
            ok = ok && (unsigned)vy < (unsigned)d.Hs && (unsigned)vx < (unsigned)d.Ws;
        }
        return ok ? (unsigned)((an[p] * d.Hs + vy) * d.Ws + vx) * pix_bytes + (unsigned)ahalf[p] * 48u : XP_OOB;
    };
    const int brow = 32 * wid + (lane >> 1);
    const unsigned bbase = (unsigned)(n0 + brow) * (unsigned)d.ldb * 6u + (unsigned)(slot ^ ((brow >> 3) & 1)) * 48u;
    const __amdgpu_buffer_rsrc_t ra = xp_rsrc(srcp), rb = xp_rsrc(wpp);

    int dj = 0, dc = 0, dkt = 0;  // (tap, k-tile within the tap), k-tile of the next DMA
    unsigned abase0 = tap_base(0, 0), abase1 = tap_base(1, 0);
    // piece g (0..8) of the next k-tile: A plane g/2 piece g&1 for g < 6, then B plane g-6
    auto piece = [&](int stage, int g) {
        unsigned char* s = lds + stage * X2_STAGE_BYTES;
        if (g < 6) {
            const int q = g >> 1, p = g & 1;
            const unsigned ab = p ? abase1 : abase0;
            const unsigned ao = ab == XP_OOB ? XP_OOB : ab + (unsigned)dc * 96u + 16u * q;
            xp_dma(ra, s + q * X2_APLANE + wid * 2048 + p * 1024, ao);
        } else {
            const int q = g - 6;
            xp_dma(rb, s + 3 * X2_APLANE + q * X2_BPLANE + wid * 1024, bbase + (unsigned)dkt * 96u + 16u * q);
        }
    };
    auto advance = [&]() {
        ++dkt;
        if (++dc == kt_per_tap) {
            dc = 0;
            ++dj;
            if (dj < d.KH * KW) { abase0 = tap_base(0, dj); abase1 = tap_base(1, dj); }
        }
    };
    auto issue_all = [&](int stage) {
#pragma unroll
        for (int g = 0; g < 9; ++g) piece(stage, g);
        advance();
    };

    floatx16 acc[4][2], t[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) { acc[i][j][r] = 0.f; t[i][j][r] = 0.f; }

    const int l32 = lane & 31, hh = lane >> 5;
    int aoff[4], boff[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = wm * 128 + i * 32 + l32;
        aoff[i] = row * 32 + 16 * (hh ^ ((row >> 3) & 1));
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int col = wn * 64 + j * 32 + l32;
        boff[j] = 3 * X2_APLANE + col * 32 + 16 * (hh ^ ((col >> 3) & 1));
    }
    // fragments: one A set [plane][block] refilled in two halves, two B sets [set][plane][block]
    bf16x8 fa[3][4], fb[2][3][2];
    auto read_a = [&](int stage, int i0) {
        const unsigned char* sb = lds + stage * X2_STAGE_BYTES;
#pragma unroll
        for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int i = i0; i < i0 + 2; ++i) fa[q][i] = *reinterpret_cast<const bf16x8*>(sb + q * X2_APLANE + aoff[i]);
    };
    auto read_b = [&](int set, int stage) {
        const unsigned char* sb = lds + stage * X2_STAGE_BYTES;
#pragma unroll
        for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int j = 0; j < 2; ++j) fb[set][q][j] = *reinterpret_cast<const bf16x8*>(sb + q * X2_BPLANE + boff[j]);
    };
    auto mfma6 = [&](int set, int i, int j) {  // smallest terms first (planes: 0 hi, 1 mid, 2 lo)
        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][i], fb[set][1][j], t[i][j], 0, 0, 0);
        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2][i], fb[set][0][j], t[i][j], 0, 0, 0);
        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fb[set][2][j], t[i][j], 0, 0, 0);
        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][i], fb[set][0][j], t[i][j], 0, 0, 0);
        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fb[set][1][j], t[i][j], 0, 0, 0);
        t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fb[set][0][j], t[i][j], 0, 0, 0);
    };

    // prologue: k-tiles 0, 1, 2 in flight; fragments of k-tile 0
    issue_all(0);
    if (nkt > 1) issue_all(1);
    if (nkt > 2) issue_all(2);
    if (nkt > 2) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
    else if (nkt > 1) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    read_a(0, 0);
    read_a(0, 2);
    read_b(0, 0);

    int stage = 0;
    for (int kt = 0; kt < nkt; kt += 2) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {  // unrolled by two: the B fragment set index is static
            const int k = kt + u;
            if (k < nkt) {
                int s3 = stage + 3;
                if (s3 >= X2_STAGES) s3 -= X2_STAGES;
                int s1 = stage + 1;
                if (s1 >= X2_STAGES) s1 -= X2_STAGES;
                const bool dma = k + 3 < nkt, next = k + 1 < nkt;
                // rows 0-63 of the wave, with the DMA pieces of k-tile k+3 between the groups
                mfma6(u, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
                if (dma) { piece(s3, 0); piece(s3, 1); piece(s3, 2); }
                __builtin_amdgcn_sched_barrier(0);
                mfma6(u, 0, 1);
                __builtin_amdgcn_sched_barrier(0);
                if (dma) { piece(s3, 3); piece(s3, 4); }
                __builtin_amdgcn_sched_barrier(0);
                mfma6(u, 1, 0);
                __builtin_amdgcn_sched_barrier(0);
                if (dma) { piece(s3, 5); piece(s3, 6); }
                __builtin_amdgcn_sched_barrier(0);
                mfma6(u, 1, 1);
                __builtin_amdgcn_sched_barrier(0);
                if (dma) { piece(s3, 7); piece(s3, 8); advance(); }
                __builtin_amdgcn_sched_barrier(0);
                if (next) {
                    // own pieces of k-tile k+1 landed (k+2, k+3 may fly), then everyone's
                    if (k + 3 < nkt) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
                    else if (k + 2 < nkt) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
                    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __builtin_amdgcn_s_barrier();
                    asm volatile("" ::: "memory");
                    read_a(s1, 0);      // rows 0-63 of k+1 (their registers are free now)
                    read_b(u ^ 1, s1);
                }
                __builtin_amdgcn_sched_barrier(0);
                // rows 64-127 of the wave
                mfma6(u, 2, 0);
                mfma6(u, 2, 1);
                mfma6(u, 3, 0);
                mfma6(u, 3, 1);
                __builtin_amdgcn_sched_barrier(0);
                if (next) read_a(s1, 2);
                __builtin_amdgcn_sched_barrier(0);
                if ((k % XP_KT2) == XP_KT2 - 1 || k + 1 == nkt) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            acc[i][j] += t[i][j];
#pragma unroll
                            for (int r = 0; r < 16; ++r) t[i][j][r] = 0.f;
                        }
                }
                if (++stage == X2_STAGES) stage = 0;
            }
        }
    }

#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int col = n0 + wn * 64 + j * 32 + l32;
        if (col >= d.Co) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wm * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
                if (row < M) out[(long long)row * d.Co + col] = acc[i][j][r];
            }
    }
}

}  // namespace
}  // namespace dcs

using namespace dcs;

extern "C" int dcs_split_x6(const float* src, int64_t n, void* dst, void* stream) {
    if (!src || !dst || n <= 0 || n % 8 || (reinterpret_cast<uintptr_t>(src) & 15) ||
        (reinterpret_cast<uintptr_t>(dst) & 15))
        return fail(DCS_E_INVALID, "split_x6: n must be a positive multiple of 8, pointers 16-byte aligned");
    const long long ng = n / 8;
    hipLaunchKernelGGL(split_x6_kernel, dim3((unsigned)cdiv(ng, 256)), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const float4*>(src), reinterpret_cast<uint4*>(dst), ng);
    return check_launch("split_x6");
}

extern "C" int dcs_conv_rows_x6p_ok(const dcs_conv_desc* dp) {
    if (!dp) return 0;
    const dcs_conv_desc& d = *dp;
    const long long src_bytes = (long long)d.N * d.Hs * d.Ws * d.Cs * 6;
    const long long w_bytes = (long long)cdiv(d.Co, XP_BN) * XP_BN * d.ldb * 6;
    return d.korder == DCS_KORDER_TAP && d.parity == 0 && d.stride == 1 && d.up == 1 && d.Cs % XP_BK == 0 &&
           d.Co % XP_BN == 0 &&
           d.csplit == d.Cs && d.pro_act == DCS_ACT_NONE && d.epi_act == DCS_ACT_NONE &&
           d.ldb >= d.KH * d.KW * d.Cs && d.ldb % 32 == 0 && d.KH * d.KW <= 64 &&
           (d.pad_mode == DCS_PAD_ZERO || d.pad_mode == DCS_PAD_REFLECT) &&
           d.Ho == d.Hs + 2 * d.pt - d.KH + 1 && d.Wo == d.Ws + 2 * d.pl - d.KW + 1 &&
           src_bytes < 0x7ffff000LL - 4096 && w_bytes < 0x7ffff000LL - 4096 &&
           (long long)d.N * d.Ho * d.Wo < (1LL << 31);
}

// srcp: dcs_split_x6 of the NHWC fp32 source; wpp: dcs_split_x6 of the N-major packed weights
// ([ncols][ldb], ncols a multiple of 128).  Output NHWC fp32 [N, Ho, Wo, Co].
extern "C" int dcs_conv_rows_x6p(const dcs_conv_desc* dp, const void* srcp, const void* wpp, float* out,
                                 void* stream) {
    if (!dp || !srcp || !wpp || !out) return fail(DCS_E_INVALID, "conv_rows_x6p: null argument");
    if (!dcs_conv_rows_x6p_ok(dp))
        return fail(DCS_E_INVALID, "conv_rows_x6p: needs stride-1 regular rows, Cs % 16 == 0, Co % 128 == 0, "
                                   "no prologue/epilogue, sources < 2 GiB");
    const dcs_conv_desc& d = *dp;
    if (d.pad_mode == DCS_PAD_REFLECT && (d.pt >= d.Hs || d.pl >= d.Ws))
        return fail(DCS_E_INVALID, "conv_rows_x6p: reflect pad larger than the input");
    const long long M = (long long)d.N * d.Ho * d.Wo;
    hipStream_t s = as_stream(stream);
    const __bf16* a = reinterpret_cast<const __bf16*>(srcp);
    const __bf16* w = reinterpret_cast<const __bf16*>(wpp);
    static const char* var_env = getenv("DCS_X6P_VARIANT");  // "3" (default), "1": 128 x 128; "2": 256 x 128
    const char* var = var_env ? var_env : "3";
    if (var[0] == '2') {
        const int gx = (int)cdiv(M, X2_BM), gy = d.Co / X2_BN;
        const dim3 grid((unsigned)(gx * gy));
        if (d.pad_mode == DCS_PAD_REFLECT)
            hipLaunchKernelGGL((conv_rows_x6p2_kernel<true>), grid, dim3(XP_NT), 0, s, d, a, w, out, gx, gy);
        else
            hipLaunchKernelGGL((conv_rows_x6p2_kernel<false>), grid, dim3(XP_NT), 0, s, d, a, w, out, gx, gy);
        return check_launch("conv_rows_x6p2");
    }
    const int gx = (int)cdiv(M, XP_BM), gy = d.Co / XP_BN;
    const dim3 grid((unsigned)(gx * gy));
    const int il = var[0] == '3' ? 2 : 1;  // "3": software-pipelined fragments, "1": DMA between MFMA groups
    if (d.pad_mode == DCS_PAD_REFLECT) {
        if (il == 2) hipLaunchKernelGGL((conv_rows_x6p_kernel<true, 2>), grid, dim3(XP_NT), 0, s, d, a, w, out, gx, gy);
        else hipLaunchKernelGGL((conv_rows_x6p_kernel<true, 1>), grid, dim3(XP_NT), 0, s, d, a, w, out, gx, gy);
    } else {
        if (il == 2) hipLaunchKernelGGL((conv_rows_x6p_kernel<false, 2>), grid, dim3(XP_NT), 0, s, d, a, w, out, gx, gy);
        else hipLaunchKernelGGL((conv_rows_x6p_kernel<false, 1>), grid, dim3(XP_NT), 0, s, d, a, w, out, gx, gy);
    }
    return check_launch("conv_rows_x6p");
}
