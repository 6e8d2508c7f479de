// 3x3 stride-1 'same' convolution over whole image rows on f16x3 operands, the source window of a
// tile staged once per 16-channel slice (the residual-block convolutions of modules/model.py:72-80:
// forward with reflection padding, and the interior of the data gradient with zero padding over
// flipped weights).
//
// conv.hip's rows pass gathers A[pixel][(tap, channel)] into LDS per k-tile: every source value is
// fetched, split into hi/lo fp16 and stored nine times (once per tap).  Here a workgroup owns 256
// consecutive pixels of one image (R = 256 / W whole rows) x 128 output channels, and per 16-channel
// slice stages the (R + 2) x (W + 2) source window once (520 pixels at W = 128: 2.0 values per output
// pixel instead of 9); the nine taps read their MFMA fragments from the window at a per-tap pixel
// offset.  The weights arrive pre-split (dcs_pack_weights_h3: hi / lo fp16 planes, slice-major K), so
// their k-tiles are copied to LDS without arithmetic.
//
// K loop: 16 slices x 3 kernel rows (ty) = 48 k-tiles of 48 k; a k-tile is three 16-k sub-tiles
// (tx = 0, 1, 2) of 2 x 2 blocks x 3 products (lo*hi, hi*lo, hi*hi) per wave.  One inner fp32
// accumulation chain per slice (144 k), added to the running sum (two-level, as conv.hip).
// 8 waves = 4 (pixels) x 2 (channels) of 64 x 64; one workgroup per CU (115 KB of LDS).  The k-tile
// schedule (LDS-DMA for B, one window unit in flight, fragments read ahead, staggered wave pairs) is
// described at conv3_win_h3_kernel.
#include "common.hpp"
#include "conv_common.hpp"
#include <type_traits>


namespace dcs {
namespace {

#ifndef WIN_TIMING
#define WIN_TIMING 0
#endif
#if WIN_TIMING  // probe build only: per-workgroup phase timestamps (scripts/r05/win_timing.py)
__device__ unsigned long long g_win_t[16384 * 5];
#endif
#ifndef CLK_PROBE
#define CLK_PROBE 0
#endif
#ifndef DCS_WGRAD16  // f16x3 residual weight gradient on the 16x16x32 kernel (0: the 32x32x16 one; A/B builds)
#define DCS_WGRAD16 1
#endif
#ifndef DCS_WW_F16_EARLY  // f16 weight gradient (wgrad3_win_h3_kernel<1>): both rows of the next barrier loaded at
                          // its start and staged by its second row, one accumulation level (0: each row's loads
                          // issued at its start and staged at its end).  1.5 % slower per launch, 0.2 % in the
                          // step (profiles/r06/ab/r06an_*): not the loads' latency; off
#define DCS_WW_F16_EARLY 0
#endif
#ifndef DCS_WGRAD16_F16  // the f16 mode's residual weight gradient on it too (NP 1, two rows per barrier): bit-compatible
                         // with the tests' bounds but 1-2 % slower per launch than wgrad3_win_h3_kernel<1> (kbench
                         // profiles/r06/ab/r06ai_kb_*), neutral in the step; off
#define DCS_WGRAD16_F16 0
#endif
#ifndef DCS_WIN16  // f16x3 residual convs on the 16x16x32 window kernel (0: the 32x32x16 one; A/B builds)
#define DCS_WIN16 1
#endif
#ifndef DCS_WW_STAGE  // where the 16x16x32 weight gradient stages the next rows (1: beside the second k-step's
                      // MFMAs, -1.5 % per launch; 0: between its k-steps; 2-4: rejected placements)
#define DCS_WW_STAGE 1
#endif
#ifndef DCS_WIN16_F16  // the f16 mode's residual convs on the 16x16x32 window kernel too (NP 1, three k-steps of
                       // 16 MFMAs per barrier, DCS_WIN16_G3; 0: conv3_win_h3_kernel<1>, one barrier per 36-MFMA
                       // slice): -5..6 % per launch, f16 step 133.5 -> 131.0 ms (profiles/r06/ab/r06ag_*)
#define DCS_WIN16_F16 1
#endif
#ifndef DCS_WIN16_G3  // NP 1 on the 16x16x32 kernel: three k-steps per barrier (0: one, as f16x3; measured neutral)
#define DCS_WIN16_G3 1
#endif
#ifndef DCS_WIN_ASYNC  // the 16x16x32 window conv's unit loads as asm with explicit vmcnt waits and four B buffers
                       // (each B DMA two k-steps to land instead of one): bit-identical, 1 % slower per launch in
                       // kbench, neutral in the step (profiles/r06/ab/r06ad_*): off
#define DCS_WIN_ASYNC 0
#endif
#ifndef DCS_RING16  // the padded-grid ring of the residual data gradient on ring16_kernel (0: the rows pass)
#define DCS_RING16 1
#endif
#if CLK_PROBE  // probe build only: core-clock and wall-clock counters per weight-gradient workgroup
__device__ unsigned long long g_clk[4096 * 4];
#endif

constexpr int WIN_BN = 128, WIN_NT = 512;  // tiles: 256 pixels (whole rows) x WIN_BN channels
constexpr int WIN_PIX = 520;             // window pixels for W <= 128: (256 / W + 2) * (W + 2) <= 520
// halves per B plane-slot: 128 rows x 16 k + 48 (96 B: the three tx slots of a row, written by
// neighbouring lanes, land on distinct banks)
constexpr int WIN_SLOT = 128 * 16 + 48;
// window staging units (pixel, 8-channel half) per thread: the interior columns only, (256 / W + 2) x W
// pixels x 2 halves <= 1024 for W <= 128
constexpr int WIN_UNITS = 2;

struct WinArgs {
    int N, H, W, C, Co;  // source NHWC [N][H][W][C]; output NHWC [N][H][W][Co]
    int reflect;         // 1: reflection padding (forward), 0: zero padding (data gradient interior)
    int R, tiles;        // image rows per tile (256 / W), tiles per image (H / R)
    int gy;              // column tiles (Co / 128)
    int rng_n;           // partial maxima of the source range record
};

typedef short shortx8 __attribute__((ext_vector_type(8)));

// half-element offset of (buffer, plane, window pixel, 8-channel half) in the window region: the
// pixels of a pair swap on odd groups of 8 pixels and the 16-byte halves of a pixel on odd groups of
// 16, so the fragment reads (every other pixel from any start: the MFMA row blocks interleave) and the
// staging writes are both conflict-free
__device__ __forceinline__ int win_off(int buf, int pl, int wpix, int h) {
    return ((buf * 2 + pl) * WIN_PIX + (wpix ^ ((wpix >> 3) & 1))) * 16 + 8 * (h ^ ((wpix >> 4) & 1));
}
// tile pixel of accumulator element r of row block i (the blocks interleave: block i holds pixels
// 2m + i of the wave's 64, so block 0 at tap tx + 1 reads the fragment block 1 read at tap tx)
__device__ __forceinline__ int win_pix(int wm, int i, int r, int kh) {
    return wm * 64 + 2 * ((r & 3) + 8 * (r >> 2) + 4 * kh) + i;
}
// B: (buffer, plane, tx, output-channel row, half)
__device__ __forceinline__ int wb_off(int buf, int pl, int tx, int row, int h) {
    return (buf * 6 + pl * 3 + tx) * WIN_SLOT + row * 16 + 8 * (h ^ ((row >> 3) & 1));
}

// one global_load_lds_dwordx4: lane L's 16 bytes land at LDS byte address lds + 16 L.  Inline asm: a
// compiler-emitted LDS-DMA makes hipcc wait for it before every later LDS read it cannot tell apart
// from the DMA's destination.  The kernel retires these itself (s_waitcnt vmcnt before the barrier
// that publishes the buffer); the compiler's own vmcnt waits only grow more conservative beside them.
__device__ __forceinline__ void win_glds(const void* base, unsigned voff, unsigned lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(base), "s"(lds)
                 : "memory");
}

// IN statistics of the tile (as conv.hip rows_in_stats, BM 256 x BN 128): per column the tile's
// count / mean / M2 / max / first argmax, merged over the four pixel waves in a fixed order
__device__ __forceinline__ void win_stats(const floatx16 (&acc)[2][2], int p0, int n0, int Co, int wm, int wn,
                                          int lane, int tid, float* lds, Part* __restrict__ parts, long long chunk) {
    Part* sp = reinterpret_cast<Part*>(lds);  // [4][128]
    const int hi = lane >> 5;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int colL = wn * 64 + j * 32 + (lane & 31);
        float s = 0.f, mx = -INFINITY;
        int am = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r)  // increasing pixel order (first maximum)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const float v = acc[i][j][r];
                s += v;
                if (v > mx) { mx = v; am = p0 + win_pix(wm, i, r, hi); }
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
        if (hi == 0) {
            const float dl = mb - mean;
            Part p;
            p.cnt = 64.f;
            p.mean = mean + 0.5f * dl;
            p.m2 = m2 + m2b + dl * dl * 16.f;
            p.mx = mx;
            p.amax = am;
            if (mxb > mx || (mxb == mx && amb < am)) { p.mx = mxb; p.amax = amb; }
            p.pad[0] = p.pad[1] = p.pad[2] = 0;
            sp[wm * WIN_BN + colL] = p;
        }
    }
    __syncthreads();
    if (tid < WIN_BN && n0 + tid < Co) {
        Part a = sp[tid];
#pragma unroll
        for (int w = 1; w < 4; ++w) {
            const Part b = sp[w * WIN_BN + tid];
            const float tot = a.cnt + b.cnt, dl = b.mean - a.mean;
            a.mean += dl * (b.cnt / tot);
            a.m2 += b.m2 + dl * dl * (a.cnt * b.cnt / tot);
            a.cnt = tot;
            if (b.mx > a.mx || (b.mx == a.mx && b.amax < a.amax)) { a.mx = b.mx; a.amax = b.amax; }
        }
        parts[chunk * Co + n0 + tid] = a;
    }
}

// The InstanceNorm backward's partial sums over a data-gradient tile (IBW instances): the output is
// da of a layer a = act(IN(y)); per channel sum g and sum g * xhat with xhat = y * sc + sh and
// g = da * act'(xhat), over the tile's pixels except the ones the reflection ring fold still adds to
// (rows 1, H - 2 and columns 1, W - 2: the fold kernel sums those with their final values).
struct IbwArgs {
    const float* y;
    const float* sc;
    const float* sh;
    Sum2* parts;  // [N][nchunk][Co]
    int act, nchunk;
};

// y of the tile's outputs, every load issued before the first use
__device__ __forceinline__ void win_ibw_load(float (&yv)[2][2][16], const IbwArgs& ib, long long obase, int p0, int Co,
                                             int n0, int wm, int wn, int lane) {
    const int kh = lane >> 5, l32 = lane & 31;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int pix = p0 + win_pix(wm, i, r, kh);
                yv[i][j][r] = ib.y[obase + (long long)pix * Co + n0 + wn * 64 + j * 32 + l32];
            }
}

__device__ __forceinline__ void win_ibw(const floatx16 (&acc)[2][2], const float (&yv)[2][2][16], const IbwArgs& ib,
                                        int n, int p0, int H, int W, int Co, int n0, int wm, int wn, int lane, int tid,
                                        int tile, float* lds) {
    const int kh = lane >> 5, l32 = lane & 31;
    Sum2* sp = reinterpret_cast<Sum2*>(lds);  // [4][128]; the k-loop's last barrier freed the LDS
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int col = n0 + wn * 64 + j * 32 + l32;
        const float s = ib.sc[(long long)n * Co + col], b = ib.sh[(long long)n * Co + col];
        float sa = 0.f, sb = 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int pix = p0 + win_pix(wm, i, r, kh);
                const int py = pix >> __builtin_ctz(W), px = pix & (W - 1);  // (W is a power of two)
                if (py == 1 || py == H - 2 || px == 1 || px == W - 2) continue;  // the ring fold's pixels
                const float xh = fmaf(yv[i][j][r], s, b);
                const float g = acc[i][j][r] * act_grad(xh, ib.act);
                sa += g;
                sb = fmaf(g, xh, sb);
            }
        sa += __shfl_xor(sa, 32, 64);  // the same operand pair on both lanes: order-free
        sb += __shfl_xor(sb, 32, 64);
        if (kh == 0) sp[wm * 128 + wn * 64 + j * 32 + l32] = Sum2{sa, sb};
    }
    __syncthreads();
    if (tid < 128 && n0 + tid < Co) {
        Sum2 t = sp[tid];
#pragma unroll
        for (int w = 1; w < 4; ++w) {
            t.a += sp[w * 128 + tid].a;
            t.b += sp[w * 128 + tid].b;
        }
        ib.parts[((long long)n * ib.nchunk + tile) * Co + n0 + tid] = t;
    }
}

// NP: products per fragment pair (3: f16x3, hi*lo + lo*hi + hi*hi; 1: f16, hi*hi with the hi planes only);
// IBW: the InstanceNorm-backward partial sums of the output (data gradients without addend)
//
// Schedule of a k-tile (one barrier each), built so that the fragment reads run ahead of the MFMAs
// that consume them within the 256-register budget of two waves per SIMD (128 of them the two-level
// accumulators):
//   * B by LDS-DMA (win_glds): tile tt + 1 is issued into the other buffer at the top of tile tt and
//     retired (vmcnt) before tile tt's barrier, so no register holds B in flight;
//   * the window of the next slice one staging unit per k-tile (units 0, 1 in kernel rows 0, 1): only
//     one unit's eight floats are live at a time.  Only the window's interior columns are loaded (two
//     units per thread); the halo columns are written by the units of source columns 1 and W - 2
//     (reflection) or zeroed once (zero padding);
//   * B fragments one tap ahead (tap tx + 1's read before tap tx's MFMAs, pinned by sched_barrier);
//   * waves 4-7 (the partners of waves 0-3 on their SIMDs) store their staging unit at the top of the
//     next k-tile instead of after their MFMAs, so the two waves of a SIMD are not in the same phase.
template <int NP, bool IBW>
__global__ __launch_bounds__(WIN_NT, 1) void conv3_win_h3_kernel(WinArgs a, const float* __restrict__ src,
                                                                 const _Float16* __restrict__ wh,
                                                                 const _Float16* __restrict__ wl,
                                                                 const float* __restrict__ rng,
                                                                 const int* __restrict__ wexp,
                                                                 const float* __restrict__ addend,
                                                                 float* __restrict__ out, Part* __restrict__ parts,
                                                                 IbwArgs ib) {
    // f16x3: B k-tiles [2][6 = plane x tx][WIN_SLOT]; f16 (NP 1): B slices [2][9 taps][WIN_SLOT] (one
    // barrier per slice, see below)
    constexpr int BHALVES = NP == 3 ? 2 * 6 * WIN_SLOT : 2 * 9 * WIN_SLOT;
    __shared__ __attribute__((aligned(16))) _Float16 smem[2 * 2 * WIN_PIX * 16 + BHALVES + 8];
    _Float16* const Wn = smem;                               // [2][2][WIN_PIX][16]
    _Float16* const Bs = smem + 2 * 2 * WIN_PIX * 16;
    _Float16* const Wspare = Bs + BHALVES;                   // 16 bytes nobody reads

#if WIN_TIMING
    const unsigned long long tm0 = wall_clock64();
    unsigned long long tm1 = 0, tm2 = 0;
#endif
    const int T = gridDim.x;
    const int L = xcd_remap(blockIdx.x, T);
    const int ntile = L % a.gy, mt = L / a.gy;
    const int n = mt / a.tiles, tile = mt - n * a.tiles;
    const int n0 = ntile * WIN_BN;
    const int y0 = tile * a.R;                 // first image row of the tile
    const int W = a.W, WP = a.W + 2, C = a.C;
    const int K = 9 * C;                       // packed K (slice-major: (c/16)*144 + tap*16 + c%16)
    const int nslice = C / 16;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int l32 = lane & 31, kh = lane >> 5;

    // the source exponent (ea, asc) is read in the prologue, its loads beside the first staging loads
    int ea = 0;
    float asc = 1.f;
    const int eb = __builtin_amdgcn_readfirstlane(wexp[0]);

    // window staging units of this thread: (pixel, 8-channel half) of the window's interior columns
    // ((R + 2) x W pixels: 2 units per thread at W <= 128).  uoff: byte offset of the unit's source
    // channel 0 (-1: zero padding); uwd: its window pixel (bits 0-15) and the halo pixel it also writes
    // (bits 16-31), each + 1 (0: none)
    const int nint = (a.R + 2) * W;
    int uoff[WIN_UNITS], uwd[WIN_UNITS];
#pragma unroll
    for (int q = 0; q < WIN_UNITS; ++q) {
        const int u = tid + q * WIN_NT;
        const int ip = u >> 1, h = u & 1;
        uoff[q] = -1;
        uwd[q] = 0;
        if (ip < nint) {
            const int wr = ip >> __builtin_ctz(W), sx = ip & (W - 1);  // (W is a power of two)
            int dup = -1;
            int sy = y0 - 1 + wr;
            bool ok = true;
            if (a.reflect) {
                sy = sy < 0 ? -sy : (sy >= a.H ? 2 * a.H - 2 - sy : sy);
                if (sx == 1) dup = wr * WP;                   // column -1 reflects column 1
                else if (sx == W - 2) dup = wr * WP + W + 1;  // column W reflects column W - 2
            } else {
                ok = sy >= 0 && sy < a.H;
            }
            uwd[q] = (wr * WP + sx + 2) | ((dup + 1) << 16);
            if (ok) uoff[q] = (((n * a.H + sy) * W + sx) * C + 8 * h) * 4;
        }
    }
    if (!a.reflect) {  // zero halo columns of both buffers and planes
        for (int i = tid; i < 2 * 2 * (a.R + 2) * 2 * 2; i += WIN_NT) {
            const int h = i & 1, side = (i >> 1) & 1, rest = i >> 2;
            const int wr = rest % (a.R + 2), bp = rest / (a.R + 2);
            *reinterpret_cast<f16x8*>(Wn + win_off(bp >> 1, bp & 1, wr * WP + side * (W + 1), h)) = f16x8{};
        }
    }
    const __amdgpu_buffer_rsrc_t srsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, 0x7fffff00, 0x00020000);
    float4 wq_[2];  // the unit in flight
    auto win_load_u = [&](int q, int s) {  // unconditional (clamped offset): see the k loop
        const int off = uoff[q] >= 0 ? uoff[q] + s * 64 : 0x7fffffbf;  // 16 channels = 64 B per slice
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(srsrc, off, 0, 0);
        u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(srsrc, off + 16, 0, 0);
        __builtin_memcpy(&wq_[0], &v0, 16);
        __builtin_memcpy(&wq_[1], &v1, 16);
    };
    // unconditional store (a unit past the window writes the spare slot): a store under a branch lets
    // the compiler sink the unit's load into the branch, next to its use
    auto win_store_u = [&](int q, int buf) {
        const int h = (tid + q * WIN_NT) & 1;
        const int wp = (uwd[q] & 0xffff) - 1, wd = (uwd[q] >> 16) - 1;
        f16x8 hi, lo;
        split8h(wq_[0], wq_[1], asc, hi, lo);
        *reinterpret_cast<f16x8*>(wp >= 0 ? Wn + win_off(buf, 0, wp, h) : Wspare) = hi;
        if constexpr (NP == 3) *reinterpret_cast<f16x8*>(wp >= 0 ? Wn + win_off(buf, 1, wp, h) : Wspare) = lo;
        if (wd >= 0) {
            *reinterpret_cast<f16x8*>(Wn + win_off(buf, 0, wd, h)) = hi;
            if constexpr (NP == 3) *reinterpret_cast<f16x8*>(Wn + win_off(buf, 1, wd, h)) = lo;
        }
    };

    // B k-tile (slice s, kernel row ty) by LDS-DMA: 2 planes x 3 tx slots x 128 rows = 24 blocks of
    // 1 KB (plane, tx slot, 32-row block), three per wave; a block's LDS image is lane-linear (lane L ->
    // row L / 2, half position L % 2), so the wb_off swizzle goes on the source side: lane L fetches
    // half (L % 2) ^ bit 3 of its row.  The lane part of the source offset is the same for the three
    // blocks (bit 3 of the row is bit 3 of L / 2); the block part and the plane are wave-uniform.
    unsigned dsu[3], ddst[3];
    const _Float16* dbase[3];
    const unsigned dlane = 2u * (unsigned)((n0 + (lane >> 1)) * K + 8 * ((lane & 1) ^ ((lane >> 4) & 1)));
    {
        const unsigned bs_lds = (unsigned)(uintptr_t)(__attribute__((address_space(3))) _Float16*)Bs;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int c = __builtin_amdgcn_readfirstlane(wid) * 3 + i, pl = c / 12, rem = c - pl * 12;
            const int tx = rem >> 2, rb = rem & 3;
            dsu[i] = 2u * (unsigned)(rb * 32 * K + tx * 16);
            dbase[i] = pl ? wl : wh;
            ddst[i] = __builtin_amdgcn_readfirstlane(bs_lds + 2u * (unsigned)((pl * 3 + tx) * WIN_SLOT + rb * 32 * 16));
        }
    }
    auto b_dma = [&](int t, int buf) {  // B tile t into buffer buf
        const int s_ = t / 3, ty_ = t - 3 * (t / 3);
        const unsigned kb = 2u * (unsigned)(s_ * 144 + ty_ * 48);
#pragma unroll
        for (int i = 0; i < 3; ++i) win_glds(dbase[i], dlane + (dsu[i] + kb), ddst[i] + 2u * (unsigned)(buf * 6 * WIN_SLOT));
    };

    // window pixel of this lane's block-0 output pixel 2m (tap (0, 0) = the window's top-left); its
    // block-1 pixel 2m + 1 is the next one (W is even: the pair shares a row)
    int wbe;
    {
        const int q = wm * 64 + 2 * l32;
        wbe = (q >> __builtin_ctz(W)) * WP + (q & (W - 1));
    }

    floatx16 acc[2][2], t[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) { acc[i][j][r] = 0.f; t[i][j][r] = 0.f; }

    if constexpr (NP == 1) {
        // f16: one product per fragment pair, so a 48-k tile holds only 12 MFMAs per wave; instead the
        // whole slice (9 taps, hi planes only) is staged per barrier: 36 MFMAs per wave between
        // barriers.  One accumulation level: the fp32 chain over all 9 C products (K <= 4608) rounds far
        // below the fp16 operands' 2^-11, so the two-level sum of the f16x3 path buys nothing here.  B slice by LDS-DMA, 36 blocks of 1 KB (tap, 32-row block), blocks w, w + 8, ...
        // of wave w.
        unsigned sdst[5], ssu[5];
        {
            const unsigned bs_lds = (unsigned)(uintptr_t)(__attribute__((address_space(3))) _Float16*)Bs;
            const int w = __builtin_amdgcn_readfirstlane(wid);
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                const int c = w + 8 * i < 36 ? w + 8 * i : 35, tap = c >> 2, rb = c & 3;
                ssu[i] = 2u * (unsigned)(rb * 32 * K + tap * 16);
                sdst[i] = __builtin_amdgcn_readfirstlane(bs_lds + 2u * (unsigned)(tap * WIN_SLOT + rb * 32 * 16));
            }
        }
        const bool fifth = wid + 32 < 36;  // wave-uniform: waves 0-3 issue a fifth block
        auto s_dma = [&](int sl, int buf) {
            const unsigned kb = 2u * (unsigned)(sl * 144);
#pragma unroll
            for (int i = 0; i < 4; ++i) win_glds(wh, dlane + (ssu[i] + kb), sdst[i] + 2u * (unsigned)(buf * 9 * WIN_SLOT));
            if (fifth) win_glds(wh, dlane + (ssu[4] + kb), sdst[4] + 2u * (unsigned)(buf * 9 * WIN_SLOT));
        };
        // prologue: every load of slice 0 (and the exponent's) in flight before the first store
        s_dma(0, 0);
        win_load_u(1, 0);
        const float4 wp1[2] = {wq_[0], wq_[1]};
        win_load_u(0, 0);
        ea = f16x3_exp(rng, a.rng_n);
        asc = __builtin_ldexpf(1.f, ea);
        win_store_u(0, 0);
        wq_[0] = wp1[0];
        wq_[1] = wp1[1];
        win_store_u(1, 0);
        __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0): the DMA has landed
        __syncthreads();
        auto sloop = [&](auto role_tag) {
            constexpr int ROLE = decltype(role_tag)::value;
            for (int s = 0; s < nslice; ++s) {
                const int buf = s & 1;
                const int sn = s + 1 < nslice ? s + 1 : s;
                // the next slice into the other buffers (last read before this slice's top barrier):
                // B by DMA now, the window's two units loaded now and stored after the kernel row that
                // is this wave's staging point (ROLE 0: the last, ROLE 1: the second)
                s_dma(sn, buf ^ 1);
                win_load_u(1, sn);  // unit 1 into wq_, moved to wq1
                const float4 wq1[2] = {wq_[0], wq_[1]};
                win_load_u(0, sn);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int ty = 0; ty < 3; ++ty) {
                    f16x8 fh[4];
#pragma unroll
                    for (int f = 0; f < 4; ++f)
                        fh[f] = *reinterpret_cast<const f16x8*>(Wn + win_off(buf, 0, wbe + ty * WP + f, kh));
                    f16x8 pb[2][2];
                    auto rd_b = [&](int tx, int slot) {
#pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            const int row = wn * 64 + j * 32 + l32;
                            pb[slot][j] = *reinterpret_cast<const f16x8*>(
                                Bs + (buf * 9 + ty * 3 + tx) * WIN_SLOT + row * 16 + 8 * (kh ^ ((row >> 3) & 1)));
                        }
                    };
                    rd_b(0, 0);
#pragma unroll
                    for (int tx = 0; tx < 3; ++tx) {
                        if (tx < 2) rd_b(tx + 1, (tx + 1) & 1);
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int i = 0; i < 2; ++i)
#pragma unroll
                            for (int j = 0; j < 2; ++j)
                                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fh[tx + i], pb[tx & 1][j], acc[i][j], 0, 0, 0);
                    }
                    if (ty == (ROLE == 0 ? 2 : 1)) {  // staging point of this wave (kernel row 2 / 1)
                        __builtin_amdgcn_sched_barrier(0);
                        win_store_u(0, buf ^ 1);
                        wq_[0] = wq1[0];
                        wq_[1] = wq1[1];
                        win_store_u(1, buf ^ 1);
                    }
                }
                __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0): this wave's DMAs landed
                __syncthreads();
            }
        };
        if (wid >= 4) sloop(std::integral_constant<int, 1>{});
        else sloop(std::integral_constant<int, 0>{});
    } else {
    // prologue: window of slice 0, B tile 0, every load (and the exponent's) in flight before the first
    // store
    b_dma(0, 0);
    win_load_u(1, 0);
    const float4 wp1[2] = {wq_[0], wq_[1]};
    win_load_u(0, 0);
    ea = f16x3_exp(rng, a.rng_n);
    asc = __builtin_ldexpf(1.f, ea);
    win_store_u(0, 0);
    wq_[0] = wp1[0];
    wq_[1] = wp1[1];
    win_store_u(1, 0);
    __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0): the DMA has landed
    __syncthreads();
#if WIN_TIMING
    tm1 = wall_clock64();
#endif

    // every global load below is unconditional (offsets clamped at the end): a load under a branch
    // makes the compiler wait for all outstanding loads (vmcnt(0)) at the next consumer
    const int last = 3 * nslice - 1;
    auto kloop = [&](auto role_tag) {
        constexpr int ROLE = decltype(role_tag)::value;
        for (int s = 0; s < nslice; ++s) {
            const int wbuf = s & 1;
            const int sn = s + 1 < nslice ? s + 1 : s;
#pragma unroll
            for (int ty = 0; ty < 3; ++ty) {
                const int tt = 3 * s + ty, bbuf = tt & 1;
                // staging of the next slice's window (buffer wbuf ^ 1: last read before the previous
                // slice's last barrier): unit ty loaded here, stored after this k-tile's MFMAs (ROLE 0)
                // or at the top of the next k-tile (ROLE 1)
                if constexpr (ROLE == 1) {
                    if (ty >= 1) win_store_u(ty - 1, wbuf ^ 1);
                }
                if (ty < WIN_UNITS) win_load_u(ty, sn);
                // B tile tt + 1 into the other buffer (last read before the previous barrier); past the
                // end a repeat nobody reads
                b_dma(tt + 1 < last ? tt + 1 : last, bbuf ^ 1);
                __builtin_amdgcn_sched_barrier(0);  // the loads stay at the top of the k-tile
                // A fragments of window pixels wbe + ty * WP + 0 .. 3: block i at tap tx takes fragment tx + i
                f16x8 fh[4], fl[4];
#pragma unroll
                for (int f = 0; f < 4; ++f) {
                    const int wpix = wbe + ty * WP + f;
                    fh[f] = *reinterpret_cast<const f16x8*>(Wn + win_off(wbuf, 0, wpix, kh));
                    if constexpr (NP == 3) fl[f] = *reinterpret_cast<const f16x8*>(Wn + win_off(wbuf, 1, wpix, kh));
                }
                // B fragments one tap ahead: tap tx + 1's are read before tap tx's MFMAs
                f16x8 pbh[2][2], pbl[2][2];
                auto rd_b = [&](int tx, int slot) {
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const int row = wn * 64 + j * 32 + l32;
                        pbh[slot][j] = *reinterpret_cast<const f16x8*>(Bs + wb_off(bbuf, 0, tx, row, kh));
                        if constexpr (NP == 3) pbl[slot][j] = *reinterpret_cast<const f16x8*>(Bs + wb_off(bbuf, 1, tx, row, kh));
                    }
                };
                rd_b(0, 0);
#pragma unroll
                for (int tx = 0; tx < 3; ++tx) {
                    if (tx < 2) rd_b(tx + 1, (tx + 1) & 1);
                    __builtin_amdgcn_sched_barrier(0);  // the reads stay ahead of this tap's MFMAs
#pragma unroll
                    for (int i = 0; i < 2; ++i)
#pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            const f16x8 bh = pbh[tx & 1][j];
                            if constexpr (NP == 3) {
                                t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fl[tx + i], bh, t[i][j], 0, 0, 0);
                                t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fh[tx + i], pbl[tx & 1][j], t[i][j], 0, 0, 0);
                            }
                            t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fh[tx + i], bh, t[i][j], 0, 0, 0);
                        }
                }
                if constexpr (ROLE == 0) {
                    // (below the MFMAs: hoisted into them, the split would wait for the unit's load there)
                    __builtin_amdgcn_sched_barrier(0);
                    if (ty < WIN_UNITS) win_store_u(ty, wbuf ^ 1);
                }
                __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0): this wave's DMAs (and window loads) landed
                __syncthreads();
            }
            // close the slice's accumulation chain (144 k)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    acc[i][j] += t[i][j];
#pragma unroll
                    for (int r = 0; r < 16; ++r) t[i][j][r] = 0.f;
                }
        }
    };
    if (wid >= 4) kloop(std::integral_constant<int, 1>{});  // (wave-uniform branch)
    else kloop(std::integral_constant<int, 0>{});
#if WIN_TIMING
    tm2 = wall_clock64();
#endif
    }

    // epilogue: undo the operand scales, + addend, NHWC store, IN statistics
    const int eab = -(ea + eb);
    const int p0 = y0 * W;  // the tile's first pixel within the image
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = __builtin_ldexpf(acc[i][j][r], eab);
    const long long obase = (long long)n * a.H * W * a.Co;
    auto ooff = [&](int i, int j, int r) {
        const int pix = p0 + win_pix(wm, i, r, kh);
        return obase + (long long)pix * a.Co + n0 + wn * 64 + j * 32 + l32;
    };

    if (addend) {  // wave-uniform: all 64 addend loads issued before the first use
        floatx16 ad[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) ad[i][j][r] = addend[ooff(i, j, r)];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) out[ooff(i, j, r)] = acc[i][j][r] + ad[i][j][r];
    } else {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) out[ooff(i, j, r)] = acc[i][j][r];
    }
    if (parts) win_stats(acc, p0, n0, a.Co, wm, wn, lane, tid, reinterpret_cast<float*>(smem), parts,
                         (long long)n * a.tiles + tile);
    if constexpr (IBW) {  // (y loaded here, after the stores: issuing them earlier spills ~70 VGPRs)
        float yv[2][2][16];
        win_ibw_load(yv, ib, obase, p0, a.Co, n0, wm, wn, lane);
        win_ibw(acc, yv, ib, n, p0, a.H, W, a.Co, n0, wm, wn, lane, tid, tile, reinterpret_cast<float*>(smem));
    }
#if WIN_TIMING
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (tid == 0 && L < 16384) {
        unsigned long long* g = g_win_t + 5 * L;
        g[0] = tm0; g[1] = tm1; g[2] = tm2; g[3] = wall_clock64(); g[4] = __smid();
    }
#endif
}

// ---------------------------------------------------------------------------------------
// The f16x3 window conv on v_mfma_f32_16x16x32_f16 (conv3_win16_kernel: same tile, operands, window
// and B staging as conv3_win_h3_kernel above).  Both MFMA shapes do the same MACs per fragment byte,
// but under the package power limit the 16x16x32 form sustains ~12 % more FLOP/s: 1758 against 1562
// TFLOP/s of f16x3 products in a bare LDS-read + MFMA loop with every CU busy on random operands
// (scripts/probes/mfma_shape_power.hip, profiles/r06b/; MI355X_MICROARCH.md, DVFS item 7).
//
// K = 32 per MFMA = two (slice, tap) units of 16 channels: the fragments' k groups 0, 1 (lanes 0-31)
// take unit 2j, k groups 2, 3 (lanes 32-63) unit 2j + 1 -- the packed B's k = 16 unit + channel, so a
// k-step is 32 consecutive packed k.  A slice has nine taps: the k-steps walk the 18 units of a PAIR
// of slices, 9 k-steps, k-step 4 taking tap 8 of the even slice and tap 0 of the odd one.  The even
// slice of a pair sits in window buffer 0, the odd one in buffer 1; the next odd slice is staged
// during k-steps 0-3 (buffer 1 is free after the previous pair's k-step 8), the next even slice
// during k-steps 5-8 (buffer 0 is free after k-step 4), one unit in flight per thread as above.
// One barrier per k-step: B (128 output-channel rows x 32 k x 2 planes, 16 KB) by LDS-DMA into the
// other of two buffers.  Per k-step and wave: 4 x 4 blocks of 16 x 16 x 3 products = 48 MFMAs.
// Row block i of wave wm holds the 16 consecutive tile pixels wm * 64 + 16 i + (lane & 15) (W >= 16:
// a block never crosses an image row), so the window needs no swizzle: the 16 lanes of a
// ds_read_b128 lane group read 16 distinct 16-byte bank groups (pixel stride 32 B, the two channel
// halves on odd / even groups).  A B row (output channel co) holds its four 8-k groups rotated by
// 2 * ((co >> 2) & 3), which makes the B reads conflict-free too.  Two-level accumulation: chains of
// 5 and 4 k-steps (160 / 128 k), added to the running sum.
constexpr int W16_BSLOT = 128 * 32;  // halves per B plane and k-step

__device__ __forceinline__ int w16_off(int buf, int pl, int wpix, int h) {
    return ((buf * 2 + pl) * WIN_PIX + wpix) * 16 + 8 * h;
}

// IN statistics of the tile from the 16x16 accumulator layout (lane: column lane & 15 of each block,
// rows 4 (lane >> 4) + r): per column over the lane's 16 pixels, merged with lanes ^ 16 and ^ 32, then
// over the four pixel waves in a fixed order (as win_stats)
__device__ __forceinline__ void win16_stats(const f32x4v (&acc)[4][4], int p0, int n0, int Co, int wm, int wn,
                                            int lane, int tid, float* lds, Part* __restrict__ parts, long long chunk) {
    Part* sp = reinterpret_cast<Part*>(lds);  // [4][128]
    const int g = lane >> 4, m16 = lane & 15;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        float s = 0.f, mx = -INFINITY;
        int am = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)  // increasing pixel order (first maximum)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float v = acc[i][j][r];
                s += v;
                if (v > mx) { mx = v; am = p0 + wm * 64 + 16 * i + 4 * g + r; }
            }
        float mean = s * (1.f / 16.f), m2 = 0.f, cnt = 16.f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float dv = acc[i][j][r] - mean;
                m2 = fmaf(dv, dv, m2);
            }
#pragma unroll
        for (int o = 16; o <= 32; o <<= 1) {  // equal counts on both sides
            const float mb = __shfl_xor(mean, o, 64), m2b = __shfl_xor(m2, o, 64), mxb = __shfl_xor(mx, o, 64);
            const int amb = __shfl_xor(am, o, 64);
            const float dl = mb - mean;
            m2 = m2 + m2b + dl * dl * (0.5f * cnt);
            mean = mean + 0.5f * dl;
            cnt *= 2.f;
            if (mxb > mx || (mxb == mx && amb < am)) { mx = mxb; am = amb; }
        }
        if (g == 0) {
            Part p;
            p.cnt = cnt;
            p.mean = mean;
            p.m2 = m2;
            p.mx = mx;
            p.amax = am;
            p.pad[0] = p.pad[1] = p.pad[2] = 0;
            sp[wm * WIN_BN + wn * 64 + j * 16 + m16] = p;
        }
    }
    __syncthreads();
    if (tid < WIN_BN && n0 + tid < Co) {
        Part a = sp[tid];
#pragma unroll
        for (int w = 1; w < 4; ++w) {
            const Part b = sp[w * WIN_BN + tid];
            const float tot = a.cnt + b.cnt, dl = b.mean - a.mean;
            a.mean += dl * (b.cnt / tot);
            a.m2 += b.m2 + dl * dl * (a.cnt * b.cnt / tot);
            a.cnt = tot;
            if (b.mx > a.mx || (b.mx == a.mx && b.amax < a.amax)) { a.mx = b.mx; a.amax = b.amax; }
        }
        parts[chunk * Co + n0 + tid] = a;
    }
}

// win_ibw for the 16x16 accumulator layout
__device__ __forceinline__ void win16_ibw(const f32x4v (&acc)[4][4], const float (&yv)[4][4][4], const IbwArgs& ib,
                                          int n, int p0, int H, int W, int Co, int n0, int wm, int wn, int lane,
                                          int tid, int tile, float* lds) {
    const int g = lane >> 4, m16 = lane & 15;
    Sum2* sp = reinterpret_cast<Sum2*>(lds);  // [4][128]; the k-loop's last barrier freed the LDS
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int col = n0 + wn * 64 + j * 16 + m16;
        const float s = ib.sc[(long long)n * Co + col], b = ib.sh[(long long)n * Co + col];
        float sa = 0.f, sb = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int pix = p0 + wm * 64 + 16 * i + 4 * g + r;
                const int py = pix >> __builtin_ctz(W), px = pix & (W - 1);  // (W is a power of two)
                if (py == 1 || py == H - 2 || px == 1 || px == W - 2) continue;  // the ring fold's pixels
                const float xh = fmaf(yv[i][j][r], s, b);
                const float gg = acc[i][j][r] * act_grad(xh, ib.act);
                sa += gg;
                sb = fmaf(gg, xh, sb);
            }
        sa += __shfl_xor(sa, 16, 64);  // the same operand pair on both lanes: order-free
        sb += __shfl_xor(sb, 16, 64);
        sa += __shfl_xor(sa, 32, 64);
        sb += __shfl_xor(sb, 32, 64);
        if (g == 0) sp[wm * 128 + wn * 64 + j * 16 + m16] = Sum2{sa, sb};
    }
    __syncthreads();
    if (tid < 128 && n0 + tid < Co) {
        Sum2 t = sp[tid];
#pragma unroll
        for (int w = 1; w < 4; ++w) {
            t.a += sp[w * 128 + tid].a;
            t.b += sp[w * 128 + tid].b;
        }
        ib.parts[((long long)n * ib.nchunk + tile) * Co + n0 + tid] = t;
    }
}

template <int NP, bool IBW, bool WIDE>  // NP: products (3: f16x3, 1: f16, hi planes only); WIDE: W >= 64
__global__ __launch_bounds__(WIN_NT, 1) void conv3_win16_kernel(WinArgs a, const float* __restrict__ src,
                                                                const _Float16* __restrict__ wh,
                                                                const _Float16* __restrict__ wl,
                                                                const float* __restrict__ rng,
                                                                const int* __restrict__ wexp,
                                                                const float* __restrict__ addend,
                                                                float* __restrict__ out, Part* __restrict__ parts,
                                                                IbwArgs ib) {
    // B buffers: the k-step in use's fragments are in registers; the next one's are read during it, so its
    // DMA must have landed by the barrier before.  DCS_WIN_ASYNC: four buffers, the DMA three k-steps ahead,
    // so each DMA has two k-steps to land; otherwise three, the DMA two ahead, and vmcnt(0) per k-step
    constexpr int NBUF = DCS_WIN_ASYNC ? 4 : 3;
    // G3 (NP 1, DCS_WIN16_G3): three k-steps per barrier, nine single-plane B buffers (one per k-step of a pair)
    constexpr bool G3 = NP == 1 && DCS_WIN16_G3;
    constexpr int BSLOTS = G3 ? 9 : NBUF * 2;
    __shared__ __attribute__((aligned(16))) _Float16 smem[2 * 2 * WIN_PIX * 16 + BSLOTS * W16_BSLOT + 8];
    _Float16* const Wn = smem;                        // [2 buffers][2 planes][WIN_PIX][16]
    _Float16* const Bs = smem + 2 * 2 * WIN_PIX * 16;  // [3 buffers][2 planes][128 rows][32 k]
    _Float16* const Wspare = Bs + BSLOTS * W16_BSLOT;  // 16 bytes nobody reads

    const int T = gridDim.x;
    const int L = xcd_remap(blockIdx.x, T);
    const int ntile = L % a.gy, mt = L / a.gy;
    const int n = mt / a.tiles, tile = mt - n * a.tiles;
    const int n0 = ntile * WIN_BN;
    const int y0 = tile * a.R;
    const int W = a.W, WP = a.W + 2, C = a.C;
    const int K = 9 * C;
    const int npair = C / 32;
    const int lw = __builtin_ctz(W);

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int m16 = lane & 15, g = lane >> 4;

    int ea = 0;
    float asc = 1.f;
    const int eb = __builtin_amdgcn_readfirstlane(wexp[0]);

    // window staging units (as conv3_win_h3_kernel)
    const int nint = (a.R + 2) * W;
    int uoff[WIN_UNITS], uwd[WIN_UNITS];
#pragma unroll
    for (int q = 0; q < WIN_UNITS; ++q) {
        const int u = tid + q * WIN_NT;
        const int ip = u >> 1, h = u & 1;
        uoff[q] = -1;
        uwd[q] = 0;
        if (ip < nint) {
            const int wr = ip >> lw, sx = ip & (W - 1);
            int dup = -1;
            int sy = y0 - 1 + wr;
            bool ok = true;
            if (a.reflect) {
                sy = sy < 0 ? -sy : (sy >= a.H ? 2 * a.H - 2 - sy : sy);
                if (sx == 1) dup = wr * WP;
                else if (sx == W - 2) dup = wr * WP + W + 1;
            } else {
                ok = sy >= 0 && sy < a.H;
            }
            uwd[q] = (wr * WP + sx + 2) | ((dup + 1) << 16);
            if (ok) uoff[q] = (((n * a.H + sy) * W + sx) * C + 8 * h) * 4;
        }
    }
    if (!a.reflect) {  // zero halo columns of both buffers and planes
        for (int i = tid; i < 2 * 2 * (a.R + 2) * 2 * 2; i += WIN_NT) {
            const int h = i & 1, side = (i >> 1) & 1, rest = i >> 2;
            const int wr = rest % (a.R + 2), bp = rest / (a.R + 2);
            *reinterpret_cast<f16x8*>(Wn + w16_off(bp >> 1, bp & 1, wr * WP + side * (W + 1), h)) = f16x8{};
        }
    }
    const __amdgpu_buffer_rsrc_t srsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, 0x7fffff00, 0x00020000);
    f32x4v wq_[2];  // (ext vectors: tied operands of the wait below)
    // DCS_WIN_ASYNC: the unit loads as inline asm, untracked by the compiler like the B DMA, so no wait of
    // the compiler's drains the k-step's own DMA (its waits for these registers counted only the tracked
    // loads: vmcnt(0) at every store); the waits are explicit (win_wait_u, the end of each k-step)
    auto win_load_into = [&](int q, int s, f32x4v (&dst)[2]) {
        const int off = uoff[q] >= 0 ? uoff[q] + s * 64 : 0x7fffffbf;
        if constexpr (DCS_WIN_ASYNC) {
            asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(dst[0]) : "v"(off), "s"(srsrc) : "memory");
            asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:16" : "=v"(dst[1]) : "v"(off), "s"(srsrc) : "memory");
        } else {
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(srsrc, off, 0, 0);
            u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(srsrc, off + 16, 0, 0);
            __builtin_memcpy(&dst[0], &v0, 16);
            __builtin_memcpy(&dst[1], &v1, 16);
        }
    };
    auto win_load_u = [&](int q, int s) { win_load_into(q, s, wq_); };
    // before a unit's store: its two loads landed, the k-step's two DMA pieces issued after them may not
    auto win_wait_u = [&]() {
        // (asm: the compiler drops waits it sees no need for; the registers as operands so no use of them
        // is scheduled above the wait)
        if constexpr (DCS_WIN_ASYNC) asm volatile("s_waitcnt vmcnt(2)" : "+v"(wq_[0]), "+v"(wq_[1]) : : "memory");
    };
    auto win_store_u = [&](int q, int buf) {
        const int h = (tid + q * WIN_NT) & 1;
        const int wp = (uwd[q] & 0xffff) - 1, wd = (uwd[q] >> 16) - 1;
        f16x8 hi, lo;
        split8h(make_float4(wq_[0][0], wq_[0][1], wq_[0][2], wq_[0][3]),
                make_float4(wq_[1][0], wq_[1][1], wq_[1][2], wq_[1][3]), asc, hi, lo);
        *reinterpret_cast<f16x8*>(wp >= 0 ? Wn + w16_off(buf, 0, wp, h) : Wspare) = hi;
        if constexpr (NP == 3) *reinterpret_cast<f16x8*>(wp >= 0 ? Wn + w16_off(buf, 1, wp, h) : Wspare) = lo;
        if (wd >= 0) {
            *reinterpret_cast<f16x8*>(Wn + w16_off(buf, 0, wd, h)) = hi;
            if constexpr (NP == 3) *reinterpret_cast<f16x8*>(Wn + w16_off(buf, 1, wd, h)) = lo;
        }
    };

    // B k-step by LDS-DMA: 16 blocks of 1 KB (plane, 16-row block), blocks 2w and 2w + 1 of wave w.  Lane
    // L of a block lands at row L / 4, 16-byte slot L % 4, which holds the row's k group
    // (L % 4 - 2 ((row >> 2) & 3)) & 3 (the rotation above; (row >> 2) & 3 = (L >> 4) & 3)
    unsigned dsu[2], ddst[2];
    const _Float16* dbase[2];
    const unsigned dlane = 2u * (unsigned)((n0 + (lane >> 2)) * K + 8 * (((lane & 3) - 2 * ((lane >> 4) & 3)) & 3));
    {
        const unsigned bs_lds = (unsigned)(uintptr_t)(__attribute__((address_space(3))) _Float16*)Bs;
#pragma unroll
        for (int i = 0; i < 2; ++i) {  // (NP 1: the hi plane's 8 blocks, block w of wave w)
            const int b = NP == 3 ? __builtin_amdgcn_readfirstlane(wid) * 2 + i : __builtin_amdgcn_readfirstlane(wid);
            const int pl = b >> 3, rb = b & 7;
            dsu[i] = 2u * (unsigned)(rb * 16 * K);
            dbase[i] = pl ? wl : wh;
            ddst[i] = __builtin_amdgcn_readfirstlane(bs_lds + 2u * (unsigned)(pl * W16_BSLOT + rb * 16 * 32));
        }
    }
    auto b_dma = [&](int j, int buf) {  // k-step j (packed k 32 j .. 32 j + 31) into B buffer buf
        const unsigned kb = 2u * (unsigned)(j * 32);
#pragma unroll
        for (int i = 0; i < (NP == 3 ? 2 : 1); ++i)
            win_glds(dbase[i], dlane + (dsu[i] + kb), ddst[i] + 2u * (unsigned)(buf * 2 * W16_BSLOT));
    };

    // fragment offsets (halves).  A: window pixel of row block i at tap (0, 0) = ublk[i] + m16 (wave-
    // uniform block part); k group g reads channel half g & 1 of the unit of its lane half.  B: row
    // wn * 64 + 16 j + m16, k group g in slot (g + 2 ((m16 >> 2) & 3)) & 3.
    // (W >= 64: the wave's four blocks are consecutive pixels of one row, block offsets 256 i halves
    // fold into the reads' immediate offsets; narrower images add a uniform offset per block)
    int ublk[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int q = wm * 64 + 16 * i;
        ublk[i] = __builtin_amdgcn_readfirstlane(((q >> lw) * WP + (q & (W - 1))) * 16);
    }
    const int alane = ublk[0] + m16 * 16 + 8 * (g & 1);
    const int blane = (wn * 64 + m16) * 32 + 8 * ((g + 2 * ((m16 >> 2) & 3)) & 3);
    const bool hiu = g >= 2;  // this lane's k groups take the k-step's second unit

    f32x4v acc[4][4], t[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) { acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f}; t[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f}; }

    if constexpr (G3) {
    // NP 1 (f16 operands, hi planes only): one product per fragment pair leaves 16 MFMAs per wave and k-step,
    // so the k-steps of a pair run in three groups of three between barriers (48 MFMAs per wave per barrier,
    // as one f16x3 k-step).  B: one single-plane buffer per k-step of a pair (buffer = js), the DMA for group
    // g + 2 issued at the top of group g.  Window: the lo-plane slots are free, so slices rotate through four
    // single-plane slots (slice s in slot s & 3): the next pair's even slice is loaded in group 0 and stored at
    // the top of group 1 (published before group 2 reads its first fragments for the next pair), the odd one
    // loaded in group 1 and stored at the top of group 2 (published before the next pair's group 1).
    const unsigned bsl = (unsigned)(uintptr_t)(__attribute__((address_space(3))) _Float16*)Bs;
    const unsigned ddst1 = __builtin_amdgcn_readfirstlane(bsl + 2u * (unsigned)(wid * 16 * 32));
    auto dma1 = [&](int j, int buf) {  // k-step j (packed k 32 j ..) into single-plane buffer buf
        win_glds(dbase[0], dlane + (dsu[0] + 2u * (unsigned)(j * 32)), ddst1 + 2u * (unsigned)(buf * W16_BSLOT));
    };
    auto dma_group = [&](int p_, int g_) {  // group g_ of pair p_
#pragma unroll
        for (int k = 0; k < 3; ++k) dma1(9 * p_ + 3 * g_ + k, 3 * g_ + k);
    };
    f32x4v wq1[2];
    auto store_slot = [&](int q, int slot, const f32x4v (&v)[2]) {
        const int h = (tid + q * WIN_NT) & 1;
        const int wp = (uwd[q] & 0xffff) - 1, wd = (uwd[q] >> 16) - 1;
        f16x8 hi, lo;
        split8h(make_float4(v[0][0], v[0][1], v[0][2], v[0][3]), make_float4(v[1][0], v[1][1], v[1][2], v[1][3]),
                asc, hi, lo);
        *reinterpret_cast<f16x8*>(wp >= 0 ? Wn + (slot * WIN_PIX + wp) * 16 + 8 * h : Wspare) = hi;
        if (wd >= 0) *reinterpret_cast<f16x8*>(Wn + (slot * WIN_PIX + wd) * 16 + 8 * h) = hi;
    };
    auto load_slice = [&](int sl) {  // both units of slice sl: unit 0 into wq_, unit 1 into wq1
        win_load_into(0, sl, wq_);
        win_load_into(1, sl, wq1);
    };
    auto store_slice = [&](int sl) {
        store_slot(0, sl & 3, wq_);
        store_slot(1, sl & 3, wq1);
    };
    // prologue: B groups 0 and 1 of pair 0, slices 0 and 1, the exponent
    dma_group(0, 0);
    dma_group(0, 1);
    load_slice(0);
    ea = f16x3_exp(rng, a.rng_n);
    asc = __builtin_ldexpf(1.f, ea);
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(wq_[0]), "+v"(wq_[1]), "+v"(wq1[0]), "+v"(wq1[1]) : : "memory");
    store_slice(0);
    load_slice(1);
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(wq_[0]), "+v"(wq_[1]), "+v"(wq1[0]), "+v"(wq1[1]) : : "memory");
    store_slice(1);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();

    f16x8 bh[4], ah[2];
    auto a_base1 = [&](int js_, int podd) {  // A base of k-step js_ (units 2 js_, 2 js_ + 1) of a pair
        const int u0 = 2 * js_, u1 = 2 * js_ + 1;
        const int t0 = u0 % 9, t1 = u1 % 9;
        const int o0 = (2 * podd + u0 / 9) * WIN_PIX * 16 + ((t0 / 3) * WP + t0 % 3) * 16;
        const int o1 = (2 * podd + u1 / 9) * WIN_PIX * 16 + ((t1 / 3) * WP + t1 % 3) * 16;
        int al_ = alane;
        asm volatile("" : "+v"(al_));
        return Wn + al_ + (hiu ? o1 : o0);
    };
    auto b_base1 = [&](int buf) {
        int bl_ = blane;
        asm volatile("" : "+v"(bl_));
        return Bs + buf * W16_BSLOT + bl_;
    };
    auto rd_a1 = [&](const _Float16* Ak, int i, int slot) {
        const int bo = WIDE ? 256 * i : ublk[i] - ublk[0];
        ah[slot] = *reinterpret_cast<const f16x8*>(Ak + bo);
    };
    {  // k-step 0's fragments
        rd_a1(a_base1(0, 0), 0, 0);
        const _Float16* const B0 = b_base1(0);
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) bh[jb] = *reinterpret_cast<const f16x8*>(B0 + jb * 16 * 32);
    }
    for (int p = 0; p < npair; ++p) {
        const int podd = p & 1;
        const bool more = p + 1 < npair;  // (block-uniform)
#pragma unroll
        for (int g_ = 0; g_ < 3; ++g_) {
            // group top: the staging of the next pair's slices, and the B DMA two groups ahead
            if (g_ == 0) {
                dma_group(p, 2);
                if (more) load_slice(2 * p + 2);
            } else if (g_ == 1) {
                if (more) {
                    store_slice(2 * p + 2);
                    dma_group(p + 1, 0);
                    load_slice(2 * p + 3);
                }
            } else {
                if (more) {
                    store_slice(2 * p + 3);
                    dma_group(p + 1, 1);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int kk = 0; kk < 3; ++kk) {
                const int js = 3 * g_ + kk;
                const _Float16* const Ak = a_base1(js, podd);
                const _Float16* const An = js < 8 ? a_base1(js + 1, podd) : a_base1(0, podd ^ 1);
                const _Float16* const Bn = b_base1(js < 8 ? js + 1 : 0);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    if (i < 3) rd_a1(Ak, i + 1, (i + 1) & 1);
                    else rd_a1(An, 0, 0);
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int jb = 0; jb < 4; ++jb) {
                        t[i][jb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i & 1], bh[jb], t[i][jb], 0, 0, 0);
                        if (i == 3) bh[jb] = *reinterpret_cast<const f16x8*>(Bn + jb * 16 * 32);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (js == 4 || js == 8) {  // close the accumulation chain (160 / 128 k)
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj) {
                            acc[i][jj] += t[i][jj];
                            asm volatile("" : "+v"(acc[i][jj]));
                            t[i][jj] = f32x4v{0.f, 0.f, 0.f, 0.f};
                        }
                }
            }
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // the group's DMAs and stores landed
            __syncthreads();
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    } else {
    // prologue: window of slice 0 (buffer 0) and B k-steps 0 and 1, every load (and the exponent's) in
    // flight before the first store
    b_dma(0, 0);
    b_dma(1, 1);
    if constexpr (NBUF == 4) b_dma(2, 2);
    f32x4v wp1[2];
    win_load_into(1, 0, wp1);
    win_load_u(0, 0);
    ea = f16x3_exp(rng, a.rng_n);
    asc = __builtin_ldexpf(1.f, ea);
    // vmcnt(0): the units (asm loads in DCS_WIN_ASYNC, so the wait is asm too, tied to their registers)
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(wq_[0]), "+v"(wq_[1]), "+v"(wp1[0]), "+v"(wp1[1]) : : "memory");
    win_store_u(0, 0);
    wq_[0] = wp1[0];
    wq_[1] = wp1[1];
    win_store_u(1, 0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // the DMAs have landed (asm: kept)
    __syncthreads();

    const int nstep = 9 * npair;
    // fragments carried across k-steps: the k-step's B (four column blocks) and the A row block in use
    // plus the next one.  Row block i's MFMAs run with block i + 1's A (or, at i = 3, the next k-step's
    // block 0) in flight, and during i = 3 each column block's B is replaced by the next k-step's right
    // after its last MFMA: the reads a k-step needs are issued during the previous one, so no wave
    // starts a k-step with its LDS reads queued behind eight waves' bursts.  That needs B k-step j + 1
    // readable during k-step j: three B buffers (k-step j in buffer j % 3 = js % 3, the DMA for j + 2
    // issued at the top of j), and each window slice published one k-step before its first fragment
    // read (see the staging windows below).
    f16x8 bh[4], bl[4], ah[2], al[2];
    auto a_base = [&](int js_) {  // this lane's A base of k-step js_ of a pair (units 2 js_, 2 js_ + 1)
        const int u0 = 2 * js_, u1 = 2 * js_ + 1;
        const int t0 = u0 % 9, t1 = u1 % 9;
        const int o0 = (u0 / 9) * 2 * WIN_PIX * 16 + ((t0 / 3) * WP + t0 % 3) * 16;
        const int o1 = (u1 / 9) * 2 * WIN_PIX * 16 + ((t1 / 3) * WP + t1 % 3) * 16;
        // (through an empty asm: hoisted out of the loop, the nine k-steps' bases stayed live and spilled)
        int al_ = alane;
        asm volatile("" : "+v"(al_));
        return Wn + al_ + (hiu ? o1 : o0);
    };
    auto b_base = [&](int buf) {
        int bl_ = blane;
        asm volatile("" : "+v"(bl_));
        return Bs + buf * 2 * W16_BSLOT + bl_;
    };
    auto rd_a = [&](const _Float16* Ak, int i, int slot) {
        const int bo = WIDE ? 256 * i : ublk[i] - ublk[0];
        if constexpr (NP == 3) al[slot] = *reinterpret_cast<const f16x8*>(Ak + bo + WIN_PIX * 16);
        ah[slot] = *reinterpret_cast<const f16x8*>(Ak + bo);
    };
    auto rd_b = [&](const _Float16* Bk, int jb) {
        bh[jb] = *reinterpret_cast<const f16x8*>(Bk + jb * 16 * 32);
        if constexpr (NP == 3) bl[jb] = *reinterpret_cast<const f16x8*>(Bk + jb * 16 * 32 + W16_BSLOT);
    };
    {  // k-step 0's fragments (published by the prologue's barrier)
        rd_a(a_base(0), 0, 0);
        const _Float16* const B0 = b_base(0);
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) rd_b(B0, jb);
    }
    auto kloop = [&](auto role_tag) {
        constexpr int ROLE = decltype(role_tag)::value;
        for (int p = 0; p < npair; ++p) {
            // staging windows (one unit in flight per thread): the odd slice 2p + 1 into window buffer 1 in
            // k-steps 0-2 (buffer 1's previous slice had its last fragment read in the previous pair's
            // k-step 8; its first read is k-step 4's block 0, issued in k-step 3), the next even slice into
            // buffer 0 in k-steps 5-7 (last read of slice 2p in k-step 4; first read of slice 2p + 2 in
            // k-step 8 for the next pair's k-step 0)
            const int s_odd = 2 * p + 1;
            const int s_even = 2 * p + 2 < 2 * npair ? 2 * p + 2 : 2 * p;  // past the end a repeat nobody reads
#pragma unroll
            for (int js = 0; js < 9; ++js) {
                const int j = 9 * p + js;
                const int ph = js < 3 ? js : (js >= 5 && js < 8 ? js - 5 : -1);  // position in a staging window
                const int sbuf = js < 3 ? 1 : 0, ssl = js < 3 ? s_odd : s_even;
                if constexpr (ROLE == 1) {  // unit ph - 1 stored at the top of the next k-step
                    if (ph == 1 || ph == 2) {
                        win_wait_u();
                        win_store_u(ph - 1, sbuf);
                    }
                }
                if (ph == 0 || ph == 1) win_load_u(ph, ssl);
                b_dma(j + NBUF - 1 < nstep ? j + NBUF - 1 : nstep - 1, (j + NBUF - 1) % NBUF);
                __builtin_amdgcn_sched_barrier(0);  // the loads stay at the top of the k-step
                const _Float16* const Ak = a_base(js);
                const _Float16* const An = a_base((js + 1) % 9);
                const _Float16* const Bn = b_base((j + 1) % NBUF);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    if (i < 3) rd_a(Ak, i + 1, (i + 1) & 1);
                    else rd_a(An, 0, 0);
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int jb = 0; jb < 4; ++jb) {
                        const int sl = i & 1;
                        if constexpr (NP == 3) {
                            t[i][jb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[sl], bh[jb], t[i][jb], 0, 0, 0);
                            t[i][jb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[sl], bl[jb], t[i][jb], 0, 0, 0);
                        }
                        t[i][jb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[sl], bh[jb], t[i][jb], 0, 0, 0);
                        if (i == 3) rd_b(Bn, jb);  // the next k-step's column block jb
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
                if constexpr (ROLE == 0) {
                    if (ph == 0 || ph == 1) {
                        win_wait_u();
                        win_store_u(ph, sbuf);
                    }
                }
                if (js == 4 || js == 8) {  // close the accumulation chain (160 / 128 k)
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj) {
                            acc[i][jj] += t[i][jj];
                            // (pinned here: sunk to the next closure, the sum kept both chains live and spilled)
                            asm volatile("" : "+v"(acc[i][jj]));
                            t[i][jj] = f32x4v{0.f, 0.f, 0.f, 0.f};
                        }
                }
                if constexpr (DCS_WIN_ASYNC) {
                    // the DMA issued one k-step ago (B k-step j + 2, read from the next k-step on) has landed
                    // once only this k-step's loads (the unit's two, if any, and the DMA's two) are in flight
                    if (ph == 0 || ph == 1) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
                    else asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
                    __builtin_amdgcn_sched_barrier(0);
                } else {
                    __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0): this wave's DMAs (and window loads) landed
                }
                __syncthreads();
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    };
    if (wid >= 4) kloop(std::integral_constant<int, 1>{});  // (wave-uniform branch)
    else kloop(std::integral_constant<int, 0>{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last (repeat) DMAs landed before the epilogue
    }

    // epilogue: undo the operand scales, + addend, NHWC store, IN statistics
    const int eab = -(ea + eb);
    const int p0 = y0 * W;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[i][j][r] = __builtin_ldexpf(acc[i][j][r], eab);
    const long long obase = (long long)n * a.H * W * a.Co;
    auto ooff = [&](int i, int j, int r) {
        const int pix = p0 + wm * 64 + 16 * i + 4 * g + r;
        return obase + (long long)pix * a.Co + n0 + wn * 64 + j * 16 + m16;
    };
    if (addend) {  // wave-uniform: all 64 addend loads issued before the first use
        float ad[4][4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) ad[i][j][r] = addend[ooff(i, j, r)];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) out[ooff(i, j, r)] = acc[i][j][r] + ad[i][j][r];
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) out[ooff(i, j, r)] = acc[i][j][r];
    }
    if (parts) win16_stats(acc, p0, n0, a.Co, wm, wn, lane, tid, reinterpret_cast<float*>(smem), parts,
                           (long long)n * a.tiles + tile);
    if constexpr (IBW) {
        float yv[4][4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) yv[i][j][r] = ib.y[ooff(i, j, r)];
        win16_ibw(acc, yv, ib, n, p0, a.H, W, a.Co, n0, wm, wn, lane, tid, tile, reinterpret_cast<float*>(smem));
    }
}

// pre-split weight pack (dcs_pack_weights_h3): the range of the raw weights first, then every block
// derives the same exponent and writes hi / lo fp16 planes of the slice-major B
__global__ __launch_bounds__(256) void wrange_kernel(const float* __restrict__ w, long long n, float* __restrict__ parts) {
    float m = 0.f;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
        m = fmaxf(m, fabsf(w[i]));
    __shared__ float red[4];
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) parts[blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (blockIdx.x == 0)  // a grid smaller than the record: the remaining partial maxima are zero
        for (int i = gridDim.x + threadIdx.x; i < DCS_RANGE_PARTS; i += blockDim.x) parts[i] = 0.f;
}

__global__ __launch_bounds__(256) void pack_h3_kernel(const float* __restrict__ w, int Cout, int Cin, int flip,
                                                      int ncols, const float* __restrict__ parts, int nparts,
                                                      _Float16* __restrict__ oh, _Float16* __restrict__ ol,
                                                      int* __restrict__ wexp) {
    const int e = f16x3_exp(parts, nparts);  // every wave derives the same exponent
    const float sc = __builtin_ldexpf(1.f, e);
    if (blockIdx.x == 0 && threadIdx.x == 0) wexp[0] = e;
    const int C = flip ? Cout : Cin;  // reduction channels per tap
    const int K = 9 * C;
    const long long total = (long long)ncols * K;
    for (long long idx = (long long)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
        const int col = (int)(idx / K), k = (int)(idx - (long long)col * K);
        const int slice = k / 144, rem = k - slice * 144;
        const int tap = rem >> 4, c = slice * 16 + (rem & 15);
        int ty = tap / 3, tx = tap - 3 * (tap / 3);
        float v = 0.f;
        if (!flip) {  // forward: B[k][co] = W[co][c][ty][tx]
            if (col < Cout) v = w[(((long long)col * Cin + c) * 3 + ty) * 3 + tx];
        } else {      // data gradient: B[k][ci] = W[c][ci][2-ty][2-tx] (c = output channel of the forward)
            if (col < Cin) v = w[(((long long)c * Cin + col) * 3 + (2 - ty)) * 3 + (2 - tx)];
        }
        const float f = v * sc;
        const _Float16 h = (_Float16)f, l = (_Float16)(f - (float)h);
        oh[idx] = h;
        ol[idx] = l;
        if (flip) {  // the tap-major copy behind the planes (k = tap * C + c: the ring kernel's B)
            const long long t = total + (long long)col * K + tap * C + c;
            oh[t] = h;
            ol[t] = l;
        }
    }
}

// ---------------------------------------------------------------------------------------
// Weight gradient of the residual 3x3 convs on a rolling source window (f16x3):
//   dW[co][ci][ty][tx] = sum_p dy[p][co] * xpad[p + (ty - 1, tx - 1)][ci]
// conv.hip's conv_wgrad_x6_kernel owns a 128 (co) x 128 ((tap, ci)) tile and gathers the source at
// each tap's offset: every source value is fetched, split and staged once per tap column group
// (nine times).  Here a workgroup owns 64 co x 64 ci x all nine taps and walks one 64-pixel-wide
// strip of an image row by row: per row it stages the dy row segment (64 px x 64 co) and ONE new
// source row segment (66 px with the halo x 64 ci) into a ring of four rows, split into hi / lo fp16
// once; the nine taps read their fragments from the ring at a per-tap (row slot, pixel) offset.
// MFMA shape: M = co (32), N = ci (32), K = 16 pixels of the row; both operands pixel-major in LDS,
// fragments by ds_read_b64_tr_b16 (8 consecutive pixels of one channel per lane).  8 waves, two per
// SIMD: waves w and w + 4 (same SIMD) own co block (w & 1) x ci block ((w >> 1) & 1), wave w taps
// 0..3 and wave w + 4 taps 5..8, tap 4 split between them by pixel sub-tile (ww_k / ww_tap), so each
// SIMD carries all nine taps of one 32 x 32 (co, ci) block, 18 MFMA groups per wave, and each wave
// five accumulators (two-level: a chain of two rows = 128 pixels, then added to
// the running sum), leaving registers for fragment reads ahead and a second wave to cover LDS
// latency.  Per row and SIMD: 4 pixel sub-tiles x 9 taps x 3 products = 108 MFMAs between barriers.
// LDS (halves): ring [4 slots][2 planes][66 px][64 ch], dy [2 buffers][2 planes][64 px][64 ch];
// 16-byte channel units swizzled by bit 1 of the pixel index (unit ^ 4), so the four consecutive
// pixels of a transposed read land on the four 64-byte quarters of the banks at any tap offset.
// Partial sums per (image, strip, row chunk) go to slabs [split][co][tap * C + ci] (the layout of
// conv.hip's split-K weight gradient), summed by its reduce kernel.
constexpr int WW_NT = 512, WW_SW = 64, WW_WP = WW_SW + 2;
constexpr int WW_XROW = 2 * WW_WP * 64;  // halves per ring slot
constexpr int WW_DROW = 2 * WW_SW * 64;  // halves per dy buffer
constexpr int WW_XU = (WW_WP * 8 + WW_NT - 1) / WW_NT;  // source-row (pixel, 8-channel unit)s per thread: 2
constexpr int WW_TPW = 5;                                // taps per wave (5 + 4)

struct WWArgs {
    int N, H, W, C, Co;  // source NHWC [N][H][W][C]; dy NHWC [N][H][W][Co]
    int reflect;         // 1: reflection padding, 0: zero padding
    int strips, rchunks, rows_per;  // 64-pixel strips per row, row chunks per strip, rows per chunk
    int gco, gci;        // 64-channel tiles of co / ci
    int rng_a_n, rng_b_n;
};

__device__ __forceinline__ int ww_swz(int pix) { return ((pix >> 1) & 1) << 2; }

typedef short wshortx4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) wshortx4 lds_wshortx4;

__device__ __forceinline__ f16x8 ww_frag(const _Float16* p) {
    const wshortx4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_wshortx4*)(p));
    const wshortx4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_wshortx4*)(p + 4 * 64));
    return __builtin_bit_cast(f16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

// (sub-tile k, tap) of a wave's j-th MFMA group in a row: the 36 pairs of a SIMD split 18 / 18
// between its two waves, tap 4 shared (role 0: taps 0..4 on sub-tiles 0, 1 and taps 0..3 on 2, 3;
// role 1: taps 5..8 on sub-tiles 0, 1 and taps 4..8 on 2, 3), so neither wave runs alone at the
// row's end; the two partial sums of tap 4 meet in the epilogue
__host__ __device__ constexpr int ww_k(int r, int j) { return r == 0 ? (j < 10 ? j / 5 : 2 + (j - 10) / 4) : (j < 8 ? j / 4 : 2 + (j - 8) / 5); }
__host__ __device__ constexpr int ww_tap(int r, int j) { return r == 0 ? (j < 10 ? j % 5 : (j - 10) % 4) : (j < 8 ? 5 + j % 4 : 4 + (j - 8) % 5); }
__host__ __device__ constexpr int ww_acc(int r, int tap) { return r == 0 ? tap : (tap == 4 ? 4 : tap - 5); }

template <int NP>  // as conv3_win_h3_kernel
__global__ __launch_bounds__(WW_NT, 1) void wgrad3_win_h3_kernel(WWArgs a, const float* __restrict__ dy,
                                                                 const float* __restrict__ src,
                                                                 const float* __restrict__ rnga,
                                                                 const float* __restrict__ rngb,
                                                                 float* __restrict__ ws) {
    // f16x3: a ring of 4 source rows [2 planes][66][64] and 2 dy buffers [2][64][64], one image row per
    // barrier.  f16 (NP 1, hi planes only): one product per fragment pair leaves 36 MFMAs per SIMD
    // and row, so two rows run per barrier: a ring of 8 source rows and 4 dy buffers.
    constexpr int RPB = NP == 3 ? 1 : 2;             // image rows per barrier
    constexpr int NXS = NP == 3 ? 4 : 8;             // source-row ring slots
    constexpr int NDB = NP == 3 ? 2 : 4;             // dy buffers
    constexpr int XROW = NP == 3 ? WW_XROW : WW_WP * 64;
    constexpr int DROW = NP == 3 ? WW_DROW : WW_SW * 64;
    __shared__ __attribute__((aligned(16))) _Float16 smem[NXS * XROW + NDB * DROW];
    _Float16* const Xr = smem;                 // [NXS][planes][66][64]
    _Float16* const Dy = smem + NXS * XROW;    // [NDB][planes][64][64]

#if CLK_PROBE
    const unsigned long long ck0 = clock64(), wc0 = wall_clock64();
#endif
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int ntile = a.gco * a.gci;
    const int tile = L % ntile, split = L / ntile;
    const int co0 = (tile % a.gco) * 64, ci0 = (tile / a.gco) * 64;
    const int rc = split % a.rchunks, rest = split / a.rchunks;
    const int strip = rest % a.strips, n = rest / a.strips;
    const int x0 = strip * WW_SW;
    const int H = a.H, W = a.W, C = a.C, Co = a.Co;
    const int y_beg = rc * a.rows_per;
    const int y_end = y_beg + a.rows_per < H ? y_beg + a.rows_per : H;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int cob = wid & 1, cib = (wid >> 1) & 1, half = wid >> 2;

    // the operand exponents are read in the prologue, beside the first rows' loads
    int ea = 0, eb = 0;
    float asc = 1.f, bsc = 1.f;

    const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dy), (short)0, 0x7fffff00, 0x00020000);
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, 0x7fffff00, 0x00020000);
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    constexpr int OOB = 0x7fffffbf;

    // dy row segment: 64 px x 8 units, one per thread; byte offset within the row
    int doff, dls;
    {
        const int pix = tid >> 3, cu = tid & 7;
        doff = ((x0 + pix) * Co + co0 + 8 * cu) * 4;
        dls = pix * 64 + 8 * (cu ^ ww_swz(pix));
    }
    // source row segment: 66 px (halo included) x 8 units; byte offset within the row (-1: none)
    int xoff[WW_XU], xls[WW_XU];
#pragma unroll
    for (int q = 0; q < WW_XU; ++q) {
        const int u = tid + q * WW_NT, wc = u >> 3, cu = u & 7;
        xoff[q] = -1;
        xls[q] = -1;
        if (wc < WW_WP) {
            int sx = x0 - 1 + wc;
            bool ok = true;
            if (a.reflect) sx = sx < 0 ? -sx : (sx >= W ? 2 * W - 2 - sx : sx);
            else ok = sx >= 0 && sx < W;
            if (ok) xoff[q] = (sx * C + ci0 + 8 * cu) * 4;
            xls[q] = wc * 64 + 8 * (cu ^ ww_swz(wc));
        }
    }
    // register sets of the rows in flight (DCS_WW_F16_EARLY, f16: both rows of the next barrier)
    constexpr bool EARLY = NP == 1 && DCS_WW_F16_EARLY;
    constexpr int NSET = EARLY ? 2 : 1;
    float4 dr_[NSET][2], xr_[NSET][WW_XU][2];
    float4 (&dr)[2] = dr_[0];
    float4 (&xr)[WW_XU][2] = xr_[0];
    auto ld_dy = [&](int y, int set = 0) {
        const int rb = ((n * H + y) * W) * Co * 4;
        u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(drs, rb + doff, 0, 0);
        u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(drs, rb + doff + 16, 0, 0);
        __builtin_memcpy(&dr_[set][0], &v0, 16);
        __builtin_memcpy(&dr_[set][1], &v1, 16);
    };
    auto ld_x = [&](int r, int set = 0) {  // logical source row r in [-1, H]
        int sy = r;
        bool ok = true;
        if (a.reflect) sy = sy < 0 ? -sy : (sy >= H ? 2 * H - 2 - sy : sy);
        else ok = sy >= 0 && sy < H;
        const int rb = ((n * H + sy) * W) * C * 4;
#pragma unroll
        for (int q = 0; q < WW_XU; ++q) {
            const int off = (ok && xoff[q] >= 0) ? rb + xoff[q] : OOB;
            u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0);
            u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(xrs, off + 16, 0, 0);
            __builtin_memcpy(&xr_[set][q][0], &v0, 16);
            __builtin_memcpy(&xr_[set][q][1], &v1, 16);
        }
    };
    auto st_dy = [&](int buf, int set = 0) {
        f16x8 hi, lo;
        split8h(dr_[set][0], dr_[set][1], asc, hi, lo);
        *reinterpret_cast<f16x8*>(Dy + buf * DROW + dls) = hi;
        if constexpr (NP == 3) *reinterpret_cast<f16x8*>(Dy + buf * DROW + WW_SW * 64 + dls) = lo;
    };
    auto st_x = [&](int slot, int set = 0) {
#pragma unroll
        for (int q = 0; q < WW_XU; ++q) {
            if (xls[q] >= 0) {
                f16x8 hi, lo;
                split8h(xr_[set][q][0], xr_[set][q][1], bsc, hi, lo);
                *reinterpret_cast<f16x8*>(Xr + slot * XROW + xls[q]) = hi;
                if constexpr (NP == 3) *reinterpret_cast<f16x8*>(Xr + slot * XROW + WW_WP * 64 + xls[q]) = lo;
            }
        }
    };

    // transposed-read lane offsets (halves): lane (r, h) of a fragment gets pixels 8h .. 8h+7 of
    // channel r of its 32-channel block; in a 16-lane group lane 4q+p reads pixel row q (+4: second
    // read), channels 4p .. 4p+3
    const int g16 = lane >> 4;
    const int rpix = 8 * (g16 >> 1) + ((lane & 15) >> 2);
    const int rcol = 16 * (g16 & 1) + 4 * (lane & 3);
    int aoff, boff[3];
    {
        const int c = 32 * cob + rcol;
        aoff = rpix * 64 + 8 * ((c >> 3) ^ ww_swz(rpix)) + (c & 7);
        const int cb = 32 * cib + rcol;
#pragma unroll
        for (int tx = 0; tx < 3; ++tx) {
            const int p = rpix + tx;
            boff[tx] = p * 64 + 8 * ((cb >> 3) ^ ww_swz(p)) + (cb & 7);
        }
    }

    floatx16 acc[WW_TPW], t[WW_TPW];
#pragma unroll
    for (int i = 0; i < WW_TPW; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) { acc[i][r] = 0.f; t[i][r] = 0.f; }

    // prologue: source rows y_beg - 1 .. y_beg + RPB into their ring slots, dy rows y_beg .. y_beg + RPB - 1;
    // every row's loads (and the exponents') in flight before the first store
    {
        float4 px_[RPB + 2][WW_XU][2], pd_[RPB][2];
#pragma unroll
        for (int i = 0; i < RPB + 2; ++i) {
            const int r = y_beg - 1 + i;
            ld_x(r <= H ? r : H);
#pragma unroll
            for (int q = 0; q < WW_XU; ++q) { px_[i][q][0] = xr[q][0]; px_[i][q][1] = xr[q][1]; }
        }
#pragma unroll
        for (int i = 0; i < RPB; ++i) {
            const int r = y_beg + i;
            ld_dy(r < y_end ? r : y_end - 1);
            pd_[i][0] = dr[0];
            pd_[i][1] = dr[1];
        }
        ea = f16x3_exp(rnga, a.rng_a_n);
        eb = f16x3_exp(rngb, a.rng_b_n);
        asc = __builtin_ldexpf(1.f, ea);
        bsc = __builtin_ldexpf(1.f, eb);
#pragma unroll
        for (int i = 0; i < RPB + 2; ++i) {
#pragma unroll
            for (int q = 0; q < WW_XU; ++q) { xr[q][0] = px_[i][q][0]; xr[q][1] = px_[i][q][1]; }
            st_x((y_beg - 1 + i) & (NXS - 1));
        }
#pragma unroll
        for (int i = 0; i < RPB; ++i) {
            dr[0] = pd_[i][0];
            dr[1] = pd_[i][1];
            st_dy((y_beg + i) & (NDB - 1));
        }
    }
    __syncthreads();

    // one row of this wave's taps T0 .. T0 + NT_ - 1: 4 pixel sub-tiles x NT_ taps, the fragments of
    // the next (sub-tile, tap) read before the MFMAs of the current one
    // (S: EARLY, the barrier's second row, which stages both rows loaded at the barrier, y0 = its first row)
    auto row = [&](int y, auto tag, auto stag) {
        constexpr int R = decltype(tag)::value;
        constexpr bool S = decltype(stag)::value;
        constexpr int NJ = 18;  // (sub-tile, tap) pairs of this wave
        const _Float16* const Db = Dy + (y & (NDB - 1)) * DROW;
        const _Float16* Xs[3];
#pragma unroll
        for (int ty = 0; ty < 3; ++ty) Xs[ty] = Xr + ((y + NXS - 1 + ty) & (NXS - 1)) * XROW;  // row y - 1 + ty
        auto rdA = [&](int k, f16x8& h, f16x8& l) {
            h = ww_frag(Db + aoff + k * 16 * 64);
            if constexpr (NP == 3) l = ww_frag(Db + WW_SW * 64 + aoff + k * 16 * 64);
        };
        auto rdB = [&](int j, f16x8& h, f16x8& l) {
            const int k = ww_k(R, j), tap = ww_tap(R, j), ty = tap / 3, tx = tap % 3;
            h = ww_frag(Xs[ty] + boff[tx] + k * 16 * 64);
            if constexpr (NP == 3) l = ww_frag(Xs[ty] + WW_WP * 64 + boff[tx] + k * 16 * 64);
        };
        f16x8 ah, al, bh, bl, nah, nal, nbh, nbl;
        rdA(0, ah, al);
        rdB(0, bh, bl);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            if (j + 1 < NJ) {
                if (ww_k(R, j + 1) != ww_k(R, j)) rdA(ww_k(R, j + 1), nah, nal);
                rdB(j + 1, nbh, nbl);
            }
            floatx16& tt = EARLY ? acc[ww_acc(R, ww_tap(R, j))] : t[ww_acc(R, ww_tap(R, j))];
            if constexpr (NP == 3) {
                tt = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, tt, 0, 0, 0);
                tt = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, tt, 0, 0, 0);
            }
            tt = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, tt, 0, 0, 0);
            // stage the rows loaded above into the buffers no row of this barrier reads: mid-row (f16x3),
            // or at the row's end (f16: a row holds a third of the MFMAs, half a row hid too little of
            // the loads' latency)
            if (!EARLY && j == (NP == 1 ? NJ - 1 : NJ / 2 - 1)) {
                st_dy((y + RPB) & (NDB - 1));
                st_x((y + RPB + 1) & (NXS - 1));
            }
            if (S && (j == NJ / 2 - 1 || j == NJ - 1)) {  // set 0 mid-row, set 1 at the end (y - 1: the first row)
                const int set = j == NJ - 1 ? 1 : 0;
                st_dy((y + 1 + set) & (NDB - 1), set);
                st_x((y + 2 + set) & (NXS - 1), set);
            }
            bh = nbh;
            bl = nbl;
            if (j + 1 < NJ && ww_k(R, j + 1) != ww_k(R, j)) {
                ah = nah;
                al = nal;
            }
        }
    };

    if constexpr (RPB == 1) {
#pragma unroll 1
        for (int y = y_beg; y < y_end; ++y) {
            // next rows in flight (unconditional: clamped past the chunk, reflected / zero past the image)
            ld_dy(y + 1 < y_end ? y + 1 : y);
            ld_x(y + 2 <= H ? y + 2 : H);
            if (half == 0) row(y, std::integral_constant<int, 0>{}, std::false_type{});
            else row(y, std::integral_constant<int, 1>{}, std::false_type{});
            if (((y - y_beg) & 1) == 1 || y + 1 == y_end) {
#pragma unroll
                for (int i = 0; i < WW_TPW; ++i) {
                    acc[i] += t[i];
#pragma unroll
                    for (int r = 0; r < 16; ++r) t[i][r] = 0.f;
                }
            }
            __syncthreads();
        }
    } else if constexpr (EARLY) {
        // both rows of the next barrier in flight from its start, staged by the second row (one accumulation
        // level: the fp16 operands' rounding dwarfs the fp32 sum's)
#pragma unroll 1
        for (int y = y_beg; y < y_end; y += 2) {
            ld_dy(y + 2 < y_end ? y + 2 : y_end - 1, 0);
            ld_dy(y + 3 < y_end ? y + 3 : y_end - 1, 1);
            ld_x(y + 3 <= H ? y + 3 : H, 0);
            ld_x(y + 4 <= H ? y + 4 : H, 1);
            if (half == 0) row(y, std::integral_constant<int, 0>{}, std::false_type{});
            else row(y, std::integral_constant<int, 1>{}, std::false_type{});
            if (y + 1 < y_end) {  // (block-uniform; otherwise no later barrier reads the staged rows)
                if (half == 0) row(y + 1, std::integral_constant<int, 0>{}, std::true_type{});
                else row(y + 1, std::integral_constant<int, 1>{}, std::true_type{});
            }
            __syncthreads();
        }
    } else {
#pragma unroll 1
        for (int y = y_beg; y < y_end; y += 2) {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int yr = y + q;
                if (yr < y_end) {  // (block-uniform)
                    // next rows in flight, staged mid-row into the buffers no row of this barrier reads
                    ld_dy(yr + 2 < y_end ? yr + 2 : y_end - 1);
                    ld_x(yr + 3 <= H ? yr + 3 : H);
                    if (half == 0) row(yr, std::integral_constant<int, 0>{}, std::false_type{});
                    else row(yr, std::integral_constant<int, 1>{}, std::false_type{});
                }
            }
#pragma unroll
            for (int i = 0; i < WW_TPW; ++i) {  // chains of two rows
                acc[i] += t[i];
#pragma unroll
                for (int r = 0; r < 16; ++r) t[i][r] = 0.f;
            }
            __syncthreads();
        }
    }

    // epilogue: the two halves of tap 4 summed through LDS (free after the loop's last barrier), then
    // undo the operand scales, slab [split][co][tap * C + ci]
    float* const t4 = reinterpret_cast<float*>(smem) + (wid & 3) * 64 * 16 + lane;
    if (half == 1) {
#pragma unroll
        for (int r = 0; r < 16; ++r) t4[r * 64] = acc[4][r];
    }
    __syncthreads();
    if (half == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[4][r] += t4[r * 64];
    }
    const int eab = -(ea + eb);
    float* const slab = ws + (long long)split * Co * 9 * C;
    const int col = ci0 + 32 * cib + (lane & 31);
#pragma unroll
    for (int i = 0; i < WW_TPW; ++i) {
        const int tap = half == 0 ? i : (i == 4 ? 9 : 5 + i);
        if (tap < 9) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = co0 + 32 * cob + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                slab[(long long)row * 9 * C + tap * C + col] = __builtin_ldexpf(acc[i][r], eab);
            }
        }
    }
#if CLK_PROBE
    if (threadIdx.x == 0 && blockIdx.x < 4096) {
        unsigned long long* g = g_clk + 4 * blockIdx.x;
        g[0] = ck0; g[1] = wc0; g[2] = clock64(); g[3] = wall_clock64();
    }
#endif
}

// ---------------------------------------------------------------------------------------
// The residual weight gradient on v_mfma_f32_16x16x32_f16 (f16x3; same workgroup, rolling window,
// staging and slabs as wgrad3_win_h3_kernel above, the MFMA shape the window conv moved to for the
// power-limited clock, conv3_win16_kernel).  M = 16 output channels, N = 16 input channels, K = 32
// pixels of the row: two k-steps per 64-pixel row.  A SIMD's waves w and w + 4 still share one
// 32 x 32 (co, ci) block = 2 x 2 sub-blocks of 16 x 16; wave w takes taps 0-3 on all four
// sub-blocks and tap 4 on the co sub-block 0, wave w + 4 taps 5-8 and tap 4 on co sub-block 1: 18
// accumulators each, no shared accumulator to merge.  Fragments by ds_read_b64_tr_b16 (lane group
// g = lane >> 4 takes pixels 8 g .. 8 g + 7 of the k-step, lane 4 q + p of the group addresses pixel
// row q (+ 4 for the second read), channels 4 p .. 4 p + 3).  The 16-byte channel units of a pixel
// row are XOR-swizzled by bits 1 and 3 of the pixel (ww16_swz), which spreads the eight pixel rows
// of a 32-lane read group (rows r .. r + 3 and r + 8 .. r + 11) over all 64 banks at any tap offset;
// the unit index's bit 1 is the 16-channel sub-block, so the second sub-block's fragment is the first
// one's offset XOR 16 halves.
// f16 (NP 1, hi planes only): a row is a third of the MFMAs, so two rows run per barrier (as
// wgrad3_win_h3_kernel<1>): a ring of 8 source rows and 4 dy buffers, the next two rows' loads issued at
// the barrier and staged in six pieces through the second row, so they have a row and a half to land.
__device__ __forceinline__ int ww16_swz(int pix) { return (((pix >> 1) & 1) << 2) | (((pix >> 3) & 1) << 1); }

__device__ __forceinline__ f16x8 ww16_frag(const _Float16* p1, const _Float16* p2) {
    const wshortx4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_wshortx4*)(p1));
    const wshortx4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_wshortx4*)(p2));
    return __builtin_bit_cast(f16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int NP>
__global__ __launch_bounds__(WW_NT, 1) void wgrad3_win16_kernel(WWArgs a, const float* __restrict__ dy,
                                                                const float* __restrict__ src,
                                                                const float* __restrict__ rnga,
                                                                const float* __restrict__ rngb,
                                                                float* __restrict__ ws) {
    constexpr int RPB = NP == 3 ? 1 : 2;  // image rows per barrier
    constexpr int NXS = NP == 3 ? 4 : 8;  // source-row ring slots
    constexpr int NDB = NP == 3 ? 2 : 4;  // dy buffers
    constexpr int XROW = NP == 3 ? WW_XROW : WW_WP * 64;
    constexpr int DROW = NP == 3 ? WW_DROW : WW_SW * 64;
    __shared__ __attribute__((aligned(16))) _Float16 smem[NXS * XROW + NDB * DROW];
    _Float16* const Xr = smem;                 // [NXS slots][planes][66][64]
    _Float16* const Dy = smem + NXS * XROW;    // [NDB buffers][planes][64][64]

    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int ntile = a.gco * a.gci;
    const int tile = L % ntile, split = L / ntile;
    const int co0 = (tile % a.gco) * 64, ci0 = (tile / a.gco) * 64;
    const int rc = split % a.rchunks, rest = split / a.rchunks;
    const int strip = rest % a.strips, n = rest / a.strips;
    const int x0 = strip * WW_SW;
    const int H = a.H, W = a.W, C = a.C, Co = a.Co;
    const int y_beg = rc * a.rows_per;
    const int y_end = y_beg + a.rows_per < H ? y_beg + a.rows_per : H;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int cob = wid & 1, cib = (wid >> 1) & 1, half = wid >> 2;

    int ea = 0, eb = 0;
    float asc = 1.f, bsc = 1.f;

    const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dy), (short)0, 0x7fffff00, 0x00020000);
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, 0x7fffff00, 0x00020000);
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    constexpr int OOB = 0x7fffffbf;

    int doff, dls;
    {
        const int pix = tid >> 3, cu = tid & 7;
        doff = ((x0 + pix) * Co + co0 + 8 * cu) * 4;
        dls = pix * 64 + 8 * (cu ^ ww16_swz(pix));
    }
    int xoff[WW_XU], xls[WW_XU];
#pragma unroll
    for (int q = 0; q < WW_XU; ++q) {
        const int u = tid + q * WW_NT, wc = u >> 3, cu = u & 7;
        xoff[q] = -1;
        xls[q] = -1;
        if (wc < WW_WP) {
            int sx = x0 - 1 + wc;
            bool ok = true;
            if (a.reflect) sx = sx < 0 ? -sx : (sx >= W ? 2 * W - 2 - sx : sx);
            else ok = sx >= 0 && sx < W;
            if (ok) xoff[q] = (sx * C + ci0 + 8 * cu) * 4;
            xls[q] = wc * 64 + 8 * (cu ^ ww16_swz(wc));
        }
    }
    // register sets i of the rows in flight (RPB of each)
    float4 dr[RPB][2], xr[RPB][WW_XU][2];
    auto ld_dy = [&](int y, int i) {
        const int rb = ((n * H + y) * W) * Co * 4;
        u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(drs, rb + doff, 0, 0);
        u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(drs, rb + doff + 16, 0, 0);
        __builtin_memcpy(&dr[i][0], &v0, 16);
        __builtin_memcpy(&dr[i][1], &v1, 16);
    };
    auto ld_x = [&](int r, int i) {  // logical source row r in [-1, H]
        int sy = r;
        bool ok = true;
        if (a.reflect) sy = sy < 0 ? -sy : (sy >= H ? 2 * H - 2 - sy : sy);
        else ok = sy >= 0 && sy < H;
        const int rb = ((n * H + sy) * W) * C * 4;
#pragma unroll
        for (int q = 0; q < WW_XU; ++q) {
            const int off = (ok && xoff[q] >= 0) ? rb + xoff[q] : OOB;
            u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0);
            u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(xrs, off + 16, 0, 0);
            __builtin_memcpy(&xr[i][q][0], &v0, 16);
            __builtin_memcpy(&xr[i][q][1], &v1, 16);
        }
    };
    auto st_dy = [&](int buf, int i) {
        f16x8 hi, lo;
        split8h(dr[i][0], dr[i][1], asc, hi, lo);
        *reinterpret_cast<f16x8*>(Dy + buf * DROW + dls) = hi;
        if constexpr (NP == 3) *reinterpret_cast<f16x8*>(Dy + buf * DROW + WW_SW * 64 + dls) = lo;
    };
    auto st_xq = [&](int slot, int q, int i) {
        if (q == 0 || xls[q] >= 0) {  // (unit 0 covers pixels 0..63 of the 66: always inside)
            f16x8 hi, lo;
            split8h(xr[i][q][0], xr[i][q][1], bsc, hi, lo);
            *reinterpret_cast<f16x8*>(Xr + slot * XROW + xls[q]) = hi;
            if constexpr (NP == 3) *reinterpret_cast<f16x8*>(Xr + slot * XROW + WW_WP * 64 + xls[q]) = lo;
        }
    };
    auto st_x = [&](int slot, int i) {
#pragma unroll
        for (int q = 0; q < WW_XU; ++q) st_xq(slot, q, i);
    };
    // staging piece p of the rows loaded for the next barrier, y = this barrier's first row (f16x3, p 0..2:
    // the dy row, source units 0 / 1; f16, p 0..5: dy rows y + 2, y + 3, then source rows y + 3, y + 4 by unit)
    auto st_piece = [&](int p, int y) {
        if constexpr (NP == 3) {
            if (p == 0) st_dy((y + 1) & 1, 0);
            else st_xq((y + 2) & 3, p - 1, 0);
        } else {
            if (p < 2) st_dy((y + 2 + p) & (NDB - 1), p);
            else st_xq((y + 3 + ((p - 2) >> 1)) & (NXS - 1), (p - 2) & 1, (p - 2) >> 1);
        }
    };

    // transposed-read lane offsets (halves) of k-step 0 and the first sub-block: A (dy) at pixel row
    // 8 g + q (+ 4: the second read, same swizzle), channel 32 cob + 4 p; B (source) at pixel row
    // 8 g + q + tx, whose second read can carry into bit 3 (its own offset)
    const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    int aoff, boff1[3], boff2[3];
    {
        const int r = 8 * g + q, c = 32 * cob + 4 * pp;
        aoff = r * 64 + 8 * ((c >> 3) ^ ww16_swz(r)) + (c & 7);
        const int cb = 32 * cib + 4 * pp;
#pragma unroll
        for (int tx = 0; tx < 3; ++tx) {
            const int p1 = r + tx, p2 = r + 4 + tx;
            boff1[tx] = p1 * 64 + 8 * ((cb >> 3) ^ ww16_swz(p1)) + (cb & 7);
            boff2[tx] = p2 * 64 + 8 * ((cb >> 3) ^ ww16_swz(p2)) + (cb & 7);
        }
    }

    f32x4v acc[18], t[18];
#pragma unroll
    for (int i = 0; i < 18; ++i) { acc[i] = f32x4v{0.f, 0.f, 0.f, 0.f}; t[i] = f32x4v{0.f, 0.f, 0.f, 0.f}; }

    // prologue: source rows y_beg - 1 .. y_beg + RPB into their ring slots, dy rows y_beg .. y_beg + RPB - 1;
    // every row's loads (and the exponents') in flight before the first store
    {
        float4 px_[RPB + 2][WW_XU][2], pd_[RPB][2];
#pragma unroll
        for (int i = 0; i < RPB + 2; ++i) {
            const int r = y_beg - 1 + i;
            ld_x(r <= H ? r : H, 0);
#pragma unroll
            for (int u = 0; u < WW_XU; ++u) { px_[i][u][0] = xr[0][u][0]; px_[i][u][1] = xr[0][u][1]; }
        }
#pragma unroll
        for (int i = 0; i < RPB; ++i) {
            const int r = y_beg + i;
            ld_dy(r < y_end ? r : y_end - 1, 0);
            pd_[i][0] = dr[0][0];
            pd_[i][1] = dr[0][1];
        }
        ea = f16x3_exp(rnga, a.rng_a_n);
        eb = f16x3_exp(rngb, a.rng_b_n);
        asc = __builtin_ldexpf(1.f, ea);
        bsc = __builtin_ldexpf(1.f, eb);
#pragma unroll
        for (int i = 0; i < RPB + 2; ++i) {
#pragma unroll
            for (int u = 0; u < WW_XU; ++u) { xr[0][u][0] = px_[i][u][0]; xr[0][u][1] = px_[i][u][1]; }
            st_x((y_beg - 1 + i) & (NXS - 1), 0);
        }
#pragma unroll
        for (int i = 0; i < RPB; ++i) {
            dr[0][0] = pd_[i][0];
            dr[0][1] = pd_[i][1];
            st_dy((y_beg + i) & (NDB - 1), 0);
        }
    }
    __syncthreads();

    // one row: two k-steps of 32 pixels; per k-step the A fragments of both co sub-blocks, then the
    // wave's five taps with the next tap's B fragments read ahead of the current one's MFMAs
    // (S: the second row of an f16 barrier, which stages the next barrier's rows)
    auto row = [&](int y, auto tag, auto stag) {
        constexpr int R = decltype(tag)::value;
        constexpr bool S = decltype(stag)::value;
        const _Float16* const Db = Dy + (y & (NDB - 1)) * DROW;
        const _Float16* Xs[3];
#pragma unroll
        for (int ty = 0; ty < 3; ++ty) Xs[ty] = Xr + ((y + NXS - 1 + ty) & (NXS - 1)) * XROW;  // row y - 1 + ty
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            f16x8 ah[2], al[2];
#pragma unroll
            for (int cs = 0; cs < 2; ++cs) {
                const int o = (aoff ^ (16 * cs)) + kk * 32 * 64;
                ah[cs] = ww16_frag(Db + o, Db + o + 4 * 64);
                if constexpr (NP == 3) al[cs] = ww16_frag(Db + WW_SW * 64 + o, Db + WW_SW * 64 + o + 4 * 64);
            }
            // (tap, ci sub-block) pairs of the wave: the next pair's B fragments read ahead of this one's MFMAs
            f16x8 bh[2], bl[2];
            auto rd_b = [&](int jp, int slot) {
                const int tt = jp >> 1, ns = jp & 1;
                const int tap = R == 0 ? tt : (tt < 4 ? 5 + tt : 4);
                const int ty = tap / 3, tx = tap % 3;
                const int o1 = (boff1[tx] ^ (16 * ns)) + kk * 32 * 64, o2 = (boff2[tx] ^ (16 * ns)) + kk * 32 * 64;
                bh[slot] = ww16_frag(Xs[ty] + o1, Xs[ty] + o2);
                if constexpr (NP == 3) bl[slot] = ww16_frag(Xs[ty] + WW_WP * 64 + o1, Xs[ty] + WW_WP * 64 + o2);
            };
            rd_b(0, 0);
#pragma unroll
            for (int jp = 0; jp < 10; ++jp) {
                if (jp < 9) rd_b(jp + 1, (jp + 1) & 1);
                __builtin_amdgcn_sched_barrier(0);
                // DCS_WW_STAGE 1 / 2 / 4: the three staging pieces inside the second k-step's pair iterations 1,
                // 3, 5 (their split VALU beside MFMAs instead of a block between the k-steps; 2: interleave
                // requested by sched_group_barrier; 4: the next row's loads issued right after the last piece,
                // in flight across the barrier); 3: iterations 3, 5, 7
                const int p0 = DCS_WW_STAGE == 3 ? 3 : 1;
                const bool piece_here = NP == 3 && DCS_WW_STAGE != 0 && (jp == p0 || jp == p0 + 2 || jp == p0 + 4);
                if (piece_here) {
                    if (kk == 1) st_piece((jp - p0) >> 1, y);
                }
                if (NP == 3 && DCS_WW_STAGE == 4 && kk == 1 && jp == 5 && y + 1 < y_end) {  // (block-uniform)
                    ld_dy(y + 2 < y_end ? y + 2 : y + 1, 0);
                    ld_x(y + 3 <= H ? y + 3 : H, 0);
                }
                // f16: pieces 0..2 in the first k-step's pair iterations 3, 5, 7, pieces 3..5 in the second's 1, 3, 5
                if (S && ((kk == 0 && (jp == 3 || jp == 5 || jp == 7)) || (kk == 1 && (jp == 1 || jp == 3 || jp == 5))))
                    st_piece(kk == 0 ? (jp - 3) >> 1 : 3 + ((jp - 1) >> 1), y - 1);
                const int tt = jp >> 1, ns = jp & 1;
                const int tap = R == 0 ? tt : (tt < 4 ? 5 + tt : 4);
                const int sl = jp & 1;
#pragma unroll
                for (int cs = 0; cs < 2; ++cs) {
                    if (tap == 4 && cs != R) continue;  // tap 4: co sub-block R only
                    const int idx = tap == 4 ? 16 + ns : (R == 0 ? tap : tap - 5) * 4 + cs * 2 + ns;
                    if constexpr (NP == 3) {
                        t[idx] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[cs], bh[sl], t[idx], 0, 0, 0);
                        t[idx] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[cs], bl[sl], t[idx], 0, 0, 0);
                        t[idx] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[cs], bh[sl], t[idx], 0, 0, 0);
                    } else {  // (one level: the fp16 operands' rounding dwarfs the fp32 sum's)
                        acc[idx] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[cs], bh[sl], acc[idx], 0, 0, 0);
                    }
                }
                if (piece_here && DCS_WW_STAGE == 2) {
                    if (kk == 1) {
#pragma unroll
                        for (int m = 0; m < 6; ++m) {
                            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
                            __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);  // then up to six VALU
                        }
                        __builtin_amdgcn_sched_group_barrier(0x200, 2, 0);      // the two LDS stores
                    }
                }
            }
            if (NP == 3 && DCS_WW_STAGE == 0 && kk == 0) {  // stage the rows loaded for the next barrier (buffers no row of this one reads)
                __builtin_amdgcn_sched_barrier(0);
                st_dy((y + 1) & 1, 0);
                st_x((y + 2) & 3, 0);
            }
        }
    };

    using F_ = std::false_type;
    using T_ = std::true_type;
    using R0_ = std::integral_constant<int, 0>;
    using R1_ = std::integral_constant<int, 1>;
    if constexpr (NP == 3) {
#pragma unroll 1
        for (int y = y_beg; y < y_end; ++y) {
            if (DCS_WW_STAGE != 4 || y == y_beg) {  // (DCS_WW_STAGE 4: issued by the previous row)
                ld_dy(y + 1 < y_end ? y + 1 : y, 0);
                ld_x(y + 2 <= H ? y + 2 : H, 0);
            }
            if (half == 0) row(y, R0_{}, F_{});
            else row(y, R1_{}, F_{});
            if (((y - y_beg) & 1) == 1 || y + 1 == y_end) {  // chains of two rows (128 pixels)
#pragma unroll
                for (int i = 0; i < 18; ++i) {
                    acc[i] += t[i];
                    asm volatile("" : "+v"(acc[i]));  // (pinned: see conv3_win16_kernel)
                    t[i] = f32x4v{0.f, 0.f, 0.f, 0.f};
                }
            }
            __syncthreads();
        }
    } else {
#pragma unroll 1
        for (int y = y_beg; y < y_end; y += 2) {
            // the next barrier's rows in flight (clamped past the chunk, reflected / zero past the image),
            // staged by the second row into buffers no row of this barrier reads
            ld_dy(y + 2 < y_end ? y + 2 : y_end - 1, 0);
            ld_dy(y + 3 < y_end ? y + 3 : y_end - 1, 1);
            ld_x(y + 3 <= H ? y + 3 : H, 0);
            ld_x(y + 4 <= H ? y + 4 : H, 1);
            if (half == 0) row(y, R0_{}, F_{});
            else row(y, R1_{}, F_{});
            if (y + 1 < y_end) {  // (block-uniform; otherwise no later barrier reads the staged rows)
                if (half == 0) row(y + 1, R0_{}, T_{});
                else row(y + 1, R1_{}, T_{});
            }
            __syncthreads();
        }
    }

    // epilogue: undo the operand scales, slab [split][co][tap * C + ci]; lane holds rows 4 g + r (co)
    // and column lane & 15 (ci) of each 16 x 16 sub-block
    const int eab = -(ea + eb);
    float* const slab = ws + (long long)split * Co * 9 * C;
#pragma unroll
    for (int i = 0; i < 18; ++i) {
        int tap, cs, ns;
        if (i >= 16) { tap = 4; cs = half; ns = i - 16; }
        else { tap = (half == 0 ? 0 : 5) + i / 4; cs = (i >> 1) & 1; ns = i & 1; }
        const int col = ci0 + 32 * cib + 16 * ns + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int rowc = co0 + 32 * cob + 16 * cs + 4 * g + r;
            slab[(long long)rowc * 9 * C + tap * C + col] = __builtin_ldexpf(acc[i][r], eab);
        }
    }
}

// ---------------------------------------------------------------------------------------
// The one-pixel ring of the residual data gradient's padded grid (dcs_conv_dgrad_reflect_win).  Over the
// (H + 2) x (W + 2) grid dx_pad[q] = sum_t B_t^T dy[q + (ty - 2, tx - 2)] (B: the window kernel's flipped
// pack, dcs_pack_weights_h3), and a ring position is reached by the three taps of one kernel row (top
// ring row: ty = 2, bottom: ty = 0) or column (left: tx = 2, right: tx = 0) only.  One GEMM per ring
// segment and tap, so B is uniform over a workgroup: M = the segment's positions over the batch (the
// top rows of all images, ...), N = the output channels, K = C; the three taps' products go to three ring
// copies (RG_COPIES), summed by the fold in tap order, so each position's sum has one fixed order
// whatever the batch.  A workgroup owns 64 positions x 256 channels: four waves of 64 x 64 (4 x 4 blocks
// of v_mfma_f32_16x16x32_f16).  A (the gathered dy pixels, fp32) arrives by LDS-DMA (the eight 16-byte
// chunks of a row rotated by bits 1-3 of the row: conflict-free fragment reads) and is split into hi / lo
// fp16 at the fragment read, where pixels outside the image are masked to zero (their DMA reads pixel 0).
// B fragments come straight from the pack's tap-major copy (L2) into registers.  RG_D = 2 of the 8 k-steps
// (C = 256) are in flight, in RG_D + 1 LDS buffers and register sets (140 VGPRs: three waves per SIMD).  The B loads are inline asm like the DMA, so the compiler inserts no wait of its
// own for them (it cannot count the DMAs, and its waits for the registers would drain later k-steps'
// loads); the one wait per k-step (vmcnt: all but the loads of the k-steps after the next) covers both.
// The tap split triples the workgroups (more waves per SIMD to overlap the fetch latency of these short
// K loops).  The generic rows pass this replaces ran the ring as 128-row tiles with K split
// over up to eight ring copies.
constexpr int RG_NT = 256, RG_BM = 64;
constexpr int RG_D = 2;  // k-steps in flight (RG_D + 1 register sets and LDS buffers; 4 measured slower: 202 VGPRs)

template <int... I, class F>
__device__ __forceinline__ void rg_unroll(std::integer_sequence<int, I...>, F&& f) {
    (f(std::integral_constant<int, I>{}), ...);
}

struct RingArgs {
    int N, H, W, C, Co;
    int tiles_tb, tiles_lr;  // 64-position tiles of the top / bottom segments and of the left / right ones
    int rng_n;
};

// 16 bytes per lane through the buffer descriptor, untracked by the compiler (see ring16_kernel)
__device__ __forceinline__ f16x8 rg_bload(__amdgpu_buffer_rsrc_t r, int off) {
    f16x8 v;
    asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(r) : "memory");
    return v;
}

template <int NP, int NK>  // NK: k-steps (C / 32)
__global__ __launch_bounds__(RG_NT) void ring16_kernel(RingArgs a, const float* __restrict__ dy,
                                                      const _Float16* __restrict__ wh,
                                                      const _Float16* __restrict__ wl,
                                                      const float* __restrict__ rng,
                                                      const int* __restrict__ wexp, float* __restrict__ ring) {
    __shared__ __attribute__((aligned(16))) float Ar[(RG_D + 1) * RG_BM * 32];  // [buffer][row][32 floats]
    const int gco = a.Co >> 8;
    const int L = blockIdx.x;
    const int ct = L % gco, jt = (L / gco) % 3, mt = L / (3 * gco);
    const int n0 = ct * 256;
    int seg, tm;
    if (mt < 2 * a.tiles_tb) {
        seg = mt >= a.tiles_tb;
        tm = mt - seg * a.tiles_tb;
    } else {
        const int r = mt - 2 * a.tiles_tb;
        seg = 2 + (r >= a.tiles_lr);
        tm = r - (seg - 2) * a.tiles_lr;
    }
    const int H = a.H, W = a.W, C = a.C, Wp = W + 2, K = 9 * C;
    const int seglen = seg < 2 ? Wp : H;  // positions per image
    const int segM = a.N * seglen, m0 = tm * RG_BM;
    const int ringlen = 2 * Wp + 2 * H;
    // the workgroup's tap (t0 + jt tstep); dy pixel of a position at tap jt: (py0 + jt sy, px0 + jt sx)
    const int t0 = seg == 0 ? 6 : (seg == 2 ? 2 : 0), tstep = seg < 2 ? 1 : 3;
    const int sy = seg < 2 ? 0 : jt, sx = seg < 2 ? jt : 0;
    auto locate = [&](int m, int& n, int& py, int& px, int& ri) {
        n = m / seglen;
        const int p = m - n * seglen;
        if (seg == 0) { py = 0; px = p - 2; ri = p; }
        else if (seg == 1) { py = H - 1; px = p - 2; ri = Wp + p; }
        else if (seg == 2) { py = p - 1; px = 0; ri = 2 * Wp + 2 * p; }  // padded row p + 1
        else { py = p - 1; px = W - 1; ri = 2 * Wp + 2 * p + 1; }
        py += sy;
        px += sx;
    };
    auto inimg = [&](int py, int px) { return py >= 0 && py < H && px >= 0 && px < W; };

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int m16 = lane & 15, g = lane >> 4;

    // A by LDS-DMA: wave w's instructions i = 0, 1 move chunks u = (2 w + i) * 64 + lane: row u >> 3,
    // LDS slot u & 7 holding channel chunk (u & 7) ^ ((row >> 1) & 7) of the k-step's 32 channels
    unsigned doff[2], dlds[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int u = (2 * wid + i) * 64 + lane, row = u >> 3, chunk = (u & 7) ^ ((row >> 1) & 7);
        int n = 0, py = 0, px = 0, ri = 0;
        if (m0 + row < segM) locate(m0 + row, n, py, px, ri);
        const bool ok = m0 + row < segM && inimg(py, px);
        doff[i] = (unsigned)((ok ? ((n * H + py) * W + px) * C * 4 : 0) + chunk * 16);
        dlds[i] = (unsigned)__builtin_amdgcn_readfirstlane((2 * wid + i) * 64 * 16);
    }
    const unsigned ar_lds = (unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)Ar;
    auto a_dma = [&](int ks, int buf) {
        const unsigned base = ar_lds + (unsigned)(buf * RG_BM * 32 * 4);
#pragma unroll
        for (int i = 0; i < 2; ++i) win_glds(dy, doff[i] + (unsigned)(ks * 128), base + dlds[i]);
    };
    // fragment rows 16 i + m16 inside the image at this tap (bit i)
    int vmask = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + 16 * i + m16;
        if (m < segM) {
            int n, py, px, ri;
            locate(m, n, py, px, ri);
            if (inimg(py, px)) vmask |= 1 << i;
        }
    }
    // B: lane (m16, g) of column block jb reads column n0 + 64 wid + 16 jb + m16, the k-step's channels
    // 8 g .. 8 g + 7 of the workgroup's tap, from the pack's tap-major copy (behind its Co x 9C planes:
    // the four lanes of a column read 64 contiguous bytes; the slice-major planes interleave the taps)
    const __amdgpu_buffer_rsrc_t bhr = __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16*>(wh), (short)0, 0x7fffff00, 0x00020000);
    const __amdgpu_buffer_rsrc_t blr = __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16*>(NP == 3 ? wl : wh), (short)0, 0x7fffff00, 0x00020000);
    const int blane = (a.Co * K + (n0 + 64 * wid + m16) * K + (t0 + jt * tstep) * C + 8 * g) * 2;
    f16x8 bq[RG_D + 1][4][2];
    auto b_load = [&](int ks, auto setc) {
        constexpr int S = decltype(setc)::value;
        const int kb = blane + ks * 32 * 2;
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) {
            bq[S][jb][0] = rg_bload(bhr, kb + jb * 16 * K * 2);
            if constexpr (NP == 3) bq[S][jb][1] = rg_bload(blr, kb + jb * 16 * K * 2);
        }
    };

    f32x4v acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) acc[i][jb] = f32x4v{0.f, 0.f, 0.f, 0.f};

    // vmcnt(n) with the other counters left alone
    auto wait_vm = [](auto nc) {
        constexpr int n = decltype(nc)::value;
        __builtin_amdgcn_s_waitcnt(0x0F70 | (n & 15) | ((n >> 4) << 14));
    };
    constexpr int PER = NP == 3 ? 10 : 6;  // loads per k-step and lane: 2 DMA + 4 or 8 B

    // prologue: the exponents first (their loads are the compiler's to wait for), then k-steps
    // 0 .. RG_D - 1 in flight, k-step 0 waited for
    const int ea = f16x3_exp(rng, a.rng_n);
    const int eb = __builtin_amdgcn_readfirstlane(wexp[0]);
    const float asc = __builtin_ldexpf(1.f, ea);
    __builtin_amdgcn_sched_barrier(0);
    rg_unroll(std::make_integer_sequence<int, (RG_D < NK ? RG_D : NK)>{}, [&](auto kc) {
        constexpr int k = decltype(kc)::value;
        a_dma(k, k);
        b_load(k, std::integral_constant<int, k>{});
    });
    wait_vm(std::integral_constant<int, ((RG_D < NK ? RG_D : NK) - 1) * PER>{});
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);

    // per lane: A rows 16 i + m16, floats 8 g .. 8 g + 7 = chunks 2 g, 2 g + 1
    int aoff[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = 16 * i + m16, f = (row >> 1) & 7;
        aoff[i][0] = row * 32 + 4 * ((2 * g) ^ f);
        aoff[i][1] = row * 32 + 4 * ((2 * g + 1) ^ f);
    }
    auto step = [&](auto ksc) {
        constexpr int ks = decltype(ksc)::value, S = ks % (RG_D + 1);
        // no load past the end (its dead destination registers the compiler would hand to other values)
        if constexpr (ks + RG_D < NK) {
            a_dma(ks + RG_D, (ks + RG_D) % (RG_D + 1));
            b_load(ks + RG_D, std::integral_constant<int, (ks + RG_D) % (RG_D + 1)>{});
        }
        __builtin_amdgcn_sched_barrier(0);
        const float* const Ab = Ar + S * RG_BM * 32;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float4 r0 = *reinterpret_cast<const float4*>(Ab + aoff[i][0]);
            const float4 r1 = *reinterpret_cast<const float4*>(Ab + aoff[i][1]);
            const float sc = (vmask >> i) & 1 ? asc : 0.f;  // pixels outside the image: zero
            f16x8 ah, al;
            split8h(r0, r1, sc, ah, al);
#pragma unroll
            for (int jb = 0; jb < 4; ++jb) {
                if constexpr (NP == 3) {
                    acc[i][jb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bq[S][jb][0], acc[i][jb], 0, 0, 0);
                    acc[i][jb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bq[S][jb][1], acc[i][jb], 0, 0, 0);
                }
                acc[i][jb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bq[S][jb][0], acc[i][jb], 0, 0, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        // k-step ks + 1 has landed once only the loads of the k-steps after it are in flight
        constexpr int last = ks + RG_D < NK - 1 ? ks + RG_D : NK - 1;
        wait_vm(std::integral_constant<int, (last > ks + 1 ? last - ks - 1 : 0) * PER>{});
        __syncthreads();
        __builtin_amdgcn_sched_barrier(0);
    };
    // fully unrolled (NK = C / 32 k-steps): the registers the asm loads fill must not meet a control-flow
    // merge, where the compiler could copy them before the data lands
    rg_unroll(std::make_integer_sequence<int, NK>{}, step);

    // epilogue: undo the scales into ring copy jt; lane (m16, g) holds rows 16 i + 4 g + r, column
    // 16 jb + m16
    const int eab = -(ea + eb);
    float* const rc = ring + (long long)jt * a.N * ringlen * a.Co;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + 16 * i + 4 * g + r;
            if (m >= segM) continue;
            int n, py, px, ri;
            locate(m, n, py, px, ri);
            float* const o = rc + ((long long)n * ringlen + ri) * a.Co + n0 + 64 * wid + m16;
#pragma unroll
            for (int jb = 0; jb < 4; ++jb) o[16 * jb] = __builtin_ldexpf(acc[i][jb][r], eab);
        }
}

struct WWPlan {
    int strips, rchunks, rows_per, nsplit;
};
WWPlan ww_plan(const dcs_conv_desc& d) {
    WWPlan p;
    p.strips = d.Ws / WW_SW;
    const long long base = (long long)d.N * p.strips * (d.Co / 64) * (d.Cs / 64);
    int rch = (int)cdiv(256, base);  // at least one workgroup per CU
    const int maxch = d.Hs / 8 > 0 ? d.Hs / 8 : 1;  // >= 8 rows per chunk
    rch = rch < 1 ? 1 : (rch > maxch ? maxch : rch);
    p.rows_per = (int)cdiv(d.Hs, rch);
    p.rchunks = (int)cdiv(d.Hs, p.rows_per);
    p.nsplit = d.N * p.strips * p.rchunks;
    return p;
}

}  // namespace

// d describes the FORWARD conv (source x, output dy)
bool wgrad_win_check(const dcs_conv_desc& d) {
    return (d.mma == DCS_MMA_F16X3 || d.mma == DCS_MMA_F16) && d.KH == 3 && d.KW == 3 && d.stride == 1 && d.up == 1 &&
           d.parity == 0 &&
           d.pt == 1 && d.pl == 1 && d.Ho == d.Hs && d.Wo == d.Ws && d.Cs % 64 == 0 && d.Co % 64 == 0 &&
           d.Ws % WW_SW == 0 && d.Hs >= 2 && d.s_c == 1 && d.s_w == d.Cs && d.s_h == (long long)d.Ws * d.Cs &&
           d.s_n == (long long)d.Hs * d.Ws * d.Cs && d.csplit == d.Cs && (d.cw == 0 || d.cw == d.Cs) &&
           d.pro_act == DCS_ACT_NONE && d.rng_a && d.rng_b && d.rng_a_n > 0 && d.rng_a_n <= 1024 &&
           d.rng_b_n > 0 && d.rng_b_n <= 1024 && (long long)d.N * d.Hs * d.Ws * d.Cs * 4 < 0x7fffff00LL - 64 &&
           (long long)d.N * d.Hs * d.Ws * d.Co * 4 < 0x7fffff00LL - 64;
}

size_t wgrad_win_workspace_size(const dcs_conv_desc& d) {
    const WWPlan p = ww_plan(d);
    return (size_t)p.nsplit * d.Co * 9 * d.Cs * sizeof(float);
}

// partial slabs into ws (wgrad_win_workspace_size bytes); returns the split count (< 0: error)
int wgrad_win_launch(const dcs_conv_desc& d, const float* dy, const float* x, float* ws, hipStream_t s) {
    const WWPlan p = ww_plan(d);
    WWArgs a;
    a.N = d.N; a.H = d.Hs; a.W = d.Ws; a.C = d.Cs; a.Co = d.Co;
    a.reflect = d.pad_mode == DCS_PAD_REFLECT;
    a.strips = p.strips; a.rchunks = p.rchunks; a.rows_per = p.rows_per;
    a.gco = d.Co / 64; a.gci = d.Cs / 64;
    a.rng_a_n = d.rng_a_n; a.rng_b_n = d.rng_b_n;
    const unsigned blocks = (unsigned)((long long)p.nsplit * a.gco * a.gci);
    if (d.mma == DCS_MMA_F16 && DCS_WGRAD16_F16)
        hipLaunchKernelGGL(wgrad3_win16_kernel<1>, dim3(blocks), dim3(WW_NT), 0, s, a, dy, x, d.rng_a, d.rng_b, ws);
    else if (d.mma == DCS_MMA_F16)
        hipLaunchKernelGGL(wgrad3_win_h3_kernel<1>, dim3(blocks), dim3(WW_NT), 0, s, a, dy, x, d.rng_a, d.rng_b, ws);
    else if (DCS_WGRAD16)
        hipLaunchKernelGGL(wgrad3_win16_kernel<3>, dim3(blocks), dim3(WW_NT), 0, s, a, dy, x, d.rng_a, d.rng_b, ws);
    else
        hipLaunchKernelGGL(wgrad3_win_h3_kernel<3>, dim3(blocks), dim3(WW_NT), 0, s, a, dy, x, d.rng_a, d.rng_b, ws);
    const int e = check_launch("wgrad3_win");
    return e ? -e : p.nsplit;
}

namespace {

int win_check(const dcs_conv_desc& d, bool fwd) {
    const bool geom = d.KH == 3 && d.KW == 3 && d.stride == 1 && d.up == 1 && !d.parity && d.Cs % 16 == 0 &&
                      d.Co % WIN_BN == 0 && d.Ws >= 2 && d.Ws <= 128 && 256 % d.Ws == 0 && d.Hs % (256 / d.Ws) == 0 &&
                      d.s_c == 1 && d.s_w == d.Cs && d.s_h == (long long)d.Ws * d.Cs &&
                      d.s_n == (long long)d.Hs * d.Ws * d.Cs && d.csplit == d.Cs &&
                      d.epi_act == DCS_ACT_NONE && (d.mma == DCS_MMA_F16X3 || d.mma == DCS_MMA_F16) && d.rng_a && d.rng_a_n > 0 &&
                      d.rng_a_n <= 1024 && (long long)d.N * d.Hs * d.Ws * d.Cs * 4 < 0x7fffff00LL &&
                      d.pro_act == DCS_ACT_NONE;
    if (!geom) return 0;
    if (fwd) return d.Ho == d.Hs && d.Wo == d.Ws && d.pt == 1 && d.pl == 1;
    return d.Ho == d.Hs + 2 && d.Wo == d.Ws + 2 && d.pt == 2 && d.pl == 2 && d.pad_mode == DCS_PAD_ZERO;
}

int launch_win(const dcs_conv_desc& d, int H, int W, int reflect, const float* src, const void* wh, const void* wl,
               const int* wexp, const float* addend, float* out, Part* parts, hipStream_t s,
               const IbwArgs* ibw = nullptr) {
    WinArgs a;
    a.N = d.N; a.H = H; a.W = W; a.C = d.Cs; a.Co = d.Co; a.reflect = reflect;
    a.R = 256 / W; a.tiles = H / a.R; a.gy = d.Co / WIN_BN; a.rng_n = d.rng_a_n;
    const unsigned blocks = (unsigned)(a.N * a.tiles * a.gy);
    const IbwArgs ib = ibw ? *ibw : IbwArgs{nullptr, nullptr, nullptr, nullptr, 0, 0};
    if (DCS_WIN16 && (d.mma == DCS_MMA_F16X3 || DCS_WIN16_F16) && W >= 16 && d.Cs % 32 == 0) {  // the 16x16x32 kernel
        const _Float16* h = reinterpret_cast<const _Float16*>(wh);
        const _Float16* l = reinterpret_cast<const _Float16*>(wl);
#define DCS_WIN16_LAUNCH(IBW_, WIDE_)                                                                              \
    if (d.mma == DCS_MMA_F16X3)                                                                                \
        hipLaunchKernelGGL((conv3_win16_kernel<3, IBW_, WIDE_>), dim3(blocks), dim3(WIN_NT), 0, s, a, src, h, l,   \
                           d.rng_a, wexp, addend, out, parts, ib);                                                 \
    else                                                                                                        \
        hipLaunchKernelGGL((conv3_win16_kernel<1, IBW_, WIDE_>), dim3(blocks), dim3(WIN_NT), 0, s, a, src, h, l,   \
                           d.rng_a, wexp, addend, out, parts, ib);
        if (W >= 64) {
            if (ibw) { DCS_WIN16_LAUNCH(true, true) } else { DCS_WIN16_LAUNCH(false, true) }
        } else {
            if (ibw) { DCS_WIN16_LAUNCH(true, false) } else { DCS_WIN16_LAUNCH(false, false) }
        }
#undef DCS_WIN16_LAUNCH
        return check_launch("conv3_win16");
    }
#define DCS_WIN_LAUNCH(NP_, IBW_)                                                                                 \
    hipLaunchKernelGGL((conv3_win_h3_kernel<NP_, IBW_>), dim3(blocks), dim3(WIN_NT), 0, s, a, src,                     \
                       reinterpret_cast<const _Float16*>(wh), reinterpret_cast<const _Float16*>(wl), d.rng_a, wexp, addend, \
                       out, parts, ib);
    if (d.mma == DCS_MMA_F16) {
        if (ibw) { DCS_WIN_LAUNCH(1, true) } else { DCS_WIN_LAUNCH(1, false) }
    } else {
        if (ibw) { DCS_WIN_LAUNCH(3, true) } else { DCS_WIN_LAUNCH(3, false) }
    }
#undef DCS_WIN_LAUNCH
    return check_launch("conv3_win");
}

// the padded-grid ring on ring16_kernel (d: the data gradient's descriptor, win_check'ed): RG_COPIES ring
// copies (one per tap)
bool ring16_ok(const dcs_conv_desc& d) {
    return DCS_RING16 && d.Cs == 256 && d.Co % 256 == 0 && d.Hs >= 2 && d.Ws >= 2;
}
int launch_ring16(const dcs_conv_desc& d, const float* dy, const void* wh, const void* wl, const int* wexp, float* ring,
                  hipStream_t s) {
    RingArgs a;
    a.N = d.N; a.H = d.Hs; a.W = d.Ws; a.C = d.Cs; a.Co = d.Co; a.rng_n = d.rng_a_n;
    a.tiles_tb = (int)cdiv((long long)d.N * (d.Ws + 2), RG_BM);
    a.tiles_lr = (int)cdiv((long long)d.N * d.Hs, RG_BM);
    const unsigned blocks = (unsigned)((2 * a.tiles_tb + 2 * a.tiles_lr) * 3 * (d.Co / 256));
    const _Float16* h = reinterpret_cast<const _Float16*>(wh);
    const _Float16* l = reinterpret_cast<const _Float16*>(wl);
    if (d.mma == DCS_MMA_F16)
        hipLaunchKernelGGL((ring16_kernel<1, 8>), dim3(blocks), dim3(RG_NT), 0, s, a, dy, h, l, d.rng_a, wexp, ring);
    else
        hipLaunchKernelGGL((ring16_kernel<3, 8>), dim3(blocks), dim3(RG_NT), 0, s, a, dy, h, l, d.rng_a, wexp, ring);
    return check_launch("ring16");
}

}  // namespace

// conv.hip: the generic rows pass (ring rows of the padded data gradient) and the ring fold
int conv_rows_impl(const dcs_conv_desc* dp, const float* src, const float* src2, const float* wpack, const float* bias,
                   const float* psc, const float* psh, float* out, Part* parts, int* bm_used, void* stream, int fold);
int reflect_ring_fold(const float* ring, float* dx, int N, int H, int W, int C, int nsplit, hipStream_t s);
int reflect_ring_fold_ibw(const float* ring, float* dx, int N, int H, int W, int C, int nsplit, const float* y,
                          const float* sc, const float* sh, int act, Sum2* parts, int nchunk, int chunk0, int nfc,
                          hipStream_t s);
int ring_ksplit(const dcs_conv_desc& d);
constexpr int IBW_FOLD_CHUNKS = 64;  // partial-sum chunks of the ring fold per image (its blocks: 64 per image)

}  // namespace dcs

using namespace dcs;

extern "C" size_t dcs_pack_weights_h3_scratch_size(void) { return DCS_RANGE_PARTS * sizeof(float); }

extern "C" int dcs_pack_weights_h3(const float* w, int Cout, int Cin, int flip, int ncols, void* out_hi, void* out_lo,
                                   float* scratch, int* wexp, void* stream) {
    if (!w || !out_hi || !out_lo || !scratch || !wexp || Cout <= 0 || Cin <= 0 || ncols <= 0 ||
        (flip ? Cout : Cin) % 16 != 0 || ncols < (flip ? Cin : Cout))
        return fail(DCS_E_INVALID, "pack_weights_h3: bad arguments (3x3, reduction channels % 16 == 0)");
    hipStream_t s = as_stream(stream);
    const long long nw = (long long)Cout * Cin * 9;
    const long long rb = cdiv(nw, 2048) < DCS_RANGE_PARTS ? cdiv(nw, 2048) : DCS_RANGE_PARTS;  // ~8 weights per thread
    hipLaunchKernelGGL(wrange_kernel, dim3((unsigned)(rb < 1 ? 1 : rb)), dim3(256), 0, s, w, nw, scratch);
    int e = check_launch("pack_weights_h3 range");
    if (e) return e;
    const long long pb = cdiv((long long)ncols * 9 * (flip ? Cout : Cin), 2048);
    hipLaunchKernelGGL(pack_h3_kernel, dim3((unsigned)(pb < 1 ? 1 : (pb > 256 ? 256 : pb))), dim3(256), 0, s, w, Cout, Cin, flip, ncols, scratch,
                       (int)DCS_RANGE_PARTS, reinterpret_cast<_Float16*>(out_hi), reinterpret_cast<_Float16*>(out_lo),
                       wexp);
    return check_launch("pack_weights_h3");
}

#if CLK_PROBE
extern "C" int dcs_probe_clk(unsigned long long* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(dcs::g_clk), (size_t)n * 4 * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
#endif
#if WIN_TIMING
extern "C" int dcs_probe_win_times(unsigned long long* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(dcs::g_win_t), (size_t)n * 5 * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
#endif

extern "C" int dcs_conv3_win_ok(const dcs_conv_desc* dp, int dgrad) { return dp ? win_check(*dp, !dgrad) : 0; }

extern "C" int dcs_conv3_win_in_stats(const dcs_conv_desc* dp, const float* src, const void* w_hi, const void* w_lo,
                                      const int* wexp, float* out, void* parts, size_t parts_bytes, int* nchunk,
                                      void* stream) {
    if (!dp || !src || !w_hi || !w_lo || !wexp || !out) return fail(DCS_E_INVALID, "conv3_win: null pointer");
    const dcs_conv_desc& d = *dp;
    if (!win_check(d, true))
        return fail(DCS_E_INVALID, "conv3_win: needs a 3x3 stride-1 'same' f16x3 conv over contiguous NHWC rows "
                                   "(W <= 128, 256 % W == 0, H % (256 / W) == 0, Cs % 16 == 0, Co % 128 == 0, "
                                   "no prologue)");
    const int tiles = d.Hs / (256 / d.Ws);
    if (parts) {
        if (!nchunk || parts_bytes < (size_t)d.N * tiles * d.Co * sizeof(Part))
            return fail(DCS_E_WORKSPACE, "conv3_win: parts buffer too small");
        *nchunk = tiles;
    }
    return launch_win(d, d.Hs, d.Ws, d.pad_mode == DCS_PAD_REFLECT, src, w_hi, w_lo, wexp, nullptr, out,
                      reinterpret_cast<Part*>(parts), as_stream(stream));
}

extern "C" int dcs_conv_dgrad_reflect_win(const dcs_conv_desc* dp, const float* dy, const float* wpack,
                                          const void* w_hi, const void* w_lo, const int* wexp, const float* addend,
                                          float* dx, float* ring, void* stream) {
    if (!dp || !dy || !wpack || !w_hi || !w_lo || !wexp || !dx || !ring)
        return fail(DCS_E_INVALID, "conv_dgrad_reflect_win: null pointer");
    const dcs_conv_desc& d = *dp;
    if (!win_check(d, false) || d.Co % 4 != 0 || d.Hs < 4 || d.Ws < 4)
        return fail(DCS_E_INVALID, "conv_dgrad_reflect_win: the padded-grid data gradient of a 3x3 reflect-pad-1 conv "
                                   "(dcs_conv_dgrad_reflect's descriptor) with an f16x3 window geometry expected");
    hipStream_t s = as_stream(stream);
    // interior: a 'same' zero-pad conv of dy over the flipped weights, straight into dx (+ addend)
    int e = launch_win(d, d.Hs, d.Ws, 0, dy, w_hi, w_lo, wexp, addend, dx, nullptr, s);
    if (e) return e;
    // the padded grid's one-pixel ring (ring16_kernel, else the generic rows pass), folded onto the border
    if (ring16_ok(d)) {
        if ((e = launch_ring16(d, dy, w_hi, w_lo, wexp, ring, s))) return e;
        return reflect_ring_fold(ring, dx, d.N, d.Ho - 2, d.Wo - 2, d.Co, RG_COPIES, s);
    }
    if ((e = conv_rows_impl(&d, dy, nullptr, wpack, nullptr, nullptr, nullptr, ring, nullptr, nullptr, stream, 2))) return e;
    return reflect_ring_fold(ring, dx, d.N, d.Ho - 2, d.Wo - 2, d.Co, ring_ksplit(d), s);
}

extern "C" size_t dcs_conv_dgrad_reflect_win_inbwd_parts_size(const dcs_conv_desc* dp) {
    if (!dp || dp->Ws <= 0 || 256 % dp->Ws) return 0;
    const int H = dp->Ho - 2, W = dp->Wo - 2;
    if (H <= 0 || W <= 0 || (long long)H * W % 256) return 0;
    return (size_t)dp->N * (H * W / 256 + IBW_FOLD_CHUNKS) * dp->Co * sizeof(Sum2);
}

extern "C" int dcs_conv_dgrad_reflect_win_inbwd(const dcs_conv_desc* dp, const float* dy, const float* wpack,
                                                const void* w_hi, const void* w_lo, const int* wexp, float* dx,
                                                float* ring, const float* y, const float* scale, const float* shift,
                                                int act, void* parts, size_t parts_bytes, int* nchunk, void* stream) {
    if (!dp || !dy || !wpack || !w_hi || !w_lo || !wexp || !dx || !ring || !y || !scale || !shift || !parts || !nchunk)
        return fail(DCS_E_INVALID, "conv_dgrad_reflect_win_inbwd: null pointer");
    const dcs_conv_desc& d = *dp;
    if (!win_check(d, false) || d.Co % 4 != 0 || 256 % (d.Co / 4) || d.Hs < 4 || d.Ws < 4)
        return fail(DCS_E_INVALID, "conv_dgrad_reflect_win_inbwd: a dcs_conv_dgrad_reflect_win geometry with Co / 4 "
                                   "dividing 256 expected");
    if (act != DCS_ACT_AFFINE && act != DCS_ACT_RELU && act != DCS_ACT_LRELU)
        return fail(DCS_E_INVALID, "conv_dgrad_reflect_win_inbwd: act must be DCS_ACT_AFFINE / _RELU / _LRELU");
    if (parts_bytes < dcs_conv_dgrad_reflect_win_inbwd_parts_size(dp))
        return fail(DCS_E_WORKSPACE, "conv_dgrad_reflect_win_inbwd: parts buffer too small");
    hipStream_t s = as_stream(stream);
    const int tiles = d.Hs * d.Ws / 256;
    const int nch = tiles + IBW_FOLD_CHUNKS;
    const IbwArgs ib{y, scale, shift, reinterpret_cast<Sum2*>(parts), act, nch};
    int e = launch_win(d, d.Hs, d.Ws, 0, dy, w_hi, w_lo, wexp, nullptr, dx, nullptr, s, &ib);
    if (e) return e;
    const bool r16 = ring16_ok(d);
    if (r16) e = launch_ring16(d, dy, w_hi, w_lo, wexp, ring, s);
    else e = conv_rows_impl(&d, dy, nullptr, wpack, nullptr, nullptr, nullptr, ring, nullptr, nullptr, stream, 2);
    if (e) return e;
    *nchunk = nch;
    return reflect_ring_fold_ibw(ring, dx, d.N, d.Hs, d.Ws, d.Co, r16 ? RG_COPIES : ring_ksplit(d), y, scale, shift, act,
                                 reinterpret_cast<Sum2*>(parts), nch, tiles, IBW_FOLD_CHUNKS, s);
}
