// The Generator stem (modules/model.py:96-98: ReflectionPad2d(3) + Conv2d(cin, 64, 7) over the image and
// mask planes packed as NHWC x 4, dcs_pack_nhwc4) forward with the InstanceNorm statistics of its
// output, on the MFMA pipe in the f16x3 / f16 operand modes.
//
// The generic rows pass runs this layer as a GEMM with K = 49 taps x 4 channels gathered per A row,
// 0.11 MFMA-busy and ~4x its 1 GB output-write time (profiles/r04a_kernel_table.md:
// conv_rows_kernel<128,64,2,4,7>).  Here a workgroup keeps the whole weight matrix in LDS (split
// once into fp16 hi / lo planes, K reordered as ty * 32 + tx * 4 + c with a zero eighth tap per
// kernel row so every 16-k step is 4 taps of one kernel row) and walks tiles of 4 output rows x
// 64 columns: per tile it stages the reflected 10 x 72 x 4 source window, split once into hi / lo
// fp16, and each lane reads its A fragments (2 taps x 4 channels of one output pixel: 16 contiguous
// bytes of a plane) from it.  One wave per output row: 2 x 32 pixels x 64 channels, 14 k-steps.
// The epilogue writes the output and the per-(tile, channel) InstanceNorm partials in the layout of
// the rows pass (Part, merged by dcs_in_stats_finish).
#include "common.hpp"
#include "conv_common.hpp"

namespace dcs {
namespace {

constexpr int ST_CO = 64;                     // output channels
constexpr int ST_TR = 4, ST_TC = 64;          // tile: 4 rows x 64 columns, one row per wave
constexpr int ST_WR = ST_TR + 6, ST_WC = 72;  // window rows / columns (64 + 6 + 1 zero-weight tap + 1)
constexpr int ST_K = 7 * 32;                  // K: 7 kernel rows x 8 taps x 4 channels
constexpr int ST_BP = ST_K + 8;               // halves per B row (464 B: conflict-free 16-lane b128 reads)
constexpr int ST_NT = 64 * ST_TR;

struct StemArgs {
    int N, H, W;
    int tiles_x, tiles_y;  // per image (nchunk = tiles_x * tiles_y)
    int ldb;               // packed weights: B[k][co] = wp[co * ldb + k], k = tap * 4 + c
    int rng_a_n, rng_b_n;
};

__device__ __forceinline__ int st_reflect(int v, int n) {
    v = v < 0 ? -v : (v >= n ? 2 * n - 2 - v : v);
    return v < 0 ? 0 : (v >= n ? n - 1 : v);
}

__device__ __forceinline__ void part_merge(Part& a, const Part& b) {  // a left of b (lower pixels first)
    const float tot = a.cnt + b.cnt, dl = b.mean - a.mean;
    a.mean += dl * (b.cnt / tot);
    a.m2 += b.m2 + dl * dl * (a.cnt * b.cnt / tot);
    a.cnt = tot;
    if (b.mx > a.mx || (b.mx == a.mx && b.amax < a.amax)) { a.mx = b.mx; a.amax = b.amax; }
}

template <int NP>
__global__ __launch_bounds__(ST_NT, 2) void stem_fwd_kernel(StemArgs a, const float* __restrict__ src,
                                                            const float* __restrict__ wp,
                                                            const float* __restrict__ rnga,
                                                            const float* __restrict__ rngb,
                                                            float* __restrict__ out, Part* __restrict__ parts) {
    constexpr int NPL = NP == 3 ? 2 : 1;
    __shared__ __attribute__((aligned(16))) _Float16 Bs[NPL][ST_CO][ST_BP];
    __shared__ __attribute__((aligned(16))) _Float16 Xw[NPL][ST_WR][ST_WC][4];  // window, split once per tile
    __shared__ Part sp[ST_TR][2][32];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int l32 = lane & 31, kh = lane >> 5;
    const int ea = f16x3_exp(rnga, a.rng_a_n), eb = f16x3_exp(rngb, a.rng_b_n);
    const float asc = __builtin_ldexpf(1.f, ea), bsc = __builtin_ldexpf(1.f, eb);
    const int eab = -(ea + eb);

    // weights: Bs[co][ty * 32 + tx * 4 + c] = W[co][c][ty][tx] (tx = 7: zero), split
    for (int i = tid; i < ST_CO * ST_K; i += ST_NT) {
        const int co = i / ST_K, k = i - co * ST_K;
        const int ty = k >> 5, tx = (k >> 2) & 7, c = k & 3;
        const float v = tx < 7 ? wp[(long long)co * a.ldb + (ty * 7 + tx) * 4 + c] * bsc : 0.f;
        const _Float16 h = (_Float16)v;
        Bs[0][co][k] = h;
        if constexpr (NP == 3) Bs[NPL - 1][co][k] = (_Float16)(v - (float)h);
    }

    const int per = a.tiles_x * a.tiles_y;
    const int ntiles = a.N * per;
    // window of a tile: rows y0 - 3 .., columns x0 - 3 .., reflected; one float4 (4 channels) per pixel,
    // ST_WU per thread, loaded one tile ahead
    constexpr int ST_WU = (ST_WR * ST_WC + ST_NT - 1) / ST_NT;
    float4 wv[ST_WU];
    auto load_win = [&](int tile) {
        const int n = tile / per, chunk = tile - n * per;
        const int tyi = chunk / a.tiles_x, txi = chunk - tyi * a.tiles_x;
        const float* sn = src + (long long)n * a.H * a.W * 4;
#pragma unroll
        for (int q = 0; q < ST_WU; ++q) {
            const int i = tid + q * ST_NT;
            const int r = i / ST_WC, c = i - r * ST_WC;
            const int sy = st_reflect(tyi * ST_TR - 3 + r, a.H), sx = st_reflect(txi * ST_TC - 3 + c, a.W);
            wv[q] = i < ST_WR * ST_WC ? *reinterpret_cast<const float4*>(sn + ((long long)sy * a.W + sx) * 4)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    if (blockIdx.x < ntiles) load_win(blockIdx.x);
#pragma unroll 1
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int n = tile / per, chunk = tile - n * per;
        const int tyi = chunk / a.tiles_x, txi = chunk - tyi * a.tiles_x;
        const int y0 = tyi * ST_TR, x0 = txi * ST_TC;
        __syncthreads();  // the previous tile's window and partials are consumed (and Bs written, first tile)
#pragma unroll
        for (int q = 0; q < ST_WU; ++q) {
            const int i = tid + q * ST_NT;
            if (i < ST_WR * ST_WC) {
                f16x4 hi, lo;
                split4h(wv[q], asc, hi, lo);
                *reinterpret_cast<f16x4*>(&Xw[0][i / ST_WC][i % ST_WC][0]) = hi;
                if constexpr (NP == 3) *reinterpret_cast<f16x4*>(&Xw[NPL - 1][i / ST_WC][i % ST_WC][0]) = lo;
            }
        }
        __syncthreads();
        if (tile + (int)gridDim.x < ntiles) load_win(tile + gridDim.x);  // in flight across this tile's MFMAs
        const int yy = y0 + wid;
        Part pm[2];
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) {
            floatx16 acc[2] = {};
#pragma unroll 2
            for (int ks = 0; ks < 14; ++ks) {
                const int ty = ks >> 1, grp = ks & 1;
                // A: pixel mb * 32 + l32, taps 4 grp + 2 kh, + 1 of kernel row ty, 4 channels each
                const int wc = mb * 32 + l32 + 4 * grp + 2 * kh;
                const f16x4 h0 = *reinterpret_cast<const f16x4*>(&Xw[0][wid + ty][wc][0]);
                const f16x4 h1 = *reinterpret_cast<const f16x4*>(&Xw[0][wid + ty][wc + 1][0]);
                const f16x8 ah = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
                f16x8 al = {};
                if constexpr (NP == 3) {
                    const f16x4 l0 = *reinterpret_cast<const f16x4*>(&Xw[NPL - 1][wid + ty][wc][0]);
                    const f16x4 l1 = *reinterpret_cast<const f16x4*>(&Xw[NPL - 1][wid + ty][wc + 1][0]);
                    al = __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7);
                }
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) {
                    const int ko = 16 * ks + 8 * kh;
                    const f16x8 bh = *reinterpret_cast<const f16x8*>(&Bs[0][nb * 32 + l32][ko]);
                    if constexpr (NP == 3) {
                        const f16x8 bl = *reinterpret_cast<const f16x8*>(&Bs[NPL - 1][nb * 32 + l32][ko]);
                        acc[nb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[nb], 0, 0, 0);
                        acc[nb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[nb], 0, 0, 0);
                    }
                    acc[nb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[nb], 0, 0, 0);
                }
            }
            // epilogue: lane (channel nb * 32 + l32) holds pixels (q & 3) + 8 (q >> 2) + 4 kh of the block
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
                const int c = nb * 32 + l32;
                float v[16];
                float s = 0.f, mx = -INFINITY;
                int am = 0;
                int nv = 0;
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int px = x0 + mb * 32 + (q & 3) + 8 * (q >> 2) + 4 * kh;
                    v[q] = __builtin_ldexpf(acc[nb][q], eab);
                    if (yy < a.H && px < a.W) {
                        out[(((long long)n * a.H + yy) * a.W + px) * ST_CO + c] = v[q];
                        s += v[q];
                        ++nv;
                        if (v[q] > mx) { mx = v[q]; am = yy * a.W + px; }
                    }
                }
                // pixels of a lane increase with q except across the 4-pixel groups of the two halves,
                // so the first maximum is the lowest index among equal values: kept by the merges below
                const float mean = nv ? s / (float)nv : 0.f;
                float m2 = 0.f;
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int px = x0 + mb * 32 + (q & 3) + 8 * (q >> 2) + 4 * kh;
                    if (yy < a.H && px < a.W) {
                        const float dv = v[q] - mean;
                        m2 = fmaf(dv, dv, m2);
                    }
                }
                Part p;
                p.cnt = (float)nv; p.mean = mean; p.m2 = m2; p.mx = mx; p.amax = am;
                p.pad[0] = p.pad[1] = p.pad[2] = 0;
                Part o;
                o.cnt = __shfl_xor(p.cnt, 32, 64); o.mean = __shfl_xor(p.mean, 32, 64);
                o.m2 = __shfl_xor(p.m2, 32, 64); o.mx = __shfl_xor(p.mx, 32, 64);
                o.amax = __shfl_xor(p.amax, 32, 64);
                if (kh == 0) {
                    if (o.cnt > 0.f) {
                        if (p.cnt > 0.f) part_merge(p, o);
                        else p = o;
                    }
                    if (mb == 0) pm[nb] = p;
                    else if (p.cnt > 0.f) {
                        if (pm[nb].cnt > 0.f) part_merge(pm[nb], p);
                        else pm[nb] = p;
                    }
                }
            }
        }
        if (parts) {
            if (kh == 0) {
                sp[wid][0][l32] = pm[0];
                sp[wid][1][l32] = pm[1];
            }
            __syncthreads();
            if (tid < ST_CO) {
                Part t = sp[0][tid >> 5][tid & 31];
#pragma unroll
                for (int w = 1; w < ST_TR; ++w) {
                    const Part b = sp[w][tid >> 5][tid & 31];
                    if (b.cnt > 0.f) {
                        if (t.cnt > 0.f) part_merge(t, b);
                        else t = b;
                    }
                }
                parts[((long long)n * per + chunk) * ST_CO + tid] = t;
            }
        }
    }
}

// Weight gradient of the stem: dW[co][k'] = sum_p dy[p][co] X[p][k'], X[p][ty * 32 + tx * 4 + c] =
// x_pad[y + ty][x + tx][c] (the same K order as the forward, tx = 7 a discarded column).  M = 64 output
// channels, N = 7 blocks of 32 (one kernel row ty each), K = output pixels.  A workgroup owns a strip of
// 64 output columns x SW_RPW rows and walks it row by row: per row it stages the dy row segment (64 px
// x 64 channels, hi / lo fp16, pixel-major with the wgrad3 swizzle) and ONE new source row (72 px x 4
// channels, hi / lo) into a ring of 8; wave ty reads its B fragments from source row y + ty - 3 by
// transposed reads of the row itself: X[p][n] sits at half 4 p + n of the row, a Toeplitz layout whose
// 8-byte lane reads stay aligned.  7 waves, one per kernel row, 2 x 32 channels each; two-level
// accumulation (a row, then the running sum); per-workgroup partials [block][co][224], summed over the
// blocks in a fixed order.
constexpr int SW_NT = 64 * 7;
constexpr int SW_TC = 64;                    // output columns per strip
constexpr int SW_XC = SW_TC + 8;             // source columns staged per row (64 + 6 + 2)
constexpr int SW_RPW = 64;                   // output rows per workgroup
constexpr int SW_XROW = 2 * SW_XC * 4;       // halves per ring slot (hi, lo planes)
constexpr int SW_DROW = 2 * SW_TC * 64;      // halves of the dy buffer (hi, lo planes)

struct StemWArgs {
    int N, H, W;
    int strips, bands;
    int rng_a_n, rng_b_n;
};

__device__ __forceinline__ int sw_swz(int pix) { return ((pix >> 1) & 1) << 2; }

typedef short swshortx4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) swshortx4 lds_swshortx4;

__device__ __forceinline__ f16x8 sw_frag(const _Float16* p, int second) {  // rows q and q + 4 (second: halves)
    const swshortx4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_swshortx4*)(p));
    const swshortx4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_swshortx4*)(p + second));
    return __builtin_bit_cast(f16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int NP>
__global__ __launch_bounds__(SW_NT, 1) void stem_wgrad_kernel(StemWArgs a, const float* __restrict__ dy,
                                                              const float* __restrict__ src,
                                                              const float* __restrict__ rnga,
                                                              const float* __restrict__ rngb,
                                                              float* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) _Float16 Dy[SW_DROW];
    __shared__ __attribute__((aligned(16))) _Float16 Xr[8][SW_XROW];

    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int strip = L % a.strips, rest = L / a.strips;
    const int band = rest % a.bands, n = rest / a.bands;
    const int x0 = strip * SW_TC, y_beg = band * SW_RPW;
    const int y_end = y_beg + SW_RPW < a.H ? y_beg + SW_RPW : a.H;
    const int tid = threadIdx.x, lane = tid & 63, ty = tid >> 6;

    const int ea = f16x3_exp(rnga, a.rng_a_n), eb = f16x3_exp(rngb, a.rng_b_n);
    const float asc = __builtin_ldexpf(1.f, ea), bsc = __builtin_ldexpf(1.f, eb);

    // dy staging: units (pixel, 8-channel group), u = tid (+ SW_NT)
    constexpr int DU = (SW_TC * 8 + SW_NT - 1) / SW_NT;  // 2
    float4 dr[DU][2];
    auto load_dy = [&](int y) {
#pragma unroll
        for (int q = 0; q < DU; ++q) {
            const int u = tid + q * SW_NT;
            const int pix = u >> 3, cu = u & 7;
            const bool ok = u < SW_TC * 8 && x0 + pix < a.W;
            const float* p = dy + (((long long)n * a.H + y) * a.W + x0 + pix) * 64 + 8 * cu;
            dr[q][0] = ok ? *reinterpret_cast<const float4*>(p) : make_float4(0.f, 0.f, 0.f, 0.f);
            dr[q][1] = ok ? *reinterpret_cast<const float4*>(p + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto store_dy = [&]() {
#pragma unroll
        for (int q = 0; q < DU; ++q) {
            const int u = tid + q * SW_NT;
            if (u < SW_TC * 8) {
                const int pix = u >> 3, cu = u & 7;
                f16x8 hi, lo;
                split8h(dr[q][0], dr[q][1], asc, hi, lo);
                const int o = pix * 64 + 8 * (cu ^ sw_swz(pix));
                *reinterpret_cast<f16x8*>(&Dy[o]) = hi;
                if constexpr (NP == 3) *reinterpret_cast<f16x8*>(&Dy[SW_TC * 64 + o]) = lo;
            }
        }
    };
    // source row staging: one pixel (4 channels) per thread, columns x0 - 3 .. x0 + 68, reflected
    float4 xv = make_float4(0.f, 0.f, 0.f, 0.f);
    const int xcol = tid < SW_XC ? st_reflect(x0 - 3 + tid, a.W) : 0;
    auto load_x = [&](int r) {  // padded row r in [y_beg - 3, y_end + 3)
        if (tid < SW_XC)
            xv = *reinterpret_cast<const float4*>(src + (((long long)n * a.H + st_reflect(r, a.H)) * a.W + xcol) * 4);
    };
    auto store_x = [&](int r) {
        if (tid < SW_XC) {
            f16x4 hi, lo;
            split4h(xv, bsc, hi, lo);
            _Float16* row = &Xr[r & 7][0];
            *reinterpret_cast<f16x4*>(row + tid * 4) = hi;
            if constexpr (NP == 3) *reinterpret_cast<f16x4*>(row + SW_XC * 4 + tid * 4) = lo;
        }
    };

    // fragment offsets (halves): in a 16-lane group lane 4q+p reads pixel row q (+4), columns 4p .. 4p+3
    const int g16 = lane >> 4;
    const int rpix = 8 * (g16 >> 1) + ((lane & 15) >> 2);
    const int rcol = 16 * (g16 & 1) + 4 * (lane & 3);
    int aoff[2];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
        const int c = 32 * mb + rcol;
        aoff[mb] = rpix * 64 + 8 * ((c >> 3) ^ sw_swz(rpix)) + (c & 7);
    }
    const int boff = 4 * rpix + rcol;  // Toeplitz row: X[p][n] at 4 p + n

    floatx16 acc[2] = {}, tt[2] = {};
    // prologue: source rows y_beg - 3 .. y_beg + 2 into the ring
#pragma unroll 1
    for (int r = y_beg - 3; r < y_beg + 3; ++r) {
        load_x(r);
        store_x(r);
    }
    load_dy(y_beg);
    load_x(y_beg + 3);
#pragma unroll 1
    for (int y = y_beg; y < y_end; ++y) {
        __syncthreads();  // the previous row's fragment reads are done
        store_dy();
        store_x(y + 3);
        if (y + 1 < y_end) {
            load_dy(y + 1);
            load_x(y + 4);
        }
        __syncthreads();
        const _Float16* xs = &Xr[(y + ty - 3) & 7][0];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const f16x8 bh = sw_frag(xs + boff + 64 * ks, 16);
            f16x8 bl = {};
            if constexpr (NP == 3) bl = sw_frag(xs + SW_XC * 4 + boff + 64 * ks, 16);
#pragma unroll
            for (int mb = 0; mb < 2; ++mb) {
                const f16x8 ah = sw_frag(&Dy[aoff[mb] + ks * 16 * 64], 4 * 64);
                if constexpr (NP == 3) {
                    const f16x8 al = sw_frag(&Dy[SW_TC * 64 + aoff[mb] + ks * 16 * 64], 4 * 64);
                    tt[mb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, tt[mb], 0, 0, 0);
                    tt[mb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, tt[mb], 0, 0, 0);
                }
                tt[mb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, tt[mb], 0, 0, 0);
            }
        }
        if (((y - y_beg) & 1) == 1 || y + 1 == y_end) {  // two-level: 128 pixels per chain
#pragma unroll
            for (int mb = 0; mb < 2; ++mb) {
                acc[mb] += tt[mb];
                tt[mb] = floatx16{};
            }
        }
    }
    const int eab = -(ea + eb);
    float* dst = part + (long long)blockIdx.x * (64 * ST_K);
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int co = 32 * mb + (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5);
            dst[co * ST_K + ty * 32 + (lane & 31)] = __builtin_ldexpf(acc[mb][q], eab);
        }
}

// dw[co][c][ty][tx] (OIHW, c < cw) = sum over the blocks of part[block][co][ty * 32 + tx * 4 + c]: 64
// outputs per workgroup, four block groups (b = g mod 4) summed in block order each, then the four in a
// fixed order
__global__ __launch_bounds__(256) void stem_wgrad_reduce_kernel(const float* __restrict__ part, int nblk, int cw,
                                                                float* __restrict__ dw) {
    __shared__ float red[4][64];
    const int o = threadIdx.x & 63, grp = threadIdx.x >> 6;
    const int i = blockIdx.x * 64 + o;  // co * 224 + k'
    const int co = i / ST_K, k = i - co * ST_K;
    const int ty = k >> 5, tx = (k >> 2) & 7, c = k & 3;
    const bool live = i < 64 * ST_K && tx < 7 && c < cw;
    float s = 0.f;
    if (live) {
#pragma unroll 8
        for (int b = grp; b < nblk; b += 4) s += part[(long long)b * (64 * ST_K) + i];
    }
    red[grp][o] = s;
    __syncthreads();
    if (grp == 0 && live) dw[((co * cw + c) * 7 + ty) * 7 + tx] = ((red[0][o] + red[1][o]) + red[2][o]) + red[3][o];
}

}  // namespace
}  // namespace dcs

using namespace dcs;

namespace {
// the stem's geometry and operand mode (both passes)
bool stem_geom(const dcs_conv_desc* dp) {
    if (!dp) return false;
    const dcs_conv_desc& d = *dp;
    return d.Cs == 4 && d.Co == ST_CO && d.KH == 7 && d.KW == 7 && d.stride == 1 && d.up == 1 && !d.parity &&
           d.pt == 3 && d.pl == 3 && d.pad_mode == DCS_PAD_REFLECT && d.Ho == d.Hs && d.Wo == d.Ws && d.Hs >= 4 &&
           d.Ws >= 4 && d.s_c == 1 && d.s_w == 4 && d.s_h == (long long)d.Ws * 4 && d.s_n == (long long)d.Hs * d.Ws * 4 &&
           d.csplit == d.Cs && d.pro_act == DCS_ACT_NONE && d.epi_act == DCS_ACT_NONE &&
           (d.mma == DCS_MMA_F16X3 || d.mma == DCS_MMA_F16) && d.rng_a && d.rng_b && d.rng_a_n > 0 &&
           d.rng_a_n <= 1024 && d.rng_b_n > 0 && d.rng_b_n <= 1024;  // f16x3_exp reads at most 1024 partials
}
}  // namespace

extern "C" int dcs_stem_fwd_ok(const dcs_conv_desc* dp) { return stem_geom(dp) && dp->ldb >= 196; }

extern "C" size_t dcs_stem_fwd_parts_size(const dcs_conv_desc* dp) {
    if (!dp) return 0;
    return (size_t)dp->N * cdiv(dp->Hs, ST_TR) * cdiv(dp->Ws, ST_TC) * ST_CO * sizeof(Part);
}

extern "C" int dcs_stem_fwd(const dcs_conv_desc* dp, const float* src, const float* wpack, float* out, void* parts,
                            size_t parts_bytes, int* nchunk, void* stream) {
    if (!dp || !src || !wpack || !out) return fail(DCS_E_INVALID, "stem_fwd: null pointer");
    if (!dcs_stem_fwd_ok(dp))
        return fail(DCS_E_INVALID, "stem_fwd: a 7x7 reflect-pad-3 conv 4 -> 64 over contiguous NHWC x 4, no prologue / "
                                   "epilogue, f16x3 / f16 operands with range records expected");
    if (parts && parts_bytes < dcs_stem_fwd_parts_size(dp)) return fail(DCS_E_WORKSPACE, "stem_fwd: parts too small");
    if ((reinterpret_cast<uintptr_t>(src) & 15) != 0) return fail(DCS_E_INVALID, "stem_fwd: source not 16-byte aligned");
    const dcs_conv_desc& d = *dp;
    StemArgs a;
    a.N = d.N; a.H = d.Hs; a.W = d.Ws;
    a.tiles_x = (int)cdiv(d.Ws, ST_TC);
    a.tiles_y = (int)cdiv(d.Hs, ST_TR);
    a.ldb = d.ldb;
    a.rng_a_n = d.rng_a_n; a.rng_b_n = d.rng_b_n;
    if (nchunk) *nchunk = a.tiles_x * a.tiles_y;
    const long long ntiles = (long long)a.N * a.tiles_x * a.tiles_y;
    const unsigned blocks = (unsigned)(ntiles < 512 ? ntiles : 512);  // persistent: 2 per CU, weights staged once per block
    hipStream_t s = as_stream(stream);
    Part* p = reinterpret_cast<Part*>(parts);
    if (d.mma == DCS_MMA_F16)
        hipLaunchKernelGGL(stem_fwd_kernel<1>, dim3(blocks), dim3(ST_NT), 0, s, a, src, wpack, d.rng_a, d.rng_b, out, p);
    else
        hipLaunchKernelGGL(stem_fwd_kernel<3>, dim3(blocks), dim3(ST_NT), 0, s, a, src, wpack, d.rng_a, d.rng_b, out, p);
    return check_launch("stem_fwd");
}

extern "C" int dcs_stem_wgrad_ok(const dcs_conv_desc* dp) {
    if (!dp) return 0;
    const dcs_conv_desc& d = *dp;
    const int cw = d.cw > 0 ? d.cw : d.Cs;
    return stem_geom(dp) && cw >= 1 && cw <= 4;
}

extern "C" size_t dcs_stem_wgrad_workspace_size(const dcs_conv_desc* dp) {
    if (!dp) return 0;
    return (size_t)dp->N * cdiv(dp->Ws, SW_TC) * cdiv(dp->Hs, SW_RPW) * 64 * ST_K * sizeof(float);
}

extern "C" int dcs_stem_wgrad(const dcs_conv_desc* dp, const float* dy, const float* src, float* dw, void* ws,
                              size_t ws_bytes, void* stream) {
    if (!dp || !dy || !src || !dw || !ws) return fail(DCS_E_INVALID, "stem_wgrad: null pointer");
    if (!dcs_stem_wgrad_ok(dp))
        return fail(DCS_E_INVALID, "stem_wgrad: the stem geometry (dcs_stem_fwd_ok) with dy / source range records expected");
    if (ws_bytes < dcs_stem_wgrad_workspace_size(dp)) return fail(DCS_E_WORKSPACE, "stem_wgrad: workspace too small");
    if ((reinterpret_cast<uintptr_t>(src) & 15) || (reinterpret_cast<uintptr_t>(dy) & 15))
        return fail(DCS_E_INVALID, "stem_wgrad: operands not 16-byte aligned");
    const dcs_conv_desc& d = *dp;
    StemWArgs a;
    a.N = d.N; a.H = d.Hs; a.W = d.Ws;
    a.strips = (int)cdiv(d.Ws, SW_TC);
    a.bands = (int)cdiv(d.Hs, SW_RPW);
    a.rng_a_n = d.rng_a_n; a.rng_b_n = d.rng_b_n;
    const unsigned blocks = (unsigned)((long long)a.N * a.strips * a.bands);
    hipStream_t s = as_stream(stream);
    float* part = reinterpret_cast<float*>(ws);
    if (d.mma == DCS_MMA_F16)
        hipLaunchKernelGGL(stem_wgrad_kernel<1>, dim3(blocks), dim3(SW_NT), 0, s, a, dy, src, d.rng_a, d.rng_b, part);
    else
        hipLaunchKernelGGL(stem_wgrad_kernel<3>, dim3(blocks), dim3(SW_NT), 0, s, a, dy, src, d.rng_a, d.rng_b, part);
    int e = check_launch("stem_wgrad");
    if (e) return e;
    hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3((unsigned)cdiv(64 * ST_K, 64)), dim3(256), 0, s, part,
                       (int)blocks, d.cw > 0 ? d.cw : d.Cs, dw);
    return check_launch("stem_wgrad_reduce");
}
