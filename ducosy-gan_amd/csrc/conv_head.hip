// The Generator head (modules/model.py:112: ReflectionPad2d(3) + Conv2d 64 -> 1, 7 x 7 + Tanh) forward
// on the MFMA pipe, by tap projection: out[y][x] = b + sum_t z[y + ty - 3][x + tx - 3][t] with
// z[p][t] = sum_c a[p][c] * W[c][t] (a = relu(IN(y_up2)), t = 7 ty + tx).  z is a GEMM (M = source
// pixels, N = 49 taps padded to 64, K = 64 channels) on v_mfma_f32_32x32x16_f16 in the f16x3 / f16
// operand modes; the 49-tap sum is a fixed-order gather from LDS.
//
// conv_narrow.hip's VALU kernel (exact f32) stages an 8-channel slice of a 22 x 70 halo per pass and
// walks the 64 channels in 8 passes, so every pass touches one 32-byte piece of each pixel's 256-byte
// row: with ~100 workgroups per XCD those rows leave the L2 between passes and the layer moved 5.3x its
// algorithmic bytes (profiles/r04a_kernel_table.md).  Here a workgroup owns a strip of 128 output
// columns x HP_RPW output rows and walks the HP_RPW + 6 source rows of the strip once: per source row it
// stages the 134 reflected pixels x 64 channels (IN + ReLU applied, split hi / lo fp16), projects them
// onto the taps, and adds each tap row's contribution to the 7 output rows it feeds (a ring of 8
// partial rows in LDS; each partial sum is updated by one thread, in source-row order, so the result
// is deterministic).  Output row y is complete after source row y + 3 and written with the bias and
// the epilogue activation then.
#include "common.hpp"
#include "conv_common.hpp"

namespace dcs {
namespace {

constexpr int HP_C = 64;                 // source channels
constexpr int HP_KS = 7, HP_R = 3;       // 7 x 7, reflection padding 3
constexpr int HP_TW = 128;               // output columns per strip
constexpr int HP_SW = HP_TW + 2 * HP_R;  // 134 source columns
constexpr int HP_MB = 5;                 // 32-row MFMA blocks over the 134 source columns (160 rows)
constexpr int HP_NT = 64 * 2 * HP_MB;    // 10 waves: one (m block, tap block) pair each
constexpr int HP_AP = 72;                // halves per staged pixel and plane (64 + 8: conflict-free b128 reads)
constexpr int HP_ZP = 65;                // floats per z row (odd: the gather's 32 lanes hit 32 banks)
constexpr int HP_RING = 8;               // partial output rows in flight (7 needed)
constexpr int HP_RPW = 32;               // output rows per workgroup
constexpr int HP_UNITS = (HP_SW * HP_C / 4 + HP_NT - 1) / HP_NT;  // float4 source units per thread (4)

struct HeadArgs {
    int N, H, W;   // source / output geometry (NHWC source [N][H][W][64], output [N][H][W])
    int strips;    // ceil(W / 128)
    int bands;     // ceil(H / HP_RPW)
    int epi_act;   // DCS_ACT_NONE / DCS_ACT_TANH
    int ldb;       // packed weight stride: W[c][t] = wp[(t * 64 + c) * ldb]
};

__device__ __forceinline__ int hp_reflect(int v, int n) {
    v = v < 0 ? -v : (v >= n ? 2 * n - 2 - v : v);
    return v < 0 ? 0 : (v >= n ? n - 1 : v);  // tiny images: fold into range (such values only feed masked outputs)
}

template <int NP>
__global__ __launch_bounds__(HP_NT, 1) void head_fwd_proj_kernel(HeadArgs a, const float* __restrict__ src,
                                                                 const float* __restrict__ wp,
                                                                 const float* __restrict__ bias,
                                                                 const float* __restrict__ psc,
                                                                 const float* __restrict__ psh,
                                                                 const float* __restrict__ xmax,
                                                                 float* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) _Float16 As[NP == 3 ? 2 : 1][32 * HP_MB][HP_AP];
    __shared__ float Zs[HP_SW][HP_ZP];
    __shared__ float Ring[HP_RING][HP_TW];

    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int strip = L % a.strips, rest = L / a.strips;
    const int band = rest % a.bands, n = rest / a.bands;
    const int x0 = strip * HP_TW, y_beg = band * HP_RPW;
    const int y_end = y_beg + HP_RPW < a.H ? y_beg + HP_RPW : a.H;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int l32 = lane & 31, kh = lane >> 5;
    const int mb = wid >> 1, nb = wid & 1;

    // operand scales: A from the IN statistics (max of relu(x * scale + shift) over the image's planes is
    // relu(xmax * scale + shift), scale > 0), B from the weights; every wave derives both itself
    const long long nc = (long long)n * HP_C + lane;
    const float am = fmaxf(fmaf(xmax[nc], psc[nc], psh[nc]), 0.f);
    float bm = 0.f;
    for (int i = lane; i < HP_KS * HP_KS * HP_C; i += 64) bm = fmaxf(bm, fabsf(wp[(long long)i * a.ldb]));
    int ea, eb;
    {
        const float m1 = wave_max(am), m2 = wave_max(bm);
        int e1 = 0, e2 = 0;
        (void)frexpf(m1, &e1);
        (void)frexpf(m2, &e2);
        ea = __builtin_amdgcn_readfirstlane(min(max(15 - e1, -100), 100));
        eb = __builtin_amdgcn_readfirstlane(min(max(15 - e2, -100), 100));
    }
    const float asc = __builtin_ldexpf(1.f, ea), bsc = __builtin_ldexpf(1.f, eb);

    // B fragments (taps nb * 32 + l32, channels ks * 16 + kh * 8 .. + 7) for the whole kernel
    f16x8 bh[4], bl[4];
    {
        const int t = nb * 32 + l32;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            float v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int c = ks * 16 + kh * 8 + i;
                v[i] = t < HP_KS * HP_KS ? wp[((long long)t * HP_C + c) * a.ldb] * bsc : 0.f;
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const _Float16 h = (_Float16)v[i];
                bh[ks][i] = h;
                bl[ks][i] = (_Float16)(v[i] - (float)h);
            }
        }
    }

    // staging units of this thread: (source column j, 4-channel group); the prologue's scale / shift
    int ucol[HP_UNITS], ucg[HP_UNITS];
    float4 usc[HP_UNITS], ush[HP_UNITS];
#pragma unroll
    for (int q = 0; q < HP_UNITS; ++q) {
        const int u = tid + q * HP_NT;
        const int j = u >> 4, cg = u & 15;
        ucol[q] = j < HP_SW ? hp_reflect(x0 - HP_R + j, a.W) : -1;
        ucg[q] = cg;
        usc[q] = *reinterpret_cast<const float4*>(psc + (long long)n * HP_C + 4 * cg);
        ush[q] = *reinterpret_cast<const float4*>(psh + (long long)n * HP_C + 4 * cg);
    }
    float4 uv[HP_UNITS];
    auto load_row = [&](int r) {  // source row r (reflected), every unit
        const int sy = hp_reflect(r, a.H);
        const float* row = src + ((long long)n * a.H + sy) * a.W * HP_C;
#pragma unroll
        for (int q = 0; q < HP_UNITS; ++q)
            uv[q] = ucol[q] >= 0 ? *reinterpret_cast<const float4*>(row + (long long)ucol[q] * HP_C + 4 * ucg[q])
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    auto store_row = [&]() {
#pragma unroll
        for (int q = 0; q < HP_UNITS; ++q) {
            const int u = tid + q * HP_NT;
            const int j = u >> 4;
            if (j < HP_SW) {
                const float v[4] = {fmaxf(fmaf(uv[q].x, usc[q].x, ush[q].x), 0.f) * asc,
                                    fmaxf(fmaf(uv[q].y, usc[q].y, ush[q].y), 0.f) * asc,
                                    fmaxf(fmaf(uv[q].z, usc[q].z, ush[q].z), 0.f) * asc,
                                    fmaxf(fmaf(uv[q].w, usc[q].w, ush[q].w), 0.f) * asc};
                f16x4 hi, lo;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    hi[i] = (_Float16)v[i];
                    lo[i] = (_Float16)(v[i] - (float)hi[i]);
                }
                *reinterpret_cast<f16x4*>(&As[0][j][4 * ucg[q]]) = hi;
                if constexpr (NP == 3) *reinterpret_cast<f16x4*>(&As[1][j][4 * ucg[q]]) = lo;
            }
        }
    };

    // zero the MFMA rows past the 134 source columns (never restaged) and the partial rows
    for (int i = tid; i < (32 * HP_MB - HP_SW) * HP_AP; i += HP_NT) {
        const int rr = HP_SW + i / HP_AP, cc = i % HP_AP;
        As[0][rr][cc] = (_Float16)0.f;
        if constexpr (NP == 3) As[1][rr][cc] = (_Float16)0.f;
    }
    for (int i = tid; i < HP_RING * HP_TW; i += HP_NT) (&Ring[0][0])[i] = 0.f;

    const float bv = bias ? bias[0] : 0.f;
    const int eab = -(ea + eb);
    const int r_beg = y_beg - HP_R, r_end = y_end + HP_R;  // source rows [r_beg, r_end)
    load_row(r_beg);
    for (int r = r_beg; r < r_end; ++r) {
        __syncthreads();  // the previous row's gathers are done with Zs / Ring, its MFMAs with As
        store_row();
        if (r + 1 < r_end) load_row(r + 1);  // in flight across this row's MFMAs and gathers
        __syncthreads();
        // z = A W for this wave's (32 source columns, 32 taps)
        floatx16 acc = {};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const f16x8 ah = *reinterpret_cast<const f16x8*>(&As[0][mb * 32 + l32][ks * 16 + kh * 8]);
            if constexpr (NP == 3) {
                const f16x8 al = *reinterpret_cast<const f16x8*>(&As[1][mb * 32 + l32][ks * 16 + kh * 8]);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[ks], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[ks], acc, 0, 0, 0);
            }
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[ks], acc, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int px = mb * 32 + (q & 3) + 8 * (q >> 2) + 4 * kh;
            if (px < HP_SW) Zs[px][nb * 32 + l32] = __builtin_ldexpf(acc[q], eab);
        }
        __syncthreads();
        // tap rows: output row y = r + 3 - ty gets sum_tx z[x + tx][7 ty + tx]; row r - 3 completes
        for (int item = tid; item < HP_KS * HP_TW; item += HP_NT) {
            const int ty = item / HP_TW, x = item - ty * HP_TW;
            const int y = r + HP_R - ty;
            if (y < y_beg || y >= y_end) continue;
            float s = 0.f;
#pragma unroll
            for (int tx = 0; tx < HP_KS; ++tx) s += Zs[x + tx][HP_KS * ty + tx];
            float* slot = &Ring[y & (HP_RING - 1)][x];
            const float v = *slot + s;
            if (ty == HP_KS - 1) {  // the last contribution to row y
                if (x0 + x < a.W) {
                    float o = v + bv;
                    if (a.epi_act != DCS_ACT_NONE) o = act_apply(o, a.epi_act);
                    out[((long long)n * a.H + y) * a.W + x0 + x] = o;
                }
                *slot = 0.f;
            } else {
                *slot = v;
            }
        }
    }
}

// Weight gradient of the head on the MFMA pipe: dW[c][t] = sum_p a[p + off_t][c] g[p] (a: the
// reflected, IN + ReLU source; g: the gradient at the pre-tanh output).  Same workgroup decomposition
// and source-row walk as the forward: per padded source row r the workgroup stages the 134 source
// columns once and adds A^T B with M = 64 channels, N = 49 taps (padded to 64), K = the 144 (134 +
// zero rows) source columns j, where B[j][t] = g[r + 3 - ty][x0 + j - tx] pairs source column j with
// the output pixel that reads it through tap t (zero outside the workgroup's band and strip, so every
// (output pixel, tap) pair is counted by exactly one workgroup).  A fragments are transposed reads of
// the pixel-major source (ds_read_b64_tr_b16, 8 columns of one channel per lane); the B fragment of a
// lane is 8 consecutive g values of its tap's shifted row, read from one of four copies of the g row
// pre-shifted by 0..3 elements so the read is 8-byte aligned at any tap offset.  g rows live in a ring
// of 8 (7 in use).  One 32 x 32 (channel, tap) block per wave, two-level accumulation (a row's 9
// k-steps, then the running sum).  Per-workgroup partial [block][t * 64 + c] summed over the blocks in
// a fixed order (deterministic).
constexpr int HW_NT = 256;                               // 4 waves: (channel block, tap block)
constexpr int HW_KP = 144;                               // source columns padded to 9 k-steps of 16
constexpr int HW_GL = 152;                               // halves per shifted g copy (u = x - x0 + 8 in [0, 152))
constexpr int HW_GI = (4 * HW_GL + HW_NT - 1) / HW_NT;   // g staging items per thread (3)
constexpr int HW_XU = (HP_SW * 8 + HW_NT - 1) / HW_NT;   // (column, 8-channel unit)s per thread (5)
constexpr int HW_TAPS = HP_KS * HP_KS;

__device__ __forceinline__ int hw_swz(int j) { return ((j >> 1) & 1) << 2; }

typedef short hshortx4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) hshortx4 lds_hshortx4;

__device__ __forceinline__ f16x8 hw_frag_tr(const _Float16* p) {  // 8 columns of one channel
    const hshortx4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_hshortx4*)(p));
    const hshortx4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_hshortx4*)(p + 4 * 64));
    return __builtin_bit_cast(f16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int NP>
__global__ __launch_bounds__(HW_NT, 2) void head_wgrad_proj_kernel(HeadArgs a, const float* __restrict__ src,
                                                                   const float* __restrict__ psc,
                                                                   const float* __restrict__ psh,
                                                                   const float* __restrict__ xmax,
                                                                   const float* __restrict__ g,
                                                                   float* __restrict__ part) {
    constexpr int NPL = NP == 3 ? 2 : 1;  // planes: hi (+ lo)
    __shared__ __attribute__((aligned(16))) _Float16 As[NPL][HW_KP * 64];
    __shared__ __attribute__((aligned(16))) _Float16 Gs[HP_RING][4][NPL][HW_GL];
    __shared__ float red[HW_NT / 64];

    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int strip = L % a.strips, rest = L / a.strips;
    const int band = rest % a.bands, n = rest / a.bands;
    const int x0 = strip * HP_TW, y_beg = band * HP_RPW;
    const int y_end = y_beg + HP_RPW < a.H ? y_beg + HP_RPW : a.H;
    const int xn = a.W - x0 < HP_TW ? a.W - x0 : HP_TW;  // output columns of this strip
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int kh = lane >> 5;
    const int mb = wid >> 1, nb = wid & 1;

    // operand scales: A as in the forward; B from max |g| over this workgroup's outputs
    const long long nc = (long long)n * HP_C + lane;
    const float am = fmaxf(fmaf(xmax[nc], psc[nc], psh[nc]), 0.f);
    float gm = 0.f;
    for (int i = tid; i < HP_RPW * HP_TW; i += HW_NT) {
        const int yy = y_beg + i / HP_TW, xx = i % HP_TW;
        if (yy < y_end && xx < xn) gm = fmaxf(gm, fabsf(g[((long long)n * a.H + yy) * a.W + x0 + xx]));
    }
    gm = wave_max(gm);
    if (lane == 0) red[wid] = gm;
    // zero the ring (rows before the band are never staged) and the padding columns of As
    for (int i = tid; i < HP_RING * 4 * NPL * HW_GL; i += HW_NT) (&Gs[0][0][0][0])[i] = (_Float16)0.f;
    for (int i = tid; i < (HW_KP - HP_SW) * 64; i += HW_NT) {
        As[0][HP_SW * 64 + i] = (_Float16)0.f;
        if constexpr (NP == 3) As[NPL - 1][HP_SW * 64 + i] = (_Float16)0.f;
    }
    __syncthreads();
    gm = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    int ea, eg;
    {
        const float m1 = wave_max(am);
        int e1 = 0, e2 = 0;
        (void)frexpf(m1, &e1);
        (void)frexpf(gm, &e2);
        ea = __builtin_amdgcn_readfirstlane(min(max(15 - e1, -100), 100));
        eg = __builtin_amdgcn_readfirstlane(min(max(15 - e2, -100), 100));
    }
    const float asc = __builtin_ldexpf(1.f, ea), gsc = __builtin_ldexpf(1.f, eg);

    // source staging: units (column j = (tid >> 3) + 32 q, channels 8 cu .. 8 cu + 7), cu fixed per thread
    const int cu = tid & 7;
    float sc[8], sh[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        sc[i] = psc[(long long)n * HP_C + 8 * cu + i];
        sh[i] = psh[(long long)n * HP_C + 8 * cu + i];
    }
    int ucol[HW_XU];
#pragma unroll
    for (int q = 0; q < HW_XU; ++q) {
        const int j = (tid >> 3) + 32 * q;
        ucol[q] = j < HP_SW ? hp_reflect(x0 - HP_R + j, a.W) : -1;
    }
    float4 uv[HW_XU][2];
    auto load_row = [&](int r) {
        const float* row = src + ((long long)n * a.H + hp_reflect(r, a.H)) * a.W * HP_C + 8 * cu;
#pragma unroll
        for (int q = 0; q < HW_XU; ++q) {
            if (ucol[q] >= 0) {
                uv[q][0] = *reinterpret_cast<const float4*>(row + (long long)ucol[q] * HP_C);
                uv[q][1] = *reinterpret_cast<const float4*>(row + (long long)ucol[q] * HP_C + 4);
            }
        }
    };
    auto store_row = [&]() {
#pragma unroll
        for (int q = 0; q < HW_XU; ++q) {
            if (ucol[q] >= 0) {
                const int j = (tid >> 3) + 32 * q;
                const float v[8] = {uv[q][0].x, uv[q][0].y, uv[q][0].z, uv[q][0].w,
                                    uv[q][1].x, uv[q][1].y, uv[q][1].z, uv[q][1].w};
                f16x8 hi, lo;
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const float f = fmaxf(fmaf(v[i], sc[i], sh[i]), 0.f) * asc;
                    hi[i] = (_Float16)f;
                    lo[i] = (_Float16)(f - (float)hi[i]);
                }
                const int o = j * 64 + 8 * (cu ^ hw_swz(j));
                *reinterpret_cast<f16x8*>(&As[0][o]) = hi;
                if constexpr (NP == 3) *reinterpret_cast<f16x8*>(&As[NPL - 1][o]) = lo;
            }
        }
    };
    // g staging: items (copy s, element v) hold g[y][x0 + v + s - 8], zero outside the band / strip
    float gv[HW_GI];
    auto load_g = [&](int y) {
        const bool yok = y >= y_beg && y < y_end;
#pragma unroll
        for (int q = 0; q < HW_GI; ++q) {
            const int it = tid + q * HW_NT;
            const int s = it / HW_GL, v = it - s * HW_GL;
            const int xx = v + s - 8;
            gv[q] = (yok && it < 4 * HW_GL && xx >= 0 && xx < xn) ? g[((long long)n * a.H + y) * a.W + x0 + xx] : 0.f;
        }
    };
    auto store_g = [&](int y) {
#pragma unroll
        for (int q = 0; q < HW_GI; ++q) {
            const int it = tid + q * HW_NT;
            if (it < 4 * HW_GL) {
                const int s = it / HW_GL, v = it - s * HW_GL;
                const float f = gv[q] * gsc;
                const _Float16 hi = (_Float16)f;
                Gs[y & (HP_RING - 1)][s][0][v] = hi;
                if constexpr (NP == 3) Gs[y & (HP_RING - 1)][s][NPL - 1][v] = (_Float16)(f - (float)hi);
            }
        }
    };

    // fragment offsets.  A (M = channel, K = column): transposed read, lane (r, h) gets columns
    // 8h .. 8h+7 of channel r; in a 16-lane group lane 4q+p reads column q (+4), channels 4p .. 4p+3
    int aoff;
    {
        const int g16 = lane >> 4;
        const int rpix = 8 * (g16 >> 1) + ((lane & 15) >> 2);
        const int c = 32 * mb + 16 * (g16 & 1) + 4 * (lane & 3);
        aoff = rpix * 64 + 8 * ((c >> 3) ^ hw_swz(rpix)) + (c & 7);
    }
    // B (K = column, N = tap): lane (t, h) reads g[r + 3 - ty][x0 + j - tx], j = 16 ks + 8 h .. + 7,
    // i.e. copy s = u & 3 at element u - s, u = 16 ks + 8 h + 8 - tx
    const int t = nb * 32 + (lane & 31);
    const bool tok = t < HW_TAPS;
    const int ty = tok ? t / HP_KS : 0, tx = tok ? t % HP_KS : 0;
    int goff[9];
#pragma unroll
    for (int ks = 0; ks < 9; ++ks) {
        const int u = 16 * ks + 8 * kh + 8 - tx;
        goff[ks] = (u & 3) * NPL * HW_GL + (u & ~3);
    }

    floatx16 acc = {};
    const int r_beg = y_beg - HP_R, r_end = y_end + HP_R;
    load_row(r_beg);
    load_g(r_beg + HP_R);
    for (int r = r_beg; r < r_end; ++r) {
        __syncthreads();  // the previous row's fragment reads are done
        store_row();
        store_g(r + HP_R);
        if (r + 1 < r_end) {
            load_row(r + 1);
            load_g(r + 1 + HP_R);
        }
        __syncthreads();
        const _Float16* gb = &Gs[(r + HP_R - ty) & (HP_RING - 1)][0][0][0];
        floatx16 tt = {};
#pragma unroll
        for (int ks = 0; ks < 9; ++ks) {
            const f16x8 ah = hw_frag_tr(&As[0][aoff + ks * 16 * 64]);
            f16x8 bh = {}, bl = {};
            if (tok) {
                const f16x4 b0 = *reinterpret_cast<const f16x4*>(gb + goff[ks]);
                const f16x4 b1 = *reinterpret_cast<const f16x4*>(gb + goff[ks] + 4);
                bh = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
                if constexpr (NP == 3) {
                    const f16x4 c0 = *reinterpret_cast<const f16x4*>(gb + HW_GL + goff[ks]);
                    const f16x4 c1 = *reinterpret_cast<const f16x4*>(gb + HW_GL + goff[ks] + 4);
                    bl = __builtin_shufflevector(c0, c1, 0, 1, 2, 3, 4, 5, 6, 7);
                }
            }
            if constexpr (NP == 3) {
                const f16x8 al = hw_frag_tr(&As[NPL - 1][aoff + ks * 16 * 64]);
                tt = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, tt, 0, 0, 0);
                tt = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, tt, 0, 0, 0);
            }
            tt = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, tt, 0, 0, 0);
        }
        acc += tt;
    }
    if (tok) {
        const int eab = -(ea + eg);
        float* dst = part + (long long)blockIdx.x * (HW_TAPS * HP_C) + (long long)t * HP_C + 32 * mb + 4 * kh;
#pragma unroll
        for (int q = 0; q < 16; ++q) dst[(q & 3) + 8 * (q >> 2)] = __builtin_ldexpf(acc[q], eab);
    }
}

// dw[c][t] (OIHW, Co = 1) = sum over the blocks of part[block][t * 64 + c]: 64 outputs per workgroup,
// four block groups (b = g mod 4) summed in block order each, then the four in a fixed order
__global__ __launch_bounds__(256) void head_wgrad_reduce_kernel(const float* __restrict__ part, int nblk,
                                                                float* __restrict__ dw) {
    __shared__ float red[4][64];
    const int o = threadIdx.x & 63, grp = threadIdx.x >> 6;
    const int i = blockIdx.x * 64 + o;  // t * 64 + c
    float s = 0.f;
    if (i < HW_TAPS * HP_C) {
#pragma unroll 8
        for (int b = grp; b < nblk; b += 4) s += part[(long long)b * (HW_TAPS * HP_C) + i];
    }
    red[grp][o] = s;
    __syncthreads();
    if (grp == 0 && i < HW_TAPS * HP_C) {
        const float t4 = ((red[0][o] + red[1][o]) + red[2][o]) + red[3][o];
        const int t = i / HP_C, c = i - t * HP_C;
        dw[c * HW_TAPS + t] = t4;
    }
}

// Data gradient of the head fused with the InstanceNorm + ReLU backward of its input
// (modules/model.py:110-112): da[p][c] = sum_t G[p][t] W[c][t], G[p][t] = sum over the padded
// positions q that reflect onto p of g[q - off_t] (the padding adjoint folded into the one-channel
// gradient, as dgrad_c1_kernel does), then dy = IN-ReLU-backward(da).  da is a GEMM (M = pixels,
// N = 64 channels, K = the 7 x 7 taps laid out as 8 kernel rows x 8 columns, the eighth of each
// zero) on the MFMA pipe and is never written: pass 0 computes it per tile and reduces the IN
// backward's per-channel sums sum(da m) and sum(da m xhat) (m: ReLU mask), pass 1 recomputes it
// (bit-identical: same tiles, scales and instruction sequence) and writes dy.  HBM traffic: y once in
// pass 0, y + dy in pass 1, against da written, re-read twice and y read twice by the separate
// dgrad / partial / apply passes.
// Tile: HB_TR rows x 64 columns, one row per wave (two 32-pixel MFMA blocks); the one-channel g over
// the tile + 3-pixel halo is staged in LDS (fp32, plus a zero margin row and column for the padding
// taps).  K step ks holds kernel rows 2 ks (lanes kh = 0) and 2 ks + 1 (kh = 1), columns 0..7, so a
// lane's 8 entries are 8 consecutive window values (one row, descending columns).  Pixels away from
// the border read them directly; the 3-pixel border sums its reflection preimages.  Workgroups are
// persistent per image (HB_PP of them), so the partial sums come in HB_PP chunks per image.
constexpr int HB_TR = 4, HB_TC = 64;
// g window rows y0 - 7 .. y0 + 12 and columns x0 - 7 .. x0 + 72 (zero outside the image): every read of
// the primary preimage (taps padded to 8 x 8) and of the reflected ones stays inside it
constexpr int HB_OFF = 7;
constexpr int HB_WR = HB_TR + 16, HB_WC = HB_TC + 16;  // 20 x 80
constexpr int HB_NT = 64 * HB_TR;
constexpr int HB_PP = 64;  // workgroups (partial-sum chunks) per image

struct HeadBwdArgs {
    int N, H, W;
    int tiles_x, tiles_y;  // per image
    int pp;                // workgroups per image
    int grng_n;            // partial maxima in g's range record
};

__device__ __forceinline__ int hb_pre(int i, int n, int* a) {  // padded-row preimages of i (pad_preimages)
    int k = 0;
    a[k++] = i + HP_R;
    if (i >= 1 && i <= HP_R) a[k++] = HP_R - i;
    if (i >= n - 1 - HP_R && i <= n - 2) a[k++] = 2 * (n - 1) - i + HP_R;
    return k;
}

template <int NP, int PASS>
__global__ __launch_bounds__(HB_NT, 2) void head_bwd_in_kernel(HeadBwdArgs a, const float* __restrict__ g,
                                                               const float* __restrict__ grng,
                                                               const float* __restrict__ wk,
                                                               const float* __restrict__ y,
                                                               const float* __restrict__ sc,
                                                               const float* __restrict__ sh,
                                                               const Sum2* __restrict__ coef,
                                                               Sum2* __restrict__ parts,
                                                               float* __restrict__ dy, float* __restrict__ rng) {
    __shared__ float Gw[HB_WR][HB_WC];  // Gw[r][c] = g[y0 - 7 + r][x0 - 7 + c], zero outside the image
    __shared__ float red[HB_NT / 64][2][HP_C];

    const int n = blockIdx.x / a.pp, wg = blockIdx.x - n * a.pp;
    const int per = a.tiles_x * a.tiles_y;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int l32 = lane & 31, kh = lane >> 5;
    const int H = a.H, W = a.W;
    const float* gn = g + (long long)n * H * W;

    // weight scale (every wave: max |W| over the 3136 weights); g scale from g's range record, two
    // binades lower since a folded entry sums up to four g values
    float wm = 0.f;
    for (int i = lane; i < HW_TAPS * HP_C; i += 64) wm = fmaxf(wm, fabsf(wk[i]));
    wm = wave_max(wm);
    const int eg = f16x3_exp(grng, a.grng_n) - 2;
    int eb;
    {
        int e2 = 0;
        (void)frexpf(wm, &e2);
        eb = __builtin_amdgcn_readfirstlane(min(max(15 - e2, -100), 100));
    }
    const float gsc = __builtin_ldexpf(1.f, eg), bsc = __builtin_ldexpf(1.f, eb);
    const int eab = -(eg + eb);

    // B fragments: lane (channel nb * 32 + l32, h) at step ks holds W[c][ty = 2 ks + h][tx = 0..7]
    f16x8 bh[2][4], bl[2][4];
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const int ty = 2 * ks + kh;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float v = (ty < HP_KS && i < HP_KS) ? wk[(ty * HP_KS + i) * HP_C + nb * 32 + l32] * bsc : 0.f;
                const _Float16 h = (_Float16)v;
                bh[nb][ks][i] = h;
                bl[nb][ks][i] = (_Float16)(v - (float)h);
            }
        }
    float sclo[2], shlo[2];
    Sum2 kk[2];
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
        sclo[nb] = sc[(long long)n * HP_C + nb * 32 + l32];
        shlo[nb] = sh[(long long)n * HP_C + nb * 32 + l32];
        kk[nb] = PASS == 1 ? coef[(long long)n * HP_C + nb * 32 + l32] : Sum2{0.f, 0.f};
    }

    float psa[2] = {0.f, 0.f}, psb[2] = {0.f, 0.f};
    float rmax = 0.f;
    // g window of a tile, HB_GU values per thread, loaded one tile ahead (unconditional loads from
    // clamped addresses, the zero fill applied at the LDS store)
    constexpr int HB_GU = (HB_WR * HB_WC + HB_NT - 1) / HB_NT;
    float gv[HB_GU];
    auto load_g = [&](int chunk) {
        const int tyi = chunk / a.tiles_x, txi = chunk - tyi * a.tiles_x;
#pragma unroll
        for (int q = 0; q < HB_GU; ++q) {
            const int i = tid + q * HB_NT;
            const int r = i / HB_WC, c = i - r * HB_WC;
            const int gy = tyi * HB_TR - HB_OFF + r, gx = txi * HB_TC - HB_OFF + c;
            gv[q] = gn[(long long)min(max(gy, 0), H - 1) * W + min(max(gx, 0), W - 1)];
        }
    };
    if (wg < per) load_g(wg);
#pragma unroll 1
    for (int chunk = wg; chunk < per; chunk += a.pp) {
        const int tyi = chunk / a.tiles_x, txi = chunk - tyi * a.tiles_x;
        const int y0 = tyi * HB_TR, x0 = txi * HB_TC;
        __syncthreads();  // the previous tile's reads of Gw are done
#pragma unroll
        for (int q = 0; q < HB_GU; ++q) {
            const int i = tid + q * HB_NT;
            const int r = i / HB_WC, c = i - r * HB_WC;
            const int gy = y0 - HB_OFF + r, gx = x0 - HB_OFF + c;
            if (i < HB_WR * HB_WC) Gw[r][c] = (gy >= 0 && gy < H && gx >= 0 && gx < W) ? gv[q] : 0.f;
        }
        __syncthreads();
        if (chunk + a.pp < per) load_g(chunk + a.pp);  // in flight across this tile
        const int yy = y0 + wid;  // this wave's pixel row
        const bool row_ok = yy < H;
        const int yc = row_ok ? yy : H - 1;
#pragma unroll 1
        for (int mb = 0; mb < 2; ++mb) {
            const int xl = mb * 32 + l32;  // the lane's A-row pixel (column within the tile)
            const int xx = x0 + xl;
            // a lane's entries at step ks: g rows r = a - ty over the padded-row preimages a of its pixel
            // row (a = yy + 3, and a reflected one within 3 pixels of the border), columns likewise:
            // Gw[7 + r - y0][7 + c - x0] (c = b - i); the second preimage, where absent, enters with
            // weight 0 (adding +0 leaves the sum unchanged, so the order of the terms is fixed)
            const bool lane_inner = yy > HP_R && yy < H - 1 - HP_R && xx > HP_R && xx < W - 1 - HP_R;
            int ay[3], ax[3];
            const int ny = hb_pre(yy, H, ay), nx = hb_pre(xx, W, ax);
            const int ry0 = HB_OFF + ay[0] - y0, ry1 = HB_OFF + (ny > 1 ? ay[1] : ay[0]) - y0;
            const int rx0 = HB_OFF + ax[0] - x0, rx1 = HB_OFF + (nx > 1 ? ax[1] : ax[0]) - x0;
            const float my = ny > 1 ? 1.f : 0.f, mx = nx > 1 ? 1.f : 0.f;
            // y of the block's outputs: all 32 loads issued before the MFMAs (clamped addresses, masked after)
            float yv[2][16];
            const long long ybase = ((long long)n * H + yc) * W;
#pragma unroll
            for (int nb = 0; nb < 2; ++nb)
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int px = x0 + mb * 32 + (q & 3) + 8 * (q >> 2) + 4 * kh;
                    yv[nb][q] = y[(ybase + (px < W ? px : W - 1)) * HP_C + nb * 32 + l32];
                }
            floatx16 acc[2] = {};
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                const int ty = 2 * ks + kh;
                float v[8];
                if (lane_inner) {
                    const float* rp = &Gw[ry0 - ty][rx0];
#pragma unroll
                    for (int i = 0; i < 8; ++i) v[i] = rp[-i];
                } else {
                    const float* p00 = &Gw[ry0 - ty][rx0];
                    const float* p01 = &Gw[ry0 - ty][rx1];
                    const float* p10 = &Gw[ry1 - ty][rx0];
                    const float* p11 = &Gw[ry1 - ty][rx1];
#pragma unroll
                    for (int i = 0; i < 8; ++i)
                        v[i] = fmaf(my * mx, p11[-i], fmaf(my, p10[-i], fmaf(mx, p01[-i], p00[-i])));
                }
                f16x8 ah, al;
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const float f = v[i] * gsc;
                    const _Float16 h = (_Float16)f;
                    ah[i] = h;
                    al[i] = (_Float16)(f - (float)h);
                }
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) {
                    if constexpr (NP == 3) {
                        acc[nb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[nb][ks], acc[nb], 0, 0, 0);
                        acc[nb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[nb][ks], acc[nb], 0, 0, 0);
                    }
                    acc[nb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[nb][ks], acc[nb], 0, 0, 0);
                }
            }
            // epilogue: lane (channel nb * 32 + l32) holds pixels (q & 3) + 8 (q >> 2) + 4 kh of the block
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
                const int c = nb * 32 + l32;
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int px = x0 + mb * 32 + (q & 3) + 8 * (q >> 2) + 4 * kh;
                    const bool ok = row_ok && px < W;
                    const float da = __builtin_ldexpf(acc[nb][q], eab);
                    const float xh = fmaf(yv[nb][q], sclo[nb], shlo[nb]);
                    const float gd = (ok && xh > 0.f) ? da : 0.f;
                    if constexpr (PASS == 0) {
                        psa[nb] += gd;
                        psb[nb] = fmaf(gd, xh, psb[nb]);
                    } else {
                        const float o = sclo[nb] * (gd - kk[nb].a - xh * kk[nb].b);
                        if (ok) {
                            dy[(ybase + px) * HP_C + c] = o;
                            rmax = fmaxf(rmax, fabsf(o));
                        }
                    }
                }
            }
        }
    }
    if constexpr (PASS == 1) {
        range_note(rng, rmax);
    } else {
        __syncthreads();
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
            psa[nb] += __shfl_xor(psa[nb], 32, 64);
            psb[nb] += __shfl_xor(psb[nb], 32, 64);
            if (kh == 0) {
                red[wid][0][nb * 32 + l32] = psa[nb];
                red[wid][1][nb * 32 + l32] = psb[nb];
            }
        }
        __syncthreads();
        if (tid < HP_C) {
            float sa = 0.f, sb = 0.f;
#pragma unroll
            for (int w = 0; w < HB_NT / 64; ++w) {
                sa += red[w][0][tid];
                sb += red[w][1][tid];
            }
            parts[((long long)n * a.pp + wg) * HP_C + tid] = Sum2{sa, sb};
        }
    }
}

// coef[n][c] = (sum of the chunks' partials) / HW, in double and chunk order
__global__ void head_bwd_finalize_kernel(const Sum2* __restrict__ parts, int N, int nchunk, int HW,
                                         Sum2* __restrict__ coef) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= N * HP_C) return;
    const int n = idx / HP_C, c = idx - n * HP_C;
    double sa = 0.0, sb = 0.0;
    for (int k = 0; k < nchunk; ++k) {
        const Sum2 p = parts[((long long)n * nchunk + k) * HP_C + c];
        sa += p.a;
        sb += p.b;
    }
    coef[idx] = Sum2{(float)(sa / HW), (float)(sb / HW)};
}

}  // namespace
}  // namespace dcs

using namespace dcs;

extern "C" int dcs_head_fwd_proj_ok(const dcs_conv_desc* dp) {
    if (!dp) return 0;
    const dcs_conv_desc& d = *dp;
    return d.Co == 1 && d.Cs == HP_C && d.KH == HP_KS && d.KW == HP_KS && d.stride == 1 && d.up == 1 && !d.parity &&
           d.pt == HP_R && d.pl == HP_R && d.pad_mode == DCS_PAD_REFLECT && d.Ho == d.Hs && d.Wo == d.Ws &&
           d.Hs >= HP_R + 1 && d.Ws >= HP_R + 1 && d.s_c == 1 && d.s_w == HP_C && d.s_h == (long long)d.Ws * HP_C &&
           d.s_n == (long long)d.Hs * d.Ws * HP_C && d.csplit == d.Cs && d.pro_act == DCS_ACT_RELU &&
           (d.epi_act == DCS_ACT_NONE || d.epi_act == DCS_ACT_TANH) && (d.mma == DCS_MMA_F16X3 || d.mma == DCS_MMA_F16);
}

extern "C" int dcs_head_fwd_proj(const dcs_conv_desc* dp, const float* src, const float* wpack, const float* bias,
                                 const float* pro_scale, const float* pro_shift, const float* xmax, float* out,
                                 void* stream) {
    if (!dp || !src || !wpack || !pro_scale || !pro_shift || !xmax || !out)
        return fail(DCS_E_INVALID, "head_fwd_proj: null pointer");
    if (!dcs_head_fwd_proj_ok(dp))
        return fail(DCS_E_INVALID, "head_fwd_proj: a 7x7 reflect-pad-3 conv 64 -> 1 over contiguous NHWC rows, IN + "
                                   "ReLU prologue, f16x3 / f16 operands expected");
    const dcs_conv_desc& d = *dp;
    if (d.ldb < 1) return fail(DCS_E_INVALID, "head_fwd_proj: ldb < 1");
    HeadArgs a;
    a.N = d.N; a.H = d.Hs; a.W = d.Ws;
    a.strips = (int)cdiv(d.Ws, HP_TW);
    a.bands = (int)cdiv(d.Hs, HP_RPW);
    a.epi_act = d.epi_act;
    a.ldb = d.ldb;
    const unsigned blocks = (unsigned)((long long)a.N * a.strips * a.bands);
    hipStream_t s = as_stream(stream);
    if (d.mma == DCS_MMA_F16)
        hipLaunchKernelGGL(head_fwd_proj_kernel<1>, dim3(blocks), dim3(HP_NT), 0, s, a, src, wpack, bias, pro_scale,
                           pro_shift, xmax, out);
    else
        hipLaunchKernelGGL(head_fwd_proj_kernel<3>, dim3(blocks), dim3(HP_NT), 0, s, a, src, wpack, bias, pro_scale,
                           pro_shift, xmax, out);
    return check_launch("head_fwd_proj");
}

extern "C" size_t dcs_head_wgrad_proj_workspace_size(const dcs_conv_desc* dp) {
    if (!dp) return 0;
    const long long blocks = (long long)dp->N * cdiv(dp->Ws, HP_TW) * cdiv(dp->Hs, HP_RPW);
    return (size_t)blocks * HW_TAPS * HP_C * sizeof(float);
}

extern "C" int dcs_head_wgrad_proj(const dcs_conv_desc* dp, const float* dy, const float* src,
                                   const float* pro_scale, const float* pro_shift, const float* xmax, float* dw,
                                   void* ws, size_t ws_bytes, void* stream) {
    if (!dp || !dy || !src || !pro_scale || !pro_shift || !xmax || !dw || !ws)
        return fail(DCS_E_INVALID, "head_wgrad_proj: null pointer");
    if (!dcs_head_fwd_proj_ok(dp))
        return fail(DCS_E_INVALID, "head_wgrad_proj: a 7x7 reflect-pad-3 conv 64 -> 1 over contiguous NHWC rows, IN + "
                                   "ReLU prologue, f16x3 / f16 operands expected");
    if (ws_bytes < dcs_head_wgrad_proj_workspace_size(dp)) return fail(DCS_E_WORKSPACE, "head_wgrad_proj: workspace too small");
    const dcs_conv_desc& d = *dp;
    HeadArgs a;
    a.N = d.N; a.H = d.Hs; a.W = d.Ws;
    a.strips = (int)cdiv(d.Ws, HP_TW);
    a.bands = (int)cdiv(d.Hs, HP_RPW);
    a.epi_act = DCS_ACT_NONE;
    a.ldb = 0;
    const unsigned blocks = (unsigned)((long long)a.N * a.strips * a.bands);
    hipStream_t s = as_stream(stream);
    float* part = reinterpret_cast<float*>(ws);
    if (d.mma == DCS_MMA_F16)
        hipLaunchKernelGGL(head_wgrad_proj_kernel<1>, dim3(blocks), dim3(HW_NT), 0, s, a, src, pro_scale, pro_shift,
                           xmax, dy, part);
    else
        hipLaunchKernelGGL(head_wgrad_proj_kernel<3>, dim3(blocks), dim3(HW_NT), 0, s, a, src, pro_scale, pro_shift,
                           xmax, dy, part);
    int e = check_launch("head_wgrad_proj");
    if (e) return e;
    hipLaunchKernelGGL(head_wgrad_reduce_kernel, dim3((unsigned)cdiv(HW_TAPS * HP_C, 64)), dim3(256), 0, s, part,
                       (int)blocks, dw);
    return check_launch("head_wgrad_proj_reduce");
}

extern "C" size_t dcs_head_dgrad_in_workspace_size(int N, int H, int W) {
    if (N <= 0 || H <= 0 || W <= 0) return 0;
    return align_up((size_t)N * HB_PP * HP_C * sizeof(Sum2), 256) + (size_t)N * HP_C * sizeof(Sum2);
}

extern "C" int dcs_head_dgrad_in(const float* dy_out, const float* dy_rng, int dy_rng_n, const float* wk, int N, int H,
                                 int W, const float* y, const float* scale, const float* shift, int act, int mma,
                                 float* dy, void* ws, size_t ws_bytes, float* rng, void* stream) {
    if (!dy_out || !dy_rng || !wk || !y || !scale || !shift || !dy || !ws)
        return fail(DCS_E_INVALID, "head_dgrad_in: null pointer");
    if (dy_rng_n <= 0 || dy_rng_n > 1024)
        return fail(DCS_E_INVALID, "head_dgrad_in: dy_rng_n must be in 1..1024 (range-record partials)");
    if (N <= 0 || H < 2 * HP_R + 2 || W < 2 * HP_R + 2 || act != DCS_ACT_RELU || (mma != DCS_MMA_F16X3 && mma != DCS_MMA_F16))
        return fail(DCS_E_INVALID, "head_dgrad_in: H, W >= 8, ReLU, f16x3 / f16 operands expected");
    if (ws_bytes < dcs_head_dgrad_in_workspace_size(N, H, W)) return fail(DCS_E_WORKSPACE, "head_dgrad_in: workspace too small");
    HeadBwdArgs a;
    a.N = N; a.H = H; a.W = W;
    a.tiles_x = (int)cdiv(W, HB_TC);
    a.tiles_y = (int)cdiv(H, HB_TR);
    a.pp = a.tiles_x * a.tiles_y < HB_PP ? a.tiles_x * a.tiles_y : HB_PP;
    a.grng_n = dy_rng_n;
    const unsigned blocks = (unsigned)((long long)N * a.pp);
    Sum2* parts = reinterpret_cast<Sum2*>(ws);
    Sum2* coef = reinterpret_cast<Sum2*>(reinterpret_cast<char*>(ws) + align_up((size_t)N * HB_PP * HP_C * sizeof(Sum2), 256));
    hipStream_t s = as_stream(stream);
    int e;
    if (mma == DCS_MMA_F16)
        hipLaunchKernelGGL((head_bwd_in_kernel<1, 0>), dim3(blocks), dim3(HB_NT), 0, s, a, dy_out, dy_rng, wk, y, scale, shift,
                           nullptr, parts, nullptr, nullptr);
    else
        hipLaunchKernelGGL((head_bwd_in_kernel<3, 0>), dim3(blocks), dim3(HB_NT), 0, s, a, dy_out, dy_rng, wk, y, scale, shift,
                           nullptr, parts, nullptr, nullptr);
    if ((e = check_launch("head_dgrad_in_partial"))) return e;
    hipLaunchKernelGGL(head_bwd_finalize_kernel, dim3((unsigned)cdiv((long long)N * HP_C, 256)), dim3(256), 0, s, parts,
                       N, a.pp, H * W, coef);
    if ((e = check_launch("head_dgrad_in_finalize"))) return e;
    if ((e = range_zero(rng, s))) return e;
    if (mma == DCS_MMA_F16)
        hipLaunchKernelGGL((head_bwd_in_kernel<1, 1>), dim3(blocks), dim3(HB_NT), 0, s, a, dy_out, dy_rng, wk, y, scale, shift,
                           coef, nullptr, dy, rng);
    else
        hipLaunchKernelGGL((head_bwd_in_kernel<3, 1>), dim3(blocks), dim3(HB_NT), 0, s, a, dy_out, dy_rng, wk, y, scale, shift,
                           coef, nullptr, dy, rng);
    return check_launch("head_dgrad_in_apply");
}
