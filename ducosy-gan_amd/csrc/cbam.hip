// CBAM tail of ResidualBlockWithCBAM (modules/model.py:6-52, 68-87) on NHWC fp32:
//   z = IN(y);  ca = sigmoid(fc(avgpool z) + fc(maxpool z));  zc = z*ca
//   s = [mean_c zc, max_c zc];  sa = sigmoid(conv7x7(s));  out = x + zc*sa
// avgpool(IN(y)) is identically 0 (IN output has zero mean per (n,c)), so the avg branch is
// evaluated on exact zeros: it contributes fc(0) = 0 forward and exactly 0 gradient.
// maxpool(IN(y)) = IN(max y) because the IN scale is positive, so the max comes from the
// statistics pass over y.  Channel reductions run 16 lanes per pixel, 4 pixels per wave (16
// channels per lane as float4 columns, 4-step xor reductions inside a 16-lane row) for C = 64,
// 128, 256, and one wave64 per pixel otherwise; the per-(n, c) sums of the backward run as
// float4 columns with pixel lanes folded through LDS.
#include "common.hpp"

#ifndef DCS_SERIAL_UNROLL
#define DCS_SERIAL_UNROLL 8  // serial fixed-order reductions: loads hoisted, additions in order
#endif

namespace dcs {

// ---- channel attention MLP (one block per image) ----------------------------------------
__global__ __launch_bounds__(256) void ca_forward_kernel(const float* __restrict__ ymax, const float* __restrict__ sc,
                                                         const float* __restrict__ sh, const float* __restrict__ w1,
                                                         const float* __restrict__ w2, int C, int Cr,
                                                         float* __restrict__ ca) {
    extern __shared__ float sm[];
    float* vmax = sm;          // [C]
    float* h = sm + C;         // [Cr] relu(W1 vmax)
    float* h0 = h + Cr;        // [Cr] relu(W1 * 0)
    const int n = blockIdx.x, tid = threadIdx.x;
    for (int c = tid; c < C; c += blockDim.x) vmax[c] = fmaf(ymax[n * C + c], sc[n * C + c], sh[n * C + c]);
    __syncthreads();
    for (int j = tid; j < Cr; j += blockDim.x) {
        float a = 0.f;
        for (int c = 0; c < C; ++c) a = fmaf(w1[j * C + c], vmax[c], a);
        h[j] = a > 0.f ? a : 0.f;
        h0[j] = 0.f;  // relu(W1 * avgpool(IN(y))) with avgpool == 0
    }
    __syncthreads();
    for (int c = tid; c < C; c += blockDim.x) {
        float oa = 0.f, om = 0.f;
        for (int j = 0; j < Cr; ++j) {
            oa = fmaf(w2[c * Cr + j], h0[j], oa);
            om = fmaf(w2[c * Cr + j], h[j], om);
        }
        ca[n * C + c] = sigmoidf_(oa + om);
    }
}

// ---- spatial attention input: per pixel mean/max over channels of zc ---------------------
__global__ __launch_bounds__(256) void sa_reduce_kernel(const float* __restrict__ y, const float* __restrict__ sc,
                                                        const float* __restrict__ sh, const float* __restrict__ ca,
                                                        int HW, int C, long long P, float* __restrict__ sin_,
                                                        int* __restrict__ sarg) {
    const long long p = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (p >= P) return;
    const int n = (int)(p / HW);
    const float* yp = y + p * C;
    const float* s = sc + (long long)n * C;
    const float* b = sh + (long long)n * C;
    const float* a = ca + (long long)n * C;
    float sum = 0.f, mx = -INFINITY;
    int am = 0;
    for (int c4 = lane; c4 < C / 4; c4 += 64) {
        float4 v = reinterpret_cast<const float4*>(yp)[c4];
        float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            int c = c4 * 4 + q;
            float zc = fmaf(e[q], s[c], b[c]) * a[c];
            sum += zc;
            if (zc > mx) { mx = zc; am = c; }
        }
    }
    sum = wave_sum(sum);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        float om = __shfl_xor(mx, o, 64);
        int oa = __shfl_xor(am, o, 64);
        if (om > mx || (om == mx && oa < am)) { mx = om; am = oa; }
    }
    if (lane == 0) {
        sin_[p * 2 + 0] = sum / (float)C;
        sin_[p * 2 + 1] = mx;
        sarg[p] = am;
    }
}

// ---- spatial attention conv + sigmoid + scale + residual add (wave per pixel) ------------
__global__ __launch_bounds__(256) void sa_apply_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                       const float* __restrict__ sc, const float* __restrict__ sh,
                                                       const float* __restrict__ ca, const float* __restrict__ sin_,
                                                       const float* __restrict__ wsa, int H, int W, int C, int ksa,
                                                       long long P, float* __restrict__ sa,
                                                       float* __restrict__ out, float* __restrict__ rng) {
    const long long p = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (p >= P) return;  // wave-uniform
    const int HW = H * W;
    const int n = (int)(p / HW);
    const int rem = (int)(p - (long long)n * HW);
    const int py = rem / W, px = rem - py * W;
    const int r = ksa / 2, taps = ksa * ksa;
    float pre = 0.f;
    for (int t = lane; t < 2 * taps; t += 64) {
        int ch = t / taps, tt = t - ch * taps;
        int ty = tt / ksa, tx = tt - ty * ksa;
        int yy = py + ty - r, xx = px + tx - r;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W)
            pre = fmaf(wsa[t], sin_[((long long)n * HW + yy * W + xx) * 2 + ch], pre);
    }
    pre = wave_sum(pre);
    const float g = sigmoidf_(pre);
    if (lane == 0) sa[p] = g;
    const float* s = sc + (long long)n * C;
    const float* b = sh + (long long)n * C;
    const float* a = ca + (long long)n * C;
    float m = 0.f;
    for (int c4 = lane; c4 < C / 4; c4 += 64) {
        float4 v = reinterpret_cast<const float4*>(y + p * C)[c4];
        float4 xv = reinterpret_cast<const float4*>(x + p * C)[c4];
        int c = c4 * 4;
        float4 o;
        o.x = xv.x + fmaf(v.x, s[c + 0], b[c + 0]) * a[c + 0] * g;
        o.y = xv.y + fmaf(v.y, s[c + 1], b[c + 1]) * a[c + 1] * g;
        o.z = xv.z + fmaf(v.z, s[c + 2], b[c + 2]) * a[c + 2] * g;
        o.w = xv.w + fmaf(v.w, s[c + 3], b[c + 3]) * a[c + 3] * g;
        reinterpret_cast<float4*>(out + p * C)[c4] = o;
        m = fmaxf(m, absmax4(o));
    }
    range_note(rng, m);
}

// ---- 16-lane-per-pixel forms (C = 64 * NQ, NQ in {1, 2, 4}) -------------------------------
// A wave holds 4 pixels; lane j of a pixel's 16-lane group owns float4 columns q*16 + j
// (q < NQ), so every load instruction moves 4 pixels x 256 contiguous bytes, the per-(image,
// channel) scale / shift / ca stay in registers across the wave's pixels (reloaded only when the
// image changes), and each reduction over channels is 4 xor steps inside a 16-lane row.
constexpr int CB_QUADS = 4;  // pixel quads per wave

template <int NQ>
struct CbRegs {
    float4 s[NQ], b[NQ], a[NQ];
    int n = -1;
    __device__ __forceinline__ void load(const float* sc, const float* sh, const float* ca, int C, int nn, int j) {
        if (nn == n) return;
        n = nn;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const long long o = (long long)nn * C + 4 * (q * 16 + j);
            s[q] = *reinterpret_cast<const float4*>(sc + o);
            b[q] = *reinterpret_cast<const float4*>(sh + o);
            a[q] = *reinterpret_cast<const float4*>(ca + o);
        }
    }
};

__device__ __forceinline__ float row16_sum(float v) {
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int NQ>
__global__ __launch_bounds__(256) void sa_reduce16_kernel(const float* __restrict__ y, const float* __restrict__ sc,
                                                          const float* __restrict__ sh, const float* __restrict__ ca,
                                                          int HW, int C, long long P, float* __restrict__ sin_,
                                                          int* __restrict__ sarg) {
    const int lane = threadIdx.x & 63, j = lane & 15, grp = lane >> 4;
    const long long wave = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    CbRegs<NQ> r;
    for (int it = 0; it < CB_QUADS; ++it) {
        const long long p = (wave * CB_QUADS + it) * 4 + grp;
        if (p >= P) break;
        r.load(sc, sh, ca, C, (int)(p / HW), j);
        const float4* yp = reinterpret_cast<const float4*>(y + p * C);
        float sum = 0.f, mx = -INFINITY;
        int am = 0;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const float4 v = yp[q * 16 + j];
            const int c = 4 * (q * 16 + j);
            const float z0 = fmaf(v.x, r.s[q].x, r.b[q].x) * r.a[q].x;
            const float z1 = fmaf(v.y, r.s[q].y, r.b[q].y) * r.a[q].y;
            const float z2 = fmaf(v.z, r.s[q].z, r.b[q].z) * r.a[q].z;
            const float z3 = fmaf(v.w, r.s[q].w, r.b[q].w) * r.a[q].w;
            sum += z0; sum += z1; sum += z2; sum += z3;
            if (z0 > mx) { mx = z0; am = c; }
            if (z1 > mx) { mx = z1; am = c + 1; }
            if (z2 > mx) { mx = z2; am = c + 2; }
            if (z3 > mx) { mx = z3; am = c + 3; }
        }
        sum = row16_sum(sum);
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) {
            const float om = __shfl_xor(mx, o, 64);
            const int oa = __shfl_xor(am, o, 64);
            if (om > mx || (om == mx && oa < am)) { mx = om; am = oa; }
        }
        if (j == 0) {
            reinterpret_cast<float2*>(sin_)[p] = make_float2(sum / (float)C, mx);
            sarg[p] = am;
        }
    }
}

template <int NQ>
__global__ __launch_bounds__(256) void sa_apply16_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                         const float* __restrict__ sc, const float* __restrict__ sh,
                                                         const float* __restrict__ ca, const float* __restrict__ sin_,
                                                         const float* __restrict__ wsa, int H, int W, int C, int ksa,
                                                         long long P, float* __restrict__ sa,
                                                         float* __restrict__ out, float* __restrict__ rng) {
    const int lane = threadIdx.x & 63, j = lane & 15, grp = lane >> 4;
    const long long wave = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int HW = H * W, r = ksa / 2, taps = ksa * ksa;
    CbRegs<NQ> rg;
    float m = 0.f;
    for (int it = 0; it < CB_QUADS; ++it) {
        const long long p = (wave * CB_QUADS + it) * 4 + grp;
        if (p >= P) break;
        const int n = (int)(p / HW);
        const int rem = (int)(p - (long long)n * HW);
        const int py = rem / W, px = rem - py * W;
        float pre = 0.f;
        for (int t = j; t < 2 * taps; t += 16) {
            const int ch = t / taps, tt = t - ch * taps;
            const int ty = tt / ksa, tx = tt - ty * ksa;
            const int yy = py + ty - r, xx = px + tx - r;
            if (yy >= 0 && yy < H && xx >= 0 && xx < W)
                pre = fmaf(wsa[t], sin_[((long long)n * HW + yy * W + xx) * 2 + ch], pre);
        }
        pre = row16_sum(pre);
        const float g = sigmoidf_(pre);
        if (j == 0) sa[p] = g;
        rg.load(sc, sh, ca, C, n, j);
        const float4* yp = reinterpret_cast<const float4*>(y + p * C);
        const float4* xp = reinterpret_cast<const float4*>(x + p * C);
        float4* op = reinterpret_cast<float4*>(out + p * C);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const float4 v = yp[q * 16 + j], xv = xp[q * 16 + j];
            float4 o;
            o.x = xv.x + fmaf(v.x, rg.s[q].x, rg.b[q].x) * rg.a[q].x * g;
            o.y = xv.y + fmaf(v.y, rg.s[q].y, rg.b[q].y) * rg.a[q].y * g;
            o.z = xv.z + fmaf(v.z, rg.s[q].z, rg.b[q].z) * rg.a[q].z * g;
            o.w = xv.w + fmaf(v.w, rg.s[q].w, rg.b[q].w) * rg.a[q].w * g;
            op[q * 16 + j] = o;
            m = fmaxf(m, absmax4(o));
        }
    }
    range_note(rng, m);  // every lane (the pixel loop breaks, never returns)
}

static inline int cb_nq(int C) { return (C == 64 || C == 128 || C == 256) ? C / 64 : 0; }
static inline unsigned cb16_blocks(long long P) { return (unsigned)cdiv(P, 4LL * 4 * CB_QUADS); }

// ---- backward ---------------------------------------------------------------------------
// b1: dpre[p] = (sum_c dout*zc) * sa*(1-sa)
__global__ __launch_bounds__(256) void cb_bwd_dsa_kernel(const float* __restrict__ dout, const float* __restrict__ y,
                                                         const float* __restrict__ sc, const float* __restrict__ sh,
                                                         const float* __restrict__ ca, const float* __restrict__ sa,
                                                         int HW, int C, long long P, float* __restrict__ dpre) {
    const long long p = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (p >= P) return;
    const int n = (int)(p / HW);
    const float* s = sc + (long long)n * C;
    const float* b = sh + (long long)n * C;
    const float* a = ca + (long long)n * C;
    float acc = 0.f;
    for (int c4 = lane; c4 < C / 4; c4 += 64) {
        float4 v = reinterpret_cast<const float4*>(y + p * C)[c4];
        float4 d = reinterpret_cast<const float4*>(dout + p * C)[c4];
        int c = c4 * 4;
        acc = fmaf(d.x, fmaf(v.x, s[c + 0], b[c + 0]) * a[c + 0], acc);
        acc = fmaf(d.y, fmaf(v.y, s[c + 1], b[c + 1]) * a[c + 1], acc);
        acc = fmaf(d.z, fmaf(v.z, s[c + 2], b[c + 2]) * a[c + 2], acc);
        acc = fmaf(d.w, fmaf(v.w, s[c + 3], b[c + 3]) * a[c + 3], acc);
    }
    acc = wave_sum(acc);
    if (lane == 0) {
        float g = sa[p];
        dpre[p] = acc * g * (1.f - g);
    }
}

// b1 for C == 256 (one float4 per lane): a wave takes PX pixels of one image (HW % PX == 0) with its
// lane's scale / shift / attention in registers and every pixel's loads issued together; per pixel
// the same sums in the same order as cb_bwd_dsa_kernel
template <int PX>
__global__ __launch_bounds__(256) void cb_bwd_dsa64x_kernel(const float* __restrict__ dout, const float* __restrict__ y,
                                                            const float* __restrict__ sc, const float* __restrict__ sh,
                                                            const float* __restrict__ ca, const float* __restrict__ sa,
                                                            int HW, long long P, float* __restrict__ dpre) {
    const long long p0 = ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * PX;
    const int lane = threadIdx.x & 63;
    if (p0 >= P) return;  // wave-uniform; P % PX == 0
    const int n = (int)(p0 / HW);
    const float4 s = reinterpret_cast<const float4*>(sc + (long long)n * 256)[lane];
    const float4 b = reinterpret_cast<const float4*>(sh + (long long)n * 256)[lane];
    const float4 a = reinterpret_cast<const float4*>(ca + (long long)n * 256)[lane];
    float4 v[PX], d[PX];
#pragma unroll
    for (int k = 0; k < PX; ++k) {
        v[k] = reinterpret_cast<const float4*>(y + (p0 + k) * 256)[lane];
        d[k] = reinterpret_cast<const float4*>(dout + (p0 + k) * 256)[lane];
    }
#pragma unroll
    for (int k = 0; k < PX; ++k) {
        float acc = 0.f;
        acc = fmaf(d[k].x, fmaf(v[k].x, s.x, b.x) * a.x, acc);
        acc = fmaf(d[k].y, fmaf(v[k].y, s.y, b.y) * a.y, acc);
        acc = fmaf(d[k].z, fmaf(v[k].z, s.z, b.z) * a.z, acc);
        acc = fmaf(d[k].w, fmaf(v[k].w, s.w, b.w) * a.w, acc);
        acc = wave_sum(acc);
        if (lane == 0) {
            const float g = sa[p0 + k];
            dpre[p0 + k] = acc * g * (1.f - g);
        }
    }
}

// b1 + the dout half of b3, for C == 256: grid (image, chunk) over b3's pixel chunks; each wave walks
// its plane's pixels of the chunk (PX at a time, every load issued together) and writes dpre[p] as
// cb_bwd_dsa64x_kernel (same sums in the same order), while accumulating per channel the part of b3's
// sums that needs dout: sum (dout g) z and sum dout g (g = sa), folded over the four planes in fixed
// order into p1[n][chunk][c].  cb_bwd_sums4_kernel<true> then adds the dsin half reading y but not
// dout, so the pair reads dout once (b1 and b3 each read it before)
template <int PX>
__global__ __launch_bounds__(256) void cb_bwd_dsa_sums_kernel(const float* __restrict__ dout, const float* __restrict__ y,
                                                              const float* __restrict__ sc, const float* __restrict__ sh,
                                                              const float* __restrict__ ca, const float* __restrict__ sa,
                                                              int HW, int nchunk, float* __restrict__ dpre,
                                                              Sum2* __restrict__ p1) {
    __shared__ float4 s_a[256], s_b[256];
    const int n = blockIdx.x, chunk = blockIdx.y, tid = threadIdx.x;
    const int lane = tid & 63, plane = tid >> 6;
    const int p_per = (HW + nchunk - 1) / nchunk;
    const int p0 = chunk * p_per;
    const int pend = min(HW, p0 + p_per);
    const float4 s = reinterpret_cast<const float4*>(sc + (long long)n * 256)[lane];
    const float4 b = reinterpret_cast<const float4*>(sh + (long long)n * 256)[lane];
    const float4 a = reinterpret_cast<const float4*>(ca + (long long)n * 256)[lane];
    float4 A = make_float4(0.f, 0.f, 0.f, 0.f), B = A;
    const long long base = (long long)n * HW;
    for (int p = p0 + plane; p < pend; p += 4 * PX) {
        float4 v[PX], d[PX];
        float gg[PX];
#pragma unroll
        for (int k = 0; k < PX; ++k) {  // pixels past the chunk: a clamped repeat, masked below
            const int pk = p + 4 * k < pend ? p + 4 * k : pend - 1;
            v[k] = reinterpret_cast<const float4*>(y + (base + pk) * 256)[lane];
            d[k] = reinterpret_cast<const float4*>(dout + (base + pk) * 256)[lane];
            gg[k] = sa[base + pk];
        }
#pragma unroll
        for (int k = 0; k < PX; ++k) {
            const bool ok = p + 4 * k < pend;  // (wave-uniform)
            const float zx = fmaf(v[k].x, s.x, b.x), zy = fmaf(v[k].y, s.y, b.y);
            const float zz = fmaf(v[k].z, s.z, b.z), zw = fmaf(v[k].w, s.w, b.w);
            float acc = 0.f;
            acc = fmaf(d[k].x, zx * a.x, acc);
            acc = fmaf(d[k].y, zy * a.y, acc);
            acc = fmaf(d[k].z, zz * a.z, acc);
            acc = fmaf(d[k].w, zw * a.w, acc);
            acc = wave_sum(acc);
            if (ok) {
                if (lane == 0) dpre[base + p + 4 * k] = acc * gg[k] * (1.f - gg[k]);
                const float g = gg[k];
                const float dx = d[k].x * g, dy_ = d[k].y * g, dz = d[k].z * g, dw = d[k].w * g;
                A.x = fmaf(dx, zx, A.x); A.y = fmaf(dy_, zy, A.y); A.z = fmaf(dz, zz, A.z); A.w = fmaf(dw, zw, A.w);
                B.x += dx; B.y += dy_; B.z += dz; B.w += dw;
            }
        }
    }
    s_a[tid] = A;
    s_b[tid] = B;
    __syncthreads();
    if (plane == 0) {
#pragma unroll
        for (int l = 1; l < 4; ++l) {
            const float4 u = s_a[l * 64 + lane], w = s_b[l * 64 + lane];
            A.x += u.x; A.y += u.y; A.z += u.z; A.w += u.w;
            B.x += w.x; B.y += w.y; B.z += w.z; B.w += w.w;
        }
        Sum2* o = p1 + ((long long)n * nchunk + chunk) * 256 + 4 * lane;
        o[0] = Sum2{A.x, B.x};
        o[1] = Sum2{A.y, B.y};
        o[2] = Sum2{A.z, B.z};
        o[3] = Sum2{A.w, B.w};
    }
}

// b2: dsin[q][ch] = sum_t wsa[ch][t] * dpre[q - (t - r)]  (adjoint of the zero-padded conv)
__global__ void cb_bwd_dsin_kernel(const float* __restrict__ dpre, const float* __restrict__ wsa, int H, int W, int ksa,
                                   long long P, float* __restrict__ dsin) {
    const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= P) return;
    const int HW = H * W;
    const int n = (int)(q / HW);
    const int rem = (int)(q - (long long)n * HW);
    const int qy = rem / W, qx = rem - qy * W;
    const int r = ksa / 2, taps = ksa * ksa;
    float a0 = 0.f, a1 = 0.f;
    for (int ty = 0; ty < ksa; ++ty) {
        int yy = qy - ty + r;
        if (yy < 0 || yy >= H) continue;
        for (int tx = 0; tx < ksa; ++tx) {
            int xx = qx - tx + r;
            if (xx < 0 || xx >= W) continue;
            float d = dpre[(long long)n * HW + yy * W + xx];
            a0 = fmaf(wsa[ty * ksa + tx], d, a0);
            a1 = fmaf(wsa[taps + ty * ksa + tx], d, a1);
        }
    }
    dsin[q * 2 + 0] = a0;
    dsin[q * 2 + 1] = a1;
}

// dwsa partials: grid (2*taps, nchunk); part[chunk][t] = sum_{p in chunk} dpre[p]*sin[p+t-r][ch]
__global__ __launch_bounds__(256) void cb_bwd_dwsa_partial_kernel(const float* __restrict__ dpre,
                                                                  const float* __restrict__ sin_, int H, int W,
                                                                  int ksa, long long P, int nchunk,
                                                                  float* __restrict__ part) {
    __shared__ float red[4];
    const int t = blockIdx.x, chunk = blockIdx.y;
    const int taps = ksa * ksa, r = ksa / 2;
    const int ch = t / taps, tt = t - ch * taps;
    const int ty = tt / ksa, tx = tt - ty * ksa;
    // 32-bit pixel index math (the host guarantees P < 2^31)
    const int per = (int)((P + nchunk - 1) / nchunk);
    const int p0 = chunk * per, p1 = (int)min(P, (long long)p0 + per);
    const int HW = H * W;
    float acc = 0.f;
#pragma unroll 4
    for (int p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
        const int n = p / HW;
        const int rem = p - n * HW;
        const int py = rem / W, px = rem - py * W;
        const int yy = py + ty - r, xx = px + tx - r;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W)
            acc = fmaf(dpre[p], sin_[(n * HW + yy * W + xx) * 2 + ch], acc);
    }
    acc = block_sum_256(acc, red);
    if (threadIdx.x == 0) part[(long long)chunk * gridDim.x + t] = acc;
}

__global__ void cb_bwd_dwsa_final_kernel(const float* __restrict__ part, int nt, int nchunk, float* __restrict__ dwsa) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nt) return;
    double s = 0.0;
#pragma unroll DCS_SERIAL_UNROLL
    for (int k = 0; k < nchunk; ++k) s += part[(long long)k * nt + t];
    dwsa[t] = (float)s;
}

struct Sum3 {
    float a, b, c;
};

// b3: per (n,c) sums over pixels of dzc*z, dz0, dz0*z
__global__ __launch_bounds__(256) void cb_bwd_sums_kernel(const float* __restrict__ dout, const float* __restrict__ y,
                                                          const float* __restrict__ sc, const float* __restrict__ sh,
                                                          const float* __restrict__ ca, const float* __restrict__ sa,
                                                          const float* __restrict__ dsin,
                                                          const int* __restrict__ sarg, int HW, int C, int nchunk,
                                                          Sum3* __restrict__ parts) {
    const int n = blockIdx.x, chunk = blockIdx.y, tid = threadIdx.x;
    const int p_per = (HW + nchunk - 1) / nchunk;
    const int p0 = chunk * p_per;
    const int p1 = min(HW, p0 + p_per);
    const bool packed = (C <= 256) && (256 % C == 0);
    const int lanes = packed ? 256 / C : 1;
    const int plane = packed ? tid / C : 0;
    __shared__ float s_a[256], s_b[256], s_c[256];
    const float invC = 1.f / (float)C;
    for (int cbase = 0; cbase < C; cbase += (packed ? C : 256)) {
        const int c = packed ? (tid % C) : (cbase + tid);
        float A = 0.f, B = 0.f, Cc = 0.f;
        if (c < C) {
            const long long nc = (long long)n * C + c;
            const float s = sc[nc], b = sh[nc], a = ca[nc];
            for (int p = p0 + plane; p < p1; p += lanes) {
                const long long pp = (long long)n * HW + p;
                const long long o = pp * C + c;
                float z = fmaf(y[o], s, b);
                float dzc = fmaf(dout[o], sa[pp], dsin[pp * 2] * invC);
                if (sarg[pp] == c) dzc += dsin[pp * 2 + 1];
                float dz0 = dzc * a;
                A = fmaf(dzc, z, A);
                B += dz0;
                Cc = fmaf(dz0, z, Cc);
            }
        }
        if (packed) {
            s_a[tid] = A; s_b[tid] = B; s_c[tid] = Cc;
            __syncthreads();
            if (plane == 0) {
                for (int l = 1; l < lanes; ++l) { A += s_a[l * C + c]; B += s_b[l * C + c]; Cc += s_c[l * C + c]; }
                parts[((long long)n * nchunk + chunk) * C + c] = Sum3{A, B, Cc};
            }
            __syncthreads();
        } else if (c < C) {
            parts[((long long)n * nchunk + chunk) * C + c] = Sum3{A, B, Cc};
        }
    }
}

// b3 (float4 form, C % 4 == 0 and C/4 dividing 256): thread t owns channels 4*(t % C4).. of
// pixel lane t / C4; a wave reads whole pixel rows (C = 256: one 1 KiB row per load), the
// pixel lanes are folded in fixed order through LDS.  Same sums as cb_bwd_sums_kernel.
// HALF: the dsin half only (no dout read), plus the dout half cb_bwd_dsa_sums_kernel left in p1
template <bool HALF>
__global__ __launch_bounds__(256) void cb_bwd_sums4_kernel(const float* __restrict__ dout, const float* __restrict__ y,
                                                           const float* __restrict__ sc, const float* __restrict__ sh,
                                                           const float* __restrict__ ca, const float* __restrict__ sa,
                                                           const float* __restrict__ dsin,
                                                           const int* __restrict__ sarg, int HW, int C, int nchunk,
                                                           Sum3* __restrict__ parts, const Sum2* __restrict__ p1) {
    __shared__ float4 s_a[256], s_b[256], s_c[256];
    const int n = blockIdx.x, chunk = blockIdx.y, tid = threadIdx.x;
    const int C4 = C >> 2, lanes = 256 / C4;
    const int c4 = tid % C4, plane = tid / C4;
    const int p_per = (HW + nchunk - 1) / nchunk;
    const int p0 = chunk * p_per;
    const int pend = min(HW, p0 + p_per);
    const int nc = n * C + 4 * c4;
    const float4 s = *reinterpret_cast<const float4*>(sc + nc);
    const float4 b = *reinterpret_cast<const float4*>(sh + nc);
    const float4 a = *reinterpret_cast<const float4*>(ca + nc);
    const float invC = 1.f / (float)C;
    float4 A = make_float4(0.f, 0.f, 0.f, 0.f), B = A, Cc = A;
    for (int p = p0 + plane; p < pend; p += lanes) {
        const long long pp = (long long)n * HW + p;
        const float4 yv = reinterpret_cast<const float4*>(y + pp * C)[c4];
        const float2 ds = reinterpret_cast<const float2*>(dsin)[pp];
        const int am = sarg[pp] - 4 * c4;
        const float d0 = ds.x * invC;
        float z, dzc, dz0;
        if constexpr (HALF) {  // A: sum dzc z, B: sum dzc (times the attention after the fold)
#define DCS_SUMS_LANE(X, K)                                   \
        z = fmaf(yv.X, s.X, b.X);                             \
        dzc = d0;                                             \
        if (am == K) dzc += ds.y;                             \
        A.X = fmaf(dzc, z, A.X);                              \
        B.X += dzc;
            DCS_SUMS_LANE(x, 0)
            DCS_SUMS_LANE(y, 1)
            DCS_SUMS_LANE(z, 2)
            DCS_SUMS_LANE(w, 3)
#undef DCS_SUMS_LANE
        } else {
            const float4 dv = reinterpret_cast<const float4*>(dout + pp * C)[c4];
            const float g = sa[pp];
#define DCS_SUMS_LANE(X, K)                                   \
        z = fmaf(yv.X, s.X, b.X);                             \
        dzc = fmaf(dv.X, g, d0);                              \
        if (am == K) dzc += ds.y;                             \
        dz0 = dzc * a.X;                                      \
        A.X = fmaf(dzc, z, A.X);                              \
        B.X += dz0;                                           \
        Cc.X = fmaf(dz0, z, Cc.X);
            DCS_SUMS_LANE(x, 0)
            DCS_SUMS_LANE(y, 1)
            DCS_SUMS_LANE(z, 2)
            DCS_SUMS_LANE(w, 3)
#undef DCS_SUMS_LANE
        }
    }
    s_a[tid] = A; s_b[tid] = B; s_c[tid] = Cc;
    __syncthreads();
    if (plane == 0) {
        for (int l = 1; l < lanes; ++l) {
            const float4 u = s_a[l * C4 + c4], v = s_b[l * C4 + c4], w = s_c[l * C4 + c4];
            A.x += u.x; A.y += u.y; A.z += u.z; A.w += u.w;
            B.x += v.x; B.y += v.y; B.z += v.z; B.w += v.w;
            Cc.x += w.x; Cc.y += w.y; Cc.z += w.z; Cc.w += w.w;
        }
        Sum3* o = parts + ((long long)n * nchunk + chunk) * C + 4 * c4;
        if constexpr (HALF) {  // + the dout half; B = a sum dzc, Cc = a sum dzc z
            const Sum2* q = p1 + ((long long)n * nchunk + chunk) * C + 4 * c4;
            const float ax = A.x + q[0].a, ay = A.y + q[1].a, az = A.z + q[2].a, aw = A.w + q[3].a;
            o[0] = Sum3{ax, a.x * (B.x + q[0].b), a.x * ax};
            o[1] = Sum3{ay, a.y * (B.y + q[1].b), a.y * ay};
            o[2] = Sum3{az, a.z * (B.z + q[2].b), a.z * az};
            o[3] = Sum3{aw, a.w * (B.w + q[3].b), a.w * aw};
        } else {
            o[0] = Sum3{A.x, B.x, Cc.x};
            o[1] = Sum3{A.y, B.y, Cc.y};
            o[2] = Sum3{A.z, B.z, Cc.z};
            o[3] = Sum3{A.w, B.w, Cc.w};
        }
    }
}

// b4: one block per image: channel-attention MLP backward + IN-backward coefficients.
// coef[n][c] = {mean(dz), mean(dz*z), dvmax}; per-image dw1/dw2 partials (summed over n by
// cb_bwd_dw_reduce_kernel in fixed order).
__global__ __launch_bounds__(256) void cb_bwd_ca_kernel(const Sum3* __restrict__ parts, int nchunk,
                                                        const float* __restrict__ ymax, const float* __restrict__ sc,
                                                        const float* __restrict__ sh, const float* __restrict__ ca,
                                                        const float* __restrict__ w1, const float* __restrict__ w2,
                                                        int HW, int C, int Cr, Sum3* __restrict__ coef,
                                                        float* __restrict__ dwpart) {
    extern __shared__ float sm[];
    float* vmax = sm;            // [C]
    float* dpc = vmax + C;       // [C] d(pre-sigmoid)
    float* hp = dpc + C;         // [Cr] W1 vmax (pre-relu)
    float* dhm = hp + Cr;        // [Cr]
    float* S1 = dhm + Cr;        // [C] sum dz0
    float* S2 = S1 + C;          // [C] sum dz0*z
    __shared__ float red[2][4];
    const int tid = threadIdx.x, n = blockIdx.x;
    for (int c = tid; c < C; c += blockDim.x) {
        const long long nc = (long long)n * C + c;
        double A = 0.0, B = 0.0, Cc = 0.0;
#pragma unroll DCS_SERIAL_UNROLL
        for (int k = 0; k < nchunk; ++k) {
            Sum3 p = parts[((long long)n * nchunk + k) * C + c];
            A += p.a; B += p.b; Cc += p.c;
        }
        vmax[c] = fmaf(ymax[nc], sc[nc], sh[nc]);
        float g = ca[nc];
        dpc[c] = (float)A * g * (1.f - g);
        S1[c] = (float)B;
        S2[c] = (float)Cc;
    }
    __syncthreads();
    for (int j = 0; j < Cr; ++j) {
        float a = 0.f, b = 0.f;
        for (int c = tid; c < C; c += blockDim.x) {
            a = fmaf(w1[j * C + c], vmax[c], a);
            b = fmaf(w2[c * Cr + j], dpc[c], b);
        }
        a = wave_sum(a);
        b = wave_sum(b);
        if ((tid & 63) == 0) { red[0][tid >> 6] = a; red[1][tid >> 6] = b; }
        __syncthreads();
        if (tid == 0) {
            float hpre = red[0][0] + red[0][1] + red[0][2] + red[0][3];
            float dh = red[1][0] + red[1][1] + red[1][2] + red[1][3];
            hp[j] = hpre;
            dhm[j] = hpre > 0.f ? dh : 0.f;   // avg branch: relu'(0) = 0 -> no gradient
        }
        __syncthreads();
    }
    float* dw1 = dwpart + (long long)n * 2 * C * Cr;
    float* dw2 = dw1 + (long long)C * Cr;
    const float inv = 1.f / (float)HW;
    for (int c = tid; c < C; c += blockDim.x) {
        float dvm = 0.f;
        for (int j = 0; j < Cr; ++j) {
            dvm = fmaf(w1[j * C + c], dhm[j], dvm);
            dw2[c * Cr + j] = dpc[c] * (hp[j] > 0.f ? hp[j] : 0.f);
            dw1[j * C + c] = dhm[j] * vmax[c];
        }
        // dz = dz0 + dvmax * [p == argmax]; sum_p z = 0 (IN output), z[argmax] = vmax
        coef[(long long)n * C + c] = Sum3{(S1[c] + dvm) * inv, (S2[c] + dvm * vmax[c]) * inv, dvm};
    }
}

__global__ void cb_bwd_dw_reduce_kernel(const float* __restrict__ dwpart, int N, int CCr, float* __restrict__ dw1,
                                        float* __restrict__ dw2) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 2 * CCr) return;
    float s = 0.f;
#pragma unroll DCS_SERIAL_UNROLL
    for (int n = 0; n < N; ++n) s += dwpart[(long long)n * 2 * CCr + i];
    if (i < CCr) dw1[i] = s;
    else dw2[i - CCr] = s;
}

// b5: dy = scale*(dz - mean(dz) - z*mean(dz*z))
__global__ void cb_bwd_apply_kernel(const float* __restrict__ dout, const float* __restrict__ y,
                                    const float* __restrict__ sc, const float* __restrict__ sh,
                                    const float* __restrict__ ca, const float* __restrict__ sa,
                                    const float* __restrict__ dsin, const int* __restrict__ sarg,
                                    const int* __restrict__ yarg, const Sum3* __restrict__ coef, int HW, int C,
                                    long long total, float* __restrict__ dy, float* __restrict__ rng) {
    const long long i0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i0 < total;
    const long long i = live ? i0 : total - 1;  // dead lanes recompute the last element, store nothing
    const int c = (int)(i % C);
    const long long pp = i / C;
    const int n = (int)(pp / HW);
    const int p = (int)(pp - (long long)n * HW);
    const long long nc = (long long)n * C + c;
    const float s = sc[nc], b = sh[nc];
    const float z = fmaf(y[i], s, b);
    float dzc = fmaf(dout[i], sa[pp], dsin[pp * 2] * (1.f / (float)C));
    if (sarg[pp] == c) dzc += dsin[pp * 2 + 1];
    const Sum3 k = coef[nc];
    float dz = dzc * ca[nc];
    if (yarg[nc] == p) dz += k.c;
    const float v = s * (dz - k.a - z * k.b);
    if (live) dy[i] = v;
    range_note(rng, fabsf(v));  // every lane
}

// b5, float4 form (C % 4 == 0): one thread per 4 channels of a pixel, 32-bit index math
__global__ __launch_bounds__(256) void cb_bwd_apply4_kernel(const float* __restrict__ dout, const float* __restrict__ y,
                                                            const float* __restrict__ sc, const float* __restrict__ sh,
                                                            const float* __restrict__ ca, const float* __restrict__ sa,
                                                            const float* __restrict__ dsin, const int* __restrict__ sarg,
                                                            const int* __restrict__ yarg, const Sum3* __restrict__ coef,
                                                            int HW, int C, int total4, float* __restrict__ dy,
                                                            float* __restrict__ rng) {
    const int i40 = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i40 < total4;
    const int i4 = live ? i40 : total4 - 1;  // dead lanes recompute the last float4, store nothing
    const int C4 = C >> 2;
    const int pp = i4 / C4;
    const int c4 = i4 - pp * C4;
    const int n = pp / HW;
    const int p = pp - n * HW;
    const int nc = n * C + 4 * c4;
    const float4 s = *reinterpret_cast<const float4*>(sc + nc);
    const float4 b = *reinterpret_cast<const float4*>(sh + nc);
    const float4 a = *reinterpret_cast<const float4*>(ca + nc);
    const int4 ya = *reinterpret_cast<const int4*>(yarg + nc);
    const float4 k0 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(coef + nc));
    const float4 k1 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(coef + nc) + 4);
    const float4 k2 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(coef + nc) + 8);
    const float4 yv = reinterpret_cast<const float4*>(y)[i4];
    const float4 dv = reinterpret_cast<const float4*>(dout)[i4];
    const float g = sa[pp];
    const float2 ds = reinterpret_cast<const float2*>(dsin)[pp];
    const int am = sarg[pp] - 4 * c4;
    const float d0 = ds.x * (1.f / (float)C);
    float4 o;
    // coef of channel j: {k.a, k.b, k.c} = floats 3j..3j+2 of (k0, k1, k2)
#define DCS_APPLY_LANE(X, K, KA, KB, KC)                      \
    {                                                         \
        const float z = fmaf(yv.X, s.X, b.X);                 \
        float dzc = fmaf(dv.X, g, d0);                        \
        if (am == K) dzc += ds.y;                             \
        float dz = dzc * a.X;                                 \
        if (ya.X == p) dz += KC;                              \
        o.X = s.X * (dz - KA - z * KB);                       \
    }
    DCS_APPLY_LANE(x, 0, k0.x, k0.y, k0.z)
    DCS_APPLY_LANE(y, 1, k0.w, k1.x, k1.y)
    DCS_APPLY_LANE(z, 2, k1.z, k1.w, k2.x)
    DCS_APPLY_LANE(w, 3, k2.y, k2.z, k2.w)
#undef DCS_APPLY_LANE
    if (live) reinterpret_cast<float4*>(dy)[i4] = o;
    range_note(rng, absmax4(o));  // every lane
}

// b5, multi-pixel float4 form (256 % (C / 4) == 0, the block's PX * 256 / (C / 4) pixels inside one image):
// a thread keeps its 4 channels' tables (scale, shift, channel attention, argmax, coefficients) in
// registers over PX pixels, so the per-image table loads and the range atomics drop by PX against
// cb_bwd_apply4_kernel; the same arithmetic per element
template <int PX>
__global__ __launch_bounds__(256) void cb_bwd_apply4x_kernel(const float* __restrict__ dout, const float* __restrict__ y,
                                                             const float* __restrict__ sc, const float* __restrict__ sh,
                                                             const float* __restrict__ ca, const float* __restrict__ sa,
                                                             const float* __restrict__ dsin, const int* __restrict__ sarg,
                                                             const int* __restrict__ yarg, const Sum3* __restrict__ coef,
                                                             int HW, int C, float* __restrict__ dy, float* __restrict__ rng) {
    const int C4 = C >> 2;
    const int ppb = 256 / C4;  // pixels per pass
    const int c4 = threadIdx.x % C4, pl = threadIdx.x / C4;
    const int pp0 = blockIdx.x * ppb * PX;
    const int n = pp0 / HW;
    const int nc = n * C + 4 * c4;
    const float4 s = *reinterpret_cast<const float4*>(sc + nc);
    const float4 b = *reinterpret_cast<const float4*>(sh + nc);
    const float4 a = *reinterpret_cast<const float4*>(ca + nc);
    const int4 ya = *reinterpret_cast<const int4*>(yarg + nc);
    const float4 k0 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(coef + nc));
    const float4 k1 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(coef + nc) + 4);
    const float4 k2 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(coef + nc) + 8);
    const float rC = 1.f / (float)C;
    float m = 0.f;
#pragma unroll
    for (int k = 0; k < PX; ++k) {
        const int pp = pp0 + k * ppb + pl;
        const int p = pp - n * HW;
        const int i4 = pp * C4 + c4;
        const float4 yv = reinterpret_cast<const float4*>(y)[i4];
        const float4 dv = reinterpret_cast<const float4*>(dout)[i4];
        const float g = sa[pp];
        const float2 ds = reinterpret_cast<const float2*>(dsin)[pp];
        const int am = sarg[pp] - 4 * c4;
        const float d0 = ds.x * rC;
        float4 o;
#define DCS_APPLY_LANE(X, K, KA, KB, KC)                      \
    {                                                         \
        const float z = fmaf(yv.X, s.X, b.X);                 \
        float dzc = fmaf(dv.X, g, d0);                        \
        if (am == K) dzc += ds.y;                             \
        float dz = dzc * a.X;                                 \
        if (ya.X == p) dz += KC;                              \
        o.X = s.X * (dz - KA - z * KB);                       \
    }
        DCS_APPLY_LANE(x, 0, k0.x, k0.y, k0.z)
        DCS_APPLY_LANE(y, 1, k0.w, k1.x, k1.y)
        DCS_APPLY_LANE(z, 2, k1.z, k1.w, k2.x)
        DCS_APPLY_LANE(w, 3, k2.y, k2.z, k2.w)
#undef DCS_APPLY_LANE
        reinterpret_cast<float4*>(dy)[i4] = o;
        m = fmaxf(m, absmax4(o));
    }
    range_note(rng, m);
}

static inline int cb_chunks(int N, int HW) {
    int want = (int)cdiv(1024, N);
    int maxc = (int)cdiv(HW, 64);
    int c = want < maxc ? want : maxc;
    return c < 1 ? 1 : c;
}
static inline int sa_wchunks(long long P) {
    long long c = cdiv(P, 4096);
    if (c < 1) c = 1;
    if (c > 64) c = 64;
    return (int)c;
}

struct CbWs {
    float* dpre;
    float* dsin;
    float* wpart;
    Sum3* parts;
    Sum2* p1;  // dout half of the b3 sums (cb_bwd_dsa_sums_kernel)
    Sum3* coef;
    float* dwpart;
    size_t total;
};
static CbWs cb_layout(void* base, int N, int H, int W, int C, int Cr, int ksa) {
    CbWs w;
    long long P = (long long)N * H * W;
    size_t off = 0;
    char* b = reinterpret_cast<char*>(base);
    w.dpre = reinterpret_cast<float*>(b + off); off = align_up(off + P * sizeof(float), 256);
    w.dsin = reinterpret_cast<float*>(b + off); off = align_up(off + 2 * P * sizeof(float), 256);
    w.wpart = reinterpret_cast<float*>(b + off); off = align_up(off + (size_t)sa_wchunks(P) * 2 * ksa * ksa * sizeof(float), 256);
    int nch = cb_chunks(N, H * W);
    w.parts = reinterpret_cast<Sum3*>(b + off); off = align_up(off + (size_t)N * nch * C * sizeof(Sum3), 256);
    w.p1 = reinterpret_cast<Sum2*>(b + off); off = align_up(off + (size_t)N * nch * C * sizeof(Sum2), 256);
    w.coef = reinterpret_cast<Sum3*>(b + off); off = align_up(off + (size_t)N * C * sizeof(Sum3), 256);
    w.dwpart = reinterpret_cast<float*>(b + off); off = align_up(off + (size_t)N * 2 * C * Cr * sizeof(float), 256);
    w.total = off;
    return w;
}

}  // namespace dcs

using namespace dcs;

extern "C" int dcs_cbam_forward(const float* x, const float* y, const float* scale, const float* shift,
                                const float* ymax, const float* w1, const float* w2, const float* wsa, int N, int H,
                                int W, int C, int Cr, int ksa, float* ca, float* sin_, int32_t* sarg, float* sa,
                                float* out, float* rng, void* stream) {
    if (!x || !y || !scale || !shift || !ymax || !w1 || !w2 || !wsa || !ca || !sin_ || !sarg || !sa || !out)
        return fail(DCS_E_INVALID, "cbam_forward: null pointer");
    if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 4 != 0 || Cr <= 0 || ksa <= 0 || (ksa & 1) == 0)
        return fail(DCS_E_INVALID, "cbam_forward: bad dims");
    hipStream_t s = as_stream(stream);
    long long P = (long long)N * H * W;
    hipLaunchKernelGGL(ca_forward_kernel, dim3(N), dim3(256), (size_t)(C + 2 * Cr) * sizeof(float), s, ymax, scale,
                       shift, w1, w2, C, Cr, ca);
    int e = check_launch("ca_forward");
    if (e) return e;
    const int nq = cb_nq(C);
#define DCS_CB16(K, NQ, ...) hipLaunchKernelGGL((K<NQ>), dim3(cb16_blocks(P)), dim3(256), 0, s, __VA_ARGS__)
    if (nq == 4) DCS_CB16(sa_reduce16_kernel, 4, y, scale, shift, ca, H * W, C, P, sin_, sarg);
    else if (nq == 2) DCS_CB16(sa_reduce16_kernel, 2, y, scale, shift, ca, H * W, C, P, sin_, sarg);
    else if (nq == 1) DCS_CB16(sa_reduce16_kernel, 1, y, scale, shift, ca, H * W, C, P, sin_, sarg);
    else hipLaunchKernelGGL(sa_reduce_kernel, dim3((unsigned)cdiv(P, 4)), dim3(256), 0, s, y, scale, shift, ca, H * W, C,
                            P, sin_, sarg);
    e = check_launch("sa_reduce");
    if (e) return e;
    if ((e = range_zero(rng, s))) return e;
    if (nq == 4) DCS_CB16(sa_apply16_kernel, 4, x, y, scale, shift, ca, sin_, wsa, H, W, C, ksa, P, sa, out, rng);
    else if (nq == 2) DCS_CB16(sa_apply16_kernel, 2, x, y, scale, shift, ca, sin_, wsa, H, W, C, ksa, P, sa, out, rng);
    else if (nq == 1) DCS_CB16(sa_apply16_kernel, 1, x, y, scale, shift, ca, sin_, wsa, H, W, C, ksa, P, sa, out, rng);
    else hipLaunchKernelGGL(sa_apply_kernel, dim3((unsigned)cdiv(P, 4)), dim3(256), 0, s, x, y, scale, shift, ca, sin_,
                            wsa, H, W, C, ksa, P, sa, out, rng);
    return check_launch("sa_apply");
}

extern "C" size_t dcs_cbam_backward_workspace_size(int N, int H, int W, int C, int Cr, int ksa) {
    if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || Cr <= 0 || ksa <= 0) return 0;
    return cb_layout(nullptr, N, H, W, C, Cr, ksa).total;
}

extern "C" int dcs_cbam_backward(const float* dout, const float* y, const float* scale, const float* shift,
                                 const float* ymax, const int32_t* yargmax, const float* w1, const float* w2,
                                 const float* wsa, const float* ca, const float* sin_, const int32_t* sarg,
                                 const float* sa, int N, int H, int W, int C, int Cr, int ksa, float* dy, float* dw1,
                                 float* dw2, float* dwsa, void* ws, size_t ws_bytes, float* rng, void* stream) {
    if (!dout || !y || !scale || !shift || !ymax || !yargmax || !w1 || !w2 || !wsa || !ca || !sin_ || !sarg || !sa ||
        !dy || !dw1 || !dw2 || !dwsa || !ws)
        return fail(DCS_E_INVALID, "cbam_backward: null pointer");
    if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 4 != 0 || Cr <= 0 || ksa <= 0)
        return fail(DCS_E_INVALID, "cbam_backward: bad dims");
    if (ws_bytes < dcs_cbam_backward_workspace_size(N, H, W, C, Cr, ksa))
        return fail(DCS_E_WORKSPACE, "cbam_backward: workspace too small");
    if ((long long)N * H * W * 2 >= (1LL << 31))
        return fail(DCS_E_INVALID, "cbam_backward: N*H*W*2 must fit in 31 bits");
    CbWs w = cb_layout(ws, N, H, W, C, Cr, ksa);
    hipStream_t s = as_stream(stream);
    const long long P = (long long)N * H * W;
    const int HW = H * W;
    // one wave per pixel: the 16-lane form (4 pixels per wave, 4 quads per wave) measured 104 vs
    // 96 us per 16-image launch here (a read-only pass wants more loads in flight per wave)
    constexpr int DPX = 4;  // pixels per wave of the C == 256 form
    const int nch = cb_chunks(N, HW);
    const bool fused = C == 256;  // b1 with the dout half of b3 (cb_bwd_dsa_sums_kernel)
    if (fused)
        hipLaunchKernelGGL(cb_bwd_dsa_sums_kernel<DPX>, dim3(N, nch), dim3(256), 0, s, dout, y, scale, shift, ca, sa, HW,
                           nch, w.dpre, w.p1);
    else if (C == 256 && HW % DPX == 0)
        hipLaunchKernelGGL(cb_bwd_dsa64x_kernel<DPX>, dim3((unsigned)cdiv(P, 4 * DPX)), dim3(256), 0, s, dout, y, scale,
                           shift, ca, sa, HW, P, w.dpre);
    else
        hipLaunchKernelGGL(cb_bwd_dsa_kernel, dim3((unsigned)cdiv(P, 4)), dim3(256), 0, s, dout, y, scale, shift, ca, sa,
                           HW, C, P, w.dpre);
    int e = check_launch("cb_bwd_dsa");
    if (e) return e;
    hipLaunchKernelGGL(cb_bwd_dsin_kernel, dim3((unsigned)cdiv(P, 256)), dim3(256), 0, s, w.dpre, wsa, H, W, ksa, P,
                       w.dsin);
    if ((e = check_launch("cb_bwd_dsin"))) return e;
    const int nt = 2 * ksa * ksa, nwc = sa_wchunks(P);
    hipLaunchKernelGGL(cb_bwd_dwsa_partial_kernel, dim3(nt, nwc), dim3(256), 0, s, w.dpre, sin_, H, W, ksa, P, nwc,
                       w.wpart);
    if ((e = check_launch("cb_bwd_dwsa_partial"))) return e;
    hipLaunchKernelGGL(cb_bwd_dwsa_final_kernel, dim3((unsigned)cdiv(nt, 128)), dim3(128), 0, s, w.wpart, nt, nwc, dwsa);
    if ((e = check_launch("cb_bwd_dwsa_final"))) return e;
    const bool v4 = (C % 4 == 0) && (C / 4 <= 256) && (256 % (C / 4) == 0);
    if (fused)
        hipLaunchKernelGGL(cb_bwd_sums4_kernel<true>, dim3(N, nch), dim3(256), 0, s, dout, y, scale, shift, ca, sa, w.dsin,
                           sarg, HW, C, nch, w.parts, w.p1);
    else if (v4)
        hipLaunchKernelGGL(cb_bwd_sums4_kernel<false>, dim3(N, nch), dim3(256), 0, s, dout, y, scale, shift, ca, sa, w.dsin,
                           sarg, HW, C, nch, w.parts, nullptr);
    else
        hipLaunchKernelGGL(cb_bwd_sums_kernel, dim3(N, nch), dim3(256), 0, s, dout, y, scale, shift, ca, sa, w.dsin,
                           sarg, HW, C, nch, w.parts);
    if ((e = check_launch("cb_bwd_sums"))) return e;
    hipLaunchKernelGGL(cb_bwd_ca_kernel, dim3(N), dim3(256), (size_t)(4 * C + 2 * Cr) * sizeof(float), s, w.parts, nch,
                       ymax, scale, shift, ca, w1, w2, HW, C, Cr, w.coef, w.dwpart);
    if ((e = check_launch("cb_bwd_ca"))) return e;
    hipLaunchKernelGGL(cb_bwd_dw_reduce_kernel, dim3((unsigned)cdiv(2LL * C * Cr, 256)), dim3(256), 0, s, w.dwpart, N,
                       C * Cr, dw1, dw2);
    if ((e = check_launch("cb_bwd_dw_reduce"))) return e;
    if ((e = range_zero(rng, s))) return e;
    const long long total = P * C;
    const int C4 = C / 4;
    constexpr int APX = 4;  // pixels per thread of the multi-pixel apply
    if (total / 4 < (1LL << 31) && (long long)N * C < (1LL << 31) && C4 <= 256 && 256 % C4 == 0 &&
        HW % (APX * (256 / C4)) == 0) {
        hipLaunchKernelGGL(cb_bwd_apply4x_kernel<APX>, dim3((unsigned)(P / (APX * (256 / C4)))), dim3(256), 0, s, dout,
                           y, scale, shift, ca, sa, w.dsin, sarg, yargmax, w.coef, HW, C, dy, rng);
    } else if (total / 4 < (1LL << 31) && (long long)N * C < (1LL << 31)) {  // C % 4 == 0 checked above
        const int total4 = (int)(total / 4);
        hipLaunchKernelGGL(cb_bwd_apply4_kernel, dim3((unsigned)cdiv(total4, 256)), dim3(256), 0, s, dout, y, scale,
                           shift, ca, sa, w.dsin, sarg, yargmax, w.coef, HW, C, total4, dy, rng);
    } else {
        hipLaunchKernelGGL(cb_bwd_apply_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s, dout, y, scale, shift,
                           ca, sa, w.dsin, sarg, yargmax, w.coef, HW, C, total, dy, rng);
    }
    return check_launch("cb_bwd_apply");
}
#undef DCS_CB16
