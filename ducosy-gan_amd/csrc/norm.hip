// InstanceNorm2d(affine=False, track_running_stats=False) on NHWC fp32 tensors
// (modules/model.py:61-63, 75-79, 94, 97, 110, 124): per-(n,c) statistics, apply (+ReLU/LReLU),
// and the fused activation+IN backward.  All reductions are two-level (per-chunk partials,
// then a fixed-order merge) and therefore deterministic.
#include "common.hpp"

#ifndef DCS_NORM_BATCH
#define DCS_NORM_BATCH 1  // IN apply / backward apply: whole-block fast path with every load issued first
#endif
#ifndef DCS_NORM_PUNROLL
#define DCS_NORM_PUNROLL 1  // IN backward partial sums: pixel-loop unroll (4 measured 1.5 % slower)
#endif

namespace dcs {

// Part (one chunk's statistics of one (n,c)): common.hpp, shared with the conv epilogue

static inline int stats_chunks(int N, int HW) {
    int want = (int)cdiv(1024, N);
    int maxc = (int)cdiv(HW, 64);
    int c = want < maxc ? want : maxc;
    if (c < 1) c = 1;
    return c;
}

// float4 path: C % 4 == 0, C/4 divides 256, 16-byte aligned pointer
static inline bool v4_ok(int C, const void* p) {
    return C % 4 == 0 && C / 4 <= 256 && 256 % (C / 4) == 0 && (reinterpret_cast<uintptr_t>(p) & 15) == 0;
}

// grid (N, nchunk); 256 threads.  Thread layout: if C <= 256 and 256 % C == 0 → C channels x
// (256/C) pixel lanes; otherwise each thread owns channels tid, tid+256, ... (one pixel lane).
__global__ __launch_bounds__(256) void in_stats_partial_kernel(const float* __restrict__ x, int HW, int C,
                                                                int nchunk, Part* __restrict__ parts) {
    const int n = blockIdx.x, chunk = blockIdx.y;
    const int p_per = (HW + nchunk - 1) / nchunk;
    const int p0 = chunk * p_per;
    const int p1 = min(HW, p0 + p_per);
    const int tid = threadIdx.x;
    const bool packed = (C <= 256) && (256 % C == 0);
    const int lanes = packed ? 256 / C : 1;
    const int plane = packed ? tid / C : 0;
    __shared__ float s_cnt[256], s_mean[256], s_m2[256], s_mx[256];
    __shared__ int s_am[256];
    const float* xb = x + (long long)n * HW * C;
    for (int cbase = 0; cbase < C; cbase += (packed ? C : 256)) {
        const int c = packed ? (tid % C) : (cbase + tid);
        float cnt = 0.f, mean = 0.f, m2 = 0.f, mx = -INFINITY;
        int am = 0;
        if (c < C) {
            float K = 0.f, s1 = 0.f, s2 = 0.f;
            bool first = true;
            for (int p = p0 + plane; p < p1; p += lanes) {
                float v = xb[(long long)p * C + c];
                if (first) { K = v; first = false; }
                float dv = v - K;
                s1 += dv;
                s2 = fmaf(dv, dv, s2);
                cnt += 1.f;
                if (v > mx) { mx = v; am = p; }
            }
            if (cnt > 0.f) {
                float d1 = s1 / cnt;
                mean = K + d1;
                m2 = fmaxf(s2 - s1 * d1, 0.f);
            }
        }
        if (packed) {
            s_cnt[tid] = cnt; s_mean[tid] = mean; s_m2[tid] = m2; s_mx[tid] = mx; s_am[tid] = am;
            __syncthreads();
            if (plane == 0) {
                for (int l = 1; l < lanes; ++l) {
                    int o = l * C + c;
                    float nb = s_cnt[o];
                    if (nb <= 0.f) continue;
                    float na = cnt, tot = na + nb;
                    float dl = s_mean[o] - mean;
                    mean = mean + dl * (nb / tot);
                    m2 = m2 + s_m2[o] + dl * dl * (na * nb / tot);
                    cnt = tot;
                    if (s_mx[o] > mx || (s_mx[o] == mx && s_am[o] < am)) { mx = s_mx[o]; am = s_am[o]; }
                }
                Part pt;
                pt.cnt = cnt; pt.mean = mean; pt.m2 = m2; pt.mx = mx; pt.amax = am;
                parts[((long long)n * nchunk + chunk) * C + c] = pt;
            }
            __syncthreads();
        } else if (c < C) {
            Part pt;
            pt.cnt = cnt; pt.mean = mean; pt.m2 = m2; pt.mx = mx; pt.amax = am;
            parts[((long long)n * nchunk + chunk) * C + c] = pt;
        }
    }
}


// Vectorised partial statistics for C % 4 == 0 with 256 % (C/4) == 0 (every layer here): a
// thread owns 4 consecutive channels (float4 loads) and one of 256/(C/4) pixel lanes; the lanes
// are merged in a fixed order (deterministic).  Same Part layout as in_stats_partial_kernel.
__global__ __launch_bounds__(256) void in_stats_partial_v4_kernel(const float4* __restrict__ x, int HW, int C,
                                                                   int nchunk, Part* __restrict__ parts) {
    const int n = blockIdx.x, chunk = blockIdx.y;
    const int p_per = (HW + nchunk - 1) / nchunk;
    const int p0 = chunk * p_per;
    const int p1 = min(HW, p0 + p_per);
    const int cq = C >> 2, lanes = 256 / cq;
    const int tid = threadIdx.x, c4 = tid % cq, plane = tid / cq;
    __shared__ float s_mean[4][256], s_m2[4][256], s_mx[4][256];
    __shared__ int s_am[4][256];
    __shared__ float s_cnt[256];
    const float4* xb = x + (long long)n * HW * cq + c4;
    float K[4] = {0.f, 0.f, 0.f, 0.f}, s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
    float mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    int am[4] = {0, 0, 0, 0};
    float cnt = 0.f;
    int p = p0 + plane;
    if (p < p1) {
        const float4 v = xb[(long long)p * cq];
        K[0] = v.x; K[1] = v.y; K[2] = v.z; K[3] = v.w;
    }
    for (; p < p1; p += lanes) {
        const float4 v4 = xb[(long long)p * cq];
        const float v[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float dv = v[e] - K[e];
            s1[e] += dv;
            s2[e] = fmaf(dv, dv, s2[e]);
            if (v[e] > mx[e]) { mx[e] = v[e]; am[e] = p; }
        }
        cnt += 1.f;
    }
    s_cnt[tid] = cnt;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        float mean = 0.f, m2 = 0.f;
        if (cnt > 0.f) {
            const float d1 = s1[e] / cnt;
            mean = K[e] + d1;
            m2 = fmaxf(s2[e] - s1[e] * d1, 0.f);
        }
        s_mean[e][tid] = mean; s_m2[e][tid] = m2; s_mx[e][tid] = mx[e]; s_am[e][tid] = am[e];
    }
    __syncthreads();
    if (plane != 0) return;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        float c0 = s_cnt[tid], mean = s_mean[e][tid], m2 = s_m2[e][tid], m = s_mx[e][tid];
        int a = s_am[e][tid];
        for (int l = 1; l < lanes; ++l) {
            const int o = l * cq + c4;
            const float nb = s_cnt[o];
            if (nb <= 0.f) continue;
            const float tot = c0 + nb, dl = s_mean[e][o] - mean;
            mean = mean + dl * (nb / tot);
            m2 = m2 + s_m2[e][o] + dl * dl * (c0 * nb / tot);
            c0 = tot;
            if (s_mx[e][o] > m || (s_mx[e][o] == m && s_am[e][o] < a)) { m = s_mx[e][o]; a = s_am[e][o]; }
        }
        Part pt;
        pt.cnt = c0; pt.mean = mean; pt.m2 = m2; pt.mx = m; pt.amax = a;
        parts[((long long)n * nchunk + chunk) * C + 4 * c4 + e] = pt;
    }
}

// finalize with 8 sub-lanes per (n,c): sub-lane s merges chunks s, s+8, ... in order, then a
// fixed xor-butterfly merges the sub-lanes (deterministic, 8x shorter dependent chain)
__device__ __forceinline__ void chan_merge(double& cnt, double& mean, double& m2, float& mx, int& am,
                                           double nb, double mb, double m2b, float mxb, int amb) {
    if (nb > 0.0) {
        const double tot = cnt + nb, dl = mb - mean;
        mean += dl * nb / tot;
        m2 += m2b + dl * dl * cnt * nb / tot;
        cnt = tot;
    }
    if (mxb > mx || (mxb == mx && amb < am)) { mx = mxb; am = amb; }
}

// SUB sub-lanes per (n,c): 8, or 32 for the many-chunk partials of the conv epilogue
// (dcs_in_stats_finish: Ho*Wo/128 chunks per image)
template <int SUB>
__global__ __launch_bounds__(256) void in_stats_finalize8_kernel(const Part* __restrict__ parts, int N, int C,
                                                                  int nchunk, float eps, float* __restrict__ scale,
                                                                  float* __restrict__ shift, float* __restrict__ xmax,
                                                                  int* __restrict__ xam) {
    constexpr int LOG = SUB == 32 ? 5 : 3;
    const int idx = blockIdx.x * (256 / SUB) + (threadIdx.x >> LOG), sub = threadIdx.x & (SUB - 1);
    const bool live = idx < N * C;
    const int n = live ? idx / C : 0, c = live ? idx - n * C : 0;
    double cnt = 0.0, mean = 0.0, m2 = 0.0;
    float mx = -INFINITY;
    int am = 0x7fffffff;
    if (live) {
        for (int k = sub; k < nchunk; k += SUB) {
            const Part p = parts[((long long)n * nchunk + k) * C + c];
            chan_merge(cnt, mean, m2, mx, am, p.cnt, p.mean, p.m2, p.mx, p.amax);
        }
    }
#pragma unroll
    for (int o = 1; o < SUB; o <<= 1) {
        const double nb = __shfl_xor(cnt, o, 64), mb = __shfl_xor(mean, o, 64), m2b = __shfl_xor(m2, o, 64);
        const float mxb = __shfl_xor(mx, o, 64);
        const int amb = __shfl_xor(am, o, 64);
        // merge in a lane-order-independent way: the lower sub-lane is always the left operand
        if ((sub & o) == 0) {
            chan_merge(cnt, mean, m2, mx, am, nb, mb, m2b, mxb, amb);
        } else {
            double c2 = nb, me2 = mb, mm2 = m2b;
            float mx2 = mxb;
            int am2 = amb;
            chan_merge(c2, me2, mm2, mx2, am2, cnt, mean, m2, mx, am);
            cnt = c2; mean = me2; m2 = mm2; mx = mx2; am = am2;
        }
    }
    if (!live || sub != 0) return;
    const double var = m2 / cnt;  // biased (InstanceNorm)
    const float rstd = (float)(1.0 / sqrt(var + (double)eps));
    scale[idx] = rstd;
    shift[idx] = (float)(-mean) * rstd;
    if (xmax) xmax[idx] = mx;
    if (xam) xam[idx] = am;
}

template <bool V4>
__global__ void in_apply_kernel(const float* __restrict__ x, const float* __restrict__ sc,
                                const float* __restrict__ sh, float* __restrict__ out, long long total, int HW,
                                int C, int act, float* __restrict__ rng) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    float m = 0.f;
    if (V4) {
        long long e = i * 4;
        if (e < total) {
            int c = (int)(e % C);
            long long n = e / ((long long)HW * C);
            float4 v = reinterpret_cast<const float4*>(x)[i];
            const float* s = sc + n * C + c;
            const float* b = sh + n * C + c;
            v.x = act_apply(fmaf(v.x, s[0], b[0]), act);
            v.y = act_apply(fmaf(v.y, s[1], b[1]), act);
            v.z = act_apply(fmaf(v.z, s[2], b[2]), act);
            v.w = act_apply(fmaf(v.w, s[3], b[3]), act);
            reinterpret_cast<float4*>(out)[i] = v;
            m = absmax4(v);
        }
    } else if (i < total) {
        int c = (int)(i % C);
        long long n = i / ((long long)HW * C);
        const float v = act_apply(fmaf(x[i], sc[n * C + c], sh[n * C + c]), act);
        out[i] = v;
        m = fabsf(v);
    }
    range_note(rng, m);
}

// Vectorised apply for power-of-two C (every Generator/PatchGAN layer): grid.y = sample, so the
// per-element index math is 32-bit shifts and masks; each thread streams 4 float4.
template <int ACT>
__global__ __launch_bounds__(256) void in_apply_pow2_kernel(const float4* __restrict__ x,
                                                            const float* __restrict__ sc,
                                                            const float* __restrict__ sh,
                                                            float4* __restrict__ out, int per_n4, int cmask,
                                                            float* __restrict__ rng) {
    const int n = blockIdx.y;
    const float* s = sc + (long long)n * (cmask + 1);
    const float* b = sh + (long long)n * (cmask + 1);
    const float4* xs = x + (long long)n * per_n4;
    float4* os = out + (long long)n * per_n4;
    const int i0 = blockIdx.x * 1024 + threadIdx.x;
    float m = 0.f;
    if (DCS_NORM_BATCH && i0 + 768 < per_n4) {  // whole block in range: the 4 loads issued together
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = xs[i0 + 256 * u];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int c = ((i0 + 256 * u) * 4) & cmask;
            const float4 s4 = *reinterpret_cast<const float4*>(s + c);
            const float4 b4 = *reinterpret_cast<const float4*>(b + c);
            float4 o;
            o.x = act_apply(fmaf(v[u].x, s4.x, b4.x), ACT);
            o.y = act_apply(fmaf(v[u].y, s4.y, b4.y), ACT);
            o.z = act_apply(fmaf(v[u].z, s4.z, b4.z), ACT);
            o.w = act_apply(fmaf(v[u].w, s4.w, b4.w), ACT);
            os[i0 + 256 * u] = o;
            m = fmaxf(m, absmax4(o));
        }
    } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = (blockIdx.x * 4 + u) * 256 + threadIdx.x;
            if (i >= per_n4) break;
            const int c = (i * 4) & cmask;
            float4 v = xs[i];
            const float4 s4 = *reinterpret_cast<const float4*>(s + c);
            const float4 b4 = *reinterpret_cast<const float4*>(b + c);
            v.x = act_apply(fmaf(v.x, s4.x, b4.x), ACT);
            v.y = act_apply(fmaf(v.y, s4.y, b4.y), ACT);
            v.z = act_apply(fmaf(v.z, s4.z, b4.z), ACT);
            v.w = act_apply(fmaf(v.w, s4.w, b4.w), ACT);
            os[i] = v;
            m = fmaxf(m, absmax4(v));
        }
    }
    range_note(rng, m);  // every lane, after both paths
}

// ---- backward of a = act(IN(y)) -------------------------------------------------------

__global__ __launch_bounds__(256) void in_bwd_partial_kernel(const float* __restrict__ da, const float* __restrict__ y,
                                                             const float* __restrict__ sc, const float* __restrict__ sh,
                                                             int HW, int C, int act, int nchunk,
                                                             Sum2* __restrict__ parts) {
    const int n = blockIdx.x, chunk = blockIdx.y;
    const int p_per = (HW + nchunk - 1) / nchunk;
    const int p0 = chunk * p_per;
    const int p1 = min(HW, p0 + p_per);
    const int tid = threadIdx.x;
    const bool packed = (C <= 256) && (256 % C == 0);
    const int lanes = packed ? 256 / C : 1;
    const int plane = packed ? tid / C : 0;
    __shared__ float s_a[256], s_b[256];
    const long long base = (long long)n * HW * C;
    for (int cbase = 0; cbase < C; cbase += (packed ? C : 256)) {
        const int c = packed ? (tid % C) : (cbase + tid);
        float sa = 0.f, sb = 0.f;
        if (c < C) {
            const float s = sc[n * C + c], b = sh[n * C + c];
            for (int p = p0 + plane; p < p1; p += lanes) {
                long long o = base + (long long)p * C + c;
                float xh = fmaf(y[o], s, b);
                float g = da[o] * act_grad(xh, act);
                sa += g;
                sb = fmaf(g, xh, sb);
            }
        }
        if (packed) {
            s_a[tid] = sa; s_b[tid] = sb;
            __syncthreads();
            if (plane == 0) {
                for (int l = 1; l < lanes; ++l) { sa += s_a[l * C + c]; sb += s_b[l * C + c]; }
                parts[((long long)n * nchunk + chunk) * C + c] = Sum2{sa, sb};
            }
            __syncthreads();
        } else if (c < C) {
            parts[((long long)n * nchunk + chunk) * C + c] = Sum2{sa, sb};
        }
    }
}

template <int ACT>
__global__ __launch_bounds__(256) void in_bwd_partial_v4_kernel(const float4* __restrict__ da, const float4* __restrict__ y,
                                                                 const float* __restrict__ sc, const float* __restrict__ sh,
                                                                 int HW, int C, int nchunk, Sum2* __restrict__ parts) {
    const int n = blockIdx.x, chunk = blockIdx.y;
    const int p_per = (HW + nchunk - 1) / nchunk;
    const int p0 = chunk * p_per;
    const int p1 = min(HW, p0 + p_per);
    const int cq = C >> 2, lanes = 256 / cq;
    const int tid = threadIdx.x, c4 = tid % cq, plane = tid / cq;
    __shared__ float s_a[4][256], s_b[4][256];
    const float4 s4 = *reinterpret_cast<const float4*>(sc + n * C + 4 * c4);
    const float4 b4 = *reinterpret_cast<const float4*>(sh + n * C + 4 * c4);
    const float s[4] = {s4.x, s4.y, s4.z, s4.w}, b[4] = {b4.x, b4.y, b4.z, b4.w};
    const long long base = (long long)n * HW * cq + c4;
    float sa[4] = {0.f, 0.f, 0.f, 0.f}, sb[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll DCS_NORM_PUNROLL
    for (int p = p0 + plane; p < p1; p += lanes) {
        const float4 g4 = da[base + (long long)p * cq], y4 = y[base + (long long)p * cq];
        const float gv[4] = {g4.x, g4.y, g4.z, g4.w}, yv[4] = {y4.x, y4.y, y4.z, y4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float xh = fmaf(yv[e], s[e], b[e]);
            const float g = gv[e] * act_grad(xh, ACT);
            sa[e] += g;
            sb[e] = fmaf(g, xh, sb[e]);
        }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) { s_a[e][tid] = sa[e]; s_b[e][tid] = sb[e]; }
    __syncthreads();
    if (plane != 0) return;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        float a = s_a[e][tid], bb = s_b[e][tid];
        for (int l = 1; l < lanes; ++l) { a += s_a[e][l * cq + c4]; bb += s_b[e][l * cq + c4]; }
        parts[((long long)n * nchunk + chunk) * C + 4 * c4 + e] = Sum2{a, bb};
    }
}

__global__ __launch_bounds__(256) void in_bwd_finalize8_kernel(const Sum2* __restrict__ parts, int N, int C, int nchunk,
                                                                int HW, Sum2* __restrict__ coef) {
    const int idx = blockIdx.x * 32 + (threadIdx.x >> 3), sub = threadIdx.x & 7;
    const bool live = idx < N * C;
    const int n = live ? idx / C : 0, c = live ? idx - n * C : 0;
    double a = 0.0, b = 0.0;
    if (live)
#pragma unroll 4
        for (int k = sub; k < nchunk; k += 8) {
            const Sum2 p = parts[((long long)n * nchunk + k) * C + c];
            a += p.a;
            b += p.b;
        }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
        a += __shfl_xor(a, o, 64);  // same operand pair on both lanes of a pair: order-free
        b += __shfl_xor(b, o, 64);
    }
    if (live && sub == 0) coef[idx] = Sum2{(float)(a / HW), (float)(b / HW)};
}

template <int ACT>
__global__ __launch_bounds__(256) void in_bwd_apply_pow2_kernel(const float4* __restrict__ da, const float4* __restrict__ y,
                                                                 const float* __restrict__ sc, const float* __restrict__ sh,
                                                                 const Sum2* __restrict__ coef, float4* __restrict__ dy,
                                                                 int per_n4, int cmask, float* __restrict__ rng) {
    const int n = blockIdx.y;
    const int C = cmask + 1;
    const long long off = (long long)n * per_n4;
    const int i0 = blockIdx.x * 1024 + threadIdx.x;
    float m = 0.f;
    if (DCS_NORM_BATCH && i0 + 768 < per_n4) {  // whole block in range: the 8 loads issued together
        float4 g4u[4], y4u[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            g4u[u] = da[off + i0 + 256 * u];
            y4u[u] = y[off + i0 + 256 * u];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int c = ((i0 + 256 * u) * 4) & cmask;
            const float4 s4 = *reinterpret_cast<const float4*>(sc + n * C + c);
            const float4 b4 = *reinterpret_cast<const float4*>(sh + n * C + c);
            const Sum2* k = coef + n * C + c;
            const float gv[4] = {g4u[u].x, g4u[u].y, g4u[u].z, g4u[u].w};
            const float yv[4] = {y4u[u].x, y4u[u].y, y4u[u].z, y4u[u].w};
            const float s[4] = {s4.x, s4.y, s4.z, s4.w}, b[4] = {b4.x, b4.y, b4.z, b4.w};
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float xh = fmaf(yv[e], s[e], b[e]);
                const float g = gv[e] * act_grad(xh, ACT);
                const Sum2 kk = k[e];
                o[e] = s[e] * (g - kk.a - xh * kk.b);
            }
            dy[off + i0 + 256 * u] = make_float4(o[0], o[1], o[2], o[3]);
            m = fmaxf(m, fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3]))));
        }
    } else {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = (blockIdx.x * 4 + u) * 256 + threadIdx.x;
        if (i >= per_n4) break;
        const int c = (i * 4) & cmask;
        const float4 g4 = da[off + i], y4 = y[off + i];
        const float4 s4 = *reinterpret_cast<const float4*>(sc + n * C + c);
        const float4 b4 = *reinterpret_cast<const float4*>(sh + n * C + c);
        const Sum2* k = coef + n * C + c;
        const float gv[4] = {g4.x, g4.y, g4.z, g4.w}, yv[4] = {y4.x, y4.y, y4.z, y4.w};
        const float s[4] = {s4.x, s4.y, s4.z, s4.w}, b[4] = {b4.x, b4.y, b4.z, b4.w};
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float xh = fmaf(yv[e], s[e], b[e]);
            const float g = gv[e] * act_grad(xh, ACT);
            const Sum2 kk = k[e];
            o[e] = s[e] * (g - kk.a - xh * kk.b);
        }
        dy[off + i] = make_float4(o[0], o[1], o[2], o[3]);
        m = fmaxf(m, fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3]))));
    }
    }
    range_note(rng, m);  // every lane, after both paths
}


__global__ void in_bwd_apply_kernel(const float* __restrict__ da, const float* __restrict__ y,
                                    const float* __restrict__ sc, const float* __restrict__ sh,
                                    const Sum2* __restrict__ coef, float* __restrict__ dy, long long total, int HW,
                                    int C, int act, float* __restrict__ rng) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    float m = 0.f;
    if (i < total) {
        int c = (int)(i % C);
        long long n = i / ((long long)HW * C);
        long long nc = n * C + c;
        float s = sc[nc], b = sh[nc];
        float xh = fmaf(y[i], s, b);
        float g = da[i] * act_grad(xh, act);
        Sum2 k = coef[nc];
        const float v = s * (g - k.a - xh * k.b);
        dy[i] = v;
        m = fabsf(v);
    }
    range_note(rng, m);
}

}  // namespace dcs

using namespace dcs;

extern "C" size_t dcs_in_stats_workspace_size(int N, int HW, int C) {
    if (N <= 0 || HW <= 0 || C <= 0) return 0;
    int nchunk = stats_chunks(N, HW);
    size_t a = (size_t)N * nchunk * C * sizeof(Part);
    size_t b = align_up((size_t)N * nchunk * C * sizeof(Sum2), 256) + (size_t)N * C * sizeof(Sum2);
    return a > b ? a : b;
}

extern "C" int dcs_in_stats(const float* x, int N, int HW, int C, float eps, float* scale, float* shift,
                            float* xmax, int32_t* xargmax, void* ws, size_t ws_bytes, void* stream) {
    if (!x || !scale || !shift || !ws || N <= 0 || HW <= 0 || C <= 0)
        return fail(DCS_E_INVALID, "in_stats: bad arguments");
    if (ws_bytes < dcs_in_stats_workspace_size(N, HW, C)) return fail(DCS_E_WORKSPACE, "in_stats: workspace too small");
    int nchunk = stats_chunks(N, HW);
    hipStream_t s = as_stream(stream);
    Part* parts = reinterpret_cast<Part*>(ws);
    if (v4_ok(C, x))
        hipLaunchKernelGGL(in_stats_partial_v4_kernel, dim3(N, nchunk), dim3(256), 0, s,
                           reinterpret_cast<const float4*>(x), HW, C, nchunk, parts);
    else
        hipLaunchKernelGGL(in_stats_partial_kernel, dim3(N, nchunk), dim3(256), 0, s, x, HW, C, nchunk, parts);
    int e = check_launch("in_stats_partial");
    if (e) return e;
    hipLaunchKernelGGL(in_stats_finalize8_kernel<8>, dim3((unsigned)cdiv((long long)N * C, 32)), dim3(256), 0, s, parts,
                       N, C, nchunk, eps, scale, shift, xmax, xargmax);
    return check_launch("in_stats_finalize");
}

// Finalize statistics whose per-chunk partials were written by a producer (the conv rows pass
// with fused statistics, dcs_conv_rows_in_stats): same merge as dcs_in_stats.
extern "C" int dcs_in_stats_finish(const void* parts, int N, int C, int nchunk, float eps, float* scale, float* shift,
                                   float* xmax, int32_t* xargmax, void* stream) {
    if (!parts || !scale || !shift || N <= 0 || C <= 0 || nchunk <= 0)
        return fail(DCS_E_INVALID, "in_stats_finish: bad arguments");
    if (nchunk >= 64)
        hipLaunchKernelGGL(in_stats_finalize8_kernel<32>, dim3((unsigned)cdiv((long long)N * C, 8)), dim3(256), 0,
                           as_stream(stream), reinterpret_cast<const Part*>(parts), N, C, nchunk, eps, scale, shift,
                           xmax, xargmax);
    else
        hipLaunchKernelGGL(in_stats_finalize8_kernel<8>, dim3((unsigned)cdiv((long long)N * C, 32)), dim3(256), 0,
                           as_stream(stream), reinterpret_cast<const Part*>(parts), N, C, nchunk, eps, scale, shift,
                           xmax, xargmax);
    return check_launch("in_stats_finish");
}

extern "C" int dcs_in_apply(const float* x, const float* scale, const float* shift, float* out, int N, int HW, int C,
                            int act, float* rng, void* stream) {
    if (!x || !scale || !shift || !out || N <= 0 || HW <= 0 || C <= 0)
        return fail(DCS_E_INVALID, "in_apply: bad arguments");
    long long total = (long long)N * HW * C;
    hipStream_t s = as_stream(stream);
    if (int e = range_zero(rng, s)) return e;
    const bool pow2 = C >= 4 && (C & (C - 1)) == 0 && ((long long)HW * C) / 4 < (1ll << 30) &&
                      ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out) |
                        reinterpret_cast<uintptr_t>(scale) | reinterpret_cast<uintptr_t>(shift)) & 15) == 0;
    if (pow2 && (act == DCS_ACT_RELU || act == DCS_ACT_LRELU || act == DCS_ACT_AFFINE)) {
        const int per_n4 = (int)((long long)HW * C / 4);
        dim3 grid((unsigned)cdiv(per_n4, 1024), (unsigned)N);
        const float4* x4 = reinterpret_cast<const float4*>(x);
        float4* o4 = reinterpret_cast<float4*>(out);
        if (act == DCS_ACT_RELU)
            hipLaunchKernelGGL(in_apply_pow2_kernel<DCS_ACT_RELU>, grid, dim3(256), 0, s, x4, scale, shift, o4, per_n4, C - 1, rng);
        else if (act == DCS_ACT_LRELU)
            hipLaunchKernelGGL(in_apply_pow2_kernel<DCS_ACT_LRELU>, grid, dim3(256), 0, s, x4, scale, shift, o4, per_n4, C - 1, rng);
        else
            hipLaunchKernelGGL(in_apply_pow2_kernel<DCS_ACT_AFFINE>, grid, dim3(256), 0, s, x4, scale, shift, o4, per_n4, C - 1, rng);
    } else if (C % 4 == 0)
        hipLaunchKernelGGL(in_apply_kernel<true>, dim3((unsigned)cdiv(total / 4, 256)), dim3(256), 0, s, x, scale,
                           shift, out, total, HW, C, act, rng);
    else
        hipLaunchKernelGGL(in_apply_kernel<false>, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s, x, scale, shift,
                           out, total, HW, C, act, rng);
    return check_launch("in_apply");
}

namespace {
// finalize (partial sums -> per-(image, channel) coefficients) + apply of the IN backward
int in_bwd_finish(const float* da, const float* y, const float* scale, const float* shift, float* dy, int N, int HW,
                  int C, int act, const Sum2* parts, int nchunk, Sum2* coef, float* rng, bool v4, hipStream_t s) {
    hipLaunchKernelGGL(in_bwd_finalize8_kernel, dim3((unsigned)cdiv((long long)N * C, 32)), dim3(256), 0, s, parts, N,
                       C, nchunk, HW, coef);
    int e = check_launch("in_bwd_finalize");
    if (e) return e;
    if ((e = range_zero(rng, s))) return e;
    const float4* da4 = reinterpret_cast<const float4*>(da);
    const float4* y4 = reinterpret_cast<const float4*>(y);
    long long total = (long long)N * HW * C;
    const bool pow2 = v4 && (C & (C - 1)) == 0 && (long long)HW * C / 4 < (1ll << 30);
    if (pow2) {
        const int per_n4 = (int)((long long)HW * C / 4);
        dim3 g((unsigned)cdiv(per_n4, 1024), (unsigned)N);
        float4* dy4 = reinterpret_cast<float4*>(dy);
        if (act == DCS_ACT_RELU)
            hipLaunchKernelGGL(in_bwd_apply_pow2_kernel<DCS_ACT_RELU>, g, dim3(256), 0, s, da4, y4, scale, shift, coef, dy4, per_n4, C - 1, rng);
        else if (act == DCS_ACT_LRELU)
            hipLaunchKernelGGL(in_bwd_apply_pow2_kernel<DCS_ACT_LRELU>, g, dim3(256), 0, s, da4, y4, scale, shift, coef, dy4, per_n4, C - 1, rng);
        else
            hipLaunchKernelGGL(in_bwd_apply_pow2_kernel<DCS_ACT_AFFINE>, g, dim3(256), 0, s, da4, y4, scale, shift, coef, dy4, per_n4, C - 1, rng);
    } else {
        hipLaunchKernelGGL(in_bwd_apply_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s, da, y, scale, shift,
                           coef, dy, total, HW, C, act, rng);
    }
    return check_launch("in_bwd_apply");
}
}  // namespace

extern "C" int dcs_in_act_backward_parts(const float* da, const float* y, const float* scale, const float* shift,
                                         float* dy, int N, int HW, int C, int act, const void* parts, int nchunk,
                                         void* ws, size_t ws_bytes, float* rng, void* stream) {
    if (!da || !y || !scale || !shift || !dy || !parts || !ws || N <= 0 || HW <= 0 || C <= 0 || nchunk <= 0)
        return fail(DCS_E_INVALID, "in_act_backward_parts: bad arguments");
    if (ws_bytes < (size_t)N * C * sizeof(Sum2)) return fail(DCS_E_WORKSPACE, "in_act_backward_parts: workspace too small");
    const bool v4 = v4_ok(C, da) && v4_ok(C, y) && v4_ok(C, dy) && v4_ok(C, scale) && v4_ok(C, shift) &&
                    (act == DCS_ACT_RELU || act == DCS_ACT_LRELU || act == DCS_ACT_AFFINE);
    return in_bwd_finish(da, y, scale, shift, dy, N, HW, C, act, reinterpret_cast<const Sum2*>(parts), nchunk,
                         reinterpret_cast<Sum2*>(ws), rng, v4, as_stream(stream));
}

extern "C" int dcs_in_act_backward(const float* da, const float* y, const float* scale, const float* shift, float* dy,
                                   int N, int HW, int C, int act, void* ws, size_t ws_bytes, float* rng, void* stream) {
    if (!da || !y || !scale || !shift || !dy || !ws || N <= 0 || HW <= 0 || C <= 0)
        return fail(DCS_E_INVALID, "in_act_backward: bad arguments");
    if (ws_bytes < dcs_in_stats_workspace_size(N, HW, C))
        return fail(DCS_E_WORKSPACE, "in_act_backward: workspace too small");
    int nchunk = stats_chunks(N, HW);
    hipStream_t s = as_stream(stream);
    Sum2* parts = reinterpret_cast<Sum2*>(ws);
    Sum2* coef = reinterpret_cast<Sum2*>(reinterpret_cast<char*>(ws) +
                                         align_up((size_t)N * nchunk * C * sizeof(Sum2), 256));
    const bool v4 = v4_ok(C, da) && v4_ok(C, y) && v4_ok(C, dy) && v4_ok(C, scale) && v4_ok(C, shift) &&
                    (act == DCS_ACT_RELU || act == DCS_ACT_LRELU || act == DCS_ACT_AFFINE);
    const float4* da4 = reinterpret_cast<const float4*>(da);
    const float4* y4 = reinterpret_cast<const float4*>(y);
    if (v4) {
        dim3 g(N, nchunk);
        if (act == DCS_ACT_RELU)
            hipLaunchKernelGGL(in_bwd_partial_v4_kernel<DCS_ACT_RELU>, g, dim3(256), 0, s, da4, y4, scale, shift, HW, C, nchunk, parts);
        else if (act == DCS_ACT_LRELU)
            hipLaunchKernelGGL(in_bwd_partial_v4_kernel<DCS_ACT_LRELU>, g, dim3(256), 0, s, da4, y4, scale, shift, HW, C, nchunk, parts);
        else
            hipLaunchKernelGGL(in_bwd_partial_v4_kernel<DCS_ACT_AFFINE>, g, dim3(256), 0, s, da4, y4, scale, shift, HW, C, nchunk, parts);
    } else {
        hipLaunchKernelGGL(in_bwd_partial_kernel, dim3(N, nchunk), dim3(256), 0, s, da, y, scale, shift, HW, C, act,
                           nchunk, parts);
    }
    int e = check_launch("in_bwd_partial");
    if (e) return e;
    return in_bwd_finish(da, y, scale, shift, dy, N, HW, C, act, parts, nchunk, coef, rng, v4, s);
}
