// Loss kernels of the G step (modules/trainer.py:22-184, 347-351, 469-512) and SSIM
// (pytorch_msssim.SSIM restated).  Every loss computes its value AND its gradient with
// respect to `pred` in the same call (the backward only rescales by the incoming scalar),
// all on single-channel planes [N,1,H,W].  Global reductions are two-level (per-block
// double partials, then one fixed-order finalize block) — deterministic.
#include "common.hpp"

namespace dcs {

constexpr int RB = 256;        // threads per block
constexpr int MAXBLK = 1024;   // reduction grid cap

static inline int red_blocks(long long n) {
    long long b = cdiv(n, RB);
    if (b > MAXBLK) b = MAXBLK;
    if (b < 1) b = 1;
    return (int)b;
}

// workspace layout (floats): [0,256) scalars, [256, 256+8*MAXBLK*2) double partials, then maps
struct LossWs {
    float* sc;      // scalars
    double* part;   // partials [MAXBLK][8]
    unsigned* hist; // 256 bins
    unsigned* st;   // radix state
    float* maps;    // map region
};
static LossWs loss_ws(void* ws) {
    LossWs w;
    char* b = reinterpret_cast<char*>(ws);
    w.sc = reinterpret_cast<float*>(b);
    w.part = reinterpret_cast<double*>(b + 1024);
    w.hist = reinterpret_cast<unsigned*>(b + 1024 + (size_t)MAXBLK * 8 * sizeof(double));
    w.st = w.hist + 256;
    w.maps = reinterpret_cast<float*>(b + 1024 + (size_t)MAXBLK * 8 * sizeof(double) + 4096);
    return w;
}
static size_t loss_ws_fixed() { return 1024 + (size_t)MAXBLK * 8 * sizeof(double) + 4096; }

template <int K>
__device__ __forceinline__ void block_partials(double (&v)[K], double* part) {
    __shared__ double red[K][4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < K; ++q) {
        double x = wave_sum_d(v[q]);
        if (lane == 0) red[q][w] = x;
    }
    __syncthreads();
    if (threadIdx.x < K) {
        int q = threadIdx.x;
        part[(long long)blockIdx.x * 8 + q] = red[q][0] + red[q][1] + red[q][2] + red[q][3];
    }
}

// sum of partials of quantity q over nb blocks, by one full wave: lane l sums blocks l, l+64, ...
// in order, then a fixed butterfly combines the lanes (deterministic; every lane gets the total)
__device__ __forceinline__ double sum_parts(const double* part, int nb, int q) {
    double s = 0.0;
    for (int b = threadIdx.x & 63; b < nb; b += 64) s += part[(long long)b * 8 + q];
    return wave_sum_d(s);
}

// ---------------------------------------------------------------------------------------
// L1 / MSE (nn.L1Loss, nn.MSELoss; trainer.py:347-349)
// ---------------------------------------------------------------------------------------
template <int KIND>  // 0 L1, 1 MSE, 2 MSE vs constant
__global__ __launch_bounds__(RB) void pointwise_kernel(const float* __restrict__ p, const float* __restrict__ t,
                                                       float tc, long long n, float* __restrict__ grad,
                                                       double* part) {
    double acc[1] = {0.0};
    const float inv = 1.f / (float)n;
    for (long long i = (long long)blockIdx.x * RB + threadIdx.x; i < n; i += (long long)gridDim.x * RB) {
        float d = p[i] - (KIND == 2 ? tc : t[i]);
        if (KIND == 0) {
            acc[0] += fabsf(d);
            if (grad) grad[i] = sgnf(d) * inv;
        } else {
            acc[0] += (double)d * d;
            if (grad) grad[i] = 2.f * d * inv;
        }
    }
    block_partials<1>(acc, part);
}

__global__ void finalize_mean_kernel(const double* part, int nb, long long n, float* out) {
    const double v = sum_parts(part, nb, 0);
    if (threadIdx.x == 0) out[0] = (float)(v / (double)n);
}

// ---------------------------------------------------------------------------------------
// GradientLoss (trainer.py:22-40)
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(RB) void gradient_loss_kernel(const float* __restrict__ p, const float* __restrict__ t,
                                                           int N, int H, int W, float* __restrict__ grad,
                                                           double* part) {
    double acc[2] = {0.0, 0.0};
    const long long n = (long long)N * H * W;
    const float ix = 1.f / (float)((long long)N * H * (W - 1));
    const float iy = 1.f / (float)((long long)N * (H - 1) * W);
    for (long long e = (long long)blockIdx.x * RB + threadIdx.x; e < n; e += (long long)gridDim.x * RB) {
        int j = (int)(e % W);
        int i = (int)((e / W) % H);
        float pv = p[e], tv = t[e];
        float g = 0.f;
        if (j + 1 < W) {  // x-difference owned by (i, j)
            float dp = p[e + 1] - pv, dt = t[e + 1] - tv;
            float ex = fabsf(dp) - fabsf(dt);
            acc[0] += fabsf(ex);
            g -= sgnf(ex) * sgnf(dp) * ix;
        }
        if (j > 0) {
            float dp = pv - p[e - 1], dt = tv - t[e - 1];
            float ex = fabsf(dp) - fabsf(dt);
            g += sgnf(ex) * sgnf(dp) * ix;
        }
        if (i + 1 < H) {
            float dp = p[e + W] - pv, dt = t[e + W] - tv;
            float ey = fabsf(dp) - fabsf(dt);
            acc[1] += fabsf(ey);
            g -= sgnf(ey) * sgnf(dp) * iy;
        }
        if (i > 0) {
            float dp = pv - p[e - W], dt = tv - t[e - W];
            float ey = fabsf(dp) - fabsf(dt);
            g += sgnf(ey) * sgnf(dp) * iy;
        }
        if (grad) grad[e] = g;
    }
    block_partials<2>(acc, part);
}

__global__ void gradient_loss_final(const double* part, int nb, int N, int H, int W, float* out) {
    double sx = sum_parts(part, nb, 0), sy = sum_parts(part, nb, 1);
    if (threadIdx.x == 0) out[0] = (float)(sx / ((double)N * H * (W - 1)) + sy / ((double)N * (H - 1) * W));
}

// ---------------------------------------------------------------------------------------
// ContrastAttentionLoss (trainer.py:43-86): AvgPool(k, s1, p k/2, count_include_pad)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ float box_mean(const float* __restrict__ x, int n, int i, int j, int H, int W, int k) {
    const int r = k / 2;
    float s = 0.f;
    for (int a = -r; a <= r; ++a) {
        int ii = i + a;
        if (ii < 0 || ii >= H) continue;
        const float* row = x + ((long long)n * H + ii) * W;
        for (int b = -r; b <= r; ++b) {
            int jj = j + b;
            if (jj >= 0 && jj < W) s += row[jj];
        }
    }
    return s / (float)(k * k);
}

__global__ __launch_bounds__(RB) void ca_loss_kernel(const float* __restrict__ p, const float* __restrict__ t,
                                                     const float* __restrict__ s, int N, int H, int W, float sigma,
                                                     float minw, float maxw, int k, float* __restrict__ gmap,
                                                     double* part) {
    double acc[1] = {0.0};
    const long long n = (long long)N * H * W;
    const float inv = 1.f / (float)n;
    for (long long e = (long long)blockIdx.x * RB + threadIdx.x; e < n; e += (long long)gridDim.x * RB) {
        int j = (int)(e % W);
        long long r = e / W;
        int i = (int)(r % H);
        int nn = (int)(r / H);
        float tb = box_mean(t, nn, i, j, H, W, k);
        float sb = box_mean(s, nn, i, j, H, W, k);
        float pb = box_mean(p, nn, i, j, H, W, k);
        float w = minw + (maxw - minw) * (1.f - expf(-fabsf(tb - sb) / sigma));
        acc[0] += (double)(w * fabsf(pb - tb));
        gmap[e] = w * sgnf(pb - tb) * inv;
    }
    block_partials<1>(acc, part);
}

__global__ void box_adjoint_kernel(const float* __restrict__ g, int N, int H, int W, int k, float* __restrict__ grad) {
    long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    long long n = (long long)N * H * W;
    if (e >= n) return;
    int j = (int)(e % W);
    long long r = e / W;
    int i = (int)(r % H);
    int nn = (int)(r / H);
    grad[e] = box_mean(g, nn, i, j, H, W, k);  // symmetric window: adjoint == same box
}

// ---------------------------------------------------------------------------------------
// ContrastRegionLoss (trainer.py:89-130)
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(RB) void cr_loss_kernel(const float* __restrict__ p, const float* __restrict__ t,
                                                     const float* __restrict__ s, int N, int H, int W, float thr,
                                                     float* __restrict__ gq, double* part, long long nq_norm) {
    // quantities: 0 region sum, 1 sum p, 2 sum p^2, 3 sum t, 4 sum t^2
    double acc[5] = {0, 0, 0, 0, 0};
    const int Hp = H / 8, Wp = W / 8;
    const long long nq = (long long)N * Hp * Wp;
    const long long n = (long long)N * H * W;
    const float invq = nq_norm > 0 ? 1.f / (float)nq_norm : 1.f;  // nq_norm 0: gq unnormalised
    for (long long e = (long long)blockIdx.x * RB + threadIdx.x; e < n; e += (long long)gridDim.x * RB) {
        float pv = p[e], tv = t[e];
        acc[1] += pv; acc[2] += (double)pv * pv;
        acc[3] += tv; acc[4] += (double)tv * tv;
    }
    for (long long q = (long long)blockIdx.x * RB + threadIdx.x; q < nq; q += (long long)gridDim.x * RB) {
        int qx = (int)(q % Wp);
        long long r = q / Wp;
        int qy = (int)(r % Hp);
        int nn = (int)(r / Hp);
        float sp = 0.f, st = 0.f, ss = 0.f;
        for (int a = 0; a < 8; ++a) {
            long long row = ((long long)nn * H + qy * 8 + a) * W + qx * 8;
            for (int b = 0; b < 8; ++b) { sp += p[row + b]; st += t[row + b]; ss += s[row + b]; }
        }
        sp /= 64.f; st /= 64.f; ss /= 64.f;
        float m = sigmoidf_(5.f * ((st - ss) - thr));
        acc[0] += (double)(m * fabsf(sp - st));
        gq[q] = m * sgnf(sp - st) * invq;
    }
    block_partials<5>(acc, part);
}

__global__ void cr_loss_final(const double* part, int nb, long long n, long long nq, float weight, float* sc,
                              float* out) {
    double reg = sum_parts(part, nb, 0);
    double s1 = sum_parts(part, nb, 1), s2 = sum_parts(part, nb, 2);
    double t1 = sum_parts(part, nb, 3), t2 = sum_parts(part, nb, 4);
    if (threadIdx.x != 0) return;
    double mp = s1 / n, mt = t1 / n;
    double sp = sqrt(fmax((s2 - n * mp * mp) / (n - 1), 0.0));
    double st = sqrt(fmax((t2 - n * mt * mt) / (n - 1), 0.0));
    double region = nq > 0 ? reg / nq : 0.0;
    double v = weight * (region + 0.5 * (fabs(mp - mt) + fabs(sp - st)));
    out[0] = (float)v;
    sc[0] = (float)mp;
    sc[1] = (float)sp;
    // d/dp of 0.5*weight*(|mp-mt| + |sp-st|): a + b*(p - mp)
    double sg1 = (mp > mt) ? 1.0 : ((mp < mt) ? -1.0 : 0.0);
    double sg2 = (sp > st) ? 1.0 : ((sp < st) ? -1.0 : 0.0);
    sc[2] = (float)(0.5 * weight * sg1 / n);
    sc[3] = (float)(sp > 0 ? 0.5 * weight * sg2 / ((n - 1) * sp) : 0.0);
    sc[5] = 1.f;  // gq already carries 1/nq
}

__global__ void cr_grad_kernel(const float* __restrict__ p, const float* __restrict__ gq, const float* __restrict__ sc,
                               int N, int H, int W, float weight, float* __restrict__ grad) {
    long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    long long n = (long long)N * H * W;
    if (e >= n) return;
    int j = (int)(e % W);
    long long r = e / W;
    int i = (int)(r % H);
    int nn = (int)(r / H);
    const int Hp = H / 8, Wp = W / 8;
    float g = sc[2] + sc[3] * (p[e] - sc[0]);
    if (i < Hp * 8 && j < Wp * 8) g += weight * sc[5] * gq[((long long)nn * Hp + i / 8) * Wp + j / 8] / 64.f;
    grad[e] = g;
}

// ---------------------------------------------------------------------------------------
// ContrastEdgeLoss (trainer.py:133-184): Sobel magnitude stats + exact top-10 % mean
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void sobel(const float* __restrict__ x, int nn, int i, int j, int H, int W, float& ex,
                                      float& ey) {
    float v[3][3];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            int ii = i + a - 1, jj = j + b - 1;
            v[a][b] = (ii >= 0 && ii < H && jj >= 0 && jj < W) ? x[((long long)nn * H + ii) * W + jj] : 0.f;
        }
    // cross-correlation with Sx = [[-1,0,1],[-2,0,2],[-1,0,1]], Sy = Sx^T
    ex = (-v[0][0] + v[0][2]) + (-2.f * v[1][0] + 2.f * v[1][2]) + (-v[2][0] + v[2][2]);
    ey = (-v[0][0] - 2.f * v[0][1] - v[0][2]) + (v[2][0] + 2.f * v[2][1] + v[2][2]);
}

__global__ __launch_bounds__(RB) void edge_maps_kernel(const float* __restrict__ p, const float* __restrict__ t, int N,
                                                       int H, int W, float* __restrict__ ep, float* __restrict__ et,
                                                       double* part) {
    double acc[4] = {0, 0, 0, 0};
    const long long n = (long long)N * H * W;
    for (long long e = (long long)blockIdx.x * RB + threadIdx.x; e < n; e += (long long)gridDim.x * RB) {
        int j = (int)(e % W);
        long long r = e / W;
        int i = (int)(r % H);
        int nn = (int)(r / H);
        float ex, ey;
        sobel(p, nn, i, j, H, W, ex, ey);
        float a = sqrtf(ex * ex + ey * ey + 1e-6f);
        sobel(t, nn, i, j, H, W, ex, ey);
        float b = sqrtf(ex * ex + ey * ey + 1e-6f);
        ep[e] = a;
        et[e] = b;
        acc[0] += a; acc[1] += (double)a * a;
        acc[2] += b; acc[3] += (double)b * b;
    }
    block_partials<4>(acc, part);
}

// radix select of the k-th largest positive float: state st = {prefix, kleft, shift_done}
__global__ void radix_init_kernel(unsigned* st, unsigned k, unsigned* hist) {
    if (threadIdx.x == 0) { st[0] = 0u; st[1] = k; }
    hist[threadIdx.x] = 0u;
}

__global__ __launch_bounds__(RB) void radix_hist_kernel(const float* __restrict__ x, long long n, int shift,
                                                        const unsigned* __restrict__ st, unsigned* hist) {
    __shared__ unsigned h[256];
    h[threadIdx.x] = 0u;
    __syncthreads();
    const unsigned prefix = st[0];
    const unsigned himask = shift >= 24 ? 0u : (0xFFFFFFFFu << (shift + 8));
    for (long long i = (long long)blockIdx.x * RB + threadIdx.x; i < n; i += (long long)gridDim.x * RB) {
        unsigned u = __float_as_uint(x[i]);
        if ((u & himask) == (prefix & himask)) atomicAdd(&h[(u >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}

__global__ void radix_select_kernel(unsigned* st, int shift, unsigned* hist) {
    if (threadIdx.x == 0) {
        unsigned k = st[1], cum = 0u;
        int b = 255;
        for (; b > 0; --b) {
            if (cum + hist[b] >= k) break;
            cum += hist[b];
        }
        st[0] |= ((unsigned)b << shift);
        st[1] = k - cum;  // still to take from elements whose bits so far equal prefix
    }
    __syncthreads();
    hist[threadIdx.x] = 0u;
}

// sum of elements > tau, count of elements == tau
__global__ __launch_bounds__(RB) void topk_sum_kernel(const float* __restrict__ x, long long n,
                                                      const unsigned* __restrict__ st, double* part) {
    double acc[2] = {0.0, 0.0};
    const float tau = __uint_as_float(st[0]);
    for (long long i = (long long)blockIdx.x * RB + threadIdx.x; i < n; i += (long long)gridDim.x * RB) {
        float v = x[i];
        if (v > tau) acc[0] += v;
        else if (v == tau) acc[1] += 1.0;
    }
    block_partials<2>(acc, part);
}

// stores in sc: [0]=tau_p [1]=kleft_p/cnt_eq_p [2..] coefficients
__global__ void edge_final_kernel(const double* part_stats, int nb_stats, const double* part_tp, int nb_tp,
                                  const double* part_tt, int nb_tt, const unsigned* st_p, const unsigned* st_t,
                                  long long n, long long k, float* sc, float* out) {
    double s1 = sum_parts(part_stats, nb_stats, 0), s2 = sum_parts(part_stats, nb_stats, 1);
    double t1 = sum_parts(part_stats, nb_stats, 2), t2 = sum_parts(part_stats, nb_stats, 3);
    const double ptp = sum_parts(part_tp, nb_tp, 0), ptt = sum_parts(part_tt, nb_tt, 0);
    const double eqp = sum_parts(part_tp, nb_tp, 1);
    if (threadIdx.x != 0) return;
    double mp = s1 / n, mt = t1 / n;
    double sp = sqrt(fmax((s2 - n * mp * mp) / (n - 1), 0.0));
    double st = sqrt(fmax((t2 - n * mt * mt) / (n - 1), 0.0));
    double taup = (double)__uint_as_float(st_p[0]), taut = (double)__uint_as_float(st_t[0]);
    double tkp = (ptp + (double)st_p[1] * taup) / (double)k;
    double tkt = (ptt + (double)st_t[1] * taut) / (double)k;
    out[0] = (float)(fabs(mp - mt) + fabs(sp - st) + fabs(tkp - tkt));
    double sg1 = (mp > mt) ? 1.0 : ((mp < mt) ? -1.0 : 0.0);
    double sg2 = (sp > st) ? 1.0 : ((sp < st) ? -1.0 : 0.0);
    double sg3 = (tkp > tkt) ? 1.0 : ((tkp < tkt) ? -1.0 : 0.0);
    sc[0] = __uint_as_float(st_p[0]);
    sc[1] = (float)(eqp > 0 ? (double)st_p[1] / eqp : 0.0);  // share of each tied element
    sc[2] = (float)(sg1 / n);
    sc[3] = (float)(sp > 0 ? sg2 / ((n - 1) * sp) : 0.0);
    sc[4] = (float)mp;
    sc[5] = (float)(sg3 / (double)k);
}

// gx = de * ex/e, gy = de * ey/e  (de = d loss / d edge_p)
__global__ void edge_grad_maps_kernel(const float* __restrict__ p, const float* __restrict__ ep,
                                      const float* __restrict__ sc, int N, int H, int W, float* __restrict__ gx,
                                      float* __restrict__ gy) {
    long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    long long n = (long long)N * H * W;
    if (e >= n) return;
    int j = (int)(e % W);
    long long r = e / W;
    int i = (int)(r % H);
    int nn = (int)(r / H);
    float v = ep[e];
    float sel = v > sc[0] ? 1.f : (v == sc[0] ? sc[1] : 0.f);
    float de = sc[2] + sc[3] * (v - sc[4]) + sc[5] * sel;
    float ex, ey;
    sobel(p, nn, i, j, H, W, ex, ey);
    gx[e] = de * ex / v;
    gy[e] = de * ey / v;
}

// adjoint of the zero-padded Sobel cross-correlations
__global__ void edge_grad_kernel(const float* __restrict__ gx, const float* __restrict__ gy, int N, int H, int W,
                                 float* __restrict__ grad) {
    long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    long long n = (long long)N * H * W;
    if (e >= n) return;
    int j = (int)(e % W);
    long long r = e / W;
    int i = (int)(r % H);
    int nn = (int)(r / H);
    const float SX[3][3] = {{-1.f, 0.f, 1.f}, {-2.f, 0.f, 2.f}, {-1.f, 0.f, 1.f}};
    const float SY[3][3] = {{-1.f, -2.f, -1.f}, {0.f, 0.f, 0.f}, {1.f, 2.f, 1.f}};
    float g = 0.f;
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            int ii = i - a + 1, jj = j - b + 1;  // output position whose window holds (i,j) at (a,b)
            if (ii >= 0 && ii < H && jj >= 0 && jj < W) {
                long long o = ((long long)nn * H + ii) * W + jj;
                g = fmaf(SX[a][b], gx[o], g);
                g = fmaf(SY[a][b], gy[o], g);
            }
        }
    grad[e] = g;
}

// ---------------------------------------------------------------------------------------
// Global statistics of the batch-coupled losses over data-parallel ranks (SURVEY.md §8e
// option ii).  The phases below leave this shard's partial sums in a caller buffer `red`
// (double) or a 512-bin histogram; the caller sums them over ranks between the phases (one
// all-reduce each), and the next phase reads the sums back, so every rank finishes with the
// loss of the WHOLE batch.  The partials are the same quantities the one-call path reduces.
// ---------------------------------------------------------------------------------------
// red[r0 + q] = sum of partial q over nb blocks (q < K); optional counts after them
__global__ void red_sum_kernel(const double* part, int nb, int K, double* red, int r0, double c0, double c1, int nc) {
    for (int q = 0; q < K; ++q) {
        const double v = sum_parts(part, nb, q);
        if (threadIdx.x == 0) red[r0 + q] = v;
    }
    if (threadIdx.x == 0) {
        if (nc > 0) red[r0 + K] = c0;
        if (nc > 1) red[r0 + K + 1] = c1;
    }
}

// region: red = {region sum, sum p, sum p^2, sum t, sum t^2, n, nq} over all ranks
__global__ void cr_final_red_kernel(const double* red, float weight, float grad_scale, float* sc, float* out) {
    if (threadIdx.x != 0) return;
    const double n = red[5], nq = red[6];
    const double mp = red[1] / n, mt = red[3] / n;
    const double sp = sqrt(fmax((red[2] - n * mp * mp) / (n - 1), 0.0));
    const double st = sqrt(fmax((red[4] - n * mt * mt) / (n - 1), 0.0));
    const double region = nq > 0 ? red[0] / nq : 0.0;
    out[0] = (float)(weight * (region + 0.5 * (fabs(mp - mt) + fabs(sp - st))));
    const double sg1 = (mp > mt) ? 1.0 : ((mp < mt) ? -1.0 : 0.0);
    const double sg2 = (sp > st) ? 1.0 : ((sp < st) ? -1.0 : 0.0);
    sc[0] = (float)mp;
    sc[1] = (float)sp;
    sc[2] = (float)(grad_scale * 0.5 * weight * sg1 / n);
    sc[3] = (float)(sp > 0 ? grad_scale * 0.5 * weight * sg2 / ((n - 1) * sp) : 0.0);
    sc[5] = (float)(nq > 0 ? grad_scale / nq : 0.0);  // gq holds m * sign, unnormalised
}

// edge: red = {sum ep, sum ep^2, sum et, sum et^2, n, sum ep>tau_p, #ep==tau_p, sum et>tau_t, #et==tau_t}
__device__ __forceinline__ long long edge_k(double n) { return (long long)(n * 0.1); }  // int(numel * 0.1)

__global__ void edge_radix_init_kernel(unsigned* st_p, unsigned* st_t, const double* red) {
    if (threadIdx.x == 0) {
        const unsigned k = (unsigned)edge_k(red[4]);
        st_p[0] = 0u; st_p[1] = k;
        st_t[0] = 0u; st_t[1] = k;
    }
}

// radix select step from a (summed) histogram, without clearing it (it is the caller's)
__global__ void radix_select_const_kernel(unsigned* st, int shift, const unsigned* hist) {
    if (threadIdx.x == 0) {
        const unsigned k = st[1];
        unsigned cum = 0u;
        int b = 255;
        for (; b > 0; --b) {
            if (cum + hist[b] >= k) break;
            cum += hist[b];
        }
        st[0] |= ((unsigned)b << shift);
        st[1] = k - cum;
    }
}

__global__ void edge_final_red_kernel(const double* red, const unsigned* st_p, const unsigned* st_t, float grad_scale,
                                      float* sc, float* out) {
    if (threadIdx.x != 0) return;
    const double n = red[4];
    const double k = (double)edge_k(n);
    const double mp = red[0] / n, mt = red[2] / n;
    const double sp = sqrt(fmax((red[1] - n * mp * mp) / (n - 1), 0.0));
    const double st = sqrt(fmax((red[3] - n * mt * mt) / (n - 1), 0.0));
    const double taup = (double)__uint_as_float(st_p[0]), taut = (double)__uint_as_float(st_t[0]);
    const double tkp = (red[5] + (double)st_p[1] * taup) / k;
    const double tkt = (red[7] + (double)st_t[1] * taut) / k;
    out[0] = (float)(fabs(mp - mt) + fabs(sp - st) + fabs(tkp - tkt));
    const double sg1 = (mp > mt) ? 1.0 : ((mp < mt) ? -1.0 : 0.0);
    const double sg2 = (sp > st) ? 1.0 : ((sp < st) ? -1.0 : 0.0);
    const double sg3 = (tkp > tkt) ? 1.0 : ((tkp < tkt) ? -1.0 : 0.0);
    sc[0] = __uint_as_float(st_p[0]);
    sc[1] = (float)(red[6] > 0 ? (double)st_p[1] / red[6] : 0.0);
    sc[2] = (float)(grad_scale * sg1 / n);
    sc[3] = (float)(sp > 0 ? grad_scale * sg2 / ((n - 1) * sp) : 0.0);
    sc[4] = (float)mp;
    sc[5] = (float)(grad_scale * sg3 / k);
}

// ---------------------------------------------------------------------------------------
// SSIM (pytorch_msssim.ssim, size_average=True, valid separable gaussian)
// ---------------------------------------------------------------------------------------
struct Gauss {
    float g[16];
};
static Gauss make_gauss(int win, float sigma) {
    Gauss G;
    float s = 0.f;
    for (int i = 0; i < win; ++i) {
        float c = (float)i - (float)(win / 2);
        G.g[i] = expf(-(c * c) / (2.f * sigma * sigma));
        s += G.g[i];
    }
    for (int i = 0; i < win; ++i) G.g[i] /= s;
    for (int i = win; i < 16; ++i) G.g[i] = 0.f;
    return G;
}

// vertical valid pass of X, Y, XX, YY, XY -> V[5][N][Hv][W]
__global__ void ssim_v_kernel(const float* __restrict__ X, const float* __restrict__ Y, int N, int H, int W, int win,
                              Gauss G, float* __restrict__ V) {
    const int Hv = H - win + 1;
    long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    long long tot = (long long)N * Hv * W;
    if (e >= tot) return;
    int j = (int)(e % W);
    long long r = e / W;
    int i = (int)(r % Hv);
    int nn = (int)(r / Hv);
    float a[5] = {0, 0, 0, 0, 0};
    for (int q = 0; q < win; ++q) {
        long long o = ((long long)nn * H + i + q) * W + j;
        float x = X[o], y = Y[o], g = G.g[q];
        a[0] = fmaf(g, x, a[0]);
        a[1] = fmaf(g, y, a[1]);
        a[2] = fmaf(g, x * x, a[2]);
        a[3] = fmaf(g, y * y, a[3]);
        a[4] = fmaf(g, x * y, a[4]);
    }
#pragma unroll
    for (int m = 0; m < 5; ++m) V[m * tot + e] = a[m];
}

// horizontal valid pass + ssim map + derivative maps D[3][N][Hv][Wv]
__global__ __launch_bounds__(RB) void ssim_h_kernel(const float* __restrict__ V, int N, int H, int W, int win, Gauss G,
                                                    float C1, float C2, float* __restrict__ D, double* part) {
    const int Hv = H - win + 1, Wv = W - win + 1;
    const long long totv = (long long)N * Hv * W;
    const long long tot = (long long)N * Hv * Wv;
    const float inv = 1.f / (float)tot;
    double acc[1] = {0.0};
    for (long long e = (long long)blockIdx.x * RB + threadIdx.x; e < tot; e += (long long)gridDim.x * RB) {
        int j = (int)(e % Wv);
        long long r = e / Wv;  // = nn*Hv + i
        float m[5] = {0, 0, 0, 0, 0};
        for (int q = 0; q < win; ++q) {
            long long o = r * W + j + q;
            float g = G.g[q];
#pragma unroll
            for (int k = 0; k < 5; ++k) m[k] = fmaf(g, V[k * totv + o], m[k]);
        }
        float mu1 = m[0], mu2 = m[1];
        float s11 = m[2] - mu1 * mu1, s22 = m[3] - mu2 * mu2, s12 = m[4] - mu1 * mu2;
        float A = 2.f * mu1 * mu2 + C1, B = mu1 * mu1 + mu2 * mu2 + C1;
        float Cc = 2.f * s12 + C2, Dd = s11 + s22 + C2;
        float cs = Cc / Dd;
        float s = (A / B) * cs;
        acc[0] += s;
        float BD = B * Dd;
        D[e] = (2.f * mu2 * (Cc - A) / BD - s * 2.f * mu1 * (1.f / B - 1.f / Dd)) * inv;  // d/d mu1
        D[tot + e] = (-s / Dd) * inv;                                                     // d/d E[XX]
        D[2 * tot + e] = (2.f * A / BD) * inv;                                            // d/d E[XY]
    }
    block_partials<1>(acc, part);
}

__global__ void ssim_final(const double* part, int nb, long long tot, float* out) {
    const double v = sum_parts(part, nb, 0);
    if (threadIdx.x == 0) out[0] = (float)(v / (double)tot);
}

// adjoint horizontal: T[3][N][Hv][W] = sum_b g[b] D[.][i][v-b]
__global__ void ssim_ht_kernel(const float* __restrict__ D, int N, int H, int W, int win, Gauss G,
                               float* __restrict__ T) {
    const int Hv = H - win + 1, Wv = W - win + 1;
    const long long tot = (long long)N * Hv * Wv, totv = (long long)N * Hv * W;
    long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= totv) return;
    int v = (int)(e % W);
    long long r = e / W;
    float a[3] = {0, 0, 0};
    for (int b = 0; b < win; ++b) {
        int jj = v - b;
        if (jj < 0 || jj >= Wv) continue;
        long long o = r * Wv + jj;
        a[0] = fmaf(G.g[b], D[o], a[0]);
        a[1] = fmaf(G.g[b], D[tot + o], a[1]);
        a[2] = fmaf(G.g[b], D[2 * tot + o], a[2]);
    }
    T[e] = a[0];
    T[totv + e] = a[1];
    T[2 * totv + e] = a[2];
}

// adjoint vertical + chain rule: dX = R0 + 2 X R1 + Y R2
__global__ void ssim_vt_kernel(const float* __restrict__ T, const float* __restrict__ X, const float* __restrict__ Y,
                               int N, int H, int W, int win, Gauss G, float* __restrict__ grad) {
    const int Hv = H - win + 1;
    const long long totv = (long long)N * Hv * W;
    long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    long long tot = (long long)N * H * W;
    if (e >= tot) return;
    int j = (int)(e % W);
    long long r = e / W;
    int u = (int)(r % H);
    int nn = (int)(r / H);
    float a[3] = {0, 0, 0};
    for (int q = 0; q < win; ++q) {
        int ii = u - q;
        if (ii < 0 || ii >= Hv) continue;
        long long o = ((long long)nn * Hv + ii) * W + j;
        a[0] = fmaf(G.g[q], T[o], a[0]);
        a[1] = fmaf(G.g[q], T[totv + o], a[1]);
        a[2] = fmaf(G.g[q], T[2 * totv + o], a[2]);
    }
    grad[e] = a[0] + 2.f * X[e] * a[1] + Y[e] * a[2];
}


// ---------------------------------------------------------------------------------------
// Fused G-step loss planes (north star: one cycle / identity / SSIM / gradient / contrast-loss
// kernel; modules/trainer.py:469-512).  One launch walks every (pred, target) plane pair of the
// step in 32 x 32 output tiles: a tile's pred / target (/ source) region with a 10-pixel halo is
// staged in LDS once, and the job's terms are evaluated from it:
//   L1     nn.L1Loss                         (trainer.py:348-349)
//   GRAD   GradientLoss                      (trainer.py:22-40)
//   SSIM   pytorch_msssim.SSIM, 11-tap valid gaussian, value and gradient in one pass: the
//          forward blur over the tile + 10 px halo, the derivative maps, and the adjoint blur
//          back onto the tile (the 4-pass ssim_v / ssim_h / ssim_ht / ssim_vt chain fused)
//   CA     ContrastAttentionLoss (7x7 box, count_include_pad; trainer.py:43-86)
//   MSEC   nn.MSELoss against a constant label (the PatchGAN terms, trainer.py:459-460, 470)
// The job's gradient plane receives the WEIGHTED SUM of its terms' d/dpred (the coefficients are
// the terms' weights in loss_G), plus up to two addends (the batch-coupled ContrastRegion /
// ContrastEdge gradients of the same plane, computed by their own phases first): one write per
// pixel, no per-term gradient planes and no adds.  Per-tile double partials of every term go to
// part[block][8]; gl_final_kernel sums them in a fixed order (deterministic) and composes the
// step's loss values from a coefficient recipe.
// ---------------------------------------------------------------------------------------
constexpr int GLT = 32, GLH = 10, GLR = GLT + 2 * GLH;  // tile, halo, staged region (52)
constexpr int GLQ = GLT + GLH;                           // SSIM window positions per tile side (42)
constexpr int GL_MAXJOB = 8;

struct GLJobK {
    const float* p;
    const float* t;
    const float* s;
    const float* add0;
    const float* add1;
    float* g;
    int nimg, flags, blk0, H, W, tiles_x, tiles, pad;
    float c_l1, c_grad, c_ssim, c_ca, c_mse, t_const, c_add0, c_add1;
};
struct GLArgsK {
    GLJobK j[GL_MAXJOB];
    int njobs;
    float gw[12];
    float C1, C2, sigma, minw, maxw;
};

__global__ __launch_bounds__(256) void gl_planes_kernel(GLArgsK a, double* __restrict__ part) {
    __shared__ float P[GLR * GLR], T[GLR * GLR], S[GLR * GLR];
    __shared__ float V[5 * GLQ * GLR];  // SSIM vertical pass; reused by the CA maps and the adjoint
    __shared__ float D[3 * GLQ * GLQ];
    const int tid = threadIdx.x;
    int jb = 0;
#pragma unroll 1
    for (int q = 1; q < a.njobs; ++q)
        if ((int)blockIdx.x >= a.j[q].blk0) jb = q;
    const GLJobK& J = a.j[jb];
    const int H = J.H, W = J.W;
    const int local = blockIdx.x - J.blk0;
    const int n = local / J.tiles, tl = local - n * J.tiles;
    const int ty = tl / J.tiles_x, tx = tl - ty * J.tiles_x;
    const int i0 = ty * GLT, j0 = tx * GLT;
    const long long base = (long long)n * H * W;
    const int fl = J.flags;

    // stage the region (zeros outside the image)
    for (int e = tid; e < GLR * GLR; e += 256) {
        const int r = e / GLR, c = e - r * GLR;
        const int y = i0 - GLH + r, x = j0 - GLH + c;
        const bool in = y >= 0 && y < H && x >= 0 && x < W;
        const long long o = base + (long long)y * W + x;
        P[e] = in ? J.p[o] : 0.f;
        T[e] = in && J.t ? J.t[o] : 0.f;
        if (fl & 8) S[e] = in ? J.s[o] : 0.f;
    }
    __syncthreads();

    double acc[5] = {0.0, 0.0, 0.0, 0.0, 0.0};  // l1, grad x, grad y, ssim, ca / mse
    float gout[4] = {0.f, 0.f, 0.f, 0.f};       // the thread's 4 pixels: (row tid/8, cols 4*(tid%8) ..)
    const int orow = tid >> 3, oc0 = (tid & 7) * 4;
    const float nhw = (float)((long long)J.nimg * H * W);
    // pointwise and gradient-difference terms
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = i0 + orow, jx = j0 + oc0 + u;
        if (i >= H || jx >= W) continue;
        const int e = (orow + GLH) * GLR + oc0 + u + GLH;
        const float pv = P[e], tv = T[e];
        float g = 0.f;
        if (fl & 1) {
            const float d = pv - tv;
            acc[0] += fabsf(d);
            g += J.c_l1 * sgnf(d) / nhw;
        }
        if (fl & 16) {
            const float d = pv - J.t_const;
            acc[4] += (double)d * d;
            g += J.c_mse * 2.f * d / nhw;
        }
        if (fl & 2) {
            const float ix = J.c_grad / (float)((long long)J.nimg * H * (W - 1));
            const float iy = J.c_grad / (float)((long long)J.nimg * (H - 1) * W);
            if (jx + 1 < W) {
                const float dp = P[e + 1] - pv, dt = T[e + 1] - tv, ex = fabsf(dp) - fabsf(dt);
                acc[1] += fabsf(ex);
                g -= sgnf(ex) * sgnf(dp) * ix;
            }
            if (jx > 0) {
                const float dp = pv - P[e - 1], dt = tv - T[e - 1], ex = fabsf(dp) - fabsf(dt);
                g += sgnf(ex) * sgnf(dp) * ix;
            }
            if (i + 1 < H) {
                const float dp = P[e + GLR] - pv, dt = T[e + GLR] - tv, ey = fabsf(dp) - fabsf(dt);
                acc[2] += fabsf(ey);
                g -= sgnf(ey) * sgnf(dp) * iy;
            }
            if (i > 0) {
                const float dp = pv - P[e - GLR], dt = tv - T[e - GLR], ey = fabsf(dp) - fabsf(dt);
                g += sgnf(ey) * sgnf(dp) * iy;
            }
        }
        gout[u] = g;
    }

    if (fl & 8) {  // ContrastAttention: box means on the tile + 3 px, gmap, adjoint box onto the tile
        constexpr int CR = 3, CN = GLT + 2 * CR;  // 38
        float* tb = V;
        float* sb = V + CN * CN;
        float* gm = V + 2 * CN * CN;
        for (int e = tid; e < CN * CN; e += 256) {
            const int r = e / CN, c = e - r * CN;
            const int rr = r + GLH - CR, cc = c + GLH - CR;  // region coords of the box centre
            float st = 0.f, ss = 0.f, sp = 0.f;
            for (int dy = -CR; dy <= CR; ++dy)
                for (int dx = -CR; dx <= CR; ++dx) {
                    const int q = (rr + dy) * GLR + cc + dx;
                    st += T[q];
                    ss += S[q];
                    sp += P[q];
                }
            st *= 1.f / 49.f; ss *= 1.f / 49.f; sp *= 1.f / 49.f;
            const int y = i0 - CR + r, x = j0 - CR + c;
            const bool in = y >= 0 && y < H && x >= 0 && x < W;
            const float w = a.minw + (a.maxw - a.minw) * (1.f - expf(-fabsf(st - ss) / a.sigma));
            tb[e] = w * fabsf(sp - st);
            gm[e] = in ? w * sgnf(sp - st) / nhw : 0.f;
            sb[e] = in ? 1.f : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = i0 + orow, jx = j0 + oc0 + u;
            if (i >= H || jx >= W) continue;
            const int r = orow + CR, c = oc0 + u + CR;
            acc[4] += tb[r * CN + c];
            float s = 0.f;
            for (int dy = -CR; dy <= CR; ++dy)
                for (int dx = -CR; dx <= CR; ++dx) s += gm[(r + dy) * CN + c + dx];
            gout[u] += J.c_ca * s * (1.f / 49.f);
        }
        __syncthreads();
    }

    if (fl & 4) {  // SSIM, value + gradient (pytorch_msssim: valid gaussian, size_average)
        const int Hv = H - 10, Wv = W - 10;
        const float inv = 1.f / (float)((long long)J.nimg * Hv * Wv);
        // vertical valid pass: window positions r (q_y = i0 - 10 + r), all 52 columns
        for (int e = tid; e < GLQ * GLR; e += 256) {
            const int r = e / GLR, c = e - r * GLR;
            float m0 = 0.f, m1 = 0.f, m2 = 0.f, m3 = 0.f, m4 = 0.f;
#pragma unroll
            for (int q = 0; q < 11; ++q) {
                const float x = P[(r + q) * GLR + c], y = T[(r + q) * GLR + c], g = a.gw[q];
                m0 = fmaf(g, x, m0); m1 = fmaf(g, y, m1);
                m2 = fmaf(g, x * x, m2); m3 = fmaf(g, y * y, m3); m4 = fmaf(g, x * y, m4);
            }
            V[e] = m0; V[GLQ * GLR + e] = m1; V[2 * GLQ * GLR + e] = m2; V[3 * GLQ * GLR + e] = m3;
            V[4 * GLQ * GLR + e] = m4;
        }
        __syncthreads();
        // horizontal pass, ssim map and its derivative maps at the 42 x 42 window positions
        for (int e = tid; e < GLQ * GLQ; e += 256) {
            const int r = e / GLQ, c = e - r * GLQ;
            const int qy = i0 - GLH + r, qx = j0 - GLH + c;
            float m[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int q = 0; q < 11; ++q) {
                const float g = a.gw[q];
#pragma unroll
                for (int k = 0; k < 5; ++k) m[k] = fmaf(g, V[k * GLQ * GLR + r * GLR + c + q], m[k]);
            }
            const bool valid = qy >= 0 && qy < Hv && qx >= 0 && qx < Wv;
            float d0 = 0.f, d1 = 0.f, d2 = 0.f;
            if (valid) {
                const float mu1 = m[0], mu2 = m[1];
                const float s11 = m[2] - mu1 * mu1, s22 = m[3] - mu2 * mu2, s12 = m[4] - mu1 * mu2;
                const float A = 2.f * mu1 * mu2 + a.C1, B = mu1 * mu1 + mu2 * mu2 + a.C1;
                const float Cc = 2.f * s12 + a.C2, Dd = s11 + s22 + a.C2;
                const float s = (A / B) * (Cc / Dd);
                if (r >= GLH && c >= GLH) acc[3] += s;  // window positions this tile owns
                const float BD = B * Dd;
                d0 = (2.f * mu2 * (Cc - A) / BD - s * 2.f * mu1 * (1.f / B - 1.f / Dd)) * inv;
                d1 = (-s / Dd) * inv;
                d2 = (2.f * A / BD) * inv;
            }
            D[e] = d0; D[GLQ * GLQ + e] = d1; D[2 * GLQ * GLQ + e] = d2;
        }
        __syncthreads();
        // adjoint horizontal onto the tile's 32 columns (all 42 window rows): Tm[r][v]
        float* Tm = V;
        for (int e = tid; e < GLQ * GLT; e += 256) {
            const int r = e / GLT, v = e - r * GLT;
            float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int b = 0; b < 11; ++b) {
                const int c = v + GLH - b;
                const float g = a.gw[b];
                s0 = fmaf(g, D[r * GLQ + c], s0);
                s1 = fmaf(g, D[GLQ * GLQ + r * GLQ + c], s1);
                s2 = fmaf(g, D[2 * GLQ * GLQ + r * GLQ + c], s2);
            }
            Tm[e] = s0; Tm[GLQ * GLT + e] = s1; Tm[2 * GLQ * GLT + e] = s2;
        }
        __syncthreads();
        // adjoint vertical + chain rule: dX = R0 + 2 X R1 + Y R2
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int v = oc0 + u;
            float r0 = 0.f, r1 = 0.f, r2 = 0.f;
#pragma unroll
            for (int b = 0; b < 11; ++b) {
                const int r = orow + GLH - b;
                const float g = a.gw[b];
                r0 = fmaf(g, Tm[r * GLT + v], r0);
                r1 = fmaf(g, Tm[GLQ * GLT + r * GLT + v], r1);
                r2 = fmaf(g, Tm[2 * GLQ * GLT + r * GLT + v], r2);
            }
            const int e = (orow + GLH) * GLR + v + GLH;
            gout[u] += J.c_ssim * (r0 + 2.f * P[e] * r1 + T[e] * r2);
        }
    }

    // one write per pixel: the weighted term gradients + the batch-coupled terms' addends
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = i0 + orow, jx = j0 + oc0 + u;
        if (i >= H || jx >= W) continue;
        const long long o = base + (long long)i * W + jx;
        float g = gout[u];
        if (J.add0) g += J.c_add0 * J.add0[o];
        if (J.add1) g += J.c_add1 * J.add1[o];
        if (J.g) J.g[o] = g;
    }
    block_partials<5>(acc, part);
}

// term values per job (fixed-order sums of the tile partials) and the composed outputs:
// out[o] = bias[o] + sum_k coef[o][k] * val[k] + sum_x coef_x[o][x] * extra[x][0]
// val[5 j + q]: q = 0 L1 mean, 1 gradient-loss x mean, 2 y mean, 3 SSIM mean, 4 CA / MSE mean
constexpr int GL_MAXOUT = 12, GL_NEXTRA = 4;
constexpr int GL_FINAL_WAVES = 8;
struct GLRecipeK {
    float bias[GL_MAXOUT];
    float coef[GL_MAXOUT][GL_MAXJOB * 5];
    float coefx[GL_MAXOUT][GL_NEXTRA];
    const float* extra[GL_NEXTRA];
    int nout;
};
__global__ void gl_final_kernel(GLArgsK a, GLRecipeK rc, const double* __restrict__ part, float* __restrict__ out) {
    // one wave per job (jobs w, w + 8, ...); each lane sums the five terms of its blocks in a
    // fixed order, then a fixed-shape wave reduction: deterministic, 5 independent load streams
    __shared__ float val[GL_MAXJOB * 5];
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    for (int j = wv; j < a.njobs; j += GL_FINAL_WAVES) {
        const int H = a.j[j].H, W = a.j[j].W;
        const int b0 = a.j[j].blk0, nb = a.j[j].nimg * a.j[j].tiles;
        const double ni = a.j[j].nimg;
        const double nrm[5] = {ni * H * W, ni * H * (W - 1), ni * (H - 1) * W, ni * (H - 10) * (W - 10), ni * H * W};
        double s[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
        for (int b = ln; b < nb; b += 64) {
            const double* pp = part + (long long)(b0 + b) * 8;
#pragma unroll
            for (int q = 0; q < 5; ++q) s[q] += pp[q];
        }
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            const double t = wave_sum_d(s[q]);
            if (ln == 0) val[5 * j + q] = nrm[q] > 0 ? (float)(t / nrm[q]) : 0.f;
        }
    }
    __syncthreads();
    if (threadIdx.x < rc.nout) {
        const int o = threadIdx.x;
        float v = rc.bias[o];
        for (int k = 0; k < 5 * a.njobs; ++k) v += rc.coef[o][k] * val[k];
        for (int x = 0; x < GL_NEXTRA; ++x)
            if (rc.extra[x]) v += rc.coefx[o][x] * rc.extra[x][0];
        out[o] = v;
    }
}

}  // namespace dcs

using namespace dcs;

extern "C" size_t dcs_loss_workspace_size(int N, int H, int W) {
    if (N <= 0 || H <= 0 || W <= 0) return 0;
    size_t n = (size_t)N * H * W;
    return loss_ws_fixed() + 10 * n * sizeof(float) + 4096;
}

#define LOSS_CHECK_WS(N, H, W)                                                        \
    if (!ws || ws_bytes < dcs_loss_workspace_size(N, H, W))                           \
        return fail(DCS_E_WORKSPACE, "loss: workspace too small");

extern "C" int dcs_loss_l1(const float* pred, const float* target, int64_t n, float* out, float* grad, void* ws,
                           size_t ws_bytes, void* stream) {
    if (!pred || !target || !out || n <= 0) return fail(DCS_E_INVALID, "loss_l1: bad arguments");
    if (!ws || ws_bytes < loss_ws_fixed()) return fail(DCS_E_WORKSPACE, "loss_l1: workspace too small");
    LossWs w = loss_ws(ws);
    hipStream_t s = as_stream(stream);
    int nb = red_blocks(n);
    hipLaunchKernelGGL(pointwise_kernel<0>, dim3(nb), dim3(RB), 0, s, pred, target, 0.f, (long long)n, grad, w.part);
    hipLaunchKernelGGL(finalize_mean_kernel, dim3(1), dim3(64), 0, s, w.part, nb, (long long)n, out);
    return check_launch("loss_l1");
}

extern "C" int dcs_loss_mse(const float* pred, const float* target, int64_t n, float* out, float* grad, void* ws,
                            size_t ws_bytes, void* stream) {
    if (!pred || !target || !out || n <= 0) return fail(DCS_E_INVALID, "loss_mse: bad arguments");
    if (!ws || ws_bytes < loss_ws_fixed()) return fail(DCS_E_WORKSPACE, "loss_mse: workspace too small");
    LossWs w = loss_ws(ws);
    hipStream_t s = as_stream(stream);
    int nb = red_blocks(n);
    hipLaunchKernelGGL(pointwise_kernel<1>, dim3(nb), dim3(RB), 0, s, pred, target, 0.f, (long long)n, grad, w.part);
    hipLaunchKernelGGL(finalize_mean_kernel, dim3(1), dim3(64), 0, s, w.part, nb, (long long)n, out);
    return check_launch("loss_mse");
}

extern "C" int dcs_loss_mse_const(const float* pred, float target, int64_t n, float* out, float* grad, void* ws,
                                  size_t ws_bytes, void* stream) {
    if (!pred || !out || n <= 0) return fail(DCS_E_INVALID, "loss_mse_const: bad arguments");
    if (!ws || ws_bytes < loss_ws_fixed()) return fail(DCS_E_WORKSPACE, "loss_mse_const: workspace too small");
    LossWs w = loss_ws(ws);
    hipStream_t s = as_stream(stream);
    int nb = red_blocks(n);
    hipLaunchKernelGGL(pointwise_kernel<2>, dim3(nb), dim3(RB), 0, s, pred, nullptr, target, (long long)n, grad, w.part);
    hipLaunchKernelGGL(finalize_mean_kernel, dim3(1), dim3(64), 0, s, w.part, nb, (long long)n, out);
    return check_launch("loss_mse_const");
}

extern "C" int dcs_loss_gradient(const float* pred, const float* target, int N, int H, int W, float* out, float* grad,
                                 void* ws, size_t ws_bytes, void* stream) {
    if (!pred || !target || !out || N <= 0 || H < 2 || W < 2) return fail(DCS_E_INVALID, "loss_gradient: bad arguments");
    LOSS_CHECK_WS(N, H, W);
    LossWs w = loss_ws(ws);
    hipStream_t s = as_stream(stream);
    long long n = (long long)N * H * W;
    int nb = red_blocks(n);
    hipLaunchKernelGGL(gradient_loss_kernel, dim3(nb), dim3(RB), 0, s, pred, target, N, H, W, grad, w.part);
    hipLaunchKernelGGL(gradient_loss_final, dim3(1), dim3(64), 0, s, w.part, nb, N, H, W, out);
    return check_launch("loss_gradient");
}

extern "C" int dcs_loss_contrast_attention(const float* pred, const float* target, const float* source, int N, int H,
                                           int W, float sigma, float min_w, float max_w, int k, float* out,
                                           float* grad, void* ws, size_t ws_bytes, void* stream) {
    if (!pred || !target || !source || !out || N <= 0 || H <= 0 || W <= 0 || k <= 0 || (k & 1) == 0)
        return fail(DCS_E_INVALID, "loss_contrast_attention: bad arguments");
    LOSS_CHECK_WS(N, H, W);
    LossWs w = loss_ws(ws);
    hipStream_t s = as_stream(stream);
    long long n = (long long)N * H * W;
    int nb = red_blocks(n);
    float* gmap = w.maps;
    hipLaunchKernelGGL(ca_loss_kernel, dim3(nb), dim3(RB), 0, s, pred, target, source, N, H, W, sigma, min_w, max_w, k,
                       gmap, w.part);
    hipLaunchKernelGGL(finalize_mean_kernel, dim3(1), dim3(64), 0, s, w.part, nb, n, out);
    if (grad)
        hipLaunchKernelGGL(box_adjoint_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, gmap, N, H, W, k, grad);
    return check_launch("loss_contrast_attention");
}

extern "C" int dcs_loss_contrast_region(const float* pred, const float* target, const float* source, int N, int H,
                                        int W, float threshold, float weight, float* out, float* grad, void* ws,
                                        size_t ws_bytes, void* stream) {
    if (!pred || !target || !source || !out || N <= 0 || H <= 0 || W <= 0 || (long long)N * H * W < 2)
        return fail(DCS_E_INVALID, "loss_contrast_region: bad arguments");
    LOSS_CHECK_WS(N, H, W);
    LossWs w = loss_ws(ws);
    hipStream_t s = as_stream(stream);
    long long n = (long long)N * H * W;
    long long nq = (long long)N * (H / 8) * (W / 8);
    int nb = red_blocks(n);
    float* gq = w.maps;
    hipLaunchKernelGGL(cr_loss_kernel, dim3(nb), dim3(RB), 0, s, pred, target, source, N, H, W, threshold, gq, w.part,
                       nq);
    hipLaunchKernelGGL(cr_loss_final, dim3(1), dim3(64), 0, s, w.part, nb, n, nq, weight, w.sc, out);
    if (grad)
        hipLaunchKernelGGL(cr_grad_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, pred, gq, w.sc, N, H, W, weight,
                           grad);
    return check_launch("loss_contrast_region");
}

extern "C" int dcs_loss_contrast_edge(const float* pred, const float* target, int N, int H, int W, float* out,
                                      float* grad, void* ws, size_t ws_bytes, void* stream) {
    if (!pred || !target || !out || N <= 0 || H <= 0 || W <= 0) return fail(DCS_E_INVALID, "loss_contrast_edge: bad arguments");
    LOSS_CHECK_WS(N, H, W);
    const long long n = (long long)N * H * W;
    const long long k = (long long)((double)n * 0.1);  // int(numel * 0.1)
    if (k < 1 || n < 2) return fail(DCS_E_INVALID, "loss_contrast_edge: too few elements for top-10%");
    LossWs w = loss_ws(ws);
    hipStream_t s = as_stream(stream);
    float* ep = w.maps;
    float* et = ep + n;
    float* gx = et + n;
    float* gy = gx + n;
    int nb = red_blocks(n);
    double* part_stats = w.part;  // slots 0-3 of each block row
    hipLaunchKernelGGL(edge_maps_kernel, dim3(nb), dim3(RB), 0, s, pred, target, N, H, W, ep, et, part_stats);
    int e = check_launch("edge_maps");
    if (e) return e;
    unsigned* stp = w.st;
    unsigned* stt = w.st + 4;
    double* part_tp = w.part + 4;  // slots 4-5 of each block row (stats use 0-3)
    double* part_tt = w.part + 6;  // slots 6-7
    const float* srcs[2] = {ep, et};
    unsigned* sts[2] = {stp, stt};
    double* parts[2] = {part_tp, part_tt};
    for (int q = 0; q < 2; ++q) {
        hipLaunchKernelGGL(radix_init_kernel, dim3(1), dim3(256), 0, s, sts[q], (unsigned)k, w.hist);
        for (int shift = 24; shift >= 0; shift -= 8) {
            hipLaunchKernelGGL(radix_hist_kernel, dim3(nb), dim3(RB), 0, s, srcs[q], n, shift, sts[q], w.hist);
            hipLaunchKernelGGL(radix_select_kernel, dim3(1), dim3(256), 0, s, sts[q], shift, w.hist);
        }
        hipLaunchKernelGGL(topk_sum_kernel, dim3(nb), dim3(RB), 0, s, srcs[q], n, sts[q], parts[q]);
    }
    if ((e = check_launch("edge_topk"))) return e;
    hipLaunchKernelGGL(edge_final_kernel, dim3(1), dim3(64), 0, s, part_stats, nb, part_tp, nb, part_tt, nb, stp, stt, n,
                       k, w.sc, out);
    if (grad) {
        hipLaunchKernelGGL(edge_grad_maps_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, pred, ep, w.sc, N, H, W,
                           gx, gy);
        hipLaunchKernelGGL(edge_grad_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, gx, gy, N, H, W, grad);
    }
    return check_launch("loss_contrast_edge");
}

extern "C" int dcs_loss_contrast_region_partial(const float* pred, const float* target, const float* source, int N,
                                                int H, int W, float threshold, double* red, void* ws, size_t ws_bytes,
                                                void* stream) {
    if (!pred || !target || !source || !red || N <= 0 || H <= 0 || W <= 0)
        return fail(DCS_E_INVALID, "loss_contrast_region_partial: bad arguments");
    LOSS_CHECK_WS(N, H, W);
    LossWs w = loss_ws(ws);
    hipStream_t s = as_stream(stream);
    const long long n = (long long)N * H * W, nq = (long long)N * (H / 8) * (W / 8);
    const int nb = red_blocks(n);
    // gq = m * sign(p - t), unnormalised: the batch's nq is only known after the reduction
    hipLaunchKernelGGL(cr_loss_kernel, dim3(nb), dim3(RB), 0, s, pred, target, source, N, H, W, threshold, w.maps,
                       w.part, 0LL);
    hipLaunchKernelGGL(red_sum_kernel, dim3(1), dim3(64), 0, s, w.part, nb, 5, red, 0, (double)n, (double)nq, 2);
    return check_launch("loss_contrast_region_partial");
}

extern "C" int dcs_loss_contrast_region_finish(const float* pred, int N, int H, int W, float weight, const double* red,
                                               float grad_scale, float* out, float* grad, void* ws, size_t ws_bytes,
                                               void* stream) {
    if (!pred || !red || !out || N <= 0 || H <= 0 || W <= 0)
        return fail(DCS_E_INVALID, "loss_contrast_region_finish: bad arguments");
    LOSS_CHECK_WS(N, H, W);
    LossWs w = loss_ws(ws);
    hipStream_t s = as_stream(stream);
    const long long n = (long long)N * H * W;
    hipLaunchKernelGGL(cr_final_red_kernel, dim3(1), dim3(64), 0, s, red, weight, grad_scale, w.sc, out);
    if (grad)
        hipLaunchKernelGGL(cr_grad_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, pred, w.maps, w.sc, N, H, W,
                           weight, grad);
    return check_launch("loss_contrast_region_finish");
}

extern "C" int dcs_loss_contrast_edge_partial(const float* pred, const float* target, int N, int H, int W, double* red,
                                              void* ws, size_t ws_bytes, void* stream) {
    if (!pred || !target || !red || N <= 0 || H <= 0 || W <= 0)
        return fail(DCS_E_INVALID, "loss_contrast_edge_partial: bad arguments");
    LOSS_CHECK_WS(N, H, W);
    LossWs w = loss_ws(ws);
    hipStream_t s = as_stream(stream);
    const long long n = (long long)N * H * W;
    const int nb = red_blocks(n);
    float* ep = w.maps;
    hipLaunchKernelGGL(edge_maps_kernel, dim3(nb), dim3(RB), 0, s, pred, target, N, H, W, ep, ep + n, w.part);
    hipLaunchKernelGGL(red_sum_kernel, dim3(1), dim3(64), 0, s, w.part, nb, 4, red, 0, (double)n, 0.0, 1);
    return check_launch("loss_contrast_edge_partial");
}

extern "C" int dcs_loss_contrast_edge_hist(int N, int H, int W, int pass, const double* red, uint32_t* hist, void* ws,
                                           size_t ws_bytes, void* stream) {
    if (!red || !hist || N <= 0 || H <= 0 || W <= 0 || pass < 0 || pass > 3)
        return fail(DCS_E_INVALID, "loss_contrast_edge_hist: bad arguments (pass 0..3)");
    LOSS_CHECK_WS(N, H, W);
    LossWs w = loss_ws(ws);
    hipStream_t s = as_stream(stream);
    const long long n = (long long)N * H * W;
    const int nb = red_blocks(n);
    if (pass == 0) hipLaunchKernelGGL(edge_radix_init_kernel, dim3(1), dim3(64), 0, s, w.st, w.st + 4, red);
    const hipError_t me = hipMemsetAsync(hist, 0, 512 * sizeof(uint32_t), s);
    if (me != hipSuccess) return fail((int)me, "loss_contrast_edge_hist: memset failed");
    const int shift = 24 - 8 * pass;
    hipLaunchKernelGGL(radix_hist_kernel, dim3(nb), dim3(RB), 0, s, w.maps, n, shift, w.st, hist);
    hipLaunchKernelGGL(radix_hist_kernel, dim3(nb), dim3(RB), 0, s, w.maps + n, n, shift, w.st + 4, hist + 256);
    return check_launch("loss_contrast_edge_hist");
}

extern "C" int dcs_loss_contrast_edge_select(int pass, const uint32_t* hist, void* ws, size_t ws_bytes, void* stream) {
    if (!hist || !ws || ws_bytes < loss_ws_fixed() || pass < 0 || pass > 3)
        return fail(DCS_E_INVALID, "loss_contrast_edge_select: bad arguments (pass 0..3)");
    LossWs w = loss_ws(ws);
    hipStream_t s = as_stream(stream);
    const int shift = 24 - 8 * pass;
    hipLaunchKernelGGL(radix_select_const_kernel, dim3(1), dim3(64), 0, s, w.st, shift, hist);
    hipLaunchKernelGGL(radix_select_const_kernel, dim3(1), dim3(64), 0, s, w.st + 4, shift, hist + 256);
    return check_launch("loss_contrast_edge_select");
}

extern "C" int dcs_loss_contrast_edge_topk(int N, int H, int W, double* red, void* ws, size_t ws_bytes, void* stream) {
    if (!red || N <= 0 || H <= 0 || W <= 0) return fail(DCS_E_INVALID, "loss_contrast_edge_topk: bad arguments");
    LOSS_CHECK_WS(N, H, W);
    LossWs w = loss_ws(ws);
    hipStream_t s = as_stream(stream);
    const long long n = (long long)N * H * W;
    const int nb = red_blocks(n);
    hipLaunchKernelGGL(topk_sum_kernel, dim3(nb), dim3(RB), 0, s, w.maps, n, w.st, w.part);
    hipLaunchKernelGGL(red_sum_kernel, dim3(1), dim3(64), 0, s, w.part, nb, 2, red, 5, 0.0, 0.0, 0);
    hipLaunchKernelGGL(topk_sum_kernel, dim3(nb), dim3(RB), 0, s, w.maps + n, n, w.st + 4, w.part);
    hipLaunchKernelGGL(red_sum_kernel, dim3(1), dim3(64), 0, s, w.part, nb, 2, red, 7, 0.0, 0.0, 0);
    return check_launch("loss_contrast_edge_topk");
}

extern "C" int dcs_loss_contrast_edge_finish(const float* pred, int N, int H, int W, const double* red,
                                             float grad_scale, float* out, float* grad, void* ws, size_t ws_bytes,
                                             void* stream) {
    if (!pred || !red || !out || N <= 0 || H <= 0 || W <= 0)
        return fail(DCS_E_INVALID, "loss_contrast_edge_finish: bad arguments");
    LOSS_CHECK_WS(N, H, W);
    LossWs w = loss_ws(ws);
    hipStream_t s = as_stream(stream);
    const long long n = (long long)N * H * W;
    float* ep = w.maps;
    float* gx = ep + 2 * n;
    float* gy = gx + n;
    hipLaunchKernelGGL(edge_final_red_kernel, dim3(1), dim3(64), 0, s, red, w.st, w.st + 4, grad_scale, w.sc, out);
    if (grad) {
        hipLaunchKernelGGL(edge_grad_maps_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, pred, ep, w.sc, N, H, W,
                           gx, gy);
        hipLaunchKernelGGL(edge_grad_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, gx, gy, N, H, W, grad);
    }
    return check_launch("loss_contrast_edge_finish");
}

extern "C" int dcs_loss_ssim(const float* X, const float* Y, int N, int H, int W, float data_range, int win,
                             float sigma, float k1, float k2, float* out, float* grad, void* ws, size_t ws_bytes,
                             void* stream) {
    if (!X || !Y || !out || N <= 0 || win <= 0 || win > 16 || (win & 1) == 0 || H < win || W < win)
        return fail(DCS_E_INVALID, "loss_ssim: bad arguments (H, W >= win required)");
    LOSS_CHECK_WS(N, H, W);
    LossWs w = loss_ws(ws);
    hipStream_t s = as_stream(stream);
    Gauss G = make_gauss(win, sigma);
    const int Hv = H - win + 1, Wv = W - win + 1;
    const long long totv = (long long)N * Hv * W, tot = (long long)N * Hv * Wv;
    float* V = w.maps;            // 5 * totv
    float* D = V + 5 * totv;      // 3 * tot
    float* T = V;                 // reuse V for the adjoint pass (3 * totv)
    const float C1 = (k1 * data_range) * (k1 * data_range), C2 = (k2 * data_range) * (k2 * data_range);
    hipLaunchKernelGGL(ssim_v_kernel, dim3((unsigned)cdiv(totv, 256)), dim3(256), 0, s, X, Y, N, H, W, win, G, V);
    int nb = red_blocks(tot);
    hipLaunchKernelGGL(ssim_h_kernel, dim3(nb), dim3(RB), 0, s, V, N, H, W, win, G, C1, C2, D, w.part);
    hipLaunchKernelGGL(ssim_final, dim3(1), dim3(64), 0, s, w.part, nb, tot, out);
    if (grad) {
        hipLaunchKernelGGL(ssim_ht_kernel, dim3((unsigned)cdiv(totv, 256)), dim3(256), 0, s, D, N, H, W, win, G, T);
        hipLaunchKernelGGL(ssim_vt_kernel, dim3((unsigned)cdiv((long long)N * H * W, 256)), dim3(256), 0, s, T, X, Y, N,
                           H, W, win, G, grad);
    }
    return check_launch("loss_ssim");
}

extern "C" size_t dcs_gen_loss_fused_ws(const dcs_gl_job* jobs, int njobs) {
    if (!jobs || njobs <= 0 || njobs > GL_MAXJOB) return 0;
    long long blocks = 0;
    for (int j = 0; j < njobs; ++j) blocks += (long long)jobs[j].n_img * cdiv(jobs[j].H, GLT) * cdiv(jobs[j].W, GLT);
    return (size_t)blocks * 8 * sizeof(double) + 256;
}

extern "C" int dcs_gen_loss_fused(const dcs_gl_job* jobs, int njobs, float ssim_data_range, float ca_sigma,
                                  float ca_min_w, float ca_max_w, const float* bias, const float* coef,
                                  const float* coefx, const float* const* extra, int nout, float* out, void* ws,
                                  size_t ws_bytes, void* stream) {
    if (!jobs || njobs <= 0 || njobs > GL_MAXJOB || nout < 0 || nout > GL_MAXOUT || (nout > 0 && (!out || !bias || !coef)))
        return fail(DCS_E_INVALID, "gen_loss_fused: bad arguments");
    if (!ws || ws_bytes < dcs_gen_loss_fused_ws(jobs, njobs)) return fail(DCS_E_WORKSPACE, "gen_loss_fused: workspace too small");
    GLArgsK a{};
    a.njobs = njobs;
    int blk = 0;
    for (int j = 0; j < njobs; ++j) {
        const dcs_gl_job& s = jobs[j];
        GLJobK& k = a.j[j];
        if (!s.pred || s.n_img <= 0 || s.H < 2 || s.W < 2) return fail(DCS_E_INVALID, "gen_loss_fused: bad job");
        if ((s.flags & ~31) || ((s.flags & (1 | 2 | 4 | 8)) && !s.target) || ((s.flags & 8) && !s.source) ||
            ((s.flags & 4) && (s.H < 11 || s.W < 11)) || ((s.flags & 8) && (s.flags & 16)))
            return fail(DCS_E_INVALID, "gen_loss_fused: bad job flags");
        k.p = s.pred; k.t = s.target; k.s = s.source; k.add0 = s.add0; k.add1 = s.add1; k.g = s.grad;
        k.nimg = s.n_img; k.flags = s.flags; k.H = s.H; k.W = s.W;
        k.tiles_x = (int)cdiv(s.W, GLT);
        k.tiles = k.tiles_x * (int)cdiv(s.H, GLT);
        k.blk0 = blk;
        blk += k.nimg * k.tiles;
        k.c_l1 = s.c_l1; k.c_grad = s.c_grad; k.c_ssim = s.c_ssim; k.c_ca = s.c_ca; k.c_mse = s.c_mse;
        k.t_const = s.t_const; k.c_add0 = s.c_add0; k.c_add1 = s.c_add1;
    }
    // pytorch_msssim: 11-tap gaussian, sigma 1.5, K = (0.01, 0.03)
    float gs = 0.f;
    for (int i = 0; i < 11; ++i) {
        const float c = (float)(i - 5);
        a.gw[i] = expf(-(c * c) / (2.f * 1.5f * 1.5f));
        gs += a.gw[i];
    }
    for (int i = 0; i < 11; ++i) a.gw[i] /= gs;
    a.gw[11] = 0.f;
    a.C1 = (0.01f * ssim_data_range) * (0.01f * ssim_data_range);
    a.C2 = (0.03f * ssim_data_range) * (0.03f * ssim_data_range);
    a.sigma = ca_sigma; a.minw = ca_min_w; a.maxw = ca_max_w;
    double* part = reinterpret_cast<double*>(ws);
    hipStream_t s = as_stream(stream);
    hipLaunchKernelGGL(gl_planes_kernel, dim3((unsigned)blk), dim3(256), 0, s, a, part);
    if (nout > 0) {
        GLRecipeK rc{};
        rc.nout = nout;
        for (int o = 0; o < nout; ++o) {
            rc.bias[o] = bias[o];
            for (int k = 0; k < 5 * njobs; ++k) rc.coef[o][k] = coef[o * 5 * njobs + k];
            for (int x = 0; x < GL_NEXTRA; ++x) rc.coefx[o][x] = coefx ? coefx[o * GL_NEXTRA + x] : 0.f;
        }
        for (int x = 0; x < GL_NEXTRA; ++x) rc.extra[x] = extra ? extra[x] : nullptr;
        hipLaunchKernelGGL(gl_final_kernel, dim3(1), dim3(64 * GL_FINAL_WAVES), 0, s, a, rc, part, out);
    }
    return check_launch("gen_loss_fused");
}
