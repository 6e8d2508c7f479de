// Error state, Adam (torch.optim.Adam semantics, modules/trainer.py:360-362) and small utilities.
#include "common.hpp"

namespace dcs {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

// registered range-record arenas (dcs_range_arena_register): [base, base + bytes)
namespace {
constexpr int ARENA_MAX = 32;
struct ArenaRange {
    uintptr_t lo, hi;
};
ArenaRange g_arenas[ARENA_MAX];
int g_narena = 0;
}  // namespace
bool in_range_arena(const void* p) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    for (int i = 0; i < g_narena; ++i)
        if (a >= g_arenas[i].lo && a < g_arenas[i].hi) return true;
    return false;
}

// One launch over the flat parameter buffer of an optimizer.  Matches torch's Adam
// (amsgrad=False, weight_decay=0):
//   m = lerp(m, g, 1-b1);  v = b2*v + (1-b2)*g*g;
//   p -= (lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps)
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, long long n, float lr, float b1, float b2, float eps,
                            float bc1, float bc2) {
    const float step_size = lr / bc1;
    const float bc2s = sqrtf(bc2);
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        float gi = g[i];
        float mi = m[i];
        mi = mi + (1.f - b1) * (gi - mi);
        float vi = fmaf(v[i], b2, (1.f - b2) * gi * gi);
        m[i] = mi;
        v[i] = vi;
        float denom = sqrtf(vi) / bc2s + eps;
        p[i] = p[i] - step_size * (mi / denom);
    }
}

__global__ void scale_add_kernel(float* __restrict__ y, const float* __restrict__ x, float a, long long n) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        y[i] = fmaf(a, x[i], y[i]);
}

}  // namespace dcs

using namespace dcs;


// ---------------------------------------------------------------------------------------
// range record of an f16x3 operand (include/ducosy_hip.h dcs_range_parts): block b of
// DCS_RANGE_PARTS reduces max |act(x * scale + shift)| (or |x|) over its contiguous share of
// the tensor's float4s; the f16x3 conv kernels reduce the DCS_RANGE_PARTS partials themselves
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(512) void range_parts_kernel(const float* __restrict__ x, long long n4, long long per_img,
                                                          int C, const float* __restrict__ sc,
                                                          const float* __restrict__ sh, int act,
                                                          float* __restrict__ parts) {
    const long long per_blk = (n4 + gridDim.x - 1) / gridDim.x;
    const long long beg = (long long)blockIdx.x * per_blk;
    const long long end = beg + per_blk < n4 ? beg + per_blk : n4;
    const float4* x4 = reinterpret_cast<const float4*>(x);
    float m = 0.f;
    auto fold = [&](float4 v, long long i) {
        if (sc) {
            const long long e = i * 4;
            const long long img = e / per_img;
            const int c = (int)(e % C);
            const float4 s = *reinterpret_cast<const float4*>(sc + img * C + c);
            const float4 h = *reinterpret_cast<const float4*>(sh + img * C + c);
            v.x = act_apply(fmaf(v.x, s.x, h.x), act);
            v.y = act_apply(fmaf(v.y, s.y, h.y), act);
            v.z = act_apply(fmaf(v.z, s.z, h.z), act);
            v.w = act_apply(fmaf(v.w, s.w, h.w), act);
        }
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    };
    long long i = beg + threadIdx.x;
    for (; i + 3 * 512 < end; i += 4 * 512) {  // four loads in flight per thread
        const float4 a = x4[i], b = x4[i + 512], c = x4[i + 1024], d = x4[i + 1536];
        fold(a, i); fold(b, i + 512); fold(c, i + 1024); fold(d, i + 1536);
    }
    for (; i < end; i += 512) fold(x4[i], i);
    __shared__ float red[8];
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float r = red[0];
        for (int w = 1; w < 8; ++w) r = fmaxf(r, red[w]);
        parts[blockIdx.x] = r;
    }
}

extern "C" const char* dcs_last_error(void) { return g_last_error.c_str(); }
extern "C" int dcs_version(void) { return 1; }

extern "C" int dcs_adam_step(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                             float beta2, float eps, float bias_c1, float bias_c2, void* stream) {
    if (!p || !g || !m || !v || n < 0) return fail(DCS_E_INVALID, "adam: bad arguments");
    if (n == 0) return DCS_OK;
    long long blocks = cdiv(n, 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), p, g, m, v, (long long)n,
                       lr, beta1, beta2, eps, bias_c1, bias_c2);
    return check_launch("adam");
}

extern "C" int dcs_scale_add(float* y, const float* x, float a, int64_t n, void* stream) {
    if (!y || !x || n < 0) return fail(DCS_E_INVALID, "scale_add: bad arguments");
    if (n == 0) return DCS_OK;
    long long blocks = cdiv(n, 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(scale_add_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), y, x, a, (long long)n);
    return check_launch("scale_add");
}

namespace dcs {

// dy = da * act'(y) for a = act(y) given the PRE-activation y (relu/lrelu), or given the
// OUTPUT y for tanh (a = tanh(.), da/dpre = 1 - a^2).
__global__ void act_backward_kernel(const float* __restrict__ da, const float* __restrict__ y,
                                    float* __restrict__ dy, long long n, int act, float* __restrict__ rng) {
    float m = 0.f;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        float v = y[i];
        float g = act == DCS_ACT_TANH ? (1.f - v * v) : act_grad(v, act);
        const float o = da[i] * g;
        dy[i] = o;
        m = fmaxf(m, fabsf(o));
    }
    range_note(rng, m);
}

// out = x * (*s)   (s a device scalar: loss backward without a host sync)
__global__ void scale_dev_kernel(const float* __restrict__ x, const float* __restrict__ s, float* __restrict__ out,
                                 long long n) {
    const float a = s[0];
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        out[i] = x[i] * a;
}

// per-channel sums of an [P][C] tensor: partials over pixel chunks, fixed-order finalize
__global__ __launch_bounds__(256) void channel_sum_partial_kernel(const float* __restrict__ x, long long P, int C,
                                                                  int nchunk, float* __restrict__ part) {
    const int chunk = blockIdx.y;
    const long long per = (P + nchunk - 1) / nchunk;
    const long long p0 = chunk * per;
    const long long p1 = min(P, p0 + per);
    for (int c = blockIdx.x * 256 + threadIdx.x; c < C; c += gridDim.x * 256) {
        float s = 0.f;
        for (long long p = p0; p < p1; ++p) s += x[p * C + c];
        part[(long long)chunk * C + c] = s;
    }
}

// per-channel sums for C a power of two <= 256: the tensor is read as flat 1024-float groups
// (a float4 per thread, coalesced); element 4t+k of a group is channel (4t+k) % C in every group,
// so each thread keeps 4 running sums and a fixed LDS tree folds them to C values per chunk
__global__ __launch_bounds__(256) void channel_sum_flat_kernel(const float* __restrict__ x, long long n, int C,
                                                               long long groups_per_chunk, float* __restrict__ part) {
    __shared__ float red[1024];
    const int t = threadIdx.x;
    const long long g0 = (long long)blockIdx.x * groups_per_chunk;
    long long g1 = g0 + groups_per_chunk;
    const long long ng = (n + 1023) / 1024;
    if (g1 > ng) g1 = ng;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (long long g = g0; g < g1; ++g) {
        const long long i = g * 1024 + 4 * t;
        float4 v;
        if (i + 3 < n) {
            v = *reinterpret_cast<const float4*>(x + i);
        } else {
            v.x = i < n ? x[i] : 0.f;
            v.y = i + 1 < n ? x[i + 1] : 0.f;
            v.z = i + 2 < n ? x[i + 2] : 0.f;
            v.w = 0.f;
        }
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    red[4 * t] = acc.x; red[4 * t + 1] = acc.y; red[4 * t + 2] = acc.z; red[4 * t + 3] = acc.w;
    __syncthreads();
    for (int stride = 512; stride >= C; stride >>= 1) {
        for (int i = t; i < stride; i += 256) red[i] += red[i + stride];
        __syncthreads();
    }
    if (t < C) part[(long long)blockIdx.x * C + t] = red[t];
}

// one wave per channel: lane l sums chunks l, l+64, ... in order, then a fixed butterfly
__global__ __launch_bounds__(64) void channel_sum_final_kernel(const float* __restrict__ part, int C, int nchunk,
                                                               float* __restrict__ out) {
    const int c = blockIdx.x;
    double s = 0.0;
    for (int k = threadIdx.x; k < nchunk; k += 64) s += part[(long long)k * C + c];
    s = wave_sum_d(s);
    if (threadIdx.x == 0) out[c] = (float)s;
}

static inline int csum_chunks(long long P) {
    long long c = cdiv(P, 256);
    if (c > 1024) c = 1024;
    if (c < 1) c = 1;
    return (int)c;
}

}  // namespace dcs

extern "C" int dcs_act_backward(const float* da, const float* y, float* dy, int64_t n, int act, float* rng,
                                void* stream) {
    if (!da || !y || !dy || n < 0) return fail(DCS_E_INVALID, "act_backward: bad arguments");
    if (int e = range_zero(rng, as_stream(stream))) return e;
    if (n == 0) return DCS_OK;
    long long blocks = cdiv(n, 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(act_backward_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), da, y, dy,
                       (long long)n, act, rng);
    return check_launch("act_backward");
}

extern "C" int dcs_scale_dev(const float* x, const float* s, float* out, int64_t n, void* stream) {
    if (!x || !s || !out || n < 0) return fail(DCS_E_INVALID, "scale_dev: bad arguments");
    if (n == 0) return DCS_OK;
    long long blocks = cdiv(n, 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(scale_dev_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), x, s, out,
                       (long long)n);
    return check_launch("scale_dev");
}

extern "C" size_t dcs_channel_sum_workspace_size(int64_t P, int C) {
    if (P <= 0 || C <= 0) return 0;
    return (size_t)csum_chunks(P) * C * sizeof(float);
}

extern "C" int dcs_channel_sum(const float* x, int64_t P, int C, float* out, void* ws, size_t ws_bytes,
                               void* stream) {
    if (!x || !out || !ws || P <= 0 || C <= 0) return fail(DCS_E_INVALID, "channel_sum: bad arguments");
    if (ws_bytes < dcs_channel_sum_workspace_size(P, C)) return fail(DCS_E_WORKSPACE, "channel_sum: workspace too small");
    int nch = csum_chunks(P);
    hipStream_t s = as_stream(stream);
    const long long n = (long long)P * C;
    if (C <= 256 && (C & (C - 1)) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
        // flat pass: chunks of whole 1024-float groups, at most csum_chunks(P) of them
        const long long ng = cdiv(n, 1024);
        long long want = cdiv(ng, 4);
        if (want > nch) want = nch;
        const long long gpc = cdiv(ng, want);
        nch = (int)cdiv(ng, gpc);
        hipLaunchKernelGGL(channel_sum_flat_kernel, dim3((unsigned)nch), dim3(256), 0, s, x, n, C, gpc,
                           reinterpret_cast<float*>(ws));
    } else {
        hipLaunchKernelGGL(channel_sum_partial_kernel, dim3((unsigned)cdiv(C, 256), nch), dim3(256), 0, s, x,
                           (long long)P, C, nch, reinterpret_cast<float*>(ws));
    }
    int e = check_launch("channel_sum_partial");
    if (e) return e;
    hipLaunchKernelGGL(channel_sum_final_kernel, dim3((unsigned)C), dim3(64), 0, s,
                       reinterpret_cast<const float*>(ws), C, nch, out);
    return check_launch("channel_sum_final");
}

extern "C" int dcs_range_parts(const float* x, int n_img, int64_t per_img, int C, const float* scale, const float* shift,
                               int act, float* parts, void* stream) {
    if (!x || !parts || n_img <= 0 || per_img <= 0 || per_img % 4 || (reinterpret_cast<uintptr_t>(x) & 15))
        return fail(DCS_E_INVALID, "range_parts: bad arguments (per_img % 4 == 0, 16-byte aligned x)");
    if ((scale != nullptr) != (shift != nullptr) || (scale && (C <= 0 || C % 4 || per_img % C)))
        return fail(DCS_E_INVALID, "range_parts: the prologue needs scale and shift, C % 4 == 0 and per_img % C == 0");
    if (!scale && act != DCS_ACT_NONE) return fail(DCS_E_INVALID, "range_parts: act without a prologue");
    hipLaunchKernelGGL(range_parts_kernel, dim3(DCS_RANGE_PARTS), dim3(512), 0, as_stream(stream), x,
                       (long long)n_img * per_img / 4, (long long)per_img, C, scale, shift, act, parts);
    return check_launch("range_parts");
}

// ---------------------------------------------------------------------------------------
// dst[i] += src[i] over a list of tensors in one launch (the second contribution to parameter
// gradients a model called twice in one step receives: one launch instead of one add per tensor)
// ---------------------------------------------------------------------------------------
namespace {
constexpr int MA_MAX = 64;
struct MultiAddArgs {
    const float* src[MA_MAX];
    float* dst[MA_MAX];
    long long n[MA_MAX];
    int count;
};
__global__ __launch_bounds__(256) void multi_add_kernel(MultiAddArgs a) {
    const int t = blockIdx.y;
    if (t >= a.count) return;  // block-uniform
    const long long n = a.n[t];
    const float* __restrict__ s = a.src[t];
    float* __restrict__ d = a.dst[t];
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) d[i] += s[i];
}
}  // namespace

extern "C" int dcs_multi_add(int count, const float* const* src, float* const* dst, const int64_t* n, void* stream) {
    if (count < 0 || (count > 0 && (!src || !dst || !n))) return fail(DCS_E_INVALID, "multi_add: bad arguments");
    for (int c0 = 0; c0 < count; c0 += MA_MAX) {
        MultiAddArgs a{};
        a.count = count - c0 < MA_MAX ? count - c0 : MA_MAX;
        long long mx = 1;
        for (int i = 0; i < a.count; ++i) {
            if (!src[c0 + i] || !dst[c0 + i] || n[c0 + i] < 0) return fail(DCS_E_INVALID, "multi_add: bad tensor");
            a.src[i] = src[c0 + i];
            a.dst[i] = dst[c0 + i];
            a.n[i] = n[c0 + i];
            mx = n[c0 + i] > mx ? n[c0 + i] : mx;
        }
        const unsigned gx = (unsigned)(cdiv(mx, 256) < 1024 ? cdiv(mx, 256) : 1024);
        hipLaunchKernelGGL(multi_add_kernel, dim3(gx, (unsigned)a.count), dim3(256), 0, as_stream(stream), a);
        const int e = check_launch("multi_add");
        if (e) return e;
    }
    return DCS_OK;
}

extern "C" int dcs_range_arena_register(const void* base, size_t bytes) {
    if (!base || bytes == 0) return fail(DCS_E_INVALID, "range_arena_register: bad arguments");
    const uintptr_t lo = reinterpret_cast<uintptr_t>(base);
    for (int i = 0; i < g_narena; ++i)
        if (g_arenas[i].lo == lo) {
            g_arenas[i].hi = lo + bytes;
            return DCS_OK;
        }
    if (g_narena >= ARENA_MAX) return fail(DCS_E_INVALID, "range_arena_register: too many arenas");
    g_arenas[g_narena++] = {lo, lo + bytes};
    return DCS_OK;
}

extern "C" int dcs_range_arena_unregister(const void* base) {
    const uintptr_t lo = reinterpret_cast<uintptr_t>(base);
    for (int i = 0; i < g_narena; ++i)
        if (g_arenas[i].lo == lo) {
            g_arenas[i] = g_arenas[--g_narena];
            return DCS_OK;
        }
    return fail(DCS_E_INVALID, "range_arena_unregister: not registered");
}
