// Input pipeline of a DuCoSy-GAN training batch on gfx950: the HU transform with soft
// squeezing (modules/preprocess.py:6-55) and the HU-threshold anatomical masks
// (modules/mask_generator.py:11-347) for a batch of 2-D slices, as modules/dataset.py:109-181
// consumes them (one NCCT slice -> masks in mask_types order, concatenated on channels).
//
// All of it is integer / byte work bounded by HBM and atomics, never a GEMM:
//   * threshold passes write one flag byte per pixel (F_* bits below);
//   * connected components (scipy.ndimage.label, 4-connectivity in 2-D) are a lock-free
//     union-find (Playne & Hawick 2018): per 4096-pixel tile in LDS, then across tile
//     borders in global memory, then path compression with wave-aggregated size counting;
//   * binary_fill_holes = background components (4-connected) that touch no image edge;
//   * the lung convex hull (scipy ConvexHull -> matplotlib Path.contains_points) is Andrew's
//     monotone chain over the per-row extreme lung pixels (the only possible hull vertices),
//     counter-clockwise like qhull's 2-D output, and the per-pixel inside test is matplotlib's
//     crossing-number rule (point_in_path, _path.h) in exact integer arithmetic.
#include "common.hpp"

namespace dcs {

enum : uint8_t {
    F_LUNGC = 1,    // lung HU window, inside body, away from the border margin
    F_LUNG = 2,     // ... and in a component of >= min_size pixels (detect_lung)
    F_INSIDE = 4,   // inside the lung convex hull (crossing rule)
    F_SEED = 8,     // bone candidate that survives the mediastinal-vessel exclusion
    F_ABONE = 16,   // all bone candidates (hu >= bone_threshold, inside body)
    F_BONE = 32,    // after region growing (components of F_ABONE holding a seed)
    F_MEDI = 64,    // mediastinum
    F_VES = 128,    // lung vessels
};

struct SliceInfo {
    int body, lung_area, nreg, cond, hull_ok, nv, pad0, pad1;
};

constexpr int MT = 256;

__device__ __forceinline__ int ld_relaxed(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int uf_find(const int* L, int x) {
    int p = ld_relaxed(L + x);
    while (p != x) {
        x = p;
        p = ld_relaxed(L + x);
    }
    return x;
}

// Parents only ever decrease (atomicMin), so stale reads are safe: the atomic returns the
// current value and the loop retries from it.
__device__ __forceinline__ void uf_union(int* L, int a, int b) {
    bool done;
    do {
        a = uf_find(L, a);
        b = uf_find(L, b);
        if (a < b) {
            const int old = atomicMin(L + b, a);
            done = old == b;
            b = old;
        } else if (b < a) {
            const int old = atomicMin(L + a, b);
            done = old == a;
            a = old;
        } else {
            done = true;
        }
    } while (!done);
}

// Tile-local labelling: a workgroup labels the UF_TILE consecutive pixels [t*UF_TILE, ...) of
// slice n in LDS (edges to the left / upper neighbour that lie inside the tile, LDS atomics) and
// writes for every foreground pixel the global index of its tile-local root (-1 elsewhere).
// Only the edges that cross into an earlier tile are then unioned in global memory
// (uf_border_kernel): W per tile instead of two per pixel.
constexpr int UF_TILE = 4096;

__device__ __forceinline__ int lds_find(int* lab, int x) {
    int p = __hip_atomic_load(lab + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (p != x) {
        x = p;
        p = __hip_atomic_load(lab + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    return x;
}

__device__ __forceinline__ void lds_union(int* lab, int a, int b) {
    bool done;
    do {
        a = lds_find(lab, a);
        b = lds_find(lab, b);
        if (a < b) {
            const int old = atomicMin(lab + b, a);
            done = old == b;
            b = old;
        } else if (b < a) {
            const int old = atomicMin(lab + a, b);
            done = old == a;
            a = old;
        } else {
            done = true;
        }
    } while (!done);
}

// Up-edge rule: for 4-connectivity the edge (j, j-W) is implied when the left pair is
// connected on both rows (j-1 ~ j-1-W and j-W ~ j-1-W), so only pixels that start a run in their
// row or sit under the start of a run in the row above need the union.
__device__ __forceinline__ bool need_up(bool left_fg, bool upleft_fg) { return !(left_fg && upleft_fg); }

constexpr int UF_SEG = UF_TILE / MT;  // consecutive pixels per thread (16)

__global__ __launch_bounds__(MT) void uf_local_kernel(const uint8_t* __restrict__ M, int* __restrict__ L, int H, int W,
                                                      int tiles) {
    __shared__ int lab[UF_TILE];
    __shared__ uint8_t fgm[UF_TILE];
    const int HW = H * W;
    const int n = blockIdx.x / tiles, t = blockIdx.x - n * tiles;
    const int p0 = t * UF_TILE;
    const int cnt = min(UF_TILE, HW - p0);
    const int g0 = n * HW + p0;
    for (int j = threadIdx.x; j < UF_TILE; j += MT) fgm[j] = j < cnt ? M[g0 + j] : 0;
    __syncthreads();
    // runs inside this thread's segment point at their first pixel (no atomics)
    const int j0 = threadIdx.x * UF_SEG;
    int x = (p0 + j0) % W;
    int run = -1;
#pragma unroll
    for (int e = 0; e < UF_SEG; ++e) {
        const int j = j0 + e;
        if (e > 0 && ++x == W) x = 0;
        if (!fgm[j]) { lab[j] = -1; run = -1; continue; }
        if (run < 0 || x == 0) run = j;
        lab[j] = run;
    }
    __syncthreads();
    // unions: the segment's first pixel with its left neighbour, and the needed up-edges
    x = (p0 + j0) % W;
#pragma unroll
    for (int e = 0; e < UF_SEG; ++e) {
        const int j = j0 + e;
        if (e > 0 && ++x == W) x = 0;
        if (j >= cnt || !fgm[j]) continue;
        const bool left = x > 0 && j > 0 && fgm[j - 1];
        if (e == 0 && left) lds_union(lab, j, j - 1);
        if (j >= W && fgm[j - W] && need_up(left, x > 0 && fgm[j - 1 - W])) lds_union(lab, j, j - W);
    }
    __syncthreads();
    for (int j = threadIdx.x; j < cnt; j += MT) L[g0 + j] = fgm[j] ? g0 + lds_find(lab, j) : -1;
}

// edges from tile t >= 1 into earlier tiles: its first min(W, UF_TILE) pixels (upper neighbour)
// and its first pixel (left neighbour, when the tile starts mid-row)
__global__ __launch_bounds__(MT) void uf_border_kernel(const uint8_t* __restrict__ M, int* L, int H, int W, int tiles,
                                                       int span, int total) {
    const int i = blockIdx.x * MT + threadIdx.x;
    if (i >= total) return;
    const int per = (tiles - 1) * span;
    const int n = i / per, r = i - n * per;
    const int t = 1 + r / span, k = r - (t - 1) * span;
    const int HW = H * W;
    const int p = t * UF_TILE + k;
    if (p >= HW) return;
    const int g = n * HW + p;
    if (!M[g]) return;
    const int x = p % W;
    const bool left = x > 0 && M[g - 1];
    if (p >= W && M[g - W] && need_up(left, x > 0 && M[g - 1 - W])) uf_union(L, g, g - W);
    if (k == 0 && left) uf_union(L, g, g - 1);
}

// L[i] = root; with count != nullptr also count[root] += 1, aggregated over runs of equal
// roots within the wave (a 100k-pixel component would otherwise serialise 100k atomics).
__global__ __launch_bounds__(MT) void uf_compress_kernel(const uint8_t* __restrict__ M, int* L, int* count, int np) {
    const int i = blockIdx.x * MT + threadIdx.x;
    const bool fg = i < np && M[i];
    int r = -1;
    if (fg) {
        r = uf_find(L, i);
        L[i] = r;
    }
    if (!count) return;
    const int lane = threadIdx.x & 63;
    const int prev = __shfl_up(r, 1, 64);
    const bool head = fg && (lane == 0 || prev != r);
    const unsigned long long heads = __ballot(head);
    const unsigned long long act = __ballot(fg);
    if (head) {
        const unsigned long long above = lane == 63 ? 0ull : (heads >> (lane + 1)) << (lane + 1);
        const int next = above ? __ffsll((long long)above) - 1 : 64;
        const unsigned long long upto = next == 64 ? ~0ull : ((1ull << next) - 1);
        const unsigned long long span = upto & ~((1ull << lane) - 1);
        atomicAdd(count + r, __popcll(act & span));
    }
}

// ---------------------------------------------------------------------------------------
// HU transform (modules/preprocess.py:43-55 + 6-40), float32 op for op like numpy:
//   hu = f32(raw) * slope + intercept ; c = clip(hu, hu_min, hu_max)
//   soft:   n = (c - hu_min) / (hu_max - hu_min); s = 1 / (1 + exp(-k (n - 0.9)))
//           r = n < 0.9 ? n : 0.9 + 0.1 s ; img = 2 r - 1
//   linear: img = 2 (c - hu_min) / (hu_max - hu_min) - 1
// ---------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(MT) void hu_transform_kernel(const T* __restrict__ raw, const float* __restrict__ slope,
                                                          const float* __restrict__ intercept, int HW, float hu_min,
                                                          float hu_max, int soft, float negk,
                                                          float* __restrict__ hu, float* __restrict__ img) {
    const int n = blockIdx.y;
    const int i = blockIdx.x * MT + threadIdx.x;
    if (i >= HW) return;
    const long long o = (long long)n * HW + i;
    const float v = __fadd_rn(__fmul_rn((float)raw[o], slope[n]), intercept[n]);
    if (hu) hu[o] = v;
    if (!img) return;
    const float c = fminf(fmaxf(v, hu_min), hu_max);
    const float range = __fsub_rn(hu_max, hu_min);
    float r;
    if (soft) {
        const float nrm = __fdiv_rn(__fsub_rn(c, hu_min), range);
        const float s = __fdiv_rn(1.0f, __fadd_rn(1.0f, expf(__fmul_rn(negk, __fsub_rn(nrm, 0.9f)))));
        const float sq = __fadd_rn(0.9f, __fmul_rn(0.1f, s));
        r = __fsub_rn(__fmul_rn(2.0f, nrm < 0.9f ? nrm : sq), 1.0f);
    } else {
        r = __fsub_rn(__fdiv_rn(__fmul_rn(2.0f, __fsub_rn(c, hu_min)), range), 1.0f);
    }
    img[o] = r;
}

// ---------------------------------------------------------------------------------------
// masks
// ---------------------------------------------------------------------------------------
struct MaskArgs {
    int N, H, W;
    float lung_lower, lung_upper, vessel_lower, vessel_upper, medi_lower, medi_upper, bone_thr;
    int min_size, border, spine_start;
};

// detect_lung thresholds (mask_generator.py:14-29) and the bone candidates (:179-183);
// per-slice body pixel count (body = hu > -1000).
__global__ __launch_bounds__(MT) void mask_seed_kernel(const float* __restrict__ hu, const uint8_t* __restrict__ lung_in,
                                                       MaskArgs a, uint8_t* __restrict__ F, uint8_t* __restrict__ M,
                                                       SliceInfo* si) {
    const int n = blockIdx.y, HW = a.H * a.W;
    int body = 0;
    for (int p = blockIdx.x * MT + threadIdx.x; p < HW; p += gridDim.x * MT) {
        const int i = n * HW + p;
        const int y = p / a.W, x = p - y * a.W;
        const float v = hu[i];
        const bool bd = v > -1000.f;
        body += bd;
        const bool inner = y >= a.border && y < a.H - a.border && x >= a.border && x < a.W - a.border;
        // a caller-supplied lung mask (detect_mediastinum(hu, lung_mask) etc.) replaces detect_lung
        const bool lc = lung_in ? lung_in[i] != 0 : bd && v >= a.lung_lower && v <= a.lung_upper && inner;
        const bool ab = bd && v >= a.bone_thr;
        F[i] = (lc ? F_LUNGC : 0) | (ab ? F_ABONE : 0);
        M[i] = lc;
    }
    __shared__ float red[4];
    const float s = block_sum_256((float)body, red);
    if (threadIdx.x == 0 && s > 0.f) atomicAdd(&si[n].body, (int)s);
}

// lung = candidate components of >= min_size pixels; per-slice area, region count and the
// per-row extreme columns (hull candidates).
__global__ __launch_bounds__(MT) void lung_final_kernel(MaskArgs a, const int* __restrict__ L, const int* __restrict__ C,
                                                        uint8_t* __restrict__ F, SliceInfo* si, int* __restrict__ rowmin,
                                                        int* __restrict__ rowmax) {
    const int n = blockIdx.y, HW = a.H * a.W;
    int lung_cnt = 0, root_cnt = 0;
    // grid-stride with a block-uniform trip count (the wave shuffles below need every lane)
    for (int p0 = blockIdx.x * MT; p0 < HW; p0 += gridDim.x * MT) {
        const int p = p0 + threadIdx.x;
        int lung = 0, y = 0, x = 0;
        if (p < HW) {
            const int i = n * HW + p;
            const uint8_t f = F[i];
            y = p / a.W;
            x = p - y * a.W;
            if (f & F_LUNGC) {
                const int r = L[i];
                if (C[r] >= a.min_size) {
                    lung = 1;
                    root_cnt += r == i;
                    F[i] = f | F_LUNG;
                }
            }
        }
        lung_cnt += lung;
        if ((a.W & 63) == 0) {  // the wave's 64 pixels share one row: one atomic pair per wave
            int mn = lung ? x : 0x7fffffff, mx = lung ? x : -1;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                mn = min(mn, __shfl_xor(mn, o, 64));
                mx = max(mx, __shfl_xor(mx, o, 64));
            }
            if ((threadIdx.x & 63) == 0 && mx >= 0) {
                atomicMin(rowmin + n * a.H + y, mn);
                atomicMax(rowmax + n * a.H + y, mx);
            }
        } else if (lung) {
            atomicMin(rowmin + n * a.H + y, x);
            atomicMax(rowmax + n * a.H + y, x);
        }
    }
    const int lung = lung_cnt, root = root_cnt;
    __shared__ float red[4];
    const float s = block_sum_256((float)lung, red);
    const float nr = block_sum_256((float)root, red);
    if (threadIdx.x == 0) {
        if (s > 0.f) atomicAdd(&si[n].lung_area, (int)s);
        if (nr > 0.f) atomicAdd(&si[n].nreg, (int)nr);
    }
}

// |coordinates| < 1024 (H, W <= 1024): every product below fits in 32 bits
__device__ __forceinline__ int cross2(int2 o, int2 a, int2 b) {
    return (a.x - o.x) * (b.y - o.y) - (a.y - o.y) * (b.x - o.x);
}

// One workgroup per slice: the gate of mask_generator.py:68/116/196 (>= 2 lung regions and
// lung/body area >= 0.1, in float64 like numpy) and the convex hull of the lung pixels,
// vertices as (row, col) counter-clockwise, no collinear points (qhull's output).
// hull_ok = 0 when there are < 3 lung pixels or they are collinear (qhull raises; the
// reference falls back to the lung mask itself / skips the exclusion).
// Andrew's monotone chain over pts[0..np) in the given direction (+1 / -1) into out; returns the
// chain length.  The top two stack entries live in registers (one LDS read per pop).
__device__ int hull_chain(const int2* pts, int np, int dir, int2* out) {
    int k = 0;
    int2 t1 = make_int2(0, 0), t2 = make_int2(0, 0);  // out[k-1], out[k-2]
    int2 nxt = np > 0 ? pts[dir > 0 ? 0 : np - 1] : make_int2(0, 0);
    for (int j = 0; j < np; ++j) {
        const int2 p = nxt;
        if (j + 1 < np) nxt = pts[dir > 0 ? j + 1 : np - 2 - j];
        while (k >= 2 && cross2(t2, t1, p) <= 0) {
            --k;
            t1 = t2;
            if (k >= 2) t2 = out[k - 2];
        }
        out[k++] = p;
        t2 = t1;
        t1 = p;
    }
    return k;
}

// One workgroup per slice: the gate of mask_generator.py:68/116/196 (>= 2 lung regions and
// lung/body area >= 0.1, in float64 like numpy) and the convex hull of the lung pixels,
// vertices as (row, col) counter-clockwise, no collinear points (qhull's output).
// hull_ok = 0 when there are < 3 lung pixels or they are collinear (qhull raises; the
// reference falls back to the lung mask itself / skips the exclusion).
__global__ __launch_bounds__(MT) void lung_hull_kernel(MaskArgs a, SliceInfo* si, const int* __restrict__ rowmin,
                                                       const int* __restrict__ rowmax, int2* __restrict__ hull,
                                                       int maxv) {
    extern __shared__ int2 sh[];  // pts[maxv], lower[maxv], upper[maxv], rows (lo, hi)[H]
    int2* pts = sh;
    int2* lo = sh + maxv;
    int2* up = sh + 2 * maxv;
    int2* rows = sh + 3 * maxv;
    __shared__ int npts, nlo, nup;
    const int n = blockIdx.x;
    SliceInfo& s = si[n];
    const int cond = s.nreg >= 2 && s.body > 0 && (double)s.lung_area / (double)s.body >= 0.1;
    if (!cond || s.lung_area < 3) {
        if (threadIdx.x == 0) { s.cond = cond; s.hull_ok = 0; s.nv = 0; }
        return;
    }
    // points sorted by (row, col): per row its leftmost then rightmost lung pixel.  Thread t owns
    // rows 4t .. 4t+3 (H <= 1024); an exclusive scan of the per-thread counts places them.
    __shared__ int wsum[MT / 64];
    int cntp[4], tot = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int y = 4 * threadIdx.x + e;
        int c = 0;
        if (y < a.H) {
            const int2 r = make_int2(rowmin[n * a.H + y], rowmax[n * a.H + y]);
            rows[y] = r;
            c = r.y < 0 ? 0 : (r.y != r.x ? 2 : 1);
        }
        cntp[e] = c;
        tot += c;
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int inc = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(inc, o, 64);
        if (lane >= o) inc += v;
    }
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    int base = inc - tot;
    for (int w2 = 0; w2 < wv; ++w2) base += wsum[w2];
    if (threadIdx.x == MT - 1) npts = base + tot;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int y = 4 * threadIdx.x + e;
        if (cntp[e] == 0) continue;
        const int2 r = rows[y];
        pts[base++] = make_int2(y, r.x);
        if (cntp[e] == 2) pts[base++] = make_int2(y, r.y);
    }
    __syncthreads();
    if (threadIdx.x == 0) nlo = hull_chain(pts, npts, +1, lo);
    if (threadIdx.x == 64) nup = hull_chain(pts, npts, -1, up);  // another wave: runs concurrently
    __syncthreads();
    // hull = lower[0 .. nlo-2] ++ upper[0 .. nup-2] (each chain ends where the other starts)
    const int kl = nlo - 1, k = kl + nup - 1;
    const int ok = k >= 3;
    for (int j = threadIdx.x; ok && j < k; j += MT) hull[(long long)n * maxv + j] = j < kl ? lo[j] : up[j - kl];
    if (threadIdx.x == 0) {
        s.cond = cond;
        s.hull_ok = ok;
        s.nv = ok ? k : 0;
    }
}

// matplotlib point_in_path (crossing number) for point (tx, ty) = (row, col) against the
// closed polygon hv[0..nv-1]: the division-free edge test of _path.h, exact on integers.
__device__ __forceinline__ bool point_in_hull(const int2* hv, int nv, int tx, int ty) {
    bool inside = false;
    int2 v0 = hv[nv - 1];
    bool f0 = v0.y >= ty;
    for (int j = 0; j < nv; ++j) {
        const int2 v1 = hv[j];
        const bool f1 = v1.y >= ty;
        if (f0 != f1) {
            const int lhs = (v1.y - ty) * (v0.x - v1.x);
            const int rhs = (v1.x - tx) * (v0.y - v1.y);
            if ((lhs >= rhs) == f1) inside = !inside;
        }
        v0 = v1;
        f0 = f1;
    }
    return inside;
}

// Lung-hull pass: mediastinum (detect_mediastinum, mask_generator.py:116-136; the candidate
// is `convex_hull - lung` in uint8, i.e. nonzero where the two differ) and the bone seeds
// (detect_bone :196-220: candidates minus hull & ~lung & ~spine rows).  Also stages the
// membership of the bone-candidate union-find.
__global__ __launch_bounds__(MT) void hull_pass_kernel(const float* __restrict__ hu, MaskArgs a, const SliceInfo* si,
                                                       const int2* __restrict__ hull, int maxv,
                                                       uint8_t* __restrict__ F, uint8_t* __restrict__ M) {
    extern __shared__ int2 hv[];
    const int n = blockIdx.y, HW = a.H * a.W;
    const int cond = si[n].cond, ok = si[n].hull_ok, nv = si[n].nv;
    if (ok)
        for (int j = threadIdx.x; j < nv; j += MT) hv[j] = hull[(long long)n * maxv + j];
    __syncthreads();
    const int p = blockIdx.x * MT + threadIdx.x;
    if (p >= HW) return;
    const int i = n * HW + p;
    const int y = p / a.W, x = p - y * a.W;
    uint8_t f = F[i];
    const bool lung = f & F_LUNG;
    bool excluded = false;
    if (cond) {
        const bool inside = ok ? point_in_hull(hv, nv, y, x) : lung;
        const float v = hu[i];
        if (inside) f |= F_INSIDE;
        if (inside != lung && v >= a.medi_lower && v <= a.medi_upper) f |= F_MEDI;
        excluded = ok && inside && !lung && y < a.spine_start;
    }
    if ((f & F_ABONE) && !excluded) f |= F_SEED;
    F[i] = f;
    M[i] = (f & F_ABONE) != 0;
}

// union-find membership = complement of a flag bit (the background of a mask)
__global__ __launch_bounds__(MT) void stage_complement_kernel(const uint8_t* __restrict__ F, int bit,
                                                              uint8_t* __restrict__ M, int np) {
    const int i = blockIdx.x * MT + threadIdx.x;
    if (i < np) M[i] = (F[i] & bit) == 0;
}

// C[root] = 1 for background components that touch an image edge (binary_fill_holes: the
// outside propagates into the background through 4-connected paths)
__global__ __launch_bounds__(MT) void mark_edge_kernel(const uint8_t* __restrict__ M, const int* __restrict__ L,
                                                       int H, int W, int* __restrict__ C, int np) {
    const int i = blockIdx.x * MT + threadIdx.x;
    if (i >= np || !M[i]) return;
    const int x = i % W, y = (i / W) % H;
    if (x == 0 || y == 0 || x == W - 1 || y == H - 1) C[L[i]] = 1;
}

// C[root] = 1 for bone-candidate components holding a seed (region growing, :224-239)
__global__ __launch_bounds__(MT) void mark_seed_kernel(const uint8_t* __restrict__ F, const int* __restrict__ L,
                                                       int* __restrict__ C, int np) {
    const int i = blockIdx.x * MT + threadIdx.x;
    if (i < np && (F[i] & F_SEED)) C[L[i]] = 1;
}

// vessels = holes of the lung mask (filled - lung) in the vessel HU window (detect_lung_vessels)
__global__ __launch_bounds__(MT) void vessel_kernel(const float* __restrict__ hu, MaskArgs a, const SliceInfo* si,
                                                    const uint8_t* __restrict__ M, const int* __restrict__ L,
                                                    const int* __restrict__ C, uint8_t* __restrict__ F) {
    const int n = blockIdx.y, HW = a.H * a.W;
    const int p = blockIdx.x * MT + threadIdx.x;
    if (p >= HW || !si[n].cond) return;
    const int i = n * HW + p;
    if (M[i] && !C[L[i]]) {
        const float v = hu[i];
        if (v >= a.vessel_lower && v <= a.vessel_upper) F[i] |= F_VES;
    }
}

__global__ __launch_bounds__(MT) void bone_grow_kernel(const int* __restrict__ L, const int* __restrict__ C,
                                                       uint8_t* __restrict__ F, int np) {
    const int i = blockIdx.x * MT + threadIdx.x;
    if (i >= np) return;
    const uint8_t f = F[i];
    if ((f & F_ABONE) && C[L[i]]) F[i] = f | F_BONE;
}

// float32 masks in the caller's channel order (fuses the reference's torch.cat); bone is
// filled here (bone | holes of bone, from the background union-find of ~bone in M/L/C)
__global__ __launch_bounds__(MT) void mask_out_kernel(MaskArgs a, const uint8_t* __restrict__ F,
                                                      const uint8_t* __restrict__ M, const int* __restrict__ L,
                                                      const int* __restrict__ C, int4 chan, int nout,
                                                      float* __restrict__ out) {
    const int n = blockIdx.y, HW = a.H * a.W;
    const int p = blockIdx.x * MT + threadIdx.x;
    if (p >= HW) return;
    const int i = n * HW + p;
    const uint8_t f = F[i];
    float* o = out + (long long)n * nout * HW + p;
    if (chan.x >= 0) o[(long long)chan.x * HW] = (f & F_LUNG) ? 1.f : 0.f;
    if (chan.y >= 0) o[(long long)chan.y * HW] = (f & F_MEDI) ? 1.f : 0.f;
    if (chan.z >= 0) {
        const bool b = (f & F_BONE) || (M[i] && !C[L[i]]);
        o[(long long)chan.z * HW] = b ? 1.f : 0.f;
    }
    if (chan.w >= 0) o[(long long)chan.w * HW] = (f & F_VES) ? 1.f : 0.f;
}

__global__ __launch_bounds__(MT) void fill_int_kernel(int* __restrict__ p, int v, int n) {
    const int i = blockIdx.x * MT + threadIdx.x;
    if (i < n) p[i] = v;
}

struct MaskWs {
    int* L;
    int* C;
    uint8_t* M;
    uint8_t* F;
    SliceInfo* si;
    int* rowmin;
    int* rowmax;
    int2* hull;
    size_t bytes;
};

static MaskWs carve(void* base, int N, int H, int W) {
    MaskWs w;
    const size_t np = (size_t)N * H * W;
    char* p = reinterpret_cast<char*>(base);
    size_t off = 0;
    auto take = [&](size_t b) {
        char* q = p ? p + off : nullptr;
        off = align_up(off + b, 256);
        return q;
    };
    w.L = reinterpret_cast<int*>(take(np * 4));
    w.C = reinterpret_cast<int*>(take(np * 4));
    w.M = reinterpret_cast<uint8_t*>(take(np));
    w.F = reinterpret_cast<uint8_t*>(take(np));
    w.si = reinterpret_cast<SliceInfo*>(take((size_t)N * sizeof(SliceInfo)));
    w.rowmin = reinterpret_cast<int*>(take((size_t)N * H * 4));
    w.rowmax = reinterpret_cast<int*>(take((size_t)N * H * 4));
    w.hull = reinterpret_cast<int2*>(take((size_t)N * (2 * H + 2) * sizeof(int2)));
    w.bytes = off;
    return w;
}

static int run_cc(MaskWs& w, int N, int H, int W, bool count, hipStream_t s) {
    const int HW = H * W, np = N * HW;
    const int tiles = (int)cdiv(HW, UF_TILE);
    const dim3 g((unsigned)cdiv(np, MT));
    hipLaunchKernelGGL(uf_local_kernel, dim3((unsigned)(N * tiles)), dim3(MT), 0, s, w.M, w.L, H, W, tiles);
    if (tiles > 1) {
        const int span = W < UF_TILE ? W : UF_TILE;
        const int total = N * (tiles - 1) * span;
        hipLaunchKernelGGL(uf_border_kernel, dim3((unsigned)cdiv(total, MT)), dim3(MT), 0, s, w.M, w.L, H, W, tiles,
                           span, total);
    }
    hipLaunchKernelGGL(fill_int_kernel, g, dim3(MT), 0, s, w.C, 0, np);
    hipLaunchKernelGGL(uf_compress_kernel, g, dim3(MT), 0, s, w.M, w.L, count ? w.C : (int*)nullptr, np);
    return check_launch("masks: connected components");
}

}  // namespace dcs

using namespace dcs;

extern "C" int dcs_hu_transform(const void* raw, int raw_dtype, const float* slope, const float* intercept, int N,
                                int H, int W, float hu_min, float hu_max, int soft, float sigma, float* hu,
                                float* img, void* stream) {
    if (!raw || !slope || !intercept || N <= 0 || H <= 0 || W <= 0 || (!hu && !img) || raw_dtype < 0 ||
        raw_dtype > 2 || (soft && !(sigma > 0.f)) || !(hu_max > hu_min))
        return fail(DCS_E_INVALID, "hu_transform: bad arguments");
    if ((long long)H * W >= (1ll << 31)) return fail(DCS_E_INVALID, "hu_transform: slice too large");
    const int HW = H * W;
    const dim3 grid((unsigned)cdiv(HW, MT), (unsigned)N);
    // k = 10.0 / sigma in float64 (python), then used as a float32 scalar on float32 arrays
    const float negk = (float)(-(10.0 / (double)sigma));
    hipStream_t s = as_stream(stream);
    if (raw_dtype == 0)
        hipLaunchKernelGGL(hu_transform_kernel<int16_t>, grid, dim3(MT), 0, s, (const int16_t*)raw, slope, intercept,
                           HW, hu_min, hu_max, soft, negk, hu, img);
    else if (raw_dtype == 1)
        hipLaunchKernelGGL(hu_transform_kernel<uint16_t>, grid, dim3(MT), 0, s, (const uint16_t*)raw, slope,
                           intercept, HW, hu_min, hu_max, soft, negk, hu, img);
    else
        hipLaunchKernelGGL(hu_transform_kernel<float>, grid, dim3(MT), 0, s, (const float*)raw, slope, intercept, HW,
                           hu_min, hu_max, soft, negk, hu, img);
    return check_launch("hu_transform");
}

extern "C" size_t dcs_masks_workspace_size(int N, int H, int W) {
    if (N <= 0 || H <= 0 || W <= 0) return 0;
    return carve(nullptr, N, H, W).bytes;
}

extern "C" int dcs_anatomical_masks(const float* hu, const uint8_t* lung_in, int N, int H, int W, const float* thresholds,
                                    const int32_t* iparams, const int32_t* chan, int nout, float* out, void* ws,
                                    size_t ws_bytes, void* stream) {
    if (!hu || !thresholds || !iparams || !chan || !out || !ws || N <= 0 || H < 1 || W < 1 || nout < 1 || nout > 4)
        return fail(DCS_E_INVALID, "anatomical_masks: bad arguments");
    if ((long long)N * H * W >= (1ll << 31) || H > 1024 || W > 1024)
        return fail(DCS_E_INVALID, "anatomical_masks: batch too large (N*H*W < 2^31, H, W <= 1024)");
    for (int c = 0; c < 4; ++c)
        if (chan[c] < -1 || chan[c] >= nout) return fail(DCS_E_INVALID, "anatomical_masks: bad channel map");
    if (ws_bytes < dcs_masks_workspace_size(N, H, W))
        return fail(DCS_E_WORKSPACE, "anatomical_masks: workspace too small");
    MaskWs w = carve(ws, N, H, W);
    MaskArgs a;
    a.N = N; a.H = H; a.W = W;
    a.lung_lower = thresholds[0]; a.lung_upper = thresholds[1];
    a.vessel_lower = thresholds[2]; a.vessel_upper = thresholds[3];
    a.medi_lower = thresholds[4]; a.medi_upper = thresholds[5];
    a.bone_thr = thresholds[6];
    a.min_size = lung_in ? 0 : iparams[0]; a.border = iparams[1]; a.spine_start = iparams[2];
    const int4 ch = make_int4(chan[0], chan[1], chan[2], chan[3]);
    const bool want_medi = ch.y >= 0, want_bone = ch.z >= 0, want_ves = ch.w >= 0;

    hipStream_t s = as_stream(stream);
    const int np = N * H * W, HW = H * W;
    const dim3 gs((unsigned)cdiv(HW, MT), (unsigned)N), gl((unsigned)cdiv(np, MT));
    const int maxv = 2 * H + 2;
    int e;

    if (hipMemsetAsync(w.si, 0, (size_t)N * sizeof(SliceInfo), s) != hipSuccess)
        return fail(DCS_E_INVALID, "anatomical_masks: memset failed");
    hipLaunchKernelGGL(fill_int_kernel, dim3((unsigned)cdiv(N * H, MT)), dim3(MT), 0, s, w.rowmin, W, N * H);
    hipLaunchKernelGGL(fill_int_kernel, dim3((unsigned)cdiv(N * H, MT)), dim3(MT), 0, s, w.rowmax, -1, N * H);
    // the per-slice counters take one atomic per block: at most 64 blocks per slice
    const dim3 gc((unsigned)(cdiv(HW, MT) < 64 ? cdiv(HW, MT) : 64), (unsigned)N);
    hipLaunchKernelGGL(mask_seed_kernel, gc, dim3(MT), 0, s, hu, lung_in, a, w.F, w.M, w.si);
    if ((e = check_launch("masks: seed"))) return e;
    // detect_lung: components of the lung candidates, size filter, gate and hull
    if ((e = run_cc(w, N, H, W, true, s))) return e;
    hipLaunchKernelGGL(lung_final_kernel, gc, dim3(MT), 0, s, a, w.L, w.C, w.F, w.si, w.rowmin, w.rowmax);
    if ((e = check_launch("masks: lung"))) return e;
    hipLaunchKernelGGL(lung_hull_kernel, dim3((unsigned)N), dim3(MT), (size_t)(3 * maxv + H) * sizeof(int2), s, a,
                       w.si, w.rowmin, w.rowmax, w.hull, maxv);
    if ((e = check_launch("masks: hull"))) return e;
    if (want_ves) {  // holes of the lung mask
        hipLaunchKernelGGL(stage_complement_kernel, gl, dim3(MT), 0, s, w.F, (int)F_LUNG, w.M, np);
        if ((e = run_cc(w, N, H, W, false, s))) return e;
        hipLaunchKernelGGL(mark_edge_kernel, gl, dim3(MT), 0, s, w.M, w.L, H, W, w.C, np);
        hipLaunchKernelGGL(vessel_kernel, gs, dim3(MT), 0, s, hu, a, w.si, w.M, w.L, w.C, w.F);
        if ((e = check_launch("masks: vessels"))) return e;
    }
    if (want_medi || want_bone) {
        hipLaunchKernelGGL(hull_pass_kernel, gs, dim3(MT), (size_t)maxv * sizeof(int2), s, hu, a, w.si, w.hull, maxv,
                           w.F, w.M);
        if ((e = check_launch("masks: hull pass"))) return e;
    }
    if (want_bone) {  // region growing over the bone candidates, then the holes of the result
        if ((e = run_cc(w, N, H, W, false, s))) return e;
        hipLaunchKernelGGL(mark_seed_kernel, gl, dim3(MT), 0, s, w.F, w.L, w.C, np);
        hipLaunchKernelGGL(bone_grow_kernel, gl, dim3(MT), 0, s, w.L, w.C, w.F, np);
        hipLaunchKernelGGL(stage_complement_kernel, gl, dim3(MT), 0, s, w.F, (int)F_BONE, w.M, np);
        if ((e = run_cc(w, N, H, W, false, s))) return e;
        hipLaunchKernelGGL(mark_edge_kernel, gl, dim3(MT), 0, s, w.M, w.L, H, W, w.C, np);
        if ((e = check_launch("masks: bone"))) return e;
    }
    hipLaunchKernelGGL(mask_out_kernel, gs, dim3(MT), 0, s, a, w.F, w.M, w.L, w.C, ch, nout, out);
    return check_launch("masks: output");
}
