// Probe: FLOP/s of the f16x3 inner loop (three products per fragment pair, fragments re-read from LDS,
// two waves per SIMD, every CU busy, random operands) on v_mfma_f32_32x32x16_f16 against
// v_mfma_f32_16x16x32_f16 at equal work per wave tile (64 x 64) and equal LDS bytes per MAC.
// MI355X_MICROARCH.md (DVFS item 7) reports the 16x16x32 bf16 loop ~1.12-1.15x faster under the
// power limit at equal cycles per FLOP; this checks it for the f16 forms this library uses.
//   hipcc -O3 --offload-arch=gfx950 mfma_shape_power.hip -o /tmp/mfma_shape_power && ./mfma_shape_power
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int NT = 512, LDSH = 32768;  // 64 KB of halves

template <int SHAPE>  // 0: 32x32x16, 1: 16x16x32
__global__ __launch_bounds__(NT, 1) void probe(const _Float16* __restrict__ src, float* __restrict__ out, int iters) {
    __shared__ __attribute__((aligned(16))) _Float16 lds[LDSH];
    for (int i = threadIdx.x * 8; i < LDSH; i += NT * 8)
        *reinterpret_cast<f16x8*>(lds + i) = *reinterpret_cast<const f16x8*>(src + ((blockIdx.x * 977 + i) & (1 << 20) - 1));
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int base = (wid * 1024 + lane * 8) & (LDSH / 2 - 1);
    if constexpr (SHAPE == 0) {
        floatx16 acc[2][2] = {};
        for (int it = 0; it < iters; ++it) {
            const int o = (base + it * 512) & (LDSH / 2 - 1);
            f16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                ah[i] = *reinterpret_cast<const f16x8*>(lds + ((o + i * 2048) & (LDSH / 2 - 1)));
                al[i] = *reinterpret_cast<const f16x8*>(lds + ((o + i * 2048 + 4096) & (LDSH / 2 - 1)));
                bh[i] = *reinterpret_cast<const f16x8*>(lds + LDSH / 2 + ((o + i * 2048) & (LDSH / 2 - 1)));
                bl[i] = *reinterpret_cast<const f16x8*>(lds + LDSH / 2 + ((o + i * 2048 + 4096) & (LDSH / 2 - 1)));
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                }
        }
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) s += acc[i][j][r];
        out[blockIdx.x * NT + threadIdx.x] = s;
    } else {
        floatx4 acc[4][4] = {};
        for (int it = 0; it < iters; it += 2) {  // one K=32 step = two K=16 steps of shape 0
            const int o = (base + it * 512) & (LDSH / 2 - 1);
            f16x8 ah[4], al[4], bh[4], bl[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                ah[i] = *reinterpret_cast<const f16x8*>(lds + ((o + i * 1024) & (LDSH / 2 - 1)));
                al[i] = *reinterpret_cast<const f16x8*>(lds + ((o + i * 1024 + 4096) & (LDSH / 2 - 1)));
                bh[i] = *reinterpret_cast<const f16x8*>(lds + LDSH / 2 + ((o + i * 1024) & (LDSH / 2 - 1)));
                bl[i] = *reinterpret_cast<const f16x8*>(lds + LDSH / 2 + ((o + i * 1024 + 4096) & (LDSH / 2 - 1)));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                }
        }
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) s += acc[i][j][r];
        out[blockIdx.x * NT + threadIdx.x] = s;
    }
}

int main() {
    const int blocks = 256 * 4, iters = 4096;
    const size_t nsrc = 1 << 20;
    std::vector<_Float16> h(nsrc);
    srand(1);
    for (auto& v : h) v = (_Float16)((rand() / (float)RAND_MAX) * 2.f - 1.f);
    _Float16* src;
    float* out;
    hipMalloc(&src, nsrc * 2);
    hipMalloc(&out, (size_t)blocks * NT * 4);
    hipMemcpy(src, h.data(), nsrc * 2, hipMemcpyHostToDevice);
    // FLOP per launch: per wave per K=16 step: 2x2 blocks x 3 products x 2*32*32*16
    const double flop = (double)blocks * 8 * iters * 12 * 2.0 * 32 * 32 * 16;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 4; ++rep) {
        for (int shape = 0; shape < 2; ++shape) {
            // ~2 s of back-to-back launches: the clock settles under the power limit
            int n = 0;
            float ms = 0.f;
            hipEventRecord(e0);
            while (true) {
                for (int k = 0; k < 10; ++k) {
                    if (shape == 0) hipLaunchKernelGGL(probe<0>, dim3(blocks), dim3(NT), 0, 0, src, out, iters);
                    else hipLaunchKernelGGL(probe<1>, dim3(blocks), dim3(NT), 0, 0, src, out, iters);
                }
                n += 10;
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                hipEventElapsedTime(&ms, e0, e1);
                if (ms > 2000.f) break;
            }
            printf("rep %d shape %s: %.3f ms/launch, %.1f TFLOP/s (f16x3 products)\n", rep,
                   shape == 0 ? "32x32x16" : "16x16x32", ms / n, flop / (ms / n * 1e-3) / 1e12);
            fflush(stdout);
        }
    }
    hipFree(src);
    hipFree(out);
    return 0;
}
