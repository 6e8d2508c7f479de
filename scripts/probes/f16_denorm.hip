// Probe: does v_mfma_f32_32x32x16_f16 honour fp16 denormal operands on gfx950, and does the
// f32 -> f16 conversion keep denormals?  Prints the MFMA output for a denormal A operand.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
__global__ void k(const float* in, float* out) {
    const int lane = threadIdx.x;
    f16x8 a, b;
    for (int i = 0; i < 8; ++i) { a[i] = (_Float16)0.f; b[i] = (_Float16)1.f; }
    // lane l < 32 supplies A[row l][k 0..7]; put the probe value at k 0 of every row
    if (lane < 32) a[0] = (_Float16)in[0];
    floatx16 acc = {};
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
    if (lane == 0) { out[0] = acc[0]; out[1] = (float)a[0]; }
}
int main() {
    float h_in[4] = {0x1p-20f, 0x1p-24f, 0x1p-14f, 3.0e-6f}, h_out[2];
    float *din, *dout;
    hipMalloc(&din, 16); hipMalloc(&dout, 8);
    for (int t = 0; t < 4; ++t) {
        hipMemcpy(din, &h_in[t], 4, hipMemcpyHostToDevice);
        k<<<1, 64>>>(din, dout);
        hipMemcpy(h_out, dout, 8, hipMemcpyDeviceToHost);
        printf("in %g: f16 cvt %g, mfma out %g\n", h_in[t], h_out[1], h_out[0]);
    }
    return 0;
}
