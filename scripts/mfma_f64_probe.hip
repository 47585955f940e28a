// Diagnostics (GPU box): sustained v_mfma_f64_16x16x4f64 rate, every CU busy, k independent
// accumulators per wave, w waves per SIMD; prints TFLOP/s and cycles per MFMA per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef double acc_t __attribute__((ext_vector_type(4)));
template <int K>
__global__ void __launch_bounds__(256) k_mfma(int iters, double *out) {
    acc_t acc[K];
    for (int k = 0; k < K; ++k) acc[k] = acc_t{0.0, 0.0, 0.0, 0.0};
    double a = 1.0 + 1e-9 * threadIdx.x, b = 1.0 - 1e-9 * threadIdx.x;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < K; ++k) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
    }
    double s = 0;
    for (int k = 0; k < K; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
template <int K>
static void run(int blocks_per_cu, int iters) {
    const int blocks = 256 * blocks_per_cu;
    double *out;
    (void)hipMalloc(&out, sizeof(double) * blocks * 256);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k_mfma<K>, dim3(blocks), dim3(256), 0, 0, iters, out);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_mfma<K>, dim3(blocks), dim3(256), 0, 0, iters, out);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double mf = (double)blocks * 4 * iters * K;   // MFMAs (4 waves per block)
    const double tf = mf * 2048 / (ms * 1e-3) / 1e12;
    printf("K=%d waves/SIMD=%d: %.3f ms, %.1f TFLOP/s, %.1f cyc/MFMA/SIMD at 2.4 GHz\n", K, blocks_per_cu, ms, tf,
           (ms * 1e-3 * 2.4e9) / (mf / 1024.0));
    (void)hipFree(out);
}
int main() {
    run<1>(1, 20000);
    run<4>(1, 5000);
    run<4>(2, 5000);
    run<8>(2, 2500);
    run<4>(4, 2500);
    return 0;
}
