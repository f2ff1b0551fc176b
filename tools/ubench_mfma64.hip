// Microbenchmark: v_mfma_f64_16x16x4_f64 throughput on every CU -- ACC independent
// accumulators per wave, W waves per workgroup (W / 4 per SIMD), one workgroup per CU,
// ITER rounds; prints TFLOP/s and the fraction of 78.6 TFLOP/s.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_mfma64.hip -o tools/ubench_mfma64
#include <hip/hip_runtime.h>
#include <cstdio>

using D4 = __attribute__((ext_vector_type(4))) double;

template <int ACC>
__global__ void mfma64_kernel(double* out, int iters, double seed) {
    D4 acc[ACC];
    for (int i = 0; i < ACC; ++i) acc[i] = D4{0.0, 0.0, 0.0, 0.0};
    double a = seed + threadIdx.x * 1e-9, b = seed * 0.5;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < ACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    double s = 0;
    for (int i = 0; i < ACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    if (s == 12345.0) out[threadIdx.x] = s;
}

template <int ACC>
void run(int waves, int cus, int iters) {
    double* out;
    (void)hipMalloc(&out, 4096 * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    mfma64_kernel<ACC><<<cus, 64 * waves>>>(out, 10, 1.0);
    (void)hipEventRecord(e0, 0);
    mfma64_kernel<ACC><<<cus, 64 * waves>>>(out, iters, 1.0);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double flops = 2.0 * 16 * 16 * 4 * 64.0 / 64 * ACC * (double)iters * waves * cus;  // per wave: ACC MFMAs x 2048 FLOP
    const double tf = flops / (ms * 1e-3) / 1e12;
    printf("ACC %2d waves/WG %2d (%d per SIMD): %8.3f ms  %6.2f TFLOP/s  %.3f of 78.6\n", ACC, waves, waves / 4, ms, tf,
           tf / 78.6);
    (void)hipFree(out);
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int iters = 20000;
    run<4>(4, cus, iters);
    run<8>(4, cus, iters);
    run<16>(4, cus, iters);
    run<4>(8, cus, iters);
    run<8>(8, cus, iters);
    run<16>(8, cus, iters);
    run<8>(16, cus, iters);
    return 0;
}
