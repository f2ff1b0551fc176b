// ubench_pass.hip — microbenchmarks that price the pieces of the fused Sinkhorn pass
// on gfx950 (N x N float32 cost, one 512-thread workgroup per CU, 16 rows each):
//   stream      : read the 64 MiB cost once (same layout as the pass), trivial reduce
//   flush R     : 256 workgroups each add 4096 floats (coalesced) into replica wg % R
//   stream+flush: both in one kernel (the pass's memory behaviour without its math)
// Build: hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics tools/ubench_pass.hip -o ubench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

using f4 = __attribute__((ext_vector_type(4))) float;
constexpr int NT = 512;

template <int ROWS, bool STREAM, bool FLUSH>
__global__ __launch_bounds__(512) void pass_like(const float* C, int n, int m, float* cs, int reps,
                                                 float* sink) {
    __shared__ float colbuf[4096];
    const int tid = threadIdx.x;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int nrb = n / ROWS;
    for (int rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
        if (STREAM) {
            f4 v[ROWS][2];
#pragma unroll
            for (int r = 0; r < ROWS; ++r)
#pragma unroll
                for (int g = 0; g < 2; ++g)
                    v[r][g] = *reinterpret_cast<const f4*>(C + (size_t)(rb * ROWS + r) * m + (tid + NT * g) * 4);
#pragma unroll
            for (int r = 0; r < ROWS; ++r)
#pragma unroll
                for (int g = 0; g < 2; ++g)
#pragma unroll
                    for (int k = 0; k < 4; ++k) acc[g * 4 + k] += v[r][g][k];
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] += 1.0f;
        }
    }
    if (FLUSH) {
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            f4 w = {acc[g * 4], acc[g * 4 + 1], acc[g * 4 + 2], acc[g * 4 + 3]};
            *reinterpret_cast<f4*>(colbuf + (tid + NT * g) * 4) = w;
        }
        __syncthreads();
        float* dst = cs + (size_t)(blockIdx.x % reps) * m;
        for (int j = tid; j < m; j += NT) atomicAdd(dst + j, colbuf[j]);
    } else {
        float s = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) s += acc[k];
        if (s == 12345.f) sink[blockIdx.x] = s;
    }
}

template <typename K>
float timeit(K launch, int iters) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    launch();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < iters; ++i) launch();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1000.f / iters;
}

int main() {
    const int n = 4096, m = 4096;
    float *C, *cs, *sink, *big;
    CK(hipMalloc(&C, (size_t)n * m * 4));
    CK(hipMalloc(&cs, (size_t)64 * m * 4));
    CK(hipMalloc(&sink, 4096 * 4));
    CK(hipMalloc(&big, (size_t)512 << 20));  // evicts the Infinity Cache
    CK(hipMemset(C, 0, (size_t)n * m * 4));
    CK(hipMemset(cs, 0, (size_t)64 * m * 4));
    const int grid = 256;
    const int it = 50;
    printf("stream(64MiB, L3-warm)         %8.2f us\n", timeit([&] { pass_like<16, true, false><<<grid, NT>>>(C, n, m, cs, 1, sink); }, it));
    printf("stream after 512MiB write       %8.2f us\n", timeit([&] { (void)hipMemsetAsync(big, 1, (size_t)512 << 20); pass_like<16, true, false><<<grid, NT>>>(C, n, m, cs, 1, sink); }, 10) -
                                                     timeit([&] { (void)hipMemsetAsync(big, 1, (size_t)512 << 20); }, 10));
    for (int reps : {1, 2, 4, 8, 16, 32, 64})
        printf("flush only reps=%-3d             %8.2f us\n", reps, timeit([&] { pass_like<16, false, true><<<grid, NT>>>(C, n, m, cs, reps, sink); }, it));
    for (int reps : {1, 8, 16, 64})
        printf("stream+flush reps=%-3d           %8.2f us\n", reps, timeit([&] { pass_like<16, true, true><<<grid, NT>>>(C, n, m, cs, reps, sink); }, it));
    printf("empty launch                    %8.2f us\n", timeit([&] { pass_like<16, false, false><<<grid, NT>>>(C, 0, m, cs, 1, sink); }, it));
    printf("stream 2 WG/CU (8 rows, 512 WGs)%8.2f us\n", timeit([&] { pass_like<8, true, false><<<512, NT>>>(C, n, m, cs, 1, sink); }, it));
    return 0;
}
