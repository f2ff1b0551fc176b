// ubench_mall.hip — what read rate can a persistent sweep get from a cost that stays in
// the 256 MiB Infinity Cache (BASELINE config 5: 128 MiB fp16), by loads in flight?
// Each workgroup streams its rows of a B-byte buffer P times (no barrier between
// passes), D 16-B loads per thread in flight (register ring), trivial reduce.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_mall.hip -o tools/ubench_mall
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
using u4 = __attribute__((ext_vector_type(4))) unsigned;

template <int NT, int D>
__global__ __launch_bounds__(NT) void stream_k(const u4* buf, long n16, int passes, unsigned* sink) {
    // chunk = NT * D vectors; workgroup w takes chunks w, w + grid, ...
    const long chunk = (long)NT * D;
    const long nchunks = n16 / chunk;
    unsigned acc = 0;
    for (int p = 0; p < passes; ++p) {
        for (long c = blockIdx.x; c < nchunks; c += gridDim.x) {
            const u4* src = buf + c * chunk + threadIdx.x;
            u4 v[D];
#pragma unroll
            for (int d = 0; d < D; ++d) v[d] = __builtin_nontemporal_load(src + (long)d * NT);
#pragma unroll
            for (int d = 0; d < D; ++d) acc ^= v[d].x + v[d].y + v[d].z + v[d].w;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <int NT, int D>
__global__ __launch_bounds__(NT) void stream_plain(const u4* buf, long n16, int passes, unsigned* sink) {
    const long chunk = (long)NT * D;
    const long nchunks = n16 / chunk;
    unsigned acc = 0;
    for (int p = 0; p < passes; ++p) {
        for (long c = blockIdx.x; c < nchunks; c += gridDim.x) {
            const u4* src = buf + c * chunk + threadIdx.x;
            u4 v[D];
#pragma unroll
            for (int d = 0; d < D; ++d) v[d] = src[(long)d * NT];
#pragma unroll
            for (int d = 0; d < D; ++d) acc ^= v[d].x + v[d].y + v[d].z + v[d].w;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <typename K>
int run(const char* name, K kern, int grid, int nt, const u4* buf, long n16, unsigned* sink, double bytes) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int passes = 20;
    kern<<<grid, nt>>>(buf, n16, 2, sink);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    kern<<<grid, nt>>>(buf, n16, passes, sink);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-28s grid %4d x %4d: %8.2f us/pass  %7.0f GB/s\n", name, grid, nt, ms * 1e3 / passes,
           bytes * passes / (ms * 1e-3) / 1e9);
    return 0;
}

int main(int argc, char** argv) {
    const long MB = argc > 1 ? atol(argv[1]) : 128;
    const long bytes = MB << 20;
    const long n16 = bytes / 16;
    u4* buf;
    unsigned* sink;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 1, bytes));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    printf("buffer %ld MiB, %d CUs\n", MB, cus);
    run("plain  512 D=2", stream_plain<512, 2>, cus, 512, buf, n16, sink, bytes);
    run("plain  512 D=4", stream_plain<512, 4>, cus, 512, buf, n16, sink, bytes);
    run("plain  512 D=8", stream_plain<512, 8>, cus, 512, buf, n16, sink, bytes);
    run("plain  512 D=16", stream_plain<512, 16>, cus, 512, buf, n16, sink, bytes);
    run("plain 1024 D=4", stream_plain<1024, 4>, cus, 1024, buf, n16, sink, bytes);
    run("plain 1024 D=8", stream_plain<1024, 8>, cus, 1024, buf, n16, sink, bytes);
    run("plain  512 D=8 2/CU", stream_plain<512, 8>, 2 * cus, 512, buf, n16, sink, bytes);
    run("nt     512 D=8", stream_k<512, 8>, cus, 512, buf, n16, sink, bytes);
    run("nt     512 D=16", stream_k<512, 16>, cus, 512, buf, n16, sink, bytes);
    return 0;
}
