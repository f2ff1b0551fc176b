// Diagnostic: the split-fp16 pairwise cost (otf_cost_pairwise_ex) at a given shape,
// timed with HIP events over reps calls (prep + cost kernels); run under
// rocprofv3 --kernel-trace --stats for the per-kernel split.  Build variants:
//   -DOTF_COST_ABLATE=1  the cost kernels skip their C stores (loop + epilogue math only)
// Build: hipcc -O3 --offload-arch=gfx950 -I include -I <pkg>/csrc tools/ubench_cost.hip -o tools/ubench_cost
// Run:   OTF_COST_RING=0|1 tools/ubench_cost [N] [d] [f32|f16in] [reps]
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_common.hip"
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_cost.hip"

#include <cstdio>
#include <cstring>
#include <vector>

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 4096;
    const int d = argc > 2 ? atoi(argv[2]) : 512;
    const bool f16 = argc > 3 && strcmp(argv[3], "f16in") == 0;
    const int reps = argc > 4 ? atoi(argv[4]) : 20;
    const size_t esz = f16 ? 2 : 4;
    std::vector<unsigned char> h((size_t)N * d * esz);
    unsigned s = 7;
    for (size_t i = 0; i < (size_t)N * d; ++i) {
        s = s * 1664525u + 1013904223u;
        const float x = (float)((s >> 8) * (1.0 / 16777216.0)) - 0.5f;
        if (f16) { const _Float16 y = (_Float16)x; memcpy(&h[i * 2], &y, 2); }
        else memcpy(&h[i * 4], &x, 4);
    }
    void *X, *Y, *C, *ws;
    float *cmax, *unit;
    (void)hipMalloc(&X, h.size());
    (void)hipMalloc(&Y, h.size());
    (void)hipMemcpy(X, h.data(), h.size(), hipMemcpyHostToDevice);
    (void)hipMemcpy(Y, h.data(), h.size(), hipMemcpyHostToDevice);
    const int cdt = f16 ? OTF_F16 : OTF_F32;
    const size_t csz = f16 ? 2 : 4;
    (void)hipMalloc(&C, (size_t)N * N * csz);
    (void)hipMalloc(&cmax, 4);
    (void)hipMalloc(&unit, 4);
    const size_t wsb = otf_cost_ex_workspace_size(N, N, d, cdt);
    (void)hipMalloc(&ws, wsb);
    auto run = [&]() {
        return otf_cost_pairwise_ex(X, d, Y, d, cdt, N, N, d, OTF_SQEUCLIDEAN, 0, C, N, cdt, cmax, unit, ws,
                                    wsb, nullptr);
    };
    int rc = run();
    (void)hipDeviceSynchronize();
    if (rc != 0) { printf("rc=%d\n", rc); return 2; }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r) run();
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1000.0 / reps;
    const double gf = 2.0 * N * (double)N * d * (f16 ? 1 : 3) / 1e9;
    printf("N=%d d=%d %s: %.1f us per call (prep + cost), %.0f TFLOP/s of fp16 MFMA work\n", N, d,
           f16 ? "f16in" : "f32", us, gf / us * 1e3);
#ifdef OTF_COST_STAMPS
    {   // the last call's ring-kernel phases (wave 0 of each workgroup, 10-ns ticks)
        std::vector<unsigned long long> st(1024 * 8);
        (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(otf::g_cst), st.size() * 8);
        int nw = 0;
        unsigned long long t0 = ~0ull, t3 = 0, s0max = 0;
        double ph[4] = {0, 0, 0, 0};
        for (int w = 0; w < 1024; ++w) {
            const unsigned long long* x = &st[w * 8];
            if (x[0] == 0 || x[3] < x[0]) continue;
            ++nw;
            ph[0] += (double)(x[1] - x[0]);
            ph[1] += (double)(x[4] - x[1]);
            ph[2] += (double)(x[2] - x[4]);
            ph[3] += (double)(x[3] - x[2]);
            t0 = x[0] < t0 ? x[0] : t0;
            t3 = x[3] > t3 ? x[3] : t3;
            s0max = x[0] > s0max ? x[0] : s0max;
        }
        if (nw) printf("stamps: %d WGs  prologue %.2f  loop 1st half %.2f  2nd half %.2f  epilogue %.2f  "
                       "span %.2f  start spread %.2f us\n", nw, ph[0] / nw / 100, ph[1] / nw / 100,
                       ph[2] / nw / 100, ph[3] / nw / 100, (t3 - t0) / 100.0, (s0max - t0) / 100.0);
    }
#endif
    return 0;
}
