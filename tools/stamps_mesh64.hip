// Diagnostic: the float64 mesh engine's iteration split into phases (wave 0 of every
// workgroup, iterations 3..13, mean over workgroups).  Builds the library sources with
// -DOTF_M64_STAMPS and runs the float64 metric shape (N = 4096, eps 0.1, 100 iterations).
// Build: hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics -DOTF_M64_STAMPS -I include \
//        tools/stamps_mesh64.hip -o tools/stamps_mesh64
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_common.hip"
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_sinkhorn.hip"
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_sweep.hip"
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_gather.hip"
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_mesh.hip"
// OTF_M64_ALT: an alternative float64 mesh source to time in place of the library's (A/B)
#ifdef OTF_M64_ALT
#include OTF_M64_ALT
#else
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_mesh64.hip"
#endif
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_comm.hip"

#include <algorithm>
#include <string>
#include <cmath>
#include <cstdio>
#include <vector>

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 4096;
    const int iters = argc > 2 ? atoi(argv[2]) : 100;
    double *C, *a, *u, *v, *P;
    otf_sinkhorn_info* info;
    (void)hipMalloc(&C, (size_t)N * N * 8);
    (void)hipMalloc(&a, N * 8);
    (void)hipMalloc(&u, N * 8);
    (void)hipMalloc(&v, N * 8);
    (void)hipMalloc(&P, (size_t)N * N * 8);
    (void)hipMalloc(&info, sizeof(otf_sinkhorn_info));
    std::vector<double> h((size_t)N * N);
    unsigned s = 1;
    for (auto& x : h) { s = s * 1664525u + 1013904223u; x = (s >> 8) * (1.0 / 16777216.0); }
    (void)hipMemcpy(C, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    std::vector<double> ha(N, 1.0 / N);
    (void)hipMemcpy(a, ha.data(), N * 8, hipMemcpyHostToDevice);
    const size_t wsb = otf_sinkhorn_workspace_size(N, N, OTF_F64, iters);
    void* ws;
    (void)hipMalloc(&ws, wsb);
    otf_sinkhorn_opts o{};
    o.reg = 0.1; o.stop_thr = 0; o.max_iter = iters; o.check_every = 10;
    o.flavor = OTF_FLAVOR_POT; o.engine = OTF_ENGINE_MESH;
    // "pw": the fused pairwise form (otf_sinkhorn_pairwise_f64) on float32 rows, d = 512
    const bool pw = argc > 3 && std::string(argv[3]) == "pw";
    const int d = 512;
    float *X = nullptr, *Y = nullptr;
    double* cmax = nullptr;
    void* wsp = nullptr;
    size_t wspb = 0;
    if (pw) {
        std::vector<float> hx((size_t)N * d);
        for (auto& x : hx) { s = s * 1664525u + 1013904223u; x = (float)((s >> 8) * (1.0 / 16777216.0)) - 0.5f; }
        (void)hipMalloc(&X, hx.size() * 4);
        (void)hipMalloc(&Y, hx.size() * 4);
        (void)hipMemcpy(X, hx.data(), hx.size() * 4, hipMemcpyHostToDevice);
        for (auto& x : hx) { s = s * 1664525u + 1013904223u; x = (float)((s >> 8) * (1.0 / 16777216.0)) - 0.5f; }
        (void)hipMemcpy(Y, hx.data(), hx.size() * 4, hipMemcpyHostToDevice);
        (void)hipMalloc(&cmax, 8);
        wspb = otf_sinkhorn_pairwise_f64_workspace_size(N, N, iters);
        (void)hipMalloc(&wsp, wspb);
    }
    for (int rep = 0; rep < 4; ++rep) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0, 0);
        const int rc = pw ? otf_sinkhorn_pairwise_f64(X, d, Y, d, N, N, d, OTF_SQEUCLIDEAN, 1, a, a, &o, u, v, P, N,
                                                      OTF_F64, cmax, info, nullptr, wsp, wspb, 0)
                          : otf_sinkhorn(a, a, C, N, N, N, OTF_F64, nullptr, &o, u, v, P, N, OTF_F64, info,
                                         nullptr, ws, wsb, 0);
        (void)hipEventRecord(e1, 0);
        (void)hipDeviceSynchronize();
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        otf_sinkhorn_info hi;
        (void)hipMemcpy(&hi, info, sizeof(hi), hipMemcpyDeviceToHost);
        printf("rc=%d status=%d engine=%d solve %.3f ms\n", rc, hi.status, hi.engine, ms);
    }
    std::vector<unsigned long long> st(256 * 16 * 8);
    (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(otf::g_m64st), st.size() * 8);
    std::vector<unsigned long long> pro(256 * 4);
    (void)hipMemcpyFromSymbol(pro.data(), HIP_SYMBOL(otf::g_m64pro), pro.size() * 8);
    double pa[3] = {0};
    unsigned long long t0 = ~0ull, tend = 0;
    for (int r = 0; r < 256; ++r) {
        for (int k = 0; k < 3; ++k) pa[k] += (double)(pro[r * 4 + k + 1] - pro[r * 4 + k]);
        t0 = std::min(t0, pro[r * 4]);
        tend = std::max(tend, pro[r * 4 + 3]);
    }
    printf("  start -> roles (registration)   %7.3f us (mean)\n", pa[0] / 256 * 0.01);
    printf("  roles -> K formed (C / cost, exp) %7.3f us\n", pa[1] / 256 * 0.01);
    printf("  K formed -> loop end            %7.3f us\n", pa[2] / 256 * 0.01);
    printf("  first start -> last loop end    %7.3f us\n", (tend - t0) * 0.01);
    if (pw) {
        std::vector<unsigned long long> q(256 * 4);
        (void)hipMemcpyFromSymbol(q.data(), HIP_SYMBOL(otf::g_m64pw), q.size() * 8);
        double m[4] = {0}, mx[4] = {0}, mn[4] = {1e30, 1e30, 1e30, 1e30};
        for (int r = 0; r < 256; ++r) {
            const unsigned long long prev[4] = {pro[r * 4 + 1], q[r * 4], q[r * 4 + 1], q[r * 4 + 2]};
            for (int k = 0; k < 4; ++k) {
                const double dt = (double)(q[r * 4 + k] - prev[k]) * 0.01;
                m[k] += dt / 256;
                mx[k] = std::max(mx[k], dt);
                mn[k] = std::min(mn[k], dt);
            }
        }
        const char* nm[4] = {"block 3 (wave 0)", "blocks 0..2 (until all waves)", "grid max (atomic + barrier)",
                             "K = exp in place"};
        for (int k = 0; k < 4; ++k)
            printf("    %-30s mean %8.3f us  min %8.3f  max %8.3f us\n", nm[k], m[k], mn[k], mx[k]);
        // when the workgroups finished their tiles, relative to the first one
        unsigned long long f0 = ~0ull;
        for (int r = 0; r < 256; ++r) f0 = std::min(f0, q[r * 4 + 1]);
        double sk[8] = {0};
        int nx[8] = {0};
        for (int r = 0; r < 256; ++r) { sk[r % 8] += (q[r * 4 + 1] - f0) * 0.01; nx[r % 8]++; }
        // effective shader clock per phase: s_memtime cycles over s_memrealtime (100 MHz) ticks
        std::vector<unsigned long long> c(256 * 5);
        (void)hipMemcpyFromSymbol(c.data(), HIP_SYMBOL(otf::g_m64pwc), c.size() * 8);
        double cyc[4] = {0}, tk[4] = {0};
        for (int r = 0; r < 256; ++r) {
            const unsigned long long rt[5] = {0, q[r * 4], q[r * 4 + 1], q[r * 4 + 2], q[r * 4 + 3]};
            for (int k = 1; k < 4; ++k) {
                cyc[k] += (double)(c[r * 5 + k + 1] - c[r * 5 + k]);
                tk[k] += (double)(rt[k + 1] - rt[k]);
            }
            cyc[0] += (double)(c[r * 5 + 1] - c[r * 5]);
        }
        printf("    shader clock: entry -> block 3 done %.1f Mcycles/WG", cyc[0] / 256 / 1e6);
        printf("; blocks 0..2 %.3f GHz, grid max %.3f GHz, exp %.3f GHz\n", cyc[1] / tk[1] / 10.0,
               cyc[2] / tk[2] / 10.0, cyc[3] / tk[3] / 10.0);
        {
            double t3 = 0;
            for (int r = 0; r < 256; ++r) t3 += (double)(q[r * 4] - pro[r * 4 + 1]);
            printf("    block 3 (roles -> block 3 done, incl. entry) %.3f GHz\n", cyc[0] / t3 / 10.0);
        }
        printf("    tile done after the first, by role %% 8:");
        for (int x = 0; x < 8; ++x) printf(" %.1f", sk[x] / nx[x]);
        printf(" us\n");
    }
    const char* names[7] = {"hop B (poll, v)", "row partials (8 rows x 16 cols)", "B1 + row publish (wave 0)",
                            "row hop gather + u", "B2", "col partials + publish", "reduce (wave 0)"};
    double acc[8] = {0};
    int cnt = 0;
    for (int r = 0; r < 256; ++r)
        for (int it = 3; it < 14; ++it) {
            const unsigned long long* q = &st[((size_t)r * 16 + it) * 8];
            const unsigned long long* qn = &st[((size_t)r * 16 + it + 1) * 8];
            if (q[0] == 0 || qn[0] == 0) continue;
            for (int k = 0; k < 7; ++k) acc[k] += (double)(q[k + 1] - q[k]);
            acc[7] += (double)(qn[0] - q[7]);
            ++cnt;
        }
    double tot = 0;
    for (int k = 0; k < 7; ++k) {
        printf("  %-30s %7.3f us\n", names[k], acc[k] / cnt * 0.01);
        tot += acc[k];
    }
    printf("  %-30s %7.3f us\n", "loop back", acc[7] / cnt * 0.01);
    tot += acc[7];
    printf("  = iteration                    %7.3f us  (%d samples)\n", tot / cnt * 0.01, cnt);
    return 0;
}
