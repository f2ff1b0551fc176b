// Diagnostic: where does the GW kernel spend its time?  Builds the library sources
// with -DOTF_GW_STAMPS and prints per-phase wall-clock totals of workgroup 0
// (s_memrealtime, 10 ns ticks): GEMMs (+ marginal mat-vecs), assignment (LAP),
// inner Sinkhorn, whole kernel.  Problem: 2 labels of n random points (CG: euclidean,
// entropic: sqeuclidean, both max-scaled), n from argv (default 64).
// Build: hipcc -O3 --offload-arch=gfx950 -DOTF_GW_STAMPS -I include -I <pkg>/csrc \
//        tools/stamps_gw.hip -o tools/stamps_gw
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_common.hip"
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_linalg.hip"
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_gw.hip"

#include <cmath>
#include <cstdio>
#include <vector>

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 64, d = 16;
    std::vector<float> h(2 * (size_t)n * d);
    unsigned s = 7;
    for (auto& x : h) { s = s * 1664525u + 1013904223u; x = (s >> 8) * (1.0f / 16777216.0f); }
    float* X;
    double *C[4], *T[2], *cm;
    (void)hipMalloc(&X, h.size() * 4);
    (void)hipMemcpy(X, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    for (auto& c : C) (void)hipMalloc(&c, (size_t)n * n * 8);
    for (auto& t : T) (void)hipMalloc(&t, (size_t)n * n * 8);
    (void)hipMalloc(&cm, 8);
    void* dws;
    const size_t dwb = otf_cost_pairwise_f64_workspace_size(n, n);
    (void)hipMalloc(&dws, dwb);
    otf_gw_info* info;
    (void)hipMalloc(&info, 2 * sizeof(otf_gw_info));
    for (int solver = 0; solver < 3; ++solver) {
        const int metric = solver == OTF_GW_CG ? OTF_EUCLIDEAN : OTF_SQEUCLIDEAN;
        for (int k = 0; k < 2; ++k) {
            otf_cost_pairwise_f64(X, d, X, d, n, n, d, metric, solver == OTF_GW_CG, 1, C[2 * k], n, cm, dws, dwb, 0);
            otf_cost_pairwise_f64(X + (size_t)n * d, d, X + (size_t)n * d, d, n, n, d, metric, solver == OTF_GW_CG, 1, C[2 * k + 1], n, cm, dws, dwb, 0);
        }
        otf_gw_problem pr[2];
        for (int k = 0; k < 2; ++k) {
            pr[k] = otf_gw_problem{C[2 * k], n, C[2 * k + 1], n, nullptr, nullptr, nullptr, nullptr, T[k], n, n, n};
        }
        otf_gw_opts o{};
        o.solver = solver; o.max_iter = solver == OTF_GW_CG ? 10000 : solver == OTF_GW_PGD ? 1000 : 2000; o.min_iter = 5;
        o.sk_max_iter = solver == OTF_GW_PGD ? 1000 : 2000; o.sk_inner = 10; o.warm_start = 1; o.tol_rel = 1e-9; o.tol_abs = 1e-9;
        o.threshold = 1e-3; o.sk_threshold = solver == OTF_GW_PGD ? 1e-9 : 1e-3; o.eps = 5e-3;
        const size_t wsb = otf_gw_workspace_size(2, pr);
        void* ws;
        (void)hipMalloc(&ws, wsb);
        for (int rep = 0; rep < 2; ++rep) {
            unsigned long long st[128], sk[4] = {0, 0, 0, 0};
            (void)hipMemcpyToSymbol(HIP_SYMBOL(otf::g_gw_sk), sk, sizeof(sk));
            int rc = otf_gw_solve(2, pr, &o, info, nullptr, 0, ws, wsb, 0);
            (void)hipDeviceSynchronize();
            (void)hipMemcpyFromSymbol(sk, HIP_SYMBOL(otf::g_gw_sk), sizeof(sk));
            (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(otf::g_gw_stamps), sizeof(st));
            otf_gw_info hi[2];
            (void)hipMemcpy(hi, info, sizeof(hi), hipMemcpyDeviceToHost);
            printf("%s n=%d rc=%d outer=%d inner=%d | gemm %.1f us  lap %.1f us  sinkhorn %.1f us  total %.1f us\n",
                   solver == OTF_GW_CG ? "cg" : solver == OTF_GW_PGD ? "pgd" : "entropic", n, rc, hi[0].n_iter, hi[0].inner_iters,
                   st[0] / 100.0, st[1] / 100.0, st[2] / 100.0, st[3] / 100.0);
            if (hi[0].inner_iters) printf("   per update: col %.2f us  row %.2f us; per check: err %.2f us\n", sk[0] / 100.0 / hi[0].inner_iters, sk[1] / 100.0 / hi[0].inner_iters, sk[2] / 100.0 / (hi[0].inner_iters / 10.0));
        }
        (void)hipFree(ws);
    }
    return 0;
}
