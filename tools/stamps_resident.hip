// Diagnostic: where does a resident-engine iteration spend its time?
// Builds the library sources with -DOTF_STAMPS, runs the bench workload shape
// (N = 4096 fp32, 100 iterations) and prints per-phase wall-clock spans averaged
// over workgroups and iterations 2..15 (s_memrealtime, 100 MHz => 10 ns ticks):
//   0->1 sums read + v + decisions   1->2 row dots + block reduction
//   2->3 u + column partials + atomics issued   3->4 atomics performed (vmcnt 0)
//   4->5 device-wide barrier            5->0' next iteration start
// Build: hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics -DOTF_STAMPS -I include \
//        -I <pkg>/csrc tools/stamps_resident.hip -o tools/stamps_resident
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_common.hip"
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_sinkhorn.hip"

#include <cmath>
#include <cstdio>
#include <vector>

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 4096;
    const bool tiled = argc > 2 && argv[2][0] == 't';  // second argument "tiled": OTF_ENGINE_TILED
    const int iters = 100;
    float *C, *a, *u, *v, *P;
    otf_sinkhorn_info* info;
    (void)hipMalloc(&C, (size_t)N * N * 4);
    (void)hipMalloc(&a, N * 4);
    (void)hipMalloc(&u, N * 4);
    (void)hipMalloc(&v, N * 4);
    (void)hipMalloc(&P, (size_t)N * N * 4);
    (void)hipMalloc(&info, sizeof(otf_sinkhorn_info));
    std::vector<float> h((size_t)N * N);
    unsigned s = 1;
    for (auto& x : h) { s = s * 1664525u + 1013904223u; x = (s >> 8) * (1.0f / 16777216.0f); }
    (void)hipMemcpy(C, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    std::vector<float> ha(N, 1.0f / N);
    (void)hipMemcpy(a, ha.data(), N * 4, hipMemcpyHostToDevice);
    const size_t wsb = otf_sinkhorn_workspace_size(N, N, OTF_F32, iters);
    void* ws;
    (void)hipMalloc(&ws, wsb);
    otf_sinkhorn_opts o{};
    o.reg = 0.1; o.stop_thr = 0; o.max_iter = iters; o.check_every = 10;
    o.flavor = OTF_FLAVOR_POT; o.engine = tiled ? OTF_ENGINE_TILED : OTF_ENGINE_RESIDENT;
    for (int rep = 0; rep < 3; ++rep) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0, 0);
        int rc = otf_sinkhorn(a, a, C, N, N, N, OTF_F32, nullptr, &o, u, v, P, N, OTF_F32, info,
                              nullptr, ws, wsb, 0);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        otf_sinkhorn_info hi;
        (void)hipMemcpy(&hi, info, sizeof(hi), hipMemcpyDeviceToHost);
        printf("rc=%d status=%d engine=%d solve %.3f ms (%.2f us/iter)\n", rc, hi.status, hi.engine,
               ms, ms * 1000 / iters);
    }
    // correctness: the resident result against the streaming engine on the same input
    {
        std::vector<float> ur(N), vr(N), us(N), vs(N);
        (void)hipMemcpy(ur.data(), u, N * 4, hipMemcpyDeviceToHost);
        (void)hipMemcpy(vr.data(), v, N * 4, hipMemcpyDeviceToHost);
        otf_sinkhorn_opts os = o;
        os.engine = OTF_ENGINE_STREAM;
        int rc = otf_sinkhorn(a, a, C, N, N, N, OTF_F32, nullptr, &os, u, v, nullptr, N, OTF_F32,
                              info, nullptr, ws, wsb, 0);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(us.data(), u, N * 4, hipMemcpyDeviceToHost);
        (void)hipMemcpy(vs.data(), v, N * 4, hipMemcpyDeviceToHost);
        // u, v are defined up to a scale (u*c, v/c): compare the products u_i v_j
        double umax = 0, vmax = 0, du = 0, dv = 0;
        const double cu = (double)ur[0] / us[0];
        for (int i = 0; i < N; ++i) {
            umax = fmax(umax, fabs((double)us[i]));
            vmax = fmax(vmax, fabs((double)vs[i]));
            du = fmax(du, fabs((double)ur[i] / cu - us[i]));
            dv = fmax(dv, fabs((double)vr[i] * cu - vs[i]));
        }
        printf("stream rc=%d  resident vs stream: rel u %.3e  rel v %.3e  %s\n", rc, du / umax,
               dv / vmax, (du / umax < 1e-4 && dv / vmax < 1e-4) ? "OK" : "MISMATCH");
    }
    std::vector<unsigned long long> st(256 * 16 * 8);
    (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(otf::g_stamps), st.size() * 8);
    int nwg = (N + 15) / 16 < 256 ? (N + 15) / 16 : 256;
    if (tiled) nwg = ((N + 127) / 128) * ((N + 511) / 512) < 256 ? ((N + 127) / 128) * ((N + 511) / 512) : 256;
    double span[6] = {0};
    int cnt = 0;
    double arrive_spread = 0;
    for (int it = 2; it < 15; ++it) {
        unsigned long long amin = ~0ull, amax = 0;
        for (int w = 0; w < nwg; ++w) {
            const unsigned long long* x = &st[(w * 16 + it) * 8];
            const unsigned long long* nx = &st[(w * 16 + it + 1) * 8];
            for (int ph = 0; ph < 5; ++ph) span[ph] += (double)(x[ph + 1] - x[ph]);
            span[5] += (double)(nx[0] - x[5]);
            amin = x[4] < amin ? x[4] : amin;
            amax = x[4] > amax ? x[4] : amax;
            ++cnt;
        }
        arrive_spread += (double)(amax - amin);
    }
    const char* rnames[6] = {"sums+v+decide", "row dots+reduce", "u+partials+atomics issue",
                             "atomics performed", "grid barrier", "loop back"};
    const char* tnames[6] = {"sums+v+decide", "row partials+group wait", "gather+u",
                             "col partials+atomics done", "grid barrier", "loop back"};
    const char* const* names = tiled ? tnames : rnames;
    for (int ph = 0; ph < 6; ++ph) printf("%-26s %8.2f us\n", names[ph], span[ph] / cnt / 100.0);
    printf("barrier arrival spread     %8.2f us\n", arrive_spread / 13 / 100.0);
    return 0;
}
