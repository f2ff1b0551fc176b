// Diagnostic: where does a resident-engine iteration spend its time?
// Builds the library sources with -DOTF_STAMPS, runs the bench workload shape
// (N = 4096 fp32, 100 iterations; "N resident double": config 2, float64, 1999 iterations) and prints per-phase wall-clock spans averaged
// over workgroups and iterations 2..15 (s_memrealtime, 100 MHz => 10 ns ticks):
//   0->1 sums read + v + decisions   1->2 row dots + block reduction
//   2->3 u + column partials + atomics issued   3->4 atomics performed (vmcnt 0)
//   4->5 device-wide barrier            5->0' next iteration start
// Build: hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics -DOTF_STAMPS -I include \
//        -I <pkg>/csrc tools/stamps_resident.hip -o tools/stamps_resident -ldl
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_common.hip"
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_sinkhorn.hip"
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_sweep.hip"
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_gather.hip"
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_mesh.hip"
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_comm.hip"

#include <cmath>
#include <cstdio>
#include <vector>

template <typename T>
int run(const int N, const char eng, const int iters, const double reg) {
    const bool tiled = eng == 't';
    const int dt = sizeof(T) == 8 ? OTF_F64 : OTF_F32;
    T *C, *a, *u, *v, *P;
    otf_sinkhorn_info* info;
    (void)hipMalloc(&C, (size_t)N * N * sizeof(T));
    (void)hipMalloc(&a, N * sizeof(T));
    (void)hipMalloc(&u, N * sizeof(T));
    (void)hipMalloc(&v, N * sizeof(T));
    (void)hipMalloc(&P, (size_t)N * N * sizeof(T));
    (void)hipMalloc(&info, sizeof(otf_sinkhorn_info));
    std::vector<T> h((size_t)N * N);
    unsigned s = 1;
    for (auto& x : h) { s = s * 1664525u + 1013904223u; x = (T)((s >> 8) * (1.0 / 16777216.0)); }
    (void)hipMemcpy(C, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice);
    std::vector<T> ha(N, (T)1 / N);
    (void)hipMemcpy(a, ha.data(), N * sizeof(T), hipMemcpyHostToDevice);
    const size_t wsb = otf_sinkhorn_workspace_size(N, N, dt, iters);
    void* ws;
    (void)hipMalloc(&ws, wsb);
    otf_sinkhorn_opts o{};
    o.reg = reg; o.stop_thr = 0; o.max_iter = iters; o.check_every = 10;
    o.flavor = OTF_FLAVOR_POT; o.engine = eng == 't' ? OTF_ENGINE_TILED : eng == 'g' ? OTF_ENGINE_GATHER : eng == 'm' ? OTF_ENGINE_MESH : OTF_ENGINE_RESIDENT;
    for (int rep = 0; rep < 3; ++rep) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0, 0);
        int rc = otf_sinkhorn(a, a, C, N, N, N, dt, nullptr, &o, u, v, P, N, dt, info,
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
        std::vector<T> ur(N), vr(N), us(N), vs(N);
        (void)hipMemcpy(ur.data(), u, N * sizeof(T), hipMemcpyDeviceToHost);
        (void)hipMemcpy(vr.data(), v, N * sizeof(T), hipMemcpyDeviceToHost);
        otf_sinkhorn_opts os = o;
        os.engine = OTF_ENGINE_STREAM;
        int rc = otf_sinkhorn(a, a, C, N, N, N, dt, nullptr, &os, u, v, nullptr, N, dt,
                              info, nullptr, ws, wsb, 0);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(us.data(), u, N * sizeof(T), hipMemcpyDeviceToHost);
        (void)hipMemcpy(vs.data(), v, N * sizeof(T), hipMemcpyDeviceToHost);
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
#ifndef OTF_STAMPS
    return 0;  // timing-only build (the library's own code, no stamp stores)
#else
    std::vector<unsigned long long> st(256 * 16 * 8);
    (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(otf::g_stamps), st.size() * 8);
    // resident grid: the rows per workgroup the library picked are in the stamps
    int nwg = 0;
    for (int w = 0; w < 256; ++w)
        if (st[(w * 16 + 2) * 8] != 0) nwg = w + 1;
    double span[6] = {0};
    int cnt = 0;
    double arrive_spread = 0;
    for (int it = 2; it < 15; ++it) {
        unsigned long long amin = ~0ull, amax = 0;
        for (int w = 0; w < nwg; ++w) {
            const unsigned long long* x = &st[(w * 16 + it) * 8];
            const unsigned long long* nx = &st[(w * 16 + it + 1) * 8];
            if (x[0] == 0 || nx[0] == 0) continue;  // a workgroup that left (gather team mode)
            for (int ph = 0; ph < 5; ++ph) span[ph] += (double)(x[ph + 1] - x[ph]);
            span[5] += (double)(nx[0] - x[5]);
            if (x[4] != 0) {
                amin = x[4] < amin ? x[4] : amin;
                amax = x[4] > amax ? x[4] : amax;
            }
            ++cnt;
        }
        arrive_spread += (double)(amax - amin);
    }
    const char* rnames[6] = {"sums+v+decide", "row dots+reduce", "u+partials+atomics issue",
                             "atomics performed", "grid barrier", "loop back"};
    const char* tnames[6] = {"sums+v+decide", "row partials+group wait", "gather+u",
                             "col partials+atomics done", "grid barrier", "loop back"};
    const char* gnames[6] = {"gather (poll) + sums", "v + decide", "row sums + u",
                             "col partials + publish", "-", "loop back"};
    const char* mnames[6] = {"hop B (poll) + v", "row partials + publish", "row hop (poll) + u",
                             "col partials + barrier", "publish + reduce (wave 0)", "loop back"};
    const char* const* names = tiled ? tnames : eng == 'g' ? gnames : eng == 'm' ? mnames : rnames;
    for (int ph = 0; ph < 6; ++ph) printf("%-26s %8.2f us\n", names[ph], span[ph] / cnt / 100.0);
    printf("barrier arrival spread     %8.2f us\n", arrive_spread / 13 / 100.0);
    return 0;
#endif
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 4096;
    const char eng = argc > 2 ? argv[2][0] : 'r';  // "tiled" / "gather" / "mesh" / "resident"
    const bool f64 = argc > 3 && argv[3][0] == 'd';     // third argument "double": config-2 form
    if (f64) return run<double>(N, eng, 1999, 1e-2);
    return run<float>(N, eng, 100, 0.1);
}
