// Diagnostic: the TWO-HOP mesh (otf_mesh2.hip) iteration split into hop latencies and
// producer skew.  Builds the library sources with -DOTF_MESH2_STAMPS, runs the bench shape
// (N = 4096 fp32, eps 0.1, 100 iterations) and pairs every consumer stamp with the
// stamps of the producers it waited for (roles rb, cb recorded per workgroup), so a hop
// reads as: consumer done - LAST producer's publish = the hop's own latency, and the
// spread of the producers' publish times = the skew the consumer had to absorb.
// s_memrealtime is the device-wide 100 MHz clock (10 ns ticks): averaged over 256
// workgroups x iterations 3..13.
// Build: hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics -DOTF_MESH2_STAMPS -I include \
//        tools/stamps_mesh2.hip -o tools/stamps_mesh2 -ldl
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_common.hip"
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_sinkhorn.hip"
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_sweep.hip"
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_gather.hip"
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_mesh.hip"
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_mesh2.hip"
#include "../ot-based-heterogeneous-multi-modal-fusion-embedding-for-ad-analysis-_amd/csrc/otf_comm.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

int main(int argc, char** argv) {
    setenv("OTF_MESH2", argc > 4 ? argv[4] : "1", 1);
    const int N = argc > 1 ? atoi(argv[1]) : 4096;
    const int iters = argc > 2 ? atoi(argv[2]) : 100;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
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
    for (auto& x : h) { s = s * 1664525u + 1013904223u; x = (float)((s >> 8) * (1.0 / 16777216.0)); }
    (void)hipMemcpy(C, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    std::vector<float> ha(N, 1.0f / N);
    (void)hipMemcpy(a, ha.data(), N * 4, hipMemcpyHostToDevice);
    const size_t wsb = otf_sinkhorn_workspace_size(N, N, OTF_F32, iters);
    void* ws;
    (void)hipMalloc(&ws, wsb);
    otf_sinkhorn_opts o{};
    o.reg = 0.1; o.stop_thr = 0; o.max_iter = iters; o.check_every = 10;
    o.flavor = OTF_FLAVOR_POT; o.engine = OTF_ENGINE_MESH;
    std::vector<float> tms;
    for (int rep = 0; rep < reps; ++rep) {
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
        if (rc != 0 || hi.status != OTF_SK_MAX_ITER) return 3;
        if (rep > 0) tms.push_back(ms * 1000 / iters);
    }
    std::sort(tms.begin(), tms.end());
    if (!tms.empty()) printf("median %.3f us/iter\n", tms[tms.size() / 2]);
    {   // correctness against the streaming engine on the same input (u_i v_j products)
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
        double umax = 0, vmax = 0, du = 0, dv = 0;
        const double cu = (double)ur[0] / us[0];
        for (int i = 0; i < N; ++i) {
            umax = fmax(umax, fabs((double)us[i]));
            vmax = fmax(vmax, fabs((double)vs[i]));
            du = fmax(du, fabs((double)ur[i] / cu - us[i]));
            dv = fmax(dv, fabs((double)vr[i] * cu - vs[i]));
        }
        const bool ok = du / umax < 1e-4 && dv / vmax < 1e-4;
        printf("stream rc=%d  mesh2 vs stream: rel u %.3e  rel v %.3e  %s\n", rc, du / umax, dv / vmax,
               ok ? "OK" : "MISMATCH");
        if (!ok) return 4;
    }
#ifdef OTF_MESH2_STAMPS
    std::vector<unsigned long long> st(256 * 16 * 16);
    std::vector<int> role(256 * 4);
    (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(otf::g_m2stamps), st.size() * 8);
    (void)hipMemcpyFromSymbol(role.data(), HIP_SYMBOL(otf::g_m2role), role.size() * 4);
    int nw = 0;
    for (int w = 0; w < 256; ++w)
        if (role[w * 4 + 3]) nw = w + 1;
    auto S = [&](int w, int it, int slot) -> double { return (double)st[(w * 16 + it) * 16 + slot]; };
    const char* names[7] = {"column gather (wait + loads)", "barrier + S + v", "row partials + publish",
                            "row hop (wave 0)", "u + col partials + barrier", "publish cols", "loop back"};
    double ph[7] = {0};
    double lat_col = 0, lat_row0 = 0, lat_row7 = 0, sk_col = 0, sk_row = 0, wsk_pub = 0, wsk_done = 0;
    int cnt = 0;
    for (int it = 3; it < 14; ++it) {
        for (int w = 0; w < nw; ++w) {
            const int rb = role[w * 4], cb = role[w * 4 + 1];
            ph[0] += S(w, it, 1) - S(w, it, 0);
            ph[1] += S(w, it, 2) - S(w, it, 1);
            ph[2] += S(w, it, 3) - S(w, it, 2);
            ph[3] += S(w, it, 4) - S(w, it, 3);
            ph[4] += S(w, it, 5) - S(w, it, 4);
            ph[5] += S(w, it, 6) - S(w, it, 5);
            ph[6] += S(w, it + 1, 0) - S(w, it, 6);
            double m3 = 0, m3min = 1e30, m10 = 0, m6 = 0, m6min = 1e30;
            for (int q = 0; q < nw; ++q) {
                if (role[q * 4] == rb) {
                    m3 = std::max(m3, S(q, it, 3));
                    m3min = std::min(m3min, S(q, it, 3));
                    m10 = std::max(m10, S(q, it, 10));
                }
                if (role[q * 4 + 1] == cb) {
                    m6 = std::max(m6, S(q, it, 6));
                    m6min = std::min(m6min, S(q, it, 6));
                }
            }
            lat_col += S(w, it + 1, 1) - m6;
            lat_row0 += S(w, it, 4) - m3;
            lat_row7 += S(w, it, 9) - m10;
            sk_col += m6 - m6min;
            sk_row += m3 - m3min;
            wsk_pub += S(w, it, 10) - S(w, it, 3);
            wsk_done += S(w, it, 9) - S(w, it, 4);
            ++cnt;
        }
    }
    const double k = 1.0 / cnt / 100.0;  // ticks (10 ns) -> us per workgroup-iteration
    printf("workgroups %d (roles), iterations 3..13\n", nw);
    double sum = 0;
    for (int i = 0; i < 7; ++i) {
        printf("  %-30s %6.3f us\n", names[i], ph[i] * k);
        sum += ph[i] * k;
    }
    printf("  %-30s %6.3f us\n", "= iteration", sum);
    printf("hop latencies (consumer done - LAST producer publish):\n");
    printf("  column hop (16 producers)      %6.3f us\n", lat_col * k);
    printf("  row hop, wave 0 / wave 7       %6.3f / %6.3f us\n", lat_row0 * k, lat_row7 * k);
    printf("producer skew (max - min publish):\n");
    printf("  column producers (16)          %6.3f us\n", sk_col * k);
    printf("  row members (16)               %6.3f us\n", sk_row * k);
    printf("wave skew in a workgroup (wave 7 - wave 0): publish %6.3f us, row hop done %6.3f us\n",
           wsk_pub * k, wsk_done * k);
#endif
    return 0;
}
