// host_asan_check.cpp -- test infrastructure: the HOST side of libotfuse (workspace
// carving, shape / argument validation, the error conventions of include/otfuse.h) built
// with -fsanitize=address,undefined (csrc/Makefile target `host-asan`, device code left
// out with --offload-host-only) and driven here without a GPU.  Every call below returns
// before the first HIP call; an out-of-bounds access, overflow or UB in the host logic
// aborts the run (tests/test_sanitizers.py).
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "otfuse.h"

static int failures = 0;
#define CHECK(cond, ...)                                         \
    do {                                                         \
        if (!(cond)) {                                           \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                        \
            fprintf(stderr, "\n");                               \
            ++failures;                                          \
        }                                                        \
    } while (0)

int main() {
    CHECK(strncmp(otf_version(), "otfuse", 6) == 0, "version %s", otf_version());
    // workspace carving over ragged shapes, both dtypes, 0 .. 5000 iterations; the shifted
    // kernel's offsets must lie inside the float32 workspace
    const int64_t ns[] = {1, 2, 63, 64, 65, 127, 513, 4096, 5000, 16384};
    const int32_t iters[] = {0, 1, 100, 2000, 5000};
    for (int64_t n : ns)
        for (int64_t m : ns)
            for (int32_t it : iters) {
                const size_t w32 = otf_sinkhorn_workspace_size(n, m, OTF_F32, it);
                const size_t w64 = otf_sinkhorn_workspace_size(n, m, OTF_F64, it);
                CHECK(w32 > 0 && w64 > 0, "workspace %lld x %lld", (long long)n, (long long)m);
                size_t oa = 0, ob = 0;
                CHECK(otf_sinkhorn_shift_offsets(n, m, OTF_F32, it, &oa, &ob) == OTF_OK, "offsets");
                CHECK(oa % 256 == 0 && ob % 256 == 0, "offsets aligned");
                CHECK(oa + 4 * (size_t)n <= w32 && ob + 4 * (size_t)m <= w32,
                      "shift offsets inside the workspace (%lld x %lld)", (long long)n, (long long)m);
                CHECK(otf_sinkhorn_shift_offsets(n, m, OTF_F64, it, &oa, &ob) == OTF_EUNSUPPORTED,
                      "float64 has no shifted kernel");
            }
    size_t oa, ob;
    CHECK(otf_sinkhorn_shift_offsets(0, 5, OTF_F32, 10, &oa, &ob) == OTF_EINVAL, "empty n");
    CHECK(otf_sinkhorn_shift_offsets(5, 5, OTF_F32, 10, nullptr, &ob) == OTF_EINVAL, "null out");
    // cost / feature / coupled / GW / EMD workspace queries
    for (int64_t n : ns) {
        CHECK(otf_cost_split16_workspace_size(n, n + 3, 512) > 0, "split16 ws");
        CHECK(otf_cost_ex_workspace_size(n, 2 * n, 1024, OTF_F16) > 0, "cost_ex ws f16");
        CHECK(otf_cost_ex_workspace_size(n, 7, 33, OTF_F32) > 0, "cost_ex ws f32");
        CHECK(otf_feature_cost_workspace_size(n, n, 64, 48) > 0, "feature ws");
        CHECK(otf_coupled_cost_workspace_size(n, 9, 17) > 0, "coupled ws");
        CHECK(otf_cost_pairwise_f64_workspace_size(n, n) > 0, "f64 cost ws");
    }
    std::vector<otf_gw_problem> probs(5);
    for (int k = 0; k < 5; ++k) {
        memset(&probs[k], 0, sizeof(otf_gw_problem));
        probs[k].n = 1 + 97 * k;
        probs[k].m = 1 + 61 * k;
    }
    CHECK(otf_gw_workspace_size(5, probs.data()) > 0, "gw ws");
    CHECK(otf_emd_max_nodes() > otf_emd_lds_nodes() && otf_emd_lds_nodes() > 0, "emd nodes");
    CHECK(otf_xpeer_handle_size() > 0, "xpeer handle");
    // argument errors: returned before any device work
    otf_sinkhorn_opts o;
    memset(&o, 0, sizeof(o));
    o.reg = 0.1;
    o.max_iter = 10;
    o.check_every = 10;
    float fake[64];
    otf_sinkhorn_info* info = reinterpret_cast<otf_sinkhorn_info*>(fake);
    CHECK(otf_sinkhorn(fake, fake, fake, 4, 4, 4, OTF_F32, nullptr, nullptr, fake, fake, nullptr, 0,
                       OTF_F32, info, nullptr, fake, 0, nullptr) == OTF_EINVAL, "null opts");
    CHECK(otf_sinkhorn(fake, fake, fake, 4, 4, 4, OTF_F32, nullptr, &o, nullptr, fake, nullptr, 0,
                       OTF_F32, info, nullptr, fake, 0, nullptr) == OTF_EINVAL, "null u_out");
    CHECK(otf_sinkhorn(fake, fake, fake, 4, 4, 3, OTF_F32, nullptr, &o, fake, fake, nullptr, 0,
                       OTF_F32, info, nullptr, fake, 0, nullptr) == OTF_EINVAL, "ldc < m");
    CHECK(otf_sinkhorn(fake, fake, fake, 4, 4, 4, OTF_F32, nullptr, &o, fake, fake, nullptr, 0,
                       OTF_F32, info, nullptr, fake, 16, nullptr) == OTF_EINVAL, "workspace too small");
    o.reg = 0.0;
    CHECK(otf_sinkhorn(fake, fake, fake, 4, 4, 4, OTF_F32, nullptr, &o, fake, fake, nullptr, 0,
                       OTF_F32, info, nullptr, fake, 1 << 30, nullptr) == OTF_EINVAL, "reg 0");
    o.reg = 0.1;
    o.shift = 1;
    o.flavor = OTF_FLAVOR_OTT;
    CHECK(otf_sinkhorn(fake, fake, fake, 4, 4, 4, OTF_F32, nullptr, &o, fake, fake, fake, 4, 7,
                       info, nullptr, fake, 1 << 30, nullptr) == OTF_EINVAL, "bad plan dtype");
    CHECK(otf_sinkhorn(fake, fake, fake, 4, 4, 4, 9, nullptr, &o, fake, fake, nullptr, 0, OTF_F32,
                       info, nullptr, fake, 1 << 30, nullptr) == OTF_EINVAL, "bad dtype");
    CHECK(otf_emd_solve(0, nullptr, 10, nullptr, nullptr) != OTF_OK, "emd no problems");
    if (failures) {
        fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    printf("host_asan_check: host logic clean\n");
    return 0;
}
