// otf_emd.hip — exact EMD with general marginals on the device: the batched launch
// (one workgroup per problem) behind otf_emd_solve.  The solver is emd_block
// (otf_emd.h).
#include "otf_emd.h"

namespace otf {
namespace {

constexpr int kEmdNT = 256;
constexpr int kEmdMaxP = 64;

struct EmdLaunch {
    otf_emd_problem prob[kEmdMaxP];
    int nprob;
};

__global__ __launch_bounds__(kEmdNT) void emd_kernel(EmdLaunch L, int64_t max_pivots, otf_emd_info* info) {
    extern __shared__ __attribute__((aligned(16))) unsigned char esm[];
    const otf_emd_info out = emd_block<kEmdNT>(L.prob[blockIdx.x], max_pivots, esm);
    if (threadIdx.x == 0) info[blockIdx.x] = out;
}

}  // namespace
}  // namespace otf
extern "C" {

int otf_emd_max_nodes(void) { return otf::kEmdMaxNodes; }

int otf_emd_solve(int32_t nprob, const otf_emd_problem* probs, int64_t max_pivots,
                  otf_emd_info* info, otf_stream_t stream) {
    if (nprob <= 0 || !probs || !info || max_pivots < 1) return OTF_EINVAL;
    for (int b = 0; b < nprob; ++b) {
        const otf_emd_problem& P = probs[b];
        if (!P.a || !P.b || !P.M || !P.T || P.n < 1 || P.m < 1) return OTF_EINVAL;
        if (P.ldm < P.m || P.ldt < P.m) return OTF_EINVAL;
        if ((int64_t)P.n + P.m + 1 > otf::kEmdMaxNodes) return OTF_EUNSUPPORTED;
    }
    hipStream_t s = (hipStream_t)stream;
    for (int first = 0; first < nprob; first += otf::kEmdMaxP) {
        otf::EmdLaunch L{};
        L.nprob = nprob - first < otf::kEmdMaxP ? nprob - first : otf::kEmdMaxP;
        int maxN = 0;
        for (int b = 0; b < L.nprob; ++b) {
            L.prob[b] = probs[first + b];
            const int N = L.prob[b].n + L.prob[b].m + 1;
            maxN = N > maxN ? N : maxN;
        }
        const size_t lds = otf::emd_lds_bytes(maxN);
        OTF_HIP(hipFuncSetAttribute((const void*)otf::emd_kernel,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        otf::emd_kernel<<<L.nprob, otf::kEmdNT, lds, s>>>(L, max_pivots, info + first);
        OTF_HIP(hipGetLastError());
    }
    return OTF_OK;
}

}  // extern "C"
