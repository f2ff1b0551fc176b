// otf_emd.hip — exact EMD with general marginals on the device: the batched launch
// (one workgroup per problem) behind otf_emd_solve.  The solver is emd_block
// (otf_emd.h).
#include <stdlib.h>

#include "otf_emd.h"

namespace otf {
namespace {

constexpr int kEmdNT = 256;
constexpr int kEmdMaxP = 64;

struct EmdLaunch {
    otf_emd_problem prob[kEmdMaxP];
    int nprob;
    unsigned char* tree;      // global-tree launches: one region per problem
    size_t tree_stride;
};

__global__ __launch_bounds__(kEmdNT) void emd_kernel(EmdLaunch L, int64_t max_pivots, otf_emd_info* info) {
    extern __shared__ __attribute__((aligned(16))) unsigned char esm[];
    const otf_emd_problem& P = L.prob[blockIdx.x];
    const size_t tb = ((size_t)(P.n + P.m + 1) * kEmdNodeBytes + 15) / 16 * 16;
    const otf_emd_info out = emd_block<kEmdNT>(P, max_pivots, esm, esm + tb);
    if (threadIdx.x == 0) info[blockIdx.x] = out;
}

// trees past the LDS: node arrays in the launch's global region, scratch in LDS
__global__ __launch_bounds__(kEmdNT) void emd_kernel_g(EmdLaunch L, int64_t max_pivots, otf_emd_info* info) {
    __shared__ __attribute__((aligned(16))) unsigned char scr[kEmdScratch];
    const otf_emd_info out =
        emd_block<kEmdNT, int>(L.prob[blockIdx.x], max_pivots, L.tree + blockIdx.x * L.tree_stride, scr);
    if (threadIdx.x == 0) info[blockIdx.x] = out;
}

}  // namespace
}  // namespace otf
extern "C" {

// n + m + 1 of the largest problem otf_emd_solve takes (n * m + n + m < 2^31 also
// holds); up to kEmdMaxNodes the tree stays in LDS
int otf_emd_max_nodes(void) { return INT32_MAX / 2; }
int otf_emd_lds_nodes(void) { return otf::kEmdMaxNodes; }

int otf_emd_solve(int32_t nprob, const otf_emd_problem* probs, int64_t max_pivots,
                  otf_emd_info* info, otf_stream_t stream) {
    if (nprob <= 0 || !probs || !info || max_pivots < 1) return OTF_EINVAL;
    for (int b = 0; b < nprob; ++b) {
        const otf_emd_problem& P = probs[b];
        if (!P.a || !P.b || !P.M || !P.T || P.n < 1 || P.m < 1) return OTF_EINVAL;
        if (P.ldm < P.m || P.ldt < P.m) return OTF_EINVAL;
        if (!otf::emd_fits_g(P.n, P.m)) return OTF_EUNSUPPORTED;
    }
    hipStream_t s = (hipStream_t)stream;
    for (int first = 0; first < nprob; first += otf::kEmdMaxP) {
        otf::EmdLaunch L{};
        L.nprob = nprob - first < otf::kEmdMaxP ? nprob - first : otf::kEmdMaxP;
        int64_t maxN = 0;
        for (int b = 0; b < L.nprob; ++b) {
            L.prob[b] = probs[first + b];
            const int64_t N = (int64_t)L.prob[b].n + L.prob[b].m + 1;
            maxN = N > maxN ? N : maxN;
        }
        // OTF_EMD_TREE=global: the global-memory tree at any size (tests: same pivots)
        const char* te = getenv("OTF_EMD_TREE");
        const bool force_g = te && te[0] == 'g';
        if (maxN <= otf::kEmdMaxNodes && !force_g) {
            const size_t lds = otf::emd_lds_bytes((int)maxN);
            OTF_HIP(hipFuncSetAttribute((const void*)otf::emd_kernel,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            otf::emd_kernel<<<L.nprob, otf::kEmdNT, lds, s>>>(L, max_pivots, info + first);
            OTF_HIP(hipGetLastError());
        } else {
            // stream-ordered tree storage, released behind the launch
            L.tree_stride = otf::emd_tree_bytes_g(maxN);
            void* tree = nullptr;
            OTF_HIP(hipMallocAsync(&tree, L.tree_stride * L.nprob, s));
            L.tree = (unsigned char*)tree;
            otf::emd_kernel_g<<<L.nprob, otf::kEmdNT, 0, s>>>(L, max_pivots, info + first);
            const hipError_t le = hipGetLastError();
            OTF_HIP(hipFreeAsync(tree, s));
            OTF_HIP(le);
        }
    }
    return OTF_OK;
}

}  // extern "C"
