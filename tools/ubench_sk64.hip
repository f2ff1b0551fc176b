// Diagnostic: latency of one POT sinkhorn_knopp update on a 64 x 64 float64 problem (the
// PGD inner solve of otf_gw.hip small_sinkhorn_knopp, perturbot match/gw.py:31-59) in
// several forms, one workgroup, a fixed number of updates (no early stop), timed with
// s_memrealtime inside the kernel.  Prints ns per update for each form.
//   v0  8 waves x 8 columns, one FMA chain of 8, IEEE division (the library form)
//   v1  v0 with two FMA chains of 4 and the division by reciprocal + 2 Newton steps
//   v2  4 waves x 16 columns (one wave per SIMD), two FMA chains of 8, IEEE division
//   v3  v2 with the reciprocal division
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_sk64.hip -o tools/ubench_sk64
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

constexpr int N = 64, WLD = 65;

template <int O> __device__ __forceinline__ double xor_f64(double x) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, x);
    unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
    auto one = [](unsigned w) -> unsigned {
        if constexpr (O == 1) return __builtin_amdgcn_update_dpp(0u, w, 0xB1, 0xF, 0xF, false);
        else if constexpr (O == 2) return __builtin_amdgcn_update_dpp(0u, w, 0x4E, 0xF, 0xF, false);
        else if constexpr (O == 4 || O == 8) {
            const unsigned up = __builtin_amdgcn_update_dpp(0u, w, 0x100 + O, 0xF, 0xF, false);
            const unsigned dn = __builtin_amdgcn_update_dpp(0u, w, 0x110 + O, 0xF, 0xF, false);
            return (__lane_id() & O) ? dn : up;
        } else if constexpr (O == 16) {
            const auto r = __builtin_amdgcn_permlane16_swap(w, w, false, false);
            return (__lane_id() & 16) ? r[0] : r[1];
        } else {
            const auto r = __builtin_amdgcn_permlane32_swap(w, w, false, false);
            return (__lane_id() & 32) ? r[0] : r[1];
        }
    };
    lo = one(lo);
    hi = one(hi);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

template <bool RCP> __device__ __forceinline__ double divide(double a, double s) {
    if constexpr (!RCP) {
        return a / s;
    } else {
        double r = __builtin_amdgcn_rcp(s);
        double e = fma(-s, r, 1.0);
        r = fma(r, e, r);
        e = fma(-s, r, 1.0);
        r = fma(r, e, r);
        const double q = a * r;
        return fma(r, fma(-s, q, a), q);  // one residual correction
    }
}

// NW waves, CPW = 64 / NW columns (rows) per wave; lane (q, sg): q = lane % CPW,
// sg = lane / CPW covers rows (cols) sg * RPS .. + RPS, RPS = CPW * 64 / 64 ... = 64 / (64 / CPW)
template <int NW, bool RCP, int CHAINS>
__global__ void sk64_kernel(const double* K, int iters, double* out, unsigned long long* ticks) {
    constexpr int CPW = N / NW;          // columns per wave
    constexpr int SEGS = 64 / CPW;       // lane segments
    constexpr int RPS = N / SEGS;        // rows per segment
    __shared__ __attribute__((aligned(16))) double s_u[N];
    __shared__ __attribute__((aligned(16))) double s_v[N];
    __shared__ int s_kf[2];
    const int l = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
    const int q = l % CPW, sg = l / CPW;
    const int jc = CPW * w + q, ir = CPW * w + q;
    double kv[RPS], ku[RPS];
    for (int r = 0; r < RPS; ++r) kv[r] = K[(RPS * sg + r) * WLD + jc];
    for (int c = 0; c < RPS; ++c) ku[c] = 64.0 * K[ir * WLD + RPS * sg + c];
    if (threadIdx.x < N) s_u[threadIdx.x] = 1.0 / N;
    if (threadIdx.x < 2) s_kf[threadIdx.x] = 0;
    const double bj = 1.0 / N;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    double u = 0, v = 0;
    for (int ii = 0; ii < iters; ++ii) {
        double s;
        {
            double acc[CHAINS];
            for (int c = 0; c < CHAINS; ++c) acc[c] = 0;
#pragma unroll
            for (int r = 0; r < RPS; ++r) acc[r % CHAINS] = fma(kv[r], s_u[RPS * sg + r], acc[r % CHAINS]);
            s = acc[0];
            for (int c = 1; c < CHAINS; ++c) s += acc[c];
            if constexpr (SEGS >= 2) s += xor_f64<CPW>(s);
            if constexpr (SEGS >= 4) s += xor_f64<CPW * 2>(s);
            if constexpr (SEGS >= 8) s += xor_f64<CPW * 4>(s);
            if constexpr (SEGS >= 16) s += xor_f64<CPW * 8>(s);
        }
        const double vn = divide<RCP>(bj, s);
        if (sg == 0) s_v[jc] = vn;
        if (__ballot(s == 0.0 || !(vn == vn)) != 0 && l == 0) s_kf[ii & 1] = 1;
        __syncthreads();
        if (threadIdx.x == 0) s_kf[(ii + 1) & 1] = 0;
        {
            double acc[CHAINS];
            for (int c = 0; c < CHAINS; ++c) acc[c] = 0;
#pragma unroll
            for (int c = 0; c < RPS; ++c) acc[c % CHAINS] = fma(ku[c], s_v[RPS * sg + c], acc[c % CHAINS]);
            s = acc[0];
            for (int c = 1; c < CHAINS; ++c) s += acc[c];
            if constexpr (SEGS >= 2) s += xor_f64<CPW>(s);
            if constexpr (SEGS >= 4) s += xor_f64<CPW * 2>(s);
            if constexpr (SEGS >= 8) s += xor_f64<CPW * 4>(s);
            if constexpr (SEGS >= 16) s += xor_f64<CPW * 8>(s);
        }
        const double un = divide<RCP>(1.0, s);
        if (sg == 0) s_u[ir] = un;
        if (__ballot(!(un == un)) != 0 && l == 0) s_kf[ii & 1] = 1;
        __syncthreads();
        if (s_kf[ii & 1]) break;
        u = un;
        v = vn;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (blockIdx.x == 0 && sg == 0) {
        out[ir] = u;
        out[N + jc] = v;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *ticks = t1 - t0;
}

int g_grid = 1;
template <int NW, bool RCP, int CHAINS>
double run(const char* name, const double* K, int iters, double* out, unsigned long long* tk,
           std::vector<double>& ref) {
    double best = 1e30;
    for (int rep = 0; rep < 3; ++rep) {
        sk64_kernel<NW, RCP, CHAINS><<<g_grid, NW * 64>>>(K, iters, out, tk);
        unsigned long long h = 0;
        (void)hipMemcpy(&h, tk, 8, hipMemcpyDeviceToHost);
        const double ns = h * 10.0 / iters;
        if (ns < best) best = ns;
    }
    std::vector<double> o(2 * N);
    (void)hipMemcpy(o.data(), out, 2 * N * 8, hipMemcpyDeviceToHost);
    double diff = 0;
    if (ref.empty()) ref = o;
    for (int i = 0; i < 2 * N; ++i) diff = fmax(diff, fabs(o[i] - ref[i]) / fabs(ref[i]));
    printf("%-40s %8.1f ns / update   max rel diff vs v0 %.2e\n", name, best, diff);
    return best;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    std::vector<double> hk(N * WLD, 0.0);
    unsigned s = 3;
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j) {
            s = s * 1664525u + 1013904223u;
            hk[i * WLD + j] = exp(-((s >> 8) * (1.0 / 16777216.0)) / 0.05);
        }
    double *K, *out;
    unsigned long long* tk;
    (void)hipMalloc(&K, hk.size() * 8);
    (void)hipMalloc(&out, 2 * N * 8);
    (void)hipMalloc(&tk, 8);
    (void)hipMemcpy(K, hk.data(), hk.size() * 8, hipMemcpyHostToDevice);
    std::vector<double> ref;
    g_grid = argc > 2 ? atoi(argv[2]) : 1;
    printf("grid %d workgroups\n", g_grid);
    run<8, false, 1>("v0 8 waves, 1 chain, IEEE div", K, iters, out, tk, ref);
    run<8, true, 2>("v1 8 waves, 2 chains, rcp div", K, iters, out, tk, ref);
    run<8, false, 2>("v1b 8 waves, 2 chains, IEEE div", K, iters, out, tk, ref);
    run<4, false, 2>("v2 4 waves, 2 chains, IEEE div", K, iters, out, tk, ref);
    run<4, true, 2>("v3 4 waves, 2 chains, rcp div", K, iters, out, tk, ref);
    run<4, true, 4>("v3b 4 waves, 4 chains, rcp div", K, iters, out, tk, ref);
    run<2, true, 4>("v4 2 waves, 4 chains, rcp div", K, iters, out, tk, ref);
    run<1, true, 8>("v5 1 wave, 8 chains, rcp div", K, iters, out, tk, ref);
    return 0;
}
