// otf_gw.hip — Gromov-Wasserstein couplings, one workgroup per
// problem (one per label), the whole outer loop resident on the device.
//
// Two solvers, both for the square loss on symmetric intra-domain costs C1 (n x n),
// C2 (m x m):
//
//  OTF_GW_CG — POT 0.9.6 ot.gromov.gromov_wasserstein(C1, C2, p, q, 'square_loss')
//    as called at MRI_PET_OT_nojax.py:80-82 (epsilon= is swallowed by **kwargs: the
//    solver is the exact conditional-gradient one).  G0 = p q^T; per iteration
//      df  = 2 (constC - hC1 G hC2^T),  constC = (C1^2 p) 1^T + 1 (C2^2 q)^T,
//            hC1 = C1, hC2 = 2 C2
//      Mi  = df + min(df);  Gc = emd(p, q, Mi)
//      line search: dot = hC1 (Gc - G) hC2^T, a = -<dot, dG>, b = -2 <dot, G>,
//                   alpha = argmin over [0, 1] of a t^2 + b t, cost += a alpha^2 + b alpha
//      stop when |dcost| / |cost| < tol_rel or |dcost| < tol_abs, or at max_iter.
//    The callers pass p = q = unif(n) with n = m (paired MRI / PET samples per label,
//    MRI_PET_OT_nojax.py:884-903), where the transportation polytope is the scaled
//    Birkhoff polytope and the exact EMD is a minimum-cost assignment / n.  It is
//    solved here by shortest augmenting paths with dual potentials (Kuhn-Munkres in
//    the Jonker-Volgenant form) on one wavefront, lanes over columns.
//
//  OTF_GW_ENTROPIC — OTT-jax 0.6.0 GromovWasserstein(epsilon, linear_solver=Sinkhorn)
//    as called at MRI_PET_OT_OT_per_epoch_attn.py:161-174 and
//    perturbot/perturbot/match/ott_egwl.py:25-296: linearisation
//      L = x 1^T + 1 y^T - 2 C1 P C2,  x = C1^2 r, y = C2^2 c  (r, c: marginals of P)
//    starting from P = a b^T, lse-mode Sinkhorn on L at epsilon (warm-started from
//    the previous potentials), reg_ot_cost = <a, f> + <b, g> + eps (1 - sum P);
//    outer stop when isclose(cost[i-2], cost[i-1], rtol=threshold) after at least
//    max(3, min_iter) iterations.  Optional labels restrict the coupling to
//    same-label pairs (L = +inf elsewhere): the labelled variant of ott_egwl.py:25-126.
//
//  OTF_GW_PGD — POT 0.9.6 ot.gromov.entropic_gromov_wasserstein(C1, C2, p, q,
//    'square_loss', epsilon, solver='PGD') as called by perturbot/perturbot/match/
//    gw.py:31-59 (egw_pgd) and :80-102 (egw_all): T0 = p q^T, constC from (p, q);
//    per iteration T = sinkhorn_knopp(p, q, 2 (constC - 2 C1 T C2), epsilon) with
//    POT's defaults (1000 updates, stopThr 1e-9); every 10th iteration
//    err = ||T - Tprev||_F; stop when err <= tol or at max_iter; gw_dist =
//    <constC - 2 C1 T C2, T>.
//
// Everything is float64 like the reference.  Matrices live in a caller workspace
// (L2-resident at the reference's sizes, <= 1024 per side), vectors in LDS.  Problems
// up to GW_HUGEN per side (POT has no cap) run the same loop with the vectors and the
// network simplex's tree in the workspace too (GwHuge); CG's linear step is then
// always the network simplex (the one-wave assignment solver keeps its columns in
// registers, <= 1024).
#include <float.h>

#include "otf_device.h"
#include "otf_emd.h"

namespace otf {
namespace {

constexpr int GW_MAXN = 1024;
constexpr int GW_HUGEN = 4096;
constexpr int GW_MAXP = 16;
constexpr double GW_INF = 1e300;
constexpr int GW_SMALLN = 64;  // problems with n, m <= this run with all matrices in LDS

// Kernel variants: SMALL keeps C1, C2, the linearised cost and the plan in LDS
// (the reference's per-label groups are <= 64 samples); the general variant keeps
// them in the (L2-resident) workspace.
template <int NT_, int MAXV_, bool SMALL_> struct GwCfg {
    static constexpr int NT = NT_;
    static constexpr int NW = NT_ / kWave;
    static constexpr int MAXV = MAXV_;
    static constexpr bool SMALL = SMALL_;
    static constexpr bool GLOBAL = MAXV_ > GW_MAXN;  // shared state in the workspace
};
using GwBig = GwCfg<256, GW_MAXN, false>;
using GwHuge = GwCfg<256, GW_HUGEN, false>;
using GwSmall = GwCfg<512, GW_SMALLN, true>;

template <class Cfg> constexpr size_t gw_sh_bytes();
struct GwLaunch {
    otf_gw_problem prob[GW_MAXP];
    double* ws[GW_MAXP];
    unsigned char* shg[GW_MAXP];   // GwHuge: GwShared, then the network simplex's tree
    int first;  // index of prob[0] in the caller's array (info / cost-log rows)
    int nprob;
};

template <int MAXV> struct GwLap {
    double minv[MAXV + 1];
    int pc[MAXV + 1];   // pc[j]: row (1-based) assigned to column j, 0 = free
    int way[MAXV + 1];  // predecessor column on the shortest path
    int sigma[MAXV];    // sigma[i]: column of row i (0-based)
    unsigned char used[MAXV + 1];
};

template <int MAXV> struct GwMarg {
    double r[MAXV];  // row marginal of the current plan
    double c[MAXV];  // column marginal
};

template <int S> struct GwMats {
    double C1[S * S], C2[S * S], L[S * (S + 1)], G[S * S];  // L rows padded: conflict-free column AND row sweeps
};
template <> struct GwMats<0> {};

template <class Cfg> struct GwShared {
    static constexpr int MV = Cfg::MAXV;
    double f[MV + 1];  // OTT: potential f; CG: LAP row duals u (1-based)
    double g[MV + 1];  // OTT: potential g; CG: LAP column duals v (1-based)
    double x[MV];      // marginal-dependent cost, rows:    (C1^2 r)_i
    double y[MV];      // marginal-dependent cost, columns: (C2^2 c)_j
    union {
        GwLap<MV> lap;
        GwMarg<MV> mg;
    };
    double pm[Cfg::NT];  // per-thread partials (max / sum)
    double ps[Cfg::NT];
    double red[32];
    int flag;
    int kflag[2];  // PGD inner Sinkhorn: numerical-error flags by update parity
    GwMats<Cfg::SMALL ? GW_SMALLN : 0> mat;
};

template <class Cfg> constexpr size_t gw_sh_bytes() { return (sizeof(GwShared<Cfg>) + 255) / 256 * 256; }

// Diagnostic build only (-DOTF_GW_STAMPS, tools/stamps_gw.hip): per-phase wall-clock
// totals of workgroup 0..15 (s_memrealtime ticks, 10 ns); compiled out of the library.
#ifdef OTF_GW_STAMPS
__device__ unsigned long long g_gw_stamps[16 * 8];
__device__ unsigned long long g_gw_sk[4];
#define GW_TBEG() unsigned long long gw_t0_ = __builtin_amdgcn_s_memrealtime()
#define GW_TEND(k) gw_acc[k] += __builtin_amdgcn_s_memrealtime() - gw_t0_
#else
#define GW_TBEG() do {} while (0)
#define GW_TEND(k) do {} while (0)
#endif

// --------------------------------------------------------------------- block helpers
__device__ __forceinline__ double blk_sum(double v, double* red) { return block_sum<double>(v, red); }

// Wave reductions of doubles over DPP (row-local exchanges + row broadcasts), result
// read from lane 63 with s_readlane: no LDS round trips (the __shfl forms are
// ds_bpermute, ~6x slower per step, and dominated the per-row LSE updates).
template <int CTRL, int RM, bool ID_ZERO>
__device__ __forceinline__ double dpp_f64(double x, double ident) {
    const int lo = __double2loint(x), hi = __double2hiint(x);
    const int olo = __double2loint(ident), ohi = __double2hiint(ident);
    const int rlo = __builtin_amdgcn_update_dpp(olo, lo, CTRL, RM, 0xf, false);
    const int rhi = __builtin_amdgcn_update_dpp(ohi, hi, CTRL, RM, 0xf, false);
    return __hiloint2double(rhi, rlo);
}
__device__ __forceinline__ double readlane_f64(double x, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(x), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(x), l);
    return __hiloint2double(hi, lo);
}
template <int OP>  // 0 sum, 1 max, 2 min
__device__ __forceinline__ double dpp_op(double a, double b) {
    return OP == 0 ? a + b : (OP == 1 ? fmax(a, b) : fmin(a, b));
}
template <int OP>
__device__ __forceinline__ double wave_reduce_f64(double x) {
    const double id = OP == 0 ? 0.0 : (OP == 1 ? -INFINITY : INFINITY);
    x = dpp_op<OP>(x, dpp_f64<0xB1, 0xf, false>(x, id));   // quad_perm [1,0,3,2]
    x = dpp_op<OP>(x, dpp_f64<0x4E, 0xf, false>(x, id));   // quad_perm [2,3,0,1]
    x = dpp_op<OP>(x, dpp_f64<0x141, 0xf, false>(x, id));  // row_half_mirror
    x = dpp_op<OP>(x, dpp_f64<0x140, 0xf, false>(x, id));  // row_mirror
    x = dpp_op<OP>(x, dpp_f64<0x142, 0xa, false>(x, id));  // row_bcast:15 -> rows 1, 3
    x = dpp_op<OP>(x, dpp_f64<0x143, 0xc, false>(x, id));  // row_bcast:31 -> rows 2, 3
    return readlane_f64(x, 63);
}
__device__ __forceinline__ int wave_min_i32(int x) {
    x = min(x, __builtin_amdgcn_update_dpp(x, x, 0xB1, 0xf, 0xf, false));
    x = min(x, __builtin_amdgcn_update_dpp(x, x, 0x4E, 0xf, 0xf, false));
    x = min(x, __builtin_amdgcn_update_dpp(x, x, 0x141, 0xf, 0xf, false));
    x = min(x, __builtin_amdgcn_update_dpp(x, x, 0x140, 0xf, 0xf, false));
    x = min(x, __builtin_amdgcn_update_dpp(0x7fffffff, x, 0x142, 0xa, 0xf, false));
    x = min(x, __builtin_amdgcn_update_dpp(0x7fffffff, x, 0x143, 0xc, 0xf, false));
    return __builtin_amdgcn_readlane(x, 63);
}

template <class Cfg>
__device__ double blk_minmax(double v, double* red, bool want_max) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double t = wave_xor_n<double>(v, o);
        v = want_max ? fmax(v, t) : fmin(v, t);
    }
    if (lane == 0) red[w] = v;
    __syncthreads();
    double r = red[0];
    for (int i = 1; i < Cfg::NW; ++i) r = want_max ? fmax(r, red[i]) : fmin(r, red[i]);
    __syncthreads();
    return r;
}

// out(i, j) = alpha * sum_k A(i, k) B(k, j) on v_mfma_f64_16x16x4_f64, one 16 x 16
// output tile per wave at a time:  A(i, k) = A[i * sai + k * sak],
// B(k, j) = B[row(k) * sbk + j * sbj] with row(k) = perm ? perm[k] : k,
// out(i, j) -> out[i * soi + j * soj].  Operand lanes: A[i0 + (l & 15)][k0 + (l >> 4)],
// B[k0 + (l >> 4)][j0 + (l & 15)]; result: col l & 15, rows (l >> 4) + 4 r.
// Callers pick strides so that the 16 lanes of a row group read consecutive doubles.
typedef double gw_f64x4 __attribute__((ext_vector_type(4)));
template <class Cfg, bool PERM>
__device__ void blk_gemm(double* out, int64_t soi, int64_t soj, const double* A, int64_t sai,
                         int64_t sak, const double* B, int64_t sbk, int64_t sbj, int n, int m,
                         int k, const int* perm, double alpha) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int tn = (n + 15) >> 4, tm = (m + 15) >> 4;
    const int li = lane & 15, lk = lane >> 4;
    for (int tile = w; tile < tn * tm; tile += Cfg::NW) {
        const int i0 = (tile / tm) * 16, j0 = (tile % tm) * 16;
        const int ia = i0 + li, jb = j0 + li;
        gw_f64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
        for (int k0 = 0; k0 < k; k0 += 4) {
            const int kk = k0 + lk;
            const bool kin = kk < k;
            const double av = (ia < n && kin) ? A[ia * sai + kk * sak] : 0.0;
            const double bv = (jb < m && kin) ? B[(int64_t)(PERM ? perm[kk] : kk) * sbk + jb * sbj] : 0.0;
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = i0 + lk + 4 * r;
            if (i < n && jb < m) out[i * soi + jb * soj] = alpha * acc[r];
        }
    }
}

// v[i] = sum_k C[k][i]^2 w[k]  (C symmetric, so this is (C^2 w)_i; column reads coalesce)
template <class Cfg>
__device__ void blk_sq_matvec(double* v, const double* C, int64_t ldc, int n, const double* w) {
    for (int i = threadIdx.x; i < n; i += Cfg::NT) {
        double s = 0;
#pragma unroll 8
        for (int k = 0; k < n; ++k) {
            const double c = C[(int64_t)k * ldc + i];
            s = fma(c * c, w[k], s);
        }
        v[i] = s;
    }
}

__device__ __forceinline__ double marg(const double* p, int i, int n) {
    return p ? p[i] : 1.0 / (double)n;
}

// Thread-to-(column, row-segment) map for column reductions: CW threads span the
// columns, S = Cfg::NT / CW segments split the rows.
template <class Cfg> struct ColMap {
    int CW, S, seg, jj;
    __device__ ColMap(int m) {
        CW = kWave;
        while (CW < m && CW < Cfg::NT) CW <<= 1;
        S = Cfg::NT / CW;
        seg = threadIdx.x / CW;
        jj = threadIdx.x - seg * CW;
    }
};

// Log-sum-exp updates, two passes over the (LDS- or L2-resident) cost: a max pass and
// a sum-of-exp pass, one exp per element; potentials in absolute units, exponents
// scaled by ieps = 1 / eps.
// One LSE sweep: for every output o < nout,
//     out[o] = eps log w_o - eps LSE_k((pot[k] - L(o, k)) / eps),  L(o, k) = Lm[o*so + k*sk],
// CW threads across the outputs, S segments across k, each thread a strided run of k
// (independent loads and exps); a max pass and a sum pass merged over the segments
// in LDS in a fixed order.  Column update: (o, k) = (j, i); row update: (i, j).
template <class Cfg>
__device__ void lse_sweep(const double* Lm, int64_t so, int64_t sk, int nout, int nk,
                          const double* pot, double* out, const double* w, double eps,
                          double ieps, GwShared<Cfg>& sh) {
    const ColMap<Cfg> cm(nout);
    for (int o0 = 0; o0 < nout; o0 += cm.CW) {
        const int o = o0 + cm.jj;
        const double* lo = Lm + (int64_t)o * so;
        double mx = -INFINITY;
        if (o < nout) {
#pragma unroll 4
            for (int k = cm.seg; k < nk; k += cm.S) mx = fmax(mx, (pot[k] - lo[k * sk]) * ieps);
        }
        sh.pm[threadIdx.x] = mx;
        __syncthreads();
        double s = 0;
        if (o < nout) {
            for (int q = 0; q < cm.S; ++q) mx = fmax(mx, sh.pm[cm.jj + q * cm.CW]);
#pragma unroll 4
            for (int k = cm.seg; k < nk; k += cm.S) s += exp((pot[k] - lo[k * sk]) * ieps - mx);
        }
        sh.ps[threadIdx.x] = s;
        __syncthreads();
        if (cm.seg == 0 && o < nout) {
            s = sh.ps[cm.jj];
            for (int q = 1; q < cm.S; ++q) s += sh.ps[cm.jj + q * cm.CW];
            out[o] = eps * log(marg(w, o, nout)) - eps * (mx + log(s));
        }
        __syncthreads();
    }
}

// L1 error of the column marginal: sum_j |sum_i exp((f_i + g_j - L_ij)/eps) - b_j|
template <class Cfg>
__device__ double lse_col_error(const double* Lm, int64_t ldl, int n, int m, const double* b,
                                double ieps, GwShared<Cfg>& sh) {
    const ColMap<Cfg> cm(m);
    double err = 0;
    for (int j0 = 0; j0 < m; j0 += cm.CW) {
        const int j = j0 + cm.jj;
        double s = 0;
        if (j < m)
            for (int i = cm.seg; i < n; i += cm.S)
                s += exp((sh.f[i] + sh.g[j] - Lm[(int64_t)i * ldl + j]) * ieps);
        sh.ps[threadIdx.x] = s;
        __syncthreads();
        if (cm.seg == 0 && j < m) {
            for (int q = 1; q < cm.S; ++q) s += sh.ps[threadIdx.x + q * cm.CW];
            err += fabs(s - marg(b, j, m));
        }
        __syncthreads();
    }
    return blk_sum(err, sh.red);
}

template <class Cfg>
__device__ bool blk_timed_out(unsigned long long deadline, GwShared<Cfg>& sh) {
    if (threadIdx.x == 0) sh.flag = __builtin_amdgcn_s_memrealtime() > deadline;
    __syncthreads();
    const bool t = sh.flag != 0;
    __syncthreads();
    return t;
}

// OTT lse-mode Sinkhorn on L (n x m) from the potentials in sh.f / sh.g:
// chunks of `inner` (g, f) updates, L1 column error after each chunk.
template <class Cfg>
__device__ int blk_sinkhorn_lse(const double* Lm, int64_t ldl, int n, int m, const double* a,
                                const double* b, double eps, double thr, int inner, int maxit,
                                GwShared<Cfg>& sh, bool& conv, unsigned long long deadline,
                                bool& timeout) {
    const double ieps = 1.0 / eps;
    int it = 0;
    conv = false;
    while (it < maxit && !conv) {
        for (int k = 0; k < inner && it < maxit; ++k, ++it) {
#ifdef OTF_GW_STAMPS
            unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            lse_sweep(Lm, 1, ldl, m, n, sh.f, sh.g, b, eps, ieps, sh);
            unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
            lse_sweep(Lm, ldl, 1, n, m, sh.g, sh.f, a, eps, ieps, sh);
            unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
            if (threadIdx.x == 0 && blockIdx.x == 0) { g_gw_sk[0] += t1 - t0; g_gw_sk[1] += t2 - t1; }
#else
            lse_sweep(Lm, 1, ldl, m, n, sh.f, sh.g, b, eps, ieps, sh);  // g from f
            lse_sweep(Lm, ldl, 1, n, m, sh.g, sh.f, a, eps, ieps, sh);  // f from g
#endif
        }
#ifdef OTF_GW_STAMPS
        unsigned long long t3 = __builtin_amdgcn_s_memrealtime();
#endif
        const double err = lse_col_error(Lm, ldl, n, m, b, ieps, sh);
#ifdef OTF_GW_STAMPS
        if (threadIdx.x == 0 && blockIdx.x == 0) g_gw_sk[2] += __builtin_amdgcn_s_memrealtime() - t3;
#endif
        if (!(err == err)) break;  // diverged
        conv = err < thr;
        if (blk_timed_out(deadline, sh)) { timeout = true; break; }
    }
    return it;
}

// POT sinkhorn_knopp (ot.bregman, POT 0.9.6), the inner solver of POT's entropic GW
// (solver='PGD'), on K = exp(M / -eps) (n x m, row stride ldk, LDS- or L2-resident):
//   u = 1/n, v = 1/m;  per update  v = b / K^T u,  u = 1 / (Kp v),  Kp = K / a (rows);
//   a zero in K^T u or a non-finite u / v keeps the previous (u, v) and stops; every
//   `every` updates err = || sum_i u_i K_ij v_j - b ||_2 < thr stops.
// (u, v) alternate between two LDS slots: slot 0 = (f, g), slot 1 = (mg.r, mg.c).
// Returns the slot holding the result; iters = update passes run (POT's loop count).
template <class Cfg>
__device__ int blk_sinkhorn_knopp(const double* K, int64_t ldk, int n, int m, const double* a,
                                  const double* b, double thr, int maxit, int every,
                                  GwShared<Cfg>& sh, bool& conv, int& iters) {
    const int t = threadIdx.x;
    for (int i = t; i < n; i += Cfg::NT) sh.f[i] = 1.0 / (double)n;
    for (int j = t; j < m; j += Cfg::NT) sh.g[j] = 1.0 / (double)m;
    if (t == 0) { sh.kflag[0] = 0; sh.kflag[1] = 0; }
    __syncthreads();
    const ColMap<Cfg> cc(m), rc(n);
    int cur = 0;
    conv = false;
    iters = maxit;
    for (int ii = 0; ii < maxit; ++ii) {
        const double* u = cur ? sh.mg.r : sh.f;
        double* un = cur ? sh.f : sh.mg.r;
        double* vn = cur ? sh.g : sh.mg.c;
        int* flag = &sh.kflag[ii & 1];
        // v = b / K^T u: threads across columns, segments across rows
        for (int j0 = 0; j0 < m; j0 += cc.CW) {
            const int j = j0 + cc.jj;
            double s = 0;
            if (j < m)
                for (int i = cc.seg; i < n; i += cc.S) s += K[(int64_t)i * ldk + j] * u[i];
            sh.ps[t] = s;
            __syncthreads();
            // the other parity's flag: every reader of it (previous update) is past this barrier
            if (t == 0) sh.kflag[(ii + 1) & 1] = 0;
            if (cc.seg == 0 && j < m) {
                for (int q = 1; q < cc.S; ++q) s += sh.ps[t + q * cc.CW];
                const double vv = marg(b, j, m) / s;
                vn[j] = vv;
                if (s == 0.0 || !finite_val(vv)) *flag = 1;
            }
            __syncthreads();
        }
        // u = 1 / (Kp v): threads across rows, segments across columns
        for (int i0 = 0; i0 < n; i0 += rc.CW) {
            const int i = i0 + rc.jj;
            double s = 0;
            if (i < n) {
                const double ia = 1.0 / marg(a, i, n);
                const double* kr = K + (int64_t)i * ldk;
                for (int j = rc.seg; j < m; j += rc.S) s += (ia * kr[j]) * vn[j];
            }
            sh.ps[t] = s;
            __syncthreads();
            if (rc.seg == 0 && i < n) {
                for (int q = 1; q < rc.S; ++q) s += sh.ps[t + q * rc.CW];
                const double uu = 1.0 / s;
                un[i] = uu;
                if (!finite_val(uu)) *flag = 1;
            }
            __syncthreads();
        }
        if (*flag) { iters = ii + 1; return cur; }  // numerical error: keep the previous pair
        cur ^= 1;
        if (ii % every == 0) {
            const double* uc = cur ? sh.mg.r : sh.f;
            const double* vc = cur ? sh.mg.c : sh.g;
            double e2 = 0;
            for (int j0 = 0; j0 < m; j0 += cc.CW) {
                const int j = j0 + cc.jj;
                double s = 0;
                if (j < m)
                    for (int i = cc.seg; i < n; i += cc.S) s += uc[i] * K[(int64_t)i * ldk + j] * vc[j];
                sh.ps[t] = s;
                __syncthreads();
                if (cc.seg == 0 && j < m) {
                    for (int q = 1; q < cc.S; ++q) s += sh.ps[t + q * cc.CW];
                    const double d = s - marg(b, j, m);
                    e2 += d * d;
                }
                __syncthreads();
            }
            e2 = blk_sum(e2, sh.red);
            if (sqrt(e2) < thr) { conv = true; iters = ii + 1; return cur; }
        }
    }
    return cur;
}

// The same sinkhorn_knopp for n, m <= 64 (the reference's per-label groups) at the
// latency of two workgroup barriers per update and no LDS traffic for K: the PGD outer
// loop runs ~1000 inner updates per outer iteration in one serial chain (562 k updates
// for the 64 x 64, eps = 5e-3 bench problem), so the update latency is the solve time.
// K (a zero-padded 64 x 65 LDS image, entries outside n x m are 0) is read into
// registers once per call, in both orientations the two half-updates need; waves 0..3
// work (one per SIMD), waves 4..7 only meet the barriers:
//   V half, v = b / K^T u:  wave w owns columns 16w .. 16w + 15; lane (q, s) = (l & 15, l >> 4)
//                           holds K[16s + r][16w + q], r < 16, and sums them against
//                           u[16s .. 16s + 15] (LDS, 8 broadcast reads) in four chains,
//                           then xor 16 / 32 (the permlane swaps);
//   U half, u = 1 / (Kp v): wave w owns rows 16w .. 16w + 15, lane (q, s) holds
//                           Kp[16w + q][16s + c] = K / a and sums them against v[16s ..].
// (tools/ubench_sk64.hip: 620 ns per update in this form against 709 for 8 waves x 8
// columns with one chain and three exchanges.)  Every lane of a column (row) group ends
// with the same sum, so every lane has the new v (u) of its column (row) and keeps the
// previous one for POT's revert-on-error rule.  POT's error check after update ii (every
// `every` updates: tmp2 = sum_i u_i K_ij v_j, err = ||tmp2 - b||) reuses the V half of
// update ii + 1 (tmp2_j = (K^T u)_j v_j, the same K^T u), so a check costs one 16-lane sum
// and one LDS word per wave; on convergence the v that half computed is dropped.  u ends
// in sh.f, v in sh.g; conv / iters are uniform.
constexpr int GW_WLD = GW_SMALLN + 1;

template <class Cfg>
__device__ __attribute__((noinline)) void small_sinkhorn_knopp(const double* K, int n, int m, const double* a, const double* b,
                                     double thr, int maxit, int every, GwShared<Cfg>& sh,
                                     bool& conv, int& iters) {
    static_assert(GW_SMALLN == 64, "16 columns / rows per wave");
    if constexpr (Cfg::NW != 8) {  // only the GwSmall kernel calls it (n, m <= 64)
        __builtin_trap();
    } else {
    __shared__ __attribute__((aligned(16))) double s_u[GW_SMALLN];
    __shared__ __attribute__((aligned(16))) double s_v[GW_SMALLN];
    __shared__ double s_e[4];
    __shared__ int s_kf[2];
    const int l = threadIdx.x & (kWave - 1);
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const bool act = w < 4;  // the working waves
    const int q = l & 15, sg = l >> 4;
    const int jc = 16 * (w & 3) + q;  // V half: this lane's column
    const int ir = 16 * (w & 3) + q;  // U half: this lane's row
    const bool cl = act && jc < m, rl = act && ir < n;
    const double bj = cl ? marg(b, jc, m) : 0.0;
    const double ia = rl ? 1.0 / marg(a, ir, n) : 0.0;
    double kv[16], ku[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) kv[r] = act ? K[(16 * sg + r) * GW_WLD + jc] : 0.0;
#pragma unroll
    for (int c = 0; c < 16; ++c) ku[c] = act ? ia * K[ir * GW_WLD + 16 * sg + c] : 0.0;  // Kp = K / a (POT)
    if (threadIdx.x < GW_SMALLN) s_u[threadIdx.x] = (int)threadIdx.x < n ? 1.0 / (double)n : 0.0;
    if (threadIdx.x < 2) s_kf[threadIdx.x] = 0;
    double u = rl ? 1.0 / (double)n : 0.0, v = cl ? 1.0 / (double)m : 0.0;  // last good pair
    __syncthreads();
    conv = false;
    iters = maxit;
    bool check = false;  // POT's error check of the previous update is pending
    int cnt = 0;         // ii % every
    using D2 = __attribute__((ext_vector_type(2))) double;
    // sum of 16 products in four chains of four, then over the 4 lane segments
    auto dot16 = [&](const double (&k)[16], const double* x) -> double {
        const D2* xp = reinterpret_cast<const D2*>(x);
        double c0 = 0, c1 = 0, c2 = 0, c3 = 0;
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const D2 x0 = xp[2 * h], x1 = xp[2 * h + 1];
            c0 = fma(k[4 * h], x0[0], c0);
            c1 = fma(k[4 * h + 1], x0[1], c1);
            c2 = fma(k[4 * h + 2], x1[0], c2);
            c3 = fma(k[4 * h + 3], x1[1], c3);
        }
        double t = (c0 + c1) + (c2 + c3);
        t += wave_xor<double, 16>(t);
        t += wave_xor<double, 32>(t);
        return t;
    };
    for (int ii = 0;; ++ii) {
        if (ii == maxit && !check) break;
        double s = 0, vn = 0;
        if (act) {
            // ---- V half: s = (K^T u)_jc; v = b / s
            s = dot16(kv, &s_u[16 * sg]);
            if (check) {
                // err of the previous update: tmp2_j = (K^T u)_j v_j
                const double d = cl ? s * v - bj : 0.0;
                double e = sg == 0 ? d * d : 0.0;
                e += wave_xor<double, 1>(e);
                e += wave_xor<double, 2>(e);
                e += wave_xor<double, 4>(e);
                e += wave_xor<double, 8>(e);
                if (l == 0) s_e[w] = e;
            }
            vn = cl ? bj / s : 0.0;
            const bool badv = cl && (s == 0.0 || !finite_val(vn));
            if (sg == 0) s_v[jc] = vn;
            if (__ballot(badv) != 0 && l == 0) s_kf[ii & 1] = 1;
        }
        __syncthreads();
        if (check) {
            const double e2 = (s_e[0] + s_e[1]) + (s_e[2] + s_e[3]);
            if (sqrt(e2) < thr) { conv = true; iters = ii; break; }  // the checked update's pair
        }
        if (ii == maxit) break;  // the last update's check only
        // every reader of the other parity's flag (update ii - 1) is past this barrier
        if (threadIdx.x == 0) s_kf[(ii + 1) & 1] = 0;
        double un = 0;
        if (act) {
            // ---- U half: s = (Kp v)_ir; u = 1 / s
            s = dot16(ku, &s_v[16 * sg]);
            un = rl ? 1.0 / s : 0.0;
            const bool badu = rl && !finite_val(un);
            if (sg == 0) s_u[ir] = un;
            if (__ballot(badu) != 0 && l == 0) s_kf[ii & 1] = 1;
        }
        __syncthreads();
        if (s_kf[ii & 1]) { iters = ii + 1; break; }  // numerical error: keep the previous pair
        u = un;
        v = vn;
        check = cnt == 0;  // ii % every == 0, as a counter (no integer division per update)
        cnt = cnt + 1 == every ? 0 : cnt + 1;
    }
    if (act && sg == 0) {
        sh.f[ir] = u;
        sh.g[jc] = v;
    }
    __syncthreads();
    }
}

// Minimum-cost assignment of the n x n matrix A (row stride lda), ONE wavefront:
// shortest augmenting paths with dual potentials (the serial form in the oracle's
// oro_lap), lanes over columns.  Column j (1-based) lives in lane (j-1) % 64, slot
// (j-1) / 64; every per-column quantity -- v, minv, used, the predecessor column
// and the row assigned to the column together with that row's dual u -- stays in
// its owner's registers, so a search step costs one load of the active row, a wave
// arg-min (ties to the lowest column, the serial scan's choice) and register
// updates; values of one column are fetched with a shuffle from its owner.
// Arithmetic and decisions are those of the serial form step by step.  Writes
// sigma (LDS, row -> column, 0-based); returns false on a non-finite cost.
template <int CPL>
__device__ bool wave_lap(const double* A, int64_t lda, int n, int* sigma, double* urow,
                         unsigned char* done) {
    const int lane = threadIdx.x & 63;
    double v[CPL], minv[CPL], ucol[CPL];
    int pc[CPL], way[CPL];
    bool used[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) { v[c] = 0; ucol[c] = 0; pc[c] = 0; way[c] = 0; }
    // j is wave-uniform: pick the slot, then s_readlane from the owner lane
    auto geti = [&](const int (&arr)[CPL], int j) {
        const int sl = (j - 1) >> 6;
        int x = arr[0];
#pragma unroll
        for (int c = 1; c < CPL; ++c) if (sl == c) x = arr[c];
        return __builtin_amdgcn_readlane(x, (j - 1) & 63);
    };
    auto getd = [&](const double (&arr)[CPL], int j) {
        const int sl = (j - 1) >> 6;
        double x = arr[0];
#pragma unroll
        for (int c = 1; c < CPL; ++c) if (sl == c) x = arr[c];
        return readlane_f64(x, (j - 1) & 63);
    };
    // column reduction v_j = min_i a_ij, then a greedy pass in row order: row i takes
    // its cheapest reduced column (lowest on ties) with u_i = that reduced cost when
    // the column is free (the oracle's oro_lap, step for step).  urow / done are
    // written with the same (wave-uniform) value by every lane and read back by each
    // lane itself, so no cross-lane ordering is involved.
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
        const int j = 1 + lane + kWave * c;
        double mn = GW_INF;
        if (j <= n)
            for (int i = 0; i < n; ++i) {
                const double a = A[(int64_t)i * lda + (j - 1)];
                if (a < mn) mn = a;
            }
        v[c] = mn;
    }
    for (int i = 1; i <= n; ++i) {
        const double* arow = A + (int64_t)(i - 1) * lda;
        double mn = GW_INF;
        int jb = 0x7fffffff;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int j = 1 + lane + kWave * c;
            if (j <= n) {
                const double r = arow[j - 1] - v[c];
                if (r < mn) { mn = r; jb = j; }
            }
        }
        const double rmin = wave_reduce_f64<2>(mn);
        jb = wave_min_i32(mn == rmin ? jb : 0x7fffffff);
        if (jb > n || !(rmin < GW_INF)) return false;
        urow[i] = rmin;
        const bool take = geti(pc, jb) == 0;
        done[i] = take ? 1 : 0;
        if (take && lane == ((jb - 1) & 63)) {
            const int sl = (jb - 1) >> 6;
#pragma unroll
            for (int c = 0; c < CPL; ++c)
                if (sl == c) { pc[c] = i; ucol[c] = rmin; }
        }
    }
    for (int i = 1; i <= n; ++i) {
        if (done[i]) continue;
        double ucur = urow[i];  // dual of row i, which sits at the virtual column 0
#pragma unroll
        for (int c = 0; c < CPL; ++c) { minv[c] = GW_INF; used[c] = false; }
        int j0 = 0;
        while (true) {
            int i0;
            double ui0;
            if (j0 == 0) { i0 = i; ui0 = ucur; }
            else { i0 = geti(pc, j0); ui0 = getd(ucol, j0); }
            const double* arow = A + (int64_t)(i0 - 1) * lda;
            double delta = GW_INF;
            int j1 = 0x7fffffff;
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int j = 1 + lane + kWave * c;
                if (j <= n && !used[c]) {
                    const double cur = arow[j - 1] - ui0 - v[c];
                    if (cur < minv[c]) { minv[c] = cur; way[c] = j0; }
                    if (minv[c] < delta) { delta = minv[c]; j1 = j; }
                }
            }
            // wave arg-min, ties to the lowest column
            const double dmin = wave_reduce_f64<2>(delta);
            j1 = wave_min_i32(delta == dmin ? j1 : 0x7fffffff);
            delta = dmin;
            if (j1 > n || !(delta < GW_INF)) return false;
            ucur += delta;
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                if (1 + lane + kWave * c > n) continue;
                if (used[c]) { ucol[c] += delta; v[c] -= delta; }
                else minv[c] -= delta;
            }
            j0 = j1;
            if (geti(pc, j0) == 0) break;
            const int sl = (j0 - 1) >> 6;
            if (lane == ((j0 - 1) & 63)) {
#pragma unroll
                for (int c = 0; c < CPL; ++c) if (sl == c) used[c] = true;
            }
        }
        // augment along the predecessor chain; each row carries its dual along
        while (j0 != 0) {
            const int jp = geti(way, j0);
            int nr;
            double nu;
            if (jp == 0) { nr = i; nu = ucur; }
            else { nr = geti(pc, jp); nu = getd(ucol, jp); }
            const int sl = (j0 - 1) >> 6;
            if (lane == ((j0 - 1) & 63)) {
#pragma unroll
                for (int c = 0; c < CPL; ++c)
                    if (sl == c) { pc[c] = nr; ucol[c] = nu; }
            }
            j0 = jp;
        }
    }
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
        const int j = 1 + lane + kWave * c;
        if (j <= n) sigma[pc[c] - 1] = j - 1;
    }
    return true;
}

// ---------------------------------------------------------------------- the kernel
// SOLV >= 0 compiles ONE solver in (the others' state leaves the register allocation: the
// small PGD instance spilled ~270 SGPRs to VGPR lanes, reloaded in its inner loop);
// SOLV = -1 takes o.solver at run time.
template <class Cfg, int SOLV = -1>
__global__ __launch_bounds__(Cfg::NT) void gw_kernel(GwLaunch Lz, otf_gw_opts o, otf_gw_info* infos,
                                                   double* costlog, int costlog_len,
                                                   unsigned long long timeout_ticks) {
    if constexpr (SOLV >= 0) o.solver = SOLV;
    GwShared<Cfg>* shp;
    if constexpr (Cfg::GLOBAL) {
        shp = reinterpret_cast<GwShared<Cfg>*>(Lz.shg[blockIdx.x]);
    } else {
        __shared__ GwShared<Cfg> sh_lds;
        shp = &sh_lds;
    }
    GwShared<Cfg>& sh = *shp;
    if ((int)blockIdx.x >= Lz.nprob) return;
    const otf_gw_problem P = Lz.prob[blockIdx.x];
    const int pid = Lz.first + blockIdx.x;
    otf_gw_info* info = infos + pid;
    double* clog = costlog ? costlog + (int64_t)pid * costlog_len : nullptr;
    const int n = (int)P.n, m = (int)P.m;
    const int64_t nm = (int64_t)n * m;
    double* D = Lz.ws[blockIdx.x];  // (C1 . G)^T      (m x n, ld n)
    double* R = D + nm;             // C1 . G . C2     (n x m, ld m)
    double* S = R + 2 * nm;         // CG: C1 . Gc . C2
    double* Lm;                     // df / linearised cost (n x m, ld ldl)
    int64_t ldl;
    double* G;                      // the plan
    int64_t ldt, ldc1, ldc2;
    const double* C1;
    const double* C2;
    if constexpr (Cfg::SMALL) {
        for (int e = threadIdx.x; e < n * n; e += Cfg::NT) sh.mat.C1[e] = P.C1[(e / n) * P.ldc1 + e % n];
        for (int e = threadIdx.x; e < m * m; e += Cfg::NT) sh.mat.C2[e] = P.C2[(e / m) * P.ldc2 + e % m];
        C1 = sh.mat.C1;
        C2 = sh.mat.C2;
        ldc1 = n;
        ldc2 = m;
        Lm = sh.mat.L;
        ldl = m + 1;
        G = sh.mat.G;
        ldt = m;
        __syncthreads();
    } else {
        C1 = P.C1;
        C2 = P.C2;
        ldc1 = P.ldc1;
        ldc2 = P.ldc2;
        Lm = R + nm;
        ldl = m;
        G = P.T;
        ldt = P.ldt;
    }
    // the wall-clock bound is per outer iteration (re-armed after each completed one):
    // a long but progressing solve runs to its iteration cap; a stuck inner loop ends
    // in OTF_GW_TIMEOUT
    unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + timeout_ticks;
    const int t = threadIdx.x;
#ifdef OTF_GW_STAMPS
    unsigned long long gw_acc[4] = {0, 0, 0, 0};
    const unsigned long long gw_start = __builtin_amdgcn_s_memrealtime();
#endif

    int status = OTF_GW_MAX_ITER, it = 0, inner_total = 0;
    bool converged = false, inner_conv = false;
    double cost = 0;

    // CG on weighted or unequal groups: the linear step is the network simplex
    // (emd_block, dynamic LDS) instead of the assignment solver
    const bool gen_cg = !Cfg::SMALL && o.solver == OTF_GW_CG && (Cfg::GLOBAL || n != m || P.p || P.q);
    if (gen_cg) {
        if constexpr (!Cfg::SMALL) {
            extern __shared__ __attribute__((aligned(16))) unsigned char gw_dyn[];
            // G0 = p q^T, constC terms from p, q (POT init_matrix)
            for (int i = t; i < n; i += Cfg::NT) sh.mg.r[i] = marg(P.p, i, n);
            for (int j = t; j < m; j += Cfg::NT) sh.mg.c[j] = marg(P.q, j, m);
            __syncthreads();
            for (int64_t e = t; e < nm; e += Cfg::NT) {
                const int i = (int)(e / m), j = (int)(e % m);
                G[i * ldt + j] = sh.mg.r[i] * sh.mg.c[j];
            }
            blk_sq_matvec<Cfg>(sh.x, C1, ldc1, n, sh.mg.r);
            blk_sq_matvec<Cfg>(sh.y, C2, ldc2, m, sh.mg.c);
            __syncthreads();
            blk_gemm<Cfg, false>(D, 1, n, C1, 1, ldc1, G, ldt, 1, n, m, n, nullptr, 1.0);
            __syncthreads();
            blk_gemm<Cfg, false>(R, m, 1, D, 1, n, C2, ldc2, 1, n, m, m, nullptr, 1.0);
            __syncthreads();
            double acc = 0;
            for (int64_t e = t; e < nm; e += Cfg::NT) {
                const int i = (int)(e / m), j = (int)(e % m);
                acc += (sh.x[i] + sh.y[j] - 2.0 * R[e]) * G[i * ldt + j];
            }
            cost = blk_sum(acc, sh.red);
            if (clog && t == 0 && costlog_len > 0) clog[0] = cost;
            while (true) {
                ++it;
                const double old = cost;
                // Mi = df + min(df), df = 2 (constC - 2 R)
                double mn = INFINITY;
                for (int64_t e = t; e < nm; e += Cfg::NT) {
                    const int i = (int)(e / m), j = (int)(e % m);
                    const double df = 2.0 * (sh.x[i] + sh.y[j] - 2.0 * R[e]);
                    Lm[i * ldl + j] = df;
                    mn = fmin(mn, df);
                }
                mn = blk_minmax<Cfg>(mn, sh.red, false);
                bool finite = true;
                for (int64_t e = t; e < nm; e += Cfg::NT) {
                    const int64_t le = (e / m) * ldl + e % m;
                    const double v = Lm[le] + mn;
                    Lm[le] = v;
                    if (!finite_val(v)) finite = false;
                }
                sh.flag = 0;
                __syncthreads();
                if (!finite) sh.flag = 1;
                __syncthreads();
                if (sh.flag) { status = OTF_GW_NUMERICAL; break; }
                // Gc = emd(p, q, Mi) (POT cg: numItermaxEmd = 1e5) into D, row-major n x m
                otf_emd_problem ep;
                ep.a = sh.mg.r;
                ep.b = sh.mg.c;
                ep.M = Lm;
                ep.ldm = ldl;
                ep.T = D;
                ep.ldt = m;
                ep.n = n;
                ep.m = m;
                __syncthreads();
                otf_emd_info ei;
                if constexpr (Cfg::GLOBAL) {
                    __shared__ __attribute__((aligned(16))) unsigned char emd_scr[kEmdScratch];
                    ei = emd_block<Cfg::NT, int>(ep, 100000, Lz.shg[blockIdx.x] + gw_sh_bytes<Cfg>(), emd_scr);
                } else {
                    ei = emd_block<Cfg::NT>(ep, 100000, gw_dyn,
                                            gw_dyn + ((size_t)(n + m + 1) * kEmdNodeBytes + 15) / 16 * 16);
                }
                __syncthreads();
                if (ei.status == OTF_EMD_INFEASIBLE || ei.status == OTF_EMD_UNBOUNDED) {
                    status = OTF_GW_NUMERICAL;
                    break;
                }
                // S = C1 Gc C2 through (C1 Gc)^T in Lm (m x n)
                blk_gemm<Cfg, false>(Lm, 1, n, C1, 1, ldc1, D, m, 1, n, m, n, nullptr, 1.0);
                __syncthreads();
                blk_gemm<Cfg, false>(S, m, 1, Lm, 1, n, C2, ldc2, 1, n, m, m, nullptr, 1.0);
                __syncthreads();
                double ta = 0, tb = 0;
                for (int64_t e = t; e < nm; e += Cfg::NT) {
                    const int i = (int)(e / m), j = (int)(e % m);
                    const double dot = 2.0 * (S[e] - R[e]);
                    const double gv = G[i * ldt + j];
                    const double gcv = D[e];
                    ta += dot * (gcv - gv);
                    tb += dot * gv;
                }
                const double a = -blk_sum(ta, sh.red);
                const double b = -2.0 * blk_sum(tb, sh.red);
                double alpha;
                if (a > 0) alpha = fmin(1.0, fmax(0.0, -b / (2.0 * a)));
                else alpha = (a + b < 0) ? 1.0 : 0.0;
                cost = cost + a * (alpha * alpha) + b * alpha;
                for (int64_t e = t; e < nm; e += Cfg::NT) {
                    const int i = (int)(e / m), j = (int)(e % m);
                    const double gv = G[i * ldt + j];
                    G[i * ldt + j] = gv + alpha * (D[e] - gv);
                }
                __syncthreads();
                if (clog && t == 0 && it < costlog_len) clog[it] = cost;
                blk_gemm<Cfg, false>(D, 1, n, C1, 1, ldc1, G, ldt, 1, n, m, n, nullptr, 1.0);
                __syncthreads();
                blk_gemm<Cfg, false>(R, m, 1, D, 1, n, C2, ldc2, 1, n, m, m, nullptr, 1.0);
                __syncthreads();
                const double absd = fabs(cost - old);
                const double reld = cost != 0.0 ? absd / fabs(cost) : NAN;
                if (reld < o.tol_rel || absd < o.tol_abs) { converged = true; status = OTF_GW_CONVERGED; break; }
                if (it >= o.max_iter) break;
                if (blk_timed_out(deadline, sh)) { status = OTF_GW_TIMEOUT; break; }
                deadline = __builtin_amdgcn_s_memrealtime() + timeout_ticks;
            }
        }
    } else if (o.solver == OTF_GW_CG) {
        // G0 = p q^T (uniform), constC terms from p, q
        const double g0 = 1.0 / ((double)n * (double)m);
        for (int64_t e = t; e < nm; e += Cfg::NT) G[(e / m) * ldt + (e % m)] = g0;
        for (int i = t; i < n; i += Cfg::NT) sh.mg.r[i] = 1.0 / n;
        for (int j = t; j < m; j += Cfg::NT) sh.mg.c[j] = 1.0 / m;
        __syncthreads();
        { GW_TBEG();
        blk_sq_matvec<Cfg>(sh.x, C1, ldc1, n, sh.mg.r);
        blk_sq_matvec<Cfg>(sh.y, C2, ldc2, m, sh.mg.c);
        __syncthreads();
        blk_gemm<Cfg, false>(D, 1, n, C1, 1, ldc1, G, ldt, 1, n, m, n, nullptr, 1.0);
        __syncthreads();
        blk_gemm<Cfg, false>(R, m, 1, D, 1, n, C2, ldc2, 1, n, m, m, nullptr, 1.0);
        __syncthreads();
        GW_TEND(0); }
        // cost(G) = <constC - 2 R, G>
        double acc = 0;
        for (int64_t e = t; e < nm; e += Cfg::NT) {
            const int i = (int)(e / m), j = (int)(e % m);
            acc += (sh.x[i] + sh.y[j] - 2.0 * R[e]) * G[i * ldt + j];
        }
        cost = blk_sum(acc, sh.red);
        if (clog && t == 0 && costlog_len > 0) clog[0] = cost;
        while (true) {
            ++it;
            const double old = cost;
            // df = 2 (constC - 2 R);  Mi = df + min(df)
            double mn = INFINITY;
            for (int64_t e = t; e < nm; e += Cfg::NT) {
                const int i = (int)(e / m), j = (int)(e % m);
                const double df = 2.0 * (sh.x[i] + sh.y[j] - 2.0 * R[e]);
                Lm[i * ldl + j] = df;
                mn = fmin(mn, df);
            }
            mn = blk_minmax<Cfg>(mn, sh.red, false);
            bool finite = true;
            for (int64_t e = t; e < nm; e += Cfg::NT) {
                const int64_t le = (e / m) * ldl + e % m;
                const double v = Lm[le] + mn;
                Lm[le] = v;
                if (!finite_val(v)) finite = false;
            }
            sh.flag = 0;
            __syncthreads();
            if (!finite) sh.flag = 1;
            __syncthreads();
            if (sh.flag) { status = OTF_GW_NUMERICAL; break; }
            __syncthreads();
            // Gc = assignment(Mi) / n
{ GW_TBEG();
            if constexpr (!Cfg::GLOBAL) {  // (GwHuge: the CG step is the network simplex)
                if (t < kWave) {
                    const bool ok = wave_lap<(Cfg::MAXV + kWave - 1) / kWave>(Lm, ldl, n, sh.lap.sigma, sh.f, sh.lap.used);
                    if (t == 0) sh.flag = ok ? 0 : 1;
                }
            }
            __syncthreads();
GW_TEND(1); }
            if (sh.flag) { status = OTF_GW_NUMERICAL; break; }
            // S = C1 Gc C2:  S_ij = (1/n) sum_k C1[i][k] C2[sigma(k)][j]
{ GW_TBEG();
            blk_gemm<Cfg, true>(S, m, 1, C1, 1, ldc1, C2, ldc2, 1, n, m, n, sh.lap.sigma, 1.0 / n);
            __syncthreads();
GW_TEND(0); }
            // dot = 2 (S - R); a = -<dot, Gc - G>; b = -2 <dot, G>
            double ta = 0, tb = 0;
            const double gc = 1.0 / n;
            for (int64_t e = t; e < nm; e += Cfg::NT) {
                const int i = (int)(e / m), j = (int)(e % m);
                const double dot = 2.0 * (S[e] - R[e]);
                const double gv = G[i * ldt + j];
                const double gcv = (sh.lap.sigma[i] == j) ? gc : 0.0;
                ta += dot * (gcv - gv);
                tb += dot * gv;
            }
            const double a = -blk_sum(ta, sh.red);
            const double b = -2.0 * blk_sum(tb, sh.red);
            double alpha;
            if (a > 0) alpha = fmin(1.0, fmax(0.0, -b / (2.0 * a)));
            else alpha = (a + b < 0) ? 1.0 : 0.0;
            cost = cost + a * (alpha * alpha) + b * alpha;
            // G += alpha (Gc - G)
            for (int64_t e = t; e < nm; e += Cfg::NT) {
                const int i = (int)(e / m), j = (int)(e % m);
                const double gv = G[i * ldt + j];
                const double gcv = (sh.lap.sigma[i] == j) ? gc : 0.0;
                G[i * ldt + j] = gv + alpha * (gcv - gv);
            }
            __syncthreads();
            if (clog && t == 0 && it < costlog_len) clog[it] = cost;
            // df(G) for the next iteration (POT recomputes it from G)
            { GW_TBEG();
            blk_gemm<Cfg, false>(D, 1, n, C1, 1, ldc1, G, ldt, 1, n, m, n, nullptr, 1.0);
            __syncthreads();
            blk_gemm<Cfg, false>(R, m, 1, D, 1, n, C2, ldc2, 1, n, m, m, nullptr, 1.0);
            __syncthreads();
            GW_TEND(0); }
            const double absd = fabs(cost - old);
            const double reld = cost != 0.0 ? absd / fabs(cost) : NAN;
            if (reld < o.tol_rel || absd < o.tol_abs) { converged = true; status = OTF_GW_CONVERGED; break; }
            if (it >= o.max_iter) break;
            if (blk_timed_out(deadline, sh)) { status = OTF_GW_TIMEOUT; break; }
            deadline = __builtin_amdgcn_s_memrealtime() + timeout_ticks;
        }
    } else if (o.solver == OTF_GW_PGD) {
        // POT entropic GW, solver='PGD'.  T0 = p q^T; constC from (p, q), fixed.
        const double* pa = P.p;
        const double* pb = P.q;
        for (int64_t e = t; e < nm; e += Cfg::NT) {
            const int i = (int)(e / m), j = (int)(e % m);
            G[i * ldt + j] = marg(pa, i, n) * marg(pb, j, m);
        }
        for (int i = t; i < n; i += Cfg::NT) sh.mg.r[i] = marg(pa, i, n);
        for (int j = t; j < m; j += Cfg::NT) sh.mg.c[j] = marg(pb, j, m);
        __syncthreads();
        blk_sq_matvec<Cfg>(sh.x, C1, ldc1, n, sh.mg.r);
        blk_sq_matvec<Cfg>(sh.y, C2, ldc2, m, sh.mg.c);
        __syncthreads();
        double err = 1.0;
        int nerr = 0;
        const double neps = -o.eps;
        // small problems: K in a zero-padded 64 x 65 LDS image for the wavefront solve
        const bool wave_sk = Cfg::SMALL && n <= kWave && m <= kWave;
        const int64_t kld = wave_sk ? GW_WLD : ldl;
        if (wave_sk) {
            for (int e = t; e < GW_SMALLN * GW_WLD; e += Cfg::NT) Lm[e] = 0.0;
            __syncthreads();
        }
        while (err > o.tol_abs && it < o.max_iter) {
            { GW_TBEG();
            blk_gemm<Cfg, false>(D, 1, n, C1, 1, ldc1, G, ldt, 1, n, m, n, nullptr, 1.0);
            __syncthreads();
            blk_gemm<Cfg, false>(R, m, 1, D, 1, n, C2, ldc2, 1, n, m, m, nullptr, 1.0);
            __syncthreads();
            GW_TEND(0); }
            // K = exp(gwggrad / -eps), gwggrad = 2 (constC - 2 C1 T C2)
            for (int64_t e = t; e < nm; e += Cfg::NT) {
                const int i = (int)(e / m), j = (int)(e % m);
                const double tens = 2.0 * (sh.x[i] + sh.y[j] - 2.0 * R[e]);
                Lm[i * kld + j] = exp(tens / neps);
            }
            __syncthreads();
            int sk_it = 0;
#ifdef OTF_GW_STAMPS
            unsigned long long gw_t0_ = __builtin_amdgcn_s_memrealtime();
#endif
            int slot = 0;
            if (wave_sk) {
                small_sinkhorn_knopp<Cfg>(Lm, n, m, pa, pb, o.sk_threshold, o.sk_max_iter,
                                          o.sk_inner, sh, inner_conv, sk_it);
            } else {
                slot = blk_sinkhorn_knopp<Cfg>(Lm, kld, n, m, pa, pb, o.sk_threshold,
                                               o.sk_max_iter, o.sk_inner, sh, inner_conv, sk_it);
            }
            GW_TEND(2);
            inner_total += sk_it;
            // T = diag(u) K diag(v) (POT: u[:, None] * K * v[None, :]); ||T - Tprev||_F
            const double* uf = slot ? sh.mg.r : sh.f;
            const double* vf = slot ? sh.mg.c : sh.g;
            double d2 = 0;
            for (int64_t e = t; e < nm; e += Cfg::NT) {
                const int i = (int)(e / m), j = (int)(e % m);
                const double tv = uf[i] * Lm[i * kld + j] * vf[j];
                const double d = tv - G[i * ldt + j];
                d2 += d * d;
                G[i * ldt + j] = tv;
            }
            d2 = blk_sum(d2, sh.red);  // (barrier inside: plan visible)
            if (it % 10 == 0) {
                err = sqrt(d2);
                if (clog && t == 0 && nerr < costlog_len) clog[nerr] = err;
                ++nerr;
            }
            ++it;
            if (blk_timed_out(deadline, sh)) { status = OTF_GW_TIMEOUT; break; }
            deadline = __builtin_amdgcn_s_memrealtime() + timeout_ticks;
        }
        converged = err <= o.tol_abs;
        if (status != OTF_GW_TIMEOUT)
            status = converged ? OTF_GW_CONVERGED : (err == err ? OTF_GW_MAX_ITER : OTF_GW_NUMERICAL);
        // log['gw_dist'] = <constC - 2 C1 T C2, T>
        blk_gemm<Cfg, false>(D, 1, n, C1, 1, ldc1, G, ldt, 1, n, m, n, nullptr, 1.0);
        __syncthreads();
        blk_gemm<Cfg, false>(R, m, 1, D, 1, n, C2, ldc2, 1, n, m, m, nullptr, 1.0);
        __syncthreads();
        double acc = 0;
        for (int64_t e = t; e < nm; e += Cfg::NT) {
            const int i = (int)(e / m), j = (int)(e % m);
            acc += (sh.x[i] + sh.y[j] - 2.0 * R[e]) * G[i * ldt + j];
        }
        cost = blk_sum(acc, sh.red);
    } else {
        // Entropic GW (OTT).  P0 = a b^T; f = g = 0.
        const double* pa = P.p;
        const double* pb = P.q;
        for (int64_t e = t; e < nm; e += Cfg::NT) {
            const int i = (int)(e / m), j = (int)(e % m);
            G[i * ldt + j] = marg(pa, i, n) * marg(pb, j, m);
        }
        for (int i = t; i < n; i += Cfg::NT) { sh.mg.r[i] = marg(pa, i, n); sh.f[i] = 0; }
        for (int j = t; j < m; j += Cfg::NT) { sh.mg.c[j] = marg(pb, j, m); sh.g[j] = 0; }
        __syncthreads();
        double cprev = 0, cprev2 = 0;
        bool timeout = false;
        while (true) {
            // linearisation at the current plan
            { GW_TBEG();
            blk_sq_matvec<Cfg>(sh.x, C1, ldc1, n, sh.mg.r);
            blk_sq_matvec<Cfg>(sh.y, C2, ldc2, m, sh.mg.c);
            blk_gemm<Cfg, false>(D, 1, n, C1, 1, ldc1, G, ldt, 1, n, m, n, nullptr, 1.0);
            __syncthreads();
            blk_gemm<Cfg, false>(R, m, 1, D, 1, n, C2, ldc2, 1, n, m, m, nullptr, 1.0);
            __syncthreads();
            GW_TEND(0); }
            for (int64_t e = t; e < nm; e += Cfg::NT) {
                const int i = (int)(e / m), j = (int)(e % m);
                double l = sh.x[i] + sh.y[j] - 2.0 * R[e];
                if (P.labels_a && P.labels_a[i] != P.labels_b[j]) l = INFINITY;
                Lm[i * ldl + j] = l;
            }
            if (!o.warm_start) {
                for (int i = t; i < n; i += Cfg::NT) sh.f[i] = 0;
                for (int j = t; j < m; j += Cfg::NT) sh.g[j] = 0;
            }
            __syncthreads();
#ifdef OTF_GW_STAMPS
            unsigned long long gw_t0_ = __builtin_amdgcn_s_memrealtime();
#endif
            int sk_it = blk_sinkhorn_lse(Lm, ldl, n, m, pa, pb, o.eps, o.sk_threshold, o.sk_inner,
                                         o.sk_max_iter, sh, inner_conv, deadline, timeout);
            GW_TEND(2);
            inner_total += sk_it;
            // plan, its marginals and mass; reg_ot_cost
            double mass = 0;
            for (int64_t e = t; e < nm; e += Cfg::NT) {
                const int i = (int)(e / m), j = (int)(e % m);
                const double pv = exp((sh.f[i] + sh.g[j] - Lm[i * ldl + j]) / o.eps);
                G[i * ldt + j] = pv;
                mass += pv;
            }
            mass = blk_sum(mass, sh.red);  // (barrier inside: plan visible)
            for (int i = t; i < n; i += Cfg::NT) {
                double s = 0;
                for (int j = 0; j < m; ++j) s += G[i * ldt + j];
                sh.mg.r[i] = s;
            }
            for (int j = t; j < m; j += Cfg::NT) {
                double s = 0;
                for (int i = 0; i < n; ++i) s += G[i * ldt + j];
                sh.mg.c[j] = s;
            }
            double fa = 0, sa = 0, sb = 0;
            for (int i = t; i < n; i += Cfg::NT) { fa += marg(pa, i, n) * sh.f[i]; sa += marg(pa, i, n); }
            for (int j = t; j < m; j += Cfg::NT) { fa += marg(pb, j, m) * sh.g[j]; sb += marg(pb, j, m); }
            fa = blk_sum(fa, sh.red);
            sa = blk_sum(sa, sh.red);
            sb = blk_sum(sb, sh.red);
            cost = fa + o.eps * (sa * sb - mass);
            if (clog && t == 0 && it < costlog_len) clog[it] = cost;
            ++it;
            cprev2 = cprev;
            cprev = cost;
            if (timeout) { status = OTF_GW_TIMEOUT; break; }
            if (!(cost == cost)) { status = OTF_GW_NUMERICAL; break; }
            // isclose(costs[i-2], costs[i-1], rtol=threshold), atol 1e-8 (jnp default)
            const bool close = it >= 2 && fabs(cprev2 - cprev) <= 1e-8 + o.threshold * fabs(cprev);
            if (it >= o.max_iter) { converged = close; if (close) status = OTF_GW_CONVERGED; break; }
            const bool keep = it < o.min_iter || it <= 2 || (isfinite(cprev) && !close);
            if (!keep) { converged = close; status = close ? OTF_GW_CONVERGED : OTF_GW_NUMERICAL; break; }
            if (blk_timed_out(deadline, sh)) { status = OTF_GW_TIMEOUT; break; }
            deadline = __builtin_amdgcn_s_memrealtime() + timeout_ticks;
        }
    }
    if constexpr (Cfg::SMALL) {
        __syncthreads();
        for (int e = t; e < (int)nm; e += Cfg::NT) P.T[(e / m) * P.ldt + e % m] = G[e];
    }
#ifdef OTF_GW_STAMPS
    gw_acc[3] = __builtin_amdgcn_s_memrealtime() - gw_start;
    if (t == 0 && blockIdx.x < 16)
        for (int k = 0; k < 4; ++k) g_gw_stamps[blockIdx.x * 8 + k] = gw_acc[k];
#endif
    if (t == 0) {
        info->n_iter = it;
        info->converged = converged ? 1 : 0;
        info->inner_converged = inner_conv ? 1 : 0;
        info->status = status;
        info->inner_iters = inner_total;
        info->pad = 0;
        info->cost = cost;
    }
}

// ------------------------------------------------------------- float64 pairwise cost
__global__ void sqnorm_f64_kernel(const float* X, int64_t ldx, int n, int d, double* out) {
    const int i = blockIdx.x * (blockDim.x / kWave) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (i >= n) return;
    double s = 0;
    for (int k = lane; k < d; k += kWave) {
        const double v = (double)X[(int64_t)i * ldx + k];
        s = fma(v, v, s);
    }
    s = wave_sum(s);
    if (lane == 0) out[i] = s;
}

// C[i][j] = -2 x_i . y_j + |x_i|^2 + |y_j|^2 for small outputs with long rows (the
// per-label GW costs: 64 x 64 samples of d = 2048): one wave per output, the float32
// rows read as 16-B vectors, the products summed in float64 over the wave (a fixed
// order), then the gemm epilogue's order (-2 acc, + row term, + column term).  The
// 64 x 64 gemm tile put the whole 64 x 64 x 2048 contraction on ONE workgroup
// (~290 us per cost, 4 per config-3 epoch call); this spreads it over n m waves.
__global__ __launch_bounds__(512) void dot_cost_f64_kernel(const float* X, int64_t ldx, const float* Y,
                                                           int64_t ldy, int n, int m, int d, int vec,
                                                           const double* nx, const double* ny, double* C,
                                                           int64_t ldc) {
    const int64_t o = (int64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (o >= (int64_t)n * m) return;
    const int i = (int)(o / m), j = (int)(o % m);
    const float* x = X + (int64_t)i * ldx;
    const float* y = Y + (int64_t)j * ldy;
    double s = 0;
    int k0 = 0;
    if (vec) {
        using F4 = __attribute__((ext_vector_type(4))) float;
        for (; k0 + 4 * kWave <= d; k0 += 4 * kWave) {
            const F4 a = *reinterpret_cast<const F4*>(x + k0 + 4 * lane);
            const F4 b = *reinterpret_cast<const F4*>(y + k0 + 4 * lane);
#pragma unroll
            for (int q = 0; q < 4; ++q) s = fma((double)a[q], (double)b[q], s);
        }
    }
    for (int k = k0 + lane; k < d; k += kWave) s = fma((double)x[k], (double)y[k], s);
    s = wave_sum(s);
    if (lane == 0) {
        double v = -2.0 * s;
        v += nx[i];
        v += ny[j];
        C[(int64_t)i * ldc + j] = v;
    }
}

// Larger outputs (the float64 metric leg: 4096 x 4096 x 512): 128 x 128 tiles of C per
// 256-thread workgroup on v_mfma_f64_16x16x4_f64 (one MFMA replaces 16 vector FMAs and
// their operand reads): 4 waves, each a 64 x 64 quarter as 4 x 4 blocks of 16 x 16; the
// float32 rows widened to float64 on the way into LDS (k-major, 16 deep, double-buffered
// through registers); per 4-deep k-step a lane reads one double of each of its 4 row
// blocks and 4 column blocks from the LDS stage (16 consecutive doubles per lane group:
// conflict-free).  The epilogue of dist_finalize_kernel is fused: v = -2 acc + |x|^2 +
// |y|^2 (POT euclidean_distances order), clamp >= 0, sqrt (euclidean), zero diagonal,
// stored once; the tile's max goes to part[tile].  Result lanes: column l & 15, rows
// (l >> 4) + 4 r.  (The generic 64 x 64 GEMM + a finalize pass over C took ~0.7 ms at the
// metric shape, the VALU form of this tile 0.45 ms -- removed in r05 -- this one 0.32 ms.)
constexpr int DT = 128, DK = 16;
__global__ __launch_bounds__(256, 2) void dist_mfma_f64_kernel(const float* __restrict__ X, int64_t ldx,
                                                               const float* __restrict__ Y, int64_t ldy,
                                                               int n, int m, int d, const double* nx,
                                                               const double* ny, int euclid, int zero_diag,
                                                               double* C, int64_t ldc, double* part, int tiles_m,
                                                               int vec) {
    __shared__ __attribute__((aligned(16))) double As[2][DK][DT];
    __shared__ __attribute__((aligned(16))) double Bs[2][DK][DT];
    __shared__ double red[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w >> 1, wn = w & 1, li = lane & 15, lk = lane >> 4;
    const int tile = blockIdx.x;
    const int i0 = (tile % tiles_m) * DT, j0 = (tile / tiles_m) * DT;
    const int lr = tid >> 1, lkk = (tid & 1) * 8;
    const int gi = i0 + lr < n ? i0 + lr : n - 1, gj = j0 + lr < m ? j0 + lr : m - 1;
    const float* xr = X + (int64_t)gi * ldx;
    const float* yr = Y + (int64_t)gj * ldy;
    float xa[8], yb[8];
    auto gload = [&](int k0) {
        const int kb = k0 + lkk;
        if (vec && kb + 8 <= d) {
            using F4 = __attribute__((ext_vector_type(4))) float;
            const F4 x0 = *reinterpret_cast<const F4*>(xr + kb), x1 = *reinterpret_cast<const F4*>(xr + kb + 4);
            const F4 y0 = *reinterpret_cast<const F4*>(yr + kb), y1 = *reinterpret_cast<const F4*>(yr + kb + 4);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                xa[q] = x0[q];
                xa[q + 4] = x1[q];
                yb[q] = y0[q];
                yb[q + 4] = y1[q];
            }
        } else {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int k = kb + q;
                xa[q] = k < d ? xr[k] : 0.f;
                yb[q] = k < d ? yr[k] : 0.f;
            }
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            As[buf][lkk + q][lr] = (double)xa[q];
            Bs[buf][lkk + q][lr] = (double)yb[q];
        }
    };
    gw_f64x4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = gw_f64x4{0.0, 0.0, 0.0, 0.0};
    const int nk = (d + DK - 1) / DK;
    gload(0);
    lstore(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) gload((kt + 1) * DK);
#pragma unroll
        for (int ks = 0; ks < DK / 4; ++ks) {
            const int k = 4 * ks + lk;
            double av[4], bv[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                av[t] = As[buf][k][wm * 64 + t * 16 + li];
                bv[t] = Bs[buf][k][wn * 64 + t * 16 + li];
            }
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[b], acc[a][b], 0, 0, 0);
        }
        if (kt + 1 < nk) lstore(buf ^ 1);
        __syncthreads();
    }
    double mx = 0.0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int j = j0 + wn * 64 + b * 16 + li;
        const bool jok = j < m;
        const double ry = jok ? ny[j] : 0.0;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = i0 + wm * 64 + a * 16 + lk + 4 * r;
                if (i >= n || !jok) continue;
                double v = -2.0 * acc[a][b][r];
                v += nx[i];
                v += ry;
                v = v > 0 ? v : 0.0;
                if (euclid) v = sqrt(v);
                if (zero_diag && i == j) v = 0.0;
                C[(int64_t)i * ldc + j] = v;
                mx = fmax(mx, v);
            }
    }
    mx = wave_max(mx);
    if (lane == 0) red[w] = mx;
    __syncthreads();
    if (tid == 0) part[tile] = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
}

// clamp >= 0, sqrt (euclidean), zero diagonal; per-block max to part[blockIdx.x]
__global__ __launch_bounds__(256) void dist_finalize_kernel(double* C, int64_t ldc, int n, int m,
                                                            int euclid, int zero_diag, double* part) {
    __shared__ double red[8];
    double mx = 0;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < (int64_t)n * m;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int i = (int)(e / m), j = (int)(e % m);
        double v = C[(int64_t)i * ldc + j];
        v = v > 0 ? v : 0.0;
        if (euclid) v = sqrt(v);
        if (zero_diag && i == j) v = 0.0;
        C[(int64_t)i * ldc + j] = v;
        mx = fmax(mx, v);
    }
    mx = wave_max(mx);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        double r = red[0];
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) r = fmax(r, red[w]);
        part[blockIdx.x] = r;
    }
}

// max over the partials -> *cmax; optionally C /= max (POT's "C /= C.max()")
__global__ __launch_bounds__(256) void dist_scale_kernel(double* C, int64_t ldc, int n, int m,
                                                         const double* part, int nparts,
                                                         int scale, double* cmax) {
    __shared__ double red[8];
    double mx = 0;
    for (int q = threadIdx.x; q < nparts; q += blockDim.x) mx = fmax(mx, part[q]);
    mx = wave_max(mx);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    double r = red[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) r = fmax(r, red[w]);
    if (cmax && blockIdx.x == 0 && threadIdx.x == 0) *cmax = r;
    if (!scale) return;
    // rows strided over the grid, columns over the block (no 64-bit division per element)
    for (int i = blockIdx.x; i < n; i += gridDim.x) {
        double* row = C + (int64_t)i * ldc;
        for (int j = threadIdx.x; j < m; j += blockDim.x) row[j] = row[j] / r;
    }
}

constexpr int DIST_PARTS = 512;

size_t align256(size_t x) { return (x + 255) / 256 * 256; }

}  // namespace

// Generic tiled GEMM from otf_linalg.hip (same template, instantiated there too).
template <typename TA, typename TB, typename TACC, typename TOUT>
int launch_gemm(const TA* A, int64_t sa0, int64_t sa1, const TB* B, int64_t sb0, int64_t sb1,
                TOUT* out, int64_t ldo, int M, int N, int K, TACC alpha, TACC beta,
                const TACC* rowadd, const TACC* coladd, hipStream_t s);

}  // namespace otf

extern "C" {

size_t otf_cost_pairwise_f64_workspace_size(int64_t n, int64_t m) {
    // per-block maxima: the finalize pass's <= DIST_PARTS blocks or one per 128 x 128 tile
    const int64_t tiles = ((n + otf::DT - 1) / otf::DT) * ((m + otf::DT - 1) / otf::DT);
    const int64_t parts = tiles > otf::DIST_PARTS ? tiles : otf::DIST_PARTS;
    return otf::align256(8 * (size_t)n) + otf::align256(8 * (size_t)m) + otf::align256(8 * (size_t)parts);
}

int otf_cost_pairwise_f64(const float* X, int64_t ldx, const float* Y, int64_t ldy, int64_t n,
                          int64_t m, int64_t d, int32_t metric, int32_t zero_diag,
                          int32_t scale_max, double* C, int64_t ldc, double* cmax,
                          void* workspace, size_t ws_bytes, otf_stream_t stream) {
    if (!X || !Y || !C || !workspace || n <= 0 || m <= 0 || d <= 0) return OTF_EINVAL;
    if (ldx < d || ldy < d || ldc < m) return OTF_EINVAL;
    if (metric != OTF_SQEUCLIDEAN && metric != OTF_EUCLIDEAN) return OTF_EINVAL;
    if (ws_bytes < otf_cost_pairwise_f64_workspace_size(n, m)) return OTF_EINVAL;
    if (n > 65535LL * 64 || m > 2147483647LL / 2) return OTF_EUNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    char* p = (char*)workspace;
    double* nx = (double*)p; p += otf::align256(8 * (size_t)n);
    double* ny = (double*)p; p += otf::align256(8 * (size_t)m);
    double* part = (double*)p;
    otf::sqnorm_f64_kernel<<<(unsigned)((n + 3) / 4), 256, 0, s>>>(X, ldx, (int)n, (int)d, nx);
    otf::sqnorm_f64_kernel<<<(unsigned)((m + 3) / 4), 256, 0, s>>>(Y, ldy, (int)m, (int)d, ny);
    OTF_HIP(hipGetLastError());
    // C = -2 X Y^T + |x|^2 + |y|^2   (POT euclidean_distances order); outputs too few to
    // fill the chip with 64 x 64 gemm tiles: one wave per output
    if (n * m <= 16384) {
        const int vec = (ldx % 4 == 0) && (ldy % 4 == 0) && ((uintptr_t)X % 16 == 0) && ((uintptr_t)Y % 16 == 0);
        otf::dot_cost_f64_kernel<<<(unsigned)((n * m + 7) / 8), 512, 0, s>>>(X, ldx, Y, ldy, (int)n, (int)m,
                                                                             (int)d, vec, nx, ny, C, ldc);
        OTF_HIP(hipGetLastError());
    } else {
        // 128 x 128 float64 tiles with the finalize epilogue fused (dist_mfma_f64_kernel)
        const int tiles_m = (int)((n + otf::DT - 1) / otf::DT), tiles_n = (int)((m + otf::DT - 1) / otf::DT);
        const int ntiles = tiles_m * tiles_n;
        const int vec = (ldx % 4 == 0) && (ldy % 4 == 0) && ((uintptr_t)X % 16 == 0) && ((uintptr_t)Y % 16 == 0);
        otf::dist_mfma_f64_kernel<<<ntiles, 256, 0, s>>>(X, ldx, Y, ldy, (int)n, (int)m, (int)d, nx, ny,
                                                         metric == OTF_EUCLIDEAN, zero_diag, C, ldc, part,
                                                         tiles_m, vec);
        OTF_HIP(hipGetLastError());
        const int64_t tot = n * m;
        int grid = (int)((tot + 255) / 256);
        if (grid > otf::DIST_PARTS) grid = otf::DIST_PARTS;
        otf::dist_scale_kernel<<<grid, 256, 0, s>>>(C, ldc, (int)n, (int)m, part, ntiles, scale_max, cmax);
        OTF_HIP(hipGetLastError());
        return OTF_OK;
    }
    const int64_t tot = n * m;
    int grid = (int)((tot + 255) / 256);
    if (grid > otf::DIST_PARTS) grid = otf::DIST_PARTS;
    otf::dist_finalize_kernel<<<grid, 256, 0, s>>>(C, ldc, (int)n, (int)m,
                                                   metric == OTF_EUCLIDEAN, zero_diag, part);
    otf::dist_scale_kernel<<<grid, 256, 0, s>>>(C, ldc, (int)n, (int)m, part, grid, scale_max, cmax);
    OTF_HIP(hipGetLastError());
    return OTF_OK;
}

namespace otf {
namespace {
bool gw_huge(const otf_gw_problem& P) { return P.n > GW_MAXN || P.m > GW_MAXN; }
// per problem: 4 n x m matrices, and for GwHuge its shared state + the simplex tree
size_t gw_prob_bytes(const otf_gw_problem& P) {
    size_t b = align256(4 * 8 * (size_t)P.n * (size_t)P.m);
    if (gw_huge(P)) b += gw_sh_bytes<GwHuge>() + emd_tree_bytes_g((int64_t)P.n + P.m + 1);
    return b;
}
}  // namespace
}  // namespace otf

size_t otf_gw_workspace_size(int32_t nprob, const otf_gw_problem* probs) {
    if (nprob <= 0 || !probs) return 0;
    size_t tot = 0;
    for (int b = 0; b < nprob; ++b) tot += otf::gw_prob_bytes(probs[b]);
    return tot;
}

static int gw_launch(const otf::GwLaunch& L, const otf_gw_opts& o, otf_gw_info* info, double* costlog,
                     int32_t costlog_len, unsigned long long ticks, bool huge, hipStream_t s) {
    using namespace otf;
    if (huge) {
        gw_kernel<GwHuge><<<L.nprob, GwHuge::NT, 0, s>>>(L, o, info, costlog, costlog_len, ticks);
        OTF_HIP(hipGetLastError());
        return OTF_OK;
    }
    {
        bool small = true;
        size_t dyn = 0;  // CG on weighted / unequal groups: the network simplex's LDS
        for (int b = 0; b < L.nprob; ++b) {
            const otf_gw_problem& P = L.prob[b];
            if (P.n > GW_SMALLN || P.m > GW_SMALLN) small = false;
            if (o.solver == OTF_GW_CG && (P.n != P.m || P.p || P.q)) {
                small = false;
                const size_t e = emd_lds_bytes((int)(P.n + P.m + 1));
                dyn = e > dyn ? e : dyn;
            }
        }
        if (small) {
            if (o.solver == OTF_GW_PGD)
                gw_kernel<GwSmall, OTF_GW_PGD><<<L.nprob, GwSmall::NT, 0, s>>>(L, o, info, costlog, costlog_len, ticks);
            else
                gw_kernel<GwSmall><<<L.nprob, GwSmall::NT, 0, s>>>(L, o, info, costlog, costlog_len, ticks);
        } else {
            if (dyn)
                OTF_HIP(hipFuncSetAttribute((const void*)gw_kernel<GwBig>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn));
            gw_kernel<GwBig><<<L.nprob, GwBig::NT, dyn, s>>>(L, o, info, costlog, costlog_len, ticks);
        }
        OTF_HIP(hipGetLastError());
    }
    return OTF_OK;
}

int otf_gw_solve(int32_t nprob, const otf_gw_problem* probs, const otf_gw_opts* opts,
                 otf_gw_info* info, double* costlog, int32_t costlog_len, void* workspace,
                 size_t ws_bytes, otf_stream_t stream) {
    using namespace otf;
    if (nprob <= 0 || !probs || !opts || !info || !workspace) return OTF_EINVAL;
    const otf_gw_opts o = *opts;
    if (o.solver != OTF_GW_CG && o.solver != OTF_GW_ENTROPIC && o.solver != OTF_GW_PGD)
        return OTF_EINVAL;
    if (o.max_iter < 1) return OTF_EINVAL;
    if (o.solver != OTF_GW_CG && (!(o.eps > 0) || o.sk_inner < 1 || o.sk_max_iter < 1))
        return OTF_EINVAL;
    if (costlog && costlog_len < 1) return OTF_EINVAL;
    if (ws_bytes < otf_gw_workspace_size(nprob, probs)) return OTF_EINVAL;
    for (int b = 0; b < nprob; ++b) {
        const otf_gw_problem& P = probs[b];
        if (!P.C1 || !P.C2 || !P.T || P.n < 1 || P.m < 1) return OTF_EINVAL;
        if (P.ldc1 < P.n || P.ldc2 < P.m || P.ldt < P.m) return OTF_EINVAL;
        if (P.n > GW_HUGEN || P.m > GW_HUGEN) return OTF_EUNSUPPORTED;
        if ((P.labels_a == nullptr) != (P.labels_b == nullptr)) return OTF_EINVAL;
        if (o.solver == OTF_GW_CG && P.labels_a) return OTF_EUNSUPPORTED;
        if (o.solver == OTF_GW_PGD && P.labels_a) return OTF_EUNSUPPORTED;
    }
    hipStream_t s = (hipStream_t)stream;
    char* wsp = (char*)workspace;
    // 20 s at 100 MHz per outer iteration, scaled up with the problem past 1024^2 pairs
    // (GwHuge: one workgroup's GEMMs and simplex grow with n m (n + m))
    unsigned long long ticks = 100000000ull * 20;
    for (int b = 0; b < nprob; ++b) {
        const double sc = (double)probs[b].n * probs[b].m * (probs[b].n + probs[b].m) / (2.0 * 1024.0 * 1024.0 * 1024.0);
        if (sc > 1.0 && 100000000ull * 20 * sc > (double)ticks) ticks = (unsigned long long)(100000000.0 * 20 * sc);
    }
    // one launch per kernel variant (GwHuge problems separately)
    for (int huge = 0; huge < 2; ++huge)
    for (int first = 0; first < nprob; first += GW_MAXP) {
        GwLaunch L{};
        L.first = first;
        L.nprob = 0;
        char* w = wsp;
        for (int b = 0; b < first; ++b) w += gw_prob_bytes(probs[b]);
        const int last = nprob - first < GW_MAXP ? nprob - first : GW_MAXP;
        // problems of this variant in [first, first + last): launched as one batch whose
        // info / log rows are addressed through L.first + slot, so keep the slots dense
        int idx[GW_MAXP];
        for (int b = 0; b < last; ++b) {
            const otf_gw_problem& P = probs[first + b];
            char* mine = w;
            w += gw_prob_bytes(P);
            if ((int)gw_huge(P) != huge) continue;
            idx[L.nprob] = first + b;
            L.prob[L.nprob] = P;
            L.ws[L.nprob] = (double*)mine;
            L.shg[L.nprob] = (unsigned char*)mine + align256(4 * 8 * (size_t)P.n * (size_t)P.m);
            ++L.nprob;
        }
        if (L.nprob == 0) continue;
        bool dense = true;  // info / cost-log rows are first + slot: contiguous problems only
        for (int b = 0; b < L.nprob; ++b) dense = dense && idx[b] == idx[0] + b;
        if (!dense) {  // mixed batch: one launch per problem
            for (int b = 0; b < L.nprob; ++b) {
                GwLaunch L1{};
                L1.first = idx[b];
                L1.nprob = 1;
                L1.prob[0] = L.prob[b];
                L1.ws[0] = L.ws[b];
                L1.shg[0] = L.shg[b];
                const int rc = gw_launch(L1, o, info, costlog, costlog_len, ticks, huge != 0, s);
                if (rc != OTF_OK) return rc;
            }
            continue;
        }
        L.first = idx[0];
        const int rc = gw_launch(L, o, info, costlog, costlog_len, ticks, huge != 0, s);
        if (rc != OTF_OK) return rc;
    }
    return OTF_OK;
}

}  // extern "C"
