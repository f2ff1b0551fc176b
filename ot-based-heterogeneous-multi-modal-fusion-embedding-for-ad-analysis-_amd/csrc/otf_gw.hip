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
// Everything is float64 like the reference.  Matrices live in a caller workspace
// (L2-resident at the reference's sizes, <= 1024 per side), vectors in LDS.
#include <float.h>

#include "otf_device.h"

namespace otf {
namespace {

constexpr int GW_NT = 256;
constexpr int GW_NW = GW_NT / kWave;
constexpr int GW_MAXN = 1024;
constexpr int GW_MAXP = 16;
constexpr double GW_INF = 1e300;

struct GwLaunch {
    otf_gw_problem prob[GW_MAXP];
    double* ws[GW_MAXP];
    int first;  // index of prob[0] in the caller's array (info / cost-log rows)
    int nprob;
};

struct GwLap {
    double minv[GW_MAXN + 1];
    int pc[GW_MAXN + 1];   // pc[j]: row (1-based) assigned to column j, 0 = free
    int way[GW_MAXN + 1];  // predecessor column on the shortest path
    int sigma[GW_MAXN];    // sigma[i]: column of row i (0-based)
    unsigned char used[GW_MAXN + 1];
};

struct GwMarg {
    double r[GW_MAXN];  // row marginal of the current plan
    double c[GW_MAXN];  // column marginal
};

struct GwShared {
    double f[GW_MAXN + 1];  // OTT: potential f; CG: LAP row duals u (1-based)
    double g[GW_MAXN + 1];  // OTT: potential g; CG: LAP column duals v (1-based)
    double x[GW_MAXN];      // marginal-dependent cost, rows:    (C1^2 r)_i
    double y[GW_MAXN];      // marginal-dependent cost, columns: (C2^2 c)_j
    union {
        GwLap lap;
        GwMarg mg;
    };
    double pm[GW_NT];  // per-thread partials (max / sum)
    double ps[GW_NT];
    double red[32];
    int flag;
};

// --------------------------------------------------------------------- block helpers
__device__ __forceinline__ double blk_sum(double v, double* red) { return block_sum<double>(v, red); }

__device__ double blk_minmax(double v, double* red, bool want_max) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double t = __shfl_xor(v, o, kWave);
        v = want_max ? fmax(v, t) : fmin(v, t);
    }
    if (lane == 0) red[w] = v;
    __syncthreads();
    double r = red[0];
    for (int i = 1; i < GW_NW; ++i) r = want_max ? fmax(r, red[i]) : fmin(r, red[i]);
    __syncthreads();
    return r;
}

// out (n x m, ld ldo) = alpha * A (n x k, lda) . B~, B~(kk, j) = B[row(kk) * ldb + j],
// row(kk) = perm ? perm[kk] : kk.  Each thread owns 4 consecutive columns of a row.
template <bool PERM>
__device__ void blk_gemm(double* out, int64_t ldo, const double* A, int64_t lda, const double* B,
                         int64_t ldb, int n, int m, int k, const int* perm, double alpha) {
    const int mq = (m + 3) >> 2;
    for (int o = threadIdx.x; o < n * mq; o += GW_NT) {
        const int i = o / mq, j = (o - i * mq) * 4;
        const double* a = A + (int64_t)i * lda;
        double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
        if (j + 3 < m) {
            for (int kk = 0; kk < k; ++kk) {
                const double av = a[kk];
                const double* b = B + (int64_t)(PERM ? perm[kk] : kk) * ldb + j;
                s0 = fma(av, b[0], s0);
                s1 = fma(av, b[1], s1);
                s2 = fma(av, b[2], s2);
                s3 = fma(av, b[3], s3);
            }
        } else {
            for (int kk = 0; kk < k; ++kk) {
                const double av = a[kk];
                const double* b = B + (int64_t)(PERM ? perm[kk] : kk) * ldb + j;
                s0 = fma(av, b[0], s0);
                if (j + 1 < m) s1 = fma(av, b[1], s1);
                if (j + 2 < m) s2 = fma(av, b[2], s2);
            }
        }
        double* d = out + (int64_t)i * ldo + j;
        d[0] = alpha * s0;
        if (j + 1 < m) d[1] = alpha * s1;
        if (j + 2 < m) d[2] = alpha * s2;
        if (j + 3 < m) d[3] = alpha * s3;
    }
}

// v[i] = sum_k C[k][i]^2 w[k]  (C symmetric, so this is (C^2 w)_i; column reads coalesce)
__device__ void blk_sq_matvec(double* v, const double* C, int64_t ldc, int n, const double* w) {
    for (int i = threadIdx.x; i < n; i += GW_NT) {
        double s = 0;
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
// columns, S = GW_NT / CW segments split the rows.
struct ColMap {
    int CW, S, seg, jj;
    __device__ ColMap(int m) {
        CW = m <= 64 ? 64 : (m <= 128 ? 128 : GW_NT);
        S = GW_NT / CW;
        seg = threadIdx.x / CW;
        jj = threadIdx.x - seg * CW;
    }
};

// Online log-sum-exp accumulator (running max, rescaled sum).
__device__ __forceinline__ void lse_add(double z, double& mx, double& s) {
    if (z > mx) {
        s = (mx == -INFINITY) ? 0.0 : s * exp(mx - z);
        mx = z;
    }
    if (z != -INFINITY) s += exp(z - mx);
}
__device__ __forceinline__ void lse_merge(double& mx, double& s, double m2, double s2) {
    if (m2 == -INFINITY) return;
    if (mx == -INFINITY) { mx = m2; s = s2; return; }
    if (m2 > mx) { s = s * exp(mx - m2) + s2; mx = m2; }
    else s += s2 * exp(m2 - mx);
}

// g_j = eps log b_j - eps LSE_i((f_i - L_ij) / eps)
__device__ void lse_col_update(const double* Lm, int64_t ldl, int n, int m, const double* b,
                               double eps, GwShared& sh) {
    const ColMap cm(m);
    for (int j0 = 0; j0 < m; j0 += cm.CW) {
        const int j = j0 + cm.jj;
        double mx = -INFINITY, s = 0;
        if (j < m)
            for (int i = cm.seg; i < n; i += cm.S) lse_add((sh.f[i] - Lm[(int64_t)i * ldl + j]) / eps, mx, s);
        sh.pm[threadIdx.x] = mx;
        sh.ps[threadIdx.x] = s;
        __syncthreads();
        if (cm.seg == 0 && j < m) {
            for (int q = 1; q < cm.S; ++q) lse_merge(mx, s, sh.pm[threadIdx.x + q * cm.CW], sh.ps[threadIdx.x + q * cm.CW]);
            const double lse = mx + log(s);
            sh.g[j] = eps * log(marg(b, j, m)) - eps * lse;
        }
        __syncthreads();
    }
}

// f_i = eps log a_i - eps LSE_j((g_j - L_ij) / eps): one wave per row, lanes over j.
__device__ void lse_row_update(const double* Lm, int64_t ldl, int n, int m, const double* a,
                               double eps, GwShared& sh) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = w; i < n; i += GW_NW) {
        const double* row = Lm + (int64_t)i * ldl;
        double mx = -INFINITY, s = 0;
        for (int j = lane; j < m; j += kWave) lse_add((sh.g[j] - row[j]) / eps, mx, s);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const double m2 = __shfl_xor(mx, o, kWave), s2 = __shfl_xor(s, o, kWave);
            lse_merge(mx, s, m2, s2);
        }
        if (lane == 0) sh.f[i] = eps * log(marg(a, i, n)) - eps * (mx + log(s));
    }
    __syncthreads();
}

// L1 error of the column marginal: sum_j |sum_i exp((f_i + g_j - L_ij)/eps) - b_j|
__device__ double lse_col_error(const double* Lm, int64_t ldl, int n, int m, const double* b,
                                double eps, GwShared& sh) {
    const ColMap cm(m);
    double err = 0;
    for (int j0 = 0; j0 < m; j0 += cm.CW) {
        const int j = j0 + cm.jj;
        double s = 0;
        if (j < m)
            for (int i = cm.seg; i < n; i += cm.S)
                s += exp((sh.f[i] + sh.g[j] - Lm[(int64_t)i * ldl + j]) / eps);
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

__device__ bool blk_timed_out(unsigned long long deadline, GwShared& sh) {
    if (threadIdx.x == 0) sh.flag = __builtin_amdgcn_s_memrealtime() > deadline;
    __syncthreads();
    const bool t = sh.flag != 0;
    __syncthreads();
    return t;
}

// OTT lse-mode Sinkhorn on L (n x m) from the potentials in sh.f / sh.g:
// chunks of `inner` (g, f) updates, L1 column error after each chunk.
__device__ int blk_sinkhorn_lse(const double* Lm, int64_t ldl, int n, int m, const double* a,
                                const double* b, double eps, double thr, int inner, int maxit,
                                GwShared& sh, bool& conv, unsigned long long deadline,
                                bool& timeout) {
    int it = 0;
    conv = false;
    while (it < maxit && !conv) {
        for (int k = 0; k < inner && it < maxit; ++k, ++it) {
            lse_col_update(Lm, ldl, n, m, b, eps, sh);
            lse_row_update(Lm, ldl, n, m, a, eps, sh);
        }
        const double err = lse_col_error(Lm, ldl, n, m, b, eps, sh);
        if (!(err == err)) break;  // diverged
        conv = err < thr;
        if (blk_timed_out(deadline, sh)) { timeout = true; break; }
    }
    return it;
}

// Minimum-cost assignment of the n x n matrix A (row stride lda), one wavefront:
// shortest augmenting paths with dual potentials, lanes over columns, ties to the
// lowest column (the serial scan's order).  Wave-synchronous LDS (volatile, one
// wave in program order).  Writes sh.lap.sigma; returns false on a non-finite cost.
__device__ bool wave_lap(const double* A, int64_t lda, int n, GwShared& sh) {
    const int lane = threadIdx.x;
    typedef volatile __attribute__((address_space(3))) double lds_d;
    typedef volatile __attribute__((address_space(3))) int lds_i;
    typedef volatile __attribute__((address_space(3))) unsigned char lds_u8;
    lds_d* u = (lds_d*)sh.f;
    lds_d* v = (lds_d*)sh.g;
    lds_d* minv = (lds_d*)sh.lap.minv;
    lds_i* pc = (lds_i*)sh.lap.pc;
    lds_i* way = (lds_i*)sh.lap.way;
    lds_u8* used = (lds_u8*)sh.lap.used;
    for (int j = lane; j <= n; j += kWave) { u[j] = 0; v[j] = 0; pc[j] = 0; way[j] = 0; }
    for (int i = 1; i <= n; ++i) {
        if (lane == 0) pc[0] = i;
        int j0 = 0;
        for (int j = lane; j <= n; j += kWave) { minv[j] = GW_INF; used[j] = 0; }
        while (true) {
            if (lane == 0) used[j0] = 1;
            const int i0 = pc[j0];
            const double ui0 = u[i0];
            const double* arow = A + (int64_t)(i0 - 1) * lda;
            double delta = GW_INF;
            int j1 = 0x7fffffff;
            for (int j = 1 + lane; j <= n; j += kWave) {
                if (!used[j]) {
                    const double cur = arow[j - 1] - ui0 - v[j];
                    if (cur < minv[j]) { minv[j] = cur; way[j] = j0; }
                    if (minv[j] < delta) { delta = minv[j]; j1 = j; }
                }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const double od = __shfl_xor(delta, o, kWave);
                const int oj = __shfl_xor(j1, o, kWave);
                if (od < delta || (od == delta && oj < j1)) { delta = od; j1 = oj; }
            }
            if (j1 > n || !(delta < GW_INF)) return false;
            for (int j = lane; j <= n; j += kWave) {
                if (used[j]) { u[pc[j]] += delta; v[j] -= delta; }
                else minv[j] -= delta;
            }
            j0 = j1;
            if (pc[j0] == 0) break;
        }
        if (lane == 0) {
            do {
                const int jp = way[j0];
                pc[j0] = pc[jp];
                j0 = jp;
            } while (j0 != 0);
        }
    }
    for (int j = 1 + lane; j <= n; j += kWave) sh.lap.sigma[pc[j] - 1] = j - 1;
    return true;
}

// ---------------------------------------------------------------------- the kernel
__global__ __launch_bounds__(GW_NT) void gw_kernel(GwLaunch Lz, otf_gw_opts o, otf_gw_info* infos,
                                                   double* costlog, int costlog_len,
                                                   unsigned long long timeout_ticks) {
    __shared__ GwShared sh;
    if ((int)blockIdx.x >= Lz.nprob) return;
    const otf_gw_problem P = Lz.prob[blockIdx.x];
    const int pid = Lz.first + blockIdx.x;
    otf_gw_info* info = infos + pid;
    double* clog = costlog ? costlog + (int64_t)pid * costlog_len : nullptr;
    const int n = (int)P.n, m = (int)P.m;
    const int64_t ldt = P.ldt;
    const int64_t nm = (int64_t)n * m;
    double* D = Lz.ws[blockIdx.x];  // C1 . G          (n x m, ld m)
    double* R = D + nm;             // C1 . G . C2     (n x m, ld m)
    double* Lm = R + nm;            // df / linearised cost (n x m, ld m)
    double* S = Lm + nm;            // CG: C1 . Gc . C2
    double* G = P.T;                // the plan, in place in the output
    const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + timeout_ticks;
    const int t = threadIdx.x;

    int status = OTF_GW_MAX_ITER, it = 0, inner_total = 0;
    bool converged = false, inner_conv = false;
    double cost = 0;

    if (o.solver == OTF_GW_CG) {
        // G0 = p q^T (uniform), constC terms from p, q
        const double g0 = 1.0 / ((double)n * (double)m);
        for (int64_t e = t; e < nm; e += GW_NT) G[(e / m) * ldt + (e % m)] = g0;
        for (int i = t; i < n; i += GW_NT) sh.mg.r[i] = 1.0 / n;
        for (int j = t; j < m; j += GW_NT) sh.mg.c[j] = 1.0 / m;
        __syncthreads();
        blk_sq_matvec(sh.x, P.C1, P.ldc1, n, sh.mg.r);
        blk_sq_matvec(sh.y, P.C2, P.ldc2, m, sh.mg.c);
        __syncthreads();
        blk_gemm<false>(D, m, P.C1, P.ldc1, G, ldt, n, m, n, nullptr, 1.0);
        __syncthreads();
        blk_gemm<false>(R, m, D, m, P.C2, P.ldc2, n, m, m, nullptr, 1.0);
        __syncthreads();
        // cost(G) = <constC - 2 R, G>
        double acc = 0;
        for (int64_t e = t; e < nm; e += GW_NT) {
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
            for (int64_t e = t; e < nm; e += GW_NT) {
                const int i = (int)(e / m), j = (int)(e % m);
                const double df = 2.0 * (sh.x[i] + sh.y[j] - 2.0 * R[e]);
                Lm[e] = df;
                mn = fmin(mn, df);
            }
            mn = blk_minmax(mn, sh.red, false);
            bool finite = true;
            for (int64_t e = t; e < nm; e += GW_NT) {
                const double v = Lm[e] + mn;
                Lm[e] = v;
                if (!finite_val(v)) finite = false;
            }
            sh.flag = 0;
            __syncthreads();
            if (!finite) sh.flag = 1;
            __syncthreads();
            if (sh.flag) { status = OTF_GW_NUMERICAL; break; }
            __syncthreads();
            // Gc = assignment(Mi) / n
            if (t < kWave) {
                const bool ok = wave_lap(Lm, m, n, sh);
                if (t == 0) sh.flag = ok ? 0 : 1;
            }
            __syncthreads();
            if (sh.flag) { status = OTF_GW_NUMERICAL; break; }
            // S = C1 Gc C2:  S_ij = (1/n) sum_k C1[i][k] C2[sigma(k)][j]
            blk_gemm<true>(S, m, P.C1, P.ldc1, P.C2, P.ldc2, n, m, n, sh.lap.sigma, 1.0 / n);
            __syncthreads();
            // dot = 2 (S - R); a = -<dot, Gc - G>; b = -2 <dot, G>
            double ta = 0, tb = 0;
            const double gc = 1.0 / n;
            for (int64_t e = t; e < nm; e += GW_NT) {
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
            for (int64_t e = t; e < nm; e += GW_NT) {
                const int i = (int)(e / m), j = (int)(e % m);
                const double gv = G[i * ldt + j];
                const double gcv = (sh.lap.sigma[i] == j) ? gc : 0.0;
                G[i * ldt + j] = gv + alpha * (gcv - gv);
            }
            __syncthreads();
            if (clog && t == 0 && it < costlog_len) clog[it] = cost;
            // df(G) for the next iteration (POT recomputes it from G)
            blk_gemm<false>(D, m, P.C1, P.ldc1, G, ldt, n, m, n, nullptr, 1.0);
            __syncthreads();
            blk_gemm<false>(R, m, D, m, P.C2, P.ldc2, n, m, m, nullptr, 1.0);
            __syncthreads();
            const double absd = fabs(cost - old);
            const double reld = cost != 0.0 ? absd / fabs(cost) : NAN;
            if (reld < o.tol_rel || absd < o.tol_abs) { converged = true; status = OTF_GW_CONVERGED; break; }
            if (it >= o.max_iter) break;
            if (blk_timed_out(deadline, sh)) { status = OTF_GW_TIMEOUT; break; }
        }
    } else {
        // Entropic GW (OTT).  P0 = a b^T; f = g = 0.
        const double* pa = P.p;
        const double* pb = P.q;
        for (int64_t e = t; e < nm; e += GW_NT) {
            const int i = (int)(e / m), j = (int)(e % m);
            G[i * ldt + j] = marg(pa, i, n) * marg(pb, j, m);
        }
        for (int i = t; i < n; i += GW_NT) { sh.mg.r[i] = marg(pa, i, n); sh.f[i] = 0; }
        for (int j = t; j < m; j += GW_NT) { sh.mg.c[j] = marg(pb, j, m); sh.g[j] = 0; }
        __syncthreads();
        double cprev = 0, cprev2 = 0;
        bool timeout = false;
        while (true) {
            // linearisation at the current plan
            blk_sq_matvec(sh.x, P.C1, P.ldc1, n, sh.mg.r);
            blk_sq_matvec(sh.y, P.C2, P.ldc2, m, sh.mg.c);
            blk_gemm<false>(D, m, P.C1, P.ldc1, G, ldt, n, m, n, nullptr, 1.0);
            __syncthreads();
            blk_gemm<false>(R, m, D, m, P.C2, P.ldc2, n, m, m, nullptr, 1.0);
            __syncthreads();
            for (int64_t e = t; e < nm; e += GW_NT) {
                const int i = (int)(e / m), j = (int)(e % m);
                double l = sh.x[i] + sh.y[j] - 2.0 * R[e];
                if (P.labels_a && P.labels_a[i] != P.labels_b[j]) l = INFINITY;
                Lm[e] = l;
            }
            if (!o.warm_start) {
                for (int i = t; i < n; i += GW_NT) sh.f[i] = 0;
                for (int j = t; j < m; j += GW_NT) sh.g[j] = 0;
            }
            __syncthreads();
            int sk_it = blk_sinkhorn_lse(Lm, m, n, m, pa, pb, o.eps, o.sk_threshold, o.sk_inner,
                                         o.sk_max_iter, sh, inner_conv, deadline, timeout);
            inner_total += sk_it;
            // plan, its marginals and mass; reg_ot_cost
            double mass = 0;
            for (int64_t e = t; e < nm; e += GW_NT) {
                const int i = (int)(e / m), j = (int)(e % m);
                const double pv = exp((sh.f[i] + sh.g[j] - Lm[e]) / o.eps);
                G[i * ldt + j] = pv;
                mass += pv;
            }
            mass = blk_sum(mass, sh.red);  // (barrier inside: plan visible)
            for (int i = t; i < n; i += GW_NT) {
                double s = 0;
                for (int j = 0; j < m; ++j) s += G[i * ldt + j];
                sh.mg.r[i] = s;
            }
            for (int j = t; j < m; j += GW_NT) {
                double s = 0;
                for (int i = 0; i < n; ++i) s += G[i * ldt + j];
                sh.mg.c[j] = s;
            }
            double fa = 0, sa = 0, sb = 0;
            for (int i = t; i < n; i += GW_NT) { fa += marg(pa, i, n) * sh.f[i]; sa += marg(pa, i, n); }
            for (int j = t; j < m; j += GW_NT) { fa += marg(pb, j, m) * sh.g[j]; sb += marg(pb, j, m); }
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
        }
    }
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
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < (int64_t)n * m;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int i = (int)(e / m), j = (int)(e % m);
        C[(int64_t)i * ldc + j] = C[(int64_t)i * ldc + j] / r;
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
    return otf::align256(8 * (size_t)n) + otf::align256(8 * (size_t)m) +
           otf::align256(8 * (size_t)otf::DIST_PARTS);
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
    // C = -2 X Y^T + |x|^2 + |y|^2   (POT euclidean_distances order)
    int rc = otf::launch_gemm<float, float, double, double>(X, ldx, 1, Y, 1, ldy, C, ldc, (int)n,
                                                            (int)m, (int)d, -2.0, 0.0, nx, ny, s);
    if (rc != OTF_OK) return rc;
    const int64_t tot = n * m;
    int grid = (int)((tot + 255) / 256);
    if (grid > otf::DIST_PARTS) grid = otf::DIST_PARTS;
    otf::dist_finalize_kernel<<<grid, 256, 0, s>>>(C, ldc, (int)n, (int)m,
                                                   metric == OTF_EUCLIDEAN, zero_diag, part);
    otf::dist_scale_kernel<<<grid, 256, 0, s>>>(C, ldc, (int)n, (int)m, part, grid, scale_max, cmax);
    OTF_HIP(hipGetLastError());
    return OTF_OK;
}

size_t otf_gw_workspace_size(int32_t nprob, const otf_gw_problem* probs) {
    if (nprob <= 0 || !probs) return 0;
    size_t tot = 0;
    for (int b = 0; b < nprob; ++b) tot += otf::align256(4 * 8 * (size_t)(probs[b].n * probs[b].m));
    return tot;
}

int otf_gw_solve(int32_t nprob, const otf_gw_problem* probs, const otf_gw_opts* opts,
                 otf_gw_info* info, double* costlog, int32_t costlog_len, void* workspace,
                 size_t ws_bytes, otf_stream_t stream) {
    using namespace otf;
    if (nprob <= 0 || !probs || !opts || !info || !workspace) return OTF_EINVAL;
    const otf_gw_opts o = *opts;
    if (o.solver != OTF_GW_CG && o.solver != OTF_GW_ENTROPIC) return OTF_EINVAL;
    if (o.max_iter < 1) return OTF_EINVAL;
    if (o.solver == OTF_GW_ENTROPIC && (!(o.eps > 0) || o.sk_inner < 1 || o.sk_max_iter < 1))
        return OTF_EINVAL;
    if (costlog && costlog_len < 1) return OTF_EINVAL;
    if (ws_bytes < otf_gw_workspace_size(nprob, probs)) return OTF_EINVAL;
    for (int b = 0; b < nprob; ++b) {
        const otf_gw_problem& P = probs[b];
        if (!P.C1 || !P.C2 || !P.T || P.n < 1 || P.m < 1) return OTF_EINVAL;
        if (P.ldc1 < P.n || P.ldc2 < P.m || P.ldt < P.m) return OTF_EINVAL;
        if (P.n > GW_MAXN || P.m > GW_MAXN) return OTF_EUNSUPPORTED;
        if ((P.labels_a == nullptr) != (P.labels_b == nullptr)) return OTF_EINVAL;
        if (o.solver == OTF_GW_CG) {
            // exact EMD as an assignment: uniform marginals on equal sizes
            if (P.n != P.m || P.p || P.q || P.labels_a) return OTF_EUNSUPPORTED;
        }
    }
    hipStream_t s = (hipStream_t)stream;
    char* wsp = (char*)workspace;
    const unsigned long long ticks = 100000000ull * 20;  // 20 s at 100 MHz
    for (int first = 0; first < nprob; first += GW_MAXP) {
        GwLaunch L{};
        L.first = first;
        L.nprob = nprob - first < GW_MAXP ? nprob - first : GW_MAXP;
        for (int b = 0; b < L.nprob; ++b) {
            L.prob[b] = probs[first + b];
            L.ws[b] = (double*)wsp;
            wsp += align256(4 * 8 * (size_t)(probs[first + b].n * probs[first + b].m));
        }
        gw_kernel<<<L.nprob, GW_NT, 0, s>>>(L, o, info, costlog, costlog_len, ticks);
        OTF_HIP(hipGetLastError());
    }
    return OTF_OK;
}

}  // extern "C"
