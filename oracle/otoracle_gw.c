/*
 * otoracle_gw.c — CPU restatement of the reference's Gromov-Wasserstein couplings.
 *
 * TEST INFRASTRUCTURE ONLY (see otoracle.c): the parity checker for the HIP GW
 * solvers (csrc/otf_gw.hip).  Never linked or called by the product path.
 *
 * Provenance (file:line into the reference tree; third-party code is absent from
 * the container, so these are restatements of the published algorithms and the
 * parity they anchor is UNPINNED by the reference's own outputs):
 *   oro_lap        exact EMD for uniform marginals on n x n (a minimum-cost
 *                  assignment / n), the inner solve of POT's CG-GW; shortest
 *                  augmenting paths with potentials, serial scan (ties -> lowest
 *                  column).  Cross-checked in tests against scipy's
 *                  linear_sum_assignment (an independent implementation).
 *   oro_gw_cg      POT 0.9.6.post1 ot.gromov.gromov_wasserstein(C1, C2, p, q,
 *                  'square_loss') -> ot.optim.cg -> generic_conditional_gradient,
 *                  with init_matrix / gwloss / gwggrad / solve_gromov_linesearch;
 *                  call site MRI_PET_OT_nojax.py:80-82 (pinned OT_environment.yml:232).
 *   oro_gw_entropic  OTT-jax 0.6.0 GromovWasserstein(epsilon, linear_solver=
 *                  Sinkhorn(max_iterations)) with PointCloud(scale_cost="max_cost"),
 *                  call sites MRI_PET_OT_OT_per_epoch_attn.py:155-174 and
 *                  perturbot/perturbot/match/ott_egwl.py:77-105,178-194,261-278
 *                  (pinned OT_environment.yml:227).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORO_EXPORT __attribute__((visibility("default")))
#define LAP_INF 1e300

/* Minimum-cost assignment of the n x n matrix A (row-major).  sigma[i] = column
 * of row i.  Returns 0, or 1 on a non-finite cost. */
ORO_EXPORT int oro_lap(const double* A, int64_t n, int* sigma) {
    double* u = (double*)calloc((size_t)n + 1, sizeof(double));
    double* v = (double*)calloc((size_t)n + 1, sizeof(double));
    double* minv = (double*)malloc(sizeof(double) * ((size_t)n + 1));
    int* p = (int*)calloc((size_t)n + 1, sizeof(int));
    int* way = (int*)calloc((size_t)n + 1, sizeof(int));
    char* used = (char*)malloc((size_t)n + 1);
    int rc = 0;
    /* column reduction v_j = min_i a_ij, then a greedy pass: row i takes its cheapest
     * reduced column (lowest index on ties) with u_i = that reduced cost when the
     * column is still free.  Potentials stay feasible (a_ij - u_i - v_j >= 0) and the
     * taken edges tight, so the shortest-path phase below completes an optimum. */
    char* done = (char*)calloc((size_t)n + 1, 1);
    for (int64_t j = 1; j <= n; ++j) {
        double mn = LAP_INF;
        for (int64_t i = 1; i <= n; ++i) if (A[(i - 1) * n + (j - 1)] < mn) mn = A[(i - 1) * n + (j - 1)];
        v[j] = mn;
    }
    for (int64_t i = 1; i <= n; ++i) {
        double mn = LAP_INF;
        int64_t jb = -1;
        for (int64_t j = 1; j <= n; ++j) {
            const double r = A[(i - 1) * n + (j - 1)] - v[j];
            if (r < mn) { mn = r; jb = j; }
        }
        if (jb < 0) { rc = 1; break; }
        u[i] = mn;
        if (p[jb] == 0) { p[jb] = (int)i; done[i] = 1; }
    }
    for (int64_t i = 1; i <= n && !rc; ++i) {
        if (done[i]) continue;
        p[0] = (int)i;
        int64_t j0 = 0;
        for (int64_t j = 0; j <= n; ++j) { minv[j] = LAP_INF; used[j] = 0; }
        do {
            used[j0] = 1;
            const int64_t i0 = p[j0];
            double delta = LAP_INF;
            int64_t j1 = -1;
            for (int64_t j = 1; j <= n; ++j) {
                if (!used[j]) {
                    const double cur = A[(i0 - 1) * n + (j - 1)] - u[i0] - v[j];
                    if (cur < minv[j]) { minv[j] = cur; way[j] = (int)j0; }
                    if (minv[j] < delta) { delta = minv[j]; j1 = j; }
                }
            }
            if (j1 < 0) { rc = 1; break; }
            for (int64_t j = 0; j <= n; ++j) {
                if (used[j]) { u[p[j]] += delta; v[j] -= delta; }
                else minv[j] -= delta;
            }
            j0 = j1;
        } while (p[j0] != 0);
        if (rc) break;
        do {
            const int64_t j1 = way[j0];
            p[j0] = p[j1];
            j0 = j1;
        } while (j0);
    }
    if (!rc)
        for (int64_t j = 1; j <= n; ++j) sigma[p[j] - 1] = (int)(j - 1);
    free(u); free(v); free(minv); free(p); free(way); free(used); free(done);
    return rc;
}

/* out = A (n x k) . B (k x m), row-major. */
static void mm(const double* A, const double* B, double* out, int64_t n, int64_t k, int64_t m) {
    for (int64_t i = 0; i < n; ++i) {
        double* o = out + i * m;
        for (int64_t j = 0; j < m; ++j) o[j] = 0.0;
        for (int64_t kk = 0; kk < k; ++kk) {
            const double a = A[i * k + kk];
            const double* b = B + kk * m;
            for (int64_t j = 0; j < m; ++j) o[j] += a * b[j];
        }
    }
}

/* tens = constC - hC1 T hC2^T, hC1 = C1, hC2 = 2 C2 (C2 symmetric) */
static void tensor_product(const double* constC, const double* C1, const double* C2,
                           const double* T, int64_t n, int64_t m, double* tmp, double* tens) {
    mm(C1, T, tmp, n, n, m);
    mm(tmp, C2, tens, n, m, m);
    for (int64_t e = 0; e < n * m; ++e) tens[e] = constC[e] - 2.0 * tens[e];
}

/* POT CG-GW, uniform p = q = 1/n, n x n.  info: [n_iter, converged, status].
 * costlog[0..] = log['loss'] (initial cost, then one per iteration). */
ORO_EXPORT int oro_gw_cg(const double* C1, const double* C2, int64_t n, int max_iter,
                         double tol_rel, double tol_abs, double* G, double* costlog,
                         int costlog_len, int64_t* info, double* cost_out) {
    const int64_t m = n, nm = n * m;
    double* constC = (double*)malloc(sizeof(double) * (size_t)nm);
    double* tmp = (double*)malloc(sizeof(double) * (size_t)nm);
    double* tens = (double*)malloc(sizeof(double) * (size_t)nm);
    double* Mi = (double*)malloc(sizeof(double) * (size_t)nm);
    double* dG = (double*)malloc(sizeof(double) * (size_t)nm);
    double* dot = (double*)malloc(sizeof(double) * (size_t)nm);
    int* sigma = (int*)malloc(sizeof(int) * (size_t)n);
    const double p = 1.0 / (double)n, q = 1.0 / (double)m;
    /* init_matrix: constC = (C1^2 p) 1^T + 1 (C2^2 q)^T */
    for (int64_t i = 0; i < n; ++i) {
        double s1 = 0.0, s2 = 0.0;
        for (int64_t k = 0; k < n; ++k) s1 += C1[i * n + k] * C1[i * n + k] * p;
        for (int64_t k = 0; k < m; ++k) s2 += C2[i * m + k] * C2[i * m + k] * q;
        tmp[i] = s1;
        dG[i] = s2;
    }
    for (int64_t i = 0; i < n; ++i)
        for (int64_t j = 0; j < m; ++j) constC[i * m + j] = tmp[i] + dG[j];
    for (int64_t e = 0; e < nm; ++e) G[e] = p * q;
    /* cost(G) = gwloss = sum(tens * G) */
    tensor_product(constC, C1, C2, G, n, m, tmp, tens);
    double cost = 0.0;
    for (int64_t e = 0; e < nm; ++e) cost += tens[e] * G[e];
    if (costlog && costlog_len > 0) costlog[0] = cost;
    int it = 0, conv = 0, status = 2;
    for (;;) {
        ++it;
        const double old = cost;
        /* df = gwggrad = 2 tens;  Mi = df + min(df) */
        tensor_product(constC, C1, C2, G, n, m, tmp, tens);
        double mn = INFINITY;
        for (int64_t e = 0; e < nm; ++e) { Mi[e] = 2.0 * tens[e]; if (Mi[e] < mn) mn = Mi[e]; }
        for (int64_t e = 0; e < nm; ++e) Mi[e] += mn;
        if (oro_lap(Mi, n, sigma)) { status = 3; break; }
        /* deltaG = Gc - G */
        for (int64_t i = 0; i < n; ++i)
            for (int64_t j = 0; j < m; ++j)
                dG[i * m + j] = (sigma[i] == j ? 1.0 / (double)n : 0.0) - G[i * m + j];
        /* solve_gromov_linesearch (symmetric): dot = hC1 dG hC2^T */
        mm(C1, dG, tmp, n, n, m);
        mm(tmp, C2, dot, n, m, m);
        double a = 0.0, b = 0.0;
        for (int64_t e = 0; e < nm; ++e) {
            dot[e] *= 2.0;
            a -= dot[e] * dG[e];
            b -= 2.0 * dot[e] * G[e];
        }
        double alpha;
        if (a > 0) alpha = fmin(1.0, fmax(0.0, -b / (2.0 * a)));
        else alpha = (a + b < 0) ? 1.0 : 0.0;
        cost = cost + a * alpha * alpha + b * alpha;
        for (int64_t e = 0; e < nm; ++e) G[e] += alpha * dG[e];
        if (costlog && it < costlog_len) costlog[it] = cost;
        const double absd = fabs(cost - old);
        const double reld = cost != 0.0 ? absd / fabs(cost) : NAN;
        if (reld < tol_rel || absd < tol_abs) { conv = 1; status = 1; break; }
        if (it >= max_iter) break;
    }
    if (info) { info[0] = it; info[1] = conv; info[2] = status; }
    if (cost_out) *cost_out = cost;
    free(constC); free(tmp); free(tens); free(Mi); free(dG); free(dot); free(sigma);
    return 0;
}

static double marg(const double* w, int64_t i, int64_t n) { return w ? w[i] : 1.0 / (double)n; }

/* OTT lse Sinkhorn on L from the potentials in f, g (updated in place).
 * Returns iterations; *conv = last error < thr. */
static int sk_lse(const double* L, int64_t n, int64_t m, const double* a, const double* b,
                  double eps, double thr, int inner, int maxit, double* f, double* g, int* conv) {
    int it = 0;
    *conv = 0;
    while (it < maxit && !*conv) {
        for (int k = 0; k < inner && it < maxit; ++k, ++it) {
            for (int64_t j = 0; j < m; ++j) {
                double mx = -INFINITY;
                for (int64_t i = 0; i < n; ++i) {
                    const double z = (f[i] - L[i * m + j]) / eps;
                    if (z > mx) mx = z;
                }
                double s = 0.0;
                for (int64_t i = 0; i < n; ++i) s += exp((f[i] - L[i * m + j]) / eps - mx);
                g[j] = eps * log(marg(b, j, m)) - eps * (mx + log(s));
            }
            for (int64_t i = 0; i < n; ++i) {
                double mx = -INFINITY;
                for (int64_t j = 0; j < m; ++j) {
                    const double z = (g[j] - L[i * m + j]) / eps;
                    if (z > mx) mx = z;
                }
                double s = 0.0;
                for (int64_t j = 0; j < m; ++j) s += exp((g[j] - L[i * m + j]) / eps - mx);
                f[i] = eps * log(marg(a, i, n)) - eps * (mx + log(s));
            }
        }
        double err = 0.0;
        for (int64_t j = 0; j < m; ++j) {
            double s = 0.0;
            for (int64_t i = 0; i < n; ++i) s += exp((f[i] + g[j] - L[i * m + j]) / eps);
            err += fabs(s - marg(b, j, m));
        }
        if (err != err) break;
        *conv = err < thr;
    }
    return it;
}

/* OTT entropic GW.  info: [n_iter, converged, inner_converged, inner_total, status].
 * la / lb (nullable): labels; the coupling is restricted to equal labels. */
ORO_EXPORT int oro_gw_entropic(const double* C1, const double* C2, int64_t n, int64_t m,
                               const double* a, const double* b, const int* la, const int* lb,
                               double eps, int max_iter, int min_iter, double threshold,
                               int sk_max, int sk_inner, double sk_thr, int warm, double* P,
                               double* costlog, int costlog_len, int64_t* info, double* cost_out) {
    const int64_t nm = n * m;
    double* tmp = (double*)malloc(sizeof(double) * (size_t)nm);
    double* R = (double*)malloc(sizeof(double) * (size_t)nm);
    double* L = (double*)malloc(sizeof(double) * (size_t)nm);
    double* f = (double*)calloc((size_t)n, sizeof(double));
    double* g = (double*)calloc((size_t)m, sizeof(double));
    double* r = (double*)malloc(sizeof(double) * (size_t)n);
    double* c = (double*)malloc(sizeof(double) * (size_t)m);
    double* x = (double*)malloc(sizeof(double) * (size_t)n);
    double* y = (double*)malloc(sizeof(double) * (size_t)m);
    for (int64_t i = 0; i < n; ++i) r[i] = marg(a, i, n);
    for (int64_t j = 0; j < m; ++j) c[j] = marg(b, j, m);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t j = 0; j < m; ++j) P[i * m + j] = r[i] * c[j];
    int it = 0, conv = 0, inner_conv = 0, inner_total = 0, status = 2;
    double cost = 0.0, cprev = 0.0, cprev2 = 0.0;
    for (;;) {
        /* linearisation: L = x 1^T + 1 y^T - C1 P (2 C2)^T,  x = C1^2 r, y = C2^2 c */
        for (int64_t i = 0; i < n; ++i) {
            double s = 0.0;
            for (int64_t k = 0; k < n; ++k) s += C1[i * n + k] * C1[i * n + k] * r[k];
            x[i] = s;
        }
        for (int64_t j = 0; j < m; ++j) {
            double s = 0.0;
            for (int64_t k = 0; k < m; ++k) s += C2[j * m + k] * C2[j * m + k] * c[k];
            y[j] = s;
        }
        mm(C1, P, tmp, n, n, m);
        mm(tmp, C2, R, n, m, m);
        for (int64_t i = 0; i < n; ++i)
            for (int64_t j = 0; j < m; ++j) {
                double l = x[i] + y[j] - 2.0 * R[i * m + j];
                if (la && la[i] != lb[j]) l = INFINITY;
                L[i * m + j] = l;
            }
        if (!warm) {
            memset(f, 0, sizeof(double) * (size_t)n);
            memset(g, 0, sizeof(double) * (size_t)m);
        }
        inner_total += sk_lse(L, n, m, a, b, eps, sk_thr, sk_inner, sk_max, f, g, &inner_conv);
        double mass = 0.0;
        for (int64_t i = 0; i < n; ++i) r[i] = 0.0;
        for (int64_t j = 0; j < m; ++j) c[j] = 0.0;
        for (int64_t i = 0; i < n; ++i)
            for (int64_t j = 0; j < m; ++j) {
                const double pv = exp((f[i] + g[j] - L[i * m + j]) / eps);
                P[i * m + j] = pv;
                mass += pv;
                r[i] += pv;
                c[j] += pv;
            }
        double fa = 0.0, sa = 0.0, sb = 0.0;
        for (int64_t i = 0; i < n; ++i) { fa += marg(a, i, n) * f[i]; sa += marg(a, i, n); }
        for (int64_t j = 0; j < m; ++j) { fa += marg(b, j, m) * g[j]; sb += marg(b, j, m); }
        cost = fa + eps * (sa * sb - mass);
        if (costlog && it < costlog_len) costlog[it] = cost;
        ++it;
        cprev2 = cprev;
        cprev = cost;
        if (cost != cost) { status = 3; break; }
        const int close = it >= 2 && fabs(cprev2 - cprev) <= 1e-8 + threshold * fabs(cprev);
        if (it >= max_iter) { conv = close; if (close) status = 1; break; }
        const int keep = it < min_iter || it <= 2 || (isfinite(cprev) && !close);
        if (!keep) { conv = close; status = close ? 1 : 3; break; }
    }
    if (info) { info[0] = it; info[1] = conv; info[2] = inner_conv; info[3] = inner_total; info[4] = status; }
    if (cost_out) *cost_out = cost;
    free(tmp); free(R); free(L); free(f); free(g); free(r); free(c); free(x); free(y);
    return 0;
}

/* POT 0.9.6 ot.gromov.entropic_gromov_wasserstein(C1, C2, p, q, 'square_loss', epsilon,
 * solver='PGD') on symmetric C1, C2, as called by perturbot/perturbot/match/gw.py:31-59
 * (egw_pgd) and :80-102 (egw_all).  T0 = p q^T; per iteration
 *     tens = gwggrad = 2 tensor_product(constC, C1, 2 C2, T) = 2 (constC - 2 C1 T C2)
 *     T    = sinkhorn_knopp(p, q, tens, eps, numItermax = sk_max, stopThr = sk_thr)
 * (ot.bregman.sinkhorn_knopp: K = exp(tens / -eps), Kp = K / p, u = 1/n, v = 1/m,
 * v = q / K^T u, u = 1 / (Kp v); a zero K^T u or non-finite u / v keeps the previous
 * pair and stops; every 10th update err = || sum_i u_i K_ij v_j - q ||_2 < stopThr
 * stops); every 10th outer iteration err = ||T - Tprev||_F; loop while err > tol and
 * it < max_iter.  info: [n_iter, converged, inner_total, n_err]; errlog = log['err'];
 * cost_out = log['gw_dist'] = sum(tensor_product(T) * T). */
ORO_EXPORT int oro_gw_pgd(const double* C1, const double* C2, int64_t n, int64_t m,
                          const double* a, const double* b, double eps, int max_iter, double tol,
                          int sk_max, double sk_thr, double* T, double* errlog, int errlog_len,
                          int64_t* info, double* cost_out) {
    const int64_t nm = n * m;
    double* constC = (double*)malloc(sizeof(double) * (size_t)nm);
    double* tmp = (double*)malloc(sizeof(double) * (size_t)nm);
    double* tens = (double*)malloc(sizeof(double) * (size_t)nm);
    double* K = (double*)malloc(sizeof(double) * (size_t)nm);
    double* Kp = (double*)malloc(sizeof(double) * (size_t)nm);
    double* u = (double*)malloc(sizeof(double) * (size_t)n);
    double* v = (double*)malloc(sizeof(double) * (size_t)m);
    double* up = (double*)malloc(sizeof(double) * (size_t)n);
    double* vp = (double*)malloc(sizeof(double) * (size_t)m);
    /* init_matrix (square loss): constC = (C1^2 p) 1^T + 1 (C2^2 q)^T */
    for (int64_t i = 0; i < n; ++i) {
        double s = 0.0;
        for (int64_t k = 0; k < n; ++k) s += C1[i * n + k] * C1[i * n + k] * marg(a, k, n);
        up[i] = s;
    }
    for (int64_t j = 0; j < m; ++j) {
        double s = 0.0;
        for (int64_t k = 0; k < m; ++k) s += C2[j * m + k] * C2[j * m + k] * marg(b, k, m);
        vp[j] = s;
    }
    for (int64_t i = 0; i < n; ++i)
        for (int64_t j = 0; j < m; ++j) {
            constC[i * m + j] = up[i] + vp[j];
            T[i * m + j] = marg(a, i, n) * marg(b, j, m);
        }
    double err = 1.0;
    int it = 0, nerr = 0, inner_total = 0;
    while (err > tol && it < max_iter) {
        tensor_product(constC, C1, C2, T, n, m, tmp, tens);
        for (int64_t e = 0; e < nm; ++e) K[e] = exp(2.0 * tens[e] / -eps);
        for (int64_t i = 0; i < n; ++i) {
            const double ia = 1.0 / marg(a, i, n);
            for (int64_t j = 0; j < m; ++j) Kp[i * m + j] = ia * K[i * m + j];
        }
        for (int64_t i = 0; i < n; ++i) u[i] = 1.0 / (double)n;
        for (int64_t j = 0; j < m; ++j) v[j] = 1.0 / (double)m;
        int ii;
        for (ii = 0; ii < sk_max; ++ii) {
            memcpy(up, u, sizeof(double) * (size_t)n);
            memcpy(vp, v, sizeof(double) * (size_t)m);
            int bad = 0;
            for (int64_t j = 0; j < m; ++j) {
                double s = 0.0;
                for (int64_t i = 0; i < n; ++i) s += K[i * m + j] * u[i];
                v[j] = marg(b, j, m) / s;
                if (s == 0.0 || !isfinite(v[j])) bad = 1;
            }
            for (int64_t i = 0; i < n; ++i) {
                double s = 0.0;
                for (int64_t j = 0; j < m; ++j) s += Kp[i * m + j] * v[j];
                u[i] = 1.0 / s;
                if (!isfinite(u[i])) bad = 1;
            }
            if (bad) {
                memcpy(u, up, sizeof(double) * (size_t)n);
                memcpy(v, vp, sizeof(double) * (size_t)m);
                break;
            }
            if (ii % 10 == 0) {
                double e2 = 0.0;
                for (int64_t j = 0; j < m; ++j) {
                    double s = 0.0;
                    for (int64_t i = 0; i < n; ++i) s += u[i] * K[i * m + j] * v[j];
                    const double d = s - marg(b, j, m);
                    e2 += d * d;
                }
                if (sqrt(e2) < sk_thr) break;
            }
        }
        inner_total += ii < sk_max ? ii + 1 : sk_max;
        double d2 = 0.0;
        for (int64_t i = 0; i < n; ++i)
            for (int64_t j = 0; j < m; ++j) {
                const double tv = u[i] * K[i * m + j] * v[j];
                const double d = tv - T[i * m + j];
                d2 += d * d;
                T[i * m + j] = tv;
            }
        if (it % 10 == 0) {
            err = sqrt(d2);
            if (errlog && nerr < errlog_len) errlog[nerr] = err;
            ++nerr;
        }
        ++it;
    }
    tensor_product(constC, C1, C2, T, n, m, tmp, tens);
    double cost = 0.0;
    for (int64_t e = 0; e < nm; ++e) cost += tens[e] * T[e];
    if (info) { info[0] = it; info[1] = err <= tol; info[2] = inner_total; info[3] = nerr; }
    if (cost_out) *cost_out = cost;
    free(constC); free(tmp); free(tens); free(K); free(Kp); free(u); free(v); free(up); free(vp);
    return 0;
}
