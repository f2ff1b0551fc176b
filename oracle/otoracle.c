/*
 * otoracle.c — CPU restatement of the reference's Sinkhorn OT fusion path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker and the timed CPU
 * baseline ("port" kind) for bench.py.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product path (the HIP
 * library under the package's csrc/) never links or calls it.
 *
 * Everything is float64, like the reference: MRI_PET_OT_nojax.py promotes the
 * float32 embeddings to float64 through Ts (np.eye(B)/B, :688) and POT runs the
 * Sinkhorn loop in the dtype of M.
 *
 * Provenance of each routine (file:line into the reference tree):
 *   oro_pairwise_cost     POT 0.9.6.post1 ot.dist -> ot.utils.euclidean_distances
 *                         (third-party, not vendored; pinned OT_environment.yml:232),
 *                         call sites MRI_PET_OT_nojax.py:70-75 (+ "/= max").
 *   oro_feature_cost      MRI_PET_OT_nojax.py:121-136 (t1 + t2 - 2 X^T Ts Y).
 *   oro_sinkhorn_knopp    POT ot.sinkhorn -> ot.bregman.sinkhorn_knopp, called at
 *                         MRI_PET_OT_nojax.py:143; vendored twin
 *                         perturbot/perturbot/match/utils.py:6-115 (sinkhorn_scaling).
 *   oro_sinkhorn_log      OTT-jax 0.6.0 log-domain Sinkhorn (lse_mode) as called by
 *                         perturbot/perturbot/match/fot.py:128-134 — OTT is absent
 *                         from the container: parity unpinned.
 *   oro_plan_apply        MRI_PET_OT_nojax.py:701-721 (NaN->1e-8, row-normalise,
 *                         pet_fused @ T^T).
 *
 * Build: see oracle/Makefile (gcc -O2 -fopenmp -shared).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORO_EXPORT __attribute__((visibility("default")))

ORO_EXPORT int oro_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
    return omp_get_max_threads();
#else
    (void)n;
    return 1;
#endif
}

/* ---------------------------------------------------------------------------
 * Pairwise cost.  POT euclidean_distances: c = -2 X Y^T + |x|^2 + |y|^2,
 * clamp at 0, sqrt for metric 'euclidean', zero the diagonal when X is Y.
 * scale_max != 0 divides by the global max (MRI_PET_OT_nojax.py:74-75).
 * Returns the max of the unscaled cost.
 * ------------------------------------------------------------------------- */
ORO_EXPORT double oro_pairwise_cost(const double* X, const double* Y, int64_t n, int64_t m,
                                    int64_t d, int euclidean, int zero_diag, int scale_max,
                                    double* C) {
    double* xx = (double*)malloc(sizeof(double) * (size_t)n);
    double* yy = (double*)malloc(sizeof(double) * (size_t)m);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        double s = 0.0;
        for (int64_t k = 0; k < d; ++k) s += X[i * d + k] * X[i * d + k];
        xx[i] = s;
    }
#pragma omp parallel for schedule(static)
    for (int64_t j = 0; j < m; ++j) {
        double s = 0.0;
        for (int64_t k = 0; k < d; ++k) s += Y[j * d + k] * Y[j * d + k];
        yy[j] = s;
    }
    double gmax = 0.0;
#pragma omp parallel for schedule(static) reduction(max : gmax)
    for (int64_t i = 0; i < n; ++i) {
        const double* xi = X + i * d;
        for (int64_t j = 0; j < m; ++j) {
            const double* yj = Y + j * d;
            double dot = 0.0;
            for (int64_t k = 0; k < d; ++k) dot += xi[k] * yj[k];
            double c = -2.0 * dot + xx[i] + yy[j];
            if (c < 0.0) c = 0.0;
            if (euclidean) c = sqrt(c);
            if (zero_diag && i == j) c = 0.0;
            C[i * m + j] = c;
            if (c > gmax) gmax = c;
        }
    }
    if (scale_max && gmax > 0.0) {
#pragma omp parallel for schedule(static)
        for (int64_t t = 0; t < n * m; ++t) C[t] = C[t] / gmax;
    }
    free(xx);
    free(yy);
    return gmax;
}

/* ---------------------------------------------------------------------------
 * Feature cost M (d x d2) = t1[:,None] + t2[None,:] - 2 X^T Ts Y with
 * w1 = Ts.sum(1), t1 = (X^2)^T w1, w2 = Ts.sum(0), t2 = (Y^2)^T w2.
 * X: n x d, Y: n2 x d2, Ts: n x n2 (all row-major).  MRI_PET_OT_nojax.py:121-136.
 * ------------------------------------------------------------------------- */
ORO_EXPORT void oro_feature_cost(const double* X, const double* Y, const double* Ts, int64_t n,
                                 int64_t n2, int64_t d, int64_t d2, int sq_f32, int fot_weights,
                                 double* M) {
    /* sq_f32: the reference's X**2 runs in float32 on its float32 embeddings, then
     * promotes through the float64 weights; fot_weights: perturbot fot.py:109-110
     * uses w1 = Ts.sum(axis=0), w2 = Ts.sum(axis=1) (needs n == n2). */
    double* w1 = (double*)calloc((size_t)n, sizeof(double));
    double* w2 = (double*)calloc((size_t)n2, sizeof(double));
    double* t1 = (double*)calloc((size_t)d, sizeof(double));
    double* t2 = (double*)calloc((size_t)d2, sizeof(double));
    double* Z = (double*)calloc((size_t)(n * d2), sizeof(double)); /* Ts @ Y */
    for (int64_t i = 0; i < n; ++i)
        for (int64_t j = 0; j < n2; ++j) {
            if (fot_weights) {
                w1[j] += Ts[i * n2 + j];
                w2[i] += Ts[i * n2 + j];
            } else {
                w1[i] += Ts[i * n2 + j];
                w2[j] += Ts[i * n2 + j];
            }
        }
    for (int64_t i = 0; i < n; ++i)
        for (int64_t k = 0; k < d; ++k) {
            const double x = X[i * d + k];
            const double sq = sq_f32 ? (double)((float)x * (float)x) : x * x;
            t1[k] += sq * w1[i];
        }
    for (int64_t j = 0; j < n2; ++j)
        for (int64_t l = 0; l < d2; ++l) {
            const double y = Y[j * d2 + l];
            const double sq = sq_f32 ? (double)((float)y * (float)y) : y * y;
            t2[l] += sq * w2[j];
        }
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i)
        for (int64_t j = 0; j < n2; ++j) {
            const double t = Ts[i * n2 + j];
            if (t == 0.0) continue;
            for (int64_t l = 0; l < d2; ++l) Z[i * d2 + l] += t * Y[j * d2 + l];
        }
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < d; ++k) {
        for (int64_t l = 0; l < d2; ++l) {
            double s = 0.0;
            for (int64_t i = 0; i < n; ++i) s += X[i * d + k] * Z[i * d2 + l];
            M[k * d2 + l] = t1[k] + t2[l] - 2.0 * s;
        }
    }
    free(w1);
    free(w2);
    free(t1);
    free(t2);
    free(Z);
}

/* ---------------------------------------------------------------------------
 * Sinkhorn-Knopp, kernel domain, exact POT sinkhorn_knopp update sequence:
 *   K = exp(-C * cscale / reg);  u = 1/n;  v = 1/m;  Kp = K / a[:,None]
 *   for ii < numItermax:
 *       uprev, vprev = u, v
 *       KtU = K^T u;  v = b / KtU;  u = 1 / (Kp v)
 *       if any(KtU == 0) or nan/inf in u, v: u, v = uprev, vprev; break
 *       if ii % check_every == 0:
 *           err = || sum_i u_i K_ij v_j - b ||_2   (squared when err_squared,
 *                                                   i.e. the vendored utils.py:88-89)
 *           if err < stopThr: break      (POT; the vendored loop tests err > stopThr)
 *   P = u K v
 * info[0] = POT log['niter'] (the last ii), info[1] = updates applied,
 * info[2] = numerical break at iteration (or -1), info[3] = #err entries.
 * errlog (optional) receives each err value.
 * ------------------------------------------------------------------------- */
ORO_EXPORT int oro_sinkhorn_knopp(const double* a, const double* b, const double* C, int64_t n,
                                  int64_t m, double reg, double cscale, int numItermax,
                                  double stopThr, int check_every, int err_squared, double* u_out,
                                  double* v_out, double* P, int64_t* info, double* errlog) {
    double* K = (double*)malloc(sizeof(double) * (size_t)(n * m));
    double* u = (double*)malloc(sizeof(double) * (size_t)n);
    double* v = (double*)malloc(sizeof(double) * (size_t)m);
    double* up = (double*)malloc(sizeof(double) * (size_t)n);
    double* vp = (double*)malloc(sizeof(double) * (size_t)m);
    double* ktu = (double*)malloc(sizeof(double) * (size_t)m);
    double* ia = (double*)malloc(sizeof(double) * (size_t)n);
    const double nreg = -reg;
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < n * m; ++t) K[t] = exp((cscale == 1.0 ? C[t] : C[t] * cscale) / nreg);
    for (int64_t i = 0; i < n; ++i) {
        u[i] = 1.0 / (double)n;
        ia[i] = 1.0 / a[i];
    }
    for (int64_t j = 0; j < m; ++j) v[j] = 1.0 / (double)m;
    int64_t niter = 0, nupd = 0, brk = -1, nerr = 0;
    int ii = 0;
    for (ii = 0; ii < numItermax; ++ii) {
        memcpy(up, u, sizeof(double) * (size_t)n);
        memcpy(vp, v, sizeof(double) * (size_t)m);
        /* K^T u : column-blocked so each thread streams contiguous row segments */
#pragma omp parallel
        {
#ifdef _OPENMP
            const int nt = omp_get_num_threads(), tid = omp_get_thread_num();
#else
            const int nt = 1, tid = 0;
#endif
            const int64_t j0 = m * tid / nt, j1 = m * (tid + 1) / nt;
            for (int64_t j = j0; j < j1; ++j) ktu[j] = 0.0;
            for (int64_t i = 0; i < n; ++i) {
                const double ui = u[i];
                const double* Ki = K + i * m;
                for (int64_t j = j0; j < j1; ++j) ktu[j] += Ki[j] * ui;
            }
        }
        int zero = 0;
        for (int64_t j = 0; j < m; ++j) {
            if (ktu[j] == 0.0) zero = 1;
            v[j] = b[j] / ktu[j];
        }
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < n; ++i) {
            const double* Ki = K + i * m;
            double acc = 0.0;
            for (int64_t j = 0; j < m; ++j) acc += (ia[i] * Ki[j]) * v[j];
            u[i] = 1.0 / acc;
        }
        int bad = zero;
        for (int64_t i = 0; i < n && !bad; ++i)
            if (isnan(u[i]) || isinf(u[i])) bad = 1;
        for (int64_t j = 0; j < m && !bad; ++j)
            if (isnan(v[j]) || isinf(v[j])) bad = 1;
        if (bad) {
            memcpy(u, up, sizeof(double) * (size_t)n);
            memcpy(v, vp, sizeof(double) * (size_t)m);
            brk = ii;
            break;
        }
        ++nupd;
        if (ii % check_every == 0) {
            /* sum_i u_i K_ij v_j = v_j (K^T u)_j with the new u */
#pragma omp parallel
            {
#ifdef _OPENMP
                const int nt = omp_get_num_threads(), tid = omp_get_thread_num();
#else
                const int nt = 1, tid = 0;
#endif
                const int64_t j0 = m * tid / nt, j1 = m * (tid + 1) / nt;
                for (int64_t j = j0; j < j1; ++j) ktu[j] = 0.0;
                for (int64_t i = 0; i < n; ++i) {
                    const double ui = u[i];
                    const double* Ki = K + i * m;
                    for (int64_t j = j0; j < j1; ++j) ktu[j] += ui * Ki[j];
                }
            }
            double e = 0.0;
            for (int64_t j = 0; j < m; ++j) {
                const double r = ktu[j] * v[j] - b[j];
                e += r * r;
            }
            const double err = err_squared ? e : sqrt(e);
            if (errlog) errlog[nerr] = err;
            ++nerr;
            if (err_squared ? !(err > stopThr) : (err < stopThr)) break;
        }
    }
    niter = (ii < numItermax) ? ii : (numItermax > 0 ? numItermax - 1 : 0);
    if (P) {
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < n; ++i)
            for (int64_t j = 0; j < m; ++j) P[i * m + j] = u[i] * K[i * m + j] * v[j];
    }
    if (u_out) memcpy(u_out, u, sizeof(double) * (size_t)n);
    if (v_out) memcpy(v_out, v, sizeof(double) * (size_t)m);
    if (info) {
        info[0] = niter;
        info[1] = nupd;
        info[2] = brk;
        info[3] = nerr;
    }
    free(K);
    free(u);
    free(v);
    free(up);
    free(vp);
    free(ktu);
    free(ia);
    return brk >= 0 ? 1 : 0;
}

/* ---------------------------------------------------------------------------
 * Log-domain Sinkhorn (OTT-jax 0.6.0 lse_mode semantics as documented; OTT is
 * not installed here, so this routine is PARITY-UNPINNED):
 *   f = g = 0;  per iteration:  g_j = reg*log b_j - reg*LSE_i((f_i - C_ij)/reg)
 *                               f_i = reg*log a_i - reg*LSE_j((g_j - C_ij)/reg)
 *   every `inner` iterations: err = sum_j |sum_i P_ij - b_j|  (norm_error = 1)
 *   converged when err < threshold; P = exp((f_i + g_j - C_ij)/reg).
 * cscale multiplies C (scale_cost="max_cost" passes 1/max C).
 * info[0] = iterations run, info[1] = converged flag.
 * ------------------------------------------------------------------------- */
ORO_EXPORT void oro_sinkhorn_log(const double* a, const double* b, const double* C, int64_t n,
                                 int64_t m, double reg, double cscale, int max_iter,
                                 double threshold, int inner, double* f_out, double* g_out,
                                 double* P, int64_t* info) {
    double* f = (double*)calloc((size_t)n, sizeof(double));
    double* g = (double*)calloc((size_t)m, sizeof(double));
    int it = 0, conv = 0;
    while (it < max_iter && !conv) {
        for (int k = 0; k < inner && it < max_iter; ++k, ++it) {
#pragma omp parallel for schedule(static)
            for (int64_t j = 0; j < m; ++j) {
                double mx = -INFINITY;
                for (int64_t i = 0; i < n; ++i) {
                    const double z = (f[i] - C[i * m + j] * cscale) / reg;
                    if (z > mx) mx = z;
                }
                double s = 0.0;
                for (int64_t i = 0; i < n; ++i) s += exp((f[i] - C[i * m + j] * cscale) / reg - mx);
                g[j] = reg * log(b[j]) - reg * (mx + log(s));
            }
#pragma omp parallel for schedule(static)
            for (int64_t i = 0; i < n; ++i) {
                double mx = -INFINITY;
                for (int64_t j = 0; j < m; ++j) {
                    const double z = (g[j] - C[i * m + j] * cscale) / reg;
                    if (z > mx) mx = z;
                }
                double s = 0.0;
                for (int64_t j = 0; j < m; ++j) s += exp((g[j] - C[i * m + j] * cscale) / reg - mx);
                f[i] = reg * log(a[i]) - reg * (mx + log(s));
            }
        }
        double err = 0.0;
        for (int64_t j = 0; j < m; ++j) {
            double s = 0.0;
            for (int64_t i = 0; i < n; ++i) s += exp((f[i] + g[j] - C[i * m + j] * cscale) / reg);
            err += fabs(s - b[j]);
        }
        if (err < threshold) conv = 1;
    }
    if (P) {
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < n; ++i)
            for (int64_t j = 0; j < m; ++j)
                P[i * m + j] = exp((f[i] + g[j] - C[i * m + j] * cscale) / reg);
    }
    if (f_out) memcpy(f_out, f, sizeof(double) * (size_t)n);
    if (g_out) memcpy(g_out, g, sizeof(double) * (size_t)m);
    if (info) {
        info[0] = it;
        info[1] = conv;
    }
    free(f);
    free(g);
}

/* ---------------------------------------------------------------------------
 * Plan post-processing + apply, MRI_PET_OT_nojax.py:701-721, in float32 like
 * the reference (torch.from_numpy(T).float()):
 *   T32 = float(T); T32[isnan] = 1e-8; rs = T32.sum(1); rs[rs==0] = 1e-8;
 *   T32 /= rs;  out = Z @ T32^T      (Z: B x d2, T: d x d2, out: B x d)
 * ------------------------------------------------------------------------- */
ORO_EXPORT void oro_plan_apply(const double* T, int64_t d, int64_t d2, const float* Z, int64_t B,
                               float* Tn, float* out) {
    for (int64_t i = 0; i < d; ++i) {
        float rs = 0.0f;
        for (int64_t j = 0; j < d2; ++j) {
            float t = (float)T[i * d2 + j];
            if (isnan(t)) t = 1e-8f;
            Tn[i * d2 + j] = t;
            rs += t;
        }
        if (rs == 0.0f) rs = 1e-8f;
        for (int64_t j = 0; j < d2; ++j) Tn[i * d2 + j] = Tn[i * d2 + j] / rs;
    }
    if (!out) return;
    for (int64_t r = 0; r < B; ++r)
        for (int64_t i = 0; i < d; ++i) {
            float s = 0.0f;
            for (int64_t j = 0; j < d2; ++j) s += Z[r * d2 + j] * Tn[i * d2 + j];
            out[r * d + i] = s;
        }
}
