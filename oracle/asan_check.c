/* asan_check.c -- test infrastructure: drives every oracle entry point (otoracle.c,
 * otoracle_gw.c) on small ragged shapes in a binary built with
 * -fsanitize=address,undefined (oracle/Makefile target `asan`, run by
 * tests/test_sanitizers.py).  Any out-of-bounds access, use-after-free, leak or UB in
 * the oracle aborts the run; the checks below only confirm that the calls did their
 * job (marginals of the plans, finite costs), the numerical parity is pinned elsewhere
 * (tests/test_oracle_golden.py). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

double oro_pairwise_cost(const double* X, const double* Y, int64_t n, int64_t m, int64_t d,
                         int euclidean, int zero_diag, int scale_max, double* C);
void oro_feature_cost(const double* X, const double* Y, const double* Ts, int64_t n, int64_t n2,
                      int64_t d, int64_t d2, int sq_f32, int fot_weights, double* M);
int oro_sinkhorn_knopp(const double* a, const double* b, const double* C, int64_t n, int64_t m,
                       double reg, double cscale, int numItermax, double stopThr, int check_every,
                       int err_squared, double* u_out, double* v_out, double* P, int64_t* info,
                       double* errlog);
void oro_sinkhorn_log(const double* a, const double* b, const double* C, int64_t n, int64_t m,
                      double reg, double cscale, int max_iter, double threshold, int inner,
                      double* f_out, double* g_out, double* P, int64_t* info);
void oro_plan_apply(const double* T, int64_t d, int64_t d2, const float* Z, int64_t B, float* Tn,
                    float* out);
int oro_lap(const double* A, int64_t n, int* sigma);
int oro_gw_cg(const double* C1, const double* C2, int64_t n, int max_iter, double tol_rel,
              double tol_abs, double* G, double* costlog, int costlog_len, int64_t* info,
              double* cost_out);
int oro_gw_entropic(const double* C1, const double* C2, int64_t n, int64_t m, const double* a,
                    const double* b, const int* la, const int* lb, double eps, int max_iter,
                    int min_iter, double threshold, int sk_max, int sk_inner, double sk_thr, int warm,
                    double* P, double* costlog, int costlog_len, int64_t* info, double* cost_out);
int oro_gw_pgd(const double* C1, const double* C2, int64_t n, int64_t m, const double* a,
               const double* b, double eps, int max_iter, double tol, int sk_max, double sk_thr,
               double* T, double* errlog, int errlog_len, int64_t* info, double* cost_out);
int oro_set_threads(int n);

static int failures = 0;
#define CHECK(cond, ...)                                              \
    do {                                                              \
        if (!(cond)) {                                                \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);      \
            fprintf(stderr, __VA_ARGS__);                             \
            fprintf(stderr, "\n");                                    \
            ++failures;                                               \
        }                                                             \
    } while (0)

static uint64_t rng = 88172645463325252ull;
static double urand(void) {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (double)(rng >> 11) / 9007199254740992.0;
}
static double* arr(int64_t k) {
    double* p = (double*)malloc(sizeof(double) * (size_t)(k > 0 ? k : 1));
    for (int64_t i = 0; i < k; ++i) p[i] = urand();
    return p;
}
static double* unif(int64_t k) {
    double* p = (double*)malloc(sizeof(double) * (size_t)k);
    for (int64_t i = 0; i < k; ++i) p[i] = 1.0 / (double)k;
    return p;
}

/* pairwise cost -> POT sinkhorn (+ plan marginals) -> OTT log sinkhorn -> plan apply */
static void linear_path(int64_t n, int64_t m, int64_t d) {
    double *X = arr(n * d), *Y = arr(m * d), *C = arr(n * m);
    const double mx = oro_pairwise_cost(X, Y, n, m, d, 0, 0, 1, C);
    CHECK(isfinite(mx) && mx >= 0, "pairwise max %g", mx);
    double *a = unif(n), *b = unif(m), *u = arr(n), *v = arr(m), *P = arr(n * m);
    double errlog[64];
    int64_t info[4];
    oro_sinkhorn_knopp(a, b, C, n, m, 0.1, 1.0, 300, 1e-9, 10, 0, u, v, P, info, errlog);
    for (int64_t i = 0; i < n; ++i) {
        double s = 0;
        for (int64_t j = 0; j < m; ++j) s += P[i * m + j];
        CHECK(fabs(s - a[i]) < 1e-6, "POT row marginal %lld: %g vs %g", (long long)i, s, a[i]);
    }
    double *f = arr(n), *g = arr(m);
    int64_t li[2];
    oro_sinkhorn_log(a, b, C, n, m, 0.1, 1.0, 500, 1e-6, 10, f, g, P, li);
    for (int64_t j = 0; j < m; ++j) {
        double s = 0;
        for (int64_t i = 0; i < n; ++i) s += P[i * m + j];
        CHECK(fabs(s - b[j]) < 1e-4, "OTT column marginal %lld: %g", (long long)j, s);
    }
    /* feature cost with a dense Ts (n x n) on d x d features, both weight modes */
    double *Ts = arr(n * n), *M = arr(d * d), *Xf = arr(n * d), *Yf = arr(n * d);
    for (int w = 0; w < 2; ++w) {
        oro_feature_cost(Xf, Yf, Ts, n, n, d, d, w, w, M);
        for (int64_t k = 0; k < d * d; ++k) CHECK(isfinite(M[k]), "feature cost not finite");
    }
    /* plan post-process + apply: T (n x m) rows normalised, Z (3 x m) */
    float *Z = (float*)malloc(sizeof(float) * 3 * (size_t)m), *Tn = (float*)malloc(sizeof(float) * (size_t)(n * m));
    float* out = (float*)malloc(sizeof(float) * 3 * (size_t)n);
    for (int64_t k = 0; k < 3 * m; ++k) Z[k] = (float)urand();
    oro_plan_apply(P, n, m, Z, 3, Tn, out);
    for (int64_t k = 0; k < 3 * n; ++k) CHECK(isfinite(out[k]), "plan apply not finite");
    free(X); free(Y); free(C); free(a); free(b); free(u); free(v); free(P); free(f); free(g);
    free(Ts); free(M); free(Xf); free(Yf); free(Z); free(Tn); free(out);
}

/* a numerical break: a column of K underflows (K^T u = 0 at iteration 0) */
static void break_path(void) {
    const int64_t n = 6, m = 4;
    double *C = arr(n * m), *a = unif(n), *b = unif(m), *u = arr(n), *v = arr(m), *P = arr(n * m);
    for (int64_t i = 0; i < n; ++i) C[i * m + 2] = 1e4;
    double errlog[8];
    int64_t info[4];
    oro_sinkhorn_knopp(a, b, C, n, m, 1.0, 1.0, 50, 0.0, 10, 1, u, v, P, info, errlog);
    CHECK(info[2] == 0, "break at iteration %lld, expected 0", (long long)info[2]);
    free(C); free(a); free(b); free(u); free(v); free(P);
}

static double* dist_matrix(int64_t n) {
    double* pts = arr(2 * n);
    double* D = (double*)malloc(sizeof(double) * (size_t)(n * n));
    for (int64_t i = 0; i < n; ++i)
        for (int64_t j = 0; j < n; ++j) {
            const double dx = pts[2 * i] - pts[2 * j], dy = pts[2 * i + 1] - pts[2 * j + 1];
            D[i * n + j] = dx * dx + dy * dy;
        }
    free(pts);
    return D;
}

static void gw_path(int64_t n, int64_t m) {
    double *C1 = dist_matrix(n), *C2 = dist_matrix(m);
    /* assignment */
    int* sigma = (int*)malloc(sizeof(int) * (size_t)n);
    CHECK(oro_lap(C1, n, sigma) == 0, "lap");
    int* seen = (int*)calloc((size_t)n, sizeof(int));
    for (int64_t i = 0; i < n; ++i) {
        CHECK(sigma[i] >= 0 && sigma[i] < n, "lap index");
        if (sigma[i] >= 0 && sigma[i] < n) seen[sigma[i]]++;
    }
    for (int64_t i = 0; i < n; ++i) CHECK(seen[i] == 1, "lap is not a permutation");
    /* CG-GW on n x n */
    double *C2n = dist_matrix(n), *G = arr(n * n), clog[32], cost = 0;
    int64_t info[5];
    oro_gw_cg(C1, C2n, n, 200, 1e-9, 1e-9, G, clog, 32, info, &cost);
    CHECK(isfinite(cost), "gw_cg cost");
    /* entropic GW (OTT), with labels, ragged n x m */
    int *la = (int*)malloc(sizeof(int) * (size_t)n), *lb = (int*)malloc(sizeof(int) * (size_t)m);
    for (int64_t i = 0; i < n; ++i) la[i] = (int)(i % 2);
    for (int64_t j = 0; j < m; ++j) lb[j] = (int)(j % 2);
    double *P = arr(n * m), elog[64];
    oro_gw_entropic(C1, C2, n, m, NULL, NULL, NULL, NULL, 0.05, 50, 5, 1e-3, 200, 10, 1e-3, 1, P,
                    elog, 64, info, &cost);
    CHECK(isfinite(cost), "gw_entropic cost");
    oro_gw_entropic(C1, C2, n, m, NULL, NULL, la, lb, 0.05, 50, 5, 1e-3, 200, 10, 1e-3, 0, P, elog,
                    64, info, &cost);
    CHECK(isfinite(cost), "gw_entropic labelled cost");
    /* POT entropic GW (PGD) */
    double *pa = unif(n), *qb = unif(m);
    oro_gw_pgd(C1, C2, n, m, pa, qb, 0.05, 20, 1e-9, 200, 1e-9, P, elog, 64, info, &cost);
    CHECK(isfinite(cost), "gw_pgd cost");
    free(C1); free(C2); free(sigma); free(seen); free(C2n); free(G); free(la); free(lb); free(P);
    free(pa); free(qb);
}

int main(void) {
    oro_set_threads(2);
    const int64_t shapes[][3] = {{1, 1, 1}, {7, 5, 3}, {33, 17, 8}, {64, 64, 16}, {5, 40, 2}};
    for (size_t s = 0; s < sizeof(shapes) / sizeof(shapes[0]); ++s)
        linear_path(shapes[s][0], shapes[s][1], shapes[s][2]);
    break_path();
    gw_path(9, 7);
    gw_path(16, 16);
    if (failures) {
        fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    printf("asan_check: all oracle entry points clean\n");
    return 0;
}
