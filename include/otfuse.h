/*
 * otfuse.h — C ABI of the MI355X-native (gfx950) Sinkhorn OT fusion path.
 *
 * Drop-in boundary for the reference's transport-plan API.  Every entry point
 * takes caller-owned DEVICE buffers (plain pointers + sizes/leading dimensions),
 * a caller-provided workspace where needed, and the hipStream_t to enqueue on.
 * Nothing here allocates device memory or synchronises the device unless the
 * function says so.  No torch types: the Python host layer (otfuse/) binds this
 * with ctypes; a C/C++ caller links libotfuse.so directly.
 *
 * Reference interfaces replaced (file:line into the reference tree):
 *   otf_cost_pairwise      ot.dist(x, y, metric) [+ "/= max"]        MRI_PET_OT_nojax.py:70-75
 *                          PointCloud(x, y, scale_cost="max_cost")   MRI_PET_OT_OT_per_epoch_attn.py:155-156,
 *                                                                    perturbot/perturbot/match/ott_egwl.py:350
 *   otf_feature_cost       cost block of get_feature_coupling_pot    MRI_PET_OT_nojax.py:100-136
 *                          init_matrix_np / M = constC - hC1 Ts hC2^T  perturbot/perturbot/match/fot.py:118-124
 *   otf_sinkhorn           ot.sinkhorn(a, b, M, reg, numItermax, stopThr)  MRI_PET_OT_nojax.py:143
 *                          (POT sinkhorn_knopp; vendored twin perturbot/perturbot/match/utils.py:6-115)
 *                          and OTT linear.solve(Geometry(M, eps, "max_cost"))  perturbot/perturbot/match/fot.py:128-134
 *   otf_plan_postprocess   NaN->1e-8 + row normalisation            MRI_PET_OT_nojax.py:702-715
 *   otf_cosine_align       cosine_loss + gradients                   MRI_PET_OT_nojax.py:552-560,721-725
 *   otf_ot_align_backward  backward of the apply + loss scaling      MRI_PET_OT_nojax.py:718-721
 *   otf_gemm_f32           ot_mri_from_pet = pet_fused @ T^T         MRI_PET_OT_nojax.py:718,
 *                                                                    MRI_PET_OT_OT_per_epoch_attn.py:728
 *
 * Error convention: every function returns OTF_OK (0), a positive argument
 * error (OTF_EINVAL / OTF_EUNSUPPORTED) or a negative HIP error (OTF_EHIP).
 * Solver outcomes (converged / max_iter / numerical break) are reported through
 * the device-side otf_sinkhorn_info, mirroring POT's "revert to the previous
 * iterate and stop" behaviour.
 */
#ifndef OTFUSE_H_
#define OTFUSE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* otf_stream_t; /* == hipStream_t */

enum {
    OTF_OK = 0,
    OTF_EINVAL = 1,
    OTF_EUNSUPPORTED = 2,
    OTF_EHIP = -1
};

typedef enum { OTF_F32 = 0, OTF_F64 = 1, OTF_F16 = 2, OTF_BF16 = 3 } otf_dtype;
typedef enum { OTF_SQEUCLIDEAN = 0, OTF_EUCLIDEAN = 1 } otf_metric;

/* Sinkhorn flavours.
 * OTF_FLAVOR_POT: POT sinkhorn_knopp — kernel-domain scaling vectors u, v,
 *   u0 = 1/n, v0 = 1/m, v-update then u-update, numerical break (zero in K^T u,
 *   nan/inf in u or v) reverts to the previous iterate and stops, the L2
 *   marginal error is checked every `check_every` iterations against stop_thr.
 * OTF_FLAVOR_OTT: OTT-jax lse_mode — log-domain potentials f, g (returned in
 *   u_out / v_out), L1 marginal error every `check_every` iterations against
 *   stop_thr (OTT's threshold).                                                */
typedef enum { OTF_FLAVOR_POT = 0, OTF_FLAVOR_OTT = 1 } otf_flavor;

/* Status codes written to otf_sinkhorn_info.status. */
enum {
    OTF_SK_RUNNING = 0,
    OTF_SK_CONVERGED = 1,
    OTF_SK_MAX_ITER = 2,
    OTF_SK_NUMERICAL_BREAK = 3,
    OTF_SK_TIMEOUT = 4  /* persistent engine: a device-wide barrier made no progress for
                           5 s (grid not co-resident); outputs are invalid            */
};

/* Solver engines (otf_sinkhorn_opts.engine).
 * OTF_ENGINE_AUTO: tiled (float32) or resident when the problem fits the register
 *   files of the chip (one tile / row block per CU), else sweep, else streaming.
 * OTF_ENGINE_STREAM: one launch per iteration, C re-read from HBM every iteration.
 * OTF_ENGINE_RESIDENT: one persistent launch for the whole solve; every workgroup
 *   keeps its rows of K = exp(-C/reg) in registers; iterations are separated by a
 *   device-wide barrier.  POT flavour only.
 * OTF_ENGINE_TILED: resident like OTF_ENGINE_RESIDENT, float32, but every workgroup
 *   keeps a 128-row x 512-column TILE of K; the row sums are combined within groups
 *   of column tiles, the column sums across the grid (8x fewer atomics).  AUTO picks
 *   it first when ceil(n/128) * ceil(m/512) <= #CUs.
 * OTF_ENGINE_SWEEP: one persistent launch for the whole solve that streams C from
 *   HBM / the Infinity Cache once per iteration (costs too large for the register
 *   files, e.g. N = 8192 fp16 or N = 16384 fp32); one workgroup per CU owns row
 *   blocks, the column sums go through a 4-slot ring of per-iteration buffers and an
 *   XCD-hierarchical barrier.  POT flavour, m <= 16384 (float) / 8192 (double).
 * OTF_ENGINE_GATHER: small problems (ceil(n / 128) float / ceil(n / 64) double row
 *   tiles <= 16, m <= 512: the per-batch feature plans of the training loop): tiles of
 *   K in registers as in TILED, but the column partials are exchanged as epoch-tagged
 *   granules that every workgroup gathers and sums in a fixed order -- no atomics, no
 *   barrier, one memory hop per iteration, bitwise reproducible.  AUTO picks it first
 *   for such shapes (and for opts.deterministic).  POT flavour.
 * OTF_ENGINE_MESH: float32, 4..64 row tiles x 1..16 column tiles of 128 x 512 (the
 *   N = 4096 metric config; config 5's 8192 columns under otf_sinkhorn_xsweep): tiles of K in registers as in TILED, but both reductions
 *   are epoch-tagged granule hops -- row partials within the row block, column partials
 *   through one reducer workgroup per column slice -- no atomics, no barrier, three
 *   memory hops per iteration, bitwise reproducible.  AUTO picks it before TILED.
 *   float64: whole 128 x 512 tiles, 4 / 8 / 16 / 32 row blocks x 1..8 column tiles,
 *   eight waves a workgroup, K in registers + LDS (AUTO picks it for those shapes).   */
typedef enum {
    OTF_ENGINE_AUTO = 0,
    OTF_ENGINE_STREAM = 1,
    OTF_ENGINE_RESIDENT = 2,
    OTF_ENGINE_TILED = 3,
    OTF_ENGINE_SWEEP = 4,
    OTF_ENGINE_GATHER = 5,
    OTF_ENGINE_MESH = 6
} otf_engine;

typedef struct {
    double reg;         /* entropic regularisation (absolute, on the scaled cost)      */
    double stop_thr;    /* POT stopThr / OTT threshold; <= 0 runs exactly max_iter     */
    int32_t max_iter;   /* POT numItermax / OTT max_iterations                         */
    int32_t check_every;/* 10 in POT and OTT (inner_iterations)                        */
    int32_t flavor;     /* otf_flavor                                                  */
    int32_t err_squared;/* 1: compare the SQUARED L2 error (vendored utils.py:88-89)   */
    int32_t sync_every; /* streaming engine: host polls the device stop flag every N
                           iterations; 0 = never (finished passes no-op)             */
    int32_t engine;     /* otf_engine                                                  */
    int32_t cost_f16;   /* 1: C is stored as fp16 (dtype must be OTF_F32; compute fp32)  */
    int32_t n_total;    /* row-sharded solve: rows of the whole problem (u0 = 1/n_total);
                           0 = n                                                      */
    int32_t deterministic; /* 1: bitwise-reproducible column sums (fixed-order reduction,
                           no float atomics; gather, mesh or sweep engine, POT flavour),
                           e.g. for parity runs; other engines: OTF_EUNSUPPORTED     */
    int32_t shift;      /* 1: shifted kernel for float32 POT at small reg (C/reg beyond
                           float32's exp range, e.g. reg < 0.0115 on a max-normalised
                           cost): the same POT iterates computed as
                             K~_ij = 2^(C_ij*cscale*(-log2 e)/reg + A_i + B_j),
                             u = 2^A * u~,  v = 2^B * v~,  P = u~ K~ v~ = u K v,
                           A, B from a log-domain first half-iteration (one column
                           log-sum-exp pass + one row max pass over C before the solve).
                           u_out / v_out receive u~, v~; the base-2 offsets A (n), B (m)
                           stay in the workspace at otf_sinkhorn_shift_offsets().
                           Engines: mesh, sweep, stream (AUTO picks among them; forcing
                           gather / tiled / resident: OTF_EUNSUPPORTED).  float64 or OTT
                           flavour: OTF_EUNSUPPORTED.                                 */
} otf_sinkhorn_opts;

/* Written on the device by otf_sinkhorn (read it after the stream completes). */
typedef struct {
    int32_t stop;       /* 1 once converged or broken                                  */
    int32_t last_good;  /* iteration whose (u, v) are returned; -1 = initial u0, v0    */
    int32_t niter;      /* POT log['niter'] (last iteration index ii)                  */
    int32_t status;     /* OTF_SK_*                                                    */
    int32_t n_err;      /* number of entries written to the err log                    */
    int32_t break_iter; /* iteration of the numerical break, or -1                     */
    int32_t engine;     /* engine that ran (otf_engine)                                */
    int32_t stalled;    /* persistent engines: 1 if any workgroup hit the stall timeout */
    int32_t fallback;   /* 1 if the persistent engine could not become co-resident and
                           the one-workgroup fallback solved the problem instead       */
} otf_sinkhorn_info;

/* Library identification; returns a static string ("otfuse <ver> gfx950"). */
const char* otf_version(void);

/* Pairwise cost C (n x m, row stride ldc) between rows of X (n x d, ldx) and Y
 * (m x d, ldy), float32 in/out, MFMA contraction (v_mfma_f32_32x32x2_f32):
 *   C_ij = max(|x_i|^2 + |y_j|^2 - 2 x_i.y_j, 0)      [sqrt if OTF_EUCLIDEAN]
 *   C_ii = 0 if zero_diag (POT's "X is Y" case).
 * If cmax != NULL the kernel also writes max_ij C_ij to *cmax (device float,
 * zeroed by the function first): scale_cost="max_cost" / "/= C.max()" without
 * a second pass over C.  Requirements: ldx, ldy multiples of 4, 16-B aligned. */
int otf_cost_pairwise(const float* X, int64_t ldx, const float* Y, int64_t ldy, int64_t n,
                      int64_t m, int64_t d, int32_t metric, int32_t zero_diag, float* C,
                      int64_t ldc, float* cmax, otf_stream_t stream);

/* Same contract as otf_cost_pairwise, fp32-accurate at the fp16 MFMA rate: each row
 * is scaled by a power of two and split into hi + lo fp16 halves (22 significant
 * bits); X Y^T = hi.hi + hi.lo + lo.hi on v_mfma_f32_32x32x16_f16 with fp32
 * accumulation.  Workspace: otf_cost_split16_workspace_size() bytes (the hi/lo
 * images, scales and squared norms).                                            */
size_t otf_cost_split16_workspace_size(int64_t n, int64_t m, int64_t d);
int otf_cost_pairwise_split16(const float* X, int64_t ldx, const float* Y, int64_t ldy, int64_t n,
                              int64_t m, int64_t d, int32_t metric, int32_t zero_diag, float* C,
                              int64_t ldc, float* cmax, void* workspace, size_t ws_bytes,
                              otf_stream_t stream);

/* General pairwise cost (BASELINE config 5: fp16 embeddings / fp16 cost storage).
 * in_dtype OTF_F32: X, Y float32, contraction as otf_cost_pairwise_split16;
 * in_dtype OTF_F16: X, Y fp16, one v_mfma_f32_32x32x16_f16 per 16-deep step,
 *   fp32 accumulation, norms in fp32 from the fp16 values.
 * c_dtype OTF_F32: C float32 holds the cost itself (*c_unit = 1);
 * c_dtype OTF_F16: C fp16 holds cost * 2^-k, k chosen from the row norms so that
 *   every stored value is <= 1 (max C <= (max|x| + max|y|)^2, no overflow, one
 *   pass); *c_unit = 2^k (device float, nullable) recovers the cost.
 * cmax (device float, nullable) receives the max of the STORED values, i.e. the
 * cost_scale that makes otf_sinkhorn see C / max(C) ("max_cost").  Rows of X/Y:
 * ldx, ldy elements; C rows 16-B aligned when it feeds otf_sinkhorn.
 * Workspace: otf_cost_ex_workspace_size() bytes.                                 */
size_t otf_cost_ex_workspace_size(int64_t n, int64_t m, int64_t d, int32_t in_dtype);
/* Profiling: with OTF_COST_PHASES=1 in the environment every otf_cost_pairwise_ex call
 * records events around its prep (split / norms) and its cost kernel; this returns the
 * last call's two durations (synchronises on that call). */
int otf_cost_last_phases(float* prep_ms, float* kernel_ms);
int otf_cost_pairwise_ex(const void* X, int64_t ldx, const void* Y, int64_t ldy,
                         int32_t in_dtype, int64_t n, int64_t m, int64_t d, int32_t metric,
                         int32_t zero_diag, void* C, int64_t ldc, int32_t c_dtype, float* cmax,
                         float* c_unit, void* workspace, size_t ws_bytes, otf_stream_t stream);

/* Divides C (n x m, ldc) by the device scalar *s (in place).  float32/64. */
int otf_scale_inplace(void* C, int64_t n, int64_t m, int64_t ldc, int32_t dtype, const void* s,
                      otf_stream_t stream);

/* Feature cost (float64 compute, like the reference):
 *   weights_mode 0 (get_feature_coupling_pot, MRI_PET_OT_nojax.py:121-136):
 *       w1 = Ts.sum(1), w2 = Ts.sum(0)
 *   weights_mode 1 (fot_numpy + init_matrix_np, perturbot/.../fot.py:108-124,
 *       utils.py:125-184; needs n == n2):  w1 = Ts.sum(0), w2 = Ts.sum(1)
 *   t1 = (X^2)^T w1, t2 = (Y^2)^T w2,
 *   M (d x d2, ldm) = t1[:,None] + t2[None,:] - 2 X^T Ts Y
 * X: n x d float32 (ldx), Y: n2 x d2 float32 (ldy).  Ts: n x n2 float64 (ldts),
 * or NULL with ts_diag (length n == n2, float64) for a diagonal Ts such as
 * np.eye(B)/B.  Workspace: otf_feature_cost_workspace_size() bytes.           */
size_t otf_feature_cost_workspace_size(int64_t n, int64_t n2, int64_t d, int64_t d2);
int otf_feature_cost(const float* X, int64_t ldx, const float* Y, int64_t ldy, int64_t n,
                     int64_t n2, int64_t d, int64_t d2, const double* Ts, int64_t ldts,
                     const double* ts_diag, int32_t weights_mode, double* M, int64_t ldm,
                     void* workspace, size_t ws_bytes, otf_stream_t stream);

/* otf_feature_cost with the embeddings stored as in_dtype = OTF_F32, OTF_BF16 or
 * OTF_F16 (BASELINE config 4: bf16 encoder outputs).  Every element is widened
 * exactly to float32 first, so the result equals otf_feature_cost on the rounded
 * values upcast to float32 (the reference's arithmetic on such arrays).           */
int otf_feature_cost_ex(const void* X, int64_t ldx, const void* Y, int64_t ldy, int32_t in_dtype,
                        int64_t n, int64_t n2, int64_t d, int64_t d2, const double* Ts,
                        int64_t ldts, const double* ts_diag, int32_t weights_mode, double* M,
                        int64_t ldm, void* workspace, size_t ws_bytes, otf_stream_t stream);

/* COOT cost (perturbot/perturbot/match/utils.py:125-184 init_matrix_np and its uses in
 * cot_labels.py:155-160, 173, 192):
 *   M (p x q, ldm) = t1[:, None] + t2[None, :] - 2 A T B^T,
 *   t1 = (A*A) w1, t2 = (B*B) w2   (squares in float32, as X**2 on float32 data)
 * A (p x r) and B (q x s) float32 addressed by element strides (a0, a1) / (b0, b1),
 * so a transposed view is free: the sample cost of label k is (A, B, T) = (X_k, Y_k,
 * Tv) with w = (v1, v2); the feature cost is (X^T, Y^T, Ts) with w = (w1, w2).
 * T (r x s, ldt), w1 (r), w2 (s), M: float64 device.
 * Workspace: otf_coupled_cost_workspace_size(p, q, r) bytes.                    */
size_t otf_coupled_cost_workspace_size(int64_t p, int64_t q, int64_t r);
int otf_coupled_cost(const float* A, int64_t a0, int64_t a1, const float* B, int64_t b0,
                     int64_t b1, int64_t p, int64_t q, int64_t r, int64_t s, const double* T,
                     int64_t ldt, const double* w1, const double* w2, double* M, int64_t ldm,
                     void* workspace, size_t ws_bytes, otf_stream_t stream);

/* Entropic OT between histograms a (n) and b (m) with cost C (n x m, ldc), all
 * of `dtype` (float32 or float64), on the device:
 *   K = exp(-C * cscale / reg)      (cscale = 1/(*cost_scale) if cost_scale != NULL)
 * POT flavour: u_out (n), v_out (m) receive the scaling vectors, P_out (n x m,
 * ldp, optional) the plan u_i K_ij v_j.  OTT flavour: u_out, v_out receive the
 * potentials f, g and P_out = exp((f_i + g_j - C_ij*cscale)/reg).
 * info (device) receives the outcome; errlog (device float64, optional, length
 * max_iter / check_every + 1) the marginal errors.
 * opts->cost_f16 = 1: C is fp16 (e.g. from otf_cost_pairwise_ex with c_dtype
 * OTF_F16, cost_scale = its cmax), dtype OTF_F32; K is formed in fp32.
 * Layout requirements: ldc and ldp multiples of 16/sizeof(dtype) and 16-B
 * aligned rows.  Workspace: otf_sinkhorn_workspace_size() bytes.
 * Host synchronisation happens only if opts->sync_every > 0.                   */
/* Number of solves (process-wide, since load) that the one-workgroup fallback had to
 * finish because a persistent engine's grid could not become co-resident within
 * OTF_REG_MS (otf_sinkhorn_info.fallback marks the solve itself).  Synchronous.     */
int otf_sinkhorn_fallback_count(uint64_t* count);

size_t otf_sinkhorn_workspace_size(int64_t n, int64_t m, int32_t dtype, int32_t max_iter);
/* Byte offsets, inside an otf_sinkhorn workspace of this shape, of the shifted kernel's
 * float32 offsets A (n values) and B (m values, base-2 logarithms): POT's scalings are
 * u_i = 2^A_i u~_i, v_j = 2^B_j v~_j.  Written by a solve with opts.shift = 1.      */
int otf_sinkhorn_shift_offsets(int64_t n, int64_t m, int32_t dtype, int32_t max_iter,
                               size_t* off_a, size_t* off_b);
int otf_sinkhorn(const void* a, const void* b, const void* C, int64_t n, int64_t m, int64_t ldc,
                 int32_t dtype, const void* cost_scale, const otf_sinkhorn_opts* opts,
                 void* u_out, void* v_out, void* P_out, int64_t ldp, int32_t P_dtype,
                 otf_sinkhorn_info* info, double* errlog, void* workspace, size_t ws_bytes,
                 otf_stream_t stream);

/* Profiling helper for bench.py: runs the same solve as otf_sinkhorn with
 * stop_thr ignored (exactly max_iter iterations) and records a hipEvent pair
 * around every iteration pass; *avg_pass_ms receives the mean pass duration.
 * Synchronises the stream.                                                     */
int otf_sinkhorn_profile(const void* a, const void* b, const void* C, int64_t n, int64_t m,
                         int64_t ldc, int32_t dtype, const void* cost_scale,
                         const otf_sinkhorn_opts* opts, void* u_out, void* v_out,
                         otf_sinkhorn_info* info, void* workspace, size_t ws_bytes,
                         float* avg_pass_ms, otf_stream_t stream);

/* Row-sharded streaming solve (POT flavour), one pass at a time — the multi-GPU
 * form of one large coupled problem: each rank owns rows R_r of C
 * (n = |R_r| rows, a = a[R_r], b and m global, opts->n_total = total rows) and
 * runs, on its stream,
 *     for pass in 0 .. max_iter:
 *         otf_sinkhorn_pass(..., pass, &colsum, &len)   -> pass 0 also initialises
 *         all-reduce(sum) of colsum[0 .. len)            (len = m_pad + 1 values of
 *                                                          dtype: the shard's K^T u
 *                                                          partials + break count)
 *     otf_sinkhorn_finish(...)                           -> u (local rows), v, P rows
 * Every rank then takes the same stop / break decisions (they depend only on the
 * reduced sums), so the result equals otf_sinkhorn on the whole problem.  The
 * arguments and workspace must be identical in every call of one solve.         */
int otf_sinkhorn_pass(const void* a, const void* b, const void* C, int64_t n, int64_t m,
                      int64_t ldc, int32_t dtype, const void* cost_scale,
                      const otf_sinkhorn_opts* opts, int32_t pass, otf_sinkhorn_info* info,
                      double* errlog, void* workspace, size_t ws_bytes, void** colsum,
                      int64_t* colsum_len, otf_stream_t stream);
int otf_sinkhorn_finish(const void* a, const void* b, const void* C, int64_t n, int64_t m,
                        int64_t ldc, int32_t dtype, const void* cost_scale,
                        const otf_sinkhorn_opts* opts, void* u_out, void* v_out, void* P_out,
                        int64_t ldp, int32_t P_dtype, otf_sinkhorn_info* info, double* errlog,
                        void* workspace, size_t ws_bytes, otf_stream_t stream);

/* Pairwise cost + Sinkhorn in float64, fused (MRI_PET_OT_nojax.py:70-75 the cost -- POT
 * euclidean_distances of the float32 embeddings, squared, divided by its max -- and :143
 * ot.sinkhorn on it).  For the float64 mesh's shapes (n a power-of-two multiple of 128 from
 * 512 to 4096, m a multiple of 512 up to 4096, d a multiple of 16, 16-B aligned rows) the
 * cost tile of every workgroup is built on v_mfma_f64_16x16x4_f64 inside the solve's
 * launch (no n x m cost in HBM); other shapes run otf_cost_pairwise_f64 + otf_sinkhorn on
 * the workspace.  metric OTF_SQEUCLIDEAN / OTF_EUCLIDEAN; scale_max: divide by the cost's
 * max (POT's M /= M.max()), returned in *cmax_out (device, nullable) either way.  POT
 * flavour; opts as otf_sinkhorn.  The fused launch also needs a plan leading dimension
 * ldp % 4 == 0 (else the two calls run).  Workspace:
 * otf_sinkhorn_pairwise_f64_workspace_size -- it always holds the n x m float64 cost, which
 * the two-call path and the fused launch's fallback (a grid that could not become
 * co-resident) build there. */
size_t otf_sinkhorn_pairwise_f64_workspace_size(int64_t n, int64_t m, int32_t max_iter);
int otf_sinkhorn_pairwise_f64(const float* X, int64_t ldx, const float* Y, int64_t ldy, int64_t n, int64_t m,
                              int64_t d, int32_t metric, int32_t scale_max, const double* a, const double* b,
                              const otf_sinkhorn_opts* opts, double* u_out, double* v_out, void* P_out,
                              int64_t ldp, int32_t P_dtype, double* cmax_out, otf_sinkhorn_info* info,
                              double* errlog, void* workspace, size_t ws_bytes, otf_stream_t stream);

/* The same segment in float32 compute (the float32 leg of bench.py): the cost is the
 * split-fp16 one of otf_cost_pairwise_ex (x.y = hi.hi + hi.lo + lo.hi on fp16 MFMA, within
 * 1e-4 of POT's float64 plan at the metric shape), the solve the float32 POT engines'.  With
 * opts->engine == OTF_ENGINE_MESH and the float32 mesh's whole-tile shapes (n a multiple of
 * 128, m a multiple of 512 up to 4096, the tiles fitting the CUs) every workgroup of the
 * solve's launch builds its 128 x 512 cost tile in its prologue from the split-fp16 images (one
 * prep launch writes them): no n x m cost in HBM, the costs -- and so the solve -- bitwise
 * those of the two calls (otf_cost_pairwise_ex + otf_sinkhorn), which run otherwise: for AUTO
 * (the two calls measured faster at the metric shape), other shapes and opts->shift (a pass
 * over C).  a, b, u, v and *cmax_out (device, nullable) are float32; the plan float32 or
 * float64 with ldp % 4 == 0.  Workspace: otf_sinkhorn_pairwise_f32_workspace_size (it holds
 * the n x m float32 cost for the two calls and for the fallback of a grid that could not
 * become co-resident). */
size_t otf_sinkhorn_pairwise_f32_workspace_size(int64_t n, int64_t m, int64_t d, int32_t max_iter);
int otf_sinkhorn_pairwise_f32(const float* X, int64_t ldx, const float* Y, int64_t ldy, int64_t n, int64_t m,
                              int64_t d, int32_t metric, int32_t scale_max, const float* a, const float* b,
                              const otf_sinkhorn_opts* opts, float* u_out, float* v_out, void* P_out,
                              int64_t ldp, int32_t P_dtype, float* cmax_out, otf_sinkhorn_info* info,
                              double* errlog, void* workspace, size_t ws_bytes, otf_stream_t stream);

/* Cross-rank persistent sweep (BASELINE config 5 on several GPUs of one node): one
 * problem's rows sharded over world <= 8 ranks, each rank one persistent launch that
 * streams its cost rows; the m column sums are exchanged INSIDE the launch as
 * epoch-tagged granules written into every rank's exchange buffer over xGMI (no RCCL
 * call, no host round trip per iteration).  Replaces the per-iteration all-reduce of
 * otf_sinkhorn_row_sharded (MRI_PET_OT_OT_per_epoch_attn.py:940-960 generalised).
 * Setup per rank: otf_xpeer_create (allocates this rank's exchange buffer, returns
 * its IPC handle, otf_xpeer_handle_size() bytes), exchange the handles (any
 * all-gather, rank order), otf_xpeer_connect.  Every rank then makes the SAME sequence
 * of otf_sinkhorn_xsweep calls (the exchange's epochs advance in lock-step); the grids
 * of all ranks must run concurrently.  float32 compute (fp32 or fp16 cost: opts.cost_f16),
 * POT flavour; opts.n_total = rows over all ranks; u / plan: this rank's rows, v: all.
 * opts.engine AUTO or MESH: when the rank's slab fits the register files (m a multiple
 * of 512, <= 16 column tiles of 512, row tiles x column tiles <= the CUs) the launch is
 * the register-resident mesh engine whose reducers do the exchange ("xmesh"); else (or
 * with OTF_ENGINE_SWEEP) the streaming sweep engine.  Both take POT's decisions at the
 * same iteration on every rank.
 * A stall (a rank that never launches) ends in OTF_SK_TIMEOUT + info.stalled. */
typedef struct otf_xpeer otf_xpeer;
size_t otf_xpeer_handle_size(void);
int otf_xpeer_create(int32_t rank, int32_t world, int64_t m, otf_xpeer** out, void* handle_out);
int otf_xpeer_connect(otf_xpeer* x, const void* handles);
/* Synchronises the device, unmaps the peers' buffers and frees this rank's.  Every rank
 * must have finished ALL its xsweep solves on this exchange first (e.g. a barrier across
 * the ranks after a device sync): a peer's grid still running would store into the freed
 * buffer. */
int otf_xpeer_destroy(otf_xpeer* x);
int otf_sinkhorn_xsweep(const void* a, const void* b, const void* C, int64_t n, int64_t m,
                        int64_t ldc, int32_t dtype, const void* cost_scale,
                        const otf_sinkhorn_opts* opts, otf_xpeer* x, void* u_out, void* v_out,
                        void* P_out, int64_t ldp, int32_t P_dtype, otf_sinkhorn_info* info,
                        double* errlog, void* workspace, size_t ws_bytes, otf_stream_t stream);

/* ---------------------------------------------------------------------------
 * RCCL communicator.  The reference has no collectives; these
 * carry the path's two exchanges: the all-gather of per-epoch embedding shards
 * (MRI_PET_OT_OT_per_epoch_attn.py:940-960 run data-parallel) and the per-iteration
 * all-reduce of the row-sharded Sinkhorn's column sums.  One process per GPU, one
 * rank each; RCCL is resolved at run time from the copy already loaded in the
 * process (PyTorch's "nccl" backend), so both share one RCCL instance.
 *   rank 0: otf_comm_unique_id(id); share the 128 id bytes (e.g. torch broadcast);
 *   every rank: otf_comm_init(&comm, id, nranks, rank) with its device current.
 * Collectives are enqueued on `stream` (stream-ordered, no host sync).
 * ------------------------------------------------------------------------- */
typedef struct otf_comm otf_comm;
enum { OTF_RED_SUM = 0, OTF_RED_MAX = 1 };
#define OTF_COMM_ID_BYTES 128

int otf_comm_unique_id(void* id_out);
int otf_comm_init(otf_comm** comm_out, const void* id, int32_t nranks, int32_t rank);
int otf_comm_destroy(otf_comm* comm);
/* In-place all-reduce of count elements (dtype OTF_F32/F64/F16/BF16, op OTF_RED_*). */
int otf_comm_all_reduce(void* buf, int64_t count, int32_t dtype, int32_t op, otf_comm* comm,
                        otf_stream_t stream);
/* recv = concat over ranks of send (count_per_rank elements each), rank order.     */
int otf_comm_all_gather(const void* send, void* recv, int64_t count_per_rank, int32_t dtype,
                        otf_comm* comm, otf_stream_t stream);

/* The whole row-sharded solve in one call: otf_sinkhorn_pass for every pass, each
 * followed by the RCCL all-reduce(sum) of its column-sum buffer on the same stream,
 * then otf_sinkhorn_finish — no host round trip per iteration (finished passes are
 * device-side no-ops).  Same arguments as the pass / finish pair; opts.n_total = rows
 * of the whole problem.  comm = NULL runs the single-rank solve through the same path. */
int otf_sinkhorn_row_sharded(const void* a, const void* b, const void* C, int64_t n, int64_t m,
                             int64_t ldc, int32_t dtype, const void* cost_scale,
                             const otf_sinkhorn_opts* opts, otf_comm* comm, void* u_out,
                             void* v_out, void* P_out, int64_t ldp, int32_t P_dtype,
                             otf_sinkhorn_info* info, double* errlog, void* workspace,
                             size_t ws_bytes, otf_stream_t stream);

/* Plan post-processing (MRI_PET_OT_nojax.py:702-715): T (d x d2, ldt, dtype
 * float32/64) -> Tn float32 (ldtn): NaN -> nan_fill, row sums (0 -> 1e-8),
 * Tn = T / rowsum.  rownorm = 0 only converts + fills.                          */
int otf_plan_postprocess(const void* T, int64_t d, int64_t d2, int64_t ldt, int32_t dtype,
                         float nan_fill, int32_t rownorm, float* Tn, int64_t ldtn,
                         otf_stream_t stream);

/* Fused post-process + apply (MRI_PET_OT_nojax.py:702-718) in ONE pass over the plan:
 * out (B x d, ldo) = Z (B x d2, ldz, float32: pet_fused) @ Tn^T with Tn the
 * post-processed plan (NaN -> nan_fill, rows / rowsum, 0 -> 1e-8); Tn (d x d2,
 * ldtn, nullable) is also written for the backward G @ Tn.                        */
int otf_plan_postprocess_apply(const void* T, int64_t d, int64_t d2, int64_t ldt, int32_t dtype,
                               float nan_fill, int32_t rownorm, const float* Z, int64_t ldz,
                               int64_t B, float* out, int64_t ldo, float* Tn, int64_t ldtn,
                               otf_stream_t stream);

/* The training-time alignment loss of one batch and its gradients, one launch
 * (cosine_loss MRI_PET_OT_nojax.py:552-560 applied at :721, NaN -> 0 at :724-725):
 * loss = 1 - mean_b cos(normalize(X_b), normalize(Y_b)) with torch's normalize /
 * cosine_similarity clamps; gx = dloss/dX, gy = dloss/dY (B x d float32).  X is
 * x_dtype OTF_F32 / OTF_BF16 / OTF_F16 (the encoder output as stored), Y float32.
 * keep = (ok == NULL || *ok) && (sk_info == NULL || the solve finished: status neither
 * RUNNING nor TIMEOUT, stop set, not stalled) && loss finite; when keep is 0 the loss
 * and both gradients are exact zeros.  sk_info (device, nullable) is the
 * otf_sinkhorn_info of the solve whose plan made Y: the check runs in this launch.
 * keep_out (device uint8, nullable) receives keep.  B <= 1024.                    */
int otf_cosine_align(const void* X, int64_t ldx, int32_t x_dtype, const float* Y, int64_t ldy,
                     int64_t B, int64_t d, const uint8_t* ok, const otf_sinkhorn_info* sk_info,
                     float* loss, float* gx, int64_t ldgx, float* gy, int64_t ldgy, uint8_t* keep_out,
                     otf_stream_t stream);

/* Backward of ot_mri_from_pet = pet @ Tn^T under the alignment loss, one launch:
 * g_pet = (g_loss * gy + g_ot) @ Tn (B x d2), g_mri = g_loss * gx (B x d).  g_loss
 * (device float), g_ot (B x d, ldgo) and keep (device uint8) are nullable; without
 * g_ot and with *keep == 0, g_pet is written as zeros (Tn may hold NaN).          */
int otf_ot_align_backward(const float* gx, int64_t ldgx, const float* gy, int64_t ldgy,
                          const float* g_ot, int64_t ldgo, const float* g_loss, const uint8_t* keep,
                          const float* Tn, int64_t ldt, int64_t B, int64_t d, int64_t d2, float* g_mri,
                          int64_t ldm, float* g_pet, int64_t ldp, otf_stream_t stream);

/* out (M x N, ldo) = alpha * op(A) op(B) (+ beta * out), float32, where
 * op(A)_{ik} = A[i*sa0 + k*sa1] and op(B)_{kj} = B[k*sb0 + j*sb1]: the plan
 * application Z @ T^T and its backward G @ T.                                  */
int otf_gemm_f32(const float* A, int64_t sa0, int64_t sa1, const float* B, int64_t sb0,
                 int64_t sb1, float* out, int64_t ldo, int64_t M, int64_t N, int64_t K,
                 float alpha, float beta, otf_stream_t stream);

/* ------------------------------------------------------------------------
 * Sample-level costs and Gromov-Wasserstein couplings.
 * ---------------------------------------------------------------------- */

/* float64 pairwise cost between float32 rows, POT euclidean_distances order
 * (C = -2 X Y^T + |x|^2 + |y|^2, clamped at 0, sqrt for OTF_EUCLIDEAN, zero
 * diagonal if zero_diag) — ot.dist(x, x, metric) at MRI_PET_OT_nojax.py:70-71
 * and PointCloud(x, x) at MRI_PET_OT_OT_per_epoch_attn.py:155-156.  *cmax
 * (device double, nullable) receives max C; scale_max = 1 also divides C by it
 * ("C1 /= C1.max()", :74-75; scale_cost="max_cost").
 * Workspace: otf_cost_pairwise_f64_workspace_size() bytes.                      */
size_t otf_cost_pairwise_f64_workspace_size(int64_t n, int64_t m);
int otf_cost_pairwise_f64(const float* X, int64_t ldx, const float* Y, int64_t ldy, int64_t n,
                          int64_t m, int64_t d, int32_t metric, int32_t zero_diag,
                          int32_t scale_max, double* C, int64_t ldc, double* cmax,
                          void* workspace, size_t ws_bytes, otf_stream_t stream);

/* GW solvers (square loss, symmetric C1 / C2):
 * OTF_GW_CG: POT 0.9.6 ot.gromov.gromov_wasserstein(C1, C2, p, q, 'square_loss')
 *   (conditional gradient, exact EMD inner solve, closed-form line search), as
 *   called by get_coupling_gromov_pot, MRI_PET_OT_nojax.py:52-88.  Requires
 *   p = q = uniform (pass NULL) and n == m — the callers' paired per-label groups
 *   — where the exact EMD is an optimal assignment (solved on the device).
 * OTF_GW_ENTROPIC: OTT-jax 0.6.0 GromovWasserstein(epsilon, linear_solver=
 *   Sinkhorn(...)) as called by get_coupling_egw_ott_fixed,
 *   MRI_PET_OT_OT_per_epoch_attn.py:129-186, and perturbot ott_egwl.py:25-296
 *   (labels_a / labels_b != NULL: coupling restricted to equal labels).
 * OTF_GW_PGD: POT 0.9.6 ot.gromov.entropic_gromov_wasserstein(C1, C2, p, q,
 *   'square_loss', epsilon, solver='PGD') as called by perturbot/perturbot/match/
 *   gw.py:31-59 (egw_pgd) and :80-102 (egw_all): sinkhorn_knopp inner solves on the
 *   gradient 2 (constC - 2 C1 T C2); opts: max_iter (1000), tol_abs = tol (1e-9),
 *   eps, sk_max_iter = numItermax (1000), sk_threshold = stopThr (1e-9), sk_inner =
 *   the inner error-check period (10); costlog = log['err'] (every 10th iteration),
 *   info.cost = log['gw_dist'].                                                   */
typedef enum { OTF_GW_CG = 0, OTF_GW_ENTROPIC = 1, OTF_GW_PGD = 2 } otf_gw_solver;
enum {
    OTF_GW_RUNNING = 0,
    OTF_GW_CONVERGED = 1,
    OTF_GW_MAX_ITER = 2,
    OTF_GW_NUMERICAL = 3,  /* non-finite cost / failed assignment                   */
    OTF_GW_TIMEOUT = 4     /* no outer iteration completed within 20 s (a stall)    */
};

typedef struct {
    int32_t solver;       /* otf_gw_solver                                              */
    int32_t max_iter;     /* POT max_iter (1e4) / OTT max_iterations                     */
    int32_t min_iter;     /* OTT min_iterations (5); CG ignores it                       */
    int32_t sk_max_iter;  /* OTT inner Sinkhorn max_iterations (2000)                    */
    int32_t sk_inner;     /* OTT inner_iterations (10)                                   */
    int32_t warm_start;   /* OTT warm_start (1: inner solves start from the previous f, g) */
    double tol_rel;       /* POT tol_rel (1e-9)                                          */
    double tol_abs;       /* POT tol_abs (1e-9)                                          */
    double threshold;     /* OTT outer threshold (1e-3, rtol of isclose on the costs)    */
    double sk_threshold;  /* OTT Sinkhorn threshold (1e-3, L1 column-marginal error)     */
    double eps;           /* OTT epsilon (absolute, on the max-scaled costs)              */
} otf_gw_opts;

/* One problem; all pointers are device pointers.  T (n x m, ldt) receives the
 * coupling.  p, q: marginals (float64) or NULL for uniform.                    */
typedef struct {
    const double* C1;
    int64_t ldc1;
    const double* C2;
    int64_t ldc2;
    const double* p;
    const double* q;
    const int32_t* labels_a;
    const int32_t* labels_b;
    double* T;
    int64_t ldt;
    int64_t n;  /* <= 1024 */
    int64_t m;  /* <= 1024 */
} otf_gw_problem;

/* Written on the device, one per problem. */
typedef struct {
    int32_t n_iter;          /* outer iterations (POT CG iterations / OTT n_iters)       */
    int32_t converged;       /* outer convergence (POT tolerance hit / OTT out.converged) */
    int32_t inner_converged; /* OTT: last linear solve converged                          */
    int32_t status;          /* OTF_GW_*                                                  */
    int32_t inner_iters;     /* OTT: total Sinkhorn updates                               */
    int32_t pad;
    double cost;             /* POT: final GW loss (log['gw_dist']); OTT: reg_gw_cost     */
} otf_gw_info;

/* Solves nprob independent problems (one workgroup each, concurrently).
 * probs: HOST array of descriptors; info: device array of nprob; costlog
 * (device, nullable): nprob rows of costlog_len doubles — POT log['loss'] /
 * OTT out.costs.  Workspace: otf_gw_workspace_size() bytes.                    */
size_t otf_gw_workspace_size(int32_t nprob, const otf_gw_problem* probs);
int otf_gw_solve(int32_t nprob, const otf_gw_problem* probs, const otf_gw_opts* opts,
                 otf_gw_info* info, double* costlog, int32_t costlog_len, void* workspace,
                 size_t ws_bytes, otf_stream_t stream);

/* ---- exact EMD, general marginals: pot.emd(a, b, M, numItermax)
 * (perturbot/perturbot/match/cot_labels.py:178,195 in get_coupling_cotl :228-276;
 * the linear step of CG-GW on weighted groups, MRI_PET_OT_nojax.py:80-82).
 * Primal network simplex on the device, one workgroup per problem.  a and b are
 * non-negative with equal sums (the caller rescales b, as POT does).            */
enum {
    OTF_EMD_OPTIMAL = 0,
    OTF_EMD_MAX_ITER = 1,   /* numItermax pivots reached (POT: "numItermax reached")    */
    OTF_EMD_INFEASIBLE = 2, /* artificial flow left (unequal masses)                   */
    OTF_EMD_UNBOUNDED = 3
};

/* One problem; all pointers are device pointers (float64). */
typedef struct {
    const double* a;  /* (n) source masses                                          */
    const double* b;  /* (m) target masses                                          */
    const double* M;  /* (n x m) costs, row stride ldm                              */
    int64_t ldm;
    double* T;        /* (n x m) optimal plan out, row stride ldt                    */
    int64_t ldt;
    int32_t n;
    int32_t m;        /* n + m + 1 <= otf_emd_max_nodes(), n * m + n + m < 2^31       */
} otf_emd_problem;

/* Written on the device, one per problem. */
typedef struct {
    double cost;                /* sum T * M                                          */
    int32_t status;             /* OTF_EMD_*                                           */
    int32_t n_pivots;
    double max_artificial_flow; /* 0 at a feasible optimum                              */
} otf_emd_info;

/* Largest n + m + 1 (n * m + n + m < 2^31 also holds).  Up to otf_emd_lds_nodes()
 * the spanning tree lives in LDS; larger problems keep it in global memory (stream-
 * ordered allocation inside otf_emd_solve), same pivots. */
int otf_emd_max_nodes(void);
int otf_emd_lds_nodes(void);
/* probs: HOST array of nprob descriptors; info: device array of nprob. */
int otf_emd_solve(int32_t nprob, const otf_emd_problem* probs, int64_t max_pivots,
                  otf_emd_info* info, otf_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* OTFUSE_H_ */
