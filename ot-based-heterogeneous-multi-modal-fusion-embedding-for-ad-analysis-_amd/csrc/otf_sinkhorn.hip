// otf_sinkhorn.hip — entropic Sinkhorn on gfx950 as fused single-read HBM sweeps.
//
// Replaces ot.sinkhorn (POT 0.9.6 sinkhorn_knopp) at MRI_PET_OT_nojax.py:143 and the
// vendored loop perturbot/perturbot/match/utils.py:6-115 (POT flavour), and OTT's
// lse-mode Sinkhorn behind perturbot/perturbot/match/fot.py:128-134 (OTT flavour).
//
// One launch = one Sinkhorn iteration = ONE read of the materialised cost C.
// Workgroup w owns blocks of R rows and ALL m columns; a row block's K values stay
// in registers between
//   (1) the row reduction with the current column scaling -> the new row scaling
//       (exact POT order: v-update first, then u-update), and
//   (2) the column update with the NEW row scaling, flushed with one float atomic
//       per column per workgroup: that is K^T u for the NEXT iteration's v-update,
//       and v_j (K^T u)_j is POT's marginal-error term, so the err check is free.
// K = exp(-C/reg) is recomputed from C in registers (one v_exp per element), so
// only C is streamed.  Both flavours run the same pass:
//   e_ij = exp(C_ij * ks + fo_i + go_j)
//   POT: fo = go = 0, row sums weighted by v_j = b_j / colsum_j, w_i = u_i = a_i / rowsum_i
//   OTT: e_ij = exp((f_prev_i + g_j - C_ij)/reg) with g_j = reg (log b_j - log colsum_j)
//        + g_prev_j; rows unweighted, w_i = a_i / rowsum_i, f_i = reg log w_i + f_prev_i.
//        Every e_ij <= 1 by construction (the previous update normalised that
//        marginal), so the shifted sums never overflow — a log-sum-exp without a
//        max pass.  The first g-update is shifted by the column minima of C.
// Control (marginal error every check_every iterations, POT's revert-and-break on
// zero / nan / inf) lives on the device: every workgroup re-derives the same
// decision from the same buffers at the top of the next launch, so no host sync
// is needed between iterations.  Column-sum buffers are triple-buffered
// (read p-1, accumulate p, zero p+1) so a pass never races the zeroing.
#include <stdlib.h>

#include <string.h>

#include "otf_persist.h"
#include <type_traits>
#include "otf_comm.h"

namespace otf {
namespace {

template <typename T> struct SkArgs {
    const void* C;         // cost, element type CT (T, or fp16 storage with fp32 compute)
    int64_t ldc;
    int n, m;
    int n_total;           // rows of the whole problem (u0 = 1/n_total; > n when row-sharded)
    const T* a;            // padded copy (workspace)
    const T* b;            // padded copy, zero beyond m (workspace)
    const T* cost_scale;   // device scalar; cost is C / cost_scale (nullable)
    double reg;
    int it;                // iteration index ii; -1 = prologue pass
    // column-sum buffers, m_pad + 1 wide: [0, m) sums K^T u, [m_pad] number of rows
    // whose scaling in that iteration is not finite (one buffer = one all-reduce in
    // the row-sharded solve)
    const T* cs_src;       // accumulated by the previous pass
    T* cs_dst;             // accumulated by this pass
    T* cs_zero;            // zeroed by this pass (accumulated by the next)
    T* u_cur;              // u (POT) / f (OTT) of iteration it
    T* v_cur;              // v / g of iteration it
    const T* u_prev;       // f of iteration it-1 (OTT)
    const T* v_prev;       // v / g of iteration it-1
    const int* cmin_key;   // OTT prologue: ordered-int column minima of C
    otf_sinkhorn_info* info;
    double* errlog;
    double stop_thr;
    int check_every;
    int check_off;         // POT checks at ii % 10 == 0, OTT after every 10th update
    int err_squared;
    int m_pad;
    // shifted POT kernel (opts.shift, float): K~_ij = exp2(C_ij ks + shA_i + shB_j), the
    // scalings start from u0v (u~0 = 2^-shA / n); null otherwise
    const T* shA;
    const T* shB;
    const T* u0v;
    const T* v0v;          // v~0 = 2^-shB / m (the initial iterate POT reverts to)
};

__device__ __forceinline__ void sk_stop(otf_sinkhorn_info* info, int last_good, int niter,
                                        int status, int break_iter) {
    info->last_good = last_good;
    info->niter = niter;
    info->status = status;
    if (break_iter >= 0) info->break_iter = break_iter;
    __hip_atomic_store(&info->stop, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The relay fallback's counters (sk_relay_kernel), ints in a workspace region zeroed by the
// init kernel: the ticket, the cost build's max (float64 bits), the abort word, and the
// completion count as 8 shards 256 B apart (a piece adds to shard blockIdx % 8, a waiter sums
// them: 32 instead of 256 arrivals on one word per pass)
constexpr int kRelayTicket = 0, kRelayMax = 16, kRelayAbort = 32, kRelayDone = 64, kRelayDoneStride = 64,
              kRelayShards = 8, kRelayInts = kRelayDone + kRelayShards * kRelayDoneStride;

// ordered int key of a float (monotone), for atomicMin on signed ints
__device__ __forceinline__ int ord_key(float x) {
    const int b = __float_as_int(x);
    return b >= 0 ? b : b ^ 0x7fffffff;
}
__device__ __forceinline__ float key_val(int k) {
    return __int_as_float(k >= 0 ? k : k ^ 0x7fffffff);
}

template <typename T> __device__ __forceinline__ T unit_log(T x);
template <> __device__ __forceinline__ float unit_log(float x) { return __builtin_amdgcn_logf(x); }   // log2
template <> __device__ __forceinline__ double unit_log(double x) { return log(x); }

template <typename T> __device__ __forceinline__ bool check_now(const SkArgs<T>& p, int it) {
    return ((it + p.check_off) % p.check_every) == 0;
}

template <typename T>
__device__ __forceinline__ bool is_conv(const SkArgs<T>& p, double err) {
    return p.err_squared ? !(err > p.stop_thr) : (err < p.stop_thr);
}

// Marginal error of iteration `it` from its column scaling and the column sums
// accumulated with its row scaling.  Block-wide, identical in every workgroup.
template <typename T, bool LOG, int G, int VEC>
__device__ __forceinline__ double marginal_err(const SkArgs<T>& p, const T* vit, const T* cs,
                                               const int (&colc)[G], const bool (&cok)[G][VEC],
                                               T* red) {
    using V = typename Vec<T>::type;
    T e = 0;
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const V s = *reinterpret_cast<const V*>(cs + colc[g]);
        const V bb = *reinterpret_cast<const V*>(p.b + colc[g]);
        V vv = *reinterpret_cast<const V*>(vit + colc[g]);
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            T r;
            if (LOG) {
                r = fabs(s[k] - bb[k]);
            } else {
                r = vv[k] * s[k] - bb[k];
                r = r * r;
            }
            e += cok[g][k] ? r : (T)0;
        }
    }
    e = block_sum<T>(e, red);
    if (LOG) return (double)e;
    return p.err_squared ? (double)e : sqrt((double)e);
}

// One fused Sinkhorn pass.  NT threads own G chunks of VEC contiguous columns each
// (chunk q = tid + NT*g), R rows per row block; K values for a row block stay in
// registers (R*G*VEC of them) between the row reduction and the column update.
// vb / vg: this workgroup's place in the pass (blockIdx.x / gridDim.x of a pass launch, a
// piece of the relay fallback's ticket sequence otherwise).  KIN: the array holds K itself
// (the relay fallback's K written once), no exp per element.
// RELAY (a piece of sk_relay_kernel): `wait` is the piece's dependency wait (poll + acquire +
// barrier, false on abort), run by the body after the first row block's loads are issued when
// `early` (the array is K, complete and L1-fresh since this workgroup's last acquire, or the
// caller's C: its rows stream during the wait; a second row block in flight measured as
// 45-330 spilled VGPRs); scalings and the zeroed sums are stored write-through (sc1) so that
// only the piece that writes the info words needs an agent release.
struct NoWait {
    __device__ bool operator()() const { return true; }
};
template <typename T, typename CT, bool LOG, int G, int R, bool SH = false, bool KIN = false, bool RELAY = false,
          typename WaitFn = NoWait>
__device__ __forceinline__ void sk_pass_body(const SkArgs<T>& p, int vb, int vg, const WaitFn& wait = WaitFn{},
                                             bool early = false) {
    static_assert(!(LOG && SH), "the shifted kernel is a POT-flavour form");
    static_assert(!(KIN && (LOG || SH)), "K input: the plain POT kernel only");
    constexpr int VEC = Vec<T>::N;
    using V = typename Vec<T>::type;
    __shared__ __attribute__((aligned(16))) T colbuf[512 * G * VEC];  // column partials
    __shared__ __attribute__((aligned(16))) T tbuf[512 * R];          // row-sum transpose
    __shared__ T red[17 * R + 17];
    const int tid = threadIdx.x;
    const int NT = blockDim.x;
    // write-through stores for the relay (see above)
    auto wstore = [](T* dst, T v) {
        if constexpr (RELAY) __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else *dst = v;
    };

    // ---- per-thread column ownership; clamped addresses + masks (branch-free loads)
    int colc[G];
    bool cok[G][VEC];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int c0 = (tid + NT * g) * VEC;
        colc[g] = c0 < p.m ? c0 : 0;
#pragma unroll
        for (int k = 0; k < VEC; ++k) cok[g][k] = c0 + k < p.m;
    }
    const int nrb = (p.n + R - 1) / R;
    auto load_block = [&](int rb, T (&dst)[R][G][VEC]) {
        const int r0 = rb * R;
        const CT* crow = (const CT*)p.C + (int64_t)r0 * p.ldc;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const CT* src = (r0 + r < p.n) ? crow : (const CT*)p.C;
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const V c = load_cost<T>(src + colc[g]);
#pragma unroll
                for (int k = 0; k < VEC; ++k) dst[r][g][k] = c[k];
            }
            crow += p.ldc;
        }
    };
    T kv[R][G][VEC];
    bool kv_loaded = false;
    if constexpr (RELAY) {
        if (early && vb < nrb) {
            load_block(vb, kv);
            kv_loaded = true;
        }
        if (!wait()) return;
    }

    // stop flag: written by an earlier launch (a flag raised by WG0 of THIS launch is
    // a decision every workgroup re-derives identically), so a uniform plain load.
    if (__builtin_amdgcn_readfirstlane(*(volatile const int*)&p.info->stop)) return;

    const bool lead = (vb == 0 && tid == 0);
    // exponent units: float works in log2 (v_exp_f32), double in natural log
    const double unit = exp_unit<T>();
    double cinv = 1.0;
    if (p.cost_scale) cinv = 1.0 / (double)p.cost_scale[0];
    const T ks = (T)(-unit / p.reg * cinv);  // multiplies C
    const T gl = (T)(unit / p.reg);          // potential -> exponent units (OTT)
    const T regn = (T)(p.reg / unit);        // unit log -> potential

    // ---- decisions about iteration it-1 (identical in every workgroup)
    if (p.it >= 1) {
        const int prev = p.it - 1;
        if (p.cs_src[p.m_pad] != (T)0) {  // row scaling of prev not finite: revert to prev-1, stop
            if (lead) sk_stop(p.info, prev - 1, prev, OTF_SK_NUMERICAL_BREAK, prev);
            return;
        }
        if (check_now(p, prev)) {
            const double err = marginal_err<T, LOG, G, VEC>(p, p.v_prev, p.cs_src, colc, cok, red);
            if (lead) {
                const int slot = (prev + p.check_off) / p.check_every - p.check_off;
                p.errlog[slot] = err;
                p.info->n_err = slot + 1;
            }
            if (is_conv(p, err)) {
                if (lead) sk_stop(p.info, prev, prev, OTF_SK_CONVERGED, -1);
                return;
            }
        }
    }

    // ---- row blocks.  The first block's cost rows are put in flight BEFORE the
    // column-scaling prologue (its loads, arithmetic and barrier), so the prologue's
    // latency hides under the stream instead of preceding it.
    const bool have_prev = p.it >= 0;
    T vw[G][VEC];  // POT: v_j (row-sum weights); OTT: 1
    T go[G][VEC];  // OTT: g_j in exponent units; POT: 0
    T colacc[G][VEC];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int k = 0; k < VEC; ++k) colacc[g][k] = 0;

    for (int rb = vb; rb < nrb || rb == vb; rb += vg) {
        const int r0 = rb * R;
        if (rb < nrb && !kv_loaded) load_block(rb, kv);
        kv_loaded = false;
        if (rb == vb) {
            // column scaling of iteration it (POT: v; OTT: g), every workgroup, all columns
            if (have_prev) {
                int badv = 0;
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    const V sv = *reinterpret_cast<const V*>(p.cs_src + colc[g]);
                    const V bv = *reinterpret_cast<const V*>(p.b + colc[g]);
                    V gp;
                    if (LOG) gp = *reinterpret_cast<const V*>(p.v_prev + colc[g]);
#pragma unroll
                    for (int k = 0; k < VEC; ++k) {
                        T val;
                        if (LOG) val = regn * (unit_log(bv[k]) - unit_log(sv[k])) + gp[k];
                        else val = bv[k] / sv[k];
                        const bool bad = (sv[k] == (T)0) || !finite_val(val);
                        badv |= (cok[g][k] && bad) ? 1 : 0;
                        val = cok[g][k] ? val : (T)0;
                        if (LOG) {
                            go[g][k] = val * gl;
                            vw[g][k] = 1;
                        } else {
                            vw[g][k] = val;
                            go[g][k] = SH && cok[g][k] ? p.shB[colc[g] + k] : (T)0;
                        }
                        if (vb == 0 && cok[g][k]) p.v_cur[colc[g] + k] = val;
                    }
                }
                badv = __syncthreads_or(badv);
                if (badv) {  // zero column sum or nan/inf column scaling: revert to it-1, stop
                    if (lead) sk_stop(p.info, p.it - 1, p.it, OTF_SK_NUMERICAL_BREAK, p.it);
                    return;
                }
            } else {
#pragma unroll
                for (int g = 0; g < G; ++g)
#pragma unroll
                    for (int k = 0; k < VEC; ++k) {
                        vw[g][k] = 1;
                        go[g][k] = SH && cok[g][k] ? p.shB[colc[g] + k] : (T)0;
                        if (LOG) {  // g_{-1} = column minima of the scaled cost: terms <= 1
                            const T h = (T)((double)key_val(p.cmin_key[colc[g] + k]) * cinv);
                            go[g][k] = cok[g][k] ? h * gl : (T)0;
                            if (vb == 0 && cok[g][k]) p.v_cur[colc[g] + k] = h;
                        }
                    }
            }
            if (rb >= nrb) break;  // more workgroups than row blocks: prologue duty only
        }
        T fo[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int row = r0 + r < p.n ? r0 + r : p.n - 1;
            fo[r] = (LOG && p.it >= 0) ? p.u_prev[row] * gl : SH ? p.shA[row] : (T)0;
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const bool rok = r0 + r < p.n;
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int k = 0; k < VEC; ++k) {
                    if constexpr (KIN) {
                        kv[r][g][k] = (rok && cok[g][k]) ? kv[r][g][k] : (T)0;
                    } else {
                        T z = kv[r][g][k] * ks;
                        if (LOG || SH) z += fo[r] + go[g][k];
                        kv[r][g][k] = (rok && cok[g][k]) ? fast_exp(z) : (T)0;
                    }
                }
        }
        T ur[R];
        if (p.it >= 0) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                T s = 0;
#pragma unroll
                for (int g = 0; g < G; ++g)
#pragma unroll
                    for (int k = 0; k < VEC; ++k) s += LOG ? kv[r][g][k] : kv[r][g][k] * vw[g][k];
                ur[r] = s;
            }
            block_sum_rows<T, R>(ur, tbuf, red);
            T outv[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const bool rok = r0 + r < p.n;
                const int row = rok ? r0 + r : p.n - 1;
                const T ar = p.a[row];
                if (LOG) {
                    ur[r] = ar / ur[r];                                // w_i = a_i / rowsum_i
                    outv[r] = regn * unit_log(ur[r]) + p.u_prev[row];  // f_i
                } else {
                    ur[r] = (T)1 / (ur[r] * ((T)1 / ar));              // POT: 1 / (Kp v)
                    outv[r] = ur[r];
                }
                if (!rok) ur[r] = 0;  // padding rows: 1/0 = inf would poison 0 * inf
            }
            if (tid < R) {
                T mine = outv[0];
                T wmine = ur[0];
#pragma unroll
                for (int r = 1; r < R; ++r)
                    if (tid == r) {
                        mine = outv[r];
                        wmine = ur[r];
                    }
                const int row = r0 + tid;
                if (row < p.n) {
                    wstore(p.u_cur + row, mine);
                    if (!finite_val(mine) || !finite_val(wmine)) atomicAdd(p.cs_dst + p.m_pad, (T)1);
                }
            }
        } else {
            const T u0 = LOG ? (T)1 : (T)1 / (T)p.n_total;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                ur[r] = u0;
                if (SH) ur[r] = r0 + r < p.n ? p.u0v[r0 + r] : (T)0;  // u~0 = 2^-shA / n
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int k = 0; k < VEC; ++k) colacc[g][k] += kv[r][g][k] * ur[r];
    }

    // ---- flush column partials: one float atomic per column per workgroup, staged
    // through LDS so every atomic wave-instruction covers 256 contiguous bytes (a
    // 16-B lane stride runs the memory-side atomics an order of magnitude slower).
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int c0 = (tid + NT * g) * VEC;
        if (c0 < p.m_pad) {
            V w;
#pragma unroll
            for (int k = 0; k < VEC; ++k) w[k] = colacc[g][k];
            *reinterpret_cast<V*>(colbuf + c0) = w;
        }
    }
    __syncthreads();
    for (int j = tid; j < p.m; j += NT) atomicAdd(p.cs_dst + j, colbuf[j]);

    // ---- zero the column-sum buffer of the next pass (nobody touches it now)
    for (int j = vb * NT + tid; j <= p.m_pad; j += vg * NT) wstore(p.cs_zero + j, (T)0);
}

template <typename T, typename CT, bool LOG, int G, int R, bool SH>
__global__ __launch_bounds__(512) void sk_pass_kernel(SkArgs<T> p) {
    sk_pass_body<T, CT, LOG, G, R, SH>(p, (int)blockIdx.x, (int)gridDim.x);
}

template <typename T>
__device__ __forceinline__ void sk_init_body(int t, int stride, const T* a, const T* b, int n, int m, int m_pad,
                                             T* a_pad, T* b_pad, T* cs, int cs_stride, T* u2, T* v2,
                                             int* cmin_key, otf_sinkhorn_info* info, uint4* zero,
                                             int64_t zero_n, int* relay) {
    // a persistent engine's granule region (mesh), zeroed here instead of by a memset launch
    for (int64_t j = t; j < zero_n; j += stride) zero[j] = make_uint4(0u, 0u, 0u, 0u);
    // the relay fallback's counters (sk_relay_kernel): fresh for every solve
    for (int j = t; j < kRelayInts; j += stride) relay[j] = 0;
    for (int j = t; j < m_pad; j += stride) {
        b_pad[j] = j < m ? b[j] : (T)0;
        cs[j] = cs[cs_stride + j] = cs[2 * cs_stride + j] = 0;
        v2[j] = v2[m_pad + j] = 0;
        cmin_key[j] = 0x7fffffff;
    }
    for (int i = t; i < n; i += stride) {
        a_pad[i] = a[i];
        u2[i] = u2[n + i] = 0;
    }
    if (t < 3) cs[t * cs_stride + m_pad] = 0;
    if (t == 0) {
        info->stop = 0;
        info->last_good = -1;
        info->niter = 0;
        info->status = OTF_SK_RUNNING;
        info->n_err = 0;
        info->break_iter = -1;
        info->engine = OTF_ENGINE_STREAM;
        info->stalled = 0;
        info->fallback = 0;
    }
}
template <typename T>
__global__ void sk_init_kernel(const T* a, const T* b, int n, int m, int m_pad, T* a_pad, T* b_pad,
                               T* cs, int cs_stride, T* u2, T* v2, int* cmin_key,
                               otf_sinkhorn_info* info, uint4* zero, int64_t zero_n, int* relay) {
    sk_init_body<T>(blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x, a, b, n, m, m_pad, a_pad,
                    b_pad, cs, cs_stride, u2, v2, cmin_key, info, zero, zero_n, relay);
}

// Column minima of C (OTT prologue shift), ordered-int atomicMin per column.
template <typename CT>
__global__ __launch_bounds__(256) void sk_colmin_kernel(const CT* C, int64_t ldc, int n, int m,
                                                        int* cmin_key) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const int rows_per = (n + gridDim.y - 1) / gridDim.y;
    const int i0 = blockIdx.y * rows_per;
    const int i1 = i0 + rows_per < n ? i0 + rows_per : n;
    float mn = INFINITY;
    for (int i = i0; i < i1; ++i) mn = fminf(mn, (float)C[(int64_t)i * ldc + j]);
    if (i0 < i1) atomicMin(cmin_key + j, ord_key(mn));
}

// ---- Shifted POT kernel (opts.shift, float32 compute) -------------------------------
// POT's K = exp(-C/reg) leaves float32's normal range once C/reg > 87 (reg < 0.0115 on a
// max-normalised cost): v_exp_f32 flushes those entries to zero, and POT's scalings,
// which grow like exp(C/reg), overflow past 88.  Both matter: at reg = 0.01 on the
// metric shape the flushed entries alone move the plan by 2.2e-3 (normwise) after 100
// iterations, and at reg = 5e-3 whole columns of K vanish (a break at iteration 0).
// The shifted form runs POT's iteration on
//     K~_ij = 2^(C_ij ks + A_i + B_j),   u = 2^A u~,   v = 2^B v~,
// which in exact arithmetic is the same sequence of iterates (the offsets cancel in
// v = b / K^T u and u = a / K v, and P = u~ K~ v~ = u K v), with offsets taken from a
// log-domain first half-iteration:
//     B_j = log2 b_j - log2 sum_i 2^(C_ij ks) / n     (= log2 of POT's first v, exactly)
//     A_i = -max_j (C_ij ks + B_j)                    (every row of K~ peaks at 1)
// and the start u~0 = 2^-A / n (POT's u0 = 1/n).  K~ is then the first half-step's plan up
// to row factors: its entries that underflow are those far below their row's mass, so
// no plan entry that matters is ever formed from a flushed value, and u~, v~ stay near 1
// (|log2| < 60 over 100 iterations at reg = 2e-3 on the metric shape).  Cost: one column
// log-sum-exp pass and one row max pass over C before the solve.
constexpr int kShChunkMax = 128;  // row chunks of the column pass (partials in the workspace)
inline int shift_chunks(int64_t n) {
    const int64_t c = (n + 31) / 32;
    return (int)(c < 1 ? 1 : c > kShChunkMax ? kShChunkMax : c);
}

__device__ __forceinline__ float shift_ks(const float* cost_scale, double reg) {
    double cinv = 1.0;
    if (cost_scale) cinv = 1.0 / (double)cost_scale[0];
    return (float)(-exp_unit<float>() / reg * cinv);
}

// (max, sum 2^(z - max)) of z = C_ij ks over one row chunk, 4 columns per thread
template <typename CT>
__global__ __launch_bounds__(256) void sk_shift_cols_kernel(const CT* C, int64_t ldc, int n, int m,
                                                            int m_pad, const float* cost_scale,
                                                            double reg, float* pmax, float* psum) {
    using V = Vec<float>::type;
    const float ks = shift_ks(cost_scale, reg);
    const int c0 = (blockIdx.x * 256 + threadIdx.x) * 4;
    if (c0 >= m_pad) return;
    const int rows_per = (n + gridDim.y - 1) / gridDim.y;
    const int i0 = blockIdx.y * rows_per;
    const int i1 = i0 + rows_per < n ? i0 + rows_per : n;
    const CT* col = C + (c0 < m ? c0 : 0);
    float mx[4], sm[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        mx[k] = -3.0e38f;
        sm[k] = 0.f;
    }
    int i = i0;
    for (; i + 4 <= i1; i += 4) {
        V c[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) c[r] = load_cost<float>(col + (int64_t)(i + r) * ldc);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float z[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) z[r] = c[r][k] * ks;
            const float bm = fmaxf(fmaxf(z[0], z[1]), fmaxf(z[2], z[3]));
            const float nm = fmaxf(mx[k], bm);
            float t = sm[k] * fast_exp(mx[k] - nm);
#pragma unroll
            for (int r = 0; r < 4; ++r) t += fast_exp(z[r] - nm);
            sm[k] = t;
            mx[k] = nm;
        }
    }
    for (; i < i1; ++i) {
        const V c = load_cost<float>(col + (int64_t)i * ldc);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float z = c[k] * ks, nm = fmaxf(mx[k], z);
            sm[k] = sm[k] * fast_exp(mx[k] - nm) + fast_exp(z - nm);
            mx[k] = nm;
        }
    }
    const int64_t o = (int64_t)blockIdx.y * m_pad + c0;
    *reinterpret_cast<V*>(pmax + o) = V{mx[0], mx[1], mx[2], mx[3]};
    *reinterpret_cast<V*>(psum + o) = V{sm[0], sm[1], sm[2], sm[3]};
}

// B_j from the chunk partials; v~0_j = 2^-B_j / m.  Columns past m: B = 0, v~0 = 0.
__global__ void sk_shift_merge_kernel(const float* pmax, const float* psum, int nch, int m, int m_pad,
                                      const float* b_pad, int n_total, float* shB, float* v0v) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m_pad) return;
    if (j >= m) {
        shB[j] = 0.f;
        v0v[j] = 0.f;
        return;
    }
    float M = -3.0e38f;
    for (int q = 0; q < nch; ++q) M = fmaxf(M, pmax[(int64_t)q * m_pad + j]);
    float S = 0.f;
    for (int q = 0; q < nch; ++q) S += psum[(int64_t)q * m_pad + j] * fast_exp(pmax[(int64_t)q * m_pad + j] - M);
    const float bj = b_pad[j];
    // a zero marginal keeps v = 0 in POT; its shift only has to be finite
    const float B = (bj > 0.f ? __builtin_amdgcn_logf(bj) : 0.f) + __builtin_amdgcn_logf((float)n_total) -
                    (M + __builtin_amdgcn_logf(S));
    shB[j] = B;
    v0v[j] = fast_exp(-B - __builtin_amdgcn_logf((float)m));
}

// A_i = -max_j (C_ij ks + B_j), u~0_i = 2^-A_i / n: one wave per row
template <typename CT>
__global__ __launch_bounds__(256) void sk_shift_rows_kernel(const CT* C, int64_t ldc, int n, int m,
                                                            const float* cost_scale, double reg,
                                                            const float* shB, int n_total,
                                                            float* shA, float* u0v) {
    using V = Vec<float>::type;
    const float ks = shift_ks(cost_scale, reg);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const float ln = __builtin_amdgcn_logf((float)n_total);
    for (int row = blockIdx.x * 4 + wv; row < n; row += gridDim.x * 4) {
        const CT* crow = C + (int64_t)row * ldc;
        float mx = -3.0e38f;
        for (int c0 = lane * 4; c0 < m; c0 += 256) {
            const V c = load_cost<float>(crow + c0);
            const V b = *reinterpret_cast<const V*>(shB + c0);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (c0 + k < m) mx = fmaxf(mx, fmaf(c[k], ks, b[k]));
        }
        mx = wave_max(mx);
        if (lane == 0) {
            shA[row] = -mx;
            u0v[row] = fast_exp(mx - ln);
        }
    }
}

// Decides the outcome of the last pass when the loop ran to max_iter.
template <typename T, bool LOG>
__device__ __forceinline__ void sk_finalize_body(const SkArgs<T>& p, int max_iter) {
    __shared__ T red[17 * 2];
    __shared__ int s_flag;
    if (threadIdx.x == 0) s_flag = __hip_atomic_load(&p.info->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (s_flag) return;
    const bool lead = threadIdx.x == 0;
    if (max_iter <= 0) {
        if (lead) sk_stop(p.info, -1, 0, OTF_SK_MAX_ITER, -1);
        return;
    }
    const int it = max_iter - 1;
    if (p.cs_src[p.m_pad] != (T)0) {
        if (lead) sk_stop(p.info, it - 1, it, OTF_SK_NUMERICAL_BREAK, it);
        return;
    }
    int status = OTF_SK_MAX_ITER;
    if (check_now(p, it)) {
        T e = 0;
        for (int j = threadIdx.x; j < p.m; j += blockDim.x) {
            T r;
            if (LOG) {
                r = fabs(p.cs_src[j] - p.b[j]);
            } else {
                r = p.v_cur[j] * p.cs_src[j] - p.b[j];
                r = r * r;
            }
            e += r;
        }
        e = block_sum<T>(e, red);
        const double err = LOG ? (double)e : (p.err_squared ? (double)e : sqrt((double)e));
        if (lead) {
            const int slot = (it + p.check_off) / p.check_every - p.check_off;
            p.errlog[slot] = err;
            p.info->n_err = slot + 1;
        }
        if (is_conv(p, err)) status = OTF_SK_CONVERGED;
    }
    if (lead) sk_stop(p.info, it, it, status, -1);
}
template <typename T, bool LOG>
__global__ __launch_bounds__(512) void sk_finalize_kernel(SkArgs<T> p, int max_iter) {
    sk_finalize_body<T, LOG>(p, max_iter);
}

// Copies the scalings of info->last_good (or the initial ones) to the outputs.
// (shifted kernel: the initial scalings are the vectors u0v, v0v)
template <typename T, bool LOG>
__global__ void sk_output_kernel(const T* u2, const T* v2, int n, int n_total, int m, int m_pad,
                                 const otf_sinkhorn_info* info, T* u_out, T* v_out,
                                 const T* u0v, const T* v0v) {
    const int lg = info->last_good;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int stride = gridDim.x * blockDim.x;
    const T u0 = LOG ? (T)0 : (T)1 / (T)n_total;
    const T v0 = LOG ? (T)0 : (T)1 / (T)m;
    for (int i = t; i < n; i += stride) u_out[i] = lg >= 0 ? u2[(lg & 1) * n + i] : u0v ? u0v[i] : u0;
    for (int j = t; j < m; j += stride) v_out[j] = lg >= 0 ? v2[(lg & 1) * m_pad + j] : v0v ? v0v[j] : v0;
}

// POT: P_ij = u_i exp(-C_ij/reg') v_j;  OTT: P_ij = exp((f_i + g_j - C_ij/scale)/reg).
// (shifted kernel, shA != null: P_ij = u_i exp2(C_ij ks + shA_i + shB_j) v_j)
template <typename T, typename CT, typename TP, bool LOG>
__global__ __launch_bounds__(256) void sk_plan_kernel(const CT* C, int64_t ldc, int n, int m,
                                                      const T* u, const T* v, const T* cost_scale,
                                                      double reg, TP* P, int64_t ldp,
                                                      const T* shA, const T* shB) {
    const double unit = exp_unit<T>();
    double cinv = 1.0;
    if (cost_scale) cinv = 1.0 / (double)cost_scale[0];
    const T ks = (T)(-unit / reg * cinv);
    const T gl = (T)(unit / reg);
    constexpr int VEC = Vec<T>::N;
    using V = typename Vec<T>::type;
    using VP = __attribute__((ext_vector_type(VEC))) TP;
    for (int row = blockIdx.x; row < n; row += gridDim.x) {
        const T ui = u[row];
        const T ai = shA ? shA[row] : (T)0;
        const CT* crow = C + (int64_t)row * ldc;
        TP* prow = P + (int64_t)row * ldp;
        for (int j0 = threadIdx.x * VEC; j0 < m; j0 += blockDim.x * VEC) {
            const V c = load_cost<T>(crow + j0);
            VP out;
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const T vj = j0 + k < m ? v[j0 + k] : (T)0;
                const T bj = (shB && j0 + k < m) ? shB[j0 + k] : (T)0;
                T val;
                if (LOG) val = fast_exp(c[k] * ks + (ui + vj) * gl);
                else val = ui * fast_exp(c[k] * ks + (ai + bj)) * vj;
                out[k] = (TP)val;
            }
            if (j0 + VEC <= m) {
                *reinterpret_cast<VP*>(prow + j0) = out;  // ldp is a multiple of VEC
            } else {
#pragma unroll
                for (int k = 0; k < VEC; ++k)
                    if (j0 + k < m) prow[j0 + k] = out[k];
            }
        }
    }
}

// ============================================================================
// Relay fallback: the whole POT solve by a grid that needs NO co-residency, enqueued behind
// every persistent engine launch on the same stream.  A persistent engine needs its whole
// grid co-resident; when other kernels hold CUs (RCCL kernels under DDP, a second solve on
// another stream) its registration gives up after OTF_REG_MS and sets info->stalled to
// kStallRegistration (a stall in the middle of a solve sets kStallMid and is reported as
// OTF_SK_TIMEOUT, never re-solved: it means a broken exchange, not a busy device).  This
// kernel then returns the right answer instead of a timeout.  When the persistent solve
// succeeded (stalled == 0, the normal case) every workgroup returns at once: one empty
// dispatch per solve, no host synchronisation either way.
//
// The solve runs as a relay of TICKETS: a workgroup takes the next ticket from a counter,
// waits until every ticket of the previous phase is done, runs the ticket's piece and counts
// it done, then takes the next one.  A workgroup only ever waits for SMALLER tickets, all of
// them held by workgroups that are already running (a ticket is taken by a running
// workgroup), so the relay always progresses whatever part of the grid the device schedules
// and whenever -- one workgroup alone finishes it.  Phases, in ticket order:
//   reset    (vg pieces)      the abandoned launch's sums, scalings and info words
//   cost     (pairwise only)  the float64 cost in 128 x 128 tiles on v_mfma_f64_16x16x4_f64
//                             into the workspace, the grid's max by a 64-bit atomic max
//   K        (pairwise only)  K = exp(-C / (reg max)) written once over C
//   passes   (vg pieces each) the streaming engine's fused pass (sk_pass_body) for the
//                             prologue and every iteration: piece q is the pass launch's
//                             workgroup q; with a written K, no exp per element
//   finalize (one piece)      POT's decision for the last iteration (sk_finalize_body)
//   outputs  (vg pieces)      u, v of last_good and the plan rows of the piece
// Once a pass has stopped the solve (info->stop), the workgroup that sees it first moves the
// ticket counter past the remaining passes in one compare-and-swap and counts them done.
// Hand-off: a piece's stores drain (vmcnt(0)) and its completion is counted after a barrier;
// an agent-scope release fence precedes the count except in pass pieces after a pass's first
// (those store only write-through words and memory-side atomics).  The waiter: one poll and
// one agent acquire by thread 0, then a barrier.  A pass piece of a workgroup whose previous
// piece was a pass piece puts its first K row block in flight BEFORE that wait (K is complete
// and L1-fresh by then).  The completion count is sharded (kRelayDone).  Measured at the
// float64 bench shape (tools/relay_probe.py): 62.6 -> 34.0 us per pass, 7.0 -> 4.0 ms per call;
// ablations of the old form: 21 us of each pass was the dependency wait, 14 the K loads, 8 the
// column atomics.  Every fallback bumps
// g_sk_fallbacks (otf_sinkhorn_fallback_count) and sets info->fallback.  (r06: replaces the
// one-workgroup re-solve, whose pass loop on a single CU took tens of ms at the metric shape.)
// ============================================================================
__device__ unsigned long long g_sk_fallbacks;

template <typename T> struct SoloArgs {
    T* cs;              // 3 x cs_stride column-sum ring (stream engine layout)
    T* u2;              // 2 x n scalings by iteration parity
    T* v2;              // 2 x m_pad
    int64_t cs_stride;
    int max_iter;
    T* u_out;
    T* v_out;
    void* P;
    int64_t ldp;
    int p_f64;
    const T* v0v;       // shifted kernel: the initial column scalings (else null)
    int* relay;         // the relay counters (kRelayInts)
    int vg;             // pieces per pass / reset / output phase
    unsigned long long stall;  // no progress for this long at a wait: OTF_SK_TIMEOUT
    // behind the pairwise meshes (otf_sinkhorn_pairwise_f64 / _f32): the float32 rows, their
    // squared norms (the norms / prep launch wrote them) and where the cost's max goes
    const float* pw_X;
    const float* pw_Y;
    int64_t pw_ldx, pw_ldy;
    int pw_d, pw_euclid, pw_scale, pw_vec;
    const double* pw_nx;   // float64 pairwise: n + m squared norms (X's, then Y's)
    const float* pw_nxf;   // float32 pairwise (pw_nx null): X's n and Y's m squared norms
    const float* pw_nyf;
    T* pw_cmax_out;
    int pw_tiles_m, pw_ntiles;
};

// One 128 x 128 tile of the pairwise float64 cost (the epilogue of dist_mfma_f64_kernel:
// -2 x.y + |x|^2 + |y|^2 in POT's euclidean_distances order, clamped at 0, the root for the
// euclidean metric) on the first 256 threads: 4 waves of 64 x 64 on v_mfma_f64_16x16x4_f64,
// the float32 rows widened into a double-buffered LDS stage.  Returns the tile's max (thread 0).
constexpr int RL_T = 128, RL_K = 16;
template <typename T>
__device__ double relay_cost_tile(const SoloArgs<T>& x, T* C, int64_t ldc, int n, int m, int tile) {
    using D4 = __attribute__((ext_vector_type(4))) double;
    __shared__ __attribute__((aligned(16))) double As[2][RL_K][RL_T];
    __shared__ __attribute__((aligned(16))) double Bs[2][RL_K][RL_T];
    __shared__ double red[8];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const bool act = tid < 256;
    const int wm = (w >> 1) & 1, wn = w & 1, li = lane & 15, lk = lane >> 4;
    const int i0 = (tile % x.pw_tiles_m) * RL_T, j0 = (tile / x.pw_tiles_m) * RL_T;
    const int lr = (tid & 255) >> 1, lkk = (tid & 1) * 8;
    const int gi = i0 + lr < n ? i0 + lr : n - 1, gj = j0 + lr < m ? j0 + lr : m - 1;
    const float* xr = x.pw_X + (int64_t)gi * x.pw_ldx;
    const float* yr = x.pw_Y + (int64_t)gj * x.pw_ldy;
    const int d = x.pw_d;
    float xa[8], yb[8];
    auto gload = [&](int k0) {
        const int kb = k0 + lkk;
        if (x.pw_vec && kb + 8 <= d) {
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
        if (!act) return;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            As[buf][lkk + q][lr] = (double)xa[q];
            Bs[buf][lkk + q][lr] = (double)yb[q];
        }
    };
    D4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = D4{0.0, 0.0, 0.0, 0.0};
    const int nk = (d + RL_K - 1) / RL_K;
    if (act) gload(0);
    lstore(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (act && kt + 1 < nk) gload((kt + 1) * RL_K);
        if (act) {
#pragma unroll
            for (int ks = 0; ks < RL_K / 4; ++ks) {
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
        }
        if (kt + 1 < nk) lstore(buf ^ 1);
        __syncthreads();
    }
    double mx = 0.0;
    if (act) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int j = j0 + wn * 64 + b * 16 + li;
            const bool jok = j < m;
            const double ry = !jok ? 0.0 : x.pw_nx ? x.pw_nx[n + j] : (double)x.pw_nyf[j];
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = i0 + wm * 64 + a * 16 + lk + 4 * r;
                    if (i >= n || !jok) continue;
                    double v = -2.0 * acc[a][b][r];
                    v += x.pw_nx ? x.pw_nx[i] : (double)x.pw_nxf[i];
                    v += ry;
                    v = v > 0 ? v : 0.0;
                    if (x.pw_euclid) v = sqrt(v);
                    const T vt = (T)v;  // float32 pairwise: the float cost, its max as stored
                    C[(int64_t)i * ldc + j] = vt;
                    mx = fmax(mx, (double)vt);
                }
        }
    }
    mx = wave_max(mx);
    if (lane == 0) red[w] = mx;
    __syncthreads();
    double r = red[0];
    for (int q = 1; q < 4; ++q) r = fmax(r, red[q]);
    return r;
}

template <typename T, typename CT, int G, int R, bool SH, bool PW>
__global__ __launch_bounds__(512) void sk_relay_kernel(SkArgs<T> p, SoloArgs<T> x) {
    static_assert(!PW || std::is_same<CT, T>::value, "pairwise: the cost (then K) in the solve's type");
    __shared__ int s_t[3];
    const int tid = threadIdx.x, NT = blockDim.x;
    // only a grid that never became co-resident (registration give-up) is re-solved here;
    // a mid-solve stall stays an OTF_SK_TIMEOUT for the caller to see
    if (tid == 0)
        s_t[0] = __hip_atomic_load(&p.info->stalled, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == kStallRegistration;
    __syncthreads();
    if (!s_t[0]) return;
    int* ctr = x.relay;
    const int VG = x.vg;
    const int s_cost = VG;                                   // [reset: VG]
    const int s_k = s_cost + (PW ? x.pw_ntiles : 0);         // [cost tiles]
    const int s_pass = s_k + (PW ? VG : 0);                  // [K: VG]
    const int s_fin = s_pass + (x.max_iter + 1) * VG;        // [passes 0..max_iter: VG each]
    const int s_out = s_fin + 1;                             // [finalize: 1]
    const int s_end = s_out + VG;                            // [outputs: VG]
    // every ticket waits for all tickets of the phases before its own (reset and the cost
    // tiles for none)
    auto need = [&](int t) -> int {
        if (t < s_k) return 0;
        if (t < s_pass) return s_k;
        if (t < s_fin) return s_pass + ((t - s_pass) / VG) * VG;
        return t < s_out ? s_fin : s_out;
    };
    auto aload = [](const int* a) { return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    // completed tickets: the sum of the shards (each a lower bound of its own count)
    auto done_count = [&]() -> int {
        int c = 0;
#pragma unroll
        for (int q = 0; q < kRelayShards; ++q) c += aload(ctr + kRelayDone + q * kRelayDoneStride);
        return c;
    };
    int* const my_done = ctr + kRelayDone + (int)(blockIdx.x % kRelayShards) * kRelayDoneStride;
    auto set_pass = [&](SkArgs<T>& q, int pass) {
        const int it = pass - 1;
        q.it = it;
        q.cs_src = pass >= 1 ? x.cs + (size_t)((pass - 1) % 3) * x.cs_stride : nullptr;
        q.cs_dst = x.cs + (size_t)(pass % 3) * x.cs_stride;
        q.cs_zero = x.cs + (size_t)((pass + 1) % 3) * x.cs_stride;
        q.u_cur = x.u2 + (size_t)(it & 1) * p.n;
        q.v_cur = x.v2 + (size_t)(it & 1) * p.m_pad;
        q.u_prev = x.u2 + (size_t)((it - 1) & 1) * p.n;
        q.v_prev = x.v2 + (size_t)((it - 1) & 1) * p.m_pad;
    };
    unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + x.stall;
    // this workgroup's previous piece was a pass piece: it acquired after K was complete, so
    // a pass piece may stream its first K rows before its own wait (the input C of a
    // non-pairwise solve never changes in the launch)
    bool prev_pass = false;
    for (;;) {
        if (tid == 0) {
            int t;
            for (;;) {
                t = aload(ctr + kRelayTicket);
                // the solve has stopped (only a pass raises stop, after the reset cleared
                // it): skip the remaining passes in one step
                if (t >= s_pass && t < s_fin && done_count() >= s_pass && aload(&p.info->stop)) {
                    int want = t;
                    if (__hip_atomic_compare_exchange_strong(ctr + kRelayTicket, &want, s_fin, __ATOMIC_RELAXED,
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                        __hip_atomic_fetch_add(my_done, s_fin - t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    continue;
                }
                t = __hip_atomic_fetch_add(ctr + kRelayTicket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            s_t[1] = t;
        }
        __syncthreads();
        const int t = s_t[1];
        if (t >= s_end) return;
        // the ticket's dependency: one poll and one agent acquire by thread 0, then the
        // barrier (false: the relay was aborted)
        auto wait = [&]() -> bool {
            if (tid == 0) {
                int ok = 1;
                const int nd = need(t);
                while (done_count() < nd) {
                    if (aload(ctr + kRelayAbort)) { ok = 0; break; }
                    __builtin_amdgcn_s_sleep(2);
                    if (__builtin_amdgcn_s_memrealtime() > deadline) {
                        __hip_atomic_store(ctr + kRelayAbort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        p.info->status = OTF_SK_TIMEOUT;
                        ok = 0;
                        break;
                    }
                }
                if (ok) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                s_t[2] = ok;
            }
            __syncthreads();
            return s_t[2] != 0;
        };
        const bool is_pass = t >= s_pass && t < s_fin;
        if (is_pass) {
            SkArgs<T> q = p;
            set_pass(q, (t - s_pass) / VG);
            sk_pass_body<T, CT, false, G, R, SH, PW, true>(q, (t - s_pass) % VG, VG, wait, PW ? prev_pass : true);
            if (!s_t[2]) return;
            prev_pass = true;
        } else {
            if (!wait()) return;
            prev_pass = false;
        }
        if (t < s_cost) {
            // reset: fresh state (the abandoned persistent solve may have written these)
            for (int64_t j = (int64_t)t * NT + tid; j < 3 * x.cs_stride; j += (int64_t)VG * NT) x.cs[j] = 0;
            for (int j = t * NT + tid; j < 2 * p.n; j += VG * NT) x.u2[j] = 0;
            for (int j = t * NT + tid; j < 2 * p.m_pad; j += VG * NT) x.v2[j] = 0;
            if (t == 0 && tid == 0) {
                p.info->stop = 0;
                p.info->last_good = -1;
                p.info->niter = 0;
                p.info->status = OTF_SK_RUNNING;
                p.info->n_err = 0;
                p.info->break_iter = -1;
            }
        } else if (t < s_k) {
            if constexpr (PW) {
                const double mx = relay_cost_tile<T>(x, (T*)p.C, p.ldc, p.n, p.m, t - s_cost);
                if (tid == 0)
                    __hip_atomic_fetch_max(reinterpret_cast<unsigned long long*>(ctr + kRelayMax),
                                           __builtin_bit_cast(unsigned long long, mx), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
            }
        } else if (t < s_pass) {
            if constexpr (PW) {
                // K = exp(-C / (reg max)) over C, rows of this piece (costs >= 0: the max's bits
                // order like its value)
                const double cmax = __builtin_bit_cast(
                    double, __hip_atomic_load(reinterpret_cast<unsigned long long*>(ctr + kRelayMax),
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                const int q = t - s_k;
                if (q == 0 && tid == 0 && x.pw_cmax_out) *x.pw_cmax_out = (T)cmax;
                // the engines' K: float64 exp, or the float32 engines' fast_exp with log2(e) folded in
                const T ks = (T)(-exp_unit<T>() / p.reg * (x.pw_scale ? 1.0 / cmax : 1.0));
                T* C = (T*)p.C;
                for (int row = q; row < p.n; row += VG) {
                    T* cr = C + (int64_t)row * p.ldc;
                    for (int j = tid; j < p.m; j += NT) {
                        if constexpr (sizeof(T) == 8) cr[j] = exp(cr[j] * ks);
                        else cr[j] = fast_exp(cr[j] * ks);
                    }
                }
            }
        } else if (is_pass) {
            // (run above)
        } else if (t < s_out) {
            SkArgs<T> q = p;
            set_pass(q, x.max_iter + 1);
            q.it = x.max_iter - 1;
            q.v_cur = x.v2 + (size_t)(q.it & 1) * p.m_pad;
            sk_finalize_body<T, false>(q, x.max_iter);
            if (tid == 0) {
                p.info->engine = OTF_ENGINE_STREAM;
                p.info->fallback = 1;
                atomicAdd(&g_sk_fallbacks, 1ull);
            }
        } else {
            // outputs: the scalings of last_good (or the initial ones) and this piece's plan rows
            const int q = t - s_out;
            const int lg = p.info->last_good;
            const T u0 = (T)1 / (T)p.n_total, v0 = (T)1 / (T)p.m;
            const T* ul = x.u2 + (size_t)(lg & 1) * p.n;
            const T* vl = x.v2 + (size_t)(lg & 1) * p.m_pad;
            for (int i = q * NT + tid; i < p.n; i += VG * NT) x.u_out[i] = lg >= 0 ? ul[i] : SH ? p.u0v[i] : u0;
            for (int j = q * NT + tid; j < p.m; j += VG * NT) x.v_out[j] = lg >= 0 ? vl[j] : SH ? x.v0v[j] : v0;
            if (x.P) {
                const double unit = exp_unit<T>();
                double cinv = 1.0;
                if (!PW && p.cost_scale) cinv = 1.0 / (double)p.cost_scale[0];
                const T ks = (T)(-unit / p.reg * cinv);
                const CT* C = (const CT*)p.C;
                for (int row = q; row < p.n; row += VG) {
                    const T ui = lg >= 0 ? ul[row] : SH ? p.u0v[row] : u0;
                    const T ai = SH ? p.shA[row] : (T)0;
                    for (int j = tid; j < p.m; j += NT) {
                        const T vj = lg >= 0 ? vl[j] : SH ? x.v0v[j] : v0;
                        T kij;
                        if constexpr (PW) kij = (T)C[(int64_t)row * p.ldc + j];
                        else kij = fast_exp((T)C[(int64_t)row * p.ldc + j] * ks + (SH ? ai + p.shB[j] : (T)0));
                        const T val = ui * kij * vj;
                        if (x.p_f64) ((double*)x.P)[(int64_t)row * x.ldp + j] = (double)val;
                        else ((float*)x.P)[(int64_t)row * x.ldp + j] = (float)val;
                    }
                }
            }
            if (q == VG - 1 && tid == 0) p.info->stalled = 0;
        }
        // completion: this piece's stores drained and released device-wide, then counted.  A
        // pass piece other than the pass's first stores only write-through (sc1) words and
        // memory-side atomics: its drained stores need no release (MI355X_MICROARCH.md,
        // hand-off table); the first piece also writes v and the info words plainly.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            if (!is_pass || (t - s_pass) % VG == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __hip_atomic_fetch_add(my_done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        deadline = __builtin_amdgcn_s_memrealtime() + x.stall;
    }
}

// ============================================================================
// Resident engine: ONE persistent launch for the whole solve (POT flavour).
//
// Workgroup w owns row block w (R rows x all m columns) and keeps K = exp(-C/reg)
// for it in registers for every iteration, so C crosses HBM once per solve.  Per
// iteration each workgroup reads the column sums K^T u of the previous iteration,
// forms v, decides convergence / numerical break exactly like the streaming pass
// (every workgroup derives the same decision from the same sums), updates u for
// its rows and adds its column partials K_w^T u_w into a FRESH per-iteration sum
// buffer with memory-side float atomics -- into one of NREP replicas picked by the
// workgroup's XCD, so ~256/NREP adders share an address instead of 256.  An
// XCD-hierarchical barrier (xcd_barrier) separates iterations; the sums are then
// read with 16-B sc1 buffer loads (the no-acquire hand-off form).  Every spin is
// bounded by wall-clock time (s_memrealtime, 100 MHz): a barrier that does not
// complete sets OTF_SK_TIMEOUT instead of hanging.  Co-residency of the grid
// (<= one workgroup per CU) is checked before the launch (launch_resident_g).
// ============================================================================

template <typename T> struct SkResArgs {
    const void* C;    // cost, element type CT
    int64_t ldc;
    int n, m, m_pad;
    const T* a;
    const T* b;
    const T* cost_scale;
    double reg;
    int max_iter, check_every, err_squared;
    double stop_thr;
    T* cs;            // ring of 4 slots (slot k % 4 = K^T u(k-1)), nrep x m_pad each, zeroed
    SkSync sync;      // hierarchical barrier words, zeroed before launch
    int nrep;         // replicas per iteration (= the kernel's NREP)
    int* bad_cnt;     // ring of 4 counters (one 256-B line each), zeroed
    int* bar;         // barrier counter, zeroed
    otf_sinkhorn_info* info;
    double* errlog;
    T* u_out;
    T* v_out;
    void* P;
    int64_t ldp;
    int p_f64;
    unsigned long long timeout_ticks;
    unsigned long long reg_ticks;  // the first wait (registration / first hop)
    // OTT flavour in scaling form (float64 only; otf_sinkhorn_opts.engine = RESIDENT):
    // U = exp(f / eps), V = exp(g / eps) with f = g = 0 at the start, so the updates are
    // POT's (V = b / K^T U, U = a / K V) from U = 1; OTT's L1 marginal error after every
    // check_every-th update; outputs f = eps ln U, g = eps ln V; a zero U or V (f or g =
    // -inf in the log form) is a numerical break like a non-finite one.  Valid while
    // K = exp(-C / (eps s)) does not underflow (the caller's contract: max C / (eps s)
    // well inside float64's exponent range, e.g. <= 300 with scale_cost = max_cost).
    int ott;
};


template <typename T, typename CT, typename TP, int G, int R, int NREP>
__global__ __launch_bounds__(512) void sk_resident_kernel(SkResArgs<T> p) {
    constexpr int VEC = Vec<T>::N;
    using V = typename Vec<T>::type;
    using VP = __attribute__((ext_vector_type(VEC))) TP;
    __shared__ __attribute__((aligned(16))) T colbuf[512 * G * VEC];
    __shared__ __attribute__((aligned(16))) T tbuf[512 * R];
    __shared__ __attribute__((aligned(16))) T vhist[2][512 * G * VEC];  // v of iterations by parity
    __shared__ T uhist[2][R];                                             // u of this block's rows
    __shared__ T red[17 * R + 17];
    __shared__ int s_flag;
    __shared__ int s_pop[3];
    const int tid = threadIdx.x;
    const int NT = blockDim.x;
    const int nwg = gridDim.x;
    const bool lead = (blockIdx.x == 0 && tid == 0);
    unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + p.reg_ticks;

    const double unit = exp_unit<T>();
    double cinv = 1.0;
    if (p.cost_scale) cinv = 1.0 / (double)p.cost_scale[0];
    const T ks = (T)(-unit / p.reg * cinv);

    int colc[G];
    bool cok[G][VEC];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int c0 = (tid + NT * g) * VEC;
        colc[g] = c0 < p.m ? c0 : 0;
#pragma unroll
        for (int k = 0; k < VEC; ++k) cok[g][k] = c0 + k < p.m;
    }

    // ---- this workgroup's rows of K, once
    const int r0 = blockIdx.x * R;
    T kv[R][G][VEC];
    {
        const CT* crow = (const CT*)p.C + (int64_t)r0 * p.ldc;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const CT* src = (r0 + r < p.n) ? crow : (const CT*)p.C;
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const V c = load_cost<T>(src + colc[g]);
#pragma unroll
                for (int k = 0; k < VEC; ++k) kv[r][g][k] = c[k];
            }
            crow += p.ldc;
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const bool rok = r0 + r < p.n;
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int k = 0; k < VEC; ++k)
                    kv[r][g][k] = (rok && cok[g][k]) ? fast_exp(kv[r][g][k] * ks) : (T)0;
        }
    }
    T ia[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int row = r0 + r < p.n ? r0 + r : p.n - 1;
        ia[r] = (T)1 / p.a[row];
    }

    // iteration history in LDS, slot = iteration & 1 (slots start as u0 = 1/n, v0 = 1/m;
    // OTT: U = V = 1): iteration it reads v(it-1) from slot (it-1)&1 and writes u(it),
    // v(it) into slot it&1 only after its checks pass, so slot it&1 still holds
    // iteration it-2 when a numerical break in it-1 has to revert two iterations.
    const bool ott = p.ott != 0;
    const T u0 = ott ? (T)1 : (T)1 / (T)p.n, v0 = ott ? (T)1 : (T)1 / (T)p.m;
    // the iteration whose marginal error is checked: POT it % ce == 0, OTT after every
    // ce-th update ((it + 1) % ce == 0); its error-log slot
    auto checked = [&](int it) -> bool { return ((it + (ott ? 1 : 0)) % p.check_every) == 0; };
    auto err_slot = [&](int it) -> int { return ott ? (it + 1) / p.check_every - 1 : it / p.check_every; };
    auto finish_err = [&](T e) -> double {
        return ott ? (double)e : (p.err_squared ? (double)e : sqrt((double)e));
    };
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            vhist[0][(tid + NT * g) * VEC + k] = v0;
            vhist[1][(tid + NT * g) * VEC + k] = v0;
        }
    if (tid < R) uhist[0][tid] = uhist[1][tid] = u0;
    int idxB = -1;
    const size_t it_stride = (size_t)NREP * p.m_pad;
    const int xcd = xcc_id();
    const int my_rep = xcd % NREP;
    // K^T u(it-1) for this thread's columns: the sum of one buffer's replicas.  Whole
    // vectors are loaded unmasked (every buffer is m_pad wide and zero past m) so all
    // G x NREP loads are in flight together; masks are applied afterwards.
    const __amdgpu_buffer_rsrc_t rs = sums_rsrc(p.cs);
    auto load_sums = [&](const T* base, T (&out)[G][VEC], T fill) {
        const uint32_t boff = (uint32_t)((base - p.cs) * sizeof(T));
        V acc[G];
#pragma unroll
        for (int g = 0; g < G; ++g) acc[g] = load_sum_vec<T>(rs, boff + colc[g] * (uint32_t)sizeof(T));
#pragma unroll
        for (int q = 1; q < NREP; ++q) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const V t = load_sum_vec<T>(
                    rs, boff + (uint32_t)((q * p.m_pad + colc[g]) * sizeof(T)));
#pragma unroll
                for (int k = 0; k < VEC; ++k) acc[g][k] += t[k];
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int k = 0; k < VEC; ++k) out[g][k] = cok[g][k] ? acc[g][k] : fill;
    };
    // target column marginal, constant over the solve (b_pad is zero past m)
    T bcol[G][VEC];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const V t = *reinterpret_cast<const V*>(p.b + colc[g]);
#pragma unroll
        for (int k = 0; k < VEC; ++k) bcol[g][k] = t[k];
    }

    auto flush = [&](const T (&w)[R], T* dst) {
        T colacc[G][VEC];
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                T s = 0;
#pragma unroll
                for (int r = 0; r < R; ++r) s += kv[r][g][k] * w[r];
                colacc[g][k] = s;
            }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int c0 = (tid + NT * g) * VEC;
            if (c0 < p.m_pad) {
                V wv;
#pragma unroll
                for (int k = 0; k < VEC; ++k) wv[k] = colacc[g][k];
                *reinterpret_cast<V*>(colbuf + c0) = wv;
            }
        }
        __syncthreads();
        dst += (size_t)my_rep * p.m_pad;
        for (int j = tid; j < p.m; j += NT) atomicAdd(dst + j, colbuf[j]);
    };

    // slot k % 4 is free once iteration k - 1 has started (S[k-4] was last read in
    // iteration k - 3): this workgroup's share of it and its break counter, write-through
    auto zero_slot = [&](int k) {
        T* zs = p.cs + (size_t)(k & 3) * it_stride;
        const int64_t per = ((int64_t)it_stride + nwg - 1) / nwg;
        const int64_t z0 = (int64_t)blockIdx.x * per;
        const int64_t z1 = z0 + per < (int64_t)it_stride ? z0 + per : (int64_t)it_stride;
        for (int64_t j = z0 + tid; j < z1; j += NT) store_wt(zs + j, (T)0);
        if (blockIdx.x == 0 && tid == 0) store_wt(p.bad_cnt + (k & 3) * 64, 0);
    };
    // ---- prologue: K^T u0 into sums[0]
    {
        T w[R];
#pragma unroll
        for (int r = 0; r < R; ++r) w[r] = (r0 + r < p.n) ? u0 : (T)0;
        flush(w, p.cs);
    }
    int last_good = -1, niter = 0, status = OTF_SK_MAX_ITER, brk = -1, n_err = 0;
    bool done = false;
    // register on this XCD's population, then the one flat barrier of the launch
    if (tid == 0)
        __hip_atomic_fetch_add(p.sync.reg + xcd * 64, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!grid_barrier(p.bar, nwg, deadline, p.timeout_ticks, &s_flag, &p.info->stalled)) {
        status = OTF_SK_TIMEOUT;
        done = true;
    }
    if (tid == 0) {
        int nact = 0;
        unsigned mask = 0;
        for (int x = 0; x < 8; ++x) {
            const int c = __hip_atomic_load(p.sync.reg + x * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (c > 0) {
                ++nact;
                mask |= 1u << x;
            }
        }
        s_pop[0] = __hip_atomic_load(p.sync.reg + xcd * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_pop[1] = nact;
        s_pop[2] = (int)mask;
    }
    __syncthreads();
    const int nx = s_pop[0], nact = s_pop[1];
    const unsigned act_mask = (unsigned)s_pop[2];

    for (int it = 0; it < p.max_iter && !done; ++it) {
        OTF_STAMP(it, 0);
        const T* cs_it = p.cs + (size_t)(it & 3) * it_stride;   // K^T u(it-1)
        T s[G][VEC], vn[G][VEC];
        int badv = 0;
        // the break flag of u(it-1) is loaded together with the sums (one round trip)
        const int prev_bad = it >= 1 ? load_agent(p.bad_cnt + ((it - 1) & 3) * 64) : 0;
        load_sums(cs_it, s, (T)1);
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const T bj = bcol[g][k];
                const T val = bj / s[g][k];
                badv |= (cok[g][k] && ((s[g][k] == (T)0) || !finite_val(val) || (ott && val == (T)0))) ? 1 : 0;
                vn[g][k] = cok[g][k] ? val : (T)0;
            }
        // numerical break in u(it-1) -> revert to it-2
        if (prev_bad > 0) {
            last_good = it - 2; niter = it - 1; status = OTF_SK_NUMERICAL_BREAK; brk = it - 1;
            break;
        }
        // marginal error of iteration it-1: v(it-1) * K^T u(it-1) - b (POT: L2, OTT: L1)
        if (it >= 1 && checked(it - 1)) {
            T e = 0;
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int k = 0; k < VEC; ++k) {
                    const T vb = vhist[(it - 1) & 1][(tid + NT * g) * VEC + k];
                    const T rr = vb * s[g][k] - bcol[g][k];
                    e += cok[g][k] ? (ott ? fabs(rr) : rr * rr) : (T)0;
                }
            e = block_sum<T>(e, red);
            const double err = finish_err(e);
            if (lead) p.errlog[err_slot(it - 1)] = err;
            n_err = err_slot(it - 1) + 1;
            if (p.err_squared ? !(err > p.stop_thr) : (err < p.stop_thr)) {
                last_good = it - 1; niter = it - 1; status = OTF_SK_CONVERGED;
                break;
            }
        }
        badv = __syncthreads_or(badv);
        OTF_STAMP(it, 1);
        if (badv) {  // zero in K^T u or nan/inf in v: revert to it-1
            last_good = it - 1; niter = it; status = OTF_SK_NUMERICAL_BREAK; brk = it;
            break;
        }
        // u(it) for this workgroup's rows
        T un[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            T acc = 0;
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int k = 0; k < VEC; ++k) acc += kv[r][g][k] * vn[g][k];
            un[r] = acc;
        }
        block_sum_rows<T, R>(un, tbuf, red);
        OTF_STAMP(it, 2);
        int badu = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const bool rok = r0 + r < p.n;
            un[r] = (T)1 / (un[r] * ia[r]);
            badu |= (rok && (!finite_val(un[r]) || (ott && un[r] == (T)0))) ? 1 : 0;
            if (!rok) un[r] = 0;
        }
        if (badu && tid == 0) atomicAdd(p.bad_cnt + (it & 3) * 64, 1);
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int k = 0; k < VEC; ++k) vhist[it & 1][(tid + NT * g) * VEC + k] = vn[g][k];
        if (tid < R) {
            T mine = un[0];
#pragma unroll
            for (int r = 1; r < R; ++r)
                if (tid == r) mine = un[r];
            uhist[it & 1][tid] = mine;
        }
        flush(un, p.cs + (size_t)((it + 1) & 3) * it_stride);
        zero_slot(it + 2);
        idxB = it;
        OTF_STAMP(it, 3);
#ifdef OTF_STAMPS
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        OTF_STAMP(it, 4);
#endif
        if (!xcd_barrier(p.sync, xcd, nx, nact, act_mask, it + 1, deadline, p.timeout_ticks, &s_flag)) {
            status = OTF_SK_TIMEOUT;
            done = true;
        }
        OTF_STAMP(it, 5);
    }
    if (status == OTF_SK_MAX_ITER && p.max_iter > 0 && idxB == p.max_iter - 1) {
        const int it = p.max_iter - 1;
        if (load_agent(p.bad_cnt + (it & 3) * 64) > 0) {
            last_good = it - 1; niter = it; status = OTF_SK_NUMERICAL_BREAK; brk = it;
        } else {
            last_good = it; niter = it;
            if (checked(it)) {
                const T* cs_last = p.cs + (size_t)(p.max_iter & 3) * it_stride;
                T e = 0, sl[G][VEC];
                load_sums(cs_last, sl, (T)0);
#pragma unroll
                for (int g = 0; g < G; ++g)
#pragma unroll
                    for (int k = 0; k < VEC; ++k) {
                        const T sk = sl[g][k];
                        const T vb = vhist[it & 1][(tid + NT * g) * VEC + k];
                        const T rr = vb * sk - bcol[g][k];
                        e += cok[g][k] ? (ott ? fabs(rr) : rr * rr) : (T)0;
                    }
                e = block_sum<T>(e, red);
                const double err = finish_err(e);
                if (lead) p.errlog[err_slot(it)] = err;
                n_err = err_slot(it) + 1;
                if (p.err_squared ? !(err > p.stop_thr) : (err < p.stop_thr)) status = OTF_SK_CONVERGED;
            }
        }
    }

    // ---- outputs from registers: (u, v) of last_good, and the plan rows
    (void)idxB;
    __syncthreads();
    const int slot = last_good & 1;
    T uo[R], vo[G][VEC];
#pragma unroll
    for (int r = 0; r < R; ++r) uo[r] = uhist[slot][r];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int k = 0; k < VEC; ++k) vo[g][k] = vhist[slot][(tid + NT * g) * VEC + k];
    if (last_good < 0) {  // initial scalings
#pragma unroll
        for (int r = 0; r < R; ++r) uo[r] = u0;
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int k = 0; k < VEC; ++k) vo[g][k] = v0;
    }
    // OTT: the potentials f = eps ln U, g = eps ln V (units of the scaled cost)
    const T epsu = (T)(p.reg / unit);
    if (tid < R && r0 + tid < p.n) {
        T mine = uo[0];
#pragma unroll
        for (int r = 1; r < R; ++r)
            if (tid == r) mine = uo[r];
        p.u_out[r0 + tid] = ott ? epsu * unit_log(mine) : mine;
    }
    if (blockIdx.x == 0) {
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int k = 0; k < VEC; ++k)
                if (cok[g][k]) p.v_out[colc[g] + k] = ott ? epsu * unit_log(vo[g][k]) : vo[g][k];
    }
    if (p.P) {
        TP* P = (TP*)p.P;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (r0 + r >= p.n) break;
            TP* prow = P + (int64_t)(r0 + r) * p.ldp;
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const int c0 = (tid + NT * g) * VEC;
                if (c0 >= p.m) continue;
                VP o;
#pragma unroll
                for (int k = 0; k < VEC; ++k) o[k] = (TP)(uo[r] * kv[r][g][k] * vo[g][k]);
                if (c0 + VEC <= p.m) {
                    *reinterpret_cast<VP*>(prow + c0) = o;
                } else {
#pragma unroll
                    for (int k = 0; k < VEC; ++k)
                        if (c0 + k < p.m) prow[c0 + k] = o[k];
                }
            }
        }
    }
    if (status == OTF_SK_TIMEOUT && threadIdx.x == 0) mark_stalled(&p.info->stalled, kStallMid);
    if (lead) {
        p.info->last_good = last_good;
        p.info->niter = niter;
        p.info->status = status;
        p.info->break_iter = brk;
        p.info->n_err = n_err;
        p.info->engine = OTF_ENGINE_RESIDENT;
        p.info->stop = 1;
    }
}

// ============================================================================
// Tiled resident engine (OTF_ENGINE_TILED): the whole solve in one launch like
// sk_resident_kernel, but each workgroup owns a 2-D TILE of K -- 512 columns x
// 128 rows for float (8 waves x 16 rows, 64 lanes x 8 columns) or 64 rows for double
// (8 waves x 8 rows) -- instead of a few full rows.  Per iteration it therefore adds only 512 column partials to the sums
// (8x fewer float atomics: they execute at the memory side at ~1.3 TB/s chip-wide,
// and 4096 per workgroup were the single largest term of an iteration), and the
// row sums K v become a two-level reduction: within the wave (butterfly), then over
// the ncb column tiles of the row block -- a GROUP of workgroups that exchange 128
// partials each through write-through (sc1) stores and a per-group arrival counter
// (placed on one XCD when the shape allows; speed only).  Every member gathers the
// ncb partials in the same fixed order, so all members compute the same u.
//
// Control differs from sk_resident_kernel only in WHEN a numerical break in v is
// seen: a workgroup sees only its own columns, so a zero / non-finite v counts into
// bad_cnt[it] (as a non-finite u always did) and every workgroup takes the break at
// the top of iteration it+1 -- the same (last_good, niter, break_iter) as POT.  The
// marginal error of iterate it-1 (every check_every) is computed by every workgroup
// from the FULL sum vectors cs[it] and cs[it-1] (v(it-1) = b / cs[it-1] is recomputed
// bit-identically), so every workgroup takes the same stop decision at once.
// ============================================================================
template <typename T> struct TileCfg {
    static constexpr int NW = 8;                        // waves per workgroup
    static constexpr int RW = sizeof(T) == 4 ? 16 : 8;  // rows per wave (per thread)
    static constexpr int VEC = Vec<T>::N;
    static constexpr int G = sizeof(T) == 4 ? 2 : 4;    // VEC-vectors per lane: 8 columns
    static constexpr int R = RW * NW;                   // rows per tile: 128 / 64
    static constexpr int C = kWave * G * VEC;           // 512 columns per tile
};
constexpr int TL_C = 512;
inline int64_t tile_rows(size_t esz) { return esz == 4 ? TileCfg<float>::R : TileCfg<double>::R; }

template <typename T> struct SkTileArgs {
    const void* C;
    int64_t ldc;
    int n, m, m_pad;
    const T* a;
    const T* b;
    const T* cost_scale;
    double reg;
    int max_iter, check_every, err_squared;
    double stop_thr;
    T* cs;            // ring of 4 slots (slot k % 4 = K^T u(k-1)), nrep x m_pad each, zeroed
    int nrep;
    int* bad_cnt;     // ring of 4 counters (one 256-B line each), zeroed
    int* bar;         // flat barrier counter, zeroed
    SkSync sync;      // hierarchical barrier words, zeroed
    T* xch;           // 2 x nrb x ncb x tile rows row partials (write-through hand-off)
    int* grp;         // nrb counters, one 256-B line each, zeroed
    int nrb, ncb;
    otf_sinkhorn_info* info;
    double* errlog;
    T* u_out;
    T* v_out;
    void* P;
    int64_t ldp;
    unsigned long long timeout_ticks;
    unsigned long long reg_ticks;  // the first wait (registration / first hop)
};


template <typename T, typename CT, typename TP, int NREP>
__global__ __launch_bounds__(512) void sk_tiled_kernel(SkTileArgs<T> p) {
    using Cf = TileCfg<T>;
    constexpr int G = Cf::G, VEC = Cf::VEC, R = Cf::RW, NW = Cf::NW, TR = Cf::R;
    static_assert(Cf::C == TL_C, "tile width");
    using V = typename Vec<T>::type;
    using VP = __attribute__((ext_vector_type(VEC))) TP;
    __shared__ __attribute__((aligned(16))) T colbuf[NW][TL_C];
    __shared__ T urow[NW][R];          // u of each wave's rows (wave-private)
    __shared__ T uhist[2][TR];          // u history (slot = iteration & 1)
    __shared__ __attribute__((aligned(16))) T vhist[2][TL_C];  // v history
    __shared__ T red[17 + 17];
    __shared__ int s_flag;
    __shared__ int s_pop[3];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int nwg = gridDim.x;
    const bool lead = (blockIdx.x == 0 && tid == 0);
    unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + p.reg_ticks;

    // tile of this workgroup; groups (row blocks) on one XCD when nrb % 8 == 0
    int rb, cb;
    {
        const int b = blockIdx.x;
        if ((p.nrb & 7) == 0) {
            const int x = b & 7, q = b >> 3;
            rb = (q / p.ncb) * 8 + x;
            cb = q % p.ncb;
        } else {
            rb = b / p.ncb;
            cb = b % p.ncb;
        }
    }
    const int row0 = rb * TR + w * R;   // this wave's first row
    const int col0 = cb * TL_C;           // this tile's first column

    const double unit = exp_unit<T>();
    double cinv = 1.0;
    if (p.cost_scale) cinv = 1.0 / (double)p.cost_scale[0];
    const T ks = (T)(-unit / p.reg * cinv);

    int colc[G];
    bool cok[G][VEC];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int c0 = col0 + (lane + kWave * g) * VEC;
        colc[g] = c0 < p.m ? c0 : 0;
#pragma unroll
        for (int k = 0; k < VEC; ++k) cok[g][k] = c0 + k < p.m;
    }
    // ---- K for this wave's 16 rows x this lane's 8 columns, once
    T kv[R][G][VEC];
    {
        const CT* crow = (const CT*)p.C + (int64_t)row0 * p.ldc;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const CT* src = (row0 + r < p.n) ? crow : (const CT*)p.C;
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const V c = load_cost<T>(src + colc[g]);
#pragma unroll
                for (int k = 0; k < VEC; ++k) kv[r][g][k] = c[k];
            }
            crow += p.ldc;
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const bool rok = row0 + r < p.n;
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int k = 0; k < VEC; ++k)
                    kv[r][g][k] = (rok && cok[g][k]) ? fast_exp(kv[r][g][k] * ks) : (T)0;
        }
    }
    // 1 / a of the row whose total this lane finishes (lanes 0..15 of each wave)
    const T ia_mine = (T)1 / p.a[row0 + (lane & (R - 1)) < p.n ? row0 + (lane & (R - 1)) : p.n - 1];
    const T u0 = (T)1 / (T)p.n, v0 = (T)1 / (T)p.m;
    for (int q = tid; q < TL_C; q += blockDim.x) vhist[0][q] = vhist[1][q] = v0;
    if (tid < TR) uhist[0][tid] = uhist[1][tid] = u0;

    const size_t it_stride = (size_t)NREP * p.m_pad;
    const int xcd = xcc_id();
    const int my_rep = xcd % NREP;
    const __amdgpu_buffer_rsrc_t rs = sums_rsrc(p.cs);
    // this lane's 8 column sums of one buffer (all replicas), unmasked 16-B sc1 loads
    auto load_sums = [&](const T* base, T (&out)[G][VEC], T fill) {
        const uint32_t boff = (uint32_t)((base - p.cs) * sizeof(T));
        V acc[G];
#pragma unroll
        for (int g = 0; g < G; ++g) acc[g] = load_sum_vec<T>(rs, boff + colc[g] * (uint32_t)sizeof(T));
#pragma unroll
        for (int q = 1; q < NREP; ++q)
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const V t = load_sum_vec<T>(rs, boff + (uint32_t)((q * p.m_pad + colc[g]) * sizeof(T)));
#pragma unroll
                for (int k = 0; k < VEC; ++k) acc[g][k] += t[k];
            }
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int k = 0; k < VEC; ++k) out[g][k] = cok[g][k] ? acc[g][k] : fill;
    };
    // full-vector L2 marginal error of iterate `itp` (needs cs[itp + 1] and cs[itp])
    auto full_error = [&](int itp) -> double {
        const uint32_t bs = (uint32_t)((size_t)((itp + 1) & 3) * it_stride * sizeof(T));
        const uint32_t bp = (uint32_t)((size_t)(itp & 3) * it_stride * sizeof(T));
        T e = 0;
        for (int c0 = tid * VEC; c0 < p.m_pad; c0 += blockDim.x * VEC) {
            V sc = load_sum_vec<T>(rs, bs + c0 * (uint32_t)sizeof(T));
            V sp = load_sum_vec<T>(rs, bp + c0 * (uint32_t)sizeof(T));
#pragma unroll
            for (int q = 1; q < NREP; ++q) {
                const V t1 = load_sum_vec<T>(rs, bs + (uint32_t)((q * p.m_pad + c0) * sizeof(T)));
                const V t2 = load_sum_vec<T>(rs, bp + (uint32_t)((q * p.m_pad + c0) * sizeof(T)));
#pragma unroll
                for (int k = 0; k < VEC; ++k) { sc[k] += t1[k]; sp[k] += t2[k]; }
            }
            const V bv = *reinterpret_cast<const V*>(p.b + c0);
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const T vb = bv[k] / sp[k];
                const T rr = vb * sc[k] - bv[k];
                e += (c0 + k < p.m) ? rr * rr : (T)0;
            }
        }
        e = block_sum<T>(e, red);
        return p.err_squared ? (double)e : sqrt((double)e);
    };
    // column partials K_tile^T w -> atomics into sums buffer dst (this tile's columns)
    auto flush = [&](const T (&wr)[R], T* dst) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            V acc;
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                T sacc = 0;
#pragma unroll
                for (int r = 0; r < R; ++r) sacc += kv[r][g][k] * wr[r];
                acc[k] = sacc;
            }
            *reinterpret_cast<V*>(&colbuf[w][(lane + kWave * g) * VEC]) = acc;
        }
        __syncthreads();
        for (int q = tid; q < TL_C; q += blockDim.x) {
            T sacc = colbuf[0][q];
#pragma unroll
            for (int ww = 1; ww < NW; ++ww) sacc += colbuf[ww][q];
            if (col0 + q < p.m) atomicAdd(dst + (size_t)my_rep * p.m_pad + col0 + q, sacc);
        }
    };

    // slot k % 4 is free once iteration k - 1 has started (S[k-4] was last read in
    // iteration k - 3): this workgroup's share of it and its break counter, write-through
    auto zero_slot = [&](int k) {
        T* zs = p.cs + (size_t)(k & 3) * it_stride;
        const int64_t per = ((int64_t)it_stride + nwg - 1) / nwg;
        const int64_t z0 = (int64_t)blockIdx.x * per;
        const int64_t z1 = z0 + per < (int64_t)it_stride ? z0 + per : (int64_t)it_stride;
        for (int64_t j = z0 + tid; j < z1; j += (int)blockDim.x) store_wt(zs + j, (T)0);
        if (blockIdx.x == 0 && tid == 0) store_wt(p.bad_cnt + (k & 3) * 64, 0);
    };
    // ---- prologue: K^T u0 into sums[0]
    {
        T wr[R];
#pragma unroll
        for (int r = 0; r < R; ++r) wr[r] = (row0 + r < p.n) ? u0 : (T)0;
        flush(wr, p.cs);
    }
    int last_good = -1, niter = 0, status = OTF_SK_MAX_ITER, brk = -1, n_err = 0;
    bool done = false;
    if (tid == 0)
        __hip_atomic_fetch_add(p.sync.reg + xcd * 64, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!grid_barrier(p.bar, nwg, deadline, p.timeout_ticks, &s_flag, &p.info->stalled)) {
        status = OTF_SK_TIMEOUT;
        done = true;
    }
    if (tid == 0) {
        int nact = 0;
        unsigned mask = 0;
        for (int x = 0; x < 8; ++x) {
            const int c = __hip_atomic_load(p.sync.reg + x * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (c > 0) { ++nact; mask |= 1u << x; }
        }
        s_pop[0] = __hip_atomic_load(p.sync.reg + xcd * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_pop[1] = nact;
        s_pop[2] = (int)mask;
    }
    __syncthreads();
    const int nx = s_pop[0], nact = s_pop[1];
    const unsigned act_mask = (unsigned)s_pop[2];
    int* gcnt = p.grp + rb * 64;
    const int rowl = butterfly_row<R>(lane);  // row whose wave total this lane holds

    for (int it = 0; it < p.max_iter && !done; ++it) {
        OTF_STAMP(it, 0);
        // a numerical break in iteration it-1 (v or u, any tile) -> revert to it-2.  The
        // flag load is issued together with the sum loads (one memory round trip, not two).
        const int prev_bad = it >= 1 ? load_agent(p.bad_cnt + ((it - 1) & 3) * 64) : 0;
        T s[G][VEC], vn[G][VEC];
        load_sums(p.cs + (size_t)(it & 3) * it_stride, s, (T)1);
        if (prev_bad > 0) {
            last_good = it - 2; niter = it - 1; status = OTF_SK_NUMERICAL_BREAK; brk = it - 1;
            break;
        }
        int badv = 0;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const V bv = *reinterpret_cast<const V*>(p.b + colc[g]);  // target marginal (L1/L2)
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const T val = bv[k] / s[g][k];
                badv |= (cok[g][k] && ((s[g][k] == (T)0) || !finite_val(val))) ? 1 : 0;
                vn[g][k] = cok[g][k] ? val : (T)0;
            }
        }
        // marginal error of iterate it-1 from the full sum vectors (same in every tile)
        if (it >= 1 && ((it - 1) % p.check_every) == 0) {
            const double err = full_error(it - 1);
            if (lead) p.errlog[(it - 1) / p.check_every] = err;
            n_err = (it - 1) / p.check_every + 1;
            if (p.err_squared ? !(err > p.stop_thr) : (err < p.stop_thr)) {
                last_good = it - 1; niter = it - 1; status = OTF_SK_CONVERGED;
                break;
            }
        }
        if (__any(badv) && lane == 0) atomicAdd(p.bad_cnt + (it & 3) * 64, 1);
        OTF_STAMP(it, 1);
        // row partials over this tile's columns, wave totals, publish to the group
        T rp[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            T acc = 0;
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int k = 0; k < VEC; ++k) acc += kv[r][g][k] * vn[g][k];
            rp[r] = acc;
        }
        wave_sum_multi<T, R>(rp, lane);
        const int slot = it & 1;
        T tot = 0;
        if (p.ncb == 1) {  // the tile spans whole rows: the wave totals are the row sums
            if (lane < R) urow[w][rowl] = rp[0];
            __builtin_amdgcn_wave_barrier();
            tot = urow[w][lane & (R - 1)];
            __builtin_amdgcn_wave_barrier();
            OTF_STAMP(it, 2);
        } else {
            T* xg = p.xch + ((size_t)slot * p.nrb + rb) * (size_t)p.ncb * TR;
            if (lane < R) store_wt(xg + (size_t)cb * TR + w * R + rowl, rp[0]);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {
                int ok = 1;
                __hip_atomic_fetch_add(gcnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const int target = p.ncb * (it + 1);
                while (load_agent(gcnt) < target) {
                    __builtin_amdgcn_s_sleep(1);
                    if (__builtin_amdgcn_s_memrealtime() > deadline) { ok = 0; break; }
                }
                s_flag = ok;
            }
            __syncthreads();
            if (!s_flag) { status = OTF_SK_TIMEOUT; done = true; break; }
            deadline = __builtin_amdgcn_s_memrealtime() + p.timeout_ticks;
            OTF_STAMP(it, 2);
            // gather the ncb partials of this wave's rows (fixed order)
            const int rr = lane & (R - 1);
            for (int mb = lane / R; mb < p.ncb; mb += kWave / R)
                tot += __hip_atomic_load(xg + (size_t)mb * TR + w * R + rr, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
            wave_sum_from<T, R>(tot);
        }
        if (lane < R) {
            const int rr = lane;
            const bool rok = row0 + rr < p.n;
            T un = (T)1 / (tot * ia_mine);
            if (!rok) un = 0;
            urow[w][rr] = un;
            uhist[slot][w * R + rr] = un;
        }
        __builtin_amdgcn_wave_barrier();  // wave-private LDS hand-off (in-order LDS queue)
        T un[R];
        int badu = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            un[r] = urow[w][r];
            badu |= (row0 + r < p.n && !finite_val(un[r])) ? 1 : 0;
        }
        if (badu && lane == 0) atomicAdd(p.bad_cnt + (it & 3) * 64, 1);
        if (w == 0) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                V vv;
#pragma unroll
                for (int q = 0; q < VEC; ++q) vv[q] = vn[g][q];
                *reinterpret_cast<V*>(&vhist[slot][(lane + kWave * g) * VEC]) = vv;
            }
        }
        OTF_STAMP(it, 3);
        flush(un, p.cs + (size_t)((it + 1) & 3) * it_stride);
        zero_slot(it + 2);
#ifdef OTF_STAMPS
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        OTF_STAMP(it, 4);
#endif
        if (!xcd_barrier(p.sync, xcd, nx, nact, act_mask, it + 1, deadline, p.timeout_ticks, &s_flag)) {
            status = OTF_SK_TIMEOUT;
            done = true;
        }
        OTF_STAMP(it, 5);
    }
    if (status == OTF_SK_MAX_ITER && p.max_iter > 0) {
        const int it = p.max_iter - 1;
        if (load_agent(p.bad_cnt + (it & 3) * 64) > 0) {
            last_good = it - 1; niter = it; status = OTF_SK_NUMERICAL_BREAK; brk = it;
        } else {
            last_good = it; niter = it;
            if ((it % p.check_every) == 0) {
                const double err = full_error(it);
                if (lead) p.errlog[it / p.check_every] = err;
                n_err = it / p.check_every + 1;
                if (p.err_squared ? !(err > p.stop_thr) : (err < p.stop_thr)) status = OTF_SK_CONVERGED;
            }
        }
    }

    // ---- outputs: (u, v) of last_good from the histories, plan from registers
    __syncthreads();
    const int hs = last_good & 1;
    T uo[R], vo[G][VEC];
#pragma unroll
    for (int r = 0; r < R; ++r) uo[r] = last_good < 0 ? u0 : uhist[hs][w * R + r];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int k = 0; k < VEC; ++k)
            vo[g][k] = last_good < 0 ? v0 : vhist[hs][(lane + kWave * g) * VEC + k];
    if (cb == 0 && lane < R && row0 + lane < p.n) {
        T mine = uo[0];
#pragma unroll
        for (int r = 1; r < R; ++r) if (lane == r) mine = uo[r];
        p.u_out[row0 + lane] = mine;
    }
    if (rb == 0 && w == 0) {
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int k = 0; k < VEC; ++k)
                if (cok[g][k]) p.v_out[colc[g] + k] = vo[g][k];
    }
    if (p.P) {
        TP* P = (TP*)p.P;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (row0 + r >= p.n) break;
            TP* prow = P + (int64_t)(row0 + r) * p.ldp;
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const int c0 = col0 + (lane + kWave * g) * VEC;
                if (c0 >= p.m) continue;
                VP o;
#pragma unroll
                for (int k = 0; k < VEC; ++k) o[k] = (TP)(uo[r] * kv[r][g][k] * vo[g][k]);
                if (c0 + VEC <= p.m) {
                    *reinterpret_cast<VP*>(prow + c0) = o;
                } else {
#pragma unroll
                    for (int k = 0; k < VEC; ++k)
                        if (c0 + k < p.m) prow[c0 + k] = o[k];
                }
            }
        }
    }
    if (status == OTF_SK_TIMEOUT && threadIdx.x == 0) mark_stalled(&p.info->stalled, kStallMid);
    if (lead) {
        p.info->last_good = last_good;
        p.info->niter = niter;
        p.info->status = status;
        p.info->break_iter = brk;
        p.info->n_err = n_err;
        p.info->engine = OTF_ENGINE_TILED;
        p.info->stop = 1;
    }
}

struct PassCfg {
    int G, R, NT;
};

// Register budget: 512-thread workgroups, one per CU (2 waves per SIMD -> up to 256
// VGPRs); each thread keeps R * G * VEC cost values of its row block live between
// the row reduction and the column update (<= 128 floats / 32 doubles).
constexpr int kPassThreads = 512;
constexpr int kMaxG = 8;

template <typename T> constexpr int pass_rows(int G) {
    return sizeof(T) == 4 ? (G == 1 ? 16 : G == 8 ? 2 : 128 / (G * 4)) : (G == 1 ? 16 : 32 / (G * 2));
}

template <typename T> PassCfg pick_cfg(int m) {
    constexpr int VEC = Vec<T>::N;
    const int chunks = (m + VEC - 1) / VEC;
    int G = 1;
    while (G < kMaxG && (chunks + G - 1) / G > kPassThreads) G *= 2;
    int nt = (chunks + G - 1) / G;
    nt = ((nt + 63) / 64) * 64;
    if (nt < 64) nt = 64;
    return {G, pass_rows<T>(G), nt};
}

// Row blocks of the pass/resident kernels for an n x m problem (host-side, no device).
template <typename T> int64_t row_blocks(int64_t n, int64_t m) {
    constexpr int64_t mmax = (int64_t)kPassThreads * kMaxG * Vec<T>::N;
    const PassCfg c = pick_cfg<T>((int)(m < 1 ? 1 : m > mmax ? mmax : m));
    return (n + c.R - 1) / c.R;
}

template <typename T, typename CT, bool LOG, bool SH>
hipError_t launch_pass_sh(const PassCfg& c, int grid, const SkArgs<T>& p, hipStream_t s) {
    switch (c.G) {
        case 1: sk_pass_kernel<T, CT, LOG, 1, pass_rows<T>(1), SH><<<grid, c.NT, 0, s>>>(p); break;
        case 2: sk_pass_kernel<T, CT, LOG, 2, pass_rows<T>(2), SH><<<grid, c.NT, 0, s>>>(p); break;
        case 4: sk_pass_kernel<T, CT, LOG, 4, pass_rows<T>(4), SH><<<grid, c.NT, 0, s>>>(p); break;
        case 8: sk_pass_kernel<T, CT, LOG, 8, pass_rows<T>(8), SH><<<grid, c.NT, 0, s>>>(p); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
// the shifted-kernel instance when the args carry offsets (float POT only)
template <typename T, typename CT, bool LOG>
hipError_t launch_pass(const PassCfg& c, int grid, const SkArgs<T>& p, hipStream_t s) {
    if constexpr (!LOG && sizeof(T) == 4)
        if (p.shA) return launch_pass_sh<T, CT, LOG, true>(c, grid, p, s);
    return launch_pass_sh<T, CT, LOG, false>(c, grid, p, s);
}

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct Workspace {
    void* a_pad;
    void* b_pad;
    void* cs;
    void* u2;
    void* v2;
    int64_t cs_stride;  // m_pad + 64: the break-count slot and alignment
    int* cmin_key;
    int* relay;         // the relay fallback's counters (kRelayInts, zeroed by the init kernel)
    double* errlog;
    void* res;        // resident / tiled engines: 4-slot sums ring | bad_cnt ring | barrier
    size_t res_bytes;
    void* sweep;      // sweep engine region (otf_sweep.hip)
    size_t sweep_bytes;
    void* gather;     // gather engine granules (otf_gather.hip); 0 bytes if not taken
    size_t gather_bytes;
    void* mesh;       // mesh engine granules (otf_mesh.hip); 0 bytes if not taken
    size_t mesh_bytes;
    // shifted kernel (float only): row / column exponent offsets, initial scalings, and the
    // column pass's chunk partials
    float* shA;
    float* shB;
    float* u0v;
    float* v0v;
    float* shpart;
    int nrep;
    size_t bytes;     // required: every engine but the float64 K stream
    void* kbuf;       // float64: K (n x m_pad) for the sweep engine's K stream, past `bytes`
    size_t bytes_k;   // bytes + the K buffer (what otf_sinkhorn_workspace_size asks for)
    int64_t m_pad;
    int64_t t_nrb, t_ncb;  // tiled engine: row / column tiles
    size_t t_xch_off;      // tiled engine: exchange region offset inside res
};

// tiled engine row exchange: two slots (iteration parity) of nrb x ncb x tile-rows partials
size_t tiled_xch_bytes(int64_t nrb, int64_t ncb, size_t esz) {
    return align_up(2 * (size_t)nrb * ncb * tile_rows(esz) * esz, 256);
}


// Column-sum replicas of the resident engine (grids of >= 128 row blocks; workgroups
// add into replica xcc_id % NREP, readers load all NREP replicas at once).  A
// function of the shape only, so the workspace size needs no device.
#ifndef OTF_RES_NREP
#define OTF_RES_NREP 4
#endif
int res_replicas(int64_t nrb) { return nrb >= 128 ? OTF_RES_NREP : 1; }

// Largest grid the resident / tiled engines are sized for (one workgroup per CU; the
// workspace size is a function of the shape only, so it cannot ask the device).
constexpr int64_t kMaxResidentWG = 1024;

Workspace carve(void* base, int64_t n, int64_t m, size_t esz, int max_iter, int64_t nrb) {
    Workspace w{};
    size_t off = 0;
    auto take = [&](size_t bytes) {
        void* p = base ? (char*)base + off : nullptr;
        off = align_up(off + bytes, 256);
        return p;
    };
    w.m_pad = (int64_t)align_up((size_t)m, 64);
    w.a_pad = take(n * esz);
    w.b_pad = take(w.m_pad * esz);
    w.cs_stride = w.m_pad + 64;
    w.cs = take(3 * w.cs_stride * esz);
    w.u2 = take(2 * n * esz);
    w.v2 = take(2 * w.m_pad * esz);
    w.cmin_key = (int*)take(sizeof(int) * (size_t)w.m_pad);
    w.relay = (int*)take(sizeof(int) * kRelayInts);
    w.errlog = (double*)take(sizeof(double) * (size_t)(max_iter + 2));
    w.nrep = res_replicas(nrb);
    // per-iteration sums live in a ring of 4 slots: O(m) whatever max_iter is
    w.res_bytes = align_up(4 * (size_t)w.nrep * w.m_pad * esz, 256) + 4 * 256 + 256 + kSyncBytes;
    // tiled engine: row-partial exchange (2 slots x nrb x ncb x tile rows) + group counters,
    // only for shapes whose tiles can all be resident (<= kMaxResidentWG)
    w.t_nrb = (n + tile_rows(esz) - 1) / tile_rows(esz);
    w.t_ncb = (m + TL_C - 1) / TL_C;
    w.t_xch_off = w.res_bytes;
    if (w.t_nrb * w.t_ncb <= kMaxResidentWG)
        w.res_bytes += tiled_xch_bytes(w.t_nrb, w.t_ncb, esz) + (size_t)w.t_nrb * 256;
    w.res = take(w.res_bytes);
    w.sweep_bytes = esz == 8 ? sweep_region_bytes<double>(w.m_pad) : sweep_region_bytes<float>(w.m_pad);
    w.sweep = take(w.sweep_bytes);
    w.gather_bytes = esz == 8 ? gather_region_bytes<double>(n, m) : gather_region_bytes<float>(n, m);
    w.gather = take(w.gather_bytes);
    w.mesh_bytes = esz == 4 ? mesh_region_bytes(n, m) : mesh64_region_bytes(n, m);
    w.mesh = take(w.mesh_bytes);
    if (esz == 4) {
        w.shA = (float*)take(sizeof(float) * (size_t)n);
        w.u0v = (float*)take(sizeof(float) * (size_t)n);
        w.shB = (float*)take(sizeof(float) * (size_t)w.m_pad);
        w.v0v = (float*)take(sizeof(float) * (size_t)w.m_pad);
        w.shpart = (float*)take(2 * sizeof(float) * (size_t)shift_chunks(n) * w.m_pad);
    }
    w.bytes = off;
    // float64: the sweep engine streams K = exp(-C / reg) written once by its prologue
    // (POT materialises K too) when the caller's workspace reaches this far; a workspace of
    // `bytes` still runs every engine (the sweep then recomputes the exp per sweep).  Only
    // for costs past 64 MiB: below that the register-resident engines take float64 K
    const size_t kb = (size_t)n * (size_t)w.m_pad * esz;
    w.kbuf = (esz == 8 && kb > ((size_t)64 << 20)) ? take(kb) : nullptr;
    w.bytes_k = off;
    return w;
}

// Plain launch of the persistent grid after an explicit residency check (every
// workgroup must be resident at once for the in-kernel barrier; plain and cooperative
// launches get identical residency, and a plain launch replays in a graph at no
// extra cost).  Every spin in the kernel is bounded, so a grid that cannot become
// resident (another persistent kernel on the device) ends in OTF_SK_TIMEOUT.
template <typename T, typename CT, typename TP, int G, int R>
hipError_t launch_resident_g(int grid, int nt, SkResArgs<T>& p, hipStream_t s) {
    void* args[] = {&p};
    const void* k = p.nrep == 1 ? (const void*)sk_resident_kernel<T, CT, TP, G, R, 1>
                                : (const void*)sk_resident_kernel<T, CT, TP, G, R, OTF_RES_NREP>;
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, nt, 0);
    if (e != hipSuccess) return e;
    if (per_cu < 1 || grid > per_cu * device_cu_count()) return hipErrorCooperativeLaunchTooLarge;
    return hipLaunchKernel(k, dim3(grid), dim3(nt), args, 0, s);
}

template <typename T, typename CT, typename TP>
hipError_t launch_resident(const PassCfg& c, int grid, SkResArgs<T>& p, hipStream_t s) {
    switch (c.G) {
        case 1: return launch_resident_g<T, CT, TP, 1, pass_rows<T>(1)>(grid, c.NT, p, s);
        case 2: return launch_resident_g<T, CT, TP, 2, pass_rows<T>(2)>(grid, c.NT, p, s);
        case 4: return launch_resident_g<T, CT, TP, 4, pass_rows<T>(4)>(grid, c.NT, p, s);
        default: return hipErrorInvalidValue;
    }
}

// Resident solve.  Returns hipSuccess, or the launch error (the caller then falls
// back to the streaming engine — nothing has been enqueued in that case).
template <typename T, typename CT>
hipError_t run_resident(const PassCfg& cfg, int grid, const CT* C, int64_t ldc, int n, int m,
                        const T* cost_scale, const otf_sinkhorn_opts& o, Workspace& w, T* u_out,
                        T* v_out, void* P_out, int64_t ldp, int P_dtype, otf_sinkhorn_info* info,
                        double* errlog, hipStream_t s, bool ott = false) {
    SkResArgs<T> p{};
    p.ott = ott ? 1 : 0;
    p.C = C;
    p.ldc = ldc;
    p.n = n;
    p.m = m;
    p.m_pad = (int)w.m_pad;
    p.a = (const T*)w.a_pad;
    p.b = (const T*)w.b_pad;
    p.cost_scale = cost_scale;
    p.reg = o.reg;
    p.max_iter = o.max_iter;
    p.check_every = o.check_every;
    p.err_squared = o.err_squared;
    p.stop_thr = o.stop_thr;
    p.cs = (T*)w.res;
    p.nrep = w.nrep;
    p.bad_cnt = (int*)((char*)w.res + align_up(4 * (size_t)w.nrep * w.m_pad * sizeof(T), 256));
    p.bar = (int*)((char*)p.bad_cnt + 4 * 256);
    p.sync = sync_words((int*)((char*)p.bar + 256));
    p.info = info;
    p.errlog = errlog;
    p.u_out = u_out;
    p.v_out = v_out;
    p.P = P_out;
    p.ldp = ldp;
    p.p_f64 = P_dtype == OTF_F64;
    p.timeout_ticks = stall_ticks();
    p.reg_ticks = reg_stall_ticks();
    hipError_t e = hipMemsetAsync(w.res, 0, w.res_bytes, s);
    if (e != hipSuccess) return e;
    if (P_out && P_dtype == OTF_F64) return launch_resident<T, CT, double>(cfg, grid, p, s);
    return launch_resident<T, CT, float>(cfg, grid, p, s);
}

// Tiled resident solve.  Same contract as run_resident.
template <typename T, typename CT, typename TP, int NREP>
hipError_t launch_tiled_g(int grid, SkTileArgs<T>& p, hipStream_t s) {
    void* args[] = {&p};
    const void* k = (const void*)sk_tiled_kernel<T, CT, TP, NREP>;
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 512, 0);
    if (e != hipSuccess) return e;
    if (per_cu < 1 || grid > per_cu * device_cu_count()) return hipErrorCooperativeLaunchTooLarge;
    return hipLaunchKernel(k, dim3(grid), dim3(512), args, 0, s);
}

template <typename T, typename CT>
hipError_t run_tiled(const CT* C, int64_t ldc, int n, int m, const T* cost_scale,
                     const otf_sinkhorn_opts& o, Workspace& w, T* u_out, T* v_out,
                     void* P_out, int64_t ldp, int P_dtype, otf_sinkhorn_info* info,
                     double* errlog, hipStream_t s) {
    SkTileArgs<T> p{};
    const int nrep = 1;
    p.C = C;
    p.ldc = ldc;
    p.n = n;
    p.m = m;
    p.m_pad = (int)w.m_pad;
    p.a = (const T*)w.a_pad;
    p.b = (const T*)w.b_pad;
    p.cost_scale = cost_scale;
    p.reg = o.reg;
    p.max_iter = o.max_iter;
    p.check_every = o.check_every;
    p.err_squared = o.err_squared;
    p.stop_thr = o.stop_thr;
    p.cs = (T*)w.res;
    p.nrep = nrep;
    p.bad_cnt = (int*)((char*)w.res + align_up(4 * (size_t)w.nrep * w.m_pad * sizeof(T), 256));
    p.bar = (int*)((char*)p.bad_cnt + 4 * 256);
    p.sync = sync_words((int*)((char*)p.bar + 256));
    p.xch = (T*)((char*)w.res + w.t_xch_off);
    p.grp = (int*)((char*)p.xch + tiled_xch_bytes(w.t_nrb, w.t_ncb, sizeof(T)));
    p.nrb = (int)w.t_nrb;
    p.ncb = (int)w.t_ncb;
    p.info = info;
    p.errlog = errlog;
    p.u_out = u_out;
    p.v_out = v_out;
    p.P = P_out;
    p.ldp = ldp;
    p.timeout_ticks = stall_ticks();
    p.reg_ticks = reg_stall_ticks();
    hipError_t e = hipMemsetAsync(w.res, 0, w.res_bytes, s);
    if (e != hipSuccess) return e;
    const int grid = (int)(w.t_nrb * w.t_ncb);
    const bool f64p = P_out && P_dtype == OTF_F64;
    if constexpr (sizeof(T) == 4) {
        if (nrep == 4) return f64p ? launch_tiled_g<T, CT, double, 4>(grid, p, s) : launch_tiled_g<T, CT, float, 4>(grid, p, s);
        if (nrep == 2) return f64p ? launch_tiled_g<T, CT, double, 2>(grid, p, s) : launch_tiled_g<T, CT, float, 2>(grid, p, s);
    }
    return f64p ? launch_tiled_g<T, CT, double, 1>(grid, p, s) : launch_tiled_g<T, CT, float, 1>(grid, p, s);
}

// Validated shape / workspace of one solve (deterministic in n, m, max_iter).
template <typename T> struct SkSetup {
    PassCfg cfg;
    int nrb, grid, m_pad;
    Workspace w;
};

template <typename T, typename CT>
int sk_prepare(const void* a, const void* b, const CT* C, int64_t n, int64_t m, int64_t ldc,
               const otf_sinkhorn_opts& o, const otf_sinkhorn_info* info, void* ws,
               size_t ws_bytes, SkSetup<T>& su) {
    constexpr int VEC = Vec<T>::N;
    if (n <= 0 || m <= 0 || !a || !b || !C || !info || !ws) return OTF_EINVAL;
    if (ldc < m || ldc % VEC != 0 || ((uintptr_t)C % 16) != 0) return OTF_EINVAL;
    if (!(o.reg > 0.0) || o.max_iter < 0 || o.check_every <= 0) return OTF_EINVAL;
    if (n > INT32_MAX || m > (int64_t)kPassThreads * kMaxG * VEC) return OTF_EUNSUPPORTED;
    su.cfg = pick_cfg<T>((int)m);
    su.nrb = (int)((n + su.cfg.R - 1) / su.cfg.R);
    su.w = carve(ws, n, m, sizeof(T), o.max_iter, su.nrb);
    if (ws_bytes < su.w.bytes) return OTF_EINVAL;
    su.m_pad = (int)su.w.m_pad;
    su.grid = su.nrb < device_cu_count() ? su.nrb : device_cu_count();
    return OTF_OK;
}

template <typename T, typename CT, bool LOG>
SkArgs<T> sk_args(const SkSetup<T>& su, const CT* C, int64_t ldc, int64_t n, int64_t m,
                  const T* cost_scale, const otf_sinkhorn_opts& o, otf_sinkhorn_info* info,
                  double* errlog, bool profile) {
    SkArgs<T> p{};
    p.C = C;
    p.ldc = ldc;
    p.n = (int)n;
    p.n_total = o.n_total > 0 ? o.n_total : (int)n;
    p.m = (int)m;
    p.a = (const T*)su.w.a_pad;
    p.b = (const T*)su.w.b_pad;
    p.cost_scale = cost_scale;
    p.reg = o.reg;
    p.cmin_key = su.w.cmin_key;
    p.info = info;
    p.errlog = errlog ? errlog : su.w.errlog;
    p.stop_thr = profile ? -1.0 : o.stop_thr;
    p.check_every = o.check_every;
    p.check_off = LOG ? 1 : 0;
    p.err_squared = LOG ? 0 : o.err_squared;
    p.m_pad = su.m_pad;
    if constexpr (!LOG && sizeof(T) == 4) {
        if (o.shift) {
            p.shA = (const T*)su.w.shA;
            p.shB = (const T*)su.w.shB;
            p.u0v = (const T*)su.w.u0v;
            p.v0v = (const T*)su.w.v0v;
        }
    }
    return p;
}

// Buffers of pass `pass` (iteration it = pass - 1; pass 0 is the prologue).
template <typename T>
void sk_set_pass(SkArgs<T>& p, const SkSetup<T>& su, int pass) {
    T* cs = (T*)su.w.cs;
    T* u2 = (T*)su.w.u2;
    T* v2 = (T*)su.w.v2;
    const size_t st = (size_t)su.w.cs_stride;
    const int it = pass - 1;
    p.it = it;
    p.cs_src = pass >= 1 ? cs + (size_t)((pass - 1) % 3) * st : nullptr;
    p.cs_dst = cs + (size_t)(pass % 3) * st;
    p.cs_zero = cs + (size_t)((pass + 1) % 3) * st;
    // iteration it writes slot (it & 1); the prologue (it = -1) writes slot 1 (OTT g_{-1})
    p.u_cur = u2 + (size_t)(it & 1) * p.n;
    p.v_cur = v2 + (size_t)(it & 1) * su.m_pad;
    p.u_prev = u2 + (size_t)((it - 1) & 1) * p.n;
    p.v_prev = v2 + (size_t)((it - 1) & 1) * su.m_pad;
}

template <typename T>
int sk_init(const SkSetup<T>& su, const T* a, const T* b, int64_t n, int64_t m,
            otf_sinkhorn_info* info, hipStream_t s, void* zero = nullptr, size_t zero_bytes = 0) {
    const int grid = zero_bytes > (1u << 20) ? 256 : 64;
    sk_init_kernel<T><<<grid, 256, 0, s>>>(a, b, (int)n, (int)m, su.m_pad, (T*)su.w.a_pad,
                                           (T*)su.w.b_pad, (T*)su.w.cs, (int)su.w.cs_stride,
                                           (T*)su.w.u2, (T*)su.w.v2, su.w.cmin_key, info,
                                           (uint4*)zero, (int64_t)(zero_bytes / 16), su.w.relay);
    OTF_HIP(hipGetLastError());
    return OTF_OK;
}

// After the last pass: decide the last iteration, write (u, v) and the plan.
template <typename T, typename CT, bool LOG>
int sk_finish(SkArgs<T>& p, const SkSetup<T>& su, const CT* C, int64_t ldc, int64_t n, int64_t m,
              const T* cost_scale, const otf_sinkhorn_opts& o, T* u_out, T* v_out, void* P_out,
              int64_t ldp, int P_dtype, otf_sinkhorn_info* info, hipStream_t s) {
    // pass max_iter (iteration max_iter-1) accumulated into cs[max_iter % 3]
    sk_set_pass(p, su, o.max_iter + 1);
    p.it = o.max_iter - 1;
    p.v_cur = (T*)su.w.v2 + (size_t)(p.it & 1) * su.m_pad;
    sk_finalize_kernel<T, LOG><<<1, 512, 0, s>>>(p, o.max_iter);
    OTF_HIP(hipGetLastError());
    sk_output_kernel<T, LOG><<<64, 256, 0, s>>>((const T*)su.w.u2, (const T*)su.w.v2, (int)n,
                                                p.n_total, (int)m, su.m_pad, info, u_out, v_out,
                                                p.u0v, p.v0v);
    OTF_HIP(hipGetLastError());
    if (P_out) {
        const int pgrid = n < 4096 ? (int)n : 4096;
        if (P_dtype == OTF_F32)
            sk_plan_kernel<T, CT, float, LOG><<<pgrid, 256, 0, s>>>(C, ldc, (int)n, (int)m, u_out, v_out,
                                                                   cost_scale, o.reg, (float*)P_out, ldp,
                                                                   p.shA, p.shB);
        else
            sk_plan_kernel<T, CT, double, LOG><<<pgrid, 256, 0, s>>>(C, ldc, (int)n, (int)m, u_out,
                                                                    v_out, cost_scale, o.reg,
                                                                    (double*)P_out, ldp, p.shA, p.shB);
        OTF_HIP(hipGetLastError());
    }
    return OTF_OK;
}

// OTF_FORCE_REG_GIVEUP=1 (tests, probes; read per call): every persistent launch (the
// engines below and the fused pairwise launches) is replaced by a registration give-up, so
// the relay fallback runs the solve at the caller's full shape without a contending grid
inline bool force_giveup() {
    const char* e = getenv("OTF_FORCE_REG_GIVEUP");
    return e && atoi(e) != 0;
}
__global__ void sk_giveup_kernel(otf_sinkhorn_info* info) {
    if (threadIdx.x == 0) mark_stalled(&info->stalled, kStallRegistration);
}
inline hipError_t forced_giveup(otf_sinkhorn_info* info, hipStream_t s) {
    sk_giveup_kernel<<<1, 64, 0, s>>>(info);
    return hipGetLastError();
}

// The relay fallback behind a persistent engine launch (sk_relay_kernel): one no-op dispatch
// unless the persistent solve's registration gave up.  pw: the pairwise float64 form (the
// relay builds the cost into C = the workspace's n x m float64 buffer, then K over it).
template <typename T, typename CT>
hipError_t launch_solo(const SkSetup<T>& su, const CT* C, int64_t ldc, int64_t n, int64_t m,
                       const T* cost_scale, const otf_sinkhorn_opts& o, T* u_out, T* v_out,
                       void* P_out, int64_t ldp, int P_dtype, otf_sinkhorn_info* info,
                       double* errlog, hipStream_t s, const SoloArgs<T>* pw = nullptr) {
    SkArgs<T> p = sk_args<T, CT, false>(su, C, ldc, n, m, cost_scale, o, info, errlog, false);
    SoloArgs<T> x{};
    if (pw) x = *pw;
    x.cs = (T*)su.w.cs;
    x.u2 = (T*)su.w.u2;
    x.v2 = (T*)su.w.v2;
    x.cs_stride = su.w.cs_stride;
    x.max_iter = o.max_iter;
    x.u_out = u_out;
    x.v_out = v_out;
    x.P = P_out;
    x.ldp = ldp;
    x.p_f64 = P_dtype == OTF_F64 ? 1 : 0;
    x.v0v = p.v0v;
    x.relay = su.w.relay;
    x.stall = stall_ticks();
    // one piece per pass-launch workgroup; the ticket count (reset + cost tiles + K + passes +
    // finalize + outputs) stays inside the int counters
    const int64_t per = (int64_t)o.max_iter + 4;
    int64_t vg = su.grid;
    const int64_t room = ((int64_t)1 << 30) - (pw ? pw->pw_ntiles : 0);
    if (vg * per > room) vg = room / per;
    if (vg < 1) return hipErrorInvalidValue;
    x.vg = (int)vg;
    const int grid = (int)vg;
    const PassCfg& c = su.cfg;
    if constexpr (std::is_same<CT, T>::value) {
        if (pw) {
            p.cost_scale = nullptr;  // the relay's passes run on K (max applied when K is formed)
            switch (c.G) {
                case 1: sk_relay_kernel<T, CT, 1, pass_rows<T>(1), false, true><<<grid, c.NT, 0, s>>>(p, x); break;
                case 2: sk_relay_kernel<T, CT, 2, pass_rows<T>(2), false, true><<<grid, c.NT, 0, s>>>(p, x); break;
                case 4: sk_relay_kernel<T, CT, 4, pass_rows<T>(4), false, true><<<grid, c.NT, 0, s>>>(p, x); break;
                case 8: sk_relay_kernel<T, CT, 8, pass_rows<T>(8), false, true><<<grid, c.NT, 0, s>>>(p, x); break;
                default: return hipErrorInvalidValue;
            }
            return hipGetLastError();
        }
    }
    if (p.shA) {
        if constexpr (sizeof(T) == 4) {
            switch (c.G) {
                case 1: sk_relay_kernel<T, CT, 1, pass_rows<T>(1), true, false><<<grid, c.NT, 0, s>>>(p, x); break;
                case 2: sk_relay_kernel<T, CT, 2, pass_rows<T>(2), true, false><<<grid, c.NT, 0, s>>>(p, x); break;
                case 4: sk_relay_kernel<T, CT, 4, pass_rows<T>(4), true, false><<<grid, c.NT, 0, s>>>(p, x); break;
                case 8: sk_relay_kernel<T, CT, 8, pass_rows<T>(8), true, false><<<grid, c.NT, 0, s>>>(p, x); break;
                default: return hipErrorInvalidValue;
            }
            return hipGetLastError();
        }
    }
    switch (c.G) {
        case 1: sk_relay_kernel<T, CT, 1, pass_rows<T>(1), false, false><<<grid, c.NT, 0, s>>>(p, x); break;
        case 2: sk_relay_kernel<T, CT, 2, pass_rows<T>(2), false, false><<<grid, c.NT, 0, s>>>(p, x); break;
        case 4: sk_relay_kernel<T, CT, 4, pass_rows<T>(4), false, false><<<grid, c.NT, 0, s>>>(p, x); break;
        case 8: sk_relay_kernel<T, CT, 8, pass_rows<T>(8), false, false><<<grid, c.NT, 0, s>>>(p, x); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// The shifted kernel's offsets (opts.shift): column log-sum-exp pass, merge, row max pass.
// Runs after sk_init (b_pad holds b).  float compute only.
template <typename CT>
int sk_shift_prepass(const SkSetup<float>& su, const CT* C, int64_t ldc, int64_t n, int64_t m,
                     int n_total, const float* cost_scale, double reg, hipStream_t s) {
    const int nch = shift_chunks(n);
    const int m_pad = su.m_pad;
    float* pmax = su.w.shpart;
    float* psum = su.w.shpart + (size_t)nch * m_pad;
    sk_shift_cols_kernel<CT><<<dim3((unsigned)((m_pad + 1023) / 1024), (unsigned)nch), 256, 0, s>>>(
        C, ldc, (int)n, (int)m, m_pad, cost_scale, reg, pmax, psum);
    OTF_HIP(hipGetLastError());
    sk_shift_merge_kernel<<<(m_pad + 255) / 256, 256, 0, s>>>(pmax, psum, nch, (int)m, m_pad,
                                                              (const float*)su.w.b_pad, n_total,
                                                              su.w.shB, su.w.v0v);
    OTF_HIP(hipGetLastError());
    const int64_t rg = (n + 3) / 4;
    sk_shift_rows_kernel<CT><<<(unsigned)(rg < 2048 ? rg : 2048), 256, 0, s>>>(
        C, ldc, (int)n, (int)m, cost_scale, reg, su.w.shB, n_total, su.w.shA, su.w.u0v);
    OTF_HIP(hipGetLastError());
    return OTF_OK;
}

// OTF_GATHER=0 keeps AUTO off the gather engine (A/B measurements); GATHER still forces it
inline bool gather_enabled() {
    static int env = -1;
    if (env < 0) {
        const char* e = getenv("OTF_GATHER");
        env = e ? atoi(e) : 1;
    }
    return env != 0;
}

// OTF_MESH=0 keeps AUTO off the mesh engine (A/B measurements); MESH still forces it
inline bool mesh_enabled() {
    static int env = -1;
    if (env < 0) {
        const char* e = getenv("OTF_MESH");
        env = e ? atoi(e) : 1;
    }
    return env != 0;
}

// float64 sweep engine: K streamed from the workspace (written by the prologue sweep) when
// the caller's workspace holds it; OTF_SWEEP_KSTREAM=0 recomputes the exp per sweep (A/B)
template <typename T> void* kstream_buf(const SkSetup<T>& su, size_t ws_bytes) {
    if (sizeof(T) != 8 || !su.w.kbuf || ws_bytes < su.w.bytes_k) return nullptr;
    const char* e = getenv("OTF_SWEEP_KSTREAM");  // read per call (a test switches it)
    return (e && atoi(e) == 0) ? nullptr : su.w.kbuf;
}

template <typename T, typename CT, bool LOG>
int run_sinkhorn(const T* a, const T* b, const CT* C, int64_t n, int64_t m, int64_t ldc,
                 const T* cost_scale, const otf_sinkhorn_opts& o, T* u_out, T* v_out, void* P_out,
                 int64_t ldp, int P_dtype, otf_sinkhorn_info* info, double* errlog_user,
                 void* ws, size_t ws_bytes, hipStream_t s, float* avg_pass_ms) {
    constexpr int VEC = Vec<T>::N;
    if (!u_out || !v_out) return OTF_EINVAL;
    if (P_out && (ldp < m || ldp % VEC != 0 || ((uintptr_t)P_out % 16) != 0)) return OTF_EINVAL;
    SkSetup<T> su;
    int rc = sk_prepare<T, CT>(a, b, C, n, m, ldc, o, info, ws, ws_bytes, su);
    if (rc != OTF_OK) return rc;
    double* errlog = errlog_user ? errlog_user : su.w.errlog;
    const bool whole = o.n_total <= 0 || o.n_total == n;
    // shifted kernel: float32 POT on the whole problem, mesh / sweep / stream engines
    const bool sh = o.shift != 0;
    if (sh && (LOG || sizeof(T) != 4 || !whole)) return OTF_EUNSUPPORTED;
    // the mesh engine's region is zeroed by the init kernel (no memset launch)
    // float64: the mesh engine's float64 form on a float64 cost of whole 128 x 512 tiles
    constexpr bool kMesh64 = sizeof(T) == 8 && std::is_same<CT, double>::value;
    bool mesh_shape_ok = false, mesh_auto_ok = true;
    if constexpr (sizeof(T) == 4) mesh_shape_ok = mesh_supported(n, m);
    else if constexpr (kMesh64) {
        mesh_shape_ok = !sh && mesh64_supported(n, m);
        // AUTO keeps the tiled engine while every float64 tile has its own CU (N <= 2048:
        // 7.36 vs 7.47 us per iteration at 2048^2, a shorter prologue); the float64 mesh
        // takes the shapes past it (N = 4096: the sweep engine otherwise)
        mesh_auto_ok = su.w.t_nrb * su.w.t_ncb > device_cu_count();
    }
    bool mesh_pick = false;
    if constexpr (sizeof(T) == 4 || kMesh64)
        mesh_pick = !LOG && !avg_pass_ms && whole && o.max_iter >= 1 && su.w.mesh_bytes > 0 &&
                    mesh_shape_ok &&
                    (o.engine == OTF_ENGINE_MESH || (o.engine == OTF_ENGINE_AUTO && mesh_enabled() && mesh_auto_ok &&
                                                     !(gather_supported<T>(n, m) && su.w.gather_bytes > 0)));
    // gather engine: small problems, one granule hop per iteration, no barrier (and
    // deterministic by construction); its region is zeroed by the init kernel too
    const bool gfits = !LOG && !sh && !avg_pass_ms && whole && o.max_iter >= 1 &&
                       gather_supported<T>(n, m) && su.w.gather_bytes > 0;
    const bool gather_pick = gfits && (o.engine == OTF_ENGINE_GATHER || (o.engine == OTF_ENGINE_AUTO && gather_enabled()));
    rc = sk_init<T>(su, a, b, n, m, info, s, mesh_pick ? su.w.mesh : gather_pick ? su.w.gather : nullptr,
                    mesh_pick ? su.w.mesh_bytes : gather_pick ? su.w.gather_bytes : 0);
    if (rc != OTF_OK) return rc;
    ShiftArgs shargs{};
    if constexpr (sizeof(T) == 4) {
        if (sh) {
            rc = sk_shift_prepass<CT>(su, C, ldc, n, m, (int)n, (const float*)cost_scale, o.reg, s);
            if (rc != OTF_OK) return rc;
            shargs = ShiftArgs{su.w.shA, su.w.shB, su.w.u0v, su.w.v0v};
        }
    }
    const ShiftArgs* shp = sh ? &shargs : nullptr;

    if (o.engine == OTF_ENGINE_GATHER && !gfits) return OTF_EUNSUPPORTED;
    if (gather_pick) {
        const hipError_t e = force_giveup() ? forced_giveup(info, s) : run_gather<T, CT>(C, ldc, (int)n, (int)m, (const T*)su.w.a_pad,
                                               (const T*)su.w.b_pad, cost_scale, o, su.w.gather, u_out,
                                               v_out, P_out, ldp, P_dtype, info, errlog,
                                               /*zeroed=*/true, s);
        if (e == hipSuccess) return check_hip(launch_solo<T, CT>(su, C, ldc, n, m, cost_scale, o, u_out, v_out, P_out, ldp, P_dtype, info, errlog, s));
        (void)hipGetLastError();
        if (o.engine == OTF_ENGINE_GATHER) return check_hip(e);
    }
    // mesh engine: float32 tiles of K in registers, three granule hops per iteration, no
    // atomics or barrier (deterministic by construction)
    bool mfits = false;
    if constexpr (sizeof(T) == 4 || kMesh64)
        mfits = !LOG && !avg_pass_ms && whole && o.max_iter >= 1 && mesh_shape_ok &&
                su.w.mesh_bytes > 0;
    if (o.engine == OTF_ENGINE_MESH && !mfits) return OTF_EUNSUPPORTED;
    if constexpr (kMesh64) {
        if (mfits && (o.engine == OTF_ENGINE_MESH || (o.engine == OTF_ENGINE_AUTO && mesh_enabled() && mesh_auto_ok))) {
            const hipError_t e = force_giveup() ? forced_giveup(info, s) : run_mesh64((const double*)C, ldc, (int)n, (int)m, (const double*)su.w.a_pad,
                                            (const double*)su.w.b_pad, (const double*)cost_scale, o, su.w.mesh,
                                            (double*)u_out, (double*)v_out, P_out, ldp, P_dtype, info, errlog,
                                            /*zeroed=*/mesh_pick, s);
            if (e == hipSuccess) return check_hip(launch_solo<T, CT>(su, C, ldc, n, m, cost_scale, o, u_out, v_out, P_out, ldp, P_dtype, info, errlog, s));
            (void)hipGetLastError();
            if (o.engine == OTF_ENGINE_MESH) return check_hip(e);
        }
    }
    if constexpr (sizeof(T) == 4) {
        if (mfits && (o.engine == OTF_ENGINE_MESH || (o.engine == OTF_ENGINE_AUTO && mesh_enabled()))) {
            const hipError_t e = force_giveup() ? forced_giveup(info, s) : run_mesh<CT>(C, ldc, (int)n, (int)m, (const float*)su.w.a_pad,
                                              (const float*)su.w.b_pad, cost_scale, o, su.w.mesh,
                                              u_out, v_out, P_out, ldp, P_dtype, info, errlog,
                                              /*zeroed=*/mesh_pick, s, shp);
            if (e == hipSuccess) return check_hip(launch_solo<T, CT>(su, C, ldc, n, m, cost_scale, o, u_out, v_out, P_out, ldp, P_dtype, info, errlog, s));
            (void)hipGetLastError();
            if (o.engine == OTF_ENGINE_MESH) return check_hip(e);
        }
    }
    // deterministic mode otherwise: the sweep engine reduces the column sums in a fixed order
    if (o.deterministic) {
        if (LOG || avg_pass_ms || !(o.engine == OTF_ENGINE_AUTO || o.engine == OTF_ENGINE_SWEEP) ||
            o.max_iter < 1 || !sweep_supported<T, CT>(n, m, ldc) || !whole)
            return OTF_EUNSUPPORTED;
        const hipError_t e = force_giveup() ? forced_giveup(info, s) : run_sweep<T, CT>(C, ldc, (int)n, (int)m, su.m_pad, (const T*)su.w.a_pad,
                                              (const T*)su.w.b_pad, cost_scale, o, su.w.sweep, u_out,
                                              v_out, P_out, ldp, P_dtype, info, errlog, s, nullptr, shp,
                                              kstream_buf(su, ws_bytes));
        if (e != hipSuccess) return check_hip(e);
        return check_hip(launch_solo<T, CT>(su, C, ldc, n, m, cost_scale, o, u_out, v_out, P_out, ldp, P_dtype, info, errlog, s));
    }
    // resident engine: the whole solve in one persistent launch when every row block
    // gets its own CU (POT flavour, no per-pass profiling requested)
    const bool fits = su.nrb <= device_cu_count() && su.cfg.G <= 4 && whole;
    // tiled engine: every (128 x 512 float / 64 x 512 double) tile on its own CU
    const bool tfits = whole && su.w.t_nrb * su.w.t_ncb <= device_cu_count() &&
                       su.w.t_nrb * su.w.t_ncb <= kMaxResidentWG;
    // AUTO takes it for float, and for the float64 whole-tile shapes the float64 mesh
    // leaves to it (every tile on its own CU, mesh_auto_ok false: 7.36 vs 7.47 us per
    // iteration at 2048^2).  Other float64 shapes (64-row tiles) measured no faster than
    // the row-block resident engine (config 2, d = 512: 12.8 vs 12.3 ms per step -- both
    // sit on the ~5 us grid-sync round trip per iteration); TILED forces it
    const bool want_tiled = !LOG && !sh && !avg_pass_ms && tfits && o.max_iter >= 1 &&
                            (o.engine == OTF_ENGINE_TILED ||
                             (o.engine == OTF_ENGINE_AUTO &&
                              (sizeof(T) == 4 || (kMesh64 && mesh_shape_ok && !mesh_auto_ok))));
    if (o.engine == OTF_ENGINE_TILED && (LOG || sh || !tfits)) return OTF_EUNSUPPORTED;
    if (want_tiled) {
        Workspace w = su.w;
        const hipError_t e = force_giveup() ? forced_giveup(info, s) : run_tiled<T, CT>(C, ldc, (int)n, (int)m, cost_scale, o, w, u_out, v_out,
                                              P_out, ldp, P_dtype, info, errlog, s);
        if (e == hipSuccess) return check_hip(launch_solo<T, CT>(su, C, ldc, n, m, cost_scale, o, u_out, v_out, P_out, ldp, P_dtype, info, errlog, s));
        (void)hipGetLastError();
        if (o.engine == OTF_ENGINE_TILED) return check_hip(e);
    }
    // AUTO reaches here only when the tiled engine did not take the solve (shape, dtype
    // or co-residency refused), so the row-block resident engine is the next choice
    const bool want_res = !LOG && !sh && !avg_pass_ms && fits && o.max_iter >= 1 &&
                          (o.engine == OTF_ENGINE_RESIDENT || o.engine == OTF_ENGINE_AUTO);
    // OTT flavour, float64, on request: the resident engine in scaling form (see
    // SkResArgs::ott for the range contract).  No one-workgroup fallback is queued (that
    // one is POT-flavour): a grid that cannot become co-resident ends in OTF_SK_TIMEOUT.
    if (LOG && o.engine == OTF_ENGINE_RESIDENT) {
        if (sizeof(T) != 8 || !fits || !whole || avg_pass_ms || o.max_iter < 1) return OTF_EUNSUPPORTED;
        Workspace w = su.w;
        return check_hip(run_resident<T, CT>(su.cfg, su.nrb, C, ldc, (int)n, (int)m, cost_scale, o, w,
                                             u_out, v_out, P_out, ldp, P_dtype, info, errlog, s,
                                             /*ott=*/true));
    }
    if (o.engine == OTF_ENGINE_RESIDENT && (LOG || sh || !fits)) return OTF_EUNSUPPORTED;
    if (want_res) {
        Workspace w = su.w;
        const hipError_t e = force_giveup() ? forced_giveup(info, s) : run_resident<T, CT>(su.cfg, su.nrb, C, ldc, (int)n, (int)m, cost_scale,
                                                 o, w, u_out, v_out, P_out, ldp, P_dtype, info,
                                                 errlog, s);
        if (e == hipSuccess) return check_hip(launch_solo<T, CT>(su, C, ldc, n, m, cost_scale, o, u_out, v_out, P_out, ldp, P_dtype, info, errlog, s));
        (void)hipGetLastError();
        if (o.engine == OTF_ENGINE_RESIDENT) return check_hip(e);
        // co-residency refused (e.g. a smaller device): fall back to the sweep engine
    }
    // sweep engine: one persistent launch that streams C once per iteration (costs
    // that do not fit the register files; POT flavour, whole problems)
    const bool sfits = !LOG && !avg_pass_ms && whole && o.max_iter >= 1 &&
                       sweep_supported<T, CT>(n, m, ldc);
    if (o.engine == OTF_ENGINE_SWEEP && !sfits) return OTF_EUNSUPPORTED;
    if (sfits && (o.engine == OTF_ENGINE_SWEEP || o.engine == OTF_ENGINE_AUTO)) {
        const hipError_t e = force_giveup() ? forced_giveup(info, s) : run_sweep<T, CT>(C, ldc, (int)n, (int)m, su.m_pad, (const T*)su.w.a_pad,
                                              (const T*)su.w.b_pad, cost_scale, o, su.w.sweep, u_out,
                                              v_out, P_out, ldp, P_dtype, info, errlog, s, nullptr, shp,
                                              kstream_buf(su, ws_bytes));
        if (e == hipSuccess) return check_hip(launch_solo<T, CT>(su, C, ldc, n, m, cost_scale, o, u_out, v_out, P_out, ldp, P_dtype, info, errlog, s));
        (void)hipGetLastError();
        if (o.engine == OTF_ENGINE_SWEEP) return check_hip(e);
    }
    if (LOG) {
        dim3 g((unsigned)((m + 255) / 256), (unsigned)(n < 64 ? n : 64));
        sk_colmin_kernel<CT><<<g, 256, 0, s>>>(C, ldc, (int)n, (int)m, su.w.cmin_key);
        OTF_HIP(hipGetLastError());
    }
    SkArgs<T> p = sk_args<T, CT, LOG>(su, C, ldc, n, m, cost_scale, o, info, errlog, avg_pass_ms);

    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double total_ms = 0.0;
    int timed = 0;
    if (avg_pass_ms) {
        OTF_HIP(hipEventCreate(&ev0));
        OTF_HIP(hipEventCreate(&ev1));
    }
    int* host_stop = nullptr;
    if (o.sync_every > 0) OTF_HIP(hipHostMalloc((void**)&host_stop, sizeof(int), hipHostMallocDefault));

    for (int pass = 0; pass <= o.max_iter; ++pass) {
        sk_set_pass(p, su, pass);
        if (avg_pass_ms && pass >= 1) OTF_HIP(hipEventRecord(ev0, s));
        OTF_HIP((launch_pass<T, CT, LOG>(su.cfg, su.grid, p, s)));
        if (avg_pass_ms && pass >= 1) {
            OTF_HIP(hipEventRecord(ev1, s));
            OTF_HIP(hipEventSynchronize(ev1));
            float ms = 0.f;
            OTF_HIP(hipEventElapsedTime(&ms, ev0, ev1));
            total_ms += ms;
            ++timed;
        }
        if (host_stop && pass >= 1 && pass % o.sync_every == 0 && pass < o.max_iter) {
            OTF_HIP(hipMemcpyAsync(host_stop, &info->stop, sizeof(int), hipMemcpyDeviceToHost, s));
            OTF_HIP(hipStreamSynchronize(s));
            if (*host_stop) break;
        }
    }
    if (host_stop) OTF_HIP(hipHostFree(host_stop));
    rc = sk_finish<T, CT, LOG>(p, su, C, ldc, n, m, cost_scale, o, u_out, v_out, P_out, ldp, P_dtype,
                               info, s);
    if (rc != OTF_OK) return rc;
    if (avg_pass_ms) {
        OTF_HIP(hipStreamSynchronize(s));
        *avg_pass_ms = timed ? (float)(total_ms / timed) : 0.f;
        (void)hipEventDestroy(ev0);
        (void)hipEventDestroy(ev1);
    }
    return OTF_OK;
}

// One pass of the row-sharded streaming solve (POT flavour).  Pass 0 also runs the
// init kernel.  *colsum receives this pass's column-sum buffer (m_pad + 1 values of
// dtype: the partial K^T u of this shard's rows and the break count), which the
// caller all-reduces (sum) across the shards before the next pass.
template <typename T, typename CT>
int sk_pass_api(const T* a, const T* b, const CT* C, int64_t n, int64_t m, int64_t ldc,
                const T* cost_scale, const otf_sinkhorn_opts& o, int pass,
                otf_sinkhorn_info* info, double* errlog, void* ws, size_t ws_bytes, void** colsum,
                int64_t* colsum_len, hipStream_t s) {
    if (o.flavor != OTF_FLAVOR_POT || o.shift) return OTF_EUNSUPPORTED;
    if (pass < 0 || pass > o.max_iter) return OTF_EINVAL;
    SkSetup<T> su;
    int rc = sk_prepare<T, CT>(a, b, C, n, m, ldc, o, info, ws, ws_bytes, su);
    if (rc != OTF_OK) return rc;
    if (pass == 0) {
        rc = sk_init<T>(su, a, b, n, m, info, s);
        if (rc != OTF_OK) return rc;
    }
    SkArgs<T> p = sk_args<T, CT, false>(su, C, ldc, n, m, cost_scale, o, info, errlog, false);
    sk_set_pass(p, su, pass);
    OTF_HIP((launch_pass<T, CT, false>(su.cfg, su.grid, p, s)));
    if (colsum) *colsum = p.cs_dst;
    if (colsum_len) *colsum_len = su.m_pad + 1;
    return OTF_OK;
}

template <typename T, typename CT>
int sk_finish_api(const T* a, const T* b, const CT* C, int64_t n, int64_t m, int64_t ldc,
                  const T* cost_scale, const otf_sinkhorn_opts& o, T* u_out, T* v_out, void* P_out,
                  int64_t ldp, int P_dtype, otf_sinkhorn_info* info, double* errlog, void* ws,
                  size_t ws_bytes, hipStream_t s) {
    constexpr int VEC = Vec<T>::N;
    if (o.flavor != OTF_FLAVOR_POT || o.shift) return OTF_EUNSUPPORTED;
    if (!u_out || !v_out) return OTF_EINVAL;
    if (P_out && (ldp < m || ldp % VEC != 0 || ((uintptr_t)P_out % 16) != 0)) return OTF_EINVAL;
    SkSetup<T> su;
    int rc = sk_prepare<T, CT>(a, b, C, n, m, ldc, o, info, ws, ws_bytes, su);
    if (rc != OTF_OK) return rc;
    SkArgs<T> p = sk_args<T, CT, false>(su, C, ldc, n, m, cost_scale, o, info, errlog, false);
    return sk_finish<T, CT, false>(p, su, C, ldc, n, m, cost_scale, o, u_out, v_out, P_out, ldp,
                                   P_dtype, info, s);
}

template <typename T, typename CT>
int dispatch_ct(const void* a, const void* b, const void* C, int64_t n, int64_t m, int64_t ldc,
                const void* cost_scale, const otf_sinkhorn_opts& o, void* u_out, void* v_out,
                void* P_out, int64_t ldp, int P_dtype, otf_sinkhorn_info* info, double* errlog,
                void* ws, size_t ws_bytes, hipStream_t s, float* avg_ms) {
    if (o.flavor == OTF_FLAVOR_POT)
        return run_sinkhorn<T, CT, false>((const T*)a, (const T*)b, (const CT*)C, n, m, ldc,
                                          (const T*)cost_scale, o, (T*)u_out, (T*)v_out, P_out, ldp,
                                          P_dtype, info, errlog, ws, ws_bytes, s, avg_ms);
    if (o.flavor == OTF_FLAVOR_OTT)
        return run_sinkhorn<T, CT, true>((const T*)a, (const T*)b, (const CT*)C, n, m, ldc,
                                         (const T*)cost_scale, o, (T*)u_out, (T*)v_out, P_out, ldp,
                                         P_dtype, info, errlog, ws, ws_bytes, s, avg_ms);
    return OTF_EINVAL;
}

// cost stored as fp16 (opts.cost_f16) is supported with fp32 compute
template <typename T>
int dispatch(const void* a, const void* b, const void* C, int64_t n, int64_t m, int64_t ldc,
             const void* cost_scale, const otf_sinkhorn_opts& o, void* u_out, void* v_out,
             void* P_out, int64_t ldp, int P_dtype, otf_sinkhorn_info* info, double* errlog,
             void* ws, size_t ws_bytes, hipStream_t s, float* avg_ms) {
    if (!o.cost_f16)
        return dispatch_ct<T, T>(a, b, C, n, m, ldc, cost_scale, o, u_out, v_out, P_out, ldp,
                                 P_dtype, info, errlog, ws, ws_bytes, s, avg_ms);
    if constexpr (sizeof(T) == 4)
        return dispatch_ct<T, _Float16>(a, b, C, n, m, ldc, cost_scale, o, u_out, v_out, P_out,
                                        ldp, P_dtype, info, errlog, ws, ws_bytes, s, avg_ms);
    return OTF_EUNSUPPORTED;
}

// Cross-rank sweep (otf_sinkhorn_xsweep): this rank's rows, the exchange of its peers.
template <typename T, typename CT>
int run_xsweep(const T* a, const T* b, const CT* C, int64_t n, int64_t m, int64_t ldc,
               const T* cost_scale, const otf_sinkhorn_opts& o, const XSweep& xs, T* u_out, T* v_out,
               void* P_out, int64_t ldp, int P_dtype, otf_sinkhorn_info* info, double* errlog_user,
               void* ws, size_t ws_bytes, hipStream_t s) {
    constexpr int VEC = Vec<T>::N;
    if (!u_out || !v_out) return OTF_EINVAL;
    if (P_out && (ldp < m || ldp % VEC != 0 || ((uintptr_t)P_out % 16) != 0)) return OTF_EINVAL;
    if (o.max_iter < 1 || xs.n_total < n) return OTF_EINVAL;
    if (o.shift) return OTF_EUNSUPPORTED;
    SkSetup<T> su;
    int rc = sk_prepare<T, CT>(a, b, C, n, m, ldc, o, info, ws, ws_bytes, su);
    if (rc != OTF_OK) return rc;
    double* errlog = errlog_user ? errlog_user : su.w.errlog;
    // the cross-rank mesh where this rank's slab fits the register files (whole 512-column
    // tiles, one workgroup per tile on this device): K stays resident for the whole solve
    // and the reducers exchange their column-sum partials; the cross-rank sweep otherwise.
    // Every rank must take the same engine (the mesh's error sums follow its tiling, so two
    // engines -- or two tilings -- round POT's error differently and could stop at different
    // checks, leaving a peer waiting on the exchange): the mesh only on equal shards
    // (n * world == n_total; otfuse.distributed.sinkhorn_xsweep agrees on the shard sizes
    // over the group before the call), so the decision depends on (n, m, device) alone
    const bool mesh_fit = (o.engine == OTF_ENGINE_AUTO || o.engine == OTF_ENGINE_MESH) &&
                          (int64_t)n * xs.world == (int64_t)xs.n_total &&
                          mesh_supported(n, m) && m % 512 == 0 && su.w.mesh_bytes > 0 &&
                          ((n + 127) / 128) * (m / 512) <= device_cu_count();
    if (o.engine == OTF_ENGINE_MESH && !mesh_fit) return OTF_EUNSUPPORTED;
    if (mesh_fit) {
        rc = sk_init<T>(su, a, b, n, m, info, s, su.w.mesh, su.w.mesh_bytes);
        if (rc != OTF_OK) return rc;
        return check_hip(run_mesh<CT>(C, ldc, (int)n, (int)m, (const float*)su.w.a_pad, (const float*)su.w.b_pad,
                                      cost_scale, o, su.w.mesh, u_out, v_out, P_out, ldp, P_dtype, info,
                                      errlog, /*zeroed=*/true, s, nullptr, &xs));
    }
    if (!sweep_supported<T, CT>(n, m, ldc)) return OTF_EUNSUPPORTED;
    rc = sk_init<T>(su, a, b, n, m, info, s);
    if (rc != OTF_OK) return rc;
    return check_hip(run_sweep<T, CT>(C, ldc, (int)n, (int)m, su.m_pad, (const T*)su.w.a_pad,
                                      (const T*)su.w.b_pad, cost_scale, o, su.w.sweep, u_out, v_out,
                                      P_out, ldp, P_dtype, info, errlog, s, &xs));
}

}  // namespace
}  // namespace otf

// One rank's side of a cross-rank exchange (include/otfuse.h, otf_xpeer_*).
struct otf_xpeer {
    int rank, world;
    int64_t m, m_pad;
    void* own;
    void* peer[otf::kXMaxRanks];
    unsigned ep_base;
    unsigned solves;  // solves issued on this exchange (their parity picks the slot set)
    int connected;
};

extern "C" {

size_t otf_xpeer_handle_size(void) { return sizeof(hipIpcMemHandle_t); }

int otf_xpeer_create(int32_t rank, int32_t world, int64_t m, otf_xpeer** out, void* handle_out) {
    if (!out || !handle_out || world < 1 || world > otf::kXMaxRanks || rank < 0 || rank >= world || m < 1)
        return OTF_EINVAL;
    otf_xpeer* x = new otf_xpeer{};
    x->rank = rank;
    x->world = world;
    x->m = m;
    x->m_pad = (int64_t)otf::align_up((size_t)m, 64);
    const size_t bytes = otf::xsweep_exchange_bytes(x->m_pad);
    hipError_t e = hipMalloc(&x->own, bytes);
    if (e == hipSuccess) e = hipMemset(x->own, 0, bytes);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipIpcGetMemHandle((hipIpcMemHandle_t*)handle_out, x->own);
    if (e != hipSuccess) {
        if (x->own) (void)hipFree(x->own);
        delete x;
        return otf::check_hip(e);
    }
    x->peer[rank] = x->own;
    *out = x;
    return OTF_OK;
}

int otf_xpeer_connect(otf_xpeer* x, const void* handles) {
    if (!x || !handles || x->connected) return OTF_EINVAL;
    const unsigned char* h = (const unsigned char*)handles;
    for (int r = 0; r < x->world; ++r) {
        if (r == x->rank) continue;
        hipIpcMemHandle_t hr;
        memcpy(&hr, h + (size_t)r * sizeof(hipIpcMemHandle_t), sizeof(hr));
        const hipError_t e = hipIpcOpenMemHandle(&x->peer[r], hr, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
            for (int q = 0; q < r; ++q)
                if (q != x->rank && x->peer[q]) (void)hipIpcCloseMemHandle(x->peer[q]);
            return otf::check_hip(e);
        }
    }
    x->connected = 1;
    return OTF_OK;
}

int otf_xpeer_destroy(otf_xpeer* x) {
    if (!x) return OTF_EINVAL;
    // this rank's own solves are finished before its exchange buffer goes away; the
    // caller's contract (include/otfuse.h) covers the peers' solves that store into it
    (void)hipDeviceSynchronize();
    if (x->connected)
        for (int r = 0; r < x->world; ++r)
            if (r != x->rank && x->peer[r]) (void)hipIpcCloseMemHandle(x->peer[r]);
    if (x->own) (void)hipFree(x->own);
    delete x;
    return OTF_OK;
}

int otf_sinkhorn_xsweep(const void* a, const void* b, const void* C, int64_t n, int64_t m,
                        int64_t ldc, int32_t dtype, const void* cost_scale,
                        const otf_sinkhorn_opts* opts, otf_xpeer* x, void* u_out, void* v_out,
                        void* P_out, int64_t ldp, int32_t P_dtype, otf_sinkhorn_info* info,
                        double* errlog, void* workspace, size_t ws_bytes, otf_stream_t stream) {
    if (!opts || !x || !x->connected || dtype != OTF_F32) return OTF_EINVAL;
    if (opts->flavor != OTF_FLAVOR_POT) return OTF_EUNSUPPORTED;
    if (m != x->m) return OTF_EINVAL;
    if (P_out && P_dtype != OTF_F32 && P_dtype != OTF_F64) return OTF_EINVAL;
    // epochs live in 30 bits of a tag and 0 is the cleared state: a window that would
    // wrap restarts at 1 (every peer slot has been rewritten many times since)
    if ((uint64_t)x->ep_base + (uint64_t)opts->max_iter + 8 >= (1ull << 30)) x->ep_base = 0;
    otf::XSweep xs{};
    xs.rank = x->rank;
    xs.world = x->world;
    xs.n_total = opts->n_total > 0 ? opts->n_total : (int)n;
    xs.ep_base = x->ep_base;
    xs.solve_par = (int)(x->solves & 1u);
    ++x->solves;
    for (int r = 0; r < x->world; ++r) xs.xr[r] = (unsigned char*)x->peer[r];
    // every rank makes the same sequence of calls: the bases stay in lock-step
    x->ep_base = x->ep_base + (unsigned)opts->max_iter + 4u;
    hipStream_t s = (hipStream_t)stream;
    if (opts->cost_f16)
        return otf::run_xsweep<float, _Float16>((const float*)a, (const float*)b, (const _Float16*)C, n,
                                                m, ldc, (const float*)cost_scale, *opts, xs,
                                                (float*)u_out, (float*)v_out, P_out, ldp, P_dtype,
                                                info, errlog, workspace, ws_bytes, s);
    return otf::run_xsweep<float, float>((const float*)a, (const float*)b, (const float*)C, n, m, ldc,
                                         (const float*)cost_scale, *opts, xs, (float*)u_out,
                                         (float*)v_out, P_out, ldp, P_dtype, info, errlog, workspace,
                                         ws_bytes, s);
}

int otf_sinkhorn_fallback_count(uint64_t* count) {
    if (!count) return OTF_EINVAL;
    unsigned long long v = 0;
    OTF_HIP(hipMemcpyFromSymbol(&v, HIP_SYMBOL(otf::g_sk_fallbacks), sizeof(v)));
    *count = (uint64_t)v;
    return OTF_OK;
}


size_t otf_sinkhorn_workspace_size(int64_t n, int64_t m, int32_t dtype, int32_t max_iter) {
    const size_t esz = dtype == OTF_F64 ? 8 : 4;
    const int64_t nrb = dtype == OTF_F64 ? otf::row_blocks<double>(n, m) : otf::row_blocks<float>(n, m);
    return otf::carve(nullptr, n, m, esz, max_iter < 0 ? 0 : max_iter, nrb).bytes_k;
}

int otf_sinkhorn_shift_offsets(int64_t n, int64_t m, int32_t dtype, int32_t max_iter,
                               size_t* off_a, size_t* off_b) {
    if (!off_a || !off_b || n <= 0 || m <= 0) return OTF_EINVAL;
    if (dtype != OTF_F32) return OTF_EUNSUPPORTED;
    const int64_t nrb = otf::row_blocks<float>(n, m);
    // carve against a non-null stand-in base (it hands out null pointers for a null one)
    char* const base = (char*)(uintptr_t)4096;
    const otf::Workspace w = otf::carve(base, n, m, 4, max_iter < 0 ? 0 : max_iter, nrb);
    *off_a = (size_t)((char*)w.shA - base);
    *off_b = (size_t)((char*)w.shB - base);
    return OTF_OK;
}

int otf_sinkhorn(const void* a, const void* b, const void* C, int64_t n, int64_t m, int64_t ldc,
                 int32_t dtype, const void* cost_scale, const otf_sinkhorn_opts* opts, void* u_out,
                 void* v_out, void* P_out, int64_t ldp, int32_t P_dtype, otf_sinkhorn_info* info,
                 double* errlog, void* workspace, size_t ws_bytes, otf_stream_t stream) {
    if (!opts) return OTF_EINVAL;
    if (P_out && P_dtype != OTF_F32 && P_dtype != OTF_F64) return OTF_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    if (dtype == OTF_F32)
        return otf::dispatch<float>(a, b, C, n, m, ldc, cost_scale, *opts, u_out, v_out, P_out, ldp,
                                    P_dtype, info, errlog, workspace, ws_bytes, s, nullptr);
    if (dtype == OTF_F64)
        return otf::dispatch<double>(a, b, C, n, m, ldc, cost_scale, *opts, u_out, v_out, P_out,
                                     ldp, P_dtype, info, errlog, workspace, ws_bytes, s, nullptr);
    return OTF_EINVAL;
}

// ---------------------------------------------------------------------------------------
// Pairwise cost + Sinkhorn, float64 (include/otfuse.h).  Workspace: [the float64 Sinkhorn
// workspace][the n x m float64 cost (the unfused path and the fallback)][the cost call's
// workspace (norms, per-tile maxima)][the max].
namespace otf {
namespace {
// the squared norms of X's and Y's float32 rows in float64 (one wave per row), for the
// pairwise mesh's epilogue (kept out of its matrix-core loops), and sk_init's work (the
// marginals, the zeroed granule region, info) in the same launch
__global__ __launch_bounds__(256) void pw_norms_kernel(const float* X, int64_t ldx, int n, const float* Y,
                                                       int64_t ldy, int m, int d, double* nx, double* ny,
                                                       const double* a, const double* b, int m_pad,
                                                       double* a_pad, double* b_pad, double* cs, int cs_stride,
                                                       double* u2, double* v2, int* cmin_key,
                                                       otf_sinkhorn_info* info, uint4* zero, int64_t zero_n,
                                                       int* relay) {
    sk_init_body<double>(blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x, a, b, n, m, m_pad, a_pad,
                         b_pad, cs, cs_stride, u2, v2, cmin_key, info, zero, zero_n, relay);
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (i >= n + m) return;
    const float* r = i < n ? X + (int64_t)i * ldx : Y + (int64_t)(i - n) * ldy;
    double s = 0;
    for (int k = lane; k < d; k += 64) s = fma((double)r[k], (double)r[k], s);
    s = wave_sum(s);
    if (lane == 0) (i < n ? nx[i] : ny[i - n]) = s;
}
struct PwLayout {
    size_t sk, c, cost, total;
};
PwLayout pw_layout(int64_t n, int64_t m, int32_t max_iter) {
    PwLayout l;
    l.sk = (otf_sinkhorn_workspace_size(n, m, OTF_F64, max_iter) + 255) / 256 * 256;
    l.c = ((size_t)n * (size_t)m * 8 + 255) / 256 * 256;
    l.cost = (otf_cost_pairwise_f64_workspace_size(n, m) + 255) / 256 * 256;
    l.total = l.sk + l.c + l.cost + 256;
    return l;
}
}  // namespace
}  // namespace otf

size_t otf_sinkhorn_pairwise_f64_workspace_size(int64_t n, int64_t m, int32_t max_iter) {
    if (n <= 0 || m <= 0) return 0;
    return otf::pw_layout(n, m, max_iter).total;
}

int otf_sinkhorn_pairwise_f64(const float* X, int64_t ldx, const float* Y, int64_t ldy, int64_t n, int64_t m,
                              int64_t d, int32_t metric, int32_t scale_max, const double* a, const double* b,
                              const otf_sinkhorn_opts* opts, double* u_out, double* v_out, void* P_out,
                              int64_t ldp, int32_t P_dtype, double* cmax_out, otf_sinkhorn_info* info,
                              double* errlog, void* workspace, size_t ws_bytes, otf_stream_t stream) {
    using namespace otf;
    if (!opts || !X || !Y || !workspace || n <= 0 || m <= 0 || d <= 0) return OTF_EINVAL;
    if (ldx < d || ldy < d) return OTF_EINVAL;
    if (metric != OTF_SQEUCLIDEAN && metric != OTF_EUCLIDEAN) return OTF_EINVAL;
    if (P_out && P_dtype != OTF_F32 && P_dtype != OTF_F64) return OTF_EINVAL;
    if (opts->flavor != OTF_FLAVOR_POT) return OTF_EUNSUPPORTED;
    const otf_sinkhorn_opts& o = *opts;
    const PwLayout L = pw_layout(n, m, o.max_iter);
    if (ws_bytes < L.total) return OTF_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    char* base = (char*)workspace;
    void* ws_sk = base;
    double* Cw = (double*)(base + L.sk);
    char* ws_cost = base + L.sk + L.c;
    double* cmax = (double*)(base + L.sk + L.c + L.cost);
    double* nx = (double*)ws_cost;  // the fallback's norms (n + m doubles)
    const bool whole = o.n_total <= 0 || o.n_total == n;
    const bool engine_ok = o.engine == OTF_ENGINE_MESH || (o.engine == OTF_ENGINE_AUTO && mesh_enabled());
    // the fused launch writes the plan in 16-B pieces of four elements (ldp % 4 == 0); decided
    // here, before any launch, so an unaligned plan takes the two calls without a wasted norms pass
    bool fused = whole && !o.shift && o.max_iter >= 1 && engine_ok && u_out && v_out &&
                 (!P_out || ldp % 4 == 0) && mesh64_pairwise_ok(n, m, d, ldx, ldy, X, Y);
    if (!u_out || !v_out) return OTF_EINVAL;
    if (P_out && (ldp < m || ldp % 2 != 0 || ((uintptr_t)P_out % 16) != 0)) return OTF_EINVAL;
    if (fused) {
        SkSetup<double> su;
        int rc = sk_prepare<double, double>(a, b, Cw, n, m, m, o, info, ws_sk, L.sk, su);
        if (rc != OTF_OK) return rc;
        // AUTO takes the float64 mesh where it takes it on a given cost (past one tiled-engine
        // tile per CU)
        if (su.w.mesh_bytes == 0 ||
            (o.engine == OTF_ENGINE_AUTO && su.w.t_nrb * su.w.t_ncb <= device_cu_count()))
            fused = false;
        if (fused) {
            double* errl = errlog ? errlog : su.w.errlog;
            pw_norms_kernel<<<(unsigned)((n + m + 3) / 4), 256, 0, s>>>(
                X, ldx, (int)n, Y, ldy, (int)m, (int)d, nx, nx + n, a, b, su.m_pad, (double*)su.w.a_pad,
                (double*)su.w.b_pad, (double*)su.w.cs, (int)su.w.cs_stride, (double*)su.w.u2, (double*)su.w.v2,
                su.w.cmin_key, info, (uint4*)su.w.mesh, (int64_t)(su.w.mesh_bytes / 16), su.w.relay);
            OTF_HIP(hipGetLastError());
            PairwiseF64 pw{X, ldx, Y, ldy, (int)d, metric == OTF_EUCLIDEAN ? 1 : 0, scale_max ? 1 : 0,
                           nx, nx + n, cmax_out, (uint32_t)(n * ldx * 4), (uint32_t)(m * ldy * 4)};
            hipError_t e;
            if (force_giveup()) {
                // test path (OTF_FORCE_REG_GIVEUP=1): the launch's registration gives up at once,
                // so the fallback runs at the caller's full shape without a contending grid
                sk_giveup_kernel<<<1, 64, 0, s>>>(info);
                e = hipGetLastError();
            } else {
                e = run_mesh64(nullptr, m, (int)n, (int)m, (const double*)su.w.a_pad, (const double*)su.w.b_pad,
                               nullptr, o, su.w.mesh, u_out, v_out, P_out, ldp, P_dtype, info, errl,
                               /*zeroed=*/true, s, &pw);
            }
            if (e == hipSuccess) {
                // the fallback (only after a registration give-up): the relay builds the cost
                // into the workspace (from the norms launch's norms), K over it, then solves
                SoloArgs<double> fb{};
                fb.pw_X = X;
                fb.pw_Y = Y;
                fb.pw_ldx = ldx;
                fb.pw_ldy = ldy;
                fb.pw_d = (int)d;
                fb.pw_euclid = metric == OTF_EUCLIDEAN ? 1 : 0;
                fb.pw_scale = scale_max ? 1 : 0;
                fb.pw_vec = (ldx % 4 == 0) && (ldy % 4 == 0) && ((uintptr_t)X % 16 == 0) && ((uintptr_t)Y % 16 == 0);
                fb.pw_cmax_out = cmax_out;
                fb.pw_nx = nx;
                fb.pw_tiles_m = (int)((n + RL_T - 1) / RL_T);
                fb.pw_ntiles = fb.pw_tiles_m * (int)((m + RL_T - 1) / RL_T);
                return check_hip(launch_solo<double, double>(su, Cw, m, n, m, nullptr, o, u_out, v_out, P_out, ldp,
                                                             P_dtype, info, errl, s, &fb));
            }
            (void)hipGetLastError();
            if (o.engine == OTF_ENGINE_MESH) return check_hip(e);
        }
    }
    // the cost, then the solve on it
    int rc = otf_cost_pairwise_f64(X, ldx, Y, ldy, n, m, d, metric, 0, 0, Cw, m, cmax, ws_cost, L.cost, stream);
    if (rc != OTF_OK) return rc;
    if (cmax_out) OTF_HIP(hipMemcpyAsync(cmax_out, cmax, 8, hipMemcpyDeviceToDevice, s));
    otf_sinkhorn_opts o2 = o;
    if (o2.engine == OTF_ENGINE_MESH && !mesh64_supported(n, m)) o2.engine = OTF_ENGINE_AUTO;
    return otf_sinkhorn(a, b, Cw, n, m, m, OTF_F64, scale_max ? cmax : nullptr, &o2, u_out, v_out, P_out, ldp,
                        P_dtype, info, errlog, ws_sk, L.sk, stream);
}

// ---------------------------------------------------------------------------------------
// Pairwise cost + Sinkhorn, float32 (include/otfuse.h).  Workspace: [the float32 Sinkhorn
// workspace][the n x m float32 cost (the unfused path and the fallback)][the split-fp16 cost
// workspace (images, row scales, norms)][the max].
namespace otf {
namespace {
PwLayout pw32_layout(int64_t n, int64_t m, int64_t d, int32_t max_iter) {
    PwLayout l;
    l.sk = (otf_sinkhorn_workspace_size(n, m, OTF_F32, max_iter) + 255) / 256 * 256;
    l.c = ((size_t)n * (size_t)m * 4 + 255) / 256 * 256;
    l.cost = (otf_cost_ex_workspace_size(n, m, d, OTF_F32) + 255) / 256 * 256;
    l.total = l.sk + l.c + l.cost + 256;
    return l;
}
}  // namespace
}  // namespace otf

size_t otf_sinkhorn_pairwise_f32_workspace_size(int64_t n, int64_t m, int64_t d, int32_t max_iter) {
    if (n <= 0 || m <= 0 || d <= 0) return 0;
    return otf::pw32_layout(n, m, d, max_iter).total;
}

int otf_sinkhorn_pairwise_f32(const float* X, int64_t ldx, const float* Y, int64_t ldy, int64_t n, int64_t m,
                              int64_t d, int32_t metric, int32_t scale_max, const float* a, const float* b,
                              const otf_sinkhorn_opts* opts, float* u_out, float* v_out, void* P_out,
                              int64_t ldp, int32_t P_dtype, float* cmax_out, otf_sinkhorn_info* info,
                              double* errlog, void* workspace, size_t ws_bytes, otf_stream_t stream) {
    using namespace otf;
    if (!opts || !X || !Y || !workspace || n <= 0 || m <= 0 || d <= 0) return OTF_EINVAL;
    if (ldx < d || ldy < d) return OTF_EINVAL;
    if (metric != OTF_SQEUCLIDEAN && metric != OTF_EUCLIDEAN) return OTF_EINVAL;
    if (P_out && P_dtype != OTF_F32 && P_dtype != OTF_F64) return OTF_EINVAL;
    if (opts->flavor != OTF_FLAVOR_POT) return OTF_EUNSUPPORTED;
    if (n > INT32_MAX || m > INT32_MAX || d > (1 << 20)) return OTF_EUNSUPPORTED;
    const otf_sinkhorn_opts& o = *opts;
    const PwLayout L = pw32_layout(n, m, d, o.max_iter);
    if (ws_bytes < L.total) return OTF_EINVAL;
    if (!u_out || !v_out) return OTF_EINVAL;
    if (P_out && (ldp < m || ldp % 4 != 0 || ((uintptr_t)P_out % 16) != 0)) return OTF_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    char* base = (char*)workspace;
    void* ws_sk = base;
    float* Cw = (float*)(base + L.sk);
    char* ws_cost = base + L.sk + L.c;
    float* cmax = (float*)(base + L.sk + L.c + L.cost);
    const bool whole = o.n_total <= 0 || o.n_total == n;
    // the fused launch on request (engine MESH) only: at the metric shape it measured 0.529 ms
    // against 0.495 ms for the two calls (its in-prologue cost build runs at ~1/4 of the fp16
    // MFMA peak, one register stage of prefetch against the L2 latency, so the 67-MB round trip
    // it saves does not pay), so AUTO keeps the two calls
    const bool engine_ok = o.engine == OTF_ENGINE_MESH;
    bool fused = whole && !o.shift && o.max_iter >= 1 && engine_ok && mesh_pairwise_ok(n, m, d) &&
                 (size_t)n * (size_t)((d + 63) / 64 * 64) * 2 < ((size_t)1 << 31) &&
                 (size_t)m * (size_t)((d + 63) / 64 * 64) * 2 < ((size_t)1 << 31);
    if (fused) {
        SkSetup<float> su;
        int rc = sk_prepare<float, float>(a, b, Cw, n, m, m, o, info, ws_sk, L.sk, su);
        if (rc != OTF_OK) return rc;
        if (su.w.mesh_bytes == 0) fused = false;
        if (fused) {
            double* errl = errlog ? errlog : su.w.errlog;
            rc = sk_init<float>(su, a, b, n, m, info, s, su.w.mesh, su.w.mesh_bytes);
            if (rc != OTF_OK) return rc;
            Split16Images im{};
            OTF_HIP(split16_images(X, ldx, (int)n, Y, ldy, (int)m, (int)d, ws_cost, im, nullptr, s));
            PairwiseF32 pw{im.Xh, im.Xl, im.Yh, im.Yl, im.ldh, im.xs, im.xx, im.ys, im.yy, (int)im.ldh,
                           metric == OTF_EUCLIDEAN ? 1 : 0, scale_max ? 1 : 0, cmax_out,
                           (uint32_t)(n * im.ldh * 2), (uint32_t)(m * im.ldh * 2)};
            hipError_t e;
            if (force_giveup()) {
                // test path (OTF_FORCE_REG_GIVEUP=1): the fallback at the caller's full shape
                sk_giveup_kernel<<<1, 64, 0, s>>>(info);
                e = hipGetLastError();
            } else {
                e = run_mesh<float>(nullptr, m, (int)n, (int)m, (const float*)su.w.a_pad, (const float*)su.w.b_pad,
                                    nullptr, o, su.w.mesh, u_out, v_out, P_out, ldp, P_dtype, info, errl,
                                    /*zeroed=*/true, s, nullptr, nullptr, &pw);
            }
            if (e == hipSuccess) {
                // the fallback (only after a registration give-up): the relay builds the float32
                // cost into the workspace on the float64 matrix cores (from the prep's norms), K
                // over it, then solves
                SoloArgs<float> fb{};
                fb.pw_X = X;
                fb.pw_Y = Y;
                fb.pw_ldx = ldx;
                fb.pw_ldy = ldy;
                fb.pw_d = (int)d;
                fb.pw_euclid = metric == OTF_EUCLIDEAN ? 1 : 0;
                fb.pw_scale = scale_max ? 1 : 0;
                fb.pw_vec = (ldx % 4 == 0) && (ldy % 4 == 0) && ((uintptr_t)X % 16 == 0) && ((uintptr_t)Y % 16 == 0);
                fb.pw_cmax_out = cmax_out;
                fb.pw_nxf = im.xx;
                fb.pw_nyf = im.yy;
                fb.pw_tiles_m = (int)((n + RL_T - 1) / RL_T);
                fb.pw_ntiles = fb.pw_tiles_m * (int)((m + RL_T - 1) / RL_T);
                return check_hip(launch_solo<float, float>(su, Cw, m, n, m, nullptr, o, u_out, v_out, P_out, ldp,
                                                           P_dtype, info, errl, s, &fb));
            }
            (void)hipGetLastError();
            if (o.engine == OTF_ENGINE_MESH) return check_hip(e);
        }
    }
    // the cost, then the solve on it (the split-fp16 cost kernel: the same costs)
    int rc = otf_cost_pairwise_ex(X, ldx, Y, ldy, OTF_F32, n, m, d, metric, 0, Cw, m, OTF_F32, cmax, nullptr, ws_cost,
                                  L.cost, stream);
    if (rc != OTF_OK) return rc;
    if (cmax_out) OTF_HIP(hipMemcpyAsync(cmax_out, cmax, 4, hipMemcpyDeviceToDevice, s));
    return otf_sinkhorn(a, b, Cw, n, m, m, OTF_F32, scale_max ? cmax : nullptr, &o, u_out, v_out, P_out, ldp,
                        P_dtype, info, errlog, ws_sk, L.sk, stream);
}

int otf_sinkhorn_profile(const void* a, const void* b, const void* C, int64_t n, int64_t m,
                         int64_t ldc, int32_t dtype, const void* cost_scale,
                         const otf_sinkhorn_opts* opts, void* u_out, void* v_out,
                         otf_sinkhorn_info* info, void* workspace, size_t ws_bytes,
                         float* avg_pass_ms, otf_stream_t stream) {
    if (!opts || !avg_pass_ms) return OTF_EINVAL;
    otf_sinkhorn_opts o = *opts;
    o.sync_every = 0;
    hipStream_t s = (hipStream_t)stream;
    if (dtype == OTF_F32)
        return otf::dispatch<float>(a, b, C, n, m, ldc, cost_scale, o, u_out, v_out, nullptr, 0,
                                    OTF_F32, info, nullptr, workspace, ws_bytes, s, avg_pass_ms);
    if (dtype == OTF_F64)
        return otf::dispatch<double>(a, b, C, n, m, ldc, cost_scale, o, u_out, v_out, nullptr, 0,
                                     OTF_F64, info, nullptr, workspace, ws_bytes, s, avg_pass_ms);
    return OTF_EINVAL;
}

int otf_sinkhorn_pass(const void* a, const void* b, const void* C, int64_t n, int64_t m,
                      int64_t ldc, int32_t dtype, const void* cost_scale,
                      const otf_sinkhorn_opts* opts, int32_t pass, otf_sinkhorn_info* info,
                      double* errlog, void* workspace, size_t ws_bytes, void** colsum,
                      int64_t* colsum_len, otf_stream_t stream) {
    if (!opts) return OTF_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const otf_sinkhorn_opts& o = *opts;
    if (dtype == OTF_F32 && o.cost_f16)
        return otf::sk_pass_api<float, _Float16>((const float*)a, (const float*)b, (const _Float16*)C,
                                                 n, m, ldc, (const float*)cost_scale, o, pass, info,
                                                 errlog, workspace, ws_bytes, colsum, colsum_len, s);
    if (dtype == OTF_F32)
        return otf::sk_pass_api<float, float>((const float*)a, (const float*)b, (const float*)C, n, m,
                                              ldc, (const float*)cost_scale, o, pass, info, errlog,
                                              workspace, ws_bytes, colsum, colsum_len, s);
    if (dtype == OTF_F64 && !o.cost_f16)
        return otf::sk_pass_api<double, double>((const double*)a, (const double*)b, (const double*)C,
                                                n, m, ldc, (const double*)cost_scale, o, pass, info,
                                                errlog, workspace, ws_bytes, colsum, colsum_len, s);
    return OTF_EINVAL;
}

int otf_sinkhorn_row_sharded(const void* a, const void* b, const void* C, int64_t n, int64_t m,
                             int64_t ldc, int32_t dtype, const void* cost_scale,
                             const otf_sinkhorn_opts* opts, otf_comm* comm, void* u_out,
                             void* v_out, void* P_out, int64_t ldp, int32_t P_dtype,
                             otf_sinkhorn_info* info, double* errlog, void* workspace,
                             size_t ws_bytes, otf_stream_t stream) {
    if (!opts) return OTF_EINVAL;
    if (opts->flavor != OTF_FLAVOR_POT) return OTF_EUNSUPPORTED;
    for (int32_t pass = 0; pass <= opts->max_iter; ++pass) {
        void* cs = nullptr;
        int64_t len = 0;
        int rc = otf_sinkhorn_pass(a, b, C, n, m, ldc, dtype, cost_scale, opts, pass, info, errlog,
                                   workspace, ws_bytes, &cs, &len, stream);
        if (rc != OTF_OK) return rc;
        if (comm) {
            rc = otf::comm_all_reduce(cs, len, dtype, OTF_RED_SUM, comm, (hipStream_t)stream);
            if (rc != OTF_OK) return rc;
        }
    }
    return otf_sinkhorn_finish(a, b, C, n, m, ldc, dtype, cost_scale, opts, u_out, v_out, P_out,
                               ldp, P_dtype, info, errlog, workspace, ws_bytes, stream);
}

int otf_sinkhorn_finish(const void* a, const void* b, const void* C, int64_t n, int64_t m,
                        int64_t ldc, int32_t dtype, const void* cost_scale,
                        const otf_sinkhorn_opts* opts, void* u_out, void* v_out, void* P_out,
                        int64_t ldp, int32_t P_dtype, otf_sinkhorn_info* info, double* errlog,
                        void* workspace, size_t ws_bytes, otf_stream_t stream) {
    if (!opts) return OTF_EINVAL;
    if (P_out && P_dtype != OTF_F32 && P_dtype != OTF_F64) return OTF_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const otf_sinkhorn_opts& o = *opts;
    if (dtype == OTF_F32 && o.cost_f16)
        return otf::sk_finish_api<float, _Float16>((const float*)a, (const float*)b, (const _Float16*)C,
                                                   n, m, ldc, (const float*)cost_scale, o, (float*)u_out,
                                                   (float*)v_out, P_out, ldp, P_dtype, info, errlog,
                                                   workspace, ws_bytes, s);
    if (dtype == OTF_F32)
        return otf::sk_finish_api<float, float>((const float*)a, (const float*)b, (const float*)C, n, m,
                                                ldc, (const float*)cost_scale, o, (float*)u_out,
                                                (float*)v_out, P_out, ldp, P_dtype, info, errlog,
                                                workspace, ws_bytes, s);
    if (dtype == OTF_F64 && !o.cost_f16)
        return otf::sk_finish_api<double, double>((const double*)a, (const double*)b, (const double*)C,
                                                  n, m, ldc, (const double*)cost_scale, o,
                                                  (double*)u_out, (double*)v_out, P_out, ldp, P_dtype,
                                                  info, errlog, workspace, ws_bytes, s);
    return OTF_EINVAL;
}

}  // extern "C"
