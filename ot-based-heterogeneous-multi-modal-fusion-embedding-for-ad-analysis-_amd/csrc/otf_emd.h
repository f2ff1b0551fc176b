// otf_emd.h — the device network simplex (exact EMD, general marginals) as a
// workgroup-level routine: otf_emd.hip's batched launch and the CG-GW linear step of
// otf_gw.hip (weighted / unequal groups) both call emd_block.
//
// Replaces pot.emd(a, b, M, numItermax) (POT 0.9.x ot.lp.emd: the network simplex of
// its emd_c) at perturbot/perturbot/match/cot_labels.py:178 (per-label sample plans)
// and :195 (the feature plan), the EMD that get_coupling_cotl (:228-276) runs, and the
// linear sub-problem of POT's CG-GW on weighted / unequal groups
// (MRI_PET_OT_nojax.py:80-82).  POT is not in the image: the algorithm below is the
// textbook primal network simplex on the bipartite transportation graph, and parity
// is anchored on scipy's HiGHS LP (tests/test_gpu_emd.py): generic costs have one
// optimal plan, so the plans agree entry-wise.
//
// Graph: supply nodes 0..n-1 (a_i), demand nodes n..n+m-1 (-b_j), a root R = n+m with
// one big-M artificial arc per node (k -> R when a_k > 0, R -> k otherwise), which
// form the initial strongly feasible spanning tree.  Real arcs i -> n+j, cost M_ij,
// unbounded.  Per pivot:
//   * pricing: block search over all arcs (blocks of max(sqrt(A), 256) arcs from a
//     rotating cursor); the workgroup's 256 threads scan a block and reduce to the
//     most negative reduced cost c_e + pi_s - pi_t (ties -> first in block order);
//   * one thread does the tree work in LDS: the join of the cycle by depth, the ratio
//     test with Cunningham's last-blocking-arc rule (keeps the tree strongly
//     feasible, so degenerate pivots cannot cycle), the flow update along the cycle,
//     the path reversal that re-hangs the cut subtree under the entering arc, and
//     the depth / potential shift of that subtree (first-child / sibling lists).
// Tree arcs have reduced cost 0, so pricing needs no arc state; the flow of a tree
// arc lives with its child node, so the plan is written once at the end.
// One workgroup per problem: a batch (the per-label plans of one COOT-L step) is one
// launch.  Per node 27 B of LDS: n + m + 1 <= kEmdMaxNodes.
#pragma once
#include "otf_device.h"

namespace otf {

constexpr int kEmdMaxNodes = 5600;
constexpr size_t kEmdScratch = 256 * (8 + 4) + 64;  // reductions of up to 256 threads

// LDS of emd_block for n + m + 1 = N nodes
inline __host__ __device__ size_t emd_lds_bytes(int N) {
    return ((size_t)N * (2 * 8 + 5 * 2 + 1) + 15) / 16 * 16 + kEmdScratch;
}

inline __device__ void argmin_pair(double& v, int& i, double v2, int i2) {
    if (v2 < v || (v2 == v && i2 < i)) {
        v = v2;
        i = i2;
    }
}

// One workgroup of NT threads solves one problem; every thread must call it.  esm:
// emd_lds_bytes(n + m + 1) bytes of LDS (16-B aligned).  P.a / P.b may point to LDS.
template <int NT>
__device__ otf_emd_info emd_block(const otf_emd_problem& P, int64_t max_pivots, unsigned char* esm) {
    static_assert(NT % 64 == 0 && NT <= 256, "whole waves; kEmdScratch holds 256 lanes");
    constexpr int kNW = NT / 64;
    const int n = P.n, m = P.m, N = n + m + 1, R = N - 1;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

    double* pi = reinterpret_cast<double*>(esm);   // node potentials
    double* tflow = pi + N;                         // flow of the tree arc (u, parent u)
    short* par = reinterpret_cast<short*>(tflow + N);
    short* fch = par + N;                           // first child
    short* nsb = fch + N;                           // next / previous sibling
    short* psb = nsb + N;
    short* dep = psb + N;                           // depth (root 0)
    signed char* sgn = reinterpret_cast<signed char*>(dep + N);  // 1: supply > 0
    unsigned char* scr = esm + ((size_t)N * (2 * 8 + 5 * 2 + 1) + 15) / 16 * 16;
    double* rv = reinterpret_cast<double*>(scr);
    int* ri = reinterpret_cast<int*>(rv + NT);
    int* flag = ri + NT;

    // zero the plan; largest |cost| for the big-M of the artificial arcs
    double mc = 0.0;
    for (int i = 0; i < n; ++i) {
        double* trow = P.T + (int64_t)i * P.ldt;
        const double* mrow = P.M + (int64_t)i * P.ldm;
        for (int j = tid; j < m; j += NT) {
            trow[j] = 0.0;
            mc = fmax(mc, fabs(mrow[j]));
        }
    }
    mc = wave_max(mc);
    if (lane == 0) rv[wid] = mc;
    __syncthreads();
    for (int w = 1; w < kNW; ++w) mc = fmax(mc, rv[w]);
    mc = fmax(mc, rv[0]);
    const double ART = (mc + 1.0) * (double)N;
    const double tol = 1e-13 * ART;  // reduced-cost zero (pi carry O(ART) rounding)
    __syncthreads();

    for (int k = tid; k < N - 1; k += NT) {
        const double sup = k < n ? P.a[k] : -P.b[k - n];
        sgn[k] = sup > 0.0 ? 1 : 0;
        par[k] = (short)R;
        tflow[k] = fabs(sup);
        pi[k] = sup > 0.0 ? -ART : ART;
        dep[k] = 1;
        fch[k] = -1;
        psb[k] = (short)(k - 1);
        nsb[k] = (short)(k + 1 < N - 1 ? k + 1 : -1);
    }
    if (tid == 0) {
        sgn[R] = 0;
        par[R] = -1;
        tflow[R] = 0.0;
        pi[R] = 0.0;
        dep[R] = 0;
        fch[R] = (short)(N > 1 ? 0 : -1);
        psb[R] = nsb[R] = -1;
        flag[0] = 0;
    }
    __syncthreads();

    const int A_real = n * m, A_tot = A_real + N - 1;
    int B = (int)ceil(sqrt((double)A_tot));
    B = B < NT ? NT : B;
    B = B > A_tot ? A_tot : B;
    auto rcost = [&](int e) -> double {
        if (e < A_real) {
            const int i = e / m, j = e - i * m;
            return P.M[(int64_t)i * P.ldm + j] + pi[i] - pi[n + j];
        }
        const int k = e - A_real;
        return sgn[k] ? ART + pi[k] - pi[R] : ART + pi[R] - pi[k];
    };
    // the tree arc between u and its parent runs u -> parent ("up")?
    auto up = [&](int u) -> bool { return par[u] == R ? sgn[u] != 0 : u < n; };

    int next = 0;
    int64_t pivots = 0;
    int status = OTF_EMD_OPTIMAL;
    for (;;) {
        // ---- pricing: block search from the cursor
        int in_arc = -1;
        double in_rc = 0.0;
        for (int scanned = 0; scanned < A_tot;) {
            const int len = A_tot - scanned < B ? A_tot - scanned : B;
            double bv = 0.0;
            int bi = INT32_MAX;
            for (int t = tid; t < len; t += NT) {
                int e = next + t;
                if (e >= A_tot) e -= A_tot;
                const double r = rcost(e);
                if (r < bv) {
                    bv = r;
                    bi = t;
                }
            }
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) {
                const double v2 = __shfl_xor(bv, o, 64);
                const int i2 = __shfl_xor(bi, o, 64);
                argmin_pair(bv, bi, v2, i2);
            }
            if (lane == 0) {
                rv[wid] = bv;
                ri[wid] = bi;
            }
            __syncthreads();
            bv = rv[0];
            bi = ri[0];
#pragma unroll
            for (int w = 1; w < kNW; ++w) argmin_pair(bv, bi, rv[w], ri[w]);
            __syncthreads();
            const int start = next;
            next += len;
            if (next >= A_tot) next -= A_tot;
            scanned += len;
            if (bv < -tol) {
                in_arc = start + bi;
                if (in_arc >= A_tot) in_arc -= A_tot;
                in_rc = bv;
                break;
            }
        }
        if (in_arc < 0) break;  // no arc prices out: optimal
        if (++pivots > max_pivots) {
            status = OTF_EMD_MAX_ITER;
            break;
        }

        // ---- tree work (one thread; everything it touches is in LDS)
        if (tid == 0) {
            int s, t;
            if (in_arc < A_real) {
                s = in_arc / m;
                t = n + (in_arc - s * m);
            } else {
                const int k = in_arc - A_real;
                s = sgn[k] ? k : R;
                t = sgn[k] ? R : k;
            }
            int u = s, v = t;
            while (u != v) {
                if (dep[u] > dep[v]) u = par[u];
                else if (dep[v] > dep[u]) v = par[v];
                else {
                    u = par[u];
                    v = par[v];
                }
            }
            const int join = u;
            // ratio test: flow runs join -> ... -> s -> t -> ... -> join; the blocking
            // arcs are those run against their direction; keep the LAST one met in that
            // order from the join (strongly feasible trees)
            double delta = INFINITY;
            int u_out = -1, side = 0;
            for (u = s; u != join; u = par[u])
                if (up(u) && tflow[u] < delta) {
                    delta = tflow[u];
                    u_out = u;
                    side = 1;
                }
            for (u = t; u != join; u = par[u])
                if (!up(u) && tflow[u] <= delta) {
                    delta = tflow[u];
                    u_out = u;
                    side = 2;
                }
            if (u_out < 0) {
                flag[0] = OTF_EMD_UNBOUNDED;
            } else {
                if (delta > 0.0) {
                    for (u = s; u != join; u = par[u]) tflow[u] += up(u) ? -delta : delta;
                    for (u = t; u != join; u = par[u]) tflow[u] += up(u) ? delta : -delta;
                }
                // re-hang the subtree of u_out from u_in (the entering arc's end inside
                // it) under v_in, reversing the path u_in .. u_out
                const int u_in = side == 1 ? s : t, v_in = side == 1 ? t : s;
                const double sigma = side == 1 ? -in_rc : in_rc;
                int prev = v_in;
                double carry = delta;
                u = u_in;
                for (;;) {
                    const int nx = par[u];
                    const double f = tflow[u];
                    // cut u from nx's children
                    if (psb[u] >= 0) nsb[psb[u]] = nsb[u];
                    else fch[nx] = nsb[u];
                    if (nsb[u] >= 0) psb[nsb[u]] = psb[u];
                    // link u as prev's first child
                    nsb[u] = fch[prev];
                    psb[u] = -1;
                    if (fch[prev] >= 0) psb[fch[prev]] = (short)u;
                    fch[prev] = (short)u;
                    par[u] = (short)prev;
                    tflow[u] = carry;
                    carry = f;
                    if (u == u_out) break;
                    prev = u;
                    u = nx;
                }
                // depth and potentials of the moved subtree (pre-order walk)
                int x = u_in;
                dep[x] = (short)(dep[v_in] + 1);
                pi[x] += sigma;
                for (;;) {
                    if (fch[x] >= 0) {
                        x = fch[x];
                    } else {
                        while (x != u_in && nsb[x] < 0) x = par[x];
                        if (x == u_in) break;
                        x = nsb[x];
                    }
                    dep[x] = (short)(dep[par[x]] + 1);
                    pi[x] += sigma;
                }
            }
        }
        __syncthreads();
        if (flag[0]) {
            status = flag[0];
            break;
        }
    }

    // ---- the plan: real tree arcs carry the flow, every other arc is 0
    double cost = 0.0, art = 0.0;
    for (int u = tid; u < N - 1; u += NT) {
        const int p = par[u];
        if (p == R) {
            art = fmax(art, tflow[u]);
        } else {
            const int i = u < n ? u : p, j = (u < n ? p : u) - n;
            P.T[(int64_t)i * P.ldt + j] = tflow[u];
            cost += tflow[u] * P.M[(int64_t)i * P.ldm + j];
        }
    }
    cost = wave_sum(cost);
    art = wave_max(art);
    __syncthreads();
    if (lane == 0) {
        rv[wid] = cost;
        rv[kNW + wid] = art;
    }
    __syncthreads();
    double tot_mass = 0.0;
    for (int i = 0; i < n; ++i) tot_mass += P.a[i];
    double c = rv[0], a = rv[kNW];
    for (int w = 1; w < kNW; ++w) {
        c += rv[w];
        a = fmax(a, rv[kNW + w]);
    }
    __syncthreads();  // rv is reused by the caller
    if (status == OTF_EMD_OPTIMAL && a > 1e-9 * (tot_mass > 0.0 ? tot_mass : 1.0))
        status = OTF_EMD_INFEASIBLE;
    otf_emd_info out;
    out.cost = c;
    out.status = status;
    out.n_pivots = (int32_t)(pivots < INT32_MAX ? pivots : INT32_MAX);
    out.max_artificial_flow = a;
    return out;
}


}  // namespace otf
