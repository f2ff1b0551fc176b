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
// unbounded.  The tree lives in LDS as parent pointers plus a PRE-ORDER ARRAY
// (ord / pos) and subtree sizes, so every subtree is one contiguous range of ord and
// x is an ancestor of y iff pos[x] <= pos[y] < pos[x] + sz[x].  Per pivot:
//   * pricing: block search over all arcs (blocks of max(sqrt(A), 256) arcs from a
//     rotating cursor); the workgroup's threads scan a block and reduce to the most
//     negative reduced cost c_e + pi_s - pi_t (ties -> first in block order);
//   * one thread: the join of the cycle (walk up from s until an ancestor of t), the
//     ratio test with Cunningham's last-blocking-arc rule (keeps the tree strongly
//     feasible, so degenerate pivots cannot cycle), the flow update along the cycle,
//     and the path u_in .. u_out that the cut subtree S is re-rooted along;
//   * all threads: S's new pre-order is the concatenation of 2k + 1 ranges of the old
//     one (each path node's own part before / after the branch towards u_in), built
//     in parallel; one thread fixes the sizes on the path and on the two ancestor
//     chains and reverses the parents; all threads then move S behind v_in (one
//     parallel block shift of ord), update pos and shift the potentials of S by the
//     entering arc's reduced cost — O(cycle + path) serial work, O(N / threads)
//     parallel work, instead of a serial walk over the moved subtree.
// Tree arcs have reduced cost 0, so pricing needs no arc state; the flow of a tree
// arc lives with its child node, so the plan is written once at the end.
// One workgroup per problem: a batch (the per-label plans of one COOT-L step) is one
// launch.  Per node 31 B of LDS (16-bit tree indices): n + m + 1 <= kEmdMaxNodes.
// Larger problems (POT's emd has no node ceiling: a feature plan at d + d' > 4799, or
// a large --max-jax-samples) keep the tree in global memory instead -- 45 B per node
// with 32-bit indices, L2-resident up to ~90 k nodes per XCC -- and only the
// workgroup's reduction scratch in LDS; same algorithm, same pivots.
#pragma once
#include "otf_device.h"

namespace otf {

#ifdef OTF_EMD_STAMPS
// diagnostic build only (tools/stamps_emd.hip): ticks in pricing / tree work, blocks
// priced, subtree nodes moved, cycle nodes walked (workgroup 0)
__device__ unsigned long long g_emd_stats[8];
#endif

constexpr int kEmdMaxNodes = 4800;                    // LDS-resident tree (16-bit indices)
constexpr size_t kEmdScratch = 256 * (8 + 4) + 128;  // reductions of up to 256 threads
// pi, tflow | par sz pos ord tmp shift path | sgn
template <typename IX> constexpr size_t emd_node_bytes() { return 2 * 8 + 7 * sizeof(IX) + 1; }
constexpr size_t kEmdNodeBytes = emd_node_bytes<short>();

// LDS of emd_block for n + m + 1 = N nodes (tree and scratch in LDS)
inline __host__ __device__ size_t emd_lds_bytes(int N) {
    return ((size_t)N * kEmdNodeBytes + 15) / 16 * 16 + kEmdScratch;
}
// global-memory tree of emd_block<NT, int> for N nodes
inline __host__ __device__ size_t emd_tree_bytes_g(int64_t N) {
    return ((size_t)N * emd_node_bytes<int>() + 255) / 256 * 256;
}
// the global-tree form: n * m real arcs + N artificial ones index as int
inline __host__ __device__ bool emd_fits_g(int64_t n, int64_t m) {
    return n * m + n + m + 1 < (int64_t)INT32_MAX;
}

inline __device__ void argmin_pair(double& v, int& i, double v2, int i2) {
    if (v2 < v || (v2 == v && i2 < i)) {
        v = v2;
        i = i2;
    }
}

// One workgroup of NT threads solves one problem; every thread must call it.  tree:
// the node arrays (N * emd_node_bytes<IX>() bytes, 16-B aligned) -- LDS for IX = short,
// a workspace in global memory for IX = int; scr: kEmdScratch bytes of LDS.  P.a / P.b
// may point to LDS.  Every access goes through generic pointers, and __syncthreads
// orders global memory within the workgroup as it does LDS.
template <int NT, typename IX = short>
__device__ otf_emd_info emd_block(const otf_emd_problem& P, int64_t max_pivots, unsigned char* tree,
                                  unsigned char* scr) {
    static_assert(NT % 64 == 0 && NT <= 256, "whole waves; kEmdScratch holds 256 lanes");
    constexpr int kNW = NT / 64;
    const int n = P.n, m = P.m, N = n + m + 1, R = N - 1;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

    double* pi = reinterpret_cast<double*>(tree);  // node potentials
    double* tflow = pi + N;                         // flow of the tree arc (u, parent u)
    IX* par = reinterpret_cast<IX*>(tflow + N);
    IX* sz = par + N;                               // subtree sizes
    IX* pos = sz + N;                               // position in the pre-order
    IX* ord = pos + N;                              // the pre-order (ord[pos[x]] = x)
    IX* tmp = ord + N;                              // new pre-order of the moved subtree
    IX* shf = tmp + N;                              // the block of ord that shifts
    IX* path = shf + N;                             // u_in .. u_out
    signed char* sgn = reinterpret_cast<signed char*>(path + N);  // 1: supply > 0
    double* rv = reinterpret_cast<double*>(scr);
    int* ri = reinterpret_cast<int*>(rv + NT);
    int* flag = ri + NT;      // [0] stop code, [1..7] pivot scalars
    double* dsc = reinterpret_cast<double*>(scr + NT * 12 + 64);  // [0] sigma

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
        par[k] = (IX)R;
        tflow[k] = fabs(sup);
        pi[k] = sup > 0.0 ? -ART : ART;
        sz[k] = 1;
        pos[k] = (IX)(k + 1);
        ord[k + 1] = (IX)k;
    }
    if (tid == 0) {
        sgn[R] = 0;
        par[R] = -1;
        tflow[R] = 0.0;
        pi[R] = 0.0;
        sz[R] = (IX)N;
        pos[R] = 0;
        ord[0] = (IX)R;
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
    auto anc = [&](int x, int y) -> bool { return pos[x] <= pos[y] && pos[y] < pos[x] + sz[x]; };

    int next = 0;
    int64_t pivots = 0;
    int status = OTF_EMD_OPTIMAL;
#ifdef OTF_EMD_STAMPS
    unsigned long long st_t0 = __builtin_amdgcn_s_memrealtime(), st_price = 0, st_tree = 0, st_blocks = 0,
                       st_sub = 0;
#endif
    for (;;) {
#ifdef OTF_EMD_STAMPS
        st_t0 = __builtin_amdgcn_s_memrealtime();
#endif
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
                const double v2 = wave_xor_n<double>(bv, o);
                const int i2 = wave_xor_n<int>(bi, o);
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
#ifdef OTF_EMD_STAMPS
            ++st_blocks;
#endif
            if (bv < -tol) {
                in_arc = start + bi;
                if (in_arc >= A_tot) in_arc -= A_tot;
                in_rc = bv;
                break;
            }
        }
#ifdef OTF_EMD_STAMPS
        {
            const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
            st_price += t1 - st_t0;
            st_t0 = t1;
        }
#endif
        if (in_arc < 0) break;  // no arc prices out: optimal
        if (++pivots > max_pivots) {
            status = OTF_EMD_MAX_ITER;
            break;
        }

        // ---- tree work.  Phase A (one thread): cycle, ratio test, flows, the path.
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
            int join = s;
            while (!anc(join, t)) join = par[join];
            // flow runs join -> ... -> s -> t -> ... -> join; the blocking arcs are
            // those run against their direction; keep the LAST one met in that order
            // from the join (strongly feasible trees)
            double delta = INFINITY;
            int u_out = -1, side = 0, u;
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
                const int u_in = side == 1 ? s : t, v_in = side == 1 ? t : s;
                int k = 0;
                path[0] = (IX)u_in;
                for (u = u_in; u != u_out;) {
                    u = par[u];
                    path[++k] = (IX)u;
                }
                flag[1] = k;
                flag[2] = u_in;
                flag[3] = v_in;
                flag[4] = u_out;
                flag[5] = join;
                dsc[0] = side == 1 ? -in_rc : in_rc;  // potential shift of the moved subtree
                dsc[1] = delta;
            }
        }
        __syncthreads();
        if (flag[0]) {
            status = flag[0];
            break;
        }
        {
            const int k = flag[1], u_in = flag[2], v_in = flag[3], u_out = flag[4], join = flag[5];
            const int L = sz[u_out], a0 = pos[u_out], q = pos[v_in];
            // Phase B (all threads): the re-rooted subtree's pre-order from the old one:
            // u_in's whole old subtree, then for each path node its part before and after
            // the branch towards u_in
            {
                int off = 0;
                int st = pos[u_in], len = sz[u_in];
                for (int e = tid; e < len; e += NT) tmp[off + e] = ord[st + e];
                off += len;
                for (int i = 1; i <= k; ++i) {
                    const int pc = path[i], pm = path[i - 1];
                    st = pos[pc];
                    len = pos[pm] - pos[pc];
                    for (int e = tid; e < len; e += NT) tmp[off + e] = ord[st + e];
                    off += len;
                    st = pos[pm] + sz[pm];
                    len = pos[pc] + sz[pc] - st;
                    for (int e = tid; e < len; e += NT) tmp[off + e] = ord[st + e];
                    off += len;
                }
            }
            // the block of ord between the old and the new place of the subtree
            const bool right = q < a0;  // the subtree moves towards the root's end
            const int b0 = right ? q + 1 : a0 + L;
            const int nb = right ? a0 - q - 1 : q - a0 - L + 1;
            __syncthreads();
            // Phase C: one thread fixes sizes and parents (old sizes read before written,
            // path nodes in descending order); the others save the shifting block
            if (tid == 0) {
                const int w = par[u_out];
                for (int x = w; x != join; x = par[x]) sz[x] = (IX)(sz[x] - L);
                for (int x = v_in; x != join; x = par[x]) sz[x] = (IX)(sz[x] + L);
                int acc = 0;
                for (int i = k; i >= 1; --i) {
                    acc += sz[path[i]] - sz[path[i - 1]];
                    sz[path[i]] = (IX)acc;
                }
                sz[u_in] = (IX)L;
                double carry = dsc[1];
                int prev = v_in;
                for (int i = 0; i <= k; ++i) {
                    const int x = path[i];
                    const double f = tflow[x];
                    par[x] = (IX)prev;
                    tflow[x] = carry;
                    carry = f;
                    prev = x;
                }
            }
            for (int e = tid; e < nb; e += NT) shf[e] = ord[b0 + e];
            __syncthreads();
            // Phase D (all threads): the block shifts by L, the subtree lands behind v_in;
            // positions and the subtree's potentials follow
            const int nb0 = right ? q + 1 + L : a0;
            const int ns0 = right ? q + 1 : a0 + nb;
            const double sigma = dsc[0];
            for (int e = tid; e < nb; e += NT) {
                const int x = shf[e];
                ord[nb0 + e] = (IX)x;
                pos[x] = (IX)(nb0 + e);
            }
            for (int e = tid; e < L; e += NT) {
                const int x = tmp[e];
                ord[ns0 + e] = (IX)x;
                pos[x] = (IX)(ns0 + e);
                pi[x] += sigma;
            }
#ifdef OTF_EMD_STAMPS
            if (tid == 0) st_sub += (unsigned long long)L;
#endif
        }
        __syncthreads();
#ifdef OTF_EMD_STAMPS
        st_tree += __builtin_amdgcn_s_memrealtime() - st_t0;
#endif
    }

#ifdef OTF_EMD_STAMPS
    if (tid == 0 && blockIdx.x == 0) {
        g_emd_stats[0] = st_price;
        g_emd_stats[1] = st_tree;
        g_emd_stats[2] = st_blocks;
        g_emd_stats[3] = st_sub;
        g_emd_stats[4] = (unsigned long long)pivots;
    }
#endif
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
