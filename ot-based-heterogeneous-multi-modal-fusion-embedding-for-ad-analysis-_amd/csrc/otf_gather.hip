// otf_gather.hip — Sinkhorn for small problems with no device-wide barrier
// (OTF_ENGINE_GATHER), POT flavour.
//
// Replaces ot.sinkhorn (POT 0.9.6 sinkhorn_knopp, MRI_PET_OT_nojax.py:143 /
// perturbot/perturbot/match/utils.py:6-115) for the per-batch feature plans of the
// training loop (BASELINE config 2: d x d = 512 x 512, float64, up to 2000 iterations
// per training step) and every other problem of <= 16 row tiles x <= 512 columns.
//
// Like the tiled engine, workgroup w keeps a 2-D tile of K = exp(-C/reg) in registers
// for the whole solve (8 waves x 8 rows for double / 16 rows for float, every lane 8
// columns); the tile spans ALL columns, so the row sums K v are finished inside the
// wave.  The column sums K^T u are the only device-wide exchange.  Instead of float
// atomics into a shared buffer followed by a grid barrier and a re-read (three memory
// round trips, 4.4 of 6.7 us per iteration at config 2), every workgroup PUBLISHES its
// column partials as epoch-tagged granules (R2 form, cdna_hip_programming.md Guideline
// 16: {value word, tag} 8-byte granules, a float per granule or a double as two, one
// 16-B write-through store per two granules) and every workgroup GATHERS all the
// partials itself, polling until every tag carries the epoch it waits for.  The data
// is its own flag: no fence, no counter, no barrier.  One memory hop per iteration.
//
// Every workgroup adds the partials in the same fixed order (workgroup 0, 1, ...), so
// every workgroup holds bit-identical column sums and takes POT's decisions
// (convergence, numerical break) at the same iteration with no further exchange, and
// the result is bitwise reproducible run to run (deterministic by construction).
//
// Tags: partials of S[k] = K^T u(k-1) carry epoch k + 1 (slot k & 1) and the OR of the
// producer's numerical-break flags of iteration k - 1 (non-finite u or v) in bit 0:
// tag = ((k + 1) << 1) | bad.  A slot is rewritten two epochs later, which no producer
// can reach before every consumer has finished reading it (producing S[k + 2] needs
// S[k + 1], which each workgroup publishes only after its gather of S[k]).  Every poll
// is bounded by s_memrealtime (re-armed after each completed gather): a stall ends in
// OTF_SK_TIMEOUT.
#include "otf_persist.h"

namespace otf {
namespace {

template <typename T> struct GatherCfg {
    static constexpr int NW = 8;                        // waves per workgroup
    static constexpr int RW = sizeof(T) == 4 ? 16 : 8;  // rows per wave
    static constexpr int VEC = Vec<T>::N;
    static constexpr int G = sizeof(T) == 4 ? 2 : 4;    // VEC-vectors per lane: 8 columns
    static constexpr int TR = RW * NW;                  // rows per workgroup: 128 / 64
    static constexpr int C = kWave * G * VEC;           // 512 columns
    static constexpr int CPC = 8 / (int)sizeof(T);      // columns per 16-B chunk (2 granules)
    static constexpr int NCH = C / CPC;                 // chunks per producer row
};
constexpr int kGatherMaxWG = 16;
constexpr uint32_t kGatherRow = 8192;  // bytes per producer row of one slot (512 chunks)

template <typename T> struct SkGatherArgs {
    const void* C;
    int64_t ldc;
    int n, m;
    const T* a;        // padded marginals (zero past n / m)
    const T* b;
    const T* cost_scale;
    double reg;
    int max_iter, check_every, err_squared;
    double stop_thr;
    void* gran;        // [2 slots][grid][kGatherRow] granules, zeroed per solve
    int* team;         // [8 x 64] workgroups per XCC, [8 * 64] the winning team's XCC + 1
    int nwg;           // workgroups of the solve (the launch has 8 x nwg in team mode)
    int team_mode;
    otf_sinkhorn_info* info;
    double* errlog;
    T* u_out;
    T* v_out;
    void* P;
    int64_t ldp;
    unsigned long long timeout_ticks;
    unsigned long long reg_ticks;  // the first wait (registration / first hop)
};

using I4 = __attribute__((ext_vector_type(4))) int;

template <typename T> __device__ __forceinline__ void chunk_values(const I4 x, T (&v)[GatherCfg<T>::CPC]) {
    if constexpr (sizeof(T) == 8) {
        v[0] = __builtin_bit_cast(double, ((unsigned long long)(unsigned)x[2] << 32) | (unsigned)x[0]);
    } else {
        // element copies first: __builtin_bit_cast of a vector ELEMENT reads the vector's
        // first word (ROCm 7.2 clang; found by the float parity test)
        const int w0 = x[0], w2 = x[2];
        v[0] = __builtin_bit_cast(float, w0);
        v[1] = __builtin_bit_cast(float, w2);
    }
}
template <typename T> __device__ __forceinline__ I4 make_chunk(const T (&v)[GatherCfg<T>::CPC], int tag) {
    I4 x;
    if constexpr (sizeof(T) == 8) {
        const unsigned long long bits = __builtin_bit_cast(unsigned long long, v[0]);
        x[0] = (int)(unsigned)bits;
        x[2] = (int)(unsigned)(bits >> 32);
    } else {
        x[0] = __builtin_bit_cast(int, v[0]);
        x[2] = __builtin_bit_cast(int, v[1]);
    }
    x[1] = tag;
    x[3] = tag;
    return x;
}

// NQ: producers polled per pass, the grid rounded up to 4 / 8 / 16 (surplus slots
// re-read the last producer, so every load is unconditional and in flight together).
// SNWG: the row tiles compiled in (0 = from the arguments): a compiled-in shape is
// SNWG whole row tiles x all C columns (BASELINE config 2: 512 x 512 float64 = 8 tiles),
// so every bound test and derived count folds away.
template <typename T, typename CT, typename TP, int NQ, int SNWG>
__global__ __launch_bounds__(512) void sk_gather_kernel(SkGatherArgs<T> p) {
    using Cf = GatherCfg<T>;
    constexpr int G = Cf::G, VEC = Cf::VEC, R = Cf::RW, NW = Cf::NW, TR = Cf::TR;
    constexpr int CPC = Cf::CPC, NCH = Cf::NCH;
    using V = typename Vec<T>::type;
    using VP = __attribute__((ext_vector_type(VEC))) TP;
    __shared__ __attribute__((aligned(16))) T colbuf[NW][Cf::C];
    __shared__ __attribute__((aligned(16))) T vcur[Cf::C];      // v = b / (gathered K^T u)
    __shared__ __attribute__((aligned(16))) T vhist[2][Cf::C];  // v by iteration parity
    __shared__ T uhist[2][TR];
    __shared__ T red[17 + 17];
    // workgroup-wide flags without a reduction: a raised flag is the EPOCH written by any
    // lane that raises it before the barrier, compared with the epoch after it (epochs
    // only grow, so no word is ever reset).  [0] publish: break in this workgroup's
    // rows; [1..3] gather: break flagged by a producer, stall, break in v.
    __shared__ int s_ep[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    constexpr bool FULL = SNWG != 0;
    const int nwg = FULL ? SNWG : p.nwg;
    const int n_ = FULL ? SNWG * TR : p.n, m_ = FULL ? Cf::C : p.m;
    auto row_in = [&](int r) -> bool { return FULL || r < n_; };
    auto col_in = [&](int c) -> bool { return FULL || c < m_; };
    unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + p.reg_ticks;
    // Team mode: the launch has 8 x nwg workgroups; each registers on its hardware XCC
    // and the first XCC whose first nwg registrants are all resident claims the solve,
    // every other workgroup returns at once.  The team's hand-offs then stay inside one
    // XCC's L2 -- the point of coherence for all its CUs -- so the granules go out as
    // plain stores (L1 is write-through; the line stays in L2) read by L1-bypassing sc1
    // loads: no write-through to the Infinity Fabric and back per iteration.  The roles
    // follow the registration (hardware ids), never an assumed placement; by pigeonhole
    // some XCC receives nwg of the 8 x nwg workgroups.
    int wgi = blockIdx.x, xl = 0;
    if (p.team_mode) {
        __shared__ int s_team[2];
        const int xcd = xcc_id();
        if (tid == 0) {
            const int slot = __hip_atomic_fetch_add(p.team + xcd * 64, 1, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
            int keep = slot < nwg ? 1 : 0;
            if (keep) {
                // wait until this XCC's team is complete or another team has claimed
                for (;;) {
                    if (load_agent(&p.info->stalled)) {  // another registrant gave up
                        keep = 0;
                        break;
                    }
                    const int claim = load_agent(p.team + 8 * 64);
                    if (claim != 0) {
                        keep = claim == xcd + 1;
                        break;
                    }
                    if (load_agent(p.team + xcd * 64) >= nwg) {
                        if (slot == 0) {
                            int expected = 0;
                            __hip_atomic_compare_exchange_strong(p.team + 8 * 64, &expected, xcd + 1,
                                                                 __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_AGENT);
                        }
                    }
                    if (__builtin_amdgcn_s_memrealtime() > deadline) {
                        // no XCC team ever claimed the solve (a slot already left, or
                        // another persistent grid holds the CUs): report the stall, or
                        // the untouched u / v / plan would read as a finished solve
                        keep = 0;
                        store_wt(&p.info->stalled, 1);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            s_team[0] = keep;
            s_team[1] = slot;
        }
        __syncthreads();
        if (!s_team[0]) return;
        wgi = s_team[1];
        xl = 1;
        deadline = __builtin_amdgcn_s_memrealtime() + p.timeout_ticks;
    }
    const bool lead = (wgi == 0 && tid == 0);
    const int row0 = wgi * TR + w * R;

    const double unit = exp_unit<T>();
    double cinv = 1.0;
    if (p.cost_scale) cinv = 1.0 / (double)p.cost_scale[0];
    const T ks = (T)(-unit / p.reg * cinv);

    int colc[G];
    bool cok[G][VEC];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int c0 = (lane + kWave * g) * VEC;
        colc[g] = col_in(c0) ? c0 : 0;
#pragma unroll
        for (int k = 0; k < VEC; ++k) cok[g][k] = col_in(c0 + k);
    }
    // ---- K for this wave's rows x this lane's 8 columns, once
    T kv[R][G][VEC];
    {
        const CT* crow = (const CT*)p.C + (int64_t)row0 * p.ldc;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const CT* src = row_in(row0 + r) ? crow : (const CT*)p.C;
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
            const bool rok = row_in(row0 + r);
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int k = 0; k < VEC; ++k)
                    kv[r][g][k] = (rok && cok[g][k]) ? fast_exp(kv[r][g][k] * ks) : (T)0;
        }
    }
    // the row whose total this lane holds after wave_row_totals: lane >> RSH
    constexpr int RSH = R == 16 ? 2 : 3;
    const int myrow = lane >> RSH;
    const T ia_mine = (T)1 / p.a[row_in(row0 + myrow) ? row0 + myrow : n_ - 1];
    // this thread's gathered columns (chunk tid): their target marginal
    T bch[CPC];
#pragma unroll
    for (int c = 0; c < CPC; ++c) {
        const int col = tid * CPC + c;
        bch[c] = (tid < NCH && col_in(col)) ? p.b[col] : (T)0;
    }
    const T u0 = (T)1 / (T)n_, v0 = (T)1 / (T)m_;
    if (tid < 4) s_ep[tid] = -1;
    for (int q = tid; q < Cf::C; q += blockDim.x) vhist[0][q] = vhist[1][q] = v0;
    if (tid < TR) uhist[0][tid] = uhist[1][tid] = u0;

    const __amdgpu_buffer_rsrc_t rs = sums_rsrc(p.gran);
    const uint32_t my_row = (uint32_t)wgi * kGatherRow + (uint32_t)tid * 16;

    // publish this workgroup's partials of S[k] = K_tile^T wr (epoch k + 1, slot k & 1)
    auto publish = [&](const T (&wr)[R], int k, int bad_local) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            V acc;
#pragma unroll
            for (int q = 0; q < VEC; ++q) {
                T sacc = 0;
#if defined(OTF_GATHER_ABLATE) && (OTF_GATHER_ABLATE & 4)
                sacc = kv[0][g][q] * wr[0];  // diagnostic: no column-partial FMAs
#else
#pragma unroll
                for (int r = 0; r < R; ++r) sacc += kv[r][g][q] * wr[r];
#endif
                acc[q] = sacc;
            }
            *reinterpret_cast<V*>(&colbuf[w][(lane + kWave * g) * VEC]) = acc;
        }
        if (bad_local) s_ep[0] = k;
        __syncthreads();
        const int bad = s_ep[0] == k ? 1 : 0;
        if (tid < NCH) {
            T val[CPC];
#pragma unroll
            for (int c = 0; c < CPC; ++c) {
                T sacc = colbuf[0][tid * CPC + c];
#pragma unroll
                for (int ww = 1; ww < NW; ++ww) sacc += colbuf[ww][tid * CPC + c];
                val[c] = sacc;
            }
            const uint32_t off = (uint32_t)(k & 1) * (uint32_t)nwg * kGatherRow + my_row;
            if (xl)  // one XCC: plain store, the line stays in its L2
                __builtin_amdgcn_raw_buffer_store_b128(make_chunk<T>(val, ((k + 1) << 1) | bad), rs, off, 0, 0);
            else
                __builtin_amdgcn_raw_buffer_store_b128(make_chunk<T>(val, ((k + 1) << 1) | bad), rs, off, 0,
                                                       16 /* sc1 */);
        }
    };
    // gather S[k]: every producer's chunk `tid`, summed in producer order, and, for those
    // columns, v = b / S[k] into vcur (once per column, not once per wave) and, when
    // eslot >= 0, this thread's terms of the marginal error of the iterate whose v is
    // vhist[eslot].  Returns bit 0 = a producer flagged a break in iteration k - 1,
    // bit 1 = stall, bit 2 = a zero sum or non-finite v (POT's break test on v).
    auto gather = [&](int k, int eslot, T& e_loc) -> int {
        int fl = 0;
        e_loc = 0;
        if (tid < NCH) {
            const unsigned ep = (unsigned)(k + 1);
            const uint32_t base = (uint32_t)(k & 1) * (uint32_t)nwg * kGatherRow + (uint32_t)tid * 16;
            I4 x[NQ];
            for (;;) {
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const uint32_t src = (uint32_t)(q < nwg ? q : nwg - 1) * kGatherRow;
                    x[q] = __builtin_bit_cast(
                        I4, __builtin_amdgcn_raw_buffer_load_b128(rs, base + src, 0, 16 /* sc1 */));
                }
                bool ok = true;
#pragma unroll
                for (int q = 0; q < NQ; ++q)
                    ok &= ((unsigned)x[q][1] >> 1) == ep && ((unsigned)x[q][3] >> 1) == ep;
#if defined(OTF_GATHER_ABLATE) && (OTF_GATHER_ABLATE & 1)
                ok = true;  // diagnostic: one load pass, no wait for the producers
#endif
                if (ok) break;
                if (__builtin_amdgcn_s_memrealtime() > deadline) {
                    fl |= 2;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            T sv[CPC];
#pragma unroll
            for (int c = 0; c < CPC; ++c) sv[c] = 0;
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                if (q < nwg) {
                    T v[CPC];
                    chunk_values<T>(x[q], v);
#pragma unroll
                    for (int c = 0; c < CPC; ++c) sv[c] += v[c];
                    fl |= x[q][1] & 1;
                }
            }
#pragma unroll
            for (int c = 0; c < CPC; ++c) {
                const int col = tid * CPC + c;
                const bool ok = col_in(col);
                const T val = bch[c] / sv[c];
                fl |= (ok && ((sv[c] == (T)0) || !finite_val(val))) ? 4 : 0;
                vcur[col] = ok ? val : (T)0;
                if (eslot >= 0) {
                    const T rr = vhist[eslot][col] * sv[c] - bch[c];
                    e_loc += ok ? rr * rr : (T)0;
                }
            }
        }
        if (fl & 1) s_ep[1] = k;
        if (fl & 2) s_ep[2] = k;
        if (fl & 4) s_ep[3] = k;
        __syncthreads();
        const int f = (s_ep[1] == k ? 1 : 0) | (s_ep[2] == k ? 2 : 0) | (s_ep[3] == k ? 4 : 0);
        deadline = __builtin_amdgcn_s_memrealtime() + p.timeout_ticks;
        return f;
    };
    auto marg_error = [&](T e_loc) -> double {
        const T e = block_sum<T>(e_loc, red);
        return p.err_squared ? (double)e : sqrt((double)e);
    };

    // ---- prologue: S[0] = K^T u0
    {
        T wr[R];
#pragma unroll
        for (int r = 0; r < R; ++r) wr[r] = row_in(row0 + r) ? u0 : (T)0;
        publish(wr, 0, 0);
    }
    int last_good = -1, niter = 0, status = OTF_SK_MAX_ITER, brk = -1, n_err = 0;
    bool done = false;

    for (int it = 0; it < p.max_iter; ++it) {
        OTF_STAMP(it, 0);
        const bool check = it >= 1 && ((it - 1) % p.check_every) == 0;
        T e_loc;
        const int fl = gather(it, check ? (it - 1) & 1 : -1, e_loc);
        OTF_STAMP(it, 1);
        if (fl & 2) {
            status = OTF_SK_TIMEOUT;
            done = true;
            break;
        }
        // a numerical break in iteration it-1 (any workgroup) -> revert to it-2
        if (fl & 1) {
            last_good = it - 2; niter = it - 1; status = OTF_SK_NUMERICAL_BREAK; brk = it - 1;
            done = true;
            break;
        }
        // marginal error of iterate it-1 (identical in every workgroup)
        if (check) {
            const double err = marg_error(e_loc);
            if (lead) p.errlog[(it - 1) / p.check_every] = err;
            n_err = (it - 1) / p.check_every + 1;
            if (p.err_squared ? !(err > p.stop_thr) : (err < p.stop_thr)) {
                last_good = it - 1; niter = it - 1; status = OTF_SK_CONVERGED;
                done = true;
                break;
            }
        }
        const int badv = (fl & 4) ? 1 : 0;   // flagged with this iteration's partials
        T vn[G][VEC];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const V t = *reinterpret_cast<const V*>(&vcur[(lane + kWave * g) * VEC]);
#pragma unroll
            for (int k = 0; k < VEC; ++k) vn[g][k] = t[k];
        }
        OTF_STAMP(it, 2);
        // row sums over all columns: wave totals are the row sums
        T rp[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            T acc = 0;
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int k = 0; k < VEC; ++k) acc += kv[r][g][k] * vn[g][k];
#if defined(OTF_GATHER_ABLATE) && (OTF_GATHER_ABLATE & 2)
            acc = kv[r][0][0] * vn[0][0];  // diagnostic: no row-sum FMAs
#endif
            rp[r] = acc;
        }
        // wave totals (lane L: row L >> RSH), u of that row in every lane, then to every
        // lane as wave-uniform values (v_readlane: no LDS round trip); the first lane of
        // each row group keeps the history
        const int slot = it & 1;
        T un[R];
        int badu = 0;
        {
            const T tot = wave_row_totals<T, R>(rp, lane);
            T um = (T)1 / (tot * ia_mine);
            if (!row_in(row0 + myrow)) um = 0;
            badu = __any(!finite_val(um)) ? 1 : 0;
#pragma unroll
            for (int r = 0; r < R; ++r)
                un[r] = map_words(um, [&](unsigned wd) { return (unsigned)__builtin_amdgcn_readlane((int)wd, r << RSH); });
            if ((lane & ((1 << RSH) - 1)) == 0) uhist[slot][w * R + myrow] = um;
        }
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
        publish(un, it + 1, badv | badu);
        OTF_STAMP(it, 4);
        OTF_STAMP(it, 5);
    }
    if (!done && p.max_iter > 0) {
        // the last iteration's break flags and K^T u(max_iter - 1)
        const int it = p.max_iter - 1;
        const bool check = (it % p.check_every) == 0;
        T e_loc;
        const int fl = gather(p.max_iter, check ? it & 1 : -1, e_loc);
        if (fl & 2) {
            status = OTF_SK_TIMEOUT;
        } else if (fl & 1) {
            last_good = it - 1; niter = it; status = OTF_SK_NUMERICAL_BREAK; brk = it;
        } else {
            last_good = it; niter = it;
            if (check) {
                const double err = marg_error(e_loc);
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
    if (lane < R && row_in(row0 + lane)) {
        T mine = uo[0];
#pragma unroll
        for (int r = 1; r < R; ++r) if (lane == r) mine = uo[r];
        p.u_out[row0 + lane] = mine;
    }
    if (wgi == 0 && w == 0) {
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
            if (!row_in(row0 + r)) break;
            TP* prow = P + (int64_t)(row0 + r) * p.ldp;
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const int c0 = (lane + kWave * g) * VEC;
                if (!col_in(c0)) continue;
                VP o;
#pragma unroll
                for (int k = 0; k < VEC; ++k) o[k] = (TP)(uo[r] * kv[r][g][k] * vo[g][k]);
                if (FULL || c0 + VEC <= m_) {
                    *reinterpret_cast<VP*>(prow + c0) = o;
                } else {
#pragma unroll
                    for (int k = 0; k < VEC; ++k)
                        if (col_in(c0 + k)) prow[c0 + k] = o[k];
                }
            }
        }
    }
    if (status == OTF_SK_TIMEOUT && tid == 0) store_wt(&p.info->stalled, 1);
    if (lead) {
        p.info->last_good = last_good;
        p.info->niter = niter;
        p.info->status = status;
        p.info->break_iter = brk;
        p.info->n_err = n_err;
        p.info->engine = OTF_ENGINE_GATHER;
        p.info->stop = 1;
    }
}

// ============================================================================
// Two-hop form (r03): reduce-scatter + all-gather inside the team's XCC.
//
// The one-hop gather above makes every workgroup read every producer's partials of all
// columns: nwg x 8 KB per workgroup per iteration through the CU's 64 B/clk port, so
// spreading the rows over more workgroups (less VALU per workgroup) costs as much in
// gather bandwidth as it saves.  Here the column partials go to REDUCERS (workgroup j
// owns chunks [j CPR, (j + 1) CPR)): one wave polls them from the nwg producers, sums
// them in producer order, forms v = b / S for its columns, POT's break test on them and
// its share of the marginal error, and publishes the v chunks; every workgroup then
// gathers one chunk per thread.  Two L2-local hops instead of one, but each moves
// 1 / nwg of the bytes, so the rows spread over 16 - 32 workgroups (R = 4 or 2 rows per
// wave for float64: 2 - 4x less VALU per iteration than R = 8).
//
// Tags of the v chunks of S[k] (epoch k + 1, slot k & 1): bit 0 = a producer's u of
// iteration k - 1 was not finite (-> break at k - 1), bit 1 = S[k] has a zero or v a
// non-finite value (-> break at k).  The error chunk (index CPR of a reducer) carries the
// reducer's terms of the marginal error of iterate k - 1 (v(k - 1) S[k] - b) when k - 1
// is a check iteration.  Every workgroup sums the nwg error terms in reducer order, so all
// take POT's decisions at the same iteration, bitwise reproducible as the one-hop form.
// Slot reuse: a producer writes slot k & 1 again for S[k + 2] after gathering the v
// chunks of S[k + 1], which every reducer published after reading its S[k + 1] partials,
// after (program order) reading those of S[k]; the v-chunk slots the same way round.
// ============================================================================
constexpr int kG2MaxWG = 32;
constexpr uint32_t kG2BStride = 1280;  // per reducer: <= 64 v chunks + the error chunk (256-B multiple)

template <typename T> struct G2Shape {
    int nwg, cpr, kq;
};
template <typename T> G2Shape<T> g2_shape(int64_t n, int R) {
    using Cf = GatherCfg<T>;
    G2Shape<T> g{};
    g.nwg = (int)((n + 8 * R - 1) / (8 * R));
    int per = (Cf::NCH + g.nwg - 1) / (g.nwg > 0 ? g.nwg : 1);
    int cpr = 1;
    while (cpr < per) cpr <<= 1;
    g.cpr = cpr;
    g.kq = (g.nwg * cpr + kWave - 1) / kWave;  // reducer loads per lane
    return g;
}

template <typename T, typename CT, typename TP, int R, int KQ>
__global__ __launch_bounds__(512) void sk_gather2_kernel(SkGatherArgs<T> p, int CPR, uint32_t off_b) {
    using Cf = GatherCfg<T>;
    constexpr int G = Cf::G, VEC = Cf::VEC, NW = Cf::NW, TR = NW * R;
    constexpr int CPC = Cf::CPC, NCH = Cf::NCH;
    constexpr int RSH = R == 16 ? 2 : R == 8 ? 3 : R == 4 ? 4 : 5;
    using V = typename Vec<T>::type;
    using VP = __attribute__((ext_vector_type(VEC))) TP;
    __shared__ __attribute__((aligned(16))) T colbuf[NW][Cf::C];
    __shared__ __attribute__((aligned(16))) T vcur[Cf::C];
    __shared__ __attribute__((aligned(16))) T vhist[2][Cf::C];
    __shared__ T uhist[2][TR];
    __shared__ T s_err;
    // raised flags hold the key of the step that raised them (keys only grow): [0] this
    // workgroup's u not finite, [1] producer break flag, [2] stall, [3] v break flag,
    // [4] reducer stall
    __shared__ int s_ep[5];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int nwg = p.nwg, n_ = p.n, m_ = p.m;
    auto row_in = [&](int r) -> bool { return r < n_; };
    auto col_in = [&](int c) -> bool { return c < m_; };
    unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + p.reg_ticks;
    // team registration (as the one-hop form): the first XCC whose first nwg registrants
    // are resident claims the solve; this form always runs as one XCC team
    int wgi;
    {
        __shared__ int s_team[2];
        const int xcd = xcc_id();
        if (tid == 0) {
            const int slot = __hip_atomic_fetch_add(p.team + xcd * 64, 1, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
            int keep = slot < nwg ? 1 : 0;
            if (keep) {
                for (;;) {
                    if (load_agent(&p.info->stalled)) {
                        keep = 0;
                        break;
                    }
                    const int claim = load_agent(p.team + 8 * 64);
                    if (claim != 0) {
                        keep = claim == xcd + 1;
                        break;
                    }
                    if (load_agent(p.team + xcd * 64) >= nwg && slot == 0) {
                        int expected = 0;
                        __hip_atomic_compare_exchange_strong(p.team + 8 * 64, &expected, xcd + 1, __ATOMIC_RELAXED,
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    if (__builtin_amdgcn_s_memrealtime() > deadline) {
                        keep = 0;
                        store_wt(&p.info->stalled, 1);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            s_team[0] = keep;
            s_team[1] = slot;
        }
        __syncthreads();
        if (!s_team[0]) return;
        wgi = s_team[1];
        deadline = __builtin_amdgcn_s_memrealtime() + p.timeout_ticks;
    }
    const bool lead = (wgi == 0 && tid == 0);
    const int row0 = wgi * TR + w * R;

    const double unit = exp_unit<T>();
    double cinv = 1.0;
    if (p.cost_scale) cinv = 1.0 / (double)p.cost_scale[0];
    const T ks = (T)(-unit / p.reg * cinv);

    int colc[G];
    bool cok[G][VEC];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int c0 = (lane + kWave * g) * VEC;
        colc[g] = col_in(c0) ? c0 : 0;
#pragma unroll
        for (int k = 0; k < VEC; ++k) cok[g][k] = col_in(c0 + k);
    }
    T kv[R][G][VEC];
    {
        const CT* crow = (const CT*)p.C + (int64_t)row0 * p.ldc;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const CT* src = row_in(row0 + r) ? crow : (const CT*)p.C;
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
            const bool rok = row_in(row0 + r);
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int k = 0; k < VEC; ++k)
                    kv[r][g][k] = (rok && cok[g][k]) ? fast_exp(kv[r][g][k] * ks) : (T)0;
        }
    }
    const int myrow = lane >> RSH;
    const T ia_mine = (T)1 / p.a[row_in(row0 + myrow) ? row0 + myrow : n_ - 1];
    const T u0 = (T)1 / (T)n_, v0 = (T)1 / (T)m_;
    if (tid < 5) s_ep[tid] = -1;
    for (int q = tid; q < Cf::C; q += blockDim.x) vhist[0][q] = vhist[1][q] = v0;
    if (tid < TR) uhist[0][tid] = uhist[1][tid] = u0;

    const __amdgpu_buffer_rsrc_t rs = sums_rsrc(p.gran);
    // reducer lanes (wave 0): chunk rc of this workgroup's range, producers rq + LPC k
    const int LPC = kWave / CPR;
    const int r_cc = lane & (CPR - 1), r_q = lane / CPR;
    const int r_ch = wgi * CPR + r_cc;
    const bool r_ok = r_ch < NCH;
    T rbv[CPC];
#pragma unroll
    for (int c = 0; c < CPC; ++c) {
        const int col = r_ch * CPC + c;
        rbv[c] = (r_ok && col_in(col)) ? p.b[col] : (T)0;
    }
    const int nred = (NCH + CPR - 1) / CPR;  // reducers holding chunks

    // partials of S[k] = K_tile^T wr, epoch k + 1, slot k & 1; bad = u not finite here
    auto publish = [&](const T (&wr)[R], int k, int bad_local) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            V acc;
#pragma unroll
            for (int q = 0; q < VEC; ++q) {
                T sacc = 0;
#pragma unroll
                for (int r = 0; r < R; ++r) sacc += kv[r][g][q] * wr[r];
                acc[q] = sacc;
            }
            *reinterpret_cast<V*>(&colbuf[w][(lane + kWave * g) * VEC]) = acc;
        }
        if (bad_local) s_ep[0] = k;
        __syncthreads();
        const int bad = s_ep[0] == k ? 1 : 0;
        if (tid < NCH) {
            T val[CPC];
#pragma unroll
            for (int c = 0; c < CPC; ++c) {
                T sacc = colbuf[0][tid * CPC + c];
#pragma unroll
                for (int ww = 1; ww < NW; ++ww) sacc += colbuf[ww][tid * CPC + c];
                val[c] = sacc;
            }
            const uint32_t off = ((uint32_t)(k & 1) * (uint32_t)nwg + (uint32_t)wgi) * kGatherRow + (uint32_t)tid * 16;
            __builtin_amdgcn_raw_buffer_store_b128(make_chunk<T>(val, ((k + 1) << 2) | bad), rs, off, 0, 0);
        }
    };
    // reducer (wave 0): S[k] of this workgroup's chunks from the nwg producers (producer
    // order), v = b / S[k], flags, and (need) the error terms of iterate k - 1 against
    // v(k - 1) = vprev; publishes the v chunks and the error chunk, epoch k + 1.
    // Returns false on a stall.
    auto reduce = [&](int k, bool need, const T* vprev) -> bool {
        const unsigned ep = (unsigned)(k + 1);
        I4 x[KQ];
        unsigned pend = 0;
#pragma unroll
        for (int q = 0; q < KQ; ++q) {
            x[q] = I4{0, 0, 0, 0};
            if (r_ok && r_q + LPC * q < nwg) pend |= 1u << q;
        }
        const uint32_t base = (uint32_t)(k & 1) * (uint32_t)nwg * kGatherRow + (uint32_t)r_ch * 16;
        bool ok = true;
        for (;;) {
#pragma unroll
            for (int q = 0; q < KQ; ++q)
                if (pend & (1u << q))
                    x[q] = gload(rs, base + (uint32_t)(r_q + LPC * q) * kGatherRow);
#pragma unroll
            for (int q = 0; q < KQ; ++q)
                if ((pend & (1u << q)) && ((unsigned)x[q][1] >> 2) == ep && ((unsigned)x[q][3] >> 2) == ep)
                    pend &= ~(1u << q);
            if (!__any(pend != 0)) break;
            if (__builtin_amdgcn_s_memrealtime() > deadline) { ok = false; break; }
            __builtin_amdgcn_s_sleep(1);
        }
        T sv[CPC];
        int fl = 0;
#pragma unroll
        for (int c = 0; c < CPC; ++c) sv[c] = 0;
#pragma unroll
        for (int q = 0; q < KQ; ++q)
            if (r_ok && r_q + LPC * q < nwg) {
                T v[CPC];
                chunk_values<T>(x[q], v);
#pragma unroll
                for (int c = 0; c < CPC; ++c) sv[c] += v[c];
                fl |= x[q][1] & 1;
            }
        // lanes of one chunk: offsets CPR, 2 CPR, ..., 32 (uniform, static DPP)
#pragma unroll
        for (int c = 0; c < CPC; ++c) {
            if (CPR <= 1) sv[c] += wave_xor<T, 1>(sv[c]);
            if (CPR <= 2) sv[c] += wave_xor<T, 2>(sv[c]);
            if (CPR <= 4) sv[c] += wave_xor<T, 4>(sv[c]);
            if (CPR <= 8) sv[c] += wave_xor<T, 8>(sv[c]);
            if (CPR <= 16) sv[c] += wave_xor<T, 16>(sv[c]);
            if (CPR <= 32) sv[c] += wave_xor<T, 32>(sv[c]);
        }
        const int pbad = __any(fl) ? 1 : 0;
        T vn[CPC];
        int vb = 0;
        T term = 0;
#pragma unroll
        for (int c = 0; c < CPC; ++c) {
            const int col = r_ch * CPC + c;
            const bool cin = r_ok && col_in(col);
            const T val = rbv[c] / sv[c];
            vb |= (cin && (sv[c] == (T)0 || !finite_val(val))) ? 1 : 0;
            vn[c] = cin ? val : (T)0;
            if (need && cin) {
                const T rr = vprev[col] * sv[c] - rbv[c];
                term += rr * rr;
            }
        }
        const int vbad = __any(vb) ? 2 : 0;
        const int tag = ((int)ep << 2) | pbad | vbad;
        const uint32_t ob = off_b + ((uint32_t)(k & 1) * (uint32_t)nwg + (uint32_t)wgi) * kG2BStride;
        if (lane < CPR && r_ok) __builtin_amdgcn_raw_buffer_store_b128(make_chunk<T>(vn, tag), rs, ob + (uint32_t)lane * 16, 0, 0);
        if (need) {
            // lanes of one chunk hold the same term: one copy per chunk, then the wave sum
            term = lane < CPR ? term : (T)0;
            term = wave_sum<T>(term);
            if (lane == 0 && wgi < nred) {
                T ev[CPC];
#pragma unroll
                for (int c = 0; c < CPC; ++c) ev[c] = c == 0 ? term : (T)0;
                __builtin_amdgcn_raw_buffer_store_b128(make_chunk<T>(ev, tag), rs, ob + (uint32_t)CPR * 16, 0, 0);
            }
        }
        deadline = __builtin_amdgcn_s_memrealtime() + p.timeout_ticks;
        return ok;
    };
    // hop B: v of S[k] (epoch k + 1) into vcur; the summed error terms into s_err when
    // need.  Returns bit 0 producer break, 1 stall, 2 v break.
    auto gather = [&](int k, bool need) -> int {
        const unsigned ep = (unsigned)(k + 1);
        int fl = 0;
        const uint32_t sb = off_b + (uint32_t)(k & 1) * (uint32_t)nwg * kG2BStride;
        if (tid < NCH) {
            const uint32_t off = sb + (uint32_t)(tid / CPR) * kG2BStride + (uint32_t)(tid & (CPR - 1)) * 16;
            I4 x;
            for (;;) {
                x = gload(rs, off);
                if (((unsigned)x[1] >> 2) == ep && ((unsigned)x[3] >> 2) == ep) break;
                if (__builtin_amdgcn_s_memrealtime() > deadline) { fl |= 2; x = I4{0, 0, 0, 0}; break; }
                __builtin_amdgcn_s_sleep(1);
            }
            fl |= (x[1] & 1) | ((x[1] & 2) << 1);  // tag bit 1 (v break) -> bit 2
            T v[CPC];
            chunk_values<T>(x, v);
#pragma unroll
            for (int c = 0; c < CPC; ++c) vcur[tid * CPC + c] = v[c];
        }
        if (need && w == NW - 1) {
            // the last wave sums the reducers' error terms in reducer order
            T e = 0;
            if (lane < nred) {
                const uint32_t off = sb + (uint32_t)lane * kG2BStride + (uint32_t)CPR * 16;
                I4 x;
                for (;;) {
                    x = gload(rs, off);
                    if (((unsigned)x[1] >> 2) == ep && ((unsigned)x[3] >> 2) == ep) break;
                    if (__builtin_amdgcn_s_memrealtime() > deadline) { fl |= 2; x = I4{0, 0, 0, 0}; break; }
                    __builtin_amdgcn_s_sleep(1);
                }
                T v[CPC];
                chunk_values<T>(x, v);
                e = v[0];
            }
            e = wave_sum<T>(e);
            if (lane == 0) s_err = e;
        }
        if (fl & 1) s_ep[1] = k;
        if (fl & 2) s_ep[2] = k;
        if (fl & 4) s_ep[3] = k;  // (bit 1 of the tag is bit 2 of fl: v break)
        __syncthreads();
        deadline = __builtin_amdgcn_s_memrealtime() + p.timeout_ticks;
        return (s_ep[1] == k ? 1 : 0) | (s_ep[2] == k ? 2 : 0) | (s_ep[3] == k ? 4 : 0) |
               (s_ep[4] == k ? 2 : 0);
    };
    auto to_err = [&](T e) -> double { return p.err_squared ? (double)e : sqrt((double)e); };
    auto stop_ok = [&](double err) -> bool { return p.err_squared ? !(err > p.stop_thr) : (err < p.stop_thr); };

    // ---- prologue: S[0] = K^T u0, its v chunks (epoch 1)
    {
        T wr[R];
#pragma unroll
        for (int r = 0; r < R; ++r) wr[r] = row_in(row0 + r) ? u0 : (T)0;
        publish(wr, 0, 0);
        if (w == 0 && !reduce(0, false, vhist[0])) s_ep[4] = 0;
    }
    int last_good = -1, niter = 0, status = OTF_SK_MAX_ITER, brk = -1, n_err = 0;
    bool done = false;
    for (int it = 0; it < p.max_iter; ++it) {
        OTF_STAMP(it, 0);
        const bool check = it >= 1 && ((it - 1) % p.check_every) == 0;
        const int fl = gather(it, check);
        OTF_STAMP(it, 1);
        if (fl & 2) { status = OTF_SK_TIMEOUT; done = true; break; }
        if (fl & 1) {  // u of iteration it - 1 not finite somewhere: revert to it - 2
            last_good = it - 2; niter = it - 1; status = OTF_SK_NUMERICAL_BREAK; brk = it - 1;
            done = true;
            break;
        }
        if (check) {
            const double err = to_err(s_err);
            if (lead) p.errlog[(it - 1) / p.check_every] = err;
            n_err = (it - 1) / p.check_every + 1;
            if (stop_ok(err)) {
                last_good = it - 1; niter = it - 1; status = OTF_SK_CONVERGED;
                done = true;
                break;
            }
        }
        if (fl & 4) {  // S[it] has a zero or v(it) is not finite: revert to it - 1
            last_good = it - 1; niter = it; status = OTF_SK_NUMERICAL_BREAK; brk = it;
            done = true;
            break;
        }
        T vn[G][VEC];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const V t = *reinterpret_cast<const V*>(&vcur[(lane + kWave * g) * VEC]);
#pragma unroll
            for (int k = 0; k < VEC; ++k) vn[g][k] = t[k];
        }
        OTF_STAMP(it, 2);
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
        const int slot = it & 1;
        T un[R];
        int badu = 0;
        {
            const T tot = wave_row_totals<T, R>(rp, lane);
            T um = (T)1 / (tot * ia_mine);
            if (!row_in(row0 + myrow)) um = 0;
            badu = __any(!finite_val(um)) ? 1 : 0;
#pragma unroll
            for (int r = 0; r < R; ++r)
                un[r] = map_words(um, [&](unsigned wd) { return (unsigned)__builtin_amdgcn_readlane((int)wd, r << RSH); });
            if ((lane & ((1 << RSH) - 1)) == 0) uhist[slot][w * R + myrow] = um;
        }
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
        publish(un, it + 1, badu);
        OTF_STAMP(it, 4);
        // S[it + 1]: the error of iterate it is checked at it + 1 when it % check_every == 0
        if (w == 0 && !reduce(it + 1, (it % p.check_every) == 0, vhist[slot])) s_ep[4] = it + 1;
        OTF_STAMP(it, 5);
    }
    if (!done && p.max_iter > 0) {
        const int it = p.max_iter - 1;
        const bool check = (it % p.check_every) == 0;
        const int fl = gather(p.max_iter, check);
        if (fl & 2) {
            status = OTF_SK_TIMEOUT;
        } else if (fl & 1) {
            last_good = it - 1; niter = it; status = OTF_SK_NUMERICAL_BREAK; brk = it;
        } else {
            last_good = it; niter = it;
            if (check) {
                const double err = to_err(s_err);
                if (lead) p.errlog[it / p.check_every] = err;
                n_err = it / p.check_every + 1;
                if (stop_ok(err)) status = OTF_SK_CONVERGED;
            }
        }
    }

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
    if (lane < R && row_in(row0 + lane)) {
        T mine = uo[0];
#pragma unroll
        for (int r = 1; r < R; ++r) if (lane == r) mine = uo[r];
        p.u_out[row0 + lane] = mine;
    }
    if (wgi == 0 && w == 0) {
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
            if (!row_in(row0 + r)) break;
            TP* prow = P + (int64_t)(row0 + r) * p.ldp;
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const int c0 = (lane + kWave * g) * VEC;
                if (!col_in(c0)) continue;
                VP o;
#pragma unroll
                for (int k = 0; k < VEC; ++k) o[k] = (TP)(uo[r] * kv[r][g][k] * vo[g][k]);
                if (c0 + VEC <= m_) {
                    *reinterpret_cast<VP*>(prow + c0) = o;
                } else {
#pragma unroll
                    for (int k = 0; k < VEC; ++k)
                        if (col_in(c0 + k)) prow[c0 + k] = o[k];
                }
            }
        }
    }
    if (status == OTF_SK_TIMEOUT && tid == 0) store_wt(&p.info->stalled, 1);
    if (lead) {
        p.info->last_good = last_good;
        p.info->niter = niter;
        p.info->status = status;
        p.info->break_iter = brk;
        p.info->n_err = n_err;
        p.info->engine = OTF_ENGINE_GATHER;
        p.info->stop = 1;
    }
}

template <typename T, typename CT, typename TP, int NQ>
hipError_t launch_gather_q(int grid, SkGatherArgs<T>& p, hipStream_t s) {
    void* args[] = {&p};
    // BASELINE config 2 (8 whole row tiles x 512 columns of float64) has its own
    // compiled-in instance
    const bool whole = p.n == p.nwg * GatherCfg<T>::TR && p.m == GatherCfg<T>::C;
    const void* k = (sizeof(T) == 8 && NQ == 8 && p.nwg == 8 && whole)
                        ? (const void*)sk_gather_kernel<T, CT, TP, NQ, (sizeof(T) == 8 && NQ == 8) ? 8 : 0>
                        : (const void*)sk_gather_kernel<T, CT, TP, NQ, 0>;
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 512, 0);
    if (e != hipSuccess) return e;
    if (per_cu < 1 || grid > per_cu * device_cu_count()) return hipErrorCooperativeLaunchTooLarge;
    return hipLaunchKernel(k, dim3(grid), dim3(512), args, 0, s);
}

// co-resident 512-thread workgroups per CU of the instance launch_gather picks (0 on error)
template <typename T, typename CT, typename TP>
int gather_per_cu_t(int nwg) {
    const void* k = nwg <= 4   ? (const void*)sk_gather_kernel<T, CT, TP, 4, 0>
                    : nwg <= 8 ? (const void*)sk_gather_kernel<T, CT, TP, 8, 0>
                               : (const void*)sk_gather_kernel<T, CT, TP, 16, 0>;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 512, 0) != hipSuccess) return 0;
    return per_cu;
}
template <typename T, typename CT>
int gather_per_cu(bool plan_f64, int nwg) {
    return plan_f64 ? gather_per_cu_t<T, CT, double>(nwg) : gather_per_cu_t<T, CT, float>(nwg);
}

template <typename T, typename CT, typename TP>
hipError_t launch_gather(int grid, SkGatherArgs<T>& p, hipStream_t s) {
    // NQ follows the solve's workgroups (p.nwg), not the launch (8 x nwg in team mode)
    if (p.nwg <= 4) return launch_gather_q<T, CT, TP, 4>(grid, p, s);
    if (p.nwg <= 8) return launch_gather_q<T, CT, TP, 8>(grid, p, s);
    return launch_gather_q<T, CT, TP, 16>(grid, p, s);
}

template <typename T> int64_t gather_grid(int64_t n) {
    return (n + GatherCfg<T>::TR - 1) / GatherCfg<T>::TR;
}

// Two-hop form: rows per wave (OTF_GATHER2_R, default 4), on (OTF_GATHER2, default 1)
inline int gather2_rows() {
    const char* e = getenv("OTF_GATHER2_R");
    const int r = e ? atoi(e) : 4;
    return r == 2 ? 2 : 4;
}
inline bool gather2_enabled() {
    const char* e = getenv("OTF_GATHER2");
    return e ? atoi(e) != 0 : true;
}
template <typename T> bool gather2_fits(int64_t n, int R) {
    const G2Shape<T> g = g2_shape<T>(n, R);
    return g.nwg >= 1 && g.nwg <= kG2MaxWG && g.cpr <= kWave;
}

template <typename T, typename CT, typename TP, int R, int KQ>
hipError_t launch_gather2_t(SkGatherArgs<T>& p, int cpr, uint32_t off_b, hipStream_t s) {
    const void* k = (const void*)sk_gather2_kernel<T, CT, TP, R, KQ>;
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 512, 0);
    if (e != hipSuccess) return e;
    const int grid = 8 * p.nwg;  // one team of nwg per XCC, the first complete one claims
    if (per_cu < 1 || grid > per_cu * device_cu_count()) return hipErrorCooperativeLaunchTooLarge;
    void* args[] = {&p, &cpr, &off_b};
    return hipLaunchKernel(k, dim3(grid), dim3(512), args, 0, s);
}
template <typename T, typename CT, typename TP, int R>
hipError_t launch_gather2_r(SkGatherArgs<T>& p, const G2Shape<T>& g, uint32_t off_b, hipStream_t s) {
    // loads per reducer lane: nwg * cpr / 64 lies in [NCH / 64, 2 NCH / 64]
    constexpr int KLO = GatherCfg<T>::NCH / kWave;
    if (g.kq <= KLO) return launch_gather2_t<T, CT, TP, R, KLO>(p, g.cpr, off_b, s);
    return launch_gather2_t<T, CT, TP, R, 2 * KLO>(p, g.cpr, off_b, s);
}

}  // namespace

template <typename T> bool gather_supported(int64_t n, int64_t m) {
    return n >= 1 && m >= 1 && m <= GatherCfg<T>::C && gather_grid<T>(n) <= kGatherMaxWG;
}

constexpr size_t kTeamBytes = 9 * 256;  // 8 XCC registration counters + the claim word

// one-hop: [2 slots][grid][kGatherRow]; two-hop: [2][<= 32 producers][kGatherRow] + the v
// chunks [2][<= 32 reducers][kG2BStride]
template <typename T> size_t gather_region_bytes(int64_t n, int64_t m) {
    if (!gather_supported<T>(n, m)) return 0;
    const size_t one = 2 * (size_t)gather_grid<T>(n) * kGatherRow;
    const size_t two = 2 * (size_t)kG2MaxWG * kGatherRow + 2 * (size_t)kG2MaxWG * kG2BStride;
    return kTeamBytes + (one > two ? one : two);
}

// OTF_GATHER_TEAM=0: one workgroup per row tile anywhere on the chip, write-through hops
inline int gather_team_mode() {
    const char* e = getenv("OTF_GATHER_TEAM");
    return e ? atoi(e) : 1;
}

template <typename T, typename CT>
hipError_t run_gather(const CT* C, int64_t ldc, int n, int m, const T* a_pad, const T* b_pad,
                      const T* cost_scale, const otf_sinkhorn_opts& o, void* region, T* u_out,
                      T* v_out, void* P_out, int64_t ldp, int P_dtype, otf_sinkhorn_info* info,
                      double* errlog, hipStream_t s) {
    if (!gather_supported<T>(n, m) || !region) return hipErrorInvalidValue;
    SkGatherArgs<T> p{};
    p.C = C;
    p.ldc = ldc;
    p.n = n;
    p.m = m;
    p.a = a_pad;
    p.b = b_pad;
    p.cost_scale = cost_scale;
    p.reg = o.reg;
    p.max_iter = o.max_iter;
    p.check_every = o.check_every;
    p.err_squared = o.err_squared;
    p.stop_thr = o.stop_thr;
    p.team = (int*)region;
    p.gran = (char*)region + kTeamBytes;
    p.info = info;
    p.errlog = errlog;
    p.u_out = u_out;
    p.v_out = v_out;
    p.P = P_out;
    p.ldp = ldp;
    p.timeout_ticks = stall_ticks();
    p.reg_ticks = reg_stall_ticks();
    hipError_t e = hipMemsetAsync(region, 0, gather_region_bytes<T>(n, m), s);
    if (e != hipSuccess) return e;
    // two-hop form: rows spread over 2 - 4x the workgroups, one XCC team
    const int R2 = gather2_rows();
    if (gather2_enabled() && gather_team_mode() && gather2_fits<T>(n, R2)) {
        const G2Shape<T> g = g2_shape<T>(n, R2);
        SkGatherArgs<T> q = p;
        q.nwg = g.nwg;
        q.team_mode = 1;
        const uint32_t off_b = 2u * (uint32_t)kG2MaxWG * kGatherRow;
        const bool f64p = P_out && P_dtype == OTF_F64;
        if (R2 == 2)
            e = f64p ? launch_gather2_r<T, CT, double, 2>(q, g, off_b, s) : launch_gather2_r<T, CT, float, 2>(q, g, off_b, s);
        else
            e = f64p ? launch_gather2_r<T, CT, double, 4>(q, g, off_b, s) : launch_gather2_r<T, CT, float, 4>(q, g, off_b, s);
        if (e != hipErrorCooperativeLaunchTooLarge) return e;
        (void)hipGetLastError();
    }
    const int grid = (int)gather_grid<T>(n);
    p.nwg = grid;
    p.team_mode = gather_team_mode();
    // team mode needs 8 x grid co-resident workgroups; on a smaller (or partitioned)
    // device fall back to one workgroup per row tile anywhere on the chip, as the mesh
    // engine does, instead of refusing the shape
    if (p.team_mode && 8 * grid > gather_per_cu<T, CT>(P_out && P_dtype == OTF_F64, grid) * device_cu_count())
        p.team_mode = 0;
    const int launch = p.team_mode ? 8 * grid : grid;
    if (P_out && P_dtype == OTF_F64) return launch_gather<T, CT, double>(launch, p, s);
    return launch_gather<T, CT, float>(launch, p, s);
}

template bool gather_supported<float>(int64_t, int64_t);
template bool gather_supported<double>(int64_t, int64_t);
template size_t gather_region_bytes<float>(int64_t, int64_t);
template size_t gather_region_bytes<double>(int64_t, int64_t);
template hipError_t run_gather<float, float>(const float*, int64_t, int, int, const float*, const float*,
                                             const float*, const otf_sinkhorn_opts&, void*, float*,
                                             float*, void*, int64_t, int, otf_sinkhorn_info*, double*,
                                             hipStream_t);
template hipError_t run_gather<float, _Float16>(const _Float16*, int64_t, int, int, const float*,
                                                const float*, const float*, const otf_sinkhorn_opts&,
                                                void*, float*, float*, void*, int64_t, int,
                                                otf_sinkhorn_info*, double*, hipStream_t);
template hipError_t run_gather<double, double>(const double*, int64_t, int, int, const double*,
                                               const double*, const double*, const otf_sinkhorn_opts&,
                                               void*, double*, double*, void*, int64_t, int,
                                               otf_sinkhorn_info*, double*, hipStream_t);

}  // namespace otf
