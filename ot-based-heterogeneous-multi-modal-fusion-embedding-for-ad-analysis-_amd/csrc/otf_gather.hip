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
// 16: {value word, tag} 8-byte granules for float, two tagged doubles per chunk for
// double -- see make_chunk -- one 16-B store per two columns) and every workgroup GATHERS all the
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
// tag = ((k + 1) << 1) | bad (double: epoch mod 4 and bad in the values' low bits).  A slot is rewritten two epochs later, which no producer
// can reach before every consumer has finished reading it (producing S[k + 2] needs
// S[k + 1], which each workgroup publishes only after its gather of S[k]).  Every poll
// is bounded by s_memrealtime (re-armed after each completed gather): a stall ends in
// OTF_SK_TIMEOUT.
#include "otf_persist.h"

namespace otf {
namespace {

// rows per wave of a float64 tile (A/B build switch; 8: 64-row tiles, 4: 32-row tiles)
#ifndef OTF_GATHER_RW64
#define OTF_GATHER_RW64 8
#endif
template <typename T> struct GatherCfg {
    static constexpr int NW = 8;                        // waves per workgroup
    static constexpr int RW = sizeof(T) == 4 ? 16 : OTF_GATHER_RW64;  // rows per wave
    static constexpr int VEC = Vec<T>::N;
    static constexpr int G = sizeof(T) == 4 ? 2 : 4;    // VEC-vectors per lane: 8 columns
    static constexpr int TR = RW * NW;                  // rows per workgroup: 128 / 64
    static constexpr int C = kWave * G * VEC;           // 512 columns
    static constexpr int CPC = 2;                       // columns per 16-B chunk
    static constexpr int NCH = C / CPC;                 // chunks per producer row
};
constexpr int kGatherMaxWG = 16;
constexpr uint32_t kGatherRow = 8192;  // bytes per producer row of one slot (256 chunks used)

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

// A 16-B chunk carries two column partials with their epoch tag.  float: two
// {value, tag} granules, tag = (epoch << 1) | bad.  double: two values whose three low
// mantissa bits ARE the tag -- epoch mod 4 (a slot holds epoch e - 2 or e, or the zero
// fill before epochs 1 and 2, so two bits tell them apart) and the bad flag -- so a chunk
// holds two columns instead of one and a gather moves half the bytes (the one-hop gather
// is bound by the CU's 64 B/clk port: nwg x 8 KB per workgroup per iteration).  The
// value is truncated to a 49-bit mantissa (relative 2^-50, below the float64 rounding
// of the sums that follow); 0 and infinities come back exact once the tag is cleared.
template <typename T> __device__ __forceinline__ void chunk_values(const I4 x, T (&v)[GatherCfg<T>::CPC]) {
    if constexpr (sizeof(T) == 8) {
        v[0] = __builtin_bit_cast(double, ((unsigned long long)(unsigned)x[1] << 32) | ((unsigned)x[0] & ~7u));
        v[1] = __builtin_bit_cast(double, ((unsigned long long)(unsigned)x[3] << 32) | ((unsigned)x[2] & ~7u));
    } else {
        // element copies first: __builtin_bit_cast of a vector ELEMENT reads the vector's
        // first word (ROCm 7.2 clang; found by the float parity test)
        const int w0 = x[0], w2 = x[2];
        v[0] = __builtin_bit_cast(float, w0);
        v[1] = __builtin_bit_cast(float, w2);
    }
}
template <typename T> __device__ __forceinline__ I4 make_chunk(const T (&v)[GatherCfg<T>::CPC], int ep, int bad) {
    I4 x;
    if constexpr (sizeof(T) == 8) {
        const unsigned low = (unsigned)(ep & 3) | ((unsigned)bad << 2);
        const unsigned long long b0 = __builtin_bit_cast(unsigned long long, v[0]);
        const unsigned long long b1 = __builtin_bit_cast(unsigned long long, v[1]);
        x[0] = (int)(((unsigned)b0 & ~7u) | low);
        x[1] = (int)(unsigned)(b0 >> 32);
        x[2] = (int)(((unsigned)b1 & ~7u) | low);
        x[3] = (int)(unsigned)(b1 >> 32);
    } else {
        const int tag = (ep << 1) | bad;
        x[0] = __builtin_bit_cast(int, v[0]);
        x[2] = __builtin_bit_cast(int, v[1]);
        x[1] = tag;
        x[3] = tag;
    }
    return x;
}
template <typename T> __device__ __forceinline__ bool chunk_at_ep(const I4 x, unsigned ep) {
    if constexpr (sizeof(T) == 8)
        return (((unsigned)x[0] & 3u) == (ep & 3u)) && (((unsigned)x[2] & 3u) == (ep & 3u));
    else
        return ((unsigned)x[1] >> 1) == ep && ((unsigned)x[3] >> 1) == ep;
}
template <typename T> __device__ __forceinline__ int chunk_bad(const I4 x) {
    if constexpr (sizeof(T) == 8)
        return (((unsigned)x[0] | (unsigned)x[2]) >> 2) & 1;
    else
        return x[1] & 1;
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
                // wait until this XCC's team is complete or another team has claimed.
                // The claim word takes exactly one value: a team (xcd + 1), or -1 when a
                // registrant whose deadline passed gave the launch up -- both by a
                // compare-and-swap from 0, so a solve is never both claimed and abandoned
                for (;;) {
                    int claim = load_agent(p.team + 8 * 64);
                    if (claim != 0) {
                        keep = claim == xcd + 1;  // -1: abandoned
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
                        // no XCC team claimed the solve in time (a slot already left, or
                        // another persistent grid holds the CUs): abandon it for the
                        // one-workgroup fallback, or the untouched u / v / plan would read
                        // as a finished solve -- unless a team claimed it meanwhile
                        int expected = 0;
                        if (__hip_atomic_compare_exchange_strong(p.team + 8 * 64, &expected, -1,
                                                                 __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_AGENT)) {
                            keep = 0;
                            mark_stalled(&p.info->stalled, kStallRegistration);
                            break;
                        }
                        continue;  // claimed: the next pass reads the owner
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
    constexpr int RSH = R == 16 ? 2 : R == 8 ? 3 : 4;
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
                __builtin_amdgcn_raw_buffer_store_b128(make_chunk<T>(val, k + 1, bad), rs, off, 0, 0);
            else
                __builtin_amdgcn_raw_buffer_store_b128(make_chunk<T>(val, k + 1, bad), rs, off, 0,
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
                    ok &= chunk_at_ep<T>(x[q], ep);
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
                    fl |= chunk_bad<T>(x[q]);
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
    if (status == OTF_SK_TIMEOUT && tid == 0) mark_stalled(&p.info->stalled, kStallMid);
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
    constexpr int S2 = 512 / GatherCfg<T>::TR;  // config 2's 512 rows in whole tiles
    const void* k = (sizeof(T) == 8 && NQ == S2 && p.nwg == S2 && whole)
                        ? (const void*)sk_gather_kernel<T, CT, TP, NQ, (sizeof(T) == 8 && NQ == S2) ? S2 : 0>
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

}  // namespace

template <typename T> bool gather_supported(int64_t n, int64_t m) {
    return n >= 1 && m >= 1 && m <= GatherCfg<T>::C && gather_grid<T>(n) <= kGatherMaxWG;
}

constexpr size_t kTeamBytes = 9 * 256;  // 8 XCC registration counters + the claim word

template <typename T> size_t gather_region_bytes(int64_t n, int64_t m) {
    return gather_supported<T>(n, m) ? kTeamBytes + 2 * (size_t)gather_grid<T>(n) * kGatherRow : 0;
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
                      double* errlog, bool zeroed, hipStream_t s) {
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
    if (!zeroed) {  // else the Sinkhorn init kernel zeroed it (no memset launch)
        const hipError_t e = hipMemsetAsync(region, 0, gather_region_bytes<T>(n, m), s);
        if (e != hipSuccess) return e;
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
                                             bool, hipStream_t);
template hipError_t run_gather<float, _Float16>(const _Float16*, int64_t, int, int, const float*,
                                                const float*, const float*, const otf_sinkhorn_opts&,
                                                void*, float*, float*, void*, int64_t, int,
                                                otf_sinkhorn_info*, double*, bool, hipStream_t);
template hipError_t run_gather<double, double>(const double*, int64_t, int, int, const double*,
                                               const double*, const double*, const otf_sinkhorn_opts&,
                                               void*, double*, double*, void*, int64_t, int,
                                               otf_sinkhorn_info*, double*, bool, hipStream_t);

}  // namespace otf
