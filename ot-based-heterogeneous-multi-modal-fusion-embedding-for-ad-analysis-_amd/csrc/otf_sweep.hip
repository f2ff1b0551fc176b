// otf_sweep.hip — persistent streaming Sinkhorn (OTF_ENGINE_SWEEP), POT flavour.
//
// Replaces ot.sinkhorn (POT 0.9.6 sinkhorn_knopp) at MRI_PET_OT_nojax.py:143 /
// perturbot/perturbot/match/utils.py:6-115 for costs too large to stay in the register
// files of the chip (BASELINE config 5: N = 8192 fp16, and past the Infinity Cache:
// N = 16384 fp32).  The whole solve is ONE launch; every iteration streams the
// materialised cost once.
//
// Grid: one 512-thread workgroup per CU.  Workgroup w owns row blocks w, w + grid, ...
// (R rows x all m columns); thread t owns G chunks of 16 bytes of every row (columns
// (t + 512 g) * VEC .. + VEC, coalesced 16-B loads).  Per iteration it:
//   1. reads K^T u(it-1) (the column sums of the previous sweep: NREP replicas of a
//      ring slot, 16-B sc1 loads) and forms v(it) = b / (K^T u) for its columns, taking
//      POT's decisions exactly like the resident engines (every workgroup derives the
//      same decision from the same sums, in a fixed reduction order);
//   2. sweeps its row blocks, the next block's cost rows in flight (two register
//      buffers, ping-pong) while the current one is reduced: e = exp(-C/reg) once per
//      element, row sums K v (wave butterfly + one LDS exchange per block, fixed order)
//      -> u = 1 / (K/a v) for those rows, then the column partials K^T u with the new u
//      in registers;
//   3. adds its m column partials into the next ring slot (memory-side float atomics,
//      staged through LDS so every wave-instruction covers 256 contiguous bytes; the
//      slot's replica is picked by the XCD), zeroes its share of the slot after next
//      (write-through), and meets the grid at the XCD-hierarchical barrier.
// The first block of the next sweep is put in flight before the barrier, so the
// barrier and the atomic drain overlap the stream.  The plan is written at the end
// from the last good (u, v) by a final sweep.
//
// Granule flush (float problems outside the deterministic mode, r03): step 3 above
// without atomics, zeroing or barriers -- every hand-off is an epoch-tagged granule
// (otf_persist.h) that the consumer polls:
//   a. every workgroup stores its m partials into its slab row (plain stores: only its
//      XCC reads them);
//   b. the XCC's workgroups, ranked by blockIdx, own the 32 column slices round-robin:
//      the owner of a slice sums it over the XCC members' rows in rank order and
//      publishes the XCC partial (write-through, parity double-buffered);
//   c. the same owner sums the slice over the active XCCs' partials in XCC order and
//      stores S into its XCC's ring slot (plain): every XCC derives the same S, bit for
//      bit, from the same partials in the same order;
//   d. the next sweep's v-update polls the XCC-local S granules.
// Across GPUs (otf_sinkhorn_xsweep: one problem's rows sharded over <= 8 ranks of one
// node, BASELINE config 5's multi-GPU form): step c sums the XCC partials into this
// rank's partial of the slice, which the first active XCC's owner stores into EVERY
// rank's exchange buffer (system-scope write-through over xGMI, parity double-buffered
// like the XCC partials); step c' then sums the slice over the world's rank partials in
// rank order -- every rank derives the same S, bit for bit -- into the XCC-local ring.
// POT's decisions follow from S alone, so every rank takes them at the same iteration.
// Epochs of an exchange continue across solves (ep_base, advanced by the host in
// lock-step on every rank), so no rank ever needs to clear a peer's buffer.
// A non-finite u travels as a tag flag (slab -> XCC partial -> S) instead of the bad
// counters.  Three hops, one of them across XCCs, instead of flush + group counter +
// atomics + grid barrier (~11 us of a 29-us config-5 sweep in r02).
//
// Ring of 4 sum slots S[k] = K^T u(k-1) (slot k % 4): iteration it reads S[it] and, on
// check iterations, S[it-1]; accumulates S[it+1]; zeroes slot (it+2) % 4 (= S[it-2],
// last read in iteration it-1).  Exits keep S[it-2..it] intact, so the outputs can be
// recomputed bit-identically from v(k) = b / S[k].  Memory is O(m), not O(max_iter m).
#include "otf_persist.h"


namespace otf {
namespace {

constexpr int kSwNT = 512;        // threads per workgroup (8 waves, one workgroup per CU)
constexpr int kSwRowMax = 1024;   // rows per workgroup kept in the LDS u history

template <typename T> struct SkSweepArgs {
    const void* C;
    int64_t ldc;
    int n, m, m_pad;
    const T* a;
    const T* b;
    const T* cost_scale;
    double reg;
    int max_iter, check_every, err_squared;
    double stop_thr;
    T* ring;            // 4 slots x slot_stride
    int64_t slot_stride;
    int* bad;           // 4 counters of non-finite u rows, one 256-B line each
    int* bar;
    SkSync sync;
    int* gcnt;          // per-XCD group arrival counters, one 256-B line each
    T* slab;            // grid x m_pad column partials (write-through), one row per workgroup
    otf_sinkhorn_info* info;
    double* errlog;
    T* u_out;
    T* v_out;
    void* P;
    int64_t ldp;
    unsigned long long stall_ticks;
    unsigned long long reg_ticks;  // the first wait (registration / first hop)
    int nt_loads;       // 1: cost larger than the Infinity Cache, stream it non-temporal
    int det;            // 1: fixed-order column sums (one group = the whole grid, no atomics)
    int nres;           // row blocks per workgroup kept in LDS (< the fewest blocks any has)
    int gran;           // 1: granule flush (float, not deterministic mode)
    unsigned char* gslab;  // [grid][m_pad] granules: column partials per workgroup
    unsigned char* gxp;    // [2 parity][8 XCC][m_pad] granules: XCC partials (sc1)
    unsigned char* gfs;    // [8 XCC][4 ring][m_pad] floats: S, read within the XCC, then
                           // [8 XCC][4 ring][32 slices] ready words: (epoch << 2) | flags
    int* xl;               // [8][256] registration lists: blockIdx per XCC slot
    // cross-rank exchange (world > 1): xr[r] = rank r's exchange buffer as mapped here,
    // [2 parity][8 ranks][m_pad] granules
    int rank, world;
    int n_total;           // rows over all ranks (POT's u0 = 1 / n)
    unsigned ep_base;      // epoch offset of this solve (the same on every rank)
    int solve_par;         // the exchange's slot set for this solve (XSweep::solve_par)
    unsigned char* xr[8];
    ShiftArgs sh;          // shifted kernel (SH instances): offsets + initial scalings
    T* kbuf;               // KS instances: K = exp(-C / reg) written by the prologue sweep,
                           // n rows x m_pad, streamed by every later sweep instead of C
};
constexpr int kSwSlices = 32;  // column slices of the granule reduction

// Slab granules (r06): FOUR float32 column partials per 16-B chunk, the tag folded into
// each value's three low mantissa bits -- bits 0..1 = (epoch mod 3) + 1 (never 0, so the
// zero fill never matches), bit 2 = the non-finite-u flag -- instead of chunk2's {value,
// tag} pairs: half the slab bytes per sweep.  A slab row is single-buffered, so a slice
// owner waiting for epoch e finds e - 1 or e there (a member writes e + 1 only after S[e],
// which needs this owner's slice), and epoch mod 3 tells them apart.  The value is
// ROUNDED to a 21-bit mantissa (relative 2^-21 on one workgroup's partial, unbiased:
// truncation's one-sided 2^-20 lifted the converged marginal-error floor of a
// 400-iteration xsweep to 1.1e-8 against 1e-8 for the float32 sums); 0 and +-inf come
// back exact once the bits are cleared.
using F4v = __attribute__((ext_vector_type(4))) float;
__device__ __forceinline__ unsigned qtag(unsigned e) { return e % 3u + 1u; }
__device__ __forceinline__ I4 chunk4(float v0, float v1, float v2, float v3, unsigned tag, int flag) {
    const unsigned low = tag | ((unsigned)flag << 2);
    // round half away from zero at bit 3 (a carry into the exponent is the correct
    // rounding; +-inf stays +-inf)
    auto rnd = [&](float v) -> int { return (int)(((__builtin_bit_cast(unsigned, v) + 4u) & ~7u) | low); };
    I4 x;
    x[0] = rnd(v0);
    x[1] = rnd(v1);
    x[2] = rnd(v2);
    x[3] = rnd(v3);
    return x;
}
__device__ __forceinline__ bool chunk4_at(const I4 x, unsigned tag) {
    return (((unsigned)x[0] & 3u) == tag) && (((unsigned)x[1] & 3u) == tag) && (((unsigned)x[2] & 3u) == tag) &&
           (((unsigned)x[3] & 3u) == tag);
}
// element copies first (ROCm 7.2: a bit_cast of a vector ELEMENT reads element 0)
__device__ __forceinline__ float chunk4_v(const I4 x, int i) {
    const unsigned w = (unsigned)x[i] & ~7u;
    return __builtin_bit_cast(float, w);
}
__device__ __forceinline__ int chunk4_flag(const I4 x) {
    return (int)((((unsigned)x[0] | (unsigned)x[1] | (unsigned)x[2] | (unsigned)x[3]) >> 2) & 1u);
}

using Raw = __attribute__((ext_vector_type(4))) unsigned int;  // 16 B of cost

template <typename CT> struct RawN {
    static constexpr int N = 16 / sizeof(CT);
};

// 16 B of cost -> compute type
template <typename T, typename CT>
__device__ __forceinline__ void widen(const Raw& r, T (&out)[RawN<CT>::N]) {
    if constexpr (sizeof(CT) == 2) {
        using H = __attribute__((ext_vector_type(8))) _Float16;
        const H h = __builtin_bit_cast(H, r);
#pragma unroll
        for (int k = 0; k < 8; ++k) out[k] = (T)h[k];
    } else if constexpr (sizeof(CT) == 4) {
        using F = __attribute__((ext_vector_type(4))) float;
        const F f = __builtin_bit_cast(F, r);
#pragma unroll
        for (int k = 0; k < 4; ++k) out[k] = (T)f[k];
    } else {
        using D = __attribute__((ext_vector_type(2))) double;
        const D d = __builtin_bit_cast(D, r);
#pragma unroll
        for (int k = 0; k < 2; ++k) out[k] = (T)d[k];
    }
}

// 16 B of cost -> pairs of (cost x ks) in the compute type.  fp16 x f32 in one
// v_fma_mix_f32 per element (the fp16 -> f32 conversion is exact, so this rounds once,
// exactly like convert-then-multiply), f32 pairs by one v_pk_mul_f32.
template <typename T> using Pair = __attribute__((ext_vector_type(2))) T;
template <typename T, typename CT>
__device__ __forceinline__ void scaled_pairs(const Raw& r, T ks, Pair<T> (&out)[RawN<CT>::N / 2]) {
    if constexpr (sizeof(CT) == 2 && sizeof(T) == 4) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float lo, hi;
            asm("v_fma_mix_f32 %0, %1, %2, 0 op_sel_hi:[1,0,0]" : "=v"(lo) : "v"(r[q]), "v"(ks));
            asm("v_fma_mix_f32 %0, %1, %2, 0 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(hi) : "v"(r[q]), "v"(ks));
            out[q] = Pair<T>{lo, hi};
        }
    } else {
        T c[RawN<CT>::N];
        widen<T, CT>(r, c);
#pragma unroll
        for (int j = 0; j < RawN<CT>::N / 2; ++j) out[j] = Pair<T>{c[2 * j], c[2 * j + 1]} * ks;
    }
}

// value of lane r (uniform result)
__device__ __forceinline__ float bcast_lane(float x, int r) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), r));
}
__device__ __forceinline__ double bcast_lane(double x, int r) {
    const long long b = __builtin_bit_cast(long long, x);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), r);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), r);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}


// SH (float only): the shifted POT kernel e = 2^(C ks + A_i + B_j) (otf_persist.h
// ShiftArgs); B of the columns and A of the workgroup's rows sit in LDS beside 1 / a.
// KS (float64 only): POT's own form -- K = exp(-M / reg) materialised once (ot.bregman
// sinkhorn_knopp, perturbot/perturbot/match/utils.py:46) -- the prologue sweep writes the
// K of the workgroup's row blocks to p.kbuf and every later sweep (and the plan) streams
// K instead of recomputing a float64 exp per element per sweep: the float64 exp (~20 FMA
// -class instructions) was the largest cost of a float64 sweep.  Same exp, same values:
// the same iterates bit for bit.
template <typename T, typename CT, typename TP, int G, int R, int NREP, bool SH, bool KS = false>
__global__ __launch_bounds__(kSwNT) void sk_sweep_kernel(SkSweepArgs<T> p) {
    constexpr int VC = RawN<CT>::N;            // cost elements per 16-B chunk
    constexpr int VT = Vec<T>::N;              // compute elements per 16-B sum load
    constexpr int NW = kSwNT / kWave;
    static_assert((VC % VT) == 0, "chunk covers whole sum vectors");
    using V = typename Vec<T>::type;
    extern __shared__ __attribute__((aligned(16))) unsigned char sw_lds[];
    // vbuf: v of this iteration for the thread's own columns (only the owning thread
    // reads it back), then reused to stage the column partials for the atomics
    T* vbuf = reinterpret_cast<T*>(sw_lds);                         // m_pad
    T* uhist = vbuf + p.m_pad;                                       // [2][kSwRowMax]
    T* ialds = uhist + 2 * kSwRowMax;                                // 1 / a of own rows
    T* gred = ialds + kSwRowMax;                                     // [kSwNT * VT] group reduce
    // the workgroup's last nres row blocks (sanitized raw cost, thread-private 16-B slots):
    // read from LDS instead of the memory system on every sweep after the prologue
    T* shBl = gred + kSwNT * VT;                                     // SH: B, m_pad
    T* shAl = shBl + (SH ? p.m_pad : 0);                             // SH: A of own rows
    Raw* resb = reinterpret_cast<Raw*>(shAl + (SH ? kSwRowMax : 0));
    __shared__ T red[2][NW][R];
    __shared__ T ered[17];
    __shared__ int s_flag;
    __shared__ int s_pop[6];
    __shared__ int mrow[256];     // granule flush: this XCC's members by blockIdx rank
    __shared__ int s_or[6][NW];  // [0..1] v-update checks, [2..3] flushes, [4..5] S slices
    __shared__ int s_fq[NW];     // granule flush stage b: the waves' slab flags
    const bool gran = sizeof(T) == 4 && p.gran;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int nwg = gridDim.x;
    const bool lead = (blockIdx.x == 0 && tid == 0);
    unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + p.reg_ticks;

    const double unit = exp_unit<T>();
    double cinv = 1.0;
    if (p.cost_scale) cinv = 1.0 / (double)p.cost_scale[0];
    const T ks = (T)(-unit / p.reg * cinv);

    // ---- column ownership: chunk g starts at column (tid + 512 g) * VC; cnt[g] of its
    // VC columns are inside the problem (loads of chunks past m are clamped to 0)
    int colc[G], cnt[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int c0 = (tid + kSwNT * g) * VC;
        colc[g] = c0 < p.m ? c0 : 0;
        const int left = p.m - c0;
        cnt[g] = left <= 0 ? 0 : (left < VC ? left : VC);
    }
    // a chunk that straddles column m: its bytes past m (row padding, any value) are
    // zeroed on load, so every e is finite; v = 0 there keeps them out of the row sums
    // and their column partials are never flushed.  A chunk wholly past m re-reads
    // column 0 (finite) with weight 0.  Rows past n read as 0 (buffer bounds) and get
    // u = 0.
    const bool ragged = (p.m % VC) != 0;
    Raw keep = {~0u, ~0u, ~0u, ~0u};
    int gk = -1;
#pragma unroll
    for (int g = 0; g < G; ++g)
        if (cnt[g] > 0 && cnt[g] < VC) {
            gk = g;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                // dword q holds elements [q * 4 / sizeof(CT), (q + 1) * 4 / sizeof(CT))
                unsigned msk = 0;
                constexpr int per = sizeof(CT) >= 4 ? 1 : 4 / (int)sizeof(CT);
                for (int s = 0; s < per; ++s) {
                    const int el = sizeof(CT) == 8 ? q / 2 : q * per + s;
                    if (el < cnt[g]) msk |= sizeof(CT) >= 4 ? ~0u : (0xffffu << (16 * s));
                }
                keep[q] = msk;
            }
        }
    const int nrb = (p.n + R - 1) / R;
    const int my_nb = nrb > (int)blockIdx.x ? (nrb - 1 - (int)blockIdx.x) / nwg + 1 : 0;
    const int res0 = my_nb - p.nres;  // first LDS-resident block (nres < every my_nb)
    const int64_t ld_bytes = p.ldc * (int64_t)sizeof(CT);
    static_assert(!KS || (sizeof(T) == 8 && sizeof(CT) == 8 && !SH), "K stream: float64 only");
    const int64_t ldk_bytes = (int64_t)p.m_pad * (int64_t)sizeof(T);
    for (int i = tid; i < my_nb * R; i += kSwNT) {
        const int row = ((int)blockIdx.x + (i / R) * nwg) * R + i % R;
        ialds[i] = (T)1 / p.a[row < p.n ? row : 0];
        if (SH) shAl[i] = row < p.n ? (T)p.sh.A[row] : (T)0;
    }
    if (SH)
        for (int j = tid; j < p.m_pad; j += kSwNT) shBl[j] = (T)p.sh.B[j];  // zero past m
    if (SH) __syncthreads();

    // R cost rows of block bi via one SGPR descriptor (rows past n read as 0).  A cost
    // larger than the Infinity Cache is loaded non-temporal (7.3 vs 6.4 TB/s from HBM,
    // tools/ubench_mall.hip; N = 16384 fp32: 195 -> 184 us per sweep); a cost that fits
    // keeps the default policy (nt measured 26.2 vs 22.3 us per config-5 sweep).
    // fromK (KS): the block of K from p.kbuf (written by this workgroup's prologue sweep)
    auto load_block = [&](int bi, Raw (&buf)[R][G], bool fromK = false) {
        const int r0 = ((int)blockIdx.x + bi * nwg) * R;
        const int nrow = p.n - r0 < R ? p.n - r0 : R;
        if (KS && fromK) {
            const __amdgpu_buffer_rsrc_t kr = __builtin_amdgcn_make_buffer_rsrc(
                (void*)((char*)p.kbuf + (int64_t)r0 * ldk_bytes), 0, (int)(nrow * ldk_bytes), 0x00020000);
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int g = 0; g < G; ++g)
                    buf[r][g] = __builtin_amdgcn_raw_buffer_load_b128(
                        kr, (uint32_t)(colc[g] * (int)sizeof(T)), (uint32_t)(r * ldk_bytes), 0);
            return;
        }
        const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc(
            (void*)((const char*)p.C + (int64_t)r0 * ld_bytes), 0, (int)(nrow * ld_bytes), 0x00020000);
        if (p.nt_loads) {
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int g = 0; g < G; ++g)
                    buf[r][g] = __builtin_amdgcn_raw_buffer_load_b128(
                        cr, (uint32_t)(colc[g] * (int)sizeof(CT)), (uint32_t)(r * ld_bytes), 2 /* nt */);
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int g = 0; g < G; ++g)
                    buf[r][g] = __builtin_amdgcn_raw_buffer_load_b128(
                        cr, (uint32_t)(colc[g] * (int)sizeof(CT)), (uint32_t)(r * ld_bytes), 0);
        }
    };
    auto sanitize = [&](Raw (&buf)[R][G]) {
        if (ragged) {
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int g = 0; g < G; ++g)
                    if (g == gk) buf[r][g] &= keep;
        }
    };

    const __amdgpu_buffer_rsrc_t rs = sums_rsrc(p.ring);
    // sums of slot k for chunk g (VC columns): all replicas summed in a fixed order
    auto load_sums_chunk = [&](int k, int g, T (&out)[VC]) {
        const uint32_t boff = (uint32_t)((size_t)(k & 3) * p.slot_stride * sizeof(T));
        V acc[VC / VT];
#pragma unroll
        for (int h = 0; h < VC / VT; ++h)
            acc[h] = load_sum_vec<T>(rs, boff + (uint32_t)((colc[g] + h * VT) * sizeof(T)));
#pragma unroll
        for (int q = 1; q < NREP; ++q)
#pragma unroll
            for (int h = 0; h < VC / VT; ++h) {
                const V t = load_sum_vec<T>(
                    rs, boff + (uint32_t)(((size_t)q * p.m_pad + colc[g] + h * VT) * sizeof(T)));
#pragma unroll
                for (int k2 = 0; k2 < VT; ++k2) acc[h][k2] += t[k2];
            }
#pragma unroll
        for (int k2 = 0; k2 < VC; ++k2) out[k2] = acc[k2 / VT][k2 % VT];
    };
    // granule form: S[k] of chunk g from this XCC's ring slot, polled until its tags carry
    // epoch k + 1; flags of every granule ORed into fl, a stall clears ok
    const int mc = p.m_pad / 2;                       // 16-B granule pairs per row
    auto load_sums_gran = [&](int k, int g, T (&out)[VC], int& fl, bool& ok) {
        // S[k] of chunk g: poll the ready word of its slice (one dword), then read the
        // VC sums (plain floats: half the bytes of tagged granules)
        const __amdgpu_buffer_rsrc_t rfs = sums_rsrc(p.gfs);
        const unsigned e = (p.ep_base + (unsigned)(k + 1)) & 0x3fffffffu;
        const int swc = 2 * ((p.m_pad / 4 + kSwSlices - 1) / kSwSlices);  // pairs per slice (flush_gran)
        const int slot = xcc_id() * 4 + (int)(e & 3);
        const uint32_t fo = (uint32_t)(32 * p.m_pad) * 4u + (uint32_t)(slot * kSwSlices + (colc[g] / 2) / swc) * 4u;
        int fw = __builtin_amdgcn_raw_buffer_load_b32(rfs, fo, 0, 16 /* sc1 */);
        while (((unsigned)fw >> 2) != e && ok) {
            __builtin_amdgcn_s_sleep(1);
            fw = __builtin_amdgcn_raw_buffer_load_b32(rfs, fo, 0, 16 /* sc1 */);
            if (((unsigned)fw >> 2) != e && __builtin_amdgcn_s_memrealtime() > deadline) ok = false;
        }
        fl |= fw & 3;
        const uint32_t base = (uint32_t)(slot * p.m_pad + colc[g]) * 4u;
#pragma unroll
        for (int h = 0; h < VC / 4; ++h) {
            using F4 = __attribute__((ext_vector_type(4))) float;
            const F4 v4 = __builtin_bit_cast(F4, __builtin_amdgcn_raw_buffer_load_b128(rfs, base + h * 16, 0, 16 /* sc1 */));
            out[4 * h] = (T)v4[0];
            out[4 * h + 1] = (T)v4[1];
            out[4 * h + 2] = (T)v4[2];
            out[4 * h + 3] = (T)v4[3];
        }
    };
    // OR of 3 flag bits over the workgroup (ballots + one barrier; par alternates)
    auto block_or = [&](int bits, int par) -> int {
        int wv = 0;
#pragma unroll
        for (int b = 0; b < 3; ++b)
            if (__ballot((bits >> b) & 1)) wv |= 1 << b;
        if (lane == 0) s_or[par][w] = wv;
        __syncthreads();
        int r = 0;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) r |= s_or[par][ww];
        return r;
    };
    auto load_b_chunk = [&](int g, T (&bv)[VC]) {
#pragma unroll
        for (int h = 0; h < VC / VT; ++h) {
            const V t = *reinterpret_cast<const V*>(p.b + colc[g] + h * VT);
#pragma unroll
            for (int k2 = 0; k2 < VT; ++k2) bv[h * VT + k2] = t[k2];
        }
    };
    // L2 marginal error of iterate k: v(k) = b / S[k] against S[k+1] (all workgroups
    // compute the same value: same data, same fixed-order block reduction)
    auto marginal_err = [&](int k) -> double {
        T e = 0;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            T sk[VC], sk1[VC], bv[VC];
            if (gran) {
                int fl = 0;
                bool ok = true;
                load_sums_gran(k, g, sk, fl, ok);
                load_sums_gran(k + 1, g, sk1, fl, ok);
            } else {
                load_sums_chunk(k, g, sk);
                load_sums_chunk(k + 1, g, sk1);
            }
            load_b_chunk(g, bv);
#pragma unroll
            for (int k2 = 0; k2 < VC; ++k2) {
                const bool ok = k2 < cnt[g];
                const T vb = bv[k2] / (ok ? sk[k2] : (T)1);
                const T rr = vb * sk1[k2] - bv[k2];
                e += ok ? rr * rr : (T)0;
            }
        }
        e = block_sum<T>(e, ered);
        return p.err_squared ? (double)e : sqrt((double)e);
    };

    const T u0 = (T)1 / (T)(p.n_total > 0 ? p.n_total : p.n);
    const int xcd = xcc_id();
#ifdef OTF_STAMPS
    if (tid == 0 && blockIdx.x < 256) g_stamps[(blockIdx.x * 16 + 15) * 8 + 7] = (unsigned long long)xcd;
#endif
    Raw bufA[R][G];
    // column partials as pairs of adjacent columns: the e * u products go out as packed
    // FMAs (v_pk_fma_f32), as do the e * v row-sum products
    using T2 = Pair<T>;
    constexpr int VP2 = VC / 2;
    T2 colacc[G][VP2];

    // One sweep over this workgroup's row blocks.  it = -1: the prologue (u = u0, no
    // row sums).  bufA holds block 0's cost on entry (already in flight).
    int badu = 0;
    auto sweep = [&](int it) {
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int k = 0; k < VP2; ++k) colacc[g][k] = T2{0, 0};
        auto process = [&](int bi, Raw (&buf)[R][G], int next) {
            const int r0 = ((int)blockIdx.x + bi * nwg) * R;
            const int nrow = p.n - r0 < R ? p.n - r0 : R;
            T2 e[R][G][VP2];
            if (KS && it >= 0) {
                // the block holds K (from p.kbuf or the LDS-resident copy)
#pragma unroll
                for (int g = 0; g < G; ++g)
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        T kk[VC];
                        widen<T, CT>(buf[r][g], kk);
#pragma unroll
                        for (int k = 0; k < VP2; ++k) e[r][g][k] = T2{kk[2 * k], kk[2 * k + 1]};
                    }
            } else {
            sanitize(buf);
            if (!KS && it < 0 && bi >= res0) {  // prologue: keep this block in LDS
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int g = 0; g < G; ++g) resb[(((bi - res0) * R + r) * G + g) * kSwNT + tid] = buf[r][g];
            }
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    T2 c[VP2];
                    scaled_pairs<T, CT>(buf[r][g], ks, c);
                    if constexpr (SH) {
                        const T sa = shAl[bi * R + r];
#pragma unroll
                        for (int k = 0; k < VP2; ++k)
                            c[k] += T2{sa, sa} + *reinterpret_cast<const T2*>(shBl + colc[g] + 2 * k);
                    }
#pragma unroll
                    for (int k = 0; k < VP2; ++k) {
#if defined(OTF_SWEEP_ABLATE) && (OTF_SWEEP_ABLATE & 1)
                        e[r][g][k] = c[k];  // diagnostic: no exponentials
#else
                        e[r][g][k] = T2{fast_exp(c[k].x), fast_exp(c[k].y)};
#endif
                    }
                }
            if constexpr (KS) {
                // prologue: K of this block to p.kbuf (rows < n, chunks inside m) and to LDS
                // when the block is LDS-resident
                char* krow = (char*)p.kbuf + (int64_t)r0 * ldk_bytes;
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int g = 0; g < G; ++g) {
                        T kk[VC];
#pragma unroll
                        for (int k = 0; k < VP2; ++k) {
                            kk[2 * k] = e[r][g][k].x;
                            kk[2 * k + 1] = e[r][g][k].y;
                        }
                        Raw kr2;
                        static_assert(sizeof(kk) == sizeof(Raw), "one 16-B chunk");
                        __builtin_memcpy(&kr2, kk, sizeof(Raw));
                        if (r < nrow && cnt[g] > 0)
                            *reinterpret_cast<Raw*>(krow + r * ldk_bytes + colc[g] * (int)sizeof(T)) = kr2;
                        if (bi >= res0) resb[(((bi - res0) * R + r) * G + g) * kSwNT + tid] = kr2;
                    }
            }
            }
            // single-buffer pipeline: the raw block is dead once widened, so the next
            // block's loads go out now and fly during this block's reductions
            // LDS-resident blocks come from LDS once the prologue sweep has put them there
#if defined(OTF_SWEEP_ABLATE) && (OTF_SWEEP_ABLATE & 2)
            if (it >= 0) {  // diagnostic: after the prologue, no cost loads (stale block)
            } else
#endif
            if (it >= 0 && next >= res0) {
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int g = 0; g < G; ++g) buf[r][g] = resb[(((next - res0) * R + r) * G + g) * kSwNT + tid];
            } else if (KS && (it >= 0 || bi + 1 >= my_nb)) {
                // K: every sweep after the prologue, and the prologue's look-ahead of the
                // first sweep's block 0 (stored by this thread earlier in this sweep)
                if (it < 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                load_block(next, buf, true);
            } else {
                load_block(next, buf);
            }
            T rp[R];
#pragma unroll
            for (int r = 0; r < R; ++r) rp[r] = 0;
            if (it >= 0) {
                T2 rp2[R];
#pragma unroll
                for (int r = 0; r < R; ++r) rp2[r] = T2{0, 0};
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    T2 vv[VP2];
                    // a chunk past m re-reads column 0's cost: weight it 0
                    const bool live = cnt[g] > 0;
#pragma unroll
                    for (int h = 0; h < VC / VT; ++h) {
                        const V t = *reinterpret_cast<const V*>(vbuf + colc[g] + h * VT);
#pragma unroll
                        for (int k2 = 0; k2 < VT; k2 += 2)
                            vv[(h * VT + k2) / 2] = live ? T2{t[k2], t[k2 + 1]} : T2{0, 0};
                    }
#pragma unroll
                    for (int r = 0; r < R; ++r)
#pragma unroll
                        for (int k = 0; k < VP2; ++k) rp2[r] = e[r][g][k] * vv[k] + rp2[r];
                }
#pragma unroll
                for (int r = 0; r < R; ++r) rp[r] = rp2[r].x + rp2[r].y;
            }
            T u[R];
            if (it >= 0) {
                // wave totals -> LDS; every wave then finishes the R row sums on lanes
                // 0..R-1 (same fixed order everywhere) and broadcasts u by readlane
                wave_sum_multi<T, R>(rp, lane);
                const int par = bi & 1;
                if (lane < R) red[par][w][butterfly_row<R>(lane)] = rp[0];
#if !(defined(OTF_SWEEP_ABLATE) && (OTF_SWEEP_ABLATE & 4))
                __syncthreads();  // (ABLATE & 4, diagnostic: no per-block barrier, racy sums)
#endif
                const int rr = lane < R ? lane : 0;
                T s = red[par][0][rr];
#pragma unroll
                for (int ww = 1; ww < NW; ++ww) s += red[par][ww][rr];
                const T un = (T)1 / (s * ialds[bi * R + rr]);  // POT: u = 1 / (K/a v)
                const bool rok = rr < nrow;
                badu |= (lane < R && rok && !finite_val(un)) ? 1 : 0;
                const T um = rok ? un : (T)0;
                if (w == 0 && lane < R) uhist[(it & 1) * kSwRowMax + bi * R + lane] = um;
#pragma unroll
                for (int r = 0; r < R; ++r) u[r] = bcast_lane(um, r);
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) u[r] = r < nrow ? (SH ? (T)p.sh.u0[r0 + r] : u0) : (T)0;
            }
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int k = 0; k < VP2; ++k) {
                    T2 acc = colacc[g][k];
#pragma unroll
                    for (int r = 0; r < R; ++r) acc = e[r][g][k] * T2{u[r], u[r]} + acc;
                    colacc[g][k] = acc;
                }
        };
        // one buffer: block bi + 1 (past the last block: the NEXT sweep's block 0, C does
        // not change) is loaded as soon as block bi is widened
        for (int bi = 0; bi < my_nb; ++bi) process(bi, bufA, bi + 1 < my_nb ? bi + 1 : 0);
    };

    // ---- registration: XCD population, this workgroup's slot in its XCD group and the
    // group's first slab row (placement changes speed only: groups are counted, not assumed)
    if (tid == 0) {
        s_pop[3] = __hip_atomic_fetch_add(p.sync.reg + xcd * 64, 1, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
        if (gran && s_pop[3] < 256) store_wt(p.xl + xcd * 256 + s_pop[3], (int)blockIdx.x);
    }
    bool reg_ok = grid_barrier(p.bar, nwg, deadline, p.stall_ticks, &s_flag, &p.info->stalled);
    if (tid == 0) {
        int nact = 0, base = 0;
        unsigned mask = 0;
        for (int x = 0; x < 8; ++x) {
            const int c = __hip_atomic_load(p.sync.reg + x * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (x < xcd) base += c;
            if (c > 0) {
                ++nact;
                mask |= 1u << x;
            }
        }
        s_pop[0] = __hip_atomic_load(p.sync.reg + xcd * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_pop[1] = nact;
        s_pop[2] = (int)mask;
        s_pop[4] = base;
    }
    __syncthreads();
    const int nx = s_pop[0], nact = s_pop[1];
    const unsigned act_mask = (unsigned)s_pop[2];
    // granule flush: the XCC's members ranked by blockIdx (a placement-independent order
    // of the slab rows within the group)
    if (gran) {
        if (tid < nx && tid < 256) {
            const int b = load_agent(p.xl + xcd * 256 + tid);
            int rk = 0;
            for (int j = 0; j < nx && j < 256; ++j) rk += load_agent(p.xl + xcd * 256 + j) < b ? 1 : 0;
            mrow[rk] = b;
            if (b == (int)blockIdx.x) s_pop[5] = rk;
        }
        __syncthreads();
    }
    const int gslot_r = gran ? s_pop[5] : 0;
    // reduction group: the workgroups of this XCD (slot = registration order), or in the
    // deterministic mode the whole grid by blockIdx (placement- and timing-independent
    // order: every column sum is added in slab-row order by one workgroup, no atomics)
    const int gsz = p.det ? nwg : nx;
    const int gslot = p.det ? (int)blockIdx.x : s_pop[3];
    const int gfirst = p.det ? 0 : s_pop[4];
    int* const gctr = p.gcnt + (p.det ? 0 : xcd * 64);
    // this workgroup's column slice of the group reduction: [sl0, sl1) of m_pad
    const int slw = ((p.m_pad + gsz * VT - 1) / (gsz * VT)) * VT;
    const int sl0 = gslot * slw < p.m_pad ? gslot * slw : p.m_pad;
    const int sl1 = sl0 + slw < p.m_pad ? sl0 + slw : p.m_pad;

    // Flush the column partials into ring slot k, zero slot k + 1's share.  Partials go
    // through the XCD group: every workgroup stores its m partials write-through into its
    // slab row, the group meets on its counter (epoch k + 1), then each member sums ONE
    // column slice over the group's rows in a fixed order and adds it to the slot with
    // memory-side atomics: 8 x m atomics per iteration instead of grid x m.
    int gep = 0;
    const __amdgpu_buffer_rsrc_t srow = sums_rsrc(p.slab + (size_t)(gfirst + gslot) * p.m_pad);
    auto flush = [&](int k) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int c0 = (tid + kSwNT * g) * VC;
            if (c0 < p.m_pad) {
#pragma unroll
                for (int h = 0; h < VC / VT; ++h) {
                    V wv;
#pragma unroll
                    for (int k2 = 0; k2 < VT; ++k2) wv[k2] = colacc[g][(h * VT + k2) / 2][k2 & 1];
                    store_sum_vec<T>(srow, (uint32_t)((c0 + h * VT) * sizeof(T)), wv);
                }
            }
        }
        ++gep;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            int ok = 1;
            __hip_atomic_fetch_add(gctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            while (load_agent(gctr) < gep * gsz) {
                __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() > deadline) { ok = 0; break; }
            }
            s_flag = ok;
        }
        __syncthreads();
        if (!s_flag) gep = -1;  // stalled: the caller reports OTF_SK_TIMEOUT
        deadline = __builtin_amdgcn_s_memrealtime() + p.stall_ticks;
        // slice reduce: thread (q, j) sums rows q, q + Q, ... of vector j of the slice
        const int nv = (sl1 - sl0) / VT;
        int Q = 1;
        while (Q * 2 <= gsz && kSwNT / (Q * 2) >= nv) Q *= 2;
        const int W = kSwNT / Q, q = tid / W, j = tid % W;
        const __amdgpu_buffer_rsrc_t sr = sums_rsrc(p.slab + (size_t)gfirst * p.m_pad);
        for (int jb = 0; jb < nv; jb += W) {
            const int jv = jb + j;
            V acc;
#pragma unroll
            for (int k2 = 0; k2 < VT; ++k2) acc[k2] = 0;
            if (jv < nv) {
#pragma unroll 4
                for (int r = q; r < gsz; r += Q) {
                    const V t = load_sum_vec<T>(sr, (uint32_t)(((size_t)r * p.m_pad + sl0 + jv * VT) * sizeof(T)));
#pragma unroll
                    for (int k2 = 0; k2 < VT; ++k2) acc[k2] += t[k2];
                }
            }
            *reinterpret_cast<V*>(gred + (size_t)tid * VT) = acc;
            __syncthreads();
            if (q == 0 && jv < nv) {
                V tot = *reinterpret_cast<const V*>(gred + (size_t)j * VT);
                for (int qq = 1; qq < Q; ++qq) {
                    const V t = *reinterpret_cast<const V*>(gred + (size_t)(qq * W + j) * VT);
#pragma unroll
                    for (int k2 = 0; k2 < VT; ++k2) tot[k2] += t[k2];
                }
                *reinterpret_cast<V*>(vbuf + jv * VT) = tot;
            }
            __syncthreads();
        }
        T* dst = p.ring + (size_t)(k & 3) * p.slot_stride;
        const int send = sl1 < p.m ? sl1 : p.m;
        if (p.det) {
            for (int c = sl0 + tid; c < send; c += kSwNT) store_wt(dst + c, vbuf[c - sl0]);
        } else {
            for (int c = sl0 + tid; c < send; c += kSwNT) atomicAdd(dst + c, vbuf[c - sl0]);
        }
        // slot k + 1 (= S[k - 3]) is free: this workgroup's share of it, write-through
        T* zs = p.ring + (size_t)((k + 1) & 3) * p.slot_stride;
        const int64_t per = (p.slot_stride + nwg - 1) / nwg;
        const int64_t z0 = (int64_t)blockIdx.x * per;
        const int64_t z1 = z0 + per < p.slot_stride ? z0 + per : p.slot_stride;
        for (int64_t jz = z0 + tid; jz < z1; jz += kSwNT) store_wt(zs + jz, (T)0);
        if (tid == 0) {
            if (blockIdx.x == 0) store_wt(p.bad + ((k + 1) & 3) * 64, 0);
            if (badu) atomicAdd(p.bad + ((k - 1) & 3) * 64, 1);  // u(k-1) not finite
        }
        badu = 0;
    };

    // Granule flush of S[k] (see the header): false on a stall
    // slab rows polled per batch (fewer at G = 8, whose registers are the tightest)
    constexpr int NBT = G >= 8 ? 4 : 8;
    auto flush_gran = [&](int k) -> bool {
        const __amdgpu_buffer_rsrc_t rsl = sums_rsrc(p.gslab);
        const __amdgpu_buffer_rsrc_t rxx = sums_rsrc(p.xr[p.world > 1 ? p.rank : 0]);
        const __amdgpu_buffer_rsrc_t rxp = sums_rsrc(p.gxp);
        const __amdgpu_buffer_rsrc_t rfs = sums_rsrc(p.gfs);
        static_assert(!(sizeof(T) == 4) || VC % 4 == 0, "slab quads: whole 4-column groups per chunk");
        const int mq = p.m_pad / 4;                              // slab quads per row
        const int sw4 = (mq + kSwSlices - 1) / kSwSlices;        // slab quads per slice (<= 128)
        const int sw = 2 * sw4;                                  // granule pairs per slice (<= 256)
        const int swp = sw4 <= 64 ? 64 : 128;                    // stage b: lanes per row group
        const int Q = kSwNT / swp, sq = tid / swp, sj = tid % swp;
        const unsigned e = (p.ep_base + (unsigned)(k + 1)) & 0x3fffffffu;
        const unsigned et = qtag(e);
        const int xsp = 2 * (p.solve_par & 1);  // exchange slot set of this solve
        bool ok = true;
        // a. this workgroup's partials -> its slab row (four columns per chunk)
        const uint32_t rowo = (uint32_t)blockIdx.x * (uint32_t)mq * 16u;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int c0 = (tid + kSwNT * g) * VC;
            if (c0 < p.m_pad) {
#pragma unroll
                for (int h = 0; h < VC / 4; ++h)
                    gstore_col(rsl, rowo + (uint32_t)(c0 / 4 + h) * 16u,
                               chunk4((float)colacc[g][2 * h].x, (float)colacc[g][2 * h].y,
                                      (float)colacc[g][2 * h + 1].x, (float)colacc[g][2 * h + 1].y, et, badu),
                               1);
            }
        }
        badu = 0;
#ifdef OTF_STAMPS
        if (k >= 1 && k - 1 < 15) {  // (slot 15 * 8 + 7 holds the XCD id)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            OTF_STAMP(k - 1, 6);
        }
#endif
        // b. owned slices: sum over the XCC's members (rank order), publish the XCC partial
        // (lane sj of row group sq: slab quad sl * sw4 + sj of members sq, sq + Q, ...).
        // A member's flag rides in every chunk of its row, so the workgroup-wide OR of the
        // flags the slice's lanes saw is the OR over the XCC's members
        for (int sl = gslot_r; sl < kSwSlices; sl += nx) {
            const int cq = sl * sw4 + sj;
            const bool act = sj < sw4 && cq < mq;
            float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
            int fl = 0;
            for (int rb = sq; rb < nx; rb += NBT * Q) {
                I4 x[NBT];
                unsigned pend = 0;
#pragma unroll
                for (int i = 0; i < NBT; ++i) {
                    const int r = rb + i * Q;
                    if (act && r < nx) {
                        x[i] = gload(rsl, (uint32_t)mrow[r] * (uint32_t)mq * 16u + (uint32_t)cq * 16u);
                        pend |= 1u << i;
                    }
                }
#pragma unroll
                for (int i = 0; i < NBT; ++i)
                    if ((pend & (1u << i)) && chunk4_at(x[i], et)) pend &= ~(1u << i);
                while (pend && ok) {
                    __builtin_amdgcn_s_sleep(1);
#pragma unroll
                    for (int i = 0; i < NBT; ++i)
                        if (pend & (1u << i))
                            x[i] = gload(rsl, (uint32_t)mrow[rb + i * Q] * (uint32_t)mq * 16u + (uint32_t)cq * 16u);
#pragma unroll
                    for (int i = 0; i < NBT; ++i)
                        if ((pend & (1u << i)) && chunk4_at(x[i], et)) pend &= ~(1u << i);
                    if (pend && __builtin_amdgcn_s_memrealtime() > deadline) ok = false;
                }
#pragma unroll
                for (int i = 0; i < NBT; ++i)
                    if (act && rb + i * Q < nx) {
                        a0 += chunk4_v(x[i], 0);
                        a1 += chunk4_v(x[i], 1);
                        a2 += chunk4_v(x[i], 2);
                        a3 += chunk4_v(x[i], 3);
                        fl |= chunk4_flag(x[i]);
                    }
            }
            float* st = reinterpret_cast<float*>(gred);
            *reinterpret_cast<F4v*>(&st[tid * 4]) = F4v{a0, a1, a2, a3};
            const bool wfl = __any(fl != 0);
            if (lane == 0) s_fq[w] = wfl ? 1 : 0;
            __syncthreads();
            if (sq == 0 && act) {
                F4v s = *reinterpret_cast<const F4v*>(&st[sj * 4]);
                int f = 0;
#pragma unroll
                for (int ww = 0; ww < NW; ++ww) f |= s_fq[ww];
                for (int qq = 1; qq < Q; ++qq) s += *reinterpret_cast<const F4v*>(&st[(qq * swp + sj) * 4]);
                const uint32_t xo = (uint32_t)(((e & 1) * 8 + xcd) * mc + 2 * cq) * 16u;
                gstore(rxp, xo, chunk2(s[0], s[1], (int)(e << 2) | f));
                gstore(rxp, xo + 16u, chunk2(s[2], s[3], (int)(e << 2) | f));
            }
            __syncthreads();
        }
#ifdef OTF_STAMPS
        if (k >= 1 && k - 1 < 15) {  // (slot 15 * 8 + 7 holds the XCD id)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            OTF_STAMP(k - 1, 7);
        }
#endif
        // c. owned slices: S = the active XCCs' partials in XCC order (across ranks: this
        // rank's partial to every rank, then the world's partials in rank order) -> this
        // XCC's ring slot as plain floats; once every owner thread's stores are done, one
        // ready word per slice carries the epoch and the OR of the flags
        int nsl = 0;
        for (int sl = gslot_r; sl < kSwSlices; sl += nx, ++nsl) {
            const int cch = sl * sw + tid;  // one thread per granule pair of the slice
            const bool act = tid < sw && cch < mc;
            float s0 = 0.f, s1 = 0.f;
            int f = 0;
            if (act) {
                I4 x[8];
                unsigned pend = 0;
#pragma unroll
                for (int xx = 0; xx < 8; ++xx)
                    if (act_mask & (1u << xx)) {
                        x[xx] = gload(rxp, (uint32_t)(((e & 1) * 8 + xx) * mc + cch) * 16u);
                        pend |= 1u << xx;
                    }
#pragma unroll
                for (int xx = 0; xx < 8; ++xx)
                    if ((pend & (1u << xx)) && chunk_at(x[xx], e)) pend &= ~(1u << xx);
                while (pend && ok) {
                    __builtin_amdgcn_s_sleep(1);
#pragma unroll
                    for (int xx = 0; xx < 8; ++xx)
                        if (pend & (1u << xx)) x[xx] = gload(rxp, (uint32_t)(((e & 1) * 8 + xx) * mc + cch) * 16u);
#pragma unroll
                    for (int xx = 0; xx < 8; ++xx)
                        if ((pend & (1u << xx)) && chunk_at(x[xx], e)) pend &= ~(1u << xx);
                    if (pend && __builtin_amdgcn_s_memrealtime() > deadline) ok = false;
                }
#pragma unroll
                for (int xx = 0; xx < 8; ++xx)
                    if (act_mask & (1u << xx)) {
                        s0 += chunk_v0(x[xx]);
                        s1 += chunk_v1(x[xx]);
                        f |= (x[xx][1] | x[xx][3]) & 3;
                    }
                if (p.world > 1) {
                    if (xcd == __builtin_ctz(act_mask)) {
                        // this rank's partial of the slice -> every rank's exchange buffer
                        const uint32_t xo = (uint32_t)(((xsp + (e & 1)) * 8 + p.rank) * mc + cch) * 16u;
                        for (int r = 0; r < p.world; ++r)
                            gstore_sys(sums_rsrc(p.xr[r]), xo, chunk2(s0, s1, (int)(e << 2) | f));
                    }
                    // c'. the world's rank partials of the slice, in rank order
                    I4 y[8];
                    unsigned pr = 0;
#pragma unroll
                    for (int r = 0; r < 8; ++r)
                        if (r < p.world) {
                            y[r] = gload_sys(rxx, (uint32_t)(((xsp + (e & 1)) * 8 + r) * mc + cch) * 16u);
                            pr |= 1u << r;
                        }
#pragma unroll
                    for (int r = 0; r < 8; ++r)
                        if ((pr & (1u << r)) && chunk_at(y[r], e)) pr &= ~(1u << r);
                    while (pr && ok) {
                        __builtin_amdgcn_s_sleep(1);
#pragma unroll
                        for (int r = 0; r < 8; ++r)
                            if (pr & (1u << r)) y[r] = gload_sys(rxx, (uint32_t)(((xsp + (e & 1)) * 8 + r) * mc + cch) * 16u);
#pragma unroll
                        for (int r = 0; r < 8; ++r)
                            if ((pr & (1u << r)) && chunk_at(y[r], e)) pr &= ~(1u << r);
                        if (pr && __builtin_amdgcn_s_memrealtime() > deadline) ok = false;
                    }
                    s0 = 0.f;
                    s1 = 0.f;
                    f = 0;
#pragma unroll
                    for (int r = 0; r < 8; ++r)
                        if (r < p.world) {
                            s0 += chunk_v0(y[r]);
                            s1 += chunk_v1(y[r]);
                            f |= (y[r][1] | y[r][3]) & 3;
                        }
                }
                using F2s = __attribute__((ext_vector_type(2))) float;
                using U2s = __attribute__((ext_vector_type(2))) unsigned int;
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(U2s, F2s{s0, s1}), rfs,
                                                      (uint32_t)((xcd * 4 + (int)(e & 3)) * p.m_pad + 2 * cch) * 4u, 0, 0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const int bits = block_or((f & 1) | (ok ? 0 : 4), 4 + ((nsl + (int)e) & 1));
            if (tid == 0 && sl * sw < mc)
                __builtin_amdgcn_raw_buffer_store_b32((int)(e << 2) | (bits & 1), rfs,
                                                      (uint32_t)(32 * p.m_pad) * 4u +
                                                          (uint32_t)((xcd * 4 + (int)(e & 3)) * kSwSlices + sl) * 4u,
                                                      0, 0);
            if (bits & 4) ok = false;
        }
        ok = !block_or(ok ? 0 : 4, 2 + (int)(e & 1));
        deadline = __builtin_amdgcn_s_memrealtime() + p.stall_ticks;
        return ok;
    };

    // ---- prologue: S[0] = K^T u0
    if (my_nb > 0) load_block(0, bufA);
    sweep(-1);
    if (gran) {
        if (reg_ok && !flush_gran(0)) gep = -1;
    } else {
        flush(0);
    }
    int last_good = -1, niter = 0, status = OTF_SK_MAX_ITER, brk = -1, n_err = 0;
    bool done = false, ran_all = false;
    if (!reg_ok || gep < 0 ||
        (!gran && !xcd_barrier(p.sync, xcd, nx, nact, act_mask, 1, deadline, p.stall_ticks, &s_flag))) {
        status = OTF_SK_TIMEOUT;
        done = true;
    }

    for (int it = 0; it < p.max_iter && !done; ++it) {
        OTF_STAMP(it, 0);
        int prev_bad = (!gran && it >= 1) ? load_agent(p.bad + ((it - 1) & 3) * 64) : 0;
        int badv = 0, gfl = 0;
        bool gok = true;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            T s[VC], bv[VC];
            if (gran)
                load_sums_gran(it, g, s, gfl, gok);
            else
                load_sums_chunk(it, g, s);
            load_b_chunk(g, bv);
            T vv[VC];
#pragma unroll
            for (int k = 0; k < VC; ++k) {
                const bool ok = k < cnt[g];
                const T val = bv[k] / (ok ? s[k] : (T)1);
                badv |= (ok && ((s[k] == (T)0) || !finite_val(val))) ? 1 : 0;
                vv[k] = ok ? val : (T)0;
            }
            const int c0 = (tid + kSwNT * g) * VC;
            if (c0 < p.m_pad) {
#pragma unroll
                for (int h = 0; h < VC / VT; ++h) {
                    V wv;
#pragma unroll
                    for (int k2 = 0; k2 < VT; ++k2) wv[k2] = vv[h * VT + k2];
                    *reinterpret_cast<V*>(vbuf + c0 + h * VT) = wv;
                }
            }
        }
        if (gran) {  // S[it]'s flags: u(it-1) not finite; a stalled poll: timeout
            const int bits = block_or((gfl & 1) | (gok ? 0 : 4), it & 1);
            if (bits & 4) {
                status = OTF_SK_TIMEOUT;
                break;
            }
            prev_bad = bits & 1;
            deadline = __builtin_amdgcn_s_memrealtime() + p.stall_ticks;
        }
        if (prev_bad > 0) {  // u(it-1) not finite: revert to it-2
            last_good = it - 2; niter = it - 1; status = OTF_SK_NUMERICAL_BREAK; brk = it - 1;
            break;
        }
        if (it >= 1 && ((it - 1) % p.check_every) == 0) {
            const double err = marginal_err(it - 1);
            if (lead) p.errlog[(it - 1) / p.check_every] = err;
            n_err = (it - 1) / p.check_every + 1;
            if (p.err_squared ? !(err > p.stop_thr) : (err < p.stop_thr)) {
                last_good = it - 1; niter = it - 1; status = OTF_SK_CONVERGED;
                break;
            }
        }
        badv = __syncthreads_or(badv);
        if (badv) {  // zero in K^T u or non-finite v: revert to it-1
            last_good = it - 1; niter = it; status = OTF_SK_NUMERICAL_BREAK; brk = it;
            break;
        }
        OTF_STAMP(it, 1);
        sweep(it);
        OTF_STAMP(it, 2);
        if (gran) {
            if (!flush_gran(it + 1)) gep = -1;
        } else {
            flush(it + 1);
        }
        OTF_STAMP(it, 3);
#ifdef OTF_STAMPS
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        OTF_STAMP(it, 4);
#endif
        if (gep < 0 ||
            (!gran && !xcd_barrier(p.sync, xcd, nx, nact, act_mask, it + 2, deadline, p.stall_ticks, &s_flag))) {
            status = OTF_SK_TIMEOUT;
            done = true;
        }
        OTF_STAMP(it, 5);
        if (it == p.max_iter - 1 && !done) ran_all = true;
    }
    if (status == OTF_SK_MAX_ITER && ran_all) {
        const int it = p.max_iter - 1;
        int ubad = 0;
        if (gran) {  // u(it)'s flag rides in S[it + 1]
            int fl = 0;
            bool ok = true;
#pragma unroll
            for (int g = 0; g < G; ++g) {
                T tmp[VC];
                load_sums_gran(it + 1, g, tmp, fl, ok);
            }
            ubad = block_or(fl & 1, (it + 1) & 1) & 1;
        } else {
            ubad = load_agent(p.bad + (it & 3) * 64) > 0;
        }
        if (ubad) {
            last_good = it - 1; niter = it; status = OTF_SK_NUMERICAL_BREAK; brk = it;
        } else {
            last_good = it; niter = it;
            if ((it % p.check_every) == 0) {
                const double err = marginal_err(it);
                if (lead) p.errlog[it / p.check_every] = err;
                n_err = it / p.check_every + 1;
                if (p.err_squared ? !(err > p.stop_thr) : (err < p.stop_thr)) status = OTF_SK_CONVERGED;
            }
        }
    }

    // ---- outputs: (u, v) of last_good, then the plan by one more sweep
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const T v0 = (T)1 / (T)p.m;
#pragma unroll
    for (int g = 0; g < G; ++g) {
        T vo[VC];
        if (last_good >= 0) {
            T sl[VC], bv[VC];
            if (gran) {
                int fl = 0;
                bool ok = true;
                load_sums_gran(last_good, g, sl, fl, ok);
            } else {
                load_sums_chunk(last_good, g, sl);
            }
            load_b_chunk(g, bv);
#pragma unroll
            for (int k = 0; k < VC; ++k) vo[k] = k < cnt[g] ? bv[k] / sl[k] : (T)0;
        } else {
#pragma unroll
            for (int k = 0; k < VC; ++k) vo[k] = SH ? (k < cnt[g] ? (T)p.sh.v0[colc[g] + k] : (T)0) : v0;
        }
#pragma unroll
        for (int k = 0; k < VC; ++k) colacc[g][k / 2][k & 1] = vo[k];  // v(last_good) from here on
        if (blockIdx.x == 0) {
#pragma unroll
            for (int k = 0; k < VC; ++k)
                if (k < cnt[g]) p.v_out[colc[g] + k] = vo[k];
        }
    }
    const T* uh = uhist + (last_good & 1) * kSwRowMax;
    for (int bi = 0; bi < my_nb; ++bi) {
        const int r0 = ((int)blockIdx.x + bi * nwg) * R;
        if (tid < R && r0 + tid < p.n)
            p.u_out[r0 + tid] = last_good >= 0 ? uh[bi * R + tid] : SH ? (T)p.sh.u0[r0 + tid] : u0;
    }
    if (p.P) {
        TP* P = (TP*)p.P;
        constexpr int VP = Vec<T>::N;
        using PV = __attribute__((ext_vector_type(VP))) TP;
        for (int bi = 0; bi < my_nb; ++bi) {
            const int r0 = ((int)blockIdx.x + bi * nwg) * R;
            load_block(bi, bufA, KS);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (r0 + r >= p.n) break;
                const T ur = last_good >= 0 ? uh[bi * R + r] : SH ? (T)p.sh.u0[r0 + r] : u0;
                const T sa = SH ? shAl[bi * R + r] : (T)0;
                TP* prow = P + (int64_t)(r0 + r) * p.ldp;
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    if (cnt[g] == 0) continue;
                    const int c0 = colc[g];
                    T c[VC];
                    widen<T, CT>(bufA[r][g], c);
                    TP o[VC];
#pragma unroll
                    for (int k = 0; k < VC; ++k) {
                        T z = c[k] * ks;
                        if (SH) z += sa + shBl[c0 + k];
                        o[k] = (TP)(ur * (KS ? c[k] : fast_exp(z)) * colacc[g][k / 2][k & 1]);
                    }
                    if (cnt[g] == VC) {
#pragma unroll
                        for (int h = 0; h < VC / VP; ++h) {
                            PV pv;
#pragma unroll
                            for (int k = 0; k < VP; ++k) pv[k] = o[h * VP + k];
                            *reinterpret_cast<PV*>(prow + c0 + h * VP) = pv;
                        }
                    } else {
#pragma unroll
                        for (int k = 0; k < VC; ++k)
                            if (k < cnt[g]) prow[c0 + k] = o[k];
                    }
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
        p.info->engine = OTF_ENGINE_SWEEP;
        p.info->stop = 1;
    }
}

// Columns per thread (G chunks of 16 B) and rows per block R.  Per thread and column:
// the column partial (sizeof(T) / 4 VGPRs), then per row of a block the e value and the
// raw cost (one buffer: refilled with the next block once widened); R is the
// largest power of two that keeps these under ~150 of the 256 VGPRs a 512-thread
// workgroup gets at one workgroup per CU (the rest: addresses, masks, reductions).
#ifndef OTF_SWEEP_RBUDGET
#define OTF_SWEEP_RBUDGET 500
#endif
constexpr int pow2_floor(int x) { return x >= 16 ? 16 : x >= 8 ? 8 : x >= 4 ? 4 : x >= 2 ? 2 : 1; }
template <typename T, typename CT> constexpr int sweep_rows(int G) {
    return pow2_floor((OTF_SWEEP_RBUDGET / (G * RawN<CT>::N) - (int)sizeof(T)) /
                      ((int)sizeof(T) + (int)sizeof(CT)));
}
constexpr int kSwMaxG = 8;
// The float64 K stream (KS) carries no exp / scaling temporaries per element: its row
// blocks may be OTF_SWEEP_KS_RMUL times taller (fewer per-block row-sum barriers per sweep;
// 2 spills 32-37 VGPRs at G = 2..4 with this register budget, so the default is 1)
#ifndef OTF_SWEEP_KS_RMUL
#define OTF_SWEEP_KS_RMUL 1
#endif
template <typename T, typename CT> constexpr int sweep_rows_ks(int G, bool ks) {
    return ks ? (sweep_rows<T, CT>(G) * OTF_SWEEP_KS_RMUL > 16 ? 16 : sweep_rows<T, CT>(G) * OTF_SWEEP_KS_RMUL)
              : sweep_rows<T, CT>(G);
}

template <typename CT> int sweep_g(int64_t m) {
    int g = 1;
    while (g < kSwMaxG && (int64_t)kSwNT * g * RawN<CT>::N < m) g *= 2;
    return (int64_t)kSwNT * g * RawN<CT>::N < m ? 0 : g;
}

#ifndef OTF_SWEEP_NREP
#define OTF_SWEEP_NREP 1
#endif
constexpr int kSwMaxGrid = 256;  // slab rows in the workspace (one per workgroup)

// LDS: vbuf | u history | 1 / a | group-reduce staging (T), then the resident blocks
template <typename T> size_t sweep_lds_base(int64_t m_pad, bool sh = false) {
    return ((size_t)m_pad + 3 * kSwRowMax + (size_t)kSwNT * Vec<T>::N +
            (sh ? (size_t)m_pad + kSwRowMax : 0)) * sizeof(T);
}
size_t sweep_block_lds(int R, int G) { return (size_t)R * G * kSwNT * 16; }
constexpr size_t kSwLdsMax = 160 * 1024 - 4096;  // the CU's LDS less the static arrays
#ifndef OTF_SWEEP_MAXRES
#define OTF_SWEEP_MAXRES 4
#endif

template <typename T, typename CT, typename TP, int G, bool SH, bool KS = false>
hipError_t launch_sweep_gs(int grid, SkSweepArgs<T>& p, hipStream_t s) {
    constexpr int R = sweep_rows_ks<T, CT>(G, KS);
    // as many whole row blocks in LDS as fit, fewer than the smallest per-workgroup count
    const int nrb = (p.n + R - 1) / R;
    const int min_nb = nrb / grid;
    const size_t base = sweep_lds_base<T>(p.m_pad, SH);
    int nres = base < kSwLdsMax ? (int)((kSwLdsMax - base) / sweep_block_lds(R, G)) : 0;
    if (nres > OTF_SWEEP_MAXRES) nres = OTF_SWEEP_MAXRES;
    if (nres > min_nb - 1) nres = min_nb - 1 > 0 ? min_nb - 1 : 0;
    p.nres = nres;
    void* args[] = {&p};
    const void* k = (const void*)sk_sweep_kernel<T, CT, TP, G, R, OTF_SWEEP_NREP, SH, KS>;
    const size_t lds = base + (size_t)p.nres * sweep_block_lds(R, G);
    if (lds > kSwLdsMax + 4096) return hipErrorInvalidValue;
    if ((int64_t)((nrb + grid - 1) / grid) * R > kSwRowMax) return hipErrorInvalidValue;
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    int per_cu = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, kSwNT, lds);
    if (e != hipSuccess) return e;
    if (per_cu < 1 || grid > per_cu * device_cu_count()) return hipErrorCooperativeLaunchTooLarge;
    return hipLaunchKernel(k, dim3(grid), dim3(kSwNT), args, lds, s);
}

template <typename T, typename CT, typename TP, int G>
hipError_t launch_sweep_g(int grid, SkSweepArgs<T>& p, hipStream_t s) {
    if constexpr (sizeof(T) == 4)
        if (p.sh.A) return launch_sweep_gs<T, CT, TP, G, true>(grid, p, s);
    if constexpr (sizeof(T) == 8 && sizeof(CT) == 8)
        if (p.kbuf) return launch_sweep_gs<T, CT, TP, G, false, true>(grid, p, s);
    return launch_sweep_gs<T, CT, TP, G, false>(grid, p, s);
}

template <typename T, typename CT, typename TP>
hipError_t launch_sweep(int G, int grid, SkSweepArgs<T>& p, hipStream_t s) {
    switch (G) {
        case 1: return launch_sweep_g<T, CT, TP, 1>(grid, p, s);
        case 2: return launch_sweep_g<T, CT, TP, 2>(grid, p, s);
        case 4: return launch_sweep_g<T, CT, TP, 4>(grid, p, s);
        case 8:
            if constexpr (sizeof(CT) == 2) return hipErrorInvalidValue;  // m <= 16384 at G = 4
            else return launch_sweep_g<T, CT, TP, 8>(grid, p, s);
        default: return hipErrorInvalidValue;
    }
}

size_t align256(size_t x) { return (x + 255) / 256 * 256; }

// region: ring (4 slots) | bad counters | barrier | sync words | group counters, all
// zeroed per solve | slab (one row of column partials per workgroup, overwritten)
size_t sweep_ctrl_bytes(int64_t m_pad, size_t esz) {
    const size_t slot = (size_t)OTF_SWEEP_NREP * m_pad + 64;
    return align256(4 * slot * esz) + 4 * 256 + 256 + align256(kSyncBytes) + 8 * 256;
}
int sweep_grid(int64_t nrb) {
    int64_t g = nrb < device_cu_count() ? nrb : device_cu_count();
    return (int)(g < kSwMaxGrid ? g : kSwMaxGrid);
}

}  // namespace

// granule flush: slab rows + 2 x 8 XCC partials + 8 x 4 S slots (8 B a column) + lists
size_t sweep_gran_bytes(int64_t m_pad) { return (size_t)(kSwMaxGrid + 16 + 32) * m_pad * 8 + 8 * 256 * 4; }
template <typename T> size_t sweep_region_bytes(int64_t m_pad) {
    return sweep_ctrl_bytes(m_pad, sizeof(T)) + (size_t)kSwMaxGrid * m_pad * sizeof(T) +
           (sizeof(T) == 4 ? sweep_gran_bytes(m_pad) : 0);
}

template <typename T, typename CT> bool sweep_supported(int64_t n, int64_t m, int64_t ldc) {
    const int G = sweep_g<CT>(m);
    if (G == 0 || (sizeof(CT) == 2 && G > 4)) return false;
    if (ldc % RawN<CT>::N != 0) return false;
    if (n > INT32_MAX) return false;
    int R = 1;
    switch (G) {
        case 1: R = sweep_rows<T, CT>(1); break;
        case 2: R = sweep_rows<T, CT>(2); break;
        case 4: R = sweep_rows<T, CT>(4); break;
        default: R = sweep_rows<T, CT>(8); break;
    }
    const int64_t nrb = (n + R - 1) / R;
    const int64_t grid = sweep_grid(nrb);
    return (nrb + grid - 1) / grid * R <= kSwRowMax;
}

template <typename T, typename CT>
hipError_t run_sweep(const CT* C, int64_t ldc, int n, int m, int m_pad, const T* a_pad,
                     const T* b_pad, const T* cost_scale, const otf_sinkhorn_opts& o, void* region,
                     T* u_out, T* v_out, void* P_out, int64_t ldp, int P_dtype,
                     otf_sinkhorn_info* info, double* errlog, hipStream_t s, const XSweep* xs,
                     const ShiftArgs* sh, void* kbuf) {
    const int G = sweep_g<CT>(m);
    if (G == 0) return hipErrorInvalidValue;
    SkSweepArgs<T> p{};
    p.C = C;
    p.ldc = ldc;
    p.n = n;
    p.m = m;
    p.m_pad = m_pad;
    p.a = a_pad;
    p.b = b_pad;
    p.cost_scale = cost_scale;
    p.reg = o.reg;
    p.max_iter = o.max_iter;
    p.check_every = o.check_every;
    p.err_squared = o.err_squared;
    p.stop_thr = o.stop_thr;
    p.ring = (T*)region;
    p.slot_stride = (int64_t)OTF_SWEEP_NREP * m_pad + 64;
    char* q = (char*)region + align256(4 * (size_t)p.slot_stride * sizeof(T));
    p.bad = (int*)q;
    p.bar = (int*)(q + 4 * 256);
    p.sync = sync_words((int*)(q + 4 * 256 + 256));
    p.gcnt = (int*)(q + 4 * 256 + 256 + align256(kSyncBytes));
    p.slab = (T*)((char*)region + sweep_ctrl_bytes(m_pad, sizeof(T)));
    p.info = info;
    p.errlog = errlog;
    p.u_out = u_out;
    p.v_out = v_out;
    p.P = P_out;
    p.ldp = ldp;
    p.stall_ticks = stall_ticks();
    p.reg_ticks = reg_stall_ticks();
    p.nt_loads = (double)n * ldc * sizeof(CT) > 192.0 * (1 << 20) ? 1 : 0;
    p.det = o.deterministic ? 1 : 0;
    // float outside the deterministic mode: the granule flush; float64 and the
    // deterministic mode: the r02 flush (slab + group counter + atomics + grid barrier)
    p.gran = (sizeof(T) == 4 && !p.det) ? 1 : 0;
    p.world = 1;
    p.n_total = n;
    // float64: stream K (written by the prologue) when the caller's workspace holds it
    if (sizeof(T) == 8 && kbuf && !(xs && xs->world > 1)) p.kbuf = (T*)kbuf;
    if (sh) {
        if (sizeof(T) != 4 || (xs && xs->world > 1)) return hipErrorInvalidValue;
        p.sh = *sh;
    }
    if (xs && xs->world > 1) {  // the cross-rank form runs on the granule flush only
        if (sizeof(T) != 4 || xs->world > kXMaxRanks) return hipErrorInvalidValue;
        p.gran = 1;
        p.rank = xs->rank;
        p.world = xs->world;
        p.n_total = xs->n_total;
        p.ep_base = xs->ep_base;
        p.solve_par = xs->solve_par;
        for (int r = 0; r < xs->world; ++r) p.xr[r] = xs->xr[r];
    }
    size_t zero_bytes = sweep_ctrl_bytes(m_pad, sizeof(T));
    if (p.gran) {
        unsigned char* gb = (unsigned char*)p.slab + (size_t)kSwMaxGrid * m_pad * sizeof(T);
        p.gslab = gb;
        p.gxp = gb + (size_t)kSwMaxGrid * m_pad * 8;
        p.gfs = p.gxp + (size_t)16 * m_pad * 8;
        p.xl = (int*)(p.gfs + (size_t)32 * m_pad * 8);
        hipError_t e0 = hipMemsetAsync(gb, 0, sweep_gran_bytes(m_pad), s);  // tags: epoch 0
        if (e0 != hipSuccess) return e0;
    }
    hipError_t e = hipMemsetAsync(region, 0, zero_bytes, s);
    if (e != hipSuccess) return e;
    const bool ks = sizeof(T) == 8 && p.kbuf != nullptr;
    int R = 1;
    switch (G) {
        case 1: R = sweep_rows_ks<T, CT>(1, ks); break;
        case 2: R = sweep_rows_ks<T, CT>(2, ks); break;
        case 4: R = sweep_rows_ks<T, CT>(4, ks); break;
        default: R = sweep_rows_ks<T, CT>(8, ks); break;
    }
    const int nrb = (n + R - 1) / R;
    int grid = sweep_grid(nrb);
    // OTF_SWEEP_GRID caps the grid (tests: two ranks' persistent grids on one device)
    if (const char* gg = getenv("OTF_SWEEP_GRID"))
        if (atoi(gg) > 0 && atoi(gg) < grid) grid = atoi(gg);
    if (P_out && P_dtype == OTF_F64) return launch_sweep<T, CT, double>(G, grid, p, s);
    return launch_sweep<T, CT, float>(G, grid, p, s);
}

template size_t sweep_region_bytes<float>(int64_t);
template size_t sweep_region_bytes<double>(int64_t);
template bool sweep_supported<float, float>(int64_t, int64_t, int64_t);
template bool sweep_supported<float, _Float16>(int64_t, int64_t, int64_t);
template bool sweep_supported<double, double>(int64_t, int64_t, int64_t);
template hipError_t run_sweep<float, float>(const float*, int64_t, int, int, int, const float*,
                                            const float*, const float*, const otf_sinkhorn_opts&,
                                            void*, float*, float*, void*, int64_t, int,
                                            otf_sinkhorn_info*, double*, hipStream_t, const XSweep*,
                                            const ShiftArgs*, void*);
template hipError_t run_sweep<float, _Float16>(const _Float16*, int64_t, int, int, int, const float*,
                                               const float*, const float*, const otf_sinkhorn_opts&,
                                               void*, float*, float*, void*, int64_t, int,
                                               otf_sinkhorn_info*, double*, hipStream_t, const XSweep*,
                                            const ShiftArgs*, void*);
template hipError_t run_sweep<double, double>(const double*, int64_t, int, int, int, const double*,
                                              const double*, const double*, const otf_sinkhorn_opts&,
                                              void*, double*, double*, void*, int64_t, int,
                                              otf_sinkhorn_info*, double*, hipStream_t, const XSweep*,
                                            const ShiftArgs*, void*);

}  // namespace otf
