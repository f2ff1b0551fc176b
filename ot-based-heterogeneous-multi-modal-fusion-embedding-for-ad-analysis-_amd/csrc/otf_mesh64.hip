// otf_mesh64.hip — the mesh engine (otf_mesh.hip) in float64: POT's sinkhorn_knopp with
// K = exp(-C/reg) held on chip for the whole solve (OTF_ENGINE_MESH on a float64 cost).
//
// Replaces ot.sinkhorn (POT 0.9.6 sinkhorn_knopp, MRI_PET_OT_nojax.py:143 /
// perturbot/perturbot/match/utils.py:6-115) in the reference's own precision for the
// whole-tile shapes whose float64 K fits the chip: up to 32 x 8 tiles of 128 x 512, i.e.
// the N = 4096 metric shape (bench.py metric_f64), where the sweep engine streams the
// 134 MB K from the Infinity Cache every iteration (27 us per iteration).
//
// Storage.  A float64 K at N = 4096 is 128 MiB -- the size of all 256 CUs' register files
// together.  Each workgroup runs ONE wave per SIMD (4 waves, 256 threads), so a lane may
// address 512 registers (256 arch + 256 acc); its 32 rows x 8 columns of K are 256
// doubles: rows 0..23 of a wave's 32 live in registers (384 words; the compiler parks
// what exceeds the arch file in the acc file), rows 24..31 in LDS (128 KiB per
// workgroup, 16-B slots laid out lane-fastest so every ds_read_b128 is conflict-free).
//
// Protocol: the float mesh's three epoch-tagged granule hops per iteration (row hop
// across the row block's ncb members, hop A column partials to the column tile's
// reducers, hop B sums back), same roles (XCC-local column tiles after registration),
// same POT decisions carried in the tags.  A 16-B chunk carries two float64 values whose
// three low mantissa bits hold the tag -- epoch mod 4 and one flag bit (the gather
// engine's encoding, otf_gather.hip make_chunk): a slot written every epoch holds epoch
// e - 2 or e when a consumer waits for e, so two bits tell them apart; the value keeps a
// 49-bit mantissa (relative 2^-50, below the float64 rounding of the sums it enters).
// The error chunks, written only every check_every epochs, carry ONE value and the full
// epoch tag instead.  Every sum has one fixed order: bitwise reproducible run to run.
#include "otf_persist.h"
#include <type_traits>

namespace otf {
namespace {

constexpr int kM64NW = 4;                   // waves per workgroup (one per SIMD)
constexpr int kM64RW = 32;                  // rows per wave
constexpr int kM64RR = 24;                  // of them in registers
constexpr int kM64RL = kM64RW - kM64RR;     // in LDS
constexpr int kM64TR = kM64NW * kM64RW;     // 128 rows per tile
constexpr int kM64TC = 512;                 // columns per tile
constexpr int kM64NCH = kM64TC / 2;         // 16-B chunks (two columns) per tile row
constexpr uint32_t kM64RowStride = 1280;    // per producer: 64 row chunks + the error chunk
constexpr uint32_t kM64ColStride = 4096;    // per producer: 256 column chunks
constexpr int kM64MinNrb = 4, kM64MaxNrb = 32, kM64MaxNcb = 8;

struct SkMesh64Args {
    const double* C;
    int64_t ldc;
    int n, m;
    const double* a;
    const double* b;
    const double* cost_scale;
    double reg;
    int max_iter, check_every, err_squared;
    double stop_thr;
    void* gran;  // granule region, zeroed per solve
    uint32_t off_row, off_cola, off_colb, bstride;
    int nrb, ncb, cpr, xcc_local;
    int* xreg;   // [8 x 64] workgroups per XCC (registration), then the flat barrier word
    otf_sinkhorn_info* info;
    double* errlog;
    double* u_out;
    double* v_out;
    void* P;
    int64_t ldp;
    unsigned long long timeout_ticks;
    unsigned long long reg_ticks;
};

using D2 = __attribute__((ext_vector_type(2))) double;
using ull = unsigned long long;

// two float64 values, tag = epoch mod 4 | flag << 2 in their three low mantissa bits
__device__ __forceinline__ I4 dchunk(double v0, double v1, int e, int flag) {
    const unsigned low = (unsigned)(e & 3) | ((unsigned)flag << 2);
    const ull b0 = __builtin_bit_cast(ull, v0), b1 = __builtin_bit_cast(ull, v1);
    I4 x;
    x[0] = (int)(((unsigned)b0 & ~7u) | low);
    x[1] = (int)(unsigned)(b0 >> 32);
    x[2] = (int)(((unsigned)b1 & ~7u) | low);
    x[3] = (int)(unsigned)(b1 >> 32);
    return x;
}
__device__ __forceinline__ bool dchunk_at(const I4 x, unsigned e) {
    return (((unsigned)x[0] & 3u) == (e & 3u)) && (((unsigned)x[2] & 3u) == (e & 3u));
}
// element copies first (ROCm 7.2: a bit_cast of a vector ELEMENT reads element 0)
__device__ __forceinline__ double dchunk_v0(const I4 x) {
    const unsigned lo = (unsigned)x[0] & ~7u, hi = (unsigned)x[1];
    return __builtin_bit_cast(double, ((ull)hi << 32) | lo);
}
__device__ __forceinline__ double dchunk_v1(const I4 x) {
    const unsigned lo = (unsigned)x[2] & ~7u, hi = (unsigned)x[3];
    return __builtin_bit_cast(double, ((ull)hi << 32) | lo);
}
__device__ __forceinline__ int dchunk_flag(const I4 x) { return (int)((((unsigned)x[0] | (unsigned)x[2]) >> 2) & 1u); }
// one float64 value and the full epoch tag (the error chunks)
__device__ __forceinline__ I4 echunk(double v, int e) {
    const ull b = __builtin_bit_cast(ull, v);
    I4 x;
    x[0] = (int)(unsigned)b;
    x[1] = (int)(unsigned)(b >> 32);
    x[2] = e << 2;
    x[3] = e << 2;
    return x;
}
__device__ __forceinline__ bool echunk_at(const I4 x, unsigned e) {
    return ((unsigned)x[2] >> 2) == e && ((unsigned)x[3] >> 2) == e;
}
__device__ __forceinline__ double echunk_v(const I4 x) {
    const unsigned lo = (unsigned)x[0], hi = (unsigned)x[1];
    return __builtin_bit_cast(double, ((ull)hi << 32) | lo);
}
template <bool ERR>
__device__ __forceinline__ bool poll64(__amdgpu_buffer_rsrc_t rs, uint32_t off, unsigned e,
                                       unsigned long long deadline, I4& x) {
    for (;;) {
        x = gload(rs, off);
        if (ERR ? echunk_at(x, e) : dchunk_at(x, e)) return true;
        if (__builtin_amdgcn_s_memrealtime() > deadline) return false;
        __builtin_amdgcn_s_sleep(1);
    }
}

__device__ __forceinline__ double lane0_f64(double x) {
    const ull b = __builtin_bit_cast(ull, x);
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)b);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(b >> 32));
    return __builtin_bit_cast(double, ((ull)hi << 32) | lo);
}

// Diagnostic build only (-DOTF_M64_STAMPS, tools/stamps_mesh64.hip): wave 0's wall clock
// at the phases of iterations 0..15, keyed by the workgroup's role rb * ncb + cb
#ifdef OTF_M64_STAMPS
__device__ unsigned long long g_m64st[256 * 16 * 8];
__device__ unsigned long long g_m64pro[256 * 4];  // kernel start, roles known, K formed, loop end
#define OTF_M64PRO(ph)                                                                          \
    do {                                                                                        \
        if (threadIdx.x == 0 && rb * ncb + cb < 256)                                            \
            g_m64pro[(rb * ncb + cb) * 4 + (ph)] = __builtin_amdgcn_s_memrealtime();           \
    } while (0)
#define OTF_M64ST(it, ph)                                                                       \
    do {                                                                                        \
        if (threadIdx.x == 0 && (it) >= 0 && (it) < 16 && rb * ncb + cb < 256)                  \
            g_m64st[((rb * ncb + cb) * 16 + (it)) * 8 + (ph)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define OTF_M64ST(it, ph) \
    do {                  \
    } while (0)
#define OTF_M64PRO(ph) \
    do {               \
    } while (0)
#endif

constexpr int pow2_ceil(int x) { return x <= 1 ? 1 : 2 * pow2_ceil((x + 1) / 2); }

// SNRB, SNCB: the shape compiled in (0 = from the arguments).  Every shape is a mesh of
// whole tiles (n = nrb * 128, m = ncb * 512), so there are no bound tests.
template <typename TP, int SNRB, int SNCB>
__global__ __launch_bounds__(256) void sk_mesh64_kernel(SkMesh64Args p) {
    using T = double;
    constexpr int NW = kM64NW, R = kM64RW, RR = kM64RR, RL = kM64RL, TR = kM64TR, TC = kM64TC;
    constexpr bool FULL = SNRB != 0 && SNCB != 0;
    constexpr int KQ = 4;  // reducer loads per lane: nrb x CPR = 256 chunks over 64 lanes
    __shared__ __attribute__((aligned(16))) D2 sK[NW][RL][4][kWave];  // K rows 24..31 of each wave
    __shared__ __attribute__((aligned(16))) T colbuf[NW][TC];
    __shared__ __attribute__((aligned(16))) T vcur[TC];
    __shared__ __attribute__((aligned(16))) T vhist[2][TC];
    __shared__ __attribute__((aligned(16))) T uhist[2][TR];
    __shared__ T s_E;
    // flags keyed by epoch / iteration (keys only grow): [0] non-finite u here, [1] hop-B
    // stall, [2] hop-B producer flag, [3] zero / non-finite v, [4] row-hop stall
    __shared__ int s_ep[5];
    __shared__ int s_reg[4];
    int tid = threadIdx.x, lane = tid & 63;
    const int w = (int)threadIdx.x >> 6;
    unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + p.reg_ticks;
#ifdef OTF_M64_STAMPS
    const unsigned long long t_start = deadline - p.reg_ticks;
#endif
    const int nrb = FULL ? SNRB : p.nrb, ncb = FULL ? SNCB : p.ncb;
    const int CPR = FULL ? pow2_ceil(kM64NCH / SNRB) : p.cpr;
    const int m_ = FULL ? SNCB * TC : p.m;
    const int n_ = FULL ? SNRB * TR : p.n;

    // roles: registration on the hardware XCC, column tile = the XCC's rank (as otf_mesh.hip)
    int rb = 0, cb = 0, xl = 0;
    if (p.xcc_local) {
        const int xcd = xcc_id();
        if (tid == 0)
            s_reg[0] = __hip_atomic_fetch_add(p.xreg + xcd * 64, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool ok = grid_barrier(p.xreg + 8 * 64, gridDim.x, deadline, p.timeout_ticks, &s_reg[3],
                                     &p.info->stalled);
        if (tid == 0) {
            int good = ok ? 1 : 0, rank = -1, nq = 0;
            for (int x = 0; x < 8; ++x) {
                const int c = load_agent(p.xreg + x * 64);
                if (c >= nrb && nq < ncb) {
                    if (x == xcd) rank = nq;
                    ++nq;
                }
            }
            if (nq < ncb) good = 0;
            s_reg[1] = good;
            s_reg[2] = rank;
        }
        __syncthreads();
        if (!s_reg[3]) {
            if (tid == 0) mark_stalled(&p.info->stalled, kStallRegistration);
            return;
        }
        if (s_reg[1]) {
            if (s_reg[2] < 0 || s_reg[0] >= nrb) return;
            rb = s_reg[0];
            cb = s_reg[2];
            xl = 1;
        }
    }
    if (!xl) {
        const int bi = blockIdx.x;
        if (bi >= nrb * ncb) return;
        rb = bi / ncb;
        cb = bi % ncb;
    }
    const bool lead = (rb == 0 && cb == 0 && tid == 0);
#ifdef OTF_M64_STAMPS
    if (threadIdx.x == 0 && rb * ncb + cb < 256) g_m64pro[(rb * ncb + cb) * 4] = t_start;
#endif
    OTF_M64PRO(1);
    const int row0 = rb * TR + w * R;
    const int col0 = cb * TC;
    const int nch = kM64NCH;
    const int nred = (nch + CPR - 1) / CPR;

    double cinv = 1.0;
    if (p.cost_scale) cinv = 1.0 / p.cost_scale[0];
    const T ks = -1.0 / p.reg * cinv;

    // ---- K: this wave's 32 rows x this lane's 8 columns (pairs j = 2 g + k2 of columns
    // (lane + 64 g) * 4 + 2 k2, + 1); rows < 24 in registers, the rest in LDS
    D2 kv[RR][4];
    {
        const T* crow = p.C + (int64_t)row0 * p.ldc + col0 + lane * 4;
#pragma unroll
        for (int r = 0; r < R; ++r) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const D2 c = *reinterpret_cast<const D2*>(crow + (j >> 1) * 256 + (j & 1) * 2);
                const D2 e = D2{exp(c[0] * ks), exp(c[1] * ks)};
                if (r < RR) kv[r][j] = e;
                else sK[w][r - RR][j][lane] = e;
            }
            crow += p.ldc;
            // one row's loads in flight at a time: hoisting all 32 rows' loads needs 512
            // registers on top of K and spills the prologue to scratch
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    OTF_M64PRO(2);
    auto kget = [&](int r, int j) -> D2 { return r < RR ? kv[r][j] : sK[w][r - RR][j][lane]; };
    // 1 / a of the rows this lane group finishes after the row hop: chunk c = lane >> 3
    // of each half (rows 2c, 2c + 1 and 16 + 2c, 16 + 2c + 1 of the wave's 32)
    const int rc = lane >> 3;
    T ia[4];
    ia[0] = 1.0 / p.a[row0 + 2 * rc];
    ia[1] = 1.0 / p.a[row0 + 2 * rc + 1];
    ia[2] = 1.0 / p.a[row0 + 16 + 2 * rc];
    ia[3] = 1.0 / p.a[row0 + 16 + 2 * rc + 1];
    // hop-B consumer: chunk tid -> columns col0 + 2 tid, + 1
    const T bch0 = p.b[col0 + 2 * tid], bch1 = p.b[col0 + 2 * tid + 1];
    // reducer (wave 0): chunk r_cc = lane % CPR of this workgroup's range, producers
    // q = lane / CPR + LPC k
    const int LPC = kWave / CPR;
    const int r_cc = lane & (CPR - 1), r_qlo = lane / CPR;
    const int r_ch = rb * CPR + r_cc;
    const bool r_ok = r_ch < nch;
    T rb0 = 0, rb1 = 0;
    if (w == 0 && r_ok) {
        rb0 = p.b[col0 + 2 * r_ch];
        rb1 = p.b[col0 + 2 * r_ch + 1];
    }
    T sp0 = 1, sp1 = 1;  // the reducer's previous sums S[k - 1]

    const T u0 = 1.0 / (T)n_, v0 = 1.0 / (T)m_;
    if (tid < 5) s_ep[tid] = -1;
    for (int q = tid; q < TC; q += blockDim.x) {
        vhist[0][q] = vhist[1][q] = v0;
        vcur[q] = 0;
    }
    if (tid < TR) uhist[0][tid] = uhist[1][tid] = u0;
    __syncthreads();

    const __amdgpu_buffer_rsrc_t rs = sums_rsrc(p.gran);
    auto rowx = [&](int e, int q) -> uint32_t {
        return p.off_row + ((uint32_t)((e & 1) * nrb + rb) * (uint32_t)ncb + (uint32_t)q) * kM64RowStride;
    };
    auto cola = [&](int e, int q) -> uint32_t {
        return p.off_cola + ((uint32_t)((e & 1) * ncb + cb) * (uint32_t)nrb + (uint32_t)q) * kM64ColStride;
    };
    auto colb = [&](int e, int j) -> uint32_t {
        return p.off_colb + ((uint32_t)((e & 1) * ncb + cb) * (uint32_t)nrb + (uint32_t)j) * p.bstride;
    };

    // column partials of rows [R0, R0 + NR) of this wave against u (LDS, wave-uniform
    // reads), accumulated into acc in ascending row order
    auto col_acc = [&](D2 (&acc)[4], const T* ur, auto r0c) {
        constexpr int R0 = decltype(r0c)::value;
#pragma unroll
        for (int r = R0; r < R0 + 16; r += 2) {
            const D2 uu = *reinterpret_cast<const D2*>(ur + r);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[j] = __builtin_elementwise_fma(kget(r, j), D2{uu[0], uu[0]}, acc[j]);
                acc[j] = __builtin_elementwise_fma(kget(r + 1, j), D2{uu[1], uu[1]}, acc[j]);
            }
        }
    };
    auto col_store = [&](const D2 (&acc)[4]) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            *reinterpret_cast<D2*>(&colbuf[w][(j >> 1) * 256 + lane * 4 + (j & 1) * 2]) = acc[j];
    };
    auto col_partials = [&](const T* ur) {
        D2 acc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = D2{0.0, 0.0};
        col_acc(acc, ur, std::integral_constant<int, 0>{});
        col_acc(acc, ur, std::integral_constant<int, 16>{});
        col_store(acc);
    };
    // hop A: the workgroup's column partials (after the barrier), epoch e; flag = non-finite u
    auto publish_cols = [&](int e, int flag) {
        D2 s = *reinterpret_cast<const D2*>(&colbuf[0][2 * tid]);
#pragma unroll
        for (int ww = 1; ww < NW; ++ww) s += *reinterpret_cast<const D2*>(&colbuf[ww][2 * tid]);
        gstore_col(rs, cola(e, rb) + (uint32_t)tid * 16, dchunk(s[0], s[1], e, flag), xl);
    };
    // reducer (wave 0): S[e - 1] of this workgroup's chunk range from the nrb producers of
    // epoch e in a fixed order; hop B carries the OR of their flags and (need) the error
    // terms of iterate e - 2.  Returns false on a stall.
    auto reduce = [&](int e, bool need) -> bool {
        I4 x[KQ];
        bool act[KQ];
#pragma unroll
        for (int k = 0; k < KQ; ++k) act[k] = r_ok && (r_qlo + LPC * k) < nrb;
        bool ok = true;
        for (;;) {
            unsigned pend = 0;
#pragma unroll
            for (int k = 0; k < KQ; ++k) {
                const int q = r_qlo + LPC * k;
                x[k] = gload(rs, cola(e, act[k] ? q : 0) + (uint32_t)(r_ok ? r_ch : 0) * 16);
            }
#pragma unroll
            for (int k = 0; k < KQ; ++k)
                if (act[k] && !dchunk_at(x[k], (unsigned)e)) pend |= 1u << k;
            if (!__any(pend != 0)) break;
            if (__builtin_amdgcn_s_memrealtime() > deadline) { ok = false; break; }
            __builtin_amdgcn_s_sleep(1);
        }
        T s0 = 0, s1 = 0;
        int fl = 0;
#pragma unroll
        for (int k = 0; k < KQ; ++k)
            if (act[k]) {
                s0 += dchunk_v0(x[k]);
                s1 += dchunk_v1(x[k]);
                fl |= dchunk_flag(x[k]);
            }
        if (CPR <= 1) { s0 += wave_xor<T, 1>(s0); s1 += wave_xor<T, 1>(s1); }
        if (CPR <= 2) { s0 += wave_xor<T, 2>(s0); s1 += wave_xor<T, 2>(s1); }
        if (CPR <= 4) { s0 += wave_xor<T, 4>(s0); s1 += wave_xor<T, 4>(s1); }
        if (CPR <= 8) { s0 += wave_xor<T, 8>(s0); s1 += wave_xor<T, 8>(s1); }
        if (CPR <= 16) { s0 += wave_xor<T, 16>(s0); s1 += wave_xor<T, 16>(s1); }
        if (CPR <= 32) { s0 += wave_xor<T, 32>(s0); s1 += wave_xor<T, 32>(s1); }
        const int bad = __any(fl) ? 1 : 0;
        T term = 0;
        if (need) {
            if (r_ok) {
                const T r0 = (rb0 / sp0) * s0 - rb0, r1 = (rb1 / sp1) * s1 - rb1;
                term = r0 * r0 + r1 * r1;
            }
            if (CPR > 1) term += wave_xor<T, 1>(term);
            if (CPR > 2) term += wave_xor<T, 2>(term);
            if (CPR > 4) term += wave_xor<T, 4>(term);
            if (CPR > 8) term += wave_xor<T, 8>(term);
            if (CPR > 16) term += wave_xor<T, 16>(term);
            if (CPR > 32) term += wave_xor<T, 32>(term);
        }
        sp0 = s0;
        sp1 = s1;
        if (lane < CPR && r_ok) gstore_col(rs, colb(e, rb) + (uint32_t)r_cc * 16, dchunk(s0, s1, e, bad), xl);
        if (need && lane == 0 && rb < nred) gstore_col(rs, colb(e, rb) + (uint32_t)CPR * 16, echunk(term, e), xl);
        deadline = __builtin_amdgcn_s_memrealtime() + p.timeout_ticks;
        return ok;
    };
    // hop B: S[e - 1] of this tile's columns -> v into vcur; the tile's error partial into
    // s_E.  Returns bit 0 = producer flag, 1 = stall, 2 = bad v.
    auto gather_b = [&](int e, bool need) -> int {
        int fl = 0;
        {
            const uint32_t off = colb(e, tid / CPR) + (uint32_t)(tid & (CPR - 1)) * 16;
            I4 x;
            if (!poll64<false>(rs, off, (unsigned)e, deadline, x)) fl |= 2;
            fl |= dchunk_flag(x);
            const T s0 = dchunk_v0(x), s1 = dchunk_v1(x);
            const T v0n = bch0 / s0, v1n = bch1 / s1;
            if (s0 == 0.0 || !finite_val(v0n) || s1 == 0.0 || !finite_val(v1n)) fl |= 4;
            *reinterpret_cast<D2*>(&vcur[2 * tid]) = D2{v0n, v1n};
        }
        if (w == 3 && need) {
            T ep = 0;
            if (lane < nred) {
                I4 x;
                if (!poll64<true>(rs, colb(e, lane) + (uint32_t)CPR * 16, (unsigned)e, deadline, x)) fl |= 2;
                ep = echunk_v(x);
            }
            ep = wave_sum<T>(ep);
            if (lane == 0) s_E = ep;
        }
        if (fl & 1) s_ep[2] = e;
        if (fl & 2) s_ep[1] = e;
        if (fl & 4) s_ep[3] = e;
        __syncthreads();
        deadline = __builtin_amdgcn_s_memrealtime() + p.timeout_ticks;
        return (s_ep[2] == e ? 1 : 0) | (s_ep[1] == e ? 2 : 0) | (s_ep[3] == e ? 4 : 0);
    };
    // total error from the ncb column tiles' partials (row-hop error chunks of epoch er)
    auto err_total = [&](int er, T& tot) -> bool {
        T ev = 0;
        bool ok = true;
        if (lane < ncb) {
            I4 x;
            ok = poll64<true>(rs, rowx(er, lane) + 64 * 16, (unsigned)er, deadline, x);
            ev = echunk_v(x);
        }
        ev += wave_xor<T, 1>(ev);
        ev += wave_xor<T, 2>(ev);
        ev += wave_xor<T, 4>(ev);
        tot = lane0_f64(ev);
        return __all(ok);
    };
    auto to_err = [&](T e) -> double { return p.err_squared ? e : sqrt(e); };
    auto stop_ok = [&](double err) -> bool { return p.err_squared ? !(err > p.stop_thr) : (err < p.stop_thr); };

    // ---- prologue: S[0] = K^T u0 (epoch 1)
    col_partials(&uhist[0][w * R]);
    __syncthreads();
    publish_cols(1, 0);
    int last_good = -1, niter = 0, status = OTF_SK_MAX_ITER, brk = -1, n_err = 0;
    bool done = false;
    if (w == 0 && !reduce(1, false)) s_ep[1] = 1;
    int chk = 0;

    for (int it = 0; it < p.max_iter; ++it) {
        asm volatile("" : "+v"(tid), "+v"(lane));
        const int e = it + 1;
        const bool check = it >= 1 && chk == 0;
        OTF_M64ST(it, 0);
        const int fl = gather_b(e, check);
        OTF_M64ST(it, 1);
        if (fl & 2) { status = OTF_SK_TIMEOUT; done = true; break; }
        if (fl & 1) {
            last_good = it - 2; niter = it - 1; status = OTF_SK_NUMERICAL_BREAK; brk = it - 1;
            done = true;
            break;
        }
        const int vbad_cb = (fl & 4) ? 1 : 0;
        D2 vn[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) vn[j] = *reinterpret_cast<const D2*>(&vcur[(j >> 1) * 256 + lane * 4 + (j & 1) * 2]);
        // Two halves of the wave's 32 rows, pipelined: each half's row partials are
        // published as soon as its wave totals are known, so the row hop of rows 0..15 is
        // in flight while rows 16..31 are summed, and rows 16..31's hop while the column
        // partials of rows 0..15 run.  Lane group c = lane >> 3 ends a half with its rows
        // 2c, 2c + 1.
        if (it >= 1) chk = chk + 1 == p.check_every ? 0 : chk + 1;
        const bool hop = ncb > 1;
        T t[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            T rp[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                D2 acc = kget(16 * h + r, 0) * vn[0];
#pragma unroll
                for (int j = 1; j < 4; ++j) acc = __builtin_elementwise_fma(kget(16 * h + r, j), vn[j], acc);
                rp[r] = acc[0] + acc[1];
            }
            const T mine = wave_row_totals<T, 16>(rp, lane), oth = dpp_lane<0x141>(mine);
            const bool odd = (lane & 4) != 0;
            t[2 * h] = odd ? oth : mine;
            t[2 * h + 1] = odd ? mine : oth;
            if (hop && (lane & 7) == 0)
                gstore(rs, rowx(e, cb) + (uint32_t)(w * 16 + 8 * h + rc) * 16, dchunk(t[2 * h], t[2 * h + 1], e, vbad_cb));
        }
        OTF_M64ST(it, 2);
        if (hop && check && w == 0 && lane == 1) gstore(rs, rowx(e, cb) + 64 * 16, echunk(s_E, e));
        T errv = hop ? 0.0 : s_E;
        int vbad = vbad_cb, stall = 0, badu = 0;
        const int q = lane & 7;
        const bool act = hop && q < ncb;
        D2 cacc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) cacc[j] = D2{0.0, 0.0};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            T th0 = t[2 * h], th1 = t[2 * h + 1];
            if (hop) {
                // gather the ncb members' chunk of this half (lane (c, q): member q)
                I4 x = I4{0, 0, 0, 0};
                if (act && !poll64<false>(rs, rowx(e, q) + (uint32_t)(w * 16 + 8 * h + rc) * 16, (unsigned)e, deadline, x))
                    stall = 1;
                th0 = act ? dchunk_v0(x) : 0.0;
                th1 = act ? dchunk_v1(x) : 0.0;
                if (__any(act && dchunk_flag(x))) vbad = 1;
                th0 += dpp_lane<0xB1>(th0);
                th1 += dpp_lane<0xB1>(th1);
                th0 += dpp_lane<0x4E>(th0);
                th1 += dpp_lane<0x4E>(th1);
                th0 += dpp_lane<0x141>(th0);
                th1 += dpp_lane<0x141>(th1);
            }
            // u of this half's two rows of the lane group; the group's first lane writes
            // them to the history, which the wave then reads back as wave-uniform values
            const T un0 = 1.0 / (th0 * ia[2 * h]), un1 = 1.0 / (th1 * ia[2 * h + 1]);
            if (__any(!finite_val(un0) || !finite_val(un1))) badu = 1;
            if ((lane & 7) == 0) *reinterpret_cast<D2*>(&uhist[it & 1][w * R + 16 * h + 2 * rc]) = D2{un0, un1};
            // the wave's own LDS writes complete before its reads (in-order LDS per wave);
            // the clobber keeps the compiler from hoisting the reads above the writes
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (h == 0) col_acc(cacc, &uhist[it & 1][w * R], std::integral_constant<int, 0>{});
            else col_acc(cacc, &uhist[it & 1][w * R], std::integral_constant<int, 16>{});
        }
        col_store(cacc);
        if (hop && check && !err_total(e, errv)) stall = 1;
        stall = __any(stall) ? 1 : 0;
        OTF_M64ST(it, 3);
        double err = 0.0;
        int dec = 0;
        if (check) {
            err = to_err(errv);
            if (stop_ok(err)) dec = 1;
        }
        if (dec == 0 && vbad) dec = 2;
        const int slot = it & 1;
        *reinterpret_cast<D2*>(&vhist[slot][2 * tid]) = *reinterpret_cast<const D2*>(&vcur[2 * tid]);
        if (badu) s_ep[0] = it;
        if (stall) s_ep[4] = it;
        OTF_M64ST(it, 4);
        __syncthreads();
        OTF_M64ST(it, 5);
        if (s_ep[4] == it) { status = OTF_SK_TIMEOUT; done = true; break; }
        if (check) {
            if (lead) p.errlog[n_err] = err;
            ++n_err;
        }
        if (dec == 1) {
            last_good = it - 1; niter = it - 1; status = OTF_SK_CONVERGED;
            done = true;
            break;
        }
        if (dec == 2) {
            last_good = it - 1; niter = it; status = OTF_SK_NUMERICAL_BREAK; brk = it;
            done = true;
            break;
        }
        publish_cols(e + 1, s_ep[0] == it ? 1 : 0);
        OTF_M64ST(it, 6);
        if (w == 0 && !reduce(e + 1, chk == 0)) s_ep[1] = e + 1;
        OTF_M64ST(it, 7);
    }
    if (!done && p.max_iter > 0) {
        const int it = p.max_iter - 1;
        const int e = p.max_iter + 1;
        const int fl = gather_b(e, (it % p.check_every) == 0);
        if (fl & 2) {
            status = OTF_SK_TIMEOUT;
        } else if (fl & 1) {
            last_good = it - 1; niter = it; status = OTF_SK_NUMERICAL_BREAK; brk = it;
        } else {
            last_good = it; niter = it;
            if ((it % p.check_every) == 0) {
                T errv = s_E;
                int stall = 0;
                if (ncb > 1) {
                    if (w == 0 && lane == 8) gstore(rs, rowx(e, cb) + 64 * 16, echunk(s_E, e));
                    if (!err_total(e, errv)) stall = 1;
                    if (stall) s_ep[4] = e;
                    __syncthreads();
                    stall = s_ep[4] == e;
                }
                if (stall) {
                    status = OTF_SK_TIMEOUT;
                } else {
                    const double err = to_err(errv);
                    if (lead) p.errlog[it / p.check_every] = err;
                    n_err = it / p.check_every + 1;
                    if (stop_ok(err)) status = OTF_SK_CONVERGED;
                }
            }
        }
    }

    // ---- outputs: (u, v) of last_good from the histories, the plan from K
    OTF_M64PRO(3);
    __syncthreads();
    const int hs = last_good & 1;
    D2 vo[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
        vo[j] = last_good >= 0 ? *reinterpret_cast<const D2*>(&vhist[hs][(j >> 1) * 256 + lane * 4 + (j & 1) * 2])
                               : D2{v0, v0};
    if (cb == 0 && lane < R) p.u_out[row0 + lane] = last_good >= 0 ? uhist[hs][w * R + lane] : u0;
    if (rb == 0 && w == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            *reinterpret_cast<D2*>(p.v_out + col0 + (j >> 1) * 256 + lane * 4 + (j & 1) * 2) = vo[j];
    }
    if (p.P) {
        TP* P = (TP*)p.P;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const T ur = last_good >= 0 ? uhist[hs][w * R + r] : u0;
            TP* prow = P + (int64_t)(row0 + r) * p.ldp + col0 + lane * 4;
#pragma unroll
            for (int g = 0; g < 2; ++g) {
                const D2 k0 = kget(r, 2 * g), k1 = kget(r, 2 * g + 1);
                const D2 o0 = (ur * k0) * vo[2 * g], o1 = (ur * k1) * vo[2 * g + 1];
                if constexpr (sizeof(TP) == 8) {
                    *reinterpret_cast<D2*>(prow + g * 256) = o0;
                    *reinterpret_cast<D2*>(prow + g * 256 + 2) = o1;
                } else {
                    using F4 = __attribute__((ext_vector_type(4))) float;
                    *reinterpret_cast<F4*>(prow + g * 256) = F4{(float)o0[0], (float)o0[1], (float)o1[0], (float)o1[1]};
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    if (status == OTF_SK_TIMEOUT && tid == 0) mark_stalled(&p.info->stalled, kStallMid);
    if (lead) {
        p.info->last_good = last_good;
        p.info->niter = niter;
        p.info->status = status;
        p.info->break_iter = brk;
        p.info->n_err = n_err;
        p.info->engine = OTF_ENGINE_MESH;
        p.info->stop = 1;
    }
}

template <typename TP>
hipError_t launch_mesh64_t(int grid, SkMesh64Args& p, hipStream_t s) {
    void* args[] = {&p};
    const void* k = (p.nrb == 32 && p.ncb == 8) ? (const void*)sk_mesh64_kernel<TP, 32, 8>
                                                : (const void*)sk_mesh64_kernel<TP, 0, 0>;
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 256, 0);
    if (e != hipSuccess) return e;
    if (per_cu < 1 || grid > per_cu * device_cu_count()) return hipErrorCooperativeLaunchTooLarge;
    return hipLaunchKernel(k, dim3(grid), dim3(256), args, 0, s);
}

constexpr size_t kM64RegBytes = 9 * 256;  // 8 XCC counters + the barrier word, 256 B each

struct Mesh64Shape {
    int nrb, ncb, cpr;
    uint32_t bstride;
    size_t row_bytes, cola_bytes, colb_bytes;
};

Mesh64Shape mesh64_shape(int64_t n, int64_t m) {
    Mesh64Shape s{};
    s.nrb = (int)(n / kM64TR);
    s.ncb = (int)(m / kM64TC);
    s.cpr = pow2_ceil(kM64NCH / (s.nrb > 0 ? s.nrb : 1));
    s.bstride = (uint32_t)((s.cpr + 1) * 16 + 255) / 256 * 256;
    s.row_bytes = 2 * (size_t)s.nrb * s.ncb * kM64RowStride;
    s.cola_bytes = 2 * (size_t)s.nrb * s.ncb * kM64ColStride;
    s.colb_bytes = 2 * (size_t)s.nrb * s.ncb * s.bstride;
    return s;
}

}  // namespace

// whole tiles only: n a multiple of 128 (4..32 row blocks, a power of two so that the
// reducers' 4 loads per lane cover the producers), m a multiple of 512 (1..8 column tiles)
bool mesh64_supported(int64_t n, int64_t m) {
    if (n < 1 || m < 1 || n % kM64TR != 0 || m % kM64TC != 0) return false;
    const int64_t nrb = n / kM64TR, ncb = m / kM64TC;
    return nrb >= kM64MinNrb && nrb <= kM64MaxNrb && (nrb & (nrb - 1)) == 0 && ncb <= kM64MaxNcb;
}

size_t mesh64_region_bytes(int64_t n, int64_t m) {
    if (!mesh64_supported(n, m)) return 0;
    const Mesh64Shape s = mesh64_shape(n, m);
    return kM64RegBytes + s.row_bytes + s.cola_bytes + s.colb_bytes;
}

hipError_t run_mesh64(const double* C, int64_t ldc, int n, int m, const double* a_pad, const double* b_pad,
                      const double* cost_scale, const otf_sinkhorn_opts& o, void* region, double* u_out,
                      double* v_out, void* P_out, int64_t ldp, int P_dtype, otf_sinkhorn_info* info,
                      double* errlog, bool zeroed, hipStream_t s) {
    if (!mesh64_supported(n, m) || !region) return hipErrorInvalidValue;
    if (ldc % 2 != 0 || ((uintptr_t)C % 16) != 0) return hipErrorInvalidValue;
    if (P_out && (ldp % 4 != 0 || ((uintptr_t)P_out % 16) != 0)) return hipErrorInvalidValue;
    const Mesh64Shape sh = mesh64_shape(n, m);
    SkMesh64Args p{};
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
    p.xreg = (int*)region;
    p.gran = (char*)region + kM64RegBytes;
    p.off_row = 0;
    p.off_cola = (uint32_t)sh.row_bytes;
    p.off_colb = (uint32_t)(sh.row_bytes + sh.cola_bytes);
    p.bstride = sh.bstride;
    p.nrb = sh.nrb;
    p.ncb = sh.ncb;
    p.cpr = sh.cpr;
    {
        const char* e = getenv("OTF_MESH_XCC");  // 0: blockIdx roles, write-through everywhere
        p.xcc_local = e ? atoi(e) : 1;
    }
    p.info = info;
    p.errlog = errlog;
    p.u_out = u_out;
    p.v_out = v_out;
    p.P = P_out;
    p.ldp = ldp;
    p.timeout_ticks = stall_ticks();
    p.reg_ticks = reg_stall_ticks();
    if (!zeroed) {
        const hipError_t e = hipMemsetAsync(region, 0, mesh64_region_bytes(n, m), s);
        if (e != hipSuccess) return e;
    }
    int grid = sh.nrb * sh.ncb;
    if (grid > device_cu_count()) return hipErrorCooperativeLaunchTooLarge;
    if (p.xcc_local && 8 * sh.nrb <= device_cu_count()) grid = 8 * sh.nrb;
    else p.xcc_local = 0;
    if (P_out && P_dtype == OTF_F32) return launch_mesh64_t<float>(grid, p, s);
    return launch_mesh64_t<double>(grid, p, s);
}

}  // namespace otf
