// otf_mesh64.hip — the mesh engine (otf_mesh.hip) in float64: POT's sinkhorn_knopp with
// K = exp(-C/reg) held on chip for the whole solve (OTF_ENGINE_MESH on a float64 cost).
//
// Replaces ot.sinkhorn (POT 0.9.6 sinkhorn_knopp, MRI_PET_OT_nojax.py:143 /
// perturbot/perturbot/match/utils.py:6-115) in the reference's own precision for the
// whole-tile shapes whose float64 K fits the chip: up to 32 x 8 tiles of 128 x 512, i.e.
// the N = 4096 metric shape (bench.py headline), where the sweep engine streams the
// 134 MB K from the Infinity Cache every iteration (27 us per iteration).
//
// Storage.  A float64 K at N = 4096 is 128 MiB -- the size of all 256 CUs' register files
// together.  Each workgroup runs EIGHT waves (two per SIMD, 256 registers a lane, all of
// them architectural: no accumulation-file reads in the loop) and holds its 128 x 512 tile
// as 8 stripes of 64 columns, one per wave.  Lane l of wave w (rr = l & 15, g = l >> 4)
// owns rows rr + 16 a (a < 8) and columns 64 w + 16 b + 4 g + i (b, i < 4) -- the
// accumulator layout of v_mfma_f64_16x16x4_f64 with the column block as the M index --
// column blocks b = 0..2 in registers (192 words), b = 3 in LDS (128 KiB per workgroup,
// lane-fastest 16-B slots: every ds_read_b128 is conflict-free).  (r04's form: four waves,
// one per SIMD, 32 rows x 8 columns a lane, ~220 of its 384 K words in the accumulation
// file: ~480 v_accvgpr_read and ~2 080 VALU per iteration against ~1 000 here.)
//
// Per iteration (epoch e = it + 1):
//   hop B    each wave polls the 32 column-sum chunks of its stripe from the reducers ->
//            v (wave-local LDS, no workgroup barrier);
//   rows     K v over the lane's 16 columns, the 4 lanes of a row (lane bits 5, 4) by two
//            permlane swaps, the 8 waves' partials through LDS -- barrier B1 -- and wave 0
//            publishes the tile's 128 row partials (64 chunks) for the row hop;
//   row hop  every thread polls one (chunk, member) of the row block's ncb column tiles,
//            8-lane DPP sums -> u of 2 rows -> LDS -- barrier B2;
//   columns  K^T u over the lane's 8 rows, the 16 lanes of a column (lane bits 3..0) by a
//            DPP halving butterfly, published per wave straight to the column tile's
//            reducers (no workgroup reduction);
//   reduce   workgroup rb owns chunks [rb CPR, +CPR) of the column tile, spread over its 8
//            waves: each sums its chunks over the nrb producers in a fixed order and
//            publishes S (and its share of POT's marginal-error terms).
// POT's decisions (zero / non-finite v, non-finite u, the error check and stop) ride in the
// tags and in LDS flags keyed by epoch, read after the barriers, so every wave of every
// workgroup takes the same decision at the same iteration.  A 16-B chunk carries two
// float64 values whose three low mantissa bits hold the tag -- epoch mod 4 and one flag
// bit (otf_gather.hip make_chunk); the error chunks, written only every check_every epochs,
// carry ONE value and the full epoch tag.  Every sum has one fixed order: bitwise
// reproducible run to run.
#include "otf_persist.h"
#include <type_traits>

namespace otf {
namespace {

constexpr int kM64NW = 8;                   // waves per workgroup (two per SIMD)
constexpr int kM64TR = 128;                 // rows per tile
constexpr int kM64TC = 512;                 // columns per tile
constexpr int kM64WC = kM64TC / kM64NW;     // 64 columns per wave
constexpr int kM64NA = 8;                   // lane rows rr + 16 a
constexpr int kM64NB = 4;                   // lane columns 16 b + 4 g + i
constexpr int kM64RB = 3;                   // column blocks in registers (b = 3 in LDS)
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
    // pairwise form (PW kernels): the cost tile built in the prologue from the float32 rows
    PairwiseF64 pw;
};

using D2 = __attribute__((ext_vector_type(2))) double;
using D4 = __attribute__((ext_vector_type(4))) double;
using F4 = __attribute__((ext_vector_type(4))) float;
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

// Diagnostic build only (-DOTF_M64_STAMPS, tools/stamps_mesh64.hip): wave 0's wall clock
// at the phases of iterations 0..15, keyed by the workgroup's role rb * ncb + cb
#ifdef OTF_M64_STAMPS
__device__ unsigned long long g_m64st[256 * 16 * 8];
__device__ unsigned long long g_m64pro[256 * 4];  // kernel start, roles known, K formed, loop end
// the pairwise prologue: block 3 built, blocks 0..2 built, the grid max known, K formed
__device__ unsigned long long g_m64pw[256 * 4];
// the shader clock (s_memtime) at the entry of the cost build and at the same four points:
// the effective core clock of each phase
__device__ unsigned long long g_m64pwc[256 * 5];
#define OTF_M64PW(ph)                                                                            \
    do {                                                                                         \
        if (threadIdx.x == 0 && sid < 256) {                                                     \
            g_m64pw[sid * 4 + (ph)] = __builtin_amdgcn_s_memrealtime();                          \
            g_m64pwc[sid * 5 + (ph) + 1] = __builtin_amdgcn_s_memtime();                         \
        }                                                                                        \
    } while (0)
#define OTF_M64PWC0()                                                                            \
    do {                                                                                         \
        if (threadIdx.x == 0 && sid < 256) g_m64pwc[sid * 5] = __builtin_amdgcn_s_memtime();     \
    } while (0)
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
#define OTF_M64PW(ph) \
    do {              \
    } while (0)
#define OTF_M64PWC0() \
    do {              \
    } while (0)
#endif

constexpr size_t kM64RegBytes = 11 * 256;  // 8 XCC counters, the registration barrier, the
                                           // PW max barrier and the PW max, 256 B each
constexpr int kM64MaxBar = 9 * 64, kM64MaxWord = 10 * 64;  // int offsets in xreg

// PW prologue (sk_mesh64_kernel<..., PW = true>): the workgroup's 128 x 512 tile of
// C = |x|^2 + |y|^2 - 2 x.y (POT euclidean_distances order, MRI_PET_OT_nojax.py:70-75) on
// v_mfma_f64_16x16x4_f64 straight from the float32 rows -- float4 buffer loads per lane,
// the k order inside each 16-deep chunk permuted the same way for both operands (lane
// group g holds k = 16 t + 4 g + q, step q takes element q), no LDS staging -- with the
// columns as the M index: Y row 4 (rr & 3) + (rr >> 2) of a 16-column block lands in
// accumulator element r of lane (rr, g) as column 4 g + r, the K layout.  Block 3 first
// (into LDS), then blocks 0..2 accumulate in the K registers themselves; clamped at 0 (and
// the square root for the euclidean metric).  The grid's max: one atomic max per workgroup
// + a flat barrier; then K = exp(-C / (reg max)) in place.  Returns false on a stall.
template <typename SK>
__device__ __forceinline__ bool pw_cost_tile(const SkMesh64Args& p, D4 (&kr)[kM64NA][kM64RB], SK& sK, int w,
                                             int lane, int rr, int g, int row0, int col0, int cw,
                                             int target, bool lead, unsigned long long& deadline,
                                             int* s_flag, double* s_red, F4* s_xs2, int sid, int* abandon) {
    (void)sid;
    OTF_M64PWC0();
    constexpr int NA = kM64NA, RB = kM64RB;
    const PairwiseF64& q = p.pw;
    const int cm = 4 * (rr & 3) + (rr >> 2);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(q.X), 0, (int)q.xbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(q.Y), 0, (int)q.ybytes, 0x00020000);
    const uint32_t yo = (uint32_t)(((int64_t)(col0 + cw + cm) * q.ldy + 4 * g) * 4);
    const uint32_t ys16 = (uint32_t)(16 * q.ldy * 4);
    const int nt = q.d / 16;
    auto ldy4 = [&](int b, int t) -> F4 {
        return __builtin_bit_cast(F4, __builtin_amdgcn_raw_buffer_load_b128(ry, yo, (uint32_t)b * ys16 + (uint32_t)t * 64u, 0));
    };
    // X is the same for the 8 waves: each chunk (128 rows x 16 k, 8 KiB) is loaded once per
    // workgroup -- thread (cr, cq) one float4 -- and staged in LDS, slot r * 4 + (q ^ (r >> 2
    // & 3)) (conflict-free: the 16 rows of a lane group spread over the 64 banks); a lane
    // reads row rr + 16 a, quarter g at rslot + 64 a
    const int cr = (int)threadIdx.x >> 2, cq = (int)threadIdx.x & 3;
    const uint32_t xco = (uint32_t)(((int64_t)(row0 + cr) * q.ldx + 4 * cq) * 4);
    const int cslot = cr * 4 + (cq ^ ((cr >> 2) & 3));
    const int rslot = rr * 4 + (g ^ ((rr >> 2) & 3));
    auto ldxc = [&](int t) -> F4 {
        return __builtin_bit_cast(F4, __builtin_amdgcn_raw_buffer_load_b128(rx, xco, (uint32_t)t * 64u, 0));
    };
    // POT's order: -2 x.y + |x|^2 + |y|^2, clamped at 0 (the euclidean root in its own pass)
    auto fin = [&](double acc, double nxi, double nyj) -> double {
        double v = -2.0 * acc;
        v += nxi;
        v += nyj;
        return v > 0 ? v : 0.0;
    };
    double lmax = 0.0;
    // block 3 -> LDS
    {
        D4 acc[NA];
#pragma unroll
        for (int a = 0; a < NA; ++a) acc[a] = D4{0.0, 0.0, 0.0, 0.0};
        // software-pipelined: chunk t + 1's operands in flight during chunk t's 32 MFMAs (the
        // norm-only loads of blocks 0..2 are consumed after them); X double-buffered in
        // wave 0's block-3 LDS area (free until the epilogue), one barrier per chunk
        // X ring of three chunks in the first block-3 areas (free until the epilogue): chunk
        // t + 1 is read into registers while chunk t's MFMAs run, chunk t + 2 is written
        F4* xs1 = reinterpret_cast<F4*>(&sK[0][0][0][0]);
        xs1[cslot] = ldxc(0);
        xs1[512 + cslot] = ldxc(nt > 1 ? 1 : 0);
        F4 yv = ldy4(3, 0);
        __syncthreads();
        F4 xv[NA];
#pragma unroll
        for (int a = 0; a < NA; ++a) xv[a] = xs1[rslot + 64 * a];
        int s1 = 1, s2 = 2;  // ring slots of chunks t + 1, t + 2
        for (int t = 0; t < nt; ++t) {
            const int t1 = t + 1 < nt ? t + 1 : t;
            const int t2 = t + 2 < nt ? t + 2 : nt - 1;
            const F4 xr = ldxc(t2), yvn = ldy4(3, t1);
            F4 xn[NA];
#pragma unroll
            for (int a = 0; a < NA; ++a) xn[a] = xs1[s1 * 512 + rslot + 64 * a];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const double yk = (double)yv[k];
#pragma unroll
                for (int a = 0; a < NA; ++a)
                    acc[a] = __builtin_amdgcn_mfma_f64_16x16x4f64(yk, (double)xv[a][k], acc[a], 0, 0, 0);
            }
            xs1[s2 * 512 + cslot] = xr;
            yv = yvn;
#pragma unroll
            for (int a = 0; a < NA; ++a) xv[a] = xn[a];
            s1 = s1 == 2 ? 0 : s1 + 1;
            s2 = s2 == 2 ? 0 : s2 + 1;
            __syncthreads();
        }
        const D4 nyv = *reinterpret_cast<const D4*>(q.ny + col0 + cw + 48 + 4 * g);
#pragma unroll
        for (int a = 0; a < NA; ++a) {
            const double nxi = q.nx[row0 + rr + 16 * a];
            D4 c;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                c[r] = fin(acc[a][r], nxi, nyv[r]);
                if (q.euclid) c[r] = sqrt(c[r]);
                lmax = fmax(lmax, c[r]);
            }
            sK[w][a][0][lane] = D2{c[0], c[1]};
            sK[w][a][1][lane] = D2{c[2], c[3]};
        }
        // block 3 lives in LDS from here: no register copy kept across the second pass
        asm volatile("" : "+v"(lmax) :: "memory");
    }
    OTF_M64PW(0);
    // blocks 0..2 in the K registers
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int b = 0; b < RB; ++b) kr[a][b] = D4{0.0, 0.0, 0.0, 0.0};
    // the 192 accumulators leave ~40 registers: X staged in LDS (one 8-KiB buffer, two
    // barriers per chunk), the next chunk's X and Y in flight during this chunk's MFMAs
    {
        F4 yv[RB], yn[RB];
#pragma unroll
        for (int b = 0; b < RB; ++b) yv[b] = ldy4(b, 0);
        s_xs2[cslot] = ldxc(0);
        __syncthreads();
        for (int t = 0; t < nt; ++t) {
            const int tn = t + 1 < nt ? t + 1 : t;
            const F4 xr = ldxc(tn);
#pragma unroll
            for (int a = 0; a < NA; ++a) {
                const F4 xv = s_xs2[rslot + 64 * a];
                if (a == NA / 2) {
#pragma unroll
                    for (int b = 0; b < RB; ++b) yn[b] = ldy4(b, tn);
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const double xk = (double)xv[k];
#pragma unroll
                    for (int b = 0; b < RB; ++b)
                        kr[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)yv[b][k], xk, kr[a][b], 0, 0, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            __syncthreads();  // every wave is done with chunk t
            s_xs2[cslot] = xr;
#pragma unroll
            for (int b = 0; b < RB; ++b) yv[b] = yn[b];
            __syncthreads();
        }
    }
#pragma unroll
    for (int b = 0; b < RB; ++b) {
        const D4 nyv = *reinterpret_cast<const D4*>(q.ny + col0 + cw + 16 * b + 4 * g);
#pragma unroll
        for (int a = 0; a < NA; ++a) {
            const double nxi = q.nx[row0 + rr + 16 * a];
#pragma unroll
            for (int r = 0; r < 4; ++r) kr[a][b][r] = fin(kr[a][b][r], nxi, nyv[r]);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    if (q.euclid) {
#pragma unroll
        for (int a = 0; a < NA; ++a)
#pragma unroll
            for (int b = 0; b < RB; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) kr[a][b][r] = sqrt(kr[a][b][r]);
    }
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int b = 0; b < RB; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) lmax = fmax(lmax, kr[a][b][r]);
    // the grid's max (costs are >= 0: the bit patterns order like the values)
    lmax = wave_max(lmax);
    if (lane == 0) s_red[w] = lmax;
    __syncthreads();
    OTF_M64PW(1);  // every wave of the workgroup done
    if (threadIdx.x == 0) {
        double mx = s_red[0];
        for (int ww = 1; ww < kM64NW; ++ww) mx = fmax(mx, s_red[ww]);
        __hip_atomic_fetch_max(reinterpret_cast<unsigned long long*>(p.xreg + kM64MaxWord),
                               __builtin_bit_cast(unsigned long long, mx), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // blockIdx roles (no registration barrier ran): this is the launch's first device-wide
    // wait, so a grid that never became co-resident gives up here as a registration give-up
    // (abandon = info->stalled) and the fallback queued behind the launch solves the problem
    if (!grid_barrier(p.xreg + kM64MaxBar, target, deadline, p.timeout_ticks, s_flag, abandon)) return false;
    OTF_M64PW(2);
    const double cmax = __builtin_bit_cast(
        double, __hip_atomic_load(reinterpret_cast<unsigned long long*>(p.xreg + kM64MaxWord), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT));
    if (lead && q.cmax_out) *q.cmax_out = cmax;
    const double cinv = q.scale ? 1.0 / cmax : 1.0;
    const double ks = -1.0 / p.reg * cinv;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
#pragma unroll
        for (int b = 0; b < RB; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) kr[a][b][r] = exp(kr[a][b][r] * ks);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const D2 c = sK[w][a][h][lane];
            sK[w][a][h][lane] = D2{exp(c[0] * ks), exp(c[1] * ks)};
        }
    }
    OTF_M64PW(3);
    return true;
}

constexpr int pow2_ceil(int x) { return x <= 1 ? 1 : 2 * pow2_ceil((x + 1) / 2); }
// u history slot of tile row r: lane rr = r & 15 reads its 8 rows rr + 16 a as one run
__device__ __forceinline__ int upos(int r) { return (r & 15) * 8 + (r >> 4); }

// SNRB, SNCB: the shape compiled in (0 = from the arguments).  Every shape is a mesh of
// whole tiles (n = nrb * 128, m = ncb * 512), so there are no bound tests.  PW: the cost
// tile is built in the prologue from the float32 rows (p.pw) instead of read from C.
template <typename TP, int SNRB, int SNCB, bool PW>
__global__ __launch_bounds__(512) void sk_mesh64_kernel(SkMesh64Args p) {
    using T = double;
    constexpr int NW = kM64NW, TR = kM64TR, TC = kM64TC, WC = kM64WC, NA = kM64NA, NB = kM64NB,
                  RB = kM64RB;
    constexpr bool FULL = SNRB != 0 && SNCB != 0;
    __shared__ __attribute__((aligned(16))) D2 sK[NW][NA][2][kWave];  // column block b = 3
    __shared__ __attribute__((aligned(16))) T rowbuf[NW][TR];         // per-wave row partials
    __shared__ __attribute__((aligned(16))) T vcur[NW][WC];           // v of this iteration
    __shared__ __attribute__((aligned(16))) T vhist[2][TC];
    __shared__ __attribute__((aligned(16))) T uhist[2][TR];           // slot upos(r)
    __shared__ __attribute__((aligned(16))) T bsh[TC];                // b of the tile's columns
    __shared__ __attribute__((aligned(16))) T iash[TR];               // 1 / a of its rows
    __shared__ __attribute__((aligned(16))) T spsh[2][kWave];         // the reducer's S[k - 1] by chunk
    __shared__ T s_err;
    // flags keyed by epoch / iteration (keys only grow): [0] non-finite u, [1] hop-B stall,
    // [2] hop-B producer flag, [3] zero / non-finite v, [4] row-hop stall, [5] a member's
    // bad-v flag in the row hop
    __shared__ int s_ep[6];
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
    const int rr = lane & 15, g = lane >> 4;
    const int row0 = rb * TR;
    const int col0 = cb * TC;
    const int cw = w * WC;
    const int nch = kM64NCH;
    const int nred = (nch + CPR - 1) / CPR;

    double cinv = 1.0;
    if (p.cost_scale) cinv = 1.0 / p.cost_scale[0];
    const T ks = -1.0 / p.reg * cinv;

    // ---- K: rows rr + 16 a, columns cw + 16 b + 4 g + (0..3) as two pairs h; blocks
    // b < 3 in registers, b = 3 in LDS
    // lane (rr, g) of wave w holds rows rr + 16 a x columns cw + 16 b + 4 g + (0..3) of
    // block b < 3 as one 4-vector (the v_mfma_f64_16x16x4_f64 accumulator of that 16 x 16
    // block with the columns as its M index: PW builds the cost right there)
    D4 kr[NA][RB];
    if constexpr (PW) {
        if (!pw_cost_tile(p, kr, sK, w, lane, rr, g, row0, col0, cw, nrb * ncb, lead, deadline, &s_reg[3],
                          &spsh[0][0], reinterpret_cast<F4*>(&vhist[0][0]),
                          rb * ncb + cb, p.xcc_local ? nullptr : &p.info->stalled)) {
            // the max barrier stalled: a mid-solve stall (OTF_SK_TIMEOUT; kept at the registration
            // give-up when the barrier gave up as one), every workgroup leaves
            if (tid == 0) {
                mark_stalled(&p.info->stalled, kStallMid);
                if (lead) p.info->status = OTF_SK_TIMEOUT;
            }
            return;
        }
    } else {
        const T* cbase = p.C + (int64_t)(row0 + rr) * p.ldc + col0 + cw + 4 * g;
#pragma unroll
        for (int a = 0; a < NA; ++a) {
            const T* crow = cbase + (int64_t)(16 * a) * p.ldc;
#pragma unroll
            for (int b = 0; b < NB; ++b) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const D2 c = *reinterpret_cast<const D2*>(crow + 16 * b + 2 * h);
                    const D2 e = D2{exp(c[0] * ks), exp(c[1] * ks)};
                    if (b < RB) {
                        kr[a][b][2 * h] = e[0];
                        kr[a][b][2 * h + 1] = e[1];
                    } else {
                        sK[w][a][h][lane] = e;
                    }
                }
            }
            // one row group's loads in flight at a time: hoisting them all needs 256
            // registers on top of K
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    OTF_M64PRO(2);
    auto kget = [&](int a, int b, int h) -> D2 {
        return b < RB ? D2{kr[a][b][2 * h], kr[a][b][2 * h + 1]} : sK[w][a][h][lane];
    };
    // row hop: thread -> chunk gc (rows 2 gc, 2 gc + 1 of the tile), member gq
    const int gc = 8 * w + (lane >> 3), gq = lane & 7;
    // hop B: lane < 32 polls chunk 32 w + lane of the tile (columns cw + 2 lane, + 1)
    const int hch = 32 * w + (lane & 31);
    // reducer, spread over the 8 waves: wave w sums chunks w + 8 j (j < CPR / 8) of this
    // workgroup's range [rb CPR, +CPR); lane l < 32 polls chunk j = l / nrb of producer
    // q = l % nrb (CPR / 8 x nrb = 32 for every nrb)
    const int r_j = (lane & 31) / nrb, r_q = (lane & 31) & (nrb - 1);
    const int r_cc = w + 8 * r_j;
    const int r_ch = rb * CPR + r_cc;
    // the marginals and the reducer's previous sums live in LDS (registers hold K)
    const T u0 = 1.0 / (T)n_, v0 = 1.0 / (T)m_;
    if (tid < 6) s_ep[tid] = -1;
    for (int q = tid; q < TC; q += blockDim.x) {
        vhist[0][q] = vhist[1][q] = v0;
        bsh[q] = p.b[col0 + q];
    }
    if (tid < TR) {
        uhist[0][tid] = uhist[1][tid] = u0;
        iash[tid] = 1.0 / p.a[row0 + tid];
    }
    if (tid < kWave) spsh[0][tid] = spsh[1][tid] = 1.0;
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

    // K^T u over the lane's 8 rows for each column block b, summed over the 16 lanes of a
    // column (lane bits 3..0: row mirror and half mirror with keep / send, then quad ^2,
    // ^1 -- every step adds two disjoint lane sets), then published per wave as chunks
    // (columns i = 0, 1 and 2, 3 of the lane group) by lanes rr = 0 and 8
    auto col_publish = [&](const T (&u)[NA], int e, int flag) {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            T c0, c1, c2, c3;
            {
                const D2 k0 = kget(0, b, 0), k1 = kget(0, b, 1);
                c0 = k0[0] * u[0];
                c1 = k0[1] * u[0];
                c2 = k1[0] * u[0];
                c3 = k1[1] * u[0];
            }
#pragma unroll
            for (int a = 1; a < NA; ++a) {
                const D2 k0 = kget(a, b, 0), k1 = kget(a, b, 1);
                c0 = fma(k0[0], u[a], c0);
                c1 = fma(k0[1], u[a], c1);
                c2 = fma(k1[0], u[a], c2);
                c3 = fma(k1[1], u[a], c3);
            }
            const D2 q01 = D2{c0, c1}, q23 = D2{c2, c3};
            const bool b3 = (lane & 8) != 0, b2 = (lane & 4) != 0;
            // bit 3: keep i in {2, 3} (upper) or {0, 1}
            const T k0 = b3 ? q23[0] : q01[0], k1 = b3 ? q23[1] : q01[1];
            const T s0 = b3 ? q01[0] : q23[0], s1 = b3 ? q01[1] : q23[1];
            const T r0 = k0 + dpp_lane<0x140>(s0), r1 = k1 + dpp_lane<0x140>(s1);
            // bit 2: keep i = 2 b3 + b2
            const T kk = b2 ? r1 : r0, ss = b2 ? r0 : r1;
            T t = kk + dpp_lane<0x141>(ss);
            t += dpp_lane<0x4E>(t);
            t += dpp_lane<0xB1>(t);
            // the chunk's second column (i + 1) sits in the lanes with bit 2 flipped
            const T o = dpp_lane<0x141>(t);
            if ((lane & 7) == 0)
                gstore_col(rs, cola(e, rb) + (uint32_t)(32 * w + 8 * b + 2 * g + (b3 ? 1 : 0)) * 16,
                           dchunk(t, o, e, flag), xl);
        }
    };
    // reducer (every wave, its chunks of this workgroup's range): S[e - 1] from the nrb
    // producers of epoch e summed over the producer lanes in a fixed order; hop B carries
    // the OR of their flags and (need) the wave's error terms of iterate e - 2 in error slot
    // w of the range.  Returns false on a stall.
    auto reduce = [&](int e, bool need) -> bool {
        I4 x;
        bool ok = true;
        const uint32_t off = cola(e, r_q) + (uint32_t)r_ch * 16;
        for (;;) {
            x = gload(rs, off);
            if (!__any(lane < 32 && !dchunk_at(x, (unsigned)e))) break;
            if (__builtin_amdgcn_s_memrealtime() > deadline) { ok = false; break; }
            __builtin_amdgcn_s_sleep(1);
        }
        T s0 = dchunk_v0(x), s1 = dchunk_v1(x);
        if (nrb > 1) { s0 += wave_xor<T, 1>(s0); s1 += wave_xor<T, 1>(s1); }
        if (nrb > 2) { s0 += wave_xor<T, 2>(s0); s1 += wave_xor<T, 2>(s1); }
        if (nrb > 4) { s0 += wave_xor<T, 4>(s0); s1 += wave_xor<T, 4>(s1); }
        if (nrb > 8) { s0 += wave_xor<T, 8>(s0); s1 += wave_xor<T, 8>(s1); }
        if (nrb > 16) { s0 += wave_xor<T, 16>(s0); s1 += wave_xor<T, 16>(s1); }
        const int bad = __any(lane < 32 && dchunk_flag(x)) ? 1 : 0;
        const bool head = lane < 32 && r_q == 0;  // the lane that owns chunk r_cc
        if (need) {
            T term = 0;
            if (head) {
                const T sp0 = spsh[0][r_cc], sp1 = spsh[1][r_cc];
                const T rb0 = bsh[2 * r_ch], rb1 = bsh[2 * r_ch + 1];
                const T r0 = (rb0 / sp0) * s0 - rb0, r1 = (rb1 / sp1) * s1 - rb1;
                term = r0 * r0 + r1 * r1;
            }
            term = wave_sum<T>(term);
            if (lane == 0) gstore_col(rs, colb(e, rb) + (uint32_t)(CPR + w) * 16, echunk(term, e), xl);
        }
        if (head) {
            spsh[0][r_cc] = s0;
            spsh[1][r_cc] = s1;
            gstore_col(rs, colb(e, rb) + (uint32_t)r_cc * 16, dchunk(s0, s1, e, bad), xl);
        }
        deadline = __builtin_amdgcn_s_memrealtime() + p.timeout_ticks;
        return ok;
    };
    // hop B (per wave): S[e - 1] of this wave's 32 chunks -> v into vcur[w]; wave 0 also
    // (need) the error terms of the nred reducers -> its tile's error partial.  Returns
    // bit 0 = producer flag, 1 = stall, 2 = bad v (this wave's columns only).
    // hop B of one chunk ch of this wave's stripe: S[e - 1] -> v of its two columns into
    // vcur[w]; returns bit 0 = producer flag, 1 = stall, 2 = bad v
    auto hop_v = [&](int e, int ch) -> int {
        int fl = 0;
        const uint32_t off = colb(e, ch / CPR) + (uint32_t)(ch & (CPR - 1)) * 16;
        I4 x;
        if (!poll64<false>(rs, off, (unsigned)e, deadline, x)) fl |= 2;
        fl |= dchunk_flag(x);
        const T s0 = dchunk_v0(x), s1 = dchunk_v1(x);
        const D2 bb = *reinterpret_cast<const D2*>(&bsh[2 * ch]);
        const T v0n = bb[0] / s0, v1n = bb[1] / s1;
        if (s0 == 0.0 || !finite_val(v0n) || s1 == 0.0 || !finite_val(v1n)) fl |= 4;
        *reinterpret_cast<D2*>(&vcur[w][2 * (ch - 32 * w)]) = D2{v0n, v1n};
        return fl;
    };
    // wave 0 on check iterations: the 8 error slots of each of the nred reducers (lane l
    // sums slots l + 64 k) -> this tile's error partial; returns bit 1 on a stall
    auto hop_err = [&](int e, T& sE) -> int {
        int fl = 0;
        T ep = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int q = lane + 64 * k;
            if (q < 8 * nred) {
                I4 x;
                if (!poll64<true>(rs, colb(e, q >> 3) + (uint32_t)(CPR + (q & 7)) * 16, (unsigned)e, deadline, x))
                    fl |= 2;
                ep += echunk_v(x);
            }
        }
        sE = wave_sum<T>(ep);
        return fl;
    };
    // hop B of the whole stripe (the post-loop check): returns the wave's flags
    auto gather_b = [&](int e, bool need, T& sE) -> int {
        int fl = 0;
        if (lane < 32) fl = hop_v(e, hch);
        if (w == 0 && need) fl |= hop_err(e, sE);
        // the wave's own LDS writes complete before its reads (in-order LDS per wave); the
        // clobber keeps the compiler from moving the reads of vcur above the writes
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const int wf = __any(fl & 1) ? 1 : 0, ws = __any(fl & 2) ? 2 : 0, wb = __any(fl & 4) ? 4 : 0;
        return wf | ws | wb;
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
        tot = ev;
        return __all(ok);
    };
    auto to_err = [&](T e) -> double { return p.err_squared ? e : sqrt(e); };
    auto stop_ok = [&](double err) -> bool { return p.err_squared ? !(err > p.stop_thr) : (err < p.stop_thr); };

    // ---- prologue: S[0] = K^T u0 (epoch 1)
    {
        T uu[NA];
#pragma unroll
        for (int a = 0; a < NA; ++a) uu[a] = u0;
        col_publish(uu, 1, 0);
    }
    int last_good = -1, niter = 0, status = OTF_SK_MAX_ITER, brk = -1, n_err = 0;
    bool done = false;
    if (!reduce(1, false) && lane == 0) s_ep[1] = 1;
    int chk = 0;
    T sE = 0;

    for (int it = 0; it < p.max_iter; ++it) {
        asm volatile("" : "+v"(tid), "+v"(lane));
        const int e = it + 1;
        const bool check = it >= 1 && chk == 0;
        OTF_M64ST(it, 0);
        if (it >= 1) chk = chk + 1 == p.check_every ? 0 : chk + 1;
        // hop B (this wave's 32 chunks, all in flight), then the row partials K v of the
        // lane's 8 rows over its 16 columns and the 4 lanes of a row (bits 5, 4: lane
        // (b5, b4) ends with rows a = 4 b5 + 2 b4 + 0, 1).  (Polling block by block and
        // summing each block as it arrives needed ~80 more spilled registers.)
        {
            {
                const int fl = gather_b(e, check, sE);
                if (lane == 0) {
                    if (fl & 2) s_ep[1] = e;
                    if (fl & 1) s_ep[2] = e;
                    if (fl & 4) s_ep[3] = e;
                }
            }
            OTF_M64ST(it, 1);
            T pr[NA];
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                const D2 va = *reinterpret_cast<const D2*>(&vcur[w][16 * b + 4 * g]);
                const D2 vb = *reinterpret_cast<const D2*>(&vcur[w][16 * b + 4 * g + 2]);
#pragma unroll
                for (int a = 0; a < NA; ++a) {
                    const D2 k0 = kget(a, b, 0), k1 = kget(a, b, 1);
                    T s = b == 0 ? k0[0] * va[0] : fma(k0[0], va[0], pr[a]);
                    s = fma(k0[1], va[1], s);
                    s = fma(k1[0], vb[0], s);
                    pr[a] = fma(k1[1], vb[1], s);
                }
            }
            T y[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) y[k] = swap_sum<32>(pr[k], pr[k + 4]);
            const T z0 = swap_sum<16>(y[0], y[2]), z1 = swap_sum<16>(y[1], y[3]);
            const int a0 = 4 * (lane >> 5) + 2 * ((lane >> 4) & 1);
            rowbuf[w][rr + 16 * a0] = z0;
            rowbuf[w][rr + 16 * a0 + 16] = z1;
        }
        OTF_M64ST(it, 2);
        __syncthreads();  // B1
        // every completed barrier re-arms the stall deadline (a stall, not a long solve,
        // times out)
        deadline = __builtin_amdgcn_s_memrealtime() + p.timeout_ticks;
        if (s_ep[1] == e) { status = OTF_SK_TIMEOUT; done = true; break; }
        if (s_ep[2] == e) {
            last_good = it - 2; niter = it - 1; status = OTF_SK_NUMERICAL_BREAK; brk = it - 1;
            done = true;
            break;
        }
        const int vbad_cb = s_ep[3] == e ? 1 : 0;
        // the tile's 128 row partials over its 512 columns (the 8 stripes in wave order):
        // wave w publishes chunks 8 w .. 8 w + 7, the ones its own lanes gather below
        if (lane < 8) {
            const int c = 8 * w + lane;
            D2 s = *reinterpret_cast<const D2*>(&rowbuf[0][2 * c]);
#pragma unroll
            for (int ww = 1; ww < NW; ++ww) s += *reinterpret_cast<const D2*>(&rowbuf[ww][2 * c]);
            gstore(rs, rowx(e, cb) + (uint32_t)c * 16, dchunk(s[0], s[1], e, vbad_cb));
        }
        if (w == 0 && check && lane == 8) gstore(rs, rowx(e, cb) + 64 * 16, echunk(sE, e));
        OTF_M64ST(it, 3);
        // row hop: the ncb members' chunk gc (lane (gc, gq): member gq), summed over the
        // 8 lanes in a fixed order -> u of rows 2 gc, 2 gc + 1
        {
            I4 x = I4{0, 0, 0, 0};
            int stall = 0;
            const bool act = gq < ncb;
            if (act && !poll64<false>(rs, rowx(e, gq) + (uint32_t)gc * 16, (unsigned)e, deadline, x)) stall = 1;
            T th0 = act ? dchunk_v0(x) : 0.0, th1 = act ? dchunk_v1(x) : 0.0;
            const int vb = act && dchunk_flag(x);
            th0 += dpp_lane<0xB1>(th0);
            th1 += dpp_lane<0xB1>(th1);
            th0 += dpp_lane<0x4E>(th0);
            th1 += dpp_lane<0x4E>(th1);
            th0 += dpp_lane<0x141>(th0);
            th1 += dpp_lane<0x141>(th1);
            const D2 ia = *reinterpret_cast<const D2*>(&iash[2 * gc]);
            const T un0 = 1.0 / (th0 * ia[0]), un1 = 1.0 / (th1 * ia[1]);
            const bool bu = gq == 0 && (!finite_val(un0) || !finite_val(un1));
            if (gq == 0) {
                uhist[it & 1][upos(2 * gc)] = un0;
                uhist[it & 1][upos(2 * gc + 1)] = un1;
            }
            if (w == 0 && check) {
                T ev;
                if (!err_total(e, ev)) stall = 1;
                if (lane == 0) s_err = ev;
            }
            const bool any_st = __any(stall), any_vb = __any(vb), any_bu = __any(bu);
            if (lane == 0) {
                if (any_st) s_ep[4] = it;
                if (any_vb) s_ep[5] = it;
                if (any_bu) s_ep[0] = it;
            }
        }
        OTF_M64ST(it, 4);
        __syncthreads();  // B2
        deadline = __builtin_amdgcn_s_memrealtime() + p.timeout_ticks;
        OTF_M64ST(it, 5);
        if (s_ep[4] == it) { status = OTF_SK_TIMEOUT; done = true; break; }
        double err = 0.0;
        int dec = 0;
        if (check) {
            err = to_err(s_err);
            if (stop_ok(err)) dec = 1;
            if (lead) p.errlog[n_err] = err;
            ++n_err;
        }
        if (dec == 0 && s_ep[5] == it) dec = 2;
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
        // v of this iteration into the history (this wave's stripe)
        if (lane < 32)
            *reinterpret_cast<D2*>(&vhist[it & 1][cw + 2 * lane]) = *reinterpret_cast<const D2*>(&vcur[w][2 * lane]);
        {
            T uu[NA];
#pragma unroll
            for (int q = 0; q < NA; q += 2) {
                const D2 t2 = *reinterpret_cast<const D2*>(&uhist[it & 1][rr * 8 + q]);
                uu[q] = t2[0];
                uu[q + 1] = t2[1];
            }
            col_publish(uu, e + 1, s_ep[0] == it ? 1 : 0);
        }
        OTF_M64ST(it, 6);
        if (!reduce(e + 1, chk == 0) && lane == 0) s_ep[1] = e + 1;
        OTF_M64ST(it, 7);
    }
    if (!done && p.max_iter > 0) {
        const int it = p.max_iter - 1;
        const int e = p.max_iter + 1;
        const bool need = (it % p.check_every) == 0;
        {
            const int fl = gather_b(e, need, sE);
            if (lane == 0) {
                if (fl & 2) s_ep[1] = e;
                if (fl & 1) s_ep[2] = e;
            }
        }
        __syncthreads();
        if (s_ep[1] == e) {
            status = OTF_SK_TIMEOUT;
        } else if (s_ep[2] == e) {
            last_good = it - 1; niter = it; status = OTF_SK_NUMERICAL_BREAK; brk = it;
        } else {
            last_good = it; niter = it;
            if (need && w == 0) {
                // only wave 0 (the lead's) needs the total: it writes the log and the status
                if (lane == 0) gstore(rs, rowx(e, cb) + 64 * 16, echunk(sE, e));
                T errv;
                if (!err_total(e, errv)) {
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
    if (cb == 0 && tid < TR) p.u_out[row0 + tid] = last_good >= 0 ? uhist[hs][upos(tid)] : u0;
    if (rb == 0 && tid < TC / 2)
        *reinterpret_cast<D2*>(p.v_out + col0 + 2 * tid) =
            last_good >= 0 ? *reinterpret_cast<const D2*>(&vhist[hs][2 * tid]) : D2{v0, v0};
    if (p.P) {
        TP* P = (TP*)p.P;
        T uo[NA];
#pragma unroll
        for (int a = 0; a < NA; ++a) uo[a] = last_good >= 0 ? uhist[hs][rr * 8 + a] : u0;
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const D2 va = last_good >= 0 ? *reinterpret_cast<const D2*>(&vhist[hs][cw + 16 * b + 4 * g]) : D2{v0, v0};
            const D2 vb = last_good >= 0 ? *reinterpret_cast<const D2*>(&vhist[hs][cw + 16 * b + 4 * g + 2]) : D2{v0, v0};
#pragma unroll
            for (int a = 0; a < NA; ++a) {
                TP* prow = P + (int64_t)(row0 + rr + 16 * a) * p.ldp + col0 + cw + 16 * b + 4 * g;
                const D2 o0 = (uo[a] * kget(a, b, 0)) * va, o1 = (uo[a] * kget(a, b, 1)) * vb;
                if constexpr (sizeof(TP) == 8) {
                    *reinterpret_cast<D2*>(prow) = o0;
                    *reinterpret_cast<D2*>(prow + 2) = o1;
                } else {
                    using F4 = __attribute__((ext_vector_type(4))) float;
                    *reinterpret_cast<F4*>(prow) = F4{(float)o0[0], (float)o0[1], (float)o1[0], (float)o1[1]};
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

template <typename TP, bool PW>
hipError_t launch_mesh64_t(int grid, SkMesh64Args& p, hipStream_t s) {
    void* args[] = {&p};
    const void* k = (p.nrb == 32 && p.ncb == 8) ? (const void*)sk_mesh64_kernel<TP, 32, 8, PW>
                                                : (const void*)sk_mesh64_kernel<TP, 0, 0, PW>;
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 512, 0);
    if (e != hipSuccess) return e;
    if (per_cu < 1 || grid > per_cu * device_cu_count()) return hipErrorCooperativeLaunchTooLarge;
    return hipLaunchKernel(k, dim3(grid), dim3(512), args, 0, s);
}


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
    s.bstride = (uint32_t)((s.cpr + kM64NW) * 16 + 255) / 256 * 256;  // S chunks + 8 error slots
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

bool mesh64_pairwise_ok(int64_t n, int64_t m, int64_t d, int64_t ldx, int64_t ldy, const void* X, const void* Y) {
    return mesh64_supported(n, m) && d >= 16 && d % 16 == 0 && ldx >= d && ldy >= d && ldx % 4 == 0 &&
           ldy % 4 == 0 && (uintptr_t)X % 16 == 0 && (uintptr_t)Y % 16 == 0 && n * ldx * 4 < (1ll << 31) &&
           m * ldy * 4 < (1ll << 31);
}

hipError_t run_mesh64(const double* C, int64_t ldc, int n, int m, const double* a_pad, const double* b_pad,
                      const double* cost_scale, const otf_sinkhorn_opts& o, void* region, double* u_out,
                      double* v_out, void* P_out, int64_t ldp, int P_dtype, otf_sinkhorn_info* info,
                      double* errlog, bool zeroed, hipStream_t s, const PairwiseF64* pw) {
    if (!mesh64_supported(n, m) || !region) return hipErrorInvalidValue;
    if (!pw && (ldc % 2 != 0 || ((uintptr_t)C % 16) != 0)) return hipErrorInvalidValue;
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
    if (pw) {
        p.pw = *pw;
        p.cost_scale = nullptr;
        if (P_out && P_dtype == OTF_F32) return launch_mesh64_t<float, true>(grid, p, s);
        return launch_mesh64_t<double, true>(grid, p, s);
    }
    if (P_out && P_dtype == OTF_F32) return launch_mesh64_t<float, false>(grid, p, s);
    return launch_mesh64_t<double, false>(grid, p, s);
}

}  // namespace otf
