// otf_mesh.hip — Sinkhorn on a mesh of register-resident K tiles with no per-iteration
// device-wide barrier and no float atomics (OTF_ENGINE_MESH), POT flavour, float32
// compute.  (One grid barrier per solve: the XCC registration before the first iteration.)
//
// Replaces ot.sinkhorn (POT 0.9.6 sinkhorn_knopp, MRI_PET_OT_nojax.py:143 /
// perturbot/perturbot/match/utils.py:6-115) for the coupled problems whose K fits the
// register files of the chip: the headline N = 4096 metric config (BASELINE.json
// configs[1]) and every shape of 4..64 row tiles x 1..8 column tiles.
//
// Workgroup (rb, cb) keeps the 128-row x 512-column tile (rb, cb) of K = exp(-C/reg)
// in registers for the whole solve (8 waves x 16 rows, every lane 8 columns), as the
// tiled engine does.  Per iteration Sinkhorn needs two reductions: the row sums K v
// over the ncb column tiles of a row block, and the column sums K^T u over the nrb row
// blocks of a column tile.  The tiled engine does the first through a write-through
// exchange + arrival counter and the second through float atomics + a grid barrier +
// a re-read: five memory-side hand-offs, 8.9 us per iteration at N = 4096.  Here all
// traffic is epoch-tagged granules (R2 form, cdna_hip_programming.md Guideline 16:
// 8-byte {value, tag} granules, two per 16-B write-through store, consumers poll the
// data itself until every tag carries the epoch they wait for -- no fence, no counter,
// no barrier), in three hops per iteration:
//
//   row hop  every WAVE publishes its 16 row partials (8 chunks) and gathers the same
//            rows' partials of the ncb members of its row block (one chunk per lane),
//            sums them in a fixed butterfly order -> u for its rows;
//   hop A    every workgroup publishes its 512 column partials K_tile^T u (256 chunks);
//   reduce   workgroup rb of column tile cb is the REDUCER of chunks [rb*CPR, ..+CPR):
//            one wave gathers them from the nrb producers and sums them in a fixed
//            order, then publishes the column sums S (hop B) -- plus its share of the
//            marginal error of the previous iterate (POT's err, utils.py:83-90);
//   hop B    every workgroup gathers the 512 sums of its column tile from the
//            reducers -> v = b / S.
//
// Every sum has one fixed order, so all members of a group hold bit-identical values
// and the result is bitwise reproducible run to run.  POT's decisions travel in the tag
// bits and the extra error chunks, so every workgroup takes them at the same point:
//   * a zero / non-finite v of iteration it (known to a column tile after hop B) rides
//     in the row-hop tags of it -> everyone knows it after the row hop of it;
//   * a non-finite u of iteration it (known to a row block after the row hop) rides in
//     the hop-A tags -> reducers -> hop-B tags -> everyone knows it at hop B of it + 1;
//   * the marginal error of iterate it - 1 = sum of the reducers' terms (hop B of it),
//     summed per column tile, then over column tiles in the row hop of it.
// which reproduces POT's order (break of iterate k before its error check, error of
// k before the break test of k + 1) with the same (last_good, niter, break_iter).
//
// Double buffering by epoch parity is enough for every hop: a member publishes epoch
// e + 2 only after its own gather of e + 1, which needed every member's publish of
// e + 1, which each made after finishing its gather of e.  Every poll is bounded by
// s_memrealtime (re-armed after each completed gather): a stall ends in OTF_SK_TIMEOUT.
#include "otf_persist.h"

namespace otf {
namespace {

constexpr int kMeshNW = 8;      // waves per workgroup
constexpr int kMeshRW = 16;     // rows per wave
constexpr int kMeshTR = 128;    // rows per tile
constexpr int kMeshTC = 512;    // columns per tile
constexpr int kMeshNCH = 256;   // 16-B chunks (two {value, tag} granules) per 512 columns
constexpr int kMeshMaxNcb = 16; // row hop: ncb members x 8 chunks <= two chunks per lane
constexpr int kMeshXccNcb = 8;   // the XCC-local column path: one column tile per XCC
constexpr int kMeshMinNrb = 4;  // reducer chunks per workgroup (CPR) <= 64
constexpr int kMeshMaxNrb = 64; // hop-B error chunks: one per lane of one wave
constexpr uint32_t kRowStride = 1280;  // per producer: 64 row chunks + the error chunk
constexpr uint32_t kColStride = 4096;  // per producer: 256 column chunks

struct SkMeshArgs {
    const void* C;
    int64_t ldc;
    int n, m;
    const float* a;  // padded marginals (zero past n / m)
    const float* b;
    const float* cost_scale;
    double reg;
    int max_iter, check_every, err_squared;
    double stop_thr;
    void* gran;  // granule region, zeroed per solve
    uint32_t off_row, off_cola, off_colb, bstride;
    int nrb, ncb, cpr, xcc_local;
    int* xreg;  // [8 x 64] workgroups per XCC (registration), then the flat barrier word
    otf_sinkhorn_info* info;
    double* errlog;
    float* u_out;
    float* v_out;
    void* P;
    int64_t ldp;
    unsigned long long timeout_ticks;
    unsigned long long reg_ticks;  // the first wait (registration / first hop)
    ShiftArgs sh;                  // shifted kernel (SH instances): offsets + initial scalings
    // cross-rank form (XR instances, otf_sinkhorn_xsweep on a shape the mesh takes): these
    // are this rank's rows of a problem of n_total rows; after summing its producers every
    // reducer stores its chunks' partial into every rank's exchange buffer (xr[r], the
    // peers' buffers as mapped here; [2 solve parities][2 epoch parities][8 ranks][mc]
    // chunks, the xsweep layout) and sums the world's partials in rank order
    int n_total, xrank, xworld, xpar, mc;
    unsigned xep;  // epoch base of this solve on the exchange (the same on every rank)
    unsigned char* xr[8];
    PairwiseF32 pw;  // PW instances: the cost tile built in the prologue (otf_persist.h)
};

// Diagnostic build only (-DOTF_MESH_STAMPS, tools/stamps_mesh.hip): per-hop wall-clock
// stamps keyed by the workgroup's ROLE (rb * ncb + cb), so the tool can pair every
// consumer with its producers and split a hop into its latency and the producers' skew.
#ifdef OTF_MESH_STAMPS
__device__ unsigned long long g_mstamps[256 * 16 * 16];
__device__ int g_mrole[256 * 4];
// the stamp buffer's address lives in a VGPR pair (set once): a stamp is then one
// s_memrealtime + one store, not a GOT load per stamp (two serial scalar round trips)
#define OTF_MSTAMP(it, slot, who)                                                            \
    do {                                                                                     \
        if (threadIdx.x == (who) && (it) >= 0 && (it) < 16 && rb * ncb + cb < 256)           \
            mst_base[((rb * ncb + cb) * 16 + (it)) * 16 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define OTF_MSTAMP(it, slot, who) \
    do {                          \
    } while (0)
#endif

using I4 = __attribute__((ext_vector_type(4))) int;
// Waves that share the reducer's gather (1, 2 or 4): each polls KQ / RW producers per lane,
// the last to finish (an LDS ticket) adds the partials in producer order and publishes
#ifndef OTF_MESH_RED_WAVES
#define OTF_MESH_RED_WAVES 1
#endif
// s_sleep units between polls of a granule that has not arrived (64 clocks each)
#ifndef OTF_MESH_SLEEP
#define OTF_MESH_SLEEP 1
#endif
// reducer polls: reload only the producers not yet seen (1) or all of them (0)
#ifndef OTF_MESH_RED_PEND
#define OTF_MESH_RED_PEND 0
#endif
using F2 = __attribute__((ext_vector_type(2))) float;

constexpr int pow2_at_least(int x) { return x <= 1 ? 1 : 2 * pow2_at_least((x + 1) / 2); }

// ---- PW prologue (sk_mesh_kernel<..., PW = true>, otf_sinkhorn_pairwise_f32; r06) ----------
// The workgroup's 128 x 512 tile of C = |x|^2 + |y|^2 - 2 x.y (MRI_PET_OT_nojax.py:70-75)
// built where its K will live instead of read from a cost the cost kernel wrote, in two column
// halves of 128 x 256: eight waves of 64 rows x 64 columns (wave w: rows 64 (w >> 2), columns
// 64 (w & 3) of the half) on v_mfma_f32_16x16x32_f16, x.y = hi.hi + hi.lo + lo.hi of the
// split-fp16 images, with the Y fragment as the A operand -- per 16 x 16 block the MFMA
// sequence and the epilogue of cost_big16_kernel (otf_cost.hip), so every cost value is
// bitwise the two-call path's.  The 32-deep stages are double-buffered in LDS (the next
// stage's images in registers during this stage's MFMAs, one barrier a stage); each half then
// moves to the mesh's K layout (wave w: 16 rows x 8 columns a lane) through LDS; one atomic
// max per workgroup + a flat barrier give the grid max(C), then K = exp(-C / (reg max)) in place.
constexpr int kPwK = 32;                        // K per stage (one 16x16x32 MFMA)
constexpr int kPwRS = 264;                      // re-layout row pitch (floats): 2-way writes
constexpr size_t kPwLds = (size_t)kMeshTR * kPwRS * 4;  // 135 168 B (a half's stages take 96 KiB of it)
constexpr int kMeshMaxBar = 9 * 64, kMeshMaxWord = 10 * 64;  // int offsets in xreg
using H8 = __attribute__((ext_vector_type(8))) _Float16;
using F4 = __attribute__((ext_vector_type(4))) float;
using U4 = __attribute__((ext_vector_type(4))) unsigned int;
// 16-B chunk kc of a 64-B stage row, XOR-permuted by the row quad (otf_cost.hip g16swz)
__device__ __forceinline__ int pw_swz(int row, int kc) {
    return row * kPwK + ((kc ^ ((0x78 >> (2 * ((row >> 2) & 3))) & 3)) << 3);
}

template <int R, int G>
__device__ __forceinline__ bool pw_cost_tile32(const SkMeshArgs& p, F2 (&kv)[R][G][2], unsigned char* lds, int rb,
                                               int cb, int target, bool lead, unsigned long long& deadline,
                                               int* s_flag, float* s_wmx, int* abandon) {
    static_assert(R == 16 && G == 2, "the mesh's K layout: 16 rows x 2 x 4 columns a lane");
    const PairwiseF32& q = p.pw;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w >> 2, wn = w & 3;
    const int row0 = rb * kMeshTR, col0 = cb * kMeshTC;
    constexpr int HC = kMeshTC / 2;                       // 256 columns per half
    constexpr int AS = kMeshTR * kPwK, BS = HC * kPwK;    // halves per image and stage buffer
    _Float16* As = reinterpret_cast<_Float16*>(lds);      // [2 buffers][2 images][128 x 32]
    _Float16* Bs = As + 4 * AS;                           // [2 buffers][2 images][256 x 32]
    const __amdgpu_buffer_rsrc_t rxh = __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16*>(q.Xh), 0, (int)q.xbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rxl = __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16*>(q.Xl), 0, (int)q.xbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t ryh = __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16*>(q.Yh), 0, (int)q.ybytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t ryl = __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16*>(q.Yl), 0, (int)q.ybytes, 0x00020000);
    // staging: X chunk (row tid >> 2, 16-B chunk tid & 3) and Y chunks tid + 512 c of a stage
    const int xr = tid >> 2, xk = tid & 3;
    const uint32_t xo = (uint32_t)(((int64_t)(row0 + xr) * q.ldh + 8 * xk) * 2);
    const int nk = q.kpad / kPwK;
    const int kc = lane >> 4;
    const int rr = wm * 64 + (lane & 15);
    float lmax = 0.f;
    float* st = reinterpret_cast<float*>(lds);
    // the tile in two column halves (operand stages double-buffered in LDS, one barrier a
    // stage); each half moves to the K layout (kv[.][h]) before the next one is built
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        uint32_t yo[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int ch = tid + 512 * c;
            yo[c] = (uint32_t)(((int64_t)(col0 + HC * h + (ch >> 2)) * q.ldh + 8 * (ch & 3)) * 2);
        }
        U4 sx[2], sy[2][2];
        auto gl = [&](int k0) {
            const uint32_t kb = (uint32_t)k0 * 2u;
            sx[0] = __builtin_bit_cast(U4, __builtin_amdgcn_raw_buffer_load_b128(rxh, xo, kb, 0));
            sx[1] = __builtin_bit_cast(U4, __builtin_amdgcn_raw_buffer_load_b128(rxl, xo, kb, 0));
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                sy[c][0] = __builtin_bit_cast(U4, __builtin_amdgcn_raw_buffer_load_b128(ryh, yo[c], kb, 0));
                sy[c][1] = __builtin_bit_cast(U4, __builtin_amdgcn_raw_buffer_load_b128(ryl, yo[c], kb, 0));
            }
        };
        auto ls = [&](int buf) {
#pragma unroll
            for (int img = 0; img < 2; ++img) {
                *reinterpret_cast<U4*>(&As[(2 * buf + img) * AS + pw_swz(xr, xk)]) = sx[img];
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const int ch = tid + 512 * c;
                    *reinterpret_cast<U4*>(&Bs[(2 * buf + img) * BS + pw_swz(ch >> 2, ch & 3)]) = sy[c][img];
                }
            }
        };
        F4 acc[4][4];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) acc[a][b] = F4{0.f, 0.f, 0.f, 0.f};
        gl(0);
        ls(0);
        __syncthreads();
        for (int kt = 0; kt < nk; ++kt) {
            const int buf = kt & 1;
            if (kt + 1 < nk) gl((kt + 1) * kPwK);
            const _Float16* A0 = As + 2 * buf * AS;
            const _Float16* B0 = Bs + 2 * buf * BS;
            H8 ah[4], al[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int ar = wm * 64 + t * 16 + (lane & 15);
                ah[t] = *reinterpret_cast<const H8*>(&A0[pw_swz(ar, kc)]);
                al[t] = *reinterpret_cast<const H8*>(&A0[AS + pw_swz(ar, kc)]);
            }
#pragma unroll
            for (int nj = 0; nj < 4; ++nj) {
                const int br = wn * 64 + nj * 16 + (lane & 15);
                const H8 bh = *reinterpret_cast<const H8*>(&B0[pw_swz(br, kc)]);
                const H8 bl = *reinterpret_cast<const H8*>(&B0[BS + pw_swz(br, kc)]);
#pragma unroll
                for (int mi = 0; mi < 4; ++mi) {
                    // cost_big16_kernel's order: hi.lo, lo.hi, then hi.hi into the same block
                    acc[mi][nj] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh, al[mi], acc[mi][nj], 0, 0, 0);
                    acc[mi][nj] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bl, ah[mi], acc[mi][nj], 0, 0, 0);
                    acc[mi][nj] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh, ah[mi], acc[mi][nj], 0, 0, 0);
                }
            }
            if (kt + 1 < nk) ls(buf ^ 1);
            __syncthreads();
        }
        // epilogue (cost_big16's): lane holds cost row rr + 16 mi at half columns cc + 16 nj + e
        const int cc = wn * 64 + 4 * (lane >> 4);
#pragma unroll
        for (int nj = 0; nj < 4; ++nj) {
            const int cl = HC * h + cc + nj * 16;
            const F4 ys4 = *reinterpret_cast<const F4*>(q.ys + col0 + cl);
            const F4 yy4 = *reinterpret_cast<const F4*>(q.yy + col0 + cl);
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) {
                const int rl = rr + mi * 16;
                const float a = -2.f * q.xs[row0 + rl], b = q.xx[row0 + rl];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float c = fmaf(acc[mi][nj][e], a * ys4[e], b + yy4[e]);
                    c = fmaxf(c, 0.f);
                    if (q.euclid) c = sqrtf(c);
                    acc[mi][nj][e] = c;
                    lmax = fmaxf(lmax, c);
                }
                *reinterpret_cast<F4*>(&st[rl * kPwRS + cc + 16 * nj]) = acc[mi][nj];
            }
        }
        __syncthreads();
        // to the K layout: wave w's 16 rows, four columns 4 lane + 256 h a lane
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const F4 v = *reinterpret_cast<const F4*>(&st[(16 * w + r) * kPwRS + 4 * lane]);
            kv[r][h][0] = F2{v[0], v[1]};
            kv[r][h][1] = F2{v[2], v[3]};
        }
        __syncthreads();  // the staging area is the next half's operand buffers
    }
    // the grid's max (costs >= 0: the bit patterns order like the values)
    lmax = wave_max(lmax);
    if (lane == 0) s_wmx[w] = lmax;
    __syncthreads();
    if (tid == 0) {
        float mx = s_wmx[0];
        for (int ww = 1; ww < kMeshNW; ++ww) mx = fmaxf(mx, s_wmx[ww]);
        __hip_atomic_fetch_max(reinterpret_cast<unsigned int*>(p.xreg + kMeshMaxWord), __float_as_uint(mx),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // blockIdx roles (no registration barrier ran): the launch's first device-wide wait gives
    // up as a registration give-up (abandon = info->stalled), so the relay fallback solves
    if (!grid_barrier(p.xreg + kMeshMaxBar, target, deadline, p.timeout_ticks, s_flag, abandon)) return false;
    const float cmax = __uint_as_float(__hip_atomic_load(reinterpret_cast<unsigned int*>(p.xreg + kMeshMaxWord),
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (lead && q.cmax_out) *q.cmax_out = cmax;
    // the two-call path's K: ks = -unit / reg / cost_scale in float64, then float32
    const double cinv = q.scale ? 1.0 / (double)cmax : 1.0;
    const float ks = (float)(-exp_unit<float>() / p.reg * cinv);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int hh = 0; hh < 2; ++hh)
                kv[r][g][hh] = F2{fast_exp(kv[r][g][hh][0] * ks), fast_exp(kv[r][g][hh][1] * ks)};
    return true;
}

// KQ: reducer loads per lane, ceil(nrb * CPR / 64): 4 when nrb is a power of two
// (nrb * CPR = 256), up to 8 otherwise.
// SNRB, SNCB: the shape compiled in (0 = read from the arguments).  A compiled-in shape
// is a mesh of WHOLE tiles (n = SNRB * 128, m = SNCB * 512): every row / column bound
// test and every derived count folds away, which also frees the scalar registers whose
// spills (v_readlane / v_writelane per branch) lengthened every phase of the generic form.
// SH: the shifted POT kernel K~ = 2^(C ks + A_i + B_j) (otf_persist.h ShiftArgs), formed
// once in the prologue like K; the loop is unchanged.
// PW: the cost tile is built in the prologue from the split-fp16 images (p.pw) instead of read
// from C (pw_cost_tile32 above).
template <typename CT, typename TP, int KQ, int SNRB, int SNCB, bool SH, bool XR = false, bool PW = false>
__global__ __launch_bounds__(512) void sk_mesh_kernel(SkMeshArgs p) {
    static_assert(!(PW && (SH || XR)), "pairwise form: the plain single-rank POT kernel");
    using T = float;
    constexpr int G = 2, VEC = 4, R = kMeshRW, NW = kMeshNW, TR = kMeshTR, TC = kMeshTC;
    using V = Vec<float>::type;
    using VP = __attribute__((ext_vector_type(VEC))) TP;
    __shared__ __attribute__((aligned(16))) T colbuf[NW][TC];
    __shared__ __attribute__((aligned(16))) T vcur[TC];      // v = b / S of this tile's columns
    __shared__ __attribute__((aligned(16))) T vhist[2][TC];  // v by iteration parity
    __shared__ T uhist[2][TR];
    __shared__ T s_E;  // this column tile's error partial (hop B)
    // workgroup-wide flags without a reduction: a raised flag holds the KEY (epoch or
    // iteration) of the step that raised it, compared after the barrier (keys only grow)
    // [0] non-finite u in this workgroup (iteration key), [1] hop-B stall, [2] hop-B
    // producer flag (non-finite u of the previous iteration), [3] zero / non-finite v
    // (epoch keys), [4] row-hop stall (iteration key)
    __shared__ int s_ep[5];
    constexpr int RW = OTF_MESH_RED_WAVES, KQW = KQ / RW;
    static_assert(KQ % RW == 0, "reducer waves must divide the reducer loads");
    __shared__ F2 red_s[RW][kWave];   // per-wave partial sums of the reducer's lanes
    __shared__ int red_f[RW][kWave];  // and their producer flags
    __shared__ F2 red_sp[kWave];      // previous sums S[k - 1] of the reducer's lanes
    __shared__ int red_cnt;           // reducer-wave ticket of this epoch
    // PW: the prologue's operand stages, then the cost tile's re-layout (kPwLds bytes)
    __shared__ __attribute__((aligned(16))) unsigned char pwb[PW ? kPwLds : 16];
    __shared__ float pw_wmx[kMeshNW];
    __shared__ int pw_flag;
    int tid = threadIdx.x, lane = tid & 63;
    const int w = (int)threadIdx.x >> 6;
    unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + p.reg_ticks;
    constexpr bool FULL = SNRB != 0 && SNCB != 0;
    const int nrb = FULL ? SNRB : p.nrb, ncb = FULL ? SNCB : p.ncb;
    const int CPR = FULL ? pow2_at_least((kMeshNCH + SNRB - 1) / (SNRB > 0 ? SNRB : 1)) : p.cpr;
    const int n_ = FULL ? SNRB * TR : p.n, m_ = FULL ? SNCB * TC : p.m;
    auto row_in = [&](int r) -> bool { return FULL || r < n_; };
    auto col_in = [&](int c) -> bool { return FULL || c < m_; };

    // Tile of this workgroup.  XCC-local column path (p.xcc_local): every workgroup
    // registers on its XCC (the hardware id, not an assumed placement), one flat
    // barrier over the launch of 8 x nrb workgroups, and when ncb XCCs hold at least nrb
    // registrants each (N = 4096: 8 x 32, one workgroup per CU), column tile cb = the
    // rank of this XCC among them and row block rb = the registration slot (the surplus
    // leaves).  A column tile's hop A, reduce and
    // hop B then stay inside one XCC's L2, which is the point of coherence for all its
    // CUs: plain stores (L1 is write-through, the line stays in L2) read by L1-bypassing
    // sc1 loads -- the single-L2 protocol; only the cross-XCC hops (row hop, error
    // chunks) need write-through stores.  Measured 7.2 -> 5.7 us per iteration; with the
    // column tiles spread over XCCs the same plain stores are never seen (the solve ends
    // in OTF_SK_TIMEOUT), which is why roles follow the registration, never blockIdx.
    // Otherwise: blockIdx roles, every hop write-through.
    int rb = 0, cb = 0, xl = 0;
    if (p.xcc_local) {
        __shared__ int s_reg[4];
        const int xcd = xcc_id();
        if (tid == 0)
            s_reg[0] = __hip_atomic_fetch_add(p.xreg + xcd * 64, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool ok = grid_barrier(p.xreg + 8 * 64, gridDim.x, deadline, p.timeout_ticks, &s_reg[3],
                                     &p.info->stalled);
        if (tid == 0) {
            // the first ncb XCCs (by id) holding >= nrb registrants are the column tiles;
            // registrants beyond slot nrb - 1 and XCCs past the ncb-th leave
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
        // a registration that timed out (the grid was not co-resident in time) must not
        // go on with blockIdx roles while the workgroups that did see the barrier complete
        // take XCC roles: it reports the stall and leaves; the rest then stall on its
        // missing data and report it too -- never a plan from mixed roles
        if (!s_reg[3]) {
            if (tid == 0) mark_stalled(&p.info->stalled, kStallRegistration);
            return;
        }
        if (s_reg[1]) {
            if (s_reg[2] < 0 || s_reg[0] >= nrb) return;  // a surplus workgroup of the launch
            rb = s_reg[0];
            cb = s_reg[2];
            xl = 1;
        }
    }
    if (!xl) {
        const int bi = blockIdx.x;
        if (bi >= nrb * ncb) return;  // the launch's surplus (XCC mode launches 8 x nrb)
        rb = bi / ncb;
        cb = bi % ncb;
    }
    const bool lead = (rb == 0 && cb == 0 && tid == 0);  // writes info and the error log
#ifdef OTF_MESH_STAMPS
    unsigned long long* mst_base = g_mstamps;
    asm volatile("" : "+v"(mst_base));
    if (tid == 0 && rb * ncb + cb < 256) {
        g_mrole[(rb * ncb + cb) * 4 + 0] = rb;
        g_mrole[(rb * ncb + cb) * 4 + 1] = cb;
        g_mrole[(rb * ncb + cb) * 4 + 2] = xcc_id();
        g_mrole[(rb * ncb + cb) * 4 + 3] = 1 + ncb * 1000 + nrb * 100000;
    }
#endif
    const int row0 = rb * TR + w * R;
    const int col0 = cb * TC;
    const int ncols = FULL ? TC : (m_ - col0 < TC ? m_ - col0 : TC);
    const int nch = (ncols + 1) >> 1;          // chunks of this column tile
    const int nred = (nch + CPR - 1) / CPR;    // reducers of this column tile

    const double unit = exp_unit<T>();
    double cinv = 1.0;
    if (p.cost_scale) cinv = 1.0 / (double)p.cost_scale[0];
    const T ks = (T)(-unit / p.reg * cinv);

    // ---- K for this wave's 16 rows x this lane's 8 columns, once (0 outside C), as
    // pairs of adjacent columns: the row and column partials run on v_pk_fma_f32
    F2 kv[R][G][2];
    if constexpr (PW) {
        if (!pw_cost_tile32<R, G>(p, kv, pwb, rb, cb, nrb * ncb, lead, deadline, &pw_flag, pw_wmx,
                                  xl ? nullptr : &p.info->stalled)) {
            // the max barrier stalled: a mid-solve stall (OTF_SK_TIMEOUT; kept at the registration
            // give-up when the barrier gave up as one), every workgroup leaves
            if (tid == 0) {
                mark_stalled(&p.info->stalled, kStallMid);
                if (lead) p.info->status = OTF_SK_TIMEOUT;
            }
            return;
        }
    } else {
        int colc[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int c0 = col0 + (lane + kWave * g) * VEC;
            colc[g] = col_in(c0) ? c0 : 0;
        }
        const CT* crow = (const CT*)p.C + (int64_t)row0 * p.ldc;
        V shb[G];  // B of this lane's columns (SH)
#pragma unroll
        for (int g = 0; g < G; ++g) {
            shb[g] = V{0, 0, 0, 0};
            if (SH) shb[g] = *reinterpret_cast<const V*>(p.sh.B + colc[g]);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const CT* src = row_in(row0 + r) ? crow : (const CT*)p.C;
            const bool rok = row_in(row0 + r);
            const T sha = SH && rok ? p.sh.A[row0 + r] : (T)0;
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const V c = load_cost<T>(src + colc[g]);
                T e[VEC];
#pragma unroll
                for (int k = 0; k < VEC; ++k) {
                    const bool ok = rok && col_in(col0 + (lane + kWave * g) * VEC + k);
                    T z = c[k] * ks;
                    if (SH) z += sha + shb[g][k];
                    e[k] = ok ? fast_exp(z) : (T)0;
                }
                kv[r][g][0] = F2{e[0], e[1]};
                kv[r][g][1] = F2{e[2], e[3]};
            }
            crow += p.ldc;
        }
    }
    // 1 / a of the rows whose u this lane finishes: row (lane & 15) when the tile spans
    // whole rows, rows 2c, 2c + 1 (c = lane & 7) after a row hop
    auto inv_a = [&](int r) -> T { return (T)1 / p.a[row_in(r) ? r : n_ - 1]; };
    // rows 2c, 2c + 1 (c = lane >> 3) of the wave's 16: the chunk a lane group finishes
    const int rc = lane >> 3;
    const T ia_c0 = inv_a(row0 + 2 * rc), ia_c1 = inv_a(row0 + 2 * rc + 1);
    // hop-B consumer: chunk t = tid - 256 of this tile -> columns col0 + 2t, + 1
    T bch0 = 0, bch1 = 0;
    if (tid >= 256) {
        const int t = tid - 256;
        if (2 * t < ncols) bch0 = p.b[col0 + 2 * t];
        if (2 * t + 1 < ncols) bch1 = p.b[col0 + 2 * t + 1];
    }
    // reducer (wave 0): chunk cc = lane % CPR of this workgroup's range, producers
    // q = lane / CPR + LPC * k
    const int LPC = kWave / CPR;
    const int r_cc = lane & (CPR - 1), r_qlo = lane / CPR;
    const int r_ch = rb * CPR + r_cc;
    const bool r_ok = r_ch < nch;
    T rb0 = 0, rb1 = 0;  // target marginal of the reducer's two columns
    if (w < OTF_MESH_RED_WAVES && r_ok) {
        if (2 * r_ch < ncols) rb0 = p.b[col0 + 2 * r_ch];
        if (2 * r_ch + 1 < ncols) rb1 = p.b[col0 + 2 * r_ch + 1];
    }
    const bool rc0 = r_ok && 2 * r_ch < ncols, rc1 = r_ok && 2 * r_ch + 1 < ncols;
    T sp0 = 1, sp1 = 1;  // the reducer's previous sums S[k - 1]

    const T u0 = (T)1 / (T)(XR ? p.n_total : n_), v0 = (T)1 / (T)m_;
    if (tid < 5) s_ep[tid] = -1;
    if (tid < kWave) red_sp[tid] = F2{1.f, 1.f};
    if (tid == 0) red_cnt = 0;
    for (int q = tid; q < TC; q += blockDim.x) {
        vhist[0][q] = vhist[1][q] = v0;
        vcur[q] = 0;  // columns past m stay 0 (their K entries are 0 too)
    }
    if (tid < TR) uhist[0][tid] = uhist[1][tid] = u0;

    const __amdgpu_buffer_rsrc_t rs = sums_rsrc(p.gran);
    auto rowx = [&](int e, int q) -> uint32_t {
        return p.off_row + ((uint32_t)((e & 1) * nrb + rb) * (uint32_t)ncb + (uint32_t)q) * kRowStride;
    };
    auto cola = [&](int e, int q) -> uint32_t {
        return p.off_cola + ((uint32_t)((e & 1) * ncb + cb) * (uint32_t)nrb + (uint32_t)q) * kColStride;
    };
    auto colb = [&](int e, int j) -> uint32_t {
        return p.off_colb + ((uint32_t)((e & 1) * ncb + cb) * (uint32_t)nrb + (uint32_t)j) * p.bstride;
    };

    // hop A: this workgroup's column partials K_tile^T wr (the per-wave partials are in
    // colbuf, after the barrier), epoch e; flag = non-finite u in this workgroup
    auto publish_cols = [&](int e, int flag) {
        if (tid < nch) {
            F2 s = *reinterpret_cast<const F2*>(&colbuf[0][2 * tid]);
#pragma unroll
            for (int ww = 1; ww < NW; ++ww) s += *reinterpret_cast<const F2*>(&colbuf[ww][2 * tid]);
            gstore_col(rs, cola(e, rb) + (uint32_t)tid * 16, chunk2(s[0], s[1], (e << 2) | flag), xl);
        }
    };
    // four independent accumulation chains (g, h) advanced together, r ascending in each
    auto col_partials = [&](const T (&wr)[R]) {
        F2 acc[G][2];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            acc[g][0] = kv[0][g][0] * wr[0];
            acc[g][1] = kv[0][g][1] * wr[0];
        }
#pragma unroll
        for (int r = 1; r < R; ++r)
#pragma unroll
            for (int g = 0; g < G; ++g) {
                acc[g][0] = __builtin_elementwise_fma(kv[r][g][0], F2{wr[r], wr[r]}, acc[g][0]);
                acc[g][1] = __builtin_elementwise_fma(kv[r][g][1], F2{wr[r], wr[r]}, acc[g][1]);
            }
#pragma unroll
        for (int g = 0; g < G; ++g)
            *reinterpret_cast<V*>(&colbuf[w][(lane + kWave * g) * VEC]) =
                V{acc[g][0][0], acc[g][0][1], acc[g][1][0], acc[g][1][1]};
    };
    // reducer (wave 0): S[e - 1] for this workgroup's chunk range from the nrb
    // producers of epoch e, fixed order; hop B carries the OR of their flags and the
    // error terms of iterate e - 2 (S[e - 1] against S[e - 2]).  Returns false on a stall.
    // need: the marginal error of this epoch is checked (POT tests it every check_every
    // iterations; the other iterations skip its two divisions and its reduction)
    auto reduce = [&](int e, bool need) -> bool {
        I4 x[KQW];
        bool act[KQW];
        unsigned pend = 0;
        const int k0 = RW > 1 ? w * KQW : 0;  // this wave's producer slice
#pragma unroll
        for (int k = 0; k < KQW; ++k) {
            const int q = r_qlo + LPC * (k0 + k);
            act[k] = r_ok && q < nrb;
            x[k] = I4{0, 0, 0, 0};
            if (act[k]) pend |= 1u << k;
        }
        bool ok = true;
        for (;;) {
#if OTF_MESH_RED_PEND
#pragma unroll
            for (int k = 0; k < KQW; ++k)
                if (pend & (1u << k)) x[k] = gload(rs, cola(e, r_qlo + LPC * (k0 + k)) + (uint32_t)r_ch * 16);
#pragma unroll
            for (int k = 0; k < KQW; ++k)
                if ((pend & (1u << k)) && chunk_at(x[k], (unsigned)e)) pend &= ~(1u << k);
#else
            // every pass reloads all KQW producers (unconditional loads, all in flight);
            // inactive slots (past nrb) re-read producer 0 and are ignored
#pragma unroll
            for (int k = 0; k < KQW; ++k) {
                const int q = r_qlo + LPC * (k0 + k);
                x[k] = gload(rs, cola(e, act[k] ? q : 0) + (uint32_t)(r_ok ? r_ch : 0) * 16);
            }
            unsigned np = 0;
#pragma unroll
            for (int k = 0; k < KQW; ++k)
                if (act[k] && !chunk_at(x[k], (unsigned)e)) np |= 1u << k;
            pend = np;
#endif
            if (!__any(pend != 0)) break;
            if (__builtin_amdgcn_s_memrealtime() > deadline) { ok = false; break; }
            __builtin_amdgcn_s_sleep(OTF_MESH_SLEEP);
        }
        OTF_MSTAMP(e - 2, 6, 0);
        T s0 = 0, s1 = 0;
        int fl = 0;
#pragma unroll
        for (int k = 0; k < KQW; ++k)
            if (act[k]) {
                s0 += chunk_v0(x[k]);
                s1 += chunk_v1(x[k]);
                fl |= x[k][1] & 1;
            }
        if (RW > 1) {
            // partials to LDS, then a ticket: the last reducer wave adds them in producer
            // order (the single-wave order: 0 + x0 + x1 + ..., bitwise the same sums)
            red_s[w][lane] = F2{s0, s1};
            red_f[w][lane] = fl;
            int t = 0;
            if (lane == 0) t = __hip_atomic_fetch_add(&red_cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            t = __builtin_amdgcn_readfirstlane(t);
            if (t != RW - 1) {
                deadline = __builtin_amdgcn_s_memrealtime() + p.timeout_ticks;
                return ok;
            }
            if (lane == 0) red_cnt = 0;  // next use is behind this iteration's barriers
            s0 = 0;
            s1 = 0;
            fl = 0;
#pragma unroll
            for (int ww = 0; ww < RW; ++ww) {
                const F2 q = red_s[ww][lane];
                s0 += q[0];
                s1 += q[1];
                fl |= red_f[ww][lane];
            }
        }
        // lanes with equal chunk: offsets CPR, 2 CPR, ..., 32 (uniform branches, static DPP)
        if (CPR <= 1) { s0 += wave_xor<T, 1>(s0); s1 += wave_xor<T, 1>(s1); }
        if (CPR <= 2) { s0 += wave_xor<T, 2>(s0); s1 += wave_xor<T, 2>(s1); }
        if (CPR <= 4) { s0 += wave_xor<T, 4>(s0); s1 += wave_xor<T, 4>(s1); }
        if (CPR <= 8) { s0 += wave_xor<T, 8>(s0); s1 += wave_xor<T, 8>(s1); }
        if (CPR <= 16) { s0 += wave_xor<T, 16>(s0); s1 += wave_xor<T, 16>(s1); }
        if (CPR <= 32) { s0 += wave_xor<T, 32>(s0); s1 += wave_xor<T, 32>(s1); }
        int bad = __any(fl) ? 1 : 0;
        if constexpr (XR) {
            // across ranks: this rank's partial of the reducer's chunks -> every rank's
            // exchange buffer (system-scope stores over xGMI), then the world's partials
            // of the same chunks from this rank's buffer, summed in rank order: every rank
            // derives the same S, bit for bit, and takes POT's decisions at the same epoch
            const unsigned ex = (p.xep + (unsigned)e) & 0x3fffffffu;
            const bool xa = lane < CPR && r_ok;
            const uint32_t gch = (uint32_t)(cb * kMeshNCH + r_ch);
            const uint32_t xs0 = (uint32_t)((2 * (p.xpar & 1) + (int)(ex & 1)) * 8);
            if (xa) {
                const I4 mine = chunk2(s0, s1, (int)(ex << 2) | bad);
                for (int r = 0; r < p.xworld; ++r)
                    gstore_sys(sums_rsrc(p.xr[r]), ((xs0 + (uint32_t)p.xrank) * (uint32_t)p.mc + gch) * 16u, mine);
            }
            const __amdgpu_buffer_rsrc_t rxx = sums_rsrc(p.xr[p.xrank]);
            I4 y[kXMaxRanks];
            for (;;) {
                unsigned pr = 0;
#pragma unroll
                for (int r = 0; r < kXMaxRanks; ++r)
                    if (xa && r < p.xworld) {
                        y[r] = gload_sys(rxx, ((xs0 + (uint32_t)r) * (uint32_t)p.mc + gch) * 16u);
                        if (!chunk_at(y[r], ex)) pr |= 1u << r;
                    }
                if (!__any(pr != 0)) break;
                if (__builtin_amdgcn_s_memrealtime() > deadline) { ok = false; break; }
                __builtin_amdgcn_s_sleep(OTF_MESH_SLEEP);
            }
            int xf = 0;
            if (xa) {
                s0 = 0;
                s1 = 0;
#pragma unroll
                for (int r = 0; r < kXMaxRanks; ++r)
                    if (r < p.xworld) {
                        s0 += chunk_v0(y[r]);
                        s1 += chunk_v1(y[r]);
                        xf |= y[r][1] & 1;
                    }
            }
            bad = __any(xf) ? 1 : 0;
        }
        // POT's marginal error of the iterate whose v = b / S[e - 2]
        const F2 sp = RW > 1 ? red_sp[lane] : F2{sp0, sp1};
        T term = 0;
        if (need) {
            if (rc0) { const T rr = (rb0 / sp[0]) * s0 - rb0; term += rr * rr; }
            if (rc1) { const T rr = (rb1 / sp[1]) * s1 - rb1; term += rr * rr; }
            if (CPR > 1) term += wave_xor<T, 1>(term);
            if (CPR > 2) term += wave_xor<T, 2>(term);
            if (CPR > 4) term += wave_xor<T, 4>(term);
            if (CPR > 8) term += wave_xor<T, 8>(term);
            if (CPR > 16) term += wave_xor<T, 16>(term);
            if (CPR > 32) term += wave_xor<T, 32>(term);
        }
        if (RW > 1) {
            red_sp[lane] = F2{s0, s1};
        } else {
            sp0 = s0;
            sp1 = s1;
        }
        const int tag = (e << 2) | bad;
        if (lane < CPR && r_ok) gstore_col(rs, colb(e, rb) + (uint32_t)r_cc * 16, chunk2(s0, s1, tag), xl);
        if (need && lane == 0 && rb < nred)
            gstore_col(rs, colb(e, rb) + (uint32_t)CPR * 16, chunk2(term, 0.f, tag), xl);
        OTF_MSTAMP(e - 2, 7, 0);
        deadline = __builtin_amdgcn_s_memrealtime() + p.timeout_ticks;
        return ok;
    };
    // hop B: the sums S[e - 1] of this tile's columns -> v into vcur; the column tile's
    // error partial into s_E.  Returns bit 0 = producer flag, 1 = stall, 2 = bad v.
    auto gather_b = [&](int e, bool need) -> int {
        int fl = 0;
        T ep = 0;
        if (tid >= 256) {
            const int t = tid - 256;
            if (t < nch) {
                const uint32_t off = colb(e, t / CPR) + (uint32_t)(t & (CPR - 1)) * 16;
                I4 x;
                if (!poll_chunk<OTF_MESH_SLEEP>(rs, off, (unsigned)e, deadline, x)) fl |= 2;
                OTF_MSTAMP(e - 1, 8, 256);
                fl |= x[1] & 1;
                const T s0 = chunk_v0(x), s1 = chunk_v1(x);
                const bool ok0 = 2 * t < ncols, ok1 = 2 * t + 1 < ncols;
                const T v0n = bch0 / s0, v1n = bch1 / s1;
                if ((ok0 && (s0 == (T)0 || !finite_val(v0n))) || (ok1 && (s1 == (T)0 || !finite_val(v1n))))
                    fl |= 4;
                vcur[2 * t] = ok0 ? v0n : (T)0;
                vcur[2 * t + 1] = ok1 ? v1n : (T)0;
            }
        } else if (w == 3 && need) {
            if (lane < nred) {
                const uint32_t off = colb(e, lane) + (uint32_t)CPR * 16;
                I4 x;
                if (!poll_chunk<OTF_MESH_SLEEP>(rs, off, (unsigned)e, deadline, x)) fl |= 2;
                ep = chunk_v0(x);
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
    // the total error from the ncb column tiles' partials (row-hop error chunks of epoch
    // er): wave-level, lanes < ncb poll.  Returns false on a stall.
    auto err_total = [&](int er, T& tot) -> bool {
        T ev = 0;
        bool ok = true;
        if (lane < ncb) {
            const uint32_t off = rowx(er, lane) + 64 * 16;
            I4 x;
            ok = poll_chunk<OTF_MESH_SLEEP>(rs, off, (unsigned)er, deadline, x);
            ev = chunk_v0(x);
        }
        ev += wave_xor<T, 1>(ev);
        ev += wave_xor<T, 2>(ev);
        ev += wave_xor<T, 4>(ev);
        if (ncb > 8) ev += wave_xor<T, 8>(ev);
        tot = __builtin_bit_cast(T, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, ev)));
        return __all(ok);
    };
    auto to_err = [&](T e) -> double { return p.err_squared ? (double)e : sqrt((double)e); };
    auto stop_ok = [&](double err) -> bool {
        return p.err_squared ? !(err > p.stop_thr) : (err < p.stop_thr);
    };

    // ---- prologue: S[0] = K^T u0 (epoch 1)
    {
        T wr[R];
#pragma unroll
        for (int r = 0; r < R; ++r) wr[r] = row_in(row0 + r) ? (SH ? p.sh.u0[row0 + r] : u0) : (T)0;
        col_partials(wr);
        __syncthreads();
        publish_cols(1, 0);
    }
    int last_good = -1, niter = 0, status = OTF_SK_MAX_ITER, brk = -1, n_err = 0;
    bool done = false;
    if (w < RW && !reduce(1, false)) s_ep[1] = 1;  // seen after the hop-B barrier of epoch 1
    int chk = 0;  // (it - 1) % check_every for it >= 1

    for (int it = 0; it < p.max_iter; ++it) {
        // re-derive the lane predicates every iteration (one v_cmp each) instead of
        // keeping ~20 hoisted 64-bit lane masks live across the loop: that set spilled
        // the SGPR file into VGPR lanes (v_readlane / v_writelane on every use)
        asm volatile("" : "+v"(tid), "+v"(lane));
        OTF_STAMP(it, 0);
        OTF_MSTAMP(it, 0, 0);
        const int e = it + 1;  // hop-B epoch of S[it]; row-hop epoch of iteration it
        // (it - 1) % check_every == 0, kept as a counter (no integer division per iteration)
        const bool check = it >= 1 && chk == 0;
        const int fl = gather_b(e, check);
        OTF_STAMP(it, 1);
        OTF_MSTAMP(it, 1, 0);
        if (fl & 2) { status = OTF_SK_TIMEOUT; done = true; break; }
        // a non-finite u in iteration it - 1 (any row block) -> revert to it - 2
        if (fl & 1) {
            last_good = it - 2; niter = it - 1; status = OTF_SK_NUMERICAL_BREAK; brk = it - 1;
            done = true;
            break;
        }
        const int vbad_cb = (fl & 4) ? 1 : 0;
        F2 vn[G][2];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const V t = *reinterpret_cast<const V*>(&vcur[(lane + kWave * g) * VEC]);
            vn[g][0] = F2{t[0], t[1]};
            vn[g][1] = F2{t[2], t[3]};
        }
        // row partials over this tile's columns, wave totals
        T rp[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            F2 acc = kv[r][0][0] * vn[0][0];
            acc = __builtin_elementwise_fma(kv[r][0][1], vn[0][1], acc);
            acc = __builtin_elementwise_fma(kv[r][1][0], vn[1][0], acc);
            acc = __builtin_elementwise_fma(kv[r][1][1], vn[1][1], acc);
            rp[r] = acc[0] + acc[1];
        }
        // wave totals: lane L holds row L >> 2; the lane group c = L >> 3 takes the chunk
        // (rows 2c, 2c + 1) from its half-mirror partner (the other row of the pair)
        T t0, t1;
        {
            const T mine = wave_row_totals<T, R>(rp, lane), oth = dpp_f<0x141>(mine);
            const bool odd = (lane & 4) != 0;
            t0 = odd ? oth : mine;
            t1 = odd ? mine : oth;
        }
        if (it >= 1) chk = chk + 1 == p.check_every ? 0 : chk + 1;
        T errv = 0;
        int vbad = vbad_cb, stall = 0;
        if (ncb == 1) {
            // the tile spans whole rows: totals, v flags and the error are already global
            errv = s_E;
            OTF_STAMP(it, 2);
            OTF_STAMP(it, 3);
        } else {
            // row hop: publish this wave's 16 row partials (8 chunks, lane 8c) and the
            // column tile's error partial, gather the ncb members' chunks of the same rows
            if ((lane & 7) == 0)
                gstore(rs, rowx(e, cb) + (uint32_t)(w * 8 + rc) * 16, chunk2(t0, t1, (e << 2) | vbad_cb));
            if (check && w == 0 && lane == 1) gstore(rs, rowx(e, cb) + 64 * 16, chunk2(s_E, 0.f, e << 2));
            OTF_STAMP(it, 2);
            OTF_MSTAMP(it, 2, 0);
            OTF_MSTAMP(it, 10, 448);
            // lane (c = lane >> 3, q = lane & 7): chunk c of member q; the member sum is a
            // butterfly over the lane's 8 (quad_perm ^1, ^2, half mirror)
            const int q = lane & 7;
            const bool act = q < ncb;
            I4 x = I4{0, 0, 0, 0};
            if (act) {
                const uint32_t off = rowx(e, q) + (uint32_t)(w * 8 + rc) * 16;
                if (!poll_chunk<OTF_MESH_SLEEP>(rs, off, (unsigned)e, deadline, x)) stall = 1;
            }
            OTF_MSTAMP(it, 3, 0);
            OTF_MSTAMP(it, 9, 448);
            t0 = act ? chunk_v0(x) : (T)0;
            t1 = act ? chunk_v1(x) : (T)0;
            int vb = act && (x[1] & 1);
            if (ncb > 8) {
                // more than 8 members (m > 4096): the lane also takes member q + 8
                const bool act2 = q + 8 < ncb;
                I4 x2 = I4{0, 0, 0, 0};
                if (act2) {
                    const uint32_t off = rowx(e, q + 8) + (uint32_t)(w * 8 + rc) * 16;
                    if (!poll_chunk<OTF_MESH_SLEEP>(rs, off, (unsigned)e, deadline, x2)) stall = 1;
                }
                t0 += act2 ? chunk_v0(x2) : (T)0;
                t1 += act2 ? chunk_v1(x2) : (T)0;
                vb |= act2 && (x2[1] & 1);
            }
            vbad = __any(vb) ? 1 : 0;
            t0 += dpp_f<0xB1>(t0);
            t1 += dpp_f<0xB1>(t1);
            t0 += dpp_f<0x4E>(t0);
            t1 += dpp_f<0x4E>(t1);
            t0 += dpp_f<0x141>(t0);
            t1 += dpp_f<0x141>(t1);
            if (check && !err_total(e, errv)) stall = 1;
            stall = __any(stall) ? 1 : 0;
            OTF_STAMP(it, 3);
        }
        // u of rows 2c, 2c + 1 in every lane of group c; to every lane as wave-uniform
        // values (v_readlane, no LDS round trip); the group's first lane keeps the history
        T un[R];
        int badu = 0;
        {
            T un0 = (T)1 / (t0 * ia_c0), un1 = (T)1 / (t1 * ia_c1);
            if (!row_in(row0 + 2 * rc)) un0 = 0;
            if (!row_in(row0 + 2 * rc + 1)) un1 = 0;
            badu = __any(!finite_val(un0) || !finite_val(un1)) ? 1 : 0;
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                un[2 * c] = __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, un0), 8 * c));
                un[2 * c + 1] = __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, un1), 8 * c));
            }
            if ((lane & 7) == 0)
                *reinterpret_cast<F2*>(&uhist[it & 1][w * R + 2 * rc]) = F2{un0, un1};
        }
        // POT's decisions for iterate it - 1 (error) and iterate it (v); identical in
        // every wave of every workgroup unless a wave stalled (then all time out)
        double err = 0.0;
        int dec = 0;
        if (check) {
            err = to_err(errv);
            if (stop_ok(err)) dec = 1;
        }
        if (dec == 0 && vbad) dec = 2;
        col_partials(un);
        // histories of iterate it (slot it & 1; only read when last_good >= it, i.e. when
        // this iteration is not the one a decision below reverts)
        const int slot = it & 1;
        vhist[slot][tid] = vcur[tid];
        if (badu) s_ep[0] = it;
        if (stall) s_ep[4] = it;
        __syncthreads();
        OTF_STAMP(it, 4);
        OTF_MSTAMP(it, 4, 0);
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
        OTF_MSTAMP(it, 5, 0);
        if (w < RW && !reduce(e + 1, chk == 0)) s_ep[1] = e + 1;  // seen after the next hop-B barrier
        OTF_STAMP(it, 5);
    }
    if (!done && p.max_iter > 0) {
        // the last iteration's u flags and S[max_iter]; its error needs one more
        // exchange of the column tiles' partials
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
                    if (w == 0 && lane == 8) gstore(rs, rowx(e, cb) + 64 * 16, chunk2(s_E, 0.f, e << 2));
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

    // ---- outputs: (u, v) of last_good from the histories, plan from registers
    __syncthreads();
    const int hs = last_good & 1;
    T uo[R], vo[G][VEC];
#pragma unroll
    for (int r = 0; r < R; ++r)
        uo[r] = last_good >= 0 ? uhist[hs][w * R + r] : SH ? (row_in(row0 + r) ? p.sh.u0[row0 + r] : (T)0) : u0;
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const int c = col0 + (lane + kWave * g) * VEC + k;
            vo[g][k] = last_good >= 0 ? vhist[hs][(lane + kWave * g) * VEC + k]
                                      : SH ? (col_in(c) ? p.sh.v0[c] : (T)0) : v0;
        }
    if (cb == 0 && lane < R && row_in(row0 + lane)) {
        T mine = uo[0];
#pragma unroll
        for (int r = 1; r < R; ++r) if (lane == r) mine = uo[r];
        p.u_out[row0 + lane] = mine;
    }
    if (rb == 0 && w == 0) {
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const int c = col0 + (lane + kWave * g) * VEC + k;
                if (col_in(c)) p.v_out[c] = vo[g][k];
            }
    }
    if (p.P) {
        TP* P = (TP*)p.P;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (!row_in(row0 + r)) break;
            TP* prow = P + (int64_t)(row0 + r) * p.ldp;
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const int c0 = col0 + (lane + kWave * g) * VEC;
                if (!col_in(c0)) continue;
                VP o;
#pragma unroll
                for (int k = 0; k < VEC; ++k) o[k] = (TP)(uo[r] * kv[r][g][k >> 1][k & 1] * vo[g][k]);
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
        p.info->engine = OTF_ENGINE_MESH;
        p.info->stop = 1;
    }
}

template <typename CT, typename TP, bool SH>
const void* mesh_kernel_for(const SkMeshArgs& p) {
    const bool pow2 = (p.nrb & (p.nrb - 1)) == 0;
    // the N = 4096 metric shape (32 x 8 whole tiles) has its own compiled-in instance
    const bool whole = p.n == p.nrb * kMeshTR && p.m == p.ncb * kMeshTC;
    return (whole && p.nrb == 32 && p.ncb == 8) ? (const void*)sk_mesh_kernel<CT, TP, 4, 32, 8, SH>
           : pow2 ? (const void*)sk_mesh_kernel<CT, TP, 4, 0, 0, SH>
                  : (const void*)sk_mesh_kernel<CT, TP, 8, 0, 0, SH>;
}
// the pairwise instances (whole tiles, float32 cost built in the prologue)
template <typename TP>
const void* pw_mesh_kernel_for(const SkMeshArgs& p) {
    const bool pow2 = (p.nrb & (p.nrb - 1)) == 0;
    return (p.nrb == 32 && p.ncb == 8) ? (const void*)sk_mesh_kernel<float, TP, 4, 32, 8, false, false, true>
           : pow2 ? (const void*)sk_mesh_kernel<float, TP, 4, 0, 0, false, false, true>
                  : (const void*)sk_mesh_kernel<float, TP, 8, 0, 0, false, false, true>;
}
// the cross-rank instances (the generic shape, no shifted kernel)
template <typename CT, typename TP>
const void* xmesh_kernel_for(const SkMeshArgs& p) {
    const bool pow2 = (p.nrb & (p.nrb - 1)) == 0;
    return pow2 ? (const void*)sk_mesh_kernel<CT, TP, 4, 0, 0, false, true>
                : (const void*)sk_mesh_kernel<CT, TP, 8, 0, 0, false, true>;
}

template <typename CT, typename TP>
hipError_t launch_mesh_t(int grid, SkMeshArgs& p, hipStream_t s) {
    void* args[] = {&p};
    const void* k = p.pw.Xh      ? pw_mesh_kernel_for<TP>(p)
                    : p.xworld > 1 ? xmesh_kernel_for<CT, TP>(p)
                    : p.sh.A     ? mesh_kernel_for<CT, TP, true>(p)
                                 : mesh_kernel_for<CT, TP, false>(p);
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 512, 0);
    if (e != hipSuccess) return e;
    if (per_cu < 1 || grid > per_cu * device_cu_count()) return hipErrorCooperativeLaunchTooLarge;
    return hipLaunchKernel(k, dim3(grid), dim3(512), args, 0, s);
}

// 8 XCC counters, the registration barrier, the PW max barrier and the PW max, 256 B each
constexpr size_t kMeshRegBytes = 11 * 256;
inline int64_t align_up_mesh(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

struct MeshShape {
    int nrb, ncb, cpr;
    uint32_t bstride;
    size_t row_bytes, cola_bytes, colb_bytes;
};

MeshShape mesh_shape(int64_t n, int64_t m) {
    MeshShape s{};
    s.nrb = (int)((n + kMeshTR - 1) / kMeshTR);
    s.ncb = (int)((m + kMeshTC - 1) / kMeshTC);
    int per = (kMeshNCH + s.nrb - 1) / (s.nrb > 0 ? s.nrb : 1);
    int cpr = 1;
    while (cpr < per) cpr <<= 1;
    s.cpr = cpr;
    s.bstride = (uint32_t)((cpr + 1) * 16 + 255) / 256 * 256;
    s.row_bytes = 2 * (size_t)s.nrb * s.ncb * kRowStride;
    s.cola_bytes = 2 * (size_t)s.nrb * s.ncb * kColStride;
    s.colb_bytes = 2 * (size_t)s.nrb * s.ncb * s.bstride;
    return s;
}

}  // namespace

bool mesh_supported(int64_t n, int64_t m) {
    if (n < 1 || m < 1) return false;
    const MeshShape s = mesh_shape(n, m);
    return s.nrb >= kMeshMinNrb && s.nrb <= kMeshMaxNrb && s.ncb <= kMeshMaxNcb && s.cpr <= 64 &&
           (int64_t)s.nrb * s.ncb <= 1024;
}

bool mesh_pairwise_ok(int64_t n, int64_t m, int64_t d) {
    return mesh_supported(n, m) && n % kMeshTR == 0 && m % kMeshTC == 0 && m / kMeshTC <= kMeshXccNcb &&
           d >= 1 && d <= (1 << 16);
}

size_t mesh_region_bytes(int64_t n, int64_t m) {
    if (!mesh_supported(n, m)) return 0;
    const MeshShape s = mesh_shape(n, m);
    return kMeshRegBytes + s.row_bytes + s.cola_bytes + s.colb_bytes;
}

template <typename CT>
hipError_t run_mesh(const CT* C, int64_t ldc, int n, int m, const float* a_pad, const float* b_pad,
                    const float* cost_scale, const otf_sinkhorn_opts& o, void* region, float* u_out,
                    float* v_out, void* P_out, int64_t ldp, int P_dtype, otf_sinkhorn_info* info,
                    double* errlog, bool zeroed, hipStream_t s, const ShiftArgs* shift,
                    const XSweep* xs, const PairwiseF32* pw) {
    if (!mesh_supported(n, m) || !region) return hipErrorInvalidValue;
    if (pw && (shift || (xs && xs->world > 1) || n % kMeshTR != 0 || m % kMeshTC != 0 || pw->kpad % kPwK != 0 ||
               pw->ldh % 8 != 0))
        return hipErrorInvalidValue;
    const bool xr = xs && xs->world > 1;
    if (xr && (shift || xs->world > kXMaxRanks || m % kMeshTC != 0)) return hipErrorInvalidValue;
    const MeshShape sh = mesh_shape(n, m);
    if (sh.nrb * sh.ncb > device_cu_count()) return hipErrorCooperativeLaunchTooLarge;
    SkMeshArgs p{};
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
    p.gran = (char*)region + kMeshRegBytes;
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
    // one column tile per XCC: more tiles than XCCs take the blockIdx roles
    if (sh.ncb > kMeshXccNcb) p.xcc_local = 0;
    p.n_total = n;
    if (xr) {
        p.n_total = xs->n_total;
        p.xrank = xs->rank;
        p.xworld = xs->world;
        p.xpar = xs->solve_par;
        p.xep = xs->ep_base;
        p.mc = (int)(align_up_mesh(m, 64) / 2);
        for (int r = 0; r < xs->world; ++r) p.xr[r] = xs->xr[r];
    }
    p.info = info;
    p.errlog = errlog;
    p.u_out = u_out;
    p.v_out = v_out;
    p.P = P_out;
    p.ldp = ldp;
    p.timeout_ticks = stall_ticks();
    p.reg_ticks = reg_stall_ticks();
    if (shift) p.sh = *shift;
    if (pw) {
        p.pw = *pw;
        p.C = nullptr;
        p.cost_scale = nullptr;  // the max is applied when K is formed
    }
    if (!zeroed) {  // else the Sinkhorn init kernel zeroed it
        const hipError_t e = hipMemsetAsync(region, 0, mesh_region_bytes(n, m), s);
        if (e != hipSuccess) return e;
    }
    // XCC mode launches nrb workgroups per XCC (8 x nrb) so that every column tile can
    // find a whole XCC of them even when ncb < 8; the surplus leaves after registration
    int grid = sh.nrb * sh.ncb;
    if (p.xcc_local && 8 * sh.nrb <= device_cu_count()) grid = 8 * sh.nrb;
    else p.xcc_local = 0;
    if (P_out && P_dtype == OTF_F64) return launch_mesh_t<CT, double>(grid, p, s);
    return launch_mesh_t<CT, float>(grid, p, s);
}

template hipError_t run_mesh<float>(const float*, int64_t, int, int, const float*, const float*,
                                    const float*, const otf_sinkhorn_opts&, void*, float*, float*,
                                    void*, int64_t, int, otf_sinkhorn_info*, double*, bool,
                                    hipStream_t, const ShiftArgs*, const XSweep*, const PairwiseF32*);
template hipError_t run_mesh<_Float16>(const _Float16*, int64_t, int, int, const float*, const float*,
                                       const float*, const otf_sinkhorn_opts&, void*, float*, float*,
                                       void*, int64_t, int, otf_sinkhorn_info*, double*, bool,
                                       hipStream_t, const ShiftArgs*, const XSweep*, const PairwiseF32*);

}  // namespace otf
