// otf_mesh2.hip — the mesh engine's two-hop form (OTF_ENGINE_MESH, build / run switch
// OTF_MESH2): POT sinkhorn_knopp (POT 0.9.6, MRI_PET_OT_nojax.py:143 ->
// perturbot/perturbot/match/utils.py:6-115), float32 compute, K resident in registers,
// for meshes of whole 256 x 256 tiles with 8 or 16 row blocks x 8 or 16 column tiles --
// the N = 4096 metric config (BASELINE.json configs[1]) is 16 x 16.
//
// otf_mesh.hip keeps 128 x 512 tiles and needs THREE exchanges per iteration: the row
// hop, the column partials to a reducer, the reduced sums back (hop B).  With 256 x 256
// tiles a column tile has only 16 producers, so every workgroup can gather all of them
// itself -- the column side becomes ONE all-gather and the reducer stage disappears:
//
//   column hop  every workgroup gathers its column tile's 16 producers' partials K^T u
//               (64 chunks each; two loads per thread), adds the pair it loaded, and
//               the 8 waves' pairs in LDS in a fixed order -> S -> v = b / S;
//   row hop     every wave publishes its 32 rows' partials K v over the tile's 256
//               columns (8 chunks) and gathers the same rows' partials of the row
//               block's ncb members (two loads per lane), fixed butterfly -> u.
//
// Granules carry FOUR floats per 16-B chunk: the epoch tag (e mod 4: a slot holds epoch
// e - 2, e, or the zero fill before epochs 1 and 2) and a flag bit ride in the three low
// mantissa bits of every value (rounded to 20 bits first: relative 2^-21, far below the
// float32 plan tolerance of 1e-4; 0 and +-inf come back exact once the bits are cleared)
// -- half the bytes of {value, tag} pairs, which the all-gather multiplies by 16.  POT's
// decisions travel as in otf_mesh.hip: a zero / non-finite v of iteration it in the
// row-hop flags of it; a non-finite u of it in the column-partial flags -> the column hop
// of it + 1; the marginal error of iterate it - 1 as one extra row-hop chunk per column
// tile.  Every sum has one fixed order, so every member of a group holds bit-identical
// values and the solve is bitwise reproducible.  Parity double buffering suffices for
// both hops (a member publishes epoch e + 2 only after its gather of e + 1, which needed
// every member's publish of e + 1, made after its own gather of e).
//
// Roles: a column tile's 16 producers must share one XCC's L2 for the plain-store column
// path (otf_mesh.hip, "XCC-local column path"): every workgroup registers on its XCC; when
// each XCC holds exactly ncb / 8 column tiles' worth of workgroups, XCC rank x gets column
// tiles x * cpx .. and the registration slot picks the row block; otherwise blockIdx roles
// with every hop write-through (correct, slower).
#include "otf_persist.h"

namespace otf {
namespace {

constexpr int kM2T = 256;            // tile rows = tile columns
constexpr int kM2NW = 8;             // waves per workgroup
constexpr int kM2RW = 32;            // rows per wave
constexpr int kM2NCH = 64;           // 16-B chunks (4 values) per 256 columns
constexpr uint32_t kM2RowStride = 1280;  // per (rb, cb): 8 waves x 8 row chunks + the error chunk
constexpr uint32_t kM2ColStride = 1024;  // per (cb, rb): 64 column chunks

struct SkMesh2Args {
    const void* C;
    int64_t ldc;
    int n, m;
    const float* a;
    const float* b;
    const float* cost_scale;
    double reg;
    int max_iter, check_every, err_squared;
    double stop_thr;
    void* gran;
    uint32_t off_row, off_col;
    int xcc_local;
    int* xreg;  // [8 x 64] registrants per XCC, then the flat barrier word
    otf_sinkhorn_info* info;
    double* errlog;
    float* u_out;
    float* v_out;
    void* P;
    int64_t ldp;
    unsigned long long timeout_ticks;
    unsigned long long reg_ticks;
    ShiftArgs sh;
};

using F2 = __attribute__((ext_vector_type(2))) float;
using F4 = __attribute__((ext_vector_type(4))) float;

// Diagnostic build only (-DOTF_MESH2_STAMPS, tools/stamps_mesh2.hip): wall-clock stamps per
// role (rb * NCB + cb), iteration 0..15, slot: 0 start, 1 column gather loaded (wave 0),
// 2 v ready (after the barrier), 3 row chunks published (wave 0), 4 row hop done (wave 0),
// 5 column partials reduced (after the barrier), 6 column chunks published, 9 / 10 the row
// hop done / published by wave 7
#ifdef OTF_MESH2_STAMPS
__device__ unsigned long long g_m2stamps[256 * 16 * 16];
__device__ int g_m2role[256 * 4];
#define OTF_M2STAMP(it, slot, who)                                                            \
    do {                                                                                      \
        if (threadIdx.x == (who) && (it) >= 0 && (it) < 16)                                   \
            g_m2stamps[((rb * NCB + cb) * 16 + (it)) * 16 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define OTF_M2STAMP(it, slot, who) \
    do {                           \
    } while (0)
#endif

// value with the tag in its three low mantissa bits: (epoch & 3) | flag << 2
__device__ __forceinline__ int tag_val(float v, int tag) {
    const unsigned b = __builtin_bit_cast(unsigned, v);
    // round to 20 mantissa bits (+-inf and NaN keep their class), then the tag
    return (int)(((b + 4u) & ~7u) | (unsigned)tag);
}
__device__ __forceinline__ float untag(int w) { return __builtin_bit_cast(float, (unsigned)w & ~7u); }
__device__ __forceinline__ I4 chunk4(F4 v, int tag) {
    return I4{tag_val(v[0], tag), tag_val(v[1], tag), tag_val(v[2], tag), tag_val(v[3], tag)};
}
__device__ __forceinline__ bool chunk4_at(const I4 x, unsigned e) {
    const unsigned t = e & 3u;
    return (((unsigned)x[0] & 3u) == t) && (((unsigned)x[1] & 3u) == t) && (((unsigned)x[2] & 3u) == t) &&
           (((unsigned)x[3] & 3u) == t);
}
__device__ __forceinline__ int chunk4_flag(const I4 x) { return (x[0] | x[1] | x[2] | x[3]) >> 2 & 1; }
__device__ __forceinline__ F4 chunk4_vals(const I4 x) {
    const int a = x[0], b = x[1], c = x[2], d = x[3];
    return F4{untag(a), untag(b), untag(c), untag(d)};
}

// Wave totals of 32 per-lane row partials (otf_device.h wave_row_totals, one level more):
// lane bits 5, 4 by the permlane swaps, 3 and 2 by row_mirror / row_half_mirror with a
// keep / send select, bit 1 by quad ^2 with a select, bit 0 summed.  Lane L ends with the
// total of row L >> 1; both lanes of a row hold bitwise the same sum.
__device__ __forceinline__ float wave_row_totals32(const float (&x)[32], int lane) {
    float y[16], z[8], w4[4], w2[2];
#pragma unroll
    for (int i = 0; i < 16; ++i) y[i] = swap_sum<32>(x[i], x[i + 16]);
#pragma unroll
    for (int i = 0; i < 8; ++i) z[i] = swap_sum<16>(y[i], y[i + 8]);
    const bool b3 = (lane & 8) != 0, b2 = (lane & 4) != 0, b1 = (lane & 2) != 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float send = b3 ? z[i] : z[i + 4], keep = b3 ? z[i + 4] : z[i];
        w4[i] = keep + dpp_lane<0x140>(send);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const float send = b2 ? w4[i] : w4[i + 2], keep = b2 ? w4[i + 2] : w4[i];
        w2[i] = keep + dpp_lane<0x141>(send);
    }
    const float send = b1 ? w2[0] : w2[1], keep = b1 ? w2[1] : w2[0];
    float t = keep + dpp_lane<0x4E>(send);
    t += dpp_lane<0xB1>(t);
    return t;
}
// polls one chunk4 until all four tags carry epoch e; false on a stall
__device__ __forceinline__ bool poll_chunk4(__amdgpu_buffer_rsrc_t rs, uint32_t off, unsigned e,
                                            unsigned long long deadline, I4& x) {
    for (;;) {
        x = gload(rs, off);
        if (chunk4_at(x, e)) return true;
        if (__builtin_amdgcn_s_memrealtime() > deadline) return false;
        __builtin_amdgcn_s_sleep(1);
    }
}
// value of lane (lane + K) within the 16-lane row (row_shl:K), 0 past the row
template <int K> __device__ __forceinline__ float row_shl(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x100 + K, 0xF, 0xF, false));
}

template <int NRB, int NCB, typename CT, typename TP, bool SH>
__global__ __launch_bounds__(512) void sk_mesh2_kernel(SkMesh2Args p) {
    using T = float;
    constexpr int NW = kM2NW, RW = kM2RW, TT = kM2T;
    constexpr int CPX = NCB / 8;  // column tiles per XCC (XCC-local roles)
    static_assert((NRB == 8 || NRB == 16) && (NCB == 8 || NCB == 16), "8 or 16 row / column tiles");
    __shared__ __attribute__((aligned(16))) F4 gbuf[NW][kM2NCH];   // column hop: per-wave pair sums
    __shared__ __attribute__((aligned(16))) T colbuf[NW][TT];      // column partials per wave
    __shared__ __attribute__((aligned(16))) T vhist[2][TT];
    __shared__ T uhist[2][TT];
    __shared__ int gfl[NW];   // column hop flags per wave: bit 0 producer (u) flag, bit 1 stall
    __shared__ int s_ep[2];   // [0] non-finite u in this workgroup (iteration key), [1] stall
    int tid = threadIdx.x, lane = tid & 63;
    const int w = (int)threadIdx.x >> 6;
    unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + p.reg_ticks;

    int rb = 0, cb = 0, xl = 0;
    if (p.xcc_local) {
        __shared__ int s_reg[4];
        const int xcd = xcc_id();
        if (tid == 0)
            s_reg[0] = __hip_atomic_fetch_add(p.xreg + xcd * 64, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool ok = grid_barrier(p.xreg + 8 * 64, gridDim.x, deadline, p.timeout_ticks, &s_reg[3],
                                     &p.info->stalled);
        if (tid == 0) {
            // XCC-local roles only when every XCC holds exactly CPX column tiles' workgroups
            int good = ok ? 1 : 0, rank = -1, nq = 0;
            for (int x = 0; x < 8; ++x) {
                const int c = load_agent(p.xreg + x * 64);
                if (c != CPX * NRB) good = 0;
                if (c > 0) {
                    if (x == xcd) rank = nq;
                    ++nq;
                }
            }
            if (nq != 8) good = 0;
            s_reg[1] = good;
            s_reg[2] = rank;
        }
        __syncthreads();
        if (!s_reg[3]) {
            if (tid == 0) mark_stalled(&p.info->stalled, kStallRegistration);
            return;
        }
        if (s_reg[1]) {
            rb = s_reg[0] % NRB;
            cb = s_reg[2] * CPX + s_reg[0] / NRB;
            xl = 1;
        }
    }
    if (!xl) {
        const int bi = blockIdx.x;
        rb = bi / NCB;
        cb = bi % NCB;
    }
    const bool lead = (rb == 0 && cb == 0 && tid == 0);
#ifdef OTF_MESH2_STAMPS
    if (tid == 0) {
        g_m2role[(rb * NCB + cb) * 4 + 0] = rb;
        g_m2role[(rb * NCB + cb) * 4 + 1] = cb;
        g_m2role[(rb * NCB + cb) * 4 + 2] = xcc_id();
        g_m2role[(rb * NCB + cb) * 4 + 3] = 1 + NCB * 1000 + NRB * 100000;
    }
#endif
    const int row0 = rb * TT + w * RW;   // this wave's first row
    const int col0 = cb * TT + 4 * lane; // this lane's first column
    const int n_ = NRB * TT, m_ = NCB * TT;

    const double unit = exp_unit<T>();
    double cinv = 1.0;
    if (p.cost_scale) cinv = 1.0 / (double)p.cost_scale[0];
    const T ks = (T)(-unit / p.reg * cinv);

    // ---- K for this wave's 32 rows x this lane's 4 columns (pairs for v_pk_fma_f32)
    F2 kv[RW][2];
    {
        const CT* crow = (const CT*)p.C + (int64_t)row0 * p.ldc + col0;
        using V = Vec<float>::type;
        V shb = V{0, 0, 0, 0};
        if (SH) shb = *reinterpret_cast<const V*>(p.sh.B + col0);
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            const V c = load_cost<T>(crow);
            const T sha = SH ? p.sh.A[row0 + r] : (T)0;
            T e[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                T z = c[k] * ks;
                if (SH) z += sha + shb[k];
                e[k] = fast_exp(z);
            }
            kv[r][0] = F2{e[0], e[1]};
            kv[r][1] = F2{e[2], e[3]};
            crow += p.ldc;
        }
    }
    // row hop lanes: chunk rc = lane & 7 (rows 4 rc .. 4 rc + 3 of the wave), members
    // mq = lane >> 3 and mq + 8
    const int rc = lane & 7, mq = lane >> 3;
    T ia[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) ia[k] = (T)1 / p.a[row0 + 4 * rc + k];
    T bcol[4];  // b of this lane's columns
    {
        const F4 bb = *reinterpret_cast<const F4*>(p.b + col0);
#pragma unroll
        for (int k = 0; k < 4; ++k) bcol[k] = bb[k];
    }
    const T u0 = (T)1 / (T)n_, v0 = (T)1 / (T)m_;
    if (tid < 2) s_ep[tid] = -1;
    for (int q = tid; q < TT; q += blockDim.x) {
        vhist[0][q] = vhist[1][q] = v0;
        uhist[0][q] = uhist[1][q] = u0;
    }

    const __amdgpu_buffer_rsrc_t rs = sums_rsrc(p.gran);
    auto rowx = [&](int e, int q) -> uint32_t {  // (rb, member q) of epoch e
        return p.off_row + ((uint32_t)((e & 1) * NRB + rb) * (uint32_t)NCB + (uint32_t)q) * kM2RowStride;
    };
    auto colx = [&](int e, int q) -> uint32_t {  // (cb, producer q) of epoch e
        return p.off_col + ((uint32_t)((e & 1) * NCB + cb) * (uint32_t)NRB + (uint32_t)q) * kM2ColStride;
    };

    // column partials K_tile^T wr -> colbuf (LDS), then (after the barrier) the 64 chunks of
    // this workgroup published by wave 0 for epoch e with flag
    auto col_partials = [&](const T (&wr)[RW]) {
        F2 a0 = kv[0][0] * wr[0], a1 = kv[0][1] * wr[0];
#pragma unroll
        for (int r = 1; r < RW; ++r) {
            a0 = __builtin_elementwise_fma(kv[r][0], F2{wr[r], wr[r]}, a0);
            a1 = __builtin_elementwise_fma(kv[r][1], F2{wr[r], wr[r]}, a1);
        }
        *reinterpret_cast<F4*>(&colbuf[w][4 * lane]) = F4{a0[0], a0[1], a1[0], a1[1]};
    };
    auto publish_cols = [&](int e, int flag) {
        if (w == 0) {
            F4 s = *reinterpret_cast<const F4*>(&colbuf[0][4 * lane]);
#pragma unroll
            for (int ww = 1; ww < NW; ++ww) s += *reinterpret_cast<const F4*>(&colbuf[ww][4 * lane]);
            gstore_col(rs, colx(e, rb) + (uint32_t)lane * 16, chunk4(s, (e & 3) | (flag << 2)), xl);
        }
    };
    // column hop of epoch e: S of this tile's columns -> sums into s4 of every lane
    // (its 4 columns); returns bit 0 = a producer's u flag, bit 1 = stall
    auto gather_cols = [&](int e, F4& s4) -> int {
        (void)e;
        const int q0 = w, q1 = w + 8;
        I4 x0 = I4{0, 0, 0, 0}, x1 = I4{0, 0, 0, 0};
        int fl = 0;
        bool d0 = false, d1 = !(q1 < NRB);
        for (;;) {
            if (!d0) x0 = gload(rs, colx(e, q0) + (uint32_t)lane * 16);
            if (!d1) x1 = gload(rs, colx(e, q1) + (uint32_t)lane * 16);
            d0 = d0 || chunk4_at(x0, (unsigned)e);
            d1 = d1 || chunk4_at(x1, (unsigned)e);
            if (__all(d0 && d1)) break;
            if (__builtin_amdgcn_s_memrealtime() > deadline) { fl |= 2; break; }
            __builtin_amdgcn_s_sleep(1);
        }
        OTF_M2STAMP(e - 1, 1, 0);
        F4 ps = chunk4_vals(x0);
        int f = chunk4_flag(x0);
        if (q1 < NRB) {
            ps += chunk4_vals(x1);
            f |= chunk4_flag(x1);
        }
        gbuf[w][lane] = ps;
        fl |= __any(f) ? 1 : 0;
        if (lane == 0) gfl[w] = fl;
        __syncthreads();
        s4 = gbuf[0][lane];
#pragma unroll
        for (int ww = 1; ww < NW; ++ww) s4 += gbuf[ww][lane];
        int all = 0;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) all |= gfl[ww];
        deadline = __builtin_amdgcn_s_memrealtime() + p.timeout_ticks;
        return all;
    };
    auto to_err = [&](T e) -> double { return p.err_squared ? (double)e : sqrt((double)e); };
    auto stop_ok = [&](double err) -> bool { return p.err_squared ? !(err > p.stop_thr) : (err < p.stop_thr); };

    // ---- prologue: S[0] = K^T u0 (epoch 1)
    {
        T wr[RW];
#pragma unroll
        for (int r = 0; r < RW; ++r) wr[r] = SH ? p.sh.u0[row0 + r] : u0;
        col_partials(wr);
        __syncthreads();
        publish_cols(1, 0);
    }
    int last_good = -1, niter = 0, status = OTF_SK_MAX_ITER, brk = -1, n_err = 0;
    bool done = false;
    int chk = 0;
    T vprev[4] = {v0, v0, v0, v0};  // v of the previous iteration (this lane's columns)
    if (SH) {
#pragma unroll
        for (int k = 0; k < 4; ++k) vprev[k] = p.sh.v0[col0 + k];
    }

    for (int it = 0; it < p.max_iter; ++it) {
        asm volatile("" : "+v"(tid), "+v"(lane));
        const int e = it + 1;
        const bool check = it >= 1 && chk == 0;
        OTF_M2STAMP(it, 0, 0);
        F4 s4;
        const int gf = gather_cols(e, s4);
        OTF_M2STAMP(it, 2, 0);
        if (gf & 2) { status = OTF_SK_TIMEOUT; done = true; break; }
        if (gf & 1) {  // a non-finite u in iteration it - 1 -> revert to it - 2
            last_good = it - 2; niter = it - 1; status = OTF_SK_NUMERICAL_BREAK; brk = it - 1;
            done = true;
            break;
        }
        T vn[4];
        int vbad = 0;
        T eterm = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            vn[k] = bcol[k] / s4[k];
            if (s4[k] == (T)0 || !finite_val(vn[k])) vbad = 1;
            if (check) {  // POT's marginal error of iterate it - 1: v(it - 1) S(it) - b
                const T rr = vprev[k] * s4[k] - bcol[k];
                eterm += rr * rr;
            }
        }
        vbad = __any(vbad) ? 1 : 0;
        if (check && w == 0) eterm = wave_sum<T>(eterm);  // this column tile's error partial
        // row partials over this tile's 256 columns, wave totals (lane L: row L >> 1)
        T rp[RW];
        {
            const F2 v01 = F2{vn[0], vn[1]}, v23 = F2{vn[2], vn[3]};
#pragma unroll
            for (int r = 0; r < RW; ++r) {
                const F2 acc = __builtin_elementwise_fma(kv[r][1], v23, kv[r][0] * v01);
                rp[r] = acc[0] + acc[1];
            }
        }
        const T tot = wave_row_totals32(rp, lane);
        if (it >= 1) chk = chk + 1 == p.check_every ? 0 : chk + 1;
        // publish: lane 8c packs rows 4c .. 4c + 3 (lanes 8c, 8c + 2, 8c + 4, 8c + 6)
        {
            const T t1 = row_shl<2>(tot), t2 = row_shl<4>(tot), t3 = row_shl<6>(tot);
            if ((lane & 7) == 0)
                gstore(rs, rowx(e, cb) + (uint32_t)(w * 8 + (lane >> 3)) * 16,
                       chunk4(F4{tot, t1, t2, t3}, (e & 3) | (vbad << 2)));
        }
        OTF_M2STAMP(it, 3, 0);
        OTF_M2STAMP(it, 10, 448);
        if (check && w == 0 && lane == 1) gstore(rs, rowx(e, cb) + 64 * 16, chunk4(F4{eterm, 0.f, 0.f, 0.f}, e & 3));
        // row hop: members mq, mq + 8 of chunk rc
        I4 x0 = I4{0, 0, 0, 0}, x1 = I4{0, 0, 0, 0};
        int stall = 0;
        {
            const uint32_t o = (uint32_t)(w * 8 + rc) * 16;
            bool d0 = !(mq < NCB), d1 = !(mq + 8 < NCB);
            for (;;) {
                if (!d0) x0 = gload(rs, rowx(e, mq) + o);
                if (!d1) x1 = gload(rs, rowx(e, mq + 8) + o);
                d0 = d0 || chunk4_at(x0, (unsigned)e);
                d1 = d1 || chunk4_at(x1, (unsigned)e);
                if (__all(d0 && d1)) break;
                if (__builtin_amdgcn_s_memrealtime() > deadline) { stall = 1; break; }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        OTF_M2STAMP(it, 4, 0);
        OTF_M2STAMP(it, 9, 448);
        F4 rt = F4{0, 0, 0, 0};
        int rflag = 0;
        if (mq < NCB) { rt = chunk4_vals(x0); rflag |= chunk4_flag(x0); }
        if (mq + 8 < NCB) { rt += chunk4_vals(x1); rflag |= chunk4_flag(x1); }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            T t = rt[k];
            t += wave_xor<T, 8>(t);
            t += wave_xor<T, 16>(t);
            t += wave_xor<T, 32>(t);
            rt[k] = t;
        }
        const int vbad_any = __any(rflag) ? 1 : 0;
        T errv = 0;
        if (check) {
            // the ncb column tiles' error partials, lanes < NCB, fixed order
            T ev = 0;
            if (lane < NCB) {
                I4 xe;
                if (!poll_chunk4(rs, rowx(e, lane) + 64 * 16, (unsigned)e, deadline, xe)) stall = 1;
                ev = chunk4_vals(xe)[0];
            }
            ev += wave_xor<T, 1>(ev);
            ev += wave_xor<T, 2>(ev);
            ev += wave_xor<T, 4>(ev);
            if (NCB > 8) ev += wave_xor<T, 8>(ev);
            errv = __builtin_bit_cast(T, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, ev)));
        }
        stall = __any(stall) ? 1 : 0;
        // u of rows 4 rc .. + 3 (every lane of chunk rc), to every lane by readlane
        T un[RW];
        int badu = 0;
        {
            T uc[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                uc[k] = (T)1 / (rt[k] * ia[k]);
                if (!finite_val(uc[k])) badu = 1;
            }
            badu = __any(badu) ? 1 : 0;
#pragma unroll
            for (int c = 0; c < 8; ++c)
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    un[4 * c + k] = __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, uc[k]), c));
            if (lane < 8)
                *reinterpret_cast<F4*>(&uhist[it & 1][w * RW + 4 * lane]) = F4{uc[0], uc[1], uc[2], uc[3]};
        }
        double err = 0.0;
        int dec = 0;
        if (check) {
            err = to_err(errv);
            if (stop_ok(err)) dec = 1;
        }
        if (dec == 0 && vbad_any) dec = 2;
        col_partials(un);
        if (w == 0) *reinterpret_cast<F4*>(&vhist[it & 1][4 * lane]) = F4{vn[0], vn[1], vn[2], vn[3]};
        if (badu) s_ep[0] = it;
        if (stall) s_ep[1] = it;
        __syncthreads();
        OTF_M2STAMP(it, 5, 0);
        if (s_ep[1] == it) { status = OTF_SK_TIMEOUT; done = true; break; }
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
        OTF_M2STAMP(it, 6, 0);
#pragma unroll
        for (int k = 0; k < 4; ++k) vprev[k] = vn[k];
    }
    if (!done && p.max_iter > 0) {
        // the last iteration's u flags ride in S[max_iter]; its error needs one more
        // exchange of the column tiles' partials
        const int it = p.max_iter - 1;
        const int e = p.max_iter + 1;
        F4 s4;
        const int gf = gather_cols(e, s4);
        if (gf & 2) {
            status = OTF_SK_TIMEOUT;
        } else if (gf & 1) {
            last_good = it - 1; niter = it; status = OTF_SK_NUMERICAL_BREAK; brk = it;
        } else {
            last_good = it; niter = it;
            if ((it % p.check_every) == 0) {
                T eterm = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const T rr = vprev[k] * s4[k] - bcol[k];
                    eterm += rr * rr;
                }
                eterm = wave_sum<T>(eterm);  // every wave, same value
                int stall = 0;
                T errv = eterm;
                if (NCB > 1) {
                    if (w == 0 && lane == 1) gstore(rs, rowx(e, cb) + 64 * 16, chunk4(F4{eterm, 0.f, 0.f, 0.f}, e & 3));
                    T ev = 0;
                    if (lane < NCB) {
                        I4 xe;
                        if (!poll_chunk4(rs, rowx(e, lane) + 64 * 16, (unsigned)e, deadline, xe)) stall = 1;
                        ev = chunk4_vals(xe)[0];
                    }
                    ev += wave_xor<T, 1>(ev);
                    ev += wave_xor<T, 2>(ev);
                    ev += wave_xor<T, 4>(ev);
                    if (NCB > 8) ev += wave_xor<T, 8>(ev);
                    errv = __builtin_bit_cast(T, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, ev)));
                    stall = __any(stall) ? 1 : 0;
                    if (stall) s_ep[1] = e;
                    __syncthreads();
                    stall = s_ep[1] == e;
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
    T uo[RW], vo[4];
#pragma unroll
    for (int r = 0; r < RW; ++r) uo[r] = last_good >= 0 ? uhist[hs][w * RW + r] : SH ? p.sh.u0[row0 + r] : u0;
#pragma unroll
    for (int k = 0; k < 4; ++k) vo[k] = last_good >= 0 ? vhist[hs][4 * lane + k] : SH ? p.sh.v0[col0 + k] : v0;
    if (cb == 0 && lane < RW) {
        T mine = uo[0];
#pragma unroll
        for (int r = 1; r < RW; ++r) if (lane == r) mine = uo[r];
        p.u_out[row0 + lane] = mine;
    }
    if (rb == 0 && w == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) p.v_out[col0 + k] = vo[k];
    }
    if (p.P) {
        using VP = __attribute__((ext_vector_type(4))) TP;
        TP* P = (TP*)p.P + (int64_t)row0 * p.ldp + col0;
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            VP o;
            o[0] = (TP)(uo[r] * kv[r][0][0] * vo[0]);
            o[1] = (TP)(uo[r] * kv[r][0][1] * vo[1]);
            o[2] = (TP)(uo[r] * kv[r][1][0] * vo[2]);
            o[3] = (TP)(uo[r] * kv[r][1][1] * vo[3]);
            *reinterpret_cast<VP*>(P) = o;
            P += p.ldp;
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

struct Mesh2Shape {
    int nrb, ncb;
    size_t row_bytes, col_bytes;
};

Mesh2Shape mesh2_shape(int64_t n, int64_t m) {
    Mesh2Shape s{};
    s.nrb = (int)(n / kM2T);
    s.ncb = (int)(m / kM2T);
    s.row_bytes = 2 * (size_t)s.nrb * s.ncb * kM2RowStride;
    s.col_bytes = 2 * (size_t)s.nrb * s.ncb * kM2ColStride;
    return s;
}
constexpr size_t kMesh2RegBytes = 9 * 256;

template <int NRB, int NCB, typename CT, typename TP>
const void* mesh2_kernel_t(bool sh) {
    return sh ? (const void*)sk_mesh2_kernel<NRB, NCB, CT, TP, true> : (const void*)sk_mesh2_kernel<NRB, NCB, CT, TP, false>;
}
template <typename CT, typename TP>
const void* mesh2_kernel_for(int nrb, int ncb, bool sh) {
    if (nrb == 16 && ncb == 16) return mesh2_kernel_t<16, 16, CT, TP>(sh);
    if (nrb == 16 && ncb == 8) return mesh2_kernel_t<16, 8, CT, TP>(sh);
    if (nrb == 8 && ncb == 16) return mesh2_kernel_t<8, 16, CT, TP>(sh);
    return mesh2_kernel_t<8, 8, CT, TP>(sh);
}

}  // namespace

bool mesh2_supported(int64_t n, int64_t m) {
    if (n % kM2T != 0 || m % kM2T != 0) return false;
    const int64_t nrb = n / kM2T, ncb = m / kM2T;
    return (nrb == 8 || nrb == 16) && (ncb == 8 || ncb == 16);
}

size_t mesh2_region_bytes(int64_t n, int64_t m) {
    if (!mesh2_supported(n, m)) return 0;
    const Mesh2Shape s = mesh2_shape(n, m);
    return kMesh2RegBytes + s.row_bytes + s.col_bytes;
}

// OTF_MESH2: 1 runs the two-hop form for the shapes it takes (read per call)
bool mesh2_enabled() {
    const char* e = getenv("OTF_MESH2");
    return e ? atoi(e) != 0 : false;
}

template <typename CT>
hipError_t run_mesh2(const CT* C, int64_t ldc, int n, int m, const float* a_pad, const float* b_pad,
                     const float* cost_scale, const otf_sinkhorn_opts& o, void* region, float* u_out,
                     float* v_out, void* P_out, int64_t ldp, int P_dtype, otf_sinkhorn_info* info,
                     double* errlog, bool zeroed, hipStream_t s, const ShiftArgs* shift) {
    if (!mesh2_supported(n, m) || !region) return hipErrorInvalidValue;
    if (ldc % 4 != 0 || (P_out && ldp % 4 != 0)) return hipErrorInvalidValue;
    const Mesh2Shape sh = mesh2_shape(n, m);
    const int grid = sh.nrb * sh.ncb;
    if (grid > device_cu_count()) return hipErrorCooperativeLaunchTooLarge;
    SkMesh2Args p{};
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
    p.gran = (char*)region + kMesh2RegBytes;
    p.off_row = 0;
    p.off_col = (uint32_t)sh.row_bytes;
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
    if (shift) p.sh = *shift;
    if (!zeroed) {
        const hipError_t e = hipMemsetAsync(region, 0, mesh2_region_bytes(n, m), s);
        if (e != hipSuccess) return e;
    }
    const bool f64p = P_out && P_dtype == OTF_F64;
    const void* k = f64p ? mesh2_kernel_for<CT, double>(sh.nrb, sh.ncb, shift != nullptr)
                         : mesh2_kernel_for<CT, float>(sh.nrb, sh.ncb, shift != nullptr);
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 512, 0);
    if (e != hipSuccess) return e;
    if (per_cu < 1 || grid > per_cu * device_cu_count()) return hipErrorCooperativeLaunchTooLarge;
    void* args[] = {&p};
    return hipLaunchKernel(k, dim3(grid), dim3(512), args, 0, s);
}

template hipError_t run_mesh2<float>(const float*, int64_t, int, int, const float*, const float*,
                                     const float*, const otf_sinkhorn_opts&, void*, float*, float*,
                                     void*, int64_t, int, otf_sinkhorn_info*, double*, bool,
                                     hipStream_t, const ShiftArgs*);
template hipError_t run_mesh2<_Float16>(const _Float16*, int64_t, int, int, const float*, const float*,
                                        const float*, const otf_sinkhorn_opts&, void*, float*, float*,
                                        void*, int64_t, int, otf_sinkhorn_info*, double*, bool,
                                        hipStream_t, const ShiftArgs*);

}  // namespace otf
