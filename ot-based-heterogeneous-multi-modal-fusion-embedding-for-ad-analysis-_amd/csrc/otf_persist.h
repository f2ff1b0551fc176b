// otf_persist.h — in-launch synchronisation for the persistent Sinkhorn engines
// (resident, tiled, sweep): XCD-hierarchical grid barrier, write-through stores and
// sc1 loads of the column sums, and the shared hand-off of per-iteration sum buffers.
//
// Hand-off form (MI355X microarch guide, inter-workgroup visibility, valid forms):
// producers add with agent-scope float atomics (performed at the memory side) or store
// write-through (sc1); every producing wave drains (s_waitcnt vmcnt(0)) before its
// workgroup arrives on a counter; EVERY consumer load of the handed-off words is a
// 16-B sc1 buffer load to registers (bypasses this CU's L1).  Every spin is bounded by
// s_memrealtime (100 MHz): a barrier that makes no progress for `timeout_ticks` ends
// the solve with OTF_SK_TIMEOUT instead of hanging.  The deadline is re-armed after
// every completed barrier, so only a stall times out, never a long healthy solve.
#pragma once
#include <stdlib.h>

#include "otf_device.h"

namespace otf {

struct SkSync {
    int* reg;   // [8 * 64]  workgroups per XCD (registration, before the first barrier)
    int* xcnt;  // [8 * 64]  arrivals per XCD
    int* top;   // [64]      XCD arrivals
    int* gen;   // [8 * 64]  published epoch per XCD
};

// hierarchical barrier words: reg[8], xcnt[8], top, gen[8], each on a 256-B line
constexpr size_t kSyncBytes = 25 * 64 * sizeof(int);

inline SkSync sync_words(int* base) {
    SkSync s;
    s.reg = base;
    s.xcnt = base + 8 * 64;
    s.top = base + 16 * 64;
    s.gen = base + 17 * 64;
    return s;
}

// Diagnostic build only (-DOTF_STAMPS, tools/stamps_resident.hip, tools/stamps_sweep.hip):
// per-phase wall-clock stamps of the persistent loops; compiled out of the library.
#ifdef OTF_STAMPS
__device__ unsigned long long g_stamps[256 * 16 * 8];
#define OTF_STAMP(it, ph)                                                                   \
    do {                                                                                    \
        if (threadIdx.x == 0 && (it) < 16 && blockIdx.x < 256)                              \
            g_stamps[(blockIdx.x * 16 + (it)) * 8 + (ph)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define OTF_STAMP(it, ph) \
    do {                  \
    } while (0)
#endif

// No progress for this long at a device-wide wait ends the solve with OTF_SK_TIMEOUT:
// 5 s at the 100 MHz s_memrealtime clock, or OTF_STALL_MS from the environment (tests)
constexpr unsigned long long kStallTicks = 500000000ull;
inline unsigned long long stall_ticks() {
    const char* e = getenv("OTF_STALL_MS");
    const long long ms = e ? atoll(e) : 0;
    return ms > 0 ? (unsigned long long)ms * 100000ull : kStallTicks;
}

// The first device-wide wait of a persistent launch (its registration, or its first
// hop) gives up much sooner: a grid that is not co-resident after OTF_REG_MS (default
// 50 ms; a healthy launch registers within microseconds of its prologue) sets
// info->stalled, and the one-workgroup fallback queued behind it (sk_solo_kernel)
// solves the problem instead of the caller waiting out the 5-s stall limit.
inline unsigned long long reg_stall_ticks() {
    const char* e = getenv("OTF_REG_MS");
    const long long ms = e ? atoll(e) : 50;
    const unsigned long long t = (unsigned long long)(ms > 0 ? ms : 50) * 100000ull;
    const unsigned long long st = stall_ticks();
    return t < st ? t : st;
}

// XCD this wave runs on (0..7).  Only speed depends on it (replica choice, grouping).
__device__ __forceinline__ int xcc_id() {
    int v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
    return v;
}

template <typename T> __device__ __forceinline__ T load_agent(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename T>
__device__ __forceinline__ void store_wt(T* p, T v) {  // write-through (sc1) store
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t sums_rsrc(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
template <typename T>
__device__ __forceinline__ typename Vec<T>::type load_sum_vec(__amdgpu_buffer_rsrc_t rs,
                                                              uint32_t byte_off) {
    const auto raw = __builtin_amdgcn_raw_buffer_load_b128(rs, byte_off, 0, 16 /* sc1 */);
    return __builtin_bit_cast(typename Vec<T>::type, raw);
}

// 16-B write-through (sc1) store: the producer side of the no-acquire hand-off
template <typename T>
__device__ __forceinline__ void store_sum_vec(__amdgpu_buffer_rsrc_t rs, uint32_t byte_off,
                                              typename Vec<T>::type v) {
    using I4 = __attribute__((ext_vector_type(4))) int;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(I4, v), rs, byte_off, 0, 16 /* sc1 */);
}

// Epoch-tagged granules (mesh, gather and sweep engines): 16 B = two {value, tag}
// pairs, tag = (epoch << 2) | flags; a consumer polls the data itself (no fence, no
// counter).  sc1 loads; stores sc1 (write-through) across XCCs, plain within one XCC.
using I4 = __attribute__((ext_vector_type(4))) int;
__device__ __forceinline__ I4 chunk2(float v0, float v1, int tag) {
    I4 x;
    x[0] = __builtin_bit_cast(int, v0);
    x[1] = tag;
    x[2] = __builtin_bit_cast(int, v1);
    x[3] = tag;
    return x;
}
__device__ __forceinline__ bool chunk_at(const I4 x, unsigned e) {
    return ((unsigned)x[1] >> 2) == e && ((unsigned)x[3] >> 2) == e;
}
// element copies first (ROCm 7.2: a bit_cast of a vector ELEMENT reads element 0)
__device__ __forceinline__ float chunk_v0(const I4 x) { const int w = x[0]; return __builtin_bit_cast(float, w); }
__device__ __forceinline__ float chunk_v1(const I4 x) { const int w = x[2]; return __builtin_bit_cast(float, w); }

template <int CTRL> __device__ __forceinline__ float dpp_f(float x) { return dpp_lane<CTRL>(x); }

__device__ __forceinline__ I4 gload(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
    return __builtin_bit_cast(I4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16 /* sc1 */));
}
__device__ __forceinline__ void gstore(__amdgpu_buffer_rsrc_t rs, uint32_t off, I4 x) {
    __builtin_amdgcn_raw_buffer_store_b128(x, rs, off, 0, 16 /* sc1 */);
}
// Polls one chunk until both its tags carry epoch e: load - wait - reload.  (Two loads in
// flight, the next issued before the previous is examined, measured slower in r03: the
// mesh's hops 0.72 -> 0.80 us -- the extra request traffic costs more than the finer
// sampling gains.)  False on a stall (deadline passed); x holds the last value loaded.
template <int SLEEP>
__device__ __forceinline__ bool poll_chunk(__amdgpu_buffer_rsrc_t rs, uint32_t off, unsigned e,
                                           unsigned long long deadline, I4& x) {
    for (;;) {
        x = gload(rs, off);
        if (chunk_at(x, e)) return true;
        if (__builtin_amdgcn_s_memrealtime() > deadline) return false;
        __builtin_amdgcn_s_sleep(SLEEP);
    }
}
// Across GPUs (peer-mapped exchange buffers): system-scope (sc0 sc1) stores reach the
// owner's memory over xGMI; the owner polls with system-scope loads
__device__ __forceinline__ I4 gload_sys(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
    return __builtin_bit_cast(I4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 17 /* sc0 sc1 */));
}
__device__ __forceinline__ void gstore_sys(__amdgpu_buffer_rsrc_t rs, uint32_t off, I4 x) {
    __builtin_amdgcn_raw_buffer_store_b128(x, rs, off, 0, 17 /* sc0 sc1 */);
}
// Column-path store: plain (xl = 1) when producer and consumers share one XCC, so the
// line stays in that XCC's L2 -- see the tile assignment in the kernel -- else
// write-through (sc1) like every cross-XCC hop
__device__ __forceinline__ void gstore_col(__amdgpu_buffer_rsrc_t rs, uint32_t off, I4 x, int xl) {
    if (xl)
        __builtin_amdgcn_raw_buffer_store_b128(x, rs, off, 0, 0);
    else
        __builtin_amdgcn_raw_buffer_store_b128(x, rs, off, 0, 16 /* sc1 */);
}

// otf_sinkhorn_info.stalled values.  A mid-solve stall (a hop or barrier that made no
// progress for the stall limit) is reported as OTF_SK_TIMEOUT and never re-solved; only
// a launch whose grid did not become co-resident at its registration is handed to the
// one-workgroup fallback (sk_solo_kernel), which clears the word again.
constexpr int kStallMid = 1;
constexpr int kStallRegistration = 2;
// raise the stalled word to at least v (a registration give-up is never downgraded by a
// workgroup that reports its own timeout afterwards)
__device__ __forceinline__ void mark_stalled(int* stalled, int v) {
    __hip_atomic_fetch_max(stalled, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr int kBarPoison = -(1 << 30);

// Device-wide flat barrier: every wave drains its own memory operations, one lane per
// workgroup arrives on the counter and polls it.  Returns false on a stall (flag
// broadcast via LDS); re-arms `deadline` on success.
// abandon (nullable, the solve's info->stalled): a REGISTRATION barrier may give up.  The
// give-up is a compare-and-swap that poisons the counter (a large negative value) only
// while it is still short of the target, so every workgroup sees exactly one outcome:
// the count completed (nobody can poison it any more) or it was poisoned (waiters and
// late arrivals fail).  The poisoning workgroup then raises abandon to
// kStallRegistration, which queues the solve for the one-workgroup fallback.
__device__ __forceinline__ bool grid_barrier(int* bar, int target, unsigned long long& deadline,
                                             unsigned long long stall, int* s_flag,
                                             int* abandon = nullptr) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        int ok = 1;
        const int old = __hip_atomic_fetch_add(bar, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old < 0) ok = 0;  // arrived after the launch gave up
        while (ok) {
            int c = load_agent(bar);
            if (c >= target) break;
            if (c < 0) { ok = 0; break; }
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() > deadline) {
                if (!abandon) { ok = 0; break; }
                if (__hip_atomic_compare_exchange_strong(bar, &c, kBarPoison, __ATOMIC_RELAXED,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    mark_stalled(abandon, kStallRegistration);
                    ok = 0;
                    break;
                }
                // the count moved since the load: look again (it may have completed)
            }
        }
        *s_flag = ok;
    }
    __syncthreads();
    deadline = __builtin_amdgcn_s_memrealtime() + stall;
    return *s_flag != 0;
}

// XCD-hierarchical grid barrier for epoch e >= 1 (all counters zeroed per call):
// each workgroup arrives on its XCD's counter (~32 adders instead of 256 on one
// word); the last arriver of an XCD (told by the value its add returned) arrives
// on the top counter; the last of those publishes e to every XCD's generation
// word, which only that XCD's workgroups poll.  Placement affects speed only: the
// per-XCD populations are counted in the launch (sync.reg), not assumed.
__device__ __forceinline__ bool xcd_barrier(const SkSync& sy, int xcd, int nx, int nact,
                                            unsigned act_mask, int e,
                                            unsigned long long& deadline,
                                            unsigned long long stall, int* s_flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        int ok = 1;
        const int old = __hip_atomic_fetch_add(sy.xcnt + xcd * 64, 1, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
        if (old == e * nx - 1) {
            const int o2 = __hip_atomic_fetch_add(sy.top, 1, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
            if (o2 == e * nact - 1) {
                for (int x = 0; x < 8; ++x)
                    if (act_mask & (1u << x))
                        __hip_atomic_store(sy.gen + x * 64, e, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        while (__hip_atomic_load(sy.gen + xcd * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < e) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() > deadline) {
                ok = 0;
                break;
            }
        }
        *s_flag = ok;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __syncthreads();
    deadline = __builtin_amdgcn_s_memrealtime() + stall;
    return *s_flag != 0;
}

// Registration on the XCD population + the one flat barrier of a launch; returns
// this XCD's population, the number of active XCDs and their mask in s_pop[0..2].
__device__ __forceinline__ bool register_grid(const SkSync& sy, int* bar, int xcd,
                                              unsigned long long& deadline,
                                              unsigned long long stall, int* s_flag,
                                              int* s_pop) {
    if (threadIdx.x == 0)
        __hip_atomic_fetch_add(sy.reg + xcd * 64, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool ok = grid_barrier(bar, gridDim.x, deadline, stall, s_flag);
    if (threadIdx.x == 0) {
        int nact = 0;
        unsigned mask = 0;
        for (int x = 0; x < 8; ++x) {
            const int c = __hip_atomic_load(sy.reg + x * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (c > 0) {
                ++nact;
                mask |= 1u << x;
            }
        }
        s_pop[0] = __hip_atomic_load(sy.reg + xcd * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_pop[1] = nact;
        s_pop[2] = (int)mask;
    }
    __syncthreads();
    return ok;
}

// Shifted POT kernel (opts.shift, float32 compute; otf_sinkhorn.hip sk_shift_prepass):
// K~_ij = 2^(C_ij ks + A_i + B_j), initial scalings u~0 = 2^-A / n, v~0 = 2^-B / m.
// Passed to the persistent engines that support it (mesh, sweep); null = plain POT kernel.
struct ShiftArgs {
    const float* A;
    const float* B;
    const float* u0;
    const float* v0;
};

// Sweep engine (otf_sweep.hip): persistent streaming solve for costs that do not fit
// the register files.  Host entry points; `region` is zeroed by the launcher.
template <typename T> size_t sweep_region_bytes(int64_t m_pad);
template <typename T, typename CT> bool sweep_supported(int64_t n, int64_t m, int64_t ldc);
// Cross-rank form (otf_sinkhorn_xsweep): this rank's place, the world's exchange buffers
// as mapped here, and the solve's epoch base (identical on every rank).
struct XSweep {
    int rank, world, n_total;
    unsigned ep_base;
    int solve_par;  // parity of this solve in the exchange's sequence (slot set)
    unsigned char* xr[8];
};
constexpr int kXMaxRanks = 8;
// [2 solve parities][2 epoch parities][8 ranks][m_pad] granules: consecutive solves use
// disjoint slot sets, so a rank that starts solve s + 1 can never overwrite a partial of
// solve s that a slower peer has still to read (solve s + 2 cannot start before every
// peer finished solve s: its first exchange needs their solve-(s + 1) partials)
inline size_t xsweep_exchange_bytes(int64_t m_pad) { return (size_t)4 * kXMaxRanks * m_pad * 8; }
template <typename T, typename CT>
hipError_t run_sweep(const CT* C, int64_t ldc, int n, int m, int m_pad, const T* a_pad,
                     const T* b_pad, const T* cost_scale, const otf_sinkhorn_opts& o, void* region,
                     T* u_out, T* v_out, void* P_out, int64_t ldp, int P_dtype,
                     otf_sinkhorn_info* info, double* errlog, hipStream_t s,
                     const XSweep* xs = nullptr, const ShiftArgs* sh = nullptr,
                     void* kbuf = nullptr);

// Gather engine (otf_gather.hip): small problems (<= 16 row tiles, m <= 512), column
// partials exchanged as epoch-tagged granules, no barrier.  `region` is zeroed by the
// launcher unless `zeroed` (the Sinkhorn init kernel did it); gather_region_bytes is 0
// for shapes it does not take.
template <typename T> bool gather_supported(int64_t n, int64_t m);
template <typename T> size_t gather_region_bytes(int64_t n, int64_t m);
template <typename T, typename CT>
hipError_t run_gather(const CT* C, int64_t ldc, int n, int m, const T* a_pad, const T* b_pad,
                      const T* cost_scale, const otf_sinkhorn_opts& o, void* region, T* u_out,
                      T* v_out, void* P_out, int64_t ldp, int P_dtype, otf_sinkhorn_info* info,
                      double* errlog, bool zeroed, hipStream_t s);

// Mesh engine (otf_mesh.hip): float32 problems of 4..64 row tiles x 1..8 column tiles
// of K in registers, row and column reductions as epoch-tagged granule hops (no atomics,
// no barrier).  `region` is zeroed by the launcher; mesh_region_bytes is 0 for shapes
// it does not take.
bool mesh_supported(int64_t n, int64_t m);
size_t mesh_region_bytes(int64_t n, int64_t m);
// float64 form (otf_mesh64.hip): whole 128 x 512 tiles, 4..32 (a power of two) x 1..8, K
// split between the register files and LDS
bool mesh64_supported(int64_t n, int64_t m);
size_t mesh64_region_bytes(int64_t n, int64_t m);
// The pairwise form of the float64 mesh (otf_sinkhorn_pairwise_f64): the cost tile is built
// in the kernel's prologue from the float32 rows X (n x d) and Y (m x d) and their squared
// norms nx, ny, and max-scaled when `scale` (the grid's max: one atomic + a barrier).
struct PairwiseF64 {
    const float* X;
    int64_t ldx;
    const float* Y;
    int64_t ldy;
    int d, euclid, scale;
    const double* nx;  // squared row norms of X (n) and Y (m), float64
    const double* ny;
    double* cmax_out;  // the cost's max (device, nullable)
    uint32_t xbytes, ybytes;
};
// d a multiple of 16, X / Y 16-B aligned with ld a multiple of 4, each < 2 GiB
bool mesh64_pairwise_ok(int64_t n, int64_t m, int64_t d, int64_t ldx, int64_t ldy, const void* X, const void* Y);
hipError_t run_mesh64(const double* C, int64_t ldc, int n, int m, const double* a_pad, const double* b_pad,
                      const double* cost_scale, const otf_sinkhorn_opts& o, void* region, double* u_out,
                      double* v_out, void* P_out, int64_t ldp, int P_dtype, otf_sinkhorn_info* info,
                      double* errlog, bool zeroed, hipStream_t s, const PairwiseF64* pw = nullptr);
// The pairwise form of the float32 mesh (otf_sinkhorn_pairwise_f32): every workgroup builds its
// 128 x 512 cost tile in the prologue on v_mfma_f32_16x16x32_f16 from the split-fp16 images of
// the float32 rows (hi / lo, power-of-two row scales: split16_prep2_kernel's), in
// cost_big16_kernel's per-block MFMA order and epilogue, so C -- and the whole solve -- is
// bitwise the two-call path's; the grid agrees on max(C) (scale) before K = exp(-C / (reg max)).
struct PairwiseF32 {
    const _Float16* Xh;  // n x ldh hi / lo images of X, m x ldh of Y (ldh = d rounded up to 64)
    const _Float16* Xl;
    const _Float16* Yh;
    const _Float16* Yl;
    int64_t ldh;
    const float* xs;  // inverse row scales and squared norms of X (n) and Y (m)
    const float* xx;
    const float* ys;
    const float* yy;
    int kpad, euclid, scale;
    float* cmax_out;  // the cost's max (device, nullable)
    uint32_t xbytes, ybytes;  // image bytes (buffer bounds)
};
// whole 128 x 512 tiles the float32 mesh takes (n % 128 == 0, m % 512 == 0)
bool mesh_pairwise_ok(int64_t n, int64_t m, int64_t d);
template <typename CT>
hipError_t run_mesh(const CT* C, int64_t ldc, int n, int m, const float* a_pad, const float* b_pad,
                    const float* cost_scale, const otf_sinkhorn_opts& o, void* region, float* u_out,
                    float* v_out, void* P_out, int64_t ldp, int P_dtype, otf_sinkhorn_info* info,
                    double* errlog, bool zeroed, hipStream_t s, const ShiftArgs* sh = nullptr,
                    const XSweep* xs = nullptr, const PairwiseF32* pw = nullptr);
// Split-fp16 images of two float32 operands (otf_cost.hip, split16_prep2_kernel) carved from
// `ws` (otf_cost_ex_workspace_size(n, m, d, OTF_F32) bytes), for the fused float32 pairwise
// solve; cmax_word (nullable) is zeroed by the same launch.
struct Split16Images {
    _Float16 *Xh, *Xl, *Yh, *Yl;
    float *xs, *xx, *ys, *yy;
    int64_t ldh;
};
hipError_t split16_images(const float* X, int64_t ldx, int n, const float* Y, int64_t ldy, int m, int d,
                          void* ws, Split16Images& out, unsigned int* cmax_word, hipStream_t s);

}  // namespace otf
