// otf_device.h — device helpers shared by the otfuse HIP kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "otfuse.h"

namespace otf {

constexpr int kWave = 64;

template <typename T> struct Vec;
template <> struct Vec<float> {
    static constexpr int N = 4;
    using type = __attribute__((ext_vector_type(4))) float;
};
template <> struct Vec<double> {
    static constexpr int N = 2;
    using type = __attribute__((ext_vector_type(2))) double;
};

// VEC consecutive cost values as the compute type: a vector load when the cost is
// stored in the compute type, else a narrower vector load (fp16 storage: 8 B for 4
// values) widened in registers.
template <typename T, typename CT>
__device__ __forceinline__ typename Vec<T>::type load_cost(const CT* p) {
    using V = typename Vec<T>::type;
    if constexpr (sizeof(T) == sizeof(CT)) {
        return *reinterpret_cast<const V*>(p);
    } else {
        using H = __attribute__((ext_vector_type(Vec<T>::N))) CT;
        return __builtin_convertvector(*reinterpret_cast<const H*>(p), V);
    }
}

__device__ __forceinline__ float fast_exp(float x) {
    // x is pre-multiplied by log2(e) by the caller: one v_exp_f32.
    return __builtin_amdgcn_exp2f(x);
}
__device__ __forceinline__ double fast_exp(double x) {
    // x is in natural-log units for double (accurate ocml exp).
    return exp(x);
}
// Scale applied to the cost before fast_exp: float wants log2(e) folded in.
template <typename T> __host__ __device__ constexpr double exp_unit();
template <> __host__ __device__ constexpr double exp_unit<float>() { return 1.4426950408889634; }
template <> __host__ __device__ constexpr double exp_unit<double>() { return 1.0; }

template <typename T> __device__ __forceinline__ bool finite_val(T x) {
    return !(isnan(x) || isinf(x));
}

// x of lane (lane ^ O) for O = 1, 2, 4, 8, 16, 32, entirely in the VALU: DPP quad_perm
// (1, 2), DPP row_shl / row_shr + a lane select (4, 8: within a 16-lane row), and the
// gfx950 v_permlane16_swap / v_permlane32_swap (16, 32).  No LDS crossbar round trip
// (ds_bpermute, what __shfl_xor lowers to): a dependent chain of exchanges -- the
// butterfly reductions below -- costs a few cycles per step instead of ~100.
// tools/ubench_xor.hip checks every offset on the device.
template <int O> __device__ __forceinline__ unsigned wave_xor_u32(unsigned x) {
    if constexpr (O == 1) {
        return (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]
    } else if constexpr (O == 2) {
        return (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, true);  // quad_perm [2,3,0,1]
    } else if constexpr (O == 4 || O == 8) {
        const unsigned from_up = (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x100 + O, 0xF, 0xF, true);  // row_shl
        const unsigned from_dn = (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x110 + O, 0xF, 0xF, true);  // row_shr
        return (__lane_id() & O) ? from_dn : from_up;
    } else if constexpr (O == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return (__lane_id() & 16) ? r[0] : r[1];
    } else {
        static_assert(O == 32, "lane offset");
        const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return (__lane_id() & 32) ? r[0] : r[1];
    }
}
template <typename T, int O> __device__ __forceinline__ T wave_xor(T x) {
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, wave_xor_u32<O>(__builtin_bit_cast(unsigned, x)));
    } else {
        static_assert(sizeof(T) == 8, "4- or 8-byte values");
        const unsigned long long b = __builtin_bit_cast(unsigned long long, x);
        const unsigned lo = wave_xor_u32<O>((unsigned)b), hi = wave_xor_u32<O>((unsigned)(b >> 32));
        return __builtin_bit_cast(T, ((unsigned long long)hi << 32) | lo);
    }
}
// runtime offset (a power of two <= 32) -> the compile-time exchange
template <typename T> __device__ __forceinline__ T wave_xor_n(T x, int o) {
    switch (o) {
        case 1: return wave_xor<T, 1>(x);
        case 2: return wave_xor<T, 2>(x);
        case 4: return wave_xor<T, 4>(x);
        case 8: return wave_xor<T, 8>(x);
        case 16: return wave_xor<T, 16>(x);
        default: return wave_xor<T, 32>(x);
    }
}

template <typename T> __device__ __forceinline__ T wave_sum(T x) {
    x += wave_xor<T, 32>(x);
    x += wave_xor<T, 16>(x);
    x += wave_xor<T, 8>(x);
    x += wave_xor<T, 4>(x);
    x += wave_xor<T, 2>(x);
    x += wave_xor<T, 1>(x);
    return x;
}

template <typename T> __device__ __forceinline__ T wave_max(T x) {
    x = fmax(x, wave_xor<T, 32>(x));
    x = fmax(x, wave_xor<T, 16>(x));
    x = fmax(x, wave_xor<T, 8>(x));
    x = fmax(x, wave_xor<T, 4>(x));
    x = fmax(x, wave_xor<T, 2>(x));
    x = fmax(x, wave_xor<T, 1>(x));
    return x;
}

// Reduce R per-lane values across the wave with the halving butterfly: after
// log2(R) exchange steps every lane holds ONE partial (of row rowOf(lane)), then
// the remaining 6 - log2(R) steps finish the sum.  R - 1 + 6 - log2 R shuffles
// instead of 6 R.  On return x[0] of lane L holds the wave total of row
// butterfly_row<R>(L).
template <int R> __device__ __forceinline__ int butterfly_row(int lane) {
    int r = 0;
#pragma unroll
    for (int s = 0, h = R / 2; h >= 1; h >>= 1, ++s)
        if (lane & (1 << s)) r += h;
    return r;
}
// One halving step per template level: H pairs, lane bit 1 << S picks which half a lane
// keeps.  Compile-time H and S keep every index static: the earlier loop form
// (for h = R/2 ...; h >>= 1, ++s) was not unrolled by ROCm 7.2 clang, so x[i] became a
// dynamic register index -- a 15-way compare/select chain per access, ~900 VALU
// instructions for R = 16 instead of ~100 (measured in the mesh engine's ISA).
template <typename T, int R, int H, int S>
__device__ __forceinline__ void wave_sum_step(T (&x)[R], int lane) {
    if constexpr (H >= 1) {
        constexpr int o = 1 << S;
        const bool upper = (lane & o) != 0;
#pragma unroll
        for (int i = 0; i < H; ++i) {
            const T send = upper ? x[i] : x[i + H];
            const T keep = upper ? x[i + H] : x[i];
            x[i] = keep + wave_xor<T, o>(send);
        }
        wave_sum_step<T, R, H / 2, S + 1>(x, lane);
    }
}
// x += x of lane ^ O, ^ 2O, ... ^ 32 (compile-time offsets)
template <typename T, int O> __device__ __forceinline__ void wave_sum_from(T& x) {
    if constexpr (O < kWave) {
        x += wave_xor<T, O>(x);
        wave_sum_from<T, O * 2>(x);
    }
}
template <typename T, int R> __device__ __forceinline__ void wave_sum_multi(T (&x)[R], int lane) {
    static_assert(R >= 1 && R <= 64 && (R & (R - 1)) == 0, "R: a power of two <= 64");
    wave_sum_step<T, R, R / 2, 0>(x, lane);
    wave_sum_from<T, (R > 1 ? R : 1)>(x[0]);
}

// ---- Row totals with the cheap exchanges first ---------------------------------
// 32-bit words of a float / double through one lane exchange
template <typename T, typename F> __device__ __forceinline__ T map_words(T x, F f) {
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, f(__builtin_bit_cast(unsigned, x)));
    } else {
        const unsigned long long b = __builtin_bit_cast(unsigned long long, x);
        const unsigned lo = f((unsigned)b), hi = f((unsigned)(b >> 32));
        return __builtin_bit_cast(T, ((unsigned long long)hi << 32) | lo);
    }
}
// x of another lane by a DPP control: quad_perm 0xB1 (^1), 0x4E (^2), row_half_mirror
// 0x141 (lane i <-> 7 - i within its 8), row_mirror 0x140 (i <-> 15 - i within its 16).
// A plain DPP move with bound_ctrl (every lane of these patterns has a source, so no
// "old" value is read): update_dpp with old = 0 made the compiler zero the destination
// before every move, one extra v_mov per 32-bit word (r05: ~100 per float64 mesh
// iteration).
template <int CTRL, typename T> __device__ __forceinline__ T dpp_lane(T x) {
    return map_words(x, [](unsigned w) { return (unsigned)__builtin_amdgcn_mov_dpp((int)w, CTRL, 0xF, 0xF, true); });
}
// v_permlane32_swap / v_permlane16_swap of (a, b), then the sum of the two results:
// lanes of the lower half (row of 16) end with their a plus the partner half's a, lanes
// of the upper half with their b plus the partner's b -- one keep / send exchange of a
// halving butterfly in two instructions per 32-bit word and one add
template <int O, typename T> __device__ __forceinline__ T swap_sum(T a, T b) {
    static_assert(O == 16 || O == 32, "swap offset");
    if constexpr (sizeof(T) == 4) {
        const auto r = O == 32 ? __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b), false, false)
                               : __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b), false, false);
        return __builtin_bit_cast(T, (unsigned)r[0]) + __builtin_bit_cast(T, (unsigned)r[1]);
    } else {
        const unsigned long long ab = __builtin_bit_cast(unsigned long long, a);
        const unsigned long long bb = __builtin_bit_cast(unsigned long long, b);
        const auto lo = O == 32 ? __builtin_amdgcn_permlane32_swap((unsigned)ab, (unsigned)bb, false, false)
                                : __builtin_amdgcn_permlane16_swap((unsigned)ab, (unsigned)bb, false, false);
        const auto hi = O == 32 ? __builtin_amdgcn_permlane32_swap((unsigned)(ab >> 32), (unsigned)(bb >> 32), false, false)
                                : __builtin_amdgcn_permlane16_swap((unsigned)(ab >> 32), (unsigned)(bb >> 32), false, false);
        const T x = __builtin_bit_cast(T, ((unsigned long long)(unsigned)hi[0] << 32) | (unsigned)lo[0]);
        const T y = __builtin_bit_cast(T, ((unsigned long long)(unsigned)hi[1] << 32) | (unsigned)lo[1]);
        return x + y;
    }
}
// Wave totals of R = 8 or 16 per-lane row partials.  A halving butterfly that spends
// its many-value levels on the cheap exchanges -- lane bits 5 and 4 by the permlane
// swaps (two instructions per pair), bit 3 (and for R = 16 bit 2) by row_mirror /
// row_half_mirror with a keep / send select -- and sums the one remaining value over
// the lanes still to be covered (half mirror, quad ^2, quad ^1).  A mirror's partner
// also differs in the low bits, which the later steps cover, so every step adds two
// disjoint lane sets and every lane that ends with a row holds bitwise the same sum.
// Lane L ends with the total of row L >> (6 - log2 R).  (The generic bits-0-first
// order needs two DPP moves and a select per bit-2 / bit-3 exchange: ~75 VALU for
// R = 16 in float against ~35 here.)
template <typename T, int R>
__device__ __forceinline__ T wave_row_totals(const T (&x)[R], int lane) {
    static_assert(R == 4 || R == 8 || R == 16, "4, 8 or 16 rows per wave");
    if constexpr (R == 4) {
        // lane bits 5 and 4 by the swaps (lane L: row L >> 4), then the 16 of a row
        T t = swap_sum<16>(swap_sum<32>(x[0], x[2]), swap_sum<32>(x[1], x[3]));
        t += dpp_lane<0x140>(t);
        t += dpp_lane<0x141>(t);
        t += dpp_lane<0xB1>(t);
        t += dpp_lane<0x4E>(t);
        return t;
    } else {
    T y[R / 2], z[R / 4];
#pragma unroll
    for (int i = 0; i < R / 2; ++i) y[i] = swap_sum<32>(x[i], x[i + R / 2]);
#pragma unroll
    for (int i = 0; i < R / 4; ++i) z[i] = swap_sum<16>(y[i], y[i + R / 4]);
    const bool b3 = (lane & 8) != 0, b2 = (lane & 4) != 0;
    T t;
    if constexpr (R == 16) {
        T w2[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const T send = b3 ? z[i] : z[i + 2], keep = b3 ? z[i + 2] : z[i];
            w2[i] = keep + dpp_lane<0x140>(send);
        }
        const T send = b2 ? w2[0] : w2[1], keep = b2 ? w2[1] : w2[0];
        t = keep + dpp_lane<0x141>(send);
    } else {
        const T send = b3 ? z[0] : z[1], keep = b3 ? z[1] : z[0];
        t = keep + dpp_lane<0x140>(send);
        t += dpp_lane<0x141>(t);
    }
    t += dpp_lane<0xB1>(t);
    t += dpp_lane<0x4E>(t);
    return t;
    }
}

// Block-wide sum of R values per thread.  `red` is LDS of >= (nwaves + 1) * R
// elements.  Deterministic (fixed order), result broadcast to every thread.
template <typename T, int R>
__device__ __forceinline__ void block_sum_multi(T (&x)[R], T* red) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    wave_sum_multi<T, R>(x, lane);
    if (lane < R) red[wid * R + butterfly_row<R>(lane)] = x[0];
    __syncthreads();
    if (threadIdx.x < R) {
        T s = 0;
        for (int w = 0; w < nw; ++w) s += red[w * R + threadIdx.x];
        red[16 * R + threadIdx.x] = s;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = red[16 * R + r];
}

// Block-wide sums of R values per thread through an LDS transpose (R divides 64,
// blockDim.x a multiple of 64):
//   1. every thread stores its R partials contiguously: tbuf[t*R + r];
//   2. thread t takes row r = t % R, slot q = t / R of Q = NT / R slots and sums
//      tbuf[(q + Q k) * R + r] over k < R — one wave's 64 lanes read 64 consecutive
//      words per step, conflict-free;
//   3. lanes with equal t % R finish with log2(64 / R) xor shuffles, one lane per
//      (wave, row) writes wbuf[w * R + r], and the R row totals are summed over waves.
// Deterministic; 3 barriers; results broadcast in x.  tbuf: NT * R, wbuf: 17 * R.
template <typename T, int R>
__device__ __forceinline__ void block_sum_rows(T (&x)[R], T* tbuf, T* wbuf) {
    static_assert(R >= 1 && R <= 64 && (64 % R) == 0, "R must divide 64");
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int NT = blockDim.x, nw = NT >> 6, Q = NT / R;
#pragma unroll
    for (int r = 0; r < R; ++r) tbuf[t * R + r] = x[r];
    __syncthreads();
    const int r = t % R, q = t / R;
    T s = 0;
#pragma unroll
    for (int k = 0; k < R; ++k) s += tbuf[(q + Q * k) * R + r];
    wave_sum_from<T, R>(s);
    if (lane < R) wbuf[wid * R + lane] = s;
    __syncthreads();
    if (t < R) {
        T tot = 0;
        for (int w = 0; w < nw; ++w) tot += wbuf[w * R + t];
        wbuf[16 * R + t] = tot;
    }
    __syncthreads();
#pragma unroll
    for (int rr = 0; rr < R; ++rr) x[rr] = wbuf[16 * R + rr];
}

template <typename T> __device__ __forceinline__ T block_sum(T x, T* red) {
    T v[1] = {x};
    block_sum_multi<T, 1>(v, red);
    return v[0];
}

}  // namespace otf

// Host-side helpers -----------------------------------------------------------
namespace otf {
int device_cu_count();
int check_hip(hipError_t e);
}  // namespace otf

#define OTF_HIP(call)                                              \
    do {                                                           \
        hipError_t e_ = (call);                                    \
        if (e_ != hipSuccess) return otf::check_hip(e_);           \
    } while (0)
