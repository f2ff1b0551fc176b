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

template <typename T> __device__ __forceinline__ T wave_sum(T x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, kWave);
    return x;
}

template <typename T> __device__ __forceinline__ T wave_max(T x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = fmax(x, __shfl_xor(x, o, kWave));
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
template <typename T, int R> __device__ __forceinline__ void wave_sum_multi(T (&x)[R], int lane) {
    int s = 0;
#pragma unroll
    for (int h = R / 2; h >= 1; h >>= 1, ++s) {
        const int o = 1 << s;
        const bool upper = (lane & o) != 0;
#pragma unroll
        for (int i = 0; i < h; ++i) {
            const T send = upper ? x[i] : x[i + h];
            const T keep = upper ? x[i + h] : x[i];
            x[i] = keep + __shfl_xor(send, o, kWave);
        }
    }
#pragma unroll
    for (int o = (R > 1 ? R : 1); o < kWave; o <<= 1) x[0] += __shfl_xor(x[0], o, kWave);
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
#pragma unroll
    for (int o = R; o < kWave; o <<= 1) s += __shfl_xor(s, o, kWave);
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
