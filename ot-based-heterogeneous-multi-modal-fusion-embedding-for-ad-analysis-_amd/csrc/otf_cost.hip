// otf_cost.hip — pairwise embedding cost on MFMA (gfx950).
//
// Replaces ot.dist(x, y, metric) (+ "C /= C.max()") at MRI_PET_OT_nojax.py:70-75 and
// PointCloud(x, y, scale_cost="max_cost") at MRI_PET_OT_OT_per_epoch_attn.py:155-156 /
// perturbot/perturbot/match/ott_egwl.py:350.  POT's euclidean_distances expansion
//     C = max(|x|^2 + |y|^2 - 2 X Y^T, 0)   [sqrt for 'euclidean'; diag = 0 when X is Y]
// with the X Y^T contraction on v_mfma_f32_32x32x2_f32 (exact f32 FMA chain: the cost
// feeds exp(-C/reg), where a bf16 contraction's ~1e-3 error would break the 1e-4
// plan tolerance).  The squared norms are folded into the same pass from the staged
// tiles, and the global max for scale_cost="max_cost" is reduced in the epilogue
// (one uint atomicMax per workgroup), so C is written exactly once.
//
// Tile: 128 x 128 per 256-thread workgroup (2 x 2 waves, 64 x 64 per wave as 2 x 2
// MFMA 32x32 tiles), BK = 32, LDS double buffer in k-major [BK][128 + 1] images
// (row-contiguous fragment reads, conflict-free transposed writes), XCD-grouped
// block order.
#include "otf_persist.h"

namespace otf {
namespace {

constexpr int BM = 128, BN = 128, BK = 32, LDSW = BM + 1;
using f32x16 = __attribute__((ext_vector_type(16))) float;

// XCD-contiguous tile index wg -> (tile row, tile column) in column bands of
// TILE_GROUP tile rows: the ~64 tiles an XCD runs at once form an 8 x 8 block, whose
// X and Y panels (2 + 2 MB in split-fp16) stay in that XCD's 4 MB L2 -- row-major
// order made them span 2 tile rows x ALL of Y, streamed from the MALL per tile row.
constexpr int TILE_GROUP = 8;
__device__ __forceinline__ void grouped_tile(int wg, int nwg, int tiles_n, int& tm, int& tn) {
    const int tiles_m = nwg / tiles_n;
    const int per_group = TILE_GROUP * tiles_n;
    const int first_m = (wg / per_group) * TILE_GROUP;
    const int gsize = min(tiles_m - first_m, TILE_GROUP);
    const int li = wg % per_group;
    tm = first_m + li % gsize;
    tn = li / gsize;
}

// Global max of non-negative floats as a uint bit pattern: ONE atomic per 256-thread
// workgroup at most (a per-wave atomic made every tile's waves queue on one address).
__device__ __forceinline__ void block_max_publish(unsigned int* cmax, float lmax) {
    __shared__ float wmx[4];
    lmax = wave_max(lmax);
    if ((threadIdx.x & 63) == 0) wmx[threadIdx.x >> 6] = lmax;
    __syncthreads();
    if (threadIdx.x == 0) {
        // cmax only grows: a coherent read at or above this tile's max makes the atomic
        // redundant, so after the first tiles almost none are issued.
        const unsigned int v = __float_as_uint(fmaxf(fmaxf(wmx[0], wmx[1]), fmaxf(wmx[2], wmx[3])));
        if (v > __hip_atomic_load(cmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(cmax, v);
    }
}

using f32x4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ f32x4 load4(const float* base, int64_t ld, int row, int nrows, int k,
                                       int kmax, bool vec_ok) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (row >= nrows) return v;
    const float* p = base + (int64_t)row * ld + k;
    if (vec_ok && k + 3 < kmax) {
        v = *reinterpret_cast<const f32x4*>(p);
    } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (k + e < kmax) v[e] = p[e];
    }
    return v;
}

__global__ __launch_bounds__(256) void cost_pairwise_kernel(
    const float* __restrict__ X, int64_t ldx, const float* __restrict__ Y, int64_t ldy, int n,
    int m, int d, int metric, int zero_diag, float* __restrict__ C, int64_t ldc,
    unsigned int* cmax, int tiles_n, bool vec_ok) {
    __shared__ float As[2][BK][LDSW];
    __shared__ float Bs[2][BK][LDSW];
    __shared__ float sxx[BM], syy[BN];

    // XCD-grouped bijective block order: blocks b and b+8 share an XCD, give each
    // XCD a contiguous run of tiles (same X row panel, streaming Y panels).
    const int nwg = gridDim.x;
    const int bid = blockIdx.x;
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    int tm, tn;
    grouped_tile(wg, nwg, tiles_n, tm, tn);
    const int i0 = tm * BM, j0 = tn * BN;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int lrow = tid >> 3, lk = (tid & 7) * 4;

    f32x4 ra[4], rb[4];
    float nx[4] = {0.f, 0.f, 0.f, 0.f}, ny[4] = {0.f, 0.f, 0.f, 0.f};
    f32x16 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

    auto gload = [&](int k0) {
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
            ra[qq] = load4(X, ldx, i0 + lrow + 32 * qq, n, k0 + lk, d, vec_ok);
            rb[qq] = load4(Y, ldy, j0 + lrow + 32 * qq, m, k0 + lk, d, vec_ok);
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                As[buf][lk + e][lrow + 32 * qq] = ra[qq][e];
                Bs[buf][lk + e][lrow + 32 * qq] = rb[qq][e];
                nx[qq] = fmaf(ra[qq][e], ra[qq][e], nx[qq]);
                ny[qq] = fmaf(rb[qq][e], rb[qq][e], ny[qq]);
            }
        }
    };

    const int nk = (d + BK - 1) / BK;
    gload(0);
    lstore(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) gload((kt + 1) * BK);
#pragma unroll
        for (int kk = 0; kk < BK / 2; ++kk) {
            const int k = 2 * kk + (lane >> 5);
            float a[2], b[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                a[t] = As[buf][k][wm * 64 + t * 32 + (lane & 31)];
                b[t] = Bs[buf][k][wn * 64 + t * 32 + (lane & 31)];
            }
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
#pragma unroll
                for (int nj = 0; nj < 2; ++nj)
                    acc[mi][nj] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[mi], b[nj], acc[mi][nj], 0, 0, 0);
        }
        if (kt + 1 < nk) lstore(buf ^ 1);
        __syncthreads();
    }

    // squared norms: the 8 lanes sharing a staged row hold its partial sums
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
        float sx = nx[qq], sy = ny[qq];
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) {
            sx += wave_xor_n<float>(sx, o);
            sy += wave_xor_n<float>(sy, o);
        }
        if ((tid & 7) == 0) {
            sxx[lrow + 32 * qq] = sx;
            syy[lrow + 32 * qq] = sy;
        }
    }
    __syncthreads();

    float lmax = 0.f;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int nj = 0; nj < 2; ++nj)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int rl = wm * 64 + mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
                const int cl = wn * 64 + nj * 32 + (lane & 31);
                const int gi = i0 + rl, gj = j0 + cl;
                float c = sxx[rl] + syy[cl] - 2.f * acc[mi][nj][e];
                c = c > 0.f ? c : 0.f;
                if (metric == OTF_EUCLIDEAN) c = sqrtf(c);
                if (zero_diag && gi == gj) c = 0.f;
                if (gi < n && gj < m) {
                    C[(int64_t)gi * ldc + gj] = c;
                    lmax = fmaxf(lmax, c);
                }
            }
    if (cmax) block_max_publish(cmax, lmax);
}

template <typename T>
__global__ void scale_inplace_kernel(T* C, int64_t n, int64_t m, int64_t ldc, const T* s) {
    const T inv = s[0];
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n * m;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = t / m, j = t % m;
        C[i * ldc + j] = C[i * ldc + j] / inv;
    }
}

// ============================================================================
// Split-fp16 path: fp32-accurate X Y^T at the fp16 MFMA rate.
// Every row is scaled by a power of two s (max |x s| in [2^14, 2^15)) and split as
// x s = hi + lo with hi = fp16(x s), lo = fp16(x s - hi): 22 significant bits.
// x.y = (hi_x hi_y + hi_x lo_y + lo_x hi_y) / (s_x s_y) + O(2^-22) — three
// v_mfma_f32_32x32x16_f16 per 16-deep K step (fp16 products are exact in the fp32
// accumulator) instead of eight v_mfma_f32_32x32x2_f32: ~5x the MFMA rate.
// ============================================================================
using f16x8 = __attribute__((ext_vector_type(8))) _Float16;
constexpr int SBK = 64;        // K per LDS stage (the fp16 images are padded to it)
constexpr int SLD = SBK + 8;   // padded LDS row (144 B): conflict-free ds_read_b128
constexpr int SCPR = SBK / 8;  // 16-B chunks per row per stage
constexpr int SCPT = BM * SCPR / 256;  // chunks per thread per image

// Split-fp16 images of both operands in ONE launch, one wavefront per row (4 rows per
// 256-thread workgroup, wave reductions, no workgroup barriers): squared norm (fp32)
// and the fp16 image(s) of the row, zero-padded to ldh.
//   SPLIT (fp32 input): power-of-two scale s, hi = fp16(x s), lo = fp16(x s - hi);
//   !SPLIT (fp16 input): hi = x, inv_scale = 1.
// max_norm (nullable): running max of the squared norms (bit pattern, >= 0).
// (Was one 256-thread workgroup per row and one launch per operand: 2 x 9 us at
// 4096 x 512.)
template <typename TI> struct PrepSide {
    const TI* X;
    int64_t ldx;
    int n;
    _Float16* hi;
    _Float16* lo;
    float* inv_scale;
    float* norm;
    unsigned int* max_norm;  // nullable
};

template <typename TI, bool SPLIT>
__global__ __launch_bounds__(256) void split16_prep2_kernel(PrepSide<TI> A, PrepSide<TI> B, int d,
                                                           int ldh, int vec, unsigned int* zero_word,
                                                           float* one_word) {
    // the cost kernel's running max (zeroed) and the fp32-storage unit (1.0), written here
    // instead of two memset launches ahead of the cost kernel
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (zero_word) *zero_word = 0u;
        if (one_word) *one_word = 1.0f;
    }
    // lane handles 8 consecutive elements per 512-wide pass: 16-B (fp16) / 2 x 16-B
    // (fp32) loads when the rows allow it, 16-B image stores; h == nullptr: norms only
    // (the fp16 input is its own image)
    using TV = __attribute__((ext_vector_type(8))) TI;
    using H8 = __attribute__((ext_vector_type(8))) _Float16;
    const int lane = threadIdx.x & 63;
    const int total = A.n + B.n;
    float nmax[2] = {0.f, 0.f};
    for (int row = blockIdx.x * 4 + (threadIdx.x >> 6); row < total; row += gridDim.x * 4) {
        const bool sb = row >= A.n;
        const PrepSide<TI>& P = sb ? B : A;
        const int r = sb ? row - A.n : row;
        const TI* x = P.X + (int64_t)r * P.ldx;
        auto load8 = [&](int k0, float (&v)[8]) {
            if (vec && k0 + 8 <= d) {
                const TV t = *reinterpret_cast<const TV*>(x + k0);
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = (float)t[e];
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = k0 + e < d ? (float)x[k0 + e] : 0.f;
            }
        };
        float mx = 0.f, s2 = 0.f;
        for (int k0 = 8 * lane; k0 < d; k0 += 512) {
            float v[8];
            load8(k0, v);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                mx = fmaxf(mx, fabsf(v[e]));
                s2 = fmaf(v[e], v[e], s2);
            }
        }
        s2 = wave_sum(s2);
        int e = 0;
        if (SPLIT) {
            mx = wave_max(mx);
            e = mx > 0.f ? ilogbf(mx) : 0;
        }
        const float sc = SPLIT ? ldexpf(1.0f, 14 - e) : 1.0f;
        if (P.hi) {
            _Float16* hrow = P.hi + (int64_t)r * ldh;
            _Float16* lrow = SPLIT ? P.lo + (int64_t)r * ldh : nullptr;
            for (int k0 = 8 * lane; k0 < ldh; k0 += 512) {
                float v[8];
                load8(k0, v);
                H8 hv, lv;
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const float w = v[q] * sc;
                    hv[q] = (_Float16)w;
                    lv[q] = (_Float16)(w - (float)hv[q]);
                }
                *reinterpret_cast<H8*>(hrow + k0) = hv;
                if (SPLIT) *reinterpret_cast<H8*>(lrow + k0) = lv;
            }
        }
        if (lane == 0) {
            P.inv_scale[r] = SPLIT ? ldexpf(1.0f, e - 14) : 1.0f;
            P.norm[r] = s2;
            nmax[sb ? 1 : 0] = fmaxf(nmax[sb ? 1 : 0], s2);
        }
    }
    // one max per workgroup, and only when it raises the running max: per-wave
    // atomics on one address serialised to ~10 ns each (16384 rows: 190 us)
    __shared__ float pmx[2][4];
    if (lane == 0) {
        pmx[0][threadIdx.x >> 6] = nmax[0];
        pmx[1][threadIdx.x >> 6] = nmax[1];
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        unsigned int* dst = threadIdx.x == 0 ? A.max_norm : B.max_norm;
        const float* v = pmx[threadIdx.x];
        const float mx = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
        if (dst && mx > 0.f &&
            __float_as_uint(mx) > __hip_atomic_load(dst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            atomicMax(dst, __float_as_uint(mx));
    }
}

// fp16 cost storage scale: 2^-k with 2^k >= the largest possible cost given the row
// norms ((|x|max + |y|max)^2, or its root for the Euclidean metric); exact in fp16.
__global__ void cost_store_scale_kernel(const unsigned int* max_norms, int metric, float* scale,
                                        float* unit) {
    const float nx = __uint_as_float(max_norms[0]), ny = __uint_as_float(max_norms[1]);
    float bound = sqrtf(nx) + sqrtf(ny);
    if (metric != OTF_EUCLIDEAN) bound = bound * bound;
    int k = 0;
    if (bound > 0.f && isfinite(bound)) {
        k = ilogbf(bound) + 1;  // 2^k > bound
        k = k < -100 ? -100 : k;
    }
    scale[0] = ldexpf(1.0f, -k);
    if (unit) unit[0] = ldexpf(1.0f, k);
}

// 128x128 output tile per 256-thread workgroup on v_mfma_f32_32x32x16_f16.
// NS = 3: split-fp16 (hi.hi + hi.lo + lo.hi, fp32-accurate); NS = 1: fp16 inputs.
// TC: stored cost type (float, or _Float16 scaled by *store_scale).
template <int NS, typename TC>
__global__ __launch_bounds__(256) void cost_split16_kernel(
    const _Float16* __restrict__ Xh, const _Float16* __restrict__ Xl, const float* __restrict__ xs,
    const float* __restrict__ xx, const _Float16* __restrict__ Yh, const _Float16* __restrict__ Yl,
    const float* __restrict__ ys, const float* __restrict__ yy, int64_t ldxh, int64_t ldyh, int n, int m, int kpad,
    int metric, int zero_diag, TC* __restrict__ C, int64_t ldc, unsigned int* cmax, int tiles_n,
    const float* __restrict__ store_scale) {
    constexpr int NI = NS == 3 ? 2 : 1;  // fp16 images per operand
    __shared__ __attribute__((aligned(16))) _Float16 As[NI][BM][SLD];  // [hi|lo][row][k]
    __shared__ __attribute__((aligned(16))) _Float16 Bs[NI][BN][SLD];
    __shared__ float sxs[BM], sxx[BM];  // row scale / squared norm of this tile's rows

    const int nwg = gridDim.x, bid = blockIdx.x;
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    int tm, tn;
    grouped_tile(wg, nwg, tiles_n, tm, tn);
    const int i0 = tm * BM, j0 = tn * BN;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;

    f32x16 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

    // staging: a 128-row x 32-half tile is 512 16-B chunks; 256 threads x 2 chunks,
    // for each of {A hi, A lo, B hi, B lo} (lo only when NS == 3)
    using u4 = __attribute__((ext_vector_type(4))) unsigned int;
    u4 st[SCPT][2 * NI];
    auto gload = [&](int k0) {
#pragma unroll
        for (int c = 0; c < SCPT; ++c) {
            const int chunk = tid + 256 * c;
            const int row = chunk / SCPR, kc = (chunk % SCPR) * 8;
            const int gi = i0 + row < n ? i0 + row : n - 1;
            const int gj = j0 + row < m ? j0 + row : m - 1;
            st[c][0] = *reinterpret_cast<const u4*>(Xh + (int64_t)gi * ldxh + k0 + kc);
            st[c][NI] = *reinterpret_cast<const u4*>(Yh + (int64_t)gj * ldyh + k0 + kc);
            if (NI == 2) {
                st[c][1] = *reinterpret_cast<const u4*>(Xl + (int64_t)gi * ldxh + k0 + kc);
                st[c][NI + 1] = *reinterpret_cast<const u4*>(Yl + (int64_t)gj * ldyh + k0 + kc);
            }
        }
    };
    auto lstore = [&]() {
#pragma unroll
        for (int c = 0; c < SCPT; ++c) {
            const int chunk = tid + 256 * c;
            const int row = chunk / SCPR, kc = (chunk % SCPR) * 8;
#pragma unroll
            for (int h = 0; h < NI; ++h) {
                *reinterpret_cast<u4*>(&As[h][row][kc]) = st[c][h];
                *reinterpret_cast<u4*>(&Bs[h][row][kc]) = st[c][NI + h];
            }
        }
    };

    // epilogue operands, fetched up front (their latency hides under the main loop):
    // the tile's 128 row factors to LDS, this lane's 2 column factors to registers
    if (tid < BM) {
        const int gi = i0 + tid < n ? i0 + tid : n - 1;
        sxs[tid] = xs[gi];
        sxx[tid] = xx[gi];
    }
    float cys[2], cyy[2];
#pragma unroll
    for (int nj = 0; nj < 2; ++nj) {
        const int gj0 = j0 + wn * 64 + nj * 32 + (lane & 31);
        const int gj = gj0 < m ? gj0 : m - 1;
        cys[nj] = ys[gj];
        cyy[nj] = yy[gj];
    }

    const int nk = kpad / SBK;
    gload(0);
    for (int kt = 0; kt < nk; ++kt) {
        __syncthreads();  // previous stage fully consumed
        lstore();
        __syncthreads();
        if (kt + 1 < nk) gload((kt + 1) * SBK);
#pragma unroll
        for (int ks = 0; ks < SBK / 16; ++ks) {
            const int kk = ks * 16 + 8 * (lane >> 5);
            f16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int ar = wm * 64 + t * 32 + (lane & 31);
                const int br = wn * 64 + t * 32 + (lane & 31);
                ah[t] = *reinterpret_cast<const f16x8*>(&As[0][ar][kk]);
                bh[t] = *reinterpret_cast<const f16x8*>(&Bs[0][br][kk]);
                if (NI == 2) {
                    al[t] = *reinterpret_cast<const f16x8*>(&As[NI - 1][ar][kk]);
                    bl[t] = *reinterpret_cast<const f16x8*>(&Bs[NI - 1][br][kk]);
                }
            }
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
#pragma unroll
                for (int nj = 0; nj < 2; ++nj) {
                    if (NS == 3) {
                        acc[mi][nj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[mi], bh[nj], acc[mi][nj], 0, 0, 0);
                        acc[mi][nj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[mi], bl[nj], acc[mi][nj], 0, 0, 0);
                    }
                    acc[mi][nj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[mi], bh[nj], acc[mi][nj], 0, 0, 0);
                }
        }
    }

    const float os = store_scale ? store_scale[0] : 1.0f;
    float lmax = 0.f;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int nj = 0; nj < 2; ++nj)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int rl = wm * 64 + mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
                const int cl = wn * 64 + nj * 32 + (lane & 31);
                const int gi = i0 + rl, gj = j0 + cl;
                if (gi < n && gj < m) {
                    const float dot = acc[mi][nj][e] * sxs[rl] * cys[nj];
                    float c = sxx[rl] + cyy[nj] - 2.f * dot;
                    c = c > 0.f ? c : 0.f;
                    if (metric == OTF_EUCLIDEAN) c = sqrtf(c);
                    if (zero_diag && gi == gj) c = 0.f;
                    const TC cs = (TC)(c * os);
#if defined(OTF_COST_ABLATE) && (OTF_COST_ABLATE & 1)
                    if (c == -12345.f)  // diagnostic (tools/ubench_cost.hip): no cost stores
#endif
                    C[(int64_t)gi * ldc + gj] = cs;
                    lmax = fmaxf(lmax, (float)cs);
                }
            }
    if (cmax) block_max_publish(cmax, lmax);
}

// 256 x 256 output tile per 512-thread workgroup for large problems (one tile per CU at
// N = 4096): twice the arithmetic intensity of the 128 x 128 tile, whose 64 KB of operand
// fetch per 48 MFMAs per wave outran the per-CU L2 / Infinity Cache rate (MFMA busy
// 20-28 %).  8 waves = 4 along M x 2 along N, each 64 x 128 = 2 x 4 MFMA 32x32 tiles
// (128 accumulators).  32-deep K stages, double-buffered in LDS (2 x 64 KB for the
// split-fp16 images); the next stage's 16-B global loads are in registers while the
// current stage computes, so one barrier per stage.  LDS rows are 64 B with the 16-B
// chunk index XORed with (row >> 2) & 3: 16 consecutive rows of one ds_read_b128 phase
// (and 4 rows x 4 chunks of a ds_write_b128 phase) hit 16 distinct 16-B bank groups.
constexpr int GBM = 256, GBN = 256, GBK = 32, GCPR = GBK / 8;

// Cost values of one 256 x 256 tile from its 8 waves' accumulators (wave (wm, wn): rows
// wm*64 .., columns wn*128 ..): c = max(sxx_r + cyy_c - 2 sxs_r cys_c acc, 0) as ONE fma
// per element -- k = -2 sxs_r cys_c is exact (the row scales are powers of two), so this
// is bit-identical to (sxx_r + cyy_c) - 2 dot -- stored through a buffer descriptor at
// the tile's corner with the row step of element e a scalar offset (no 64-bit address
// per element).  The metric and the whole-tile test are template arguments (one uniform
// branch per tile, not per element); a row's norm terms are read once for its 4 column
// blocks.  Returns the max of the stored values (the fp16 rounding is monotone).
template <typename TC, bool EUC, bool WHOLE>
__device__ __forceinline__ float epilogue_tile256_t(const f32x16 (&acc)[2][4], const float* sxs, const float* sxx,
                                                    const float (&cys)[4], const float (&cyy)[4], int wm, int wn,
                                                    int lane, int i0, int j0, int n, int m, int zero_diag, TC* C,
                                                    int64_t ldc, float os) {
    const __amdgpu_buffer_rsrc_t ct =
        __builtin_amdgcn_make_buffer_rsrc((void*)(C + (int64_t)i0 * ldc + j0), 0, 0x7fffffff, 0x00020000);
    const int r0 = wm * 64 + 4 * (lane >> 5);
    float cy2[4];
    int cl[4];
#pragma unroll
    for (int nj = 0; nj < 4; ++nj) {
        cy2[nj] = -2.f * cys[nj];
        cl[nj] = wn * 128 + nj * 32 + (lane & 31);
    }
    float lmax = 0.f;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
        __builtin_amdgcn_sched_barrier(0);
        uint32_t vb[4];
#pragma unroll
        for (int nj = 0; nj < 4; ++nj) {
            vb[nj] = (uint32_t)((r0 + mi * 32) * (int)ldc + cl[nj]) * (uint32_t)sizeof(TC);
            asm volatile("" : "+v"(vb[nj]));
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int rl = r0 + mi * 32 + (e & 3) + 8 * (e >> 2);
            const float a = sxs[rl], b = sxx[rl];
            const uint32_t so = (uint32_t)(((e & 3) + 8 * (e >> 2)) * (int)ldc) * (uint32_t)sizeof(TC);
#pragma unroll
            for (int nj = 0; nj < 4; ++nj) {
                float c = fmaf(acc[mi][nj][e], a * cy2[nj], b + cyy[nj]);
                c = fmaxf(c, 0.f);  // (a NaN maps to 0 either way)
                if constexpr (EUC) c = sqrtf(c);
                if constexpr (!WHOLE) {
                    if (i0 + rl >= n || j0 + cl[nj] >= m) continue;
                    if (zero_diag && i0 + rl == j0 + cl[nj]) c = 0.f;
                }
                lmax = fmaxf(lmax, c);
#if defined(OTF_COST_ABLATE) && (OTF_COST_ABLATE & 1)
                if (c == -12345.f)  // diagnostic (tools/ubench_cost.hip): no cost stores
#endif
                {
                    if constexpr (sizeof(TC) == 4)
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, c * os), ct, vb[nj], so, 0);
                    else
                        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, (TC)(c * os)), ct, vb[nj], so, 0);
                }
            }
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    return (float)(TC)(lmax * os);
}
template <typename TC>
__device__ __forceinline__ float epilogue_tile256(const f32x16 (&acc)[2][4], const float* sxs, const float* sxx,
                                                  const float (&cys)[4], const float (&cyy)[4], int wm, int wn,
                                                  int lane, int i0, int j0, int n, int m, int metric,
                                                  int zero_diag, TC* C, int64_t ldc, float os) {
    const bool whole = i0 + 256 <= n && j0 + 256 <= m && !(zero_diag && i0 == j0);
    if (metric == OTF_EUCLIDEAN) {
        if (whole)
            return epilogue_tile256_t<TC, true, true>(acc, sxs, sxx, cys, cyy, wm, wn, lane, i0, j0, n, m, zero_diag, C, ldc, os);
        return epilogue_tile256_t<TC, true, false>(acc, sxs, sxx, cys, cyy, wm, wn, lane, i0, j0, n, m, zero_diag, C, ldc, os);
    }
    if (whole)
        return epilogue_tile256_t<TC, false, true>(acc, sxs, sxx, cys, cyy, wm, wn, lane, i0, j0, n, m, zero_diag, C, ldc, os);
    return epilogue_tile256_t<TC, false, false>(acc, sxs, sxx, cys, cyy, wm, wn, lane, i0, j0, n, m, zero_diag, C, ldc, os);
}
__device__ __forceinline__ int gswz(int row, int kc) { return row * GBK + ((kc ^ ((row >> 2) & 3)) << 3); }

// Diagnostic build only (-DOTF_COST_STAMPS, tools/ubench_cost.hip): wave 0's wall clock
// at the phases of the 256x256 cost kernels per workgroup
#ifdef OTF_COST_STAMPS
__device__ unsigned long long g_cst[1024 * 8];
#define OTF_CST(k)                                                                            \
    do {                                                                                      \
        if (threadIdx.x == 0 && blockIdx.x < 1024)                                            \
            g_cst[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime();                   \
    } while (0)
#else
#define OTF_CST(k) \
    do {           \
    } while (0)
#endif
template <int NS, typename TC>
__global__ __launch_bounds__(512) void cost_big_kernel(
    const _Float16* __restrict__ Xh, const _Float16* __restrict__ Xl, const float* __restrict__ xs,
    const float* __restrict__ xx, const _Float16* __restrict__ Yh, const _Float16* __restrict__ Yl,
    const float* __restrict__ ys, const float* __restrict__ yy, int64_t ldxh, int64_t ldyh, int n, int m, int kpad,
    int metric, int zero_diag, TC* __restrict__ C, int64_t ldc, unsigned int* cmax, int tiles_n,
    const float* __restrict__ store_scale) {
    constexpr int NI = NS == 3 ? 2 : 1;           // fp16 images per operand
    constexpr int NCH = GBM * GCPR / 512;         // 16-B chunks per thread per image per stage
    __shared__ __attribute__((aligned(16))) _Float16 As[2][NI][GBM * GBK];
    __shared__ __attribute__((aligned(16))) _Float16 Bs[2][NI][GBN * GBK];
    __shared__ float sxs[GBM], sxx[GBM];
    __shared__ float wmx[8];

    OTF_CST(0);
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    int tm, tn;
    grouped_tile(wg, nwg, tiles_n, tm, tn);
    const int i0 = tm * GBM, j0 = tn * GBN;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;

    f32x16 acc[2][4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

    using u4 = __attribute__((ext_vector_type(4))) unsigned int;
    u4 st[NCH][2 * NI];
    auto gload = [&](int k0) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int chunk = tid + 512 * c;
            const int row = chunk / GCPR, kc = (chunk % GCPR) * 8;
            const int gi = i0 + row < n ? i0 + row : n - 1;
            const int gj = j0 + row < m ? j0 + row : m - 1;
            st[c][0] = *reinterpret_cast<const u4*>(Xh + (int64_t)gi * ldxh + k0 + kc);
            st[c][NI] = *reinterpret_cast<const u4*>(Yh + (int64_t)gj * ldyh + k0 + kc);
            if (NI == 2) {
                st[c][1] = *reinterpret_cast<const u4*>(Xl + (int64_t)gi * ldxh + k0 + kc);
                st[c][NI + 1] = *reinterpret_cast<const u4*>(Yl + (int64_t)gj * ldyh + k0 + kc);
            }
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int chunk = tid + 512 * c;
            const int row = chunk / GCPR, kc = chunk % GCPR;
#pragma unroll
            for (int h = 0; h < NI; ++h) {
                *reinterpret_cast<u4*>(&As[buf][h][gswz(row, kc)]) = st[c][h];
                *reinterpret_cast<u4*>(&Bs[buf][h][gswz(row, kc)]) = st[c][NI + h];
            }
        }
    };

    if (tid < GBM) {
        const int gi = i0 + tid < n ? i0 + tid : n - 1;
        sxs[tid] = xs[gi];
        sxx[tid] = xx[gi];
    }
    float cys[4], cyy[4];
#pragma unroll
    for (int nj = 0; nj < 4; ++nj) {
        const int gj0 = j0 + wn * 128 + nj * 32 + (lane & 31);
        const int gj = gj0 < m ? gj0 : m - 1;
        cys[nj] = ys[gj];
        cyy[nj] = yy[gj];
    }

    OTF_CST(1);
    const int nk = kpad / GBK;
    gload(0);
    lstore(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        if (kt == nk / 2) OTF_CST(4);
        const int buf = kt & 1;
#if defined(OTF_COST_ABLATE) && (OTF_COST_ABLATE & 4)
        // diagnostic: no operand loads after the prologue (the loop re-reads stale stages)
        if (false)
#else
        if (kt + 1 < nk)
#endif
            gload((kt + 1) * GBK);
#pragma unroll
        for (int ks = 0; ks < GBK / 16; ++ks) {
            const int kc = ks * 2 + (lane >> 5);
            f16x8 ah[2], al[2], bh[4], bl[4];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int ar = wm * 64 + t * 32 + (lane & 31);
                ah[t] = *reinterpret_cast<const f16x8*>(&As[buf][0][gswz(ar, kc)]);
                if (NI == 2) al[t] = *reinterpret_cast<const f16x8*>(&As[buf][NI - 1][gswz(ar, kc)]);
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int br = wn * 128 + t * 32 + (lane & 31);
                bh[t] = *reinterpret_cast<const f16x8*>(&Bs[buf][0][gswz(br, kc)]);
                if (NI == 2) bl[t] = *reinterpret_cast<const f16x8*>(&Bs[buf][NI - 1][gswz(br, kc)]);
            }
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
#pragma unroll
                for (int nj = 0; nj < 4; ++nj) {
#if defined(OTF_COST_ABLATE) && (OTF_COST_ABLATE & 2)
                    // diagnostic: no MFMAs (the fragments still feed one add each)
                    acc[mi][nj][0] += (float)ah[mi][0] + (float)bh[nj][0] + (NI == 2 ? (float)al[mi][0] + (float)bl[nj][0] : 0.f);
#else
                    if (NS == 3) {
                        acc[mi][nj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[mi], bh[nj], acc[mi][nj], 0, 0, 0);
                        acc[mi][nj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[mi], bl[nj], acc[mi][nj], 0, 0, 0);
                    }
                    acc[mi][nj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[mi], bh[nj], acc[mi][nj], 0, 0, 0);
#endif
                }
        }
#if defined(OTF_COST_ABLATE) && (OTF_COST_ABLATE & 4)
        if (false)
#else
        if (kt + 1 < nk)
#endif
            lstore(buf ^ 1);
        __syncthreads();
    }

    OTF_CST(2);
    const float os = store_scale ? store_scale[0] : 1.0f;
    float lmax = epilogue_tile256<TC>(acc, sxs, sxx, cys, cyy, wm, wn, lane, i0, j0, n, m, metric, zero_diag, C,
                                      ldc, os);
    OTF_CST(3);
    if (cmax) {
        lmax = wave_max(lmax);
        if (lane == 0) wmx[wid] = lmax;
        __syncthreads();
        if (tid == 0) {
            float v = wmx[0];
#pragma unroll
            for (int w = 1; w < 8; ++w) v = fmaxf(v, wmx[w]);
            const unsigned int u = __float_as_uint(v);
            if (u > __hip_atomic_load(cmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(cmax, u);
        }
    }
}

// The same 256 x 256 tile on v_mfma_f32_16x16x32_f16 (OTF_COST_MFMA16): one MFMA per
// 32-deep stage and 16 x 16 output block, so a wave's 64 x 128 block is 4 x 8 MFMA
// blocks (128 accumulators, as before) and the LDS reads per stage are the same 24
// ds_read_b128 per wave; the point is the clock: MFMA-dense loops hold a higher clock on
// the 16x16 shape (MI355X_MICROARCH.md, DVFS item 7: 1.12-1.15x the FLOP/s of 32x32x16).
// Fragment of rows r..r+15: lane l reads row r + (l & 15), 16-B chunk l >> 4 of the
// 64-B row.  The chunk is XOR-permuted by the row quad q = (row >> 2) & 3 through
// g(q) = {0, 2, 3, 1}: every 16-lane group of ds_read_b128 ({0-3,12-15,20-27}, ...)
// then hits 16 distinct 16-B slots of the 256-B bank row, and the 8-lane groups of the
// ds_write_b128 staging stores (rows 2j, 2j + 1, chunks 0..3) cover 128 B exactly.
__device__ __forceinline__ int g16swz(int row, int kc) {
    return row * GBK + ((kc ^ ((0x78 >> (2 * ((row >> 2) & 3))) & 3)) << 3);
}
// Cost values of one 256 x 256 tile from the 16x16x32 kernel's accumulators.  The MFMAs
// run with the Y fragment as the A operand, so each 16 x 16 accumulator block is the
// TRANSPOSED cost block: lane l holds cost row (l & 15) at the four consecutive columns
// 4 (l >> 4) + e -- one 16-B (fp32) / 8-B (fp16) store per lane per block instead of
// four 4-B stores (the epilogue's store issue, not bandwidth, is its cost).  Column norm
// terms come from LDS (sys / syy, four consecutive in one read).  VEC: whole tile with a
// 16-B aligned row pitch; otherwise one element at a time with the bounds tests.
template <typename TC, bool EUC, bool VEC>
__device__ __forceinline__ float epilogue_tile256_16t(const f32x4 (&acc)[4][8], const float* sxs, const float* sxx,
                                                      const float* sys, const float* syy, int wm, int wn, int lane,
                                                      int i0, int j0, int n, int m, int zero_diag, TC* C,
                                                      int64_t ldc, float os) {
    const __amdgpu_buffer_rsrc_t ct =
        __builtin_amdgcn_make_buffer_rsrc((void*)(C + (int64_t)i0 * ldc + j0), 0, 0x7fffffff, 0x00020000);
    const int rr = wm * 64 + (lane & 15), cc = wn * 128 + 4 * (lane >> 4);
    float lmax = 0.f;
#pragma unroll
    for (int nj = 0; nj < 8; ++nj) {
        __builtin_amdgcn_sched_barrier(0);
        const int cl = cc + nj * 16;
        const f32x4 ys4 = *reinterpret_cast<const f32x4*>(&sys[cl]);
        const f32x4 yy4 = *reinterpret_cast<const f32x4*>(&syy[cl]);
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
            const int rl = rr + mi * 16;
            const float a = -2.f * sxs[rl], b = sxx[rl];
            uint32_t vo = (uint32_t)(rl * (int)ldc + cl) * (uint32_t)sizeof(TC);
            float cv[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float c = fmaf(acc[mi][nj][e], a * ys4[e], b + yy4[e]);
                c = fmaxf(c, 0.f);
                if constexpr (EUC) c = sqrtf(c);
                cv[e] = c;
            }
            if constexpr (VEC) {
#pragma unroll
                for (int e = 0; e < 4; ++e) lmax = fmaxf(lmax, cv[e]);
#if defined(OTF_COST_ABLATE) && (OTF_COST_ABLATE & 1)
                if (cv[0] == -12345.f)  // diagnostic (tools/ubench_cost.hip): no cost stores
#endif
                {
                    if constexpr (sizeof(TC) == 4) {
                        using U4 = __attribute__((ext_vector_type(4))) unsigned int;
                        const U4 w = {__builtin_bit_cast(uint32_t, cv[0] * os), __builtin_bit_cast(uint32_t, cv[1] * os),
                                      __builtin_bit_cast(uint32_t, cv[2] * os), __builtin_bit_cast(uint32_t, cv[3] * os)};
                        __builtin_amdgcn_raw_buffer_store_b128(w, ct, vo, 0, 0);
                    } else {
                        using U2 = __attribute__((ext_vector_type(2))) unsigned int;
                        const uint32_t h0 = __builtin_bit_cast(uint16_t, (TC)(cv[0] * os)) |
                                            ((uint32_t)__builtin_bit_cast(uint16_t, (TC)(cv[1] * os)) << 16);
                        const uint32_t h1 = __builtin_bit_cast(uint16_t, (TC)(cv[2] * os)) |
                                            ((uint32_t)__builtin_bit_cast(uint16_t, (TC)(cv[3] * os)) << 16);
                        __builtin_amdgcn_raw_buffer_store_b64(U2{h0, h1}, ct, vo, 0, 0);
                    }
                }
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float c = cv[e];
                    if (i0 + rl >= n || j0 + cl + e >= m) continue;
                    if (zero_diag && i0 + rl == j0 + cl + e) c = 0.f;
                    lmax = fmaxf(lmax, c);
                    const uint32_t ve = vo + (uint32_t)(e * (int)sizeof(TC));
                    if constexpr (sizeof(TC) == 4)
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, c * os), ct, ve, 0, 0);
                    else
                        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, (TC)(c * os)), ct, ve, 0, 0);
                }
            }
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    return (float)(TC)(lmax * os);
}

// F32IN (split-fp16 only): X / Y are the float32 embeddings themselves (Xh / Yh cast back,
// ldxh / ldyh in floats, d a multiple of the 64-deep image padding, rows 16-B aligned);
// every stage is split into its hi / lo fp16 images in registers on the way to LDS with
// the row's power-of-two scale 1 / xs (the prep kernel then writes only the norms and
// scales): the same images as split16_prep2_kernel's, so the same bits, without their
// 33.7 MB HBM round trip (fp32 operand bytes = hi + lo image bytes).
// first column block after which a split piece runs (build switch; 4 pieces)
#ifndef OTF_COST_ILV_AT
#define OTF_COST_ILV_AT 3
#endif
// ILV (F32IN only, OTF_COST_ILV=1): the next stage's split + LDS writes run in four pieces
// between the MFMA groups of the current stage (after column blocks 3..6) instead of after
// all of them, and every stage issues its loads (the last one reloads itself into the idle
// buffer), so the loop body is one basic block the scheduler can interleave.
template <int NS, typename TC, bool F32IN = false, bool ILV = false>
__global__ __launch_bounds__(512) void cost_big16_kernel(
    const _Float16* __restrict__ Xh, const _Float16* __restrict__ Xl, const float* __restrict__ xs,
    const float* __restrict__ xx, const _Float16* __restrict__ Yh, const _Float16* __restrict__ Yl,
    const float* __restrict__ ys, const float* __restrict__ yy, int64_t ldxh, int64_t ldyh, int n, int m, int kpad,
    int metric, int zero_diag, TC* __restrict__ C, int64_t ldc, unsigned int* cmax, int tiles_n,
    const float* __restrict__ store_scale) {
    constexpr int NI = NS == 3 ? 2 : 1;
    constexpr int NCH = GBM * GCPR / 512;
    __shared__ __attribute__((aligned(16))) _Float16 As[2][NI][GBM * GBK];
    __shared__ __attribute__((aligned(16))) _Float16 Bs[2][NI][GBN * GBK];
    __shared__ float sxs[GBM], sxx[GBM];
    __shared__ __attribute__((aligned(16))) float sys[GBN], syy[GBN];
    __shared__ float wmx[8];

    OTF_CST(0);
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    int tm, tn;
    grouped_tile(wg, nwg, tiles_n, tm, tn);
    const int i0 = tm * GBM, j0 = tn * GBN;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;

    f32x4 acc[4][8];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

    using u4 = __attribute__((ext_vector_type(4))) unsigned int;
    static_assert(!F32IN || NI == 2, "float32 operands are split into two images");
    u4 st[NCH][2 * NI];
    // F32IN: the row scales of this thread's staging rows (fixed across stages)
    float scx[NCH], scy[NCH];
    if constexpr (F32IN) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int row = (tid + 512 * c) / GCPR;
            scx[c] = 1.0f / xs[i0 + row < n ? i0 + row : n - 1];
            scy[c] = 1.0f / ys[j0 + row < m ? j0 + row : m - 1];
        }
    }
    auto gload = [&](int k0) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int chunk = tid + 512 * c;
            const int row = chunk / GCPR, kc = (chunk % GCPR) * 8;
            const int gi = i0 + row < n ? i0 + row : n - 1;
            const int gj = j0 + row < m ? j0 + row : m - 1;
            if constexpr (F32IN) {
                // 8 consecutive floats = the same 32 B the two fp16 images would take
                const float* xr = reinterpret_cast<const float*>(Xh) + (int64_t)gi * ldxh + k0 + kc;
                const float* yr = reinterpret_cast<const float*>(Yh) + (int64_t)gj * ldyh + k0 + kc;
                st[c][0] = *reinterpret_cast<const u4*>(xr);
                st[c][1] = *reinterpret_cast<const u4*>(xr + 4);
                st[c][NI] = *reinterpret_cast<const u4*>(yr);
                st[c][NI + 1] = *reinterpret_cast<const u4*>(yr + 4);
            } else {
                st[c][0] = *reinterpret_cast<const u4*>(Xh + (int64_t)gi * ldxh + k0 + kc);
                st[c][NI] = *reinterpret_cast<const u4*>(Yh + (int64_t)gj * ldyh + k0 + kc);
                if (NI == 2) {
                    st[c][1] = *reinterpret_cast<const u4*>(Xl + (int64_t)gi * ldxh + k0 + kc);
                    st[c][NI + 1] = *reinterpret_cast<const u4*>(Yl + (int64_t)gj * ldyh + k0 + kc);
                }
            }
        }
    };
    // x s = hi + lo, hi = fp16(x s), lo = fp16(x s - hi): split16_prep2_kernel's images
    auto split8 = [&](u4 a, u4 b, float sc, u4& h, u4& l) {
        using H8 = __attribute__((ext_vector_type(8))) _Float16;
        H8 hv, lv;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const float w = __builtin_bit_cast(float, q < 4 ? a[q] : b[q - 4]) * sc;
            hv[q] = (_Float16)w;
            lv[q] = (_Float16)(w - (float)hv[q]);
        }
        h = __builtin_bit_cast(u4, hv);
        l = __builtin_bit_cast(u4, lv);
    };
    // one quarter of lstore (F32IN): chunk part >> 1, operand X (part even) or Y
    auto lstore_part = [&](int buf, int part) {
        if constexpr (!F32IN) return;
        const int c = part >> 1;
        const int chunk = tid + 512 * c;
        const int row = chunk / GCPR, kc = chunk % GCPR;
        u4 h, l;
        if ((part & 1) == 0) {
            split8(st[c][0], st[c][1], scx[c], h, l);
            *reinterpret_cast<u4*>(&As[buf][0][g16swz(row, kc)]) = h;
            *reinterpret_cast<u4*>(&As[buf][1][g16swz(row, kc)]) = l;
        } else {
            split8(st[c][NI], st[c][NI + 1], scy[c], h, l);
            *reinterpret_cast<u4*>(&Bs[buf][0][g16swz(row, kc)]) = h;
            *reinterpret_cast<u4*>(&Bs[buf][1][g16swz(row, kc)]) = l;
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int chunk = tid + 512 * c;
            const int row = chunk / GCPR, kc = chunk % GCPR;
            if constexpr (F32IN) {
                u4 h, l;
                split8(st[c][0], st[c][1], scx[c], h, l);
                *reinterpret_cast<u4*>(&As[buf][0][g16swz(row, kc)]) = h;
                *reinterpret_cast<u4*>(&As[buf][1][g16swz(row, kc)]) = l;
                split8(st[c][NI], st[c][NI + 1], scy[c], h, l);
                *reinterpret_cast<u4*>(&Bs[buf][0][g16swz(row, kc)]) = h;
                *reinterpret_cast<u4*>(&Bs[buf][1][g16swz(row, kc)]) = l;
            } else {
#pragma unroll
                for (int h = 0; h < NI; ++h) {
                    *reinterpret_cast<u4*>(&As[buf][h][g16swz(row, kc)]) = st[c][h];
                    *reinterpret_cast<u4*>(&Bs[buf][h][g16swz(row, kc)]) = st[c][NI + h];
                }
            }
        }
    };

    if (tid < GBM) {
        const int gi = i0 + tid < n ? i0 + tid : n - 1;
        sxs[tid] = xs[gi];
        sxx[tid] = xx[gi];
    } else if (tid < GBM + GBN) {
        const int c = tid - GBM;
        const int gj = j0 + c < m ? j0 + c : m - 1;
        sys[c] = ys[gj];
        syy[c] = yy[gj];
    }

    OTF_CST(1);
    const int nk = kpad / GBK;
    gload(0);
    lstore(0);
    __syncthreads();
    const int kc = lane >> 4;
    for (int kt = 0; kt < nk; ++kt) {
        if (kt == nk / 2) OTF_CST(4);
        const int buf = kt & 1;
        if constexpr (ILV) {
            gload((kt + 1 < nk ? kt + 1 : kt) * GBK);
            __builtin_amdgcn_sched_barrier(0);  // the next stage's loads go out first
        } else {
#if defined(OTF_COST_ABLATE) && (OTF_COST_ABLATE & 4)
        if (false)
#else
        if (kt + 1 < nk)
#endif
            gload((kt + 1) * GBK);
        }
        f16x8 ah[4], al[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int ar = wm * 64 + t * 16 + (lane & 15);
            ah[t] = *reinterpret_cast<const f16x8*>(&As[buf][0][g16swz(ar, kc)]);
            if (NI == 2) al[t] = *reinterpret_cast<const f16x8*>(&As[buf][NI - 1][g16swz(ar, kc)]);
        }
#pragma unroll
        for (int nj = 0; nj < 8; ++nj) {
            const int br = wn * 128 + nj * 16 + (lane & 15);
            const f16x8 bh = *reinterpret_cast<const f16x8*>(&Bs[buf][0][g16swz(br, kc)]);
            f16x8 bl;
            if (NI == 2) bl = *reinterpret_cast<const f16x8*>(&Bs[buf][NI - 1][g16swz(br, kc)]);
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) {
#if defined(OTF_COST_ABLATE) && (OTF_COST_ABLATE & 2)
                acc[mi][nj][0] += (float)ah[mi][0] + (float)bh[0] + (NI == 2 ? (float)al[mi][0] + (float)bl[0] : 0.f);
#else
                // Y fragment as the A operand: the accumulator block is the transposed
                // cost block (row-contiguous stores in the epilogue)
                if (NS == 3) {
                    acc[mi][nj] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh, al[mi], acc[mi][nj], 0, 0, 0);
                    acc[mi][nj] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bl, ah[mi], acc[mi][nj], 0, 0, 0);
                }
                acc[mi][nj] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh, ah[mi], acc[mi][nj], 0, 0, 0);
#endif
            }
            if constexpr (ILV) {
                if (nj >= OTF_COST_ILV_AT && nj < OTF_COST_ILV_AT + 4) lstore_part(buf ^ 1, nj - OTF_COST_ILV_AT);
            }
        }
        if constexpr (!ILV) {
#if defined(OTF_COST_ABLATE) && (OTF_COST_ABLATE & 4)
        if (false)
#else
        if (kt + 1 < nk)
#endif
            lstore(buf ^ 1);
        }
        __syncthreads();
    }

    OTF_CST(2);
    const float os = store_scale ? store_scale[0] : 1.0f;
    // vector stores: whole tile, no diagonal in it, rows 16-B (fp32) / 8-B (fp16) aligned
    const bool vec = i0 + 256 <= n && j0 + 256 <= m && !(zero_diag && i0 == j0) && (ldc % 4) == 0 &&
                     ((uintptr_t)C % 16) == 0;
    float lmax;
    if (metric == OTF_EUCLIDEAN)
        lmax = vec ? epilogue_tile256_16t<TC, true, true>(acc, sxs, sxx, sys, syy, wm, wn, lane, i0, j0, n, m, zero_diag, C, ldc, os)
                   : epilogue_tile256_16t<TC, true, false>(acc, sxs, sxx, sys, syy, wm, wn, lane, i0, j0, n, m, zero_diag, C, ldc, os);
    else
        lmax = vec ? epilogue_tile256_16t<TC, false, true>(acc, sxs, sxx, sys, syy, wm, wn, lane, i0, j0, n, m, zero_diag, C, ldc, os)
                   : epilogue_tile256_16t<TC, false, false>(acc, sxs, sxx, sys, syy, wm, wn, lane, i0, j0, n, m, zero_diag, C, ldc, os);
    OTF_CST(3);
    if (cmax) {
        lmax = wave_max(lmax);
        if (lane == 0) wmx[wid] = lmax;
        __syncthreads();
        if (tid == 0) {
            float v = wmx[0];
#pragma unroll
            for (int w = 1; w < 8; ++w) v = fmaxf(v, wmx[w]);
            const unsigned int u = __float_as_uint(v);
            if (u > __hip_atomic_load(cmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(cmax, u);
        }
    }
}



// ---------------------------------------------------------------------------------------
// The 256 x 256 tile as an 8-phase LDS-DMA pipeline (cdna_hip_programming.md "The 256²
// 8-phase template"): operands move global -> LDS by global_load_lds_dwordx4 only, in
// HALF-TILES of 16 KB (128 operand rows x 64 B x 2 sub-buffers: the two 32-deep k halves of
// a 64-deep K-tile for fp16 operands, NI = 1; the hi and lo images of a 32-deep K-tile for
// split-fp16, NI = 2), two K-tiles of four half-tiles in 128 KB of LDS.  The waves are
// 2 (Y, the MFMA A operand) x 4 (X) of 128 Y x 64 X -- cost_big16_kernel's per-wave block,
// so its epilogue -- and a K-tile runs as four PHASES, one output quadrant each
// (Y half x X half: A0.B0, A0.B1, A1.B1, A1.B0 -- each phase reads only the fragments the
// previous one did not leave in registers): ds_read the new fragments, put one half-tile of
// the NEXT K-tile in flight (2 glds a thread), a counted vmcnt, raw barrier, lgkmcnt(0), the
// quadrant's 16 (NI = 1) / 24 (NI = 2) MFMAs at raised priority, raw barrier.  Half-tile
// order per K-tile A0, B0, B1, A1 (first use order): vmcnt(4) in phases 0, 1, 3 retires what
// the next phase reads and keeps two half-tiles in flight across every barrier; a half-tile
// is restaged >= 2 phases after its last read.  Each 16 x 16 block gets cost_big16's MFMA
// sequence (for NI = 2: hi.lo, lo.hi, hi.hi per 32-deep step, in k order), so the same bits.
// LDS rows are 64 B with cost_big16's XOR chunk permutation (g16swz), applied to each lane's
// SOURCE chunk since the DMA writes lane-linear (rule 21).  All LDS is one array (a second
// __shared__ object makes hipcc drain the DMA early).
typedef __attribute__((address_space(3))) void p8_lds_t;
typedef __attribute__((address_space(1))) void p8_gbl_t;
constexpr int P8_SUB = 8192, P8_HT = 2 * P8_SUB, P8_BUF = 4 * P8_HT;
constexpr int P8_LDS = 2 * P8_BUF + 4 * 256 * 4 + 64;
__device__ __forceinline__ int p8_byte(int row, int kc) {
    return row * 64 + ((kc ^ ((0x78 >> (2 * ((row >> 2) & 3))) & 3)) << 4);
}
template <int N> __device__ __forceinline__ void p8_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <int NI, typename TC>
__global__ __launch_bounds__(512) void cost_8ph_kernel(
    const _Float16* __restrict__ Xh, const _Float16* __restrict__ Xl, const float* __restrict__ xs,
    const float* __restrict__ xx, const _Float16* __restrict__ Yh, const _Float16* __restrict__ Yl,
    const float* __restrict__ ys, const float* __restrict__ yy, int64_t ldxh, int64_t ldyh, int n, int m, int kpad,
    int metric, int zero_diag, TC* __restrict__ C, int64_t ldc, unsigned int* cmax, int tiles_n,
    const float* __restrict__ store_scale) {
    __shared__ __attribute__((aligned(16))) char smem[P8_LDS];
    float* sxs = reinterpret_cast<float*>(smem + 2 * P8_BUF);
    float* sxx = sxs + 256;
    float* sys = sxx + 256;
    float* syy = sys + 256;
    float* wmx = syy + 256;

    const int nwg = gridDim.x, bid = blockIdx.x;
    const int q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
    int tm, tn;
    grouped_tile(wg, nwg, tiles_n, tm, tn);
    const int i0 = tm * GBM, j0 = tn * GBN;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wn = wid >> 2, wm = wid & 3;  // Y half (128 columns), X quarter (64 rows)

    // norms first: ordinary loads, none while a DMA is in flight
    if (tid < 256) {
        const int gi = i0 + tid < n ? i0 + tid : n - 1;
        sxs[tid] = xs[gi];
        sxx[tid] = xx[gi];
    } else {
        const int c = tid - 256;
        const int gj = j0 + c < m ? j0 + c : m - 1;
        sys[c] = ys[gj];
        syy[c] = yy[gj];
    }

    // this thread's DMA sources: slot tid of every sub-buffer = local row tid / 4, stored
    // chunk tid % 4, which holds logical chunk (tid % 4) ^ g(row)
    const int drow = tid >> 2;
    const int dkc = (tid & 3) ^ ((0x78 >> (2 * ((drow >> 2) & 3))) & 3);
    const _Float16* src[4][2];
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        const bool isy = h < 2;
        const int hh = h & 1;
        const int tr = isy ? (drow >> 6) * 128 + hh * 64 + (drow & 63) : (drow >> 5) * 64 + hh * 32 + (drow & 31);
        const int gr = isy ? (j0 + tr < m ? j0 + tr : m - 1) : (i0 + tr < n ? i0 + tr : n - 1);
        const _Float16* hi = isy ? Yh + (int64_t)gr * ldyh : Xh + (int64_t)gr * ldxh;
        if constexpr (NI == 2) {
            const _Float16* lo = isy ? Yl + (int64_t)gr * ldyh : Xl + (int64_t)gr * ldxh;
            src[h][0] = hi + dkc * 8;
            src[h][1] = lo + dkc * 8;
        } else {
            src[h][0] = hi + dkc * 8;
            src[h][1] = hi + 32 + dkc * 8;
        }
    }
    constexpr int BK = NI == 1 ? 64 : 32;
    // half-tile h of K-tile kt into buffer b
    auto stage = [&](int h, int kt, int b) {
        char* dst = smem + b * P8_BUF + h * P8_HT + wid * 1024;
        const int k0 = kt * BK;
        __builtin_amdgcn_global_load_lds((p8_gbl_t*)(src[h][0] + k0), (p8_lds_t*)dst, 16, 0, 0);
        __builtin_amdgcn_global_load_lds((p8_gbl_t*)(src[h][1] + k0), (p8_lds_t*)(dst + P8_SUB), 16, 0, 0);
    };

    f32x4 acc[4][8];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    f16x8 fa[4][2], fb[2][2];  // Y fragments of the current Y half, X fragments of the current X half
    const int kc = lane >> 4, lr = lane & 15;
    auto read_a = [&](int b, int yh) {
        const char* base = smem + b * P8_BUF + yh * P8_HT;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int off = p8_byte(wn * 64 + t * 16 + lr, kc);
            fa[t][0] = *reinterpret_cast<const f16x8*>(base + off);
            fa[t][1] = *reinterpret_cast<const f16x8*>(base + P8_SUB + off);
        }
    };
    auto read_b = [&](int b, int xh) {
        const char* base = smem + b * P8_BUF + (2 + xh) * P8_HT;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int off = p8_byte(wm * 32 + t * 16 + lr, kc);
            fb[t][0] = *reinterpret_cast<const f16x8*>(base + off);
            fb[t][1] = *reinterpret_cast<const f16x8*>(base + P8_SUB + off);
        }
    };
    auto mfma_quadrant = [&](int yh, int xh) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                f32x4& a = acc[xh * 2 + u][yh * 4 + t];
                if constexpr (NI == 2) {
                    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[t][0], fb[u][1], a, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[t][1], fb[u][0], a, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[t][0], fb[u][0], a, 0, 0, 0);
                } else {
                    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[t][0], fb[u][0], a, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[t][1], fb[u][1], a, 0, 0, 0);
                }
            }
        __builtin_amdgcn_s_setprio(0);
    };
    auto sync_compute = [&](int yh, int xh) {
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        mfma_quadrant(yh, xh);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");  // the next phase's reads and DMA stay behind the barrier
    };

    // prologue: K-tile 0 in the order A0, B0, B1, A1; A0 and B0 landed before the first phase
    const int nk = kpad / BK;
    stage(0, 0, 0);
    stage(2, 0, 0);
    stage(3, 0, 0);
    stage(1, 0, 0);
    p8_vmcnt<4>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // the two wave groups (wn, one wave of each on every SIMD) run one barrier apart, so one
    // group's MFMAs overlap the other's fragment reads and DMA issue (the template's
    // stagger); every read stays one phase behind its wait and every restage >= 2 phases
    // behind its last read, which is what that offset needs
    const int wsg = __builtin_amdgcn_readfirstlane(wn);
    if (wsg == 1) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    for (int kt = 0; kt < nk; ++kt) {
        const int b = kt & 1;
        const bool more = kt + 1 < nk;
        // phase 0: A0 x B0
        read_b(b, 0);
        __builtin_amdgcn_sched_barrier(0);
        read_a(b, 0);
        if (more) {
            stage(0, kt + 1, b ^ 1);
            p8_vmcnt<4>();  // B1 of this K-tile landed
        } else {
            p8_vmcnt<2>();
        }
        sync_compute(0, 0);
        // phase 1: A0 x B1
        read_b(b, 1);
        if (more) {
            stage(2, kt + 1, b ^ 1);
            p8_vmcnt<4>();  // A1 of this K-tile landed
        } else {
            p8_vmcnt<0>();
        }
        sync_compute(0, 1);
        // phase 2: A1 x B1
        read_a(b, 1);
        if (more) stage(3, kt + 1, b ^ 1);
        sync_compute(1, 1);
        // phase 3: A1 x B0
        read_b(b, 0);
        if (more) {
            stage(1, kt + 1, b ^ 1);
            p8_vmcnt<4>();  // A0, B0 of the next K-tile landed
        }
        sync_compute(1, 0);
    }
    if (wsg == 0) __builtin_amdgcn_s_barrier();  // the groups' barrier counts agree again

    const float os = store_scale ? store_scale[0] : 1.0f;
    const bool vec = i0 + 256 <= n && j0 + 256 <= m && !(zero_diag && i0 == j0) && (ldc % 4) == 0 &&
                     ((uintptr_t)C % 16) == 0;
    float lmax;
    if (metric == OTF_EUCLIDEAN)
        lmax = vec ? epilogue_tile256_16t<TC, true, true>(acc, sxs, sxx, sys, syy, wm, wn, lane, i0, j0, n, m, zero_diag, C, ldc, os)
                   : epilogue_tile256_16t<TC, true, false>(acc, sxs, sxx, sys, syy, wm, wn, lane, i0, j0, n, m, zero_diag, C, ldc, os);
    else
        lmax = vec ? epilogue_tile256_16t<TC, false, true>(acc, sxs, sxx, sys, syy, wm, wn, lane, i0, j0, n, m, zero_diag, C, ldc, os)
                   : epilogue_tile256_16t<TC, false, false>(acc, sxs, sxx, sys, syy, wm, wn, lane, i0, j0, n, m, zero_diag, C, ldc, os);
    if (cmax) {
        lmax = wave_max(lmax);
        if (lane == 0) wmx[wid] = lmax;
        __syncthreads();
        if (tid == 0) {
            float v = wmx[0];
#pragma unroll
            for (int w = 1; w < 8; ++w) v = fmaxf(v, wmx[w]);
            const unsigned int u = __float_as_uint(v);
            if (u > __hip_atomic_load(cmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(cmax, u);
        }
    }
}

}  // namespace

// Split-fp16 images + row scales + squared norms of two float32 operands in the workspace
// layout of otf_cost_pairwise_ex (one split16_prep2_kernel launch): the fused float32
// pairwise solve's prologue reads them (otf_persist.h PairwiseF32); the same bits as the
// images the 256 x 256 cost kernel splits in registers, so the same costs.
hipError_t split16_images(const float* X, int64_t ldx, int n, const float* Y, int64_t ldy, int m, int d,
                          void* ws, Split16Images& out, unsigned int* cmax_word, hipStream_t s) {
    const int64_t ldh = (d + SBK - 1) / SBK * SBK;
    char* p = (char*)ws;
    auto take = [&](size_t bytes) { void* q = p; p += (bytes + 255) / 256 * 256; return q; };
    out.Xh = (_Float16*)take((size_t)n * ldh * 2);
    out.Xl = (_Float16*)take((size_t)n * ldh * 2);
    out.Yh = (_Float16*)take((size_t)m * ldh * 2);
    out.Yl = (_Float16*)take((size_t)m * ldh * 2);
    out.xs = (float*)take((size_t)n * 4);
    out.xx = (float*)take((size_t)n * 4);
    out.ys = (float*)take((size_t)m * 4);
    out.yy = (float*)take((size_t)m * 4);
    out.ldh = ldh;
    const int rows = n + m;
    const int nblk = (rows + 3) / 4 < 1024 ? (rows + 3) / 4 : 1024;
    const int vec = (ldx * 4 % 16 == 0 && ldy * 4 % 16 == 0 && (uintptr_t)X % 16 == 0 && (uintptr_t)Y % 16 == 0) ? 1 : 0;
    const PrepSide<float> A{X, ldx, n, out.Xh, out.Xl, out.xs, out.xx, nullptr};
    const PrepSide<float> B{Y, ldy, m, out.Yh, out.Yl, out.ys, out.yy, nullptr};
    split16_prep2_kernel<float, true><<<nblk, 256, 0, s>>>(A, B, d, (int)ldh, vec, cmax_word, nullptr);
    return hipGetLastError();
}
}  // namespace otf

extern "C" {

int otf_cost_pairwise(const float* X, int64_t ldx, const float* Y, int64_t ldy, int64_t n,
                      int64_t m, int64_t d, int32_t metric, int32_t zero_diag, float* C,
                      int64_t ldc, float* cmax, otf_stream_t stream) {
    if (!X || !Y || !C || n <= 0 || m <= 0 || d <= 0) return OTF_EINVAL;
    if (ldx < d || ldy < d || ldc < m) return OTF_EINVAL;
    if (metric != OTF_SQEUCLIDEAN && metric != OTF_EUCLIDEAN) return OTF_EINVAL;
    if (n > INT32_MAX || m > INT32_MAX || d > INT32_MAX) return OTF_EUNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    const bool vec_ok = (ldx % 4 == 0) && (ldy % 4 == 0) && ((uintptr_t)X % 16 == 0) &&
                        ((uintptr_t)Y % 16 == 0);
    if (cmax) OTF_HIP(hipMemsetAsync(cmax, 0, sizeof(float), s));
    const int tiles_m = (int)((n + otf::BM - 1) / otf::BM);
    const int tiles_n = (int)((m + otf::BN - 1) / otf::BN);
    const int64_t nwg = (int64_t)tiles_m * tiles_n;
    if (nwg > INT32_MAX) return OTF_EUNSUPPORTED;
    otf::cost_pairwise_kernel<<<(int)nwg, 256, 0, s>>>(X, ldx, Y, ldy, (int)n, (int)m, (int)d,
                                                       metric, zero_diag, C, ldc,
                                                       (unsigned int*)cmax, tiles_n, vec_ok);
    OTF_HIP(hipGetLastError());
    return OTF_OK;
}

static size_t otf_al(size_t x) { return (x + 255) / 256 * 256; }

// The 16x16x32 form of the 256 x 256 kernel for float32 cost storage (metric shape: 52
// vs 56 us, r03 stamps); the fp16-storage config-5 cost keeps the 32x32x16 form (its
// 8-B transposed stores measured no faster).  Float32 operands are split into hi / lo fp16
// inside the 16x16x32 kernel (F32IN, the next stage's split interleaved between the MFMA
// groups: r04 kernel 59.0 -> 56.2 us) where the rows are whole 16-B aligned stages; other
// float32 rows go through the prep's fp16 images (the same bits, tests/test_gpu_parity.py).
// Measured and removed in r05 (numbers in DESIGN.md 4.2): the LDS-DMA ring and the
// warp-specialised persistent kernels, the 128 x 128 tile at every shape, the split after
// the MFMA groups.
// r06: every 256 x 256 tile runs cost_8ph_kernel (OTF_COST_8PH=0 restores the kernels
// above): same bits as cost_big16_kernel for float32 storage; measured in one process
// (tools/cost8_probe.py) 66.2 -> 54.0 us at the metric shape (the prep then writes the
// images: 8.3 -> 13.3 us), config 5 166.5 -> 146.0 us.

size_t otf_cost_ex_workspace_size(int64_t n, int64_t m, int64_t d, int32_t in_dtype) {
    const size_t ldh = (size_t)((d + otf::SBK - 1) / otf::SBK * otf::SBK);
    const size_t ni = in_dtype == OTF_F16 ? 1 : 2;
    return ni * otf_al((size_t)n * ldh * 2) + ni * otf_al((size_t)m * ldh * 2) +
           2 * otf_al((size_t)n * 4) + 2 * otf_al((size_t)m * 4) + 256;
}

size_t otf_cost_split16_workspace_size(int64_t n, int64_t m, int64_t d) {
    return otf_cost_ex_workspace_size(n, m, d, OTF_F32);
}

// OTF_COST_PHASES=1 (read per call): events around the prep and the cost kernel of
// every otf_cost_pairwise_ex call; otf_cost_last_phases reports the last call's split
static hipEvent_t g_cost_ev[3];
static int g_cost_ev_state = 0;  // 0 none, 1 created, 2 recorded
// OTF_COST_8PH (read per call; default 1): the 8-phase LDS-DMA kernel (cost_8ph_kernel) for
// the 256 x 256 tile instead of the register-staged kernels; 0 keeps cost_big16_kernel /
// cost_big_kernel (A/B and bit-identity tests)
static bool cost_8ph_on() {
    const char* e = getenv("OTF_COST_8PH");
    return !(e && atoi(e) == 0);
}

static bool cost_phases_on() {
    const char* e = getenv("OTF_COST_PHASES");
    if (!(e && atoi(e) != 0)) return false;
    if (g_cost_ev_state == 0) {
        for (auto& ev : g_cost_ev)
            if (hipEventCreate(&ev) != hipSuccess) return false;
        g_cost_ev_state = 1;
    }
    return true;
}

int otf_cost_last_phases(float* prep_ms, float* kernel_ms) {
    if (!prep_ms || !kernel_ms || g_cost_ev_state != 2) return OTF_EINVAL;
    OTF_HIP(hipEventSynchronize(g_cost_ev[2]));
    OTF_HIP(hipEventElapsedTime(prep_ms, g_cost_ev[0], g_cost_ev[1]));
    OTF_HIP(hipEventElapsedTime(kernel_ms, g_cost_ev[1], g_cost_ev[2]));
    return OTF_OK;
}

int otf_cost_pairwise_ex(const void* X, int64_t ldx, const void* Y, int64_t ldy,
                         int32_t in_dtype, int64_t n, int64_t m, int64_t d, int32_t metric,
                         int32_t zero_diag, void* C, int64_t ldc, int32_t c_dtype, float* cmax,
                         float* c_unit, void* workspace, size_t ws_bytes, otf_stream_t stream) {
    if (!X || !Y || !C || !workspace || n <= 0 || m <= 0 || d <= 0) return OTF_EINVAL;
    if (ldx < d || ldy < d || ldc < m) return OTF_EINVAL;
    if (metric != OTF_SQEUCLIDEAN && metric != OTF_EUCLIDEAN) return OTF_EINVAL;
    if (in_dtype != OTF_F32 && in_dtype != OTF_F16) return OTF_EINVAL;
    if (c_dtype != OTF_F32 && c_dtype != OTF_F16) return OTF_EINVAL;
    if (ws_bytes < otf_cost_ex_workspace_size(n, m, d, in_dtype)) return OTF_EINVAL;
    if (n > INT32_MAX || m > INT32_MAX || d > (1 << 20)) return OTF_EUNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    const bool phases = cost_phases_on();
    if (phases) OTF_HIP(hipEventRecord(g_cost_ev[0], s));
    const bool split = in_dtype == OTF_F32;
    const int ldh = (int)((d + otf::SBK - 1) / otf::SBK * otf::SBK);
    char* p = (char*)workspace;
    auto take = [&](size_t bytes) { void* q = p; p += otf_al(bytes); return q; };
    _Float16* Xh = (_Float16*)take((size_t)n * ldh * 2);
    _Float16* Xl = split ? (_Float16*)take((size_t)n * ldh * 2) : nullptr;
    _Float16* Yh = (_Float16*)take((size_t)m * ldh * 2);
    _Float16* Yl = split ? (_Float16*)take((size_t)m * ldh * 2) : nullptr;
    float* xs = (float*)take((size_t)n * 4);
    float* xx = (float*)take((size_t)n * 4);
    float* ys = (float*)take((size_t)m * 4);
    float* yy = (float*)take((size_t)m * 4);
    float* small = (float*)take(256);  // [0..1] max squared norms, [2] store scale
    const bool f16out = c_dtype == OTF_F16;
    unsigned int* mn = f16out ? (unsigned int*)small : nullptr;
    if (f16out) OTF_HIP(hipMemsetAsync(small, 0, 2 * sizeof(float), s));
    const bool same = (X == Y && n == m && ldx == ldy);
    // fp16 rows that are whole K stages, 16-B aligned, are their own MFMA image
    const bool alias = !split && d % otf::SBK == 0 && ldx % 8 == 0 && ldy % 8 == 0 &&
                       (uintptr_t)X % 16 == 0 && (uintptr_t)Y % 16 == 0;
    int64_t ldxh = ldh, ldyh = ldh;
    // float32 operands split inside the 256 x 256 16x16x32 kernel (F32IN): decided before
    // the prep, which then writes only the norms and the row scales
    // Tile choice by rounds of resident workgroups (two 128 x 128 per CU, one 256 x 256):
    // a round of 256 x 256 tiles took 1.8x a round of 128 x 128 ones at N = 4096
    // (68 vs 38 us), so big tiles win when they need fewer than 1 / 1.8 of the rounds
    // (N = 4096: 1 vs 2 rounds; config 5: 4 vs 8), not for a ragged 17 x 16 grid (2 vs 3).
    const int64_t cus0 = otf::device_cu_count();
    const int64_t big_rounds = (((n + otf::GBM - 1) / otf::GBM) * ((m + otf::GBN - 1) / otf::GBN) + cus0 - 1) / cus0;
    const int64_t small_rounds = (((n + otf::BM - 1) / otf::BM) * ((m + otf::BN - 1) / otf::BN) + 2 * cus0 - 1) / (2 * cus0);
    const bool big0 = 18 * big_rounds < 10 * small_rounds;
    const bool mfma16 = !f16out;
    const bool p8 = big0 && cost_8ph_on();
    const bool f32in = !p8 && split && big0 && mfma16 && d % otf::SBK == 0 && ldx % 4 == 0 &&
                       ldy % 4 == 0 && (uintptr_t)X % 16 == 0 && (uintptr_t)Y % 16 == 0;
    {
        const int rows = (int)n + (same ? 0 : (int)m);
        const int nblk = (rows + 3) / 4 < 1024 ? (rows + 3) / 4 : 1024;
        const size_t isz = split ? 4 : 2;
        const int vec = (ldx * isz % 16 == 0 && ldy * isz % 16 == 0 && (uintptr_t)X % 16 == 0 &&
                         (uintptr_t)Y % 16 == 0) ? 1 : 0;
        if (split) {
            const otf::PrepSide<float> A{(const float*)X, ldx, (int)n, f32in ? nullptr : Xh, Xl, xs, xx, mn};
            const otf::PrepSide<float> B{(const float*)Y, ldy, same ? 0 : (int)m, f32in ? nullptr : Yh, Yl,
                                         ys, yy, mn ? mn + 1 : nullptr};
            otf::split16_prep2_kernel<float, true><<<nblk, 256, 0, s>>>(A, B, (int)d, ldh, vec,
                                                                       (unsigned int*)cmax,
                                                                       f16out ? nullptr : c_unit);
        } else {
            if (alias) {
                Xh = (_Float16*)X;
                Yh = (_Float16*)Y;
                ldxh = ldx;
                ldyh = ldy;
            }
            const otf::PrepSide<_Float16> A{(const _Float16*)X, ldx, (int)n, alias ? nullptr : Xh,
                                            nullptr, xs, xx, mn};
            const otf::PrepSide<_Float16> B{(const _Float16*)Y, ldy, same ? 0 : (int)m,
                                            alias ? nullptr : Yh, nullptr, ys, yy,
                                            mn ? mn + 1 : nullptr};
            otf::split16_prep2_kernel<_Float16, false><<<nblk, 256, 0, s>>>(A, B, (int)d, ldh, vec,
                                                                           (unsigned int*)cmax,
                                                                           f16out ? nullptr : c_unit);
        }
    }
    OTF_HIP(hipGetLastError());
    if (same) {
        Yh = Xh; Yl = Xl; ys = xs; yy = xx; ldyh = ldxh;
        if (f16out) OTF_HIP(hipMemcpyAsync(mn + 1, mn, sizeof(float), hipMemcpyDeviceToDevice, s));
    }
    const float* store_scale = nullptr;
    if (f16out) {
        otf::cost_store_scale_kernel<<<1, 1, 0, s>>>(mn, metric, small + 2, c_unit);
        OTF_HIP(hipGetLastError());
        store_scale = small + 2;
    }
    // cmax = 0 and c_unit = 1 (fp32 storage) were written by the prep kernel
    const bool big = big0;
    const int BMx = big ? otf::GBM : otf::BM, BNx = big ? otf::GBN : otf::BN;
    const int tiles_m = (int)((n + BMx - 1) / BMx);
    const int tiles_n = (int)((m + BNx - 1) / BNx);
    const int64_t nwg = (int64_t)tiles_m * tiles_n;
    if (nwg > INT32_MAX) return OTF_EUNSUPPORTED;
#define OTF_COST_LAUNCH(NS, TC)                                                                   \
    do {                                                                                          \
        if (p8)                                                                                   \
            otf::cost_8ph_kernel<NS == 3 ? 2 : 1, TC><<<(int)nwg, 512, 0, s>>>(                  \
                Xh, Xl, xs, xx, Yh, Yl, ys, yy, ldxh, ldyh, (int)n, (int)m, ldh, metric,         \
                zero_diag, (TC*)C, ldc, (unsigned int*)cmax, tiles_n, store_scale);              \
        else if (big && mfma16 && f32in)                                                          \
            otf::cost_big16_kernel<NS, TC, NS == 3, NS == 3><<<(int)nwg, 512, 0, s>>>(           \
                (const _Float16*)X, nullptr, xs, xx, (const _Float16*)Y, nullptr, ys, yy, ldx,   \
                ldy, (int)n, (int)m, (int)d, metric, zero_diag, (TC*)C, ldc, (unsigned int*)cmax, \
                tiles_n, store_scale);                                                            \
        else if (big && mfma16)                                                                   \
            otf::cost_big16_kernel<NS, TC><<<(int)nwg, 512, 0, s>>>(                             \
                Xh, Xl, xs, xx, Yh, Yl, ys, yy, ldxh, ldyh, (int)n, (int)m, ldh, metric,         \
                zero_diag, (TC*)C, ldc, (unsigned int*)cmax, tiles_n, store_scale);              \
        else if (big)                                                                             \
            otf::cost_big_kernel<NS, TC><<<(int)nwg, 512, 0, s>>>(                               \
                Xh, Xl, xs, xx, Yh, Yl, ys, yy, ldxh, ldyh, (int)n, (int)m, ldh, metric,         \
                zero_diag, (TC*)C, ldc, (unsigned int*)cmax, tiles_n, store_scale);              \
        else                                                                                      \
            otf::cost_split16_kernel<NS, TC><<<(int)nwg, 256, 0, s>>>(                          \
                Xh, Xl, xs, xx, Yh, Yl, ys, yy, ldxh, ldyh, (int)n, (int)m, ldh, metric,         \
                zero_diag, (TC*)C, ldc, (unsigned int*)cmax, tiles_n, store_scale);              \
    } while (0)
    if (phases) OTF_HIP(hipEventRecord(g_cost_ev[1], s));
    if (split && !f16out) OTF_COST_LAUNCH(3, float);
    else if (split) OTF_COST_LAUNCH(3, _Float16);
    else if (!f16out) OTF_COST_LAUNCH(1, float);
    else OTF_COST_LAUNCH(1, _Float16);
#undef OTF_COST_LAUNCH
    OTF_HIP(hipGetLastError());
    if (phases) {
        OTF_HIP(hipEventRecord(g_cost_ev[2], s));
        g_cost_ev_state = 2;
    }
    return OTF_OK;
}

int otf_cost_pairwise_split16(const float* X, int64_t ldx, const float* Y, int64_t ldy, int64_t n,
                              int64_t m, int64_t d, int32_t metric, int32_t zero_diag, float* C,
                              int64_t ldc, float* cmax, void* workspace, size_t ws_bytes,
                              otf_stream_t stream) {
    return otf_cost_pairwise_ex(X, ldx, Y, ldy, OTF_F32, n, m, d, metric, zero_diag, C, ldc,
                                OTF_F32, cmax, nullptr, workspace, ws_bytes, stream);
}

int otf_scale_inplace(void* C, int64_t n, int64_t m, int64_t ldc, int32_t dtype, const void* s,
                      otf_stream_t stream) {
    if (!C || !s || n <= 0 || m <= 0 || ldc < m) return OTF_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == OTF_F32)
        otf::scale_inplace_kernel<float><<<1024, 256, 0, st>>>((float*)C, n, m, ldc, (const float*)s);
    else if (dtype == OTF_F64)
        otf::scale_inplace_kernel<double><<<1024, 256, 0, st>>>((double*)C, n, m, ldc, (const double*)s);
    else
        return OTF_EINVAL;
    OTF_HIP(hipGetLastError());
    return OTF_OK;
}

}  // extern "C"
