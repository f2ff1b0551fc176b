// otf_linalg.hip — feature cost (float64), plan post-processing and the small
// GEMMs that apply a plan.
//
// Feature cost, MRI_PET_OT_nojax.py:121-136 (get_feature_coupling_pot):
//     w1 = Ts.sum(1); t1 = (X**2).T @ w1;  w2 = Ts.sum(0); t2 = (Y**2).T @ w2
//     M  = t1[:, None] + t2[None, :] - 2 X^T Ts Y
// computed in float64 like the reference (X, Y are float32 numpy arrays that numpy
// promotes through the float64 Ts; X**2 is squared in float32 first, as there).
// Plan post-processing, MRI_PET_OT_nojax.py:702-715, and application
// ot_mri_from_pet = pet_fused @ T^T (:718; MRI_PET_OT_OT_per_epoch_attn.py:728).
#include "otf_device.h"

namespace otf {
namespace {

// bf16 storage (BASELINE config 4: bf16 encoder outputs): the upper 16 bits of an fp32,
// so the widening is exact and the reference's float32 arithmetic on the bf16-rounded
// embeddings is reproduced bit for bit
struct bf16 {
    uint16_t bits;
    __device__ __forceinline__ operator float() const { return __uint_as_float((uint32_t)bits << 16); }
    __device__ __forceinline__ operator double() const { return (double)(float)*this; }
};

// Generic tiled GEMM  out[i][j] = alpha * sum_k A(i,k) B(k,j) + beta * out[i][j]
//                                 + rowadd[i] + coladd[j]
// with A(i,k) = A[i*sa0 + k*sa1], B(k,j) = B[k*sb0 + j*sb1].  64 x 64 tile, BK 16,
// 256 threads, 4 x 4 outputs per thread, accumulation in TACC.
constexpr int GT = 64, GK = 16;

template <typename TA, typename TB, typename TACC, typename TOUT>
__global__ __launch_bounds__(256) void gemm_kernel(const TA* __restrict__ A, int64_t sa0,
                                                   int64_t sa1, const TB* __restrict__ B,
                                                   int64_t sb0, int64_t sb1, TOUT* out,
                                                   int64_t ldo, int M, int N, int K, TACC alpha,
                                                   TACC beta, const TACC* rowadd,
                                                   const TACC* coladd) {
    __shared__ TACC As[GK][GT + 1];
    __shared__ TACC Bs[GK][GT + 1];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int i0 = blockIdx.y * GT, j0 = blockIdx.x * GT;
    TACC acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = 0;
    for (int k0 = 0; k0 < K; k0 += GK) {
        for (int t = threadIdx.x; t < GK * GT; t += 256) {
            // A tile: element (i, k) with i fastest when sa0 == 1, else k fastest
            int ii, kk;
            if (sa0 == 1) { ii = t % GT; kk = t / GT; } else { kk = t % GK; ii = t / GK; }
            const int gi = i0 + ii, gk = k0 + kk;
            As[kk][ii] = (gi < M && gk < K) ? (TACC)A[(int64_t)gi * sa0 + (int64_t)gk * sa1] : (TACC)0;
            int jj, kb;
            if (sb1 == 1) { jj = t % GT; kb = t / GT; } else { kb = t % GK; jj = t / GK; }
            const int gj = j0 + jj, gkb = k0 + kb;
            Bs[kb][jj] = (gj < N && gkb < K) ? (TACC)B[(int64_t)gkb * sb0 + (int64_t)gj * sb1] : (TACC)0;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < GK; ++kk) {
            TACC av[4], bv[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) av[a] = As[kk][ty + 16 * a];
#pragma unroll
            for (int b = 0; b < 4; ++b) bv[b] = Bs[kk][tx + 16 * b];
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) acc[a][b] = fma(av[a], bv[b], acc[a][b]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        const int gi = i0 + ty + 16 * a;
        if (gi >= M) continue;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int gj = j0 + tx + 16 * b;
            if (gj >= N) continue;
            TACC v = alpha * acc[a][b];
            if (beta != (TACC)0) v += beta * (TACC)out[(int64_t)gi * ldo + gj];
            if (rowadd) v += rowadd[gi];
            if (coladd) v += coladd[gj];
            out[(int64_t)gi * ldo + gj] = (TOUT)v;
        }
    }
}

// w1[i] = sum_j Ts[i][j] (rows), w2[j] = sum_i Ts[i][j] (cols); diag form copies.
// mode 1 swaps them (fot_numpy's w1 = Ts.sum(axis=0), w2 = Ts.sum(axis=1)).
__global__ void ts_sums_kernel(const double* Ts, int64_t ldts, const double* diag, int n, int n2,
                               int mode, double* w1, double* w2) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (diag) {
        if (t < n) w1[t] = w2[t] = diag[t];
        return;
    }
    double* rows = mode ? w2 : w1;
    double* cols = mode ? w1 : w2;
    if (t < n) {
        double s = 0.0;
        for (int j = 0; j < n2; ++j) s += Ts[(int64_t)t * ldts + j];
        rows[t] = s;
    }
    if (t < n2) {
        double s = 0.0;
        for (int i = 0; i < n; ++i) s += Ts[(int64_t)i * ldts + t];
        cols[t] = s;
    }
}

// t[k] = sum_i float(x_ik * x_ik) * w[i]   ((X**2).T @ w with X**2 in float32)
template <typename TI>
__global__ void weighted_sq_colsum_kernel(const TI* X, int64_t ldx, int n, int d,
                                          const double* w, double* t) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= d) return;
    double s = 0.0;
    for (int i = 0; i < n; ++i) {
        const float x = (float)X[(int64_t)i * ldx + k];
        s += (double)(x * x) * w[i];
    }
    t[k] = s;
}

// t[o] = sum_k A(o, k)^2 w[k], A(o, k) = A[o * so + k * sk]; the square in float32
// as the reference's X**2 on float32 data, the weighted sum in float64.
__global__ void weighted_sq_strided_kernel(const float* A, int64_t so, int64_t sk, int nout, int nk,
                                           const double* w, double* t) {
    const int o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= nout) return;
    double s = 0.0;
    for (int k = 0; k < nk; ++k) {
        const float x = A[(int64_t)o * so + (int64_t)k * sk];
        s += (double)(x * x) * w[k];
    }
    t[o] = s;
}

// Z[i][l] = diag[i] * Y[i][l]   (Ts diagonal, e.g. np.eye(B)/B)
template <typename TI>
__global__ void diag_scale_kernel(const TI* Y, int64_t ldy, int n, int d2, const double* diag,
                                  double* Z) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < (int64_t)n * d2;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int i = (int)(t / d2), l = (int)(t % d2);
        Z[t] = diag[i] * (double)(float)Y[(int64_t)i * ldy + l];
    }
}

// One workgroup per row: Tn = fill_nan(float(T)) / rowsum (0 -> 1e-8).
template <typename T>
__global__ __launch_bounds__(256) void postprocess_kernel(const T* Tm, int d, int d2, int64_t ldt,
                                                          float nan_fill, int rownorm, float* Tn,
                                                          int64_t ldtn) {
    __shared__ float red[17];
    for (int row = blockIdx.x; row < d; row += gridDim.x) {
        const T* src = Tm + (int64_t)row * ldt;
        float* dst = Tn + (int64_t)row * ldtn;
        float s = 0.f;
        for (int j = threadIdx.x; j < d2; j += blockDim.x) {
            float v = (float)src[j];
            if (isnan(v)) v = nan_fill;
            dst[j] = v;
            s += v;
        }
        if (!rownorm) continue;
        s = block_sum<float>(s, red);
        if (s == 0.f) s = 1e-8f;
        for (int j = threadIdx.x; j < d2; j += blockDim.x) dst[j] = dst[j] / s;
        __syncthreads();
    }
}

// Fused post-process + apply (MRI_PET_OT_nojax.py:702-718): one workgroup per plan
// row i, ONE pass over the row: v = fill_nan(float(T[i][j])), rowsum s and the B
// dot products z_b . v together; out[b][i] = (z_b . v) / s (= pet_fused @ Tn^T),
// then Tn[i][j] = v / s (kept for the backward G @ Tn) from the L2-resident row.
constexpr int kPaB = 16;   // batch rows per register block
template <typename T>
__global__ __launch_bounds__(256) void postprocess_apply_kernel(
    const T* Tm, int d, int d2, int64_t ldt, float nan_fill, int rownorm, const float* Z,
    int64_t ldz, int B, float* out, int64_t ldo, float* Tn, int64_t ldtn) {
    __shared__ float red[17 * kPaB];
    __shared__ float red1[17];
    for (int row = blockIdx.x; row < d; row += gridDim.x) {
        const T* src = Tm + (int64_t)row * ldt;
        float s = 0.f;
        for (int b0 = 0; b0 < B; b0 += kPaB) {
            float acc[kPaB];
            float sp = 0.f;
#pragma unroll
            for (int b = 0; b < kPaB; ++b) acc[b] = 0.f;
            for (int j = threadIdx.x; j < d2; j += blockDim.x) {
                float v = (float)src[j];
                if (isnan(v)) v = nan_fill;
                sp += v;
#pragma unroll
                for (int b = 0; b < kPaB; ++b)
                    if (b0 + b < B) acc[b] += Z[(int64_t)(b0 + b) * ldz + j] * v;
            }
            block_sum_multi<float, kPaB>(acc, red);
            s = block_sum<float>(sp, red1);
            const float sd = (rownorm && s == 0.f) ? 1e-8f : s;
            if (threadIdx.x < kPaB && b0 + (int)threadIdx.x < B) {
                float mine = acc[0];
#pragma unroll
                for (int b = 1; b < kPaB; ++b)
                    if ((int)threadIdx.x == b) mine = acc[b];
                out[(int64_t)(b0 + threadIdx.x) * ldo + row] = rownorm ? mine / sd : mine;
            }
            __syncthreads();
        }
        if (Tn) {
            const float sd = (rownorm && s == 0.f) ? 1e-8f : s;
            float* dst = Tn + (int64_t)row * ldtn;
            for (int j = threadIdx.x; j < d2; j += blockDim.x) {
                float v = (float)src[j];
                if (isnan(v)) v = nan_fill;
                dst[j] = rownorm ? v / sd : v;
            }
        }
    }
}

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---------------------------------------------------------------------------------
// The training step's alignment loss and its gradients in ONE workgroup launch
// (cosine_loss, MRI_PET_OT_nojax.py:552-560, applied at :721 with the NaN -> 0 swap of
// :724-725): torch's chain  xh = x / max(|x|, 1e-12)  (F.normalize),
// xt = xh / max(|xh|, 1e-8)  (the norm clamp inside F.cosine_similarity),
// cos_b = xt_b . yt_b,  L = 1 - mean_b cos_b,  and the backward of that chain:
//   g_xt = -(1/B) yt,  g_xh = (g_xt - (xt . g_xt) xt) / max(|xh|, 1e-8),
//   g_x  = (g_xh - (xh . g_xh) xh) / |x|   (|x| > 1e-12; else g_xh / 1e-12)
// with xt . g_xt = -cos / B and xh . g_xh = (cos / B)(|xh|^2 / max(|xh|,1e-8)^2 - 1).
// keep = ok && finite(L): otherwise L, g_x, g_y are exact zeros (the reference
// replaces a NaN loss by a constant 0) and keep_out tells the backward.  Replaces the
// ~40 small torch launches of the autograd form per training step.
template <typename TX>
__global__ __launch_bounds__(1024) void cosine_align_kernel(const TX* X, int64_t ldx, const float* Y,
                                                            int64_t ldy, int B, int d, const uint8_t* ok,
                                                            const otf_sinkhorn_info* sk_info,
                                                            float* loss, float* gx, int64_t ldgx,
                                                            float* gy, int64_t ldgy, uint8_t* keep_out) {
    __shared__ float s_cos[1024];
    __shared__ int s_keep;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int b = w; b < B; b += nw) {
        const TX* x = X + (int64_t)b * ldx;
        const float* y = Y + (int64_t)b * ldy;
        float sxx = 0.f, syy = 0.f;
        for (int k = lane; k < d; k += kWave) {
            const float xv = (float)x[k], yv = y[k];
            sxx += xv * xv;
            syy += yv * yv;
        }
        sxx = wave_sum<float>(sxx);
        syy = wave_sum<float>(syy);
        const float dx = fmaxf(sqrtf(sxx), 1e-12f), dy = fmaxf(sqrtf(syy), 1e-12f);
        float ah = 0.f, bh = 0.f, c = 0.f;
        for (int k = lane; k < d; k += kWave) {
            const float xh = (float)x[k] / dx, yh = y[k] / dy;
            ah += xh * xh;
            bh += yh * yh;
            c += xh * yh;
        }
        ah = wave_sum<float>(ah);
        bh = wave_sum<float>(bh);
        c = wave_sum<float>(c);
        const float ax = fmaxf(sqrtf(ah), 1e-8f), ay = fmaxf(sqrtf(bh), 1e-8f);
        if (lane == 0) s_cos[b] = c / (ax * ay);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float sum = 0.f;
        for (int b = 0; b < B; ++b) sum += s_cos[b];   // fixed order
        const float L = 1.f - sum / (float)B;
        // the solve that made the plan finished (final status, stop set, no stalled
        // workgroup): checked here, not by extra launches on the caller's side
        const bool solved = sk_info == nullptr ||
                            (sk_info->status != OTF_SK_TIMEOUT && sk_info->status != OTF_SK_RUNNING &&
                             sk_info->stop != 0 && sk_info->stalled == 0);
        const int keep = (ok == nullptr || ok[0] != 0) && solved && finite_val(L);
        s_keep = keep;
        loss[0] = keep ? L : 0.f;
        if (keep_out) keep_out[0] = (uint8_t)keep;
    }
    __syncthreads();
    const bool keep = s_keep != 0;
    const float invB = 1.f / (float)B;
    for (int b = w; b < B; b += nw) {
        const TX* x = X + (int64_t)b * ldx;
        const float* y = Y + (int64_t)b * ldy;
        float* ox = gx + (int64_t)b * ldgx;
        float* oy = gy + (int64_t)b * ldgy;
        if (!keep) {
            for (int k = lane; k < d; k += kWave) ox[k] = oy[k] = 0.f;
            continue;
        }
        // the row's norms again (bitwise the values of the first pass: same order)
        float sxx = 0.f, syy = 0.f;
        for (int k = lane; k < d; k += kWave) {
            const float xv = (float)x[k], yv = y[k];
            sxx += xv * xv;
            syy += yv * yv;
        }
        sxx = wave_sum<float>(sxx);
        syy = wave_sum<float>(syy);
        const float nx = sqrtf(sxx), ny = sqrtf(syy);
        const float dx = fmaxf(nx, 1e-12f), dy = fmaxf(ny, 1e-12f);
        float ah = 0.f, bh = 0.f;
        for (int k = lane; k < d; k += kWave) {
            const float xh = (float)x[k] / dx, yh = y[k] / dy;
            ah += xh * xh;
            bh += yh * yh;
        }
        ah = wave_sum<float>(ah);
        bh = wave_sum<float>(bh);
        const float ax = fmaxf(sqrtf(ah), 1e-8f), ay = fmaxf(sqrtf(bh), 1e-8f);
        const float cs = s_cos[b];
        const float tx = -cs * invB;                               // xt . g_xt (= yt . g_yt)
        const float sx = cs * invB * (ah / (ax * ax) - 1.f);       // xh . g_xh
        const float sy = cs * invB * (bh / (ay * ay) - 1.f);
        const bool cx = nx > 1e-12f, cy = ny > 1e-12f;
        for (int k = lane; k < d; k += kWave) {
            const float xh = (float)x[k] / dx, yh = y[k] / dy;
            const float xt = xh / ax, yt = yh / ay;
            const float gxh = (-invB * yt - tx * xt) / ax;
            const float gyh = (-invB * xt - tx * yt) / ay;
            ox[k] = cx ? (gxh - sx * xh) / dx : gxh / dx;
            oy[k] = cy ? (gyh - sy * yh) / dy : gyh / dy;
        }
    }
}

// Backward of the plan apply ot = pet @ Tn^T together with the loss scaling, ONE launch:
//   g_pet[b][j] = sum_i G[b][i] Tn[i][j],  G = g_loss * gy + g_ot   (B x d2)
//   g_mri       = g_loss * gx                                       (B x d)
// A skinny product (B <= a few tens of rows): workgroup = 64 output columns, its 8
// waves split the d rows of Tn (coalesced 256-B row segments), G staged transposed
// in LDS (8 batch rows per pass: two 16-B broadcast reads per Tn element), the 8
// slices added in a fixed order.  The generic 64 x 64-tile GEMM ran one workgroup
// per 64 output columns with K in 16-deep steps: 84 us for 8 x 512 x 512.  Without
// g_ot and keep = 0 the plan may hold NaN: g_pet is written as exact zeros.
constexpr int kAbB = 8;        // batch rows per pass
constexpr int kAbS = 8;        // row slices (waves)
__global__ __launch_bounds__(512) void ot_align_backward_kernel(
    const float* gx, int64_t ldgx, const float* gy, int64_t ldgy, const float* g_ot, int64_t ldgo,
    const float* g_loss, const uint8_t* keep, const float* Tn, int64_t ldt, int B, int d, int d2,
    float* g_mri, int64_t ldm, float* g_pet, int64_t ldp) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* Gt = smem;                        // [d][kAbB]
    float* red = smem + (size_t)d * kAbB;    // [kAbS][kAbB][64]
    const int tid = threadIdx.x, jl = tid & 63, ks = tid >> 6;
    const float gl = g_loss ? g_loss[0] : 0.f;
    const bool zero = g_ot == nullptr && keep != nullptr && keep[0] == 0;
    // g_mri: grid-strided elementwise share of every workgroup
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + tid; e < (int64_t)B * d; e += (int64_t)gridDim.x * blockDim.x) {
        const int b = (int)(e / d), i = (int)(e % d);
        g_mri[(int64_t)b * ldm + i] = gl * gx[(int64_t)b * ldgx + i];
    }
    const int j = blockIdx.x * 64 + jl;
    const int i0 = (int)((int64_t)d * ks / kAbS), i1 = (int)((int64_t)d * (ks + 1) / kAbS);
    for (int b0 = 0; b0 < B; b0 += kAbB) {
        __syncthreads();
        for (int e = tid; e < d * kAbB; e += blockDim.x) {
            const int i = e / kAbB, bb = e % kAbB, b = b0 + bb;
            float g = 0.f;
            if (b < B) {
                g = gl * gy[(int64_t)b * ldgy + i];
                if (g_ot) g += g_ot[(int64_t)b * ldgo + i];
            }
            Gt[e] = g;
        }
        __syncthreads();
        float acc[kAbB];
#pragma unroll
        for (int bb = 0; bb < kAbB; ++bb) acc[bb] = 0.f;
        if (j < d2 && !zero) {
            // unrolled so 16 independent Tn loads per lane are in flight (the rolled loop
            // waited one memory latency per row: 23.8 us at d = d2 = 512, B = 8)
#pragma unroll 16
            for (int i = i0; i < i1; ++i) {
                const float t = Tn[(int64_t)i * ldt + j];
                const float4 g0 = *reinterpret_cast<const float4*>(&Gt[i * kAbB]);
                const float4 g1 = *reinterpret_cast<const float4*>(&Gt[i * kAbB + 4]);
                acc[0] += g0.x * t; acc[1] += g0.y * t; acc[2] += g0.z * t; acc[3] += g0.w * t;
                acc[4] += g1.x * t; acc[5] += g1.y * t; acc[6] += g1.z * t; acc[7] += g1.w * t;
            }
        }
#pragma unroll
        for (int bb = 0; bb < kAbB; ++bb) red[(ks * kAbB + bb) * 64 + jl] = acc[bb];
        __syncthreads();
        if (ks == 0 && j < d2) {
            for (int bb = 0; bb < kAbB && b0 + bb < B; ++bb) {
                float sum = red[bb * 64 + jl];
#pragma unroll
                for (int q = 1; q < kAbS; ++q) sum += red[(q * kAbB + bb) * 64 + jl];
                g_pet[(int64_t)(b0 + bb) * ldp + j] = sum;
            }
        }
    }
}

}  // namespace

// Host launcher for the tiled GEMM, shared with the other translation units.
template <typename TA, typename TB, typename TACC, typename TOUT>
int launch_gemm(const TA* A, int64_t sa0, int64_t sa1, const TB* B, int64_t sb0, int64_t sb1,
                TOUT* out, int64_t ldo, int M, int N, int K, TACC alpha, TACC beta,
                const TACC* rowadd, const TACC* coladd, hipStream_t s) {
    if (M > 65535 * GT) return OTF_EUNSUPPORTED;
    dim3 grid((unsigned)((N + GT - 1) / GT), (unsigned)((M + GT - 1) / GT));
    gemm_kernel<TA, TB, TACC, TOUT><<<grid, 256, 0, s>>>(A, sa0, sa1, B, sb0, sb1, out, ldo, M, N,
                                                         K, alpha, beta, rowadd, coladd);
    OTF_HIP(hipGetLastError());
    return OTF_OK;
}
template int launch_gemm<float, float, double, double>(const float*, int64_t, int64_t,
                                                       const float*, int64_t, int64_t, double*,
                                                       int64_t, int, int, int, double, double,
                                                       const double*, const double*, hipStream_t);
}  // namespace otf

extern "C" {

size_t otf_feature_cost_workspace_size(int64_t n, int64_t n2, int64_t d, int64_t d2) {
    using otf::align_up;
    return align_up(8 * (size_t)n, 256) + align_up(8 * (size_t)n2, 256) +
           align_up(8 * (size_t)d, 256) + align_up(8 * (size_t)d2, 256) +
           align_up(8 * (size_t)(n * d2), 256);
}

}  // extern "C"

namespace otf {
namespace {
template <typename TI>
int feature_cost_t(const TI* X, int64_t ldx, const TI* Y, int64_t ldy, int64_t n, int64_t n2,
                   int64_t d, int64_t d2, const double* Ts, int64_t ldts, const double* ts_diag,
                   int32_t weights_mode, double* M, int64_t ldm, void* workspace, size_t ws_bytes,
                   hipStream_t s) {
    if (!X || !Y || !M || !workspace || n <= 0 || n2 <= 0 || d <= 0 || d2 <= 0) return OTF_EINVAL;
    if (!Ts && !ts_diag) return OTF_EINVAL;
    if ((ts_diag || weights_mode == 1) && n != n2) return OTF_EINVAL;
    if (weights_mode != 0 && weights_mode != 1) return OTF_EINVAL;
    if (ldx < d || ldy < d2 || ldm < d2 || (Ts && ldts < n2)) return OTF_EINVAL;
    if (ws_bytes < otf_feature_cost_workspace_size(n, n2, d, d2)) return OTF_EINVAL;
    if (n > 65535 * 64 || d > 65535 * 64 || d2 > 65535 * 64) return OTF_EUNSUPPORTED;
    char* p = (char*)workspace;
    double* w1 = (double*)p; p += align_up(8 * (size_t)n, 256);
    double* w2 = (double*)p; p += align_up(8 * (size_t)n2, 256);
    double* t1 = (double*)p; p += align_up(8 * (size_t)d, 256);
    double* t2 = (double*)p; p += align_up(8 * (size_t)d2, 256);
    double* Z = (double*)p;

    const int nmax = (int)(n > n2 ? n : n2);
    ts_sums_kernel<<<(nmax + 255) / 256, 256, 0, s>>>(Ts, ldts, ts_diag, (int)n, (int)n2,
                                                      weights_mode, w1, w2);
    OTF_HIP(hipGetLastError());
    weighted_sq_colsum_kernel<TI><<<(int)((d + 255) / 256), 256, 0, s>>>(X, ldx, (int)n, (int)d, w1, t1);
    weighted_sq_colsum_kernel<TI><<<(int)((d2 + 255) / 256), 256, 0, s>>>(Y, ldy, (int)n2, (int)d2, w2, t2);
    OTF_HIP(hipGetLastError());
    // Z = Ts @ Y  (n x d2)
    if (ts_diag) {
        diag_scale_kernel<TI><<<256, 256, 0, s>>>(Y, ldy, (int)n, (int)d2, ts_diag, Z);
    } else {
        dim3 grid((unsigned)((d2 + GT - 1) / GT), (unsigned)((n + GT - 1) / GT));
        gemm_kernel<double, TI, double, double><<<grid, 256, 0, s>>>(
            Ts, ldts, 1, Y, ldy, 1, Z, d2, (int)n, (int)d2, (int)n2, 1.0, 0.0, nullptr, nullptr);
    }
    OTF_HIP(hipGetLastError());
    // M = -2 X^T Z + t1[:, None] + t2[None, :]   (d x d2, sum over the n samples)
    dim3 grid((unsigned)((d2 + GT - 1) / GT), (unsigned)((d + GT - 1) / GT));
    gemm_kernel<TI, double, double, double><<<grid, 256, 0, s>>>(
        X, 1, ldx, Z, d2, 1, M, ldm, (int)d, (int)d2, (int)n, -2.0, 0.0, t1, t2);
    OTF_HIP(hipGetLastError());
    return OTF_OK;
}
}  // namespace
}  // namespace otf

extern "C" {

int otf_feature_cost(const float* X, int64_t ldx, const float* Y, int64_t ldy, int64_t n,
                     int64_t n2, int64_t d, int64_t d2, const double* Ts, int64_t ldts,
                     const double* ts_diag, int32_t weights_mode, double* M, int64_t ldm,
                     void* workspace, size_t ws_bytes, otf_stream_t stream) {
    return otf::feature_cost_t<float>(X, ldx, Y, ldy, n, n2, d, d2, Ts, ldts, ts_diag, weights_mode,
                                      M, ldm, workspace, ws_bytes, (hipStream_t)stream);
}

int otf_feature_cost_ex(const void* X, int64_t ldx, const void* Y, int64_t ldy, int32_t in_dtype,
                        int64_t n, int64_t n2, int64_t d, int64_t d2, const double* Ts,
                        int64_t ldts, const double* ts_diag, int32_t weights_mode, double* M,
                        int64_t ldm, void* workspace, size_t ws_bytes, otf_stream_t stream) {
    hipStream_t s = (hipStream_t)stream;
    switch (in_dtype) {
        case OTF_F32:
            return otf::feature_cost_t<float>((const float*)X, ldx, (const float*)Y, ldy, n, n2, d, d2,
                                              Ts, ldts, ts_diag, weights_mode, M, ldm, workspace,
                                              ws_bytes, s);
        case OTF_BF16:
            return otf::feature_cost_t<otf::bf16>((const otf::bf16*)X, ldx, (const otf::bf16*)Y, ldy, n,
                                                  n2, d, d2, Ts, ldts, ts_diag, weights_mode, M, ldm,
                                                  workspace, ws_bytes, s);
        case OTF_F16:
            return otf::feature_cost_t<_Float16>((const _Float16*)X, ldx, (const _Float16*)Y, ldy, n,
                                                 n2, d, d2, Ts, ldts, ts_diag, weights_mode, M, ldm,
                                                 workspace, ws_bytes, s);
        default:
            return OTF_EINVAL;
    }
}

size_t otf_coupled_cost_workspace_size(int64_t p, int64_t q, int64_t r) {
    using otf::align_up;
    return align_up(8 * (size_t)p, 256) + align_up(8 * (size_t)q, 256) +
           align_up(8 * (size_t)(r * q), 256);
}

int otf_coupled_cost(const float* A, int64_t a0, int64_t a1, const float* B, int64_t b0,
                     int64_t b1, int64_t p, int64_t q, int64_t r, int64_t s_, const double* T,
                     int64_t ldt, const double* w1, const double* w2, double* M, int64_t ldm,
                     void* workspace, size_t ws_bytes, otf_stream_t stream) {
    using otf::align_up;
    if (!A || !B || !T || !w1 || !w2 || !M || !workspace) return OTF_EINVAL;
    if (p <= 0 || q <= 0 || r <= 0 || s_ <= 0 || ldt < s_ || ldm < q) return OTF_EINVAL;
    if (ws_bytes < otf_coupled_cost_workspace_size(p, q, r)) return OTF_EINVAL;
    if (p > 65535LL * otf::GT || r > 65535LL * otf::GT || q > 2147483647LL || s_ > 2147483647LL)
        return OTF_EUNSUPPORTED;
    hipStream_t st = (hipStream_t)stream;
    char* w = (char*)workspace;
    double* t1 = (double*)w; w += align_up(8 * (size_t)p, 256);
    double* t2 = (double*)w; w += align_up(8 * (size_t)q, 256);
    double* Z = (double*)w;
    otf::weighted_sq_strided_kernel<<<(int)((p + 255) / 256), 256, 0, st>>>(A, a0, a1, (int)p, (int)r, w1, t1);
    otf::weighted_sq_strided_kernel<<<(int)((q + 255) / 256), 256, 0, st>>>(B, b0, b1, (int)q, (int)s_, w2, t2);
    OTF_HIP(hipGetLastError());
    // Z = T B^T  (r x q)
    {
        dim3 grid((unsigned)((q + otf::GT - 1) / otf::GT), (unsigned)((r + otf::GT - 1) / otf::GT));
        otf::gemm_kernel<double, float, double, double><<<grid, 256, 0, st>>>(
            T, ldt, 1, B, b1, b0, Z, q, (int)r, (int)q, (int)s_, 1.0, 0.0, nullptr, nullptr);
    }
    // M = -2 A Z + t1[:, None] + t2[None, :]
    {
        dim3 grid((unsigned)((q + otf::GT - 1) / otf::GT), (unsigned)((p + otf::GT - 1) / otf::GT));
        otf::gemm_kernel<float, double, double, double><<<grid, 256, 0, st>>>(
            A, a0, a1, Z, q, 1, M, ldm, (int)p, (int)q, (int)r, -2.0, 0.0, t1, t2);
    }
    OTF_HIP(hipGetLastError());
    return OTF_OK;
}

int otf_plan_postprocess(const void* T, int64_t d, int64_t d2, int64_t ldt, int32_t dtype,
                         float nan_fill, int32_t rownorm, float* Tn, int64_t ldtn,
                         otf_stream_t stream) {
    if (!T || !Tn || d <= 0 || d2 <= 0 || ldt < d2 || ldtn < d2) return OTF_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const int grid = d < 4096 ? (int)d : 4096;
    if (dtype == OTF_F64)
        otf::postprocess_kernel<double><<<grid, 256, 0, s>>>((const double*)T, (int)d, (int)d2, ldt,
                                                             nan_fill, rownorm, Tn, ldtn);
    else if (dtype == OTF_F32)
        otf::postprocess_kernel<float><<<grid, 256, 0, s>>>((const float*)T, (int)d, (int)d2, ldt,
                                                            nan_fill, rownorm, Tn, ldtn);
    else
        return OTF_EINVAL;
    OTF_HIP(hipGetLastError());
    return OTF_OK;
}

int otf_plan_postprocess_apply(const void* T, int64_t d, int64_t d2, int64_t ldt, int32_t dtype,
                               float nan_fill, int32_t rownorm, const float* Z, int64_t ldz,
                               int64_t B, float* out, int64_t ldo, float* Tn, int64_t ldtn,
                               otf_stream_t stream) {
    if (!T || !Z || !out || d <= 0 || d2 <= 0 || B <= 0 || ldt < d2 || ldz < d2 || ldo < d ||
        (Tn && ldtn < d2))
        return OTF_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const int grid = d < 4096 ? (int)d : 4096;
    if (dtype == OTF_F64)
        otf::postprocess_apply_kernel<double><<<grid, 256, 0, s>>>(
            (const double*)T, (int)d, (int)d2, ldt, nan_fill, rownorm, Z, ldz, (int)B, out, ldo, Tn, ldtn);
    else if (dtype == OTF_F32)
        otf::postprocess_apply_kernel<float><<<grid, 256, 0, s>>>(
            (const float*)T, (int)d, (int)d2, ldt, nan_fill, rownorm, Z, ldz, (int)B, out, ldo, Tn, ldtn);
    else
        return OTF_EINVAL;
    OTF_HIP(hipGetLastError());
    return OTF_OK;
}

int otf_gemm_f32(const float* A, int64_t sa0, int64_t sa1, const float* B, int64_t sb0,
                 int64_t sb1, float* out, int64_t ldo, int64_t M, int64_t N, int64_t K,
                 float alpha, float beta, otf_stream_t stream) {
    if (!A || !B || !out || M <= 0 || N <= 0 || K <= 0 || ldo < N) return OTF_EINVAL;
    if (M > 65535LL * otf::GT || N > 2147483647LL) return OTF_EUNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    dim3 grid((unsigned)((N + otf::GT - 1) / otf::GT), (unsigned)((M + otf::GT - 1) / otf::GT));
    otf::gemm_kernel<float, float, float, float><<<grid, 256, 0, s>>>(
        A, sa0, sa1, B, sb0, sb1, out, ldo, (int)M, (int)N, (int)K, alpha, beta, nullptr, nullptr);
    OTF_HIP(hipGetLastError());
    return OTF_OK;
}

int otf_cosine_align(const void* X, int64_t ldx, int32_t x_dtype, const float* Y, int64_t ldy,
                     int64_t B, int64_t d, const uint8_t* ok, const otf_sinkhorn_info* sk_info,
                     float* loss, float* gx, int64_t ldgx, float* gy, int64_t ldgy, uint8_t* keep_out,
                     otf_stream_t stream) {
    if (!X || !Y || !loss || !gx || !gy || B <= 0 || d <= 0 || ldx < d || ldy < d || ldgx < d ||
        ldgy < d)
        return OTF_EINVAL;
    if (B > 1024) return OTF_EUNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    if (x_dtype == OTF_F32)
        otf::cosine_align_kernel<float><<<1, 1024, 0, s>>>((const float*)X, ldx, Y, ldy, (int)B, (int)d, ok,
                                                           sk_info, loss, gx, ldgx, gy, ldgy, keep_out);
    else if (x_dtype == OTF_BF16)
        otf::cosine_align_kernel<otf::bf16><<<1, 1024, 0, s>>>((const otf::bf16*)X, ldx, Y, ldy, (int)B,
                                                               (int)d, ok, sk_info, loss, gx, ldgx, gy, ldgy, keep_out);
    else if (x_dtype == OTF_F16)
        otf::cosine_align_kernel<_Float16><<<1, 1024, 0, s>>>((const _Float16*)X, ldx, Y, ldy, (int)B,
                                                              (int)d, ok, sk_info, loss, gx, ldgx, gy, ldgy, keep_out);
    else
        return OTF_EINVAL;
    OTF_HIP(hipGetLastError());
    return OTF_OK;
}

int otf_ot_align_backward(const float* gx, int64_t ldgx, const float* gy, int64_t ldgy,
                          const float* g_ot, int64_t ldgo, const float* g_loss, const uint8_t* keep,
                          const float* Tn, int64_t ldt, int64_t B, int64_t d, int64_t d2, float* g_mri,
                          int64_t ldm, float* g_pet, int64_t ldp, otf_stream_t stream) {
    if (!gx || !gy || !Tn || !g_mri || !g_pet || B <= 0 || d <= 0 || d2 <= 0 || ldgx < d ||
        ldgy < d || ldt < d2 || ldm < d || ldp < d2 || (g_ot && ldgo < d))
        return OTF_EINVAL;
    const size_t lds = ((size_t)d * otf::kAbB + (size_t)otf::kAbS * otf::kAbB * 64) * sizeof(float);
    if (lds > 160 * 1024) return OTF_EUNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    const int grid = (int)((d2 + 63) / 64);
    otf::ot_align_backward_kernel<<<grid, 512, lds, s>>>(gx, ldgx, gy, ldgy, g_ot, ldgo, g_loss, keep, Tn,
                                                        ldt, (int)B, (int)d, (int)d2, g_mri, ldm, g_pet,
                                                        ldp);
    OTF_HIP(hipGetLastError());
    return OTF_OK;
}

}  // extern "C"
