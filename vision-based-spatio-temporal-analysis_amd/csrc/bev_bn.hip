// bev_bn.hip -- BatchNorm with batch statistics for training the backbone trunk (timm's BN in
// model.train(), reference train.py:222), on NHWC activations viewed as rows [M][C] (M = N*H*W), fp32:
//
//   forward   k_bn_partial<Stats>  per block of rows: per-channel (sum z, sum z^2) in double
//             k_bn_finalize        mean, biased var, rstd = 1/sqrt(var + eps), scale = gamma*rstd,
//                                  shift = beta - mean*scale; running_mean / running_var updated with
//                                  the momentum rule and the unbiased variance (torch's train-mode BN)
//             k_bn_apply           y = act(z*scale + shift (+ residual)), act = none / ReLU / SiLU (float4)
//   backward  k_bn_partial<GradsT> per channel (sum g, sum g*xhat), g = dy * act'(u) (ReLU: y > 0 from the
//                                  saved output, or -- no residual -- u = z*scale + shift > 0 recomputed from
//                                  z (act 3); SiLU: u recomputed), xhat = (z - mean) * rstd
//             k_bn_bwd_finalize    k1 = sum g / M, k2 = sum g xhat / M, dbeta, dgamma
//             k_bn_bwd_apply       dz = gamma * rstd * (g - k1 - xhat * k2); d(residual) = g
//   Under autocast the forward statistics come from the fp16 conv's epilogue instead (bev_conv2d_h16_bnstats_f32):
//             k_bn_finalize_tiles  per-tile (sum, M2 about the tile mean) combined in double (two passes)
//   A BN module in eval() inside a training model ("frozen": running statistics) uses the same apply and
//   backward with k1 = k2 = 0 (its statistics are constants).
//
// Per-image channel sums (the SqueezeExcite squeeze and its backward, EfficientNet training):
//             k_img_partial / k_img_finalize   out[n][c] = sum_p x[n][p][c] (* x2[n][p][c])
//             k_chan_affine                     y[n][p][c] = x[n][p][c] * a[n][c] (+ b[n][c])
//
// The partials are one per (row block, channel): deterministic, no float atomics.  Every pass is a
// streaming read of the activation (HBM-bound; a few us per trunk layer at BEV-rig sizes).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bev_mi355x.h"
#include "bev_act.h"

namespace {

constexpr int BN_T = 256;
constexpr int BN_ROWS = 1024;  // rows per block
constexpr int BN_QB = 64;      // channel quads per block (256 channels)
constexpr int BN_U = 4;        // rows per load batch of the streaming passes

struct Stats {  // (z, z^2)
    const float *z;
    __device__ void at(int64_t i, int, float4 &a, float4 &b) const {
        const float4 v = *(const float4 *)(z + i);
        a = v;
        b = make_float4(v.x * v.x, v.y * v.y, v.z * v.z, v.w * v.w);
    }
};

// u = z * scale + shift, two roundings (the library builds with -ffp-contract=off: no fma) -- the one expression
// k_bn_apply writes and the backward's recomputed ReLU mask / SiLU argument use, so they agree bit for bit
__device__ __forceinline__ float bn_u(float z, float s, float h) { return z * s + h; }

// SiLU' (u) = s (1 + u (1 - s)), s = sigmoid(u) = 1 / (1 + exp(-u)) (torch's SiLU backward)
__device__ __forceinline__ float silu_grad(float u) {
    const float sg = sigmoid_hw(u);
    return sg * (1.0f + u * (1.0f - sg));
}

// g = dy * act'(u) for the 4 channels c .. c+3 of element i (act 1: y > 0 from the saved output; act 3: ReLU of a
// layer without residual, y > 0 recomputed from z so y is not read; act 4: ReLU, y > 0 from the forward's mask
// bytes (k_bn_apply_q's `mask`: 1 B per 4 elements instead of re-reading the 4-B y twice); act 2: u = z * scale +
// shift)
__device__ __forceinline__ void act_grad(float (&g)[4], const float4 d, const float *y, const float4 v,
                                         const float *scale, const float *shift, int act, int64_t i, int c) {
    g[0] = d.x;
    g[1] = d.y;
    g[2] = d.z;
    g[3] = d.w;
    if (act == 1) {
        const float4 o = *(const float4 *)(y + i);
        const float ov[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) g[u] = ov[u] > 0.f ? g[u] : 0.f;
    } else if (act == 4) {  // ReLU, the forward's mask bytes (bit u of byte i / 4: y[i + u] > 0) instead of y
        const unsigned m = reinterpret_cast<const uint8_t *>(y)[i >> 2];
#pragma unroll
        for (int u = 0; u < 4; ++u) g[u] = (m >> u) & 1u ? g[u] : 0.f;
    } else if (act == 3) {  // ReLU without residual: y > 0 <=> u > 0, u exactly as k_bn_apply computed it
        const float zv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) g[u] = bn_u(zv[u], scale[c + u], shift[c + u]) > 0.f ? g[u] : 0.f;
    } else if (act == 2) {
        const float zv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) g[u] *= silu_grad(bn_u(zv[u], scale[c + u], shift[c + u]));
    }
}

// act_grad with the activation as a template parameter (no per-element branch, so the batched row loops below keep
// every load of a batch in flight): the same expressions, so the same values
template <int ACT>
__device__ __forceinline__ void act_side(const float *y, int64_t i, float4 &o, unsigned &m) {
    if constexpr (ACT == 1) o = *(const float4 *)(y + i);
    if constexpr (ACT == 4) m = reinterpret_cast<const uint8_t *>(y)[i >> 2];
}
template <int ACT>
__device__ __forceinline__ void act_grad_t(float (&g)[4], const float4 d, const float4 o, const unsigned m,
                                           const float4 v, const float *sc, const float *sh) {
    g[0] = d.x;
    g[1] = d.y;
    g[2] = d.z;
    g[3] = d.w;
    const float ov[4] = {o.x, o.y, o.z, o.w}, zv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        if constexpr (ACT == 1) g[u] = ov[u] > 0.f ? g[u] : 0.f;
        if constexpr (ACT == 4) g[u] = (m >> u) & 1u ? g[u] : 0.f;
        if constexpr (ACT == 3) g[u] = bn_u(zv[u], sc[u], sh[u]) > 0.f ? g[u] : 0.f;
        if constexpr (ACT == 2) g[u] *= silu_grad(bn_u(zv[u], sc[u], sh[u]));
    }
}

template <int ACT>
struct GradsT {  // Grads with a compile-time activation
    const float *dy, *y, *z, *mean, *rstd, *scale, *shift;
    __device__ void at(int64_t i, int c, float4 &a, float4 &b) const {
        const float4 d = *(const float4 *)(dy + i), v = *(const float4 *)(z + i);
        float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
        unsigned m = 0;
        act_side<ACT>(y, i, o, m);
        float sc[4] = {0.f, 0.f, 0.f, 0.f}, sh[4] = {0.f, 0.f, 0.f, 0.f};
        if constexpr (ACT == 2 || ACT == 3) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                sc[u] = scale[c + u];
                sh[u] = shift[c + u];
            }
        }
        float g[4];
        act_grad_t<ACT>(g, d, o, m, v, sc, sh);
        const float zv[4] = {v.x, v.y, v.z, v.w};
        float h[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) h[u] = g[u] * ((zv[u] - mean[c + u]) * rstd[c + u]);
        a = make_float4(g[0], g[1], g[2], g[3]);
        b = make_float4(h[0], h[1], h[2], h[3]);
    }
};

// grid (row blocks, channel slices of BN_QB quads); part [nb][C][2]
template <class F>
__device__ __forceinline__ void k_bn_partial_body(const F &f, int64_t M, int C, double *__restrict__ part) {
    __shared__ double red[BN_T][4][2];
    const int C4 = C / 4, tid = threadIdx.x, blk = blockIdx.x;
    const int qb = C4 < BN_QB ? C4 : BN_QB;  // quads handled per block
    const int q = tid % qb, ph = tid / qb, nph = BN_T / qb;
    const int qg = blockIdx.y * BN_QB + q;
    const int64_t r0 = (int64_t)blk * BN_ROWS, r1 = r0 + BN_ROWS < M ? r0 + BN_ROWS : M;
    double s[4] = {0, 0, 0, 0}, t[4] = {0, 0, 0, 0};
    if (ph < nph && qg < C4) {
        // rows in batches of BN_U: the batch's loads all in flight before the first use (one row at a time left
        // ~2 float4 loads per wave outstanding: latency-, not HBM-bound); the sums still run row by row, in order
        int64_t r = r0 + ph;
        for (; r + (BN_U - 1) * nph < r1; r += BN_U * nph) {
            float4 a[BN_U], b[BN_U];
#pragma unroll
            for (int u = 0; u < BN_U; ++u) f.at((r + u * nph) * C + 4 * qg, 4 * qg, a[u], b[u]);
#pragma unroll
            for (int u = 0; u < BN_U; ++u) {
                s[0] += a[u].x; s[1] += a[u].y; s[2] += a[u].z; s[3] += a[u].w;
                t[0] += b[u].x; t[1] += b[u].y; t[2] += b[u].z; t[3] += b[u].w;
            }
        }
        for (; r < r1; r += nph) {
            float4 a, b;
            f.at(r * C + 4 * qg, 4 * qg, a, b);
            s[0] += a.x; s[1] += a.y; s[2] += a.z; s[3] += a.w;
            t[0] += b.x; t[1] += b.y; t[2] += b.z; t[3] += b.w;
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        red[tid][u][0] = s[u];
        red[tid][u][1] = t[u];
    }
    __syncthreads();
    if (tid < 4 * qb) {
        const int qq = tid / 4, u = tid % 4, c = 4 * (blockIdx.y * BN_QB + qq) + u;
        if (c < C) {
            double a = 0.0, b = 0.0;
            for (int p = 0; p < nph; ++p) {
                a += red[p * qb + qq][u][0];
                b += red[p * qb + qq][u][1];
            }
            double *o = part + ((size_t)blk * C + c) * 2;
            o[0] = a;
            o[1] = b;
        }
    }
}

template <class F>
__global__ __launch_bounds__(BN_T) void k_bn_partial(F f, int64_t M, int C, double *__restrict__ part) {
    k_bn_partial_body(f, M, C, part);
}

// Column sums of part [nb][C][2] for 16 channels per block: 16 row-block phases per channel, LDS reduce.
constexpr int FIN_C = 16, FIN_P = 16;
__device__ inline bool fin_sums(const double *__restrict__ part, int nb, int C, double &a, double &b) {
    __shared__ double red[FIN_P][FIN_C][2];
    const int cl = threadIdx.x % FIN_C, ph = threadIdx.x / FIN_C, c = blockIdx.x * FIN_C + cl;
    double s = 0.0, t = 0.0;
    if (c < C) {
#pragma unroll 4
        for (int k = ph; k < nb; k += FIN_P) {
            s += part[((size_t)k * C + c) * 2];
            t += part[((size_t)k * C + c) * 2 + 1];
        }
    }
    red[ph][cl][0] = s;
    red[ph][cl][1] = t;
    __syncthreads();
    if (ph != 0 || c >= C) return false;
    a = 0.0;
    b = 0.0;
    for (int p = 0; p < FIN_P; ++p) {
        a += red[p][cl][0];
        b += red[p][cl][1];
    }
    return true;
}

__global__ __launch_bounds__(FIN_C * FIN_P) void k_bn_finalize(const double *__restrict__ part, int nb, int64_t M, int C, float eps, float momentum,
                              const float *__restrict__ gamma, const float *__restrict__ beta,
                              float *__restrict__ running_mean, float *__restrict__ running_var,
                              float *__restrict__ mean, float *__restrict__ rstd, float *__restrict__ scale,
                              float *__restrict__ shift) {
    double a, b;
    if (!fin_sums(part, nb, C, a, b)) return;
    const int c = blockIdx.x * FIN_C + threadIdx.x;
    const double mu = a / (double)M;
    double var = b / (double)M - mu * mu;
    var = var > 0.0 ? var : 0.0;
    const float r = (float)(1.0 / __builtin_sqrt(var + (double)eps));
    const float sc = gamma[c] * r;
    mean[c] = (float)mu;
    rstd[c] = r;
    scale[c] = sc;
    shift[c] = beta[c] - (float)mu * sc;
    if (running_mean) {
        const float unb = (float)(M > 1 ? var * (double)M / (double)(M - 1) : var);
        running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mu;
        running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
    }
}

// BatchNorm statistics from the conv epilogue's per-tile partials (k_conv_h16b with stats): channel c's tiles
// part[c][k] = (sum, M2 about the tile mean) over n_k = min(rows, M - k rows) rows, fp32.  One workgroup per
// channel, two passes over its (contiguous) tiles in double: mean = sum_k sum_k / M, then
// M2 = sum_k (M2_k + n_k (mean_k - mean)^2) -- the exact combination (Chan et al.), no per-tile division chain.
// Same outputs and running-stat rule as k_bn_finalize.
constexpr int FT_T = 256;
__device__ __forceinline__ double ft_block_sum(double v, double *red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __syncthreads();  // red[] free (previous use consumed)
    if (lane == 0) red[w] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(FT_T) void k_bn_finalize_tiles(const float *__restrict__ part, int ntiles, int rows,
                                                              int64_t M, int C, float eps, float momentum,
                                                              const float *__restrict__ gamma,
                                                              const float *__restrict__ beta,
                                                              float *__restrict__ running_mean,
                                                              float *__restrict__ running_var,
                                                              float *__restrict__ mean, float *__restrict__ rstd,
                                                              float *__restrict__ scale, float *__restrict__ shift) {
    __shared__ double red[4];
    const int c = blockIdx.x;
    const float2 *pc = reinterpret_cast<const float2 *>(part) + (size_t)c * ntiles;
    double s = 0.0;
    for (int k = threadIdx.x; k < ntiles; k += FT_T) s += (double)pc[k].x;
    const double mu = ft_block_sum(s, red) / (double)M;
    double q = 0.0;
    for (int k = threadIdx.x; k < ntiles; k += FT_T) {
        const int64_t left = M - (int64_t)k * rows;
        const double nk = (double)(left < rows ? left : rows);
        const float2 t = pc[k];
        const double d = (double)t.x / nk - mu;
        q += (double)t.y + nk * d * d;
    }
    const double m2 = ft_block_sum(q, red);
    if (threadIdx.x != 0) return;
    double var = m2 / (double)M;
    var = var > 0.0 ? var : 0.0;
    const float r = (float)(1.0 / __builtin_sqrt(var + (double)eps));
    const float sc = gamma[c] * r;
    mean[c] = (float)mu;
    rstd[c] = r;
    scale[c] = sc;
    shift[c] = beta[c] - (float)mu * sc;
    if (running_mean) {
        const float unb = (float)(M > 1 ? m2 / (double)(M - 1) : var);
        running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mu;
        running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
    }
}

// IT: uint32_t when the element count fits (no 64-bit divisions in the channel decode), else int64_t
// store 4 values: fp32, or fp16 (RNE) when the only readers are fp16-operand kernels (bit-identical to their rounding)
__device__ __forceinline__ void st4(float *p, int64_t e, float4 o) { *(float4 *)(p + e) = o; }
__device__ __forceinline__ void st4(_Float16 *p, int64_t e, float4 o) {
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    *(h4 *)(p + e) = (h4){(_Float16)o.x, (_Float16)o.y, (_Float16)o.z, (_Float16)o.w};
}

template <typename IT, typename OT>
__global__ void k_bn_apply(const float *__restrict__ z, int C, const float *__restrict__ scale,
                           const float *__restrict__ shift, const float *__restrict__ res, int act,
                           OT *__restrict__ y, IT total4) {
    const IT C4 = (IT)(C / 4);
    for (IT i = (IT)blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += (IT)gridDim.x * blockDim.x) {
        const int64_t e = 4 * (int64_t)i;
        const int c = 4 * (int)(i % C4);
        const float4 v = *(const float4 *)(z + e);
        const float4 s = *(const float4 *)(scale + c), h = *(const float4 *)(shift + c);
        float4 o = make_float4(bn_u(v.x, s.x, h.x), bn_u(v.y, s.y, h.y), bn_u(v.z, s.z, h.z), bn_u(v.w, s.w, h.w));
        if (res) {
            const float4 r = *(const float4 *)(res + e);
            o = make_float4(o.x + r.x, o.y + r.y, o.z + r.z, o.w + r.w);
        }
        if (act == 1) o = make_float4(fmaxf(o.x, 0.f), fmaxf(o.y, 0.f), fmaxf(o.z, 0.f), fmaxf(o.w, 0.f));
        if (act == 2)  // torch SiLU: x / (1 + exp(-x))
            o = make_float4(silu_hw(o.x), silu_hw(o.y), silu_hw(o.z), silu_hw(o.w));
        st4(y, e, o);
    }
}

// coef [C][2] = (sum g / M, sum g xhat / M)
__global__ __launch_bounds__(FIN_C * FIN_P) void k_bn_bwd_finalize(const double *__restrict__ part, int nb, int64_t M,
                                                                    int C, int frozen, float *__restrict__ coef,
                                                                    float *__restrict__ dgamma,
                                                                    float *__restrict__ dbeta) {
    double a, b;
    if (!fin_sums(part, nb, C, a, b)) return;
    const int c = blockIdx.x * FIN_C + threadIdx.x;
    dbeta[c] = (float)a;
    dgamma[c] = (float)b;
    coef[2 * c] = frozen ? 0.f : (float)(a / (double)M);
    coef[2 * c + 1] = frozen ? 0.f : (float)(b / (double)M);
}

template <typename IT, typename OT>
__global__ void k_bn_bwd_apply(const float *__restrict__ dy, const float *__restrict__ y, const float *__restrict__ z,
                               int C, const float *__restrict__ mean, const float *__restrict__ rstd,
                               const float *__restrict__ gamma, const float *__restrict__ scale,
                               const float *__restrict__ shift, int act, const float *__restrict__ coef,
                               OT *__restrict__ dz, float *__restrict__ dres, IT total4) {
    const IT C4 = (IT)(C / 4);
    for (IT i = (IT)blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += (IT)gridDim.x * blockDim.x) {
        const int64_t e = 4 * (int64_t)i;
        const int c0 = 4 * (int)(i % C4);
        const float4 d = *(const float4 *)(dy + e), v = *(const float4 *)(z + e);
        float g[4];
        act_grad(g, d, y, v, scale, shift, act, e, c0);
        const float zv[4] = {v.x, v.y, v.z, v.w};
        float o[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int c = c0 + u;
            const float xh = (zv[u] - mean[c]) * rstd[c];
            o[u] = gamma[c] * rstd[c] * (g[u] - coef[2 * c] - xh * coef[2 * c + 1]);
        }
        st4(dz, e, make_float4(o[0], o[1], o[2], o[3]));
        if (dres) *(float4 *)(dres + e) = make_float4(g[0], g[1], g[2], g[3]);
    }
}


// Row-block forms of the two streaming passes (round 5), used when 256 % (C / 4) == 0 (every ResNet trunk width):
// grid = blocks of BNQ_ROWS rows, thread = (channel quad q, row phase), the quad's per-channel constants in registers
// for the whole block -- the grid-stride forms above decode the channel per float4 and re-load 4-7 per-channel
// values per element.  Same arithmetic per element, so identical results.
constexpr int BNQ_ROWS = 256;

template <typename OT, int ACT, bool RES>
__device__ __forceinline__ void bn_apply_one(const float4 v, const float4 rr, const float4 s, const float4 h, OT *y,
                                             uint8_t *mask, int64_t e) {
    float4 o = make_float4(bn_u(v.x, s.x, h.x), bn_u(v.y, s.y, h.y), bn_u(v.z, s.z, h.z), bn_u(v.w, s.w, h.w));
    if constexpr (RES) o = make_float4(o.x + rr.x, o.y + rr.y, o.z + rr.z, o.w + rr.w);
    if constexpr (ACT == 1) o = make_float4(fmaxf(o.x, 0.f), fmaxf(o.y, 0.f), fmaxf(o.z, 0.f), fmaxf(o.w, 0.f));
    if constexpr (ACT == 2) o = make_float4(silu_hw(o.x), silu_hw(o.y), silu_hw(o.z), silu_hw(o.w));
    st4(y, e, o);
    if (mask)  // act 1: bit u = (y[e + u] > 0), what the backward's act 4 reads instead of y
        mask[e >> 2] = (uint8_t)((o.x > 0.f) | ((o.y > 0.f) << 1) | ((o.z > 0.f) << 2) | ((o.w > 0.f) << 3));
}

template <typename OT, int ACT, bool RES>
__global__ __launch_bounds__(256) void k_bn_apply_q(const float *__restrict__ z, int64_t M, int C,
                                                    const float *__restrict__ scale, const float *__restrict__ shift,
                                                    const float *__restrict__ res, OT *__restrict__ y,
                                                    uint8_t *__restrict__ mask) {
    const int tid = threadIdx.x, QP = C / 4, q = tid % QP, ph = tid / QP, nph = 256 / QP;
    const int64_t r0 = (int64_t)blockIdx.x * BNQ_ROWS, r1 = r0 + BNQ_ROWS < M ? r0 + BNQ_ROWS : M;
    const float4 s = *(const float4 *)(scale + 4 * q), h = *(const float4 *)(shift + 4 * q);
    const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
    int64_t r = r0 + ph;
    for (; r + (BN_U - 1) * nph < r1; r += BN_U * nph) {  // BN_U rows' loads in flight at once
        float4 v[BN_U], rr[BN_U];
#pragma unroll
        for (int u = 0; u < BN_U; ++u) {
            const int64_t e = (r + u * nph) * C + 4 * q;
            v[u] = *(const float4 *)(z + e);
            rr[u] = RES ? *(const float4 *)(res + e) : zero;
        }
#pragma unroll
        for (int u = 0; u < BN_U; ++u) bn_apply_one<OT, ACT, RES>(v[u], rr[u], s, h, y, mask, (r + u * nph) * C + 4 * q);
    }
    for (; r < r1; r += nph) {
        const int64_t e = r * C + 4 * q;
        bn_apply_one<OT, ACT, RES>(*(const float4 *)(z + e), RES ? *(const float4 *)(res + e) : zero, s, h, y, mask, e);
    }
}

template <typename OT>
static void launch_bn_apply_q(dim3 g, hipStream_t st, const float *z, int64_t M, int C, const float *scale,
                              const float *shift, const float *res, int act, OT *y, uint8_t *mask) {
#define BN_APPLY_Q(A, R) hipLaunchKernelGGL((k_bn_apply_q<OT, A, R>), g, dim3(256), 0, st, z, M, C, scale, shift, res, y, mask)
    if (res) {
        if (act == 1) BN_APPLY_Q(1, true); else if (act == 2) BN_APPLY_Q(2, true); else BN_APPLY_Q(0, true);
    } else {
        if (act == 1) BN_APPLY_Q(1, false); else if (act == 2) BN_APPLY_Q(2, false); else BN_APPLY_Q(0, false);
    }
#undef BN_APPLY_Q
}

template <typename OT, int ACT>
__global__ __launch_bounds__(256) void k_bn_bwd_apply_q(const float *__restrict__ dy, const float *__restrict__ y,
                                                        const float *__restrict__ z, int64_t M, int C,
                                                        const float *__restrict__ mean, const float *__restrict__ rstd,
                                                        const float *__restrict__ gamma,
                                                        const float *__restrict__ scale,
                                                        const float *__restrict__ shift,
                                                        const float *__restrict__ coef, OT *__restrict__ dz,
                                                        float *__restrict__ dres) {
    const int tid = threadIdx.x, QP = C / 4, q = tid % QP, ph = tid / QP, nph = 256 / QP;
    const int64_t r0 = (int64_t)blockIdx.x * BNQ_ROWS, r1 = r0 + BNQ_ROWS < M ? r0 + BNQ_ROWS : M;
    const int c0 = 4 * q;
    float mu[4], rs[4], gr[4], k1[4], k2[4], sc[4] = {0.f, 0.f, 0.f, 0.f}, sh[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        mu[u] = mean[c0 + u];
        rs[u] = rstd[c0 + u];
        gr[u] = gamma[c0 + u] * rstd[c0 + u];
        k1[u] = coef[2 * (c0 + u)];
        k2[u] = coef[2 * (c0 + u) + 1];
        if constexpr (ACT == 2 || ACT == 3) {
            sc[u] = scale[c0 + u];
            sh[u] = shift[c0 + u];
        }
    }
    auto one = [&](const float4 d, const float4 v, const float4 o, const unsigned m, const int64_t e) {
        float g[4];
        act_grad_t<ACT>(g, d, o, m, v, sc, sh);
        const float zv[4] = {v.x, v.y, v.z, v.w};
        float out[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const float xh = (zv[u] - mu[u]) * rs[u];
            out[u] = gr[u] * (g[u] - k1[u] - xh * k2[u]);
        }
        st4(dz, e, make_float4(out[0], out[1], out[2], out[3]));
        if (dres) *(float4 *)(dres + e) = make_float4(g[0], g[1], g[2], g[3]);
    };
    int64_t r = r0 + ph;
    for (; r + (BN_U - 1) * nph < r1; r += BN_U * nph) {  // BN_U rows' loads in flight at once
        float4 d[BN_U], v[BN_U], o[BN_U];
        unsigned m[BN_U];
#pragma unroll
        for (int u = 0; u < BN_U; ++u) {
            const int64_t e = (r + u * nph) * C + c0;
            d[u] = *(const float4 *)(dy + e);
            v[u] = *(const float4 *)(z + e);
            o[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            m[u] = 0;
            act_side<ACT>(y, e, o[u], m[u]);
        }
#pragma unroll
        for (int u = 0; u < BN_U; ++u) one(d[u], v[u], o[u], m[u], (r + u * nph) * C + c0);
    }
    for (; r < r1; r += nph) {
        const int64_t e = r * C + c0;
        float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
        unsigned m = 0;
        act_side<ACT>(y, e, o, m);
        one(*(const float4 *)(dy + e), *(const float4 *)(z + e), o, m, e);
    }
}

template <typename OT>
static void launch_bn_bwd_apply_q(dim3 g, hipStream_t st, const float *dy, const float *y, const float *z, int64_t M,
                                  int C, const float *mean, const float *rstd, const float *gamma, const float *scale,
                                  const float *shift, int act, const float *coef, OT *dz, float *dres) {
#define BN_BWD_Q(A) hipLaunchKernelGGL((k_bn_bwd_apply_q<OT, A>), g, dim3(256), 0, st, dy, y, z, M, C, mean, rstd, \
                                       gamma, scale, shift, coef, dz, dres)
    switch (act) {
        case 1: BN_BWD_Q(1); break;
        case 2: BN_BWD_Q(2); break;
        case 3: BN_BWD_Q(3); break;
        case 4: BN_BWD_Q(4); break;
        default: BN_BWD_Q(0); break;
    }
#undef BN_BWD_Q
}

// ---- per-image channel sums and channel affine (SqueezeExcite training) -------------------------------
struct Prod {  // (x * x2, unused)
    const float *x, *x2;
    __device__ void at(int64_t i, int, float4 &a, float4 &b) const {
        const float4 v = *(const float4 *)(x + i);
        if (x2) {
            const float4 w = *(const float4 *)(x2 + i);
            a = make_float4(v.x * w.x, v.y * w.y, v.z * w.z, v.w * w.w);
        } else {
            a = v;
        }
        b = make_float4(0.f, 0.f, 0.f, 0.f);
    }
};

// grid (row blocks, channel slices, images): image n's rows are [n P, (n+1) P); part [N][nb][C][2]
__global__ __launch_bounds__(BN_T) void k_img_partial(Prod f, int64_t P, int C, double *__restrict__ part) {
    const int n = blockIdx.z;
    const int64_t off = (int64_t)n * P * C;
    Prod g{f.x + off, f.x2 ? f.x2 + off : nullptr};
    k_bn_partial_body(g, P, C, part + (size_t)n * gridDim.x * C * 2);
}

__global__ __launch_bounds__(FIN_C * FIN_P) void k_img_finalize(const double *__restrict__ part, int nb, int C,
                                                               float *__restrict__ out) {
    const int n = blockIdx.y;
    double a, b;
    if (!fin_sums(part + (size_t)n * nb * C * 2, nb, C, a, b)) return;
    out[(size_t)n * C + blockIdx.x * FIN_C + threadIdx.x] = (float)a;
}

template <typename IT>
__global__ void k_chan_affine(const float *__restrict__ x, int C, IT P4, const float *__restrict__ a,
                              const float *__restrict__ b, float *__restrict__ y, IT total4) {
    const IT C4 = (IT)(C / 4);
    for (IT i = (IT)blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += (IT)gridDim.x * blockDim.x) {
        const int64_t e = 4 * (int64_t)i;
        const int64_t nc = (int64_t)(i / P4) * C + 4 * (int64_t)(i % C4);  // image n = i / (P * C4)
        const float4 v = *(const float4 *)(x + e), s = *(const float4 *)(a + nc);
        float4 o = make_float4(v.x * s.x, v.y * s.y, v.z * s.z, v.w * s.w);
        if (b) {
            const float4 t = *(const float4 *)(b + nc);
            o = make_float4(o.x + t.x, o.y + t.y, o.z + t.z, o.w + t.w);
        }
        *(float4 *)(y + e) = o;
    }
}

inline int row_blocks(int64_t M) { return (int)((M + BN_ROWS - 1) / BN_ROWS); }
inline bool bn_shape_ok(int64_t M, int C) { return M > 0 && C > 0 && C % 4 == 0 && row_blocks(M) < (1 << 30); }

inline unsigned stream_blocks(int64_t total4) {
    int64_t b = (total4 + 255) / 256;
    return (unsigned)(b > 8192 ? 8192 : b);
}

}  // namespace

extern "C" {

int64_t bev_batchnorm_workspace_bytes(int64_t M, int C) {
    if (!bn_shape_ok(M, C)) return -1;
    return (int64_t)row_blocks(M) * C * 2 * (int64_t)sizeof(double) + (int64_t)C * 2 * (int64_t)sizeof(float);
}

int bev_batchnorm_train_fwd_f32(const float *z, int64_t M, int C, float eps, float momentum, const float *gamma,
                                const float *beta, float *running_mean, float *running_var, float *mean, float *rstd,
                                float *scale, float *shift, void *workspace, void *stream) {
    if (!z || !gamma || !beta || !mean || !rstd || !scale || !shift || !workspace || !bn_shape_ok(M, C) ||
        (!running_mean) != (!running_var))
        return BEV_ERR_ARGS;
    hipStream_t st = (hipStream_t)stream;
    const int nb = row_blocks(M);
    double *part = (double *)workspace;
    const dim3 grid(nb, (C / 4 + BN_QB - 1) / BN_QB);
    hipLaunchKernelGGL(k_bn_partial<Stats>, grid, dim3(BN_T), 0, st, Stats{z}, M, C, part);
    hipLaunchKernelGGL(k_bn_finalize, dim3((C + FIN_C - 1) / FIN_C), dim3(FIN_C * FIN_P), 0, st, part, nb, M, C, eps, momentum, gamma,
                       beta, running_mean, running_var, mean, rstd, scale, shift);
    return (int)hipGetLastError();
}

int bev_batchnorm_finalize_tiles_f32(const float *tile_stats, int ntiles, int rows_per_tile, int64_t M, int C,
                                     float eps, float momentum, const float *gamma, const float *beta,
                                     float *running_mean, float *running_var, float *mean, float *rstd, float *scale,
                                     float *shift, void *stream) {
    if (!tile_stats || !gamma || !beta || !mean || !rstd || !scale || !shift || M <= 0 || C <= 0 ||
        rows_per_tile <= 0 || ntiles != (M + rows_per_tile - 1) / rows_per_tile || (!running_mean) != (!running_var))
        return BEV_ERR_ARGS;
    hipLaunchKernelGGL(k_bn_finalize_tiles, dim3(C), dim3(FT_T), 0, (hipStream_t)stream,
                       tile_stats, ntiles, rows_per_tile, M, C, eps, momentum, gamma, beta, running_mean, running_var,
                       mean, rstd, scale, shift);
    return (int)hipGetLastError();
}

int bev_batchnorm_apply_ex_f32(const float *z, int64_t M, int C, const float *scale, const float *shift,
                               const float *residual, int act, void *y, int y_half, void *stream) {
    if (!z || !scale || !shift || !y || !bn_shape_ok(M, C) || act < 0 || act > 2) return BEV_ERR_ARGS;
    const int64_t total4 = M * C / 4;
    const dim3 g(stream_blocks(total4));
    hipStream_t st = (hipStream_t)stream;
    if (256 % (C / 4) == 0) {
        const dim3 gq((unsigned)((M + BNQ_ROWS - 1) / BNQ_ROWS));
        if (y_half)
            launch_bn_apply_q<_Float16>(gq, st, z, M, C, scale, shift, residual, act, (_Float16 *)y, nullptr);
        else
            launch_bn_apply_q<float>(gq, st, z, M, C, scale, shift, residual, act, (float *)y, nullptr);
        return (int)hipGetLastError();
    }
    const bool small = total4 < ((int64_t)1 << 32) - 65536 * 256;
    if (y_half && small)
        hipLaunchKernelGGL((k_bn_apply<uint32_t, _Float16>), g, dim3(256), 0, st, z, C, scale, shift, residual, act,
                           (_Float16 *)y, (uint32_t)total4);
    else if (y_half)
        hipLaunchKernelGGL((k_bn_apply<int64_t, _Float16>), g, dim3(256), 0, st, z, C, scale, shift, residual, act,
                           (_Float16 *)y, total4);
    else if (small)
        hipLaunchKernelGGL((k_bn_apply<uint32_t, float>), g, dim3(256), 0, st, z, C, scale, shift, residual, act,
                           (float *)y, (uint32_t)total4);
    else
        hipLaunchKernelGGL((k_bn_apply<int64_t, float>), g, dim3(256), 0, st, z, C, scale, shift, residual, act,
                           (float *)y, total4);
    return (int)hipGetLastError();
}

int bev_batchnorm_apply_mask_f32(const float *z, int64_t M, int C, const float *scale, const float *shift,
                                 const float *residual, float *y, uint8_t *mask, void *stream) {
    if (!z || !scale || !shift || !y || !mask || !bn_shape_ok(M, C) || 256 % (C / 4) != 0) return BEV_ERR_ARGS;
    launch_bn_apply_q<float>(dim3((unsigned)((M + BNQ_ROWS - 1) / BNQ_ROWS)), (hipStream_t)stream, z, M, C, scale,
                             shift, residual, 1, y, mask);
    return (int)hipGetLastError();
}

int bev_batchnorm_apply_f32(const float *z, int64_t M, int C, const float *scale, const float *shift,
                            const float *residual, int act, float *y, void *stream) {
    return bev_batchnorm_apply_ex_f32(z, M, C, scale, shift, residual, act, y, 0, stream);
}

int bev_batchnorm_bwd_ex_f32(const float *dy, const float *y, const float *z, int64_t M, int C, const float *mean,
                             const float *rstd, const float *gamma, const float *scale, const float *shift, int act,
                             int frozen, void *dz, int dz_half, float *dres, float *dgamma, float *dbeta,
                             void *workspace, void *stream) {
    if (!dy || !z || !mean || !rstd || !gamma || !dz || !dgamma || !dbeta || !workspace || !bn_shape_ok(M, C) ||
        act < 0 || act > 4 || ((act == 1 || act == 4) && !y) || ((act == 2 || act == 3) && (!scale || !shift)) ||
        (act == 3 && dres))  // act 3: ReLU recomputed from z, only for a layer without residual
        return BEV_ERR_ARGS;
    hipStream_t st = (hipStream_t)stream;
    const int nb = row_blocks(M);
    double *part = (double *)workspace;
    float *coef = (float *)(part + (size_t)nb * C * 2);
    const dim3 grid(nb, (C / 4 + BN_QB - 1) / BN_QB);
#define BN_PART_G(A) hipLaunchKernelGGL(k_bn_partial<GradsT<A>>, grid, dim3(BN_T), 0, st, \
                                      GradsT<A>{dy, y, z, mean, rstd, scale, shift}, M, C, part)
    switch (act) {
        case 1: BN_PART_G(1); break;
        case 2: BN_PART_G(2); break;
        case 3: BN_PART_G(3); break;
        case 4: BN_PART_G(4); break;
        default: BN_PART_G(0); break;
    }
#undef BN_PART_G
    hipLaunchKernelGGL(k_bn_bwd_finalize, dim3((C + FIN_C - 1) / FIN_C), dim3(FIN_C * FIN_P), 0, st, part, nb, M, C,
                       frozen, coef, dgamma, dbeta);
    const int64_t total4 = M * C / 4;
    const dim3 g(stream_blocks(total4));
    if (256 % (C / 4) == 0) {
        const dim3 gq((unsigned)((M + BNQ_ROWS - 1) / BNQ_ROWS));
        if (dz_half)
            launch_bn_bwd_apply_q<_Float16>(gq, st, dy, y, z, M, C, mean, rstd, gamma, scale, shift, act, coef,
                                            (_Float16 *)dz, dres);
        else
            launch_bn_bwd_apply_q<float>(gq, st, dy, y, z, M, C, mean, rstd, gamma, scale, shift, act, coef,
                                         (float *)dz, dres);
        return (int)hipGetLastError();
    }
    const bool small = total4 < ((int64_t)1 << 32) - 65536 * 256;
    if (dz_half && small)
        hipLaunchKernelGGL((k_bn_bwd_apply<uint32_t, _Float16>), g, dim3(256), 0, st, dy, y, z, C, mean, rstd, gamma,
                           scale, shift, act, coef, (_Float16 *)dz, dres, (uint32_t)total4);
    else if (dz_half)
        hipLaunchKernelGGL((k_bn_bwd_apply<int64_t, _Float16>), g, dim3(256), 0, st, dy, y, z, C, mean, rstd, gamma,
                           scale, shift, act, coef, (_Float16 *)dz, dres, total4);
    else if (small)
        hipLaunchKernelGGL((k_bn_bwd_apply<uint32_t, float>), g, dim3(256), 0, st, dy, y, z, C, mean, rstd, gamma,
                           scale, shift, act, coef, (float *)dz, dres, (uint32_t)total4);
    else
        hipLaunchKernelGGL((k_bn_bwd_apply<int64_t, float>), g, dim3(256), 0, st, dy, y, z, C, mean, rstd, gamma,
                           scale, shift, act, coef, (float *)dz, dres, total4);
    return (int)hipGetLastError();
}

int bev_batchnorm_bwd_f32(const float *dy, const float *y, const float *z, int64_t M, int C, const float *mean,
                          const float *rstd, const float *gamma, const float *scale, const float *shift, int act,
                          int frozen, float *dz, float *dres, float *dgamma, float *dbeta, void *workspace,
                          void *stream) {
    return bev_batchnorm_bwd_ex_f32(dy, y, z, M, C, mean, rstd, gamma, scale, shift, act, frozen, dz, 0, dres, dgamma,
                                    dbeta, workspace, stream);
}

int64_t bev_channel_sums_workspace_bytes(int N, int64_t P, int C) {
    if (N <= 0 || !bn_shape_ok(P, C)) return -1;
    return (int64_t)N * row_blocks(P) * C * 2 * (int64_t)sizeof(double);
}

int bev_channel_sums_f32(const float *x, const float *x2, int N, int64_t P, int C, float *out, void *workspace,
                         void *stream) {
    if (!x || !out || !workspace || N <= 0 || N > 65535 || !bn_shape_ok(P, C)) return BEV_ERR_ARGS;
    hipStream_t st = (hipStream_t)stream;
    const int nb = row_blocks(P);
    double *part = (double *)workspace;
    hipLaunchKernelGGL(k_img_partial, dim3(nb, (C / 4 + BN_QB - 1) / BN_QB, N), dim3(BN_T), 0, st, Prod{x, x2}, P, C,
                       part);
    hipLaunchKernelGGL(k_img_finalize, dim3((C + FIN_C - 1) / FIN_C, N), dim3(FIN_C * FIN_P), 0, st, part, nb, C, out);
    return (int)hipGetLastError();
}

int bev_channel_affine_f32(const float *x, int N, int64_t P, int C, const float *a, const float *b, float *y,
                           void *stream) {
    if (!x || !a || !y || N <= 0 || P <= 0 || C <= 0 || C % 4 != 0 ||
        (((uintptr_t)x | (uintptr_t)a | (uintptr_t)b | (uintptr_t)y) & 15) != 0)
        return BEV_ERR_ARGS;
    const int64_t total4 = (int64_t)N * P * C / 4, P4 = P * (C / 4);
    if (total4 < ((int64_t)1 << 32) - 65536 * 256)
        hipLaunchKernelGGL(k_chan_affine<uint32_t>, dim3(stream_blocks(total4)), dim3(256), 0, (hipStream_t)stream, x,
                           C, (uint32_t)P4, a, b, y, (uint32_t)total4);
    else
        hipLaunchKernelGGL(k_chan_affine<int64_t>, dim3(stream_blocks(total4)), dim3(256), 0, (hipStream_t)stream, x, C,
                           P4, a, b, y, total4);
    return (int)hipGetLastError();
}

}  // extern "C"
