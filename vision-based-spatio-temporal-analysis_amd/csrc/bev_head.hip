// bev_head.hip -- GroupNorm(+ReLU) of the CenterNet BEV head.
//
// Replaces the torch GroupNorm(32) + ReLU of BEVDetector.stem (detector.py:16-30, forward
// detector.py:47-62) on NHWC activations [N][P][C] (P = H*W pixels), fp32:
//
//   k_gn_partial   per (image, block of pixels): sum and sum of squares of every channel group,
//                  in double (deterministic: one partial per block, no atomics)
//   k_gn_finalize  per (image, group): mean, rstd = 1/sqrt(var + eps) (biased variance, like torch);
//                  per (image, channel): scale = rstd * gamma, shift = beta - mean * scale -- the
//                  affine the NEXT conv applies while loading its operand (bev_conv2d_nhwc_ex_f32
//                  in_scale / in_shift / in_relu), so in inference the normalised tensor is never
//                  written; training materialises it with k_gn_apply
//   k_gn_apply     y = relu(x * scale + shift)  (float4)
//   k_gn_bwd_partial / k_gn_bwd_finalize / k_gn_bwd_apply
//                  backward of relu(groupnorm(x)): with g = dy * (y > 0) and xhat = (x - mean) rstd,
//                  dgamma[c] = sum g xhat, dbeta[c] = sum g, and per (image, group)
//                  dx = rstd (g gamma - mean(g gamma) - xhat mean(g gamma xhat)).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bev_mi355x.h"

namespace {

constexpr int GN_T = 256;
// Pixels per partial block.  Round 5: 512 (was 2048 -> 338 workgroups for the 691 k-cell head maps, ~1.3 per CU: the
// partial passes ran at 2.3-3.4 TB/s, latency-bound on their serial double chains); the finalizes reduce the
// partials in parallel (one workgroup per (image, group) / per 16 channels) instead of one thread per output.
constexpr int GN_PIX_PER_BLOCK = 512;

// thread -> (channel quad q, pixel phase): QP = C / 4 quads per pixel, 256 % QP == 0
__global__ __launch_bounds__(GN_T) void k_gn_partial(const float *__restrict__ x, int64_t P, int C, int G,
                                                     double *__restrict__ part /* [N][nb][G][2] */) {
    __shared__ double red[GN_T][2];
    const int n = blockIdx.y, nb = gridDim.x, blk = blockIdx.x, tid = threadIdx.x;
    const int QP = C / 4, q = tid % QP, ph = tid / QP, nph = GN_T / QP;
    const int64_t p0 = (int64_t)blk * GN_PIX_PER_BLOCK, p1 = p0 + GN_PIX_PER_BLOCK < P ? p0 + GN_PIX_PER_BLOCK : P;
    const float *xb = x + (size_t)n * P * C;
    double s0 = 0.0, ss0 = 0.0, s1 = 0.0, ss1 = 0.0;  // two independent chains (pixels p, p + nph)
    int64_t p = p0 + ph;
    for (; p + nph < p1; p += 2 * nph) {
        const float4 v = *(const float4 *)(xb + p * C + 4 * q), w = *(const float4 *)(xb + (p + nph) * C + 4 * q);
        s0 += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
        ss0 += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
        s1 += (double)w.x + (double)w.y + (double)w.z + (double)w.w;
        ss1 += (double)w.x * w.x + (double)w.y * w.y + (double)w.z * w.z + (double)w.w * w.w;
    }
    if (p < p1) {
        const float4 v = *(const float4 *)(xb + p * C + 4 * q);
        s0 += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
        ss0 += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
    }
    red[tid][0] = s0 + s1;
    red[tid][1] = ss0 + ss1;
    __syncthreads();
    // per quad: sum over the phases (fixed order), then per group over its quads
    if (tid < QP) {
        double a = 0.0, b = 0.0;
        for (int t = tid; t < GN_T; t += QP) {
            a += red[t][0];
            b += red[t][1];
        }
        red[tid][0] = a;  // row tid is read only by this thread above (t == tid first)
        red[tid][1] = b;
    }
    __syncthreads();
    const int qpg = C / G / 4;
    if (tid < G) {
        double a = 0.0, b = 0.0;
        for (int t = tid * qpg; t < (tid + 1) * qpg; ++t) {
            a += red[t][0];
            b += red[t][1];
        }
        double *o = part + (((size_t)n * nb + blk) * G + tid) * 2;
        o[0] = a;
        o[1] = b;
    }
}

// fixed-order block sum of two doubles over GN_T threads
__device__ __forceinline__ void gn_block_sum2(double &a, double &b, double (*red)[2]) {
    const int tid = threadIdx.x;
    red[tid][0] = a;
    red[tid][1] = b;
    __syncthreads();
    for (int o = GN_T / 2; o > 0; o >>= 1) {
        if (tid < o) {
            red[tid][0] += red[tid + o][0];
            red[tid][1] += red[tid + o][1];
        }
        __syncthreads();
    }
    a = red[0][0];
    b = red[0][1];
}

// one workgroup per (image, group): the nb partials summed in parallel, then the group's channels' affine
__global__ __launch_bounds__(GN_T) void k_gn_finalize(const double *__restrict__ part, int nb, int64_t P, int C, int G,
                                                      float eps, const float *__restrict__ gamma,
                                                      const float *__restrict__ beta, float *__restrict__ mean,
                                                      float *__restrict__ rstd, float *__restrict__ scale,
                                                      float *__restrict__ shift) {
    __shared__ double red[GN_T][2];
    const int n = blockIdx.x / G, g = blockIdx.x % G, cpg = C / G;
    double a = 0.0, b = 0.0;
    for (int k = threadIdx.x; k < nb; k += GN_T) {
        const double *o = part + (((size_t)n * nb + k) * G + g) * 2;
        a += o[0];
        b += o[1];
    }
    gn_block_sum2(a, b, red);
    const double cnt = (double)P * cpg;
    const double mu = a / cnt;
    double var = b / cnt - mu * mu;
    var = var > 0.0 ? var : 0.0;
    const float r = (float)(1.0 / __builtin_sqrt(var + (double)eps));
    const float m = (float)mu;
    for (int j = threadIdx.x; j < cpg; j += GN_T) {
        const int c = g * cpg + j;
        const float sc = r * gamma[c];
        scale[(size_t)n * C + c] = sc;
        shift[(size_t)n * C + c] = beta[c] - m * sc;
    }
    if (threadIdx.x == 0) {
        mean[(size_t)n * G + g] = m;
        rstd[(size_t)n * G + g] = r;
    }
}

// 4 values out: fp32, or fp16 (RNE) for an output read only by fp16-operand kernels (bit-identical to their rounding)
__device__ __forceinline__ void gn_st4(float *p, int64_t e, float4 o) { *(float4 *)(p + e) = o; }
__device__ __forceinline__ void gn_st4(_Float16 *p, int64_t e, float4 o) {
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    *(h4 *)(p + e) = (h4){(_Float16)o.x, (_Float16)o.y, (_Float16)o.z, (_Float16)o.w};
}

// Streaming passes: grid (pixel blocks of GN_APPLY_PIX, images), thread = (channel quad q, pixel phase), the quad's
// per-channel constants held in registers for the whole block (the round-4 form decoded (image, channel) with
// 64-bit divisions and re-loaded the constants for every float4: 1.3 ms for the 1.4 GB map's backward apply).
constexpr int GN_APPLY_PIX = 256;

template <typename OT>
__global__ __launch_bounds__(GN_T) void k_gn_apply(const float *__restrict__ x, int64_t P, int C,
                                                   const float *__restrict__ scale, const float *__restrict__ shift,
                                                   int relu, OT *__restrict__ y) {
    const int n = blockIdx.y, tid = threadIdx.x;
    const int QP = C / 4, q = tid % QP, ph = tid / QP, nph = GN_T / QP;
    const int64_t p0 = (int64_t)blockIdx.x * GN_APPLY_PIX;
    const int64_t p1 = p0 + GN_APPLY_PIX < P ? p0 + GN_APPLY_PIX : P;
    const float4 s = *(const float4 *)(scale + (size_t)n * C + 4 * q), h = *(const float4 *)(shift + (size_t)n * C + 4 * q);
    const size_t base = (size_t)n * P * C + 4 * q;
    for (int64_t p = p0 + ph; p < p1; p += nph) {
        const int64_t e = base + p * C;
        const float4 v = *(const float4 *)(x + e);
        float4 o = make_float4(v.x * s.x + h.x, v.y * s.y + h.y, v.z * s.z + h.z, v.w * s.w + h.w);
        if (relu) o = make_float4(fmaxf(o.x, 0.f), fmaxf(o.y, 0.f), fmaxf(o.z, 0.f), fmaxf(o.w, 0.f));
        gn_st4(y, e, o);
    }
}

// ---- backward ------------------------------------------------------------------------------------
// part: [N][nb][G][2] (sum g*gamma, sum g*gamma*xhat), cpart: [N][nb][C][2] (sum g*xhat, sum g)
__global__ __launch_bounds__(GN_T) void k_gn_bwd_partial(const float *__restrict__ x, const float *__restrict__ dy,
                                                         int64_t P, int C, int G, const float *__restrict__ mean,
                                                         const float *__restrict__ rstd,
                                                         const float *__restrict__ gamma,
                                                         const float *__restrict__ scale,
                                                         const float *__restrict__ shift, int relu,
                                                         double *__restrict__ part, double *__restrict__ cpart) {
    __shared__ double red[GN_T][4][2];  // per thread, per channel of its quad: (g xhat, g)
    __shared__ double chan[1024][2];    // per channel of this block: (g xhat, g)
    const int n = blockIdx.y, nb = gridDim.x, blk = blockIdx.x, tid = threadIdx.x;
    const int QP = C / 4, q = tid % QP, ph = tid / QP, nph = GN_T / QP;
    const int cpg = C / G;
    const int64_t p0 = (int64_t)blk * GN_PIX_PER_BLOCK, p1 = p0 + GN_PIX_PER_BLOCK < P ? p0 + GN_PIX_PER_BLOCK : P;
    const float *xb = x + (size_t)n * P * C, *db = dy + (size_t)n * P * C;
    float mu[4], rs[4], sc[4], sh[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int c = 4 * q + u, g = c / cpg;
        mu[u] = mean[(size_t)n * G + g];
        rs[u] = rstd[(size_t)n * G + g];
        sc[u] = scale[(size_t)n * C + c];
        sh[u] = shift[(size_t)n * C + c];
    }
    double sgx[4] = {0, 0, 0, 0}, sg[4] = {0, 0, 0, 0};
    for (int64_t p = p0 + ph; p < p1; p += nph) {
        const float4 v = *(const float4 *)(xb + p * C + 4 * q), d = *(const float4 *)(db + p * C + 4 * q);
        const float xv[4] = {v.x, v.y, v.z, v.w}, dv[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const float gr = (relu && !(xv[u] * sc[u] + sh[u] > 0.f)) ? 0.f : dv[u];
            const float xh = (xv[u] - mu[u]) * rs[u];
            sgx[u] += (double)gr * xh;
            sg[u] += (double)gr;
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        red[tid][u][0] = sgx[u];
        red[tid][u][1] = sg[u];
    }
    __syncthreads();
    // per channel: sum over phases
    for (int c = tid; c < C; c += GN_T) {
        const int qq = c / 4, u = c % 4;
        double a = 0.0, b = 0.0;
        for (int t = qq; t < GN_T; t += QP) {
            a += red[t][u][0];
            b += red[t][u][1];
        }
        double *o = cpart + (((size_t)n * nb + blk) * C + c) * 2;
        o[0] = a;
        o[1] = b;
        chan[c][0] = a;
        chan[c][1] = b;
    }
    __syncthreads();
    // per group: sum over its channels of gamma * (.)
    for (int g = tid; g < G; g += GN_T) {
        double a = 0.0, b = 0.0;
        for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
            a += (double)gamma[c] * chan[c][1];
            b += (double)gamma[c] * chan[c][0];
        }
        double *o = part + (((size_t)n * nb + blk) * G + g) * 2;
        o[0] = a;  // sum g * gamma
        o[1] = b;  // sum g * gamma * xhat
    }
}

// dgamma / dbeta [C]: sums of cpart over images and blocks, 16 channels x 16 phases per workgroup
constexpr int GF_C = 16, GF_P = 16;
__global__ __launch_bounds__(GF_C * GF_P) void k_gn_bwd_fin_chan(const double *__restrict__ cpart, int N, int nb,
                                                                 int C, float *__restrict__ dgamma,
                                                                 float *__restrict__ dbeta) {
    __shared__ double red[GF_P][GF_C][2];
    const int cl = threadIdx.x % GF_C, ph = threadIdx.x / GF_C, c = blockIdx.x * GF_C + cl;
    double a = 0.0, b = 0.0;
    if (c < C)
        for (int k = ph; k < N * nb; k += GF_P) {  // k = n * nb + block
            const double *o = cpart + ((size_t)k * C + c) * 2;
            a += o[0];
            b += o[1];
        }
    red[ph][cl][0] = a;
    red[ph][cl][1] = b;
    __syncthreads();
    if (ph != 0 || c >= C) return;
    for (int t = 1; t < GF_P; ++t) {
        a += red[t][cl][0];
        b += red[t][cl][1];
    }
    dgamma[c] = (float)a;
    dbeta[c] = (float)b;
}

// coef [N][G][2] = (mean(g gamma), mean(g gamma xhat)): one workgroup per (image, group)
__global__ __launch_bounds__(GN_T) void k_gn_bwd_fin_group(const double *__restrict__ part, int nb, int64_t P, int C,
                                                           int G, float *__restrict__ coef) {
    __shared__ double red[GN_T][2];
    const int n = blockIdx.x / G, g = blockIdx.x % G;
    double a = 0.0, b = 0.0;
    for (int k = threadIdx.x; k < nb; k += GN_T) {
        const double *o = part + (((size_t)n * nb + k) * G + g) * 2;
        a += o[0];
        b += o[1];
    }
    gn_block_sum2(a, b, red);
    if (threadIdx.x == 0) {
        const double cnt = (double)P * (C / G);
        coef[(size_t)blockIdx.x * 2] = (float)(a / cnt);
        coef[(size_t)blockIdx.x * 2 + 1] = (float)(b / cnt);
    }
}

template <typename OT>
__global__ __launch_bounds__(GN_T) void k_gn_bwd_apply(const float *__restrict__ x, const float *__restrict__ dy,
                                                       int64_t P, int C, int G, const float *__restrict__ mean,
                                                       const float *__restrict__ rstd,
                                                       const float *__restrict__ gamma,
                                                       const float *__restrict__ scale,
                                                       const float *__restrict__ shift, int relu,
                                                       const float *__restrict__ coef, OT *__restrict__ dx) {
    const int n = blockIdx.y, tid = threadIdx.x;
    const int QP = C / 4, q = tid % QP, ph = tid / QP, nph = GN_T / QP;
    const int64_t p0 = (int64_t)blockIdx.x * GN_APPLY_PIX;
    const int64_t p1 = p0 + GN_APPLY_PIX < P ? p0 + GN_APPLY_PIX : P;
    const size_t ng = (size_t)n * G + (4 * q) / (C / G);  // the quad's group ((C / G) % 4 == 0)
    const float mu = mean[ng], rs = rstd[ng], k1 = coef[2 * ng], k2 = coef[2 * ng + 1];
    float sc[4], sh[4], ga[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int c = 4 * q + u;
        sc[u] = scale[(size_t)n * C + c];
        sh[u] = shift[(size_t)n * C + c];
        ga[u] = gamma[c];
    }
    const size_t base = (size_t)n * P * C + 4 * q;
    for (int64_t p = p0 + ph; p < p1; p += nph) {
        const int64_t e = base + p * C;
        const float4 v = *(const float4 *)(x + e), d = *(const float4 *)(dy + e);
        const float xv[4] = {v.x, v.y, v.z, v.w}, dv[4] = {d.x, d.y, d.z, d.w};
        float o[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const float gr = (relu && !(xv[u] * sc[u] + sh[u] > 0.f)) ? 0.f : dv[u];
            const float xh = (xv[u] - mu) * rs;
            o[u] = rs * (gr * ga[u] - k1 - xh * k2);
        }
        gn_st4(dx, e, make_float4(o[0], o[1], o[2], o[3]));
    }
}

inline int nblocks(int64_t P) { return (int)((P + GN_PIX_PER_BLOCK - 1) / GN_PIX_PER_BLOCK); }

bool gn_shape_ok(int N, int64_t P, int C, int G) {
    if (N <= 0 || P <= 0 || C <= 0 || G <= 0 || C % G != 0 || C % 4 != 0 || C > 1024) return false;
    const int QP = C / 4;
    return GN_T % QP == 0 && (C / G) % 4 == 0 && N <= 65535;
}


// ---------------------------------------------------------------------------------------------------------------
// BEVNet head operand (model_wrapper.py:69-75): x[b, h, w, :] = [proj(concat)(b, :, h, w) + bias, pos_enc(:, h, w),
// 0 ... 0] -- the fused warp-sum output (NCHW) plus the BEV projection's bias, the 2 positional channels and the
// zero pad, written channels-last with `cp` channels per cell (what the head's convs read).  One workgroup per
// (frame, BEV row, 64-cell run): the run's P channel rows are read coalesced along w into an LDS tile [64][P + 1],
// the cells' cp channels are written coalesced (the 64 cells' rows form one contiguous block).  The backward
// (k_head_operand_bwd) transposes the first P channels of the gradient back to NCHW the same way.  Values are
// moved unchanged except the one fp32 add s + bias (the reference's own rounding of proj's bias add).
constexpr int HO_T = 256, HO_RUN = 64;

__global__ __launch_bounds__(HO_T) void k_head_operand(const float *__restrict__ s, const float *__restrict__ bias,
                                                       const float *__restrict__ pos, int P, int Hb, int Wb, int cp,
                                                       float *__restrict__ x) {
    extern __shared__ float tile[];  // [HO_RUN][P + 1]
    const int w0 = blockIdx.x * HO_RUN, h = blockIdx.y, b = blockIdx.z, tid = threadIdx.x;
    const int nw = min(HO_RUN, Wb - w0);
    const size_t plane = (size_t)Hb * Wb;
    for (int e = tid; e < P * HO_RUN; e += HO_T) {
        const int c = e / HO_RUN, k = e - c * HO_RUN;
        if (k < nw) tile[k * (P + 1) + c] = s[((size_t)b * P + c) * plane + (size_t)h * Wb + w0 + k] + bias[c];
    }
    __syncthreads();
    float *xr = x + (((size_t)b * Hb + h) * Wb + w0) * cp;
    for (int e = tid; e < nw * cp; e += HO_T) {
        const int k = e / cp, c = e - k * cp;
        float v = 0.0f;
        if (c < P) v = tile[k * (P + 1) + c];
        else if (c < P + 2) v = pos[(size_t)(c - P) * plane + (size_t)h * Wb + w0 + k];
        xr[e] = v;
    }
}

__global__ __launch_bounds__(HO_T) void k_head_operand_bwd(const float *__restrict__ gx, int P, int Hb, int Wb,
                                                           int cp, float *__restrict__ gs) {
    extern __shared__ float tile[];  // [HO_RUN][P + 1]
    const int w0 = blockIdx.x * HO_RUN, h = blockIdx.y, b = blockIdx.z, tid = threadIdx.x;
    const int nw = min(HO_RUN, Wb - w0);
    const size_t plane = (size_t)Hb * Wb;
    const float *gr = gx + (((size_t)b * Hb + h) * Wb + w0) * cp;
    for (int e = tid; e < nw * cp; e += HO_T) {
        const int k = e / cp, c = e - k * cp;
        if (c < P) tile[k * (P + 1) + c] = gr[e];
    }
    __syncthreads();
    for (int e = tid; e < P * HO_RUN; e += HO_T) {
        const int c = e / HO_RUN, k = e - c * HO_RUN;
        if (k < nw) gs[((size_t)b * P + c) * plane + (size_t)h * Wb + w0 + k] = tile[k * (P + 1) + c];
    }
}

// 16-B forms (Wb % 4 == 0, cp % 4 == 0, 16-B aligned buffers -- the bench geometry): sixteen lanes read one
// channel row's 64 cells as float4 (256 B), the cells' block of 64 cp-channel rows is written as float4.  The
// scalar forms above move 4 B per lane and divide by cp per element: 420 / 317 us at 480 x 1440 x P 128 (r05o).
__global__ __launch_bounds__(HO_T) void k_head_operand_v4(const float *__restrict__ s, const float *__restrict__ bias,
                                                          const float *__restrict__ pos, int P, int Hb, int Wb,
                                                          int cp, float *__restrict__ x) {
    extern __shared__ float tile[];  // [HO_RUN][P + 1]
    const int w0 = blockIdx.x * HO_RUN, h = blockIdx.y, b = blockIdx.z, tid = threadIdx.x;
    const int nw = min(HO_RUN, Wb - w0), nq = nw / 4;  // Wb % 4 == 0: whole quads
    const size_t plane = (size_t)Hb * Wb;
    const float *sb = s + (size_t)b * P * plane + (size_t)h * Wb + w0;
    for (int e = tid; e < P * (HO_RUN / 4); e += HO_T) {
        const int c = e / (HO_RUN / 4), k4 = e % (HO_RUN / 4);
        if (k4 < nq) {
            const float4 v = *(const float4 *)(sb + (size_t)c * plane + 4 * k4);
            const float bc = bias[c];
            float *t = tile + 4 * k4 * (P + 1) + c;
            t[0] = v.x + bc;
            t[P + 1] = v.y + bc;
            t[2 * (P + 1)] = v.z + bc;
            t[3 * (P + 1)] = v.w + bc;
        }
    }
    __syncthreads();
    const int cq = cp / 4;
    float4 *xr = reinterpret_cast<float4 *>(x + (((size_t)b * Hb + h) * Wb + w0) * cp);
    const float *pr = pos + (size_t)h * Wb + w0;
    for (int e = tid; e < nw * cq; e += HO_T) {
        const int k = e / cq, c = 4 * (e - k * cq);
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int cc = c + u;
            v[u] = cc < P ? tile[k * (P + 1) + cc] : cc < P + 2 ? pr[(size_t)(cc - P) * plane + k] : 0.0f;
        }
        xr[e] = make_float4(v[0], v[1], v[2], v[3]);
    }
}

// BIAS: also the block's per-channel sums of its nw cells (fp32, in cell order) into bpart[block][P], which
// k_head_bias_fin adds in double -- the BEV projection bias's gradient without a separate pass over gs
template <bool BIAS = false>
__global__ __launch_bounds__(HO_T) void k_head_operand_bwd_v4(const float *__restrict__ gx, int P, int Hb, int Wb,
                                                              int cp, float *__restrict__ gs,
                                                              float *__restrict__ bpart = nullptr) {
    extern __shared__ float tile[];  // [HO_RUN][P + 1]
    const int w0 = blockIdx.x * HO_RUN, h = blockIdx.y, b = blockIdx.z, tid = threadIdx.x;
    const int nw = min(HO_RUN, Wb - w0), nq = nw / 4, cq = cp / 4, pq = (P + 3) / 4;
    const size_t plane = (size_t)Hb * Wb;
    const float4 *gr = reinterpret_cast<const float4 *>(gx + (((size_t)b * Hb + h) * Wb + w0) * cp);
    for (int e = tid; e < nw * pq; e += HO_T) {
        const int k = e / pq, c = 4 * (e - k * pq);
        const float4 v = gr[(size_t)k * cq + c / 4];
        const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (c + u < P) tile[k * (P + 1) + c + u] = vv[u];
    }
    __syncthreads();
    float *gb = gs + (size_t)b * P * plane + (size_t)h * Wb + w0;
    for (int e = tid; e < P * (HO_RUN / 4); e += HO_T) {
        const int c = e / (HO_RUN / 4), k4 = e % (HO_RUN / 4);
        if (k4 < nq) {
            const float *t = tile + 4 * k4 * (P + 1) + c;
            *(float4 *)(gb + (size_t)c * plane + 4 * k4) = make_float4(t[0], t[P + 1], t[2 * (P + 1)], t[3 * (P + 1)]);
        }
    }
    if constexpr (BIAS) {
        const size_t blk = ((size_t)b * Hb + h) * gridDim.x + blockIdx.x;
        for (int c = tid; c < P; c += HO_T) {
            float acc = 0.0f;
            for (int k = 0; k < nw; ++k) acc += tile[k * (P + 1) + c];
            bpart[blk * P + c] = acc;
        }
    }
}

// gbias[c] = sum over the blocks' partials (double, fixed order: deterministic); one workgroup per channel
__global__ __launch_bounds__(256) void k_head_bias_fin(const float *__restrict__ bpart, int64_t nblk, int P,
                                                       float *__restrict__ gbias) {
    __shared__ double red[256];
    const int c = blockIdx.x, tid = threadIdx.x;
    double acc = 0.0;
    for (int64_t i = tid; i < nblk; i += 256) acc += (double)bpart[i * P + c];
    red[tid] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) red[tid] += red[tid + o];
        __syncthreads();
    }
    if (tid == 0) gbias[c] = (float)red[0];
}

}  // namespace

extern "C" {

int64_t bev_groupnorm_workspace_bytes(int N, int64_t P, int C, int G) {
    if (!gn_shape_ok(N, P, C, G)) return -1;
    const int64_t nb = nblocks(P);
    return (int64_t)N * nb * (G + C) * 2 * (int64_t)sizeof(double) + (int64_t)N * G * 2 * (int64_t)sizeof(float);
}

int bev_groupnorm_fwd_f32(const float *x, int N, int64_t P, int C, int G, float eps, const float *gamma,
                          const float *beta, float *mean, float *rstd, float *scale, float *shift, void *workspace,
                          void *stream) {
    if (!x || !gamma || !beta || !mean || !rstd || !scale || !shift || !workspace || !gn_shape_ok(N, P, C, G))
        return BEV_ERR_ARGS;
    hipStream_t st = (hipStream_t)stream;
    const int nb = nblocks(P);
    double *part = (double *)workspace;
    hipLaunchKernelGGL(k_gn_partial, dim3(nb, N), dim3(GN_T), 0, st, x, P, C, G, part);
    hipLaunchKernelGGL(k_gn_finalize, dim3(N * G), dim3(GN_T), 0, st, part, nb, P, C, G, eps, gamma, beta, mean, rstd,
                       scale, shift);
    return (int)hipGetLastError();
}

int bev_groupnorm_apply_ex_f32(const float *x, int N, int64_t P, int C, const float *scale, const float *shift,
                               int relu, void *y, int y_half, void *stream) {
    if (!x || !scale || !shift || !y || N <= 0 || N > 65535 || P <= 0 || C <= 0 || C % 4 != 0 || GN_T % (C / 4) != 0)
        return BEV_ERR_ARGS;
    const dim3 grid((unsigned)((P + GN_APPLY_PIX - 1) / GN_APPLY_PIX), N);
    if (y_half)
        hipLaunchKernelGGL(k_gn_apply<_Float16>, grid, dim3(GN_T), 0, (hipStream_t)stream, x, P, C, scale, shift, relu,
                           (_Float16 *)y);
    else
        hipLaunchKernelGGL(k_gn_apply<float>, grid, dim3(GN_T), 0, (hipStream_t)stream, x, P, C, scale, shift, relu,
                           (float *)y);
    return (int)hipGetLastError();
}

int bev_groupnorm_apply_f32(const float *x, int N, int64_t P, int C, const float *scale, const float *shift, int relu,
                            float *y, void *stream) {
    return bev_groupnorm_apply_ex_f32(x, N, P, C, scale, shift, relu, y, 0, stream);
}

int bev_groupnorm_bwd_ex_f32(const float *x, const float *dy, int N, int64_t P, int C, int G, const float *mean,
                             const float *rstd, const float *gamma, const float *scale, const float *shift, int relu,
                             void *dx, int dx_half, float *dgamma, float *dbeta, void *workspace, void *stream) {
    if (!x || !dy || !mean || !rstd || !gamma || !scale || !shift || !dx || !dgamma || !dbeta || !workspace ||
        !gn_shape_ok(N, P, C, G))
        return BEV_ERR_ARGS;
    hipStream_t st = (hipStream_t)stream;
    const int nb = nblocks(P);
    double *part = (double *)workspace;                     // [N][nb][G][2]
    double *cpart = part + (size_t)N * nb * G * 2;          // [N][nb][C][2]
    // coef [N][G][2] floats after cpart (bev_groupnorm_workspace_bytes sizes all three)
    hipLaunchKernelGGL(k_gn_bwd_partial, dim3(nb, N), dim3(GN_T), 0, st, x, dy, P, C, G, mean, rstd, gamma, scale,
                       shift, relu, part, cpart);
    float *coef = (float *)(cpart + (size_t)N * nb * C * 2);
    hipLaunchKernelGGL(k_gn_bwd_fin_chan, dim3((C + GF_C - 1) / GF_C), dim3(GF_C * GF_P), 0, st, cpart, N, nb, C,
                       dgamma, dbeta);
    hipLaunchKernelGGL(k_gn_bwd_fin_group, dim3(N * G), dim3(GN_T), 0, st, part, nb, P, C, G, coef);
    const dim3 grid((unsigned)((P + GN_APPLY_PIX - 1) / GN_APPLY_PIX), N);
    if (dx_half)
        hipLaunchKernelGGL(k_gn_bwd_apply<_Float16>, grid, dim3(GN_T), 0, st, x, dy, P, C, G, mean, rstd, gamma, scale,
                           shift, relu, coef, (_Float16 *)dx);
    else
        hipLaunchKernelGGL(k_gn_bwd_apply<float>, grid, dim3(GN_T), 0, st, x, dy, P, C, G, mean, rstd, gamma, scale,
                           shift, relu, coef, (float *)dx);
    return (int)hipGetLastError();
}

int bev_groupnorm_bwd_f32(const float *x, const float *dy, int N, int64_t P, int C, int G, const float *mean,
                          const float *rstd, const float *gamma, const float *scale, const float *shift, int relu,
                          float *dx, float *dgamma, float *dbeta, void *workspace, void *stream) {
    return bev_groupnorm_bwd_ex_f32(x, dy, N, P, C, G, mean, rstd, gamma, scale, shift, relu, dx, 0, dgamma, dbeta,
                                    workspace, stream);
}

int bev_head_operand_f32(const float *s, const float *bias, const float *pos, int B, int P, int Hb, int Wb, int cp,
                         float *x, void *stream) {
    if (!s || !bias || !pos || !x || B < 0 || P <= 0 || Hb < 0 || Wb < 0 || cp < P + 2 || B > 65535 || Hb > 65535 ||
        P > 512)
        return BEV_ERR_ARGS;
    if (B == 0 || Hb == 0 || Wb == 0) return 0;
    const size_t lds = (size_t)HO_RUN * (P + 1) * sizeof(float);
    const dim3 grid((Wb + HO_RUN - 1) / HO_RUN, Hb, B);
    if (Wb % 4 == 0 && cp % 4 == 0 && (((uintptr_t)s | (uintptr_t)pos | (uintptr_t)x) & 15) == 0)
        hipLaunchKernelGGL(k_head_operand_v4, grid, dim3(HO_T), lds, (hipStream_t)stream, s, bias, pos, P, Hb, Wb, cp, x);
    else
        hipLaunchKernelGGL(k_head_operand, grid, dim3(HO_T), lds, (hipStream_t)stream, s, bias, pos, P, Hb, Wb, cp, x);
    return (int)hipGetLastError();
}

int64_t bev_head_operand_bwd_bias_partials(int B, int P, int Hb, int Wb) {
    if (B <= 0 || P <= 0 || Hb <= 0 || Wb <= 0) return BEV_ERR_ARGS;
    return (int64_t)B * Hb * ((Wb + HO_RUN - 1) / HO_RUN) * P;
}

int bev_head_operand_bwd_bias_f32(const float *gx, int B, int P, int Hb, int Wb, int cp, float *gs, float *gbias,
                                  float *partials, void *stream) {
    if (!gx || !gs || !gbias || !partials || B <= 0 || P <= 0 || Hb <= 0 || Wb <= 0 || cp < P || B > 65535 ||
        Hb > 65535 || P > 512)
        return BEV_ERR_ARGS;
    if (Wb % 4 != 0 || cp % 4 != 0 || (((uintptr_t)gx | (uintptr_t)gs) & 15) != 0) return BEV_ERR_ARGS;  // 16-B form
    const size_t lds = (size_t)HO_RUN * (P + 1) * sizeof(float);
    const dim3 grid((Wb + HO_RUN - 1) / HO_RUN, Hb, B);
    hipLaunchKernelGGL(k_head_operand_bwd_v4<true>, grid, dim3(HO_T), lds, (hipStream_t)stream, gx, P, Hb, Wb, cp, gs,
                       partials);
    hipLaunchKernelGGL(k_head_bias_fin, dim3(P), dim3(256), 0, (hipStream_t)stream, partials,
                       (int64_t)B * Hb * grid.x, P, gbias);
    return (int)hipGetLastError();
}

int bev_head_operand_bwd_f32(const float *gx, int B, int P, int Hb, int Wb, int cp, float *gs, void *stream) {
    if (!gx || !gs || B < 0 || P <= 0 || Hb < 0 || Wb < 0 || cp < P || B > 65535 || Hb > 65535 || P > 512)
        return BEV_ERR_ARGS;
    if (B == 0 || Hb == 0 || Wb == 0) return 0;
    const size_t lds = (size_t)HO_RUN * (P + 1) * sizeof(float);
    const dim3 grid((Wb + HO_RUN - 1) / HO_RUN, Hb, B);
    if (Wb % 4 == 0 && cp % 4 == 0 && (((uintptr_t)gx | (uintptr_t)gs) & 15) == 0)
        hipLaunchKernelGGL(k_head_operand_bwd_v4<false>, grid, dim3(HO_T), lds, (hipStream_t)stream, gx, P, Hb, Wb, cp,
                           gs, nullptr);
    else
        hipLaunchKernelGGL(k_head_operand_bwd, grid, dim3(HO_T), lds, (hipStream_t)stream, gx, P, Hb, Wb, cp, gs);
    return (int)hipGetLastError();
}

}  // extern "C"

// ---- CenterNet focal heatmap loss (model_wrapper.py:235-247) -------------------------------------------------------
// p = clamp(sigmoid(x), 1e-4, 1 - 1e-4); pos = log p (1 - p)^a where gt == 1, neg = log(1 - p) p^a (1 - gt)^b where
// gt < 1; loss = -(sum pos + sum neg) / max(#(gt == 1), 1).  Forward: per-block partial sums in double, one finalize
// block (loss, and 1 / max(npos, 1) kept on the device for the backward); backward: dx = -g inv d(pos + neg)/dp dp/dx
// with torch's clamp rule (gradient where 1e-4 <= sigmoid(x) <= 1 - 1e-4) and sigmoid'(x) = s (1 - s).  Two launches
// forward and one backward instead of torch's ~60 elementwise / reduction launches for the same loss (a training step
// runs them at the host's launch pace, between the head's forward and its backward).
namespace {
constexpr int FL_T = 256, FL_MAXB = 1024;

__device__ __forceinline__ float fl_p(float x, float &s) {
    s = 1.0f / (1.0f + expf(-x));
    const float lo = (float)1e-4, hi = (float)(1.0 - 1e-4);
    return fminf(fmaxf(s, lo), hi);
}

__device__ __forceinline__ double fl_block_sum(double v, double *red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(FL_T) void k_focal_partial(const float *__restrict__ x, const float *__restrict__ gt,
                                                        int64_t n, float alpha, float beta, double *__restrict__ part) {
    __shared__ double red[4];
    double sp = 0.0, sn = 0.0, np = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * FL_T + threadIdx.x; i < n; i += (int64_t)gridDim.x * FL_T) {
        float s;
        const float p = fl_p(x[i], s), g = gt[i];
        if (g == 1.0f) {
            sp += (double)(logf(p) * powf(1.0f - p, alpha));
            np += 1.0;
        }
        if (g < 1.0f) sn += (double)(logf(1.0f - p) * powf(p, alpha) * powf(1.0f - g, beta));
    }
    sp = fl_block_sum(sp, red);
    sn = fl_block_sum(sn, red);
    np = fl_block_sum(np, red);
    if (threadIdx.x == 0) {
        part[3 * blockIdx.x] = sp;
        part[3 * blockIdx.x + 1] = sn;
        part[3 * blockIdx.x + 2] = np;
    }
}

__global__ __launch_bounds__(FL_T) void k_focal_finalize(const double *__restrict__ part, int nb, float *__restrict__ loss,
                                                         float *__restrict__ inv) {
    __shared__ double red[4];
    double sp = 0.0, sn = 0.0, np = 0.0;
    for (int b = threadIdx.x; b < nb; b += FL_T) {
        sp += part[3 * b];
        sn += part[3 * b + 1];
        np += part[3 * b + 2];
    }
    sp = fl_block_sum(sp, red);
    sn = fl_block_sum(sn, red);
    np = fl_block_sum(np, red);
    if (threadIdx.x == 0) {
        const double den = np > 1.0 ? np : 1.0;
        loss[0] = (float)(-(sp + sn) / den);
        inv[0] = (float)(1.0 / den);
    }
}

__global__ __launch_bounds__(FL_T) void k_focal_bwd(const float *__restrict__ x, const float *__restrict__ gt, int64_t n,
                                                    float alpha, float beta, const float *__restrict__ gout,
                                                    const float *__restrict__ inv, float *__restrict__ dx) {
    const float scale = -gout[0] * inv[0];
    const float lo = (float)1e-4, hi = (float)(1.0 - 1e-4);
    for (int64_t i = (int64_t)blockIdx.x * FL_T + threadIdx.x; i < n; i += (int64_t)gridDim.x * FL_T) {
        float s;
        const float p = fl_p(x[i], s), g = gt[i];
        float d = 0.0f;
        if (g == 1.0f) d += powf(1.0f - p, alpha) / p - alpha * logf(p) * powf(1.0f - p, alpha - 1.0f);
        if (g < 1.0f) {
            const float w = powf(1.0f - g, beta);
            d += -powf(p, alpha) * w / (1.0f - p) + alpha * logf(1.0f - p) * powf(p, alpha - 1.0f) * w;
        }
        const float dp = (s >= lo && s <= hi) ? s * (1.0f - s) : 0.0f;
        dx[i] = scale * d * dp;
    }
}

inline int fl_blocks(int64_t n) {
    const int64_t b = (n + FL_T - 1) / FL_T;
    return (int)(b < FL_MAXB ? (b > 0 ? b : 1) : FL_MAXB);
}
}  // namespace

extern "C" {

int64_t bev_focal_loss_workspace_bytes(int64_t n) {
    if (n < 0) return BEV_ERR_ARGS;
    return (int64_t)fl_blocks(n) * 3 * (int64_t)sizeof(double);
}

int bev_focal_loss_fwd_f32(const float *logits, const float *gt, int64_t n, float alpha, float beta, float *loss,
                           float *inv_norm, void *workspace, int64_t workspace_bytes, void *stream) {
    if (!logits || !gt || !loss || !inv_norm || !workspace || n < 0 ||
        workspace_bytes < bev_focal_loss_workspace_bytes(n))
        return BEV_ERR_ARGS;
    const int nb = fl_blocks(n);
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_focal_partial, dim3(nb), dim3(FL_T), 0, st, logits, gt, n, alpha, beta, (double *)workspace);
    hipLaunchKernelGGL(k_focal_finalize, dim3(1), dim3(FL_T), 0, st, (const double *)workspace, nb, loss, inv_norm);
    return (int)hipGetLastError();
}

int bev_focal_loss_bwd_f32(const float *logits, const float *gt, int64_t n, float alpha, float beta,
                           const float *grad_loss, const float *inv_norm, float *dlogits, void *stream) {
    if (!logits || !gt || !grad_loss || !inv_norm || !dlogits || n < 0) return BEV_ERR_ARGS;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_focal_bwd, dim3(fl_blocks(n)), dim3(FL_T), 0, (hipStream_t)stream, logits, gt, n, alpha, beta,
                       grad_loss, inv_norm, dlogits);
    return (int)hipGetLastError();
}

}  // extern "C"

// ---- CenterNet L1 offset / log-size losses (model_wrapper.py:109-116) ---------------------------------------------
// off = sum_{b,k,c} |offset[b][c][idx[b][k]] - off_t[b][k][c]| m[b][k] / n, size likewise on size_raw / size_t,
// n = sum m + 1e-4 (fp32 terms, double sums): one workgroup over the B x M slots.  Backward: the gathers' gradients
// scattered back, g sign(x) m / n (torch's abs rule, sign(0) = 0), added per cell (two objects may share one).
namespace {
__global__ __launch_bounds__(FL_T) void k_l1_fwd(const float *__restrict__ off, const float *__restrict__ sz, int64_t HW,
                                                 const int64_t *__restrict__ idx, const float *__restrict__ m,
                                                 const float *__restrict__ offt, const float *__restrict__ szt, int B,
                                                 int M, int ldi, float *__restrict__ out) {
    __shared__ double red[4];
    double so = 0.0, ss = 0.0, sm = 0.0;
    for (int e = threadIdx.x; e < B * M; e += FL_T) {
        const int b = e / M, k = e - b * M;
        const float mk = m[(int64_t)b * ldi + k];
        const int64_t i = idx[(int64_t)b * ldi + k];
        sm += (double)mk;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int64_t t = ((int64_t)b * ldi + k) * 2 + c;
            so += (double)fabsf((off[((int64_t)b * 2 + c) * HW + i] - offt[t]) * mk);
            ss += (double)fabsf((sz[((int64_t)b * 2 + c) * HW + i] - szt[t]) * mk);
        }
    }
    so = fl_block_sum(so, red);
    ss = fl_block_sum(ss, red);
    sm = fl_block_sum(sm, red);
    if (threadIdx.x == 0) {
        const float n = (float)sm + 1e-4f;  // torch: m.sum() (fp32) + 1e-4
        out[0] = (float)(so / (double)n);
        out[1] = (float)(ss / (double)n);
        out[2] = 1.0f / n;
    }
}

__global__ __launch_bounds__(FL_T) void k_l1_bwd(const float *__restrict__ off, const float *__restrict__ sz, int64_t HW,
                                                 const int64_t *__restrict__ idx, const float *__restrict__ m,
                                                 const float *__restrict__ offt, const float *__restrict__ szt, int B,
                                                 int M, int ldi, const float *__restrict__ gl,
                                                 const float *__restrict__ fwd, float *__restrict__ doff,
                                                 float *__restrict__ dsz) {
    const float go = gl[0] * fwd[2], gs = gl[1] * fwd[2];
    for (int e = blockIdx.x * FL_T + threadIdx.x; e < B * M * 2; e += gridDim.x * FL_T) {
        const int c = e & 1, bk = e >> 1, b = bk / M, k = bk - b * M;
        const float mk = m[(int64_t)b * ldi + k];
        if (mk == 0.0f) continue;
        const int64_t i = idx[(int64_t)b * ldi + k];
        const int64_t t = ((int64_t)b * ldi + k) * 2 + c, o = ((int64_t)b * 2 + c) * HW + i;
        const float xo = (off[o] - offt[t]) * mk, xs = (sz[o] - szt[t]) * mk;
        const float so = xo > 0.0f ? 1.0f : (xo < 0.0f ? -1.0f : 0.0f), ss = xs > 0.0f ? 1.0f : (xs < 0.0f ? -1.0f : 0.0f);
        atomicAdd(doff + o, go * so * mk);
        atomicAdd(dsz + o, gs * ss * mk);
    }
}
}  // namespace

extern "C" {

int bev_l1_losses_fwd_f32(const float *offset, const float *size, int B, int64_t HW, const int64_t *indices,
                          const float *mask, const float *off_t, const float *size_t_, int M, int ld, float *out,
                          void *stream) {
    if (!offset || !size || !indices || !mask || !off_t || !size_t_ || !out || B < 0 || M < 0 || ld < M || HW <= 0)
        return BEV_ERR_ARGS;
    hipLaunchKernelGGL(k_l1_fwd, dim3(1), dim3(FL_T), 0, (hipStream_t)stream, offset, size, HW, indices, mask, off_t,
                       size_t_, B, M, ld, out);
    return (int)hipGetLastError();
}

int bev_l1_losses_bwd_f32(const float *offset, const float *size, int B, int64_t HW, const int64_t *indices,
                          const float *mask, const float *off_t, const float *size_t_, int M, int ld,
                          const float *grad_losses, const float *fwd_out, float *d_offset, float *d_size,
                          void *stream) {
    if (!offset || !size || !indices || !mask || !off_t || !size_t_ || !grad_losses || !fwd_out || !d_offset ||
        !d_size || B < 0 || M < 0 || ld < M || HW <= 0)
        return BEV_ERR_ARGS;
    const int n = B * M * 2;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_l1_bwd, dim3((n + FL_T - 1) / FL_T), dim3(FL_T), 0, (hipStream_t)stream, offset, size, HW,
                       indices, mask, off_t, size_t_, B, M, ld, grad_losses, fwd_out, d_offset, d_size);
    return (int)hipGetLastError();
}

}  // extern "C"

// ---- CenterNet gaussian radius (model_wrapper.py:205-233, BEVNet._gaussian_radius_tensor) --------------------------
// The torch float32 op sequence replayed op by op in one launch instead of ~45 (the library builds with
// -ffp-contract=off: no fused multiply-adds): a tensor times a Python scalar is x * (float)s, a tensor over a Python
// scalar x * (1.0f / (float)s) (torch's CUDA division by a CPU scalar; the caller passes that reciprocal), tensor over
// tensor a true division, x ** 2 a product, clamp / min propagate NaN like torch's.
namespace {
__device__ __forceinline__ float gr_clamp_min(float x, float lo) { return x < lo ? lo : x; }  // NaN stays NaN
__device__ __forceinline__ float gr_min(float a, float b) { return a != a ? a : (b != b ? b : (b < a ? b : a)); }
__device__ __forceinline__ float gr_root(float a, float b, float c) {
    const float t = gr_clamp_min(b * b - (a * 4.0f) * c, 0.0f);  // b ** 2 - 4 * a * c, clamp(min=0)
    return b + sqrtf(t);
}
__global__ void k_gauss_radius(const float *__restrict__ wc, const float *__restrict__ hc, int n, float f_1mov,
                               float rcp_1pov, float f_4ov, float f_m2ov, float f_ovm1, int ov_zero, float minr,
                               int64_t *__restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float w = gr_clamp_min(wc[i], 1.0f), h = gr_clamp_min(hc[i], 1.0f);
    const float r1 = gr_root(1.0f, h + w, ((w * h) * f_1mov) * rcp_1pov) * 0.5f;
    const float a2 = 4.0f;
    const float r2 = gr_root(a2, (h + w) * 2.0f, (w * f_1mov) * h) / (a2 * 2.0f);
    float r = gr_min(r1, r2);
    if (!ov_zero) {
        const float a3 = f_4ov;
        const float r3 = gr_root(a3, (h + w) * f_m2ov, (w * f_ovm1) * h) / (a3 * 2.0f);
        r = gr_min(r, r3);
    }
    out[i] = (int64_t)floorf(gr_clamp_min(r, minr));
}
}  // namespace

extern "C" {
int bev_gaussian_radius_f32(const float *width_cells, const float *height_cells, int n, float f_1mov,
                            float rcp_1pov, float f_4ov, float f_m2ov, float f_ovm1, int ov_zero, float min_radius,
                            int64_t *radius, void *stream) {
    if (!width_cells || !height_cells || !radius || n < 0) return BEV_ERR_ARGS;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_gauss_radius, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, width_cells,
                       height_cells, n, f_1mov, rcp_1pov, f_4ov, f_m2ov, f_ovm1, ov_zero, min_radius, radius);
    return (int)hipGetLastError();
}
}  // extern "C"
