// bev_effnet.hip -- the non-GEMM layers of the EfficientNet trunk for gfx950.
//
// The reference builds its per-camera backbone with timm (cnn_encoder.py:26,
// `features_only=True`, feature index out_index=2 -> stride 8); for
// efficientnet_b3 that trunk is conv_stem -> blocks.0 (depthwise-separable)
// -> blocks.1, blocks.2 (inverted residuals, SiLU, squeeze-excitation).  The
// 1x1 / stem convolutions run on the MFMA implicit GEMM (bev_conv.hip, act =
// SiLU); this file holds what is not a GEMM:
//
//   k_dwconv      depthwise KxK conv (BN folded) + SiLU, NHWC, float4 per
//                 thread over channels; the thread's K*K weight quads stay in
//                 VGPRs; the per-workgroup channel sums of the OUTPUT (the
//                 squeeze of the SE block) are reduced in LDS and written as
//                 deterministic partials [N][nb][C] (no atomics).
//   k_se_gate     per image: mean = sum(partials) / (Ho*Wo), conv_reduce +
//                 SiLU, conv_expand + sigmoid -> gate [N][C].
//   k_chan_scale  x[n, p, c] *= gate[n, c] in place (the SE excitation).
//   k_dw_wgrad    training: depthwise weight gradient dW[t][c] = sum_{n,p} dz[n,p,c] x[n, tap t of p, c], the
//                 k_dwconv thread layout with K*K float4 accumulators per thread, reduced over the workgroup's
//                 pixel lanes in LDS and added to dW with float atomics (one per workgroup, tap and channel).
//
// All three are HBM-bound streaming kernels (bytes per output element: the
// input taps come from L1/L2 after the first touch, so ~4 B in + 4 B out).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bev_mi355x.h"
#include "bev_act.h"

namespace {

constexpr int DW_NT = 256;      // threads per workgroup
constexpr int DW_STEPS = 8;     // pixel steps per thread: output pixels per workgroup = DW_STEPS * (pixels per step)

// Channel quads per workgroup (larger C is split over blockIdx.z) and pixels per workgroup.
inline int dw_ch4(int C) { return C / 4 <= DW_NT ? C / 4 : DW_NT / 2; }
inline int dw_ppb(int C) { return DW_STEPS * (DW_NT / dw_ch4(C)); }

__device__ __forceinline__ float act_f(float t, int act) {
    if (act == 1) return t > 0.0f ? t : 0.0f;
    if (act == 2) return silu_hw(t);  // torch SiLU x / (1 + exp(-x)), hardware exp2 / rcp (bev_act.h)
    return t;
}

template <int K>
__global__ __launch_bounds__(DW_NT) void k_dwconv(const float *__restrict__ x, int H, int W, int C,
                                                  const float *__restrict__ wt, const float *__restrict__ bias,
                                                  int stride, int pad, int act, float *__restrict__ y, int Ho, int Wo,
                                                  float *__restrict__ psum, int nb, int ppb) {
    __shared__ float4 red[DW_NT];
    const int C4 = C >> 2;
    const int CH4 = C4 <= DW_NT ? C4 : DW_NT / 2;  // channel quads per workgroup (blockIdx.z chunks)
    const int PB = DW_NT / CH4;                     // pixels per step
    const int tid = threadIdx.x;
    const int pl = tid / CH4, c4 = blockIdx.z * CH4 + (tid - pl * CH4);
    const bool active = pl < PB && c4 < C4;
    const int n = blockIdx.y, blk = blockIdx.x;
    const int64_t HWo = (int64_t)Ho * Wo;
    const int64_t p0 = (int64_t)blk * ppb, p1 = min(p0 + ppb, HWo);
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (active) {
        float4 w[K * K];
#pragma unroll
        for (int t = 0; t < K * K; ++t) w[t] = *(const float4 *)(wt + (int64_t)t * C + c4 * 4);
        const float4 b = *(const float4 *)(bias + c4 * 4);
        const float *xn = x + (int64_t)n * H * W * C + c4 * 4;
        float *yn = y + (int64_t)n * HWo * C + c4 * 4;
        for (int64_t p = p0 + pl; p < p1; p += PB) {
            const int oy = (int)(p / Wo), ox = (int)(p - (int64_t)oy * Wo);
            const int iy0 = oy * stride - pad, ix0 = ox * stride - pad;
            float4 acc = b;
#pragma unroll
            for (int ky = 0; ky < K; ++ky) {
                const int iy = iy0 + ky;
                if (iy < 0 || iy >= H) continue;
#pragma unroll
                for (int kx = 0; kx < K; ++kx) {
                    const int ix = ix0 + kx;
                    if (ix < 0 || ix >= W) continue;
                    const float4 v = *(const float4 *)(xn + ((int64_t)iy * W + ix) * C);
                    const float4 ww = w[ky * K + kx];
                    acc.x = __builtin_fmaf(v.x, ww.x, acc.x);
                    acc.y = __builtin_fmaf(v.y, ww.y, acc.y);
                    acc.z = __builtin_fmaf(v.z, ww.z, acc.z);
                    acc.w = __builtin_fmaf(v.w, ww.w, acc.w);
                }
            }
            acc.x = act_f(acc.x, act);
            acc.y = act_f(acc.y, act);
            acc.z = act_f(acc.z, act);
            acc.w = act_f(acc.w, act);
            *(float4 *)(yn + p * C) = acc;
            s.x += acc.x;
            s.y += acc.y;
            s.z += acc.z;
            s.w += acc.w;
        }
    }
    if (psum == nullptr) return;
    red[tid] = s;
    __syncthreads();
    if (pl == 0 && c4 < C4) {  // fixed order over the step lanes: deterministic partial
        for (int q = 1; q < PB; ++q) {
            const float4 t = red[q * CH4 + (tid - pl * CH4)];
            s.x += t.x;
            s.y += t.y;
            s.z += t.z;
            s.w += t.w;
        }
        *(float4 *)(psum + ((int64_t)n * nb + blk) * C + c4 * 4) = s;
    }
}


// Row-run depthwise K x K for narrow channel counts (C / 4 <= 64 quads, where the LDS tile loses: B3's 540 x 960 C 24 /
// C 40 and 270 x 480 C 144 stride-2 layers).  A thread owns one channel quad of R consecutive outputs of one row;
// for each kernel row it loads the (R - 1) * S + K input pixels the run needs once into registers and applies them
// to all R outputs, so every input quad is fetched once per kernel row and run instead of K times per output (the
// per-pixel kernel's K * K tap loads per output were bound by the L1 / address rate, 0.28 of HBM on those layers).
// The C / 4 lanes of a run read each pixel as one contiguous segment.  Per output the taps are applied in
// k_dwconv's order (ky-major, kx-minor; out-of-range rows skipped, out-of-range columns read as 0, so y matches
// k_dwconv up to the sign of an exact zero); SE partials per workgroup in a fixed order.
// BEV_TUNE_DW_RUN: 0 keeps these layers on k_dwconv; 1 row runs; 2 row runs with every kernel row's loads issued up
// front for 3 x 3 (more VGPRs, fewer exposed latencies); 3 (default) = 2 also for the widths the LDS tile took.
// r03i (EfficientNet-B3 bench, profiles/r03i_dw_run_ab.txt): per-pixel -> runs -> up front: 540 x 960 C 24
// 623 -> 421 -> 401 us, C 40 1031 -> 701 -> 671, 270 x 480 C 144 s2 1271 -> 1039 -> 980 (120.1 -> 126.8 frames/s);
// LDS tile -> runs: 270 x 480 C 192 k3 819 -> 706, 135 x 240 C 288 k5 645 -> 439, C 192 k5 s2 1105 -> 522 us
// (127.1 -> 136.0 frames/s).
int g_dw_run = 3;
template <int S> constexpr int dw_run_len() { return S == 1 ? 8 : 4; }
inline int dw_run_ch4(int C) {
    const int C4 = C / 4;
    for (int d = 1; d <= 16; ++d)
        if (C4 % d == 0 && C4 / d <= 64) return C4 / d;
    return 0;
}

template <int K, int S, bool UP>
__global__ __launch_bounds__(DW_NT) void k_dwconv_r(const float *__restrict__ x, int H, int W, int C,
                                                    const float *__restrict__ wt, const float *__restrict__ bias,
                                                    int pad, int act, float *__restrict__ y, int Ho, int Wo,
                                                    float *__restrict__ psum, int nb, int CH4) {
    constexpr int R = dw_run_len<S>(), IC = (R - 1) * S + K;
    __shared__ float4 red[DW_NT];
    const int PB = DW_NT / CH4;  // runs per workgroup; CH4 channel quads per workgroup (blockIdx.z chunks)
    const int tid = threadIdx.x, pl = tid / CH4, q = blockIdx.z * CH4 + (tid - pl * CH4);
    const int n = blockIdx.y, blk = blockIdx.x;
    const int rpr = (Wo + R - 1) / R;
    const int64_t ri = (int64_t)blk * PB + pl;
    const bool active = pl < PB && ri < (int64_t)Ho * rpr;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (active) {
        const int oy = (int)(ri / rpr), ox0 = (int)(ri - (int64_t)oy * rpr) * R;
        const int ix0 = ox0 * S - pad;
        float4 w[K * K];
#pragma unroll
        for (int t = 0; t < K * K; ++t) w[t] = *(const float4 *)(wt + (int64_t)t * C + q * 4);
        const float4 b = *(const float4 *)(bias + q * 4);
        float4 acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = b;
        const float *xn = x + (int64_t)n * H * W * C + q * 4;
        float4 vu[UP ? K : 1][IC];
        if (UP) {  // every row's loads in flight at once (out-of-range rows read as 0)
#pragma unroll
            for (int ky = 0; ky < K; ++ky) {
                const int iy = oy * S - pad + ky;
                const bool rin = iy >= 0 && iy < H;
                const float *xr = xn + (int64_t)(rin ? iy : 0) * W * C;
#pragma unroll
                for (int c = 0; c < IC; ++c) {
                    const int ix = ix0 + c;
                    vu[UP ? ky : 0][c] = (rin && ix >= 0 && ix < W) ? *(const float4 *)(xr + (int64_t)ix * C)
                                                                    : make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
        }
#pragma unroll
        for (int ky = 0; ky < K; ++ky) {
            const int iy = oy * S - pad + ky;
            float4 v[IC];
            if (UP) {
#pragma unroll
                for (int c = 0; c < IC; ++c) v[c] = vu[UP ? ky : 0][c];
            } else {
                if (iy < 0 || iy >= H) continue;
                const float *xr = xn + (int64_t)iy * W * C;
#pragma unroll
                for (int c = 0; c < IC; ++c) {
                    const int ix = ix0 + c;
                    v[c] = (ix >= 0 && ix < W) ? *(const float4 *)(xr + (int64_t)ix * C) : make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
#pragma unroll
                for (int kx = 0; kx < K; ++kx) {
                    const float4 vv = v[r * S + kx], ww = w[ky * K + kx];
                    acc[r].x = __builtin_fmaf(vv.x, ww.x, acc[r].x);
                    acc[r].y = __builtin_fmaf(vv.y, ww.y, acc[r].y);
                    acc[r].z = __builtin_fmaf(vv.z, ww.z, acc[r].z);
                    acc[r].w = __builtin_fmaf(vv.w, ww.w, acc[r].w);
                }
            }
        }
        float *yr = y + (((int64_t)n * Ho + oy) * Wo + ox0) * C + q * 4;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (ox0 + r >= Wo) break;
            float4 o = acc[r];
            o.x = act_f(o.x, act);
            o.y = act_f(o.y, act);
            o.z = act_f(o.z, act);
            o.w = act_f(o.w, act);
            *(float4 *)(yr + (int64_t)r * C) = o;
            s.x += o.x;
            s.y += o.y;
            s.z += o.z;
            s.w += o.w;
        }
    }
    if (psum == nullptr) return;
    red[tid] = s;
    __syncthreads();
    if (pl == 0) {  // fixed order over the runs: deterministic partial
        for (int l = 1; l < PB; ++l) {
            const float4 t = red[l * CH4 + (tid - pl * CH4)];
            s.x += t.x;
            s.y += t.y;
            s.z += t.z;
            s.w += t.w;
        }
        *(float4 *)(psum + ((int64_t)n * nb + blk) * C + q * 4) = s;
    }
}

// LDS-tiled depthwise conv: a workgroup owns an 8-row output-pixel tile x DQ channel quads (DQ = 8: 32 channels =
// one 128-B line of every pixel, 8 columns; DQ = 4: 8 columns; DQ = 2: 16 columns).  The tile's input patch is
// staged in LDS once (pixel stride DQ + 1 quads: conflict-free ds_read_b128 for stride 1 and 2), so the K*K taps
// of every output read LDS instead of re-streaming whole pixels from L2 (the per-pixel kernel's K=5 working set
// over 1-KB pixels exceeds the 32-KB L1).  Per output the taps are applied in the same order as k_dwconv
// (ky-major, kx-minor, out-of-range taps skipped), so y is bit-identical to it; the SE partial sums are per tile
// (fixed order), so their rounding differs from k_dwconv's partition.
constexpr int DT_R = 8;  // output tile rows
__host__ __device__ constexpr int dt_cols(int dq) { return dq == 2 ? 16 : 8; }

inline int dw_dq(int C) {
    const int C4 = C / 4;
    return C4 % 8 == 0 ? 8 : C4 % 4 == 0 ? 4 : C4 % 2 == 0 ? 2 : 0;
}
inline int dt_tiles(int Ho, int Wo, int dq) {
    return ((Ho + DT_R - 1) / DT_R) * ((Wo + dt_cols(dq) - 1) / dt_cols(dq));
}

template <int K, int S, int DQ>
__global__ __launch_bounds__(256) void k_dwconv_t(const float *__restrict__ x, int H, int W, int C,
                                                  const float *__restrict__ wt, const float *__restrict__ bias,
                                                  int pad, int act, float *__restrict__ y, int Ho, int Wo,
                                                  float *__restrict__ psum, int nb) {
    constexpr int TC = dt_cols(DQ), NPL = 256 / DQ, OPT = DT_R * TC / NPL, RS = DT_R / OPT;
    constexpr int PRR = (DT_R - 1) * S + K, PRC = (TC - 1) * S + K, PS = DQ + 1;
    __shared__ float4 patch[PRR * PRC * PS];
    __shared__ float4 red[256];
    const int tid = threadIdx.x, q = tid % DQ, pl = tid / DQ, c = pl % TC, r = pl / TC;  // r < RS
    const int n = blockIdx.y, tile = blockIdx.x, cq = blockIdx.z * DQ + q;
    const int ntx = (Wo + TC - 1) / TC;
    const int oy0 = (tile / ntx) * DT_R, ox0 = (tile % ntx) * TC;
    const int iy0 = oy0 * S - pad, ix0 = ox0 * S - pad;
    const float *xn = x + (int64_t)n * H * W * C + blockIdx.z * DQ * 4;
    for (int e = tid; e < PRR * PRC * DQ; e += 256) {
        const int qq = e % DQ, pp = e / DQ, pr = pp / PRC, pc = pp - pr * PRC;
        const int iy = iy0 + pr, ix = ix0 + pc;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
            v = *(const float4 *)(xn + ((int64_t)iy * W + ix) * C + qq * 4);
        patch[(pr * PRC + pc) * PS + qq] = v;
    }
    __syncthreads();
    float4 s4 = make_float4(0.f, 0.f, 0.f, 0.f);
    {
        float4 w[K * K];
#pragma unroll
        for (int t = 0; t < K * K; ++t) w[t] = *(const float4 *)(wt + (int64_t)t * C + cq * 4);
        const float4 b = *(const float4 *)(bias + cq * 4);
        const int ox = ox0 + c;
#pragma unroll
        for (int h = 0; h < OPT; ++h) {
            const int rr = r + RS * h, oy = oy0 + rr;
            if (oy >= Ho || ox >= Wo) continue;
            float4 acc = b;
#pragma unroll
            for (int ky = 0; ky < K; ++ky) {
                const int iy = iy0 + rr * S + ky;
                if (iy < 0 || iy >= H) continue;
#pragma unroll
                for (int kx = 0; kx < K; ++kx) {
                    const int ix = ix0 + c * S + kx;
                    if (ix < 0 || ix >= W) continue;
                    const float4 v = patch[((rr * S + ky) * PRC + c * S + kx) * PS + q];
                    const float4 ww = w[ky * K + kx];
                    acc.x = __builtin_fmaf(v.x, ww.x, acc.x);
                    acc.y = __builtin_fmaf(v.y, ww.y, acc.y);
                    acc.z = __builtin_fmaf(v.z, ww.z, acc.z);
                    acc.w = __builtin_fmaf(v.w, ww.w, acc.w);
                }
            }
            acc.x = act_f(acc.x, act);
            acc.y = act_f(acc.y, act);
            acc.z = act_f(acc.z, act);
            acc.w = act_f(acc.w, act);
            *(float4 *)(y + (((int64_t)n * Ho + oy) * Wo + ox) * C + cq * 4) = acc;
            s4.x += acc.x;
            s4.y += acc.y;
            s4.z += acc.z;
            s4.w += acc.w;
        }
    }
    if (psum == nullptr) return;
    red[tid] = s4;
    __syncthreads();
    if (pl == 0) {  // fixed order over the pixel lanes: deterministic partial
        for (int l = 1; l < NPL; ++l) {
            const float4 t = red[l * DQ + q];
            s4.x += t.x;
            s4.y += t.y;
            s4.z += t.z;
            s4.w += t.w;
        }
        *(float4 *)(psum + ((int64_t)n * nb + tile) * C + cq * 4) = s4;
    }
}

template <int K, int S>
void launch_dwconv_t(int dq, dim3 grid, hipStream_t st, const float *x, int H, int W, int C, const float *wt,
                     const float *bias, int pad, int act, float *y, int Ho, int Wo, float *psum, int nb) {
    if (dq == 8)
        hipLaunchKernelGGL((k_dwconv_t<K, S, 8>), grid, dim3(256), 0, st, x, H, W, C, wt, bias, pad, act, y, Ho, Wo,
                           psum, nb);
    else if (dq == 4)
        hipLaunchKernelGGL((k_dwconv_t<K, S, 4>), grid, dim3(256), 0, st, x, H, W, C, wt, bias, pad, act, y, Ho, Wo,
                           psum, nb);
    else
        hipLaunchKernelGGL((k_dwconv_t<K, S, 2>), grid, dim3(256), 0, st, x, H, W, C, wt, bias, pad, act, y, Ho, Wo,
                           psum, nb);
}

constexpr int SE_NT = 1024;  // threads of the SE gate workgroup (one per image)

__global__ __launch_bounds__(SE_NT) void k_se_gate(const float *__restrict__ psum, int nb, int C, float hw,
                                                 const float *__restrict__ w1, const float *__restrict__ b1, int rd,
                                                 const float *__restrict__ w2, const float *__restrict__ b2,
                                                 float *__restrict__ gate) {
    extern __shared__ float sh[];  // mean[C], r[rd]
    __shared__ float part[SE_NT];  // [16 partial lanes][64 channels]
    float *mean = sh, *r = sh + C;
    const int n = blockIdx.x, tid = threadIdx.x;
    // squeeze: 64 channels x 16 interleaved partial sums per pass, combined in a fixed order
    for (int c0 = 0; c0 < C; c0 += 64) {
        const int c = c0 + (tid & 63), q0 = tid >> 6;
        // 8 independent chains (loads in flight instead of one latency-bound chain), fixed combine order
        float t8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (c < C) {
            const float *ps = psum + (int64_t)n * nb * C + c;
            constexpr int ST = SE_NT / 64;
            int q = q0;
            for (; q + 7 * ST < nb; q += 8 * ST) {
#pragma unroll
                for (int u = 0; u < 8; ++u) t8[u] += ps[(int64_t)(q + u * ST) * C];
            }
            for (int u = 0; q < nb; q += ST, ++u) t8[u & 7] += ps[(int64_t)q * C];
        }
        const float s = ((t8[0] + t8[1]) + (t8[2] + t8[3])) + ((t8[4] + t8[5]) + (t8[6] + t8[7]));
        part[tid] = s;
        __syncthreads();
        if (tid < 64 && c < C) {
            float t = part[tid];
            for (int k = 1; k < SE_NT / 64; ++k) t += part[k * 64 + tid];
            mean[c] = t / hw;
        }
        __syncthreads();
    }
    for (int j = threadIdx.x; j < rd; j += blockDim.x) {
        float t = b1[j];
        for (int c = 0; c < C; ++c) t = __builtin_fmaf(w1[(int64_t)j * C + c], mean[c], t);
        r[j] = silu_hw(t);  // SiLU (conv_reduce -> act1)
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        float t = b2[c];
        for (int j = 0; j < rd; ++j) t = __builtin_fmaf(w2[(int64_t)c * rd + j], r[j], t);
        gate[(int64_t)n * C + c] = sigmoid_hw(t);  // conv_expand -> sigmoid gate
    }
}

__global__ __launch_bounds__(256) void k_chan_scale(float *__restrict__ y, int64_t P, int C,
                                                    const float *__restrict__ gate, int64_t total4) {
    const int C4 = C >> 2;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total4;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int c4 = (int)(i % C4);
        const int64_t n = i / C4 / P;
        float4 v = *(float4 *)(y + i * 4);
        const float4 g = *(const float4 *)(gate + n * C + c4 * 4);
        v.x *= g.x;
        v.y *= g.y;
        v.z *= g.z;
        v.w *= g.w;
        *(float4 *)(y + i * 4) = v;
    }
}


template <int K>
__global__ __launch_bounds__(DW_NT) void k_dw_wgrad(const float *__restrict__ x, int H, int W, int C,
                                                    const float *__restrict__ dz, int stride, int pad, int Ho, int Wo,
                                                    int ppb, float *__restrict__ dW) {
    __shared__ float4 red[DW_NT];
    const int C4 = C >> 2;
    const int CH4 = C4 <= DW_NT ? C4 : DW_NT / 2;
    const int PB = DW_NT / CH4;
    const int tid = threadIdx.x;
    const int pl = tid / CH4, c4 = blockIdx.z * CH4 + (tid - pl * CH4);
    const bool active = pl < PB && c4 < C4;
    const int n = blockIdx.y, blk = blockIdx.x;
    const int64_t HWo = (int64_t)Ho * Wo;
    const int64_t p0 = (int64_t)blk * ppb, p1 = min(p0 + ppb, HWo);
    float4 acc[K * K];
#pragma unroll
    for (int t = 0; t < K * K; ++t) acc[t] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (active) {
        const float *xn = x + (int64_t)n * H * W * C + c4 * 4;
        const float *dn = dz + (int64_t)n * HWo * C + c4 * 4;
        for (int64_t p = p0 + pl; p < p1; p += PB) {
            const int oy = (int)(p / Wo), ox = (int)(p - (int64_t)oy * Wo);
            const int iy0 = oy * stride - pad, ix0 = ox * stride - pad;
            const float4 g = *(const float4 *)(dn + p * C);
#pragma unroll
            for (int ky = 0; ky < K; ++ky) {
                const int iy = iy0 + ky;
                if (iy < 0 || iy >= H) continue;
#pragma unroll
                for (int kx = 0; kx < K; ++kx) {
                    const int ix = ix0 + kx;
                    if (ix < 0 || ix >= W) continue;
                    const float4 v = *(const float4 *)(xn + ((int64_t)iy * W + ix) * C);
                    float4 &a = acc[ky * K + kx];
                    a.x = __builtin_fmaf(g.x, v.x, a.x);
                    a.y = __builtin_fmaf(g.y, v.y, a.y);
                    a.z = __builtin_fmaf(g.z, v.z, a.z);
                    a.w = __builtin_fmaf(g.w, v.w, a.w);
                }
            }
        }
    }
#pragma unroll
    for (int t = 0; t < K * K; ++t) {
        red[tid] = acc[t];
        __syncthreads();
        if (pl == 0 && c4 < C4) {
            float4 s = acc[t];
            for (int q = 1; q < PB; ++q) {
                const float4 u = red[q * CH4 + tid];
                s.x += u.x;
                s.y += u.y;
                s.z += u.z;
                s.w += u.w;
            }
            float *o = dW + (int64_t)t * C + c4 * 4;
            atomicAdd(o, s.x);
            atomicAdd(o + 1, s.y);
            atomicAdd(o + 2, s.z);
            atomicAdd(o + 3, s.w);
        }
        __syncthreads();
    }
}

// k_stem3: the EfficientNet stem (timm conv_stem, cnn_encoder.py:26: 3x3, stride 2, pad 1, 3 input channels; BN
// folded, SiLU) from the NCHW fp32 images straight to NHWC, on the vector ALU.  K = 27 is far too short for the MFMA
// implicit GEMM (the generic k_conv ran it at 2.1 ms per 14 x 1080p images, 0.7 TB/s); here a workgroup stages the
// 3 x 17 x 129 input window of an 8 x 64 output tile in LDS (coalesced rows, zero padding), each lane computes two
// output pixels (rows 2w and 2w + 1 of its wave, one column) as 27 x CO fp32 FMAs with the weights as scalar
// operands (wave-uniform: s_load, no LDS or VGPR traffic), and each wave writes its 64-pixel row runs back as whole
// NHWC runs (the CO values of a pixel staged at an odd LDS stride, then 16 B per lane, 1 KiB per instruction).
// Per output: sum over (ci, ky, kx) ascending of fmaf(x, w), from +0, then + bias, then the activation.
constexpr int S3_TR = 8, S3_TC = 64;                          // output tile rows / columns
constexpr int S3_IR = 2 * S3_TR + 1, S3_IC = 2 * S3_TC + 1;  // its input window (stride 2, 3 taps)
constexpr int S3_ICP = S3_IC + 3;                             // padded window row (floats)

int g_stem3_stage = 2;  // BEV_TUNE_STEM3_STAGE (r06u micro, 14 x 1080p B3 stem: 64-pixel passes 545 us, 32-pixel 481, registers 3483)

template <int CO, int SP>  // SP: output pixels staged per wave and pass (64 / 32), 0 = stores from registers
__global__ __launch_bounds__(256) void k_stem3(const float *__restrict__ x, int H, int W, const float *__restrict__ wt,
                                               const float *__restrict__ bias, int act, float *__restrict__ y, int Ho,
                                               int Wo, int tiles_x) {
    constexpr int CP = CO + 1;                 // staged pixel stride (odd: conflict-free dword writes)
    constexpr int IN_F = 3 * S3_IR * S3_ICP;   // input window floats
    constexpr int ST_F = 4 * SP * CP;          // output staging floats (4 waves x SP pixels)
    __shared__ float lds[IN_F > ST_F ? IN_F : ST_F];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n = blockIdx.y;
    const int ty = blockIdx.x / tiles_x, tx = blockIdx.x - ty * tiles_x;
    const int r0 = ty * S3_TR, c0 = tx * S3_TC;
    const int iy0 = 2 * r0 - 1, ix0 = 2 * c0 - 1;
    const float *xn = x + (int64_t)n * 3 * H * W;
    constexpr int NE = 3 * S3_IR * S3_IC, NL = (NE + 255) / 256;  // window elements, loads per thread
    float win[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k) {  // every load in flight before the first LDS write
        const int e = tid + 256 * k;
        const int ci = e / (S3_IR * S3_IC), rem = e - ci * (S3_IR * S3_IC);
        const int rr = rem / S3_IC, cc = rem - rr * S3_IC;
        const int iy = iy0 + rr, ix = ix0 + cc;
        const bool in = e < NE && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
        win[k] = in ? xn[((int64_t)ci * H + iy) * W + ix] : 0.0f;
    }
#pragma unroll
    for (int k = 0; k < NL; ++k) {
        const int e = tid + 256 * k;
        const int ci = e / (S3_IR * S3_IC), rem = e - ci * (S3_IR * S3_IC);
        const int rr = rem / S3_IC, cc = rem - rr * S3_IC;
        if (e < NE) lds[(ci * S3_IR + rr) * S3_ICP + cc] = win[k];
    }
    __syncthreads();
    float acc0[CO], acc1[CO];
#pragma unroll
    for (int c = 0; c < CO; ++c) acc0[c] = acc1[c] = 0.0f;
#pragma unroll
    for (int ci = 0; ci < 3; ++ci)
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
                const int t = (ci * 3 + ky) * 3 + kx;
                const float v0 = lds[(ci * S3_IR + 4 * wave + ky) * S3_ICP + 2 * lane + kx];
                const float v1 = lds[(ci * S3_IR + 4 * wave + 2 + ky) * S3_ICP + 2 * lane + kx];
#pragma unroll
                for (int c = 0; c < CO; ++c) {
                    acc0[c] = __builtin_fmaf(v0, wt[t * CO + c], acc0[c]);
                    acc1[c] = __builtin_fmaf(v1, wt[t * CO + c], acc1[c]);
                }
            }
    if constexpr (SP == 0) {  // straight from registers: 16 B per lane, lanes a pixel (CO floats) apart
        const int c = c0 + lane;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int r = r0 + 2 * wave + i;
            if (r >= Ho || c >= Wo) continue;
            float *dst = y + (((int64_t)n * Ho + r) * Wo + c) * CO;
#pragma unroll
            for (int q = 0; q < CO / 4; ++q) {
                float o[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) o[u] = act_f((i ? acc1[4 * q + u] : acc0[4 * q + u]) + bias[4 * q + u], act);
                *(float4 *)(dst + 4 * q) = make_float4(o[0], o[1], o[2], o[3]);
            }
        }
        return;
    }
    __syncthreads();  // the window is no longer read: the staging reuses the LDS
    float *stg = lds + wave * SP * CP;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r = r0 + 2 * wave + i;
#pragma unroll
        for (int hb = 0; hb < 64 / SP; ++hb) {  // pixels hb SP .. hb SP + SP - 1 of the row run
            if (lane / SP == hb) {
#pragma unroll
                for (int c = 0; c < CO; ++c)
                    stg[(lane - hb * SP) * CP + c] = act_f((i ? acc1[c] : acc0[c]) + bias[c], act);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const int np = min(SP, Wo - c0 - hb * SP);  // pixels of this run piece
            if (r < Ho && np > 0) {
                float *dst = y + (((int64_t)n * Ho + r) * Wo + c0 + hb * SP) * CO;
                for (int f = lane * 4; f < np * CO; f += 256) {  // CO % 4 == 0: a quad never straddles two pixels
                    const int p = f / CO, c = f - p * CO;
                    const float *s = stg + p * CP + c;
                    *(float4 *)(dst + f) = make_float4(s[0], s[1], s[2], s[3]);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
}

// k_irdw: an EfficientNet inverted residual's expansion and depthwise conv as ONE pass (timm InvertedResidual
// conv_pw -> bn1 -> SiLU -> conv_dw -> bn2 -> SiLU, cnn_encoder.py:26), plus the SE squeeze partial sums.  The
// expanded tensor h (Cm = 6 Ci channels at the block's input resolution: 4.2 GB per B3 bench step in blocks.1.0
// alone) never reaches HBM: a workgroup owns a strip of TC output columns x IR_RSEG output rows x 48 channels (3
// waves x 16) and walks down its rows; each input row the strip needs is staged once (IR_IC = 32 pixels x CI, zero
// outside the image), expanded by each wave on the fp32 matrix cores (v_mfma_f32_16x16x4_f32: 16 pixels x 16
// channels, K = CI; BN folded, SiLU; h = 0 outside the image -- the depthwise conv's zero padding) into the wave's
// ring of the last K rows in LDS, and every output row is then the K x K taps of that ring (float4 per lane: 16
// pixels x 4 channel quads), + bias, SiLU, stored NHWC and summed into the squeeze partials.
// Numerics: h = SiLU(fp32 dot over CI + bias) (k order of the MFMA: fp32-tolerance equal to the 1x1 conv kernels);
// the depthwise taps in k_dwconv's order from the bias (ky-major, kx-minor; zero taps exact).  psum[n][blk][c] over
// the workgroup's outputs (blk = strip + strips * segment).
constexpr int IR_W = 3;       // waves per workgroup (16 expanded channels each: 48 per workgroup)
constexpr int IR_IC = 32;     // input columns per strip: two 16-pixel MFMA groups
constexpr int IR_RSEG = 16;   // output rows per workgroup
constexpr int IR_HS = 20;     // ring pixel stride (floats): conflict-free h writes, 16-B aligned quads
template <int K, int S> constexpr int ir_tc() { return (IR_IC - K) / S + 1; }  // output columns per strip

typedef float irf4 __attribute__((ext_vector_type(4)));

template <int K, int S, int CI>
__global__ __launch_bounds__(64 * IR_W) void k_irdw(const float *__restrict__ x, int H, int W,
                                                    const float *__restrict__ we, const float *__restrict__ be,
                                                    const float *__restrict__ wd, const float *__restrict__ bd, int Cm,
                                                    float *__restrict__ y, int Ho, int Wo, float *__restrict__ psum,
                                                    int strips, int segs) {
    constexpr int TC = ir_tc<K, S>(), PAD = K / 2, CQ = CI / 4, XS = CI + 1;
    static_assert(CI % 4 == 0 && CI <= 64, "CI");
    __shared__ float xs[IR_IC * XS];                                          // one staged input row
    __shared__ __attribute__((aligned(16))) float ring[IR_W][K][IR_IC * IR_HS];  // the last K expanded rows per wave
    __shared__ __attribute__((aligned(16))) float wds[K * K][16 * IR_W];      // depthwise weights of the 48 channels
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int blk = blockIdx.x, sxi = blk % strips, syi = blk / strips, n = blockIdx.y;
    const int chw = blockIdx.z * 16 * IR_W, ch0 = chw + wave * 16;
    const int c0 = sxi * TC, r0 = syi * IR_RSEG;
    const int ix0 = c0 * S - PAD;
    const int rows_out = min(IR_RSEG, Ho - r0);
    // expansion B operand (k = lane / 16 + 4 step, channel ch0 + lane % 16) and bias
    float bw[CQ];
#pragma unroll
    for (int st = 0; st < CQ; ++st) bw[st] = we[(int64_t)(ch0 + (lane & 15)) * CI + 4 * st + (lane >> 4)];
    const float bexp = be[ch0 + (lane & 15)];
    for (int e = tid; e < K * K * 16 * IR_W; e += 64 * IR_W) {
        const int t = e / (16 * IR_W), c = e - t * (16 * IR_W);
        wds[t][c] = wd[(int64_t)t * Cm + chw + c];
    }
    const int p = lane >> 2, q = lane & 3;  // depthwise: output pixel p (+16 per pass), channel quad q
    const irf4 bdw = *(const irf4 *)(bd + ch0 + 4 * q);
    irf4 ssum = {0.f, 0.f, 0.f, 0.f};
    const float *xn = x + (int64_t)n * H * W * CI;
    float *hr = &ring[wave][0][0];
    // input rows are loaded one row ahead into registers (the next row's loads fly during this row's expansion and
    // the output rows it completes), then written to xs at the next expand_row
    constexpr int NPF = (IR_IC * CQ + 64 * IR_W - 1) / (64 * IR_W);
    irf4 pre[NPF];
    auto load_row = [&](int iy) {
        const bool rin = (unsigned)iy < (unsigned)H;
#pragma unroll
        for (int k = 0; k < NPF; ++k) {
            const int e = tid + 64 * IR_W * k;
            const int px = e / CQ, cq = e - px * CQ, ix = ix0 + px;
            irf4 v = {0.f, 0.f, 0.f, 0.f};
            if (e < IR_IC * CQ && rin && (unsigned)ix < (unsigned)W)
                v = *(const irf4 *)(xn + ((int64_t)iy * W + ix) * CI + 4 * cq);
            pre[k] = v;
        }
    };
    auto expand_row = [&](int iy) {  // stage + expand input row iy into ring slot iy mod K (iy may be outside)
        __syncthreads();  // the previous row's staged pixels are no longer read
        const bool rin = (unsigned)iy < (unsigned)H;
#pragma unroll
        for (int k = 0; k < NPF; ++k) {
            const int e = tid + 64 * IR_W * k;
            const int px = e / CQ, cq = e - px * CQ;
            if (e < IR_IC * CQ) {
#pragma unroll
                for (int u = 0; u < 4; ++u) xs[px * XS + 4 * cq + u] = pre[k][u];
            }
        }
        load_row(iy + 1);
        __syncthreads();
        const int slot = ((iy % K) + K) % K;
#pragma unroll
        for (int g = 0; g < IR_IC / 16; ++g) {
            irf4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int st = 0; st < CQ; ++st)
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xs[(g * 16 + (lane & 15)) * XS + 4 * st + (lane >> 4)], bw[st],
                                                           acc, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int px = g * 16 + 4 * (lane >> 4) + r, ix = ix0 + px;
                const bool in = rin && (unsigned)ix < (unsigned)W;
                hr[slot * IR_IC * IR_HS + px * IR_HS + (lane & 15)] = in ? silu_hw(acc[r] + bexp) : 0.0f;
            }
        }
    };
    int iy_next = r0 * S - PAD;
    load_row(iy_next);
    for (int ro = 0; ro < rows_out; ++ro) {
        const int r = r0 + ro, iy_top = r * S - PAD;
        while (iy_next < iy_top + K) expand_row(iy_next++);
        // this wave's ring writes precede its reads (LDS is in order within a wave)
#pragma unroll
        for (int pp = 0; pp < (TC + 15) / 16; ++pp) {
            const int px = pp * 16 + p, c = c0 + px;
            if (px < TC && c < Wo) {
                irf4 acc = bdw;
#pragma unroll
                for (int ky = 0; ky < K; ++ky) {
                    const int slot = (((iy_top + ky) % K) + K) % K;
#pragma unroll
                    for (int kx = 0; kx < K; ++kx) {
                        const irf4 h = *(const irf4 *)(hr + slot * IR_IC * IR_HS + (px * S + kx) * IR_HS + 4 * q);
                        const irf4 w = *(const irf4 *)(&wds[ky * K + kx][wave * 16 + 4 * q]);
#pragma unroll
                        for (int u = 0; u < 4; ++u) acc[u] = __builtin_fmaf(h[u], w[u], acc[u]);
                    }
                }
                irf4 o;
#pragma unroll
                for (int u = 0; u < 4; ++u) o[u] = silu_hw(acc[u]);
                *(irf4 *)(y + (((int64_t)n * Ho + r) * Wo + c) * Cm + ch0 + 4 * q) = o;
                ssum += o;
            }
        }
    }
    // squeeze partials: the 16 pixel lanes of each channel quad, fixed order
#pragma unroll
    for (int o = 4; o < 64; o <<= 1) {
#pragma unroll
        for (int u = 0; u < 4; ++u) ssum[u] += __shfl_xor(ssum[u], o);
    }
    if (p == 0) *(irf4 *)(psum + ((int64_t)n * strips * segs + blk) * Cm + ch0 + 4 * q) = ssum;
}

inline int last() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

}  // namespace

extern "C" {

// Which kernel: k_dwconv_t with 8-quad (32-channel) chunks whenever C % 32 == 0 -- r02r micro (7 x 1080p B3 shapes):
// C 192 k3 659 -> 435 us, 192 k5 s2 735 -> 572, 288 k5 927 -> 340 -- and with 4- / 2-quad chunks only for outputs of
// at most 64 Ki pixels per image: r02r, B0's k5 layers at 135 x 240 (C 144 / 240) gain (B0 training step 44.6 ->
// 42.9 ms) while B3's 540 x 960 C 40 and 270 x 480 C 144 layers lose badly (572 -> 1360, 665 -> 1042 us: 32- / 64-B
// pixel segments per patch load).  The tiled kernel takes stride 1 or 2; other strides run the per-pixel kernel.
// The choice depends on (Ho, Wo, C, stride) only, so the SE partial count below always matches the kernel that runs.
inline int dw_tiled_dq(int Ho, int Wo, int C, int stride) {
    const int dq = dw_dq(C);
    if (stride != 1 && stride != 2) return 0;
    if (g_dw_run == 3 && dw_run_ch4(C) > 0) return 0;  // row runs for every width
    return (dq == 8 || (dq > 0 && (int64_t)Ho * Wo <= 65536)) ? dq : 0;
}

// k_dwconv_r: stride 1 / 2; channel quads per workgroup = C / 4 split into equal chunks of at most 64
inline bool dw_use_run(int stride, int C) {
    return g_dw_run && (stride == 1 || stride == 2) && (C / 4 <= 64 || (g_dw_run == 3 && dw_run_ch4(C) > 0));
}
inline int dw_run_blocks(int Ho, int Wo, int C, int stride) {
    const int R = stride == 1 ? dw_run_len<1>() : dw_run_len<2>(), PB = DW_NT / dw_run_ch4(C);
    return (int)(((int64_t)Ho * ((Wo + R - 1) / R) + PB - 1) / PB);
}

}  // namespace

namespace bev {
int stem3_tune(int value) {
    if (value < 0 || value > 2) return BEV_ERR_ARGS;
    const int old = g_stem3_stage;
    g_stem3_stage = value;
    return old;
}
int dw_tune(int value) {
    if (value < 0 || value > 3) return BEV_ERR_ARGS;
    const int old = g_dw_run;
    g_dw_run = value;
    return old;
}
}  // namespace bev

extern "C" {

int bev_dwconv_psum_blocks(int Ho, int Wo, int C, int stride) {
    if (Ho <= 0 || Wo <= 0 || C <= 0 || C % 4 != 0 || stride <= 0) return BEV_ERR_ARGS;
    const int dq = dw_tiled_dq(Ho, Wo, C, stride);
    if (dq) return dt_tiles(Ho, Wo, dq);  // one SE partial per output tile
    if (dw_use_run(stride, C)) return dw_run_blocks(Ho, Wo, C, stride);
    const int ppb = dw_ppb(C);
    return (int)(((int64_t)Ho * Wo + ppb - 1) / ppb);
}

int bev_dwconv2d_f32(const float *x, int N, int H, int W, int C, const float *wt, const float *bias, int K, int stride,
                     int pad, int act, float *y, int Ho, int Wo, float *psum, void *stream) {
    if (!x || !wt || !bias || !y || N < 0 || H <= 0 || W <= 0 || C <= 0 || C % 4 != 0 ||
        stride <= 0 || pad < 0 || act < 0 || act > 2)
        return BEV_ERR_ARGS;
    if (K != 3 && K != 5) return BEV_ERR_ARGS;
    if (Ho != (H + 2 * pad - K) / stride + 1 || Wo != (W + 2 * pad - K) / stride + 1 || Ho <= 0 || Wo <= 0)
        return BEV_ERR_ARGS;
    if ((((uintptr_t)x | (uintptr_t)wt | (uintptr_t)bias | (uintptr_t)y | (uintptr_t)psum) & 15) != 0)
        return BEV_ERR_ARGS;
    if (N == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const int dq = dw_tiled_dq(Ho, Wo, C, stride);
    if (!dq && dw_use_run(stride, C)) {
        const int nb = dw_run_blocks(Ho, Wo, C, stride), CH4 = dw_run_ch4(C);
        dim3 grid(nb, N, C / 4 / CH4);
        if (g_dw_run >= 2 && K == 3) {
            if (stride == 1)
                hipLaunchKernelGGL((k_dwconv_r<3, 1, true>), grid, dim3(DW_NT), 0, st, x, H, W, C, wt, bias, pad, act, y,
                                   Ho, Wo, psum, nb, CH4);
            else
                hipLaunchKernelGGL((k_dwconv_r<3, 2, true>), grid, dim3(DW_NT), 0, st, x, H, W, C, wt, bias, pad, act, y,
                                   Ho, Wo, psum, nb, CH4);
            return last();
        }
        if (K == 3 && stride == 1)
            hipLaunchKernelGGL((k_dwconv_r<3, 1, false>), grid, dim3(DW_NT), 0, st, x, H, W, C, wt, bias, pad, act, y, Ho, Wo,
                               psum, nb, CH4);
        else if (K == 3)
            hipLaunchKernelGGL((k_dwconv_r<3, 2, false>), grid, dim3(DW_NT), 0, st, x, H, W, C, wt, bias, pad, act, y, Ho, Wo,
                               psum, nb, CH4);
        else if (stride == 1)
            hipLaunchKernelGGL((k_dwconv_r<5, 1, false>), grid, dim3(DW_NT), 0, st, x, H, W, C, wt, bias, pad, act, y, Ho, Wo,
                               psum, nb, CH4);
        else
            hipLaunchKernelGGL((k_dwconv_r<5, 2, false>), grid, dim3(DW_NT), 0, st, x, H, W, C, wt, bias, pad, act, y, Ho, Wo,
                               psum, nb, CH4);
        return last();
    }
    if (!dq) {
        const int nb = bev_dwconv_psum_blocks(Ho, Wo, C, stride), ppb = dw_ppb(C);
        const int C4 = C / 4, CH4 = dw_ch4(C);
        dim3 grid(nb, N, (C4 + CH4 - 1) / CH4);
        if (K == 3)
            hipLaunchKernelGGL(k_dwconv<3>, grid, dim3(DW_NT), 0, st, x, H, W, C, wt, bias, stride, pad, act, y, Ho,
                               Wo, psum, nb, ppb);
        else
            hipLaunchKernelGGL(k_dwconv<5>, grid, dim3(DW_NT), 0, st, x, H, W, C, wt, bias, stride, pad, act, y, Ho,
                               Wo, psum, nb, ppb);
        return last();
    }
    const int nb = dt_tiles(Ho, Wo, dq);
    dim3 grid(nb, N, C / 4 / dq);
    if (K == 3 && stride == 1) launch_dwconv_t<3, 1>(dq, grid, st, x, H, W, C, wt, bias, pad, act, y, Ho, Wo, psum, nb);
    else if (K == 3) launch_dwconv_t<3, 2>(dq, grid, st, x, H, W, C, wt, bias, pad, act, y, Ho, Wo, psum, nb);
    else if (stride == 1) launch_dwconv_t<5, 1>(dq, grid, st, x, H, W, C, wt, bias, pad, act, y, Ho, Wo, psum, nb);
    else launch_dwconv_t<5, 2>(dq, grid, st, x, H, W, C, wt, bias, pad, act, y, Ho, Wo, psum, nb);
    return last();
}

int bev_ir_expand_dw_blocks(int Ho, int Wo, int K, int stride) {
    if (Ho <= 0 || Wo <= 0 || (K != 3 && K != 5) || (stride != 1 && stride != 2)) return BEV_ERR_ARGS;
    const int tc = (IR_IC - K) / stride + 1;
    return ((Wo + tc - 1) / tc) * ((Ho + IR_RSEG - 1) / IR_RSEG);
}

int bev_ir_expand_dw_f32(const float *x, int N, int H, int W, int Ci, const float *we, const float *be, int Cm,
                         const float *wd, const float *bd, int K, int stride, float *y, int Ho, int Wo, float *psum,
                         void *stream) {
    if (!x || !we || !be || !wd || !bd || !y || !psum || N < 0 || H <= 0 || W <= 0 || Cm <= 0 || Cm % 48 != 0)
        return BEV_ERR_ARGS;
    if ((Ci != 16 && Ci != 24 && Ci != 32 && Ci != 40 && Ci != 48) || (K != 3 && K != 5) || (stride != 1 && stride != 2))
        return BEV_ERR_ARGS;
    const int pad = K / 2;
    if (Ho != (H + 2 * pad - K) / stride + 1 || Wo != (W + 2 * pad - K) / stride + 1) return BEV_ERR_ARGS;
    if ((((uintptr_t)x | (uintptr_t)bd | (uintptr_t)y | (uintptr_t)psum) & 15) != 0) return BEV_ERR_ARGS;
    if ((int64_t)H * W * Ci >= ((int64_t)1 << 31) || (int64_t)Ho * Wo * Cm >= ((int64_t)1 << 31)) return BEV_ERR_ARGS;
    if (N == 0) return 0;
    const int tc = (IR_IC - K) / stride + 1, strips = (Wo + tc - 1) / tc, segs = (Ho + IR_RSEG - 1) / IR_RSEG;
    const dim3 grid(strips * segs, N, Cm / 48), block(64 * IR_W);
    hipStream_t st = (hipStream_t)stream;
#define IRDW(KK, SS, CC)                                                                                           \
    hipLaunchKernelGGL((k_irdw<KK, SS, CC>), grid, block, 0, st, x, H, W, we, be, wd, bd, Cm, y, Ho, Wo, psum, strips, \
                       segs)
#define IRDW_CI(KK, SS)                                                                                            \
    do {                                                                                                           \
        if (Ci == 16) IRDW(KK, SS, 16);                                                                            \
        else if (Ci == 24) IRDW(KK, SS, 24);                                                                       \
        else if (Ci == 32) IRDW(KK, SS, 32);                                                                       \
        else if (Ci == 40) IRDW(KK, SS, 40);                                                                       \
        else IRDW(KK, SS, 48);                                                                                     \
    } while (0)
    if (K == 3 && stride == 1) IRDW_CI(3, 1);
    else if (K == 3) IRDW_CI(3, 2);
    else if (stride == 1) IRDW_CI(5, 1);
    else IRDW_CI(5, 2);
#undef IRDW_CI
#undef IRDW
    return last();
}

int bev_conv2d_stem3_f32(const float *x, int N, int H, int W, const float *wt, const float *bias, int Co, int act,
                         float *y, int Ho, int Wo, void *stream) {
    if (!x || !wt || !bias || !y || N < 0 || H <= 0 || W <= 0 || act < 0 || act > 2 ||
        (Co != 32 && Co != 40 && Co != 48 && Co != 64))
        return BEV_ERR_ARGS;
    if (Ho != (H - 1) / 2 + 1 || Wo != (W - 1) / 2 + 1 || (((uintptr_t)y) & 15) != 0) return BEV_ERR_ARGS;
    if ((int64_t)3 * H * W >= ((int64_t)1 << 31)) return BEV_ERR_ARGS;
    if (N == 0) return 0;
    const int tiles_x = (Wo + S3_TC - 1) / S3_TC, tiles = ((Ho + S3_TR - 1) / S3_TR) * tiles_x;
    const dim3 grid(tiles, N);
    hipStream_t st = (hipStream_t)stream;
#define STEM3_LAUNCH(CO)                                                                                          \
    do {                                                                                                         \
        if (g_stem3_stage == 1)                                                                                  \
            hipLaunchKernelGGL((k_stem3<CO, 64>), grid, dim3(256), 0, st, x, H, W, wt, bias, act, y, Ho, Wo, tiles_x);  \
        else if (g_stem3_stage == 2)                                                                             \
            hipLaunchKernelGGL((k_stem3<CO, 32>), grid, dim3(256), 0, st, x, H, W, wt, bias, act, y, Ho, Wo, tiles_x);  \
        else                                                                                                     \
            hipLaunchKernelGGL((k_stem3<CO, 0>), grid, dim3(256), 0, st, x, H, W, wt, bias, act, y, Ho, Wo, tiles_x);   \
    } while (0)
    if (Co == 32) STEM3_LAUNCH(32);
    else if (Co == 40) STEM3_LAUNCH(40);
    else if (Co == 48) STEM3_LAUNCH(48);
    else STEM3_LAUNCH(64);
#undef STEM3_LAUNCH
    return last();
}

int bev_se_gate_f32(const float *psum, int N, int nb, int C, int hw, const float *w1, const float *b1, int rd,
                    const float *w2, const float *b2, float *gate, void *stream) {
    if (!psum || !w1 || !b1 || !w2 || !b2 || !gate || N < 0 || nb <= 0 || C <= 0 || rd <= 0 || hw <= 0 ||
        (C + rd) > 12288)
        return BEV_ERR_ARGS;
    if (N == 0) return 0;
    hipLaunchKernelGGL(k_se_gate, dim3(N), dim3(SE_NT), (C + rd) * sizeof(float), (hipStream_t)stream, psum, nb, C,
                       (float)hw, w1, b1, rd, w2, b2, gate);
    return last();
}

int bev_channel_scale_f32(float *y, int N, int64_t P, int C, const float *gate, void *stream) {
    if (!y || !gate || N < 0 || P < 0 || C <= 0 || C % 4 != 0 || (((uintptr_t)y | (uintptr_t)gate) & 15) != 0)
        return BEV_ERR_ARGS;
    const int64_t total4 = (int64_t)N * P * (C / 4);
    if (total4 == 0) return 0;
    const int64_t blocks = (total4 + 255) / 256 < 256 * 64 ? (total4 + 255) / 256 : 256 * 64;
    hipLaunchKernelGGL(k_chan_scale, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, y, P, C, gate,
                       total4);
    return last();
}

int bev_dwconv_wgrad_f32(const float *x, int N, int H, int W, int C, const float *dz, int Ho, int Wo, int K, int stride,
                         int pad, float *dW, void *stream) {
    if (!x || !dz || !dW || N < 0 || H <= 0 || W <= 0 || C <= 0 || C % 4 != 0 || stride <= 0 || pad < 0)
        return BEV_ERR_ARGS;
    if (K != 3 && K != 5) return BEV_ERR_ARGS;
    if (Ho != (H + 2 * pad - K) / stride + 1 || Wo != (W + 2 * pad - K) / stride + 1 || Ho <= 0 || Wo <= 0)
        return BEV_ERR_ARGS;
    if ((((uintptr_t)x | (uintptr_t)dz | (uintptr_t)dW) & 15) != 0) return BEV_ERR_ARGS;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(dW, 0, (size_t)K * K * C * sizeof(float), st) != hipSuccess) return last();
    if (N == 0) return 0;
    const int ppb = dw_ppb(C), nb = (int)(((int64_t)Ho * Wo + ppb - 1) / ppb);  // its own pixel partition
    const int C4 = C / 4, CH4 = dw_ch4(C);
    dim3 grid(nb, N, (C4 + CH4 - 1) / CH4);
    if (K == 3)
        hipLaunchKernelGGL(k_dw_wgrad<3>, grid, dim3(DW_NT), 0, st, x, H, W, C, dz, stride, pad, Ho, Wo, ppb, dW);
    else
        hipLaunchKernelGGL(k_dw_wgrad<5>, grid, dim3(DW_NT), 0, st, x, H, W, C, dz, stride, pad, Ho, Wo, ppb, dW);
    return last();
}

}  // extern "C"
