// bev_train.hip -- backward kernels of the backbone trunk for gfx950 (training, BASELINE config 3).
//
// The reference trains its timm trunk through torch autograd (train.py:249-255, the optimizer holds the
// trunk parameters: model_wrapper.py lazy modules do not exist yet when it is built, quirk Q2).  Here
// every conv + (frozen, folded) BN + ReLU of the trunk has an autograd node whose backward runs:
//
//   k_relu_bwd     dz = dy * (y > 0)                                   (ReLU mask from the saved output)
//   k_dilate       zero-inserted, padded copy of dz for strided dgrad  (so dgrad is a stride-1 conv)
//   bev_conv2d_f32 dx = conv(dilate(dz), flip(W)^T)                    (the forward MFMA kernel)
//   k_wgrad        dW[co][k] = sum_m dz[m][co] * im2col(x)[m][k]       (LDS-tiled, split over m, f32 atomics;
//                  k_wgrad_v4 = float4 staging without index divisions when Ci % 4 == 0 and Co % 4 == 0)
//   k_colsum       db[co] = sum_m dz[m][co]
//   k_maxpool_bwd  dx = sum of dy over the windows whose first maximum is this input (gather, no atomics;
//                  k_maxpool_bwd_v4: four channels per thread when C % 4 == 0; bev_maxpool2d_bwd_ws_nhwc_f32:
//                  window argmax bytes once, then the gather -- k_maxpool_argmax_v4 + k_maxpool_bwd_idx_v4)
//
// All tensors NHWC fp32.  Float atomics in k_wgrad / k_colsum: the last bits of the weight gradients
// may vary run to run (summation order); the activations' gradients are deterministic.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bev_mi355x.h"
#include "bev_tune.h"

namespace {

int g_wgrad_mfma = 2;  // bev_tune(BEV_TUNE_WGRAD_MFMA): 2 = k_wgrad_nat (default), 1 = k_wgrad_mfma, 0 = k_wgrad_v4
typedef float wf32x16 __attribute__((ext_vector_type(16)));
typedef float wf32x4 __attribute__((ext_vector_type(4)));

inline int last() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

__global__ __launch_bounds__(256) void k_relu_bwd(const float *__restrict__ dy, const float *__restrict__ y,
                                                  float *__restrict__ dz, int64_t n4) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 g = ((const float4 *)dy)[i], v = ((const float4 *)y)[i];
        ((float4 *)dz)[i] = make_float4(v.x > 0.f ? g.x : 0.f, v.y > 0.f ? g.y : 0.f, v.z > 0.f ? g.z : 0.f,
                                        v.w > 0.f ? g.w : 0.f);
    }
}

// out [N][Hd][Wd][C] (zero everywhere else): out[n][top + oy*s][left + ox*s][c] = dz[n][oy][ox][c]; Q = one
// channel quad (float4 for fp32, uint2 for fp16 elements: a copy, so any 4-element type)
template <typename Q>
__global__ __launch_bounds__(256) void k_dilate(const Q *__restrict__ dz, int N, int Ho, int Wo, int C, int s,
                                                int top, int left, int Hd, int Wd, Q *__restrict__ out) {
    const int64_t total = (int64_t)N * Hd * Wd * (C / 4);
    const int C4 = C / 4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int c4 = (int)(i % C4);
        int64_t t = i / C4;
        const int x = (int)(t % Wd);
        t /= Wd;
        const int y = (int)(t % Hd);
        const int n = (int)(t / Hd);
        const int yy = y - top, xx = x - left;
        Q v = {};
        if (yy >= 0 && xx >= 0 && yy % s == 0 && xx % s == 0 && yy / s < Ho && xx / s < Wo)
            v = dz[(((int64_t)n * Ho + yy / s) * Wo + xx / s) * C4 + c4];
        out[i] = v;
    }
}

// The input gradient of a 1x1 / stride-s / pad-0 conv without dilation: out [N][H][W][C] = residual (or 0) plus, at
// (s*oy, s*ox), y[n][oy][ox] = dz W -- one pass over out (the dilated form wrote the zero-inserted 4x map and ran the
// 1x1 conv over it).  Grid (pixel blocks, images), thread = (channel quad, pixel phase) as the streaming passes.
__global__ __launch_bounds__(256) void k_place_strided(const float4 *__restrict__ y, int Ho, int Wo, int C4, int s,
                                                       int H, int W, const float4 *__restrict__ res,
                                                       float4 *__restrict__ out) {
    const int n = blockIdx.y, tid = threadIdx.x, q = tid % C4, ph = tid / C4, nph = 256 / C4;
    const int64_t p0 = (int64_t)blockIdx.x * 256, p1 = p0 + 256 < (int64_t)H * W ? p0 + 256 : (int64_t)H * W;
    for (int64_t p = p0 + ph; p < p1; p += nph) {
        const int yy = (int)(p / W), xx = (int)(p - (int64_t)yy * W);
        const int64_t e = ((int64_t)n * H * W + p) * C4 + q;
        float4 v = res ? res[e] : make_float4(0.f, 0.f, 0.f, 0.f);
        if (yy % s == 0 && xx % s == 0 && yy / s < Ho && xx / s < Wo) {
            const float4 u = y[(((int64_t)n * Ho + yy / s) * Wo + xx / s) * C4 + q];
            v = res ? make_float4(v.x + u.x, v.y + u.y, v.z + u.z, v.w + u.w) : u;  // no residual: y itself (-0 kept)
        }
        out[e] = v;
    }
}

// dW[co][k], k = (ky*KW + kx)*Ci + ci.  Workgroup = 64 (co) x 64 (k) outputs, 256 threads x (4 x 4);
// loops over its slice of m in steps of 16 with both operands staged in LDS.
constexpr int WG_T = 64, WG_M = 16;
__global__ __launch_bounds__(256) void k_wgrad(const float *__restrict__ x, const float *__restrict__ dz, int N, int H,
                                               int W, int Ci, int Ho, int Wo, int Co, int KH, int KW, int stride,
                                               int pad, int dil, int64_t mchunk, float *__restrict__ dW) {
    __shared__ float sa[WG_M][WG_T + 4];  // im2col(x)[m][k]
    __shared__ float sd[WG_M][WG_T + 4];  // dz[m][co]
    const int K = KH * KW * Ci;
    const int k0 = blockIdx.x * WG_T, co0 = blockIdx.y * WG_T;
    const int64_t M = (int64_t)N * Ho * Wo;
    const int64_t mb = (int64_t)blockIdx.z * mchunk, me = mb + mchunk < M ? mb + mchunk : M;
    const int tid = threadIdx.x, tr = tid >> 4, tc = tid & 15;  // 16 x 16 threads, 4 x 4 each
    float acc[4][4] = {};
    for (int64_t m = mb; m < me; m += WG_M) {
        // stage: 16 rows x 64 columns of each operand, 4 elements per thread each
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int idx = tid + 256 * e, r = idx >> 6, c = idx & 63;
            const int64_t mm = m + r;
            float av = 0.f, dv = 0.f;
            if (mm < me) {
                const int ox = (int)(mm % Wo);
                const int64_t t = mm / Wo;
                const int oy = (int)(t % Ho), n = (int)(t / Ho);
                const int k = k0 + c;
                if (k < K) {
                    const int ci = k % Ci, rr = k / Ci, kx = rr % KW, ky = rr / KW;
                    const int iy = oy * stride - pad + ky * dil, ix = ox * stride - pad + kx * dil;
                    if (iy >= 0 && iy < H && ix >= 0 && ix < W) av = x[(((int64_t)n * H + iy) * W + ix) * Ci + ci];
                }
                if (co0 + c < Co) dv = dz[mm * Co + co0 + c];
            }
            sa[r][c] = av;
            sd[r][c] = dv;
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < WG_M; ++r) {
            float a4[4], d4[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                d4[i] = sd[r][tr * 4 + i];
                a4[i] = sa[r][tc * 4 + i];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_fmaf(d4[i], a4[j], acc[i][j]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int co = co0 + tr * 4 + i;
        if (co >= Co) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = k0 + tc * 4 + j;
            if (k < K) atomicAdd(dW + (int64_t)co * K + k, acc[i][j]);
        }
    }
}

// Same contraction for Ci % 4 == 0 and Co % 4 == 0 (every trunk / head conv once the stem's 3 input channels
// and the head's 5 outputs are zero-padded to 4 / 8 by the host).  Each thread stages one float4 of each
// operand per m step (row tid >> 4, columns 4 (tid & 15)); its k column (tap ky, kx and channel ci) is fixed
// for the whole loop and decoded once, and the output pixel (n, oy, ox) of its row advances incrementally --
// no integer division in the loop (the generic kernel spends most of its time in the per-element 64-bit index
// decode).
__global__ __launch_bounds__(256) void k_wgrad_v4(const float *__restrict__ x, const float *__restrict__ dz, int N,
                                                  int H, int W, int Ci, int Ho, int Wo, int Co, int KW, int K,
                                                  int stride, int pad, int dil, int64_t mchunk, float *__restrict__ dW) {
    __shared__ __attribute__((aligned(16))) float sa[WG_M][WG_T + 4];
    __shared__ __attribute__((aligned(16))) float sd[WG_M][WG_T + 4];
    const int k0 = blockIdx.x * WG_T, co0 = blockIdx.y * WG_T;
    const int64_t M = (int64_t)N * Ho * Wo;
    const int64_t mb = (int64_t)blockIdx.z * mchunk, me = mb + mchunk < M ? mb + mchunk : M;
    const int tid = threadIdx.x, tr = tid >> 4, tc = tid & 15;
    const int r = tid >> 4, c4 = tid & 15;
    const int kk = k0 + 4 * c4;  // this thread's staged k column (4 channels of one tap)
    const bool k_ok = kk < K;
    const int rr = k_ok ? kk / Ci : 0, ci = kk - rr * Ci, kx = rr % KW, ky = rr / KW;
    const bool dz_ok = co0 + 4 * c4 < Co;
    // output pixel of row mb + r
    int64_t mm = mb + r;
    int ox, oy, n;
    {
        const int64_t m0 = mm < M ? mm : 0;
        ox = (int)(m0 % Wo);
        const int64_t t = m0 / Wo;
        oy = (int)(t % Ho);
        n = (int)(t / Ho);
    }
    float acc[4][4] = {};
    for (int64_t m = mb; m < me; m += WG_M, mm += WG_M) {
        float4 av = make_float4(0.f, 0.f, 0.f, 0.f), dv = av;
        if (mm < me) {
            const int iy = oy * stride - pad + ky * dil, ix = ox * stride - pad + kx * dil;
            if (k_ok && iy >= 0 && iy < H && ix >= 0 && ix < W)
                av = *(const float4 *)(x + (((int64_t)n * H + iy) * W + ix) * Ci + ci);
            if (dz_ok) dv = *(const float4 *)(dz + mm * Co + co0 + 4 * c4);
        }
        *(float4 *)&sa[r][4 * c4] = av;
        *(float4 *)&sd[r][4 * c4] = dv;
        ox += WG_M;
        while (ox >= Wo) {
            ox -= Wo;
            if (++oy == Ho) {
                oy = 0;
                ++n;
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < WG_M; ++q) {
            const float4 d = *(const float4 *)&sd[q][tr * 4];
            const float4 a = *(const float4 *)&sa[q][tc * 4];
            const float d4[4] = {d.x, d.y, d.z, d.w}, a4[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_fmaf(d4[i], a4[j], acc[i][j]);
        }
        __syncthreads();
    }
    const int kc = k0 + tc * 4;
    if (kc >= K) return;  // K % 4 == 0: the thread's 4 columns are all valid or all not
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int co = co0 + tr * 4 + i;
        if (co >= Co) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) atomicAdd(dW + (int64_t)co * K + kc + j, acc[i][j]);
    }
}


// ---- weight gradient on the MFMA, natural-layout operands by LDS-DMA (default) ----------------------
// v_mfma_f32_32x32x2_f32 takes ONE A and ONE B value per lane: A[i][kk] from lane i + 32 kk, B[kk][j] from
// lane j + 32 kk.  For dW = dz^T im2col(x) the MFMA's reduction index kk is the output pixel m, so a lane needs
// dz[m0 + kk][co0 + i] and im2col(x)[m0 + kk][k0 + j]: 32 consecutive elements of ONE pixel row per half-wave,
// i.e. both operands in their natural [pixel][channel] layout.  Each step therefore copies 32 pixel rows of
// both operands global -> LDS with global_load_lds_dwordx4 (no staging registers, no transposing ds_writes;
// invalid taps / rows read a zero quad), double-buffered, and the fragments are conflict-free ds_read_b32 of
// consecutive dwords.  Same tiles, m split and float-atomic epilogue as k_wgrad_mfma below.
__device__ __attribute__((aligned(16))) float g_wzero4[4] = {0.f, 0.f, 0.f, 0.f};  // never written

__device__ __forceinline__ unsigned wg_lds_base(const void *p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) unsigned char *)p;
}

__device__ __forceinline__ void wg_dma16(const float *src, unsigned dst_any) {
    const unsigned dst = (unsigned)__builtin_amdgcn_readfirstlane((int)dst_any);  // wave-uniform LDS address
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(dst)
        : "memory");
}

template <int WCO, int TM, int TN>
__global__ __launch_bounds__(256, TN == 4 ? 1 : 2) void k_wgrad_nat(const float *__restrict__ x, const float *__restrict__ dz, int N,
                                                      int H, int W, int Ci, int Ho, int Wo, int Co, int KW, int K,
                                                      int stride, int pad, int dil, int64_t mchunk, int ctiles,
                                                      int ntiles, float *__restrict__ dW) {
    constexpr int WK = 4 / WCO, CT = WCO * TM * 32, KT = WK * TN * 32;
    constexpr int AF = CT / 4, BF = KT / 4;             // float4 per pixel row of each operand
    constexpr int QA = 32 * AF / 256, QB = 32 * BF / 256;  // DMA instructions per wave and step
    constexpr int STAGE = 32 * (CT + KT);               // floats per stage
    static_assert((32 * AF) % 256 == 0 && (32 * BF) % 256 == 0, "whole DMA instructions per wave");
    __shared__ __attribute__((aligned(16))) float lds[2 * STAGE];
    unsigned bid = blockIdx.x;
    {
        const unsigned nb = gridDim.x, q = nb / 8, r = nb % 8, xc = bid % 8;
        bid = (xc < r ? xc * (q + 1) : r * (q + 1) + (xc - r) * q) + bid / 8;
    }
    const int tile = (int)(bid % (unsigned)ntiles);
    const int64_t split = bid / (unsigned)ntiles;
    const int co0 = (tile % ctiles) * CT, k0 = (tile / ctiles) * KT;
    const int64_t M = (int64_t)N * Ho * Wo;
    const int64_t mb = split * mchunk, me = mb + mchunk < M ? mb + mchunk : M;
    if (mb >= me) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wco = wave / WK, wk = wave % WK;

    // first pixel of the step being copied, as (image, row, column); each DMA instruction's pixel rows and
    // channel columns are decoded on the fly (few registers: up to 16 instructions per wave and step)
    int mpx, mpy, mpn;
    {
        const int64_t t = mb / Wo;
        mpx = (int)(mb - t * Wo);
        mpy = (int)(t % Ho);
        mpn = (int)(t / Ho);
    }
    const unsigned lbase = wg_lds_base(lds);
    int64_t ms = mb;
    auto issue = [&](int buf) {
        const unsigned d0 = lbase + (unsigned)(buf * STAGE * 4);
#pragma unroll
        for (int q = 0; q < QA; ++q) {
            const int f = (wave + 4 * q) * 64 + lane, row = f / AF, col = f % AF;
            const int64_t m = ms + row;
            const float *src = (m < me && co0 + 4 * col < Co) ? dz + m * Co + co0 + 4 * col : g_wzero4;
            wg_dma16(src, d0 + (unsigned)((wave + 4 * q) * 1024));
        }
#pragma unroll
        for (int q = 0; q < QB; ++q) {
            const int f = (wave + 4 * q) * 64 + lane, row = f / BF;
            const int k = k0 + 4 * (f % BF);
            const int tap = k / Ci, ci = k - tap * Ci, ky = tap / KW, kx = tap - ky * KW;
            int px = mpx + row, py = mpy, pn = mpn;
            while (px >= Wo) {  // rows of one step span at most 32 pixels
                px -= Wo;
                if (++py == Ho) {
                    py = 0;
                    ++pn;
                }
            }
            const int iy = py * stride - pad + ky * dil, ix = px * stride - pad + kx * dil;
            const bool in = ms + row < me && k < K && iy >= 0 && iy < H && ix >= 0 && ix < W;
            const float *src = in ? x + (((int64_t)pn * H + iy) * W + ix) * Ci + ci : g_wzero4;
            wg_dma16(src, d0 + (unsigned)(CT * 32 * 4 + (wave + 4 * q) * 1024));
        }
        ms += 32;
        mpx += 32;
        while (mpx >= Wo) {
            mpx -= Wo;
            if (++mpy == Ho) {
                mpy = 0;
                ++mpn;
            }
        }
    };
    wf32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (wf32x16){0};
    const int nsteps = (int)((me - mb + 31) / 32);
    issue(0);
    const int r32 = lane & 31, h = lane >> 5;
    for (int st = 0; st < nsteps; ++st) {
        if (st + 1 < nsteps) {
            issue((st + 1) & 1);
            // this wave's copies of step st are done; the ones of step st + 1 stay in flight
            if (QA + QB == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            else if (QA + QB == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else if (QA + QB == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            else if (QA + QB == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else if (QA + QB == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();  // every wave's share of step st is in LDS
        const float *As = lds + (st & 1) * STAGE, *Bs = As + CT * 32;
#pragma unroll
        for (int p = 0; p < 16; ++p) {
            const int row = 2 * p + h;
            float fa[TM], fb[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) fa[i] = As[row * CT + wco * TM * 32 + i * 32 + r32];
#pragma unroll
            for (int j = 0; j < TN; ++j) fb[j] = Bs[row * KT + wk * TN * 32 + j * 32 + r32];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();  // step st's buffer is free for step st + 2
    }
    // D[row][col]: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int k = k0 + wk * TN * 32 + j * 32 + r32;
            if (k >= K) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int co = co0 + wco * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (co < Co) atomicAdd(dW + (int64_t)co * K + k, acc[i][j][r]);
            }
        }
}

template <int WCO, int TM, int TN>
int launch_wgrad_nat(const float *x, const float *dz, int N, int H, int W, int Ci, int Ho, int Wo, int Co, int KW,
                     int K, int stride, int pad, int dil, float *dW, hipStream_t st) {
    constexpr int CT = WCO * TM * 32, KT = (4 / WCO) * TN * 32;
    const int64_t M = (int64_t)N * Ho * Wo;
    const int ct = (Co + CT - 1) / CT, kt = (K + KT - 1) / KT, nt = ct * kt;
    int64_t sp = 1024 / nt + 1;  // >= ~1024 workgroups (2 per CU resident)
    int64_t mc = (M + sp - 1) / sp;
    mc = ((mc + 31) / 32) * 32;
    sp = (M + mc - 1) / mc;
    if (sp * nt >= ((int64_t)1 << 31)) return BEV_ERR_ARGS;
    hipLaunchKernelGGL((k_wgrad_nat<WCO, TM, TN>), dim3((unsigned)(sp * nt)), dim3(256), 0, st, x, dz, N, H, W, Ci, Ho,
                       Wo, Co, KW, K, stride, pad, dil, mc, ct, nt, dW);
    return 0;
}

// ---- weight gradient on the MFMA, transposed staging (BEV_TUNE_WGRAD_MFMA = 1) ------------------------
// dW[co][k] = sum_m dz[m][co] * im2col(x)[m][k] as a GEMM whose reduction runs over the output pixels m.
// Workgroup tile CT (co) x KT (k) = (WCO x TM x 32) x (WK x TN x 32), WCO x WK = 4 waves of TM x TN
// v_mfma_f32_32x32x2_f32 tiles -- 128 x 128 in general, 64 x 256 for 64-channel layers, 256 x 64 for K = 64,
// 32 x 512 for the BEV head's 5 (-> 8) outputs, so the MFMA tiles are not half empty on the narrow layers.
// Each step stages 32 pixels of both operands TRANSPOSED into LDS ([co][m] and [k][m], 144-B rows) so the
// MFMA fragments are contiguous float4 reads along m, exactly like k_conv's A/B panels; the next step's global
// loads are issued into registers before the current step's MFMAs.  A thread's staged k column (one tap, 4
// channels) is decoded once, and the output pixels of its rows advance incrementally.  The m range is split
// over a 1-D XCD-aware grid (the tiles of one m split run on one XCD and share its L2); partial tiles are
// added with float atomics (summation order varies in the last bits, as in k_wgrad).
constexpr int WM_BM = 32, WM_LROW = 36;

// LDS element (row c, pixel m) of a staged operand: 36-float rows; the 16-B group of m is XOR-swizzled by
// c >> 4 so the transposed staging writes (lanes = consecutive float4 columns c = 4 ac + u) hit distinct
// banks, while the float4 fragment reads (16 consecutive rows share one key) stay contiguous and
// conflict-free.
__device__ __forceinline__ int wsw(int c, int m) { return c * WM_LROW + ((((m >> 2) ^ ((c >> 4) & 7)) << 2) | (m & 3)); }

template <int WCO, int TM, int TN, int NBUF>
__global__ __launch_bounds__(256, TN == 4 ? 1 : 2) void k_wgrad_mfma(const float *__restrict__ x, const float *__restrict__ dz,
                                                       int N, int H, int W, int Ci, int Ho, int Wo, int Co, int KW,
                                                       int K, int stride, int pad, int dil, int64_t mchunk,
                                                       int ctiles, int ntiles, float *__restrict__ dW) {
    constexpr int WK = 4 / WCO, CT = WCO * TM * 32, KT = WK * TN * 32;
    constexpr int ACOLS = CT / 4, ARPP = 256 / ACOLS, AQ = WM_BM / ARPP;  // float4 columns, rows per pass, passes
    constexpr int BCOLS = KT / 4, BRPP = 256 / BCOLS, BQ = WM_BM / BRPP;
    constexpr int STAGE = (CT + KT) * WM_LROW;
    __shared__ __attribute__((aligned(16))) float lds[NBUF * STAGE];
    unsigned bid = blockIdx.x;
    {
        const unsigned nb = gridDim.x, q = nb / 8, r = nb % 8, xc = bid % 8;
        bid = (xc < r ? xc * (q + 1) : r * (q + 1) + (xc - r) * q) + bid / 8;
    }
    const int tile = (int)(bid % (unsigned)ntiles);
    const int64_t split = bid / (unsigned)ntiles;
    const int co0 = (tile % ctiles) * CT, k0 = (tile / ctiles) * KT;
    const int64_t M = (int64_t)N * Ho * Wo;
    const int64_t mb = split * mchunk, me = mb + mchunk < M ? mb + mchunk : M;
    if (mb >= me) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wco = wave / WK, wk = wave % WK;
    const int ac = tid % ACOLS, ar = tid / ACOLS;  // A staging: float4 column ac, rows ar + ARPP q
    const int bc = tid % BCOLS, br = tid / BCOLS;  // B staging: float4 column bc, rows br + BRPP q
    const bool c_ok = co0 + 4 * ac < Co;
    const int kk = k0 + 4 * bc;
    const bool k_ok = kk < K;
    const int tap = k_ok ? kk / Ci : 0, ci = kk - tap * Ci, kx = tap % KW, ky = tap / KW;
    int px[BQ], py[BQ], pn[BQ];
#pragma unroll
    for (int q = 0; q < BQ; ++q) {
        int64_t m = mb + br + BRPP * q;
        m = m < M ? m : 0;
        px[q] = (int)(m % Wo);
        const int64_t t = m / Wo;
        py[q] = (int)(t % Ho);
        pn[q] = (int)(t / Ho);
    }
    wf32x4 ra[AQ], rx[BQ];
    int64_t ms = mb;  // first pixel of the step being loaded
    auto gload = [&]() {
#pragma unroll
        for (int q = 0; q < AQ; ++q) {
            const int64_t m = ms + ar + ARPP * q;
            ra[q] = (wf32x4){0.f, 0.f, 0.f, 0.f};
            if (m < me && c_ok) ra[q] = *(const wf32x4 *)(dz + m * Co + co0 + 4 * ac);
        }
#pragma unroll
        for (int q = 0; q < BQ; ++q) {
            const int64_t m = ms + br + BRPP * q;
            rx[q] = (wf32x4){0.f, 0.f, 0.f, 0.f};
            if (m < me) {
                const int iy = py[q] * stride - pad + ky * dil, ix = px[q] * stride - pad + kx * dil;
                if (k_ok && iy >= 0 && iy < H && ix >= 0 && ix < W)
                    rx[q] = *(const wf32x4 *)(x + (((int64_t)pn[q] * H + iy) * W + ix) * Ci + ci);
            }
            px[q] += WM_BM;
            while (px[q] >= Wo) {
                px[q] -= Wo;
                if (++py[q] == Ho) {
                    py[q] = 0;
                    ++pn[q];
                }
            }
        }
        ms += WM_BM;
    };
    auto swrite = [&](int buf) {
        float *As = lds + buf * STAGE, *Bs = As + CT * WM_LROW;
#pragma unroll
        for (int q = 0; q < AQ; ++q)
#pragma unroll
            for (int u = 0; u < 4; ++u) As[wsw(4 * ac + u, ar + ARPP * q)] = ra[q][u];
#pragma unroll
        for (int q = 0; q < BQ; ++q)
#pragma unroll
            for (int u = 0; u < 4; ++u) Bs[wsw(4 * bc + u, br + BRPP * q)] = rx[q][u];
    };
    wf32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (wf32x16){0};
    const int nsteps = (int)((me - mb + WM_BM - 1) / WM_BM);
    gload();
    swrite(0);
    __syncthreads();
    const int r32 = lane & 31, h = lane >> 5;
    for (int st = 0; st < nsteps; ++st) {
        const bool more = st + 1 < nsteps;
        if (more) gload();
        const float *As = lds + (NBUF == 2 ? (st & 1) : 0) * STAGE, *Bs = As + CT * WM_LROW;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            wf32x4 fa[TM][2], fb[TN][2];
            const int m0 = h * 16 + half * 8;
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int c = wco * TM * 32 + i * 32 + r32;
                fa[i][0] = *(const wf32x4 *)(As + wsw(c, m0));
                fa[i][1] = *(const wf32x4 *)(As + wsw(c, m0 + 4));
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int c = wk * TN * 32 + j * 32 + r32;
                fb[j][0] = *(const wf32x4 *)(Bs + wsw(c, m0));
                fb[j][1] = *(const wf32x4 *)(Bs + wsw(c, m0 + 4));
            }
#pragma unroll
            for (int p = 0; p < 8; ++p)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][p >> 2][p & 3], fb[j][p >> 2][p & 3],
                                                                         acc[i][j], 0, 0, 0);
        }
        if (NBUF == 2) {  // write the other buffer while slower waves still read this one
            if (more) swrite((st + 1) & 1);
            __syncthreads();
        } else {
            __syncthreads();
            if (more) {
                swrite(0);
                __syncthreads();
            }
        }
    }
    // D[row][col]: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int k = k0 + wk * TN * 32 + j * 32 + r32;
            if (k >= K) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int co = co0 + wco * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (co < Co) atomicAdd(dW + (int64_t)co * K + k, acc[i][j][r]);
            }
        }
}

template <int WCO, int TM, int TN, int NBUF = 1>
int launch_wgrad_mfma(const float *x, const float *dz, int N, int H, int W, int Ci, int Ho, int Wo, int Co, int KW,
                      int K, int stride, int pad, int dil, float *dW, hipStream_t st) {
    constexpr int CT = WCO * TM * 32, KT = (4 / WCO) * TN * 32;
    const int64_t M = (int64_t)N * Ho * Wo;
    const int ct = (Co + CT - 1) / CT, kt = (K + KT - 1) / KT, nt = ct * kt;
    int64_t sp = 1024 / nt + 1;  // >= ~1024 workgroups (2 per CU resident)
    int64_t mc = (M + sp - 1) / sp;
    mc = ((mc + WM_BM - 1) / WM_BM) * WM_BM;
    sp = (M + mc - 1) / mc;
    if (sp * nt >= ((int64_t)1 << 31)) return BEV_ERR_ARGS;
    hipLaunchKernelGGL((k_wgrad_mfma<WCO, TM, TN, NBUF>), dim3((unsigned)(sp * nt)), dim3(256), 0, st, x, dz, N, H, W, Ci,
                       Ho, Wo, Co, KW, K, stride, pad, dil, mc, ct, nt, dW);
    return 0;
}

__global__ __launch_bounds__(256) void k_colsum(const float *__restrict__ dz, int64_t M, int C, int64_t mchunk,
                                                float *__restrict__ db) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const int64_t mb = (int64_t)blockIdx.y * mchunk, me = mb + mchunk < M ? mb + mchunk : M;
    float s = 0.f;
    for (int64_t m = mb; m < me; ++m) s += dz[m * C + c];
    atomicAdd(db + c, s);
}

// db[c] = sum_m dz[m][c] for C % 4 == 0 with C / 4 a power of two <= 256 (ResNet widths): the block's
// 256 threads cover 256 / (C / 4) rows x C columns per step with float4 loads (whole contiguous rows per
// wave instead of one 4-byte column per thread), reduce their row groups in LDS, then one atomic per
// column and block.
__global__ __launch_bounds__(256) void k_colsum_v4(const float *__restrict__ dz, int64_t M, int C, int64_t mchunk,
                                                   float *__restrict__ db) {
    __shared__ float4 part[256];
    const int C4 = C >> 2, G = 256 / C4;
    const int c4 = threadIdx.x % C4, g = threadIdx.x / C4;
    const int64_t mb = (int64_t)blockIdx.x * mchunk, me = mb + mchunk < M ? mb + mchunk : M;
    float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
    int64_t m = mb + g;
    for (; m + G < me; m += 2 * G) {  // two independent load chains
        const float4 a = ((const float4 *)dz)[m * C4 + c4], b = ((const float4 *)dz)[(m + G) * C4 + c4];
        s0.x += a.x, s0.y += a.y, s0.z += a.z, s0.w += a.w;
        s1.x += b.x, s1.y += b.y, s1.z += b.z, s1.w += b.w;
    }
    if (m < me) {
        const float4 a = ((const float4 *)dz)[m * C4 + c4];
        s0.x += a.x, s0.y += a.y, s0.z += a.z, s0.w += a.w;
    }
    part[threadIdx.x] = make_float4(s0.x + s1.x, s0.y + s1.y, s0.z + s1.z, s0.w + s1.w);
    __syncthreads();
    if (g == 0) {
        float4 t = part[c4];
        for (int q = 1; q < G; ++q) {
            const float4 u = part[q * C4 + c4];
            t.x += u.x, t.y += u.y, t.z += u.z, t.w += u.w;
        }
        atomicAdd(db + 4 * c4, t.x);
        atomicAdd(db + 4 * c4 + 1, t.y);
        atomicAdd(db + 4 * c4 + 2, t.z);
        atomicAdd(db + 4 * c4 + 3, t.w);
    }
}

// torch max_pool2d CPU/GPU semantics: the FIRST maximum in window scan order (ky, kx) wins; NaN wins.
__global__ __launch_bounds__(256) void k_maxpool_bwd(const float *__restrict__ x, const float *__restrict__ dy, int N,
                                                     int H, int W, int C, int k, int s, int p, int Ho, int Wo,
                                                     float *__restrict__ dx) {
    const int64_t total = (int64_t)N * H * W * C;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        int64_t t = i / C;
        const int ix = (int)(t % W);
        t /= W;
        const int iy = (int)(t % H);
        const int n = (int)(t / H);
        float g = 0.f;
        // output windows covering (iy, ix): oy*s - p <= iy <= oy*s - p + k - 1
        const int oy_lo = max(0, (iy + p - k + s) / s), oy_hi = min(Ho - 1, (iy + p) / s);
        const int ox_lo = max(0, (ix + p - k + s) / s), ox_hi = min(Wo - 1, (ix + p) / s);
        for (int oy = oy_lo; oy <= oy_hi; ++oy)
            for (int ox = ox_lo; ox <= ox_hi; ++ox) {
                // ATen max_pool2d: maxval = -inf, index = first in-bounds tap; update if (v > maxval || isnan(v))
                int by = -1, bx = -1;
                float best = -__builtin_inff();
                for (int ky = 0; ky < k; ++ky) {
                    const int yy = oy * s - p + ky;
                    if (yy < 0 || yy >= H) continue;
                    for (int kx = 0; kx < k; ++kx) {
                        const int xx = ox * s - p + kx;
                        if (xx < 0 || xx >= W) continue;
                        const float v = x[(((int64_t)n * H + yy) * W + xx) * C + c];
                        if (by < 0) {
                            by = yy;
                            bx = xx;
                        }
                        if (v > best || v != v) {
                            best = v;
                            by = yy;
                            bx = xx;
                        }
                    }
                }
                if (by == iy && bx == ix) g += dy[(((int64_t)n * Ho + oy) * Wo + ox) * C + c];
            }
        dx[i] = g;
    }
}

// Same gather for C % 4 == 0, four channels per thread (float4 loads; the window / index arithmetic
// is shared by the four channels, which the scalar kernel repeats per element).
__global__ __launch_bounds__(256) void k_maxpool_bwd_v4(const float *__restrict__ x, const float *__restrict__ dy,
                                                        int N, int H, int W, int C, int k, int s, int p, int Ho,
                                                        int Wo, float *__restrict__ dx) {
    const int C4 = C >> 2;
    const int64_t total = (int64_t)N * H * W * C4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int c4 = (int)(i % C4);
        int64_t t = i / C4;
        const int ix = (int)(t % W);
        t /= W;
        const int iy = (int)(t % H);
        const int n = (int)(t / H);
        float g[4] = {0.f, 0.f, 0.f, 0.f};
        const int oy_lo = max(0, (iy + p - k + s) / s), oy_hi = min(Ho - 1, (iy + p) / s);
        const int ox_lo = max(0, (ix + p - k + s) / s), ox_hi = min(Wo - 1, (ix + p) / s);
        for (int oy = oy_lo; oy <= oy_hi; ++oy)
            for (int ox = ox_lo; ox <= ox_hi; ++ox) {
                int by[4] = {-1, -1, -1, -1}, bx[4] = {-1, -1, -1, -1};
                float best[4] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
                for (int ky = 0; ky < k; ++ky) {
                    const int yy = oy * s - p + ky;
                    if (yy < 0 || yy >= H) continue;
                    for (int kx = 0; kx < k; ++kx) {
                        const int xx = ox * s - p + kx;
                        if (xx < 0 || xx >= W) continue;
                        const float4 q = ((const float4 *)x)[(((int64_t)n * H + yy) * W + xx) * C4 + c4];
                        const float v[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            if (by[u] < 0) {
                                by[u] = yy;
                                bx[u] = xx;
                            }
                            if (v[u] > best[u] || v[u] != v[u]) {
                                best[u] = v[u];
                                by[u] = yy;
                                bx[u] = xx;
                            }
                        }
                    }
                }
                const bool hit = (by[0] == iy && bx[0] == ix) || (by[1] == iy && bx[1] == ix) ||
                                 (by[2] == iy && bx[2] == ix) || (by[3] == iy && bx[3] == ix);
                if (hit) {
                    const float4 d = ((const float4 *)dy)[(((int64_t)n * Ho + oy) * Wo + ox) * C4 + c4];
                    const float dv[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (by[u] == iy && bx[u] == ix) g[u] += dv[u];
                }
            }
        ((float4 *)dx)[i] = make_float4(g[0], g[1], g[2], g[3]);
    }
}

inline unsigned grid_for(int64_t n) {
    const int64_t b = (n + 255) / 256;
    return (unsigned)(b < 256 * 64 ? (b > 0 ? b : 1) : 256 * 64);
}

// Two-pass max-pool backward for C % 4 == 0 (the trunk's 3x3 / 2 stem pool): k_maxpool_argmax_v4 scans every window
// once with k_maxpool_bwd_v4's rule (first valid tap, then v > best or v NaN) and stores the winning tap ky * k + kx
// per (output, channel) as one byte; k_maxpool_bwd_idx_v4 gathers, per input, dy of the windows whose byte names it,
// in the same (oy, ox) order -- bit-identical to k_maxpool_bwd_v4, which re-scans every covering window per input
// (4 windows x 9 taps of float4 loads per input for 3x3 / 2, against 2.25 here).
__global__ __launch_bounds__(256) void k_maxpool_argmax_v4(const float *__restrict__ x, int N, int H, int W, int C,
                                                           int k, int s, int p, int Ho, int Wo,
                                                           uchar4 *__restrict__ arg) {
    const int C4 = C >> 2;
    const int64_t total = (int64_t)N * Ho * Wo * C4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int c4 = (int)(i % C4);
        int64_t t = i / C4;
        const int ox = (int)(t % Wo);
        t /= Wo;
        const int oy = (int)(t % Ho);
        const int n = (int)(t / Ho);
        int bi[4] = {-1, -1, -1, -1};
        float best[4] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
        for (int ky = 0; ky < k; ++ky) {
            const int yy = oy * s - p + ky;
            if (yy < 0 || yy >= H) continue;
            for (int kx = 0; kx < k; ++kx) {
                const int xx = ox * s - p + kx;
                if (xx < 0 || xx >= W) continue;
                const float4 q = ((const float4 *)x)[(((int64_t)n * H + yy) * W + xx) * C4 + c4];
                const float v[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (bi[u] < 0) bi[u] = ky * k + kx;
                    if (v[u] > best[u] || v[u] != v[u]) {
                        best[u] = v[u];
                        bi[u] = ky * k + kx;
                    }
                }
            }
        }
        arg[i] = make_uchar4((unsigned char)bi[0], (unsigned char)bi[1], (unsigned char)bi[2], (unsigned char)bi[3]);
    }
}

__global__ __launch_bounds__(256) void k_maxpool_bwd_idx_v4(const uchar4 *__restrict__ arg,
                                                            const float *__restrict__ dy, int N, int H, int W, int C,
                                                            int k, int s, int p, int Ho, int Wo,
                                                            float *__restrict__ dx) {
    const int C4 = C >> 2;
    const int64_t total = (int64_t)N * H * W * C4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int c4 = (int)(i % C4);
        int64_t t = i / C4;
        const int ix = (int)(t % W);
        t /= W;
        const int iy = (int)(t % H);
        const int n = (int)(t / H);
        float g[4] = {0.f, 0.f, 0.f, 0.f};
        const int oy_lo = max(0, (iy + p - k + s) / s), oy_hi = min(Ho - 1, (iy + p) / s);
        const int ox_lo = max(0, (ix + p - k + s) / s), ox_hi = min(Wo - 1, (ix + p) / s);
        for (int oy = oy_lo; oy <= oy_hi; ++oy)
            for (int ox = ox_lo; ox <= ox_hi; ++ox) {
                const int me = (iy - (oy * s - p)) * k + (ix - (ox * s - p));
                const int64_t o = (((int64_t)n * Ho + oy) * Wo + ox) * C4 + c4;
                const uchar4 a = arg[o];
                const bool h0 = a.x == me, h1 = a.y == me, h2 = a.z == me, h3 = a.w == me;
                if (h0 || h1 || h2 || h3) {
                    const float4 d = ((const float4 *)dy)[o];
                    if (h0) g[0] += d.x;
                    if (h1) g[1] += d.y;
                    if (h2) g[2] += d.z;
                    if (h3) g[3] += d.w;
                }
            }
        ((float4 *)dx)[i] = make_float4(g[0], g[1], g[2], g[3]);
    }
}

// Training forward max-pool that also keeps the backward's window argmax bytes (C % 4 == 0): one float4 of channels
// per thread on a (row piece, output row, image) grid with 32-bit indices; the pooled value by k_maxpool_rows' rule
// and the winning tap by k_maxpool_argmax_v4's (the same comparisons: first valid tap, then v > best or v NaN), so
// the backward's argmax pass over the input disappears.
__global__ __launch_bounds__(256) void k_maxpool_fwd_arg_v4(const float4 *__restrict__ x, int H, int W, int CV, int k,
                                                            int s, int p, float4 *__restrict__ y,
                                                            uchar4 *__restrict__ arg, int Ho, int Wo) {
    const int oy = blockIdx.y, n = blockIdx.z;
    const int t = blockIdx.x * 256 + threadIdx.x;  // (ox, c4) within the output row
    if (t >= Wo * CV) return;
    const int ox = t / CV, c = t - ox * CV;
    float best[4] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
    int bi[4] = {-1, -1, -1, -1};
    const int iy0 = oy * s - p, ix0 = ox * s - p;
    for (int ky = 0; ky < k; ++ky) {
        const int iy = iy0 + ky;
        if (iy < 0 || iy >= H) continue;
        const float4 *row = x + ((size_t)n * H + iy) * (size_t)W * CV + c;
        for (int kx = 0; kx < k; ++kx) {
            const int ix = ix0 + kx;
            if (ix < 0 || ix >= W) continue;
            const float4 q = row[(size_t)ix * CV];
            const float v[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (bi[u] < 0) bi[u] = ky * k + kx;
                if (v[u] > best[u] || v[u] != v[u]) {
                    best[u] = v[u];
                    bi[u] = ky * k + kx;
                }
            }
        }
    }
    const size_t o = ((size_t)n * Ho + oy) * (size_t)Wo * CV + t;
    y[o] = make_float4(best[0], best[1], best[2], best[3]);
    arg[o] = make_uchar4((unsigned char)bi[0], (unsigned char)bi[1], (unsigned char)bi[2], (unsigned char)bi[3]);
}

// k_maxpool_bwd_idx_v4 on an (input row piece, input row, image) grid with 32-bit indices; same windows in the
// same (oy, ox) order: bit-identical.  W2 (windows per axis <= 2, e.g. 3x3 / 2): the up to 2 x 2 covering windows'
// argmax bytes and dy are all loaded up front (dy unconditionally, from L2), so a thread waits for memory once
// instead of twice per window (the looped form ran at ~2.3 TB/s, latency-bound).
template <bool W2>
__global__ __launch_bounds__(256) void k_maxpool_bwd_arg_v4(const uchar4 *__restrict__ arg,
                                                            const float4 *__restrict__ dy, int H, int W, int CV, int k,
                                                            int s, int p, int Ho, int Wo, float4 *__restrict__ dx) {
    const int iy = blockIdx.y, n = blockIdx.z;
    const int t = blockIdx.x * 256 + threadIdx.x;  // (ix, c4) within the input row
    if (t >= W * CV) return;
    const int ix = t / CV, c = t - ix * CV;
    float g[4] = {0.f, 0.f, 0.f, 0.f};
    const int oy_lo = max(0, (iy + p - k + s) / s), oy_hi = min(Ho - 1, (iy + p) / s);
    const int ox_lo = max(0, (ix + p - k + s) / s), ox_hi = min(Wo - 1, (ix + p) / s);
    if constexpr (W2) {
        uchar4 a[2][2];
        float4 d[2][2];
        bool ok[2][2];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int v = 0; v < 2; ++v) {
                const int oy = oy_lo + u, ox = ox_lo + v;
                ok[u][v] = oy <= oy_hi && ox <= ox_hi;
                const size_t o = ((size_t)n * Ho + (ok[u][v] ? oy : min(oy_lo, Ho - 1))) * (size_t)Wo * CV +
                                 (size_t)(ok[u][v] ? ox : min(ox_lo, Wo - 1)) * CV + c;  // any in-range address
                a[u][v] = arg[o];
                d[u][v] = dy[o];
            }
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int v = 0; v < 2; ++v) {
                const int me = (iy - ((oy_lo + u) * s - p)) * k + (ix - ((ox_lo + v) * s - p));
                if (!ok[u][v]) continue;
                if (a[u][v].x == me) g[0] += d[u][v].x;
                if (a[u][v].y == me) g[1] += d[u][v].y;
                if (a[u][v].z == me) g[2] += d[u][v].z;
                if (a[u][v].w == me) g[3] += d[u][v].w;
            }
        dx[((size_t)n * H + iy) * (size_t)W * CV + t] = make_float4(g[0], g[1], g[2], g[3]);
        return;
    }
    for (int oy = oy_lo; oy <= oy_hi; ++oy)
        for (int ox = ox_lo; ox <= ox_hi; ++ox) {
            const int me = (iy - (oy * s - p)) * k + (ix - (ox * s - p));
            const size_t o = ((size_t)n * Ho + oy) * (size_t)Wo * CV + (size_t)ox * CV + c;
            const uchar4 a = arg[o];
            const bool h0 = a.x == me, h1 = a.y == me, h2 = a.z == me, h3 = a.w == me;
            if (h0 || h1 || h2 || h3) {
                const float4 d = dy[o];
                if (h0) g[0] += d.x;
                if (h1) g[1] += d.y;
                if (h2) g[2] += d.z;
                if (h3) g[3] += d.w;
            }
        }
    dx[((size_t)n * H + iy) * (size_t)W * CV + t] = make_float4(g[0], g[1], g[2], g[3]);
}

}  // namespace

extern "C" {

int bev_maxpool2d_fwd_arg_nhwc_f32(const float *x, int N, int H, int W, int C, int k, int stride, int pad, float *y,
                                   uint8_t *argmax, int Ho, int Wo, void *stream) {
    if (!x || !y || !argmax || N < 0 || H <= 0 || W <= 0 || C <= 0 || C % 4 != 0 || k <= 0 || k * k > 255 ||
        stride <= 0 || pad < 0 || N >= 65536 || Ho >= 65536)
        return BEV_ERR_ARGS;
    if (Ho != (H + 2 * pad - k) / stride + 1 || Wo != (W + 2 * pad - k) / stride + 1 || Ho <= 0 || Wo <= 0)
        return BEV_ERR_ARGS;
    if ((((uintptr_t)x | (uintptr_t)y) & 15) != 0 || ((uintptr_t)argmax & 3) != 0) return BEV_ERR_ARGS;
    if ((int64_t)Wo * (C / 4) >= (1ll << 30)) return BEV_ERR_ARGS;
    if (N == 0) return 0;
    hipLaunchKernelGGL(k_maxpool_fwd_arg_v4, dim3((unsigned)(((int64_t)Wo * (C / 4) + 255) / 256), Ho, N), dim3(256), 0,
                       (hipStream_t)stream, reinterpret_cast<const float4 *>(x), H, W, C / 4, k, stride, pad,
                       reinterpret_cast<float4 *>(y), reinterpret_cast<uchar4 *>(argmax), Ho, Wo);
    return last();
}

int bev_maxpool2d_bwd_arg_nhwc_f32(const uint8_t *argmax, const float *dy, int N, int H, int W, int C, int k,
                                   int stride, int pad, int Ho, int Wo, float *dx, void *stream) {
    if (!argmax || !dy || !dx || N < 0 || H <= 0 || W <= 0 || C <= 0 || C % 4 != 0 || k <= 0 || k * k > 255 ||
        stride <= 0 || pad < 0 || N >= 65536 || H >= 65536)
        return BEV_ERR_ARGS;
    if (Ho != (H + 2 * pad - k) / stride + 1 || Wo != (W + 2 * pad - k) / stride + 1 || Ho <= 0 || Wo <= 0)
        return BEV_ERR_ARGS;
    if ((((uintptr_t)dy | (uintptr_t)dx) & 15) != 0 || ((uintptr_t)argmax & 3) != 0) return BEV_ERR_ARGS;
    if ((int64_t)W * (C / 4) >= (1ll << 30)) return BEV_ERR_ARGS;
    if (N == 0) return 0;
    const bool w2 = (k + stride - 1) / stride <= 2;  // covering windows per axis
    hipLaunchKernelGGL(w2 ? k_maxpool_bwd_arg_v4<true> : k_maxpool_bwd_arg_v4<false>,
                       dim3((unsigned)(((int64_t)W * (C / 4) + 255) / 256), H, N), dim3(256), 0,
                       (hipStream_t)stream, reinterpret_cast<const uchar4 *>(argmax),
                       reinterpret_cast<const float4 *>(dy), H, W, C / 4, k, stride, pad, Ho, Wo,
                       reinterpret_cast<float4 *>(dx));
    return last();
}

int bev_relu_bwd_f32(const float *dy, const float *y, float *dz, int64_t n, void *stream) {
    if (!dy || !y || !dz || n < 0 || n % 4 != 0) return BEV_ERR_ARGS;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_relu_bwd, dim3(grid_for(n / 4)), dim3(256), 0, (hipStream_t)stream, dy, y, dz, n / 4);
    return last();
}

int bev_dilate_nhwc_ex(const void *dz, int elem_bytes, int N, int Ho, int Wo, int C, int s, int top, int left, int Hd,
                       int Wd, void *out, void *stream) {
    if (!dz || !out || N < 0 || Ho <= 0 || Wo <= 0 || C <= 0 || C % 4 != 0 || s <= 0 || top < 0 || left < 0 ||
        top + s * (Ho - 1) >= Hd || left + s * (Wo - 1) >= Wd || (elem_bytes != 4 && elem_bytes != 2))
        return BEV_ERR_ARGS;
    const int64_t total = (int64_t)N * Hd * Wd * (C / 4);
    if (total == 0) return 0;
    if (elem_bytes == 4)
        hipLaunchKernelGGL(k_dilate<float4>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream,
                           (const float4 *)dz, N, Ho, Wo, C, s, top, left, Hd, Wd, (float4 *)out);
    else
        hipLaunchKernelGGL(k_dilate<uint2>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream,
                           (const uint2 *)dz, N, Ho, Wo, C, s, top, left, Hd, Wd, (uint2 *)out);
    return last();
}

int bev_place_strided_f32(const float *y, int N, int Ho, int Wo, int C, int s, int H, int W, const float *residual,
                          float *out, void *stream) {
    if (!y || !out || N <= 0 || N > 65535 || Ho <= 0 || Wo <= 0 || C <= 0 || C % 4 != 0 || 256 % (C / 4) != 0 ||
        s <= 0 || s * (Ho - 1) >= H || s * (Wo - 1) >= W ||
        (((uintptr_t)y | (uintptr_t)out | (uintptr_t)residual) & 15) != 0)
        return BEV_ERR_ARGS;
    const dim3 grid((unsigned)(((int64_t)H * W + 255) / 256), N);
    hipLaunchKernelGGL(k_place_strided, grid, dim3(256), 0, (hipStream_t)stream, (const float4 *)y, Ho, Wo, C / 4, s,
                       H, W, (const float4 *)residual, (float4 *)out);
    return last();
}

int bev_dilate_nhwc_f32(const float *dz, int N, int Ho, int Wo, int C, int s, int top, int left, int Hd, int Wd,
                        float *out, void *stream) {
    return bev_dilate_nhwc_ex(dz, 4, N, Ho, Wo, C, s, top, left, Hd, Wd, out, stream);
}

int bev_conv_wgrad_f32(const float *x, int N, int H, int W, int Ci, const float *dz, int Ho, int Wo, int Co, int KH,
                       int KW, int stride, int pad, float *dW, void *stream) {
    return bev_conv_wgrad_ex_f32(x, N, H, W, Ci, dz, Ho, Wo, Co, KH, KW, stride, pad, 1, dW, stream);
}

int bev_conv_wgrad_ex_f32(const float *x, int N, int H, int W, int Ci, const float *dz, int Ho, int Wo, int Co, int KH,
                          int KW, int stride, int pad, int dilation, float *dW, void *stream) {
    if (!x || !dz || !dW || N < 0 || H <= 0 || W <= 0 || Ci <= 0 || Co <= 0 || KH <= 0 || KW <= 0 || stride <= 0 ||
        pad < 0 || dilation <= 0)
        return BEV_ERR_ARGS;
    const int dil = dilation;
    if (Ho != (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1 || Wo != (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1)
        return BEV_ERR_ARGS;
    const int K = KH * KW * Ci;
    const int64_t M = (int64_t)N * Ho * Wo;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(dW, 0, (size_t)Co * K * sizeof(float), st) != hipSuccess) return last();
    if (M == 0) return 0;
    const int gx = (K + WG_T - 1) / WG_T, gy = (Co + WG_T - 1) / WG_T;
    int64_t splits = 2048 / ((int64_t)gx * gy) + 1;  // >= ~2048 workgroups
    int64_t mchunk = (M + splits - 1) / splits;
    mchunk = ((mchunk + WG_M - 1) / WG_M) * WG_M;
    splits = (M + mchunk - 1) / mchunk;
    if (splits > 65535) return BEV_ERR_ARGS;
    if (Ci % 4 == 0 && Co % 4 == 0 && g_wgrad_mfma) {
        // tile shape by the narrow dimension: 32 x 512 (Co <= 32), 64 x 256 (Co <= 64), 256 x 64 (K <= 64),
        // else 128 x 128
        int rc;
        if (g_wgrad_mfma == 2) {
            if (Co <= 32)
                rc = launch_wgrad_nat<1, 1, 4>(x, dz, N, H, W, Ci, Ho, Wo, Co, KW, K, stride, pad, dil, dW, st);
            else if (Co <= 64)
                rc = launch_wgrad_nat<1, 2, 2>(x, dz, N, H, W, Ci, Ho, Wo, Co, KW, K, stride, pad, dil, dW, st);
            else if (K <= 64)
                rc = launch_wgrad_nat<4, 2, 2>(x, dz, N, H, W, Ci, Ho, Wo, Co, KW, K, stride, pad, dil, dW, st);
            else
                rc = launch_wgrad_nat<2, 2, 2>(x, dz, N, H, W, Ci, Ho, Wo, Co, KW, K, stride, pad, dil, dW, st);
        } else if (Co <= 32)
            rc = launch_wgrad_mfma<1, 1, 4>(x, dz, N, H, W, Ci, Ho, Wo, Co, KW, K, stride, pad, dil, dW, st);
        else if (Co <= 64)
            rc = launch_wgrad_mfma<1, 2, 2>(x, dz, N, H, W, Ci, Ho, Wo, Co, KW, K, stride, pad, dil, dW, st);
        else if (K <= 64)
            rc = launch_wgrad_mfma<4, 2, 2>(x, dz, N, H, W, Ci, Ho, Wo, Co, KW, K, stride, pad, dil, dW, st);
        else
            rc = launch_wgrad_mfma<2, 2, 2, 2>(x, dz, N, H, W, Ci, Ho, Wo, Co, KW, K, stride, pad, dil, dW, st);
        if (rc) return rc;
    } else if (Ci % 4 == 0 && Co % 4 == 0)
        hipLaunchKernelGGL(k_wgrad_v4, dim3(gx, gy, (unsigned)splits), dim3(256), 0, st, x, dz, N, H, W, Ci, Ho, Wo,
                           Co, KW, K, stride, pad, dil, mchunk, dW);
    else
        hipLaunchKernelGGL(k_wgrad, dim3(gx, gy, (unsigned)splits), dim3(256), 0, st, x, dz, N, H, W, Ci, Ho, Wo, Co,
                           KH, KW, stride, pad, dil, mchunk, dW);
    return last();
}

int bev_colsum_f32(const float *dz, int64_t M, int C, float *db, void *stream) {
    if (!dz || !db || M < 0 || C <= 0) return BEV_ERR_ARGS;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(db, 0, (size_t)C * sizeof(float), st) != hipSuccess) return last();
    if (M == 0) return 0;
    const int C4 = C / 4;
    if (C % 4 == 0 && C4 <= 256 && (C4 & (C4 - 1)) == 0) {
        const int64_t splits = M < 4096 ? 1 : 2048;
        const int64_t mchunk = (M + splits - 1) / splits;
        hipLaunchKernelGGL(k_colsum_v4, dim3((unsigned)((M + mchunk - 1) / mchunk)), dim3(256), 0, st, dz, M, C,
                           mchunk, db);
        return last();
    }
    const int64_t splits = M < 1024 ? 1 : 1024;
    const int64_t mchunk = (M + splits - 1) / splits;
    hipLaunchKernelGGL(k_colsum, dim3((C + 255) / 256, (unsigned)((M + mchunk - 1) / mchunk)), dim3(256), 0, st, dz,
                       M, C, mchunk, db);
    return last();
}

int bev_maxpool2d_bwd_nhwc_f32(const float *x, const float *dy, int N, int H, int W, int C, int k, int stride, int pad,
                               int Ho, int Wo, float *dx, void *stream) {
    if (!x || !dy || !dx || N < 0 || H <= 0 || W <= 0 || C <= 0 || k <= 0 || stride <= 0 || pad < 0) return BEV_ERR_ARGS;
    if (Ho != (H + 2 * pad - k) / stride + 1 || Wo != (W + 2 * pad - k) / stride + 1) return BEV_ERR_ARGS;
    const int64_t total = (int64_t)N * H * W * C;
    if (total == 0) return 0;
    if (C % 4 == 0)
        hipLaunchKernelGGL(k_maxpool_bwd_v4, dim3(grid_for(total / 4)), dim3(256), 0, (hipStream_t)stream, x, dy, N, H,
                           W, C, k, stride, pad, Ho, Wo, dx);
    else
        hipLaunchKernelGGL(k_maxpool_bwd, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, x, dy, N, H, W, C,
                           k, stride, pad, Ho, Wo, dx);
    return last();
}

int bev_maxpool2d_bwd_ws_nhwc_f32(const float *x, const float *dy, int N, int H, int W, int C, int k, int stride,
                                  int pad, int Ho, int Wo, float *dx, uint8_t *argmax, void *stream) {
    if (!x || !dy || !dx || !argmax || N < 0 || H <= 0 || W <= 0 || C <= 0 || C % 4 != 0 || k <= 0 || k * k > 255 ||
        stride <= 0 || pad < 0)
        return BEV_ERR_ARGS;
    if (Ho != (H + 2 * pad - k) / stride + 1 || Wo != (W + 2 * pad - k) / stride + 1 || Ho <= 0 || Wo <= 0)
        return BEV_ERR_ARGS;
    if ((((uintptr_t)x | (uintptr_t)dy | (uintptr_t)dx) & 15) != 0 || ((uintptr_t)argmax & 3) != 0) return BEV_ERR_ARGS;
    const int64_t total = (int64_t)N * H * W * C;
    if (total == 0) return 0;
    const int64_t outs = (int64_t)N * Ho * Wo * C;
    hipLaunchKernelGGL(k_maxpool_argmax_v4, dim3(grid_for(outs / 4)), dim3(256), 0, (hipStream_t)stream, x, N, H, W, C,
                       k, stride, pad, Ho, Wo, (uchar4 *)argmax);
    hipLaunchKernelGGL(k_maxpool_bwd_idx_v4, dim3(grid_for(total / 4)), dim3(256), 0, (hipStream_t)stream,
                       (const uchar4 *)argmax, dy, N, H, W, C, k, stride, pad, Ho, Wo, dx);
    return last();
}

}  // extern "C"

namespace bev {
int train_tune(int knob, int value) {
    if (knob != BEV_TUNE_WGRAD_MFMA || value < 0 || value > 2) return BEV_ERR_ARGS;
    const int old = g_wgrad_mfma;
    g_wgrad_mfma = value;
    return old;
}
}  // namespace bev
