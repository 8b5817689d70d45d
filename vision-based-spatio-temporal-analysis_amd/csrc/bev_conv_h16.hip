// bev_conv_h16.hip -- the convolutions of a training step under torch.autocast(float16) (BASELINE config 3).
//
// The reference trains with RUNTIME.USE_AMP: true (configs/wildtrack.yaml:45): inside
// autocast(dtype=float16) (train.py:238-247) every nn.Conv2d of the timm trunk and of BEVDetector runs on fp16
// operands (autocast rounds the fp32 activation and the fp32 weight to fp16, round-to-nearest-even) with fp32
// accumulation, forward and backward.  This kernel is that arithmetic on the MI355X matrix cores:
//     y[m][n] = act( sum_k f16(A[m][k]) * f16(W[k][n]) + bias[n] (+ res[m][n]) )     (fp32 sum)
// on v_mfma_f32_32x32x16_f16 (16x the fp32 MFMA rate; the products of two fp16 values are exact in fp32, so the
// result equals an fp32 convolution of the fp16-rounded operands up to the order of the fp32 additions).
// Activations stay fp32 NHWC in HBM (the BatchNorm / GroupNorm / loss kernels around the convs run in fp32, as
// under autocast); A is converted to fp16 as it is staged into LDS, the weights are packed to fp16 once.
//
// Implicit GEMM, m = (image, oy, ox), n = output channel, k = (ky, kx, ci) with Ci % 32 == 0 (one tap and 32
// consecutive channels per K step).  256 threads = 2 x 2 waves of 64 x 64 outputs (2 x 2 MFMA tiles of 32 x 32),
// block tile 128 x 128, K step 32 (two 16-deep MFMA k-slices), operands [row][k] in LDS with 80-B rows (5 odd
// 16-B slots: conflict-free ds_read_b128 fragments), double-buffered: the next step's global loads are issued
// before this step's MFMAs.  Fragment map (cdna_hip_programming.md §3): lane l holds A[row l & 31][k 8 (l >> 5)
// + j] and B[k 8 (l >> 5) + j][col l & 31], j = 0..7.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bev_mi355x.h"
#include "bev_act.h"

namespace {

typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));  // native vector: stays in VGPRs (uint4 arrays went to scratch)

constexpr int HBM = 128, HBN = 128, HBK = 32;
int g_h16_kernel = 0;  // BEV_TUNE_CONV_H16_KERNEL: 0 = k_conv_h16b where Ci % 64 == 0 and k_wgrad_h16b, 1 = k_conv_h16
                       // and k_wgrad_h16 always
constexpr int HROW = 40;  // halves per LDS row: 32 + 8 pad = 80 B = 5 slots (odd: 16 rows -> 16 distinct slots)

__device__ __attribute__((aligned(16))) float g_hzero4[4] = {0.f, 0.f, 0.f, 0.f};  // never written

__host__ __device__ inline int64_t kpad_h(int K) { return (K + HBK - 1) / HBK * HBK; }
__host__ __device__ inline int64_t copad_h(int Co) { return (Co + HBN - 1) / HBN * HBN; }

// OIHW fp32 -> [Co_pad][K_pad] fp16 (RNE, like autocast's weight cast), k = (ky*KW + kx)*Ci + ci
__global__ void k_pack_h16(const float *__restrict__ w, int Co, int Ci, int KH, int KW, int64_t Kp, int64_t Cop,
                           _Float16 *__restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= Kp * Cop) return;
    const int n = (int)(t / Kp);
    const int k = (int)(t % Kp);
    const int K = Ci * KH * KW;
    float v = 0.0f;
    if (n < Co && k < K) {
        const int ci = k % Ci, r = k / Ci, kx = r % KW, ky = r / KW;
        v = w[(((int64_t)n * Ci + ci) * KH + ky) * KW + kx];
    }
    out[t] = (_Float16)v;
}

struct ConvH {
    const float *__restrict__ x;
    const _Float16 *__restrict__ xh;  // k_conv_h16b<true>: the operand stored in fp16 (what the kernel rounds x to)
    const _Float16 *__restrict__ wp;
    const float *__restrict__ bias;
    const float *__restrict__ res;
    float *__restrict__ y;
    float *__restrict__ stats;  // k_conv_h16b: per (row tile, channel) BatchNorm partials (sum, M2) of the output, or null
    int N, H, W, Ci, Co, KH, KW, stride, pad, dil, Ho, Wo, act, ldy, Kp;
    int64_t M;
};

__device__ __forceinline__ float act_h(float t, int act) {
    if (act == 2) return silu_hw(t);
    if (act == 1) return t > 0.0f ? t : 0.0f;
    return t;
}

__global__ __launch_bounds__(256, 2) void k_conv_h16(ConvH a) {
    __shared__ __attribute__((aligned(16))) _Float16 lds[2][(HBM + HBN) * HROW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int ntn = (a.Co + HBN - 1) / HBN;
    const int64_t ntm = (a.M + HBM - 1) / HBM;
    unsigned bid = blockIdx.x;
    {  // XCD-aware order: consecutive blocks (the N tiles of one M block) on one XCD
        const unsigned nb = gridDim.x, q = nb / 8, r = nb % 8, xc = bid % 8;
        bid = (xc < r ? xc * (q + 1) : r * (q + 1) + (xc - r) * q) + bid / 8;
    }
    const int64_t mt = bid / (unsigned)ntn;
    const int nt = (int)(bid % (unsigned)ntn);
    if (mt >= ntm) return;
    const int64_t m0 = mt * HBM;
    const int n0 = nt * HBN;

    // A staging: rows (tid >> 3) + 32 q, channel quad tid & 7 (4 channels -> 4 halves)
    const int aq = tid & 7;
    int64_t pix[4];
    int iy0[4], ix0[4];
    bool rok[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t m = m0 + (tid >> 3) + 32 * q;
        rok[q] = m < a.M;
        const int64_t mm = rok[q] ? m : 0;
        const int ox = (int)(mm % a.Wo);
        const int64_t t = mm / a.Wo;
        const int oy = (int)(t % a.Ho);
        const int n = (int)(t / a.Ho);
        pix[q] = (int64_t)n * a.H * a.W * a.Ci;
        iy0[q] = oy * a.stride - a.pad;
        ix0[q] = ox * a.stride - a.pad;
    }
    // B staging: weight row n0 + (tid >> 1), halves 16 (tid & 1) .. + 15 of the K step
    const _Float16 *wrow = a.wp + (int64_t)(n0 + (tid >> 1)) * a.Kp + 16 * (tid & 1);

    f32x4 ra[4];
    u32x4 rb[2];
    int ky = 0, kx = 0, ci0 = 0;  // tap and channel offset of the K step being loaded
    int64_t kb = 0;
    auto gload = [&]() {
        const int dy = ky * a.dil, dx = kx * a.dil;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int iy = iy0[q] + dy, ix = ix0[q] + dx;
            const bool in = rok[q] && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
            const float *src = in ? a.x + pix[q] + ((int64_t)iy * a.W + ix) * a.Ci + ci0 + 4 * aq : g_hzero4;
            ra[q] = *(const f32x4 *)src;
        }
        rb[0] = *(const u32x4 *)(wrow + kb);
        rb[1] = *(const u32x4 *)(wrow + kb + 8);
        kb += HBK;
        ci0 += HBK;
        if (ci0 == a.Ci) {
            ci0 = 0;
            if (++kx == a.KW) {
                kx = 0;
                ++ky;
            }
        }
    };
    auto swrite = [&](int buf) {
        _Float16 *As = lds[buf], *Bs = As + HBM * HROW;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const h16x4 h = {(_Float16)ra[q][0], (_Float16)ra[q][1], (_Float16)ra[q][2], (_Float16)ra[q][3]};
            *(h16x4 *)(As + ((tid >> 3) + 32 * q) * HROW + 4 * aq) = h;
        }
        *(u32x4 *)(Bs + (tid >> 1) * HROW + 16 * (tid & 1)) = rb[0];
        *(u32x4 *)(Bs + (tid >> 1) * HROW + 16 * (tid & 1) + 8) = rb[1];
    };

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = (f32x16){0};
    const int nsteps = a.Kp / HBK;
    gload();
    swrite(0);
    __syncthreads();
    const int r32 = lane & 31, h = lane >> 5;
    for (int st = 0; st < nsteps; ++st) {
        const bool more = st + 1 < nsteps;
        if (more) gload();
        const _Float16 *As = lds[st & 1], *Bs = As + HBM * HROW;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            h16x8 fa[2], fb[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) fa[i] = *(const h16x8 *)(As + (wm * 64 + i * 32 + r32) * HROW + kk * 16 + 8 * h);
#pragma unroll
            for (int j = 0; j < 2; ++j) fb[j] = *(const h16x8 *)(Bs + (wn * 64 + j * 32 + r32) * HROW + kk * 16 + 8 * h);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
        if (more) swrite((st + 1) & 1);  // the other buffer: its last readers passed the previous barrier
        __syncthreads();
    }
    // D[row][col]: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int col = n0 + wn * 64 + j * 32 + r32;
            if (col >= a.Co) continue;
            const float bv = a.bias ? a.bias[col] : 0.0f;
            float rv[16];  // all residual loads first: interleaved with the stores they would serialise (y may alias)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                rv[r] = (a.res && row < a.M) ? a.res[row * a.Co + col] : 0.0f;
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (row >= a.M) continue;
                float v = acc[i][j][r] + bv;
                if (a.res) v += rv[r];
                a.y[row * a.ldy + col] = act_h(v, a.act);
            }
        }
}

// ---- k_conv_h16b: Ci % 64 == 0 (the ResNet trunk) -----------------------------------------------------------------
// k_conv_h16's K step of 32 gives each wave only 8 MFMAs (256 cycles) per barrier and prefetches one step ahead, so
// the global-load latency is exposed.  Here a K step is 64 deep (one tap, 64 channels: 16 MFMAs per wave and step)
// and the operands of steps s + 1 and s + 2 are in flight in two register sets while step s runs (ping-pong, two
// steps per trip, no copies).  Same fragment map, same per-output K order (16-deep slices in increasing k): results
// identical to k_conv_h16.
constexpr int HBK2 = 64, HROW2 = 72;
// H16B_LINES 1: the fp16 operand and the weight panel are staged with eight lanes per 128-B K-step row, so every
// wave load instruction reads whole lines (round 5); 0: the round-4 maps (4 / 2 lanes per row, 32-64 B pieces).
#ifndef H16B_LINES
#define H16B_LINES 1
#endif
#ifndef H16B_BUF
#define H16B_BUF 1
#endif  // halves per LDS row: 64 + 8 pad = 144 B = 9 odd 16-B slots

// BatchNorm statistics of the conv output z = acc + bias (training forward, BN with batch statistics), fused into
// the epilogue so z is not read back: per output column of the 128 x 128 tile, over the tile's valid rows,
// (sum, M2 = sum (z - sum / n)^2) in fp32 -> stats[col][row tile][2] (channel-major: the finalize reads each
// channel's tiles contiguously); bev_batchnorm_finalize_tiles_f32 combines the tiles in double.  Two-pass around the tile mean, so the variance
// has no E[z^2] - E[z]^2 cancellation.  Column col = n0 + wn 64 + j 32 + r32 is held by 32 rows of each lane,
// the lane pair (h = 0, 1) and the two wm waves: lane sums, one xor-32 exchange, one LDS exchange.
template <int BN, int TI>
__device__ __forceinline__ void h16_tile_stats(const ConvH &a, const f32x16 (&acc)[TI][2], _Float16 *ldsh, int64_t m0,
                                               int n0, int wm, int wn, int r32, int h) {
    constexpr int NRW = BN == 128 ? 2 : 4, WROWS = BN == 128 ? 64 : 32;  // row-waves sharing a column, rows each
    float *red = reinterpret_cast<float *>(ldsh);  // [NRW][BN cols]
    const int64_t nv64 = a.M - m0;
    const int nv = nv64 < HBM ? (int)nv64 : HBM;
    float mean[2], sum[2];
    __syncthreads();  // the last K step's fragment reads of this buffer are done
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int c = wn * 64 + j * 32 + r32;
        const float bv = (a.bias && n0 + c < a.Co) ? a.bias[n0 + c] : 0.0f;
        float s = 0.0f;
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = wm * WROWS + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (row < nv) s += acc[i][j][r] + bv;
            }
        s += __shfl_xor(s, 32);
        if (h == 0) red[wm * BN + c] = s;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int c = wn * 64 + j * 32 + r32;
        float t = 0.0f;
#pragma unroll
        for (int w = 0; w < NRW; ++w) t += red[w * BN + c];
        sum[j] = t;
        mean[j] = sum[j] / (float)nv;
    }
    __syncthreads();  // sums consumed before the M2 exchange reuses red
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int c = wn * 64 + j * 32 + r32;
        const float bv = (a.bias && n0 + c < a.Co) ? a.bias[n0 + c] : 0.0f;
        float q = 0.0f;
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = wm * WROWS + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                const float d = acc[i][j][r] + bv - mean[j];
                if (row < nv) q = fmaf(d, d, q);
            }
        q += __shfl_xor(q, 32);
        if (h == 0) red[wm * BN + c] = q;
    }
    __syncthreads();
    if (wm == 0 && h == 0) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int c = wn * 64 + j * 32 + r32;
            if (n0 + c < a.Co) {
                float t = 0.0f;
#pragma unroll
                for (int w = 0; w < NRW; ++w) t += red[w * BN + c];
                float *o = a.stats + ((int64_t)(n0 + c) * ((a.M + HBM - 1) / HBM) + m0 / HBM) * 2;
                o[0] = sum[j];
                o[1] = t;
            }
        }
    }
}

// HIN: the operand arrives in fp16 (a.xh) -- the value the fp32 path rounds it to while staging, so the result is
// bit-identical; 8-B loads instead of 16 and no conversion.
// BN: output columns per workgroup.  128: 2 x 2 waves of 64 x 64 (2 x 2 MFMA tiles each); 64 (outputs of <= 64
// channels: no zero half of the panel loaded or multiplied): 4 x 1 waves of 32 x 64 (1 x 2 tiles).  Per output the
// K order is the same, so both give identical conv results.
// BUF (fp16 operand, H16B_LINES, operand and panel < 2 GiB): the staging loads are raw buffer loads with 32-bit
// offsets -- per row a constant base, per K step one uniform tap offset (SGPR), and taps outside the image read
// through an out-of-range offset, which the buffer returns as zeros; the weight panel's K step is the SGPR soffset.
// Same values in LDS, so results are identical to the pointer form (r05q counters: ~7 VALU per MFMA there, mostly
// 64-bit address arithmetic).
template <bool HIN, int BN, bool BUF = false>
__global__ __launch_bounds__(256, 2) void k_conv_h16b(ConvH a) {
    constexpr int TI = BN == 128 ? 2 : 1, WROWS = BN == 128 ? 64 : 32, NBU = BN == 128 ? 4 : 2;
    __shared__ __attribute__((aligned(16))) _Float16 lds[2][(HBM + BN) * HROW2];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = BN == 128 ? wave >> 1 : wave, wn = BN == 128 ? wave & 1 : 0;
    const int ntn = (a.Co + BN - 1) / BN;
    const int64_t ntm = (a.M + HBM - 1) / HBM;
    unsigned bid = blockIdx.x;
    {
        const unsigned nb = gridDim.x, q = nb / 8, r = nb % 8, xc = bid % 8;
        bid = (xc < r ? xc * (q + 1) : r * (q + 1) + (xc - r) * q) + bid / 8;
    }
    const int64_t mt = bid / (unsigned)ntn;
    const int nt = (int)(bid % (unsigned)ntn);
    if (mt >= ntm) return;
    const int64_t m0 = mt * HBM;
    const int n0 = nt * BN;
    // A staging.  fp32 operand: rows (tid >> 2) + 64 q (q < 2), channel quads (tid & 3) + 4 u (u < 4), 16-B loads.
    // fp16 operand (H16B_LINES): rows (tid >> 3) + 32 q (q < 4), halves 8 (tid & 7) .. + 7 -- eight lanes read one
    // pixel's 128-B K step, so each wave load is 8 whole lines instead of 16 rows x 32 B.
    constexpr bool LN = HIN && H16B_LINES;
    constexpr int NQ = LN ? 4 : 2, ARS = LN ? 32 : 64;
    const int aq = LN ? (tid & 7) : (tid & 3), arow = LN ? (tid >> 3) : (tid >> 2);
    int64_t pix[NQ];
    int iy0[NQ], ix0[NQ];
    bool rok[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int64_t m = m0 + arow + ARS * q;
        rok[q] = m < a.M;
        const int64_t mm = rok[q] ? m : 0;
        const int ox = (int)(mm % a.Wo);
        const int64_t t = mm / a.Wo;
        const int oy = (int)(t % a.Ho);
        const int n = (int)(t / a.Ho);
        pix[q] = (int64_t)n * a.H * a.W * a.Ci + (LN ? 8 : 4) * aq;
        iy0[q] = oy * a.stride - a.pad;
        ix0[q] = ox * a.stride - a.pad;
    }
    // B staging (H16B_LINES): weight rows n0 + (tid >> 3) + 32 u (u < NBU), halves 8 (tid & 7) .. + 7 of the K step
    // (whole 128-B lines per wave load).  Otherwise row n0 + (tid >> 1), halves 32 (tid & 1) .. + 31 (BN 64: row
    // n0 + (tid >> 2), halves 16 (tid & 3) .. + 15).
    const int brow = H16B_LINES ? tid >> 3 : BN == 128 ? tid >> 1 : tid >> 2;
    const int bcol = H16B_LINES ? 8 * (tid & 7) : BN == 128 ? 32 * (tid & 1) : 16 * (tid & 3);
    const int64_t bstep = H16B_LINES ? 32 * (int64_t)a.Kp : 8;  // halves between a thread's NBU weight loads
    const int bls = H16B_LINES ? 32 * HROW2 : 8;                 // ... and between its LDS stores
    const _Float16 *wrow = a.wp + (int64_t)(n0 + brow) * a.Kp + bcol;
    static_assert(!BUF || LN, "buffer staging: fp16 operand, whole-line map");
    __amdgpu_buffer_rsrc_t rsx, rsw;
    int xrb[NQ], wvo[NBU];  // BUF: byte offsets of row q's (0, 0) tap piece / of weight load u at K step 0
    if constexpr (BUF) {
        rsx = __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16 *>(a.xh), 0,
                                                (int)((int64_t)a.N * a.H * a.W * a.Ci * 2), 0x00020000);
        rsw = __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16 *>(a.wp), 0,
                                                (int)(copad_h(a.Co) * (int64_t)a.Kp * 2), 0x00020000);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int n = (int)((pix[q] - 8 * aq) / ((int64_t)a.H * a.W * a.Ci));
            xrb[q] = (((n * a.H + iy0[q]) * a.W + ix0[q]) * a.Ci + 8 * aq) * 2;
        }
#pragma unroll
        for (int u = 0; u < NBU; ++u) wvo[u] = ((n0 + brow + 32 * u) * a.Kp + bcol) * 2;
    }
    int ky = 0, kx = 0, ci0 = 0;
    int64_t kb = 0;
    f32x4 ra0[8], ra1[8];
    h16x8 rh0[4], rh1[4];  // LN: one 16-B line piece per row q; else pairs of the old map's 8-B quads
    u32x4 rb0[NBU], rb1[NBU];
#define H16_GLOAD(RA, RH, RB)                                                                              \
    do {                                                                                                   \
        const int dy = ky * a.dil, dx = kx * a.dil;                                                        \
        if constexpr (BUF) {                                                                               \
            const int toff = ((dy * a.W + dx) * a.Ci + ci0) * 2; /* uniform */                             \
            _Pragma("unroll") for (int q = 0; q < NQ; ++q) {                                               \
                const int iy = iy0[q] + dy, ix = ix0[q] + dx;                                              \
                const bool in = rok[q] && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;    \
                RH[q] = __builtin_bit_cast(h16x8, __builtin_amdgcn_raw_buffer_load_b128(                   \
                                                      rsx, in ? xrb[q] + toff : (int)0x80000000, 0, 0));   \
            }                                                                                              \
        } else if constexpr (LN) {                                                                         \
            _Pragma("unroll") for (int q = 0; q < NQ; ++q) {                                               \
                const int iy = iy0[q] + dy, ix = ix0[q] + dx;                                              \
                const bool in = rok[q] && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;    \
                const int64_t e = pix[q] + ((int64_t)iy * a.W + ix) * a.Ci + ci0;                          \
                RH[q] = *(const h16x8 *)(in ? a.xh + e : (const _Float16 *)g_hzero4);                      \
            }                                                                                              \
        } else {                                                                                           \
            _Pragma("unroll") for (int q = 0; q < 2; ++q) {                                                \
                const int iy = iy0[q] + dy, ix = ix0[q] + dx;                                              \
                const bool in = rok[q] && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;    \
                const int64_t e = pix[q] + ((int64_t)iy * a.W + ix) * a.Ci + ci0;                          \
                const int st = in ? 16 : 0; /* the zero quad is re-read for every u */                     \
                if constexpr (HIN) {                                                                       \
                    const _Float16 *src = in ? a.xh + e : (const _Float16 *)g_hzero4;                      \
                    _Pragma("unroll") for (int u = 0; u < 4; ++u) {                                        \
                        const h16x4 v = *(const h16x4 *)(src + st * u);                                    \
                        RH[(4 * q + u) >> 1][4 * (u & 1) + 0] = v[0];                                      \
                        RH[(4 * q + u) >> 1][4 * (u & 1) + 1] = v[1];                                      \
                        RH[(4 * q + u) >> 1][4 * (u & 1) + 2] = v[2];                                      \
                        RH[(4 * q + u) >> 1][4 * (u & 1) + 3] = v[3];                                      \
                    }                                                                                      \
                } else {                                                                                   \
                    const float *src = in ? a.x + e : g_hzero4;                                            \
                    _Pragma("unroll") for (int u = 0; u < 4; ++u) RA[4 * q + u] = *(const f32x4 *)(src + st * u); \
                }                                                                                          \
            }                                                                                              \
        }                                                                                                  \
        if constexpr (BUF) {                                                                               \
            _Pragma("unroll") for (int u = 0; u < NBU; ++u) RB[u] = __builtin_bit_cast(                    \
                u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsw, wvo[u], (int)kb * 2, 0));                \
        } else {                                                                                           \
            _Pragma("unroll") for (int u = 0; u < NBU; ++u) RB[u] = *(const u32x4 *)(wrow + kb + bstep * u); \
        }                                                                                                  \
        kb += HBK2;                                                                                        \
        ci0 += HBK2;                                                                                       \
        if (ci0 == a.Ci) {                                                                                 \
            ci0 = 0;                                                                                       \
            if (++kx == a.KW) {                                                                            \
                kx = 0;                                                                                    \
                ++ky;                                                                                      \
            }                                                                                              \
        }                                                                                                  \
    } while (0)
#define H16_SWRITE(BUF, RA, RH, RB)                                                                        \
    do {                                                                                                   \
        _Float16 *As = lds[BUF], *Bs = As + HBM * HROW2;                                                   \
        if constexpr (LN) {                                                                                \
            _Pragma("unroll") for (int q = 0; q < NQ; ++q)                                                 \
                *(h16x8 *)(As + (arow + 32 * q) * HROW2 + 8 * aq) = RH[q];                                 \
        } else {                                                                                           \
            _Pragma("unroll") for (int q = 0; q < 8; ++q) {                                                \
                h16x4 hv;                                                                                  \
                if constexpr (HIN) hv = (h16x4){RH[q >> 1][4 * (q & 1)], RH[q >> 1][4 * (q & 1) + 1],      \
                                                RH[q >> 1][4 * (q & 1) + 2], RH[q >> 1][4 * (q & 1) + 3]}; \
                else hv = (h16x4){(_Float16)RA[q][0], (_Float16)RA[q][1], (_Float16)RA[q][2], (_Float16)RA[q][3]}; \
                *(h16x4 *)(As + (arow + 64 * (q >> 2)) * HROW2 + 4 * aq + 16 * (q & 3)) = hv;              \
            }                                                                                              \
        }                                                                                                  \
        _Pragma("unroll") for (int u = 0; u < NBU; ++u)                                                    \
            *(u32x4 *)(Bs + brow * HROW2 + bcol + bls * u) = RB[u];                                        \
    } while (0)
    f32x16 acc[TI][2];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = (f32x16){0};
    const int r32 = lane & 31, h = lane >> 5;
#define H16_MFMA(BUF)                                                                                      \
    do {                                                                                                   \
        const _Float16 *As = lds[BUF], *Bs = As + HBM * HROW2;                                             \
        _Pragma("unroll") for (int kk = 0; kk < 4; ++kk) {                                                 \
            h16x8 fa[TI], fb[2];                                                                           \
            _Pragma("unroll") for (int i = 0; i < TI; ++i)                                                 \
                fa[i] = *(const h16x8 *)(As + (wm * WROWS + i * 32 + r32) * HROW2 + kk * 16 + 8 * h);      \
            _Pragma("unroll") for (int j = 0; j < 2; ++j)                                                  \
                fb[j] = *(const h16x8 *)(Bs + (wn * 64 + j * 32 + r32) * HROW2 + kk * 16 + 8 * h);         \
            _Pragma("unroll") for (int i = 0; i < TI; ++i)                                                 \
                _Pragma("unroll") for (int j = 0; j < 2; ++j)                                              \
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[i], fb[j], acc[i][j], 0, 0, 0);  \
            __builtin_amdgcn_sched_barrier(0); /* one slice of fragments live at a time (VGPR budget) */   \
        }                                                                                                  \
    } while (0)
    const int nk = a.Kp / HBK2;
    H16_GLOAD(ra0, rh0, rb0);
    if (nk > 1) H16_GLOAD(ra1, rh1, rb1);
    H16_SWRITE(0, ra0, rh0, rb0);
    __syncthreads();
    int ks = 0;  // loop head: LDS buffer 0 holds step ks, register set 1 step ks + 1
    for (; ks + 3 < nk; ks += 2) {
        H16_GLOAD(ra0, rh0, rb0);
        H16_MFMA(0);
        H16_SWRITE(1, ra1, rh1, rb1);
        __syncthreads();
        H16_GLOAD(ra1, rh1, rb1);
        H16_MFMA(1);
        H16_SWRITE(0, ra0, rh0, rb0);
        __syncthreads();
    }
    if (ks + 2 < nk) {
        H16_GLOAD(ra0, rh0, rb0);
        H16_MFMA(0);
        H16_SWRITE(1, ra1, rh1, rb1);
        __syncthreads();
        H16_MFMA(1);
        H16_SWRITE(0, ra0, rh0, rb0);
        __syncthreads();
        H16_MFMA(0);
    } else if (ks + 1 < nk) {
        H16_MFMA(0);
        H16_SWRITE(1, ra1, rh1, rb1);
        __syncthreads();
        H16_MFMA(1);
    } else {
        H16_MFMA(0);
    }
#undef H16_MFMA
#undef H16_SWRITE
#undef H16_GLOAD
    if (a.stats) h16_tile_stats<BN, TI>(a, acc, lds[0], m0, n0, wm, wn, r32, h);
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int col = n0 + wn * 64 + j * 32 + r32;
            if (col >= a.Co) continue;
            const float bv = a.bias ? a.bias[col] : 0.0f;
            float rv[16];  // all residual loads first: interleaved with the stores they would serialise (y may alias)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t row = m0 + wm * WROWS + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                rv[r] = (a.res && row < a.M) ? a.res[row * a.Co + col] : 0.0f;
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t row = m0 + wm * WROWS + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (row >= a.M) continue;
                float v = acc[i][j][r] + bv;
                if (a.res) v += rv[r];
                a.y[row * a.ldy + col] = act_h(v, a.act);
            }
        }
}

// ---- weight gradient under autocast(float16): dW[co][k] = sum_m f16(dz[m][co]) * f16(im2col(x)[m][k]) ----------
// The reduction index of v_mfma_f32_32x32x16_f16 is the output pixel m: lane l needs 8 consecutive pixels of one
// channel (A = dz^T, B = im2col(x)), so both operands are staged TRANSPOSED into LDS as fp16 [channel][pixel]
// rows of 40 halves (the forward kernel's conflict-free 80-B rows).  Each thread loads four pixel rows of one
// channel quad (float4, coalesced along channels), rounds them to fp16 and writes each channel's four pixels
// as one ds_write_b64.  Block tile 128 (co) x 128 (k), 2 x 2 waves of 64 x 64, 32 pixels per step, registers
// prefetched one step ahead, double-buffered LDS; the pixel range is split over workgroups and the partial
// tiles are added with float atomics (summation order varies in the last bits, as in the fp32 kernels).
constexpr int WT = 128, WMS = 32;

__global__ __launch_bounds__(256, 2) void k_wgrad_h16(const float *__restrict__ x, const float *__restrict__ dz,
                                                       int N, int H, int W, int Ci, int Ho, int Wo, int Co, int KW,
                                                       int K, int stride, int pad, int dil, int64_t mchunk, int ctiles,
                                                       int ntiles, float *__restrict__ dW) {
    __shared__ __attribute__((aligned(16))) _Float16 lds[2][2 * WT * HROW];
    unsigned bid = blockIdx.x;
    {
        const unsigned nb = gridDim.x, q = nb / 8, r = nb % 8, xc = bid % 8;
        bid = (xc < r ? xc * (q + 1) : r * (q + 1) + (xc - r) * q) + bid / 8;
    }
    const int tile = (int)(bid % (unsigned)ntiles);
    const int64_t split = bid / (unsigned)ntiles;
    const int co0 = (tile % ctiles) * WT, k0 = (tile / ctiles) * WT;
    const int64_t M = (int64_t)N * Ho * Wo;
    const int64_t mb = split * mchunk, me = mb + mchunk < M ? mb + mchunk : M;
    if (mb >= me) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
    const int rg = tid >> 5, q = tid & 31;  // staging: pixel rows 4 rg .. 4 rg + 3, channel quad q
    const int co = co0 + 4 * q;
    const bool co_ok = co < Co;
    const int k = k0 + 4 * q;  // 4 consecutive k inside one tap (Ci % 4 == 0)
    const bool k_ok = k < K;
    const int tap = k_ok ? k / Ci : 0, ci = k - tap * Ci, ky = tap / KW, kx = tap - ky * KW;
    // (image, row, column) of this thread's first pixel row in the current step
    int px, py, pn;
    {
        const int64_t m = mb + 4 * rg, t = m / Wo;
        px = (int)(m - t * Wo);
        py = (int)(t % Ho);
        pn = (int)(t / Ho);
    }
    int64_t ms = mb;
    f32x4 ra[4], rb[4];
    auto gload = [&]() {
        int x1 = px, y1 = py, n1 = pn;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t m = ms + 4 * rg + r;
            const bool mok = m < me;
            ra[r] = (mok && co_ok) ? *(const f32x4 *)(dz + m * Co + co) : (f32x4){0.f, 0.f, 0.f, 0.f};
            const int iy = y1 * stride - pad + ky * dil, ix = x1 * stride - pad + kx * dil;
            const bool in = mok && k_ok && iy >= 0 && iy < H && ix >= 0 && ix < W;
            rb[r] = in ? *(const f32x4 *)(x + (((int64_t)n1 * H + iy) * W + ix) * Ci + ci) : (f32x4){0.f, 0.f, 0.f, 0.f};
            if (++x1 == Wo) {
                x1 = 0;
                if (++y1 == Ho) {
                    y1 = 0;
                    ++n1;
                }
            }
        }
        ms += WMS;
        px += WMS;
        while (px >= Wo) {
            px -= Wo;
            if (++py == Ho) {
                py = 0;
                ++pn;
            }
        }
    };
    auto swrite = [&](int buf) {
        _Float16 *As = lds[buf], *Bs = As + WT * HROW;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const h16x4 ha = {(_Float16)ra[0][c], (_Float16)ra[1][c], (_Float16)ra[2][c], (_Float16)ra[3][c]};
            const h16x4 hb = {(_Float16)rb[0][c], (_Float16)rb[1][c], (_Float16)rb[2][c], (_Float16)rb[3][c]};
            *(h16x4 *)(As + (4 * q + c) * HROW + 4 * rg) = ha;
            *(h16x4 *)(Bs + (4 * q + c) * HROW + 4 * rg) = hb;
        }
    };
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = (f32x16){0};
    const int nsteps = (int)((me - mb + WMS - 1) / WMS);
    gload();
    swrite(0);
    __syncthreads();
    const int r32 = lane & 31, h = lane >> 5;
    for (int st = 0; st < nsteps; ++st) {
        const bool more = st + 1 < nsteps;
        if (more) gload();
        const _Float16 *As = lds[st & 1], *Bs = As + WT * HROW;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            h16x8 fa[2], fb[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) fa[i] = *(const h16x8 *)(As + (wm * 64 + i * 32 + r32) * HROW + kk * 16 + 8 * h);
#pragma unroll
            for (int j = 0; j < 2; ++j) fb[j] = *(const h16x8 *)(Bs + (wn * 64 + j * 32 + r32) * HROW + kk * 16 + 8 * h);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
        if (more) swrite((st + 1) & 1);
        __syncthreads();
    }
    // D[row][col]: row = co (A rows), col = k; row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5), col = lane & 31
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int kc = k0 + wn * 64 + j * 32 + r32;
            if (kc >= K) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int cr = co0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (cr < Co) atomicAdd(dW + (int64_t)cr * K + kc, acc[i][j][r]);
            }
        }
}

// ---- k_wgrad_h16b: 64 pixels per K step, two steps of operands in flight -----------------------------------------
// k_wgrad_h16's 32-pixel step gives a wave 8 MFMAs (~256 cycles) per barrier with one step of loads in flight: the
// global-load latency is exposed (the weight gradient was 15 % of the AMP training step).  Here a step is 64 pixels
// (16 MFMAs per wave) and, as in k_conv_h16b, the loads of steps s + 1 and s + 2 sit in two register sets while
// step s runs.  Staging: thread (rg = tid >> 5, q = tid & 31) loads pixel rows 8 rg .. 8 rg + 7 of channel quad q
// of both operands and writes each channel's 8 pixels as ONE ds_write_b128 ([channel][pixel] rows of 72 halves:
// 9 odd 16-B slots, conflict-free fragment reads).  Same per-element products; pixel chunks per workgroup are
// multiples of 64 (fp32-tolerance equal to k_wgrad_h16, float atomics across chunks as there).
// XH / DH: x / dz arrive in fp16 (the values the fp32 path rounds them to: bit-identical products).
constexpr int WMS2 = 64, WROW2 = 72;

template <bool XH, bool DH>
__global__ __launch_bounds__(256, 2) void k_wgrad_h16b(const float *__restrict__ x, const float *__restrict__ dz,
                                                        int N, int H, int W, int Ci, int Ho, int Wo, int Co, int KW,
                                                        int K, int stride, int pad, int dil, int64_t mchunk, int ctiles,
                                                        int ntiles, float *__restrict__ dW) {
    __shared__ __attribute__((aligned(16))) _Float16 lds[2][2 * WT * WROW2];
    unsigned bid = blockIdx.x;
    {
        const unsigned nb = gridDim.x, q = nb / 8, r = nb % 8, xc = bid % 8;
        bid = (xc < r ? xc * (q + 1) : r * (q + 1) + (xc - r) * q) + bid / 8;
    }
    const int tile = (int)(bid % (unsigned)ntiles);
    const int64_t split = bid / (unsigned)ntiles;
    const int co0 = (tile % ctiles) * WT, k0 = (tile / ctiles) * WT;
    const int64_t M = (int64_t)N * Ho * Wo;
    const int64_t mb = split * mchunk, me = mb + mchunk < M ? mb + mchunk : M;
    if (mb >= me) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int rg = tid >> 5, q = tid & 31;  // staging: pixel rows 8 rg .. 8 rg + 7, channel quad q
    const int co = co0 + 4 * q;
    const bool co_ok = co < Co;
    const int k = k0 + 4 * q;
    const bool k_ok = k < K;
    const int tap = k_ok ? k / Ci : 0, ci = k - tap * Ci, ky = tap / KW, kx = tap - ky * KW;
    const int dyo = ky * dil - pad, dxo = kx * dil - pad;
    int px, py, pn;  // (column, row, image) of this thread's first pixel row of the next step to load
    {
        const int64_t m = mb + 8 * rg, t = m / Wo;
        px = (int)(m - t * Wo);
        py = (int)(t % Ho);
        pn = (int)(t / Ho);
    }
    int64_t ms = mb;
    const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
#define WG16_LOAD(RA, RB)                                                                                      \
    do {                                                                                                       \
        int x1 = px, y1 = py, n1 = pn;                                                                         \
        _Pragma("unroll") for (int r = 0; r < 8; ++r) {                                                        \
            const int64_t m = ms + 8 * rg + r;                                                                 \
            const bool mok = m < me;                                                                           \
            if constexpr (DH)                                                                                  \
                RA##h[r] = (mok && co_ok) ? *(const h16x4 *)((const _Float16 *)dz + m * Co + co) : h4z;        \
            else                                                                                               \
                RA[r] = (mok && co_ok) ? *(const f32x4 *)(dz + m * Co + co) : z4;                              \
            const int iy = y1 * stride + dyo, ix = x1 * stride + dxo;                                          \
            const bool in = mok && k_ok && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;           \
            const int64_t xe = (((int64_t)n1 * H + iy) * W + ix) * Ci + ci;                                    \
            if constexpr (XH)                                                                                  \
                RB##h[r] = in ? *(const h16x4 *)((const _Float16 *)x + xe) : h4z;                              \
            else                                                                                               \
                RB[r] = in ? *(const f32x4 *)(x + xe) : z4;                                                    \
            if (++x1 == Wo) {                                                                                  \
                x1 = 0;                                                                                        \
                if (++y1 == Ho) {                                                                              \
                    y1 = 0;                                                                                    \
                    ++n1;                                                                                      \
                }                                                                                              \
            }                                                                                                  \
        }                                                                                                      \
        ms += WMS2;                                                                                            \
        px += WMS2;                                                                                            \
        while (px >= Wo) {                                                                                     \
            px -= Wo;                                                                                          \
            if (++py == Ho) {                                                                                  \
                py = 0;                                                                                        \
                ++pn;                                                                                          \
            }                                                                                                  \
        }                                                                                                      \
    } while (0)
#define WG16_STORE(BUF, RA, RB)                                                                                \
    do {                                                                                                       \
        _Float16 *As = lds[BUF], *Bs = As + WT * WROW2;                                                        \
        _Pragma("unroll") for (int c = 0; c < 4; ++c) {                                                        \
            h16x8 ha, hb;                                                                                      \
            _Pragma("unroll") for (int r = 0; r < 8; ++r) {                                                    \
                if constexpr (DH) ha[r] = RA##h[r][c];                                                         \
                else ha[r] = (_Float16)RA[r][c];                                                               \
                if constexpr (XH) hb[r] = RB##h[r][c];                                                         \
                else hb[r] = (_Float16)RB[r][c];                                                               \
            }                                                                                                  \
            *(h16x8 *)(As + (4 * q + c) * WROW2 + 8 * rg) = ha;                                                \
            *(h16x8 *)(Bs + (4 * q + c) * WROW2 + 8 * rg) = hb;                                                \
        }                                                                                                      \
    } while (0)
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = (f32x16){0};
    const int r32 = lane & 31, h = lane >> 5;
#define WG16_MFMA(BUF)                                                                                         \
    do {                                                                                                       \
        const _Float16 *As = lds[BUF], *Bs = As + WT * WROW2;                                                  \
        _Pragma("unroll") for (int kk = 0; kk < 4; ++kk) {                                                     \
            h16x8 fa[2], fb[2];                                                                                \
            _Pragma("unroll") for (int i = 0; i < 2; ++i)                                                      \
                fa[i] = *(const h16x8 *)(As + (wm * 64 + i * 32 + r32) * WROW2 + kk * 16 + 8 * h);             \
            _Pragma("unroll") for (int j = 0; j < 2; ++j)                                                      \
                fb[j] = *(const h16x8 *)(Bs + (wn * 64 + j * 32 + r32) * WROW2 + kk * 16 + 8 * h);             \
            _Pragma("unroll") for (int i = 0; i < 2; ++i)                                                      \
                _Pragma("unroll") for (int j = 0; j < 2; ++j)                                                  \
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[i], fb[j], acc[i][j], 0, 0, 0);      \
            __builtin_amdgcn_sched_barrier(0);                                                                 \
        }                                                                                                      \
    } while (0)
    f32x4 ra0[8], rb0[8], ra1[8], rb1[8];
    h16x4 ra0h[8], rb0h[8], ra1h[8], rb1h[8];
    const h16x4 h4z = {(_Float16)0.0f, (_Float16)0.0f, (_Float16)0.0f, (_Float16)0.0f};
    const int nk = (int)((me - mb + WMS2 - 1) / WMS2);
    WG16_LOAD(ra0, rb0);
    if (nk > 1) WG16_LOAD(ra1, rb1);
    WG16_STORE(0, ra0, rb0);
    __syncthreads();
    int ks = 0;  // loop head: LDS buffer 0 holds step ks, register set 1 step ks + 1
    for (; ks + 3 < nk; ks += 2) {
        WG16_LOAD(ra0, rb0);
        WG16_MFMA(0);
        WG16_STORE(1, ra1, rb1);
        __syncthreads();
        WG16_LOAD(ra1, rb1);
        WG16_MFMA(1);
        WG16_STORE(0, ra0, rb0);
        __syncthreads();
    }
    if (ks + 2 < nk) {
        WG16_LOAD(ra0, rb0);
        WG16_MFMA(0);
        WG16_STORE(1, ra1, rb1);
        __syncthreads();
        WG16_MFMA(1);
        WG16_STORE(0, ra0, rb0);
        __syncthreads();
        WG16_MFMA(0);
    } else if (ks + 1 < nk) {
        WG16_MFMA(0);
        WG16_STORE(1, ra1, rb1);
        __syncthreads();
        WG16_MFMA(1);
    } else {
        WG16_MFMA(0);
    }
#undef WG16_MFMA
#undef WG16_STORE
#undef WG16_LOAD
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int kc = k0 + wn * 64 + j * 32 + r32;
            if (kc >= K) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int cr = co0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (cr < Co) atomicAdd(dW + (int64_t)cr * K + kc, acc[i][j][r]);
            }
        }
}

// ---- k_wgrad_h16c: natural [pixel][channel] LDS images read back with the transposing ds_read_b64_tr_b16 --------
// k_wgrad_h16b transposes in registers (each thread gathers 8 pixels of a channel into one ds_write_b128): ~20 VALU
// per MFMA and 0.20 MFMA utilisation in its counters (profiles/r05q_conv_h16_pmc.txt).  Here each thread loads 16-B
// pieces of pixel rows -- dz[m][co0 + 8 c .. + 7] and the tap's x[pixel][ci .. ci + 7] -- and stores them unchanged
// into [64 pixels][128 channels] images (256-B rows, XOR-swizzled 16-B chunks, cdna_hip_programming.md T10 (b):
// conflict-free for the 32x32x16 transposed reads); the MFMA fragments (8 consecutive pixels of one channel per
// lane) are two ds_read_b64_tr_b16 each.  Same tiles, pixel chunks and per-slice pixel order as k_wgrad_h16b, so
// every workgroup's partial tile is bit-identical to it; only the float-atomic order across chunks varies (as
// there).  dz (DH) and x (XH) in fp16, or fp32 rounded to fp16 in the staging write (as k_wgrad_h16b does).
// Requires Ci % 8 == 0 and Co % 8 == 0 (a 16-B piece inside one tap / one output row) and 16-B aligned operands.
#ifndef H16_WGRAD_TR
#define H16_WGRAD_TR 1
#endif
typedef short s16x4v __attribute__((vector_size(8)));

__device__ __forceinline__ h16x4 lds_tr16(const _Float16 *p) {
    return __builtin_bit_cast(
        h16x4, __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4v *)(_Float16 *)p));
}

__device__ __forceinline__ int tr_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

template <bool XH, bool DH>
__global__ __launch_bounds__(256, 2) void k_wgrad_h16c(const float *__restrict__ x, const void *__restrict__ dzv,
                                                        int N, int H, int W, int Ci, int Ho, int Wo, int Co, int KW,
                                                        int K, int stride, int pad, int dil, int64_t mchunk, int ctiles,
                                                        int ntiles, float *__restrict__ dW) {
    constexpr int IMG = WMS2 * WT;  // halves per operand image: 64 pixel rows x 128 channels
    __shared__ __attribute__((aligned(16))) _Float16 lds[2][2 * IMG];
    const _Float16 *dz = (const _Float16 *)dzv;  // DH: fp16 gradient; else fp32 (dzf), rounded while staging
    const float *dzf = (const float *)dzv;
    unsigned bid = blockIdx.x;
    {
        const unsigned nb = gridDim.x, q = nb / 8, r = nb % 8, xc = bid % 8;
        bid = (xc < r ? xc * (q + 1) : r * (q + 1) + (xc - r) * q) + bid / 8;
    }
    const int tile = (int)(bid % (unsigned)ntiles);
    const int split = (int)(bid / (unsigned)ntiles);
    const int co0 = (tile % ctiles) * WT, k0 = (tile / ctiles) * WT;
    const int M = N * Ho * Wo;  // the launcher checks that every offset fits in 31 bits
    const int mb = split * (int)mchunk, me = mb + (int)mchunk < M ? mb + (int)mchunk : M;
    if (mb >= me) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    // staging: ONE pixel row per thread and step, prow = tid >> 2, its 16-B pieces cq + 4 u (u < 4), cq = tid & 3:
    // one address per operand and step; four lanes cover 64 contiguous bytes of a row per load instruction
    const int prow = tid >> 2, cq = tid & 3;
    int dzo = (mb + prow) * Co + co0 + 8 * cq;  // dz offset of piece 0 (pieces u at + 32 u halves)
    unsigned cmask = 0;                         // pieces inside [0, Co) / [0, K)
    int xoff[4], xdy[4], xdx[4];                // per piece: offset from the pixel's (0, 0) tap, tap displacement
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int c = co0 + 8 * (cq + 4 * u), k = k0 + 8 * (cq + 4 * u);
        if (c < Co) cmask |= 1u << u;
        const bool kok = k < K;
        if (kok) cmask |= 16u << u;
        const int tap = kok ? k / Ci : 0, ci = k - tap * Ci, ky = tap / KW, kx = tap - ky * KW;
        xdy[u] = ky * dil - pad;
        xdx[u] = kx * dil - pad;
        xoff[u] = (xdy[u] * W + xdx[u]) * Ci + ci;
    }
    int px, py, pn;  // (column, row, image) of this thread's pixel row in the next step to load
    {
        const int m = mb + prow, t = m / Wo;
        px = m - t * Wo;
        py = t % Ho;
        pn = t / Ho;
    }
    int ms = mb;
    const int soff = tr_swz(prow);  // rows prow: chunk c of the row sits at c ^ soff
    const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
    const h16x8 hz = {(_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f,
                      (_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
#define WG16C_LOAD(RD, RX, RF, RG)                                                                             \
    do {                                                                                                       \
        const bool mok = ms + prow < me;                                                                       \
        const int iy0 = py * stride, ix0 = px * stride;                                                        \
        const int xb = ((pn * H + iy0) * W + ix0) * Ci;                                                        \
        _Pragma("unroll") for (int u = 0; u < 4; ++u) {                                                        \
            const bool dok = mok && (cmask >> u & 1);                                                          \
            if constexpr (DH) {                                                                                \
                RD[u] = dok ? *(const h16x8 *)(dz + dzo + 32 * u) : hz;                                        \
            } else {                                                                                           \
                RG[2 * u] = dok ? *(const f32x4 *)(dzf + dzo + 32 * u) : z4;                                   \
                RG[2 * u + 1] = dok ? *(const f32x4 *)(dzf + dzo + 32 * u + 4) : z4;                           \
            }                                                                                                  \
            const int iy = iy0 + xdy[u], ix = ix0 + xdx[u];                                                    \
            const bool in = mok && (cmask >> (4 + u) & 1) && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W; \
            if constexpr (XH) {                                                                                \
                RX[u] = in ? *(const h16x8 *)((const _Float16 *)x + (xb + xoff[u])) : hz;                      \
            } else {                                                                                           \
                RF[2 * u] = in ? *(const f32x4 *)(x + (xb + xoff[u])) : z4;                                    \
                RF[2 * u + 1] = in ? *(const f32x4 *)(x + (xb + xoff[u] + 4)) : z4;                            \
            }                                                                                                  \
        }                                                                                                      \
        dzo += WMS2 * Co;                                                                                      \
        ms += WMS2;                                                                                            \
        px += WMS2;                                                                                            \
        while (px >= Wo) {                                                                                     \
            px -= Wo;                                                                                          \
            if (++py == Ho) {                                                                                  \
                py = 0;                                                                                        \
                ++pn;                                                                                          \
            }                                                                                                  \
        }                                                                                                      \
    } while (0)
#define WG16C_STORE(BUF, RD, RX, RF, RG)                                                                       \
    do {                                                                                                       \
        _Float16 *Ds = lds[BUF] + prow * WT, *Xs = Ds + IMG;                                                   \
        _Pragma("unroll") for (int u = 0; u < 4; ++u) {                                                        \
            const int o = 8 * ((cq + 4 * u) ^ soff);                                                           \
            if constexpr (DH) {                                                                                \
                *(h16x8 *)(Ds + o) = RD[u];                                                                    \
            } else {                                                                                           \
                const f32x4 c_ = RG[2 * u], d_ = RG[2 * u + 1];                                                \
                *(h16x8 *)(Ds + o) = (h16x8){(_Float16)c_[0], (_Float16)c_[1], (_Float16)c_[2], (_Float16)c_[3], \
                                             (_Float16)d_[0], (_Float16)d_[1], (_Float16)d_[2], (_Float16)d_[3]}; \
            }                                                                                                  \
            if constexpr (XH) {                                                                                \
                *(h16x8 *)(Xs + o) = RX[u];                                                                    \
            } else {                                                                                           \
                const f32x4 a_ = RF[2 * u], b_ = RF[2 * u + 1];                                                \
                *(h16x8 *)(Xs + o) = (h16x8){(_Float16)a_[0], (_Float16)a_[1], (_Float16)a_[2], (_Float16)a_[3], \
                                             (_Float16)b_[0], (_Float16)b_[1], (_Float16)b_[2], (_Float16)b_[3]}; \
            }                                                                                                  \
        }                                                                                                      \
    } while (0)
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = (f32x16){0};
    // transposed fragment reads: 16-lane group g = lane >> 4 reads rows kk 16 + 8 (g >> 1) + {0..3} and {4..7} of
    // the 16 columns cb + 16 (g & 1) ..; lane 4 q + p of the group addresses row q, columns 4 p .. 4 p + 3
    const int li = lane & 15, g = lane >> 4, q = li >> 2, p = li & 3;
    const int rq = 8 * (g >> 1) + q;                                                    // row within a 16-row slice
    const int cg = 2 * (g & 1) + (p >> 1), sw0 = tr_swz(rq), sw1 = tr_swz(rq + 4), hp = 4 * (p & 1);
    const int r32 = lane & 31, h = lane >> 5;
#define WG16C_FRAG(IMGP, KK, CB, F)                                                                            \
    do {                                                                                                       \
        const int ch_ = (CB) / 8 + cg;                                                                         \
        const h16x4 lo_ = lds_tr16((IMGP) + ((KK) * 16 + rq) * WT + 8 * (ch_ ^ sw0) + hp);                     \
        const h16x4 hi_ = lds_tr16((IMGP) + ((KK) * 16 + rq + 4) * WT + 8 * (ch_ ^ sw1) + hp);                 \
        F = __builtin_shufflevector(lo_, hi_, 0, 1, 2, 3, 4, 5, 6, 7);                                         \
    } while (0)
#define WG16C_MFMA(BUF)                                                                                        \
    do {                                                                                                       \
        const _Float16 *Ds = lds[BUF], *Xs = Ds + IMG;                                                         \
        _Pragma("unroll") for (int kk = 0; kk < 4; ++kk) {                                                     \
            h16x8 fa[2], fb[2];                                                                                \
            _Pragma("unroll") for (int i = 0; i < 2; ++i) WG16C_FRAG(Ds, kk, wm * 64 + i * 32, fa[i]);         \
            _Pragma("unroll") for (int j = 0; j < 2; ++j) WG16C_FRAG(Xs, kk, wn * 64 + j * 32, fb[j]);         \
            _Pragma("unroll") for (int i = 0; i < 2; ++i)                                                      \
                _Pragma("unroll") for (int j = 0; j < 2; ++j)                                                  \
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[i], fb[j], acc[i][j], 0, 0, 0);      \
            __builtin_amdgcn_sched_barrier(0);                                                                 \
        }                                                                                                      \
    } while (0)
    h16x8 rd0[4], rd1[4], rx0[4], rx1[4];
    f32x4 rf0[8], rf1[8], rg0[8], rg1[8];
    const int nk = (int)((me - mb + WMS2 - 1) / WMS2);
    WG16C_LOAD(rd0, rx0, rf0, rg0);
    if (nk > 1) WG16C_LOAD(rd1, rx1, rf1, rg1);
    WG16C_STORE(0, rd0, rx0, rf0, rg0);
    __syncthreads();
    int ks = 0;  // loop head: LDS buffer 0 holds step ks, register set 1 step ks + 1
    for (; ks + 3 < nk; ks += 2) {
        WG16C_LOAD(rd0, rx0, rf0, rg0);
        WG16C_MFMA(0);
        WG16C_STORE(1, rd1, rx1, rf1, rg1);
        __syncthreads();
        WG16C_LOAD(rd1, rx1, rf1, rg1);
        WG16C_MFMA(1);
        WG16C_STORE(0, rd0, rx0, rf0, rg0);
        __syncthreads();
    }
    if (ks + 2 < nk) {
        WG16C_LOAD(rd0, rx0, rf0, rg0);
        WG16C_MFMA(0);
        WG16C_STORE(1, rd1, rx1, rf1, rg1);
        __syncthreads();
        WG16C_MFMA(1);
        WG16C_STORE(0, rd0, rx0, rf0, rg0);
        __syncthreads();
        WG16C_MFMA(0);
    } else if (ks + 1 < nk) {
        WG16C_MFMA(0);
        WG16C_STORE(1, rd1, rx1, rf1, rg1);
        __syncthreads();
        WG16C_MFMA(1);
    } else {
        WG16C_MFMA(0);
    }
#undef WG16C_MFMA
#undef WG16C_FRAG
#undef WG16C_STORE
#undef WG16C_LOAD
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int kc = k0 + wn * 64 + j * 32 + r32;
            if (kc >= K) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int cr = co0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (cr < Co) atomicAdd(dW + (int64_t)cr * K + kc, acc[i][j][r]);
            }
        }
}

}  // namespace

namespace bev {
int conv_h16_tune(int value) {
    if (value < 0 || value > 3) return BEV_ERR_ARGS;
    const int old = g_h16_kernel;
    g_h16_kernel = value;
    return old;
}
}  // namespace bev

extern "C" {

int bev_conv_wgrad_h16_ex_f32(const void *xv, int x_half, int N, int H, int W, int Ci, const void *dzv, int dz_half,
                              int Ho, int Wo, int Co, int KH, int KW, int stride, int pad, int dilation, float *dW,
                              void *stream) {
    const float *x = (const float *)xv, *dz = (const float *)dzv;
    if (!x || !dz || !dW || N < 0 || H <= 0 || W <= 0 || Ci <= 0 || Co <= 0 || KH <= 0 || KW <= 0 || stride <= 0 ||
        pad < 0 || dilation <= 0)
        return BEV_ERR_ARGS;
    if (Ci % 4 != 0 || Co % 4 != 0 || (((uintptr_t)x | (uintptr_t)dz) & 7) != 0) return BEV_ERR_ARGS;
    if ((!x_half && ((uintptr_t)x & 15) != 0) || (!dz_half && ((uintptr_t)dz & 15) != 0)) return BEV_ERR_ARGS;
    if (Ho != (H + 2 * pad - dilation * (KH - 1) - 1) / stride + 1 ||
        Wo != (W + 2 * pad - dilation * (KW - 1) - 1) / stride + 1 || Ho <= 0 || Wo <= 0)
        return BEV_ERR_ARGS;
    const int K = KH * KW * Ci;
    const int64_t M = (int64_t)N * Ho * Wo;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(dW, 0, (size_t)Co * K * sizeof(float), st) != hipSuccess) return (int)hipGetLastError();
    if (M == 0) return 0;
    const int ct = (Co + WT - 1) / WT, kt = (K + WT - 1) / WT, nt = ct * kt;
    const bool deep = g_h16_kernel != 1 || x_half || dz_half;  // k_wgrad_h16b (64-pixel steps, two in flight); 1:
                                                               // k_wgrad_h16 (fp32 operands only)
    const int step = deep ? WMS2 : WMS;
    int64_t sp = 1024 / nt + 1;  // >= ~1024 workgroups
    int64_t mc = (M + sp - 1) / sp;
    mc = ((mc + step - 1) / step) * step;
    sp = (M + mc - 1) / mc;
    if (sp * nt >= ((int64_t)1 << 31)) return BEV_ERR_ARGS;
    const bool tr = H16_WGRAD_TR && deep && Ci % 8 == 0 && Co % 8 == 0 &&
                    (((uintptr_t)x | (uintptr_t)dz) & 15) == 0 && M * Co < ((int64_t)1 << 31) - WMS2 * Co &&
                    (int64_t)N * H * W * Ci < ((int64_t)1 << 31);  // k_wgrad_h16c: 32-bit offsets
    if (tr) {
        auto kern = x_half ? (dz_half ? k_wgrad_h16c<true, true> : k_wgrad_h16c<true, false>)
                           : (dz_half ? k_wgrad_h16c<false, true> : k_wgrad_h16c<false, false>);
        hipLaunchKernelGGL(kern, dim3((unsigned)(sp * nt)), dim3(256), 0, st, x, (const void *)dz, N, H, W, Ci,
                           Ho, Wo, Co, KW, K, stride, pad, dilation, mc, ct, nt, dW);
    } else if (deep) {
        auto kern = x_half ? (dz_half ? k_wgrad_h16b<true, true> : k_wgrad_h16b<true, false>)
                           : (dz_half ? k_wgrad_h16b<false, true> : k_wgrad_h16b<false, false>);
        hipLaunchKernelGGL(kern, dim3((unsigned)(sp * nt)), dim3(256), 0, st, x, dz, N, H, W, Ci, Ho, Wo, Co, KW, K,
                           stride, pad, dilation, mc, ct, nt, dW);
    }
    else
        hipLaunchKernelGGL(k_wgrad_h16, dim3((unsigned)(sp * nt)), dim3(256), 0, st, x, dz, N, H, W, Ci, Ho, Wo, Co, KW,
                           K, stride, pad, dilation, mc, ct, nt, dW);
    return (int)hipGetLastError();
}


int bev_conv_wgrad_h16_f32(const float *x, int N, int H, int W, int Ci, const float *dz, int Ho, int Wo, int Co,
                           int KH, int KW, int stride, int pad, int dilation, float *dW, void *stream) {
    return bev_conv_wgrad_h16_ex_f32(x, 0, N, H, W, Ci, dz, 0, Ho, Wo, Co, KH, KW, stride, pad, dilation, dW, stream);
}

int64_t bev_conv_packed_size_h16(int Co, int Ci, int KH, int KW) {
    if (Co <= 0 || Ci <= 0 || KH <= 0 || KW <= 0) return BEV_ERR_ARGS;
    return copad_h(Co) * kpad_h(Ci * KH * KW);
}

int bev_conv_pack_weights_h16(const float *w, int Co, int Ci, int KH, int KW, uint16_t *packed, void *stream) {
    if (!w || !packed || Co <= 0 || Ci <= 0 || KH <= 0 || KW <= 0) return BEV_ERR_ARGS;
    const int64_t Kp = kpad_h(Ci * KH * KW), Cop = copad_h(Co), n = Kp * Cop;
    hipLaunchKernelGGL(k_pack_h16, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, w, Co, Ci, KH,
                       KW, Kp, Cop, (_Float16 *)packed);
    return (int)hipGetLastError();
}

static int conv_h16(const void *xv, int x_half, int N, int H, int W, int Ci, const uint16_t *packed, const float *bias,
                    const float *residual, int Co, int KH, int KW, int stride, int pad, int dilation, int act, float *y,
                    int ldy, int Ho, int Wo, float *stats, void *stream) {
    const float *x = (const float *)xv;
    if (!x || !packed || !y || N < 0 || H <= 0 || W <= 0 || Ci <= 0 || Co <= 0 || KH <= 0 || KW <= 0 ||
        stride <= 0 || pad < 0 || dilation <= 0 || act < 0 || act > 2 || ldy < Co)
        return BEV_ERR_ARGS;
    if (Ci % HBK != 0) return BEV_ERR_ARGS;  // one tap and 32 channels per K step
    if (Ho != (H + 2 * pad - dilation * (KH - 1) - 1) / stride + 1 ||
        Wo != (W + 2 * pad - dilation * (KW - 1) - 1) / stride + 1 || Ho <= 0 || Wo <= 0)
        return BEV_ERR_ARGS;
    if ((((uintptr_t)x | (uintptr_t)packed) & 15) != 0) return BEV_ERR_ARGS;
    if (residual && ldy != Co) return BEV_ERR_ARGS;
    // CONV_H16_KERNEL 1 (the 32-deep kernel, A/B) applies only where that kernel can run: epilogue statistics
    // and fp16-stored operands exist on k_conv_h16b alone, so those calls keep it (as the weight gradient does)
    const bool wide = Ci % HBK2 == 0 && (g_h16_kernel != 1 || stats != nullptr || x_half);
    if (stats && (!wide || act != 0 || residual)) return BEV_ERR_ARGS;  // statistics of the raw conv output, k_conv_h16b
    if (x_half && !wide) return BEV_ERR_ARGS;                         // fp16 operands: k_conv_h16b only
    if (x_half && ((uintptr_t)x & 7) != 0) return BEV_ERR_ARGS;
    if (N == 0) return 0;
    ConvH a;
    a.x = x_half ? nullptr : x;
    a.xh = x_half ? (const _Float16 *)xv : nullptr;
    a.wp = (const _Float16 *)packed;
    a.bias = bias;
    a.res = residual;
    a.y = y;
    a.stats = stats;
    a.N = N, a.H = H, a.W = W, a.Ci = Ci, a.Co = Co, a.KH = KH, a.KW = KW, a.stride = stride, a.pad = pad;
    a.dil = dilation, a.Ho = Ho, a.Wo = Wo, a.act = act, a.ldy = ldy;
    a.Kp = (int)kpad_h(Ci * KH * KW);
    a.M = (int64_t)N * Ho * Wo;
    // 64-column tiles for Co <= 64 (2: the 128-column tile always; 3: 64-column tiles always -- A/B, same results)
    const bool n64 = wide && ((Co <= 64 && g_h16_kernel != 2) || g_h16_kernel == 3);
    const int64_t blocks = ((a.M + HBM - 1) / HBM) * (n64 ? (Co + 63) / 64 : (Co + HBN - 1) / HBN);
    if (blocks >= ((int64_t)1 << 31)) return BEV_ERR_ARGS;
    const dim3 g((unsigned)blocks), b(256);
    hipStream_t st = (hipStream_t)stream;
    if (wide) {
        // 32-bit buffer offsets: operand and panel below 2 GiB (every in-image byte offset, and the out-of-range
        // sentinel 2^31 above them all)
        const bool buf = H16B_BUF && H16B_LINES && x_half &&
                         (int64_t)N * H * W * Ci * 2 < ((int64_t)1 << 31) - 16 &&
                         copad_h(Co) * (int64_t)a.Kp * 2 < ((int64_t)1 << 31) - 16;
        void (*kern)(ConvH) = n64 ? (x_half ? (buf ? k_conv_h16b<true, 64, true> : k_conv_h16b<true, 64>)
                                            : k_conv_h16b<false, 64>)
                                  : (x_half ? (buf ? k_conv_h16b<true, 128, true> : k_conv_h16b<true, 128>)
                                            : k_conv_h16b<false, 128>);
        hipLaunchKernelGGL(kern, g, b, 0, st, a);
    }
    else
        hipLaunchKernelGGL(k_conv_h16, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a);
    return (int)hipGetLastError();
}

int bev_conv2d_h16_f32(const float *x, int N, int H, int W, int Ci, const uint16_t *packed, const float *bias,
                       const float *residual, int Co, int KH, int KW, int stride, int pad, int dilation, int act,
                       float *y, int ldy, int Ho, int Wo, void *stream) {
    return conv_h16(x, 0, N, H, W, Ci, packed, bias, residual, Co, KH, KW, stride, pad, dilation, act, y, ldy, Ho, Wo,
                    nullptr, stream);
}

int64_t bev_conv_h16_stat_tiles(int64_t M) { return M > 0 ? (M + HBM - 1) / HBM : BEV_ERR_ARGS; }

int bev_conv2d_h16_bnstats_f32(const float *x, int N, int H, int W, int Ci, const uint16_t *packed, const float *bias,
                               int Co, int KH, int KW, int stride, int pad, int dilation, float *y, int Ho, int Wo,
                               float *tile_stats, void *stream) {
    if (!tile_stats) return BEV_ERR_ARGS;
    return conv_h16(x, 0, N, H, W, Ci, packed, bias, nullptr, Co, KH, KW, stride, pad, dilation, 0, y, Co, Ho, Wo,
                    tile_stats, stream);
}

int bev_conv2d_h16_ex_f32(const void *x, int x_half, int N, int H, int W, int Ci, const uint16_t *packed,
                          const float *bias, const float *residual, int Co, int KH, int KW, int stride, int pad,
                          int dilation, int act, float *y, int ldy, int Ho, int Wo, float *tile_stats, void *stream) {
    return conv_h16(x, x_half, N, H, W, Ci, packed, bias, residual, Co, KH, KW, stride, pad, dilation, act, y, ldy, Ho,
                    Wo, tile_stats, stream);
}

}  // extern "C"
