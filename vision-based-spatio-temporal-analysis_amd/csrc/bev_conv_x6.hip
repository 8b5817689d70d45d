// bev_conv_x6.hip -- fp32 convolutions on the bf16 matrix cores through an exact three-way operand split.
//
// Same contract as bev_conv2d_f32 (the timm trunk convs of CNNEncoder._encode_single, cnn_encoder.py:26,41-46):
//     y[m][n] = act( sum_k A[m][k] * W[k][n] + bias[n] (+ res[m][n]) )
// with fp32 operands and fp32 accumulation.  Every fp32 value v is written EXACTLY as the sum of three bf16
// values by round-to-nearest-even splitting:
//     h = bf16(v),  m = bf16(v - h),  l = bf16(v - h - m)        v == h + m + l  (8 + 8 + 8 significand bits;
// both subtractions are exact in fp32 because each residual is a multiple of ulp(v) below half an ulp of the
// previous term), |m| <= 2^-9 |v|, |l| <= 2^-18 |v|.  A product a*b is then the sum of nine bf16 x bf16
// products, each EXACT in fp32; the six kept here are those larger than 2^-27 |a b|:
//     hh + hm + mh + hl + lh + mm          (dropped: ml + lm + ll <= 2^-26 |a b|, below fp32's 2^-24 rounding)
// and all of them accumulate into the fp32 MFMA accumulator.  The result is an fp32 GEMM whose per-product error
// (<= 2^-26 relative) is below the fp32 rounding of the running sum it is added to, so it is exactly as accurate as
// the exact-f32 MFMA path (tests/test_conv_x6_gpu.py measures both against float64), at 6 bf16 MFMAs per 16-deep
// k slice instead of 8 fp32 32x32x2 MFMAs per 16: v_mfma_f32_32x32x16_bf16 is 32 cycles, v_mfma_f32_32x32x2_f32
// 64 (MI355X_MICROARCH.md), so the matrix-core time per output falls from 512 to 192 cycles (2.67x).
// Summation order differs from the fp32 kernel: fp32-tolerance equal, not bitwise.
//
// Implicit GEMM, m = (image, oy, ox), n = output channel, k = (ky, kx, ci), NHWC activations with Ci % 16 == 0
// (a K step = one tap and 16 consecutive channels), or the dual-source 1x1 form of bev_conv2d_dual_f32 (bottleneck
// conv3 + downsample shortcut as one GEMM over K = [h | x[::s]]).  256 threads = WM x WN waves, each TM x TN MFMA
// tiles of 32 x 32.  Per K step the block stages A (global fp32 -> registers -> split -> three bf16 LDS planes) and
// B (weights split once at pack time: panel [Co_pad][K_pad / 16][3][16] bf16, one 96-B run per row and step);
// LDS rows of 24 bf16 (48 B = 3 odd 16-B slots: the 16-lane ds_read_b128 fragment groups are conflict-free);
// double-buffered LDS, two register sets prefetched two K steps ahead, one barrier per step.  Fragment map
// (cdna_hip_programming.md §3): lane l holds A[row l & 31][k 8 (l >> 5) + j] and B[k 8 (l >> 5) + j][col l & 31].
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/bev_mi355x.h"
#include "bev_act.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

// pre-split chains without a fused next conv: 1 = conv3 transposed (x6_chain_epilogue_t), 0 = x6_chain_epilogue.
// r06m A/B (7 x 1080p ResNet-50 encoder): the transposed epilogue's per-pixel float4 residual loads / y stores (32
// rows x 32 B per instruction) cost ~0.1 ms per launch over the row-contiguous dword form, so only the chains that
// run the next conv (NT3 > 0, which needs the transposed layout) take it.
#ifndef X6S_T_EPI
#define X6S_T_EPI 0
#endif
#ifndef X6S_ABLATE
#define X6S_ABLATE 0  // timing builds only (chains) (wrong results): 1 no chain epilogue, 2 no mainloop MFMAs, 4 no operand DMA
#endif
constexpr int XBK = 16;   // K step
constexpr int XROW = 24;  // bf16 per LDS row (48 B)

__device__ __attribute__((aligned(16))) float g_xzero4[4] = {0.f, 0.f, 0.f, 0.f};  // never written

__host__ __device__ inline int64_t kpad_x(int K) { return (K + XBK - 1) / XBK * XBK; }
__host__ __device__ inline int64_t copad_x(int Co) { return (Co + 127) / 128 * 128; }

// v == h + m + l exactly (see the header); RNE conversions (v_cvt_pk_bf16_f32), exact fp32 residuals.
__device__ __forceinline__ void split3(float v, __bf16 &h, __bf16 &m, __bf16 &l) {
    h = (__bf16)v;
    const float r = v - (float)h;
    m = (__bf16)r;
    l = (__bf16)(r - (float)m);
}

// OIHW fp32 -> split panel in MFMA B-fragment order: [Co_pad / 32][K_pad / 16][plane h, m, l][lane 64][8] bf16,
// lane l of the (32-column block, 16-deep slice, plane) fragment holds W[32 cb + (l & 31)][16 s + 8 (l >> 5) + j],
// j = 0..7 -- one coalesced 1-KiB load per wave and fragment (k = (ky*KW + kx)*Ci + ci).
__host__ __device__ inline int64_t frag_index(int n, int k, int p, int64_t S) {
    return (((int64_t)(n >> 5) * S + (k >> 4)) * 3 + p) * 512 + (((k >> 3) & 1) * 32 + (n & 31)) * 8 + (k & 7);
}

__global__ void k_pack_x6(const float *__restrict__ w, int Co, int Ci, int KH, int KW, int64_t Kp, int64_t Cop,
                          __bf16 *__restrict__ out) {
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
    __bf16 h, m, l;
    split3(v, h, m, l);
    const int64_t S = Kp / XBK;
    out[frag_index(n, k, 0, S)] = h;
    out[frag_index(n, k, 1, S)] = m;
    out[frag_index(n, k, 2, S)] = l;
}

struct ConvX {
    const float *__restrict__ x;
    const __bf16 *__restrict__ wp;
    const float *__restrict__ bias;
    const float *__restrict__ res;
    float *__restrict__ y;
    int N, H, W, Ci, Co, KH, KW, stride, pad, dil, Ho, Wo, act, ldy, Kp;
    int64_t M;
    // dual-source 1x1: k in [Ci, Ci + Ci2) reads x2 [N][H2][W2][Ci2] at (oy*stride2, ox*stride2)
    const float *__restrict__ x2;
    int Ci2, H2, W2, stride2;
    // pre-split operand / output planes: xs [3][N][H][W][Ci], ys [3][M][Co] bf16 (plane strides xps / yps)
    const __bf16 *__restrict__ xs;
    __bf16 *__restrict__ ys;
    int64_t xps, yps;
    // chained pointwise conv (k_conv_x6b CHAIN): y = act2(h (*) W2 + bias2 + res), h = act(this conv + bias)
    const __bf16 *__restrict__ wp2;
    const float *__restrict__ bias2;
    int Co2, act2;
    int nta = 0;  // 1: A (activation) loads non-temporal (BEV_TUNE_CONV_X6_NT, the last layer of a trunk)
    // the next block's 1x1 conv fused into a chain's epilogue (x6_chain_epilogue_t NT3 > 0): h3 = act3(y (*) W3 + b3)
    // from the block output y the chain just computed, written split (ys3 [3][M][Co3] bf16) or fp32 (y3 [M][Co3])
    const __bf16 *__restrict__ wp3 = nullptr;
    const float *__restrict__ bias3 = nullptr;
    __bf16 *__restrict__ ys3 = nullptr;
    float *__restrict__ y3 = nullptr;
    int Co3 = 0, act3 = 0;
};

__device__ __forceinline__ float act_x(float t, int act) {
    if (act == 2) return silu_hw(t);
    if (act == 1) return t > 0.0f ? t : 0.0f;
    return t;
}

// The wave's (TM*32) x (TN*32) accumulator tile goes through LDS, 32 rows per pass (4 * 32 * (TN * 32 + 4) floats
// for the block), so every lane stores whole float4 row pieces; each pass issues all its residual loads at once (the
// memory-bound 1x1 layers).  Same scheme as bev_conv.hip's epilogue.  With a.ys the result is stored split.
template <int TN>
__host__ __device__ constexpr int x6_epi_bytes() { return 4 * 32 * (TN * 32 + 4) * 4; }

template <int TM, int TN>
__device__ __forceinline__ void x6_epilogue(const ConvX &a, float *lds, const f32x16 (&acc)[TM][TN], int wave,
                                            int lane, int wn, int wm, int64_t m0, int n0) {
    const int r32 = lane & 31, h = lane >> 5;
    constexpr int WC = TN * 32, ER = WC + 4;
    constexpr int C4 = WC / 4, RPI = 64 / C4, NQ = 32 / RPI;
    float *E = lds + wave * (32 * ER);
    const int c4 = lane % C4, rq = lane / C4;
    const int n = n0 + wn * WC + c4 * 4;
    const bool nvec = ((a.Co & 3) == 0) && ((a.ldy & 3) == 0) && (n + 3 < a.Co);
    // each pass's residual loads go out before its LDS traffic (the first pass's before the barrier)
    float4 rv[NQ];
    auto res_load = [&](int i) {
        const int64_t mb = m0 + wm * TM * 32 + i * 32;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int64_t m = mb + rq + RPI * q;
            rv[q] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (a.res && m < a.M && nvec) rv[q] = *(const float4 *)(a.res + m * a.Co + n);
        }
    };
    res_load(0);
    __syncthreads();  // every wave is done with the staging buffers
    float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.bias) {
        if (nvec) bv = *(const float4 *)(a.bias + n);
        else {
            bv.x = n < a.Co ? a.bias[n] : 0.f;
            bv.y = n + 1 < a.Co ? a.bias[n + 1] : 0.f;
            bv.z = n + 2 < a.Co ? a.bias[n + 2] : 0.f;
            bv.w = n + 3 < a.Co ? a.bias[n + 3] : 0.f;
        }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        // same-wave LDS operations complete in order: the previous pass's reads precede these writes
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) E[((r & 3) + 8 * (r >> 2) + 4 * h) * ER + j * 32 + r32] = acc[i][j][r];
        const int64_t mbase = m0 + wm * TM * 32 + i * 32;
        if (i > 0) res_load(i);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int row = rq + RPI * q;
            const int64_t m = mbase + row;
            if (m >= a.M) continue;
            const float4 v = *(const float4 *)(E + row * ER + c4 * 4);
            float o[4] = {v.x + bv.x, v.y + bv.y, v.z + bv.z, v.w + bv.w};
            if (a.ys) {  // split output planes (the next conv's pre-split operand); ldy == Co, Co % 4 == 0
                if (a.res) {
                    const float4 rr = rv[q];
                    o[0] += rr.x, o[1] += rr.y, o[2] += rr.z, o[3] += rr.w;
                }
                bf16x4 hv, mv, lv;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    __bf16 h_, m_, l_;
                    split3(act_x(o[u], a.act), h_, m_, l_);
                    hv[u] = h_, mv[u] = m_, lv[u] = l_;
                }
                __bf16 *yp = a.ys + m * a.Co + n;
                if (n < a.Co) {
                    *(bf16x4 *)yp = hv;
                    *(bf16x4 *)(yp + a.yps) = mv;
                    *(bf16x4 *)(yp + 2 * a.yps) = lv;
                }
                continue;
            }
            float *yp = a.y + m * a.ldy + n;
            if (nvec) {
                if (a.res) {
                    o[0] += rv[q].x;
                    o[1] += rv[q].y;
                    o[2] += rv[q].z;
                    o[3] += rv[q].w;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) o[u] = act_x(o[u], a.act);
                *(float4 *)yp = make_float4(o[0], o[1], o[2], o[3]);
            } else {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (n + u >= a.Co) break;
                    float t = o[u];
                    if (a.res) t += a.res[m * a.Co + n + u];
                    yp[u] = act_x(t, a.act);
                }
            }
        }
    }
}

template <int WM, int WN, int TM, int TN, bool DUAL>
__global__ __launch_bounds__(256, 2) void k_conv_x6(ConvX a) {
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
    constexpr int APL = BM * XROW, BPL = BN * XROW;  // bf16 per operand plane
    constexpr int STAGE = 3 * (APL + BPL);            // bf16 per LDS stage
    constexpr int AQ = BM / 64;                       // A float4 per thread and K step: rows tid / 4 + 64 q
    // B staging: the step's BN rows x 96 B in pieces of PB bytes (16, or 8 when 16-B pieces do not divide evenly
    // over the 256 threads), BQ whole pieces per thread -- no conditional loads
    constexpr int PB = ((BN * 6) % 256 == 0) ? 16 : 8;
    constexpr int PPR = 96 / PB;  // pieces per row
    constexpr int BQ = BN * PPR / 256;
    static_assert(BN * PPR % 256 == 0, "B pieces per thread");
    typedef typename std::conditional<PB == 16, u32x4, u32x2>::type bpiece;  // native vectors stay in VGPRs
    constexpr int EPIB = x6_epi_bytes<TN>();
    constexpr int LDSB = (2 * STAGE * 2 > EPIB) ? 2 * STAGE * 2 : EPIB;
    static_assert(BM % 64 == 0, "A staging rows");
    __shared__ __attribute__((aligned(16))) unsigned char lds_raw[LDSB];
    __bf16 *lds = (__bf16 *)lds_raw;

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
    const int wm = wave / WN, wn = wave % WN;
    const int n_tiles = (a.Co + BN - 1) / BN;
    unsigned bid = blockIdx.x;
    {  // XCD-aware order: the n_tiles blocks reading the same A rows run on one XCD (shared L2)
        const unsigned nb = gridDim.x, q = nb / 8, r = nb % 8, xc = bid % 8;
        bid = (xc < r ? xc * (q + 1) : r * (q + 1) + (xc - r) * q) + bid / 8;
    }
    const int64_t m0 = (int64_t)(bid / n_tiles) * BM;
    const int n0 = (bid % n_tiles) * BN;

    // A staging rows: (tid >> 2) + 64 q, channel quad aq of the 16-channel K step
    const int aq = tid & 3;
    int64_t pb[AQ], p2[AQ];
    int iy0[AQ], ix0[AQ];
    bool rok[AQ];
#pragma unroll
    for (int q = 0; q < AQ; ++q) {
        const int64_t m = m0 + (tid >> 2) + 64 * q;
        rok[q] = m < a.M;
        const int64_t mm = rok[q] ? m : 0;
        const int ox = (int)(mm % a.Wo);
        const int64_t t = mm / a.Wo;
        const int oy = (int)(t % a.Ho);
        const int64_t n = t / a.Ho;
        if (DUAL) {
            pb[q] = mm * a.Ci + 4 * aq;
            p2[q] = ((n * a.H2 + (int64_t)oy * a.stride2) * a.W2 + (int64_t)ox * a.stride2) * a.Ci2 + 4 * aq;
            iy0[q] = ix0[q] = 0;
        } else {
            pb[q] = n * a.H * a.W * a.Ci + 4 * aq;
            p2[q] = 0;
            iy0[q] = oy * a.stride - a.pad;
            ix0[q] = ox * a.stride - a.pad;
        }
    }
    const int64_t bstep = 3 * 512;  // bf16 per 16-deep slice of a 32-column block (fragment-order panel)
    const __bf16 *brow[BQ];
    int bdst[BQ];  // LDS offset (bf16) of the piece inside the B part of a stage
#pragma unroll
    for (int i = 0; i < BQ; ++i) {
        const int pc = tid + 256 * i;
        const int row = pc / PPR, byte = (pc % PPR) * PB;  // byte of the row's 96-B (plane, 16 k) run
        const int pl = byte / 32, hk = (byte % 32) / 16, sub = (byte % 16) / 2;
        brow[i] = a.wp + frag_index(n0 + row, 8 * hk, pl, a.Kp / XBK) + sub;
        bdst[i] = pl * BPL + row * XROW + 8 * hk + sub;
    }
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){0};

    f32x4 va0[AQ], va1[AQ];
    bpiece vb0[BQ], vb1[BQ];
    int ky = 0, kx = 0, ci0 = 0, k0 = 0;  // tap / channel (or dual k) of the step being loaded
    int64_t kb = 0;                       // bf16 offset of that step in a panel row
#define X6_GLOAD(VA, VB)                                                                                   \
    do {                                                                                                   \
        if (DUAL) {                                                                                        \
            const bool first = k0 < a.Ci;                                                                  \
            const float *src = first ? a.x + k0 : a.x2 + (k0 - a.Ci);                                      \
            _Pragma("unroll") for (int q = 0; q < AQ; ++q) VA[q] =                                         \
                *(const f32x4 *)(rok[q] ? src + (first ? pb[q] : p2[q]) : g_xzero4);                      \
            k0 += XBK;                                                                                     \
        } else {                                                                                           \
            const int dy = ky * a.dil, dx = kx * a.dil;                                                    \
            _Pragma("unroll") for (int q = 0; q < AQ; ++q) {                                               \
                const int iy = iy0[q] + dy, ix = ix0[q] + dx;                                              \
                const bool in = rok[q] && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;    \
                VA[q] = *(const f32x4 *)(in ? a.x + pb[q] + ((int64_t)iy * a.W + ix) * a.Ci + ci0 : g_xzero4); \
            }                                                                                              \
            ci0 += XBK;                                                                                    \
            if (ci0 == a.Ci) {                                                                             \
                ci0 = 0;                                                                                   \
                if (++kx == a.KW) {                                                                        \
                    kx = 0;                                                                                \
                    ++ky;                                                                                  \
                }                                                                                          \
            }                                                                                              \
        }                                                                                                  \
        _Pragma("unroll") for (int i = 0; i < BQ; ++i) VB[i] = *(const bpiece *)(brow[i] + kb);          \
        kb += bstep;                                                                                       \
    } while (0)
#define X6_SWRITE(BUF, VA, VB)                                                                             \
    do {                                                                                                   \
        __bf16 *As = lds + (BUF) * STAGE;                                                                  \
        __bf16 *Bs = As + 3 * APL;                                                                         \
        _Pragma("unroll") for (int q = 0; q < AQ; ++q) {                                                   \
            bf16x4 hv, mv, lv;                                                                             \
            _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                                \
                __bf16 h_, m_, l_;                                                                         \
                split3(VA[q][e], h_, m_, l_);                                                              \
                hv[e] = h_;                                                                                \
                mv[e] = m_;                                                                                \
                lv[e] = l_;                                                                                \
            }                                                                                              \
            __bf16 *d = As + ((tid >> 2) + 64 * q) * XROW + 4 * aq;                                        \
            *(bf16x4 *)d = hv;                                                                             \
            *(bf16x4 *)(d + APL) = mv;                                                                     \
            *(bf16x4 *)(d + 2 * APL) = lv;                                                                 \
        }                                                                                                  \
        _Pragma("unroll") for (int i = 0; i < BQ; ++i) *(bpiece *)(Bs + bdst[i]) = VB[i];                \
    } while (0)
    const int r32 = lane & 31, h = lane >> 5;
    // one 16-deep k slice: 6 MFMAs per (A tile, B tile) pair (hh, hm, mh, hl, lh, mm)
#define X6_MFMA(BUF)                                                                                       \
    do {                                                                                                   \
        const __bf16 *As = lds + (BUF) * STAGE;                                                            \
        const __bf16 *Bs = As + 3 * APL;                                                                   \
        bf16x8 fa[TM][3], fb[TN][3];                                                                       \
        _Pragma("unroll") for (int i = 0; i < TM; ++i)                                                     \
            _Pragma("unroll") for (int p = 0; p < 3; ++p)                                                  \
                fa[i][p] = *(const bf16x8 *)(As + p * APL + (wm * TM * 32 + i * 32 + r32) * XROW + 8 * h); \
        _Pragma("unroll") for (int j = 0; j < TN; ++j)                                                     \
            _Pragma("unroll") for (int p = 0; p < 3; ++p)                                                  \
                fb[j][p] = *(const bf16x8 *)(Bs + p * BPL + (wn * TN * 32 + j * 32 + r32) * XROW + 8 * h); \
        _Pragma("unroll") for (int i = 0; i < TM; ++i)                                                     \
            _Pragma("unroll") for (int j = 0; j < TN; ++j) {                                               \
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][0], acc[i][j], 0, 0, 0); \
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][1], acc[i][j], 0, 0, 0); \
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[j][0], acc[i][j], 0, 0, 0); \
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][2], acc[i][j], 0, 0, 0); \
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][2], fb[j][0], acc[i][j], 0, 0, 0); \
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[j][1], acc[i][j], 0, 0, 0); \
            }                                                                                              \
    } while (0)

    const int nk = a.Kp / XBK;
    X6_GLOAD(va0, vb0);
    if (nk > 1) X6_GLOAD(va1, vb1);
    X6_SWRITE(0, va0, vb0);
    __syncthreads();
    // Invariant at the loop head: LDS buffer 0 holds step ks, register set 1 holds step ks + 1.
    int ks = 0;
    for (; ks + 3 < nk; ks += 2) {
        X6_GLOAD(va0, vb0);  // step ks + 2
        X6_MFMA(0);
        X6_SWRITE(1, va1, vb1);  // step ks + 1 (buffer 1's readers passed the last barrier)
        __syncthreads();
        X6_GLOAD(va1, vb1);  // step ks + 3
        X6_MFMA(1);
        X6_SWRITE(0, va0, vb0);  // step ks + 2
        __syncthreads();
    }
    if (ks + 2 < nk) {
        X6_GLOAD(va0, vb0);
        X6_MFMA(0);
        X6_SWRITE(1, va1, vb1);
        __syncthreads();
        X6_MFMA(1);
        X6_SWRITE(0, va0, vb0);
        __syncthreads();
        X6_MFMA(0);
    } else if (ks + 1 < nk) {
        X6_MFMA(0);
        X6_SWRITE(1, va1, vb1);
        __syncthreads();
        X6_MFMA(1);
    } else {
        X6_MFMA(0);
    }
#undef X6_MFMA
#undef X6_SWRITE
#undef X6_GLOAD
    x6_epilogue<TM, TN>(a, (float *)lds_raw, acc, wave, lane, wn, wm, m0, n0);
}

// ---------------------------------------------------------------------------
// Chained bottleneck body in the split arithmetic (bev_conv2d_chain_x6_f32): timm Bottleneck without a downsample,
// act3(bn3(conv3(act2(bn2(conv2(h1))))) + x).  The block's BM x BN tile of h2 = act(conv2 + b2) holds EVERY channel
// of h2 for its BM pixels (BN == Co), so it is split once into three bf16 planes in LDS ([3][BM][BN + 8]: rows of
// odd 16-B slot counts) and conv3 (1x1, K2 = BN) runs on it there: h2 never makes its HBM round trip.  Wave w takes
// rows 32 w .. 32 w + 31 and walks Co2 in 64-column chunks (2 MFMA tiles); the W3 fragments come from the
// fragment-order panel by buffer loads (SGPR soffset); the chunk's residual is loaded before its MFMAs; residual and
// output are addressed by buffer instructions (row in the VGPR offset, so rows past M read 0 / are dropped).
// ---------------------------------------------------------------------------
__device__ __forceinline__ __amdgpu_buffer_rsrc_t x6_rsrc(const void *p, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, (int)(uint32_t)bytes, 0x00020000);
}

// X2S > 0: the dual form (block 0 of a stage, bev_conv2d_chain_dual_x6_f32): conv3's K continues with the X2S
// 16-deep slices of the shortcut operand x2 at the lane row's strided pixel (the 1x1 downsample), split in registers
// once per wave and reused by every chunk; the panel is the dual tail's [W3 | Wds].
template <int WM, int WN, int TM, int TN, int X2S = 0>
__device__ __forceinline__ void x6_chain_epilogue(const ConvX &a, unsigned char *lds_raw, const f32x16 (&acc)[TM][TN],
                                                  int wave, int lane, int wm, int wn, int64_t m0) {
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32, HR = BN + 8, HPL = BM * HR;
    constexpr int NB = BM / 32, WPB = 4 / NB;  // 32-row bands; waves per band (each a share of the Co2 chunks)
    static_assert(NB * WPB == 4, "chain epilogue: 4 waves over the 32-row bands");
    __bf16 *H = (__bf16 *)lds_raw;
    const int r32 = lane & 31, hh = lane >> 5;
    // residual of this wave's first chunk: requested before the h2 staging, so its latency overlaps it
    const int band = (wave % NB) * 32, part = wave / NB;
    const int64_t rows = (a.M - m0 < BM) ? a.M - m0 : BM;
    const int64_t base = m0 * a.Co2;
    const __amdgpu_buffer_rsrc_t rr = x6_rsrc(a.res ? a.res + base : a.y + base, rows * a.Co2 * 4);
    const int vo = ((band + 4 * hh) * a.Co2 + r32) * 4;  // lane part of a res / y address
    const int nch = a.Co2 / 64 / WPB;                     // this wave's 64-column chunks: [part * nch, (part + 1) * nch)
    float rvn[2][16];
    auto res_load = [&](int c0) {
        if (!a.res) return;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                rvn[j][r] = __builtin_bit_cast(
                    float, __builtin_amdgcn_raw_buffer_load_b32(rr, vo + ((r & 3) + 8 * (r >> 2)) * a.Co2 * 4,
                                                                (c0 + 32 * j) * 4, 0));
    };
    res_load(64 * part * nch);
    __syncthreads();  // every wave is done with the staging buffers
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = wn * TN * 32 + j * 32 + r32;
            const float bj = a.bias ? a.bias[col] : 0.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                __bf16 h_, m_, l_;
                split3(act_x(acc[i][j][r] + bj, a.act), h_, m_, l_);
                const int row = wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
                H[row * HR + col] = h_;
                H[HPL + row * HR + col] = m_;
                H[2 * HPL + row * HR + col] = l_;
            }
        }
    __syncthreads();
    constexpr int S2 = BN / 16;      // 16-deep slices of conv3's K from h2
    constexpr int ST = S2 + X2S;     // slices of the panel
    bf16x8 fx[X2S > 0 ? X2S : 1][3];  // the shortcut operand, split (dual form)
    if constexpr (X2S > 0) {
        int64_t m = m0 + band + r32;
        const bool ok = m < a.M;
        m = ok ? m : 0;
        const int ox = (int)(m % a.Wo);
        const int64_t q = m / a.Wo;
        const int oy = (int)(q % a.Ho);
        const int64_t n = q / a.Ho;
        const float *xp = a.x2 + ((n * a.H2 + (int64_t)oy * a.stride2) * a.W2 + (int64_t)ox * a.stride2) * a.Ci2 + 8 * hh;
#pragma unroll
        for (int t = 0; t < X2S; ++t) {
            f32x4 v0 = ok ? *(const f32x4 *)(xp + 16 * t) : (f32x4){0.f, 0.f, 0.f, 0.f};
            f32x4 v1 = ok ? *(const f32x4 *)(xp + 16 * t + 4) : (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                __bf16 h_, m_, l_;
                split3(e < 4 ? v0[e] : v1[e - 4], h_, m_, l_);
                fx[t][0][e] = h_, fx[t][1][e] = m_, fx[t][2][e] = l_;
            }
        }
    }
    const __bf16 *ap = H + (band + r32) * HR + 8 * hh;
    const __amdgpu_buffer_rsrc_t ry = x6_rsrc(a.y + base, rows * a.Co2 * 4);
    const __amdgpu_buffer_rsrc_t rw = x6_rsrc(a.wp2, copad_x(a.Co2) / 32 * (int64_t)ST * 3072);
    const int vl = lane * 16;
    for (int nc = part * nch; nc < (part + 1) * nch; ++nc) {
        const int c0 = 64 * nc;
        float rv[2][16];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) rv[j][r] = rvn[j][r];
        if (nc + 1 < (part + 1) * nch) res_load(c0 + 64);  // the next chunk's residual, during these MFMAs
        f32x16 acc2[2] = {(f32x16){0}, (f32x16){0}};
#pragma unroll
        for (int t = 0; t < ST; ++t) {
            bf16x8 fa[3], fb[2][3];
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                if constexpr (X2S > 0) fa[p] = t < S2 ? *(const bf16x8 *)(ap + p * HPL + 16 * (t < S2 ? t : 0))
                                                      : fx[t >= S2 ? t - S2 : 0][p];
                else fa[p] = *(const bf16x8 *)(ap + p * HPL + 16 * t);
            }
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    fb[j][p] = __builtin_bit_cast(
                        bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, vl, (((c0 >> 5) + j) * ST + t) * 3072 + p * 1024, 0));
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                acc2[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[j][0], acc2[j], 0, 0, 0);
                acc2[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[j][1], acc2[j], 0, 0, 0);
                acc2[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[j][0], acc2[j], 0, 0, 0);
                acc2[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[j][2], acc2[j], 0, 0, 0);
                acc2[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2], fb[j][0], acc2[j], 0, 0, 0);
                acc2[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[j][1], acc2[j], 0, 0, 0);
            }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const float bj = a.bias2 ? a.bias2[c0 + 32 * j + r32] : 0.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                float o = acc2[j][r] + bj;
                if (a.res) o += rv[j][r];
                o = act_x(o, a.act2);
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o), ry,
                                                      vo + ((r & 3) + 8 * (r >> 2)) * a.Co2 * 4, (c0 + 32 * j) * 4, 0);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// The chain epilogue with conv3 computed TRANSPOSED (x6_chain_epilogue_t, the pre-split chains of k_conv_x6s):
// D^T = W3^T h2^T -- the same fragments as x6_chain_epilogue with the MFMA operands swapped (A = the W3 panel
// fragment, rows = output channels; B = the h2 fragment, columns = the band's 32 pixels) and the six products issued
// in the same order, so every output element accumulates the same products in the same sequence.  Lane (p, hh)
// then holds pixel band + p, channels c0 + 32 j + 8 g + 4 hh + u (g, u = 0..3) of the chunk: the residual and the
// output move as float4 (four per tile and lane instead of sixteen dwords), and -- NT3 > 0 -- the block output y is
// already the B operand of the NEXT block's 1x1 conv (h3 = act3(y (*) W3' + b3), Co3 = 32 NT3 output channels):
// per 16-deep slice a lane keeps one 4-channel group of each plane and trades the other with lane p + 32 (one
// __shfl_xor per plane and dword), so the next conv runs on y straight from registers -- its launch, its HBM read of
// y (1 KiB per pixel in layer1) and its operand split per N tile disappear.  h3 leaves split (ys3) or fp32 (y3).
// Same K order per output as the stand-alone conv (slices ascending, six products per slice).  Needs every Co2 chunk
// of a band in one wave (WPB == 1: the 128-row tiles).
template <int WM, int WN, int TM, int TN, int X2S = 0, int NT3 = 0>
__device__ __forceinline__ void x6_chain_epilogue_t(const ConvX &a, unsigned char *lds_raw,
                                                    const f32x16 (&acc)[TM][TN], int wave, int lane, int wm, int wn,
                                                    int64_t m0) {
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32, HR = BN + 8, HPL = BM * HR;
    constexpr int NB = BM / 32, WPB = 4 / NB;
    static_assert(NB * WPB == 4, "chain epilogue: 4 waves over the 32-row bands");
    static_assert(NT3 == 0 || WPB == 1, "the fused next conv needs all of a band's Co2 chunks in one wave");
    __bf16 *H = (__bf16 *)lds_raw;
    const int r32 = lane & 31, hh = lane >> 5;
    const int band = (wave % NB) * 32, part = wave / NB;
    const int64_t rows = (a.M - m0 < BM) ? a.M - m0 : BM;
    const int64_t base = m0 * a.Co2;
    const __amdgpu_buffer_rsrc_t rr = x6_rsrc(a.res ? a.res + base : a.y + base, rows * a.Co2 * 4);
    const int vrow = (band + r32) * a.Co2 * 4 + 16 * hh;  // this lane's pixel row + its 4-channel half (bytes)
    const int nch = a.Co2 / 64 / WPB;
    f32x4 rvn[2][4];
    auto res_load = [&](int c0) {
        if (!a.res) return;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g)
                rvn[j][g] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, vrow + 32 * g,
                                                                                           (c0 + 32 * j) * 4, 0));
    };
    res_load(64 * part * nch);
    __syncthreads();  // every wave is done with the staging buffers
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = wn * TN * 32 + j * 32 + r32;
            const float bj = a.bias ? a.bias[col] : 0.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                __bf16 h_, m_, l_;
                split3(act_x(acc[i][j][r] + bj, a.act), h_, m_, l_);
                const int row = wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
                H[row * HR + col] = h_;
                H[HPL + row * HR + col] = m_;
                H[2 * HPL + row * HR + col] = l_;
            }
        }
    __syncthreads();
    constexpr int S2 = BN / 16;
    constexpr int ST = S2 + X2S;
    bf16x8 fx[X2S > 0 ? X2S : 1][3];
    if constexpr (X2S > 0) {
        int64_t m = m0 + band + r32;
        const bool ok = m < a.M;
        m = ok ? m : 0;
        const int ox = (int)(m % a.Wo);
        const int64_t q = m / a.Wo;
        const int oy = (int)(q % a.Ho);
        const int64_t n = q / a.Ho;
        const float *xp = a.x2 + ((n * a.H2 + (int64_t)oy * a.stride2) * a.W2 + (int64_t)ox * a.stride2) * a.Ci2 + 8 * hh;
#pragma unroll
        for (int t = 0; t < X2S; ++t) {
            f32x4 v0 = ok ? *(const f32x4 *)(xp + 16 * t) : (f32x4){0.f, 0.f, 0.f, 0.f};
            f32x4 v1 = ok ? *(const f32x4 *)(xp + 16 * t + 4) : (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                __bf16 h_, m_, l_;
                split3(e < 4 ? v0[e] : v1[e - 4], h_, m_, l_);
                fx[t][0][e] = h_, fx[t][1][e] = m_, fx[t][2][e] = l_;
            }
        }
    }
    const __bf16 *ap = H + (band + r32) * HR + 8 * hh;
    const __amdgpu_buffer_rsrc_t ry = x6_rsrc(a.y + base, rows * a.Co2 * 4);
    const __amdgpu_buffer_rsrc_t rw = x6_rsrc(a.wp2, copad_x(a.Co2) / 32 * (int64_t)ST * 3072);
    const int vl = lane * 16;
    constexpr int N3 = NT3 > 0 ? NT3 : 1;
    const int S3 = a.Co2 / 16;  // 16-deep slices of the fused conv's K (= Co2)
    const __amdgpu_buffer_rsrc_t rw3 = x6_rsrc(NT3 > 0 ? a.wp3 : a.wp2, NT3 > 0 ? copad_x(a.Co3) / 32 * (int64_t)S3 * 3072 : 0);
    f32x16 acc3[N3];
#pragma unroll
    for (int q = 0; q < N3; ++q) acc3[q] = (f32x16){0};
    for (int nc = part * nch; nc < (part + 1) * nch; ++nc) {
        const int c0 = 64 * nc;
        f32x4 rv[2][4];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) rv[j][g] = rvn[j][g];
        if (nc + 1 < (part + 1) * nch) res_load(c0 + 64);  // the next chunk's residual, during these MFMAs
        f32x16 acc2[2] = {(f32x16){0}, (f32x16){0}};
#pragma unroll
        for (int t = 0; t < ST; ++t) {
            bf16x8 fh[3], fw[2][3];
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                if constexpr (X2S > 0) fh[p] = t < S2 ? *(const bf16x8 *)(ap + p * HPL + 16 * (t < S2 ? t : 0))
                                                      : fx[t >= S2 ? t - S2 : 0][p];
                else fh[p] = *(const bf16x8 *)(ap + p * HPL + 16 * t);
            }
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    fw[j][p] = __builtin_bit_cast(
                        bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, vl, (((c0 >> 5) + j) * ST + t) * 3072 + p * 1024, 0));
#pragma unroll
            for (int j = 0; j < 2; ++j) {  // x6_chain_epilogue's products, operands swapped
                acc2[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[j][0], fh[0], acc2[j], 0, 0, 0);
                acc2[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[j][1], fh[0], acc2[j], 0, 0, 0);
                acc2[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[j][0], fh[1], acc2[j], 0, 0, 0);
                acc2[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[j][2], fh[0], acc2[j], 0, 0, 0);
                acc2[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[j][0], fh[2], acc2[j], 0, 0, 0);
                acc2[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[j][1], fh[1], acc2[j], 0, 0, 0);
            }
        }
        // y = act2(acc2 + b2 + res): channel c0 + 32 j + 8 g + 4 hh + u of this lane's pixel
        unsigned ys[NT3 > 0 ? 2 : 1][4][3][2];  // NT3: y split, [j][g][plane][2 packed bf16 pairs]
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int c = c0 + 32 * j + 8 * g + 4 * hh;
                const f32x4 bv = a.bias2 ? *(const f32x4 *)(a.bias2 + c) : (f32x4){0.f, 0.f, 0.f, 0.f};
                f32x4 o;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    float t_ = acc2[j][4 * g + u] + bv[u];
                    if (a.res) t_ += rv[j][g][u];
                    o[u] = act_x(t_, a.act2);
                }
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), ry, vrow + 32 * g,
                                                       (c0 + 32 * j) * 4, 0);
                if constexpr (NT3 > 0) {
                    __bf16 hv[4], mv[4], lv[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) split3(o[u], hv[u], mv[u], lv[u]);
                    auto pk = [](__bf16 x0, __bf16 x1) {
                        return (unsigned)__builtin_bit_cast(unsigned short, x0) |
                               ((unsigned)__builtin_bit_cast(unsigned short, x1) << 16);
                    };
                    ys[j][g][0][0] = pk(hv[0], hv[1]), ys[j][g][0][1] = pk(hv[2], hv[3]);
                    ys[j][g][1][0] = pk(mv[0], mv[1]), ys[j][g][1][1] = pk(mv[2], mv[3]);
                    ys[j][g][2][0] = pk(lv[0], lv[1]), ys[j][g][2][1] = pk(lv[2], lv[3]);
                }
            }
        if constexpr (NT3 > 0) {
            // the next conv's K slices of this chunk: (j, sl), channels c0 + 32 j + 16 sl .. + 15.  Lane hh = 0 needs
            // channels 0-7 of the slice (its own group g = 2 sl, the partner's 4-7), hh = 1 needs 8-15 (the partner's
            // group 2 sl + 1, its own 12-15): each lane sends the group it does not keep
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int sl = 0; sl < 2; ++sl) {
                    bf16x8 fy[3];
#pragma unroll
                    for (int p = 0; p < 3; ++p) {
                        const unsigned k0 = ys[j][2 * sl][p][0], k1 = ys[j][2 * sl][p][1];
                        const unsigned q0 = ys[j][2 * sl + 1][p][0], q1 = ys[j][2 * sl + 1][p][1];
                        const unsigned s0 = hh ? k0 : q0, s1 = hh ? k1 : q1;  // the group the partner keeps
                        const unsigned r0 = (unsigned)__shfl_xor((int)s0, 32), r1 = (unsigned)__shfl_xor((int)s1, 32);
                        const u32x4 f = hh ? (u32x4){r0, r1, q0, q1} : (u32x4){k0, k1, r0, r1};
                        fy[p] = __builtin_bit_cast(bf16x8, f);
                    }
                    const int ks = (c0 + 32 * j + 16 * sl) >> 4;  // slice of the next conv's K
#pragma unroll
                    for (int q = 0; q < NT3; ++q) {
                        bf16x8 fw3[3];
#pragma unroll
                        for (int p = 0; p < 3; ++p)
                            fw3[p] = __builtin_bit_cast(
                                bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw3, vl, (q * S3 + ks) * 3072 + p * 1024, 0));
                        acc3[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw3[0], fy[0], acc3[q], 0, 0, 0);
                        acc3[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw3[1], fy[0], acc3[q], 0, 0, 0);
                        acc3[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw3[0], fy[1], acc3[q], 0, 0, 0);
                        acc3[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw3[2], fy[0], acc3[q], 0, 0, 0);
                        acc3[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw3[0], fy[2], acc3[q], 0, 0, 0);
                        acc3[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw3[1], fy[1], acc3[q], 0, 0, 0);
                    }
                }
        }
    }
    if constexpr (NT3 > 0) {  // h3 = act3(acc3 + b3) of this lane's pixel, channels 32 q + 8 g + 4 hh + u
        const int64_t prow = m0 + band + r32;
        if (prow < a.M) {
#pragma unroll
            for (int q = 0; q < NT3; ++q)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int c = 32 * q + 8 * g + 4 * hh;
                    const f32x4 bv = a.bias3 ? *(const f32x4 *)(a.bias3 + c) : (f32x4){0.f, 0.f, 0.f, 0.f};
                    f32x4 o;
#pragma unroll
                    for (int u = 0; u < 4; ++u) o[u] = act_x(acc3[q][4 * g + u] + bv[u], a.act3);
                    if (a.ys3) {
                        bf16x4 hv, mv, lv;
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            __bf16 h_, m_, l_;
                            split3(o[u], h_, m_, l_);
                            hv[u] = h_, mv[u] = m_, lv[u] = l_;
                        }
                        __bf16 *yp = a.ys3 + prow * a.Co3 + c;
                        const int64_t pl = a.M * a.Co3;
                        *(bf16x4 *)yp = hv;
                        *(bf16x4 *)(yp + pl) = mv;
                        *(bf16x4 *)(yp + 2 * pl) = lv;
                    } else {
                        *(f32x4 *)(a.y3 + prow * a.Co3 + c) = o;
                    }
                }
        }
    }
}

// ---------------------------------------------------------------------------
// k_conv_x6b: Ci % 32 == 0 (every ResNet trunk layer).  K step 32 (two 16-deep slices, 48 MFMAs per wave and
// step for a 64 x 64 wave tile: twice the work per barrier of k_conv_x6).  Only A goes through LDS (three bf16
// planes, rows of 40 bf16 = 80 B = 5 odd 16-B slots: conflict-free fragment groups); the B fragments are read
// straight from the fragment-order panel into registers (one coalesced 1-KiB load per fragment and plane), one
// slice ahead of their MFMAs, so the LDS per stage is A's alone (30 KiB for 128 rows).
// ---------------------------------------------------------------------------
constexpr int YBK = 32;
constexpr int YROW = 40;

// CHAIN: 0 none, 1 chain, 2 chain + shortcut; NT: non-temporal activation loads (BEV_TUNE_CONV_X6_NT)
template <int WM, int WN, int TM, int TN, bool DUAL, int CHAIN = 0, bool NT = false>
__global__ __launch_bounds__(256, 2) void k_conv_x6b(ConvX a) {
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
    constexpr int APL = BM * YROW;                 // bf16 per A plane
    constexpr int STAGE = 3 * APL;                 // bf16 per LDS stage
    constexpr int AQ = BM / 32;                    // A float4 per thread and K step: rows tid / 8 + 32 q
    constexpr int EPIB = CHAIN ? 3 * BM * (BN + 8) * 2 : x6_epi_bytes<TN>();
    constexpr int LDSB = (2 * STAGE * 2 > EPIB) ? 2 * STAGE * 2 : EPIB;
    __shared__ __attribute__((aligned(16))) unsigned char lds_raw[LDSB];
    __bf16 *lds = (__bf16 *)lds_raw;

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
    const int wm = wave / WN, wn = wave % WN;
    const int n_tiles = (a.Co + BN - 1) / BN;
    unsigned bid = blockIdx.x;
    {
        const unsigned nb = gridDim.x, q = nb / 8, r = nb % 8, xc = bid % 8;
        bid = (xc < r ? xc * (q + 1) : r * (q + 1) + (xc - r) * q) + bid / 8;
    }
    const int64_t m0 = (int64_t)(bid / n_tiles) * BM;
    const int n0 = (bid % n_tiles) * BN;

    const int aq = tid & 7;
    int64_t pb[AQ], p2[AQ];
    int iy0[AQ], ix0[AQ];
    bool rok[AQ];
#pragma unroll
    for (int q = 0; q < AQ; ++q) {
        const int64_t m = m0 + (tid >> 3) + 32 * q;
        rok[q] = m < a.M;
        const int64_t mm = rok[q] ? m : 0;
        const int ox = (int)(mm % a.Wo);
        const int64_t t = mm / a.Wo;
        const int oy = (int)(t % a.Ho);
        const int64_t n = t / a.Ho;
        if (DUAL) {
            pb[q] = mm * a.Ci + 4 * aq;
            p2[q] = ((n * a.H2 + (int64_t)oy * a.stride2) * a.W2 + (int64_t)ox * a.stride2) * a.Ci2 + 4 * aq;
            iy0[q] = ix0[q] = 0;
        } else {
            pb[q] = n * a.H * a.W * a.Ci + 4 * aq;
            p2[q] = 0;
            iy0[q] = oy * a.stride - a.pad;
            ix0[q] = ox * a.stride - a.pad;
        }
    }
    // B: this wave's fragments of column blocks (n0 + wn TN 32) / 32 + j; slice g of block cb, plane p at
    // wb + (cb_rel * S + g) * 1536 + p * 512 (bf16), lane part l * 8
    const int64_t S = a.Kp / XBK;
    const __bf16 *wb = a.wp + ((int64_t)((n0 + wn * TN * 32) >> 5) * S) * 1536 + lane * 8;
    const int nslice = a.Kp / XBK;

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){0};

    f32x4 va0[AQ], va1[AQ];
    bf16x8 bs0[TN][3], bs1[TN][3];  // B fragments of the even / odd slices
    int ky = 0, kx = 0, ci0 = 0, k0 = 0;
#define X6B_GLOAD(VA)                                                                                      \
    do {                                                                                                   \
        if (DUAL) {                                                                                        \
            const bool first = k0 < a.Ci;                                                                  \
            const float *src = first ? a.x + k0 : a.x2 + (k0 - a.Ci);                                      \
            _Pragma("unroll") for (int q = 0; q < AQ; ++q) VA[q] =                                         \
                *(const f32x4 *)(rok[q] ? src + (first ? pb[q] : p2[q]) : g_xzero4);                      \
            k0 += YBK;                                                                                     \
        } else {                                                                                           \
            const int dy = ky * a.dil, dx = kx * a.dil;                                                    \
            _Pragma("unroll") for (int q = 0; q < AQ; ++q) {                                               \
                const int iy = iy0[q] + dy, ix = ix0[q] + dx;                                              \
                const bool in = rok[q] && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;    \
                const f32x4 *ap_ = (const f32x4 *)(in ? a.x + pb[q] + ((int64_t)iy * a.W + ix) * a.Ci + ci0 : g_xzero4); \
                if (NT) VA[q] = __builtin_nontemporal_load(ap_);                                          \
                else VA[q] = *ap_;                                                                        \
            }                                                                                              \
            ci0 += YBK;                                                                                    \
            if (ci0 == a.Ci) {                                                                             \
                ci0 = 0;                                                                                   \
                if (++kx == a.KW) {                                                                        \
                    kx = 0;                                                                                \
                    ++ky;                                                                                  \
                }                                                                                          \
            }                                                                                              \
        }                                                                                                  \
    } while (0)
#define X6B_SWRITE(BUF, VA)                                                                                \
    do {                                                                                                   \
        __bf16 *As = lds + (BUF) * STAGE;                                                                  \
        _Pragma("unroll") for (int q = 0; q < AQ; ++q) {                                                   \
            bf16x4 hv, mv, lv;                                                                             \
            _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                                \
                __bf16 h_, m_, l_;                                                                         \
                split3(VA[q][e], h_, m_, l_);                                                              \
                hv[e] = h_;                                                                                \
                mv[e] = m_;                                                                                \
                lv[e] = l_;                                                                                \
            }                                                                                              \
            __bf16 *d = As + ((tid >> 3) + 32 * q) * YROW + 4 * aq;                                        \
            *(bf16x4 *)d = hv;                                                                             \
            *(bf16x4 *)(d + APL) = mv;                                                                     \
            *(bf16x4 *)(d + 2 * APL) = lv;                                                                 \
        }                                                                                                  \
    } while (0)
#define X6B_BLOAD(BS, G)                                                                                   \
    do {                                                                                                   \
        const int g_ = (G) < nslice ? (G) : nslice - 1; /* past the end: a harmless re-read */             \
        _Pragma("unroll") for (int j = 0; j < TN; ++j)                                                     \
            _Pragma("unroll") for (int p = 0; p < 3; ++p)                                                  \
                BS[j][p] = *(const bf16x8 *)(wb + ((int64_t)j * S + g_) * 1536 + p * 512);                \
    } while (0)
    const int r32 = lane & 31, h = lane >> 5;
#define X6B_SLICE(AS, KK, BC)                                                                              \
    do {                                                                                                   \
        bf16x8 fa[TM][3];                                                                                  \
        _Pragma("unroll") for (int i = 0; i < TM; ++i)                                                     \
            _Pragma("unroll") for (int p = 0; p < 3; ++p)                                                  \
                fa[i][p] = *(const bf16x8 *)(AS + p * APL + (wm * TM * 32 + i * 32 + r32) * YROW + 16 * (KK) + 8 * h); \
        _Pragma("unroll") for (int i = 0; i < TM; ++i)                                                     \
            _Pragma("unroll") for (int j = 0; j < TN; ++j) {                                               \
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], BC[j][0], acc[i][j], 0, 0, 0); \
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], BC[j][1], acc[i][j], 0, 0, 0); \
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], BC[j][0], acc[i][j], 0, 0, 0); \
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], BC[j][2], acc[i][j], 0, 0, 0); \
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][2], BC[j][0], acc[i][j], 0, 0, 0); \
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], BC[j][1], acc[i][j], 0, 0, 0); \
            }                                                                                              \
    } while (0)
    // MFMAs of K step KS from LDS buffer BUF: slice 2 KS (B in bs0), slice 2 KS + 1 (B in bs1, loaded by the caller
    // BEFORE the step's A prefetch), the next step's slice 0 loaded into bs0 in between.  Order matters: vmcnt
    // retires loads in issue order, so a B fragment loaded after an A prefetch would make its first use wait for
    // that prefetch too (half a K step of cover instead of a whole one).
#define X6B_MFMA(BUF, KS)                                                                                  \
    do {                                                                                                   \
        const __bf16 *As = lds + (BUF) * STAGE;                                                            \
        X6B_SLICE(As, 0, bs0);                                                                             \
        X6B_BLOAD(bs0, 2 * (KS) + 2);                                                                      \
        X6B_SLICE(As, 1, bs1);                                                                             \
    } while (0)

    const int nk = a.Kp / YBK;
    X6B_BLOAD(bs0, 0);
    X6B_GLOAD(va0);
    if (nk > 1) X6B_GLOAD(va1);
    X6B_SWRITE(0, va0);
    __syncthreads();
    int ks = 0;
    for (; ks + 3 < nk; ks += 2) {
        X6B_BLOAD(bs1, 2 * ks + 1);
        X6B_GLOAD(va0);  // step ks + 2
        X6B_MFMA(0, ks);
        X6B_SWRITE(1, va1);  // step ks + 1
        __syncthreads();
        X6B_BLOAD(bs1, 2 * ks + 3);
        X6B_GLOAD(va1);  // step ks + 3
        X6B_MFMA(1, ks + 1);
        X6B_SWRITE(0, va0);  // step ks + 2
        __syncthreads();
    }
    if (ks + 2 < nk) {
        X6B_BLOAD(bs1, 2 * ks + 1);
        X6B_GLOAD(va0);
        X6B_MFMA(0, ks);
        X6B_SWRITE(1, va1);
        __syncthreads();
        X6B_BLOAD(bs1, 2 * ks + 3);
        X6B_MFMA(1, ks + 1);
        X6B_SWRITE(0, va0);
        __syncthreads();
        X6B_BLOAD(bs1, 2 * ks + 5);
        X6B_MFMA(0, ks + 2);
    } else if (ks + 1 < nk) {
        X6B_BLOAD(bs1, 2 * ks + 1);
        X6B_MFMA(0, ks);
        X6B_SWRITE(1, va1);
        __syncthreads();
        X6B_BLOAD(bs1, 2 * ks + 3);
        X6B_MFMA(1, ks + 1);
    } else {
        X6B_BLOAD(bs1, 2 * ks + 1);
        X6B_MFMA(0, ks);
    }
#undef X6B_MFMA
#undef X6B_SLICE
#undef X6B_BLOAD
#undef X6B_SWRITE
#undef X6B_GLOAD
    if constexpr (CHAIN > 0) {
        if (X6S_ABLATE & 1) {  // timing only: one store per lane keeps the mainloop live
            float s_ = 0.0f;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) s_ += acc[i][j][0] + acc[i][j][15];
            if (m0 + tid < a.M) a.y[(m0 + tid) * a.Co2] = s_;
            return;
        }
        x6_chain_epilogue<WM, WN, TM, TN, CHAIN == 2 ? 4 : 0>(a, lds_raw, acc, wave, lane, wm, wn, m0);
        return;
    }
    x6_epilogue<TM, TN>(a, (float *)lds_raw, acc, wave, lane, wn, wm, m0, n0);
}

// ---------------------------------------------------------------------------
// k_conv_x6s: A from PRE-SPLIT activation planes (xs [3][N][H][W][Ci] bf16, written split by the producing conv's
// epilogue -- the 3x3 bottleneck conv2 reads the conv1 output it would otherwise split 9 times, once per tap)
// staged global -> LDS by LDS-DMA (global_load_lds_dwordx4: no staging VGPRs, no ds_write, no split VALU).  One
// DMA instruction moves 16 rows x 64 B of one plane; the 16-B chunk c of row r sits at chunk c ^ ((r >> 2) & 3),
// so the 16-lane fragment groups (16 consecutive rows, one chunk) hit 16 distinct slots.  B fragments by buffer
// loads from the fragment-order panel: the lane part of the address in the VGPR, the (block, slice, plane) part in
// the SGPR soffset (no address VALU).  NHWC, Ci % 32 == 0.  Same per-output K order as k_conv_x6 / k_conv_x6b:
// bit-identical results on the same split operands.
// ---------------------------------------------------------------------------
__device__ __forceinline__ unsigned lds_addr(const void *p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

__device__ __forceinline__ void dma16(const void *src, unsigned dst_any) {
    const unsigned dst = (unsigned)__builtin_amdgcn_readfirstlane((int)dst_any);  // wave-uniform LDS address
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(dst)
        : "memory");
}

// CHAIN (bev_conv2d_chain_x6_f32 / _dual_ with a pre-split xs): the mainloop above, then x6_chain_epilogue exactly
// as k_conv_x6b's chain runs it -- the layer1 / layer2 bottleneck bodies take conv1's split output, so conv2 (the
// 3x3, whose fp32 operand the register-staged kernel splits once per tap) stages by DMA alone.
// BLDS (the chains): B goes through LDS too -- the K step's BN / 32 x 2 slices x 3 planes of the fragment-order panel
// are 1-KiB runs, one DMA instruction each, read back as conflict-free ds_read_b128 (lane l at 16 l) -- so every
// vector-memory operation of the loop is a DMA issued one K step ahead and waited for at the step's end.  (With B
// in registers hipcc re-issued the fragment loads next to their MFMAs and waited on each: L2 latency per slice.)
template <int WM, int WN, int TM, int TN, int CHAIN = 0, bool BLDS = (CHAIN > 0), int NT3 = 0>
__global__ __launch_bounds__(256, CHAIN ? 2 : 3) void k_conv_x6s(ConvX a) {
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
    constexpr int APL = BM * 32;     // bf16 per A plane per stage (64-B rows)
    constexpr int BST = BLDS ? BN / 32 * 6 * 512 : 0;  // bf16 of B per stage: [cb][slice][plane][64 lanes][8]
    constexpr int STAGE = 3 * APL + BST;  // bf16 per stage
    constexpr int RW = BM / 4;       // rows staged by each wave
    constexpr int RG = RW / 16;      // 16-row DMA groups per wave and plane
    constexpr int BPW = BLDS ? BN / 32 * 6 / 4 : 0;  // B pieces (1 KiB) per wave and K step
    constexpr int EPIB = CHAIN ? 3 * BM * (BN + 8) * 2 : x6_epi_bytes<TN>();
    constexpr int LDSB = (2 * STAGE * 2 > EPIB) ? 2 * STAGE * 2 : EPIB;
    static_assert(RW % 16 == 0, "whole DMA groups per wave");
    static_assert(!BLDS || (BN / 32 * 6) % 4 == 0, "whole B pieces per wave");
    __shared__ __attribute__((aligned(16))) unsigned char lds_raw[LDSB];
    const __bf16 *lds = (const __bf16 *)lds_raw;

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
    const int wm = wave / WN, wn = wave % WN;
    const int n_tiles = (a.Co + BN - 1) / BN;
    unsigned bid = blockIdx.x;
    {
        const unsigned nb = gridDim.x, q = nb / 8, r = nb % 8, xc = bid % 8;
        bid = (xc < r ? xc * (q + 1) : r * (q + 1) + (xc - r) * q) + bid / 8;
    }
    const int64_t m0 = (int64_t)(bid / n_tiles) * BM;
    const int n0 = (bid % n_tiles) * BN;

    // DMA rows of this lane: wave * RW + 16 g + (lane >> 2); physical chunk lane & 3 holds logical chunk
    // (lane & 3) ^ ((row >> 2) & 3)
    int64_t abase[RG];
    int aiy[RG], aix[RG];
    bool aok[RG];
#pragma unroll
    for (int g = 0; g < RG; ++g) {
        const int row = wave * RW + 16 * g + (lane >> 2);
        const int lc = (lane & 3) ^ ((row >> 2) & 3);
        const int64_t m = m0 + row;
        aok[g] = m < a.M;
        const int64_t mm = aok[g] ? m : 0;
        const int ox = (int)(mm % a.Wo);
        const int64_t t = mm / a.Wo;
        const int oy = (int)(t % a.Ho);
        const int64_t n = t / a.Ho;
        aiy[g] = oy * a.stride - a.pad;
        aix[g] = ox * a.stride - a.pad;
        abase[g] = ((n * a.H + aiy[g]) * a.W + aix[g]) * a.Ci + 8 * lc;
    }
    const unsigned lbase = (unsigned)__builtin_amdgcn_readfirstlane((int)lds_addr(lds_raw));
    const int S = a.Kp / XBK;  // 16-deep slices
    int ky = 0, kx = 0, ci0 = 0, kstep = 0;
    const __bf16 *bsrc = a.wp + (int64_t)(n0 >> 5) * S * 1536 + lane * 8;  // the block's first column block
    auto issue = [&](int buf) {
        if (X6S_ABLATE & 4) return;
        if constexpr (BLDS) {  // piece q = (cb, slice, plane) of this K step: panel run ((cb S + 2 ks + sl) 3 + p)
            const unsigned db = lbase + (unsigned)(buf * STAGE * 2 + 3 * APL * 2);
#pragma unroll
            for (int i = 0; i < BPW; ++i) {
                const int q = wave + 4 * i, cbl = q / 6, r = q % 6;
                dma16(bsrc + ((int64_t)cbl * S + 2 * kstep + r / 3) * 1536 + (r % 3) * 512,
                      db + (unsigned)(q * 1024));
            }
            ++kstep;
        }
        const int64_t toff = ((int64_t)ky * a.dil * a.W + kx * a.dil) * a.Ci + ci0;
        const unsigned d0 = lbase + (unsigned)(buf * STAGE * 2) + (unsigned)(wave * RW * 64);
#pragma unroll
        for (int g = 0; g < RG; ++g) {
            const int iy = aiy[g] + ky * a.dil, ix = aix[g] + kx * a.dil;
            const bool in = aok[g] && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
            const __bf16 *src = a.xs + abase[g] + toff;
#pragma unroll
            for (int p = 0; p < 3; ++p)
                dma16(in ? (const void *)(src + p * a.xps) : (const void *)g_xzero4,
                      d0 + (unsigned)(p * APL * 2 + g * 1024));
        }
        ci0 += YBK;
        if (ci0 == a.Ci) {
            ci0 = 0;
            if (++kx == a.KW) {
                kx = 0;
                ++ky;
            }
        }
    };

    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<__bf16 *>(a.wp), 0, (int)(uint32_t)(copad_x(a.Co) / 32 * (int64_t)S * 3072), 0x00020000);
    const int cb0 = (n0 + wn * TN * 32) >> 5;
    const int vl = lane * 16;
    bf16x8 bs0[TN][3], bs1[TN][3];
#define X6S_BLOAD(BS, G)                                                                                   \
    do {                                                                                                   \
        const int g_ = (G) < S ? (G) : S - 1;                                                              \
        _Pragma("unroll") for (int j = 0; j < TN; ++j)                                                     \
            _Pragma("unroll") for (int p = 0; p < 3; ++p)                                                  \
                BS[j][p] = __builtin_bit_cast(                                                             \
                    bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, vl, (((cb0 + j) * S + g_) * 3 + p) * 1024, 0)); \
    } while (0)
    const int r32 = lane & 31, h = lane >> 5;
#define X6S_SLICE(AS, KK, BC)                                                                              \
    do {                                                                                                   \
        bf16x8 fa[TM][3];                                                                                  \
        _Pragma("unroll") for (int i = 0; i < TM; ++i) {                                                   \
            const int R = wm * TM * 32 + i * 32 + r32;                                                     \
            const int ph = (2 * (KK) + h) ^ ((R >> 2) & 3);                                                \
            _Pragma("unroll") for (int p = 0; p < 3; ++p)                                                  \
                fa[i][p] = *(const bf16x8 *)(AS + p * APL + R * 32 + ph * 8);                              \
        }                                                                                                  \
        if (X6S_ABLATE & 2) {                                                                              \
            _Pragma("unroll") for (int i = 0; i < TM; ++i)                                                 \
                _Pragma("unroll") for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(fa[i][0]), "v"(fa[i][1]), \
                                                                  "v"(fa[i][2]), "v"(BC[j][0]), "v"(BC[j][1]), "v"(BC[j][2])); \
            break;                                                                                         \
        }                                                                                                  \
        _Pragma("unroll") for (int i = 0; i < TM; ++i)                                                     \
            _Pragma("unroll") for (int j = 0; j < TN; ++j) {                                               \
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], BC[j][0], acc[i][j], 0, 0, 0); \
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], BC[j][1], acc[i][j], 0, 0, 0); \
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], BC[j][0], acc[i][j], 0, 0, 0); \
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], BC[j][2], acc[i][j], 0, 0, 0); \
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][2], BC[j][0], acc[i][j], 0, 0, 0); \
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], BC[j][1], acc[i][j], 0, 0, 0); \
            }                                                                                              \
    } while (0)

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){0};
    const int nk = a.Kp / YBK;
    if constexpr (BLDS) {
        issue(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (int ks = 0; ks < nk; ++ks) {
            const int cur = ks & 1;
            if (ks + 1 < nk) issue(cur ^ 1);
            const __bf16 *As = lds + cur * STAGE;
            const __bf16 *Bs = As + 3 * APL + lane * 8;
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                bf16x8 fb[TN][3];
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int p = 0; p < 3; ++p) fb[j][p] = *(const bf16x8 *)(Bs + (((wn * TN + j) * 2 + kk) * 3 + p) * 512);
                X6S_SLICE(As, kk, fb);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMAs of step ks + 1 landed
            __syncthreads();                                   // everyone's; buffer cur is free again
        }
    } else {
        X6S_BLOAD(bs0, 0);
        issue(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (int ks = 0; ks < nk; ++ks) {
            const int cur = ks & 1;
            if (ks + 1 < nk) issue(cur ^ 1);
            const __bf16 *As = lds + cur * STAGE;
            X6S_BLOAD(bs1, 2 * ks + 1);
            X6S_SLICE(As, 0, bs0);
            X6S_BLOAD(bs0, 2 * ks + 2);
            X6S_SLICE(As, 1, bs1);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of step ks + 1 landed
            __syncthreads();                                   // all of it; buffer cur is free again
        }
    }
#undef X6S_SLICE
#undef X6S_BLOAD
    if constexpr (CHAIN > 0) {
        if (X6S_ABLATE & 1) {  // timing only: one store per lane keeps the mainloop live
            float s_ = 0.0f;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) s_ += acc[i][j][0] + acc[i][j][15];
            if (m0 + tid < a.M) a.y[(m0 + tid) * a.Co2] = s_;
            return;
        }
        if (X6S_T_EPI || NT3 > 0) x6_chain_epilogue_t<WM, WN, TM, TN, CHAIN == 2 ? 4 : 0, NT3>(a, lds_raw, acc, wave, lane, wm, wn, m0);
        else x6_chain_epilogue<WM, WN, TM, TN, CHAIN == 2 ? 4 : 0>(a, lds_raw, acc, wave, lane, wm, wn, m0);
        return;
    }
    x6_epilogue<TM, TN>(a, (float *)lds_raw, acc, wave, lane, wn, wm, m0, n0);
}

template <int WM, int WN, int TM, int TN, int CHAIN = 0, int NT3 = 0>
int launch_x6s(const ConvX &a, hipStream_t st) {
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
    const int64_t blocks = ((a.M + BM - 1) / BM) * ((a.Co + BN - 1) / BN);
    if (blocks >= ((int64_t)1 << 31)) return BEV_ERR_ARGS;
    hipLaunchKernelGGL((k_conv_x6s<WM, WN, TM, TN, CHAIN, (CHAIN > 0), NT3>), dim3((unsigned)blocks), dim3(256), 0, st,
                       a);
    return (int)hipGetLastError();
}

__global__ void k_split3(const float *__restrict__ x, int64_t n, __bf16 *__restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    __bf16 h, m, l;
    split3(x[t], h, m, l);
    out[t] = h;
    out[t + n] = m;
    out[t + 2 * n] = l;
}

template <int WM, int WN, int TM, int TN, bool DUAL, int CHAIN = 0, bool NT = false>
int launch_x6b(const ConvX &a, hipStream_t st) {
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
    const int64_t blocks = ((a.M + BM - 1) / BM) * ((a.Co + BN - 1) / BN);
    if (blocks >= ((int64_t)1 << 31)) return BEV_ERR_ARGS;
    hipLaunchKernelGGL((k_conv_x6b<WM, WN, TM, TN, DUAL, CHAIN, NT>), dim3((unsigned)blocks), dim3(256), 0, st, a);
    return (int)hipGetLastError();
}

template <int WM, int WN, int TM, int TN, bool DUAL>
int launch_x6(const ConvX &a, hipStream_t st) {
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
    const int64_t blocks = ((a.M + BM - 1) / BM) * ((a.Co + BN - 1) / BN);
    if (blocks >= ((int64_t)1 << 31)) return BEV_ERR_ARGS;
    hipLaunchKernelGGL((k_conv_x6<WM, WN, TM, TN, DUAL>), dim3((unsigned)blocks), dim3(256), 0, st, a);
    return (int)hipGetLastError();
}

int g_x6_tile = 0;  // 0 automatic, 1 = 128 x 128, 2 = 128 x 64
int g_x6_nt = 0;    // BEV_TUNE_CONV_X6_NT: 1 = non-temporal activation loads in the 32-deep kernels
int g_x6_kernel = 0;  // 0 automatic, 1 = k_conv_x6 (16-deep K steps) everywhere, 2 = k_conv_x6b wherever it applies

template <bool DUAL>
int dispatch_x6(const ConvX &a0, hipStream_t st) {
    ConvX a = a0;
    a.nta = g_x6_nt;
    const int t = g_x6_tile ? g_x6_tile : (a.Co <= 64 ? 2 : 1);
    if (!DUAL && a.xs) {
        if (t == 2) return launch_x6s<4, 1, 1, 2>(a, st);
        return launch_x6s<2, 2, 2, 2>(a, st);
    }
    // automatic = the 32-deep-step kernel wherever it applies: single 1x1 layers measured faster on the 16-deep
    // kernel in isolation, but the ResNet-50 encoder (two stream groups) is fastest with the 32-deep kernel
    // everywhere (r03 tools/trunk_ab.py: 16.24 ms vs 16.34 with 1x1 / dual layers on the 16-deep one, 16.43 all)
    const bool wide = a.Ci % YBK == 0 && (!DUAL || a.Ci2 % YBK == 0) && g_x6_kernel != 1;
    if (wide) {
        if (t == 2 && !DUAL && a.nta) return launch_x6b<4, 1, 1, 2, false, 0, true>(a, st);
        if (t == 2) return launch_x6b<4, 1, 1, 2, DUAL>(a, st);
        return launch_x6b<2, 2, 2, 2, DUAL>(a, st);
    }
    if (t == 2) return launch_x6<4, 1, 1, 2, DUAL>(a, st);
    return launch_x6<2, 2, 2, 2, DUAL>(a, st);
}

// ---------------------------------------------------------------------------
// ResNet stem (7x7 / stride 2 / pad 3 over Ci = 3 NCHW images, Co <= 64) on the split arithmetic
// ---------------------------------------------------------------------------
// timm conv1 (cnn_encoder.py:26; first layer of CNNEncoder._encode_single) -- the same contract as bev_conv.hip's
// exact-f32 k_stem, with the products of the other trunk layers: per 16-deep k slice six v_mfma_f32_32x32x16_bf16
// (32 cycles each) instead of eight v_mfma_f32_32x32x2_f32 (64 cycles), 2.67x fewer matrix-core cycles.
// Workgroup = 8 waves, tile = 8 output rows x 64 columns x 64 channels, wave w owns output row w (2 x 2 MFMA tiles
// of 32 pixels x 32 channels).  The tile's input patch (3 ch x 21 rows x 133 cols) sits in LDS as fp32 even / odd
// column planes exactly as k_stem keeps it (stride 2: tap kx of output column ox is plane kx & 1 at ox + kx / 2),
// so each A element is a ds_read_b32 at a compile-time offset; a lane's 8 consecutive k (the split panel's order,
// k = (ky * 7 + kx) * 3 + ci, 147 taps padded to 160) are read, split into h / m / l and fed as three bf16
// fragments.  The weights' split panel (fragment order, the first two 32-column blocks: 60 KiB) is copied into LDS
// once per workgroup, so B fragments are conflict-free ds_read_b128.  Persistent over tiles; the next tile's patch
// is fetched into registers during the MFMAs.  fp32-tolerance equal to k_stem (summation order), as every split
// conv is to its exact-f32 counterpart.
namespace stem6 {
constexpr int TW = 64, TH = 8, NTHR = 512;
constexpr int PR = 2 * TH + 5;  // 21 input rows
constexpr int PC = 2 * TW + 5;  // 133 input columns
constexpr int PP = 80;          // plane pitch (67 used; = 16 mod 32 -> conflict-free stores)
constexpr int RP = 2 * PP, CP = PR * RP, PATCH = 3 * CP;
constexpr int NE = 3 * PR * PC;
constexpr int PER_T = (NE + NTHR - 1) / NTHR;
constexpr int NS = 10;            // 16-deep k slices (147 -> 160)
constexpr int WB = 2 * NS * 3 * 512;  // bf16 of the panel's first two 32-column blocks
// STEM6_PRESPLIT 1: the patch is split into h / m / l once, when it is written to LDS (a dword plane of (h, m) pairs
// and a 16-bit plane of l): each input value serves ~12 (tap, pixel) products, so splitting per use (0: fp32 patch,
// split3 on every A element) costs ~12x the conversions.
// LDS float offset of panel k (k = (ky * 7 + kx) * 3 + ci) relative to (output row 0, output column 0) of the patch;
// the padding k >= 147 reads tap 0 (its weight is zero)
__host__ __device__ constexpr int koff(int k) {
    return k >= 147 ? 0 : (k % 3) * CP + (k / 21) * RP + (((k / 3) % 7) & 1) * PP + (((k / 3) % 7) >> 1);
}
}  // namespace stem6

#ifndef STEM6_PRESPLIT
#define STEM6_PRESPLIT 1
#endif

struct StemX6Args {
    const float *__restrict__ x;
    const __bf16 *__restrict__ wp;
    const float *__restrict__ bias;
    float *__restrict__ y;  // the stem output [N, Ho, Wo, Co], or (POOL) the max-pooled one [N, Hp, Wp, 64]
    int H, W, Co, Ho, Wo, relu, nTx, nTy;
    int64_t ntiles;
    // POOL only: per tile, the horizontally pooled last stem row (the next tile row's pooled row 0 needs it:
    // [ntiles][32][64]) and the last stem column's vertical window maxima for pooled rows 0..4 ([ntiles][5][64])
    float *__restrict__ edge_b, *__restrict__ edge_r;
    int Hp, Wp;
};

__device__ __forceinline__ void stem6_fetch(const StemX6Args &a, int64_t t, int tid, float (&pv)[stem6::PER_T]) {
    using namespace stem6;
    const int tx = (int)(t % a.nTx);
    const int64_t r_ = t / a.nTx;
    const int ty = (int)(r_ % a.nTy);
    const int64_t img = r_ / a.nTy;
    const int row0 = 2 * ty * TH - 3, col0 = 2 * tx * TW - 3;
    const float *xi = a.x + img * 3 * (int64_t)a.H * a.W;
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
        const int e = tid + NTHR * i;
        const int cr = e / PC, c = e - cr * PC;
        const int ci = cr / PR, r = cr - ci * PR;
        const int gy = row0 + r, gx = col0 + c;
        const bool in = e < NE && gy >= 0 && gy < a.H && gx >= 0 && gx < a.W;
        pv[i] = *(in ? xi + ((int64_t)ci * a.H + gy) * a.W + gx : (const float *)g_xzero4);
    }
}

__device__ __forceinline__ void stem6_put(float *pl, int tid, const float (&pv)[stem6::PER_T]) {
    using namespace stem6;
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
        const int e = tid + NTHR * i;
        if (e < NE) {
            const int cr = e / PC, c = e - cr * PC;
            const int ci = cr / PR, r = cr - ci * PR;
            const int o = ci * CP + r * RP + (c & 1) * PP + (c >> 1);
            if (STEM6_PRESPLIT) {  // pl = the (h, m) dword plane, followed by the l plane (PATCH bf16)
                __bf16 hh, mm, ll;
                split3(pv[i], hh, mm, ll);
                reinterpret_cast<unsigned *>(pl)[o] = (unsigned)__builtin_bit_cast(unsigned short, hh) |
                                                      ((unsigned)__builtin_bit_cast(unsigned short, mm) << 16);
                reinterpret_cast<__bf16 *>(pl + PATCH)[o] = ll;
            } else {
                pl[o] = pv[i];
            }
        }
    }
}

// the pooled maximum of relu'd stem values (>= +0, never NaN: the ReLU maps NaN to 0)
__device__ __forceinline__ float pool_mx(float m, float v) { return __builtin_fmaxf(m, v); }

// POOL: timm's stem max-pool (3x3 / s2 / p1, cnn_encoder.py:26 features_only) fused into the epilogue.  The stem
// output is relu'd (>= +0), so a window's padding and the tile's rows / columns past the image may count as +0 without
// changing any maximum: every pooled value is the max over a set of non-negative values, whatever the grouping --
// bit-identical to k_maxpool_rows over the stem output.  Tile (ty, tx) = stem rows 8ty..8ty+7 x columns
// 64tx..64tx+63 owns pooled rows 4ty..4ty+3 x columns 32tx..32tx+31; pooled row 4ty needs stem row 8ty-1 (tile ty-1)
// and pooled column 32tx stem column 64tx-1 (tile tx-1): each tile stores its own part of those seam outputs and
// exports its last row / column parts (edge_b / edge_r), which k_stem_pool_seams folds in afterwards.
// Lane (h, r32) holds channel r32 (+32) of stem columns 32mt + 8b + 4h + u (u = 0..3): pooled columns 16mt + 4b + 2h
// (+1) are 3-maxima of its own values and, for the even one, the other half-wave's u = 3 value of the preceding
// group (a cross-half shuffle); wave w = stem row w: the odd waves hand their 34 row maxima to the even ones through
// LDS, the even wave 2p combines rows 2p-1..2p+1 into pooled row p.
template <bool POOL>
__global__ __launch_bounds__(stem6::NTHR, 1) void k_stem_x6(StemX6Args a) {
    using namespace stem6;
    __shared__ __attribute__((aligned(16))) unsigned char lds_raw[WB * 2 + PATCH * (STEM6_PRESPLIT ? 6 : 4)];
    __bf16 *wl = (__bf16 *)lds_raw;
    float *pl = (float *)(lds_raw + WB * 2);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r32 = lane & 31;
    // the split panel's blocks 0 and 1 ([cb][slice][plane][64 lanes][8]) are its first WB bf16: a straight copy
    for (int e = tid; e < WB / 8; e += NTHR) reinterpret_cast<u32x4 *>(wl)[e] = reinterpret_cast<const u32x4 *>(a.wp)[e];
    float pv[PER_T];
    int64_t t = blockIdx.x;
    stem6_fetch(a, t < a.ntiles ? t : 0, tid, pv);
    stem6_put(pl, tid, pv);
    __syncthreads();

    const float *P = pl + wave * 2 * RP + r32;  // output row `wave`, column r32 (+ 32 for the second M tile)
    const __bf16 *PL = reinterpret_cast<const __bf16 *>(pl + PATCH) + wave * 2 * RP + r32;  // its l plane (PRESPLIT)
    const float b0 = (r32 < a.Co) ? a.bias[r32] : 0.0f;
    const float b1 = (32 + r32 < a.Co) ? a.bias[32 + r32] : 0.0f;
    for (; t < a.ntiles; t += gridDim.x) {
        const int64_t tn = t + gridDim.x;
        stem6_fetch(a, tn < a.ntiles ? tn : t, tid, pv);  // in flight during the MFMAs
        f32x16 acc[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = (f32x16){0};
#pragma unroll
        for (int sl = 0; sl < NS; ++sl) {
            int hv = h;
            asm volatile("" : "+v"(hv));  // per slice: the h selects stay cndmasks, not 160 hoisted lane offsets
            const __bf16 *wlb = wl + lane * 8;
            asm volatile("" : "+v"(wlb));  // per slice: the weight fragments are re-read, not held across tiles
            bf16x8 fb[2][3];
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    fb[j][p] = *(const bf16x8 *)(wlb + ((j * NS + sl) * 3 + p) * 512);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                bf16x8 fa[3];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const int o0 = koff(16 * sl + e), o1 = koff(16 * sl + 8 + e);
                    const int o = 32 * mt + (hv ? o1 : o0);
                    if (STEM6_PRESPLIT) {
                        const unsigned hm = reinterpret_cast<const unsigned *>(P)[o];
                        fa[0][e] = __builtin_bit_cast(__bf16, (unsigned short)(hm & 0xffffu));
                        fa[1][e] = __builtin_bit_cast(__bf16, (unsigned short)(hm >> 16));
                        fa[2][e] = PL[o];
                    } else {
                        __bf16 hh, mm, ll;
                        split3(P[o], hh, mm, ll);
                        fa[0][e] = hh;
                        fa[1][e] = mm;
                        fa[2][e] = ll;
                    }
                }
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    f32x16 &c = acc[mt][j];
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[j][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[j][1], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[j][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[j][2], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2], fb[j][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[j][1], c, 0, 0, 0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);  // one slice of operands live at a time
        }
        // epilogue: D[row][col], col = channel r32 (+32), row = pixel (r & 3) + 8 (r >> 2) + 4 h (+32)
        if constexpr (POOL) {
            const int tx = (int)(t % a.nTx);
            const int64_t r_ = t / a.nTx;
            const int ty = (int)(r_ % a.nTy);
            const int64_t img = r_ / a.nTy;
            const int oy = ty * TH + wave;
            const int oxb = tx * TW;
            float hp[2][4][2][2];  // [mt][b][pc][j]: pooled column 16 mt + 4 b + 2 h + pc, channel r32 + 32 j
            float pa3[2][2][4];    // the other half-wave's u = 3 value of group (mt, b)
            float c63[2];          // stem column 63 (lanes h = 1)
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        float v[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int ox = oxb + 32 * mt + 8 * b + 4 * h + u;
                            const float z = acc[mt][j][4 * b + u] + (j ? b1 : b0);
                            v[u] = oy < a.Ho && ox < a.Wo && z > 0.0f ? z : 0.0f;  // the stem's ReLU (NaN -> 0)
                        }
                        pa3[mt][j][b] = __shfl_xor(v[3], 32);
                        hp[mt][b][1][j] = pool_mx(pool_mx(v[1], v[2]), v[3]);
                        hp[mt][b][0][j] = pool_mx(v[0], v[1]);
                        if (mt == 1 && b == 3) c63[j] = v[3];
                    }
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        const float prev0 = b > 0 ? pa3[mt][j][b - 1] : (mt > 0 ? pa3[mt - 1][j][3] : 0.0f);
                        hp[mt][b][0][j] = pool_mx(hp[mt][b][0][j], h ? pa3[mt][j][b] : prev0);
                    }
            __syncthreads();  // every wave is done reading the patch: its LDS holds the row exchange
            float *xl = pl;   // [odd wave][34][64 lanes]
            if (wave & 1) {
                float *o = xl + (wave >> 1) * 34 * 64 + lane;
#pragma unroll
                for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                    for (int b = 0; b < 4; ++b)
#pragma unroll
                        for (int pc = 0; pc < 2; ++pc)
#pragma unroll
                            for (int j = 0; j < 2; ++j) o[(((mt * 4 + b) * 2 + pc) * 2 + j) * 64] = hp[mt][b][pc][j];
                o[32 * 64] = c63[0];
                o[33 * 64] = c63[1];
            }
            __syncthreads();
            const int64_t tile = t;
            if (wave == TH - 1) {  // the last row: next tile row's pooled row 0, and column 63 alone (pooled row 4)
                float *eb = a.edge_b + tile * (32 * 64);
#pragma unroll
                for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                    for (int b = 0; b < 4; ++b)
#pragma unroll
                        for (int pc = 0; pc < 2; ++pc)
#pragma unroll
                            for (int j = 0; j < 2; ++j)
                                eb[(16 * mt + 4 * b + 2 * h + pc) * 64 + r32 + 32 * j] = hp[mt][b][pc][j];
                if (h) {
                    a.edge_r[(tile * 5 + 4) * 64 + r32] = c63[0];
                    a.edge_r[(tile * 5 + 4) * 64 + 32 + r32] = c63[1];
                }
            } else if (!(wave & 1)) {
                const int p = wave >> 1;
                const float *up = xl + (p - 1) * 34 * 64 + lane, *dn = xl + p * 34 * 64 + lane;
#pragma unroll
                for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                    for (int b = 0; b < 4; ++b)
#pragma unroll
                        for (int pc = 0; pc < 2; ++pc)
#pragma unroll
                            for (int j = 0; j < 2; ++j) {
                                const int e = (((mt * 4 + b) * 2 + pc) * 2 + j) * 64;
                                float m = pool_mx(hp[mt][b][pc][j], dn[e]);
                                if (p > 0) m = pool_mx(m, up[e]);
                                hp[mt][b][pc][j] = m;
                            }
                float e0 = pool_mx(c63[0], dn[32 * 64]), e1 = pool_mx(c63[1], dn[33 * 64]);
                if (p > 0) {
                    e0 = pool_mx(e0, up[32 * 64]);
                    e1 = pool_mx(e1, up[33 * 64]);
                }
                if (h) {
                    a.edge_r[(tile * 5 + p) * 64 + r32] = e0;
                    a.edge_r[(tile * 5 + p) * 64 + 32 + r32] = e1;
                }
                const int prow = ty * (TH / 2) + p;
                if (prow < a.Hp) {
                    float *yr = a.y + ((img * a.Hp + prow) * (int64_t)a.Wp) * 64;
#pragma unroll
                    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                        for (int b = 0; b < 4; ++b)
#pragma unroll
                            for (int pc = 0; pc < 2; ++pc) {
                                const int Q = tx * (TW / 2) + 16 * mt + 4 * b + 2 * h + pc;
                                if (Q < a.Wp) {
                                    yr[(int64_t)Q * 64 + r32] = hp[mt][b][pc][0];
                                    yr[(int64_t)Q * 64 + 32 + r32] = hp[mt][b][pc][1];
                                }
                            }
                }
            }
        } else {
            const int tx = (int)(t % a.nTx);
            const int64_t r_ = t / a.nTx;
            const int ty = (int)(r_ % a.nTy);
            const int64_t img = r_ / a.nTy;
            const int oy = ty * TH + wave;
            const int oxb = tx * TW;
            if (oy < a.Ho) {
                float *yr = a.y + ((img * a.Ho + oy) * (int64_t)a.Wo) * a.Co;
#pragma unroll
                for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int ox = oxb + 32 * mt + (r & 3) + 8 * (r >> 2) + 4 * h;
                        if (ox < a.Wo) {
                            float v0 = acc[mt][0][r] + b0, v1 = acc[mt][1][r] + b1;
                            if (a.relu) {
                                v0 = v0 > 0.0f ? v0 : 0.0f;
                                v1 = v1 > 0.0f ? v1 : 0.0f;
                            }
                            float *yp = yr + (int64_t)ox * a.Co;
                            if (r32 < a.Co) yp[r32] = v0;
                            if (32 + r32 < a.Co) yp[32 + r32] = v1;
                        }
                    }
            }
        }
        __syncthreads();  // every wave is done reading the patch
        stem6_put(pl, tid, pv);
        __syncthreads();
    }
}

// The seam outputs of the fused stem max-pool: pooled row 4ty of tile (ty, tx) takes edge_b of tile (ty-1, tx),
// pooled column 32tx edge_r of tile (ty, tx-1), their corner edge_r row 4 of tile (ty-1, tx-1).  One thread per
// (tile, seam output, 4 channels): 35 seam outputs (32 columns of row 0, rows 1..3 of column 0) x 16 float4.
__global__ __launch_bounds__(256) void k_stem_pool_seams(float *__restrict__ y, const float *__restrict__ edge_b,
                                                         const float *__restrict__ edge_r, int nTx, int nTy,
                                                         int64_t ntiles, int Hp, int Wp) {
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t tile = g / (35 * 16);
    if (tile >= ntiles) return;
    const int k = (int)(g - tile * (35 * 16)), s = k >> 4, c4 = k & 15;
    const int tx = (int)(tile % nTx);
    const int64_t r_ = tile / nTx;
    const int ty = (int)(r_ % nTy);
    const int64_t img = r_ / nTy;
    const int p = s < 32 ? 0 : s - 31, q = s < 32 ? s : 0;
    const int P = ty * (stem6::TH / 2) + p, Q = tx * (stem6::TW / 2) + q;
    if (P >= Hp || Q >= Wp || (p == 0 && ty == 0 && (q > 0 || tx == 0))) return;  // no seam contribution
    float4 *yp = reinterpret_cast<float4 *>(y + (((img * Hp + P) * (int64_t)Wp + Q) * 64)) + c4;
    float4 m = *yp;
    auto mx = [](float4 a, float4 b) {
        return make_float4(pool_mx(a.x, b.x), pool_mx(a.y, b.y), pool_mx(a.z, b.z), pool_mx(a.w, b.w));
    };
    if (p == 0 && ty > 0) m = mx(m, reinterpret_cast<const float4 *>(edge_b + ((tile - nTx) * 32 + q) * 64)[c4]);
    if (q == 0 && tx > 0) {
        m = mx(m, reinterpret_cast<const float4 *>(edge_r + ((tile - 1) * 5 + p) * 64)[c4]);
        if (p == 0 && ty > 0)
            m = mx(m, reinterpret_cast<const float4 *>(edge_r + ((tile - nTx - 1) * 5 + 4) * 64)[c4]);
    }
    *yp = m;
}

}  // namespace

namespace bev {
int conv_x6_tune(int knob, int value) {
    int *slot = knob == BEV_TUNE_CONV_X6_TILE ? &g_x6_tile : knob == BEV_TUNE_CONV_X6_NT ? &g_x6_nt : &g_x6_kernel;
    if (value < 0 || value > 2 || (knob == BEV_TUNE_CONV_X6_NT && value > 1)) return BEV_ERR_ARGS;
    const int old = *slot;
    *slot = value;
    return old;
}
}  // namespace bev

extern "C" {

int64_t bev_conv_packed_size_x6(int Co, int Ci, int KH, int KW) {
    if (Co <= 0 || Ci <= 0 || KH <= 0 || KW <= 0) return BEV_ERR_ARGS;
    return copad_x(Co) * kpad_x(Ci * KH * KW) * 3;
}

int bev_conv_pack_weights_x6(const float *w, int Co, int Ci, int KH, int KW, uint16_t *packed, void *stream) {
    if (!w || !packed || Co <= 0 || Ci <= 0 || KH <= 0 || KW <= 0) return BEV_ERR_ARGS;
    const int64_t Kp = kpad_x(Ci * KH * KW), Cop = copad_x(Co), n = Kp * Cop;
    hipLaunchKernelGGL(k_pack_x6, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, w, Co, Ci, KH,
                       KW, Kp, Cop, (__bf16 *)packed);
    return (int)hipGetLastError();
}

int bev_conv2d_x6_f32(const float *x, const uint16_t *xs, int N, int H, int W, int Ci, const uint16_t *packed,
                      const float *bias, const float *residual, int Co, int KH, int KW, int stride, int pad,
                      int dilation, int act, float *y, uint16_t *ys, int ldy, int Ho, int Wo, void *stream) {
    if ((!x == !xs) || !packed || (!y == !ys) || N < 0 || H <= 0 || W <= 0 || Ci <= 0 || Co <= 0 || KH <= 0 ||
        KW <= 0 || stride <= 0 || pad < 0 || dilation <= 0 || act < 0 || act > 2 || ldy < Co)
        return BEV_ERR_ARGS;
    if (Ci % (xs ? YBK : XBK) != 0) return BEV_ERR_ARGS;  // one tap and 16 (split input: 32) channels per K step
    if (Ho != (H + 2 * pad - dilation * (KH - 1) - 1) / stride + 1 ||
        Wo != (W + 2 * pad - dilation * (KW - 1) - 1) / stride + 1 || Ho <= 0 || Wo <= 0)
        return BEV_ERR_ARGS;
    if ((((uintptr_t)x | (uintptr_t)xs | (uintptr_t)packed) & 15) != 0) return BEV_ERR_ARGS;
    if (residual && ldy != Co) return BEV_ERR_ARGS;
    if (ys && (ldy != Co || Co % 4 != 0 || ((uintptr_t)ys & 7) != 0)) return BEV_ERR_ARGS;
    if (N == 0) return 0;
    ConvX a;
    a.x = x;
    a.wp = (const __bf16 *)packed;
    a.bias = bias;
    a.res = residual;
    a.y = y;
    a.N = N, a.H = H, a.W = W, a.Ci = Ci, a.Co = Co, a.KH = KH, a.KW = KW, a.stride = stride, a.pad = pad;
    a.dil = dilation, a.Ho = Ho, a.Wo = Wo, a.act = act, a.ldy = ldy;
    a.Kp = (int)kpad_x(Ci * KH * KW);
    a.M = (int64_t)N * Ho * Wo;
    a.x2 = nullptr;
    a.Ci2 = a.H2 = a.W2 = a.stride2 = 0;
    a.xs = (const __bf16 *)xs;
    a.ys = (__bf16 *)ys;
    a.xps = (int64_t)N * H * W * Ci;
    a.yps = a.M * Co;
    a.wp2 = nullptr;
    a.bias2 = nullptr;
    a.Co2 = a.act2 = 0;
    return dispatch_x6<false>(a, (hipStream_t)stream);
}

int bev_split3_f32(const float *x, int64_t n, uint16_t *planes, void *stream) {
    if (!x || !planes || n < 0) return BEV_ERR_ARGS;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_split3, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, n,
                       (__bf16 *)planes);
    return (int)hipGetLastError();
}

int bev_conv2d_dual_x6_f32(const float *x, int N, int Ho, int Wo, int Ci, const float *x2, int H2, int W2, int Ci2,
                           int stride2, const uint16_t *packed, const float *bias, int Co, int act, float *y,
                           void *stream) {
    if (!x || !x2 || !packed || !y || N < 0 || Ho <= 0 || Wo <= 0 || Ci <= 0 || Ci2 <= 0 || H2 <= 0 || W2 <= 0 ||
        stride2 <= 0 || Co <= 0 || act < 0 || act > 2)
        return BEV_ERR_ARGS;
    if (Ci % XBK != 0 || Ci2 % XBK != 0) return BEV_ERR_ARGS;
    if (Ho != (H2 - 1) / stride2 + 1 || Wo != (W2 - 1) / stride2 + 1) return BEV_ERR_ARGS;
    if ((((uintptr_t)x | (uintptr_t)x2 | (uintptr_t)packed) & 15) != 0) return BEV_ERR_ARGS;
    if (N == 0) return 0;
    ConvX a;
    a.x = x;
    a.wp = (const __bf16 *)packed;
    a.bias = bias;
    a.res = nullptr;
    a.y = y;
    a.N = N, a.H = Ho, a.W = Wo, a.Ci = Ci, a.Co = Co, a.KH = 1, a.KW = 1, a.stride = 1, a.pad = 0;
    a.dil = 1, a.Ho = Ho, a.Wo = Wo, a.act = act, a.ldy = Co;
    a.Kp = (int)kpad_x(Ci + Ci2);
    a.M = (int64_t)N * Ho * Wo;
    a.x2 = x2;
    a.Ci2 = Ci2, a.H2 = H2, a.W2 = W2, a.stride2 = stride2;
    a.xs = nullptr;
    a.ys = nullptr;
    a.xps = a.yps = 0;
    a.wp2 = nullptr;
    a.bias2 = nullptr;
    a.Co2 = a.act2 = 0;
    return dispatch_x6<true>(a, (hipStream_t)stream);
}

int bev_conv2d_chain_x6_f32(const float *x, const uint16_t *xs, int N, int H, int W, int Ci,
                            const uint16_t *packed, const float *bias, int Co, int KH, int KW, int stride, int pad,
                            int act, const uint16_t *packed2, const float *bias2, int Co2, const float *residual,
                            int act2, float *y, int Ho, int Wo, void *stream) {
    if ((!x == !xs) || !packed || !packed2 || !y || N < 0 || H <= 0 || W <= 0 || KH <= 0 || KW <= 0 ||
        stride <= 0 || pad < 0 || act < 0 || act > 2 || act2 < 0 || act2 > 2)
        return BEV_ERR_ARGS;
    if (Ci % YBK != 0 || (Co != 64 && Co != 128) || Co2 <= 0 || Co2 % 64 != 0 ||
        (((uintptr_t)x | (uintptr_t)xs | (uintptr_t)packed | (uintptr_t)packed2) & 15) != 0)
        return BEV_ERR_ARGS;
    if (Ho != (H + 2 * pad - KH) / stride + 1 || Wo != (W + 2 * pad - KW) / stride + 1 || Ho <= 0 || Wo <= 0)
        return BEV_ERR_ARGS;
    if (N == 0) return 0;
    ConvX a;
    a.x = x;
    a.wp = (const __bf16 *)packed;
    a.bias = bias;
    a.res = residual;
    a.y = y;
    a.N = N, a.H = H, a.W = W, a.Ci = Ci, a.Co = Co, a.KH = KH, a.KW = KW, a.stride = stride, a.pad = pad;
    a.dil = 1, a.Ho = Ho, a.Wo = Wo, a.act = act, a.ldy = Co2;
    a.Kp = (int)kpad_x(Ci * KH * KW);
    a.M = (int64_t)N * Ho * Wo;
    a.x2 = nullptr;
    a.Ci2 = a.H2 = a.W2 = a.stride2 = 0;
    a.xs = (const __bf16 *)xs;
    a.ys = nullptr;
    a.xps = (int64_t)N * H * W * Ci;
    a.yps = 0;
    a.wp2 = (const __bf16 *)packed2;
    a.bias2 = bias2;
    a.Co2 = Co2;
    a.act2 = act2;
    if (Co != 64 && Co2 % 128 != 0) return BEV_ERR_ARGS;  // two waves share each 32-row band of the 64-row tile
    if (xs) {  // conv1 handed over its output split: conv2's operand by LDS-DMA (k_conv_x6s), same K order
        if (Co == 64) return launch_x6s<4, 1, 1, 2, 1>(a, (hipStream_t)stream);
        return launch_x6s<2, 2, 1, 2, 1>(a, (hipStream_t)stream);
    }
    if (Co == 64) return launch_x6b<4, 1, 1, 2, false, 1>(a, (hipStream_t)stream);
    return launch_x6b<2, 2, 1, 2, false, 1>(a, (hipStream_t)stream);  // 64 x 128: h2 planes 52 KiB of LDS
}

int bev_conv2d_chain_dual_x6_f32(const float *x, const uint16_t *xs, int N, int H, int W, int Ci,
                                 const uint16_t *packed, const float *bias, int Co, int KH, int KW, int stride,
                                 int pad, int act, const float *x2, int H2, int W2, int Ci2, int stride2,
                                 const uint16_t *packed2, const float *bias2, int Co2, int act2, float *y, int Ho,
                                 int Wo, void *stream) {
    if ((!x == !xs) || !x2 || !packed || !packed2 || !y || N < 0 || H <= 0 || W <= 0 || KH <= 0 || KW <= 0 ||
        stride <= 0 || pad < 0 || act < 0 || act > 2 || act2 < 0 || act2 > 2 || stride2 <= 0 || H2 <= 0 || W2 <= 0)
        return BEV_ERR_ARGS;
    // the layer1 block-0 shape: 64-channel h2 and a 64-channel shortcut operand (4 slices kept in registers)
    if (Ci % YBK != 0 || Co != 64 || Ci2 != 64 || Co2 <= 0 || Co2 % 64 != 0 ||
        (((uintptr_t)x | (uintptr_t)xs | (uintptr_t)x2 | (uintptr_t)packed | (uintptr_t)packed2) & 15) != 0)
        return BEV_ERR_ARGS;
    if (Ho != (H + 2 * pad - KH) / stride + 1 || Wo != (W + 2 * pad - KW) / stride + 1 || Ho <= 0 || Wo <= 0 ||
        Ho != (H2 - 1) / stride2 + 1 || Wo != (W2 - 1) / stride2 + 1)
        return BEV_ERR_ARGS;
    if (N == 0) return 0;
    ConvX a;
    a.x = x;
    a.wp = (const __bf16 *)packed;
    a.bias = bias;
    a.res = nullptr;
    a.y = y;
    a.N = N, a.H = H, a.W = W, a.Ci = Ci, a.Co = Co, a.KH = KH, a.KW = KW, a.stride = stride, a.pad = pad;
    a.dil = 1, a.Ho = Ho, a.Wo = Wo, a.act = act, a.ldy = Co2;
    a.Kp = (int)kpad_x(Ci * KH * KW);
    a.M = (int64_t)N * Ho * Wo;
    a.x2 = x2;
    a.Ci2 = Ci2, a.H2 = H2, a.W2 = W2, a.stride2 = stride2;
    a.xs = (const __bf16 *)xs;
    a.ys = nullptr;
    a.xps = (int64_t)N * H * W * Ci;
    a.yps = 0;
    a.wp2 = (const __bf16 *)packed2;
    a.bias2 = bias2;
    a.Co2 = Co2;
    a.act2 = act2;
    if (xs) return launch_x6s<4, 1, 1, 2, 2>(a, (hipStream_t)stream);
    return launch_x6b<4, 1, 1, 2, false, 2>(a, (hipStream_t)stream);
}

int bev_conv2d_chain_next_x6_f32(const uint16_t *xs, int N, int H, int W, int Ci, const uint16_t *packed,
                                 const float *bias, int Co, int KH, int KW, int stride, int pad, int act,
                                 const float *x2, int H2, int W2, int Ci2, int stride2, const uint16_t *packed2,
                                 const float *bias2, int Co2, const float *residual, int act2, float *y, int Ho, int Wo,
                                 const uint16_t *packed3, const float *bias3, int Co3, int act3, float *y3,
                                 uint16_t *ys3, void *stream) {
    if (!xs || !packed || !packed2 || !packed3 || !y || (!y3 == !ys3) || N < 0 || H <= 0 || W <= 0 || KH <= 0 ||
        KW <= 0 || stride <= 0 || pad < 0 || act < 0 || act > 2 || act2 < 0 || act2 > 2 || act3 < 0 || act3 > 2)
        return BEV_ERR_ARGS;
    // the 128-row tile (every Co2 chunk of a band in one wave), conv2 64 channels; the next conv Co3 in {64, 128}
    if (Ci % YBK != 0 || Co != 64 || Co2 <= 0 || Co2 % 64 != 0 || (Co3 != 64 && Co3 != 128) ||
        (((uintptr_t)xs | (uintptr_t)packed | (uintptr_t)packed2 | (uintptr_t)packed3 | (uintptr_t)y |
          (uintptr_t)y3 | (uintptr_t)residual | (uintptr_t)bias2 | (uintptr_t)bias3) & 15) != 0 ||
        ((uintptr_t)ys3 & 7) != 0)
        return BEV_ERR_ARGS;
    if (Ho != (H + 2 * pad - KH) / stride + 1 || Wo != (W + 2 * pad - KW) / stride + 1 || Ho <= 0 || Wo <= 0)
        return BEV_ERR_ARGS;
    // The dual (block 0) form is not offered: its instantiation (k_conv_x6s<4,1,1,2,2,1,2>, 256 VGPRs) wrote y
    // channels 24-31 of each 32 wrongly for lanes 12-15 of every 16, differently from run to run, at the bench size
    // (r06o tools/chain_next_determinism.py; every other form repeatable) -- x2 is refused until that is understood.
    if (x2) return BEV_ERR_ARGS;
    (void)H2, (void)W2, (void)Ci2, (void)stride2;
    if (N == 0) return 0;
    ConvX a;
    a.x = nullptr;
    a.wp = (const __bf16 *)packed;
    a.bias = bias;
    a.res = residual;
    a.y = y;
    a.N = N, a.H = H, a.W = W, a.Ci = Ci, a.Co = Co, a.KH = KH, a.KW = KW, a.stride = stride, a.pad = pad;
    a.dil = 1, a.Ho = Ho, a.Wo = Wo, a.act = act, a.ldy = Co2;
    a.Kp = (int)kpad_x(Ci * KH * KW);
    a.M = (int64_t)N * Ho * Wo;
    a.x2 = x2;
    a.Ci2 = x2 ? Ci2 : 0, a.H2 = x2 ? H2 : 0, a.W2 = x2 ? W2 : 0, a.stride2 = x2 ? stride2 : 0;
    a.xs = (const __bf16 *)xs;
    a.ys = nullptr;
    a.xps = (int64_t)N * H * W * Ci;
    a.yps = 0;
    a.wp2 = (const __bf16 *)packed2;
    a.bias2 = bias2;
    a.Co2 = Co2;
    a.act2 = act2;
    a.wp3 = (const __bf16 *)packed3;
    a.bias3 = bias3;
    a.Co3 = Co3;
    a.act3 = act3;
    a.y3 = y3;
    a.ys3 = (__bf16 *)ys3;
    const hipStream_t st = (hipStream_t)stream;
    return Co3 == 64 ? launch_x6s<4, 1, 1, 2, 1, 2>(a, st) : launch_x6s<4, 1, 1, 2, 1, 4>(a, st);
}

int bev_conv2d_stem_x6_f32(const float *x, int N, int H, int W, const uint16_t *packed, const float *bias, int Co,
                           int relu, float *y, int Ho, int Wo, void *stream) {
    if (!x || !packed || !bias || !y || N <= 0 || H <= 0 || W <= 0 || Co <= 0 || Co > 64 ||
        Ho != (H + 6 - 7) / 2 + 1 || Wo != (W + 6 - 7) / 2 + 1 || (((uintptr_t)packed) & 15) != 0)
        return BEV_ERR_ARGS;
    static int num_cu = 0;
    if (num_cu == 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        num_cu = n;
    }
    StemX6Args a;
    a.x = x;
    a.wp = (const __bf16 *)packed;
    a.bias = bias;
    a.y = y;
    a.H = H, a.W = W, a.Co = Co, a.Ho = Ho, a.Wo = Wo, a.relu = relu;
    a.nTx = (Wo + stem6::TW - 1) / stem6::TW;
    a.nTy = (Ho + stem6::TH - 1) / stem6::TH;
    a.ntiles = (int64_t)N * a.nTx * a.nTy;
    a.edge_b = a.edge_r = nullptr;
    a.Hp = a.Wp = 0;
    const int64_t grid = a.ntiles < num_cu ? a.ntiles : num_cu;
    hipLaunchKernelGGL(k_stem_x6<false>, dim3((unsigned)grid), dim3(stem6::NTHR), 0, (hipStream_t)stream, a);
    return (int)hipGetLastError();
}

int64_t bev_conv2d_stem_pool_x6_workspace(int N, int H, int W) {
    if (N <= 0 || H <= 0 || W <= 0) return BEV_ERR_ARGS;
    const int Ho = (H + 6 - 7) / 2 + 1, Wo = (W + 6 - 7) / 2 + 1;
    const int64_t nt = (int64_t)N * ((Wo + stem6::TW - 1) / stem6::TW) * ((Ho + stem6::TH - 1) / stem6::TH);
    return nt * (32 + 5) * 64 * (int64_t)sizeof(float);
}

int bev_conv2d_stem_pool_x6_f32(const float *x, int N, int H, int W, const uint16_t *packed, const float *bias,
                                int Co, float *y, int Hp, int Wp, void *workspace, int64_t workspace_bytes,
                                void *stream) {
    const int Ho = (H + 6 - 7) / 2 + 1, Wo = (W + 6 - 7) / 2 + 1;
    if (!x || !packed || !bias || !y || !workspace || N <= 0 || H <= 0 || W <= 0 || Co != 64 ||
        Hp != (Ho + 2 - 3) / 2 + 1 || Wp != (Wo + 2 - 3) / 2 + 1 || (((uintptr_t)packed | (uintptr_t)y |
                                                                       (uintptr_t)workspace) & 15) != 0)
        return BEV_ERR_ARGS;
    if (workspace_bytes < bev_conv2d_stem_pool_x6_workspace(N, H, W)) return BEV_ERR_ARGS;
    static int num_cu = 0;
    if (num_cu == 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        num_cu = n;
    }
    StemX6Args a;
    a.x = x;
    a.wp = (const __bf16 *)packed;
    a.bias = bias;
    a.y = y;
    a.H = H, a.W = W, a.Co = Co, a.Ho = Ho, a.Wo = Wo, a.relu = 1;
    a.nTx = (Wo + stem6::TW - 1) / stem6::TW;
    a.nTy = (Ho + stem6::TH - 1) / stem6::TH;
    a.ntiles = (int64_t)N * a.nTx * a.nTy;
    a.edge_b = (float *)workspace;
    a.edge_r = a.edge_b + a.ntiles * 32 * 64;
    a.Hp = Hp, a.Wp = Wp;
    const int64_t grid = a.ntiles < num_cu ? a.ntiles : num_cu;
    hipLaunchKernelGGL(k_stem_x6<true>, dim3((unsigned)grid), dim3(stem6::NTHR), 0, (hipStream_t)stream, a);
    const int64_t nthr = a.ntiles * 35 * 16;
    hipLaunchKernelGGL(k_stem_pool_seams, dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, (hipStream_t)stream, y,
                       a.edge_b, a.edge_r, a.nTx, a.nTy, a.ntiles, Hp, Wp);
    return (int)hipGetLastError();
}

}  // extern "C"
