// bev_conv.hip -- per-camera backbone convolutions for gfx950 (MI355X).
//
// Replaces the convolution stack the reference runs per camera in
// CNNEncoder._encode_single (cnn_encoder.py:39-48): the timm ResNet
// `features_only` graph (cnn_encoder.py:26,41-42) + the lazy 1x1 projection
// (cnn_encoder.py:43-46), or the fallback 2-conv stack (cnn_encoder.py:31-37).
//
// Convolution = implicit GEMM on the exact-f32 MFMA (v_mfma_f32_32x32x2_f32,
// 64 FLOP/clk/SIMD, bitwise an fmaf chain):
//     y[m][n] = act( sum_k A[m][k] * W[k][n] + bias[n] (+ res[m][n]) )
//     m = (image, oy, ox), n = output channel, k = (ky, kx, ci)
// Activations are channels-last (NHWC) so that a 16-deep K step of a layer
// with Ci % 16 == 0 is one contiguous 64-B run per output pixel.  The stem
// (Ci = 3, images NCHW straight from the caller) uses a per-element loader.
//
// Tiling: 256 threads = 4 waves as WM x WN, each wave 64 x 64 outputs
// (2 x 2 MFMA tiles of 32 x 32, 64 accumulator VGPRs).  K step BK = 16 staged
// global -> registers -> LDS, double-buffered (issue the next step's global
// loads before the MFMAs of this one, write them to the other LDS buffer
// after; one barrier per step).  Inside a K step the MFMA's two k-slots are
// mapped to k = 8*h + p (h = lane >> 5, p = 0..7) so each lane's eight A and
// eight B operands are two contiguous ds_read_b128 from [row][k] images padded
// to 80-B rows (conflict-free 16-lane groups).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "../../include/bev_mi355x.h"
#include "bev_act.h"
#include "bev_tune.h"

namespace {

constexpr int BK = 32;        // K step
constexpr int LROW = BK + 4;  // LDS row stride in floats (144 B: 9 slots, odd -> conflict-free b128 rows)

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));  // native vector: promotes to VGPRs reliably

// 16 zero bytes in device memory: out-of-range operand taps load from here (an unconditional load
// through a selected pointer), so the K loop has no branches around loads and hipcc's vmcnt
// bookkeeping stays exact (a select on the loaded VALUE gets sunk into a branch around the load).
__device__ __attribute__((aligned(16))) float g_zero4[4] = {0.f, 0.f, 0.f, 0.f};  // never written

__host__ __device__ inline int64_t kpad(int K) { return (K + BK - 1) / BK * BK; }
__host__ __device__ inline int64_t copad(int Co) { return (Co + 127) / 128 * 128; }

// ---------------------------------------------------------------------------
// weight packing: OIHW -> [Co_pad][K_pad], k = (ky*KW + kx)*Ci + ci
// ---------------------------------------------------------------------------
__global__ void k_pack(const float *__restrict__ w, int Co, int Ci, int KH, int KW, int64_t Kp, int64_t Cop,
                       float *__restrict__ out) {
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
    out[t] = v;
}

// Epilogue activation: 1 = ReLU, 2 = SiLU (torch: x / (1 + exp(-x)); EfficientNet trunk).
__device__ __forceinline__ float act_fn(float t, int act) {
    if (act == 2) return silu_hw(t);
    return t > 0.0f ? t : 0.0f;
}

struct ConvArgs {
    const float *__restrict__ x;
    const float *__restrict__ wp;
    const float *__restrict__ bias;
    const float *__restrict__ res;
    float *__restrict__ y;
    int N, H, W, Ci, Co, KH, KW, stride, pad, Ho, Wo;
    int relu;
    int in_nchw;  // generic loader only: input is NCHW instead of NHWC
    int64_t M;
    int K;
    int Kp;
    // dual-source 1x1 (LOADER 3): k in [Ci, Ci + Ci2) reads x2 [N][H2][W2][Ci2] at (oy*s2, ox*s2)
    const float *__restrict__ x2;
    int Ci2, H2, W2, stride2;
    // per-(image, input channel) multiplier of the A operand (SqueezeExcite excitation folded into
    // the projection conv's loader: conv(x * gate)); NULL = none.  Fast and contiguous loaders only.
    const float *__restrict__ ascale;
    // with ascale: per-(image, input channel) shift added after the scale, then ReLU when arelu
    // (a GroupNorm + ReLU of the previous layer applied on the fly; out-of-range taps stay 0)
    const float *__restrict__ ashift;
    int arelu;
    int dil;  // dilation of the taps (input offset ky * dil, kx * dil)
    int ldy;  // row stride of y in floats (>= Co; a channel slice of a wider NHWC buffer)
    int xcd;  // 1: XCD-aware block order (the N tiles of one M block run on one XCD, sharing its L2)
    // chained pointwise conv (EPI 1, bev_conv2d_chain_f32): y = act2(h (*) W2 + bias2 + res), h = this conv's output
    const float *__restrict__ wp2;
    const float *__restrict__ bias2;
    int Co2, Kp2, relu2;
    int pwvec;  // k_pw_mfma: float4 epilogue through LDS (set by try_pw_mfma)
};

// Per-thread view of the A tile rows it loads: rows (tid >> 3) + 32 r, one 16-B quad.
template <int ROWS>
struct RowsA {
    int64_t pix[ROWS];  // element offset of the row's image
    int iy0[ROWS], ix0[ROWS], img[ROWS];
    bool ok[ROWS];
    bool uni;  // every row of the tile lies in one image (img[0]): one gate quad per K step
    __device__ void init(const ConvArgs &a, int64_t m0, int tid) {
        {
            const int64_t hw = (int64_t)a.Ho * a.Wo, last = (m0 + 32 * ROWS - 1 < a.M) ? m0 + 32 * ROWS - 1 : a.M - 1;
            uni = (m0 / hw) == (last / hw);
        }
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            const int64_t m = m0 + (tid >> 3) + 32 * r;
            ok[r] = m < a.M;
            const int64_t mm = ok[r] ? m : 0;
            const int ox = (int)(mm % a.Wo);
            const int64_t t = mm / a.Wo;
            const int oy = (int)(t % a.Ho);
            const int n = (int)(t / a.Ho);
            pix[r] = (int64_t)n * a.H * a.W * a.Ci;
            img[r] = n;
            iy0[r] = oy * a.stride - a.pad;
            ix0[r] = ox * a.stride - a.pad;
        }
    }
};

// A loader, fast path: NHWC, Ci % 32 == 0 -> a K step is one (ky, kx) and 32
// consecutive channels, i.e. one contiguous 128-B run per output pixel.  The
// (ky, kx, ci0) position advances incrementally (no divisions in the loop).
// SCALE: multiply by the per-(image, channel) ascale (SE excitation; LOADER 6).
template <int ROWS, bool SCALE = false>
struct LoaderFast {
    static constexpr int NV = ROWS;  // float4 per thread and K step
    RowsA<ROWS> rows;
    int quad, ky, kx, ci0;
    __device__ void init(const ConvArgs &a, int64_t m0, int tid) {
        rows.init(a, m0, tid);
        quad = tid & 7;
        ky = kx = ci0 = 0;
    }
    // A tile image: row (tid >> 3) + 32 r, k columns quad*4 .. +3
    __device__ void store(float *As, int tid, const f32x4 (&v)[NV]) const {
#pragma unroll
        for (int r = 0; r < ROWS; ++r) *(f32x4 *)(As + ((tid >> 3) + 32 * r) * LROW + quad * 4) = v[r];
    }
    __device__ void load(const ConvArgs &a, f32x4 (&v)[NV]) {
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            const int iy = rows.iy0[r] + ky, ix = rows.ix0[r] + kx;
            const bool in = rows.ok[r] && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
            const float *src = in ? a.x + rows.pix[r] + ((int64_t)iy * a.W + ix) * a.Ci + ci0 + quad * 4 : g_zero4;
            v[r] = *(const f32x4 *)src;
            if (SCALE && !rows.uni && in)
                v[r] *= *(const f32x4 *)(a.ascale + (int64_t)rows.img[r] * a.Ci + ci0 + quad * 4);
        }
        if (SCALE && rows.uni) {
            const f32x4 g = *(const f32x4 *)(a.ascale + (int64_t)rows.img[0] * a.Ci + ci0 + quad * 4);
#pragma unroll
            for (int r = 0; r < ROWS; ++r) v[r] *= g;  // out-of-range rows are 0 and stay 0
        }
    }
    __device__ void advance(const ConvArgs &a) {
        ci0 += BK;
        if (ci0 == a.Ci) {
            ci0 = 0;
            if (++kx == a.KW) {
                kx = 0;
                ++ky;
            }
        }
    }
};

// A loader, fast path with a dilated tap grid and the previous layer's GroupNorm + ReLU applied on the
// fly (BEV head, bev_conv2d_nhwc_ex_f32): x' = relu?(x * ascale[n][ci] + ashift[n][ci]) for in-range
// taps.  A separate instantiation keeps LoaderFast's register budget (and the trunk's occupancy).
template <int ROWS>
struct LoaderFastEx : LoaderFast<ROWS> {
    using LoaderFast<ROWS>::rows;
    using LoaderFast<ROWS>::quad;
    using LoaderFast<ROWS>::ky;
    using LoaderFast<ROWS>::kx;
    using LoaderFast<ROWS>::ci0;
    static constexpr int NV = ROWS;
    __device__ void load(const ConvArgs &a, f32x4 (&v)[NV]) {
        bool inr[ROWS];
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            const int iy = rows.iy0[r] + ky * a.dil, ix = rows.ix0[r] + kx * a.dil;
            const bool in = rows.ok[r] && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
            inr[r] = in;
            v[r] = in ? *(const f32x4 *)(a.x + rows.pix[r] + ((int64_t)iy * a.W + ix) * a.Ci + ci0 + quad * 4)
                      : (f32x4){0.f, 0.f, 0.f, 0.f};
            if (a.ascale && !rows.uni && in) {
                const int64_t o = (int64_t)rows.img[r] * a.Ci + ci0 + quad * 4;
                v[r] *= *(const f32x4 *)(a.ascale + o);
                if (a.ashift) v[r] += *(const f32x4 *)(a.ashift + o);
                if (a.arelu) v[r] = __builtin_elementwise_max(v[r], (f32x4){0.f, 0.f, 0.f, 0.f});
            }
        }
        if (a.ascale && rows.uni) {
            const int64_t o = (int64_t)rows.img[0] * a.Ci + ci0 + quad * 4;
            const f32x4 g = *(const f32x4 *)(a.ascale + o);
            if (!a.ashift) {
#pragma unroll
                for (int r = 0; r < ROWS; ++r) v[r] *= g;  // out-of-range rows are 0 and stay 0
            } else {
                const f32x4 sh = *(const f32x4 *)(a.ashift + o);
#pragma unroll
                for (int r = 0; r < ROWS; ++r) {
                    f32x4 t = v[r] * g + sh;
                    if (a.arelu) t = __builtin_elementwise_max(t, (f32x4){0.f, 0.f, 0.f, 0.f});
                    v[r] = inr[r] ? t : v[r];  // zero padding is applied after the normalisation
                }
            }
        }
    }
};

// A loader, dual-source 1x1 (bottleneck conv3 + downsample shortcut in ONE GEMM):
// K = [0, Ci) reads x [M][Ci] (the conv3 input, one pixel per output pixel),
// K = [Ci, Ci + Ci2) reads x2 at the strided pixel (oy*s2, ox*s2) -- the
// downsample's 1x1/stride-s2 input.  Ci, Ci2 % 32 == 0.
template <int ROWS>
struct LoaderDual {
    static constexpr int NV = ROWS;
    int64_t p1[ROWS], p2[ROWS];
    bool ok[ROWS];
    int quad, k0;
    __device__ void init(const ConvArgs &a, int64_t m0, int tid) {
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            const int64_t m = m0 + (tid >> 3) + 32 * r;
            ok[r] = m < a.M;
            const int64_t mm = ok[r] ? m : 0;
            const int ox = (int)(mm % a.Wo);
            const int64_t t = mm / a.Wo;
            const int oy = (int)(t % a.Ho);
            const int64_t n = t / a.Ho;
            p1[r] = mm * a.Ci;
            p2[r] = ((n * a.H2 + (int64_t)oy * a.stride2) * a.W2 + (int64_t)ox * a.stride2) * a.Ci2;
        }
        quad = tid & 7;
        k0 = 0;
    }
    __device__ void store(float *As, int tid, const f32x4 (&v)[NV]) const {
#pragma unroll
        for (int r = 0; r < ROWS; ++r) *(f32x4 *)(As + ((tid >> 3) + 32 * r) * LROW + quad * 4) = v[r];
    }
    __device__ void load(const ConvArgs &a, f32x4 (&v)[NV]) {
        const bool first = k0 < a.Ci;  // wave-uniform
        const float *src = first ? a.x + k0 : a.x2 + (k0 - a.Ci);
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            const int64_t off = (first ? p1[r] : p2[r]) + quad * 4;
            v[r] = *(const f32x4 *)(ok[r] ? src + off : g_zero4);
        }
    }
    __device__ void advance(const ConvArgs &) { k0 += BK; }
};

// A loader, pointwise 1x1 / stride 1 / pad 0 over NHWC with Ci % 4 == 0 (but not
// % 32: EfficientNet widths 24, 40, 48, 144): row m's A data is x[m][0 .. Ci),
// one contiguous run; a K step reads quads k0 + 4 quad, zero past Ci (K padding).
template <int ROWS>
struct LoaderContig {
    static constexpr int NV = ROWS;
    int64_t p[ROWS], g[ROWS];
    bool ok[ROWS], uni;
    int quad, k0;
    __device__ void init(const ConvArgs &a, int64_t m0, int tid) {
        const int64_t hw = (int64_t)a.Ho * a.Wo;
        const int64_t last = (m0 + 32 * ROWS - 1 < a.M) ? m0 + 32 * ROWS - 1 : a.M - 1;
        uni = (m0 / hw) == (last / hw);
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            const int64_t m = m0 + (tid >> 3) + 32 * r;
            ok[r] = m < a.M;
            p[r] = (ok[r] ? m : 0) * a.Ci;
            g[r] = a.ascale ? ((ok[r] ? m : 0) / hw) * a.Ci : 0;
        }
        quad = tid & 7;
        k0 = 0;
    }
    __device__ void store(float *As, int tid, const f32x4 (&v)[NV]) const {
#pragma unroll
        for (int r = 0; r < ROWS; ++r) *(f32x4 *)(As + ((tid >> 3) + 32 * r) * LROW + quad * 4) = v[r];
    }
    __device__ void load(const ConvArgs &a, f32x4 (&v)[NV]) {
        const int k = k0 + quad * 4;
        const bool kin = k < a.Ci;
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            v[r] = (ok[r] && kin) ? *(const f32x4 *)(a.x + p[r] + k) : (f32x4){0.f, 0.f, 0.f, 0.f};
            if (a.ascale && !uni && ok[r] && kin) v[r] *= *(const f32x4 *)(a.ascale + g[r] + k);
        }
        if (a.ascale && uni && kin) {
            const f32x4 gq = *(const f32x4 *)(a.ascale + g[0] + k);
#pragma unroll
            for (int r = 0; r < ROWS; ++r) v[r] *= gq;  // out-of-range rows are 0 and stay 0
        }
    }
    __device__ void advance(const ConvArgs &) { k0 += BK; }
};

// A loader, generic path (any Ci, NHWC or NCHW input), element-wise.  Each
// thread owns ONE output pixel (row) of the tile and a contiguous run of KPT
// k's, so for a given k the 64 lanes of a wave read 64 neighbouring output
// pixels (coalesced) and the k -> (ky, kx, ci) decode is wave-uniform.
// CI / KWc > 0 bake the geometry in (the ResNet stem: Ci = 3, 7 x 7, NCHW).
template <int BM, int CI = 0, int KWc = 0>
struct LoaderRow {
    static constexpr int TPR = 256 / BM;  // threads per row
    static constexpr int KPT = BK / TPR;  // k's per thread and K step
    static constexpr int NV = KPT / 4;
    int64_t pix;
    int iy0, ix0, row, kq, k0;
    bool ok, nchw;
    __device__ void init(const ConvArgs &a, int64_t m0, int tid) {
        row = tid % BM;
        kq = tid / BM;
        const int64_t m = m0 + row;
        ok = m < a.M;
        const int64_t mm = ok ? m : 0;
        const int ox = (int)(mm % a.Wo);
        const int64_t t = mm / a.Wo;
        const int oy = (int)(t % a.Ho);
        const int n = (int)(t / a.Ho);
        pix = (int64_t)n * a.H * a.W * a.Ci;
        iy0 = oy * a.stride - a.pad;
        ix0 = ox * a.stride - a.pad;
        k0 = 0;
        nchw = a.in_nchw != 0;
    }
    __device__ void store(float *As, int, const f32x4 (&v)[NV]) const {
#pragma unroll
        for (int i = 0; i < KPT / 4; ++i) *(f32x4 *)(As + row * LROW + kq * KPT + 4 * i) = v[i];
    }
    __device__ void load(const ConvArgs &a, f32x4 (&v)[NV]) {
        const int Ci = CI > 0 ? CI : a.Ci, KW = KWc > 0 ? KWc : a.KW;
        float e[KPT];
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const int k = k0 + kq * KPT + j;  // uniform across the wave
            const int ci = k % Ci, rr = k / Ci, kx = rr % KW, ky = rr / KW;
            const int dil = CI > 0 ? 1 : a.dil;  // the stem instantiation keeps its constant geometry
            const int iy = iy0 + ky * dil, ix = ix0 + kx * dil;
            const bool in = ok && (k < a.K) && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
            const int64_t off = nchw ? pix + ((int64_t)ci * a.H + iy) * a.W + ix : pix + ((int64_t)iy * a.W + ix) * Ci + ci;
            e[j] = in ? a.x[off] : 0.0f;
        }
#pragma unroll
        for (int i = 0; i < KPT / 4; ++i) v[i] = (f32x4){e[4 * i], e[4 * i + 1], e[4 * i + 2], e[4 * i + 3]};
    }
    __device__ void advance(const ConvArgs &) { k0 += BK; }
};

template <int R>
__device__ __forceinline__ void load_rows(f32x4 (&v)[R], const float *__restrict__ p, int64_t ld, int k) {
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = *(const f32x4 *)(p + (int64_t)(32 * r) * ld + k);
}

template <int R>
__device__ __forceinline__ void store_rows(float *p, const f32x4 (&v)[R]) {
#pragma unroll
    for (int r = 0; r < R; ++r) *(f32x4 *)(p + 32 * r * LROW) = v[r];
}

// Standard epilogue: the wave's (TM*32) x (TN*32) accumulator tile goes to LDS (4 * 32 TM x (32 TN + 4)
// floats for the block; the caller sizes its LDS for it), then every lane issues ALL its residual float4
// loads at once (deep memory parallelism for the memory-bound 1x1 layers), combines and stores whole
// float4 row pieces.
template <int TM, int TN>
__device__ __forceinline__ void conv_epilogue(const ConvArgs &a, float *lds, const f32x16 (&acc)[TM][TN], int wave,
                                              int lane, int wm, int wn, int64_t m0, int n0) {
    const int r32 = lane & 31, h = lane >> 5;
    // D[row][col]: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5).
    constexpr int WR = TM * 32, WC = TN * 32, ER = WC + 4;  // wave tile, LDS row stride
    constexpr int C4 = WC / 4;                              // float4 per row
    constexpr int RPI = 64 / C4;                            // rows per wave-instruction
    constexpr int NQ = WR / RPI;                            // float4 per lane
    __syncthreads();  // every wave is done reading the staging buffers
    float *E = lds + wave * (WR * ER);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) E[(i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * ER + j * 32 + r32] = acc[i][j][r];
    // same-wave LDS ops complete in order: no barrier needed
    const int c4 = lane % C4, rq = lane / C4;
    const int n = n0 + wn * WC + c4 * 4;
    const bool nvec = ((a.Co & 3) == 0) && ((a.ldy & 3) == 0) && (n + 3 < a.Co);
    const int64_t mbase = m0 + wm * WR;
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
    float4 rv[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int64_t m = mbase + rq + RPI * q;
        rv[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (a.res && m < a.M && nvec) rv[q] = *(const float4 *)(a.res + m * a.Co + n);
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int row = rq + RPI * q;
        const int64_t m = mbase + row;
        if (m >= a.M) continue;
        const float4 v = *(const float4 *)(E + row * ER + c4 * 4);
        float o[4] = {v.x + bv.x, v.y + bv.y, v.z + bv.z, v.w + bv.w};
        float *yp = a.y + m * a.ldy + n;
        if (nvec) {
            if (a.res) {
                o[0] += rv[q].x;
                o[1] += rv[q].y;
                o[2] += rv[q].z;
                o[3] += rv[q].w;
            }
            if (a.relu) {
#pragma unroll
                for (int u = 0; u < 4; ++u) o[u] = act_fn(o[u], a.relu);
            }
            *(float4 *)yp = make_float4(o[0], o[1], o[2], o[3]);
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (n + u >= a.Co) break;
                float t = o[u];
                if (a.res) t += a.res[m * a.Co + n + u];
                if (a.relu) t = act_fn(t, a.relu);
                yp[u] = t;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Chained pointwise epilogue (EPI 1; bev_conv2d_chain_f32)
// ---------------------------------------------------------------------------
// timm Bottleneck.forward without a downsample: act3(bn3(conv3(act2(bn2(conv2(h1))))) + x).
// The block's BM x BN tile of h2 = act(conv2(h1) + b2) holds EVERY channel of h2 for its BM
// pixels (BN == Co), so conv3 (1x1, K2 = Co) runs on it straight from LDS:
//     y = act2( h2 (*) W3 + b3 + res )
// and h2 never makes its HBM round trip (write + read of M x Co floats).  Each wave computes its
// 32 rows x (Co2 / WN) columns in 64-column chunks (2 MFMA tiles); the W3 fragments stream from
// L2 (the panel is shared by every block) one 16-deep half step ahead; the chunk's residual is
// loaded before its MFMAs.  K2 order = the main loop's (k-slot h of MFMA p reads 16 h + 8 half + p
// inside each 32-deep step), so y is bit-identical to the two-launch chain.
// Buffer resources (base, byte size): the lane's row is in the VGPR offset (the part the range
// check sees), so loads / stores of rows past the block's last one return 0 / are dropped; the
// uniform column / k offset goes to the SGPR soffset.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t chain_rsrc(const float *p, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(p), 0, (int)(uint32_t)bytes, 0x00020000);
}

// W2 fragments of half step t (k = 32 (t >> 1) + 16 hh + 8 (t & 1) + 0..7) for columns c0 + 32 j + r32.
__device__ __forceinline__ void chain_load_b(__amdgpu_buffer_rsrc_t rw, int kp2, int voff, int c0, int t,
                                             f32x4 (&w)[2][2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int so = ((c0 + 32 * j) * kp2 + 32 * (t >> 1) + 8 * (t & 1) + 4 * q) * 4;
            w[j][q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rw, voff, so, 0));
        }
}

__device__ __forceinline__ void chain_mfma_r(f32x16 (&acc)[2], const f32x4 &a0, const f32x4 &a1,
                                             const f32x4 (&w)[2][2]) {
#pragma unroll
    for (int p = 0; p < 8; ++p) {
        const float av = (p < 4 ? a0 : a1)[p & 3];
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, w[j][p >> 2][p & 3], acc[j], 0, 0, 0);
    }
}

__device__ __forceinline__ void chain_mfma(f32x16 (&acc)[2], const float *ap, int t, const f32x4 (&w)[2][2]) {
    const float *pa = ap + 32 * (t >> 1) + 8 * (t & 1);
    chain_mfma_r(acc, *(const f32x4 *)pa, *(const f32x4 *)(pa + 4), w);
}

// x2 (shortcut) operand of half step t >= BN / 16: k2 = 32 (t >> 1) + 16 hh + 8 (t & 1) - BN of the
// lane's strided pixel (16 hh is in voff).  With no x2 the resource has 0 records: the load returns 0.
__device__ __forceinline__ void chain_load_x(__amdgpu_buffer_rsrc_t rx, int voff, int t, int bn, f32x4 (&x)[2]) {
    const int so = (32 * (t >> 1) + 8 * (t & 1) - bn) * 4;
    x[0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, voff, so, 0));
    x[1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, voff, so + 16, 0));
}

template <int WM, int WN, int TM, int TN>
__device__ __forceinline__ void chain_epilogue(const ConvArgs &a, float *lds, const f32x16 (&acc)[TM][TN], int wm,
                                               int wn, int lane, int64_t m0) {
    static_assert(TM == 1 && TN == 2, "chain epilogue: each wave owns 32 rows x 64 channels of h2");
    constexpr int BM = WM * 32, BN = WN * 64, LA = BN + 4;  // h2 image [BM][LA]: 4 LA B = odd 16-B slot count
    constexpr int HS = BN / 16;                              // 16-deep half steps of the h2 part (K = BN)
    const int r32 = lane & 31, hh = lane >> 5;
    __syncthreads();  // every wave is done with the staging buffers
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int col = wn * 64 + j * 32 + r32;
        const float bj = a.bias ? a.bias[col] : 0.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            float o = acc[0][j][r] + bj;
            if (a.relu) o = act_fn(o, a.relu);
            lds[(wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh) * LA + col] = o;
        }
    }
    __syncthreads();
    const int ncols = a.Co2 / WN, nch = ncols / 64;
    const int cb = wn * ncols;
    const float *ap = lds + (wm * 32 + r32) * LA + 16 * hh;
    // this block's rows of res / y: [m0, min(m0 + BM, M)) x Co2 (ldy == Co2)
    const int64_t rows = (a.M - m0 < BM) ? a.M - m0 : BM;
    const int64_t base = m0 * a.Co2;
    const __amdgpu_buffer_rsrc_t ry = chain_rsrc(a.y + base, rows * a.Co2 * 4);
    const __amdgpu_buffer_rsrc_t rr = chain_rsrc(a.res ? a.res + base : a.y + base, rows * a.Co2 * 4);
    const __amdgpu_buffer_rsrc_t rw = chain_rsrc(a.wp2, (int64_t)copad(a.Co2) * a.Kp2 * 4);
    const int vw = (r32 * a.Kp2 + 16 * hh) * 4;                // lane part of a W2 address
    const int vo = ((wm * 32 + 4 * hh) * a.Co2 + r32) * 4;     // lane part of a res / y address
    // dual (downsample shortcut): K2 = [h2 | x2 at the lane row's strided pixel], x2 [N][H2][W2][Ci2]
    const int hs2 = a.x2 ? a.Ci2 / 16 : 0;
    __amdgpu_buffer_rsrc_t rx = chain_rsrc(a.y, 0);
    int vx = 0;
    if (a.x2) {
        int64_t m = m0 + wm * 32 + r32;
        m = m < a.M ? m : a.M - 1;
        const int ox = (int)(m % a.Wo);
        const int64_t q = m / a.Wo;
        const int oy = (int)(q % a.Ho);
        const int64_t n = q / a.Ho;
        rx = chain_rsrc(a.x2, (int64_t)a.N * a.H2 * a.W2 * a.Ci2 * 4);
        vx = (int)((((n * a.H2 + (int64_t)oy * a.stride2) * a.W2 + (int64_t)ox * a.stride2) * a.Ci2 + 16 * hh) * 4);
    }
    f32x4 wA[2][2], wB[2][2], xA[2], xB[2];
    chain_load_b(rw, a.Kp2, vw, cb, 0, wA);
    for (int nc = 0; nc < nch; ++nc) {
        const int c0 = cb + 64 * nc, cn = nc + 1 < nch ? c0 + 64 : c0;  // next chunk (clamped)
        float rv[2][16];
        if (a.res) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    rv[j][r] = __builtin_bit_cast(
                        float, __builtin_amdgcn_raw_buffer_load_b32(rr, vo + ((r & 3) + 8 * (r >> 2)) * a.Co2 * 4,
                                                                    (c0 + 32 * j) * 4, 0));
        }
        f32x16 acc2[2] = {(f32x16){0}, (f32x16){0}};
#pragma unroll
        for (int t = 0; t < HS; t += 2) {
            chain_load_b(rw, a.Kp2, vw, c0, t + 1, wB);
            chain_mfma(acc2, ap, t, wA);
            // after the h2 part's last half step: the x2 part's first, or the next chunk's first
            // (unconditional loads: clamped chunk; x2 loads read 0 without an x2)
            const bool lst = (t + 2 == HS);
            if (lst) {
                chain_load_b(rw, a.Kp2, vw, hs2 ? c0 : cn, hs2 ? HS : 0, wA);
                chain_load_x(rx, vx, HS, BN, xA);
            } else {
                chain_load_b(rw, a.Kp2, vw, c0, t + 2, wA);
            }
            chain_mfma(acc2, ap, t + 1, wB);
            __builtin_amdgcn_sched_barrier(0);  // one half step of W2 in flight (VGPR budget of 3 blocks / CU)
        }
        for (int t = HS; t < HS + hs2; t += 2) {
            chain_load_b(rw, a.Kp2, vw, c0, t + 1, wB);
            chain_load_x(rx, vx, t + 1, BN, xB);
            chain_mfma_r(acc2, xA[0], xA[1], wA);
            const bool lst = (t + 2 == HS + hs2);
            chain_load_b(rw, a.Kp2, vw, lst ? cn : c0, lst ? 0 : t + 2, wA);
            chain_load_x(rx, vx, lst ? t + 1 : t + 2, BN, xA);
            chain_mfma_r(acc2, xB[0], xB[1], wB);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const float bj = a.bias2 ? a.bias2[c0 + 32 * j + r32] : 0.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                float o = acc2[j][r] + bj;
                if (a.res) o += rv[j][r];
                if (a.relu2) o = act_fn(o, a.relu2);
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o), ry,
                                                      vo + ((r & 3) + 8 * (r >> 2)) * a.Co2 * 4, (c0 + 32 * j) * 4, 0);
            }
        }
    }
}

// Block = WM x WN waves; each wave owns TM x TN MFMA tiles of 32 x 32.
// LOADER: 0 generic, 1 fast (NHWC, Ci % 32 == 0), 2 stem (NCHW, Ci = 3, 7 x 7), 3 dual 1x1,
// 4 contiguous 1x1 (NHWC, Ci % 4 == 0), 5 fast + dilation + GroupNorm/ReLU operand affine,
// 6 fast + per-(image, channel) operand scale
// NBUF: LDS staging buffers.  2 = one barrier per K step; 1 = half the LDS (a
// third workgroup per CU for the <= 170-VGPR tiles) at two barriers per K step.
template <int WM, int WN, int TM, int TN, int LOADER, int NBUF, int CHAIN = 0>
__global__ __launch_bounds__(256, NBUF == 1 ? 3 : 2) void k_conv(ConvArgs a) {
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
    constexpr int AROWS = BM / 32;  // A rows per thread (rows tid/8 + 32 r)
    constexpr int BROWS = BN / 32;
    constexpr int STAGE = (BM + BN) * LROW;
    constexpr int EPI = 4 * (TM * 32) * (TN * 32 + 4);  // epilogue tile (see below)
    constexpr int LDSF = NBUF * STAGE > EPI ? NBUF * STAGE : EPI;
    __shared__ __attribute__((aligned(16))) float lds[LDSF];

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int n_tiles = (a.Co + BN - 1) / BN;
    // Consecutive blockIdx.x go round-robin over the 8 XCDs; with a.xcd the logical tile order is
    // remapped so each XCD walks a contiguous run: the n_tiles blocks that read the same A rows are
    // dispatched together on one XCD and share its L2 instead of fetching A once per XCD.
    unsigned bid = blockIdx.x;
    if (a.xcd) {
        const unsigned nb = gridDim.x, q = nb / 8, r = nb % 8, x = bid % 8;
        bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
    }
    const int64_t m0 = (int64_t)(bid / n_tiles) * BM;
    const int n0 = (bid % n_tiles) * BN;

    typename std::conditional<
        LOADER == 1, LoaderFast<AROWS>, typename std::conditional<LOADER == 6, LoaderFast<AROWS, true>,
        typename std::conditional<LOADER == 5, LoaderFastEx<AROWS>,
        typename std::conditional<LOADER == 2, LoaderRow<BM, 3, 7>,
                                  typename std::conditional<
                                      LOADER == 3, LoaderDual<AROWS>,
                                      typename std::conditional<LOADER == 4, LoaderContig<AROWS>,
                                                                LoaderRow<BM>>::type>::type>::type>::type>::type>::type la;
    la.init(a, m0, tid);
    const int bq = tid & 7;
    const float *wrow = a.wp + (int64_t)(n0 + (tid >> 3)) * a.Kp + bq * 4;

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){0};

    // global -> register prefetch, TWO K steps ahead (macros, not lambdas: register
    // arrays captured by reference were address-taken and landed in scratch).
    // Step ks: register set ks&1 receives step ks+2 while the MFMAs consume LDS
    // buffer ks&1; the other set (step ks+1) is then written to the other LDS buffer.
    constexpr int NV = decltype(la)::NV;
    f32x4 va0[NV], va1[NV], rb0[BROWS], rb1[BROWS];
    int kb = 0;  // k offset of the B panel
#define BEV_GLOAD(VA, RB)                     \
    do {                                      \
        la.load(a, VA);                       \
        load_rows<BROWS>(RB, wrow, a.Kp, kb); \
        la.advance(a);                        \
        kb += BK;                             \
    } while (0)
#define BEV_SWRITE(buf, VA, RB)                                                                        \
    do {                                                                                               \
        la.store(lds + (NBUF == 2 ? (buf) : 0) * STAGE, tid, VA);                                      \
        store_rows<BROWS>(lds + (NBUF == 2 ? (buf) : 0) * STAGE + (BM + (tid >> 3)) * LROW + bq * 4, RB); \
    } while (0)

    const int nk = a.Kp / BK;
    BEV_GLOAD(va0, rb0);
    if (nk > 1) BEV_GLOAD(va1, rb1);
    BEV_SWRITE(0, va0, rb0);
    __syncthreads();
    const int r32 = lane & 31, h = lane >> 5;
    // MFMAs of one K step from LDS buffer BUF.  MFMA k-slot h of step p reads k = 16 h + p
    // (p = 0..15): per half of the step each lane reads two contiguous float4 of its row per tile.
#define BEV_MFMA_STEP(BUF)                                                                           \
    do {                                                                                             \
        const float *As = lds + (NBUF == 2 ? (BUF) : 0) * STAGE;                                     \
        const float *Bs = As + BM * LROW;                                                            \
        _Pragma("unroll") for (int half = 0; half < 2; ++half) {                                     \
            f32x4 fa[TM][2], fb[TN][2];                                                              \
            _Pragma("unroll") for (int i = 0; i < TM; ++i) {                                         \
                const float *pa = As + (wm * TM * 32 + i * 32 + r32) * LROW + h * 16 + half * 8;     \
                fa[i][0] = *(const f32x4 *)pa;                                                       \
                fa[i][1] = *(const f32x4 *)(pa + 4);                                                 \
            }                                                                                        \
            _Pragma("unroll") for (int j = 0; j < TN; ++j) {                                         \
                const float *pb = Bs + (wn * TN * 32 + j * 32 + r32) * LROW + h * 16 + half * 8;     \
                fb[j][0] = *(const f32x4 *)pb;                                                       \
                fb[j][1] = *(const f32x4 *)(pb + 4);                                                 \
            }                                                                                        \
            _Pragma("unroll") for (int p = 0; p < 8; ++p) {                                          \
                _Pragma("unroll") for (int i = 0; i < TM; ++i) {                                     \
                    const float av = fa[i][p >> 2][p & 3];                                           \
                    _Pragma("unroll") for (int j = 0; j < TN; ++j) {                                 \
                        const float bv = fb[j][p >> 2][p & 3];                                       \
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[i][j], 0, 0, 0); \
                    }                                                                                \
                }                                                                                    \
            }                                                                                        \
        }                                                                                            \
    } while (0)
    // Two K steps per trip with the register sets in ping-pong (no copies), so the loads of step
    // ks + 2 stay in flight across step ks + 1 and are waited for only when written to LDS.  The
    // loop body issues its loads unconditionally (the last steps are peeled off below): with no
    // path that skips a load, hipcc's waitcnt pass keeps the counted vmcnt for the older set.
#define BEV_SYNC_WRITE(BUF, VA, RB)                                      \
    do {                                                                 \
        if (NBUF == 1) __syncthreads(); /* single buffer: reads done */ \
        BEV_SWRITE(BUF, VA, RB);                                         \
        __syncthreads();                                                 \
    } while (0)
    int ks = 0;
    for (; ks + 3 < nk; ks += 2) {
        BEV_GLOAD(va0, rb0);  // step ks + 2 -> set 0
        BEV_MFMA_STEP(0);
        BEV_SYNC_WRITE(1, va1, rb1);  // step ks + 1
        BEV_GLOAD(va1, rb1);  // step ks + 3 -> set 1
        BEV_MFMA_STEP(1);
        BEV_SYNC_WRITE(0, va0, rb0);  // step ks + 2
    }
    // 1, 2 or 3 steps left (set 1 holds step ks + 1 when it exists)
    if (ks + 2 < nk) {
        BEV_GLOAD(va0, rb0);  // step ks + 2
        BEV_MFMA_STEP(0);
        BEV_SYNC_WRITE(1, va1, rb1);
        BEV_MFMA_STEP(1);
        BEV_SYNC_WRITE(0, va0, rb0);
        BEV_MFMA_STEP(0);
    } else if (ks + 1 < nk) {
        BEV_MFMA_STEP(0);
        BEV_SYNC_WRITE(1, va1, rb1);
        BEV_MFMA_STEP(1);
    } else {
        BEV_MFMA_STEP(0);
    }
#undef BEV_SYNC_WRITE
#undef BEV_MFMA_STEP
#undef BEV_GLOAD
#undef BEV_SWRITE
    if constexpr (CHAIN == 1) {
        static_assert(WM * 32 * (WN * TN * 32 + 4) <= LDSF, "chain epilogue: h tile must fit the LDS");
        chain_epilogue<WM, WN, TM, TN>(a, lds, acc, wm, wn, lane, m0);
        return;
    }

    conv_epilogue<TM, TN>(a, lds, acc, wave, lane, wm, wn, m0, n0);
}

// ---------------------------------------------------------------------------
// LDS-DMA operand path (NHWC, Ci % 32 == 0: the fast loader's layers): k_conv_dma
// ---------------------------------------------------------------------------
// Same tiles, MFMA order (bit-identical results) and epilogues as k_conv<.., LOADER 1, ..>; the K-step
// operands go global -> LDS by global_load_lds_dwordx4 instead of through registers: no staging VGPRs,
// no ds_write, double-buffered, one barrier per K step.  One DMA instruction moves 8 rows x 32 k
// (1 KiB) and writes lane l's 16 B at slot l, so rows are 128 B with no padding; the 16-B chunk c of
// row r is stored at chunk c ^ ((r >> 1) & 7) (each lane fetches the logical chunk its slot holds),
// which makes the fragment reads conflict-free: every 16-lane ds_read_b128 group covers 8 even and
// 8 odd rows whose swizzles are all distinct.  Out-of-range taps and rows read a zero quad.
__device__ __forceinline__ unsigned lds_base(const unsigned char *p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) unsigned char *)p;
}

__device__ __forceinline__ void lds_dma16(const float *src, unsigned dst_any) {
    const unsigned dst = (unsigned)__builtin_amdgcn_readfirstlane((int)dst_any);  // wave-uniform LDS address
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(dst)
        : "memory");
}

template <int WM, int WN, int TM, int TN, int CHAIN>
__global__ __launch_bounds__(256, (TM * TN > 2) ? 2 : 3) void k_conv_dma(ConvArgs a) {
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
    constexpr int STAGE = (BM + BN) * 32;  // floats per stage
    constexpr int EPI = 4 * (TM * 32) * (TN * 32 + 4);
    constexpr int CHT = CHAIN ? WM * 32 * (WN * TN * 32 + 4) : 0;
    constexpr int L0 = 2 * STAGE > EPI ? 2 * STAGE : EPI;
    constexpr int LDSF = CHT > L0 ? CHT : L0;
    constexpr int NA = BM / 8, NB = BN / 8;  // DMA instructions (1 KiB) per stage for A and B
    constexpr int QA = NA / 4, QB = NB / 4;  // per wave
    static_assert(NA % 4 == 0 && NB % 4 == 0, "whole DMA instructions per wave");
    __shared__ __attribute__((aligned(16))) float lds[LDSF];

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int n_tiles = (a.Co + BN - 1) / BN;
    unsigned bid = blockIdx.x;
    if (a.xcd) {
        const unsigned nb = gridDim.x, q = nb / 8, r = nb % 8, x = bid % 8;
        bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
    }
    const int64_t m0 = (int64_t)(bid / n_tiles) * BM;
    const int n0 = (bid % n_tiles) * BN;

    // this lane's DMA slots: instruction i = wave + 4 q, row 8 i + lane / 8 (of the A or the B tile),
    // logical chunk (lane & 7) ^ ((row >> 1) & 7)
    const int rsub = lane >> 3;
    int64_t abase[QA];  // element offset of (image, iy0, ix0) + chunk, valid only with the tap in range
    int aiy[QA], aix[QA];
    bool aok[QA];
#pragma unroll
    for (int q = 0; q < QA; ++q) {
        const int row = 8 * (wave + 4 * q) + rsub;
        const int c = (lane & 7) ^ ((row >> 1) & 7);
        const int64_t m = m0 + row;
        aok[q] = m < a.M;
        const int64_t mm = aok[q] ? m : 0;
        const int ox = (int)(mm % a.Wo);
        const int64_t t = mm / a.Wo;
        const int oy = (int)(t % a.Ho);
        const int64_t n = t / a.Ho;
        aiy[q] = oy * a.stride - a.pad;
        aix[q] = ox * a.stride - a.pad;
        abase[q] = ((n * a.H + aiy[q]) * a.W + aix[q]) * a.Ci + 4 * c;
    }
    const float *bsrc[QB];
#pragma unroll
    for (int q = 0; q < QB; ++q) {
        const int row = 8 * (wave + 4 * q) + rsub;
        const int c = (lane & 7) ^ ((row >> 1) & 7);
        bsrc[q] = a.wp + (int64_t)(n0 + row) * a.Kp + 4 * c;
    }
    const unsigned lbase = (unsigned)__builtin_amdgcn_readfirstlane((int)lds_base((const unsigned char *)lds));
    int ky = 0, kx = 0, ci0 = 0, kb = 0;
    auto issue = [&](int buf) {
        const unsigned d0 = lbase + (unsigned)(buf * STAGE * 4);
        const int64_t toff = ((int64_t)ky * a.W + kx) * a.Ci + ci0;
#pragma unroll
        for (int q = 0; q < QA; ++q) {
            const int iy = aiy[q] + ky, ix = aix[q] + kx;
            const bool in = aok[q] && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
            lds_dma16(in ? a.x + abase[q] + toff : g_zero4, d0 + (unsigned)((wave + 4 * q) * 1024));
        }
#pragma unroll
        for (int q = 0; q < QB; ++q)
            lds_dma16(bsrc[q] + kb, d0 + (unsigned)((NA + wave + 4 * q) * 1024));
        kb += BK;
        ci0 += BK;
        if (ci0 == a.Ci) {
            ci0 = 0;
            if (++kx == a.KW) {
                kx = 0;
                ++ky;
            }
        }
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){0};
    const int r32 = lane & 31, h = lane >> 5, sw = (r32 >> 1) & 7;
    // fragment chunk offsets (floats) of half 0 / 1: logical chunks 4 h + 2 half + {0, 1}
    const int f00 = ((4 * h) ^ sw) * 4, f01 = ((4 * h + 1) ^ sw) * 4;
    const int f10 = ((4 * h + 2) ^ sw) * 4, f11 = ((4 * h + 3) ^ sw) * 4;

    const int nk = a.Kp / BK;
    issue(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int ks = 0; ks < nk; ++ks) {
        const int cur = ks & 1;
        if (ks + 1 < nk) issue(cur ^ 1);
        const float *As = lds + cur * STAGE;
        const float *Bs = As + BM * 32;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            const int o0 = half ? f10 : f00, o1 = half ? f11 : f01;
            f32x4 fa[TM][2], fb[TN][2];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const float *pa = As + (wm * TM * 32 + i * 32 + r32) * 32;
                fa[i][0] = *(const f32x4 *)(pa + o0);
                fa[i][1] = *(const f32x4 *)(pa + o1);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const float *pb = Bs + (wn * TN * 32 + j * 32 + r32) * 32;
                fb[j][0] = *(const f32x4 *)(pb + o0);
                fb[j][1] = *(const f32x4 *)(pb + o1);
            }
#pragma unroll
            for (int p = 0; p < 8; ++p) {
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const float av = fa[i][p >> 2][p & 3];
#pragma unroll
                    for (int j = 0; j < TN; ++j) {
                        const float bv = fb[j][p >> 2][p & 3];
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[i][j], 0, 0, 0);
                    }
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of step ks + 1 landed
        __syncthreads();                                   // all of it; buffer cur is free again
    }
    if constexpr (CHAIN == 1) {
        chain_epilogue<WM, WN, TM, TN>(a, lds, acc, wm, wn, lane, m0);
        return;
    }
    conv_epilogue<TM, TN>(a, lds, acc, wave, lane, wm, wn, m0, n0);
}

// ---------------------------------------------------------------------------
// ResNet stem: 7x7 / stride 2 / pad 3 over Ci = 3 NCHW images, Co <= 64
// ---------------------------------------------------------------------------
// timm conv1 (cnn_encoder.py:26 backbone; first layer of CNNEncoder._encode_single).
// Persistent workgroups; one output tile = 4 rows x 64 columns x Co channels, wave w owns
// output row w (2 x 2 MFMA tiles of 32 pixels x 32 channels, 64 accumulators).  The tile's
// input patch (3 ch x 13 rows x 133 cols) is read once with coalesced row loads and kept in
// LDS as even / odd column planes: with stride 2, tap kx of output column ox reads column
// 2 ox + kx, i.e. plane (kx & 1) at index ox + kx / 2, so every A operand is a conflict-free
// ds_read_b32 at a per-(tap, k-slot) constant offset.  The 147 taps t = (ci * 7 + ky) * 7 + kx
// are packed densely into 74 MFMA k-pairs (k-slot h of pair q is tap 2 q + h; the one padding
// slot has zero weight), 12 % fewer MFMAs than pairing (kx, kx + 1) within a row.  The next
// tile's patch is fetched into registers during the MFMAs and written to the single LDS patch
// buffer between two barriers, so weights (39 KiB) + patch (24 KiB) leave room for two
// workgroups per CU.  Weights are re-laid out into LDS once per workgroup from the packed panel.
namespace stem {
constexpr int TW = 64, TH = 4;
constexpr int PR = 2 * TH + 5;                     // 13 input rows
constexpr int PC = 2 * TW + 5;                     // 133 input columns
constexpr int PP = 80;                             // plane pitch: 67 used; = 16 mod 32 -> conflict-free stores
constexpr int RP = 2 * PP, CP = PR * RP, PATCH = 3 * CP;
constexpr int NT = 147;                            // taps
constexpr int NQ = (NT + 1) / 2;                   // 74 k pairs
constexpr int NQP = 76;                            // per-k-slot weight run (multiple of 4)
constexpr int WP = 2 * NQP + 4;                    // weight row pitch (156 floats = 39 odd 16-B slots)
constexpr int NE = 3 * PR * PC;                    // patch elements
constexpr int PER_T = (NE + 255) / 256;            // per thread (21)
// LDS offset of tap t relative to (output row 0, output column 0) of the patch
__host__ __device__ constexpr int tap_off(int t) {
    return (t / 49) * CP + ((t % 49) / 7) * RP + ((t % 7) & 1) * PP + ((t % 7) >> 1);
}
}  // namespace stem

struct StemArgs {
    const float *__restrict__ x;
    const float *__restrict__ wp;
    const float *__restrict__ bias;
    float *__restrict__ y;
    int N, H, W, Kp, Co, Ho, Wo, relu, nTx, nTy;
    int64_t ntiles;
};

__device__ __forceinline__ void stem_fetch(const StemArgs &a, int64_t t, int tid, float (&pv)[stem::PER_T]) {
    using namespace stem;
    const int tx = (int)(t % a.nTx);
    const int64_t r_ = t / a.nTx;
    const int ty = (int)(r_ % a.nTy);
    const int64_t img = r_ / a.nTy;
    const int row0 = 2 * ty * TH - 3, col0 = 2 * tx * TW - 3;
    const float *xi = a.x + img * 3 * (int64_t)a.H * a.W;
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
        const int e = tid + 256 * i;
        const int cr = e / PC, c = e - cr * PC;
        const int ci = cr / PR, r = cr - ci * PR;
        const int gy = row0 + r, gx = col0 + c;
        const bool in = e < NE && gy >= 0 && gy < a.H && gx >= 0 && gx < a.W;
        // unconditional load through a selected pointer (no branch around the load)
        pv[i] = *(in ? xi + ((int64_t)ci * a.H + gy) * a.W + gx : (const float *)g_zero4);
    }
}

__device__ __forceinline__ void stem_put(float *pl, int tid, const float (&pv)[stem::PER_T]) {
    using namespace stem;
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
        const int e = tid + 256 * i;
        if (e < NE) {
            const int cr = e / PC, c = e - cr * PC;
            const int ci = cr / PR, r = cr - ci * PR;
            pl[ci * CP + r * RP + (c & 1) * PP + (c >> 1)] = pv[i];
        }
    }
}

__global__ __launch_bounds__(256, 2) void k_stem(StemArgs a) {
    using namespace stem;
    __shared__ __attribute__((aligned(16))) float lds[64 * WP + PATCH];
    float *wl = lds, *pl = lds + 64 * WP;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r32 = lane & 31;

    // weights: wl[n][h * NQP + q] = W[n][tap 2 q + h]; packed k = (ky * 7 + kx) * 3 + ci
    for (int e = tid; e < 64 * 2 * NQP; e += 256) {
        const int n = e / (2 * NQP), hq = e - n * (2 * NQP), hh = hq / NQP, q = hq - hh * NQP;
        const int tp = 2 * q + hh;
        float v = 0.0f;
        if (n < a.Co && tp < NT) {
            const int ci = tp / 49, ky = (tp % 49) / 7, kx = tp % 7;
            v = a.wp[(int64_t)n * a.Kp + (ky * 7 + kx) * 3 + ci];
        }
        wl[n * WP + hq] = v;
    }
    float pv[PER_T];
    int64_t t = blockIdx.x;
    stem_fetch(a, t < a.ntiles ? t : 0, tid, pv);
    stem_put(pl, tid, pv);
    __syncthreads();

    const float *P = pl + wave * 2 * RP + r32;  // output row `wave`, column r32 (+ 32 for the second M tile)
    const float *wb0 = wl + r32 * WP + h * NQP, *wb1 = wl + (32 + r32) * WP + h * NQP;
    const float b0 = (r32 < a.Co) ? a.bias[r32] : 0.0f;
    const float b1 = (32 + r32 < a.Co) ? a.bias[32 + r32] : 0.0f;
    for (; t < a.ntiles; t += gridDim.x) {
        const int64_t tn = t + gridDim.x;
        stem_fetch(a, tn < a.ntiles ? tn : t, tid, pv);  // in flight during the MFMAs
        f32x16 acc00 = (f32x16){0}, acc01 = (f32x16){0}, acc10 = (f32x16){0}, acc11 = (f32x16){0};
        int hv = h;
        asm volatile("" : "+v"(hv));  // per-tile opaque: the 74 per-pair lane offsets are not hoisted into VGPRs
#pragma unroll
        for (int q4 = 0; q4 < NQ; q4 += 4) {
            const f32x4 w0 = *(const f32x4 *)(wb0 + q4), w1 = *(const f32x4 *)(wb1 + q4);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int q = q4 + u;
                if (q >= NQ) break;
                // k-slot h reads tap 2 q + h (the padding slot 147 re-reads tap 146 with zero weight)
                const int o0 = tap_off(2 * q), o1 = tap_off(2 * q + 1 < NT ? 2 * q + 1 : NT - 1);
                const float *pa = P + (hv ? o1 - o0 : 0);  // k-slot 1 lanes: the odd tap
                const float av0 = pa[o0], av1 = pa[o0 + 32];
                acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(av0, w0[u], acc00, 0, 0, 0);
                acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(av0, w1[u], acc01, 0, 0, 0);
                acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(av1, w0[u], acc10, 0, 0, 0);
                acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(av1, w1[u], acc11, 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);  // bound the operand reads in flight (VGPR budget of 2 waves / SIMD)
        }
        // epilogue: D[row][col], col = channel r32 (+32), row = pixel (r & 3) + 8 (r >> 2) + 4 h (+32)
        {
            const int tx = (int)(t % a.nTx);
            const int64_t r_ = t / a.nTx;
            const int ty = (int)(r_ % a.nTy);
            const int64_t img = r_ / a.nTy;
            const int oy = ty * TH + wave;
            const int oxb = tx * TW;
            if (oy < a.Ho) {
                float *yr = a.y + ((img * a.Ho + oy) * (int64_t)a.Wo) * a.Co;
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) {
                    const f32x16 &c0 = mt ? acc10 : acc00;
                    const f32x16 &c1 = mt ? acc11 : acc01;
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int ox = oxb + 32 * mt + (r & 3) + 8 * (r >> 2) + 4 * h;
                        if (ox < a.Wo) {
                            float v0 = c0[r] + b0, v1 = c1[r] + b1;
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
        }
        __syncthreads();  // every wave is done reading the patch
        stem_put(pl, tid, pv);
        __syncthreads();
    }
}

int g_num_cu = 0;

int launch_stem(const float *x, int N, int H, int W, const float *packed, int Kp, const float *bias, int Co,
                float *y, int Ho, int Wo, int relu, hipStream_t st) {
    if (g_num_cu == 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                    hipSuccess || n <= 0)
            n = 256;
        g_num_cu = n;
    }
    StemArgs a;
    a.x = x;
    a.wp = packed;
    a.bias = bias;
    a.y = y;
    a.N = N;
    a.H = H;
    a.W = W;
    a.Kp = Kp;
    a.Co = Co;
    a.Ho = Ho;
    a.Wo = Wo;
    a.relu = relu;
    a.nTx = (Wo + stem::TW - 1) / stem::TW;
    a.nTy = (Ho + stem::TH - 1) / stem::TH;
    a.ntiles = (int64_t)N * a.nTx * a.nTy;
    const int64_t grid = a.ntiles < 2 * (int64_t)g_num_cu ? a.ntiles : 2 * (int64_t)g_num_cu;
    hipLaunchKernelGGL(k_stem, dim3((unsigned)grid), dim3(256), 0, st, a);
    return (int)hipGetLastError();
}

// NHWC max-pool (padding counts as -inf, as torch.nn.MaxPool2d); one float4
// of channels per thread when C % 4 == 0.
template <bool VEC>
__global__ void k_maxpool(const float *__restrict__ x, int N, int H, int W, int C, int k, int s, int p,
                          float *__restrict__ y, int Ho, int Wo) {
    const int CV = VEC ? C / 4 : C;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)N * Ho * Wo * CV;
    if (t >= total) return;
    const int c = (int)(t % CV);
    int64_t r = t / CV;
    const int ox = (int)(r % Wo);
    r /= Wo;
    const int oy = (int)(r % Ho);
    const int n = (int)(r / Ho);
    const float ninf = -__builtin_inff();
    float m[4] = {ninf, ninf, ninf, ninf};
    for (int ky = 0; ky < k; ++ky) {
        const int iy = oy * s - p + ky;
        if (iy < 0 || iy >= H) continue;
        for (int kx = 0; kx < k; ++kx) {
            const int ix = ox * s - p + kx;
            if (ix < 0 || ix >= W) continue;
            const int64_t base = (((int64_t)n * H + iy) * W + ix) * C;
            if (VEC) {
                const float4 v = *(const float4 *)(x + base + 4 * c);
                const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int u = 0; u < 4; ++u) m[u] = (vv[u] > m[u] || vv[u] != vv[u]) ? vv[u] : m[u];
            } else {
                const float v = x[base + c];
                m[0] = (v > m[0] || v != v) ? v : m[0];
            }
        }
    }
    if (VEC) *(float4 *)(y + t * 4) = make_float4(m[0], m[1], m[2], m[3]);
    else y[t] = m[0];
}

// 32x32 tiled transposes between [N][C][HW] and [N][HW][C]
__global__ void k_transpose(const float *__restrict__ x, int R, int S, float *__restrict__ y) {
    // x [N][R][S] -> y [N][S][R]
    __shared__ float tile[32][33];
    const int n = blockIdx.z;
    const int s0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
    const float *xn = x + (int64_t)n * R * S;
    float *yn = y + (int64_t)n * R * S;
    for (int q = threadIdx.y; q < 32; q += 8) {
        const int r = r0 + q, s = s0 + threadIdx.x;
        if (r < R && s < S) tile[q][threadIdx.x] = xn[(int64_t)r * S + s];
    }
    __syncthreads();
    for (int q = threadIdx.y; q < 32; q += 8) {
        const int s = s0 + q, r = r0 + threadIdx.x;
        if (r < R && s < S) yn[(int64_t)s * R + r] = tile[threadIdx.x][q];
    }
}

inline int last() { return (int)hipGetLastError(); }

// BEV_TUNE_CONV_DMA: fast-loader layers stage their operands by LDS-DMA (k_conv_dma).  1 = on the 64-column
// tiles only: r02l A/B over the ResNet-50 layers (7 x 1080p), LDS-DMA vs register staging: 128 x 64 and 64 x 64
// tiles (layer1) -1..-4 %, 64 x 128 tiles (layer2) +1..+3 %.  2 = every tile, 0 = none.
int g_conv_dma = 1;
inline bool use_dma(int bn) { return g_conv_dma == 2 || (g_conv_dma == 1 && bn == 64); }

template <int WM, int WN, int TM, int TN, int NBUF = 2>
int launch_conv(const ConvArgs &a, int loader, hipStream_t st) {
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
    const int64_t m_tiles = (a.M + BM - 1) / BM;
    const int n_tiles = (a.Co + BN - 1) / BN;
    const int64_t blocks = m_tiles * n_tiles;
    if (blocks > 0x7fffffff) return BEV_ERR_ARGS;
    const dim3 g((unsigned)blocks), b(256);
    if (loader == 1 && use_dma(BN)) hipLaunchKernelGGL((k_conv_dma<WM, WN, TM, TN, 0>), g, b, 0, st, a);
    else if (loader == 1) hipLaunchKernelGGL((k_conv<WM, WN, TM, TN, 1, NBUF>), g, b, 0, st, a);
    else if (loader == 2) hipLaunchKernelGGL((k_conv<WM, WN, TM, TN, 2, NBUF>), g, b, 0, st, a);
    else if (loader == 3) hipLaunchKernelGGL((k_conv<WM, WN, TM, TN, 3, NBUF>), g, b, 0, st, a);
    else if (loader == 4) hipLaunchKernelGGL((k_conv<WM, WN, TM, TN, 4, NBUF>), g, b, 0, st, a);
    else if (loader == 5) hipLaunchKernelGGL((k_conv<WM, WN, TM, TN, 5, NBUF>), g, b, 0, st, a);
    else if (loader == 6) hipLaunchKernelGGL((k_conv<WM, WN, TM, TN, 6, NBUF>), g, b, 0, st, a);
    else hipLaunchKernelGGL((k_conv<WM, WN, TM, TN, 0, NBUF>), g, b, 0, st, a);
    return last();
}

// ---------------------------------------------------------------------------
// Narrow pointwise convs (1x1, Co <= 48: the EfficientNet projections to 24 / 32 / 40 / 48 channels, up to
// 518 400 pixels per image): an MFMA tile is >= 64 columns wide, so 33-62 % of its work is padding and the K loop
// (Ci = 24 .. 288) is one to nine steps -- these layers ran at 1/3 of the HBM rate.  One thread per output pixel
// computes its Co outputs on the VALU from the pixel's Ci inputs (two float4 loads per 8 channels, the
// per-(image, channel) SE gate applied to them as in the MFMA loaders).  The weights are wave-uniform, so they come
// through the scalar cache into SGPRs (s_load of 8 consecutive k of one output channel, read straight from the
// fp32 panel [Co][Kp]) and feed packed FMAs: acc[co] = {sum over even k, sum over odd k} on v_pk_fma_f32, added at
// the end.  Epilogue bias, residual, activation as conv_epilogue.  HBM-bound: (Ci + Co (+ Co)) floats per pixel.
// Measured (profiles/r03h_pw_small_ab.txt, EfficientNet-B3 bench): 107.9 frames/s against 121.9 on the MFMA
// tiles -- the per-lane rows (stride Ci floats) thrash the L1 and every 8 k the wave waits on the scalar cache
// (55 KB of weights for 288 -> 48 does not fit it), so the layers stay on the MFMA tiles (BEV_TUNE_CONV_PW_SMALL
// 0) or k_pw_mfma below (2, default; 3; 4); 1 selects this kernel.
int g_conv_pw_small = 2;

template <int CO>
__global__ __launch_bounds__(256) void k_pw_small(ConvArgs a) {
    const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (m >= a.M) return;
    const int Ci = a.Ci, Kp = a.Kp;
    const float *xp = a.x + m * Ci;
    const float *gp = a.ascale ? a.ascale + (m / ((int64_t)a.Ho * a.Wo)) * Ci : nullptr;
    const float *__restrict__ wp = a.wp;
    f32x2 acc[CO];
#pragma unroll
    for (int co = 0; co < CO; ++co) acc[co] = (f32x2){0.f, 0.f};
    f32x4 x0 = *(const f32x4 *)xp, x1 = *(const f32x4 *)(xp + 4);
    for (int c0 = 0; c0 < Ci; c0 += 8) {
        f32x4 u0 = x0, u1 = x1;
        if (c0 + 8 < Ci) {  // next 8 channels in flight during these FMAs
            x0 = *(const f32x4 *)(xp + c0 + 8);
            x1 = *(const f32x4 *)(xp + c0 + 12);
        }
        if (gp) {
            u0 *= *(const f32x4 *)(gp + c0);
            u1 *= *(const f32x4 *)(gp + c0 + 4);
        }
        const f32x2 xa = {u0[0], u0[1]}, xb = {u0[2], u0[3]}, xc = {u1[0], u1[1]}, xd = {u1[2], u1[3]};
#pragma unroll
        for (int co = 0; co < CO; ++co) {
            const float *w = wp + co * Kp + c0;  // wave-uniform: scalar loads
            acc[co] = __builtin_elementwise_fma(xa, (f32x2){w[0], w[1]}, acc[co]);
            acc[co] = __builtin_elementwise_fma(xb, (f32x2){w[2], w[3]}, acc[co]);
            acc[co] = __builtin_elementwise_fma(xc, (f32x2){w[4], w[5]}, acc[co]);
            acc[co] = __builtin_elementwise_fma(xd, (f32x2){w[6], w[7]}, acc[co]);
        }
    }
    float *yp = a.y + m * a.ldy;
    const float *rp = a.res ? a.res + m * a.Co : nullptr;
#pragma unroll
    for (int q = 0; q < CO / 4; ++q) {
        f32x4 o = {acc[4 * q][0] + acc[4 * q][1], acc[4 * q + 1][0] + acc[4 * q + 1][1],
                   acc[4 * q + 2][0] + acc[4 * q + 2][1], acc[4 * q + 3][0] + acc[4 * q + 3][1]};
        if (a.bias) o += *(const f32x4 *)(a.bias + 4 * q);
        if (rp) o += *(const f32x4 *)(rp + 4 * q);
        if (a.relu) {
#pragma unroll
            for (int u = 0; u < 4; ++u) o[u] = act_fn(o[u], a.relu);
        }
        *(f32x4 *)(yp + 4 * q) = o;
    }
}

// Wave-streaming 1x1 conv for tiny K (Ci in {24, 32, 40, 48}: EfficientNet's 24 -> 144 expansion and 40 / 24 -> 24
// projections at 540 x 960), BEV_TUNE_CONV_PW_SMALL = 2.  The tiled kernels spend one K step per tile between an
// operand load and an epilogue (nothing to overlap: 0.3 of HBM).  Here every wave owns 32 pixels and is independent
// (no LDS, no barrier): lane (i = pixel, h = k half) loads its pixel's k in [h K/2, (h + 1) K/2) straight into
// registers (float4 pieces of one contiguous row) and the matching weight row piece of output channel i of each
// 32-channel block, so MFMA k-slot h of step s multiplies x[m][h K/2 + s] by W[co][h K/2 + s] -- a permutation
// of the k order (fp32-tolerance equal to the tiles); D[(r & 3) + 8 (r >> 2) + 4 h][lane & 31] gets bias,
// residual, activation and is stored 32 channels (128 B) per half-wave.

template <int KH2>
__device__ __forceinline__ void pw_load_b(const ConvArgs &a, int co, int h, float (&bv)[KH2]) {
    const float *wr = a.wp + (int64_t)co * a.Kp + h * KH2;  // panel rows are zero-padded to 128
#pragma unroll
    for (int u = 0; u < KH2 / 4; ++u) {
        const f32x4 v = *(const f32x4 *)(wr + 4 * u);
#pragma unroll
        for (int e = 0; e < 4; ++e) bv[4 * u + e] = v[e];
    }
}

__device__ __forceinline__ void pw_store(const ConvArgs &a, const f32x16 &acc, int64_t mw, int h, int co) {
    if (co >= a.Co) return;
    const float b = a.bias ? a.bias[co] : 0.f;
    float rv[16];  // every residual load issued before the first store (the compiler cannot reorder them past it)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t mo = mw + (r & 3) + 8 * (r >> 2) + 4 * h;
        rv[r] = (a.res && mo < a.M) ? a.res[mo * a.Co + co] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t mo = mw + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (mo >= a.M) continue;
        float o = acc[r] + b;
        if (a.res) o += rv[r];
        if (a.relu) o = act_fn(o, a.relu);
        a.y[mo * a.ldy + co] = o;
    }
}

// Vector epilogue (Co % 4 == 0, 16-B aligned y / res / bias, ldy % 4 == 0): the 32 x 32 block goes through a
// wave-private LDS tile and leaves as float4 rows -- 4 store instructions per block instead of 16 dword ones.
__device__ __forceinline__ void pw_store_v(const ConvArgs &a, const f32x16 &acc, int64_t mw, int lane, int nb,
                                           float *E) {
    constexpr int ER = 36;  // row stride (floats): float4 reads of 8 lanes per row spread over the banks
    const int h = lane >> 5, c = lane & 31;
#pragma unroll
    for (int r = 0; r < 16; ++r) E[((r & 3) + 8 * (r >> 2) + 4 * h) * ER + c] = acc[r];
    const int c4 = lane & 7, co = nb * 32 + 4 * c4;
    if (co >= a.Co) return;
    const f32x4 b = a.bias ? *(const f32x4 *)(a.bias + co) : (f32x4){0.f, 0.f, 0.f, 0.f};
    f32x4 rv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t mo = mw + (lane >> 3) + 8 * q;
        rv[q] = (a.res && mo < a.M) ? *(const f32x4 *)(a.res + mo * a.Co + co) : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int pr = (lane >> 3) + 8 * q;
        const int64_t mo = mw + pr;
        if (mo >= a.M) continue;
        f32x4 o = *(const f32x4 *)(E + pr * ER + 4 * c4) + b;
        if (a.res) o += rv[q];
        if (a.relu) {
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = act_fn(o[e], a.relu);
        }
        *(f32x4 *)(a.y + mo * a.ldy + co) = o;
    }
}

// NP output blocks of 32 channels per pass: NP independent MFMA chains interleaved (NP = 1 launched: see below)
template <int KH2, int NP>
__global__ __launch_bounds__(256) void k_pw_mfma(ConvArgs a) {
    __shared__ __attribute__((aligned(16))) float epi[4][32 * 36];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, i = lane & 31, h = lane >> 5;
    const bool vec = a.pwvec != 0;
    const int64_t mw = ((int64_t)blockIdx.x * 4 + wave) * 32;  // the wave's first pixel
    if (mw >= a.M) return;
    const int64_t m = mw + i < a.M ? mw + i : a.M - 1;
    const int Ci = a.Ci;
    float av[KH2];
    {
        const float *xp = a.x + m * Ci + h * KH2;
        const float *gp = a.ascale ? a.ascale + (m / ((int64_t)a.Ho * a.Wo)) * Ci + h * KH2 : nullptr;
#pragma unroll
        for (int u = 0; u < KH2 / 4; ++u) {
            f32x4 v = *(const f32x4 *)(xp + 4 * u);
            if (gp) v *= *(const f32x4 *)(gp + 4 * u);
#pragma unroll
            for (int e = 0; e < 4; ++e) av[4 * u + e] = v[e];
        }
    }
    const int nbt = (a.Co + 31) / 32;
    for (int nb = 0; nb < nbt; nb += NP) {
        float bv[NP][KH2];
        f32x16 acc[NP];
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            pw_load_b<KH2>(a, (nb + p) * 32 + i, h, bv[p]);  // rows past Co: zero padding (< copad)
            acc[p] = (f32x16){};
        }
#pragma unroll
        for (int st = 0; st < KH2; ++st)
#pragma unroll
            for (int p = 0; p < NP; ++p) acc[p] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[st], bv[p][st], acc[p], 0, 0, 0);
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            if (vec) pw_store_v(a, acc[p], mw, lane, nb + p, epi[wave]);
            else pw_store(a, acc[p], mw, h, (nb + p) * 32 + i);
        }
    }
}

// BEV_TUNE_CONV_PW_SMALL: 2 (default) = narrow outputs (Co <= 32) only, 3 = every tiny-K 1x1 layer, 4 = narrow only
// with the dword epilogue.  3 is faster for inference but not the default: its k order on the wide expansions
// moves one EfficientNet-B0 training gradient (test_effnet_trunk_backward_vs_torch_autograd, blocks.0.0.bn2.bias)
// to 1.007e-3 relative against float64 autograd, past the test's 1e-3 bound (r03q); the default path's worst in that
// test is 5.74e-4 (b0, batch statistics: blocks.0.0.bn2.bias; b3 5.06e-4; frozen BN ~1e-6; gpurun_out r04t, round 4).  r03p micro (profiles/r03p_pw_mfma_vec_ab.txt, 7 x 1080p, us; tiles -> dword epilogue ->
// float4 epilogue): 40 -> 24 420 -> 344 -> 270, 24 -> 24 + residual 337 -> 294 -> 223, 24 -> 144 927 -> (921) -> 747,
// 32 -> 192 287 -> 242.  (r03j: with the dword epilogue the wide expansions were within +-5 % of the tiles, and each
// residual load waited behind the previous store until all 16 were issued first.)
bool try_pw_mfma(const ConvArgs &a, int loader, hipStream_t st, int &rc) {
    if (g_conv_pw_small < 2 || (g_conv_pw_small != 3 && a.Co > 32) || !(loader == 1 || loader == 4 || loader == 6) || a.KH != 1 || a.KW != 1 ||
        a.stride != 1 || a.pad != 0 || a.in_nchw || a.ashift || a.arelu || a.dil != 1 || a.Kp < a.Ci ||
        !(a.Ci == 24 || a.Ci == 32 || a.Ci == 40 || a.Ci == 48) ||
        ((((uintptr_t)a.x) | ((uintptr_t)a.wp) | ((uintptr_t)a.ascale)) & 15))
        return false;
    const int64_t blocks = (a.M + 127) / 128;
    if (blocks > 0x7fffffff) return false;
    const dim3 g((unsigned)blocks), b(256);
    ConvArgs av = a;  // float4 epilogue when the output rows allow it (knob 4: dword stores, for A/B)
    av.pwvec = g_conv_pw_small != 4 && a.Co % 4 == 0 && a.ldy % 4 == 0 &&
               ((((uintptr_t)a.y) | ((uintptr_t)a.res) | ((uintptr_t)a.bias)) & 15) == 0;
    {  // NP = 2 (two chains in flight, 188 VGPRs) measured slower on 24 -> 144: 953 -> 1230 us (r03m)
        switch (a.Ci) {
            case 24: hipLaunchKernelGGL((k_pw_mfma<12, 1>), g, b, 0, st, av); break;
            case 32: hipLaunchKernelGGL((k_pw_mfma<16, 1>), g, b, 0, st, av); break;
            case 40: hipLaunchKernelGGL((k_pw_mfma<20, 1>), g, b, 0, st, av); break;
            default: hipLaunchKernelGGL((k_pw_mfma<24, 1>), g, b, 0, st, av); break;
        }
    }
    rc = last();
    return true;
}

// the layer takes k_pw_small (true) -- launched here -- or the MFMA tiles (false)
bool try_pw_small(const ConvArgs &a, int loader, hipStream_t st, int &rc) {
    if (g_conv_pw_small != 1 || !(loader == 1 || loader == 4 || loader == 6) || a.KH != 1 || a.KW != 1 ||
        a.stride != 1 || a.pad != 0 || a.in_nchw || a.ashift || a.arelu || a.dil != 1 || a.ldy != a.Co ||
        a.Ci % 8 != 0 || a.Ci > 512 || a.Kp < a.Ci ||
        ((((uintptr_t)a.x) | ((uintptr_t)a.y) | ((uintptr_t)a.bias) | ((uintptr_t)a.res) | ((uintptr_t)a.ascale)) & 15))
        return false;
    const int64_t blocks = (a.M + 255) / 256;
    if (blocks > 0x7fffffff) return false;
    const size_t sh = 0;
    switch (a.Co) {
        case 16: hipLaunchKernelGGL(k_pw_small<16>, dim3((unsigned)blocks), dim3(256), sh, st, a); break;
        case 24: hipLaunchKernelGGL(k_pw_small<24>, dim3((unsigned)blocks), dim3(256), sh, st, a); break;
        case 32: hipLaunchKernelGGL(k_pw_small<32>, dim3((unsigned)blocks), dim3(256), sh, st, a); break;
        case 40: hipLaunchKernelGGL(k_pw_small<40>, dim3((unsigned)blocks), dim3(256), sh, st, a); break;
        case 48: hipLaunchKernelGGL(k_pw_small<48>, dim3((unsigned)blocks), dim3(256), sh, st, a); break;
        default: return false;
    }
    rc = last();
    return true;
}

int g_conv_tile = 0;

// XCD-aware block order (k_conv): on by default since the smaller r01f/r01g tiles put 2-4 N tiles
// on every A row block; A/B over ResNet-50 (r01g, same box): 3x3 layers -3..-6 %, tails -2..-4 %,
// 1x1 conv3 / proj -5 %, sum over the layers -1.6 %.  BEV_TUNE_CONV_XCD = 0 restores plain order.
int g_conv_xcd = 1;   // BEV_TUNE_CONV_XCD
int g_conv_nbuf = 0;  // BEV_TUNE_CONV_NBUF
inline int conv_xcd() { return g_conv_xcd; }

// Tile choice + launch.  Cost model (measured on MI355X, tools/conv_micro.py
// A/B): time ~ rounds of resident blocks x tile area; ties go to the larger
// tile (better operand reuse).  Candidates: 1 = 128x128 (2 blocks per CU),
// 3 = 64x128 and 2 = 128x64, both with ONE LDS staging buffer so 3 blocks
// fit per CU (r01e A/B over the ResNet-50 layers: the extra resident block
// hides more of the load / epilogue latency than the second barrier per K
// step costs -- 1x1 layers -4..-13 %, 3x3 layers -4..-7 %, bottleneck tails
// -8..-13 %).  Small-M 128x64 launches (< 2 full rounds) keep the double
// buffer.  BEV_TUNE_CONV_NBUF = 1|2 forces the staging depth of tiles 2 / 3.
int launch_tiled(const ConvArgs &a, int loader, hipStream_t st) {
    int rc_pw = 0;
    if (g_conv_tile == 0 && try_pw_small(a, loader, st, rc_pw)) return rc_pw;
    if (g_conv_tile == 0 && try_pw_mfma(a, loader, st, rc_pw)) return rc_pw;
    const int64_t M = a.M;
    const int Co = a.Co;
    const int nbuf_env = g_conv_nbuf;
    auto nbuf1_for = [&](int tile) {
        if (nbuf_env == 1 || nbuf_env == 2) return nbuf_env == 1;
        return tile == 3 || M >= 400000;
    };
    int tile = g_conv_tile;
    if (tile == 0) {
        auto cost = [&](int bm, int bn, int resident) {
            const int64_t blocks = ((M + bm - 1) / bm) * ((Co + bn - 1) / bn);
            return (double)((blocks + resident - 1) / resident) * bm * bn;
        };
        const double c1 = cost(128, 128, 512), c3 = cost(64, 128, nbuf1_for(3) ? 768 : 512),
                     c2 = cost(128, 64, nbuf1_for(2) ? 768 : 512);
        tile = 1;
        double best = c1;
        if (c3 < 0.95 * best) { tile = 3; best = c3; }
        if (c2 < 0.95 * best) { tile = 2; best = c2; }
        // Single-source 1x1 layers over NHWC (Ci % 32 == 0) are HBM-bound: the 64 x 64 tile (one
        // 32 x 32 MFMA tile per wave, ~4 resident blocks per CU) trades operand reuse for memory
        // parallelism.  r01f A/B over ResNet-50: every such layer -1..-19 % (proj 209 -> 170 us,
        // layer1 conv1 400 -> 352 us); 3x3 layers and the dual-source tails are slower with it.
        if (a.KH == 1 && a.KW == 1 && (loader == 1 || loader == 6) && M >= 200000) tile = 4;
        // The same for the contiguous-row loader (Ci % 4 == 0: EfficientNet's 24 / 40 / 144-channel inputs) when
        // the output is narrow or K is not tiny: r03i micro (profiles/r03i_b3_pointwise_tile_micro.txt, 7 x 1080p
        // B3 layers) 40 -> 24 480 -> 420 us, 24 -> 24 375 -> 338, 144 -> 32 236 -> 204, 48 -> 288 164 -> 141;
        // 24 -> 144 is slower with it (968 -> 1030) and keeps 128 x 64.
        if (a.KH == 1 && a.KW == 1 && loader == 4 && M >= 200000 && (Co <= 64 || a.Ci >= 48)) tile = 4;
    }
    if (tile == 2)
        return nbuf1_for(2) ? launch_conv<4, 1, 1, 2, 1>(a, loader, st) : launch_conv<4, 1, 1, 2>(a, loader, st);
    if (tile == 3)
        return nbuf1_for(3) ? launch_conv<2, 2, 1, 2, 1>(a, loader, st) : launch_conv<2, 2, 1, 2>(a, loader, st);
    if (tile == 4) return launch_conv<2, 2, 1, 1, 1>(a, loader, st);  // 64 x 64
    return launch_conv<2, 2, 2, 2>(a, loader, st);                 // 128 x 128 tiles
}

// Chained conv (EPI 1): one M block holds all Co channels of the first conv -- 128 x 64 tiles
// for Co = 64 (ResNet layer1), 64 x 128 for Co = 128 (layer2); one LDS staging buffer (3 blocks / CU).
int launch_chain(const ConvArgs &a, hipStream_t st) {
    const int bm = a.Co == 64 ? 128 : 64;
    const int64_t blocks = (a.M + bm - 1) / bm;
    if (blocks > 0x7fffffff) return BEV_ERR_ARGS;
    const dim3 g((unsigned)blocks), b(256);
    if (use_dma(a.Co)) {
        if (a.Co == 64) hipLaunchKernelGGL((k_conv_dma<4, 1, 1, 2, 1>), g, b, 0, st, a);
        else hipLaunchKernelGGL((k_conv_dma<2, 2, 1, 2, 1>), g, b, 0, st, a);
    } else if (a.Co == 64) hipLaunchKernelGGL((k_conv<4, 1, 1, 2, 1, 1, 1>), g, b, 0, st, a);
    else hipLaunchKernelGGL((k_conv<2, 2, 1, 2, 1, 1, 1>), g, b, 0, st, a);
    return last();
}

}  // namespace

extern "C" {

int bev_tune(int knob, int value) {
    if (knob == BEV_TUNE_CONV_TILE) {
        if (value < 0 || value > 4) return BEV_ERR_ARGS;
        const int old = g_conv_tile;
        g_conv_tile = value;
        return old;
    }
    if (knob == BEV_TUNE_CONV_DMA) {
        if (value < 0 || value > 2) return BEV_ERR_ARGS;
        const int old = g_conv_dma;
        g_conv_dma = value;
        return old;
    }
    if (knob == BEV_TUNE_CONV_XCD || knob == BEV_TUNE_CONV_NBUF) {
        int *slot = knob == BEV_TUNE_CONV_XCD ? &g_conv_xcd : &g_conv_nbuf;
        if (value < 0 || value > (knob == BEV_TUNE_CONV_XCD ? 1 : 2)) return BEV_ERR_ARGS;
        const int old = *slot;
        *slot = value;
        return old;
    }
    if (knob == BEV_TUNE_WGRAD_MFMA) return bev::train_tune(knob, value);
    if (knob == BEV_TUNE_CONV_X6_TILE || knob == BEV_TUNE_CONV_X6_KERNEL || knob == BEV_TUNE_CONV_X6_NT)
        return bev::conv_x6_tune(knob, value);
    if (knob == BEV_TUNE_CONV_H16_KERNEL) return bev::conv_h16_tune(value);
    if (knob == BEV_TUNE_DW_RUN) return bev::dw_tune(value);
    if (knob == BEV_TUNE_STEM3_STAGE) return bev::stem3_tune(value);
    if (knob == BEV_TUNE_CONV_PW_SMALL) {
        if (value < 0 || value > 4) return BEV_ERR_ARGS;
        const int old = g_conv_pw_small;
        g_conv_pw_small = value;
        return old;
    }
    return bev::warp_tune(knob, value);
}

int64_t bev_conv_packed_size(int Co, int Ci, int KH, int KW) {
    if (Co <= 0 || Ci <= 0 || KH <= 0 || KW <= 0) return 0;
    return copad(Co) * kpad(Ci * KH * KW);
}

int bev_conv_pack_weights_f32(const float *w, int Co, int Ci, int KH, int KW, float *packed, void *stream) {
    if (!w || !packed || Co <= 0 || Ci <= 0 || KH <= 0 || KW <= 0) return BEV_ERR_ARGS;
    const int64_t Kp = kpad(Ci * KH * KW), Cop = copad(Co);
    const int64_t total = Kp * Cop;
    hipLaunchKernelGGL(k_pack, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, w, Co, Ci,
                       KH, KW, Kp, Cop, packed);
    return last();
}

static int conv2d_impl(const float *x, int in_nchw, int N, int H, int W, int Ci, const float *packed,
                       const float *bias, const float *residual, int Co, int KH, int KW, int stride, int pad, int relu,
                       float *y, int Ho, int Wo, const float *ascale, void *stream, int dil, int ldy,
                       const float *ashift, int arelu);

int bev_conv2d_f32(const float *x, int in_nchw, int N, int H, int W, int Ci, const float *packed, const float *bias,
                   const float *residual, int Co, int KH, int KW, int stride, int pad, int relu, float *y, int Ho,
                   int Wo, void *stream) {
    return conv2d_impl(x, in_nchw, N, H, W, Ci, packed, bias, residual, Co, KH, KW, stride, pad, relu, y, Ho, Wo,
                       nullptr, stream, 1, Co, nullptr, 0);
}

int bev_conv2d_nhwc_ex_f32(const float *x, int N, int H, int W, int Ci, const float *in_scale, const float *in_shift,
                           int in_relu, const float *packed, const float *bias, int Co, int KH, int KW, int stride,
                           int pad, int dilation, int relu, float *y, int ldy, int Ho, int Wo, void *stream) {
    if ((in_shift || in_relu) && !in_scale) return BEV_ERR_ARGS;
    if (in_scale && (Ci % BK != 0 || ((((uintptr_t)in_scale) | ((uintptr_t)in_shift) | ((uintptr_t)x)) & 15) != 0))
        return BEV_ERR_ARGS;  // the per-channel affine is applied by the fast NHWC loader only
    return conv2d_impl(x, 0, N, H, W, Ci, packed, bias, nullptr, Co, KH, KW, stride, pad, relu, y, Ho, Wo, in_scale,
                       stream, dilation, ldy, in_shift, in_relu != 0);
}

int bev_conv2d_chscale_f32(const float *x, int N, int H, int W, int Ci, const float *gate, const float *packed,
                           const float *bias, const float *residual, int Co, int KH, int KW, int stride, int pad,
                           int relu, float *y, int Ho, int Wo, void *stream) {
    if (!gate || ((((uintptr_t)gate) | ((uintptr_t)x)) & 15) != 0 || Ci % 4 != 0) return BEV_ERR_ARGS;
    const bool fast = Ci % BK == 0;
    const bool contig = KH == 1 && KW == 1 && stride == 1 && pad == 0;
    if (!fast && !contig) return BEV_ERR_ARGS;  // only the fast / contiguous loaders apply the scale
    return conv2d_impl(x, 0, N, H, W, Ci, packed, bias, residual, Co, KH, KW, stride, pad, relu, y, Ho, Wo, gate,
                       stream, 1, Co, nullptr, 0);
}

static int conv2d_impl(const float *x, int in_nchw, int N, int H, int W, int Ci, const float *packed,
                       const float *bias, const float *residual, int Co, int KH, int KW, int stride, int pad, int relu,
                       float *y, int Ho, int Wo, const float *ascale, void *stream, int dil, int ldy,
                       const float *ashift, int arelu) {
    if (!x || !packed || !y || N < 0 || H <= 0 || W <= 0 || Ci <= 0 || Co <= 0 || KH <= 0 || KW <= 0 ||
        stride <= 0 || pad < 0 || relu < 0 || relu > 2 || dil <= 0 || ldy < Co || (residual && ldy != Co))
        return BEV_ERR_ARGS;
    if (Ho != (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1 || Wo != (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1 ||
        Ho <= 0 || Wo <= 0)
        return BEV_ERR_ARGS;
    if (N == 0) return 0;
    ConvArgs a;
    a.x = x;
    a.wp = packed;
    a.bias = bias;
    a.res = residual;
    a.y = y;
    a.N = N;
    a.H = H;
    a.W = W;
    a.Ci = Ci;
    a.Co = Co;
    a.KH = KH;
    a.KW = KW;
    a.stride = stride;
    a.pad = pad;
    a.Ho = Ho;
    a.Wo = Wo;
    a.relu = relu;
    a.M = (int64_t)N * Ho * Wo;
    a.K = Ci * KH * KW;
    a.Kp = (int)kpad(a.K);
    a.in_nchw = in_nchw;
    const bool pw = !in_nchw && KH == 1 && KW == 1 && stride == 1 && pad == 0 && Ci % 4 == 0 &&
                    ((uintptr_t)x & 15) == 0;
    int loader = (!in_nchw && Ci % BK == 0) ? 1 : (in_nchw && Ci == 3 && KH == 7 && KW == 7) ? 2 : pw ? 4 : 0;
    if (loader == 1 && (ashift || arelu || dil != 1)) loader = 5;
    else if (loader == 1 && ascale) loader = 6;
    if ((ashift || arelu) && loader != 5) return BEV_ERR_ARGS;
    a.x2 = nullptr;
    a.Ci2 = a.H2 = a.W2 = a.stride2 = 0;
    a.ascale = ascale;
    a.ashift = ashift;
    a.arelu = arelu;
    a.dil = dil;
    a.ldy = ldy;
    a.xcd = conv_xcd();
    if (in_nchw && Ci == 3 && KH == 7 && KW == 7 && stride == 2 && pad == 3 && Co <= 64 && !residual && bias &&
        g_conv_tile == 0 && relu <= 1 && !ascale && dil == 1 && ldy == Co)
        return launch_stem(x, N, H, W, packed, a.Kp, bias, Co, y, Ho, Wo, relu, (hipStream_t)stream);
    return launch_tiled(a, loader, (hipStream_t)stream);
}

int bev_conv2d_dual_f32(const float *x, int N, int Ho, int Wo, int Ci, const float *x2, int H2, int W2, int Ci2,
                        int stride2, const float *packed, const float *bias, int Co, int relu, float *y,
                        void *stream) {
    if (!x || !x2 || !packed || !y || N < 0 || Ho <= 0 || Wo <= 0 || Ci <= 0 || Ci2 <= 0 || H2 <= 0 || W2 <= 0 ||
        stride2 <= 0 || Co <= 0)
        return BEV_ERR_ARGS;
    if (Ci % BK != 0 || Ci2 % BK != 0) return BEV_ERR_ARGS;
    if (Ho != (H2 - 1) / stride2 + 1 || Wo != (W2 - 1) / stride2 + 1) return BEV_ERR_ARGS;
    if (N == 0) return 0;
    ConvArgs a;
    a.x = x;
    a.wp = packed;
    a.bias = bias;
    a.res = nullptr;
    a.y = y;
    a.N = N;
    a.H = Ho;
    a.W = Wo;
    a.Ci = Ci;
    a.Co = Co;
    a.KH = a.KW = 1;
    a.stride = 1;
    a.pad = 0;
    a.Ho = Ho;
    a.Wo = Wo;
    a.relu = relu;
    a.M = (int64_t)N * Ho * Wo;
    a.K = Ci + Ci2;
    a.Kp = (int)kpad(a.K);
    a.in_nchw = 0;
    a.x2 = x2;
    a.ascale = nullptr;
    a.ashift = nullptr;
    a.arelu = 0;
    a.dil = 1;
    a.ldy = Co;
    a.xcd = conv_xcd();
    a.Ci2 = Ci2;
    a.H2 = H2;
    a.W2 = W2;
    a.stride2 = stride2;
    return launch_tiled(a, 3, (hipStream_t)stream);
}

int bev_conv2d_chain_f32(const float *x, int N, int H, int W, int Ci, const float *packed, const float *bias, int Co,
                         int KH, int KW, int stride, int pad, int relu, const float *packed2, const float *bias2,
                         int Co2, const float *residual, int relu2, float *y, int Ho, int Wo, void *stream) {
    if (!x || !packed || !packed2 || !y || N < 0 || H <= 0 || W <= 0 || KH <= 0 || KW <= 0 || stride <= 0 ||
        pad < 0 || relu < 0 || relu > 2 || relu2 < 0 || relu2 > 2)
        return BEV_ERR_ARGS;
    if (Ci % BK != 0 || (Co != 64 && Co != 128) || Co2 <= 0 || Co2 % 128 != 0 || ((uintptr_t)x & 15) != 0 ||
        (((uintptr_t)packed | (uintptr_t)packed2) & 15) != 0)
        return BEV_ERR_ARGS;
    if (Ho != (H + 2 * pad - KH) / stride + 1 || Wo != (W + 2 * pad - KW) / stride + 1 || Ho <= 0 || Wo <= 0)
        return BEV_ERR_ARGS;
    if (N == 0) return 0;
    ConvArgs a{};
    a.x = x;
    a.wp = packed;
    a.bias = bias;
    a.res = residual;
    a.y = y;
    a.N = N;
    a.H = H;
    a.W = W;
    a.Ci = Ci;
    a.Co = Co;
    a.KH = KH;
    a.KW = KW;
    a.stride = stride;
    a.pad = pad;
    a.Ho = Ho;
    a.Wo = Wo;
    a.relu = relu;
    a.M = (int64_t)N * Ho * Wo;
    a.K = Ci * KH * KW;
    a.Kp = (int)kpad(a.K);
    a.dil = 1;
    a.ldy = Co2;
    a.xcd = conv_xcd();
    a.wp2 = packed2;
    a.bias2 = bias2;
    a.Co2 = Co2;
    a.Kp2 = (int)kpad(Co);
    a.relu2 = relu2;
    a.x2 = nullptr;
    a.Ci2 = a.H2 = a.W2 = a.stride2 = 0;
    return launch_chain(a, (hipStream_t)stream);
}

int bev_conv2d_chain_dual_f32(const float *x, int N, int H, int W, int Ci, const float *packed, const float *bias,
                              int Co, int KH, int KW, int stride, int pad, int relu, const float *x2, int H2, int W2,
                              int Ci2, int stride2, const float *packed2, const float *bias2, int Co2, int relu2,
                              float *y, int Ho, int Wo, void *stream) {
    if (!x2 || Ci2 <= 0 || Ci2 % BK != 0 || H2 <= 0 || W2 <= 0 || stride2 <= 0 || ((uintptr_t)x2 & 15) != 0)
        return BEV_ERR_ARGS;
    if (Ho != (H2 - 1) / stride2 + 1 || Wo != (W2 - 1) / stride2 + 1) return BEV_ERR_ARGS;
    if ((int64_t)N * H2 * W2 * Ci2 * 4 > (int64_t)0xffffffff) return BEV_ERR_ARGS;  // 32-bit buffer offsets
    // validate / fill the common part through the plain entry point's checks, then launch with x2
    if (!x || !packed || !packed2 || !y || N < 0 || H <= 0 || W <= 0 || KH <= 0 || KW <= 0 || stride <= 0 ||
        pad < 0 || relu < 0 || relu > 2 || relu2 < 0 || relu2 > 2)
        return BEV_ERR_ARGS;
    if (Ci % BK != 0 || (Co != 64 && Co != 128) || Co2 <= 0 || Co2 % 128 != 0 || ((uintptr_t)x & 15) != 0 ||
        (((uintptr_t)packed | (uintptr_t)packed2) & 15) != 0)
        return BEV_ERR_ARGS;
    if (Ho != (H + 2 * pad - KH) / stride + 1 || Wo != (W + 2 * pad - KW) / stride + 1 || Ho <= 0 || Wo <= 0)
        return BEV_ERR_ARGS;
    if (N == 0) return 0;
    ConvArgs a{};
    a.x = x;
    a.wp = packed;
    a.bias = bias;
    a.res = nullptr;
    a.y = y;
    a.N = N;
    a.H = H;
    a.W = W;
    a.Ci = Ci;
    a.Co = Co;
    a.KH = KH;
    a.KW = KW;
    a.stride = stride;
    a.pad = pad;
    a.Ho = Ho;
    a.Wo = Wo;
    a.relu = relu;
    a.M = (int64_t)N * Ho * Wo;
    a.K = Ci * KH * KW;
    a.Kp = (int)kpad(a.K);
    a.dil = 1;
    a.ldy = Co2;
    a.xcd = conv_xcd();
    a.wp2 = packed2;
    a.bias2 = bias2;
    a.Co2 = Co2;
    a.Kp2 = (int)kpad(Co + Ci2);
    a.relu2 = relu2;
    a.x2 = x2;
    a.Ci2 = Ci2;
    a.H2 = H2;
    a.W2 = W2;
    a.stride2 = stride2;
    return launch_chain(a, (hipStream_t)stream);
}

// The same pooling with a (pixel-row-piece, output row, image) grid: 32-bit index arithmetic (the flat kernel's
// 64-bit divisions and modulos made it ALU-bound at ~1.6 TB/s on the ResNet stem output), one float4 of channels per
// thread, the window's rows read as coalesced float4 runs along the row.
__global__ __launch_bounds__(256) void k_maxpool_rows(const float4 *__restrict__ x, int H, int W, int CV, int k,
                                                      int s, int p, float4 *__restrict__ y, int Ho, int Wo) {
    const int oy = blockIdx.y, n = blockIdx.z;
    const int t = blockIdx.x * 256 + threadIdx.x;  // (ox, c4) within the output row
    if (t >= Wo * CV) return;
    const int ox = t / CV, c = t - ox * CV;
    const float ninf = -__builtin_inff();
    float m[4] = {ninf, ninf, ninf, ninf};
    const int iy0 = oy * s - p, ix0 = ox * s - p;
    for (int ky = 0; ky < k; ++ky) {
        const int iy = iy0 + ky;
        if (iy < 0 || iy >= H) continue;
        const float4 *row = x + ((size_t)n * H + iy) * (size_t)W * CV + c;
        for (int kx = 0; kx < k; ++kx) {
            const int ix = ix0 + kx;
            if (ix < 0 || ix >= W) continue;
            const float4 v = row[(size_t)ix * CV];
            const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int u = 0; u < 4; ++u) m[u] = (vv[u] > m[u] || vv[u] != vv[u]) ? vv[u] : m[u];
        }
    }
    y[((size_t)n * Ho + oy) * (size_t)Wo * CV + t] = make_float4(m[0], m[1], m[2], m[3]);
}

int bev_maxpool2d_nhwc_f32(const float *x, int N, int H, int W, int C, int k, int stride, int pad, float *y, int Ho,
                           int Wo, void *stream) {
    if (!x || !y || N < 0 || H <= 0 || W <= 0 || C <= 0 || k <= 0 || stride <= 0 || pad < 0) return BEV_ERR_ARGS;
    if (Ho != (H + 2 * pad - k) / stride + 1 || Wo != (W + 2 * pad - k) / stride + 1) return BEV_ERR_ARGS;
    const bool vec = (C % 4 == 0) && (((uintptr_t)x & 15) == 0) && (((uintptr_t)y & 15) == 0);
    const int64_t total = (int64_t)N * Ho * Wo * (vec ? C / 4 : C);
    if (total == 0) return 0;
    if (vec && (int64_t)Wo * (C / 4) < (1ll << 30) && Ho < 65536 && N < 65536)
        hipLaunchKernelGGL(k_maxpool_rows, dim3((unsigned)(((int64_t)Wo * (C / 4) + 255) / 256), Ho, N), dim3(256), 0,
                           (hipStream_t)stream, reinterpret_cast<const float4 *>(x), H, W, C / 4, k, stride, pad,
                           reinterpret_cast<float4 *>(y), Ho, Wo);
    else if (vec)
        hipLaunchKernelGGL(k_maxpool<true>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                           x, N, H, W, C, k, stride, pad, y, Ho, Wo);
    else
        hipLaunchKernelGGL(k_maxpool<false>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                           x, N, H, W, C, k, stride, pad, y, Ho, Wo);
    return last();
}

// 3-channel images (the stem's input, for its weight gradient): 4 pixels per thread, one float4 from each plane in,
// three float4 of interleaved channels out (the 32 x 32 tiles of k_transpose would use 3 of their 32 rows)
__global__ __launch_bounds__(256) void k_nchw3_to_nhwc(const float4 *__restrict__ x, int64_t S4, int64_t total,
                                                       float4 *__restrict__ y) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= total) return;
    const int64_t n = t / S4, q = t - n * S4;
    const float4 *xn = x + n * 3 * S4 + q;
    const float4 a = xn[0], b = xn[S4], c = xn[2 * S4];
    float4 *yp = y + t * 3;
    yp[0] = make_float4(a.x, b.x, c.x, a.y);
    yp[1] = make_float4(b.y, c.y, a.z, b.z);
    yp[2] = make_float4(c.z, a.w, b.w, c.w);
}

// C <= 4 channels to 4-channel pixels (zero padding): one float4 per pixel -- the stem's input as the float4 operand
// of its weight gradient, without a separate zero-pad copy
__global__ __launch_bounds__(256) void k_nchw_to_nhwc4(const float *__restrict__ x, int C, int64_t S, int64_t total,
                                                       float4 *__restrict__ y) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= total) return;
    const int64_t n = t / S, q = t - n * S;
    const float *xn = x + n * C * S + q;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < C; ++c) v[c] = xn[c * S];
    y[t] = make_float4(v[0], v[1], v[2], v[3]);
}

int bev_nchw_to_nhwc4_f32(const float *x, int N, int C, int H, int W, float *y, void *stream) {
    if (!x || !y || N < 0 || C <= 0 || C > 4 || H <= 0 || W <= 0 || ((uintptr_t)y & 15) != 0) return BEV_ERR_ARGS;
    const int64_t S = (int64_t)H * W, total = (int64_t)N * S;
    if (total == 0) return 0;
    hipLaunchKernelGGL(k_nchw_to_nhwc4, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, C,
                       S, total, reinterpret_cast<float4 *>(y));
    return last();
}

int bev_nchw_to_nhwc_f32(const float *x, int N, int C, int H, int W, float *y, void *stream) {
    if (!x || !y || N < 0 || C <= 0 || H <= 0 || W <= 0) return BEV_ERR_ARGS;
    if (N == 0) return 0;
    const int S = H * W;
    if (C == 3 && S % 4 == 0 && (((uintptr_t)x | (uintptr_t)y) & 15) == 0) {
        const int64_t total = (int64_t)N * (S / 4);
        hipLaunchKernelGGL(k_nchw3_to_nhwc, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                           reinterpret_cast<const float4 *>(x), (int64_t)(S / 4), total, reinterpret_cast<float4 *>(y));
        return last();
    }
    hipLaunchKernelGGL(k_transpose, dim3((S + 31) / 32, (C + 31) / 32, N), dim3(32, 8), 0, (hipStream_t)stream, x, C,
                       S, y);
    return last();
}

int bev_nhwc_to_nchw_f32(const float *x, int N, int C, int H, int W, float *y, void *stream) {
    if (!x || !y || N < 0 || C <= 0 || H <= 0 || W <= 0) return BEV_ERR_ARGS;
    if (N == 0) return 0;
    const int S = H * W;
    hipLaunchKernelGGL(k_transpose, dim3((C + 31) / 32, (S + 31) / 32, N), dim3(32, 8), 0, (hipStream_t)stream, x, S,
                       C, y);
    return last();
}

}  // extern "C"
