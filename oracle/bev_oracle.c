/*
 * bev_oracle.c -- CPU restatement of the reference's multi-view -> BEV hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker (the "oracle"):
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it.  The product path (the HIP library in
 * vision-based-spatio-temporal-analysis_amd/csrc) never calls it.
 *
 * Parity status: PINNED.  Every function below is checked bit-for-bit against
 * the golden fixtures in the tests/golden fixtures, which were produced by importing
 * the reference's own modules (tests/golden/make_golden.py).
 *
 * It restates, in plain IEEE fp32 with explicit FMA placement, what the
 * reference computes through torch on the CPU:
 *   - linspace of the BEV cell centres       geometry.py:26-27 (torch.linspace)
 *   - H = K @ [r1 r2 t]                        geometry.py:33-64 (MKL sgemm, 3-term dot)
 *   - uvw = H @ [x y 1]^T, w_safe, u, v        geometry.py:144-149
 *   - feature-space rescale and [-1,1] norm    geometry.py:151-158
 *   - F.grid_sample(bilinear, zeros, align_corners=False)  geometry.py:161
 *     (ATen grid_sampler_2d CPU vectorised kernel semantics)
 *   - SimpleFusion sum / mean / max over views fusion.py:17-22
 *   - a direct NCHW conv2d (+bias, optional ReLU) for the fallback encoder
 *     cnn_encoder.py:31-37 (tolerance check only: MKL-DNN's accumulation order
 *     is not restated).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off).  -ffp-contract=off is
 * essential: every fused multiply-add below is written as fmaf() explicitly.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

/* torch.linspace on the CPU.  lo/hi are Python
 * doubles rounded to f32; step in f32; the first half counts up from lo, the
 * second half counts down from hi (both with a single FMA). */
int oracle_linspace_f32(double lo, double hi, int n, float *out) {
    if (n <= 0) return 0;
    float lo_f = (float)lo, hi_f = (float)hi;
    if (n == 1) { out[0] = lo_f; return 0; }
    float step = (hi_f - lo_f) / (float)(n - 1);
    int half = n / 2;
    for (int i = 0; i < n; ++i) {
        if (i < half) out[i] = fmaf(step, (float)i, lo_f);
        else out[i] = fmaf(-step, (float)(n - 1 - i), hi_f);
    }
    return 0;
}

/* 3-term dot product as MKL sgemm rounds it.
 * variant 0 = AVX-512 kernel: fma(a2,b2, fma(a1,b1, fma(a0,b0, +0)))
 *             (the accumulator starts at +0: a -0 product becomes +0, which the
 *             homography fixtures with a zero translation column pin down)
 * variant 1 = AVX2 kernel:    fma(a2,b2, a0*b0 + a1*b1)                        */
static inline float dot3(float a0, float a1, float a2, float b0, float b1, float b2, int variant) {
    if (variant == 0) return fmaf(a2, b2, fmaf(a1, b1, fmaf(a0, b0, 0.0f)));
    float p0 = a0 * b0, p1 = a1 * b1;
    return fmaf(a2, b2, p0 + p1);
}

/* geometry.py:60-63: H = K[:3,:3] @ G with G = [r1 r2 t] (3x3, row-major). */
int oracle_homography_f32(const float *K, const float *G, int n, float *H, int variant) {
    for (int k = 0; k < n; ++k) {
        const float *Kk = K + 9 * k, *Gk = G + 9 * k;
        float *Hk = H + 9 * k;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                Hk[3 * i + j] = dot3(Kk[3 * i], Kk[3 * i + 1], Kk[3 * i + 2], Gk[j], Gk[3 + j], Gk[6 + j], variant);
    }
    return 0;
}

/* geometry.py:144-158 for one BEV cell: returns the normalised grid (gx, gy)
 * that the reference hands to grid_sample.  sx = f32(Wf / W_img), sy likewise. */
static inline void cell_grid(const float *H, float x, float y, int Hf, int Wf, float sx, float sy, int variant,
                             float *gx, float *gy) {
    float u0 = dot3(H[0], H[1], H[2], x, y, 1.0f, variant);
    float u1 = dot3(H[3], H[4], H[5], x, y, 1.0f, variant);
    float w = dot3(H[6], H[7], H[8], x, y, 1.0f, variant);
    float ws = (fabsf(w) < 1e-6f) ? 1.0f : w;
    float u = u0 / ws, v = u1 / ws;
    float fx = u * sx, fy = v * sy;
    *gx = ((fx + 0.5f) / (float)Wf) * 2.0f - 1.0f;
    *gy = ((fy + 0.5f) / (float)Hf) * 2.0f - 1.0f;
}

/* Grid for N views: grid[N][Hb][Wb][2] (gx, gy) exactly as geometry.py:159 builds it. */
int oracle_grid_f32(const float *Hmat, const float *xs, const float *ys, int n, int Hf, int Wf, float sx, float sy,
                    int Hb, int Wb, float *grid, int variant) {
    for (int k = 0; k < n; ++k)
        for (int i = 0; i < Hb; ++i)
            for (int j = 0; j < Wb; ++j) {
                float *g = grid + (((size_t)k * Hb + i) * Wb + j) * 2;
                cell_grid(Hmat + 9 * k, xs[j], ys[i], Hf, Wf, sx, sy, variant, &g[0], &g[1]);
            }
    return 0;
}

/* ATen grid_sampler_2d (CPU, vectorised, bilinear, zeros, align_corners=False)
 * for one grid point.  Outputs the integer corner (x0,y0), the four bilinear
 * weights, and a validity bit per tap (bit0 nw, bit1 ne, bit2 sw, bit3 se). */
static inline void bilinear_taps(float gx, float gy, int Hf, int Wf, int *x0, int *y0, float wts[4], int *valid) {
    float ix = fmaf(gx + 1.0f, (float)Wf / 2.0f, -0.5f);
    float iy = fmaf(gy + 1.0f, (float)Hf / 2.0f, -0.5f);
    float xw = floorf(ix), yn = floorf(iy);
    float we = ix - xw, e = 1.0f - we;
    float n = iy - yn, s = 1.0f - n;
    wts[0] = s * e;   /* nw */
    wts[1] = s * we;  /* ne */
    wts[2] = n * e;   /* sw */
    wts[3] = n * we;  /* se */
    /* validity decided in float: exact for every representable corner and
     * immune to int overflow when |ix| is huge near the horizon. */
    int vx0 = (xw >= 0.0f) && (xw < (float)Wf);
    int vx1 = (xw + 1.0f >= 0.0f) && (xw + 1.0f < (float)Wf);
    int vy0 = (yn >= 0.0f) && (yn < (float)Hf);
    int vy1 = (yn + 1.0f >= 0.0f) && (yn + 1.0f < (float)Hf);
    *valid = (vx0 && vy0) | ((vx1 && vy0) << 1) | ((vx0 && vy1) << 2) | ((vx1 && vy1) << 3);
    *x0 = (vx0 || vx1) ? (int)xw : 0;
    *y0 = (vy0 || vy1) ? (int)yn : 0;
}

/* Per-view warp: feats [N][C][Hf][Wf] (NCHW) -> out [N][C][Hb][Wb].
 * Equivalent to geometry.py:142-162 for every (b,v) (N = B*V). */
int oracle_warp_f32(const float *feats, const float *Hmat, const float *xs, const float *ys, int n, int C, int Hf,
                    int Wf, float sx, float sy, int Hb, int Wb, float *out, int variant) {
    size_t plane = (size_t)Hf * Wf, oplane = (size_t)Hb * Wb;
    for (int k = 0; k < n; ++k)
        for (int i = 0; i < Hb; ++i)
            for (int j = 0; j < Wb; ++j) {
                float gx, gy, w[4];
                int x0, y0, valid;
                cell_grid(Hmat + 9 * k, xs[j], ys[i], Hf, Wf, sx, sy, variant, &gx, &gy);
                bilinear_taps(gx, gy, Hf, Wf, &x0, &y0, w, &valid);
                for (int c = 0; c < C; ++c) {
                    const float *f = feats + ((size_t)k * C + c) * plane;
                    float vnw = (valid & 1) ? f[(size_t)y0 * Wf + x0] : 0.0f;
                    float vne = (valid & 2) ? f[(size_t)y0 * Wf + x0 + 1] : 0.0f;
                    float vsw = (valid & 4) ? f[(size_t)(y0 + 1) * Wf + x0] : 0.0f;
                    float vse = (valid & 8) ? f[(size_t)(y0 + 1) * Wf + x0 + 1] : 0.0f;
                    float r = fmaf(vse, w[3], fmaf(vsw, w[2], fmaf(vne, w[1], vnw * w[0])));
                    out[((size_t)k * C + c) * oplane + (size_t)i * Wb + j] = r;
                }
            }
    return 0;
}

/* Bilinear corner dump for index-exactness checks: x0y0 [N][Hb][Wb][2] int32,
 * wts [N][Hb][Wb][4], valid [N][Hb][Wb] uint8. */
int oracle_taps_f32(const float *Hmat, const float *xs, const float *ys, int n, int Hf, int Wf, float sx, float sy,
                    int Hb, int Wb, int32_t *x0y0, float *wts, uint8_t *valid, int variant) {
    for (int k = 0; k < n; ++k)
        for (int i = 0; i < Hb; ++i)
            for (int j = 0; j < Wb; ++j) {
                size_t cell = ((size_t)k * Hb + i) * Wb + j;
                float gx, gy;
                int x0, y0, vb;
                cell_grid(Hmat + 9 * k, xs[j], ys[i], Hf, Wf, sx, sy, variant, &gx, &gy);
                bilinear_taps(gx, gy, Hf, Wf, &x0, &y0, wts + 4 * cell, &vb);
                x0y0[2 * cell] = x0;
                x0y0[2 * cell + 1] = y0;
                valid[cell] = (uint8_t)vb;
            }
    return 0;
}

/* fusion.py:17-22 over x [B][V][M]: mode 0 sum, 1 mean, 2 max -> out [B][M].
 * sum: sequential v = 0..V-1 starting from +0; mean: that sum / f32(V) (true
 * division); max: NaN-propagating elementwise max (torch.max semantics). */
int oracle_fuse_f32(const float *x, int B, int V, long long M, int mode, float *out) {
    for (int b = 0; b < B; ++b)
        for (long long m = 0; m < M; ++m) {
            const float *p = x + (size_t)b * V * M + m;
            float acc;
            if (mode == 2) {
                acc = p[0];
                for (int v = 1; v < V; ++v) {
                    float t = p[(size_t)v * M];
                    if (isnan(t) || t > acc) acc = isnan(acc) ? acc : t;
                }
            } else {
                acc = 0.0f;
                for (int v = 0; v < V; ++v) acc = acc + p[(size_t)v * M];
                if (mode == 1) acc = acc / (float)V;
            }
            out[(size_t)b * M + m] = acc;
        }
    return 0;
}

/* Direct NCHW conv2d with bias and optional ReLU (cnn_encoder.py:31-37 fallback
 * stack, and the torch-free check of the HIP conv kernels).  Accumulates in
 * double: the comparison against MKL-DNN / MFMA is tolerance-based. */
int oracle_conv2d_f32(const float *x, const float *w, const float *bias, int N, int Ci, int H, int W, int Co, int KH,
                      int KW, int stride, int pad, int relu, float *y) {
    int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
    for (int n = 0; n < N; ++n)
        for (int co = 0; co < Co; ++co)
            for (int oy = 0; oy < Ho; ++oy)
                for (int ox = 0; ox < Wo; ++ox) {
                    double acc = bias ? bias[co] : 0.0;
                    for (int ci = 0; ci < Ci; ++ci)
                        for (int ky = 0; ky < KH; ++ky) {
                            int iy = oy * stride - pad + ky;
                            if (iy < 0 || iy >= H) continue;
                            for (int kx = 0; kx < KW; ++kx) {
                                int ix = ox * stride - pad + kx;
                                if (ix < 0 || ix >= W) continue;
                                acc += (double)x[(((size_t)n * Ci + ci) * H + iy) * W + ix] *
                                       (double)w[(((size_t)co * Ci + ci) * KH + ky) * KW + kx];
                            }
                        }
                    float r = (float)acc;
                    if (relu && r < 0.0f) r = 0.0f;
                    y[(((size_t)n * Co + co) * Ho + oy) * Wo + ox] = r;
                }
    return 0;
}
