// bev_warp.hip -- IPM homography warp + N-view BEV fusion for gfx950 (MI355X).
//
// Replaces the reference's per-(b,v) Python loop in
// GeometryTransformer.forward (geometry.py:120-162: homography, grid build,
// F.grid_sample, bev_out[b,v] = ...) and SimpleFusion (fusion.py:17-22).
//
// Kernels
//   k_homography     H = K @ [r1 r2 t]                      (geometry.py:60-63)
//   k_taps           integer corners / weights dump         (geometry.py:161)
//   k_warp           per-view warp, out [N][C][Hb][Wb]      (geometry.py:142-162)
//   k_warp_fuse      warp + view reduce, out [B][C][Hb][Wb] (+ fusion.py:17-22)
//   k_warp_bwd       d out / d feats (float atomics)
//   k_view_fuse      SimpleFusion on materialised maps      (fusion.py:19-22)
//
// The fused kernel is the hot one.  One workgroup owns a TILE_H x TILE_W tile
// of BEV cells (one lane per cell, a wavefront = one 64-cell row segment, so
// every per-channel output store is a contiguous 256-B row piece).  For each
// view it computes the cell's bilinear taps once (bit-exact recipe), reduces
// the tile's source-footprint bounding box across the workgroup, and - when
// the footprint fits - stages that feature rectangle (all channels of the
// current chunk) into LDS as [pixel][channel] so each tap of four channels is
// ONE ds_read_b128; the view's samples are accumulated in registers in the
// reference order (v = 0..V-1).  Footprints that do not fit (cells near the
// horizon map to huge source regions) fall back to direct global gathers for
// that (tile, view).  Output is written once, non-temporally.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bev_geometry.h"
#include "../../include/bev_mi355x.h"

using namespace bev;

namespace {

constexpr int TILE_W = 64;  // cells per wavefront row (one wave = one row piece)
constexpr int TILE_H = 4;   // wavefronts per workgroup
constexpr int NT = TILE_W * TILE_H;

// -------------------------------------------------------------------------
// H = K @ G   (one thread per matrix entry)
// -------------------------------------------------------------------------
__global__ void k_homography(const float *__restrict__ K, const float *__restrict__ G, int n, float *__restrict__ H) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * 9) return;
    const int k = t / 9, ij = t % 9, i = ij / 3, j = ij % 3;
    const float *Kk = K + 9 * k, *Gk = G + 9 * k;
    H[t] = dot3(Kk[3 * i], Kk[3 * i + 1], Kk[3 * i + 2], Gk[j], Gk[3 + j], Gk[6 + j]);
}

__device__ __forceinline__ void load_h(const float *__restrict__ Hmat, int n, float h[9]) {
#pragma unroll
    for (int q = 0; q < 9; ++q) h[q] = Hmat[9 * n + q];
}

// -------------------------------------------------------------------------
// tap dump
// -------------------------------------------------------------------------
__global__ void k_taps(const float *__restrict__ Hmat, const float *__restrict__ xs, const float *__restrict__ ys,
                       int Hf, int Wf, float sx, float sy, int Hb, int Wb, int32_t *__restrict__ x0y0,
                       float *__restrict__ wts, uint8_t *__restrict__ valid) {
    const int j = blockIdx.x * TILE_W + threadIdx.x;
    const int i = blockIdx.y * TILE_H + threadIdx.y;
    const int n = blockIdx.z;
    if (i >= Hb || j >= Wb) return;
    float h[9];
    load_h(Hmat, n, h);
    const Taps t = cell_taps(h, xs[j], ys[i], Hf, Wf, sx, sy);
    const size_t cell = ((size_t)n * Hb + i) * Wb + j;
    x0y0[2 * cell] = t.x0;
    x0y0[2 * cell + 1] = t.y0;
#pragma unroll
    for (int q = 0; q < 4; ++q) wts[4 * cell + q] = t.w[q];
    valid[cell] = (uint8_t)t.valid;
}

// Global-memory tap offsets (element offsets inside one feature map; invalid
// taps point at offset 0 and are masked to zero).
struct GOff {
    int64_t o[4];
};

__device__ __forceinline__ GOff global_offsets(const Taps &t, int64_t sH, int64_t sW) {
    GOff g;
    const int64_t base = (int64_t)t.y0 * sH + (int64_t)t.x0 * sW;
    g.o[0] = (t.valid & 1) ? base : 0;
    g.o[1] = (t.valid & 2) ? base + sW : 0;
    g.o[2] = (t.valid & 4) ? base + sH : 0;
    g.o[3] = (t.valid & 8) ? base + sH + sW : 0;
    return g;
}

__device__ __forceinline__ float sample_global(const float *__restrict__ f, const GOff &g, const Taps &t) {
    const float a = f[g.o[0]], b = f[g.o[1]], c = f[g.o[2]], d = f[g.o[3]];
    return bilerp((t.valid & 1) ? a : 0.0f, (t.valid & 2) ? b : 0.0f, (t.valid & 4) ? c : 0.0f,
                  (t.valid & 8) ? d : 0.0f, t.w);
}

// -------------------------------------------------------------------------
// per-view warp: out [N][C][Hb][Wb]
// -------------------------------------------------------------------------
__global__ __launch_bounds__(NT) void k_warp(const float *__restrict__ feats, int64_t sN, int64_t sC, int64_t sH,
                                             int64_t sW, const float *__restrict__ Hmat, const float *__restrict__ xs,
                                             const float *__restrict__ ys, int C, int Hf, int Wf, float sx, float sy,
                                             int Hb, int Wb, float *__restrict__ out) {
    const int j = blockIdx.x * TILE_W + threadIdx.x;
    const int i = blockIdx.y * TILE_H + threadIdx.y;
    const int n = blockIdx.z;
    if (i >= Hb || j >= Wb) return;
    float h[9];
    load_h(Hmat, n, h);
    const Taps t = cell_taps(h, xs[j], ys[i], Hf, Wf, sx, sy);
    const GOff g = global_offsets(t, sH, sW);
    const float *f = feats + (int64_t)n * sN;
    const size_t plane = (size_t)Hb * Wb;
    float *o = out + (size_t)n * C * plane + (size_t)i * Wb + j;
    if (t.valid == 0) {
        for (int c = 0; c < C; ++c) __builtin_nontemporal_store(0.0f, o + (size_t)c * plane);
        return;
    }
    for (int c = 0; c < C; ++c) {
        const float r = sample_global(f + (int64_t)c * sC, g, t);
        __builtin_nontemporal_store(r, o + (size_t)c * plane);
    }
}

// -------------------------------------------------------------------------
// fused warp + reduce: out [B][C][Hb][Wb]
// -------------------------------------------------------------------------
// LDS image of one view's footprint for a chunk of CK channels:
//   pixel p (row-major inside the bbox) at byte p*PSTRIDE, channels packed.
// PSTRIDE = CK*4 + 16 keeps consecutive pixels on different 16-B bank slots
// (stride in slots = CK/4 + 1, odd) so the 16-lane groups of ds_read_b128 hit
// distinct slots; lanes sampling the same pixel broadcast.
// One extra all-zero pixel at index npix serves every invalid tap.
constexpr int LDS_BYTES = 40 * 1024;

template <int CK>
struct Stage {
    static constexpr int PSTRIDE = CK * 4 + 16;
    static constexpr int MAXPIX = LDS_BYTES / PSTRIDE - 1;
};

__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}

template <int CK, int MODE>
__global__ __launch_bounds__(NT) void k_warp_fuse(const float *__restrict__ feats, int64_t sN, int64_t sC, int64_t sH,
                                                  int64_t sW, const float *__restrict__ Hmat,
                                                  const float *__restrict__ xs, const float *__restrict__ ys, int V,
                                                  int C, int Hf, int Wf, float sx, float sy, int Hb, int Wb,
                                                  float *__restrict__ out) {
    using S = Stage<CK>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    int (*red)[TILE_H] = reinterpret_cast<int (*)[TILE_H]>(smem + LDS_BYTES);  // [4][TILE_H] bbox partials

    const int tx = threadIdx.x, ty = threadIdx.y, tid = ty * TILE_W + tx;
    const int j = blockIdx.x * TILE_W + tx;
    const int i = blockIdx.y * TILE_H + ty;
    const int b = blockIdx.z;
    const bool inside = (i < Hb) && (j < Wb);
    const float cx = xs[inside ? j : 0], cy = ys[inside ? i : 0];
    const size_t plane = (size_t)Hb * Wb;
    float *o = out + (size_t)b * C * plane + (size_t)(inside ? i : 0) * Wb + (inside ? j : 0);

    for (int c0 = 0; c0 < C; c0 += CK) {
        const int ck = min(CK, C - c0);
        float acc[CK];
#pragma unroll
        for (int q = 0; q < CK; ++q) acc[q] = 0.0f;

        for (int v = 0; v < V; ++v) {
            const int n = b * V + v;
            float h[9];
            load_h(Hmat, n, h);
            Taps t = cell_taps(h, cx, cy, Hf, Wf, sx, sy);
            if (!inside) t.valid = 0;
            // footprint bbox over valid taps of the workgroup
            int bx0 = 0x7fffffff, by0 = 0x7fffffff, bx1 = -1, by1 = -1;
            if (t.valid) {
                bx0 = (t.valid & 5) ? t.x0 : t.x0 + 1;
                bx1 = (t.valid & 10) ? t.x0 + 1 : t.x0;
                by0 = (t.valid & 3) ? t.y0 : t.y0 + 1;
                by1 = (t.valid & 12) ? t.y0 + 1 : t.y0;
            }
            bx0 = wave_min(bx0);
            by0 = wave_min(by0);
            bx1 = wave_max(bx1);
            by1 = wave_max(by1);
            __syncthreads();  // previous view's LDS reads are done before red[] / smem reuse
            if (tx == 0) {
                red[0][ty] = bx0;
                red[1][ty] = by0;
                red[2][ty] = bx1;
                red[3][ty] = by1;
            }
            __syncthreads();
#pragma unroll
            for (int w = 0; w < TILE_H; ++w) {
                bx0 = min(bx0, red[0][w]);
                by0 = min(by0, red[1][w]);
                bx1 = max(bx1, red[2][w]);
                by1 = max(by1, red[3][w]);
            }
            if (bx1 < 0) {
                // no cell of the tile sees this view: every sample is +0
                if (MODE == BEV_FUSE_MAX) {
#pragma unroll
                    for (int q = 0; q < CK; ++q) acc[q] = (v == 0) ? 0.0f : nan_max(acc[q], 0.0f);
                }
                continue;  // sum / mean: acc + (+0) == acc (acc is never -0 here)
            }
            const int bw = bx1 - bx0 + 1, bh = by1 - by0 + 1;
            const int npix = bw * bh;
            const float *f = feats + (int64_t)n * sN + (int64_t)c0 * sC;
            float smp[CK];
            if (npix <= S::MAXPIX) {
                // ---- stage the footprint: [pixel][channel] ------------------------
                // element e -> (pixel p = e / ck, channel q = e % ck); consecutive lanes
                // walk channels first (contiguous in NHWC, strided in NCHW).
                const int total = npix * ck;
                for (int e = tid; e < total; e += NT) {
                    const int p = e / ck, q = e - p * ck;
                    const int py = p / bw, px = p - py * bw;
                    const float val = f[(int64_t)q * sC + (int64_t)(by0 + py) * sH + (int64_t)(bx0 + px) * sW];
                    *(float *)(smem + p * S::PSTRIDE + q * 4) = val;
                }
                if (ck < CK) {  // zero the unused channel slots of every pixel
                    for (int e = tid; e < npix * (CK - ck); e += NT) {
                        const int p = e / (CK - ck), q = ck + e - p * (CK - ck);
                        *(float *)(smem + p * S::PSTRIDE + q * 4) = 0.0f;
                    }
                }
                for (int q = tid; q < CK; q += NT) *(float *)(smem + npix * S::PSTRIDE + q * 4) = 0.0f;
                __syncthreads();
                // ---- gather from LDS ----------------------------------------------
                const int lx = t.x0 - bx0, ly = t.y0 - by0;
                const int pb = ly * bw + lx;
                const int a0 = ((t.valid & 1) ? pb : npix) * S::PSTRIDE;
                const int a1 = ((t.valid & 2) ? pb + 1 : npix) * S::PSTRIDE;
                const int a2 = ((t.valid & 4) ? pb + bw : npix) * S::PSTRIDE;
                const int a3 = ((t.valid & 8) ? pb + bw + 1 : npix) * S::PSTRIDE;
#pragma unroll
                for (int q = 0; q < CK; q += 4) {
                    const float4 vnw = *(const float4 *)(smem + a0 + q * 4);
                    const float4 vne = *(const float4 *)(smem + a1 + q * 4);
                    const float4 vsw = *(const float4 *)(smem + a2 + q * 4);
                    const float4 vse = *(const float4 *)(smem + a3 + q * 4);
                    smp[q + 0] = bilerp(vnw.x, vne.x, vsw.x, vse.x, t.w);
                    smp[q + 1] = bilerp(vnw.y, vne.y, vsw.y, vse.y, t.w);
                    smp[q + 2] = bilerp(vnw.z, vne.z, vsw.z, vse.z, t.w);
                    smp[q + 3] = bilerp(vnw.w, vne.w, vsw.w, vse.w, t.w);
                }
            } else {
                // ---- footprint too large: direct global gathers -----------------------
                const GOff g = global_offsets(t, sH, sW);
#pragma unroll
                for (int q = 0; q < CK; ++q) smp[q] = (q < ck) ? sample_global(f + (int64_t)q * sC, g, t) : 0.0f;
            }
            if (MODE == BEV_FUSE_MAX) {
#pragma unroll
                for (int q = 0; q < CK; ++q) acc[q] = (v == 0) ? smp[q] : nan_max(acc[q], smp[q]);
            } else {
#pragma unroll
                for (int q = 0; q < CK; ++q) acc[q] = acc[q] + smp[q];
            }
        }
        if (inside) {
            const float fv = (float)V;
#pragma unroll
            for (int q = 0; q < CK; ++q) {
                if (q < ck) {
                    const float r = (MODE == BEV_FUSE_MEAN) ? acc[q] / fv : acc[q];
                    __builtin_nontemporal_store(r, o + (size_t)(c0 + q) * plane);
                }
            }
        }
    }
}

// -------------------------------------------------------------------------
// backward (grad w.r.t. feats): scatter-add with float atomics
// -------------------------------------------------------------------------
__global__ __launch_bounds__(NT) void k_warp_bwd(const float *__restrict__ gout, const float *__restrict__ Hmat,
                                                 const float *__restrict__ xs, const float *__restrict__ ys, int V,
                                                 int C, int Hf, int Wf, float sx, float sy, int Hb, int Wb, float scale,
                                                 int per_view_gout, float *__restrict__ gfeats) {
    const int j = blockIdx.x * TILE_W + threadIdx.x;
    const int i = blockIdx.y * TILE_H + threadIdx.y;
    const int n = blockIdx.z;  // feature map index b*V + v
    if (i >= Hb || j >= Wb) return;
    float h[9];
    load_h(Hmat, n, h);
    const Taps t = cell_taps(h, xs[j], ys[i], Hf, Wf, sx, sy);
    if (t.valid == 0) return;
    const size_t plane = (size_t)Hb * Wb, fplane = (size_t)Hf * Wf;
    const int src = per_view_gout ? n : n / V;
    const float *g = gout + (size_t)src * C * plane + (size_t)i * Wb + j;
    float *gf = gfeats + (size_t)n * C * fplane;
    const size_t base = (size_t)t.y0 * Wf + t.x0;
    for (int c = 0; c < C; ++c) {
        float go = g[(size_t)c * plane];
        if (scale != 1.0f) go = go / scale;  // mean backward: grad / V
        float *p = gf + (size_t)c * fplane + base;
        if (t.valid & 1) atomicAdd(p, t.w[0] * go);
        if (t.valid & 2) atomicAdd(p + 1, t.w[1] * go);
        if (t.valid & 4) atomicAdd(p + Wf, t.w[2] * go);
        if (t.valid & 8) atomicAdd(p + Wf + 1, t.w[3] * go);
    }
}

// -------------------------------------------------------------------------
// SimpleFusion on materialised maps: x [B][V][M] -> out [B][M]
// -------------------------------------------------------------------------
template <int MODE>
__global__ void k_view_fuse(const float *__restrict__ x, int V, int64_t M, float *__restrict__ out) {
    const int b = blockIdx.y;
    const float *xb = x + (size_t)b * V * M;
    float *ob = out + (size_t)b * M;
    const float fv = (float)V;
    for (int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; m < M; m += (int64_t)gridDim.x * blockDim.x) {
        float acc;
        if (MODE == BEV_FUSE_MAX) {
            acc = xb[m];
            for (int v = 1; v < V; ++v) acc = nan_max(acc, xb[(size_t)v * M + m]);
        } else {
            acc = 0.0f;
            for (int v = 0; v < V; ++v) acc = acc + xb[(size_t)v * M + m];
            if (MODE == BEV_FUSE_MEAN) acc = acc / fv;
        }
        ob[m] = acc;
    }
}

inline int err(hipError_t e) { return (int)e; }
inline int last() { return (int)hipGetLastError(); }

template <int CK>
int launch_fuse(const float *feats, int64_t sN, int64_t sC, int64_t sH, int64_t sW, const float *Hmat, const float *xs,
                const float *ys, int B, int V, int C, int Hf, int Wf, float sx, float sy, int Hb, int Wb, int mode,
                float *out, hipStream_t st) {
    dim3 grid((Wb + TILE_W - 1) / TILE_W, (Hb + TILE_H - 1) / TILE_H, B), block(TILE_W, TILE_H);
    const size_t lds = LDS_BYTES + 4 * TILE_H * sizeof(int);
    switch (mode) {
        case BEV_FUSE_SUM:
            hipLaunchKernelGGL((k_warp_fuse<CK, BEV_FUSE_SUM>), grid, block, lds, st, feats, sN, sC, sH, sW, Hmat, xs,
                               ys, V, C, Hf, Wf, sx, sy, Hb, Wb, out);
            break;
        case BEV_FUSE_MEAN:
            hipLaunchKernelGGL((k_warp_fuse<CK, BEV_FUSE_MEAN>), grid, block, lds, st, feats, sN, sC, sH, sW, Hmat,
                               xs, ys, V, C, Hf, Wf, sx, sy, Hb, Wb, out);
            break;
        default:
            hipLaunchKernelGGL((k_warp_fuse<CK, BEV_FUSE_MAX>), grid, block, lds, st, feats, sN, sC, sH, sW, Hmat, xs,
                               ys, V, C, Hf, Wf, sx, sy, Hb, Wb, out);
    }
    return last();
}

}  // namespace

extern "C" {

int bev_abi_version(void) { return 1; }

int bev_linspace_f32(double lo, double hi, int n, float *out) {
    if (n < 0 || (n > 0 && !out)) return BEV_ERR_ARGS;
    if (n == 0) return 0;
    const float lo_f = (float)lo, hi_f = (float)hi;
    if (n == 1) {
        out[0] = lo_f;
        return 0;
    }
    const float step = (hi_f - lo_f) / (float)(n - 1);
    const int half = n / 2;
    for (int i = 0; i < n; ++i)
        out[i] = (i < half) ? __builtin_fmaf(step, (float)i, lo_f) : __builtin_fmaf(-step, (float)(n - 1 - i), hi_f);
    return 0;
}

int bev_homography_f32(const float *K, const float *G, int n, float *H, void *stream) {
    if (n < 0 || (n > 0 && (!K || !G || !H))) return BEV_ERR_ARGS;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_homography, dim3((n * 9 + 255) / 256), dim3(256), 0, (hipStream_t)stream, K, G, n, H);
    return last();
}

int bev_ipm_taps_f32(const float *Hmat, const float *xs, const float *ys, int N, int Hf, int Wf, float sx, float sy,
                     int Hb, int Wb, int32_t *x0y0, float *wts, uint8_t *valid, void *stream) {
    if (N < 0 || Hf <= 0 || Wf <= 0 || Hb < 0 || Wb < 0) return BEV_ERR_ARGS;
    if (N == 0 || Hb == 0 || Wb == 0) return 0;
    dim3 grid((Wb + TILE_W - 1) / TILE_W, (Hb + TILE_H - 1) / TILE_H, N), block(TILE_W, TILE_H);
    hipLaunchKernelGGL(k_taps, grid, block, 0, (hipStream_t)stream, Hmat, xs, ys, Hf, Wf, sx, sy, Hb, Wb, x0y0, wts,
                       valid);
    return last();
}

int bev_ipm_warp_f32(const float *feats, int64_t sN, int64_t sC, int64_t sH, int64_t sW, const float *Hmat,
                     const float *xs, const float *ys, int N, int C, int Hf, int Wf, float sx, float sy, int Hb,
                     int Wb, float *out, void *stream) {
    if (N < 0 || C < 0 || Hf <= 0 || Wf <= 0 || Hb < 0 || Wb < 0 || N > 65535) return BEV_ERR_ARGS;
    if (N == 0 || C == 0 || Hb == 0 || Wb == 0) return 0;
    dim3 grid((Wb + TILE_W - 1) / TILE_W, (Hb + TILE_H - 1) / TILE_H, N), block(TILE_W, TILE_H);
    hipLaunchKernelGGL(k_warp, grid, block, 0, (hipStream_t)stream, feats, sN, sC, sH, sW, Hmat, xs, ys, C, Hf, Wf,
                       sx, sy, Hb, Wb, out);
    return last();
}

int bev_ipm_warp_fuse_f32(const float *feats, int64_t sN, int64_t sC, int64_t sH, int64_t sW, const float *Hmat,
                          const float *xs, const float *ys, int B, int V, int C, int Hf, int Wf, float sx, float sy,
                          int Hb, int Wb, int mode, float *out, void *stream) {
    if (B < 0 || V <= 0 || C < 0 || Hf <= 0 || Wf <= 0 || Hb < 0 || Wb < 0 || B > 65535) return BEV_ERR_ARGS;
    if (mode < BEV_FUSE_SUM || mode > BEV_FUSE_MAX) return BEV_ERR_ARGS;
    if (B == 0 || C == 0 || Hb == 0 || Wb == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    if (C <= 4) return launch_fuse<4>(feats, sN, sC, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, st);
    if (C <= 8) return launch_fuse<8>(feats, sN, sC, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, st);
    return launch_fuse<16>(feats, sN, sC, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, st);
}

int bev_ipm_warp_bwd_f32(const float *gout, const float *Hmat, const float *xs, const float *ys, int N, int C, int Hf,
                         int Wf, float sx, float sy, int Hb, int Wb, float *gfeats, void *stream) {
    if (N < 0 || C < 0 || Hf <= 0 || Wf <= 0 || Hb < 0 || Wb < 0 || N > 65535) return BEV_ERR_ARGS;
    hipStream_t st = (hipStream_t)stream;
    if (N == 0 || C == 0) return 0;
    hipError_t e = hipMemsetAsync(gfeats, 0, sizeof(float) * (size_t)N * C * Hf * Wf, st);
    if (e != hipSuccess) return err(e);
    if (Hb == 0 || Wb == 0) return 0;
    dim3 grid((Wb + TILE_W - 1) / TILE_W, (Hb + TILE_H - 1) / TILE_H, N), block(TILE_W, TILE_H);
    hipLaunchKernelGGL(k_warp_bwd, grid, block, 0, st, gout, Hmat, xs, ys, 1, C, Hf, Wf, sx, sy, Hb, Wb, 1.0f, 1,
                       gfeats);
    return last();
}

int bev_ipm_warp_fuse_bwd_f32(const float *gout, const float *Hmat, const float *xs, const float *ys, int B, int V,
                              int C, int Hf, int Wf, float sx, float sy, int Hb, int Wb, int mode, float *gfeats,
                              void *stream) {
    if (B < 0 || V <= 0 || C < 0 || Hf <= 0 || Wf <= 0 || Hb < 0 || Wb < 0 || B * V > 65535) return BEV_ERR_ARGS;
    if (mode != BEV_FUSE_SUM && mode != BEV_FUSE_MEAN) return BEV_ERR_ARGS;
    hipStream_t st = (hipStream_t)stream;
    if (B == 0 || C == 0) return 0;
    hipError_t e = hipMemsetAsync(gfeats, 0, sizeof(float) * (size_t)B * V * C * Hf * Wf, st);
    if (e != hipSuccess) return err(e);
    if (Hb == 0 || Wb == 0) return 0;
    dim3 grid((Wb + TILE_W - 1) / TILE_W, (Hb + TILE_H - 1) / TILE_H, B * V), block(TILE_W, TILE_H);
    hipLaunchKernelGGL(k_warp_bwd, grid, block, 0, st, gout, Hmat, xs, ys, V, C, Hf, Wf, sx, sy, Hb, Wb,
                       mode == BEV_FUSE_MEAN ? (float)V : 1.0f, 0, gfeats);
    return last();
}

int bev_view_fuse_f32(const float *x, int B, int V, int64_t M, int mode, float *out, void *stream) {
    if (B < 0 || V <= 0 || M < 0 || B > 65535 || mode < BEV_FUSE_SUM || mode > BEV_FUSE_MAX) return BEV_ERR_ARGS;
    if (B == 0 || M == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const int threads = 256;
    int64_t blocks = (M + threads - 1) / threads;
    if (blocks > 4096) blocks = 4096;
    dim3 grid((unsigned)blocks, B);
    if (mode == BEV_FUSE_SUM) hipLaunchKernelGGL(k_view_fuse<BEV_FUSE_SUM>, grid, dim3(threads), 0, st, x, V, M, out);
    else if (mode == BEV_FUSE_MEAN) hipLaunchKernelGGL(k_view_fuse<BEV_FUSE_MEAN>, grid, dim3(threads), 0, st, x, V, M, out);
    else hipLaunchKernelGGL(k_view_fuse<BEV_FUSE_MAX>, grid, dim3(threads), 0, st, x, V, M, out);
    return last();
}

}  // extern "C"
