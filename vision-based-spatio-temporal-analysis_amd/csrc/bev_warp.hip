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
//   k_warp_fuse_v2   warp + view reduce, out [B][C][Hb][Wb] (+ fusion.py:17-22):
//                    the default for NHWC features with C % 64 == 0 -- corner-bounded
//                    footprints staged by LDS-DMA, one workgroup barrier per view
//   k_warp_fuse      the same reduction for any strides / channel count,
//                    register-staged footprint images (NCHW, C % 64 != 0)
//   (the backward, d out / d feats, is bev_warp_bwd.hip)
//   k_view_fuse      SimpleFusion on materialised maps      (fusion.py:19-22)
//   k_view_max_bwd   backward of the max over views (torch max(dim) index rule)
//
// Every fused kernel computes a cell's bilinear taps once per view with the
// bit-exact recipe (bev_geometry.h), stages the tile's source footprint in LDS
// as [pixel][channel] so each tap of four channels is ONE ds_read_b128, and
// accumulates the views in the reference order (v = 0..V-1).  Output is written
// once, non-temporally.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "bev_geometry.h"
#include <algorithm>

#include "bev_tune.h"
#include "../../include/bev_mi355x.h"

// Timing experiments only (tools/warp_ablate.py builds separate libraries with these bits; the product library
// is built with 0): 1 no mean division, 2 no footprint staging, 4 no LDS sampling, 8 no tap arithmetic,
// 16 no output stores.  Any non-zero value gives wrong results.
#ifndef WARP_ABLATE
#define WARP_ABLATE 0
#endif
#ifndef WARP_HSCALAR
#define WARP_HSCALAR 1  // fused warp: homographies of the tap recipe by scalar loads (1) or from the LDS table (0)
#endif
// Fused-warp variants under A/B (results identical): 1 corner boxes by wave 0 only, shared through LDS.
#ifndef WARP_OPT
#define WARP_OPT 1
#endif
#ifndef WARP_DMA_POLICY
#define WARP_DMA_POLICY ""  // footprint LDS-DMA cache policy suffix (A/B builds: " nt")
#endif

using namespace bev;

// V = 1..64 for which Markstein's fp32 division by V (+ NaN fix-up) equals a / V for every float but -0
// (tools/verify_div_markstein_fix.c, exhaustive): bit V - 1.
#define MARKSTEIN_EXACT_V 0xd5555555d555d5dfull

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

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
    const Grid grid = make_grid(Hf, Wf);
    const Taps t = cell_taps(h, xs[j], ys[i], grid, sx, sy);
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
    const Grid grid = make_grid(Hf, Wf);
    const Taps t = cell_taps(h, xs[j], ys[i], grid, sx, sy);
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
// Tile = FT_H x FT_W = 8 x 32 BEV cells, 256 threads, one cell per lane; wave
// w owns rows 2w, 2w+1 (lanes 0-31 / 32-63), so each per-channel output store
// is two full 128-B lines.
//
// LDS image of one view's source footprint for a chunk of CK channels:
//   pixel p (row-major inside the tile's bbox) at byte p*PSTRIDE, CK channels
//   packed.  PSTRIDE = CK*4 + 16 (odd number of 16-B slots) so distinct pixels
//   of a 16-lane ds_read_b128 group sit on distinct bank slots; lanes sampling
//   the same pixel broadcast.  Pixel index npix is an all-zero pixel that
//   every out-of-range tap reads (zeros padding, no branch in the inner loop).
// Per view: taps -> wave bbox (shuffles) -> [barrier] -> block bbox -> stage
// (global float4 -> ds_write_b128) -> [barrier] -> 4 ds_read_b128 per 4
// channels + bilinear + accumulate.  The bbox partials are double-buffered by
// view parity, so two barriers per view suffice.
constexpr int FT_W = 32, FT_H = 8, FT_NT = FT_W * FT_H;

template <int CK>
struct Stage {
    static constexpr int PSTRIDE = CK * 4 + 16;
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

// exact p / d for 0 <= p < 2^22, 1 <= d < 2^22 (float estimate + one correction)
__device__ __forceinline__ int fast_div(int p, int d, float inv_d) {
    int q = (int)((float)p * inv_d);
    const int r = p - q * d;
    q += (r >= d) - (r < 0);
    return q;
}

template <int CK, int MODE, bool VEC>
__global__ __launch_bounds__(FT_NT, 2) void k_warp_fuse(const float *__restrict__ feats, int64_t sN, int64_t sC,
                                                        int64_t sH, int64_t sW, const float *__restrict__ Hmat,
                                                        const float *__restrict__ xs, const float *__restrict__ ys,
                                                        int V, int C, int Hf, int Wf, float sx, float sy, int Hb,
                                                        int Wb, float *__restrict__ out, int img_bytes) {
    constexpr int PS = Stage<CK>::PSTRIDE;
    constexpr int G4 = CK / 4;  // float4 groups per pixel
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    int *red = reinterpret_cast<int *>(smem + img_bytes);  // [2 parity][4 values][4 waves]
    const int maxpix = img_bytes / PS - 1;

    // XCD-aware tile order: consecutive tiles (which share source pixels) are
    // dealt to the same XCD (blocks b, b+8, ... share one); bijective remap.
    const int ntx = (Wb + FT_W - 1) / FT_W, nty = (Hb + FT_H - 1) / FT_H, nt = ntx * nty;
    int tile = blockIdx.x;
    {
        const int q = nt / 8, r = nt % 8, x = tile % 8;
        tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + tile / 8;
    }
    const int tyb = tile / ntx, txb = tile - tyb * ntx;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int i = tyb * FT_H + wave * 2 + (lane >> 5);
    const int j = txb * FT_W + (lane & 31);
    const int b = blockIdx.y;
    const bool inside = (i < Hb) && (j < Wb);
    const float cx = xs[inside ? j : 0], cy = ys[inside ? i : 0];
    const size_t plane = (size_t)Hb * Wb;
    const Grid grid = make_grid(Hf, Wf);
    const double rV = recip_uniform(V);  // mean: acc / V via div_rcp (exact)
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
            Taps t = cell_taps(h, cx, cy, grid, sx, sy);
            if (!inside) t.valid = 0;
            int bx0 = 0x7fffffff, by0 = 0x7fffffff, bx1 = -1, by1 = -1;
            if (t.valid) {
                bx0 = (t.valid & 5) ? t.x0 : t.x0 + 1;
                bx1 = (t.valid & 10) ? t.x0 + 1 : t.x0;
                by0 = (t.valid & 3) ? t.y0 : t.y0 + 1;
                by1 = (t.valid & 12) ? t.y0 + 1 : t.y0;
            }
            const bool wave_any = __ballot(t.valid != 0) != 0ull;
            bx0 = wave_min(bx0);
            by0 = wave_min(by0);
            bx1 = wave_max(bx1);
            by1 = wave_max(by1);
            int *rp = red + (v & 1) * 16;
            if (lane == 0) {
                rp[wave] = bx0;
                rp[4 + wave] = by0;
                rp[8 + wave] = bx1;
                rp[12 + wave] = by1;
            }
            __syncthreads();  // (A) bbox partials visible; previous view's LDS reads are done
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                bx0 = min(bx0, rp[w]);
                by0 = min(by0, rp[4 + w]);
                bx1 = max(bx1, rp[8 + w]);
                by1 = max(by1, rp[12 + w]);
            }
            if (bx1 < 0) {  // no cell of the tile sees this view: every sample is +0
                if (MODE == BEV_FUSE_MAX) {
#pragma unroll
                    for (int q = 0; q < CK; ++q) acc[q] = (v == 0) ? 0.0f : nan_max(acc[q], 0.0f);
                }
                continue;  // sum / mean: acc + (+0) == acc (acc is never -0 here)
            }
            const int bw = bx1 - bx0 + 1, bh = by1 - by0 + 1;
            const float *f = feats + (int64_t)n * sN + (int64_t)c0 * sC;
            // Split the footprint into blocks that fit the LDS budget.  Blocks
            // overlap by one pixel in x and y, so every lane's 2x2 tap quad lies
            // inside the block it is assigned to; almost always there is one block.
            int wb = bw, hb = bh, nbx = 1, nby = 1;
            if (bw * bh > maxpix) {
                wb = (2 * bw <= maxpix) ? bw : maxpix / 2;
                hb = min(bh, maxpix / wb);
                nbx = (wb >= bw) ? 1 : (bw - 2) / (wb - 1) + 1;
                nby = (hb >= bh) ? 1 : (bh - 2) / (hb - 1) + 1;
            }
            const bool single = (nbx == 1) && (nby == 1);
            int mkx = 0, mky = 0;
            if (!single && t.valid) {
                const int xlo = (t.valid & 5) ? t.x0 : t.x0 + 1, ylo = (t.valid & 3) ? t.y0 : t.y0 + 1;
                mkx = (nbx == 1) ? 0 : min((xlo - bx0) / (wb - 1), nbx - 1);
                mky = (nby == 1) ? 0 : min((ylo - by0) / (hb - 1), nby - 1);
            }
            if (!single && MODE == BEV_FUSE_MAX && !t.valid) {
#pragma unroll
                for (int q = 0; q < CK; ++q) acc[q] = (v == 0) ? 0.0f : nan_max(acc[q], 0.0f);
            }
            for (int ky = 0; ky < nby; ++ky) {
                for (int kx = 0; kx < nbx; ++kx) {
                    const int sx0 = bx0 + kx * (wb - 1), sy0 = by0 + ky * (hb - 1);
                    const int sbw = min(wb, bx1 - sx0 + 1), sbh = min(hb, by1 - sy0 + 1);
                    const int npix = sbw * sbh;
                    if (!single) __syncthreads();  // previous block's LDS reads are done
                    // ---- stage the block as [pixel][channel] ----------------------------
                    const float inv_bw = 1.0f / (float)sbw;
                    if (VEC) {  // channels contiguous (NHWC), ck % 4 == 0
                        const int total = npix * G4;
                        for (int e = tid; e < total; e += FT_NT) {
                            const int p = e / G4, g = e - p * G4;
                            const int py = fast_div(p, sbw, inv_bw), px = p - py * sbw;
                            float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
                            if (g * 4 < ck)
                                val = *(const float4 *)(f + (int64_t)(sy0 + py) * sH + (int64_t)(sx0 + px) * sW + g * 4);
                            *(float4 *)(smem + p * PS + g * 16) = val;
                        }
                    } else {  // generic strides
                        const int total = npix * CK;
                        for (int e = tid; e < total; e += FT_NT) {
                            const int p = e / CK, q = e - p * CK;
                            const int py = fast_div(p, sbw, inv_bw), px = p - py * sbw;
                            float val = 0.0f;
                            if (q < ck) val = f[(int64_t)q * sC + (int64_t)(sy0 + py) * sH + (int64_t)(sx0 + px) * sW];
                            *(float *)(smem + p * PS + q * 4) = val;
                        }
                    }
                    if (tid < G4) *(float4 *)(smem + npix * PS + tid * 16) = make_float4(0.f, 0.f, 0.f, 0.f);
                    __syncthreads();  // (B) image ready
                    // single block: every lane of an active wave samples (invalid taps
                    // read the zero pixel -> +0, which is the reference's sample too).
                    const bool mine = single ? true : (t.valid != 0 && mkx == kx && mky == ky);
                    const bool go = single ? wave_any : (__ballot(mine) != 0ull);
                    if (go) {
                        const int pb = (t.y0 - sy0) * sbw + (t.x0 - sx0);
                        const unsigned char *a0 = smem + ((mine && (t.valid & 1)) ? pb : npix) * PS;
                        const unsigned char *a1 = smem + ((mine && (t.valid & 2)) ? pb + 1 : npix) * PS;
                        const unsigned char *a2 = smem + ((mine && (t.valid & 4)) ? pb + sbw : npix) * PS;
                        const unsigned char *a3 = smem + ((mine && (t.valid & 8)) ? pb + sbw + 1 : npix) * PS;
#pragma unroll
                        for (int g = 0; g < G4; ++g) {
                            const float4 vnw = *(const float4 *)(a0 + g * 16);
                            const float4 vne = *(const float4 *)(a1 + g * 16);
                            const float4 vsw = *(const float4 *)(a2 + g * 16);
                            const float4 vse = *(const float4 *)(a3 + g * 16);
                            const float sm[4] = {bilerp(vnw.x, vne.x, vsw.x, vse.x, t.w),
                                                 bilerp(vnw.y, vne.y, vsw.y, vse.y, t.w),
                                                 bilerp(vnw.z, vne.z, vsw.z, vse.z, t.w),
                                                 bilerp(vnw.w, vne.w, vsw.w, vse.w, t.w)};
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                float &a = acc[4 * g + u];
                                float r;
                                if (MODE == BEV_FUSE_MAX) r = (v == 0) ? sm[u] : nan_max(a, sm[u]);
                                else r = a + sm[u];
                                a = mine ? r : a;
                            }
                            // bound the LDS-read lookahead (registers): at most 4 groups in flight
                            if ((g & 3) == 3) __builtin_amdgcn_sched_barrier(0);
                        }
                    } else if (single && MODE == BEV_FUSE_MAX) {
#pragma unroll
                        for (int q = 0; q < CK; ++q) acc[q] = (v == 0) ? 0.0f : nan_max(acc[q], 0.0f);
                    }
                }
            }
        }
        if (inside) {
#pragma unroll
            for (int q = 0; q < CK; ++q) {
                if (q < ck) {
                    const float r = (MODE == BEV_FUSE_MEAN) ? div_rcp(acc[q], rV) : acc[q];
                    __builtin_nontemporal_store(r, o + (size_t)(c0 + q) * plane);
                }
            }
        }
    }
}

// -------------------------------------------------------------------------
// LDS-DMA helpers (NHWC features, 64-channel chunks)
// -------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;
typedef int v4i_t __attribute__((ext_vector_type(4)));


__device__ __forceinline__ unsigned lds_base(const unsigned char *p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) unsigned char *)p;
}

// Issue the DMA of footprint block (sx0, sy0, sbw x sbh) into LDS byte offset `off`.
// Element offsets are 32-bit (the launcher checks that a feature map fits).
template <int S = 17>
__device__ __forceinline__ void dma_block(const float *__restrict__ f, int sH, int sW, int sx0, int sy0, int sbw,
                                          int npix, unsigned char *smem, int off, int wave, int lane,
                                          int nwaves = FT_NT / 64) {
    if (WARP_ABLATE & 2) return;
    const int ninstr = (npix * S + 63) >> 6;
    const float inv_bw = 1.0f / (float)sbw;
    const int base = sy0 * sH + sx0 * sW;
    for (int k = wave; k < ninstr; k += nwaves) {
        const int slot = k * 64 + lane;
        const int p = slot / S, sl = slot - p * S;
        const int py = fast_div(p, sbw, inv_bw), px = p - py * sbw;
        const int eo = base + py * sH + px * sW + ((sl < S - 1) ? sl * 4 : 0);
        const float *src = f + ((p < npix) ? eo : 0);  // tail lanes: any valid address
        // Inline asm on purpose: hipcc treats the builtin's LDS write as aliasing every
        // later ds_read and drains vmcnt before them, which would serialise the
        // prefetch.  Completion is waited for explicitly (vmcnt(0) + barrier) before
        // the image is read.  M0 is saved/restored inside the statement.
        const unsigned dst = (unsigned)__builtin_amdgcn_readfirstlane((int)(lds_base(smem) + off + k * 1024));
        unsigned keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %1, off" WARP_DMA_POLICY "\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(src), "s"(dst)
            : "memory");
    }
}

#ifndef WARP_DMA_ROWS
#define WARP_DMA_ROWS 0  // fused warp v2 staging: 3 pixels of one box row per LDS-DMA instruction (1, A/B: neutral on K2, +4 % on K5) or dma_block (0)
#endif

// The same image as dma_block (pixel p = py * sbw + px at `off` + 272 p, 17 slots of 16 B: 64 channels + pad) from
// one LDS-DMA instruction per 3 pixels of a box row.  Lane l moves chunk l % 17 of pixel l / 17 of the instruction
// (the pad slot and lanes 51-63 stay idle), so its global byte offset from the instruction's first pixel is a
// per-lane constant; the pixel address itself is an SGPR base (global_load_lds_dwordx4 with saddr) and M0 the
// instruction's first slot -- the per-instruction work is scalar.  Instructions are dealt round-robin over the
// waves (row-major), so every wave issues about sbh * ceil(sbw / 3) / nwaves of them.  Element offsets are 32-bit
// (the launcher checks that a feature map fits).
__device__ __forceinline__ void dma_rows(const float *__restrict__ f, int sH, int sW, int sx0, int sy0, int sbw,
                                         int sbh, unsigned char *smem, int off, int wave, int lane,
                                         int nwaves = FT_NT / 64) {
    if (WARP_ABLATE & 2) return;
    const int lp = (lane * 241) >> 12;  // lane / 17 for lane < 64
    const int ls = lane - 17 * lp;
    const bool slot_ok = lp < 3 && ls < 16;
    const unsigned voff = (unsigned)((lp * sW + ls * 4) * (int)sizeof(float));
    const int per_row = (sbw + 2) / 3;
    const unsigned lds0 = (unsigned)__builtin_amdgcn_readfirstlane((int)(lds_base(smem) + (unsigned)off));
    int py = 0, i = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform: the loop runs on the scalar unit
    while (i >= per_row && py < sbh) {  // instruction `wave` of the row-major order
        i -= per_row;
        ++py;
    }
    for (; py < sbh;) {
        const int rem = sbw - 3 * i;  // pixels left in the row from this instruction's first (>= 1)
        const float *src = f + (sy0 + py) * sH + (sx0 + 3 * i) * sW;
        const unsigned dst = lds0 + (unsigned)((py * sbw + 3 * i) * 272);
        if (slot_ok && lp < rem) {
            unsigned keep;
            asm volatile(
                "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                "global_load_lds_dwordx4 %1, %3" WARP_DMA_POLICY "\n\ts_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(voff), "s"(dst), "s"(src)
                : "memory");
        }
        i += nwaves;
        while (i >= per_row && py < sbh) {
            i -= per_row;
            ++py;
        }
    }
}

// Span staging (see row_span): a footprint staged row by row, row r = the `len` pixels from column `sx` of box row r,
// rows back to back from LDS byte offset `off` (pixel exc_r + k of the image = column sx_r + k of row r; exc = the
// exclusive prefix sum of len over the rows).  Lane r of len / sx / exc holds row r's values (r < nrows <= 32).  The
// same instruction form as dma_rows (3 pixels of one row per LDS-DMA instruction, scalar source base and M0); the
// instructions of all rows are dealt round-robin over the waves.
__device__ __forceinline__ void dma_spans(const float *__restrict__ f, int sH, int sW, int sy0, int nrows, int len,
                                          int sxr, int exc, unsigned char *smem, int off, int wave, int lane,
                                          int nwaves = FT_NT / 64) {
    if (WARP_ABLATE & 2) return;
    const int lp = (lane * 241) >> 12;  // lane / 17 for lane < 64
    const int ls = lane - 17 * lp;
    const bool slot_ok = lp < 3 && ls < 16;
    const unsigned voff = (unsigned)((lp * sW + ls * 4) * (int)sizeof(float));
    const unsigned lds0 = (unsigned)__builtin_amdgcn_readfirstlane((int)(lds_base(smem) + (unsigned)off));
    int r = 0, i = __builtin_amdgcn_readfirstlane(wave);
    int rl = __builtin_amdgcn_readlane(len, 0), per = (rl + 2) / 3;
    while (r < nrows) {
        if (i < per) {
            const int rsx = __builtin_amdgcn_readlane(sxr, r), rex = __builtin_amdgcn_readlane(exc, r);
            const float *src = f + (sy0 + r) * sH + (rsx + 3 * i) * sW;
            const unsigned dst = lds0 + (unsigned)((rex + 3 * i) * 272);
            if (slot_ok && lp < rl - 3 * i) {
                unsigned keep;
                asm volatile(
                    "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                    "global_load_lds_dwordx4 %1, %3" WARP_DMA_POLICY "\n\ts_mov_b32 m0, %0"
                    : "=&s"(keep)
                    : "v"(voff), "s"(dst), "s"(src)
                    : "memory");
            }
            i += nwaves;
        } else {
            i -= per;
            ++r;
            if (r < nrows) {
                rl = __builtin_amdgcn_readlane(len, r);
                per = (rl + 2) / 3;
            }
        }
    }
}

// bytes of the output from element `base` on, as a buffer bound (clamped to 32 bits: a chunk of 64 planes is < 4 GiB)
__device__ __forceinline__ uint32_t out_range(size_t total_bytes, size_t base) {
    const size_t r = total_bytes - base * sizeof(float);
    return r > 0xffffffffull ? 0xffffffffu : (uint32_t)r;
}

#ifndef WARP_TAPS_AHEAD
#define WARP_TAPS_AHEAD 0  // fused warp v2: the next live view's taps computed before the end-of-view wait (1), inside
                           // this view's LDS sampling after group WARP_TAPS_AHEAD - 2 (>= 2), or at its start (0)
#endif
#ifndef WARP_STAGE_ALL
#define WARP_STAGE_ALL 0  // fused warp v2: all live views staged at once when they fit the pool (1, A/B: neutral) or per view (0)
#endif
// LDS bytes of an np-pixel footprint image (17-slot pixels); dma_block rounds to its 1-KiB instructions
#ifndef WARP_CK
#define WARP_CK 64  // fused warp v2 channels per workgroup: 64 (one workgroup per tile and frame) or 32 (A/B: two
                    // workgroups per tile, each staging and sampling every other 32-channel group -- half the LDS image
                    // and accumulator per workgroup, the taps computed twice)
#endif
static_assert(WARP_CK == 64 || WARP_CK == 32, "WARP_CK: 64 or 32");
static_assert(WARP_CK == 64 || WARP_DMA_ROWS == 0, "the row DMA stages 64-channel pixels");
constexpr int V2_SL = WARP_CK / 4 + 1;  // DMA slots of 16 B per staged pixel (WARP_CK channels + pad)
constexpr int V2_SPLIT = 64 / WARP_CK;  // workgroups per (tile, frame)

__device__ __forceinline__ int stage_bytes(int np) {
    return WARP_DMA_ROWS ? np * 272 : ((np * V2_SL + 63) >> 6) * 1024;
}

#ifndef WARP_STORE_AUX
#define WARP_STORE_AUX 2  // fused warp output stores: buffer cache policy (2 = nt, streaming; 0 = default)
#endif
#ifndef WARP_PIPE
#define WARP_PIPE 1  // fused warp v2: LDS sampling software-pipelined by one 4-channel group (1) or not (0)
#endif
#ifndef WARP_STAMP
#define WARP_STAMP 0  // timing builds only (tools/warp_stamps.py): per-workgroup s_memtime stamps of the v2 phases
#endif
#if WARP_STAMP
// per workgroup: [0..4] phases, [5] HW_ID | XCC_ID << 32, [6 + 3 v + k] view v < 6: taps done, sampled, barrier
constexpr int STAMP_N = 24;
__device__ unsigned long long g_warp_stamp[16384 * STAMP_N];
#define STAMP_AT(k)                                                                                          \
    do {                                                                                                     \
        const unsigned sb_ = blockIdx.x + blockIdx.y * gridDim.x;                                            \
        if (threadIdx.x == 0 && sb_ < 16384) g_warp_stamp[sb_ * STAMP_N + (k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#define STAMP(k)                                                                                             \
    do {                                                                                                     \
        STAMP_AT(k);                                                                                         \
        const unsigned sb_ = blockIdx.x + blockIdx.y * gridDim.x;                                            \
        if ((k) == 0 && threadIdx.x == 0 && sb_ < 16384)                                                     \
            g_warp_stamp[sb_ * STAMP_N + 5] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |  \
                                              ((unsigned long long)__builtin_amdgcn_s_getreg((15 << 11) | 20) << 32); \
    } while (0)
#define STAMP_VIEW(n, k) \
    do {                 \
        if ((n) < 6) STAMP_AT(6 + 3 * (n) + (k)); \
    } while (0)
#else
#define STAMP(k) ((void)0)
#define STAMP_VIEW(n, k) ((void)0)
#endif

#ifndef WARP_LANESKIP
#define WARP_LANESKIP 1  // fused warp v2: lanes with no valid tap skip the view's LDS sampling (1, r03 A/B: 1-8 % faster) or read the zero pixel (0)
#endif
// Output stores of a 64-channel chunk through a buffer descriptor: SGPR base of
// the chunk, per-lane byte offset of the cell, SGPR byte offset of the channel
// plane -> no per-store address arithmetic.  The dispatcher guarantees the
// chunk (64 planes) spans < 4 GiB.  aux 2 = nt (streaming, written once).
#ifndef WARP_MEAN_FP32
#define WARP_MEAN_FP32 0  // fused warp v2 mean: Markstein fp32 division for the exhaustively verified V (1, A/B: slower), or div_rcp (0)
#endif
// acc / V for the mean: for V with bit V - 1 of MARKSTEIN_EXACT_V, q0 = a * RN(1/V) and one correction step
// q0 + RN(a - q0 V) * RN(1/V) (two FMAs) is the correctly rounded quotient for every float but -0 (the view sum is
// never -0) -- tools/verify_div_markstein_fix.c, exhaustive over all 2^32 inputs; infinities give NaN in the
// correction, which the fix-up maps back to q0 (= +-inf, the IEEE quotient).  Other V: div_rcp through double.
struct MeanDiv {
    float vf, rf;
    double rV;
    bool fast;
};
__device__ __forceinline__ MeanDiv mean_div_of(int V) {
    MeanDiv m;
    m.vf = (float)V;
    m.rV = recip_uniform(V);
    m.rf = (float)m.rV;
    m.fast = WARP_MEAN_FP32 && V >= 1 && V <= 64 && ((MARKSTEIN_EXACT_V >> (V - 1)) & 1ull);
    return m;
}
__device__ __forceinline__ float mean_div(float a, const MeanDiv &m) {
    if (m.fast) {
        const float q0 = a * m.rf;
        const float q = __builtin_fmaf(__builtin_fmaf(-q0, m.vf, a), m.rf, q0);
        return q != q ? q0 : q;
    }
    return div_rcp(a, m.rV);
}

template <int N>
__device__ __forceinline__ void store_chunk(float *chunk, size_t plane, int voff, const float (&acc)[N], int mode,
                                            const MeanDiv &md, uint32_t range) {
    // range: bytes addressable from `chunk` (the buffer's bound: an offset past it drops the store)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(chunk, 0, (int)range, 0x00020000);
    static_assert(N % 8 == 0, "stores in groups of 8 channels");
    if (WARP_ABLATE & 32) {  // timing only: the same bytes as 1-KiB coalesced 16-B-per-lane stores (wrong layout)
        const int wb = __builtin_amdgcn_readfirstlane(voff) * N;
        const int lane = threadIdx.x & 63;
#pragma unroll
        for (int q = 0; q < N; q += 4) {
            const float4 v = make_float4(acc[q], acc[q + 1], acc[q + 2], acc[q + 3]);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i_t, v), rs, lane * 16, wb + q * 256, 2);
        }
        return;
    }
#pragma unroll
    for (int q0 = 0; q0 < N; q0 += 8) {
        // eight independent divisions, then their stores: the group is pinned after the previous group's
        // stores (no hoisted doubles for all N channels), the chains inside it overlap
        float a[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) a[u] = acc[q0 + u];
        asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]),
                     "+v"(a[7])::"memory");
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const float r = (mode == BEV_FUSE_MEAN && !(WARP_ABLATE & 1)) ? mean_div(a[u], md) : a[u];
            if ((WARP_ABLATE & 16) && r != 1.2345e-30f) continue;
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, r), rs, voff,
                                                  (int)(uint32_t)((q0 + u) * plane * sizeof(float)),
                                                  WARP_STORE_AUX);
        }
    }
}

// Footprint bbox of the workgroup for one view (wave partials -> red[] -> block).
struct Box {
    int x0, y0, x1, y1;
};

// Packed (x, y) 16-bit pairs: min of (x0, y0) and min of (-x1, -y1) -> 2 shuffles per step.
typedef short short2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int pk_min(int a, int b) {
    short2_t x = __builtin_bit_cast(short2_t, a), y = __builtin_bit_cast(short2_t, b);
    return __builtin_bit_cast(int, __builtin_elementwise_min(x, y));
}

__device__ __forceinline__ int pk2(int lo, int hi) { return (lo & 0xffff) | (hi << 16); }
__device__ __forceinline__ int pk_lo(int v) { return (int)(short)(v & 0xffff); }
__device__ __forceinline__ int pk_hi(int v) { return v >> 16; }

__device__ __forceinline__ Box wave_box(const Taps &t) {
    // sentinels: x0/y0 -> 32767, -x1/-y1 -> 32767 (empty); coordinates are < 2^14
    int mn = pk2(32767, 32767), mx = pk2(32767, 32767);
    if (t.valid) {
        const int x0 = (t.valid & 5) ? t.x0 : t.x0 + 1, x1 = (t.valid & 10) ? t.x0 + 1 : t.x0;
        const int y0 = (t.valid & 3) ? t.y0 : t.y0 + 1, y1 = (t.valid & 12) ? t.y0 + 1 : t.y0;
        mn = pk2(x0, y0);
        mx = pk2(-x1, -y1);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mn = pk_min(mn, __shfl_xor(mn, o));
        mx = pk_min(mx, __shfl_xor(mx, o));
    }
    Box b;
    if (pk_lo(mn) == 32767) {
        b = Box{0x7fffffff, 0x7fffffff, -1, -1};
    } else {
        b = Box{pk_lo(mn), pk_hi(mn), -pk_lo(mx), -pk_hi(mx)};
    }
    return b;
}

template <int NW = 4>
__device__ __forceinline__ void put_box(int *rp, const Box &b, int wave, int lane) {
    if (lane == 0) {
        rp[wave] = b.x0;
        rp[NW + wave] = b.y0;
        rp[2 * NW + wave] = b.x1;
        rp[3 * NW + wave] = b.y1;
    }
}

template <int NW = 4>
__device__ __forceinline__ Box get_box(const int *rp) {
    Box b{rp[0], rp[NW], rp[2 * NW], rp[3 * NW]};
#pragma unroll
    for (int w = 1; w < NW; ++w) {
        b.x0 = min(b.x0, rp[w]);
        b.y0 = min(b.y0, rp[NW + w]);
        b.x1 = max(b.x1, rp[2 * NW + w]);
        b.y1 = max(b.y1, rp[3 * NW + w]);
    }
    b.x0 = __builtin_amdgcn_readfirstlane(b.x0);
    b.y0 = __builtin_amdgcn_readfirstlane(b.y0);
    b.x1 = __builtin_amdgcn_readfirstlane(b.x1);
    b.y1 = __builtin_amdgcn_readfirstlane(b.y1);
    return b;
}

// Sample one view for the lanes with `mine` from an image at LDS byte offset
// `ib` (origin sx0, sy0, width sbw); invalid taps read the zero pixel `zp`.
template <int MODE, int WIN, int N = 64>
__device__ __forceinline__ void sample_view(float (&acc)[N], const Taps &t, bool mine, int v,
                                            const unsigned char *smem, int ib, int sx0, int sy0, int sbw, int zp) {
    constexpr int PS = (N / 4 + 1) * 16;  // staged pixel stride (N channels + one pad slot)
    const int pb = ib + ((t.y0 - sy0) * sbw + (t.x0 - sx0)) * PS;
    const unsigned char *a0 = smem + ((mine && (t.valid & 1)) ? pb : zp);
    const unsigned char *a1 = smem + ((mine && (t.valid & 2)) ? pb + PS : zp);
    const unsigned char *a2 = smem + ((mine && (t.valid & 4)) ? pb + sbw * PS : zp);
    const unsigned char *a3 = smem + ((mine && (t.valid & 8)) ? pb + (sbw + 1) * PS : zp);
#pragma unroll
    for (int g = 0; g < N / 4; ++g) {
        const float4 vnw = *(const float4 *)(a0 + g * 16);
        const float4 vne = *(const float4 *)(a1 + g * 16);
        const float4 vsw = *(const float4 *)(a2 + g * 16);
        const float4 vse = *(const float4 *)(a3 + g * 16);
        const float sm[4] = {bilerp(vnw.x, vne.x, vsw.x, vse.x, t.w), bilerp(vnw.y, vne.y, vsw.y, vse.y, t.w),
                             bilerp(vnw.z, vne.z, vsw.z, vse.z, t.w), bilerp(vnw.w, vne.w, vsw.w, vse.w, t.w)};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            float &a = acc[4 * g + u];
            const float r = (MODE == BEV_FUSE_MAX) ? nan_max(a, sm[u]) : a + sm[u];
            a = mine ? r : a;
        }
        if ((g % WIN) == WIN - 1) __builtin_amdgcn_sched_barrier(0);  // bound LDS-read lookahead
    }
}

template <int MODE, int N>
__device__ __forceinline__ void zero_view(float (&acc)[N], int v) {
    if (MODE == BEV_FUSE_MAX) {
#pragma unroll
        for (int q = 0; q < N; ++q) acc[q] = nan_max(acc[q], 0.0f);
    }
}

// -------------------------------------------------------------------------
// fused warp + reduce v2: corner-bounded footprints (default DMA path)
// -------------------------------------------------------------------------
// Same tile, lane mapping, LDS image layout, ring and block decomposition as
// k_warp_fuse_dma; what changes is how a (tile, view) footprint is found and
// therefore the per-view critical path.  The image of the tile's cell-centre
// rectangle under x -> (H x)_{0,1} / (H x)_2 is a convex quadrilateral whenever
// w = (H x)_2 keeps one sign on it, so the bilinear taps of every cell lie in
// the bbox of the four corner projections widened by a bound on the fp32
// rounding of the tap recipe.  Every wave computes that box for all views at
// once (lane v -> view v, in double) and reads it back with readlane: no
// cross-lane bbox reduction, no LDS exchange, and a view whose box misses the
// feature map costs no tap arithmetic at all.  Tiles where the bound does not
// apply (w may change sign or come near the 1e-6 clamp of geometry.py:147)
// take the exact per-cell reduction of k_warp_fuse_dma for that view.
// Per view:  [stage synchronously if it did not fit] -> issue LDS-DMA of
// view v+1 -> taps of view v -> software-pipelined LDS sampling (the next 4
// channels' four ds_read_b128 are in flight during this group's FMAs) ->
// vmcnt(0) + one barrier.
constexpr double EPS32 = 5.9604644775390625e-08;  // 2^-24
// Footprint-box workspace: a 16-B header {BOX_MAGIC, maxpix, V, TH} (the fit test and tiling the boxes were made
// for, written by k_warp_boxes) and then the boxes.  The fused kernel checks the header and, on a mismatch (boxes
// made for another mode's pool, another pool knob, another V or tile shape), ignores the boxes and computes its own.
constexpr unsigned BOX_MAGIC = 0x42455642u;  // "BVEB"
constexpr int BOX_HDR = 16;                   // header bytes before the boxes
constexpr int V2_MAXV = 64;                         // one view per lane
constexpr int WQ_WORDS = 16;  // queue words after the boxes: [0..7] tickets per queue, [8] finished workgroups
// Span tables after the queue words ([frame][tile][view][SPAN_ROWS] words, written for the views flagged span-staged:
// box word a, bit 30).  Header word w = TH | SPAN_FLAG when k_warp_boxes made them.
constexpr int SPAN_ROWS = 32;          // span staging applies to boxes of at most this many rows
constexpr int SPAN_HDR = 144;          // LDS bytes before a span-staged image: the row bases of rows -1 .. 32 (34 ints)
constexpr unsigned SPAN_FLAG = 0x100u;
#ifndef WARP_SPAN_PCT
#define WARP_SPAN_PCT 0  // fused warp v2, BEV_TUNE_WARP_SPAN's default: a footprint that fits the pool as a box is
                         // span-staged when its spans need at most this percentage of the box's pixels (oversized boxes
                         // always); 0 = span staging off (default: the span pass costs k_warp_boxes 5-8 us per
                         // launch, as much as it saves the fused kernel on K5 -- profiles/r06at_warp_span_staging.txt)
#endif

// The projected corners of the BEV rectangle (image coordinates, order: c & 1 -> xb, c & 2 -> yb) and the fp32
// margins of the tap recipe, for the per-row spans (row_spans).
struct Quad {
    double x[4], y[4], mx, my;
    double s[4];  // dx / dy of polygon edge e (corner ord[e] -> ord[e + 1]; 0 for a horizontal edge): quad_slopes
};
constexpr int QUAD_ORD[4] = {0, 1, 3, 2};  // the corners in polygon order

__device__ __forceinline__ void quad_slopes(Quad &q) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int a = QUAD_ORD[e], c = QUAD_ORD[(e + 1) & 3];
        q.s[e] = q.y[a] != q.y[c] ? (q.x[c] - q.x[a]) / (q.y[c] - q.y[a]) : 0.0;
    }
}

// Conservative tap bbox of the BEV rectangle [xa, xb] x [ya, yb] (cell
// centres) for homography h; ok = false when the corner bound does not apply.
__device__ Box corner_box(const float *hf, float xa, float xb, float ya, float yb, float sx, float sy, int Wf, int Hf,
                          bool &ok, Quad *quad = nullptr) {
    double h[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) h[q] = (double)hf[q];
    double ixmin = __builtin_inf(), ixmax = -__builtin_inf(), iymin = __builtin_inf(), iymax = -__builtin_inf();
    double wmin = __builtin_inf(), swmax = 0.0, sumax = 0.0, svmax = 0.0, umax = 0.0, vmax = 0.0, aix = 0.0, aiy = 0.0;
    int npos = 0, nneg = 0;
    bool fin = true;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const double x = (double)((c & 1) ? xb : xa), y = (double)((c & 2) ? yb : ya);
        const double a0 = h[0] * x, a1 = h[1] * y, b0 = h[3] * x, b1 = h[4] * y, c0 = h[6] * x, c1 = h[7] * y;
        const double u = a0 + a1 + h[2], v = b0 + b1 + h[5], w = c0 + c1 + h[8];
        sumax = fmax(sumax, fabs(a0) + fabs(a1) + fabs(h[2]));
        svmax = fmax(svmax, fabs(b0) + fabs(b1) + fabs(h[5]));
        swmax = fmax(swmax, fabs(c0) + fabs(c1) + fabs(h[8]));
        npos += w > 0.0;
        nneg += w < 0.0;
        wmin = fmin(wmin, fabs(w));
        double rw = __builtin_amdgcn_rcp(w);  // + one Newton step: ~1e-15 relative, far inside the margin
        rw = rw * (2.0 - w * rw);
        const double U = u * rw, Vv = v * rw;
        const double ix = U * (double)sx, iy = Vv * (double)sy;
        fin = fin && __builtin_isfinite(ix) && __builtin_isfinite(iy) && __builtin_isfinite(w);
        umax = fmax(umax, fabs(U));
        vmax = fmax(vmax, fabs(Vv));
        aix = fmax(aix, fabs(ix));
        aiy = fmax(aiy, fabs(iy));
        if (quad) {
            quad->x[c] = ix;
            quad->y[c] = iy;
        }
        ixmin = fmin(ixmin, ix);
        ixmax = fmax(ixmax, ix);
        iymin = fmin(iymin, iy);
        iymax = fmax(iymax, iy);
    }
    ok = fin && (npos == 4 || nneg == 4) && wmin > 1e-6 + 4.0 * EPS32 * swmax;
    Box b{0x7fffffff, 0x7fffffff, -1, -1};
    if (!ok) return b;
    // |fp32 tap coordinate - exact| <= (dot3 error + division) / |w| + normalisation steps; x4 safety
    const double mx = 4.0 * ((double)sx * 3.0 * EPS32 * (sumax + umax * swmax) / wmin +
                             16.0 * EPS32 * (aix + (double)Wf + 1.0)) + 1e-3;
    const double my = 4.0 * ((double)sy * 3.0 * EPS32 * (svmax + vmax * swmax) / wmin +
                             16.0 * EPS32 * (aiy + (double)Hf + 1.0)) + 1e-3;
    if (quad) {
        quad->mx = mx;
        quad->my = my;
    }
    const double lox = fmin(fmax(ixmin - mx, -4.0), (double)Wf + 4.0);
    const double hix = fmin(fmax(ixmax + mx, -4.0), (double)Wf + 4.0);
    const double loy = fmin(fmax(iymin - my, -4.0), (double)Hf + 4.0);
    const double hiy = fmin(fmax(iymax + my, -4.0), (double)Hf + 4.0);
    const int x0 = max((int)floor(lox), 0), x1 = min((int)floor(hix) + 1, Wf - 1);
    const int y0 = max((int)floor(loy), 0), y1 = min((int)floor(hiy) + 1, Hf - 1);
    if (x0 <= x1 && y0 <= y1) b = Box{x0, y0, x1, y1};
    return b;
}

// Span of box row r (image row bx.y0 + r) of box bx (span table word: x0 | len << 16; 0: no tap of the tile there).
// A cell puts taps on row y iff its fp32 iy is in [y - 1, y + 1), so its exact iy (a point of the quad) is in the
// band [y - 1 - my, y + 1 + my]; the exact ix of such cells lies in the x extent [lo, hi] of the quad's part inside
// that band (a convex polygon: its vertices inside the band and its edges' crossings of the band's lines), so their
// fp32 ix is in [lo - mx, hi + mx] and their tap columns in [floor(lo - mx), floor(hi + mx) + 1] -- clipped to the
// (conservative) box.  Every valid tap of the tile on row y lies in the span.  Evaluated in fp32 relative to the box
// origin (QuadF): the corners, slopes and margins are rounded once, and the margins widened by 1e-2 pixel plus a
// bound on fp32 rounding at the corners' magnitude -- far above the error of the few fp32 operations per row.
struct QuadF {
    float x[4], y[4], s[4], mx, my;
};
__device__ __forceinline__ QuadF quad_f(const Quad &q, const Box &bx) {
    QuadF f;
    double amax = 0.0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const double x = q.x[c] - (double)bx.x0, y = q.y[c] - (double)bx.y0;
        f.x[c] = (float)x;
        f.y[c] = (float)y;
        amax = fmax(amax, fmax(fabs(x), fabs(y)));
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) f.s[e] = (float)q.s[e];
    const double extra = 1e-2 + 1e-6 * amax;
    f.mx = (float)(q.mx + extra);
    f.my = (float)(q.my + extra);
    return f;
}
__device__ __forceinline__ unsigned row_span(const QuadF &q, const Box &bx, int r) {
    const float lo = (float)r - 1.0f - q.my, hi = (float)r + 1.0f + q.my;
    float xl = __builtin_inff(), xh = -__builtin_inff();
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const float px = q.x[QUAD_ORD[e]], py = q.y[QUAD_ORD[e]], qy = q.y[QUAD_ORD[(e + 1) & 3]];
        if (py >= lo && py <= hi) {
            xl = fminf(xl, px);
            xh = fmaxf(xh, px);
        }
        if (py != qy) {
            const float s = q.s[e];
            if ((lo - py) * (lo - qy) <= 0.0f) {
                const float x = px + (lo - py) * s;
                xl = fminf(xl, x);
                xh = fmaxf(xh, x);
            }
            if ((hi - py) * (hi - qy) <= 0.0f) {
                const float x = px + (hi - py) * s;
                xl = fminf(xl, x);
                xh = fmaxf(xh, x);
            }
        }
    }
    if (!(xl <= xh)) return 0u;
    const int bw = bx.x1 - bx.x0;  // relative box columns 0 .. bw
    const float l = fminf(fmaxf(xl - q.mx, -1.0f), (float)bw + 2.0f);
    const float h = fmaxf(fminf(xh + q.mx, (float)bw + 1.0f), -2.0f);
    const int x0 = max((int)floorf(l), 0), x1 = min((int)floorf(h) + 1, bw);
    return x0 <= x1 ? (unsigned)(x0 + bx.x0) | ((unsigned)(x1 - x0 + 1) << 16) : 0u;
}

// bilerp (bev_geometry.h) of 4 channels as two independent packed chains,
// written in interleaved order so that no packed op waits on its predecessor
// (a dependent v_pk_* pair needs a wait state): per element exactly
// fma(se, wse, fma(sw, wsw, fma(ne, wne, nw * wnw))), then acc + s / max.
typedef float f32x2 __attribute__((ext_vector_type(2)));
template <int MODE, int N>
__device__ __forceinline__ void bilerp4(float (&acc)[N], int q0, const f32x4 &nw, const f32x4 &ne, const f32x4 &sw,
                                        const f32x4 &se, const float w[4]) {
    const f32x2 w0 = (f32x2){w[0], w[0]}, w1 = (f32x2){w[1], w[1]}, w2 = (f32x2){w[2], w[2]},
                w3 = (f32x2){w[3], w[3]};
    f32x2 a = nw.xy * w0, b = nw.zw * w0;
    a = __builtin_elementwise_fma(ne.xy, w1, a);
    b = __builtin_elementwise_fma(ne.zw, w1, b);
    a = __builtin_elementwise_fma(sw.xy, w2, a);
    b = __builtin_elementwise_fma(sw.zw, w2, b);
    a = __builtin_elementwise_fma(se.xy, w3, a);
    b = __builtin_elementwise_fma(se.zw, w3, b);
    if (MODE == BEV_FUSE_MAX) {
        acc[q0] = nan_max(acc[q0], a.x);
        acc[q0 + 1] = nan_max(acc[q0 + 1], a.y);
        acc[q0 + 2] = nan_max(acc[q0 + 2], b.x);
        acc[q0 + 3] = nan_max(acc[q0 + 3], b.y);
    } else {
        f32x2 s0 = (f32x2){acc[q0], acc[q0 + 1]}, s1 = (f32x2){acc[q0 + 2], acc[q0 + 3]};
        s0 = s0 + a;
        s1 = s1 + b;
        acc[q0] = s0.x;
        acc[q0 + 1] = s0.y;
        acc[q0 + 2] = s1.x;
        acc[q0 + 3] = s1.y;
    }
}

// LDS sampling of one view, software-pipelined by one 4-channel group (PIPE; else
// each group's reads are issued right before its use -- fewer live registers, the
// max reduction's choice).  Invalid taps read the zero pixel `zp` (the nw tap: `zp0`,
// see k_warp_fuse_pc's blocked views).
struct NoMid {
    __device__ __forceinline__ void operator()() const {}
};
// `mid` runs between LDS groups MID_G and MID_G + 1 (the next view's taps while this view's reads are in flight)
// (the taps' LDS pixels: (x0, y0) at byte pb, (x0, y0 + 1) at byte pbs, each row's x0 + 1 one pixel further)
template <int MODE, int N, bool PIPE = true, int MID_G = -1, class Mid = NoMid>
__device__ __forceinline__ void sample_pipe_at(float (&acc)[N], const Taps &t, const unsigned char *smem, int pb,
                                               int pbs, int zp, int zp0, Mid mid = Mid()) {
    constexpr int PS = (N / 4 + 1) * 16, NG = N / 4;
    const unsigned char *a0 = smem + ((t.valid & 1) ? pb : zp0);
    const unsigned char *a1 = smem + ((t.valid & 2) ? pb + PS : zp);
    const unsigned char *a2 = smem + ((t.valid & 4) ? pbs : zp);
    const unsigned char *a3 = smem + ((t.valid & 8) ? pbs + PS : zp);
    if (!PIPE) {
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const f32x4 c0 = *(const f32x4 *)(a0 + g * 16), c1 = *(const f32x4 *)(a1 + g * 16);
            const f32x4 c2 = *(const f32x4 *)(a2 + g * 16), c3 = *(const f32x4 *)(a3 + g * 16);
            bilerp4<MODE>(acc, 4 * g, c0, c1, c2, c3, t.w);
            if (g == MID_G) mid();
            __builtin_amdgcn_sched_barrier(0);
        }
        return;
    }
    f32x4 c0 = *(const f32x4 *)a0, c1 = *(const f32x4 *)a1, c2 = *(const f32x4 *)a2, c3 = *(const f32x4 *)a3;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        f32x4 n0, n1, n2, n3;
        if (g < NG - 1) {
            n0 = *(const f32x4 *)(a0 + (g + 1) * 16);
            n1 = *(const f32x4 *)(a1 + (g + 1) * 16);
            if (WARP_ABLATE & 128) {  // timing only: half the LDS reads, the same arithmetic
                n2 = n0;
                n3 = n1;
            } else {
                n2 = *(const f32x4 *)(a2 + (g + 1) * 16);
                n3 = *(const f32x4 *)(a3 + (g + 1) * 16);
            }
        }
        if ((WARP_ABLATE & 256) && (g & 1)) {  // timing only: half the arithmetic, the same LDS reads
            acc[4 * g] += c0.x + c1.y + c2.z + c3.w;
        } else
        bilerp4<MODE>(acc, 4 * g, c0, c1, c2, c3, t.w);
        if (g == MID_G) mid();
        __builtin_amdgcn_sched_barrier(0);  // at most two groups of reads in flight
        if (g < NG - 1) {
            c0 = n0;
            c1 = n1;
            c2 = n2;
            c3 = n3;
        }
    }
}

// ... from a box image at LDS byte `ib` (origin sx0, sy0, width sbw)
template <int MODE, int N, bool PIPE = true, int MID_G = -1, class Mid = NoMid>
__device__ __forceinline__ void sample_view_pipe(float (&acc)[N], const Taps &t, const unsigned char *smem, int ib,
                                                 int sx0, int sy0, int sbw, int zp, int zp0, Mid mid = Mid()) {
    constexpr int PS = (N / 4 + 1) * 16;
    const int pb = ib + ((t.y0 - sy0) * sbw + (t.x0 - sx0)) * PS;
    sample_pipe_at<MODE, N, PIPE, MID_G, Mid>(acc, t, smem, pb, pb + sbw * PS, zp, zp0, mid);
}

// Tile shapes of k_warp_fuse_v2 (TH rows x TW cells, 256 lanes, one cell per lane):
//   TH = 8:  8 x 32, wave w owns rows 2w, 2w + 1 (lanes 0-31 / 32-63): every output store is two full 128-B lines;
//   TH = 16: 16 x 16, wave w owns rows 4w .. 4w + 3 and each of the four ds_read_b128 lane groups of a wave
//            ({0-3,12-15,20-27}, {4-11,16-19,28-31} and the same +32, MI355X_MICROARCH §LDS) is ONE row of 16
//            cells, so the lanes that can bank-conflict sample neighbouring cells of one BEV row; stores are
//            64-B row segments.  A square tile's footprint is smaller: on the Appendix-B rig (7 cams, 1080p,
//            480 x 1440) 0.61 staged pixels per cell against 0.81 (tools/ model in DESIGN.md §4).
template <int TH>
__device__ __forceinline__ void tile_cell(int lane, int wave, int &r, int &c) {
    if (TH == 8) {
        r = wave * 2 + (lane >> 5);
        c = lane & 31;
    } else {
        const int lp = lane & 31;
        const bool gb = (lp >= 4 && lp < 12) || (lp >= 16 && lp < 20) || lp >= 28;
        c = gb ? (lp < 12 ? lp - 4 : (lp < 20 ? lp - 8 : lp - 16)) : (lp < 4 ? lp : (lp < 16 ? lp - 8 : lp - 12));
        r = wave * 4 + 2 * (lane >> 5) + (gb ? 1 : 0);
    }
}

template <int MODE, int OCC, int TH = 8, bool CHUNK = false, bool NHWC = false>
__global__ __launch_bounds__(FT_NT, OCC) void k_warp_fuse_v2(const float *__restrict__ feats, int64_t sN, int64_t sH,
                                                          int64_t sW, const float *__restrict__ Hmat,
                                                          const float *__restrict__ xs, const float *__restrict__ ys,
                                                          int B, int V, int C, int Hf, int Wf, float sx, float sy,
                                                          int Hb, int Wb, float *__restrict__ out, int pool,
                                                          const uint2 *__restrict__ boxes_in, int rpr, int tband) {
    constexpr int NW = FT_NT / 64;  // 4 waves
    constexpr int TW = FT_NT / TH;  // tile width in cells
    constexpr int CK = WARP_CK, SL = V2_SL, PS = SL * 16;  // channels / DMA slots / bytes per staged pixel (+ pad)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int zp = pool;                                    // zero pixel (256 B)
    int *red = reinterpret_cast<int *>(smem + pool + 256);  // [4 * NW] exact-bbox exchange
    float *htab = reinterpret_cast<float *>(smem + pool + 256 + 4 * NW * sizeof(int));  // [V][9] homographies
    const int maxpix = pool / PS - 4;                      // ~1 KiB DMA rounding slack

    const int ntx = (Wb + TW - 1) / TW, nty = (Hb + TH - 1) / TH, nt = ntx * nty;
    int tile = blockIdx.x;
    {
        const int q = nt / 8, r = nt % 8, x = tile % 8;
        tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + tile / 8;
    }
    if (tband > 1) {  // order index -> tile: bands of tband tile rows walked column by column (BEV_TUNE_WARP_TILE_BAND)
        const int band = tile / (tband * ntx), k = tile - band * (tband * ntx);
        const int bh = min(tband, nty - band * tband);
        tile = (band * tband + k % bh) * ntx + k / bh;
    }
    const int tyb = tile / ntx, txb = tile - tyb * ntx;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    STAMP(0);
    int tr, tc;
    tile_cell<TH>(lane, wave, tr, tc);
    auto dma = [&](const float *fp, int x0, int y0, int w, int h, int o) {
        if (WARP_DMA_ROWS) dma_rows(fp, (int)sH, (int)sW, x0, y0, w, h, smem, o, wave, lane, NW);
        else dma_block<SL>(fp, (int)sH, (int)sW, x0, y0, w, w * h, smem, o, wave, lane, NW);
    };
    const int i = tyb * TH + tr;
    const int j = txb * TW + tc;
    const int b = V2_SPLIT == 1 ? (int)blockIdx.y : (int)blockIdx.y / V2_SPLIT;
    const int cfirst = V2_SPLIT == 1 ? 0 : ((int)blockIdx.y % V2_SPLIT) * CK;  // this workgroup's first channel
    const bool inside = (i < Hb) && (j < Wb);
    const float cx = xs[inside ? j : 0], cy = ys[inside ? i : 0];
    const size_t plane = (size_t)Hb * Wb;
    // output layout: [B][C][Hb][Wb] (rpr == Hb), or rank-chunk-major [ceil(Hb / rpr)][B][C][rpr][Wb] for the camera-shard
    // reduce-scatter (BEV row r -> chunk r / rpr, its row r % rpr); the chunk is a per-lane byte offset (the launcher
    // checks the whole output is < 2 GiB), the (frame, channel) base and the channel plane stay uniform
    // (CHUNK only: the plain layout keeps the round-4 addressing -- no extra live registers in the default kernel)
    const size_t oplane = CHUNK ? (size_t)rpr * Wb : plane;
    auto store_out = [&](int c0, const float (&acc)[CK], const MeanDiv &md) {
        if (!CHUNK) {
            store_chunk(out + ((size_t)b * C + c0) * plane, plane, (i * Wb + j) * (int)sizeof(float), acc, MODE, md,
                        (uint32_t)(plane * CK * sizeof(float)));
            return;
        }
        const int ck = i / rpr;
        const int ovoff = (int)(((size_t)ck * B * C * oplane + (size_t)(i - ck * rpr) * Wb + j) * sizeof(float));
        const size_t orange = (size_t)((Hb + rpr - 1) / rpr) * B * C * oplane * sizeof(float);  // whole output
        store_chunk(out + ((size_t)b * C + c0) * oplane, oplane, ovoff, acc, MODE, md,
                    out_range(orange, ((size_t)b * C + c0) * oplane));
    };
    // NHWC: channels-last output [B][Hb][Wb][C] (bev_ipm_warp_fuse_nhwc_f32).  A cell's C values are one contiguous
    // run, so a wave's 4 x 16 (TH 16) cells are 4 row runs of 16 x C floats: each lane parks its 32-channel half in
    // the (free) pool, and the wave writes it back 16 B per lane, 8 cells x 128 B (whole cache lines) per store --
    // 1 KiB per instruction instead of the NCHW layout's 64-B row segments per channel plane
    // (tools/store_pattern_micro.hip: 65.5 vs 104.5 us for the 354 MB of a batch-2 launch).  Same values.
    auto store_nhwc = [&](int c0, const float (&acc)[CK], const MeanDiv &md) {
        constexpr int RW = TH / NW, NS = 36;  // rows per wave; floats per parked cell (32 + 4 pad)
        __syncthreads();                      // every wave is done with the pool
        float *stg = reinterpret_cast<float *>(smem) + wave * 64 * NS;
        const int cl = (tr - wave * RW) * TW + tc;  // this lane's cell among the wave's 64
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            out + (size_t)b * plane * C, 0, (int)(uint32_t)(plane * C * sizeof(float)), 0x00020000);
#pragma unroll
        for (int hh = 0; hh < CK / 32; ++hh) {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                // four divisions at a time, pinned after the previous group's LDS write (as store_chunk groups its
                // divisions): no hoisted doubles for all 64 channels, no spills
                float v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = acc[32 * hh + 4 * q + u];
                asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3])::"memory");
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (MODE == BEV_FUSE_MEAN && !(WARP_ABLATE & 1)) v[u] = mean_div(v[u], md);
                *reinterpret_cast<float4 *>(stg + cl * NS + 4 * q) = make_float4(v[0], v[1], v[2], v[3]);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int cc = 8 * k + (lane >> 3), pc = lane & 7;
                const float4 v = *reinterpret_cast<const float4 *>(stg + cc * NS + 4 * pc);
                const int gi = tyb * TH + wave * RW + cc / TW, gj = txb * TW + cc % TW;
                if (gi < Hb && gj < Wb)
                    __builtin_amdgcn_raw_buffer_store_b128(
                        __builtin_bit_cast(v4i_t, v), rs,
                        (int)((((size_t)gi * Wb + gj) * C + c0 + 32 * hh) * sizeof(float)) + pc * 16, 0, WARP_STORE_AUX);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        if (c0 + CK < C) __syncthreads();  // the next chunk stages into the pool
    };
    const Grid grid = make_grid(Hf, Wf);
    const MeanDiv md = mean_div_of(V);  // mean: acc / V (exact)
    if (tid < 16) *(float4 *)(smem + zp + tid * 16) = make_float4(0.f, 0.f, 0.f, 0.f);
    unsigned *btab = reinterpret_cast<unsigned *>(htab + V2_MAXV * 9);  // [V][2] corner boxes
    bool box_hdr_ok = false;  // boxes made for this kernel's fit test and tiling? (else: computed here)
    bool span_ok = false;     // ... and span tables for the views flagged span-staged
    if (boxes_in != nullptr) {
        const uint4 hd = reinterpret_cast<const uint4 *>(boxes_in)[-1];
        box_hdr_ok = hd.x == BOX_MAGIC && (int)hd.y == maxpix && (int)hd.z == V && (int)(hd.w & ~SPAN_FLAG) == TH;
        span_ok = box_hdr_ok && (hd.w & SPAN_FLAG) && CK == 64 && WARP_HSCALAR && !WARP_STAGE_ALL;
    }
    const uint2 *__restrict__ boxes = box_hdr_ok ? boxes_in : nullptr;
    const unsigned *__restrict__ spans =
        span_ok ? reinterpret_cast<const unsigned *>(boxes_in + (int64_t)B * nt * V) + WQ_WORDS : nullptr;

    // corner boxes of this tile for frame bb, lane v <-> view v, packed in two VGPRs (wave 0 computes them in
    // double, the others read them): lba = x0 | y0 << 16 | (!ok) << 31,  lbb = (x1 + 1) | (y1 + 1) << 16
    // (x1 + 1 == 0: empty).
    unsigned lba = 0, lbb = 0;
    auto prologue = [&](int bb) {
        if (WARP_HSCALAR && boxes != nullptr) {  // precomputed by k_warp_boxes: every wave reads them
            const uint2 bx = lane < V ? boxes[((int64_t)bb * nt + tile) * V + lane] : make_uint2(0u, 0u);
            lba = bx.x;
            lbb = bx.y;
            return;
        }
        if (wave == 0) {
            const int ia = tyb * TH, ib = min(ia + TH - 1, Hb - 1);
            const int ja = txb * TW, jb = min(ja + TW - 1, Wb - 1);
            Box cb{0x7fffffff, 0x7fffffff, -1, -1};
            bool ok = true;
            if (lane < V) {
                float hv[9];
                load_h(Hmat, bb * V + lane, hv);
#pragma unroll
                for (int q = 0; q < 9; ++q) htab[lane * 9 + q] = hv[q];  // visible after the barrier below
                cb = corner_box(hv, xs[ja], xs[jb], ys[ia], ys[ib], sx, sy, Wf, Hf, ok);
                // large footprints: the exact per-cell box (usually much smaller near the
                // horizon, where adjacent cell rows map far apart) decides the staging
                if (ok && cb.x1 >= 0 && (cb.x1 - cb.x0 + 1) * (cb.y1 - cb.y0 + 1) > maxpix) ok = false;
            }
            const bool emp = cb.x1 < 0;
            if (lane < V) {
                btab[2 * lane] = (emp ? 0u : (unsigned)cb.x0 | ((unsigned)cb.y0 << 16)) | (ok ? 0u : 0x80000000u);
                btab[2 * lane + 1] = emp ? 0u : (unsigned)(cb.x1 + 1) | ((unsigned)(cb.y1 + 1) << 16);
            }
        }
        __syncthreads();
        lba = lane < V ? btab[2 * lane] : 0u;
        lbb = lane < V ? btab[2 * lane + 1] : 0u;
    };
    prologue(b);
    STAMP(1);
    auto box_of = [&](int v) {
        const unsigned a = (unsigned)__builtin_amdgcn_readlane((int)lba, v);
        const unsigned c = (unsigned)__builtin_amdgcn_readlane((int)lbb, v);
        return Box{(int)(a & 0xffffu), (int)((a >> 16) & 0x3fffu), (int)(c & 0xffffu) - 1, (int)(c >> 16) - 1};
    };
    auto ok_of = [&](int v) { return ((unsigned)__builtin_amdgcn_readlane((int)lba, v) >> 31) == 0u; };
    auto span_of = [&](int v) {
        return spans != nullptr && ((unsigned)__builtin_amdgcn_readlane((int)lba, v) & 0x40000000u) != 0u;
    };
    // span table of view v (lane r < SPAN_ROWS: row r's word) -- a plain load, consumed (and so waited for by the
    // compiler) only after an explicit vmcnt(0), so its wait never covers LDS-DMA still in flight
    auto load_span = [&](int v) -> unsigned {
        return lane < SPAN_ROWS ? spans[(((int64_t)b * nt + tile) * V + v) * SPAN_ROWS + lane] : 0u;
    };
    // span staging of a view (box rows y0 .. y0 + nrows - 1, table spw) at LDS byte o: the row bases first (wave 0:
    // int [34] for rows -1 .. 32, absolute LDS pixel-0 offsets, read by the sampling after the end-of-view barrier),
    // then the rows' pixels from o + SPAN_HDR.  span_bytes: the LDS bytes it takes.
    auto span_scan = [&](unsigned spw, int nrows, int &len, int &sxr, int &exc) {
        len = lane < nrows ? (int)(spw >> 16) : 0;
        sxr = (int)(spw & 0xffffu);
        int inc = len;
#pragma unroll
        for (int d = 1; d < SPAN_ROWS; d <<= 1) {
            const int u = __shfl_up(inc, d);
            if (lane >= d) inc += u;
        }
        exc = inc - len;
        return SPAN_HDR + __builtin_amdgcn_readlane(inc, SPAN_ROWS - 1) * PS;
    };
    auto stage_span = [&](const float *fp, int y0, int nrows, int len, int sxr, int exc, int o) {
        const int rb = __shfl(exc - sxr, lane > 0 ? lane - 1 : 0);  // lane l: row l - 1's pixel of column 0
        if (wave == 0 && lane < SPAN_ROWS + 2)
            reinterpret_cast<int *>(smem + o)[lane] = o + SPAN_HDR + ((lane >= 1 && lane <= nrows) ? rb * PS : 0);
        dma_spans(fp, (int)sH, (int)sW, y0, nrows, len, sxr, exc, smem, o + SPAN_HDR, wave, lane, NW);
    };
    // the taps' LDS pixels (sample_pipe_at) in a span image at o (box origin row y0) or a box image (origin, width)
    auto span_addr = [&](const Taps &t, int o, int y0, int &pb, int &pbs) {
        const int *hdr = reinterpret_cast<const int *>(smem + o);
        const int r0 = min(max(t.y0 - y0 + 1, 0), SPAN_ROWS + 1), r1 = min(r0 + 1, SPAN_ROWS + 1);
        pb = hdr[r0] + t.x0 * PS;
        pbs = hdr[r1] + t.x0 * PS;
    };

    float ccx = cx, ccy = cy;  // made opaque per chunk (see the chunk loop)
    const int hbase = b * V;   // homography row of view 0 of this frame
    auto taps_of = [&](int v) {
        Taps t;
        float h[9];
#pragma unroll
        for (int q = 0; q < 9; ++q) {  // wave-uniform address: scalar loads (no LDS cycles on the sampling path)
#if WARP_HSCALAR
            h[q] = Hmat[__builtin_amdgcn_readfirstlane((hbase + v) * 9) + q];
#else
            h[q] = htab[v * 9 + q];
#endif
        }
        float ix, iy;
        cell_ixy(h, ccx, ccy, grid, sx, sy, ix, iy);
        t = taps_from_ixy(ix, iy, grid);
        if (WARP_ABLATE & 8) {
            const Box bb = box_of(v);
            t.x0 = bb.x0 + (lane & 1);
            t.y0 = bb.y0;
            t.valid = (bb.x1 > bb.x0 + 1 && bb.y1 > bb.y0) ? 15u : 0u;
            t.w[0] = t.w[1] = t.w[2] = t.w[3] = 0.25f;
        }
        if (!inside) t.valid = 0;
        return t;
    };

    {
      for (int c0 = cfirst; c0 < C; c0 += 64) {
        ccx = cx;
        ccy = cy;
        asm volatile("" : "+v"(ccx), "+v"(ccy));  // keep taps per chunk (no hoisting + spills)
        float acc[CK];
#pragma unroll
        for (int q = 0; q < CK; ++q) acc[q] = (MODE == BEV_FUSE_MAX) ? -__builtin_inff() : 0.0f;
        const float *fb = feats + (int64_t)(b * V) * sN + c0;

        // Views whose corner box is empty (the tile is outside that camera's feature map)
        // contribute +0 (sum / mean: skipping them is exact, the accumulator is never -0)
        // or max(acc, 0): they get no iteration, no DMA and no barrier.
        auto live = [&](int u) { return !ok_of(u) || box_of(u).x1 >= 0; };
        auto next_live = [&](int u) {
            ++u;
            while (u < V && !live(u)) {
                zero_view<MODE>(acc, u);
                ++u;
            }
            return u;
        };
        if (WARP_STAGE_ALL) {
            // ---- every live view's footprint at once: when all corner boxes apply and the images fit the pool
            // together, they are staged back to back up front and the views are sampled with ONE wait + barrier
            // per tile (instead of one per view) -- same taps, same view order, same arithmetic
            int need = 0;  // lane v < V: view v's image bytes (0: empty view; huge: the corner box does not apply)
            if (lane < V) {
                const int x0 = (int)(lba & 0xffffu), y0 = (int)((lba >> 16) & 0x3fffu);
                const int x1 = (int)(lbb & 0xffffu) - 1, y1 = (int)(lbb >> 16) - 1;
                const int np = (x1 - x0 + 1) * (y1 - y0 + 1);
                need = (lba >> 31) ? (1 << 26) : (x1 < 0 ? 0 : stage_bytes(np));
            }
            int tot = need;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
            tot = __builtin_amdgcn_readfirstlane(tot);
            if (tot <= pool) {
                int off = 0;
                for (int u = 0; u < V; ++u) {
                    const Box bx = box_of(u);
                    if (bx.x1 < 0) continue;
                    const int w = bx.x1 - bx.x0 + 1, h = bx.y1 - bx.y0 + 1;
                    dma(fb + (int64_t)u * sN, bx.x0, bx.y0, w, h, off);
                    off += stage_bytes(w * h);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();  // every image and the zero pixel
                off = 0;
                for (int u = 0; u < V; ++u) {
                    const Box bx = box_of(u);
                    if (bx.x1 < 0) {
                        zero_view<MODE>(acc, u);
                        continue;
                    }
                    const int w = bx.x1 - bx.x0 + 1;
                    const Taps t = taps_of(u);
                    if (__ballot(t.valid != 0) != 0ull && (!WARP_LANESKIP || t.valid))
                        sample_view_pipe<MODE, CK, WARP_PIPE != 0>(acc, t, smem, off, bx.x0, bx.y0, w, zp, zp);
                    else
                        zero_view<MODE>(acc, u);
                    off += stage_bytes(w * (bx.y1 - bx.y0 + 1));
                }
                if constexpr (NHWC) store_nhwc(c0, acc, md);
                else if (inside) store_out(c0, acc, md);
                if (c0 + 64 < C) __syncthreads();  // the next chunk re-stages the pool
                continue;
            }
        }
        const int v_first = next_live(-1);
        auto peek_live = [&](int u) {  // next_live without the skipped views' max(acc, 0)
            ++u;
            while (u < V && !live(u)) ++u;
            return u;
        };
        // prologue: DMA of the first live view (if its corner box applies and fits, or its spans do).  Span tables:
        // spc = the current view's, spn = the next live view's (loaded during the view before, consumed after the
        // end-of-view wait), both 0 for views without one.
        Box bn = box_of(v_first < V ? v_first : 0);
        int offn = -1, bytesn = 0;  // the next image's LDS byte offset (-1: not staged ahead) and size
        bool spsn = false;          // ... staged by spans
        unsigned spc = 0u, spn = 0u;
        if (v_first < V) {
            const int npix = (bn.x1 - bn.x0 + 1) * (bn.y1 - bn.y0 + 1);
            if (span_of(v_first)) {
                spc = load_span(v_first);
                asm volatile("" : "+v"(spc));  // its wait: nothing else in flight
                int len, sxr, exc;
                bytesn = span_scan(spc, bn.y1 - bn.y0 + 1, len, sxr, exc);
                stage_span(fb + (int64_t)v_first * sN, bn.y0, bn.y1 - bn.y0 + 1, len, sxr, exc, 0);
                offn = 0;
                spsn = true;
            } else if (ok_of(v_first) && bn.x1 >= 0 && npix <= maxpix) {
                offn = 0;
                bytesn = ((npix * SL + 63) >> 6) * 1024;
                dma(fb + (int64_t)v_first * sN, bn.x0, bn.y0, bn.x1 - bn.x0 + 1, bn.y1 - bn.y0 + 1, 0);
            }
            const int vs = peek_live(v_first);
            if (vs < V && span_of(vs)) spn = load_span(vs);
        }
        // the first live view's taps while its footprint lands (exact-bbox views reduce their taps first)
        Taps tf;
        bool have_f = false;
        if (v_first < V && ok_of(v_first)) {
            tf = taps_of(v_first);
            have_f = true;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // zero pixel + image of the first live view
        asm volatile("" : "+v"(spn));
        STAMP(2);

        int nview = 0;  // live views done (timing stamps)
        for (int v = v_first, vn; v < V; v = vn) {
            vn = next_live(v);
            Box bx = bn;
            const int off = offn, bytesc = bytesn;
            const bool spsc = spsn;
            const float *f = fb + (int64_t)v * sN;
            Taps t;
            bool have_t = false;
            if (have_f) {
                t = tf;
                have_t = true;
                have_f = false;
            }
            if (!ok_of(v)) {
                // exact footprint by per-cell reduction (horizon tiles); staged synchronously
                t = taps_of(v);
                have_t = true;
                put_box<NW>(red, wave_box(t), wave, lane);
                __syncthreads();
                bx = get_box<NW>(red);
            }
            const bool empty = bx.x1 < 0;
            const int bw = bx.x1 - bx.x0 + 1, bh = bx.y1 - bx.y0 + 1;
            bool done = empty;
            if (!done && off < 0 && span_of(v)) {
                // ---- synchronous span staging (no room was left beside the previous image) ----
                int len, sxr, exc;
                span_scan(spc, bh, len, sxr, exc);
                stage_span(f, bx.y0, bh, len, sxr, exc, 0);
                if (!have_t) {
                    t = taps_of(v);
                    have_t = true;
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (__ballot(t.valid != 0) != 0ull && (!WARP_LANESKIP || t.valid)) {
                    int pb, pbs;
                    span_addr(t, 0, bx.y0, pb, pbs);
                    sample_pipe_at<MODE, CK, WARP_PIPE != 0>(acc, t, smem, pb, pbs, zp, zp);
                } else
                    zero_view<MODE>(acc, v);
                done = true;
                __syncthreads();  // the pool is free again
            }
            if (!done && off < 0) {
                // ---- synchronous staging, overlapping blocks if larger than the pool ----
                int wb = bw, hb = bh, nbx = 1, nby = 1;
                if (bw * bh > maxpix) {
                    wb = (2 * bw <= maxpix) ? bw : maxpix / 2;
                    hb = min(bh, maxpix / wb);
                    nbx = (wb >= bw) ? 1 : (bw - 2) / (wb - 1) + 1;
                    nby = (hb >= bh) ? 1 : (bh - 2) / (hb - 1) + 1;
                }
                const bool single = (nbx == 1) && (nby == 1);
                if (single)  // the common case: start the copy (the pool is free since the last
                             // end-of-view barrier), compute the taps while it lands
                    dma(f, bx.x0, bx.y0, bw, bh, 0);
                if (!have_t) {
                    t = taps_of(v);
                    have_t = true;
                }
                int mkx = 0, mky = 0;
                if (!single && t.valid) {
                    const int xlo = (t.valid & 5) ? t.x0 : t.x0 + 1, ylo = (t.valid & 3) ? t.y0 : t.y0 + 1;
                    mkx = (nbx == 1) ? 0 : min((xlo - bx.x0) / (wb - 1), nbx - 1);
                    mky = (nby == 1) ? 0 : min((ylo - bx.y0) / (hb - 1), nby - 1);
                }
                const bool wave_any = __ballot(t.valid != 0) != 0ull;
                if (!single && !t.valid) zero_view<MODE>(acc, v);
                for (int ky = 0; ky < nby; ++ky)
                    for (int kx = 0; kx < nbx; ++kx) {
                        const int sx0 = bx.x0 + kx * (wb - 1), sy0 = bx.y0 + ky * (hb - 1);
                        const int sbw = min(wb, bx.x1 - sx0 + 1), sbh = min(hb, bx.y1 - sy0 + 1);
                        if (!single) {
                            __syncthreads();  // earlier LDS images are no longer read
                            dma(f, sx0, sy0, sbw, sbh, 0);
                        }
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        __syncthreads();
                        const bool mine = single ? true : (t.valid != 0 && mkx == kx && mky == ky);
                        const bool go = single ? wave_any : (__ballot(mine) != 0ull);
                        if (go) sample_view<MODE, 1, CK>(acc, t, mine, v, smem, 0, sx0, sy0, sbw, zp);
                        else if (single) zero_view<MODE>(acc, v);
                    }
                done = true;
                __syncthreads();  // every wave is done with the staged blocks before DMA(v+1) reuses the pool
            }
            // ---- look ahead: DMA of the next live view beside the live image of view v ----
            unsigned spnn = 0u;  // the span table of the live view after vn
            if (vn < V) {
                bn = box_of(vn);
                offn = -1;
                spsn = false;
                const int npix = (bn.x1 - bn.x0 + 1) * (bn.y1 - bn.y0 + 1);
                const bool sp = span_of(vn);
                if (ok_of(vn) && bn.x1 >= 0 && (sp || npix <= maxpix)) {
                    // consecutive images anchor at opposite ends of the pool: they coexist
                    // whenever their sizes add up to at most the pool
                    int len = 0, sxr = 0, exc = 0;
                    const int need = sp ? span_scan(spn, bn.y1 - bn.y0 + 1, len, sxr, exc)
                                        : ((npix * SL + 63) >> 6) * 1024;
                    if (done || off < 0) offn = 0;
                    else if (off == 0) {
                        if (bytesc + need <= pool) offn = pool - need;
                    } else if (need <= off) offn = 0;
                    if (offn >= 0) {
                        if (sp) stage_span(fb + (int64_t)vn * sN, bn.y0, bn.y1 - bn.y0 + 1, len, sxr, exc, offn);
                        else dma(fb + (int64_t)vn * sN, bn.x0, bn.y0, bn.x1 - bn.x0 + 1, bn.y1 - bn.y0 + 1, offn);
                        bytesn = need;
                        spsn = sp;
                    }
                }
                const int vnn = peek_live(vn);
                if (vnn < V && span_of(vnn)) spnn = load_span(vnn);
            }
            // ---- sample view v from its prefetched image ------------------------------
            if (!done) {
                if (!have_t) t = taps_of(v);
                STAMP_VIEW(nview, 0);
                int pb, pbs;  // the taps' LDS pixels
                if (spsc) {
                    span_addr(t, off, bx.y0, pb, pbs);
                } else {
                    pb = off + ((t.y0 - bx.y0) * bw + (t.x0 - bx.x0)) * PS;
                    pbs = pb + bw * PS;
                }
                if (WARP_ABLATE & 4) acc[0] += t.w[0] * t.w[3] + (float)(t.x0 + t.y0 + (int)t.valid);
                else if (__ballot(t.valid != 0) != 0ull) {
                    // WARP_LANESKIP: lanes without a valid tap leave the LDS reads to the others (their sample is
                    // +0: acc + 0 == acc exactly, max(acc, 0) for the max mode)
                    if (WARP_TAPS_AHEAD && vn < V && ok_of(vn)) {
                        // the next view's taps inside this view's sampling, by every lane (a lane without a valid tap
                        // reads the zero pixel: its sample is +0, i.e. acc + 0 == acc, or max(acc, +0) -- what the
                        // lane skip gives)
                        sample_pipe_at<MODE, CK, WARP_PIPE != 0, WARP_TAPS_AHEAD - 2>(
                            acc, t, smem, pb, pbs, zp, zp, [&]() { tf = taps_of(vn); });
                        if (WARP_TAPS_AHEAD == 1) tf = taps_of(vn);  // after the sampling, before the DMA wait
                        have_f = true;
                    } else if (!WARP_LANESKIP || t.valid)
                        sample_pipe_at<MODE, CK, WARP_PIPE != 0>(acc, t, smem, pb, pbs, zp, zp);
                    else zero_view<MODE>(acc, v);
                } else zero_view<MODE>(acc, v);
            } else if (empty) {
                zero_view<MODE>(acc, v);
            }
            STAMP_VIEW(nview, 1);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of view v+1 landed
            __syncthreads();  // all of it landed; image of view v and red[] are free
            spc = spn;
            spn = spnn;
            asm volatile("" : "+v"(spn));  // landed with the DMA
            STAMP_VIEW(nview, 2);
            ++nview;
        }
        STAMP(3);
        if constexpr (NHWC) {
            store_nhwc(c0, acc, md);
        } else if (inside) {
            store_out(c0, acc, md);
        }
        STAMP(4);
      }
    }
}

// -------------------------------------------------------------------------
// fused warp + sum / mean, persistent (k_warp_fuse_p; BEV_TUNE_WARP_PERSIST 1 / 2, an A/B option: measured SLOWER)
// -------------------------------------------------------------------------
// Measured (r06w-r06y, tools/warp_persist_ab.py, interleaved, us per launch): bench 7 cams B = 2 per-tile 135-137,
// persistent 8 queues 150-154, 1 queue 144-146 (8 queues + stealing from the next queue at the tail: 194);
// K5 16 cams 4K 218-224 vs 245-252.  Bit-identical in every form (test_fused_persistent_equals_per_tile_kernel).
// Why it loses: the in-order vmcnt hides the first DMA behind the previous item's stores (vmcnt(63)), but EVERY
// later DMA wait of the item (the end of each view) also waits for those 64 stores, so their drain lands on the
// item's first view; a workgroup of v2 simply ends after its stores and the drain overlaps its successor's start.
// k_warp_fuse_v2's per-item work (one frame x 16 x 16 BEV tile, 64 channels: taps, footprint DMA one view ahead,
// LDS sampling, view order from +0, the mean by the same division) in CUs x OCC resident workgroups that pull items
// from work queues instead of one workgroup per item.  What the loop buys (v2's s_memtime timeline: per workgroup
// ~34 k cycles = prologue 1.6 k + first view's DMA 4.2 k + views 25.2 k + stores 3.1 k, and 2 k from a workgroup's
// end to its successor's start): the next item's boxes and first-view DMA are issued BEFORE this item's output
// stores, so that DMA lands while the 64 store instructions issue and the next item's taps are computed; the wait
// before its first sampling is `vmcnt(63)` (every vector-memory op counts in issue order, MI355X_MICROARCH.md
// §vmcnt: with >= 64 stores younger than the DMA, <= 63 outstanding means the DMA is done, the stores need not be),
// and the barrier after it a raw s_barrier (no fence drain of the stores).  No workgroup launch gap.
// Queues: q = blockIdx % 8 (the XCD under round-robin dispatch) owns the contiguous item range
// [total q / 8, total (q + 1) / 8) (item = frame x tiles + tile): an XCD walks neighbouring tiles, whose footprints
// share source pixels in its L2.  A workgroup's first item is static (lo + blockIdx / 8), the next ones a ticket
// (atomicAdd on the queue word, fetched at the start of the current item and read after its views).  The queue
// words live after the boxes in the workspace: zeroed by k_warp_boxes and reset by the last workgroup to finish
// (a finished-count word), so every launch starts from zero.  Each workgroup exits once its queue is drained --
// no inter-workgroup waits, so residency is not needed for progress.
// Same per-cell arithmetic and view order as v2 => bit-identical output.

template <int MODE, int OCC, bool CHUNK>
__global__ __launch_bounds__(FT_NT, OCC) void k_warp_fuse_p(const float *__restrict__ feats, int64_t sN, int64_t sH,
                                                         int64_t sW, const float *__restrict__ Hmat,
                                                         const float *__restrict__ xs, const float *__restrict__ ys,
                                                         int B, int V, int C, int Hf, int Wf, float sx, float sy,
                                                         int Hb, int Wb, float *__restrict__ out, int pool,
                                                         const uint2 *__restrict__ boxes_in, int rpr,
                                                         unsigned *__restrict__ queue, int nqs) {
    static_assert(MODE != BEV_FUSE_MAX, "sum / mean");
    constexpr int NW = FT_NT / 64, TH = 16, TW = FT_NT / TH, CK = 64, SL = V2_SL, PS = SL * 16;
    static_assert(WARP_CK == 64, "one workgroup per (tile, frame)");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int zp = pool;
    int *red = reinterpret_cast<int *>(smem + pool + 256);
    int *slot = reinterpret_cast<int *>(smem + pool + 256 + 4 * NW * sizeof(int));  // the next ticket (htab area)
    const int maxpix = pool / PS - 4;
    const int ntx = (Wb + TW - 1) / TW, nty = (Hb + TH - 1) / TH, nt = ntx * nty;
    const int total = nt * B;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int tr, tc;
    tile_cell<TH>(lane, wave, tr, tc);
    const int qi = (int)(blockIdx.x % (unsigned)nqs);
    const int nq = (int)(gridDim.x / (unsigned)nqs);  // workgroups per queue (gridDim.x % nqs == 0)
    const int lo = (int)((int64_t)total * qi / nqs), hi = (int)((int64_t)total * (qi + 1) / nqs);
    bool hdr_ok = false;
    {
        const uint4 hd = reinterpret_cast<const uint4 *>(boxes_in)[-1];
        hdr_ok = hd.x == BOX_MAGIC && (int)hd.y == maxpix && (int)hd.z == V && (int)hd.w == TH;
    }
    const Grid grid = make_grid(Hf, Wf);
    const MeanDiv md = mean_div_of(V);
    if (tid < 16) *(float4 *)(smem + zp + tid * 16) = make_float4(0.f, 0.f, 0.f, 0.f);
    const size_t plane = (size_t)Hb * Wb;
    const size_t oplane = CHUNK ? (size_t)rpr * Wb : plane;
    auto dma = [&](const float *fp, int x0, int y0, int w, int h, int o) {
        dma_block<SL>(fp, (int)sH, (int)sW, x0, y0, w, w * h, smem, o, wave, lane, NW);
    };

    // the item being set up: frame, tile origin, this lane's cell, its centre, the boxes of its views
    int b = 0, tyb = 0, txb = 0, ci = 0, cj = 0;
    bool inside = false;
    float cx = 0.f, cy = 0.f;
    unsigned lba = 0, lbb = 0;
    auto load_item = [&](int it) {
        b = it / nt;
        const int tile = it - b * nt;
        tyb = tile / ntx;
        txb = tile - tyb * ntx;
        ci = tyb * TH + tr;
        cj = txb * TW + tc;
        inside = (ci < Hb) && (cj < Wb);
        cx = xs[inside ? cj : 0];
        cy = ys[inside ? ci : 0];
        if (hdr_ok) {
            const uint2 bx = lane < V ? boxes_in[((int64_t)b * nt + tile) * V + lane] : make_uint2(0u, 0u);
            lba = bx.x;
            lbb = bx.y;
        } else {  // boxes made for another pool / V / tiling: every view by the exact per-cell reduction
            lba = lane < V ? 0x80000000u : 0u;
            lbb = 0u;
        }
    };
    auto box_of = [&](int v) {
        const unsigned a = (unsigned)__builtin_amdgcn_readlane((int)lba, v);
        const unsigned c = (unsigned)__builtin_amdgcn_readlane((int)lbb, v);
        return Box{(int)(a & 0xffffu), (int)((a >> 16) & 0x7fffu), (int)(c & 0xffffu) - 1, (int)(c >> 16) - 1};
    };
    auto ok_of = [&](int v) { return ((unsigned)__builtin_amdgcn_readlane((int)lba, v) >> 31) == 0u; };
    auto live = [&](int u) { return !ok_of(u) || box_of(u).x1 >= 0; };
    auto next_live = [&](int u) {  // sum / mean: views with an empty box contribute +0 -- skipped exactly
        ++u;
        while (u < V && !live(u)) ++u;
        return u;
    };
    float ccx = 0.f, ccy = 0.f;
    auto taps_of = [&](int v, bool in) {
        float h[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) h[k] = Hmat[__builtin_amdgcn_readfirstlane((b * V + v) * 9) + k];
        float ix, iy;
        cell_ixy(h, ccx, ccy, grid, sx, sy, ix, iy);
        Taps t = taps_from_ixy(ix, iy, grid);
        if (!in) t.valid = 0;
        return t;
    };
    // the first live view of the item just loaded, its DMA issued now (offn = 0) when its corner box fits the pool
    int v_first = V, offn = -1;
    Box bn{0, 0, -1, -1};
    auto first_dma = [&]() {
        v_first = next_live(-1);
        bn = box_of(v_first < V ? v_first : 0);
        offn = -1;
        if (v_first < V) {
            const int npix = (bn.x1 - bn.x0 + 1) * (bn.y1 - bn.y0 + 1);
            if (ok_of(v_first) && bn.x1 >= 0 && npix <= maxpix) {
                offn = 0;
                dma(feats + (int64_t)(b * V + v_first) * sN, bn.x0, bn.y0, bn.x1 - bn.x0 + 1, bn.y1 - bn.y0 + 1, 0);
            }
        }
    };

    int item = lo + (int)(blockIdx.x / (unsigned)nqs);
    if (item < hi) {
        load_item(item);
        first_dma();
    }
    bool stores_out = false;  // this wave issued the previous item's 64 output stores after the current first DMA
    while (item < hi) {
        int tkt = 0;
        if (tid == 0) tkt = (int)atomicAdd(&queue[qi], 1u);  // the next ticket, read after this item's views
        const int bi = b, ii = ci, jj = cj;
        const bool in = inside;
        ccx = cx;
        ccy = cy;
        asm volatile("" : "+v"(ccx), "+v"(ccy));  // keep the taps per item (no hoisting + spills)
        float acc[CK];
#pragma unroll
        for (int k = 0; k < CK; ++k) acc[k] = 0.0f;
        const float *fb = feats + (int64_t)(bi * V) * sN;
        Taps tf;
        bool have_f = false;
        if (v_first < V && ok_of(v_first)) {
            tf = taps_of(v_first, in);
            have_f = true;
        }
        // the first live view's image (and the zero pixel); the previous item's stores may still be in flight
        if (stores_out) asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        for (int v = v_first, vn; v < V; v = vn) {
            vn = next_live(v);
            Box bx = bn;
            const int off = offn;
            const float *f = fb + (int64_t)v * sN;
            Taps t;
            bool have_t = false;
            if (have_f) {
                t = tf;
                have_t = true;
                have_f = false;
            }
            if (!ok_of(v)) {  // exact footprint by per-cell reduction (horizon tiles); staged synchronously
                t = taps_of(v, in);
                have_t = true;
                put_box<NW>(red, wave_box(t), wave, lane);
                __syncthreads();
                bx = get_box<NW>(red);
            }
            const bool empty = bx.x1 < 0;
            const int bw = bx.x1 - bx.x0 + 1, bh = bx.y1 - bx.y0 + 1;
            bool done = empty;
            if (!done && off < 0) {  // synchronous staging, overlapping blocks if larger than the pool (as v2)
                int wb = bw, hb = bh, nbx = 1, nby = 1;
                if (bw * bh > maxpix) {
                    wb = (2 * bw <= maxpix) ? bw : maxpix / 2;
                    hb = min(bh, maxpix / wb);
                    nbx = (wb >= bw) ? 1 : (bw - 2) / (wb - 1) + 1;
                    nby = (hb >= bh) ? 1 : (bh - 2) / (hb - 1) + 1;
                }
                const bool single = (nbx == 1) && (nby == 1);
                if (single) dma(f, bx.x0, bx.y0, bw, bh, 0);
                if (!have_t) {
                    t = taps_of(v, in);
                    have_t = true;
                }
                int mkx = 0, mky = 0;
                if (!single && t.valid) {
                    const int xlo = (t.valid & 5) ? t.x0 : t.x0 + 1, ylo = (t.valid & 3) ? t.y0 : t.y0 + 1;
                    mkx = (nbx == 1) ? 0 : min((xlo - bx.x0) / (wb - 1), nbx - 1);
                    mky = (nby == 1) ? 0 : min((ylo - bx.y0) / (hb - 1), nby - 1);
                }
                const bool wave_any = __ballot(t.valid != 0) != 0ull;
                for (int ky = 0; ky < nby; ++ky)
                    for (int kx = 0; kx < nbx; ++kx) {
                        const int sx0 = bx.x0 + kx * (wb - 1), sy0 = bx.y0 + ky * (hb - 1);
                        const int sbw = min(wb, bx.x1 - sx0 + 1), sbh = min(hb, bx.y1 - sy0 + 1);
                        if (!single) {
                            __syncthreads();
                            dma(f, sx0, sy0, sbw, sbh, 0);
                        }
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        __syncthreads();
                        const bool mine = single ? true : (t.valid != 0 && mkx == kx && mky == ky);
                        const bool go = single ? wave_any : (__ballot(mine) != 0ull);
                        if (go) sample_view<MODE, 1, CK>(acc, t, mine, v, smem, 0, sx0, sy0, sbw, zp);
                    }
                done = true;
                __syncthreads();
            }
            if (vn < V) {  // look ahead: DMA of the next live view beside the live image of view v
                bn = box_of(vn);
                offn = -1;
                const int npix = (bn.x1 - bn.x0 + 1) * (bn.y1 - bn.y0 + 1);
                if (ok_of(vn) && bn.x1 >= 0 && npix <= maxpix) {
                    const int need = ((npix * SL + 63) >> 6) * 1024;
                    if (done || off < 0) offn = 0;
                    else if (off == 0) {
                        if (((bw * bh * SL + 63) >> 6) * 1024 + need <= pool) offn = pool - need;
                    } else if (need <= off) offn = 0;
                    if (offn >= 0) dma(fb + (int64_t)vn * sN, bn.x0, bn.y0, bn.x1 - bn.x0 + 1, bn.y1 - bn.y0 + 1, offn);
                }
            }
            if (!done) {
                if (!have_t) t = taps_of(v, in);
                if (__ballot(t.valid != 0) != 0ull && (!WARP_LANESKIP || t.valid))
                    sample_view_pipe<MODE, CK, WARP_PIPE != 0>(acc, t, smem, off, bx.x0, bx.y0, bw, zp, zp);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of view v+1 landed
            __syncthreads();  // all of it landed; image of view v and red[] are free
        }
        // the next item: its ticket, boxes and first-view DMA before this item's stores (the pool is free: every
        // view of this item ended with a barrier after its last LDS read)
        if (tid == 0) *slot = tkt;
        __syncthreads();
        const int nxt = lo + nq + __builtin_amdgcn_readfirstlane(*slot);
        if (nxt < hi) {
            load_item(nxt);
            first_dma();
        }
        item = nxt;
        if (in) {
            if (!CHUNK) {
                store_chunk(out + (size_t)bi * C * plane, plane, (ii * Wb + jj) * (int)sizeof(float), acc, MODE, md,
                            (uint32_t)(plane * CK * sizeof(float)));
            } else {
                const int ck = ii / rpr;
                const int ovoff = (int)(((size_t)ck * B * C * oplane + (size_t)(ii - ck * rpr) * Wb + jj) * sizeof(float));
                const size_t orange = (size_t)((Hb + rpr - 1) / rpr) * B * C * oplane * sizeof(float);
                store_chunk(out + (size_t)bi * C * oplane, oplane, ovoff, acc, MODE, md,
                            out_range(orange, (size_t)bi * C * oplane));
            }
        }
        stores_out = __ballot(in) != 0ull;
    }
    // queue bookkeeping: the last workgroup to finish resets the words for the next launch
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const unsigned d = atomicAdd(&queue[8], 1u);
        if (d == gridDim.x - 1) {
#pragma unroll
            for (int k = 0; k < 9; ++k) atomicExch(&queue[k], 0u);
        }
    }
}

template <int TH, int TW = FT_NT / TH>
__global__ __launch_bounds__(256) void k_warp_boxes(const float *__restrict__ Hmat, const float *__restrict__ xs,
                                                    const float *__restrict__ ys, int V, int Hf, int Wf, float sx,
                                                    float sy, int Hb, int Wb, int maxpix, int nty,
                                                    uint2 *__restrict__ boxes, unsigned *__restrict__ queue,
                                                    unsigned *__restrict__ spans, int span_pct) {
    const int ntx = (Wb + TW - 1) / TW, nt = ntx * nty;  // nty >= ceil(Hb / TH) box-tile rows (extra rows: empty)
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int b = blockIdx.y;
    if (t == 0 && b == 0)
        reinterpret_cast<uint4 *>(boxes)[-1] =
            make_uint4(BOX_MAGIC, (unsigned)maxpix, (unsigned)V, (unsigned)TH | (spans ? SPAN_FLAG : 0u));
    if (queue != nullptr && b == 0 && t < WQ_WORDS) queue[t] = 0u;  // k_warp_fuse_p's work queues start at zero
    if (t >= (int64_t)nt * V) return;
    const int tile = (int)(t / V), v = (int)(t - (int64_t)tile * V);
    const int tyb = tile / ntx, txb = tile - tyb * ntx;
    const int ia = tyb * TH, ib = min(ia + TH - 1, Hb - 1);
    const int ja = txb * TW, jb = min(ja + TW - 1, Wb - 1);
    bool ok = true, span = false;
    Box cb{0x7fffffff, 0x7fffffff, -1, -1};
    Quad q;
    if (ia < Hb) {
        float hv[9];
        load_h(Hmat, b * V + v, hv);
        cb = corner_box(hv, xs[ja], xs[jb], ys[ia], ys[ib], sx, sy, Wf, Hf, ok, spans ? &q : nullptr);
    }
    if (ok && cb.x1 >= 0) {
        const int bpix = (cb.x1 - cb.x0 + 1) * (cb.y1 - cb.y0 + 1), nrows = cb.y1 - cb.y0 + 1;
        // the spans of a row band of height 2 hold at least the quad's width across it, and every point of the quad
        // lies in two bands: the spans total at least the quad's area -- a box that fits and is less than
        // 100 / span_pct times that area cannot qualify (no row pass)
        double area = 0.0;
        if (spans) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int a = QUAD_ORD[e], c = QUAD_ORD[(e + 1) & 3];
                area += q.x[a] * q.y[c] - q.x[c] * q.y[a];
            }
            area = 0.5 * fabs(area);
        }
        if (spans && nrows <= SPAN_ROWS && (bpix > maxpix || area * 100.0 <= (double)bpix * span_pct)) {
            // span staging: when the box does not fit the pool but its rows' spans do, or when they save enough
            // one pass: the table is written whether or not the view ends up flagged (the fused kernel reads only
            // flagged views' tables)
            quad_slopes(q);
            const QuadF qf = quad_f(q, cb);
            unsigned *o = spans + (((int64_t)b * nt + tile) * V + v) * SPAN_ROWS;
            int tot = 1;  // + the row-base header (144 B < one pixel)
            for (int r = 0; r < nrows; ++r) {
                const unsigned w = row_span(qf, cb, r);
                o[r] = w;
                tot += (int)(w >> 16);
            }
            span = bpix > maxpix ? tot <= maxpix : tot * 100 <= bpix * span_pct;
        }
        if (!span && bpix > maxpix) ok = false;
    }
    const bool emp = cb.x1 < 0;
    boxes[((int64_t)b * nt + tile) * V + v] =
        make_uint2((emp ? 0u : (unsigned)cb.x0 | ((unsigned)cb.y0 << 16)) | (ok ? 0u : 0x80000000u) |
                       (span ? 0x40000000u : 0u),
                   emp ? 0u : (unsigned)(cb.x1 + 1) | ((unsigned)(cb.y1 + 1) << 16));
}

// -------------------------------------------------------------------------
// fused warp + sum / mean v3: DPP row runs (default for NHWC features with C % 64 == 0, modes SUM / MEAN)
// -------------------------------------------------------------------------
// Workgroup = one (frame, 16 x 16 BEV tile), 4 waves, wave w = tile rows 4w .. 4w + 3, one 16-lane DPP row per tile
// row.  Lane l of a row computes the taps of cell l of its row (once per view, the bit-exact recipe) and holds, for
// ALL 16 cells of the row, the 4 channels 4l .. 4l + 3 of the 64-channel chunk: acc[16][4].  A row walks its cells
// k = 0..15: cell k's quad key, tap addresses and weights come from lane k by DPP row broadcast (row_newbcast), the
// row reads the quad's four 256-B pixels with one ds_read_b128 per tap (lane l: bytes 16l .. 16l + 15 -- every
// 16-lane LDS group reads whole pixels, conflict-free on the unpadded 256-B pixel layout), and the bilinear combine is
// the reference's FMA chain per channel.  Consecutive cells usually share a quad (Appendix-B rig: 80 % have their
// left neighbour's): the reads are skipped whenever no row of the wave enters a new quad (wave-uniform ballot) --
// half of the steps on the rig, so half the LDS reads of one read per (cell, view, tap).
// Footprints: conservative corner boxes from k_warp_boxes (workspace).  The views of a tile are staged in batches:
// as many consecutive views as fit the pool, each box row one contiguous NHWC run moved by LDS-DMA (4 pixels per
// 1-KiB instruction, no per-lane index arithmetic), ONE vmcnt wait + barrier per batch, then the batch's views are
// walked in view order (the reference's v = 0..V-1 accumulation from +0).  Views whose box does not apply (w sign
// change / |w| near 1e-6) or does not fit the pool read their taps straight from global memory (same walk).
// Output: each lane stores its 4 channel planes x 16 cells as 16-B non-temporal stores; the mean divides by V in
// fp32 (Markstein's correction step, exact for the verified V -- tools/verify_div_markstein_fix.c) or through
// div_rcp.  Bit-identical to k_warp_fuse_v2 (same taps, weights, FMA chain, view order, division result).
constexpr int W3_PIX = 256;  // staged bytes per pixel (one unpadded 64-channel chunk)

template <int K>
__device__ __forceinline__ int rbc(int v) {  // lane K of this lane's 16-lane DPP row
    return __builtin_amdgcn_update_dpp(0, v, 0x150 + K, 0xf, 0xf, true);  // bound_ctrl: no "old" operand to set up
}
template <int K>
__device__ __forceinline__ float rbcf(float v) {
    return __builtin_bit_cast(float, rbc<K>(__builtin_bit_cast(int, v)));
}

// one lane's cell for one view, broadcast along its row during the walk
struct CellTap {
    int key;    // (x0 + 1) | (y0 + 1) << 14 | valid << 28; 0 = no valid tap (never a real key; -1 neither)
    int a[4];   // staged: LDS byte address of each tap (the zero pixel if invalid); direct: element offset or -1
    float w[4]; // bilinear weights nw, ne, sw, se (all 0 when no tap is valid)
};

template <int K>
__device__ __forceinline__ void w3_step(float (&acc)[16][4], f32x4 (&qv)[4], int &cur, CellTap &c,
                                        const unsigned char *smem, __amdgpu_buffer_rsrc_t rs, bool direct, int l16) {
    // the broadcast sources are re-defined per step: no hoisting of all 16 steps' broadcasts (register pressure)
    asm volatile("" : "+v"(c.key), "+v"(c.a[0]), "+v"(c.a[1]), "+v"(c.a[2]), "+v"(c.a[3]), "+v"(c.w[0]),
                 "+v"(c.w[1]), "+v"(c.w[2]), "+v"(c.w[3]));
    const int kk = rbc<K>(c.key);
    if (__ballot(kk != cur) != 0ull) {  // wave-uniform: some row enters a new quad -> every row reads its quad
        int at[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) at[t] = rbc<K>(c.a[t]);
        if (direct) {  // (uniform) buffer loads: an invalid tap's out-of-range offset reads 0
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int vo = at[t] >= 0 ? at[t] * 4 + 16 * l16 : 0x7ffffff0;
                qv[t] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, 0, 0));
            }
        } else {
#pragma unroll
            for (int t = 0; t < 4; ++t) qv[t] = *reinterpret_cast<const f32x4 *>(smem + at[t] + 16 * l16);
        }
    }
    cur = kk;
    const float w0 = rbcf<K>(c.w[0]), w1 = rbcf<K>(c.w[1]), w2 = rbcf<K>(c.w[2]), w3 = rbcf<K>(c.w[3]);
    // grid_sampler_2d's chain (bilerp) per channel, then the view sum -- as packed fp32 (v_pk_mul / v_pk_fma /
    // v_pk_add: two channels per instruction, each half the scalar op exactly)
    const f32x2 W0 = (f32x2){w0, w0}, W1 = (f32x2){w1, w1}, W2 = (f32x2){w2, w2}, W3 = (f32x2){w3, w3};
    f32x2 a = qv[0].xy * W0, b = qv[0].zw * W0;
    a = __builtin_elementwise_fma(qv[1].xy, W1, a);
    b = __builtin_elementwise_fma(qv[1].zw, W1, b);
    a = __builtin_elementwise_fma(qv[2].xy, W2, a);
    b = __builtin_elementwise_fma(qv[2].zw, W2, b);
    a = __builtin_elementwise_fma(qv[3].xy, W3, a);
    b = __builtin_elementwise_fma(qv[3].zw, W3, b);
    const f32x2 s0 = (f32x2){acc[K][0], acc[K][1]} + a, s1 = (f32x2){acc[K][2], acc[K][3]} + b;
    acc[K][0] = s0.x;
    acc[K][1] = s0.y;
    acc[K][2] = s1.x;
    acc[K][3] = s1.y;
    // and the step's sums are complete here: without this the compiler defers the FMAs of many steps (keeping
    // their broadcast weights and quads live -- spills)
    asm volatile("" : "+v"(acc[K][0]), "+v"(acc[K][1]), "+v"(acc[K][2]), "+v"(acc[K][3]));
}

template <int K>
__device__ __forceinline__ void w3_walk(float (&acc)[16][4], f32x4 (&qv)[4], int &cur, CellTap &c,
                                        const unsigned char *smem, __amdgpu_buffer_rsrc_t rs, bool direct, int l16) {
    w3_step<K>(acc, qv, cur, c, smem, rs, direct, l16);
    if constexpr (K + 1 < 16) w3_walk<K + 1>(acc, qv, cur, c, smem, rs, direct, l16);
}

// Stage one view's box (bx0, by0, bw x bh pixels of the map at chunk channel 0) into LDS at byte offset img: row r at
// img + r * bw4 * 256 (bw4 = bw rounded up to 4 pixels), 4 pixels per LDS-DMA instruction, rows round-robin over
// the waves.  Lane l moves bytes 16 (l & 15) .. of pixel 4i + (l >> 4) of the row.
__device__ __forceinline__ void w3_stage(const float *__restrict__ map, int64_t sH, int64_t sW, int bx0, int by0,
                                         int bw, int bh, unsigned char *smem, int img, int wave, int lane) {
    if (WARP_ABLATE & 2) return;
    const int bw4 = (bw + 3) & ~3, nins = bw4 >> 2;
    const int px = lane >> 4, cb = (lane & 15) * 4;
    for (int r = wave; r < bh; r += FT_NT / 64) {
        const float *row = map + (int64_t)(by0 + r) * sH + (int64_t)bx0 * sW + cb;
        const int dst0 = (int)lds_base(smem) + img + r * bw4 * W3_PIX;
        for (int i = 0; i < nins; ++i) {
            const int x = 4 * i + px;
            const unsigned dst = (unsigned)__builtin_amdgcn_readfirstlane(dst0 + i * 1024);
            if (x < bw) {
                const float *src = row + (int64_t)x * sW;
                unsigned keep;
                asm volatile(
                    "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                    "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                    : "=&s"(keep)
                    : "v"(src), "s"(dst)
                    : "memory");
            }
        }
    }
}

// a / V in fp32: Markstein's correction step + the NaN fix-up (exact for every float but -0 when V is in the verified
// set; the view sum is never -0), else div_rcp through double.
__device__ __forceinline__ float w3_div(float a, float vf, float r, double rV, bool fast) {
    if (fast) {
        const float q0 = a * r;
        const float q = __builtin_fmaf(__builtin_fmaf(-q0, vf, a), r, q0);
        return q != q ? q0 : q;
    }
    return div_rcp(a, rV);
}

template <int MODE>
__global__ __launch_bounds__(FT_NT, 3) void k_warp_fuse_v3(const float *__restrict__ feats, int64_t sN, int64_t sH,
                                                           int64_t sW, const float *__restrict__ Hmat,
                                                           const float *__restrict__ xs, const float *__restrict__ ys,
                                                           int B, int V, int C, int Hf, int Wf, float sx, float sy,
                                                           int Hb, int Wb, float *__restrict__ out, int pool,
                                                           const uint2 *__restrict__ boxes, int fastdiv) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int zp = pool;  // the zero pixel (256 B) after the pool
    const int ntx = (Wb + 15) / 16, nty = (Hb + 15) / 16, nt = ntx * nty;
    int tile = blockIdx.x;
    {  // XCD-aware order: neighbouring tiles (shared source pixels) on one XCD's L2
        const int q = nt / 8, r = nt % 8, x = tile % 8;
        tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + tile / 8;
    }
    const int ty = tile / ntx, tx = tile - ty * ntx;
    const int b = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l16 = lane & 15;
    const int i = ty * 16 + wave * 4 + (lane >> 4), j0 = tx * 16, j = j0 + l16;
    const bool inside = i < Hb && j < Wb;
    const float cx = xs[inside ? j : 0], cy = ys[inside ? i : 0];
    const Grid grid = make_grid(Hf, Wf);
    if (tid < 16) *(float4 *)(smem + zp + tid * 16) = make_float4(0.f, 0.f, 0.f, 0.f);
    // boxes of this (frame, tile): lane v of every wave holds view v's (k_warp_boxes format)
    uint2 bxv = make_uint2(0u, 0u);
    if (lane < V) bxv = boxes[((int64_t)b * nt + tile) * V + lane];
    // consume the load here: its wait would otherwise sit at the head of the staging loop and, every iteration,
    // also wait for the LDS-DMA issued so far (the compiler cannot see those in the asm) -- serialising the views
    asm volatile("" : "+v"(bxv.x), "+v"(bxv.y));
    auto box_of = [&](int v) {
        const unsigned a = (unsigned)__builtin_amdgcn_readlane((int)bxv.x, v);
        const unsigned c = (unsigned)__builtin_amdgcn_readlane((int)bxv.y, v);
        return Box{(int)(a & 0xffffu), (int)((a >> 16) & 0x7fffu), (int)(c & 0xffffu) - 1, (int)(c >> 16) - 1};
    };
    auto ok_of = [&](int v) { return ((unsigned)__builtin_amdgcn_readlane((int)bxv.x, v) >> 31) == 0u; };
    auto need_of = [&](const Box &bo) { return (bo.y1 - bo.y0 + 1) * (((bo.x1 - bo.x0 + 1) + 3) & ~3) * W3_PIX; };
    const float vf = (float)V, rf = (float)(1.0 / (double)V);
    const double rV = recip_uniform(V);
    const size_t plane = (size_t)Hb * Wb;

    for (int c0 = 0; c0 < C; c0 += 64) {
        float acc[16][4];
#pragma unroll
        for (int k = 0; k < 16; ++k)
#pragma unroll
            for (int u = 0; u < 4; ++u) acc[k][u] = 0.0f;
        const float *fb = feats + (int64_t)(b * V) * sN + c0;
        for (int v = 0; v < V;) {
            // ---- stage a batch: consecutive views while their images fit the pool ----
            int off = 0, u = v;
            for (; u < V; ++u) {
                const Box bo = box_of(u);
                if (bo.x1 < 0 || !ok_of(u)) continue;  // empty (no work) or direct (no staging)
                const int need = need_of(bo);
                if (need > pool) continue;  // direct
                if (off + need > pool) break;
                w3_stage(fb + (int64_t)u * sN, sH, sW, bo.x0, bo.y0, bo.x1 - bo.x0 + 1, bo.y1 - bo.y0 + 1, smem, off,
                         wave, lane);
                off += need;
            }
            const int vend = u;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA landed
            __syncthreads();                                  // every wave's (and the zero pixel)
            // ---- walk the batch's views in view order ----
            off = 0;
            for (u = v; u < vend; ++u) {
                const Box bo = box_of(u);
                if (bo.x1 < 0) continue;  // the tile misses this view: +0 for every cell, exact to skip
                const int need = need_of(bo);
                const bool direct = !ok_of(u) || need > pool;
                const int img = off;
                if (!direct) off += need;
                float h[9];
#pragma unroll
                for (int q = 0; q < 9; ++q) h[q] = Hmat[__builtin_amdgcn_readfirstlane((b * V + u) * 9) + q];
                float ix, iy;
                cell_ixy(h, cx, cy, grid, sx, sy, ix, iy);
                Taps t = taps_from_ixy(ix, iy, grid);
                if (!inside) t.valid = 0;
                CellTap c;
                c.key = t.valid ? (t.x0 + 1) | ((t.y0 + 1) << 14) | ((int)t.valid << 28) : 0;
                const bool any = t.valid != 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) c.w[q] = any ? t.w[q] : 0.0f;
                if (direct) {
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        c.a[q] = (t.valid & (1u << q))
                                     ? (int)((int64_t)(t.y0 + (q >> 1)) * sH + (int64_t)(t.x0 + (q & 1)) * sW)
                                     : -1;
                } else {
                    const int bw4 = ((bo.x1 - bo.x0 + 1) + 3) & ~3;
                    const int p0 = img + ((t.y0 - bo.y0) * bw4 + (t.x0 - bo.x0)) * W3_PIX;
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        c.a[q] = (t.valid & (1u << q)) ? p0 + ((q >> 1) * bw4 + (q & 1)) * W3_PIX : zp;
                }
                f32x4 qv[4];
                int cur = -1;
                if (WARP_ABLATE & 4) continue;
                // direct views: the view's map at this chunk as a buffer (bytes: every pixel's 64 channels)
                const int nbytes = direct ? (int)(((int64_t)(Hf - 1) * sH + (int64_t)(Wf - 1) * sW + 64) * 4) : 0;
                const __amdgpu_buffer_rsrc_t rs =
                    __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(fb + (int64_t)u * sN), 0, nbytes, 0x00020000);
                w3_walk<0>(acc, qv, cur, c, smem, rs, direct, l16);
            }
            __syncthreads();  // the pool is free for the next batch
            v = vend;
        }
        // ---- output: channel planes 4 l16 .. 4 l16 + 3, cells j0 .. j0 + 15 of row i ----
        if (i < Hb && !(WARP_ABLATE & 16)) {
            float *ob = out + ((size_t)b * C + c0 + 4 * l16) * plane + (size_t)i * Wb + j0;
            const bool mean = MODE == BEV_FUSE_MEAN && !(WARP_ABLATE & 1);
            if (j0 + 16 <= Wb && (Wb & 3) == 0) {
#pragma unroll
                for (int uu = 0; uu < 4; ++uu)
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        f32x4 o;
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const float a = acc[4 * m + e][uu];
                            o[e] = mean ? w3_div(a, vf, rf, rV, fastdiv != 0) : a;
                        }
                        // plain stores: a lane's 64-B run of one channel row is 4 of these, merged in L2 (16-B
                        // non-temporal stores from 64 different rows per instruction went to HBM as partial writes)
                        *reinterpret_cast<f32x4 *>(ob + uu * plane + 4 * m) = o;
                    }
            } else {
#pragma unroll
                for (int uu = 0; uu < 4; ++uu)
#pragma unroll
                    for (int k = 0; k < 16; ++k)
                        if (j0 + k < Wb) {
                            const float a = acc[k][uu];
                            ob[uu * plane + k] = mean ? w3_div(a, vf, rf, rV, fastdiv != 0) : a;
                        }
            }
        }
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
    const double rV = recip_uniform(V);  // mean: acc / V via div_rcp (exact)
    for (int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; m < M; m += (int64_t)gridDim.x * blockDim.x) {
        float acc;
        if (MODE == BEV_FUSE_MAX) {
            acc = xb[m];
            for (int v = 1; v < V; ++v) acc = nan_max(acc, xb[(size_t)v * M + m]);
        } else {
            acc = 0.0f;
            for (int v = 0; v < V; ++v) acc = acc + xb[(size_t)v * M + m];
            if (MODE == BEV_FUSE_MEAN) acc = div_rcp(acc, rV);
        }
        ob[m] = acc;
    }
}

// Backward of the max over views (fusion.py:22, bev_maps.max(dim=1).values): the gradient goes to the view torch's
// CPU max(dim) returns as the index -- the first NaN if any element is NaN, else the first maximal element (ties,
// -0 vs +0 included, go to the lowest view) -- and every other view gets 0.  gx [B][V][M], all of it written.
__global__ void k_view_max_bwd(const float *__restrict__ x, const float *__restrict__ g, int V, int64_t M,
                               float *__restrict__ gx) {
    const int b = blockIdx.y;
    const float *xb = x + (size_t)b * V * M;
    float *gb = gx + (size_t)b * V * M;
    for (int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; m < M; m += (int64_t)gridDim.x * blockDim.x) {
        float best = xb[m];
        int arg = 0;
        for (int v = 1; v < V; ++v) {
            const float t = xb[(size_t)v * M + m];
            if (best == best && (t > best || t != t)) {  // nan_max's choice; a NaN best is kept
                best = t;
                arg = v;
            }
        }
        const float gm = g[(size_t)b * M + m];
        for (int v = 0; v < V; ++v) gb[(size_t)v * M + m] = (v == arg) ? gm : 0.0f;
    }
}

inline int err(hipError_t e) { return (int)e; }
inline int last() { return (int)hipGetLastError(); }

// ---- performance knobs (bev_tune; results never depend on them) -------------
int g_warp_pool_kb = 0;  // BEV_TUNE_WARP_POOL_KB: LDS image pool / ring per workgroup, 0 = automatic
int g_warp_kernel = 0;   // BEV_TUNE_WARP_KERNEL: 0 default (= 2), 1 register-staged k_warp_fuse, 2 per-view LDS-DMA
                         // k_warp_fuse_v2, 3 DPP-row k_warp_fuse_v3 (sum / mean with a workspace)
int g_warp_bwd_pool = 0; // BEV_TUNE_WARP_BWD_POOL: backward LDS image in floats, 0 = WARP_BWD_POOL_MAX
// BEV_TUNE_WARP_PERSIST: 0 (default) = k_warp_fuse_v2; 1 = k_warp_fuse_p with 8 work queues, 2 = with one queue.
// r06x A/B (tools/warp_persist_ab.py, us per launch, bench / K5): per-tile 136.2 / 220.0, persistent 8 queues
// 150.2 / 247.6, 1 queue 145.6 / 245.7 -- slower: see k_warp_fuse_p (the store drain the next DMA waits behind).
int g_warp_persist = 0;
int g_warp_span_pct = WARP_SPAN_PCT;  // BEV_TUNE_WARP_SPAN: span staging threshold in percent, 0 = off
// BEV_TUNE_WARP_TILE_BAND: fused warp v2 tile order, 1 = row-major, n = bands of n tile rows walked column by column,
// 0 = automatic: bands of 4 for >= 12 views (read-heavy: the 16-camera 4K rig's warp 228.9 -> 220.5 us and its reads
// 479 -> 366 MB per launch), row-major otherwise (store-heavy: the 7-camera bench rig's output rows stay contiguous
// across the resident tiles; bands of 4 there 134.5 -> 137.4 us) -- profiles/r06bf_warp_tile_band_ab.txt
int g_warp_tile_band = 0;

constexpr int FUSE_LDS_BYTES = 60 * 1024;  // register-staged kernel's footprint image

int cu_count() {
    static int cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    if (cache[dev] == 0) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
        cache[dev] = c;
    }
    return cache[dev];
}

template <int CK, bool VEC>
int launch_fuse(const float *feats, int64_t sN, int64_t sC, int64_t sH, int64_t sW, const float *Hmat, const float *xs,
                const float *ys, int B, int V, int C, int Hf, int Wf, float sx, float sy, int Hb, int Wb, int mode,
                float *out, hipStream_t st) {
    const int ntiles = ((Wb + FT_W - 1) / FT_W) * ((Hb + FT_H - 1) / FT_H);
    dim3 grid(ntiles, B), block(FT_NT);
    const int img = FUSE_LDS_BYTES;
    const size_t lds = img + 32 * sizeof(int);
    switch (mode) {
        case BEV_FUSE_SUM:
            hipLaunchKernelGGL((k_warp_fuse<CK, BEV_FUSE_SUM, VEC>), grid, block, lds, st, feats, sN, sC, sH, sW, Hmat,
                               xs, ys, V, C, Hf, Wf, sx, sy, Hb, Wb, out, img);
            break;
        case BEV_FUSE_MEAN:
            hipLaunchKernelGGL((k_warp_fuse<CK, BEV_FUSE_MEAN, VEC>), grid, block, lds, st, feats, sN, sC, sH, sW,
                               Hmat, xs, ys, V, C, Hf, Wf, sx, sy, Hb, Wb, out, img);
            break;
        default:
            hipLaunchKernelGGL((k_warp_fuse<CK, BEV_FUSE_MAX, VEC>), grid, block, lds, st, feats, sN, sC, sH, sW, Hmat,
                               xs, ys, V, C, Hf, Wf, sx, sy, Hb, Wb, out, img);
    }
    return last();
}

template <int CK>
int launch_fuse_ck(const float *feats, int64_t sN, int64_t sC, int64_t sH, int64_t sW, const float *Hmat,
                   const float *xs, const float *ys, int B, int V, int C, int Hf, int Wf, float sx, float sy, int Hb,
                   int Wb, int mode, float *out, hipStream_t st) {
    const bool vec = (sC == 1) && (C % 4 == 0) && (((uintptr_t)feats & 15) == 0) && (sW % 4 == 0) && (sH % 4 == 0) &&
                     (sN % 4 == 0);
    if (vec)
        return launch_fuse<CK, true>(feats, sN, sC, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out,
                                     st);
    return launch_fuse<CK, false>(feats, sN, sC, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, st);
}

#ifndef WARP_TILE_H
#define WARP_TILE_H 16  // fused-warp tile: 16 x 16 (default) or 8 x 32 cells (A/B builds)
#endif
#ifndef WARP_OCC
#define WARP_OCC 3   // workgroups per CU the default (mean / sum) kernel is compiled and sized for
#endif
constexpr int V2_FIXED = 256 + 4 * (FT_NT / 64) * (int)sizeof(int) + V2_MAXV * 9 * (int)sizeof(float) +
                         (2 * V2_MAXV + 4) * (int)sizeof(unsigned);  // zero pixel, red, htab, btab

// k_warp_boxes' span tables (after the queue words), or none: span staging off (knob 0), or boxes for a kernel that
// does not read them (the persistent kernel; v2 builds with 32-channel workgroups, staging everything up front or
// the LDS homography prologue)
inline unsigned *span_tables(unsigned *queue, bool persist) {
    if (!queue || persist || g_warp_span_pct <= 0 || WARP_CK != 64 || WARP_STAGE_ALL || !WARP_HSCALAR) return nullptr;
    return queue + WQ_WORDS;
}

template <int OCC>
int launch_fuse_v2_occ(const float *feats, int64_t sN, int64_t sH, int64_t sW, const float *Hmat, const float *xs,
                       const float *ys, int B, int V, int C, int Hf, int Wf, float sx, float sy, int Hb, int Wb,
                       int mode, float *out, hipStream_t st, int pool, uint2 *boxes, bool boxes_ready, int rpr) {
    constexpr int TH = WARP_TILE_H, TW = FT_NT / TH;
    const int ntiles = ((Wb + TW - 1) / TW) * ((Hb + TH - 1) / TH);
    dim3 grid(ntiles, B * V2_SPLIT), block(FT_NT);
    const size_t lds = (size_t)pool + V2_FIXED;
    if (!WARP_HSCALAR) boxes = nullptr;  // the in-kernel prologue (LDS homographies)
    unsigned *queue = boxes ? reinterpret_cast<unsigned *>(boxes + (int64_t)B * ntiles * V) : nullptr;
    const bool nhwc = rpr == 0;          // channels-last output (bev_ipm_warp_fuse_nhwc_f32)
    const bool ck = !nhwc && rpr < Hb;  // rank-chunk-major output (camera-shard partials)
    const bool persist = g_warp_persist && boxes && !nhwc && C == 64 && mode != BEV_FUSE_MAX && TH == 16 &&
                         WARP_CK == 64 && !WARP_STAGE_ALL && !WARP_TAPS_AHEAD;
    if (boxes && !boxes_ready) {  // else bev_ipm_warp_fuse_boxes_f32 wrote them (same geometry, pool and knobs)
        const int maxpix = pool / (V2_SL * 16) - 4;  // the kernel's own pool test
        hipLaunchKernelGGL((k_warp_boxes<TH>), dim3((unsigned)(((int64_t)ntiles * V + 255) / 256), B), dim3(256), 0,
                           st, Hmat, xs, ys, V, Hf, Wf, sx, sy, Hb, Wb, maxpix, (Hb + TH - 1) / TH, boxes, queue,
                           span_tables(queue, persist), g_warp_span_pct);
    }
    if (persist) {
        // persistent: OCC resident workgroups per CU, a multiple of 8 (one work queue per XCD)
        const int nq = (cu_count() * OCC + 7) / 8;
        const dim3 pgrid((unsigned)(8 * nq)), pblock(FT_NT);
        auto gop = [&](auto kern) {
            hipLaunchKernelGGL(kern, pgrid, pblock, lds, st, feats, sN, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy,
                               Hb, Wb, out, pool, boxes, rpr, queue, g_warp_persist == 2 ? 1 : 8);
        };
        if (mode == BEV_FUSE_SUM) ck ? gop(k_warp_fuse_p<BEV_FUSE_SUM, OCC, true>) : gop(k_warp_fuse_p<BEV_FUSE_SUM, OCC, false>);
        else ck ? gop(k_warp_fuse_p<BEV_FUSE_MEAN, OCC, true>) : gop(k_warp_fuse_p<BEV_FUSE_MEAN, OCC, false>);
        return last();
    }
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, block, lds, st, feats, sN, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb,
                           out, pool, boxes, rpr, g_warp_tile_band > 0 ? g_warp_tile_band : (V >= 12 ? 4 : 1));
    };
    if (nhwc) {
        if (mode == BEV_FUSE_SUM) go(k_warp_fuse_v2<BEV_FUSE_SUM, OCC, TH, false, true>);
        else if (mode == BEV_FUSE_MEAN) go(k_warp_fuse_v2<BEV_FUSE_MEAN, OCC, TH, false, true>);
        else go(k_warp_fuse_v2<BEV_FUSE_MAX, OCC, TH, false, true>);
    } else if (mode == BEV_FUSE_SUM)
        ck ? go(k_warp_fuse_v2<BEV_FUSE_SUM, OCC, TH, true>) : go(k_warp_fuse_v2<BEV_FUSE_SUM, OCC, TH, false>);
    else if (mode == BEV_FUSE_MEAN)
        ck ? go(k_warp_fuse_v2<BEV_FUSE_MEAN, OCC, TH, true>) : go(k_warp_fuse_v2<BEV_FUSE_MEAN, OCC, TH, false>);
    else
        ck ? go(k_warp_fuse_v2<BEV_FUSE_MAX, OCC, TH, true>) : go(k_warp_fuse_v2<BEV_FUSE_MAX, OCC, TH, false>);
    return last();
}

// V for which k_warp_fuse_v3's fp32 mean division (w3_div) is exact for every input but -0: bit V - 1, from the
// exhaustive check tools/verify_div_markstein_fix.c (other V divide through double, div_rcp).
constexpr uint64_t W3_FASTDIV_V = MARKSTEIN_EXACT_V;

int launch_fuse_v3(const float *feats, int64_t sN, int64_t sH, int64_t sW, const float *Hmat, const float *xs,
                   const float *ys, int B, int V, int C, int Hf, int Wf, float sx, float sy, int Hb, int Wb, int mode,
                   float *out, hipStream_t st, uint2 *boxes) {
    const int ntx = (Wb + 15) / 16, nty = (Hb + 15) / 16, ntiles = ntx * nty;
    // 3 workgroups per CU: pool + zero pixel <= 160 KiB / 3
    const int pool = g_warp_pool_kb ? g_warp_pool_kb * 1024 : ((163840 / 3 - 256 - 64) & ~1023);
    hipLaunchKernelGGL((k_warp_boxes<16, 16>), dim3((unsigned)(((int64_t)ntiles * V + 255) / 256), B), dim3(256), 0,
                       st, Hmat, xs, ys, V, Hf, Wf, sx, sy, Hb, Wb, pool / W3_PIX, nty, boxes, nullptr, nullptr, 0);
    const int fastdiv = (V >= 1 && V <= 64 && ((W3_FASTDIV_V >> (V - 1)) & 1)) ? 1 : 0;
    const size_t lds = (size_t)pool + 256;
    if (mode == BEV_FUSE_SUM)
        hipLaunchKernelGGL(k_warp_fuse_v3<BEV_FUSE_SUM>, dim3(ntiles, B), dim3(FT_NT), lds, st, feats, sN, sH, sW, Hmat,
                           xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, out, pool, boxes, fastdiv);
    else
        hipLaunchKernelGGL(k_warp_fuse_v3<BEV_FUSE_MEAN>, dim3(ntiles, B), dim3(FT_NT), lds, st, feats, sN, sH, sW,
                           Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, out, pool, boxes, fastdiv);
    return last();
}

// LDS image pool of k_warp_fuse_v2 for `mode` (the corner boxes' fit test depends on it)
inline int v2_pool_bytes(int mode) {
    const int kb = g_warp_pool_kb > 0 && g_warp_pool_kb < 8 ? 8 : g_warp_pool_kb;  // v2 needs >= 8 KiB
    if (mode == BEV_FUSE_MAX) return kb ? kb * 1024 : 72 * 1024;  // MAX: 2 workgroups per CU
    const int pool3 = (163840 / WARP_OCC - V2_FIXED - 64) & ~1023;
    return kb ? kb * 1024 : (pool3 < 49 * 1024 ? pool3 : 49 * 1024);
}

inline int launch_fuse_v2(const float *feats, int64_t sN, int64_t sH, int64_t sW, const float *Hmat,
                          const float *xs, const float *ys, int B, int V, int C, int Hf, int Wf, float sx, float sy,
                          int Hb, int Wb, int mode, float *out, hipStream_t st, uint2 *boxes, bool boxes_ready, int rpr) {
    if (mode == BEV_FUSE_MAX)  // MAX's extra live state spills at 3 workgroups per CU
        return launch_fuse_v2_occ<2>(feats, sN, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, st,
                                     v2_pool_bytes(mode), boxes, boxes_ready, rpr);
    return launch_fuse_v2_occ<WARP_OCC>(feats, sN, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out,
                                        st, v2_pool_bytes(mode), boxes, boxes_ready, rpr);
}

int warp_fuse_impl(const float *feats, int64_t sN, int64_t sC, int64_t sH, int64_t sW, const float *Hmat,
                   const float *xs, const float *ys, int B, int V, int C, int Hf, int Wf, float sx, float sy, int Hb,
                   int Wb, int mode, float *out, void *workspace, int64_t workspace_bytes, void *stream,
                   bool boxes_ready, int rpr);

}  // namespace

namespace bev {
int warp_bwd_pool_floats() { return g_warp_bwd_pool > 0 ? g_warp_bwd_pool : WARP_BWD_POOL_MAX; }

int warp_tune(int knob, int value) {
    int *slot = nullptr;
    bool ok = false;
    switch (knob) {
        case BEV_TUNE_WARP_POOL_KB:
            slot = &g_warp_pool_kb;
            ok = value >= 0 && value <= 150;  // v3 takes any pool; v2 clamps to >= 8 KiB
            break;
        case BEV_TUNE_WARP_KERNEL:
            slot = &g_warp_kernel;
            ok = value >= 0 && value <= 3;
            break;
        case BEV_TUNE_WARP_BWD_POOL:
            slot = &g_warp_bwd_pool;
            ok = value >= 0 && value <= WARP_BWD_POOL_MAX;
            break;
        case BEV_TUNE_WARP_PERSIST:
            slot = &g_warp_persist;
            ok = value >= 0 && value <= 2;
            break;
        case BEV_TUNE_WARP_SPAN:
            slot = &g_warp_span_pct;
            ok = value >= 0 && value <= 100;
            break;
        case BEV_TUNE_WARP_TILE_BAND:
            slot = &g_warp_tile_band;
            ok = value >= 0 && value <= 64;
            break;
        default:
            return BEV_ERR_ARGS;
    }
    if (!ok) return BEV_ERR_ARGS;
    const int old = *slot;
    *slot = value;
    return old;
}
}  // namespace bev

extern "C" {

int bev_abi_version(void) { return 12; }

#if WARP_STAMP
int bev_warp_stamp_read(unsigned long long *host, int n) {  // timing builds only
    if (n > 16384 * STAMP_N) n = 16384 * STAMP_N;
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_warp_stamp), (size_t)n * sizeof(unsigned long long), 0,
                                    hipMemcpyDeviceToHost);
}
#endif

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
    if (N < 0 || Hf <= 0 || Wf <= 0 || Hb < 0 || Wb < 0 || N > 65535) return BEV_ERR_ARGS;
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

int64_t bev_ipm_warp_fuse_workspace_bytes(int B, int V, int Hb, int Wb) {
    if (B < 0 || V <= 0 || Hb < 0 || Wb < 0) return BEV_ERR_ARGS;
    // per-(frame, tile, view) footprint boxes (16 x 16 tiles, v2 and v3; A/B builds of v2 with 8 x 32 tiles have as
    // many), the work-queue words and the span tables
    constexpr int TH = WARP_TILE_H, TW = FT_NT / TH;
    const int64_t nt = (((int64_t)Wb + TW - 1) / TW) * (((int64_t)Hb + TH - 1) / TH);
    return BOX_HDR + (int64_t)B * nt * V * (int64_t)sizeof(uint2) + WQ_WORDS * (int64_t)sizeof(unsigned) +
           (int64_t)B * nt * V * SPAN_ROWS * (int64_t)sizeof(unsigned);
}

int bev_ipm_warp_fuse_f32(const float *feats, int64_t sN, int64_t sC, int64_t sH, int64_t sW, const float *Hmat,
                          const float *xs, const float *ys, int B, int V, int C, int Hf, int Wf, float sx, float sy,
                          int Hb, int Wb, int mode, float *out, void *stream) {
    return bev_ipm_warp_fuse_ws_f32(feats, sN, sC, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out,
                                    nullptr, 0, stream);
}

int bev_ipm_warp_fuse_ws_f32(const float *feats, int64_t sN, int64_t sC, int64_t sH, int64_t sW, const float *Hmat,
                             const float *xs, const float *ys, int B, int V, int C, int Hf, int Wf, float sx, float sy,
                             int Hb, int Wb, int mode, float *out, void *workspace, int64_t workspace_bytes,
                             void *stream) {
    return warp_fuse_impl(feats, sN, sC, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, workspace,
                          workspace_bytes, stream, false, Hb);
}

int bev_ipm_warp_fuse_pre_f32(const float *feats, int64_t sN, int64_t sC, int64_t sH, int64_t sW, const float *Hmat,
                              const float *xs, const float *ys, int B, int V, int C, int Hf, int Wf, float sx, float sy,
                              int Hb, int Wb, int mode, float *out, void *workspace, int64_t workspace_bytes,
                              void *stream) {
    return warp_fuse_impl(feats, sN, sC, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, workspace,
                          workspace_bytes, stream, true, Hb);
}

int bev_ipm_warp_fuse_nhwc_f32(const float *feats, int64_t sN, int64_t sC, int64_t sH, int64_t sW, const float *Hmat,
                               const float *xs, const float *ys, int B, int V, int C, int Hf, int Wf, float sx,
                               float sy, int Hb, int Wb, int mode, float *out, void *workspace,
                               int64_t workspace_bytes, int boxes_ready, void *stream) {
    return warp_fuse_impl(feats, sN, sC, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, workspace,
                          workspace_bytes, stream, boxes_ready != 0, 0);
}

int bev_ipm_warp_fuse_chunked_f32(const float *feats, int64_t sN, int64_t sC, int64_t sH, int64_t sW,
                                  const float *Hmat, const float *xs, const float *ys, int B, int V, int C, int Hf,
                                  int Wf, float sx, float sy, int Hb, int Wb, int mode, int rows_per_chunk, float *out,
                                  void *workspace, int64_t workspace_bytes, int boxes_ready, void *stream) {
    if (rows_per_chunk <= 0 || Hb <= 0) return BEV_ERR_ARGS;
    return warp_fuse_impl(feats, sN, sC, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, workspace,
                          workspace_bytes, stream, boxes_ready != 0, rows_per_chunk < Hb ? rows_per_chunk : Hb);
}

int bev_ipm_warp_fuse_boxes_f32(const float *Hmat, const float *xs, const float *ys, int B, int V, int Hf, int Wf,
                                float sx, float sy, int Hb, int Wb, int mode, void *workspace, int64_t workspace_bytes,
                                void *stream) {
    if (!Hmat || !xs || !ys || B < 0 || V <= 0 || V > V2_MAXV || Hf <= 0 || Wf <= 0 || Hb < 0 || Wb < 0 || B > 65535)
        return BEV_ERR_ARGS;
    if (mode < BEV_FUSE_SUM || mode > BEV_FUSE_MAX || Hf >= 16384 || Wf >= 16384) return BEV_ERR_ARGS;
    const int64_t need = bev_ipm_warp_fuse_workspace_bytes(B, V, Hb, Wb);
    if (!workspace || workspace_bytes < need || ((uintptr_t)workspace & 15) != 0) return BEV_ERR_ARGS;
    if (B == 0 || Hb == 0 || Wb == 0) return 0;
    constexpr int TH = WARP_TILE_H, TW = FT_NT / TH;
    const int ntiles = ((Wb + TW - 1) / TW) * ((Hb + TH - 1) / TH);
    const int maxpix = v2_pool_bytes(mode) / (V2_SL * 16) - 4;  // k_warp_fuse_v2's own pool test
    unsigned *queue = reinterpret_cast<unsigned *>(reinterpret_cast<unsigned char *>(workspace) + BOX_HDR +
                                                   (int64_t)B * ntiles * V * (int64_t)sizeof(uint2));
    hipLaunchKernelGGL((k_warp_boxes<TH>), dim3((unsigned)(((int64_t)ntiles * V + 255) / 256), B), dim3(256), 0,
                       (hipStream_t)stream, Hmat, xs, ys, V, Hf, Wf, sx, sy, Hb, Wb, maxpix, (Hb + TH - 1) / TH,
                       reinterpret_cast<uint2 *>(reinterpret_cast<unsigned char *>(workspace) + BOX_HDR), queue,
                       span_tables(queue, g_warp_persist != 0), g_warp_span_pct);
    return last();
}

}  // extern "C"

namespace {
int warp_fuse_impl(const float *feats, int64_t sN, int64_t sC, int64_t sH, int64_t sW, const float *Hmat,
                   const float *xs, const float *ys, int B, int V, int C, int Hf, int Wf, float sx, float sy, int Hb,
                   int Wb, int mode, float *out, void *workspace, int64_t workspace_bytes, void *stream,
                   bool boxes_ready, int rpr) {
    if (B < 0 || V <= 0 || C < 0 || Hf <= 0 || Wf <= 0 || Hb < 0 || Wb < 0 || B > 65535) return BEV_ERR_ARGS;
    if ((int64_t)Hf * Wf >= (1 << 22)) return BEV_ERR_ARGS;  // fast_div range of the footprint index
    if (mode < BEV_FUSE_SUM || mode > BEV_FUSE_MAX) return BEV_ERR_ARGS;
    if (B == 0 || C == 0 || Hb == 0 || Wb == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    // LDS-DMA kernels: NHWC 64-channel chunks, 16-B aligned pixels, 32-bit element offsets
    // inside a map, and 64 output planes addressable by one buffer descriptor (store_chunk)
    const bool dma_ok = (sC == 1) && (C % 64 == 0) && V <= V2_MAXV && Hf < 16384 && Wf < 16384 &&
                        ((int64_t)Hf * sH < (1ll << 31)) && ((int64_t)Wf * sW < (1ll << 31)) &&
                        (((uintptr_t)feats & 15) == 0) && (sW % 4 == 0) && (sH % 4 == 0) && (sN % 4 == 0) &&
                        (int64_t)Hb * Wb * 64 * (int64_t)sizeof(float) < (1ll << 32);
    if (rpr == 0) {  // channels-last output: the LDS-DMA kernel only, a frame's output < 2 GiB (per-lane offsets),
                     // the parking area (4 waves x 64 cells x 144 B) inside the pool
        if (!dma_ok || g_warp_kernel == 1 || (int64_t)Hb * Wb * C * (int64_t)sizeof(float) >= (1ll << 31) ||
            v2_pool_bytes(mode) < 4 * 64 * 36 * (int)sizeof(float))
            return BEV_ERR_ARGS;
    } else if (rpr != Hb) {  // rank-chunk-major output: the LDS-DMA kernel only, whole output < 2 GiB (per-lane offsets)
        const int64_t nck = ((int64_t)Hb + rpr - 1) / rpr;
        if (!dma_ok || g_warp_kernel == 1 || nck * rpr * (int64_t)B * C * Wb * (int64_t)sizeof(float) >= (1ll << 31))
            return BEV_ERR_ARGS;
    }
    if (dma_ok && g_warp_kernel != 1) {
        const int64_t need = bev_ipm_warp_fuse_workspace_bytes(B, V, Hb, Wb);
        uint2 *boxes = (workspace && workspace_bytes >= need && ((uintptr_t)workspace & 15) == 0)
                           ? reinterpret_cast<uint2 *>(reinterpret_cast<unsigned char *>(workspace) + BOX_HDR)
                           : nullptr;
        // default: the per-view LDS-DMA kernel; 3: the DPP-row kernel (sum / mean, footprint boxes in the workspace;
        // measured slower at the bench geometry, profiles/r04g_warp_v3_vs_v2.txt)
        if (g_warp_kernel == 3 && boxes && mode != BEV_FUSE_MAX && rpr == Hb &&
            (int64_t)Hf * sH + (int64_t)Wf * sW < (1ll << 31))
            return launch_fuse_v3(feats, sN, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, st,
                                  boxes);
        return launch_fuse_v2(feats, sN, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, st, boxes,
                              boxes_ready, rpr);
    }
    if (C <= 4)
        return launch_fuse_ck<4>(feats, sN, sC, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, st);
    if (C <= 16)
        return launch_fuse_ck<16>(feats, sN, sC, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, st);
    if (C <= 32)
        return launch_fuse_ck<32>(feats, sN, sC, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, st);
    return launch_fuse_ck<64>(feats, sN, sC, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, st);
}
}  // namespace

extern "C" {

int bev_view_max_bwd_f32(const float *x, const float *gout, int B, int V, int64_t M, float *gx, void *stream) {
    if (B < 0 || V <= 0 || M < 0 || B > 65535) return BEV_ERR_ARGS;
    if (B == 0 || M == 0) return 0;
    int64_t blocks = (M + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_view_max_bwd, dim3((unsigned)blocks, B), dim3(256), 0, (hipStream_t)stream, x, gout, V, M, gx);
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
