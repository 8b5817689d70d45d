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

using namespace bev;

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
            "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(src), "s"(dst)
            : "memory");
    }
}

// The same DMA through a buffer descriptor based at the block origin (byte strides sH4 / sW4 < 2^24, every
// byte offset of the feature map < 2^31 -- the launcher checks): per lane only 24-bit integer products and a
// 32-bit offset, no 64-bit address arithmetic (slot / 17 as (slot * 61681) >> 20, exact for slot < 69632,
// i.e. footprints < 4096 pixels).  The pad slot (sl == 16) re-reads channel group 0 (any in-range address).
typedef int v4i_t __attribute__((ext_vector_type(4)));
template <int S = 17>
__device__ __forceinline__ void dma_block_buf(const float *__restrict__ f, int sH4, int sW4, int sx0, int sy0, int sbw,
                                              int npix, unsigned char *smem, int off, int wave, int lane,
                                              int nwaves = FT_NT / 64) {
    static_assert(S == 17, "slot decomposition assumes 17 slots per pixel");
    if (WARP_ABLATE & 2) return;
    const int ninstr = (npix * S + 63) >> 6;
    const float inv_bw = 1.0f / (float)sbw;
    const uint64_t a = (uint64_t)(uintptr_t)f + (uint64_t)((int64_t)sy0 * sH4 + (int64_t)sx0 * sW4);
    const v4i_t rsrc = {__builtin_amdgcn_readfirstlane((int)(uint32_t)a),
                        __builtin_amdgcn_readfirstlane((int)((uint32_t)(a >> 32) & 0xffffu)), 0x7fffffff, 0x00020000};
    for (int k = wave; k < ninstr; k += nwaves) {
        const unsigned slot = (unsigned)(k * 64 + lane);
        const unsigned p = __umul24(slot, 61681u) >> 20;
        const unsigned sl = slot - ((p << 4) + p);
        int q = (int)((float)p * inv_bw);
        int r = (int)p - (int)__umul24((unsigned)q, (unsigned)sbw);
        const bool hi = r >= sbw, lo = r < 0;
        q += (int)hi - (int)lo;
        r += (lo ? sbw : 0) - (hi ? sbw : 0);
        unsigned voff = __umul24((unsigned)q, (unsigned)sH4) + __umul24((unsigned)r, (unsigned)sW4) + ((sl & 15u) << 4);
        voff = ((int)p < npix) ? voff : 0u;  // tail lanes: any in-range address
        const unsigned dst = (unsigned)__builtin_amdgcn_readfirstlane((int)(lds_base(smem) + off + k * 1024));
        unsigned keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
            "buffer_load_dwordx4 %1, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(voff), "s"(dst), "s"(rsrc)
            : "memory");
    }
}

#ifndef WARP_PIPE
#define WARP_PIPE 1  // fused warp v2: LDS sampling software-pipelined by one 4-channel group (1) or not (0)
#endif
#ifndef WARP_STAMP
#define WARP_STAMP 0  // timing builds only (tools/warp_stamps.py): per-workgroup s_memtime stamps of the v2 phases
#endif
#if WARP_STAMP
__device__ unsigned long long g_warp_stamp[16384 * 6];
#define STAMP(k)                                                                                             \
    do {                                                                                                     \
        const unsigned sb_ = blockIdx.x + blockIdx.y * gridDim.x;                                            \
        if (threadIdx.x == 0 && sb_ < 16384) g_warp_stamp[sb_ * 6 + (k)] = __builtin_amdgcn_s_memtime();      \
    } while (0)
#else
#define STAMP(k) ((void)0)
#endif

#ifndef WARP_TSTORE
#define WARP_TSTORE 0  // fused warp v2: 16-B output stores through a per-wave LDS transpose (1) or 4-B stores (0)
#endif
#ifndef WARP_LANESKIP
#define WARP_LANESKIP 1  // fused warp v2: lanes with no valid tap skip the view's LDS sampling (1, r03 A/B: 1-8 % faster) or read the zero pixel (0)
#endif
#ifndef WARP_DMABUF
#define WARP_DMABUF 0  // fused warp v2: footprint DMA through a buffer descriptor (1; r03m A/B: 1-8 % slower) or 64-bit global addresses (0)
#endif

// Output stores of a 64-channel chunk through a buffer descriptor: SGPR base of
// the chunk, per-lane byte offset of the cell, SGPR byte offset of the channel
// plane -> no per-store address arithmetic.  The dispatcher guarantees the
// chunk (64 planes) spans < 4 GiB.  aux 2 = nt (streaming, written once).
template <int N>
__device__ __forceinline__ void store_chunk(float *chunk, size_t plane, int cell, const float (&acc)[N], int mode,
                                            double rV) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(chunk, 0, (int)(uint32_t)(plane * N * sizeof(float)), 0x00020000);
    const int voff = cell * (int)sizeof(float);
    static_assert(N % 8 == 0, "stores in groups of 8 channels");
    if (WARP_ABLATE & 32) {  // timing only: the same bytes as 1-KiB coalesced 16-B-per-lane stores (wrong layout)
        const int wb = __builtin_amdgcn_readfirstlane(cell) * N * (int)sizeof(float);
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
            const float r = (mode == BEV_FUSE_MEAN && !(WARP_ABLATE & 1)) ? div_rcp(a[u], rV) : a[u];
            if ((WARP_ABLATE & 16) && r != 1.2345e-30f) continue;
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, r), rs, voff,
                                                  (int)(uint32_t)((q0 + u) * plane * sizeof(float)), 2);
        }
    }
}

// Output stores of a whole in-range tile through a per-wave LDS transpose (WARP_TSTORE): each lane holds one
// cell's 64 channels, but the [C][Hb][Wb] output is contiguous along cells, so the lanes first write their values
// (after the mean division) to LDS as [channel][wave's 64 cells], then read back 4 consecutive cells of one
// channel and store them as ONE 16-B store: 16 1-KiB store instructions per wave instead of 64 of 256 B.
// Two passes of 32 channels (8 KiB of LDS per wave).  Cell slot of a lane: its row inside the wave's band x TW +
// its column.  Same values, same addresses as store_chunk: bit-identical output.
template <int TH, int N>
__device__ __forceinline__ void store_tile_t(float *chunk, size_t plane, int row0, int col0, int Wb, int tr, int tc,
                                             const float (&acc)[N], int mode, double rV, unsigned char *smem,
                                             int wave, int lane) {
    constexpr int TW = FT_NT / TH, RB = TH / 4;  // tile width; rows per wave
    static_assert(RB * TW == 64 && TW % 4 == 0, "one wave = 64 cells in whole 4-cell quads");
    float *E = reinterpret_cast<float *>(smem) + wave * (32 * 64);
    const int slot = (tr - wave * RB) * TW + tc;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(chunk, 0, (int)(uint32_t)(plane * N * sizeof(float)), 0x00020000);
    const int g = lane & 15, cq = lane >> 4;            // quad of cells, channel within the instruction's four
    const int r = wave * RB + (4 * g) / TW, c = (4 * g) % TW;
    const int voff = ((row0 + r) * Wb + col0 + c) * (int)sizeof(float);
#pragma unroll
    for (int h = 0; h < N; h += 32) {
#pragma unroll
        for (int u = 0; u < 32; ++u) {
            const float a = acc[h + u];
            E[u * 64 + slot] = (mode == BEV_FUSE_MEAN && !(WARP_ABLATE & 1)) ? div_rcp(a, rV) : a;
        }
        // same-wave LDS ops complete in order: the reads below see these writes
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int ch = 4 * k + cq;
            const f32x4 v = *(const f32x4 *)(E + ch * 64 + 4 * g);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i_t, v), rs, voff,
                                                   (int)(uint32_t)((h + ch) * plane * sizeof(float)), 2);
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
constexpr int V2_MAXV = 64;                         // one view per lane

// Conservative tap bbox of the BEV rectangle [xa, xb] x [ya, yb] (cell
// centres) for homography h; ok = false when the corner bound does not apply.
__device__ Box corner_box(const float *hf, float xa, float xb, float ya, float yb, float sx, float sy, int Wf, int Hf,
                          bool &ok) {
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
    const double lox = fmin(fmax(ixmin - mx, -4.0), (double)Wf + 4.0);
    const double hix = fmin(fmax(ixmax + mx, -4.0), (double)Wf + 4.0);
    const double loy = fmin(fmax(iymin - my, -4.0), (double)Hf + 4.0);
    const double hiy = fmin(fmax(iymax + my, -4.0), (double)Hf + 4.0);
    const int x0 = max((int)floor(lox), 0), x1 = min((int)floor(hix) + 1, Wf - 1);
    const int y0 = max((int)floor(loy), 0), y1 = min((int)floor(hiy) + 1, Hf - 1);
    if (x0 <= x1 && y0 <= y1) b = Box{x0, y0, x1, y1};
    return b;
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
template <int MODE, int N, bool PIPE = true>
__device__ __forceinline__ void sample_view_pipe(float (&acc)[N], const Taps &t, const unsigned char *smem, int ib,
                                                 int sx0, int sy0, int sbw, int zp, int zp0) {
    constexpr int PS = (N / 4 + 1) * 16, NG = N / 4;
    const int pb = ib + ((t.y0 - sy0) * sbw + (t.x0 - sx0)) * PS;
    const unsigned char *a0 = smem + ((t.valid & 1) ? pb : zp0);
    const unsigned char *a1 = smem + ((t.valid & 2) ? pb + PS : zp);
    const unsigned char *a2 = smem + ((t.valid & 4) ? pb + sbw * PS : zp);
    const unsigned char *a3 = smem + ((t.valid & 8) ? pb + (sbw + 1) * PS : zp);
    if (!PIPE) {
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const f32x4 c0 = *(const f32x4 *)(a0 + g * 16), c1 = *(const f32x4 *)(a1 + g * 16);
            const f32x4 c2 = *(const f32x4 *)(a2 + g * 16), c3 = *(const f32x4 *)(a3 + g * 16);
            bilerp4<MODE>(acc, 4 * g, c0, c1, c2, c3, t.w);
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
            n2 = *(const f32x4 *)(a2 + (g + 1) * 16);
            n3 = *(const f32x4 *)(a3 + (g + 1) * 16);
        }
        bilerp4<MODE>(acc, 4 * g, c0, c1, c2, c3, t.w);
        __builtin_amdgcn_sched_barrier(0);  // at most two groups of reads in flight
        if (g < NG - 1) {
            c0 = n0;
            c1 = n1;
            c2 = n2;
            c3 = n3;
        }
    }
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

// Frames per workgroup (FPW = 2, tcache >= 0): a static rig gives every frame of a batch the same homographies
// (Wildtrack's cameras do not move), so the workgroup of a tile runs the frames one after the other and the
// second pass reads each cell's taps from an LDS record written by the first instead of recomputing them:
// (x0, y0) as int16 (-32768: no valid tap along that axis) + the fractional offsets we = ix - floor(ix) and
// n = iy - floor(iy), from which the weights and validity bits are rebuilt with the same fp32 operations
// (bit-identical).  The geometry is compared per view in the prologue; frames that differ take a full pass.
// The same records serve every further 64-channel chunk of a frame.
template <int MODE, int OCC, int TH = 8, int FPW = 1>
__global__ __launch_bounds__(FT_NT, OCC) void k_warp_fuse_v2(const float *__restrict__ feats, int64_t sN, int64_t sH,
                                                          int64_t sW, const float *__restrict__ Hmat,
                                                          const float *__restrict__ xs, const float *__restrict__ ys,
                                                          int B, int V, int C, int Hf, int Wf, float sx, float sy,
                                                          int Hb, int Wb, float *__restrict__ out, int pool,
                                                          int tcache, const uint2 *__restrict__ boxes) {
    constexpr int NW = FT_NT / 64;  // 4 waves
    constexpr int TW = FT_NT / TH;  // tile width in cells
    constexpr int SL = 17, PS = SL * 16;  // DMA slots / bytes per staged pixel (64 channels + pad)
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
    const int tyb = tile / ntx, txb = tile - tyb * ntx;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    STAMP(0);
    int tr, tc;
    tile_cell<TH>(lane, wave, tr, tc);
    // footprint DMA: buffer-descriptor form when the byte strides fit 24 bits and the map 2^31 bytes (uniform)
    const bool bufdma = WARP_DMABUF && sH * 4 < (1 << 24) && sW * 4 < (1 << 24) &&
                        ((int64_t)Hf * sH + (int64_t)Wf * sW) * 4 < (1ll << 31);
    auto dma = [&](const float *fp, int x0, int y0, int w, int n, int o) {
        if (bufdma) dma_block_buf<SL>(fp, (int)sH * 4, (int)sW * 4, x0, y0, w, n, smem, o, wave, lane, NW);
        else dma_block<SL>(fp, (int)sH, (int)sW, x0, y0, w, n, smem, o, wave, lane, NW);
    };
    const int i = tyb * TH + tr;
    const int j = txb * TW + tc;
    const int b0 = blockIdx.y * FPW;
    const bool inside = (i < Hb) && (j < Wb);
    const float cx = xs[inside ? j : 0], cy = ys[inside ? i : 0];
    const size_t plane = (size_t)Hb * Wb;
    const Grid grid = make_grid(Hf, Wf);
    const double rV = recip_uniform(V);  // mean: acc / V via div_rcp (exact)
    if (tid < 16) *(float4 *)(smem + zp + tid * 16) = make_float4(0.f, 0.f, 0.f, 0.f);
    unsigned *btab = reinterpret_cast<unsigned *>(htab + V2_MAXV * 9);  // [V][2] corner boxes, [2 V] same flag
    unsigned *tc0 = reinterpret_cast<unsigned *>(smem + (tcache >= 0 ? tcache : 0));  // [V][256] packed x0, y0
    float2 *tc1 = reinterpret_cast<float2 *>(tc0 + V * FT_NT);                         // [V][256] (we, n)

    // corner boxes of this tile for frame bb, lane v <-> view v, packed in two VGPRs (wave 0 computes them in
    // double, the others read them): lba = x0 | y0 << 16 | (!ok) << 31,  lbb = (x1 + 1) | (y1 + 1) << 16
    // (x1 + 1 == 0: empty).  With FPW = 2 wave 0 also compares frame bb + 1's homographies with bb's.
    unsigned lba = 0, lbb = 0;
    bool same = false;
    auto prologue = [&](int bb, bool check_next) {
        if (WARP_HSCALAR && boxes != nullptr) {  // precomputed by k_warp_boxes (FPW = 1): every wave reads them
            const uint2 bx = lane < V ? boxes[((int64_t)bb * nt + tile) * V + lane] : make_uint2(0u, 0u);
            lba = bx.x;
            lbb = bx.y;
            same = false;
            return;
        }
        if (wave == 0) {
            const int ia = tyb * TH, ib = min(ia + TH - 1, Hb - 1);
            const int ja = txb * TW, jb = min(ja + TW - 1, Wb - 1);
            Box cb{0x7fffffff, 0x7fffffff, -1, -1};
            bool ok = true, eq = true;
            if (lane < V) {
                float hv[9];
                load_h(Hmat, bb * V + lane, hv);
#pragma unroll
                for (int q = 0; q < 9; ++q) htab[lane * 9 + q] = hv[q];  // visible after the barrier below
                if (check_next) {
                    float hn[9];
                    load_h(Hmat, (bb + 1) * V + lane, hn);
#pragma unroll
                    for (int q = 0; q < 9; ++q) eq = eq && (__float_as_uint(hn[q]) == __float_as_uint(hv[q]));
                }
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
            const bool all_eq = check_next && __ballot(lane < V && !eq) == 0ull;
            if (lane == 0) btab[2 * V2_MAXV] = all_eq ? 1u : 0u;
        }
        __syncthreads();
        lba = lane < V ? btab[2 * lane] : 0u;
        lbb = lane < V ? btab[2 * lane + 1] : 0u;
        same = btab[2 * V2_MAXV] != 0u;
    };
    prologue(b0, FPW > 1 && b0 + 1 < B && tcache >= 0);
    STAMP(1);
    auto box_of = [&](int v) {
        const unsigned a = (unsigned)__builtin_amdgcn_readlane((int)lba, v);
        const unsigned c = (unsigned)__builtin_amdgcn_readlane((int)lbb, v);
        return Box{(int)(a & 0xffffu), (int)((a >> 16) & 0x7fffu), (int)(c & 0xffffu) - 1, (int)(c >> 16) - 1};
    };
    auto ok_of = [&](int v) { return ((unsigned)__builtin_amdgcn_readlane((int)lba, v) >> 31) == 0u; };

    float ccx = cx, ccy = cy;  // made opaque per chunk (see the chunk loop)
    bool cache_rd = false;     // this chunk reads the tap records (written by an earlier chunk / frame)
    int hbase = b0 * V;        // homography row of view 0 of the frame being sampled
    auto taps_of = [&](int v) {
        Taps t;
        if (cache_rd) {
            const unsigned pk = tc0[v * FT_NT + tid];
            const float2 f = tc1[v * FT_NT + tid];
            const int x0s = (int)(short)(pk & 0xffffu), y0s = (int)(short)(pk >> 16);
            const float e = 1.0f - f.x, s = 1.0f - f.y;  // taps_from_ixy's arithmetic
            t.w[0] = s * e;
            t.w[1] = s * f.x;
            t.w[2] = f.y * e;
            t.w[3] = f.y * f.x;
            const bool vx0 = x0s >= 0 && x0s < Wf, vx1 = x0s >= -1 && x0s + 1 < Wf;
            const bool vy0 = y0s >= 0 && y0s < Hf, vy1 = y0s >= -1 && y0s + 1 < Hf;
            t.valid = (unsigned)(vx0 & vy0) | ((unsigned)(vx1 & vy0) << 1) | ((unsigned)(vx0 & vy1) << 2) |
                      ((unsigned)(vx1 & vy1) << 3);
            t.x0 = (vx0 | vx1) ? x0s : 0;
            t.y0 = (vy0 | vy1) ? y0s : 0;
            return t;
        }
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
        if (FPW > 1 && tcache >= 0) {
            const float xw = __builtin_floorf(ix), yn = __builtin_floorf(iy);
            const bool xv = xw >= -1.0f && xw < grid.fWf, yv = yn >= -1.0f && yn < grid.fHf;  // vx0 | vx1, vy0 | vy1
            const int x0s = (inside && xv) ? t.x0 : -32768, y0s = (inside && yv) ? t.y0 : -32768;
            tc0[v * FT_NT + tid] = ((unsigned)x0s & 0xffffu) | ((unsigned)y0s << 16);
            tc1[v * FT_NT + tid] = make_float2(ix - xw, iy - yn);
        }
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

    for (int pass = 0; pass < FPW; ++pass) {
      const int b = b0 + pass;
      if (b >= B) break;
      hbase = b * V;
      if (pass > 0 && !same) {  // this frame's geometry differs: its own boxes and homographies
          __syncthreads();
          prologue(b, false);
      }
      for (int c0 = 0; c0 < C; c0 += 64) {
        cache_rd = FPW > 1 && tcache >= 0 && (c0 > 0 || (pass > 0 && same));
        ccx = cx;
        ccy = cy;
        asm volatile("" : "+v"(ccx), "+v"(ccy));  // keep taps per chunk (no hoisting + spills)
        float acc[64];
#pragma unroll
        for (int q = 0; q < 64; ++q) acc[q] = (MODE == BEV_FUSE_MAX) ? -__builtin_inff() : 0.0f;
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
        const int v_first = next_live(-1);
        // prologue: DMA of the first live view (if its corner box applies and fits)
        Box bn = box_of(v_first < V ? v_first : 0);
        int offn = -1;
        if (v_first < V) {
            const int npix = (bn.x1 - bn.x0 + 1) * (bn.y1 - bn.y0 + 1);
            if (ok_of(v_first) && bn.x1 >= 0 && npix <= maxpix) {
                offn = 0;
                dma(fb + (int64_t)v_first * sN, bn.x0, bn.y0, bn.x1 - bn.x0 + 1, npix, 0);
            }
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
        STAMP(2);

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
                    dma(f, bx.x0, bx.y0, bw, bw * bh, 0);
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
                            dma(f, sx0, sy0, sbw, sbw * sbh, 0);
                        }
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        __syncthreads();
                        const bool mine = single ? true : (t.valid != 0 && mkx == kx && mky == ky);
                        const bool go = single ? wave_any : (__ballot(mine) != 0ull);
                        if (go) sample_view<MODE, 1, 64>(acc, t, mine, v, smem, 0, sx0, sy0, sbw, zp);
                        else if (single) zero_view<MODE>(acc, v);
                    }
                done = true;
                __syncthreads();  // every wave is done with the staged blocks before DMA(v+1) reuses the pool
            }
            // ---- look ahead: DMA of the next live view beside the live image of view v ----
            if (vn < V) {
                bn = box_of(vn);
                offn = -1;
                const int npix = (bn.x1 - bn.x0 + 1) * (bn.y1 - bn.y0 + 1);
                if (ok_of(vn) && bn.x1 >= 0 && npix <= maxpix) {
                    // consecutive images anchor at opposite ends of the pool: they coexist
                    // whenever their sizes add up to at most the pool
                    const int need = ((npix * SL + 63) >> 6) * 1024;
                    if (done || off < 0) offn = 0;
                    else if (off == 0) {
                        if (((bw * bh * SL + 63) >> 6) * 1024 + need <= pool) offn = pool - need;
                    } else if (need <= off) offn = 0;
                    if (offn >= 0)
                        dma(fb + (int64_t)vn * sN, bn.x0, bn.y0, bn.x1 - bn.x0 + 1, npix, offn);
                }
            }
            // ---- sample view v from its prefetched image ------------------------------
            if (!done) {
                if (!have_t) t = taps_of(v);
                if (WARP_ABLATE & 4) acc[0] += t.w[0] * t.w[3] + (float)(t.x0 + t.y0 + (int)t.valid);
                else if (__ballot(t.valid != 0) != 0ull) {
                    // WARP_LANESKIP: lanes without a valid tap leave the LDS reads to the others (their sample is
                    // +0: acc + 0 == acc exactly, max(acc, 0) for the max mode)
                    if (!WARP_LANESKIP || t.valid)
                        sample_view_pipe<MODE, 64, WARP_PIPE != 0>(acc, t, smem, off, bx.x0, bx.y0, bw, zp, zp);
                    else zero_view<MODE>(acc, v);
                } else zero_view<MODE>(acc, v);
            } else if (empty) {
                zero_view<MODE>(acc, v);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of view v+1 landed
            __syncthreads();  // all of it landed; image of view v and red[] are free
        }
        STAMP(3);
        if (WARP_TSTORE && pool >= 4 * 32 * 64 * 4 && (tyb + 1) * TH <= Hb && (txb + 1) * TW <= Wb && Wb % 4 == 0) {
            store_tile_t<TH>(out + ((size_t)b * C + c0) * plane, plane, tyb * TH, txb * TW, Wb, tr, tc, acc, MODE, rV,
                             smem, wave, lane);
            __syncthreads();  // the transpose's LDS is free before the next chunk / frame stages into the pool
        } else if (inside) {
            store_chunk(out + ((size_t)b * C + c0) * plane, plane, i * Wb + j, acc, MODE, rV);
        }
        STAMP(4);
      }
    }
}

// -------------------------------------------------------------------------
// persistent form of k_warp_fuse_v2 (C == 64, corner boxes from the workspace; BEV_TUNE_WARP_KERNEL 3)
// -------------------------------------------------------------------------
// The ablation of k_warp_fuse_v2 shows its phases adding up: the ~5400 workgroups of a batch-2 launch
// run in ~7 lock-step rounds, each computing and then storing, so the 354 MB of output stores (61 us alone) barely
// overlap the sampling.  Here a workgroup walks (frame, tile) items with stride gridDim.x, and before it stores item
// k it already reads item k + 1's corner boxes, issues the LDS-DMA of k + 1's first live footprint and computes that
// view's taps: the stores then drain while the next item starts.  vmcnt counts loads, stores and LDS-DMA in issue
// order, so the DMA must be OLDER than the stores to be waited for without them: the wait is vmcnt(63) (every
// operation but the 63 youngest -- the stores -- is complete).  Per item the arithmetic, the view order and the
// LDS images are exactly k_warp_fuse_v2's: bit-identical output.
template <int MODE, int OCC, int TH>
__global__ __launch_bounds__(FT_NT, OCC) void k_warp_fuse_p(const float *__restrict__ feats, int64_t sN, int64_t sH,
                                                         int64_t sW, const float *__restrict__ Hmat,
                                                         const float *__restrict__ xs, const float *__restrict__ ys,
                                                         int B, int V, int Hf, int Wf, float sx, float sy, int Hb,
                                                         int Wb, float *__restrict__ out, int pool,
                                                         const uint2 *__restrict__ boxes) {
    constexpr int NW = FT_NT / 64;
    constexpr int TW = FT_NT / TH;
    constexpr int SL = 17, PS = SL * 16;
    constexpr int C = 64;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int zp = pool;
    int *red = reinterpret_cast<int *>(smem + pool + 256);
    const int maxpix = pool / PS - 4;
    const int ntx = (Wb + TW - 1) / TW, nty = (Hb + TH - 1) / TH, nt = ntx * nty;
    const int nitems = nt * B;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int tr, tc;
    tile_cell<TH>(lane, wave, tr, tc);
    const size_t plane = (size_t)Hb * Wb;
    const Grid grid = make_grid(Hf, Wf);
    const double rV = recip_uniform(V);
    if (tid < 16) *(float4 *)(smem + zp + tid * 16) = make_float4(0.f, 0.f, 0.f, 0.f);
    auto dma = [&](const float *fp, int x0, int y0, int w, int n, int o) {
        dma_block<SL>(fp, (int)sH, (int)sW, x0, y0, w, n, smem, o, wave, lane, NW);
    };
    // per-item state
    struct Item {
        int b, tyb, txb, i, j;
        bool inside;
        float cx, cy;
        unsigned lba, lbb;
    };
    auto setup = [&](int item, Item &it) {
        it.b = item / nt;
        int tile = item - it.b * nt;
        {  // XCD-aware tile order within a frame, as k_warp_fuse_v2
            const int q = nt / 8, r = nt % 8, x = tile % 8;
            tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + tile / 8;
        }
        it.tyb = tile / ntx;
        it.txb = tile - it.tyb * ntx;
        it.i = it.tyb * TH + tr;
        it.j = it.txb * TW + tc;
        it.inside = (it.i < Hb) && (it.j < Wb);
        it.cx = xs[it.inside ? it.j : 0];
        it.cy = ys[it.inside ? it.i : 0];
        const uint2 bx = lane < V ? boxes[((int64_t)it.b * nt + tile) * V + lane] : make_uint2(0u, 0u);
        it.lba = bx.x;
        it.lbb = bx.y;
    };
    auto box_of = [&](const Item &it, int v) {
        const unsigned a = (unsigned)__builtin_amdgcn_readlane((int)it.lba, v);
        const unsigned c = (unsigned)__builtin_amdgcn_readlane((int)it.lbb, v);
        return Box{(int)(a & 0xffffu), (int)((a >> 16) & 0x7fffu), (int)(c & 0xffffu) - 1, (int)(c >> 16) - 1};
    };
    auto ok_of = [&](const Item &it, int v) {
        return ((unsigned)__builtin_amdgcn_readlane((int)it.lba, v) >> 31) == 0u;
    };
    auto live = [&](const Item &it, int u) { return !ok_of(it, u) || box_of(it, u).x1 >= 0; };
    auto taps_of = [&](const Item &it, int v, float ccx, float ccy) {
        float h[9];
#pragma unroll
        for (int q = 0; q < 9; ++q) h[q] = Hmat[__builtin_amdgcn_readfirstlane((it.b * V + v) * 9) + q];
        float ix, iy;
        cell_ixy(h, ccx, ccy, grid, sx, sy, ix, iy);
        Taps t = taps_from_ixy(ix, iy, grid);
        if (!it.inside) t.valid = 0;
        return t;
    };
    // head of an item: its first live view, the DMA of that view's footprint (when its corner box applies and fits)
    // and that view's taps -- everything before the first barrier of the item
    struct Head {
        int v_first, offn;
        Box bn;
        Taps tf;
        bool have_f;
    };
    auto head = [&](const Item &it, Head &hd) {
        int u = 0;
        while (u < V && !live(it, u)) ++u;
        hd.v_first = u;
        hd.bn = box_of(it, u < V ? u : 0);
        hd.offn = -1;
        hd.have_f = false;
        if (u < V) {
            const Box &bn = hd.bn;
            const int npix = (bn.x1 - bn.x0 + 1) * (bn.y1 - bn.y0 + 1);
            if (ok_of(it, u) && bn.x1 >= 0 && npix <= maxpix) {
                hd.offn = 0;
                dma(feats + (int64_t)(it.b * V + u) * sN, bn.x0, bn.y0, bn.x1 - bn.x0 + 1, npix, 0);
            }
            if (ok_of(it, u)) {
                float ccx = it.cx, ccy = it.cy;
                asm volatile("" : "+v"(ccx), "+v"(ccy));
                hd.tf = taps_of(it, u, ccx, ccy);
                hd.have_f = true;
            }
        }
    };

    int item = blockIdx.x;
    if (item >= nitems) return;
    Item cur;
    Head hd;
    setup(item, cur);
    head(cur, hd);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // zero pixel + image of the first live view
    while (true) {
        float ccx = cur.cx, ccy = cur.cy;
        asm volatile("" : "+v"(ccx), "+v"(ccy));  // taps per view, not hoisted
        float acc[C];
#pragma unroll
        for (int q = 0; q < C; ++q) acc[q] = (MODE == BEV_FUSE_MAX) ? -__builtin_inff() : 0.0f;
        if (hd.v_first > 0) zero_view<MODE>(acc, 0);  // views before the first live one contribute 0 (max: max(acc, 0))
        const float *fb = feats + (int64_t)(cur.b * V) * sN;
        auto next_live = [&](int u) {
            ++u;
            while (u < V && !live(cur, u)) {
                zero_view<MODE>(acc, u);
                ++u;
            }
            return u;
        };
        Box bn = hd.bn;
        int offn = hd.offn;
        bool have_f = hd.have_f;
        for (int v = hd.v_first, vn; v < V; v = vn) {
            vn = next_live(v);
            Box bx = bn;
            const int off = offn;
            const float *f = fb + (int64_t)v * sN;
            Taps t;
            bool have_t = false;
            if (have_f) {
                t = hd.tf;
                have_t = true;
                have_f = false;
            }
            if (!ok_of(cur, v)) {
                t = taps_of(cur, v, ccx, ccy);
                have_t = true;
                put_box<NW>(red, wave_box(t), wave, lane);
                __syncthreads();
                bx = get_box<NW>(red);
            }
            const bool empty = bx.x1 < 0;
            const int bw = bx.x1 - bx.x0 + 1, bh = bx.y1 - bx.y0 + 1;
            bool done = empty;
            if (!done && off < 0) {
                int wb = bw, hb = bh, nbx = 1, nby = 1;
                if (bw * bh > maxpix) {
                    wb = (2 * bw <= maxpix) ? bw : maxpix / 2;
                    hb = min(bh, maxpix / wb);
                    nbx = (wb >= bw) ? 1 : (bw - 2) / (wb - 1) + 1;
                    nby = (hb >= bh) ? 1 : (bh - 2) / (hb - 1) + 1;
                }
                const bool single = (nbx == 1) && (nby == 1);
                if (single) dma(f, bx.x0, bx.y0, bw, bw * bh, 0);
                if (!have_t) {
                    t = taps_of(cur, v, ccx, ccy);
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
                            __syncthreads();
                            dma(f, sx0, sy0, sbw, sbw * sbh, 0);
                        }
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        __syncthreads();
                        const bool mine = single ? true : (t.valid != 0 && mkx == kx && mky == ky);
                        const bool go = single ? wave_any : (__ballot(mine) != 0ull);
                        if (go) sample_view<MODE, 1, 64>(acc, t, mine, v, smem, 0, sx0, sy0, sbw, zp);
                        else if (single) zero_view<MODE>(acc, v);
                    }
                done = true;
                __syncthreads();
            }
            if (vn < V) {
                bn = box_of(cur, vn);
                offn = -1;
                const int npix = (bn.x1 - bn.x0 + 1) * (bn.y1 - bn.y0 + 1);
                if (ok_of(cur, vn) && bn.x1 >= 0 && npix <= maxpix) {
                    const int need = ((npix * SL + 63) >> 6) * 1024;
                    if (done || off < 0) offn = 0;
                    else if (off == 0) {
                        if (((bw * bh * SL + 63) >> 6) * 1024 + need <= pool) offn = pool - need;
                    } else if (need <= off) offn = 0;
                    if (offn >= 0) dma(fb + (int64_t)vn * sN, bn.x0, bn.y0, bn.x1 - bn.x0 + 1, npix, offn);
                }
            }
            if (!done) {
                if (!have_t) t = taps_of(cur, v, ccx, ccy);
                if (__ballot(t.valid != 0) != 0ull) {
                    if (!WARP_LANESKIP || t.valid)
                        sample_view_pipe<MODE, 64, WARP_PIPE != 0>(acc, t, smem, off, bx.x0, bx.y0, bw, zp, zp);
                    else zero_view<MODE>(acc, v);
                } else zero_view<MODE>(acc, v);
            } else if (empty) {
                zero_view<MODE>(acc, v);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();  // image of view v and red[] are free
        }
        // the next item's boxes, first footprint DMA and first taps go out BEFORE this item's stores
        const int nitem = item + gridDim.x;
        const bool more = nitem < nitems;
        Item nxt;
        Head nh;
        if (more) {
            setup(nitem, nxt);
            head(nxt, nh);
        }
        const bool any_in = __ballot(cur.inside) != 0ull;  // the wave issues its 64 stores (else none at all)
        if (cur.inside)
            store_chunk(out + (size_t)cur.b * C * plane, plane, cur.i * Wb + cur.j, acc, MODE, rV);
        if (!more) break;
        // the DMA is older than this wave's 64 stores: all but the 63 youngest operations = the DMA has landed
        if (any_in) asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        cur = nxt;
        hd = nh;
        item = nitem;
    }
}

template <int OCC>
int launch_fuse_p(const float *feats, int64_t sN, int64_t sH, int64_t sW, const float *Hmat, const float *xs,
                  const float *ys, int B, int V, int Hf, int Wf, float sx, float sy, int Hb, int Wb, int mode,
                  float *out, hipStream_t st, int pool, uint2 *boxes);

// Corner boxes of every (frame, tile, view) for k_warp_fuse_v2 (FPW = 1), one thread each: the tile prologue's
// arithmetic (corner_box + the pool-size test) moved out of the sampling kernel, whose workgroups then start
// with one 8-byte load per view instead of a double-precision latency chain on one wave while three wait.
template <int TH, int TW = FT_NT / TH>
__global__ __launch_bounds__(256) void k_warp_boxes(const float *__restrict__ Hmat, const float *__restrict__ xs,
                                                    const float *__restrict__ ys, int V, int Hf, int Wf, float sx,
                                                    float sy, int Hb, int Wb, int maxpix, int nty,
                                                    uint2 *__restrict__ boxes) {
    const int ntx = (Wb + TW - 1) / TW, nt = ntx * nty;  // nty >= ceil(Hb / TH) box-tile rows (extra rows: empty)
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int b = blockIdx.y;
    if (t >= (int64_t)nt * V) return;
    const int tile = (int)(t / V), v = (int)(t - (int64_t)tile * V);
    const int tyb = tile / ntx, txb = tile - tyb * ntx;
    const int ia = tyb * TH, ib = min(ia + TH - 1, Hb - 1);
    const int ja = txb * TW, jb = min(ja + TW - 1, Wb - 1);
    bool ok = true;
    Box cb{0x7fffffff, 0x7fffffff, -1, -1};
    if (ia < Hb) {
        float hv[9];
        load_h(Hmat, b * V + v, hv);
        cb = corner_box(hv, xs[ja], xs[jb], ys[ia], ys[ib], sx, sy, Wf, Hf, ok);
    }
    if (ok && cb.x1 >= 0 && (cb.x1 - cb.x0 + 1) * (cb.y1 - cb.y0 + 1) > maxpix) ok = false;
    const bool emp = cb.x1 < 0;
    boxes[((int64_t)b * nt + tile) * V + v] =
        make_uint2((emp ? 0u : (unsigned)cb.x0 | ((unsigned)cb.y0 << 16)) | (ok ? 0u : 0x80000000u),
                   emp ? 0u : (unsigned)(cb.x1 + 1) | ((unsigned)(cb.y1 + 1) << 16));
}

// -------------------------------------------------------------------------
// fused warp + reduce, wave-independent (k_warp_fuse_w): no workgroup barrier
// -------------------------------------------------------------------------
// The workgroup's four waves share nothing but the launch: wave w owns the 4 x 16 cells of rows 4w .. 4w + 3 of
// the 16 x 16 tile (the same cells, lanes, taps, sampling order and stores as k_warp_fuse_v2<.., 16, 1>, hence
// bit-identical results), and stages, for each view, the footprint of ITS cells into its own slice of LDS (pool
// `wpool` bytes + a zero pixel).  Its own LDS-DMA completes under its own vmcnt, so the per-view workgroup barrier
// of v2 is gone: the waves drift apart and hide each other's DMA / tap / sampling latency.  Footprints are
// per-wave corner boxes (k_warp_boxes over 4 x 16 tiles; in-lane if no workspace); the ring anchors consecutive
// images at opposite ends of the pool; a footprint larger than what is free is staged synchronously, in
// overlapping blocks when larger than the pool; tiles where the corner bound does not apply reduce their exact
// per-cell box by shuffles.  Staging volume ~2x v2's (smaller tiles overlap more), LDS-read and VALU work equal.
template <int MODE, int OCC>
__global__ __launch_bounds__(FT_NT, OCC) void k_warp_fuse_w(const float *__restrict__ feats, int64_t sN, int64_t sH,
                                                         int64_t sW, const float *__restrict__ Hmat,
                                                         const float *__restrict__ xs, const float *__restrict__ ys,
                                                         int B, int V, int C, int Hf, int Wf, float sx, float sy,
                                                         int Hb, int Wb, float *__restrict__ out, int wpool,
                                                         const uint2 *__restrict__ boxes) {
    constexpr int TH = 16, TW = 16, SL = 17, PS = SL * 16;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int ib = wave * (wpool + 256);  // this wave's pool (byte offset in smem), zero pixel after it
    const int zp = ib + wpool;
    const int maxpix = wpool / PS - 4;
    const int ntx = (Wb + TW - 1) / TW, nty = (Hb + TH - 1) / TH, nt = ntx * nty;
    int tile = blockIdx.x;
    {
        const int q = nt / 8, r = nt % 8, x = tile % 8;
        tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + tile / 8;
    }
    const int tyb = tile / ntx, txb = tile - tyb * ntx;
    const int wtile = (tyb * 4 + wave) * ntx + txb;  // this wave's 4 x 16 box tile
    STAMP(0);
    int tr, tc;
    tile_cell<TH>(lane, wave, tr, tc);
    const bool bufdma = WARP_DMABUF && sH * 4 < (1 << 24) && sW * 4 < (1 << 24) &&
                        ((int64_t)Hf * sH + (int64_t)Wf * sW) * 4 < (1ll << 31);
    auto dma = [&](const float *fp, int x0, int y0, int w, int n, int o) {
        if (bufdma) dma_block_buf<SL>(fp, (int)sH * 4, (int)sW * 4, x0, y0, w, n, smem, o, 0, lane, 1);
        else dma_block<SL>(fp, (int)sH, (int)sW, x0, y0, w, n, smem, o, 0, lane, 1);
    };
    const int i = tyb * TH + tr;
    const int j = txb * TW + tc;
    const int b = blockIdx.y;
    const bool inside = (i < Hb) && (j < Wb);
    const float cx = xs[inside ? j : 0], cy = ys[inside ? i : 0];
    const size_t plane = (size_t)Hb * Wb;
    const Grid grid = make_grid(Hf, Wf);
    const double rV = recip_uniform(V);
    if (lane < 16) *(float4 *)(smem + zp + lane * 16) = make_float4(0.f, 0.f, 0.f, 0.f);  // read after, same wave

    // per-wave corner boxes, lane v <-> view v (v2's packing)
    unsigned lba = 0, lbb = 0;
    if (boxes != nullptr) {
        const uint2 bx = lane < V ? boxes[((int64_t)b * (nt * 4) + wtile) * V + lane] : make_uint2(0u, 0u);
        lba = bx.x;
        lbb = bx.y;
    } else if (lane < V) {
        const int ia = tyb * TH + 4 * wave, ibr = min(ia + 3, Hb - 1);
        const int ja = txb * TW, jb = min(ja + TW - 1, Wb - 1);
        Box cb{0x7fffffff, 0x7fffffff, -1, -1};
        bool ok = true;
        if (ia < Hb) {
            float hv[9];
            load_h(Hmat, b * V + lane, hv);
            cb = corner_box(hv, xs[ja], xs[jb], ys[ia], ys[ibr], sx, sy, Wf, Hf, ok);
            if (ok && cb.x1 >= 0 && (cb.x1 - cb.x0 + 1) * (cb.y1 - cb.y0 + 1) > maxpix) ok = false;
        }
        const bool emp = cb.x1 < 0;
        lba = (emp ? 0u : (unsigned)cb.x0 | ((unsigned)cb.y0 << 16)) | (ok ? 0u : 0x80000000u);
        lbb = emp ? 0u : (unsigned)(cb.x1 + 1) | ((unsigned)(cb.y1 + 1) << 16);
    }
    STAMP(1);
    auto box_of = [&](int v) {
        const unsigned a = (unsigned)__builtin_amdgcn_readlane((int)lba, v);
        const unsigned c = (unsigned)__builtin_amdgcn_readlane((int)lbb, v);
        return Box{(int)(a & 0xffffu), (int)((a >> 16) & 0x7fffu), (int)(c & 0xffffu) - 1, (int)(c >> 16) - 1};
    };
    auto ok_of = [&](int v) { return ((unsigned)__builtin_amdgcn_readlane((int)lba, v) >> 31) == 0u; };
    const int hbase = b * V;
    float ccx = cx, ccy = cy;
    auto taps_of = [&](int v) {
        float h[9];
#pragma unroll
        for (int q = 0; q < 9; ++q) h[q] = Hmat[__builtin_amdgcn_readfirstlane((hbase + v) * 9) + q];
        float ix, iy;
        cell_ixy(h, ccx, ccy, grid, sx, sy, ix, iy);
        Taps t = taps_from_ixy(ix, iy, grid);
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

    for (int c0 = 0; c0 < C; c0 += 64) {
        ccx = cx;
        ccy = cy;
        asm volatile("" : "+v"(ccx), "+v"(ccy));  // taps per chunk (no hoisting + spills)
        float acc[64];
#pragma unroll
        for (int q = 0; q < 64; ++q) acc[q] = (MODE == BEV_FUSE_MAX) ? -__builtin_inff() : 0.0f;
        const float *fb = feats + (int64_t)(b * V) * sN + c0;
        auto live = [&](int u) { return !ok_of(u) || box_of(u).x1 >= 0; };
        auto next_live = [&](int u) {
            ++u;
            while (u < V && !live(u)) {
                zero_view<MODE>(acc, u);
                ++u;
            }
            return u;
        };
        const int v_first = next_live(-1);
        Box bn = box_of(v_first < V ? v_first : 0);
        int offn = -1;
        if (v_first < V) {
            const int npix = (bn.x1 - bn.x0 + 1) * (bn.y1 - bn.y0 + 1);
            if (ok_of(v_first) && bn.x1 >= 0 && npix <= maxpix) {
                offn = ib;
                dma(fb + (int64_t)v_first * sN, bn.x0, bn.y0, bn.x1 - bn.x0 + 1, npix, ib);
            }
        }
        Taps tf;
        bool have_f = false;
        if (v_first < V && ok_of(v_first)) {
            tf = taps_of(v_first);
            have_f = true;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's own DMA: visible to its own reads
        STAMP(2);

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
            if (!ok_of(v)) {  // exact per-cell box of this wave's cells (shuffle reduction, no exchange)
                t = taps_of(v);
                have_t = true;
                bx = wave_box(t);
            }
            const bool empty = bx.x1 < 0;
            const int bw = bx.x1 - bx.x0 + 1, bh = bx.y1 - bx.y0 + 1;
            bool done = empty;
            if (!done && off < 0) {
                // synchronous staging (overlapping blocks if larger than the pool); the pool's previous
                // images have been read: every earlier ds_read's result was consumed by its FMAs
                int wb = bw, hb = bh, nbx = 1, nby = 1;
                if (bw * bh > maxpix) {
                    wb = (2 * bw <= maxpix) ? bw : maxpix / 2;
                    hb = min(bh, maxpix / wb);
                    nbx = (wb >= bw) ? 1 : (bw - 2) / (wb - 1) + 1;
                    nby = (hb >= bh) ? 1 : (bh - 2) / (hb - 1) + 1;
                }
                const bool single = (nbx == 1) && (nby == 1);
                if (single) dma(f, bx.x0, bx.y0, bw, bw * bh, ib);
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
                            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // previous block's reads returned
                            dma(f, sx0, sy0, sbw, sbw * sbh, ib);
                        }
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        const bool mine = single ? true : (t.valid != 0 && mkx == kx && mky == ky);
                        const bool go = single ? wave_any : (__ballot(mine) != 0ull);
                        if (go) sample_view<MODE, 1, 64>(acc, t, mine, v, smem, ib, sx0, sy0, sbw, zp);
                        else if (single) zero_view<MODE>(acc, v);
                    }
                done = true;
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the pool is free for the next DMA
            }
            // look ahead: DMA of the next live view beside the live image of view v
            if (vn < V) {
                bn = box_of(vn);
                offn = -1;
                const int npix = (bn.x1 - bn.x0 + 1) * (bn.y1 - bn.y0 + 1);
                if (ok_of(vn) && bn.x1 >= 0 && npix <= maxpix) {
                    const int need = ((npix * SL + 63) >> 6) * 1024;
                    if (done || off < 0) offn = ib;
                    else if (off == ib) {
                        if (((bw * bh * SL + 63) >> 6) * 1024 + need <= wpool) offn = ib + wpool - need;
                    } else if (need <= off - ib) offn = ib;
                    if (offn >= 0) dma(fb + (int64_t)vn * sN, bn.x0, bn.y0, bn.x1 - bn.x0 + 1, npix, offn);
                }
            }
            if (!done) {
                if (!have_t) t = taps_of(v);
                if (WARP_ABLATE & 4) acc[0] += t.w[0] * t.w[3] + (float)(t.x0 + t.y0 + (int)t.valid);
                else if (__ballot(t.valid != 0) != 0ull)
                    sample_view_pipe<MODE, 64>(acc, t, smem, off, bx.x0, bx.y0, bw, zp, zp);
                else zero_view<MODE>(acc, v);
            } else if (empty) {
                zero_view<MODE>(acc, v);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // view v + 1's image landed
        }
        STAMP(3);
        if (inside) store_chunk(out + ((size_t)b * C + c0) * plane, plane, i * Wb + j, acc, MODE, rV);
        STAMP(4);
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
int g_warp_kernel = 0;   // BEV_TUNE_WARP_KERNEL: 0 LDS-DMA kernel (k_warp_fuse_v2, default), 1 register-staged
int g_warp_bwd_pool = 0; // BEV_TUNE_WARP_BWD_POOL: backward LDS image in floats, 0 = WARP_BWD_POOL_MAX

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
#ifndef WARP_PAIR
#define WARP_PAIR 0  // frames per workgroup with the LDS tap records: 0 off (default), 1 on (A/B builds; r03d:
                     // 176 vs 131 us for the batch-2 bench launch -- half the workgroups, a tail and a smaller pool)
#endif
#ifndef WARP_OCC
#define WARP_OCC 3   // workgroups per CU the default (mean / sum) kernel is compiled and sized for
#endif
constexpr int V2_FIXED = 256 + 4 * (FT_NT / 64) * (int)sizeof(int) + V2_MAXV * 9 * (int)sizeof(float) +
                         (2 * V2_MAXV + 4) * (int)sizeof(unsigned);  // zero pixel, red, htab, btab + flag
constexpr int V2_TC_MAXV = 8;  // tap records only for rigs of up to 8 cameras (12 B per cell and view)

template <int OCC, int FPW>
int launch_fuse_v2_occ(const float *feats, int64_t sN, int64_t sH, int64_t sW, const float *Hmat, const float *xs,
                       const float *ys, int B, int V, int C, int Hf, int Wf, float sx, float sy, int Hb, int Wb,
                       int mode, float *out, hipStream_t st, int pool, int tc_bytes, uint2 *boxes) {
    constexpr int TH = WARP_TILE_H, TW = FT_NT / TH;
    const int ntiles = ((Wb + TW - 1) / TW) * ((Hb + TH - 1) / TH);
    dim3 grid(ntiles, (B + FPW - 1) / FPW), block(FT_NT);
    const int tcache = tc_bytes > 0 ? pool + V2_FIXED : -1;
    const size_t lds = (size_t)pool + V2_FIXED + (tc_bytes > 0 ? tc_bytes : 0);
    if (FPW != 1 || !WARP_HSCALAR) boxes = nullptr;  // the in-kernel prologue (frame pairs / LDS homographies)
    if (boxes) {
        const int maxpix = pool / (17 * 16) - 4;  // the kernel's own pool test
        hipLaunchKernelGGL((k_warp_boxes<TH>), dim3((unsigned)(((int64_t)ntiles * V + 255) / 256), B), dim3(256), 0,
                           st, Hmat, xs, ys, V, Hf, Wf, sx, sy, Hb, Wb, maxpix, (Hb + TH - 1) / TH, boxes);
    }
    if (mode == BEV_FUSE_SUM)
        hipLaunchKernelGGL((k_warp_fuse_v2<BEV_FUSE_SUM, OCC, TH, FPW>), grid, block, lds, st, feats, sN, sH, sW, Hmat,
                           xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, out, pool, tcache, boxes);
    else if (mode == BEV_FUSE_MEAN)
        hipLaunchKernelGGL((k_warp_fuse_v2<BEV_FUSE_MEAN, OCC, TH, FPW>), grid, block, lds, st, feats, sN, sH, sW, Hmat,
                           xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, out, pool, tcache, boxes);
    else
        hipLaunchKernelGGL((k_warp_fuse_v2<BEV_FUSE_MAX, OCC, TH, FPW>), grid, block, lds, st, feats, sN, sH, sW, Hmat,
                           xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, out, pool, tcache, boxes);
    return last();
}

template <int OCC>
int launch_fuse_p(const float *feats, int64_t sN, int64_t sH, int64_t sW, const float *Hmat, const float *xs,
                  const float *ys, int B, int V, int Hf, int Wf, float sx, float sy, int Hb, int Wb, int mode,
                  float *out, hipStream_t st, int pool, uint2 *boxes) {
    constexpr int TH = WARP_TILE_H, TW = FT_NT / TH;
    const int nty = (Hb + TH - 1) / TH, ntiles = ((Wb + TW - 1) / TW) * nty;
    const int maxpix = pool / (17 * 16) - 4;
    hipLaunchKernelGGL((k_warp_boxes<TH>), dim3((unsigned)(((int64_t)ntiles * V + 255) / 256), B), dim3(256), 0, st,
                       Hmat, xs, ys, V, Hf, Wf, sx, sy, Hb, Wb, maxpix, nty, boxes);
    const int64_t nitems = (int64_t)ntiles * B;
    const unsigned g = (unsigned)(nitems < (int64_t)OCC * cu_count() ? nitems : (int64_t)OCC * cu_count());
    const size_t lds = (size_t)pool + V2_FIXED;
    if (mode == BEV_FUSE_SUM)
        hipLaunchKernelGGL((k_warp_fuse_p<BEV_FUSE_SUM, OCC, TH>), dim3(g), dim3(FT_NT), lds, st, feats, sN, sH, sW,
                           Hmat, xs, ys, B, V, Hf, Wf, sx, sy, Hb, Wb, out, pool, boxes);
    else if (mode == BEV_FUSE_MEAN)
        hipLaunchKernelGGL((k_warp_fuse_p<BEV_FUSE_MEAN, OCC, TH>), dim3(g), dim3(FT_NT), lds, st, feats, sN, sH, sW,
                           Hmat, xs, ys, B, V, Hf, Wf, sx, sy, Hb, Wb, out, pool, boxes);
    else if constexpr (OCC == 2)  // MAX's extra live state spills at 3 workgroups per CU
        hipLaunchKernelGGL((k_warp_fuse_p<BEV_FUSE_MAX, OCC, TH>), dim3(g), dim3(FT_NT), lds, st, feats, sN, sH, sW,
                           Hmat, xs, ys, B, V, Hf, Wf, sx, sy, Hb, Wb, out, pool, boxes);
    else
        return BEV_ERR_ARGS;
    return last();
}

// wave-independent kernel: 4 x (pool + zero pixel) per workgroup, OCC workgroups per CU
template <int OCC>
int launch_fuse_w_occ(const float *feats, int64_t sN, int64_t sH, int64_t sW, const float *Hmat, const float *xs,
                      const float *ys, int B, int V, int C, int Hf, int Wf, float sx, float sy, int Hb, int Wb, int mode,
                      float *out, hipStream_t st, uint2 *boxes) {
    const int ntx = (Wb + 15) / 16, nty = (Hb + 15) / 16;
    const int wpool = g_warp_pool_kb ? g_warp_pool_kb * 1024 / 4 : ((163840 / OCC - 64) / 4 - 256) & ~1023;
    if (wpool < 4096) return BEV_ERR_ARGS;
    if (boxes) {
        const int maxpix = wpool / (17 * 16) - 4;
        hipLaunchKernelGGL((k_warp_boxes<4, 16>), dim3((unsigned)(((int64_t)ntx * nty * 4 * V + 255) / 256), B),
                           dim3(256), 0, st, Hmat, xs, ys, V, Hf, Wf, sx, sy, Hb, Wb, maxpix, nty * 4, boxes);
    }
    dim3 grid(ntx * nty, B), block(FT_NT);
    const size_t lds = (size_t)4 * (wpool + 256);
    if (mode == BEV_FUSE_SUM)
        hipLaunchKernelGGL((k_warp_fuse_w<BEV_FUSE_SUM, OCC>), grid, block, lds, st, feats, sN, sH, sW, Hmat, xs, ys, B,
                           V, C, Hf, Wf, sx, sy, Hb, Wb, out, wpool, boxes);
    else if (mode == BEV_FUSE_MEAN)
        hipLaunchKernelGGL((k_warp_fuse_w<BEV_FUSE_MEAN, OCC>), grid, block, lds, st, feats, sN, sH, sW, Hmat, xs, ys,
                           B, V, C, Hf, Wf, sx, sy, Hb, Wb, out, wpool, boxes);
    else if constexpr (OCC == 2)  // MAX's extra live state spills at 3 workgroups per CU
        hipLaunchKernelGGL((k_warp_fuse_w<BEV_FUSE_MAX, OCC>), grid, block, lds, st, feats, sN, sH, sW, Hmat, xs, ys, B,
                           V, C, Hf, Wf, sx, sy, Hb, Wb, out, wpool, boxes);
    else
        return BEV_ERR_ARGS;
    return last();
}

inline int launch_fuse_v2(const float *feats, int64_t sN, int64_t sH, int64_t sW, const float *Hmat,
                          const float *xs, const float *ys, int B, int V, int C, int Hf, int Wf, float sx, float sy,
                          int Hb, int Wb, int mode, float *out, hipStream_t st, uint2 *boxes) {
    if (mode == BEV_FUSE_MAX)  // MAX's extra live state spills at 3 workgroups per CU
        return launch_fuse_v2_occ<2, 1>(feats, sN, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out,
                                        st, g_warp_pool_kb ? g_warp_pool_kb * 1024 : 72 * 1024, 0, boxes);
    // tap records: worth it when a workgroup runs two frames or several 64-channel chunks
    const int tc_bytes = V * FT_NT * 12;
    const bool pair = WARP_PAIR && V <= V2_TC_MAXV && (B > 1 || C > 64);
    // 3 workgroups per CU: pool + fixed + records <= 160 KiB / 3 (the pool shrinks by the records)
    const int budget = 163840 / 3 - V2_FIXED - 64;
    const int pool = g_warp_pool_kb ? g_warp_pool_kb * 1024 : ((pair ? budget - tc_bytes : 49 * 1024) & ~1023);
    if (pair && pool >= 16 * 1024 && pool + V2_FIXED + tc_bytes <= 160 * 1024)
        return launch_fuse_v2_occ<3, 2>(feats, sN, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, st,
                                        pool, tc_bytes, boxes);
    return launch_fuse_v2_occ<WARP_OCC, 1>(feats, sN, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out,
                                           st, g_warp_pool_kb ? g_warp_pool_kb * 1024 :
                                           ((163840 / WARP_OCC - V2_FIXED - 64) & ~1023) < 49 * 1024 ?
                                           ((163840 / WARP_OCC - V2_FIXED - 64) & ~1023) : 49 * 1024, 0, boxes);
}

}  // namespace

namespace bev {
int warp_bwd_pool_floats() { return g_warp_bwd_pool > 0 ? g_warp_bwd_pool : WARP_BWD_POOL_MAX; }

int warp_tune(int knob, int value) {
    int *slot = nullptr;
    bool ok = false;
    switch (knob) {
        case BEV_TUNE_WARP_POOL_KB:
            slot = &g_warp_pool_kb;
            ok = value == 0 || (value >= 8 && value <= 150);
            break;
        case BEV_TUNE_WARP_KERNEL:
            slot = &g_warp_kernel;
            ok = value >= 0 && value <= 3;
            break;
        case BEV_TUNE_WARP_BWD_POOL:
            slot = &g_warp_bwd_pool;
            ok = value >= 0 && value <= WARP_BWD_POOL_MAX;
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

int bev_abi_version(void) { return 6; }

#if WARP_STAMP
int bev_warp_stamp_read(unsigned long long *host, int n) {  // timing builds only
    if (n > 16384 * 6) n = 16384 * 6;
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
    // the larger of the two box tables: v2's (TH x TW tiles) and the wave-independent kernel's (4 x 16)
    constexpr int TH = WARP_TILE_H, TW = FT_NT / TH;
    const int64_t v2 = (((int64_t)Wb + TW - 1) / TW) * (((int64_t)Hb + TH - 1) / TH);
    const int64_t wv = (((int64_t)Wb + 15) / 16) * (((int64_t)Hb + 15) / 16) * 4;
    return (int64_t)B * (v2 > wv ? v2 : wv) * V * (int64_t)sizeof(uint2);
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
    if (dma_ok && g_warp_kernel != 1)
    {
        const int64_t need = bev_ipm_warp_fuse_workspace_bytes(B, V, Hb, Wb);
        uint2 *boxes = (workspace && workspace_bytes >= need && ((uintptr_t)workspace & 7) == 0)
                           ? reinterpret_cast<uint2 *>(workspace) : nullptr;
        if (g_warp_kernel == 3 && boxes && C == 64 && (int64_t)B * ((Hb + 15) / 16) * ((Wb + 15) / 16) < (1ll << 31)) {
            const int occ_pool = g_warp_pool_kb ? g_warp_pool_kb * 1024 : 49 * 1024;
            return mode == BEV_FUSE_MAX
                       ? launch_fuse_p<2>(feats, sN, sH, sW, Hmat, xs, ys, B, V, Hf, Wf, sx, sy, Hb, Wb, mode, out, st,
                                          g_warp_pool_kb ? occ_pool : 72 * 1024, boxes)
                       : launch_fuse_p<3>(feats, sN, sH, sW, Hmat, xs, ys, B, V, Hf, Wf, sx, sy, Hb, Wb, mode, out, st,
                                          occ_pool, boxes);
        }
        if (g_warp_kernel == 2)
            return mode == BEV_FUSE_MAX
                       ? launch_fuse_w_occ<2>(feats, sN, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out,
                                              st, boxes)
                       : launch_fuse_w_occ<3>(feats, sN, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out,
                                              st, boxes);
        return launch_fuse_v2(feats, sN, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, st, boxes);
    }
    if (C <= 4)
        return launch_fuse_ck<4>(feats, sN, sC, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, st);
    if (C <= 16)
        return launch_fuse_ck<16>(feats, sN, sC, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, st);
    if (C <= 32)
        return launch_fuse_ck<32>(feats, sN, sC, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, st);
    return launch_fuse_ck<64>(feats, sN, sC, sH, sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, st);
}

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
