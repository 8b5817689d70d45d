// bev_warp_bwd.hip -- backward of the IPM warp (+ view sum / mean) w.r.t. the features, for gfx950 (MI355X).
//
// Replaces autograd through geometry.py:161 (grid_sampler_2d_backward, input gradient only: the grid comes from
// the calibration, which carries no gradient) and, for the fused path, fusion.py:19-21 (sum / mean over views:
// d mean / d x_v = gout / V).  For every source pixel p of view v and channel c:
//     gfeats[v][c][p] = sum over BEV cells q and taps t of q with tap(q, t) == p, valid:  w_t(q) * g_v[c][q]
// with g_v = gout (sum) or gout / V (mean), or the view's own gout (per-view warp).  The taps and weights are
// the forward's bit-exact recipe (bev_geometry.h).  Float addition order differs from torch's scatter (float
// atomics across tiles): equal to the reference's backward within fp32 tolerance, not bit for bit.
//
// k_warp_bwd_runs -- one workgroup per (frame, 16 x 16 BEV tile), ALL views of the frame in one workgroup, so the
// fused gradient gout is read from HBM once (not once per view).  Lane mapping ("runs"): a 16-lane DPP row owns
// one tile row = a run of 16 consecutive cells along the BEV x axis; lane l holds channels 4l .. 4l + 3 of a
// 64-channel chunk for all 16 cells of the run (64 VGPRs), and computes the taps of cell l.  The row walks its 16
// cells in order; cell k's tap key, weights and image addresses come from lane k by DPP row broadcast
// (row_newbcast), and the four tap gradients w_t * g are accumulated in registers while consecutive cells share
// the same 2x2 source quad -- on the Appendix-B rig 80 % of the cells have their left neighbour's quad (DESIGN.md
// §4) -- and are added to the LDS image of the tile's footprint only when the quad changes.
// No LDS float atomics: on gfx950 a ds_add_f32 wave instruction costs ~40x a ds_add_u32 / ~160x a ds_write_b32
// (tools/lds_atomic_micro.hip, profiles/r04c_lds_atomic_micro.txt).  Instead every wave owns a copy of the image and
// its four rows add their run sums by plain read-modify-write (ds_read_b128 + add + ds_write_b128), one row at a
// time (the rows of a wave may hit the same pixel; a wave's LDS operations complete in order).  The four copies are
// summed per (pixel, channel) and go to the gradient with one global float atomic per touched (pixel, channel),
// coalesced along channels for NHWC gradients (one 256-B wave instruction per pixel) or along x for NCHW.
// A footprint whose four copies do not fit the LDS pool is done in two halves of the tile (two waves each, two copies
// of the half's own box); only a half whose box still does not fit adds its run sums straight to global memory.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bev_geometry.h"
#include "bev_tune.h"
#include "../../include/bev_mi355x.h"

using namespace bev;

namespace {

constexpr int RB_NT = 256;   // 4 waves = 16 DPP rows = 16 runs
constexpr int RB_T = 16;     // tile = 16 rows x 16 cells
constexpr int RB_PIX = 256;  // image bytes per pixel (64 channels, unpadded: a row's b128 access is one pixel)

static inline int rb_err(hipError_t e) { return e == hipSuccess ? 0 : (int)e; }

// lane k of this lane's 16-lane DPP row, to every lane of the row
template <int K>
__device__ __forceinline__ int row_bcast(int v) {
    return __builtin_amdgcn_update_dpp(0, v, 0x150 + K, 0xf, 0xf, true);  // bound_ctrl: no "old" operand to set up
}
template <int K>
__device__ __forceinline__ float row_bcast_f(float v) {
    return __builtin_bit_cast(float, row_bcast<K>(__builtin_bit_cast(int, v)));
}

// Quad key of a cell: (x0 + 1) | (y0 + 1) << 14 | valid << 28; 0 = no valid tap (never equal to a real key).
__device__ __forceinline__ int quad_key(const Taps &t) {
    if (!t.valid) return 0;
    return (t.x0 + 1) | ((t.y0 + 1) << 14) | ((int)t.valid << 28);
}
__device__ __forceinline__ int key_x0(int k) { return (k & 0x3fff) - 1; }
__device__ __forceinline__ int key_y0(int k) { return ((k >> 14) & 0x3fff) - 1; }
__device__ __forceinline__ unsigned key_valid(int k) { return ((unsigned)k >> 28) & 15u; }

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

struct Box4 {
    int x0, y0, x1, y1;
};

// Where a run's four tap sums go: the wave's copy of the LDS image (byte addresses of the four taps from the run's
// last cell, lane offset included; an invalid tap points at the copy's trash pixel, never flushed), or without an
// image (footprint too large) the global gradient, by float atomics on the valid taps.
struct GSink {
    float *gf;           // global gradient of this view at the chunk's first channel
    int64_t sC, sH, sW;  // its element strides
    int lane16, cmax;
};

__device__ __forceinline__ void run_flush(bool img, int key, const int (&a)[4], const f32x4 (&q)[4],
                                          unsigned char *smem, const GSink &gs) {
    if (img) {  // uniform in the row
        // the four taps are distinct pixels (or the trash pixel, never read back): all reads, ONE wait, all writes
        // (a read-wait-write per tap costs four LDS round trips)
        f32x4 *p[4];
        f32x4 o[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            p[t] = reinterpret_cast<f32x4 *>(smem + a[t] + 16 * gs.lane16);
            o[t] = *p[t];
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const f32x2 lo = o[t].xy + q[t].xy, hi = o[t].zw + q[t].zw;  // v_pk_add_f32
            *p[t] = (f32x4){lo.x, lo.y, hi.x, hi.y};
        }
    } else {
        const unsigned vb = key_valid(key);
        const int x0 = key_x0(key), y0 = key_y0(key);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            if (!(vb & (1u << t))) continue;
            float *p = gs.gf + (int64_t)(y0 + (t >> 1)) * gs.sH + (int64_t)(x0 + (t & 1)) * gs.sW;
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (4 * gs.lane16 + u < gs.cmax) unsafeAtomicAdd(p + (int64_t)(4 * gs.lane16 + u) * gs.sC, q[t][u]);
        }
    }
}

// Step K of a row's walk: accumulate cell K's four tap gradients (key / weights from lane K by DPP row broadcast);
// when cell K ends its run (cell K + 1 has another quad, or K is the last cell), add the run's sums at cell K's tap
// addresses -- the rows of the wave one after the other -- and restart them.  The restart is a select, so the
// accumulators carry no control-flow merges.
template <int K>
__device__ __forceinline__ void walk_step(const float (&g)[16][4], f32x4 (&q)[4], int &key, int (&a)[4],
                                          float (&w)[4], bool img, int rw, unsigned char *smem, const GSink &gs) {
    // the broadcast sources are "redefined" at every step, so the compiler cannot hoist all 16 steps' broadcasts
    // to the top of the walk (9 x 16 extra live VGPRs)
    asm volatile("" : "+v"(key), "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(a[0]), "+v"(a[1]), "+v"(a[2]),
                 "+v"(a[3]));
    const int kk = row_bcast<K>(key);
    int kn = 0;
    if constexpr (K + 1 < 16) kn = row_bcast<K + 1>(key);
    const f32x2 g01 = (f32x2){g[K][0], g[K][1]}, g23 = (f32x2){g[K][2], g[K][3]};
#pragma unroll
    for (int t = 0; t < 4; ++t) {  // packed fp32: two channels per v_pk_fma_f32 (each half fmaf exactly)
        const float wt = row_bcast_f<K>(w[t]);
        const f32x2 W = (f32x2){wt, wt};
        const f32x2 lo = __builtin_elementwise_fma(W, g01, q[t].xy), hi = __builtin_elementwise_fma(W, g23, q[t].zw);
        q[t] = (f32x4){lo.x, lo.y, hi.x, hi.y};
    }
    const bool end = kn != kk;
    const bool fl = end && kk != 0;
    if (__ballot(fl) != 0ull) {  // wave-uniform
        int at[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) at[t] = row_bcast<K>(a[t]);
#pragma unroll 1
        for (int r = 0; r < 4; ++r) {  // one row at a time: plain read-modify-write of the wave's image copy
            // compiler barrier: per thread the rows' accesses look independent, but row r + 1 must read what row r
            // wrote (the hardware keeps a wave's LDS operations in order)
            asm volatile("" ::: "memory");
            if (rw == r && fl) run_flush(img, kk, at, q, smem, gs);
        }
        asm volatile("" ::: "memory");
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) q[t] = end ? (f32x4){0.0f, 0.0f, 0.0f, 0.0f} : q[t];
    // the step's sums exist here (no deferral of many steps' FMAs: register pressure)
    asm volatile("" : "+v"(q[0]), "+v"(q[1]), "+v"(q[2]), "+v"(q[3]));
}

template <int K>
__device__ __forceinline__ void walk_from(const float (&g)[16][4], f32x4 (&q)[4], int &key, int (&a)[4],
                                          float (&w)[4], bool img, int rw, unsigned char *smem, const GSink &gs) {
    walk_step<K>(g, q, key, a, w, img, rw, smem, gs);
    if constexpr (K + 1 < 16) walk_from<K + 1>(g, q, key, a, w, img, rw, smem, gs);
}

// One row's walk over its 16 cells for one view.
__device__ __forceinline__ void walk_row(const float (&g)[16][4], int key, const int (&a0)[4], const float (&w0)[4],
                                         bool img, int rw, unsigned char *smem, const GSink &gs) {
    int a[4] = {a0[0], a0[1], a0[2], a0[3]};
    float w[4] = {w0[0], w0[1], w0[2], w0[3]};
    f32x4 q[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) q[t] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
    walk_from<0>(g, q, key, a, w, img, rw, smem, gs);
}

// Exact bbox of the valid taps of the workgroup's cells (wave shuffles + LDS exchange).
__device__ __forceinline__ Box4 block_box(const Taps &t, int *red, int wave, int lane) {
    int x0 = 0x7fffffff, y0 = 0x7fffffff, x1 = -1, y1 = -1;
    if (t.valid) {
        x0 = (t.valid & 5) ? t.x0 : t.x0 + 1;
        x1 = (t.valid & 10) ? t.x0 + 1 : t.x0;
        y0 = (t.valid & 3) ? t.y0 : t.y0 + 1;
        y1 = (t.valid & 12) ? t.y0 + 1 : t.y0;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        x0 = min(x0, __shfl_xor(x0, o));
        y0 = min(y0, __shfl_xor(y0, o));
        x1 = max(x1, __shfl_xor(x1, o));
        y1 = max(y1, __shfl_xor(y1, o));
    }
    if (lane == 0) {
        red[wave] = x0;
        red[4 + wave] = y0;
        red[8 + wave] = x1;
        red[12 + wave] = y1;
    }
    __syncthreads();
    Box4 b{red[0], red[4], red[8], red[12]};
#pragma unroll
    for (int w = 1; w < 4; ++w) {
        b.x0 = min(b.x0, red[w]);
        b.y0 = min(b.y0, red[4 + w]);
        b.x1 = max(b.x1, red[8 + w]);
        b.y1 = max(b.y1, red[12 + w]);
    }
    return b;
}

// grid (tiles, B); gout [B][Cg][Hb][Wb] (per_view: [B*V][C][Hb][Wb]), gfeats element strides (sN, sC, sH, sW)
__global__ __launch_bounds__(RB_NT, 2) void k_warp_bwd_runs(const float *__restrict__ gout, const float *__restrict__ Hmat,
                                                         const float *__restrict__ xs, const float *__restrict__ ys,
                                                         int V, int C, int Hf, int Wf, float sx, float sy, int Hb,
                                                         int Wb, int mean, int per_view, float *__restrict__ gfeats,
                                                         int64_t sN, int64_t sC, int64_t sH, int64_t sW, int pool) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float *img = reinterpret_cast<float *>(smem);
    int *red = reinterpret_cast<int *>(smem + pool);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l16 = lane & 15;
    const int ntx = (Wb + RB_T - 1) / RB_T;
    const int ty = blockIdx.x / ntx, tx = blockIdx.x - ty * ntx;
    const int b = blockIdx.y;
    const int row = wave * 4 + (lane >> 4);  // the run (tile row) of this lane's DPP row
    const int i = ty * RB_T + row, j0 = tx * RB_T, j = j0 + l16;
    const bool inside = i < Hb && j < Wb, row_in = i < Hb;
    const float cx = xs[inside ? j : 0], cy = ys[inside ? i : 0];
    const Grid grid = make_grid(Hf, Wf);
    const int64_t plane = (int64_t)Hb * Wb;
    const bool vec = row_in && (Wb % 4 == 0) && j0 + RB_T <= Wb;
    const double rV = recip_uniform(V);
    const int maxpix = pool / (4 * RB_PIX) - 1;  // four copies, each + its trash pixel (whole-tile footprints)
    const int rw = lane >> 4;                     // the lane's row within its wave

    for (int c0 = 0; c0 < C; c0 += 64) {
        const int cmax = min(64, C - c0);
        float g[16][4];
        auto load_g = [&](const float *src) {  // src = gradient map of this frame (or view) [C][Hb][Wb]
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int c = c0 + 4 * l16 + m;
                const float *p = src + (int64_t)(c < C ? c : 0) * plane + (int64_t)(row_in ? i : 0) * Wb + j0;
                if (vec && c < C) {
#pragma unroll
                    for (int k4 = 0; k4 < 4; ++k4) {
                        const float4 v = *reinterpret_cast<const float4 *>(p + 4 * k4);
                        g[4 * k4][m] = v.x;
                        g[4 * k4 + 1][m] = v.y;
                        g[4 * k4 + 2][m] = v.z;
                        g[4 * k4 + 3][m] = v.w;
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < 16; ++k) g[k][m] = (row_in && c < C && j0 + k < Wb) ? p[k] : 0.0f;
                }
                if (mean) {
#pragma unroll
                    for (int k = 0; k < 16; ++k) g[k][m] = div_rcp(g[k][m], rV);  // gout / V, IEEE-exact
                }
            }
        };
        if (!per_view) load_g(gout + (int64_t)b * C * plane);

        for (int v = 0; v < V; ++v) {
            const int n = b * V + v;
            float h[9];
#pragma unroll
            for (int q = 0; q < 9; ++q) h[q] = Hmat[__builtin_amdgcn_readfirstlane(n * 9) + q];
            Taps t = cell_taps(h, cx, cy, grid, sx, sy);
            if (!inside) t.valid = 0;
            const Box4 bxt = block_box(t, red, wave, lane);  // one barrier; red[] reused after the next barrier
            if (bxt.x1 < 0) {
                __syncthreads();  // red[] is read by every wave before the next view rewrites it
                continue;
            }
            if (per_view) load_g(gout + (int64_t)n * C * plane);
            // A footprint too large for four per-wave copies is done in two halves of the tile (waves 0-1, then
            // 2-3), each with its own (smaller) box and two copies of twice the size -- instead of adding every run
            // straight to global memory.
            const int npt = (bxt.x1 - bxt.x0 + 1) * (bxt.y1 - bxt.y0 + 1);
            const int parts = npt <= maxpix ? 1 : 2;
            for (int part = 0; part < parts; ++part) {
                const bool active = parts == 1 || (wave >> 1) == part;
                Taps tp = t;
                if (!active) tp.valid = 0;
                Box4 bx = bxt;
                if (parts > 1) {
                    __syncthreads();  // red[] consumed before block_box rewrites it
                    bx = block_box(tp, red, wave, lane);
                    if (bx.x1 < 0) {
                        __syncthreads();
                        continue;
                    }
                }
                const int ncop = parts == 1 ? 4 : 2, copy = parts == 1 ? wave : (wave & 1);
                const int bw = bx.x1 - bx.x0 + 1, npix = bw * (bx.y1 - bx.y0 + 1);
                const bool use_img = npix <= pool / (ncop * RB_PIX) - 1;
                const int cpy = (npix + 1) * RB_PIX;  // bytes of one image copy (+ its trash pixel)
                if (use_img) {
                    float4 *z = reinterpret_cast<float4 *>(img);
                    for (int k = tid; k < ncop * cpy / 16; k += RB_NT) z[k] = make_float4(0.f, 0.f, 0.f, 0.f);
                }
                __syncthreads();  // image zeroed; red[] consumed

                if (active) {  // wave-uniform
                    const int key = quad_key(tp);
                    const GSink gs{gfeats + (int64_t)n * sN + (int64_t)c0 * sC, sC, sH, sW, l16, cmax};
                    // byte addresses of this cell's four taps in its wave's image copy, WITHOUT the lane's channel
                    // offset (the addresses are row-broadcast from the owning lane; run_flush adds 16 * lane16);
                    // invalid taps -> the copy's trash pixel
                    const int cb = copy * cpy;
                    const int px = tp.x0 - bx.x0, py = tp.y0 - bx.y0;
                    int a[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        a[u] = use_img && (tp.valid & (1u << u)) ? cb + ((py + (u >> 1)) * bw + px + (u & 1)) * RB_PIX
                                                                 : cb + npix * RB_PIX;
                    walk_row(g, key, a, tp.w, use_img, rw, smem, gs);
                }

                if (use_img) {
                    __syncthreads();  // every row's quad sums are in the image
                    float *gfv = gfeats + (int64_t)n * sN + (int64_t)c0 * sC;
                    if (sC == 1) {  // channels contiguous: one pixel per wave instruction, lane = channel
                        for (int p0 = wave * 4; p0 < npix; p0 += 16) {  // 4 pixels per wave in flight
                            float val[4];
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                val[u] = 0.0f;
                                if (p0 + u < npix) {
#pragma unroll
                                    for (int w = 0; w < 4; ++w)
                                        if (w < ncop) val[u] += img[(w * cpy) / 4 + (p0 + u) * 64 + lane];
                                }
                            }
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                const int p = p0 + u, qy = p / bw, qx = p - qy * bw;
                                if (val[u] != 0.0f && lane < cmax)
                                    unsafeAtomicAdd(gfv + (int64_t)(bx.y0 + qy) * sH + (int64_t)(bx.x0 + qx) * sW + lane,
                                                    val[u]);
                            }
                        }
                    } else {  // lanes along x: for each (channel, footprint row), 64 consecutive pixels per step
                        const int bh = npix / bw;
                        for (int r = wave; r < cmax * bh; r += 4) {
                            const int c = r / bh, qy = r - c * bh;
                            for (int qx = lane; qx < bw; qx += 64) {
                                float val = 0.0f;
#pragma unroll
                                for (int w = 0; w < 4; ++w)
                                    if (w < ncop) val += img[(w * cpy) / 4 + (qy * bw + qx) * 64 + c];
                                if (val != 0.0f)
                                    unsafeAtomicAdd(gfv + (int64_t)c * sC + (int64_t)(bx.y0 + qy) * sH +
                                                        (int64_t)(bx.x0 + qx) * sW,
                                                    val);
                            }
                        }
                    }
                }
                __syncthreads();  // the image is free for the next part / view
            }
        }
    }
}

}  // namespace

// Shared launcher: zero the gradient, then one workgroup per (frame, tile).
static int warp_bwd_runs(const float *gout, const float *Hmat, const float *xs, const float *ys, int B, int V, int C,
                         int Hf, int Wf, float sx, float sy, int Hb, int Wb, int mean, int per_view, float *gfeats,
                         int64_t sN, int64_t sC, int64_t sH, int64_t sW, hipStream_t st) {
    // zero the [B*V] maps (any strides that cover a dense block: NCHW or NHWC)
    const int64_t n_el = (int64_t)B * V * C * Hf * Wf;
    hipError_t e = hipMemsetAsync(gfeats, 0, sizeof(float) * (size_t)n_el, st);
    if (e != hipSuccess) return rb_err(e);
    if (Hb == 0 || Wb == 0) return 0;
    const int ntiles = ((Wb + RB_T - 1) / RB_T) * ((Hb + RB_T - 1) / RB_T);
    const int pool = (warp_bwd_pool_floats() * 4) & ~15;  // LDS image bytes (default 48 KiB: 3 workgroups per CU)
    hipLaunchKernelGGL(k_warp_bwd_runs, dim3(ntiles, B), dim3(RB_NT), pool + 16 * sizeof(int), st, gout, Hmat, xs, ys,
                       V, C, Hf, Wf, sx, sy, Hb, Wb, mean, per_view, gfeats, sN, sC, sH, sW, pool);
    return rb_err(hipGetLastError());
}

static bool dense_nchw_or_nhwc(int C, int Hf, int Wf, int64_t sN, int64_t sC, int64_t sH, int64_t sW) {
    const int64_t P = (int64_t)Hf * Wf;
    const bool nchw = sW == 1 && sH == Wf && sC == P && sN == C * P;
    const bool nhwc = sC == 1 && sW == C && sH == (int64_t)Wf * C && sN == C * P;
    return nchw || nhwc;
}

extern "C" {

int bev_ipm_warp_bwd_f32(const float *gout, const float *Hmat, const float *xs, const float *ys, int N, int C, int Hf,
                         int Wf, float sx, float sy, int Hb, int Wb, float *gfeats, void *stream) {
    return bev_ipm_warp_bwd_ex_f32(gout, Hmat, xs, ys, N, C, Hf, Wf, sx, sy, Hb, Wb, gfeats, (int64_t)C * Hf * Wf,
                                   (int64_t)Hf * Wf, Wf, 1, stream);
}

int bev_ipm_warp_bwd_ex_f32(const float *gout, const float *Hmat, const float *xs, const float *ys, int N, int C,
                            int Hf, int Wf, float sx, float sy, int Hb, int Wb, float *gfeats, int64_t sN, int64_t sC,
                            int64_t sH, int64_t sW, void *stream) {
    if (N < 0 || C < 0 || Hf <= 0 || Wf <= 0 || Hb < 0 || Wb < 0 || N > 65535) return BEV_ERR_ARGS;
    if (Hf >= 16383 || Wf >= 16383 || !dense_nchw_or_nhwc(C, Hf, Wf, sN, sC, sH, sW)) return BEV_ERR_ARGS;
    if (N == 0 || C == 0) return 0;
    // per-view gradient maps: one "frame" per map, V = 1
    return warp_bwd_runs(gout, Hmat, xs, ys, N, 1, C, Hf, Wf, sx, sy, Hb, Wb, 0, 1, gfeats, sN, sC, sH, sW,
                         (hipStream_t)stream);
}

int bev_ipm_warp_fuse_bwd_f32(const float *gout, const float *Hmat, const float *xs, const float *ys, int B, int V,
                              int C, int Hf, int Wf, float sx, float sy, int Hb, int Wb, int mode, float *gfeats,
                              void *stream) {
    return bev_ipm_warp_fuse_bwd_ex_f32(gout, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, gfeats,
                                        (int64_t)C * Hf * Wf, (int64_t)Hf * Wf, Wf, 1, stream);
}

int bev_ipm_warp_fuse_bwd_ex_f32(const float *gout, const float *Hmat, const float *xs, const float *ys, int B,
                                 int V, int C, int Hf, int Wf, float sx, float sy, int Hb, int Wb, int mode,
                                 float *gfeats, int64_t sN, int64_t sC, int64_t sH, int64_t sW, void *stream) {
    if (B < 0 || V <= 0 || C < 0 || Hf <= 0 || Wf <= 0 || Hb < 0 || Wb < 0 || B > 65535) return BEV_ERR_ARGS;
    if (mode != BEV_FUSE_SUM && mode != BEV_FUSE_MEAN) return BEV_ERR_ARGS;
    if (Hf >= 16383 || Wf >= 16383 || !dense_nchw_or_nhwc(C, Hf, Wf, sN, sC, sH, sW)) return BEV_ERR_ARGS;
    if (B == 0 || C == 0) return 0;
    return warp_bwd_runs(gout, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode == BEV_FUSE_MEAN, 0, gfeats, sN, sC,
                         sH, sW, (hipStream_t)stream);
}

}  // extern "C"
