// bev_warp_fuse.hip -- fused IPM warp + N-view reduce for gfx950: the "unit
// pipeline" kernel behind bev_ipm_warp_fuse_f32 (GeometryTransformer.forward
// per-(b,v) grid_sample loop, geometry.py:120-162, followed by SimpleFusion,
// fusion.py:17-22, without materialising the [B,V,C,Hb,Wb] intermediate).
//
// One 256-thread workgroup owns an 8 x 32 tile of BEV cells (lane = cell; wave
// w holds rows 2w and 2w+1, so every per-channel store is two full 128-B
// lines).  Work per tile:
//
//  1. Taps, all views at once.  Every lane computes (ix, iy) of its cell in
//     each view of a group of up to 8 views (bit-exact recipe, bev_geometry.h)
//     and keeps them in registers; the exact bounding box of the valid taps is
//     reduced per wave (packed 16-bit shuffles) and per tile (LDS, one
//     barrier).  Eight independent tap chains per lane hide each other's
//     latency; nothing is recomputed later.
//  2. Plan.  Each view's footprint image is staged into LDS in "units" of ck
//     channels (ck = 64, 32, 16 or 8; pixel stride 4*ck + 16 B = an odd number
//     of 16-B slots, so ds_read_b128 is conflict-free).  ck is the largest that
//     lets the unit sit beside its predecessor in the pool; consecutive units
//     are anchored at opposite ends of the pool.  A footprint too large even at
//     8 channels is sampled straight from global memory ("direct" unit).
//  3. Pipeline.  Unit u+1 is copied global -> LDS with LDS-DMA
//     (global_load_lds_dwordx4) while unit u is sampled (four ds_read_b128 per
//     4 channels, packed bilinear FMAs, software-pipelined by one group);
//     then vmcnt(0) + one barrier.  No synchronous staging.
//  4. Store.  acc (64 channels per pass) -> nt buffer stores, mean divides by V.
//
// Exactness: taps are the bit recipe; per channel the views are accumulated
// in order v = 0..V-1 from +0 (or -inf for max).  Skipping a view for a wave
// whose cells have no valid tap adds nothing for sum/mean (the sample is +0
// and the accumulator is never -0); max applies max(acc, +0) at that point in
// the view order.  Cells whose tap coordinate is not finite get NaN weights in
// the reference (0 * NaN), i.e. NaN output: reproduced explicitly.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "bev_geometry.h"
#include "bev_warp_fuse.h"
#include "../../include/bev_mi355x.h"

using namespace bev;

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int UT_H = 8, UT_W = 32, UT_NT = UT_H * UT_W;
constexpr int VG = 8;                 // views per tap group
constexpr int ZP_BYTES = 256;         // all-zero pixel (64 channels)
constexpr int RED_BYTES = VG * 4 * 8; // per (view, wave) packed boxes
constexpr int CODE_DIRECT = 5;        // plan code: sample from global memory

__device__ __forceinline__ unsigned lds_addr(const unsigned char *p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) unsigned char *)p;
}

// exact p / d for 0 <= p < 2^22, 1 <= d < 2^22 (float estimate + one correction)
__device__ __forceinline__ int fdiv(int p, int d, float inv_d) {
    int q = (int)((float)p * inv_d);
    const int r = p - q * d;
    q += (r >= d) - (r < 0);
    return q;
}

// bytes of a unit image: whole 1-KiB DMA pieces of (ck/4 + 1) 16-B slots per pixel
__device__ __forceinline__ int unit_bytes(int npix, int code) {
    const int S = (16 >> (4 - code)) + 1;  // code 4: 17, 3: 9, 2: 5, 1: 3
    return ((npix * S + 63) >> 6) << 10;
}

__device__ __forceinline__ int pk2(int lo, int hi) { return (lo & 0xffff) | (hi << 16); }
__device__ __forceinline__ int pk_lo(int v) { return (int)(short)(v & 0xffff); }
__device__ __forceinline__ int pk_hi(int v) { return v >> 16; }
typedef short short2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int pk_min(int a, int b) {
    return __builtin_bit_cast(int, __builtin_elementwise_min(__builtin_bit_cast(short2_t, a),
                                                             __builtin_bit_cast(short2_t, b)));
}

// a[k] for a wave-uniform k as a v_cndmask chain (the opaque copies keep LLVM
// from turning the chain back into a dynamic index, which it lowers to scratch).
template <int N>
__device__ __forceinline__ float pick(const float (&a)[N], int k) {
    float r = a[0];
#pragma unroll
    for (int i = 1; i < N; ++i) {
        float t = a[i];
        asm("" : "+v"(t));
        r = (k == i) ? t : r;
    }
    return r;
}

// Issue the LDS-DMA of one unit: footprint (x0, y0, bw x bh = npix pixels) of
// channels [c, c + ck) of view base f, into LDS byte offset off.  Slot s of the
// image (16 B) is pixel s / S, channel group s % S; the pad group re-reads
// group 0.  Element offsets are 32-bit (checked by the launcher).
__device__ __forceinline__ void dma_unit(const float *__restrict__ f, int sH, int sW, int x0, int y0, int bw,
                                         int npix, int code, unsigned char *smem, int off, int wave, int lane) {
    const int S = (16 >> (4 - code)) + 1;
    const int ninstr = (npix * S + 63) >> 6;
    const float inv_S = 1.0f / (float)S, inv_bw = 1.0f / (float)bw;
    const int base = y0 * sH + x0 * sW;
    for (int k = wave; k < ninstr; k += UT_NT / 64) {
        const int slot = k * 64 + lane;
        const int p = fdiv(slot, S, inv_S), sl = slot - p * S;
        const int py = fdiv(p, bw, inv_bw), px = p - py * bw;
        const int eo = base + py * sH + px * sW + ((sl < S - 1) ? sl * 4 : 0);
        const float *src = f + ((p < npix) ? eo : 0);  // tail lanes: any valid address
        // inline asm: the builtin makes hipcc drain vmcnt before later ds_reads,
        // which would serialise the prefetch; completion is awaited explicitly.
        const unsigned dst = (unsigned)__builtin_amdgcn_readfirstlane((int)(lds_addr(smem) + off + k * 1024));
        unsigned keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(src), "s"(dst)
            : "memory");
    }
}

// bilerp of 4 channels as two packed chains: per element exactly
// fma(se, wse, fma(sw, wsw, fma(ne, wne, nw * wnw))), then acc + s or max.
template <int MODE>
__device__ __forceinline__ void bilerp4(float (&acc)[64], int q0, const f32x4 &nw, const f32x4 &ne, const f32x4 &sw,
                                        const f32x4 &se, const float (&w)[4]) {
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

// Sample channels [Q*CK, Q*CK + CK) of the accumulator from a unit image; a0..a3
// are the LDS byte addresses of the four taps (the zero pixel for invalid ones).
template <int MODE, int CK, int Q>
__device__ __forceinline__ void sample_unit(float (&acc)[64], const unsigned char *smem, int a0, int a1, int a2,
                                            int a3, const float (&w)[4]) {
    constexpr int G = CK / 4;
    const unsigned char *p0 = smem + a0, *p1 = smem + a1, *p2 = smem + a2, *p3 = smem + a3;
    f32x4 c0 = *(const f32x4 *)p0, c1 = *(const f32x4 *)p1, c2 = *(const f32x4 *)p2, c3 = *(const f32x4 *)p3;
#pragma unroll
    for (int g = 0; g < G; ++g) {
        f32x4 n0, n1, n2, n3;
        if (g + 1 < G) {
            n0 = *(const f32x4 *)(p0 + (g + 1) * 16);
            n1 = *(const f32x4 *)(p1 + (g + 1) * 16);
            n2 = *(const f32x4 *)(p2 + (g + 1) * 16);
            n3 = *(const f32x4 *)(p3 + (g + 1) * 16);
        }
        bilerp4<MODE>(acc, Q * CK + 4 * g, c0, c1, c2, c3, w);
        __builtin_amdgcn_sched_barrier(0);  // at most two groups of reads in flight
        if (g + 1 < G) {
            c0 = n0;
            c1 = n1;
            c2 = n2;
            c3 = n3;
        }
    }
}

template <int MODE>
__device__ __forceinline__ void sample_code(float (&acc)[64], int code, int q, const unsigned char *smem, int a0,
                                            int a1, int a2, int a3, const float (&w)[4]) {
#define SU(CK, Q) sample_unit<MODE, CK, Q>(acc, smem, a0, a1, a2, a3, w)
    switch (code) {
        case 4: SU(64, 0); break;
        case 3: if (q == 0) SU(32, 0); else SU(32, 1); break;
        case 2:
            switch (q) {
                case 0: SU(16, 0); break;
                case 1: SU(16, 1); break;
                case 2: SU(16, 2); break;
                default: SU(16, 3);
            }
            break;
        default:
            switch (q) {
                case 0: SU(8, 0); break;
                case 1: SU(8, 1); break;
                case 2: SU(8, 2); break;
                case 3: SU(8, 3); break;
                case 4: SU(8, 4); break;
                case 5: SU(8, 5); break;
                case 6: SU(8, 6); break;
                default: SU(8, 7);
            }
    }
#undef SU
}

// Direct unit: all 64 channels of one view gathered from global memory.
template <int MODE>
__device__ __forceinline__ void sample_direct(float (&acc)[64], const float *__restrict__ f, int sH, int sW, int x0,
                                             int y0, unsigned val, const float (&w)[4]) {
    const int base = y0 * sH + x0 * sW;
    const float *p0 = f + ((val & 1) ? base : 0), *p1 = f + ((val & 2) ? base + sW : 0);
    const float *p2 = f + ((val & 4) ? base + sH : 0), *p3 = f + ((val & 8) ? base + sH + sW : 0);
    const f32x4 z = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < 16; ++g) {
        f32x4 c0 = *(const f32x4 *)(p0 + 4 * g), c1 = *(const f32x4 *)(p1 + 4 * g);
        f32x4 c2 = *(const f32x4 *)(p2 + 4 * g), c3 = *(const f32x4 *)(p3 + 4 * g);
        c0 = (val & 1) ? c0 : z;
        c1 = (val & 2) ? c1 : z;
        c2 = (val & 4) ? c2 : z;
        c3 = (val & 8) ? c3 : z;
        bilerp4<MODE>(acc, 4 * g, c0, c1, c2, c3, w);
        __builtin_amdgcn_sched_barrier(0);  // bounded register footprint (rare path)
    }
}

template <int MODE>
__device__ __forceinline__ void zero_view(float (&acc)[64]) {
    if (MODE == BEV_FUSE_MAX) {
#pragma unroll
        for (int q = 0; q < 64; ++q) acc[q] = nan_max(acc[q], 0.0f);
    }
}

// nt stores of one 64-channel chunk through a buffer descriptor (chunk < 4 GiB,
// checked by the launcher); mean divides by V exactly (div_rcp).
template <int MODE>
__device__ __forceinline__ void store_chunk(float *chunk, size_t plane, int cell, const float (&acc)[64], double rV) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(chunk, 0, (int)(uint32_t)(plane * 64 * sizeof(float)), 0x00020000);
    const int voff = cell * (int)sizeof(float);
#pragma unroll
    for (int q = 0; q < 64; ++q) {
        float a = acc[q];
        asm volatile("" : "+v"(a)::"memory");  // convert after the previous store (no hoisted doubles)
        const float r = (MODE == BEV_FUSE_MEAN) ? div_rcp(a, rV) : a;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, r), rs, voff,
                                              (int)(uint32_t)(q * plane * sizeof(float)), 2);
    }
}

// index of the first non-zero 4-bit plan code above view k (8 = none)
__device__ __forceinline__ int next_view(unsigned plan, int k) {
    const unsigned m = (k + 1 >= 8) ? 0u : (plan >> (4 * (k + 1)));
    const unsigned nz = (m | (m >> 1) | (m >> 2) | (m >> 3)) & 0x11111111u;
    return nz ? k + 1 + (__builtin_ctz(nz) >> 2) : 8;
}

template <int MODE, int OCC>
__global__ __launch_bounds__(UT_NT, OCC) void k_warp_fuse_units(const float *__restrict__ feats, int64_t sN, int sH,
                                                              int sW, const float *__restrict__ Hmat,
                                                              const float *__restrict__ xs,
                                                              const float *__restrict__ ys, int V, int C, int Hf,
                                                              int Wf, float sx, float sy, int Hb, int Wb,
                                                              float *__restrict__ out, int pool, int dbg) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int zp = pool;
    int *red = reinterpret_cast<int *>(smem + pool + ZP_BYTES);

    // XCD-aware tile order: consecutive blockIdx go round-robin over the 8 XCDs;
    // remap so each XCD walks a contiguous run of tiles (shared source pixels in one L2).
    const int ntx = (Wb + UT_W - 1) / UT_W, nty = (Hb + UT_H - 1) / UT_H, nt = ntx * nty;
    int tile = blockIdx.x;
    {
        const int q = nt / 8, r = nt % 8, x = tile % 8;
        tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + tile / 8;
    }
    const int tyb = tile / ntx, txb = tile - tyb * ntx;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int i = tyb * UT_H + wave * 2 + (lane >> 5);
    const int j = txb * UT_W + (lane & 31);
    const int b = blockIdx.y;
    const bool inside = (i < Hb) && (j < Wb);
    const float cx = xs[inside ? j : 0], cy = ys[inside ? i : 0];
    const size_t plane = (size_t)Hb * Wb;
    const Grid grid = make_grid(Hf, Wf);
    const double rV = recip_uniform(V);
    const int ng = (V + VG - 1) / VG;
    if (tid < ZP_BYTES / 16) *(f32x4 *)(smem + zp + tid * 16) = (f32x4){0.f, 0.f, 0.f, 0.f};

    float ixs[VG], iys[VG];
    unsigned vbits = 0, poison = 0, wany = 0, plan = 0;
    int P0 = 0, P1 = 0, NP = 0;  // lane k: box origin (x0 | y0 << 16), size (bw | bh << 16), npix of view k

    for (int c0 = 0; c0 < C; c0 += 64) {
        float acc[64];
#pragma unroll
        for (int q = 0; q < 64; ++q) acc[q] = (MODE == BEV_FUSE_MAX) ? -__builtin_inff() : 0.0f;

        for (int g = 0; g < ng; ++g) {
            const int v0 = g * VG, nv = min(VG, V - v0);
            if (c0 == 0 || ng > 1) {
                // ---- 1. taps of all views of the group, wave boxes -> red[] -------------
                if (c0 > 0 || g > 0) __syncthreads();  // red[] of the previous group is read
                vbits = 0;
                wany = 0;
#pragma unroll
                for (int k = 0; k < VG; ++k) {
                    if (k < nv) {
                        const float *hp = Hmat + 9 * (b * V + v0 + k);
                        float h[9];
#pragma unroll
                        for (int e = 0; e < 9; ++e) h[e] = hp[e];
                        float ix, iy;
                        cell_ixy(h, cx, cy, grid, sx, sy, ix, iy);
                        const unsigned val = inside ? ixy_valid(ix, iy, grid) : 0u;
                        ixs[k] = ix;
                        iys[k] = iy;
                        vbits |= val << (4 * k);
                        poison |= (inside && !(__builtin_isfinite(ix) && __builtin_isfinite(iy))) ? 1u : 0u;
                        int mn = pk2(32767, 32767), mx = pk2(32767, 32767);
                        if (val) {
                            const int x0 = (int)__builtin_floorf(ix), y0 = (int)__builtin_floorf(iy);
                            const int xl = (val & 5) ? x0 : x0 + 1, xh = (val & 10) ? x0 + 1 : x0;
                            const int yl = (val & 3) ? y0 : y0 + 1, yh = (val & 12) ? y0 + 1 : y0;
                            mn = pk2(xl, yl);
                            mx = pk2(-xh, -yh);
                        }
#pragma unroll
                        for (int o = 32; o > 0; o >>= 1) {
                            mn = pk_min(mn, __shfl_xor(mn, o));
                            mx = pk_min(mx, __shfl_xor(mx, o));
                        }
                        if (lane == 0) {
                            red[(k * 4 + wave) * 2] = mn;
                            red[(k * 4 + wave) * 2 + 1] = mx;
                        }
                        wany |= (__ballot(val != 0u) != 0ull) ? (1u << k) : 0u;
                    }
                    __builtin_amdgcn_sched_barrier(0);  // one view's chain at a time (register bound)
                }
                __syncthreads();
                // ---- 2. tile boxes (lane k <-> view k) and the unit plan ----------------
                P0 = P1 = NP = 0;
                if (lane < nv) {
                    int mn = red[(lane * 4) * 2], mx = red[(lane * 4) * 2 + 1];
#pragma unroll
                    for (int w = 1; w < 4; ++w) {
                        mn = pk_min(mn, red[(lane * 4 + w) * 2]);
                        mx = pk_min(mx, red[(lane * 4 + w) * 2 + 1]);
                    }
                    if (pk_lo(mn) != 32767) {
                        const int x0 = pk_lo(mn), y0 = pk_hi(mn), x1 = -pk_lo(mx), y1 = -pk_hi(mx);
                        const int bw = x1 - x0 + 1, bh = y1 - y0 + 1;
                        P0 = pk2(x0, y0);
                        P1 = pk2(bw, bh);
                        NP = bw * bh;
                    }
                }
                plan = 0;
                int prev = 0;
                for (int k = 0; k < nv; ++k) {
                    const int npix = __builtin_amdgcn_readlane(NP, k);
                    if (npix == 0) continue;
                    int code = CODE_DIRECT, sz = 0;
                    for (int c = 4; c >= 1; --c) {
                        const int s = unit_bytes(npix, c);
                        if (s + prev <= pool && (c == 4 || 2 * s <= pool)) {
                            code = c;
                            sz = s;
                            break;
                        }
                    }
                    if (dbg & 1) code = CODE_DIRECT;
                    prev = sz;
                    plan |= (unsigned)code << (4 * k);
                }
            }

            // ---- 3. unit pipeline ----------------------------------------------------
            const float *fg = feats + (int64_t)(b * V + v0) * sN + c0;
            int k = (plan & 15u) ? 0 : next_view(plan, 0);
            if (k >= nv) {
                zero_view<MODE>(acc);  // no view of the group has a valid tap in this tile
                continue;
            }
            int code = (plan >> (4 * k)) & 15, q = 0, off = 0, par = 0, lastk = -1;
            auto issue = [&](int kk, int qq, int cd, int of) {
                const int p0 = __builtin_amdgcn_readlane(P0, kk), p1 = __builtin_amdgcn_readlane(P1, kk);
                const int bw = p1 & 0xffff, bh = p1 >> 16;
                dma_unit(fg + (int64_t)kk * sN + qq * (4 << cd), sH, sW, pk_lo(p0), pk_hi(p0), bw, bw * bh, cd, smem,
                         of, wave, lane);
            };
            if (code != CODE_DIRECT) issue(k, 0, code, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            while (true) {
                // next unit: DMA beside the live image (opposite end of the pool)
                int nk = k, nq = q + 1;
                if (code == CODE_DIRECT || nq >= (16 >> code)) {
                    nk = next_view(plan, k);
                    nq = 0;
                }
                int ncode = 0, noff = 0;
                if (nk < nv) {
                    ncode = (plan >> (4 * nk)) & 15;
                    if (ncode != CODE_DIRECT) {
                        const int np = __builtin_amdgcn_readlane(NP, nk);
                        noff = par ? 0 : pool - unit_bytes(np, ncode);
                        if (!(dbg & 8)) issue(nk, nq, ncode, noff);
                    }
                }
                // sample the current unit
                if (MODE == BEV_FUSE_MAX && q == 0 && k > lastk + 1) zero_view<MODE>(acc);
                if (!((wany >> k) & 1u)) {
                    if (q == 0) zero_view<MODE>(acc);
                } else if (!(dbg & 2)) {
                    const float ix = pick(ixs, k), iy = pick(iys, k);
                    const unsigned val = (vbits >> (4 * k)) & 15u;
                    const float xw = __builtin_floorf(ix), yn = __builtin_floorf(iy);
                    const float we = ix - xw, e = 1.0f - we, n = iy - yn, s = 1.0f - n;
                    const float w[4] = {s * e, s * we, n * e, n * we};
                    const int x0 = val ? (int)xw : 0, y0 = val ? (int)yn : 0;
                    if (code == CODE_DIRECT) {
                        sample_direct<MODE>(acc, fg + (int64_t)k * sN, sH, sW, x0, y0, val, w);
                    } else {
                        const int p0 = __builtin_amdgcn_readlane(P0, k), p1 = __builtin_amdgcn_readlane(P1, k);
                        const int bw = p1 & 0xffff, ps = (4 << code) * 4 + 16;
                        const int pb = off + ((y0 - pk_hi(p0)) * bw + (x0 - pk_lo(p0))) * ps;
                        const int a0 = (val & 1) ? pb : zp, a1 = (val & 2) ? pb + ps : zp;
                        const int a2 = (val & 4) ? pb + bw * ps : zp, a3 = (val & 8) ? pb + (bw + 1) * ps : zp;
                        sample_code<MODE>(acc, code, q, smem, a0, a1, a2, a3, w);
                    }
                }
                lastk = k;
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of the next unit landed
                __syncthreads();                                   // all of it; the current image is free
                if (nk >= nv) break;
                k = nk;
                q = nq;
                code = ncode;
                off = noff;
                par ^= 1;
            }
            if (MODE == BEV_FUSE_MAX && lastk < nv - 1) zero_view<MODE>(acc);
        }
        if (poison && !(dbg & 4)) {
#pragma unroll
            for (int q = 0; q < 64; ++q) acc[q] = __builtin_nanf("");
        }
        if (inside && !(dbg & 4)) store_chunk<MODE>(out + ((size_t)b * C + c0) * plane, plane, i * Wb + j, acc, rV);
        if (dbg & 4) {
            float z = 0.f;
#pragma unroll
            for (int q = 0; q < 64; ++q) z += acc[q];
            if (z == 12345.f) out[0] = z;  // keep acc live
        }
    }
}

// -------------------------------------------------------------------------
// per-wave variant: every wave owns a 4 x 16 cell tile, its own LDS pool and
// its own unit pipeline -> no workgroup barrier, no cross-wave reduction.
// -------------------------------------------------------------------------
// Min over the wave of packed 16-bit pairs by DPP (quad perms, row rotates,
// row broadcasts; the full-wave result lands in lane 63).
__device__ __forceinline__ int wave_pkmin(int x) {
    x = pk_min(x, __builtin_amdgcn_update_dpp(x, x, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
    x = pk_min(x, __builtin_amdgcn_update_dpp(x, x, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
    x = pk_min(x, __builtin_amdgcn_update_dpp(x, x, 0x124, 0xF, 0xF, false));  // row_ror:4
    x = pk_min(x, __builtin_amdgcn_update_dpp(x, x, 0x128, 0xF, 0xF, false));  // row_ror:8
    x = pk_min(x, __builtin_amdgcn_update_dpp(x, x, 0x142, 0xA, 0xF, false));  // row_bcast:15
    x = pk_min(x, __builtin_amdgcn_update_dpp(x, x, 0x143, 0xC, 0xF, false));  // row_bcast:31
    return __builtin_amdgcn_readlane(x, 63);
}

// exact unit image bytes (per-wave DMA masks the tail lanes)
__device__ __forceinline__ int unit_bytes_exact(int npix, int code) { return npix * ((16 >> (4 - code)) + 1) * 16; }

// LDS-DMA of one unit issued entirely by the calling wave (tail lanes masked).
__device__ __forceinline__ void dma_unit_wave(const float *__restrict__ f, int sH, int sW, int x0, int y0, int bw,
                                              int npix, int code, unsigned dst0, int lane) {
    const int S = (16 >> (4 - code)) + 1;
    const int total = npix * S, ninstr = (total + 63) >> 6;
    const float inv_S = 1.0f / (float)S, inv_bw = 1.0f / (float)bw;
    const int base = y0 * sH + x0 * sW;
    for (int k = 0; k < ninstr; ++k) {
        const int slot = k * 64 + lane;
        const int p = fdiv(slot, S, inv_S), sl = slot - p * S;
        const int py = fdiv(p, bw, inv_bw), px = p - py * bw;
        const int eo = base + py * sH + px * sW + ((sl < S - 1) ? sl * 4 : 0);
        const float *src = f + ((p < npix) ? eo : 0);
        const unsigned dst = (unsigned)__builtin_amdgcn_readfirstlane((int)(dst0 + k * 1024));
        if (slot < total) {
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

constexpr int WT_H = 4, WT_W = 16;  // per-wave cell tile (4 x 64-B store pieces per channel)

template <int MODE, int OCC>
__global__ __launch_bounds__(UT_NT, OCC) void k_warp_fuse_waves(const float *__restrict__ feats, int64_t sN, int sH,
                                                              int sW, const float *__restrict__ Hmat,
                                                              const float *__restrict__ xs,
                                                              const float *__restrict__ ys, int V, int C, int Hf,
                                                              int Wf, float sx, float sy, int Hb, int Wb,
                                                              float *__restrict__ out, int wpool, int dbg) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int ntx = (Wb + UT_W - 1) / UT_W, nty = (Hb + UT_H - 1) / UT_H, nt = ntx * nty;
    int tile = blockIdx.x;
    {
        const int q = nt / 8, r = nt % 8, x = tile % 8;
        tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + tile / 8;
    }
    const int tyb = tile / ntx, txb = tile - tyb * ntx;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int i = tyb * UT_H + (wave >> 1) * WT_H + (lane >> 4);
    const int j = txb * UT_W + (wave & 1) * WT_W + (lane & 15);
    const int b = blockIdx.y;
    const bool inside = (i < Hb) && (j < Wb);
    const float cx = xs[inside ? j : 0], cy = ys[inside ? i : 0];
    const size_t plane = (size_t)Hb * Wb;
    const Grid grid = make_grid(Hf, Wf);
    const double rV = recip_uniform(V);
    const int ng = (V + VG - 1) / VG;
    // this wave's LDS: [zero pixel 256 B][pool]
    const int zp = wave * wpool, pbase = zp + ZP_BYTES, pool = wpool - ZP_BYTES;
    const unsigned lbase = lds_addr(smem);
    if (lane < ZP_BYTES / 16) *(f32x4 *)(smem + zp + lane * 16) = (f32x4){0.f, 0.f, 0.f, 0.f};

    float ixs[VG], iys[VG];
    unsigned vbits = 0, poison = 0, plan = 0;
    int P0 = 0, P1 = 0;  // lane k: wave box origin (x0 | y0 << 16) and size (bw | bh << 16) of view k

    long long tm[6] = {(long long)__builtin_amdgcn_s_memtime(), 0, 0, 0, 0, 0};
    int nunits = 0;
    for (int c0 = 0; c0 < C; c0 += 64) {
        float acc[64];
#pragma unroll
        for (int q = 0; q < 64; ++q) acc[q] = (MODE == BEV_FUSE_MAX) ? -__builtin_inff() : 0.0f;

        for (int g = 0; g < ng; ++g) {
            const int v0 = g * VG, nv = min(VG, V - v0);
            const float *fg = feats + (int64_t)(b * V + v0) * sN + c0;
            auto issue = [&](int kk, int qq, int cd, int of) {
                const int p0 = __builtin_amdgcn_readlane(P0, kk), p1 = __builtin_amdgcn_readlane(P1, kk);
                const int bw = p1 & 0xffff, bh = p1 >> 16;
                dma_unit_wave(fg + (int64_t)kk * sN + qq * (4 << cd), sH, sW, pk_lo(p0), pk_hi(p0), bw, bw * bh, cd,
                              lbase + pbase + of, lane);
            };
            bool first_issued = false;
            if (c0 == 0 || ng > 1) {
                vbits = 0;
                P0 = P1 = 0;
                plan = 0;
                int prev = 0;
                // the group's homographies, lane q <-> entry q (read back with readlane: no
                // scalar-load latency per view)
                const int hb = 9 * (b * V + v0), hn = 9 * nv;
                const float hv0 = (lane < hn) ? Hmat[hb + lane] : 0.0f;
                const float hv1 = (lane + 64 < hn) ? Hmat[hb + 64 + lane] : 0.0f;
#pragma unroll
                for (int k = 0; k < VG; ++k) {
                    if (k < nv) {
                        float h[9];
#pragma unroll
                        for (int e = 0; e < 9; ++e) {
                            const int q = 9 * k + e;
                            h[e] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(
                                                                 __builtin_bit_cast(int, q < 64 ? hv0 : hv1), q & 63));
                        }
                        float ix, iy;
                        cell_ixy(h, cx, cy, grid, sx, sy, ix, iy);
                        const unsigned val = inside ? ixy_valid(ix, iy, grid) : 0u;
                        ixs[k] = ix;
                        iys[k] = iy;
                        vbits |= val << (4 * k);
                        poison |= (inside && !(__builtin_isfinite(ix) && __builtin_isfinite(iy))) ? 1u : 0u;
                        if (__ballot(val != 0u) != 0ull) {
                            int mn = pk2(32767, 32767), mx = pk2(32767, 32767);
                            if (val) {
                                const int x0 = (int)__builtin_floorf(ix), y0 = (int)__builtin_floorf(iy);
                                const int xl = (val & 5) ? x0 : x0 + 1, xh = (val & 10) ? x0 + 1 : x0;
                                const int yl = (val & 3) ? y0 : y0 + 1, yh = (val & 12) ? y0 + 1 : y0;
                                mn = pk2(xl, yl);
                                mx = pk2(-xh, -yh);
                            }
                            mn = wave_pkmin(mn);
                            mx = wave_pkmin(mx);
                            const int bx0 = pk_lo(mn), by0 = pk_hi(mn);
                            const int bw = -pk_lo(mx) - bx0 + 1, bh = -pk_hi(mx) - by0 + 1;
                            P0 = (lane == k) ? pk2(bx0, by0) : P0;
                            P1 = (lane == k) ? pk2(bw, bh) : P1;
                            // unit plan of view k: largest ck whose image fits beside the
                            // previous unit's; the group's first unit starts copying now
                            const int npix = bw * bh;
                            int code = CODE_DIRECT, sz = 0;
                            for (int c = 4; c >= 1; --c) {
                                const int sb = unit_bytes_exact(npix, c);
                                if (sb + prev <= pool && (c == 4 || 2 * sb <= pool)) {
                                    code = c;
                                    sz = sb;
                                    break;
                                }
                            }
                            if (dbg & 1) code = CODE_DIRECT;
                            prev = sz;
                            plan |= (unsigned)code << (4 * k);
                            if (!first_issued) {
                                first_issued = true;
                                if (code != CODE_DIRECT && !(dbg & 8)) issue(k, 0, code, 0);
                            }
                        }
                    }
                }
                tm[1] = (long long)__builtin_amdgcn_s_memtime();
            }

            tm[2] = (long long)__builtin_amdgcn_s_memtime();
            int k = (plan & 15u) ? 0 : next_view(plan, 0);
            if (k >= nv) {
                zero_view<MODE>(acc);
                continue;
            }
            int code = (plan >> (4 * k)) & 15, q = 0, off = 0, par = 0, lastk = -1;
            if (!first_issued && code != CODE_DIRECT && !(dbg & 8)) issue(k, 0, code, 0);  // chunk loop c0 > 0
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            while (true) {
                int nk = k, nq = q + 1;
                if (code == CODE_DIRECT || nq >= (16 >> code)) {
                    nk = next_view(plan, k);
                    nq = 0;
                }
                int ncode = 0, noff = 0;
                if (nk < nv) {
                    ncode = (plan >> (4 * nk)) & 15;
                    if (ncode != CODE_DIRECT) {
                        const int p1 = __builtin_amdgcn_readlane(P1, nk);
                        noff = par ? 0 : pool - unit_bytes_exact((p1 & 0xffff) * (p1 >> 16), ncode);
                        if (!(dbg & 8)) issue(nk, nq, ncode, noff);
                    }
                }
                if (MODE == BEV_FUSE_MAX && q == 0 && k > lastk + 1) zero_view<MODE>(acc);
                if (!(dbg & 2)) {
                    const float ix = pick(ixs, k), iy = pick(iys, k);
                    const unsigned val = (vbits >> (4 * k)) & 15u;
                    const float xw = __builtin_floorf(ix), yn = __builtin_floorf(iy);
                    const float we = ix - xw, e = 1.0f - we, n = iy - yn, s = 1.0f - n;
                    const float w[4] = {s * e, s * we, n * e, n * we};
                    const int x0 = val ? (int)xw : 0, y0 = val ? (int)yn : 0;
                    if (code == CODE_DIRECT) {
                        sample_direct<MODE>(acc, fg + (int64_t)k * sN, sH, sW, x0, y0, val, w);
                    } else {
                        const int p0 = __builtin_amdgcn_readlane(P0, k), p1 = __builtin_amdgcn_readlane(P1, k);
                        const int bw = p1 & 0xffff, ps = (4 << code) * 4 + 16;
                        const int pb = pbase + off + ((y0 - pk_hi(p0)) * bw + (x0 - pk_lo(p0))) * ps;
                        const int a0 = (val & 1) ? pb : zp, a1 = (val & 2) ? pb + ps : zp;
                        const int a2 = (val & 4) ? pb + bw * ps : zp, a3 = (val & 8) ? pb + (bw + 1) * ps : zp;
                        sample_code<MODE>(acc, code, q, smem, a0, a1, a2, a3, w);
                    }
                }
                ++nunits;
                lastk = k;
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next unit's image landed
                if (nk >= nv) break;
                k = nk;
                q = nq;
                code = ncode;
                off = noff;
                par ^= 1;
            }
            if (MODE == BEV_FUSE_MAX && lastk < nv - 1) zero_view<MODE>(acc);
        }
        tm[3] = (long long)__builtin_amdgcn_s_memtime();
        if (poison && !(dbg & 4)) {
#pragma unroll
            for (int q = 0; q < 64; ++q) acc[q] = __builtin_nanf("");
        }
        if (inside && !(dbg & 4)) store_chunk<MODE>(out + ((size_t)b * C + c0) * plane, plane, i * Wb + j, acc, rV);
        if (dbg & 4) {
            float z = 0.f;
#pragma unroll
            for (int q = 0; q < 64; ++q) z += acc[q];
            if (z == 12345.f) out[0] = z;  // keep acc live
        }
        tm[4] = (long long)__builtin_amdgcn_s_memtime();
        if ((dbg & 64) && lane == 0) {
            int *rec = reinterpret_cast<int *>(out) + ((size_t)(blockIdx.y * gridDim.x + blockIdx.x) * 4 + wave) * 8;
            rec[0] = (int)(tm[1] - tm[0]);
            rec[1] = (int)(tm[2] - tm[1]);
            rec[2] = (int)(tm[3] - tm[2]);
            rec[3] = (int)(tm[4] - tm[3]);
            rec[4] = nunits;
            rec[5] = (int)(plan & 0x7fffffff);
            rec[6] = (int)(tm[0] & 0x7fffffff);
            rec[7] = (int)(tm[4] & 0x7fffffff);
        }
    }
}

// -------------------------------------------------------------------------
// "rounds" variant (default): 8 x 32 tile per workgroup, whole views staged per
// round.  After the taps of all views (one barrier for the tile boxes), the
// units (view k, channel chunk q) are packed in view order into rounds that
// fill one half of the pool; round r+1 is copied (LDS-DMA, spread over the four
// waves) while round r is sampled, so a tile pays ~ (rounds + 1) barriers and
// one exposed copy latency instead of one per view.
// -------------------------------------------------------------------------
__device__ __forceinline__ void dma_unit_wg(const float *__restrict__ f, int sH, int sW, int x0, int y0, int bw,
                                            int npix, int code, unsigned dst0, int first, int lane) {
    const int S = (16 >> (4 - code)) + 1;
    const int total = npix * S, ninstr = (total + 63) >> 6;
    const float inv_S = 1.0f / (float)S, inv_bw = 1.0f / (float)bw;
    const int base = y0 * sH + x0 * sW;
    for (int k = first; k < ninstr; k += UT_NT / 64) {
        const int slot = k * 64 + lane;
        const int p = fdiv(slot, S, inv_S), sl = slot - p * S;
        const int py = fdiv(p, bw, inv_bw), px = p - py * bw;
        const int eo = base + py * sH + px * sW + ((sl < S - 1) ? sl * 4 : 0);
        const float *src = f + ((p < npix) ? eo : 0);
        const unsigned dst = (unsigned)__builtin_amdgcn_readfirstlane((int)(dst0 + k * 1024));
        if (slot < total) {
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

template <int MODE, int OCC>
__global__ __launch_bounds__(UT_NT, OCC) void k_warp_fuse_rounds(const float *__restrict__ feats, int64_t sN, int sH,
                                                               int sW, const float *__restrict__ Hmat,
                                                               const float *__restrict__ xs,
                                                               const float *__restrict__ ys, int V, int C, int Hf,
                                                               int Wf, float sx, float sy, int Hb, int Wb,
                                                               float *__restrict__ out, int half, int dbg) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int zp = 2 * half;
    int *red = reinterpret_cast<int *>(smem + zp + ZP_BYTES);
    const unsigned lbase = lds_addr(smem);

    const int ntx = (Wb + UT_W - 1) / UT_W, nty = (Hb + UT_H - 1) / UT_H, nt = ntx * nty;
    int tile = blockIdx.x;
    {
        const int q = nt / 8, r = nt % 8, x = tile % 8;
        tile = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + tile / 8;
    }
    const int tyb = tile / ntx, txb = tile - tyb * ntx;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int i = tyb * UT_H + wave * 2 + (lane >> 5);
    const int j = txb * UT_W + (lane & 31);
    const int b = blockIdx.y;
    const bool inside = (i < Hb) && (j < Wb);
    const size_t plane = (size_t)Hb * Wb;
    const Grid grid = make_grid(Hf, Wf);
    const double rV = recip_uniform(V);
    const int ng = (V + VG - 1) / VG;
    if (tid < ZP_BYTES / 16) *(f32x4 *)(smem + zp + tid * 16) = (f32x4){0.f, 0.f, 0.f, 0.f};

    float ixs[VG], iys[VG];
    unsigned vbits = 0, poison = 0, wany = 0, plan = 0;
    int P0 = 0, P1 = 0;  // lane k: tile box origin (x0 | y0 << 16) and size (bw | bh << 16) of view k
    long long tm[5] = {(long long)__builtin_amdgcn_s_memtime(), 0, 0, 0, 0};
    int nrounds = 0;

    for (int c0 = 0; c0 < C; c0 += 64) {
        float acc[64];
#pragma unroll
        for (int q = 0; q < 64; ++q) acc[q] = (MODE == BEV_FUSE_MAX) ? -__builtin_inff() : 0.0f;

        for (int g = 0; g < ng; ++g) {
            const int v0 = g * VG, nv = min(VG, V - v0);
            if (c0 == 0 || ng > 1) {
                // ---- taps of all views of the group; wave boxes -> red[] ------------------
                if (c0 > 0 || g > 0) __syncthreads();  // red[] of the previous group is consumed
                const float cx = xs[inside ? j : 0], cy = ys[inside ? i : 0];
                const int hb = 9 * (b * V + v0), hn = 9 * nv;
                const float hv0 = (lane < hn) ? Hmat[hb + lane] : 0.0f;
                const float hv1 = (lane + 64 < hn) ? Hmat[hb + 64 + lane] : 0.0f;
                vbits = 0;
                wany = 0;
#pragma unroll
                for (int k = 0; k < VG; ++k) {
                    if (k < nv) {
                        float h[9];
#pragma unroll
                        for (int e = 0; e < 9; ++e) {
                            const int q = 9 * k + e;
                            h[e] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(
                                                                 __builtin_bit_cast(int, q < 64 ? hv0 : hv1), q & 63));
                        }
                        float ix, iy;
                        cell_ixy(h, cx, cy, grid, sx, sy, ix, iy);
                        const unsigned val = inside ? ixy_valid(ix, iy, grid) : 0u;
                        ixs[k] = ix;
                        iys[k] = iy;
                        vbits |= val << (4 * k);
                        poison |= (inside && !(__builtin_isfinite(ix) && __builtin_isfinite(iy))) ? 1u : 0u;
                        int mn = pk2(32767, 32767), mx = pk2(32767, 32767);
                        if (__ballot(val != 0u) != 0ull) {
                            wany |= 1u << k;
                            if (val) {
                                const int x0 = (int)__builtin_floorf(ix), y0 = (int)__builtin_floorf(iy);
                                const int xl = (val & 5) ? x0 : x0 + 1, xh = (val & 10) ? x0 + 1 : x0;
                                const int yl = (val & 3) ? y0 : y0 + 1, yh = (val & 12) ? y0 + 1 : y0;
                                mn = pk2(xl, yl);
                                mx = pk2(-xh, -yh);
                            }
                            mn = wave_pkmin(mn);
                            mx = wave_pkmin(mx);
                        }
                        if (lane == 0) {
                            red[(k * 4 + wave) * 2] = mn;
                            red[(k * 4 + wave) * 2 + 1] = mx;
                        }
                    }
                }
                __syncthreads();
                // ---- tile boxes (lane k <-> view k) and the unit codes -----------------
                P0 = P1 = 0;
                if (lane < nv) {
                    int mn = red[(lane * 4) * 2], mx = red[(lane * 4) * 2 + 1];
#pragma unroll
                    for (int w = 1; w < 4; ++w) {
                        mn = pk_min(mn, red[(lane * 4 + w) * 2]);
                        mx = pk_min(mx, red[(lane * 4 + w) * 2 + 1]);
                    }
                    if (pk_lo(mn) != 32767) {
                        const int x0 = pk_lo(mn), y0 = pk_hi(mn);
                        P0 = pk2(x0, y0);
                        P1 = pk2(-pk_lo(mx) - x0 + 1, -pk_hi(mx) - y0 + 1);
                    }
                }
                plan = 0;
                for (int k = 0; k < nv; ++k) {
                    const int p1 = __builtin_amdgcn_readlane(P1, k);
                    const int npix = (p1 & 0xffff) * (p1 >> 16);
                    if (npix == 0) continue;
                    int code = CODE_DIRECT;
                    for (int c = 4; c >= 1; --c)
                        if (unit_bytes_exact(npix, c) <= half) {
                            code = c;
                            break;
                        }
                    if (dbg & 1) code = CODE_DIRECT;
                    plan |= (unsigned)code << (4 * k);
                }
                tm[1] = (long long)__builtin_amdgcn_s_memtime();
            }

            // ---- rounds ---------------------------------------------------------------
            const float *fg = feats + (int64_t)(b * V + v0) * sN + c0;
            int k = (plan & 15u) ? 0 : next_view(plan, 0);
            if (k >= nv) {
                zero_view<MODE>(acc);
                continue;
            }
            // Walk the units of one round starting at (k, q) in half h; ISSUE or SAMPLE each;
            // returns the first unit of the next round in (k, q).
            int lastk = -1;
            auto walk = [&](int &wk, int &wq, int h, bool sample) {
                int off = 0, gi = 0;
                while (wk < nv) {
                    const int code = (plan >> (4 * wk)) & 15;
                    const int p1 = __builtin_amdgcn_readlane(P1, wk), p0 = __builtin_amdgcn_readlane(P0, wk);
                    const int bw = p1 & 0xffff, npix = bw * (p1 >> 16);
                    const int sz = (code == CODE_DIRECT) ? 0 : unit_bytes_exact(npix, code);
                    if (off + sz > half && off > 0) break;
                    const int ub = h * half + off;
                    if (!sample) {
                        if (code != CODE_DIRECT && !(dbg & 8)) {
                            const int ni = (npix * ((16 >> (4 - code)) + 1) + 63) >> 6;
                            dma_unit_wg(fg + (int64_t)wk * sN + wq * (4 << code), sH, sW, pk_lo(p0), pk_hi(p0), bw,
                                        npix, code, lbase + ub, (wave - gi) & 3, lane);
                            gi += ni;
                        }
                    } else {
                        if (MODE == BEV_FUSE_MAX && wq == 0 && wk > lastk + 1) zero_view<MODE>(acc);
                        if (!((wany >> wk) & 1u)) {
                            if (wq == 0) zero_view<MODE>(acc);
                        } else if (!(dbg & 2)) {
                            const float ix = pick(ixs, wk), iy = pick(iys, wk);
                            const unsigned val = (vbits >> (4 * wk)) & 15u;
                            const float xw = __builtin_floorf(ix), yn = __builtin_floorf(iy);
                            const float we = ix - xw, e = 1.0f - we, n = iy - yn, s = 1.0f - n;
                            const float w[4] = {s * e, s * we, n * e, n * we};
                            const int x0 = val ? (int)xw : 0, y0 = val ? (int)yn : 0;
                            if (code == CODE_DIRECT) {
                                sample_direct<MODE>(acc, fg + (int64_t)wk * sN, sH, sW, x0, y0, val, w);
                            } else {
                                const int ps = (4 << code) * 4 + 16;
                                const int pb = ub + ((y0 - pk_hi(p0)) * bw + (x0 - pk_lo(p0))) * ps;
                                const int a0 = (val & 1) ? pb : zp, a1 = (val & 2) ? pb + ps : zp;
                                const int a2 = (val & 4) ? pb + bw * ps : zp, a3 = (val & 8) ? pb + (bw + 1) * ps : zp;
                                sample_code<MODE>(acc, code, wq, smem, a0, a1, a2, a3, w);
                            }
                        }
                        lastk = wk;
                    }
                    off += sz;
                    if (code != CODE_DIRECT && wq + 1 < (16 >> code)) ++wq;
                    else {
                        wk = next_view(plan, wk);
                        wq = 0;
                    }
                }
            };
            int q = 0, nk = k, nq = 0, r = 0;
            walk(nk, nq, 0, false);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            while (k < nv) {
                int nk2 = nk, nq2 = nq;
                if (nk2 < nv) walk(nk2, nq2, (r + 1) & 1, false);  // next round's copy
                walk(k, q, r & 1, true);                           // sample this round: ends at (nk, nq)
                ++nrounds;
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                k = nk;
                q = nq;
                nk = nk2;
                nq = nq2;
                ++r;
            }
            if (MODE == BEV_FUSE_MAX && lastk < nv - 1) zero_view<MODE>(acc);
        }
        tm[2] = (long long)__builtin_amdgcn_s_memtime();
        if (poison && !(dbg & 4)) {
#pragma unroll
            for (int q = 0; q < 64; ++q) acc[q] = __builtin_nanf("");
        }
        if (inside && !(dbg & 4)) store_chunk<MODE>(out + ((size_t)b * C + c0) * plane, plane, i * Wb + j, acc, rV);
        if (dbg & 4) {
            float z = 0.f;
#pragma unroll
            for (int q = 0; q < 64; ++q) z += acc[q];
            if (z == 12345.f) out[0] = z;  // keep acc live
        }
        tm[3] = (long long)__builtin_amdgcn_s_memtime();
    }
    if ((dbg & 64) && lane == 0) {
        int *rec = reinterpret_cast<int *>(out) + ((size_t)(blockIdx.y * gridDim.x + blockIdx.x) * 4 + wave) * 8;
        rec[0] = (int)(tm[1] - tm[0]);
        rec[1] = 0;
        rec[2] = (int)(tm[2] - tm[1]);
        rec[3] = (int)(tm[3] - tm[2]);
        rec[4] = nrounds;
        rec[5] = (int)(plan & 0x7fffffff);
        rec[6] = (int)(tm[0] & 0x7fffffff);
        rec[7] = (int)(tm[3] & 0x7fffffff);
    }
}

inline int env_int(const char *name, int dflt) {
    const char *e = getenv(name);
    return e ? atoi(e) : dflt;
}

template <int OCC>
int launch_occ(const float *feats, int64_t sN, int sH, int sW, const float *Hmat, const float *xs, const float *ys,
               int B, int V, int C, int Hf, int Wf, float sx, float sy, int Hb, int Wb, int mode, float *out,
               hipStream_t st, int pool, int dbg) {
    const int ntiles = ((Wb + UT_W - 1) / UT_W) * ((Hb + UT_H - 1) / UT_H);
    dim3 grid(ntiles, B), block(UT_NT);
    const size_t lds = (size_t)pool + ZP_BYTES + RED_BYTES;
#define L(M)                                                                                                          \
    hipLaunchKernelGGL((k_warp_fuse_units<M, OCC>), grid, block, lds, st, feats, sN, sH, sW, Hmat, xs, ys, V, C, Hf, \
                       Wf, sx, sy, Hb, Wb, out, pool, dbg)
    if (mode == BEV_FUSE_SUM) L(BEV_FUSE_SUM);
    else if (mode == BEV_FUSE_MEAN) L(BEV_FUSE_MEAN);
    else L(BEV_FUSE_MAX);
#undef L
    return (int)hipGetLastError();
}


template <int OCC>
int launch_waves(const float *feats, int64_t sN, int sH, int sW, const float *Hmat, const float *xs, const float *ys,
                 int B, int V, int C, int Hf, int Wf, float sx, float sy, int Hb, int Wb, int mode, float *out,
                 hipStream_t st, int pool_kb, int dbg) {
    const int ntiles = ((Wb + UT_W - 1) / UT_W) * ((Hb + UT_H - 1) / UT_H);
    dim3 grid(ntiles, B), block(UT_NT);
    // per wave: 1/(4 OCC) of the CU's 160 KiB unless a pool is forced
    int wpool = pool_kb > 0 ? pool_kb * 1024 + ZP_BYTES : ((160 * 1024 / (4 * OCC)) & ~255);
    if (wpool > 40 * 1024) wpool = 40 * 1024;
    const size_t lds = (size_t)4 * wpool;
#define L(M)                                                                                                          \
    hipLaunchKernelGGL((k_warp_fuse_waves<M, OCC>), grid, block, lds, st, feats, sN, sH, sW, Hmat, xs, ys, V, C, Hf, \
                       Wf, sx, sy, Hb, Wb, out, wpool, dbg)
    if (mode == BEV_FUSE_SUM) L(BEV_FUSE_SUM);
    else if (mode == BEV_FUSE_MEAN) L(BEV_FUSE_MEAN);
    else L(BEV_FUSE_MAX);
#undef L
    return (int)hipGetLastError();
}


template <int OCC>
int launch_rounds(const float *feats, int64_t sN, int sH, int sW, const float *Hmat, const float *xs, const float *ys,
                  int B, int V, int C, int Hf, int Wf, float sx, float sy, int Hb, int Wb, int mode, float *out,
                  hipStream_t st, int pool_kb, int dbg) {
    const int ntiles = ((Wb + UT_W - 1) / UT_W) * ((Hb + UT_H - 1) / UT_H);
    dim3 grid(ntiles, B), block(UT_NT);
    // the CU's 160 KiB over OCC workgroups: two halves + zero pixel + box exchange
    int half = pool_kb > 0 ? pool_kb * 512 : ((160 * 1024 / OCC - ZP_BYTES - RED_BYTES) / 2) & ~15;
    if (half < 1024) half = 1024;
    const size_t lds = (size_t)2 * half + ZP_BYTES + RED_BYTES;
#define L(M)                                                                                                           \
    hipLaunchKernelGGL((k_warp_fuse_rounds<M, OCC>), grid, block, lds, st, feats, sN, sH, sW, Hmat, xs, ys, V, C, Hf, \
                       Wf, sx, sy, Hb, Wb, out, half, dbg)
    if (mode == BEV_FUSE_SUM) L(BEV_FUSE_SUM);
    else if (mode == BEV_FUSE_MEAN) L(BEV_FUSE_MEAN);
    else L(BEV_FUSE_MAX);
#undef L
    return (int)hipGetLastError();
}

}  // namespace

namespace bev {

static int g_pool_kb = -1;  // -1: BEV_WARP_POOL_KB env (or automatic)

int warp_fuse_set_pool_kb(int kb) {
    const int old = g_pool_kb < 0 ? 0 : g_pool_kb;
    g_pool_kb = kb;
    return old;
}

static int g_units = -1;  // -1: BEV_WARP_UNITS env (default off)

int warp_fuse_set_units(int on) {
    const int old = warp_fuse_units_enabled() ? 1 : 0;
    g_units = on ? 1 : 0;
    return old;
}

bool warp_fuse_units_enabled() {
    static const int env_on = env_int("BEV_WARP_UNITS", 0);
    return g_units < 0 ? env_on != 0 : g_units != 0;
}

bool warp_fuse_units_ok(int64_t sN, int64_t sC, int64_t sH, int64_t sW, const float *feats, int C, int Hf, int Wf,
                        int Hb, int Wb) {
    return sC == 1 && C % 64 == 0 && Hf < 16384 && Wf < 16384 && (int64_t)Hf * sH < (1ll << 31) &&
           (int64_t)Wf * sW < (1ll << 31) && (int64_t)(Hf - 1) * sH + (int64_t)(Wf - 1) * sW + C < (1ll << 31) &&
           ((uintptr_t)feats & 15) == 0 && sW % 4 == 0 && sH % 4 == 0 && sN % 4 == 0 &&
           (int64_t)Hb * Wb * 64 * (int64_t)sizeof(float) < (1ll << 32);
}

int warp_fuse_units(const float *feats, int64_t sN, int64_t sH, int64_t sW, const float *Hmat, const float *xs,
                    const float *ys, int B, int V, int C, int Hf, int Wf, float sx, float sy, int Hb, int Wb, int mode,
                    float *out, hipStream_t st) {
    // LDS per workgroup: 4 workgroups (16 waves) per CU at OCC 4 -> 40 KiB each.
    static const int occ = env_int("BEV_WARP_OCC", 2) == 4 ? 4 : 2;
    static const int env_pool_kb = env_int("BEV_WARP_POOL_KB", 0);
    const int pool_kb = g_pool_kb < 0 ? env_pool_kb : g_pool_kb;
    static const int dbg = env_int("BEV_WARP_DEBUG", 0);
    static const int impl = env_int("BEV_WARP_IMPL", 2);  // 2 rounds, 1 per-wave, 0 per-unit workgroup
    static const int wocc = env_int("BEV_WARP_WOCC", 3);
    if (impl == 2) {
        if (wocc == 1)
            return launch_rounds<1>(feats, sN, (int)sH, (int)sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode,
                                    out, st, pool_kb, dbg);
        return launch_rounds<2>(feats, sN, (int)sH, (int)sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out,
                                st, pool_kb, dbg);
    }
    if (impl == 1) {
        if (wocc == 4 && mode != BEV_FUSE_MAX)
            return launch_waves<4>(feats, sN, (int)sH, (int)sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode,
                                   out, st, pool_kb, dbg);
        if (wocc == 2 || mode == BEV_FUSE_MAX)
            return launch_waves<2>(feats, sN, (int)sH, (int)sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode,
                                   out, st, pool_kb, dbg);
        return launch_waves<3>(feats, sN, (int)sH, (int)sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out,
                               st, pool_kb, dbg);
    }
    int pool = pool_kb > 0 ? pool_kb * 1024 : (occ == 4 ? 39 * 1024 : 79 * 1024);
    if (pool < 2048) pool = 2048;
    if (pool > 150 * 1024) pool = 150 * 1024;
    if (occ == 2 || mode == BEV_FUSE_MAX)
        return launch_occ<2>(feats, sN, (int)sH, (int)sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out,
                             st, pool, dbg);
    return launch_occ<4>(feats, sN, (int)sH, (int)sW, Hmat, xs, ys, B, V, C, Hf, Wf, sx, sy, Hb, Wb, mode, out, st,
                         pool, dbg);
}

}  // namespace bev
