// bev_geometry.h -- device-side IPM geometry shared by the warp kernels.
//
// Restates, for one BEV cell, the arithmetic the reference performs through
// torch on the CPU (bit-exact):
//   geometry.py:144-149  uvw = H @ [x y 1]^T (MKL AVX-512 3-term dot), w_safe, u, v
//   geometry.py:151-158  feature-space rescale and [-1,1] normalisation
//   geometry.py:161      grid_sampler_2d unnormalise + floor + bilinear weights
// Everything is plain IEEE fp32 (divisions by launch constants are evaluated
// through an exactly-equivalent double product, div_rcp); FMAs are explicit
// (__builtin_fmaf) and the library is compiled with -ffp-contract=off so no
// other contraction happens.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bev {

// MKL AVX-512 sgemm 3-term dot: accumulator starts at +0 (App. A.2).
__device__ __forceinline__ float dot3(float a0, float a1, float a2, float b0, float b1, float b2) {
    return __builtin_fmaf(a2, b2, __builtin_fmaf(a1, b1, __builtin_fmaf(a0, b0, 0.0f)));
}

// a / b rounded to f32 exactly as IEEE division, for a divisor b that is fixed
// per launch, given rb = 1.0 / (double)b.  Proof: the double product has
// relative error < 2^-52 (two roundings to 53 bits), while the exact quotient
// of two 24-bit-significand floats is never an f32 rounding midpoint and lies at
// least 1 / (2^24 * 2^25) = 2^-49 (relative) away from every midpoint.  So the
// product and a/b round to the same float (zeros, infinities, NaNs and f32
// subnormal results included).  3 VALU instead of the 11-instruction f32
// division sequence.
__device__ __forceinline__ float div_rcp(float a, double rb) { return (float)((double)a * rb); }

// A wave-uniform double held in SGPRs (the VALU double division that produced
// it leaves it in VGPRs otherwise).
__device__ __forceinline__ double uniform_d(double d) {
    const uint64_t b = __builtin_bit_cast(uint64_t, d);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double recip_uniform(int n) { return uniform_d(1.0 / (double)n); }

// Per-launch constants of the feature-map grid.
struct Grid {
    float fWf, fHf;  // (float)Wf, (float)Hf
    double rWf, rHf; // 1 / Wf, 1 / Hf in double (div_rcp)
};
__device__ __forceinline__ Grid make_grid(int Hf, int Wf) {
    return Grid{(float)Wf, (float)Hf, recip_uniform(Wf), recip_uniform(Hf)};
}

// Bilinear taps of one BEV cell in one feature map.
struct Taps {
    int x0, y0;       // top-left corner (only meaningful for valid taps)
    float w[4];       // nw, ne, sw, se
    unsigned valid;   // bit0 nw, bit1 ne, bit2 sw, bit3 se
};

// Unnormalised sampling coordinates (ix, iy) of one BEV cell in one feature map.
// h[9] = world->image homography, (x, y) = BEV cell centre on the ground plane.
__device__ __forceinline__ void cell_ixy(const float h[9], float x, float y, const Grid &g, float sx, float sy,
                                         float &ix, float &iy) {
    // geometry.py:144-149
    const float u0 = dot3(h[0], h[1], h[2], x, y, 1.0f);
    const float u1 = dot3(h[3], h[4], h[5], x, y, 1.0f);
    const float w = dot3(h[6], h[7], h[8], x, y, 1.0f);
    const float ws = (__builtin_fabsf(w) < 1e-6f) ? 1.0f : w;
    // u0 / ws and u1 / ws as IEEE f32 divisions, through ONE double reciprocal of ws: rcp_f64 refined by two
    // Newton steps is within ~2^-53 of 1/ws, so (double)u0 * rws lies within 2^-51 (relative) of the exact
    // quotient, inside div_rcp's 2^-49 midpoint margin -> the same float as u0 / ws (12 VALU instead of the
    // two 13-instruction f32 division sequences).  Why the margin suffices (normal quotients): a float rounds
    // differently only if q = u0 / ws lies within 2^-51 of a rounding midpoint m (25 significant bits, odd at that
    // width).  q == m exactly would need u0 = m * ws, an odd 25-bit times a >= 1-bit odd significand in 24 bits:
    // impossible; and q != m gives |q - m| = |u0 - m ws| / |ws| >= 2^-49 |q| (u0 - m ws is a nonzero multiple of
    // the product's last bit).  Covered by the argument, not exhaustively checked: subnormal quotients (|u0|
    // below ~1e-38 |ws|; the geometry's u0 are pixel-scale or exactly 0, and 0 * rws keeps IEEE's sign) and
    // ws = +-inf (handled explicitly above).  |ws| >= 1e-6 by the clamp, so rws never overflows.  Randomized host
    // check, tools/verify_div_rcp_ws.c: 3e8 samples (|ws| 1e-6..1e6, |u0| 1e-45..3e38, subnormal and overflowing
    // quotients included, rcp start emulated with up to 2^-20 error): 0 mismatches against u0 / ws.
    const double wd = (double)ws;
    double rws = __builtin_amdgcn_rcp(wd);
    rws = __builtin_fma(rws, __builtin_fma(-wd, rws, 1.0), rws);
    rws = __builtin_fma(rws, __builtin_fma(-wd, rws, 1.0), rws);
    if (__builtin_isinf(ws)) rws = __builtin_copysign(0.0, wd);  // x / inf (the Newton step would give NaN)
    const float u = div_rcp(u0, rws);
    const float v = div_rcp(u1, rws);
    // geometry.py:151-158
    const float fx = u * sx;
    const float fy = v * sy;
    const float gx = div_rcp(fx + 0.5f, g.rWf) * 2.0f - 1.0f;  // ((fx + 0.5) / Wf) * 2 - 1
    const float gy = div_rcp(fy + 0.5f, g.rHf) * 2.0f - 1.0f;
    // grid_sampler_2d (align_corners=False): ix = (gx + 1) * Wf/2 - 0.5 as one FMA
    ix = __builtin_fmaf(gx + 1.0f, g.fWf / 2.0f, -0.5f);
    iy = __builtin_fmaf(gy + 1.0f, g.fHf / 2.0f, -0.5f);
}

// Validity bits of the four taps at (ix, iy): bit0 nw, bit1 ne, bit2 sw, bit3 se.
// Decided in float (immune to int overflow for |ix| >> 2^31; NaN -> invalid).
__device__ __forceinline__ unsigned ixy_valid(float ix, float iy, const Grid &g) {
    const float xw = __builtin_floorf(ix), yn = __builtin_floorf(iy);
    const bool vx0 = (xw >= 0.0f) & (xw < g.fWf);
    const bool vx1 = (xw + 1.0f >= 0.0f) & (xw + 1.0f < g.fWf);
    const bool vy0 = (yn >= 0.0f) & (yn < g.fHf);
    const bool vy1 = (yn + 1.0f >= 0.0f) & (yn + 1.0f < g.fHf);
    return (unsigned)(vx0 & vy0) | ((unsigned)(vx1 & vy0) << 1) | ((unsigned)(vx0 & vy1) << 2) |
           ((unsigned)(vx1 & vy1) << 3);
}

// grid_sampler_2d bilinear taps at (ix, iy) (geometry.py:161).
__device__ __forceinline__ Taps taps_from_ixy(float ix, float iy, const Grid &g) {
    const float xw = __builtin_floorf(ix);
    const float yn = __builtin_floorf(iy);
    const float we = ix - xw, e = 1.0f - we;
    const float n = iy - yn, s = 1.0f - n;
    Taps t;
    t.w[0] = s * e;
    t.w[1] = s * we;
    t.w[2] = n * e;
    t.w[3] = n * we;
    const bool vx0 = (xw >= 0.0f) & (xw < g.fWf);
    const bool vx1 = (xw + 1.0f >= 0.0f) & (xw + 1.0f < g.fWf);
    const bool vy0 = (yn >= 0.0f) & (yn < g.fHf);
    const bool vy1 = (yn + 1.0f >= 0.0f) & (yn + 1.0f < g.fHf);
    t.valid = (unsigned)(vx0 & vy0) | ((unsigned)(vx1 & vy0) << 1) | ((unsigned)(vx0 & vy1) << 2) |
              ((unsigned)(vx1 & vy1) << 3);
    t.x0 = (vx0 | vx1) ? (int)xw : 0;
    t.y0 = (vy0 | vy1) ? (int)yn : 0;
    return t;
}

__device__ __forceinline__ Taps cell_taps(const float h[9], float x, float y, const Grid &g, float sx, float sy) {
    float ix, iy;
    cell_ixy(h, x, y, g, sx, sy, ix, iy);
    return taps_from_ixy(ix, iy, g);
}

// grid_sampler_2d bilinear combine: ((nw*wnw + ne*wne) + sw*wsw) + se*wse,
// contracted exactly as ATen's vectorised CPU kernel does (App. A.3).
__device__ __forceinline__ float bilerp(float vnw, float vne, float vsw, float vse, const float w[4]) {
    return __builtin_fmaf(vse, w[3], __builtin_fmaf(vsw, w[2], __builtin_fmaf(vne, w[1], vnw * w[0])));
}

// torch.max semantics (NaN propagates).
__device__ __forceinline__ float nan_max(float acc, float t) {
    return (t > acc || t != t) ? (acc != acc ? acc : t) : acc;
}

}  // namespace bev
