// bev_geometry.h -- device-side IPM geometry shared by the warp kernels.
//
// Restates, for one BEV cell, the arithmetic the reference performs through
// torch on the CPU (bit-exact):
//   geometry.py:144-149  uvw = H @ [x y 1]^T (MKL AVX-512 3-term dot), w_safe, u, v
//   geometry.py:151-158  feature-space rescale and [-1,1] normalisation
//   geometry.py:161      grid_sampler_2d unnormalise + floor + bilinear weights
// Everything is plain IEEE fp32; FMAs are explicit (__builtin_fmaf) and the
// library is compiled with -ffp-contract=off so no other contraction happens.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bev {

// MKL AVX-512 sgemm 3-term dot: accumulator starts at +0 (App. A.2).
__device__ __forceinline__ float dot3(float a0, float a1, float a2, float b0, float b1, float b2) {
    return __builtin_fmaf(a2, b2, __builtin_fmaf(a1, b1, __builtin_fmaf(a0, b0, 0.0f)));
}

// Bilinear taps of one BEV cell in one feature map.
struct Taps {
    int x0, y0;       // top-left corner (only meaningful for valid taps)
    float w[4];       // nw, ne, sw, se
    unsigned valid;   // bit0 nw, bit1 ne, bit2 sw, bit3 se
};

// h[9] = world->image homography, (x, y) = BEV cell centre on the ground plane.
__device__ __forceinline__ Taps cell_taps(const float h[9], float x, float y, int Hf, int Wf, float sx, float sy) {
    // geometry.py:144-149
    const float u0 = dot3(h[0], h[1], h[2], x, y, 1.0f);
    const float u1 = dot3(h[3], h[4], h[5], x, y, 1.0f);
    const float w = dot3(h[6], h[7], h[8], x, y, 1.0f);
    const float ws = (__builtin_fabsf(w) < 1e-6f) ? 1.0f : w;
    const float u = u0 / ws;
    const float v = u1 / ws;
    // geometry.py:151-158
    const float fx = u * sx;
    const float fy = v * sy;
    const float fWf = (float)Wf, fHf = (float)Hf;
    const float gx = ((fx + 0.5f) / fWf) * 2.0f - 1.0f;
    const float gy = ((fy + 0.5f) / fHf) * 2.0f - 1.0f;
    // grid_sampler_2d (align_corners=False): ix = (gx + 1) * Wf/2 - 0.5 as one FMA
    const float ix = __builtin_fmaf(gx + 1.0f, fWf / 2.0f, -0.5f);
    const float iy = __builtin_fmaf(gy + 1.0f, fHf / 2.0f, -0.5f);
    const float xw = __builtin_floorf(ix);
    const float yn = __builtin_floorf(iy);
    const float we = ix - xw, e = 1.0f - we;
    const float n = iy - yn, s = 1.0f - n;
    Taps t;
    t.w[0] = s * e;
    t.w[1] = s * we;
    t.w[2] = n * e;
    t.w[3] = n * we;
    // validity decided in float (immune to int overflow for |ix| >> 2^31)
    const bool vx0 = (xw >= 0.0f) & (xw < fWf);
    const bool vx1 = (xw + 1.0f >= 0.0f) & (xw + 1.0f < fWf);
    const bool vy0 = (yn >= 0.0f) & (yn < fHf);
    const bool vy1 = (yn + 1.0f >= 0.0f) & (yn + 1.0f < fHf);
    t.valid = (unsigned)(vx0 & vy0) | ((unsigned)(vx1 & vy0) << 1) | ((unsigned)(vx0 & vy1) << 2) |
              ((unsigned)(vx1 & vy1) << 3);
    t.x0 = (vx0 | vx1) ? (int)xw : 0;
    t.y0 = (vy0 | vy1) ? (int)yn : 0;
    return t;
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
