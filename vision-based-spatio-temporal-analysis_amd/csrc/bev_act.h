// bev_act.h -- internal: activation functions shared by the conv / depthwise / BatchNorm kernels.
#pragma once
#include <hip/hip_runtime.h>

// SiLU t * sigmoid(t) on the hardware exp2 / reciprocal (v_exp_f32, v_rcp_f32): a few ulp from torch's
// x / (1 + exp(-x)) (relative error <= ~1e-6 for |t| < 100), at ~5 VALU instead of libm expf + an IEEE division
// (~30): the SiLU epilogues of the EfficientNet trunk are a large share of its memory-bound layers' issue time.
__device__ __forceinline__ float silu_hw(float t) {
    return t * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(t * -1.4426950408889634f));
}
__device__ __forceinline__ float sigmoid_hw(float t) {
    return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(t * -1.4426950408889634f));
}
