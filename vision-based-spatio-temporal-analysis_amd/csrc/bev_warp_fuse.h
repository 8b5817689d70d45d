// bev_warp_fuse.h -- internal entry of the unit-pipeline fused warp (bev_warp_fuse.hip),
// called by the bev_ipm_warp_fuse_f32 dispatcher (bev_warp.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bev {

// Whether the unit-pipeline kernel takes this layout: NHWC (channel stride 1),
// C % 64 == 0, 16-B aligned pixels, 32-bit element offsets inside one map.
bool warp_fuse_units_ok(int64_t sN, int64_t sC, int64_t sH, int64_t sW, const float *feats, int C, int Hf, int Wf,
                        int Hb, int Wb);

int warp_fuse_units(const float *feats, int64_t sN, int64_t sH, int64_t sW, const float *Hmat, const float *xs,
                    const float *ys, int B, int V, int C, int Hf, int Wf, float sx, float sy, int Hb, int Wb, int mode,
                    float *out, hipStream_t st);

// Pool knob (BEV_TUNE_WARP_POOL_KB): 0 = automatic, else KiB of LDS image pool.
int warp_fuse_set_pool_kb(int kb);

// Route knob (BEV_TUNE_WARP_UNITS, env BEV_WARP_UNITS): whether the dispatcher uses this kernel.
int warp_fuse_set_units(int on);
bool warp_fuse_units_enabled();

}  // namespace bev
