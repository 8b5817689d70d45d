// bev_tune.h -- internal: performance knobs of the warp (bev_warp.hip) and training (bev_train.hip) kernels, set through
// bev_tune() (bev_conv.hip).  Results never depend on them.
#pragma once

namespace bev {

// knob = BEV_TUNE_WARP_* (include/bev_mi355x.h); returns the previous value or BEV_ERR_ARGS.
int warp_tune(int knob, int value);

// LDS image of the warp backward (bev_warp_bwd.hip) in floats: BEV_TUNE_WARP_BWD_POOL, 0 = the maximum.
constexpr int WARP_BWD_POOL_MAX = 19968;  // 78 KiB: two workgroups per CU (k_warp_bwd_runs holds 256 VGPRs)
int warp_bwd_pool_floats();

// knob = BEV_TUNE_WGRAD_MFMA (bev_train.hip).
int train_tune(int knob, int value);

// BEV_TUNE_CONV_X6_TILE / BEV_TUNE_CONV_X6_KERNEL (bev_conv_x6.hip).
int conv_x6_tune(int knob, int value);

// BEV_TUNE_CONV_H16_KERNEL (bev_conv_h16.hip).
int conv_h16_tune(int value);

// BEV_TUNE_DW_RUN (bev_effnet.hip).
int dw_tune(int value);
int stem3_tune(int value);

}  // namespace bev
