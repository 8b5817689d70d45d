/*
 * bev_mi355x.h -- C ABI of the MI355X-native multi-view -> BEV hot path.
 *
 * One shared library, libbev_mi355x.so (built from
 * vision-based-spatio-temporal-analysis_amd/csrc/ for gfx950), exports these
 * entry points.  Plain pointers and sizes only: no torch / HIP types appear in
 * the signatures (`stream` is a hipStream_t passed as void*, NULL = the null
 * stream).  All tensor pointers are DEVICE pointers unless the parameter says
 * "host".  Memory is caller-owned; no entry point allocates, frees or
 * synchronises, so every call is stream-ordered and hipGraph-capturable.
 * Return value: 0 on success, otherwise a hipError_t (as int) or
 * BEV_ERR_ARGS (-1) for an argument the kernel cannot take.
 *
 * Each function cites the reference interface it replaces
 * (sea-sky-web/Vision-based-Spatio-Temporal-Analysis @ 2025-11-14, paths
 * relative to project/).  The reference is pure Python/torch, so "replaces"
 * means: the torch op sequence at that file:line, which its modules call on
 * the hot path.  INTEGRATION.md shows the ctypes binding a maintainer adds.
 */
#ifndef BEV_MI355X_H
#define BEV_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BEV_ERR_ARGS (-1)

/* fusion modes (fusion.py:11-22; AttentionFusion fusion.py:25-36 == MEAN) */
#define BEV_FUSE_SUM 0
#define BEV_FUSE_MEAN 1
#define BEV_FUSE_MAX 2

/* ABI version (bumped on any signature change). */
int bev_abi_version(void);

/* host: provenance -- the first 16 hex digits of sha256 over the library's HIP sources and headers (the
 * Makefile's SRCS then HDRS), fixed at build time; bev_native.source_hash() recomputes it from a source tree. */
const char *bev_build_source_hash(void);

/* host: performance knobs (no effect on results); returns the previous value, or
 * BEV_ERR_ARGS for an unknown knob / out-of-range value.
 * BEV_TUNE_CONV_TILE: 0 = automatic, 1 = 128x128, 2 = 128x64, 3 = 64x128, 4 = 64x64
 *   output tiles for bev_conv2d_f32.
 * BEV_TUNE_WARP_POOL_KB: LDS footprint-image pool per workgroup of the fused warp in KiB, 0 = automatic,
 *   else 1..150 (small pools force one-view batches / direct views in the default kernel and block
 *   decomposition in the per-view LDS-DMA kernel, which uses at least 8).
 * BEV_TUNE_WARP_KERNEL: fused warp kernel for NHWC C % 64 == 0 features:
 *   0 = default (= 2), 1 = register-staged, 2 = per-view LDS-DMA kernel, 3 = DPP-row kernel with batched
 *   footprint staging (SUM / MEAN with a workspace; else 2).
 * BEV_TUNE_WARP_BWD_POOL: LDS image of the warp backward in floats (<= 19968), 0 = 19968.
 * BEV_TUNE_CONV_XCD: 1 (default) = XCD-aware conv block order, 0 = plain.
 * BEV_TUNE_CONV_NBUF: 0 = automatic, 1 / 2 = LDS staging depth of the 128x64 / 64x128 conv tiles.
 * BEV_TUNE_WGRAD_MFMA: conv weight gradient on the MFMA with natural-layout operands copied by LDS-DMA
 *   (2, default), on the MFMA with transposed register staging (1), or the VALU float4 kernel (0).
 * BEV_TUNE_CONV_DMA: NHWC Ci % 32 == 0 convs stage their operands global -> LDS by LDS-DMA on
 *   1 (default) = the 64-column output tiles, 2 = every tile, 0 = none (through registers); same
 *   results bit for bit.
 * BEV_TUNE_CONV_X6_TILE: output tile of the split-bf16 fp32 convs (bev_conv2d_x6_f32 / _dual_x6_f32):
 *   0 = automatic, 1 = 128x128, 2 = 128x64.
 * BEV_TUNE_CONV_X6_KERNEL: 0 (default) / 2 = 32-deep K steps with B fragments read straight from the panel
 *   wherever Ci (and Ci2) % 32 == 0, 1 = the 16-deep-step kernel (both operands through LDS) for every shape.
 *   Same results bit for bit.
 * BEV_TUNE_CONV_H16_KERNEL: autocast fp16 convs: 0 (default) = 64-deep K steps, two steps in flight, where Ci % 64 ==
 *   0 (64-column tiles for Co <= 64), and the 64-pixel-step weight gradient; 1 = the 32-deep-step conv and
 *   32-pixel-step weight gradient always; 2 = as 0 with 128-column tiles always.  Same conv results bit for bit;
 *   weight gradients equal to fp32 tolerance (pixel chunks differ).
 * BEV_TUNE_CONV_PW_SMALL: narrow / tiny-K 1x1 convs (EfficientNet): 0 = the MFMA tiles; 1 = Co in
 *   {16, 24, 32, 40, 48} on a per-pixel VALU kernel (measured slower, kept for A/B); 2 (default) = 1x1 with
 *   Ci in {24, 32, 40, 48} and Co <= 32 on a wave-streaming MFMA kernel (k_pw_mfma, float4 epilogue through
 *   LDS); 3 = every 1x1 with Ci in {24, 32, 40, 48} on it (faster inference); 4 = as 2 with dword stores.
 *   All fp32-tolerance equal.
 * BEV_TUNE_DW_RUN: depthwise convs with <= 256 channels that the LDS tile does not take: 0 = per pixel (k_dwconv),
 *   1 = row runs (k_dwconv_r), 2 = row runs with the 3 x 3 rows' loads issued up front, 3 (default) = 2 for every
 *   width (also where the LDS tile k_dwconv_t ran).  Same y up to the sign of an exact zero; the SE partial count
 *   per bev_dwconv_psum_blocks, which follows the knob.
 * BEV_TUNE_CONV_X6_NT: 1 = non-temporal (streaming) activation loads in the split-arithmetic 1x1 / 3x3 convs with
 *   Co <= 64 tiles, 0 (default) = cached loads.  For the LAST reader of a large tensor: CNNEncoder sets it around its
 *   projection so the feature maps that conv writes stay in the Infinity Cache for the warp.  Same results.
 * BEV_TUNE_STEM3_STAGE: bev_conv2d_stem3_f32 output stores: staged in LDS and written as whole NHWC row runs (1 KiB
 *   per instruction), 64 pixels per wave and pass (1) or 32 (2, default: half the LDS, more resident workgroups);
 *   0 = straight from registers (16 B per lane at a pixel stride).  Same results.
 * BEV_TUNE_WARP_PERSIST: fused warp sum / mean with C == 64, NCHW or rank-chunk-major output and a footprint-box
 *   workspace: 0 (default) = one workgroup per (tile, frame); 1 / 2 = the persistent work-queue kernel with 8 queues
 *   (one per XCD) / one queue (A/B options, measured slower).  Same results.
 * BEV_TUNE_WARP_SPAN: fused warp with a footprint-box workspace: span staging (each box row's tap span only) for
 *   footprints of <= 32 rows -- always where the box does not fit the LDS pool but the spans do, and where it fits
 *   when the spans need at most `value` percent of its pixels (1..100, e.g. 50); 0 (default) = box staging only.
 *   An A/B option: at 50 the fused kernel is ~3 % faster on the 16-camera 4K rig, but the span pass adds 5-8 us to
 *   the box pre-pass, so the geometry stage is unchanged there and slower on the bench rig.  Same results.
 * BEV_TUNE_WARP_TILE_BAND: fused warp (per-tile kernel) tile order inside each XCD's contiguous range: 1 = row-major
 *   tiles, n (2..64) = bands of n tile rows walked column by column, so vertically neighbouring tiles (which share
 *   source pixels) are resident together and share that XCD's L2; 0 (default) = bands of 4 for >= 12 views,
 *   row-major otherwise (measured: 16-camera 4K rig -3.7 %, 7-camera rig +2.2 % with bands of 4).  Same results. */
#define BEV_TUNE_CONV_TILE 1
#define BEV_TUNE_WARP_POOL_KB 2
#define BEV_TUNE_WARP_KERNEL 3
#define BEV_TUNE_WARP_BWD_POOL 5
#define BEV_TUNE_CONV_XCD 6
#define BEV_TUNE_CONV_NBUF 7
#define BEV_TUNE_WGRAD_MFMA 8
#define BEV_TUNE_CONV_DMA 9
#define BEV_TUNE_CONV_X6_TILE 10
#define BEV_TUNE_CONV_X6_KERNEL 11
#define BEV_TUNE_CONV_H16_KERNEL 12
#define BEV_TUNE_CONV_PW_SMALL 13
#define BEV_TUNE_DW_RUN 14
#define BEV_TUNE_CONV_X6_NT 16
#define BEV_TUNE_STEM3_STAGE 17
#define BEV_TUNE_WARP_PERSIST 18
#define BEV_TUNE_WARP_SPAN 19
#define BEV_TUNE_WARP_TILE_BAND 20
int bev_tune(int knob, int value);

/* ---------------------------------------------------------------------------
 * Geometry helpers
 * ------------------------------------------------------------------------- */

/* host: BEV cell-centre axis, bit-identical to torch.linspace on the CPU.
 * Replaces geometry.py:26-27 (torch.linspace(min+0.5res, max-0.5res, n)). */
int bev_linspace_f32(double lo, double hi, int n, float *out_host);

/* device: H[n][3][3] = K[n][3][3] @ G[n][3][3], G = [r1 r2 t], with the
 * reference CPU's rounding (MKL AVX-512 3-term dot).
 * Replaces geometry.py:60-63 (`H = K @ G` inside _compute_homography); the
 * shape-tolerance branches geometry.py:35-59 are resolved by the host into
 * (K, G) before the call. */
int bev_homography_f32(const float *K, const float *G, int n, float *H, void *stream);

/* ---------------------------------------------------------------------------
 * IPM warp (GeometryTransformer, grid_sample branch)
 *
 * feats: N = B*V feature maps of C x Hf x Wf fp32, addressed with element
 *   strides (sN, sC, sH, sW) so NCHW and channels-last (NHWC) both work.
 * Hmat: [N][9] world->image homographies (bev_homography_f32 output).
 * xs [Wb], ys [Hb]: BEV cell-centre axes (bev_linspace_f32 output).
 * sx = (float)(Wf / (double)W_img), sy = (float)(Hf / (double)H_img).
 * ------------------------------------------------------------------------- */

/* Per-view warp: out [N][C][Hb][Wb] contiguous.  Bit-identical to
 * geometry.py:142-162 (grid build + F.grid_sample(bilinear, zeros,
 * align_corners=False) + bev_out[b,v] = sampled) for every (b,v). */
int bev_ipm_warp_f32(const float *feats, int64_t sN, int64_t sC, int64_t sH, int64_t sW, const float *Hmat,
                     const float *xs, const float *ys, int N, int C, int Hf, int Wf, float sx, float sy, int Hb,
                     int Wb, float *out, void *stream);

/* Fused warp + view reduction: out [B][C][Hb][Wb] contiguous, mode one of
 * BEV_FUSE_*.  Bit-identical to SimpleFusion(mode)(GeometryTransformer(...))
 * i.e. geometry.py:120-162 followed by fusion.py:17-22, without materialising
 * the [B,V,C,Hb,Wb] intermediate.  Feature map b*V+v is view v of frame b. */
int bev_ipm_warp_fuse_f32(const float *feats, int64_t sN, int64_t sC, int64_t sH, int64_t sW, const float *Hmat,
                          const float *xs, const float *ys, int B, int V, int C, int Hf, int Wf, float sx, float sy,
                          int Hb, int Wb, int mode, float *out, void *stream);

/* bev_ipm_warp_fuse_f32 with a caller-owned device workspace of at least
 * bev_ipm_warp_fuse_workspace_bytes(B, V, Hb, Wb) bytes (16-B aligned, stream-ordered like the output): the
 * fused kernel's per-(frame, tile, view) footprint boxes are then computed by a separate small launch instead of
 * inside every workgroup (same results, bit for bit).  A null or short workspace = bev_ipm_warp_fuse_f32. */
int64_t bev_ipm_warp_fuse_workspace_bytes(int B, int V, int Hb, int Wb);
int bev_ipm_warp_fuse_ws_f32(const float *feats, int64_t sN, int64_t sC, int64_t sH, int64_t sW, const float *Hmat,
                             const float *xs, const float *ys, int B, int V, int C, int Hf, int Wf, float sx, float sy,
                             int Hb, int Wb, int mode, float *out, void *workspace, int64_t workspace_bytes,
                             void *stream);
/* The footprint-box pre-pass of bev_ipm_warp_fuse_ws_f32 on its own (so it can run on a side stream, e.g. while the
 * encoder runs: it needs only the homographies), and the fused warp that takes the boxes from the workspace instead of
 * recomputing them.  bev_ipm_warp_fuse_pre_f32 requires a prior bev_ipm_warp_fuse_boxes_f32 on the same workspace with
 * the same Hmat / xs / ys / B / V / Hf / Wf / sx / sy / Hb / Wb / mode and tuning knobs, ordered before it (same stream
 * or an event); otherwise it is bev_ipm_warp_fuse_ws_f32.  Same results.  The workspace starts with a 16-B header
 * recording the fit test (LDS pool), V and tile shape the boxes were made for; a fused launch whose own differ (another
 * mode's pool, a changed pool knob) ignores the boxes and derives its footprints itself -- still the same results.
 * Replaces the same reference ops (geometry.py:120-162 + fusion.py:17-22). */
int bev_ipm_warp_fuse_boxes_f32(const float *Hmat, const float *xs, const float *ys, int B, int V, int Hf, int Wf,
                                float sx, float sy, int Hb, int Wb, int mode, void *workspace, int64_t workspace_bytes,
                                void *stream);
int bev_ipm_warp_fuse_pre_f32(const float *feats, int64_t sN, int64_t sC, int64_t sH, int64_t sW, const float *Hmat,
                              const float *xs, const float *ys, int B, int V, int C, int Hf, int Wf, float sx, float sy,
                              int Hb, int Wb, int mode, float *out, void *workspace, int64_t workspace_bytes,
                              void *stream);
/* bev_ipm_warp_fuse_pre_f32 (boxes_ready != 0) or _ws_f32 (boxes_ready == 0) writing the fused map channels-last:
 * out [B][Hb][Wb][C] (a [B][C][Hb][Wb] tensor in torch.channels_last memory format), the layout the reference's next
 * consumer -- the BEV projection / detector convs (model_wrapper.py:72-84) -- reads best, and one a 16 x 16 tile writes
 * as whole 128-B lines (1 KiB per store instruction) instead of 64-B row segments per channel plane.  Same values as the
 * plain call.  Needs the LDS-DMA kernel's layout (NHWC features, C % 64 == 0, ...) and one frame's output < 2 GiB; else
 * BEV_ERR_ARGS.  Replaces geometry.py:120-162 + fusion.py:17-22 (the fused inference path, GeometryTransformer
 * .forward_fused). */
int bev_ipm_warp_fuse_nhwc_f32(const float *feats, int64_t sN, int64_t sC, int64_t sH, int64_t sW, const float *Hmat,
                               const float *xs, const float *ys, int B, int V, int C, int Hf, int Wf, float sx,
                               float sy, int Hb, int Wb, int mode, float *out, void *workspace,
                               int64_t workspace_bytes, int boxes_ready, void *stream);
/* bev_ipm_warp_fuse_pre_f32 (boxes_ready != 0) or _ws_f32 (boxes_ready == 0) writing the fused map in
 * rank-chunk-major row order for the camera-shard exchange: out [ceil(Hb / rows_per_chunk)][B][C][rows_per_chunk][Wb],
 * BEV row r of frame b at chunk r / rows_per_chunk, row r % rows_per_chunk -- the layout reduce_scatter over BEV rows
 * takes as is (bev_dist.reduce_partial_bev), so the partial map is not permuted by a copy.  Rows past Hb in the last
 * chunk are not written.  rows_per_chunk >= Hb is the plain [B][C][Hb][Wb] layout.  Same values as the plain call.
 * Needs the LDS-DMA kernel's layout (NHWC C % 64 == 0 ...) and a whole output < 2 GiB; else BEV_ERR_ARGS.  Replaces
 * geometry.py:120-162 + fusion.py:17-22 per rank, and the partial-map permute of the exchange. */
int bev_ipm_warp_fuse_chunked_f32(const float *feats, int64_t sN, int64_t sC, int64_t sH, int64_t sW,
                                  const float *Hmat, const float *xs, const float *ys, int B, int V, int C, int Hf,
                                  int Wf, float sx, float sy, int Hb, int Wb, int mode, int rows_per_chunk, float *out,
                                  void *workspace, int64_t workspace_bytes, int boxes_ready, void *stream);

/* Bilinear corners for index-exactness checks: x0y0 [N][Hb][Wb][2] int32
 * (0 when both taps of an axis are out of range), wts [N][Hb][Wb][4] (nw, ne,
 * sw, se), valid [N][Hb][Wb] uint8 bitmask (1 nw, 2 ne, 4 sw, 8 se).  The
 * integer indices torch's grid_sampler_2d derives at geometry.py:161. */
int bev_ipm_taps_f32(const float *Hmat, const float *xs, const float *ys, int N, int Hf, int Wf, float sx, float sy,
                     int Hb, int Wb, int32_t *x0y0, float *wts, uint8_t *valid, void *stream);

/* Backward of bev_ipm_warp_f32 w.r.t. feats (the grid is constant: calibration
 * carries no gradient).  gfeats [N][C][Hf][Wf] contiguous is OVERWRITTEN.
 * gout [N][C][Hb][Wb] contiguous.  Float atomics: the summation order, and
 * therefore the last bits, may vary run to run.  Replaces autograd through
 * geometry.py:161 (grid_sampler_2d_backward, input grad only). */
int bev_ipm_warp_bwd_f32(const float *gout, const float *Hmat, const float *xs, const float *ys, int N, int C, int Hf,
                         int Wf, float sx, float sy, int Hb, int Wb, float *gfeats, void *stream);

/* The same with the gradient's element strides (sN, sC, sH, sW): dense NCHW (sW == 1) or dense channels-last
 * NHWC (sC == 1, the layout CNNEncoder hands over); anything else is BEV_ERR_ARGS.  Hf, Wf < 16383. */
int bev_ipm_warp_bwd_ex_f32(const float *gout, const float *Hmat, const float *xs, const float *ys, int N, int C,
                            int Hf, int Wf, float sx, float sy, int Hb, int Wb, float *gfeats, int64_t sN, int64_t sC,
                            int64_t sH, int64_t sW, void *stream);

/* Backward of bev_ipm_warp_fuse_f32 for mode SUM / MEAN: gout [B][C][Hb][Wb],
 * gfeats [B*V][C][Hf][Wf] contiguous, OVERWRITTEN.  Replaces autograd through geometry.py:161 and
 * fusion.py:19-21 (d mean / d x_v = gout / V). */
int bev_ipm_warp_fuse_bwd_f32(const float *gout, const float *Hmat, const float *xs, const float *ys, int B, int V,
                              int C, int Hf, int Wf, float sx, float sy, int Hb, int Wb, int mode, float *gfeats,
                              void *stream);

/* The same with the gradient's element strides (dense NCHW or dense NHWC, as bev_ipm_warp_bwd_ex_f32). */
int bev_ipm_warp_fuse_bwd_ex_f32(const float *gout, const float *Hmat, const float *xs, const float *ys, int B,
                                 int V, int C, int Hf, int Wf, float sx, float sy, int Hb, int Wb, int mode,
                                 float *gfeats, int64_t sN, int64_t sC, int64_t sH, int64_t sW, void *stream);

/* ---------------------------------------------------------------------------
 * View fusion on materialised per-view maps (SimpleFusion / AttentionFusion)
 * x [B][V][M] contiguous -> out [B][M].  Replaces fusion.py:19-22
 * (bev_maps.sum(1) / .mean(1) / .max(1).values; AttentionFusion fusion.py:36).
 * ------------------------------------------------------------------------- */
int bev_view_fuse_f32(const float *x, int B, int V, int64_t M, int mode, float *out, void *stream);

/* Backward of the max fusion (fusion.py:22, autograd of bev_maps.max(dim=1).values): gx [B][V][M] (written in full)
 * = gout [B][M] at the view torch's max(dim) selects -- the first NaN, else the first maximal element (ties to the
 * lowest view) -- and 0 at every other view.  x [B][V][M] are the fused maps of the forward. */
int bev_view_max_bwd_f32(const float *x, const float *gout, int B, int V, int64_t M, float *gx, void *stream);

/* ---------------------------------------------------------------------------
 * Backbone (CNNEncoder, cnn_encoder.py:39-70): convolutions on MFMA.
 *
 * Activations are channels-last (NHWC) fp32.  Weights are packed by
 * bev_conv_pack_weights_f32 into a [Co padded to 128][K padded to 32] panel,
 * K index k = (ky*KW + kx)*Ci + ci (the implicit-GEMM reduction order).
 * y = act( conv(x, w) + bias (+ residual) ),  act by `relu`: 0 none, 1 ReLU,
 * 2 SiLU (x / (1 + exp(-x)); the EfficientNet trunk's pointwise convs).
 * Batch-norm (eval) is folded into (w, bias) by the host.
 * x may instead be NCHW (in_nchw = 1): the stem reads the caller's images
 * [B*V,3,H,W] directly (cnn_encoder.py:66-67 view).
 * ------------------------------------------------------------------------- */

/* Size in floats of the packed weight panel for (Co, Ci, KH, KW). */
int64_t bev_conv_packed_size(int Co, int Ci, int KH, int KW);

/* device: w [Co][Ci][KH][KW] (torch OIHW) -> packed panel (see above). */
int bev_conv_pack_weights_f32(const float *w, int Co, int Ci, int KH, int KW, float *packed, void *stream);

/* device: NHWC (or NCHW input) implicit-GEMM convolution on fp32 MFMA.
 * residual (NHWC, same shape as y) and bias may be NULL. */
int bev_conv2d_f32(const float *x, int in_nchw, int N, int H, int W, int Ci, const float *packed, const float *bias,
                   const float *residual, int Co, int KH, int KW, int stride, int pad, int relu, float *y, int Ho,
                   int Wo, void *stream);

/* device: as bev_conv2d_f32 (NHWC input) with every input channel scaled per image first:
 *   y = act( conv(x * gate[n, ci], w) + bias (+ residual) )
 * gate [N][Ci] -- the SqueezeExcite excitation of an EfficientNet block folded into the
 * projection conv's operand load (timm InvertedResidual: se -> conv_pwl; the product x * gate
 * is rounded to fp32 exactly as the separate `x * gate` of SqueezeExcite.forward).
 * Needs Ci % 32 == 0, or a 1x1 / stride-1 / pad-0 conv with Ci % 4 == 0; 16-B aligned x, gate. */
int bev_conv2d_chscale_f32(const float *x, int N, int H, int W, int Ci, const float *gate, const float *packed,
                           const float *bias, const float *residual, int Co, int KH, int KW, int stride, int pad,
                           int relu, float *y, int Ho, int Wo, void *stream);

/* device: bottleneck tail as ONE GEMM (NHWC, both 1x1):
 *   y = act( x (*) W1  +  x2[:, ::s2, ::s2, :] (*) W2  + bias )
 * x [N][Ho][Wo][Ci] is conv3's input, x2 [N][H2][W2][Ci2] the block input the
 * downsample shortcut reads with stride s2 (Ho = (H2-1)/s2 + 1, same for W).
 * packed = bev_conv_pack_weights_f32 of the concatenated [Co][Ci + Ci2][1][1]
 * weight [W1 | W2] (BN folded), bias = b1 + b2.  Ci, Ci2 % 32 == 0.
 * Replaces timm Bottleneck.forward's conv3 -> bn3 -> (+ downsample(shortcut):
 * conv1x1/stride + BN) -> act3 inside the features_only trunk
 * (cnn_encoder.py:26, 41-42): the shortcut tensor is never materialised. */
int bev_conv2d_dual_f32(const float *x, int N, int Ho, int Wo, int Ci, const float *x2, int H2, int W2, int Ci2,
                        int stride2, const float *packed, const float *bias, int Co, int relu, float *y,
                        void *stream);

/* device: two chained convolutions in ONE launch (NHWC):
 *   h = act(conv(x, W1) + bias)               (KH x KW, stride, pad; Co = 64 or 128 channels)
 *   y = act2(h (*) W2 + bias2 + residual)     (1x1, Co -> Co2, Co2 % 128 == 0)
 * h never leaves the chip: each workgroup holds all Co channels of h for its pixels in LDS and
 * runs the 1x1 GEMM on them.  packed / packed2 = bev_conv_pack_weights_f32 of W1 [Co][Ci][KH][KW]
 * and W2 [Co2][Co][1][1] (BN folded); residual [N][Ho][Wo][Co2] or NULL; Ci % 32 == 0; 16-B aligned
 * x / panels.  Bit-identical to bev_conv2d_f32(x -> h) followed by bev_conv2d_f32(h -> y).
 * Replaces timm Bottleneck.forward's conv2 -> bn2 -> act2 -> conv3 -> bn3 (+ shortcut) -> act3 for
 * the blocks without a downsample, inside the features_only trunk (cnn_encoder.py:26, 41-42). */
int bev_conv2d_chain_f32(const float *x, int N, int H, int W, int Ci, const float *packed, const float *bias, int Co,
                         int KH, int KW, int stride, int pad, int relu, const float *packed2, const float *bias2,
                         int Co2, const float *residual, int relu2, float *y, int Ho, int Wo, void *stream);

/* device: as bev_conv2d_chain_f32 for a bottleneck WITH a downsample shortcut (block 0 of a stage):
 *   h = act(conv(x, W1) + bias)
 *   y = act2( [h | x2[:, ::s2, ::s2, :]] (*) W2 + bias2 )     (1x1 over K2 = Co + Ci2)
 * x2 [N][H2][W2][Ci2] is the block input the 1x1/stride-s2 downsample reads (Ho = (H2-1)/s2 + 1);
 * packed2 = bev_conv_pack_weights_f32 of [W3 | Wds] as [Co2][Co + Ci2][1][1], bias2 = b3 + bds
 * (the bev_conv2d_dual_f32 panel).  Ci2 % 32 == 0, x2 < 4 GiB, 16-B aligned.  Bit-identical to
 * bev_conv2d_f32(x -> h) followed by bev_conv2d_dual_f32(h, x2 -> y).  Replaces timm
 * Bottleneck.forward's conv2 -> bn2 -> act2 -> conv3 -> bn3 (+ downsample(shortcut)) -> act3. */
int bev_conv2d_chain_dual_f32(const float *x, int N, int H, int W, int Ci, const float *packed, const float *bias,
                              int Co, int KH, int KW, int stride, int pad, int relu, const float *x2, int H2, int W2,
                              int Ci2, int stride2, const float *packed2, const float *bias2, int Co2, int relu2,
                              float *y, int Ho, int Wo, void *stream);

/* device: NHWC max-pool (timm ResNet stem: 3x3, stride 2, pad 1). */
int bev_maxpool2d_nhwc_f32(const float *x, int N, int H, int W, int C, int k, int stride, int pad, float *y, int Ho,
                           int Wo, void *stream);

/* device: layout conversions between NCHW and NHWC. */
int bev_nchw_to_nhwc_f32(const float *x, int N, int C, int H, int W, float *y, void *stream);
int bev_nhwc_to_nchw_f32(const float *x, int N, int C, int H, int W, float *y, void *stream);
/* device: NCHW [N][C][H][W] with C <= 4 -> NHWC [N][H][W][4], channels >= C zero (y 16-B aligned): the training
 * stem's input as the float4 operand of its weight gradient (trunk_grad.py ConvBNTrain). */
int bev_nchw_to_nhwc4_f32(const float *x, int N, int C, int H, int W, float *y, void *stream);

/* ---------------------------------------------------------------------------
 * EfficientNet trunk (timm efficientnet_b3 features_only, cnn_encoder.py:26,
 * feature index out_index = 2): the layers that are not GEMMs.  All NHWC fp32,
 * C % 4 == 0, 16-B aligned pointers.
 * ------------------------------------------------------------------------- */

/* Number of per-workgroup SE partial sums per image that bev_dwconv2d_f32
 * writes for an Ho x Wo x C output at `stride` (psum is [N][nb][C]). */
int bev_dwconv_psum_blocks(int Ho, int Wo, int C, int stride);

/* device: depthwise KxK conv (K = 3 or 5; torch groups = C), BN folded:
 *   y[n,oy,ox,c] = act( sum_{ky,kx} x[n, oy*s-pad+ky, ox*s-pad+kx, c] * wt[ky*K+kx][c] + bias[c] )
 * (timm conv_dw -> bn -> SiLU, _efficientnet_blocks.py InvertedResidual /
 * DepthwiseSeparableConv).  wt is tap-major [K*K][C].  act as bev_conv2d_f32.
 * If psum != NULL, also writes the channel sums of y per workgroup
 * (deterministic partials, [N][bev_dwconv_psum_blocks(Ho,Wo,C,stride)][C]) -- the
 * squeeze of the block's SqueezeExcite.  C % 32 == 0 (and C % 8 == 0 for outputs of <= 65536 pixels)
 * at stride 1 or 2 runs an LDS-tiled kernel (8-row output tiles x 32 / 16 / 8 channels per workgroup);
 * every other shape and stride the per-pixel kernel. */
int bev_dwconv2d_f32(const float *x, int N, int H, int W, int C, const float *wt, const float *bias, int K, int stride,
                     int pad, int act, float *y, int Ho, int Wo, float *psum, void *stream);

/* device: an EfficientNet inverted residual's expansion and depthwise conv in one pass (timm InvertedResidual
 * conv_pw -> bn1 -> SiLU -> conv_dw -> bn2 -> SiLU, cnn_encoder.py:26), BN folded:
 *   h[n,iy,ix,c] = SiLU( sum_k x[n,iy,ix,k] * we[c][k] + be[c] )   (0 outside the image: the conv_dw zero padding)
 *   y[n,oy,ox,c] = SiLU( bd[c] + sum_{ky,kx} h[n, oy*s-pad+ky, ox*s-pad+kx, c] * wd[ky*K+kx][c] ),  pad = K / 2
 * and, as bev_dwconv2d_f32's psum, the channel sums of y per workgroup: psum [N][nb][Cm], nb =
 * bev_ir_expand_dw_blocks(Ho, Wo, K, stride).  h is never stored.  x [N][H][W][Ci] NHWC fp32 with Ci in {16, 24, 32,
 * 40, 48}, Cm % 48 == 0, K in {3, 5}, stride in {1, 2}; x, bd, y, psum 16-B aligned. */
int bev_ir_expand_dw_blocks(int Ho, int Wo, int K, int stride);
int bev_ir_expand_dw_f32(const float *x, int N, int H, int W, int Ci, const float *we, const float *be, int Cm,
                         const float *wd, const float *bd, int K, int stride, float *y, int Ho, int Wo, float *psum,
                         void *stream);

/* device: the EfficientNet stem (timm conv_stem -> bn1 -> SiLU, cnn_encoder.py:26: 3x3, stride 2, pad 1, 3 input
 * channels), BN folded, from NCHW images to NHWC:
 *   y[n,oy,ox,c] = act( sum_{ci,ky,kx ascending} x[n, ci, 2 oy - 1 + ky, 2 ox - 1 + kx] * wt[(ci*3+ky)*3+kx][c] + bias[c] )
 * x [N][3][H][W] fp32, wt tap-major [27][Co], Co in {32, 40, 48, 64} (timm B0-B5 stems), y [N][Ho][Wo][Co] 16-B
 * aligned, Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1; act as bev_conv2d_f32.  fp32 FMAs on the vector ALU. */
int bev_conv2d_stem3_f32(const float *x, int N, int H, int W, const float *wt, const float *bias, int Co, int act,
                         float *y, int Ho, int Wo, void *stream);

/* device: depthwise conv weight gradient (training): dW [K*K][C] (tap-major, like wt) =
 * sum over n, output pixels of dz[n][p][c] * x[n][tap t of p][c]; OVERWRITTEN (float atomics inside). */
int bev_dwconv_wgrad_f32(const float *x, int N, int H, int W, int C, const float *dz, int Ho, int Wo, int K, int stride,
                         int pad, float *dW, void *stream);

/* device: SqueezeExcite gate from the dwconv partials (timm SqueezeExcite.forward):
 *   mean = sum(psum[n]) / hw;  r = SiLU(w1 @ mean + b1);  gate[n] = sigmoid(w2 @ r + b2)
 * w1 = conv_reduce.weight [rd][C], w2 = conv_expand.weight [C][rd]. */
int bev_se_gate_f32(const float *psum, int N, int nb, int C, int hw, const float *w1, const float *b1, int rd,
                    const float *w2, const float *b2, float *gate, void *stream);

/* device: in place y[n, p, c] *= gate[n, c] for y [N][P][C] (SE excitation, x * gate). */
int bev_channel_scale_f32(float *y, int N, int64_t P, int C, const float *gate, void *stream);

/* ---------------------------------------------------------------------------
 * Trunk backward (training, BASELINE config 3: train.py:249-255 backpropagates
 * through the timm trunk).  NHWC fp32.  BatchNorm in training uses batch statistics
 * (bev_batchnorm_* below) or, for a BN module in eval(), the folded running statistics.
 * ------------------------------------------------------------------------- */

/* dz = dy * (y > 0): ReLU backward from the saved output.  n % 4 == 0. */
int bev_relu_bwd_f32(const float *dy, const float *y, float *dz, int64_t n, void *stream);

/* out [N][Hd][Wd][C] = 0 except out[n][top + s*oy][left + s*ox][c] = dz[n][oy][ox][c]
 * (zero-inserted, padded gradient: turns a strided conv's dgrad into a stride-1 conv). */
int bev_dilate_nhwc_f32(const float *dz, int N, int Ho, int Wo, int C, int s, int top, int left, int Hd, int Wd,
                        float *out, void *stream);

/* out [N][H][W][C] = residual (or 0 when NULL) + (y [N][Ho][Wo][C] placed at (s*oy, s*ox), zero elsewhere): the input
 * gradient of a 1x1 / stride-s / pad-0 conv from y = dz W (the zero-inserted dgrad without the zeros' work);
 * 256 % (C / 4) == 0, 16-B aligned. */
int bev_place_strided_f32(const float *y, int N, int Ho, int Wo, int C, int s, int H, int W, const float *residual,
                          float *out, void *stream);

/* bev_dilate_nhwc_f32 for elements of elem_bytes 4 (fp32) or 2 (fp16 storage): a copy, any 4-channel quad type. */
int bev_dilate_nhwc_ex(const void *dz, int elem_bytes, int N, int Ho, int Wo, int C, int s, int top, int left, int Hd,
                       int Wd, void *out, void *stream);

/* dW [Co][KH*KW*Ci] (k = (ky*KW + kx)*Ci + ci, OVERWRITTEN) = sum over output pixels of
 * dz[m][co] * im2col(x)[m][k] (conv weight gradient; float atomics across m-splits). */
int bev_conv_wgrad_f32(const float *x, int N, int H, int W, int Ci, const float *dz, int Ho, int Wo, int Co, int KH,
                       int KW, int stride, int pad, float *dW, void *stream);

/* db [C] (OVERWRITTEN) = sum over m of dz[m][c] (bias / BN-shift gradient). */
int bev_colsum_f32(const float *dz, int64_t M, int C, float *db, void *stream);
/* CenterNet penalty-reduced focal heatmap loss of model_wrapper.py:235-247 (BEVNet._heatmap_focal_loss) over n cells:
 * p = clamp(sigmoid(logits), 1e-4, 1 - 1e-4), loss[0] = -(sum_{gt == 1} log p (1-p)^alpha + sum_{gt < 1} log(1-p)
 * p^alpha (1-gt)^beta) / max(#{gt == 1}, 1) (fp32 terms, double sums), inv_norm[0] = 1 / max(#{gt == 1}, 1) for the
 * backward; workspace >= bev_focal_loss_workspace_bytes(n).  Backward: dlogits = -grad_loss[0] * inv_norm[0] *
 * d(terms)/dp * sigmoid', torch's clamp rule (no gradient where sigmoid(x) is outside [1e-4, 1 - 1e-4]). */
/* CenterNet masked L1 losses of model_wrapper.py:109-116 (BEVNet.loss): offset / size [B][2][HW] fp32 (NCHW maps),
 * indices [B][ld] int64 cell ids, mask [B][ld], off_t / size_t [B][ld][2] (the first M slots of rows of ld):
 * out[0] = sum |offset[b][c][idx] - off_t| m / n, out[1] = the same on size / size_t, out[2] = 1 / n,
 * n = sum m + 1e-4 (fp32 terms, double sums).  Backward: d_offset / d_size (zeroed by the caller) += g sign(x) m / n
 * at the gathered cells (torch's abs rule), grad_losses = the two losses' gradients. */
int bev_l1_losses_fwd_f32(const float *offset, const float *size, int B, int64_t HW, const int64_t *indices,
                          const float *mask, const float *off_t, const float *size_t_, int M, int ld, float *out,
                          void *stream);
int bev_l1_losses_bwd_f32(const float *offset, const float *size, int B, int64_t HW, const int64_t *indices,
                          const float *mask, const float *off_t, const float *size_t_, int M, int ld,
                          const float *grad_losses, const float *fwd_out, float *d_offset, float *d_size,
                          void *stream);
/* CenterNet gaussian radius of model_wrapper.py:205-233 per object (BEVNet._gaussian_radius_tensor, as torch's
 * float32 ops compute it on the device): width / height in cells -> radius[i] (int64).  The Python-scalar operands
 * come as torch casts them: f_1mov = (float)(1 - ov), rcp_1pov = 1.0f / (float)(1 + ov), f_4ov = (float)(4 ov),
 * f_m2ov = (float)(-2 ov), f_ovm1 = (float)(ov - 1); ov_zero: the r3 root is +inf (ov == 0). */
int bev_gaussian_radius_f32(const float *width_cells, const float *height_cells, int n, float f_1mov,
                            float rcp_1pov, float f_4ov, float f_m2ov, float f_ovm1, int ov_zero, float min_radius,
                            int64_t *radius, void *stream);
int64_t bev_focal_loss_workspace_bytes(int64_t n);
int bev_focal_loss_fwd_f32(const float *logits, const float *gt, int64_t n, float alpha, float beta, float *loss,
                           float *inv_norm, void *workspace, int64_t workspace_bytes, void *stream);
int bev_focal_loss_bwd_f32(const float *logits, const float *gt, int64_t n, float alpha, float beta,
                           const float *grad_loss, const float *inv_norm, float *dlogits, void *stream);

/* dx [N][H][W][C] (OVERWRITTEN): max-pool backward with ATen's window argmax rule
 * (first maximum in scan order, NaN wins). */
int bev_maxpool2d_bwd_nhwc_f32(const float *x, const float *dy, int N, int H, int W, int C, int k, int stride, int pad,
                               int Ho, int Wo, float *dx, void *stream);

/* The same dx (bit-identical) in two passes for C % 4 == 0, k * k <= 255: each window's argmax tap is found once and
 * kept as a byte in argmax [N][Ho][Wo][C] (uint8 workspace, 4-B aligned), then every input gathers the dy of the
 * windows whose byte names it.  Replaces MaxPool2d's backward of timm's stem pool (cnn_encoder.py:26). */
int bev_maxpool2d_bwd_ws_nhwc_f32(const float *x, const float *dy, int N, int H, int W, int C, int k, int stride,
                                  int pad, int Ho, int Wo, float *dx, uint8_t *argmax, void *stream);

/* Training form of the same pair, split at the forward: the pooled y [N][Ho][Wo][C] (bev_maxpool2d_nhwc_f32's
 * values) together with the window argmax bytes, so the backward needs neither x nor the argmax pass; the backward
 * gathers exactly as bev_maxpool2d_bwd_ws_nhwc_f32 does (bit-identical dx).  C % 4 == 0, k * k <= 255, x / y / dy /
 * dx 16-B aligned, argmax 4-B aligned. */
int bev_maxpool2d_fwd_arg_nhwc_f32(const float *x, int N, int H, int W, int C, int k, int stride, int pad, float *y,
                                   uint8_t *argmax, int Ho, int Wo, void *stream);
int bev_maxpool2d_bwd_arg_nhwc_f32(const uint8_t *argmax, const float *dy, int N, int H, int W, int C, int k,
                                   int stride, int pad, int Ho, int Wo, float *dx, void *stream);

/* ---------------------------------------------------------------------------
 * Mixed precision (train.py:238-247, configs/wildtrack.yaml:45 USE_AMP): the convolutions a training step
 * runs under torch.autocast(float16) -- fp16 operands (round to nearest even, as autocast's casts), fp32
 * accumulation -- on the fp16 matrix cores.  Activations stay fp32 NHWC; NHWC Ci % 32 == 0.
 * ------------------------------------------------------------------------- */

/* host: number of fp16 elements of a packed weight panel ([Co pad 128][K pad 32]). */
int64_t bev_conv_packed_size_h16(int Co, int Ci, int KH, int KW);

/* device: OIHW fp32 weights -> fp16 panel (k = (ky*KW + kx)*Ci + ci), packed [size] uint16 storage. */
int bev_conv_pack_weights_h16(const float *w, int Co, int Ci, int KH, int KW, uint16_t *packed, void *stream);

/* device: y[m][n] (row pitch ldy) = act(sum_k f16(x)[m][k] * packed[n][k] + bias[n] (+ residual[m][n])),
 * fp32 sum, NHWC x [N][H][W][Ci] fp32, stride / pad / dilation as bev_conv2d_nhwc_ex_f32; act 0 none,
 * 1 ReLU, 2 SiLU; bias / residual may be NULL (residual needs ldy == Co).  Replaces nn.Conv2d under autocast
 * (cnn_encoder.py:26 timm trunk, detector.py:16-30 head) forward and input-gradient convolutions. */
int bev_conv2d_h16_f32(const float *x, int N, int H, int W, int Ci, const uint16_t *packed, const float *bias,
                       const float *residual, int Co, int KH, int KW, int stride, int pad, int dilation, int act,
                       float *y, int ldy, int Ho, int Wo, void *stream);

/* host: number of 128-row tiles of the BatchNorm statistics bev_conv2d_h16_bnstats_f32 writes for M output rows. */
int64_t bev_conv_h16_stat_tiles(int64_t M);

/* device: bev_conv2d_h16_f32 (act 0, no residual, ldy == Co; Ci % 64 == 0) that also writes the BatchNorm batch
 * statistics of its output, so the train-mode BN after the conv does not read it back: tile_stats
 * [Co][bev_conv_h16_stat_tiles(M)][2] = per channel and 128-row tile (sum, sum of squared deviations from the tile
 * mean), fp32; combine with bev_batchnorm_finalize_tiles_f32.  Replaces the conv -> BatchNorm2d(train) pair of the
 * timm trunk under autocast (cnn_encoder.py:26, train.py:238-247). */
int bev_conv2d_h16_bnstats_f32(const float *x, int N, int H, int W, int Ci, const uint16_t *packed, const float *bias,
                               int Co, int KH, int KW, int stride, int pad, int dilation, float *y, int Ho, int Wo,
                               float *tile_stats, void *stream);

/* bev_conv2d_h16_f32 / _bnstats_f32 in one entry, with the operand x optionally STORED in fp16 (x_half = 1: uint16
 * storage of _Float16, 8-B aligned, Ci % 64 == 0) -- the values the fp32-operand kernel rounds x to while staging,
 * so the result is bit-identical; tile_stats may be NULL (else act 0, no residual, ldy == Co). */
int bev_conv2d_h16_ex_f32(const void *x, int x_half, int N, int H, int W, int Ci, const uint16_t *packed,
                          const float *bias, const float *residual, int Co, int KH, int KW, int stride, int pad,
                          int dilation, int act, float *y, int ldy, int Ho, int Wo, float *tile_stats, void *stream);

/* Weight gradient of a convolution under autocast(float16): dW[co][(ky*KW + kx)*Ci + ci] =
 * sum over output pixels of f16(dz) * f16(x) with fp32 accumulation (the fp16 matrix cores), dW [Co][KH*KW*Ci]
 * fp32 (zeroed by the call).  x [N,H,W,Ci], dz [N,Ho,Wo,Co] NHWC fp32, Ci % 4 == 0, Co % 4 == 0, 16-B aligned.
 * Replaces the conv weight gradient autograd computes for the reference's autocast branch (train.py:238-247). */
int bev_conv_wgrad_h16_f32(const float *x, int N, int H, int W, int Ci, const float *dz, int Ho, int Wo, int Co,
                           int KH, int KW, int stride, int pad, int dilation, float *dW, void *stream);

/* bev_conv_wgrad_h16_f32 with x and / or dz optionally stored in fp16 (x_half / dz_half = 1; 8-B aligned): the
 * values the fp32-operand kernel rounds them to, so the products are identical. */
int bev_conv_wgrad_h16_ex_f32(const void *x, int x_half, int N, int H, int W, int Ci, const void *dz, int dz_half,
                              int Ho, int Wo, int Co, int KH, int KW, int stride, int pad, int dilation, float *dW,
                              void *stream);

/* ---------------------------------------------------------------------------
 * fp32 convolutions on the bf16 matrix cores (exact three-way operand split; bev_conv_x6.hip)
 * Every fp32 operand v is stored as bf16 h + m + l with v == h + m + l exactly; the six bf16 x bf16 partial
 * products above 2^-27 |a b| are summed in the fp32 accumulator (the dropped three are below fp32 rounding),
 * so the result is an fp32 convolution as accurate as the exact-f32 MFMA kernels of bev_conv2d_f32, at 2.67x
 * their matrix-core rate.  Summation order differs from bev_conv2d_f32: fp32-tolerance equal, not bitwise.
 * ------------------------------------------------------------------------- */

/* host: number of bf16 elements of a split weight panel (MFMA fragment order: [Co pad 128 / 32][K pad 16 / 16]
 * [3 planes][64 lanes][8]). */
int64_t bev_conv_packed_size_x6(int Co, int Ci, int KH, int KW);

/* device: OIHW fp32 weights -> split bf16 panel (k = (ky*KW + kx)*Ci + ci), packed [size] uint16 storage. */
int bev_conv_pack_weights_x6(const float *w, int Co, int Ci, int KH, int KW, uint16_t *packed, void *stream);

/* device: y[m][n] (row pitch ldy) = act(sum_k x[m][k] * w[n][k] + bias[n] (+ residual[m][n])) in fp32 through the
 * split panel; NHWC x [N][H][W][Ci] fp32 with Ci % 16 == 0, 16-B aligned -- or, with x NULL, the operand already
 * split: xs [3][N][H][W][Ci] bf16 planes (h, m, l as bev_split3_f32 / a split output writes them; Ci % 32 == 0);
 * stride / pad / dilation as bev_conv2d_nhwc_ex_f32; act 0 none, 1 ReLU, 2 SiLU; bias / residual may be NULL
 * (residual needs ldy == Co).  Output fp32 y, or, with y NULL, the result split into ys [3][N][Ho][Wo][Co] bf16
 * planes (ldy == Co, Co % 4 == 0) -- the pre-split operand of the next conv.  Replaces the nn.Conv2d (+ folded
 * eval BN) layers of the timm trunk and the lazy 1x1 projection (cnn_encoder.py:26,41-46) -- the contract of
 * bev_conv2d_f32 for NHWC inputs. */
int bev_conv2d_x6_f32(const float *x, const uint16_t *xs, int N, int H, int W, int Ci, const uint16_t *packed,
                      const float *bias, const float *residual, int Co, int KH, int KW, int stride, int pad,
                      int dilation, int act, float *y, uint16_t *ys, int ldy, int Ho, int Wo, void *stream);

/* device: bev_conv2d_chain_f32 (bottleneck conv2 -> conv3 + identity residual in one launch, the conv2 output kept
 * in LDS) in the split arithmetic: packed / packed2 are the split panels of conv2 [Co][Ci][KH][KW] and conv3
 * [Co2][Co][1][1]; NHWC x, Ci % 32 == 0, Co in {64, 128}, Co2 % 64 == 0; residual [N][Ho][Wo][Co2] (or NULL).
 * Exactly one of x / xs: xs = conv2's operand already split ([3][N][H][W][Ci] bf16 planes, as the conv1 launch's
 * split output ys writes them; 16-B aligned) -- staged by LDS-DMA, bit-identical to the fp32 x. */
int bev_conv2d_chain_x6_f32(const float *x, const uint16_t *xs, int N, int H, int W, int Ci,
                            const uint16_t *packed, const float *bias, int Co, int KH, int KW, int stride, int pad,
                            int act, const uint16_t *packed2, const float *bias2, int Co2, const float *residual,
                            int act2, float *y, int Ho, int Wo, void *stream);

/* device: bev_conv2d_chain_dual_f32 (block 0 of a stage: conv2 -> [conv3 | 1x1/s2 downsample of x2] in one launch)
 * in the split arithmetic; packed2 = the split panel of [W3 | Wds] as [Co2][Co + Ci2][1][1]; Co == Ci2 == 64 (the
 * layer1 shape), Ci % 32 == 0, Co2 % 64 == 0.  x / xs as bev_conv2d_chain_x6_f32 (x2 stays fp32). */
int bev_conv2d_chain_dual_x6_f32(const float *x, const uint16_t *xs, int N, int H, int W, int Ci,
                                 const uint16_t *packed, const float *bias, int Co, int KH, int KW, int stride,
                                 int pad, int act, const float *x2, int H2, int W2, int Ci2, int stride2,
                                 const uint16_t *packed2, const float *bias2, int Co2, int act2, float *y, int Ho,
                                 int Wo, void *stream);

/* device: a pre-split chained bottleneck body (bev_conv2d_chain_x6_f32 with xs, identity residual) that also runs
 * the NEXT block's 1x1 conv on the block output it has just computed: y = the block output [N][Ho][Wo][Co2] fp32 as
 * before, and h3 = act3(y (*) W3 + bias3) with packed3 the split panel of [Co3][Co2][1][1], written split (ys3
 * [3][N][Ho][Wo][Co3] bf16, 8-B aligned) or fp32 (y3 [N][Ho][Wo][Co3]) -- exactly one of them.  h3 equals
 * bev_conv2d_x6_f32 over y (same K order); y never makes the HBM round trip the separate 1x1 launch would read it by
 * (timm Bottleneck.conv1 of block k + 1, cnn_encoder.py:26).  Co == 64 (the 128-row tile), Co3 in {64, 128},
 * Co2 % 64 == 0, 16-B aligned operands.  x2 (the dual block-0 form) is reserved: non-NULL returns BEV_ERR_ARGS
 * (its kernel was not repeatable at the bench size). */
int bev_conv2d_chain_next_x6_f32(const uint16_t *xs, int N, int H, int W, int Ci, const uint16_t *packed,
                                 const float *bias, int Co, int KH, int KW, int stride, int pad, int act,
                                 const float *x2, int H2, int W2, int Ci2, int stride2, const uint16_t *packed2,
                                 const float *bias2, int Co2, const float *residual, int act2, float *y, int Ho, int Wo,
                                 const uint16_t *packed3, const float *bias3, int Co3, int act3, float *y3,
                                 uint16_t *ys3, void *stream);

/* device: the ResNet stem (timm conv1: 7x7, stride 2, pad 3, Ci = 3; cnn_encoder.py:26, the first layer of
 * CNNEncoder._encode_single) in the split arithmetic: x NCHW [N][3][H][W] fp32 images, packed = the split panel of
 * the (BN-folded) [Co][3][7][7] weights (bev_conv_pack_weights_x6, 16-B aligned), Co <= 64; y NHWC [N][Ho][Wo][Co]
 * = act(conv + bias), act 0 / 1 (ReLU).  fp32-tolerance equal to the exact-f32 stem of bev_conv2d_f32. */
int bev_conv2d_stem_x6_f32(const float *x, int N, int H, int W, const uint16_t *packed, const float *bias, int Co,
                           int relu, float *y, int Ho, int Wo, void *stream);

/* device: the same stem (Co = 64, ReLU) followed by timm's stem max-pool (3x3, stride 2, pad 1; cnn_encoder.py:26,
 * features_only's maxpool) in one pass: y NHWC [N][Hp][Wp][64], Hp = (Ho - 1) / 2 + 1 (Wp alike), bit-identical to
 * bev_conv2d_stem_x6_f32 + bev_maxpool2d_nhwc_f32 without writing the stem output.  workspace (16-B aligned) holds
 * the tile seams: at least bev_conv2d_stem_pool_x6_workspace(N, H, W) bytes. */
int64_t bev_conv2d_stem_pool_x6_workspace(int N, int H, int W);
int bev_conv2d_stem_pool_x6_f32(const float *x, int N, int H, int W, const uint16_t *packed, const float *bias,
                                int Co, float *y, int Hp, int Wp, void *workspace, int64_t workspace_bytes,
                                void *stream);

/* device: split n fp32 values into planes [3][n] bf16 with x == h + m + l exactly (the operand format of
 * bev_conv2d_x6_f32's xs). */
int bev_split3_f32(const float *x, int64_t n, uint16_t *planes, void *stream);

/* device: bev_conv2d_dual_f32 (bottleneck conv3 + downsample shortcut as one GEMM over K = [x | x2[::s2]]) through
 * the split panel of the concatenated [Co][Ci + Ci2] weights; Ci, Ci2 % 16 == 0; act as above. */
int bev_conv2d_dual_x6_f32(const float *x, int N, int Ho, int Wo, int Ci, const float *x2, int H2, int W2, int Ci2,
                           int stride2, const uint16_t *packed, const float *bias, int Co, int act, float *y,
                           void *stream);

/* ---------------------------------------------------------------------------
 * CenterNet BEV head (BEVDetector, detector.py:16-62): dilated convs, GroupNorm(32) + ReLU
 * ------------------------------------------------------------------------- */

/* device: NHWC conv on fp32 MFMA with an optional per-(image, input channel) affine + ReLU applied
 * to the operand as it is loaded: x' = relu?(x * in_scale[n][ci] + in_shift[n][ci]) for in-range
 * taps (zero padding stays 0) -- the previous layer's GroupNorm + ReLU, never materialised.
 * in_scale / in_shift [N][Ci] (both NULL: plain conv; needs Ci % 32 == 0 otherwise).  dilation
 * >= 1 (Ho = (H + 2 pad - dilation (KH - 1) - 1) / stride + 1); y rows are ldy >= Co floats apart
 * (a channel slice of a wider NHWC buffer).  Replaces nn.Conv2d(..., dilation) of detector.py:16-30
 * followed by GroupNorm + ReLU of the layer before. */
int bev_conv2d_nhwc_ex_f32(const float *x, int N, int H, int W, int Ci, const float *in_scale, const float *in_shift,
                           int in_relu, const float *packed, const float *bias, int Co, int KH, int KW, int stride,
                           int pad, int dilation, int relu, float *y, int ldy, int Ho, int Wo, void *stream);

/* bev_conv_wgrad_f32 for a dilated conv. */
int bev_conv_wgrad_ex_f32(const float *x, int N, int H, int W, int Ci, const float *dz, int Ho, int Wo, int Co, int KH,
                          int KW, int stride, int pad, int dilation, float *dW, void *stream);

/* host: bytes of the workspace bev_groupnorm_fwd_f32 / _bwd_f32 need for x [N][P][C], G groups
 * (-1: unsupported shape -- C % G == 0, (C / G) % 4 == 0, 256 % (C / 4) == 0, C <= 1024). */
int64_t bev_groupnorm_workspace_bytes(int N, int64_t P, int C, int G);

/* device: GroupNorm statistics of x [N][P][C] (NHWC, G groups of C/G channels, biased variance,
 * torch.nn.GroupNorm semantics): mean, rstd [N][G]; and the per-(image, channel) affine of the
 * normalised output, scale = rstd * gamma, shift = beta - mean * scale [N][C]. */
int bev_groupnorm_fwd_f32(const float *x, int N, int64_t P, int C, int G, float eps, const float *gamma,
                          const float *beta, float *mean, float *rstd, float *scale, float *shift, void *workspace,
                          void *stream);

/* device: y = x * scale + shift (+ ReLU), NHWC [N][P][C]; y may alias x. */
int bev_groupnorm_apply_f32(const float *x, int N, int64_t P, int C, const float *scale, const float *shift, int relu,
                            float *y, void *stream);

/* bev_groupnorm_apply_f32 with y stored in fp16 when y_half = 1 (an output read only by fp16-operand convs, which
 * round it to exactly these values). */
int bev_groupnorm_apply_ex_f32(const float *x, int N, int64_t P, int C, const float *scale, const float *shift,
                               int relu, void *y, int y_half, void *stream);

/* device: backward of y = relu?(groupnorm(x)) (the forward's mean, rstd, scale, shift): dx [N][P][C],
 * dgamma, dbeta [C], all OVERWRITTEN. */
int bev_groupnorm_bwd_f32(const float *x, const float *dy, int N, int64_t P, int C, int G, const float *mean,
                          const float *rstd, const float *gamma, const float *scale, const float *shift, int relu,
                          float *dx, float *dgamma, float *dbeta, void *workspace, void *stream);

/* bev_groupnorm_bwd_f32 with dx stored in fp16 when dx_half = 1 (read only by the fp16 dgrad / weight gradient). */
int bev_groupnorm_bwd_ex_f32(const float *x, const float *dy, int N, int64_t P, int C, int G, const float *mean,
                             const float *rstd, const float *gamma, const float *scale, const float *shift, int relu,
                             void *dx, int dx_half, float *dgamma, float *dbeta, void *workspace, void *stream);

/* ---------------------------------------------------------------------------
 * BatchNorm with batch statistics (training the trunk in model.train(), reference train.py:222;
 * torch.nn.BatchNorm2d train-mode semantics) on NHWC activations viewed as rows z [M][C], M = N*H*W.
 * Replaces the train-mode BN of timm's trunk (cnn_encoder.py:26 -> timm ResNet bn1/bn2/bn3).
 * ------------------------------------------------------------------------- */

/* host: workspace bytes for bev_batchnorm_train_fwd_f32 / _bwd_f32 (-1: C % 4 != 0 or M <= 0). */
int64_t bev_batchnorm_workspace_bytes(int64_t M, int C);

/* device: per-channel batch mean, rstd = 1/sqrt(biased var + eps), scale = gamma * rstd, shift = beta - mean *
 * scale [C]; running_mean / running_var (both or neither) <- (1 - momentum) * running + momentum * batch value
 * (unbiased variance M/(M-1)). */
int bev_batchnorm_train_fwd_f32(const float *z, int64_t M, int C, float eps, float momentum, const float *gamma,
                                const float *beta, float *running_mean, float *running_var, float *mean, float *rstd,
                                float *scale, float *shift, void *workspace, void *stream);

/* device: bev_batchnorm_train_fwd_f32's outputs (mean, rstd, scale, shift, running-stat update) from per-tile
 * partials (sum, M2 about the tile mean) [C][ntiles][2] of z [M][C] in tiles of rows_per_tile rows (the last
 * one ragged), combined in double: mean = sum of sums / M, M2 = sum of (M2_k + n_k (mean_k - mean)^2). */
int bev_batchnorm_finalize_tiles_f32(const float *tile_stats, int ntiles, int rows_per_tile, int64_t M, int C,
                                     float eps, float momentum, const float *gamma, const float *beta,
                                     float *running_mean, float *running_var, float *mean, float *rstd, float *scale,
                                     float *shift, void *stream);

/* device: y = act(z * scale + shift (+ residual [M][C])), per channel (product and sum each rounded to fp32);
 * act 0 none, 1 ReLU, 2 SiLU. */
int bev_batchnorm_apply_f32(const float *z, int64_t M, int C, const float *scale, const float *shift,
                            const float *residual, int act, float *y, void *stream);

/* bev_batchnorm_apply_f32 with y stored in fp16 when y_half = 1 (round to nearest even) -- for an output whose only
 * readers round it to fp16 anyway (the autocast convs' operands), so storing it rounded changes no result. */
int bev_batchnorm_apply_ex_f32(const float *z, int64_t M, int C, const float *scale, const float *shift,
                               const float *residual, int act, void *y, int y_half, void *stream);

/* device: bev_batchnorm_apply_f32 with act 1 (ReLU), also writing mask [M * C / 4] bytes: bit u of byte k is
 * (y[4 k + u] > 0) -- the ReLU mask the backward's act 4 reads (1 B per 4 elements) instead of y; 256 % (C / 4) == 0.
 * Replaces the residual-add + ReLU of timm's Bottleneck.forward (conv3 / bn3 + shortcut) in training. */
int bev_batchnorm_apply_mask_f32(const float *z, int64_t M, int C, const float *scale, const float *shift,
                                 const float *residual, float *y, uint8_t *mask, void *stream);

/* device: backward of y = act(batchnorm(z) (+ residual)): act 1 (ReLU) takes its mask from the forward output
 * y, act 4 (ReLU) from the mask bytes of bev_batchnorm_apply_mask_f32 passed as y (bit-identical to act 1), act 3 (ReLU of a layer WITHOUT residual; dres must be NULL, y is not read) recomputes it exactly as
 * z * scale + shift > 0 (apply's rounding), act 2 (SiLU) recomputes u = z * scale + shift; frozen = 1 for running statistics (the mean / variance are
 * constants: dz = gamma * rstd * g).  dz [M][C], dres [M][C] (the gradient reaching the residual; may be NULL),
 * dgamma, dbeta [C], all OVERWRITTEN. */
int bev_batchnorm_bwd_f32(const float *dy, const float *y, const float *z, int64_t M, int C, const float *mean,
                          const float *rstd, const float *gamma, const float *scale, const float *shift, int act,
                          int frozen, float *dz, float *dres, float *dgamma, float *dbeta, void *workspace,
                          void *stream);

/* bev_batchnorm_bwd_f32 with dz stored in fp16 when dz_half = 1 (for a dz read only by fp16-operand kernels). */
int bev_batchnorm_bwd_ex_f32(const float *dy, const float *y, const float *z, int64_t M, int C, const float *mean,
                             const float *rstd, const float *gamma, const float *scale, const float *shift, int act,
                             int frozen, void *dz, int dz_half, float *dres, float *dgamma, float *dbeta,
                             void *workspace, void *stream);

/* host: workspace bytes of bev_channel_sums_f32 (-1: C % 4 != 0 or an empty shape). */
int64_t bev_channel_sums_workspace_bytes(int N, int64_t P, int C);

/* device: per-image channel sums out[n][c] = sum_p x[n][p][c] (* x2[n][p][c] when x2 != NULL), NHWC, double
 * partials (the SqueezeExcite squeeze of timm's SqueezeExcite.forward, and its gate gradient). */
int bev_channel_sums_f32(const float *x, const float *x2, int N, int64_t P, int C, float *out, void *workspace,
                         void *stream);

/* device: y[n][p][c] = x[n][p][c] * a[n][c] (+ b[n][c] when b != NULL), out of place (the SE excitation and
 * its input gradient). */
int bev_channel_affine_f32(const float *x, int N, int64_t P, int C, const float *a, const float *b, float *y,
                           void *stream);

/* ---------------------------------------------------------------------------
 * BEVDetector.decode (detector.py:64-125) on the device: no per-pair host sync.
 * ------------------------------------------------------------------------- */

/* device: heat [B][H][W] (the sigmoid heatmap).  Every cell whose `_nms2d` score
 * v * (v == maxpool3x3(v)) exceeds thresh is appended to its frame's candidate list:
 * cand_idx [B][cap] (cell y*W + x), cand_score [B][cap]; count [B] is OVERWRITTEN with the
 * number of candidates (may exceed cap: then only cap were stored). */
int bev_decode_peaks_f32(const float *heat, int B, int H, int W, float thresh, int cap, int32_t *cand_idx,
                         float *cand_score, int32_t *count, void *stream);

/* device: per frame, candidates sorted by (score desc, cell asc), boxes
 * [cx, cy, w, h] = [x_min + (x + off_x) * res_x, y_min + (y + off_y) * res_y, size_w * res_x,
 * size_h * res_y] (offset, size [B][2][H][W]), greedy centre-distance NMS (kept when every
 * kept centre is >= nms_dist away).  boxes [B][cap][4], scores [B][cap] in keep order,
 * nkept [B] (-1: more candidates than cap or bev_decode_max_candidates(); such frames are
 * finished by bev_decode_nms_large_f32). */
int bev_decode_nms_f32(const int32_t *cand_idx, const float *cand_score, const int32_t *count, int B, int cap,
                       const float *offset, const float *size, int H, int W, float x_min, float y_min, float res_x,
                       float res_y, float nms_dist, float *boxes, float *scores, int32_t *nkept, void *stream);

/* host: the largest candidate count per frame bev_decode_nms_f32 handles (its LDS sort). */
int bev_decode_max_candidates(void);

/* device: the same sort + greedy NMS for frames with more than bev_decode_max_candidates()
 * candidates (count[b] <= cap; other frames are left untouched): keys sorted in global memory
 * (keys [B][P] workspace, P a power of two >= every such count, P >= 2 * max_candidates), the
 * greedy NMS in blocks of 64 candidates -- each block is tested against every centre kept so far
 * in parallel, then resolved in order inside one wave.  Same outputs as bev_decode_nms_f32 would
 * give without its LDS limit, so a reference-valid heatmap never fails (detector.py:71-125 has
 * no candidate limit). */
int bev_decode_nms_large_f32(const int32_t *cand_idx, const float *cand_score, const int32_t *count, int B, int cap,
                             int P, const float *offset, const float *size, int H, int W, float x_min, float y_min,
                             float res_x, float res_y, float nms_dist, uint64_t *keys, float *boxes, float *scores,
                             int32_t *nkept, void *stream);

/* Camera-image ingest (data/transforms.py:12-19 T.ToTensor + T.Normalize, applied per image in
 * data/wildtrack_loader.py:368-374): src [N][H][W][3] uint8 RGB (device) -> out [N][3][H][W]
 * fp32, out = (float(src) / 255 - mean[c]) / std[c] with torch's rounding (bit-exact).
 * mean, std: host float[3]. */
int bev_image_normalize_u8_f32(const uint8_t *src, int N, int H, int W, const float *mean, const float *std,
                               float *out, void *stream);

/* BEVNet head operand (model_wrapper.py:69-75 -- proj bias add, pos-enc concat; the reference's torch.cat of the
 * projection [B,P,Hb,Wb] and pos_enc [2,Hb,Wb]): x [B][Hb][Wb][cp] channels-last = (s + bias, pos, 0...) per cell, s the
 * fused warp-sum of the projected views [B][P][Hb][Wb]; cp >= P + 2 (the head's padded input width), P <= 512.  The
 * backward moves the first P channels of the head-input gradient gx [B][Hb][Wb][cp] back to gs [B][P][Hb][Wb] (the
 * warp-sum's gradient).  Values bit-identical to torch's add + cat / slice + permute. */
int bev_head_operand_f32(const float *s, const float *bias, const float *pos, int B, int P, int Hb, int Wb, int cp,
                         float *x, void *stream);
int bev_head_operand_bwd_f32(const float *gx, int B, int P, int Hb, int Wb, int cp, float *gs, void *stream);
/* The same backward with the BEV projection bias's gradient (the sum of gx[..., :P] over every cell: torch's
 * reduction of the broadcast add's gradient, model_wrapper.py:69-75) from the same pass: per-block fp32 partials
 * (`partials`, bev_head_operand_bwd_bias_partials(B, P, Hb, Wb) floats) added in double into gbias [P].  Needs the
 * 16-B form (Wb % 4 == 0, cp % 4 == 0, 16-B aligned gx / gs). */
int64_t bev_head_operand_bwd_bias_partials(int B, int P, int Hb, int Wb);
int bev_head_operand_bwd_bias_f32(const float *gx, int B, int P, int Hb, int Wb, int cp, float *gs, float *gbias,
                                  float *partials, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* BEV_MI355X_H */
