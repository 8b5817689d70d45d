"""ctypes binding of libbev_mi355x.so (include/bev_mi355x.h) for torch tensors.

This is the only door from the Python module surface (models/) to the HIP
kernels.  There is NO CPU or PyTorch fallback: if the library is missing or a
tensor is not on a ROCm device, the call raises.  torch is imported before the
library is loaded so its HIP runtime (soname libamdhip64.so.7) is the one the
kernels bind to -- one runtime, one set of streams.
"""
from __future__ import annotations

import collections.abc
import contextlib
import ctypes
import functools
import os
import subprocess
import threading

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libbev_mi355x.so")
ABI_VERSION = 12
BEV_ERR_ARGS = -1  # include/bev_mi355x.h: an argument the kernel cannot take

FUSE_MODES = {"sum": 0, "mean": 1, "max": 2}

_lib = None

_vp = ctypes.c_void_p
_i = ctypes.c_int
_i64 = ctypes.c_int64
_f = ctypes.c_float
_d = ctypes.c_double

# name -> (restype, argtypes); must match include/bev_mi355x.h
SIGNATURES = {
    "bev_abi_version": (_i, []),
    "bev_batchnorm_apply_mask_f32": (_i, [_vp, _i64, _i, _vp, _vp, _vp, _vp, _vp, _vp]),
    "bev_place_strided_f32": (_i, [_vp, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp]),
    "bev_conv2d_stem_x6_f32": (_i, [_vp, _i, _i, _i, _vp, _vp, _i, _i, _vp, _i, _i, _vp]),
    "bev_conv2d_stem_pool_x6_workspace": (_i64, [_i, _i, _i]),
    "bev_conv2d_stem_pool_x6_f32": (_i, [_vp, _i, _i, _i, _vp, _vp, _i, _vp, _i, _i, _vp, _i64, _vp]),
    "bev_build_source_hash": (ctypes.c_char_p, []),
    "bev_tune": (_i, [_i, _i]),
    "bev_linspace_f32": (_i, [_d, _d, _i, _vp]),
    "bev_homography_f32": (_i, [_vp, _vp, _i, _vp, _vp]),
    "bev_ipm_warp_f32": (_i, [_vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _i, _i, _i, _i, _f, _f, _i, _i, _vp, _vp]),
    "bev_ipm_warp_fuse_f32": (_i, [_vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _i, _i, _i, _i, _i, _f, _f, _i, _i,
                                   _i, _vp, _vp]),
    "bev_ipm_warp_fuse_workspace_bytes": (_i64, [_i, _i, _i, _i]),
    "bev_ipm_warp_fuse_ws_f32": (_i, [_vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _i, _i, _i, _i, _i, _f, _f, _i, _i,
                                      _i, _vp, _vp, _i64, _vp]),
    "bev_ipm_warp_fuse_pre_f32": (_i, [_vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _i, _i, _i, _i, _i, _f, _f, _i, _i,
                                      _i, _vp, _vp, _i64, _vp]),
    "bev_ipm_warp_fuse_boxes_f32": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _f, _f, _i, _i, _i, _vp, _i64, _vp]),
    "bev_head_operand_f32": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _vp, _vp]),
    "bev_head_operand_bwd_f32": (_i, [_vp, _i, _i, _i, _i, _i, _vp, _vp]),
    "bev_head_operand_bwd_bias_partials": (_i64, [_i, _i, _i, _i]),
    "bev_head_operand_bwd_bias_f32": (_i, [_vp, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp]),
    "bev_l1_losses_fwd_f32": (_i, [_vp, _vp, _i, _i64, _vp, _vp, _vp, _vp, _i, _i, _vp, _vp]),
    "bev_l1_losses_bwd_f32": (_i, [_vp, _vp, _i, _i64, _vp, _vp, _vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp]),
    "bev_gaussian_radius_f32": (_i, [_vp, _vp, _i, _f, _f, _f, _f, _f, _i, _f, _vp, _vp]),
    "bev_focal_loss_workspace_bytes": (_i64, [_i64]),
    "bev_focal_loss_fwd_f32": (_i, [_vp, _vp, _i64, _f, _f, _vp, _vp, _vp, _i64, _vp]),
    "bev_focal_loss_bwd_f32": (_i, [_vp, _vp, _i64, _f, _f, _vp, _vp, _vp, _vp]),
    "bev_ipm_warp_fuse_nhwc_f32": (_i, [_vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _i, _i, _i, _i, _i, _f, _f, _i,
                                        _i, _i, _vp, _vp, _i64, _i, _vp]),
    "bev_ipm_warp_fuse_chunked_f32": (_i, [_vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _i, _i, _i, _i, _i, _f, _f, _i,
                                           _i, _i, _i, _vp, _vp, _i64, _i, _vp]),
    "bev_ipm_taps_f32": (_i, [_vp, _vp, _vp, _i, _i, _i, _f, _f, _i, _i, _vp, _vp, _vp, _vp]),
    "bev_ipm_warp_bwd_f32": (_i, [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _f, _f, _i, _i, _vp, _vp]),
    "bev_ipm_warp_bwd_ex_f32": (_i, [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _f, _f, _i, _i, _vp, _i64, _i64, _i64, _i64,
                                     _vp]),
    "bev_ipm_warp_fuse_bwd_f32": (_i, [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _f, _f, _i, _i, _i, _vp, _vp]),
    "bev_ipm_warp_fuse_bwd_ex_f32": (_i, [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _f, _f, _i, _i, _i, _vp, _i64, _i64,
                                          _i64, _i64, _vp]),
    "bev_view_fuse_f32": (_i, [_vp, _i, _i, _i64, _i, _vp, _vp]),
    "bev_view_max_bwd_f32": (_i, [_vp, _vp, _i, _i, _i64, _vp, _vp]),
    "bev_conv_packed_size": (_i64, [_i, _i, _i, _i]),
    "bev_conv_pack_weights_f32": (_i, [_vp, _i, _i, _i, _i, _vp, _vp]),
    "bev_conv2d_f32": (_i, [_vp, _i, _i, _i, _i, _i, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _i, _i, _vp]),
    "bev_conv2d_chscale_f32": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _i, _i,
                                    _vp]),
    "bev_relu_bwd_f32": (_i, [_vp, _vp, _vp, _i64, _vp]),
    "bev_dilate_nhwc_f32": (_i, [_vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp]),
    "bev_conv_wgrad_f32": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _i, _i, _i, _i, _i, _i, _vp, _vp]),
    "bev_colsum_f32": (_i, [_vp, _i64, _i, _vp, _vp]),
    "bev_maxpool2d_bwd_nhwc_f32": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp]),
    "bev_maxpool2d_bwd_ws_nhwc_f32": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp]),
    "bev_maxpool2d_fwd_arg_nhwc_f32": (_i, [_vp, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _i, _i, _vp]),
    "bev_maxpool2d_bwd_arg_nhwc_f32": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp]),
    "bev_conv2d_dual_f32": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _i, _i, _i, _vp, _vp, _i, _i, _vp, _vp]),
    "bev_conv2d_chain_f32": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _vp, _i, _vp, _i, _vp,
                                  _i, _i, _vp]),
    "bev_conv2d_chain_dual_f32": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _i, _i, _i, _i,
                                       _vp, _vp, _i, _i, _vp, _i, _i, _vp]),
    "bev_maxpool2d_nhwc_f32": (_i, [_vp, _i, _i, _i, _i, _i, _i, _i, _vp, _i, _i, _vp]),
    "bev_nchw_to_nhwc_f32": (_i, [_vp, _i, _i, _i, _i, _vp, _vp]),
    "bev_nchw_to_nhwc4_f32": (_i, [_vp, _i, _i, _i, _i, _vp, _vp]),
    "bev_nhwc_to_nchw_f32": (_i, [_vp, _i, _i, _i, _i, _vp, _vp]),
    "bev_dwconv_psum_blocks": (_i, [_i, _i, _i, _i]),
    "bev_dwconv2d_f32": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _i, _i, _i, _i, _vp, _i, _i, _vp, _vp]),
    "bev_se_gate_f32": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _vp]),
    "bev_conv2d_stem3_f32": (_i, [_vp, _i, _i, _i, _vp, _vp, _i, _i, _vp, _i, _i, _vp]),
    "bev_ir_expand_dw_blocks": (_i, [_i, _i, _i, _i]),
    "bev_ir_expand_dw_f32": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _i, _i, _vp, _i, _i, _vp, _vp]),
    "bev_channel_scale_f32": (_i, [_vp, _i, _i64, _i, _vp, _vp]),
    "bev_decode_peaks_f32": (_i, [_vp, _i, _i, _i, _f, _i, _vp, _vp, _vp, _vp]),
    "bev_decode_nms_f32": (_i, [_vp, _vp, _vp, _i, _i, _vp, _vp, _i, _i, _f, _f, _f, _f, _f, _vp, _vp, _vp, _vp]),
    "bev_decode_max_candidates": (_i, []),
    "bev_decode_nms_large_f32": (_i, [_vp, _vp, _vp, _i, _i, _i, _vp, _vp, _i, _i, _f, _f, _f, _f, _f, _vp, _vp, _vp,
                                      _vp, _vp]),
    "bev_conv2d_nhwc_ex_f32": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _vp, _i,
                                    _i, _i, _vp]),
    "bev_conv_wgrad_ex_f32": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp]),
    "bev_groupnorm_workspace_bytes": (_i64, [_i, _i64, _i, _i]),
    "bev_batchnorm_workspace_bytes": (_i64, [_i64, _i]),
    "bev_batchnorm_train_fwd_f32": (_i, [_vp, _i64, _i, _f, _f, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "bev_batchnorm_apply_f32": (_i, [_vp, _i64, _i, _vp, _vp, _vp, _i, _vp, _vp]),
    "bev_batchnorm_bwd_f32": (_i, [_vp, _vp, _vp, _i64, _i, _vp, _vp, _vp, _vp, _vp, _i, _i, _vp, _vp, _vp, _vp,
                                   _vp, _vp]),
    "bev_channel_sums_workspace_bytes": (_i64, [_i, _i64, _i]),
    "bev_channel_sums_f32": (_i, [_vp, _vp, _i, _i64, _i, _vp, _vp, _vp]),
    "bev_channel_affine_f32": (_i, [_vp, _i, _i64, _i, _vp, _vp, _vp, _vp]),
    "bev_dwconv_wgrad_f32": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _i, _i, _i, _i, _vp, _vp]),
    "bev_groupnorm_fwd_f32": (_i, [_vp, _i, _i64, _i, _i, _f, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "bev_groupnorm_apply_f32": (_i, [_vp, _i, _i64, _i, _vp, _vp, _i, _vp, _vp]),
    "bev_image_normalize_u8_f32": (_i, [_vp, _i, _i, _i, _vp, _vp, _vp, _vp]),
    "bev_groupnorm_bwd_f32": (_i, [_vp, _vp, _i, _i64, _i, _i, _vp, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp]),
    "bev_conv_packed_size_h16": (_i64, [_i, _i, _i, _i]),
    "bev_conv_pack_weights_h16": (_i, [_vp, _i, _i, _i, _i, _vp, _vp]),
    "bev_conv2d_h16_f32": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _vp, _i, _i, _i, _vp]),
    "bev_conv_wgrad_h16_f32": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp]),
    "bev_conv_h16_stat_tiles": (_i64, [_i64]),
    "bev_conv2d_h16_ex_f32": (_i, [_vp, _i, _i, _i, _i, _i, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _vp, _i, _i, _i,
                                   _vp, _vp]),
    "bev_conv_wgrad_h16_ex_f32": (_i, [_vp, _i, _i, _i, _i, _i, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp]),
    "bev_batchnorm_apply_ex_f32": (_i, [_vp, _i64, _i, _vp, _vp, _vp, _i, _vp, _i, _vp]),
    "bev_batchnorm_bwd_ex_f32": (_i, [_vp, _vp, _vp, _i64, _i, _vp, _vp, _vp, _vp, _vp, _i, _i, _vp, _i, _vp, _vp, _vp,
                                      _vp, _vp]),
    "bev_dilate_nhwc_ex": (_i, [_vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp]),
    "bev_groupnorm_apply_ex_f32": (_i, [_vp, _i, _i64, _i, _vp, _vp, _i, _vp, _i, _vp]),
    "bev_groupnorm_bwd_ex_f32": (_i, [_vp, _vp, _i, _i64, _i, _i, _vp, _vp, _vp, _vp, _vp, _i, _vp, _i, _vp, _vp, _vp,
                                      _vp]),
    "bev_conv2d_h16_bnstats_f32": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _i, _i, _vp, _vp]),
    "bev_batchnorm_finalize_tiles_f32": (_i, [_vp, _i, _i, _i64, _i, _f, _f, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                               _vp]),
    "bev_conv_packed_size_x6": (_i64, [_i, _i, _i, _i]),
    "bev_conv_pack_weights_x6": (_i, [_vp, _i, _i, _i, _i, _vp, _vp]),
    "bev_conv2d_x6_f32": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _i, _i, _i,
                               _vp]),
    "bev_split3_f32": (_i, [_vp, _i64, _vp, _vp]),
    "bev_conv2d_chain_dual_x6_f32": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _i, _i, _i, _i,
                                          _vp, _vp, _i, _i, _vp, _i, _i, _vp]),
    "bev_conv2d_chain_x6_f32": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _vp, _i, _vp, _i,
                                     _vp, _i, _i, _vp]),
    "bev_conv2d_dual_x6_f32": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _i, _i, _i, _vp, _vp, _i, _i, _vp, _vp]),
    "bev_conv2d_chain_next_x6_f32": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _i, _i, _i, _i,
                                          _vp, _vp, _i, _vp, _i, _vp, _i, _i, _vp, _vp, _i, _i, _vp, _vp, _vp]),
}


# ---------------------------------------------------------------------------
# launch timing: HIP events recorded on the launch stream around each kernel
# launch of a class ("conv", "warp_fuse"), so a benchmark can price exactly
# those kernels (bench.py roofline) without a profiler.  Off by default.
# ---------------------------------------------------------------------------
_SPANS = None  # dict name -> list of (start, end) events while recording


def spans_start():
    global _SPANS
    _SPANS = {}


def spans_stop() -> dict:
    """Stop recording; returns name -> list of per-launch durations in ms (synchronises)."""
    global _SPANS
    spans, _SPANS = _SPANS or {}, None
    torch.cuda.synchronize()
    return {k: [a.elapsed_time(b) for a, b in v] for k, v in spans.items()}


@contextlib.contextmanager
def _span(name: str, t: torch.Tensor):
    if _SPANS is None:
        yield
        return
    st = torch.cuda.current_stream(t.device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    yield
    e1.record(st)
    _SPANS.setdefault(name, []).append((e0, e1))


def build(force: bool = False) -> str:
    """Compile libbev_mi355x.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    cmd = ["make", "-s", "-C", HERE] + (["-B"] if force else [])
    subprocess.check_call(cmd)
    return LIB_PATH


def lib():
    """Load the HIP library (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libbev_mi355x.so not built ({LIB_PATH}); run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        v = L.bev_abi_version()
        if v != ABI_VERSION:
            raise ImportError(f"libbev_mi355x.so ABI {v} != expected {ABI_VERSION}; rebuild")
        _lib = L
    return _lib


def source_hash() -> str:
    """sha256 (first 16 hex digits) of the library's sources and headers in the Makefile's order (SRCS, then HDRS):
    the digest the Makefile compiles into bev_build_source_hash()."""
    import hashlib
    mk = open(os.path.join(HERE, "Makefile")).read()
    files = []
    for var in ("SRCS", "HDRS"):
        line = next(l for l in mk.splitlines() if l.startswith(var + " ="))
        files += line.split("=", 1)[1].split()
    h = hashlib.sha256()
    for f in files:
        with open(os.path.join(HERE, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def provenance() -> dict:
    """Which sources the loaded library was built from, and whether they are the sources in this tree."""
    built = lib().bev_build_source_hash().decode()
    try:
        tree = source_hash()
    except OSError:
        tree = None
    return {"lib": LIB_PATH, "lib_source_hash": built, "tree_source_hash": tree, "matches_tree": built == tree}


# performance knobs (include/bev_mi355x.h BEV_TUNE_*); results never depend on them
TUNE_CONV_TILE = 1
TUNE_WARP_POOL_KB = 2
TUNE_WARP_KERNEL = 3
TUNE_WARP_BWD_POOL = 5
TUNE_CONV_XCD = 6
TUNE_CONV_NBUF = 7
TUNE_WGRAD_MFMA = 8
TUNE_CONV_DMA = 9
TUNE_CONV_X6_TILE = 10
TUNE_CONV_X6_KERNEL = 11
TUNE_CONV_H16_KERNEL = 12
TUNE_CONV_PW_SMALL = 13
TUNE_DW_RUN = 14
TUNE_CONV_X6_NT = 16
TUNE_STEM3_STAGE = 17
TUNE_WARP_PERSIST = 18
TUNE_WARP_SPAN = 19
TUNE_WARP_TILE_BAND = 20
WARP_KERNEL_DMA, WARP_KERNEL_REGISTER = 0, 1


def tune(knob: int, value: int) -> int:
    """Set a performance knob (include/bev_mi355x.h BEV_TUNE_*); returns the previous value."""
    rc = lib().bev_tune(knob, value)
    if rc < 0:
        raise ValueError(f"bad tuning knob/value {knob}/{value}")
    return rc


@contextlib.contextmanager
def tuned(**knobs):
    """Temporarily set knobs by name: `with tuned(WARP_POOL_KB=8, WARP_KERNEL=2): ...`."""
    old = []
    try:
        for name, value in knobs.items():
            k = globals()["TUNE_" + name]
            old.append((k, tune(k, value)))
        yield
    finally:
        for k, v in reversed(old):
            tune(k, v)


class HipError(RuntimeError):
    pass


# Mixed precision (the reference trains under torch.autocast(float16) + GradScaler, train.py:168-173,238-247):
# every native autograd Function runs its forward with autocast disabled and its floating inputs cast to fp32,
# and its backward in the forward's precision mode -- torch's custom-extension contract (torch.amp.custom_fwd /
# custom_bwd).  What autocast(float16) puts on fp16 in the reference -- its convolutions, forward, input gradient
# and weight gradient -- runs here on fp16 operands with fp32 accumulation too (bev_conv2d_h16_f32 /
# bev_conv_wgrad_h16_f32, the fp16 matrix cores) when AMP_HALF_CONVS is on (default) and the conv has
# Ci % 32 == 0; BatchNorm / GroupNorm / the warp / the loss stay fp32 as under autocast.  AMP_HALF_CONVS = False
# keeps every kernel in fp32 under autocast (wider than the reference).
AMP_HALF_CONVS = True
_AMP_LOCAL = threading.local()


# fp32 arithmetic of the inference trunk convs (ResNet FoldedConv / FoldedTail, the encoder's 1x1 proj):
# "bf16x6" = bev_conv2d_x6_f32 / bev_conv2d_dual_x6_f32 -- every fp32 operand split exactly into three bf16 terms,
# the six partial products above 2^-27 relative on the bf16 matrix cores, fp32 accumulation: an fp32 convolution as
# accurate as the exact-f32 MFMA kernels at 2.67x their matrix-core rate (tests/test_conv_x6_gpu.py measures both
# against float64); "f32" = bev_conv2d_f32 and the chained bottleneck kernels (exact-f32 MFMA, bitwise an fmaf chain).
CONV_ARITHS = ("f32", "bf16x6")
_ARITH = {"mode": "bf16x6"}


def conv_arith() -> str:
    return _ARITH["mode"]


def set_conv_arith(mode: str) -> str:
    """Select the trunk conv arithmetic (CONV_ARITHS); returns the previous mode."""
    if mode not in CONV_ARITHS:
        raise ValueError(f"conv arithmetic {mode!r} not in {CONV_ARITHS}")
    prev, _ARITH["mode"] = _ARITH["mode"], mode
    return prev


@contextlib.contextmanager
def conv_arith_mode(mode: str):
    prev = set_conv_arith(mode)
    try:
        yield
    finally:
        set_conv_arith(prev)


def half_convs() -> bool:
    """True inside the forward / backward of a native Function called under autocast(float16)."""
    return getattr(_AMP_LOCAL, "half", False)


@contextlib.contextmanager
def _half_mode(on: bool):
    prev = half_convs()
    _AMP_LOCAL.half = on
    try:
        yield
    finally:
        _AMP_LOCAL.half = prev


def amp_half_active() -> bool:
    """True where a native Function called now would run its convolutions in the fp16 AMP arithmetic."""
    return bool(torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.float16
                and AMP_HALF_CONVS)


def amp_fwd(fn):
    @functools.wraps(fn)
    def forward(ctx, *args, **kwargs):
        on = (torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.float16
              and AMP_HALF_CONVS)
        ctx._bev_half = on
        with torch.autocast("cuda", enabled=False), _half_mode(on):
            args = [a.float() if isinstance(a, torch.Tensor) and a.is_floating_point() and a.dtype != torch.float32
                    else a for a in args]
            return fn(ctx, *args, **kwargs)
    return forward


def amp_bwd(fn):
    @functools.wraps(fn)
    def backward(ctx, *grads):
        with torch.autocast("cuda", enabled=False), _half_mode(getattr(ctx, "_bev_half", False)):
            return fn(ctx, *[g.float() if isinstance(g, torch.Tensor) and g.is_floating_point() else g
                             for g in grads])
    return backward


def _check(rc: int, name: str):
    if rc != 0:
        if rc == -1:
            raise HipError(f"{name}: invalid arguments (BEV_ERR_ARGS)")
        raise HipError(f"{name}: hipError {rc}")


def _stream(t: torch.Tensor):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _require_gpu(*ts):
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise HipError("libbev_mi355x kernels need ROCm device tensors (got a CPU tensor); "
                           "this package has no CPU fallback")
        if t.dtype != torch.float32:
            raise HipError(f"fp32 tensors expected, got {t.dtype}")


# ---------------------------------------------------------------------------
# geometry
# ---------------------------------------------------------------------------
def linspace(lo: float, hi: float, n: int) -> torch.Tensor:
    out = torch.empty(max(n, 0), dtype=torch.float32)
    _check(lib().bev_linspace_f32(lo, hi, n, _ptr(out)), "bev_linspace_f32")
    return out


def homography(K33: torch.Tensor, G33: torch.Tensor) -> torch.Tensor:
    """K33, G33 [n,3,3] device fp32 -> H [n,9] (bit-identical to the reference CPU matmul)."""
    K33 = K33.contiguous()
    G33 = G33.contiguous()
    _require_gpu(K33, G33)
    n = K33.shape[0]
    H = torch.empty(n, 9, device=K33.device, dtype=torch.float32)
    _check(lib().bev_homography_f32(_ptr(K33), _ptr(G33), n, _ptr(H), _stream(K33)), "bev_homography_f32")
    return H


def _scales(Hf, Wf, img_hw):
    return float(torch.tensor(Wf / float(img_hw[1]), dtype=torch.float32)), \
        float(torch.tensor(Hf / float(img_hw[0]), dtype=torch.float32))


def warp(feats: torch.Tensor, H: torch.Tensor, xs: torch.Tensor, ys: torch.Tensor, img_hw) -> torch.Tensor:
    """feats [N,C,Hf,Wf] (any strides) -> out [N,C,Hb,Wb]."""
    _require_gpu(feats, H, xs, ys)
    N, C, Hf, Wf = feats.shape
    Hb, Wb = ys.numel(), xs.numel()
    sx, sy = _scales(Hf, Wf, img_hw)
    out = torch.empty(N, C, Hb, Wb, device=feats.device, dtype=torch.float32)
    s = feats.stride()
    _check(lib().bev_ipm_warp_f32(_ptr(feats), s[0], s[1], s[2], s[3], _ptr(H), _ptr(xs), _ptr(ys), N, C, Hf, Wf, sx,
                                  sy, Hb, Wb, _ptr(out), _stream(feats)), "bev_ipm_warp_f32")
    return out


def warp_fuse_boxes(H: torch.Tensor, xs, ys, B: int, V: int, Hf: int, Wf: int, img_hw, mode: str) -> torch.Tensor:
    """The fused warp's footprint-box pre-pass alone (bev_ipm_warp_fuse_boxes_f32) into a new workspace, on the
    current stream; pass it to `warp_fuse(..., boxes=)` with the same geometry and mode."""
    _require_gpu(H, xs, ys)
    Hb, Wb = ys.numel(), xs.numel()
    sx, sy = _scales(Hf, Wf, img_hw)
    nws = lib().bev_ipm_warp_fuse_workspace_bytes(B, V, Hb, Wb)
    ws = torch.empty(max(nws, 8), device=H.device, dtype=torch.uint8)
    with _span("warp_boxes", H):
        rc = lib().bev_ipm_warp_fuse_boxes_f32(_ptr(H), _ptr(xs), _ptr(ys), B, V, Hf, Wf, sx, sy, Hb, Wb, FUSE_MODES[mode],
                                               _ptr(ws), nws, _stream(H))
    _check(rc, "bev_ipm_warp_fuse_boxes_f32")
    return ws


def warp_fuse(feats: torch.Tensor, H: torch.Tensor, xs, ys, img_hw, mode: str, out: torch.Tensor = None,
              boxes: torch.Tensor = None, rows_per_chunk: int = None, channels_last: bool = False,
              num_chunks: int = None):
    """feats [B,V,C,Hf,Wf] (any strides within a map; maps b*V+v) -> out [B,C,Hb,Wb].  `boxes`: a workspace filled
    by `warp_fuse_boxes` for this geometry and mode (the pre-pass is then not launched again).
    `rows_per_chunk` (< Hb): the rank-chunk-major layout of bev_ipm_warp_fuse_chunked_f32 instead,
    out [ceil(Hb / rpr), B, C, rpr, Wb] with the rows past Hb zero (the camera-shard reduce-scatter's input), or
    [num_chunks, B, C, rpr, Wb] when `num_chunks` (>= ceil(Hb / rpr), the world size) is given: the chunks past the
    map are all zero.  Layouts the chunk-major kernel does not take (not channels-last, C % 64 != 0, ...) run the
    plain fused launch and one rearranging copy on the device, with the same values.
    `channels_last`: bev_ipm_warp_fuse_nhwc_f32 -- the same [B,C,Hb,Wb] values in torch.channels_last memory format
    (storage [B,Hb,Wb,C]); needs NHWC features with C % 64 == 0 (the LDS-DMA kernel), else HipError."""
    if rows_per_chunk is not None and (rows_per_chunk < ys.numel() or num_chunks):
        return _warp_fuse_chunked(feats, H, xs, ys, img_hw, mode, int(rows_per_chunk), boxes, num_chunks)
    if channels_last:
        return _warp_fuse_nhwc(feats, H, xs, ys, img_hw, mode, out, boxes)
    _require_gpu(feats, H, xs, ys)
    B, V, C, Hf, Wf = feats.shape
    if B * V > 0 and feats.stride(0) != V * feats.stride(1):
        feats = feats.contiguous()
    Hb, Wb = ys.numel(), xs.numel()
    sx, sy = _scales(Hf, Wf, img_hw)
    if out is None:
        out = torch.empty(B, C, Hb, Wb, device=feats.device, dtype=torch.float32)
    s = feats.stride()
    # the per-(frame, tile, view) footprint boxes go to a stream-ordered workspace: for the LDS-DMA kernels (NHWC,
    # C % 64 == 0) a launch of their own BEFORE the timed span, so "warp_fuse" spans time the fused kernel alone
    # (as rocprofv3 lists it); other layouts let the library decide
    nws = lib().bev_ipm_warp_fuse_workspace_bytes(B, V, Hb, Wb)
    if boxes is None and s[2] == 1 and C % 64 == 0 and V <= 64 and Hf < 16384 and Wf < 16384 and B * Hb * Wb > 0:
        boxes = warp_fuse_boxes(H, xs, ys, B, V, Hf, Wf, img_hw, mode)
    if boxes is not None:
        assert boxes.numel() >= nws and boxes.device == feats.device, "boxes workspace for another geometry"
        fn, ws = lib().bev_ipm_warp_fuse_pre_f32, boxes
    else:
        fn, ws = lib().bev_ipm_warp_fuse_ws_f32, torch.empty(max(nws, 8), device=feats.device, dtype=torch.uint8)
    with _span("warp_fuse", feats):
        rc = fn(_ptr(feats), s[1], s[2], s[3], s[4], _ptr(H), _ptr(xs), _ptr(ys), B, V, C, Hf, Wf, sx, sy, Hb, Wb,
                FUSE_MODES[mode], _ptr(out), _ptr(ws), nws, _stream(feats))
    _check(rc, "bev_ipm_warp_fuse")
    return out


def _warp_fuse_nhwc(feats, H, xs, ys, img_hw, mode, out=None, boxes=None):
    _require_gpu(feats, H, xs, ys)
    B, V, C, Hf, Wf = feats.shape
    if B * V > 0 and feats.stride(0) != V * feats.stride(1):
        feats = feats.contiguous()
    Hb, Wb = ys.numel(), xs.numel()
    sx, sy = _scales(Hf, Wf, img_hw)
    if out is None:
        out = torch.empty(B, Hb, Wb, C, device=feats.device, dtype=torch.float32).permute(0, 3, 1, 2)
    assert out.shape == (B, C, Hb, Wb) and out.permute(0, 2, 3, 1).is_contiguous(), "channels-last [B,C,Hb,Wb] out"
    s = feats.stride()
    nws = lib().bev_ipm_warp_fuse_workspace_bytes(B, V, Hb, Wb)
    ready = boxes is not None
    if boxes is None and s[2] == 1 and C % 64 == 0 and V <= 64 and Hf < 16384 and Wf < 16384 and B * Hb * Wb > 0:
        boxes, ready = warp_fuse_boxes(H, xs, ys, B, V, Hf, Wf, img_hw, mode), True
    if boxes is not None:
        assert boxes.numel() >= nws and boxes.device == feats.device, "boxes workspace for another geometry"
    ws = boxes if boxes is not None else torch.empty(max(nws, 8), device=feats.device, dtype=torch.uint8)
    with _span("warp_fuse", feats):
        rc = lib().bev_ipm_warp_fuse_nhwc_f32(_ptr(feats), s[1], s[2], s[3], s[4], _ptr(H), _ptr(xs), _ptr(ys), B, V,
                                              C, Hf, Wf, sx, sy, Hb, Wb, FUSE_MODES[mode], _ptr(out), _ptr(ws), nws,
                                              int(ready), _stream(feats))
    if rc == -1 and boxes is not None:  # a kernel choice without the channels-last store (BEV_TUNE_WARP_KERNEL 1 / a
        # small WARP_POOL_KB, A/B knobs): the NCHW launch, then one layout copy on the device
        out.copy_(warp_fuse(feats, H, xs, ys, img_hw, mode, boxes=boxes if ready else None))
        return out
    _check(rc, "bev_ipm_warp_fuse_nhwc_f32")
    return out


def _warp_fuse_chunked(feats, H, xs, ys, img_hw, mode, rpr, boxes=None, num_chunks=None):
    _require_gpu(feats, H, xs, ys)
    B, V, C, Hf, Wf = feats.shape
    if B * V > 0 and feats.stride(0) != V * feats.stride(1):
        feats = feats.contiguous()
    Hb, Wb = ys.numel(), xs.numel()
    sx, sy = _scales(Hf, Wf, img_hw)
    if rpr <= 0:
        raise ValueError("rows_per_chunk must be positive")
    nmap = -(-Hb // rpr)  # chunks that hold map rows
    nck = nmap if num_chunks is None else int(num_chunks)
    if nck < nmap:
        raise ValueError(f"num_chunks {nck} < ceil(Hb / rows_per_chunk) = {nmap}")
    out = torch.empty(nck, B, C, rpr, Wb, device=feats.device, dtype=torch.float32)
    if nmap * rpr > Hb:
        out[nmap - 1, :, :, Hb - (nmap - 1) * rpr:].zero_()  # padding rows: no cell writes them
    if nck > nmap:
        out[nmap:].zero_()  # whole chunks past the map (a world larger than ceil(Hb / rpr))
    s = feats.stride()
    nws = lib().bev_ipm_warp_fuse_workspace_bytes(B, V, Hb, Wb)
    ready = boxes is not None
    if boxes is None and s[2] == 1 and C % 64 == 0 and V <= 64 and Hf < 16384 and Wf < 16384 and B * Hb * Wb > 0:
        boxes, ready = warp_fuse_boxes(H, xs, ys, B, V, Hf, Wf, img_hw, mode), True
    ws = boxes if boxes is not None else torch.empty(max(nws, 8), device=feats.device, dtype=torch.uint8)
    with _span("warp_fuse", feats):
        rc = lib().bev_ipm_warp_fuse_chunked_f32(_ptr(feats), s[1], s[2], s[3], s[4], _ptr(H), _ptr(xs), _ptr(ys), B,
                                                 V, C, Hf, Wf, sx, sy, Hb, Wb, FUSE_MODES[mode], rpr, _ptr(out),
                                                 _ptr(ws), nws, int(ready), _stream(feats))
    if rc == BEV_ERR_ARGS:
        # a layout the chunk-major LDS-DMA kernel does not take (NCHW or C % 64 != 0 features, V > 64, an A/B knob):
        # the plain fused launch, then its rows copied into chunk order on the device (same values)
        plain = warp_fuse(feats, H, xs, ys, img_hw, mode, boxes=boxes if ready else None)
        padded = torch.zeros(B, C, nmap * rpr, Wb, device=feats.device, dtype=torch.float32)
        padded[:, :, :Hb] = plain
        out[:nmap] = padded.view(B, C, nmap, rpr, Wb).permute(2, 0, 1, 3, 4)
        return out
    _check(rc, "bev_ipm_warp_fuse_chunked_f32")
    return out


def head_operand(s: torch.Tensor, bias: torch.Tensor, pos: torch.Tensor, cp: int) -> torch.Tensor:
    """s [B,P,Hb,Wb] contiguous, bias [P], pos [2,Hb,Wb] -> x [B,Hb,Wb,cp] channels-last (s + bias, pos, zeros)."""
    _require_gpu(s, bias, pos)
    s, bias, pos = s.contiguous(), bias.contiguous().float(), pos.contiguous().float()
    B, P, Hb, Wb = s.shape
    x = torch.empty(B, Hb, Wb, cp, device=s.device, dtype=torch.float32)
    _check(lib().bev_head_operand_f32(_ptr(s), _ptr(bias), _ptr(pos), B, P, Hb, Wb, cp, _ptr(x), _stream(s)),
           "bev_head_operand_f32")
    return x


def head_operand_bwd(gx: torch.Tensor, P: int) -> torch.Tensor:
    """gx [B,Hb,Wb,cp] (channels contiguous) -> gs [B,P,Hb,Wb] = gx[..., :P] in NCHW."""
    _require_gpu(gx)
    gx = gx.contiguous()
    B, Hb, Wb, cp = gx.shape
    gs = torch.empty(B, P, Hb, Wb, device=gx.device, dtype=torch.float32)
    _check(lib().bev_head_operand_bwd_f32(_ptr(gx), B, P, Hb, Wb, cp, _ptr(gs), _stream(gx)),
           "bev_head_operand_bwd_f32")
    return gs


def head_operand_bwd_bias(gx: torch.Tensor, P: int):
    """(gs, gbias): head_operand_bwd's gs and the BEV projection bias's gradient sum(gx[..., :P]) over (b, h, w) from
    the same pass (bev_head_operand_bwd_bias_f32; block partials added in double), or None for gbias when the 16-B
    form does not apply (the caller reduces gs itself)."""
    _require_gpu(gx)
    gx = gx.contiguous()
    B, Hb, Wb, cp = gx.shape
    gs = torch.empty(B, P, Hb, Wb, device=gx.device, dtype=torch.float32)
    if Wb % 4 != 0 or cp % 4 != 0 or gx.data_ptr() % 16 != 0 or B * Hb * Wb == 0:
        _check(lib().bev_head_operand_bwd_f32(_ptr(gx), B, P, Hb, Wb, cp, _ptr(gs), _stream(gx)),
               "bev_head_operand_bwd_f32")
        return gs, None
    n = int(lib().bev_head_operand_bwd_bias_partials(B, P, Hb, Wb))
    _check(min(n, 0), "bev_head_operand_bwd_bias_partials")
    part = torch.empty(n, device=gx.device, dtype=torch.float32)
    gb = torch.empty(P, device=gx.device, dtype=torch.float32)
    _check(lib().bev_head_operand_bwd_bias_f32(_ptr(gx), B, P, Hb, Wb, cp, _ptr(gs), _ptr(gb), _ptr(part),
                                               _stream(gx)), "bev_head_operand_bwd_bias_f32")
    return gs, gb


def taps(H, xs, ys, Hf, Wf, img_hw):
    _require_gpu(H, xs, ys)
    N = H.shape[0]
    Hb, Wb = ys.numel(), xs.numel()
    sx, sy = _scales(Hf, Wf, img_hw)
    dev = H.device
    x0y0 = torch.empty(N, Hb, Wb, 2, device=dev, dtype=torch.int32)
    wts = torch.empty(N, Hb, Wb, 4, device=dev, dtype=torch.float32)
    valid = torch.empty(N, Hb, Wb, device=dev, dtype=torch.uint8)
    _check(lib().bev_ipm_taps_f32(_ptr(H), _ptr(xs), _ptr(ys), N, Hf, Wf, sx, sy, Hb, Wb, _ptr(x0y0), _ptr(wts),
                                  _ptr(valid), _stream(H)), "bev_ipm_taps_f32")
    return x0y0, wts, valid


def _grad_maps(lead, C, Hf, Wf, dev, channels_last):
    """Gradient buffer [*lead, C, Hf, Wf]: dense NCHW, or a channels-last view of [*lead, Hf, Wf, C] storage (the
    layout CNNEncoder hands its features over in, so the gradient needs no transpose on its way back)."""
    if not channels_last:
        return torch.empty(*lead, C, Hf, Wf, device=dev, dtype=torch.float32)
    nl = len(lead)
    buf = torch.empty(*lead, Hf, Wf, C, device=dev, dtype=torch.float32)
    return buf.permute(*range(nl), nl + 2, nl, nl + 1)


def warp_bwd(gout, H, xs, ys, Hf, Wf, img_hw, channels_last=True):
    """d feats of the per-view warp (k_warp_bwd_runs); [N,C,Hf,Wf], channels-last storage by default."""
    gout = gout.contiguous()
    _require_gpu(gout, H, xs, ys)
    N, C, Hb, Wb = gout.shape
    sx, sy = _scales(Hf, Wf, img_hw)
    g = _grad_maps((N,), C, Hf, Wf, gout.device, channels_last)
    s = g.stride()
    with _span("warp_bwd", gout):
        rc = lib().bev_ipm_warp_bwd_ex_f32(_ptr(gout), _ptr(H), _ptr(xs), _ptr(ys), N, C, Hf, Wf, sx, sy, Hb, Wb,
                                           _ptr(g), s[0], s[1], s[2], s[3], _stream(gout))
    _check(rc, "bev_ipm_warp_bwd_ex_f32")
    return g


def warp_fuse_bwd(gout, H, xs, ys, V, Hf, Wf, img_hw, mode, channels_last=True):
    """d feats of the fused warp + sum / mean (k_warp_bwd_runs); [B,V,C,Hf,Wf], channels-last storage by
    default."""
    gout = gout.contiguous()
    _require_gpu(gout, H, xs, ys)
    B, C, Hb, Wb = gout.shape
    sx, sy = _scales(Hf, Wf, img_hw)
    g = _grad_maps((B, V), C, Hf, Wf, gout.device, channels_last)
    s = g.stride()
    with _span("warp_bwd", gout):
        rc = lib().bev_ipm_warp_fuse_bwd_ex_f32(_ptr(gout), _ptr(H), _ptr(xs), _ptr(ys), B, V, C, Hf, Wf, sx, sy, Hb,
                                                Wb, FUSE_MODES[mode], _ptr(g), s[1], s[2], s[3], s[4], _stream(gout))
    _check(rc, "bev_ipm_warp_fuse_bwd_ex_f32")
    return g


def view_fuse(x: torch.Tensor, mode: str) -> torch.Tensor:
    """x [B,V,...] -> [B,...] (SimpleFusion)."""
    x = x.contiguous()
    _require_gpu(x)
    B, V = x.shape[:2]
    M = x[0, 0].numel() if B * V > 0 else 0
    out = torch.empty((B,) + tuple(x.shape[2:]), device=x.device, dtype=torch.float32)
    _check(lib().bev_view_fuse_f32(_ptr(x), B, V, M, FUSE_MODES[mode], _ptr(out), _stream(x)), "bev_view_fuse_f32")
    return out


def view_max_bwd(x: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
    """Gradient of the max over dim 1 of x [B,V,...] for the upstream gradient g [B,...] (torch's index rule)."""
    x = x.contiguous()
    g = g.contiguous().float()
    _require_gpu(x, g)
    B, V = x.shape[:2]
    M = x[0, 0].numel() if B * V > 0 else 0
    gx = torch.empty_like(x, dtype=torch.float32)
    _check(lib().bev_view_max_bwd_f32(_ptr(x), _ptr(g), B, V, M, _ptr(gx), _stream(x)), "bev_view_max_bwd_f32")
    return gx


# ---------------------------------------------------------------------------
# backbone
# ---------------------------------------------------------------------------
def pack_conv_weight(w: torch.Tensor) -> torch.Tensor:
    """OIHW fp32 (device) -> packed MFMA panel: fp32, or fp16 (torch.float16 storage) inside a native Function
    run under autocast(float16) when the conv takes the fp16 kernel (Ci % 32 == 0) -- the conv calls below
    dispatch on the panel's dtype."""
    w = w.detach().contiguous()
    _require_gpu(w)
    Co, Ci, KH, KW = w.shape
    if half_convs() and Ci % 32 == 0:
        n = lib().bev_conv_packed_size_h16(Co, Ci, KH, KW)
        out = torch.empty(n, device=w.device, dtype=torch.float16)
        _check(lib().bev_conv_pack_weights_h16(_ptr(w), Co, Ci, KH, KW, _ptr(out), _stream(w)),
               "bev_conv_pack_weights_h16")
        return out
    n = lib().bev_conv_packed_size(Co, Ci, KH, KW)
    out = torch.empty(n, device=w.device, dtype=torch.float32)
    _check(lib().bev_conv_pack_weights_f32(_ptr(w), Co, Ci, KH, KW, _ptr(out), _stream(w)), "bev_conv_pack_weights_f32")
    return out


def pack_conv_weight_x6(w: torch.Tensor) -> torch.Tensor:
    """OIHW fp32 (device) -> split-bf16 panel (torch.bfloat16 storage) of bev_conv2d_x6_f32 / _dual_x6_f32; the
    conv calls below dispatch on the panel's dtype."""
    w = w.detach().contiguous().float()
    _require_gpu(w)
    Co, Ci, KH, KW = w.shape
    n = lib().bev_conv_packed_size_x6(Co, Ci, KH, KW)
    out = torch.empty(n, device=w.device, dtype=torch.bfloat16)
    _check(lib().bev_conv_pack_weights_x6(_ptr(w), Co, Ci, KH, KW, _ptr(out), _stream(w)), "bev_conv_pack_weights_x6")
    return out


class Split3:
    """An fp32 NHWC activation held split into three bf16 planes (planes [3, N, H, W, C] bf16, x == h + m + l
    exactly): the pre-split operand format of bev_conv2d_x6_f32 (xs / ys)."""

    def __init__(self, planes: torch.Tensor):
        assert planes.dtype == torch.bfloat16 and planes.dim() == 5 and planes.shape[0] == 3
        self.planes = planes

    @property
    def shape(self):
        return tuple(self.planes.shape[1:])

    @property
    def device(self):
        return self.planes.device

    def to_float(self) -> torch.Tensor:
        p = self.planes.float()
        return (p[0] + p[1]) + p[2]


def split3(x: torch.Tensor) -> Split3:
    """fp32 tensor [N, H, W, C] -> Split3 (bev_split3_f32)."""
    x = x.contiguous()
    _require_gpu(x)
    out = torch.empty((3,) + tuple(x.shape), device=x.device, dtype=torch.bfloat16)
    _check(lib().bev_split3_f32(_ptr(x), x.numel(), _ptr(out), _stream(x)), "bev_split3_f32")
    return Split3(out)


def conv2d_nhwc_x6(x, packed: torch.Tensor, bias, Co: int, KH: int, KW: int, stride: int, pad: int,
                   dilation: int = 1, act: int = 0, residual: torch.Tensor = None, out: torch.Tensor = None,
                   split_out: bool = False):
    """fp32 conv through the split-bf16 panel (bev_conv2d_x6_f32): x [N,H,W,Ci] fp32 NHWC (Ci % 16 == 0) or a
    Split3 (Ci % 32 == 0) -> y [N,Ho,Wo,Co] fp32 (or the first Co channels of a wider NHWC `out`), or a Split3
    with split_out."""
    xs = x if isinstance(x, Split3) else None
    if xs is None:
        x = x.contiguous()
        _require_gpu(x)
    _require_gpu(bias, residual)
    if not packed.is_cuda or packed.dtype != torch.bfloat16:
        raise HipError("conv2d_nhwc_x6 needs the split-bf16 weight panel on the device")
    N, H, W, Ci = x.shape
    dev = x.device
    Ho, Wo = (H + 2 * pad - dilation * (KH - 1) - 1) // stride + 1, (W + 2 * pad - dilation * (KW - 1) - 1) // stride + 1
    ys = None
    if split_out:
        assert out is None
        ys = torch.empty(3, N, Ho, Wo, Co, device=dev, dtype=torch.bfloat16)
        ldy = Co
    else:
        if out is None:
            out = torch.empty(N, Ho, Wo, Co, device=dev, dtype=torch.float32)
        assert out.shape[:3] == (N, Ho, Wo) and out.shape[3] >= Co and out.is_contiguous() and out.dtype == torch.float32
        ldy = out.shape[3]
    if residual is not None:
        residual = residual.contiguous()
        assert residual.shape == (N, Ho, Wo, Co) and ldy == Co
    with _span("conv", xs.planes if xs is not None else x):
        rc = lib().bev_conv2d_x6_f32(None if xs is not None else _ptr(x), _ptr(xs.planes) if xs is not None else None,
                                     N, H, W, Ci, _ptr(packed), _ptr(bias), _ptr(residual), Co, KH, KW, stride, pad,
                                     dilation, int(act), _ptr(out), _ptr(ys), ldy, Ho, Wo,
                                     _stream(xs.planes if xs is not None else x))
    _check(rc, "bev_conv2d_x6_f32")
    return Split3(ys) if split_out else out


def conv2d_stem_x6(x: torch.Tensor, packed: torch.Tensor, bias: torch.Tensor, Co: int, relu: bool,
                   out: torch.Tensor = None) -> torch.Tensor:
    """The ResNet stem (7x7 / s2 / p3 over NCHW [N,3,H,W] fp32 images) on the split arithmetic: packed = the split
    panel of the [Co,3,7,7] weights (pack_conv_weight_x6) -> y [N,Ho,Wo,Co] NHWC fp32 (bev_conv2d_stem_x6_f32)."""
    x = x.contiguous()
    _require_gpu(x, bias)
    N, Ci, H, W = x.shape
    if Ci != 3 or not packed.is_cuda or packed.dtype != torch.bfloat16:
        raise HipError("conv2d_stem_x6 takes NCHW 3-channel images and the split (bf16) weight panel on the device")
    Ho, Wo = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
    if out is None:
        out = torch.empty(N, Ho, Wo, Co, device=x.device, dtype=torch.float32)
    with _span("conv", x):
        rc = lib().bev_conv2d_stem_x6_f32(_ptr(x), N, H, W, _ptr(packed), _ptr(bias.contiguous().float()), Co,
                                          int(relu), _ptr(out), Ho, Wo, _stream(x))
    _check(rc, "bev_conv2d_stem_x6_f32")
    return out


def conv2d_stem_pool_x6(x: torch.Tensor, packed: torch.Tensor, bias: torch.Tensor, Co: int = 64) -> torch.Tensor:
    """conv2d_stem_x6 with ReLU followed by maxpool_nhwc(3, 2, 1) in one pass (bev_conv2d_stem_pool_x6_f32; Co = 64):
    NCHW [N,3,H,W] images -> the pooled NHWC [N,Hp,Wp,64], bit-identical to the two calls."""
    x = x.contiguous()
    _require_gpu(x, bias)
    N, Ci, H, W = x.shape
    if Ci != 3 or Co != 64 or not packed.is_cuda or packed.dtype != torch.bfloat16:
        raise HipError("conv2d_stem_pool_x6 takes NCHW 3-channel images, Co 64 and the split (bf16) weight panel")
    Ho, Wo = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
    Hp, Wp = (Ho - 1) // 2 + 1, (Wo - 1) // 2 + 1
    ws_bytes = int(lib().bev_conv2d_stem_pool_x6_workspace(N, H, W))
    _check(min(ws_bytes, 0), "bev_conv2d_stem_pool_x6_workspace")
    ws = torch.empty(ws_bytes, device=x.device, dtype=torch.uint8)
    out = torch.empty(N, Hp, Wp, 64, device=x.device, dtype=torch.float32)
    with _span("conv", x):
        rc = lib().bev_conv2d_stem_pool_x6_f32(_ptr(x), N, H, W, _ptr(packed), _ptr(bias.contiguous().float()), Co,
                                               _ptr(out), Hp, Wp, _ptr(ws), ws_bytes, _stream(x))
    _check(rc, "bev_conv2d_stem_pool_x6_f32")
    return out


def conv2d_nhwc(x: torch.Tensor, packed: torch.Tensor, bias, Co: int, KH: int, KW: int, stride: int, pad: int,
                relu: bool, residual: torch.Tensor = None, in_nchw: bool = False, out: torch.Tensor = None,
                ascale: torch.Tensor = None):
    """x: [N,H,W,Ci] NHWC (or [N,Ci,H,W] with in_nchw) -> y [N,Ho,Wo,Co] NHWC.
    ascale [N, Ci]: per-image input-channel multiplier applied in the operand load (SE excitation).
    The kernel follows the panel: fp32 (bev_conv2d_f32), split bf16 (bev_conv2d_x6_f32), fp16 (autocast)."""
    if packed.dtype == torch.bfloat16:
        if ascale is not None or in_nchw:
            raise HipError("the split-bf16 conv takes NHWC inputs without an operand channel scale")
        return conv2d_nhwc_x6(x, packed, bias, Co, KH, KW, stride, pad, 1, int(relu), residual=residual, out=out)
    x = x.contiguous()
    if packed.dtype == torch.float16:  # autocast(float16): the fp16 matrix-core kernel
        if ascale is not None:
            raise HipError("the fp16 conv takes no operand channel scale (the SE gate is applied apart in training)")
        if in_nchw:
            x = nchw_to_nhwc(x)
        return conv2d_nhwc_h16(x, packed, bias, Co, KH, KW, stride, pad, 1, int(relu), residual=residual, out=out)
    _require_gpu(x, packed, bias, residual)
    if in_nchw:
        N, Ci, H, W = x.shape
    else:
        N, H, W, Ci = x.shape
    Ho, Wo = (H + 2 * pad - KH) // stride + 1, (W + 2 * pad - KW) // stride + 1
    if out is None:
        out = torch.empty(N, Ho, Wo, Co, device=x.device, dtype=torch.float32)
    if residual is not None:
        residual = residual.contiguous()
        assert residual.shape == out.shape
    with _span("conv", x):
        if ascale is not None:
            assert not in_nchw and ascale.shape == (N, Ci) and ascale.is_contiguous()
            rc = lib().bev_conv2d_chscale_f32(_ptr(x), N, H, W, Ci, _ptr(ascale), _ptr(packed), _ptr(bias),
                                              _ptr(residual), Co, KH, KW, stride, pad, int(relu), _ptr(out), Ho, Wo,
                                              _stream(x))
        else:
            rc = lib().bev_conv2d_f32(_ptr(x), int(in_nchw), N, H, W, Ci, _ptr(packed), _ptr(bias), _ptr(residual),
                                      Co, KH, KW, stride, pad, int(relu), _ptr(out), Ho, Wo, _stream(x))
    _check(rc, "bev_conv2d_f32")
    return out


ACT_NONE, ACT_RELU, ACT_SILU = 0, 1, 2  # `relu` argument of conv2d_nhwc / dwconv2d_nhwc
ACT_RELU_FROM_Z = 3  # batchnorm_bwd only: ReLU of a layer without residual, mask recomputed from z (y not read)
ACT_RELU_MASK = 4  # batchnorm_bwd only: ReLU, mask from batchnorm_apply_mask's bytes (passed as y; bit-identical to 1)
H16_STAT_ROWS = 128  # rows per BatchNorm statistics tile of conv2d_nhwc_h16_bnstats


def conv2d_nhwc_h16_bnstats(x: torch.Tensor, packed: torch.Tensor, Co: int, KH: int, KW: int, stride: int, pad: int):
    """The fp16-operand conv of a train-mode BatchNorm layer (no bias, no activation; Ci % 64 == 0) with the BN batch
    statistics taken in its epilogue: -> (z [N,Ho,Wo,Co] fp32, tile partials [tiles, Co, 2] = per 128-row tile
    (sum, sum of squared deviations from the tile mean), channel-major [Co, tiles, 2]) for batchnorm_finalize_tiles."""
    x = x.contiguous()
    _require_gpu(x)
    if not packed.is_cuda or packed.dtype != torch.float16:
        raise HipError("conv2d_nhwc_h16_bnstats needs the fp16 weight panel on the device")
    N, H, W, Ci = x.shape
    Ho, Wo = (H + 2 * pad - KH) // stride + 1, (W + 2 * pad - KW) // stride + 1
    z = torch.empty(N, Ho, Wo, Co, device=x.device, dtype=torch.float32)
    nt = lib().bev_conv_h16_stat_tiles(N * Ho * Wo)
    _check(0 if nt > 0 else nt, "bev_conv_h16_stat_tiles")
    tiles = torch.empty(Co, nt, 2, device=x.device, dtype=torch.float32)
    with _span("conv", x):
        rc = lib().bev_conv2d_h16_bnstats_f32(_ptr(x), N, H, W, Ci, _ptr(packed), None, Co, KH, KW, stride, pad, 1,
                                              _ptr(z), Ho, Wo, _ptr(tiles), _stream(x))
    _check(rc, "bev_conv2d_h16_bnstats_f32")
    return z, tiles


# ---- fp16-STORED operands of the autocast convs (bit-identical: the kernels round these operands to fp16 anyway) ----
def _require_gpu_h(*ts):
    """Like _require_gpu, but fp16 tensors are accepted (operands stored in the precision the kernel computes in)."""
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise HipError("libbev_mi355x kernels need ROCm device tensors (got a CPU tensor); "
                           "this package has no CPU fallback")
        if t.dtype not in (torch.float32, torch.float16):
            raise HipError(f"fp32 / fp16 tensors expected, got {t.dtype}")


def conv2d_h16_any(x: torch.Tensor, packed: torch.Tensor, Co: int, KH: int, KW: int, stride: int, pad: int,
                   stats: bool = False, residual: torch.Tensor = None, bias: torch.Tensor = None, dilation: int = 1,
                   out: torch.Tensor = None):
    """The autocast fp16 conv with x [N,H,W,Ci] stored in fp32 or fp16 (Ci % 64 == 0 for fp16) -> z fp32
    [N,Ho,Wo,Co] (+ residual), and with `stats` the BatchNorm tile partials (conv2d_nhwc_h16_bnstats).  `out`: a
    wider NHWC fp32 buffer [N,Ho,Wo,>=Co] whose first Co channels receive z (the rest are left as they are)."""
    x = x.contiguous()
    _require_gpu_h(x)
    _require_gpu(residual, bias)
    if not packed.is_cuda or packed.dtype != torch.float16:
        raise HipError("conv2d_h16_any needs the fp16 weight panel on the device")
    N, H, W, Ci = x.shape
    Ho = (H + 2 * pad - dilation * (KH - 1) - 1) // stride + 1
    Wo = (W + 2 * pad - dilation * (KW - 1) - 1) // stride + 1
    if out is not None:
        assert (out.shape[:3] == (N, Ho, Wo) and out.shape[3] >= Co and out.is_contiguous() and out.is_cuda
                and out.dtype == torch.float32 and residual is None and not stats)
        z = out
    else:
        z = torch.empty(N, Ho, Wo, Co, device=x.device, dtype=torch.float32)
    tiles = None
    if stats:
        nt = lib().bev_conv_h16_stat_tiles(N * Ho * Wo)
        _check(0 if nt > 0 else nt, "bev_conv_h16_stat_tiles")
        tiles = torch.empty(Co, nt, 2, device=x.device, dtype=torch.float32)
    if residual is not None:
        residual = residual.contiguous()
    with _span("conv", x):
        rc = lib().bev_conv2d_h16_ex_f32(_ptr(x), int(x.dtype == torch.float16), N, H, W, Ci, _ptr(packed),
                                         _ptr(bias), _ptr(residual), Co, KH, KW, stride, pad, dilation, 0, _ptr(z),
                                         z.shape[3], Ho, Wo, _ptr(tiles), _stream(x))
    _check(rc, "bev_conv2d_h16_ex_f32")
    return (z, tiles) if stats else z


def conv_wgrad_h16_any(x: torch.Tensor, dz: torch.Tensor, KH: int, KW: int, stride: int, pad: int,
                       dilation: int = 1) -> torch.Tensor:
    """The autocast weight gradient with x / dz stored in fp32 or fp16 (Ci, Co % 4 == 0) -> dW [Co, Ci, KH, KW]."""
    x, dz = x.contiguous(), dz.contiguous()
    _require_gpu_h(x, dz)
    N, H, W, Ci = x.shape
    _, Ho, Wo, Co = dz.shape
    dW = torch.empty(Co, KH, KW, Ci, device=x.device, dtype=torch.float32)
    _check(lib().bev_conv_wgrad_h16_ex_f32(_ptr(x), int(x.dtype == torch.float16), N, H, W, Ci, _ptr(dz),
                                           int(dz.dtype == torch.float16), Ho, Wo, Co, KH, KW, stride, pad, dilation,
                                           _ptr(dW), _stream(x)), "bev_conv_wgrad_h16_ex_f32")
    return dW.permute(0, 3, 1, 2).contiguous()


def place_strided(y: torch.Tensor, s: int, H: int, W: int, residual: torch.Tensor = None) -> torch.Tensor:
    """y [N,Ho,Wo,C] fp32 -> out [N,H,W,C] = residual (or 0) + y at (s*oy, s*ox) (bev_place_strided_f32): the input
    gradient of a 1x1 / stride-s / pad-0 conv from y = dz W."""
    y = y.contiguous()
    _require_gpu(y, residual)
    N, Ho, Wo, C = y.shape
    out = torch.empty(N, H, W, C, device=y.device, dtype=torch.float32)
    if residual is not None:
        residual = residual.contiguous().float()
        assert residual.shape == out.shape
    _check(lib().bev_place_strided_f32(_ptr(y), N, Ho, Wo, C, s, H, W, _ptr(residual), _ptr(out), _stream(y)),
           "bev_place_strided_f32")
    return out


def dilate_nhwc_any(dz: torch.Tensor, s: int, top: int, left: int, Hd: int, Wd: int) -> torch.Tensor:
    dz = dz.contiguous()
    _require_gpu_h(dz)
    N, Ho, Wo, C = dz.shape
    out = torch.empty(N, Hd, Wd, C, device=dz.device, dtype=dz.dtype)
    _check(lib().bev_dilate_nhwc_ex(_ptr(dz), dz.element_size(), N, Ho, Wo, C, s, top, left, Hd, Wd, _ptr(out),
                                    _stream(dz)), "bev_dilate_nhwc_ex")
    return out


def batchnorm_apply_half(z: torch.Tensor, scale, shift, act: int = 0) -> torch.Tensor:
    """batchnorm_apply (no residual) with the output stored in fp16: for a y whose only readers are fp16-operand
    kernels (the next autocast conv and its weight gradient), which round it to exactly these values."""
    _require_gpu(z, scale, shift)
    assert z.is_contiguous()
    C = z.shape[-1]
    y = torch.empty(z.shape, device=z.device, dtype=torch.float16)
    _check(lib().bev_batchnorm_apply_ex_f32(_ptr(z), z.numel() // C, C, _ptr(scale), _ptr(shift), None, int(act),
                                            _ptr(y), 1, _stream(z)), "bev_batchnorm_apply_ex_f32")
    return y


def batchnorm_apply_mask(z: torch.Tensor, scale, shift, residual=None):
    """y = relu(z * scale + shift (+ residual)) and its ReLU mask bytes (bit u of byte k: y[4k + u] > 0) for the
    backward's ACT_RELU_MASK (bev_batchnorm_apply_mask_f32) -> (y fp32, mask uint8 [numel / 4])."""
    _require_gpu(z, scale, shift, residual)
    assert z.is_contiguous()
    if residual is not None:
        residual = residual.contiguous()
        assert residual.shape == z.shape
    C = z.shape[-1]
    y = torch.empty_like(z)
    mask = torch.empty(z.numel() // 4, device=z.device, dtype=torch.uint8)
    _check(lib().bev_batchnorm_apply_mask_f32(_ptr(z), z.numel() // C, C, _ptr(scale), _ptr(shift), _ptr(residual),
                                              _ptr(y), _ptr(mask), _stream(z)), "bev_batchnorm_apply_mask_f32")
    return y, mask


def batchnorm_bwd_half(dy: torch.Tensor, y, z: torch.Tensor, mean, rstd, gamma, want_dres: bool, act: int = 1,
                       scale=None, shift=None, frozen: bool = False):
    """batchnorm_bwd with dz stored in fp16 (for a dz read only by the fp16-operand dgrad / weight gradient).
    act ACT_RELU_MASK: `y` is the forward's ReLU mask bytes (batchnorm_apply_mask)."""
    dy = dy.contiguous()
    if act == ACT_RELU_MASK:
        if y is None or not y.is_cuda or y.dtype != torch.uint8 or y.numel() * 4 != z.numel():
            raise HipError("ACT_RELU_MASK needs the forward's uint8 mask (batchnorm_apply_mask)")
        _require_gpu(dy, z, mean, rstd, gamma, scale, shift)
    else:
        _require_gpu(dy, y, z, mean, rstd, gamma, scale, shift)
    C = z.shape[-1]
    M = z.numel() // C
    dz = torch.empty(z.shape, device=z.device, dtype=torch.float16)
    dres = torch.empty_like(z) if want_dres else None
    dg = torch.empty(C, device=z.device)
    db = torch.empty(C, device=z.device)
    ws = _bn_workspace(M, C, z.device)
    _check(lib().bev_batchnorm_bwd_ex_f32(_ptr(dy), _ptr(y), _ptr(z), M, C, _ptr(mean), _ptr(rstd),
                                          _ptr(gamma.detach().contiguous()), _ptr(scale), _ptr(shift), int(act),
                                          int(frozen), _ptr(dz), 1, _ptr(dres), _ptr(dg), _ptr(db), _ptr(ws),
                                          _stream(z)), "bev_batchnorm_bwd_ex_f32")
    return dz, dres, dg, db


def groupnorm_apply_half(x: torch.Tensor, scale, shift, relu: bool) -> torch.Tensor:
    """groupnorm_apply with the output stored in fp16 (read only by the next fp16 conv and its weight gradient)."""
    _require_gpu(x, scale, shift)
    assert x.is_contiguous()
    N, C = x.shape[0], x.shape[-1]
    y = torch.empty(x.shape, device=x.device, dtype=torch.float16)
    _check(lib().bev_groupnorm_apply_ex_f32(_ptr(x), N, x.numel() // (N * C), C, _ptr(scale), _ptr(shift), int(relu),
                                            _ptr(y), 1, _stream(x)), "bev_groupnorm_apply_ex_f32")
    return y


def groupnorm_bwd_half(x: torch.Tensor, dy: torch.Tensor, G: int, mean, rstd, gamma, scale, shift, relu: bool):
    """groupnorm_bwd with dx stored in fp16 (read only by the conv's fp16 dgrad and weight gradient)."""
    x, dy = x.contiguous(), dy.contiguous().float()
    _require_gpu(x, dy, mean, rstd, gamma, scale, shift)
    N, C = x.shape[0], x.shape[-1]
    P = x.numel() // (N * C)
    dx = torch.empty(x.shape, device=x.device, dtype=torch.float16)
    dg = torch.empty(C, device=x.device)
    db = torch.empty(C, device=x.device)
    ws = _gn_workspace(N, P, C, G, x.device)
    _check(lib().bev_groupnorm_bwd_ex_f32(_ptr(x), _ptr(dy), N, P, C, G, _ptr(mean), _ptr(rstd),
                                          _ptr(gamma.detach().contiguous()), _ptr(scale), _ptr(shift), int(relu),
                                          _ptr(dx), 1, _ptr(dg), _ptr(db), _ptr(ws), _stream(x)),
           "bev_groupnorm_bwd_ex_f32")
    return dx, dg, db


def batchnorm_finalize_tiles(tiles: torch.Tensor, M: int, gamma, beta, running_mean, running_var, eps: float,
                             momentum: float):
    """batchnorm_train_fwd's outputs (mean, rstd, scale, shift; running stats updated in place if given) from the
    per-tile partials of conv2d_nhwc_h16_bnstats over M rows."""
    _require_gpu(tiles, gamma, beta, running_mean, running_var)
    C, nt, _ = tiles.shape
    dev = tiles.device
    mean, rstd, scale, shift = (torch.empty(C, device=dev) for _ in range(4))
    with _span("batchnorm", tiles):
        rc = lib().bev_batchnorm_finalize_tiles_f32(_ptr(tiles), nt, H16_STAT_ROWS, M, C, float(eps), float(momentum),
                                                    _ptr(gamma.detach().contiguous()),
                                                    _ptr(beta.detach().contiguous()), _ptr(running_mean),
                                                    _ptr(running_var), _ptr(mean), _ptr(rstd), _ptr(scale),
                                                    _ptr(shift), _stream(tiles))
    _check(rc, "bev_batchnorm_finalize_tiles_f32")
    return mean, rstd, scale, shift


def conv2d_nhwc_h16(x: torch.Tensor, packed: torch.Tensor, bias, Co: int, KH: int, KW: int, stride: int, pad: int,
                    dilation: int = 1, act: int = 0, residual: torch.Tensor = None, out: torch.Tensor = None):
    """fp16-operand / fp32-accumulate conv (autocast(float16) arithmetic): x [N,H,W,Ci] fp32 NHWC, packed = the
    fp16 panel of pack_conv_weight under half_convs() -> y [N,Ho,Wo,Co] fp32 (or the first Co channels of a wider
    NHWC `out`)."""
    x = x.contiguous()
    _require_gpu(x, bias, residual)
    if not packed.is_cuda or packed.dtype != torch.float16:
        raise HipError("conv2d_nhwc_h16 needs the fp16 weight panel on the device")
    N, H, W, Ci = x.shape
    Ho, Wo = (H + 2 * pad - dilation * (KH - 1) - 1) // stride + 1, (W + 2 * pad - dilation * (KW - 1) - 1) // stride + 1
    if out is None:
        out = torch.empty(N, Ho, Wo, Co, device=x.device, dtype=torch.float32)
    assert out.shape[:3] == (N, Ho, Wo) and out.shape[3] >= Co and out.is_contiguous() and out.dtype == torch.float32
    if residual is not None:
        residual = residual.contiguous()
        assert residual.shape == (N, Ho, Wo, Co) and out.shape[3] == Co
    with _span("conv", x):
        rc = lib().bev_conv2d_h16_f32(_ptr(x), N, H, W, Ci, _ptr(packed), _ptr(bias), _ptr(residual), Co, KH, KW,
                                      stride, pad, dilation, int(act), _ptr(out), out.shape[3], Ho, Wo, _stream(x))
    _check(rc, "bev_conv2d_h16_f32")
    return out


def dwconv2d_nhwc(x: torch.Tensor, wt: torch.Tensor, bias: torch.Tensor, K: int, stride: int, pad: int, act: int,
                  want_psum: bool = False):
    """Depthwise KxK conv, NHWC: x [N,H,W,C], wt [K*K, C] (tap-major, BN folded), bias [C].
    Returns y [N,Ho,Wo,C] and, with want_psum, the SE partial channel sums [N, nb, C]."""
    x = x.contiguous()
    _require_gpu(x, wt, bias)
    N, H, W, C = x.shape
    Ho, Wo = (H + 2 * pad - K) // stride + 1, (W + 2 * pad - K) // stride + 1
    y = torch.empty(N, Ho, Wo, C, device=x.device, dtype=torch.float32)
    psum = None
    if want_psum:
        nb = lib().bev_dwconv_psum_blocks(Ho, Wo, C, stride)
        _check(0 if nb > 0 else nb, "bev_dwconv_psum_blocks")
        psum = torch.empty(N, nb, C, device=x.device, dtype=torch.float32)
    with _span("dwconv", x):
        rc = lib().bev_dwconv2d_f32(_ptr(x), N, H, W, C, _ptr(wt), _ptr(bias), K, stride, pad, int(act), _ptr(y), Ho,
                                    Wo, _ptr(psum), _stream(x))
    _check(rc, "bev_dwconv2d_f32")
    return y, psum


def conv2d_stem3(x: torch.Tensor, wt: torch.Tensor, bias: torch.Tensor, act: int) -> torch.Tensor:
    """EfficientNet stem (3x3 / s2 / p1, 3 input channels, BN folded) on the vector ALU: x [N,3,H,W] NCHW fp32,
    wt [27, Co] tap-major ((ci*3+ky)*3+kx), bias [Co] -> y [N,Ho,Wo,Co] NHWC (bev_conv2d_stem3_f32)."""
    x = x.contiguous()
    _require_gpu(x, wt, bias)
    N, Ci, H, W = x.shape
    Co = wt.shape[1]
    if Ci != 3 or wt.shape[0] != 27:
        raise HipError("conv2d_stem3 takes 3-channel images and a [27, Co] weight")
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    y = torch.empty(N, Ho, Wo, Co, device=x.device, dtype=torch.float32)
    with _span("conv", x):
        rc = lib().bev_conv2d_stem3_f32(_ptr(x), N, H, W, _ptr(wt.contiguous()), _ptr(bias.contiguous()), Co, int(act),
                                        _ptr(y), Ho, Wo, _stream(x))
    _check(rc, "bev_conv2d_stem3_f32")
    return y


def ir_expand_dw(x: torch.Tensor, we: torch.Tensor, be: torch.Tensor, wd: torch.Tensor, bd: torch.Tensor, K: int,
                 stride: int):
    """An inverted residual's expansion (1x1, BN folded, SiLU) and depthwise KxK / stride conv (BN folded, SiLU,
    pad K // 2) in one pass (bev_ir_expand_dw_f32): x [N,H,W,Ci] NHWC, we [Cm, Ci], be [Cm], wd [K*K, Cm] tap-major,
    bd [Cm] -> (y [N,Ho,Wo,Cm] NHWC, SE partial sums [N, nb, Cm]) like dwconv2d_nhwc(want_psum=True) over the
    expanded tensor, which is never stored."""
    x = x.contiguous()
    _require_gpu(x, we, be, wd, bd)
    N, H, W, Ci = x.shape
    Cm = we.shape[0]
    pad = K // 2
    Ho, Wo = (H + 2 * pad - K) // stride + 1, (W + 2 * pad - K) // stride + 1
    nb = lib().bev_ir_expand_dw_blocks(Ho, Wo, K, stride)
    _check(0 if nb > 0 else nb, "bev_ir_expand_dw_blocks")
    y = torch.empty(N, Ho, Wo, Cm, device=x.device, dtype=torch.float32)
    psum = torch.empty(N, nb, Cm, device=x.device, dtype=torch.float32)
    with _span("dwconv", x):
        rc = lib().bev_ir_expand_dw_f32(_ptr(x), N, H, W, Ci, _ptr(we.contiguous()), _ptr(be.contiguous()), Cm,
                                        _ptr(wd.contiguous()), _ptr(bd.contiguous()), K, stride, _ptr(y), Ho, Wo,
                                        _ptr(psum), _stream(x))
    _check(rc, "bev_ir_expand_dw_f32")
    return y, psum


def se_gate(psum: torch.Tensor, hw: int, w1: torch.Tensor, b1: torch.Tensor, w2: torch.Tensor, b2: torch.Tensor):
    """SqueezeExcite gate [N, C] from dwconv partial sums [N, nb, C]; w1 [rd, C], w2 [C, rd]."""
    _require_gpu(psum, w1, b1, w2, b2)
    N, nb, C = psum.shape
    rd = w1.shape[0]
    gate = torch.empty(N, C, device=psum.device, dtype=torch.float32)
    rc = lib().bev_se_gate_f32(_ptr(psum), N, nb, C, int(hw), _ptr(w1.contiguous()), _ptr(b1.contiguous()), rd,
                               _ptr(w2.contiguous()), _ptr(b2.contiguous()), _ptr(gate), _stream(psum))
    _check(rc, "bev_se_gate_f32")
    return gate


def channel_scale_(y: torch.Tensor, gate: torch.Tensor) -> torch.Tensor:
    """In place y[n, ..., c] *= gate[n, c] for NHWC y."""
    _require_gpu(y, gate)
    assert y.is_contiguous() and gate.is_contiguous()
    N, C = y.shape[0], y.shape[-1]
    P = y.numel() // (N * C)
    rc = lib().bev_channel_scale_f32(_ptr(y), N, P, C, _ptr(gate), _stream(y))
    _check(rc, "bev_channel_scale_f32")
    return y


def conv2d_dual_nhwc(x: torch.Tensor, x2: torch.Tensor, stride2: int, packed: torch.Tensor, bias, Co: int,
                     relu: bool, out: torch.Tensor = None):
    """act(x (*) W1 + x2[:, ::s2, ::s2] (*) W2 + bias), both 1x1, NHWC: x [N,Ho,Wo,Ci], x2 [N,H2,W2,Ci2]."""
    x = x.contiguous()
    x2 = x2.contiguous()
    _require_gpu(x, x2, bias, packed if packed.dtype != torch.bfloat16 else None)
    if not packed.is_cuda:
        raise HipError("conv2d_dual_nhwc needs the weight panel on the device")
    N, Ho, Wo, Ci = x.shape
    _, H2, W2, Ci2 = x2.shape
    if out is None:
        out = torch.empty(N, Ho, Wo, Co, device=x.device, dtype=torch.float32)
    if packed.dtype == torch.bfloat16:
        with _span("conv", x):
            rc = lib().bev_conv2d_dual_x6_f32(_ptr(x), N, Ho, Wo, Ci, _ptr(x2), H2, W2, Ci2, stride2, _ptr(packed),
                                              _ptr(bias), Co, int(relu), _ptr(out), _stream(x))
        _check(rc, "bev_conv2d_dual_x6_f32")
        return out
    with _span("conv", x):
        rc = lib().bev_conv2d_dual_f32(_ptr(x), N, Ho, Wo, Ci, _ptr(x2), H2, W2, Ci2, stride2, _ptr(packed),
                                       _ptr(bias), Co, int(relu), _ptr(out), _stream(x))
    _check(rc, "bev_conv2d_dual_f32")
    return out


def conv2d_chain_nhwc(x: torch.Tensor, packed: torch.Tensor, bias, Co: int, KH: int, KW: int, stride: int, pad: int,
                      relu: int, packed2: torch.Tensor, bias2, Co2: int, relu2: int, residual: torch.Tensor = None,
                      out: torch.Tensor = None):
    """act2(act(conv(x) + bias) (*) W2 + bias2 + residual) in one launch; x [N,H,W,Ci] NHWC -> [N,Ho,Wo,Co2].  In the
    split arithmetic x may be a Split3 (conv1's split output): conv2's operand is then staged by LDS-DMA with no
    split in the kernel (bit-identical to the fp32 x it holds)."""
    xs = x if isinstance(x, Split3) else None
    if xs is not None and packed.dtype != torch.bfloat16:
        raise HipError("a pre-split operand needs the split-bf16 panels")
    if xs is None:
        x = x.contiguous()
    src = xs.planes if xs is not None else x
    _require_gpu(x if xs is None else None, bias, bias2, residual,
                 *([packed, packed2] if packed.dtype != torch.bfloat16 else []))
    if xs is not None and not src.is_cuda:
        raise HipError("the pre-split operand must be on the device")
    if not (packed.is_cuda and packed2.is_cuda and packed.dtype == packed2.dtype):
        raise HipError("conv2d_chain_nhwc needs both weight panels on the device, in one arithmetic")
    N, H, W, Ci = x.shape
    Ho, Wo = (H + 2 * pad - KH) // stride + 1, (W + 2 * pad - KW) // stride + 1
    if out is None:
        out = torch.empty(N, Ho, Wo, Co2, device=x.device, dtype=torch.float32)
    if residual is not None:
        residual = residual.contiguous()
        assert residual.shape == out.shape
    if packed.dtype == torch.bfloat16:  # split-bf16 arithmetic (both panels from pack_conv_weight_x6)
        with _span("conv", src):
            rc = lib().bev_conv2d_chain_x6_f32(None if xs is not None else _ptr(x), _ptr(xs.planes) if xs is not None
                                               else None, N, H, W, Ci, _ptr(packed), _ptr(bias), Co, KH, KW, stride,
                                               pad, int(relu), _ptr(packed2), _ptr(bias2), Co2, _ptr(residual),
                                               int(relu2), _ptr(out), Ho, Wo, _stream(src))
        _check(rc, "bev_conv2d_chain_x6_f32")
        return out
    with _span("conv", x):
        rc = lib().bev_conv2d_chain_f32(_ptr(x), N, H, W, Ci, _ptr(packed), _ptr(bias), Co, KH, KW, stride, pad,
                                        int(relu), _ptr(packed2), _ptr(bias2), Co2, _ptr(residual), int(relu2),
                                        _ptr(out), Ho, Wo, _stream(x))
    _check(rc, "bev_conv2d_chain_f32")
    return out


def conv2d_chain_next_nhwc(xs: "Split3", packed: torch.Tensor, bias, Co: int, KH: int, KW: int, stride: int, pad: int,
                           relu: int, packed2: torch.Tensor, bias2, Co2: int, relu2: int, packed3: torch.Tensor, bias3,
                           Co3: int, relu3: int, residual: torch.Tensor = None, x2: torch.Tensor = None,
                           stride2: int = 1, out: torch.Tensor = None, split3_out: bool = True):
    """A pre-split chained bottleneck body (conv2d_chain_nhwc with a Split3 x; with x2 the dual form of
    conv2d_chain_dual_nhwc) that also runs the next block's 1x1 conv on the block output it computes
    (bev_conv2d_chain_next_x6_f32): returns (y [N,Ho,Wo,Co2] fp32, h3) with h3 = act3(y (*) W3 + bias3) as a Split3
    (split3_out) or fp32 [N,Ho,Wo,Co3] -- bit-identical to conv2d_nhwc_x6 over y, without reading y back."""
    if not isinstance(xs, Split3) or not (packed.dtype == packed2.dtype == packed3.dtype == torch.bfloat16):
        raise HipError("conv2d_chain_next_nhwc takes a Split3 operand and split-bf16 panels")
    if not xs.planes.is_cuda:
        raise HipError("the pre-split operand must be on the device")
    _require_gpu(bias, bias2, bias3, residual, x2)
    N, H, W, Ci = xs.shape
    Ho, Wo = (H + 2 * pad - KH) // stride + 1, (W + 2 * pad - KW) // stride + 1
    dev = xs.device
    if out is None:
        out = torch.empty(N, Ho, Wo, Co2, device=dev, dtype=torch.float32)
    assert out.shape == (N, Ho, Wo, Co2) and out.is_contiguous()
    if residual is not None:
        residual = residual.contiguous()
        assert residual.shape == out.shape
    H2 = W2 = Ci2 = 0
    if x2 is not None:
        x2 = x2.contiguous()
        _, H2, W2, Ci2 = x2.shape
    if split3_out:
        ys3, y3 = torch.empty(3, N, Ho, Wo, Co3, device=dev, dtype=torch.bfloat16), None
    else:
        ys3, y3 = None, torch.empty(N, Ho, Wo, Co3, device=dev, dtype=torch.float32)
    with _span("conv", xs.planes):
        rc = lib().bev_conv2d_chain_next_x6_f32(
            _ptr(xs.planes), N, H, W, Ci, _ptr(packed), _ptr(bias), Co, KH, KW, stride, pad, int(relu), _ptr(x2), H2,
            W2, Ci2, stride2, _ptr(packed2), _ptr(bias2), Co2, _ptr(residual), int(relu2), _ptr(out), Ho, Wo,
            _ptr(packed3), _ptr(bias3), Co3, int(relu3), _ptr(y3), _ptr(ys3), _stream(xs.planes))
    _check(rc, "bev_conv2d_chain_next_x6_f32")
    return out, (Split3(ys3) if split3_out else y3)


def conv2d_chain_dual_nhwc(x: torch.Tensor, packed: torch.Tensor, bias, Co: int, KH: int, KW: int, stride: int,
                           pad: int, relu: int, x2: torch.Tensor, stride2: int, packed2: torch.Tensor, bias2, Co2: int,
                           relu2: int, out: torch.Tensor = None):
    """act2([act(conv(x) + bias) | x2[:, ::s2, ::s2]] (*) W2 + bias2) in one launch (bottleneck with downsample).
    x may be a Split3 in the split arithmetic, as for conv2d_chain_nhwc."""
    xs = x if isinstance(x, Split3) else None
    if xs is not None and packed.dtype != torch.bfloat16:
        raise HipError("a pre-split operand needs the split-bf16 panels")
    if xs is None:
        x = x.contiguous()
    src = xs.planes if xs is not None else x
    x2 = x2.contiguous()
    _require_gpu(x if xs is None else None, bias, x2, bias2,
                 *([packed, packed2] if packed.dtype != torch.bfloat16 else []))
    if xs is not None and not src.is_cuda:
        raise HipError("the pre-split operand must be on the device")
    if not (packed.is_cuda and packed2.is_cuda and packed.dtype == packed2.dtype):
        raise HipError("conv2d_chain_dual_nhwc needs both weight panels on the device, in one arithmetic")
    N, H, W, Ci = x.shape
    _, H2, W2, Ci2 = x2.shape
    Ho, Wo = (H + 2 * pad - KH) // stride + 1, (W + 2 * pad - KW) // stride + 1
    if out is None:
        out = torch.empty(N, Ho, Wo, Co2, device=x.device, dtype=torch.float32)
    if packed.dtype == torch.bfloat16:  # split-bf16 arithmetic
        with _span("conv", src):
            rc = lib().bev_conv2d_chain_dual_x6_f32(None if xs is not None else _ptr(x),
                                                    _ptr(xs.planes) if xs is not None else None, N, H, W, Ci,
                                                    _ptr(packed), _ptr(bias), Co, KH, KW, stride, pad, int(relu),
                                                    _ptr(x2), H2, W2, Ci2, stride2, _ptr(packed2), _ptr(bias2), Co2,
                                                    int(relu2), _ptr(out), Ho, Wo, _stream(src))
        _check(rc, "bev_conv2d_chain_dual_x6_f32")
        return out
    with _span("conv", x):
        rc = lib().bev_conv2d_chain_dual_f32(_ptr(x), N, H, W, Ci, _ptr(packed), _ptr(bias), Co, KH, KW, stride, pad,
                                             int(relu), _ptr(x2), H2, W2, Ci2, stride2, _ptr(packed2), _ptr(bias2),
                                             Co2, int(relu2), _ptr(out), Ho, Wo, _stream(x))
    _check(rc, "bev_conv2d_chain_dual_f32")
    return out


def maxpool_nhwc(x: torch.Tensor, k: int, stride: int, pad: int) -> torch.Tensor:
    x = x.contiguous()
    _require_gpu(x)
    N, H, W, C = x.shape
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    y = torch.empty(N, Ho, Wo, C, device=x.device, dtype=torch.float32)
    _check(lib().bev_maxpool2d_nhwc_f32(_ptr(x), N, H, W, C, k, stride, pad, _ptr(y), Ho, Wo, _stream(x)),
           "bev_maxpool2d_nhwc_f32")
    return y


def nchw_to_nhwc(x: torch.Tensor) -> torch.Tensor:
    x = x.contiguous()
    _require_gpu(x)
    N, C, H, W = x.shape
    y = torch.empty(N, H, W, C, device=x.device, dtype=torch.float32)
    _check(lib().bev_nchw_to_nhwc_f32(_ptr(x), N, C, H, W, _ptr(y), _stream(x)), "bev_nchw_to_nhwc_f32")
    return y


def nchw_to_nhwc4(x: torch.Tensor) -> torch.Tensor:
    """[N,C,H,W] (C <= 4) -> [N,H,W,4] NHWC with zero channels past C (bev_nchw_to_nhwc4_f32): the stem's input as
    its weight gradient's float4 operand."""
    x = x.contiguous()
    _require_gpu(x)
    N, C, H, W = x.shape
    y = torch.empty(N, H, W, 4, device=x.device, dtype=torch.float32)
    _check(lib().bev_nchw_to_nhwc4_f32(_ptr(x), N, C, H, W, _ptr(y), _stream(x)), "bev_nchw_to_nhwc4_f32")
    return y


def nhwc_to_nchw(x: torch.Tensor) -> torch.Tensor:
    x = x.contiguous()
    _require_gpu(x)
    N, H, W, C = x.shape
    y = torch.empty(N, C, H, W, device=x.device, dtype=torch.float32)
    _check(lib().bev_nhwc_to_nchw_f32(_ptr(x), N, C, H, W, _ptr(y), _stream(x)), "bev_nhwc_to_nchw_f32")
    return y


# ---------------------------------------------------------------------------
# trunk backward (training)
# ---------------------------------------------------------------------------
def relu_bwd(dy: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    dy, y = dy.contiguous(), y.contiguous()
    _require_gpu(dy, y)
    dz = torch.empty_like(y)
    _check(lib().bev_relu_bwd_f32(_ptr(dy), _ptr(y), _ptr(dz), y.numel(), _stream(y)), "bev_relu_bwd_f32")
    return dz


def dilate_nhwc(dz: torch.Tensor, s: int, top: int, left: int, Hd: int, Wd: int) -> torch.Tensor:
    dz = dz.contiguous()
    _require_gpu(dz)
    N, Ho, Wo, C = dz.shape
    out = torch.empty(N, Hd, Wd, C, device=dz.device, dtype=torch.float32)
    _check(lib().bev_dilate_nhwc_f32(_ptr(dz), N, Ho, Wo, C, s, top, left, Hd, Wd, _ptr(out), _stream(dz)),
           "bev_dilate_nhwc_f32")
    return out


def _pad_last(t: torch.Tensor, m: int) -> torch.Tensor:
    c = t.shape[-1]
    return t if c % m == 0 else torch.nn.functional.pad(t, (0, m - c % m))


def conv_wgrad(x: torch.Tensor, dz: torch.Tensor, KH: int, KW: int, stride: int, pad: int) -> torch.Tensor:
    """x [N,H,W,Ci], dz [N,Ho,Wo,Co] (NHWC) -> dW [Co, Ci, KH, KW] (torch OIHW)."""
    return conv_wgrad_ex(x, dz, KH, pad, 1, stride=stride, KW=KW)


def colsum(dz: torch.Tensor) -> torch.Tensor:
    dz = dz.contiguous()
    _require_gpu(dz)
    C = dz.shape[-1]
    db = torch.empty(C, device=dz.device, dtype=torch.float32)
    _check(lib().bev_colsum_f32(_ptr(dz), dz.numel() // C, C, _ptr(db), _stream(dz)), "bev_colsum_f32")
    return db


def maxpool_fwd_arg_nhwc(x: torch.Tensor, k: int, stride: int, pad: int):
    """Training max-pool: (y [N,Ho,Wo,C], argmax uint8 [N,Ho,Wo,C]) -- maxpool_nhwc's values and the window argmax
    bytes maxpool_bwd_arg_nhwc consumes (C % 4 == 0, k * k <= 255)."""
    x = x.contiguous()
    _require_gpu(x)
    N, H, W, C = x.shape
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    y = torch.empty(N, Ho, Wo, C, device=x.device, dtype=torch.float32)
    arg = torch.empty(N, Ho, Wo, C, device=x.device, dtype=torch.uint8)
    _check(lib().bev_maxpool2d_fwd_arg_nhwc_f32(_ptr(x), N, H, W, C, k, stride, pad, _ptr(y), _ptr(arg), Ho, Wo,
                                                _stream(x)), "bev_maxpool2d_fwd_arg_nhwc_f32")
    return y, arg


def maxpool_bwd_arg_nhwc(arg: torch.Tensor, dy: torch.Tensor, H: int, W: int, k: int, stride: int,
                         pad: int) -> torch.Tensor:
    """dx [N,H,W,C] of the max-pool from its forward's argmax bytes (maxpool_fwd_arg_nhwc): bit-identical to
    maxpool_bwd_nhwc."""
    dy = dy.contiguous()
    _require_gpu(dy)
    if not arg.is_cuda or arg.dtype != torch.uint8 or arg.shape != dy.shape:
        raise HipError("maxpool_bwd_arg_nhwc needs the forward's uint8 argmax of dy's shape")
    N, Ho, Wo, C = dy.shape
    dx = torch.empty(N, H, W, C, device=dy.device, dtype=torch.float32)
    _check(lib().bev_maxpool2d_bwd_arg_nhwc_f32(_ptr(arg), _ptr(dy), N, H, W, C, k, stride, pad, Ho, Wo, _ptr(dx),
                                                _stream(dy)), "bev_maxpool2d_bwd_arg_nhwc_f32")
    return dx


def maxpool_bwd_nhwc(x: torch.Tensor, dy: torch.Tensor, k: int, stride: int, pad: int) -> torch.Tensor:
    x, dy = x.contiguous(), dy.contiguous()
    _require_gpu(x, dy)
    N, H, W, C = x.shape
    Ho, Wo = dy.shape[1], dy.shape[2]
    dx = torch.empty_like(x)
    if C % 4 == 0 and k * k <= 255:  # window argmax bytes once, then the gather (bit-identical, ~16x fewer loads)
        arg = torch.empty(N, Ho, Wo, C, device=x.device, dtype=torch.uint8)
        _check(lib().bev_maxpool2d_bwd_ws_nhwc_f32(_ptr(x), _ptr(dy), N, H, W, C, k, stride, pad, Ho, Wo, _ptr(dx),
                                                   _ptr(arg), _stream(x)), "bev_maxpool2d_bwd_ws_nhwc_f32")
        return dx
    _check(lib().bev_maxpool2d_bwd_nhwc_f32(_ptr(x), _ptr(dy), N, H, W, C, k, stride, pad, Ho, Wo, _ptr(dx),
                                            _stream(x)), "bev_maxpool2d_bwd_nhwc_f32")
    return dx


# ---------------------------------------------------------------------------
# decode (detector.py:64-125)
# ---------------------------------------------------------------------------
class _PendingDecode:
    """A decode whose kernels are queued: the kept / candidate counts travel to pinned host memory behind an
    event, and the host waits for them only when a result is first read (`get`)."""

    def __init__(self, finish):
        self._finish, self._val = finish, None

    def get(self):
        if self._val is None:
            self._val, self._finish = self._finish(), None
        return self._val


class DetectionList(collections.abc.Sequence):
    """Per-frame boxes (which 0) or scores (which 1) of a decode queued by decode(lazy=True): a read-only sequence
    of device tensors, materialised -- one host synchronisation for the batch -- on first access.  A training step
    that never reads the detections of its forward (train.py:238-243 reads only the loss) therefore never waits for
    them, and the loss and backward launches queue behind the forward instead of after a drained GPU."""

    def __init__(self, pending: _PendingDecode, which: int):
        self._p, self._w = pending, which

    def __getitem__(self, i):
        return self._p.get()[self._w][i]

    def __len__(self):
        return len(self._p.get()[self._w])

    def __repr__(self):
        return repr(list(self))


def decode(heatmap: torch.Tensor, offset: torch.Tensor, size: torch.Tensor, bounds, conf_thresh: float,
           nms_dist: float, lazy: bool = False):
    """heatmap [B,1,H,W], offset / size [B,2,H,W] (device) -> (boxes list of [K,4], scores list of [K]).
    Like the reference there is no candidate limit: a frame with more candidates than the LDS sort holds
    (bev_decode_max_candidates) is finished by the global-memory sort + blocked NMS (bev_decode_nms_large_f32).
    One host synchronisation per batch (two when some frame needs the large path).  lazy: return two
    DetectionList sequences instead; the synchronisation happens when one of them is first read."""
    heatmap, offset, size = heatmap.contiguous().float(), offset.contiguous().float(), size.contiguous().float()
    _require_gpu(heatmap, offset, size)
    B, _, H, W = heatmap.shape
    cap = H * W  # every cell can be a candidate (plateaus): the candidate list never overflows
    dev = heatmap.device
    idx = torch.empty(B, cap, device=dev, dtype=torch.int32)
    sc = torch.empty(B, cap, device=dev, dtype=torch.float32)
    cnt = torch.empty(B, device=dev, dtype=torch.int32)
    st = _stream(heatmap)
    _check(lib().bev_decode_peaks_f32(_ptr(heatmap), B, H, W, float(conf_thresh), cap, _ptr(idx), _ptr(sc), _ptr(cnt),
                                      st), "bev_decode_peaks_f32")
    x_min, x_max, y_min, y_max = bounds
    res_x, res_y = (x_max - x_min) / float(W), (y_max - y_min) / float(H)
    boxes = torch.empty(B, cap, 4, device=dev, dtype=torch.float32)
    scores = torch.empty(B, cap, device=dev, dtype=torch.float32)
    nk = torch.empty(B, device=dev, dtype=torch.int32)
    args = (float(x_min), float(y_min), float(res_x), float(res_y), float(nms_dist))
    _check(lib().bev_decode_nms_f32(_ptr(idx), _ptr(sc), _ptr(cnt), B, cap, _ptr(offset), _ptr(size), H, W, *args,
                                    _ptr(boxes), _ptr(scores), _ptr(nk), st), "bev_decode_nms_f32")
    kc = torch.empty(2, B, dtype=torch.int32, pin_memory=True)
    kc.copy_(torch.stack([nk, cnt]), non_blocking=True)
    queued_on = torch.cuda.current_stream(dev)
    ready = torch.cuda.Event()
    ready.record(queued_on)

    def finish():
        ready.synchronize()
        kept, counts = kc[0].tolist(), kc[1].tolist()
        if min(kept, default=0) < 0:
            big = max(c for k, c in zip(kept, counts) if k < 0)
            P = max(2 * DECODE_SORT_CHUNK, 1 << (big - 1).bit_length())
            keys = torch.empty(B, P, device=dev, dtype=torch.int64)
            with torch.cuda.stream(queued_on):  # the large path on the stream the decode was queued on
                _check(lib().bev_decode_nms_large_f32(_ptr(idx), _ptr(sc), _ptr(cnt), B, cap, P, _ptr(offset),
                                                      _ptr(size), H, W, *args, _ptr(keys), _ptr(boxes), _ptr(scores),
                                                      _ptr(nk), st), "bev_decode_nms_large_f32")
                kept = nk.cpu().tolist()
            if min(kept, default=0) < 0:
                raise HipError("decode: large-candidate path left a frame unfinished")
        return [boxes[b, :k] for b, k in enumerate(kept)], [scores[b, :k] for b, k in enumerate(kept)]

    if not lazy:
        return finish()
    pending = _PendingDecode(finish)
    return DetectionList(pending, 0), DetectionList(pending, 1)


def focal_loss(logits: torch.Tensor, gt: torch.Tensor, alpha: float, beta: float):
    """CenterNet focal heatmap loss (model_wrapper.py:235-247) over same-shaped fp32 logits / gt on the device ->
    (loss [] fp32, inv_norm [1] = 1 / max(#peaks, 1) for focal_loss_bwd)."""
    logits, gt = logits.contiguous(), gt.contiguous()
    _require_gpu(logits, gt)
    if logits.dtype != torch.float32 or gt.dtype != torch.float32 or logits.shape != gt.shape:
        raise HipError("focal_loss: fp32 logits / gt of one shape")
    n = logits.numel()
    ws = torch.empty(lib().bev_focal_loss_workspace_bytes(n), device=logits.device, dtype=torch.uint8)
    loss = torch.empty((), device=logits.device, dtype=torch.float32)
    inv = torch.empty(1, device=logits.device, dtype=torch.float32)
    _check(lib().bev_focal_loss_fwd_f32(_ptr(logits), _ptr(gt), n, float(alpha), float(beta), _ptr(loss), _ptr(inv),
                                        _ptr(ws), ws.numel(), _stream(logits)), "bev_focal_loss_fwd_f32")
    return loss, inv


def focal_loss_bwd(logits, gt, alpha: float, beta: float, grad_loss: torch.Tensor, inv: torch.Tensor) -> torch.Tensor:
    logits, gt, grad_loss = logits.contiguous(), gt.contiguous(), grad_loss.contiguous().float()
    _require_gpu(logits, gt, grad_loss, inv)
    dx = torch.empty_like(logits)
    _check(lib().bev_focal_loss_bwd_f32(_ptr(logits), _ptr(gt), logits.numel(), float(alpha), float(beta),
                                        _ptr(grad_loss), _ptr(inv), _ptr(dx), _stream(logits)), "bev_focal_loss_bwd_f32")
    return dx


def _l1_operands(offset, size, indices, mask, off_t, size_t):
    """The L1 losses' slot operands as rows of a common length ld (the targets' [B, M + 1] buffers viewed [:, :M])."""
    B, M = indices.shape
    ld = indices.stride(0)
    ok = (indices.stride(1) == 1 and mask.stride() == (ld, 1) and off_t.stride() == (2 * ld, 2, 1)
          and size_t.stride() == (2 * ld, 2, 1) and indices.dtype == torch.int64 and mask.dtype == torch.float32
          and off_t.dtype == torch.float32 and size_t.dtype == torch.float32)
    if not ok:
        indices, mask = indices.contiguous().long(), mask.contiguous().float()
        off_t, size_t, ld = off_t.contiguous().float(), size_t.contiguous().float(), M
    offset, size = offset.contiguous().float(), size.contiguous().float()
    _require_gpu(offset, size, mask, off_t, size_t)
    if not indices.is_cuda or indices.device != offset.device:
        raise HipError("l1_losses: indices must be an int64 tensor on the maps' device")
    if offset.shape != size.shape or offset.shape[:2] != (B, 2):
        raise HipError("l1_losses: offset / size [B, 2, H, W]")
    return offset, size, indices, mask, off_t, size_t, B, M, ld, offset.shape[2] * offset.shape[3]


def l1_losses(offset, size, indices, mask, off_t, size_t) -> torch.Tensor:
    """model_wrapper.py:109-116's masked L1 offset / log-size losses on the device -> [3] = (offset loss, size loss,
    1 / n) (bev_l1_losses_fwd_f32)."""
    o, sz, idx, m, ot, st, B, M, ld, HW = _l1_operands(offset, size, indices, mask, off_t, size_t)
    out = torch.empty(3, device=o.device, dtype=torch.float32)
    _check(lib().bev_l1_losses_fwd_f32(_ptr(o), _ptr(sz), B, HW, _ptr(idx), _ptr(m), _ptr(ot), _ptr(st), M, ld,
                                       _ptr(out), _stream(o)), "bev_l1_losses_fwd_f32")
    return out


def l1_losses_bwd(offset, size, indices, mask, off_t, size_t, grad_losses, fwd_out):
    o, sz, idx, m, ot, st, B, M, ld, HW = _l1_operands(offset, size, indices, mask, off_t, size_t)
    d_off, d_sz = torch.zeros_like(o), torch.zeros_like(sz)
    g = grad_losses.contiguous().float()
    _require_gpu(g, fwd_out)
    _check(lib().bev_l1_losses_bwd_f32(_ptr(o), _ptr(sz), B, HW, _ptr(idx), _ptr(m), _ptr(ot), _ptr(st), M, ld,
                                       _ptr(g), _ptr(fwd_out), _ptr(d_off), _ptr(d_sz), _stream(o)),
           "bev_l1_losses_bwd_f32")
    return d_off, d_sz


def gaussian_radius(width_cells: torch.Tensor, height_cells: torch.Tensor, overlap: float, min_radius: int):
    """BEVNet._gaussian_radius_tensor (model_wrapper.py:205-233) in one launch, the same float32 values as torch's ops
    on the device -> int64 radii."""
    import numpy as np
    w, h = width_cells.contiguous(), height_cells.contiguous()
    _require_gpu(w, h)
    out = torch.empty(w.shape, device=w.device, dtype=torch.int64)
    f32 = np.float32
    _check(lib().bev_gaussian_radius_f32(_ptr(w), _ptr(h), w.numel(), float(f32(1 - overlap)),
                                         float(f32(1.0) / f32(1 + overlap)), float(f32(4 * overlap)),
                                         float(f32(-2 * overlap)), float(f32(overlap - 1)), int(overlap == 0),
                                         float(min_radius), _ptr(out), _stream(w)), "bev_gaussian_radius_f32")
    return out


DECODE_SORT_CHUNK = 8192  # keys per LDS chunk of the large-path sort (bev_decode.hip SORT_CHUNK)


# ---------------------------------------------------------------------------
# BEV head (detector.py:16-62): dilated / operand-affine convs, GroupNorm
# ---------------------------------------------------------------------------
def conv2d_nhwc_ex(x: torch.Tensor, packed: torch.Tensor, bias, Co: int, K: int, pad: int, dilation: int = 1,
                   in_scale: torch.Tensor = None, in_shift: torch.Tensor = None, in_relu: bool = False,
                   out: torch.Tensor = None, relu: bool = False) -> torch.Tensor:
    """Stride-1 KxK conv over NHWC x [N,H,W,Ci] with dilation and the previous layer's GroupNorm + ReLU
    applied to the operand (in_scale / in_shift [N, Ci]).  `out` may be a wider NHWC buffer [N,Ho,Wo,>=Co]
    whose first Co channels receive y."""
    x = x.contiguous()
    if packed.dtype == torch.float16:  # autocast(float16): the fp16 matrix-core kernel
        if in_scale is not None or in_shift is not None:
            raise HipError("the fp16 conv takes no operand affine (GroupNorm is materialised in training)")
        return conv2d_nhwc_h16(x, packed, bias, Co, K, K, 1, pad, dilation, int(relu), out=out)
    _require_gpu(x, packed, bias, in_scale, in_shift)
    N, H, W, Ci = x.shape
    Ho, Wo = H + 2 * pad - dilation * (K - 1), W + 2 * pad - dilation * (K - 1)
    if out is None:
        out = torch.empty(N, Ho, Wo, Co, device=x.device, dtype=torch.float32)
    assert out.shape[:3] == (N, Ho, Wo) and out.shape[3] >= Co and out.stride(3) == 1 and out.is_contiguous()
    with _span("conv", x):
        rc = lib().bev_conv2d_nhwc_ex_f32(_ptr(x), N, H, W, Ci, _ptr(in_scale), _ptr(in_shift), int(in_relu),
                                          _ptr(packed), _ptr(bias), Co, K, K, 1, pad, dilation, int(relu), _ptr(out),
                                          out.shape[3], Ho, Wo, _stream(x))
    _check(rc, "bev_conv2d_nhwc_ex_f32")
    return out


def conv_wgrad_ex(x: torch.Tensor, dz: torch.Tensor, K: int, pad: int, dilation: int, stride: int = 1,
                  KW: int = None) -> torch.Tensor:
    """Conv weight gradient (dilation, stride): x [N,H,W,Ci], dz [N,Ho,Wo,Co] -> dW [Co, Ci, K, KW] (OIHW view).
    Ci and Co are zero-padded to multiples of 4 here (the stem's 3 input channels, the head's 5 outputs) so
    every call takes the float4 kernel; the padding's gradient rows / columns are sliced off."""
    KH, KW = K, (K if KW is None else KW)
    N, H, W, Ci = x.shape
    _, Ho, Wo, Co = dz.shape
    xp, dzp = _pad_last(x.contiguous(), 4).contiguous(), _pad_last(dz.contiguous(), 4).contiguous()
    _require_gpu(xp, dzp)
    Cip, Cop = xp.shape[-1], dzp.shape[-1]
    dW = torch.empty(Cop, KH, KW, Cip, device=x.device, dtype=torch.float32)
    if half_convs() and Ci % 32 == 0:  # autocast(float16): the weight gradient of an fp16 conv on the fp16 MFMA
        _check(lib().bev_conv_wgrad_h16_f32(_ptr(xp), N, H, W, Cip, _ptr(dzp), Ho, Wo, Cop, KH, KW, stride, pad,
                                            dilation, _ptr(dW), _stream(x)), "bev_conv_wgrad_h16_f32")
        return dW[:Co, :, :, :Ci].permute(0, 3, 1, 2).contiguous()
    _check(lib().bev_conv_wgrad_ex_f32(_ptr(xp), N, H, W, Cip, _ptr(dzp), Ho, Wo, Cop, KH, KW, stride, pad, dilation,
                                       _ptr(dW), _stream(x)), "bev_conv_wgrad_ex_f32")
    return dW[:Co, :, :, :Ci].permute(0, 3, 1, 2).contiguous()  # the parameter's OIHW strides (DDP bucket views)


def _gn_workspace(N, P, C, G, device):
    nbytes = lib().bev_groupnorm_workspace_bytes(N, P, C, G)
    if nbytes < 0:
        raise HipError(f"GroupNorm shape not supported: C={C}, G={G}")
    return torch.empty((nbytes + 7) // 8, device=device, dtype=torch.float64)


def groupnorm_fwd(x: torch.Tensor, G: int, gamma: torch.Tensor, beta: torch.Tensor, eps: float):
    """x [N,H,W,C] NHWC -> (mean [N,G], rstd [N,G], scale [N,C], shift [N,C])."""
    _require_gpu(x, gamma, beta)
    assert x.is_contiguous()
    N, C = x.shape[0], x.shape[-1]
    P = x.numel() // (N * C)
    dev = x.device
    mean = torch.empty(N, G, device=dev)
    rstd = torch.empty(N, G, device=dev)
    scale = torch.empty(N, C, device=dev)
    shift = torch.empty(N, C, device=dev)
    ws = _gn_workspace(N, P, C, G, dev)
    with _span("groupnorm", x):
        rc = lib().bev_groupnorm_fwd_f32(_ptr(x), N, P, C, G, float(eps), _ptr(gamma.detach().contiguous()),
                                         _ptr(beta.detach().contiguous()), _ptr(mean), _ptr(rstd), _ptr(scale),
                                         _ptr(shift), _ptr(ws), _stream(x))
    _check(rc, "bev_groupnorm_fwd_f32")
    return mean, rstd, scale, shift


def groupnorm_apply(x: torch.Tensor, scale: torch.Tensor, shift: torch.Tensor, relu: bool) -> torch.Tensor:
    _require_gpu(x, scale, shift)
    assert x.is_contiguous()
    N, C = x.shape[0], x.shape[-1]
    y = torch.empty_like(x)
    _check(lib().bev_groupnorm_apply_f32(_ptr(x), N, x.numel() // (N * C), C, _ptr(scale), _ptr(shift), int(relu),
                                         _ptr(y), _stream(x)), "bev_groupnorm_apply_f32")
    return y


def groupnorm_bwd(x, dy, G, mean, rstd, gamma, scale, shift, relu: bool):
    """-> (dx [N,H,W,C], dgamma [C], dbeta [C]) of y = relu?(groupnorm(x))."""
    x, dy = x.contiguous(), dy.contiguous()
    _require_gpu(x, dy, mean, rstd, gamma, scale, shift)
    N, C = x.shape[0], x.shape[-1]
    P = x.numel() // (N * C)
    dx = torch.empty_like(x)
    dg = torch.empty(C, device=x.device)
    db = torch.empty(C, device=x.device)
    ws = _gn_workspace(N, P, C, G, x.device)
    _check(lib().bev_groupnorm_bwd_f32(_ptr(x), _ptr(dy), N, P, C, G, _ptr(mean), _ptr(rstd),
                                       _ptr(gamma.detach().contiguous()), _ptr(scale), _ptr(shift), int(relu), _ptr(dx),
                                       _ptr(dg), _ptr(db), _ptr(ws), _stream(x)), "bev_groupnorm_bwd_f32")
    return dx, dg, db


# ---------------------------------------------------------------------------
# BatchNorm with batch statistics (trunk training, train.py:222)
# ---------------------------------------------------------------------------
def _bn_workspace(M, C, device):
    nbytes = lib().bev_batchnorm_workspace_bytes(M, C)
    if nbytes < 0:
        raise HipError(f"BatchNorm shape not supported: M={M}, C={C}")
    return torch.empty((nbytes + 7) // 8, device=device, dtype=torch.float64)


def batchnorm_train_fwd(z: torch.Tensor, gamma, beta, running_mean, running_var, eps: float, momentum: float):
    """z [..., C] NHWC contiguous -> (mean, rstd, scale, shift) [C]; running stats updated in place (if given)."""
    _require_gpu(z, gamma, beta, running_mean, running_var)
    assert z.is_contiguous()
    C = z.shape[-1]
    M = z.numel() // C
    dev = z.device
    mean, rstd, scale, shift = (torch.empty(C, device=dev) for _ in range(4))
    ws = _bn_workspace(M, C, dev)
    with _span("batchnorm", z):
        rc = lib().bev_batchnorm_train_fwd_f32(_ptr(z), M, C, float(eps), float(momentum),
                                               _ptr(gamma.detach().contiguous()), _ptr(beta.detach().contiguous()),
                                               _ptr(running_mean), _ptr(running_var), _ptr(mean), _ptr(rstd), _ptr(scale),
                                               _ptr(shift), _ptr(ws), _stream(z))
    _check(rc, "bev_batchnorm_train_fwd_f32")
    return mean, rstd, scale, shift


def batchnorm_apply(z: torch.Tensor, scale, shift, residual=None, act: int = 0) -> torch.Tensor:
    """y = act(z * scale + shift (+ residual)), act 0 none / 1 ReLU / 2 SiLU (ACT_*)."""
    _require_gpu(z, scale, shift, residual)
    assert z.is_contiguous()
    if residual is not None:
        residual = residual.contiguous()
        assert residual.shape == z.shape
    C = z.shape[-1]
    y = torch.empty_like(z)
    _check(lib().bev_batchnorm_apply_f32(_ptr(z), z.numel() // C, C, _ptr(scale), _ptr(shift), _ptr(residual),
                                         int(act), _ptr(y), _stream(z)), "bev_batchnorm_apply_f32")
    return y


def batchnorm_bwd(dy: torch.Tensor, y, z: torch.Tensor, mean, rstd, gamma, want_dres: bool, act: int = 1,
                  scale=None, shift=None, frozen: bool = False):
    """-> (dz, dres or None, dgamma, dbeta) of y = act(batchnorm(z) (+ res)).  act 1 needs the forward output y,
    act 2 (SiLU) and 3 (ReLU without residual, mask from z) the forward's scale / shift; frozen: running statistics
    (no batch-statistic terms)."""
    dy = dy.contiguous()
    _require_gpu(dy, y, z, mean, rstd, gamma, scale, shift)
    C = z.shape[-1]
    M = z.numel() // C
    dz = torch.empty_like(z)
    dres = torch.empty_like(z) if want_dres else None
    dg = torch.empty(C, device=z.device)
    db = torch.empty(C, device=z.device)
    ws = _bn_workspace(M, C, z.device)
    _check(lib().bev_batchnorm_bwd_f32(_ptr(dy), _ptr(y), _ptr(z), M, C, _ptr(mean), _ptr(rstd),
                                       _ptr(gamma.detach().contiguous()), _ptr(scale), _ptr(shift), int(act),
                                       int(frozen), _ptr(dz), _ptr(dres), _ptr(dg), _ptr(db), _ptr(ws), _stream(z)),
           "bev_batchnorm_bwd_f32")
    return dz, dres, dg, db


# ---------------------------------------------------------------------------
# SqueezeExcite / depthwise training helpers (EfficientNet trunk)
# ---------------------------------------------------------------------------
def channel_sums(x: torch.Tensor, x2: torch.Tensor = None) -> torch.Tensor:
    """x (and x2) [N, H, W, C] NHWC -> [N, C] per-image channel sums of x (* x2)."""
    x = x.contiguous()
    x2 = x2.contiguous() if x2 is not None else None
    _require_gpu(x, x2)
    N, C = x.shape[0], x.shape[-1]
    P = x.numel() // (N * C)
    nbytes = lib().bev_channel_sums_workspace_bytes(N, P, C)
    if nbytes < 0:
        raise HipError(f"channel_sums shape not supported: {tuple(x.shape)}")
    ws = torch.empty((nbytes + 7) // 8, device=x.device, dtype=torch.float64)
    out = torch.empty(N, C, device=x.device)
    _check(lib().bev_channel_sums_f32(_ptr(x), _ptr(x2), N, P, C, _ptr(out), _ptr(ws), _stream(x)),
           "bev_channel_sums_f32")
    return out


def channel_affine(x: torch.Tensor, a: torch.Tensor, b: torch.Tensor = None) -> torch.Tensor:
    """y[n, ..., c] = x[n, ..., c] * a[n, c] (+ b[n, c]) for NHWC x, out of place."""
    x = x.contiguous()
    a = a.contiguous()
    b = b.contiguous() if b is not None else None
    _require_gpu(x, a, b)
    N, C = x.shape[0], x.shape[-1]
    y = torch.empty_like(x)
    _check(lib().bev_channel_affine_f32(_ptr(x), N, x.numel() // (N * C), C, _ptr(a), _ptr(b), _ptr(y), _stream(x)),
           "bev_channel_affine_f32")
    return y


def dwconv_wgrad(x: torch.Tensor, dz: torch.Tensor, K: int, stride: int, pad: int) -> torch.Tensor:
    """Depthwise weight gradient: x [N,H,W,C], dz [N,Ho,Wo,C] -> dW [K*K, C] (tap-major)."""
    x, dz = x.contiguous(), dz.contiguous()
    _require_gpu(x, dz)
    N, H, W, C = x.shape
    _, Ho, Wo, _ = dz.shape
    dW = torch.empty(K * K, C, device=x.device)
    _check(lib().bev_dwconv_wgrad_f32(_ptr(x), N, H, W, C, _ptr(dz), Ho, Wo, K, stride, pad, _ptr(dW), _stream(x)),
           "bev_dwconv_wgrad_f32")
    return dW


def image_normalize_u8(src: torch.Tensor, mean, std, out: torch.Tensor = None) -> torch.Tensor:
    """[N, H, W, 3] uint8 RGB on the GPU -> [N, 3, H, W] fp32 (ToTensor + Normalize, bit-exact)."""
    if not src.is_cuda:
        raise HipError("image_normalize_u8 needs a ROCm device tensor (got a CPU tensor); no CPU fallback")
    if src.dtype != torch.uint8 or src.dim() != 4 or src.shape[3] != 3:
        raise ValueError(f"image_normalize_u8 expects [N, H, W, 3] uint8, got {tuple(src.shape)} {src.dtype}")
    src = src.contiguous()
    N, H, W, _ = src.shape
    if out is None:
        out = torch.empty(N, 3, H, W, device=src.device, dtype=torch.float32)
    m = (ctypes.c_float * 3)(*[float(v) for v in mean])
    s = (ctypes.c_float * 3)(*[float(v) for v in std])
    _check(lib().bev_image_normalize_u8_f32(_ptr(src), N, H, W, m, s, _ptr(out), _stream(src)),
           "bev_image_normalize_u8_f32")
    return out
