"""ctypes binding of the C-ABI in include/ducosy_hip.h (lib/libducosy_hip.so).

The product path has no fallback: if the library is missing, importing the ops raises.
Build it with ``make -C ducosy-gan_amd`` (or ``python -c "import __graft_entry__ as g; g.build()"``).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_float, c_int, c_int32, c_int64, c_size_t, c_void_p, c_char_p

PKG_ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
LIB_PATH = os.environ.get("DUCOSY_HIP_LIB", os.path.join(PKG_ROOT, "lib", "libducosy_hip.so"))

DCS_PAD_ZERO, DCS_PAD_REFLECT = 0, 1
ACT_NONE, ACT_AFFINE, ACT_RELU, ACT_LRELU, ACT_TANH = 0, 1, 2, 3, 4
MMA_F32, MMA_BF16, MMA_BF16X3, MMA_BF16X6, MMA_F16X3, MMA_F16 = 0, 1, 3, 6, 7, 8
RANGE_PARTS = 512  # DCS_RANGE_PARTS: partial maxima of an f16x3 operand's range record
KORDER_TAP, KORDER_SLICE, PACK_KSLICE = 0, 1, 8


class ConvDesc(ctypes.Structure):
    """Mirror of dcs_conv_desc (include/ducosy_hip.h)."""
    _fields_ = [
        ("N", c_int32), ("Hs", c_int32), ("Ws", c_int32), ("Cs", c_int32),
        ("s_n", c_int64), ("s_c", c_int64), ("s_h", c_int64), ("s_w", c_int64),
        ("csplit", c_int32), ("cw", c_int32),
        ("s2_n", c_int64), ("s2_c", c_int64), ("s2_h", c_int64), ("s2_w", c_int64),
        ("up", c_int32), ("pad_mode", c_int32),
        ("KH", c_int32), ("KW", c_int32), ("pt", c_int32), ("pl", c_int32),
        ("stride", c_int32), ("parity", c_int32),
        ("Ho", c_int32), ("Wo", c_int32), ("Co", c_int32),
        ("ldb", c_int32), ("pro_act", c_int32), ("epi_act", c_int32), ("mma", c_int32),
        ("korder", c_int32),
        ("rng_a_n", c_int32), ("rng_b_n", c_int32), ("rng_a", c_void_p), ("rng_b", c_void_p),
        ("b_h3", c_void_p),
    ]


class PackJob(ctypes.Structure):
    """Mirror of dcs_pack_job (include/ducosy_hip.h): one weight pack of dcs_pack_batch."""
    _fields_ = [
        ("w", c_void_p),
        ("Cout", c_int32), ("Cin", c_int32), ("KH", c_int32), ("KW", c_int32), ("kind", c_int32),
        ("ci_count", c_int32), ("Kpad", c_int32), ("ncols", c_int32), ("nmajor", c_int32), ("h3", c_int32),
        ("h3_flip", c_int32), ("h3_ncols", c_int32),
        ("out", c_void_p), ("rng", c_void_p), ("planes", c_void_p), ("h3_hi", c_void_p), ("h3_lo", c_void_p),
        ("h3_wexp", c_void_p), ("h3_scratch", c_void_p),
        ("b0", c_int32), ("b1", c_int32), ("p0", c_int32), ("p1", c_int32),
    ]


class GLJob(ctypes.Structure):
    """Mirror of dcs_gl_job (include/ducosy_hip.h): one plane set of the fused G-step loss kernel."""
    _fields_ = [
        ("pred", c_void_p), ("target", c_void_p), ("source", c_void_p), ("add0", c_void_p), ("add1", c_void_p),
        ("grad", c_void_p), ("n_img", c_int32), ("H", c_int32), ("W", c_int32), ("flags", c_int32),
        ("c_l1", c_float), ("c_grad", c_float), ("c_ssim", c_float), ("c_ca", c_float), ("c_mse", c_float),
        ("t_const", c_float), ("c_add0", c_float), ("c_add1", c_float),
    ]


GL_L1, GL_GRAD, GL_SSIM, GL_CA, GL_MSEC = 1, 2, 4, 8, 16

P = c_void_p
DP = POINTER(ConvDesc)

# name -> (restype, argtypes)
SIGNATURES = {
    "dcs_last_error": (c_char_p, []),
    "dcs_version": (c_int, []),
    "dcs_pack_weights": (c_int, [P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, P]),
    "dcs_pack_weights_r": (c_int, [P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, P, P]),
    "dcs_range_parts": (c_int, [P, c_int, c_int64, c_int, P, P, c_int, P, P]),
    "dcs_pack_weights_h3_scratch_size": (c_size_t, []),
    "dcs_pack_weights_h3": (c_int, [P, c_int, c_int, c_int, c_int, P, P, P, P, P]),
    "dcs_conv3_win_ok": (c_int, [DP, c_int]),
    "dcs_conv3_win_in_stats": (c_int, [DP, P, P, P, P, P, P, c_size_t, P, P]),
    "dcs_pack_split_h3": (c_int, [P, c_int, c_int, P, c_int, P, P]),
    "dcs_pack_plan": (c_int, [P, c_int, POINTER(c_int), POINTER(c_int)]),
    "dcs_pack_subpix_h3": (c_int, [P, c_int, c_int, c_int, P, P, P, P, P]),
    "dcs_subpix_win_dgrad_ok": (c_int, [DP]),
    "dcs_subpix_win_dgrad": (c_int, [DP, P, P, P, P, P, P]),
    "dcs_phase_win_dgrad_inbwd_parts_size": (c_size_t, [DP, c_int]),
    "dcs_phase_win_dgrad_inbwd": (c_int, [DP, c_int, P, P, P, P, P, P, P, P, c_int, P, c_size_t, POINTER(c_int), P]),
    "dcs_stride2_win_ok": (c_int, [DP]),
    "dcs_stride2_win_parts_size": (c_size_t, [DP]),
    "dcs_stride2_win": (c_int, [DP, P, P, P, P, P, P, P, P, c_size_t, POINTER(c_int), P]),
    "dcs_subpix_win_ok": (c_int, [DP]),
    "dcs_subpix_win_parts_size": (c_size_t, [DP]),
    "dcs_subpix_win": (c_int, [DP, P, P, P, P, P, P, c_size_t, POINTER(c_int), P]),
    "dcs_pack_batch": (c_int, [P, c_int, c_int, c_int, P]),
    "dcs_stem_fwd_ok": (c_int, [DP]),
    "dcs_stem_fwd_parts_size": (c_size_t, [DP]),
    "dcs_stem_fwd": (c_int, [DP, P, P, P, P, c_size_t, POINTER(c_int), P]),
    "dcs_stem_wgrad_ok": (c_int, [DP]),
    "dcs_stem_wgrad_workspace_size": (c_size_t, [DP]),
    "dcs_stem_wgrad": (c_int, [DP, P, P, P, P, c_size_t, P]),
    "dcs_head_fwd_proj_ok": (c_int, [DP]),
    "dcs_head_fwd_proj": (c_int, [DP, P, P, P, P, P, P, P, P]),
    "dcs_head_wgrad_proj_workspace_size": (c_size_t, [DP]),
    "dcs_head_wgrad_proj": (c_int, [DP, P, P, P, P, P, P, P, c_size_t, P]),
    "dcs_head_dgrad_in_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "dcs_head_dgrad_in": (c_int, [P, P, c_int, P, c_int, c_int, c_int, P, P, P, c_int, c_int, P, P, c_size_t, P, P]),
    "dcs_conv_dgrad_reflect_win": (c_int, [DP, P, P, P, P, P, P, P, P, P]),
    "dcs_conv_dgrad_reflect_win_inbwd_parts_size": (c_size_t, [DP]),
    "dcs_conv_dgrad_reflect_win_inbwd": (c_int, [DP, P, P, P, P, P, P, P, P, P, P, c_int, P, c_size_t, P, P]),
    "dcs_conv_rows": (c_int, [DP, P, P, P, P, P, P, P, P]),
    "dcs_conv_rows_in_stats_parts_size": (c_size_t, [DP]),
    "dcs_conv_rows_in_stats": (c_int, [DP, P, P, P, P, P, P, P, P, c_size_t, P, P]),
    "dcs_in_stats_finish": (c_int, [P, c_int, c_int, c_int, c_float, P, P, P, P, P]),
    "dcs_conv_dgrad_c1": (c_int, [P, c_int, c_int, c_int, P, c_int, c_int, c_int, c_int, P, P]),
    "dcs_conv_dgrad_to1_workspace_size": (c_size_t, [c_int, c_int, c_int, c_int]),
    "dcs_conv_dgrad_to1": (c_int, [P, c_int, c_int, c_int, c_int, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                   P, P, c_size_t, P]),
    "dcs_conv_wgrad_workspace_size": (c_size_t, [DP]),
    "dcs_conv_wgrad": (c_int, [DP, P, P, P, P, P, P, P, c_size_t, P]),
    "dcs_conv_dgrad_reflect_ring_size": (c_size_t, [P]),
    "dcs_conv_dgrad_reflect": (c_int, [P, P, P, P, P, P, P]),
    "dcs_reflect_fold": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, P]),
    "dcs_pack_nhwc4": (c_int, [P, c_int, P, c_int, c_int, c_int, c_int, P, P, P]),
    "dcs_upsample2_grad": (c_int, [P, P, c_int, c_int, c_int, c_int, P]),
    "dcs_in_stats_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "dcs_in_stats": (c_int, [P, c_int, c_int, c_int, c_float, P, P, P, P, P, c_size_t, P]),
    "dcs_in_apply": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, P, P]),
    "dcs_in_act_backward": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_int, P, c_size_t, P, P]),
    "dcs_in_act_backward_parts": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_int, P, c_int, P, c_size_t, P, P]),
    "dcs_conv_rows_narrow": (c_int, [DP, P, P, P, P, P, P, P, P]),
    "dcs_conv_wgrad_narrow_workspace_size": (c_size_t, [DP]),
    "dcs_conv_wgrad_narrow": (c_int, [DP, P, P, P, P, P, P, P, c_size_t, P]),
    "dcs_cbam_forward": (c_int, [P, P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int,
                                 P, P, P, P, P, P, P]),
    "dcs_cbam_backward_workspace_size": (c_size_t, [c_int, c_int, c_int, c_int, c_int, c_int]),
    "dcs_cbam_backward": (c_int, [P, P, P, P, P, P, P, P, P, P, P, P, P, c_int, c_int, c_int, c_int,
                                  c_int, c_int, P, P, P, P, P, c_size_t, P, P]),
    "dcs_loss_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "dcs_gen_loss_fused_ws": (c_size_t, [P, c_int]),
    "dcs_gen_loss_fused": (c_int, [P, c_int, c_float, c_float, c_float, c_float, P, P, P, P, c_int, P, P, c_size_t, P]),
    "dcs_multi_add": (c_int, [c_int, P, P, P, P]),
    "dcs_range_arena_register": (c_int, [P, c_size_t]),
    "dcs_range_arena_unregister": (c_int, [P]),
    "dcs_loss_l1": (c_int, [P, P, c_int64, P, P, P, c_size_t, P]),
    "dcs_loss_mse": (c_int, [P, P, c_int64, P, P, P, c_size_t, P]),
    "dcs_loss_mse_const": (c_int, [P, c_float, c_int64, P, P, P, c_size_t, P]),
    "dcs_loss_gradient": (c_int, [P, P, c_int, c_int, c_int, P, P, P, c_size_t, P]),
    "dcs_loss_contrast_attention": (c_int, [P, P, P, c_int, c_int, c_int, c_float, c_float, c_float,
                                            c_int, P, P, P, c_size_t, P]),
    "dcs_loss_contrast_region": (c_int, [P, P, P, c_int, c_int, c_int, c_float, c_float, P, P, P,
                                         c_size_t, P]),
    "dcs_loss_contrast_edge": (c_int, [P, P, c_int, c_int, c_int, P, P, P, c_size_t, P]),
    "dcs_loss_contrast_region_partial": (c_int, [P, P, P, c_int, c_int, c_int, c_float, P, P, c_size_t, P]),
    "dcs_loss_contrast_region_finish": (c_int, [P, c_int, c_int, c_int, c_float, P, c_float, P, P, P, c_size_t, P]),
    "dcs_loss_contrast_edge_partial": (c_int, [P, P, c_int, c_int, c_int, P, P, c_size_t, P]),
    "dcs_loss_contrast_edge_hist": (c_int, [c_int, c_int, c_int, c_int, P, P, P, c_size_t, P]),
    "dcs_loss_contrast_edge_select": (c_int, [c_int, P, P, c_size_t, P]),
    "dcs_loss_contrast_edge_topk": (c_int, [c_int, c_int, c_int, P, P, c_size_t, P]),
    "dcs_loss_contrast_edge_finish": (c_int, [P, c_int, c_int, c_int, P, c_float, P, P, P, c_size_t, P]),
    "dcs_loss_ssim": (c_int, [P, P, c_int, c_int, c_int, c_float, c_int, c_float, c_float, c_float,
                              P, P, P, c_size_t, P]),
    "dcs_adam_step": (c_int, [P, P, P, P, c_int64, c_float, c_float, c_float, c_float, c_float,
                              c_float, P]),
    "dcs_scale_add": (c_int, [P, P, c_float, c_int64, P]),
    "dcs_scale_dev": (c_int, [P, P, P, c_int64, P]),
    "dcs_act_backward": (c_int, [P, P, P, c_int64, c_int, P, P]),
    "dcs_channel_sum_workspace_size": (c_size_t, [c_int64, c_int]),
    "dcs_channel_sum": (c_int, [P, c_int64, c_int, P, P, c_size_t, P]),
    "dcs_hu_transform": (c_int, [P, c_int, P, P, c_int, c_int, c_int, c_float, c_float, c_int, c_float,
                                 P, P, P]),
    "dcs_masks_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "dcs_anatomical_masks": (c_int, [P, P, c_int, c_int, c_int, P, P, P, c_int, P, P, c_size_t, P]),
}


class HipLibraryError(RuntimeError):
    pass


_lib = None


def load() -> ctypes.CDLL:
    """Load the kernel library (once).  Raises loudly when it is missing: no CPU fallback."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.isfile(LIB_PATH):
        raise HipLibraryError(
            f"HIP kernel library not found at {LIB_PATH}; build it with `make -C {PKG_ROOT}`")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def exported_symbols():
    return sorted(SIGNATURES)


_SYNC_CHECK = os.environ.get("DUCOSY_SYNC_CHECK", "0") == "1"


def call(name: str, *args) -> None:
    """Call an int-returning entry point and raise on a non-zero status.  With
    DUCOSY_SYNC_CHECK=1 every call is followed by a device synchronisation so an
    asynchronous fault is attributed to the entry point that launched it (debug only)."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.dcs_last_error()
        raise HipLibraryError(f"{name} failed (status {rc}): {msg.decode() if msg else ''}")
    if _SYNC_CHECK:
        import torch
        try:
            torch.cuda.synchronize()
        except Exception as e:  # pragma: no cover - debug path
            raise HipLibraryError(f"device fault after {name}: {e}") from e


def query(name: str, *args) -> int:
    return int(getattr(load(), name)(*args))
