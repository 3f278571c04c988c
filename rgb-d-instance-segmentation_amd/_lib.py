"""ctypes binding of librgbd_hip.so (the C ABI declared in include/rgbd_hip.h).

There is no fallback: if the library is missing or fails to load, every op raises.
``import torch`` happens first so that torch's HIP runtime (soname libamdhip64.so.7) is the
one the library binds to — one HIP runtime per process.
"""
import ctypes
import os
from pathlib import Path

import numpy as np

# RGBD_HIP_LIB overrides the in-tree library (A/B timing of two builds on one box)
LIB_PATH = Path(os.environ.get("RGBD_HIP_LIB", Path(__file__).resolve().parent / "librgbd_hip.so"))

RGBD_F32 = 0
RGBD_BF16 = 1
NBINS = 512

# rgbd_decomp_info (include/rgbd_hip.h) as a numpy structured dtype: 2116 bytes, no padding
DECOMP_INFO_DTYPE = np.dtype([
    ("status", "<i4"), ("n_modes", "<i4"), ("n_masks", "<i4"), ("peak_bin", "<i4", 3),
    ("first_edge", "<f4"), ("last_edge", "<f4"), ("center", "<f4", 3),
    ("lo", "<f4", 3), ("hi", "<f4", 3), ("hist", "<i4", NBINS)])
assert DECOMP_INFO_DTYPE.itemsize == 2116

_P = ctypes.c_void_p
_I = ctypes.c_int
_LL = ctypes.c_longlong
_SZ = ctypes.c_size_t

# name -> (restype, argtypes); must list every symbol the header declares
SIGNATURES = {
    "rgbd_version": (ctypes.c_char_p, []),
    "rgbd_assemble_workspace_size": (_SZ, [_I]),
    "rgbd_assemble_pixel_values": (_I, [_P, _P, _I, _I, _I, _P, _P, _P]),
    "rgbd_instance_presence": (_I, [_P, _I, _I, _I, _P, _P]),
    "rgbd_instance_masks": (_I, [_P, _I, _I, _P, _P, _I, _P, _P]),
    "rgbd_pp_instance_workspace_size": (_SZ, [_I, _I]),
    "rgbd_pp_instance": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P, ctypes.c_double, _P, _P, _P, _P, _P, _P]),
    "rgbd_pp_binary_maps": (_I, [_P, _I, _I, _I, _I, _I, _P, _P, _P]),
    "rgbd_pack_mask_bits": (_I, [_P, _I, _LL, _P, _P, _P]),
    "rgbd_mask_intersections": (_I, [_P, _I, _P, _I, _LL, _P, _P]),
    "rgbd_resize_workspace_size": (_SZ, [_I, _I, _I, _I, _I, _I]),
    "rgbd_resize_pil_bilinear": (_I, [_P, _I, _I, _I, _I, _I, _I, _P, _P, _P]),
    "rgbd_resize_pil_nearest": (_I, [_P, _I, _I, _I, _I, _I, _I, _P, _P, _P]),
    "rgbd_resize_cv2_linear": (_I, [_P, _I, _I, _I, _I, _I, _P, _P, _P]),
    "rgbd_edsam_decompose_workspace_size": (_SZ, [_I]),
    "rgbd_edsam_decompose": (_I, [_P, _LL, _I, _I, _I, _I, _P, _I, _P, _P, _P, _P, _P, _P]),
    "rgbd_edsam_decompose_masks": (_I, [_P, _LL, _I, _I, _I, _I, _P, _I, _P, _P, _P, _P, _P, _P, _P]),
    "rgbd_edsam_modes_workspace_size": (_SZ, [_I, _I, _I]),
    "rgbd_edsam_modes": (_I, [_P, _LL, _I, _I, _I, _I, _P, _P, _I, _P, _P]),
    "rgbd_edsam_codes": (_I, [_P, _I, _I, _I, _P, _I, _P, _P, _P, _P, _P, _P]),
    "rgbd_dggm_fuse_fwd": (_I, [_I, _P, _P, _P, _P, _LL, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P]),
    "rgbd_dggm_fuse_bwd_workspace_size": (_SZ, [_I, _I, _I, _I]),
    "rgbd_dggm_fuse_bwd": (_I, [_I, _P, _P, _P, _LL, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P]),
    "rgbd_dggm_fuse_fwd_multi": (_I, [_I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _LL, _I, _I, _I, _P]),
    "rgbd_dggm_fuse_fwd_multi_mixed": (_I, [_I, _I, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _LL, _I, _I, _I,
                                            _P]),
    "rgbd_dggm_fuse_bwd_multi_workspace_size": (_SZ, [_I, _P, _P, _P, _I]),
    "rgbd_dggm_fuse_bwd_multi": (_I, [_I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _LL, _I, _I, _I, _P, _P]),
    "rgbd_nchw_to_nhwc": (_I, [_I, _P, _P, _I, _I, _I, _I, _P]),
    "rgbd_nchw_to_nhwc_multi": (_I, [_I, _P, _P]),
    "rgbd_adamw_multi": (_I, [_I, _P, _P, _P, _P, _P, _P, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                             ctypes.c_double, ctypes.c_double, _P]),
    "rgbd_adamw_multi_shadow": (_I, [_I, _P, _P, _P, _P, _P, _P, _P, ctypes.c_double, ctypes.c_double,
                                     ctypes.c_double, ctypes.c_double, ctypes.c_double, _P]),
    "rgbd_dsam_packed_elems": (_LL, [_I, _I, _I]),
    "rgbd_dsam_pack_weights": (_I, [_I, _P, _P, _I, _I, _P, _P, _P, _P]),
    "rgbd_dsam_code_masks": (_I, [_I, _P, _P, _P, _P]),
    "rgbd_dsam_conv_workspace_size": (_SZ, [_I, _I, _I, _I, _I, _I]),
    "rgbd_dsam_fwd": (_I, [_I, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P]),
    "rgbd_dsam_fwd_nhwc": (_I, [_I, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P]),
    "rgbd_dsam_bwd_data": (_I, [_I, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P]),
    "rgbd_dsam_bwd_weight_workspace_size": (_SZ, [_I, _I, _I, _I, _I, _I]),
    "rgbd_dsam_bwd_weight": (_I, [_I, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P]),
    "rgbd_dsam_plan_size": (_SZ, [_I, _I, _I, _I, _I, _I]),
    "rgbd_dsam_run_workspace_size": (_SZ, [_I, _I, _I, _I, _I, _I]),
    "rgbd_dsam_plan": (_I, [_I, _P, _P]),
    "rgbd_dsam_fwd_nhwc_planned": (_I, [_I, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P]),
    "rgbd_dsam_bwd_data_planned": (_I, [_I, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "rgbd_dsam_bwd_weight_planned": (_I, [_I, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P]),
    "rgbd_dsam_bwd_weight_planned_multi": (_I, [_I, _P, _P, _P]),
    "rgbd_point_sample": (_I, [_P, _I, _I, _I, _P, _I, _I, _P, _P]),
    "rgbd_point_sample_t": (_I, [_I, _P, _I, _I, _I, _P, _I, _I, _P, _P]),
    "rgbd_point_sample_sets": (_I, [_I, _P, _I, _I, _I, _P, _P, _I, _P, _P]),
    "rgbd_topk_rows_max_n": (_SZ, []),
    "rgbd_topk_rows": (_I, [_P, _I, _I, _I, _P, _P]),
    "rgbd_point_sample_bwd": (_I, [_P, _I, _I, _I, _P, _I, _I, _P, _P]),
    "rgbd_match_cost": (_I, [_P, _I, _I, _I, _P, _P, _P, _P, ctypes.c_float, ctypes.c_float, ctypes.c_float, _P, _P]),
    "rgbd_match_cost_probs": (_I, [_P, _I, _I, _I, _P, _P, _P, _I, _P, _P, ctypes.c_float, ctypes.c_float,
                                   ctypes.c_float, _P, _P]),
    "rgbd_point_losses": (_I, [_P, _P, _I, _I, _P, _P, _P, _P]),
    "rgbd_point_losses_bwd": (_I, [_P, _P, _I, _I, _P, _P, _P, _P, _P]),
    "rgbd_msda_fwd": (_I, [_I, _P, _I, _I, _P, _I, _I, _I, _I, _P, _P, _P, _P]),
    "rgbd_msda_bwd": (_I, [_I, _P, _I, _I, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P]),
    "rgbd_level_memory_workspace_size": (_SZ, [_I, _I, _I]),
    "rgbd_level_memory_fwd": (_I, [_I, _P, _P, _I, _I, _I, _P, _P]),
    "rgbd_level_memory_bwd": (_I, [_I, _P, _I, _I, _I, _P, _P, _P, _P]),
    "rgbd_msda_locations": (_I, [_I, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P]),
    "rgbd_msda_locations_bwd": (_I, [_I, _P, _P, _I, _I, _I, _I, _I, _P, _P]),
    "rgbd_lsa_lds_bytes": (_SZ, [_I, _I]),
    "rgbd_lsa_batch": (_I, [_I, _P, _P, _I, _I, _P, _P, _P, _P]),
    "rgbd_mask_logits": (_I, [_I, _P, _P, _I, _I, _I, _I, _I, _P, _P]),
    "rgbd_mask_attention": (_I, [_I, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P]),
    "rgbd_masked_attn_fwd_workspace_size": (_SZ, [_I, _I, _I]),
    "rgbd_masked_attn_fwd": (_I, [_I, _P, _P, _P, _P, _I, _I, _I, _I, ctypes.c_float, _P, _P, _P, _P]),
    "rgbd_masked_attn_bwd_workspace_size": (_SZ, [_I, _I, _I]),
    "rgbd_masked_attn_bwd": (_I, [_I, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, ctypes.c_float, _P, _P, _P, _P,
                                  _P]),
    "rgbd_gemm_workspace_size": (_SZ, [_I, _I, _I, _I]),
    "rgbd_gemm": (_I, [_I, _I, _I, _I, _I, _I, _P, _LL, _LL, _P, _LL, _LL, _P, _I, _P, _LL, _LL, _P, _LL, _LL, _I,
                       _I, _I, _P, _P]),
    "rgbd_im2col": (_I, [_I, _P, _I, _I, _I, _I, _I, _P, _P]),
    "rgbd_colsum_workspace_size": (_SZ, [_I, _I]),
    "rgbd_colsum": (_I, [_I, _P, _I, _I, _LL, _P, _P, _P]),
    "rgbd_layernorm_fwd": (_I, [_I, _P, _P, _P, _I, _I, ctypes.c_float, _I, _P, _P, _P, _P]),
    "rgbd_add_layernorm_fwd": (_I, [_I, _P, _I, _P, _P, _P, _I, _I, ctypes.c_float, ctypes.c_float, _I, _P, _P, _P,
                                    _P, _P, _P]),
    "rgbd_add_layernorm_bwd": (_I, [_I, _P, _I, _P, _P, _P, _P, _P, _I, _I, ctypes.c_float, _P, _P, _P, _P, _P,
                                    _P]),
    "rgbd_layernorm_bwd_workspace_size": (_SZ, [_I, _I]),
    "rgbd_layernorm_bwd": (_I, [_I, _P, _I, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P]),
    "rgbd_groupnorm_workspace_size": (_SZ, [_I, _I]),
    "rgbd_groupnorm_fwd": (_I, [_I, _P, _P, _P, _I, _I, _I, _I, ctypes.c_float, _I, _I, _P, _P, _P, _P]),
    "rgbd_groupnorm_bwd": (_I, [_I, _P, _I, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P]),
    "rgbd_swin_window_attn": (_I, [_I, _P, _P, _P, _LL, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, ctypes.c_float, _P,
                                   _LL, _P]),
    "rgbd_timing_enable": (_I, [_I]),
    "rgbd_timing_read": (ctypes.c_double, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]),
    "rgbd_ratio_packed_size": (_SZ, [_I]),
    "rgbd_ratio_pack": (_I, [_I, _P, _P, _P]),
    "rgbd_ratio_workspace_size": (_SZ, [_I, _I, _I, _I]),
    "rgbd_ratio_features_offset": (_SZ, [_I, _I, _I, _I]),
    "rgbd_ratio_pooled_offset": (_SZ, [_I, _I, _I, _I]),
    "rgbd_ratio_forward": (_I, [_I, _I, ctypes.c_float, _P, _LL, _I, _I, _I, _P, _P, ctypes.c_ulonglong, _P, _P,
                                _P, _P]),
    "rgbd_ratio_forward_ex": (_I, [_I, _I, ctypes.c_float, _P, _LL, _I, _I, _I, _P, _P, ctypes.c_ulonglong, _P, _P,
                                   _P, _I, _P]),
}

# the diagnostic build's extra entry points (include/rgbd_hip_diag.h; librgbd_hip_diag.so via
# RGBD_HIP_LIB), bound only when the loaded library exports them
DIAG_SIGNATURES = {
    "rgbd_debug_conv5_stamps": (_I, [_P]),
    "rgbd_debug_chain_stamps": (_I, [_P]),
    "rgbd_debug_dsam_stamps": (_I, [_P, _I]),
    "rgbd_debug_stem_lag_stamps": (_I, [_P]),
    "rgbd_debug_conv5_mode": (_I, [_I]),
    "rgbd_debug_dsam_mode": (_I, [_I]),
}

_lib = None


class RgbdHipError(RuntimeError):
    pass


def lib():
    """Load (once) and return the CDLL with argtypes set.  Raises if unavailable."""
    global _lib
    if _lib is None:
        import torch  # noqa: F401  (bind to torch's HIP runtime)
        if not LIB_PATH.exists():
            raise RgbdHipError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(there is no CPU fallback for the rgbd_amd kernels)")
        h = ctypes.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        for name, (res, args) in DIAG_SIGNATURES.items():
            if hasattr(h, name):
                fn = getattr(h, name)
                fn.restype = res
                fn.argtypes = args
        _lib = h
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        kind = {-1: "bad argument", -2: "unsupported shape", -3: "unsupported dtype"}.get(rc, "HIP error")
        raise RgbdHipError(f"{what} failed: {kind} (code {rc})")


def header_symbols():
    """Function names declared in include/rgbd_hip.h (parsed, for the export test)."""
    import re
    hdr = Path(__file__).resolve().parents[1] / "include" / "rgbd_hip.h"
    txt = hdr.read_text()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?(?:\w+\*?\s+)+\*?(rgbd_\w+)\s*\(", txt, flags=re.M)))
