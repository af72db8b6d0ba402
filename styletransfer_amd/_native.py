"""ctypes binding of libstx.so (the C-ABI declared in include/stx.h).

The product path has no fallback: if the library is missing or fails to load,
`lib()` raises, and every op that needs it fails loudly.  `lib()` is lazy so
that host-only code (argument checking, state_dict handling) imports on a
machine without a GPU.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("STX_LIB", os.path.join(_HERE, "libstx.so"))

STX_IN_RAW, STX_IN_RELU, STX_IN_RELU_POOL2, STX_IN_UPSAMPLE2, STX_IN_DILATE2 = range(5)
STX_AMAX_SLOTS = 32  # an "amax" is a group of 32 floats whose max is the value (stx.h)
STX_GRAM_GROUP = 8  # fused Gram partials per in-kernel group sum (stx_conv_params.gram_cnt)
STX_ABI_VERSION = 7  # include/stx.h: the library must report the same revision


def knob(name: str, default: str) -> str:
    """A measurement-only A/B switch of the Python host path: read from the environment
    only when STX_AB=1 (tools/ab_engine.py and the other same-box A/B scripts), otherwise
    the product default -- the product path is environment-independent, like the
    library's compile-time STX_KNOBs (common.h; only `make AB=1` builds read those)."""
    if os.environ.get("STX_AB") != "1":
        return default
    return os.environ.get(name, default)

vp = C.c_void_p
i32 = C.c_int
i64 = C.c_longlong
f32 = C.c_float
sz = C.c_size_t


class ConvParams(C.Structure):
    """Mirror of `stx_conv_params` (include/stx.h)."""
    _fields_ = [
        ("x", vp), ("wt", vp), ("bias", vp), ("y", vp), ("mask", vp), ("aux", vp),
        ("aux_scale", f32), ("acc_scale", vp), ("accumulate", i32), ("relu_out", i32),
        ("n", i32), ("cin", i32), ("h", i32), ("w", i32),
        ("cout", i32), ("ks", i32), ("stride", i32), ("pad", i32),
        ("in_mode", i32), ("hv", i32), ("wv", i32), ("ho", i32), ("wo", i32),
        ("cin_pad", i32), ("cout_pad", i32), ("wt_batch_stride", i64),
        ("p2_z", vp), ("p2_wt", vp), ("p2_scale", vp), ("p2_c", i32), ("p2_wt_batch_stride", i64),
        ("up_dp", vp), ("up_z", vp),
        ("wt16", vp), ("w_amax", vp), ("in_amax", vp), ("out_amax", vp),
        ("pool_out", vp), ("p2_amax", vp), ("gram_part", vp), ("pool_sum", i32),
        ("gram_cnt", vp), ("p2_wt_amax", vp), ("mse_ref", vp), ("mse_parts", vp),
        ("wt16_up", vp), ("unpool_out", i32),
    ]


class ImageMeta(C.Structure):
    """Mirror of `stx_image_meta` (include/stx.h)."""
    _fields_ = [("offset", i64), ("h", i32), ("w", i32), ("top", i32), ("left", i32),
                ("y0", i32), ("y1", i32), ("resize_w", i32), ("resize_h", i32),
                ("xcoef", i32), ("ycoef", i32), ("xk", i32), ("yk", i32), ("tmp_offset", i64)]


class WprepJob(C.Structure):
    """Mirror of `stx_wprep_job` (include/stx.h)."""
    _fields_ = [("w", vp), ("slab", vp), ("w_amax", vp), ("kind", i32), ("cout", i32),
                ("cin", i32), ("ks", i32), ("transpose", i32), ("pad_", i32)]


STX_WPREP_MAX, STX_WPREP_F32, STX_WPREP_F16, STX_WPREP_F16UP = 48, 0, 1, 2


class PGradJob(C.Structure):
    """Mirror of `stx_in_pgrad_job` (include/stx.h)."""
    _fields_ = [("parts", vp), ("dgamma", vp), ("dbeta", vp), ("dbias_in", vp), ("n", i32),
                ("c", i32), ("accumulate", i32), ("pad_", i32)]


STX_PGRAD_MAX = 32


class LossParts(C.Structure):
    """Mirror of `stx_loss_parts` (include/stx.h)."""
    _fields_ = [("parts", vp * 8), ("nparts", i32 * 8), ("inv", f32 * 8), ("k", i32)]


class GramFinJob(C.Structure):
    """Mirror of `stx_gram_fin_job` (include/stx.h)."""
    _fields_ = [("parts", vp), ("g_out", vp), ("target", vp), ("coef", vp), ("loss_parts", vp),
                ("mse_parts", vp), ("mse_out", vp), ("t_bstride", i64), ("mse_n", C.c_double),
                ("scale", f32), ("cA", f32), ("alpha", f32), ("c", i32), ("nsplit", i32),
                ("b", i32), ("cpad", i32), ("mse_nparts", i32), ("coef_amax", vp)]


STX_FIN_MAX = 8


# name -> (restype, argtypes); every symbol include/stx.h declares
SIGNATURES = {
    "stx_version": (i32, []),
    "stx_abi_layout": (i32, [vp, i32]),
    "stx_last_error_string": (C.c_char_p, []),
    "stx_abi_version": (i32, []),
    "stx_conv_weight_dims": (i32, [i32, i32, i32, C.POINTER(i32), C.POINTER(i32)]),
    "stx_conv_weight_prep": (i32, [vp, vp, i32, i32, i32, i32, vp]),
    "stx_conv2d": (i32, [C.POINTER(ConvParams), vp]),
    "stx_conv_gram_tiles": (i32, [C.POINTER(ConvParams)]),
    "stx_conv_gram_groups": (i32, [C.POINTER(ConvParams)]),
    "stx_conv_weight16_bytes": (sz, [i32, i32, i32, i32]),
    "stx_conv_weight_prep16": (i32, [vp, vp, vp, i32, i32, i32, i32, vp]),
    "stx_conv_weight_prep16_pair": (i32, [vp, vp, vp, vp, i32, i32, i32, vp]),
    "stx_conv_weight16up_bytes": (sz, [i32, i32]),
    "stx_conv_weight_prep16_up": (i32, [vp, vp, vp, i32, i32, vp]),
    "stx_conv_weight_compose16": (i32, [vp, i32, vp, vp, vp, i32, i32, vp, vp, vp, vp]),
    "stx_amax": (i32, [vp, i64, vp, vp]),
    "stx_conv_weight_prep_batch": (i32, [C.POINTER(WprepJob), i32, vp]),
    "stx_conv2d_wgrad_ws": (sz, [i32, i32, i32, i32, i32, i32, i32]),
    "stx_conv2d_wgrad": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32,
                               i32, i32, i32, i32, vp, sz, vp]),
    "stx_conv2d_wgrad16_ws": (sz, [i32, i32, i32, i32, i32, i32]),
    "stx_conv2d_wgrad16": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp,
                                 vp, sz, vp]),
    "stx_conv2d_wgrad16_s2_ws": (sz, [i32, i32, i32, i32, i32]),
    "stx_conv2d_wgrad16_s2": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp,
                                    vp, sz, vp]),
    "stx_conv2d_wgrad_few16_ws": (sz, [i32, i32, i32, i32, i32, i32]),
    "stx_conv2d_wgrad_few16": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp,
                                     vp, sz, vp]),
    "stx_vec_ws": (sz, []),
    "stx_vec_reduce": (i32, [vp, vp, i64, i32, vp, vp, vp, f32, vp, sz, vp]),
    "stx_vec_axpby": (i32, [vp, vp, i64, f32, vp, f32, f32, vp]),
    "stx_scalar_op": (i32, [vp, i32, i32, i32, i32, vp]),
    "stx_lbfgs_state_bytes": (sz, [i32]),
    "stx_lbfgs_hist_bytes": (sz, [i64, i32]),
    "stx_lbfgs_ws": (sz, [i64, i32]),
    "stx_lbfgs_direction": (i32, [vp, vp, vp, vp, i64, i32, f32, f32, vp, vp, vp, sz, vp]),
    "stx_lbfgs_grad_stats": (i32, [vp, i64, vp, vp, vp, i32, vp, sz, vp]),
    "stx_bias_grad_ws": (sz, [i32, i32]),
    "stx_bias_grad": (i32, [vp, vp, i32, i32, i32, i32, vp, sz, vp]),
    "stx_gram_ws": (sz, [i32, i32, i32]),
    "stx_gram": (i32, [vp, vp, i32, i32, i32, f32, vp, vp, sz, vp]),
    "stx_gram_coef_pitch": (i32, [i32]),
    "stx_style_loss": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, i32, f32, f32, vp, vp, sz,
                             vp]),
    "stx_style_loss_from_parts": (i32, [vp, i32, vp, vp, vp, vp, i32, i32, i32, i32, f32, f32,
                                        vp, sz, vp]),
    "stx_style_content_loss_from_parts": (i32, [vp, i32, vp, vp, vp, i32, i32, i32, i32, f32,
                                                f32, vp, vp, vp, sz, vp]),
    "stx_style_content_ws": (sz, [i32, i32, i32]),
    "stx_style_content_loss": (i32, [vp, vp, vp, vp, i32, i32, i32, i32, f32, f32, vp, vp, vp,
                                     vp, sz, vp]),
    "stx_style_loss_deferred": (i32, [vp, vp, vp, i32, i32, i32, i32, f32, f32, vp, vp, sz,
                                      C.POINTER(GramFinJob), vp]),
    "stx_style_content_loss_deferred": (i32, [vp, vp, vp, i32, i32, i32, i32, f32, f32, vp, vp,
                                              vp, vp, sz, C.POINTER(GramFinJob), vp]),
    "stx_style_loss_from_parts_deferred": (i32, [vp, i32, vp, vp, i32, i32, i32, i32, f32, f32,
                                                 vp, sz, C.POINTER(GramFinJob), vp]),
    "stx_style_content_loss_from_parts_deferred": (i32, [vp, i32, vp, vp, i32, i32, i32, i32,
                                                         f32, f32, vp, vp, vp, sz,
                                                         C.POINTER(GramFinJob), vp]),
    "stx_gram_finalize_batch": (i32, [C.POINTER(GramFinJob), i32, vp]),
    "stx_gram_bwd": (i32, [vp, vp, vp, i32, i32, i32, i32, vp, vp, vp, f32, i32, vp]),
    "stx_mse_ws": (sz, [i64]),
    "stx_mse": (i32, [vp, vp, i64, i32, i32, vp, vp, f32, vp, sz, vp]),
    "stx_diff_scale": (i32, [vp, vp, vp, i64, f32, vp, vp, i32, i32, vp]),
    "stx_loss_combine": (i32, [vp, i32, C.POINTER(f32), vp, vp]),
    "stx_style_loss_parts": (sz, [i32, i32, i32, C.POINTER(i32)]),
    "stx_loss_finalize": (i32, [C.POINTER(LossParts), vp, vp, i32, C.POINTER(f32), vp, vp]),
    "stx_maxpool2x2_fwd": (i32, [vp, vp, vp, i32, i32, i32, i32, vp]),
    "stx_maxpool2x2_bwd": (i32, [vp, vp, vp, i32, i32, i32, vp]),
    "stx_relupool_bwd": (i32, [vp, vp, vp, i32, i32, i32, vp]),
    "stx_relu_fwd": (i32, [vp, vp, i64, vp]),
    "stx_relu_bwd": (i32, [vp, vp, vp, i64, vp]),
    "stx_adam_ws": (sz, []),
    "stx_adam_step": (i32, [vp, vp, vp, vp, i64, f32, f32, f32, f32, vp, vp, vp]),
    "stx_adam_step_clear": (i32, [vp, vp, vp, vp, i64, f32, f32, f32, f32, vp, vp, vp, i32, vp]),
    "stx_instnorm_fwd": (i32, [vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, f32, i32, vp, vp]),
    "stx_instnorm_bwd_ws": (sz, [i32, i32]),
    "stx_instnorm_param_grads": (i32, [C.POINTER(PGradJob), i32, vp]),
    "stx_instnorm_bwd": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32,
                               i32, i32, vp, vp, sz, vp]),
    "stx_upsample2x_fwd": (i32, [vp, vp, i32, i32, i32, vp]),
    "stx_upsample2x_bwd": (i32, [vp, vp, i32, i32, i32, vp]),
    "stx_tv_ws": (sz, [i32, i32, i32, i32]),
    "stx_tv_loss": (i32, [vp, vp, vp, f32, vp, i32, i32, i32, i32, f32, vp, sz, vp]),
    "stx_resample_coeffs": (i32, [i32, i32, vp, vp, i32]),
    "stx_image_condition": (i32, [vp, vp, i32, i32, vp, i32, vp, vp, vp, vp, sz, vp]),
    "stx_temporal_loss_ws": (sz, []),
    "stx_temporal_loss": (i32, [vp, vp, vp, vp, i64, f32, vp, vp, sz, vp]),
    "stx_temporal_loss_bwd": (i32, [vp, vp, i64, vp, f32, vp, vp, i32, vp]),
}

_lib = None
_lock = threading.Lock()


class NativeError(RuntimeError):
    pass


def lib():
    """Load libstx.so (raises NativeError if absent — there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise NativeError(
                    f"libstx.so not found at {LIB_PATH}; build it with "
                    f"`python -c 'import __graft_entry__ as g; g.build()'` "
                    f"(make -C styletransfer_amd/csrc)")
            try:
                L = C.CDLL(LIB_PATH)
            except OSError as e:  # pragma: no cover
                raise NativeError(f"failed to load {LIB_PATH}: {e}") from e
            # the ABI revision must match, whatever else: an older library whose entry
            # points read an argument differently would be driven out of bounds (a
            # round-5 libstx_prev.so read stx_instnorm_bwd's beta as a whole y plane)
            abi = L.stx_abi_version() if hasattr(L, "stx_abi_version") else None
            if abi != STX_ABI_VERSION:
                raise NativeError(f"{LIB_PATH}: ABI revision {abi}, this binding needs "
                                  f"{STX_ABI_VERSION} (include/stx.h STX_ABI_VERSION)")
            # STX_LIB_PARTIAL=1: an older build of the same ABI revision for same-box A/B
            # timing may lack newer entry points
            partial = os.environ.get("STX_LIB_PARTIAL") == "1"
            for name, (res, args) in SIGNATURES.items():
                if partial and not hasattr(L, name):
                    continue
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib().stx_last_error_string().decode(errors="replace")
        raise NativeError(f"{what or 'libstx'} failed (code {rc}): {msg}")
