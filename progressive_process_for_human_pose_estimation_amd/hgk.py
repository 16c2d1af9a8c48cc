"""ctypes binding of libhgk.so (include/hgk.h) + thin tensor-level wrappers.

The HIP library is the only compute path: if libhgk.so is missing or cannot be loaded, every
wrapper raises — there is no CPU / eager-PyTorch fallback.
"""
import ctypes
import os

import torch  # noqa: F401  (must be imported first: libhgk resolves libamdhip64 to torch's copy)

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "libhgk.so")

F32, BF16 = 0, 1
UP_BILINEAR_AC, UP_NEAREST = 0, 1
ABI_VERSION = 39

_c_void_p = ctypes.c_void_p
_c_int = ctypes.c_int
_c_long = ctypes.c_long
_c_float = ctypes.c_float
_c_size_t = ctypes.c_size_t
_c_intp = ctypes.POINTER(ctypes.c_int)



class WgradSrc(ctypes.Structure):
    """struct hgk_wgrad_src (include/hgk.h): one use of a weight for hgk_conv_wgrad_accum_multi."""
    _fields_ = [("x", _c_void_p), ("dy", _c_void_p), ("pre_scale", _c_void_p),
                ("pre_shift", _c_void_p), ("pre_relu", _c_int), ("N", _c_int), ("H", _c_int),
                ("W", _c_int)]


class WgradJob(ctypes.Structure):
    """struct hgk_wgrad_job (include/hgk.h): one use of one weight for hgk_conv_wgrad_accum_batch."""
    _fields_ = [("src", WgradSrc), ("slabs", _c_void_p), ("slab_cap", _c_int), ("slabs_init", _c_int),
                ("with_bias", _c_int), ("Cin", _c_int), ("Cout", _c_int), ("KH", _c_int),
                ("KW", _c_int), ("stride", _c_int), ("pad", _c_int), ("dil", _c_int)]


class PackDesc(ctypes.Structure):
    """struct hgk_pack_desc (include/hgk.h): one weight layout for hgk_pack_conv_weight_multi."""
    _fields_ = [("w", _c_void_p), ("packed", _c_void_p), ("w_ld", _c_int), ("Cout", _c_int),
                ("Cin", _c_int), ("KH", _c_int), ("KW", _c_int), ("for_dgrad", _c_int),
                ("Cout_store", _c_int), ("Cin_store", _c_int), ("rows_store", _c_int)]


class WgradFin(ctypes.Structure):
    """struct hgk_wgrad_fin (include/hgk.h): one weight for hgk_conv_wgrad_finish_multi."""
    _fields_ = [("slabs", _c_void_p), ("slab_cap", _c_int), ("nslabs", _c_int), ("dw", _c_void_p),
                ("db", _c_void_p), ("Cin", _c_int), ("Cout", _c_int), ("KH", _c_int), ("KW", _c_int),
                ("Cin_log", _c_int), ("Cout_log", _c_int)]


class BnVgrad(ctypes.Structure):
    """struct hgk_bn_vgrad (include/hgk.h): a BN-backward apply folded into a conv's staging."""
    _fields_ = [("y", _c_void_p), ("scale", _c_void_p), ("shift", _c_void_p), ("coef", _c_void_p),
                ("relu", _c_int), ("out", _c_void_p),
                # folded finalize (ABI 27; partial = None: coef is final)
                ("partial", _c_void_p), ("rows", _c_int), ("M", _c_long), ("mean", _c_void_p),
                ("invstd", _c_void_p), ("training", _c_int), ("dgamma", _c_void_p),
                ("dbeta", _c_void_p), ("add", _c_void_p)]


class BnFold(ctypes.Structure):
    """struct hgk_bn_fold (include/hgk.h): a BN finalize folded into the consuming conv."""
    _fields_ = [("partial", _c_void_p), ("rows", _c_int), ("M", _c_long), ("gamma", _c_void_p),
                ("beta", _c_void_p), ("eps", _c_float), ("stat", _c_void_p), ("rec", _c_void_p)]


class ConvSeg(ctypes.Structure):
    """struct hgk_conv_seg (include/hgk.h): one segment of hgk_conv_fwd_twin."""
    _fields_ = [("x", _c_void_p), ("res", _c_void_p), ("y", _c_void_p), ("pre_scale", _c_void_p),
                ("pre_shift", _c_void_p), ("stats", _c_void_p), ("rows_out", _c_intp),
                ("N", _c_int), ("H", _c_int), ("W", _c_int), ("bb_y", _c_void_p),
                ("bb_scale", _c_void_p), ("bb_shift", _c_void_p), ("bb_mean", _c_void_p),
                ("bb_invstd", _c_void_p), ("bb_partial", _c_void_p), ("bb_relu", _c_int),
                ("bb_rows", _c_intp), ("vg", ctypes.POINTER(BnVgrad)),
                ("fold", ctypes.POINTER(BnFold))]


class BnSeg(ctypes.Structure):
    """struct hgk_bn_seg (include/hgk.h): one use for hgk_bn_finalize_deferred."""
    _fields_ = [("partial", _c_void_p), ("rows", _c_int), ("M", _c_long), ("rec", _c_void_p),
                ("stat", _c_void_p)]


class BnFinJob(ctypes.Structure):
    """struct hgk_bn_fin_job (include/hgk.h): one BN of a multi-BN forward finalize."""
    _fields_ = [("partial", _c_void_p), ("rows", _c_int), ("M", ctypes.c_long), ("C", _c_int),
                ("gamma", _c_void_p), ("beta", _c_void_p), ("eps", ctypes.c_float),
                ("rec", _c_void_p), ("stat", _c_void_p)]


class BnbFinJob(ctypes.Structure):
    """struct hgk_bnb_fin_job (include/hgk.h): one BN of a multi-BN backward finalize."""
    _fields_ = [("partial", _c_void_p), ("rows", _c_int), ("M", ctypes.c_long), ("C", _c_int),
                ("scale", _c_void_p), ("mean", _c_void_p), ("invstd", _c_void_p),
                ("training", _c_int), ("dgamma", _c_void_p), ("dbeta", _c_void_p),
                ("coef", _c_void_p)]


class BnbSide(ctypes.Structure):
    """struct hgk_bnb_side (include/hgk.h): one BN of a summed pair, backward (hgk_bn_bwd_pair)."""
    _fields_ = [("y", _c_void_p), ("scale", _c_void_p), ("shift", _c_void_p), ("mean", _c_void_p),
                ("invstd", _c_void_p), ("relu", _c_int), ("partial", _c_void_p), ("rows", _c_int),
                ("coef", _c_void_p), ("dgamma", _c_void_p), ("dbeta", _c_void_p), ("dy", _c_void_p)]


class BnSide(ctypes.Structure):
    """struct hgk_bn_side (include/hgk.h): one BN of a pair whose outputs are summed."""
    _fields_ = [("y", _c_void_p), ("scale", _c_void_p), ("shift", _c_void_p), ("mean", _c_void_p),
                ("invstd", _c_void_p), ("relu", _c_int), ("partial", _c_void_p)]


class BnRunning(ctypes.Structure):
    """struct hgk_bn_running (include/hgk.h): one deferred running-statistics update."""
    _fields_ = [("running_mean", _c_void_p), ("running_var", _c_void_p), ("rec", _c_void_p),
                ("C", _c_int), ("momentum", _c_float)]


class BnbSeg(ctypes.Structure):
    """struct hgk_bnb_seg (include/hgk.h): one use for hgk_bn_bwd_twin."""
    _fields_ = [("partial", _c_void_p), ("rows", _c_int), ("M", _c_long), ("stat", _c_void_p),
                ("dA", _c_void_p), ("y", _c_void_p), ("add", _c_void_p), ("dy", _c_void_p),
                ("accumulate", _c_int)]


# name -> (restype, argtypes); the single source of truth for what include/hgk.h exports
SIGNATURES = {
    "hgk_abi_version": (_c_int, []),
    "hgk_last_error": (ctypes.c_char_p, []),
    "hgk_max_stats_rows": (_c_int, []),
    "hgk_set_route": (_c_long, [_c_int, _c_long]),
    "hgk_get_route": (_c_long, [_c_int]),
    "hgk_conv_fwd_kernel_family": (_c_int, [_c_int] * 14),
    "hgk_conv_fwd": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p,
                              _c_void_p, _c_void_p, _c_void_p, _c_int, _c_int, _c_void_p, _c_intp,
                              _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int,
                              _c_int, _c_void_p, _c_size_t]),
    "hgk_conv_fwd_workspace": (_c_size_t, [_c_int] * 11),
    "hgk_conv_fwd_twin": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_int, _c_void_p] + [_c_int] * 9
                          + [ctypes.POINTER(ConvSeg), _c_void_p, _c_size_t]),
    "hgk_conv_fwd_twin_workspace": (_c_size_t, [_c_int] * 14),
    "hgk_pack_conv_weight_multi": (_c_int, [_c_void_p, _c_int, ctypes.POINTER(PackDesc), _c_int]),
    "hgk_pack_conv_weight": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_int, _c_int, _c_int,
                                      _c_int, _c_int, _c_int, _c_int, _c_int]),
    "hgk_conv_w_ld": (_c_int, [_c_int]),
    "hgk_conv_wgrad_workspace": (_c_size_t, [_c_int] * 11),
    "hgk_conv_wgrad": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int,
                                _c_void_p, _c_void_p, _c_void_p, _c_size_t] + [_c_int] * 12),
    "hgk_conv_fwd_bnbwd": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_int, _c_void_p,
                                    _c_void_p] + [_c_int] * 10 + [_c_void_p, _c_size_t,
                                    _c_void_p, _c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p,
                                    _c_void_p, _c_intp]),
    "hgk_conv_fwd_bnbwd_vg": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_int, _c_void_p,
                                       _c_void_p] + [_c_int] * 10 + [_c_void_p, _c_size_t,
                                       _c_void_p, _c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p,
                                       _c_void_p, _c_intp, ctypes.POINTER(BnVgrad)]),
    "hgk_conv_vgrad_ok": (_c_int, [_c_int] * 15),
    "hgk_conv_vgrad_fin_ok": (_c_int, [_c_int] * 18),
    "hgk_conv_fwd_fold": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p,
                                   _c_void_p, _c_int, _c_int, _c_void_p, _c_intp] + [_c_int] * 10
                          + [_c_void_p, _c_size_t, ctypes.POINTER(BnFold)]),
    "hgk_conv_fold_ok": (_c_int, [_c_int] * 16),
    "hgk_conv_wgrad_max_splits": (_c_int, []),
    "hgk_conv_wgrad_slab_bytes": (_c_size_t, [_c_int] * 5),
    "hgk_conv_wgrad_accum": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                      _c_int, _c_void_p, _c_int, _c_int, _c_int, _c_intp]
                             + [_c_int] * 10),
    "hgk_conv_wgrad_finish": (_c_int, [_c_void_p, _c_void_p, _c_int, _c_int, _c_void_p, _c_void_p]
                              + [_c_int] * 6),
    "hgk_conv_wgrad_finish_multi": (_c_int, [_c_void_p, ctypes.POINTER(WgradFin), _c_int]),
    "hgk_conv_wgrad_accum_multi": (_c_int, [_c_void_p, _c_int, ctypes.POINTER(WgradSrc), _c_int,
                                            _c_void_p, _c_int, _c_int, _c_int, _c_intp]
                                   + [_c_int] * 7),
    "hgk_gauss_targets": (_c_int, [_c_void_p] * 4 + [_c_int] * 5 + [_c_float, _c_void_p]),
    "hgk_pckh": (_c_int, [_c_void_p] * 4 + [_c_int] * 4 + [_c_void_p] * 4),
    "hgk_bn_stats": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_long, _c_int, _c_void_p, _c_intp]),
    "hgk_bn_finalize": (_c_int, [_c_void_p, _c_void_p, _c_int, _c_long, _c_int, _c_void_p, _c_void_p,
                                 _c_void_p, _c_void_p, _c_float, _c_float, _c_int, _c_void_p, _c_void_p,
                                 _c_void_p, _c_void_p, _c_void_p]),
    "hgk_bn_finalize_scratch": (_c_size_t, [_c_int, _c_int]),
    "hgk_bn_apply": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_long, _c_int, _c_void_p, _c_void_p,
                              _c_int, _c_void_p]),
    "hgk_bn_bwd_reduce": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_long, _c_int, _c_void_p,
                                   _c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_intp]),
    "hgk_conv_wgrad_accum_batch": (_c_int, [_c_void_p, _c_int, ctypes.POINTER(WgradJob), _c_int,
                                            ctypes.POINTER(_c_int)]),
    "hgk_bn_apply2_add": (_c_int, [_c_void_p, _c_int, ctypes.POINTER(BnSide), ctypes.POINTER(BnSide),
                                   _c_void_p, _c_long, _c_int, _c_void_p, _c_intp]),
    "hgk_bn_bwd_reduce2": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_long, _c_int,
                                    ctypes.POINTER(BnSide), ctypes.POINTER(BnSide), _c_intp]),
    "hgk_bn_finalize_multi": (_c_int, [_c_void_p, ctypes.POINTER(BnFinJob), _c_int]),
    "hgk_bn_bwd_finalize_multi": (_c_int, [_c_void_p, ctypes.POINTER(BnbFinJob), _c_int]),
    "hgk_bn_bwd_finalize_multi_min_rows": (_c_int, []),
    "hgk_bn_bwd_pair": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_long, _c_int, _c_int,
                                 ctypes.POINTER(BnbSide), ctypes.POINTER(BnbSide)]),
    "hgk_bn_bwd_finalize": (_c_int, [_c_void_p, _c_void_p, _c_int, _c_long, _c_int, _c_void_p,
                                     _c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p,
                                     _c_void_p]),
    "hgk_bn_bwd_apply": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_long, _c_int, _c_void_p,
                                  _c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_int]),
    "hgk_bn_bwd_fused_max_rows": (_c_int, []),
    "hgk_bn_finalize_deferred": (_c_int, [_c_void_p, ctypes.POINTER(BnSeg), _c_int, _c_int, _c_void_p,
                                          _c_void_p, _c_float]),
    "hgk_bn_running_update": (_c_int, [_c_void_p, ctypes.POINTER(BnRunning), _c_int]),
    "hgk_bn_bwd_twin": (_c_int, [_c_void_p, _c_int, ctypes.POINTER(BnbSeg), _c_int, _c_int, _c_int,
                                 _c_int, _c_void_p, _c_void_p, _c_void_p]),
    "hgk_bn_bwd_finalize_apply": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_int, _c_long, _c_int,
                                           _c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p,
                                           _c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                           _c_void_p, _c_void_p, _c_int]),
    "hgk_maxpool2_fwd": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_int, _c_int, _c_int,
                                  _c_int]),
    "hgk_maxpool2_bwd": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_int, _c_int,
                                  _c_int, _c_int, _c_int]),
    "hgk_upsample2_add_fwd": (_c_int, [_c_void_p, _c_int, _c_int, _c_void_p, _c_void_p, _c_void_p,
                                       _c_int, _c_int, _c_int, _c_int]),
    "hgk_upsample2_bwd": (_c_int, [_c_void_p, _c_int, _c_int, _c_void_p, _c_void_p, _c_int, _c_int,
                                   _c_int, _c_int, _c_int]),
    "hgk_mse_fwd_bwd": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_long, _c_void_p, _c_intp,
                                 _c_void_p, _c_float]),
    "hgk_mse_finalize": (_c_int, [_c_void_p, _c_void_p, _c_int, _c_long, _c_void_p, _c_int]),
    "hgk_mse_heads_nhwc": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_int, _c_void_p, _c_int,
                                    _c_int, _c_int, _c_int, _c_int, _c_float, _c_void_p, _c_void_p]),
    "hgk_mse_heads_partial_rows": (_c_int, []),
    "hgk_nchw_to_nhwc": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_int, _c_int, _c_int,
                                  _c_int, _c_int]),
    "hgk_nhwc_to_nchw": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_int, _c_int, _c_int,
                                  _c_int, _c_int]),
    "hgk_channel_copy": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_int, _c_int, _c_void_p, _c_int,
                                  _c_int, _c_int, _c_long, _c_int]),
    "hgk_maxpool2_fwd_stats": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_int, _c_int,
                                        _c_int, _c_int, _c_void_p, ctypes.POINTER(_c_int)]),
    "hgk_upsample2_add_fwd_stats": (_c_int, [_c_void_p, _c_int, _c_int, _c_void_p, _c_void_p,
                                             _c_void_p, _c_int, _c_int, _c_int, _c_int, _c_void_p,
                                             ctypes.POINTER(_c_int)]),
    "hgk_add": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_long, _c_int]),
    "hgk_ce_pixels": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int, _c_int, _c_long,
                               _c_void_p, _c_void_p]),
    "hgk_ce_grad": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int, _c_int,
                             _c_long, _c_void_p, _c_float, _c_void_p]),
    "hgk_ce_fwd_bwd": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_int, _c_int, _c_long, _c_void_p,
                                _c_intp, _c_void_p, _c_float, _c_void_p]),
    "hgk_sqdiff": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int, _c_int, _c_long,
                            _c_void_p]),
    "hgk_sqdiff_grad": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int,
                                 _c_int, _c_long, _c_void_p, _c_float, _c_void_p]),
    "hgk_topk_select": (_c_int, [_c_void_p, _c_void_p, _c_int, _c_long, _c_long, _c_void_p,
                                 _c_void_p]),
    "hgk_zero_insert": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_int, _c_int, _c_int,
                                 _c_int, _c_int, _c_int, _c_int]),
    "hgk_spatial_sum": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_int, _c_int, _c_int,
                                 _c_float, _c_int]),
    "hgk_spatial_broadcast": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_int, _c_int,
                                       _c_int, _c_float, _c_int]),
    "hgk_adam_step": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_long, _c_float,
                               _c_float, _c_float, _c_float, _c_float, _c_void_p]),
}

_lib = None


class HgkError(RuntimeError):
    pass


def load_library(path=None):
    """Load libhgk.so and bind every exported symbol. Raises if anything is missing.
    HGK_LIB overrides the path (kernel ablation builds, scripts/ only)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("HGK_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise HgkError(f"libhgk.so not found at {path}: build it with "
                       "`python -m progressive_process_for_human_pose_estimation_amd.build_ext` "
                       "(there is no CPU fallback)")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError -> loud failure
        fn.restype = res
        fn.argtypes = args
    if lib.hgk_abi_version() != ABI_VERSION:
        raise HgkError("libhgk ABI version mismatch")
    _lib = lib
    for name, knob in ROUTES.items():   # the compiled defaults, before anything sets a route
        _ROUTE_DEFAULT.setdefault(name, lib.hgk_get_route(knob))
    return lib


def lib():
    return _lib if _lib is not None else load_library()


def check(rc):
    if rc != 0:
        raise HgkError(f"libhgk error {rc}: {lib().hgk_last_error().decode()}")


KFAM = {0: "implicit", 1: "smallc", 2: "halo", 3: "ring", 4: "row3", 5: "img", 6: "split", 7: "stem"}

# kernel routing knobs of the library (include/hgk.h HGK_ROUTE_*): compiled defaults, changed only
# by an explicit set_route / route() call (A/B experiments and tests), never by the environment
ROUTES = {"ring_nw": 0, "ring_minm": 1, "ring_small": 2, "row3": 3, "splitk_fixup": 4, "img": 5,
          "wg_full": 6, "wg_dma": 7, "wg_batch_target": 8, "row3_alt": 9, "halo_bn64": 10, "wg_batch_slab_x10": 11,
          "stem": 12, "img_narrow": 13, "wg_ring": 14, "wg_halo_multi": 15}
_ROUTE_SET = {}  # knobs moved off their compiled default through set_route (graph-cache keys)
_ROUTE_DEFAULT = {}  # the library's compiled defaults, read once at load


def set_route(name, value):
    """Set a library routing knob (value < 0: its compiled default); returns the previous value."""
    if name not in ROUTES:
        raise HgkError(f"unknown library route {name!r}: expected one of {sorted(ROUTES)}")
    prev = lib().hgk_set_route(ROUTES[name], int(value))
    if prev < 0:
        check(prev)
    now = lib().hgk_get_route(ROUTES[name])
    if now == _ROUTE_DEFAULT.get(name):
        _ROUTE_SET.pop(name, None)
    else:
        _ROUTE_SET[name] = now
    return prev


def route_key():
    """The library routes changed from their defaults, as a hashable key: a captured hipGraph
    froze the launches of the routes in force at capture (modules._signature)."""
    return tuple(sorted(_ROUTE_SET.items()))


def get_route(name):
    if name not in ROUTES:
        raise HgkError(f"unknown library route {name!r}: expected one of {sorted(ROUTES)}")
    return lib().hgk_get_route(ROUTES[name])


class route:
    """Context manager: `with hgk.route(ring_minm=0): ...` runs the block on another kernel
    route and restores the previous values on exit."""

    def __init__(self, **knobs):
        self.knobs = knobs
        self.prev = {}

    def __enter__(self):
        for k, v in self.knobs.items():
            self.prev[k] = set_route(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.prev.items():
            set_route(k, v)
        return False


def dtype_code(dt):
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    raise HgkError(f"unsupported activation dtype {dt}")


def stream_handle():
    return torch.cuda.current_stream().cuda_stream


def ptr(t):
    return None if t is None else t.data_ptr()


def _require_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise HgkError("libhgk tensors must live on the GPU")
