"""ctypes binding of libartsbir_hip.so (the C-ABI declared in include/artsbir.h).

This module is the only place Python touches the native library.  It loads the
in-tree shared object (built by ``make`` in this directory / ``__graft_entry__.build``)
and fails loudly when it is missing: the product path has no CPU or PyTorch
fallback.  ``import torch`` happens first so that the HIP runtime torch ships is
the one the library binds to (same soname, loaded once per process).
"""
from __future__ import annotations

import ctypes
import os
import time

import torch  # noqa: F401  (must be imported before the library is dlopen'ed)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ARTSBIR_LIB") or os.path.join(_HERE, "libartsbir_hip.so")

DT_F32 = 0
DT_BF16 = 1
NSLOT = 32

_c_int = ctypes.c_int
_c_ll = ctypes.c_longlong
_c_float = ctypes.c_float
_vp = ctypes.c_void_p


class ConvDesc(ctypes.Structure):
    _fields_ = [("dtype", _c_int), ("N", _c_int), ("H", _c_int), ("W", _c_int), ("C", _c_int),
                ("Cout", _c_int), ("R", _c_int), ("S", _c_int), ("stride", _c_int), ("pad", _c_int)]


class BnBwdDesc(ctypes.Structure):
    _fields_ = [("dtype", _c_int), ("kind", _c_int), ("pool", _c_int), ("d", _vp), ("mask", _vp),
                ("mask_bn", _vp), ("ntarget", _c_int), ("y", _vp * 2),
                ("mean", _vp * 2), ("istd", _vp * 2), ("slots", _vp * 2), ("coef", _vp * 2), ("dy", _vp * 2),
                ("gout", _vp), ("B", _c_int), ("H", _c_int), ("W", _c_int), ("C", _c_int), ("nseg", _c_int),
                ("pstride", _c_ll), ("cstride", _c_ll), ("sstride", _c_ll)]


class AdamTensor(ctypes.Structure):
    _fields_ = [("param", _vp), ("grad", _vp), ("exp_avg", _vp), ("exp_avg_sq", _vp), ("numel", _c_ll)]


class PackDesc(ctypes.Structure):
    """artsbir_pack_desc (include/artsbir.h): one entry of the batched weight re-pack"""
    _fields_ = [("src", _vp), ("dst", _vp), ("Co", _c_int), ("Ci", _c_int), ("R", _c_int), ("S", _c_int),
                ("ci_pad", _c_int), ("mode", _c_int), ("ldo", _c_ll), ("blk0", _c_ll)]


class ImageDesc(ctypes.Structure):
    """artsbir_image_desc (include/artsbir.h)"""
    _fields_ = [("src", ctypes.c_void_p), ("H", ctypes.c_int), ("W", ctypes.c_int), ("C", ctypes.c_int),
                ("pitch", ctypes.c_int), ("rw", ctypes.c_int), ("rh", ctypes.c_int), ("left", ctypes.c_int),
                ("top", ctypes.c_int)]


class WarpDesc(ctypes.Structure):
    """artsbir_warp_desc (include/artsbir.h)"""
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("kind", ctypes.c_int),
                ("coeffs", ctypes.c_double * 8), ("fill", ctypes.c_ubyte * 3)]


class EraseDesc(ctypes.Structure):
    """artsbir_erase_desc (include/artsbir.h)"""
    _fields_ = [("src", ctypes.c_void_p), ("nrect", ctypes.c_int), ("rect", (ctypes.c_int * 4) * 4),
                ("value", ctypes.c_float * 4)]


_P = ctypes.POINTER(ConvDesc)
_PI = ctypes.POINTER(ImageDesc)
_PB = ctypes.POINTER(BnBwdDesc)

# name -> argtypes (restype is always int status unless listed in _RESTYPES)
SIGNATURES = {
    "artsbir_clip_preprocess_workspace": [ctypes.c_int, _PI, ctypes.c_int],
    "artsbir_resize_u8": [ctypes.c_int, _PI, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong,
                          ctypes.c_void_p],
    "artsbir_warp_u8": [ctypes.c_int, ctypes.POINTER(WarpDesc), ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                        ctypes.c_longlong, ctypes.c_void_p],
    "artsbir_erase_normalize": [ctypes.c_int, ctypes.POINTER(EraseDesc), ctypes.c_int, ctypes.c_int,
                                ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float), ctypes.c_void_p,
                                ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p],
    "artsbir_clip_preprocess": [ctypes.c_int, _PI, ctypes.c_int, ctypes.POINTER(ctypes.c_float),
                                ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong,
                                ctypes.c_void_p],
    "artsbir_version": [],
    "artsbir_last_error": [],
    "artsbir_last_kernel": [],
    "artsbir_tune_save": [ctypes.c_char_p],
    "artsbir_tune_load": [ctypes.c_char_p],
    "artsbir_stream_create_cu_mask": [ctypes.POINTER(ctypes.c_uint), _c_int, ctypes.POINTER(_vp)],
    "artsbir_stream_destroy": [_vp],
    "artsbir_conv2d_fwd": [_P, _vp, _vp, _vp, _c_ll, _c_int, _c_int, _vp, _vp, _vp, _c_int, _vp, _vp],
    "artsbir_conv2d_wgrad": [_P, _vp, _vp, _vp, _vp, _c_int, _vp, _vp],
    "artsbir_gemm_nt": [_c_int, _c_ll, _c_int, _c_int, _vp, _c_ll, _vp, _vp, _c_ll, _c_int, _c_int, _vp, _vp, _vp],
    "artsbir_gemm_nt_gate": [_c_ll, _c_int, _c_int, _vp, _c_ll, _vp, _vp, _c_ll, _vp, _vp, _vp],
    "artsbir_gemm_tn": [_c_int, _c_ll, _c_int, _c_int, _vp, _c_ll, _vp, _c_ll, _vp, _vp],
    "artsbir_conv2d_dgrad": [_P, _vp, _vp, _vp, _vp, _c_int, _vp],
    "artsbir_conv2d_fwd_seg": [_P, _vp, _vp, _vp, _c_int, _vp, _vp],
    "artsbir_conv2d_fwd_act": [_P, _vp, _vp, _vp, _vp, _vp, _c_int, _c_int, _vp],
    "artsbir_bn_fold": [_vp, _c_int, _c_ll, _vp, _vp, _vp, _vp, ctypes.c_float, _vp, _vp, _vp],
    "artsbir_conv2d_dgrad_bnb": [_P, _vp, _vp, _vp, _vp, _c_int, _PB, _c_int, _c_ll, _vp],
    "artsbir_conv1x1_dgrad_fold": [_P, _vp, _vp, _vp, _vp, _vp, _PB, _c_int, _c_ll, _vp],
    "artsbir_conv1x1_dgrad_fold_wg": [_P, _vp, _vp, _vp, _vp, _vp, _PB, _c_int, _c_ll, _vp, _vp, _vp],
    "artsbir_conv1x1_dgrad_fold_y": [_P, _vp, _vp, _vp, _vp, _vp, _vp, _c_int, _PB, _c_int, _c_ll, _vp],
    "artsbir_bn_fold_bwd_prep_y": [_c_int, _c_int, _c_int, _vp, _vp, _vp, _c_ll, _c_int, _vp, _vp, _vp],
    "artsbir_bn_fold_wgrad_combine_y": [_c_int, _c_int, _c_int, _vp, _vp, _vp, _c_int, _vp, _vp, _c_ll, _vp, _vp],
    "artsbir_bn_fold_bwd_prep": [_c_int, _c_int, _c_int, _vp, _vp, _vp, _c_ll, _c_int, _vp, _vp, _vp, _vp],
    "artsbir_bn_fold_wgrad_combine": [_c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _c_int, _vp, _vp, _vp, _c_ll, _vp,
                                      _vp, _vp],
    "artsbir_act_pool_colsum": [_c_int, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp,
                                _vp],
    "artsbir_gemm_tn2": [_c_int, _c_ll, _c_int, _c_int, _c_int, _vp, _c_ll, _vp, _c_ll, _vp, _c_ll, _vp, _vp, _vp],
    "artsbir_pack_input": [_c_int, _vp, _c_int, _c_int, _c_int, _c_int, _vp, _vp],
    "artsbir_pack_weight": [_c_int, _vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_ll, _vp, _vp],
    "artsbir_pack_weights": [_c_int, _vp, _c_int, _c_ll, _vp],
    "artsbir_unpack_wgrad": [_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp],
    "artsbir_cast": [_c_int, _vp, _c_int, _vp, _c_ll, _vp],
    "artsbir_bn_finalize": [_vp, _c_int, ctypes.c_double, _vp, _vp, _vp, _vp, _vp, _c_float, _c_float, _c_int,
                            _vp, _vp, _vp, _vp, _vp],
    "artsbir_bn_stats_det": [_c_int, _vp, _c_int, _c_ll, _c_int, _vp, _c_ll, _vp],
    "artsbir_act_pool": [_c_int, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp],
    "artsbir_block_out": [_c_int, _vp, _vp, _vp, _vp, _vp, _c_ll, _c_int, _c_int, _vp, _vp],
    "artsbir_block_out_mask": [_c_int, _vp, _vp, _vp, _vp, _vp, _c_ll, _c_int, _c_int, _vp, _vp, _vp],
    "artsbir_block_out_colsum": [_c_int, _vp, _vp, _vp, _vp, _vp, _c_ll, _c_int, _c_int, _vp, _vp, _vp, _vp],
    "artsbir_layernorm_fwd": [_c_int, _vp, _vp, _vp, _c_ll, _c_int, ctypes.c_float, _vp, _vp],
    "artsbir_quickgelu": [_c_int, _vp, _c_ll, _vp, _vp],
    "artsbir_mha_fwd": [_c_int, _vp, _c_int, _c_int, _c_int, _vp, _vp, _vp],
    "artsbir_mha_fwd_lse": [_c_int, _vp, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp],
    "artsbir_layernorm_bwd": [_c_int, _vp, _vp, _vp, _c_ll, _c_int, ctypes.c_float, _vp, _vp, _vp, _vp, _vp],
    "artsbir_layernorm_fwd_pmax": [_c_int, _vp, _vp, _vp, _c_ll, _c_int, ctypes.c_float, _vp, _vp, _vp],
    "artsbir_quickgelu_pmax": [_c_int, _vp, _c_ll, _vp, _vp, _vp],
    "artsbir_mha_fwd_lse_pmax": [_c_int, _vp, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp],
    "artsbir_quantize_fp8_pmax": [_c_int, _vp, _c_ll, _vp, _c_int, _vp, _vp, _vp],
    "artsbir_layernorm_bwd_sums": [_c_int, _vp, _vp, _vp, _c_ll, _c_int, ctypes.c_float, _vp, _vp, _vp, _vp, _vp, _vp,
                                   _vp],
    "artsbir_quickgelu_bwd_sum": [_c_int, _vp, _vp, _c_ll, _c_int, _vp, _vp, _vp],
    "artsbir_quickgelu_bwd": [_c_int, _vp, _vp, _c_ll, _vp, _vp],
    "artsbir_mha_bwd": [_c_int, _vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp],
    "artsbir_vit_patchify": [_c_int, _vp, _c_int, _c_int, _c_int, _vp, _vp],
    "artsbir_quantize_fp8": [_c_int, _vp, _c_ll, _vp, _vp, _vp],
    "artsbir_gemm_nt_fp8": [_c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp, _vp, _c_int, _c_int, _vp],
    "artsbir_gemm_nt_fp8_gelu": [_c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "artsbir_gemm_nt_fp8_ex": [_c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp, _vp, _c_int, _c_int, _vp, _vp, _c_int,
                               _vp],
    "artsbir_vit_tokens": [_c_int, _vp, _vp, _vp, _c_int, _c_int, _c_int, _vp, _vp],
    "artsbir_vit_tokens_bwd": [_c_int, _vp, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp],
    "artsbir_bn_finalize_seg": [_vp, _c_int, _c_ll, _c_int, ctypes.c_double, _vp, _vp, _vp, _vp, _vp, _c_float,
                                _c_float, _c_int, _vp, _vp],
    "artsbir_bn_bwd_finalize_seg": [_vp, _c_int, _c_ll, _c_int, ctypes.c_double, _vp, _vp, _c_ll, _vp, _vp, _vp,
                                    _vp],
    "artsbir_bn_bwd_reduce": [_PB, _vp],
    "artsbir_set_deterministic": [_c_int],
    "artsbir_set_wgrad_cus": [_c_int],
    "artsbir_bn_bwd_finalize": [_vp, _c_int, ctypes.c_double, _vp, _vp, _vp, _vp, _vp, _vp],
    "artsbir_bn_bwd_apply": [_PB, _vp],
    "artsbir_colsum": [_c_int, _vp, _c_ll, _c_ll, _c_ll, _vp, _vp],
    "artsbir_tokens_fwd": [_c_int, _vp, _vp, _c_int, _c_int, _c_int, _vp, _vp],
    "artsbir_tokens_bwd": [_c_int, _vp, _c_int, _c_int, _c_int, _vp, _vp],
    "artsbir_tokens_bwd_ex": [_c_int, _vp, _vp, _c_int, _c_int, _c_int, _vp, _vp],
    "artsbir_attnpool_fwd": [_c_int, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp],
    "artsbir_attnpool_bwd": [_c_int, _vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp],
    "artsbir_triplet_fwd": [_vp, _vp, _vp, _c_int, _c_int, _c_float, _c_float, _vp, _vp, _vp],
    "artsbir_triplet_bwd": [_vp, _vp, _vp, _c_int, _c_int, _c_float, _c_float, _vp, _vp, _vp, _vp, _vp, _vp],
    "artsbir_adam_table_blocks": [_vp, _c_int, _c_ll],
    "artsbir_adam_fill_table": [_vp, _c_int, _c_ll, _vp],
    "artsbir_adam_step": [_vp, _vp, _c_ll, _c_ll, _c_float, _c_float, _c_float, _c_float, _c_float, _c_ll, _vp],
    "artsbir_pairwise_l2": [_vp, _c_ll, _vp, _c_ll, _c_int, _c_float, _vp, _vp],
    "artsbir_rows_prep": [_c_int, _vp, _c_int, _c_int, _vp, _vp, _c_int, _vp],
    "artsbir_knn_band": [_vp, _vp, _vp, _c_ll, _c_ll, _vp, _c_float, _c_int, _c_int, _c_float, _vp, _vp, _vp, _vp],
    "artsbir_knn_band_from_dpos": [_vp, _vp, _c_float, _c_int, _c_float, _vp, _vp, _vp],
    "artsbir_knn_candidates_per_query": [_c_int, _c_int],
    "artsbir_knn_scan": [_c_int, _vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _c_int,
                         _vp, _vp, _vp],
    "artsbir_rows_prep_aug": [_vp, _c_int, _c_int, _c_int, _vp, _vp, _vp],
    "artsbir_knn_scan_aug_supported": [_c_int],
    "artsbir_knn_scan_aug": [_vp, _vp, _vp, _c_float, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _c_int, _c_float,
                             _vp, _vp, _vp, _vp, _c_int, _vp, _vp, _vp],
    "artsbir_knn_merge": [_vp, _vp, _c_int, _c_int, _c_int, _vp, _vp, _vp, _c_float, _c_float, _c_ll, _c_int, _vp,
                          _vp, _vp, _vp],
    "artsbir_knn_uncertain": [_vp, _vp, _c_int, _vp, _c_int, _vp, _vp, _c_ll, _vp, _vp],
    "artsbir_knn_exact_all": [_vp, _vp, _c_int, _c_int, _vp, _vp],
    "artsbir_pairwise_l2_topk_workspace": [_c_int, _c_int, _c_ll, _c_int, _c_int, _c_int],
    "artsbir_pairwise_l2_topk": [_c_int, _c_int, _vp, _c_int, _vp, _c_ll, _c_int, _c_int, _vp, _vp, _c_ll, _c_int,
                                 _vp, _vp, _vp, _vp, _vp, _c_ll, _vp],
    "artsbir_scan_profile": [_c_int],
    "artsbir_knn_set_unc_cap": [_c_int],
    "artsbir_scan_profile_read": [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_c_int)],
    "artsbir_knn_stat_read": [ctypes.POINTER(ctypes.c_ulonglong), _c_int],
    "artsbir_topk_merge": [_c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp],
    "artsbir_positive_key": [_c_int, _vp, _c_int, _vp, _c_ll, _c_int, _vp, _c_ll, _vp, _vp],
    "artsbir_pairwise_l2_bwd": [_vp, _c_ll, _vp, _c_ll, _c_int, _c_float, _vp, _vp, _vp, _vp, _vp],
    "artsbir_linear_fwd": [_vp, _vp, _vp, _c_int, _c_int, _c_int, _vp, _vp],
    "artsbir_linear_bwd": [_vp, _vp, _vp, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp],
    "artsbir_cross_entropy_fwd": [_vp, _vp, _c_int, _c_int, _c_ll, _vp, _vp, _vp],
    "artsbir_cross_entropy_bwd": [_vp, _vp, _c_int, _c_int, _c_ll, _vp, _vp, _vp, _vp],
    "artsbir_cosine_fwd": [_vp, _c_ll, _vp, _c_ll, _c_int, _c_float, _vp, _vp, _vp],
    "artsbir_cosine_bwd": [_vp, _c_ll, _vp, _c_ll, _c_int, _vp, _vp, _vp, _vp, _vp, _vp],
    "artsbir_hinge_fwd": [_vp, _vp, _c_int, _c_float, _vp, _vp],
    "artsbir_hinge_bwd": [_vp, _vp, _c_int, _c_float, _vp, _vp, _vp, _vp],
}
_RESTYPES = {"artsbir_last_error": ctypes.c_char_p, "artsbir_last_kernel": ctypes.c_char_p, "artsbir_adam_table_blocks": _c_ll,
             "artsbir_knn_candidates_per_query": _c_int, "artsbir_pairwise_l2_topk_workspace": _c_ll,
             "artsbir_clip_preprocess_workspace": _c_ll}

_lib = None


def lib() -> ctypes.CDLL:
    """Load (once) and return the native library; raise if it is not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libartsbir_hip.so not found at {LIB_PATH}: build it with `make -C art-sbir_amd` "
                "or __graft_entry__.build(); there is no fallback path")
        handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, argtypes in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.argtypes = argtypes
            fn.restype = _RESTYPES.get(name, _c_int)
        _lib = handle
    return _lib


class HipError(RuntimeError):
    pass


# Optional live per-launch timing (bench.py): when PROFILE is a list, every call
# that declares its algorithmic work is bracketed by two timing events on the
# current stream and (kernel, flops, bytes, start, end, tag, stream) is appended.
PROFILE = None
HOST_TS = None  # list: host time of every profiled launch (diagnostics)
# Optional call trace (tests): when TRACE is a list, every successful call appends
# (entry point, kernel, tag) — kernel is the variant the library launched for a
# kernel="auto" call (artsbir_last_kernel), the declared name otherwise — so a
# test can assert which kernels a whole forward / backward actually ran
TRACE = None


def call(name: str, *args, kernel: str | None = None, flops: float = 0.0, nbytes: float = 0.0,
         tag: str | None = None) -> None:
    """Invoke a status-returning entry point; map a non-zero status to HipError."""
    prof = PROFILE
    if HOST_TS is not None and prof is not None and kernel is not None:
        HOST_TS.append(time.perf_counter())  # host enqueue time of this launch (tools/step_gaps.py --host)
    if prof is not None and kernel is not None:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = getattr(lib(), name)(*args)
        e1.record()
        if kernel == "auto":  # the variant the library chose for this call
            kernel = lib().artsbir_last_kernel().decode()
        prof.append((kernel, flops, nbytes, e0, e1, tag, torch.cuda.current_stream().cuda_stream))
    else:
        rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = lib().artsbir_last_error().decode(errors="replace")
        raise HipError(f"{name} failed ({rc}): {msg}")
    tr = TRACE
    if tr is not None:
        if kernel == "auto":
            kernel = lib().artsbir_last_kernel().decode()
        tr.append((name, kernel, tag))


def ptr(t) -> int | None:
    """Raw device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return DT_F32
    if dt == torch.bfloat16:
        return DT_BF16
    raise TypeError(f"unsupported compute dtype {dt}")


def conv_desc(dt: torch.dtype, N, H, W, C, Cout, R, S, stride, pad) -> ConvDesc:
    return ConvDesc(dtype_code(dt), N, H, W, C, Cout, R, S, stride, pad)
