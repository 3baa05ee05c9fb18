"""ctypes binding of ``liblss_hip.so`` (the C ABI of ``include/lss_hip.h`` and ``include/lss_convs.h``).

The library is built in-tree by ``__graft_entry__.build()`` (or
``python -m lss_carla_amd.build``). There is no fallback: if the library is
missing or a call fails, a RuntimeError is raised.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch  # noqa: F401  -- loads the HIP runtime (soname libamdhip64.so.7) before our library

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liblss_hip.so")
DEBUG_LIB_PATH = os.path.join(_HERE, "liblss_hip_debug.so")  # LSS_DEBUG=1: device-side index checks

F32, BF16 = 0, 1
NCHW, NHWC = 0, 1
ABI_VERSION = 23


class Dims(ctypes.Structure):
    _fields_ = [("B", ctypes.c_int32), ("N", ctypes.c_int32), ("D", ctypes.c_int32),
                ("H", ctypes.c_int32), ("W", ctypes.c_int32), ("C", ctypes.c_int32)]


class ImgAug(ctypes.Structure):
    """lss_img_aug_t of include/lss_simbev.h."""
    _fields_ = [("src_h", ctypes.c_int32), ("src_w", ctypes.c_int32), ("rs_w", ctypes.c_int32),
                ("rs_h", ctypes.c_int32), ("crop", ctypes.c_int32 * 4), ("flip", ctypes.c_int32),
                ("rot_mode", ctypes.c_int32), ("affine", ctypes.c_int32 * 6), ("h_off", ctypes.c_int32),
                ("h_ksize", ctypes.c_int32), ("v_off", ctypes.c_int32), ("v_ksize", ctypes.c_int32)]


class Grid(ctypes.Structure):
    _fields_ = [("lo", ctypes.c_float * 3), ("dx", ctypes.c_float * 3), ("nx", ctypes.c_int32 * 3)]


_p = ctypes.c_void_p
_i32 = ctypes.c_int32
_DIMS = ctypes.POINTER(Dims)
_GRID = ctypes.POINTER(Grid)

# name -> (restype, argtypes); must match include/lss_hip.h exactly.
SIGNATURES = {
    "lss_abi_version": (ctypes.c_int, []),
    "lss_error_string": (ctypes.c_char_p, [ctypes.c_int]),
    "lss_debug_checks": (ctypes.c_int, []),
    "lss_debug_status": (ctypes.c_int, [_p, _i32]),
    "lss_event_create": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p)]),
    "lss_event_destroy": (ctypes.c_int, [_p]),
    "lss_event_elapsed_ms": (ctypes.c_int, [_p, _p, ctypes.POINTER(ctypes.c_float)]),
    "lss_event_record": (ctypes.c_int, [_p, _p]),
    "lss_ceiling_store": (ctypes.c_int, [_p, ctypes.c_size_t, _i32, _i32, _p, _p, _p]),
    "lss_ceiling_read": (ctypes.c_int, [_p, ctypes.c_size_t, _p, _p]),
    "lss_geometry_cells": (ctypes.c_int, [_p, _p, _p, _p, _p, _p, _DIMS, _GRID, _p, _p, _p, _p, _p]),
    "lss_cells_from_geom": (ctypes.c_int, [_p, _i32, _i32, _GRID, _p, _p, _p, _p]),
    "lss_csr_scratch_bytes": (ctypes.c_size_t, [_i32, _i32]),
    "lss_csr_build": (ctypes.c_int, [_p, _p, _i32, _p, _i32, _DIMS, _p, _p, _p, _p, _p]),
    "lss_csr_workspace_bytes": (ctypes.c_size_t, [_i32]),
    "lss_csr_build_ws": (ctypes.c_int, [_p, _p, _i32, _p, _i32, _DIMS, _p, _p, _p, _p, _p, _p]),
    "lss_csr_lists_bytes": (ctypes.c_size_t, [_i32, _i32]),
    "lss_geometry_cells_ordered": (ctypes.c_int, [_p, _p, _p, _p, _p, _p, _DIMS, _GRID, _p, _p, _p, _p, _p, _p, _p]),
    "lss_cells_from_geom_ordered": (ctypes.c_int, [_p, _i32, _i32, _GRID, _p, _p, _p, _p, _p, _p]),
    "lss_csr_build_ordered": (ctypes.c_int, [_p, _p, _i32, _p, _i32, _DIMS, _p, _p, _p, _p, _p, _p]),
    "lss_lift_prep": (ctypes.c_int, [_p, _i32, _DIMS, _p, _p, _i32, _p]),
    "lss_depthnet_lift": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _DIMS, _p, _p, _i32, _p]),
    "lss_depthnet_lift_nhwc": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _DIMS, _p, _p, _i32, _p]),
    "lss_depthnet_pack": (ctypes.c_int, [_p, _p, _i32, _i32, _i32, _p, _p, _p, _p]),
    "lss_flat_cast_bf16": (ctypes.c_int, [_p, _p, ctypes.c_int64, _p, _i32, _i32, _p, _p]),
    "lss_depthnet_lift_nhwc_packed": (ctypes.c_int, [_p, _p, _p, _i32, _DIMS, _p, _p, _i32, _p]),
    "lss_splat_fwd": (ctypes.c_int, [_p, _p, _i32, _p, _p, _p, _p, _DIMS, _GRID, _p, _i32, _i32, _p, _p, _p]),
    "lss_bev_rows": (ctypes.c_int, [_p, _i32, _p, _DIMS, _GRID, _p, _p]),
    "lss_splat_bwd": (ctypes.c_int, [_p, _i32, _i32, _p, _p, _p, _i32, _DIMS, _GRID, _p, _i32, _p]),
    "lss_splat_bwd_lifted": (ctypes.c_int, [_p, _i32, _i32, _p, _i32, _DIMS, _GRID, _p, _p]),
    "lss_segment_scratch_bytes": (ctypes.c_size_t, [_i32]),
    "lss_segment_build": (ctypes.c_int, [_p, _i32, _p, _p, _p, _p, _p]),
    "lss_segment_sum": (ctypes.c_int, [_p, _i32, _p, _i32, _p, _i32, _p, _p, _p]),
    "lss_segment_gather": (ctypes.c_int, [_p, _i32, _p, _i32, _p, _p]),
    # include/lss_simbev.h (SimBEV input path, same library)
    "lss_resample_ksize": (ctypes.c_int, [_i32, _i32]),
    "lss_resample_coeffs": (ctypes.c_int, [_i32, _i32, _p]),
    "lss_simbev_images": (ctypes.c_int, [_p, _i32, _i32, _i32, _p, _p, _i32, _i32, _p, _p]),
    "lss_simbev_vehicle_mask": (ctypes.c_int, [_p, _i32, _i32, _i32, _i32, _p, _p]),
    # include/lss_convs.h (conv-stack kernels, same library)
    "lss_dwconv_fwd": (ctypes.c_int, [_p, _i32, _p] + [_i32] * 10 + [_p, _p]),
    "lss_dwconv_bwd_data": (ctypes.c_int, [_p, _i32, _p] + [_i32] * 10 + [_p, _p]),
    "lss_dwconv_bwd_weight": (ctypes.c_int, [_p, _p, _i32] + [_i32] * 11 + [_p, _p]),
    "lss_dwconv_bwd_weight2": (ctypes.c_int, [_p, _p] + [_i32] * 12 + [_p, _p, _p, _p]),
    "lss_head1_blocks": (ctypes.c_int, [_i32]),
    "lss_head1_fwd": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _p, _p]),
    "lss_head1_bwd": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _p, _p, _p]),
    "lss_head1_fwd2": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _p, _p, _p]),
    "lss_head1_bwd2": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _p, _p, _p, _p]),
    "lss_bn_bwd_rank1": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _i32, _p, _p, _p, _p, _p,
                                        _p]),
    "lss_scale_add": (ctypes.c_int, [_p, _p, ctypes.c_float, _p, ctypes.c_int64, ctypes.c_int64, _p, _p]),
    "lss_dropout": (ctypes.c_int, [_p, _i32, ctypes.c_int64, _p, ctypes.c_float, _p, _p, ctypes.c_int64, _p]),
    "lss_bce_logits": (ctypes.c_int, [_p, _i32, _p, ctypes.c_int64, ctypes.c_float, _p, _p, _p, _p]),
    "lss_bce_partials": (ctypes.c_int64, [ctypes.c_int64]),
    "lss_channel_sums": (ctypes.c_int, [_p, _i32, _i32, _i32, _i32, _p, _p]),
    "lss_conv_flip_weight": (ctypes.c_int, [_p, _i32, _i32, _i32, _i32, _i32, _p, _p]),
    "lss_clip_adam_partials": (ctypes.c_int, []),
    "lss_clip_adam": (ctypes.c_int, [_i32, _p, _p, _p, _p, _p, _p, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                     ctypes.c_float, ctypes.c_float, ctypes.c_float, _p, _p]),
    "lss_bce_logits_bwd": (ctypes.c_int, [_p, _i32, ctypes.c_int64, _p, _p, _p]),
    "lss_pw_wrw_workspace_bytes": (ctypes.c_int64, [_i32, _i32, _i32, _i32]),
    "lss_pw_wrw": (ctypes.c_int, [_p, _p, _i32, _i32, _i32, _i32, _p, _i32, _p, ctypes.c_int64, _p]),
    "lss_pw_conv": (ctypes.c_int, [_p, _p, _i32, _i32, _i32, _i32, _i32, _p, _p]),
    "lss_bn_groups": (ctypes.c_int, [_i32, _i32, _i32, _i32]),
    "lss_bn_fwd": (ctypes.c_int, [_p, _p, _i32, _i32, _i32, _i32, _i32, _p, _p, ctypes.c_float, ctypes.c_float,
                                  _p, _p, _p, _i32, _i32, _p, _p, _p, _p, _p, _p, _p]),
    "lss_bn_bwd": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _i32, _p, _p,
                                  _p, _p, _p, _p, _p]),
    "lss_bn_sync_words": (ctypes.c_int, []),
    "lss_bn_fwd2": (ctypes.c_int, [_p, _p, _i32, _i32, _i32, _i32, _i32, _p, _p, ctypes.c_float, ctypes.c_float,
                                   _p, _p, _p, _i32, _i32, _p, _p, _p, _p, _p, _p, _p, _p]),
    "lss_bn_bwd2": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _i32, _p, _p,
                                   _p, _p, _p, _p, _p, _p]),
    "lss_upsample_cat_fwd": (ctypes.c_int, [_p, _p] + [_i32] * 7 + [_p, _p]),
    "lss_upsample_bwd": (ctypes.c_int, [_p] + [_i32] * 7 + [_p, _p]),
    "lss_upsample_cat_fwd2": (ctypes.c_int, [_p, _p, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _p, _p, _p]),
    "lss_upsample_bwd2": (ctypes.c_int, [_p, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _p, _p, _p]),
    "lss_se_fwd": (ctypes.c_int, [_p, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _p, _p, _p, _p, _p, _p]),
    "lss_se_bwd": (ctypes.c_int, [_p, _p, _i32, _i32, _i32, _p, _p, _i32, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "lss_se_wgrad": (ctypes.c_int, [_p, _p, _p, _p, _i32, _i32, _i32, _p, _p, _p, _p, _p]),
}

_lib: Optional[ctypes.CDLL] = None


def DN_PACKED_BYTES(K: int) -> int:
    """LSS_DN_PACKED_BYTES(K) of include/lss_hip.h: bytes of lss_depthnet_pack's fragment buffer."""
    return K * 256


def open_library(path: str) -> ctypes.CDLL:
    """dlopen a build of the C ABI and attach the signatures (also used for tuning variants)."""
    if not os.path.exists(path):
        raise RuntimeError(
            f"lss_carla_amd: HIP library not found at {path}. Build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950). "
            "There is no CPU fallback.")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.lss_abi_version() != ABI_VERSION:
        raise RuntimeError(f"lss_carla_amd: ABI mismatch ({lib.lss_abi_version()} != {ABI_VERSION}); rebuild")
    return lib


def load() -> ctypes.CDLL:
    """Load (once) and type the product library; raise if it is absent or of another ABI."""
    global _lib
    if _lib is None:  # LSS_LIB: another build of the same ABI (A/B timing of tuning builds)
        default = DEBUG_LIB_PATH if os.environ.get("LSS_DEBUG", "0") == "1" else LIB_PATH
        _lib = open_library(os.environ.get("LSS_LIB") or default)
    return _lib


def debug_status(clear: bool = True):
    """(failures, first check code, value, bound) recorded by a LSS_DEBUG build's device checks; all
    zero for the product library. Synchronous."""
    out = (ctypes.c_int32 * 4)()
    check(load().lss_debug_status(ctypes.cast(out, ctypes.c_void_p), int(clear)), "lss_debug_status")
    return tuple(out)


def check(code: int, what: str) -> None:
    if code != 0:
        msg = load().lss_error_string(code)
        raise RuntimeError(f"{what} failed: {msg.decode() if msg else code} (code {code})")


def ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_handle(device: torch.device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    raise RuntimeError(f"lss_carla_amd: unsupported dtype {dt} (float32 / bfloat16 only)")
