"""Bilinear upsampling (align_corners=True) + Up's channel concatenation on lss_upsample_* kernels.

``upsample_cat(x, skip, scale)`` = ``torch.cat([skip, nn.Upsample(scale, 'bilinear',
align_corners=True)(x)], 1)`` (src/models.py:19, 33, 109) for channels-last bf16 CUDA maps, as the
BevEncode Up stages see them under bf16 autocast. The reference computes the upsample in fp32
(autocast's fp32 list) and the next conv casts the concatenation back to bf16; the kernel blends in
fp32 and writes that bf16 concatenation directly. Backward: a gather kernel for d(x) (fp32 sums,
no atomics), a view of the incoming gradient for d(skip). Anything else -- fp32 maps (no autocast),
NCHW, CPU -- runs the stock PyTorch ops.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from . import _lib

USE_HIP_UPSAMPLE = True


def _eligible(t: Optional[torch.Tensor]) -> bool:
    return (t is None or (t.is_cuda and t.dtype == torch.bfloat16 and t.dim() == 4 and t.shape[1] % 8 == 0
                          and t.is_contiguous(memory_format=torch.channels_last)))


class _UpsampleCat(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, skip, Ho: int, Wo: int, chan_scale=None):
        lib = _lib.load()
        N, C1, Hi, Wi = x.shape
        C2 = skip.shape[1] if skip is not None else 0
        y = torch.empty(N, C2 + C1, Ho, Wo, device=x.device, dtype=torch.bfloat16,
                        memory_format=torch.channels_last)
        _lib.check(lib.lss_upsample_cat_fwd2(_lib.ptr(x), _lib.ptr(skip), N, Hi, Wi, C1, C2, Ho, Wo,
                                             _lib.ptr(chan_scale), _lib.ptr(y), _lib.stream_handle(x.device)),
                   "lss_upsample_cat_fwd2")
        ctx.geo = (N, Hi, Wi, C1, C2, Ho, Wo)
        ctx.save_for_backward(chan_scale)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _lib.load()
        N, Hi, Wi, C1, C2, Ho, Wo = ctx.geo
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = torch.empty(N, C1, Hi, Wi, device=dy.device, dtype=torch.bfloat16, memory_format=torch.channels_last)
        (chan_scale,) = ctx.saved_tensors
        _lib.check(lib.lss_upsample_bwd2(_lib.ptr(dy), N, Hi, Wi, C1, C2, Ho, Wo, _lib.ptr(chan_scale), _lib.ptr(dx),
                                         _lib.stream_handle(dy.device)), "lss_upsample_bwd2")
        dskip = dy[:, :C2] if C2 else None
        return dx, dskip, None, None, None


def upsample_cat(x: torch.Tensor, skip: Optional[torch.Tensor], scale_factor: int,
                 chan_scale: Optional[torch.Tensor] = None) -> torch.Tensor:
    """cat([skip, bilinear_upsample(x * chan_scale, scale_factor, align_corners=True)], dim=1); skip and
    chan_scale (an (N, C) per-channel factor: a Dropout2d mask) may be None."""
    Ho, Wo = x.shape[2] * scale_factor, x.shape[3] * scale_factor
    if chan_scale is not None:
        chan_scale = chan_scale.reshape(x.shape[0], x.shape[1]).float().contiguous()
    if (USE_HIP_UPSAMPLE and _eligible(x) and _eligible(skip) and x.shape[2] > 1 and x.shape[3] > 1
            and (skip is None or (skip.shape[0] == x.shape[0] and tuple(skip.shape[2:]) == (Ho, Wo)))):
        return _UpsampleCat.apply(x, skip, Ho, Wo, chan_scale)
    if chan_scale is not None:
        x = x * chan_scale.view(x.shape[0], x.shape[1], 1, 1).to(x.dtype)
    up = F.interpolate(x, scale_factor=scale_factor, mode="bilinear", align_corners=True)
    return up if skip is None else torch.cat([skip, up], dim=1)
