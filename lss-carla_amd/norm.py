"""nn.BatchNorm2d + activation (+ residual) for the conv stacks, on the lss_bn_* kernels.

``bn_act(bn, x, act, residual)`` computes ``act(bn(x) [+ residual])`` for a BatchNorm2d module in
training mode with the module's own parameters and buffers (running statistics updated as PyTorch
does, ``num_batches_tracked`` incremented), so state_dicts are unchanged. Used where the reference
applies BN followed by swish (EfficientNet-B0) or ReLU (``Up``, ResNet-18 BevEncode). In eval mode,
on CPU tensors, or with ``USE_HIP_BN = False``, it runs the same computation with stock PyTorch ops.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F
from torch import nn

from . import _lib

USE_HIP_BN = True
# channels-last ReLU without a residual: the backward recomputes the output from x (lss_bn_bwd with
# y = NULL) instead of keeping and re-reading it
RECOMPUTE_RELU_Y = True
ACT = {"none": 0, "relu": 1, "swish": 2}
NCHW, NHWC = 0, 1
# NCHW maps with several groups per channel: statistics + apply in one launch per direction (the
# lss_bn_*2 cluster kernels), through a per-device sync workspace (zero-filled once, left zero-filled)
USE_BN_CLUSTER = True
_SYNC = {}


def _sync(dev: torch.device):
    if not USE_BN_CLUSTER:
        return None
    w = _SYNC.get(dev)
    if w is None:
        if torch.cuda.is_current_stream_capturing():
            return None  # (created by the eager warm-up steps, before any capture)
        w = torch.zeros(int(_lib.load().lss_bn_sync_words()), device=dev, dtype=torch.int32)
        _SYNC[dev] = w
    return w


def _layout(x: torch.Tensor) -> Optional[int]:
    if x.is_contiguous():
        return NCHW
    if x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last):
        return NHWC
    return None


def running_args(bn: nn.BatchNorm2d):
    """(momentum, num_batches_tracked counter or None, running_mean, running_var) for lss_bn_fwd*, with
    PyTorch's update rule (the counter is incremented by the kernel; a cumulative average needs it here)."""
    momentum = bn.momentum if bn.momentum is not None else 0.0
    counter = None
    if bn.track_running_stats and bn.num_batches_tracked is not None:
        if bn.momentum is None:  # cumulative moving average: the factor needs the count on the host
            bn.num_batches_tracked.add_(1)
            momentum = 1.0 / float(bn.num_batches_tracked.item())
        else:
            counter = bn.num_batches_tracked
    rm = bn.running_mean if bn.track_running_stats else None
    rv = bn.running_var if bn.track_running_stats else None
    return momentum, counter, rm, rv


class _BnAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, bn: nn.BatchNorm2d, act: int, layout: int):
        lib = _lib.load()
        N, C, H, W = x.shape
        HW = H * W
        dev = x.device
        st = _lib.stream_handle(dev)
        if residual is not None:
            residual = residual.to(x.dtype)
            residual = residual.contiguous(memory_format=torch.channels_last if layout == NHWC else
                                           torch.contiguous_format)
        y = torch.empty_like(x)
        groups = int(lib.lss_bn_groups(N, C, HW, layout))
        f32 = dict(device=dev, dtype=torch.float32)
        partial = torch.empty(C, groups, 2, **f32)
        stats = torch.empty(4, C, **f32)  # save_mean, save_rstd, scale, shift
        momentum, counter, rm, rv = running_args(bn)
        _lib.check(lib.lss_bn_fwd2(_lib.ptr(x), _lib.ptr(residual), _lib.dtype_code(x.dtype), layout, N, C, HW,
                                   _lib.ptr(weight), _lib.ptr(bias), float(bn.eps), float(momentum), _lib.ptr(rm),
                                   _lib.ptr(rv), _lib.ptr(counter), act, groups, _lib.ptr(partial),
                                   _lib.ptr(stats[0]), _lib.ptr(stats[1]), _lib.ptr(stats[2]), _lib.ptr(stats[3]),
                                   _lib.ptr(y), _lib.ptr(_sync(dev)), st), "lss_bn_fwd2")
        # ReLU's backward needs y; in channels-last without a residual the kernels recompute it from x
        # (lss_bn_bwd), so y is neither kept nor read again
        keep_y = act == ACT["relu"] and (layout == NCHW or residual is not None or not RECOMPUTE_RELU_Y)
        ctx.save_for_backward(x, y if keep_y else None, stats)
        ctx.conf = (act, layout, groups, residual is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _lib.load()
        x, y, stats = ctx.saved_tensors
        act, layout, groups, has_res = ctx.conf
        N, C, H, W = x.shape
        dev = x.device
        dy = dy.to(x.dtype).contiguous(memory_format=torch.channels_last if layout == NHWC else
                                       torch.contiguous_format)
        f32 = dict(device=dev, dtype=torch.float32)
        partial = torch.empty(C, groups, 2, **f32)
        coef = torch.empty(C, 2, **f32)
        dgamma = torch.empty(C, **f32)
        dbeta = torch.empty(C, **f32)
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if has_res else None
        _lib.check(lib.lss_bn_bwd2(_lib.ptr(dy), _lib.ptr(x), _lib.ptr(y), _lib.dtype_code(x.dtype), layout, N, C,
                                   H * W, _lib.ptr(stats[2]), _lib.ptr(stats[3]), _lib.ptr(stats[0]),
                                   _lib.ptr(stats[1]), act, groups, _lib.ptr(partial), _lib.ptr(coef),
                                   _lib.ptr(dgamma), _lib.ptr(dbeta), _lib.ptr(dx), _lib.ptr(dres),
                                   _lib.ptr(_sync(dev)), _lib.stream_handle(dev)), "lss_bn_bwd2")
        return dx, dgamma, dbeta, dres, None, None, None


def _torch_bn_act(bn: nn.BatchNorm2d, x: torch.Tensor, act: str, residual: Optional[torch.Tensor]):
    y = bn(x)
    if residual is not None:
        y = y + residual
    if act == "relu":
        return F.relu(y)
    if act == "swish":
        return F.silu(y)
    return y


def bn_act(bn: nn.BatchNorm2d, x: torch.Tensor, act: str = "none", residual: Optional[torch.Tensor] = None):
    """act(bn(x) [+ residual]) with act in {'none', 'relu', 'swish'}."""
    layout = _layout(x)
    use = (USE_HIP_BN and bn.training and x.is_cuda and x.dim() == 4 and layout is not None and bn.affine
           and x.dtype in (torch.float32, torch.bfloat16)
           and (layout == NCHW or (x.shape[1] % 8 == 0 and 256 % (x.shape[1] // 8) == 0)))
    if not use:
        return _torch_bn_act(bn, x, act, residual)
    return _BnAct.apply(x, bn.weight, bn.bias, residual, bn, ACT[act], layout)
