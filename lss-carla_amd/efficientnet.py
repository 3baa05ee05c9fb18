"""EfficientNet-B0 trunk with efficientnet_pytorch's module names and numerics.

The reference builds its camera trunk with
``EfficientNet.from_pretrained("efficientnet-b0")`` (``src/models.py:43``,
``efficientnet-pytorch>=0.7.1`` in ``requirements.txt:8``). That package is not
available here and its pretrained weights need the network, so this is a
from-scratch module with the same architecture and the same state_dict keys
(``_conv_stem``, ``_bn0``, ``_blocks.{i}._expand_conv/_bn0/_depthwise_conv/_bn1/
_se_reduce/_se_expand/_project_conv/_bn2``, ``_conv_head``, ``_bn1``, ``_fc``), so a
checkpoint of the reference loads into it. Weights are randomly initialised
(PyTorch defaults, as the package does before loading weights).

Architecture facts restated from the published B0 definition: width = depth =
1.0, image_size 224, batch-norm momentum 0.01 / eps 1e-3, drop-connect 0.2,
SE ratio 0.25, TF "static same" padding computed for 224x224 inputs, swish.
Runs as stock PyTorch-ROCm convolutions (MIOpen, MFMA via the library), except the depthwise
convolutions, which run on this package's HIP kernels (include/lss_convs.h) on the GPU.
"""
from __future__ import annotations

import math
import os
from types import SimpleNamespace
from typing import List, Tuple

import torch
import torch.nn.functional as F
from torch import nn

from .norm import bn_act

# (repeats, kernel, stride, expand, in, out) for the 7 stages of B0, SE ratio 0.25.
B0_STAGES = (
    (1, 3, 1, 1, 32, 16),
    (2, 3, 2, 6, 16, 24),
    (2, 5, 2, 6, 24, 40),
    (3, 3, 2, 6, 40, 80),
    (3, 5, 1, 6, 80, 112),
    (4, 5, 2, 6, 112, 192),
    (1, 3, 1, 6, 192, 320),
)
BN_MOMENTUM = 1 - 0.99
# depthwise weight gradient folded by each channel's last block (lss_dwconv_bwd_weight2); LSS_DW_FOLD=0 keeps
# the partial buffer + torch reduction (A/B in profiles/r06/dw_wgrad_fold.txt)
DW_FOLD = os.environ.get("LSS_DW_FOLD", "1") != "0"
BN_EPS = 1e-3
IMAGE_SIZE = 224


def _out_size(size: Tuple[int, int], stride: int) -> Tuple[int, int]:
    return (int(math.ceil(size[0] / stride)), int(math.ceil(size[1] / stride)))


class Conv2dStaticSamePadding(nn.Conv2d):
    """Conv2d with TF-'same' padding frozen for a nominal input size (efficientnet_pytorch semantics).

    Symmetric pads go to the convolution itself (no padded copy); asymmetric ones
    (stride-2 layers at even sizes pad 0 before / 1 after) use a ZeroPad2d module.
    """

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, groups=1, bias=True,
                 image_size: Tuple[int, int] = (IMAGE_SIZE, IMAGE_SIZE)):
        super().__init__(in_channels, out_channels, kernel_size, stride, 0, groups=groups, bias=bias)
        ih, iw = image_size
        kh, kw = self.weight.shape[-2:]
        sh, sw = self.stride
        oh, ow = math.ceil(ih / sh), math.ceil(iw / sw)
        pad_h = max((oh - 1) * sh + (kh - 1) * self.dilation[0] + 1 - ih, 0)
        pad_w = max((ow - 1) * sw + (kw - 1) * self.dilation[1] + 1 - iw, 0)
        pads = (pad_w // 2, pad_w - pad_w // 2, pad_h // 2, pad_h - pad_h // 2)
        if pads[0] == pads[1] and pads[2] == pads[3]:
            self.padding = (pads[2], pads[0])
            self.static_padding = nn.Identity()
        else:
            self.static_padding = nn.ZeroPad2d(pads)

    def forward(self, x):
        return self._conv_forward(self.static_padding(x), self.weight, self.bias)


class _NativeConv2d(torch.autograd.Function):
    """conv2d forward AND backward with MIOpen disabled, i.e. on PyTorch's native kernels.

    PyTorch picks the convolution backend again in backward (from the global cuDNN/MIOpen
    flag), so disabling MIOpen around the forward alone is not enough. Used for the depthwise
    convolutions, for which MIOpen has no bf16 NCHW solver and falls back to naive kernels.
    """

    @staticmethod
    def forward(ctx, x, w, stride, padding, dilation, groups):
        if x.is_cuda and torch.is_autocast_enabled("cuda"):
            dt = torch.get_autocast_dtype("cuda")
            x, w = x.to(dt), w.to(dt)
        with torch.autocast("cuda", enabled=False), torch.backends.cudnn.flags(enabled=False):
            y = F.conv2d(x, w, None, stride, padding, dilation, groups)
        ctx.save_for_backward(x, w)
        ctx.conf = (stride, padding, dilation, groups)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        stride, padding, dilation, groups = ctx.conf
        with torch.autocast("cuda", enabled=False), torch.backends.cudnn.flags(enabled=False):
            gx, gw, _ = torch.ops.aten.convolution_backward(
                gy.to(x.dtype).contiguous(), x, w, None, list(stride), list(padding), list(dilation), False, [0, 0],
                groups, [ctx.needs_input_grad[0], ctx.needs_input_grad[1], False])
        return gx, gw, None, None, None, None


class _HipDepthwise(torch.autograd.Function):
    """Depthwise conv (groups = C) on the lss_dwconv_* kernels of include/lss_convs.h.

    Activations in the autocast dtype (as the reference's ``nn.Conv2d`` under autocast), the fp32
    weight parameter read as is, fp32 accumulation; the weight gradient is fp32 (summed per image
    group on the device, then over the groups in a fixed order).
    """

    @staticmethod
    def forward(ctx, x, weight, stride: int, pads: Tuple[int, int, int, int]):
        from . import _lib
        lib = _lib.load()
        if torch.is_autocast_enabled("cuda"):
            x = x.to(torch.get_autocast_dtype("cuda"))
        if x.dtype not in (torch.float32, torch.bfloat16):
            x = x.float()
        x = x.contiguous()
        N, C, Hi, Wi = x.shape
        K = weight.shape[-1]
        pl, pr, pt, pb = pads
        Ho, Wo = (Hi + pt + pb - K) // stride + 1, (Wi + pl + pr - K) // stride + 1
        w = weight.detach().float().reshape(C, K * K).contiguous()
        y = torch.empty(N, C, Ho, Wo, device=x.device, dtype=x.dtype)
        _lib.check(lib.lss_dwconv_fwd(_lib.ptr(x), _lib.dtype_code(x.dtype), _lib.ptr(w), N, C, Hi, Wi, K, stride,
                                      pt, pl, Ho, Wo, _lib.ptr(y), _lib.stream_handle(x.device)), "lss_dwconv_fwd")
        ctx.save_for_backward(x, w)
        ctx.conf = (stride, pt, pl, Ho, Wo, weight.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import _lib
        lib = _lib.load()
        x, w = ctx.saved_tensors
        stride, pt, pl, Ho, Wo, wdtype = ctx.conf
        N, C, Hi, Wi = x.shape
        K = int(round((w.shape[1]) ** 0.5))
        dy = dy.to(x.dtype).contiguous()
        st = _lib.stream_handle(x.device)
        code = _lib.dtype_code(x.dtype)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            _lib.check(lib.lss_dwconv_bwd_data(_lib.ptr(dy), code, _lib.ptr(w), N, C, Hi, Wi, K, stride, pt, pl, Ho,
                                               Wo, _lib.ptr(dx), st), "lss_dwconv_bwd_data")
        if ctx.needs_input_grad[1]:
            groups = max(1, min(N, (N * Ho * Wo) // 8192))
            part = torch.empty(C, groups, K * K, device=x.device, dtype=torch.float32)
            from .norm import _sync
            sync = _sync(x.device) if C <= 4096 and DW_FOLD else None
            if sync is not None:
                # the channel's last block folds the partials (lss_dwconv_bwd_weight2): no reduction launch
                dw32 = torch.empty(C, K * K, device=x.device, dtype=torch.float32)
                _lib.check(lib.lss_dwconv_bwd_weight2(_lib.ptr(x), _lib.ptr(dy), code, N, C, Hi, Wi, K, stride, pt,
                                                      pl, Ho, Wo, groups, _lib.ptr(part), _lib.ptr(sync),
                                                      _lib.ptr(dw32), st), "lss_dwconv_bwd_weight2")
                dw = dw32.view(C, 1, K, K).to(wdtype)
            else:
                _lib.check(lib.lss_dwconv_bwd_weight(_lib.ptr(x), _lib.ptr(dy), code, N, C, Hi, Wi, K, stride, pt,
                                                     pl, Ho, Wo, groups, _lib.ptr(part), st), "lss_dwconv_bwd_weight")
                dw = part.sum(1).view(C, 1, K, K).to(wdtype)
        return dx, dw, None, None


class _HipPointwise(torch.autograd.Function):
    """1x1 conv (stride 1, no bias) over NCHW activations in bf16 (the autocast conv's operands): forward
    and backward-data on ``lss_pw_conv`` (MFMA, pixels as the GEMM rows; MIOpen's per-image batched
    GEMMs when USE_HIP_PW_GEMM is off or the shapes do not fit), the weight gradient on ``lss_pw_wrw``
    (include/lss_convs.h) -- an MFMA GEMM reading both operands in place, written in the weight's
    dtype, where MIOpen's NCHW path transposes both activations, accumulates atomically in an fp32
    workspace it zero-fills, and casts the result."""

    @staticmethod
    def forward(ctx, x, weight):
        from . import _lib
        xb = x.to(torch.bfloat16).contiguous()
        wb = weight.to(torch.bfloat16)
        N, Cin, H, W = xb.shape
        Cout = wb.shape[0]
        gemm = USE_HIP_PW_GEMM and Cin % 8 == 0 and Cout % 8 == 0 and xb.data_ptr() % 16 == 0
        if gemm:
            if wb.data_ptr() % 16 or not wb.is_contiguous():
                wb = wb.contiguous().clone()  # (a flat-parameter view need not be 16-B aligned)
            y = torch.empty(N, Cout, H, W, device=xb.device, dtype=torch.bfloat16)
            _lib.check(_lib.load().lss_pw_conv(_lib.ptr(xb), _lib.ptr(wb), 0, N, Cin, Cout, H * W, _lib.ptr(y),
                                               _lib.stream_handle(xb.device)), "lss_pw_conv")
        else:
            with torch.autocast("cuda", enabled=False):
                y = F.conv2d(xb, wb)
        ctx.save_for_backward(xb, wb)
        ctx.dtypes = (x.dtype, weight.dtype)
        ctx.gemm = gemm
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import _lib
        lib = _lib.load()
        xb, wb = ctx.saved_tensors
        xdt, wdt = ctx.dtypes
        dy = dy.to(torch.bfloat16).contiguous()
        dx = dw = None
        if ctx.needs_input_grad[0]:
            if ctx.gemm and dy.data_ptr() % 16 == 0:
                N, Cin, H, W = xb.shape
                dx = torch.empty_like(xb)
                _lib.check(lib.lss_pw_conv(_lib.ptr(dy), _lib.ptr(wb), 1, N, dy.shape[1], Cin, H * W, _lib.ptr(dx),
                                           _lib.stream_handle(xb.device)), "lss_pw_conv")
                dx = dx.to(xdt)
            else:
                with torch.autocast("cuda", enabled=False):
                    dx = torch.ops.aten.convolution_backward(dy, xb, wb, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                                             [True, False, False])[0].to(xdt)
        if ctx.needs_input_grad[1]:
            N, Cin, H, W = xb.shape
            Cout = dy.shape[1]
            nbytes = int(lib.lss_pw_wrw_workspace_bytes(N, Cin, Cout, H * W))
            ws = torch.empty(nbytes, device=xb.device, dtype=torch.uint8)
            dw = torch.empty(Cout, Cin, 1, 1, device=xb.device, dtype=wdt)
            _lib.check(lib.lss_pw_wrw(_lib.ptr(xb), _lib.ptr(dy), N, Cin, Cout, H * W, _lib.ptr(dw), _lib.dtype_code(wdt),
                                      _lib.ptr(ws), nbytes, _lib.stream_handle(xb.device)), "lss_pw_wrw")
        return dx, dw


# the trunk's 1x1 convs (MBConv expand / project) take _HipPointwise when their activations are bf16 NCHW;
# USE_HIP_PW_GEMM: its forward and backward-data on lss_pw_conv too (else MIOpen)
USE_HIP_PW_WRW = True
USE_HIP_PW_GEMM = True


def pointwise_conv(conv: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    if (USE_HIP_PW_WRW and x.is_cuda and x.dim() == 4 and conv.kernel_size == (1, 1) and conv.stride == (1, 1)
            and conv.groups == 1 and conv.bias is None and conv.padding == (0, 0) and conv.dilation == (1, 1)
            and isinstance(getattr(conv, "static_padding", None), (nn.Identity, type(None)))
            and x.is_contiguous() and (x.shape[2] * x.shape[3]) % 4 == 0
            and conv.weight.dtype in (torch.float32, torch.bfloat16)
            and ((torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16)
                 or (x.dtype == torch.bfloat16 and conv.weight.dtype == torch.bfloat16))
            and _pw_fits(x.shape[0], x.shape[1], conv.weight.shape[0], x.shape[2] * x.shape[3])):
        return _HipPointwise.apply(x, conv.weight)
    return conv(x)


_INT_MAX = 2**31 - 1


def _pw_fits(N: int, Cin: int, Cout: int, HW: int) -> bool:
    """The index limits lss_pw_conv / lss_pw_wrw enforce (they return EINVAL past them): larger
    activations stay on MIOpen instead of raising."""
    return N * max(Cin, Cout) * HW < _INT_MAX and N * ((HW + 31) // 32) < _INT_MAX


def depthwise_same_pads(conv: "Conv2dStaticSamePadding") -> Tuple[int, int, int, int]:
    """(left, right, top, bottom) padding of a static-same conv, whether it pads itself or via ZeroPad2d."""
    if isinstance(conv.static_padding, nn.ZeroPad2d):
        return tuple(conv.static_padding.padding)
    ph, pw = conv.padding
    return (pw, pw, ph, ph)


def drop_connect(x: torch.Tensor, p: float, training: bool) -> torch.Tensor:
    """Per-sample stochastic depth (efficientnet_pytorch ``drop_connect``)."""
    if not training or not p:
        return x
    keep = 1.0 - p
    mask = torch.floor(keep + torch.rand((x.shape[0], 1, 1, 1), dtype=x.dtype, device=x.device))
    return x / keep * mask


USE_HIP_DROP_ADD = True


class _HipScaleAdd(torch.autograd.Function):
    """y = bf16(x * scale[n] + res), scale[n] = floor(keep + u[n]) / keep computed in the kernel from
    the sample's draw u (``lss_scale_add``: one launch instead of the mask's add / floor and the
    divide, multiply and add); backward dx = bf16(dy * scale[n]), dres = dy."""

    @staticmethod
    def forward(ctx, x, res, u, keep):
        from . import _lib
        lib = _lib.load()
        y = torch.empty_like(x)
        N = x.shape[0]
        _lib.check(lib.lss_scale_add(_lib.ptr(x), _lib.ptr(u), keep, _lib.ptr(res), N, x.numel() // N, _lib.ptr(y),
                                     _lib.stream_handle(x.device)), "lss_scale_add")
        ctx.save_for_backward(u)
        ctx.keep = keep
        ctx.fmt = torch.channels_last if not x.is_contiguous() else torch.contiguous_format
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import _lib
        lib = _lib.load()
        (u,) = ctx.saved_tensors
        dy = dy.to(torch.bfloat16).contiguous(memory_format=ctx.fmt)
        if dy.data_ptr() % 16:  # a contiguous view at an unaligned offset: the kernel's 16-B loads need a copy
            dy = dy.clone(memory_format=ctx.fmt)
        dx = torch.empty_like(dy)
        N = dy.shape[0]
        _lib.check(lib.lss_scale_add(_lib.ptr(dy), _lib.ptr(u), ctx.keep, None, N, dy.numel() // N, _lib.ptr(dx),
                                     _lib.stream_handle(dy.device)), "lss_scale_add")
        return dx, dy, None, None


def _scale_add_eligible(x: torch.Tensor, res: torch.Tensor) -> bool:
    if not (USE_HIP_DROP_ADD and x.is_cuda and x.dtype == torch.bfloat16 and res.dtype == torch.bfloat16
            and x.dim() == 4 and x.shape == res.shape and (x.numel() // x.shape[0]) % 8 == 0):
        return False
    for fmt in (torch.contiguous_format, torch.channels_last):
        if x.is_contiguous(memory_format=fmt) and res.is_contiguous(memory_format=fmt):
            return all(t.data_ptr() % 16 == 0 for t in (x, res))
    return False


def drop_connect_add(x: torch.Tensor, inputs: torch.Tensor, p: float, training: bool) -> torch.Tensor:
    """``drop_connect(x, p, training) + inputs`` (the MBConv skip, src/models.py:43 via
    efficientnet_pytorch): the same per-sample draw (``rand`` in x's dtype; the mask
    ``floor(keep + rand)`` is formed in the kernel exactly as torch forms it), applied as one fused
    scale-and-add on bf16 activations (fp32 arithmetic, one rounding instead of three)."""
    if not training or not p:
        return x + inputs
    if not _scale_add_eligible(x, inputs):
        return drop_connect(x, p, training) + inputs
    u = torch.rand((x.shape[0],), dtype=x.dtype, device=x.device)  # the same draw as drop_connect's
    return _HipScaleAdd.apply(x, inputs, u, 1.0 - p)


class MBConvBlock(nn.Module):
    def __init__(self, k: int, stride: int, expand: int, in_f: int, out_f: int, image_size, se_ratio=0.25):
        super().__init__()
        self.in_f, self.out_f, self.stride, self.expand = in_f, out_f, stride, expand
        mid = in_f * expand
        if expand != 1:
            self._expand_conv = Conv2dStaticSamePadding(in_f, mid, 1, bias=False, image_size=image_size)
            self._bn0 = nn.BatchNorm2d(mid, momentum=BN_MOMENTUM, eps=BN_EPS)
        self._depthwise_conv = Conv2dStaticSamePadding(mid, mid, k, stride=stride, groups=mid, bias=False,
                                                       image_size=image_size)
        self._bn1 = nn.BatchNorm2d(mid, momentum=BN_MOMENTUM, eps=BN_EPS)
        image_size = _out_size(image_size, stride)
        sq = max(1, int(in_f * se_ratio))
        self._se_reduce = Conv2dStaticSamePadding(mid, sq, 1, image_size=(1, 1))
        self._se_expand = Conv2dStaticSamePadding(sq, mid, 1, image_size=(1, 1))
        # the lss_se_* kernels read these fp32 masters and round them to bf16 themselves
        self._se_reduce.lss_fp32_params = self._se_expand.lss_fp32_params = True
        self._project_conv = Conv2dStaticSamePadding(mid, out_f, 1, bias=False, image_size=image_size)
        self._bn2 = nn.BatchNorm2d(out_f, momentum=BN_MOMENTUM, eps=BN_EPS)
        # depthwise conv backend on the GPU: 'hip' (lss_dwconv_* kernels), 'miopen', 'native' (PyTorch's
        # own kernels), 'fp32' (MIOpen outside autocast)
        self.depthwise_impl = "hip"

    def forward(self, inputs: torch.Tensor, drop_connect_rate=None) -> torch.Tensor:
        x = inputs
        if self.expand != 1:
            x = bn_act(self._bn0, pointwise_conv(self._expand_conv, x), "swish")
        dw = self._depthwise_conv
        if self.depthwise_impl == "hip" and x.is_cuda:
            x = _HipDepthwise.apply(x, dw.weight, dw.stride[0], depthwise_same_pads(dw))
        elif self.depthwise_impl == "native" and x.is_cuda:
            x = _NativeConv2d.apply(dw.static_padding(x), dw.weight, dw.stride, dw.padding, dw.dilation, dw.groups)
        elif self.depthwise_impl == "fp32" and x.is_cuda and torch.is_autocast_enabled("cuda"):
            with torch.autocast("cuda", enabled=False):
                x = self._depthwise_conv(x.float())
        else:
            x = self._depthwise_conv(x)
        x = bn_act(self._bn1, x, "swish")
        x = squeeze_excite(x, self._se_reduce, self._se_expand)
        x = bn_act(self._bn2, pointwise_conv(self._project_conv, x))
        if self.stride == 1 and self.in_f == self.out_f:
            x = drop_connect_add(x, inputs, drop_connect_rate, self.training)
        return x


USE_HIP_SE = True


class _HipSqueezeExcite(torch.autograd.Function):
    """x * sigmoid(W2 swish(W1 avg_pool(x) + b1) + b2) on the lss_se_* kernels (NCHW bf16 x, fp32
    weights rounded to bf16 in-kernel as autocast's conv would). Backward: two streaming kernels
    (sum_hw dy*x, then dx = dy*sig + dm/HW) around a per-image MLP backward; the four weight /
    bias gradients in one more launch (lss_se_wgrad)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        from . import _lib
        lib = _lib.load()
        N, C, H, W = x.shape
        sq = w1.shape[0]
        f32 = dict(device=x.device, dtype=torch.float32)
        W1 = w1.detach().reshape(sq, C).float().contiguous()
        W2 = w2.detach().reshape(C, sq).float().contiguous()
        B1, B2 = b1.detach().float().contiguous(), b2.detach().float().contiguous()
        m, sig = torch.empty(N, C, **f32), torch.empty(N, C, **f32)
        r, h = torch.empty(N, sq, **f32), torch.empty(N, sq, **f32)
        y = torch.empty_like(x)
        _lib.check(lib.lss_se_fwd(_lib.ptr(x), N, C, H * W, _lib.ptr(W1), _lib.ptr(B1), _lib.ptr(W2), _lib.ptr(B2), sq,
                                  _lib.ptr(m), _lib.ptr(r), _lib.ptr(h), _lib.ptr(sig), _lib.ptr(y),
                                  _lib.stream_handle(x.device)), "lss_se_fwd")
        ctx.save_for_backward(x, W1, W2, m, r, h, sig)
        ctx.shapes = (w1.shape, w1.dtype, b1.dtype, w2.shape, w2.dtype, b2.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import _lib
        lib = _lib.load()
        x, W1, W2, m, r, h, sig = ctx.saved_tensors
        w1s, w1t, b1t, w2s, w2t, b2t = ctx.shapes
        N, C, H, W = x.shape
        sq = W1.shape[0]
        dy = dy.to(torch.bfloat16).contiguous()
        f32 = dict(device=x.device, dtype=torch.float32)
        t, de, dm = torch.empty(N, C, **f32), torch.empty(N, C, **f32), torch.empty(N, C, **f32)
        dr = torch.empty(N, sq, **f32)
        dh_part = torch.empty(N, (C + 63) // 64, sq, **f32)
        dx = torch.empty_like(x)
        _lib.check(lib.lss_se_bwd(_lib.ptr(dy), _lib.ptr(x), N, C, H * W, _lib.ptr(W1), _lib.ptr(W2), sq, _lib.ptr(r),
                                  _lib.ptr(sig), _lib.ptr(t), _lib.ptr(dh_part), _lib.ptr(de), _lib.ptr(dr),
                                  _lib.ptr(dm), _lib.ptr(dx), _lib.stream_handle(x.device)), "lss_se_bwd")
        dw1, db1 = torch.empty(sq, C, **f32), torch.empty(sq, **f32)
        dw2, db2 = torch.empty(C, sq, **f32), torch.empty(C, **f32)
        _lib.check(lib.lss_se_wgrad(_lib.ptr(de), _lib.ptr(h), _lib.ptr(dr), _lib.ptr(m), N, C, sq, _lib.ptr(dw1),
                                    _lib.ptr(db1), _lib.ptr(dw2), _lib.ptr(db2), _lib.stream_handle(x.device)),
                   "lss_se_wgrad")
        return dx, dw1.reshape(w1s).to(w1t), db1.to(b1t), dw2.reshape(w2s).to(w2t), db2.to(b2t)


def squeeze_excite(x: torch.Tensor, se_reduce: nn.Conv2d, se_expand: nn.Conv2d) -> torch.Tensor:
    """x * sigmoid(se_expand(swish(se_reduce(avg_pool(x))))) (efficientnet_pytorch MBConvBlock)."""
    if (USE_HIP_SE and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.is_contiguous()
            and (x.shape[2] * x.shape[3]) % 4 == 0 and x.shape[1] <= 2048 and se_reduce.weight.shape[0] <= 64
            and se_reduce.bias is not None and se_expand.bias is not None):
        return _HipSqueezeExcite.apply(x, se_reduce.weight, se_reduce.bias, se_expand.weight, se_expand.bias)
    s = F.adaptive_avg_pool2d(x, 1)
    s = se_expand(F.silu(se_reduce(s)))
    return torch.sigmoid(s) * x


def set_depthwise_impl(module: nn.Module, impl: str) -> None:
    """Depthwise-conv backend of every MBConv block under `module`: 'hip', 'miopen', 'native' or 'fp32'."""
    if impl not in ("hip", "miopen", "native", "fp32"):
        raise ValueError(f"unknown depthwise implementation {impl!r}")
    for m in module.modules():
        if isinstance(m, MBConvBlock):
            m.depthwise_impl = impl


class _NativeBatchNorm2d(nn.BatchNorm2d):
    """BatchNorm2d on PyTorch's native kernels (MIOpen disabled for the forward, which also
    fixes the backward: the autograd node is NativeBatchNormBackward)."""

    def forward(self, x):
        with torch.backends.cudnn.flags(enabled=False):
            return super().forward(x)


def set_batchnorm_native(module: nn.Module) -> int:
    """Swap the class of every BatchNorm2d under `module` (state_dict unchanged)."""
    n = 0
    for m in module.modules():
        if type(m) is nn.BatchNorm2d:
            m.__class__ = _NativeBatchNorm2d
            n += 1
    return n


def load_state_dict_file(path: str) -> dict:
    """A state dict from a file, by loaders that execute nothing from it: safetensors for
    ``.safetensors``, else ``torch.load(weights_only=True)`` (a ``{"state_dict": ...}`` wrapper is
    unwrapped). CPU tensors."""
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return dict(load_file(path, device="cpu"))
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "state_dict" in sd and isinstance(sd["state_dict"], dict):
        sd = sd["state_dict"]
    if not isinstance(sd, dict) or not all(isinstance(v, torch.Tensor) for v in sd.values()):
        raise RuntimeError(f"{path}: not a state dict of tensors")
    return sd


class EfficientNetB0(nn.Module):
    """The trunk of ``CamEncode`` (module names of efficientnet_pytorch.EfficientNet)."""

    def __init__(self, num_classes: int = 1000):
        super().__init__()
        self._global_params = SimpleNamespace(drop_connect_rate=0.2, dropout_rate=0.2, image_size=IMAGE_SIZE,
                                              batch_norm_momentum=0.99, batch_norm_epsilon=BN_EPS)
        size = (IMAGE_SIZE, IMAGE_SIZE)
        self._conv_stem = Conv2dStaticSamePadding(3, 32, 3, stride=2, bias=False, image_size=size)
        self._bn0 = nn.BatchNorm2d(32, momentum=BN_MOMENTUM, eps=BN_EPS)
        size = _out_size(size, 2)
        blocks: List[nn.Module] = []
        for repeats, k, s, e, i, o in B0_STAGES:
            blocks.append(MBConvBlock(k, s, e, i, o, size))
            size = _out_size(size, s)
            for _ in range(repeats - 1):
                blocks.append(MBConvBlock(k, 1, e, o, o, size))
        self._blocks = nn.ModuleList(blocks)
        self._conv_head = Conv2dStaticSamePadding(320, 1280, 1, bias=False, image_size=size)
        self._bn1 = nn.BatchNorm2d(1280, momentum=BN_MOMENTUM, eps=BN_EPS)
        self._avg_pooling = nn.AdaptiveAvgPool2d(1)
        self._dropout = nn.Dropout(0.2)
        self._fc = nn.Linear(1280, num_classes)

    @classmethod
    def from_pretrained(cls, model_name: str = "efficientnet-b0", weights_path: str | None = None,
                        load_fc: bool = True, num_classes: int = 1000) -> "EfficientNetB0":
        """``EfficientNet.from_pretrained`` (src/models.py:43) from a LOCAL file: nothing is fetched.

        weights_path: an efficientnet_pytorch-format state dict of B0 (the package's published
        ``efficientnet-b0-355c32eb.pth``, or any ``torch.save(model.state_dict())`` of either
        module; ``.safetensors`` also read). Default: $LSS_EFFICIENTNET_B0_WEIGHTS. Loaded with a
        loader that executes nothing from the file (``torch.load(weights_only=True)`` /
        safetensors). As the package's ``load_pretrained_weights``: every key of the model must be
        in the file (``num_batches_tracked`` excepted: older checkpoints lack it), the ``_fc``
        keys are skipped with ``load_fc=False`` (then ``num_classes`` may differ), and a key the
        model does not have is an error."""
        if model_name != "efficientnet-b0":
            raise ValueError(f"only efficientnet-b0 is built here, not {model_name!r}")
        import os
        path = weights_path or os.environ.get("LSS_EFFICIENTNET_B0_WEIGHTS")
        if not path:
            raise RuntimeError("EfficientNetB0.from_pretrained needs a local weights file (weights_path= or "
                               "$LSS_EFFICIENTNET_B0_WEIGHTS): there is no download")
        sd = load_state_dict_file(path)
        if not load_fc:
            sd = {k: v for k, v in sd.items() if not k.startswith("_fc.")}
        model = cls(num_classes)
        ret = model.load_state_dict(sd, strict=False)
        missing = [k for k in ret.missing_keys if not k.endswith("num_batches_tracked")
                   and (load_fc or not k.startswith("_fc."))]
        if missing or ret.unexpected_keys:
            raise RuntimeError(f"{path}: not an efficientnet-b0 state dict (missing {missing[:5]}, "
                               f"unexpected {ret.unexpected_keys[:5]})")
        return model

    @staticmethod
    def _swish(x: torch.Tensor) -> torch.Tensor:
        return F.silu(x)

    def forward(self, x: torch.Tensor) -> torch.Tensor:  # classification head (unused by LSS)
        x = bn_act(self._bn0, self._conv_stem(x), "swish")
        for idx, block in enumerate(self._blocks):
            x = block(x, self._global_params.drop_connect_rate * idx / len(self._blocks))
        x = self._swish(self._bn1(self._conv_head(x)))
        return self._fc(self._dropout(self._avg_pooling(x).flatten(1)))
