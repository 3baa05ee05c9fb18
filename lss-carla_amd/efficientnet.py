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
Runs as stock PyTorch-ROCm convolutions (MIOpen) -- MFMA via the library.
"""
from __future__ import annotations

import math
from types import SimpleNamespace
from typing import List, Tuple

import torch
import torch.nn.functional as F
from torch import nn

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


def drop_connect(x: torch.Tensor, p: float, training: bool) -> torch.Tensor:
    """Per-sample stochastic depth (efficientnet_pytorch ``drop_connect``)."""
    if not training or not p:
        return x
    keep = 1.0 - p
    mask = torch.floor(keep + torch.rand((x.shape[0], 1, 1, 1), dtype=x.dtype, device=x.device))
    return x / keep * mask


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
        self._project_conv = Conv2dStaticSamePadding(mid, out_f, 1, bias=False, image_size=image_size)
        self._bn2 = nn.BatchNorm2d(out_f, momentum=BN_MOMENTUM, eps=BN_EPS)
        self.depthwise_fp32 = False  # run the depthwise conv outside autocast (MIOpen solver choice)
        self.depthwise_native = False  # run the depthwise conv on PyTorch's native kernels (not MIOpen)

    def forward(self, inputs: torch.Tensor, drop_connect_rate=None) -> torch.Tensor:
        x = inputs
        if self.expand != 1:
            x = F.silu(self._bn0(self._expand_conv(x)))
        if self.depthwise_native and x.is_cuda:
            dw = self._depthwise_conv
            x = _NativeConv2d.apply(dw.static_padding(x), dw.weight, dw.stride, dw.padding, dw.dilation, dw.groups)
        elif self.depthwise_fp32 and x.is_cuda and torch.is_autocast_enabled("cuda"):
            with torch.autocast("cuda", enabled=False):
                x = self._depthwise_conv(x.float())
        else:
            x = self._depthwise_conv(x)
        x = F.silu(self._bn1(x))
        s = F.adaptive_avg_pool2d(x, 1)
        s = self._se_expand(F.silu(self._se_reduce(s)))
        x = torch.sigmoid(s) * x
        x = self._bn2(self._project_conv(x))
        if self.stride == 1 and self.in_f == self.out_f:
            if drop_connect_rate:
                x = drop_connect(x, drop_connect_rate, self.training)
            x = x + inputs
        return x


def set_depthwise_fp32(module: nn.Module, flag: bool = True) -> None:
    for m in module.modules():
        if isinstance(m, MBConvBlock):
            m.depthwise_fp32 = flag


def set_depthwise_native(module: nn.Module, flag: bool = True) -> None:
    for m in module.modules():
        if isinstance(m, MBConvBlock):
            m.depthwise_native = flag


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

    @staticmethod
    def _swish(x: torch.Tensor) -> torch.Tensor:
        return F.silu(x)

    def forward(self, x: torch.Tensor) -> torch.Tensor:  # classification head (unused by LSS)
        x = self._swish(self._bn0(self._conv_stem(x)))
        for idx, block in enumerate(self._blocks):
            x = block(x, self._global_params.drop_connect_rate * idx / len(self._blocks))
        x = self._swish(self._bn1(self._conv_head(x)))
        return self._fc(self._dropout(self._avg_pooling(x).flatten(1)))
