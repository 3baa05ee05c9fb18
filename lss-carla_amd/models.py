"""LiftSplatShoot with the reference's module surface, MI355X-native hot path.

Drop-in for ``src/models.py`` of shdragron/LSS-Carla:

* ``compile_model(grid_conf, data_aug_conf, outC)`` / ``LiftSplatShoot(...)`` with
  the same dict schemas (``src/models.py:133-155, 262``);
* ``forward(x, rots, trans, intrins, post_rots, post_trans)`` -> (B, outC, X, Y)
  logits (``src/models.py:256-259``);
* the same attribute and state_dict names: ``dx``, ``bx``, ``nx``, ``frustum``
  (non-trainable Parameters), ``camencode.trunk.*`` (efficientnet_pytorch names),
  ``camencode.up1.*``, ``camencode.depthnet.*``, ``bevencode.*`` (torchvision
  resnet18 names); ``use_quickcumsum`` and ``get_geometry``/``get_cam_feats``/
  ``voxel_pooling``/``get_voxels`` keep their signatures.

What runs where: geometry, voxel assignment, the lift (depth softmax x context
outer product) and the splat run as gfx950 HIP kernels (``ops.py`` ->
``liblss_hip.so``); the EfficientNet-B0 trunk and the ResNet-18 BEV encoder are
stock PyTorch-ROCm modules (MIOpen / MFMA). The hot path refuses CPU tensors.

Extra knobs (not in the reference, defaults reproduce it):
  ``bev_layout``     'nhwc' (default: channels-last BEV strides, feeds a channels-last BevEncode
                     without a transpose) or 'nchw' (the reference's contiguous strides). Same shape and
                     values either way; strides are not part of the reference interface
  ``static_inverses`` (pinv, kinv) device buffers staged from the host's torch.inverse before a
                     captured step (ops.HostInverses); None: computed per forward, as the reference
  ``fuse_depthnet``  under bf16 autocast, run the depthnet 1x1 conv inside the lift kernel
                     (MFMA); off: the conv runs as its own op (MIOpen)
"""
from __future__ import annotations

import os
import sys

import torch
import torch.nn.functional as F
from torch import nn

from . import _lib, ops
from .efficientnet import EfficientNetB0
from . import resample
from . import norm
from .norm import bn_act
from .tools import gen_dx_bx

# CamEncode.up1 on channels-last maps under bf16 autocast (see get_eff_depth); False: NCHW (the unfused
# channel-plane lift, k_depthnet_lift2; tests switch it)
UP1_CHANNELS_LAST = True


# Stride-1 3x3 convolutions (BevEncode's layer1-3 / up1 / up2 convs, CamEncode.up1) with the backward-data
# pass run as a FORWARD convolution of dy with the flipped, transposed weight (dx = conv2d(dy, W'),
# W'[i, o, a, b] = W[o, i, 2 - a, 2 - b]: the transposed convolution of stride 1, padding 1). MIOpen's
# find gives these shapes its CK forward kernels (0.29-0.33 of the bf16 MFMA peak at c3) where its
# backward-data solvers (ASM implicit GEMM) run at 0.13-0.29; the weight gradient stays MIOpen's.
USE_FLIP_BWD = True


def _flip_eligible(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    return (USE_FLIP_BWD and x.is_cuda and x.dim() == 4 and conv.kernel_size == (3, 3) and conv.stride == (1, 1)
            and conv.padding == (1, 1) and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None
            and conv.padding_mode == "zeros" and torch.is_grad_enabled()
            and (x.requires_grad or conv.weight.requires_grad))


class _Conv3x3(torch.autograd.Function):
    """conv2d(x, w, stride 1, padding 1); backward-data as conv2d(dy, flip(w^T)) (see USE_FLIP_BWD)."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.bfloat16)
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return F.conv2d(x, w, None, 1, 1)

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        need = ctx.needs_input_grad
        dx = dw = None
        if need[0]:
            dx = F.conv2d(dy, _flip_weight(w), None, 1, 1)
        if need[1]:
            dw = torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                                     [False, True, False])[1]
        return dx, dw


def _flip_weight(w: torch.Tensor) -> torch.Tensor:
    """W'[i, o, a, b] = W[o, i, 2 - a, 2 - b], channels-last, in one lss_conv_flip_weight launch."""
    O, I, K, _ = w.shape
    if w.is_contiguous(memory_format=torch.channels_last):
        lay = _lib.NHWC
    else:
        w, lay = w.contiguous(), _lib.NCHW
    wt = torch.empty(I, O, K, K, device=w.device, dtype=w.dtype, memory_format=torch.channels_last)
    lib = _lib.load()
    _lib.check(lib.lss_conv_flip_weight(_lib.ptr(w), _lib.dtype_code(w.dtype), O, I, K, lay, _lib.ptr(wt),
                                        _lib.stream_handle(w.device)), "lss_conv_flip_weight")
    return wt


def conv3x3(conv: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    """conv(x), through _Conv3x3 where eligible (same parameters, same forward)."""
    if _flip_eligible(conv, x):
        return _Conv3x3.apply(x, conv.weight)
    return conv(x)


class Up(nn.Module):
    """Upsample x1, concatenate with x2, two conv-BN-ReLU (src/models.py:15-34)."""

    def __init__(self, in_channels, out_channels, scale_factor=2):
        super().__init__()
        self.up = nn.Upsample(scale_factor=scale_factor, mode="bilinear", align_corners=True)
        self.conv = nn.Sequential(
            nn.Conv2d(in_channels, out_channels, kernel_size=3, padding=1, bias=False),
            nn.BatchNorm2d(out_channels),
            nn.ReLU(inplace=True),
            nn.Conv2d(out_channels, out_channels, kernel_size=3, padding=1, bias=False),
            nn.BatchNorm2d(out_channels),
            nn.ReLU(inplace=True),
        )

    def forward(self, x1, x2):
        c = self.conv  # conv-BN-ReLU twice; BN + ReLU fused (lss_bn_*)
        if resample.USE_HIP_UPSAMPLE and resample._eligible(x1) and resample._eligible(x2):
            # channels-last bf16 (BevEncode under autocast): upsample + cat in one kernel
            x = resample.upsample_cat(x1, x2, int(self.up.scale_factor))
            x = bn_act(c[1], conv3x3(c[0], x), "relu")
            return bn_act(c[4], conv3x3(c[3], x), "relu")
        if x1.is_cuda and not x1.is_contiguous(memory_format=torch.channels_last):
            # PyTorch's NCHW bilinear kernel parallelises over output pixels only (a 8x22 map:
            # 176 threads, each looping over N*C); the channels-last kernel covers every element.
            x1 = self.up(x1.contiguous(memory_format=torch.channels_last)).contiguous()
        else:
            x1 = self.up(x1)
        x = bn_act(c[1], conv3x3(c[0], torch.cat([x2, x1], dim=1)), "relu")
        return bn_act(c[4], conv3x3(c[3], x), "relu")


_TRUNK_WEIGHTS_NOTED = set()


def _note_trunk_weights(path: str) -> None:
    """Say once per path (stderr) that the trunk starts from local weights: the environment variable
    changes every model built in the process, parity and benchmark runs included."""
    if path not in _TRUNK_WEIGHTS_NOTED:
        _TRUNK_WEIGHTS_NOTED.add(path)
        print(f"[lss_carla_amd] CamEncode trunk: EfficientNet-B0 weights from {path} "
              "($LSS_EFFICIENTNET_B0_WEIGHTS)", file=sys.stderr, flush=True)


class _HipDropout(torch.autograd.Function):
    """Training-mode dropout on ``lss_dropout`` (include/lss_convs.h): the mask is a function of a 64-bit
    seed drawn from torch's CUDA generator (graph-capturable) and the element index, so the backward
    regenerates it instead of saving it."""

    @staticmethod
    def forward(ctx, x, p, prefetch):
        lib = _lib.load()
        seed = torch.randint(0, 2 ** 62, (1,), device=x.device, dtype=torch.int64)
        y = torch.empty_like(x)
        keep = 1.0 - p
        pf_bytes = prefetch.numel() * prefetch.element_size() if prefetch is not None else 0
        _lib.check(lib.lss_dropout(_lib.ptr(x), _lib.dtype_code(x.dtype), x.numel(), _lib.ptr(seed), keep, _lib.ptr(y),
                                   _lib.ptr(prefetch) if pf_bytes else None, pf_bytes, _lib.stream_handle(x.device)),
                   "lss_dropout")
        ctx.save_for_backward(seed)
        ctx.keep = keep
        # the mask follows the elements' memory order: the gradient is read in the input's format
        ctx.fmt = torch.contiguous_format if x.is_contiguous() else torch.channels_last
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _lib.load()
        (seed,) = ctx.saved_tensors
        fmt = ctx.fmt
        dy = dy.contiguous(memory_format=fmt)
        if dy.data_ptr() % 16:
            dy = dy.clone(memory_format=fmt)
        dx = torch.empty_like(dy)
        _lib.check(lib.lss_dropout(_lib.ptr(dy), _lib.dtype_code(dy.dtype), dy.numel(), _lib.ptr(seed), ctx.keep,
                                   _lib.ptr(dx), None, 0, _lib.stream_handle(dy.device)), "lss_dropout")
        return dx, None, None


USE_HIP_DROPOUT = True
# where the plan kernels run: "trunk" (in front of the trunk), "dropout" (between the trunk's last conv
# and the dropout), "lift" (between the dropout and the fused lift)
PLAN_AT = "dropout"


class LssDropout(nn.Dropout):
    """``nn.Dropout`` (same attributes, no state) whose training-mode CUDA forward is ``lss_dropout``:
    the same Bernoulli(1 - p) mask distribution and 1 / (1 - p) scaling as torch's (not the same draws),
    written in the XCD-contiguous eighths the fused lift reads, and warming the lift's packed weights
    (``prefetch``, set by ``LiftSplatShoot.get_voxels``) into every XCD's L2."""

    prefetch = None

    def forward(self, x):
        if (USE_HIP_DROPOUT and self.training and 0.0 < self.p < 1.0 and x.is_cuda
                and x.dtype in (torch.float32, torch.bfloat16) and x.data_ptr() % 16 == 0
                and (x.numel() * x.element_size()) % 16 == 0
                and (x.is_contiguous() or (x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)))):
            pf = self.prefetch if self.prefetch is not None and self.prefetch.device == x.device else None
            return _HipDropout.apply(x, self.p, pf)
        return super().forward(x)


class CamEncode(nn.Module):
    """Image -> depthnet output (src/models.py:37-89)."""

    def __init__(self, D, C, downsample):
        super().__init__()
        self.D, self.C = D, C
        # src/models.py:43 loads ImageNet weights with EfficientNet.from_pretrained("efficientnet-b0"),
        # a download; here they come from a local file when $LSS_EFFICIENTNET_B0_WEIGHTS names one
        # (an unchanged train_simbev.py then trains from them), else the trunk is randomly initialised
        wpath = os.environ.get("LSS_EFFICIENTNET_B0_WEIGHTS")
        if wpath:
            _note_trunk_weights(wpath)
        self.trunk = EfficientNetB0.from_pretrained("efficientnet-b0", wpath) if wpath else EfficientNetB0()
        self.up1 = Up(320 + 112, 512)
        self.dropout = LssDropout(0.2)
        self.depthnet = nn.Conv2d(512, self.D + self.C, kernel_size=1, padding=0)

    def get_eff_depth(self, x):
        """Endpoints reduction_4 / reduction_5 of the trunk, fused by ``up1`` (src/models.py:63-84)."""
        t = self.trunk
        x = bn_act(t._bn0, t._conv_stem(x), "swish")
        endpoints = []
        prev = x
        nblk = len(t._blocks)
        for idx, block in enumerate(t._blocks):
            rate = t._global_params.drop_connect_rate
            if rate:
                rate *= float(idx) / nblk
            x = block(x, drop_connect_rate=rate)
            if prev.size(2) > x.size(2):
                endpoints.append(prev)
            prev = x
        endpoints.append(x)
        x5, x4 = endpoints[4], endpoints[3]
        if UP1_CHANNELS_LAST and x5.is_cuda and x5.dtype == torch.bfloat16 and x4.dtype == torch.bfloat16:
            # up1 channels-last (bf16 autocast): upsample + cat in one kernel, NHWC convs without
            # layout transposes, and a pixel-major feature map -- each pixel's 512 channels one
            # contiguous row -- for the fused depthnet lift (lss_depthnet_lift_nhwc)
            x5 = x5.contiguous(memory_format=torch.channels_last)
            x4 = x4.contiguous(memory_format=torch.channels_last)
        return self.up1(x5, x4)

    def depthnet_out(self, x):
        """(B*N, 3, H, W) images -> (B*N, D+C, H/16, W/16) depth logits + context."""
        return self.depthnet(self.dropout(self.get_eff_depth(x)))

    def get_depth_dist(self, x, eps=1e-20):
        return x.softmax(dim=1)

    def get_depth_feat(self, x):
        """(depth, lifted features) as the reference returns them (src/models.py:52-61).

        API compatibility only: the training forward never materialises the lifted
        volume (the lift is fused into the splat kernel).
        """
        x = self.depthnet_out(x)
        depth = self.get_depth_dist(x[:, :self.D])
        new_x = depth.unsqueeze(1) * x[:, self.D:(self.D + self.C)].unsqueeze(2)
        return depth, new_x

    def forward(self, x):
        return self.get_depth_feat(x)[1]


class BasicBlock(nn.Module):
    """torchvision ResNet BasicBlock (names conv1/bn1/conv2/bn2/downsample)."""
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        if self.downsample is None:
            identity = x
        else:
            identity = bn_act(self.downsample[1], conv1x1(self.downsample[0], x))
        out = bn_act(self.bn1, conv3x3(self.conv1, x), "relu")
        return bn_act(self.bn2, conv3x3(self.conv2, out), "relu", residual=identity)


def _resnet_layer(inplanes, planes, blocks, stride):
    down = None
    if stride != 1 or inplanes != planes:
        down = nn.Sequential(nn.Conv2d(inplanes, planes, 1, stride, bias=False), nn.BatchNorm2d(planes))
    layers = [BasicBlock(inplanes, planes, stride, down)]
    layers += [BasicBlock(planes, planes) for _ in range(1, blocks)]
    return nn.Sequential(*layers)


class _Head1x1(torch.autograd.Function):
    """A 1x1 conv to ONE output channel over channels-last bf16 maps on lss_head1_* (include/lss_convs.h):
    as a GEMM it is a GEMV whose weight gradient -- a reduction over every pixel of the BEV -- ran on a
    handful of hipBLASLt workgroups (~210 us per c3 step); here one pass over the input each way."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.bfloat16)
    def forward(ctx, x, weight, bias):
        lib = _lib.load()
        N, C, H, W = x.shape
        x = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = weight.detach().to(torch.bfloat16).reshape(C).float()  # the bf16 operand, as fp32
        b = bias.detach().to(torch.bfloat16).float().reshape(1) if bias is not None else None
        y = torch.empty(N, 1, H, W, device=x.device, dtype=torch.bfloat16)
        _lib.check(lib.lss_head1_fwd(_lib.ptr(x), _lib.ptr(w), _lib.ptr(b), N * H * W, C, _lib.ptr(y),
                                     _lib.stream_handle(x.device)), "lss_head1_fwd")
        ctx.save_for_backward(x, w)
        ctx.meta = (weight.shape, weight.dtype, None if bias is None else bias.dtype)
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dy):
        lib = _lib.load()
        x, w = ctx.saved_tensors
        wshape, wdtype, bdtype = ctx.meta
        N, C, H, W = x.shape
        P = N * H * W
        dy = dy.to(torch.bfloat16).contiguous()
        dx = torch.empty_like(x)  # channels-last, as x
        part = torch.empty(int(lib.lss_head1_blocks(P)), C + 1, device=x.device, dtype=torch.float32)
        _lib.check(lib.lss_head1_bwd(_lib.ptr(x), _lib.ptr(dy), _lib.ptr(w), P, C, _lib.ptr(dx), _lib.ptr(part),
                                     _lib.stream_handle(x.device)), "lss_head1_bwd")
        tot = part.sum(0)
        dw = tot[:C].reshape(wshape).to(wdtype)
        db = tot[C:].to(bdtype) if bdtype is not None else None
        return dx, dw, db


def _head1_eligible(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    C = x.shape[1] if x.dim() == 4 else 0
    bf16 = x.dtype == torch.bfloat16 or (torch.is_autocast_enabled("cuda")
                                          and torch.get_autocast_dtype("cuda") == torch.bfloat16)
    return (USE_HIP_HEAD1 and conv.out_channels == 1 and x.is_cuda and x.dim() == 4 and bf16 and C % 8 == 0
            and C // 8 > 0 and 64 % (C // 8) == 0 and x.is_contiguous(memory_format=torch.channels_last))


USE_HIP_HEAD1 = True  # BevEncode's last conv (one output channel) on lss_head1_* instead of a hipBLASLt GEMV
# BevEncode's up2 tail, BN + ReLU + that conv, without the normalised map (_BnReluHead1)
USE_BN_HEAD = True


class _BnReluHead1(torch.autograd.Function):
    """conv1x1_to_one_channel(relu(bn(x))) for channels-last bf16 maps in training mode (BevEncode.up2[2:5],
    src/models.py:111-115), the normalised map never written: lss_bn_fwd2 with y = NULL (statistics,
    running stats), then lss_head1_fwd2 applies scale / shift / ReLU to each value as it reads x (the
    value the BN apply would have stored); backward: lss_head1_bwd2 (head weight / bias gradients from
    the recomputed map, no input gradient written) and lss_bn_bwd_rank1 (the BN backward with the head's
    gradient bf16(dout[p] w[c]) computed in its kernels). The same kernels' arithmetic in the same order
    as bn_act + _Head1x1: bit-identical outputs and gradients (tests/test_gpu_convs.py). At c3 this
    skips 82 MB written and 82 MB read in the forward, 82 MB written and 164 MB read in the backward."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda")
    def forward(ctx, x, gamma, beta, hw, hb, bn: nn.BatchNorm2d):
        lib = _lib.load()
        N, C, H, W = x.shape
        HW, P = H * W, N * H * W
        dev = x.device
        st = _lib.stream_handle(dev)
        groups = int(lib.lss_bn_groups(N, C, HW, norm.NHWC))
        f32 = dict(device=dev, dtype=torch.float32)
        partial = torch.empty(C, groups, 2, **f32)
        stats = torch.empty(4, C, **f32)  # save_mean, save_rstd, scale, shift
        momentum, counter, rm, rv = norm.running_args(bn)
        _lib.check(lib.lss_bn_fwd2(_lib.ptr(x), None, _lib.BF16, norm.NHWC, N, C, HW, _lib.ptr(gamma), _lib.ptr(beta),
                                   float(bn.eps), float(momentum), _lib.ptr(rm), _lib.ptr(rv), _lib.ptr(counter),
                                   norm.ACT["relu"], groups, _lib.ptr(partial), _lib.ptr(stats[0]), _lib.ptr(stats[1]),
                                   _lib.ptr(stats[2]), _lib.ptr(stats[3]), None, None, st), "lss_bn_fwd2")
        w = hw.detach().to(torch.bfloat16).reshape(C).float()  # the bf16 operands, as _Head1x1 takes them
        b = hb.detach().to(torch.bfloat16).float().reshape(1) if hb is not None else None
        y = torch.empty(N, 1, H, W, device=dev, dtype=torch.bfloat16)
        _lib.check(lib.lss_head1_fwd2(_lib.ptr(x), _lib.ptr(w), _lib.ptr(b), P, C, _lib.ptr(stats), _lib.ptr(y), st),
                   "lss_head1_fwd2")
        ctx.save_for_backward(x, stats, w)
        # under autocast the head's operands are its bf16 casts, so its parameter gradients come back
        # rounded to bf16 (as _Head1x1's, whose inputs autocast casts)
        cast = torch.is_autocast_enabled("cuda")
        ctx.meta = (groups, hw.shape, torch.bfloat16 if cast else hw.dtype, hw.dtype,
                    None if hb is None else (torch.bfloat16 if cast else hb.dtype), None if hb is None else hb.dtype)
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dout):
        lib = _lib.load()
        x, stats, w = ctx.saved_tensors
        groups, wshape, wdtype, wdtype_out, bdtype, bdtype_out = ctx.meta
        N, C, H, W = x.shape
        P = N * H * W
        dev = x.device
        st = _lib.stream_handle(dev)
        dout = dout.to(torch.bfloat16).contiguous()
        part = torch.empty(int(lib.lss_head1_blocks(P)), C + 1, device=dev, dtype=torch.float32)
        _lib.check(lib.lss_head1_bwd2(_lib.ptr(x), _lib.ptr(dout), _lib.ptr(w), P, C, _lib.ptr(stats), None,
                                      _lib.ptr(part), st), "lss_head1_bwd2")
        tot = part.sum(0)
        dw = tot[:C].reshape(wshape).to(wdtype).to(wdtype_out)
        db = tot[C:].to(bdtype).to(bdtype_out) if bdtype is not None else None
        f32 = dict(device=dev, dtype=torch.float32)
        partial = torch.empty(C, groups, 2, **f32)
        coef = torch.empty(C, 2, **f32)
        dgamma = torch.empty(C, **f32)
        dbeta = torch.empty(C, **f32)
        dx = torch.empty_like(x)
        _lib.check(lib.lss_bn_bwd_rank1(_lib.ptr(dout), _lib.ptr(w), _lib.ptr(x), N, C, H * W, _lib.ptr(stats[2]),
                                        _lib.ptr(stats[3]), _lib.ptr(stats[0]), _lib.ptr(stats[1]), norm.ACT["relu"],
                                        groups, _lib.ptr(partial), _lib.ptr(coef), _lib.ptr(dgamma), _lib.ptr(dbeta),
                                        _lib.ptr(dx), st), "lss_bn_bwd_rank1")
        return dx, dgamma, dbeta, dw, db, None


def bn_relu_head1(bn: nn.BatchNorm2d, head: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    """head(relu(bn(x))) with head a 1x1 conv to one channel: _BnReluHead1 where eligible (the benched
    BevEncode: training mode, channels-last bf16 under autocast), else bn_act + conv1x1."""
    C = x.shape[1] if x.dim() == 4 else 0
    ok = (USE_BN_HEAD and norm.USE_HIP_BN and USE_HIP_HEAD1 and bn.training and bn.affine and x.is_cuda
          and x.dim() == 4 and x.dtype == torch.bfloat16 and x.is_contiguous(memory_format=torch.channels_last)
          and head.out_channels == 1 and head.kernel_size == (1, 1) and head.stride == (1, 1) and head.groups == 1
          and C % 8 == 0 and 64 % (C // 8) == 0 and 256 % (C // 8) == 0 and _head1_eligible(head, x))
    if not ok:
        return conv1x1(head, bn_act(bn, x, "relu"))
    return _BnReluHead1.apply(x, bn.weight, bn.bias, head.weight, head.bias, bn)


class _Subsample(torch.autograd.Function):
    """x[:, :, ::s, ::s] as a channels-last copy (what F.linear over the pixels needs anyway), its gradient
    scattered into one zero-filled map: two SliceBackward nodes each allocated, zero-filled and copied a
    map of their own (the H slice's at full size), and matmul cloned the strided view in the forward."""

    @staticmethod
    def forward(ctx, x, s):
        fmt = torch.contiguous_format if x.is_contiguous() else torch.channels_last
        ctx.meta = (x.shape, s, fmt)
        return x[:, :, ::s, ::s].contiguous(memory_format=torch.channels_last)

    @staticmethod
    def backward(ctx, g):
        shape, s, fmt = ctx.meta
        dx = torch.empty(shape, device=g.device, dtype=g.dtype, memory_format=fmt).zero_()
        dx[:, :, ::s, ::s] = g
        return dx, None


def conv1x1(conv: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    """A 1x1 nn.Conv2d (stride s, no padding) applied as a GEMM over the channels of every s-th pixel
    (F.linear: hipBLASLt) on CUDA maps, with the module's own weight and bias (same math). MIOpen's
    channels-last 1x1 backward is not safe to replay from a hipGraph: from the second replay of the
    captured training step on, the weight gradient of BevEncode's last conv (up2.4, 128 -> outC = 1
    channels, src/models.py:115) came out as garbage (1e35 / 1e-31), and that of the depthnet's 1x1
    conv on channels-last features as zeros (tests/test_gpu_captured_step.py). BevEncode's stride-2
    downsample convs (torchvision BasicBlock, layer2 / layer3) are channels-last 1x1 convs too and
    take this path for the same reason."""
    if not (x.is_cuda and x.dim() == 4) or conv.kernel_size != (1, 1) or conv.groups != 1 \
            or conv.stride[0] != conv.stride[1] or conv.padding not in ((0, 0), "valid"):
        return conv(x)
    s = conv.stride[0]
    if s == 1 and _head1_eligible(conv, x):
        return _Head1x1.apply(x, conv.weight, conv.bias)
    if s > 1:
        x = _Subsample.apply(x, s)
    w = conv.weight.reshape(conv.out_channels, conv.in_channels)
    y = F.linear(x.permute(0, 2, 3, 1), w, conv.bias)  # (N, H, W, O)
    return y.permute(0, 3, 1, 2)  # (N, O, H, W), channels-last strides


def _dropout2d_scale(d: nn.Dropout2d, x: torch.Tensor):
    """The (N, C) factor nn.Dropout2d multiplies x by (0 or 1 / (1 - p) per image and channel, drawn the
    way torch's feature dropout draws it: bernoulli_(1 - p) then div_(1 - p) in x's dtype), or None when
    it is the identity (eval, p = 0)."""
    if not d.training or d.p == 0:
        return None
    if d.p == 1:
        return torch.zeros(x.shape[0], x.shape[1], device=x.device)
    noise = torch.empty(x.shape[0], x.shape[1], device=x.device, dtype=x.dtype)
    return noise.bernoulli_(1 - d.p).div_(1 - d.p).float()


class BevEncode(nn.Module):
    """ResNet-18 stem + layer1-3 + two Up stages (src/models.py:92-130).

    Initialised like ``torchvision.models.resnet18(pretrained=False,
    zero_init_residual=True)`` for the parts taken from it (kaiming fan_out convs,
    unit BN, zeroed last BN of every residual block); ``conv1`` and the Up stages
    keep PyTorch defaults as in the reference.
    """

    def __init__(self, inC, outC):
        super().__init__()
        # registration order = the reference's (parameters() order keys optimizer state)
        self.conv1 = nn.Conv2d(inC, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.layer1 = _resnet_layer(64, 64, 2, 1)
        self.layer2 = _resnet_layer(64, 128, 2, 2)
        self.layer3 = _resnet_layer(128, 256, 2, 2)
        for m in (self.bn1, self.layer1, self.layer2, self.layer3):
            for mm in m.modules():
                if isinstance(mm, nn.Conv2d):
                    nn.init.kaiming_normal_(mm.weight, mode="fan_out", nonlinearity="relu")
                elif isinstance(mm, nn.BatchNorm2d):
                    nn.init.constant_(mm.weight, 1)
                    nn.init.constant_(mm.bias, 0)
        for mm in self.modules():
            if isinstance(mm, BasicBlock):
                nn.init.constant_(mm.bn2.weight, 0)
        self.up1 = Up(64 + 256, 256, scale_factor=4)
        self.dropout = nn.Dropout2d(0.1)
        self.up2 = nn.Sequential(
            nn.Upsample(scale_factor=2, mode="bilinear", align_corners=True),
            nn.Conv2d(256, 128, kernel_size=3, padding=1, bias=False),
            nn.BatchNorm2d(128),
            nn.ReLU(inplace=True),
            nn.Conv2d(128, outC, kernel_size=1, padding=0),
        )

    def forward(self, x):
        x = bn_act(self.bn1, self.conv1(x), "relu")
        x1 = self.layer1(x)
        x = self.layer3(self.layer2(x1))
        x = self.up1(x, x1)
        u = self.up2  # Upsample, conv, BN, ReLU, conv
        if resample.USE_HIP_UPSAMPLE and resample._eligible(x):
            # Dropout2d folded into the upsample: its (N, C) mask scales the interpolated channels (and
            # the gradient) inside lss_upsample_cat_fwd2 / lss_upsample_bwd2, not as two passes over x
            x = resample.upsample_cat(x, None, int(u[0].scale_factor), _dropout2d_scale(self.dropout, x))
        else:
            x = u[0](self.dropout(x))
        return bn_relu_head1(u[2], u[4], conv3x3(u[1], x))


class LiftSplatShoot(nn.Module):
    def __init__(self, grid_conf, data_aug_conf, outC):
        super().__init__()
        self.grid_conf = grid_conf
        self.data_aug_conf = data_aug_conf
        dx, bx, nx = gen_dx_bx(grid_conf["xbound"], grid_conf["ybound"], grid_conf["zbound"])
        self.dx = nn.Parameter(dx, requires_grad=False)
        self.bx = nn.Parameter(bx, requires_grad=False)
        self.nx = nn.Parameter(nx, requires_grad=False)
        self.downsample = 16
        self.camC = 64
        self.frustum = self.create_frustum()
        self.D, _, _, _ = self.frustum.shape
        self.camencode = CamEncode(self.D, self.camC, self.downsample)
        self.bevencode = BevEncode(inC=self.camC, outC=outC)
        # toggle kept for API compatibility (src/models.py:155); both settings run the same kernels.
        self.use_quickcumsum = True
        # channels-last BEV by default, also for the reference's own fp32 training (train_simbev.py
        # runs without autocast): c3 fp32 step 268.1 vs 255.8 frames/s, its splat 17.1 vs 20.8 us in the
        # graph replays (0.64 vs 0.53 of HBM); c2 fp32 forward 660.9 vs 639.8 (profiles/r05)
        self.bev_layout = "nhwc"
        # BevEncode's weights channels-last too (same values and state_dict), so its convolutions take
        # the BEV as it comes instead of converting a weight per call
        self.bevencode.to(memory_format=torch.channels_last)
        self.fuse_depthnet = True  # bf16 autocast: depthnet conv fused into the lift kernel
        # (pinv, kinv) device buffers filled from host torch.inverse by ops.HostInverses before the
        # step (captured training step); None: get_voxels computes them (host torch.inverse)
        self.static_inverses = None
        self._grid = ops.GridSpec.from_conf(grid_conf)

    def create_frustum(self):
        """(D, fH, fW, 3) grid of (u, v, depth), built on the host with torch (src/models.py:157-168)."""
        ogfH, ogfW = self.data_aug_conf["final_dim"]
        fH, fW = ogfH // self.downsample, ogfW // self.downsample
        ds = torch.arange(*self.grid_conf["dbound"], dtype=torch.float).view(-1, 1, 1).expand(-1, fH, fW)
        D, _, _ = ds.shape
        xs = torch.linspace(0, ogfW - 1, fW, dtype=torch.float).view(1, 1, fW).expand(D, fH, fW)
        ys = torch.linspace(0, ogfH - 1, fH, dtype=torch.float).view(1, fH, 1).expand(D, fH, fW)
        return nn.Parameter(torch.stack((xs, ys, ds), -1), requires_grad=False)

    # ------------------------------------------------------------------ hot path pieces
    def _layout(self) -> int:
        return _lib.NHWC if self.bev_layout == "nhwc" else _lib.NCHW

    def _bev_dtype(self, device) -> torch.dtype:
        if device.type == "cuda" and torch.is_autocast_enabled("cuda"):
            return torch.get_autocast_dtype("cuda")
        return torch.float32

    def plan(self, rots, trans, intrins, post_rots, post_trans, want_geom=False) -> ops.SplatPlan:
        """Geometry + voxel assignment + CSR of points by cell for one batch of rigs."""
        return ops.plan_from_cameras(self.frustum, rots, trans, intrins, post_rots, post_trans, self._grid,
                                     want_geom=want_geom)

    def get_geometry(self, rots, trans, intrins, post_rots, post_trans):
        """(B, N, D, fH, fW, 3) ego-frame points (src/models.py:170-190), HIP kernel."""
        p = ops.plan_from_cameras(self.frustum, rots, trans, intrins, post_rots, post_trans, self._grid,
                                  want_geom=True, want_csr=False)
        return p.geom

    def get_cam_feats(self, x):
        """(B, N, D, fH, fW, C) lifted features (src/models.py:192-202); API compatibility."""
        B, N, C, imH, imW = x.shape
        x = self.camencode(x.view(B * N, C, imH, imW))
        x = x.view(B, N, self.camC, self.D, imH // self.downsample, imW // self.downsample)
        return x.permute(0, 1, 3, 4, 5, 2)

    def voxel_pooling(self, geom_feats, x):
        """Splat given geometry + lifted features (src/models.py:204-246), HIP kernels."""
        B, N, D, H, W, C = x.shape
        plan = ops.plan_from_geom(geom_feats, self._grid)
        return ops.voxel_pool_rows(x.reshape(B * N * D * H * W, C), plan, self._layout())

    def get_voxels(self, x, rots, trans, intrins, post_rots, post_trans):
        """Fused hot path: trunk, geometry/CSR, lift+splat (src/models.py:248-254).

        Schedule: the camera inverses first (the host's torch.inverse copies the rig to the host,
        which must not wait behind the trunk), then the trunk, the plan kernels, the dropout (it writes
        the features where the fused lift's blocks read them, right before the lift), then the fused
        lift and the splat (the plan's CSR still in the L2s).
        """
        B, N, C, imH, imW = x.shape
        inv = self.static_inverses
        if inv is None:
            inv = ops.camera_inverses(post_rots, intrins)
        ce = self.camencode
        plan = None

        def make_plan():
            return ops.plan_from_cameras(self.frustum, rots, trans, intrins, post_rots, post_trans, self._grid,
                                         inverses=inv)

        if PLAN_AT == "trunk":
            plan = make_plan()
        out_dtype = self._bev_dtype(x.device)
        fused = self.fuse_depthnet and out_dtype == torch.bfloat16 and self.D + self.camC <= 128
        packed = None
        if fused:
            w = ce.depthnet.weight
            pk = getattr(ce.depthnet, "lss_packed_weight", None)  # (buffer, the bf16 view's address)
            packed = pk[0] if pk is not None and w.dtype == torch.bfloat16 and w.data_ptr() == pk[1] else None
        ce.dropout.prefetch = packed
        try:
            feat = ce.get_eff_depth(x.view(B * N, C, imH, imW))
            if PLAN_AT == "dropout":
                plan = make_plan()
            feat = ce.dropout(feat)
        finally:
            ce.dropout.prefetch = None
        if plan is None:
            plan = make_plan()
        if fused:
            # depthnet 1x1 conv + softmax + context layout in one MFMA kernel; its
            # tile holds D + C <= 128 output channels (a larger dbound runs the conv as its own op)
            return ops.depthnet_lift_splat(feat, w, ce.depthnet.bias, plan, out_dtype, self._layout(), packed)
        return ops.lift_splat(ce.depthnet(feat), plan, out_dtype, self._layout())

    def forward(self, x, rots, trans, intrins, post_rots, post_trans):
        x = self.get_voxels(x, rots, trans, intrins, post_rots, post_trans)
        return self.bevencode(x)


def compile_model(grid_conf, data_aug_conf, outC):
    return LiftSplatShoot(grid_conf, data_aug_conf, outC)
