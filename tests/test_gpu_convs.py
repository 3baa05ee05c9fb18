"""HIP depthwise convolutions of the EfficientNet-B0 trunk (include/lss_convs.h) vs an fp64
PyTorch reference of the same op (conv2d with groups = C after the static-same zero padding)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs an MI355X", allow_module_level=True)

from lss_carla_amd import efficientnet as E  # noqa: E402

DEV = torch.device("cuda:0")

# (K, stride, (left, right, top, bottom) pads, H, W): the B0 depthwise layers at 128x352 input, plus odd sizes
CASES = [
    (3, 1, (1, 1, 1, 1), 64, 176),
    (3, 2, (0, 1, 0, 1), 64, 176),
    (5, 2, (1, 2, 1, 2), 32, 88),
    (5, 1, (2, 2, 2, 2), 16, 44),
    (3, 2, (0, 1, 0, 1), 16, 44),
    (5, 1, (2, 2, 2, 2), 8, 22),
    (5, 2, (1, 2, 1, 2), 8, 22),
    (3, 1, (1, 1, 1, 1), 4, 11),
    (5, 1, (2, 2, 2, 2), 4, 11),
    (5, 2, (2, 2, 2, 2), 7, 9),
]


def _reference(x, w, stride, pads, dy):
    xr = x.detach().cpu().double().requires_grad_(True)
    wr = w.detach().cpu().double().requires_grad_(True)
    y = F.conv2d(F.pad(xr, pads), wr, stride=stride, groups=x.shape[1])
    y.backward(dy.detach().cpu().double())
    return y.detach(), xr.grad, wr.grad


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("K,stride,pads,H,W", CASES)
def test_depthwise_fwd_bwd_vs_fp64(K, stride, pads, H, W, dtype):
    g = torch.Generator().manual_seed(K * 100 + stride * 10 + H)
    N, C = 3, 24
    x = torch.randn(N, C, H, W, generator=g).to(dtype)
    w = torch.randn(C, 1, K, K, generator=g) * 0.2
    xd = x.to(DEV).requires_grad_(True)
    wd = w.to(DEV).requires_grad_(True)
    y = E._HipDepthwise.apply(xd, wd, stride, pads)
    dy = torch.randn(y.shape, generator=g).to(dtype)
    y.backward(dy.to(DEV))
    y_ref, dx_ref, dw_ref = _reference(x, w, stride, pads, dy)
    assert y.shape == y_ref.shape and y.dtype == dtype
    tol = dict(rtol=1e-5, atol=1e-5) if dtype == torch.float32 else dict(rtol=1e-2, atol=2e-2)
    torch.testing.assert_close(y.detach().cpu().double(), y_ref, **tol)
    torch.testing.assert_close(xd.grad.cpu().double(), dx_ref, **tol)
    assert wd.grad.dtype == torch.float32  # fp32 accumulation into the fp32 parameter's gradient
    torch.testing.assert_close(wd.grad.cpu().double(), dw_ref, rtol=1e-4, atol=1e-3 if dtype == torch.float32 else 5e-2)


def test_trunk_hip_vs_miopen_depthwise():
    """The whole B0 trunk (16 MBConv blocks, real paddings) with either depthwise backend, fp32."""
    torch.manual_seed(0)
    trunk = E.EfficientNetB0().to(DEV).eval()
    x = torch.randn(2, 3, 128, 352, device=DEV)
    outs = []
    for impl in ("hip", "miopen"):
        E.set_depthwise_impl(trunk, impl)
        trunk.zero_grad(set_to_none=True)
        h = trunk._swish(trunk._bn0(trunk._conv_stem(x)))
        for blk in trunk._blocks:
            h = blk(h)
        h.square().mean().backward()
        outs.append((h.detach(), trunk._blocks[3]._depthwise_conv.weight.grad.clone()))
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(outs[0][1], outs[1][1], rtol=1e-3, atol=1e-5)


# ----------------------------------------------------------------------------- batch norm + activation
from lss_carla_amd import norm as Nm  # noqa: E402

BN_CASES = [  # (N, C, H, W, layout)
    (3, 32, 64, 176, "nchw"),
    (4, 96, 8, 22, "nchw"),
    (5, 40, 4, 11, "nchw"),
    (2, 16, 5, 7, "nchw"),     # one group per channel (the fused single-launch kernels), V = 1
    (48, 8, 8, 22, "nchw"),    # the trunk's 8 x 22 maps at B*N = 48: one group, V = 8, 8 vectors a thread
    (96, 8, 4, 11, "nchw"),    # 4 x 11 maps: one group, V = 4, 8 vectors a thread (register-resident)
    (2, 64, 100, 100, "nhwc"),
    (2, 256, 25, 25, "nhwc"),
    (3, 24, 7, 9, "nhwc"),
]


def _bn_reference(x, w, b, rm, rv, eps, mom, act, res, dy):
    xr = x.detach().cpu().double().requires_grad_(True)
    wr = w.detach().cpu().double().requires_grad_(True)
    br = b.detach().cpu().double().requires_grad_(True)
    rr = res.detach().cpu().double().requires_grad_(True) if res is not None else None
    rm, rv = rm.cpu().double(), rv.cpu().double()
    y = F.batch_norm(xr, rm, rv, wr, br, training=True, momentum=mom, eps=eps)
    if rr is not None:
        y = y + rr
    y = {"none": y, "relu": F.relu(y), "swish": F.silu(y)}[act]
    y.backward(dy.detach().cpu().double())
    return y.detach(), xr.grad, wr.grad, br.grad, (rr.grad if rr is not None else None), rm, rv


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("act,with_res", [("none", False), ("swish", False), ("relu", False), ("relu", True)])
@pytest.mark.parametrize("N,C,H,W,layout", BN_CASES)
def test_bn_act_vs_fp64(N, C, H, W, layout, act, with_res, dtype):
    g = torch.Generator().manual_seed(N * 1000 + C + H)
    x = (torch.randn(N, C, H, W, generator=g) * 2 + 3).to(dtype)  # offset mean: exercises the shifted sums
    res = torch.randn(N, C, H, W, generator=g).to(dtype) if with_res else None
    bn = torch.nn.BatchNorm2d(C, eps=1e-3, momentum=0.01).to(DEV).train()
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(C, generator=g) * 0.1)
        bn.running_mean.copy_(torch.randn(C, generator=g))
        bn.running_var.copy_(torch.rand(C, generator=g) + 0.5)
    rm0, rv0 = bn.running_mean.clone(), bn.running_var.clone()
    mf = torch.channels_last if layout == "nhwc" else torch.contiguous_format
    xd = x.to(DEV).contiguous(memory_format=mf).requires_grad_(True)
    rd = res.to(DEV).contiguous(memory_format=mf).requires_grad_(True) if with_res else None
    y = Nm.bn_act(bn, xd, act, rd)
    assert y.dtype == dtype and y.is_contiguous(memory_format=mf)
    dy = torch.randn(y.shape, generator=g).to(dtype)
    y.backward(dy.to(DEV).contiguous(memory_format=mf))
    ref = _bn_reference(x, bn.weight, bn.bias, rm0, rv0, bn.eps, bn.momentum, act, res, dy)
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(y.detach().cpu().double(), ref[0], **tol)
    torch.testing.assert_close(xd.grad.cpu().double(), ref[1], **tol)
    gtol = dict(rtol=1e-3, atol=1e-2) if dtype == torch.float32 else dict(rtol=3e-2, atol=1.0)
    torch.testing.assert_close(bn.weight.grad.cpu().double(), ref[2], **gtol)
    torch.testing.assert_close(bn.bias.grad.cpu().double(), ref[3], **gtol)
    if with_res:
        torch.testing.assert_close(rd.grad.cpu().double(), ref[4], **tol)
    torch.testing.assert_close(bn.running_mean.cpu().double(), ref[5], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bn.running_var.cpu().double(), ref[6], rtol=1e-3, atol=1e-4)
    assert int(bn.num_batches_tracked) == 1


# ----------------------------------------------------------------------------- bilinear upsample + cat
from lss_carla_amd import resample as R  # noqa: E402

UP_CASES = [  # (N, C1, Hi, Wi, C2, scale): BevEncode.up1 / up2, CamEncode.up1 (channels-last), odd sizes
    (2, 256, 25, 25, 64, 4),
    (2, 256, 100, 100, 0, 2),
    (3, 320, 4, 11, 112, 2),
    (1, 16, 5, 7, 8, 3),
]


@pytest.mark.parametrize("N,C1,H,W,C2,s", UP_CASES)
def test_upsample_cat_vs_fp64(N, C1, H, W, C2, s):
    g = torch.Generator().manual_seed(N * 7 + C1 + H)
    cl = torch.channels_last
    x = torch.randn(N, C1, H, W, generator=g).bfloat16()
    skip = torch.randn(N, C2, H * s, W * s, generator=g).bfloat16() if C2 else None
    xd = x.to(DEV).contiguous(memory_format=cl).requires_grad_(True)
    sd = skip.to(DEV).contiguous(memory_format=cl).requires_grad_(True) if C2 else None
    y = R.upsample_cat(xd, sd, s)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=cl) and y.shape == (N, C1 + C2, H * s, W * s)
    # reference: the fp64 upsample of the same bf16 values, concatenated as src/models.py:33 does
    xr = x.double().requires_grad_(True)
    up = F.interpolate(xr, scale_factor=s, mode="bilinear", align_corners=True)
    ref = torch.cat([skip.double(), up], 1) if C2 else up
    torch.testing.assert_close(y.detach().cpu().double(), ref.detach(), rtol=8e-3, atol=8e-3)  # one bf16 rounding
    if C2:
        assert torch.equal(y[:, :C2].detach().cpu(), skip)
    # the autocast reference: PyTorch's fp32 kernel, cast to bf16 -- equal but for FMA-contraction ulps
    with torch.no_grad():
        t32 = F.interpolate(xd.float(), scale_factor=s, mode="bilinear", align_corners=True).bfloat16()
    assert (y[:, C2:].detach() == t32).float().mean().item() > 0.99
    dy = torch.randn(y.shape, generator=g).bfloat16()
    y.backward(dy.to(DEV).contiguous(memory_format=cl))
    ref.backward(dy.double())
    assert xd.grad.dtype == torch.bfloat16
    torch.testing.assert_close(xd.grad.cpu().double(), xr.grad, rtol=1e-2, atol=2e-2)
    if C2:
        assert torch.equal(sd.grad.cpu(), dy[:, :C2])
    # deterministic backward (gather, no atomics)
    g1 = xd.grad.clone()
    xd.grad = None
    R.upsample_cat(xd, sd, s).backward(dy.to(DEV).contiguous(memory_format=cl))
    assert torch.equal(xd.grad, g1)


def test_bevencode_hip_upsample_vs_torch():
    """BevEncode under bf16 autocast: fused upsample+cat kernels vs PyTorch's fp32 upsample + cat."""
    from lss_carla_amd.models import BevEncode
    torch.manual_seed(5)
    m = BevEncode(64, 1).to(DEV).to(memory_format=torch.channels_last).train()
    m.dropout.p = 0.0
    x = torch.randn(2, 64, 200, 200, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    outs = []
    for use in (True, False):
        R.USE_HIP_UPSAMPLE = use
        try:
            m.zero_grad(set_to_none=True)
            xi = x.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = m(xi)
            y.float().square().mean().backward()
            outs.append((y.detach().float(), xi.grad.float(), m.up1.conv[0].weight.grad.clone(),
                         m.layer3[0].conv1.weight.grad.clone()))
        finally:
            R.USE_HIP_UPSAMPLE = True
    for a, b in zip(outs[0], outs[1]):
        err = (a - b).abs().max() / b.abs().max().clamp_min(1e-6)
        assert err < 3e-2, float(err)


# ----------------------------------------------------------------------------- squeeze-and-excitation
SE_CASES = [  # (N, C, H, W, sq): MBConv blocks of the trunk at config-3 resolutions (fewer images)
    (4, 32, 64, 176, 8),
    (3, 96, 32, 88, 4),
    (6, 240, 16, 44, 10),
    (5, 1152, 4, 11, 48),
]


def _rel(a, b):
    return float((a.double().cpu() - b.double().cpu()).abs().max() / b.double().abs().max().clamp_min(1e-12))


@pytest.mark.parametrize("N,C,H,W,sq", SE_CASES)
def test_squeeze_excite_vs_fp64(N, C, H, W, sq):
    g = torch.Generator().manual_seed(C + H)
    torch.manual_seed(C)
    x = (torch.randn(N, C, H, W, generator=g) * 2).bfloat16()
    red = torch.nn.Conv2d(C, sq, 1).to(DEV)
    exp = torch.nn.Conv2d(sq, C, 1).to(DEV)
    xd = x.to(DEV).requires_grad_(True)
    y = E.squeeze_excite(xd, red, exp)
    assert y.dtype == torch.bfloat16 and y.shape == x.shape
    dy = torch.randn(y.shape, generator=g).bfloat16()
    y.backward(dy.to(DEV))
    # fp64 reference on the bf16-rounded weights (what the autocast convs multiply with)
    ps = [t.detach().cpu().bfloat16().double().requires_grad_(True)
          for t in (red.weight, red.bias, exp.weight, exp.bias)]
    xr = x.double().requires_grad_(True)
    s = F.conv2d(F.silu(F.conv2d(xr.mean((2, 3), keepdim=True), ps[0], ps[1])), ps[2], ps[3])
    yr = torch.sigmoid(s) * xr
    yr.backward(dy.double())
    torch.testing.assert_close(y.detach().cpu().double(), yr.detach(), rtol=2e-2, atol=3e-2)
    assert _rel(xd.grad, xr.grad) < 2e-2
    for got, ref_p in zip((red.weight.grad, red.bias.grad, exp.weight.grad, exp.bias.grad), ps):
        assert got.dtype == torch.float32
        assert _rel(got, ref_p.grad) < 5e-2, _rel(got, ref_p.grad)


def test_mbconv_hip_se_vs_torch_autocast():
    """An MBConv block under bf16 autocast: lss_se_* vs PyTorch's SE ops (same block, same input)."""
    torch.manual_seed(11)
    blk = E.MBConvBlock(5, 1, 6, 40, 40, image_size=(16, 44)).to(DEV).train()
    x = torch.randn(6, 40, 16, 44, device=DEV).bfloat16()
    outs = []
    for use in (True, False):
        E.USE_HIP_SE = use
        try:
            blk.zero_grad(set_to_none=True)
            xi = x.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = blk(xi)
            y.float().square().mean().backward()
            outs.append((y.detach(), xi.grad, blk._se_reduce.weight.grad.clone(), blk._se_expand.bias.grad.clone(),
                         blk._expand_conv.weight.grad.clone()))
        finally:
            E.USE_HIP_SE = True
    for a, b in zip(*outs):
        assert _rel(a, b) < 5e-2, _rel(a, b)


@pytest.mark.parametrize("shape", [(8, 128, 200, 200), (2, 64, 7, 9), (1, 256, 3, 5)])
def test_head1x1_matches_fp32_conv(shape):
    """BevEncode's last conv (one output channel, src/models.py:115) on lss_head1_*: forward and the
    three gradients vs the fp32 conv of the same bf16 operands."""
    from lss_carla_amd import models
    N, C, H, W = shape
    g = torch.Generator().manual_seed(C + H)
    conv = torch.nn.Conv2d(C, 1, 1).to(DEV)
    x = torch.randn(N, C, H, W, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xr = x.detach().clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        assert models._head1_eligible(conv, xr)
        y = models.conv1x1(conv, xr)
    assert y.shape == (N, 1, H, W) and y.dtype == torch.bfloat16
    gy = torch.randn(N, 1, H, W, generator=g).to(DEV, torch.bfloat16)
    y.backward(gy)
    w = conv.weight.detach().to(torch.bfloat16).double()
    b = conv.bias.detach().to(torch.bfloat16).double()
    xd = x.double().requires_grad_(True)
    wd = w.clone().requires_grad_(True)
    bd = b.clone().requires_grad_(True)
    want = torch.nn.functional.conv2d(xd, wd, bd)
    want.backward(gy.double())
    torch.testing.assert_close(y.double(), want, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(xr.grad.double(), xd.grad, rtol=2e-2, atol=1e-3)
    for got, ref_ in ((conv.weight.grad, wd.grad), (conv.bias.grad, bd.grad)):
        # the gradient of autocast's bf16 operand is bf16 (as the conv's own): rounding 2^-9
        rel = ((got.double() - ref_).norm() / ref_.norm()).item()
        assert rel < 4e-3, rel


# ----------------------------------------------------------------------------- drop_connect + skip
from lss_carla_amd import efficientnet as E  # noqa: E402


@pytest.mark.parametrize("shape,cl", [((48, 40, 16, 44), False), ((48, 80, 8, 22), True), ((6, 24, 5, 7), False)])
def test_drop_connect_add_vs_fp64(shape, cl):
    """The fused MBConv skip with stochastic depth (lss_scale_add) against the reference's
    ``inputs / keep * floor(keep + rand) + skip`` in fp64 on the same Bernoulli draw; (6, 24, 5, 7)
    (per-sample size not a multiple of 8) takes the torch composition."""
    g = torch.Generator().manual_seed(shape[1])
    mf = torch.channels_last if cl else torch.contiguous_format
    x = torch.randn(shape, generator=g).bfloat16().to(DEV).contiguous(memory_format=mf).requires_grad_(True)
    r = torch.randn(shape, generator=g).bfloat16().to(DEV).contiguous(memory_format=mf).requires_grad_(True)
    p, keep = 0.2, 0.8
    torch.cuda.manual_seed(7)
    y = E.drop_connect_add(x, r, p, True)
    torch.cuda.manual_seed(7)
    mask = torch.floor(keep + torch.rand((shape[0], 1, 1, 1), dtype=torch.bfloat16, device=DEV))
    if shape[0] >= 48:
        assert 0 < int(mask.sum()) < shape[0]  # some samples dropped, some kept
    dy = torch.randn(shape, generator=g).bfloat16().to(DEV).contiguous(memory_format=mf)
    y.backward(dy)
    md = mask.double().cpu()
    ref = x.detach().double().cpu() / keep * md + r.detach().double().cpu()
    torch.testing.assert_close(y.detach().double().cpu(), ref, rtol=8e-3, atol=8e-3)
    torch.testing.assert_close(x.grad.double().cpu(), dy.double().cpu() / keep * md, rtol=8e-3, atol=8e-3)
    assert torch.equal(r.grad, dy)
    assert y.is_contiguous(memory_format=mf)
    # the in-kernel mask is torch's floor(keep + rand) bit for bit: dropped samples are the skip exactly
    drop = mask.reshape(-1) == 0
    assert torch.equal(y.detach()[drop], r.detach()[drop]) and torch.equal(x.grad[drop], torch.zeros_like(x.grad[drop]))


def test_drop_connect_add_eval_is_plain_add():
    x = torch.randn(4, 16, 4, 4, device=DEV).bfloat16()
    r = torch.randn(4, 16, 4, 4, device=DEV).bfloat16()
    assert torch.equal(E.drop_connect_add(x, r, 0.2, False), x + r)
    assert torch.equal(E.drop_connect_add(x, r, None, True), x + r)


# ----------------------------------------------------------------------------- BN backward without y
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bn_relu_nhwc_backward_recomputes_output(dtype):
    """Channels-last ReLU without a residual: lss_bn_bwd with y = NULL (the output recomputed from x and
    the saved scale / shift) gives the same bits as with the forward's y, with 2,500 partial groups per
    channel through the C ABI (the fold's batched loads and its tail), and against torch's BN on the GPU."""
    from lss_carla_amd import _lib
    lib = _lib.load()
    N, C, H, W = 4, 128, 200, 200
    g = torch.Generator().manual_seed(11)
    cl = torch.channels_last
    x = (torch.randn(N, C, H, W, generator=g) + 0.3).to(dtype).to(DEV).contiguous(memory_format=cl)
    dy = torch.randn(N, C, H, W, generator=g).to(dtype).to(DEV).contiguous(memory_format=cl)
    bn = torch.nn.BatchNorm2d(C).to(DEV).train()
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(C, generator=g) * 0.1)
    xd = x.clone().requires_grad_(True)
    y = Nm.bn_act(bn, xd, "relu")
    y.backward(dy)
    # the C-ABI passes below use more partial groups than lss_bn_groups picks (625 here), so the fold's
    # batched loop (32 loads per lane) and its tail both run
    groups = 2500
    assert groups > 64 * 32 and groups <= 4096
    # the same forward again for its saved statistics, then both backward forms through the C ABI
    stats = torch.empty(4, C, device=DEV)
    partial = torch.empty(C, groups, 2, device=DEV)
    y2 = torch.empty_like(x)
    st = _lib.stream_handle(DEV)
    _lib.check(lib.lss_bn_fwd(_lib.ptr(x), None, _lib.dtype_code(dtype), Nm.NHWC, N, C, H * W, _lib.ptr(bn.weight),
                              _lib.ptr(bn.bias), 1e-5, 0.0, None, None, None, Nm.ACT["relu"], groups,
                              _lib.ptr(partial), _lib.ptr(stats[0]), _lib.ptr(stats[1]), _lib.ptr(stats[2]),
                              _lib.ptr(stats[3]), _lib.ptr(y2), st), "fwd")
    outs = []
    for yy in (y2, None):
        coef = torch.empty(C, 2, device=DEV)
        dg, db = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        dx = torch.empty_like(x)
        _lib.check(lib.lss_bn_bwd(_lib.ptr(dy), _lib.ptr(x), _lib.ptr(yy), _lib.dtype_code(dtype), Nm.NHWC, N, C, H * W,
                                  _lib.ptr(stats[2]), _lib.ptr(stats[3]), _lib.ptr(stats[0]), _lib.ptr(stats[1]),
                                  Nm.ACT["relu"], groups, _lib.ptr(partial), _lib.ptr(coef), _lib.ptr(dg), _lib.ptr(db),
                                  _lib.ptr(dx), None, st), "bwd")
        outs.append((dx, dg, db))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    # bn_act (lss_bn_groups' 625 groups) vs these 2,500: the same sums in another fold order
    close = dict(rtol=1e-5, atol=1e-6) if dtype == torch.float32 else dict(rtol=1e-2, atol=1e-3)
    torch.testing.assert_close(outs[1][0].float(), xd.grad.float(), **close)
    # torch's fp32 BN + ReLU on the GPU
    xr = x.float().requires_grad_(True)
    ref = F.relu(F.batch_norm(xr, None, None, bn.weight.detach(), bn.bias.detach(), training=True, eps=1e-5))
    ref.backward(dy.float())
    tol = dict(rtol=1e-3, atol=1e-3) if dtype == torch.float32 else dict(rtol=2e-2, atol=5e-2)
    torch.testing.assert_close(y.float(), ref.detach(), **tol)
    torch.testing.assert_close(xd.grad.float(), xr.grad, **tol)


@pytest.mark.parametrize("Hi,Wi,Ho,Wo", [(10, 13, 37, 50), (7, 9, 13, 29), (25, 25, 101, 99)])
def test_upsample_noninteger_ratio_vs_fp64(Hi, Wi, Ho, Wo):
    """lss_upsample_* at output sizes that are not integer multiples (align_corners ratios r = (Hi - 1) /
    (Ho - 1) whose r * o rounds across line boundaries): every nonzero tap reaches the backward, whether
    k_up_bwd_taps holds it in its list or falls back to the plain loop."""
    g = torch.Generator().manual_seed(Hi * 100 + Wo)
    cl = torch.channels_last
    x = torch.randn(2, 16, Hi, Wi, generator=g).bfloat16()
    xd = x.to(DEV).contiguous(memory_format=cl).requires_grad_(True)
    y = R._UpsampleCat.apply(xd, None, Ho, Wo)
    xr = x.double().requires_grad_(True)
    ref = F.interpolate(xr, size=(Ho, Wo), mode="bilinear", align_corners=True)
    torch.testing.assert_close(y.detach().cpu().double(), ref.detach(), rtol=8e-3, atol=8e-3)
    dy = torch.randn(y.shape, generator=g).bfloat16()
    y.backward(dy.to(DEV).contiguous(memory_format=cl))
    ref.backward(dy.double())
    torch.testing.assert_close(xd.grad.cpu().double(), xr.grad, rtol=1e-2, atol=2e-2)


def _bn_run(x, res, act, dy, seed):
    """one bn_act forward + backward on a fresh module; every output the kernels produce"""
    C = x.shape[1]
    torch.manual_seed(seed)
    bn = torch.nn.BatchNorm2d(C, eps=1e-3, momentum=0.01).to(DEV).train()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.normal_(0.0, 0.1)
    xd = x.clone().requires_grad_(True)
    rd = res.clone().requires_grad_(True) if res is not None else None
    y = Nm.bn_act(bn, xd, act, rd)
    y.backward(dy)
    out = [y.detach(), xd.grad, bn.weight.grad, bn.bias.grad, bn.running_mean.clone(), bn.running_var.clone()]
    return out + ([rd.grad] if rd is not None else [])


@pytest.mark.parametrize("spin", [0, 1])
@pytest.mark.parametrize("act,with_res", [("swish", False), ("none", True), ("relu", False)])
@pytest.mark.parametrize("N,C,H,W", [(48, 144, 32, 88), (48, 24, 32, 88), (48, 80, 16, 44), (16, 16, 33, 40)])
def test_bn_cluster_kernels_bit_identical(N, C, H, W, act, with_res, spin):
    """NCHW bf16 with several groups per channel: the one-launch cluster kernels (lss_bn_fwd2 / lss_bn_bwd2
    with a sync workspace) against the two-launch statistics + apply kernels, bit for bit -- outputs,
    gradients, running statistics. spin = 1 sets the workspace's wait bound to 0 polls, so every block
    takes the timeout path (recomputes every group's statistics itself): still bit-identical. The
    workspace's counters come back zero-filled."""
    g = torch.Generator().manual_seed(N + C + H)
    x = (torch.randn(N, C, H, W, generator=g) * 2 + 3).bfloat16().to(DEV)
    res = torch.randn(N, C, H, W, generator=g).bfloat16().to(DEV) if with_res else None
    dy = torch.randn(N, C, H, W, generator=g).bfloat16().to(DEV)
    from lss_carla_amd import _lib
    lib = _lib.load()
    assert lib.lss_bn_groups(N, C, H * W, 0) > 1
    old = Nm.USE_BN_CLUSTER
    try:
        Nm.USE_BN_CLUSTER = False
        want = _bn_run(x, res, act, dy, 1)
        Nm.USE_BN_CLUSTER = True
        sync = Nm._sync(DEV)
        sync[-1] = spin
        got = _bn_run(x, res, act, dy, 1)
        torch.cuda.synchronize()
    finally:
        Nm.USE_BN_CLUSTER = old
        Nm._sync(DEV)[-1] = 0
    for a, b in zip(got, want):
        assert torch.equal(a, b)
    assert int(Nm._sync(DEV)[:-1].abs().sum()) == 0, "cluster counters not re-zeroed"


# ----------------------------------------------------------------------------- BevEncode up2 tail
@pytest.mark.parametrize("shape", [(2, 128, 64, 64), (1, 64, 30, 50)])
def test_bn_relu_head1_fused_bit_identical(shape):
    """models._BnReluHead1 (BN statistics only, the head applying scale / shift / ReLU as it reads, the BN
    backward taking the head's rank-1 gradient) == bn_act + _Head1x1 bit for bit: the output, d(x), the BN
    weight / bias gradients, the head weight / bias gradients and the running statistics."""
    import copy
    from lss_carla_amd import models as M
    N, C, H, W = shape
    torch.manual_seed(C + H)
    bn = torch.nn.BatchNorm2d(C).to(DEV).train()
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C) + 0.5)
        bn.bias.copy_(torch.randn(C) * 0.2)
    head = torch.nn.Conv2d(C, 1, 1).to(DEV).to(memory_format=torch.channels_last)
    x = (torch.randn(N, C, H, W, device=DEV) + 0.2).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dout = torch.randn(N, 1, H, W, device=DEV).to(torch.bfloat16)
    res = []
    for fused in (True, False):
        b, h = copy.deepcopy(bn), copy.deepcopy(head)
        xi = x.clone().requires_grad_(True)
        M.USE_BN_HEAD = fused
        try:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = M.bn_relu_head1(b, h, xi)
        finally:
            M.USE_BN_HEAD = True
        out.backward(dout)
        torch.cuda.synchronize()
        res.append((out.detach(), xi.grad, b.weight.grad, b.bias.grad, h.weight.grad, h.bias.grad,
                    b.running_mean, b.running_var, b.num_batches_tracked))
    for a, c in zip(*res):
        assert torch.equal(a, c)
    assert int(res[0][-1]) == 1


# ----------------------------------------------------------------------------- Dropout2d in the upsample
@pytest.mark.parametrize("N,C,H,W,s", [(2, 256, 25, 25, 2), (3, 64, 10, 13, 4)])
def test_upsample_channel_scale_vs_fp64(N, C, H, W, s):
    """upsample_cat(x, None, s, chan_scale=m) == bilinear_upsample(x * m) (fp64 of the same bf16 values,
    one bf16 rounding), and d(x) = m * upsample_bwd(dy); m a Dropout2d mask with zeroed channels."""
    g = torch.Generator().manual_seed(N + C + H)
    cl = torch.channels_last
    x = torch.randn(N, C, H, W, generator=g).bfloat16()
    m = (torch.rand(N, C, generator=g) > 0.3).float() * (1 / 0.7)
    xd = x.to(DEV).contiguous(memory_format=cl).requires_grad_(True)
    y = R.upsample_cat(xd, None, s, m.to(DEV))
    xr = x.double().requires_grad_(True)
    ref = F.interpolate(xr * m.double().view(N, C, 1, 1), scale_factor=s, mode="bilinear", align_corners=True)
    torch.testing.assert_close(y.detach().cpu().double(), ref.detach(), rtol=8e-3, atol=8e-3)
    zero = m == 0
    assert (y.detach().cpu()[zero] == 0).all()  # dropped channels exactly zero
    dy = torch.randn(y.shape, generator=g).bfloat16()
    y.backward(dy.to(DEV).contiguous(memory_format=cl))
    ref.backward(dy.double())
    torch.testing.assert_close(xd.grad.cpu().double(), xr.grad, rtol=1e-2, atol=2e-2)
    assert (xd.grad.cpu()[zero] == 0).all()


def test_bevencode_dropout2d_mask_matches_torch():
    """models._dropout2d_scale draws the mask torch's Dropout2d draws (same generator calls, same dtype):
    with the same seed, x * mask == F.dropout2d(x) bit for bit; eval and p = 0 give None."""
    from lss_carla_amd import models as M
    d = torch.nn.Dropout2d(0.1).train()
    x = torch.randn(8, 256, 4, 4, device=DEV).bfloat16()
    torch.manual_seed(5)
    m = M._dropout2d_scale(d, x)
    torch.manual_seed(5)
    ref = F.dropout2d(x, 0.1, True)
    got = x * m.view(8, 256, 1, 1).to(x.dtype)
    assert torch.equal(got, ref)
    assert 0 < int((m == 0).sum()) < m.numel()
    assert M._dropout2d_scale(d.eval(), x) is None
    assert M._dropout2d_scale(torch.nn.Dropout2d(0.0).train(), x) is None


@pytest.mark.parametrize("N,C,H,W,K,S,pad,Ho", [(48, 40, 32, 88, 3, 1, 1, 32), (48, 24, 22, 22, 5, 1, 2, 22),
                                                 (48, 24, 11, 11, 5, 1, 2, 11), (48, 16, 22, 22, 3, 2, 0, 11)],
                         ids=["lds-3x3", "planes-22", "planes-11-one-group", "planes-s2"])
def test_depthwise_weight_grad_folded_in_kernel(N, C, H, W, K, S, pad, Ho):
    """lss_dwconv_bwd_weight2: the channel's last block folds the group partials (no torch reduction):
    equal to the unfolded partials summed in group order up to fp32 rounding, the same bits on every call,
    and the sync workspace left zero-filled."""
    from lss_carla_amd import _lib, norm
    lib = _lib.load()
    g = torch.Generator().manual_seed(3)
    x = torch.randn(N, C, H, W, generator=g).to(torch.bfloat16).to(DEV)
    dy = torch.randn(N, C, Ho, Ho, generator=g).to(torch.bfloat16).to(DEV)
    groups = max(1, min(N, (N * Ho * Ho) // 8192))
    # fp64 reference: padded (TF 'same' pads the far side for stride 2) grouped-conv weight gradient
    far = (Ho - 1) * S + K - H - pad
    xp = torch.nn.functional.pad(x.double(), (pad, far, pad, far))
    ref = torch.nn.grad.conv2d_weight(xp, (C, 1, K, K), dy.double(), stride=S, groups=C).view(C, K * K)
    st = _lib.stream_handle(DEV)
    part = torch.empty(C, groups, K * K, device=DEV)
    _lib.check(lib.lss_dwconv_bwd_weight(_lib.ptr(x), _lib.ptr(dy), _lib.BF16, N, C, H, W, K, S, pad, pad, Ho, Ho, groups,
                                         _lib.ptr(part), st), "unfolded")
    want = part.double().sum(1)
    sync = norm._sync(DEV)
    outs = []
    for _ in range(2):
        part2 = torch.empty(C, groups, K * K, device=DEV)
        dw = torch.empty(C, K * K, device=DEV)
        _lib.check(lib.lss_dwconv_bwd_weight2(_lib.ptr(x), _lib.ptr(dy), _lib.BF16, N, C, H, W, K, S, pad, pad, Ho, Ho, groups,
                                              _lib.ptr(part2), _lib.ptr(sync), _lib.ptr(dw), st), "folded")
        torch.cuda.synchronize()
        outs.append(dw.clone())
    assert torch.equal(outs[0], outs[1])
    torch.testing.assert_close(outs[0].double(), want, rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(outs[0].double(), ref, rtol=1e-4, atol=1e-2)
    assert int(sync.abs().sum()) == 0
