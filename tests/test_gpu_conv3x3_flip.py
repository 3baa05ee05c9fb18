"""Stride-1 3x3 convolutions with the backward-data pass as a forward convolution of the flipped,
transposed weight (models._Conv3x3, USE_FLIP_BWD): same forward, same gradients as nn.Conv2d's autograd
(MIOpen's backward-data solver) within the rounding of the operands -- bf16 channels-last (the benched
BevEncode / CamEncode.up1 path) and fp32 (the reference caller's precision) -- at BevEncode's and
CamEncode.up1's channel counts; and BevEncode's gradients with the switch on and off."""
import pytest
import torch
from torch import nn

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs an MI355X", allow_module_level=True)

from lss_carla_amd import models  # noqa: E402

DEV = torch.device("cuda:0")


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("shape", [(2, 64, 64, 25, 25), (2, 320, 256, 20, 24), (4, 432, 512, 8, 22)],
                         ids=["64x64", "320x256", "432x512"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32], ids=["bf16", "fp32"])
def test_flip_bwd_matches_conv_autograd(shape, dtype):
    N, Cin, Cout, H, W = shape
    torch.manual_seed(0)
    conv = nn.Conv2d(Cin, Cout, 3, padding=1, bias=False).to(DEV).to(memory_format=torch.channels_last)
    x = torch.randn(N, Cin, H, W, device=DEV).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, Cout, H, W, device=DEV).contiguous(memory_format=torch.channels_last)
    outs = []
    for flip in (True, False):
        models.USE_FLIP_BWD = flip
        conv.zero_grad(set_to_none=True)
        xi = x.clone().requires_grad_(True)
        try:
            if dtype == torch.bfloat16:
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    y = models.conv3x3(conv, xi)
            else:
                y = models.conv3x3(conv, xi)
        finally:
            models.USE_FLIP_BWD = True
        y.backward(dy.to(y.dtype))
        torch.cuda.synchronize()
        outs.append((y.detach().float(), xi.grad.float(), conv.weight.grad.float()))
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-5
    # the forward is the same convolution (MIOpen may pick another fp32 solver per call: summation order)
    assert _rel(outs[0][0], outs[1][0]) < (1e-6 if dtype == torch.float32 else 1e-30) or \
        torch.equal(outs[0][0], outs[1][0])
    assert _rel(outs[0][1], outs[1][1]) < tol
    assert _rel(outs[0][2], outs[1][2]) < tol


def test_flip_bwd_fp64_reference():
    """dx of the flipped form against an fp64 torch convolution's autograd (fp32 operands)."""
    torch.manual_seed(1)
    conv = nn.Conv2d(48, 40, 3, padding=1, bias=False).to(DEV)
    x = torch.randn(2, 48, 13, 17, device=DEV, requires_grad=True)
    y = models.conv3x3(conv, x)
    g = torch.randn_like(y)
    y.backward(g)
    x64 = x.detach().double().requires_grad_(True)
    w64 = conv.weight.detach().double().requires_grad_(True)
    y64 = torch.nn.functional.conv2d(x64, w64, None, 1, 1)
    y64.backward(g.double())
    assert _rel(x.grad, x64.grad) < 1e-6
    assert _rel(conv.weight.grad, w64.grad) < 1e-6


def test_bevencode_flip_on_off():
    torch.manual_seed(2)
    enc = models.BevEncode(64, 1).to(DEV).to(memory_format=torch.channels_last).train()
    enc.dropout.p = 0.0  # the same forward on both passes
    x = torch.randn(2, 64, 200, 200, device=DEV).contiguous(memory_format=torch.channels_last)
    grads = []
    for flip in (True, False):
        models.USE_FLIP_BWD = flip
        enc.zero_grad(set_to_none=True)
        try:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = enc(x)
        finally:
            models.USE_FLIP_BWD = True
        out.float().square().mean().backward()
        torch.cuda.synchronize()
        grads.append({n: p.grad.detach().float().clone() for n, p in enc.named_parameters() if p.grad is not None})
    assert grads[0].keys() == grads[1].keys()
    for n in grads[0]:
        assert _rel(grads[0][n], grads[1][n]) < 3e-2, n


@pytest.mark.parametrize("cl", [True, False], ids=["channels_last", "contiguous"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32], ids=["bf16", "fp32"])
@pytest.mark.parametrize("O,I,K", [(256, 320, 3), (128, 256, 3), (40, 48, 5)])
def test_flip_weight_kernel_exact(O, I, K, dtype, cl):
    """lss_conv_flip_weight == w.transpose(0, 1).flip(2, 3), bit for bit, channels-last output."""
    torch.manual_seed(O + I + K)
    w = torch.randn(O, I, K, K, device=DEV).to(dtype)
    if cl:
        w = w.contiguous(memory_format=torch.channels_last)
    got = models._flip_weight(w)
    torch.cuda.synchronize()
    want = w.transpose(0, 1).flip(2, 3)
    assert got.shape == (I, O, K, K) and got.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(got, want)
