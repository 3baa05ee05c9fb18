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
