"""lss_pw_wrw (include/lss_convs.h): the weight gradient of the trunk's 1x1 convs (MBConv expand /
project, src/models.py:43 via efficientnet_pytorch) against an fp64 reference of the same bf16
operands, at the trunk's shapes (both fragment-load widths: HW % 8 == 0 and HW % 4 == 0), plus the
autograd path (efficientnet._HipPointwise) against nn.Conv2d under autocast."""
import pytest
import torch

import lss_carla_amd  # noqa: F401
from lss_carla_amd import _lib, efficientnet

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")

# (N, Cin, Cout, H, W): c3 trunk layers at reduced N, plus ragged channel counts and tiny cases
SHAPES = [
    (2, 16, 96, 64, 176),    # b1 expand (HW 11264)
    (3, 96, 24, 32, 88),     # b1 project
    (4, 40, 240, 16, 44),    # b4 expand (HW 704)
    (4, 672, 112, 8, 22),    # b10 project (HW 176: a half-filled last K step)
    (5, 192, 1152, 4, 11),   # b12 expand (HW 44: 8-B fragment loads)
    (3, 1152, 320, 4, 11),   # b15 project
    (2, 3, 5, 2, 2),         # one ragged fragment each way, HW 4
    (1, 70, 130, 4, 6),      # tiles past 64 in both dims, HW 24
]


def _run(x, dy, out_dtype):
    lib = _lib.load()
    N, Cin, H, W = x.shape
    Cout = dy.shape[1]
    nbytes = int(lib.lss_pw_wrw_workspace_bytes(N, Cin, Cout, H * W))
    ws = torch.empty(nbytes, device=DEV, dtype=torch.uint8)
    dw = torch.full((Cout, Cin), float("nan"), device=DEV, dtype=out_dtype)
    _lib.check(lib.lss_pw_wrw(_lib.ptr(x), _lib.ptr(dy), N, Cin, Cout, H * W, _lib.ptr(dw), _lib.dtype_code(out_dtype),
                              _lib.ptr(ws), nbytes, _lib.stream_handle(DEV)), "lss_pw_wrw")
    return dw


def _inputs(N, Cin, Cout, H, W, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, Cin, H, W, generator=g).to(DEV, torch.bfloat16)
    dy = torch.randn(N, Cout, H, W, generator=g).to(DEV, torch.bfloat16)
    return x, dy


def _ref(x, dy):
    return torch.einsum("nohw,nihw->oi", dy.double(), x.double())


@pytest.mark.parametrize("shape", SHAPES)
def test_pw_wrw_vs_fp64(shape):
    x, dy = _inputs(*shape)
    ref = _ref(x, dy)
    K = shape[0] * shape[3] * shape[4]
    got = _run(x, dy, torch.float32).double()
    # fp32 accumulation of K products of bf16 values (exact in fp32): error ~ sqrt(K) * 2^-24 * |terms|
    tol = 4e-6 * K + 1e-5
    assert torch.isfinite(got).all()
    assert (got - ref).abs().max().item() <= tol, ((got - ref).abs().max().item(), tol)
    gb = _run(x, dy, torch.bfloat16)
    assert torch.equal(gb, got.float().to(torch.bfloat16))  # the bf16 output is the fp32 sum rounded once


def test_pw_wrw_deterministic():
    x, dy = _inputs(4, 112, 672, 8, 22, seed=3)
    a = _run(x, dy, torch.float32)
    b = _run(x, dy, torch.float32)
    assert torch.equal(a, b)


def test_pw_wrw_rejects_bad_arguments():
    lib = _lib.load()
    x, dy = _inputs(1, 8, 8, 3, 3)  # HW 9: not a multiple of 4
    ws = torch.empty(1 << 16, device=DEV, dtype=torch.uint8)
    dw = torch.empty(8, 8, device=DEV)
    rc = lib.lss_pw_wrw(_lib.ptr(x), _lib.ptr(dy), 1, 8, 8, 9, _lib.ptr(dw), 0, _lib.ptr(ws), ws.numel(),
                        _lib.stream_handle(DEV))
    assert rc == -1
    x, dy = _inputs(2, 16, 96, 8, 8)
    rc = lib.lss_pw_wrw(_lib.ptr(x), _lib.ptr(dy), 2, 16, 96, 64, _lib.ptr(dw), 0, _lib.ptr(ws), 4,
                        _lib.stream_handle(DEV))  # workspace too small
    assert rc == -1


@pytest.fixture
def miopen_fwd():
    efficientnet.USE_HIP_PW_GEMM = False  # forward / backward-data on MIOpen: only the weight gradient differs
    yield
    efficientnet.USE_HIP_PW_GEMM = True


@pytest.mark.parametrize("wdtype", [torch.float32, torch.bfloat16])
def test_pointwise_conv_autograd_matches_conv2d(wdtype, miopen_fwd):
    torch.manual_seed(0)
    conv = efficientnet.Conv2dStaticSamePadding(96, 24, 1, bias=False, image_size=(32, 88)).to(DEV)
    if wdtype == torch.bfloat16:
        conv = conv.to(torch.bfloat16)
    x = torch.randn(6, 96, 32, 88, device=DEV).to(torch.bfloat16).requires_grad_(True)
    gy = torch.randn(6, 24, 32, 88, device=DEV).to(torch.bfloat16)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = efficientnet.pointwise_conv(conv, x)
    y.backward(gy)
    gx, gw = x.grad.clone(), conv.weight.grad.clone()
    assert gw.dtype == wdtype
    x.grad = None
    conv.weight.grad = None
    efficientnet.USE_HIP_PW_WRW = False
    try:
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y2 = efficientnet.pointwise_conv(conv, x)
        y2.backward(gy)
    finally:
        efficientnet.USE_HIP_PW_WRW = True
    assert torch.equal(y, y2)  # the same MIOpen forward
    assert torch.equal(gx, x.grad)  # the same MIOpen backward-data
    ref = _ref(x.detach(), gy).float()
    tol = 2e-2 * ref.abs().max().item()
    assert (gw.float().view_as(ref) - ref).abs().max().item() <= tol
    assert (conv.weight.grad.float().view_as(ref) - ref).abs().max().item() <= tol


CONV_SHAPES = [
    (2, 16, 96, 64, 176),    # b1 expand (K 16: one 32-k stage, half of it masked)
    (3, 96, 24, 32, 88),     # b1 project
    (4, 40, 240, 16, 44),
    (4, 672, 112, 8, 22),    # HW 176
    (5, 192, 1152, 4, 11),   # HW 44: 8-B pixel loads, tiles straddling images
    (3, 1152, 320, 4, 11),   # K 1152: nine 128-k stages
    (2, 8, 8, 2, 2),
    (1, 136, 72, 3, 4),      # ragged tiles in k, m and pixels
]


@pytest.mark.parametrize("layout", [0, 1])
@pytest.mark.parametrize("shape", CONV_SHAPES)
def test_pw_conv_vs_fp64(shape, layout):
    lib = _lib.load()
    N, Cin, Cout, H, W = shape
    g = torch.Generator().manual_seed(7)
    K, M = (Cin, Cout) if layout == 0 else (Cout, Cin)  # layout 1: the backward-data, dx = W^T dy
    x = torch.randn(N, K, H, W, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(Cout, Cin, generator=g) / K ** 0.5).to(DEV, torch.bfloat16)
    y = torch.full((N, M, H, W), float("nan"), device=DEV, dtype=torch.bfloat16)
    _lib.check(lib.lss_pw_conv(_lib.ptr(x), _lib.ptr(w), layout, N, K, M, H * W, _lib.ptr(y), _lib.stream_handle(DEV)),
               "lss_pw_conv")
    a = w.double() if layout == 0 else w.double().t()  # (M, K)
    ref = torch.einsum("mk,nkhw->nmhw", a, x.double())
    assert torch.isfinite(y.float()).all()
    # fp32 accumulation, one bf16 rounding of the result
    err = (y.double() - ref).abs() - 2.0 ** -8 * ref.abs()
    assert err.max().item() <= 1e-4 * K ** 0.5, err.max().item()


def test_pointwise_gemm_autograd_matches_miopen():
    torch.manual_seed(1)
    conv = efficientnet.Conv2dStaticSamePadding(112, 672, 1, bias=False, image_size=(8, 22)).to(DEV)
    x = torch.randn(6, 112, 8, 22, device=DEV).to(torch.bfloat16).requires_grad_(True)
    gy = torch.randn(6, 672, 8, 22, device=DEV).to(torch.bfloat16)
    outs = []
    for gemm in (True, False):
        efficientnet.USE_HIP_PW_GEMM = gemm
        try:
            x.grad = None
            conv.weight.grad = None
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = efficientnet.pointwise_conv(conv, x)
            y.backward(gy)
            outs.append((y.detach().float(), x.grad.float(), conv.weight.grad.clone()))
        finally:
            efficientnet.USE_HIP_PW_GEMM = True
    (y1, gx1, gw1), (y2, gx2, gw2) = outs
    torch.testing.assert_close(y1, y2, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(gx1, gx2, rtol=1e-2, atol=2e-2)
    assert torch.equal(gw1, gw2)  # the same lss_pw_wrw either way
