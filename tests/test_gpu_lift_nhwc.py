"""Fused depthnet lift on channels-last features (lss_depthnet_lift_nhwc, k_depthnet_lift3).

The kernel must give the same bits as the NCHW kernel (k_depthnet_lift2) on the same values -- same
MFMA operands, same K order, same epilogue -- at every BASELINE config it serves, with the weights as
they lie or in lss_depthnet_pack's fragment order; at pixel counts the NCHW kernel does not tile (odd
feature maps, fewer pixels than CUs) it is checked against the fp64 conv + the oracle's lift
(src/models.py:47, 52-59).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU CI, skipped there
    pytest.skip("needs an MI355X", allow_module_level=True)

from oracle import lss_ref as ref  # noqa: E402
import lss_carla_amd as L  # noqa: E402
from lss_carla_amd import _lib, ops  # noqa: E402
from lss_carla_amd import synthetic as syn  # noqa: E402

DEV = torch.device("cuda:0")


def _inputs(B, N, H, W, D, seed=0):
    g = torch.Generator().manual_seed(seed)
    feat = torch.randn(B * N, 512, H, W, generator=g).to(torch.bfloat16)
    weight = (torch.randn(D + 64, 512, generator=g) * 0.05).to(torch.bfloat16)
    bias = (torch.randn(D + 64, generator=g) * 0.1).to(torch.bfloat16)
    return feat, weight, bias


def _run(fn, feat, weight, bias, dims):
    B, N, D, H, W = dims.B, dims.N, dims.D, dims.H, dims.W
    depth = torch.full((B * N, D, H, W), float("nan"), device=DEV)
    ctx_t = torch.full((B * N * H * W, 64), float("nan"), device=DEV, dtype=torch.bfloat16)
    _lib.check(fn(_lib.ptr(feat), _lib.ptr(weight), _lib.ptr(bias), _lib.BF16, 512, dims, _lib.ptr(depth),
                  _lib.ptr(ctx_t), _lib.BF16, _lib.stream_handle(DEV)), "depthnet_lift")
    torch.cuda.synchronize()
    return depth, ctx_t


@pytest.mark.parametrize("name", ["c1", "c3", "c5"])
def test_nhwc_kernel_bit_identical_to_nchw_kernel(name):
    cfg, gc, _ = syn.config_confs(name)
    B, N, fd = cfg["B"], cfg["N"], cfg["final_dim"]
    rig = {k: v.to(DEV) for k, v in syn.make_rig(B, N, fd, seed=2).items()}
    frustum = ref.create_frustum(fd, gc["dbound"]).to(DEV)
    D, H, W = frustum.shape[:3]
    plan = ops.plan_from_cameras(frustum, **rig, grid=ops.GridSpec.from_conf(gc))
    feat, weight, bias = (t.to(DEV) for t in _inputs(B, N, H, W, D, seed=5))
    feat_cl = feat.contiguous(memory_format=torch.channels_last)
    lib = _lib.load()
    d0, c0 = _run(lib.lss_depthnet_lift, feat, weight, bias, plan.c_dims)
    d1, c1 = _run(lib.lss_depthnet_lift_nhwc, feat_cl, weight, bias, plan.c_dims)
    assert torch.equal(d0, d1) and torch.equal(c0, c1)


def _pack(weight, bias):
    O, K = weight.shape
    packed = torch.full((_lib.DN_PACKED_BYTES(K) // 2,), float("nan"), device=DEV, dtype=torch.bfloat16)
    plain = torch.full((O, K), float("nan"), device=DEV, dtype=torch.bfloat16)
    b16 = torch.full((O,), float("nan"), device=DEV, dtype=torch.bfloat16)
    _lib.check(_lib.load().lss_depthnet_pack(_lib.ptr(weight), _lib.ptr(bias), _lib.dtype_code(weight.dtype), O, K,
                                             _lib.ptr(packed), _lib.ptr(plain), _lib.ptr(b16),
                                             _lib.stream_handle(DEV)), "pack")
    torch.cuda.synchronize()
    return packed, plain, b16


@pytest.mark.parametrize("name", ["c1", "c3", "c5"])
@pytest.mark.parametrize("wdtype", [torch.float32, torch.bfloat16])
def test_packed_weights_bit_identical(name, wdtype):
    """lss_depthnet_pack (fp32 master or bf16 weights -> the fragment order, the plain bf16 copy and the
    bf16 bias: torch's round to nearest even) + lss_depthnet_lift_nhwc_packed give the bits of
    lss_depthnet_lift_nhwc on the torch-rounded weights."""
    cfg, gc, _ = syn.config_confs(name)
    B, N, fd = cfg["B"], cfg["N"], cfg["final_dim"]
    D, H, W = ref.create_frustum(fd, gc["dbound"]).shape[:3]
    g = torch.Generator().manual_seed(3)
    feat = torch.randn(B * N, 512, H, W, generator=g).to(torch.bfloat16).to(DEV)
    weight = (torch.randn(D + 64, 512, generator=g) * 0.05).to(wdtype).to(DEV)
    bias = (torch.randn(D + 64, generator=g) * 0.1).to(wdtype).to(DEV)
    feat_cl = feat.contiguous(memory_format=torch.channels_last)
    dims = _lib.Dims(B, N, D, H, W, 64)
    packed, plain, b16 = _pack(weight, bias)
    assert torch.equal(plain, weight.to(torch.bfloat16)) and torch.equal(b16, bias.to(torch.bfloat16))
    lib = _lib.load()
    d0, c0 = _run(lib.lss_depthnet_lift_nhwc, feat_cl, plain, b16, dims)
    depth = torch.full_like(d0, float("nan"))
    ctx_t = torch.full_like(c0, float("nan"))
    _lib.check(lib.lss_depthnet_lift_nhwc_packed(_lib.ptr(feat_cl), _lib.ptr(packed), _lib.ptr(b16), 512, dims,
                                                 _lib.ptr(depth), _lib.ptr(ctx_t), _lib.BF16,
                                                 _lib.stream_handle(DEV)), "lift packed")
    torch.cuda.synchronize()
    assert torch.equal(depth, d0) and torch.equal(ctx_t, c0)


def test_pack_rejects_bad_arguments():
    lib = _lib.load()
    w = torch.zeros(105, 512, device=DEV)
    buf = torch.empty(_lib.DN_PACKED_BYTES(512) // 2, device=DEV, dtype=torch.bfloat16)
    st = _lib.stream_handle(DEV)
    assert lib.lss_depthnet_pack(_lib.ptr(w), _lib.ptr(w), _lib.F32, 105, 500, _lib.ptr(buf), None, None, st) == -2
    assert lib.lss_depthnet_pack(_lib.ptr(w), _lib.ptr(w), _lib.F32, 129, 512, _lib.ptr(buf), None, None, st) == -2
    assert lib.lss_depthnet_pack(_lib.ptr(w), None, _lib.F32, 105, 512, _lib.ptr(buf), None, _lib.ptr(buf), st) == -1


@pytest.mark.parametrize("shape", [(1, 3, 5, 7, 41), (2, 5, 9, 13, 41), (1, 1, 8, 22, 60), (8, 6, 8, 22, 41)])
def test_nhwc_kernel_vs_fp64_conv(shape):
    """Odd maps, fewer pixels than CUs, D = 60: logits rounded to bf16 as the autocast conv's output,
    then the oracle's softmax / context layout."""
    B, N, H, W, D = shape
    feat, weight, bias = _inputs(B, N, H, W, D, seed=11)
    dims = _lib.Dims(B, N, D, H, W, 64)
    lib = _lib.load()
    depth, ctx_t = _run(lib.lss_depthnet_lift_nhwc, feat.to(DEV).contiguous(memory_format=torch.channels_last),
                           weight.to(DEV), bias.to(DEV), dims)
    logits = torch.einsum("nkhw,ok->nohw", feat.double(), weight.double()) + bias.double().view(1, -1, 1, 1)
    dn = logits.to(torch.bfloat16)
    want_depth, _ = ref.lift(dn.float(), D, 64)
    want_ctx = dn[:, D:].permute(0, 2, 3, 1).reshape(-1, 64)
    got_ctx = ctx_t.cpu()
    assert (got_ctx != want_ctx).float().mean().item() < 1e-3  # a logit on a bf16 rounding boundary may flip
    np.testing.assert_allclose(got_ctx.float().numpy(), want_ctx.float().numpy(), rtol=1e-2, atol=1e-2)
    np.testing.assert_allclose(depth.cpu().numpy(), want_depth.numpy(), rtol=2e-2, atol=1e-4)


def test_module_up1_channels_last_feeds_nhwc_lift():
    """Under bf16 autocast CamEncode.up1 runs channels-last, so the fused lift takes the pixel-row
    kernel; the BEV and the depthnet gradient match the NCHW up1 path."""
    cfg, gc, dac = syn.config_confs("c2")
    torch.manual_seed(0)
    m = L.compile_model(gc, dac, 1).to(DEV).eval()
    m.bev_layout = "nhwc"
    rig = {k: v.to(DEV) for k, v in syn.make_rig(cfg["B"], cfg["N"], cfg["final_dim"], seed=1).items()}
    imgs = syn.make_images(cfg["B"], cfg["N"], cfg["final_dim"]).to(DEV)
    seen = []
    orig = ops.DepthnetLiftSplat.forward

    def spy(ctx, feat, *a):
        seen.append(feat.is_contiguous(memory_format=torch.channels_last) and not feat.is_contiguous())
        return orig(ctx, feat, *a)
    outs = []
    from lss_carla_amd import models
    try:
        ops.DepthnetLiftSplat.forward = staticmethod(spy)
        for cl in (True, False):
            models.UP1_CHANNELS_LAST = cl
            m.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                bev = m.get_voxels(imgs, **rig)
            bev.float().square().mean().backward()
            outs.append((bev.detach().float(), m.camencode.depthnet.weight.grad.clone()))
    finally:
        models.UP1_CHANNELS_LAST = True
        ops.DepthnetLiftSplat.forward = orig
    assert seen == [True, False]
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=3e-2, atol=3e-2)
    rel = (outs[0][1] - outs[1][1]).norm() / outs[1][1].norm()
    assert rel < 3e-2, rel.item()


def test_flat_params_cast_writes_the_packed_depthnet_weight():
    """flat_params.FlatParams materialises the bf16 working copy and the depthnet weight in fragment
    order in one launch (lss_flat_cast_bf16): the copy equals torch's .to(bfloat16) of the fp32 master,
    the packed weight equals lss_depthnet_pack's, and the model's fused lift picks it up."""
    from lss_carla_amd.flat_params import FlatParams
    cfg, gc, dac = syn.config_confs("c1")
    torch.manual_seed(0)
    m = L.compile_model(gc, dac, 1).to(DEV)
    fp = FlatParams(m, cast_dtype=torch.bfloat16)
    assert fp.dn is not None
    with torch.no_grad():
        fp.master.add_(torch.randn_like(fp.master) * 1e-3)  # values a stale copy would not have
    t = fp.tensors()
    torch.cuda.synchronize()
    assert torch.equal(fp.work16, fp.master[:fp.n16].to(torch.bfloat16))
    w, b = t["camencode.depthnet.weight"], t["camencode.depthnet.bias"]
    packed, plain, b16 = _pack(m.camencode.depthnet.weight.detach().reshape(w.shape[0], -1), m.camencode.depthnet.bias.detach())
    assert torch.equal(fp.dn_packed, packed) and torch.equal(w.reshape(plain.shape), plain) and torch.equal(b, b16)
    assert m.camencode.depthnet.lss_packed_weight[1] == w.data_ptr()


def test_model_under_flat_params_takes_the_prepacked_weight():
    """The BEV of the model run on FlatParams' working copies (the prepacked depthnet weight, no pack
    launch) equals the BEV of the same model under plain autocast (the pack kernel on the fp32 weight)."""
    from lss_carla_amd.flat_params import FlatParams
    cfg, gc, dac = syn.config_confs("c2")
    torch.manual_seed(1)
    m = L.compile_model(gc, dac, 1).to(DEV).eval()
    m.bev_layout = "nhwc"
    fp = FlatParams(m, cast_dtype=torch.bfloat16)
    rig = {k: v.to(DEV) for k, v in syn.make_rig(cfg["B"], cfg["N"], cfg["final_dim"], seed=2).items()}
    imgs = syn.make_images(cfg["B"], cfg["N"], cfg["final_dim"], seed=2).to(DEV)
    seen = []
    m.bevencode.register_forward_pre_hook(lambda mod, a: seen.append(a[0].detach().clone()))
    calls = []
    orig = ops.DepthnetLiftSplat.forward

    def spy(ctx, *a):
        calls.append(a[-1] is not None)  # the prepacked weight handed over?
        return orig(ctx, *a)
    try:
        ops.DepthnetLiftSplat.forward = staticmethod(spy)
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            m(imgs, **rig)
            fp.bind(m)(imgs, **rig)
    finally:
        ops.DepthnetLiftSplat.forward = orig
    torch.cuda.synchronize()
    assert calls == [False, True]
    assert torch.equal(seen[0], seen[1])


def test_depthnet_wgrad_partials_fp32_vs_fp64():
    """The split-K depthnet weight gradient (ops._bmm_f32 + a slice-order sum) on zero-mean pixel
    gradients, whose sums cancel: every element within one bf16 rounding of the fp64 GEMM of the same
    bf16 operands (bf16 partials, rounded before the sum, were not)."""
    from lss_carla_amd import ops
    g = torch.Generator().manual_seed(5)
    npix, O, K = 8448, 105, 512
    dd = (torch.randn(npix, O, generator=g) * 1e-2).bfloat16()
    fm = torch.randn(npix, K, generator=g).bfloat16()
    S = ops._wgrad_splits(npix)
    ddd, fmd = dd.to(DEV), fm.to(DEV)
    part = ops._bmm_f32(ddd.view(S, npix // S, O).transpose(1, 2), fmd.view(S, npix // S, K))
    assert part.dtype == torch.float32
    got = part.sum(0).bfloat16().double().cpu()
    want = dd.double().t() @ fm.double()
    err = (got - want).abs()
    bound = want.abs() * 2.0 ** -8 + 1e-6 * want.abs().max()
    assert bool((err <= bound).all()), float((err / (want.abs() + 1e-30)).max())
