"""The splat forward in two parts (lss_splat_zero_empty + lss_splat_fwd_occupied, ops.prefill_empty_rows):
the empty rows written on a second stream, the occupied rows by the splat, every element once, the same
bits as lss_splat_fwd (src/models.py:239-246: the dense BEV, empty cells zero)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU CI, skipped there
    pytest.skip("needs an MI355X", allow_module_level=True)

from oracle import lss_ref as ref  # noqa: E402
from lss_carla_amd import _lib, ops  # noqa: E402
from lss_carla_amd import synthetic as syn  # noqa: E402

DEV = torch.device("cuda:0")


def _setup(name, seed=1):
    cfg, gc, _ = syn.config_confs(name)
    B, N, fd = cfg["B"], cfg["N"], cfg["final_dim"]
    rig = {k: v.to(DEV) for k, v in syn.make_rig(B, N, fd, seed=seed).items()}
    frustum = ref.create_frustum(fd, gc["dbound"]).to(DEV)
    plan = ops.plan_from_cameras(frustum, **rig, grid=ops.GridSpec.from_conf(gc))
    D, H, W = frustum.shape[:3]
    return plan, B, N, D, H, W


@pytest.mark.parametrize("name", ["c1", "c3", "c5"])
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
def test_two_part_splat_bit_identical(name, out_dtype):
    plan, B, N, D, H, W = _setup(name)
    g = torch.Generator(device=DEV).manual_seed(2)
    dn = torch.randn(B * N, D + 64, H, W, device=DEV, generator=g).to(out_dtype)
    want = ops.lift_splat(dn, plan, out_dtype, _lib.NHWC)
    X, Y, Z = plan.grid.nx
    out = torch.full((B, Z * 64, X, Y), float("nan"), device=DEV, dtype=out_dtype).contiguous(
        memory_format=torch.channels_last)
    lib = _lib.load()
    st = _lib.stream_handle(DEV)
    _lib.check(lib.lss_splat_zero_empty(_lib.ptr(plan.cell_start), plan.c_dims, plan.grid.c_struct(), _lib.ptr(out),
                                        _lib.dtype_code(out_dtype), _lib.NHWC, st), "zero")
    torch.cuda.synchronize()
    empty = (plan.cell_start[1:] == plan.cell_start[:-1]).view(B, Z, X, Y)
    rows = out.view(B, Z, 64, X, Y).permute(0, 1, 3, 4, 2)
    assert torch.all(rows[empty] == 0) and torch.all(torch.isnan(rows[~empty].float()))
    depth = torch.empty(B * N, D, H, W, device=DEV)
    ctx_t = torch.empty(B * N * H * W, 64, device=DEV, dtype=out_dtype)
    _lib.check(lib.lss_lift_prep(_lib.ptr(dn), _lib.dtype_code(dn.dtype), plan.c_dims, _lib.ptr(depth),
                                 _lib.ptr(ctx_t), _lib.dtype_code(out_dtype), st), "prep")
    _lib.check(lib.lss_splat_fwd_occupied(_lib.ptr(depth), _lib.ptr(ctx_t), _lib.dtype_code(out_dtype), None,
                                          _lib.ptr(plan.cell_start), _lib.ptr(plan.sorted_key),
                                          _lib.ptr(plan.sorted_row), plan.c_dims, plan.grid.c_struct(),
                                          _lib.ptr(out), _lib.dtype_code(out_dtype), _lib.NHWC, st, None, None), "occ")
    torch.cuda.synchronize()
    assert torch.equal(out, want)


@pytest.mark.parametrize("name", ["c2", "c3"])
def test_prefill_through_ops_bit_identical(name):
    """ops.prefill_empty_rows on the side stream, joined by the splat: the fused and unfused autograd
    paths give the BEV of the one-kernel splat, and the same gradients."""
    plan, B, N, D, H, W = _setup(name, seed=4)
    g = torch.Generator(device=DEV).manual_seed(3)
    dn = torch.randn(B * N, D + 64, H, W, device=DEV, generator=g).to(torch.bfloat16).requires_grad_(True)
    want = ops.lift_splat(dn, plan, torch.bfloat16, _lib.NHWC)
    (gw,) = torch.autograd.grad(want.float().square().sum(), dn)
    got = ops.lift_splat(dn, plan, torch.bfloat16, _lib.NHWC, ops.prefill_empty_rows(plan, torch.bfloat16))
    (gg,) = torch.autograd.grad(got.float().square().sum(), dn)
    assert torch.equal(got, want) and torch.equal(gg, gw)
    feat = torch.randn(B * N, 512, H, W, device=DEV, generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn(D + 64, 512, 1, 1, device=DEV, generator=g) * 0.05
    b = torch.randn(D + 64, device=DEV, generator=g) * 0.1
    with torch.autocast("cuda", dtype=torch.bfloat16):
        a = ops.depthnet_lift_splat(feat, w, b, plan, torch.bfloat16, _lib.NHWC)
        c = ops.depthnet_lift_splat(feat, w, b, plan, torch.bfloat16, _lib.NHWC,
                                    ops.prefill_empty_rows(plan, torch.bfloat16))
    assert torch.equal(a, c)


def test_two_part_splat_rejects_nchw():
    plan, B, N, D, H, W = _setup("c1")
    X, Y, Z = plan.grid.nx
    out = torch.empty(B, Z * 64, X, Y, device=DEV)
    lib = _lib.load()
    assert lib.lss_splat_zero_empty(_lib.ptr(plan.cell_start), plan.c_dims, plan.grid.c_struct(), _lib.ptr(out),
                                    _lib.F32, _lib.NCHW, _lib.stream_handle(DEV)) == -2
    with pytest.raises(RuntimeError):
        ops.lift_splat(torch.zeros(B * N, D + 64, H, W, device=DEV), plan, torch.float32, _lib.NCHW,
                       ops.prefill_empty_rows(plan, torch.float32))
