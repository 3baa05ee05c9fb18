"""Plans without the canonical pass (ops.plan_from_cameras(canonical=False), lss_csr_build_ws without
sorted_row) and the channels-last splat that orders each cell itself (LSS_SPLAT_UNORDERED).

The unordered CSR must hold exactly the canonical CSR's entries per cell (the reference's stable
argsort, src/models.py:225-231, up to the order inside a cell) with the same cell_start and sentinel
tail, and the splat over it must give the canonical splat's bits: fused bf16 / fp32 rows, lifted rows,
cells longer than a chunk window (the big-cell path, in LDS and by selection from memory).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU CI, skipped there
    pytest.skip("needs an MI355X", allow_module_level=True)

from oracle import lss_ref as ref  # noqa: E402
import lss_carla_amd as L  # noqa: E402
from lss_carla_amd import _lib, models, ops  # noqa: E402
from lss_carla_amd import synthetic as syn  # noqa: E402

DEV = torch.device("cuda:0")


def _plans(name, seed=0, aug=False, gc=None):
    cfg, gc0, _ = syn.config_confs(name)
    gc = gc or gc0
    B, N, fd = cfg["B"], cfg["N"], cfg["final_dim"]
    rig = {k: v.to(DEV) for k, v in syn.make_rig(B, N, fd, seed=seed, aug=aug).items()}
    frustum = ref.create_frustum(fd, gc["dbound"]).to(DEV)
    grid = ops.GridSpec.from_conf(gc)
    canon = ops.plan_from_cameras(frustum, **rig, grid=grid)
    unord = ops.plan_from_cameras(frustum, **rig, grid=grid, canonical=False)
    return canon, unord


def _check_csr(canon, unord):
    assert canon.canonical and not unord.canonical and unord.sorted_row is None
    assert torch.equal(canon.cell_of, unord.cell_of) and torch.equal(canon.cell_start, unord.cell_start)
    kept = int(canon.cell_start[-1])
    # grouped by ascending cell: sorting the whole key list only reorders inside cells
    assert torch.equal((unord.sorted_key[:kept] >> 32), (canon.sorted_key[:kept] >> 32))
    assert torch.equal(torch.sort(unord.sorted_key[:kept]).values, canon.sorted_key[:kept])
    assert (unord.sorted_key[kept:] == -1).all() and (canon.sorted_key[kept:] == -1).all()
    return kept


def _splat(plan, depth, ctx, out_dtype, x_rows=None):
    B, N, D, H, W = plan.dims
    X, Y, Z = plan.grid.nx
    out = torch.full((B, Z * 64, X, Y), float("nan"), device=DEV, dtype=out_dtype).contiguous(
        memory_format=torch.channels_last)
    ops._splat_fwd_launch(plan, depth, ctx, x_rows, out, _lib.NHWC)
    torch.cuda.synchronize()
    return out


def _lift_inputs(plan, ctx_dtype, seed=3):
    B, N, D, H, W = plan.dims
    dn = syn.make_depthnet_out(B, N, D, H, W, seed=seed).to(DEV)
    depth = torch.softmax(dn[:, :D], dim=1).contiguous()
    ctx = dn[:, D:].permute(0, 2, 3, 1).reshape(-1, 64).to(ctx_dtype).contiguous()
    return depth, ctx


@pytest.mark.parametrize("name,aug", [("c1", False), ("c3", False), ("c3", True), ("c5", False), ("c5", True)])
def test_unordered_plan_and_splat_match_canonical(name, aug):
    canon, unord = _plans(name, seed=4, aug=aug)
    _check_csr(canon, unord)
    for ctx_dtype, out_dtype in ((torch.bfloat16, torch.bfloat16), (torch.float32, torch.float32),
                                 (torch.bfloat16, torch.float32)):
        depth, ctx = _lift_inputs(canon, ctx_dtype)
        a = _splat(canon, depth, ctx, out_dtype)
        b = _splat(unord, depth, ctx, out_dtype)
        assert torch.equal(a, b), (name, aug, ctx_dtype, out_dtype)


def test_unordered_lifted_rows_match_canonical():
    canon, unord = _plans("c2", seed=1)
    rows = torch.randn(canon.nprime, 64, generator=torch.Generator().manual_seed(5)).to(DEV)
    assert torch.equal(_splat(canon, None, None, torch.float32, x_rows=rows),
                       _splat(unord, None, None, torch.float32, x_rows=rows))


@pytest.mark.parametrize("xy", [(-50.0, 50.0, 5.0), (-50.0, 50.0, 12.5)])
def test_unordered_big_cells(xy):
    """Coarse grids: cells of hundreds to thousands of points (the big-cell path, in LDS up to 512
    entries and by selection beyond)."""
    gc = syn.grid_conf(xy=xy)
    canon, unord = _plans("c2", seed=2, gc=gc)
    _check_csr(canon, unord)
    cnt = canon.cell_start[1:] - canon.cell_start[:-1]
    assert int(cnt.max()) > 512  # the selection path too
    assert int(((cnt > 64) & (cnt <= 512)).sum()) > 0
    for ctx_dtype in (torch.bfloat16, torch.float32):
        depth, ctx = _lift_inputs(canon, ctx_dtype)
        assert torch.equal(_splat(canon, depth, ctx, torch.float32), _splat(unord, depth, ctx, torch.float32))


def test_unordered_plan_refused_by_the_nchw_splat():
    canon, unord = _plans("c1")
    depth, ctx = _lift_inputs(canon, torch.float32)
    B, N, D, H, W = unord.dims
    X, Y, Z = unord.grid.nx
    out = torch.empty(B, Z * 64, X, Y, device=DEV)
    with pytest.raises(RuntimeError, match="unordered plan"):
        ops._splat_fwd_launch(unord, depth, ctx, None, out, _lib.NCHW)


def test_module_unordered_plan_same_bev_and_grads():
    cfg, gc, dac = syn.config_confs("c2")
    torch.manual_seed(0)
    m = L.compile_model(gc, dac, 1).to(DEV).eval()
    m.bev_layout = "nhwc"
    rig = {k: v.to(DEV) for k, v in syn.make_rig(cfg["B"], cfg["N"], cfg["final_dim"], seed=1, aug=True).items()}
    imgs = syn.make_images(cfg["B"], cfg["N"], cfg["final_dim"]).to(DEV)
    outs, prev = [], models.UNORDERED_PLAN
    try:
        for flag in (True, False):
            models.UNORDERED_PLAN = flag
            m.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                bev = m.get_voxels(imgs, **rig)
            bev.float().square().mean().backward()
            outs.append((bev.detach(), m.camencode.depthnet.weight.grad.clone()))
    finally:
        models.UNORDERED_PLAN = prev
    assert torch.equal(outs[0][0], outs[1][0])  # the BEV bit for bit
    # the gradient within run-to-run noise (BevEncode's MIOpen backward is not bitwise reproducible)
    rel = ((outs[0][1] - outs[1][1]).norm() / outs[1][1].norm()).item()
    assert rel < 1e-3, rel
