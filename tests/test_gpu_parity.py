"""HIP hot path vs the CPU oracle (pinned to the reference by test_oracle_golden.py).

Bar (BASELINE.json north_star): voxel indices bit-exact, fp32 outputs within 1e-4.
The reference's own fp32 cumsum trick is off the exact segment sum by up to
~3e-5 at these sizes, so the BEV is compared against the fp64
segment sum with atol 1e-4 and against the reference-restating oracle with 1e-4.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU CI, skipped there
    pytest.skip("needs an MI355X", allow_module_level=True)

from oracle import lss_ref as ref  # noqa: E402
import lss_carla_amd as L  # noqa: E402
from lss_carla_amd import _lib, ops  # noqa: E402
from lss_carla_amd import synthetic as syn  # noqa: E402

DEV = torch.device("cuda:0")
ATOL = 1e-4


def _rig_dev(rig):
    return {k: v.to(DEV) for k, v in rig.items()}


def _setup(name, seed=0, aug=False):
    cfg, gc, dac = syn.config_confs(name)
    B, N, fd = cfg["B"], cfg["N"], cfg["final_dim"]
    rig = syn.make_rig(B, N, fd, seed=seed, aug=aug)
    frustum = ref.create_frustum(fd, gc["dbound"])
    D, H, W = frustum.shape[:3]
    dn = syn.make_depthnet_out(B, N, D, H, W, seed=seed)
    return cfg, gc, rig, frustum, dn


def _oracle_cells(frustum, rig, gc):
    geom = ref.get_geometry(frustum, **rig)
    dx, bx, nx = ref.gen_dx_bx(gc["xbound"], gc["ybound"], gc["zbound"])
    ids, kept = ref.quantize(geom, dx, bx, nx)
    cell = np.where(kept, ref.output_cell(ids, nx), -1).astype(np.int32)
    return geom, cell, (dx, bx, nx)


# ----------------------------------------------------------------------------- geometry
@pytest.mark.parametrize("tag", ["plain", "aug"])
def test_geometry_vs_golden(tag):
    z = np.load(os.path.join(GOLDEN, "geom_small.npz"))
    rig = {k: torch.from_numpy(z[f"{tag}_{k}"]).to(DEV) for k in ("rots", "trans", "intrins", "post_rots", "post_trans")}
    plan = ops.plan_from_cameras(torch.from_numpy(z["frustum"]).to(DEV), **rig,
                                 grid=ops.GridSpec.from_conf(syn.grid_conf()), want_geom=True, want_csr=False)
    np.testing.assert_array_equal(plan.geom.cpu().numpy(), z[f"{tag}_geom"])  # bit-exact


@pytest.mark.parametrize("name", ["c1", "c2", "c3", "c5"])
def test_voxel_ids_bit_exact_full_size(name):
    cfg, gc, rig, frustum, _ = _setup(name)
    geom, cell, _ = _oracle_cells(frustum, rig, gc)
    m_grid = ops.GridSpec.from_conf(gc)
    plan = ops.plan_from_cameras(frustum.to(DEV), **_rig_dev(rig), grid=m_grid, want_geom=True)
    np.testing.assert_array_equal(plan.cell_of.cpu().numpy(), cell)
    np.testing.assert_array_equal(plan.geom.cpu().numpy(), geom)
    _check_canonical_csr(plan, cell, m_grid.ncells(cfg["B"]))


def _check_canonical_csr(plan, cell, ncells):
    """lss_csr_build: ascending cell, then ascending point id (= the reference's stable argsort of
    ranks, src/models.py:228-231); sorted_row = the pixel of each point."""
    cs = plan.cell_start.cpu().numpy().astype(np.int64)
    total = int(cs[-1])
    sk = plan.sorted_key.cpu().numpy()[:total]
    kept = cell >= 0
    assert total == kept.sum()
    counts = np.bincount(cell[kept], minlength=ncells)
    np.testing.assert_array_equal(np.diff(cs), counts)
    want_p = np.nonzero(kept)[0][np.argsort(cell[kept], kind="stable")]
    np.testing.assert_array_equal(sk & 0xFFFFFFFF, want_p)
    np.testing.assert_array_equal(sk >> 32, np.repeat(np.arange(counts.size), counts))
    B, N, D, H, W = plan.dims
    cam, rem = np.divmod(want_p, D * H * W)
    np.testing.assert_array_equal(plan.sorted_row.cpu().numpy()[:total], cam * H * W + rem % (H * W))


def test_splat_chunk_and_tile_kernels_agree():
    """The channels-last chunk kernel and the NCHW tile kernel differ only in how a cell cut by a
    lane-group boundary is associated (both fp32, FMA per point)."""
    *_, bev_nhwc = _lift_splat("c3", _lib.NHWC)
    *_, bev_nchw = _lift_splat("c3", _lib.NCHW)
    torch.testing.assert_close(bev_nhwc.contiguous(), bev_nchw, rtol=0, atol=1e-5)
    # cells whose points all fall in one lane group are summed in the same order: most rows agree bitwise
    same = (bev_nhwc.contiguous() == bev_nchw).all(dim=1).float().mean().item()
    assert same > 0.9, same


def _dense_cell_geom(B, N, D, H, W, seed=0):
    """A geometry with a few very full cells (> 64 and > 128 points: the kernels' long-cell paths)
    and the rest scattered; grid 16 x 16 x 1 over [-8, 8)."""
    rng = np.random.default_rng(seed)
    nprime = B * N * D * H * W
    g = rng.uniform(-8, 8, size=(nprime, 3)).astype(np.float32)
    g[:, 2] = rng.uniform(-1, 1, size=nprime).astype(np.float32)
    perm = rng.permutation(nprime // B)  # the full cells in batch 0
    for n, xy in ((300, (0.25, 0.25)), (129, (3.5, -2.5)), (65, (-7.5, 7.5)), (64, (-0.75, 0.25))):
        pts, perm = perm[:n], perm[n:]
        g[pts, 0], g[pts, 1] = xy
    g[perm[:50], 0] = 100.0  # out of grid
    return g.reshape(B, N, D, H, W, 3)


@pytest.mark.parametrize("layout", [_lib.NCHW, _lib.NHWC])
def test_dense_cells_long_paths(layout):
    gc = syn.grid_conf(xy=(-8.0, 8.0, 1.0), z=(-2.0, 2.0, 4.0), dbound=(4.0, 45.0, 1.0))
    B, N, D, H, W = 2, 2, 41, 4, 22
    geom = _dense_cell_geom(B, N, D, H, W)
    dx, bx, nx = ref.gen_dx_bx(gc["xbound"], gc["ybound"], gc["zbound"])
    ids, kept = ref.quantize(geom, dx, bx, nx)
    cell = np.where(kept, ref.output_cell(ids, nx), -1).astype(np.int32)
    assert np.bincount(cell[cell >= 0]).max() >= 300
    grid = ops.GridSpec.from_conf(gc)
    plan = ops.plan_from_geom(torch.from_numpy(geom).to(DEV), grid)
    np.testing.assert_array_equal(plan.cell_of.cpu().numpy(), cell)
    _check_canonical_csr(plan, cell, grid.ncells(B))
    dn = syn.make_depthnet_out(B, N, D, H, W, seed=5)
    bev = ops.lift_splat(dn.to(DEV), plan, torch.float32, layout)
    _, new_x = ref.lift(dn, D, 64)
    x = ref.cam_feats_layout(new_x, B, N)
    exact = ref.voxel_pooling_fp64(geom, x.numpy(), dx, bx, nx)
    np.testing.assert_allclose(bev.float().cpu().numpy(), exact, rtol=0, atol=ATOL)
    # lifted rows through the same plan
    m = L.compile_model(gc, syn.data_aug_conf((64, 352)), 1).to(DEV)
    m.bev_layout = "nhwc" if layout == _lib.NHWC else "nchw"
    bev2 = m.voxel_pooling(torch.from_numpy(geom).to(DEV), x.to(DEV))
    np.testing.assert_allclose(bev2.float().cpu().numpy(), exact, rtol=0, atol=ATOL)


# ----------------------------------------------------------------------------- splat forward
def _lift_splat(name, layout, out_dtype=torch.float32, dn_dtype=torch.float32, seed=0):
    cfg, gc, rig, frustum, dn = _setup(name, seed)
    plan = ops.plan_from_cameras(frustum.to(DEV), **_rig_dev(rig), grid=ops.GridSpec.from_conf(gc))
    bev = ops.lift_splat(dn.to(DEV, dn_dtype), plan, out_dtype, layout)
    return cfg, gc, rig, frustum, dn, plan, bev


@pytest.mark.parametrize("name", ["c1", "c2", "c3"])
@pytest.mark.parametrize("layout", [_lib.NCHW, _lib.NHWC])
def test_lift_splat_fwd_vs_oracle(name, layout):
    cfg, gc, rig, frustum, dn, plan, bev = _lift_splat(name, layout)
    if layout == _lib.NHWC:
        assert bev.is_contiguous(memory_format=torch.channels_last)
    else:
        assert bev.is_contiguous()
    geom, _, (dx, bx, nx) = _oracle_cells(frustum, rig, gc)
    _, new_x = ref.lift(dn, geom.shape[2], 64)
    x = ref.cam_feats_layout(new_x, cfg["B"], cfg["N"])
    exact = ref.voxel_pooling_fp64(geom, x.numpy(), dx, bx, nx)
    got = bev.float().cpu().numpy()
    np.testing.assert_allclose(got, exact, rtol=0, atol=ATOL)
    want_ref = ref.voxel_pooling(geom, x, dx, bx, nx, use_quickcumsum=True).numpy()
    np.testing.assert_allclose(got, want_ref, rtol=0, atol=ATOL)
    # empty cells are exact zeros, occupied cells are written
    occ = np.abs(exact).sum(1) > 0
    assert not got.transpose(0, 2, 3, 1)[~occ].any()


def test_lift_splat_config5_hbm_stress():
    cfg, gc, rig, frustum, dn, plan, bev = _lift_splat("c5", _lib.NCHW)
    geom, _, (dx, bx, nx) = _oracle_cells(frustum, rig, gc)
    _, new_x = ref.lift(dn, geom.shape[2], 64)
    exact = ref.voxel_pooling_fp64(geom, ref.cam_feats_layout(new_x, cfg["B"], cfg["N"]).numpy(), dx, bx, nx)
    np.testing.assert_allclose(bev.cpu().numpy(), exact, rtol=0, atol=ATOL)


def test_lift_splat_bf16_io():
    cfg, gc, rig, frustum, dn, plan, bev = _lift_splat("c2", _lib.NHWC, torch.bfloat16, torch.bfloat16)
    assert bev.dtype == torch.bfloat16
    geom, _, (dx, bx, nx) = _oracle_cells(frustum, rig, gc)
    dnb = dn.to(torch.bfloat16).float()  # the kernel sees bf16-rounded logits / context
    _, new_x = ref.lift(dnb, geom.shape[2], 64)
    exact = ref.voxel_pooling_fp64(geom, ref.cam_feats_layout(new_x, cfg["B"], cfg["N"]).numpy(), dx, bx, nx)
    np.testing.assert_allclose(bev.float().cpu().numpy(), exact, rtol=1e-2, atol=2e-2)


def test_golden_pool_small():
    z = np.load(os.path.join(GOLDEN, "pool_small.npz"))
    g = z["grid"]
    gc = syn.grid_conf(xy=tuple(g[0:3]), z=tuple(g[3:6]), dbound=tuple(g[6:9]))
    frustum = ref.create_frustum((64, 176), gc["dbound"]).to(DEV)
    rig = {k: torch.from_numpy(z[k]).to(DEV) for k in ("rots", "trans", "intrins", "post_rots", "post_trans")}
    plan = ops.plan_from_cameras(frustum, **rig, grid=ops.GridSpec.from_conf(gc))
    bev = ops.lift_splat(torch.from_numpy(z["depthnet_out"]).to(DEV), plan).cpu().numpy()
    np.testing.assert_allclose(bev, z["bev_fp64"], rtol=0, atol=ATOL)
    np.testing.assert_allclose(bev, z["bev_quick"], rtol=0, atol=ATOL)


@pytest.mark.parametrize("layout", [_lib.NCHW, _lib.NHWC])
def test_deterministic_bitwise(layout):
    outs = [_lift_splat("c3", layout)[-1].cpu() for _ in range(2)]
    assert torch.equal(outs[0], outs[1])


def test_all_points_out_of_grid():
    cfg, gc, rig, frustum, dn = _setup("c2")
    rig = dict(rig)
    rig["trans"] = rig["trans"] + 1000.0
    plan = ops.plan_from_cameras(frustum.to(DEV), **_rig_dev(rig), grid=ops.GridSpec.from_conf(gc))
    assert int(plan.cell_start[-1]) == 0
    dnd = dn.to(DEV).requires_grad_(True)
    bev = ops.lift_splat(dnd, plan)
    assert not bev.any()
    bev.backward(torch.ones_like(bev))
    assert not dnd.grad.any()


# ----------------------------------------------------------------------------- backward
def _bwd(name, layout, g_dtype=torch.float32, seed=0):
    cfg, gc, rig, frustum, dn = _setup(name, seed)
    plan = ops.plan_from_cameras(frustum.to(DEV), **_rig_dev(rig), grid=ops.GridSpec.from_conf(gc))
    dnd = dn.to(DEV).requires_grad_(True)
    bev = ops.lift_splat(dnd, plan, torch.float32, layout)
    torch.manual_seed(seed + 11)
    dbev = torch.randn(bev.shape)
    gdev = dbev.to(DEV, g_dtype)
    if layout == _lib.NHWC:
        gdev = gdev.contiguous(memory_format=torch.channels_last)
    bev.backward(gdev)
    geom, _, (dx, bx, nx) = _oracle_cells(frustum, rig, gc)
    want = ref.lift_splat_backward_fp64(dn.numpy(), geom, gdev.float().cpu().numpy(), dx, bx, nx, geom.shape[2], 64)
    return dnd.grad.float().cpu().numpy(), want


@pytest.mark.parametrize("name", ["c1", "c2", "c3"])
@pytest.mark.parametrize("layout", [_lib.NCHW, _lib.NHWC])
def test_lift_splat_bwd_vs_oracle(name, layout):
    got, want = _bwd(name, layout)
    np.testing.assert_allclose(got, want, rtol=1e-4, atol=ATOL)


def test_lift_splat_bwd_golden_small():
    z = np.load(os.path.join(GOLDEN, "pool_small.npz"))
    gz = np.load(os.path.join(GOLDEN, "grad_small.npz"))
    g = z["grid"]
    gc = syn.grid_conf(xy=tuple(g[0:3]), z=tuple(g[3:6]), dbound=tuple(g[6:9]))
    frustum = ref.create_frustum((64, 176), gc["dbound"]).to(DEV)
    rig = {k: torch.from_numpy(z[k]).to(DEV) for k in ("rots", "trans", "intrins", "post_rots", "post_trans")}
    plan = ops.plan_from_cameras(frustum, **rig, grid=ops.GridSpec.from_conf(gc))
    dn = torch.from_numpy(z["depthnet_out"]).to(DEV).requires_grad_(True)
    bev = ops.lift_splat(dn, plan)
    bev.backward(torch.from_numpy(gz["dbev"]).to(DEV))
    np.testing.assert_allclose(dn.grad.cpu().numpy(), gz["d_depthnet_out_quick"], rtol=1e-4, atol=ATOL)


def test_bwd_bf16_grad():
    got, want = _bwd("c2", _lib.NHWC, torch.bfloat16)
    np.testing.assert_allclose(got, want, rtol=1e-3, atol=1e-3)


# ----------------------------------------------------------------------------- voxel_pooling(geom, x) boundary
def test_voxel_pooling_api_lifted():
    cfg, gc, rig, frustum, dn = _setup("c2")
    geom, _, (dx, bx, nx) = _oracle_cells(frustum, rig, gc)
    _, new_x = ref.lift(dn, geom.shape[2], 64)
    x = ref.cam_feats_layout(new_x, cfg["B"], cfg["N"])
    m = L.compile_model(gc, syn.data_aug_conf(cfg["final_dim"]), 1).to(DEV)
    xd = x.to(DEV).requires_grad_(True)
    bev = m.voxel_pooling(torch.from_numpy(geom).to(DEV), xd)
    exact = ref.voxel_pooling_fp64(geom, x.numpy(), dx, bx, nx)
    np.testing.assert_allclose(bev.cpu().detach().numpy(), exact, rtol=0, atol=ATOL)
    # QuickCumsum backward is a pure gather: bit-exact against the reference's grad
    torch.manual_seed(3)
    gup = torch.randn(bev.shape)
    bev.backward(gup.to(DEV))
    xr = x.clone().requires_grad_(True)
    ref.voxel_pooling(geom, xr, dx, bx, nx, use_quickcumsum=True).backward(gup)
    np.testing.assert_array_equal(xd.grad.cpu().numpy(), xr.grad.numpy())


def test_get_geometry_api():
    cfg, gc, rig, frustum, _ = _setup("c2")
    m = L.compile_model(gc, syn.data_aug_conf(cfg["final_dim"]), 1).to(DEV)
    geom = m.get_geometry(**_rig_dev(rig))
    np.testing.assert_array_equal(geom.cpu().numpy(), ref.get_geometry(frustum, **rig))


# ----------------------------------------------------------------------------- whole module
def test_module_get_voxels_matches_oracle_with_same_trunk():
    cfg, gc, rig, frustum, _ = _setup("c1")
    m = L.compile_model(gc, syn.data_aug_conf(cfg["final_dim"]), 1).to(DEV).eval()
    imgs = syn.make_images(cfg["B"], cfg["N"], cfg["final_dim"]).to(DEV)
    with torch.no_grad():
        bev = m.get_voxels(imgs, **_rig_dev(rig))
        dn = m.camencode.depthnet_out(imgs.view(-1, *imgs.shape[2:])).cpu()
    geom, _, (dx, bx, nx) = _oracle_cells(frustum, rig, gc)
    _, new_x = ref.lift(dn, geom.shape[2], 64)
    exact = ref.voxel_pooling_fp64(geom, ref.cam_feats_layout(new_x, cfg["B"], cfg["N"]).numpy(), dx, bx, nx)
    np.testing.assert_allclose(bev.cpu().numpy(), exact, rtol=1e-5, atol=ATOL)


def test_module_train_step_bf16_nhwc():
    cfg, gc, rig, frustum, _ = _setup("c2")
    m = L.compile_model(gc, syn.data_aug_conf(cfg["final_dim"]), 1).to(DEV).train()
    m.bev_layout = "nhwc"
    m.bevencode.to(memory_format=torch.channels_last)
    imgs = syn.make_images(cfg["B"], cfg["N"], cfg["final_dim"]).to(DEV)
    labels = syn.make_labels(cfg["B"], 200, 200).to(DEV)
    loss_fn = L.SimpleLoss(2.13).to(DEV)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-7)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = m(imgs, **_rig_dev(rig))
        loss = loss_fn(out.float(), labels)
    loss.backward()
    torch.nn.utils.clip_grad_norm_(m.parameters(), 5.0)
    opt.step()
    assert out.shape == (cfg["B"], 1, 200, 200)
    assert torch.isfinite(loss).item()
    g = m.camencode.depthnet.weight.grad
    assert g is not None and torch.isfinite(g).all() and g.abs().sum() > 0


def test_cpu_tensors_fail_loudly():
    cfg, gc, rig, frustum, _ = _setup("c1")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.plan_from_cameras(frustum, **rig, grid=ops.GridSpec.from_conf(gc))


# ----------------------------------------------------------------------------- depthnet fused into the lift (§8f row 1)
def _depthnet_inputs(name, seed=0, K=512):
    cfg, gc, rig, frustum, _ = _setup(name, seed)
    D, H, W = frustum.shape[:3]
    BN = cfg["B"] * cfg["N"]
    g = torch.Generator().manual_seed(seed + 100)
    feat = torch.randn(BN, K, H, W, generator=g).to(torch.bfloat16)
    weight = (torch.randn(D + 64, K, 1, 1, generator=g) * 0.05).to(torch.bfloat16)
    bias = (torch.randn(D + 64, generator=g) * 0.1).to(torch.bfloat16)
    plan = ops.plan_from_cameras(frustum.to(DEV), **_rig_dev(rig), grid=ops.GridSpec.from_conf(gc))
    return cfg, gc, rig, frustum, feat, weight, bias, plan


@pytest.mark.parametrize("name", ["c1", "c3"])
def test_depthnet_lift_kernel_vs_conv_then_lift_prep(name):
    """lss_depthnet_lift == bf16(conv1x1 in fp32) followed by lss_lift_prep, up to the rounding of a
    logit that lies on a bf16 rounding boundary (GEMM accumulation order)."""
    cfg, gc, rig, frustum, feat, weight, bias, plan = _depthnet_inputs(name)
    lib = _lib.load()
    B, N, D, H, W = plan.dims
    f, w, b = feat.to(DEV), weight.to(DEV), bias.to(DEV)
    depth = torch.empty(B * N, D, H, W, device=DEV)
    ctx_t = torch.empty(B * N * H * W, 64, device=DEV, dtype=torch.bfloat16)
    _lib.check(lib.lss_depthnet_lift(_lib.ptr(f), _lib.ptr(w.reshape(D + 64, -1).contiguous()), _lib.ptr(b),
                                     _lib.BF16, 512, plan.c_dims, _lib.ptr(depth), _lib.ptr(ctx_t), _lib.BF16,
                                     _lib.stream_handle(DEV)), "depthnet_lift")
    # reference: the conv in fp64 from the same bf16 operands, rounded to bf16 like the autocast conv output
    logits = torch.einsum("nkhw,ok->nohw", feat.double(), weight.double().flatten(1)) + bias.double().view(1, -1, 1, 1)
    dn = logits.to(torch.bfloat16)
    want_depth, _ = ref.lift(dn.float(), D, 64)
    want_ctx = dn[:, D:].permute(0, 2, 3, 1).reshape(-1, 64)
    got_ctx = ctx_t.cpu()
    ulp_flips = (got_ctx != want_ctx)
    assert ulp_flips.float().mean().item() < 1e-3
    np.testing.assert_allclose(got_ctx.float().numpy(), want_ctx.float().numpy(), rtol=1e-2, atol=1e-2)
    np.testing.assert_allclose(depth.cpu().numpy(), want_depth.numpy(), rtol=2e-2, atol=1e-4)


def test_depthnet_lift_splat_fwd_bwd_vs_unfused():
    """Fused depthnet+lift+splat vs the unfused path (MIOpen conv under autocast, then lift_splat)."""
    cfg, gc, rig, frustum, feat, weight, bias, plan = _depthnet_inputs("c2")
    fw = [t.to(DEV).float().requires_grad_(True) for t in (feat, weight, bias)]
    uw = [t.to(DEV).float().requires_grad_(True) for t in (feat, weight, bias)]
    with torch.autocast("cuda", dtype=torch.bfloat16):
        fused = ops.depthnet_lift_splat(fw[0], fw[1], fw[2], plan, torch.bfloat16, _lib.NHWC)
        dn = torch.nn.functional.conv2d(uw[0], uw[1], uw[2])
        unfused = ops.lift_splat(dn, plan, torch.bfloat16, _lib.NHWC)
    assert fused.dtype == torch.bfloat16 and fused.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(fused.float(), unfused.float(), rtol=2e-2, atol=2e-2)
    g = torch.randn(fused.shape, generator=torch.Generator().manual_seed(7)).to(DEV)
    g = g.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    fused.backward(g)
    unfused.backward(g)
    for a, b_, what in zip(fw, uw, ("feat", "weight", "bias")):
        assert a.grad is not None and torch.isfinite(a.grad).all(), what
        rel = (a.grad - b_.grad).norm() / b_.grad.norm()
        assert rel < 3e-2, (what, rel.item())


def test_module_fused_depthnet_train_step():
    cfg, gc, rig, frustum, _ = _setup("c2")
    torch.manual_seed(0)
    m = L.compile_model(gc, syn.data_aug_conf(cfg["final_dim"]), 1).to(DEV).eval()
    m.bev_layout = "nhwc"
    imgs = syn.make_images(cfg["B"], cfg["N"], cfg["final_dim"]).to(DEV)
    outs = []
    for fuse in (True, False):
        m.fuse_depthnet = fuse
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            bev = m.get_voxels(imgs, **_rig_dev(rig))
        bev.float().square().mean().backward()
        outs.append((bev.detach().float(), m.camencode.depthnet.weight.grad.clone()))
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=2e-2, atol=2e-2)
    rel = (outs[0][1] - outs[1][1]).norm() / outs[1][1].norm()
    assert rel < 3e-2, rel.item()


