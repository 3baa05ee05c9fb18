"""The reference's op-level boundary -- QuickCumsum / cumsum_trick (src/tools.py:182-219) -- on the
HIP segment kernels, against the reference's own outputs (golden pool_small / grad_small) and the
CPU oracle. Also the cumsum_check A/B of src/explore.py:119-191 (SURVEY.md §4 tier 4): the fused
module path vs the op-level pipeline, BEV output and depthnet.weight gradient.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs an MI355X", allow_module_level=True)

from oracle import lss_ref as ref  # noqa: E402
import lss_carla_amd as L  # noqa: E402
from lss_carla_amd import ops  # noqa: E402
from lss_carla_amd import synthetic as syn  # noqa: E402

DEV = torch.device("cuda:0")
ATOL = 1e-4


def hip_segment(fn):
    """segment_fn for oracle.voxel_pooling: the product operator on the device, results back on the CPU
    (autograd flows through the .to() copies)."""
    def run(x, geom_feats, ranks):
        xs, gs = fn(x.to(DEV), geom_feats.to(DEV), ranks.to(DEV))
        return xs.cpu(), gs.cpu()
    return run


def _golden_setup():
    z = np.load(os.path.join(GOLDEN, "pool_small.npz"))
    g = z["grid"]
    gc = syn.grid_conf(xy=tuple(g[0:3]), z=tuple(g[3:6]), dbound=tuple(g[6:9]))
    dx, bx, nx = ref.gen_dx_bx(gc["xbound"], gc["ybound"], gc["zbound"])
    return z, z["geom"], (dx, bx, nx)


@pytest.mark.parametrize("op", ["QuickCumsum", "cumsum_trick"])
def test_golden_pool_small_through_operator(op):
    z, geom, (dx, bx, nx) = _golden_setup()
    dn = torch.from_numpy(z["depthnet_out"])
    B, N = z["trans"].shape[:2]
    _, new_x = ref.lift(dn, 41, 64)
    x = ref.cam_feats_layout(new_x, B, N)
    fn = L.QuickCumsum.apply if op == "QuickCumsum" else L.cumsum_trick
    bev = ref.voxel_pooling(geom, x, dx, bx, nx, segment_fn=hip_segment(fn)).numpy()
    np.testing.assert_allclose(bev, z["bev_fp64"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(bev, z["bev_quick"], rtol=0, atol=ATOL)
    np.testing.assert_allclose(bev, z["bev_autograd"], rtol=0, atol=ATOL)


def test_golden_grad_small_through_operator():
    """d(loss)/d(depthnet_out) with the HIP QuickCumsum in the reference's voxel_pooling: the
    operator's backward is the reference's gather, so the gradient is the reference's."""
    z, geom, (dx, bx, nx) = _golden_setup()
    gz = np.load(os.path.join(GOLDEN, "grad_small.npz"))
    dn = torch.from_numpy(z["depthnet_out"]).requires_grad_(True)
    B, N = z["trans"].shape[:2]
    _, new_x = ref.lift(dn, 41, 64)
    bev = ref.voxel_pooling(geom, ref.cam_feats_layout(new_x, B, N), dx, bx, nx,
                            segment_fn=hip_segment(L.QuickCumsum.apply))
    (bev * torch.from_numpy(gz["dbev"])).sum().backward()
    np.testing.assert_allclose(dn.grad.numpy(), gz["d_depthnet_out_quick"], rtol=0, atol=1e-6)


def _random_runs(n, C, nruns, seed, long_run=0):
    g = torch.Generator().manual_seed(seed)
    ranks = torch.sort(torch.randint(0, nruns, (n,), generator=g)).values
    if long_run:
        ranks[:long_run] = -1  # one run of long_run rows at the front
    x = torch.randn(n, C, generator=g)
    geom = torch.randint(0, 200, (n, 4), generator=g)
    return x, geom, ranks


@pytest.mark.parametrize("n,C,nruns,long_run", [(1, 64, 1, 0), (7, 3, 2, 0), (1000, 64, 100, 0),
                                                (5000, 64, 4000, 0), (4096 * 3 + 5, 17, 50, 0),
                                                (3000, 64, 10, 1500)])
def test_operator_vs_reference_quickcumsum(n, C, nruns, long_run):
    x, geom, ranks = _random_runs(n, C, nruns, seed=n + C, long_run=long_run)
    want_x, want_g = ref.QuickCumsum.apply(x, geom, ranks)
    xd = x.to(DEV).requires_grad_(True)
    got_x, got_g = L.QuickCumsum.apply(xd, geom.to(DEV), ranks.to(DEV))
    assert got_x.shape == want_x.shape and got_g.dtype == torch.int64
    np.testing.assert_array_equal(got_g.cpu().numpy(), want_g.numpy())  # geom_feats[kept]: exact
    # exact run sums in fp64 (tolerance anchor) and the reference's prefix-difference result
    seg = torch.zeros(n, dtype=torch.long)
    seg[1:] = (ranks[1:] != ranks[:-1]).long().cumsum(0)
    exact = torch.zeros(want_x.shape, dtype=torch.float64).index_add_(0, seg, x.double())
    # fp32 sums of runs of up to 1,500 N(0,1) rows: absolute 1e-4 plus a relative 1e-5 for the long ones
    # (the reference's own prefix-difference error grows with the prefix: ~ulp of the running sum)
    np.testing.assert_allclose(got_x.detach().cpu().numpy(), exact.numpy(), rtol=1e-5, atol=ATOL)
    np.testing.assert_allclose(got_x.detach().cpu().numpy(), want_x.numpy(), rtol=1e-5, atol=ATOL)
    # backward: the reference's gather, bit for bit
    gup = torch.randn(want_x.shape, generator=torch.Generator().manual_seed(9))
    got_x.backward(gup.to(DEV))
    xr = x.clone().requires_grad_(True)
    ref.QuickCumsum.apply(xr, geom, ranks)[0].backward(gup)
    np.testing.assert_array_equal(xd.grad.cpu().numpy(), xr.grad.numpy())


def test_operator_empty_input():
    x = torch.empty(0, 64, device=DEV, requires_grad=True)
    out, g = L.QuickCumsum.apply(x, torch.empty(0, 4, dtype=torch.long, device=DEV),
                                 torch.empty(0, dtype=torch.long, device=DEV))
    assert out.shape == (0, 64) and g.shape == (0, 4)


def test_operator_cpu_tensors_fail_loudly():
    x, geom, ranks = _random_runs(10, 4, 3, seed=1)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        L.QuickCumsum.apply(x, geom, ranks)


@pytest.mark.parametrize("name", ["c2", "c3"])
def test_operator_full_size_vs_fused_splat(name):
    """At the BASELINE sizes: the op-level pipeline (lifted rows, ranks, argsort, QuickCumsum,
    griddify) and the fused CSR splat give the same BEV within 1e-4 (both within 1e-5 of fp64)."""
    cfg, gc, dac = syn.config_confs(name)
    B, N, fd = cfg["B"], cfg["N"], cfg["final_dim"]
    rig = syn.make_rig(B, N, fd, seed=0)
    frustum = ref.create_frustum(fd, gc["dbound"])
    D, H, W = frustum.shape[:3]
    dn = syn.make_depthnet_out(B, N, D, H, W, seed=0)
    geom = ref.get_geometry(frustum, **rig)
    dx, bx, nx = ref.gen_dx_bx(gc["xbound"], gc["ybound"], gc["zbound"])
    _, new_x = ref.lift(dn, D, 64)
    x = ref.cam_feats_layout(new_x, B, N)
    op_bev = ref.voxel_pooling(geom, x, dx, bx, nx, segment_fn=hip_segment(L.QuickCumsum.apply))
    plan = ops.plan_from_cameras(frustum.to(DEV), **{k: v.to(DEV) for k, v in rig.items()},
                                 grid=ops.GridSpec.from_conf(gc))
    fused = ops.lift_splat(dn.to(DEV), plan).cpu()
    np.testing.assert_allclose(op_bev.numpy(), fused.numpy(), rtol=0, atol=ATOL)


def test_cumsum_check_ab_module_vs_operator_pipeline():
    """src/explore.py:119-191 re-expressed: the same model in eval(), the BEV and
    camencode.depthnet.weight.grad through (A) the fused HIP module path and (B) the reference's
    voxel_pooling with the HIP QuickCumsum operator; plus the module's use_quickcumsum toggle."""
    cfg, gc, dac = syn.config_confs("c1")
    B, N, fd = 2, 6, cfg["final_dim"]
    rig = syn.make_rig(B, N, fd, seed=1)
    torch.manual_seed(0)
    m = L.compile_model(gc, syn.data_aug_conf(fd), 1).to(DEV).eval()
    imgs = syn.make_images(B, N, fd, seed=1).to(DEV)
    rdev = {k: v.to(DEV) for k, v in rig.items()}
    outs = {}
    for quick in (False, True):  # the reference toggles use_quickcumsum; both must agree
        m.use_quickcumsum = quick
        m.zero_grad(set_to_none=True)
        out = m(imgs, **rdev)
        out.mean().backward()
        outs[quick] = (out.detach().cpu(), m.camencode.depthnet.weight.grad.detach().cpu().clone())
    torch.testing.assert_close(outs[False][0], outs[True][0], rtol=0, atol=0)
    # the weight gradient passes MIOpen's backward convolutions, whose reductions are not bitwise
    # reproducible run to run: compare as a relative norm
    rel0 = ((outs[False][1] - outs[True][1]).norm() / outs[True][1].norm()).item()
    assert rel0 < 1e-4, rel0
    # (B): the op-level pipeline on the same trunk output, bevencode on the device
    m.zero_grad(set_to_none=True)
    frustum = m.frustum.detach().cpu()
    dx, bx, nx = ref.gen_dx_bx(gc["xbound"], gc["ybound"], gc["zbound"])
    feat = m.camencode.get_eff_depth(imgs.view(B * N, *imgs.shape[2:]))
    dn = m.camencode.depthnet(feat).cpu()
    bev = ref.get_voxels(frustum, dn, rig["rots"], rig["trans"], rig["intrins"], rig["post_rots"], rig["post_trans"],
                         dx, bx, nx, m.D, segment_fn=hip_segment(L.QuickCumsum.apply))
    out_b = m.bevencode(bev.to(DEV))
    out_b.mean().backward()
    np.testing.assert_allclose(out_b.detach().cpu().numpy(), outs[True][0].numpy(), rtol=1e-3, atol=1e-4)
    ga, gb = outs[True][1], m.camencode.depthnet.weight.grad.cpu()
    rel = ((ga - gb).norm() / gb.norm()).item()
    assert rel < 1e-3, rel
