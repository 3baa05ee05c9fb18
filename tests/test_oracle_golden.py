"""Pin the CPU oracle to vectors produced by the reference itself (tests/golden/make_golden.py).

These run without a GPU. They establish that ``oracle/lss_ref.py`` *is* the
reference's hot path (bit-exact geometry and voxel ids, bit-exact QuickCumsum
forward/backward), so the GPU parity tests may use it as the checker.
"""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

from oracle import lss_ref as ref
import lss_carla_amd.synthetic as syn

from conftest import GOLDEN


def _load(name):
    return np.load(os.path.join(GOLDEN, name))


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


@pytest.fixture(scope="module")
def facts():
    with open(os.path.join(GOLDEN, "facts.json")) as f:
        return json.load(f)


def test_gen_dx_bx_matches_reference_defaults():
    dx, bx, nx = ref.gen_dx_bx([-50.0, 50.0, 0.5], [-50.0, 50.0, 0.5], [-10.0, 10.0, 20.0])
    assert dx.tolist() == [0.5, 0.5, 20.0]
    assert bx.tolist() == [-49.75, -49.75, 0.0]
    assert nx.tolist() == [200, 200, 1]


def test_frustum_bit_exact():
    z = _load("geom_small.npz")
    fr = ref.create_frustum((64, 176), (4.0, 45.0, 1.0)).numpy()
    assert fr.shape == (41, 4, 11, 3)
    np.testing.assert_array_equal(fr, z["frustum"])


@pytest.mark.parametrize("tag", ["plain", "aug"])
def test_geometry_bit_exact(tag):
    z = _load("geom_small.npz")
    rig = {k: _t(z[f"{tag}_{k}"]) for k in ("rots", "trans", "intrins", "post_rots", "post_trans")}
    geom = ref.get_geometry(z["frustum"], **rig)
    assert geom.dtype == np.float32
    np.testing.assert_array_equal(geom, z[f"{tag}_geom"])


def test_synthetic_rig_reproduces_fixture_inputs():
    z = _load("geom_small.npz")
    rig = syn.make_rig(2, 6, (64, 176), seed=3, aug=True)
    for k, v in rig.items():
        np.testing.assert_array_equal(v.numpy(), z[f"aug_{k}"])


@pytest.mark.parametrize("name", ["c1", "c2", "c3", "c5"])
def test_full_size_voxel_ids_digest(name, facts):
    """Bit-exact voxel ids at full size, via SHA-256 of the reference's own ids."""
    f = facts[name]
    cfg, gcf, dacf = syn.config_confs(name)
    rig = syn.make_rig(cfg["B"], cfg["N"], cfg["final_dim"], seed=0)
    fr = ref.create_frustum(cfg["final_dim"], gcf["dbound"])
    geom = ref.get_geometry(fr, **rig)
    dx, bx, nx = ref.gen_dx_bx(gcf["xbound"], gcf["ybound"], gcf["zbound"])
    ids, kept = ref.quantize(geom, dx, bx, nx)
    assert hashlib.sha256(geom.tobytes()).hexdigest() == f["sha256_geom_f32"]
    assert hashlib.sha256(ids[:, :3].astype(np.int32).tobytes()).hexdigest() == f["sha256_ids_int32"]
    assert hashlib.sha256(kept.astype(np.uint8).tobytes()).hexdigest() == f["sha256_kept_u8"]
    st = ref.voxel_stats(geom, dx, bx, nx)
    for k in ("nprime", "kept", "occupied", "max_per_voxel", "trunc_ne_floor"):
        assert st[k] == f[k], k


def test_known_answer_facts_config3(facts):
    f = facts["c3"]
    assert (f["kept"], f["occupied"], f["max_per_voxel"], f["trunc_ne_floor"]) == (344720, 40727, 40, 9432)
    f5 = facts["c5"]
    assert (f5["kept"], f5["occupied"], f5["max_per_voxel"]) == (794837, 48404, 64)


def test_lift_matches_reference():
    z = _load("lift_small.npz")
    conv = torch.nn.Conv2d(512, 105, 1)
    with torch.no_grad():
        conv.weight.copy_(_t(z["weight"]))
        conv.bias.copy_(_t(z["bias"]))
        dn = conv(_t(z["feat"]))
        depth, new_x = ref.lift(dn, 41, 64)
    np.testing.assert_array_equal(depth.numpy(), z["depth"])
    np.testing.assert_array_equal(new_x.numpy(), z["new_x"])


def _pool_inputs():
    z = _load("pool_small.npz")
    g = z["grid"]
    gc = syn.grid_conf(xy=tuple(g[0:3]), z=tuple(g[3:6]), dbound=tuple(g[6:9]))
    rig = {k: _t(z[k]) for k in ("rots", "trans", "intrins", "post_rots", "post_trans")}
    dx, bx, nx = ref.gen_dx_bx(gc["xbound"], gc["ybound"], gc["zbound"])
    fr = ref.create_frustum((64, 176), gc["dbound"])
    return z, rig, dx, bx, nx, fr


@pytest.mark.parametrize("quick", [True, False])
def test_voxel_pooling_matches_reference(quick):
    z, rig, dx, bx, nx, fr = _pool_inputs()
    geom = ref.get_geometry(fr, **rig)
    np.testing.assert_array_equal(geom, z["geom"])
    dn = _t(z["depthnet_out"])
    _, new_x = ref.lift(dn, 41, 64)
    x = ref.cam_feats_layout(new_x, 2, 6)
    assert hashlib.sha256(x.contiguous().numpy().tobytes()).hexdigest() == str(z["x_lifted_sha256"])
    bev = ref.voxel_pooling(geom, x, dx, bx, nx, use_quickcumsum=quick).numpy()
    want = z["bev_quick" if quick else "bev_autograd"]
    # argsort is unstable, so the within-voxel order (and thus the last bits) can differ.
    np.testing.assert_allclose(bev, want, rtol=0, atol=2e-5)
    exact = ref.voxel_pooling_fp64(geom, x.detach().numpy(), dx, bx, nx)
    np.testing.assert_allclose(exact, z["bev_fp64"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(bev, exact, rtol=0, atol=3e-5)


def test_splat_backward_matches_reference():
    z, rig, dx, bx, nx, fr = _pool_inputs()
    gz = _load("grad_small.npz")
    geom = ref.get_geometry(fr, **rig)
    dn = _t(z["depthnet_out"]).requires_grad_(True)
    _, new_x = ref.lift(dn, 41, 64)
    bev = ref.voxel_pooling(geom, ref.cam_feats_layout(new_x, 2, 6), dx, bx, nx, use_quickcumsum=True)
    (bev * _t(gz["dbev"])).sum().backward()
    np.testing.assert_allclose(dn.grad.numpy(), gz["d_depthnet_out_quick"], rtol=1e-5, atol=1e-6)
    analytic = ref.lift_splat_backward_fp64(z["depthnet_out"], geom, gz["dbev"], dx, bx, nx, 41, 64)
    np.testing.assert_allclose(analytic, gz["d_depthnet_out_quick"], rtol=1e-4, atol=2e-5)
    np.testing.assert_allclose(analytic, gz["d_depthnet_out_autograd"], rtol=1e-4, atol=5e-5)


def test_all_points_out_of_grid_gives_zero_bev():
    z, rig, dx, bx, nx, fr = _pool_inputs()
    geom = ref.get_geometry(fr, **rig) + np.float32(1000.0)
    _, new_x = ref.lift(_t(z["depthnet_out"]), 41, 64)
    exact = ref.voxel_pooling_fp64(geom, ref.cam_feats_layout(new_x, 2, 6).numpy(), dx, bx, nx)
    assert not exact.any()
