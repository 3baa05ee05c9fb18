"""The LSS_DEBUG library (liblss_hip_debug.so): every data-derived global index of the kernels is checked
on the device (include/lss_hip.h, lss_debug_status).

* test_debug_build_parity_subset: the geometry / CSR / splat / backward / QuickCumsum parity tests and
  the fp32 NCHW module test (the one an illegal-address fault was once seen in, round 2) re-run in a
  child process on the debug library; conftest's fixture fails any test after which a check fired.
* test_debug_checks_fire: in that child, a deliberately corrupted CSR (a context row and a point id out
  of range, a total past the buffer) is reported by the checks instead of faulting the GPU.
"""
import os
import subprocess
import sys

import pytest
import torch

from conftest import REPO

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs an MI355X", allow_module_level=True)

IN_DEBUG = os.environ.get("LSS_DEBUG", "0") == "1"
SUBSET = ["tests/test_gpu_parity.py", "tests/test_gpu_quickcumsum.py",
          "tests/test_gpu_parity2.py::test_single_pass_scan_matches_two_kernel_csr",
          "tests/test_gpu_parity2.py::test_lookback_timeout_path_is_exact",
          "tests/test_gpu_parity2.py::test_plan_workspace_is_ordered_across_streams",
          "tests/test_gpu_parity2.py::test_csr_build_ws_direct",
          "tests/test_gpu_parity2.py::test_two_z_bins_vs_reference",
          "tests/test_gpu_debug.py::test_debug_checks_fire"]


@pytest.mark.skipif(IN_DEBUG, reason="the parent run starts the debug child")
def test_debug_build_parity_subset():
    lib = os.path.join(REPO, "lss-carla_amd", "liblss_hip_debug.so")
    assert os.path.exists(lib), "liblss_hip_debug.so not built (__graft_entry__.build())"
    env = dict(os.environ, LSS_DEBUG="1", LSS_HYP_EXAMPLES="5")
    env.pop("LSS_LIB", None)  # (an A/B run's release variant: the child takes the debug build)
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "gpu",
                        "--timeout", "120", "--timeout-method", "thread"] + SUBSET,
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    tail = (r.stdout + r.stderr)[-3000:]
    print(tail)
    assert r.returncode == 0, tail
    assert " passed" in r.stdout and " failed" not in r.stdout


@pytest.mark.skipif(not IN_DEBUG, reason="runs in the LSS_DEBUG child")
def test_debug_checks_fire():
    from oracle import lss_ref as ref
    from lss_carla_amd import _lib, ops, synthetic as syn

    lib = _lib.load()
    assert lib.lss_debug_checks() == 1
    dev = torch.device("cuda:0")
    cfg, gc, _ = syn.config_confs("c1")
    B, N, fd = 2, 6, cfg["final_dim"]
    frustum = ref.create_frustum(fd, gc["dbound"]).to(dev)
    rig = {k: v.to(dev) for k, v in syn.make_rig(B, N, fd, seed=1).items()}
    plan = ops.plan_from_cameras(frustum, **rig, grid=ops.GridSpec.from_conf(gc))
    D, H, W = frustum.shape[:3]
    dn = syn.make_depthnet_out(B, N, D, H, W, seed=1).to(dev)
    torch.cuda.synchronize()
    assert _lib.debug_status() == (0, 0, 0, 0)
    for layout, code in ((_lib.NHWC, 6), (_lib.NCHW, 6)):
        bad = ops.SplatPlan(plan.dims, plan.grid, plan.cell_of, plan.cell_start, plan.sorted_key,
                            plan.sorted_row.clone(), None)
        bad.sorted_row[3] = 10 ** 8  # a context row far outside the buffer
        ops.lift_splat(dn, bad, torch.float32, layout)
        torch.cuda.synchronize()
        st = _lib.debug_status()
        assert st[0] > 0 and st[1] == code and st[2] == 10 ** 8, st
    # a point id out of range in the keys (the depth-weight gather)
    bad = ops.SplatPlan(plan.dims, plan.grid, plan.cell_of, plan.cell_start, plan.sorted_key.clone(),
                        plan.sorted_row, None)
    bad.sorted_key[5] = (bad.sorted_key[5] >> 32 << 32) | (plan.nprime + 7)
    ops.lift_splat(dn, bad, torch.float32, _lib.NCHW)
    torch.cuda.synchronize()
    st = _lib.debug_status()
    assert st[0] > 0 and st[1] == 5 and st[2] == plan.nprime + 7, st
    # counts that do not start from zero (the stale-workspace hazard): the scatter and the CSR check fire
    counts = torch.full((plan.grid.ncells(B),), 10, device=dev, dtype=torch.int32)  # total 800,000 > nprime
    slot = torch.zeros(plan.nprime, device=dev, dtype=torch.int32)
    ops._build_csr(plan.cell_of, slot, counts, plan.dims, plan.grid.ncells(B), dev, None)
    torch.cuda.synchronize()
    st = _lib.debug_status()
    assert st[0] > 0 and st[1] in (1, 2), st
