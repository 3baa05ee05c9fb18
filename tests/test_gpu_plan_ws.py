"""lss_plan_ws (the whole plan in one call, the scan's block prefixes from group sums left by the
geometry kernel) vs lss_geometry_cells + lss_csr_build_ws (look-back scan): the same cell_of,
cell_start, sorted_key, sorted_row bit for bit -- the reference's ids and stable argsort order
(src/models.py:205-231), pinned elsewhere against the golden SHA-256 of the ids -- over repeated calls
on one persistent workspace (left zero-filled by every call) and over random rigs."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU CI, skipped there
    pytest.skip("needs an MI355X", allow_module_level=True)

from oracle import lss_ref as ref  # noqa: E402
from lss_carla_amd import ops  # noqa: E402
from lss_carla_amd import synthetic as syn  # noqa: E402

DEV = torch.device("cuda:0")


def _plan(frustum, rig, grid, whole):
    old = ops.USE_PLAN_WS_CALL
    ops.USE_PLAN_WS_CALL = whole
    try:
        return ops.plan_from_cameras(frustum, **rig, grid=grid)
    finally:
        ops.USE_PLAN_WS_CALL = old


@pytest.mark.parametrize("name", ["c1", "c3", "c5"])
def test_plan_ws_matches_two_call_plan(name):
    cfg, gc, _ = syn.config_confs(name)
    B, N, fd = cfg["B"], cfg["N"], cfg["final_dim"]
    frustum = ref.create_frustum(fd, gc["dbound"]).to(DEV)
    grid = ops.GridSpec.from_conf(gc)
    for seed, aug in ((0, False), (3, True), (0, False)):
        rig = {k: v.to(DEV) for k, v in syn.make_rig(B, N, fd, seed=seed, aug=aug).items()}
        a = _plan(frustum, rig, grid, True)
        b = _plan(frustum, rig, grid, False)
        kept = int(b.cell_start[-1])
        for t in ("cell_of", "cell_start", "sorted_key"):
            assert torch.equal(getattr(a, t), getattr(b, t)), (name, seed, t)
        assert torch.equal(a.sorted_row[:kept], b.sorted_row[:kept])  # (defined for the kept entries)
    ws = ops.PLAN_WS.get(DEV, grid.ncells(B), B * N * frustum.shape[0] * frustum.shape[1] * frustum.shape[2], False)
    torch.cuda.synchronize()
    assert ws is not None and int(ws.counts.abs().sum()) == 0 and int(ws.workspace.abs().sum()) == 0


def test_plan_ws_coarse_grid_many_groups():
    """A grid of 4 x 10^6 cells per sample (977 scan blocks) and a 5 m grid (one scan block)."""
    for xy in ((-50.0, 50.0, 0.05), (-50.0, 50.0, 5.0)):
        gc = syn.grid_conf(xy=xy)
        B, N, fd = 2, 6, (128, 352)
        frustum = ref.create_frustum(fd, gc["dbound"]).to(DEV)
        grid = ops.GridSpec.from_conf(gc)
        rig = {k: v.to(DEV) for k, v in syn.make_rig(B, N, fd, seed=1).items()}
        a = _plan(frustum, rig, grid, True)
        b = _plan(frustum, rig, grid, False)
        assert torch.equal(a.cell_start, b.cell_start) and torch.equal(a.sorted_key, b.sorted_key)
