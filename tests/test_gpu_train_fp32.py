"""The module in the reference's own training precision: fp32, ``train()`` mode, no autocast, eager,
torch Adam -- what an unchanged ``train_simbev.py`` runs (/root/reference/train_simbev.py:229-248).

One training forward/backward at a BASELINE size (config 2: B=4 x 6 cams x 128x352, D=41, 200x200),
dropout and drop-connect active as in training. Forward hooks capture what the hot path actually
received (the depthnet input and output of this very step) and what it produced (the BEV handed to
BevEncode, with its incoming gradient), so the oracle is applied to the same operands:

- the BEV vs ``ref.voxel_pooling_fp64`` of the captured depthnet output (src/models.py:204-246), 1e-4;
- d(depthnet output) vs ``ref.lift_splat_backward_fp64`` of the captured dBEV (src/tools.py:212-219,
  src/models.py:58-59), relative 1e-4;
- d(camencode.depthnet.weight) / d(bias) vs the fp64 1x1-conv backward of the captured depthnet
  input and that oracle gradient, relative 1e-4.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU CI, skipped there
    pytest.skip("needs an MI355X", allow_module_level=True)

from oracle import lss_ref as ref  # noqa: E402
import lss_carla_amd as L  # noqa: E402
from lss_carla_amd import synthetic as syn  # noqa: E402

DEV = torch.device("cuda:0")


def _rel(a, b) -> float:
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.parametrize("name", ["c2"])
def test_fp32_train_mode_module_vs_oracle(name):
    cfg, gc, dac = syn.config_confs(name)
    B, N, fd = cfg["B"], cfg["N"], cfg["final_dim"]
    torch.manual_seed(0)
    m = L.compile_model(gc, dac, 1).to(DEV).train()
    assert m.bev_layout == "nhwc"  # the module default an unchanged caller gets
    rig = syn.make_rig(B, N, fd, seed=3)
    rdev = {k: v.to(DEV) for k, v in rig.items()}
    imgs = syn.make_images(B, N, fd, seed=3).to(DEV)
    labels = syn.make_labels(B, 200, 200, seed=3).to(DEV)
    loss_fn = L.SimpleLoss(2.13).to(DEV)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-7)

    cap = {}

    def dn_hook(mod, inp, out):
        cap["feat"] = inp[0].detach()
        out.retain_grad()
        cap["dn"] = out

    def bev_hook(mod, inp):
        inp[0].retain_grad()
        cap["bev"] = inp[0]

    h1 = m.camencode.depthnet.register_forward_hook(dn_hook)
    h2 = m.bevencode.register_forward_pre_hook(bev_hook)
    try:
        # train_simbev.py:229-248, unchanged
        opt.zero_grad()
        preds = m(imgs, **rdev)
        loss = loss_fn(preds, labels)
        loss.backward()
        # (read before clip_grad_norm_ rescales them in place)
        dw = m.camencode.depthnet.weight.grad.detach().double().cpu().numpy()
        db = m.camencode.depthnet.bias.grad.detach().double().cpu().numpy()
        torch.nn.utils.clip_grad_norm_(m.parameters(), 5.0)
        opt.step()
    finally:
        h1.remove()
        h2.remove()
    assert preds.dtype == torch.float32 and preds.shape == (B, 1, 200, 200)
    assert torch.isfinite(loss).item()
    assert "dn" in cap, "the fp32 path no longer runs depthnet as its own conv; capture moved"

    frustum = m.frustum.detach().cpu()
    D = frustum.shape[0]
    dx, bx, nx = ref.gen_dx_bx(gc["xbound"], gc["ybound"], gc["zbound"])
    geom = ref.get_geometry(frustum, **rig)
    dn = cap["dn"].detach().float().cpu()
    _, new_x = ref.lift(dn, D, 64)
    exact = ref.voxel_pooling_fp64(geom, ref.cam_feats_layout(new_x, B, N).numpy(), dx, bx, nx)
    bev = cap["bev"].detach().float().cpu().numpy()
    np.testing.assert_allclose(bev, exact, rtol=1e-5, atol=1e-4)

    dbev = cap["bev"].grad.detach().double().cpu().numpy()
    d_dn = ref.lift_splat_backward_fp64(dn.numpy(), geom, dbev, dx, bx, nx, D, 64)
    got_d_dn = cap["dn"].grad.detach().double().cpu().numpy()
    r = _rel(got_d_dn, d_dn)
    assert r < 1e-4, f"d(depthnet output) rel {r:.2e}"

    feat = cap["feat"].double().cpu()
    w_shape = m.camencode.depthnet.weight.shape
    dw_ref = torch.nn.grad.conv2d_weight(feat, w_shape, torch.from_numpy(d_dn)).numpy()
    db_ref = d_dn.sum(axis=(0, 2, 3))
    r_w = _rel(dw, dw_ref)
    r_b = _rel(db, db_ref)
    assert r_w < 1e-4, f"d(depthnet.weight) rel {r_w:.2e}"
    assert r_b < 1e-4, f"d(depthnet.bias) rel {r_b:.2e}"
    assert all(torch.isfinite(p).all() for p in m.parameters())  # the update ran on finite values
