"""SURVEY §8f row 4 on the device: the validation loop (src/tools.py:243-270, train_simbev.py:334) with
its loss / IoU accumulators on the MI355X and no host synchronisation per batch.

* the reference's get_val_info / get_batch_iou results (tests/golden/val_info.json, made by importing
  the reference) from a fixed toy model and loader, computed on the device;
* a LiftSplatShoot model over compile_data's DeviceLoader (the SimBEV test tree): the whole loop --
  JPEG pixels through the HIP augmentation kernels, the host torch.inverse of the rig (from the host
  copies the loader attaches), the hot path, the loss and IoU -- runs under
  torch.cuda.set_sync_debug_mode("error"), which raises on any synchronising call; the one read
  happens after the loop."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs an MI355X", allow_module_level=True)

import lss_carla_amd as L  # noqa: E402
from lss_carla_amd import simbev, tools as T  # noqa: E402

DEV = torch.device("cuda:0")


class _SyncErrors:
    def __enter__(self):
        torch.cuda.synchronize()
        torch.cuda.set_sync_debug_mode("error")

    def __exit__(self, *exc):
        torch.cuda.set_sync_debug_mode("default")


def _toy():
    z = np.load(os.path.join(GOLDEN, "val_inputs.npz"))

    class Toy(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter(torch.from_numpy(z["w"]))
            self.register_buffer("grid", torch.arange(400.0).view(1, 1, 20, 20))

        def forward(self, x, rots, trans, intrins, post_rots, post_trans):
            s = x.mean(dim=(1, 2, 3, 4)).view(-1, 1, 1, 1)
            return torch.sin(self.grid * self.w[0] + s * 3.0) * 2.0 + self.w[1]

    batches = []
    for i in range(3):
        x = torch.from_numpy(z[f"x{i}"]).to(DEV)
        zeros = [torch.zeros(s, device=DEV) for s in ((2, 6, 3, 3), (2, 6, 3), (2, 6, 3, 3), (2, 6, 3, 3), (2, 6, 3))]
        batches.append((x, *zeros, torch.from_numpy(z[f"y{i}"]).to(DEV)))

    class Loader(list):
        dataset = list(range(6))

    return Toy().to(DEV), Loader(batches)


def test_get_val_info_on_device_matches_reference():
    want = json.load(open(os.path.join(GOLDEN, "val_info.json")))
    model, loader = _toy()
    loss_fn = T.SimpleLoss(2.13).to(DEV)
    got = T.get_val_info(model, loader, loss_fn, DEV, use_tqdm=False)
    assert got["iou"] == pytest.approx(want["get_val_info"]["iou"], rel=1e-12)
    assert got["loss"] == pytest.approx(want["get_val_info"]["loss"], rel=1e-6)
    model.eval()
    with _SyncErrors():
        tl, ti, tu = T.val_totals(model, loader, loss_fn, DEV)
    assert (ti / tu).item() == pytest.approx(want["get_val_info"]["iou"], rel=1e-12)
    preds = model(*loader[0][:6])
    assert list(T.get_batch_iou(preds, loader[0][6])) == pytest.approx(want["get_batch_iou"], rel=1e-12)


def test_val_loop_over_device_loader_never_syncs():
    root = os.path.join(GOLDEN, "simbev_small")
    gc = {"xbound": [-50.0, 50.0, 0.5], "ybound": [-50.0, 50.0, 0.5], "zbound": [-10.0, 10.0, 20.0],
          "dbound": [4.0, 45.0, 1.0]}
    dac = {"resize_lim": (1.6, 1.8), "final_dim": (64, 192), "rot_lim": (-5.4, 5.4), "H": 56, "W": 120,
           "rand_flip": True, "bot_pct_lim": (0.0, 0.22), "Ncams": 6}
    tl, vl = simbev.compile_data("", root, dac, gc, bsz=2, nworkers=0, parser_name="segmentationdata", device=DEV)
    torch.manual_seed(0)
    model = L.compile_model(gc, dac, outC=1).to(DEV)
    loss_fn = T.SimpleLoss(2.13).to(DEV)
    model.eval()
    batches = list(vl) + list(tl)  # the loaders' batches, made once (their augmentation draws are random)
    torch.cuda.synchronize()
    with _SyncErrors():
        tot = T.val_totals(model, batches, loss_fn, DEV)
        with torch.no_grad():
            for b in tl:  # the loader itself (workers' raw samples -> device batches) inside the check too
                model(*b[:6])
    loss, inter, union = (t.item() for t in tot)
    # the same totals batch by batch with the reference's per-batch reads (src/tools.py:253-266)
    ref_loss, ref_i, ref_u = 0.0, 0.0, 0.0
    with torch.no_grad():
        for b in batches:
            preds = model(*b[:6])
            ref_loss += loss_fn(preds, b[6]).item() * preds.shape[0]
            i, u, _ = T.get_batch_iou(preds, b[6])
            ref_i += i
            ref_u += u
    assert np.isfinite(loss) and union > 0
    assert loss == pytest.approx(ref_loss, rel=1e-6) and inter == ref_i and union == ref_u
