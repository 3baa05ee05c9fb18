"""Round-2 golden fixtures, generated from the REFERENCE itself (build container only).

Same recipe as make_golden.py: the reference's ``src`` package imported with inert
stubs for third-party modules its hot path does not use, ``Tensor.cuda`` the identity, no bytecode
written into the read-only mount. What it stores (data only):

  simbev_small/      a synthetic SimBEV directory tree (SimBEV_cvt_label/scene_*/yaw0pitch0/meta.json,
                     bev_*.npz, sweeps/RGB-CAM_*/*.jpg) -- the input of the loader fixtures
  simbev_ref.npz     the reference's SegmentationData (src/data_simbev.py) on that tree, train split
                     with augmentation (resize / crop / flip / rotate draws, np.random seeded) and val
                     split: the camera images right after img_transform as uint8 (normalize_img --
                     torchvision, absent here -- is captured before it runs, see below), rots, trans,
                     intrins, post_rots, post_trans, binimg
  pool_z2.npz        the reference's voxel_pooling on a two-z-bin grid (zbound [-10, 10, 10]): the
                     z*C + c channel order of the collapsed BEV (src/models.py:239-244)
  val_info.json      the reference's get_val_info / get_batch_iou (src/tools.py:232-270) on a fixed
                     toy model and loader

normalize_img is torchvision's ToTensor + Normalize; torchvision is not installed, so the fixture
captures the PIL image handed to it (as uint8) and the normalisation is checked against its published
formula in tests/test_simbev.py.

Usage:  PYTHONDONTWRITEBYTECODE=1 python -B tests/golden/make_golden_r2.py
"""
from __future__ import annotations

import json
import os
import shutil
import sys

sys.dont_write_bytecode = True

import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
from make_golden import _import_reference, _ref_module  # noqa: E402

SMALL_H, SMALL_W = 56, 120          # a 224x480 SimBEV camera at 1/4 scale
FINAL_DIM = (32, 88)


def make_dataset(root: str, n_scenes: int = 5, per_scene: int = 2, seed: int = 0) -> None:
    """Synthetic SimBEV tree: smooth coloured images with noise (JPEG), 8-class BEV npz (bool)."""
    from PIL import Image
    rng = np.random.default_rng(seed)
    cams = ["CAM_FRONT_LEFT", "CAM_FRONT", "CAM_FRONT_RIGHT", "CAM_BACK_LEFT", "CAM_BACK", "CAM_BACK_RIGHT"]
    yy, xx = np.mgrid[0:SMALL_H, 0:SMALL_W].astype(np.float64)
    for s in range(n_scenes):
        meta_dir = os.path.join(root, "SimBEV_cvt_label", f"scene_{s:04d}", "yaw0pitch0")
        os.makedirs(meta_dir, exist_ok=True)
        samples = []
        for k in range(per_scene):
            token = f"s{s}_{k}"
            images = []
            for ci, cam in enumerate(cams):
                d = os.path.join(root, "sweeps", f"RGB-{cam}")
                os.makedirs(d, exist_ok=True)
                f0, f1 = rng.uniform(3, 12, 2)
                img = np.stack([128 + 90 * np.sin(xx / f0 + c) * np.cos(yy / f1 - c) for c in range(3)], -1)
                img = np.clip(img + rng.normal(0, 12, img.shape), 0, 255).astype(np.uint8)
                rel = os.path.join("sweeps", f"RGB-{cam}", f"{token}.jpg")
                Image.fromarray(img).save(os.path.join(root, rel), quality=90)
                images.append(rel)
            fx = SMALL_W / (2 * np.tan(np.radians(35.0)))
            K = [[fx, 0, SMALL_W / 2], [0, fx, SMALL_H / 2], [0, 0, 1]]
            extr = []
            for ci in range(6):
                yaw = np.radians([55, 0, -55, 110, 180, -110][ci])
                E = np.eye(4)
                E[:3, :3] = np.array([[np.cos(yaw), -np.sin(yaw), 0], [np.sin(yaw), np.cos(yaw), 0], [0, 0, 1]]) @ \
                    np.array([[0, 0, 1], [-1, 0, 0], [0, -1, 0]])
                E[:3, 3] = [1.5 * np.cos(yaw), 0.5 * np.sin(yaw), 1.6 + rng.normal(0, 0.05)]
                extr.append(E.tolist())
            bev = rng.random((8, 200, 200)) < 0.02
            bev_name = f"bev_{token}.npz"
            np.savez_compressed(os.path.join(meta_dir, bev_name), bev=bev)
            samples.append({"token": token, "images": images, "intrinsics": [K] * 6, "extrinsics": extr,
                            "bev": bev_name})
        with open(os.path.join(meta_dir, "meta.json"), "w") as f:
            json.dump(samples, f)


def main():
    sys.path.insert(0, REPO)
    ref_models, ref_tools = _import_reference()
    from src import data_simbev as ref_data  # noqa: E402

    root = os.path.join(HERE, "simbev_small")
    shutil.rmtree(root, ignore_errors=True)
    make_dataset(root)

    # normalize_img is torchvision (absent): capture the PIL image handed to it, as uint8 HWC
    ref_data.normalize_img = lambda img: torch.from_numpy(np.asarray(img, dtype=np.uint8).copy())
    gc = {"xbound": [-50.0, 50.0, 0.5], "ybound": [-50.0, 50.0, 0.5], "zbound": [-10.0, 10.0, 20.0],
          "dbound": [4.0, 45.0, 1.0]}
    out = {}
    for split, is_train, dac in (
            ("train", True, {"resize_lim": (0.6, 0.9), "final_dim": FINAL_DIM, "rot_lim": (-5.4, 5.4),
                             "H": SMALL_H, "W": SMALL_W, "rand_flip": True, "bot_pct_lim": (0.0, 0.22),
                             "Ncams": 6}),
            ("val", False, {"resize_lim": (1.0, 1.0), "final_dim": FINAL_DIM, "rot_lim": (0.0, 0.0),
                            "H": SMALL_H, "W": SMALL_W, "rand_flip": False, "bot_pct_lim": (0.0, 0.0),
                            "Ncams": 6})):
        ds = ref_data.SegmentationData(root, is_train=is_train, data_aug_conf=dac, grid_conf=gc)
        for i in range(len(ds)):
            np.random.seed(100 + i)
            imgs, rots, trans, intrins, post_rots, post_trans, binimg = ds[i]
            for name, t in (("imgs_u8", imgs), ("rots", rots), ("trans", trans), ("intrins", intrins),
                            ("post_rots", post_rots), ("post_trans", post_trans), ("binimg", binimg)):
                out[f"{split}{i}_{name}"] = t.numpy()
        out[f"{split}_len"] = np.array(len(ds))
        out[f"{split}_aug"] = np.array(json.dumps(dac, default=list))
    np.savez_compressed(os.path.join(HERE, "simbev_ref.npz"), **out)

    # ---------------------------------------------------------------- two z bins (Z = 2)
    import lss_carla_amd.synthetic as syn
    small_dim = (64, 176)
    gcz = syn.grid_conf(xy=(-12.5, 12.5, 0.5), z=(-10.0, 10.0, 10.0))
    dac = syn.data_aug_conf(small_dim)
    B, N, D, C = 2, 6, 41, 64
    rig = syn.make_rig(B, N, small_dim, seed=7)
    dn = syn.make_depthnet_out(B, N, D, small_dim[0] // 16, small_dim[1] // 16, C, seed=3)
    m = _ref_module(ref_models, ref_tools, gcz, dac, use_quickcumsum=True)
    geom = m.get_geometry(rig["rots"], rig["trans"], rig["intrins"], rig["post_rots"], rig["post_trans"])
    depth = dn[:, :D].softmax(dim=1)
    new_x = depth.unsqueeze(1) * dn[:, D:D + C].unsqueeze(2)
    x = new_x.view(B, N, C, D, small_dim[0] // 16, small_dim[1] // 16).permute(0, 1, 3, 4, 5, 2)
    bev = m.voxel_pooling(geom, x)
    z = {"depthnet_out": dn.numpy(), "bev_quick": bev.detach().numpy(), "geom": geom.numpy(),
         "grid": np.array(gcz["xbound"] + gcz["zbound"] + gcz["dbound"], dtype=np.float64)}
    z.update({k: v.numpy() for k, v in rig.items()})
    np.savez_compressed(os.path.join(HERE, "pool_z2.npz"), **z)

    # ---------------------------------------------------------------- get_val_info / get_batch_iou
    torch.manual_seed(0)

    class Toy(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter(torch.randn(3))

        def forward(self, x, rots, trans, intrins, post_rots, post_trans):
            s = x.mean(dim=(1, 2, 3, 4)).view(-1, 1, 1, 1)
            return torch.sin(torch.arange(400.0).view(1, 1, 20, 20) * self.w[0] + s * 3.0) * 2.0 + self.w[1]

    g = torch.Generator().manual_seed(5)
    batches = []
    for _ in range(3):
        batches.append((torch.randn(2, 6, 3, 8, 8, generator=g), torch.zeros(2, 6, 3, 3), torch.zeros(2, 6, 3),
                        torch.zeros(2, 6, 3, 3), torch.zeros(2, 6, 3, 3), torch.zeros(2, 6, 3),
                        (torch.rand(2, 1, 20, 20, generator=g) < 0.3).float()))

    class Loader(list):
        dataset = list(range(6))

    loader = Loader(batches)
    loss_fn = ref_tools.SimpleLoss(2.13)
    toy = Toy()
    info = ref_tools.get_val_info(toy, loader, loss_fn, torch.device("cpu"), use_tqdm=False)
    preds = toy(*batches[0][:6])
    inter, union, iou = ref_tools.get_batch_iou(preds, batches[0][6])
    arrays = {"w": toy.w.detach().numpy()}
    for i, b in enumerate(batches):
        arrays[f"x{i}"] = b[0].numpy()
        arrays[f"y{i}"] = b[6].numpy()
    np.savez_compressed(os.path.join(HERE, "val_inputs.npz"), **arrays)
    with open(os.path.join(HERE, "val_info.json"), "w") as f:
        json.dump({"get_val_info": info, "get_batch_iou": [inter, union, iou],
                   "generator": "tests/golden/make_golden_r2.py"}, f, indent=1)
    print("val_info", info, (inter, union, iou))


if __name__ == "__main__":
    main()
