"""SimBEV input path on the device (lss_simbev_images / lss_simbev_vehicle_mask) vs the Pillow
restatement (oracle/simbev_ref.py, itself pinned to Pillow in test_simbev.py), vs Pillow directly, and
end to end through compile_data vs the reference loader's own output (tests/golden/simbev_ref.npz).
Bar: bit-exact (uint8 pixel arithmetic, then the same fp32 normalisation)."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs an MI355X", allow_module_level=True)

from PIL import Image  # noqa: E402

from oracle import simbev_ref as S  # noqa: E402
from lss_carla_amd import simbev  # noqa: E402

DEV = torch.device("cuda:0")


def _imgs(rng, n, H, W):
    yy, xx = np.mgrid[0:H, 0:W]
    out = []
    for i in range(n):
        base = np.sin(xx / (3 + i))[..., None] * 90 + np.cos(yy / (2 + i))[..., None] * 90 + 128
        out.append(np.clip(base + rng.normal(0, 20, (H, W, 3)), 0, 255).astype(np.uint8))
    return np.stack(out)


def _check(imgs, augs, fd):
    got = simbev.augment_images(torch.from_numpy(imgs).to(DEV), augs, fd).cpu().numpy()
    for i, a in enumerate(augs):
        u8 = S.img_transform(imgs[i], a["resize_dims"], a["crop"], a["flip"], a["rotate"])
        np.testing.assert_array_equal(got[i], S.normalize_img(u8), err_msg=str(a))
    return got


@pytest.mark.parametrize("H,W,fd", [(224, 480, (128, 352)), (56, 120, (32, 88)), (448, 960, (256, 704))])
def test_val_mode_augmentation(H, W, fd):
    """The SimBEV val crop (src/data_simbev.py:135-143) at the BASELINE sizes."""
    fH, fW = fd
    resize = max(fH / H, fW / W)
    rd = (int(W * resize), int(H * resize))
    crop_h = int(rd[1]) - fH
    crop_w = int(max(0, rd[0] - fW) / 2)
    a = {"resize_dims": rd, "crop": (crop_w, crop_h, crop_w + fW, crop_h + fH), "flip": False, "rotate": 0}
    _check(_imgs(np.random.default_rng(0), 3, H, W), [a] * 3, fd)


def test_train_mode_augmentation_random_draws():
    """Random resize / crop (partly outside the image) / flip / rotate draws, one per image."""
    rng = np.random.default_rng(1)
    H, W, fd = 112, 240, (64, 176)
    imgs = _imgs(rng, 12, H, W)
    augs = []
    for i in range(12):
        r = rng.uniform(0.55, 1.1)
        rd = (int(W * r), int(H * r))
        ch = int((1 - rng.uniform(0, 0.22)) * rd[1]) - fd[0]
        cw = int(rng.uniform(0, max(0, rd[0] - fd[1])))
        rot = [0.0, 180.0, -3.1, 5.4, 360.0, float(rng.uniform(-5.4, 5.4))][i % 6]
        augs.append({"resize_dims": rd, "crop": (cw, ch, cw + fd[1], ch + fd[0]), "flip": bool(i % 2), "rotate": rot})
    _check(imgs, augs, fd)


def test_square_crop_quarter_turns_and_pillow_directly():
    rng = np.random.default_rng(2)
    imgs = _imgs(rng, 4, 80, 100)
    augs = [{"resize_dims": (70, 56), "crop": (5, 3, 45, 43), "flip": f, "rotate": r}
            for f, r in ((False, 90.0), (True, 270.0), (False, -90.0), (True, 33.0))]
    got = _check(imgs, augs, (40, 40))
    for i, a in enumerate(augs):  # and against Pillow itself
        im = Image.fromarray(imgs[i]).resize(a["resize_dims"]).crop(a["crop"])
        if a["flip"]:
            im = im.transpose(Image.FLIP_LEFT_RIGHT)
        np.testing.assert_array_equal(got[i], S.normalize_img(np.asarray(im.rotate(a["rotate"]))))


def test_vehicle_mask():
    rng = np.random.default_rng(3)
    bev = (rng.random((3, 8, 200, 200)) < 0.05).astype(np.uint8) * rng.integers(1, 255, (3, 8, 200, 200)).astype(np.uint8)
    got = simbev.vehicle_masks(torch.from_numpy(bev).to(DEV)).cpu().numpy()
    for i in range(3):
        np.testing.assert_array_equal(got[i], S.vehicle_mask(bev[i]))
    got_b = simbev.vehicle_masks(torch.from_numpy(bev > 0).to(DEV)).cpu().numpy()  # bool maps
    np.testing.assert_array_equal(got_b, got)


def test_compile_data_end_to_end_vs_reference_loader():
    """Device batches from compile_data's loaders == the reference SegmentationData's samples
    (images through the reference's PIL path, normalised with torchvision's formula)."""
    z = np.load(os.path.join(GOLDEN, "simbev_ref.npz"))
    root = os.path.join(GOLDEN, "simbev_small")
    gc = {"xbound": [-50.0, 50.0, 0.5], "ybound": [-50.0, 50.0, 0.5], "zbound": [-10.0, 10.0, 20.0],
          "dbound": [4.0, 45.0, 1.0]}
    for split in ("train", "val"):
        dac = json.loads(str(z[f"{split}_aug"]))
        dac = {k: tuple(v) if isinstance(v, list) else v for k, v in dac.items()}
        ds = simbev.SegmentationData(root, is_train=split == "train", data_aug_conf=dac, grid_conf=gc)
        for i in range(len(ds)):
            np.random.seed(100 + i)
            raw = ds[i]
            batch = torch.utils.data.default_collate([raw])
            imgs, rots, trans, intrins, post_rots, post_trans, binimgs = simbev.finish_batch(batch, dac["final_dim"],
                                                                                              DEV)
            assert imgs.is_cuda and imgs.shape == (1, 6, 3) + tuple(dac["final_dim"])
            want = np.stack([S.normalize_img(u8) for u8 in z[f"{split}{i}_imgs_u8"]])
            np.testing.assert_array_equal(imgs[0].cpu().numpy(), want, err_msg=f"{split}{i}")
            np.testing.assert_array_equal(binimgs[0].cpu().numpy(), z[f"{split}{i}_binimg"])
            np.testing.assert_array_equal(post_rots[0].cpu().numpy(), z[f"{split}{i}_post_rots"])


def test_device_loader_batches():
    root = os.path.join(GOLDEN, "simbev_small")
    gc = {"xbound": [-50.0, 50.0, 0.5], "ybound": [-50.0, 50.0, 0.5], "zbound": [-10.0, 10.0, 20.0],
          "dbound": [4.0, 45.0, 1.0]}
    dac = {"resize_lim": (0.6, 0.9), "final_dim": (32, 88), "rot_lim": (-5.4, 5.4), "H": 56, "W": 120,
           "rand_flip": True, "bot_pct_lim": (0.0, 0.22), "Ncams": 6}
    tl, vl = simbev.compile_data("", root, dac, gc, bsz=2, nworkers=0, parser_name="segmentationdata", device=DEV)
    n = 0
    for batch in tl:
        assert len(batch) == 7 and batch[0].shape == (2, 6, 3, 32, 88) and batch[6].shape == (2, 1, 200, 200)
        assert all(t.is_cuda for t in batch)
        n += 1
    assert n == len(tl) == 4 and len(vl.dataset) == 2
