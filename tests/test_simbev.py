"""SimBEV input path, host side (CPU): the Pillow restatement (oracle/simbev_ref.py) against Pillow
itself, the product's coefficient tables / rotation coefficients / post-homography / dataset against
that restatement and against the reference's own loader output (tests/golden/simbev_ref.npz), and the
reference's validation helpers (tests/golden/val_info.json)."""
import json
import os

import numpy as np
import pytest
import torch
from hypothesis import given, settings, strategies as st
from PIL import Image

from conftest import GOLDEN
from oracle import simbev_ref as S
from lss_carla_amd import simbev
from lss_carla_amd import tools as T

SMALL = os.path.join(GOLDEN, "simbev_small")


def _img(rng, H, W, smooth):
    if smooth:
        yy, xx = np.mgrid[0:H, 0:W]
        base = np.sin(xx / 6.0)[..., None] * 90 + np.cos(yy / 4.0)[..., None] * 90 + 128
        return np.clip(base + rng.normal(0, 15, (H, W, 3)), 0, 255).astype(np.uint8)
    return rng.integers(0, 256, (H, W, 3), dtype=np.uint8)


# ----------------------------------------------------------------------------- oracle pinned to Pillow
@settings(max_examples=30, deadline=None)
@given(H=st.integers(8, 120), W=st.integers(8, 240), H2=st.integers(4, 160), W2=st.integers(4, 300),
       smooth=st.booleans(), seed=st.integers(0, 10_000))
def test_oracle_resize_is_pillow(H, W, H2, W2, smooth, seed):
    img = _img(np.random.default_rng(seed), H, W, smooth)
    np.testing.assert_array_equal(S.resize(img, (W2, H2)), np.asarray(Image.fromarray(img).resize((W2, H2))))


@settings(max_examples=30, deadline=None)
@given(H=st.integers(8, 100), W=st.integers(8, 200), angle=st.floats(-360, 360, allow_nan=False),
       seed=st.integers(0, 10_000))
def test_oracle_rotate_is_pillow(H, W, angle, seed):
    img = _img(np.random.default_rng(seed), H, W, False)
    np.testing.assert_array_equal(S.rotate(img, angle), np.asarray(Image.fromarray(img).rotate(angle)))


@pytest.mark.parametrize("angle", [0.0, 90.0, 180.0, 270.0, -90.0, 5.4, -5.4, 360.0])
@pytest.mark.parametrize("shape", [(40, 40), (32, 88)])
def test_oracle_rotate_fast_paths(angle, shape):
    img = _img(np.random.default_rng(1), *shape, False)
    np.testing.assert_array_equal(S.rotate(img, angle), np.asarray(Image.fromarray(img).rotate(angle)))


@pytest.mark.parametrize("box", [(0, 0, 60, 50), (-5, 3, 40, 70), (10, -4, 70, 20), (30, 30, 30, 40)])
def test_oracle_crop_flip_is_pillow(box):
    img = _img(np.random.default_rng(2), 50, 60, False)
    np.testing.assert_array_equal(S.crop(img, box), np.asarray(Image.fromarray(img).crop(box)))
    np.testing.assert_array_equal(S.flip_lr(img), np.asarray(Image.fromarray(img).transpose(Image.FLIP_LEFT_RIGHT)))


# ----------------------------------------------------------------------------- product host pieces
@pytest.mark.parametrize("inn,outn", [(480, 352), (224, 164), (120, 88), (56, 41), (10, 300), (300, 7), (5, 5)])
def test_resample_tables_match_pillow_coefficients(inn, outn):
    k, tab = simbev.resample_table(inn, outn)
    if inn == outn:
        assert k == 0
        return
    bounds, coeffs = S.resample_coeffs(inn, outn)
    t = tab.reshape(outn, 2 + k)
    np.testing.assert_array_equal(t[:, :2], bounds)
    np.testing.assert_array_equal(t[:, 2:], coeffs)


@settings(max_examples=40, deadline=None)
@given(angle=st.floats(-30, 30, allow_nan=False), w=st.integers(8, 400), h=st.integers(8, 300))
def test_rotation_coefficients_match_pillow_path(angle, w, h):
    mode, co = simbev.rotation_mode(angle, w, h)
    a = angle % 360.0
    if a == 0:
        assert mode == 0
    elif a == 180:
        assert mode == 1
    elif mode == 2:
        assert co == S.affine_fixed(S.rotate_matrix(angle, w, h))


def _ref():
    return np.load(os.path.join(GOLDEN, "simbev_ref.npz"))


def test_post_homography_matches_reference_loader():
    z = _ref()
    # the draws of the reference's sample_augmentation, replayed with the same seeds
    for split, is_train in (("train", True), ("val", False)):
        dac = json.loads(str(z[f"{split}_aug"]))
        ds = _dataset(is_train, dac)
        assert len(ds) == int(z[f"{split}_len"])
        for i in range(len(ds)):
            np.random.seed(100 + i)
            raw = ds[i]
            imgs_u8, rots, trans, intrins, post_rots, post_trans, aug, rot, bev = raw
            for name, t in (("rots", rots), ("trans", trans), ("intrins", intrins), ("post_rots", post_rots),
                            ("post_trans", post_trans)):
                np.testing.assert_array_equal(t.numpy(), z[f"{split}{i}_{name}"], err_msg=f"{split}{i} {name}")
            # the pixel path on these draws (restated) == the reference's PIL output
            a = aug.tolist()
            for c in range(imgs_u8.shape[0]):
                got = S.img_transform(imgs_u8[c].numpy(), (a[0], a[1]), a[2:6], bool(a[6]), float(rot))
                np.testing.assert_array_equal(got, z[f"{split}{i}_imgs_u8"][c], err_msg=f"{split}{i} cam {c}")
            np.testing.assert_array_equal(S.vehicle_mask(bev.numpy()), z[f"{split}{i}_binimg"])


def _dataset(is_train, dac):
    gc = {"xbound": [-50.0, 50.0, 0.5], "ybound": [-50.0, 50.0, 0.5], "zbound": [-10.0, 10.0, 20.0],
          "dbound": [4.0, 45.0, 1.0]}
    dac = dict(dac)
    dac["final_dim"] = tuple(dac["final_dim"])
    for k in ("resize_lim", "rot_lim", "bot_pct_lim"):
        dac[k] = tuple(dac[k])
    return simbev.SegmentationData(SMALL, is_train=is_train, data_aug_conf=dac, grid_conf=gc)


def test_normalize_restates_torchvision():
    """ToTensor (uint8 / 255, fp32) then Normalize ((x - mean) / std, fp32): torchvision's published
    formula, evaluated with torch's own fp32 ops (torchvision itself is not installed)."""
    img = _img(np.random.default_rng(3), 7, 9, False)
    t = torch.from_numpy(img).permute(2, 0, 1).contiguous().to(torch.float32).div(255)
    mean = torch.as_tensor([0.485, 0.456, 0.406], dtype=torch.float32)[:, None, None]
    std = torch.as_tensor([0.229, 0.224, 0.225], dtype=torch.float32)[:, None, None]
    np.testing.assert_array_equal(S.normalize_img(img), t.sub(mean).div(std).numpy())


# ----------------------------------------------------------------------------- validation helpers (f4)
def _val_setup():
    z = np.load(os.path.join(GOLDEN, "val_inputs.npz"))

    class Toy(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter(torch.from_numpy(z["w"]))

        def forward(self, x, rots, trans, intrins, post_rots, post_trans):
            s = x.mean(dim=(1, 2, 3, 4)).view(-1, 1, 1, 1)
            return torch.sin(torch.arange(400.0).view(1, 1, 20, 20) * self.w[0] + s * 3.0) * 2.0 + self.w[1]

    batches = []
    for i in range(3):
        x = torch.from_numpy(z[f"x{i}"])
        batches.append((x, torch.zeros(2, 6, 3, 3), torch.zeros(2, 6, 3), torch.zeros(2, 6, 3, 3),
                        torch.zeros(2, 6, 3, 3), torch.zeros(2, 6, 3), torch.from_numpy(z[f"y{i}"])))

    class Loader(list):
        dataset = list(range(6))

    return Toy(), Loader(batches)


def test_get_val_info_matches_reference():
    want = json.load(open(os.path.join(GOLDEN, "val_info.json")))
    model, loader = _val_setup()
    got = T.get_val_info(model, loader, T.SimpleLoss(2.13), torch.device("cpu"), use_tqdm=False)
    assert set(got) == {"loss", "iou"}
    assert got["iou"] == pytest.approx(want["get_val_info"]["iou"], rel=1e-12)
    assert got["loss"] == pytest.approx(want["get_val_info"]["loss"], rel=1e-6)
    assert model.training  # restored to train mode, as the reference does
    preds = model(*loader[0][:6])
    assert list(T.get_batch_iou(preds, loader[0][6])) == pytest.approx(want["get_batch_iou"], rel=1e-12)


def test_val_info_empty_union_raises_like_reference():
    model, loader = _val_setup()
    empty = type(loader)([(b[0], *b[1:6], torch.zeros_like(b[6])) for b in loader])

    class Neg(torch.nn.Module):
        def forward(self, x, *a):
            return -torch.ones(x.shape[0], 1, 20, 20)

    with pytest.raises(ZeroDivisionError):
        T.get_val_info(Neg(), empty, T.SimpleLoss(2.13), torch.device("cpu"), use_tqdm=False)
    assert T.get_batch_iou(-torch.ones(1, 1, 4, 4), torch.zeros(1, 1, 4, 4))[2] == 1.0  # (union 0) -> 1.0
