"""CPU restatement of the SimBEV image / label path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module (as the checker of ``lss_carla_amd.simbev``'s HIP kernels).

The reference's per-camera image path is ``img_transform`` + ``normalize_img``
(``src/tools.py:120-144, 167-171``), driven by ``SimBEVDataset.sample_augmentation`` /
``get_image_data`` (``src/data_simbev.py:119-218``); the label path is ``get_binimg``
(``src/data_simbev.py:220-246``). The pixel arithmetic lives in a third-party dependency absent
from /root/reference: Pillow (12.2.0 in this image, ``requirements.txt`` pins none), whose published
C algorithms are restated here in numpy:

* ``Image.resize(size)`` -- default filter BICUBIC (a = -0.5, support 2), separable two-pass
  resample (``libImaging/Resample.c``: ``precompute_coeffs`` in double, coefficients normalised
  to 22-bit fixed point -- ``PRECISION_BITS = 32 - 8 - 2`` -- rounded half away from zero,
  int32 accumulation starting at ``1 << 21``, clip to [0, 255] after ``>> 22``); horizontal pass
  first, over the rows the vertical pass needs, then the vertical pass;
* ``Image.crop(box)`` -- integer box, pixels outside the source are 0;
* ``Image.transpose(FLIP_LEFT_RIGHT)``;
* ``Image.rotate(angle)`` -- NEAREST, expand=False, centre (w/2, h/2), fill 0: the inverse affine
  matrix of ``Image.rotate`` (Python double arithmetic, ``round(.., 15)``), then
  ``ImagingTransformAffine``'s 16.16 fixed-point nearest-neighbour walk (``libImaging/Geometry.c``:
  ``a2 = FIX(a[2] + a[1]*0.5 + a[0]*0.5)``, ``xin = xx >> 16``); angle % 360 == 0 is a copy.
* ``normalize_img`` -- ``ToTensor`` (uint8 / 255 in fp32) then ``Normalize(mean, std)``
  (``(x - mean) / std`` in fp32), torchvision's published behaviour.

Pinned by: Pillow itself (tests/test_simbev.py compares every function here with PIL on random
images) and by fixtures produced from the reference's own ``img_transform`` / ``get_binimg``
(tests/golden/make_golden_r2.py).
"""
from __future__ import annotations

import math
from typing import Sequence, Tuple

import numpy as np

PRECISION_BITS = 32 - 8 - 2
MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)
STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)


# ----------------------------------------------------------------------------- resize (Resample.c)
def _bicubic(x: float) -> float:
    a = -0.5
    if x < 0.0:
        x = -x
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def resample_coeffs(in_size: int, out_size: int, support_base: float = 2.0):
    """(bounds (out, 2) int: xmin, count; coeffs (out, ksize) int32) of one resample pass."""
    scale = float(in_size) / out_size
    filterscale = max(scale, 1.0)
    support = support_base * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), dtype=np.int64)
    kk = np.zeros((out_size, ksize), dtype=np.float64)
    for xx in range(out_size):
        center = 0.0 + (xx + 0.5) * scale
        ww = 0.0
        ss = 1.0 / filterscale
        xmin = int(center - support + 0.5)
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        for x in range(xmax):
            w = _bicubic((x + xmin - center + 0.5) * ss)
            kk[xx, x] = w
            ww += w
        for x in range(xmax):
            if ww != 0.0:
                kk[xx, x] /= ww
        bounds[xx] = (xmin, xmax)
    fixed = np.where(kk < 0, np.trunc(-0.5 + kk * (1 << PRECISION_BITS)),
                     np.trunc(0.5 + kk * (1 << PRECISION_BITS))).astype(np.int64)
    return bounds, fixed


def _clip8(acc: np.ndarray) -> np.ndarray:
    return np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)


def _pass(img: np.ndarray, bounds, coeffs, axis: int) -> np.ndarray:
    """One pass over `axis` (1 = horizontal / x, 0 = vertical / y) of an (H, W, C) uint8 image."""
    out_n = bounds.shape[0]
    src = img.astype(np.int64)
    shape = list(img.shape)
    shape[axis] = out_n
    acc = np.full(shape, 1 << (PRECISION_BITS - 1), dtype=np.int64)
    for o in range(out_n):
        xmin, cnt = bounds[o]
        for k in range(cnt):
            if axis == 1:
                acc[:, o] += src[:, xmin + k] * coeffs[o, k]
            else:
                acc[o] += src[xmin + k] * coeffs[o, k]
    return _clip8(acc)


def resize(img: np.ndarray, size: Tuple[int, int]) -> np.ndarray:
    """``Image.resize((W, H))`` with the default BICUBIC filter, (H, W, 3) uint8 -> (H', W', 3)."""
    W2, H2 = size
    H, W = img.shape[:2]
    if (W2, H2) == (W, H):
        return img.copy()
    need_h = W2 != W
    need_v = H2 != H
    bh, ch = resample_coeffs(W, W2)
    bv, cv = resample_coeffs(H, H2)
    out = img
    if need_h:
        y0 = int(bv[0, 0])
        y1 = int(bv[-1, 0] + bv[-1, 1])
        out = _pass(img[y0:y1], bh, ch, axis=1)
        bv = bv.copy()
        bv[:, 0] -= y0
    if need_v:
        out = _pass(out, bv, cv, axis=0)
    return out


# ----------------------------------------------------------------------------- crop / flip / rotate
def crop(img: np.ndarray, box: Sequence[int]) -> np.ndarray:
    x0, y0, x1, y1 = (int(round(v)) for v in box)
    H, W = img.shape[:2]
    out = np.zeros((y1 - y0, x1 - x0) + img.shape[2:], dtype=img.dtype)
    sx0, sy0, sx1, sy1 = max(x0, 0), max(y0, 0), min(x1, W), min(y1, H)
    if sx1 > sx0 and sy1 > sy0:
        out[sy0 - y0:sy1 - y0, sx0 - x0:sx1 - x0] = img[sy0:sy1, sx0:sx1]
    return out


def flip_lr(img: np.ndarray) -> np.ndarray:
    return img[:, ::-1].copy()


def rotate_matrix(angle: float, w: int, h: int):
    """The inverse affine matrix Image.rotate builds (Python doubles, as Pillow computes it)."""
    center = (w / 2, h / 2)
    a = -math.radians(angle)
    m = [round(math.cos(a), 15), round(math.sin(a), 15), 0.0, round(-math.sin(a), 15), round(math.cos(a), 15), 0.0]
    tx, ty = -center[0], -center[1]
    m[2], m[5] = m[0] * tx + m[1] * ty + m[2], m[3] * tx + m[4] * ty + m[5]
    m[2] += center[0]
    m[5] += center[1]
    return m


def affine_fixed(m) -> Tuple[int, int, int, int, int, int]:
    """16.16 fixed-point coefficients of ImagingTransformAffine's nearest path: (a0, a1, a2, a3, a4, a5)."""
    fix = lambda v: int(math.floor(v * 65536.0 + 0.5))  # noqa: E731
    return (fix(m[0]), fix(m[1]), fix(m[2] + m[1] * 0.5 + m[0] * 0.5), fix(m[3]), fix(m[4]),
            fix(m[5] + m[4] * 0.5 + m[3] * 0.5))


def rotate(img: np.ndarray, angle: float) -> np.ndarray:
    """``Image.rotate(angle)`` (NEAREST, expand=False, fill 0)."""
    angle = angle % 360.0
    if angle == 0:
        return img.copy()
    H, W = img.shape[:2]
    if angle == 180:
        return img[::-1, ::-1].copy()
    if angle in (90, 270) and W == H:
        return np.rot90(img, 1 if angle == 90 else 3).copy()
    a0, a1, a2, a3, a4, a5 = affine_fixed(rotate_matrix(angle, W, H))
    ys, xs = np.meshgrid(np.arange(H, dtype=np.int64), np.arange(W, dtype=np.int64), indexing="ij")
    # the incremental int32 sums of the C loop: xx = a2 + y*a1 + x*a0 (two's complement)
    xx = (a2 + ys * a1 + xs * a0).astype(np.int64)
    yy = (a5 + ys * a4 + xs * a3).astype(np.int64)
    xx = ((xx + 2 ** 31) % 2 ** 32) - 2 ** 31
    yy = ((yy + 2 ** 31) % 2 ** 32) - 2 ** 31
    xin, yin = xx >> 16, yy >> 16
    ok = (xin >= 0) & (xin < W) & (yin >= 0) & (yin < H)
    out = np.zeros_like(img)
    out[ok] = img[yin[ok], xin[ok]]
    return out


# ----------------------------------------------------------------------------- reference composition
def img_transform(img: np.ndarray, resize_dims, crop_box, flip: bool, rotate_deg: float) -> np.ndarray:
    """The image half of ``img_transform`` (src/tools.py:120-128): resize, crop, flip, rotate."""
    out = resize(img, tuple(resize_dims))
    out = crop(out, crop_box)
    if flip:
        out = flip_lr(out)
    return rotate(out, rotate_deg)


def normalize_img(img: np.ndarray) -> np.ndarray:
    """``normalize_img`` (src/tools.py:167-171): ToTensor + Normalize, (H, W, 3) uint8 -> (3, H, W) fp32."""
    x = img.astype(np.float32).transpose(2, 0, 1) / np.float32(255)
    return ((x - MEAN[:, None, None]) / STD[:, None, None]).astype(np.float32)


def vehicle_mask(bev: np.ndarray) -> np.ndarray:
    """``get_binimg`` (src/data_simbev.py:236-244): classes 1-3 merged, flipped up-down, (1, X, Y) fp32."""
    m = ((bev[1] > 0) | (bev[2] > 0) | (bev[3] > 0)).astype(np.float32)
    return np.flipud(m).copy()[None]
