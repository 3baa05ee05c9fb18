"""Seeded SimBEV-shaped synthetic inputs.

The SimBEV dataset is not available offline, so every parity test and the
benchmark drive the hot path with a synthetic 6-camera rig built the same way
the reference's SimBEV loader builds real ones:

* intrinsics of a 224x480 pinhole camera with a 70 deg horizontal FOV
  (``train_simbev.py:29-30`` H/W defaults),
* camera yaws in ``CAMERA_ORDER`` (``src/data_simbev.py:17-20``),
* the validation-mode resize/crop of ``sample_augmentation``
  (``src/data_simbev.py:136-141``) turned into ``post_rots``/``post_trans``
  exactly as ``img_transform`` does (``src/tools.py:120-144``),
* optionally a training-mode rotation + flip, so that ``post_rots`` is not
  diagonal (exercises the general 3x3 inverse path).

All tensors are float32 on CPU; callers move them to the device.
"""
from __future__ import annotations

import math
from typing import Dict, Sequence, Tuple

import torch

# Yaw (degrees) of front_left, front, front_right, back_left, back, back_right.
CAMERA_YAWS_DEG = (55.0, 0.0, -55.0, 110.0, 180.0, -110.0)
# Camera frame (x right, y down, z forward) -> ego frame (x fwd, y left, z up).
_CAM_TO_EGO_BASE = ((0.0, 0.0, 1.0), (-1.0, 0.0, 0.0), (0.0, -1.0, 0.0))

IMG_H, IMG_W = 224, 480
HFOV_DEG = 70.0

# The five BASELINE.json configurations (SURVEY.md §8d "Per config").
CONFIGS: Dict[str, dict] = {
    "c1": dict(B=1, N=1, final_dim=(128, 352), dbound=(4.0, 45.0, 1.0), xy=(-50.0, 50.0, 0.5)),
    "c2": dict(B=4, N=6, final_dim=(128, 352), dbound=(4.0, 45.0, 1.0), xy=(-50.0, 50.0, 0.5)),
    "c3": dict(B=8, N=6, final_dim=(128, 352), dbound=(4.0, 45.0, 1.0), xy=(-50.0, 50.0, 0.5)),
    "c4": dict(B=8, N=6, final_dim=(128, 352), dbound=(4.0, 45.0, 1.0), xy=(-50.0, 50.0, 0.5)),
    "c5": dict(B=4, N=6, final_dim=(256, 704), dbound=(4.0, 64.0, 1.0), xy=(-50.0, 50.0, 0.25)),
}


def grid_conf(xy=(-50.0, 50.0, 0.5), z=(-10.0, 10.0, 20.0), dbound=(4.0, 45.0, 1.0)) -> dict:
    """grid_conf dict with the schema of ``train_simbev.py:104-109``."""
    return {"xbound": list(xy), "ybound": list(xy), "zbound": list(z), "dbound": list(dbound)}


def data_aug_conf(final_dim=(128, 352), ncams=6) -> dict:
    """data_aug_conf dict with the schema of ``train_simbev.py:111-120``."""
    return {
        "resize_lim": (1.0, 1.0), "final_dim": tuple(final_dim), "rot_lim": (0.0, 0.0),
        "H": IMG_H, "W": IMG_W, "rand_flip": False, "bot_pct_lim": (0.0, 0.0), "Ncams": ncams,
    }


def config_confs(name: str) -> Tuple[dict, dict, dict]:
    c = CONFIGS[name]
    return c, grid_conf(xy=c["xy"], dbound=c["dbound"]), data_aug_conf(c["final_dim"], c["N"])


def _rot2(theta: float) -> torch.Tensor:
    c, s = math.cos(theta), math.sin(theta)
    return torch.tensor([[c, s], [-s, c]], dtype=torch.float32)


def _post_homography(final_dim, flip: bool, rotate_deg: float):
    """Resize/crop(/flip/rotate) -> 3x3 post_rot and 3-vector post_tran.

    Follows the arithmetic of ``img_transform`` (``src/tools.py:131-144``)
    with the val-mode crop of ``src/data_simbev.py:136-141``.
    """
    fH, fW = final_dim
    resize = max(fH / IMG_H, fW / IMG_W)
    newW, newH = int(IMG_W * resize), int(IMG_H * resize)
    crop_h = int(newH) - fH
    crop_w = int(max(0, newW - fW) / 2)
    crop = (crop_w, crop_h, crop_w + fW, crop_h + fH)
    post_rot = torch.eye(2) * resize
    post_tran = torch.zeros(2) - torch.tensor(crop[:2], dtype=torch.float32)
    if flip:
        A = torch.tensor([[-1.0, 0.0], [0.0, 1.0]])
        b = torch.tensor([float(crop[2] - crop[0]), 0.0])
        post_rot = A.matmul(post_rot)
        post_tran = A.matmul(post_tran) + b
    A = _rot2(rotate_deg / 180.0 * math.pi)
    b = torch.tensor([float(crop[2] - crop[0]), float(crop[3] - crop[1])]) / 2
    b = A.matmul(-b) + b
    post_rot = A.matmul(post_rot)
    post_tran = A.matmul(post_tran) + b
    R3 = torch.eye(3)
    R3[:2, :2] = post_rot
    t3 = torch.zeros(3)
    t3[:2] = post_tran
    return R3, t3


def make_rig(B: int, N: int = 6, final_dim: Sequence[int] = (128, 352), seed: int = 0,
             aug: bool = False) -> Dict[str, torch.Tensor]:
    """Calibration tensors of the §8d rig: rots/intrins/post_rots (B,N,3,3), trans/post_trans (B,N,3)."""
    assert 1 <= N <= len(CAMERA_YAWS_DEG)
    gen = torch.Generator().manual_seed(seed)
    fx = IMG_W / (2.0 * math.tan(math.radians(HFOV_DEG / 2.0)))
    K = torch.tensor([[fx, 0.0, IMG_W / 2.0], [0.0, fx, IMG_H / 2.0], [0.0, 0.0, 1.0]], dtype=torch.float64)
    base = torch.tensor(_CAM_TO_EGO_BASE, dtype=torch.float64)
    rots, trans_mean = [], []
    for yaw in CAMERA_YAWS_DEG[:N]:
        a = math.radians(yaw)
        Rz = torch.tensor([[math.cos(a), -math.sin(a), 0.0], [math.sin(a), math.cos(a), 0.0], [0.0, 0.0, 1.0]],
                          dtype=torch.float64)
        rots.append(Rz @ base)
        trans_mean.append([1.5 * math.cos(a), 0.5 * math.sin(a), 1.6])
    rots = torch.stack(rots).to(torch.float32).unsqueeze(0).expand(B, N, 3, 3).contiguous()
    trans = (torch.tensor(trans_mean, dtype=torch.float32).unsqueeze(0)
             + 0.05 * torch.randn((B, N, 3), generator=gen)).contiguous()
    intrins = K.to(torch.float32).expand(B, N, 3, 3).contiguous()
    post_rots = torch.empty(B, N, 3, 3)
    post_trans = torch.empty(B, N, 3)
    for b in range(B):
        if aug:
            flip = bool(torch.randint(0, 2, (1,), generator=gen).item())
            rot = float(torch.empty(1).uniform_(-5.4, 5.4, generator=gen).item())
        else:
            flip, rot = False, 0.0
        R3, t3 = _post_homography(final_dim, flip, rot)
        post_rots[b] = R3
        post_trans[b] = t3
    return {"rots": rots, "trans": trans, "intrins": intrins, "post_rots": post_rots, "post_trans": post_trans}


def make_depthnet_out(B: int, N: int, D: int, fH: int, fW: int, C: int = 64, seed: int = 0,
                      dtype=torch.float32) -> torch.Tensor:
    """Depthnet output (B*N, D+C, fH, fW): N(0,1) depth logits then N(0,1) context (§8d order)."""
    torch.manual_seed(seed)
    logits = torch.randn(B * N, D, fH, fW)
    ctx = torch.randn(B * N, C, fH, fW)
    return torch.cat([logits, ctx], 1).to(dtype).contiguous()


def make_images(B: int, N: int, final_dim: Sequence[int], seed: int = 0) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed + 1)
    return torch.randn((B, N, 3, final_dim[0], final_dim[1]), generator=g)


def make_labels(B: int, X: int, Y: int, seed: int = 0) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed + 2)
    return (torch.rand((B, 1, X, Y), generator=g) < 0.03).to(torch.float32)
