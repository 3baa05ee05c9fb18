"""SimBEV input path with the pixel work on the MI355X.

Drop-in for ``src/data_simbev.py`` of shdragron/LSS-Carla: ``SimBEVDataset`` / ``SegmentationData`` /
``VizData`` / ``compile_data(version, dataroot, data_aug_conf, grid_conf, bsz, nworkers, parser_name)``
with the same directory layout, split, augmentation draws and returned 7-tuple
``(imgs, rots, trans, intrins, post_rots, post_trans, binimgs)``.

Where the work runs:
  host (DataLoader workers)  meta.json parsing, JPEG decode (PIL), the augmentation draws
                             (``sample_augmentation``, np.random, src/data_simbev.py:119-145) and the
                             post-homography arithmetic (torch, src/tools.py:130-142), the BEV npz read
  device (main process)      ``lss_simbev_images``: Image.resize (bicubic) -> crop -> flip -> rotate
                             -> ToTensor -> Normalize per camera, bit for bit with Pillow / torchvision;
                             ``lss_simbev_vehicle_mask``: classes 1-3 merged + np.flipud
So a training step at hundreds of frames/s is not bound by PIL's per-camera resampling on the CPU:
the workers only decode. The loader yields device tensors; the reference's ``.to(device)`` calls in
train_simbev.py become no-ops.
"""
from __future__ import annotations

import ctypes
import json
import math
import os
from functools import lru_cache
from pathlib import Path
from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch

from . import _lib

CAMERA_ORDER = ["front_left", "front", "front_right", "back_left", "back", "back_right"]  # src/data_simbev.py:17-20


# ----------------------------------------------------------------------------- augmentation arithmetic (host)
def get_rot(h):
    """src/tools.py:113-117."""
    return torch.Tensor([[np.cos(h), np.sin(h)], [-np.sin(h), np.cos(h)]])


def draw_augmentation(conf: dict, train: bool):
    """One sample's augmentation (src/data_simbev.py:119-145): (scale, (W', H') after scaling, crop box
    (left, top, right, bottom) of final_dim, flip, rotation in degrees).

    The crop keeps the image's bottom band: its top edge sits `bottom` of the scaled height above the
    bottom minus the final height; horizontally the window starts `left` pixels in. Training draws,
    in order, from np.random: scale ~ U(resize_lim), bottom ~ U(bot_pct_lim), left ~ U(0, slack), a
    flip coin only when rand_flip is set, rotation ~ U(rot_lim). Validation: the scale that fits the
    final width, the mean of bot_pct_lim, the window centred, no flip or rotation."""
    src_h, src_w = conf["H"], conf["W"]
    out_h, out_w = conf["final_dim"]
    rnd = np.random
    scale = rnd.uniform(*conf["resize_lim"]) if train else max(out_h / src_h, out_w / src_w)
    scaled = (int(src_w * scale), int(src_h * scale))
    slack = max(0, scaled[0] - out_w)
    bottom = rnd.uniform(*conf["bot_pct_lim"]) if train else np.mean(conf["bot_pct_lim"])
    top = int((1 - bottom) * scaled[1]) - out_h
    left = int(rnd.uniform(0, slack)) if train else int(slack / 2)
    flip = bool(train and conf["rand_flip"] and rnd.choice([0, 1]))
    rotate = rnd.uniform(*conf["rot_lim"]) if train else 0
    return scale, scaled, (left, top, left + out_w, top + out_h), flip, rotate


def post_homography(resize, crop, flip, rotate):
    """(post_rot (3, 3), post_tran (3,)) of one camera: img_transform's post-homography arithmetic
    (src/tools.py:130-142) then the 3x3 embedding of get_image_data (src/data_simbev.py:204-208),
    with the same torch fp32 ops in the same order."""
    post_rot = torch.eye(2)
    post_tran = torch.zeros(2)
    post_rot *= resize
    post_tran -= torch.Tensor(crop[:2])
    if flip:
        A = torch.Tensor([[-1, 0], [0, 1]])
        b = torch.Tensor([crop[2] - crop[0], 0])
        post_rot = A.matmul(post_rot)
        post_tran = A.matmul(post_tran) + b
    A = get_rot(rotate / 180 * np.pi)
    b = torch.Tensor([crop[2] - crop[0], crop[3] - crop[1]]) / 2
    b = A.matmul(-b) + b
    post_rot = A.matmul(post_rot)
    post_tran = A.matmul(post_tran) + b
    post_tran_3 = torch.zeros(3)
    post_rot_3 = torch.eye(3)
    post_tran_3[:2] = post_tran
    post_rot_3[:2, :2] = post_rot
    return post_rot_3, post_tran_3


def rotation_mode(angle: float, w: int, h: int) -> Tuple[int, Tuple[int, ...]]:
    """(rot_mode, 16.16 affine coefficients) for Image.rotate(angle) of a w x h image (NEAREST,
    expand=False): the fast paths of Image.rotate, else its inverse matrix (Python doubles, as
    Pillow computes it) in ImagingTransformAffine's fixed point."""
    angle = angle % 360.0
    if angle == 0:
        return 0, (0,) * 6
    if angle == 180:
        return 1, (0,) * 6
    if angle in (90, 270) and w == h:
        return (3 if angle == 90 else 4), (0,) * 6
    center = (w / 2, h / 2)
    a = -math.radians(angle)
    m = [round(math.cos(a), 15), round(math.sin(a), 15), 0.0, round(-math.sin(a), 15), round(math.cos(a), 15), 0.0]
    x, y = -center[0], -center[1]
    m[2], m[5] = m[0] * x + m[1] * y + m[2], m[3] * x + m[4] * y + m[5]
    m[2] += center[0]
    m[5] += center[1]
    fix = lambda v: int(math.floor(v * 65536.0 + 0.5))  # noqa: E731  (Geometry.c FIX)
    coeffs = (fix(m[0]), fix(m[1]), fix(m[2] + m[1] * 0.5 + m[0] * 0.5), fix(m[3]), fix(m[4]),
              fix(m[5] + m[4] * 0.5 + m[3] * 0.5))
    # check_fixed: the fixed-point walk is Pillow's path while every corner maps inside +-32768
    for cx, cy in ((0, 0), (w, h), (0, h), (w, 0)):
        if abs(m[0] * cx + m[1] * cy + m[2]) >= 32768.0 or abs(m[3] * cx + m[4] * cy + m[5]) >= 32768.0:
            raise NotImplementedError("rotation outside Pillow's fixed-point range (image > 32k pixels)")
    return 2, coeffs


@lru_cache(maxsize=64)
def resample_table(in_size: int, out_size: int) -> Tuple[int, np.ndarray]:
    """(ksize, int32 table) of one Image.resize pass (lss_resample_coeffs: Pillow's bicubic coefficients);
    ksize 0 = the pass is skipped (same size)."""
    if in_size == out_size:
        return 0, np.zeros(0, dtype=np.int32)
    lib = _lib.load()
    k = int(lib.lss_resample_ksize(in_size, out_size))
    tab = np.zeros(out_size * (2 + k), dtype=np.int32)
    _lib.check(lib.lss_resample_coeffs(in_size, out_size, ctypes.c_void_p(tab.ctypes.data)), "lss_resample_coeffs")
    return k, tab


_DEVICE_TABLES: Dict[Tuple[int, int, int], torch.Tensor] = {}


def _device_table(inn: int, outn: int, dev: torch.device) -> Tuple[int, torch.Tensor]:
    """(ksize, device int32 table) of one resize pass, uploaded once per (device, in, out) through
    pinned memory without blocking the host (the pinned block is not reused before the copy ran)."""
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), inn, outn)
    k, tab = resample_table(inn, outn)
    t = _DEVICE_TABLES.get(key)
    if t is None:
        host = torch.from_numpy(tab if tab.size else np.zeros(1, dtype=np.int32)).pin_memory()
        t = host.to(dev, non_blocking=True)
        _DEVICE_TABLES[key] = t
    return k, t


def _to_device_pinned(buf: bytes, dev: torch.device) -> torch.Tensor:
    """Host bytes -> a device uint8 tensor through a pinned staging block, non-blocking."""
    host = torch.empty(len(buf), dtype=torch.uint8, pin_memory=True)
    host.numpy()[:] = np.frombuffer(buf, dtype=np.uint8)
    return host.to(dev, non_blocking=True)


# ----------------------------------------------------------------------------- device kernels
def augment_images(imgs_u8: torch.Tensor, augs: Sequence[dict], final_dim: Sequence[int]) -> torch.Tensor:
    """(n, H, W, 3) uint8 device images + one aug dict per image (resize_dims, crop, flip, rotate) ->
    (n, 3, fH, fW) fp32 = normalize_img(img_transform(img)) (src/tools.py:120-128, 167-171)."""
    if not imgs_u8.is_cuda:
        raise RuntimeError("lss_carla_amd.simbev: images must be on the MI355X (no CPU fallback)")
    if imgs_u8.dtype != torch.uint8 or imgs_u8.dim() != 4 or imgs_u8.shape[-1] != 3:
        raise RuntimeError(f"expected (n, H, W, 3) uint8 images, got {imgs_u8.dtype} {tuple(imgs_u8.shape)}")
    n, H, W, _ = imgs_u8.shape
    if len(augs) != n:
        raise RuntimeError(f"{len(augs)} augmentation records for {n} images")
    fH, fW = int(final_dim[0]), int(final_dim[1])
    lib = _lib.load()
    dev = imgs_u8.device
    params = (_lib.ImgAug * n)()
    # the batch's resize tables: device-resident per (in, out) size, concatenated on the device (no
    # host round trip per batch; the first use of a size uploads it without blocking)
    tables: List[torch.Tensor] = []
    offsets: Dict[Tuple[int, int], Tuple[int, int]] = {}
    off = 0

    def table(inn, outn):
        nonlocal off
        key = (inn, outn)
        if key not in offsets:
            k, tab = _device_table(inn, outn, dev)
            offsets[key] = (off, k)
            if k:
                tables.append(tab)
                off += tab.numel()
        return offsets[key]

    for i, a in enumerate(augs):
        rs_w, rs_h = (int(v) for v in a["resize_dims"])
        crop = [int(round(v)) for v in a["crop"]]
        if crop[2] - crop[0] != fW or crop[3] - crop[1] != fH:
            raise RuntimeError(f"crop {crop} is not final_dim {final_dim}")
        p = params[i]
        p.src_h, p.src_w, p.rs_w, p.rs_h = H, W, rs_w, rs_h
        for j in range(4):
            p.crop[j] = crop[j]
        p.flip = 1 if a["flip"] else 0
        mode, co = rotation_mode(float(a["rotate"]), fW, fH)
        p.rot_mode = mode
        for j in range(6):
            p.affine[j] = co[j]
        p.h_off, p.h_ksize = table(W, rs_w)
        p.v_off, p.v_ksize = table(H, rs_h)
    tab_d = (tables[0] if len(tables) == 1 else torch.cat(tables)) if tables else \
        torch.zeros(1, device=dev, dtype=torch.int32)
    par_d = _to_device_pinned(bytes(params), dev)
    src = imgs_u8.contiguous()
    out = torch.empty(n, 3, fH, fW, device=dev, dtype=torch.float32)
    _lib.check(lib.lss_simbev_images(_lib.ptr(src), n, H, W, _lib.ptr(par_d), _lib.ptr(tab_d), fH, fW,
                                     _lib.ptr(out), _lib.stream_handle(dev)), "lss_simbev_images")
    return out


def vehicle_masks(bev_u8: torch.Tensor) -> torch.Tensor:
    """(n, C, X, Y) uint8 device BEV maps -> (n, 1, X, Y) fp32 binimgs (src/data_simbev.py:236-244)."""
    if not bev_u8.is_cuda:
        raise RuntimeError("lss_carla_amd.simbev: BEV maps must be on the MI355X (no CPU fallback)")
    if bev_u8.dtype == torch.bool:
        bev_u8 = bev_u8.view(torch.uint8)
    if bev_u8.dtype != torch.uint8:
        bev_u8 = (bev_u8 > 0).to(torch.uint8)
    n, C, X, Y = bev_u8.shape
    out = torch.empty(n, 1, X, Y, device=bev_u8.device, dtype=torch.float32)
    b = bev_u8.contiguous()
    _lib.check(_lib.load().lss_simbev_vehicle_mask(_lib.ptr(b), n, C, X, Y, _lib.ptr(out),
                                                   _lib.stream_handle(b.device)), "lss_simbev_vehicle_mask")
    return out


# ----------------------------------------------------------------------------- dataset (host side)
class SimBEVDataset(torch.utils.data.Dataset):
    """src/data_simbev.py:23-265: same layout (SimBEV_cvt_label/scene_*/yaw0pitch0/meta.json, 80/20
    scene split), same augmentation draws. ``__getitem__`` returns the raw sample (decoded uint8
    images + calibration + augmentation + uint8 BEV); ``compile_data``'s loader finishes it on the device."""

    def __init__(self, dataroot, is_train, data_aug_conf, grid_conf):
        self.dataroot = Path(dataroot)
        self.is_train = is_train
        self.data_aug_conf = data_aug_conf
        self.grid_conf = grid_conf
        self.samples = self._load_all_samples()
        from .tools import gen_dx_bx
        dx, bx, nx = gen_dx_bx(grid_conf["xbound"], grid_conf["ybound"], grid_conf["zbound"])
        self.dx, self.bx, self.nx = dx.numpy(), bx.numpy(), nx.numpy()
        print(self)

    def _load_all_samples(self):
        labels_dir = self.dataroot / "SimBEV_cvt_label"
        if not labels_dir.exists():
            raise FileNotFoundError(f"Labels directory not found: {labels_dir}")
        scene_dirs = sorted([d for d in labels_dir.iterdir() if d.is_dir() and d.name.startswith("scene_")])
        if not scene_dirs:
            raise FileNotFoundError(f"No scene directories found in {labels_dir}")
        train_split = int(0.8 * len(scene_dirs))
        selected = scene_dirs[:train_split] if self.is_train else scene_dirs[train_split:]
        out = []
        for scene_dir in selected:
            meta_path = scene_dir / "yaw0pitch0" / "meta.json"
            if not meta_path.exists():
                continue
            with open(meta_path) as f:
                for s in json.load(f):
                    s["scene_dir"] = scene_dir
                    s["meta_dir"] = meta_path.parent
                    out.append(s)
        if not out:
            raise FileNotFoundError(f"No samples found for {'train' if self.is_train else 'val'} split in {labels_dir}")
        return out

    def sample_augmentation(self):
        """(resize, resize_dims, crop box, flip, rotate) of one sample (src/data_simbev.py:119-145).

        Training draws from numpy's global generator in the reference's order -- scale, bottom-crop
        fraction, horizontal crop offset, the flip coin (only when rand_flip is on), rotation -- so a
        seeded run reproduces the reference loader's augmentations; validation uses the fixed
        fit-to-width scale, the mean bottom fraction and a centred window."""
        return draw_augmentation(self.data_aug_conf, self.is_train)

    def get_image_data(self, sample, cam_indices):
        """Decoded images and calibration (src/data_simbev.py:147-218 without the pixel work)."""
        from PIL import Image
        resize, resize_dims, crop, flip, rotate = self.sample_augmentation()
        imgs, rots, trans, intrins, post_rots, post_trans = [], [], [], [], [], []
        for cam_idx in cam_indices:
            img = Image.open(self.dataroot / sample["images"][cam_idx]).convert("RGB")
            imgs.append(torch.from_numpy(np.asarray(img, dtype=np.uint8).copy()))
            intrins.append(torch.Tensor(sample["intrinsics"][cam_idx]))
            extrin = np.array(sample["extrinsics"][cam_idx])
            rots.append(torch.Tensor(extrin[:3, :3]))
            trans.append(torch.Tensor(extrin[:3, 3]))
            pr, pt = post_homography(resize, crop, flip, rotate)
            post_rots.append(pr)
            post_trans.append(pt)
        aug = torch.tensor([resize_dims[0], resize_dims[1], crop[0], crop[1], crop[2], crop[3], int(flip)],
                           dtype=torch.int64)
        return (torch.stack(imgs), torch.stack(rots), torch.stack(trans), torch.stack(intrins),
                torch.stack(post_rots), torch.stack(post_trans), aug, torch.tensor(float(rotate), dtype=torch.float64))

    def get_bev_raw(self, sample):
        """The BEV npz's (n_classes, X, Y) map as uint8 (value > 0 kept), src/data_simbev.py:227-232."""
        bev = np.load(sample["meta_dir"] / sample["bev"])["bev"]
        return torch.from_numpy((bev > 0).astype(np.uint8) if bev.dtype != np.uint8 else bev.copy())

    def choose_cams(self):
        all_cams = list(range(len(CAMERA_ORDER)))
        if self.is_train and "Ncams" in self.data_aug_conf:
            Ncams = self.data_aug_conf["Ncams"]
            if Ncams < len(CAMERA_ORDER):
                return sorted(np.random.choice(all_cams, Ncams, replace=False).tolist())
        return all_cams

    def __len__(self):
        return len(self.samples)

    def __str__(self):
        return f"SimBEVDataset ({'train' if self.is_train else 'val'}): {len(self)} samples"


class VizData(SimBEVDataset):
    def __getitem__(self, index):
        sample = self.samples[index]
        raw = self.get_image_data(sample, self.choose_cams())
        return raw + (torch.empty(3, 0), self.get_bev_raw(sample))


class SegmentationData(SimBEVDataset):
    def __getitem__(self, index):
        sample = self.samples[index]
        raw = self.get_image_data(sample, self.choose_cams())
        return raw + (self.get_bev_raw(sample),)


def worker_rnd_init(x):
    np.random.seed(13 + x)  # src/data_simbev.py:310-312


def finish_batch(batch, final_dim, device):
    """A collated raw batch -> the reference's (imgs, rots, trans, intrins, post_rots, post_trans,
    [lidar,] binimgs) on `device`, the pixel work done by the HIP kernels."""
    imgs_u8, rots, trans, intrins, post_rots, post_trans, aug, rot = batch[:8]
    rest = batch[8:]
    B, N = imgs_u8.shape[:2]
    src = imgs_u8.reshape(B * N, *imgs_u8.shape[2:]).to(device, non_blocking=True)
    augs = []
    for b in range(B):
        a = aug[b].tolist()
        rec = {"resize_dims": (a[0], a[1]), "crop": tuple(a[2:6]), "flip": bool(a[6]), "rotate": float(rot[b])}
        augs.extend([rec] * N)
    imgs = augment_images(src, augs, final_dim).view(B, N, 3, int(final_dim[0]), int(final_dim[1]))
    out = [imgs] + [t.to(device, non_blocking=True) for t in (rots, trans, intrins, post_rots, post_trans)]
    # the host copies ride along: the model's host torch.inverse (src/models.py:180,186) reads them
    # instead of copying the device tensors back (ops.camera_inverses), so no batch syncs the host
    out[3]._lss_host, out[3]._lss_host_version = intrins, out[3]._version
    out[4]._lss_host, out[4]._lss_host_version = post_rots, out[4]._version
    for t in rest[:-1]:
        out.append(t)  # lidar placeholder (VizData)
    out.append(vehicle_masks(rest[-1].to(device, non_blocking=True)))
    return tuple(out)


class DeviceLoader:
    """Iterates a DataLoader of raw samples and yields finished device batches (finish_batch)."""

    def __init__(self, loader, final_dim, device):
        self.loader, self.final_dim, self.device = loader, final_dim, torch.device(device)
        self.dataset = loader.dataset
        self.batch_size = loader.batch_size

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        for batch in self.loader:
            yield finish_batch(batch, self.final_dim, self.device)


def compile_data(version, dataroot, data_aug_conf, grid_conf, bsz, nworkers, parser_name, device="cuda"):
    """src/data_simbev.py:315-354 with the same loaders' settings; returns DeviceLoaders."""
    parser = {"vizdata": VizData, "segmentationdata": SegmentationData}[parser_name]
    traindata = parser(dataroot, is_train=True, data_aug_conf=data_aug_conf, grid_conf=grid_conf)
    valdata = parser(dataroot, is_train=False, data_aug_conf=data_aug_conf, grid_conf=grid_conf)
    trainloader = torch.utils.data.DataLoader(traindata, batch_size=bsz, shuffle=True, num_workers=nworkers,
                                              drop_last=True, worker_init_fn=worker_rnd_init, pin_memory=True)
    valloader = torch.utils.data.DataLoader(valdata, batch_size=bsz, shuffle=False, num_workers=nworkers,
                                            pin_memory=True)
    fd = data_aug_conf["final_dim"]
    return DeviceLoader(trainloader, fd, device), DeviceLoader(valloader, fd, device)
