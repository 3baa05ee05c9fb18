"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Runs only in the build container, where the reference is mounted at
/root/reference (read-only; never shipped). It imports the reference's own
``src.models`` / ``src.tools`` (SURVEY.md §8c recipe): third-party modules the
hot path does not use (torchvision, efficientnet_pytorch, pyquaternion,
nuscenes) are replaced by inert stubs, ``Tensor.cuda`` is made the identity
because ``get_geometry`` hard-codes ``.cuda()`` (``src/models.py:180,186``),
and no bytecode is written into the mount.

What it stores (data only -- inputs and the reference's outputs):
  geom_small.npz   G-geom  : rig + reference get_geometry at B=2, 64x176 (fH x fW = 4 x 11),
                             plain and with rotation/flip augmentation
  pool_small.npz   G-pool  : reference voxel_pooling (QuickCumsum and cumsum_trick) on a
                             50x50 grid, the lifted input, and the fp64 segment sum
  grad_small.npz   G-grad  : reference autograd d(loss)/d(depthnet_out) through lift + splat
                             for a seeded upstream grad, both cumsum modes
  lift_small.npz   G-lift  : reference CamEncode.get_depth_feat tail for a seeded 1x1 conv
  facts.json       known-answer facts + SHA-256 digests of full-size voxel ids (configs 2, 3, 5)

Usage:  PYTHONDONTWRITEBYTECODE=1 python -B tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import types

sys.dont_write_bytecode = True

import numpy as np  # noqa: E402
import torch  # noqa: E402
from torch import nn  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"


def _install_stubs():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    class _Transform:
        def __init__(self, *a, **k):
            pass

        def __call__(self, x):
            return x

    tv = mod("torchvision")
    tv.transforms = mod("torchvision.transforms", Normalize=_Transform, Compose=_Transform,
                        ToTensor=_Transform, ToPILImage=_Transform)
    tv.models = mod("torchvision.models")

    def _no_resnet(*a, **k):
        raise RuntimeError("torchvision stub: resnet18 not available in the golden generator")

    tv.models.resnet = mod("torchvision.models.resnet", resnet18=_no_resnet)

    class _NoEff:
        @staticmethod
        def from_pretrained(*a, **k):
            raise RuntimeError("efficientnet stub: network weights are never fetched")

    mod("efficientnet_pytorch", EfficientNet=_NoEff)
    mod("pyquaternion", Quaternion=object)
    mod("nuscenes")
    mod("nuscenes.utils")
    mod("nuscenes.utils.data_classes", LidarPointCloud=object)
    mod("nuscenes.utils.geometry_utils", transform_matrix=lambda *a, **k: None)
    mod("nuscenes.map_expansion")
    mod("nuscenes.map_expansion.map_api", NuScenesMap=object)


def _import_reference():
    _install_stubs()
    torch.Tensor.cuda = lambda self, *a, **k: self
    sys.path.insert(0, REF)
    from src import models as ref_models  # noqa: E402
    from src import tools as ref_tools  # noqa: E402
    return ref_models, ref_tools


def _ref_module(ref_models, ref_tools, grid_conf, data_aug_conf, use_quickcumsum=True):
    """LiftSplatShoot without its conv stacks (SURVEY.md §8c recipe, step 3)."""
    m = ref_models.LiftSplatShoot.__new__(ref_models.LiftSplatShoot)
    nn.Module.__init__(m)
    m.grid_conf = grid_conf
    m.data_aug_conf = data_aug_conf
    dx, bx, nx = ref_tools.gen_dx_bx(grid_conf["xbound"], grid_conf["ybound"], grid_conf["zbound"])
    m.dx = nn.Parameter(dx, requires_grad=False)
    m.bx = nn.Parameter(bx, requires_grad=False)
    m.nx = nn.Parameter(nx, requires_grad=False)
    m.downsample = 16
    m.camC = 64
    m.frustum = m.create_frustum()
    m.D = m.frustum.shape[0]
    m.use_quickcumsum = use_quickcumsum
    return m


def _ref_camencode(ref_models, D, C, seed):
    ce = ref_models.CamEncode.__new__(ref_models.CamEncode)
    nn.Module.__init__(ce)
    ce.D, ce.C = D, C
    torch.manual_seed(seed)
    ce.depthnet = nn.Conv2d(512, D + C, kernel_size=1, padding=0)
    ce.dropout = nn.Dropout(0.2)
    ce.get_eff_depth = lambda x: x
    ce.eval()
    return ce


def _sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    sys.path.insert(0, REPO)
    import lss_carla_amd.synthetic as syn  # noqa: E402

    ref_models, ref_tools = _import_reference()

    # ---------------------------------------------------------------- G-geom
    small_dim = (64, 176)
    gc = syn.grid_conf()
    dac = syn.data_aug_conf(small_dim)
    m = _ref_module(ref_models, ref_tools, gc, dac)
    out = {"frustum": m.frustum.detach().numpy()}
    for tag, aug in (("plain", False), ("aug", True)):
        rig = syn.make_rig(2, 6, small_dim, seed=3, aug=aug)
        with torch.no_grad():
            geom = m.get_geometry(rig["rots"], rig["trans"], rig["intrins"], rig["post_rots"], rig["post_trans"])
        for k, v in rig.items():
            out[f"{tag}_{k}"] = v.numpy()
        out[f"{tag}_geom"] = geom.numpy()
    np.savez_compressed(os.path.join(HERE, "geom_small.npz"), **out)

    # ---------------------------------------------------------------- G-pool / G-grad
    gc_small = syn.grid_conf(xy=(-12.5, 12.5, 0.5))
    D, C = 41, 64
    B, N = 2, 6
    fH, fW = small_dim[0] // 16, small_dim[1] // 16
    rig = syn.make_rig(B, N, small_dim, seed=5)
    dn = syn.make_depthnet_out(B, N, D, fH, fW, C, seed=0)
    pool = {"depthnet_out": dn.numpy()}
    for k, v in rig.items():
        pool[k] = v.numpy()
    grad = {}
    torch.manual_seed(1)
    X = Y = 50
    g_up = torch.randn(B, C, X, Y)
    grad["dbev"] = g_up.numpy()
    for mode, quick in (("quick", True), ("autograd", False)):
        m = _ref_module(ref_models, ref_tools, gc_small, dac, use_quickcumsum=quick)
        geom = m.get_geometry(rig["rots"], rig["trans"], rig["intrins"], rig["post_rots"], rig["post_trans"])
        dn_req = dn.clone().requires_grad_(True)
        depth = dn_req[:, :D].softmax(dim=1)                          # CamEncode.get_depth_feat tail
        new_x = depth.unsqueeze(1) * dn_req[:, D:D + C].unsqueeze(2)
        x = new_x.view(B, N, C, D, fH, fW).permute(0, 1, 3, 4, 5, 2)  # get_cam_feats layout
        bev = m.voxel_pooling(geom, x)
        pool[f"bev_{mode}"] = bev.detach().numpy()
        (bev * g_up).sum().backward()
        grad[f"d_depthnet_out_{mode}"] = dn_req.grad.numpy()
        if mode == "quick":
            pool["geom"] = geom.detach().numpy()
            pool["x_lifted"] = x.detach().contiguous().numpy()
    # fp64 segment sum of the same lifted input (tolerance anchor)
    xl = pool["x_lifted"].astype(np.float64).reshape(-1, C)
    gm = pool["geom"].reshape(-1, 3)
    dxv, bxv, nxv = [t.numpy() for t in ref_tools.gen_dx_bx(gc_small["xbound"], gc_small["ybound"], gc_small["zbound"])]
    q = ((gm - (bxv - dxv / 2.0).astype(np.float32)) / dxv).astype(np.float32)
    ids = np.trunc(q).astype(np.int64)
    bix = np.repeat(np.arange(B), ids.shape[0] // B)
    kept = (ids >= 0).all(1) & (ids < nxv).all(1)
    acc = np.zeros((B, 1, X, Y, C))
    np.add.at(acc, (bix[kept], ids[kept, 2], ids[kept, 0], ids[kept, 1]), xl[kept])
    pool["bev_fp64"] = acc.transpose(0, 1, 4, 2, 3).reshape(B, C, X, Y)
    pool["grid"] = np.array(gc_small["xbound"] + gc_small["zbound"] + gc_small["dbound"], dtype=np.float64)
    pool["x_lifted_sha256"] = np.array(_sha(pool.pop("x_lifted")))
    np.savez_compressed(os.path.join(HERE, "pool_small.npz"), **pool)
    np.savez_compressed(os.path.join(HERE, "grad_small.npz"), **grad)

    # ---------------------------------------------------------------- G-lift
    ce = _ref_camencode(ref_models, D, C, seed=7)
    torch.manual_seed(8)
    feat = torch.randn(1, 512, 4, 11)
    with torch.no_grad():
        depth, new_x = ce.get_depth_feat(feat)
    np.savez_compressed(os.path.join(HERE, "lift_small.npz"), feat=feat.numpy(),
                        weight=ce.depthnet.weight.detach().numpy(), bias=ce.depthnet.bias.detach().numpy(),
                        depth=depth.numpy(), new_x=new_x.numpy())

    # ---------------------------------------------------------------- facts (full sizes)
    facts = {"generator": "tests/golden/make_golden.py", "reference": "shdragron/LSS-Carla @ 2025-11-21"}
    for name in ("c1", "c2", "c3", "c5"):
        cfg, gcf, dacf = syn.config_confs(name)
        m = _ref_module(ref_models, ref_tools, gcf, dacf)
        rig = syn.make_rig(cfg["B"], cfg["N"], cfg["final_dim"], seed=0)
        with torch.no_grad():
            geom = m.get_geometry(rig["rots"], rig["trans"], rig["intrins"], rig["post_rots"], rig["post_trans"])
            gf = ((geom - (m.bx - m.dx / 2.)) / m.dx).long().view(-1, 3)
        Bc = cfg["B"]
        nprime = gf.shape[0]
        bix = torch.cat([torch.full([nprime // Bc, 1], ix, dtype=torch.long) for ix in range(Bc)])
        gf4 = torch.cat((gf, bix), 1)
        kept = ((gf4[:, 0] >= 0) & (gf4[:, 0] < m.nx[0]) & (gf4[:, 1] >= 0) & (gf4[:, 1] < m.nx[1])
                & (gf4[:, 2] >= 0) & (gf4[:, 2] < m.nx[2]))
        gk = gf4[kept]
        ranks = gk[:, 0] * (m.nx[1] * m.nx[2] * Bc) + gk[:, 1] * (m.nx[2] * Bc) + gk[:, 2] * Bc + gk[:, 3]
        _, counts = torch.unique(ranks, return_counts=True)
        qf = ((geom - (m.bx - m.dx / 2.)) / m.dx).view(-1, 3)
        facts[name] = {
            "B": Bc, "N": cfg["N"], "final_dim": list(cfg["final_dim"]), "grid_conf": gcf,
            "nprime": int(nprime), "kept": int(kept.sum()), "occupied": int(counts.numel()),
            "max_per_voxel": int(counts.max()),
            "trunc_ne_floor": int((qf.trunc() != qf.floor()).any(1).sum()),
            "sha256_ids_int32": _sha(gf.numpy().astype(np.int32)),
            "sha256_kept_u8": _sha(kept.numpy().astype(np.uint8)),
            "sha256_geom_f32": _sha(geom.numpy().astype(np.float32)),
        }
    with open(os.path.join(HERE, "facts.json"), "w") as f:
        json.dump(facts, f, indent=1, sort_keys=True)
    print(json.dumps({k: {kk: vv for kk, vv in v.items() if not kk.startswith("sha")} if isinstance(v, dict) else v
                      for k, v in facts.items()}, indent=1))


if __name__ == "__main__":
    main()
