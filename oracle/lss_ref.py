"""CPU oracle for the Lift-Splat hot path -- TEST INFRASTRUCTURE ONLY.

This module is the *checker*, never the product: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it. The product path (``lss_carla_amd``) never routes through it and fails
loudly when its HIP library is missing.

It restates, on the CPU, the semantics of the reference
(shdragron/LSS-Carla @ 2025-11-21, pure PyTorch) for every row of SURVEY.md
§8a. Each function cites the reference file:line it follows.

Numerics:

* geometry is fp32 with the reference's op order; both 3x3 mat-vecs are
  sequential ``acc = acc + M[i,k]*v[k]`` sums with no FMA, which is what the
  CPU ``torch.matmul`` of ``src/models.py:180,187`` computes for 3x3 operands;
  the inverses are host ``torch.inverse`` results (``src/models.py:180,186``);
* quantisation truncates toward zero (``.long()``, ``src/models.py:212``);
* the reference's cumsum trick accumulates the prefix sum in double and
  stores fp32 (CPU ``torch.cumsum``), then differences in fp32.

Parity pin: ``tests/golden/*`` hold vectors produced by importing the
reference itself in the build container (``tests/golden/make_golden.py``);
``tests/test_oracle_golden.py`` checks this module against them.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F


# ----------------------------------------------------------------------------- a1
def gen_dx_bx(xbound, ybound, zbound):
    """Cell size, first-cell centre and cell count per axis (``src/tools.py:174-179``).

    Returns dx, bx as float32 (python doubles rounded once, like ``torch.Tensor``)
    and nx as int64 (python ``int`` of the double quotient, like ``torch.LongTensor``).
    """
    rows = (xbound, ybound, zbound)
    dx = np.array([r[2] for r in rows], dtype=np.float32)
    bx = np.array([r[0] + r[2] / 2.0 for r in rows], dtype=np.float32)
    nx = np.array([int((r[1] - r[0]) / r[2]) for r in rows], dtype=np.int64)
    return dx, bx, nx


# ----------------------------------------------------------------------------- a3
def create_frustum(final_dim, dbound, downsample: int = 16) -> torch.Tensor:
    """(D, fH, fW, 3) grid of (u, v, depth) (``src/models.py:157-168``).

    Uses torch's own ``arange``/``linspace`` so the fp32 rounding of the grid is
    the reference's.
    """
    ogfH, ogfW = final_dim
    fH, fW = ogfH // downsample, ogfW // downsample
    ds = torch.arange(*dbound, dtype=torch.float).view(-1, 1, 1).expand(-1, fH, fW)
    D = ds.shape[0]
    xs = torch.linspace(0, ogfW - 1, fW, dtype=torch.float).view(1, 1, fW).expand(D, fH, fW)
    ys = torch.linspace(0, ogfH - 1, fH, dtype=torch.float).view(1, fH, 1).expand(D, fH, fW)
    return torch.stack((xs, ys, ds), -1).contiguous()


# ----------------------------------------------------------------------------- a4
def _matvec_seq(M: np.ndarray, v: np.ndarray) -> np.ndarray:
    """out[..., i] = ((0 + M[i,0] v0) + M[i,1] v1) + M[i,2] v2, every op rounded to fp32."""
    out = np.empty(np.broadcast_shapes(M.shape[:-1], v.shape), dtype=np.float32)
    for i in range(3):
        acc = M[..., i, 0] * v[..., 0]
        acc = acc + M[..., i, 1] * v[..., 1]
        acc = acc + M[..., i, 2] * v[..., 2]
        out[..., i] = acc
    return out


def _matmul_seq(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    out = np.empty(A.shape, dtype=np.float32)
    for j in range(3):
        out[..., :, j] = _matvec_seq(A, B[..., :, j])
    return out


def camera_matrices(rots, intrins, post_rots):
    """Host inverses and ``combine = rots @ inv(intrins)`` (``src/models.py:180,186``)."""
    pinv = torch.inverse(post_rots.detach().cpu().float()).numpy()
    kinv = torch.inverse(intrins.detach().cpu().float()).numpy()
    combine = _matmul_seq(rots.detach().cpu().float().numpy(), kinv)
    return pinv.astype(np.float32), combine


def get_geometry(frustum, rots, trans, intrins, post_rots, post_trans) -> np.ndarray:
    """Frustum -> ego-frame xyz, (B, N, D, fH, fW, 3) float32 (``src/models.py:170-190``)."""
    fr = np.asarray(frustum.detach().cpu().numpy() if torch.is_tensor(frustum) else frustum, dtype=np.float32)
    B, N = trans.shape[:2]
    pinv, combine = camera_matrices(rots, intrins, post_rots)
    pt = post_trans.detach().cpu().float().numpy().reshape(B, N, 1, 1, 1, 3)
    tr = trans.detach().cpu().float().numpy().reshape(B, N, 1, 1, 1, 3)
    p = fr[None, None] - pt                                       # models.py:179
    p = _matvec_seq(pinv.reshape(B, N, 1, 1, 1, 3, 3), p)         # models.py:180
    p = np.stack((p[..., 0] * p[..., 2], p[..., 1] * p[..., 2], p[..., 2]), -1)  # 183-185
    p = _matvec_seq(combine.reshape(B, N, 1, 1, 1, 3, 3), p)      # models.py:186-187
    return (p + tr).astype(np.float32)                            # models.py:188


# ----------------------------------------------------------------------------- a7
def quantize(geom: np.ndarray, dx, bx, nx) -> Tuple[np.ndarray, np.ndarray]:
    """Voxel ids (Nprime, 4) = (x, y, z, b) int64 and the in-grid mask (``src/models.py:211-223``).

    ``.long()`` truncates toward zero; points in (-1 cell, 0) therefore land in cell 0.
    """
    B = geom.shape[0]
    g = geom.reshape(-1, 3).astype(np.float32)
    lo = (bx - dx / np.float32(2.0)).astype(np.float32)
    with np.errstate(invalid="ignore"):
        q = (g - lo) / dx
        ids = np.trunc(q)
        ok = np.isfinite(ids).all(1)
        ids = np.where(np.isfinite(ids), ids, -1).astype(np.int64)
    nprime = ids.shape[0]
    bix = np.repeat(np.arange(B, dtype=np.int64), nprime // B)[:, None]   # models.py:214-216
    ids = np.concatenate([ids, bix], 1)
    kept = ok & (ids[:, 0] >= 0) & (ids[:, 0] < nx[0]) & (ids[:, 1] >= 0) & (ids[:, 1] < nx[1]) \
        & (ids[:, 2] >= 0) & (ids[:, 2] < nx[2])
    return ids, kept


def ranks_of(ids: np.ndarray, nx, B: int) -> np.ndarray:
    """Sort key x*(Y*Z*B) + y*(Z*B) + z*B + b (``src/models.py:226-229``)."""
    return ids[:, 0] * (nx[1] * nx[2] * B) + ids[:, 1] * (nx[2] * B) + ids[:, 2] * B + ids[:, 3]


def output_cell(ids: np.ndarray, nx) -> np.ndarray:
    """Flat index of a voxel in the (B, Z, X, Y) output grid (griddify, ``src/models.py:240-244``)."""
    X, Y, Z = int(nx[0]), int(nx[1]), int(nx[2])
    return ((ids[:, 3] * Z + ids[:, 2]) * X + ids[:, 0]) * Y + ids[:, 1]


# ----------------------------------------------------------------------------- a5
def lift(depthnet_out: torch.Tensor, D: int, C: int):
    """depth = softmax over D; new_x = depth (x) context (``src/models.py:49-61``)."""
    depth = depthnet_out[:, :D].softmax(dim=1)
    new_x = depth.unsqueeze(1) * depthnet_out[:, D:D + C].unsqueeze(2)
    return depth, new_x


def cam_feats_layout(new_x: torch.Tensor, B: int, N: int) -> torch.Tensor:
    """(B*N, C, D, fH, fW) -> (B, N, D, fH, fW, C) view (``src/models.py:199-200``)."""
    BN, C, D, fH, fW = new_x.shape
    return new_x.view(B, N, C, D, fH, fW).permute(0, 1, 3, 4, 5, 2)


# ----------------------------------------------------------------------------- a9-a11
def _segment_boundaries(ranks: torch.Tensor) -> torch.Tensor:
    last = torch.ones(ranks.shape[0], dtype=torch.bool)
    last[:-1] = ranks[1:] != ranks[:-1]
    return last


def cumsum_trick(x, geom_feats, ranks):
    """Plain-autograd segmented sum (``src/tools.py:182-190``)."""
    c = x.cumsum(0)
    last = _segment_boundaries(ranks)
    c, geom_feats = c[last], geom_feats[last]
    return torch.cat((c[:1], c[1:] - c[:-1])), geom_feats


class QuickCumsum(torch.autograd.Function):
    """Segmented sum with a gather backward (``src/tools.py:193-219``)."""

    @staticmethod
    def forward(ctx, x, geom_feats, ranks):
        c = x.cumsum(0)
        last = _segment_boundaries(ranks)
        c, geom_feats = c[last], geom_feats[last]
        out = torch.cat((c[:1], c[1:] - c[:-1]))
        ctx.save_for_backward(last)
        ctx.mark_non_differentiable(geom_feats)
        return out, geom_feats

    @staticmethod
    def backward(ctx, gradx, gradgeom):
        last, = ctx.saved_tensors
        seg = torch.cumsum(last, 0)
        seg[last] -= 1
        return gradx[seg], None, None


# ----------------------------------------------------------------------------- a7-a12
def voxel_pooling(geom: np.ndarray, x: torch.Tensor, dx, bx, nx, use_quickcumsum: bool = True,
                  segment_fn: Optional[Callable] = None) -> torch.Tensor:
    """Reference splat: (B, N, D, fH, fW, C) features -> (B, Z*C, X, Y) (``src/models.py:204-246``).

    Differentiable in ``x``. ``geom`` is the float32 geometry from :func:`get_geometry`.
    ``segment_fn(x, geom_feats, ranks)``, if given, replaces the cumsum step (``src/models.py:233-237``):
    the op-level parity tests plug the product's HIP ``QuickCumsum`` in here.
    """
    B, N, D, H, W, C = x.shape
    nprime = B * N * D * H * W
    xf = x.reshape(nprime, C)
    ids, kept = quantize(geom, dx, bx, nx)
    keep_t = torch.from_numpy(kept)
    xf = xf[keep_t]
    ids_t = torch.from_numpy(ids[kept])
    ranks = torch.from_numpy(ranks_of(ids[kept], nx, B))
    order = ranks.argsort()
    xf, ids_t, ranks = xf[order], ids_t[order], ranks[order]
    if segment_fn is not None:
        xf, ids_t = segment_fn(xf, ids_t, ranks)
    elif use_quickcumsum:
        xf, ids_t = QuickCumsum.apply(xf, ids_t, ranks)
    else:
        xf, ids_t = cumsum_trick(xf, ids_t, ranks)
    X, Y, Z = int(nx[0]), int(nx[1]), int(nx[2])
    final = torch.zeros((B, C, Z, X, Y), dtype=xf.dtype)
    final[ids_t[:, 3], :, ids_t[:, 2], ids_t[:, 0], ids_t[:, 1]] = xf
    return torch.cat(final.unbind(dim=2), 1)


def voxel_pooling_fp64(geom: np.ndarray, x: np.ndarray, dx, bx, nx) -> np.ndarray:
    """Exact segment sums in float64 -- the tolerance anchor (SURVEY.md §7 'Tolerance')."""
    B, N, D, H, W, C = x.shape
    xf = np.asarray(x, dtype=np.float64).reshape(-1, C)
    ids, kept = quantize(geom, dx, bx, nx)
    X, Y, Z = int(nx[0]), int(nx[1]), int(nx[2])
    cell = output_cell(ids[kept], nx)
    acc = np.zeros((B * Z * X * Y, C), dtype=np.float64)
    np.add.at(acc, cell, xf[kept])
    return acc.reshape(B, Z, X, Y, C).transpose(0, 1, 4, 2, 3).reshape(B, Z * C, X, Y)


# ----------------------------------------------------------------------------- backward, analytic
def lift_splat_backward_fp64(depthnet_out: np.ndarray, geom: np.ndarray, dbev: np.ndarray,
                             dx, bx, nx, D: int, C: int) -> np.ndarray:
    """d loss / d depthnet_out for out = voxel_pooling(lift(depthnet_out)), in float64.

    The reference's backward is a gather (``src/tools.py:212-219``) followed by the
    autograd of the outer product and softmax (``src/models.py:58-59``).
    """
    BN, _, fH, fW = depthnet_out.shape
    B = geom.shape[0]
    N = BN // B
    X, Y, Z = int(nx[0]), int(nx[1]), int(nx[2])
    logits = depthnet_out[:, :D].astype(np.float64)
    ctxf = depthnet_out[:, D:D + C].astype(np.float64)                 # (BN, C, fH, fW)
    e = np.exp(logits - logits.max(1, keepdims=True))
    depth = e / e.sum(1, keepdims=True)                                  # (BN, D, fH, fW)
    ids, kept = quantize(geom, dx, bx, nx)
    cell = np.where(kept, output_cell(ids, nx), 0)
    g = dbev.astype(np.float64).reshape(B, Z, C, X, Y).transpose(0, 1, 3, 4, 2).reshape(-1, C)
    gp = g[cell] * kept[:, None]                                          # (Nprime, C)
    gp = gp.reshape(BN, D, fH, fW, C)
    ctx_t = ctxf.transpose(0, 2, 3, 1)                                    # (BN, fH, fW, C)
    d_depth = np.einsum("ndhwc,nhwc->ndhw", gp, ctx_t)
    d_ctx = np.einsum("ndhwc,ndhw->nchw", gp, depth)
    d_logits = depth * (d_depth - (depth * d_depth).sum(1, keepdims=True))
    return np.concatenate([d_logits, d_ctx], 1)


# ----------------------------------------------------------------------------- a13
def get_voxels(frustum, depthnet_out: torch.Tensor, rots, trans, intrins, post_rots, post_trans,
               dx, bx, nx, D: int, C: int = 64, use_quickcumsum: bool = True,
               segment_fn: Optional[Callable] = None) -> torch.Tensor:
    """geometry -> lift -> splat, i.e. ``get_voxels`` with the trunk already applied
    (``src/models.py:248-254``); ``depthnet_out`` is (B*N, D+C, fH, fW)."""
    B, N = trans.shape[:2]
    geom = get_geometry(frustum, rots, trans, intrins, post_rots, post_trans)
    _, new_x = lift(depthnet_out, D, C)
    x = cam_feats_layout(new_x, B, N)
    return voxel_pooling(geom, x, dx, bx, nx, use_quickcumsum, segment_fn)


def full_forward(trunk: Callable[[torch.Tensor], torch.Tensor], bevencode: Callable[[torch.Tensor], torch.Tensor],
                 frustum, x, rots, trans, intrins, post_rots, post_trans, dx, bx, nx, D: int, C: int = 64,
                 use_quickcumsum: bool = True) -> torch.Tensor:
    """Whole ``LiftSplatShoot.forward`` on the CPU (``src/models.py:256-259``).

    ``trunk`` maps (B*N, 3, H, W) images to the depthnet output (B*N, D+C, fH, fW);
    ``bevencode`` maps the BEV to logits. The conv stacks are supplied by the caller
    (the reference's come from efficientnet_pytorch / torchvision, absent here).
    """
    B, N = x.shape[:2]
    dn = trunk(x.reshape(B * N, *x.shape[2:]))
    bev = get_voxels(frustum, dn, rots, trans, intrins, post_rots, post_trans, dx, bx, nx, D, C, use_quickcumsum)
    return bevencode(bev)


def voxel_stats(geom: np.ndarray, dx, bx, nx) -> dict:
    """Known-answer facts of SURVEY.md §8c (kept, occupied voxels, max per voxel, trunc != floor)."""
    ids, kept = quantize(geom, dx, bx, nx)
    cell = output_cell(ids[kept], nx)
    _, counts = np.unique(cell, return_counts=True)
    lo = (bx - dx / np.float32(2.0)).astype(np.float32)
    q = (geom.reshape(-1, 3) - lo) / dx
    trunc_ne_floor = int((np.trunc(q) != np.floor(q)).any(1).sum())
    return {"nprime": int(ids.shape[0]), "kept": int(kept.sum()), "occupied": int(counts.size),
            "max_per_voxel": int(counts.max()) if counts.size else 0, "trunc_ne_floor": trunc_ne_floor}
