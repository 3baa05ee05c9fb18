"""Training-side helpers with the reference's names (src/tools.py).

Only what the LiftSplatShoot training step needs: the grid helper, the loss
and the IoU metric. The reference's nuScenes/visualisation helpers are out of
scope.
"""
from __future__ import annotations

import torch


def gen_dx_bx(xbound, ybound, zbound):
    """Cell size, first-cell centre and cell count per axis (src/tools.py:174-179)."""
    rows = (xbound, ybound, zbound)
    dx = torch.tensor([r[2] for r in rows], dtype=torch.float32)
    bx = torch.tensor([r[0] + r[2] / 2.0 for r in rows], dtype=torch.float32)
    nx = torch.tensor([int((r[1] - r[0]) / r[2]) for r in rows], dtype=torch.long)
    return dx, bx, nx


class SimpleLoss(torch.nn.Module):
    """BCE-with-logits with a positive-class weight (src/tools.py:222-230)."""

    def __init__(self, pos_weight: float):
        super().__init__()
        self.loss_fn = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([float(pos_weight)]))

    def forward(self, ypred, ytgt):
        return self.loss_fn(ypred, ytgt)


def get_batch_iou(preds: torch.Tensor, binimgs: torch.Tensor):
    """Intersection, union and IoU of (logit > 0) vs the labels, as Python floats (src/tools.py:232-240)."""
    intersect, union = get_batch_iou_device(preds, binimgs)
    intersect, union = intersect.item(), union.item()
    return intersect, union, intersect / union if union > 0 else 1.0


def get_batch_iou_device(preds: torch.Tensor, binimgs: torch.Tensor):
    """Same counts as device tensors, without a host sync."""
    with torch.no_grad():
        pred = preds > 0
        tgt = binimgs.bool()
        return (pred & tgt).sum().float(), (pred | tgt).sum().float()


def get_val_info(model, valloader, loss_fn, device, use_tqdm: bool = False):
    """Validation loss / IoU over a loader (src/tools.py:243-270); one host sync per epoch, not per batch."""
    model.eval()
    total_loss = torch.zeros((), device=device)
    inter = torch.zeros((), device=device)
    union = torch.zeros((), device=device)
    n = 0
    with torch.no_grad():
        for allimgs, rots, trans, intrins, post_rots, post_trans, binimgs in valloader:
            preds = model(allimgs.to(device), rots.to(device), trans.to(device), intrins.to(device),
                          post_rots.to(device), post_trans.to(device))
            binimgs = binimgs.to(device)
            total_loss += loss_fn(preds, binimgs) * preds.shape[0]
            i, u = get_batch_iou_device(preds, binimgs)
            inter += i
            union += u
            n += preds.shape[0]
    model.train()
    return {"loss": total_loss.item() / max(len(getattr(valloader, "dataset", [])) or n, 1),
            "iou": inter.item() / union.item() if union.item() > 0 else 1.0}
