"""Training-side helpers with the reference's names (src/tools.py).

What the LiftSplatShoot training step and its callers use: the grid helper, the op-level
segmented sum (``QuickCumsum`` / ``cumsum_trick``, HIP-backed), the loss and the IoU metric. The
reference's nuScenes/visualisation helpers are out of scope; its
image/label helpers live in ``simbev.py``.
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


# ----------------------------------------------------------------------------- op-level segmented sum
class QuickCumsum(torch.autograd.Function):
    """``QuickCumsum.apply(x, geom_feats, ranks)`` of src/tools.py:193-219 on HIP kernels.

    x (n, C) rows sorted by ``ranks`` (n,) int64; geom_feats (n, k) int64. Returns one row per run
    of equal ranks: (x_seg (nseg, C), geom_seg (nseg, k)) with geom_seg = the geom_feats row of the
    run's last row, as the reference's ``geom_feats[kept]``. Forward: lss_segment_build +
    lss_segment_sum (each run summed in row order in fp32 -- the reference differences two
    fp32-rounded prefix sums, which is off the exact sum by ~ulp(prefix); this is not). Backward:
    lss_segment_gather, the reference's ``gradx[back]`` (identical values). The number of runs is
    read back once, as the reference's boolean indexing does. Device tensors only.
    """

    @staticmethod
    def forward(ctx, x, geom_feats, ranks):
        from . import ops
        if x.dim() != 2 or ranks.dim() != 1 or ranks.shape[0] != x.shape[0] or geom_feats.shape[0] != x.shape[0]:
            raise RuntimeError(f"QuickCumsum: x {tuple(x.shape)}, geom_feats {tuple(geom_feats.shape)} and ranks "
                               f"{tuple(ranks.shape)} do not describe the same rows")
        ops._require_cuda(x, geom_feats, ranks)
        n, C = x.shape
        if n == 0:
            seg_of = torch.empty(0, device=x.device, dtype=torch.int32)
            out, gout = x.new_empty(0, C), geom_feats.new_empty((0,) + tuple(geom_feats.shape[1:]))
        else:
            seg_of, seg_start, nseg = ops.segment_runs(ranks)
            out, gout = ops.segment_sum(x, seg_start, nseg, geom_feats)
            out = out.to(x.dtype)
        ctx.save_for_backward(seg_of)
        ctx.x_dtype = x.dtype
        ctx.mark_non_differentiable(gout)
        return out, gout

    @staticmethod
    def backward(ctx, gradx, gradgeom):
        from . import ops
        seg_of, = ctx.saved_tensors
        if seg_of.numel() == 0:
            return gradx.new_empty(0, gradx.shape[1]), None, None
        return ops.segment_gather(gradx, seg_of).to(ctx.x_dtype), None, None


def cumsum_trick(x, geom_feats, ranks):
    """src/tools.py:182-190: the same segmented sum, differentiable in x (the reference reaches the
    same gradient through autograd of cumsum / indexing / cat; here it is the gather directly)."""
    return QuickCumsum.apply(x, geom_feats, ranks)


# ----------------------------------------------------------------------------- loss / metrics
class _BceLogits(torch.autograd.Function):
    """BCEWithLogitsLoss(pos_weight), mean, on ``lss_bce_logits`` (include/lss_convs.h): the loss and
    its input gradient in one pass plus a fixed-order fold of the block sums -- two launches where
    torch's decomposition runs about twenty elementwise / reduction kernels per step. The backward
    scales the stored gradient by the incoming one (``lss_bce_logits_bwd``, read on the device)."""

    @staticmethod
    def forward(ctx, x, target, pos_weight: float):
        from . import _lib
        lib = _lib.load()
        n = x.numel()
        partial = torch.empty(int(lib.lss_bce_partials(n)), device=x.device, dtype=torch.float32)
        loss = torch.empty((), device=x.device, dtype=torch.float32)
        grad = torch.empty_like(x)
        _lib.check(lib.lss_bce_logits(_lib.ptr(x), _lib.dtype_code(x.dtype), _lib.ptr(target), n, float(pos_weight),
                                      _lib.ptr(partial), _lib.ptr(loss), _lib.ptr(grad),
                                      _lib.stream_handle(x.device)), "lss_bce_logits")
        ctx.save_for_backward(grad)
        return loss

    @staticmethod
    def backward(ctx, g):
        from . import _lib
        (grad,) = ctx.saved_tensors
        g = g.float().contiguous()
        dx = torch.empty_like(grad)
        _lib.check(_lib.load().lss_bce_logits_bwd(_lib.ptr(grad), _lib.dtype_code(grad.dtype), grad.numel(),
                                                  _lib.ptr(g), _lib.ptr(dx), _lib.stream_handle(grad.device)),
                   "lss_bce_logits_bwd")
        return dx, None, None


class SimpleLoss(torch.nn.Module):
    """BCE-with-logits with a positive-class weight (src/tools.py:222-230).

    On the GPU (fp32 or bf16 logits, fp32 labels of the same shape, contiguous) the loss and its
    gradient come from the fused ``lss_bce_logits`` kernel, computed in fp32 (a bf16 input gives the
    loss of its exact fp32 cast); otherwise ``loss_fn`` (the reference's ``BCEWithLogitsLoss``). The
    weight is the constructor's value (reading the module's device buffer back would synchronise)."""

    computes_in_fp32 = True  # callers may pass bf16 logits without casting them first (train_step)

    def __init__(self, pos_weight: float):
        super().__init__()
        self.loss_fn = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([float(pos_weight)]))
        self.pos_weight_value = float(pos_weight)

    def forward(self, ypred, ytgt):
        if (ypred.is_cuda and ypred.dtype in (torch.float32, torch.bfloat16) and ytgt.dtype == torch.float32
                and ytgt.device == ypred.device and ytgt.shape == ypred.shape and ypred.is_contiguous()
                and ytgt.is_contiguous() and ypred.data_ptr() % 16 == 0 and ytgt.data_ptr() % 16 == 0
                and ypred.numel() > 0):
            return _BceLogits.apply(ypred, ytgt, self.pos_weight_value)
        return self.loss_fn(ypred.float() if ypred.dtype == torch.bfloat16 else ypred, ytgt)


def get_batch_iou(preds: torch.Tensor, binimgs: torch.Tensor):
    """Intersection, union and IoU of (logit > 0) vs the labels, as Python floats (src/tools.py:232-240)."""
    intersect, union = get_batch_iou_device(preds, binimgs)
    intersect, union = intersect.item(), union.item()
    return intersect, union, intersect / union if (union > 0) else 1.0


def get_batch_iou_device(preds: torch.Tensor, binimgs: torch.Tensor):
    """Same counts as device tensors, without a host sync."""
    with torch.no_grad():
        pred = preds > 0
        tgt = binimgs.bool()
        return (pred & tgt).sum().float(), (pred | tgt).sum().float()


def val_totals(model, loader, loss_fn, device):
    """The device accumulators of get_val_info: (sum of loss x batch size, intersection, union) as
    float64 device tensors; nothing in the loop synchronises the host."""
    total_loss = torch.zeros((), device=device, dtype=torch.float64)
    total_intersect = torch.zeros((), device=device, dtype=torch.float64)
    total_union = torch.zeros((), device=device, dtype=torch.float64)
    with torch.no_grad():
        for batch in loader:
            allimgs, rots, trans, intrins, post_rots, post_trans, binimgs = batch
            preds = model(allimgs.to(device), rots.to(device), trans.to(device), intrins.to(device),
                          post_rots.to(device), post_trans.to(device))
            binimgs = binimgs.to(device)
            total_loss += loss_fn(preds, binimgs).double() * preds.shape[0]
            i, u = get_batch_iou_device(preds, binimgs)
            total_intersect += i.double()
            total_union += u.double()
    return total_loss, total_intersect, total_union


def get_val_info(model, valloader, loss_fn, device, use_tqdm=True):
    """Validation loss / IoU over a loader (src/tools.py:243-270).

    Same results and the same return dict as the reference, but the per-batch ``.item()`` syncs
    are gone: loss (x batch size) and the intersection / union counts accumulate on the device in
    float64 (val_totals) and are read once at the end. As in the reference, the loss is divided by
    ``len(valloader.dataset)`` and an empty union raises ZeroDivisionError.
    """
    model.eval()
    print("running eval...")
    loader = valloader
    if use_tqdm:
        from tqdm import tqdm
        loader = tqdm(valloader, desc="Validation")
    total_loss, total_intersect, total_union = val_totals(model, loader, loss_fn, device)
    model.train()
    return {
        "loss": total_loss.item() / len(valloader.dataset),
        "iou": total_intersect.item() / total_union.item(),
    }
