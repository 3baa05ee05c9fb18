"""Flat fp32 master parameters with per-step bf16 working copies (mixed precision in two kernels).

Under bf16 autocast every conv casts its fp32 weight (and bias) to bf16 on each call and the
backward casts each bf16 weight gradient back to fp32: ~250 small copy kernels per step at config
3, each a few microseconds, plus one gradient-accumulation, Adam and clip pass per parameter tensor.
``FlatParams`` keeps the trainable parameters of a module in ONE fp32 buffer (``master``, the only
tensor the optimizer and the all-reduce see; the module's nn.Parameters become views of it, so
state_dict and in-place updates stay coherent) and materialises, once per forward:

  * the weights/biases autocast would cast (nn.Conv2d with groups == 1, nn.Linear) as bf16 views of
    one buffer -- ``master[:n16].to(bf16)``, one kernel, the same round-to-nearest-even values the
    autocast cast produces;
  * the rest (BatchNorm affine parameters, depthwise weights consumed in fp32 by the lss_dwconv_*
    kernels) as fp32 views of one copy.

``forward(*args)`` runs the module with these tensors swapped in (torch.func.functional_call).
Backward gathers the per-view gradients into one flat bf16 and one flat fp32 buffer with
multi-tensor copies and returns ``master``'s fp32 gradient in one piece (it lands in
``master.grad`` without an accumulation kernel). Numerics are those of autocast: identical bf16
operands and fp32 gradients; only the summation order of clip_grad_norm_'s norm changes.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import os

import torch
from torch import nn


def autocast_cast_names(model: nn.Module) -> set:
    """Names of parameters a bf16 autocast region would cast on use: weights and biases of
    non-grouped nn.Conv2d and of nn.Linear (depthwise convs stay fp32: lss_dwconv_* reads fp32)."""
    names = set()
    for mname, m in model.named_modules():
        if getattr(m, "lss_fp32_params", False):  # consumed in fp32 by a HIP kernel (rounds them itself)
            continue
        if (isinstance(m, nn.Conv2d) and m.groups == 1) or isinstance(m, nn.Linear):
            for pname, _ in m.named_parameters(recurse=False):
                names.add(f"{mname}.{pname}" if mname else pname)
    return names


def _dense(p: torch.Tensor) -> bool:
    return p.is_contiguous() or (p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last))


def _views(buf: torch.Tensor, like: List[torch.Tensor]) -> List[torch.Tensor]:
    out, off = [], buf.storage_offset()  # as_strided offsets are absolute in the storage
    for p in like:
        out.append(buf.as_strided(p.shape, p.stride(), off))
        off += p.numel()
    return out


class _Materialize(torch.autograd.Function):
    @staticmethod
    def forward(ctx, master: torch.Tensor, fp: "FlatParams"):
        n16 = fp.n16
        if n16 and fp.dn is not None:
            # one launch: the bf16 copy and the depthnet weight in the fused lift's fragment order
            from . import _lib
            w_off, O, K = fp.dn
            _lib.check(_lib.load().lss_flat_cast_bf16(_lib.ptr(master), _lib.ptr(fp.work16), n16,
                                                      _lib.ptr(master[w_off:w_off + O * K]), O, K,
                                                      _lib.ptr(fp.dn_packed), _lib.stream_handle(master.device)),
                       "lss_flat_cast_bf16")
        elif n16:
            fp.work16.copy_(master[:n16])
        fp.work32.copy_(master[n16:])
        ctx.fp = fp
        # fresh view objects per call (each carries this call's autograd history)
        return tuple(_views(fp.work16, fp.like16) + _views(fp.work32, fp.like32))

    @staticmethod
    def backward(ctx, *grads):
        fp: FlatParams = ctx.fp
        n16, k16 = fp.n16, len(fp.like16)
        dev = fp.master.device
        d_master = torch.empty(fp.numel, device=dev, dtype=torch.float32)
        if n16:
            g16 = torch.empty(n16, device=dev, dtype=fp.cast_dtype)
            _gather(_views(g16, fp.like16), grads[:k16], g16)
            d_master[:n16].copy_(g16)
        _gather(_views(d_master[n16:], fp.like32), grads[k16:], d_master[n16:])
        return d_master, None


GATHER_SPLIT = os.environ.get("LSS_FLAT_GATHER_SPLIT", "1") != "0"


def _gather(dst_views, grads, buf) -> None:
    """Copy the per-parameter gradients into their views of buf (unused parameters: zero)."""
    if any(g is None for g in grads):
        buf.zero_()
    pairs = [(d, _restride(g, d)) for d, g in zip(dst_views, grads) if g is not None]
    # _foreach_copy_ takes its multi-tensor route only when EVERY pair has the same dtype and strides;
    # one odd pair (a channels-last conv weight gradient into a contiguous view) would send all of them
    # through a strided copy each: the odd ones are copied on their own
    if not GATHER_SPLIT:  # (A/B: the single _foreach_copy_ of round 5)
        torch._foreach_copy_([d for d, _ in pairs], [g.to(d.dtype) for d, g in pairs])
        return
    fast = [(d, g) for d, g in pairs if g.dtype == d.dtype and g.stride() == d.stride()]
    if fast:
        torch._foreach_copy_([d for d, _ in fast], [g for _, g in fast])
    for d, g in pairs:
        if g.dtype != d.dtype or g.stride() != d.stride():
            d.copy_(g)


def _restride(g: torch.Tensor, d: torch.Tensor) -> torch.Tensor:
    """g re-viewed with d's strides when the two differ only on size-1 dimensions (a 1x1 conv weight's
    gradient in (O, I, 1, 1) contiguous strides against a channels-last parameter view): the same memory
    order, so _foreach_copy_ keeps its one-launch multi-tensor route instead of a strided copy per tensor."""
    if g.shape != d.shape or g.stride() == d.stride() or not g.is_contiguous():
        return g
    if all(gs == ds for gs, ds, n in zip(g.stride(), d.stride(), d.shape) if n != 1):
        return g.as_strided(d.shape, d.stride())
    return g


class FlatParams:
    def __init__(self, model: nn.Module, cast_dtype=torch.bfloat16, prefixes=None):
        """prefixes: only the parameters whose dotted names start with one of these (a group of
        FlatParamGroups); None: every trainable parameter."""
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        if prefixes is not None:
            named = [(n, p) for n, p in named if any(n == pre or n.startswith(pre + ".") for pre in prefixes)]
        if not named:
            raise ValueError("FlatParams: no trainable parameters")
        for n, p in named:
            if p.dtype != torch.float32 or not _dense(p):
                raise ValueError(f"FlatParams: {n} must be a dense fp32 tensor")
        cast = autocast_cast_names(model) if cast_dtype is not None else set()
        self.names16 = [n for n, _ in named if n in cast]
        self.names32 = [n for n, _ in named if n not in cast]
        byname = dict(named)
        self.like16 = [byname[n] for n in self.names16]
        self.like32 = [byname[n] for n in self.names32]
        self.cast_dtype = cast_dtype
        self.n16 = sum(p.numel() for p in self.like16)
        self.numel = self.n16 + sum(p.numel() for p in self.like32)
        dev = named[0][1].device
        master = torch.empty(self.numel, device=dev, dtype=torch.float32)
        with torch.no_grad():
            for v, p in zip(_views(master, self.like16 + self.like32), self.like16 + self.like32):
                v.copy_(p)
                p.data = v  # the module's Parameters now alias the master buffer
        self.master = nn.Parameter(master)
        self.work16 = torch.empty(self.n16, device=dev, dtype=cast_dtype or torch.float32)
        self.work32 = torch.empty(self.numel - self.n16, device=dev, dtype=torch.float32)
        # the depthnet 1x1 conv (CamEncode.depthnet, src/models.py:47) of a fused-lift model: its bf16
        # weight is also kept in the lift kernel's fragment order, written by the same cast launch
        # (lss_flat_cast_bf16), and handed to the module through the weight view's storage address
        self.dn, self.dn_packed = None, None
        dn = getattr(model, "camencode", None)
        dn = getattr(dn, "depthnet", None)
        wname = next((n for n in self.names16 if n.endswith("camencode.depthnet.weight")), None)
        if (dn is not None and wname is not None and dev.type == "cuda" and cast_dtype == torch.bfloat16
                and dn.weight.shape[1] % 32 == 0 and dn.weight.shape[1] <= 512 and dn.weight.shape[0] <= 128):
            from . import _lib
            off = 0
            for n, p in zip(self.names16, self.like16):
                if n == wname:
                    break
                off += p.numel()
            O, K = dn.weight.shape[0], dn.weight.shape[1]
            self.dn = (off, O, K)
            self.dn_packed = torch.empty(_lib.DN_PACKED_BYTES(K) // 2, device=dev, dtype=torch.bfloat16)
            dn.lss_packed_weight = (self.dn_packed, self.work16.data_ptr() + 2 * off)

    def tensors(self) -> Dict[str, torch.Tensor]:
        outs = _Materialize.apply(self.master, self)
        return dict(zip(self.names16 + self.names32, outs))

    def bind(self, model: nn.Module):
        """A callable running `model` on the materialised working parameters."""
        def run(*args, **kwargs):
            return torch.func.functional_call(model, self.tensors(), args, kwargs, strict=False)
        return run

    def views_of(self, flat: torch.Tensor) -> Dict[str, torch.Tensor]:
        """Per-parameter views (the original shapes/strides) of a flat tensor laid out like master."""
        return dict(zip(self.names16 + self.names32, _views(flat, self.like16 + self.like32)))


class FlatParamGroups:
    """Several FlatParams over disjoint parameter groups, run as one module: one fp32 master (and one
    gradient) per group. A group's gradient is complete as soon as the backward has passed all of its
    parameters, so groups listed in the order the backward finishes them (the BEV encoder first, the
    trunk's early blocks last) let TrainStep all-reduce each one while the backward continues."""

    def __init__(self, model: nn.Module, groups, cast_dtype=torch.bfloat16):
        trainable = [n for n, p in model.named_parameters() if p.requires_grad]
        taken = set()
        self.groups = []
        for prefixes in groups:
            names = [n for n in trainable if n not in taken and any(n == pre or n.startswith(pre + ".") for pre in prefixes)]
            if names:
                taken.update(names)
                self.groups.append(FlatParams(model, cast_dtype=cast_dtype, prefixes=names))
        rest = [n for n in trainable if n not in taken]
        if rest:
            self.groups.append(FlatParams(model, cast_dtype=cast_dtype, prefixes=rest))

    @property
    def masters(self) -> List[nn.Parameter]:
        return [g.master for g in self.groups]

    def views(self, grads: bool = False) -> Dict[str, torch.Tensor]:
        """name -> view of the masters (or of their gradients)."""
        out = {}
        for g in self.groups:
            out.update(g.views_of(g.master.grad if grads else g.master.detach()))
        return out

    def bind(self, model: nn.Module):
        def run(*args, **kwargs):
            tensors = {}
            for g in self.groups:
                tensors.update(g.tensors())
            return torch.func.functional_call(model, tensors, args, kwargs, strict=False)
        return run


def lss_backward_groups(prefix: str = "") -> list:
    """LiftSplatShoot's parameters in the order the backward completes them: BevEncode, then the
    camera encoder's head (up1, depthnet) with the trunk's last blocks, then (the remainder group
    FlatParamGroups adds) the rest of the trunk. `prefix`: the model's name inside a wrapper."""
    late = [f"{prefix}camencode.trunk._blocks.{i}" for i in range(11, 16)]
    return [[f"{prefix}bevencode"], [f"{prefix}camencode.up1", f"{prefix}camencode.depthnet"] + late]
