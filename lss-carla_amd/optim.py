"""The training step's update on the GPU: clip_grad_norm_ + torch.optim.Adam as two launches.

``ClipAdam(opt).step(max_norm)`` does what ``torch.nn.utils.clip_grad_norm_(params, max_norm)`` followed by
``opt.step()`` does for an ``Adam`` over fp32 CUDA tensors (train_simbev.py:245-248): it keeps the
optimizer's own state tensors (``step``, ``exp_avg``, ``exp_avg_sq``, created as torch creates them), so
``opt.state_dict()`` stays what torch would save and either path can continue the other. The gradient
norm is fp32 over all the tensors' gradients; the gradients themselves are left unclipped (nothing reads
them after the step). Kernels: ``lss_clip_adam`` (include/lss_convs.h). Anything it does not cover
(amsgrad, maximize, several parameter groups, tensor learning rates, CPU tensors, other dtypes, an Adam
that is neither ``capturable`` nor ``fused``, whose ``step`` torch keeps on the host) keeps torch's path
(``supported``).
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import torch

from . import _lib

USE_HIP_ADAM = True
MAX_TENSORS = 32  # LSS_ADAM_MAX_TENSORS


def supported(opt: torch.optim.Optimizer, params: Sequence[torch.Tensor]) -> bool:
    if not USE_HIP_ADAM or type(opt) is not torch.optim.Adam or len(opt.param_groups) != 1:
        return False
    g = opt.param_groups[0]
    if g.get("amsgrad") or g.get("maximize") or g.get("differentiable") or g.get("decoupled_weight_decay"):
        return False
    if not (g.get("capturable") or g.get("fused")):
        # torch keeps such an Adam's `step` on the host; the device step this path keeps would change
        # its state_dict and cost the next torch step a sync per tensor
        return False
    if any(isinstance(g[k], torch.Tensor) for k in ("lr", "eps", "weight_decay")) or \
            any(isinstance(b, torch.Tensor) for b in g["betas"]):
        return False
    ps = list(g["params"])
    if len(ps) != len(params) or any(a is not b for a, b in zip(ps, params)) or not 0 < len(ps) <= MAX_TENSORS:
        return False
    for p in ps:
        if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and p.grad is not None
                and p.grad.dtype == torch.float32 and p.grad.is_contiguous() and p.grad.device == p.device):
            return False
    return True


class ClipAdam:
    def __init__(self, opt: torch.optim.Adam):
        self.opt = opt
        self._partial = None

    def _state(self, p: torch.Tensor):
        st = self.opt.state[p]
        if len(st) == 0:  # as torch.optim.Adam initialises it (fused / capturable: the step on the device)
            st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        elif st["step"].device != p.device or st["step"].dtype != torch.float32:
            st["step"] = st["step"].to(device=p.device, dtype=torch.float32)
        return st

    def step(self, max_norm: float) -> None:
        lib = _lib.load()
        g = self.opt.param_groups[0]
        ps = list(g["params"])
        n = len(ps)
        sts = [self._state(p) for p in ps]
        dev = ps[0].device
        if self._partial is None or self._partial.device != dev:
            self._partial = torch.empty(int(lib.lss_clip_adam_partials()), device=dev, dtype=torch.float32)
        arr = lambda ts: (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])  # noqa: E731
        numel = (ctypes.c_int64 * n)(*[p.numel() for p in ps])
        b1, b2 = g["betas"]
        _lib.check(lib.lss_clip_adam(n, arr(ps), arr([p.grad for p in ps]), arr([s["exp_avg"] for s in sts]),
                                     arr([s["exp_avg_sq"] for s in sts]), arr([s["step"] for s in sts]), numel,
                                     float(max_norm), float(g["lr"]), float(b1), float(b2), float(g["eps"]),
                                     float(g["weight_decay"]), _lib.ptr(self._partial), _lib.stream_handle(dev)),
                   "lss_clip_adam")
