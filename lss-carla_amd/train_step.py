"""The training step of train_simbev.py:229-248 -- forward, SimpleLoss, backward,
clip_grad_norm_(max_grad_norm), Adam -- eager, or replayed as two HIP graphs.

A B=8 step launches ~2000 kernels (conv stacks, BN, the lift/splat path, optimizer); eager, the
host's Python + launch cost per kernel is longer than many of the kernels, so the GPU idles.
Captured (``torch.cuda.CUDAGraph``, i.e. hipGraph), the step is two graph launches:

  graph A  forward under bf16 autocast, loss, backward
  (eager)  all-reduce of the gradients over RCCL (world size > 1)
  graph B  divide by the world size, clip_grad_norm_, fused Adam (capturable)

With ``overlap_all_reduce`` (and ``flat_params.FlatParamGroups``: one master per parameter group, in
the order the backward completes them) each group's all-reduce starts from its post-accumulate hook
on a side stream while the backward continues, captured into graph A; the eager all-reduce between
the graphs is then skipped.

With ``flat_params.FlatParams`` the trainable parameters are one fp32 tensor, so the gradient is one
tensor too: one ~50 MB ring all-reduce over xGMI per step (the same averaged gradient as DDP), a
single-tensor Adam and norm. Every op of the LSS path is capturable: its kernels take device
pointers only and the plan's sizes come from the static shapes; the one host round trip of the
reference (torch.inverse on the CPU, src/models.py:180,186) moves out of the captured region:
``pre_step`` inverts the host copy of the rig with the same call and stages the results into static
device buffers (ops.HostInverses) before each replay, so the captured step reads bit-identical
inverses. (A device fp64 adjugate inverse, not bit-exact, was removed in round 4 with the other
off-by-default options; its measurements stay in profiles/r03.)
"""
from __future__ import annotations

import time
from typing import Callable, Optional, Sequence

import torch
import torch.distributed as dist


class TrainStep:
    """forward(*inputs) -> preds; params: what the optimizer updates (e.g. [FlatParams.master]);
    all_reduce: average params' gradients over the process group here (False under DDP)."""

    def __init__(self, forward: Callable[..., torch.Tensor], inputs: Sequence[torch.Tensor], labels: torch.Tensor,
                 loss_fn: Callable, opt: torch.optim.Optimizer, params: Sequence[torch.Tensor],
                 all_reduce: bool = False, amp_dtype: Optional[torch.dtype] = torch.bfloat16,
                 max_grad_norm: float = 5.0, pre_step: Optional[Callable[[], None]] = None,
                 overlap_all_reduce: bool = False, force_collectives: bool = False):
        """overlap_all_reduce: all-reduce each parameter's gradient (e.g. each FlatParamGroups
        master) from its post-accumulate hook, on a side stream, while the backward continues -- inside
        the captured graph too; the step waits for them before the update. force_collectives: issue
        the collectives even at world size 1 (tests of the captured path on one GPU)."""
        self.forward, self.inputs, self.labels = forward, tuple(inputs), labels
        # host work staged into the step's static device inputs before each step is launched
        # (e.g. ops.HostInverses.update: the reference's host torch.inverse of the rig)
        self.pre_step = pre_step
        self.loss_fn, self.opt, self.params = loss_fn, opt, list(params)
        self.amp_dtype, self.max_grad_norm = amp_dtype, max_grad_norm
        on = all_reduce and dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size() if on else 1
        self.collectives = on and (self.world > 1 or force_collectives)
        self.overlap = bool(overlap_all_reduce) and self.collectives
        self._works = []
        self._side = None
        if self.overlap:
            for p in self.params:
                p.register_post_accumulate_grad_hook(self._reduce_ready)
        self.graphs = None
        self.graph_grads = None
        self.static_loss = None

    @property
    def captured(self) -> bool:
        return self.graphs is not None

    def forward_backward(self) -> torch.Tensor:
        self.opt.zero_grad(set_to_none=True)  # backward's gradient is stolen, not accumulated
        dev_type = self.labels.device.type
        # autocast's cast cache must be off while capturing (its entries would outlive the capture)
        capturing = dev_type == "cuda" and torch.cuda.is_current_stream_capturing()
        with torch.autocast(dev_type, dtype=self.amp_dtype or torch.bfloat16, enabled=self.amp_dtype is not None,
                            cache_enabled=not capturing):
            preds = self.forward(*self.inputs)
        # (a loss that computes in fp32 itself, tools.SimpleLoss, takes the bf16 logits: no cast kernels)
        loss = self.loss_fn(preds if getattr(self.loss_fn, "computes_in_fp32", False) else preds.float(), self.labels)
        loss.backward()
        if self.overlap:  # the collectives the hooks started: the update waits for them
            for w in self._works:
                w.wait()
            if self._side is not None:
                torch.cuda.current_stream(self.labels.device).wait_stream(self._side)
            self._works = []
        return loss

    def _reduce_ready(self, p: torch.Tensor) -> None:
        """post-accumulate-grad hook: p.grad is final; start its all-reduce beside the backward."""
        if p.grad is None:
            return
        if p.grad.is_cuda:
            dev = p.grad.device
            if self._side is None:
                self._side = torch.cuda.Stream(dev)
            self._side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(self._side):
                self._works.append(dist.all_reduce(p.grad, async_op=True))
        else:
            self._works.append(dist.all_reduce(p.grad, async_op=True))

    def all_reduce(self, grads=None) -> None:
        """Sum the gradients over ranks (eager: outside any capture); no-op when the hooks did it."""
        if self.collectives and not self.overlap:
            for g in (grads if grads is not None else [p.grad for p in self.params]):
                if g is not None:
                    dist.all_reduce(g)

    def update(self) -> None:
        if self.world > 1:
            for p in self.params:
                if p.grad is not None:
                    p.grad.mul_(1.0 / self.world)
        from . import optim
        if optim.supported(self.opt, self.params):  # both in two launches on the GPU (lss_clip_adam)
            if getattr(self, "_clip_adam", None) is None or self._clip_adam.opt is not self.opt:
                self._clip_adam = optim.ClipAdam(self.opt)
            self._clip_adam.step(self.max_grad_norm)
            return
        torch.nn.utils.clip_grad_norm_(self.params, self.max_grad_norm)
        self.opt.step()

    def eager(self) -> torch.Tensor:
        if self.pre_step is not None:
            self.pre_step()
        loss = self.forward_backward()
        self.all_reduce()
        self.update()
        return loss

    def capture(self, warmup: int = 2, on_warmup: Optional[Callable[[int], None]] = None) -> None:
        """`warmup` eager steps on a side stream (MIOpen find, optimizer state, allocator), then
        capture (the optimizer must be built with capturable=True)."""
        dev = self.labels.device
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for i in range(max(warmup, 1)):
                self.eager()
                if on_warmup is not None:
                    on_warmup(i)
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        mode = "global"
        if self.collectives:
            # the process group's watchdog thread polls the warm-up's all-reduce events (every 100 ms)
            # until it reaps them; one such query during a global-mode capture aborts the process
            # ("operation not permitted when stream is capturing", seen in a world-size-1 RCCL run).
            # Let it reap the completed works, and restrict the capture's checks to this thread.
            time.sleep(0.5)
            mode = "thread_local"
        g_fb, g_up = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_fb, capture_error_mode=mode):
            # detached: holding the captured autograd graph would keep its AccumulateGrad nodes
            # (bound to the capture stream) alive into later eager steps. The gradients allocated
            # here (graph pool) are what graph B and the all-reduce read on every replay.
            self.static_loss = self.forward_backward().detach()
        self.graph_grads = [p.grad for p in self.params]
        with torch.cuda.graph(g_up, pool=g_fb.pool(), capture_error_mode=mode):
            self.update()
        self.graphs = (g_fb, g_up)

    def __call__(self) -> torch.Tensor:
        if self.graphs is None:
            return self.eager()
        g_fb, g_up = self.graphs
        if self.pre_step is not None:
            self.pre_step()
        g_fb.replay()  # with overlap_all_reduce the collectives are inside this graph
        self.all_reduce(self.graph_grads)
        g_up.replay()
        return self.static_loss
