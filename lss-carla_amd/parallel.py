"""Data-parallel training over the GPUs of a node: one process per GPU, RCCL gradient all-reduce.

The reference trains on one device (``train_simbev.py:179``); this is the build's
only parallel strategy. Every rank runs geometry, lift, splat and
both conv stacks on its own B samples -- ranks include the batch index, so the
splat never mixes samples -- and gradients are averaged by DDP's bucketed
all-reduce (backend "nccl" = RCCL over xGMI on MI355X), overlapped with backward.
BatchNorm stays per-replica, as in the reference (plain ``nn.BatchNorm2d``).
"""
from __future__ import annotations

import os
from typing import Iterable

import torch
import torch.distributed as dist

# The trunk's classification head is never used by LSS (src/models.py:63-84 stops at the
# blocks): it never receives gradients, so it is kept out of DDP's buckets.
UNUSED_PREFIXES = ("camencode.trunk._conv_head", "camencode.trunk._bn1", "camencode.trunk._fc")


def freeze_unused(model: torch.nn.Module, prefixes: Iterable[str] = UNUSED_PREFIXES) -> int:
    """requires_grad_(False) on parameters that never get a gradient; returns how many were frozen."""
    n = 0
    prefixes = tuple(prefixes)
    for name, p in model.named_parameters():
        dotted = "." + name + "."  # match as a path component, also under a wrapper module
        if any(("." + pre + ".") in dotted for pre in prefixes) and p.requires_grad:
            p.requires_grad_(False)
            n += p.numel()
    return n


def init_from_env(backend: str = "nccl") -> tuple:
    """(world, rank, local_rank, device) from torchrun's environment; initialises the process group if world > 1."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "nccl":
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local if world > 1 else 0)
        device = torch.device("cuda", local if world > 1 else 0)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            dist.init_process_group(backend, device_id=device)
        else:
            dist.init_process_group(backend)
    return world, rank, local, device


def make_data_parallel(model: torch.nn.Module, device: torch.device, bucket_cap_mb: int = 25):
    """Wrap for DP (no-op at world size 1). Bucket size: ~25 MB keeps two buckets of the ~50 MB
    fp32 gradient in flight behind backward, large enough for xGMI ring bandwidth."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return model
    freeze_unused(model)
    ids = [device.index] if device.type == "cuda" else None
    return torch.nn.parallel.DistributedDataParallel(model, device_ids=ids, bucket_cap_mb=bucket_cap_mb,
                                                     broadcast_buffers=False, gradient_as_bucket_view=True)


def broadcast_state(model: torch.nn.Module, src: int = 0) -> None:
    """Parameters and buffers of rank `src` on every rank (what DDP does at construction)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    with torch.no_grad():
        for t in list(model.parameters()) + list(model.buffers()):
            dist.broadcast(t.data, src)


def max_over_ranks(value: float, device: torch.device) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return value
    t = torch.tensor([value], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
