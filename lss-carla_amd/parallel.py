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


# ----------------------------------------------------------------------------- one-shot N > 1 safety
# The driver's multi-GPU bench runs once, unattended: every decision that could send ranks down
# different paths (a graph capture that raised on one rank only) is taken collectively, over a
# host-side gloo group that does not depend on the state of the RCCL communicator, and the replicas
# are checked bit for bit after the untimed replays (train_simbev.py:245-248 is the update they must
# agree on).
_CONTROL = None


def control_group():
    """A gloo group over all ranks for host-side decisions; created collectively on first use (every
    rank must call it at the same point). The world group itself when that is already gloo."""
    global _CONTROL
    if not (dist.is_available() and dist.is_initialized()):
        return None
    if _CONTROL is None:
        _CONTROL = dist.group.WORLD if dist.get_backend() == "gloo" else dist.new_group(backend="gloo")
    return _CONTROL


def all_ranks_ok(ok: bool) -> bool:
    """True iff `ok` holds on every rank (MIN over the control group); `ok` itself at world size 1."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return bool(ok)
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=control_group())
    return bool(t.item())


def replica_checksums(tensors) -> torch.Tensor:
    """(n, 2) int64 per tensor: the sum of its elements' bit patterns and a position-weighted sum of
    them (weights 1..65521), wrapped mod 2^64 -- equal on two replicas iff (with overwhelming
    probability) the tensors are bit-identical. Computed where the tensors live; returned on the CPU."""
    rows = []
    for t in tensors:
        flat = t.detach().contiguous().reshape(-1)
        int_dt = {4: torch.int32, 2: torch.int16, 8: torch.int64}.get(flat.element_size())
        bits = (flat.view(int_dt) if int_dt is not None else flat.view(torch.uint8)).to(torch.int64)
        w = torch.arange(bits.numel(), device=bits.device, dtype=torch.int64) % 65521 + 1
        rows.append(torch.stack([bits.sum(), (bits * w).sum()]))
    return torch.stack(rows).cpu() if rows else torch.zeros(0, 2, dtype=torch.int64)


def replicas_in_sync(tensors) -> bool:
    """True iff every rank holds bit-identical `tensors` (e.g. the masters after an update): the
    checksums of all ranks gathered over the control group and compared with rank 0's."""
    c = replica_checksums(tensors)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return True
    allc = [torch.empty_like(c) for _ in range(dist.get_world_size())]
    dist.all_gather(allc, c, group=control_group())
    return all(torch.equal(x, allc[0]) for x in allc)


def capture_collectively(step, warmup: int, fallback=None, on_warmup=None, fail: bool = False):
    """Capture `step` (train_step.TrainStep or anything with .capture(warmup, on_warmup)) on every
    rank, or on none: each rank's success is agreed over the control group before any replay, so a
    capture that raised on one rank sends EVERY rank to `fallback()` (a factory of the step to use
    instead, captured here with 2 warm-up steps). The fallback's capture is voted on the same way;
    if it fails on any rank, every rank raises (no rank replays while another has given up).
    Returns (step, reason) -- reason None when `step` itself was captured everywhere, else why the
    fallback was taken. fail: force this rank's capture to raise (tests of the decision).

    Not covered by the vote: a rank that hangs (rather than raises) inside the eager warm-up steps,
    whose collectives the other ranks then wait on -- that case ends by the bench's watchdog."""
    err = None
    try:
        if fail:
            raise RuntimeError("capture failure forced on this rank")
        step.capture(warmup=warmup, on_warmup=on_warmup)
    except Exception as e:  # any failure must reach the vote, or the peers block in it
        err = e
    if all_ranks_ok(err is None):
        return step, None
    if fallback is None:
        raise RuntimeError(f"graph capture failed on {'this' if err else 'another'} rank") from err
    reason = f"this rank's capture raised: {err}" if err is not None else "another rank's capture raised"
    return recapture_collectively(fallback, reason), reason


def recapture_collectively(factory, why: str = ""):
    """factory() captured with 2 warm-up steps on every rank, agreed over the control group: returns
    the captured step, or raises on EVERY rank if the capture raised on any."""
    new, err = None, None
    try:
        new = factory()
        new.capture(warmup=2)
    except Exception as e:
        err = e
    if not all_ranks_ok(err is None):
        raise RuntimeError(f"fallback capture failed on {'this' if err else 'another'} rank"
                           + (f" ({why})" if why else "")) from err
    return new


def max_over_ranks(value: float, device: torch.device) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return value
    t = torch.tensor([value], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
