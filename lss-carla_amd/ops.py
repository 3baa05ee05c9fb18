"""Host orchestration of the HIP hot path: geometry, CSR, fused lift+splat autograd.

Every function here takes device tensors, launches on the current HIP stream
of that device, never synchronises with the host (except camera_inverses, which
mirrors the reference's ``torch.inverse(x.cpu())`` exactly, when the rig carries no
host copy) and never falls back to another implementation.

Reference boundary replaced (shdragron/LSS-Carla):
  get_geometry            src/models.py:170-190
  get_depth_dist/feat     src/models.py:49-61  (lift; fused into the splat)
  get_cam_feats layout    src/models.py:192-202
  voxel_pooling           src/models.py:204-246
  QuickCumsum fwd/bwd     src/tools.py:193-219
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib

C_CAM = 64  # camC, src/models.py:148


# ----------------------------------------------------------------------------- grid
@dataclass(frozen=True)
class GridSpec:
    """Voxel grid of a grid_conf (``gen_dx_bx``, src/tools.py:174-179; lo = bx - dx/2, src/models.py:212)."""
    lo: Tuple[float, float, float]
    dx: Tuple[float, float, float]
    nx: Tuple[int, int, int]  # X, Y, Z

    @staticmethod
    def from_conf(grid_conf: dict) -> "GridSpec":
        rows = (grid_conf["xbound"], grid_conf["ybound"], grid_conf["zbound"])
        dx = np.array([r[2] for r in rows], dtype=np.float32)
        bx = np.array([r[0] + r[2] / 2.0 for r in rows], dtype=np.float32)
        nx = tuple(int((r[1] - r[0]) / r[2]) for r in rows)
        lo = (bx - dx / np.float32(2.0)).astype(np.float32)
        return GridSpec(tuple(float(v) for v in lo), tuple(float(v) for v in dx), nx)

    def c_struct(self) -> _lib.Grid:
        g = _lib.Grid()
        for i in range(3):
            g.lo[i] = self.lo[i]
            g.dx[i] = self.dx[i]
            g.nx[i] = self.nx[i]
        return g

    def ncells(self, B: int) -> int:
        X, Y, Z = self.nx
        return B * Z * X * Y


def make_dims(B: int, N: int, D: int, H: int, W: int) -> _lib.Dims:
    return _lib.Dims(B, N, D, H, W, C_CAM)


def _require_cuda(*ts: Optional[torch.Tensor]) -> torch.device:
    dev = None
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("lss_carla_amd: the hot path runs only on MI355X (HIP) tensors; "
                               f"got a {t.device} tensor. There is no CPU fallback.")
        dev = t.device if dev is None else dev
    return dev


def _f32c(t: torch.Tensor) -> torch.Tensor:
    return t.detach().to(torch.float32).contiguous()


# ----------------------------------------------------------------------------- cameras
def camera_inverses(post_rots: torch.Tensor, intrins: torch.Tensor):
    """inv(post_rots), inv(intrins) as (B*N, 9) fp32 device tensors: torch.inverse on the CPU, exactly as
    src/models.py:180,186 (one D2H + H2D copy; no D2H copy when the device tensors carry their host
    copies, ``t._lss_host``, as simbev.finish_batch attaches them: then nothing synchronises the host).
    """
    dev = _require_cuda(post_rots, intrins)
    ncam = post_rots.shape[0] * post_rots.shape[1]

    def host_copy(t):
        # the attached host copy only while the device tensor is unchanged since it was attached
        # (an in-place copy_ into a reused batch buffer bumps _version: then read the device tensor)
        h = getattr(t, "_lss_host", None)
        if (h is not None and tuple(h.shape) == tuple(t.shape) and not h.is_cuda
                and getattr(t, "_lss_host_version", None) == t._version):
            return h
        return t.detach().cpu()
    pinv = torch.inverse(host_copy(post_rots).float()).reshape(ncam, 9).pin_memory()
    kinv = torch.inverse(host_copy(intrins).float()).reshape(ncam, 9).pin_memory()
    return pinv.to(dev, non_blocking=True), kinv.to(dev, non_blocking=True)


class HostInverses:
    """Host ``torch.inverse`` results (src/models.py:180,186, bit for bit) in static device buffers.

    ``inverse='host'`` is a device->host->device round trip inside the forward, which a captured
    (hipGraph) step cannot contain. In training the rig arrives on the host anyway (the loader
    builds it there), so ``update(post_rots, intrins)`` inverts the host copy with the reference's
    own call and stages the result through pinned memory into ``pinv`` / ``kinv``, on the current
    stream, before the step is launched; ``LiftSplatShoot.static_inverses = (pinv, kinv)`` makes
    the forward read them. Two pinned staging buffers alternate; a buffer is rewritten only after
    the copy that last read it has executed (the host never runs more than two steps ahead).
    """

    def __init__(self, n_cams: int, device: torch.device):
        self.pinv = torch.empty(n_cams, 9, device=device, dtype=torch.float32)
        self.kinv = torch.empty(n_cams, 9, device=device, dtype=torch.float32)
        self._host = [torch.empty(2, n_cams, 9, dtype=torch.float32).pin_memory() for _ in range(2)]
        self._done = [None, None]
        self._i = 0
        self.n_cams = n_cams

    def update(self, post_rots: torch.Tensor, intrins: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        if post_rots.is_cuda or intrins.is_cuda:
            raise RuntimeError("HostInverses.update takes the host copies of post_rots / intrins")
        i = self._i
        self._i ^= 1
        if self._done[i] is not None:
            self._done[i].synchronize()
        h = self._host[i]
        h[0].copy_(torch.inverse(post_rots.float()).reshape(self.n_cams, 9))
        h[1].copy_(torch.inverse(intrins.float()).reshape(self.n_cams, 9))
        self.pinv.copy_(h[0], non_blocking=True)
        self.kinv.copy_(h[1], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.pinv.device))
        self._done[i] = ev
        return self.pinv, self.kinv


# ----------------------------------------------------------------------------- plan
@dataclass
class SplatPlan:
    """Per-forward voxel assignment: cell of every point and the CSR of points by cell."""
    dims: Tuple[int, int, int, int, int]  # B, N, D, H, W
    grid: GridSpec
    cell_of: torch.Tensor      # (Nprime,) int32, -1 = dropped
    cell_start: Optional[torch.Tensor]  # (ncells+1,) int32 (None: geometry only, want_csr=False)
    sorted_key: Optional[torch.Tensor]  # (Nprime,) int64 (cell << 32 | point): ascending cell, then point
                               # id; key -1 past the first cell_start[-1] entries
    sorted_row: Optional[torch.Tensor]  # (Nprime,) int32 context row (pixel) of each sorted entry
    geom: Optional[torch.Tensor] = None

    @property
    def c_dims(self) -> _lib.Dims:
        return make_dims(*self.dims)

    @property
    def nprime(self) -> int:
        B, N, D, H, W = self.dims
        return B * N * D * H * W

    def tensors(self):
        return [t for t in (self.cell_of, self.cell_start, self.sorted_key, self.sorted_row, self.geom)
                if t is not None]


class PlanWs:
    """Persistent state of the plans of one shape on one device (lss_csr_build_ws): the cell counts,
    the single-pass scan's workspace (zero-filled once here and left zero-filled by every
    lss_csr_build_ws, so a plan needs no count memset and no scan reset) and the counting sort's
    scratch. The C ABI allows one plan at a time per workspace; the order between plans on different
    streams is kept here: every eager plan records an event on its stream after its CSR build, and a
    plan on another stream first waits for that event. A captured plan (hipGraph) records nothing:
    torch.cuda.graph synchronises the device before capturing, and the graph's replays must be
    ordered with other plans of the shape on that device (TrainStep replays and eager steps run on
    one stream)."""

    def __init__(self, dev: torch.device, ncells: int, nprime: int):
        lib = _lib.load()
        self.counts = torch.zeros(ncells, device=dev, dtype=torch.int32)
        self.workspace = torch.zeros(int(lib.lss_csr_workspace_bytes(ncells)), device=dev, dtype=torch.uint8)
        self.scratch = torch.empty(int(lib.lss_csr_scratch_bytes(ncells, nprime)), device=dev, dtype=torch.uint8)
        # ordered plans' per-cell block records (no initialisation needed)
        self.lists = torch.empty(int(lib.lss_csr_lists_bytes(ncells, nprime)), device=dev, dtype=torch.uint8)
        self.last_stream = None
        self.last_event = None

    def __iter__(self):  # (counts, workspace, scratch)
        return iter((self.counts, self.workspace, self.scratch))

    def acquire(self, dev: torch.device, capturing: bool) -> None:
        if capturing or self.last_event is None:
            return
        cur = torch.cuda.current_stream(dev)
        if cur != self.last_stream:
            cur.wait_event(self.last_event)

    def release(self, dev: torch.device, capturing: bool) -> None:
        if capturing:
            return
        cur = torch.cuda.current_stream(dev)
        ev = torch.cuda.Event()
        ev.record(cur)
        self.last_stream, self.last_event = cur, ev

    def restore(self) -> None:
        """After a failed plan: counts and scan state back to zeros (on the current stream)."""
        self.counts.zero_()
        self.workspace.zero_()


class _PlanWorkspace:
    """PlanWs per (device, ncells, nprime). Created outside graph capture (the eager warm-up
    steps); a plan captured before its workspace exists takes the stateless path."""

    def __init__(self):
        self._ws = {}

    def get(self, dev: torch.device, ncells: int, nprime: int, create: bool) -> Optional[PlanWs]:
        key = (dev.index, ncells, nprime)
        w = self._ws.get(key)
        if w is None and create:
            w = PlanWs(dev, ncells, nprime)
            self._ws[key] = w
        return w

    def clear(self):
        self._ws.clear()


PLAN_WS = _PlanWorkspace()
USE_PLAN_WS = True  # False: a count memset + lss_csr_build (two-kernel scan) per plan
# with a persistent workspace: ordered plans (lss_geometry_cells_ordered + lss_csr_build_ordered, three
# kernels, every point written at its canonical position) instead of lss_geometry_cells +
# lss_csr_build_ws (four kernels: arrival-order slots, then k_csr_canon sorts each cell)
USE_PLAN_ORDERED = True
_ORD_MAX_SAMPLE_POINTS = (1 << 20) - 512  # lss_geometry_cells_ordered's limit (points per sample)


def _ordered(ws, points_per_sample: int) -> bool:
    return ws is not None and USE_PLAN_ORDERED and points_per_sample < _ORD_MAX_SAMPLE_POINTS


def _plan_counts(dev: torch.device, ncells: int, nprime: int):
    """(counts, PlanWs) for one plan: the persistent zero-filled state (acquired: ordered after its
    last user), or fresh zeros and None."""
    if USE_PLAN_WS:
        capturing = dev.type == "cuda" and torch.cuda.is_current_stream_capturing()
        w = PLAN_WS.get(dev, ncells, nprime, create=not capturing)
        if w is not None:
            w.acquire(dev, capturing)
            return w.counts, w
    return torch.zeros(ncells, device=dev, dtype=torch.int32), None


def _counted_plan(dev: torch.device, ws: Optional[PlanWs], launch_cells, build_csr):
    """launch_cells() counts into the plan's cell counts, build_csr() turns them into the CSR. With a
    persistent workspace, a failure anywhere in between restores its zero-filled state (the counts
    may already hold this plan's points), and success records its last use."""
    if ws is None:
        launch_cells()
        return build_csr()
    capturing = dev.type == "cuda" and torch.cuda.is_current_stream_capturing()
    try:
        launch_cells()
        out = build_csr()
    except Exception:
        if not capturing:
            ws.restore()
        raise
    ws.release(dev, capturing)
    return out


def _build_csr(cell_of, slot_of, counts, dims, ncells: int, dev, ws=None, ordered=False):
    """Counting sort into the canonical CSR (lss_csr_build[_ws|_ordered]): cell_start, sorted_key,
    sorted_row."""
    lib = _lib.load()
    B, N, D, H, W = dims
    nprime = B * N * D * H * W
    cell_start = torch.empty(ncells + 1, device=dev, dtype=torch.int32)
    sorted_key = torch.empty(nprime, device=dev, dtype=torch.int64)
    sorted_row = torch.empty(nprime, device=dev, dtype=torch.int32)
    if ordered:
        _lib.check(lib.lss_csr_build_ordered(_lib.ptr(cell_of), _lib.ptr(slot_of), nprime, _lib.ptr(counts), ncells,
                                             make_dims(*dims), _lib.ptr(ws.lists), _lib.ptr(cell_start),
                                             _lib.ptr(sorted_key), _lib.ptr(sorted_row), _lib.ptr(ws.workspace),
                                             _lib.stream_handle(dev)), "lss_csr_build_ordered")
        return cell_start, sorted_key, sorted_row
    if ws is not None:
        _lib.check(lib.lss_csr_build_ws(_lib.ptr(cell_of), _lib.ptr(slot_of), nprime, _lib.ptr(counts), ncells,
                                        make_dims(*dims), _lib.ptr(cell_start), _lib.ptr(sorted_key),
                                        _lib.ptr(sorted_row), _lib.ptr(ws.scratch), _lib.ptr(ws.workspace),
                                        _lib.stream_handle(dev)), "lss_csr_build_ws")
        return cell_start, sorted_key, sorted_row
    scratch = torch.empty(int(lib.lss_csr_scratch_bytes(ncells, nprime)), device=dev, dtype=torch.uint8)
    _lib.check(lib.lss_csr_build(_lib.ptr(cell_of), _lib.ptr(slot_of), nprime, _lib.ptr(counts), ncells,
                                 make_dims(*dims), _lib.ptr(cell_start), _lib.ptr(sorted_key), _lib.ptr(sorted_row),
                                 _lib.ptr(scratch), _lib.stream_handle(dev)), "lss_csr_build")
    return cell_start, sorted_key, sorted_row


def plan_from_cameras(frustum: torch.Tensor, rots, trans, intrins, post_rots, post_trans, grid: GridSpec,
                      want_geom: bool = False, want_csr: bool = True,
                      inverses: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> SplatPlan:
    """get_geometry + quantise + filter + counting sort, all on the device (src/models.py:170-231).

    `inverses` = a (pinv, kinv) pair from camera_inverses / HostInverses, if already computed
    (models.py computes them before the trunk, so the host round trip never waits for device work).
    """
    dev = _require_cuda(frustum, rots, trans, intrins, post_rots, post_trans)
    lib = _lib.load()
    B, N = trans.shape[:2]
    D, H, W = frustum.shape[:3]
    nprime = B * N * D * H * W
    ncells = grid.ncells(B)
    pinv, kinv = inverses if inverses is not None else camera_inverses(post_rots, intrins)
    fr, ro, tr, pt = _f32c(frustum), _f32c(rots), _f32c(trans), _f32c(post_trans)
    cell_of = torch.empty(nprime, device=dev, dtype=torch.int32)
    geom = torch.empty(B, N, D, H, W, 3, device=dev, dtype=torch.float32) if want_geom else None
    counts = slot_of = ws = None
    if want_csr:
        counts, ws = _plan_counts(dev, ncells, nprime)
        slot_of = torch.empty(nprime, device=dev, dtype=torch.int32)
    dims = make_dims(B, N, D, H, W)
    g = grid.c_struct()
    ordered = want_csr and _ordered(ws, N * D * H * W)

    def launch_cells():
        if ordered:
            _lib.check(lib.lss_geometry_cells_ordered(
                _lib.ptr(fr), _lib.ptr(ro), _lib.ptr(tr), _lib.ptr(kinv), _lib.ptr(pinv), _lib.ptr(pt), dims, g,
                _lib.ptr(geom), _lib.ptr(cell_of), _lib.ptr(counts), _lib.ptr(slot_of), _lib.ptr(ws.lists),
                _lib.ptr(ws.workspace), _lib.stream_handle(dev)), "lss_geometry_cells_ordered")
            return
        _lib.check(lib.lss_geometry_cells(_lib.ptr(fr), _lib.ptr(ro), _lib.ptr(tr), _lib.ptr(kinv), _lib.ptr(pinv),
                                          _lib.ptr(pt), dims, g, _lib.ptr(geom), _lib.ptr(cell_of), _lib.ptr(counts),
                                          _lib.ptr(slot_of), _lib.stream_handle(dev)), "lss_geometry_cells")

    if not want_csr:
        launch_cells()
        return SplatPlan((B, N, D, H, W), grid, cell_of, None, None, None, geom)
    cell_start, sorted_key, sorted_row = _counted_plan(
        dev, ws, launch_cells,
        lambda: _build_csr(cell_of, slot_of, counts, (B, N, D, H, W), ncells, dev, ws, ordered))
    return SplatPlan((B, N, D, H, W), grid, cell_of, cell_start, sorted_key, sorted_row, geom)


def plan_from_geom(geom: torch.Tensor, grid: GridSpec) -> SplatPlan:
    """Quantise a given (B, N, D, H, W, 3) geometry (voxel_pooling(geom_feats, x) boundary)."""
    dev = _require_cuda(geom)
    lib = _lib.load()
    B, N, D, H, W, _ = geom.shape
    nprime = B * N * D * H * W
    ncells = grid.ncells(B)
    gm = _f32c(geom)
    cell_of = torch.empty(nprime, device=dev, dtype=torch.int32)
    counts, ws = _plan_counts(dev, ncells, nprime)
    slot_of = torch.empty(nprime, device=dev, dtype=torch.int32)
    ordered = _ordered(ws, nprime // B)

    def launch_cells():
        if ordered:
            _lib.check(lib.lss_cells_from_geom_ordered(_lib.ptr(gm), nprime, nprime // B, grid.c_struct(),
                                                       _lib.ptr(cell_of), _lib.ptr(counts), _lib.ptr(slot_of),
                                                       _lib.ptr(ws.lists), _lib.ptr(ws.workspace),
                                                       _lib.stream_handle(dev)), "lss_cells_from_geom_ordered")
            return
        _lib.check(lib.lss_cells_from_geom(_lib.ptr(gm), nprime, nprime // B, grid.c_struct(), _lib.ptr(cell_of),
                                           _lib.ptr(counts), _lib.ptr(slot_of), _lib.stream_handle(dev)),
                   "lss_cells_from_geom")

    cell_start, sorted_key, sorted_row = _counted_plan(
        dev, ws, launch_cells,
        lambda: _build_csr(cell_of, slot_of, counts, (B, N, D, H, W), ncells, dev, ws, ordered))
    return SplatPlan((B, N, D, H, W), grid, cell_of, cell_start, sorted_key, sorted_row, None)


# ----------------------------------------------------------------------------- profiling hook
class _SplatProfile:
    """Opt-in timing of every lss_splat_fwd launch (used by bench.py).

    The ABI stamps a pair of hipEvents with the kernel's own start/end (hipExtLaunchKernel), so
    the average is kernel time only -- the same quantity rocprofv3 --kernel-trace reports.
    """

    def __init__(self):
        self.enabled = False
        self.pairs = []

    def reset(self, enabled: bool = True):
        self.release()
        self.enabled = enabled

    def new_pair(self):
        lib = _lib.load()
        a, b = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.check(lib.lss_event_create(ctypes.byref(a)), "lss_event_create")
        _lib.check(lib.lss_event_create(ctypes.byref(b)), "lss_event_create")
        self.pairs.append((a, b))
        return a, b

    def avg_ms(self) -> Optional[float]:
        if not self.pairs:
            return None
        lib = _lib.load()
        tot = 0.0
        for a, b in self.pairs:
            ms = ctypes.c_float()
            _lib.check(lib.lss_event_elapsed_ms(a, b, ctypes.byref(ms)), "lss_event_elapsed_ms")
            tot += ms.value
        return tot / len(self.pairs)

    def release(self):
        if self.pairs:
            lib = _lib.load()
            for a, b in self.pairs:
                lib.lss_event_destroy(a)
                lib.lss_event_destroy(b)
        self.pairs = []


SPLAT_PROFILE = _SplatProfile()


def _new_bev(B, Z, X, Y, dtype, layout, dev) -> torch.Tensor:
    if layout == _lib.NHWC:
        return torch.empty(B, Z * C_CAM, X, Y, device=dev, dtype=dtype, memory_format=torch.channels_last)
    return torch.empty(B, Z * C_CAM, X, Y, device=dev, dtype=dtype)


def _splat_fwd_launch(plan: SplatPlan, depth, ctx_t, x_rows, out: torch.Tensor, layout: int):
    lib = _lib.load()
    dev = out.device
    e0, e1 = SPLAT_PROFILE.new_pair() if SPLAT_PROFILE.enabled else (None, None)
    ctx_code = _lib.dtype_code(ctx_t.dtype) if ctx_t is not None else _lib.F32
    _lib.check(lib.lss_splat_fwd(_lib.ptr(depth), _lib.ptr(ctx_t), ctx_code, _lib.ptr(x_rows), _lib.ptr(plan.cell_start),
                                 _lib.ptr(plan.sorted_key), _lib.ptr(plan.sorted_row), plan.c_dims,
                                 plan.grid.c_struct(), _lib.ptr(out), _lib.dtype_code(out.dtype), layout,
                                 _lib.stream_handle(dev), e0, e1), "lss_splat_fwd")


def _grad_rows(plan: SplatPlan, dbev: torch.Tensor) -> Tuple[torch.Tensor, int]:
    """Gradient rows of the occupied cells: the channels-last dbev itself, or compacted from NCHW."""
    if dbev.dtype not in (torch.float32, torch.bfloat16):
        dbev = dbev.float()
    if dbev.dim() == 4 and dbev.is_contiguous(memory_format=torch.channels_last) and not dbev.is_contiguous():
        return dbev, _lib.NHWC
    dbev = dbev.contiguous()
    lib = _lib.load()
    B = plan.dims[0]
    rows = torch.empty(plan.grid.ncells(B) * C_CAM, device=dbev.device, dtype=dbev.dtype)
    _lib.check(lib.lss_bev_rows(_lib.ptr(dbev), _lib.dtype_code(dbev.dtype), _lib.ptr(plan.cell_start),
                                plan.c_dims, plan.grid.c_struct(), _lib.ptr(rows), _lib.stream_handle(dbev.device)),
               "lss_bev_rows")
    return rows, _lib.NCHW


# ----------------------------------------------------------------------------- autograd: fused lift + splat
class LiftSplat(torch.autograd.Function):
    """depthnet output (B*N, D+C, H, W) -> BEV (B, Z*C, X, Y).

    Forward = softmax over depth bins, outer product with the context features
    and voxel pooling (src/models.py:49-61, 192-246), without materialising the
    (B*N, C, D, H, W) lifted volume. Backward = QuickCumsum's gather
    (src/tools.py:212-219) fused with the outer-product and softmax backward.
    """

    @staticmethod
    def forward(ctx, depthnet_out: torch.Tensor, plan: SplatPlan, out_dtype: torch.dtype, layout: int):
        dev = _require_cuda(depthnet_out)
        lib = _lib.load()
        B, N, D, H, W = plan.dims
        if depthnet_out.shape != (B * N, D + C_CAM, H, W):
            raise RuntimeError(f"depthnet output shape {tuple(depthnet_out.shape)} != {(B * N, D + C_CAM, H, W)}")
        dn = depthnet_out.detach()
        if dn.dtype not in (torch.float32, torch.bfloat16):
            dn = dn.float()
        dn = dn.contiguous()
        depth = torch.empty(B * N, D, H, W, device=dev, dtype=torch.float32)
        # context rows keep the input's element type: bf16 rows are exact for a bf16 depthnet output
        # and halve the splat's gathered bytes
        ctx_t = torch.empty(B * N * H * W, C_CAM, device=dev, dtype=dn.dtype)
        X, Y, Z = plan.grid.nx
        out = _new_bev(B, Z, X, Y, out_dtype, layout, dev)
        _lib.check(lib.lss_lift_prep(_lib.ptr(dn), _lib.dtype_code(dn.dtype), plan.c_dims, _lib.ptr(depth),
                                     _lib.ptr(ctx_t), _lib.dtype_code(ctx_t.dtype), _lib.stream_handle(dev)),
                   "lss_lift_prep")
        _splat_fwd_launch(plan, depth, ctx_t, None, out, layout)
        ctx.save_for_backward(depth, ctx_t)
        ctx.plan = plan
        ctx.dn_dtype = depthnet_out.dtype
        return out

    @staticmethod
    def backward(ctx, dbev: torch.Tensor):
        depth, ctx_t = ctx.saved_tensors
        plan: SplatPlan = ctx.plan
        lib = _lib.load()
        rows, layout = _grad_rows(plan, dbev)
        B, N, D, H, W = plan.dims
        d_dn = torch.empty(B * N, D + C_CAM, H, W, device=depth.device, dtype=ctx.dn_dtype)
        _lib.check(lib.lss_splat_bwd(_lib.ptr(rows), _lib.dtype_code(rows.dtype), layout, _lib.ptr(plan.cell_of),
                                     _lib.ptr(depth), _lib.ptr(ctx_t), _lib.dtype_code(ctx_t.dtype), plan.c_dims,
                                     plan.grid.c_struct(),
                                     _lib.ptr(d_dn), _lib.dtype_code(d_dn.dtype), _lib.stream_handle(depth.device)),
                   "lss_splat_bwd")
        return d_dn, None, None, None


def lift_splat(depthnet_out: torch.Tensor, plan: SplatPlan, out_dtype: torch.dtype = torch.float32,
               layout: int = _lib.NCHW) -> torch.Tensor:
    return LiftSplat.apply(depthnet_out, plan, out_dtype, layout)


def _wgrad_splits(npix: int) -> int:
    """Slices of the pixel (reduction) axis for the depthnet weight gradient's batched GEMM: up to 16,
    each a whole number of pixels."""
    for s in (16, 8, 4, 2):
        if npix % s == 0 and npix // s >= 256:
            return s
    return 1


# ----------------------------------------------------------------------------- autograd: depthnet + lift + splat
class DepthnetLiftSplat(torch.autograd.Function):
    """depthnet(feat) -> lift -> splat in two kernels: lss_depthnet_lift (the 1x1 conv on MFMA fused
    with the depth softmax and the context-row layout, src/models.py:47, 55-59) and lss_splat_fwd.
    The (B*N, D+C, H, W) depthnet output is never materialised in the forward.

    bf16 only (the autocast training path): under autocast the operands are rounded to bf16 as the
    reference's ``nn.Conv2d`` would see them -- the features by a cast, the weight and bias by
    lss_depthnet_pack on the channels-last path (one launch: the lift kernel's fragment order, the
    plain bf16 weight for the backward and the bf16 bias), by casts otherwise. Backward:
    lss_splat_bwd gives d(logits); the conv's own backward turns it into d(feat), d(weight), d(bias).
    """

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda")
    def forward(ctx, feat: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, plan: SplatPlan,
                out_dtype: torch.dtype, layout: int, packed: Optional[torch.Tensor] = None):
        dev = _require_cuda(feat, weight, bias)
        lib = _lib.load()
        B, N, D, H, W = plan.dims
        O, K = weight.shape[0], weight.shape[1]
        bf = torch.bfloat16
        if torch.is_autocast_enabled("cuda"):
            feat = feat.to(bf)
        elif feat.dtype != bf or weight.dtype != bf or bias.dtype != bf:
            raise RuntimeError("lss_carla_amd: the fused depthnet path is bf16 (run it under torch.autocast)")
        if weight.dtype not in (torch.float32, bf) or bias.dtype != weight.dtype:
            raise RuntimeError(f"lss_carla_amd: depthnet weight / bias of dtype {weight.dtype} / {bias.dtype}")
        if feat.shape != (B * N, K, H, W) or O != D + C_CAM or tuple(weight.shape[2:]) != (1, 1):
            raise RuntimeError(f"depthnet shapes feat {tuple(feat.shape)} weight {tuple(weight.shape)} do not match "
                               f"the plan (B*N={B * N}, D+C={D + C_CAM}, H={H}, W={W})")
        # a channels-last feature map (pixel-major rows, as CamEncode's channels-last up1 gives it) goes
        # to the pixel-row kernel; anything else is made NCHW-contiguous for the channel-plane kernel
        # (k_depthnet_lift3 reads 16-B vectors of the rows: a view at an unaligned offset is copied)
        nhwc = K == 512 and feat.dim() == 4 and feat.is_contiguous(memory_format=torch.channels_last)
        f = feat.detach() if nhwc else feat.detach().contiguous()
        if f.data_ptr() % 16:
            f = f.clone(memory_format=torch.channels_last if nhwc else torch.contiguous_format)
        depth = torch.empty(B * N, D, H, W, device=dev, dtype=torch.float32)
        ctx_t = torch.empty(B * N * H * W, C_CAM, device=dev, dtype=bf)
        X, Y, Z = plan.grid.nx
        out = _new_bev(B, Z, X, Y, out_dtype, layout, dev)
        st = _lib.stream_handle(dev)
        if nhwc and packed is not None and weight.dtype == bf and bias.dtype == bf:
            # weights already in fragment order (flat_params: the same launch as their bf16 copy);
            # the kernel reads DN_PACKED_BYTES(K) from it, so a buffer of another size, type or device
            # is refused rather than read out of bounds
            if (packed.dtype != bf or packed.device != dev or not packed.is_contiguous()
                    or packed.numel() * 2 != _lib.DN_PACKED_BYTES(K) or packed.data_ptr() % 16):
                raise RuntimeError(f"lss_carla_amd: prepacked depthnet weight {packed.dtype} x {packed.numel()} on "
                                   f"{packed.device} does not match K={K} ({_lib.DN_PACKED_BYTES(K)} bytes, bf16, "
                                   f"16-B aligned, on {dev})")
            w, b = weight.detach().reshape(O, K), bias.detach()
        elif nhwc:
            packed = torch.empty(_lib.DN_PACKED_BYTES(K) // 2, device=dev, dtype=bf)
            w = torch.empty(O, K, device=dev, dtype=bf)
            b = torch.empty(O, device=dev, dtype=bf)
            _lib.check(lib.lss_depthnet_pack(_lib.ptr(weight.detach().reshape(O, K).contiguous()),
                                             _lib.ptr(bias.detach().contiguous()), _lib.dtype_code(weight.dtype),
                                             O, K, _lib.ptr(packed), _lib.ptr(w), _lib.ptr(b), st), "lss_depthnet_pack")
        if nhwc:
            _lib.check(lib.lss_depthnet_lift_nhwc_packed(_lib.ptr(f), _lib.ptr(packed), _lib.ptr(b), K, plan.c_dims,
                                                         _lib.ptr(depth), _lib.ptr(ctx_t), _lib.BF16, st),
                       "lss_depthnet_lift_nhwc_packed")
        else:
            w = weight.detach().to(bf).reshape(O, K).contiguous()
            b = bias.detach().to(bf).contiguous()
            _lib.check(lib.lss_depthnet_lift(_lib.ptr(f), _lib.ptr(w), _lib.ptr(b), _lib.BF16, K, plan.c_dims,
                                             _lib.ptr(depth), _lib.ptr(ctx_t), _lib.BF16, st), "lss_depthnet_lift")
        _splat_fwd_launch(plan, depth, ctx_t, None, out, layout)
        ctx.save_for_backward(f, w.view(weight.shape), depth, ctx_t)
        ctx.plan = plan
        return out

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dbev: torch.Tensor):
        feat, weight, depth, ctx_t = ctx.saved_tensors
        plan: SplatPlan = ctx.plan
        lib = _lib.load()
        rows, layout = _grad_rows(plan, dbev)
        B, N, D, H, W = plan.dims
        d_dn = torch.empty(B * N, D + C_CAM, H, W, device=depth.device, dtype=torch.bfloat16)
        _lib.check(lib.lss_splat_bwd(_lib.ptr(rows), _lib.dtype_code(rows.dtype), layout, _lib.ptr(plan.cell_of),
                                     _lib.ptr(depth), _lib.ptr(ctx_t), _lib.BF16, plan.c_dims, plan.grid.c_struct(),
                                     _lib.ptr(d_dn), _lib.BF16, _lib.stream_handle(depth.device)), "lss_splat_bwd")
        need = ctx.needs_input_grad
        if feat.dim() == 4 and feat.is_contiguous(memory_format=torch.channels_last) and not feat.is_contiguous():
            # channels-last features: the 1x1 conv's backward as plain GEMMs over pixel-major rows
            # (hipBLASLt). MIOpen's channels-last 1x1 backward-weights solver is not replay-safe in a
            # hipGraph (its weight gradient reads back as zeros from the first replay on).
            O, K = weight.shape[0], weight.shape[1]
            npix = B * N * H * W
            dd = d_dn.permute(0, 2, 3, 1).reshape(npix, O)          # (pixels, O), one copy
            fm = feat.permute(0, 2, 3, 1).reshape(npix, K)          # a view: the channels-last rows
            w2 = weight.reshape(O, K).to(dd.dtype)
            d_feat = d_w = d_b = None
            if need[0]:
                d_feat = torch.mm(dd, w2).view(B * N, H, W, K).permute(0, 3, 1, 2)  # channels-last
            if need[1]:
                # split-K as a batched GEMM: one (O x npix) x (npix x K) product gives hipBLASLt only
                # (O / 64) x (K / 64) = 16 tiles for 8,448-long dot products (76 us at c3); KSPLIT slices of
                # the pixels fill the chip, their partials kept in fp32 (bf16 partials would be rounded
                # before the sum, and pixel-gradient sums cancel) and summed in slice order
                S = _wgrad_splits(npix)
                part = _bmm_f32(dd.view(S, npix // S, O).transpose(1, 2), fm.view(S, npix // S, K))
                d_w = part.sum(0).view(weight.shape).to(weight.dtype)
            if need[2]:
                # per-channel sums straight from the NCHW d(logits) (torch's dim-0 reduction of the
                # pixel-major copy ran on 128 threads: 89 us at c3)
                d_b32 = torch.empty(O, device=d_dn.device, dtype=torch.float32)
                _lib.check(lib.lss_channel_sums(_lib.ptr(d_dn), _lib.BF16, B * N, O, H * W, _lib.ptr(d_b32),
                                                _lib.stream_handle(d_dn.device)), "lss_channel_sums")
                d_b = d_b32.to(weight.dtype)
            return d_feat, d_w, d_b, None, None, None, None
        d_feat, d_w, d_b = torch.ops.aten.convolution_backward(
            d_dn, feat, weight, [weight.shape[0]], [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
            [need[0], need[1], need[2]])
        return d_feat, d_w, d_b, None, None, None, None


_BMM_F32_OUT = {}


def _bmm_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """bf16 x bf16 batched GEMM with fp32 outputs (torch.bmm's out_dtype overload, one rounding per
    element); where this torch build lacks that overload for the device, an fp32 GEMM of the same
    bf16 values (exact products, fp32 sums). Probed once per device, outside any capture (the eager
    warm-up steps come first)."""
    dev = a.device
    ok = _BMM_F32_OUT.get(dev)
    if ok is None:
        try:
            t = torch.ones(1, 2, 2, device=dev, dtype=torch.bfloat16)
            ok = torch.bmm(t, t, out_dtype=torch.float32).dtype == torch.float32
        except (RuntimeError, TypeError, NotImplementedError):
            ok = False
        _BMM_F32_OUT[dev] = ok
    if ok:
        return torch.bmm(a, b, out_dtype=torch.float32)
    return torch.bmm(a.float(), b.float())


def depthnet_lift_splat(feat: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, plan: SplatPlan,
                        out_dtype: torch.dtype = torch.bfloat16, layout: int = _lib.NHWC,
                        packed: Optional[torch.Tensor] = None) -> torch.Tensor:
    """packed: the weight in lss_depthnet_pack's order, already written (flat_params.FlatParams);
    used only with a bf16 weight and bias."""
    return DepthnetLiftSplat.apply(feat, weight, bias, plan, out_dtype, layout, packed)


# ----------------------------------------------------------------------------- autograd: unfused voxel pooling
class VoxelPool(torch.autograd.Function):
    """(Nprime, C) lifted rows -> BEV (voxel_pooling(geom_feats, x) boundary, src/models.py:204-246)."""

    @staticmethod
    def forward(ctx, x_rows: torch.Tensor, plan: SplatPlan, layout: int):
        dev = _require_cuda(x_rows)
        xr = x_rows.detach().to(torch.float32).contiguous()
        X, Y, Z = plan.grid.nx
        out = _new_bev(plan.dims[0], Z, X, Y, torch.float32, layout, dev)
        _splat_fwd_launch(plan, None, None, xr, out, layout)
        ctx.plan = plan
        ctx.x_dtype = x_rows.dtype
        return out

    @staticmethod
    def backward(ctx, dbev: torch.Tensor):
        plan: SplatPlan = ctx.plan
        lib = _lib.load()
        rows, layout = _grad_rows(plan, dbev)
        dx = torch.empty(plan.nprime, C_CAM, device=rows.device, dtype=torch.float32)
        _lib.check(lib.lss_splat_bwd_lifted(_lib.ptr(rows), _lib.dtype_code(rows.dtype), layout,
                                            _lib.ptr(plan.cell_of), plan.nprime, plan.c_dims,
                                            plan.grid.c_struct(), _lib.ptr(dx), _lib.stream_handle(rows.device)),
                   "lss_splat_bwd_lifted")
        return dx.to(ctx.x_dtype), None, None


def voxel_pool_rows(x_rows: torch.Tensor, plan: SplatPlan, layout: int = _lib.NCHW) -> torch.Tensor:
    return VoxelPool.apply(x_rows, plan, layout)


# ----------------------------------------------------------------------------- op-level boundary: runs of ranks
def _f32_rows(t: torch.Tensor) -> torch.Tensor:
    """Contiguous fp32 copy/view with a 16-B aligned base (the gather's vector loads need it)."""
    t = t.detach().to(torch.float32).contiguous()
    return t if t.data_ptr() % 16 == 0 else t.clone()


def segment_runs(ranks: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, int]:
    """(seg_of, seg_start, nseg) of a sorted int64 rank vector (lss_segment_build).

    The number of runs sizes the outputs of QuickCumsum, so it is read back to the host -- the same
    synchronisation as the reference's boolean-mask indexing ``x[kept]`` (src/tools.py:200).
    """
    dev = _require_cuda(ranks)
    lib = _lib.load()
    r = ranks.detach()
    if r.dtype != torch.int64:
        r = r.to(torch.int64)
    r = r.contiguous()
    n = r.numel()
    seg_of = torch.empty(n, device=dev, dtype=torch.int32)
    seg_start = torch.empty(n + 1, device=dev, dtype=torch.int32)
    nseg = torch.empty(1, device=dev, dtype=torch.int32)
    scratch = torch.empty(int(lib.lss_segment_scratch_bytes(n)), device=dev, dtype=torch.uint8)
    _lib.check(lib.lss_segment_build(_lib.ptr(r), n, _lib.ptr(seg_of), _lib.ptr(seg_start), _lib.ptr(nseg),
                                     _lib.ptr(scratch), _lib.stream_handle(dev)), "lss_segment_build")
    return seg_of, seg_start, int(nseg.item())


def segment_sum(x: torch.Tensor, seg_start: torch.Tensor, nseg: int,
                keys: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Per-run row sums (nseg, C) fp32 and the keys row of each run's last row (lss_segment_sum)."""
    dev = _require_cuda(x, seg_start, keys)
    lib = _lib.load()
    xr = _f32_rows(x)
    C = xr.shape[1]
    out = torch.empty(nseg, C, device=dev, dtype=torch.float32)
    key_out = None
    kp = None
    kw = 0
    if keys is not None:
        if keys.dtype != torch.int64 or keys.dim() != 2:
            raise RuntimeError(f"lss_carla_amd: keys (geom_feats) must be a 2-D int64 tensor, got {keys.dtype} "
                               f"{tuple(keys.shape)}")
        kp = keys.detach().contiguous()
        kw = kp.shape[1]
        key_out = torch.empty(nseg, kw, device=dev, dtype=torch.int64)
    _lib.check(lib.lss_segment_sum(_lib.ptr(xr), C, _lib.ptr(seg_start), nseg, _lib.ptr(kp), kw, _lib.ptr(key_out),
                                   _lib.ptr(out), _lib.stream_handle(dev)), "lss_segment_sum")
    return out, key_out


def segment_gather(g: torch.Tensor, seg_of: torch.Tensor) -> torch.Tensor:
    """dx[i] = g[seg_of[i]] (lss_segment_gather): QuickCumsum's backward."""
    dev = _require_cuda(g, seg_of)
    lib = _lib.load()
    gr = _f32_rows(g)
    n, C = seg_of.numel(), gr.shape[1]
    dx = torch.empty(n, C, device=dev, dtype=torch.float32)
    _lib.check(lib.lss_segment_gather(_lib.ptr(gr), C, _lib.ptr(seg_of), n, _lib.ptr(dx), _lib.stream_handle(dev)),
               "lss_segment_gather")
    return dx
