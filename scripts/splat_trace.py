"""Per-wave timeline of the channels-last splat from a LSS_TRACE=1 build (diagnostics only).

  python scripts/splat_trace.py --build [--lib NAME] [-D KNOB=V ...]   # here: builds variants/NAME.so
  python scripts/splat_trace.py [--lib NAME]               # GPU box: step-mode launch, prints the timeline
"""
import argparse
import ctypes as ct
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("-D", action="append", default=[])
    ap.add_argument("--mode", default="step", choices=["warm", "step"])
    ap.add_argument("--lib", default="trace")
    a = ap.parse_args()
    if a.build:
        from lss_carla_amd import build
        print(build.build_variant(a.lib, ["LSS_TRACE=1"] + a.D))
        return
    import torch
    from lss_carla_amd import _lib, ops, synthetic as syn
    from oracle import lss_ref as ref
    l = _lib.open_library(os.path.join(REPO, "lss-carla_amd", "variants", a.lib + ".so"))
    l.lss_debug_trace.argtypes = [ct.c_void_p, ct.c_int]
    dev = torch.device("cuda:0")
    cfg, gc, _ = syn.config_confs("c3")
    B, N, fd = cfg["B"], cfg["N"], cfg["final_dim"]
    rig = {k: v.to(dev) for k, v in syn.make_rig(B, N, fd).items()}
    frustum = ref.create_frustum(fd, gc["dbound"]).to(dev)
    D, H, W = frustum.shape[:3]
    grid = ops.GridSpec.from_conf(gc)
    X, Y, Z = grid.nx
    dn = syn.make_depthnet_out(B, N, D, H, W).to(dev, torch.bfloat16)
    st = _lib.stream_handle(dev)
    plan = ops.plan_from_cameras(frustum, **rig, grid=grid)  # product library's CSR
    dims, g = plan.c_dims, grid.c_struct()
    depth = torch.empty(B * N, D, H, W, device=dev)
    ctx = torch.empty(B * N * H * W, 64, device=dev, dtype=torch.bfloat16)
    out = torch.empty(B, Z * 64, X, Y, device=dev, dtype=torch.bfloat16, memory_format=torch.channels_last)
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    for it in range(4):
        if a.mode == "step":
            flush.zero_()
            plan = ops.plan_from_cameras(frustum, **rig, grid=grid)
        _lib.check(l.lss_lift_prep(_lib.ptr(dn), _lib.BF16, dims, _lib.ptr(depth), _lib.ptr(ctx), _lib.BF16, st),
                   "lift")
        e0, e1 = ct.c_void_p(), ct.c_void_p()
        l.lss_event_create(ct.byref(e0))
        l.lss_event_create(ct.byref(e1))
        _lib.check(l.lss_splat_fwd(_lib.ptr(depth), _lib.ptr(ctx), _lib.BF16, None, _lib.ptr(plan.cell_start),
                                   _lib.ptr(plan.sorted_key), _lib.ptr(plan.sorted_row), dims, g, _lib.ptr(out),
                                   _lib.BF16, _lib.NHWC, st, e0, e1), "fwd")
        ms = ct.c_float()
        l.lss_event_elapsed_ms(e0, e1, ct.byref(ms))
    torch.cuda.synchronize()
    nchunk_waves = ((plan.nprime + 63) // 64 + 3) // 4 * 4
    buf = np.zeros((16384, 5), dtype=np.uint64)
    _lib.check(l.lss_debug_trace(buf.ctypes.data, 16384), "trace")
    t = buf[:, :4].astype(np.int64)
    live = t[:, 0] > 0
    t0 = t[live, 0].min()
    rel = (t - t0) * 10 / 1000.0  # 100 MHz ticks -> us
    print(f"kernel (events) {ms.value * 1e3:.2f} us; stamped span {(t[live, 3].max() - t0) / 100:.2f} us; "
          f"waves stamped {live.sum()}")
    ch = np.arange(16384) < nchunk_waves
    c = live & ch & (t[:, 3] > 0)
    z = live & ~ch & (t[:, 3] > 0)

    def q(x):
        return " ".join(f"{v:6.2f}" for v in np.percentile(x, [0, 10, 50, 90, 99, 100]))
    print("percentiles            p0     p10    p50    p90    p99    max  (us)")
    print("chunk start          ", q(rel[c, 0]))
    print("chunk rt1 (t1-t0)    ", q(rel[c, 1] - rel[c, 0]))
    has2 = c & (t[:, 2] > 0)
    print("chunk rt2 (t2-t1)    ", q(rel[has2, 2] - rel[has2, 1]))
    print("chunk rest (t3-t2)   ", q(rel[has2, 3] - rel[has2, 2]))
    print("chunk total (t3-t0)  ", q(rel[c, 3] - rel[c, 0]))
    print("chunk end            ", q(rel[c, 3]))
    if z.any():
        print("zero start           ", q(rel[z, 0]))
        print("zero total           ", q(rel[z, 3] - rel[z, 0]))
        print("zero end             ", q(rel[z, 3]))
    # start skew between XCDs: per XCC, the waves' start-time percentiles (is the ramp dispatch or XCD start?)
    xcc = (buf[:, 4] >> np.uint64(32)).astype(np.int64)
    for x in range(8):
        for nm, msk in (("chunk", c), ("zero", z)):
            sel = msk & (xcc == x)
            if sel.any():
                print(f"xcc {x} {nm:5s} waves {sel.sum():5d} start p0 {rel[sel, 0].min():5.2f} p10 "
                      f"{np.percentile(rel[sel, 0], 10):5.2f} p50 {np.percentile(rel[sel, 0], 50):5.2f} "
                      f"max {rel[sel, 0].max():5.2f}  end max {rel[sel, 3].max():5.2f}")
    # the slowest chunk waves and their chunks
    sk = plan.sorted_key.cpu().numpy()
    tot = int(plan.cell_start[-1])
    cells = (sk[:tot] >> 32).astype(np.int64)
    cidx = np.nonzero(c)[0]
    slow = cidx[np.argsort(rel[c, 3] - rel[c, 0])[-8:]]
    for w in slow:
        base = 64 * w
        win = cells[max(base - 1, 0):min(base + 128, tot)]
        own = cells[base:min(base + 64, tot)]
        print(f"slow chunk w={w}: start {rel[w, 0]:.2f} t1 {rel[w, 1]:.2f} t2 {rel[w, 2]:.2f} end {rel[w, 3]:.2f}  "
              f"xcc {buf[w, 4] >> 32} hwid {buf[w, 4] & 0xffffffff:#x}; distinct cells in chunk {len(np.unique(own))}, "
              f"max run {np.max(np.unique(win, return_counts=True)[1]) if len(win) else 0}, tail={base + 64 >= tot}")
    # concurrency over time
    for tt in np.arange(0, rel[live, 3].max() + 0.5, 0.5):
        act_c = ((rel[c, 0] <= tt) & (rel[c, 3] > tt)).sum()
        act_z = ((rel[z, 0] <= tt) & (rel[z, 3] > tt)).sum()
        print(f"t={tt:5.1f} us  active chunk waves {act_c:5d}  zero waves {act_z:5d}")


if __name__ == "__main__":
    main()
