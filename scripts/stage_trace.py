"""Per-wave stage timeline of the fused depthnet lift (k_depthnet_lift2), the tiled splat backward
(k_splat_bwd_tile) or the geometry / cell count kernel (k_geometry_cells: 1 after the geometry, 2 after
the cell index, 3 after the counted slot) from a LSS_TRACE=1 build (diagnostics only; stamps 0 start, 1 after the staging
barrier, 2 after the MFMA / the gathers and reductions, 3 end).

  python scripts/splat_trace.py --build        # here: builds variants/trace.so (-D KNOB=V for others)
  python scripts/stage_trace.py lift|bwd       # GPU box
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
    ap.add_argument("kernel", choices=["lift", "lift3", "bwd", "geom", "nchw", "scan"])
    ap.add_argument("--config", default="c3")
    ap.add_argument("--cold", type=int, default=1)
    ap.add_argument("--lib", default="trace", help="variants/<name>.so, a LSS_TRACE=1 build")
    a = ap.parse_args()
    import torch
    from lss_carla_amd import _lib, ops, synthetic as syn
    from oracle import lss_ref as ref
    l = _lib.open_library(os.path.join(REPO, "lss-carla_amd", "variants", a.lib + ".so"))
    l.lss_debug_trace.argtypes = [ct.c_void_p, ct.c_int]
    dev = torch.device("cuda:0")
    cfg, gc, _ = syn.config_confs(a.config)
    B, N, fd = cfg["B"], cfg["N"], cfg["final_dim"]
    rig = {k: v.to(dev) for k, v in syn.make_rig(B, N, fd).items()}
    frustum = ref.create_frustum(fd, gc["dbound"]).to(dev)
    D, H, W = frustum.shape[:3]
    grid = ops.GridSpec.from_conf(gc)
    X, Y, Z = grid.nx
    st = _lib.stream_handle(dev)
    plan = ops.plan_from_cameras(frustum, **rig, grid=grid)
    dims, g = plan.c_dims, grid.c_struct()
    depth = torch.empty(B * N, D, H, W, device=dev)
    ctx = torch.empty(B * N * H * W, 64, device=dev, dtype=torch.bfloat16)
    feat = torch.randn(B * N, 512, H, W, device=dev).to(torch.bfloat16)
    feat_cl = feat.contiguous(memory_format=torch.channels_last)
    wdn = (torch.randn(D + 64, 512, 1, 1, device=dev) * 0.05).to(torch.bfloat16)
    bdn = torch.zeros(D + 64, device=dev, dtype=torch.bfloat16)
    gbev = torch.randn(B, Z * 64, X, Y, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    d_dn = torch.empty(B * N, D + 64, H, W, device=dev, dtype=torch.bfloat16)
    dnf = syn.make_depthnet_out(B, N, D, H, W).to(dev)
    ctxf = torch.empty(B * N * H * W, 64, device=dev)
    bevf = torch.empty(B, Z * 64, X, Y, device=dev)
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    pinv, kinv = ops.camera_inverses(rig["post_rots"], rig["intrins"])
    ro, tr, pt = [t.float().contiguous() for t in (rig["rots"], rig["trans"], rig["post_trans"])]
    ms = ct.c_float()
    for it in range(4):
        if a.cold:
            flush.zero_()
        e0, e1 = ct.c_void_p(), ct.c_void_p()
        l.lss_event_create(ct.byref(e0))
        l.lss_event_create(ct.byref(e1))
        l.lss_event_record(e0, st)
        if a.kernel == "scan":  # k_scan_lookback: 1 after the ticket, 2 after the block scan, 3 end
            if it == 0:
                prod = _lib.load()
                ncells = grid.ncells(B)
                counts = torch.zeros(ncells, device=dev, dtype=torch.int32)
                slot = torch.empty(plan.nprime, device=dev, dtype=torch.int32)
                cell_of = torch.empty(plan.nprime, device=dev, dtype=torch.int32)
                wsb = torch.zeros(int(l.lss_csr_workspace_bytes(ncells)), device=dev, dtype=torch.uint8)
                scr = torch.empty(int(l.lss_csr_scratch_bytes(ncells, plan.nprime)), device=dev, dtype=torch.uint8)
                cs = torch.empty(ncells + 1, device=dev, dtype=torch.int32)
                sk = torch.empty(plan.nprime, device=dev, dtype=torch.int64)
                sr = torch.empty(plan.nprime, device=dev, dtype=torch.int32)
            _lib.check(prod.lss_geometry_cells(_lib.ptr(frustum), _lib.ptr(ro), _lib.ptr(tr), _lib.ptr(kinv),
                                               _lib.ptr(pinv), _lib.ptr(pt), dims, g, None, _lib.ptr(cell_of),
                                               _lib.ptr(counts), _lib.ptr(slot), st), "geom")
            _lib.check(l.lss_csr_build_ws(_lib.ptr(cell_of), _lib.ptr(slot), plan.nprime, _lib.ptr(counts), ncells,
                                          dims, _lib.ptr(cs), _lib.ptr(sk), _lib.ptr(sr), _lib.ptr(scr),
                                          _lib.ptr(wsb), st), "csr")
            if it == 3:
                assert torch.equal(cs, plan.cell_start), "trace build CSR differs"
        elif a.kernel == "geom":
            counts = torch.zeros(grid.ncells(B), device=dev, dtype=torch.int32)
            slot = torch.empty(plan.nprime, device=dev, dtype=torch.int32)
            cell_of = torch.empty(plan.nprime, device=dev, dtype=torch.int32)
            _lib.check(l.lss_geometry_cells(_lib.ptr(frustum), _lib.ptr(ro), _lib.ptr(tr), _lib.ptr(kinv),
                                            _lib.ptr(pinv), _lib.ptr(pt), dims, g, None, _lib.ptr(cell_of),
                                            _lib.ptr(counts), _lib.ptr(slot), st), "geom")
        elif a.kernel == "nchw":  # config 2's forward: fp32 context rows, fp32 NCHW BEV
            _lib.check(l.lss_lift_prep(_lib.ptr(dnf), _lib.F32, dims, _lib.ptr(depth), _lib.ptr(ctxf), _lib.F32, st),
                       "lift")
            _lib.check(l.lss_splat_fwd(_lib.ptr(depth), _lib.ptr(ctxf), _lib.F32, None, _lib.ptr(plan.cell_start),
                                       _lib.ptr(plan.sorted_key), _lib.ptr(plan.sorted_row), dims, g,
                                       _lib.ptr(bevf), _lib.F32, _lib.NCHW, st, None, None), "fwd")
        elif a.kernel == "lift3":  # channels-last features (k_depthnet_lift3), weights in fragment order
            if it == 0:
                packed = torch.empty(_lib.DN_PACKED_BYTES(512) // 2, device=dev, dtype=torch.bfloat16)
                _lib.check(l.lss_depthnet_pack(_lib.ptr(wdn), _lib.ptr(bdn), _lib.BF16, wdn.shape[0], 512,
                                               _lib.ptr(packed), None, None, st), "pack")
            _lib.check(l.lss_depthnet_lift_nhwc_packed(_lib.ptr(feat_cl), _lib.ptr(packed), _lib.ptr(bdn), 512, dims,
                                                       _lib.ptr(depth), _lib.ptr(ctx), _lib.BF16, st), "lift3")
        elif a.kernel == "lift":
            _lib.check(l.lss_depthnet_lift(_lib.ptr(feat), _lib.ptr(wdn), _lib.ptr(bdn), _lib.BF16, 512, dims,
                                           _lib.ptr(depth), _lib.ptr(ctx), _lib.BF16, st), "lift")
        else:
            _lib.check(l.lss_splat_bwd(_lib.ptr(gbev), _lib.BF16, _lib.NHWC, _lib.ptr(plan.cell_of), _lib.ptr(depth),
                                       _lib.ptr(ctx), _lib.BF16, dims, g, _lib.ptr(d_dn), _lib.BF16, st), "bwd")
        l.lss_event_record(e1, st)
        torch.cuda.synchronize()
        l.lss_event_elapsed_ms(e0, e1, ct.byref(ms))
    torch.cuda.synchronize()
    buf = np.zeros((16384, 5), dtype=np.uint64)
    _lib.check(l.lss_debug_trace(buf.ctypes.data, 16384), "trace")
    t = buf[:, :5].astype(np.int64)
    live = (t[:, 0] > 0) & (t[:, 3] > 0)
    t0 = t[live, 0].min()
    rel = (t - t0) / 100.0  # 100 MHz ticks -> us
    print(f"{a.kernel} [{a.lib}]: events {ms.value * 1e3:.2f} us; stamped span {rel[live, 3].max():.2f} us; waves {live.sum()}")

    def q(x):
        return " ".join(f"{v:6.2f}" for v in np.percentile(x, [0, 10, 50, 90, 99, 100]))
    print("percentiles             p0     p10    p50    p90    p99    max  (us)")
    print("start                ", q(rel[live, 0]))
    print("stage (t1-t0)        ", q(rel[live, 1] - rel[live, 0]))
    print("compute (t2-t1)      ", q(rel[live, 2] - rel[live, 1]))
    print("tail (t3-t2)         ", q(rel[live, 3] - rel[live, 2]))
    if a.kernel == "nchw":  # stamp 4: after the tile zeroing + group search barrier (occupied tiles)
        occ = live & (t[:, 4] > 0)
        print("setup (t4-t1)        ", q(rel[occ, 4] - rel[occ, 1]))
        print("sums (t2-t4)         ", q(rel[occ, 2] - rel[occ, 4]))
        print(f"occupied tiles: {occ.sum()} of {live.sum()} waves")
    print("total (t3-t0)        ", q(rel[live, 3] - rel[live, 0]))
    print("end                  ", q(rel[live, 3]))
    for tt in np.arange(0, rel[live, 3].max() + 0.5, 0.5):
        act = ((rel[live, 0] <= tt) & (rel[live, 3] > tt)).sum()
        print(f"t={tt:5.1f} us  active waves {act:5d}")


if __name__ == "__main__":
    main()
