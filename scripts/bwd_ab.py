"""Splat backward A/B across library builds: lss_splat_bwd (channels-last bf16 dBEV -> bf16 d_depthnet_out)
of one config, outputs compared with the product build's bit for bit, times from events around the
launch on its stream in two cache states (warm: back to back; read: after a 512 MiB read sweep).

  python scripts/bwd_ab.py --config c3 --libs product,bwd81,dpp0
"""
import argparse
import ctypes as ct
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--libs", default="product")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    import torch
    from lss_carla_amd import _lib, ops, synthetic as syn
    from oracle import lss_ref as ref

    dev = torch.device("cuda:0")
    cfg, gc, _ = syn.config_confs(args.config)
    B, N, fd = cfg["B"], cfg["N"], cfg["final_dim"]
    rig = {k: v.to(dev) for k, v in syn.make_rig(B, N, fd).items()}
    frustum = ref.create_frustum(fd, gc["dbound"]).to(dev)
    D, H, W = frustum.shape[:3]
    grid = ops.GridSpec.from_conf(gc)
    X, Y, Z = grid.nx
    lib = _lib.load()
    st = _lib.stream_handle(dev)
    dn = syn.make_depthnet_out(B, N, D, H, W).to(dev, torch.bfloat16)
    plan = ops.plan_from_cameras(frustum, **rig, grid=grid)
    dims, g = plan.c_dims, grid.c_struct()
    depth = torch.empty(B * N, D, H, W, device=dev)
    ctx = torch.empty(B * N * H * W, 64, device=dev, dtype=torch.bfloat16)
    _lib.check(lib.lss_lift_prep(_lib.ptr(dn), _lib.BF16, dims, _lib.ptr(depth), _lib.ptr(ctx), _lib.BF16, st), "lift")
    gen = torch.Generator(device="cpu").manual_seed(0)
    gbev = torch.randn(B, Z * 64, X, Y, generator=gen).to(dev, torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    d_dn = torch.empty(B * N, D + 64, H, W, device=dev, dtype=torch.bfloat16)
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)

    def run(l):
        _lib.check(l.lss_splat_bwd(_lib.ptr(gbev), _lib.BF16, _lib.NHWC, _lib.ptr(plan.cell_of), _lib.ptr(depth),
                                   _lib.ptr(ctx), _lib.BF16, dims, g, _lib.ptr(d_dn), _lib.BF16, st), "bwd")

    def timed(l, mode):
        ts = []
        for i in range(args.iters + 3):
            if mode == "read":
                _lib.check(lib.lss_ceiling_read(_lib.ptr(flush), flush.numel(), _lib.ptr(sink), st), "read")
            a, b = ct.c_void_p(), ct.c_void_p()
            lib.lss_event_create(ct.byref(a))
            lib.lss_event_create(ct.byref(b))
            lib.lss_event_record(a, st)
            run(l)
            lib.lss_event_record(b, st)
            torch.cuda.synchronize()
            ms = ct.c_float()
            lib.lss_event_elapsed_ms(a, b, ct.byref(ms))
            lib.lss_event_destroy(a)
            lib.lss_event_destroy(b)
            if i >= 3:
                ts.append(ms.value * 1e3)
        ts.sort()
        return {"avg": round(sum(ts) / len(ts), 2), "p50": round(ts[len(ts) // 2], 2), "min": round(ts[0], 2)}

    run(lib)
    torch.cuda.synchronize()
    want = d_dn.clone()
    res = {"config": args.config, "pixels": B * N * H * W, "D": D}
    for name in args.libs.split(","):
        l = lib if name == "product" else _lib.open_library(
            os.path.join(REPO, "lss-carla_amd", "variants", name + ".so"))
        d_dn.fill_(7.0)
        run(l)
        torch.cuda.synchronize()
        row = {"equal_to_product": bool(torch.equal(d_dn, want)),
               "max_abs_diff": float((d_dn.float() - want.float()).abs().max())}
        for m in ("warm", "read"):
            row[m] = timed(l, m)
        res[f"bwd[{name}]"] = row
        print(f"bwd[{name}] {json.dumps(row)}", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
