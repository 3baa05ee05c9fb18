"""Hot-kernel A/B across library builds, outputs compared with the product build's bit for bit, times
from events around the launch on its stream in two cache states (warm: back to back; read: after a
512 MiB read sweep):
  bwd   lss_splat_bwd (channels-last bf16 dBEV -> bf16 d_depthnet_out)
  lift  lss_depthnet_lift_nhwc_packed (channels-last bf16 features, fragment-order weights -> depth, context rows)

  python scripts/kernel_ab.py --config c3 --libs product,bwd81,dpp0 [--kernel lift]
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
    ap.add_argument("--kernel", default="bwd", choices=["bwd", "lift"])
    ap.add_argument("--producer", default="none", choices=["none", "dropout", "torch"],
                    help="lift: after the read sweep, rewrite the features with lss_dropout (keep 1: an XCD-"
                         "contiguous copy, + the packed weights warmed) or torch's copy, as a step's last kernel")
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

    feat = torch.randn(B * N, 512, H, W, generator=gen).to(dev, torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    wdn = (torch.randn(D + 64, 512, 1, 1, generator=gen) * 0.05).to(dev, torch.bfloat16)
    bdn = (torch.randn(D + 64, generator=gen) * 0.1).to(dev, torch.bfloat16)
    packed = torch.empty(_lib.DN_PACKED_BYTES(512) // 2, device=dev, dtype=torch.bfloat16)
    _lib.check(lib.lss_depthnet_pack(_lib.ptr(wdn), _lib.ptr(bdn), _lib.BF16, wdn.shape[0], 512, _lib.ptr(packed),
                                     None, None, st), "pack")

    def run(l):
        if args.kernel == "bwd":
            _lib.check(l.lss_splat_bwd(_lib.ptr(gbev), _lib.BF16, _lib.NHWC, _lib.ptr(plan.cell_of), _lib.ptr(depth),
                                       _lib.ptr(ctx), _lib.BF16, dims, g, _lib.ptr(d_dn), _lib.BF16, st), "bwd")
        else:
            _lib.check(l.lss_depthnet_lift_nhwc_packed(_lib.ptr(feat), _lib.ptr(packed), _lib.ptr(bdn), 512, dims,
                                                       _lib.ptr(depth), _lib.ptr(ctx), _lib.BF16, st), "lift3")

    def output():
        return d_dn if args.kernel == "bwd" else torch.cat([depth.flatten(), ctx.float().flatten()])

    feat_src = feat.clone(memory_format=torch.channels_last) if args.kernel == "lift" else None
    seed = torch.zeros(1, device=dev, dtype=torch.int64)

    def produce():
        if args.producer == "dropout":
            _lib.check(lib.lss_dropout(_lib.ptr(feat_src), _lib.BF16, feat.numel(), _lib.ptr(seed), 1.0, _lib.ptr(feat),
                                       _lib.ptr(packed), packed.numel() * 2, st), "dropout")
        elif args.producer == "torch":
            feat.copy_(feat_src)

    def timed(l, mode):
        ts = []
        for i in range(args.iters + 3):
            if mode == "read":
                _lib.check(lib.lss_ceiling_read(_lib.ptr(flush), flush.numel(), _lib.ptr(sink), st), "read")
            if args.kernel == "lift":
                produce()
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
    want = output().clone()
    res = {"config": args.config, "kernel": args.kernel, "producer": args.producer, "pixels": B * N * H * W, "D": D}
    for name in args.libs.split(","):
        l = lib if name == "product" else _lib.open_library(
            os.path.join(REPO, "lss-carla_amd", "variants", name + ".so"))
        if args.kernel == "bwd":
            d_dn.fill_(7.0)
        else:  # (the lift's outputs; for the backward they are inputs)
            depth.fill_(7.0)
            ctx.fill_(7.0)
        run(l)
        torch.cuda.synchronize()
        got = output()
        row = {"equal_to_product": bool(torch.equal(got, want)),
               "max_abs_diff": float((got.float() - want.float()).abs().max())}
        for m in ("warm", "read"):
            row[m] = timed(l, m)
        res[f"{args.kernel}[{name}]"] = row
        print(f"{args.kernel}[{name}] {json.dumps(row)}", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
