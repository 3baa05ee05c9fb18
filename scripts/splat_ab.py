"""Splat forward A/B across library builds, plus the HBM write ceiling, in the cache states of a step.

For each library (the product build or lss-carla_amd/variants/<name>.so) the splat forward of one
config is launched with kernel-stamped events (hipExtLaunchKernelGGL: the kernel alone) after
  dirty  512 MiB written (L2 + Infinity Cache full of dirty lines, the old bench.py ceiling state)
  read   512 MiB read (caches full of clean lines)
  step   dirty, then the plan and the lift rebuilt (the order of a training step)
and its output is compared with the product build's, bit for bit.
The ceiling rows time lss_ceiling_store (16-B stores over the BEV buffer) in the same states.

  python scripts/splat_ab.py --config c3 --libs product,zu8_o2 [--ceiling 1]
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
    ap.add_argument("--layout", default="nhwc", choices=["nhwc", "nchw"])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--libs", default="product")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--modes", default="dirty,read,step")
    ap.add_argument("--ceiling", type=int, default=1)
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
    st = lambda: _lib.stream_handle(dev)  # noqa: E731
    dn = syn.make_depthnet_out(B, N, D, H, W).to(dev, torch.bfloat16)
    inv = ops.camera_inverses(rig["post_rots"], rig["intrins"])
    plan = ops.plan_from_cameras(frustum, **rig, grid=grid, inverses=inv)
    dims, g = plan.c_dims, grid.c_struct()
    kept = int(plan.cell_start[-1])
    odt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    ctx_dt = odt
    depth = torch.empty(B * N, D, H, W, device=dev)
    ctx = torch.empty(B * N * H * W, 64, device=dev, dtype=ctx_dt)
    layout = _lib.NHWC if args.layout == "nhwc" else _lib.NCHW
    mf = torch.channels_last if args.layout == "nhwc" else torch.contiguous_format
    bev = torch.empty(B, Z * 64, X, Y, device=dev, dtype=odt, memory_format=mf)
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)

    def lift():
        _lib.check(lib.lss_lift_prep(_lib.ptr(dn), _lib.BF16, dims, _lib.ptr(depth), _lib.ptr(ctx),
                                     _lib.dtype_code(ctx.dtype), st()), "lift")

    def replan():
        ops.plan_from_cameras(frustum, **rig, grid=grid, inverses=inv)

    def prepare(mode):
        if mode in ("dirty", "step"):
            flush.zero_()
        elif mode == "read":
            _lib.check(lib.lss_ceiling_read(_lib.ptr(flush), flush.numel(), _lib.ptr(sink), st()), "read")
        if mode == "step":
            replan()
            lift()

    def stamped(launch, mode):
        tot, ts = 0.0, []
        for i in range(args.iters + 3):
            prepare(mode)
            a, b = ct.c_void_p(), ct.c_void_p()
            lib.lss_event_create(ct.byref(a))
            lib.lss_event_create(ct.byref(b))
            launch(a, b)
            ms = ct.c_float()
            lib.lss_event_elapsed_ms(a, b, ct.byref(ms))
            if i >= 3:
                ts.append(ms.value * 1e3)
            lib.lss_event_destroy(a)
            lib.lss_event_destroy(b)
        ts.sort()
        return {"avg": round(sum(ts) / len(ts), 2), "p50": round(ts[len(ts) // 2], 2), "min": round(ts[0], 2)}

    lift()
    res = {"config": args.config, "layout": args.layout, "dtype": args.dtype, "kept": kept}
    nbytes = (plan.nprime * 4 + B * N * H * W * 64 * ctx.element_size() + kept * 4
              + (grid.ncells(B) + 1) * 4 + bev.numel() * bev.element_size())
    res["alg_bytes"] = nbytes
    modes = args.modes.split(",")

    def splat_fn(l):
        def launch(a, b):
            _lib.check(l.lss_splat_fwd(_lib.ptr(depth), _lib.ptr(ctx), _lib.dtype_code(ctx.dtype), None,
                                       _lib.ptr(plan.cell_start), _lib.ptr(plan.sorted_key),
                                       _lib.ptr(plan.sorted_row), dims, g, _lib.ptr(bev),
                                       _lib.dtype_code(bev.dtype), layout, st(), a, b), "fwd")
        return launch

    splat_fn(lib)(None, None)
    want = bev.clone()
    for name in args.libs.split(","):
        l = lib if name == "product" else _lib.open_library(
            os.path.join(REPO, "lss-carla_amd", "variants", name + ".so"))
        bev.fill_(1.0)
        splat_fn(l)(None, None)
        torch.cuda.synchronize()
        same = bool(torch.equal(bev, want))
        row = {"equal_to_product": same}
        for m in modes:
            t = stamped(splat_fn(l), m)
            t["frac"] = round(nbytes / (t["avg"] * 1e3) / 8000.0, 4)
            row[m] = t
        res[f"splat[{name}]"] = row
        print(f"splat[{name}] {json.dumps(row)}", flush=True)
    if args.ceiling:
        nb = bev.numel() * bev.element_size()
        for pt in (1, 4):
            for fl in (0, 1, 2):
                row = {}
                for m in ("dirty", "read"):
                    t = stamped(lambda a, b: _lib.check(lib.lss_ceiling_store(_lib.ptr(bev), nb, pt, fl, st(), a, b),
                                                        "ceiling"), m)
                    t["GB/s"] = round(nb / (t["avg"] * 1e3), 1)
                    row[m] = t
                res[f"ceiling[pt={pt},{('plain', 'nt', 'sc1')[fl]}]"] = row
                print(f"ceiling[pt={pt},{('plain', 'nt', 'sc1')[fl]}] {json.dumps(row)}", flush=True)
        row = {}
        for m in ("dirty", "read"):
            tot = []
            for i in range(args.iters + 3):
                prepare(m)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                bev.zero_()
                e1.record()
                torch.cuda.synchronize()
                if i >= 3:
                    tot.append(e0.elapsed_time(e1) * 1e3)
            row[m] = round(sum(tot) / len(tot), 2)
        res["torch_memset_us"] = row
        print(f"torch memset {json.dumps(row)}", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
