"""Kernel micro-benchmark: every hot-path op of config 3 timed in isolation (HIP events), plus
tuning variants of lss_splat_fwd built with -D knobs (lss-carla_amd/variants/*.so).

  python scripts/kbench.py --build-variants     # here (hipcc), before gpurun
  python scripts/kbench.py                      # on the GPU box
"""
import argparse
import ctypes
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

VARIANTS = {
    "g64": ["LSS_ITEM_G=64"],
    "g96": ["LSS_ITEM_G=96"],
    "g128": ["LSS_ITEM_G=128"],
    "g192": ["LSS_ITEM_G=192"],
    "g256": ["LSS_ITEM_G=256"],
    "g128_pf8": ["LSS_ITEM_G=128", "LSS_FWD_PREFETCH=8"],
    "g128_pf32": ["LSS_ITEM_G=128", "LSS_FWD_PREFETCH=32"],
}


def build_variants():
    from lss_carla_amd import build
    for name, defs in VARIANTS.items():
        print(name, build.build_variant(name, defs), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build-variants", action="store_true")
    ap.add_argument("--config", default="c3")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--only", default="", help="run only ops whose name contains this (for rocprofv3 --pmc)")
    args = ap.parse_args()
    if args.build_variants:
        build_variants()
        return
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
    dn = syn.make_depthnet_out(B, N, D, H, W).to(dev, torch.bfloat16)
    lib = _lib.load()
    st = lambda: _lib.stream_handle(dev)  # noqa: E731

    def timeit(fn, iters=args.iters):
        if args.only and args.only not in timeit.name:
            return float("nan")
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters * 1e3  # us

    res = {}

    def named(name, fn, *a):
        timeit.name = name
        return timeit(fn, *a)
    plan = ops.plan_from_cameras(frustum, **rig, grid=grid, inverse="device")
    kept = int(plan.cell_start[-1])
    dims, g = plan.c_dims, grid.c_struct()
    depth = torch.empty(B * N, D, H, W, device=dev)
    ctx_t = torch.empty(B * N * H * W, 64, device=dev)
    bev_bf = torch.empty(B, Z * 64, X, Y, device=dev, dtype=torch.bfloat16, memory_format=torch.channels_last)
    bev_f = torch.empty(B, Z * 64, X, Y, device=dev)
    res["memset_bev_bf16_41MB"] = named("memset_bev_bf16_41MB", lambda: bev_bf.zero_())
    res["memset_bev_f32_82MB"] = named("memset_bev_f32_82MB", lambda: bev_f.zero_())
    res["copy_bev_f32_82MB"] = named("copy_bev_f32_82MB", lambda: bev_f.copy_(bev_bf))
    res["plan_total(device inv)"] = named("plan_total(device inv)", lambda: ops.plan_from_cameras(frustum, **rig, grid=grid, inverse="device"))
    res["lift_prep"] = named("lift_prep", lambda: _lib.check(lib.lss_lift_prep(_lib.ptr(dn), _lib.BF16, dims, _lib.ptr(depth),
                                                                    _lib.ptr(ctx_t), st()), "lift"))

    def fwd(l, out, layout):
        return lambda: _lib.check(l.lss_splat_fwd(_lib.ptr(depth), _lib.ptr(ctx_t), None, _lib.ptr(plan.cell_start),
                                                  _lib.ptr(plan.sorted_key), _lib.ptr(items), dims, g, _lib.ptr(out),
                                                  _lib.dtype_code(out.dtype), layout, st(), None, None), "fwd")

    items = plan.item_start
    res["splat_fwd nhwc bf16"] = named("splat_fwd nhwc bf16", fwd(lib, bev_bf, _lib.NHWC))
    items = None
    res["splat_fwd nhwc bf16 [tile kernel]"] = named("splat_fwd nhwc bf16 [tile kernel]", fwd(lib, bev_bf, _lib.NHWC))
    items = plan.item_start
    res["splat_fwd nchw f32"] = named("splat_fwd nchw f32", fwd(lib, bev_f, _lib.NCHW))
    for path in sorted(glob.glob(os.path.join(REPO, "lss-carla_amd", "variants", "*.so"))):
        vl = _lib.open_library(path)
        name = os.path.basename(path)[:-3]
        res[f"splat_fwd nhwc bf16 [{name}]"] = named(f"splat_fwd nhwc bf16 [{name}]", fwd(vl, bev_bf, _lib.NHWC))
    g_bf = torch.randn(B, Z * 64, X, Y, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    d_dn = torch.empty_like(dn)
    res["splat_bwd nhwc bf16"] = named("splat_bwd nhwc bf16", lambda: _lib.check(lib.lss_splat_bwd(
        _lib.ptr(g_bf), _lib.BF16, _lib.NHWC, _lib.ptr(plan.cell_of), _lib.ptr(depth), _lib.ptr(ctx_t), dims, g,
        _lib.ptr(d_dn), _lib.BF16, st()), "bwd"))
    rows = torch.empty(grid.ncells(B) * 64, device=dev)
    g_f = torch.randn(B, Z * 64, X, Y, device=dev)
    res["bev_rows nchw f32"] = named("bev_rows nchw f32", lambda: _lib.check(lib.lss_bev_rows(
        _lib.ptr(g_f), _lib.F32, _lib.ptr(plan.cell_start), dims, g, _lib.ptr(rows), st()), "rows"))
    nbytes = (B * N * D * H * W * 4 + B * N * H * W * 64 * 4 + kept * 4 + (grid.ncells(B) + 1) * 4
              + grid.ncells(B) * 64 * 2)
    for k, v in res.items():
        extra = f"  {nbytes / v / 1e3:7.1f} GB/s alg" if k.startswith("splat_fwd nhwc bf16") else ""
        print(f"{k:40s} {v:9.2f} us{extra}")
    print(json.dumps({"kept": kept, "alg_bytes_fwd_bf16": nbytes}))


if __name__ == "__main__":
    main()
