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
    "lds_b8": ["LSS_GROUPS=0", "LSS_BATCH=8"],
    "lds_b16": ["LSS_GROUPS=0", "LSS_BATCH=16"],
    "u2": ["LSS_UNROLL=2"],
    "u3": ["LSS_UNROLL=3"],
    "u6": ["LSS_UNROLL=6"],
    "wpc16": ["LSS_WAVES_PER_CU=16"],
    "wpc0": ["LSS_WAVES_PER_CU=0"],
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
    ap.add_argument("--variants", type=int, default=1, help="also time the variants/*.so builds")
    ap.add_argument("--cold", type=int, default=1, help="also time splat_fwd with caches flushed before each launch")
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

    def lib_plan(l):
        """cell_start / sorted_key / sorted_row built by library `l`."""
        import ctypes as ct
        ncells = grid.ncells(B)
        nprime = plan.nprime
        counts = torch.zeros(ncells, device=dev, dtype=torch.int32)
        slot = torch.empty(nprime, device=dev, dtype=torch.int32)
        cell_of = torch.empty(nprime, device=dev, dtype=torch.int32)
        pinv, kinv = ops.camera_inverses(rig["post_rots"], rig["intrins"], "device")
        ro, tr, pt = [t.float().contiguous() for t in (rig["rots"], rig["trans"], rig["post_trans"])]
        _lib.check(l.lss_geometry_cells(_lib.ptr(frustum), _lib.ptr(ro), _lib.ptr(tr), _lib.ptr(kinv),
                                        _lib.ptr(pinv), _lib.ptr(pt), dims, g, None, _lib.ptr(cell_of),
                                        _lib.ptr(counts), _lib.ptr(slot), st()), "geom")
        cs = torch.empty(ncells + 1, device=dev, dtype=torch.int32)
        sk = torch.empty(nprime, device=dev, dtype=torch.int64)
        sr = torch.empty(nprime, device=dev, dtype=torch.int32)
        scr = torch.empty(int(l.lss_csr_scratch_bytes(ncells, nprime)), device=dev, dtype=torch.uint8)
        _lib.check(l.lss_csr_build(_lib.ptr(cell_of), _lib.ptr(slot), nprime, _lib.ptr(counts), ncells, dims,
                                   _lib.ptr(cs), _lib.ptr(sk), _lib.ptr(sr), _lib.ptr(scr), st()), "csr")
        return cs, sk, sr

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

    pcsr = (plan.cell_start, plan.sorted_key, plan.sorted_row)

    def fwd(l, out, layout, csr=pcsr):
        cs, sk, its = csr
        return lambda: _lib.check(l.lss_splat_fwd(_lib.ptr(depth), _lib.ptr(ctx_t), None, _lib.ptr(cs),
                                                  _lib.ptr(sk), _lib.ptr(its), dims, g, _lib.ptr(out),
                                                  _lib.dtype_code(out.dtype), layout, st(), None, None), "fwd")

    res["splat_fwd nhwc bf16"] = named("splat_fwd nhwc bf16", fwd(lib, bev_bf, _lib.NHWC))
    res["splat_fwd nchw f32"] = named("splat_fwd nchw f32", fwd(lib, bev_f, _lib.NCHW))
    fwd(lib, bev_bf, _lib.NHWC)()
    ref_out = bev_bf.clone()
    variants = {}
    for path in sorted(glob.glob(os.path.join(REPO, "lss-carla_amd", "variants", "*.so"))) if args.variants else []:
        vl = _lib.open_library(path)
        name = os.path.basename(path)[:-3]
        variants[name] = (vl, lib_plan(vl))
        res[f"splat_fwd nhwc bf16 [{name}]"] = named(f"splat_fwd nhwc bf16 [{name}]",
                                                     fwd(vl, bev_bf, _lib.NHWC, variants[name][1]))
        if not torch.equal(bev_bf, ref_out):
            print(f"WARNING variant {name}: output differs from the product kernel", flush=True)
    if args.cold:
        # cold caches, as inside a training step (the trunk runs between the CSR build and the splat):
        # 512 MiB written before every launch, kernel time from kernel-stamped events (hipExtLaunchKernel)
        flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)

        def cold(l, out, layout, csr, iters=20):
            import ctypes as ct
            cs, sk, its = csr
            tot = 0.0
            for _ in range(iters):
                flush.zero_()
                a, b = ct.c_void_p(), ct.c_void_p()
                l.lss_event_create(ct.byref(a))
                l.lss_event_create(ct.byref(b))
                _lib.check(l.lss_splat_fwd(_lib.ptr(depth), _lib.ptr(ctx_t), None, _lib.ptr(cs),
                                           _lib.ptr(sk), _lib.ptr(its), dims, g, _lib.ptr(out),
                                           _lib.dtype_code(out.dtype), layout, st(), a, b), "fwd")
                ms = ct.c_float()
                l.lss_event_elapsed_ms(a, b, ct.byref(ms))
                tot += ms.value
                l.lss_event_destroy(a)
                l.lss_event_destroy(b)
            return tot / iters * 1e3

        if not args.only or "cold" in args.only:
            res["COLD splat_fwd nhwc bf16"] = cold(lib, bev_bf, _lib.NHWC, pcsr)
            for name, (vl, csr) in variants.items():
                res[f"COLD splat_fwd nhwc bf16 [{name}]"] = cold(vl, bev_bf, _lib.NHWC, csr)
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
        extra = f"  {nbytes / v / 1e3:7.1f} GB/s alg" if "splat_fwd nhwc bf16" in k else ""
        print(f"{k:40s} {v:9.2f} us{extra}")
    print(json.dumps({"kept": kept, "alg_bytes_fwd_bf16": nbytes}))


if __name__ == "__main__":
    main()
