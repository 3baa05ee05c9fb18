"""Kernel micro-benchmark: every hot-path op of one config timed in isolation (launch to launch, warm
caches), and the splat forward with kernel-stamped events (hipExtLaunchKernelGGL: the kernel alone) in
the cache states of a training step:
  warm  back-to-back launches
  step  512 MiB written before each launch (L2 + Infinity Cache full of dirty lines), then the plan
        and the lift rebuilt right before the splat -- the order of a training step
Variants built with -D knobs (lss-carla_amd/variants/<name>.so, build.build_variant) are timed with
--libs; scripts/splat_ab.py does the splat-only A/B with the write ceiling.

  python scripts/kbench.py [--config c3] [--libs product,zu8_o2]     # on the GPU box
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
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--libs", default="product")
    ap.add_argument("--only", default="", help="run only ops whose name contains this (for rocprofv3 --pmc)")
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
    st = lambda: _lib.stream_handle(dev)  # noqa: E731
    inv = ops.camera_inverses(rig["post_rots"], rig["intrins"])
    pinv, kinv = inv
    plan = ops.plan_from_cameras(frustum, **rig, grid=grid, inverses=inv)
    kept = int(plan.cell_start[-1])
    dims, g = plan.c_dims, grid.c_struct()
    ncells, nprime = grid.ncells(B), plan.nprime
    ro, tr, pt = [t.float().contiguous() for t in (rig["rots"], rig["trans"], rig["post_trans"])]
    dn = syn.make_depthnet_out(B, N, D, H, W).to(dev, torch.bfloat16)
    depth = torch.empty(B * N, D, H, W, device=dev)
    ctx_t = torch.empty(B * N * H * W, 64, device=dev, dtype=torch.bfloat16)
    ctx_f = torch.empty(B * N * H * W, 64, device=dev)
    feat = torch.randn(B * N, 512, H, W, device=dev).to(torch.bfloat16)
    feat_cl = feat.contiguous(memory_format=torch.channels_last)
    wdn = (torch.randn(D + 64, 512, device=dev) * 0.05).to(torch.bfloat16)
    bdn = torch.zeros(D + 64, device=dev, dtype=torch.bfloat16)
    bev_bf = torch.empty(B, Z * 64, X, Y, device=dev, dtype=torch.bfloat16, memory_format=torch.channels_last)
    bev_f = torch.empty(B, Z * 64, X, Y, device=dev)
    g_bf = torch.randn(B, Z * 64, X, Y, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    d_dn = torch.empty_like(dn)
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)

    def timeit(name, fn, iters=args.iters):
        """Launch-to-launch time (includes the host's launch overhead for short kernels)."""
        if args.only and args.only not in name:
            return None
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / iters * 1e3, 2)

    def lib_ops(l):
        ws = ops.PlanWs(dev, ncells, nprime)
        cell_of = torch.empty(nprime, device=dev, dtype=torch.int32)
        slot = torch.empty(nprime, device=dev, dtype=torch.int32)
        cs = torch.empty(ncells + 1, device=dev, dtype=torch.int32)
        sk = torch.empty(nprime, device=dev, dtype=torch.int64)
        sr = torch.empty(nprime, device=dev, dtype=torch.int32)

        def plan_ws():
            _lib.check(l.lss_geometry_cells(_lib.ptr(frustum), _lib.ptr(ro), _lib.ptr(tr), _lib.ptr(kinv),
                                            _lib.ptr(pinv), _lib.ptr(pt), dims, g, None, _lib.ptr(cell_of),
                                            _lib.ptr(ws.counts), _lib.ptr(slot), st()), "geom")
            _lib.check(l.lss_csr_build_ws(_lib.ptr(cell_of), _lib.ptr(slot), nprime, _lib.ptr(ws.counts), ncells,
                                          dims, _lib.ptr(cs), _lib.ptr(sk), _lib.ptr(sr), _lib.ptr(ws.scratch),
                                          _lib.ptr(ws.workspace), st()), "csr_ws")

        def lift_prep(ctx, code):
            return lambda: _lib.check(l.lss_lift_prep(_lib.ptr(dn), _lib.BF16, dims, _lib.ptr(depth), _lib.ptr(ctx),
                                                      code, st()), "lift_prep")

        def splat(out, layout, ctx, a=None, b=None):
            _lib.check(l.lss_splat_fwd(_lib.ptr(depth), _lib.ptr(ctx), _lib.dtype_code(ctx.dtype), None,
                                       _lib.ptr(cs), _lib.ptr(sk), _lib.ptr(sr), dims, g, _lib.ptr(out),
                                       _lib.dtype_code(out.dtype), layout, st(), a, b), "fwd")

        def stamped(out, layout, ctx, mode, iters=20):
            tot = 0.0
            for i in range(iters + 3):
                if mode == "step":
                    flush.zero_()
                    plan_ws()
                    lift_prep(ctx, _lib.dtype_code(ctx.dtype))()
                a, b = ct.c_void_p(), ct.c_void_p()
                l.lss_event_create(ct.byref(a))
                l.lss_event_create(ct.byref(b))
                splat(out, layout, ctx, a, b)
                ms = ct.c_float()
                l.lss_event_elapsed_ms(a, b, ct.byref(ms))
                if i >= 3:
                    tot += ms.value
                l.lss_event_destroy(a)
                l.lss_event_destroy(b)
            return round(tot / iters * 1e3, 2)

        r = {}
        r["plan (geometry + csr_build_ws)"] = timeit("plan", plan_ws)
        plan_ws()
        if not (torch.equal(cs, plan.cell_start) and torch.equal(sk, plan.sorted_key)):
            print("WARNING: CSR differs from the product plan", flush=True)
        r["lift_prep bf16 ctx"] = timeit("lift_prep", lift_prep(ctx_t, _lib.BF16))
        r["depthnet_lift (NCHW feat)"] = timeit("depthnet_lift", lambda: _lib.check(l.lss_depthnet_lift(
            _lib.ptr(feat), _lib.ptr(wdn), _lib.ptr(bdn), _lib.BF16, 512, dims, _lib.ptr(depth), _lib.ptr(ctx_t),
            _lib.BF16, st()), "lift2"))
        r["depthnet_lift_nhwc (channels-last feat)"] = timeit("depthnet_lift_nhwc", lambda: _lib.check(
            l.lss_depthnet_lift_nhwc(_lib.ptr(feat_cl), _lib.ptr(wdn), _lib.ptr(bdn), _lib.BF16, 512, dims,
                                     _lib.ptr(depth), _lib.ptr(ctx_t), _lib.BF16, st()), "lift3"))
        if hasattr(l, "lss_depthnet_pack"):
            packed = torch.empty(_lib.DN_PACKED_BYTES(512) // 2, device=dev, dtype=torch.bfloat16)
            _lib.check(l.lss_depthnet_pack(_lib.ptr(wdn), _lib.ptr(bdn), _lib.BF16, D + 64, 512, _lib.ptr(packed),
                                           None, None, st()), "pack")
            r["depthnet_lift_nhwc_packed (fragment-order weights)"] = timeit("depthnet_lift_nhwc_packed", lambda: _lib.check(
                l.lss_depthnet_lift_nhwc_packed(_lib.ptr(feat_cl), _lib.ptr(packed), _lib.ptr(bdn), 512, dims,
                                                _lib.ptr(depth), _lib.ptr(ctx_t), _lib.BF16, st()), "lift3p"))
            wf, bfl = wdn.float().contiguous(), bdn.float()
            r["depthnet_pack (fp32 -> fragments + plain + bias)"] = timeit("depthnet_pack", lambda: _lib.check(
                l.lss_depthnet_pack(_lib.ptr(wf), _lib.ptr(bfl), _lib.F32, D + 64, 512, _lib.ptr(packed),
                                    _lib.ptr(wdn), _lib.ptr(bdn), st()), "pack"))
        lift_prep(ctx_t, _lib.BF16)()
        lift_prep(ctx_f, _lib.F32)()
        if not args.only or "splat_fwd" in args.only:
            for m in ("warm", "step"):
                r[f"{m} splat_fwd nhwc bf16"] = stamped(bev_bf, _lib.NHWC, ctx_t, m)
                r[f"{m} splat_fwd nchw f32"] = stamped(bev_f, _lib.NCHW, ctx_f, m)
        r["splat_bwd nhwc bf16"] = timeit("splat_bwd", lambda: _lib.check(l.lss_splat_bwd(
            _lib.ptr(g_bf), _lib.BF16, _lib.NHWC, _lib.ptr(plan.cell_of), _lib.ptr(depth), _lib.ptr(ctx_t),
            _lib.BF16, dims, g, _lib.ptr(d_dn), _lib.BF16, st()), "bwd"))
        return r

    res = {"config": args.config, "kept": kept}
    nbytes = nprime * 4 + B * N * H * W * 64 * 2 + kept * 4 + (ncells + 1) * 4 + ncells * 64 * 2
    res["splat_alg_bytes_bf16"] = nbytes
    for name in args.libs.split(","):
        l = _lib.load() if name == "product" else _lib.open_library(
            os.path.join(REPO, "lss-carla_amd", "variants", name + ".so"))
        r = lib_ops(l)
        res[name] = r
        for k, v in r.items():
            extra = f"  {nbytes / v / 1e3:7.1f} GB/s alg" if (v and "nhwc bf16" in k and "splat_fwd" in k) else ""
            print(f"[{name}] {k:44s} {v} us{extra}", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
