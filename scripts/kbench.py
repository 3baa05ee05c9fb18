"""Kernel micro-benchmark: every hot-path op of config 3 timed in isolation, plus tuning variants of
lss_splat_fwd built with -D knobs (lss-carla_amd/variants/*.so).

Splat times come from kernel-stamped events (hipExtLaunchKernel: the kernel alone, no launch
overhead) in three cache states:
  warm  back-to-back launches
  cold  512 MiB written before each launch (L2 and Infinity Cache flushed)
  step  caches flushed, then the CSR and the lift prep rebuilt right before the splat -- the order of
        a training step, where the plan is built after the trunk (models.LiftSplatShoot.get_voxels)
  hot   as step, with ~0.3 ms of bf16 GEMMs before the plan (the trunk's clock / power state)

  python scripts/kbench.py --build-variants     # here (hipcc), before gpurun
  python scripts/kbench.py                      # on the GPU box
"""
import argparse
import ctypes as ct
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

VARIANTS = {
    "cpw2": ["LSS_CHUNKS_PER_WAVE=2"],     # two chunks per chunk wave (half the chunk waves)
    "cpw2_o0": ["LSS_CHUNKS_PER_WAVE=2", "LSS_INTERLEAVE=0"],
    "cpw3": ["LSS_CHUNKS_PER_WAVE=3"],
    "o0": ["LSS_INTERLEAVE=0"],            # chunks first always
}
VARIANTS_R1 = {  # round-1 knobs of the two-role kernel (kept for reference; pass --r1-variants)
    "skip_chunks": ["LSS_SPLAT_IMPL=0", "LSS_FWD_SKIP=1"],  # zero units only (timing decomposition; wrong output)
    "skip_zero": ["LSS_SPLAT_IMPL=0", "LSS_FWD_SKIP=2"],    # chunks only (timing decomposition; wrong output)
    "interleave": ["LSS_SPLAT_IMPL=0", "LSS_INTERLEAVE=1"],
    "gap8": ["LSS_SPLAT_IMPL=0", "LSS_CHUNK_GAP=8"],
}


def build_variants(r1=False):
    from lss_carla_amd import build
    import shutil
    vdir = os.path.join(REPO, "lss-carla_amd", "variants")
    shutil.rmtree(vdir, ignore_errors=True)  # stale variants of older ABIs would fail to load
    for name, defs in (VARIANTS_R1 if r1 else VARIANTS).items():
        print(name, build.build_variant(name, defs), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build-variants", action="store_true")
    ap.add_argument("--r1-variants", action="store_true", help="with --build-variants: the round-1 knob set")
    ap.add_argument("--config", default="c3")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--only", default="", help="run only ops whose name contains this (for rocprofv3 --pmc)")
    ap.add_argument("--variants", type=int, default=1, help="also time the variants/*.so builds")
    ap.add_argument("--variant-filter", default="", help="only variants whose name contains this")
    ap.add_argument("--cold", type=int, default=1, help="also time splat_fwd in the cold and step cache states")
    ap.add_argument("--lib", default="", help="use variants/<name>.so as THE library (ops included), for rocprofv3")
    args = ap.parse_args()
    if args.build_variants:
        build_variants(args.r1_variants)
        return
    import torch
    from lss_carla_amd import _lib, ops, synthetic as syn
    from oracle import lss_ref as ref

    if args.lib:
        _lib._lib = _lib.open_library(os.path.join(REPO, "lss-carla_amd", "variants", args.lib + ".so"))
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
        """Launch-to-launch time (includes the host's launch overhead for short kernels)."""
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
    ops.SORTED_DEPTH = True  # the plan carries pos_of, so the "(sorted depth)" rows get real weights
    plan = ops.plan_from_cameras(frustum, **rig, grid=grid, inverse="device")
    assert plan.pos_of is not None
    kept = int(plan.cell_start[-1])
    dims, g = plan.c_dims, grid.c_struct()
    ncells, nprime = grid.ncells(B), plan.nprime
    pinv, kinv = ops.camera_inverses(rig["post_rots"], rig["intrins"], "device")
    ro, tr, pt = [t.float().contiguous() for t in (rig["rots"], rig["trans"], rig["post_trans"])]

    def lib_plan(l, into=None):
        """cell_start / sorted_key / sorted_row built by library `l` (into the given buffers, if any)."""
        counts = torch.zeros(ncells, device=dev, dtype=torch.int32)
        slot = torch.empty(nprime, device=dev, dtype=torch.int32)
        cell_of = torch.empty(nprime, device=dev, dtype=torch.int32)
        _lib.check(l.lss_geometry_cells(_lib.ptr(frustum), _lib.ptr(ro), _lib.ptr(tr), _lib.ptr(kinv),
                                        _lib.ptr(pinv), _lib.ptr(pt), dims, g, None, _lib.ptr(cell_of),
                                        _lib.ptr(counts), _lib.ptr(slot), st()), "geom")
        if into is not None:
            cs, sk, sr, po = into
        else:
            cs = torch.empty(ncells + 1, device=dev, dtype=torch.int32)
            sk = torch.empty(nprime, device=dev, dtype=torch.int64)
            sr = torch.empty(nprime, device=dev, dtype=torch.int32)
            po = torch.empty(nprime, device=dev, dtype=torch.int32)
        scr = torch.empty(int(l.lss_csr_scratch_bytes(ncells, nprime)), device=dev, dtype=torch.uint8)
        _lib.check(l.lss_csr_build(_lib.ptr(cell_of), _lib.ptr(slot), nprime, _lib.ptr(counts), ncells, dims,
                                   _lib.ptr(cs), _lib.ptr(sk), _lib.ptr(sr), _lib.ptr(po), _lib.ptr(scr), st()), "csr")
        return cs, sk, sr, po

    def named(name, fn, *a):
        timeit.name = name
        return timeit(fn, *a)

    def lib_rows(l, tag):
        """Launch-to-launch rows of library `l` for the plan pieces, the fused lift and the splat bwd."""
        counts = torch.zeros(ncells, device=dev, dtype=torch.int32)
        slot = torch.empty(nprime, device=dev, dtype=torch.int32)
        cell_of = torch.empty(nprime, device=dev, dtype=torch.int32)
        cs = torch.empty(ncells + 1, device=dev, dtype=torch.int32)
        sk = torch.empty(nprime, device=dev, dtype=torch.int64)
        sr = torch.empty(nprime, device=dev, dtype=torch.int32)
        po = torch.empty(nprime, device=dev, dtype=torch.int32)
        scr = torch.empty(int(l.lss_csr_scratch_bytes(ncells, nprime)), device=dev, dtype=torch.uint8)
        geom = lambda: _lib.check(l.lss_geometry_cells(  # noqa: E731
            _lib.ptr(frustum), _lib.ptr(ro), _lib.ptr(tr), _lib.ptr(kinv), _lib.ptr(pinv), _lib.ptr(pt), dims, g,
            None, _lib.ptr(cell_of), _lib.ptr(counts), _lib.ptr(slot), st()), "geom")
        csr = lambda: _lib.check(l.lss_csr_build(  # noqa: E731
            _lib.ptr(cell_of), _lib.ptr(slot), nprime, _lib.ptr(counts), ncells, dims, _lib.ptr(cs), _lib.ptr(sk),
            _lib.ptr(sr), _lib.ptr(po), _lib.ptr(scr), st()), "csr")

        def geom_only():
            counts.zero_()
            geom()

        def plan3():
            counts.zero_()
            geom()
            csr()
        wsb = torch.zeros(int(l.lss_csr_workspace_bytes(ncells)), device=dev, dtype=torch.uint8)
        counts_ws = torch.zeros(ncells, device=dev, dtype=torch.int32)

        def plan_ws():  # persistent zero-filled counts + look-back scan workspace (what ops uses)
            _lib.check(l.lss_geometry_cells(_lib.ptr(frustum), _lib.ptr(ro), _lib.ptr(tr), _lib.ptr(kinv),
                                            _lib.ptr(pinv), _lib.ptr(pt), dims, g, None, _lib.ptr(cell_of),
                                            _lib.ptr(counts_ws), _lib.ptr(slot), st()), "geom")
            _lib.check(l.lss_csr_build_ws(_lib.ptr(cell_of), _lib.ptr(slot), nprime, _lib.ptr(counts_ws), ncells, dims,
                                          _lib.ptr(cs), _lib.ptr(sk), _lib.ptr(sr), _lib.ptr(po), _lib.ptr(scr),
                                          _lib.ptr(wsb), st()), "csr_ws")
        axes = ops.frustum_axes(frustum)

        def plan_ws_axes():  # + the frustum as its three axes (what ops uses for create_frustum's frustum)
            _lib.check(l.lss_geometry_cells_axes(_lib.ptr(axes), _lib.ptr(ro), _lib.ptr(tr), _lib.ptr(kinv),
                                                 _lib.ptr(pinv), _lib.ptr(pt), dims, g, None, _lib.ptr(cell_of),
                                                 _lib.ptr(counts_ws), _lib.ptr(slot), st()), "geom")
            _lib.check(l.lss_csr_build_ws(_lib.ptr(cell_of), _lib.ptr(slot), nprime, _lib.ptr(counts_ws), ncells, dims,
                                          _lib.ptr(cs), _lib.ptr(sk), _lib.ptr(sr), _lib.ptr(po), _lib.ptr(scr),
                                          _lib.ptr(wsb), st()), "csr_ws")
        res[f"geometry+csr_build_ws (no memset){tag}"] = named("csr_build", plan_ws)
        res[f"geometry_axes+csr_build_ws (no memset){tag}"] = named("csr_build", plan_ws_axes)
        plan_ws()
        if not (torch.equal(cs, plan.cell_start) and torch.equal(sk, plan.sorted_key)):
            print(f"WARNING {tag}: workspace CSR differs from the product plan", flush=True)
        res[f"memset counts{tag}"] = named("memset counts", lambda: counts.zero_())
        res[f"memset+geometry_cells{tag}"] = named("geometry_cells", geom_only)
        res[f"memset+geometry+csr_build{tag}"] = named("csr_build", plan3)
        plan3()
        if not (torch.equal(cs, plan.cell_start) and torch.equal(sk, plan.sorted_key)):
            print(f"WARNING {tag}: CSR differs from the product plan", flush=True)
        res[f"depthnet_lift (fused, MFMA){tag}"] = named("depthnet_lift", lambda: _lib.check(l.lss_depthnet_lift(
            _lib.ptr(feat), _lib.ptr(wdn), _lib.ptr(bdn), _lib.BF16, 512, dims, _lib.ptr(depth), _lib.ptr(ctx_t),
            _lib.BF16, None, None, None, None, None, 0, st()), "depthnet_lift"))
        res[f"splat_bwd nhwc bf16{tag}"] = named("splat_bwd nhwc bf16", lambda: _lib.check(l.lss_splat_bwd(
            _lib.ptr(g_bf), _lib.BF16, _lib.NHWC, _lib.ptr(plan.cell_of), _lib.ptr(depth), _lib.ptr(ctx_t),
            _lib.BF16, dims, g, _lib.ptr(d_dn), _lib.BF16, st()), "bwd"))

    depth = torch.empty(B * N, D, H, W, device=dev)
    ctx_t = torch.empty(B * N * H * W, 64, device=dev, dtype=torch.bfloat16)  # as ops.LiftSplat for bf16 input
    bev_bf = torch.empty(B, Z * 64, X, Y, device=dev, dtype=torch.bfloat16, memory_format=torch.channels_last)
    bev_f = torch.empty(B, Z * 64, X, Y, device=dev)
    res["memset_bev_bf16_41MB"] = named("memset_bev_bf16_41MB", lambda: bev_bf.zero_())
    res["memset_bev_f32_82MB"] = named("memset_bev_f32_82MB", lambda: bev_f.zero_())
    res["copy_bev_f32_82MB"] = named("copy_bev_f32_82MB", lambda: bev_f.copy_(bev_bf))
    res["plan_total(device inv)"] = named("plan_total(device inv)",
                                          lambda: ops.plan_from_cameras(frustum, **rig, grid=grid, inverse="device"))
    sdepth = torch.empty(nprime, device=dev)  # depth weights in CSR order (lift with pos_of)
    res["lift_prep"] = named("lift_prep", lambda: _lib.check(lib.lss_lift_prep(
        _lib.ptr(dn), _lib.BF16, dims, _lib.ptr(depth), _lib.ptr(ctx_t), _lib.BF16, None, None, None, None, None, 0, st()), "lift"))
    res["lift_prep (+sorted depth)"] = named("lift_prep (+sorted depth)", lambda: _lib.check(lib.lss_lift_prep(
        _lib.ptr(dn), _lib.BF16, dims, _lib.ptr(depth), _lib.ptr(ctx_t), _lib.BF16, _lib.ptr(plan.pos_of),
        _lib.ptr(sdepth), None, None, None, 0, st()), "lift"))
    feat = torch.randn(B * N, 512, H, W, device=dev).to(torch.bfloat16)
    wdn = (torch.randn(D + 64, 512, 1, 1, device=dev) * 0.05).to(torch.bfloat16)
    bdn = torch.zeros(D + 64, device=dev, dtype=torch.bfloat16)
    res["depthnet conv (MIOpen, bf16)"] = named("depthnet conv (MIOpen, bf16)",
                                                lambda: torch.nn.functional.conv2d(feat, wdn, bdn))
    res["depthnet_lift (fused, MFMA)"] = named("depthnet_lift (fused, MFMA)", lambda: _lib.check(lib.lss_depthnet_lift(
        _lib.ptr(feat), _lib.ptr(wdn), _lib.ptr(bdn), _lib.BF16, 512, dims, _lib.ptr(depth), _lib.ptr(ctx_t), _lib.BF16,
        None, None, None, None, None, 0, st()), "depthnet_lift"))
    res["depthnet_lift (+sorted depth)"] = named("depthnet_lift (+sorted depth)", lambda: _lib.check(
        lib.lss_depthnet_lift(_lib.ptr(feat), _lib.ptr(wdn), _lib.ptr(bdn), _lib.BF16, 512, dims, _lib.ptr(depth),
                              _lib.ptr(ctx_t), _lib.BF16, _lib.ptr(plan.pos_of), _lib.ptr(sdepth), None, None, None, 0, st()),
        "depthnet_lift"))
    ctx_f = torch.empty(B * N * H * W, 64, device=dev)
    _lib.check(lib.lss_lift_prep(_lib.ptr(dn), _lib.BF16, dims, _lib.ptr(depth), _lib.ptr(ctx_f), _lib.F32,
                                 _lib.ptr(plan.pos_of), _lib.ptr(sdepth), None, None, None, 0, st()), "lift")

    pcsr = (plan.cell_start, plan.sorted_key, plan.sorted_row, plan.pos_of)

    def fwd(l, out, layout, csr=pcsr, ctx=None, sd=None):
        cs, sk, its, _ = csr
        ctx = ctx_t if ctx is None else ctx
        return lambda: _lib.check(l.lss_splat_fwd(_lib.ptr(depth), _lib.ptr(ctx), _lib.dtype_code(ctx.dtype), None,
                                                  _lib.ptr(cs), _lib.ptr(sk), _lib.ptr(its), _lib.ptr(sd), dims, g,
                                                  _lib.ptr(out), _lib.dtype_code(out.dtype), layout, 0, st(), None, None),
                                  "fwd")

    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    gemm_a = torch.randn(4096, 4096, device=dev).to(torch.bfloat16)
    gemm_c = torch.empty_like(gemm_a)

    def memset_after(mode):
        """41 MB bf16 BEV memset in the given cache / clock state (kernel time only, hipEvents)."""
        tot = 0.0
        for i in range(23):
            flush.zero_()
            if mode == "hot":
                for _ in range(4):
                    torch.matmul(gemm_a, gemm_a, out=gemm_c)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            bev_bf.zero_()
            e1.record()
            torch.cuda.synchronize()
            if i >= 3:
                tot += e0.elapsed_time(e1)
        return tot / 20 * 1e3
    if not args.only:
        res["memset_bev_bf16_41MB (flushed)"] = memset_after("cold")
        res["memset_bev_bf16_41MB (flushed, after GEMMs)"] = memset_after("hot")

    def stamped(l, out, layout, csr=pcsr, ctx=None, mode="warm", iters=20, sd=None):
        cs, sk, its, po = csr
        ctx = ctx_t if ctx is None else ctx
        tot = 0.0
        for i in range(iters + 3):
            if mode in ("cold", "step", "hot"):
                flush.zero_()
            if mode == "hot":
                for _ in range(4):
                    torch.matmul(gemm_a, gemm_a, out=gemm_c)
            if mode in ("step", "hot"):
                lib_plan(l, csr)
                _lib.check(l.lss_lift_prep(_lib.ptr(dn), _lib.BF16, dims, _lib.ptr(depth), _lib.ptr(ctx),
                                           _lib.dtype_code(ctx.dtype), _lib.ptr(po if sd is not None else None),
                                           _lib.ptr(sd), None, None, None, 0, st()), "lift")
            a, b = ct.c_void_p(), ct.c_void_p()
            l.lss_event_create(ct.byref(a))
            l.lss_event_create(ct.byref(b))
            _lib.check(l.lss_splat_fwd(_lib.ptr(depth), _lib.ptr(ctx), _lib.dtype_code(ctx.dtype), None, _lib.ptr(cs),
                                       _lib.ptr(sk), _lib.ptr(its), _lib.ptr(sd), dims, g, _lib.ptr(out),
                                       _lib.dtype_code(out.dtype), layout, 0, st(), a, b), "fwd")
            ms = ct.c_float()
            l.lss_event_elapsed_ms(a, b, ct.byref(ms))
            if i >= 3:
                tot += ms.value
            l.lss_event_destroy(a)
            l.lss_event_destroy(b)
        return tot / iters * 1e3

    modes = ["warm"] + (["cold", "step", "hot"] if args.cold else [])
    fwd(lib, bev_bf, _lib.NHWC)()
    ref_out = bev_bf.clone()
    if not args.only or "splat_fwd" in args.only:
        res["launch-to-launch splat_fwd nhwc bf16"] = named("splat_fwd nhwc bf16", fwd(lib, bev_bf, _lib.NHWC))
        fwd(lib, bev_bf, _lib.NHWC, sd=sdepth)()
        if not torch.equal(bev_bf, ref_out):
            print("WARNING: sorted-depth splat differs from the gather splat", flush=True)
        for m in modes:
            res[f"{m} splat_fwd nhwc bf16"] = stamped(lib, bev_bf, _lib.NHWC, mode=m)
            res[f"{m} splat_fwd nhwc bf16 (sorted depth)"] = stamped(lib, bev_bf, _lib.NHWC, mode=m, sd=sdepth)
            res[f"{m} splat_fwd nhwc bf16 (f32 ctx)"] = stamped(lib, bev_bf, _lib.NHWC, ctx=ctx_f, mode=m)
        res["warm splat_fwd nchw f32"] = stamped(lib, bev_f, _lib.NCHW)
        res["step splat_fwd nchw f32"] = stamped(lib, bev_f, _lib.NCHW, mode="step")
        res["warm splat_fwd nchw f32 (f32 ctx)"] = stamped(lib, bev_f, _lib.NCHW, ctx=ctx_f)
    # the timing modes above rewrote ctx_t (the "step" mode reruns the lift): fresh reference output
    fwd(lib, bev_bf, _lib.NHWC)()
    ref_out = bev_bf.clone()
    g_bf = torch.randn(B, Z * 64, X, Y, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    d_dn = torch.empty_like(dn)
    def restore_lift():  # lib_rows rewrites depth / ctx_t through the fused lift
        _lib.check(lib.lss_lift_prep(_lib.ptr(dn), _lib.BF16, dims, _lib.ptr(depth), _lib.ptr(ctx_t), _lib.BF16, None,
                                     None, None, None, None, 0, st()), "lift")
    lib_rows(lib, "")
    restore_lift()
    for path in sorted(glob.glob(os.path.join(REPO, "lss-carla_amd", "variants", "*.so"))) if args.variants else []:
        name = os.path.basename(path)[:-3]
        if args.variant_filter and args.variant_filter not in name:
            continue
        vl = _lib.open_library(path)
        lib_rows(vl, f" [{name}]")
        restore_lift()
        vcsr = lib_plan(vl)
        fwd(vl, bev_bf, _lib.NHWC, vcsr)()
        if not torch.equal(bev_bf, ref_out):
            print(f"WARNING variant {name}: output differs from the product kernel", flush=True)
        vsd = torch.empty(nprime, device=dev)
        _lib.check(vl.lss_lift_prep(_lib.ptr(dn), _lib.BF16, dims, _lib.ptr(depth), _lib.ptr(ctx_t), _lib.BF16,
                                    _lib.ptr(vcsr[3]), _lib.ptr(vsd), None, None, None, 0, st()), "lift")
        for m in modes:
            res[f"{m} splat_fwd nhwc bf16 [{name}]"] = stamped(vl, bev_bf, _lib.NHWC, vcsr, mode=m)
            res[f"{m} splat_fwd nhwc bf16 (sorted depth) [{name}]"] = stamped(vl, bev_bf, _lib.NHWC, vcsr, mode=m,
                                                                               sd=vsd)
        # NCHW fp32 (the reference layout): output vs the product kernel, then timed
        ref_f = bev_f.clone()
        fwd(lib, ref_f, _lib.NCHW)()
        fwd(vl, bev_f, _lib.NCHW, vcsr)()
        if not torch.equal(bev_f, ref_f):
            print(f"WARNING variant {name}: NCHW output differs from the product kernel", flush=True)
        res[f"warm splat_fwd nchw f32 [{name}]"] = stamped(vl, bev_f, _lib.NCHW, vcsr)
        res[f"step splat_fwd nchw f32 [{name}]"] = stamped(vl, bev_f, _lib.NCHW, vcsr, mode="step")
        res[f"warm splat_fwd nchw f32 (f32 ctx) [{name}]"] = stamped(vl, bev_f, _lib.NCHW, vcsr, ctx=ctx_f)
    rows = torch.empty(ncells * 64, device=dev)
    g_f = torch.randn(B, Z * 64, X, Y, device=dev)
    res["bev_rows nchw f32"] = named("bev_rows nchw f32", lambda: _lib.check(lib.lss_bev_rows(
        _lib.ptr(g_f), _lib.F32, _lib.ptr(plan.cell_start), dims, g, _lib.ptr(rows), st()), "rows"))
    nbytes = (nprime * 4 + B * N * H * W * 64 * 2 + kept * 4 + (ncells + 1) * 4 + ncells * 64 * 2)
    for k, v in res.items():
        extra = f"  {nbytes / v / 1e3:7.1f} GB/s alg" if "splat_fwd nhwc bf16" in k else ""
        print(f"{k:52s} {v:9.2f} us{extra}")
    print(json.dumps({"kept": kept, "alg_bytes_fwd_bf16_ctx": nbytes}))


if __name__ == "__main__":
    main()
