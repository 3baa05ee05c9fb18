"""LSS fwd+bwd frames/sec (BASELINE.json metric) on 1..8 MI355X, one process per GPU.

Workload (config 3 of BASELINE.json): B=8 samples x 6 cameras x 128x352 per GPU,
D=41, 200x200 BEV, bf16 autocast, full training step of train_simbev.py:229-248
(forward, SimpleLoss, backward, clip_grad_norm_(5.0), Adam step). Synthetic
SimBEV-shaped inputs, random-init weights. The step is replayed as
two HIP graphs (train_step.TrainStep: fwd+loss+bwd | clip+Adam) with one RCCL
all-reduce of the flat fp32 gradient between them; --graph 0 runs it eagerly (DDP).
For N>1: torchrun, one rank per GPU, B=8 per rank (weak scaling).

Also reported on the same JSON line:
  roofline      the fused lift+splat forward kernel (lss_splat_fwd): algorithmic
                bytes per launch / its average launch time (HIP events on the
                launch stream, over the timed steps) vs 8 TB/s HBM peak
  cpu_baseline  the CPU oracle (restatement of the reference's path, fp32 eager,
                conv stacks on the CPU) timed on this host, rank 0, N=1 only
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# MIOpen find results (which conv solver per shape) and compiled kernels, kept in-tree so a
# fresh box does not repeat the exhaustive search (tuning/README.md). Must precede torch init.
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(REPO, "tuning", "miopen", "db"))
os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", os.path.join(REPO, "tuning", "miopen", "cache"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "LSS fwd+bwd frames/sec at B=8, 6×128×352, D=41 → 200×200 BEV; 1/2/4/8 GPU"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8, help="samples per GPU")
    ap.add_argument("--config", default="c3")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--bev-layout", default="nhwc", choices=["nhwc", "nchw"])
    ap.add_argument("--trunk-channels-last", type=int, default=0)
    ap.add_argument("--trunk-fp32", type=int, default=0, help="run CamEncode outside autocast")
    ap.add_argument("--dw-impl", default="hip", choices=["hip", "miopen", "native", "fp32"],
                    help="depthwise convs of the trunk: HIP kernels, MIOpen, PyTorch native, MIOpen in fp32")
    ap.add_argument("--miopen-find", type=int, default=1, help="torch.backends.cudnn.benchmark (MIOpen find)")
    ap.add_argument("--hip-bn", type=int, default=1, help="BatchNorm + activation on the lss_bn_* kernels")
    ap.add_argument("--bn-native", default="", help="with --hip-bn 0: BatchNorm on PyTorch's native kernels: "
                                                    "'', 'trunk', 'bev', 'all'")
    ap.add_argument("--inverse", default="host", choices=["host", "device"])
    ap.add_argument("--fuse-depthnet", type=int, default=1, help="depthnet 1x1 conv inside the lift kernel (MFMA)")
    ap.add_argument("--graph", type=int, default=1,
                    help="replay the step as two HIP graphs (fwd+bwd, clip+Adam) with the gradient all-reduce "
                         "between them; 0 = eager (DDP for N>1)")
    ap.add_argument("--flat-params", type=int, default=1,
                    help="trainable parameters as one fp32 master tensor with one bf16 working copy per step")
    ap.add_argument("--graph-splat-timing", type=int, default=0,
                    help="also bracket the captured splat launch with event-record nodes (upper bound)")
    ap.add_argument("--profile-steps", type=int, default=8,
                    help="steps after the timed region on which the splat kernel is timed (graph replays, then eager)")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "splat_fwd_traffic.json"))
    return ap.parse_args()


def setup_dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, torch.device("cuda", local if world > 1 else 0)


def splat_fwd_bytes(B, N, D, H, W, X, Y, Z, kept, out_bytes, ctx_bytes) -> int:
    """Algorithmic bytes of one lss_splat_fwd launch."""
    nprime = B * N * D * H * W
    ncells = B * Z * X * Y
    return (nprime * 4                    # depth (fp32)
            + B * N * H * W * 64 * ctx_bytes  # context rows (the depthnet output's type: bf16 under autocast)
            + kept * 4                    # sorted point ids
            + (ncells + 1) * 4            # cell_start
            + ncells * 64 * out_bytes)    # dense BEV, every element written once


def build_model(args, dev, cfg, gc, dac):
    import lss_carla_amd as L

    model = L.compile_model(gc, dac, outC=1).to(dev)
    model.bev_layout = args.bev_layout
    model.inverse = args.inverse
    model.fuse_depthnet = bool(args.fuse_depthnet)
    if args.bev_layout == "nhwc":
        model.bevencode.to(memory_format=torch.channels_last)
    if args.trunk_channels_last:
        model.camencode.to(memory_format=torch.channels_last)
    from lss_carla_amd import norm
    norm.USE_HIP_BN = bool(args.hip_bn)
    from lss_carla_amd.efficientnet import set_depthwise_impl
    set_depthwise_impl(model.camencode.trunk, args.dw_impl)
    if args.bn_native:
        from lss_carla_amd.efficientnet import set_batchnorm_native
        if args.bn_native in ("trunk", "all"):
            set_batchnorm_native(model.camencode)
        if args.bn_native in ("bev", "all"):
            set_batchnorm_native(model.bevencode)
    if args.trunk_fp32:
        ce = model.camencode
        fwd = ce.depthnet_out

        def depthnet_out_fp32(x):
            with torch.autocast("cuda", enabled=False):
                return fwd(x.float())
        ce.depthnet_out = depthnet_out_fp32
    model.train()
    return model


def cpu_baseline(model, cfg, gc, seconds: float):
    """Reference path on the host: oracle geometry/lift/splat + the same conv stacks, fp32, eager."""
    import copy

    from oracle import lss_ref as ref
    from lss_carla_amd import synthetic as syn
    import lss_carla_amd as L

    threads = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    torch.set_num_threads(threads)
    cpu_model = copy.deepcopy(model).to("cpu").float()
    cpu_model.bevencode.to(memory_format=torch.contiguous_format)
    cpu_model.camencode.to(memory_format=torch.contiguous_format)
    cpu_model.train()
    B = 1
    rig = syn.make_rig(B, cfg["N"], cfg["final_dim"], seed=0)
    imgs = syn.make_images(B, cfg["N"], cfg["final_dim"])
    labels = syn.make_labels(B, 200, 200)
    frustum = cpu_model.frustum.detach()
    dx, bx, nx = ref.gen_dx_bx(gc["xbound"], gc["ybound"], gc["zbound"])
    loss_fn = L.SimpleLoss(2.13)
    opt = torch.optim.Adam(cpu_model.parameters(), lr=1e-3, weight_decay=1e-7)

    def step():
        opt.zero_grad()
        out = ref.full_forward(cpu_model.camencode.depthnet_out, cpu_model.bevencode, frustum, imgs, rig["rots"],
                               rig["trans"], rig["intrins"], rig["post_rots"], rig["post_trans"], dx, bx, nx,
                               cpu_model.D)
        loss = loss_fn(out, labels)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(cpu_model.parameters(), 5.0)
        opt.step()

    step()  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        step()
        n += 1
        el = time.perf_counter() - t0
        if (el >= seconds and n >= 2) or el >= 2 * seconds:
            break
    return {"value": round(B * n / el, 4), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"B=1 x {cfg['N']} cams x {cfg['final_dim'][0]}x{cfg['final_dim'][1]}, {n} full training "
                      f"steps (fwd+bwd+clip+Adam) in {el:.1f} s, fp32 eager, oracle lift/splat + same conv stacks"}


def main():
    args = parse()
    world, rank, dev = setup_dist()
    torch.backends.cudnn.benchmark = bool(args.miopen_find)
    from lss_carla_amd import ops, parallel, synthetic as syn
    from lss_carla_amd.flat_params import FlatParams
    from lss_carla_amd.train_step import TrainStep
    import lss_carla_amd as L

    cfg, gc, dac = syn.config_confs(args.config)
    B, N, fd = args.batch, cfg["N"], cfg["final_dim"]
    torch.manual_seed(1234 + rank)
    if args.graph:
        args.inverse = "device"  # inverse='host' is a device->host round trip: not capturable
    model = build_model(args, dev, cfg, gc, dac)
    amp_dtype = torch.bfloat16 if args.dtype == "bf16" else None
    flat = None
    if args.graph or args.flat_params:
        # one process per GPU without DDP: identical replicas, one flat gradient all-reduce
        parallel.broadcast_state(model)
        parallel.freeze_unused(model)
        flat = FlatParams(model, cast_dtype=amp_dtype) if args.flat_params else None
    if flat is not None:
        fwd, params = flat.bind(model), [flat.master]
    else:
        fwd = model if (args.graph or world == 1) else parallel.make_data_parallel(model, dev)
        params = [p for p in model.parameters() if p.requires_grad]
    loss_fn = L.SimpleLoss(2.13).to(dev)
    opt = torch.optim.Adam(params, lr=1e-3, weight_decay=1e-7, fused=True, capturable=bool(args.graph))
    rig = {k: v.to(dev) for k, v in syn.make_rig(B, N, fd, seed=rank).items()}
    imgs = syn.make_images(B, N, fd, seed=rank).to(dev)
    if args.trunk_channels_last:
        imgs = imgs.contiguous()
    X, Y, Z = ops.GridSpec.from_conf(gc).nx
    labels = syn.make_labels(B, X, Y, seed=rank).to(dev)

    train = TrainStep(fwd, (imgs, rig["rots"], rig["trans"], rig["intrins"], rig["post_rots"], rig["post_trans"]),
                      labels, loss_fn, opt, params, all_reduce=bool(args.graph or args.flat_params),
                      amp_dtype=amp_dtype, max_grad_norm=5.0)
    t_w = time.perf_counter()

    def first(i):
        if i == 0:
            torch.cuda.synchronize()
            log(f"[rank {rank}] first step done in {time.perf_counter() - t_w:.1f} s")

    if args.graph:
        # eager warm-up on a side stream (MIOpen find, optimizer state), capture, 2 untimed replays
        # opt-in: event-record nodes around the captured splat launch (an upper bound: each node
        # adds a marker packet to the interval; measured 14.6 us bracket vs ~12 us kernel in rocprof)
        ops.SPLAT_PROFILE.capture = bool(args.graph_splat_timing)
        train.capture(warmup=max(args.warmup, 2), on_warmup=first)
        ops.SPLAT_PROFILE.capture = False
        for _ in range(2):
            train()
    else:
        for i in range(args.warmup):
            train()
            first(i)
    torch.cuda.synchronize()
    log(f"[rank {rank}] warmup {args.warmup} steps in {time.perf_counter() - t_w:.1f} s"
        + (" (incl. graph capture)" if args.graph else ""))

    ops.SPLAT_PROFILE.reset(not args.graph)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = train()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    graph_bracket_ms = graph_marker_ms = None
    if args.graph:
        # Primary: the captured splat launch, bracketed by hipEvent-record nodes in the graph,
        # read after each of `profile_steps` further replays (same cache state as the timed steps).
        if ops.SPLAT_PROFILE.graph_pairs:
            gms = []
            try:
                for _ in range(args.profile_steps):
                    train()
                    torch.cuda.synchronize()
                    gms.append(ops.SPLAT_PROFILE.graph_ms())
                graph_bracket_ms = sum(g[0] for g in gms) / len(gms)
                graph_marker_ms = sum(g[1] for g in gms) / len(gms)
            except RuntimeError as e:  # event-record nodes unsupported: fall back to the eager timing
                log(f"[rank {rank}] captured splat timing unavailable ({e}); timing eager steps")
        # Secondary: kernel-stamped events (hipExtLaunchKernel) on eager steps, same inputs
        train.eager()  # the first eager step after the replays runs cold: not timed
        torch.cuda.synchronize()
        ops.SPLAT_PROFILE.reset(True)
        for _ in range(args.profile_steps):
            train.eager()
        torch.cuda.synchronize()
    ops.SPLAT_PROFILE.enabled = False
    splat_eager_ms = ops.SPLAT_PROFILE.avg_ms()
    ops.SPLAT_PROFILE.release()
    splat_ms = splat_eager_ms
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    log(f"[rank {rank}] {args.steps} steps in {elapsed:.3f} s, loss {loss.item():.4f}")

    if rank == 0:
        D, H, W = model.frustum.shape[:3]
        with torch.no_grad():
            plan = model.plan(rig["rots"], rig["trans"], rig["intrins"], rig["post_rots"], rig["post_trans"])
            kept = int(plan.cell_start[-1].item())
        out_bytes = 2 if amp_dtype is not None else 4
        nbytes = splat_fwd_bytes(B, N, D, H, W, X, Y, Z, kept, out_bytes, ctx_bytes=out_bytes)
        achieved = nbytes / (splat_ms * 1e-3) / 1e9 if splat_ms else None
        traffic = None
        if os.path.exists(args.traffic_json):
            try:
                with open(args.traffic_json) as f:
                    tj = json.load(f)
                if tj.get("config") == args.config and tj.get("out_bytes") == out_bytes:
                    traffic = tj.get("hbm_bytes_per_launch")
            except (OSError, ValueError):
                traffic = None
        frames = world * B * args.steps
        res = {
            "metric": METRIC, "value": round(frames / elapsed, 3), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (SimBEV-shaped rig, random-init weights)",
            "config": {"workload": f"{args.config}: B={B}/GPU x {N} cams x {fd[0]}x{fd[1]}, D={D}, {X}x{Y} BEV, "
                                   "full train step (fwd+loss+bwd+clip+Adam)",
                       "global_batch": world * B, "parallelism": f"dp{world}", "bev_layout": args.bev_layout,
                       "inverse": args.inverse, "fuse_depthnet": bool(args.fuse_depthnet),
                       "depthwise": args.dw_impl, "batchnorm": "hip" if args.hip_bn else "miopen",
                       "step": "hipgraph" if args.graph else "eager", "flat_params": bool(args.flat_params)},
            "roofline": {"kernel": "lss_splat_fwd", "bound": "hbm",
                         "achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None, "traffic": traffic,
                         "algorithmic_bytes": nbytes, "avg_launch_us": round(splat_ms * 1e3, 2) if splat_ms else None,
                         "timed_in": "eager steps after the timed replays, kernel-stamped hipEvents",
                         **({"graph_bracket_us": round(graph_bracket_ms * 1e3, 2),
                             "graph_empty_pair_us": round(graph_marker_ms * 1e3, 2)} if graph_bracket_ms else {})},
        }
        if args.cpu_baseline and world == 1:
            log("[rank 0] timing the CPU baseline ...")
            res["cpu_baseline"] = cpu_baseline(model, cfg, gc, args.cpu_seconds)
        else:
            res["cpu_baseline"] = None
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
