"""The splat forward of one BASELINE config, alone, for rocprofv3 --pmc passes (bench.py runs this as a
child process under `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` to measure the kernel's HBM
traffic in the same run that times it).

  rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_splat_fwd -d DIR -o run --output-format csv -- \
      python3 scripts/splat_pmc.py --config c3 --dtype bf16 --layout nhwc
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--batch", type=int, default=0, help="samples (0: the config's own B)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--layout", default="nhwc", choices=["nhwc", "nchw"])
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    import torch
    from lss_carla_amd import _lib, ops, synthetic as syn

    dev = torch.device("cuda:0")
    cfg, gc, dac = syn.config_confs(args.config)
    B, N, fd = args.batch or cfg["B"], cfg["N"], cfg["final_dim"]
    import lss_carla_amd as L
    m = L.compile_model(gc, dac, 1)
    frustum = m.frustum.detach().to(dev)
    D, H, W = frustum.shape[:3]
    rig = {k: v.to(dev) for k, v in syn.make_rig(B, N, fd).items()}
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    layout = _lib.NHWC if args.layout == "nhwc" else _lib.NCHW
    dn = syn.make_depthnet_out(B, N, D, H, W).to(dev, dt)
    with torch.no_grad():
        for _ in range(args.iters):
            plan = ops.plan_from_cameras(frustum, **rig, grid=ops.GridSpec.from_conf(gc))
            ops.lift_splat(dn, plan, dt, layout)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
