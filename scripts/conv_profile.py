"""torch.profiler view of one bench training step, grouped by op and input shape (conv-stack triage)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(REPO, "tuning", "miopen", "db"))
os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", os.path.join(REPO, "tuning", "miopen", "cache"))

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402


def main():
    sys.argv = ["bench.py"] + sys.argv[1:]
    args = bench.parse()
    torch.backends.cudnn.benchmark = bool(args.miopen_find)
    from lss_carla_amd import synthetic as syn
    import lss_carla_amd as L
    dev = torch.device("cuda:0")
    cfg, gc, dac = syn.config_confs("c3")
    model = bench.build_model(args, dev, cfg, gc, dac)
    B, N, fd = 8, 6, cfg["final_dim"]
    rig = {k: v.to(dev) for k, v in syn.make_rig(B, N, fd).items()}
    imgs = syn.make_images(B, N, fd).to(dev)
    labels = syn.make_labels(B, 200, 200).to(dev)
    loss_fn = L.SimpleLoss(2.13).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True)

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(imgs, rig["rots"], rig["trans"], rig["intrins"], rig["post_rots"], rig["post_trans"])
        loss_fn(out.float(), labels).backward()
        opt.step()

    for _ in range(4):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for _ in range(2):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=60,
                                                            max_name_column_width=40, max_shapes_column_width=110))


if __name__ == "__main__":
    main()
