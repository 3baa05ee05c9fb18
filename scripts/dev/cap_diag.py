"""Diagnostics of the captured c3 TrainStep: gradient buffers after graph replays vs eager steps."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(REPO, "tuning", "miopen", "db"))
os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", os.path.join(REPO, "tuning", "miopen", "cache"))

import torch  # noqa: E402

import lss_carla_amd as L  # noqa: E402
from lss_carla_amd import ops, parallel, synthetic as syn  # noqa: E402
from lss_carla_amd.flat_params import FlatParamGroups, FlatParams, lss_backward_groups  # noqa: E402
from lss_carla_amd.train_step import TrainStep  # noqa: E402

DEV = torch.device("cuda:0")
groups = int(sys.argv[1]) if len(sys.argv) > 1 else 1
torch.backends.cudnn.benchmark = True
cfg, gc, dac = syn.config_confs("c3")
B, N, fd = cfg["B"], cfg["N"], cfg["final_dim"]
torch.manual_seed(7)
model = L.compile_model(gc, dac, outC=1).to(DEV)
model.bev_layout, model.fuse_depthnet, model.inverse = "nhwc", True, "device"
model.bevencode.to(memory_format=torch.channels_last)
model.camencode.dropout.p = 0.0
model.bevencode.dropout.p = 0.0
model.camencode.trunk._global_params.drop_connect_rate = 0.0
parallel.freeze_unused(model)
flat = FlatParamGroups(model, lss_backward_groups(), cast_dtype=torch.bfloat16) if groups else \
    FlatParams(model, cast_dtype=torch.bfloat16)
masters = flat.masters if groups else [flat.master]
rig = {k: v.to(DEV) for k, v in syn.make_rig(B, N, fd, seed=0).items()}
X, Y, _ = ops.GridSpec.from_conf(gc).nx
imgs = syn.make_images(B, N, fd, seed=3).to(DEV)
labels = syn.make_labels(B, X, Y, seed=3).to(DEV)
inputs = (imgs, rig["rots"], rig["trans"], rig["intrins"], rig["post_rots"], rig["post_trans"])
opt = torch.optim.Adam(masters, lr=1e-3, weight_decay=1e-7, fused=True, capturable=True)
step = TrainStep(flat.bind(model), inputs, labels, L.SimpleLoss(2.13).to(DEV), opt, masters, all_reduce=True,
                 amp_dtype=torch.bfloat16, max_grad_norm=5.0)
mode = sys.argv[2] if len(sys.argv) > 2 else "normal"
if mode == "nopool":  # g_up in its own memory pool
    import types

    def capture(self, warmup=2):
        dev = self.labels.device
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for i in range(warmup):
                self.eager()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        g_fb, g_up = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_fb):
            self.static_loss = self.forward_backward().detach()
        self.graph_grads = [p.grad for p in self.params]
        with torch.cuda.graph(g_up):
            self.update()
        self.graphs = (g_fb, g_up)
    step.capture = types.MethodType(capture, step)
step.capture(warmup=2)
if mode == "fbonly":
    g_fb, g_up = step.graphs
    for g in step.graph_grads:
        g.zero_()  # whatever the capture-time memory held
    prev = None
    for r in range(3):
        g_fb.replay()
        torch.cuda.synchronize()
        print(f"fb-only replay {r}: loss {step.static_loss.item():.6f} grad norms",
              [f"{g.norm().item():.4e}" for g in step.graph_grads])
        views = {k: v.detach().float().clone() for k, v in flat.views(grads=True).items()}
        if prev is not None:
            for k, v in views.items():
                d = (v - prev[k]).abs().max().item()
                if d != 0 or not torch.isfinite(v).all():
                    print(f"   changed {k}: max diff {d:.3e} finite {bool(torch.isfinite(v).all())} "
                          f"norm {v.norm().item():.3e} prev {prev[k].norm().item():.3e}")
        prev = views
    g_up.replay()
    g_fb.replay()
    torch.cuda.synchronize()
    print("after up + fb:", [f"{g.norm().item():.4e}" for g in step.graph_grads])
    sys.exit(0)
print("graph grads", [(g.data_ptr(), g.numel()) for g in step.graph_grads])
print("master.grad", [(m.grad.data_ptr() if m.grad is not None else None) for m in masters])
for r in range(3):
    step()
    torch.cuda.synchronize()
    print(f"replay {r}: loss {step.static_loss.item():.6f} grad norms", [f"{g.norm().item():.4e}" for g in step.graph_grads])
for r in range(2):
    loss = step.eager()
    torch.cuda.synchronize()
    print(f"eager {r}: loss {loss.item():.6f} grad norms", [f"{m.grad.norm().item():.4e}" for m in masters])
