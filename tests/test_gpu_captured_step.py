"""Parity of the exact benched step: the config-3 training step captured as HIP graphs the way bench.py
builds it (train_step.TrainStep over FlatParamGroups masters, fused depthnet + lift on MFMA,
channels-last bf16 BEV, host torch.inverse staged by ops.HostInverses.update as pre_step, the plan's
persistent workspace pointers baked into the graph), replayed over two different rigs.

Each replay is compared with an eager step from the same parameters and inputs (the BEV bit for bit,
the loss, camencode.depthnet.weight's clipped gradient), and the replayed BEV with the fp64 oracle on
the same bf16 operands (reference: train_simbev.py:231-248 -> src/models.py:248-259). Run twice: with
dropout and drop-connect off, and with both at their defaults (the benched step: torch.rand's draw
feeding lss_scale_add's in-kernel mask) -- then the CUDA generator is seeded identically before the
replay and before the eager step (graph-safe Philox: the same draws), and two replays without a
reseed must draw different masks."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs an MI355X", allow_module_level=True)

from oracle import lss_ref as ref  # noqa: E402
import lss_carla_amd as L  # noqa: E402
from lss_carla_amd import ops, parallel, synthetic as syn  # noqa: E402
from lss_carla_amd.flat_params import FlatParamGroups, lss_backward_groups  # noqa: E402
from lss_carla_amd.train_step import TrainStep  # noqa: E402

DEV = torch.device("cuda:0")
BF16_U = 2.0 ** -8


def _oracle_bev(feat, weight, bias, rig, frustum, gc, B, N):
    """Autocast's bf16 conv output of the same bf16 operands, then the reference's lift + splat (fp64)."""
    D = frustum.shape[0]
    logits = torch.einsum("nkhw,ok->nohw", feat.double(), weight.double().flatten(1)) + bias.double().view(1, -1, 1, 1)
    dn = logits.to(torch.bfloat16).float()
    geom = ref.get_geometry(frustum, **rig)
    dx, bx, nx = ref.gen_dx_bx(gc["xbound"], gc["ybound"], gc["zbound"])
    _, new_x = ref.lift(dn, D, 64)
    return ref.voxel_pooling_fp64(geom, ref.cam_feats_layout(new_x, B, N).numpy(), dx, bx, nx)


@pytest.fixture
def miopen_find():
    """MIOpen's find (as bench.py runs it), restored afterwards: left on, every later test's new conv
    shape would run the exhaustive search."""
    old = torch.backends.cudnn.benchmark
    torch.backends.cudnn.benchmark = True
    yield
    torch.backends.cudnn.benchmark = old


@pytest.mark.parametrize("stochastic", [False, True], ids=["deterministic", "dropout_dropconnect"])
def test_captured_c3_step_matches_eager_and_oracle_over_two_rigs(miopen_find, stochastic):
    cfg, gc, dac = syn.config_confs("c3")
    B, N, fd = cfg["B"], cfg["N"], cfg["final_dim"]
    torch.manual_seed(7)
    model = L.compile_model(gc, dac, outC=1).to(DEV)
    model.bev_layout, model.fuse_depthnet = "nhwc", True
    model.bevencode.to(memory_format=torch.channels_last)
    if not stochastic:
        model.camencode.dropout.p = 0.0
        model.bevencode.dropout.p = 0.0
        model.camencode.trunk._global_params.drop_connect_rate = 0.0
    else:
        assert model.camencode.trunk._global_params.drop_connect_rate == 0.2
    model.train()
    parallel.freeze_unused(model)
    flat = FlatParamGroups(model, lss_backward_groups(), cast_dtype=torch.bfloat16)
    masters = flat.masters

    rigs = [syn.make_rig(B, N, fd, seed=0), syn.make_rig(B, N, fd, seed=5, aug=True)]
    assert not torch.equal(rigs[0]["post_rots"], rigs[1]["post_rots"])
    static = {k: v.to(DEV) for k, v in rigs[0].items()}  # the graph's static rig inputs
    host = {k: rigs[0][k].clone().pin_memory() for k in ("post_rots", "intrins")}
    hinv = ops.HostInverses(B * N, DEV)
    model.static_inverses = (hinv.pinv, hinv.kinv)
    X, Y, _ = ops.GridSpec.from_conf(gc).nx
    imgs = syn.make_images(B, N, fd, seed=3).to(DEV)
    labels = syn.make_labels(B, X, Y, seed=3).to(DEV)
    inputs = (imgs, static["rots"], static["trans"], static["intrins"], static["post_rots"], static["post_trans"])
    seen = {}
    # (detached: a stored tensor with autograd history would keep the captured graph's nodes alive)
    model.bevencode.register_forward_pre_hook(lambda m, a: seen.__setitem__("bev", a[0].detach()))
    model.camencode.dropout.register_forward_hook(lambda m, a, out: seen.__setitem__("feat", out.detach()))
    opt = torch.optim.Adam(masters, lr=1e-3, weight_decay=1e-7, fused=True, capturable=True)
    step = TrainStep(flat.bind(model), inputs, labels, L.SimpleLoss(2.13).to(DEV), opt, masters, all_reduce=True,
                     amp_dtype=torch.bfloat16, max_grad_norm=5.0,
                     pre_step=lambda: hinv.update(host["post_rots"], host["intrins"]))
    step.capture(warmup=2)
    g_bev = seen["bev"]  # written by every replay (graph pool)
    def graph_grad_views():
        out = {}
        for grp, gg in zip(flat.groups, step.graph_grads):
            out.update(grp.views_of(gg))
        return out
    g_dw = graph_grad_views()["camencode.depthnet.weight"]
    assert g_bev.dtype == torch.bfloat16 and g_bev.is_contiguous(memory_format=torch.channels_last)
    snap = [m.detach().clone() for m in masters]

    def restore():
        with torch.no_grad():
            for m, s in zip(masters, snap):
                m.copy_(s)

    def set_rig(r):
        for k in static:
            static[k].copy_(r[k])
        for k in host:
            host[k].copy_(r[k])

    frustum = model.frustum.detach().cpu()
    results = []
    for i, r in enumerate(rigs):
        set_rig(r)
        restore()
        torch.cuda.manual_seed(1000 + i)  # the same Philox stream for the replay and the eager step
        step()  # pre_step + graph replays
        torch.cuda.synchronize()
        rep = (g_bev.clone(), g_dw.clone(), step.static_loss.clone())
        # the replay's gradients live in the graph's own buffers (step.graph_grads): after an eager
        # step the masters' .grad point elsewhere
        rep_all = {k: v.detach().clone() for k, v in graph_grad_views().items()}
        restore()
        w = model.camencode.depthnet.weight.detach().to(torch.bfloat16).cpu()  # this step's bf16 operands
        b = model.camencode.depthnet.bias.detach().to(torch.bfloat16).cpu()
        torch.cuda.manual_seed(1000 + i)
        loss_e = step.eager()
        torch.cuda.synchronize()
        e_dw = flat.views(grads=True)["camencode.depthnet.weight"].clone()
        eag = (seen["bev"].clone(), e_dw, loss_e.detach().clone(), seen["feat"].detach())
        # replay == eager: the BEV bit for bit (same kernels, same operands), loss and gradient close
        # (MIOpen's backward-weight reductions are not bitwise reproducible run to run)
        d = (rep[0].float() - eag[0].float()).abs()
        print(f"rig {i}: bev |rep| {rep[0].float().norm().item():.4f} |eag| {eag[0].float().norm().item():.4f} "
              f"max diff {d.max().item():.3e} ndiff {(d > 0).sum().item()} loss {rep[2].item():.6f} "
              f"{eag[2].item():.6f} |g_rep| {rep[1].norm().item():.4e} |g_eag| {eag[1].norm().item():.4e}")
        assert torch.equal(rep[0], eag[0]), f"rig {i}: replayed BEV != eager BEV"
        torch.testing.assert_close(rep[2], eag[2], rtol=1e-5, atol=1e-6)
        rel = ((rep[1] - eag[1]).norm() / eag[1].norm()).item()
        assert rel < 1e-3, (i, rel, rep[1].norm().item(), eag[1].norm().item())
        # every parameter's gradient, not only the hot path's: a conv solver that is not replay-safe
        # shows up as a replayed gradient of zeros (or garbage) next to the eager one
        diffs = []
        for k, e in flat.views(grads=True).items():
            en = e.norm().item()
            if en < 1e-6:
                continue
            diffs.append((((rep_all[k] - e).norm() / en).item(), k, en, rep_all[k].norm().item(), e.numel()))
        diffs.sort(reverse=True)
        for d_ in diffs[:3]:
            print(f"rig {i}: grad rel diff {d_[0]:.3e} {d_[1]} |eag| {d_[2]:.3e} |rep| {d_[3]:.3e} n {d_[4]}")
        # a replay-safe step reproduces every gradient to MIOpen's run-to-run noise (~1e-4, also the
        # ill-conditioned BN biases); a solver that is not replay-safe is off by O(1)
        assert diffs[0][0] < 2e-2, diffs[0][:2]
        # replayed BEV vs the fp64 oracle on the eager step's bf16 operands
        exact = _oracle_bev(eag[3].to(torch.bfloat16).cpu(), w, b, r, frustum, gc, B, N)
        got = rep[0].float().cpu().numpy()
        err = np.abs(got - exact)
        bound = 2 * BF16_U * np.abs(exact) + 2e-3
        assert (err <= bound).all(), (i, float(err.max()), int((err > bound).sum()))
        assert not got.transpose(0, 2, 3, 1)[np.abs(exact).sum(1) == 0].any()  # empty cells exactly zero
        results.append(rep[0])
    # the two rigs really produced different BEVs through the same graph
    assert not torch.equal(results[0], results[1])
    if stochastic:  # two replays, same rig and parameters, no reseed: new dropout / drop-connect masks
        bevs = []
        for _ in range(2):
            restore()
            step()
            torch.cuda.synchronize()
            bevs.append(g_bev.clone())
        assert not torch.equal(bevs[0], bevs[1]), "the replays drew the same masks"
