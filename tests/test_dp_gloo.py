"""World-size-2 data parallelism on CPU (gloo): DDP-averaged gradients of the LSS model equal the
average of per-replica single-process gradients (BatchNorm is per replica, as in the reference).

The HIP hot path has no CPU implementation, so on CPU the hot path runs through the oracle
(test infrastructure) while the conv stacks, the DP wrapper and the all-reduce are the product's.
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import lss_carla_amd as L
from lss_carla_amd import parallel
from lss_carla_amd.flat_params import FlatParams, FlatParamGroups, lss_backward_groups
from lss_carla_amd.train_step import TrainStep
from lss_carla_amd import synthetic as syn

FD = (64, 192)
GC = syn.grid_conf(xy=(-16.0, 16.0, 0.5))  # 64x64 BEV (BevEncode needs X, Y multiples of 8)


class _CpuLSS(torch.nn.Module):
    """Wraps the product model; forward goes through the oracle hot path (CPU only)."""

    def __init__(self, model):
        super().__init__()
        self.model = model

    def forward(self, x, rots, trans, intrins, post_rots, post_trans):
        from oracle import lss_ref as ref
        m = self.model
        dx, bx, nx = ref.gen_dx_bx(GC["xbound"], GC["ybound"], GC["zbound"])
        return ref.full_forward(m.camencode.depthnet_out, m.bevencode, m.frustum.detach(), x, rots, trans, intrins,
                                post_rots, post_trans, dx, bx, nx, m.D)


def _model():
    torch.manual_seed(0)
    m = L.compile_model(GC, syn.data_aug_conf(FD, 2), outC=1)
    for mod in m.modules():
        if isinstance(mod, (torch.nn.Dropout, torch.nn.Dropout2d)):
            mod.p = 0.0
    m.camencode.trunk._global_params.drop_connect_rate = 0.0
    m.train()
    return m


def _batch(seed):
    rig = syn.make_rig(1, 2, FD, seed=seed)
    imgs = syn.make_images(1, 2, FD, seed=seed)
    labels = syn.make_labels(1, 64, 64, seed=seed)
    return imgs, rig, labels


def _grads(module, seed):
    imgs, rig, labels = _batch(seed)
    out = module(imgs, rig["rots"], rig["trans"], rig["intrins"], rig["post_rots"], rig["post_trans"])
    L.SimpleLoss(2.13)(out, labels).backward()


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    w, r, _, dev = parallel.init_from_env("gloo")
    assert (w, r) == (world, rank)
    m = _model()
    ddp = parallel.make_data_parallel(_CpuLSS(m), dev)
    assert isinstance(ddp, torch.nn.parallel.DistributedDataParallel)
    _grads(ddp, seed=10 + rank)
    if rank == 0:
        torch.save({n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None},
                   os.path.join(outdir, "ddp.pt"))
    # the captured-step path: broadcast replicas, flat master parameters, one all-reduce
    m2 = _model()
    if rank == 1:
        with torch.no_grad():
            for p in m2.parameters():
                if p.is_floating_point():
                    p.add_(1.0)
    parallel.broadcast_state(m2)
    parallel.freeze_unused(m2)
    wrapped = _CpuLSS(m2)
    flat = FlatParams(wrapped, cast_dtype=None)
    _grads(flat.bind(wrapped), seed=10 + rank)
    dist.all_reduce(flat.master.grad)
    flat.master.grad.mul_(1.0 / world)
    if rank == 0:
        g = {n.removeprefix("model."): v.clone().contiguous() for n, v in flat.views_of(flat.master.grad).items()}
        torch.save(g, os.path.join(outdir, "flat.pt"))
    t = parallel.max_over_ranks(float(rank), dev)
    assert t == world - 1
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(600)
def test_ddp_gradients_equal_mean_of_replicas():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        ddp = torch.load(os.path.join(d, "ddp.pt"), weights_only=True)
        flat = torch.load(os.path.join(d, "flat.pt"), weights_only=True)
    ref = {}
    nthreads = torch.get_num_threads()
    torch.set_num_threads(2)  # the workers' thread count: same conv algorithms and reduction order
    for rank in range(world):
        m = _model()
        parallel.freeze_unused(m)
        _grads(_CpuLSS(m), seed=10 + rank)
        for n, p in m.named_parameters():
            if p.grad is not None:
                ref[n] = ref.get(n, 0) + p.grad / world
    torch.set_num_threads(nthreads)
    assert set(ddp) == set(ref)
    for n in ref:
        scale = ref[n].abs().max().clamp_min(1e-12)
        err = (ddp[n] - ref[n]).abs().max() / scale
        assert err < 1e-3, (n, float(err), float(scale))
    assert not any(n.startswith(parallel.UNUSED_PREFIXES) for n in ddp)
    # FlatParams + one all-reduce (bench.py --graph): same averaged gradients, frozen head excluded
    assert set(flat) == set(ref)
    for n in ref:
        scale = ref[n].abs().max().clamp_min(1e-12)
        err = (flat[n] - ref[n]).abs().max() / scale
        assert err < 1e-3, (n, float(err), float(scale))


def test_freeze_unused_through_wrapper():
    w = _CpuLSS(_model())
    assert parallel.freeze_unused(w) == parallel.freeze_unused(_model()) > 0


def test_freeze_unused_counts_head_params():
    m = _model()
    frozen = parallel.freeze_unused(m)
    assert frozen == 320 * 1280 + 2 * 1280 + 1280 * 1000 + 1000
    assert all(not p.requires_grad for n, p in m.named_parameters() if n.startswith(parallel.UNUSED_PREFIXES))


def test_flat_params_match_autocast_gradients():
    """FlatParams under CPU bf16 autocast: same forward and parameter gradients as the module run
    with its own Parameters (autocast casting each weight), channels-last weights included."""
    torch.manual_seed(3)
    net = torch.nn.Sequential(torch.nn.Conv2d(8, 16, 3, padding=1), torch.nn.BatchNorm2d(16), torch.nn.ReLU(),
                              torch.nn.Conv2d(16, 16, 3, padding=1, groups=16, bias=False),
                              torch.nn.Conv2d(16, 4, 1)).to(memory_format=torch.channels_last)
    x = torch.randn(2, 8, 10, 12).contiguous(memory_format=torch.channels_last)
    with torch.autocast("cpu", dtype=torch.bfloat16):
        y0 = net(x)
    y0.float().square().mean().backward()
    want = {n: p.grad.clone() for n, p in net.named_parameters()}
    flat = FlatParams(net, cast_dtype=torch.bfloat16)
    assert set(flat.names16) == {"0.weight", "0.bias", "4.weight", "4.bias"}  # depthwise + BN stay fp32
    assert flat.numel == sum(p.numel() for p in net.parameters())
    for p in net.parameters():  # the module's Parameters alias the master buffer
        base, end = flat.master.data_ptr(), flat.master.data_ptr() + 4 * flat.numel
        assert base <= p.data_ptr() < end
    with torch.autocast("cpu", dtype=torch.bfloat16):
        y1 = flat.bind(net)(x)
    assert torch.equal(y0, y1)
    y1.float().square().mean().backward()
    got = flat.views_of(flat.master.grad)
    for n in want:
        torch.testing.assert_close(got[n], want[n], rtol=0, atol=0)
    # an optimizer step on master is seen by the module
    with torch.no_grad():
        flat.master.add_(1.0)
    assert torch.equal(net[0].bias.detach(), flat.views_of(flat.master.detach())["0.bias"])


def _train_step(model, seed, world_reduce, overlap=False):
    """One TrainStep (flat fp32 master, SimpleLoss, backward, all-reduce, clip 5.0, Adam) on `model`;
    overlap: one master per backward group, each all-reduced from its gradient hook."""
    parallel.freeze_unused(model)
    wrapped = _CpuLSS(model)
    if overlap:
        flat = FlatParamGroups(wrapped, lss_backward_groups("model."), cast_dtype=None)
        params = flat.masters
    else:
        flat = FlatParams(wrapped, cast_dtype=None)
        params = [flat.master]
    imgs, rig, labels = _batch(seed)
    opt = torch.optim.Adam(params, lr=1e-3, weight_decay=1e-7)
    inputs = (imgs, rig["rots"], rig["trans"], rig["intrins"], rig["post_rots"], rig["post_trans"])
    step = TrainStep(flat.bind(wrapped), inputs, labels, L.SimpleLoss(2.13), opt, params,
                     all_reduce=world_reduce, amp_dtype=None, max_grad_norm=5.0, overlap_all_reduce=overlap)
    return step, flat


def _worker_trainstep(rank, world, port, outdir, overlap=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    parallel.init_from_env("gloo")
    m = _model()
    parallel.broadcast_state(m)
    step, flat = _train_step(m, seed=20 + rank, world_reduce=True, overlap=overlap)
    assert step.world == world and step.overlap == overlap
    if overlap:  # the summed gradients the hooks produced, then the update
        loss = step.forward_backward()
        grads = {n.removeprefix("model."): v.clone().contiguous() for n, v in flat.views(grads=True).items()}
        step.update()
    else:
        loss = step.eager()
    assert torch.isfinite(loss)
    assert parallel.replicas_in_sync(step.params)  # bench.py's check after the untimed replays
    if rank == 0:
        if overlap:
            torch.save({"grads": grads, "params": {n.removeprefix("model."): v.clone().contiguous()
                                                   for n, v in flat.views().items()}},
                       os.path.join(outdir, "ts_overlap.pt"))
        else:
            torch.save({"master": flat.master.detach().clone()}, os.path.join(outdir, "ts.pt"))
    dist.destroy_process_group()


def _worker_trainstep_overlap(rank, world, port, outdir):
    _worker_trainstep(rank, world, port, outdir, overlap=True)


@pytest.mark.timeout(600)
def test_train_step_world2_equals_single_process_average():
    """TrainStep's world > 1 path (the captured bench step's eager twin): all-reduce sum, / world,
    clip_grad_norm_(5), Adam -- equals one process applying the mean of the two ranks' gradients."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker_trainstep, args=(world, _free_port(), d), nprocs=world, join=True)
        got = torch.load(os.path.join(d, "ts.pt"), weights_only=True)["master"]
    nthreads = torch.get_num_threads()
    torch.set_num_threads(2)
    grads = []
    for rank in range(world):
        step, flat = _train_step(_model(), seed=20 + rank, world_reduce=False)
        step.forward_backward()
        grads.append(flat.master.grad.clone())
    step, flat = _train_step(_model(), seed=20, world_reduce=False)
    flat.master.grad = (grads[0] + grads[1]) * (1.0 / world)
    step.update()
    torch.set_num_threads(nthreads)
    want = flat.master.detach()
    assert got.shape == want.shape
    torch.testing.assert_close(got, want, rtol=1e-6, atol=1e-7)


@pytest.mark.timeout(600)
def test_train_step_world2_overlapped_all_reduce():
    """overlap_all_reduce: three parameter groups, each all-reduced from its gradient hook while the
    backward continues -- the summed gradients are bit-identical to one all-reduce of the flat
    gradient; the parameters after clip + Adam agree to the last bits (the clip norm is summed over
    three tensors instead of one)."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker_trainstep_overlap, args=(world, _free_port(), d), nprocs=world, join=True)
        got = torch.load(os.path.join(d, "ts_overlap.pt"), weights_only=True)
        mp.spawn(_worker_trainstep, args=(world, _free_port(), d), nprocs=world, join=True)
        ref_master = torch.load(os.path.join(d, "ts.pt"), weights_only=True)["master"]
    nthreads = torch.get_num_threads()
    torch.set_num_threads(2)
    gsum = None
    for rank in range(world):  # the reference sum of the two ranks' flat gradients
        step, flat = _train_step(_model(), seed=20 + rank, world_reduce=False)
        step.forward_backward()
        gsum = flat.master.grad.clone() if gsum is None else gsum + flat.master.grad
    torch.set_num_threads(nthreads)
    want_g = {n.removeprefix("model."): v for n, v in flat.views_of(gsum).items()}
    want_p = {n.removeprefix("model."): v for n, v in flat.views_of(ref_master).items()}
    assert set(got["grads"]) == set(want_g) == set(want_p)
    for n in want_g:
        assert torch.equal(got["grads"][n], want_g[n]), n
        torch.testing.assert_close(got["params"][n], want_p[n], rtol=0, atol=1e-5, msg=n)


class _FakeStep:
    """Stands in for train_step.TrainStep in the capture decision: capture() records its call."""

    def __init__(self, name):
        self.name, self.captured_with = name, None

    def capture(self, warmup=2, on_warmup=None):
        self.captured_with = warmup


def _worker_capture_decision(rank, world, port, outdir, fail_rank):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    parallel.init_from_env("gloo")
    assert parallel.control_group() is not None
    step, reason = parallel.capture_collectively(_FakeStep("overlapped"), 3, fallback=lambda: _FakeStep("serial"),
                                                 fail=(rank == fail_rank))
    # replicas: identical tensors agree; a one-ulp change on rank 1 is seen by every rank
    t = [torch.linspace(-1, 1, 1000), torch.arange(7, dtype=torch.float32)]
    same = parallel.replicas_in_sync(t)
    if rank == 1:
        t[0][500] = torch.nextafter(t[0][500], torch.tensor(2.0))
    diff = parallel.replicas_in_sync(t)
    torch.save({"step": step.name, "warmup": step.captured_with, "reason": reason, "same": same, "diff": diff},
               os.path.join(outdir, f"cap{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("fail_rank", [-1, 0, 1])
def test_capture_fallback_is_a_collective_decision(fail_rank):
    """bench.py's N > 1 capture path (parallel.capture_collectively): when one rank's capture raises,
    EVERY rank takes the serial all-reduce step (captured with 2 warm-up steps); when none does, every
    rank keeps its captured step. parallel.replicas_in_sync: True on identical replicas, False on every
    rank when one element of one rank differs by one ulp."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker_capture_decision, args=(world, _free_port(), d, fail_rank), nprocs=world, join=True)
        got = [torch.load(os.path.join(d, f"cap{r}.pt"), weights_only=True) for r in range(world)]
    for r, g in enumerate(got):
        if fail_rank < 0:
            assert (g["step"], g["warmup"], g["reason"]) == ("overlapped", 3, None)
        else:
            assert (g["step"], g["warmup"]) == ("serial", 2)
            assert ("this rank" if r == fail_rank else "another rank") in g["reason"]
        assert g["same"] is True and g["diff"] is False


def test_replica_checksums_single_process():
    """World size 1: always in sync; the checksum tells bit patterns apart (-0.0 vs 0.0, bf16 views)."""
    a = torch.zeros(10)
    b = a.clone()
    b[3] = -0.0
    assert not torch.equal(parallel.replica_checksums([a]), parallel.replica_checksums([b]))
    assert torch.equal(parallel.replica_checksums([a.bfloat16()]), parallel.replica_checksums([a.bfloat16()]))
    assert parallel.replicas_in_sync([a]) is True
