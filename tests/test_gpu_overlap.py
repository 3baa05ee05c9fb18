"""The overlapped gradient all-reduce inside a captured training step (TrainStep(overlap_all_reduce=
True) + FlatParamGroups) on one GPU: an RCCL process group of world size 1 with the collectives forced
on, so the per-group all-reduces started from the gradient hooks are captured into the hipGraph on
a side stream. Same parameters after three replays as the serial path (all-reduce between graphs)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs an MI355X", allow_module_level=True)

from lss_carla_amd.flat_params import FlatParamGroups  # noqa: E402
from lss_carla_amd.train_step import TrainStep  # noqa: E402

DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def pg():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=DEV)
    dist.all_reduce(torch.ones(1, device=DEV))  # communicator up before any capture
    yield
    dist.destroy_process_group()


def _step(overlap):
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.ReLU(), torch.nn.Linear(256, 256),
                              torch.nn.ReLU(), torch.nn.Linear(256, 1)).to(DEV)
    flat = FlatParamGroups(net, [["4"], ["2"]], cast_dtype=None)
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.randn(512, 64, generator=g).to(DEV)
    y = torch.randn(512, 1, generator=g).to(DEV)
    opt = torch.optim.Adam(flat.masters, lr=1e-3, fused=True, capturable=True)
    step = TrainStep(flat.bind(net), (x,), y, torch.nn.functional.mse_loss, opt, flat.masters, all_reduce=True,
                     amp_dtype=None, max_grad_norm=5.0, overlap_all_reduce=overlap, force_collectives=True)
    return step, flat


@pytest.mark.timeout(120)
def test_overlapped_all_reduce_captured(pg):
    res = []
    for overlap in (False, True):
        step, flat = _step(overlap)
        assert step.collectives and step.overlap == overlap
        step.capture(warmup=2)
        for _ in range(3):
            loss = step()
        torch.cuda.synchronize()
        assert torch.isfinite(loss)
        res.append({n: v.clone() for n, v in flat.views().items()})
    for n in res[0]:
        torch.testing.assert_close(res[1][n], res[0][n], rtol=1e-6, atol=1e-7, msg=n)
