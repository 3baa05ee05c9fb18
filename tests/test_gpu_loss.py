"""SimpleLoss on lss_bce_logits (include/lss_convs.h) vs the reference's BCEWithLogitsLoss(pos_weight)
(src/tools.py:222-230): loss and input gradient, fp32 and bf16 logits, ragged sizes, determinism."""
import pytest
import torch

from lss_carla_amd import tools as T

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(8, 1, 200, 200), (2, 1, 13, 7), (1, 1, 1, 5), (3, 2, 40, 41)])
def test_fused_bce_vs_reference(shape, dtype):
    g = torch.Generator().manual_seed(sum(shape))
    x = (torch.randn(shape, generator=g) * 4).to(dtype)
    x.view(-1)[:3] = torch.tensor([60.0, -60.0, 0.0]).to(dtype)  # saturated logits and zero
    t = (torch.rand(shape, generator=g) < 0.3).float()
    loss_fn = T.SimpleLoss(2.13).to(DEV)
    xd = x.to(DEV).requires_grad_(True)
    loss = loss_fn(xd, t.to(DEV))
    assert loss.dtype == torch.float32 and loss.shape == ()
    loss.backward(torch.tensor(0.75, device=DEV))
    # reference: torch's BCEWithLogitsLoss on the fp64 cast of the same values
    xr = x.double().requires_grad_(True)
    ref = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([2.13], dtype=torch.float64))(xr, t.double())
    (ref * 0.75).backward()
    torch.testing.assert_close(loss.detach().cpu().double(), ref.detach(), rtol=2e-6, atol=1e-7)
    assert xd.grad.dtype == dtype
    if dtype == torch.float32:
        torch.testing.assert_close(xd.grad.cpu().double(), xr.grad, rtol=1e-5, atol=1e-12)
    else:  # the fp32 gradient rounded once to bf16
        torch.testing.assert_close(xd.grad.cpu().double(), xr.grad, rtol=8e-3, atol=1e-12)


def test_fused_bce_deterministic_and_matches_torch_gpu():
    g = torch.Generator().manual_seed(3)
    x = torch.randn(8, 1, 200, 200, generator=g).to(DEV)
    t = (torch.rand(8, 1, 200, 200, generator=g) < 0.1).float().to(DEV)
    loss_fn = T.SimpleLoss(2.13).to(DEV)
    a, b = loss_fn(x, t), loss_fn(x, t)
    assert torch.equal(a, b)
    torch.testing.assert_close(a, loss_fn.loss_fn(x, t), rtol=1e-6, atol=0)


def test_non_contiguous_logits_take_torch_path():
    x = torch.randn(4, 1, 10, 12, device=DEV).transpose(2, 3)
    t = (torch.rand(4, 1, 12, 10, device=DEV) < 0.5).float()
    loss_fn = T.SimpleLoss(2.13).to(DEV)
    torch.testing.assert_close(loss_fn(x, t), loss_fn.loss_fn(x, t))
