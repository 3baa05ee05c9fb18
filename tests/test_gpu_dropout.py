"""CamEncode.dropout on lss_dropout (models.LssDropout): mask distribution, scaling, backward with the
forward's mask (regenerated from the seed), determinism under torch's CUDA seed, memory formats.

The reference's nn.Dropout(0.2) (src/models.py:44, 53) draws its mask from torch's Philox stream; this
one from Philox4x32-10 keyed by a seed drawn from the same generator -- the same distribution, not the
same draws, so the checks are the dropout contract (kept elements scaled by 1 / keep, the rest zero,
keep rate within binomial noise, the backward applying the same mask), not a fixture."""
import pytest
import torch

import lss_carla_amd  # noqa: F401
from lss_carla_amd import models

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _x(fmt, dtype, shape=(48, 512, 8, 22), seed=0):
    g = torch.Generator().manual_seed(seed)
    x = (torch.rand(shape, generator=g) + 0.5).to(DEV, dtype)  # nonzero everywhere: zeros are the mask
    return x.contiguous(memory_format=fmt)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("fmt", [torch.channels_last, torch.contiguous_format])
def test_dropout_forward_backward(dtype, fmt):
    m = models.LssDropout(0.2).train()
    x = _x(fmt, dtype).requires_grad_(True)
    torch.cuda.manual_seed(11)
    y = m(x)
    assert y.dtype == dtype and y.is_contiguous(memory_format=fmt)
    kept = y != 0
    rate = kept.float().mean().item()
    assert abs(rate - 0.8) < 0.002, rate  # n = 8.65 M: binomial sd 1.4e-4
    want = (x.detach().float() * 1.25).to(dtype)  # 1 / keep = 1.25 exactly, one rounding
    assert torch.equal(y[kept], want[kept])
    # backward: the same mask, dy in another memory format than x
    gy = torch.randn(x.shape, generator=torch.Generator().manual_seed(3)).to(DEV, dtype)
    gy = gy.contiguous(memory_format=torch.contiguous_format if fmt == torch.channels_last else torch.channels_last)
    y.backward(gy)
    gwant = torch.where(kept, (gy.float() * 1.25).to(dtype), torch.zeros((), device=DEV, dtype=dtype))
    assert torch.equal(x.grad, gwant)


def test_dropout_seeded_and_varies_per_call():
    m = models.LssDropout(0.2).train()
    x = _x(torch.channels_last, torch.bfloat16)
    torch.cuda.manual_seed(5)
    a = m(x)
    b = m(x)
    torch.cuda.manual_seed(5)
    c = m(x)
    assert torch.equal(a, c)
    assert not torch.equal(a != 0, b != 0)
    # masks of different calls independent: overlap of kept sets ~ 0.8^2
    both = ((a != 0) & (b != 0)).float().mean().item()
    assert abs(both - 0.64) < 0.003, both


def test_dropout_eval_and_fallbacks_match_torch_semantics():
    m = models.LssDropout(0.2)
    x = _x(torch.channels_last, torch.bfloat16)
    m.eval()
    assert m(x) is x or torch.equal(m(x), x)
    m.train()
    xc = x.cpu()
    y = m(xc)  # CPU tensor: torch's own dropout
    assert y.device.type == "cpu" and abs((y != 0).float().mean().item() - 0.8) < 0.01
    m0 = models.LssDropout(0.0).train()
    assert torch.equal(m0(x), x)


def test_dropout_prefetch_argument_is_harmless():
    m = models.LssDropout(0.2).train()
    x = _x(torch.channels_last, torch.bfloat16)
    pf = torch.randn(512 * 256 // 2, device=DEV).to(torch.bfloat16)  # the packed depthnet weights' size
    torch.cuda.manual_seed(2)
    a = m(x)
    m.prefetch = pf
    torch.cuda.manual_seed(2)
    b = m(x)
    m.prefetch = None
    assert torch.equal(a, b)
