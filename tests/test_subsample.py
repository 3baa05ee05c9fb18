"""models._Subsample (the stride-s pixel pick in front of BevEncode's stride-2 1x1 downsample convs):
the same values and input gradient as x[:, :, ::s, ::s] under autograd, channels-last output, the
gradient in the input's layout. CPU."""
import pytest
import torch

from lss_carla_amd.models import _Subsample


@pytest.mark.parametrize("cl", [True, False], ids=["channels_last", "contiguous"])
@pytest.mark.parametrize("shape,s", [((2, 4, 9, 10), 2), ((1, 8, 100, 100), 2), ((3, 2, 7, 7), 3)])
def test_subsample_matches_slicing(shape, s, cl):
    torch.manual_seed(0)
    x = torch.randn(shape)
    if cl:
        x = x.contiguous(memory_format=torch.channels_last)
    a = x.clone().requires_grad_(True)
    b = x.clone().requires_grad_(True)
    ya, yb = _Subsample.apply(a, s), b[:, :, ::s, ::s]
    g = torch.randn_like(yb)
    ya.backward(g)
    yb.backward(g)
    assert torch.equal(ya, yb) and ya.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(a.grad, b.grad)
    assert a.grad.is_contiguous(memory_format=torch.channels_last if cl else torch.contiguous_format)
