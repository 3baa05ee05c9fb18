"""flat_params._gather (the flat-gradient copy in _Materialize's backward): gradients whose layout differs
from their flat view -- a channels-last 3x3 weight gradient into a contiguous view, a 1x1 gradient whose
strides differ only on size-1 dimensions, another dtype -- land bit-exact, copied apart from the
same-layout pairs, which keep the one multi-tensor copy. CPU."""
import torch

from lss_carla_amd import flat_params as fpm


def _case():
    torch.manual_seed(0)
    like = [torch.empty(8, 4, 3, 3), torch.empty(16, 8, 1, 1).contiguous(memory_format=torch.channels_last),
            torch.empty(5, 7), torch.empty(6, 3, 3, 3)]
    grads = [torch.randn(8, 4, 3, 3).contiguous(memory_format=torch.channels_last),  # odd layout
             torch.randn(16, 8, 1, 1),                                              # size-1 strides only
             torch.randn(5, 7, dtype=torch.float64),                                # odd dtype
             torch.randn(6, 3, 3, 3)]                                               # same layout
    return like, grads


def test_gather_odd_layouts_exact():
    like, grads = _case()
    n = sum(p.numel() for p in like)
    buf = torch.full((n,), float("nan"))
    fpm._gather(fpm._views(buf, like), grads, buf)
    for v, g in zip(fpm._views(buf, like), grads):
        assert torch.equal(v, g.to(v.dtype))


def test_gather_unused_parameter_zero_and_split_matches_single_copy():
    like, grads = _case()
    grads[2] = None
    n = sum(p.numel() for p in like)
    outs = []
    for split in (True, False):
        fpm.GATHER_SPLIT = split
        try:
            buf = torch.full((n,), float("nan"))
            fpm._gather(fpm._views(buf, like), grads, buf)
        finally:
            fpm.GATHER_SPLIT = True
        outs.append(buf)
    assert torch.equal(outs[0], outs[1])
    assert not torch.isnan(outs[0]).any()
    assert torch.equal(fpm._views(outs[0], like)[2], torch.zeros(5, 7))


def test_restride_only_size1_dims():
    d = torch.empty(16, 8, 1, 1).as_strided((16, 8, 1, 1), (8, 1, 8, 8))
    g = torch.randn(16, 8, 1, 1)
    r = fpm._restride(g, d)
    assert r.stride() == d.stride() and torch.equal(r, g)
    d3 = torch.empty(8, 4, 3, 3).contiguous(memory_format=torch.channels_last)
    g3 = torch.randn(8, 4, 3, 3)
    assert fpm._restride(g3, d3) is g3
