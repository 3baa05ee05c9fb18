"""Inputs the kernels' fast paths must not trip over (round-3 advisor findings): tensors at storage
offsets that are not 16-B aligned reach the 16-B vector kernels only after a copy, and a device rig
updated in place after its host copy was attached is inverted from its new values."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU CI, skipped there
    pytest.skip("needs an MI355X", allow_module_level=True)

from oracle import lss_ref as ref  # noqa: E402
from lss_carla_amd import ops, synthetic as syn  # noqa: E402
from lss_carla_amd.efficientnet import _HipScaleAdd  # noqa: E402

DEV = torch.device("cuda:0")


def _unaligned_like(t: torch.Tensor, memory_format=torch.contiguous_format) -> torch.Tensor:
    """A copy of t living at storage offset 1 (2 B for bf16: never 16-B aligned), same strides."""
    dense = t.contiguous(memory_format=memory_format)
    buf = torch.empty(dense.numel() + 1, dtype=t.dtype, device=t.device)
    v = buf[1:].as_strided(dense.shape, dense.stride())
    v.copy_(dense)
    assert v.data_ptr() % 16 != 0 and torch.equal(v, t)
    return v


def test_scale_add_backward_with_unaligned_gradient():
    """lss_scale_add's backward (the MBConv skip with drop-connect) given a gradient at an unaligned
    offset: the same gradients, bit for bit, as from the aligned copy."""
    g = torch.Generator(device=DEV).manual_seed(0)
    x0 = torch.randn(4, 16, 8, 8, device=DEV, generator=g).to(torch.bfloat16)
    r0 = torch.randn(4, 16, 8, 8, device=DEV, generator=g).to(torch.bfloat16)
    u = torch.tensor([0.1, 0.9, 0.5, 0.95], device=DEV, dtype=torch.bfloat16)
    dy = torch.randn(x0.shape, device=DEV, generator=g).to(torch.bfloat16)
    grads = []
    for d in (dy, _unaligned_like(dy)):
        x, res = x0.clone().requires_grad_(True), r0.clone().requires_grad_(True)
        _HipScaleAdd.apply(x, res, u, 0.8).backward(d)
        grads.append((x.grad, res.grad))
    assert torch.equal(grads[0][0], grads[1][0]) and torch.equal(grads[0][1], grads[1][1])
    assert torch.equal(grads[0][1], dy) and grads[0][0][0].abs().sum() == 0  # sample 0 dropped (0.8 + 0.1 < 1)


def test_depthnet_lift_nhwc_with_unaligned_features():
    cfg, gc, _ = syn.config_confs("c1")
    B, N, fd = cfg["B"], cfg["N"], cfg["final_dim"]
    rig = {k: v.to(DEV) for k, v in syn.make_rig(B, N, fd, seed=1).items()}
    frustum = ref.create_frustum(fd, gc["dbound"]).to(DEV)
    D, H, W = frustum.shape[:3]
    plan = ops.plan_from_cameras(frustum, **rig, grid=ops.GridSpec.from_conf(gc))
    g = torch.Generator().manual_seed(3)
    feat = torch.randn(B * N, 512, H, W, generator=g).to(DEV, torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(D + 64, 512, 1, 1, generator=g) * 0.05).to(DEV, torch.bfloat16)
    b = (torch.randn(D + 64, generator=g) * 0.1).to(DEV, torch.bfloat16)
    want = ops.depthnet_lift_splat(feat, w, b, plan, torch.bfloat16, 1)
    got = ops.depthnet_lift_splat(_unaligned_like(feat, torch.channels_last), w, b, plan, torch.bfloat16, 1)
    torch.cuda.synchronize()
    assert torch.equal(got, want)


def test_host_inverse_copy_is_not_used_after_an_in_place_update():
    cfg, _, _ = syn.config_confs("c1")
    rig_a = syn.make_rig(1, 6, cfg["final_dim"], seed=0)
    rig_b = syn.make_rig(1, 6, cfg["final_dim"], seed=4, aug=True)
    assert not torch.equal(rig_a["post_rots"], rig_b["post_rots"])
    pr, it = rig_a["post_rots"].to(DEV), rig_a["intrins"].to(DEV)
    pr._lss_host, pr._lss_host_version = rig_a["post_rots"], pr._version  # as simbev.finish_batch attaches it
    it._lss_host, it._lss_host_version = rig_a["intrins"], it._version
    pinv, _ = ops.camera_inverses(pr, it)
    assert torch.equal(pinv.cpu(), torch.inverse(rig_a["post_rots"]).reshape(-1, 9))
    pr.copy_(rig_b["post_rots"].to(DEV))  # a reused batch buffer: the attached host copy is stale now
    pinv, _ = ops.camera_inverses(pr, it)
    assert torch.equal(pinv.cpu(), torch.inverse(rig_b["post_rots"]).reshape(-1, 9))
