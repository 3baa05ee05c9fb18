"""CPU-only checks: the C ABI library loads and exports every declared symbol, host logic, module surface."""
import os
import re

import numpy as np
import pytest
import torch

from conftest import REPO
from oracle import lss_ref as ref
import lss_carla_amd as L
from lss_carla_amd import _lib, ops
from lss_carla_amd import synthetic as syn

HEADERS = [os.path.join(REPO, "include", h) for h in ("lss_hip.h", "lss_convs.h", "lss_simbev.h")]


def _declared():
    text = "".join(open(h).read() for h in HEADERS)
    return set(re.findall(r"^\s*(?:int|int32_t|int64_t|size_t|const char\*)\s+(lss_\w+)\s*\(", text, re.M))


def test_header_declarations_match_binding():
    assert _declared() == set(_lib.SIGNATURES), _declared() ^ set(_lib.SIGNATURES)


def test_library_loads_and_exports_all_symbols():
    lib = _lib.load()  # built by __graft_entry__.build(); raises if missing
    for name in _declared():
        assert hasattr(lib, name), name
    assert lib.lss_abi_version() == _lib.ABI_VERSION
    assert lib.lss_error_string(0) == b"success"
    assert b"invalid" in lib.lss_error_string(-1)
    # host-side argument validation (no device work): NULL pointers are rejected
    assert lib.lss_geometry_cells(None, None, None, None, None, None, None, None, None, None, None, None, None) == -1
    assert lib.lss_ceiling_store(None, 16, 1, 0, None, None, None) == -1
    assert lib.lss_csr_scratch_bytes(4096, 100) == 256 + 8 * 100  # scan partials (aligned) + unsorted keys
    assert lib.lss_debug_checks() == (1 if os.environ.get("LSS_DEBUG", "0") == "1" else 0)


def test_debug_library_loads_and_exports_all_symbols():
    """liblss_hip_debug.so (LSS_DEBUG=1: device-side index checks) exposes the same ABI."""
    dbg = _lib.open_library(_lib.DEBUG_LIB_PATH)
    for name in _declared():
        assert hasattr(dbg, name), name
    assert dbg.lss_debug_checks() == 1
    assert dbg.lss_debug_status(None, 0) == -1  # NULL output rejected without touching a device


def test_gridspec_matches_reference_quantiser_constants():
    gs = ops.GridSpec.from_conf(syn.grid_conf())
    dx, bx, nx = ref.gen_dx_bx([-50.0, 50.0, 0.5], [-50.0, 50.0, 0.5], [-10.0, 10.0, 20.0])
    assert gs.nx == tuple(nx.tolist())
    assert np.array_equal(np.array(gs.lo, dtype=np.float32), (bx - dx / np.float32(2)).astype(np.float32))
    assert gs.ncells(8) == 8 * 200 * 200


def test_module_surface_and_state_dict():
    gc, dac = syn.grid_conf(), syn.data_aug_conf()
    m = L.compile_model(gc, dac, outC=1)
    assert isinstance(m, L.LiftSplatShoot)
    sd = m.state_dict()
    keys = list(sd)
    assert keys[:4] == ["dx", "bx", "nx", "frustum"]
    assert m.dx.requires_grad is False and m.nx.dtype == torch.long
    assert m.D == 41 and m.camC == 64 and m.downsample == 16 and m.use_quickcumsum is True
    np.testing.assert_array_equal(m.frustum.detach().numpy(), ref.create_frustum((128, 352), gc["dbound"]).numpy())
    for k in ("camencode.trunk._conv_stem.weight", "camencode.trunk._blocks.15._project_conv.weight",
              "camencode.trunk._blocks.1._expand_conv.weight", "camencode.trunk._blocks.0._se_reduce.bias",
              "camencode.trunk._fc.weight", "camencode.up1.conv.4.running_var", "camencode.depthnet.weight",
              "bevencode.conv1.weight", "bevencode.layer2.0.downsample.1.weight", "bevencode.up2.4.bias"):
        assert k in sd, k
    assert "camencode.trunk._blocks.0._expand_conv.weight" not in sd  # expand ratio 1 block
    assert len(m.camencode.trunk._blocks) == 16
    assert sum(p.numel() for p in m.parameters()) == 14313575
    assert m.camencode.depthnet.out_channels == 41 + 64
    # zero_init_residual of the torchvision trunk parts
    assert m.bevencode.layer1[0].bn2.weight.abs().sum() == 0
    assert m.bevencode.layer1[0].bn1.weight.sum() == 64
    # BevEncode parameter order = the reference's (conv1 first)
    names = [n for n, _ in m.bevencode.named_parameters()]
    assert names[0] == "conv1.weight" and names[1] == "bn1.weight"


def test_efficientnet_static_same_padding():
    m = L.compile_model(syn.grid_conf(), syn.data_aug_conf(), outC=1)
    t = m.camencode.trunk
    assert isinstance(t._conv_stem.static_padding, torch.nn.ZeroPad2d)
    assert t._conv_stem.static_padding.padding == (0, 1, 0, 1)
    assert t._blocks[3]._depthwise_conv.static_padding.padding == (1, 2, 1, 2)
    assert t._blocks[4]._depthwise_conv.padding == (2, 2)
    # endpoints on a 128x352 image: the depthnet output is 8x22
    m.eval()
    with torch.no_grad():
        feats = m.camencode.get_eff_depth(torch.randn(1, 3, 128, 352))
    assert feats.shape == (1, 512, 8, 22)


def test_cpu_forward_fails_loudly():
    gc = syn.grid_conf()
    m = L.compile_model(gc, syn.data_aug_conf((64, 176)), outC=1)
    rig = syn.make_rig(1, 2, (64, 176))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m(torch.randn(1, 2, 3, 64, 176), **rig)


def test_synthetic_rig_shapes():
    rig = syn.make_rig(3, 6, (128, 352))
    assert rig["rots"].shape == (3, 6, 3, 3) and rig["post_trans"].shape == (3, 6, 3)
    # val-mode crop of the 224x480 image to 128x352: resize 352/480, crop_h = 164 - 128
    assert np.isclose(rig["post_rots"][0, 0, 0, 0].item(), 352 / 480)
    assert rig["post_trans"][0, 0].tolist() == [0.0, -36.0, 0.0]
    dn = syn.make_depthnet_out(1, 1, 41, 8, 22)
    assert dn.shape == (1, 105, 8, 22)


def test_bench_gpus_flag_launches_one_rank_per_gpu(monkeypatch):
    """`bench.py --gpus N` without a torchrun environment re-launches itself as N ranks (torchrun on
    127.0.0.1) before touching the GPU, and exits with the job's status."""
    import importlib.util
    import sys as _sys
    spec = importlib.util.spec_from_file_location("_bench", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 7

    monkeypatch.setattr(bench.subprocess, "call", fake_call)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(_sys, "argv", ["bench.py", "--gpus", "8", "--steps", "3"])
    args = bench.parse()
    with pytest.raises(SystemExit) as e:
        bench.maybe_launch_ranks(args)
    assert e.value.code == 7
    cmd = seen["cmd"]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"] and "--nproc-per-node=8" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"] and seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    monkeypatch.setenv("WORLD_SIZE", "8")  # under torchrun: no second launch
    assert bench.maybe_launch_ranks(args) is None
    assert args.config == "c3" and args.batch == 8 and args.mode == "train" and args.bev_layout == "nhwc"


def test_hip_adam_only_for_plain_cuda_adam():
    """optim.supported: the lss_clip_adam path is never taken for CPU tensors or other optimizers."""
    import torch
    from lss_carla_amd import optim
    ps = [torch.zeros(4, requires_grad=True), torch.zeros(3, requires_grad=True)]
    for p in ps:
        p.grad = torch.ones_like(p)
    assert not optim.supported(torch.optim.Adam(ps, lr=1e-3), ps)  # CPU tensors
    assert not optim.supported(torch.optim.SGD(ps, lr=1e-3), ps)


def test_pointwise_conv_size_guard():
    """pointwise_conv routes to lss_pw_conv / lss_pw_wrw only inside the index limits those kernels check
    (EINVAL past them); larger activations stay on the framework conv."""
    from lss_carla_amd import efficientnet as E
    assert E._pw_fits(48, 512, 105, 176)
    assert not E._pw_fits(4096, 1152, 192, 704)        # N * C * HW >= 2^31
    assert E._pw_fits(1, 2**20, 1, 2047) and not E._pw_fits(1, 2**20, 1, 2048)
