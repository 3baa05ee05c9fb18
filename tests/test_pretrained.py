"""EfficientNetB0.from_pretrained from a local efficientnet_pytorch-format state dict (src/models.py:43
downloads ImageNet weights; here nothing is fetched). The synthetic checkpoint is built from the
package's published B0 block strings, independently of this repo's module, so the key names and
shapes are those a real efficientnet-b0-355c32eb.pth holds."""
import os

import pytest
import torch

import lss_carla_amd as L
from lss_carla_amd import synthetic as syn
from lss_carla_amd.efficientnet import EfficientNetB0

# efficientnet_pytorch.utils.efficientnet(): blocks_args of B0 (width = depth = 1.0)
B0_BLOCKS_ARGS = ["r1_k3_s11_e1_i32_o16_se0.25", "r2_k3_s22_e6_i16_o24_se0.25", "r2_k5_s22_e6_i24_o40_se0.25",
                  "r3_k3_s22_e6_i40_o80_se0.25", "r3_k5_s11_e6_i80_o112_se0.25", "r4_k5_s22_e6_i112_o192_se0.25",
                  "r1_k3_s11_e6_i192_o320_se0.25"]


def _bn(prefix, c, sd, g):
    sd[prefix + ".weight"] = torch.rand(c, generator=g) + 0.5
    sd[prefix + ".bias"] = torch.randn(c, generator=g)
    sd[prefix + ".running_mean"] = torch.randn(c, generator=g)
    sd[prefix + ".running_var"] = torch.rand(c, generator=g) + 0.5


def published_b0_state_dict(seed=0, num_classes=1000):
    """Keys and shapes of efficientnet_pytorch's B0 (no num_batches_tracked, as the published file)."""
    g = torch.Generator().manual_seed(seed)
    sd = {"_conv_stem.weight": torch.randn(32, 3, 3, 3, generator=g)}
    _bn("_bn0", 32, sd, g)
    i = 0
    for s in B0_BLOCKS_ARGS:
        a = {t[0]: t[1:] for t in s.split("_")}
        r, k, e, cin, cout = int(a["r"]), int(a["k"]), int(a["e"]), int(a["i"]), int(a["o"])
        for j in range(r):
            fin = cin if j == 0 else cout
            mid = fin * e
            p = f"_blocks.{i}"
            if e != 1:
                sd[p + "._expand_conv.weight"] = torch.randn(mid, fin, 1, 1, generator=g)
                _bn(p + "._bn0", mid, sd, g)
            sd[p + "._depthwise_conv.weight"] = torch.randn(mid, 1, k, k, generator=g)
            _bn(p + "._bn1", mid, sd, g)
            sq = max(1, int(fin * 0.25))
            sd[p + "._se_reduce.weight"] = torch.randn(sq, mid, 1, 1, generator=g)
            sd[p + "._se_reduce.bias"] = torch.randn(sq, generator=g)
            sd[p + "._se_expand.weight"] = torch.randn(mid, sq, 1, 1, generator=g)
            sd[p + "._se_expand.bias"] = torch.randn(mid, generator=g)
            sd[p + "._project_conv.weight"] = torch.randn(cout, mid, 1, 1, generator=g)
            _bn(p + "._bn2", cout, sd, g)
            i += 1
    sd["_conv_head.weight"] = torch.randn(1280, 320, 1, 1, generator=g)
    _bn("_bn1", 1280, sd, g)
    sd["_fc.weight"] = torch.randn(num_classes, 1280, generator=g)
    sd["_fc.bias"] = torch.randn(num_classes, generator=g)
    return sd


def test_from_pretrained_round_trip(tmp_path):
    sd = published_b0_state_dict()
    path = str(tmp_path / "efficientnet-b0.pth")
    torch.save(sd, path)
    m = EfficientNetB0.from_pretrained("efficientnet-b0", weights_path=path)
    got = m.state_dict()
    for k, v in sd.items():
        assert torch.equal(got[k], v), k
    assert set(got) - set(sd) == {k for k in got if k.endswith("num_batches_tracked")}


def test_from_pretrained_safetensors_and_no_fc(tmp_path):
    from safetensors.torch import save_file
    sd = published_b0_state_dict(seed=1)
    path = str(tmp_path / "b0.safetensors")
    save_file(sd, path)
    m = EfficientNetB0.from_pretrained("efficientnet-b0", weights_path=path, load_fc=False, num_classes=10)
    assert m._fc.weight.shape == (10, 1280)
    assert torch.equal(m._blocks[15]._project_conv.weight, sd["_blocks.15._project_conv.weight"])


def test_from_pretrained_rejects_other_files(tmp_path):
    sd = published_b0_state_dict()
    sd["_blocks.16._depthwise_conv.weight"] = torch.zeros(1)  # a B1-style extra block
    path = str(tmp_path / "bad.pth")
    torch.save(sd, path)
    with pytest.raises(RuntimeError, match="unexpected"):
        EfficientNetB0.from_pretrained("efficientnet-b0", weights_path=path)
    del sd["_blocks.16._depthwise_conv.weight"]
    del sd["_conv_head.weight"]
    torch.save(sd, path)
    with pytest.raises(RuntimeError, match="missing"):
        EfficientNetB0.from_pretrained("efficientnet-b0", weights_path=path)
    with pytest.raises(RuntimeError, match="no download"):
        EfficientNetB0.from_pretrained("efficientnet-b0")
    with pytest.raises(ValueError):
        EfficientNetB0.from_pretrained("efficientnet-b1", weights_path=path)


def test_compile_model_picks_up_local_weights(tmp_path, monkeypatch):
    """An unchanged train_simbev.py (compile_model) trains from the local ImageNet weights when
    $LSS_EFFICIENTNET_B0_WEIGHTS names them -- the reference's from_pretrained without the download."""
    sd = published_b0_state_dict(seed=2)
    path = str(tmp_path / "b0.pth")
    torch.save(sd, path)
    monkeypatch.setenv("LSS_EFFICIENTNET_B0_WEIGHTS", path)
    m = L.compile_model(syn.grid_conf(), syn.data_aug_conf((128, 352), 6), outC=1)
    got = m.state_dict()
    for k, v in sd.items():
        assert torch.equal(got["camencode.trunk." + k], v), k
