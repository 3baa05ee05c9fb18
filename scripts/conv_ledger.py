"""Every convolution of the c3 training step with its shapes and FLOPs (forward, and the two backward
GEMMs: data and weight gradients), from forward hooks on the model's Conv2d modules run on the CPU
(shapes only: the trunk on the 48 camera images, the depthnet, BevEncode on the 8 BEVs).

  python scripts/conv_ledger.py > profiles/r06/conv_ledger_c3.json

Kinds (which kernels run them in the bf16 training step): "dense" (k x k, groups 1: MIOpen / CK
igemm and grouped-conv kernels, hipBLASLt GEMMs for the stride-2 1x1 downsamples), "pointwise" (the
trunk's 1x1 expand / project convs: lss_pw_conv / lss_pw_wrw), "depthwise" (lss_dw_*), "se" (the
squeeze-excite 1x1 convs on 1x1 maps: lss_se_*), "depthnet" (fused into k_depthnet_lift3), "head"
(BevEncode's last 1x1 conv, one output channel: lss_head1_*).
"""
import json
import os
import sys

import torch
import torch.nn as nn

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import lss_carla_amd as L
    from lss_carla_amd import synthetic as syn
    cfg, gc, dac = syn.config_confs("c3")
    B, N, (H, W) = cfg["B"], cfg["N"], cfg["final_dim"]
    torch.manual_seed(0)
    m = L.compile_model(gc, dac, 1).float().train()
    m.bevencode.to(memory_format=torch.contiguous_format)
    rows = []

    def hook(mod, inp, out):
        x = inp[0]
        n, cin, hi, wi = x.shape
        _, cout, ho, wo = out.shape
        kh, kw = mod.kernel_size
        g = mod.groups
        macs = n * ho * wo * cout * (cin // g) * kh * kw
        if mod is m.camencode.depthnet:
            kind = "depthnet"
        elif g > 1:
            kind = "depthwise"
        elif hi == 1 and wi == 1:
            kind = "se"
        elif mod.out_channels == 1:
            kind = "head"
        elif (kh, kw) == (1, 1) and mod.stride == (1, 1) and mod.bias is None and n == B * N:
            kind = "pointwise"
        else:
            kind = "dense"
        rows.append({"name": names[mod], "kind": kind, "in": [n, cin, hi, wi], "out": [n, cout, ho, wo],
                     "k": [kh, kw], "stride": list(mod.stride), "groups": g,
                     "flops_fwd": 2 * macs, "flops_fwd_bwd": 6 * macs})

    names = {mod: nm for nm, mod in m.named_modules()}
    hs = [mod.register_forward_hook(hook) for mod in m.modules() if isinstance(mod, nn.Conv2d)]
    with torch.no_grad():
        x = torch.randn(B * N, 3, H, W)
        feat = m.camencode.get_eff_depth(x)
        m.camencode.depthnet(feat)
        X, Y = 200, 200
        m.bevencode(torch.randn(B, 64, X, Y))
    for h in hs:
        h.remove()
    tot = {}
    for r in rows:
        t = tot.setdefault(r["kind"], {"convs": 0, "flops_fwd_bwd": 0})
        t["convs"] += 1
        t["flops_fwd_bwd"] += r["flops_fwd_bwd"]
    print(json.dumps({"config": "c3: B=8 x 6 cams x 128x352 (trunk on 48 images), BEV 8 x 64 x 200 x 200",
                      "flops_note": "fwd = 2*MACs; fwd+bwd = 3x (data and weight gradients; the stem's data "
                                    "gradient is not needed, counted anyway)",
                      "totals": tot, "total_flops_fwd_bwd": sum(t["flops_fwd_bwd"] for t in tot.values()),
                      "convs": rows}, indent=1))


if __name__ == "__main__":
    main()
