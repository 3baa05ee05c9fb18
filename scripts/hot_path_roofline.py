"""Roofline fraction of every hot-path kernel of the c3 training step, from a rocprofv3 steady-state
summary (scripts/steady_summary.py output) and the algorithmic bytes / flops of DESIGN.md §4.

usage: python scripts/hot_path_roofline.py profiles/r02/bench_c3_steady_summary.json > profiles/r02/hot_path_roofline.json
"""
import json
import sys

HBM = 8000.0         # GB/s, MI355X HBM3E peak
BF16_DENSE = 2500.0  # TFLOP/s, dense bf16 MFMA

# c3: B=8, N=6, D=41, fH x fW = 8 x 22, 200 x 200 BEV, Z=1, C=64; kept points from the bench plan
B, N, D, H, W, C, X, Y = 8, 6, 41, 8, 22, 64, 200, 200
NPRIME = B * N * D * H * W
PIX = B * N * H * W
CELLS = B * X * Y
KEPT = 344720

KERNELS = {  # name fragment -> (algorithmic bytes, flops, what the bytes are)
    "k_geometry_cells": (20 * NPRIME + 4 * CELLS, None,
                         "frustum 12 B + cell_of 4 B + slot 4 B per point, counts 4 B per cell"),
    "k_scan_lookback": (8 * CELLS, None, "counts read + cell_start written, 4 B each per cell"),
    "k_scatter_ws": (20 * NPRIME + 4 * CELLS, None,
                     "cell_of + slot read, key 8 B + row 4 B written per point; counts re-zeroed"),
    "k_csr_canon": (24 * KEPT, None, "key 8 B + row 4 B read and written per entry"),
    "k_depthnet_lift2": (PIX * (512 * 2 + D * 4 + C * 2 + 2 * 2) + (D + C) * 512 * 2, 2 * PIX * 512 * (D + C),
                         "features 1024 B + depth 164 B + context row 128 B per pixel, weights once"),
    "k_splat_fwd_nhwc": (NPRIME * 4 + PIX * C * 2 + KEPT * 4 + (CELLS + 1) * 4 + CELLS * C * 2, None,
                         "depth weights, context rows, point ids, cell_start, dense bf16 BEV"),
    "k_splat_bwd_tile": (PIX * (D * 4 * 2 + 128 + (D + C) * 2) + KEPT * 128, None,
                         "depth + cell_of, context row, d_depthnet_out per pixel; one 128-B gradient row "
                         "per kept point (L2 / Infinity Cache gathers)"),
}


def main():
    summ = json.load(open(sys.argv[1]))["hot_path_kernels"]
    out = {"source": sys.argv[1], "peak_hbm_GBps": HBM, "peak_bf16_TFLOPs": BF16_DENSE, "kernels": {}}
    total_us = 0.0
    for frag, (nbytes, flops, what) in KERNELS.items():
        hit = [v for k, v in summ.items() if frag in k]
        if not hit:
            continue
        us = hit[0]["avg_us"]
        total_us += us
        row = {"avg_us_in_step": us, "algorithmic_bytes": nbytes, "bytes_are": what,
               "achieved_GBps": round(nbytes / us / 1e3, 1), "hbm_frac": round(nbytes / us / 1e3 / HBM, 4)}
        if flops:
            row["flops"] = flops
            row["mfma_frac"] = round(flops / us / 1e6 / BF16_DENSE, 4)
        out["kernels"][frag] = row
    out["hot_path_total_us"] = round(total_us, 2)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
