"""Per-kernel summary of a rocprofv3 --kernel-trace CSV of bench.py: the LSS hot-path kernels (every
dispatch: graph replays + eager profiling steps) and the step's top kernels by total time.

  python scripts/steady_summary.py gpurun_out/r2/prof_c3/run_kernel_trace.csv > profiles/r02/bench_c3_steady_summary.json
"""
import csv
import json
import re
import statistics
import sys

HOT = ("k_splat_fwd", "k_splat_bwd", "k_depthnet_lift", "k_lift_prep", "k_geometry_cells", "k_scan", "k_scatter",
       "k_csr_canon", "k_camera_inverse", "k_bev_rows", "k_seg_", "k_flat_cast")


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    return name.split("(")[0][:90]


def main(path):
    per = {}
    for r in csv.DictReader(open(path)):
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        per.setdefault(short(r["Kernel_Name"]), []).append(d)
    hot = {k: {"calls": len(v), "avg_us": round(statistics.mean(v), 2), "median_us": round(statistics.median(v), 2),
               "min_us": round(min(v), 2)} for k, v in per.items() if any(h in k for h in HOT)}
    top = sorted(((k, sum(v)) for k, v in per.items()), key=lambda t: -t[1])[:25]
    print(json.dumps({"source": path, "hot_path_kernels": hot,
                      "top_kernels_total_us": {k: round(t, 1) for k, t in top}}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
