"""Steady-state per-step kernel summary from a rocprofv3 kernel trace of bench.py.

Steps are delimited by the k_geometry_cells dispatch (one per training step); the first
`--skip` steps (warm-up, MIOpen find) are dropped. Also writes the splat PMC traffic json.
usage: python scripts/trace_summary.py <round_dir> <out_dir> [--skip N]
"""
import argparse
import collections
import csv
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("round_dir")
ap.add_argument("out_dir")
ap.add_argument("--skip", type=int, default=4)
ap.add_argument("--config", default="c3")
ap.add_argument("--out-bytes", type=int, default=2)
a = ap.parse_args()
os.makedirs(a.out_dir, exist_ok=True)

rows = list(csv.DictReader(open(os.path.join(a.round_dir, "trace", "run_kernel_trace.csv"))))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "k_geometry_cells" in r["Kernel_Name"]]
# bench.py computes one extra plan after timing (for `kept`): ignore dispatches after the last step
first = marks[a.skip]
last = marks[-1]
steady = rows[first:last]
nsteps = len(marks) - 1 - a.skip
agg = collections.defaultdict(lambda: [0, 0.0])
for r in steady:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    agg[r["Kernel_Name"]][0] += 1
    agg[r["Kernel_Name"]][1] += d
tot = sum(v[1] for v in agg.values())
span = (int(rows[last]["Start_Timestamp"]) - int(rows[first]["Start_Timestamp"])) / 1e3
with open(os.path.join(a.out_dir, "bench_steady_kernels.csv"), "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["kernel", "calls_per_step", "us_per_step", "avg_us", "pct_of_kernel_time"])
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        w.writerow([k[:160], round(n / nsteps, 2), round(t / nsteps, 2), round(t / n, 2), round(100 * t / tot, 2)])
summary = {"steps": nsteps, "kernel_us_per_step": round(tot / nsteps, 1), "wall_us_per_step": round(span / nsteps, 1),
           "lss_kernels_us_per_step": round(sum(t for k, (n, t) in agg.items() if "::k_" in k) / nsteps, 1)}
lss = {k[k.find("::k_") + 2:].split("(")[0]: round(t / n, 2) for k, (n, t) in agg.items() if "::k_" in k}
summary["lss_kernel_avg_us"] = lss


def pmc(counter):
    p = os.path.join(a.round_dir, f"pmc_{counter}", "run_counter_collection.csv")
    if not os.path.exists(p):
        return None
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(p)) if "k_splat_fwd" in r["Kernel_Name"]]
    return sum(v) / len(v) if v else None


fetch, write = pmc("FETCH_SIZE"), pmc("WRITE_SIZE")
if fetch is not None and write is not None:
    traffic = {"config": a.config, "out_bytes": a.out_bytes, "kernel": "k_splat_fwd",
               "fetch_size_kb": round(fetch, 1), "write_size_kb": round(write, 1),
               "hbm_bytes_per_launch": int((fetch + write) * 1024),
               "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over the bench's training steps, "
                       "KB x1024, averaged over the splat launches. FETCH_SIZE counts the reads that left L2 for the "
                       "fabric (Infinity Cache or HBM); the context-row gathers are 16-B lane slices of L2-resident "
                       "rows, not a streaming read, so no x2 correction is applied. WRITE_SIZE is exact for the "
                       "16-B row stores."}
    with open(os.path.join(a.out_dir, "splat_fwd_traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1)
    summary["splat_fwd_traffic"] = traffic
with open(os.path.join(a.out_dir, "bench_steady_summary.json"), "w") as f:
    json.dump(summary, f, indent=1)
print(json.dumps(summary, indent=1))
