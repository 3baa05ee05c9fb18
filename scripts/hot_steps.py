"""Hot-path kernels per training step from a rocprofv3 --kernel-trace CSV of bench.py, over the steps
[s0, s1) (steps delimited by k_geometry_cells; with --profile-steps 0 and warmup 3, steps 5.. are the
timed graph replays): average in-step duration of each hot kernel and the hot path's sum.

  python scripts/hot_steps.py <kernel_trace.csv> [s0 s1]
"""
import collections
import csv
import re
import sys

HOT = ("k_splat_fwd", "k_splat_bwd", "k_depthnet_lift", "k_lift_prep", "k_geometry_cells", "k_scan", "k_scatter",
       "k_csr_canon", "k_bev_rows", "k_depthnet_pack")
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
geo = [i for i, r in enumerate(rows) if "k_geometry_cells" in r["Kernel_Name"]]
s0 = int(sys.argv[2]) if len(sys.argv) > 2 else 5
s1 = int(sys.argv[3]) if len(sys.argv) > 3 else min(len(geo) - 1, s0 + 8)
sel = rows[geo[s0]:geo[s1]]
n = s1 - s0
agg = collections.defaultdict(list)
for r in sel:
    k = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0]
    if any(h in k for h in HOT):
        agg[k[:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = 0.0
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    per = sum(v) / n
    tot += per
    print(f"{k:60s} {len(v) / n:4.1f}x  avg {sum(v) / len(v):7.2f} us  min {min(v):7.2f}  per step {per:7.2f}")
span = (int(rows[geo[s1]]["Start_Timestamp"]) - int(rows[geo[s0]]["Start_Timestamp"])) / n / 1e3
print(f"hot path per step {tot:.1f} us; step span {span:.0f} us ({len(geo)} steps in trace, steps {s0}..{s1})")
