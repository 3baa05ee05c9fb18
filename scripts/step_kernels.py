"""Per-step kernel breakdown of a rocprofv3 kernel trace of bench.py (graph replays).

usage: python scripts/step_kernels.py <kernel_trace.csv> [first_step last_step] [top]
Steps are delimited by k_geometry_cells (one per step).
"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
geo = [i for i, r in enumerate(rows) if "k_geometry_cells" in r["Kernel_Name"]]
s0 = int(sys.argv[2]) if len(sys.argv) > 2 else 6
s1 = int(sys.argv[3]) if len(sys.argv) > 3 else 14
top = int(sys.argv[4]) if len(sys.argv) > 4 else 45
a, b = geo[s0], geo[s1]
sel, n = rows[a:b], s1 - s0
dur = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])  # noqa: E731
busy = sum(dur(r) for r in sel) / n / 1e3
span = (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / n / 1e3
print(f"{len(geo)} steps; per step: span {span:.0f} us, kernel busy {busy:.0f} us, {len(sel) / n:.0f} kernels")
agg = collections.defaultdict(lambda: [0, 0])
for r in sel:
    k = r["Kernel_Name"][:100]
    agg[k][0] += 1
    agg[k][1] += dur(r)
tot = sum(v[1] for v in agg.values())
for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
    print(f"{t / n / 1e3:8.1f} us {c / n:5.1f}x {t / c / 1e3:7.1f} avg {100 * t / tot:5.1f}%  {k}")
