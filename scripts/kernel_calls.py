"""Every call of the kernels matching a pattern in one step of a rocprofv3 kernel trace of bench.py, in
launch order, with grid size and duration (per-layer view of a conv kernel).

usage: python scripts/kernel_calls.py <kernel_trace.csv> <pattern> [step]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
geo = [i for i, r in enumerate(rows) if "k_geometry_cells" in r["Kernel_Name"]]
st = int(sys.argv[3]) if len(sys.argv) > 3 else 8
a, b = geo[st], geo[st + 1]
tot = 0.0
for r in rows[a:b]:
    if sys.argv[2] in r["Kernel_Name"]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        grid = r.get("Grid_Size_X", r.get("Grid_Size", "?"))
        print(f"{d:8.2f} us  grid {grid:>8}  {r['Kernel_Name'][:90]}")
print(f"total {tot:.1f} us")
