"""Average PMC counters per dispatch for kernels matching a pattern (gpurun_out/pmc/p*/.../*counter_collection.csv)."""
import collections
import csv
import glob
import sys

pat = sys.argv[1] if len(sys.argv) > 1 else "k_splat"
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            name = r["Kernel_Name"]
            key = name[name.find("::k_"):][:70] if "::k_" in name else name[:70]
            vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    print(k)
    for c in sorted(d):
        v = d[c]
        print(f"   {c:28s} {sum(v) / len(v):16.1f}   (n={len(v)})")
