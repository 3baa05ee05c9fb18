"""Step-level roofline of the c3 training step: the top kernels of the captured step by time, each with
its bytes per call (rocprofv3 PMC FETCH_SIZE / WRITE_SIZE of the same kernel in eager steps of the same
bench, FETCH doubled per MI355X_MICROARCH.md's gfx950 correction), the achieved GB/s and its fraction
of the bench's own measured ceilings (the hand-written streaming-store ceiling and torch's copy of the
BEV buffer, bench.py `roofline.write_ceiling`), and for the convolution kernels the FLOPs of the
convolutions they run (scripts/conv_ledger.py) against the dense bf16 MFMA peak.

  python scripts/step_roofline.py <kernel_trace.csv> <pmc_fetch_dir> <pmc_write_dir> <conv_ledger.json> \
      <bench.json> [top] > profiles/r06/step_roofline.json

Kernel time per step: steps delimited by the geometry kernel, steps 5..23 of a `measure.py trace` run
(the timed graph replays). PMC bytes: per-dispatch averages over the eager steps of a `measure.py pmc`
run. FETCH_SIZE is calibrated only for 16-B-per-lane streaming reads; narrower or gathered reads are
read as-is (noted per row as `fetch_calibrated`: false where the kernel's reads are not all 16-B wide
is not known here, so the doubling is applied to every kernel and flagged).
"""
import collections
import csv
import glob
import json
import re
import sys

HBM = 8000.0  # GB/s
BF16 = 2500.0  # TFLOP/s dense

# kernel-name patterns -> the convolution kind of conv_ledger.py whose FLOPs they run
CONV_FAMILIES = [
    (r"igemm_|grouped_conv|conv_fwd|conv_bwd|conv_wrw|Cijk_|gemm_xdl|naive_conv", "dense"),
    (r"k_pw_gemm|k_pw_wrw(?!_reduce)", "pointwise"),
    (r"k_dw_", "depthwise"),
    (r"k_depthnet_lift", "depthnet"),
]


def short(name: str) -> str:
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    n = re.sub(r"^void ", "", n)
    return n.split("(")[0][:90]


def per_step_times(trace_csv, s0=5, s1=23):
    rows = list(csv.DictReader(open(trace_csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    geo = [i for i, r in enumerate(rows) if "k_geometry_cells" in r["Kernel_Name"]]
    s1 = min(s1, len(geo) - 1)
    sel = rows[geo[s0]:geo[s1]]
    n = s1 - s0
    agg = collections.defaultdict(list)
    for r in sel:
        agg[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    busy = sum(sum(v) for v in agg.values()) / n
    return agg, n, busy


def pmc_bytes(path, counter):
    vals = collections.defaultdict(list)
    files = [path] if path.endswith(".csv") else glob.glob(f"{path}/**/*counter_collection.csv", recursive=True)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)  # KiB
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    trace, fdir, wdir, ledger_p, bench_p = sys.argv[1:6]  # (the PMC arguments: a counter CSV or a directory)
    top = int(sys.argv[6]) if len(sys.argv) > 6 else 30
    agg, nsteps, busy = per_step_times(trace)
    fetch, write = pmc_bytes(fdir, "FETCH_SIZE"), pmc_bytes(wdir, "WRITE_SIZE")
    ledger = json.load(open(ledger_p))
    bench = json.loads(open(bench_p).read().strip().splitlines()[-1])
    wc = bench["roofline"]["write_ceiling"]
    store_ceiling, copy_ceiling = wc["GB/s"], wc["copy_GB/s"]
    kinds_time = collections.defaultdict(float)
    for k, v in agg.items():
        for pat, kind in CONV_FAMILIES:
            if re.search(pat, k):
                kinds_time[kind] += sum(v) / nsteps
                break
    kinds = {}
    for kind, t in kinds_time.items():
        fl = ledger["totals"].get(kind, {}).get("flops_fwd_bwd", 0)
        kinds[kind] = {"us_per_step": round(t, 1), "flops_per_step": fl,
                       "TFLOP/s": round(fl / t / 1e6, 1) if t and fl else None,
                       "mfma_frac": round(fl / t / 1e6 / BF16, 4) if t and fl else None}
    rows = []
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
        per_step = sum(v) / nsteps
        calls = len(v) / nsteps
        avg = sum(v) / len(v)
        row = {"kernel": k, "calls_per_step": round(calls, 2), "us_per_step": round(per_step, 1),
               "avg_us": round(avg, 2), "share_of_busy": round(per_step / busy, 4)}
        fam = next((kind for pat, kind in CONV_FAMILIES if re.search(pat, k)), None)
        if fam:
            row["conv_family"] = fam
        if k in fetch or k in write:
            b = 2.0 * fetch.get(k, 0.0) + write.get(k, 0.0)
            row.update({"pmc_bytes_per_call": round(b), "read_bytes": round(2.0 * fetch.get(k, 0.0)),
                        "write_bytes": round(write.get(k, 0.0)), "GB/s": round(b / avg / 1e3, 1),
                        "hbm_frac": round(b / avg / 1e3 / HBM, 4),
                        "frac_of_store_ceiling": round(b / avg / 1e3 / store_ceiling, 4),
                        "frac_of_copy_ceiling": round(b / avg / 1e3 / copy_ceiling, 4)})
        rows.append(row)
    out = {"source": {"trace": trace, "pmc_fetch": fdir, "pmc_write": wdir, "ledger": ledger_p, "bench": bench_p},
           "steps": nsteps, "kernel_busy_us_per_step": round(busy, 1),
           "ceilings_GBps": {"hbm_peak": HBM, "store_measured": store_ceiling, "copy_measured": copy_ceiling},
           "conv_families": kinds, "top_kernels": rows,
           "notes": "bytes = 2 x FETCH_SIZE + WRITE_SIZE per dispatch (eager steps, PMC); the doubling is "
                    "calibrated for 16-B-per-lane streaming reads only, so for gather-heavy kernels the read "
                    "bytes are an estimate; graph replays and eager steps run the same kernels"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
