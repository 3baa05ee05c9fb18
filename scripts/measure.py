"""One parameterised GPU measurement runner (replaces the one-shot gpu_r4_* / gpu_r5_* scripts).

Runs the steps given on the command line in order, each under its own time limit, and stops at the
first step that fails (no retries). Outputs go to gpurun_out/<tag>/; copy what should be judged into
profiles/rNN/ (scripts/README.md lists which profile came from which step).

  python scripts/measure.py --tag r6a tests smoke "bench:c3" "trace:c3" \
      "bench:c3_caller:--caller reference --cpu-baseline 0 --pmc-traffic 0" \
      "pmc:plan:TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum:k_scan|k_scatter|k_csr|k_geometry:--graph 0"

Steps:
  tests[:pytest args]                 GPU suite (one process), log + summary line
  smoke                               __graft_entry__.smoke()
  bench:NAME[:bench.py args]          bench.py, its JSON line kept as NAME.json
  trace:NAME[:bench.py args]          rocprofv3 --kernel-trace --stats of bench.py (20 timed replays):
                                      NAME_kernel_stats.csv, NAME_hot_steps.txt, NAME_step_kernels.txt,
                                      NAME_steady_summary.json
  pmc:NAME:COUNTERS:REGEX[:args]      one rocprofv3 --pmc pass (COUNTERS space-separated, one block's
                                      limits) over bench.py (eager steps) for kernels matching REGEX:
                                      per-kernel averages in NAME.txt
  kbench:NAME:args                    scripts/kbench.py with args, log kept
  py:NAME:script args                 python scripts/<script> args (a diagnostics script), log kept
  lib:VARIANT                         later steps load lss-carla_amd/variants/VARIANT.so (product: the default)
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import re
import shlex
import shutil
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY = sys.executable


def run(cmd, log_path, limit, env=None, cwd=REPO) -> int:
    """cmd under `timeout -k 10 limit`, stdout+stderr to log_path; prints a progress line."""
    t0 = time.time()
    full = ["timeout", "-k", "10", str(limit)] + cmd
    with open(log_path, "w") as fh:
        proc = subprocess.Popen(full, stdout=fh, stderr=subprocess.STDOUT, env=env, cwd=cwd)
        while True:  # a heartbeat: a first step compiling library kernels can be silent for minutes
            try:
                rc = proc.wait(timeout=50)
                break
            except subprocess.TimeoutExpired:
                print(f"  ... {os.path.basename(log_path)} running, {time.time() - t0:.0f} s", flush=True)
    print(f"  rc={rc} in {time.time() - t0:.0f} s ({os.path.basename(log_path)})", flush=True)
    return rc


def tail(path, n=3) -> str:
    try:
        with open(path, errors="replace") as fh:
            return "".join(fh.readlines()[-n:])
    except OSError:
        return ""


def prof_env():
    return dict(os.environ, TMPDIR="/tmp")


def bench_args(extra: str) -> list:
    return shlex.split(extra) if extra else []


def step_tests(out, spec):
    args = shlex.split(spec) if spec else []
    if not any(a.startswith("tests") for a in args):
        args = ["tests"] + args
    log = os.path.join(out, "gpu_tests.log")
    rc = run([PY, "-u", "-m", "pytest", "-m", "gpu", "-q", "-rs", "-p", "no:cacheprovider",
              "--timeout", "200", "--timeout-method", "thread"] + args, log, 1000)
    print(tail(log, 3), flush=True)
    return rc


def step_smoke(out, _):
    log = os.path.join(out, "smoke.log")
    rc = run([PY, "-u", "-c", "import __graft_entry__ as g; g.smoke()"], log, 300)
    print(tail(log, 1), flush=True)
    return rc


def step_bench(out, spec):
    name, _, extra = spec.partition(":")
    log = os.path.join(out, f"{name}.log")
    rc = run([PY, "-u", "bench.py"] + bench_args(extra), log, 1000)
    last = tail(log, 1).strip()
    if rc == 0 and last.startswith("{"):
        with open(os.path.join(out, f"{name}.json"), "w") as fh:
            fh.write(last + "\n")
        print(last[:400], flush=True)
    else:
        print(tail(log, 15), flush=True)
    return rc


def step_trace(out, spec):
    name, _, extra = spec.partition(":")
    d = f"/tmp/measure_trace_{name}"
    shutil.rmtree(d, ignore_errors=True)
    log = os.path.join(out, f"{name}_trace.log")
    cmd = ["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", d, "-o", "run", "--",
           PY, "-u", os.path.join(REPO, "bench.py"), "--steps", "20", "--warmup", "3", "--profile-steps", "0",
           "--cpu-baseline", "0", "--pmc-traffic", "0", "--in-graph-prof", "0"] + bench_args(extra)
    rc = run(cmd, log, 700, env=prof_env(), cwd="/tmp")
    if rc != 0:
        print(tail(log, 15), flush=True)
        return rc
    tr = (glob.glob(f"{d}/**/run_kernel_trace.csv", recursive=True) or [None])[0]
    st = (glob.glob(f"{d}/**/run_kernel_stats.csv", recursive=True) or [None])[0]
    if st:
        shutil.copy(st, os.path.join(out, f"{name}_kernel_stats.csv"))
    if tr:
        for script, suffix, args in (("hot_steps.py", "hot_steps.txt", ["5", "23"]),
                                     ("step_kernels.py", "step_kernels.txt", ["5", "23", "400"]),
                                     ("steady_summary.py", "steady_summary.json", [])):
            with open(os.path.join(out, f"{name}_{suffix}"), "w") as fh:
                subprocess.call([PY, os.path.join(REPO, "scripts", script), tr] + args, stdout=fh,
                                stderr=subprocess.STDOUT)
        keep = os.path.join(out, f"{name}_kernel_trace.csv")
        # gpurun copies back at most 64 MiB of gpurun_out/: keep a trace only while the tag stays < 40 MiB
        used = sum(os.path.getsize(os.path.join(out, f)) for f in os.listdir(out))
        if used + os.path.getsize(tr) < 40 << 20:
            shutil.copy(tr, keep)
        print(tail(os.path.join(out, f"{name}_hot_steps.txt"), 12), flush=True)
    shutil.rmtree(d, ignore_errors=True)
    return 0


def step_pmc(out, spec):
    name, counters, regex, *rest = spec.split(":", 3)
    extra = rest[0] if rest else ""
    d = f"/tmp/measure_pmc_{name}"
    shutil.rmtree(d, ignore_errors=True)
    log = os.path.join(out, f"{name}_pmc.log")
    cmd = (["timeout", "-s", "KILL", "240", "rocprofv3", "--pmc"] + counters.split()
           + ["--output-format", "csv", "-d", d, "-o", "run", "--", PY, "-u", os.path.join(REPO, "bench.py"),
              "--steps", "6", "--warmup", "3", "--profile-steps", "0", "--graph", "0", "--cpu-baseline", "0",
              "--pmc-traffic", "0", "--in-graph-prof", "0"] + bench_args(extra))
    rc = run(cmd, log, 260, env=prof_env(), cwd="/tmp")
    if rc != 0:
        print(tail(log, 10), flush=True)
        return rc
    pat = re.compile(regex)
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if files and os.path.getsize(files[0]) < 32 << 20:  # kept for scripts/step_roofline.py
        shutil.copy(files[0], os.path.join(out, f"{name}_counter_collection.csv"))
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if pat.search(k):
                key = re.sub(r"\(anonymous namespace\)::", "", k).split("(")[0][:70]
                vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    with open(os.path.join(out, f"{name}.txt"), "w") as fh:
        fh.write(f"# rocprofv3 --pmc {counters} over bench.py --graph 0 {extra}; per-dispatch averages "
                 f"(first 2 dispatches of each kernel dropped)\n")
        for k, dd in sorted(vals.items()):
            fh.write(k + "\n")
            for c in sorted(dd):
                v = dd[c][2:] if len(dd[c]) > 4 else dd[c]
                fh.write(f"   {c:28s} {sum(v) / len(v):16.1f}   (n={len(v)})\n")
    print(open(os.path.join(out, f"{name}.txt")).read()[:3000], flush=True)
    shutil.rmtree(d, ignore_errors=True)
    return 0


def step_kbench(out, spec):
    name, _, extra = spec.partition(":")
    log = os.path.join(out, f"{name}.log")
    rc = run([PY, "-u", os.path.join("scripts", "kbench.py")] + bench_args(extra), log, 600)
    print(tail(log, 25), flush=True)
    return rc


def step_py(out, spec):
    name, _, extra = spec.partition(":")
    args = shlex.split(extra)
    log = os.path.join(out, f"{name}.log")
    rc = run([PY, "-u", os.path.join("scripts", args[0])] + args[1:], log, 600)
    print(tail(log, 40), flush=True)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("steps", nargs="+")
    a = ap.parse_args()
    out = os.path.join(REPO, "gpurun_out", a.tag)
    os.makedirs(out, exist_ok=True)
    os.chdir(REPO)
    fns = {"tests": step_tests, "smoke": step_smoke, "bench": step_bench, "trace": step_trace, "pmc": step_pmc,
           "kbench": step_kbench, "py": step_py}
    for s in a.steps:
        kind, _, spec = s.partition(":")
        print(f"== {s}", flush=True)
        if kind == "lib":
            if spec in ("", "product"):
                os.environ.pop("LSS_LIB", None)
            else:
                os.environ["LSS_LIB"] = os.path.join(REPO, "lss-carla_amd", "variants", spec + ".so")
            continue
        if kind == "env":  # env:NAME=VALUE for the steps that follow (env:NAME= unsets)
            k, _, v = spec.partition("=")
            if v:
                os.environ[k] = v
            else:
                os.environ.pop(k, None)
            continue
        rc = fns[kind](out, spec)
        if rc != 0:
            print(f"step {s!r} failed (rc={rc}); stopping", flush=True)
            sys.exit(rc if 0 < rc < 256 else 1)


if __name__ == "__main__":
    main()
