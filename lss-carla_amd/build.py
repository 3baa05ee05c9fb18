"""Build ``liblss_hip.so`` in-tree with hipcc for gfx950.

``python -m lss_carla_amd.build`` or ``__graft_entry__.build()``. The shared
library lands next to this file so it travels with the repo snapshot to the
GPU box (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SOURCES = [os.path.join(HERE, "csrc", f) for f in ("lss_hip.hip", "lss_convs.hip", "lss_bnorm.hip",
                                                            "lss_resample.hip", "lss_se.hip", "lss_simbev.hip",
                                                            "lss_ceiling.hip", "lss_optim.hip")]
HEADERS = [os.path.join(REPO, "include", h) for h in ("lss_hip.h", "lss_convs.h", "lss_simbev.h")]
OUT = os.path.join(HERE, "liblss_hip.so")
# LSS_DEBUG build: every data-derived index checked on the device (include/lss_hip.h, lss_debug_status);
# loaded instead of the product library when LSS_DEBUG=1 (_lib.py)
OUT_DEBUG = os.path.join(HERE, "liblss_hip_debug.so")
ARCH = os.environ.get("LSS_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build liblss_hip.so)")


def command(out: str = OUT, defines=()):
    # -ffp-contract=off: the geometry must keep the reference's un-fused fp32 op order.
    return [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
            "-Wall", "-Wno-unused-function", f"-I{os.path.join(REPO, 'include')}"] + \
        [f"-D{d}" for d in defines] + ["-o", out] + SOURCES


def build_variant(name: str, defines) -> str:
    """Tuning build with extra -D knobs into lss-carla_amd/variants/<name>.so (scripts/kbench.py)."""
    vdir = os.path.join(HERE, "variants")
    os.makedirs(vdir, exist_ok=True)
    out = os.path.join(vdir, f"{name}.so")
    r = subprocess.run(command(out, defines), capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"hipcc failed building variant {name}")
    return out


def up_to_date(out: str = OUT) -> bool:
    if not os.path.exists(out):
        return False
    t = os.path.getmtime(out)
    return all(os.path.getmtime(s) <= t for s in SOURCES + HEADERS + [__file__])


def build(force: bool = False, verbose: bool = True, debug: bool = True) -> str:
    """The product library and (debug=True) the LSS_DEBUG library, compiled concurrently."""
    jobs = [(OUT, ())] + ([(OUT_DEBUG, ("LSS_DEBUG=1",))] if debug else [])
    procs = []
    for out, defines in jobs:
        if not force and up_to_date(out):
            continue
        cmd = command(out, defines)
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((out, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)))
    for out, p in procs:
        so, se = p.communicate()
        if p.returncode != 0:
            sys.stderr.write(so + se)
            raise RuntimeError(f"hipcc failed ({p.returncode}) building {out}")
        if verbose and se.strip():
            sys.stderr.write(se)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
