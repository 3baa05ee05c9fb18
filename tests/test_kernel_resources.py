"""The hot-path kernels of the built library use no scratch memory (no register spills, no private
arrays left in memory). A spilled value costs a store and a reload through the memory pipeline, and the
reload's wait also waits for every load issued before it (one vmcnt for all): round 4 found the lane's
column of the channels-last splat spilled (a reload round trip at every chunk wave's end) and the
feature tile of k_depthnet_lift3 kept in scratch (its stage serialised). Reads the kernel descriptors
of the gfx950 code objects embedded in liblss_hip.so (AMDGPU metadata notes); no GPU needed."""
import glob
import os
import re
import shutil
import subprocess
import tempfile

import pytest

from lss_carla_amd import _lib

LLVM = "/opt/rocm/lib/llvm/bin"
HOT = ("k_geometry_cells", "k_scan_lookback", "k_scatter_ws", "k_scatter_ord", "k_cells_from_geom_ord", "k_csr_canon", "k_lift_prep", "k_depthnet_lift2",
       "k_depthnet_lift3", "k_splat_fwd_nhwc", "k_splat_fwd_nchw2", "k_splat_bwd_tile", "k_splat_bwd_reg",
       "k_bev_rows")


def _kernel_notes(lib_path):
    objdump, readelf = os.path.join(LLVM, "llvm-objdump"), os.path.join(LLVM, "llvm-readelf")
    if not (os.path.exists(objdump) and os.path.exists(readelf) and os.path.exists(lib_path)):
        pytest.skip("ROCm llvm tools or the built library missing")
    with tempfile.TemporaryDirectory() as d:
        so = os.path.join(d, "lib.so")
        shutil.copy(lib_path, so)  # the bundles are extracted next to the input file
        subprocess.run([objdump, "--offloading", so], cwd=d, check=True, capture_output=True)
        notes = ""
        for obj in sorted(glob.glob(os.path.join(d, "lib.so.*gfx950"))):
            notes += subprocess.run([readelf, "--notes", obj], check=True, capture_output=True, text=True).stdout
    kernels = {}
    cur = None
    for line in notes.splitlines():
        m = re.match(r"\s*\.name:\s+(\S+)", line)
        if m:
            cur = m.group(1)
            kernels[cur] = {}
            continue
        m = re.match(r"\s*\.(private_segment_fixed_size|vgpr_spill_count|sgpr_spill_count):\s+(\d+)", line)
        if m and cur is not None:
            kernels[cur][m.group(1)] = int(m.group(2))
    return kernels


def test_hot_path_kernels_use_no_scratch():
    # (the product library only: the debug build's index checks may spill, it is not timed)
    kernels = _kernel_notes(_lib.LIB_PATH)
    hot = {k: v for k, v in kernels.items() if any(h in k for h in HOT)}
    assert len(hot) >= len(HOT), sorted(hot)
    bad = {k: v for k, v in hot.items()
           if v.get("private_segment_fixed_size", 0) or v.get("vgpr_spill_count", 0)}
    assert not bad, bad
