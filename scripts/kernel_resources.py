"""Print VGPR/SGPR/LDS/occupancy/scratch per kernel of lss_hip.hip (hipcc -Rpass-analysis)."""
import re
import subprocess
import sys

cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-Iinclude", "-c",
       "-o", "/tmp/_lss_res.o", "lss-carla_amd/csrc/lss_hip.hip", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, []
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    txt = m.group(1)
    if txt.startswith("Function Name:"):
        cur = {"name": txt.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in txt:
        k, v = txt.split(":", 1)
        cur[k.strip()] = v.strip()
pat = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if pat in r["name"]:
        short = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", r["name"])[:60]
        print(f"{short:60s} vgpr={r.get('VGPRs','?'):>4} agpr={r.get('AGPRs','?'):>3} sgpr={r.get('SGPRs','?'):>3} "
              f"lds={r.get('LDS Size [bytes/block]','?'):>6} occ={r.get('Occupancy [waves/SIMD]','?'):>2} "
              f"scratch={r.get('ScratchSize [bytes/lane]','?')}")
