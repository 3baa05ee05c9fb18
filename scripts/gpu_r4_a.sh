# Round 4, experiment A: splat forward variants (zero-fill units x dispatch order) and the HBM write
# ceiling in the step's cache states (scripts/splat_ab.py), then the in-step (graph replay) splat time
# of a few builds (scripts/gpu_prof_ab.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4a
timeout -k 10 300 python -u scripts/splat_ab.py --config c3 --libs product,skipzero,skipchunk,o2,zu2_o2,zu4_o2,zu8_o2,zu16_o2,zu8_o1 \
  > gpurun_out/r4a/splat_ab_c3.log 2>&1 || { tail -30 gpurun_out/r4a/splat_ab_c3.log; exit 1; }
grep -v '^{' gpurun_out/r4a/splat_ab_c3.log | grep -v amdgpu.ids
bash scripts/gpu_prof_ab.sh product zu8_o2 zu16_o2 zu4_o2 2>&1 | tee gpurun_out/r4a/prof_ab.txt
