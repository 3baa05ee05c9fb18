# Round 4: splat role split (chunk waves alone / zero fill alone) and chunk-wave priority, splat-only
# A/B and in-step (graph replay) A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4e; mkdir -p $OUT
timeout -k 10 300 python -u scripts/splat_ab.py --config c3 --libs product,chunkonly,zeroonly,prio1,prio3 --ceiling 0 \
  > $OUT/splat_ab_c3.log 2>&1 || { tail -30 $OUT/splat_ab_c3.log; exit 1; }
grep -v '^{' $OUT/splat_ab_c3.log | grep -v amdgpu.ids
bash scripts/gpu_prof_ab.sh product prio1 prio3 product chunkonly 2>&1 | tee $OUT/prof_ab.txt || exit 1
