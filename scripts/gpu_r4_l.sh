# Round 4: the first zero-fill waves held back (s_sleep) so the chunk waves' two round trips meet
# an idle memory system; splat-only and in-step A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4l; mkdir -p $OUT
timeout -k 10 300 python -u scripts/splat_ab.py --config c3 --libs product,zs16,zs32,zs64,zs32all --ceiling 0 \
  > $OUT/splat_ab_c3.log 2>&1 || { tail -30 $OUT/splat_ab_c3.log; exit 1; }
grep -v '^{' $OUT/splat_ab_c3.log | grep -v amdgpu.ids
bash scripts/gpu_prof_ab.sh product zs32 zs64 product 2>&1 | tee $OUT/prof_ab.txt || exit 1
