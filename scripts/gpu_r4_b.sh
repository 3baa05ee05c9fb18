# Round 4, after pruning the ABI (v17): the GPU suite, then the splat variants (zero-fill units x
# dispatch order; the NCHW tile kernel's channel split) with the write ceiling (scripts/splat_ab.py),
# then the in-step splat of a few builds (scripts/gpu_prof_ab.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4b; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1; rc=$?
tail -15 $OUT/gpu_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/splat_ab.py --config c3 --libs product,o2,zu2_o2,zu4_o2,zu8_o2,zu16_o2,zu8_o1,zu4_o0 \
  > $OUT/splat_ab_c3.log 2>&1 || { tail -30 $OUT/splat_ab_c3.log; exit 1; }
grep -v '^{' $OUT/splat_ab_c3.log | grep -v amdgpu.ids
for cfg in c2 c3; do
  timeout -k 10 300 python -u scripts/splat_ab.py --config $cfg --layout nchw --dtype f32 --libs product,nq2,nq4 \
    --modes dirty,step --ceiling 0 > $OUT/splat_ab_${cfg}_nchw.log 2>&1 || { tail -30 $OUT/splat_ab_${cfg}_nchw.log; exit 1; }
  grep -v '^{' $OUT/splat_ab_${cfg}_nchw.log | grep -v amdgpu.ids
done
bash scripts/gpu_prof_ab.sh product zu8_o2 zu4_o2 zu16_o2 2>&1 | tee $OUT/prof_ab.txt
