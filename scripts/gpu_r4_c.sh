# Round 4: the GPU suite at HEAD, then A/B of the splat / lift builds: the product, `h69` (the splat
# gather loop before the straight-line weight broadcast), `pre` (ABI 17 before the scratch fixes),
# zero-fill units x dispatch order (splat_ab.py with the write ceiling), the NCHW tile kernel's
# channel split, kernel micro-bench, and the in-step (graph replay) hot-path kernels of a few builds
# (gpu_prof_ab.sh). A failing test is reported but does not stop the measurements (they use the
# product path the tests check); a failing or timed-out measurement ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4c; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1; trc=$?
tail -8 $OUT/gpu_tests.log; echo "tests rc=$trc"
case $trc in 0|1) ;; *) exit $trc ;; esac  # a crash / timeout: stop using the GPU
timeout -k 10 400 python -u scripts/splat_ab.py --config c3 --libs product,h69,pre,o2,zu4_o2,zu8_o2,zu16_o2,zu8_o1,zu4_o0 \
  > $OUT/splat_ab_c3.log 2>&1 || { tail -30 $OUT/splat_ab_c3.log; exit 1; }
grep -v '^{' $OUT/splat_ab_c3.log | grep -v amdgpu.ids
for cfg in c2 c3; do
  timeout -k 10 300 python -u scripts/splat_ab.py --config $cfg --layout nchw --dtype f32 --libs product,nq2,nq4 \
    --modes dirty,step --ceiling 0 > $OUT/splat_ab_${cfg}_nchw.log 2>&1 || { tail -30 $OUT/splat_ab_${cfg}_nchw.log; exit 1; }
  grep -v '^{' $OUT/splat_ab_${cfg}_nchw.log | grep -v amdgpu.ids
done
timeout -k 10 300 python -u scripts/kbench.py --libs product,h69,pre > $OUT/kbench.log 2>&1 || { tail -20 $OUT/kbench.log; exit 1; }
grep -v '^{' $OUT/kbench.log | grep -v amdgpu.ids
bash scripts/gpu_prof_ab.sh product h69 pre zu8_o2 2>&1 | tee $OUT/prof_ab.txt || exit 1
exit $trc
