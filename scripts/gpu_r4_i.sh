# Round 4: the fused lift's new epilogue (GPU suite for parity), its stage trace, the weight-copies
# experiment (kbench + trace), and in-step times.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4i; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1; trc=$?
tail -4 $OUT/gpu_tests.log; echo "tests rc=$trc"
[ $trc -ne 0 ] && exit $trc
timeout -k 10 300 python -u scripts/kbench.py --libs product,wc8,wc2 --only depthnet_lift > $OUT/kbench.log 2>&1 || { tail -20 $OUT/kbench.log; exit 1; }
grep -v '^{' $OUT/kbench.log | grep -v amdgpu.ids
for lib in trace trace_wc8; do
  timeout -k 10 200 python -u scripts/stage_trace.py lift3 --config c3 --lib $lib > $OUT/trace_lift3_$lib.txt 2>&1 || { tail -20 $OUT/trace_lift3_$lib.txt; exit 1; }
  head -8 $OUT/trace_lift3_$lib.txt
done
bash scripts/gpu_prof_ab.sh product 2>&1 | tee $OUT/prof_ab.txt || exit 1
