# Round 5: splat backward reductions on DPP / permlane (no ds_bpermute butterflies): bit-equality and
# standalone times across tile shapes, parity subset, per-wave traces, in-step A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5e; mkdir -p $OUT
timeout -k 10 200 python3 -u scripts/bwd_ab.py --config c3 --libs product,dpp0,bwd81,bwd81dpp0 > $OUT/bwd_ab_c3.log 2>&1 || { tail -20 $OUT/bwd_ab_c3.log; exit 1; }
grep "^bwd" $OUT/bwd_ab_c3.log
timeout -k 10 200 python3 -u scripts/bwd_ab.py --config c5 --libs product,dpp0 > $OUT/bwd_ab_c5.log 2>&1 || { tail -20 $OUT/bwd_ab_c5.log; exit 1; }
grep "^bwd" $OUT/bwd_ab_c5.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity2.py tests/test_gpu_captured_step.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in trace trace81; do
  timeout -k 10 120 python3 -u scripts/stage_trace.py bwd --lib $v --cold 0 > $OUT/trace_bwd_$v.txt 2>&1 || { tail -20 $OUT/trace_bwd_$v.txt; exit 1; }
  head -9 $OUT/trace_bwd_$v.txt
done
bash scripts/gpu_prof_ab.sh product bwd81 dpp0 product 2>&1 | tee $OUT/prof_ab.txt || exit 1
