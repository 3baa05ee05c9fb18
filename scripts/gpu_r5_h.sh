# Round 5: splat backward with two tiles per block (both tiles' staging in one round trip): bit-equality,
# standalone times, parity subset, trace, in-step A/B vs one tile per block.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5h; mkdir -p $OUT
timeout -k 10 200 python3 -u scripts/kernel_ab.py --config c3 --libs product,tpb1,tpb2w6 > $OUT/bwd_ab_c3.log 2>&1 || { tail -20 $OUT/bwd_ab_c3.log; exit 1; }
grep "^bwd" $OUT/bwd_ab_c3.log
timeout -k 10 200 python3 -u scripts/kernel_ab.py --config c5 --libs product,tpb1 > $OUT/bwd_ab_c5.log 2>&1 || { tail -20 $OUT/bwd_ab_c5.log; exit 1; }
grep "^bwd" $OUT/bwd_ab_c5.log
timeout -k 10 120 python3 -u scripts/stage_trace.py bwd --lib trace --cold 0 > $OUT/trace_bwd_tpb2.txt 2>&1 || { tail -20 $OUT/trace_bwd_tpb2.txt; exit 1; }
head -9 $OUT/trace_bwd_tpb2.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity2.py tests/test_gpu_captured_step.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash scripts/gpu_prof_ab.sh product tpb1 tpb2w6 product tpb1 2>&1 | tee $OUT/prof_ab.txt || exit 1
