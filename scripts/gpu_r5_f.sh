# Round 5: DPP / permlane primitive probe; splat backward reductions on them (bit-equal to the butterfly
# build?) across tile shapes; lift with 32-row MFMA waves; parity subset; in-step A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5f; mkdir -p $OUT
timeout -k 10 60 ./scripts/probes/dpp_check > $OUT/dpp_check.txt 2>&1 || { cat $OUT/dpp_check.txt; exit 1; }
cat $OUT/dpp_check.txt
timeout -k 10 200 python3 -u scripts/kernel_ab.py --config c3 --libs product,dpp0,bwd81,bwd81dpp0 > $OUT/bwd_ab_c3.log 2>&1 || { tail -20 $OUT/bwd_ab_c3.log; exit 1; }
grep "^bwd" $OUT/bwd_ab_c3.log
timeout -k 10 200 python3 -u scripts/kernel_ab.py --config c5 --libs product,dpp0 > $OUT/bwd_ab_c5.log 2>&1 || { tail -20 $OUT/bwd_ab_c5.log; exit 1; }
grep "^bwd" $OUT/bwd_ab_c5.log
timeout -k 10 200 python3 -u scripts/kernel_ab.py --kernel lift --config c3 --libs product,dn3rt2 > $OUT/lift_ab_c3.log 2>&1 || { tail -20 $OUT/lift_ab_c3.log; exit 1; }
grep "^lift" $OUT/lift_ab_c3.log
timeout -k 10 300 python3 -u scripts/splat_ab.py --config c3 --libs product,wa0 --modes step,read --ceiling 0 > $OUT/splat_ab_c3.log 2>&1 || { tail -30 $OUT/splat_ab_c3.log; exit 1; }
grep -v '^{' $OUT/splat_ab_c3.log | cut -c1-260
timeout -k 10 300 python3 -u scripts/splat_ab.py --config c5 --libs product,wa0 --modes step --ceiling 0 > $OUT/splat_ab_c5.log 2>&1 || { tail -30 $OUT/splat_ab_c5.log; exit 1; }
grep -v '^{' $OUT/splat_ab_c5.log | cut -c1-260
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity2.py tests/test_gpu_captured_step.py tests/test_gpu_lift_nhwc.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash scripts/gpu_prof_ab.sh product wa0 bwd81 dpp0 dn3rt2 product 2>&1 | tee $OUT/prof_ab.txt || exit 1
