# Round 5: splat forward weight broadcast on DPP (vs ds_bpermute); backward DPP bit-equality; backward
# trace with the DPP reductions; MIOpen solver-switch step A/B (helper kernels).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5g; mkdir -p $OUT
timeout -k 10 200 python3 -u scripts/kernel_ab.py --config c3 --libs product,dpp0 > $OUT/bwd_ab_c3.log 2>&1 || { tail -20 $OUT/bwd_ab_c3.log; exit 1; }
grep "^bwd" $OUT/bwd_ab_c3.log
timeout -k 10 300 python3 -u scripts/splat_ab.py --config c3 --libs product,dppw0,product,dppw0 --modes step,read --ceiling 0 > $OUT/splat_ab_c3.log 2>&1 || { tail -30 $OUT/splat_ab_c3.log; exit 1; }
grep -v '^{' $OUT/splat_ab_c3.log | cut -c1-260
timeout -k 10 120 python3 -u scripts/stage_trace.py bwd --lib trace --cold 0 > $OUT/trace_bwd_dpp.txt 2>&1 || { tail -20 $OUT/trace_bwd_dpp.txt; exit 1; }
head -9 $OUT/trace_bwd_dpp.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity2.py tests/test_gpu_captured_step.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash scripts/gpu_prof_ab.sh product dppw0 product dppw0 2>&1 | tee $OUT/prof_ab.txt || exit 1
bash scripts/gpu_miopen_ab.sh 2>&1 | tee $OUT/miopen_ab.txt || exit 1
