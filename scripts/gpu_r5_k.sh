# Round 5: CamEncode.dropout on lss_dropout (XCD-contiguous write + weight warm-up) and the plan moved in
# front of the trunk: dropout tests, lift times after each producer, captured step + parity, in-step A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5k; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropout.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests_dropout.log 2>&1 || { tail -30 $OUT/tests_dropout.log; exit 1; }
tail -2 $OUT/tests_dropout.log
for pr in none dropout torch; do
  timeout -k 10 200 python3 -u scripts/kernel_ab.py --kernel lift --config c3 --libs product --producer $pr > $OUT/lift_ab_$pr.log 2>&1 || { tail -20 $OUT/lift_ab_$pr.log; exit 1; }
  echo "producer=$pr $(grep '^lift' $OUT/lift_ab_$pr.log)"
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_captured_step.py tests/test_gpu_parity.py tests/test_gpu_parity2.py tests/test_gpu_lift_nhwc.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash scripts/gpu_prof_ab.sh product product 2>&1 | tee $OUT/prof_ab_hipdrop.txt || exit 1
BENCH_ARGS="--hip-dropout 0" bash scripts/gpu_prof_ab.sh product product 2>&1 | tee $OUT/prof_ab_torchdrop.txt || exit 1
