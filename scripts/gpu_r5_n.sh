# Round 5: geometry blocks as column strips (LSS_GEO_STRIPS, product) vs 256 consecutive points (geo0),
# and the plan kernels between the trunk and the dropout (--plan-at dropout) vs before the lift; c3 + c5.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5n; mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_parity2.py tests/test_gpu_robustness.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for cfg in c3 c5; do
  echo "## $cfg strips (product) vs geo0"
  BENCH_ARGS="--config $cfg" bash scripts/gpu_prof_ab.sh product geo0 2>&1 | tee -a $OUT/prof_ab_geo.txt || exit 1
  echo "## $cfg plan-at dropout"
  BENCH_ARGS="--config $cfg --plan-at dropout" bash scripts/gpu_prof_ab.sh product 2>&1 | tee -a $OUT/prof_ab_plan_at.txt || exit 1
done
