# Round 5: channels-last BN + ReLU backward with the output recomputed from x (product) vs kept and re-read,
# same box: kernel trace of one c3 step each (batch-norm calls), then the plain bench each, twice.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5u; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_loss.py \
  > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for m in recompute keep; do
  rm -rf /tmp/prof_u
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_u -o run -- \
    python3 -u bench.py --steps 10 --warmup 3 --profile-steps 0 --cpu-baseline 0 --pmc-traffic 0 --in-graph-prof 0 --bn-relu-y $m \
    > $OUT/bench_prof_$m.log 2>&1 || { tail -20 $OUT/bench_prof_$m.log; exit 1; }
  csv=$(ls /tmp/prof_u/*/run_kernel_trace.csv /tmp/prof_u/run_kernel_trace.csv 2>/dev/null | head -1)
  python3 scripts/kernel_calls.py "$csv" "" 8 > $OUT/all_calls_$m.txt && python3 scripts/step_kernels.py "$csv" 3 12 60 > $OUT/step_kernels_$m.txt || exit 1
  echo "== $m"; head -1 $OUT/step_kernels_$m.txt; grep -E "k_bn_bwd_(stats|apply)_nhwc" $OUT/all_calls_$m.txt | head -8 | cut -c1-60
done
bash scripts/gpu_ab_lib.sh "product|" "product|--bn-relu-y keep" "product|" "product|--bn-relu-y keep" 2>&1 | tee $OUT/ab.txt
