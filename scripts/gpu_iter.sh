# One development iteration on the GPU box: selected GPU tests (PYTEST_ARGS, default: none), a short
# bench line (BENCH_ARGS), then a kernel trace of a short bench run with the per-step hot-path and
# whole-step breakdowns. Logs under gpurun_out/iter (OUT overrides).
set -o pipefail
OUT=${OUT:-gpurun_out/iter}; mkdir -p $OUT
if [ -n "${PYTEST_ARGS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -v -rs -p no:cacheprovider --timeout 120 --timeout-method thread \
      $PYTEST_ARGS > $OUT/tests.log 2>&1; rc=$?
  echo "tests=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/tests.log | tail -25; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.log; rc=$?
echo "bench=$rc"; tail -c 1200 $OUT/bench.json; [ $rc -ne 0 ] && { tail -8 $OUT/bench.log; exit $rc; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/itrace
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/itrace -o run -- python3 -u bench.py --steps 10 \
    --warmup 3 --profile-steps 0 --cpu-baseline 0 --pmc-traffic 0 --in-graph-prof 0 ${BENCH_ARGS:-} \
    > $OUT/trace_bench.json 2> $OUT/trace_bench.log; rc=$?
echo "trace=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/trace_bench.log; exit $rc; }
csv=$(find /tmp/itrace -name '*kernel_trace.csv' | head -1)
python3 scripts/hot_steps.py $csv 5 12 > $OUT/hot_steps.txt; cat $OUT/hot_steps.txt
python3 scripts/step_kernels.py $csv 5 12 80 > $OUT/step_kernels.txt; head -45 $OUT/step_kernels.txt
exit 0
