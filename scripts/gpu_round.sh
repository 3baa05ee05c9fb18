# Round measurement: GPU parity tests, default bench (+CPU baseline), kernel trace, splat PMC passes.
set -o pipefail
OUT=gpurun_out/round; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
echo "tests=$rc"; tail -3 $OUT/gpu_tests.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1; rc=$?; echo "bench=$rc"; tail -1 $OUT/bench.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 > $OUT/trace_bench.log 2>&1; rc=$?
echo "trace=$rc"; tail -1 $OUT/trace_bench.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-include-regex k_splat_fwd --output-format csv -d $OUT/pmc_$c -o run -- \
      python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 --graph 0 > $OUT/pmc_$c.log 2>&1; rc=$?
  echo "pmc $c=$rc"; [ $rc -ne 0 ] && { tail -3 $OUT/pmc_$c.log; exit $rc; }
done
exit 0
