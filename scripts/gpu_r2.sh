# Round-2 iteration: GPU tests, kernel micro-bench (+variants), default bench line.
# usage: bash scripts/gpu_r2.sh [tests|kbench|bench]...   (default: all three)
set -o pipefail
OUT=gpurun_out/r2; mkdir -p $OUT
steps="${*:-tests kbench bench}"
for s in $steps; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
      echo "tests=$rc"; tail -15 $OUT/gpu_tests.log; [ $rc -ne 0 ] && exit $rc ;;
    kbench)
      timeout -k 10 400 python -u scripts/kbench.py > $OUT/kbench.log 2>&1; rc=$?
      echo "kbench=$rc"; grep -v Warn $OUT/kbench.log | tail -100; [ $rc -ne 0 ] && exit $rc ;;
    bench)
      timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1; rc=$?
      echo "bench=$rc"; grep "^\[" $OUT/bench.log | tail -8; tail -1 $OUT/bench.log; [ $rc -ne 0 ] && exit $rc ;;
  esac
done
exit 0
