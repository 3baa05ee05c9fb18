# Round 3 (second session): the whole GPU suite unserialized (one process), then the default bench
# line and a kernel trace of a short bench run (per-step breakdown). Logs under gpurun_out/r3b.
set -o pipefail
OUT=${OUT:-gpurun_out/r3b}; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rs -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $OUT/gpu_tests.log 2>&1; rc=$?
echo "tests=$rc"; tail -4 $OUT/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
OUT=$OUT bash scripts/gpu_iter.sh
