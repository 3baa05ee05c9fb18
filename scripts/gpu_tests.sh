# GPU parity suite, unserialized, one process; log under gpurun_out/tests.
set -o pipefail
OUT=gpurun_out/tests; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rs -p no:cacheprovider --timeout 300 --timeout-method thread \
    ${PYTEST_ARGS:-} > $OUT/gpu_tests.log 2>&1; rc=$?
echo "tests=$rc"; grep -E "passed|failed|error" $OUT/gpu_tests.log | tail -15
exit $rc
