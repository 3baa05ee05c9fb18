# GPU parity suite, unserialized, one process; log under gpurun_out/tests.
set -o pipefail
OUT=gpurun_out/tests; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs -p no:cacheprovider --timeout 300 --timeout-method thread \
    ${PYTEST_ARGS:-} > $OUT/gpu_tests.log 2>&1; rc=$?
echo "tests=$rc"; tail -15 $OUT/gpu_tests.log
exit $rc
