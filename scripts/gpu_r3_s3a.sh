# Round 3, third session, part 1: the whole GPU suite unserialized (one process), then the default
# bench line and the rocprofv3 --kernel-trace --stats run (gpu_r3_lines.sh c3 prof). gpurun_out/r3s3.
set -o pipefail
OUT=gpurun_out/r3s3; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -rs -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $OUT/gpu_tests.log 2>&1; rc=$?
echo "tests=$rc"; tail -4 $OUT/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
OUT=$OUT bash scripts/gpu_r3_lines.sh c3 prof
