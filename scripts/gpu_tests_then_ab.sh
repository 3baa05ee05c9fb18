set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_lift_nhwc.py tests/test_gpu_captured_step.py > gpurun_out/x_tests.log 2>&1; rc=$?; tail -2 gpurun_out/x_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_prof_ab.sh product product
