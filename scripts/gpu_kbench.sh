set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -rf -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "tests=$rc"; tail -25 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/kbench.py > gpurun_out/kbench.log 2>&1; rc=$?; echo "kbench=$rc"; cat gpurun_out/kbench.log | grep -v Warn
exit $rc
