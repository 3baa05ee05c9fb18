set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "tests=$rc"; tail -25 gpurun_out/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench=$rc"; tail -5 gpurun_out/bench.log
exit $rc
