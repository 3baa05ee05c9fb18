set -o pipefail
mkdir -p gpurun_out/lt
for v in "lift trace" "lift3 trace" "lift3 trace_p48"; do
  set -- $v
  timeout -k 10 120 python scripts/stage_trace.py $1 --lib $2 > gpurun_out/lt/$1_$2.txt 2>&1 || { echo "fail $v"; tail -5 gpurun_out/lt/$1_$2.txt; exit 1; }
  echo "== $v"; sed -n 2,8p gpurun_out/lt/$1_$2.txt
done
LSS_CAPTURE_DIAG=1 timeout -k 10 600 python -u -m pytest -x -s -q -p no:cacheprovider --timeout 500 --timeout-method thread tests/test_gpu_captured_step.py > gpurun_out/diag.log 2>&1; grep -E "rig [01]|passed|failed" gpurun_out/diag.log
OUT=gpurun_out/iter bash scripts/gpu_iter.sh
