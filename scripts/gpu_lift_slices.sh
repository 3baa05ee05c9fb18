# k_depthnet_lift3 K slices (LSS_DN3_SLICES 1 / 2 / 4): stage timelines, the lift parity tests, then
# the usual iteration (bench line + in-step kernel trace) on the product build.
set -o pipefail
mkdir -p gpurun_out/lsl
for v in trace_sl1 trace trace_sl4 trace_sl1 trace; do
  timeout -k 10 120 python scripts/stage_trace.py lift3 --lib $v > gpurun_out/lsl/$v.txt 2>&1 || { echo "fail $v"; tail -5 gpurun_out/lsl/$v.txt; exit 1; }
  echo "== $v"; sed -n 2,8p gpurun_out/lsl/$v.txt
done
PYTEST_ARGS="tests/test_gpu_lift_nhwc.py tests/test_gpu_captured_step.py" bash scripts/gpu_iter.sh
