# Stage timelines of k_depthnet_lift3 with its feature / weight loads replaced by constants
# (LSS_DN_SKIP=1 weights, 2 features, 3 both): where the stage phase's time goes.
set -o pipefail
mkdir -p gpurun_out/lskip
for v in trace trace_s1 trace_s2 trace_s3 trace_rot trace; do
  timeout -k 10 120 python scripts/stage_trace.py lift3 --lib $v > gpurun_out/lskip/$v.txt 2>&1 || { echo "fail $v"; tail -5 gpurun_out/lskip/$v.txt; exit 1; }
  echo "== $v"; sed -n 2,8p gpurun_out/lskip/$v.txt
done
