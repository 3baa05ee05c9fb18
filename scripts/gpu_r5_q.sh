# Round 5: trunk 1x1 conv forward / backward-data on lss_pw_conv (--hip-pw 2) vs MIOpen (--hip-pw 1), plus
# the hybrid depthwise dispatch: tests, then the c3 step under rocprofv3 for each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5q; mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pointwise.py tests/test_gpu_convs.py tests/test_gpu_captured_step.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for pw in 2 1; do
  rm -rf /tmp/prof_q
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_q -o run -- \
    python3 -u bench.py --steps 20 --warmup 3 --profile-steps 0 --cpu-baseline 0 --pmc-traffic 0 --in-graph-prof 0 --hip-pw $pw \
    > $OUT/bench_pw$pw.log 2>&1 || { tail -20 $OUT/bench_pw$pw.log; exit 1; }
  csv=$(ls /tmp/prof_q/*/run_kernel_trace.csv /tmp/prof_q/run_kernel_trace.csv 2>/dev/null | head -1)
  python3 scripts/step_kernels.py "$csv" 5 18 60 > $OUT/step_kernels_pw$pw.txt || exit 1
  python3 scripts/kernel_calls.py "$csv" "" > $OUT/all_calls_pw$pw.txt || exit 1
  echo "== pw=$pw"; head -1 $OUT/step_kernels_pw$pw.txt; grep -E "pw_gemm|Cijk|k_dw" $OUT/step_kernels_pw$pw.txt | cut -c1-110
done
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pmc-traffic 0 --in-graph-prof 0 > $OUT/bench_plain.log 2>&1 || { tail -20 $OUT/bench_plain.log; exit 1; }
tail -1 $OUT/bench_plain.log | cut -c1-300
