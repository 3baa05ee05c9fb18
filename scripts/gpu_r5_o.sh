# Round 5: the trunk's 1x1 conv weight gradients on lss_pw_wrw -- its tests, the captured step, then the
# c3 bench with --hip-pw 1 / 0 under rocprofv3 (whole step by kernel) and plain bench lines.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5o; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_pointwise.py tests/test_gpu_captured_step.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
grep -E "passed|failed" $OUT/tests.log | tail -2
for pw in 1 0; do
  rm -rf /tmp/prof_pw
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_pw -o run -- \
    python3 -u bench.py --steps 20 --warmup 3 --profile-steps 0 --cpu-baseline 0 --pmc-traffic 0 --in-graph-prof 0 --hip-pw $pw \
    > $OUT/bench_pw$pw.log 2>&1 || { tail -20 $OUT/bench_pw$pw.log; exit 1; }
  csv=$(ls /tmp/prof_pw/*/run_kernel_trace.csv /tmp/prof_pw/run_kernel_trace.csv 2>/dev/null | head -1)
  python3 scripts/step_kernels.py "$csv" 5 18 60 > $OUT/step_kernels_pw$pw.txt || exit 1
  echo "== pw=$pw"; tail -1 $OUT/bench_pw$pw.log | cut -c1-200; head -25 $OUT/step_kernels_pw$pw.txt | cut -c1-150
  grep -E "pw_wrw" $OUT/step_kernels_pw$pw.txt | cut -c1-150
  python3 scripts/kernel_calls.py "$csv" pw_wrw > $OUT/pw_calls_pw$pw.txt
  python3 scripts/kernel_calls.py "$csv" "" > $OUT/all_calls_pw$pw.txt
  if [ $pw = 1 ]; then cat $OUT/pw_calls_pw$pw.txt; fi
done
