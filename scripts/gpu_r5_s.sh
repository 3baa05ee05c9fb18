# Round 5: every kernel call of one c3 training step in launch order (rocprofv3 kernel trace of bench.py),
# for the per-layer view of the batch-norm and conv kernels.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5s; mkdir -p $OUT
rm -rf /tmp/prof_s
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_s -o run -- \
  python3 -u bench.py --steps 10 --warmup 3 --profile-steps 0 --cpu-baseline 0 --pmc-traffic 0 --in-graph-prof 0 \
  > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
csv=$(ls /tmp/prof_s/*/run_kernel_trace.csv /tmp/prof_s/run_kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/kernel_calls.py "$csv" "" 8 > $OUT/all_calls_c3.txt || exit 1
tail -1 $OUT/all_calls_c3.txt
