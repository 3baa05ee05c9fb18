# Round 5 evidence at HEAD: GPU suite, smoke, the default
# bench line (c3, CPU baseline, PMC traffic, in-graph splat + backward), and a rocprofv3 --kernel-trace --stats
# run of the same bench (per-kernel summary, hot path per step, whole step by kernel).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${R5OUT:-r5final_b}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1; trc=$?
tail -3 $OUT/gpu_tests.log; echo "tests rc=$trc"
[ $trc -ne 0 ] && exit $trc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u bench.py > $OUT/bench_c3.log 2>&1 || { tail -20 $OUT/bench_c3.log; exit 1; }
tail -1 $OUT/bench_c3.log > $OUT/bench_c3.json; cut -c1-400 $OUT/bench_c3.json
rm -rf /tmp/prof_c3
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_c3 -o run -- \
  python3 -u bench.py --steps 20 --warmup 3 --profile-steps 0 --cpu-baseline 0 --pmc-traffic 0 --in-graph-prof 0 \
  > $OUT/bench_c3_under_rocprof.log 2>&1 || { tail -20 $OUT/bench_c3_under_rocprof.log; exit 1; }
csv=$(ls /tmp/prof_c3/*/run_kernel_trace.csv /tmp/prof_c3/run_kernel_trace.csv 2>/dev/null | head -1)
st=$(ls /tmp/prof_c3/*/run_kernel_stats.csv /tmp/prof_c3/run_kernel_stats.csv 2>/dev/null | head -1)
cp "$st" $OUT/bench_c3_kernel_stats.csv
python3 scripts/hot_steps.py "$csv" 5 23 > $OUT/hot_steps_c3.txt && python3 scripts/step_kernels.py "$csv" 5 23 40 > $OUT/step_kernels_c3.txt \
  && python3 scripts/steady_summary.py "$csv" > $OUT/bench_c3_steady_summary.json
tail -12 $OUT/hot_steps_c3.txt
