# Round-3 measurement: default bench line (PMC + in-graph child trace + CPU baseline), then a kernel trace
# of a short bench run for the per-step breakdown. Logs under gpurun_out/r3.
set -o pipefail
OUT=gpurun_out/r3; mkdir -p $OUT
timeout -k 10 700 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.log; rc=$?
echo "bench=$rc"; tail -c 600 $OUT/bench.json; [ $rc -ne 0 ] && { tail -5 $OUT/bench.log; exit $rc; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 --pmc-traffic 0 --in-graph-prof 0 ${BENCH_ARGS:-} \
    > $OUT/trace_bench.json 2> $OUT/trace_bench.log; rc=$?
echo "trace=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/trace_bench.log; exit $rc; }
python scripts/step_kernels.py $(ls $OUT/trace/*/run_kernel_trace.csv 2>/dev/null || find $OUT/trace -name "*kernel_trace.csv" | head -1) 6 14 60 > $OUT/step_kernels.txt; head -70 $OUT/step_kernels.txt
exit 0
