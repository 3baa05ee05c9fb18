# Round 3: the reference-layout fp32 training line (MIOpen immediate mode: its fp32 shapes are not in the
# in-tree find db), the default bench line, a kernel trace of the default bench for the per-step breakdown.
set -o pipefail
OUT=gpurun_out/r3; mkdir -p $OUT
timeout -k 10 500 python bench.py --config c3 --dtype fp32 --bev-layout nchw --cpu-baseline 0 --miopen-find 0 --in-graph-prof 0 > $OUT/bench_c3_fp32_nchw.json 2> $OUT/bench_c3_fp32_nchw.log; rc=$?
echo "fp32=$rc"; tail -c 400 $OUT/bench_c3_fp32_nchw.json; [ $rc -ne 0 ] && { tail -5 $OUT/bench_c3_fp32_nchw.log; exit $rc; }
timeout -k 10 700 python bench.py > $OUT/bench.json 2> $OUT/bench.log; rc=$?
echo "bench=$rc"; tail -c 1500 $OUT/bench.json; [ $rc -ne 0 ] && tail -5 $OUT/bench.log
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/r3trace -o run -- python3 -u bench.py --steps 10 --warmup 3 --profile-steps 0 --cpu-baseline 0 --pmc-traffic 0 --in-graph-prof 0 > $OUT/trace_bench.json 2> $OUT/trace_bench.log; rc=$?
echo "trace=$rc"; [ $rc -ne 0 ] && exit $rc
csv=$(find /tmp/r3trace -name '*kernel_trace.csv' | head -1)
python3 scripts/step_kernels.py $csv 5 14 70 > $OUT/step_kernels_c3.txt; python3 scripts/hot_steps.py $csv 5 14 > $OUT/hot_steps_c3.txt; head -40 $OUT/step_kernels_c3.txt
exit 0
