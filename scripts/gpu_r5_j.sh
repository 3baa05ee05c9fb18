# Round 5: per-wave splat timeline at HEAD (step mode) after the wait/broadcast/hold-back changes; c5 bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5j; mkdir -p $OUT
timeout -k 10 60 ./scripts/probes/xcc_probe > $OUT/xcc_probe.txt 2>&1 || { cat $OUT/xcc_probe.txt; exit 1; }
cat $OUT/xcc_probe.txt
timeout -k 10 120 python3 -u scripts/splat_trace.py --lib trace --mode step > $OUT/trace_splat_c3_step.txt 2>&1 || { tail -20 $OUT/trace_splat_c3_step.txt; exit 1; }
head -45 $OUT/trace_splat_c3_step.txt
timeout -k 10 600 python -u bench.py --config c5 --cpu-baseline 0 > $OUT/bench_c5.log 2>&1 || { tail -20 $OUT/bench_c5.log; exit 1; }
tail -1 $OUT/bench_c5.log > $OUT/bench_c5.json; cut -c1-300 $OUT/bench_c5.json
