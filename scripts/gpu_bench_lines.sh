# Bench lines of round 2: config 3 (default), config 2 (fp32 NCHW forward), config 5 per-GPU shard;
# then a rocprofv3 kernel trace (--stats) of the default step.  usage: bash scripts/gpu_bench_lines.sh [c3 c2 c5 prof]
set -o pipefail
OUT=gpurun_out/r2; mkdir -p $OUT
for s in ${*:-c3 c2 c5 prof}; do
  case $s in
    c3) timeout -k 10 600 python3 -u bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.log; rc=$? ;;
    c2) timeout -k 10 400 python3 -u bench.py --config c2 --cpu-baseline 0 > $OUT/bench_c2.json 2> $OUT/bench_c2.log; rc=$? ;;
    c5) timeout -k 10 500 python3 -u bench.py --config c5 --cpu-baseline 0 > $OUT/bench_c5.json 2> $OUT/bench_c5.log; rc=$? ;;
    prof) cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
          timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python3 -u bench.py --steps 10 \
            --cpu-baseline 0 --pmc-traffic 0 > $OUT/prof_c3.log 2>&1; rc=$? ;;
  esac
  echo "$s rc=$rc"; [ -f $OUT/bench_$s.json ] && cat $OUT/bench_$s.json | cut -c1-600
  [ $rc -ne 0 ] && { tail -20 $OUT/bench_$s.log $OUT/prof_c3.log 2>/dev/null; exit $rc; }
done
exit 0
