# Round 3 (second session) measurement at HEAD, logs under gpurun_out/r3s2: the default bench line
# (c3 training step: PMC traffic passes, in-graph splat timing, CPU baseline), a rocprofv3
# --kernel-trace --stats run of the same bench (per-kernel summary + per-step breakdown), the c5 and
# c2 lines and the reference-layout fp32 NCHW training line.  usage: bash scripts/gpu_r3_lines.sh [steps...]
set -o pipefail
OUT=${OUT:-gpurun_out/r3s2}; mkdir -p $OUT
for s in ${*:-c3 prof c5 c2 fp32}; do
  case $s in
    c3) timeout -k 10 600 python3 -u bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.log; rc=$? ;;
    prof) cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && rm -rf /tmp/r3s2prof && \
          timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r3s2prof -o run -- \
            python3 -u bench.py --steps 10 --warmup 3 --profile-steps 0 --cpu-baseline 0 --pmc-traffic 0 \
            --in-graph-prof 0 > $OUT/prof_c3.json 2> $OUT/prof_c3.log; rc=$?
          if [ $rc -eq 0 ]; then
            cp $(find /tmp/r3s2prof -name '*kernel_stats.csv' | head -1) $OUT/bench_c3_kernel_stats.csv
            csv=$(find /tmp/r3s2prof -name '*kernel_trace.csv' | head -1)
            python3 scripts/hot_steps.py $csv 5 12 > $OUT/hot_steps_c3.txt
            python3 scripts/step_kernels.py $csv 5 12 80 > $OUT/step_kernels_c3.txt
          fi ;;
    c5) timeout -k 10 500 python3 -u bench.py --config c5 --cpu-baseline 0 > $OUT/bench_c5.json 2> $OUT/bench_c5.log; rc=$? ;;
    c2) timeout -k 10 400 python3 -u bench.py --config c2 --cpu-baseline 0 > $OUT/bench_c2.json 2> $OUT/bench_c2.log; rc=$? ;;
    fp32) timeout -k 10 500 python3 -u bench.py --dtype fp32 --bev-layout nchw --cpu-baseline 0 --miopen-find 0 \
            --in-graph-prof 0 > $OUT/bench_c3_fp32_nchw_train.json 2> $OUT/bench_c3_fp32_nchw_train.log; rc=$? ;;
  esac
  echo "$s rc=$rc"; [ -f $OUT/bench_$s.json ] && cut -c1-300 $OUT/bench_$s.json
  [ $rc -ne 0 ] && { tail -20 $OUT/*$s*.log 2>/dev/null; exit $rc; }
done
exit 0
