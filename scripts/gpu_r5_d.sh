# Round 5: per-wave traces of the splat backward (4x3 vs 8x1 tiles) and the fused lift (7 vs 8 waves);
# in-step A/B of the lift (7 waves + unrolled softmax vs 8 waves / loop softmax); caller's fp32 path.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5d; mkdir -p $OUT
for v in "bwd trace" "bwd trace81" "lift3 trace" "lift3 trace_w8"; do
  set -- $v
  for cold in 0 1; do
    timeout -k 10 120 python3 -u scripts/stage_trace.py $1 --lib $2 --cold $cold > $OUT/trace_$1_$2_cold$cold.txt 2>&1 || { tail -20 $OUT/trace_$1_$2_cold$cold.txt; exit 1; }
    head -9 $OUT/trace_$1_$2_cold$cold.txt
  done
done
bash scripts/gpu_prof_ab.sh product dn8 smu0 product 2>&1 | tee $OUT/prof_ab.txt || exit 1
Q="--pmc-traffic 0 --cpu-baseline 0 --miopen-find 0"
for v in "c3 fp32 nchw train" "c3 fp32 nhwc train" "c2 fp32 nchw fwd" "c2 fp32 nhwc fwd"; do
  set -- $v
  timeout -k 10 400 python -u bench.py --config $1 --dtype $2 --bev-layout $3 --mode $4 $Q > $OUT/bench_$1_$2_$3_$4.log 2>&1 || { tail -20 $OUT/bench_$1_$2_$3_$4.log; exit 1; }
  tail -1 $OUT/bench_$1_$2_$3_$4.log | cut -c1-700
done
