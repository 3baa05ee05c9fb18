# Round 5: GPU suite + smoke at HEAD, default bench line, and the caller's fp32 path with both BEV layouts.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5b; mkdir -p $OUT
bash scripts/gpu_tests.sh || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
Q="--pmc-traffic 0 --cpu-baseline 0"
for v in "c3 fp32 nchw train" "c3 fp32 nhwc train" "c2 fp32 nchw fwd" "c2 fp32 nhwc fwd"; do
  set -- $v
  timeout -k 10 300 python -u bench.py --config $1 --dtype $2 --bev-layout $3 --mode $4 $Q > $OUT/bench_$1_$2_$3_$4.log 2>&1 || { tail -20 $OUT/bench_$1_$2_$3_$4.log; exit 1; }
  tail -1 $OUT/bench_$1_$2_$3_$4.log | cut -c1-400
done
timeout -k 10 600 python -u bench.py > $OUT/bench_c3.log 2>&1 || { tail -20 $OUT/bench_c3.log; exit 1; }
tail -1 $OUT/bench_c3.log > $OUT/bench_c3.json; cut -c1-300 $OUT/bench_c3.json
