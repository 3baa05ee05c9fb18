# Round 5: the one-round backward tile (4 waves x 3 pixels) -- parity subset, in-step A/B vs the 8x1 tile
# and 4x4; then the caller's fp32 path with both BEV layouts (MIOpen find off: fp32 find runs for minutes).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5c; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity2.py tests/test_gpu_captured_step.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash scripts/gpu_prof_ab.sh product bwd81 bwd44 product 2>&1 | tee $OUT/prof_ab.txt || exit 1
Q="--pmc-traffic 0 --cpu-baseline 0 --miopen-find 0"
for v in "c3 fp32 nchw train" "c3 fp32 nhwc train" "c2 fp32 nchw fwd" "c2 fp32 nhwc fwd"; do
  set -- $v
  timeout -k 10 300 python -u bench.py --config $1 --dtype $2 --bev-layout $3 --mode $4 $Q > $OUT/bench_$1_$2_$3_$4.log 2>&1 || { tail -20 $OUT/bench_$1_$2_$3_$4.log; exit 1; }
  tail -1 $OUT/bench_$1_$2_$3_$4.log | cut -c1-600
done
