# Round 5: after the persistent-chunk code removal -- captured step + parity subset; splat zero hold-back
# (s_sleep heuristic) still needed now that the gathers retire before the row stores?
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5i; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_captured_step.py tests/test_gpu_parity.py tests/test_gpu_parity2.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python3 -u scripts/splat_ab.py --config c3 --libs product,hold0,product,hold0 --modes step,read --ceiling 0 > $OUT/splat_ab_c3.log 2>&1 || { tail -30 $OUT/splat_ab_c3.log; exit 1; }
grep -v '^{' $OUT/splat_ab_c3.log | cut -c1-260
bash scripts/gpu_prof_ab.sh product hold0 product hold0 2>&1 | tee $OUT/prof_ab.txt || exit 1
