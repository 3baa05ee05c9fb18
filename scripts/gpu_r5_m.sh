# Round 5: splat forward -- a finished row parked in LDS across a group's second batch of gathers
# (HOLDROW, at 6 waves/SIMD: it needs the registers) vs 6 waves/SIMD alone vs the product; c3 + c5.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5m; mkdir -p $OUT
timeout -k 10 300 python3 -u scripts/splat_ab.py --config c3 --libs product,hr1o6,o6,product,hr1o6,o6 --modes step --ceiling 0 > $OUT/splat_ab_c3.log 2>&1 || { tail -30 $OUT/splat_ab_c3.log; exit 1; }
grep -v '^{' $OUT/splat_ab_c3.log | cut -c1-200
timeout -k 10 300 python3 -u scripts/splat_ab.py --config c5 --libs product,hr1o6,o6 --modes step --ceiling 0 > $OUT/splat_ab_c5.log 2>&1 || { tail -30 $OUT/splat_ab_c5.log; exit 1; }
grep -v '^{' $OUT/splat_ab_c5.log | cut -c1-200
bash scripts/gpu_prof_ab.sh product hr1o6 o6 product hr1o6 2>&1 | tee $OUT/prof_ab.txt || exit 1
