# Round 5: c5 splat regression hunt -- kernel variants standalone at c5, and the step order (plan before /
# after the trunk) x dropout (lss_dropout / torch) in-step at c3 and c5.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5l; mkdir -p $OUT
timeout -k 10 300 python3 -u scripts/splat_ab.py --config c5 --libs product,wa0,dppw0 --modes step --ceiling 0 > $OUT/splat_ab_c5.log 2>&1 || { tail -30 $OUT/splat_ab_c5.log; exit 1; }
grep -v '^{' $OUT/splat_ab_c5.log | cut -c1-200
for cfg in c3 c5; do
  for v in "lift 1" "trunk 1" "lift 0"; do
    set -- $v
    echo "## $cfg plan-at=$1 hip-dropout=$2"
    BENCH_ARGS="--config $cfg --plan-at $1 --hip-dropout $2" bash scripts/gpu_prof_ab.sh product 2>&1 | tee -a $OUT/prof_ab_order.txt || exit 1
  done
done
