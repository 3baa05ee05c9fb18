# Round 5: persistent pipelined chunk waves -- splat-only A/B (bit-equal + cache states), then in-step.
# (the LSS_SPLAT_K switch this script measured was removed after it; results in profiles/r05)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5a; mkdir -p $OUT
timeout -k 10 300 python3 -u scripts/splat_ab.py --config c3 --libs product,k3o5,k3o5z2,k2o5,k4o5,k3o5zf,k6o5 --modes step,read --ceiling 0 > $OUT/splat_ab_c3.log 2>&1 || { tail -30 $OUT/splat_ab_c3.log; exit 1; }
grep -v '^{' $OUT/splat_ab_c3.log | cut -c1-260
bash scripts/gpu_prof_ab.sh product k3o5 k3o5z2 k4o5 k3o5zf product 2>&1 | tee $OUT/prof_ab.txt || exit 1
