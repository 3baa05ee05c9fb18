# Round 5: fp32-row splat forward with one gather batch per typical lane group (LSS_SPLAT_KU32 = 12 / 16
# entries in flight, occupancy 4-6) vs the product (8): kernel-stamped A/B at c2 and c3 (fp32 BEV).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5r; mkdir -p $OUT
for c in c2 c3; do
  timeout -k 10 240 python3 -u scripts/splat_ab.py --config $c --dtype f32 --libs product,ku16o4,ku16o5,ku12o6,product \
    --modes read,step --ceiling 0 > $OUT/splat_ab_${c}_f32.log 2>&1 || { tail -20 $OUT/splat_ab_${c}_f32.log; exit 1; }
  cat $OUT/splat_ab_${c}_f32.log
done
