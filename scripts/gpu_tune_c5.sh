# Config-5 per-GPU shard bench line with a fresh MIOpen find for its shapes; the find database is
# written under gpurun_out/miopen/db (seeded with tuning/miopen/db) to be copied back into tuning/.
set -o pipefail
OUT=gpurun_out/r2; mkdir -p $OUT gpurun_out/miopen/db
cp tuning/miopen/db/* gpurun_out/miopen/db/
( while sleep 50; do echo "[heartbeat] $(date +%T)"; done ) & HB=$!
MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen/db MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache_c5 \
  timeout -k 10 1000 python3 -u bench.py --config c5 --cpu-baseline 0 > $OUT/bench_c5.json 2> $OUT/bench_c5.log
rc=$?
kill $HB
echo "c5 rc=$rc"; cat $OUT/bench_c5.json | cut -c1-400; tail -3 $OUT/bench_c5.log
exit $rc
