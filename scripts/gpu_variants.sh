# Bench variants back to back (one JSON line each). MIOpen's user find-db and kernel cache go to
# gpurun_out/miopen so they can be inspected / reused.
set -o pipefail
# MIOpen uses the in-tree find-db (tuning/miopen) unless CAPTURE_MIOPEN=1 (fresh db under gpurun_out).
mkdir -p gpurun_out/prof
if [ "${CAPTURE_MIOPEN:-0}" = 1 ]; then
  mkdir -p gpurun_out/miopen/db gpurun_out/miopen/cache
  export MIOPEN_USER_DB_PATH="$PWD/gpurun_out/miopen/db" MIOPEN_CUSTOM_CACHE_DIR="$PWD/gpurun_out/miopen/cache"
fi
for v in "$@"; do
  echo "== variant: $v"
  t0=$(date +%s)
  timeout -k 10 420 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 $v > gpurun_out/var.log 2>&1; rc=$?
  grep -h "first step\|warmup" gpurun_out/var.log | tr '\n' ' '; echo "(wall $(( $(date +%s) - t0 )) s)"
  if [ $rc -ne 0 ]; then tail -3 gpurun_out/var.log; exit $rc; fi
  tail -1 gpurun_out/var.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done
[ "${CAPTURE_MIOPEN:-0}" = 1 ] && du -sh gpurun_out/miopen/db gpurun_out/miopen/cache
exit 0
