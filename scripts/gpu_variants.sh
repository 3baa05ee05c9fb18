# Bench variants back to back (one JSON line each), then a kernel-trace profile of one of them.
set -o pipefail
mkdir -p gpurun_out/prof
for v in "$@"; do
  echo "== variant: $v"
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 $v > gpurun_out/var.log 2>&1; rc=$?
  tail -1 gpurun_out/var.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])" || tail -5 gpurun_out/var.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
