# Bench A/B: one JSON summary line per flag set (args: quoted flag sets). MIOpen db in-tree.
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  timeout -k 10 420 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 $v > gpurun_out/ab.log 2>&1; rc=$?
  if [ $rc -ne 0 ]; then echo "== $v FAILED rc=$rc"; tail -5 gpurun_out/ab.log; exit $rc; fi
  tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('== $v:', d['value'], 'fps', d['ms_per_step'], 'ms/step; splat', d['roofline']['avg_launch_us'], 'us frac', d['roofline']['frac'])"
done
exit 0
