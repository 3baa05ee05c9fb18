# Bench A/B across library builds: each arg is "<lib>|<bench flags>", lib = product or a
# variants/<name>.so build (loaded through LSS_LIB). One summary line per run.
#   bash scripts/gpu_ab_lib.sh "product|" "old|" "product|--config c2" "old|--config c2"
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  lib="${v%%|*}"; flags="${v#*|}"
  path=""; [ "$lib" != product ] && path="$GRAFT_REPO_ROOT/lss-carla_amd/variants/$lib.so"
  LSS_LIB="$path" timeout -k 10 420 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pmc-traffic 0 $flags \
    > gpurun_out/ab.json 2> gpurun_out/ab.log; rc=$?
  if [ $rc -ne 0 ]; then echo "== $v FAILED rc=$rc"; tail -5 gpurun_out/ab.log; exit $rc; fi
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('== $v:', d['value'], 'fps', d['ms_per_step'], 'ms/step; splat', d['roofline']['avg_launch_us'], 'us frac', d['roofline']['frac'])"
done
exit 0
