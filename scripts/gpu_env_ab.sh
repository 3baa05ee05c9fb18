# In-step A/B of environment settings (e.g. "LSS_FILL_IN_LIFT=1" "LSS_FILL_IN_LIFT=0"): a rocprofv3
# kernel trace of a short bench run per setting, the hot-path kernels per timed replay (hot_steps.py).
#   [BENCH_ARGS="--config c5"] bash scripts/gpu_env_ab.sh "A=1" "A=0" "A=1" "A=0"
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/envab
i=0
for setting in "$@"; do
  i=$((i + 1))
  rm -rf /tmp/eab
  env $setting timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/eab -o run -- \
    python3 -u bench.py --steps 10 --warmup 3 --profile-steps 0 --cpu-baseline 0 --pmc-traffic 0 --in-graph-prof 0 \
    ${BENCH_ARGS:-} > gpurun_out/envab/$i.json 2> gpurun_out/envab/$i.log || { tail -5 gpurun_out/envab/$i.log; exit 1; }
  csv=$(find /tmp/eab -name "*kernel_trace.csv" | head -1)
  echo "== $i $setting: $(python3 -c "import json;d=json.load(open('gpurun_out/envab/$i.json'));print(d['value'], 'frames/s', d['ms_per_step'], 'ms')")"
  python3 scripts/hot_steps.py "$csv" 5 14 | tee gpurun_out/envab/$i.hot.txt
done
exit 0
