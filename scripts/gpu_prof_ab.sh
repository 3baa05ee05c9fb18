# rocprofv3 kernel-trace A/B of library builds inside the c3 training step (graph replays):
# per build, the hot-path kernels' in-step averages (scripts/steady_summary.py).
#   [BENCH_ARGS="--config c5"] bash scripts/gpu_prof_ab.sh product nt0 product nt0
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/profab
i=0
for lib in "$@"; do
  i=$((i + 1))
  path=""; [ "$lib" != product ] && path="$GRAFT_REPO_ROOT/lss-carla_amd/variants/$lib.so"
  rm -rf /tmp/pab
  LSS_LIB="$path" timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pab -o run -- \
    python3 -u bench.py --steps 10 --cpu-baseline 0 --pmc-traffic 0 ${BENCH_ARGS:-} > gpurun_out/profab/${i}_$lib.log 2>&1 || exit 1
  csv=$(ls /tmp/pab/*/run_kernel_trace.csv /tmp/pab/run_kernel_trace.csv 2>/dev/null | head -1)
  echo "== $i $lib"
  python3 scripts/steady_summary.py "$csv" | python3 -c "import json,sys; d=json.load(sys.stdin)['hot_path_kernels']; [print(f'{k[:40]:40s} {v[\"avg_us\"]:7.2f} {v[\"median_us\"]:7.2f}') for k, v in d.items()]"
  rm -rf /tmp/pab
done
exit 0
