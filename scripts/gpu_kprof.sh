# Per-kernel durations (rocprofv3 kernel trace) of the kbench rows, product library and each variant
# run as THE library in its own process, so same-named kernels do not mix.
# usage: bash scripts/gpu_kprof.sh [variant ...]     ("product" = the in-tree library)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/kprof; mkdir -p $OUT
for v in ${*:-product}; do
  lib=""; [ "$v" != product ] && lib="--lib $v"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$v -o run -- \
    python3 -u scripts/kbench.py --variants 0 --cold 0 --iters 20 $lib > $OUT/$v.log 2>&1; rc=$?
  echo "$v rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/$v.log; exit $rc; }
  f=$(ls $OUT/$v/*/run_kernel_stats.csv 2>/dev/null | head -1)
  [ -z "$f" ] && f=$(ls $OUT/$v/run_kernel_stats.csv 2>/dev/null)
  python3 - "$f" <<'PY'
import csv, sys
for r in sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))[:24]:
    print(f"  {r['Name'][:90]:90s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:8.2f} us")
PY
done
exit 0
