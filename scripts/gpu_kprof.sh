# Per-kernel durations (rocprofv3 kernel trace) of the kbench rows, product library and each variant
# run as THE library in its own process, so same-named kernels do not mix. Keeps only the text
# summaries (gpurun_out/kprof/summary.txt): the trace databases are deleted on the box.
# usage: bash scripts/gpu_kprof.sh [variant ...]     ("product" = the in-tree library)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/kprof; mkdir -p $OUT; : > $OUT/summary.txt
for v in ${*:-product}; do
  lib=""; [ "$v" != product ] && lib="--lib $v"
  rm -rf /tmp/kprof_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kprof_$v -o run -- \
    python3 -u scripts/kbench.py --variants 0 --cold 0 --iters 20 $lib > $OUT/$v.log 2>&1; rc=$?
  echo "$v rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/$v.log; exit $rc; }
  db=$(ls /tmp/kprof_$v/*/run_results.db /tmp/kprof_$v/run_results.db 2>/dev/null | head -1)
  echo "== $v" >> $OUT/summary.txt
  python3 scripts/kprof_summary.py "$db" >> $OUT/summary.txt
  rm -rf /tmp/kprof_$v
done
exit 0
