# Profile the bench's kernels: rocprofv3 kernel trace + stats (no PMC in this pass). Args: extra bench flags.
# PROF_DIR (default gpurun_out/prof) receives the trace and the bench log.
set -o pipefail
D=${PROF_DIR:-gpurun_out/prof}
mkdir -p "$D"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$D" -o run -- \
    python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 "$@" > "$D.log" 2>&1
rc=$?; echo "prof=$rc"; tail -1 "$D.log" | cut -c1-300
exit $rc
