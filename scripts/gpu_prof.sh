# Profile the bench's kernels: rocprofv3 kernel trace + stats (no PMC in this pass). Args: extra bench flags.
set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 "$@" > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "prof=$rc"; tail -1 gpurun_out/prof_bench.log | cut -c1-300
exit $rc
