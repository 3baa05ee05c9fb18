set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4d; mkdir -p $OUT
timeout -k 10 200 python -u scripts/splat_trace.py --lib trace --mode step > $OUT/trace_step.txt 2>&1 || { tail -20 $OUT/trace_step.txt; exit 1; }
timeout -k 10 200 python -u scripts/splat_trace.py --lib trace --mode warm > $OUT/trace_warm.txt 2>&1 || { tail -20 $OUT/trace_warm.txt; exit 1; }
head -30 $OUT/trace_step.txt
