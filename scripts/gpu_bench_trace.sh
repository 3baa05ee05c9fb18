set -o pipefail
OUT=gpurun_out/g2; mkdir -p $OUT
timeout -k 10 600 python bench.py --cpu-baseline 0 > $OUT/bench.log 2>&1; rc=$?; echo "bench=$rc"; tail -1 $OUT/bench.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --cpu-baseline 0 > $OUT/trace_bench.log 2>&1; rc=$?
echo "trace=$rc"; tail -1 $OUT/trace_bench.log | cut -c1-300
