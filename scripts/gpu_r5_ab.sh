# Round 5: GPU suite and smoke at HEAD.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5ab; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1; trc=$?; tail -1 $OUT/gpu_tests.log; [ $trc -ne 0 ] && { tail -30 $OUT/gpu_tests.log; exit $trc; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
