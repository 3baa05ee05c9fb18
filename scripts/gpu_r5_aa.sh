# Round 5: upsample backward with each output row's taps loaded together (k_up_bwd_taps) vs the branchy gather
# (variant upold): the upsample tests, then the c3 bench A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5aa; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_convs.py -k "upsample or up_" \
  > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash scripts/gpu_ab_lib.sh "product|" "upold|" "product|" "upold|" 2>&1 | tee $OUT/ab.txt
