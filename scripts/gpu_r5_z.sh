# Round 5: channels-last BN statistics with 8 rows in flight (and 1,024 groups) vs 4 rows (product): c3 bench A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5z; mkdir -p $OUT
bash scripts/gpu_ab_lib.sh "product|" "sr8|" "sr8g1k|" "product|" "sr8|" "sr8g1k|" 2>&1 | tee $OUT/ab.txt
