# Round 5: channels-last BN statistics with 8 rows in flight (and 1,024 groups) vs 4 rows (product): the GPU suite
# on the product, the batch-norm tests on the variant library, then the c3 bench A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5y; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
LSS_LIB=$GRAFT_REPO_ROOT/lss-carla_amd/variants/sr8g1k.so timeout -k 10 300 python -u -m pytest tests/test_gpu_convs.py -q -k bn \
  -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/bn_tests_sr8g1k.log 2>&1 || { tail -30 $OUT/bn_tests_sr8g1k.log; exit 1; }
tail -1 $OUT/bn_tests_sr8g1k.log
bash scripts/gpu_ab_lib.sh "product|" "sr8|" "sr8g1k|" "product|" "sr8|" "sr8g1k|" 2>&1 | tee $OUT/ab.txt
