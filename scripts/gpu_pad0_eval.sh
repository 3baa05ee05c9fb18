# The NCHW tile kernel's tighter LDS stride (LSS_NCHW_PAD=0), on evidence: (1) the debug-checked subset
# (geometry / CSR / splat / backward / QuickCumsum parity and the fp32 NCHW module test) on a PAD=0
# LSS_DEBUG build, (2) the full GPU suite on the PAD=0 release build, unserialized, (3) c2 in-step A/B.
set -o pipefail
OUT=gpurun_out/pad0; mkdir -p $OUT
V=$GRAFT_REPO_ROOT/lss-carla_amd/variants
LSS_DEBUG=1 LSS_LIB=$V/pad0_debug.so timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider -m gpu \
    --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_quickcumsum.py \
    tests/test_gpu_parity2.py tests/test_gpu_debug.py::test_debug_checks_fire > $OUT/debug_subset.log 2>&1; rc=$?
echo "debug_subset=$rc"; grep -E " passed| failed|Error" $OUT/debug_subset.log | tail -3; [ $rc -ne 0 ] && exit $rc
LSS_LIB=$V/pad0.so timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider -m gpu --timeout 300 \
    --timeout-method thread tests > $OUT/full.log 2>&1; rc=$?
echo "full=$rc"; grep -E " passed| failed|Error" $OUT/full.log | tail -3; [ $rc -ne 0 ] && exit $rc
BENCH_ARGS="--config c2" bash scripts/gpu_prof_ab.sh product pad0 product pad0 > $OUT/ab_c2.txt 2>&1; rc=$?
cat $OUT/ab_c2.txt | grep -E "==|nchw"
exit $rc
