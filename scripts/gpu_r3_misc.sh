# Round 3: splat per-wave trace (step mode), the reference-layout fp32 training line, the default bench.
set -o pipefail
OUT=gpurun_out/r3; mkdir -p $OUT
timeout -k 10 200 python scripts/splat_trace.py > $OUT/splat_trace.txt 2>&1; rc=$?; echo "trace=$rc"; head -20 $OUT/splat_trace.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -m pytest tests/test_gpu_parity2.py -k fill_in_lift -q -p no:cacheprovider > $OUT/fill_test.log 2>&1; rc=$?; echo "filltest=$rc"; tail -2 $OUT/fill_test.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python bench.py --config c3 --dtype fp32 --bev-layout nchw --cpu-baseline 0 > $OUT/bench_c3_fp32_nchw.json 2> $OUT/bench_c3_fp32_nchw.log; rc=$?
echo "fp32=$rc"; tail -c 400 $OUT/bench_c3_fp32_nchw.json; [ $rc -ne 0 ] && { tail -5 $OUT/bench_c3_fp32_nchw.log; exit $rc; }
timeout -k 10 700 python bench.py > $OUT/bench.json 2> $OUT/bench.log; rc=$?
echo "bench=$rc"; tail -c 1500 $OUT/bench.json; [ $rc -ne 0 ] && tail -5 $OUT/bench.log
exit $rc
