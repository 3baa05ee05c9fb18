# Round 4 evidence, part B: the other bench lines -- c5 (B=4 per GPU, 256x704, D=60, 400x400),
# c2 forward in the reference's precision and layout (fp32, NCHW BEV), and the c3 training step in
# fp32 with the NCHW BEV (the reference's train_simbev.py path), each with its splat roofline.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4final; mkdir -p $OUT
timeout -k 10 600 python -u bench.py --config c5 --cpu-baseline 0 > $OUT/bench_c5.log 2>&1 || { tail -20 $OUT/bench_c5.log; exit 1; }
tail -1 $OUT/bench_c5.log > $OUT/bench_c5.json; cut -c1-300 $OUT/bench_c5.json
timeout -k 10 600 python -u bench.py --config c2 --cpu-baseline 0 > $OUT/bench_c2.log 2>&1 || { tail -20 $OUT/bench_c2.log; exit 1; }
tail -1 $OUT/bench_c2.log > $OUT/bench_c2.json; cut -c1-300 $OUT/bench_c2.json
timeout -k 10 700 python -u bench.py --config c3 --dtype fp32 --bev-layout nchw --miopen-find 0 --cpu-baseline 0 \
  > $OUT/bench_c3_fp32_nchw_train.log 2>&1 || { tail -20 $OUT/bench_c3_fp32_nchw_train.log; exit 1; }
tail -1 $OUT/bench_c3_fp32_nchw_train.log > $OUT/bench_c3_fp32_nchw_train.json; cut -c1-300 $OUT/bench_c3_fp32_nchw_train.json
