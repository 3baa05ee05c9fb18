# Round 5: the other configs' bench lines at HEAD: c2 (fp32 forward, the reference's precision; channels-last BEV,
# the module default) and c5 (256x704, D=60, 400x400, B=4 per GPU, bf16 training).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5final_e; mkdir -p $OUT
Q="--pmc-traffic 0 --cpu-baseline 0"
timeout -k 10 400 python -u bench.py --config c2 --dtype fp32 --mode fwd $Q > $OUT/bench_c2.log 2>&1 || { tail -20 $OUT/bench_c2.log; exit 1; }
tail -1 $OUT/bench_c2.log > $OUT/bench_c2_fp32_fwd.json; cut -c1-300 $OUT/bench_c2_fp32_fwd.json
timeout -k 10 500 python -u bench.py --config c5 $Q > $OUT/bench_c5.log 2>&1 || { tail -20 $OUT/bench_c5.log; exit 1; }
tail -1 $OUT/bench_c5.log > $OUT/bench_c5.json; cut -c1-300 $OUT/bench_c5.json
