# Round 5: fused squeeze-excite launches (k_se_scale_mlp2, k_se_dx_mlpb2) vs the unfused build (bit-equality and
# launch times at the trunk's shapes), row-walking channels-last BN apply passes vs the grid-stride ones; the conv
# tests, then the c3 bench A/B and a kernel trace of the product.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5v; mkdir -p $OUT
timeout -k 10 200 python3 -u scripts/se_ab.py --lib sefused0 > $OUT/se_ab.txt 2>&1; rc=$?; cat $OUT/se_ab.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_convs.py tests/test_gpu_captured_step.py \
  > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash scripts/gpu_ab_lib.sh "product|" "sefused0|" "bnrows0|" "product|" "sefused0|" "bnrows0|" 2>&1 | tee $OUT/ab.txt || exit 1
rm -rf /tmp/prof_v
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_v -o run -- \
  python3 -u bench.py --steps 10 --warmup 3 --profile-steps 0 --cpu-baseline 0 --pmc-traffic 0 --in-graph-prof 0 \
  > $OUT/bench_prof.log 2>&1 || { tail -20 $OUT/bench_prof.log; exit 1; }
csv=$(ls /tmp/prof_v/*/run_kernel_trace.csv /tmp/prof_v/run_kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/kernel_calls.py "$csv" "" 8 > $OUT/all_calls_c3.txt && python3 scripts/step_kernels.py "$csv" 3 12 60 > $OUT/step_kernels_c3.txt || exit 1
head -1 $OUT/step_kernels_c3.txt
