# Round 5: depthnet weight gradient as a split-K batched GEMM and its bias gradient on lss_channel_sums: the fused
# lift / parity tests, the c3 bench, and a kernel trace of one step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5w; mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lift_nhwc.py tests/test_gpu_parity.py \
  tests/test_gpu_captured_step.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash scripts/gpu_ab_lib.sh "product|" "product|" 2>&1 | tee $OUT/ab.txt || exit 1
rm -rf /tmp/prof_w
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_w -o run -- \
  python3 -u bench.py --steps 10 --warmup 3 --profile-steps 0 --cpu-baseline 0 --pmc-traffic 0 --in-graph-prof 0 \
  > $OUT/bench_prof.log 2>&1 || { tail -20 $OUT/bench_prof.log; exit 1; }
csv=$(ls /tmp/prof_w/*/run_kernel_trace.csv /tmp/prof_w/run_kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/kernel_calls.py "$csv" "" 8 > $OUT/all_calls_c3.txt && python3 scripts/step_kernels.py "$csv" 3 12 60 > $OUT/step_kernels_c3.txt || exit 1
head -1 $OUT/step_kernels_c3.txt; grep -n -A8 "k_splat_bwd_tile" $OUT/all_calls_c3.txt | cut -c1-120
