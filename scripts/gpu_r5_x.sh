# Round 5: clip_grad_norm_ + Adam on lss_clip_adam: optimizer tests, the captured-step tests, then the c3 bench A/B
# (--hip-adam 1 / 0) and a kernel trace of the product.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5x; mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_optim.py tests/test_gpu_captured_step.py \
  tests/test_gpu_overlap.py tests/test_gpu_loss.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash scripts/gpu_ab_lib.sh "product|" "product|--hip-adam 0" "product|" "product|--hip-adam 0" 2>&1 | tee $OUT/ab.txt || exit 1
rm -rf /tmp/prof_x
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_x -o run -- \
  python3 -u bench.py --steps 10 --warmup 3 --profile-steps 0 --cpu-baseline 0 --pmc-traffic 0 --in-graph-prof 0 \
  > $OUT/bench_prof.log 2>&1 || { tail -20 $OUT/bench_prof.log; exit 1; }
csv=$(ls /tmp/prof_x/*/run_kernel_trace.csv /tmp/prof_x/run_kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/kernel_calls.py "$csv" "" 8 > $OUT/all_calls_c3.txt && python3 scripts/step_kernels.py "$csv" 3 12 60 > $OUT/step_kernels_c3.txt || exit 1
head -1 $OUT/step_kernels_c3.txt; grep -E "k_clip" $OUT/all_calls_c3.txt | cut -c1-100
