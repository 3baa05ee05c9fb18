# Round 5: LDS-staged depthwise kernels (product) vs the register-tiled ones (dwold variant): conv tests,
# then the c3 step under rocprofv3 for each (whole step by kernel, per-call depthwise list).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5p; mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_convs.py tests/test_gpu_pointwise.py tests/test_gpu_captured_step.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for lib in product dwold; do
  path=""; [ "$lib" != product ] && path="$GRAFT_REPO_ROOT/lss-carla_amd/variants/$lib.so"
  rm -rf /tmp/prof_dw
  LSS_LIB="$path" timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_dw -o run -- \
    python3 -u bench.py --steps 20 --warmup 3 --profile-steps 0 --cpu-baseline 0 --pmc-traffic 0 --in-graph-prof 0 \
    > $OUT/bench_$lib.log 2>&1 || { tail -20 $OUT/bench_$lib.log; exit 1; }
  csv=$(ls /tmp/prof_dw/*/run_kernel_trace.csv /tmp/prof_dw/run_kernel_trace.csv 2>/dev/null | head -1)
  python3 scripts/step_kernels.py "$csv" 5 18 60 > $OUT/step_kernels_$lib.txt || exit 1
  python3 scripts/kernel_calls.py "$csv" k_dw > $OUT/dw_calls_$lib.txt || exit 1
  echo "== $lib"; head -1 $OUT/step_kernels_$lib.txt; grep -E "k_dw" $OUT/step_kernels_$lib.txt | cut -c1-120; tail -1 $OUT/dw_calls_$lib.txt
done
