# Round 4: zero-fill hold-back, repeated in-step A/B (alternating builds on one box), plus the
# flat cast at 16 elements per thread (product) -- GPU tests of the lift / captured step first.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4m; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_lift_nhwc.py tests/test_gpu_captured_step.py -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -20 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
bash scripts/gpu_prof_ab.sh product zs32 product zs32 zs24 zs40 zs32g28 2>&1 | tee $OUT/prof_ab.txt || exit 1
