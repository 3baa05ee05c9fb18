# Round 4: the splat with each entry's context row computed from its point id (no sorted_row in the
# CSR): GPU suite for parity, kbench A/B (rows loaded vs derived), in-step times.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4k; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1; trc=$?
tail -3 $OUT/gpu_tests.log; echo "tests rc=$trc"
[ $trc -ne 0 ] && exit $trc
timeout -k 10 300 python -u scripts/kbench.py --libs product > $OUT/kbench.log 2>&1 || { tail -20 $OUT/kbench.log; exit 1; }
grep -v '^{' $OUT/kbench.log | grep -v amdgpu.ids
bash scripts/gpu_prof_ab.sh product product 2>&1 | tee $OUT/prof_ab.txt || exit 1
