# Round 4: GPU suite (packed depthnet weights, ABI 18), store flavours of the channels-last splat
# (chunk rows / zero rows: plain, nt, sc1 = written through the XCD's L2), waves per splat block,
# the write-ceiling forms; splat-only and in-step A/B; the fused lift with packed weights.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4g; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1; trc=$?
tail -4 $OUT/gpu_tests.log; echo "tests rc=$trc"
case $trc in 0|1) ;; *) exit $trc ;; esac
timeout -k 10 400 python -u scripts/kbench.py --libs product > $OUT/kbench.log 2>&1 || { tail -20 $OUT/kbench.log; exit 1; }
grep -v '^{' $OUT/kbench.log | grep -v amdgpu.ids
timeout -k 10 500 python -u scripts/splat_ab.py --config c3 --libs product,cnt,csc1,csc1_zsc1,cnt_zplain,chunkonly,chunkonly_csc1,w2,w7,w8 \
  > $OUT/splat_ab_c3.log 2>&1 || { tail -30 $OUT/splat_ab_c3.log; exit 1; }
grep -v '^{' $OUT/splat_ab_c3.log | grep -v amdgpu.ids
bash scripts/gpu_prof_ab.sh product csc1 cnt w7 2>&1 | tee $OUT/prof_ab.txt || exit 1
exit $trc
