# Round 4: store flavours of the channels-last splat (chunk rows / zero rows: plain, nt, sc1 = written
# through the XCD's L2) and of the write-ceiling kernel; splat-only and in-step A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4g; mkdir -p $OUT
timeout -k 10 400 python -u scripts/splat_ab.py --config c3 --libs product,cnt,csc1,csc1_zsc1,cnt_zplain,chunkonly,chunkonly_csc1 \
  > $OUT/splat_ab_c3.log 2>&1 || { tail -30 $OUT/splat_ab_c3.log; exit 1; }
grep -v '^{' $OUT/splat_ab_c3.log | grep -v amdgpu.ids
bash scripts/gpu_prof_ab.sh product csc1 csc1_zsc1 cnt product 2>&1 | tee $OUT/prof_ab.txt || exit 1
