# Round 4: where the channels-last splat's chunk phase goes (gathers replaced by L1-resident rows /
# one depth line, chunk waves alone), then per-wave stage traces of the NCHW tile kernel (c2) and
# the fused lift.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4f; mkdir -p $OUT
timeout -k 10 300 python -u scripts/splat_ab.py --config c3 --libs product,chunkonly,c_skiprow,c_skipdep,c_skipboth,skipboth,zeroonly --ceiling 0 \
  > $OUT/splat_ab_c3.log 2>&1 || { tail -30 $OUT/splat_ab_c3.log; exit 1; }
grep -v '^{' $OUT/splat_ab_c3.log | grep -v amdgpu.ids
timeout -k 10 200 python -u scripts/stage_trace.py nchw --config c2 > $OUT/trace_nchw_c2.txt 2>&1 || { tail -20 $OUT/trace_nchw_c2.txt; exit 1; }
head -40 $OUT/trace_nchw_c2.txt
timeout -k 10 200 python -u scripts/stage_trace.py lift3 --config c3 > $OUT/trace_lift3_c3.txt 2>&1 || { tail -20 $OUT/trace_lift3_c3.txt; exit 1; }
head -30 $OUT/trace_lift3_c3.txt
