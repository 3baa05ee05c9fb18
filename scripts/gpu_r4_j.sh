# Round 4: the fused lift's loads non-temporal (L1-bypassing: weights / features / both) -- kbench,
# stage traces, in-step times.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4j; mkdir -p $OUT
timeout -k 10 300 python -u scripts/kbench.py --libs product,nt1,nt2,nt3 --only depthnet_lift > $OUT/kbench.log 2>&1 || { tail -20 $OUT/kbench.log; exit 1; }
grep -v '^{' $OUT/kbench.log | grep -v amdgpu.ids | grep -v None
for lib in trace trace_nt3; do
  timeout -k 10 200 python -u scripts/stage_trace.py lift3 --config c3 --lib $lib > $OUT/trace_lift3_$lib.txt 2>&1 || { tail -20 $OUT/trace_lift3_$lib.txt; exit 1; }
  head -8 $OUT/trace_lift3_$lib.txt
done
bash scripts/gpu_prof_ab.sh product nt3 nt1 2>&1 | tee $OUT/prof_ab.txt || exit 1
