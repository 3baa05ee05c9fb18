# Round 4: GPU suite (two-part splat, prefill in the captured step), the c3 bench with the BEV's empty
# rows written inside the splat / beside the lift / beside the trunk, the chunk phase decomposed,
# its per-wave trace alone, the packed lift's stage trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4h; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1; trc=$?
tail -4 $OUT/gpu_tests.log; echo "tests rc=$trc"
[ $trc -ne 0 ] && exit $trc
for pf in none lift trunk; do
  timeout -k 10 600 python -u bench.py --cpu-baseline 0 --pmc-traffic 0 --bev-prefill $pf > $OUT/bench_c3_prefill_$pf.log 2>&1 \
    || { tail -20 $OUT/bench_c3_prefill_$pf.log; exit 1; }
  tail -1 $OUT/bench_c3_prefill_$pf.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$pf', d['value'], d['ms_per_step'], json.dumps(r['in_graph']))"
done
timeout -k 10 300 python -u scripts/splat_ab.py --config c3 --libs product,chunkonly,c_nostore,c_nostore_skipall --ceiling 0 \
  > $OUT/splat_ab_c3.log 2>&1 || { tail -30 $OUT/splat_ab_c3.log; exit 1; }
grep -v '^{' $OUT/splat_ab_c3.log | grep -v amdgpu.ids
timeout -k 10 200 python -u scripts/stage_trace.py lift3 --config c3 --lib trace > $OUT/trace_lift3_packed.txt 2>&1 || { tail -20 $OUT/trace_lift3_packed.txt; exit 1; }
head -9 $OUT/trace_lift3_packed.txt
timeout -k 10 200 python -u scripts/splat_trace.py --lib trace_chunkonly --mode step > $OUT/trace_chunkonly_step.txt 2>&1 || { tail -20 $OUT/trace_chunkonly_step.txt; exit 1; }
head -12 $OUT/trace_chunkonly_step.txt
