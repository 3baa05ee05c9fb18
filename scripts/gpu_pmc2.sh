# PMC passes over kbench's splat_fwd (product kernel + one variant): one rocprofv3 run per counter group.
# usage: bash scripts/gpu_pmc2.sh <variant-filter>
set -o pipefail
OUT=gpurun_out/pmc2; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
VF="$1"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS" \
           "TCC_HIT_sum TCC_MISS_sum" "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex k_splat_fwd --output-format csv -d $OUT/p$i -o run -- \
      python3 scripts/kbench.py --only splat_fwd --iters 20 --variant-filter "$VF" > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
python3 - <<'PY'
import collections, csv, glob
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc2/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        key = n[n.find("k_splat"):][:60]
        vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    print(k)
    for c in sorted(d):
        v = d[c]
        print(f"   {c:28s} {sum(v) / len(v):16.1f}   (n={len(v)})")
PY
