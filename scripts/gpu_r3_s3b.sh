# Round 3, third session, part 2: smoke(), then the c5, c2 and fp32 NCHW lines (gpu_r3_lines.sh). gpurun_out/r3s3.
set -o pipefail
OUT=gpurun_out/r3s3; mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
echo "smoke=$rc"; tail -3 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
OUT=$OUT bash scripts/gpu_r3_lines.sh c5 c2 fp32
