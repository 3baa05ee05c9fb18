# Stage timelines (LSS_TRACE=1 builds in variants/): usage  bash scripts/gpu_trace.sh "lift:trace bwd:trace ..."
set -o pipefail
OUT=gpurun_out/tr; mkdir -p $OUT
for kv in $1; do
  k=${kv%%:*}; v=${kv#*:}
  timeout -k 10 200 python3 -u scripts/stage_trace.py $k --lib $v > $OUT/${k}_$v.txt 2>&1; rc=$?
  echo "$k $v rc=$rc"; grep -v Warn $OUT/${k}_$v.txt | grep -v "^t=" | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
done
exit 0
