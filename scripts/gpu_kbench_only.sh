set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python scripts/kbench.py "$@" > gpurun_out/kbench.log 2>&1; rc=$?; echo "kbench=$rc"; grep -v Warn gpurun_out/kbench.log
exit $rc
