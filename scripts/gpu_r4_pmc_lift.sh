# Round 4: PMC counters of the fused lift (packed weights), one rocprofv3 pass per counter group.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc
bash scripts/gpu_pmc.sh depthnet_lift_nhwc_packed || exit 1
python3 scripts/pmc_summary.py k_depthnet_lift3 | tee gpurun_out/pmc/lift3_pmc_summary.txt
