# In-step A/B of CamEncode.up1 channels-last (lift3) vs NCHW (lift2), alternating on one box.
set -o pipefail
for v in 1 0 1 0; do
  echo "== LSS_UP1_CL=$v"; LSS_UP1_CL=$v bash scripts/gpu_prof_ab.sh product | grep -v "^=="
done
