# Round 4: zero-fill hold-back variants -- after the cell_start loads, paced stores -- in-step A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4n; mkdir -p $OUT
bash scripts/gpu_prof_ab.sh product hbafter32 hbafter48 pace1 pace4 product 2>&1 | tee $OUT/prof_ab.txt || exit 1
