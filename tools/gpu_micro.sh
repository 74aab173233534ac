# Microbenchmarks (each under its own limit): hash-to-G2 phases, combine phases, bucket MSM vs the
# combine's per-lane MSM, coin check parts -- or the named ones.
# Usage: gpurun -- bash tools/gpu_micro.sh <tag> ["bench1 bench2 ..."]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=${1:-m}
for b in ${2:-hashg2 combine msm_bucket coin_parts}; do
  if [ -x tools/microbench/$b ]; then
    echo "== $b"
    timeout -k 10 120 tools/microbench/$b || { echo "$b failed"; exit 1; }
  fi
done > gpurun_out/${tag}_micro.txt 2>&1
cat gpurun_out/${tag}_micro.txt
