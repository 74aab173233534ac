# Targeted GPU tests (pytest -k expression over the -m gpu tests), then an optional profile.
# Usage: gpurun -- bash tools/gpu_check.sh <tag> "<pytest -k expr>" [prof [micro]]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-c}
K=${2:-}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/${tag}_pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${tag}_pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/${tag}_pytest_gpu.txt
if [ "${3:-}" = "prof" ]; then
  bash tools/gpu_prof.sh ${tag} ${4:-} || exit 1
fi
echo done
