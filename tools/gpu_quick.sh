# Quick GPU iteration: the threshold parity tests, the N=256 bench line without CPU legs, and a
# rocprofv3 kernel-trace summary of it -- each step under its own limit, stopping at the first failure.
# Usage: gpurun -- bash tools/gpu_quick.sh <tag> [pytest -k expression]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-q}
K=${2:-}
timeout -k 10 300 python -u -m pytest tests/test_gpu_threshold.py -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/${tag}_pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${tag}_pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/${tag}_pytest_gpu.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --configs= > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
cut -c1-1500 gpurun_out/${tag}_bench.json
if [ "${PROF:-1}" = "1" ]; then
  R="$GRAFT_REPO_ROOT"
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${tag}_prof" -o run -- python3 -u "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --in-flight 1 --configs= > "$R/gpurun_out/${tag}_prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/${tag}_prof.log"; exit 1; }
  python3 "$R/tools/kstats.py" "$R/gpurun_out/${tag}_prof/run_results.db" > "$R/gpurun_out/${tag}_kernel_stats.txt" && cat "$R/gpurun_out/${tag}_kernel_stats.txt"
fi
echo done
