# Full GPU check: every -m gpu test, then the quick bench + rocprof summary (tools/gpu_quick.sh
# without its pytest step).  Usage: gpurun -- bash tools/gpu_full.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-full}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/${tag}_pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/${tag}_pytest_gpu.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --configs= > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
cut -c1-1200 gpurun_out/${tag}_bench.json
R="$GRAFT_REPO_ROOT"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${tag}_prof" -o run -- python3 -u "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --in-flight 1 --configs= > "$R/gpurun_out/${tag}_prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/${tag}_prof.log"; exit 1; }
python3 "$R/tools/kstats.py" "$R/gpurun_out/${tag}_prof/run_results.db" > "$R/gpurun_out/${tag}_kernel_stats.txt" && head -24 "$R/gpurun_out/${tag}_kernel_stats.txt"
echo done
