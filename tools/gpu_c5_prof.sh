# rocprofv3 kernel summary of the C5 (Broadcast) config alone.  Usage: gpurun -- bash tools/gpu_c5_prof.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-c5p}
R="$GRAFT_REPO_ROOT"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${tag}_prof" -o run -- python3 -u "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --in-flight 1 --configs=C5 > "$R/gpurun_out/${tag}_prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/${tag}_prof.log"; exit 1; }
python3 "$R/tools/kstats.py" "$R/gpurun_out/${tag}_prof/run_results.db" > "$R/gpurun_out/${tag}_kernel_stats.txt" && head -40 "$R/gpurun_out/${tag}_kernel_stats.txt"
rm -f "$R/gpurun_out/${tag}_prof/run_results.db"
