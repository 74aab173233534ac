set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp HBX_SPLIT_PREP=1
R="$GRAFT_REPO_ROOT"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r05q_prof" -o run -- python3 -u "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --in-flight 1 --configs= > "$R/gpurun_out/r05q_prof.log" 2>&1 || { echo "rocprof failed"; tail -5 "$R/gpurun_out/r05q_prof.log"; exit 1; }
python3 "$R/tools/kstats.py" "$R/gpurun_out/r05q_prof/run_results.db" > "$R/gpurun_out/r05q_kernel_stats.txt" && head -16 "$R/gpurun_out/r05q_kernel_stats.txt"
