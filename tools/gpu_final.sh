# Round-end check: every GPU test, the default bench line (all configs, CPU baselines), the
# shard-of-8 rehearsal, a rocprof kernel summary of the N=256 epoch and of the C4 round, and the
# PMC passes of the one-lane share check.  Usage: gpurun -- bash tools/gpu_final.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-final}
R="$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${tag}_pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/${tag}_pytest_gpu.txt
timeout -k 10 900 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
cut -c1-400 gpurun_out/${tag}_bench.json
timeout -k 10 300 python -u bench.py --shard-of 8 --no-cpu-baseline --configs= > gpurun_out/${tag}_bench_shard8.json 2> gpurun_out/${tag}_shard8.err || { echo "shard8 failed"; tail -20 gpurun_out/${tag}_shard8.err; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${tag}_prof" -o run -- python3 -u "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --in-flight 1 --configs=C4 > "$R/gpurun_out/${tag}_prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/${tag}_prof.log"; exit 1; }
python3 "$R/tools/kstats.py" "$R/gpurun_out/${tag}_prof/run_results.db" > "$R/gpurun_out/${tag}_kernel_stats.txt" && head -30 "$R/gpurun_out/${tag}_kernel_stats.txt"
cd "$R" && bash tools/gpu_pmc_fe.sh ${tag} 1 > /dev/null 2>&1 || echo "pmc failed"
echo done
