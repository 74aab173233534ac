set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05d}
bash tools/gpu_check.sh $tag "host_api or degenerate or fallback or one_lane_checks or test_epoch_matches_golden or fused_epoch" || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --configs= > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/${tag}_bench.json')); print(d['ms_per_step'], d['kernels_ms'], d['roofline']['frac'], d.get('epochs_in_flight',{}).get('ms_per_epoch'))"
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${tag}_prof" -o run -- python3 -u "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --in-flight 1 --configs= > "$R/gpurun_out/${tag}_prof.log" 2>&1 || { echo "rocprof failed"; exit 1; }
python3 "$R/tools/kstats.py" "$R/gpurun_out/${tag}_prof/run_results.db" > "$R/gpurun_out/${tag}_kernel_stats.txt" && head -24 "$R/gpurun_out/${tag}_kernel_stats.txt"
cd "$R" && timeout -k 10 120 tools/microbench/combsig > gpurun_out/${tag}_combsig.txt 2>&1; cat gpurun_out/${tag}_combsig.txt
echo done
