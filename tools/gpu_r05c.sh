set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_check.sh r05c "host_api or degenerate or fallback or one_lane_checks or test_epoch_matches_golden" || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --configs= > gpurun_out/r05c_bench.json 2> gpurun_out/r05c_bench.err || { echo "bench failed"; tail -20 gpurun_out/r05c_bench.err; exit 1; }
cut -c1-900 gpurun_out/r05c_bench.json
bash tools/gpu_prof.sh r05c micro
