# Round-end check: every GPU test, the default bench line (all configs, CPU baselines), the
# shard-of-8 rehearsal, a rocprof kernel summary of the N=256 epoch and of the C4 round, and the
# PMC passes (wave states, FETCH_SIZE, WRITE_SIZE) with the traffic records of the one-lane share
# check and the two-lane coin check.  Usage: COMMIT=<sha> gpurun -- bash tools/gpu_final.sh <tag>
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
cd "$R" && bash tools/gpu_prof.sh ${tag}p > /dev/null 2>&1 || { echo "pmc failed"; exit 1; }
# HBM-traffic records of the dominant regions (bench.py traffic_record): the one-lane share check
# and the two-lane coin check, from the same FETCH / WRITE passes
python3 tools/pmc_json.py gpurun_out/${tag}p_f/run_results.db gpurun_out/${tag}p_p/run_results.db \
  "k_verify_shares_ml,k_fe1<0>,k_fe1<1>,k_fe1<3>,k_fe1<5>,k_verify_shares(" ${COMMIT:-unknown} > gpurun_out/${tag}_pmc_hbm.json || echo "pmc json failed"
python3 tools/pmc_json.py gpurun_out/${tag}p_f/run_results.db gpurun_out/${tag}p_p/run_results.db \
  "k_verify_sig_shares2(,k_verify_sig_shares2_fe<true>" ${COMMIT:-unknown} --skip-empty > gpurun_out/${tag}_pmc_coin.json || echo "pmc coin json failed"
cat gpurun_out/${tag}_pmc_hbm.json gpurun_out/${tag}_pmc_coin.json
echo done
