# One GPU round trip: parity tests, the default bench line (with the CPU baseline), the
# shard-of-8 rehearsal and a rocprofv3 kernel-trace summary of the bench -- each step under its
# own limit, stopping at the first failure.  Usage: gpurun -- bash tools/gpu_round.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${tag}_pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/${tag}_pytest_gpu.txt
timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
cat gpurun_out/${tag}_bench.json
timeout -k 10 200 python -u bench.py --shard-of 8 --no-cpu-baseline > gpurun_out/${tag}_bench_shard8.json 2> gpurun_out/${tag}_bench_shard8.err || { echo "shard8 failed"; tail -20 gpurun_out/${tag}_bench_shard8.err; exit 1; }
cat gpurun_out/${tag}_bench_shard8.json
if [ "${PROF:-1}" = "1" ]; then
  R="$GRAFT_REPO_ROOT"
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${tag}_prof" -o run -- python3 -u "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --in-flight 1 > "$R/gpurun_out/${tag}_prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/${tag}_prof.log"; exit 1; }
  python3 "$R/tools/kstats.py" "$R/gpurun_out/${tag}_prof/run_results.db" > "$R/gpurun_out/${tag}_kernel_stats.txt" && cat "$R/gpurun_out/${tag}_kernel_stats.txt"
fi
if [ "${PMC:-0}" = "1" ]; then
  # HBM bytes of one N=256 epoch step: FETCH_SIZE and WRITE_SIZE in separate passes
  R="$GRAFT_REPO_ROOT"
  cd /tmp
  B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --in-flight 1 --configs="
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/${tag}_pf" -o run -- python3 -u $B > "$R/gpurun_out/${tag}_pf.log" 2>&1 || { echo "pmc fetch failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/${tag}_pw" -o run -- python3 -u $B > "$R/gpurun_out/${tag}_pw.log" 2>&1 || { echo "pmc write failed"; exit 1; }
  python3 "$R/tools/pmcsum.py" "$R/gpurun_out/${tag}_pf/run_results.db" "$R/gpurun_out/${tag}_pw/run_results.db" > "$R/gpurun_out/${tag}_pmc_hbm.txt" 2>&1 || true
  cat "$R/gpurun_out/${tag}_pmc_hbm.txt"
  python3 "$R/tools/pmc_json.py" "$R/gpurun_out/${tag}_pf/run_results.db" "$R/gpurun_out/${tag}_pw/run_results.db" "${PMC_KERNEL:-k_verify_shares}" "${COMMIT:-unknown}" > "$R/gpurun_out/${tag}_pmc_hbm.json" && cat "$R/gpurun_out/${tag}_pmc_hbm.json"
fi
echo done
