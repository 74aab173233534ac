# Profile the shipped library: rocprofv3 kernel summary of the N=256 epoch + the C4 coin round, then
# PMC passes (wave states + instruction mix, FETCH_SIZE, WRITE_SIZE -- one pass each) over one bench
# step with the C4 round, so the share check's and the coin kernels' traffic come from the same
# build.  Optional first step: the issue-rate microbenchmark.
# Usage: gpurun -- bash tools/gpu_prof.sh <tag> [micro]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-p}
R="$GRAFT_REPO_ROOT"
if [ "${2:-}" = "micro" ] && [ -x tools/microbench/issue ]; then
  timeout -k 10 120 tools/microbench/issue > gpurun_out/${tag}_issue.txt 2>&1 || { echo "issue failed"; tail gpurun_out/${tag}_issue.txt; exit 1; }
  cat gpurun_out/${tag}_issue.txt
fi
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${tag}_prof" -o run -- python3 -u "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --in-flight 1 --configs=C4 > "$R/gpurun_out/${tag}_prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/${tag}_prof.log"; exit 1; }
python3 "$R/tools/kstats.py" "$R/gpurun_out/${tag}_prof/run_results.db" > "$R/gpurun_out/${tag}_kernel_stats.txt" && head -40 "$R/gpurun_out/${tag}_kernel_stats.txt"
B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --in-flight 1 --configs=C4"
W="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
timeout -s KILL 120 rocprofv3 --pmc $W --kernel-trace -d "$R/gpurun_out/${tag}_w" -o run -- python3 -u $B > "$R/gpurun_out/${tag}_w.log" 2>&1 || { echo "pmc wave failed"; tail -5 "$R/gpurun_out/${tag}_w.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/${tag}_f" -o run -- python3 -u $B > "$R/gpurun_out/${tag}_f.log" 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/${tag}_p" -o run -- python3 -u $B > "$R/gpurun_out/${tag}_p.log" 2>&1 || { echo "pmc write failed"; exit 1; }
python3 "$R/tools/pmcsum.py" "$R/gpurun_out/${tag}_w/run_results.db" "$R/gpurun_out/${tag}_f/run_results.db" "$R/gpurun_out/${tag}_p/run_results.db" > "$R/gpurun_out/${tag}_pmc.txt" 2>&1
grep -E "verify_shares|k_fe1|sig_shares|combine_sigs|hash_nonces" "$R/gpurun_out/${tag}_pmc.txt"
echo done
