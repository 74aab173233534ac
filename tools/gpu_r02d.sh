# Round-2 check: GPU tests, hash-to-G2 phases, bench (N=256 and shard-of-8), PMC HBM bytes of
# the share-check kernel (FETCH_SIZE and WRITE_SIZE in separate passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r02d}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${tag}_pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/${tag}_pytest_gpu.txt
timeout -k 10 120 ./tools/microbench/hashg2 > gpurun_out/${tag}_hashg2.txt 2>&1 || { echo "hashg2 failed"; exit 1; }
cat gpurun_out/${tag}_hashg2.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${tag}_bench.json')); print('N256', d['ms_per_step'], d['kernels_ms'], d['roofline']['frac'])"
timeout -k 10 200 python -u bench.py --shard-of 8 --no-cpu-baseline > gpurun_out/${tag}_bench_shard8.json 2> gpurun_out/${tag}_bench_shard8.err || { echo "shard8 failed"; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${tag}_bench_shard8.json')); print('shard8', d['ms_per_step'], d['kernels_ms'])"
cd /tmp
R="$GRAFT_REPO_ROOT"
B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/${tag}_pf" -o run -- python3 -u $B > "$R/gpurun_out/${tag}_pf.log" 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/${tag}_pw" -o run -- python3 -u $B > "$R/gpurun_out/${tag}_pw.log" 2>&1 || { echo "pmc write failed"; exit 1; }
python3 "$R/tools/pmcsum.py" "$R/gpurun_out/${tag}_pf/run_results.db" "$R/gpurun_out/${tag}_pw/run_results.db" | grep -E "verify_shares|prepare_ct|combine:" 
echo done
