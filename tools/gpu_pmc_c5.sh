# HBM bytes of the C5 (Broadcast) kernels: FETCH_SIZE and WRITE_SIZE passes over a bench run with
# only the C5 config, then per-launch records for the RS coding and Merkle leaf kernels.
# Usage: gpurun -- bash tools/gpu_pmc_c5.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-c5}
R="$GRAFT_REPO_ROOT"
B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --in-flight 1 --configs=C5"
cd /tmp
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/${tag}_f" -o run -- python3 -u $B > "$R/gpurun_out/${tag}_f.log" 2>&1 || { echo "pmc fetch failed"; tail -5 "$R/gpurun_out/${tag}_f.log"; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/${tag}_p" -o run -- python3 -u $B > "$R/gpurun_out/${tag}_p.log" 2>&1 || { echo "pmc write failed"; exit 1; }
for k in k_rs_code_perm3 k_merkle_leaves_sha256 k_merkle_leaves_sha3 k_merkle_validate; do
  python3 "$R/tools/pmc_json.py" "$R/gpurun_out/${tag}_f/run_results.db" "$R/gpurun_out/${tag}_p/run_results.db" "$k" "${COMMIT:-unknown}" || true
done > "$R/gpurun_out/${tag}_pmc_c5.jsonl"
cat "$R/gpurun_out/${tag}_pmc_c5.jsonl"
