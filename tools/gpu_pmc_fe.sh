# PMC passes over one N=256 epoch: wave states + instruction mix, and HBM bytes (FETCH_SIZE and
# WRITE_SIZE in passes of their own), for the one-lane share check (Miller kernel + k_fe1 steps)
# and, for comparison, the single-kernel one-lane check (--verify-lanes 7).
# Usage: gpurun -- bash tools/gpu_pmc_fe.sh <tag> [lanes ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-f}
shift
LANES=${@:-1 7}
R="$GRAFT_REPO_ROOT"
cd /tmp
W="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
for L in $LANES; do
  B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --in-flight 1 --configs= --verify-lanes $L"
  timeout -s KILL 120 rocprofv3 --pmc $W --kernel-trace -d "$R/gpurun_out/${tag}_w$L" -o run -- python3 -u $B > "$R/gpurun_out/${tag}_w$L.log" 2>&1 || { echo "pmc wave $L failed"; tail -5 "$R/gpurun_out/${tag}_w$L.log"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/${tag}_f$L" -o run -- python3 -u $B > "$R/gpurun_out/${tag}_f$L.log" 2>&1 || { echo "pmc fetch $L failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/${tag}_p$L" -o run -- python3 -u $B > "$R/gpurun_out/${tag}_p$L.log" 2>&1 || { echo "pmc write $L failed"; exit 1; }
  echo "== lanes $L"
  python3 "$R/tools/pmcsum.py" "$R/gpurun_out/${tag}_w$L/run_results.db" "$R/gpurun_out/${tag}_f$L/run_results.db" "$R/gpurun_out/${tag}_p$L/run_results.db" | grep -E "verify_shares|k_fe1"
done > "$R/gpurun_out/${tag}_pmc.txt" 2>&1
cat "$R/gpurun_out/${tag}_pmc.txt"
