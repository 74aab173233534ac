# Wave-state PMC pass of the share check: full N=256 epoch (one-lane kernel) and the shard-of-8
# slice (three-lane kernel), one epoch each.  Usage: gpurun -- bash tools/gpu_pmc_wave.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-w}
R="$GRAFT_REPO_ROOT"
cd /tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d "$R/gpurun_out/${tag}_full" -o run -- python3 -u "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --in-flight 1 --configs= > "$R/gpurun_out/${tag}_full.log" 2>&1 || { echo "pmc full failed"; tail -5 "$R/gpurun_out/${tag}_full.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d "$R/gpurun_out/${tag}_s8" -o run -- python3 -u "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --in-flight 1 --configs= --shard-of 8 > "$R/gpurun_out/${tag}_s8.log" 2>&1 || { echo "pmc s8 failed"; tail -5 "$R/gpurun_out/${tag}_s8.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d "$R/gpurun_out/${tag}_s8l1" -o run -- python3 -u "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --in-flight 1 --shard-of 8 --verify-lanes 1 --configs= > "$R/gpurun_out/${tag}_s8l1.log" 2>&1 || { echo "pmc s8l1 failed"; tail -5 "$R/gpurun_out/${tag}_s8l1.log"; exit 1; }
for v in full s8 s8l1; do echo "== $v"; python3 "$R/tools/pmcsum.py" "$R/gpurun_out/${tag}_${v}/run_results.db" | grep -E "verify_shares|combine|prepare"; done > "$R/gpurun_out/${tag}_pmc_wave.txt" 2>&1
cat "$R/gpurun_out/${tag}_pmc_wave.txt"
