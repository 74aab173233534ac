# Pairing parts microbenchmark: timings + PMC waits per part kernel.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
tag=${1:-parts}
timeout -k 10 120 "$R/tools/microbench/parts" > "$R/gpurun_out/${tag}.txt" 2>&1 || { echo "parts failed"; cat "$R/gpurun_out/${tag}.txt"; exit 1; }
cat "$R/gpurun_out/${tag}.txt"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM --kernel-trace -d "$R/gpurun_out/${tag}_p1" -o run -- "$R/tools/microbench/parts" > "$R/gpurun_out/${tag}_p1.log" 2>&1 || { echo "pmc failed"; tail -5 "$R/gpurun_out/${tag}_p1.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_IFETCH SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-trace -d "$R/gpurun_out/${tag}_p2" -o run -- "$R/tools/microbench/parts" > "$R/gpurun_out/${tag}_p2.log" 2>&1 || { echo "pmc2 failed"; tail -5 "$R/gpurun_out/${tag}_p2.log"; }
echo done
