# PMC passes over one N=256 bench step (instruction mix, waits, HBM bytes) + VALU op-rate microbench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
tag=${1:-pmc}
B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 60 "$R/tools/microbench/valu" > "$R/gpurun_out/${tag}_valu.txt" 2>&1 || { echo "valu failed"; exit 1; }
cat "$R/gpurun_out/${tag}_valu.txt"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SMEM" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d "$R/gpurun_out/${tag}_p$i" -o run -- python3 -u $B > "$R/gpurun_out/${tag}_p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$R/gpurun_out/${tag}_p$i.log"; exit 1; }
done
echo done
