# Two PMC passes (instruction mix, waits) over one N=256 bench step.
set -e
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 --kernel-trace -d "$R/gpurun_out/pmcA" -o run -- python3 -u $B > "$R/gpurun_out/pmcA.log" 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH --kernel-trace -d "$R/gpurun_out/pmcB" -o run -- python3 -u $B > "$R/gpurun_out/pmcB.log" 2>&1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/pmcC" -o run -- python3 -u $B > "$R/gpurun_out/pmcC.log" 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/pmcD" -o run -- python3 -u $B > "$R/gpurun_out/pmcD.log" 2>&1
