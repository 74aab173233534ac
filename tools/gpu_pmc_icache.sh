# Counter discovery + instruction-cache and LDS counters for k_verify_shares (bench step) and the
# C5 RS kernel (bench_aux c5).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
tag=${1:-ic}
timeout -s KILL 60 rocprofv3 --list-avail > "$R/gpurun_out/${tag}_avail.txt" 2>&1 || echo "list-avail rc=$?"
grep -o "SQC_[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_[A-Z_]*LDS[A-Z_]*" "$R/gpurun_out/${tag}_avail.txt" | sort -u | tr '\n' ' '; echo
B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --kernel-trace -d "$R/gpurun_out/${tag}_p1" -o run -- python3 -u $B > "$R/gpurun_out/${tag}_p1.log" 2>&1 || { echo "pass 1 failed"; tail -5 "$R/gpurun_out/${tag}_p1.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace -d "$R/gpurun_out/${tag}_p2" -o run -- python3 -u $B > "$R/gpurun_out/${tag}_p2.log" 2>&1 || { echo "pass 2 failed"; tail -5 "$R/gpurun_out/${tag}_p2.log"; exit 1; }
C="$R/tools/bench_aux.py --only c5 --steps 2"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace -d "$R/gpurun_out/${tag}_p3" -o run -- python3 -u $C > "$R/gpurun_out/${tag}_p3.log" 2>&1 || { echo "pass 3 failed"; tail -5 "$R/gpurun_out/${tag}_p3.log"; exit 1; }
echo done
