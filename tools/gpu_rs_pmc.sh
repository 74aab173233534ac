# PMC passes over one C5 bench step (RS coding, Merkle leaves): wave states + instruction mix, and
# FETCH_SIZE / WRITE_SIZE, one pass each.  Usage: gpurun -- bash tools/gpu_rs_pmc.sh <tag> [lib]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-rsp}
R="$GRAFT_REPO_ROOT"
[ -n "${2:-}" ] && export HBX_LIB_PATH="$R/$2"
cd /tmp
B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --in-flight 1 --configs=C5"
W="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS"
timeout -s KILL 120 rocprofv3 --pmc $W GRBM_GUI_ACTIVE --kernel-trace -d "$R/gpurun_out/${tag}_w" -o run -- python3 -u $B > "$R/gpurun_out/${tag}_w.log" 2>&1 || { echo "pmc wave failed"; tail -5 "$R/gpurun_out/${tag}_w.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM --kernel-trace -d "$R/gpurun_out/${tag}_x" -o run -- python3 -u $B > "$R/gpurun_out/${tag}_x.log" 2>&1 || { echo "pmc x failed"; tail -5 "$R/gpurun_out/${tag}_x.log"; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/${tag}_f" -o run -- python3 -u $B > "$R/gpurun_out/${tag}_f.log" 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/${tag}_p" -o run -- python3 -u $B > "$R/gpurun_out/${tag}_p.log" 2>&1 || { echo "pmc write failed"; exit 1; }
ls "$R"/gpurun_out/${tag}_x/run_results.db > /dev/null 2>&1 && X="$R/gpurun_out/${tag}_x/run_results.db" || X=
python3 "$R/tools/pmcsum.py" "$R/gpurun_out/${tag}_w/run_results.db" $X "$R/gpurun_out/${tag}_f/run_results.db" "$R/gpurun_out/${tag}_p/run_results.db" > "$R/gpurun_out/${tag}_pmc.txt" 2>&1
grep -E "rs_code|merkle" "$R/gpurun_out/${tag}_pmc.txt"
echo done
