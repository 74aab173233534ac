# HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of the coin check for the shipped library and a variant
# (tools/build_variant.py).  Usage: gpurun -- bash tools/gpu_pmc_variants.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
for v in main as; do
  lib=$R/hbbft_amd/libhbx.so; [ "$v" = "main" ] || lib=$R/hbbft_amd/libhbx_$v.so
  cd /tmp
  B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --in-flight 1 --configs=C4"
  HBX_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/r06o_${v}_f" -o run -- python3 -u $B > "$R/gpurun_out/r06o_${v}_f.log" 2>&1 || { echo "fetch $v failed"; exit 1; }
  HBX_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/r06o_${v}_p" -o run -- python3 -u $B > "$R/gpurun_out/r06o_${v}_p.log" 2>&1 || { echo "write $v failed"; exit 1; }
  cd "$R"
  python3 tools/pmc_json.py gpurun_out/r06o_${v}_f/run_results.db gpurun_out/r06o_${v}_p/run_results.db "k_verify_sig_shares2(,k_verify_sig_shares2_fe<true>" $v --skip-empty > gpurun_out/r06o_${v}_pmc_coin.json
  cat gpurun_out/r06o_${v}_pmc_coin.json; echo
done
