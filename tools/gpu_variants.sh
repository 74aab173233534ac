# Kernel variants side by side (tools/build_variant.py -> hbbft_amd/libhbx_<name>.so; "main" = the
# shipped libhbx.so): the N=256 epoch bench line of each (its last step checked: validity bitmap and
# plaintexts), one after another, each under its own limit.
# Usage: gpurun -- bash tools/gpu_variants.sh <tag> "main vA vB ..."   (CONFIGS=C4 adds the coin round)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=${1:-v}
for v in ${2:-main}; do
  lib=hbbft_amd/libhbx.so
  [ "$v" = "main" ] || lib=hbbft_amd/libhbx_$v.so
  HBX_LIB_PATH=$PWD/$lib timeout -k 10 240 python -u bench.py --no-cpu-baseline --configs=${CONFIGS:-} --in-flight 1 --steps 10 \
    > gpurun_out/${tag}_${v}.json 2> gpurun_out/${tag}_${v}.err || { echo "$v failed"; tail -5 gpurun_out/${tag}_${v}.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c4=d.get('configs',{}).get('C4',{}); print(sys.argv[2], d['ms_per_step'], d['kernels_ms'], d['roofline']['frac'], c4.get('kernels_ms'), c4.get('round_ms_kernels'))" gpurun_out/${tag}_${v}.json $v
done | tee gpurun_out/${tag}_variants.txt
