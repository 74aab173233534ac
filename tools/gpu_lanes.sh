# Shard rehearsals (rank 0's slice of a G-way strong-scaled N=256 epoch) at each lane count.
# Usage: gpurun -- bash tools/gpu_lanes.sh <tag> "<G:lanes> ..."
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=$1
for gl in $2; do
  G=${gl%%:*}; L=${gl##*:}
  timeout -k 10 200 python -u bench.py --shard-of $G --verify-lanes $L --no-cpu-baseline --configs= --in-flight 1 > gpurun_out/${tag}_g${G}l${L}.json 2> gpurun_out/${tag}.err || { echo "G=$G lanes=$L failed"; tail -5 gpurun_out/${tag}.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/${tag}_g${G}l${L}.json').read().strip().splitlines()[-1]);print('G',sys.argv[1],'lanes',sys.argv[2],'->',d['verify_lanes'],d['ms_per_step'],d['kernels_ms'])" $G $L
done
