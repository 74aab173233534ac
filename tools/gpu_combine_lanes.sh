# The N=256 epoch with the Lagrange combine on one lane per term (k_combine, the default at N=256)
# and on quads of lanes per term (k_combine_q), each bench line's last step checked.
# Usage: gpurun -- bash tools/gpu_combine_lanes.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=${1:-cl}
for L in 1 4; do
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --configs= --in-flight 1 --steps 10 --combine-lanes $L \
    > gpurun_out/${tag}_c$L.json 2> gpurun_out/${tag}_c$L.err || { echo "combine lanes $L failed"; tail -5 gpurun_out/${tag}_c$L.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('combine lanes', sys.argv[2], d['ms_per_step'], d['kernels_ms'])" gpurun_out/${tag}_c$L.json $L
done | tee gpurun_out/${tag}_combine_lanes.txt
