# RS coding tiles (HBX_RS_TILE: output rows x dwords per lane of k_rs_code_perm) on the C5 config,
# with the broadcast tests on the candidate tiles.  Usage: gpurun -- bash tools/gpu_rs_tiles.sh <tag> "<tiles>" [lib]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=${1:-rs}
LIB=${3:-$PWD/hbbft_amd/libhbx.so}
for t in ${2:-0}; do
  HBX_RS_TILE=$t HBX_LIB_PATH=$LIB timeout -k 10 300 python -u -m pytest tests/test_gpu_broadcast.py tests/test_gpu_broadcast_host.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/${tag}_t${t}_pytest.txt 2>&1 || { echo "tile $t tests failed"; tail -5 gpurun_out/${tag}_t${t}_pytest.txt; exit 1; }
  HBX_RS_TILE=$t HBX_LIB_PATH=$LIB timeout -k 10 300 python -u bench.py --no-cpu-baseline --configs=C5 --in-flight 1 --steps 5 \
    > gpurun_out/${tag}_t$t.json 2> gpurun_out/${tag}_t$t.err || { echo "tile $t failed"; tail -5 gpurun_out/${tag}_t$t.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['configs']['C5']; r=c['rs_encode']; print('tile', sys.argv[2], c['value'], r.get('ms'), r['roofline']['achieved'], '|', open(sys.argv[3]).read().strip().splitlines()[-1])" gpurun_out/${tag}_t$t.json $t gpurun_out/${tag}_t${t}_pytest.txt
done | tee gpurun_out/${tag}_tiles.txt
