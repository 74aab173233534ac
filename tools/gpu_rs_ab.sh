# A/B of RS coding builds on the C5 config: the broadcast GPU tests and a C5 bench line per library
# (automatic tile).  Usage: gpurun -- bash tools/gpu_rs_ab.sh <tag> <lib> [<lib> ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=$1; shift
for lib in "$@"; do
  n=$(basename "$lib" .so)
  HBX_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_broadcast.py tests/test_gpu_broadcast_host.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/${tag}_${n}_pytest.txt 2>&1 || { echo "$n tests failed"; tail -5 gpurun_out/${tag}_${n}_pytest.txt; exit 1; }
  HBX_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --configs=C5 --in-flight 1 --steps 10 \
    > gpurun_out/${tag}_${n}.json 2> gpurun_out/${tag}_${n}.err || { echo "$n bench failed"; tail -5 gpurun_out/${tag}_${n}.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['configs']['C5']; m=c['merkle_sha256']; r=c['rs_encode']; print(sys.argv[2], c['value'], m['ms'], r.get('ms'), r['roofline']['achieved'], '|', open(sys.argv[3]).read().strip().splitlines()[-1])" gpurun_out/${tag}_${n}.json $n gpurun_out/${tag}_${n}_pytest.txt
done | tee gpurun_out/${tag}_ab.txt
