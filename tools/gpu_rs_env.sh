# RS coding settings swept on the C5 config: per setting ("VAR=value[,VAR=value]" or "-" for none)
# the broadcast GPU tests and a C5 bench line.  Usage: gpurun -- bash tools/gpu_rs_env.sh <tag> <lib> <setting> ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=$1; lib=$PWD/$2; shift 2
i=0
for st in "$@"; do
  i=$((i + 1))
  envs=(HBX_LIB_PATH=$lib)
  [ "$st" != "-" ] && IFS=, read -ra extra <<< "$st" && envs+=("${extra[@]}")
  env "${envs[@]}" timeout -k 10 300 python -u -m pytest tests/test_gpu_broadcast.py tests/test_gpu_broadcast_host.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/${tag}_${i}_pytest.txt 2>&1 || { echo "$st tests failed"; tail -5 gpurun_out/${tag}_${i}_pytest.txt; exit 1; }
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --no-cpu-baseline --configs=C5 --in-flight 1 --steps 10 \
    > gpurun_out/${tag}_${i}.json 2> gpurun_out/${tag}_${i}.err || { echo "$st bench failed"; tail -5 gpurun_out/${tag}_${i}.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['configs']['C5']; m=c['merkle_sha256']; r=c['rs_encode']; print(sys.argv[2], c['value'], m['ms'], r.get('ms'), r['roofline']['achieved'], '|', open(sys.argv[3]).read().strip().splitlines()[-1])" gpurun_out/${tag}_${i}.json "$st" gpurun_out/${tag}_${i}_pytest.txt
done | tee gpurun_out/${tag}_env.txt
