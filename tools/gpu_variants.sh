# Bench the in-tree library variants (hbbft_amd/libhbx*.so): shard-of-8 rehearsal (auto lanes)
# and the full N=256 epoch (auto lanes and forced 3 lanes).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-var}
timeout -k 10 300 python -u -m pytest tests/test_gpu_threshold.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_pytest.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${tag}_pytest.txt; exit 1; }
tail -1 gpurun_out/${tag}_pytest.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_coin.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_coin.txt 2>&1 || { echo "coin pytest failed"; tail -30 gpurun_out/${tag}_coin.txt; exit 1; }
tail -1 gpurun_out/${tag}_coin.txt
timeout -k 10 300 python -u tools/bench_aux.py --only c4 > gpurun_out/${tag}_c4.json 2>&1 || { echo "c4 failed"; tail -20 gpurun_out/${tag}_c4.json; exit 1; }
cat gpurun_out/${tag}_c4.json
for lib in hbbft_amd/libhbx*.so; do
  v=$(basename $lib .so)
  for mode in "--shard-of 8" ""; do
    HBX_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 3 $mode > gpurun_out/${tag}_run.json 2> gpurun_out/${tag}_run.err || { echo "$v $mode failed"; tail -5 gpurun_out/${tag}_run.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/${tag}_run.json')); print('$v', '$mode', d['ms_per_step'], d['kernels_ms'])" | tee -a gpurun_out/${tag}_summary.txt
  done
done
