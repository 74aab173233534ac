# GPU check of the broadcast byte path: parity tests, C5 aux bench, rocprof kernel stats of it
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-rs}
timeout -k 10 600 python -u -m pytest tests/test_gpu_broadcast.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest.txt 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${tag}_pytest.txt; exit 1; }
tail -2 gpurun_out/${tag}_pytest.txt
for t in 0 4; do
  HBX_RS_TILE=$t timeout -k 10 300 python -u tools/bench_aux.py --only c5 > gpurun_out/${tag}_c5_t$t.json 2> gpurun_out/${tag}_c5.err || { echo "c5 failed"; tail -20 gpurun_out/${tag}_c5.err; exit 1; }
  echo "tile $t"; cat gpurun_out/${tag}_c5_t$t.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o c5 -- python3 tools/bench_aux.py --only c5 > gpurun_out/${tag}_prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/${tag}_prof.log; exit 1; }
find gpurun_out/${tag}_prof -name '*kernel_stats.csv' | head -1 | xargs cut -d, -f1-8 | head -20
timeout -k 10 60 ./tools/microbench/valu > gpurun_out/${tag}_valu.txt 2>&1 || { echo "valu failed"; exit 1; }
cat gpurun_out/${tag}_valu.txt
