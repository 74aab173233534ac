# Round-2 GPU session: tests, bench (N=1 default), 8-way shard rehearsal, rocprof kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r02}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${tag}_pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/${tag}_pytest_gpu.txt
timeout -k 10 300 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
cat gpurun_out/${tag}_bench.json
timeout -k 10 200 python -u bench.py --shard-of 8 --no-cpu-baseline > gpurun_out/${tag}_bench_shard8.json 2> gpurun_out/${tag}_bench_shard8.err || { echo "shard8 failed"; exit 1; }
cat gpurun_out/${tag}_bench_shard8.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o prof -- python3 bench.py --steps 3 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/${tag}_prof.log; exit 1; }
echo done
timeout -k 10 300 python -u tools/bench_aux.py > gpurun_out/${tag}_aux.jsonl 2> gpurun_out/${tag}_aux.err || { echo "aux failed"; tail -20 gpurun_out/${tag}_aux.err; exit 1; }
cat gpurun_out/${tag}_aux.jsonl
for b in tools/microbench/hashg2 tools/microbench/parts tools/microbench/parts_w2; do
  [ -x "$b" ] || continue
  echo "== $b"; timeout -k 10 120 ./$b > gpurun_out/${tag}_$(basename $b).txt 2>&1 || { echo "$b failed"; cat gpurun_out/${tag}_$(basename $b).txt; exit 1; }
  cat gpurun_out/${tag}_$(basename $b).txt
done
