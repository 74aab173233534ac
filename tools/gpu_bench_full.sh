# The coin / threshold / shard GPU tests, then the full bench line (every config, CPU baselines)
# and the PMC passes of the one-lane share check.  Usage: gpurun -- bash tools/gpu_bench_full.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-bf}
timeout -k 10 400 python -u -m pytest tests/test_gpu_threshold.py tests/test_gpu_coin.py tests/test_coin_replay.py tests/test_shard_rounds.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${tag}_pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/${tag}_pytest_gpu.txt
timeout -k 10 900 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
cut -c1-600 gpurun_out/${tag}_bench.json
bash tools/gpu_pmc_fe.sh ${tag} 1

if [ -x tools/microbench/coin_parts ]; then
  timeout -k 10 120 tools/microbench/coin_parts > gpurun_out/${tag}_coin_parts.txt 2>&1 && cat gpurun_out/${tag}_coin_parts.txt
fi
echo done
