# quick GPU check: threshold tests + bench at N=256 (1 lane auto) + shard-of-8 rehearsal (3 lanes auto)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-q}
timeout -k 10 600 python -u -m pytest tests/test_gpu_threshold.py tests/test_replay.py tests/test_shard_gloo.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest.txt 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${tag}_pytest.txt; exit 1; }
tail -2 gpurun_out/${tag}_pytest.txt
timeout -k 10 200 python -u bench.py --shard-of 8 --no-cpu-baseline > gpurun_out/${tag}_shard8.json 2> gpurun_out/${tag}_shard8.err || { echo "shard8 failed"; tail -20 gpurun_out/${tag}_shard8.err; exit 1; }
cat gpurun_out/${tag}_shard8.json
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
cat gpurun_out/${tag}_bench.json
