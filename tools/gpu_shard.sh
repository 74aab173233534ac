# Shard-of-8 rehearsal and the C2 epoch (both on the six-lane check), plus the threshold tests.
# Usage: gpurun -- bash tools/gpu_shard.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=${1:-sh}
timeout -k 10 300 python -u -m pytest tests/test_gpu_threshold.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_pytest.txt 2>&1 || { tail -30 gpurun_out/${tag}_pytest.txt; exit 1; }
tail -1 gpurun_out/${tag}_pytest.txt
timeout -k 10 300 python -u bench.py --shard-of 8 --no-cpu-baseline --configs=C2 > gpurun_out/${tag}_bench_shard8.json 2> gpurun_out/${tag}_shard8.err || { tail -20 gpurun_out/${tag}_shard8.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/${tag}_bench_shard8.json').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['kernels_ms'],d['epochs_in_flight']['ms_per_epoch']);c=d['configs']['C2'];print('C2',c['ms_per_epoch'],c['kernels_ms'])"
