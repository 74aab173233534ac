# Coin checks: the coin GPU tests (fixtures incl. cofactor-torsion shares, both lane counts, replay)
# and the C4 bench leg.  Usage: gpurun -- bash tools/gpu_coin.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=${1:-coin}
timeout -k 10 300 python -u -m pytest tests/test_gpu_coin.py tests/test_coin_replay.py tests/test_shard_rounds.py tests/test_reference_properties.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_pytest.txt 2>&1 || { tail -30 gpurun_out/${tag}_pytest.txt; exit 1; }
tail -1 gpurun_out/${tag}_pytest.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --configs=C4 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/${tag}_bench.json').read().strip().splitlines()[-1]);c=d['configs']['C4'];print(d['ms_per_step'],c['kernels_ms'],c['round_ms_kernels'],c['round_ms_wall'],c['value'])"
