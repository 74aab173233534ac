set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_coin.py tests/test_coin_replay.py tests/test_gpu_threshold.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04h_pytest.txt 2>&1 || { tail -30 gpurun_out/r04h_pytest.txt; exit 1; }
tail -1 gpurun_out/r04h_pytest.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --configs=C4 > gpurun_out/r04h_bench.json 2> gpurun_out/r04h_bench.err || { tail -20 gpurun_out/r04h_bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r04h_bench.json').read().strip().splitlines()[-1]);c=d['configs']['C4'];print(d['ms_per_step'],d['kernels_ms'],c['kernels_ms'],c['round_ms_kernels'],c['round_ms_wall'])"
bash tools/gpu_micro.sh r04h
COMMIT=$(cat .commit 2>/dev/null || echo unknown) bash tools/gpu_pmc_c5.sh r04h
