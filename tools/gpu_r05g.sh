# Round-5 check + profile: threshold/coin/broadcast-host GPU tests, the N=256 bench line with the C4
# round, the shard-of-8 slice, then tools/gpu_prof.sh (kernel stats + wave-state / FETCH / WRITE PMC
# passes).  Usage: gpurun -- bash tools/gpu_r05g.sh <tag> [pytest -k expr]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r05g}
K=${2:-threshold or coin or host_api}
bash tools/gpu_check.sh $tag "$K" || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --configs=C4 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/${tag}_bench.json')); c=d['configs']['C4']
print('epoch', d['ms_per_step'], d['kernels_ms'], 'frac', d['roofline']['frac'], 'inflight', d.get('epochs_in_flight',{}).get('ms_per_epoch'))
print('C4', c.get('round_ms_kernels'), c.get('round_ms_wall'), c.get('kernels_ms'))"
timeout -k 10 300 python -u bench.py --shard-of 8 --no-cpu-baseline --configs= > gpurun_out/${tag}_bench_shard8.json 2> gpurun_out/${tag}_shard8.err || { echo "shard8 failed"; tail -20 gpurun_out/${tag}_shard8.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/${tag}_bench_shard8.json')); print('shard8', d['ms_per_step'], d['kernels_ms'], d.get('verify_lanes'))"
bash tools/gpu_prof.sh $tag || exit 1
echo done
