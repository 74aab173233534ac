# Stochastic PC sampling over one N=256 bench step (where k_verify_shares waves stall).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
tag=${1:-pcs}
method=${2:-stochastic}
timeout -s KILL 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $method --pc-sampling-unit cycles --pc-sampling-interval 1048576 --output-format csv -d "$R/gpurun_out/${tag}" -o pcs -- python3 -u "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$R/gpurun_out/${tag}.log" 2>&1 || { echo "pc sampling rc=$?"; tail -15 "$R/gpurun_out/${tag}.log"; exit 1; }
ls -la "$R/gpurun_out/${tag}"
echo done
