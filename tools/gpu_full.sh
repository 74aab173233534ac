# Round-end style run: parity tests, the default bench line (with CPU baseline), rocprof summary.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --shard-of 8 > gpurun_out/bench_shard8.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 -u "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
