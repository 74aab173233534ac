# Kernel trace with k_prepare_ct split into its hash and decode launches (HBX_SPLIT_PREP=1), for
# the full N=256 epoch and the shard-of-8 rehearsal.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
tag=${1:-split}
export HBX_SPLIT_PREP=1
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${tag}_full" -o run -- python3 -u "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/${tag}_full.log" 2>&1 || { echo "full failed"; tail -5 "$R/gpurun_out/${tag}_full.log"; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${tag}_s8" -o run -- python3 -u "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --shard-of 8 > "$R/gpurun_out/${tag}_s8.log" 2>&1 || { echo "s8 failed"; tail -5 "$R/gpurun_out/${tag}_s8.log"; exit 1; }

for b in tools/microbench/parts tools/microbench/parts_inl; do
  [ -x "$R/$b" ] || continue
  echo "== $b"; timeout -k 10 120 "$R/$b" || { echo "$b failed"; exit 1; }
done
echo done
