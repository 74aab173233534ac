# Pairing-parts microbenchmark over build variants (tools/microbench/parts_*).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=${1:-pv}
for b in tools/microbench/parts_*; do
  echo "== $b"
  timeout -k 10 120 ./$b > gpurun_out/${tag}_$(basename $b).txt 2>&1 || { echo "$b failed"; cat gpurun_out/${tag}_$(basename $b).txt; exit 1; }
  cat gpurun_out/${tag}_$(basename $b).txt
done
