#!/bin/bash
# Strong-scaling evidence on one GPU: the shard curve (fixed per-run cost) and the bench lines
# of rank 0's half, quarter and eighth of c3 (parity against the whole-genome list).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04}
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/shard_curve.py > gpurun_out/${T}_shard_curve.txt 2>&1 || { echo "curve rc=$?"; tail -5 gpurun_out/${T}_shard_curve.txt; exit 1; }
tail -12 gpurun_out/${T}_shard_curve.txt
for n in 8 4 2; do
  timeout -k 10 300 python -u bench.py --shard-of $n --steps 30 --warmup 5 --no-cpu-baseline --no-e2e > gpurun_out/${T}_shard${n}.log 2>&1 || { echo "shard $n rc=$?"; exit 1; }
  tail -1 gpurun_out/${T}_shard${n}.log | cut -c1-300
done
