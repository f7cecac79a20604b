#!/bin/bash
# Round 6: tail_kernel's fixed cost at small shards: references only (80), up to the bucket
# head (81), survivors counted not stored (82: no buffer, no barriers, no flush atomics),
# against the product, at 1/8 and 1/64 of c3.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for k in 8 64; do
  timeout -k 10 400 python3 -u scripts/ablate.py --no-build --config c3 --shard-of $k --steps 20 --variants 0,80,81,82,0,80,81,82 \
      > gpurun_out/r6u_sh$k.log 2>&1 || { echo "ablate sh$k failed rc=$?"; tail -5 gpurun_out/r6u_sh$k.log; exit 1; }
  echo "== 1/$k"; grep '^variant' gpurun_out/r6u_sh$k.log
done
