#!/bin/bash
# Round 6: how much of pair_kernel is the primer-1 compare (ablation 54: dropped), c4 and c3,
# before building 32-B survivors that carry the primer-1 window.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for c in c4 c3; do
  timeout -k 10 400 python3 -u scripts/ablate.py --no-build --config $c --steps 5 --variants 0,54,0,54 \
      > gpurun_out/r6k_$c.log 2>&1 || { echo "ablate $c failed rc=$?"; tail -5 gpurun_out/r6k_$c.log; exit 1; }
  grep '^variant' gpurun_out/r6k_$c.log
done
