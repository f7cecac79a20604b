#!/bin/bash
# Round 6: what record-line locality could save in pair_kernel (ablation 57), what the hit writes cost (55), and non-temporal genome loads (58).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for c in c4 c3; do
  timeout -k 10 400 python3 -u scripts/ablate.py --no-build --config $c --steps 5 --variants 0,58,0,58 \
      > gpurun_out/r6w_$c.log 2>&1 || { echo "ablate $c failed rc=$?"; tail -5 gpurun_out/r6w_$c.log; exit 1; }
  echo "== $c"; grep '^variant' gpurun_out/r6w_$c.log
done
