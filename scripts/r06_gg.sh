#!/bin/bash
# Round 6: a level 1.5 in the L1, emulated (ablations 11 and 12, scripts/ablate_variants.py): c3, c2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for c in c3 c2; do
  timeout -k 10 400 python3 -u scripts/ablate.py --no-build --config $c --steps 5 --variants 0,11,12,0,11,12 \
      > gpurun_out/r6gg_$c.log 2>&1 || { echo "ablate $c failed rc=$?"; tail -5 gpurun_out/r6gg_$c.log; exit 1; }
  echo "== $c"; grep '^variant' gpurun_out/r6gg_$c.log
done
