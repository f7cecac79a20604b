#!/bin/bash
# Round 6: scan time against the level-1 positive rate (ablations 9 / 7 / 10: 1/16, 1/8, 1/4 of
# windows pass a hashed level 1 with no LDS reads), c3, same box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u scripts/ablate.py --no-build --config c3 --steps 5 --variants 0,9,7,10,0,9,7,10 \
    > gpurun_out/r6q_c3.log 2>&1 || { echo "ablate failed rc=$?"; tail -5 gpurun_out/r6q_c3.log; exit 1; }
grep '^variant' gpurun_out/r6q_c3.log
