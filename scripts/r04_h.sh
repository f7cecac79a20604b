#!/bin/bash
# Stage split of the c4 scan (timing-only variants 1-3, scripts/ablate_variants.py): the wide
# key groups (kgrp4) against the rank-word path (MP_NO_KGRP4=1), and c3 for reference.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
T=${1:-r4h}
timeout -k 10 400 python -u scripts/ablate.py --variants 0,1,2,3 --config c4 --no-build --steps 5 > gpurun_out/${T}_c4_k4.log 2>&1 || { echo "c4 k4 failed"; tail -5 gpurun_out/${T}_c4_k4.log; exit 1; }
tail -6 gpurun_out/${T}_c4_k4.log
MP_NO_KGRP4=1 timeout -k 10 400 python -u scripts/ablate.py --variants 0,1,2,3 --config c4 --no-build --steps 5 > gpurun_out/${T}_c4_rank.log 2>&1 || { echo "c4 rank failed"; tail -5 gpurun_out/${T}_c4_rank.log; exit 1; }
tail -6 gpurun_out/${T}_c4_rank.log
timeout -k 10 400 python -u scripts/ablate.py --variants 0,1,2,3 --config c3 --no-build --steps 5 > gpurun_out/${T}_c3.log 2>&1 || { echo "c3 failed"; tail -5 gpurun_out/${T}_c3.log; exit 1; }
tail -6 gpurun_out/${T}_c3.log
