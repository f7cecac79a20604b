#!/bin/bash
# Whole GPU suite with the wide key groups as the c4 default, then c4's profile and bench line
# (CPU oracle over the whole genome).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
T=${1:-r4m}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1 \
    || { echo "gpu tests failed rc=$?"; grep -n "FAILED\|Error" gpurun_out/${T}_gputest.log | head; tail -5 gpurun_out/${T}_gputest.log; exit 1; }
tail -1 gpurun_out/${T}_gputest.log
bash scripts/r04_prof.sh r04b_c4 c4 600 || exit 1
