#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
T=${1:-r4f}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1 \
    || { echo "gpu tests failed rc=$?"; tail -30 gpurun_out/${T}_gputest.log; exit 1; }
tail -1 gpurun_out/${T}_gputest.log
SHARD=1 CFG=c4 bash scripts/r04_ab.sh ${T}_c4 prod= r03=R03 prod2= r03b=R03 || exit 1
SHARD=1 CFG=c3 bash scripts/r04_ab.sh ${T}_c3 prod= r03=R03 || exit 1
